#!/bin/bash
# round-4 evidence, second pass (tracker / keyframe changes): smoke, the headline / track / keyframe lines with their
# CPU baselines, rocprofv3 kernel trace + stats of the track line, and its PMC roof passes (tools/r04_pmc.sh)
TAG=${1:-r04_ev2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed rc=$?"; tail -30 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
head -c 400 $OUT/bench.json; echo
timeout -k 10 300 python bench.py --workload track --cpu-seconds 8 > $OUT/bench_track.json 2> $OUT/bench_track.err || { echo "bench track failed"; tail -20 $OUT/bench_track.err; exit 1; }
timeout -k 10 300 python bench.py --workload keyframe --cpu-seconds 6 > $OUT/bench_keyframe.json 2> $OUT/bench_keyframe.err || { echo "bench keyframe failed"; tail -20 $OUT/bench_keyframe.err; exit 1; }
for W in track keyframe; do python3 -c "import json;d=json.load(open('$OUT/bench_$W.json'));print('$W',round(d['ms_per_step'],4),'ms',d.get('speedup_vs_cpu'))"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_track -o track -- python3 $GRAFT_REPO_ROOT/bench.py --workload track --no-cpu > $OUT/prof_track.json 2> $OUT/prof_track.err
echo "rocprof rc=$?"
find $OUT/prof_track -name "*kernel_stats.csv" -exec head -6 {} \;
bash $GRAFT_REPO_ROOT/tools/r04_pmc.sh ${TAG}_pmc track
