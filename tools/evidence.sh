#!/bin/bash
# round-6 evidence (as rounds 4-5): smoke, every bench line (CPU baselines included), the sweep, rocprofv3 kernel trace + stats of
# the headline.  usage: tools/evidence.sh TAG   (outputs under gpurun_out/TAG/)
TAG=${1:-ev}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed rc=$?"; tail -30 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
head -c 700 $OUT/bench.json; echo
for W in trace track act refine select; do
  timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 3 --cpu-seconds 8 > $OUT/bench_$W.json 2> $OUT/bench_$W.err || { echo "bench $W failed rc=$?"; tail -20 $OUT/bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$W.json'));print('$W',round(d['ms_per_step'],4),'ms',d.get('speedup_vs_cpu'))"
done
timeout -k 10 300 python bench.py --workload ba-kitti --steps 50 --warmup 5 --cpu-seconds 6 > $OUT/bench_ba_kitti.json 2> $OUT/bench_ba_kitti.err || { echo "bench ba-kitti failed"; tail -20 $OUT/bench_ba_kitti.err; exit 1; }
timeout -k 10 300 python bench.py --workload keyframe --steps 10 --warmup 2 --cpu-seconds 6 > $OUT/bench_keyframe.json 2> $OUT/bench_keyframe.err || { echo "bench keyframe failed"; tail -20 $OUT/bench_keyframe.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_ba_kitti.json'));print('kitti',round(d['ms_per_step']*1e3,2),'us')"
head -c 600 $OUT/bench_keyframe.json; echo
for P in 20000 200000 2000000; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --points $P > $OUT/p$P.json 2> $OUT/p$P.err || { echo "sweep $P failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/p$P.json'));print('$P',round(d['ms_per_step']*1e3,1),'us/step',d['roofline']['kernel'],round(d['roofline']['avg_launch_ms']*1e3,1),'us frac',round(d['roofline']['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "rocprof rc=$?"
find $OUT/prof -name "*kernel_stats.csv" -exec head -8 {} \;
