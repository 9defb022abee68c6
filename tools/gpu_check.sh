#!/bin/bash
# GPU check on the gpurun box: smoke -> pytest -m gpu -> bench -> rocprofv3 kernel stats.
# usage: tools/gpu_check.sh TAG   (outputs under gpurun_out/TAG/)
TAG=${1:-check}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed rc=$?"; tail -30 $OUT/smoke.txt; exit 1; }
tail -3 $OUT/smoke.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -30 $OUT/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 50 --warmup 5 --cpu-seconds 8 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/trace_bench.json 2> $OUT/trace.txt || { echo "trace run failed rc=$?"; tail -30 $OUT/trace.txt; exit 1; }
grep "hs trace" $OUT/trace.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "rocprof rc=$?"
find $OUT/prof -name "*stats*"
