#!/bin/bash
# GPU check of the DirectRefinement path: parity tests, bench, rocprof kernel stats.  usage: tools/refine_check.sh TAG
TAG=${1:-refine}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_refine.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_refine.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 $OUT/pytest_refine.txt
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --workload refine --steps 50 --warmup 3 --cpu-seconds 8 > $OUT/refine_bench.json 2> $OUT/refine_bench.err || { echo "bench failed"; tail -20 $OUT/refine_bench.err; exit 1; }
cat $OUT/refine_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o refine -- python3 $GRAFT_REPO_ROOT/bench.py --workload refine --steps 50 --warmup 3 --no-cpu > $OUT/prof_refine.json 2> $OUT/prof_refine.err
echo "rocprof rc=$?"
