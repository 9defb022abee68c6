#!/bin/bash
# round-3 GPU iteration: pytest -m gpu (all), the headline bench.  usage: tools/r03_run.sh TAG [pytest-args]
TAG=${1:-r03}
shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
T=${@:-tests}
timeout -k 10 600 python -u -m pytest $T -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_gpu.txt | tail -5; tail -25 $OUT/pytest_gpu.txt | grep -v PASSED
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
head -c 600 $OUT/bench.json; echo
