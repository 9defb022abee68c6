#!/bin/bash
# round-4 GPU iteration: pytest -m gpu (given tests, default all), then the driver's bench command.
# usage: tools/r04_run.sh TAG [pytest-args]
TAG=${1:-r04}
shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
T=${@:-tests}
timeout -k 10 900 python -u -m pytest $T -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -cE "PASSED" $OUT/pytest_gpu.txt; tail -25 $OUT/pytest_gpu.txt | grep -v PASSED
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
head -c 1500 $OUT/bench.json; echo
