#!/bin/bash
# multi-rank path checks (rank group, one-block select, 1-rank RCCL), then the end-of-round evidence suite
TAG=${1:-r03_mr}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_threshold.py tests/test_gpu_ba.py -k "shard or group or threshold or rank or communicator" -v --timeout 120 --timeout-method thread > $OUT/pytest_mr.txt 2>&1
rc=$?
echo "multi-rank tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_mr.txt | tail -8
if [ $rc -gt 1 ]; then exit $rc; fi
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/trace.json 2> $OUT/trace.txt || { echo "trace failed"; tail -5 $OUT/trace.txt; exit 1; }
grep "chain\|span" $OUT/trace.txt | tail -6
bash tools/all_bench.sh ${TAG}_all
