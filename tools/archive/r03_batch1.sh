#!/bin/bash
# round-3 batch 1: multi-rank checks + chain trace, fused reduce+stitch A/B, lin8 variants, multi-workgroup tracker
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_b1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_threshold.py tests/test_gpu_ba.py -k "shard or group or threshold or rank or communicator" -v --timeout 120 --timeout-method thread > $OUT/pytest_mr.txt 2>&1
rc=$?
echo "multi-rank tests rc=$rc"; grep -E "FAILED|ERROR|passed|failed" $OUT/pytest_mr.txt | tail -8 | cut -c1-200
[ $rc -gt 1 ] && exit $rc
bash tools/r03_exp1.sh r03_b1_exp1 "ldsacc2 ldsacc1 product" || exit $?
bash tools/r03_trk.sh r03_b1_trk || exit $?
