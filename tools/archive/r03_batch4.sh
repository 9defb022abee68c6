#!/bin/bash
# round-3 batch 4: the whole GPU suite, then the evidence (every bench line, sweep, rocprof)
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_v4
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.txt | head -5 | cut -c1-300; tail -2 $OUT/pytest_gpu.txt
[ $rc -gt 1 ] && exit $rc
bash tools/r03_evidence.sh r03_v4
