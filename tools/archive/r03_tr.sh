#!/bin/bash
# chain trace of the headline (per-kernel checkpoints)
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_tr${1:-}
mkdir -p $OUT
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/tr.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/tr.txt | tail -1
