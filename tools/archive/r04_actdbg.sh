#!/bin/bash
# hs_k_act_dist experiment: kernel stats with parts switched off (HS_ACT_DBG bits)
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_actdbg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for D in 0 1 2 4; do
  HS_ACT_DBG=$D timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/d$D -o act -- python3 $GRAFT_REPO_ROOT/bench.py --workload act --steps 5 --warmup 1 --no-cpu > /dev/null 2>&1 || { echo "dbg $D failed"; exit 1; }
  echo "== HS_ACT_DBG=$D"; find $OUT/d$D -name "*kernel_stats.csv" -exec grep -E "act_dist|act_select" {} \;
done
