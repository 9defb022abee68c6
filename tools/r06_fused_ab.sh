#!/bin/bash
# hs_k_lin8 back-to-back: the fused-step launch (the GN loop's) against the plain one; needs a temporary HS_TIME_FUSED switch in
# hs_ba_time_linearize (launch_linearize(c, 1) instead of (c, 0); not kept, profiles/r06_fused_ab.txt)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_fused; mkdir -p $O
for P in 200000 2000000; do
 for V in plain fused plain fused; do
  L=""; [ $V = fused ] && L="HS_TIME_FUSED=1"
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
