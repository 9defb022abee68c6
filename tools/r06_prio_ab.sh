#!/bin/bash
# hs_k_lin8's issue-priority scheme on the final build: L8_PRIO 4 (the product: SIMD pairs take turns) against 0 (none)
# and 1 (alternate per group, all waves in phase), interleaved
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_prio; mkdir -p $O
for P in 200000 2000000 25000; do
 for V in prod p0 p1 prod p0 p1; do
  L=""; [ $V != prod ] && L="HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_$V.so"
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
