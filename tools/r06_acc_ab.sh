#!/bin/bash
# hs_k_lin8 with parts of its accumulation compiled out (timing only: the systems are wrong): what the
# AccumulatorApprox reduce-scatter (notop) and the Schur accumulators (noschur) cost per launch.  The variants were
# built with temporary #ifndef XB_NOTOP / XB_NOSCHUR guards around the two blocks of hs_lin8_kernels.hip (not kept):
# make variant V=notop X=-DXB_NOTOP, V=noschur X=-DXB_NOSCHUR, V=noacc X="-DXB_NOTOP -DXB_NOSCHUR"
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_acc; mkdir -p $O
for P in 200000 2000000; do
 for V in base notop noschur noacc base2; do
  L=""; [ $V != base ] && [ $V != base2 ] && L="HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_$V.so"
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
