#!/bin/bash
# hs_k_lin8 with the AccumulatorApprox T slice in registers across the point groups (an experiment patch, not kept:
# L8_T_REG=1, 256 VGPRs; profiles/r06_treg_ab.txt) against the product (the T slice read-modify-written in LDS)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_treg; mkdir -p $O
cd $R && HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_treg.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lin8.py tests/test_gpu_shard.py > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc = 0 ] || exit $rc
for P in 200000 2000000 25000; do
 for V in prod treg prod treg; do
  L=""; [ $V = treg ] && L="HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_treg.so"
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
