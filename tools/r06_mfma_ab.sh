#!/bin/bash
# hs_k_lin8 with the Schur accumulators on MFMA (product build) against the per-lane form (variants/old), and the
# lin8 parity tests
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_mfma; mkdir -p $O
cd $R && timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_lin8.py tests/test_gpu_shard.py > $O/pytest.txt 2>&1; rc=$?; tail -3 $O/pytest.txt; [ $rc = 0 ] || exit $rc
for P in 200000 2000000 20000; do
 for V in old new old2 new2; do
  L=""; case $V in old*) L="HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_old.so";; esac
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
