#!/bin/bash
# the product (Schur accumulators on VALU, L8_MFMA_SC=0, filled grid) against the MFMA-accumulator build (variants/mfma) and
# the packed-pair accD / accE updates (variants/pk, L8_PK_SC=1)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_nomfma; mkdir -p $O
cd $R && timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lin8.py tests/test_gpu_shard.py > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc = 0 ] || exit $rc
for P in 200000 2000000 25000; do
 for V in valu mfma pk valu mfma pk; do
  L=""; [ $V != valu ] && L="HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_$V.so"
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
