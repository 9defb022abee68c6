#!/bin/bash
# hs_k_lin8 workgroup -> block map giving each XCD one contiguous image band (an experiment patch, measured and not kept:
# profiles/r06_xcd_ab.txt) against the identity order (HS_LIN8_XCDMAP=0)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_xcd; mkdir -p $O
cd $R && timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lin8.py tests/test_gpu_shard.py > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc = 0 ] || exit $rc
for P in 200000 2000000 25000 100000; do
 for V in map ident map ident; do
  L=""; [ $V = ident ] && L="HS_LIN8_XCDMAP=0"
  echo -n "$V "; env $L timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
