#!/bin/bash
# LDLT variants: BA parity tests on the product build, then per variant the 2k headline line and the solve's
# in-kernel trace (HS_SOLVE_DBG=8: the LDLT runs twice, slots 20-22 give its cycles).  usage: tools/r03_solve.sh TAG [variants]
TAG=${1:-r03_solve}
VARS=${2:-"product ldlt4"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_window.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_ba.txt 2>&1
rc=$?; echo "ba tests rc=$rc"; tail -3 $OUT/pytest_ba.txt; [ $rc -ne 0 ] && exit $rc
for V in $VARS; do
  if [ $V = product ]; then unset HSLAM_AMD_LIB; else export HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_$V.so; fi
  for rep in 1 2; do
    timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu > $OUT/${V}_2k_$rep.json 2> $OUT/${V}_2k_$rep.err || { echo "$V bench failed"; tail -5 $OUT/${V}_2k_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${V}_2k_$rep.json'));print('$V 2k',round(d['value']/1e6,1),'Mpres/s',round(d['ms_per_step']*1e3,2),'us/step')"
  done
  HS_KTRACE=1 HS_SOLVE_DBG=8 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/${V}_tr.json 2> $OUT/${V}_tr.txt || { echo "$V trace failed"; exit 1; }
  grep "solve" $OUT/${V}_tr.txt | tail -6
done
