#!/bin/bash
# lin8 variants: parity tests per variant build, then the 200k / 2M sweep points.  usage: tools/r03_lin8.sh TAG "variants"
TAG=${1:-r03_lin8}
VARS=${2:-"product ldsacc2"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for V in $VARS; do
  if [ $V = product ]; then unset HSLAM_AMD_LIB; else export HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_$V.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_lin8.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_lin8_$V.txt 2>&1
  rc=$?; echo "$V lin8 tests rc=$rc"; tail -2 $OUT/pytest_lin8_$V.txt
  [ $rc -ne 0 ] && exit $rc
  for P in 200000 2000000; do
    timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --points $P > $OUT/${V}_p$P.json 2> $OUT/${V}_p$P.err || { echo "$V $P failed"; tail -5 $OUT/${V}_p$P.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/${V}_p$P.json'));print('$V',$P,round(d['value']/1e6),'Mpres/s',round(d['ms_per_step']*1e3,1),'us/step lin',round(d['roofline']['avg_launch_ms']*1e3,1),'us frac',round(d['roofline']['frac'],3))"
  done
done
