#!/bin/bash
# experiments: fused reduce + stitch (HS_FUSE_RS) parity + 2k step A/B with chain traces; lin8 variants at 200k / 2M
TAG=${1:-r03_exp1}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -k "fused" -v --timeout 120 --timeout-method thread > $OUT/pytest_fused.txt 2>&1
rc=$?; echo "fused tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_fused.txt | tail -4
[ $rc -gt 1 ] && exit $rc
for V in product linwt product linwt; do
  if [ $V = product ]; then unset HSLAM_AMD_LIB; else export HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_$V.so; fi
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/wt_$V.json 2> $OUT/wt_$V.err || { echo "$V failed"; tail -5 $OUT/wt_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/wt_$V.json'));print('$V',round(d['ms_per_step']*1e3,2),'us/step')"
done
unset HSLAM_AMD_LIB
for F in 0 1 0 1; do
  HS_FUSE_RS=$F timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/fuse$F.json 2> $OUT/fuse$F.err || { echo "fuse $F failed"; tail -5 $OUT/fuse$F.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/fuse$F.json'));print('fuse $F',round(d['ms_per_step']*1e3,2),'us/step')"
done
for F in 0 1; do
  HS_FUSE_RS=$F HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr$F.json 2> $OUT/tr$F.txt || { echo "trace failed"; exit 1; }
  grep "chain" $OUT/tr$F.txt | tail -1
done
bash tools/r03_lin8.sh ${TAG}_lin8 "${2:-ldsacc2 ldsacc1 product}" || exit $?
