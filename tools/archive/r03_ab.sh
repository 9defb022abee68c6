#!/bin/bash
# A/B of a variant library against the product: headline at 300 steps (alternating, 2 each) + the variant's chain trace
# usage: tools/r03_ab.sh TAG VARIANT
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/$1
V=$2
mkdir -p $OUT
for r in 1 2; do
  for L in product $V; do
    if [ $L = product ]; then unset HSLAM_AMD_LIB; else export HSLAM_AMD_LIB=$GRAFT_REPO_ROOT/h-slam_amd/lib/variants/libhslam_amd_$L.so; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/$L$r.json 2> $OUT/$L$r.err || { echo "bench $L failed"; tail -5 $OUT/$L$r.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/$L$r.json'));print('$L',round(d['ms_per_step']*1e3,2),'us/step')"
  done
done
export HSLAM_AMD_LIB=$GRAFT_REPO_ROOT/h-slam_amd/lib/variants/libhslam_amd_$V.so
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/tr.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/tr.txt | tail -1
