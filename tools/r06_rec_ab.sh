#!/bin/bash
# the fused point step's slot-dot gathers from one LDS record per point (an experiment patch, L8_STEP_REC=1, not kept:
# profiles/r06_rec_ab.txt) against ds_bpermute (the product): the lin8 tests on the variant, then the GN loop's launch
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_rec; mkdir -p $O
cd $R && HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_rec.so timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_lin8.py tests/test_gpu_shard.py > $O/pytest.txt 2>&1; rc=$?; tail -2 $O/pytest.txt; [ $rc = 0 ] || exit $rc
for P in 200000 2000000 25000; do
 for V in prod rec prod rec; do
  L=""; [ $V = rec ] && L="HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_rec.so"
  env $L timeout -k 10 200 python3 $R/bench.py --points $P --steps 10 --warmup 2 --no-cpu > $O/${V}_$P.json 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/${V}_$P.json'));r=d['roofline'];print('$V $P', round(r['avg_launch_ms_gn_loop']*1e3,1), 'us in loop', round(r['avg_launch_ms']*1e3,1), 'us plain', round(d['ms_per_step']*1e3,1), 'us/step')"
 done
done
