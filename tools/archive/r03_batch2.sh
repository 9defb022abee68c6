#!/bin/bash
# round-3 batch 2: the whole GPU suite on the new defaults (lin8 occupancy 2, tracker G = 8 + reduce-scatter), then
# A/B: hs_k_lin write-through partials (2k), lin8 vs lin at 20k / 60k, the C2 track line, the headline chain trace
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_b2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.txt | head -5 | cut -c1-300; tail -2 $OUT/pytest_gpu.txt
[ $rc -gt 1 ] && exit $rc
for V in product linwt product linwt; do
  if [ $V = product ]; then unset HSLAM_AMD_LIB; else export HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_$V.so; fi
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/wt_$V.json 2> $OUT/wt_$V.err || { echo "$V failed"; tail -5 $OUT/wt_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/wt_$V.json'));print('$V',round(d['ms_per_step']*1e3,2),'us/step')"
done
unset HSLAM_AMD_LIB
for P in 20000 60000; do
  for L in 0 1; do
    HS_LIN8=$L timeout -k 10 200 python bench.py --points $P --steps 50 --warmup 5 --no-cpu > $OUT/p${P}_l$L.json 2> $OUT/p${P}_l$L.err || { echo "p$P lin8=$L failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/p${P}_l$L.json'));print('$P lin8=$L',round(d['ms_per_step']*1e3,1),'us/step lin',round(d['roofline']['avg_launch_ms']*1e3,1), d['roofline']['kernel'])"
  done
done
timeout -k 10 200 python bench.py --workload track --steps 20 --warmup 3 --no-cpu > $OUT/trk.json 2> $OUT/trk.err || { echo "track failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/trk.json'));print('track',round(d['ms_per_step'],4),'ms device',round(d['config']['device_ms_per_track'],4))"
HS_KTRACE=1 timeout -k 10 200 python bench.py --workload track --steps 2 --warmup 1 --no-cpu > $OUT/trktr.json 2> $OUT/trktr.txt || { echo "trace failed"; exit 1; }
grep "trk trace" $OUT/trktr.txt | tail -1
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/tr.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/tr.txt | tail -1
