#!/bin/bash
# round-3 batch 3: the whole GPU suite (threshold beside the solve, tracker granule meeting), lin / lin8 crossover at
# 5k / 10k, the C2 track line + phase trace, the headline + chain trace
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_b3
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_gpu.txt | head -5 | cut -c1-300; tail -2 $OUT/pytest_gpu.txt
[ $rc -gt 1 ] && exit $rc
for P in 2000 5000 10000; do
  for L in 0 1; do
    HS_LIN8=$L timeout -k 10 200 python bench.py --points $P --steps 100 --warmup 5 --no-cpu > $OUT/p${P}_l$L.json 2> $OUT/p${P}_l$L.err || { echo "p$P lin8=$L failed"; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/p${P}_l$L.json'));print('$P lin8=$L',round(d['ms_per_step']*1e3,1),'us/step lin',round(d['roofline']['avg_launch_ms']*1e3,1), d['roofline']['kernel'])"
  done
done
timeout -k 10 200 python bench.py --workload track --steps 20 --warmup 3 --no-cpu > $OUT/trk.json 2> $OUT/trk.err || { echo "track failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/trk.json'));print('track',round(d['ms_per_step'],4),'ms device',round(d['config']['device_ms_per_track'],4))"
HS_KTRACE=1 timeout -k 10 200 python bench.py --workload track --steps 2 --warmup 1 --no-cpu > $OUT/trktr.json 2> $OUT/trktr.txt || { echo "trace failed"; exit 1; }
grep "trk trace" $OUT/trktr.txt | tail -1
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/head$r.json 2> $OUT/head$r.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/head$r.json'));print('headline',round(d['ms_per_step']*1e3,2),'us/step',round(d['value']/1e6,1),'M pres/s')"
done
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/tr.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/tr.txt | tail -1
HS_LIN_PPW=2 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/ppw2.json 2> $OUT/ppw2.err || { echo "ppw2 failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/ppw2.json'));print('ppw2',round(d['ms_per_step']*1e3,2),'us/step lin',round(d['roofline']['avg_launch_ms']*1e3,2))"
HS_LIN_PPW=2 HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/trppw2.json 2> $OUT/trppw2.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/trppw2.txt | tail -1
HS_LIN8=1 HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/trl8.json 2> $OUT/trl8.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/trl8.txt | tail -1
