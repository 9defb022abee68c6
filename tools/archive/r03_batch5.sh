#!/bin/bash
# round-3 batch 5: stitch split (diagonal host-f Schur blocks) -- BA / stitch / shard / lin8 tests, the headline +
# chain trace, tracker G sweep
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_b5
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_stitch.py tests/test_gpu_shard.py tests/test_gpu_ba.py tests/test_gpu_window.py tests/test_gpu_lin8.py tests/test_gpu_c_caller.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_ba.txt 2>&1
rc=$?; echo "ba tests rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_ba.txt | head -5 | cut -c1-300; tail -2 $OUT/pytest_ba.txt
[ $rc -gt 1 ] && exit $rc
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-cpu > $OUT/head$r.json 2> $OUT/head$r.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/head$r.json'));print('headline',round(d['ms_per_step']*1e3,2),'us/step',round(d['value']/1e6,1),'M pres/s')"
done
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/tr.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/tr.txt | tail -1
for G in 4 8 16; do
  HS_TRK_G=$G timeout -k 10 200 python bench.py --workload track --steps 20 --warmup 3 --no-cpu > $OUT/trk$G.json 2> $OUT/trk$G.err || { echo "track failed"; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/trk$G.json'));print('track G=$G',round(d['ms_per_step'],4),'ms device',round(d['config']['device_ms_per_track'],4))"
done
