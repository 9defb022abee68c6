#!/bin/bash
# round-3 batch 6: LDS-staged host-f terms in the solve, kernel-argument counter reset, zero-copy result readback --
# BA / stitch / shard / graph tests, the headline at the driver's 20 steps and at 300, chain trace
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r03_b6${1:-}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_stitch.py tests/test_gpu_shard.py tests/test_gpu_ba.py tests/test_gpu_window.py tests/test_gpu_c_caller.py tests/test_gpu_threshold.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest_ba.txt 2>&1
rc=$?; echo "ba tests rc=$rc"; grep -E "FAILED|ERROR" $OUT/pytest_ba.txt | head -5 | cut -c1-300; tail -2 $OUT/pytest_ba.txt
[ $rc -gt 1 ] && exit $rc
for s in 20 300; do
timeout -k 10 200 python bench.py --gpus 1 --steps $s --warmup 5 --no-cpu > $OUT/head$s.json 2> $OUT/head$s.err || { echo "bench failed"; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/head$s.json'));print('headline steps $s',round(d['ms_per_step']*1e3,2),'us/step',round(d['value']/1e6,1),'M pres/s')"
done
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/tr.txt || { echo "trace failed"; exit 1; }
grep "chain" $OUT/tr.txt | tail -1
