#!/bin/bash
# hs_k_lin8 check: its GPU parity tests, then the BA bench at 2k / 20k / 200k points with hs_k_lin8 forced off / on.
# usage: tools/lin8_check.sh TAG   (outputs under gpurun_out/TAG/)
TAG=${1:-lin8}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_lin8.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_lin8.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|Error|assert" $OUT/pytest_lin8.txt | head -40
if [ $rc -gt 1 ]; then exit $rc; fi
for P in 2000 20000 200000; do
  for M in 0 1; do
    HS_LIN8=$M timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --points $P > $OUT/p${P}_l$M.json 2> $OUT/p${P}_l$M.err || { echo "bench $P $M failed"; tail -20 $OUT/p${P}_l$M.err; exit 1; }
    python3 -c "
import json,sys
d=json.loads(open('$OUT/p${P}_l$M.json').read().strip().splitlines()[-1])
print('P=$P lin8=$M', round(d['value']/1e6,1), 'Mpres/s', round(d['ms_per_step']*1e3,1), 'us/step lin', round(d['roofline']['avg_launch_ms']*1e3,2), 'us frac', round(d['roofline']['frac'],3))"
  done
done
