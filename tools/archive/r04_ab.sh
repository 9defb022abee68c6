#!/bin/bash
# A/B of an experiment flag on the headline step: parity tests with the flag, then bench with / without it
# usage: tools/r04_ab.sh TAG VAR=VALUE [pytest -k expr]
TAG=$1; FLAG=$2; K=${3:-"solve or optimize or step or graph"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
if [ -x tools/micro/ldlt_wave ]; then timeout -k 10 60 tools/micro/ldlt_wave > $OUT/ldlt_wave.txt 2>&1; echo "ldlt_wave rc=$?"; cat $OUT/ldlt_wave.txt; fi
env $FLAG timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py -m gpu -x -v --timeout 180 --timeout-method thread -k "$K" > $OUT/pytest_flag.txt 2>&1
rc=$?
echo "pytest(flag) rc=$rc"; grep -cE "PASSED" $OUT/pytest_flag.txt; grep -E "FAILED|Error" $OUT/pytest_flag.txt | head -10
if [ $rc -gt 1 ]; then exit $rc; fi
FLAG2=${4:-}
for rep in 1 2; do
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/base$rep.json 2> $OUT/base$rep.err || { echo "bench failed"; tail -5 $OUT/base$rep.err; exit 1; }
  env $FLAG timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/flag$rep.json 2> $OUT/flag$rep.err || { echo "bench(flag) failed"; tail -5 $OUT/flag$rep.err; exit 1; }
  if [ -n "$FLAG2" ]; then env $FLAG2 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/flagb$rep.json 2> $OUT/flagb$rep.err || { echo "bench(flag2) failed"; exit 1; }; fi
done
for f in $OUT/base1.json $OUT/flag1.json $OUT/flagb1.json $OUT/base2.json $OUT/flag2.json $OUT/flagb2.json; do [ -f $f ] || continue; python3 -c "
import json,sys; r=json.load(open('$f')); print('$f'.split('/')[-1], round(r['ms_per_step']*1e3,2), 'us/step', {k: round(v*1e3,2) for k,v in r['phase_ms_per_step'].items() if isinstance(v,float)}, r.get('calls_ms'))"; done
