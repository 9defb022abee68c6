#!/bin/bash
# full GPU suite, then the track / keyframe / headline lines
TAG=${1:-r04_v2}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.txt | tail -8 | cut -c1-200
[ $rc -ne 0 ] && exit $rc
for W in track keyframe; do
  timeout -k 10 300 python bench.py --workload $W > $OUT/bench_$W.json 2> $OUT/bench_$W.err || { echo "bench $W failed"; tail -5 $OUT/bench_$W.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$W.json'));print('$W',d['value'],d['unit'],round(d['ms_per_step'],4),'ms', d.get('cpu_baseline',{}).get('value'))"
done
