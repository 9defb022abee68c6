#!/bin/bash
# GPU check of the BA / tracker paths after a kernel change: the parity suites named in $2 (default: BA + lin8 +
# tracker), then the headline bench, the C2 tracker line and the 20k / 200k sweep points.
# usage: tools/ba_suite.sh TAG ["test files"]
TAG=${1:-suite}
TESTS=${2:-"tests/test_gpu_ba.py tests/test_gpu_lin8.py tests/test_gpu_threshold.py tests/test_gpu_stitch.py tests/test_gpu_track.py"}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "FAIL|ERROR|Error|assert|passed|failed" $OUT/pytest.txt | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --steps 100 --warmup 5 --no-cpu > $OUT/b2k.json 2> $OUT/b2k.err || { echo "bench failed"; tail -20 $OUT/b2k.err; exit 1; }
timeout -k 10 200 python bench.py --workload track --steps 20 --warmup 3 --no-cpu > $OUT/track.json 2> $OUT/track.err || { echo "bench track failed"; tail -20 $OUT/track.err; exit 1; }
for P in 20000 200000; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --points $P > $OUT/p$P.json 2> $OUT/p$P.err || { echo "bench $P failed"; tail -20 $OUT/p$P.err; exit 1; }
done
python3 - <<PY
import json
for f in ['b2k','p20000','p200000','track']:
    d=json.loads(open('$OUT/%s.json'%f).read().strip().splitlines()[-1])
    r=d.get('roofline') or {}
    print(f, round(d['value'],1), d['unit'], round(d['ms_per_step']*1e3,2), 'us/step; kernel', round((r.get('avg_launch_ms') or 0)*1e3,2), 'us frac', round(r.get('frac') or 0,4))
PY
