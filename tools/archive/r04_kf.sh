#!/bin/bash
# keyframe path: window tests, keyframe bench with per-call times
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_kf}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests/test_gpu_window.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_window.txt 2>&1
rc=$?; tail -2 $OUT/pytest_window.txt; grep -E "FAILED|Error" $OUT/pytest_window.txt | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --workload keyframe --steps 20 --warmup 3 --no-cpu > $OUT/kf.json 2> $OUT/kf.err || { echo "kf bench failed"; tail -20 $OUT/kf.err; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/kf.json')); print('kf', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d['phase_ms_per_keyframe'].items()})
print({k: round(v,3) for k,v in d['call_ms_per_keyframe'].items()})"
