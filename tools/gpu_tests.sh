#!/bin/bash
# Selected GPU tests, then a short headline bench.  usage: tools/gpu_tests.sh TAG [pytest selectors...]
TAG=${1:-t}; shift
SEL=${@:-tests}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 120 --timeout-method thread > $OUT/pytest.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|PASS|FAIL|Error|relinearized" $OUT/pytest.txt | tail -40
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['ms_per_step'],d.get('phase_ms_per_step'))"
exit $rc
