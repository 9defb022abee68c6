#!/bin/bash
# activation tests + bench, then the PMC roof passes (tools/r04_pmc.sh)
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_t3}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_act.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest_act.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -cE "PASSED" $OUT/pytest_act.txt; grep -E "FAILED|Error" $OUT/pytest_act.txt | head -10
if [ $rc -ne 0 ]; then exit $rc; fi
HS_ACT_PROF=1 timeout -k 10 200 python bench.py --workload act --steps 10 --warmup 2 > $OUT/act.json 2> $OUT/act.err || { echo "act bench failed"; tail -20 $OUT/act.err; exit 1; }
tail -2 $OUT/act.err; python3 -c "import json;d=json.load(open('$OUT/act.json'));print('act',round(d['ms_per_step'],3),'ms',d.get('speedup_vs_cpu'))"
bash tools/r04_pmc.sh ${2:-r04_pmc} 2000 200000 2000000 trace
