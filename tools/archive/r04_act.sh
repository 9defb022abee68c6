#!/bin/bash
# activation: GPU tests, bench with the in-kernel profile, rocprofv3 kernel stats
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_act}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_act.py -m gpu -x -q --timeout 180 --timeout-method thread > $OUT/pytest_act.txt 2>&1
rc=$?; tail -2 $OUT/pytest_act.txt; grep -E "FAILED|Error" $OUT/pytest_act.txt | head -5
if [ $rc -ne 0 ]; then exit $rc; fi
HS_ACT_PROF=1 timeout -k 10 200 python bench.py --workload act --steps 10 --warmup 2 > $OUT/act.json 2> $OUT/act.err || { echo "act bench failed"; tail -20 $OUT/act.err; exit 1; }
tail -2 $OUT/act.err; python3 -c "import json;d=json.load(open('$OUT/act.json'));print('act',round(d['ms_per_step'],3),'ms',d.get('speedup_vs_cpu'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o act -- python3 $GRAFT_REPO_ROOT/bench.py --workload act --steps 10 --warmup 2 --no-cpu > /dev/null 2>&1
find $OUT/prof -name "*kernel_stats.csv" -exec head -8 {} \;
