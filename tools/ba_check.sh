#!/bin/bash
# BA parity tests + per-phase kernel trace + short bench.  usage: tools/ba_check.sh TAG
TAG=${1:-bac}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
timeout -k 10 300 python -u -m pytest tests/test_gpu_ba.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/$TAG/pytest.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/$TAG/pytest.txt; [ $rc -ne 0 ] && exit $rc
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/$TAG/tr.json 2> gpurun_out/$TAG/trace.txt || exit 1
grep "hs trace" gpurun_out/$TAG/trace.txt | tail -24
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu > gpurun_out/$TAG/b.json 2> gpurun_out/$TAG/b.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/$TAG/b.json'));print(round(d['value']/1e6,2), 'Mpres/s', round(d['ms_per_step']*1e3,2), 'us/step; lin', round(d['roofline']['avg_launch_ms']*1e3,2), 'us')"
