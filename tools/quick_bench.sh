#!/bin/bash
# quick GPU timing: tests + bench with and without per-kernel HIP events + trace
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/qb
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/qb/pytest.txt 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/qb/pytest.txt
timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu > gpurun_out/qb/ev.json 2>gpurun_out/qb/ev.err || exit 1
HS_EVENT_TIMING=0 timeout -k 10 200 python bench.py --steps 200 --warmup 10 --no-cpu > gpurun_out/qb/noev.json 2>gpurun_out/qb/noev.err || exit 1
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/qb/tr.json 2> gpurun_out/qb/trace.txt || exit 1
python3 -c "
import json
for f in ('ev','noev'):
    d=json.load(open('gpurun_out/qb/%s.json'%f)); print(f, d['value'], d['ms_per_step'], d['phase_ms_per_step'])"
grep "hs trace" gpurun_out/qb/trace.txt | tail -24
