#!/bin/bash
# round-1 first GPU check: smoke, bench, gpu tests, rocprof kernel trace
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.txt 2>&1 || { echo "smoke failed rc=$?"; cat gpurun_out/smoke.txt | tail -30; exit 1; }
cat gpurun_out/smoke.txt | tail -3
timeout -k 10 400 python bench.py --steps 30 --warmup 5 --cpu-seconds 5 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.txt
if [ $rc -gt 1 ]; then exit $rc; fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --no-cpu > $GRAFT_REPO_ROOT/gpurun_out/prof_bench.json 2> $GRAFT_REPO_ROOT/gpurun_out/prof_bench.err
echo "rocprof rc=$?"
find $GRAFT_REPO_ROOT/gpurun_out/prof_r01 -name "*stats*" | head
