#!/bin/bash
# traceOn parity + all GPU tests + trace/track/BA bench lines.  usage: tools/trace_check.sh TAG
TAG=${1:-trc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_trace.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_trace.txt 2>&1
rc=$?; echo "trace pytest rc=$rc"; tail -15 $OUT/pytest_trace.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "all gpu pytest rc=$rc"; tail -5 $OUT/pytest_gpu.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --workload trace --steps 20 --warmup 3 --cpu-seconds 6 > $OUT/bench_trace.json 2> $OUT/bench_trace.err || { echo "trace bench rc=$?"; tail -20 $OUT/bench_trace.err; exit 1; }
cat $OUT/bench_trace.json
timeout -k 10 200 python bench.py --workload track --steps 50 --warmup 3 --cpu-seconds 6 > $OUT/bench_track.json 2> $OUT/bench_track.err || { echo "track bench rc=$?"; tail -20 $OUT/bench_track.err; exit 1; }
cat $OUT/bench_track.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --workload trace --steps 20 --warmup 2 --no-cpu > $OUT/prof_trace.json 2> $OUT/prof_trace.err
echo "rocprof rc=$?"
cat $OUT/prof_trace/*kernel_stats.csv
