#!/bin/bash
# BA-focused GPU check: smoke -> pytest tests/test_gpu_ba.py -> bench ba + ba-kitti -> rocprofv3 kernel stats.
# usage: tools/r02_ba.sh TAG [pytest -k expr]   (outputs under gpurun_out/TAG/)
TAG=${1:-ba}
KEXPR=${2:-}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { echo "smoke failed rc=$?"; tail -30 $OUT/smoke.txt; exit 1; }
tail -2 $OUT/smoke.txt
if [ -n "$KEXPR" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" > $OUT/pytest_ba.txt 2>&1
else
  timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py -m gpu -v --timeout 120 --timeout-method thread > $OUT/pytest_ba.txt 2>&1
fi
rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" $OUT/pytest_ba.txt | tail -40
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --cpu-seconds 6 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json; echo
timeout -k 10 300 python bench.py --workload ba-kitti --steps 50 --warmup 5 --cpu-seconds 6 > $OUT/bench_kitti.json 2> $OUT/bench_kitti.err || { echo "bench kitti failed rc=$?"; tail -30 $OUT/bench_kitti.err; exit 1; }
cat $OUT/bench_kitti.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "rocprof rc=$?"
find $OUT/prof -name "*kernel_stats*" -exec head -8 {} \;
