#!/bin/bash
# round-4 check: BA / window / shard / activation GPU tests, the headline bench, keyframe and activation benches
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r04_t1}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests/test_act.py tests/test_gpu_track.py tests/test_gpu_ba.py tests/test_gpu_window.py tests/test_gpu_shard.py -m gpu -x -v --timeout 180 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?
echo "pytest rc=$rc"; grep -cE "PASSED" $OUT/pytest_gpu.txt; grep -E "FAILED|Error|error" $OUT/pytest_gpu.txt | head -20
if [ $rc -gt 1 ]; then exit $rc; fi
HS_ACT_PROF=1 timeout -k 10 200 python bench.py --workload act --steps 10 --warmup 2 > $OUT/act.json 2> $OUT/act.err || { echo "act bench failed"; tail -20 $OUT/act.err; exit 1; }
tail -3 $OUT/act.err; head -c 1200 $OUT/act.json; echo
timeout -k 10 200 python bench.py --workload track --steps 50 --warmup 5 > $OUT/track.json 2> $OUT/track.err || { echo "track bench failed"; tail -20 $OUT/track.err; exit 1; }
head -c 800 $OUT/track.json; echo
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed rc=$?"; tail -30 $OUT/bench.err; exit 1; }
head -c 3000 $OUT/bench.json; echo
timeout -k 10 200 python bench.py --workload keyframe --steps 20 --warmup 3 > $OUT/kf.json 2> $OUT/kf.err || { echo "kf bench failed"; tail -20 $OUT/kf.err; exit 1; }
head -c 2500 $OUT/kf.json; echo
