#!/bin/bash
# HBM traffic per launch of the kernels as they stand, per workload key (separate FETCH_SIZE / WRITE_SIZE rocprofv3
# passes, kernel trace only): C4 windows of N points, "kitti<N>" (--workload ba-kitti), "trace", "track".
# usage: tools/r03_pmc.sh TAG [keys...]
TAG=${1:-pmc}; shift
KEYS=${@:-2000 20000 200000 2000000 kitti2000 trace track}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for K in $KEYS; do
  case $K in
    kitti*) ARGS="--workload ba-kitti --points ${K#kitti} --steps 10 --warmup 2 --no-cpu" ;;
    trace|track) ARGS="--workload $K --steps 5 --warmup 1 --no-cpu" ;;
    *) ARGS="--points $K --steps 10 --warmup 2 --no-cpu" ;;
  esac
  mkdir -p $OUT/p$K
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 170 rocprofv3 --pmc $C --output-format csv -d $OUT/p$K/$C -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$K/$C.json 2> $OUT/p$K/$C.err || { echo "pmc $K $C failed rc=$?"; tail -20 $OUT/p$K/$C.err; exit 1; }
  done
  echo "pmc $K done"
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py --sizes $OUT $KEYS > $OUT/traffic.json && head -c 3000 $OUT/traffic.json
