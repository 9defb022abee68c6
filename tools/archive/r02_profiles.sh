#!/bin/bash
# Round-2 BA evidence: rocprofv3 kernel-trace --stats of the bench at the headline (C4 2k), 200k, and C5 (KITTI
# 2k / 20k); FETCH_SIZE / WRITE_SIZE passes at 2k and 200k (tools/r02_pmc.sh); the HBM stream micro benchmark.
# usage: tools/r02_profiles.sh TAG
TAG=${1:-prof}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
run_stats() {  # name, bench args...
  local NAME=$1; shift
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$NAME -o k -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu "$@" > $OUT/$NAME.json 2> $OUT/$NAME.err || { echo "stats $NAME failed"; tail -20 $OUT/$NAME.err; exit 1; }
  echo "== $NAME"; head -7 $(find $OUT/$NAME -name "*kernel_stats.csv")
}
run_stats ba2k --steps 200 --warmup 10
run_stats ba200k --steps 30 --warmup 3 --points 200000
run_stats kitti2k --workload ba-kitti --steps 200 --warmup 10
run_stats kitti20k --workload ba-kitti --steps 100 --warmup 5 --points 20000
bash $GRAFT_REPO_ROOT/tools/r02_pmc.sh $TAG/pmc 2000 200000 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -30 $OUT/pmc.log; exit 1; }
tail -5 $OUT/pmc.log
