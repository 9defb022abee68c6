#!/bin/bash
# HBM traffic per kernel from PMC counters (MI355X_MICROARCH.md "HBM/rocprofv3"): FETCH_SIZE and
# WRITE_SIZE in SEPARATE --pmc passes (FETCH_SIZE uses 3 TCC counters, WRITE_SIZE 2), kernel trace
# only, no sys/runtime trace.  usage: tools/pmc.sh TAG [bench args...]
TAG=${1:-pmc}; shift
ARGS=${@:---steps 20 --warmup 2 --no-cpu}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/$C -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/$C.json 2> $OUT/$C.err || { echo "pmc $C failed rc=$?"; tail -20 $OUT/$C.err; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT > $OUT/traffic.json && cat $OUT/traffic.json
