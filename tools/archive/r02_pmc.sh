#!/bin/bash
# HBM traffic per launch of the BA kernels at several window sizes (separate FETCH_SIZE / WRITE_SIZE passes, kernel
# trace only), the achievable-bandwidth micro benchmark, and a kernel-trace --stats profile at the largest size.
# usage: tools/r02_pmc.sh TAG [points...]     (default 2000 200000)
TAG=${1:-pmc}; shift
SIZES=${@:-2000 200000}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT/tools/micro && hipcc --offload-arch=gfx950 -O3 -o /tmp/hs_stream stream.hip && timeout -k 10 60 /tmp/hs_stream > $OUT/stream.jsonl || { echo "stream failed"; exit 1; }
cat $OUT/stream.jsonl
cd /tmp && export TMPDIR=/tmp
for P in $SIZES; do
  mkdir -p $OUT/p$P
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $C --output-format csv -d $OUT/p$P/$C -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --no-cpu --points $P > $OUT/p$P/$C.json 2> $OUT/p$P/$C.err || { echo "pmc $P $C failed rc=$?"; tail -20 $OUT/p$P/$C.err; exit 1; }
  done
  echo "pmc $P done"
done
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py --sizes $OUT $SIZES > $OUT/traffic.json && cat $OUT/traffic.json
LAST=${SIZES##* }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu --points $LAST > $OUT/stats_bench.json 2> $OUT/stats_bench.err || { echo "stats failed"; exit 1; }
find $OUT/stats -name "*kernel_stats*" -exec head -8 {} \;
