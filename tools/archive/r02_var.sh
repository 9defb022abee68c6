#!/bin/bash
# BA timing variants: kernel trace of the headline bench + HS_LIN_PPW sweep + point sweep (no CPU leg).
# usage: tools/r02_var.sh TAG
TAG=${1:-var}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
HS_KTRACE=1 timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu > $OUT/tr.json 2> $OUT/trace.txt || { echo "trace failed"; tail -20 $OUT/trace.txt; exit 1; }
grep "hs trace" $OUT/trace.txt | tail -24
for P in 1 2 4; do
  HS_LIN_PPW=$P timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu > $OUT/ppw$P.json 2> $OUT/ppw$P.err || { echo "ppw $P failed"; tail -20 $OUT/ppw$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/ppw$P.json'));print('ppw $P', round(d['value']/1e6,1), 'Mpres/s', round(d['ms_per_step']*1e3,2), 'us/step; lin', round(d['roofline']['avg_launch_ms']*1e3,2), 'us')"
done
for N in 20000 200000; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --points $N > $OUT/p$N.json 2> $OUT/p$N.err || { echo "points $N failed"; tail -20 $OUT/p$N.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/p$N.json'));print('points $N', round(d['value']/1e6,1), 'Mpres/s', round(d['ms_per_step']*1e3,2), 'us/step; lin', round(d['roofline']['avg_launch_ms']*1e3,2), 'us', round(d['roofline']['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o bench -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-cpu > $OUT/prof_bench.json 2> $OUT/prof_bench.err
echo "rocprof rc=$?"
find $OUT/prof -name "*kernel_stats*" -exec head -6 {} \;
