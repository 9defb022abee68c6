#!/bin/bash
# headline + C5 bench lines with their CPU baselines, and the 2M-point sweep line (no CPU leg)
OUT=$GRAFT_REPO_ROOT/gpurun_out/${1:-r02_cpu}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 200 --warmup 10 > $OUT/ba.json 2> $OUT/ba.err || { echo "ba failed"; tail $OUT/ba.err; exit 1; }
echo "ba done"
timeout -k 10 300 python bench.py --workload ba-kitti --steps 200 --warmup 10 > $OUT/kitti.json 2> $OUT/kitti.err || { echo "kitti failed"; tail $OUT/kitti.err; exit 1; }
echo "kitti done"
timeout -k 10 500 python -u bench.py --points 2000000 --steps 5 --warmup 1 --no-cpu > $OUT/p2m.json 2> $OUT/p2m.err || { echo "2M failed"; tail $OUT/p2m.err; exit 1; }
echo "2M done"
