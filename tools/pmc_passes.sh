#!/bin/bash
# Round-4 roof evidence per workload key: three rocprofv3 passes (each with --kernel-trace --stats only beside the
# counters), then tools/pmc_roof.py: HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE), DRAM GB/s over the
# kernel-trace duration, and the SQ issue / wait split (VALU busy per SIMD, wave-cycle fractions).
# keys: C4 point counts (2000 20000 200000 2000000), kitti<N>, trace, track
# usage: tools/pmc_passes.sh TAG [keys...]
TAG=${1:-pmc}; shift
KEYS=${@:-2000 200000 2000000 trace}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || echo "counter list rc=$?"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
for K in $KEYS; do
  case $K in
    kitti*) ARGS="--workload ba-kitti --points ${K#kitti} --steps 10 --warmup 2 --no-cpu --no-phase-split" ;;
    trace|track) ARGS="--workload $K --steps 5 --warmup 1 --no-cpu" ;;
    *) ARGS="--points $K --steps 10 --warmup 2 --no-cpu --no-phase-split" ;;
  esac
  mkdir -p $OUT/p$K
  for P in FETCH_SIZE WRITE_SIZE SQ; do
    C=$P; [ $P = SQ ] && C=$SQ
    timeout -s KILL 170 rocprofv3 --kernel-trace --stats --pmc $C --output-format csv -d $OUT/p$K/$P -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $OUT/p$K/$P.json 2> $OUT/p$K/$P.err || { echo "pmc $K $P failed rc=$?"; tail -20 $OUT/p$K/$P.err; exit 1; }
  done
  echo "pmc $K done"
done
python3 $GRAFT_REPO_ROOT/tools/pmc_roof.py $OUT $KEYS > $OUT/roof.json && head -c 4000 $OUT/roof.json
