#!/bin/bash
# Instruction mix and wave-cycle breakdown of the BA kernels (two SQ passes, kernel trace only).
# usage: tools/sq_pass.sh TAG POINTS
TAG=${1:-sq}; P=${2:-200000}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH"
B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
i=0
for C in "$A" "$B"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $OUT/pass$i -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu --points $P > $OUT/pass$i.json 2> $OUT/pass$i.err || { echo "pass $i failed rc=$?"; tail -20 $OUT/pass$i.err; exit 1; }
done
python3 $GRAFT_REPO_ROOT/tools/sq_summary.py $OUT > $OUT/sq.json && cat $OUT/sq.json
