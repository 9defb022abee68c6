#!/bin/bash
# HS_SYNC_POLL A/B (1 = event polling, the default; 0 = hipStreamSynchronize) over the per-call bench lines,
# after the full GPU suite
TAG=${1:-r04_sync}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; grep -E "passed|failed|FAILED|ERROR" $OUT/pytest_gpu.txt | tail -8 | cut -c1-200
[ $rc -ne 0 ] && exit $rc
for P in 1 0 1 0; do
  for W in track keyframe act trace refine select; do
    HS_SYNC_POLL=$P timeout -k 10 300 python bench.py --workload $W --no-cpu > $OUT/b_${W}_$P.json 2> $OUT/b_${W}_$P.err || { echo "bench $W failed"; tail -5 $OUT/b_${W}_$P.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/b_${W}_$P.json'));print('P=$P $W',round(d['value'],1),d['unit'],round(d['ms_per_step'],4),'ms')"
  done
done
