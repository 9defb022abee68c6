#!/bin/bash
# multi-workgroup tracker: parity tests, then the C2 track line at HS_TRK_G = 1 / default, with the phase trace
TAG=${1:-r03_trk}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
HS_TRK_G=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_track.py -v --timeout 120 --timeout-method thread > $OUT/pytest_trk.txt 2>&1
rc=$?; echo "track tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_trk.txt | tail -25 | cut -c1-150
[ $rc -gt 1 ] && exit $rc
for G in 1 32 8 16; do
  HS_TRK_G=$G timeout -k 10 200 python bench.py --workload track --steps 20 --warmup 3 --no-cpu > $OUT/trk$G.json 2> $OUT/trk$G.err || { echo "track G=$G failed"; tail -5 $OUT/trk$G.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/trk$G.json'));print('G=$G',round(d['ms_per_step'],4),'ms/track device',round(d['config']['device_ms_per_track'],4), 'passes', d['config']['passes'])"
  HS_TRK_G=$G HS_KTRACE=1 timeout -k 10 200 python bench.py --workload track --steps 2 --warmup 1 --no-cpu > $OUT/trktr$G.json 2> $OUT/trktr$G.txt || { echo "trace failed"; exit 1; }
  grep "trk trace" $OUT/trktr$G.txt | tail -1
done
