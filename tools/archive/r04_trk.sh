#!/bin/bash
# tracker: parity tests, then the C2 track line per HS_TRK_SOLVE (0 = Gauss-Jordan on 64 lanes, 1 = Eigen-order
# LDLT on 8 row lanes) and per member count HS_TRK_G, and the phase trace
TAG=${1:-r04_trk}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_track.py -v --timeout 120 --timeout-method thread > $OUT/pytest_trk.txt 2>&1
rc=$?; echo "track tests rc=$rc"; grep -E "PASSED|FAILED|ERROR" $OUT/pytest_trk.txt | tail -25 | cut -c1-150
[ $rc -gt 1 ] && exit $rc
for V in S0 Z0 S1 G4 G12 G16 S0 Z0; do
  case $V in S*) export HS_TRK_SOLVE=${V#S} HS_TRK_ZC=1; unset HS_TRK_G ;; Z*) export HS_TRK_SOLVE=0 HS_TRK_ZC=0; unset HS_TRK_G ;; G*) export HS_TRK_SOLVE=0 HS_TRK_ZC=1 HS_TRK_G=${V#G} ;; esac
  timeout -k 10 200 python bench.py --workload track --steps 30 --warmup 3 --no-cpu > $OUT/trk$V.json 2> $OUT/trk$V.err || { echo "track $V failed"; tail -5 $OUT/trk$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/trk$V.json'));print('$V',round(d['ms_per_step'],4),'ms/track device',round(d['config']['device_ms_per_track'],4), 'passes', d['config']['passes'])"
done
unset HS_TRK_G
for S in 0; do
  HS_TRK_SOLVE=$S HS_KTRACE=1 timeout -k 10 200 python bench.py --workload track --steps 2 --warmup 1 --no-cpu > $OUT/trktr$S.json 2> $OUT/trktr$S.txt || { echo "trace failed"; exit 1; }
  grep "trk trace" $OUT/trktr$S.txt | tail -2
done
