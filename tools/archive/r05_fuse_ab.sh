#!/bin/bash
# GPU tests of the iterate path, then the 200-step headline with and without the fused solve + linearize launch.
# usage: tools/fuse_ab.sh TAG
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-fz}; mkdir -p $O
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_ba.py tests/test_gpu_window.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
rc=$?; [ -n "$NOTEST" ] || tail -3 $O/pytest.txt; [ -n "$NOTEST" ] || [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for F in 1 0; do
    HS_FUSE_SL=$F timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu --no-phase-split --points ${P:-2000} > $O/b_${F}_$r.json 2>$O/b_${F}_$r.err || exit 1
    python3 -c "import json;d=json.load(open('$O/b_${F}_$r.json'));print('fuse=$F',round(d['ms_per_step']*1e3,2),'us')"
  done
done
HS_FUSE_SL=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu --no-phase-split > $O/b20.json 2>$O/b20.err || exit 1
python3 -c "import json;d=json.load(open('$O/b20.json'));print('fuse 20 steps',round(d['ms_per_step']*1e3,2),'us')"
