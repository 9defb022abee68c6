#!/bin/bash
# solve-kernel trace + points sweep (linearize roofline regime).  usage: tools/sweep.sh TAG
TAG=${1:-sweep}
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG
HS_KTRACE=1 timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/$TAG/tr.json 2> gpurun_out/$TAG/trace.txt || exit 1
grep "hs trace" gpurun_out/$TAG/trace.txt | tail -24
for P in 2000 20000 200000; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 3 --no-cpu --points $P > gpurun_out/$TAG/p$P.json 2> gpurun_out/$TAG/p$P.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/$TAG/p$P.json'));print($P, d['config']['point_residuals'], round(d['value']/1e6,1), 'Mpres/s', round(d['ms_per_step'],4), 'ms/step lin', round(d['roofline']['avg_launch_ms'],4), 'ms', round(d['roofline']['achieved'],1), 'GB/s')"
done
