#!/bin/bash
# per-rank step of a point shard at the strong-200k projection's sizes (the MFMA Schur build)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_sw3; mkdir -p $O
for P in 25000 50000 100000 200000; do
  timeout -k 10 200 python3 $R/bench.py --points $P --steps 40 --warmup 5 --no-cpu > $O/p$P.json 2> $O/p$P.err || { echo "$P failed"; tail -5 $O/p$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/p$P.json'));print($P, round(d['ms_per_step']*1e3,1),'us/step', round(d['roofline']['avg_launch_ms']*1e3,1), 'us lin8', {k: round(v*1e3,1) for k,v in d['phase_ms_per_step'].items() if isinstance(v,float)})"
done
