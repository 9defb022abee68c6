#!/bin/bash
# Per-kernel rocprofv3 stats (kernel trace only, no counters) + the bench line for a few runs.
# usage: tools/kstats.sh TAG "NAME|ENV ASSIGNMENTS|bench args" ...
#   e.g. tools/kstats.sh r06_k1 "p200k|HS_TH_BESIDE=0|--points 200000 --steps 20 --warmup 3 --no-cpu"
# Outputs gpurun_out/TAG/NAME/{bench.json,bench.err,prof/...kernel_stats.csv}; prints value, step and the top kernels.
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for SPEC in "$@"; do
  NAME=${SPEC%%|*}; REST=${SPEC#*|}; ENVS=${REST%%|*}; ARGS=${REST#*|}
  D=$OUT/$NAME; mkdir -p $D
  env $ENVS timeout -k 10 200 python3 $GRAFT_REPO_ROOT/bench.py $ARGS > $D/bench.json 2> $D/bench.err || { echo "$NAME bench failed rc=$?"; tail -20 $D/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$D/bench.json'));print('$NAME', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step', {k: round(v*1e3,2) for k, v in (d.get('phase_ms_per_step') or {}).items() if isinstance(v, float)})"
  # the profiler preloads into the program itself: the environment goes through `env` BEFORE rocprofv3, never after --
  env $ENVS timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $D/prof -o k -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS --no-phase-split > $D/prof.json 2> $D/prof.err || { echo "$NAME rocprof failed rc=$?"; tail -20 $D/prof.err; exit 1; }
  F=$(find $D/prof -name "*kernel_stats.csv" | head -1)
  python3 - "$F" <<'EOF'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:9]:
    print("   %-28s calls %6s avg %8.2f us  %5.1f%%" % (r["Name"][:28], r["Calls"], float(r["AverageNs"]) / 1e3, float(r["Percentage"])))
EOF
done
