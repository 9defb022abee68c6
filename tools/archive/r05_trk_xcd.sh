cd $GRAFT_REPO_ROOT && O=gpurun_out/$1 && mkdir -p $O; shift
for V in "$@"; do
  X=${V%%:*}; M=${V#*:}
  HS_TRK_SPIN=${SPIN:-2000000} HS_TRK_XCD=$X HS_TRK_MEET=$M timeout -k 10 120 python bench.py --workload track --steps 50 --warmup 5 --no-cpu > $O/track_$X$M.json 2>$O/track_$X$M.err || { echo "track $V failed"; tail -5 $O/track_$X$M.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/track_$X$M.json'));print('xcd:meet $V', round(d['ms_per_step'],4), 'ms  device', round(d['config']['device_ms_per_track'],4))"
  HS_TRK_SPIN=${SPIN:-2000000} HS_KTRACE=1 HS_TRK_XCD=$X HS_TRK_MEET=$M timeout -k 10 120 python bench.py --workload track --steps 3 --warmup 1 --no-cpu > $O/trace_$X$M.json 2>$O/trace_$X$M.err || exit 1
  grep "trk trace" $O/trace_$X$M.err | tail -1
done
