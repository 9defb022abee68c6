# tracker A/B over HS_TRK_GMIN (levels below it run on one member).  usage: tools/trk_exp.sh TAG [values...]
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-trk} && mkdir -p $O; shift
for V in ${@:-0 4096}; do
  HS_TRK_GMIN=$V timeout -k 10 120 python bench.py --workload track --steps 50 --warmup 5 --no-cpu > $O/track_$V.json 2>$O/track_$V.err || { echo "track $V failed"; tail -5 $O/track_$V.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/track_$V.json'));print('gmin $V', round(d['ms_per_step'],4), 'ms  device', round(d['config']['device_ms_per_track'],4), 'passes', d['config']['passes'])"
done
for V in ${TRACE_GMIN:-}; do
  HS_KTRACE=1 HS_TRK_GMIN=$V timeout -k 10 120 python bench.py --workload track --steps 3 --warmup 1 --no-cpu > $O/trace_$V.json 2>$O/trace_$V.err || exit 1
  echo "gmin $V"; grep "trk trace" $O/trace_$V.err | tail -2
done
