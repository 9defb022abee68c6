cd $GRAFT_REPO_ROOT && O=gpurun_out/$1 && mkdir -p $O
for V in 0 1 0 1; do
  HS_TRK_NOEVT=$V timeout -k 10 120 python bench.py --workload track --steps 100 --warmup 5 --no-cpu > $O/track_$V.json 2>$O/track_$V.err || exit 1
  python3 -c "import json;d=json.load(open('$O/track_$V.json'));print('noevt $V', round(d['ms_per_step'],4))"
done
