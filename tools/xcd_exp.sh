# A/B of the XCD-aware linearize block order (HS_XCD=0/1) at 2k / 200k / 2M, plus a FETCH_SIZE pass at 200k
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-xcd} && mkdir -p $O
for P in 2000 200000 2000000; do
  for X in 0 1; do
    HS_XCD=$X timeout -k 10 200 python bench.py --points $P --steps 30 --warmup 3 --no-cpu --no-phase-split > $O/p${P}_x$X.json 2>$O/p${P}_x$X.err || { echo "bench $P $X failed"; tail -5 $O/p${P}_x$X.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/p${P}_x$X.json'));r=d['roofline'];print('$P xcd=$X', round(d['ms_per_step']*1e3,2),'us/step', r['kernel'], round(r['avg_launch_ms']*1e3,2),'us frac', round(r['frac'],3))"
  done
done
cd /tmp && export TMPDIR=/tmp
for X in 0 1; do
  HS_XCD=$X timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE --output-format csv -d $GRAFT_REPO_ROOT/$O/pmc_x$X -o pmc -- python3 $GRAFT_REPO_ROOT/bench.py --points 200000 --steps 10 --warmup 2 --no-cpu --no-phase-split > $GRAFT_REPO_ROOT/$O/pmc_x$X.json 2> $GRAFT_REPO_ROOT/$O/pmc_x$X.err || { echo "pmc $X failed"; exit 1; }
done
echo done
