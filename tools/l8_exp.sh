#!/bin/bash
# lin8 A/B at the large windows: variant libraries (h-slam_amd/lib/variants, `make variant`) at 200k and 2M points.
# usage: tools/l8_exp.sh TAG [variant[:ENV=value] ...]   (e.g. w8:HS_LIN8_BLOCKS=256)
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-l8}; mkdir -p $O; shift
for VS in ${@:-f0 f7}; do
  V=${VS%%:*}; E=""; [ "$VS" != "$V" ] && E=${VS#*:}
  for P in ${L8_POINTS:-200000 2000000}; do
    env $E HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_$V.so timeout -k 10 200 python bench.py --points $P --steps 20 --warmup 3 --no-cpu --no-phase-split --no-large-strong > $O/b_${V}_$P.json 2> $O/b_${V}_$P.err || { echo "bench $V $P failed"; tail -5 $O/b_${V}_$P.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_${V}_$P.json'));r=d['roofline'];print('$VS',$P,round(d['ms_per_step'],4),r.get('frac'),r.get('achieved'))"
  done
done
