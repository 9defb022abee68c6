cd $GRAFT_REPO_ROOT && O=gpurun_out/$1; mkdir -p $O; shift
for VS in "$@"; do
  V=${VS%%:*}; E=""; [ "$VS" != "$V" ] && E=${VS#*:}
  env $E HS_KTRACE=1 HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_$V.so timeout -k 10 200 python bench.py --points 200000 --steps 3 --warmup 1 --no-cpu --no-phase-split --no-large-strong > $O/t_$V.json 2> $O/t_$V.err || exit 1
  echo "== $VS"; grep "hs trace] linearize" $O/t_$V.err | tail -22 | grep -v "cp2 \|span"
done
