# A/B of the step + in-kernel chain trace.  usage: tools/kexp.sh TAG [variants: B D16 D32]
cd $GRAFT_REPO_ROOT && O=gpurun_out/${1:-r05_k1} && mkdir -p $O; shift
for V in ${@:-B}; do
  unset HS_SOLVE_DBG HS_LIN_PPW HSLAM_AMD_LIB
  case $V in B) ;; D16) export HS_SOLVE_DBG=16;; D32) export HS_SOLVE_DBG=32;; PPW2) export HS_LIN_PPW=2;; lib_*) export HSLAM_AMD_LIB=h-slam_amd/lib/variants/libhslam_amd_${V#lib_}.so;; esac
  timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu --no-phase-split > $O/b_$V.json 2>$O/b_$V.err || exit 1
  HS_KTRACE=1 timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu --no-phase-split > $O/t_$V.json 2>$O/t_$V.err || exit 1
  python3 -c "import json;d=json.load(open('$O/b_$V.json'));print('$V',d['value'],d['ms_per_step']*1e3)"
  grep "hs trace" $O/t_$V.err | tail -40 | grep "solve\|chain\|linearize"
done
