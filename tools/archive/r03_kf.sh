cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03_kf1
timeout -k 10 300 python bench.py --workload keyframe --steps 10 --warmup 2 --no-cpu > gpurun_out/r03_kf1/kf.json 2> gpurun_out/r03_kf1/kf.err
echo rc=$?; tail -5 gpurun_out/r03_kf1/kf.err; cat gpurun_out/r03_kf1/kf.json
