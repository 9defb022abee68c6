#!/bin/bash
# accumulate split-size sweep: HS_ACC_SPLIT_POINTS in {64, 32, 16, 8}; trace + bench per setting
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/split
for SP in 64 32 16 8; do
  HS_ACC_SPLIT_POINTS=$SP HS_KTRACE=1 timeout -k 10 120 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/split/tr$SP.json 2> gpurun_out/split/tr$SP.txt || exit 1
  HS_ACC_SPLIT_POINTS=$SP timeout -k 10 120 python bench.py --steps 200 --warmup 10 --no-cpu > gpurun_out/split/b$SP.json 2> gpurun_out/split/b$SP.err || exit 1
  echo "split $SP: $(python3 -c "import json;d=json.load(open('gpurun_out/split/b$SP.json'));print(round(d['ms_per_step']*1e3,2),'us/step')") $(grep -E 'accumulate   blocks|stitch       blocks' gpurun_out/split/tr$SP.txt | tr '\n' ' ')"
done
