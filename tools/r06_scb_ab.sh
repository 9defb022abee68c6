#!/bin/bash
# hs_k_lin8 variants interleaved, launch durations: the Schur MFMA tiles in batches of 1 / 5 / 10 (L8_SC_BATCH: b1 / b5 / b10), then b5 against t4 (the T slice as lane-consecutive float4s)
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r06_scb; mkdir -p $O
for P in 200000 2000000; do
 for V in b5 t4 b5 t4; do
  echo -n "$V "; HSLAM_AMD_LIB=$R/h-slam_amd/lib/variants/libhslam_amd_$V.so timeout -k 10 200 python3 $R/tools/lin8_time.py $P 64 2> $O/${V}_$P.err || { echo "$V $P failed"; tail -5 $O/${V}_$P.err; exit 1; }
 done
done
