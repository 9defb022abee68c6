#!/bin/bash
# hs_k_lin against hs_k_lin8 at shard sizes (the strong-200k projection's per-rank step)
R=$GRAFT_REPO_ROOT
bash $R/tools/kstats.sh r06_sw2 "p25k_lin8||--points 25000 --steps 40 --warmup 5 --no-cpu" "p25k_lin|HS_LIN8=0|--points 25000 --steps 40 --warmup 5 --no-cpu" "p12k_lin8||--points 12500 --steps 40 --warmup 5 --no-cpu" "p12k_lin|HS_LIN8=0|--points 12500 --steps 40 --warmup 5 --no-cpu"
