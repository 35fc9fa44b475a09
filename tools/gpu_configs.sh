#!/bin/bash
# Bench lines of the other BASELINE configs (C1, C2, C4, C5) with their CPU baselines:
#   tools/gpu_configs.sh [tag] [configs...]
cd "$GRAFT_REPO_ROOT" || exit 2
T=${1:-configs}; shift
out=gpurun_out/$T; mkdir -p $out
for cfg in ${@:-1 2 4 5}; do
  timeout -k 10 400 python bench.py --config $cfg --steps 200 --warmup 10 --cpu-seconds 10 > $out/bench_c$cfg.log 2>&1 || exit $?
  echo "C$cfg: $(tail -1 $out/bench_c$cfg.log | cut -c1-300)"
done
