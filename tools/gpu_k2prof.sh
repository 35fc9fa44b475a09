#!/bin/bash
# K2 per-wave profile only (no test suite): tools/gpu_k2prof.sh [tag] [configs...]
cd "$GRAFT_REPO_ROOT" || exit 2
T=${1:-k2prof}; shift
mkdir -p gpurun_out/$T
for cfg in ${@:-3}; do
  rm -f /tmp/k2prof_c$cfg.bin
  SR_K2_PROFILE="/tmp/k2prof_c$cfg.bin" timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 \
    --e2e-reps 0 --no-cpu-baseline > gpurun_out/$T/bench_prof_c$cfg.log 2>&1 || exit $?
  python tools/k2_profile.py /tmp/k2prof_c$cfg.bin > gpurun_out/$T/k2prof_c$cfg.txt 2>&1
  echo "== C$cfg"; cat gpurun_out/$T/k2prof_c$cfg.txt; rm -f /tmp/k2prof_c$cfg.bin
done
