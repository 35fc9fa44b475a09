#!/bin/bash
# K2 per-wave profiles of one config under two environment settings:
#   tools/gpu_k2prof_ab.sh tag config "ENV=a" "ENV=b"
cd "$GRAFT_REPO_ROOT" || exit 2
T=$1; cfg=$2; shift 2
mkdir -p gpurun_out/$T
i=0
for arm in "$@"; do
  i=$((i + 1))
  rm -f /tmp/k2prof_ab.bin
  env $arm SR_K2_PROFILE=/tmp/k2prof_ab.bin timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 \
    --e2e-reps 0 --no-cpu-baseline ${K2AB_ARGS:-} > gpurun_out/$T/bench_$i.log 2>&1 || exit $?
  python tools/k2_profile.py /tmp/k2prof_ab.bin > gpurun_out/$T/k2prof_$i.txt 2>&1
  echo "== $arm"; head -22 gpurun_out/$T/k2prof_$i.txt; rm -f /tmp/k2prof_ab.bin
done
