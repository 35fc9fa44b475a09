#!/bin/bash
# rocprof kernel stats of the C3 steady tick: K0-less runs vs K0 on every run (SR_K0_SKIP=0)
#   tools/gpu_k0skip_prof.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/k0skip"; mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for arm in skip noskip; do
  case $arm in
    skip) env_=""; args="";;
    noskip) env_="SR_K0_SKIP=0"; args="";;
    cold) env_=""; args="--tick cold";;
  esac
  if [ $arm = noskip ]; then export SR_K0_SKIP=0; else unset SR_K0_SKIP; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof_$arm" -o run --output-format csv -- \
    python3 "$R/bench.py" --config 3 --steps 400 --warmup 10 --no-cpu-baseline --e2e-reps 0 $args > "$out/prof_$arm.log" 2>&1 || exit $?
  f=$(find "$out/prof_$arm" -name '*kernel_stats.csv' | head -1); echo "== $arm"; cut -d, -f1-8 "$f" | cut -c1-200
  grep '^{' "$out/prof_$arm.log" | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms/step', d['ms_per_step'], d['kernels_ms'], 'lat', d['latency_ms'])" || true
done
