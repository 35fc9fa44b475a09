#!/bin/bash
# Copy the judged summaries of a tools/gpu_round.sh run into profiles/<round>/
#   tools/save_profiles.sh gpurun_out/<tag> profiles/r01 [config]
src=$1; dst=$2; cfg=${3:-3}
for f in bench.log bench_podorder.log prof/run_kernel_stats.csv k2prof.txt "pmc_traffic_c${cfg}.json" pytest_gpu.log; do
  [ -s "$src/$f" ] || { echo "save_profiles: $src/$f missing or empty; nothing copied" >&2; exit 1; }
done
mkdir -p "$dst"
tail -1 "$src/bench.log" > "$dst/c${cfg}_bench.json"
tail -1 "$src/bench_podorder.log" > "$dst/c${cfg}_bench_pod_order_k2.json"
cp "$src/prof/run_kernel_stats.csv" "$dst/c${cfg}_kernel_stats.csv"
cp "$src/k2prof.txt" "$dst/c${cfg}_k2_wave_profile.txt"
cp "$src/pmc_traffic_c${cfg}.json" "$dst/c${cfg}_pmc_traffic.json"
cp "$src/pmc_traffic_c${cfg}.json" "$(dirname "$dst")/pmc_traffic_c${cfg}.json"
tail -3 "$src/pytest_gpu.log" > "$dst/pytest_gpu_tail.txt"
ls -la "$dst"
