#!/bin/bash
# K2 per-wave profile + rocprof kernel stats of one bench configuration.
#   tools/gpu_prof05.sh tag "bench args" [ENV=v ...]
tag=${1:-run}; bargs=${2:---config 3}; shift 2
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
out="$R/gpurun_out/$tag"
mkdir -p "$out"
for kv in "$@"; do export "$kv"; done
rm -f /tmp/k2prof_$tag.bin
SR_K2_PROFILE="/tmp/k2prof_$tag.bin" timeout -k 10 300 python bench.py $bargs --steps 3 --warmup 3 \
  --e2e-reps 0 --no-cpu-baseline > "$out/bench_prof.log" 2>&1 || exit $?
python tools/k2_profile.py "/tmp/k2prof_$tag.bin" > "$out/k2prof.txt" 2>&1; head -30 "$out/k2prof.txt"
rm -f /tmp/k2prof_$tag.bin
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" $bargs --steps 200 --warmup 10 --no-cpu-baseline --e2e-reps 0 > "$out/prof.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc"; tail -1 "$out/prof.log" | cut -c1-200
[ $rc -ne 0 ] && exit $rc
f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-220 "$f"
exit 0
