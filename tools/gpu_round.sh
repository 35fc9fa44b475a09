#!/bin/bash
# One GPU session: parity tests, bench (default K2 + pod-order A/B), K2 per-wave
# (rocprof and PMC passes run without the end-to-end ticks, whose prefix-batch
# launches would pull the per-launch averages below the full tick's),
# profile, rocprofv3 kernel trace and the two PMC traffic passes.
#   tools/gpu_round.sh [tag] [config] [skip-tests]
# Every GPU step has its own time limit; the script stops at the first step
# that crashes or times out (pytest rc 1 = assertion failures: reported, and
# the measurement steps still run).
tag=${1:-run}; cfg=${2:-3}; skip=${3:-}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
out="$R/gpurun_out/$tag"
mkdir -p "$out"
if [ -z "$skip" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -6 "$out/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
  tail -1 "$out/smoke.log"
fi
timeout -k 10 300 python bench.py --config "$cfg" --steps 200 --warmup 10 --cpu-seconds 10 > "$out/bench.log" 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 "$out/bench.log" | cut -c1-600
[ $rc -ne 0 ] && exit $rc
SR_K2_MODE=1 timeout -k 10 300 python bench.py --config "$cfg" --steps 200 --warmup 10 --no-cpu-baseline \
  > "$out/bench_podorder.log" 2>&1
rc=$?; echo "bench(pod order) rc=$rc"; tail -1 "$out/bench_podorder.log" | cut -c1-400
[ $rc -ne 0 ] && exit $rc
# the raw per-wave records (tens of MB) stay on the box: only the summary comes back
rm -f /tmp/k2prof_$tag.bin
SR_K2_PROFILE="/tmp/k2prof_$tag.bin" timeout -k 10 300 python bench.py --config "$cfg" --steps 3 --warmup 3 \
  --e2e-reps 0 --no-cpu-baseline > "$out/bench_prof.log" 2>&1 || exit $?
python tools/k2_profile.py "/tmp/k2prof_$tag.bin" > "$out/k2prof.txt" 2>&1; cat "$out/k2prof.txt"
rm -f /tmp/k2prof_$tag.bin
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python3 "$R/bench.py" --config "$cfg" --steps 200 --warmup 10 --no-cpu-baseline --e2e-reps 0 > "$out/prof.log" 2>&1
rc=$?; echo "rocprof trace rc=$rc"; tail -1 "$out/prof.log" | cut -c1-300
[ $rc -ne 0 ] && exit $rc
f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-200 "$f"
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pmc_fetch" -o run --output-format csv -- \
  python3 "$R/bench.py" --config "$cfg" --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 0 > "$out/pmc_fetch.log" 2>&1
rc=$?; echo "pmc FETCH_SIZE rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/pmc_write" -o run --output-format csv -- \
  python3 "$R/bench.py" --config "$cfg" --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 0 > "$out/pmc_write.log" 2>&1
rc=$?; echo "pmc WRITE_SIZE rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$R" && python tools/pmc_traffic.py "$out/pmc_fetch" "$out/pmc_write" "$out/pmc_traffic_c$cfg.json"
