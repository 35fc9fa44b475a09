#!/bin/bash
# GPU session: parity tests, bench, K2 per-wave profile, rocprofv3 kernel trace.
#   tools/gpu_check.sh [tag] [config]
tag=${1:-run}; cfg=${2:-3}
cd "$GRAFT_REPO_ROOT" || exit 2
out="$GRAFT_REPO_ROOT/gpurun_out/$tag"
mkdir -p "$out"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > "$out/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc"; tail -15 "$out/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
timeout -k 10 400 python bench.py --config "$cfg" --steps 200 --warmup 10 --cpu-seconds 5 > "$out/bench.log" 2>&1
rc=$?
echo "bench rc=$rc"; tail -3 "$out/bench.log"
[ $rc -ne 0 ] && exit $rc
rm -f "$out/k2prof.bin"
SR_K2_PROFILE="$out/k2prof.bin" timeout -k 10 300 python bench.py --config "$cfg" --steps 3 --warmup 3 --no-cpu-baseline > "$out/bench_prof.log" 2>&1
rc=$?
echo "k2prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
python tools/k2_profile.py "$out/k2prof.bin" > "$out/k2prof.txt" 2>&1; cat "$out/k2prof.txt"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config "$cfg" --steps 50 --warmup 2 --no-cpu-baseline > "$out/prof.log" 2>&1
rc=$?
echo "rocprof rc=$rc"; tail -2 "$out/prof.log"
f=$(find "$out/prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cut -c1-160 "$f"
exit $rc
