#!/bin/bash
# GPU session: the -m gpu suite, smoke, then bench lines for the given configs.
#   tools/gpu_tests.sh [tag] [configs...]      e.g. tools/gpu_tests.sh r02a 3 5
# Every GPU step has its own time limit; the script stops at the first step
# that crashes or times out (pytest rc 1 = assertion failures: reported, the
# bench steps still run).  SKIP_TESTS=1 skips pytest and smoke.
tag=${1:-run}; shift
cfgs=${*:-3}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
out="$R/gpurun_out/$tag"
mkdir -p "$out"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$out/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" "$out/pytest_gpu.log" | tail -5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
  tail -1 "$out/smoke.log"
fi
for cfg in $cfgs; do
  steps=200; [ "$cfg" = 4 ] && steps=50
  timeout -k 10 400 python bench.py --config "$cfg" --steps $steps --warmup 10 --cpu-seconds ${CPU_SECONDS:-10} \
    > "$out/bench_c$cfg.log" 2>&1
  rc=$?; echo "bench c$cfg rc=$rc"; tail -1 "$out/bench_c$cfg.log" | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
done
exit 0
