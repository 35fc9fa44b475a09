#!/bin/bash
# Round-5 GPU session: selected -m gpu modules, then bench lines.
#   tools/gpu_r05.sh tag "pytest files" "bench args;ENV=v ENV2=w|bench args;..."
# (a bench entry "ENVS|ARGS" runs bench.py with those environment variables)
# Every GPU step has its own time limit and the script stops at the first
# step that crashes or times out (pytest rc 1 = assertion failures: reported,
# the bench steps still run).
tag=${1:-run}; files=${2:-}; benches=${3:-}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
out="$R/gpurun_out/$tag"
mkdir -p "$out"
if [ -n "$files" ]; then
  timeout -k 10 1000 python -u -m pytest $files -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$out/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" "$out/pytest_gpu.log" | tail -5
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
i=0
IFS=';' read -ra B <<< "$benches"
for entry in "${B[@]}"; do
  i=$((i+1))
  envs=""; args="$entry"
  if [[ "$entry" == *"|"* ]]; then envs="${entry%%|*}"; args="${entry#*|}"; fi
  eval "$envs timeout -k 10 400 python bench.py $args" > "$out/bench_$i.log" 2>&1
  rc=$?; echo "bench $i ($entry) rc=$rc"; tail -1 "$out/bench_$i.log" | cut -c1-400
  [ $rc -ne 0 ] && exit $rc
done
exit 0
