#!/bin/bash
# Round-4 GPU session: the -m gpu suite, smoke, the driver's bench command, the
# realistic variant, then same-box A/B arms (tools/gpu_ab.sh).  Every GPU step
# has its own time limit; the script stops at the first step that crashes.
#   tools/gpu_r04.sh tag [skip-tests]
tag=${1:-r04}; skip=${2:-}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
if [ -z "$skip" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -4 "$out/pytest_gpu.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
  tail -1 "$out/smoke.log"
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/driver_cmd.json" 2> "$out/driver_cmd.err" || exit $?
echo "driver line:"; cut -c1-200 "$out/driver_cmd.json"
timeout -k 10 300 python bench.py --config 3 --variant realistic --steps 100 --warmup 10 --cpu-seconds 5 \
  > "$out/realistic_c3.json" 2> "$out/realistic_c3.err" || exit $?
python - "$out/realistic_c3.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
cb = d.get("cpu_baseline", {})
print("realistic C3: ms/step %.4f fallback %d ratio %s identical %s" % (d["ms_per_step"], d["fallback_candidates"],
      cb.get("fallback_ratio"), cb.get("plans_identical_to_gpu")))
PY
for arms in C5 C3; do
  if [ $arms = C5 ]; then
    AB_CONFIG=5 bash tools/gpu_ab.sh "$tag/ab_c5" "SR_PLANNER_LIB=libsrplanner.so" "SR_PLANNER_LIB=libsrplanner_oset.so" \
      "SR_PLANNER_LIB=libsrplanner_opred.so" || exit $?
  else
    AB_CONFIG=3 bash tools/gpu_ab.sh "$tag/ab_c3" "SR_K2_WPB=4" "SR_K2_WPB=1" "SR_K2_WPB=2" \
      "SR_PLANNER_LIB=libsrplanner_oset.so" || exit $?
  fi
done
exit 0
