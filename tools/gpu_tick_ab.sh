#!/bin/bash
# Same-box A/B of the C3 device tick (ms_per_step, latency_ms, K2) at the
# driver's step count and at 200 steps, each arm three times, interleaved:
#   tools/gpu_tick_ab.sh tag "ENV=val ..." "ENV=val ..." ...
# (an arm "SR_PLANNER_LIB=libsrplanner_<name>.so" loads a `make ab` build).
tag=$1; shift
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
cfg=${AB_CONFIG:-3}
for steps in 20 200; do
  for rep in 1 2 3; do
    i=0
    for arm in "$@"; do
      i=$((i+1))
      f="$out/s${steps}_arm${i}_rep${rep}.log"
      env $arm timeout -k 10 200 python bench.py --config $cfg --steps $steps --warmup 20 --no-cpu-baseline \
        --e2e-reps 0 $BENCH_ARGS > "$f" 2>&1 || exit $?
      python - "$f" "$arm" "$steps" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernels_ms"]
print("steps %-4s %-44s ms/step %.5f  latency %.5f  K0 %.5f  K2 %.5f  K2(timed) %.5f" % (sys.argv[3], sys.argv[2],
      d["ms_per_step"], d.get("latency_ms", 0), k["k0_tables"], k["k2_placement"], d["roofline"]["kernel_ms"]))
PY
    done
  done
done
