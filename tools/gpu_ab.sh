#!/bin/bash
# A/B of planner variants in ONE GPU session (same box, same clocks):
#   tools/gpu_ab.sh tag "ENV=val ..." "ENV=val ..." ...   (each arm run twice, interleaved)
# Two builds: `make -C k8s-spot-rescheduler_amd ab AB_FLAGS=-DNAME=value` builds
# lib/libsrplanner_ab.so; the arm SR_PLANNER_LIB=libsrplanner_ab.so loads it.
tag=$1; shift
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
for rep in 1 2; do
  i=0
  for arm in "$@"; do
    i=$((i+1))
    env $arm timeout -k 10 200 python bench.py --config ${AB_CONFIG:-3} --steps 300 --warmup 20 --no-cpu-baseline $BENCH_ARGS > "$out/arm${i}_rep${rep}.log" 2>&1 || exit $?
    python - "$out/arm${i}_rep${rep}.log" "$arm" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
e = d.get("end_to_end_tick") or {}
k = d["kernels_ms"]
print("%-40s ms/step %.4f  latency %.4f  K0 %.4f  K2 %.4f  K3 %.4f  e2e %.4f  all %.3f" % (sys.argv[2],
      d["ms_per_step"], d.get("latency_ms", 0), k["k0_tables"], k["k2_placement"],
      k.get("k3_winner", k.get("k3_winner_and_collective", 0)), e.get("median_ms", 0),
      (e.get("all_candidates") or {}).get("median_ms", 0)))
PY
  done
done
