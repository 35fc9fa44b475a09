#!/bin/bash
# K2 per-wave profiles only (SR_K2_PROFILE), per "cfg:variant":
#   tools/gpu_k2prof.sh tag "3:realistic 3:baseline"
tag=${1:-k2prof}; entries=${2:-3:baseline}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
out="$R/gpurun_out/$tag"
mkdir -p "$out"
for e in $entries; do
  cfg=${e%%:*}; var=${e#*:}
  name="c${cfg}$([ "$var" = baseline ] || echo "_$var")"
  rm -f "/tmp/k2prof_$name.bin"
  SR_K2_PROFILE="/tmp/k2prof_$name.bin" timeout -k 10 300 python bench.py --config $cfg --variant $var --steps 3 \
    --warmup 3 --e2e-reps 0 --no-cpu-baseline > "$out/${name}_bench_prof.log" 2>&1 || exit $?
  python tools/k2_profile.py "/tmp/k2prof_$name.bin" > "$out/${name}_k2_wave_profile.txt" 2>&1
  rm -f "/tmp/k2prof_$name.bin"
  echo "== $name"; cat "$out/${name}_k2_wave_profile.txt"
done
exit 0
