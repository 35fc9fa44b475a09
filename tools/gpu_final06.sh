#!/bin/bash
# Round-6 measurement session: per configuration (and variant) the bench line,
# the K2 per-wave profile, the rocprofv3 kernel statistics and the two PMC
# traffic passes (FETCH_SIZE, WRITE_SIZE: separate runs, kernel trace only).
#   tools/gpu_final06.sh tag "3:baseline 4:baseline 3:affinity ..."
# Every GPU step has its own time limit; the script stops at the first step
# that fails or times out.
tag=${1:-final}; entries=${2:-3:baseline}
R="$GRAFT_REPO_ROOT"
cd "$R" || exit 2
out="$R/gpurun_out/$tag"
mkdir -p "$out"
for e in $entries; do
  cfg=${e%%:*}; var=${e#*:}
  name="c${cfg}$([ "$var" = baseline ] || echo "_$var")"
  vargs="--config $cfg --variant $var"
  cpu="--cpu-seconds 10"; [ "$cfg" = 4 ] && cpu="--cpu-seconds 6"
  [ "$var" != baseline ] && cpu="--cpu-seconds 3"
  timeout -k 10 400 python bench.py $vargs --steps 200 --warmup 10 $cpu > "$out/${name}_bench.log" 2>&1
  rc=$?; echo "$name bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
  tail -1 "$out/${name}_bench.log" > "$out/${name}_bench.json"
  rm -f "/tmp/k2prof_$name.bin"
  SR_K2_PROFILE="/tmp/k2prof_$name.bin" timeout -k 10 300 python bench.py $vargs --steps 3 --warmup 3 \
    --e2e-reps 0 --no-cpu-baseline > "$out/${name}_bench_prof.log" 2>&1 || exit $?
  python tools/k2_profile.py "/tmp/k2prof_$name.bin" > "$out/${name}_k2_wave_profile.txt" 2>&1
  rm -f "/tmp/k2prof_$name.bin"
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/${name}_prof" -o run \
    --output-format csv -- python3 "$R/bench.py" $vargs --steps 200 --warmup 10 --no-cpu-baseline --e2e-reps 0 \
    > "$out/${name}_prof.log" 2>&1)
  rc=$?; echo "$name rocprof rc=$rc"; [ $rc -ne 0 ] && exit $rc
  f=$(find "$out/${name}_prof" -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" "$out/${name}_kernel_stats.csv"
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/${name}_pmc_fetch" \
    -o run --output-format csv -- python3 "$R/bench.py" $vargs --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 0 \
    > "$out/${name}_pmc_fetch.log" 2>&1)
  rc=$?; echo "$name pmc FETCH_SIZE rc=$rc"; [ $rc -ne 0 ] && exit $rc
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$out/${name}_pmc_write" \
    -o run --output-format csv -- python3 "$R/bench.py" $vargs --steps 20 --warmup 2 --no-cpu-baseline --e2e-reps 0 \
    > "$out/${name}_pmc_write.log" 2>&1)
  rc=$?; echo "$name pmc WRITE_SIZE rc=$rc"; [ $rc -ne 0 ] && exit $rc
  python tools/pmc_traffic.py "$out/${name}_pmc_fetch" "$out/${name}_pmc_write" "$out/pmc_traffic_${name}.json"
  rm -rf "$out/${name}_pmc_fetch" "$out/${name}_pmc_write" "$out/${name}_prof"
done
exit 0
