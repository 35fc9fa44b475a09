#!/bin/bash
# Round-4 evidence beyond tools/gpu_round.sh: bench lines of C1/C2/C4/C5 with their CPU baselines, the
# driver's exact bench command, the realistic variant of C3, K2 wave profiles of C4 and C5.
#   tools/gpu_r04.sh tag
tag=${1:-r04}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > "$out/driver_cmd.json" 2> "$out/driver_cmd.err" || exit $?
echo "driver: $(cut -c1-160 "$out/driver_cmd.json")"
for cfg in 1 2 5 4; do
  timeout -k 10 400 python3 bench.py --config $cfg --steps 200 --warmup 10 --cpu-seconds 10 > "$out/bench_c$cfg.json" \
    2> "$out/bench_c$cfg.err" || exit $?
  echo "C$cfg: $(cut -c1-120 "$out/bench_c$cfg.json")"
done
timeout -k 10 300 python3 bench.py --config 3 --variant realistic --steps 200 --warmup 10 --cpu-seconds 5 \
  > "$out/realistic_c3.json" 2> "$out/realistic_c3.err" || exit $?
echo "realistic: $(cut -c1-120 "$out/realistic_c3.json")"
bash tools/gpu_k2prof.sh "$tag/k2" 4 5 > "$out/k2prof.log" 2>&1 || exit $?
tail -3 "$out/k2prof.log"
exit 0
