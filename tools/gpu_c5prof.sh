# C5 K2: wave profile and placement-path A/B
cd "$GRAFT_REPO_ROOT" || exit 2
out=gpurun_out/${TAG:-c5prof}
mkdir -p $out
rm -f $out/k2prof.bin
SR_K2_PROFILE="$out/k2prof.bin" timeout -k 10 300 python bench.py --config 5 --steps 3 --warmup 3 \
  --no-cpu-baseline > "$out/bench_prof.log" 2>&1 || exit $?
python tools/k2_profile.py "$out/k2prof.bin" > "$out/k2prof.txt" 2>&1; tail -24 "$out/k2prof.txt"
BENCH_ARGS="--config 5" bash tools/gpu_ab.sh ${TAG:-c5prof}/ab "SR_X=0" "SR_K2_SCAN_MIN=65" "SR_K2_MODE=1"
