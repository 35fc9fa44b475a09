cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-r02c}
mkdir -p gpurun_out/$T
for a in "3 64" "3 1500" "4"; do
  echo "== encode_stats $a" >> gpurun_out/$T/encode_stats.txt
  timeout -k 10 120 k8s-spot-rescheduler_amd/bin/encode_stats $a >> gpurun_out/$T/encode_stats.txt 2>&1 || exit $?
done
# K0 A/B: atoms from global memory
SR_K0_LDS=0 timeout -k 10 300 python bench.py --config 3 --steps 200 --warmup 10 --cpu-seconds 1 \
  > gpurun_out/$T/bench_c3_k0global.log 2>&1 || exit $?
bash tools/gpu_tests.sh $T 3 4 5
