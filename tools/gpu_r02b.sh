cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out/r02b
for a in "3 64" "3 1500" "4"; do
  echo "== encode_stats $a" >> gpurun_out/r02b/encode_stats.txt
  timeout -k 10 120 k8s-spot-rescheduler_amd/bin/encode_stats $a >> gpurun_out/r02b/encode_stats.txt 2>&1 || exit $?
done
bash tools/gpu_tests.sh r02b 3 4 5
