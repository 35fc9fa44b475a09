#!/bin/bash
# Round-6 GPU session: the -m gpu suite, smoke, the C3 bench line (driver
# command), and the N = 2 path rehearsed on the box's one GPU (two ranks on
# device 0 through the shared-memory transport, strong line + weak beside).
#   tools/gpu_r06.sh tag [pytest -k expr]
tag=${1:-r06}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 \
    --timeout-method thread ${2:+-k "$2"} > "$out/pytest_gpu.log" 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" "$out/pytest_gpu.log" | tail -3
  [ $rc -ne 0 ] && exit $rc
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || exit $?
  tail -1 "$out/smoke.log"
fi
timeout -k 10 400 python bench.py --steps 20 --warmup 20 > "$out/bench_c3.log" 2>&1 || exit $?
tail -1 "$out/bench_c3.log" | cut -c1-400
SR_BENCH_DEVICE=0 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 10 --e2e-reps 2 \
  > "$out/bench_c3_n2_shm.log" 2>&1 || exit $?
tail -1 "$out/bench_c3_n2_shm.log" | cut -c1-400
exit 0
