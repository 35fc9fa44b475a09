# current build vs the A/B build (previous commit): GPU parity first, then C5 and C3 A/B
cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-eo}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/$T/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
BENCH_ARGS="--config 5" bash tools/gpu_ab.sh $T/c5 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so" || exit $?
bash tools/gpu_ab.sh $T/c3 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so"
