# GPU suite, then C3/C5: window prefetch (default build vs A/B build) and the event-polling completion wait
cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-win}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/$T/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab.sh $T/c3 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so" "SR_WAIT_EVENT=1" || exit $?
BENCH_ARGS="--config 5" bash tools/gpu_ab.sh $T/c5 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so"
