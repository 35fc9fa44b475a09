# the A/B build through the parity tests, then C3 / C5 A/B against the default build
cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-abtest}
mkdir -p gpurun_out/$T
SR_PLANNER_LIB=libsrplanner_ab.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "parity or known_answer or domain" > gpurun_out/$T/pytest_ab.log 2>&1
rc=$?; echo "pytest(ab) rc=$rc"; tail -2 gpurun_out/$T/pytest_ab.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab.sh $T/c3 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so" || exit $?
BENCH_ARGS="--config 5" bash tools/gpu_ab.sh $T/c5 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so"
