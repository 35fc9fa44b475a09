# placement variants: current build vs the A/B build (previous variants), C5 and C3
cd "$GRAFT_REPO_ROOT" || exit 2
BENCH_ARGS="--config 5" bash tools/gpu_ab.sh ${TAG:-eo}/c5 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so" || exit $?
bash tools/gpu_ab.sh ${TAG:-eo}/c3 "SR_X=0" "SR_PLANNER_LIB=libsrplanner_ab.so" "SR_K2_SCAN_MIN=3"
