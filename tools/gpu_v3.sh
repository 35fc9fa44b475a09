#!/bin/bash
# Round-3 K2 change: parity suite subset on the new build, then A/B against the
# round-2 code (libsrplanner_ab.so built with -DSR_K2_V3=0) and a K2 profile.
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
tag=${1:-v3}; out="$R/gpurun_out/$tag"; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  > "$out/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$out/pytest_gpu.log"
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh "$tag/ab" "SR_PLANNER_LIB=libsrplanner_ab.so" "SR_K2_V3_ARM=1" || exit $?
bash tools/gpu_k2prof.sh "$tag/prof" 3 5 > "$out/k2prof.txt" 2>&1 || exit $?
grep -E "wave dur|cycles/visit|latest|^ *[0-9]+ " "$out/k2prof.txt" | head -12
