#!/bin/bash
# One GPU session for a K2 change: the -m gpu suite (stops on a crash), then a
# same-box A/B of this build against lib/libsrplanner_ab.so on C3 and C5, then
# K2 wave profiles of C3 and C5 (AB_CONFIGS="3 5" by default).   tools/gpu_win.sh tag
tag=${1:-win}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 "$out/pytest.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
[ $rc -eq 1 ] && exit 1
for c in ${AB_CONFIGS:-3 5}; do
  AB_CONFIG=$c bash tools/gpu_ab.sh "$tag/c$c" "SR_ARM=new" "SR_PLANNER_LIB=libsrplanner_ab.so" || exit $?
done
bash tools/gpu_k2prof.sh "$tag" ${AB_CONFIGS:-3 5}
