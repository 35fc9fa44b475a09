#!/bin/bash
# Domain-path change: the -m gpu suite, then tools/domain_bench.py (zone spread
# and zone anti-affinity replica candidates) for this build and
# lib/libsrplanner_ab.so, interleaved on one box.   tools/gpu_domain_ab.sh tag
tag=${1:-dom}
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
out="$R/gpurun_out/$tag"; mkdir -p "$out"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > "$out/pytest.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 "$out/pytest.log"
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for lib in libsrplanner.so libsrplanner_ab.so; do
    for kind in spread anti; do
      SR_PLANNER_LIB=$lib timeout -k 10 300 python tools/domain_bench.py --kind $kind --runs 20 \
        > "$out/${kind}_${lib}_$rep.log" 2>&1 || exit $?
      echo "$lib $(tail -1 "$out/${kind}_${lib}_$rep.log")"
    done
  done
done
