#!/bin/bash
# Parity first, then a same-box A/B of env arms, then a K2 wave profile:
#   tools/gpu_try.sh tag "ENV=val ..." "ENV=val ..." ...
tag=$1
R="$GRAFT_REPO_ROOT"; cd "$R" || exit 2
mkdir -p gpurun_out/$tag
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > gpurun_out/$tag/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/$tag/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/gpu_ab.sh "$@" || exit $?
bash tools/gpu_k2prof.sh "$tag" ${PROF_CFGS:-3}
