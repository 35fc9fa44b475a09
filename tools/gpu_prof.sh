# GPU suite, then a K2 wave profile for C3 and C5
cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-prof}
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread > gpurun_out/$T/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/$T/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for cfg in 3 5; do
  rm -f gpurun_out/$T/k2prof_c$cfg.bin
  SR_K2_PROFILE="gpurun_out/$T/k2prof_c$cfg.bin" timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 3 \
    --no-cpu-baseline > gpurun_out/$T/bench_prof_c$cfg.log 2>&1 || exit $?
  python tools/k2_profile.py gpurun_out/$T/k2prof_c$cfg.bin > gpurun_out/$T/k2prof_c$cfg.txt 2>&1
  echo "== C$cfg"; tail -13 gpurun_out/$T/k2prof_c$cfg.txt; rm -f gpurun_out/$T/k2prof_c$cfg.bin
done
