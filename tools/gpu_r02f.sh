# K2 prologue A/B: parity (node-order paths) on the default build, then
# default vs the A/B build vs sequential placement, then a K2 wave profile.
cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-r02f}
out=gpurun_out/$T
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "parity or known_answer or ticks" > $out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_ab.sh $T/ab ${ARMS:-"SR_X=0" "SR_K2_SCAN_MIN=65" "SR_K2_SCALAR=0" "SR_K2_SCAN_MIN=4" "SR_K2_SCAN_MIN=8"} || exit $?
rm -f $out/k2prof.bin
SR_K2_PROFILE="$out/k2prof.bin" timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 3 \
  --no-cpu-baseline > "$out/bench_prof.log" 2>&1 || exit $?
python tools/k2_profile.py "$out/k2prof.bin" > "$out/k2prof.txt" 2>&1; tail -22 "$out/k2prof.txt"
