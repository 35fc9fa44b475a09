# K2 prefix-sum placement: parity with the pass forced everywhere, then the
# full suite at the default, then C3/C4 bench A/B over SR_K2_SCAN_MIN.
cd "$GRAFT_REPO_ROOT" || exit 2
T=${TAG:-r02d}
out=gpurun_out/$T
mkdir -p $out
SR_K2_SCAN_MIN=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "parity or known_answer or distributed or ticks" > $out/pytest_scan1.log 2>&1
rc=$?; echo "pytest scan_min=1 rc=$rc"; tail -2 $out/pytest_scan1.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for m in 65 1 2 3 4 6; do
  SR_K2_SCAN_MIN=$m timeout -k 10 300 python bench.py --config 3 --steps 200 --warmup 10 --no-cpu-baseline \
    > $out/bench_c3_scan$m.log 2>&1 || exit $?
  echo "c3 scan_min=$m $(tail -1 $out/bench_c3_scan$m.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"],d["kernels_ms"])')"
done
for m in 65 2; do
  SR_K2_SCAN_MIN=$m timeout -k 10 300 python bench.py --config 4 --steps 50 --warmup 10 --no-cpu-baseline \
    > $out/bench_c4_scan$m.log 2>&1 || exit $?
  echo "c4 scan_min=$m $(tail -1 $out/bench_c4_scan$m.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["ms_per_step"],d["kernels_ms"])')"
done
rm -f $out/k2prof.bin
SR_K2_PROFILE="$out/k2prof.bin" timeout -k 10 300 python bench.py --config 3 --steps 3 --warmup 3 \
  --no-cpu-baseline > "$out/bench_prof.log" 2>&1 || exit $?
python tools/k2_profile.py "$out/k2prof.bin" > "$out/k2prof.txt" 2>&1; head -30 "$out/k2prof.txt"
