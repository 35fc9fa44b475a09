#!/bin/bash
# round-1 GPU session B: parity tests, bench, kernel trace, PMC traffic passes
cd "$GRAFT_REPO_ROOT" || exit 2
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --cpu-seconds 5 > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
R="$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r1" -o run --output-format csv -- python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline > "$R/gpurun_out/prof_r1.log" 2>&1 || exit $?
echo "trace ok"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$R/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/pmc_fetch.log" 2>&1 || exit $?
echo "pmc fetch ok"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$R/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 2 --no-cpu-baseline > "$R/gpurun_out/pmc_write.log" 2>&1 || exit $?
echo "pmc write ok"
ls -R "$R/gpurun_out" | head -40
