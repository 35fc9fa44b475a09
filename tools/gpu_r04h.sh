set -o pipefail
mkdir -p gpurun_out/r04h
timeout -k 10 300 python -u -m pytest tests/test_gpu_ticks.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04h/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r04h/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -n "^FAILED\|Error" gpurun_out/r04h/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/tick_stress.py --seconds 20 --reuse > gpurun_out/r04h/tick_stress_reuse.txt 2>&1 || exit $?
tail -1 gpurun_out/r04h/tick_stress_reuse.txt
timeout -k 10 300 python tools/tick_stress.py --seconds 20 --reuse --wide > gpurun_out/r04h/tick_stress_reuse_wide.txt 2>&1 || exit $?
tail -1 gpurun_out/r04h/tick_stress_reuse_wide.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 --cpu-seconds 3 > gpurun_out/r04h/c3.json 2> gpurun_out/r04h/c3.err || exit $?
SR_K0_SKIP=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 --no-cpu-baseline > gpurun_out/r04h/c3_noskip.json 2> gpurun_out/r04h/c3_noskip.err || exit $?
timeout -k 10 300 python3 bench.py --config 5 --steps 200 --warmup 10 --cpu-seconds 3 > gpurun_out/r04h/c5.json 2> gpurun_out/r04h/c5.err || exit $?
python - <<'PY'
import json
for f in ("c3", "c3_noskip", "c5"):
    d = json.loads(open("gpurun_out/r04h/%s.json" % f).read().strip().splitlines()[-1])
    e = d.get("end_to_end_tick") or {}
    cb = d.get("cpu_baseline") or {}
    print(f, "ms/step %.4f" % d["ms_per_step"], d.get("kernels_ms"), d["config"].get("k0"), "lat", d.get("latency_ms"),
          "identical", cb.get("plans_identical_to_gpu"), "e2e", e.get("median_ms"), "all", (e.get("all_candidates") or {}).get("median_ms"))
PY
