set -o pipefail
mkdir -p gpurun_out/r04g
timeout -k 10 300 python -u -m pytest tests/test_gpu_ticks.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04g/pytest_ticks.log 2>&1
rc=$?; tail -2 gpurun_out/r04g/pytest_ticks.log; if [ $rc -ne 0 ]; then grep -n "^FAILED\|Error" gpurun_out/r04g/pytest_ticks.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/tick_stress.py --seconds 60 --reuse > gpurun_out/r04g/tick_stress_reuse.txt 2>&1 || exit $?
tail -1 gpurun_out/r04g/tick_stress_reuse.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04g/c3.json 2> gpurun_out/r04g/c3.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 --cpu-seconds 3 > gpurun_out/r04g/c3_200.json 2> gpurun_out/r04g/c3_200.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 --tick cold --cpu-seconds 3 > gpurun_out/r04g/c3_cold.json 2> gpurun_out/r04g/c3_cold.err || exit $?
timeout -k 10 600 python3 bench.py --config 4 --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/r04g/c4.json 2> gpurun_out/r04g/c4.err || exit $?
timeout -k 10 300 python3 bench.py --config 5 --steps 200 --warmup 10 --cpu-seconds 3 > gpurun_out/r04g/c5.json 2> gpurun_out/r04g/c5.err || exit $?
python - <<'PY'
import json
for f in ("c3", "c3_200", "c3_cold", "c4", "c5"):
    d = json.loads(open("gpurun_out/r04g/%s.json" % f).read().strip().splitlines()[-1])
    e = d.get("end_to_end") or {}
    print(f, "ms/step %.4f" % d["ms_per_step"], d.get("kernels_ms"), d["config"].get("k0"), "lat", d.get("latency_ms"),
          "e2e", e.get("median_ms"), "all", json.dumps(e.get("all_candidates"))[:300],
          "full_tick", e.get("full_tick_median_ms"), json.dumps(e.get("full_tick_stages_median_ms")))
PY
