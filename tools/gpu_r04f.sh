set -o pipefail
mkdir -p gpurun_out/r04f
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/r04f/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/r04f/pytest_gpu.log; if [ $rc -ne 0 ]; then grep -n "^FAILED\|Error" gpurun_out/r04f/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python tools/tick_stress.py --seconds 60 --reuse > gpurun_out/r04f/tick_stress_reuse.txt 2>&1 || exit $?
tail -1 gpurun_out/r04f/tick_stress_reuse.txt
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r04f/c3.json 2> gpurun_out/r04f/c3.err || exit $?
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 --tick cold --cpu-seconds 3 > gpurun_out/r04f/c3_cold.json 2> gpurun_out/r04f/c3.err || exit $?
timeout -k 10 600 python3 bench.py --config 4 --steps 20 --warmup 5 --cpu-seconds 5 > gpurun_out/r04f/c4.json 2> gpurun_out/r04f/c4.err || exit $?
python - <<'PY'
import json
for f in ("c3", "c3_cold", "c4"):
    d = json.loads(open("gpurun_out/r04f/%s.json" % f).read().strip().splitlines()[-1])
    e = d.get("end_to_end") or {}
    print(f, "ms/step %.4f" % d["ms_per_step"], d.get("kernels_ms"), d["config"].get("tick"), d["config"].get("k0"), "e2e", e.get("median_ms"), "all", json.dumps(e.get("all_candidates"))[:400],
          "full_tick", e.get("full_tick_median_ms"), json.dumps(e.get("full_tick_stages_median_ms")))
PY
