"""One line per bench JSON log: device tick, latency, K2, host-to-host ticks,
reuse, fallback and parity (tools/gpu_r05.sh output)."""
import json
import sys

for path in sys.argv[1:]:
    try:
        d = json.loads(open(path).read().strip().splitlines()[-1])
    except Exception as e:  # noqa: BLE001
        print(path, "unreadable:", e)
        continue
    e = d.get("end_to_end_tick") or {}
    a = e.get("all_candidates") or {}
    cb = d.get("cpu_baseline") or {}
    k = d["kernels_ms"]
    print("%-28s %-9s step %.4f lat %.4f K0 %.4f K2 %.4f | dpl %s enc %s | all %s enc %s reused %s | full %s | fb %s "
          "parity %s frac %.4f" % (
              path.split("/")[-1], d["config"].get("variant", "?"), d["ms_per_step"], d["latency_ms"],
              k.get("k0_tables", 0), k.get("k2_placement", 0), e.get("median_ms"), e.get("encode_ms_last_batch"),
              a.get("median_ms"), a.get("encode_ms"), a.get("candidate_side_reused"), e.get("full_tick_median_ms"),
              d.get("fallback_candidates"), cb.get("plans_identical_to_gpu"), d["roofline"]["frac"]))
