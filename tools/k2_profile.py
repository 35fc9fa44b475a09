#!/usr/bin/env python3
"""Summarise K2 per-wave profiles written with SR_K2_PROFILE=<file>.

Each sr_plan_run appends {int64 n_cand, int64 n_k0} + n_cand x 16 u64 (K2)
+ n_k0 x 2 u64 (K0 waves: start, end; zero = not launched):
  [0] s_memrealtime at wave start (100 MHz)
 [1] at the arrival of the work-list entry
  [2] at the end                               [3] s_memtime cycles start->end
  [4] pod steps executed                       [5] 1 if rerun with 512 slots
  [6] speculative-record misses                [7] wave_min count | far-chunk count << 32
  [8..11] cycles per step section: a = start -> answer, b = answer -> slot
          update, c = wait for the next rows, d = next pod's first clean node
          + DMA issue;  [12] cycles waiting for speculative records
Node-order waves ([5] == 2) reuse the fields: [6] placements, [7] visits |
windows << 32, [8] prologue (F heads) cycles, [9] min + window load,
[10] placement (window visits), [11] pointer moves (+ far resolution), [14]
cycles from wave start to the pod records and window 0 in registers, [15] 1
if the candidate's window visits use 32-bit scaled state.
The last of the widest runs in the file is summarised (earlier ones are
warmup; narrower ones are prefix batches of sr_plan_first)."""
import sys

import numpy as np


def load(path):
    raw = np.fromfile(path, dtype=np.uint64)
    runs, k0s, i = [], [], 0
    while i + 2 <= len(raw):
        n, m = int(raw[i]), int(raw[i + 1]); i += 2
        runs.append(raw[i:i + 16 * n].reshape(n, 16)); i += 16 * n
        k0s.append(raw[i:i + 2 * m].reshape(m, 2)); i += 2 * m
    return runs, k0s


def main():
    runs, k0s = load(sys.argv[1])
    last_run = max(range(len(runs)), key=lambda i: (len(runs[i]), i))
    r = runs[last_run].astype(np.int64)
    k0 = k0s[last_run].astype(np.int64)
    k0 = k0[k0[:, 0] != 0]
    t0 = r[:, 0].min()
    if len(k0):
        is_s = k0[:, 0] < 0  # bit 63 of the start stamp: an S-row wave
        k0[:, 0] &= (1 << 63) - 1
        z = k0[:, 0].min()
        for name, m in (("S", is_s), ("T", ~is_s)):
            if m.any():
                print("K0 %s waves %d: start p50/p90/max %s us; duration p50/p90/max %s us; last end %.2f us"
                      % (name, int(m.sum()),
                         " ".join("%.2f" % x for x in np.percentile((k0[m, 0] - z) / 100.0, [50, 90, 100])),
                         " ".join("%.2f" % x for x in np.percentile((k0[m, 1] - k0[m, 0]) / 100.0, [50, 90, 100])),
                         (k0[m, 1].max() - z) / 100.0))
        print("K0 waves %d: start p50/p90/max %s us; duration p50/p90/max %s us; last end %.2f us; K2 first start %.2f us"
              % (len(k0), " ".join("%.2f" % x for x in np.percentile((k0[:, 0] - z) / 100.0, [50, 90, 100])),
                 " ".join("%.2f" % x for x in np.percentile((k0[:, 1] - k0[:, 0]) / 100.0, [50, 90, 100])),
                 (k0[:, 1].max() - z) / 100.0, (t0 - z) / 100.0))
    start = (r[:, 0] - t0) / 100.0          # us
    pro = (r[:, 1] - r[:, 0]) / 100.0
    end = (r[:, 2] - t0) / 100.0
    dur = (r[:, 2] - r[:, 0]) / 100.0
    steps = r[:, 4]
    loop_us = (r[:, 2] - r[:, 1]) / 100.0
    pct = lambda a: " ".join("%.2f" % x for x in np.percentile(a, [50, 90, 99, 100]))
    print("runs %d  waves %d" % (len(runs), len(r)))
    print("start skew us  p50/p90/p99/max:", pct(start))
    print("entry->list us p50/p90/p99/max:", pct(pro))
    print("wave dur us    p50/p90/p99/max:", pct(dur))
    print("end us         p50/p90/p99/max:", pct(end))
    print("steps          p50/p90/p99/max:", pct(steps))
    ok = steps > 0
    per = loop_us[ok] / steps[ok]
    print("loop us/step   p50/p90/p99/max:", pct(per))
    cyc = r[:, 3] / np.maximum(1, dur)     # cycles per us -> clock
    print("clock MHz (memtime/realtime) p50:", "%.0f" % np.median(cyc[dur > 0]))
    mode = r[:, 5]
    nodeo = mode == 2
    print("waves: node order %d, pod order %d (of which rerun with 512 slots %d)"
          % (int(nodeo.sum()), int((~nodeo).sum()), int((mode == 1).sum())))
    if nodeo.any():
        q = r[nodeo]
        vis = (q[:, 7] & 0xffffffff).astype(np.int64)
        print("node order: visits p50/p90/max %s; placements/visit %.2f; windows/wave %.2f"
              % (" ".join("%d" % x for x in np.percentile(vis, [50, 90, 100])),
                 q[:, 6].sum() / max(1, vis.sum()), (q[:, 7] >> 32).sum() / len(q)))
        print("node order: entry->records cycles p50/p90/max %s; prologue (F heads) cycles p50/p90/max %s" % (
            " ".join("%.0f" % x for x in np.percentile(q[:, 14], [50, 90, 100])),
            " ".join("%.0f" % x for x in np.percentile(q[:, 8], [50, 90, 100]))))
        sv = max(1, vis.sum())
        print("node order: cycles/visit min+window %.0f, placement %.0f, pointer moves %.0f"
              % (q[:, 9].sum() / sv, q[:, 10].sum() / sv, q[:, 11].sum() / sv))
        print("node order: placement cycles per placed pod %.0f" % (q[:, 10].sum() / max(1, q[:, 6].sum())))
        res = q[:, 12] & ((1 << 40) - 1)
        print("node order: of min+window, far resolution %.0f cycles/visit (%d chunk rounds, %d pods found no node), "
              "window loads %.0f cycles/visit" % (res.sum() / sv, int(((q[:, 12] >> 40) & 0xffff).sum()),
                                                 int((q[:, 12] >> 56).sum()), q[:, 13].sum() / sv))
        print("node order: wave dur us p50/p90/max %s" % pct(dur[nodeo]))
        print("node order: 32-bit scaled window visits in %d of %d waves" % (int((q[:, 15] & 1).sum()), len(q)))
        idle = (q[:, 6] == 0) & (vis == 0)  # no placement, no window visit: a pod with no feasible node first
        dq = dur[nodeo]
        print("node order: waves with no visit and no placement %d (%.1f %% of wave-us, p50 %.2f us)"
              % (int(idle.sum()), 100.0 * dq[idle].sum() / max(1e-9, dq.sum()),
                 float(np.median(dq[idle])) if idle.any() else 0.0))
    if (~nodeo).any():
        print("pod order:  wave dur us p50/p90/max %s" % pct(dur[~nodeo]))
    r = r[~nodeo] if (~nodeo).any() else r
    print("spec misses total %d, wave_min total %d, far chunks total %d" %
          (r[:, 6].sum(), (r[:, 7] & 0xffffffff).sum(), (r[:, 7] >> 32).sum()))
    tot = r[:, 8:13].sum(axis=0)
    if not (~nodeo).any():
        tot[4] = 0  # node-order records hold placement counters there
    st = max(1, (steps[~nodeo] if (~nodeo).any() else steps).sum())
    print("cycles/step by section a,b,c,d,spec-wait:", " ".join("%.0f" % (x / st) for x in tot))
    last = np.argsort(-end)[:8]
    full = runs[last_run].astype(np.int64)
    cols = ("wave start_us dur_us steps mode | visits placements windows | "
            "cycles: entry->records prologue min+window placement moves | 32-bit (+2: cooperative block) | "
            "resolve (chunk rounds, dead) window-loads")

    def row(c):
        f = full[c]
        nod = mode[c] == 2
        print("  %5d %6.2f %6.2f %4d %2d | %3d %3d %3d | %6d %6d %6d %6d %6d | %d | %6d (%d, %d) %6d"
              % (c, start[c], dur[c], steps[c], mode[c], f[7] & 0xffffffff, f[6], f[7] >> 32, f[14],
                 f[8], f[9], f[10], f[11], f[15] & 3, (f[12] & ((1 << 40) - 1)) if nod else 0,
                 ((f[12] >> 40) & 0xffff) if nod else 0, (f[12] >> 56) if nod else 0, f[13] if nod else 0))
    print("latest-ending waves: " + cols)
    for c in last:
        row(c)
    print("longest waves: " + cols)
    for c in np.argsort(-dur, kind="stable")[:8]:
        row(int(c))


if __name__ == "__main__":
    main()
