#!/usr/bin/env python3
"""K2 domain-path timing on large replica candidates (tools only; GPU).

A pool of spot nodes over zones, and candidates of Deployment replicas that
count each other, so every candidate takes the domain path (encode.cpp
analyse_spread / analyse_anti, kernels.hip k2_domain).  Kinds: zone spread
(maxSkew 1), hostname spread (maxSkew 2; the oracle takes minutes there: use
--no-oracle or few candidates), zone anti-affinity within groups of 3
replicas.  Prints K2's HIP-event time over back-to-back runs and the time per
pod of a candidate; checks every candidate's plan against the oracle once.

  python tools/domain_bench.py [--spot 3500] [--cands 64] [--pods 100] [--kind spread|anti|host]
"""
import argparse
import os
import random
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "k8s-spot-rescheduler_amd")]

import numpy as np  # noqa: E402

from helpers import Scenario  # noqa: E402
from oracle_lib import oracle_plan  # noqa: E402
from spotplanner import capi  # noqa: E402
from spotplanner.model import (Container, LabelSelector, Node, Pod, PodAffinityTerm,  # noqa: E402
                               TopologySpreadConstraint)
from spotplanner.planner import PredicateChecker  # noqa: E402

Z, H = "topology.kubernetes.io/zone", "kubernetes.io/hostname"


def scenario(n_spot, n_cand, n_pods, kind, seed=7):
    r = random.Random(seed)
    zones = ["z%d" % i for i in range(3)]
    nodes = [Node("s%d" % i, cpu_milli=r.choice([16000, 32000, 64000]), memory=256 * 2 ** 30, pods=110,
                  labels={Z: zones[i % 3], H: "s%d" % i}) for i in range(n_spot)]
    apps = ["app%d" % i for i in range(16)]
    spot_pods = [[Pod("b%d_%d" % (i, j), namespace="default",
                      containers=[Container(cpu_milli=r.choice([100, 250, 500, 1000]))],
                      labels={"app": r.choice(apps)}) for j in range(r.randrange(1, 12))] for i in range(n_spot)]
    cands = []
    for c in range(n_cand):
        app = apps[c % len(apps)]
        sel = LabelSelector(match_labels={"app": app})
        pods = []
        for j in range(n_pods):
            p = Pod("c%d_%d" % (c, j), namespace="default", containers=[Container(cpu_milli=r.choice([100, 250, 500]))],
                    labels={"app": app})
            if kind == "spread":
                p.topology_spread = [TopologySpreadConstraint(1, Z, "DoNotSchedule", sel)]
            elif kind == "host":
                p.topology_spread = [TopologySpreadConstraint(2, H, "DoNotSchedule", sel)]
            else:  # anti: groups of 3 replicas, each refusing zones that host another of its group
                p.labels = {"app": app, "grp": "c%d_g%d" % (c, j // 3)}
                p.pod_anti_affinity = [PodAffinityTerm(Z, LabelSelector(match_labels={"grp": "c%d_g%d" % (c, j // 3)}))]
            pods.append(p)
        cands.append(pods)
    return nodes, spot_pods, cands


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spot", type=int, default=3500)
    ap.add_argument("--cands", type=int, default=64)
    ap.add_argument("--pods", type=int, default=100)
    ap.add_argument("--kind", default="spread", choices=["spread", "anti", "host"])
    ap.add_argument("--runs", type=int, default=50)
    ap.add_argument("--no-oracle", action="store_true")
    a = ap.parse_args()
    nodes, spot_pods, cands = scenario(a.spot, a.cands, a.pods, a.kind)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    chk = PredicateChecker(0)
    lib = chk.lib
    h = sc.product_snapshot()
    cs = capi.sr_candidates(len(cands), capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32), None)
    status = np.zeros(len(cands), np.int32)
    node_of = np.zeros(len(flat), np.int32)
    out = capi.sr_plan_out()
    out.status = capi.ptr(status, capi.P32)
    out.node_of_pod = capi.ptr(node_of, capi.P32)
    t0 = time.perf_counter()
    assert lib.sr_plan_prepare(chk.handle, h, sc.ptr, ctypes_ref(cs)) == capi.SR_OK, chk.last_error()
    prep_ms = 1e3 * (time.perf_counter() - t0)
    k2 = []
    for _ in range(a.runs):  # timing() accumulates since set_timing: one run per window
        chk.set_timing(2)
        assert lib.sr_plan_run(chk.handle, ctypes_ref(out)) == capi.SR_OK, chk.last_error()
        t = chk.timing()
        k2.append(t.ms_placement / max(1, t.n_runs))
    n_fb = int(np.sum(status == capi.SR_CAND_FALLBACK))
    line = {"kind": a.kind, "spot": a.spot, "cands": a.cands, "pods_per_cand": a.pods,
            "k2_ms_median": round(float(np.median(k2)), 4), "us_per_pod_longest": round(
                1e3 * float(np.median(k2)) / a.pods, 3), "prepare_ms": round(prep_ms, 2), "fallback_cands": n_fb,
            "ok_cands": int(np.sum(status == capi.SR_CAND_OK))}
    if not a.no_oracle:
        o = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1, threads=16)
        same = all(int(o["status"][c]) == int(status[c]) and (int(status[c]) == capi.SR_CAND_FALLBACK or np.array_equal(
            o["node_of_pod"][cand_off[c]:cand_off[c + 1]], node_of[cand_off[c]:cand_off[c + 1]]))
            for c in range(len(cands)))
        line["plans_equal_oracle"] = bool(same)
    print(line, flush=True)
    lib.sr_snapshot_destroy(h)
    chk.close()
    return 0 if line.get("plans_equal_oracle", True) else 1


def ctypes_ref(x):
    import ctypes
    return ctypes.byref(x)


if __name__ == "__main__":
    sys.exit(main())
