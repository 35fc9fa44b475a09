#!/usr/bin/env python3
"""Tick stress (tools only): one planner encodes tick after tick of a synthetic
cluster whose spot nodes gain random pods (1-3 per tick, host ports at C5), on
fresh snapshots, alternating the reference-faithful sr_plan_first and the
every-candidate plan, each against the oracle on the same mutated snapshot.
Exercises the persistent encoder's caches (state patches, port-conflict rows,
staging arena, node-record patch uploads).  GPU required.

  python tools/tick_stress.py [--seconds 150] [--wide] [--reuse] [--moves]

--moves: pods on spot nodes also change their cpu requests (and stamps)
between ticks, so NewNodeMap re-sorts the spot list; the node map comes from a
node map cache and the snapshot is the previous tick's, refreshed
(sr_snapshot_refresh), while the oracle rebuilds both from scratch.
"""
import ctypes
import argparse
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "k8s-spot-rescheduler_amd")]

from oracle_lib import OracleSnapshot, oracle_plan  # noqa: E402
from spotplanner import capi  # noqa: E402
from spotplanner.planner import PredicateChecker  # noqa: E402
from spotplanner.rescheduler import plan_arrays  # noqa: E402
from spotplanner.synth import SynthCluster, build_candidates, new_node_map  # noqa: E402
import test_gpu_ticks as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=150.0)
    ap.add_argument("--wide", action="store_true", help="C4-shaped clusters (5,000-node pools: rows over 64 words)")
    ap.add_argument("--reuse", action="store_true",
                    help="every tick plans all candidates on one planner per cluster: the same stamped input tick "
                         "after tick, so the candidate side is reused (CandReuse) and its records patched on the device")
    ap.add_argument("--moves", action="store_true",
                    help="spot pods change cpu requests between ticks (the spot order moves); kept node map cache and "
                         "refreshed snapshot")
    a = ap.parse_args()
    lib = capi.load_planner()
    os.environ["SR_NODE_PATCH"] = "0"  # the second planner uploads a changed node section whole
    patcher = PredicateChecker(0)
    del os.environ["SR_NODE_PATCH"]
    default = PredicateChecker(0)
    t0, ticks = time.time(), 0
    rng = np.random.default_rng(11)
    if a.wide:
        clusters = [SynthCluster(4, seed=3, n_on_demand=150, n_spot=5000), SynthCluster(4, seed=4, n_on_demand=100, n_spot=4300)]
    else:
        clusters = [SynthCluster(5, seed=3, n_on_demand=120, n_spot=400), SynthCluster(3, seed=4, n_on_demand=150, n_spot=500)]
    maps = []
    for sc in clusters:
        nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
        maps.append((nm, *build_candidates(nm, sc.pod_flags())))
    extra = [[], []]
    caches, kept = [], [None, None]
    if a.moves:
        from oracle_lib import oracle_new_node_map
        for _ in clusters:
            caches.append(ctypes.c_void_p())
            assert lib.sr_node_map_cache_create(ctypes.byref(caches[-1])) == capi.SR_OK
        views = []
        for sc in clusters:
            cl = sc.cluster
            views.append(([np.ctypeslib.as_array(x, shape=(sc.n_pods,)) for x in
                           (cl.pods.cpu_sort_milli, cl.pods.req_milli_cpu, cl.acc_milli_cpu) if x],
                          np.ctypeslib.as_array(cl.pod_stamp, shape=(sc.n_pods,))))
    per_cluster = [PredicateChecker(0), PredicateChecker(0)] if a.reuse else []
    reused = patches = 0
    while time.time() - t0 < a.seconds:
        ci = (ticks // 10) % 2  # ten ticks of one cluster, then ten of the other
        sc, (nm, cand_off, cand_pods) = clusters[ci], maps[ci]
        ck = per_cluster[ci] if a.reuse else patcher if ticks % 3 == 0 else default
        if rng.random() < 0.3 and extra[ci]:
            extra[ci].pop(int(rng.integers(len(extra[ci]))))  # a pod leaves again
        for _ in range(int(rng.integers(1, 4))):
            extra[ci].append((int(cand_pods[rng.integers(len(cand_pods))]), int(rng.integers(len(nm.spot)))))
        extra[ci] = extra[ci][-6:]
        if a.moves:
            cpu, stamps = views[ci]
            for _ in range(int(rng.integers(1, 4))):  # pods on spot nodes change requests: the spot order moves
                node = nm.spot[rng.integers(len(nm.spot))]
                lo, hi = nm.node_pod_off[node], nm.node_pod_off[node + 1]
                if hi > lo:
                    pod = nm.node_pod_idx[rng.integers(lo, hi)]
                    d = int(rng.integers(-150, 250))
                    for x in cpu:
                        x[pod] = max(0, int(x[pod]) + d)
                    stamps[pod] += 2
            nm = new_node_map(lambda cp, pp, mp: lib.sr_new_node_map_cached(caches[ci], cp, pp, mp, None), sc.ptr,
                              sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            orc = oracle_new_node_map(sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            assert np.array_equal(nm.spot, orc.spot) and np.array_equal(nm.node_pod_idx, orc.node_pod_idx), ticks
            maps[ci] = (nm, cand_off, cand_pods)
            args = (sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(nm.node_pod_off, capi.P32),
                    capi.ptr(nm.node_pod_idx, capi.P32))
            if kept[ci] is None:
                kept[ci] = ctypes.c_void_p()
                assert lib.sr_snapshot_create(*args, ctypes.byref(kept[ci])) == capi.SR_OK
            else:
                assert lib.sr_snapshot_refresh(kept[ci], *args, None) == capi.SR_OK
            h = kept[ci]
        else:
            h = T._snapshot(lib, sc, nm)
        osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
        for pod, pos in extra[ci]:
            assert lib.sr_snapshot_add_pod(h, sc.ptr, pod, pos) == capi.SR_OK
            osnap.lib.oracle_snapshot_add_pod(osnap.h, sc.ptr, pod, pos)
        ref_all = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
        if a.reuse:
            p = plan_arrays(ck, h, sc.ptr, cand_off, cand_pods)
            t = ck.timing()
            reused += t.enc_reused
            patches += t.enc_pod_patches
            assert np.array_equal(p.status, ref_all["status"]), ticks
            assert np.array_equal(p.node_of_pod, ref_all["node_of_pod"]), ticks
            assert p.winner == ref_all["winner"], ticks
        elif ticks % 2 == 0:
            ref_early = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=0)
            o, status, nodes, wmap = T.plan_first(ck, h, sc.ptr, cand_off, cand_pods)
            T.check_first(o, status, nodes, wmap, ref_all, ref_early, cand_off)
        else:
            p = plan_arrays(ck, h, sc.ptr, cand_off, cand_pods)
            assert np.array_equal(p.status, ref_all["status"]), ticks
            assert np.array_equal(p.node_of_pod, ref_all["node_of_pod"]), ticks
            assert p.winner == ref_all["winner"], ticks
        if not a.moves:
            lib.sr_snapshot_destroy(h)
        ticks += 1
        if ticks % 20 == 0:
            print("  %d ticks, %.0f s" % (ticks, time.time() - t0), flush=True)
    patcher.close()
    default.close()
    for ck in per_cluster:
        ck.close()
    for h in kept:
        if h is not None:
            lib.sr_snapshot_destroy(h)
    for cache in caches:
        lib.sr_node_map_cache_destroy(cache)
    print("tick stress: %d ticks in %.0f s, every plan equal to the oracle%s" % (
        ticks, time.time() - t0, " (%d reused, %d pod patches)" % (reused, patches) if a.reuse else ""))
    return 0


if __name__ == "__main__":
    sys.exit(main())
