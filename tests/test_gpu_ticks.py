"""Consecutive ticks through one planner (the persistent encoder)
and the reference-faithful prefix-batched tick (sr_plan_first).

run() rebuilds its model every housekeeping tick (rescheduler.go:195,215) and
stops at the first drainable candidate (:280-286).  The planner keeps what it
derived from the previous tick (spot-node views, specs, requirement rows) and
re-encodes what changed; these tests change one thing at a time between ticks
-- a pod added on one spot node, node labels and taints, a different cluster,
a different string interner -- and check every tick against the oracle."""
import ctypes
import os

import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import OracleSnapshot, oracle_plan
from plan_first_cases import check_plan_first, plan_first_scenario
from randcluster import rand_scenario
from spotplanner import capi
from spotplanner.model import Interner, Taint
from spotplanner.rescheduler import plan_arrays
from spotplanner.synth import SynthCluster, build_candidates, new_node_map

pytestmark = pytest.mark.gpu
SKIPPED = capi.SR_CAND_SKIPPED


def plan_first(checker, h, cluster_ptr, cand_off, cand_pods, full=True):
    lib = capi.load_planner()
    n = len(cand_off) - 1
    c = capi.sr_candidates(n, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32), None)
    status = np.full(max(1, n), -99, np.int32)
    nodes = np.full(max(1, int(cand_off[-1]) if n else 1), -99, np.int32)
    wmap = np.full(max(1, int(np.max(np.diff(cand_off))) if n else 1), -1, np.int32)
    o = capi.sr_plan_out()
    if full:
        o.status = capi.ptr(status, capi.P32)
        o.node_of_pod = capi.ptr(nodes, capi.P32)
    o.winner_map = capi.ptr(wmap, capi.P32)
    st = lib.sr_plan_first(checker.handle, h, cluster_ptr, ctypes.byref(c), ctypes.byref(o))
    assert st == capi.SR_OK, checker.last_error()
    return o, status[:n], nodes[: int(cand_off[-1]) if n else 0], wmap[: o.winner_npods]


def check_first(o, status, nodes, wmap, ref_all, ref_early, cand_off, full=True):
    segs = [nodes[int(cand_off[c]):int(cand_off[c + 1])] for c in range(len(cand_off) - 1)]
    check_plan_first(o.first_ok, o.first_fallback, o.winner, wmap, status, segs, ref_all, ref_early, cand_off, full)


@pytest.fixture(scope="module")
def small_batch_checker():
    from spotplanner.planner import PredicateChecker
    os.environ["SR_PREFIX_BATCH"] = "2"
    try:
        c = PredicateChecker(0)
    finally:
        del os.environ["SR_PREFIX_BATCH"]
    yield c
    c.close()


@pytest.mark.parametrize("seed", range(24))
@pytest.mark.parametrize("which", ["default", "batch2"])
def test_plan_first_matches_reference_loop(checker, small_batch_checker, seed, which):
    """Fallback candidates before, right after, far after and instead of the
    first drainable one, across prefix-batch boundaries, with hostname / zone
    (anti-)affinity on three seeds in four: the winner, -1 when a fallback
    candidate precedes it, the first fallback, every evaluated status and
    mapping, equal to the oracle's loop."""
    ck = checker if which == "default" else small_batch_checker
    nodes, spot_pods, cands, pattern, win, fb = plan_first_scenario(seed)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    ref_all = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1)
    ref_early = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=0)
    for c in fb:  # the injected candidates take the reference path on both sides
        assert ref_all["status"][c] == capi.SR_CAND_FALLBACK
    h = sc.product_snapshot()
    try:
        for full in (True, False):
            o, status, nodes_o, wmap = plan_first(ck, h, sc.ptr, cand_off, cand_pods, full)
            check_first(o, status, nodes_o, wmap, ref_all, ref_early, cand_off, full)
    finally:
        capi.load_planner().sr_snapshot_destroy(h)


@pytest.mark.parametrize("config,variant", [(1, None), (2, None), (3, None), (5, None), (3, "realistic"),
                                            (3, "affinity")])
def test_plan_first_synthetic_configs(checker, small_batch_checker, config, variant):
    # the variants: extension records on the node-order kernel (realistic), and
    # each prefix batch keeping only the anti-affinity terms its candidates have
    # or are selected by, with zone-spread replicas on the domain path (affinity)
    from spotplanner.synth import AFFINITY, REALISTIC
    sc = SynthCluster(config, **{"realistic": REALISTIC, "affinity": AFFINITY}.get(variant, {}))
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
    ref_all = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
    ref_early = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=0)
    h = ctypes.c_void_p()
    assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                  capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                  ctypes.byref(h)) == capi.SR_OK
    try:
        for ck in (checker, small_batch_checker):
            o, status, nodes_o, wmap = plan_first(ck, h, sc.ptr, cand_off, cand_pods)
            check_first(o, status, nodes_o, wmap, ref_all, ref_early, cand_off)
            assert o.checks > 0 and ck.timing().prefix_batches >= 1
    finally:
        lib.sr_snapshot_destroy(h)


def _snapshot(lib, sc, nm):
    h = ctypes.c_void_p()
    assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                  capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                  ctypes.byref(h)) == capi.SR_OK
    return h


@pytest.fixture(scope="module")
def whole_checker():
    """A planner that uploads a changed node section whole (SR_NODE_PATCH=0; by
    default the records of up to 8 changed nodes ride in the call's copy and K0
    writes them into the resident section)."""
    from spotplanner.planner import PredicateChecker
    os.environ["SR_NODE_PATCH"] = "0"
    try:
        c = PredicateChecker(0)
    finally:
        del os.environ["SR_NODE_PATCH"]
    yield c
    c.close()


@pytest.mark.parametrize("config", [3, 5])
@pytest.mark.parametrize("which", ["default", "whole"])
def test_consecutive_ticks_one_node_changed(checker, whole_checker, which, config):
    """Tick after tick on fresh snapshots of one cluster, each with one more
    pod placed on some spot node (its state changes, the static view not):
    every full plan equals the oracle on the same mutated snapshot.  `default`:
    the changed nodes' records go to the device with the call's copy and K0
    applies them; `whole`: the changed node section goes up whole.  Config 5: the
    added pods carry host ports, so the cached base port-conflict rows are
    patched node by node."""
    other = whole_checker
    checker = whole_checker if which == "whole" else checker
    sc = SynthCluster(config, seed=21, n_on_demand=200, n_spot=450)
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    rng = np.random.default_rng(5)
    extra = []
    for tick in range(8):
        h = _snapshot(lib, sc, nm)
        osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
        if tick:  # one more pod on one spot node (several ticks accumulate on different nodes)
            extra.append((int(cand_pods[rng.integers(len(cand_pods))]), int(rng.integers(len(nm.spot)))))
        for pod, pos in extra[-1:]:
            assert lib.sr_snapshot_add_pod(h, sc.ptr, pod, pos) == capi.SR_OK
            osnap.lib.oracle_snapshot_add_pod(osnap.h, sc.ptr, pod, pos)
        p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
        t = checker.timing()
        if which == "default":  # the same tick through the whole-section planner: its upload for comparison
            plan_arrays(other, h, sc.ptr, cand_off, cand_pods)
            up_whole = other.timing().bytes_uploaded
        o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
        assert np.array_equal(p.status, o["status"]), tick
        assert np.array_equal(p.node_of_pod, o["node_of_pod"]), tick
        assert p.winner == o["winner"]
        if tick >= 2:  # steady state: one node's state re-encoded, no spec is new
            assert t.enc_static_rebuilt == 0 and t.enc_state_nodes <= 2 and t.enc_new_specs == 0, \
                (t.enc_static_rebuilt, t.enc_state_nodes, t.enc_new_specs)
            if which == "default":  # <= 2 node patches in the call's copy instead of the section
                n_pad = (len(nm.spot) + 127) // 128 * 128
                assert up_whole - t.bytes_uploaded >= n_pad * 88 - 256, (up_whole, t.bytes_uploaded)
        lib.sr_snapshot_destroy(h)


@pytest.mark.parametrize("config", [3, 5])
def test_ticks_candidate_side_reuse(config):
    """Candidate-side reuse (host.hpp CandReuse) through the planner (C5: host-port candidates): tick
    after tick the same stamped candidate input on fresh snapshots whose spot
    nodes gain pods (one at a time, bursts of 20, then all leave again).  From
    the third tick on the encoder keeps the candidate side, the device keeps
    its pod records and K0 re-points the ones whose thresholds moved (pod
    patches), or launches no K0 at all while at most 16 nodes changed since its
    tables were written (K2 recomputes those nodes' bits); every plan equals the
    oracle.  In between: a prepare whose
    patches no run applies (the next tick uploads the records whole), and
    sr_plan_first's prefix batches on the same planner (other inputs, other
    workload slots: the every-candidate input stays reused)."""
    from spotplanner.planner import PredicateChecker
    ck = PredicateChecker(0)
    try:
        sc = SynthCluster(config, seed=22, n_on_demand=200, n_spot=450)
        lib = capi.load_planner()
        nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
        cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
        n_rec_bytes = int(cand_off[-1]) * 48
        rng = np.random.default_rng(9)
        extra, patched, reused, k0_cols, k0_less = [], 0, 0, 0, 0
        for tick in range(16):
            h = _snapshot(lib, sc, nm)
            osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
            if tick == 11:
                extra.clear()
            elif tick:
                for _ in range(20 if tick % 4 == 3 else 1):
                    extra.append((int(cand_pods[rng.integers(len(cand_pods))]), int(rng.integers(len(nm.spot)))))
            for pod, pos in extra:
                assert lib.sr_snapshot_add_pod(h, sc.ptr, pod, pos) == capi.SR_OK
                osnap.lib.oracle_snapshot_add_pod(osnap.h, sc.ptr, pod, pos)
            o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
            if tick == 6:  # prepared, never run: its pod patches never reach the device
                c = capi.sr_candidates(len(cand_off) - 1, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32),
                                       None)
                assert lib.sr_plan_prepare(ck.handle, h, sc.ptr, ctypes.byref(c)) == capi.SR_OK
            if tick in (9, 10):  # the reference-faithful tick first: its batches take other slots
                ref_early = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=0)
                fo, status, nodes, wmap = plan_first(ck, h, sc.ptr, cand_off, cand_pods)
                check_first(fo, status, nodes, wmap, o, ref_early, cand_off)
            p = plan_arrays(ck, h, sc.ptr, cand_off, cand_pods)
            t = ck.timing()
            assert np.array_equal(p.status, o["status"]), tick
            assert np.array_equal(p.node_of_pod, o["node_of_pod"]), tick
            assert p.winner == o["winner"], tick
            if tick >= 2:
                assert t.enc_reused == 1, (tick, t.enc_reused)
                if tick not in (6, 9, 10):  # no K0 (<= 16 nodes changed since the tables), or K0 on the changed
                    # word columns only: never every row
                    assert t.k0_columns >= 0 or t.k0_columns == -2, (tick, t.k0_columns)
                    k0_cols += max(0, t.k0_columns)
                    k0_less += t.k0_columns == -2
                reused += 1
                patched += t.enc_pod_patches
                if tick != 6:  # the records stay on the device: the copy holds atoms, thresholds, patches and
                    # the node section (whole when many nodes changed), not the 48-B pod records
                    assert t.bytes_uploaded < n_rec_bytes // 2, (tick, t.bytes_uploaded, n_rec_bytes)
            lib.sr_snapshot_destroy(h)
        # C5: the added pods carry host ports, so the port conflict atoms change and K0 rewrites their columns
        assert reused == 14 and patched > 0 and k0_cols > 0 and (k0_less > 0 or config == 5), \
            (reused, patched, k0_cols, k0_less)
    finally:
        ck.close()


def test_ticks_alternating_clusters_and_interners(checker):
    """Static-view changes between ticks: two clusters in turn (different
    spot pools and specs), and the same random scenario encoded through two
    interners whose ids differ: no cached row, spec or taint set may leak
    from one into the other."""
    lib = capi.load_planner()
    a = SynthCluster(3, seed=31, n_on_demand=120, n_spot=300)
    b = SynthCluster(2, seed=32, n_on_demand=100, n_spot=250)
    plans = {}
    for sc in (a, b, a, b, a):
        nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
        cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
        h = _snapshot(lib, sc, nm)
        p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
        lib.sr_snapshot_destroy(h)
        o = oracle_plan(OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx), sc.ptr, cand_off,
                        cand_pods, mode=1, threads=8)
        assert np.array_equal(p.status, o["status"]) and np.array_equal(p.node_of_pod, o["node_of_pod"])
        plans.setdefault(id(sc), []).append(p.node_of_pod.copy())
    for runs in plans.values():
        assert all(np.array_equal(runs[0], r) for r in runs)
    nodes, spot_pods, cands = rand_scenario(777, n_spot=20, n_cand=10, max_pods=8)
    flat = [p for c in cands for p in c]
    first = None
    for warm in (Interner(), Interner()):
        for s in ("zone", "team", "type", "dedicated", "x", "a", "b"):  # shifts every later id
            warm.id("pad-" + s)
        sc = Scenario(nodes, spot_pods, flat, interner=warm)
        cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
        cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
        h = sc.product_snapshot()
        p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
        lib.sr_snapshot_destroy(h)
        o = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1)
        assert np.array_equal(p.status, o["status"]) and np.array_equal(p.node_of_pod, o["node_of_pod"])
        first = p if first is None else first
        assert np.array_equal(p.node_of_pod, first.node_of_pod)


def test_ticks_node_labels_and_taints_change(checker):
    """The same spot pool with one node's labels, then its taints changed:
    requirement rows and taint rows are rebuilt for the new static view."""
    lib = capi.load_planner()
    nodes, spot_pods, cands = rand_scenario(4242, n_spot=16, n_cand=10, max_pods=8)
    flat = [p for c in cands for p in c]
    cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    variants = [list(nodes)]
    import copy
    n2 = copy.deepcopy(nodes)
    n2[0].labels = dict(n2[0].labels, zone="b", team="a")
    variants.append(n2)
    n3 = copy.deepcopy(n2)
    n3[1].taints = n3[1].taints + [Taint("dedicated", "a", "NoSchedule")]
    n3[2].unschedulable = not n3[2].unschedulable
    variants.append(n3)
    variants.append(list(nodes))
    interner = Interner()
    for ns in variants:
        sc = Scenario(ns, spot_pods, flat, interner=interner)
        cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
        h = sc.product_snapshot()
        p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
        lib.sr_snapshot_destroy(h)
        o = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1)
        assert np.array_equal(p.status, o["status"]) and np.array_equal(p.node_of_pod, o["node_of_pod"])


@pytest.mark.parametrize("seed", range(6))
def test_ticks_with_pod_stamps(checker, seed):
    """sr_cluster.pod_stamp: the encoder keeps each stamped pod's spec id and candidate checks across calls.
    Ticks alternate between two versions of the candidate pods (specs, requests and accounting of some pods
    changed, with new stamps), then repeat a version with its old stamps; every tick equals the oracle, and a
    stamped tick equals the same tick without stamps."""
    import copy
    import random
    from spotplanner.model import Container
    nodes, spot_pods, cands = rand_scenario(9900 + seed, n_spot=12 + seed, n_cand=8, max_pods=6)
    r = random.Random(seed)
    alt = copy.deepcopy(cands)
    changed = []
    for ci, c in enumerate(alt):
        for pi, p in enumerate(c):
            if r.random() < 0.3:
                p.node_selector = {} if p.node_selector else {"zone": "z1"}
                p.containers = [Container(cpu_milli=p.containers[0].cpu_milli + 150 if p.containers else 150)]
                p.init_containers = [Container(cpu_milli=900)] if r.random() < 0.5 else []
                changed.append((ci, pi))
    n_spot_pods = sum(len(ps) for ps in spot_pods)

    def stamps_of(version, flat_len):  # distinct per seed: the planner is shared by the session's tests
        tag = (seed + 1) << 40
        base = [tag + 1000 + i for i in range(n_spot_pods)]
        flat = [(ci, pi) for ci, c in enumerate(cands) for pi in range(len(c))]
        return base + [tag + (5000 if version and k in changed else 3000) + i for i, k in enumerate(flat)][:flat_len]

    interner = Interner()  # one string dictionary per process: the stamps' contract
    for version in (0, 1, 0, 1, 1, 0):
        cs = alt if version else cands
        flat = [p for c in cs for p in c]
        for st in (stamps_of(version, len(flat)), None):
            sc = Scenario(nodes, spot_pods, flat, interner=interner, stamps=st)
            off = np.cumsum([0] + [len(c) for c in cs]).astype(np.int32)
            cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
            o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, cand_pods, mode=1)
            h = sc.product_snapshot()
            try:
                p = plan_arrays(checker, h, sc.ptr, off, cand_pods)
            finally:
                capi.load_planner().sr_snapshot_destroy(h)
            from test_gpu_parity import compare_plans
            compare_plans(o, p, off, None)


@pytest.mark.parametrize("config", [3, 5])
def test_ticks_kept_node_map_and_snapshot(checker, config):
    """A long-running planner's housekeeping ticks: the cluster changes between
    ticks (pods change requests, move, leave; stamps with them), the node map
    comes from the node map cache and the snapshot is the previous tick's,
    refreshed (sr_snapshot_refresh_cached, linked to the cache's node map:
    the nodes it found unchanged are kept without gathering their stamps;
    every third tick the plain sr_snapshot_refresh).  Every tick's node map
    equals the oracle's and every plan equals the oracle's on a snapshot built
    from scratch."""
    from oracle_lib import oracle_new_node_map
    sc = SynthCluster(config, seed=23, n_on_demand=200, n_spot=450)
    lib = capi.load_planner()
    cl = sc.cluster
    cpu = [np.ctypeslib.as_array(a, shape=(sc.n_pods,)) for a in
           (cl.pods.cpu_sort_milli, cl.pods.req_milli_cpu, cl.acc_milli_cpu) if a]
    node = np.ctypeslib.as_array(cl.pods.node, shape=(sc.n_pods,))
    stamps = np.ctypeslib.as_array(cl.pod_stamp, shape=(sc.n_pods,))
    saved = [a.copy() for a in cpu] + [node.copy(), stamps.copy()]
    cache = ctypes.c_void_p()
    assert lib.sr_node_map_cache_create(ctypes.byref(cache)) == capi.SR_OK
    rng = np.random.default_rng(config)
    h, rebuilt_total = None, 0
    try:
        for tick in range(10):
            if tick:
                for p in rng.integers(0, sc.n_pods, 6):
                    for a in cpu:
                        a[p] = max(0, int(a[p]) + int(rng.integers(-50, 200)))
                    stamps[p] += 2
                for p in rng.integers(0, sc.n_pods, 2):
                    node[p] = rng.integers(-1, sc.n_nodes)
                    stamps[p] += 2
            nm = new_node_map(lambda cp, pp, mp: lib.sr_new_node_map_cached(cache, cp, pp, mp, None), sc.ptr,
                              sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            orc = oracle_new_node_map(sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            for f in ("spot", "on_demand", "node_pod_off", "node_pod_idx", "requested_cpu"):
                assert np.array_equal(getattr(nm, f), getattr(orc, f)), (tick, f)
            args = (sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(nm.node_pod_off, capi.P32),
                    capi.ptr(nm.node_pod_idx, capi.P32))
            if h is None:
                h = ctypes.c_void_p()
                assert lib.sr_snapshot_create(*args, ctypes.byref(h)) == capi.SR_OK
            else:
                rebuilt = ctypes.c_int32()
                if tick % 3 == 2:
                    assert lib.sr_snapshot_refresh(h, *args, ctypes.byref(rebuilt)) == capi.SR_OK
                else:
                    assert lib.sr_snapshot_refresh_cached(h, cache, *args, ctypes.byref(rebuilt)) == capi.SR_OK
                rebuilt_total += rebuilt.value
            cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
            osnap = OracleSnapshot(sc.ptr, orc.spot, orc.node_pod_off, orc.node_pod_idx)
            p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
            o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
            assert np.array_equal(p.status, o["status"]), tick
            assert np.array_equal(p.node_of_pod, o["node_of_pod"]), tick
            assert p.winner == o["winner"], tick
        assert 0 < rebuilt_total < 9 * len(nm.spot) // 4, rebuilt_total  # only the changed nodes
    finally:
        for a, b in zip(cpu + [node, stamps], saved):
            a[:] = b
        if h is not None:
            lib.sr_snapshot_destroy(h)
        lib.sr_node_map_cache_destroy(cache)


@pytest.mark.parametrize("config", [3, 5])
def test_ticks_realistic_variant_reuse(checker, config):
    """The realistic variant (StatefulSet pods with EBS claims, init
    containers, GPU pods): the candidates read the spot nodes' scalar usage and
    attachable volumes.  Tick after tick pods on spot nodes change requests
    (stamps with them, the spot order moves), the snapshot is refreshed; the
    candidate side is reused (its scalar and volume-limit rows and shared
    scalar rows recomputed) and every plan equals the oracle's."""
    from spotplanner.synth import REALISTIC
    sc = SynthCluster(config, seed=24, n_on_demand=150, n_spot=400, **REALISTIC)
    lib = capi.load_planner()
    cl = sc.cluster
    cpu = [np.ctypeslib.as_array(a, shape=(sc.n_pods,)) for a in
           (cl.pods.cpu_sort_milli, cl.pods.req_milli_cpu, cl.acc_milli_cpu) if a]
    stamps = np.ctypeslib.as_array(cl.pod_stamp, shape=(sc.n_pods,))
    saved = [a.copy() for a in cpu] + [stamps.copy()]
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    spot_pods = np.concatenate([nm.node_pod_idx[nm.node_pod_off[n]:nm.node_pod_off[n + 1]] for n in nm.spot])
    rng = np.random.default_rng(config)
    h, reused = None, 0
    try:
        for tick in range(10):
            if tick:
                for p in rng.choice(spot_pods, 3):
                    for a in cpu:
                        a[p] = max(0, int(a[p]) + int(rng.integers(-100, 300)))
                    stamps[p] += 2
            nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            args = (sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(nm.node_pod_off, capi.P32),
                    capi.ptr(nm.node_pod_idx, capi.P32))
            if h is None:
                h = ctypes.c_void_p()
                assert lib.sr_snapshot_create(*args, ctypes.byref(h)) == capi.SR_OK
            else:
                assert lib.sr_snapshot_refresh(h, *args, None) == capi.SR_OK
            co, cp = build_candidates(nm, sc.pod_flags())
            assert np.array_equal(co, cand_off) and np.array_equal(cp, cand_pods)  # the on-demand side is untouched
            osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
            p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
            reused += checker.timing().enc_reused
            o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
            assert np.array_equal(p.status, o["status"]), tick
            assert np.array_equal(p.node_of_pod, o["node_of_pod"]), tick
            assert p.winner == o["winner"], tick
        assert reused >= 5, reused
    finally:
        for a, b in zip(cpu + [stamps], saved):
            a[:] = b
        if h is not None:
            lib.sr_snapshot_destroy(h)


def _with_extra(nm, n_nodes, extra):
    """node_pod_off / node_pod_idx with the (pod, spot position) pairs of
    `extra` appended to their spot nodes' lists (a pod of the cluster placed
    there as well, as sr_snapshot_add_pod does)."""
    add = {}
    for pod, pos in extra:
        add.setdefault(int(nm.spot[pos]), []).append(pod)
    off, idx = [0], []
    for n in range(n_nodes):
        idx.extend(nm.node_pod_idx[nm.node_pod_off[n]:nm.node_pod_off[n + 1]].tolist())
        idx.extend(add.get(n, []))
        off.append(len(idx))
    return np.asarray(off, np.int32), np.asarray(idx, np.int32)


@pytest.mark.parametrize("config", [2, 3])
def test_ticks_affinity_variant_reuse(checker, config):
    """The affinity variant (Deployments with hostname anti-affinity and zone
    DoNotSchedule spread): the candidates read the spot nodes' pods through
    the DA / DB rows, the spread rows and the domain path's base counts.  Tick
    after tick a fresh snapshot holds a changing set of extra replicas on
    random spot nodes (added a few at a time, dropped every fifth tick); the
    candidate side is reused (AntiReuse / SpreadReuse patch the changed nodes)
    and every plan equals the oracle's."""
    from spotplanner.synth import AFFINITY
    sc = SynthCluster(config, seed=31, n_on_demand=150, n_spot=400, **AFFINITY)
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    rng = np.random.default_rng(config)
    extra, reused = [], 0
    for tick in range(12):
        if tick % 5 == 4:
            extra.clear()
        for _ in range(int(rng.integers(1, 4))):
            extra.append((int(rng.choice(cand_pods)), int(rng.integers(len(nm.spot)))))
        off, idx = _with_extra(nm, sc.n_nodes, extra)
        h = ctypes.c_void_p()
        assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(off, capi.P32),
                                      capi.ptr(idx, capi.P32), ctypes.byref(h)) == capi.SR_OK
        try:
            osnap = OracleSnapshot(sc.ptr, nm.spot, off, idx)
            p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
            reused += checker.timing().enc_reused
            o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
            assert np.array_equal(p.status, o["status"]), tick
            assert np.array_equal(p.node_of_pod, o["node_of_pod"]), tick
            assert p.winner == o["winner"], tick
        finally:
            lib.sr_snapshot_destroy(h)
    assert reused >= 6, reused
