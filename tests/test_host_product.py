"""CPU tests of the product's host side (no GPU): the C-ABI library loads and
exports every declared symbol, NewNodeMap (Go-exact sort.Slice, spot /
on-demand split, priority filter) matches the oracle, and the reference's
nodes_test.go golden vectors hold through the product's Python mirror."""
import ctypes

import numpy as np
import pytest

from helpers import fixture_node, fixture_pod, golden, header_functions
from oracle_lib import load_oracle, oracle_new_node_map
from spotplanner import capi
from spotplanner.model import Interner, encode_cluster, label_flag
from spotplanner.synth import SynthCluster, build_candidates, new_node_map

G = golden()


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(capi.PLANNER_LIB)
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(capi.EXPORTED) == declared
    capi.load_planner()  # argtypes for every symbol


def test_build_info_names_gfx950():
    assert b"gfx950" in capi.load_planner().sr_build_info()


def test_abi_version_matches_header_and_build_info():
    """the library reports the SR_ABI_VERSION it was built with (sr_abi_version and sr_build_info),
    and the binding refuses a library whose version differs from the header's."""
    lib = capi.load_planner()
    assert lib.sr_abi_version() == capi.SR_ABI_VERSION
    assert ("abi=%d " % capi.SR_ABI_VERSION).encode() in lib.sr_build_info()

    class Old:
        def sr_abi_version(self):
            return capi.SR_ABI_VERSION - 1
    import pytest
    with pytest.raises(capi.PlannerAbiMismatch):
        capi.check_abi(Old())


def test_sr_create_without_device_fails_loudly():
    import torch
    if torch.cuda.device_count() > 0:
        pytest.skip("a HIP device is present")
    lib = capi.load_planner()
    h = ctypes.c_void_p()
    assert lib.sr_create(0, ctypes.byref(h)) == capi.SR_ERR_NO_DEVICE


# ---------------------------------------------------------------- Go sort
def go_sort_py(a, less):
    """Third restatement of Go 1.16 sort.Slice (pure Python, small inputs)."""
    def lt(i, j):
        return less(a[i], a[j])

    def sw(i, j):
        a[i], a[j] = a[j], a[i]

    def ins(lo, hi):
        for i in range(lo + 1, hi):
            j = i
            while j > lo and lt(j, j - 1):
                sw(j, j - 1)
                j -= 1

    def sift(lo, hi, first):
        root = lo
        while True:
            child = 2 * root + 1
            if child >= hi:
                return
            if child + 1 < hi and lt(first + child, first + child + 1):
                child += 1
            if not lt(first + root, first + child):
                return
            sw(first + root, first + child)
            root = child

    def heap(lo, hi):
        first, n = lo, hi - lo
        for i in range((n - 1) // 2, -1, -1):
            sift(i, n, first)
        for i in range(n - 1, -1, -1):
            sw(first, first + i)
            sift(0, i, first)

    def med3(m1, m0, m2):
        if lt(m1, m0):
            sw(m1, m0)
        if lt(m2, m1):
            sw(m2, m1)
            if lt(m1, m0):
                sw(m1, m0)

    def pivot(lo, hi):
        m = (lo + hi) >> 1
        if hi - lo > 40:
            s = (hi - lo) // 8
            med3(lo, lo + s, lo + 2 * s)
            med3(m, m - s, m + s)
            med3(hi - 1, hi - 1 - s, hi - 1 - 2 * s)
        med3(lo, m, hi - 1)
        p, x, c = lo, lo + 1, hi - 1
        while x < c and lt(x, p):
            x += 1
        b = x
        while True:
            while b < c and not lt(p, b):
                b += 1
            while b < c and lt(p, c - 1):
                c -= 1
            if b >= c:
                break
            sw(b, c - 1)
            b += 1
            c -= 1
        protect = hi - c < 5
        if not protect and hi - c < (hi - lo) // 4:
            dups = 0
            if not lt(p, hi - 1):
                sw(c, hi - 1)
                c += 1
                dups += 1
            if not lt(b - 1, p):
                b -= 1
                dups += 1
            if not lt(m, p):
                sw(m, b - 1)
                b -= 1
                dups += 1
            protect = dups > 1
        if protect:
            while True:
                while x < b and not lt(b - 1, p):
                    b -= 1
                while x < b and lt(x, p):
                    x += 1
                if x >= b:
                    break
                sw(x, b - 1)
                x += 1
                b -= 1
        sw(p, b - 1)
        return b - 1, c

    def quick(lo, hi, depth):
        while hi - lo > 12:
            if depth == 0:
                heap(lo, hi)
                return
            depth -= 1
            mlo, mhi = pivot(lo, hi)
            if mlo - lo < hi - mhi:
                quick(lo, mlo, depth)
                lo = mhi
            else:
                quick(mhi, hi, depth)
                hi = mlo
        if hi - lo > 1:
            for i in range(lo + 6, hi):
                if lt(i, i - 6):
                    sw(i, i - 6)
            ins(lo, hi)

    n = len(a)
    depth, i = 0, n
    while i > 0:
        depth += 1
        i >>= 1
    quick(0, n, 2 * depth)
    return a


@pytest.mark.parametrize("n", [0, 1, 2, 5, 12, 13, 20, 40, 41, 64, 100, 257, 1000])
def test_oracle_go_sort_matches_python_restatement(n):
    lib = load_oracle()
    rng = np.random.default_rng(n)
    for trial in range(5):
        keys = rng.integers(0, max(2, n // (trial + 2)), size=n).astype(np.int64)  # tie-heavy
        for desc in (0, 1):
            ids = np.arange(n, dtype=np.int32)
            lib.oracle_go_sort_by_key(capi.ptr(ids, capi.P32), n, capi.ptr(keys, capi.P64), desc)
            want = go_sort_py(list(range(n)), (lambda x, y: keys[x] > keys[y]) if desc else
                              (lambda x, y: keys[x] < keys[y]))
            assert ids.tolist() == want
            if n:
                k = keys[ids]
                assert np.all(k[:-1] >= k[1:]) if desc else np.all(k[:-1] <= k[1:])


def test_go_sort_is_not_stable_on_ties():
    # The reason the product reproduces Go's algorithm instead of using a stable
    # sort: Go's sort.Slice permutes equal keys.
    keys = [1, 5, 5, 1] * 10
    order = go_sort_py(list(range(40)), lambda x, y: keys[x] > keys[y])
    fives = [i for i in order if keys[i] == 5]
    assert fives != sorted(fives)


# ------------------------------------------------------------ NewNodeMap
@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_product_new_node_map_matches_oracle(config):
    sc = SynthCluster(config)
    lib = capi.load_planner()
    prod = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    orc = oracle_new_node_map(sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    for f in ("spot", "on_demand", "node_pod_off", "node_pod_idx", "requested_cpu", "free_cpu"):
        assert np.array_equal(getattr(prod, f), getattr(orc, f)), f
    off, pods = build_candidates(prod, sc.pod_flags())
    assert len(off) - 1 == len(prod.on_demand)
    assert np.all(np.diff(off) >= 0)


def test_product_new_node_map_parallel_sort_matches_oracle():
    """Pools above 8,192 nodes: the product sorts the spot and on-demand
    lists (nodes/nodes.go:95-101) with Go's quickSort_func split over a thread
    pool (gosort.hpp go_sort_slice_parallel); tie-heavy RequestedCPU sums must
    still come out in the serial sort's exact order."""
    sc = SynthCluster(3, seed=41, n_on_demand=9000, n_spot=12000)
    lib = capi.load_planner()
    prod = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    orc = oracle_new_node_map(sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    assert len(prod.spot) > 8192 and len(prod.on_demand) > 8192
    assert len(np.unique(prod.requested_cpu[prod.spot])) < len(prod.spot) // 2  # ties everywhere
    for f in ("spot", "on_demand", "node_pod_off", "node_pod_idx", "requested_cpu"):
        assert np.array_equal(getattr(prod, f), getattr(orc, f)), f


def test_product_new_node_map_priority_threshold_matches_oracle():
    sc = SynthCluster(3, n_on_demand=200, n_spot=400)
    lib = capi.load_planner()
    for thr in (-5, 0, 1):
        prod = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label, thr)
        orc = oracle_new_node_map(sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label, thr)
        assert np.array_equal(prod.node_pod_idx, orc.node_pod_idx)
        assert np.array_equal(prod.spot, orc.spot)


def test_new_node_map_golden_through_product_api():
    from spotplanner import nodes as N
    fx = G["TestNewNodeMap"]

    class FakeClient:  # the reactor of nodes/nodes_test.go:387-450
        def list_pods(self, node_name):
            return [fixture_pod(p) for p in fx["pods_by_node"][node_name]]

    N.OnDemandNodeLabel, N.SpotNodeLabel = fx["on_demand_label"], fx["spot_label"]
    node_map = N.NewNodeMap(FakeClient(), [fixture_node(n) for n in fx["nodes"]])
    od, sp = node_map[N.OnDemand], node_map[N.Spot]
    assert [(n.Node.name, len(n.Pods)) for n in od] == [(e["name"], e["npods"]) for e in fx["expect"]["on_demand"]]
    assert [(n.Node.name, len(n.Pods)) for n in sp] == [(e["name"], e["npods"]) for e in fx["expect"]["spot"]]
    assert od[0].RequestedCPU <= od[1].RequestedCPU
    for ni in list(od) + list(sp):
        cpus = [N.getPodCPURequests(p) for p in ni.Pods]
        assert all(a >= b for a, b in zip(cpus, cpus[1:]))
        assert ni.RequestedCPU == fx["expect"]["requested_cpu"][ni.Node.name]


def test_get_pods_on_node_golden_through_product_api():
    from spotplanner import nodes as N
    fx = G["TestGetPodsOnNode"]

    class FakeClient:
        def list_pods(self, node_name):
            return [fixture_pod(p) for p in fx["pods_by_node"][node_name]]

    N.OnDemandNodeLabel, N.SpotNodeLabel, N.PriorityThreshold = \
        "kubernetes.io/role=worker", "kubernetes.io/role=spot-worker", 0
    for n in fx["nodes"]:
        got = [p.name for p in N.getPodsOnNode(FakeClient(), fixture_node(n))]
        assert got == fx["expect_kept_list_order"][n["name"]]


def test_is_spot_node_golden_through_product_api():
    from spotplanner import nodes as N
    for key, fn, glob in (("TestIsSpotNode", N.isSpotNode, "SpotNodeLabel"),
                          ("TestIsOnDemandNode", N.isOnDemandNode, "OnDemandNodeLabel")):
        fx = G[key]
        node = fixture_node({"name": "fooNode", "cpu_milli": 2000, "memory": 1, "pods": 100, "labels": fx["labels"]})
        for case in fx["cases"]:
            setattr(N, glob, case["flag"])
            assert fn(node) == case["expect"], case
    N.OnDemandNodeLabel, N.SpotNodeLabel = "kubernetes.io/role=worker", "kubernetes.io/role=spot-worker"


def test_label_flag_missing_key_reads_empty():
    # "k=" matches nodes WITHOUT key k: labels[k] of a missing key is "" (nodes/nodes.go:183).
    from spotplanner import nodes as N
    from spotplanner.model import Node
    N.SpotNodeLabel = "lifecycle="
    assert N.isSpotNode(Node("n", 1000, labels={}))
    assert not N.isSpotNode(Node("n", 1000, labels={"lifecycle": "spot"}))
    N.SpotNodeLabel = "kubernetes.io/role=spot-worker"


def test_validate_args_golden():
    from spotplanner.rescheduler import validateArgs
    for case in G["TestNodeLabelValidation"]["cases"]:
        err = validateArgs(case["on_demand"], case["spot"])
        assert (str(err) if err else None) == case["error"]


def test_nil_priority_panics_like_reference():
    from spotplanner import nodes as N
    from spotplanner.model import Container, Node, Pod

    class C:
        def list_pods(self, name):
            return [Pod("p", containers=[Container(100)], priority=None)]

    with pytest.raises(N.NilPriorityPanic):
        N.NewNodeMap(C(), [Node("n", 1000, labels={"kubernetes.io/role": "worker"})])


def test_snapshot_fork_revert_host():
    # ClusterSnapshot bookkeeping is host logic: Fork / AddPod / Revert restores state.
    from helpers import Scenario
    node = fixture_node({"name": "n1", "cpu_milli": 2000, "memory": 1 << 31, "pods": 100})
    sc = Scenario([node], [[fixture_pod({"name": "a", "cpu_milli": 300})]],
                  [fixture_pod({"name": "q", "cpu_milli": 500})])
    lib = capi.load_planner()
    h = sc.product_snapshot()
    req = np.zeros(3, np.int64)
    n = ctypes.c_int32()
    assert lib.sr_snapshot_fork(h) == capi.SR_OK
    assert lib.sr_snapshot_fork(h) == capi.SR_ERR_STATE
    lib.sr_snapshot_add_pod(h, sc.ptr, sc.qidx(0), 0)
    lib.sr_snapshot_node_state(h, 0, capi.ptr(req, capi.P64), ctypes.byref(n))
    assert req[0] == 800 and n.value == 2
    lib.sr_snapshot_revert(h)
    lib.sr_snapshot_node_state(h, 0, capi.ptr(req, capi.P64), ctypes.byref(n))
    assert req[0] == 300 and n.value == 1
    assert lib.sr_snapshot_revert(h) == capi.SR_OK
    lib.sr_snapshot_destroy(h)


def test_bench_plan_parity_rule():
    # bench.py's cpu_baseline parity: fallback candidates are the reference path's,
    # every device-evaluated candidate must match the oracle pod by pod.
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "bench_mod", os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    FB, OK = capi.SR_CAND_FALLBACK, capi.SR_CAND_OK
    cand_off = np.array([0, 2, 3, 5], np.int32)
    o = {"status": np.array([OK, 0, OK], np.int32), "node_of_pod": np.array([1, 2, -1, 0, 0], np.int32)}
    gpu_nodes = np.array([1, 2, -1, 0, 0], np.int32)
    assert bench.plan_parity(o, np.array([OK, 0, OK], np.int32), gpu_nodes, cand_off) == (True, 0, 0)
    assert bench.plan_parity(o, np.array([OK, FB, OK], np.int32), gpu_nodes, cand_off) == (True, 1, 1)
    assert not bench.plan_parity(o, np.array([OK, 0, FB + 10], np.int32), gpu_nodes, cand_off)[0]
    bad = gpu_nodes.copy()
    bad[4] = 1
    assert not bench.plan_parity(o, np.array([OK, 0, OK], np.int32), bad, cand_off)[0]
    assert bench.plan_parity(o, np.array([OK, 0, FB], np.int32), bad, cand_off) == (True, 1, 2)
