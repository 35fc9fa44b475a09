"""Pins the CPU oracle against every golden vector of the reference's own tests
(tests/golden/reference_tests.json, transcribed from rescheduler_test.go and
nodes/nodes_test.go)."""
import ctypes

import numpy as np

from helpers import Scenario, fixture_node, fixture_pod, golden
from oracle_lib import load_oracle, oracle_new_node_map
from spotplanner import capi
from spotplanner.model import Interner, encode_cluster, label_flag

G = golden()


def _scenario(fx, queries):
    nodes = [fixture_node(s["node"]) for s in fx["spot"]]
    pods = [[fixture_pod(p) for p in s["pods"]] for s in fx["spot"]]
    return Scenario(nodes, pods, queries)


def test_find_spot_node_for_pod_golden():
    fx = G["TestFindSpotNodeForPod"]
    sc = _scenario(fx, [fixture_pod(q["pod"]) for q in fx["queries"]])
    snap = sc.oracle_snapshot()
    lib = load_oracle()
    names = [n.name for n in sc.nodes]
    for i, q in enumerate(fx["queries"]):
        pos = lib.oracle_find_spot_node_for_pod(snap.h, sc.ptr, sc.qidx(i))
        got = names[pos] if pos >= 0 else ""
        assert got == q["expect"], q


def test_can_drain_node_golden():
    fx = G["TestCanDrainNode"]
    calls = fx["calls"]
    q = [fixture_pod(p) for c in calls for p in c["pods"]]
    sc = _scenario(fx, q)
    snap = sc.oracle_snapshot()
    lib = load_oracle()
    names = [n.name for n in sc.nodes]
    base = 0
    for c in calls:  # one snapshot reused, no Fork/Revert (rescheduler_test.go:140-150)
        n = len(c["pods"])
        pods = np.arange(sc.qidx(base), sc.qidx(base) + n, dtype=np.int32)
        mapping = np.full(n, -1, np.int32)
        r = lib.oracle_can_drain_node(snap.h, sc.ptr, capi.ptr(pods, capi.P32), n, capi.ptr(mapping, capi.P32))
        assert (r == -1) == c["expect_ok"]
        if "derived_mapping" in c:
            assert [names[k] for k in mapping] == c["derived_mapping"]
        if "derived_fail_pod" in c:
            assert r == c["derived_fail_pod"]
        base += n


def _reactor_cluster(fx):
    nodes = [fixture_node(n) for n in fx["nodes"]]
    pods, pod_node = [], []
    for i, n in enumerate(nodes):
        for p in fx["pods_by_node"].get(n.name, []):
            pods.append(fixture_pod(p))
            pod_node.append(i)
    it = Interner()
    enc = encode_cluster(nodes, pods, it, pod_node=pod_node)
    return nodes, pods, enc, it


def test_new_node_map_golden():
    fx = G["TestNewNodeMap"]
    nodes, pods, enc, it = _reactor_cluster(fx)
    nm = oracle_new_node_map(enc.ptr, len(nodes), len(pods), label_flag(fx["on_demand_label"], it),
                             label_flag(fx["spot_label"], it))
    exp = fx["expect"]
    od = [(nodes[i].name, int(nm.node_pod_off[i + 1] - nm.node_pod_off[i])) for i in nm.on_demand]
    sp = [(nodes[i].name, int(nm.node_pod_off[i + 1] - nm.node_pod_off[i])) for i in nm.spot]
    assert od == [(e["name"], e["npods"]) for e in exp["on_demand"]]
    assert sp == [(e["name"], e["npods"]) for e in exp["spot"]]
    for i, n in enumerate(nodes):
        cpus = [pods[j].cpu_sort_milli() for j in nm.node_pod_idx[nm.node_pod_off[i]:nm.node_pod_off[i + 1]]]
        assert all(a >= b for a, b in zip(cpus, cpus[1:]))
        assert nm.requested_cpu[i] == exp["requested_cpu"][n.name]


def test_get_pods_on_node_golden():
    fx = G["TestGetPodsOnNode"]
    nodes, pods, enc, it = _reactor_cluster(fx)
    nm = oracle_new_node_map(enc.ptr, len(nodes), len(pods), label_flag("kubernetes.io/role=worker", it),
                             label_flag("kubernetes.io/role=spot-worker", it))
    for i, n in enumerate(nodes):
        kept = {pods[j].name for j in nm.node_pod_idx[nm.node_pod_off[i]:nm.node_pod_off[i + 1]]}
        assert kept == set(fx["expect_kept_list_order"][n.name])


def test_add_pod_and_requested_cpu_golden():
    fx = G["TestAddPod"]
    node = fixture_node(fx["node"])
    adds = [fixture_pod(a["pod"]) for a in fx["adds"]]
    sc = Scenario([node], [[]], adds)
    snap = sc.oracle_snapshot()
    lib = load_oracle()
    for i, a in enumerate(fx["adds"]):
        lib.oracle_snapshot_add_pod(snap.h, sc.ptr, sc.qidx(i), 0)
        req, npods = snap.node_state(0)
        assert req[0] == a["requested"] and node.cpu_milli - req[0] == a["free"] and npods == a["npods"]


def test_calculate_requested_cpu_golden():
    for case in G["TestCalculateRequestedCPU"]["cases"]:
        node = fixture_node({"name": "n", "cpu_milli": 2000, "memory": 1, "pods": 100,
                             "labels": {"kubernetes.io/role": "worker"}})
        pods = [fixture_pod({"name": "p%d" % i, "cpu_milli": c}) for i, c in enumerate(case["cpus"])]
        it = Interner()
        enc = encode_cluster([node], pods, it, pod_node=[0] * len(pods))
        nm = oracle_new_node_map(enc.ptr, 1, len(pods), label_flag("kubernetes.io/role=worker", it),
                                 label_flag("kubernetes.io/role=spot-worker", it))
        assert nm.requested_cpu[0] == case["expect"]
    for case in G["TestGetPodCPURequests"]["cases"]:
        assert fixture_pod({"name": "p", "cpu_milli": case["cpu"]}).cpu_sort_milli() == case["expect"]


def test_is_spot_and_on_demand_node_golden():
    lib = load_oracle()
    for key in ("TestIsSpotNode", "TestIsOnDemandNode"):
        fx = G[key]
        node = fixture_node({"name": "fooNode", "cpu_milli": 2000, "memory": 1, "pods": 100, "labels": fx["labels"]})
        for case in fx["cases"]:
            it = Interner()
            enc = encode_cluster([node], [], it)
            lab = label_flag(case["flag"], it)
            assert bool(lib.oracle_node_has_label(enc.ptr, 0, ctypes.byref(lab))) == case["expect"], case


def test_node_label_validation_golden():
    lib = load_oracle()
    for case in G["TestNodeLabelValidation"]["cases"]:
        ok = lib.oracle_validate_label_flag(len(case["on_demand"].split("="))) and \
            lib.oracle_validate_label_flag(len(case["spot"].split("=")))
        assert bool(ok) == (case["error"] is None)


def test_copy_node_infos_golden():
    # CopyNodeInfos is pure host bookkeeping: check the fixture's invariants hold
    # for the product's mirror (no GPU needed).
    from spotplanner.nodes import NodeInfo, NodeInfoArray
    fx = G["TestCopyNodeInfos"]
    arr = NodeInfoArray()
    for n in fx["nodes"]:
        node = fixture_node(n["node"])
        pods = [fixture_pod({"name": "p%d" % i, "cpu_milli": c}) for i, c in enumerate(n["cpus"])]
        arr.append(NodeInfo(node, pods, n["requested"], node.cpu_milli - n["requested"]))
    cp = arr.CopyNodeInfos()
    for ni in cp:
        ni.AddPod(fixture_pod({"name": "x", "cpu_milli": fx["add_cpu"]}))
    for orig, copy, n in zip(arr, cp, fx["nodes"]):
        assert len(copy.Pods) == len(n["cpus"]) + 1
        assert len(orig.Pods) == len(n["cpus"])
