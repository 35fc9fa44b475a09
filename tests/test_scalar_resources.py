"""Scalar resources (extended resources, hugepages) and NodeInfo.AddPod's
accounting: the NodeResourcesFit ScalarResources loop behind CheckPredicates
(rescheduler.go:344; k8s v1.19.2 noderesources/fit.go fitsRequest, upstream,
not vendored: parity unpinned beyond the hand-derived answers here and in
tests/known_answer.py).

The planner encodes a pod's scalar checks as base-snapshot atoms.  That is
exact while no earlier pod of the same candidate can change the node's
Requested for the same name, so a candidate where two pods list one scalar
resource goes to the reference path, as does a pod whose AddPod accounting
differs from its fit request (init containers) when later pods of its
candidate follow it.  Checked on the oracle (CPU) and the GPU (C-ABI)."""
import ctypes

import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import load_oracle, oracle_plan
from randcluster import rand_scenario
from spotplanner import capi
from spotplanner.model import Container, GiB, Node, Pod

G = "nvidia.com/gpu"
OK, FB = capi.SR_CAND_OK, capi.SR_CAND_FALLBACK


def gpod(name, gpu=1, cpu=100, init_gpu=None, init_cpu=None):
    init = []
    if init_gpu is not None or init_cpu is not None:
        init = [Container(cpu_milli=init_cpu or 0, scalar={G: init_gpu} if init_gpu is not None else {})]
    return Pod(name, containers=[Container(cpu_milli=cpu, scalar={G: gpu} if gpu is not None else {})],
               init_containers=init)


def nodes3():
    return [Node("a", cpu_milli=4000, memory=8 * GiB, scalar={G: 1}),
            Node("b", cpu_milli=4000, memory=8 * GiB),
            Node("c", cpu_milli=4000, memory=8 * GiB, scalar={G: 4})]


def cases():
    """(name, spot pods, candidates, expected oracle statuses, expected mappings)"""
    yield ("one_gpu_pod", [[], [], []], [[gpod("p")]], [OK], [[0]])
    yield ("two_pods_share_a_name_fall_back", [[], [], []], [[gpod("p"), gpod("q")]], [FB], [[-1, -1]])
    yield ("different_names_are_independent", [[], [], []],
           [[gpod("p"), Pod("q", containers=[Container(cpu_milli=10, scalar={"hugepages-2Mi": 0})])]], [OK], [[0, 0]])
    yield ("base_usage_counts", [[gpod("u")], [], []], [[gpod("p")]], [OK], [[2]])
    yield ("listed_zero_with_zero_cpu_falls_back", [[], [], []], [[gpod("p", gpu=0, cpu=0)]], [FB], [[-1]])
    yield ("init_container_pod_before_others_falls_back", [[], [], []],
           [[Pod("i", containers=[Container(cpu_milli=100)], init_containers=[Container(cpu_milli=900)]),
             Pod("q", containers=[Container(cpu_milli=100)])]], [FB], [[-1, -1]])
    yield ("init_container_pod_last_is_planned", [[], [], []],
           [[Pod("q", containers=[Container(cpu_milli=100)]),
             Pod("i", containers=[Container(cpu_milli=100)], init_containers=[Container(cpu_milli=3950)])]],
           [OK], [[0, 1]])
    yield ("base_init_container_not_accounted", [[Pod("u", containers=[Container(cpu_milli=100)],
                                                      init_containers=[Container(cpu_milli=3900)])], [], []],
           [[Pod("q", containers=[Container(cpu_milli=3800)])]], [OK], [[0]])


@pytest.mark.parametrize("case", list(cases()), ids=lambda c: c[0])
def test_oracle_scalar_cases(case):
    _, spot_pods, cands, want_status, want_map = case
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes3(), spot_pods, flat)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32), mode=1)
    assert [int(x) for x in o["status"]] == want_status
    for k, m in enumerate(want_map):
        if want_status[k] != FB:
            assert [int(x) for x in o["node_of_pod"][off[k]:off[k + 1]]] == m


def test_oracle_without_scalar_tables_flags_and_tracks_unknown_usage():
    """A shim without scalar tables flags pods that list scalars
    (SR_POD_FB_SCALAR_RESOURCES); a snapshot holding such a pod does not know
    its node's scalar usage, so candidates asking for any scalar fall back
    while the others are planned."""
    from spotplanner.model import encode_cluster
    nodes = nodes3()
    spot_pods = [[gpod("u")], [], []]
    flat = [gpod("p"), Pod("q", containers=[Container(cpu_milli=100)])]
    pods = [p for ps in spot_pods for p in ps] + flat
    enc = encode_cluster(nodes, pods, pod_node=[0, -1, -1], scalar_tables=False)
    assert enc.a["flags"][0] & capi.SR_POD_FB_SCALAR_RESOURCES
    olib = load_oracle()
    from oracle_lib import OracleSnapshot
    snap = OracleSnapshot(enc.ptr, np.arange(3, dtype=np.int32), np.array([0, 1, 1, 1], np.int32),
                          np.array([0], np.int32))
    assert olib.oracle_find_spot_node_for_pod(snap.h, enc.ptr, 1) == -2
    assert olib.oracle_find_spot_node_for_pod(snap.h, enc.ptr, 2) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(cases()), ids=lambda c: c[0])
def test_gpu_scalar_cases(checker, case):
    from spotplanner.rescheduler import plan_arrays
    _, spot_pods, cands, want_status, want_map = case
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes3(), spot_pods, flat)
    off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, off, np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32))
    finally:
        capi.load_planner().sr_snapshot_destroy(h)
    assert [int(x) for x in p.status] == want_status
    for k, m in enumerate(want_map):
        if want_status[k] != FB:
            assert [int(x) for x in p.node_of_pod[off[k]:off[k + 1]]] == m


@pytest.mark.gpu
def test_gpu_without_scalar_tables(checker):
    from spotplanner.model import encode_cluster
    from spotplanner.rescheduler import plan_arrays
    nodes = nodes3()
    pods = [gpod("u"), gpod("p"), Pod("q", containers=[Container(cpu_milli=100)])]
    enc = encode_cluster(nodes, pods, pod_node=[0, -1, -1], scalar_tables=False)
    lib = capi.load_planner()
    h = ctypes.c_void_p()
    assert lib.sr_snapshot_create(enc.ptr, capi.ptr(np.arange(3, dtype=np.int32), capi.P32), 3,
                                  capi.ptr(np.array([0, 1, 1, 1], np.int32), capi.P32),
                                  capi.ptr(np.array([0], np.int32), capi.P32), ctypes.byref(h)) == capi.SR_OK
    try:
        p = plan_arrays(checker, h, enc.ptr, np.array([0, 1, 2], np.int32), np.array([1, 2], np.int32))
    finally:
        lib.sr_snapshot_destroy(h)
    assert [int(x) for x in p.status] == [FB, OK] and [int(x) for x in p.node_of_pod] == [-1, 0]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_gpu_random_scalar_clusters(checker, seed):
    """Scalar-heavy random clusters: every candidate the device plans equals the
    oracle; the fallback candidates are the oracle's."""
    from test_gpu_parity import run_scenario
    nodes, spot_pods, cands = rand_scenario(8800 + seed, n_spot=6 + seed % 15, n_cand=12, max_pods=5 + seed % 6)
    import random
    r = random.Random(seed)
    for n in nodes:  # most nodes carry GPUs, most candidates ask for one in a single pod
        if r.random() < 0.7:
            n.scalar = {G: r.choice([0, 1, 2, 4]), "hugepages-2Mi": r.choice([0, 4 << 20])}
    for c in cands:
        if c and r.random() < 0.7:
            p = c[r.randrange(len(c))]
            p.containers[0].scalar = {G: r.choice([0, 1, 2])}
            if p.containers[0].cpu_milli == 0:
                p.containers[0].cpu_milli = 10
    _, o, p = run_scenario(checker, nodes, spot_pods, cands)
    assert sum(int(s) != FB for s in p.status) >= 1
