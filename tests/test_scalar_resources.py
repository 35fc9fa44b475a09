"""Scalar resources (extended resources, hugepages) and NodeInfo.AddPod's
accounting: the NodeResourcesFit ScalarResources loop behind CheckPredicates
(rescheduler.go:344; k8s v1.19.2 noderesources/fit.go fitsRequest, upstream,
not vendored: parity unpinned beyond the hand-derived answers here and in
tests/known_answer.py).

The planner encodes a pod's scalar checks as base-snapshot atoms, exact while
no earlier pod of the same candidate changes the node's Requested for the
same name.  A candidate where two pods list one scalar resource (up to two
such names), or where a pod whose AddPod accounting differs from its fit
request (init containers) is followed by others, is planned with extension
records: K2's running state per touched node subtracts the accounting
(calculateResource: regular containers + Overhead) and keeps the shared
scalars' free values.  Rules assumed (k8s v1.19.2, parity unpinned):
fitsRequest checks alloc[s] >= request[s] + requested[s] for every listed
name, the request being max(sum of containers, each init container) +
Overhead; NodeInfo.AddPod adds the containers' sum + Overhead only.
Checked on the oracle (CPU) and the GPU (C-ABI)."""
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



@pytest.fixture(params=["node_order", "pod_order"])
def checker(request, checker):
    """Every GPU case of this module under both K2 settings: the default
    (extension-record candidates on the node-order window kernel) and
    SR_K2_MODE=1 (pod order)."""
    return checker if request.param == "node_order" else request.getfixturevalue("podorder_checker")

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
    # a has one GPU: p takes it, q sees p's AddPod there and goes to c
    yield ("two_pods_share_a_name", [[], [], []], [[gpod("p"), gpod("q")]], [OK], [[0, 2]])
    # c's four GPUs hold four more; the sixth pod finds none left
    yield ("shared_name_runs_out", [[], [], []], [[gpod("p%d" % i) for i in range(5)]], [OK], [[0, 2, 2, 2, 2]])
    yield ("shared_name_exhausted_fails", [[], [], []], [[gpod("p%d" % i) for i in range(6)]], [5],
           [[0, 2, 2, 2, 2, -1]])
    # two GPUs per pod: a (1, used by u) never fits, c takes two pods, the third fits nowhere
    yield ("shared_name_two_each", [[gpod("u", gpu=1)], [], []],
           [[gpod("p", gpu=2), gpod("q", gpu=2)], [gpod("p", gpu=2), gpod("q", gpu=2), gpod("r", gpu=2)]],
           [OK, 2], [[2, 2], [2, 2, -1]])
    # an init container's GPU is in the fit request, not in AddPod's accounting: a fits both
    yield ("shared_name_init_container_not_accounted", [[], [], []],
           [[gpod("i", gpu=0, init_gpu=1), gpod("j", gpu=0, init_gpu=1)]], [OK], [[0, 0]])
    # two names in the running slots: hugepages listed with 0 on nodes allocating none still passes
    yield ("two_shared_names", [[], [], []],
           [[Pod("p", containers=[Container(cpu_milli=100, scalar={G: 1, "hugepages-2Mi": 0})]),
             Pod("q", containers=[Container(cpu_milli=100, scalar={G: 1, "hugepages-2Mi": 0})])]],
           [OK], [[0, 2]])
    # three names listed by two pods each: beyond the two running scalar slots
    yield ("three_shared_names_fall_back", [[], [], []],
           [[Pod("p", containers=[Container(cpu_milli=100, scalar={G: 1, "x.io/a": 1, "x.io/b": 1})]),
             Pod("q", containers=[Container(cpu_milli=100, scalar={G: 1, "x.io/a": 1, "x.io/b": 1})])]],
           [FB], [[-1, -1]])
    yield ("different_names_are_independent", [[], [], []],
           [[gpod("p"), Pod("q", containers=[Container(cpu_milli=10, scalar={"hugepages-2Mi": 0})])]], [OK], [[0, 0]])
    yield ("base_usage_counts", [[gpod("u")], [], []], [[gpod("p")]], [OK], [[2]])
    yield ("listed_zero_with_zero_cpu_falls_back", [[], [], []], [[gpod("p", gpu=0, cpu=0)]], [FB], [[-1]])
    # i fits a with its init container's 3950m but AddPod adds only 100m: q (3800m) still fits a
    # (subtracting the fit request instead would send q to b)
    yield ("init_container_pod_before_others", [[], [], []],
           [[Pod("i", containers=[Container(cpu_milli=100)], init_containers=[Container(cpu_milli=3950)]),
             Pod("q", containers=[Container(cpu_milli=3800)])]], [OK], [[0, 0]])
    # fit 3000m, accounting 1000m: two per 4000m node (a after one: 3000 free, after two: 2000 < 3000)
    yield ("init_container_pods_fill_a_node", [[], [], []],
           [[Pod("i%d" % k, containers=[Container(cpu_milli=1000)], init_containers=[Container(cpu_milli=3000)])
             for k in range(5)]], [OK], [[0, 0, 1, 1, 2]])
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


def init_and_gpu_scenario(seed):
    """Random clusters where most pods carry init containers (fit request !=
    AddPod accounting) and most candidates list one GPU name in several pods
    (a running scalar state per touched node), some hugepages too."""
    import random
    nodes, spot_pods, cands = rand_scenario(9100 + seed, n_spot=6 + seed % 20, n_cand=12, max_pods=4 + seed % 12,
                                            features=seed % 2 == 0)
    r = random.Random(seed)
    for n in nodes:
        if r.random() < 0.8:
            n.scalar = {G: r.choice([0, 1, 2, 4, 8]), "hugepages-2Mi": r.choice([0, 8 << 20])}
    for c in cands:
        gpu_cand = r.random() < 0.7
        for p in c:
            if r.random() < 0.5:
                p.init_containers = [Container(cpu_milli=r.choice([200, 1500, 3000]),
                                               memory=r.choice([0, 1 * GiB, 6 * GiB]),
                                               scalar={G: r.choice([1, 2])} if gpu_cand and r.random() < 0.3 else {})]
            if gpu_cand and r.random() < 0.6:
                p.containers[0].scalar = {G: r.choice([0, 1, 1, 2])}
                if r.random() < 0.2:
                    p.containers[0].scalar["hugepages-2Mi"] = r.choice([2 << 20, 4 << 20])
                if p.containers[0].cpu_milli == 0:
                    p.containers[0].cpu_milli = 10
    return nodes, spot_pods, cands


def test_oracle_plans_init_and_shared_scalar_candidates():
    """The extension cases are planned (not fallback) by the oracle for most candidates of the random clusters
    below, and some of them fail late (the running state matters)."""
    planned = shared = 0
    for seed in range(20):
        nodes, spot_pods, cands = init_and_gpu_scenario(seed)
        flat = [p for c in cands for p in c]
        sc = Scenario(nodes, spot_pods, flat)
        off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
        o = oracle_plan(sc.oracle_snapshot(), sc.ptr, off, np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32),
                        mode=1)
        for k, c in enumerate(cands):
            if int(o["status"][k]) == FB:
                continue
            planned += 1
            shared += sum(1 for p in c if any(G in ct.scalar for ct in p.containers + p.init_containers)) >= 2
    assert planned >= 120 and shared >= 40, (planned, shared)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(20))
def test_gpu_random_init_and_shared_scalar_candidates(checker, seed):
    """Init-container-heavy and GPU-sharing candidates on the device's extension records, bit-exact with the
    oracle (every status and every pod's node)."""
    from test_gpu_parity import run_scenario
    nodes, spot_pods, cands = init_and_gpu_scenario(seed)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.gpu
def test_gpu_large_extension_candidates(checker):
    """Extension records on candidates of 65-300 pods (pod order with 64 and 512 touched-node slots)."""
    from test_gpu_parity import run_scenario
    nodes = [Node("n%d" % i, cpu_milli=4000 + 1000 * (i % 5), memory=64 * GiB, scalar={G: 2 * (i % 4)})
             for i in range(160)]
    cands = []
    for npods in (65, 130, 300):
        c = []
        for k in range(npods):
            c.append(Pod("p%d_%d" % (npods, k), containers=[Container(cpu_milli=100 + 50 * (k % 7), scalar={G: 1})],
                         init_containers=[Container(cpu_milli=1500)] if k % 3 == 0 else []))
        cands.append(c)
    _, o, p = run_scenario(checker, nodes, [[] for _ in nodes], cands)
    assert all(int(s) != FB for s in o["status"])
