"""Parity of the HIP path (through the C-ABI) with the CPU oracle: bit-exact
drain plans (per-candidate status and the full pod -> spot node mapping),
findSpotNodeForPod answers and canDrainNode side effects, on seeded random
clusters, on the BASELINE.json synthetic configs and on edge cases."""
import ctypes

import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import OracleSnapshot, load_oracle, oracle_new_node_map, oracle_plan
from randcluster import rand_scenario
from spotplanner import capi
from spotplanner.model import Container, ContainerPort, GiB, Node, OwnerReference, Pod
from spotplanner.rescheduler import plan_arrays
from spotplanner.synth import SynthCluster, build_candidates, new_node_map

pytestmark = pytest.mark.gpu

OK, FB, EMPTY = capi.SR_CAND_OK, capi.SR_CAND_FALLBACK, capi.SR_CAND_EMPTY


def compare_plans(o, p, cand_off, extra_fallback=None):
    n = len(cand_off) - 1
    exp_ok, exp_fb = -1, -1
    for c in range(n):
        os_, ps = int(o["status"][c]), int(p.status[c])
        if os_ == FB:
            assert ps == FB, (c, os_, ps)
        elif ps == FB:
            assert extra_fallback is not None and extra_fallback(c), (c, os_, ps)
        else:
            assert ps == os_, (c, os_, ps)
            seg = slice(cand_off[c], cand_off[c + 1])
            assert np.array_equal(p.node_of_pod[seg], o["node_of_pod"][seg]), c
            if ps == OK and exp_ok < 0:
                exp_ok = c
        if ps == FB and exp_fb < 0:
            exp_fb = c
    assert p.first_ok == exp_ok
    assert p.first_fallback == exp_fb
    want_winner = exp_ok if exp_ok >= 0 and (exp_fb < 0 or exp_fb > exp_ok) else -1
    assert p.winner == want_winner
    if exp_ok >= 0:
        assert np.array_equal(p.winner_map, o["node_of_pod"][cand_off[exp_ok]:cand_off[exp_ok + 1]])


def run_scenario(checker, nodes, spot_pods, cands, extra_fallback=None):
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    o = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1)
    h = sc.product_snapshot()
    try:
        # winner only first (single rank: K2 writes each candidate's outcome to
        # the host and the run returns at the winner), then every output
        q = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods, full=False)
        p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
    finally:
        capi.load_planner().sr_snapshot_destroy(h)
    compare_plans(o, p, cand_off, extra_fallback)
    assert (q.first_ok, q.first_fallback, q.winner) == (p.first_ok, p.first_fallback, p.winner)
    assert np.array_equal(q.winner_map, p.winner_map)
    if np.array_equal(p.status, o["status"]):  # same candidates evaluated: the same reference-equivalent work
        assert p.checks == o["checks"]
    return sc, o, p


@pytest.mark.parametrize("seed", range(40))
def test_random_plans_match_oracle(checker, seed):
    nodes, spot_pods, cands = rand_scenario(seed, n_spot=6 + seed % 40, n_cand=10, max_pods=6 + seed % 10)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.parametrize("seed", range(10))
def test_random_plans_with_fallback_features(checker, seed):
    nodes, spot_pods, cands = rand_scenario(1000 + seed, n_spot=20, n_cand=12, max_pods=8, fallback=True)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.parametrize("seed", range(10))
def test_random_plans_resources_only(checker, seed):
    nodes, spot_pods, cands = rand_scenario(2000 + seed, n_spot=30, n_cand=16, max_pods=12, features=False)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.parametrize("seed", range(10))
def test_find_spot_nodes_match_oracle(checker, seed):
    nodes, spot_pods, cands = rand_scenario(3000 + seed, n_spot=25, n_cand=6, max_pods=10)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    osnap = sc.oracle_snapshot()
    olib = load_oracle()
    want = [olib.oracle_find_spot_node_for_pod(osnap.h, sc.ptr, sc.qidx(i)) for i in range(len(flat))]
    h = sc.product_snapshot()
    lib = capi.load_planner()
    idx = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    out = np.full(max(1, len(flat)), -7, np.int32)
    fb = np.zeros(max(1, len(flat)), np.uint8)
    assert lib.sr_find_spot_nodes(checker.handle, h, sc.ptr, capi.ptr(idx, capi.P32), len(flat),
                                  capi.ptr(out, capi.P32), capi.ptr(fb, capi.PU8)) == capi.SR_OK
    for i, w in enumerate(want):
        if w == -2:
            assert fb[i] == 1
        else:
            assert fb[i] == 0 and out[i] == w, (i, w, out[i], fb[i])
    lib.sr_snapshot_destroy(h)


@pytest.mark.parametrize("seed", range(8))
def test_can_drain_node_sequence_mutates_like_oracle(checker, seed):
    """Several canDrainNode calls on ONE snapshot, without Fork/Revert
    (rescheduler_test.go:140-150): results and snapshot state stay equal."""
    nodes, spot_pods, cands = rand_scenario(4000 + seed, n_spot=10, n_cand=6, max_pods=6)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    osnap = sc.oracle_snapshot()
    olib = load_oracle()
    h = sc.product_snapshot()
    lib = capi.load_planner()
    base = sc.q0
    for c in cands:
        n = len(c)
        pods = np.arange(base, base + n, dtype=np.int32)
        base += n
        omap = np.full(max(n, 1), -1, np.int32)
        r = olib.oracle_can_drain_node(osnap.h, sc.ptr, capi.ptr(pods, capi.P32), n, capi.ptr(omap, capi.P32))
        pmap = np.full(max(n, 1), -1, np.int32)
        fail = ctypes.c_int32()
        fb = ctypes.c_uint8()
        assert lib.sr_can_drain_node(checker.handle, h, sc.ptr, capi.ptr(pods, capi.P32), n,
                                     capi.ptr(pmap, capi.P32), ctypes.byref(fail), ctypes.byref(fb)) == capi.SR_OK
        if r == -2:
            assert fb.value == 1
            continue
        assert fb.value == 0
        assert fail.value == r
        assert np.array_equal(pmap[:n], omap[:n])
        for pos in range(len(nodes)):
            req = np.zeros(3, np.int64)
            k = ctypes.c_int32()
            lib.sr_snapshot_node_state(h, pos, capi.ptr(req, capi.P64), ctypes.byref(k))
            assert (tuple(req), k.value) == osnap.node_state(pos)
    lib.sr_snapshot_destroy(h)


@pytest.mark.parametrize("seed", range(30))
def test_random_plans_with_pod_anti_affinity(checker, seed):
    """Required pod anti-affinity (static base conflicts, state-bit pairs
    between the pods of a candidate on node-local keys, the domain path on
    shared keys): every candidate planned on the device, no fallback."""
    nodes, spot_pods, cands = rand_scenario(6000 + seed, n_spot=8 + seed % 12, n_cand=10, max_pods=4 + seed % 8,
                                            features=seed % 3 != 0, anti=0.3 + 0.02 * seed)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.parametrize("seed", range(30))
def test_random_plans_with_pod_affinity(checker, seed):
    """Required pod affinity (static SAT / KEYS rows per term set) together with
    anti-affinity; candidates whose pods interact through an affinity set or
    an anti-affinity term on a shared key are planned on the domain path."""
    nodes, spot_pods, cands = rand_scenario(6600 + seed, n_spot=8 + seed % 14, n_cand=10, max_pods=3 + seed % 7,
                                            features=seed % 2 == 0, anti=0.15, aff=0.25 + 0.02 * seed)
    run_scenario(checker, nodes, spot_pods, cands)


def test_pod_anti_affinity_exercises_the_state_bits(checker):
    """Some seeds above must plan candidates whose pods interact through the
    hostname (the state-bit path), not only static conflicts or fallbacks."""
    from randcluster import HOST, term_selects
    hits = 0
    for seed in range(30):
        nodes, spot_pods, cands = rand_scenario(6000 + seed, n_spot=8 + seed % 12, n_cand=10,
                                                max_pods=4 + seed % 8, features=seed % 3 != 0,
                                                anti=0.3 + 0.02 * seed)
        for c in cands:
            hits += any(t.topology_key == HOST and any(j != i and term_selects(a, t, b) for j, b in enumerate(c))
                        for i, a in enumerate(c) for t in a.pod_anti_affinity or [])
    assert hits >= 20


def test_replicas_spread_by_hostname_anti_affinity(checker):
    from spotplanner.model import LabelSelector, PodAffinityTerm
    HOST = "kubernetes.io/hostname"
    nodes = [Node(name="n%d" % i, cpu_milli=4000, memory=8 * GiB, pods=110, labels={HOST: "n%d" % i})
             for i in range(3)]
    t = [PodAffinityTerm(HOST, LabelSelector({"app": "web"}))]
    reps = [Pod(name="r%d" % i, namespace="default", containers=[Container(cpu_milli=100)],
                labels={"app": "web"}, pod_anti_affinity=t) for i in range(4)]
    other = Pod(name="x", namespace="default", containers=[Container(cpu_milli=100)], labels={"app": "db"})
    _, o, p = run_scenario(checker, nodes, [[], [], []], [reps[:3] + [other], reps])
    assert list(p.status) == [OK, 3]
    assert list(p.node_of_pod[:4]) == [0, 1, 2, 0]


@pytest.mark.parametrize("seed", range(6))
def test_find_spot_nodes_with_pod_anti_affinity(checker, seed):
    nodes, spot_pods, cands = rand_scenario(7000 + seed, n_spot=15, n_cand=6, max_pods=10, anti=0.5)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    osnap = sc.oracle_snapshot()
    olib = load_oracle()
    want = [olib.oracle_find_spot_node_for_pod(osnap.h, sc.ptr, sc.qidx(i)) for i in range(len(flat))]
    h = sc.product_snapshot()
    lib = capi.load_planner()
    idx = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    out = np.full(max(1, len(flat)), -7, np.int32)
    fb = np.zeros(max(1, len(flat)), np.uint8)
    assert lib.sr_find_spot_nodes(checker.handle, h, sc.ptr, capi.ptr(idx, capi.P32), len(flat),
                                  capi.ptr(out, capi.P32), capi.ptr(fb, capi.PU8)) == capi.SR_OK
    for i, w in enumerate(want):
        if w == -2:
            assert fb[i] == 1, i
        else:
            assert fb[i] == 0 and out[i] == w, (i, w, out[i], fb[i])  # one pod: nothing interacts
    lib.sr_snapshot_destroy(h)


@pytest.mark.parametrize("seed", range(6))
def test_can_drain_node_sequence_with_pod_anti_affinity(checker, seed):
    """canDrainNode calls on ONE snapshot: the pods placed by earlier calls
    (and their terms) are base pods of the later ones."""
    nodes, spot_pods, cands = rand_scenario(8000 + seed, n_spot=10, n_cand=6, max_pods=6, anti=0.5)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    osnap = sc.oracle_snapshot()
    olib = load_oracle()
    h = sc.product_snapshot()
    lib = capi.load_planner()
    base = sc.q0
    for c in cands:
        n = len(c)
        pods = np.arange(base, base + n, dtype=np.int32)
        base += n
        omap = np.full(max(n, 1), -1, np.int32)
        r = olib.oracle_can_drain_node(osnap.h, sc.ptr, capi.ptr(pods, capi.P32), n, capi.ptr(omap, capi.P32))
        pmap = np.full(max(n, 1), -1, np.int32)
        fail = ctypes.c_int32()
        fb = ctypes.c_uint8()
        assert lib.sr_can_drain_node(checker.handle, h, sc.ptr, capi.ptr(pods, capi.P32), n,
                                     capi.ptr(pmap, capi.P32), ctypes.byref(fail), ctypes.byref(fb)) == capi.SR_OK
        if r == -2:
            assert fb.value == 1
            continue
        assert fb.value == 0
        assert fail.value == r
        assert np.array_equal(pmap[:n], omap[:n])
    lib.sr_snapshot_destroy(h)


@pytest.mark.parametrize("seed", range(8))
def test_random_large_candidates(checker, seed):
    # 65..300 pods per candidate: K2's node-order path with 2 and 4 pod groups
    # (a failing pod in any group) and, above 256 pods, the pod-order path
    nodes, spot_pods, cands = rand_scenario(5000 + seed, n_spot=20 + 5 * seed, n_cand=4, max_pods=70 + 33 * seed,
                                            features=seed % 2 == 0)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.parametrize("seed", range(4))
def test_random_large_candidates_with_pod_anti_affinity(checker, seed):
    # the state-bit pairs through 2 and 4 pod groups and the pod-order path
    nodes, spot_pods, cands = rand_scenario(5100 + seed, n_spot=40 + 10 * seed, n_cand=4, max_pods=70 + 66 * seed,
                                            features=False, anti=0.15, hostname_only=True)
    run_scenario(checker, nodes, spot_pods, cands)


def test_pod_order_mode_matches_oracle():
    # SR_K2_MODE=1 forces K2's pod-order path everywhere (the A/B arm of the bench)
    import os
    from spotplanner.planner import PredicateChecker
    os.environ["SR_K2_MODE"] = "1"
    try:
        c = PredicateChecker(0)
    finally:
        del os.environ["SR_K2_MODE"]
    try:
        for seed in range(6):
            nodes, spot_pods, cands = rand_scenario(6000 + seed, n_spot=8 + 7 * seed, n_cand=8, max_pods=12)
            run_scenario(c, nodes, spot_pods, cands)
        for seed in range(10):  # anti-affinity state bits through the pod-order placement
            nodes, spot_pods, cands = rand_scenario(6100 + seed, n_spot=8 + 3 * seed, n_cand=10, max_pods=10,
                                                    anti=0.5)
            run_scenario(c, nodes, spot_pods, cands)
        tick_parity(c, SynthCluster(3, seed=13, n_on_demand=300, n_spot=900))
    finally:
        c.close()


# ------------------------------------------------------------------ edge cases
def test_no_spot_nodes(checker):
    cands = [[Pod("a", containers=[Container(100)])], [], [Pod("z", containers=[Container(0)])]]
    _, o, p = run_scenario(checker, [], [], cands)
    assert list(p.status) == [0, EMPTY, 0]


def test_no_candidates(checker):
    node = Node("n0", 1000)
    _, o, p = run_scenario(checker, [node], [[]], [])
    assert p.winner == -1 and p.first_ok == -1


def test_zero_request_pods_skip_resource_checks(checker):
    # overcommitted node: a zero-request pod still fits (only the pod count is checked)
    node = Node("n0", 1000, pods=3)
    spot = [[Pod("big", containers=[Container(5000)])]]
    cands = [[Pod("z1", containers=[Container(0)]), Pod("z2", containers=[Container(0)]),
              Pod("z3", containers=[Container(0)])], [Pod("c", containers=[Container(1)])]]
    _, o, p = run_scenario(checker, [node], spot, cands)
    assert list(p.status) == [2, 0]  # third zero pod exceeds allocatable pods (3)


def test_intra_candidate_host_port_conflict(checker):
    nodes = [Node("n0", 4000), Node("n1", 4000)]
    mk = lambda name: Pod(name, containers=[Container(100, ports=[ContainerPort(80)])])
    cands = [[mk("a"), mk("b"), mk("c")]]
    _, o, p = run_scenario(checker, nodes, [[], []], cands)
    assert list(p.status) == [2]
    assert list(p.node_of_pod) == [0, 1, -1]


@pytest.mark.parametrize("seed", range(8))
def test_gpu_exclusive_port_candidates(checker, seed):
    """Candidates whose pods all ask for one host port (no two can share a
    node: K2's taken-mask step, place_window32 X) next to ones with mixed ports
    and host IPs (the regular step), 5-160 pods over several windows, spot
    nodes already using the port or full, uneven requests: against the oracle."""
    import random
    r = random.Random(4400 + seed)
    n = r.randint(60, 220)
    nodes = [Node("n%d" % i, r.choice([500, 1000, 2000, 4000]), memory=r.choice([1, 2, 4]) * GiB,
                  pods=r.choice([2, 5, 110])) for i in range(n)]
    port = lambda p_, ip="": ContainerPort(p_, host_ip=ip)  # noqa: E731
    spot = [[Pod("s%d_%d" % (i, k), containers=[Container(r.choice([50, 400, 900]),
                                                          ports=[port(80)] if r.random() < 0.15 else [])])
             for k in range(r.randint(0, 2))] for i in range(n)]
    cands = []
    for c in range(6):
        m = r.randint(5, 160)
        excl = c % 2 == 0
        pods = []
        for k in range(m):
            ports = [port(80)] if excl else ([port(r.choice([80, 443]), r.choice(["", "10.0.0.1"]))]
                                             if r.random() < 0.6 else [])
            if excl and r.random() < 0.3:
                ports.append(port(9100))  # a second port, still exclusive through port 80
            pods.append(Pod("c%d_%d" % (c, k), containers=[Container(r.choice([0, 10, 100, 700]),
                                                                     memory=r.choice([0, 64, 512]) * 2 ** 20,
                                                                     ports=ports)]))
        cands.append(pods)
    run_scenario(checker, nodes, spot, cands)


def test_host_ip_conflicts_inside_a_candidate(checker):
    # HostPortInfo.CheckConflict between the candidate's own pods and the base
    # UsedPorts: 0.0.0.0 conflicts with every IP of (protocol, port), a
    # specific IP with 0.0.0.0 and itself
    nodes = [Node("n0", 4000), Node("n1", 4000), Node("n2", 4000)]
    mk = lambda name, ip="", port=80, proto="TCP": Pod(name, containers=[Container(100, ports=[  # noqa: E731
        ContainerPort(port, protocol=proto, host_ip=ip)])])
    spot = [[mk("base", "10.0.0.1")], [], []]
    cands = [[mk("a", "10.0.0.2"), mk("b"), mk("c", "10.0.0.1"), mk("d", "10.0.0.1"), mk("e", proto="UDP")],
             [mk("f", "10.0.0.3"), mk("g", "10.0.0.3"), mk("h", "10.0.0.3"), mk("i", "10.0.0.3")]]
    _, o, p = run_scenario(checker, nodes, spot, cands)
    assert list(p.status) == [3, 3]
    assert list(p.node_of_pod[:5]) == [0, 1, 2, -1, -1]
    assert list(p.node_of_pod[5:]) == [0, 1, 2, -1]


def test_more_than_128_touched_nodes(checker):
    # every spot node has room for exactly one more pod: 200 pods touch 200 nodes
    nodes = [Node("n%d" % i, 1000, pods=1) for i in range(260)]
    cands = [[Pod("p%d" % k, containers=[Container(10)]) for k in range(200)],
             [Pod("q%d" % k, containers=[Container(10)]) for k in range(300)]]
    _, o, p = run_scenario(checker, nodes, [[] for _ in nodes], cands)
    assert p.status[0] == OK and p.status[1] == 260
    assert list(p.node_of_pod[:200]) == list(range(200))


@pytest.mark.parametrize("n_touch", [63, 64, 65, 129])
def test_touched_slot_boundaries(checker, n_touch):
    # K2 keeps 64 touched-node slots in registers and reruns a candidate that
    # needs more with 512: both sides of the boundary, plus pods that keep
    # landing on already-touched nodes afterwards
    nodes = [Node("n%d" % i, 1000, pods=1) for i in range(n_touch)] + [Node("big", 100000)]
    pods = [Pod("p%d" % k, containers=[Container(10)]) for k in range(n_touch + 20)]
    _, o, p = run_scenario(checker, nodes, [[] for _ in nodes], [pods, pods[:5]])
    assert p.status[0] == OK and p.status[1] == OK
    assert list(p.node_of_pod[:n_touch + 20]) == list(range(n_touch)) + [n_touch] * 20


def test_many_chunks_of_spot_nodes(checker):
    # > 4096 spot nodes: bitmask rows span several 64-word chunks
    nodes = [Node("n%d" % i, 100) for i in range(9000)] + [Node("big", 10000)]
    cands = [[Pod("a", containers=[Container(500)]), Pod("b", containers=[Container(50)])]]
    _, o, p = run_scenario(checker, nodes, [[] for _ in nodes], cands)
    assert list(p.node_of_pod) == [9000, 0]


@pytest.mark.parametrize("seed", range(6))
def test_wide_pool_sparse_capacity(checker, seed):
    # rows of 133 words (three 64-word chunks): capacity only on scattered nodes,
    # some right at the chunk boundaries, so pods resolve beyond the head, run
    # out of a chunk's mask and move on to the next chunk
    import random
    r = random.Random(seed)
    n = 2 * 4096 + 300
    big = set(r.sample(range(n), 40)) | {511, 512, 4095, 4096, 4097, 8191, 8192, n - 1}
    if seed % 2:
        big -= set(range(0, 512))  # nothing in the head: every pod starts unresolved
    nodes = [Node("n%d" % i, r.choice([1000, 1500, 2500]) if i in big else 100) for i in range(n)]
    cands = []
    for c in range(8):
        cands.append([Pod("c%d_%d" % (c, k), containers=[Container(r.choice([200, 400, 600, 900]))])
                      for k in range(r.randint(3, 40))])
    run_scenario(checker, nodes, [[] for _ in nodes], cands)


@pytest.mark.parametrize("seed", range(4))
def test_wide_pool_random_features(checker, seed):
    # every encoded feature (selectors, node affinity, taints, host ports,
    # anti-affinity state bits) on pools of 4,100-9,000 nodes: sparse S rows
    # beyond the head and across chunk boundaries
    nodes, spot_pods, cands = rand_scenario(7300 + seed, n_spot=4100 + 1600 * seed, n_cand=10, max_pods=20,
                                            anti=0.2, hostname_only=True)
    run_scenario(checker, nodes, spot_pods, cands)


@pytest.mark.parametrize("head_only", [0, 1])
def test_wide_pool_head_only_s_rows(head_only):
    # SR_S_HEAD_ONLY=1 (the default on rows wider than 64 words): K0 writes only
    # the heads of the S rows and K2 evaluates the rest from the class programs
    import os
    from spotplanner.planner import PredicateChecker
    os.environ["SR_S_HEAD_ONLY"] = str(head_only)
    try:
        c = PredicateChecker(0)
    finally:
        del os.environ["SR_S_HEAD_ONLY"]
    try:
        for seed in range(6):
            nodes, spot_pods, cands = rand_scenario(7400 + seed, n_spot=4200 + 900 * seed, n_cand=10, max_pods=24)
            run_scenario(c, nodes, spot_pods, cands)
        tick_parity(c, SynthCluster(4, seed=5, n_on_demand=400, n_spot=6000))
    finally:
        c.close()


# ------------------------------------------------------------ synthetic configs
def tick_parity(checker, sc: SynthCluster, max_cands=None, oracle_threads=8):
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    if max_cands is not None:
        cand_off = cand_off[: max_cands + 1]
        cand_pods = cand_pods[: cand_off[-1]]
    h = ctypes.c_void_p()
    assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                  capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                  ctypes.byref(h)) == capi.SR_OK
    q = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods, full=False)  # winner only (returns at the winner)
    p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
    lib.sr_snapshot_destroy(h)
    assert (q.first_ok, q.first_fallback, q.winner) == (p.first_ok, p.first_fallback, p.winner)
    assert np.array_equal(q.winner_map, p.winner_map)
    osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
    o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=oracle_threads)
    compare_plans(o, p, cand_off)
    assert np.array_equal(p.status, o["status"])  # nothing outside the encoded set in the synthetic configs
    assert p.checks == o["checks"]
    return o, p


@pytest.mark.parametrize("config", [1, 2, 3, 5])
def test_synthetic_config_plans_match_oracle(checker, config):
    o, p = tick_parity(checker, SynthCluster(config))
    assert p.checks > 0


def test_synthetic_config3_other_seeds(checker):
    for seed in (11, 12):
        tick_parity(checker, SynthCluster(3, seed=seed, n_on_demand=500, n_spot=1200, pinned_fraction=0.05))


def test_synthetic_config4_full_tick(checker):
    # BASELINE C4 as defined: every one of the 15,000 on-demand candidates of the
    # 50k-node / 1.5M-pod cluster in one tick, over the 35k-node spot pool
    # (9 chunks per row: the pod-order K2), against the multi-threaded oracle
    import os
    sc = SynthCluster(4)
    o, p = tick_parity(checker, sc, oracle_threads=min(16, os.cpu_count() or 8))
    assert len(p.status) == 15000 and np.sum(p.status == OK) > 0


def test_rccl_single_rank_collective_path_matches(checker):
    """The multi-GPU tick (K0 + K2, ncclAllReduce(min) of d_min over RCCL, K3
    on the owning rank) run with a one-rank communicator: same plan as the
    single-GPU path.  The sharding itself is covered with gloo at world sizes
    2 and 3 (test_distributed.py)."""
    from spotplanner.planner import PredicateChecker
    nodes, spot_pods, cands = rand_scenario(9100, n_spot=30, n_cand=20, max_pods=10)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    lib = capi.load_planner()
    h = sc.product_snapshot()
    comm_checker = PredicateChecker(0)
    try:
        uid = (ctypes.c_uint8 * capi.SR_UNIQUE_ID_BYTES)()
        assert lib.sr_comm_unique_id(uid) == capi.SR_OK
        assert lib.sr_comm_init(comm_checker.handle, uid, 1, 0) == capi.SR_OK, comm_checker.last_error()
        want = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
        got = plan_arrays(comm_checker, h, sc.ptr, cand_off, cand_pods)
        assert (got.winner, got.first_ok, got.first_fallback) == (want.winner, want.first_ok, want.first_fallback)
        assert np.array_equal(got.status, want.status)
        assert np.array_equal(got.node_of_pod, want.node_of_pod)
        assert np.array_equal(got.winner_map, want.winner_map)
        # the split prepare / run form the bench times goes through the collective too
        c = capi.sr_candidates(len(cand_off) - 1, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32), None)
        assert lib.sr_plan_prepare(comm_checker.handle, h, sc.ptr, ctypes.byref(c)) == capi.SR_OK
        wmap = np.full(max(1, int(np.max(np.diff(cand_off)))), -1, np.int32)
        out = capi.sr_plan_out()
        out.winner_map = capi.ptr(wmap, capi.P32)
        for _ in range(3):
            assert lib.sr_plan_run(comm_checker.handle, ctypes.byref(out)) == capi.SR_OK, comm_checker.last_error()
            assert out.winner == want.winner
            assert np.array_equal(wmap[:out.winner_npods], want.winner_map)
    finally:
        comm_checker.close()
        lib.sr_snapshot_destroy(h)


def test_many_deployments_with_hostname_anti_affinity(checker):
    """A cluster shaped like production anti-affinity use: 120 Deployments,
    each spreading its replicas one per host (required anti-affinity on
    kubernetes.io/hostname selecting its own app label), on spot and
    on-demand nodes alike; some Deployments also keep away from a database.
    Exercises the term index, the static DA/DB sets and the state-bit pairs
    with many distinct terms (more than the 32 pairs: candidates needing more
    fall back, the rest must match the oracle)."""
    import random
    from spotplanner.model import LabelSelector, PodAffinityTerm
    HOST = "kubernetes.io/hostname"
    r = random.Random(77)
    nodes = [Node(name="n%d" % i, cpu_milli=r.choice([2000, 4000, 8000]), memory=64 * GiB, pods=110,
                  labels={HOST: "n%d" % i}) for i in range(150)]

    def replica(app, i):
        anti = [PodAffinityTerm(HOST, LabelSelector({"app": app}))]
        if r.random() < 0.2:
            anti.append(PodAffinityTerm(HOST, LabelSelector({"app": "db"})))
        return Pod(name="%s-%d" % (app, i), namespace="default", labels={"app": app},
                   containers=[Container(cpu_milli=r.choice([100, 250, 500]), memory=r.choice([1, 2]) * GiB)],
                   pod_anti_affinity=anti if r.random() < 0.9 else None)

    apps = ["app%d" % k for k in range(120)] + ["db"]
    hot = apps[:10]  # the Deployments being drained also crowd the first spot nodes
    spot_pods = [[] for _ in nodes]
    for n in range(len(nodes)):
        for k in range(r.randint(4, 12)):
            spot_pods[n].append(replica(r.choice(hot if r.random() < 0.6 else apps), 100 * n + k))
    cands = []
    for c in range(60):  # 1-3 Deployments per on-demand node, 2-5 replicas each
        cands.append([replica(a, 100000 + 100 * c + 10 * j + k) for j, a in enumerate(r.sample(hot, r.randint(1, 3)))
                      for k in range(r.randint(2, 5))])
    _, o, p = run_scenario(checker, nodes, spot_pods, cands)
    assert len(set(int(x) for x in p.node_of_pod if x >= 0)) > 8  # conflicts push replicas past the first nodes


# ------------------------------------------- node order: 32-bit scaled run passes
def _granular_scenario(seed: int):
    """Many small pods onto few nodes (run passes of several pods), with request
    granularities that do and do not allow the scaled 32-bit sums: MiB multiples,
    odd byte counts, scaled values at the 2^26 limit (run passes) and the 2^23
    limit (window visits), nodes whose scaled free memory is clamped at 2^31 - 1
    (window visits), sums landing exactly on a node's free value (not itself a
    multiple of the granularity), and overcommitted nodes (negative free
    values)."""
    import random
    r = random.Random(seed)
    mode = seed % 6
    unit = {0: 1 << 20, 1: 1, 2: 1 << 20, 3: 3, 4: 1 << 20, 5: 1 << 20}[mode]
    n_spot = 3 + seed % 5
    nodes = []
    for i in range(n_spot):
        mem = r.choice([1, 2, 4]) * GiB + r.choice([0, 1, 12345])
        if mode == 2:
            mem = (1 << 46) + r.choice([0, 1, 1 << 20])  # scaled by 2^20: just around 2^26
        elif mode >= 4:
            mem = r.choice([1 << 52, (1 << 51) - 1, (1 << 30) + 5])  # scaled by 2^20: around and above 2^31
        nodes.append(Node(name="n%d" % i, cpu_milli=r.choice([1000, 2000, 4001]), memory=mem, pods=110,
                          ephemeral=r.choice([0, 10 * GiB + 7]), labels={"kubernetes.io/hostname": "n%d" % i}))
    spot_pods = []
    for i, n in enumerate(nodes):
        ps = []
        if r.random() < 0.3:  # overcommitted: free values below zero
            ps.append(Pod(name="big%d" % i, containers=[Container(cpu_milli=n.cpu_milli + 100,
                                                                  memory=n.memory + unit)]))
        spot_pods.append(ps)
    cands = []
    for c in range(10):
        pods = []
        for k in range(r.randint(2, 24)):
            if mode == 2:
                mem = r.choice([(1 << 45), (1 << 44) + (1 << 20), ((1 << 26) - 1) << 20, 1 << 20])
            elif mode == 4:  # scaled requests at the window visits' 2^23 limit, some beyond it
                mem = r.choice([((1 << 23) - 1) << 20, (1 << 23) << 20, (1 << 22) << 20, 1 << 20, 3 << 20])
            elif mode == 5:  # every scaled request below 2^23: 32-bit window state on clamped nodes
                mem = r.choice([((1 << 23) - 1) << 20, (1 << 21) << 20, 5 << 20, 1 << 20])
            else:
                mem = r.randint(1, 600) * unit * (1 if mode != 0 else r.choice([1, 1, 64]))
            cpu = r.choice([0, 50, 100, 250, 333, 1000])
            eph = r.choice([0, 0, unit * r.randint(1, 1 << 20)])
            pods.append(Pod(name="c%d_%d" % (c, k), containers=[Container(cpu_milli=cpu, memory=mem, ephemeral=eph)],
                            owner_references=[OwnerReference("ReplicaSet")]))
        # a pod sized to the remaining free memory of node 0 exactly
        if c % 3 == 0 and not spot_pods[0]:
            pods.append(Pod(name="c%d_fill" % c, containers=[Container(memory=nodes[0].memory - sum(
                p.containers[0].memory for p in pods) % nodes[0].memory)], owner_references=[OwnerReference("ReplicaSet")]))
        cands.append(pods)
    return nodes, spot_pods, cands


@pytest.mark.parametrize("narrow", [0, 1])
def test_scaled_run_pass_matches_oracle(narrow):
    # SR_K2_NARROW=0 keeps every placement on 64-bit values; 1 (the default)
    # scales a candidate's requests (and, in window visits, the window's free
    # values) to 32 bits where that is exact
    import os
    from spotplanner.planner import PredicateChecker
    os.environ["SR_K2_NARROW"] = str(narrow)
    try:
        c = PredicateChecker(0)
    finally:
        del os.environ["SR_K2_NARROW"]
    try:
        for seed in range(36):
            nodes, spot_pods, cands = _granular_scenario(7000 + seed)
            run_scenario(c, nodes, spot_pods, cands)
        for seed in range(10):
            nodes, spot_pods, cands = rand_scenario(7100 + seed, n_spot=4 + seed, n_cand=12, max_pods=30,
                                                    features=False)
            run_scenario(c, nodes, spot_pods, cands)
        for seed in range(16):  # host ports and hostname anti-affinity next to scaled runs
            nodes, spot_pods, cands = rand_scenario(7200 + seed, n_spot=4 + seed % 8, n_cand=12, max_pods=24,
                                                    anti=0.3, hostname_only=True)
            run_scenario(c, nodes, spot_pods, cands)
        tick_parity(c, SynthCluster(5, seed=21))
    finally:
        c.close()


@pytest.mark.parametrize("mode", ["node_order", "pod_order"])
def test_synthetic_config3_realistic_plans_match_oracle(checker, podorder_checker, mode):
    # bench --variant realistic at full C3 size: StatefulSet EBS claims under a
    # CSINode limit, init containers, GPU pods -- extension-record candidates on
    # the node-order window kernel (default) and on the pod-order path
    from spotplanner.synth import REALISTIC
    c = checker if mode == "node_order" else podorder_checker
    o, p = tick_parity(c, SynthCluster(3, **REALISTIC), oracle_threads=16)
    assert p.checks > 0


@pytest.mark.parametrize("mode", ["node_order", "pod_order"])
def test_synthetic_config3_affinity_plans_match_oracle(checker, podorder_checker, mode):
    # bench --variant affinity at full C3 size: every pod in a Deployment, 10 %
    # of them with required hostname anti-affinity (spot replicas included), 10 %
    # with a zone DoNotSchedule spread constraint -- state-bit pairs, the domain
    # path for replicas that count each other, and the pruned term set
    from spotplanner.synth import AFFINITY
    c = checker if mode == "node_order" else podorder_checker
    o, p = tick_parity(c, SynthCluster(3, **AFFINITY), oracle_threads=16)
    assert p.checks > 0

