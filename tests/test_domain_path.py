"""K2's domain path (candidates whose pods interact through inter-pod
(anti-)affinity across nodes): the hand-derived plans of domain_cases.py on the
oracle (CPU) and on the GPU through the C-ABI, random clusters with shared-key
terms planned without fallback, and the path's limits."""
import numpy as np
import pytest

from domain_cases import cases, nodes
from helpers import Scenario
from oracle_lib import oracle_plan
from randcluster import aff_interacts, anti_interacts_off_node, rand_scenario
from spotplanner import capi
from spotplanner.rescheduler import plan_arrays

CASES = cases()
IDS = [c.name for c in CASES]


def _plan(sc, n, use_gpu, checker=None):
    cand_off = np.array([0, n], np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + n, dtype=np.int32)
    if not use_gpu:
        o = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1)
        return int(o["status"][0]), list(o["node_of_pod"])
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, cand_off, cand_pods)
    finally:
        capi.load_planner().sr_snapshot_destroy(h)
    return int(p.status[0]), list(p.node_of_pod)


def _expect(case):
    return (capi.SR_CAND_OK if case.fail < 0 else case.fail), case.want


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_oracle_domain_case(case):
    sc = Scenario(nodes(), [[] for _ in range(4)], case.pods)
    assert _plan(sc, len(case.pods), False) == _expect(case), case.why


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_gpu_domain_case(checker, case):
    sc = Scenario(nodes(), [[] for _ in range(4)], case.pods)
    assert _plan(sc, len(case.pods), True, checker) == _expect(case), case.why


def test_random_scenarios_reach_the_domain_path():
    """The random parity seeds below plan candidates that interact across
    nodes (not only static conflicts): both kinds must occur."""
    anti = aff = 0
    for seed in range(30):
        nodes_, _, cands = rand_scenario(7000 + seed, n_spot=8 + seed % 10, n_cand=10, max_pods=3 + seed % 8,
                                         features=seed % 2 == 0, anti=0.3, aff=0.3, shared_keys=True)
        anti += sum(anti_interacts_off_node(nodes_, c) for c in cands)
        aff += sum(aff_interacts(c) for c in cands)
    assert anti >= 30 and aff >= 30, (anti, aff)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(30))
def test_gpu_random_shared_key_plans(checker, seed):
    """Anti-affinity and affinity on zone / team keys (shared, missing on some
    nodes) between the pods of a candidate: planned on the device, bit-exact
    with the oracle, no fallback."""
    from test_gpu_parity import run_scenario
    nodes_, spot_pods, cands = rand_scenario(7000 + seed, n_spot=8 + seed % 10, n_cand=10, max_pods=3 + seed % 8,
                                             features=seed % 2 == 0, anti=0.3, aff=0.3, shared_keys=True)
    run_scenario(checker, nodes_, spot_pods, cands)


@pytest.mark.gpu
def test_gpu_domain_path_up_to_512_pods(checker):
    """Up to 512 pods interacting across nodes are planned on the device
    (8 groups of 64 lanes: candidates of 300 and 512 pods, and 257 / 256 / 65 /
    64 around the group boundaries), bit-exact with the oracle; a 513-pod
    candidate exceeds the planner's per-candidate limit (MAX_CAND_PODS) and
    takes the fallback path.  The oracle plans every one of them."""
    from domain_cases import pod, term
    from test_gpu_parity import run_scenario
    sizes = [511, 299, 256, 255, 64, 63]  # web pods; each candidate adds one db pod
    big = [[pod("w%d" % i, "web", anti=[term("zone", "db")]) for i in range(n)] + [pod("d", "db")] for n in sizes]
    big.append([pod("w%d" % i, "web", anti=[term("zone", "db")]) for i in range(512)] + [pod("d", "db")])  # 513
    _, o, p = run_scenario(checker, nodes(), [[] for _ in range(4)], big, extra_fallback=lambda c: c == len(sizes))
    assert [int(x) for x in p.status[:len(sizes)]] == [int(x) for x in o["status"][:len(sizes)]]
    assert all(int(x) != capi.SR_CAND_FALLBACK for x in p.status[:len(sizes)])
    assert int(p.status[len(sizes)]) == capi.SR_CAND_FALLBACK


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(4))
def test_gpu_large_domain_candidates_300_512(checker, seed):
    """Zone anti-affinity / affinity candidates of 300-512 pods with init containers and scalars on the
    8-group domain path, against the oracle."""
    from test_gpu_parity import run_scenario
    nodes_, spot_pods, cands = rand_scenario(7600 + seed, n_spot=48 + 8 * seed, n_cand=2, max_pods=200,
                                             features=False, anti=0.2, aff=0.15 if seed % 2 else 0.0,
                                             shared_keys=True, valid_selectors=True)
    for i, c in enumerate(cands):  # 300 .. 512 pods each
        want = 300 + 212 * i
        while len(c) < want:
            c.extend(cands[(i + 1) % 2][:want - len(c)] or [c[0]])
    _, o, p = run_scenario(checker, nodes_, spot_pods, cands)
    assert all(int(s) != capi.SR_CAND_FALLBACK for s in o["status"])


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_gpu_large_shared_key_candidates(checker, seed):
    """65-200 pods per candidate interacting through zone / team anti-affinity
    (and affinity on half the seeds): the domain path with 2-4 pod groups,
    bit-exact with the oracle and without fallback -- init containers and
    scalar resources included (extension records)."""
    from test_gpu_parity import run_scenario
    nodes_, spot_pods, cands = rand_scenario(7400 + seed, n_spot=24 + 4 * seed, n_cand=3, max_pods=200,
                                             features=False, anti=0.2, aff=0.15 if seed % 2 else 0.0,
                                             shared_keys=True, valid_selectors=True)

    for i, c in enumerate(cands):  # 65 .. 200 pods each
        while len(c) < 65 + 45 * i:
            c.extend(cands[(i + 1) % 3][:65 + 45 * i - len(c)] or [c[0]])
    _, o, p = run_scenario(checker, nodes_, spot_pods, cands)
    assert all(int(s) != capi.SR_CAND_FALLBACK for s in o["status"])
    assert any(anti_interacts_off_node(nodes_, c) or aff_interacts(c) for c in cands)
