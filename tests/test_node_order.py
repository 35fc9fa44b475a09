"""Node-order and window-order first fit == pod-order first fit (canDrainNode).

K2's node-order path (kernels.hip `k2_node_order`) rests on
these identities: visiting the spot nodes in NodeInfoArray order and, at each
node, placing the candidate's unplaced pods in pod order wherever they fit --
or, as K2 does, visiting windows of consecutive nodes (64 on the device) and
placing the unplaced pods in pod order, each on its first node of the window
that fits -- gives the same failing pod and the same pod -> node mapping as the
reference's sequential first fit (rescheduler.go:357-370).  Checked here on
the oracle itself (CPU): a node-order planner whose only predicate is the
oracle's CheckPredicates restatement against the evolving snapshot, compared
with oracle_can_drain_node on random clusters that use every encoded
predicate (resources, pod count, host ports incl. intra-candidate conflicts,
selectors, affinity, taints, unschedulable)."""
import numpy as np
import pytest

from helpers import Scenario
from oracle_lib import load_oracle
from randcluster import rand_scenario
from spotplanner import capi


def node_order_can_drain(olib, snap, cptr, pods, n_spot):
    """Returns (failing pod or -1, node per pod) or None for a fallback pod."""
    base = []
    for p in pods:
        row = [olib.oracle_check_predicates(snap.h, cptr, p, n) for n in range(n_spot)]
        if -1 in row:
            return None
        base.append(row)

    def next_feasible(k, after):
        return next((m for m in range(after + 1, n_spot) if base[k][m] == 1), None)

    ptr = [next_feasible(k, -1) for k in range(len(pods))]
    dead = next((k for k in range(len(pods)) if ptr[k] is None), len(pods))
    node = [-1] * len(pods)
    active = set(range(dead))
    assert olib.oracle_snapshot_fork(snap.h) == 0
    visited = set()
    while active:
        n = min(ptr[k] for k in active)
        assert n not in visited  # each node is visited at most once
        visited.add(n)
        for k in sorted(k for k in active if ptr[k] == n):
            if k >= dead:
                continue
            if olib.oracle_check_predicates(snap.h, cptr, pods[k], n) == 1:
                node[k] = n
                olib.oracle_snapshot_add_pod(snap.h, cptr, pods[k], n)
                active.discard(k)
            else:
                ptr[k] = next_feasible(k, n)
                if ptr[k] is None:
                    dead = min(dead, k)
                    active = {a for a in active if a < dead}
    olib.oracle_snapshot_revert(snap.h)
    return (dead if dead < len(pods) else -1), [node[k] if k < dead else -1 for k in range(len(pods))]


def window_order_can_drain(olib, snap, cptr, pods, n_spot, win):
    """K2's window visits on the oracle: windows of `win` nodes in order, the
    pods pointing into a window placed one by one in pod order on its first
    base-feasible node there that fits the snapshot; (failing pod or -1, node
    per pod) or None for a fallback pod."""
    base = []
    for p in pods:
        row = [olib.oracle_check_predicates(snap.h, cptr, p, n) for n in range(n_spot)]
        if -1 in row:
            return None
        base.append(row)

    def next_feasible(k, after):
        return next((m for m in range(after + 1, n_spot) if base[k][m] == 1), None)

    ptr = [next_feasible(k, -1) for k in range(len(pods))]
    dead = next((k for k in range(len(pods)) if ptr[k] is None), len(pods))
    node = [-1] * len(pods)
    active = set(range(dead))
    assert olib.oracle_snapshot_fork(snap.h) == 0
    visited = set()
    while active:
        w = min(ptr[k] for k in active) // win
        assert w not in visited  # each window is visited at most once
        visited.add(w)
        for k in sorted(k for k in active if ptr[k] // win == w):
            if k >= dead:
                continue
            hit = next((m for m in range(ptr[k], min(n_spot, (w + 1) * win))
                        if base[k][m] == 1 and olib.oracle_check_predicates(snap.h, cptr, pods[k], m) == 1), None)
            if hit is not None:
                node[k] = hit
                olib.oracle_snapshot_add_pod(snap.h, cptr, pods[k], hit)
                active.discard(k)
            else:
                ptr[k] = next_feasible(k, (w + 1) * win - 1)
                if ptr[k] is None:
                    dead = min(dead, k)
                    active = {a for a in active if a < dead}
    olib.oracle_snapshot_revert(snap.h)
    return (dead if dead < len(pods) else -1), [node[k] if k < dead else -1 for k in range(len(pods))]


@pytest.mark.parametrize("seed", range(60))
def test_node_order_first_fit_equals_pod_order(seed):
    nodes, spot_pods, cands = rand_scenario(7000 + seed, n_spot=5 + seed % 17, n_cand=6, max_pods=4 + seed % 9,
                                            features=seed % 3 != 0)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    olib = load_oracle()
    snap = sc.oracle_snapshot()
    q = sc.q0
    compared = 0
    for c in cands:
        pods = list(range(q, q + len(c)))
        q += len(c)
        got = node_order_can_drain(olib, snap, sc.ptr, pods, len(nodes))
        if got is None:
            continue
        # window visits of 1 (node order), 2, 3 and 4 nodes and of the whole pool
        for win in (1, 2, 3, 4, len(nodes)):
            assert window_order_can_drain(olib, snap, sc.ptr, pods, len(nodes), win) == got, (seed, win)
        arr = np.array(pods, np.int32)
        want_map = np.full(max(1, len(pods)), -1, np.int32)
        assert olib.oracle_snapshot_fork(snap.h) == 0
        want = olib.oracle_can_drain_node(snap.h, sc.ptr, capi.ptr(arr, capi.P32), len(pods),
                                          capi.ptr(want_map, capi.P32))
        olib.oracle_snapshot_revert(snap.h)
        if want == -2:  # candidate-level fallback (an init-container pod before others)
            continue
        assert got[0] == want, (seed, got, want)
        assert got[1] == [int(x) for x in want_map[:len(pods)]], (seed, got, want_map)
        compared += 1
    assert compared > 0 or not any(cands)
