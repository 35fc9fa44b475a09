"""K2's dispatch forms against the oracle at test size.

Three paths are on by default only on large work lists, so the full-size
configs reach them only in the bench (C4: 15,000 candidates):

- the split launch (planner.cpp `k2_split`): a list with domain-path
  candidates and more entries than SR_K2_SPLIT_MIN (4,096) runs in two kernels
  side by side, the node-order candidates on the node-order kernel and the rest
  on the general kernel on a second stream; both write d_min and the
  single-rank result words;
- the cost-ordered work list (`list_cost`, lists above SR_LIST_COST_MIN =
  1,024 entries): the first run of a candidate generation records each
  candidate's wave duration, and the reused workloads of the next ticks
  dispatch the longest waves first;
- four waves per block (lists above 2,048 entries).

Each planner here lowers those thresholds per context (environment at
sr_create) so a 300-candidate cluster takes them, and every tick's statuses,
mappings, first_ok / first_fallback / winner and winner-only result are
compared with the oracle.  The winner is the first drainable candidate
whatever the dispatch order (rescheduler.go:269-287)."""
import ctypes
import os

import numpy as np
import pytest

from oracle_lib import OracleSnapshot, oracle_plan
from spotplanner import capi
from spotplanner.rescheduler import plan_arrays
from spotplanner.synth import AFFINITY, SynthCluster, build_candidates, new_node_map
from test_gpu_parity import compare_plans
from test_gpu_ticks import _with_extra

pytestmark = pytest.mark.gpu


def make_checker(**env):
    from spotplanner.planner import PredicateChecker
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: str(v) for k, v in env.items()})
    try:
        return PredicateChecker(0)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


DISPATCH = {
    # split launch + cost order, a short list head (head and rest parts in each split part)
    "split_cost_head32": dict(SR_K2_SPLIT_MIN=64, SR_LIST_COST_MIN=0, SR_LIST_HEAD=32),
    # split launch + cost order, four waves per block, the default list head (one part)
    "split_cost_wpb4": dict(SR_K2_SPLIT_MIN=64, SR_LIST_COST_MIN=0, SR_K2_WPB=4),
    # the split launch's fork / join as marker packets (the default: dispatch completion signals)
    "split_marker_events": dict(SR_K2_SPLIT_MIN=64, SR_LIST_COST_MIN=0, SR_K2_DISPATCH_EVENTS=0),
    # cost order without the split (one kernel: the general one)
    "cost_nosplit": dict(SR_K2_SPLIT=0, SR_LIST_COST_MIN=0, SR_LIST_HEAD=16),
}


def _ticks(ck, sc, n_ticks, rng, expect_split, per_tick_extra=(1, 4)):
    """Fresh snapshots of `sc`, each with a changing set of extra pods on random
    spot nodes (the candidate input stays the same, so the encoder reuses its
    candidate side from the third tick); every tick planned in full and
    winner-only, both against the oracle."""
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    extra, by_cost, reused, splits = [], 0, 0, 0
    _ticks.coop = 0  # runs with cooperative blocks
    for tick in range(n_ticks):
        if tick % 6 == 5:
            extra.clear()
        if tick:
            for _ in range(int(rng.integers(*per_tick_extra))):
                extra.append((int(rng.choice(cand_pods)), int(rng.integers(len(nm.spot)))))
        off, idx = _with_extra(nm, sc.n_nodes, extra)
        h = ctypes.c_void_p()
        assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(off, capi.P32),
                                      capi.ptr(idx, capi.P32), ctypes.byref(h)) == capi.SR_OK
        try:
            o = oracle_plan(OracleSnapshot(sc.ptr, nm.spot, off, idx), sc.ptr, cand_off, cand_pods, mode=1,
                            threads=8)
            q = plan_arrays(ck, h, sc.ptr, cand_off, cand_pods, full=False)  # winner only: returns at the winner
            tq = ck.timing()
            p = plan_arrays(ck, h, sc.ptr, cand_off, cand_pods)
            t = ck.timing()
        finally:
            lib.sr_snapshot_destroy(h)
        compare_plans(o, p, cand_off)
        assert np.array_equal(p.status, o["status"]), tick
        assert (q.first_ok, q.first_fallback, q.winner) == (p.first_ok, p.first_fallback, p.winner), tick
        assert np.array_equal(q.winner_map, p.winner_map), tick
        for tt in (tq, t):
            assert tt.k2_launches == (2 if expect_split else 1), (tick, tt.k2_launches)
            splits += tt.k2_launches == 2
            _ticks.coop += tt.k2_coop > 0
        if tick >= 2:
            reused += t.enc_reused
            by_cost += tq.k2_list_by_cost + t.k2_list_by_cost
    return reused, by_cost, splits


@pytest.mark.parametrize("which", sorted(DISPATCH))
def test_affinity_ticks_split_launch_and_cost_order(which):
    """The affinity variant (hostname anti-affinity state bits, zone-spread
    replicas on the domain path) over ten ticks: from the third tick the
    candidate side is reused and the work list runs in cost order."""
    ck = make_checker(**DISPATCH[which])
    try:
        sc = SynthCluster(3, seed=41, n_on_demand=300, n_spot=600, **AFFINITY)
        reused, by_cost, splits = _ticks(ck, sc, 10, np.random.default_rng(41), expect_split=which != "cost_nosplit")
        assert reused >= 6, reused
        assert by_cost >= 10, by_cost  # both runs of most reused ticks
    finally:
        ck.close()


def test_affinity_domain_path_candidates_exist():
    """The split needs domain-path candidates in the list: the affinity cluster
    above has them (the domain path plans zone-spread replicas that count each
    other)."""
    ck = make_checker(SR_K2_SPLIT_MIN=64)
    try:
        sc = SynthCluster(3, seed=41, n_on_demand=300, n_spot=600, **AFFINITY)
        lib = capi.load_planner()
        nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
        cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
        h = ctypes.c_void_p()
        assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                      capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                      ctypes.byref(h)) == capi.SR_OK
        try:
            plan_arrays(ck, h, sc.ptr, cand_off, cand_pods)
            assert ck.timing().k2_launches == 2
        finally:
            lib.sr_snapshot_destroy(h)
    finally:
        ck.close()


@pytest.mark.parametrize("config", [3, 5])
def test_cost_order_k0_less_ticks(config):
    """The cost-ordered list on the node-order kernel with K0-less steady ticks
    (one to three pods added on spot nodes between ticks: K2 recomputes the
    changed nodes' bits) and host-port candidates (C5)."""
    ck = make_checker(SR_LIST_COST_MIN=0, SR_LIST_HEAD=64)
    try:
        sc = SynthCluster(config, seed=43, n_on_demand=300, n_spot=600)
        reused, by_cost, _ = _ticks(ck, sc, 10, np.random.default_rng(config), expect_split=False)
        assert reused >= 6 and by_cost >= 10, (reused, by_cost)
    finally:
        ck.close()


def test_timed_runs_across_k0_and_k0_less_ticks():
    """Timing on (every kernel bracketed with events) while ticks alternate
    between runs that launch K0 and K0-less ones: an event pair is taken only
    for a kernel that is launched, so reading the times back never meets an
    unrecorded event (an A/B arm once failed here with `invalid resource
    handle`)."""
    ck = make_checker()
    try:
        sc = SynthCluster(3, seed=44, n_on_demand=200, n_spot=450)
        lib = capi.load_planner()
        nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
        cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
        c = capi.sr_candidates(len(cand_off) - 1, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32), None)
        wmap = np.full(int(np.max(np.diff(cand_off))), -1, np.int32)
        out = capi.sr_plan_out()
        out.winner_map = capi.ptr(wmap, capi.P32)
        ck.set_timing(7)
        k0_less, k0_runs, runs = 0, 0, 0
        rng = np.random.default_rng(44)
        extra = []
        for tick in range(8):
            if tick >= 2:
                extra.append((int(rng.choice(cand_pods)), int(rng.integers(len(nm.spot)))))
            off, idx = _with_extra(nm, sc.n_nodes, extra)
            h = ctypes.c_void_p()
            assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(off, capi.P32),
                                          capi.ptr(idx, capi.P32), ctypes.byref(h)) == capi.SR_OK
            try:
                assert lib.sr_plan_prepare(ck.handle, h, sc.ptr, ctypes.byref(c)) == capi.SR_OK, ck.last_error()
                cols = ck.timing().k0_columns
                k0_less += cols == -2
                k0_runs += cols != -2
                for _ in range(3):
                    assert lib.sr_plan_run(ck.handle, ctypes.byref(out)) == capi.SR_OK, ck.last_error()
                    runs += 1
                o = oracle_plan(OracleSnapshot(sc.ptr, nm.spot, off, idx), sc.ptr, cand_off, cand_pods, mode=1,
                                threads=8)
                assert out.winner == o["winner"], tick
            finally:
                lib.sr_snapshot_destroy(h)
            t = capi.sr_timing()
            assert lib.sr_get_timing(ck.handle, ctypes.byref(t)) == capi.SR_OK, ck.last_error()
            assert t.n_runs == runs and t.ms_placement > 0
        assert k0_less >= 2 and k0_runs >= 2, (k0_less, k0_runs)
    finally:
        ck.close()


# Every planner switch that is not the default, against the oracle: consecutive
# ticks of a host-port cluster (exclusive-port candidates, K0-less and
# incremental-K0 ticks, candidate-side reuse) and random scenarios on a pool
# wider than 64 words (rows over several chunks, head-only S rows).
SWITCHES = {
    "node_kernel_off": dict(SR_K2_NODE_KERNEL=0),   # every launch on the general kernel
    "excl_off": dict(SR_K2_EXCL=0),                 # exclusive candidates on the regular window step
    "one_slot": dict(SR_PLAN_SLOTS=1),              # one workload slot: every other input re-encodes
    "k0_inc_off": dict(SR_K0_INCREMENTAL=0),        # K0 rewrites every row whenever it runs
    "k0_skip_off": dict(SR_K0_SKIP=0),              # every run launches K0
    "wpb1": dict(SR_K2_WPB=1), "wpb2": dict(SR_K2_WPB=2), "wpb4": dict(SR_K2_WPB=4),
    "list_cost_off": dict(SR_LIST_COST=0, SR_LIST_COST_MIN=0),
    "prefix_batch_3": dict(SR_PREFIX_BATCH=3),
}


@pytest.mark.parametrize("which", sorted(SWITCHES))
def test_planner_switches_match_oracle(which):
    from randcluster import rand_scenario
    from test_gpu_parity import run_scenario, test_gpu_exclusive_port_candidates
    ck = make_checker(**SWITCHES[which])
    try:
        sc = SynthCluster(5, seed=51, n_on_demand=150, n_spot=400)
        _ticks(ck, sc, 6, np.random.default_rng(51), expect_split=False)
        for seed in range(2):
            nodes, spot_pods, cands = rand_scenario(7500 + seed, n_spot=4200 + 700 * seed, n_cand=8, max_pods=20,
                                                    anti=0.2, hostname_only=True)
            run_scenario(ck, nodes, spot_pods, cands)
        for seed in range(2):
            test_gpu_exclusive_port_candidates(ck, seed)
    finally:
        ck.close()


@pytest.mark.parametrize("case", ["c3", "c4_wide_head_only", "affinity_split", "c3_all", "c3_off"])
def test_cooperative_blocks(case):
    """Cooperative blocks (SR_K2_COOP): the costliest entries of a cost-ordered
    list, on a node-order launch of four waves per block, are planned by one
    block each whose other waves scan far resolutions with the chain wave; the
    plan is the oracle's.  C3-shaped rows (10 words: resolutions beyond the
    512-node head), a 6,000-node pool (94-word rows, head-only S rows: the
    scans evaluate the class programs), and the affinity variant's split launch
    (its node-order part cooperative); every entry cooperative (c3_all) and
    none (c3_off) on the same ticks."""
    env = dict(SR_LIST_COST_MIN=0, SR_K2_WPB=4, SR_K2_COOP={"c3_all": 4096, "c3_off": 0}.get(case, 32))
    if case == "affinity_split":
        env["SR_K2_SPLIT_MIN"] = 64
    ck = make_checker(**env)
    try:
        sc = {"c3": lambda: SynthCluster(3, seed=45, n_on_demand=300, n_spot=600),
              "c3_all": lambda: SynthCluster(3, seed=45, n_on_demand=300, n_spot=600),
              "c3_off": lambda: SynthCluster(3, seed=45, n_on_demand=300, n_spot=600),
              "c4_wide_head_only": lambda: SynthCluster(4, seed=5, n_on_demand=400, n_spot=6000),
              "affinity_split": lambda: SynthCluster(3, seed=41, n_on_demand=300, n_spot=600, **AFFINITY)}[case]()
        reused, by_cost, _ = _ticks(ck, sc, 8, np.random.default_rng(45), expect_split=case == "affinity_split")
        assert reused >= 4 and by_cost >= 8, (reused, by_cost)
        if case == "c3_off":
            assert _ticks.coop == 0, _ticks.coop
        else:
            assert _ticks.coop >= 8, _ticks.coop
    finally:
        ck.close()


@pytest.mark.parametrize("config", [3, 5])
def test_consecutive_runs_match_oracle(config):
    """Consecutive runs of one prepared workload, as the bench's timed region
    issues them: forty runs per tick -- winner-only runs (each returns once the
    candidates up to the winner are planned, the rest of the grid finishing
    behind the next launch), full runs with every output and runs with K2
    timed interleaved -- each with the oracle's winner and mapping, then the
    next tick's prepare (one more pod on a spot node: K0-less runs)."""
    ck = make_checker()
    try:
        sc = SynthCluster(config, seed=47, n_on_demand=300, n_spot=600)
        lib = capi.load_planner()
        nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
        cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
        n = len(cand_off) - 1
        c = capi.sr_candidates(n, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32), None)
        wmap = np.full(int(np.max(np.diff(cand_off))), -1, np.int32)
        status = np.zeros(n, np.int32)
        nodes = np.zeros(int(cand_off[-1]), np.int32)
        rng = np.random.default_rng(config)
        extra, k0_less = [], 0
        for tick in range(6):
            if tick:
                extra.append((int(rng.choice(cand_pods)), int(rng.integers(len(nm.spot)))))
            off, idx = _with_extra(nm, sc.n_nodes, extra)
            h = ctypes.c_void_p()
            assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot), capi.ptr(off, capi.P32),
                                          capi.ptr(idx, capi.P32), ctypes.byref(h)) == capi.SR_OK
            try:
                o = oracle_plan(OracleSnapshot(sc.ptr, nm.spot, off, idx), sc.ptr, cand_off, cand_pods, mode=1,
                                threads=8)
                want_map = o["node_of_pod"][cand_off[o["first_ok"]]:cand_off[o["first_ok"] + 1]] \
                    if o["first_ok"] >= 0 else None
                for _ in range(2 if tick == 0 else 1):
                    assert lib.sr_plan_prepare(ck.handle, h, sc.ptr, ctypes.byref(c)) == capi.SR_OK, ck.last_error()
                k0_less += ck.timing().k0_columns == -2
                for r in range(40):
                    out = capi.sr_plan_out()
                    out.winner_map = capi.ptr(wmap, capi.P32)
                    if r % 13 == 5:  # every output: waits for the other stream first
                        out.status = capi.ptr(status, capi.P32)
                        out.node_of_pod = capi.ptr(nodes, capi.P32)
                    timed = r % 11 == 7
                    if timed:
                        ck.set_timing(2)
                    assert lib.sr_plan_run(ck.handle, ctypes.byref(out)) == capi.SR_OK, ck.last_error()
                    if timed:
                        assert ck.timing().n_runs == 1
                        ck.set_timing(0)
                    assert (out.first_ok, out.winner) == (o["first_ok"], o["winner"]), (tick, r)
                    if want_map is not None:
                        assert np.array_equal(wmap[:out.winner_npods], want_map), (tick, r)
                    if r % 13 == 5:  # candidates outside the encoded set (C5: > 64 state bits) take the reference path
                        fb = status == capi.SR_CAND_FALLBACK
                        assert np.all(fb | (status == o["status"])), (tick, r)
                        for k in np.flatnonzero(~fb):
                            seg = slice(int(cand_off[k]), int(cand_off[k + 1]))
                            assert np.array_equal(nodes[seg], o["node_of_pod"][seg]), (tick, r, k)
            finally:
                lib.sr_snapshot_destroy(h)
        assert k0_less >= 3, k0_less
    finally:
        ck.close()
