"""The product's sharded path at world size 2 on one GPU, through its own
transports: two processes each plan their shard of the candidates through
libsrplanner with a communicator attached, either
- `host_fn` (sr_comm_init_host: RCCL does not run two ranks on one device, so
  the allreduce(min) of the planner's three result words goes over gloo):
  K0 + K2 per shard, the collective on the packed {global << 32 | local}
  words, K3 on every rank (the owner writes the mapping); or
- `shm` (sr_comm_init_shm, bench.py's default on one node): every rank's K2
  writes its outcome words into one shared-memory segment and each rank's
  host walks them in global order -- no collective, no K3;
and sr_plan_first's prefix batches stopping on the reduced bound.

Checked against the oracle (rescheduler.go:228-287 evaluates the same
candidates serially): sr_plan with interleaved shards (statuses, mappings,
winner, the owner's mapping); sr_plan_first with interleaved AND contiguous
shards, prefix batches of 2 and 16, on scenarios whose fallback candidates
sit before, after and instead of the first drainable one (the shared-memory
transport takes interleaved shards only and refuses contiguous ones)."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
WORLD = 2
SEEDS = [0, 1, 4, 5, 6, 11, 14, 23]   # every plan_first_cases pattern, winners 1..18 and none


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _contiguous(cand_off, cand_pods, rank, world):
    n = len(cand_off) - 1
    lo, hi = n * rank // world, n * (rank + 1) // world
    idx = np.arange(lo, hi, dtype=np.int32)
    off = (cand_off[lo:hi + 1] - cand_off[lo]).astype(np.int32)
    return off, np.ascontiguousarray(cand_pods[cand_off[lo]:cand_off[hi]], np.int32), idx


def _run_first(lib, ck, h, cptr, loff, lpods, gidx):
    import ctypes

    from spotplanner import capi
    n = len(loff) - 1
    c = capi.sr_candidates(n, capi.ptr(loff, capi.P32), capi.ptr(lpods, capi.P32), capi.ptr(gidx, capi.P32))
    status = np.full(max(1, n), -99, np.int32)
    nodes = np.full(max(1, int(loff[-1])), -99, np.int32)
    wmap = np.full(max(1, int(np.max(np.diff(loff))) if n else 1), -1, np.int32)
    o = capi.sr_plan_out()
    o.status = capi.ptr(status, capi.P32)
    o.node_of_pod = capi.ptr(nodes, capi.P32)
    o.winner_map = capi.ptr(wmap, capi.P32)
    st = lib.sr_plan_first(ck.handle, h, cptr, ctypes.byref(c), ctypes.byref(o))
    assert st == capi.SR_OK, ck.last_error()
    mine = {int(g): (int(status[k]), [int(x) for x in nodes[loff[k]:loff[k + 1]]]) for k, g in enumerate(gidx)}
    return dict(first_ok=int(o.first_ok), first_fallback=int(o.first_fallback), winner=int(o.winner),
                wmap=[int(x) for x in wmap[:o.winner_npods]] if o.winner_npods else None, mine=mine,
                batches=int(ck.timing().prefix_batches))


def _worker(rank, world, port, out, transport):
    import ctypes
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "k8s-spot-rescheduler_amd"), os.path.join(repo, "tests")]
    import torch
    import torch.distributed as dist

    from helpers import Scenario
    from plan_first_cases import plan_first_scenario
    from spotplanner import capi
    from spotplanner.planner import PredicateChecker
    from spotplanner.rescheduler import plan_arrays
    from spotplanner.synth import SynthCluster, build_candidates, new_node_map, shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    bias = 1 << 63

    def allreduce_min(vals):  # uint64 words: order-preserving shift into int64
        t = torch.tensor([v - bias for v in vals], dtype=torch.int64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return [int(x) + bias for x in t]

    def attach(ck, name):
        if transport == "shm":  # one segment per planner, the same name and session on both ranks
            ck.attach_shared_memory("/srtest-%d-%s" % (port, name), port * 7919, world, rank, 4096)
        else:
            ck.attach_collective(world, rank, allreduce_min)

    results = {}
    try:
        lib = capi.load_planner()
        checkers = {}
        for b in (16, 2):
            os.environ["SR_PREFIX_BATCH"] = str(b)
            checkers[b] = PredicateChecker(0)
            attach(checkers[b], "b%d" % b)
        del os.environ["SR_PREFIX_BATCH"]
        dist.barrier()  # every rank attached before any plans (or rank 0's planner could unlink the name)
        # sr_plan over synthetic clusters: every candidate, interleaved shards
        for cfg in [(3, 240, 600, 0.3), (5, 200, 500, -1.0)]:
            config, n_od, n_spot, pinned = cfg
            sc = SynthCluster(config, n_on_demand=n_od, n_spot=n_spot, pinned_fraction=pinned)
            nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
            loff, lpods, gidx = shard(cand_off, cand_pods, rank, world)
            h = ctypes.c_void_p()
            assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                          capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                          ctypes.byref(h)) == capi.SR_OK
            p = plan_arrays(checkers[16], h, sc.ptr, loff, lpods, cand_global=gidx)
            q = plan_arrays(checkers[16], h, sc.ptr, loff, lpods, cand_global=gidx, full=False)
            results[("plan", cfg)] = dict(
                first_ok=p.first_ok, first_fallback=p.first_fallback, winner=p.winner,
                wmap=[int(x) for x in p.winner_map] if len(p.winner_map) else None,
                q=(q.first_ok, q.first_fallback, q.winner, [int(x) for x in q.winner_map]),
                mine={int(g): (int(s), [int(x) for x in p.node_of_pod[loff[k]:loff[k + 1]]])
                      for k, (g, s) in enumerate(zip(gidx, p.status))})
            results[("first_synth", cfg)] = _run_first(lib, checkers[2], h, sc.ptr, loff, lpods, gidx)
            lib.sr_snapshot_destroy(h)
            if config == 3:  # steady ticks through the collective: reuse, K0-less and incremental K0 runs
                ck = PredicateChecker(0)
                attach(ck, "steady")
                dist.barrier()
                rng = np.random.default_rng(77)  # the same changes on both ranks
                extra = []
                for t in range(8):
                    if t:
                        for _ in range(1 if t % 3 else 12):
                            extra.append((int(cand_pods[rng.integers(len(cand_pods))]), int(rng.integers(len(nm.spot)))))
                    h = ctypes.c_void_p()
                    assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                                  capi.ptr(nm.node_pod_off, capi.P32),
                                                  capi.ptr(nm.node_pod_idx, capi.P32), ctypes.byref(h)) == capi.SR_OK
                    for pod, pos in extra:
                        assert lib.sr_snapshot_add_pod(h, sc.ptr, pod, pos) == capi.SR_OK
                    p = plan_arrays(ck, h, sc.ptr, loff, lpods, cand_global=gidx)
                    tm = ck.timing()
                    results[("steady", t)] = dict(
                        first_ok=p.first_ok, first_fallback=p.first_fallback, winner=p.winner,
                        wmap=[int(x) for x in p.winner_map] if len(p.winner_map) else None,
                        k0=int(tm.k0_columns), reused=int(tm.enc_reused), extra=list(extra),
                        mine={int(g): (int(s_), [int(x) for x in p.node_of_pod[loff[k]:loff[k + 1]]])
                              for k, (g, s_) in enumerate(zip(gidx, p.status))})
                    lib.sr_snapshot_destroy(h)
                dist.barrier()
                ck.close()
        # sr_plan_first: fallback patterns, both shardings, both batch sizes
        for seed in SEEDS:
            nodes, spot_pods, cands, _, _, _ = plan_first_scenario(seed)
            flat = [p for c in cands for p in c]
            sc = Scenario(nodes, spot_pods, flat)
            cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
            cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
            h = sc.product_snapshot()
            for split, fn in (("interleaved", shard), ("contiguous", _contiguous)):
                loff, lpods, gidx = fn(cand_off, cand_pods, rank, world)
                for b, ck in checkers.items():
                    if transport == "shm" and split == "contiguous":  # refused before anything is planned
                        c = capi.sr_candidates(len(loff) - 1, capi.ptr(loff, capi.P32), capi.ptr(lpods, capi.P32),
                                               capi.ptr(gidx, capi.P32))
                        o = capi.sr_plan_out()
                        results[("first", seed, split, b)] = {
                            "refused": lib.sr_plan_first(ck.handle, h, sc.ptr, ctypes.byref(c), ctypes.byref(o))}
                        continue
                    results[("first", seed, split, b)] = _run_first(lib, ck, h, sc.ptr, loff, lpods, gidx)
            lib.sr_snapshot_destroy(h)
        dist.barrier()  # no rank closes (rank 0: unlinks) a segment another still plans through
        for ck in checkers.values():
            ck.close()
        gathered = [None] * world
        dist.all_gather_object(gathered, results)
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module", params=["host_fn", "shm"])
def two_rank_results(request):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, WORLD, port, q, request.param)) for r in range(WORLD)]
    for p in procs:
        p.start()
    gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return gathered


def _merged(gathered, key):
    merged = {}
    for res in gathered:
        merged.update(res[key]["mine"])
    return merged


def _synth(cfg):
    import ctypes

    from oracle_lib import OracleSnapshot
    from spotplanner import capi
    from spotplanner.synth import SynthCluster, build_candidates, new_node_map
    config, n_od, n_spot, pinned = cfg
    sc = SynthCluster(config, n_on_demand=n_od, n_spot=n_spot, pinned_fraction=pinned)
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    osnap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
    return sc, osnap, cand_off, cand_pods, ctypes


@pytest.mark.parametrize("cfg", [(3, 240, 600, 0.3), (5, 200, 500, -1.0)])
def test_two_ranks_plan_every_candidate_through_the_collective(two_rank_results, cfg):
    from oracle_lib import oracle_plan
    sc, osnap, cand_off, cand_pods, _ = _synth(cfg)
    o = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
    merged = _merged(two_rank_results, ("plan", cfg))
    n = len(cand_off) - 1
    assert sorted(merged) == list(range(n))
    for c in range(n):
        s, m = merged[c]
        assert s == int(o["status"][c]), c
        assert m == list(o["node_of_pod"][int(cand_off[c]):int(cand_off[c + 1])]), c
    owners = []
    for rank, res in enumerate(two_rank_results):
        r = res[("plan", cfg)]
        # every rank sees the reduced first_ok / first_fallback / winner (K3 after the collective)
        assert (r["first_ok"], r["first_fallback"], r["winner"]) == (o["first_ok"], o["first_fallback"], o["winner"])
        assert r["q"][:3] == (o["first_ok"], o["first_fallback"], o["winner"])  # the winner-only run too
        if r["wmap"] is not None:
            owners.append((rank, r["wmap"]))
    if o["first_ok"] >= 0:  # only the rank owning the global first_ok writes its mapping
        assert len(owners) == 1 and owners[0][0] == o["first_ok"] % WORLD
        assert owners[0][1] == list(o["winner_map"])


def _check_first(two_rank_results, key, ref_all, ref_early, cand_off):
    from plan_first_cases import check_plan_first
    from spotplanner import capi
    n = len(cand_off) - 1
    results = [res[key] for res in two_rank_results]
    if "refused" in results[0]:  # the shared-memory transport and contiguous shards
        assert all(r["refused"] == capi.SR_ERR_INVALID_ARG for r in results), results
        return
    for r in results:  # the reduced outcome is the same on every rank
        assert (r["first_ok"], r["first_fallback"], r["winner"], r["batches"]) == \
            (results[0]["first_ok"], results[0]["first_fallback"], results[0]["winner"], results[0]["batches"])
    owners = [r["wmap"] for r in results if r["wmap"] is not None]
    r0 = results[0]
    wmap = owners[0] if owners else None
    if r0["first_ok"] >= 0:
        assert len(owners) == 1
    merged = _merged(two_rank_results, key)
    assert sorted(merged) == list(range(n))
    glob = sorted(merged)
    status = [merged[c][0] for c in glob]
    nodes = [merged[c][1] for c in glob]
    check_plan_first(r0["first_ok"], r0["first_fallback"], r0["winner"], wmap, status, nodes, ref_all, ref_early,
                     cand_off, True, glob)


@pytest.mark.parametrize("cfg", [(3, 240, 600, 0.3), (5, 200, 500, -1.0)])
def test_two_ranks_plan_first_synthetic(two_rank_results, cfg):
    from oracle_lib import oracle_plan
    sc, osnap, cand_off, cand_pods, _ = _synth(cfg)
    ref_all = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
    ref_early = oracle_plan(osnap, sc.ptr, cand_off, cand_pods, mode=0)
    _check_first(two_rank_results, ("first_synth", cfg), ref_all, ref_early, cand_off)


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.parametrize("split", ["interleaved", "contiguous"])
@pytest.mark.parametrize("batch", [16, 2])
def test_two_ranks_plan_first_fallback_patterns(two_rank_results, seed, split, batch):
    from helpers import Scenario
    from oracle_lib import oracle_plan
    from plan_first_cases import plan_first_scenario
    nodes, spot_pods, cands, _, _, _ = plan_first_scenario(seed)
    flat = [p for c in cands for p in c]
    sc = Scenario(nodes, spot_pods, flat)
    cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
    cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
    ref_all = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=1)
    ref_early = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=0)
    _check_first(two_rank_results, ("first", seed, split, batch), ref_all, ref_early, cand_off)


def test_two_ranks_steady_ticks_through_the_collective(two_rank_results):
    """Consecutive ticks of one cluster through the collective, the same
    stamped candidate shards every tick and a few more pods on spot nodes each
    time: the candidate side is reused, K0 is skipped while few nodes changed
    (K2 sets the run's d_min words for the allreduce) or runs on the changed
    columns; every tick's merged plan equals the oracle on the mutated snapshot."""
    from oracle_lib import OracleSnapshot, oracle_plan
    from spotplanner import capi
    from spotplanner.synth import new_node_map
    sc, _, cand_off, cand_pods, _ = _synth((3, 240, 600, 0.3))
    lib = capi.load_planner()
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    n = len(cand_off) - 1
    kinds = set()
    for t in range(8):
        r0 = two_rank_results[0][("steady", t)]
        osn = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
        for pod, pos in r0["extra"]:
            osn.lib.oracle_snapshot_add_pod(osn.h, sc.ptr, pod, pos)
        o = oracle_plan(osn, sc.ptr, cand_off, cand_pods, mode=1, threads=8)
        merged = _merged(two_rank_results, ("steady", t))
        assert sorted(merged) == list(range(n))
        for c in range(n):
            s_, m = merged[c]
            assert s_ == int(o["status"][c]), (t, c)
            assert m == list(o["node_of_pod"][int(cand_off[c]):int(cand_off[c + 1])]), (t, c)
        for res in two_rank_results:
            r = res[("steady", t)]
            assert (r["first_ok"], r["winner"]) == (int(o["first_ok"]), int(o["winner"])), t
            if t >= 2:
                assert r["reused"] == 1, t
                kinds.add(r["k0"])
    assert -2 in kinds  # at least one K0-less tick on some rank
