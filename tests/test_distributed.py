"""N > 1 planning on CPU: candidates sharded c % world == rank (bench.py's
layout), each rank plans its shard, one allreduce(min) picks the first
drainable candidate.  The GPU path does the same reduction with RCCL inside
sr_plan_run; here gloo and the oracle stand in, checking the sharding and
reduction logic against a single-process plan of all candidates."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, config, n_od, n_spot, pinned, out):
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(repo, "k8s-spot-rescheduler_amd"), os.path.join(repo, "tests")]
    from oracle_lib import OracleSnapshot, oracle_plan
    from spotplanner import capi
    from spotplanner.synth import SynthCluster, build_candidates, new_node_map, shard

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sc = SynthCluster(config, n_on_demand=n_od, n_spot=n_spot, pinned_fraction=pinned)
    nm = new_node_map(capi.load_planner().sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label,
                      sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    loff, lpods, gidx = shard(cand_off, cand_pods, rank, world)
    snap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
    r = oracle_plan(snap, sc.ptr, loff, lpods, mode=1, cand_global=gidx)
    big = np.iinfo(np.int64).max
    t = torch.tensor([r["first_ok"] if r["first_ok"] >= 0 else big,
                      r["first_fallback"] if r["first_fallback"] >= 0 else big], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    local_status = {int(g): int(s) for g, s in zip(gidx, r["status"])}
    gathered = [None] * world
    dist.all_gather_object(gathered, local_status)
    if rank == 0:
        merged = {}
        for d in gathered:
            merged.update(d)
        out.put((int(t[0]), int(t[1]), merged))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_plan_min_reduce_matches_single_process(world):
    from oracle_lib import OracleSnapshot, oracle_plan
    from spotplanner import capi
    from spotplanner.synth import SynthCluster, build_candidates, new_node_map

    config, n_od, n_spot, pinned = 3, 120, 300, 0.3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, config, n_od, n_spot, pinned, q)) for r in range(world)]
    for p in procs:
        p.start()
    first_ok, first_fb, merged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    sc = SynthCluster(config, n_on_demand=n_od, n_spot=n_spot, pinned_fraction=pinned)
    nm = new_node_map(capi.load_planner().sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label,
                      sc.spot_label)
    cand_off, cand_pods = build_candidates(nm, sc.pod_flags())
    r = oracle_plan(OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx), sc.ptr, cand_off, cand_pods,
                    mode=1)
    big = np.iinfo(np.int64).max
    assert first_ok == (r["first_ok"] if r["first_ok"] >= 0 else big)
    assert first_fb == (r["first_fallback"] if r["first_fallback"] >= 0 else big)
    assert [merged[c] for c in range(len(cand_off) - 1)] == list(r["status"])
    # the reference-faithful serial run drains the same node
    early = oracle_plan(OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx), sc.ptr, cand_off,
                        cand_pods, mode=0)
    assert early["winner"] == r["winner"]
