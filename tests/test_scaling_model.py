"""The multi-GPU tick model and the bench's per-rank fields:
CPU only.  The model predicts a rank's device tick from measured one-GPU parts
(K2, its longest chain, the launch gap, K3) and an allreduce latency; bench.py
--scaling auto shards a config's own tick only where that shortens it."""
import multiprocessing as mp
import os
import socket
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "k8s-spot-rescheduler_amd"))
import bench  # noqa: E402
from spotplanner import scaling  # noqa: E402


def test_one_gpu_tick_is_k2_plus_gap():
    for c, p in scaling.PARTS.items():
        assert scaling.predict_tick_us(p, 1, "strong") == pytest.approx(max(p["chain"], p["k2"]) + p["gap"])
        assert scaling.predict_tick_us(p, 1, "weak") == scaling.predict_tick_us(p, 1, "strong")


def test_chain_bounds_the_sharded_tick():
    p = dict(k2=100.0, chain=30.0, gap=1.0, k3=4.0)
    # 100 / 8 < 30: the longest candidate's chain sets K2 on every rank
    assert scaling.predict_tick_us(p, 8, "strong") == pytest.approx(30.0 + 1.0 + scaling.allreduce_us(8) + 4.0)
    assert scaling.predict_tick_us(p, 2, "strong") == pytest.approx(50.0 + 1.0 + scaling.allreduce_us(2) + 4.0)
    assert scaling.predict_tick_us(p, 2, "weak") == pytest.approx(100.0 + 1.0 + scaling.allreduce_us(2) + 4.0)


@pytest.mark.parametrize("n", [2, 4, 8])
@pytest.mark.parametrize("transport", ["rccl", "shm"])
def test_c3_does_not_shard_its_own_tick(n, transport):
    # C3's K2 is one chain (12.2 of 14.5 us): a strong-scaled tick is slower
    r = scaling.predict(3, n, transport)
    assert not r["strong_pays"] and r["strong_tick_us"] > r["tick1_us"]
    assert scaling.choose_scaling(3, n, transport)[0] == "weak"


def test_throughput_bound_tick_shards():
    # a K2 well above its chain (C4 before its work list ran longest wave first:
    # 67.8 us against a 41.3 us wave) is shortened by splitting the candidates
    p = dict(k2=67.8, chain=41.3, gap=0.0, k3=4.5)
    assert scaling.predict_tick_us(p, 2, "strong") < scaling.predict_tick_us(p, 1, "strong")


@pytest.mark.parametrize("c", [1, 2, 3, 5])
def test_chain_bound_configs_keep_their_own_tick_whole(c):
    # round 6: C1-C3 and C5's K2 is within a few us of its longest wave
    for transport in ("rccl", "shm"):
        assert scaling.choose_scaling(c, 2, transport)[0] == "weak"


@pytest.mark.parametrize("n", [2, 4, 8])
def test_c4_shards_over_shared_memory(n):
    # round 6: the cooperative blocks cut C4's longest wave to 28.8 us of a 44.4 us
    # K2, so splitting its 15,000 candidates pays where the exchange is cheap
    r = scaling.predict(4, n, "shm")
    assert r["strong_pays"] and r["strong_tick_us"] == pytest.approx(
        scaling.PARTS[4]["chain"] + scaling.PARTS[4]["gap"] + scaling.SHM_US)
    assert scaling.choose_scaling(4, n, "shm")[0] == "strong"


def test_efficiencies_follow_the_driver_rule():
    # weak: N x the work in tick(N) -> t1 / tN; strong: the same work -> t1 / (N tN)
    for c in scaling.PARTS:
        for n in (2, 4, 8):
            r = scaling.predict(c, n)
            assert r["weak_efficiency"] == pytest.approx(r["tick1_us"] / r["weak_tick_us"], abs=1e-3)
            assert r["strong_efficiency"] == pytest.approx(r["tick1_us"] / (n * r["strong_tick_us"]), abs=1e-3)


def test_one_gpu_needs_no_choice():
    assert scaling.choose_scaling(3, 1)[0] == "strong"


def test_rank_record_fields():
    rec = bench.rank_record(1, 750, 21000, 0.0032, 200,
                            {"k0_tables": 0.0, "k2_placement": 0.0138, "k3_winner": 0.0045, "collective": 0.02})
    assert rec == {"rank": 1, "candidates": 750, "candidate_pods": 21000, "ms_per_step_local": 0.016,
                   "k0_tables_ms": 0.0, "k2_placement_ms": 0.0138, "k3_winner_ms": 0.0045, "collective_ms": 0.02}


def _gather_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec = bench.rank_record(rank, 10 + rank, 100 * rank, 0.001 * (rank + 1), 10,
                            {"k2_placement": 0.01 * (rank + 1), "collective": 0.02})
    q.put((rank, bench.gather_per_rank(rec, world)))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_per_rank_records_gathered_in_rank_order(world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_gather_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for r in range(world):
        recs = got[r]
        assert [x["rank"] for x in recs] == list(range(world))
        assert [x["candidates"] for x in recs] == [10 + k for k in range(world)]
        assert recs[world - 1]["k2_placement_ms"] == pytest.approx(0.01 * world)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_shared_memory_transport_adds_no_device_exchange(n):
    # transport "shm" (sr_comm_init_shm): the ranks' hosts walk the outcome words K2 wrote; no allreduce, no K3,
    # only the host walk (SHM_US) on top of the one-GPU tick
    for c, p in scaling.PARTS.items():
        assert scaling.predict_tick_us(p, n, "weak", "shm") == pytest.approx(
            scaling.predict_tick_us(p, 1, "weak") + scaling.SHM_US)
        assert scaling.predict_tick_us(p, n, "weak", "shm") < scaling.predict_tick_us(p, n, "weak", "rccl")
        assert scaling.predict(c, n, "shm")["transport"] == "shm"
