"""bench.py --gpus N without torch.distributed.run: the launcher starts N
rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, LOCAL_RANK =
the GPU ordinal), never touches the GPU itself, refuses N > visible devices,
and fails when a rank fails.  CPU-only: the ranks here are a stub script."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402

STUB = """
import json, os, sys
out = sys.argv[sys.argv.index("--out") + 1]
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys} | {"argv": sys.argv[1:]}, f)
if "--fail-rank" in sys.argv and os.environ["RANK"] == sys.argv[sys.argv.index("--fail-rank") + 1]:
    sys.exit(7)
"""


@pytest.fixture
def stub(tmp_path):
    p = tmp_path / "stub.py"
    p.write_text(STUB)
    return str(p)


@pytest.mark.parametrize("n", [2, 4, 8])
def test_launcher_starts_n_ranks_with_their_environment(stub, tmp_path, n):
    rc = bench.launch_ranks(n, ["--gpus", str(n), "--out", str(tmp_path)], script=stub, devices=n)
    assert rc == 0
    seen = [json.load(open(tmp_path / ("rank%d.json" % r))) for r in range(n)]
    ports = {s["MASTER_PORT"] for s in seen}
    assert len(ports) == 1
    for r, s in enumerate(seen):
        assert s["RANK"] == s["LOCAL_RANK"] == str(r)
        assert s["WORLD_SIZE"] == s["LOCAL_WORLD_SIZE"] == str(n)
        assert s["MASTER_ADDR"] == "127.0.0.1"
        assert s["argv"][:2] == ["--gpus", str(n)]


def test_launcher_refuses_more_ranks_than_devices(stub, tmp_path):
    assert bench.launch_ranks(4, ["--out", str(tmp_path)], script=stub, devices=2) == 2
    assert not list(tmp_path.glob("rank*.json"))


def test_launcher_fails_when_a_rank_fails(stub, tmp_path):
    assert bench.launch_ranks(3, ["--out", str(tmp_path), "--fail-rank", "1"], script=stub, devices=3) == 7


def test_bench_gpus_2_without_a_gpu_fails_loudly():
    """No HIP device here: `bench.py --gpus 2` refuses instead of running one rank."""
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "1"],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "refusing" in r.stderr and r.stdout == ""


def _fake_kfd(tmp_path, simds):
    base = tmp_path / "kfd_nodes"
    for i, s in enumerate(simds):
        d = base / str(i)
        d.mkdir(parents=True)
        (d / "properties").write_text("cpu_cores_count 0\nsimd_count %d\nmem_banks_count 1\n" % s)
    return str(base)


def test_visible_devices_counts_gpu_agents_without_hip(tmp_path):
    """The launcher counts GPUs from the KFD topology (simd_count > 0), never through HIP."""
    kfd = _fake_kfd(tmp_path, [0, 1024, 1024, 1024, 0])  # two CPU agents, three GPUs
    assert bench.visible_devices(kfd, environ={}) == 3
    assert bench.visible_devices(kfd, environ={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.visible_devices(kfd, environ={"ROCR_VISIBLE_DEVICES": "2"}) == 1
    assert bench.visible_devices(str(tmp_path / "missing"), environ={}) == 0
    assert "torch" not in bench.visible_devices.__code__.co_names


@pytest.fixture(scope="module")
def c3_lists():
    sys.path.insert(0, os.path.join(REPO, "k8s-spot-rescheduler_amd"))
    import ctypes

    from spotplanner import capi
    from spotplanner.synth import SynthCluster, new_node_map, pods_for_deletion
    lib = capi.load_planner()
    sc = SynthCluster(3, n_on_demand=bench.cluster_on_demand(3, 8, "strong"))
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    off, pods, _, _, st = pods_for_deletion(lib.sr_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain),
                                            nm.on_demand, nm.node_pod_off, nm.node_pod_idx)
    assert st == capi.SR_OK
    return sc, nm, off, pods


@pytest.mark.parametrize("n", [2, 4, 8])
def test_strong_scaling_shards_the_c3_cluster(c3_lists, n):
    """--scaling strong keeps BASELINE's C3 cluster (5,000 nodes: 1,500 on-demand / 3,500 spot) at
    every N and splits its 1,500 candidates c % N; the workload string names the counts actually planned."""
    from spotplanner.synth import shard
    sc, nm, off, pods = c3_lists
    assert bench.cluster_on_demand(3, n, "strong") == 1500
    assert (sc.n_nodes, len(nm.on_demand), len(nm.spot)) == (5000, 1500, 3500)
    sizes = bench.shard_sizes(len(off) - 1, n)
    assert sum(sizes) == 1500 and max(sizes) - min(sizes) <= 1
    assert sizes == [len(range(r, 1500, n)) for r in range(n)]
    seen = []
    for r in range(n):
        lo, lp, gidx = shard(off, pods, r, n)
        assert len(lo) - 1 == sizes[r]
        assert np.array_equal(gidx, np.arange(r, 1500, n))
        assert len(lp) == sum(int(off[g + 1] - off[g]) for g in gidx)
        seen.extend(gidx.tolist())
    assert sorted(seen) == list(range(1500))
    w = bench.workload_name(3, sc.n_nodes, len(nm.on_demand), len(nm.spot), sc.n_pods, n, "strong")
    assert w.startswith("C3 5000 nodes (1500 od / 3500 spot) / %d pods" % sc.n_pods)
    assert "strong scaling: 1500 candidates sharded c %% %d" % n in w


@pytest.mark.parametrize("n", [2, 8])
def test_weak_scaling_multiplies_candidates_and_says_so(n):
    assert bench.cluster_on_demand(3, n, "weak") == 1500 * n
    assert bench.cluster_on_demand(4, 8, "strong") == 15000
    w = bench.workload_name(3, 3500 + 1500 * n, 1500 * n, 3500, 1, n, "weak")
    assert w.startswith("C3 %d nodes (%d od / 3500 spot)" % (3500 + 1500 * n, 1500 * n))
    assert "weak scaling" in w


def test_bench_defaults_to_strong_scaling_with_weak_beside():
    # BASELINE names C3 on 1/2/4/8 GPUs: the parsed line is the config's own cluster split over the ranks
    # (strong); the weak-scaled tick (N x the candidates) is measured beside it and labelled, never the value
    src = open(os.path.join(REPO, "bench.py")).read()
    assert 'ap.add_argument("--scaling", default="strong"' in src and '"scaling": args.scaling' in src
    assert '"weak_scaling": weak_scaling' in src and "not the line's value" in src
    assert 'ap.add_argument("--transport", default="shm"' in src
