"""bench.py --gpus N without torch.distributed.run: the launcher starts N
rank processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, LOCAL_RANK =
the GPU ordinal), never touches the GPU itself, refuses N > visible devices,
and fails when a rank fails.  CPU-only: the ranks here are a stub script."""
import json
import os
import subprocess
import sys

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
