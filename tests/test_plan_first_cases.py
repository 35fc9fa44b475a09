"""CPU checks of the sr_plan_first scenarios (tests/plan_first_cases.py) on
the oracle: the seeds the GPU tests use reach every fallback pattern."""
import numpy as np

from helpers import Scenario
from oracle_lib import oracle_plan
from plan_first_cases import PATTERNS, plan_first_scenario


def test_plan_first_scenarios_cover_every_pattern():
    """The seeds above reach every pattern, a winner masked by a preceding
    fallback candidate, and winners on both sides of the batch boundaries."""
    seen, masked, wins = set(), 0, set()
    for seed in range(24):
        nodes, spot_pods, cands, pattern, win, fb = plan_first_scenario(seed)
        flat = [p for c in cands for p in c]
        sc = Scenario(nodes, spot_pods, flat)
        cand_off = np.cumsum([0] + [len(c) for c in cands]).astype(np.int32)
        cand_pods = np.arange(sc.q0, sc.q0 + len(flat), dtype=np.int32)
        e = oracle_plan(sc.oracle_snapshot(), sc.ptr, cand_off, cand_pods, mode=0)
        seen.add(pattern)
        masked += e["first_ok"] >= 0 and e["winner"] < 0
        if e["winner"] >= 0:
            wins.add(e["winner"])
    assert seen == set(PATTERNS) and masked >= 4
    assert max(wins) >= 16 and any(2 <= w < 6 for w in wins) and any(6 <= w < 14 for w in wins)
