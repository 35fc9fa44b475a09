#!/usr/bin/env python3
"""Randomised parity stress (tools only): product vs oracle on many seeded
scenarios, mixing every encoded feature, inter-pod (anti-)affinity on hostname
and shared keys, topology spread, large candidates and wide pools.  Runs until --seconds elapse
and prints the first mismatch.  GPU required.

  python tools/parity_stress.py [--seconds 180] [--seed0 100000]
"""
import argparse
import os
import sys
import time
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "k8s-spot-rescheduler_amd")]

from randcluster import rand_scenario  # noqa: E402
from spotplanner.planner import PredicateChecker  # noqa: E402
import test_gpu_parity as P  # noqa: E402
import test_topology_spread as S  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=180.0)
    ap.add_argument("--seed0", type=int, default=100000)
    a = ap.parse_args()
    chk = PredicateChecker(0)
    t0, n, seed = time.time(), 0, a.seed0
    kinds = {}
    try:
        while time.time() - t0 < a.seconds:
            k = seed % 11
            if k == 0:
                args = dict(n_spot=5 + seed % 60, n_cand=12, max_pods=4 + seed % 30)
            elif k == 1:
                args = dict(n_spot=8 + seed % 30, n_cand=10, max_pods=12, anti=0.4, hostname_only=True)
            elif k == 2:
                args = dict(n_spot=6 + seed % 20, n_cand=8, max_pods=10, anti=0.3, shared_keys=True,
                            valid_selectors=True)
            elif k == 3:
                args = dict(n_spot=6 + seed % 20, n_cand=8, max_pods=10, aff=0.3, shared_keys=seed % 2 == 0,
                            valid_selectors=True)
            elif k == 4:
                args = dict(n_spot=10 + seed % 40, n_cand=6, max_pods=70 + seed % 200, features=seed % 2 == 0)
            elif k == 5:
                args = dict(n_spot=4100 + seed % 3000, n_cand=6, max_pods=20)
            elif k == 6:
                args = dict(n_spot=20, n_cand=12, max_pods=8, fallback=True)
            elif k == 7:  # the domain path with 2-4 pod groups (65-230 interacting pods)
                args = dict(n_spot=20 + seed % 30, n_cand=3, max_pods=65 + seed % 165, features=False, anti=0.2,
                            aff=0.15 if seed % 2 else 0.0, shared_keys=True, valid_selectors=True)
            elif k == 8:  # scalar resources on most nodes and candidates
                args = dict(n_spot=6 + seed % 20, n_cand=12, max_pods=4 + seed % 8)
            if k == 9:  # topology spread, static and between the pods of a candidate
                nodes, spot_pods, cands = S.rand_spread_scenario(seed)
            elif k == 10:  # replica candidates of 65-230 pods spread over zones / hostnames
                nodes, spot_pods, cands = S.rand_spread_replicas(seed)
            else:
                nodes, spot_pods, cands = rand_scenario(seed, **args)
            if k == 7:
                for c in cands:  # no init containers / scalars: nothing sends them to the fallback path
                    for p in c:
                        p.init_containers = []
                        for ct in p.containers:
                            ct.scalar = {}
            if k == 8:
                import random
                r = random.Random(seed)
                for nd in nodes:
                    if r.random() < 0.7:
                        nd.scalar = {"nvidia.com/gpu": r.choice([0, 1, 2, 4]), "hugepages-2Mi": r.choice([0, 4 << 20])}
                for c in cands:
                    if c and r.random() < 0.7:
                        p = c[r.randrange(len(c))]
                        p.containers[0].scalar = {"nvidia.com/gpu": r.choice([0, 1, 2])}
                        p.containers[0].cpu_milli = max(p.containers[0].cpu_milli, 10)
            P.run_scenario(chk, nodes, spot_pods, cands)
            kinds[k] = kinds.get(k, 0) + 1
            n += 1
            seed += 1
            if n % 25 == 0:
                print("  %d scenarios, %.0f s" % (n, time.time() - t0), flush=True)
    except Exception:
        print("MISMATCH at seed %d kind %d" % (seed, seed % 11))
        traceback.print_exc()
        return 1
    finally:
        chk.close()
    print("parity stress: %d scenarios in %.0f s, all equal to the oracle (by kind: %s)" % (n, time.time() - t0, kinds))
    return 0


if __name__ == "__main__":
    sys.exit(main())
