"""Scenarios and checks for the reference-faithful tick (sr_plan_first): run()
walks the on-demand candidates in order, routes nothing anywhere, and drains
the first one whose pods all fit (rescheduler.go:228-287, break at :286).  The
product plans prefix batches; a candidate outside the encoded predicate set
goes to the reference path (SR_CAND_FALLBACK), and the product may name a
winner only when no such candidate precedes it.

`plan_first_scenario(seed)` places a drainable candidate at a chosen index
(earlier candidates carry a pod that fits nowhere, at a random position, so
their partial mappings are exercised), then routes chosen candidates to the
fallback path (a PVC) before, right after, far after, or instead of it -- on
both sides of the prefix-batch boundaries of batch sizes 2 (2, 6, 14, 30) and
16 -- with hostname or zone (anti-)affinity on some seeds."""
from __future__ import annotations

import random

import numpy as np

from randcluster import rand_scenario
from spotplanner import capi
from spotplanner.model import Container, Pod, Toleration

PATTERNS = ("fallback_just_before_winner", "fallback_in_first_batch", "fallback_right_after_winner",
            "fallback_far_after_winner", "no_drainable_candidate", "winner_itself_falls_back")


def plan_first_scenario(seed: int, n_cand: int = 24):
    r = random.Random(77_000 + seed)
    kw = {}
    if seed % 4 == 1:
        kw = dict(anti=0.35, hostname_only=True)
    elif seed % 4 == 2:
        kw = dict(anti=0.3, shared_keys=True, valid_selectors=True)
    elif seed % 4 == 3:
        kw = dict(anti=0.15, aff=0.3, valid_selectors=True)
    nodes, spot_pods, cands = rand_scenario(9600 + seed, n_spot=8 + seed % 9, n_cand=n_cand, max_pods=6, **kw)
    for c in cands:  # only the injected candidates leave the encoded set
        for p in c:
            p.init_containers = []
            for ct in p.containers:
                ct.scalar = {}
    pattern = PATTERNS[seed % len(PATTERNS)]
    win = 1 + (seed * 5) % (n_cand - 6)  # 1..18: before and after the boundaries 2, 6, 14, 16
    ns = cands[0][0].namespace if cands[0] else "default"
    easy = Pod("easy%d" % seed, namespace=ns, containers=[Container(cpu_milli=1)],
               tolerations=[Toleration("", "Exists")])
    if kw:
        easy.labels = {"app": "other"}
    for c in range(n_cand):
        if c < win or pattern == "no_drainable_candidate":
            # fits nowhere: this candidate fails at that pod, after placing the ones before it
            huge = Pod("huge%d_%d" % (seed, c), namespace=ns, containers=[Container(cpu_milli=10 ** 9)])
            cands[c].insert(r.randint(0, len(cands[c])), huge)
        elif c == win:
            cands[c] = [easy]
    fb = []
    if pattern == "fallback_just_before_winner":
        fb = [win - 1]
    elif pattern == "fallback_in_first_batch":
        fb = [0]
    elif pattern == "fallback_right_after_winner":
        fb = [win + 1]
    elif pattern == "fallback_far_after_winner":
        fb = [min(n_cand - 1, win + 15)]
    elif pattern == "no_drainable_candidate":
        fb = [win, min(n_cand - 1, win + 3)]
    elif pattern == "winner_itself_falls_back":
        fb = [win]
    for c in fb:
        if not cands[c]:
            cands[c] = [Pod("pvc%d" % c, namespace=ns, containers=[Container(cpu_milli=1)])]
        cands[c][r.randrange(len(cands[c]))].has_pvc = True  # VolumeBinding et al.: outside the encoded set
    return nodes, spot_pods, cands, pattern, win, fb


def check_plan_first(first_ok, first_fallback, winner, wmap, status, nodes, ref_all, ref_early, cand_off,
                     full=True, cand_global=None):
    """sr_plan_first against the oracle: the early-exit loop's first drainable
    candidate, winner (-1 when a fallback candidate precedes it) and mapping;
    the first fallback before the winner; every candidate the product evaluated
    (`status` != SKIPPED, per global index) equal to the all-candidates oracle,
    and every candidate below the winner evaluated."""
    assert first_ok == ref_early["first_ok"] == ref_all["first_ok"], (first_ok, ref_early["first_ok"])
    assert winner == ref_early["winner"], (winner, ref_early["winner"])
    if first_ok >= 0 and wmap is not None:
        seg = slice(int(cand_off[first_ok]), int(cand_off[first_ok + 1]))
        assert list(wmap) == list(ref_all["node_of_pod"][seg]) == list(ref_early["winner_map"])
    fb_before = ref_early["first_fallback"]  # the early loop stops at first_ok: fallbacks before it only
    if fb_before >= 0:
        assert first_fallback == fb_before, (first_fallback, fb_before)
    else:
        assert first_fallback < 0 or (first_ok >= 0 and first_fallback > first_ok), (first_fallback, first_ok)
    if winner < 0 and first_ok >= 0:
        assert 0 <= first_fallback < first_ok
    if not full:
        return
    n = len(cand_off) - 1
    glob = np.arange(n) if cand_global is None else np.asarray(cand_global)
    for k, c in enumerate(glob):
        c = int(c)
        if status[k] == capi.SR_CAND_SKIPPED:
            assert first_ok >= 0 and c > first_ok, c  # nothing below the winner is skipped
            continue
        assert status[k] == ref_all["status"][c], (c, status[k], ref_all["status"][c])
        if status[k] != capi.SR_CAND_FALLBACK:
            seg = slice(int(cand_off[c]), int(cand_off[c + 1]))
            assert list(nodes[k]) == list(ref_all["node_of_pod"][seg]), c
