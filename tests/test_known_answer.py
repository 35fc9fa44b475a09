"""Known-answer tests for the scheduler filters (tests/known_answer.py): every
hand-derived answer on the oracle (CPU) and on the GPU path through the C-ABI:
sr_find_spot_nodes one spot node at a time (the per-node answer) and sr_plan
over all nodes of the case (first fit = the first node whose answer is yes)."""
import dataclasses

import numpy as np
import pytest

from helpers import Scenario
from known_answer import cases
from oracle_lib import load_oracle
from spotplanner import capi
from spotplanner.model import Taint

CASES = cases()
IDS = [c.name for c in CASES]


@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_oracle_known_answer(case):
    sc = Scenario(case.nodes, case.base, [case.pod])
    osnap = sc.oracle_snapshot()
    lib = load_oracle()
    got = [lib.oracle_check_predicates(osnap.h, sc.ptr, sc.qidx(0), i) for i in range(len(case.nodes))]
    assert got == [1 if f else 0 for f in case.fits], (case.rule, got)
    first = next((i for i, f in enumerate(case.fits) if f), -1)
    assert lib.oracle_find_spot_node_for_pod(osnap.h, sc.ptr, sc.qidx(0)) == first


def test_known_answer_covers_every_filter():
    names = " ".join(IDS)
    for word in ("memory", "ephemeral", "pod_count", "zero_request", "init_container", "overhead",
                 "prefer_no_schedule", "empty_effect", "empty_key_exists", "equal_with_empty_value",
                 "unschedulable_without", "unschedulable_tolerated", "not_in_missing_key",
                 "does_not_exist_missing_key", "empty_term_list", "empty_term_matches", "node_selector_and_terms",
                 "match_fields_name", "wildcard_against_specific", "protocol_separates"):
        assert word in names, word


def _gpu_first_fit(checker, sc, n_nodes):
    lib = capi.load_planner()
    h = sc.product_snapshot()
    try:
        idx = np.array([sc.qidx(0)], np.int32)
        out = np.full(1, -7, np.int32)
        fb = np.zeros(1, np.uint8)
        st = lib.sr_find_spot_nodes(checker.handle, h, sc.ptr, capi.ptr(idx, capi.P32), 1, capi.ptr(out, capi.P32),
                                    capi.ptr(fb, capi.PU8))
        assert st == capi.SR_OK, checker.last_error()
        assert fb[0] == 0
        return int(out[0])
    finally:
        lib.sr_snapshot_destroy(h)


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES, ids=IDS)
def test_gpu_known_answer(checker, case):
    inter_pod = case.name.startswith(("aff_", "anti_"))
    for i, node in enumerate(case.nodes):  # the answer of every node on its own
        if inter_pod:
            # the topology domain spans the other nodes' pods: keep every node,
            # and keep the pod off the others with a taint it does not tolerate
            others = [dataclasses.replace(n, taints=list(n.taints) + [Taint("ka-only-this-node")]) if j != i else n
                      for j, n in enumerate(case.nodes)]
            sc = Scenario(others, case.base, [case.pod])
            want = i if case.fits[i] else -1
        else:
            sc = Scenario([node], [case.base[i]], [case.pod])
            want = 0 if case.fits[i] else -1
        assert _gpu_first_fit(checker, sc, len(sc.nodes)) == want, (case.rule, node.name)
    # first fit over all nodes, through the batched planner (one candidate)
    sc = Scenario(case.nodes, case.base, [case.pod])
    first = next((i for i, f in enumerate(case.fits) if f), -1)
    assert _gpu_first_fit(checker, sc, len(case.nodes)) == first
    from spotplanner.rescheduler import plan_arrays
    lib = capi.load_planner()
    h = sc.product_snapshot()
    try:
        p = plan_arrays(checker, h, sc.ptr, np.array([0, 1], np.int32), np.array([sc.qidx(0)], np.int32))
    finally:
        lib.sr_snapshot_destroy(h)
    assert list(p.status) == [capi.SR_CAND_OK if first >= 0 else 0]
    assert list(p.node_of_pod) == [first]
