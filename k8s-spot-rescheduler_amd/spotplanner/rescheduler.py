"""Mirror of the reference's planning functions (rescheduler.go, package main).

findSpotNodeForPod (rescheduler.go:338-353), canDrainNode (:357-370),
validateArgs (:407-417), podID (:402-404), and plan_arrays: the planning
segment of run() (:228-287) evaluated for every candidate at once on the GPU.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import capi
from .model import EncodedDrain, NilControllerPanic, Node, Pod, PodDisruptionBudget, encode_cluster, pod_id
from .planner import ClusterSnapshot, FallbackRequired, PlannerError, PredicateChecker
from .synth import pods_for_deletion

podID = pod_id


class GoError(Exception):
    """A Go `error` value: str(err) is its Error() text."""


def validateArgs(OnDemandNodeLabel: str, SpotNodeLabel: str) -> Optional[GoError]:
    """rescheduler.go:407-417."""
    if len(OnDemandNodeLabel.split("=")) > 2:
        return GoError("the on demand node label is not correctly formatted: expected '<label_name>' or "
                       "'<label_name>=<label_value>', but got %s" % OnDemandNodeLabel)
    if len(SpotNodeLabel.split("=")) > 2:
        return GoError("the spot node label is not correctly formatted: expected '<label_name>' or "
                       "'<label_name>=<label_value>', but got %s" % SpotNodeLabel)
    return None


@dataclass
class BlockingPod:
    """drain.BlockingPod: the pod that stops a node from being drained and why (capi.SR_BLOCK_*)."""
    Pod: Pod
    Reason: int


def _block_error(pod: Pod, reason: int) -> GoError:
    """The error texts of drain.GetPodsForDeletionOnNodeDrain [upstream CA @03f60a4c3818]."""
    if reason == capi.SR_BLOCK_NOT_REPLICATED:
        return GoError("%s/%s is not replicated" % (pod.namespace, pod.name))
    if reason == capi.SR_BLOCK_UNMOVABLE_KUBE_SYSTEM:
        return GoError("non-daemonset, non-mirrored, non-pdb-assigned kube-system pod present: %s" % pod.name)
    if reason == capi.SR_BLOCK_LOCAL_STORAGE:
        return GoError("pod with local storage present: %s" % pod.name)
    if reason == capi.SR_BLOCK_NOT_SAFE_TO_EVICT:
        return GoError("pod annotated as not safe to evict present: %s" % pod.name)
    return GoError("error matching pods to pdbs")


def podsForDeletion(podList: Sequence[Pod], pdbs: Sequence[PodDisruptionBudget], deleteNonReplicatedPods: bool = False):
    """The pods run() moves off one on-demand node (rescheduler.go:231-256):
    GetPodsForDeletionOnNodeDrain(nodeInfo.Pods, pdbs, *deleteNonReplicatedPods,
    false, false, nil, 0, now), then the DaemonSet-owner filter.  Returns
    (podsForDeletion, blockingPod, err); evaluated by the planner library
    (sr_pods_for_deletion).  A nil OwnerReference.Controller reached by the
    filter raises NilControllerPanic, as the reference panics."""
    pods = list(podList)
    enc = encode_cluster([Node("node", 0)], pods, pod_node=[0] * len(pods))
    drain = EncodedDrain(pods, list(pdbs))
    lib = capi.load_planner()
    off, idx, bp, br, st = pods_for_deletion(lib.sr_pods_for_deletion, enc.ptr, drain.ptr, np.zeros(1, np.int32),
                                             np.array([0, len(pods)], np.int32), np.arange(len(pods), dtype=np.int32),
                                             deleteNonReplicatedPods)
    if st == capi.SR_ERR_NIL_CONTROLLER:
        raise NilControllerPanic("nil OwnerReference.Controller (rescheduler.go:244)")
    if st != capi.SR_OK:
        raise PlannerError("sr_pods_for_deletion: status %d" % st)
    if bp[0] >= 0:
        blocking = pods[int(bp[0])]
        return [], BlockingPod(blocking, int(br[0])), _block_error(blocking, int(br[0]))
    return [pods[int(i)] for i in idx], None, None


def updateSpotNodeMetrics(spotNodeInfos, pdbs: Sequence[PodDisruptionBudget], deleteNonReplicatedPods: bool = False):
    """updateSpotNodeMetrics (rescheduler.go:388-399): per spot node, the number of
    pods GetPodsForDeletionOnNodeDrain returns (the pods the rescheduler
    understands), {node name: count}; nodes whose call errors are skipped, as the
    reference logs and continues.  The Prometheus gauge itself stays in the Go
    shim (metrics.UpdateNodePodsCount(SpotNodeLabel, name, count))."""
    infos = list(spotNodeInfos)
    pods, pod_node = [], []
    for i, ni in enumerate(infos):
        pods.extend(ni.Pods)
        pod_node.extend([i] * len(ni.Pods))
    enc = encode_cluster([ni.Node for ni in infos], pods, pod_node=pod_node)
    drain = EncodedDrain(pods, list(pdbs))
    off = np.zeros(len(infos) + 1, np.int32)
    off[1:] = np.cumsum([len(ni.Pods) for ni in infos])
    out_off, _, bp, _, st = pods_for_deletion(capi.load_planner().sr_pods_for_deletion, enc.ptr, drain.ptr,
                                              np.arange(len(infos), dtype=np.int32), off,
                                              np.arange(len(pods), dtype=np.int32), deleteNonReplicatedPods,
                                              owner_filter=False)
    if st != capi.SR_OK:
        raise PlannerError("sr_pods_for_deletion: status %d" % st)
    return {ni.Node.name: int(out_off[i + 1] - out_off[i]) for i, ni in enumerate(infos) if bp[i] < 0}


def _node_names(nodes) -> List[str]:
    return [ni.Node.name for ni in nodes]


def _check_order(snapshot: ClusterSnapshot, nodes):
    snapshot.materialize()
    if _node_names(nodes) != snapshot.node_names():
        raise PlannerError("NodeInfoArray order must be the snapshot's node order")


def findSpotNodeForPod(predicateChecker: PredicateChecker, spotSnapshot: ClusterSnapshot, nodes,
                       pod: Pod) -> str:
    """First spot node in NodeInfoArray order whose predicates pass, else ""."""
    if len(nodes) == 0:
        return ""
    pod.node_name = ""  # :341 — pretend the pod is not scheduled
    _check_order(spotSnapshot, nodes)
    enc = spotSnapshot.encode_pods([pod])
    idx = np.zeros(1, np.int32)
    out = np.full(1, -1, np.int32)
    fb = np.zeros(1, np.uint8)
    lib = predicateChecker.lib
    st = lib.sr_find_spot_nodes(predicateChecker.handle, spotSnapshot.handle, enc.ptr, capi.ptr(idx, capi.P32), 1,
                                capi.ptr(out, capi.P32), capi.ptr(fb, capi.PU8))
    if st != capi.SR_OK:
        raise PlannerError("sr_find_spot_nodes: %d %s" % (st, predicateChecker.last_error()))
    if fb[0]:
        raise FallbackRequired(pod_id(pod))
    return nodes[int(out[0])].Node.name if out[0] >= 0 else ""


def canDrainNode(predicateChecker: PredicateChecker, spotSnapshot: ClusterSnapshot, nodes,
                 pods: Sequence[Pod]) -> Optional[GoError]:
    """Places pods one by one (first fit) and adds each to the snapshot; returns
    the reference's error for the first pod that fits nowhere, else None."""
    if len(pods) == 0:
        return None
    _check_order(spotSnapshot, nodes)
    enc = spotSnapshot.encode_pods(list(pods))
    idx = np.arange(len(pods), dtype=np.int32)
    mapping = np.full(len(pods), -1, np.int32)
    fail = ctypes.c_int32(-1)
    fb = ctypes.c_uint8(0)
    lib = predicateChecker.lib
    st = lib.sr_can_drain_node(predicateChecker.handle, spotSnapshot.handle, enc.ptr, capi.ptr(idx, capi.P32),
                               len(pods), capi.ptr(mapping, capi.P32), ctypes.byref(fail), ctypes.byref(fb))
    if st != capi.SR_OK:
        raise PlannerError("sr_can_drain_node: %d %s" % (st, predicateChecker.last_error()))
    if fb.value:
        raise FallbackRequired(", ".join(pod_id(p) for p in pods))
    if len(nodes) > 0:
        # :341 runs for every pod findSpotNodeForPod evaluates: up to and
        # including the first pod that fits nowhere (canDrainNode returns there)
        evaluated = pods if fail.value < 0 else pods[:fail.value + 1]
        for p in evaluated:
            p.node_name = ""
    canDrainNode.last_mapping = [nodes[int(k)].Node.name if k >= 0 else "" for k in mapping]
    if fail.value >= 0:
        return GoError("pod %s can't be rescheduled on any existing spot node" % pod_id(pods[fail.value]))
    return None


canDrainNode.last_mapping = []


@dataclass
class PlanResult:
    winner: int            # index of the candidate run() drains, -1 none / unresolved
    first_ok: int
    first_fallback: int
    status: np.ndarray     # per candidate: SR_CAND_* or failing pod index
    node_of_pod: np.ndarray  # flat, spot position per candidate pod (-1 not placed)
    winner_map: np.ndarray
    checks: int
    fallback_pods: int


def plan_arrays(predicateChecker: PredicateChecker, snapshot_handle, cluster_ptr, cand_off: np.ndarray,
                cand_pods: np.ndarray, cand_global: Optional[np.ndarray] = None, full: bool = True) -> PlanResult:
    """sr_plan over caller-built arrays (the batched drop-in of rescheduler.go:228-287)."""
    lib = predicateChecker.lib
    n = len(cand_off) - 1
    c = capi.sr_candidates(n, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32),
                           capi.ptr(cand_global, capi.P32) if cand_global is not None else None)
    maxp = int(np.max(np.diff(cand_off))) if n > 0 else 0
    status = np.zeros(max(n, 1), np.int32)
    nodes = np.zeros(max(int(cand_off[-1]) if n > 0 else 0, 1), np.int32)
    wmap = np.full(max(maxp, 1), -1, np.int32)
    o = capi.sr_plan_out()
    o.status = capi.ptr(status, capi.P32) if full else None
    o.node_of_pod = capi.ptr(nodes, capi.P32) if full else None
    o.winner_map = capi.ptr(wmap, capi.P32)
    st = lib.sr_plan(predicateChecker.handle, snapshot_handle, cluster_ptr, ctypes.byref(c), ctypes.byref(o))
    if st != capi.SR_OK:
        raise PlannerError("sr_plan: %d %s" % (st, predicateChecker.last_error()))
    return PlanResult(o.winner, o.first_ok, o.first_fallback, status[:n], nodes[: int(cand_off[-1]) if n else 0],
                      wmap[: o.winner_npods], int(o.checks), int(o.fallback_pods))
