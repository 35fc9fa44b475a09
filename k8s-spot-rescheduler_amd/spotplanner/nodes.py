"""Mirror of package nodes (nodes/nodes.go): NodeInfo, NodeInfoArray, NewNodeMap.

Names, globals and semantics follow the reference; the work is done by the
C++ host side of libsrplanner.so (sr_new_node_map: Go-exact sort.Slice, spot /
on-demand classification, priority filter).
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import numpy as np

from . import capi
from .model import Interner, Node, Pod, encode_cluster, label_flag
from .planner import ClusterSnapshot, PlannerError

# Package globals (nodes/nodes.go:31-42); run() sets them from flags.
OnDemandNodeLabel = "kubernetes.io/role=worker"
SpotNodeLabel = "kubernetes.io/role=spot-worker"
OnDemand = 0
Spot = 1
PriorityThreshold = 0


class NilPriorityPanic(RuntimeError):
    """nodes/nodes.go:139 dereferences *Spec.Priority: the reference panics on nil."""


class NodeInfo:
    """nodes.NodeInfo (nodes/nodes.go:44-50)."""

    def __init__(self, node: Node, pods: List[Pod], requested_cpu: int, free_cpu: int):
        self.Node = node
        self.Pods = pods
        self.RequestedCPU = requested_cpu
        self.FreeCPU = free_cpu

    def AddPod(self, pod: Pod):
        """NodeInfo.AddPod (nodes/nodes.go:122-126)."""
        self.Pods = self.Pods + [pod]
        self.RequestedCPU = calculateRequestedCPU(self.Pods)
        self.FreeCPU = self.Node.cpu_milli - self.RequestedCPU


class NodeInfoArray(list):
    """nodes.NodeInfoArray (nodes/nodes.go:55)."""

    def CopyNodeInfos(self) -> "NodeInfoArray":
        """nodes/nodes.go:212-224: new NodeInfo structs sharing Node and Pods."""
        return NodeInfoArray(NodeInfo(n.Node, n.Pods, n.RequestedCPU, n.FreeCPU) for n in self)

    def GetClusterSnapshot(self, interner: Optional[Interner] = None) -> ClusterSnapshot:
        """nodes/nodes.go:226-232: AddNodeWithPods per node, in array order."""
        snap = ClusterSnapshot(interner)
        for ni in self:
            snap.AddNodeWithPods(ni.Node, ni.Pods)
        snap.materialize()
        return snap


def getPodCPURequests(pod: Pod) -> int:
    """nodes/nodes.go:159-165 (the shim's Quantity conversion of each container)."""
    return pod.cpu_sort_milli()


def calculateRequestedCPU(pods: List[Pod]) -> int:
    """nodes/nodes.go:149-156."""
    return sum(getPodCPURequests(p) for p in pods)


def _has_label(node: Node, flag: str) -> bool:
    lib = capi.load_planner()
    it = Interner()
    enc = encode_cluster([node], [], it)
    lab = label_flag(flag, it)
    return bool(lib.sr_node_has_label(enc.ptr, 0, ctypes.byref(lab)))


def isSpotNode(node: Node) -> bool:
    """nodes/nodes.go:168-187."""
    return _has_label(node, SpotNodeLabel)


def isOnDemandNode(node: Node) -> bool:
    """nodes/nodes.go:190-209."""
    return _has_label(node, OnDemandNodeLabel)


def getPodsOnNode(client, node: Node) -> List[Pod]:
    """nodes/nodes.go:129-145: the LIST (client.list_pods) minus pods below
    PriorityThreshold on spot nodes; list order kept."""
    out = []
    spot = isSpotNode(node)
    for p in client.list_pods(node.name):
        if p.priority is None:
            raise NilPriorityPanic("nil Spec.Priority on %s/%s" % (p.namespace, p.name))
        if p.priority < PriorityThreshold and spot:
            continue
        out.append(p)
    return out


def NewNodeMap(client, nodes: List[Node], interner: Optional[Interner] = None) -> Dict[int, NodeInfoArray]:
    """nodes.NewNodeMap (nodes/nodes.go:63-104).  `client.list_pods(node_name)`
    plays the per-node LIST of getPodsOnNode; everything after it (filter,
    sums, Go sort.Slice, classification) runs in sr_new_node_map."""
    lib = capi.load_planner()
    it = interner or Interner()
    pods, pod_node = [], []
    for i, n in enumerate(nodes):
        listed = client.list_pods(n.name)
        pods.extend(listed)
        pod_node.extend([i] * len(listed))
    enc = encode_cluster(nodes, pods, it, pod_node=pod_node)
    params = capi.sr_node_map_params(label_flag(OnDemandNodeLabel, it), label_flag(SpotNodeLabel, it),
                                     PriorityThreshold)
    nn, np_ = len(nodes), len(pods)
    spot = np.zeros(max(nn, 1), np.int32)
    od = np.zeros(max(nn, 1), np.int32)
    ns, nod = np.zeros(1, np.int32), np.zeros(1, np.int32)
    off = np.zeros(nn + 1, np.int32)
    idx = np.zeros(max(np_, 1), np.int32)
    req = np.zeros(max(nn, 1), np.int64)
    free = np.zeros(max(nn, 1), np.int64)
    m = capi.sr_node_map(capi.ptr(spot, capi.P32), capi.ptr(ns, capi.P32), capi.ptr(od, capi.P32),
                         capi.ptr(nod, capi.P32), capi.ptr(off, capi.P32), capi.ptr(idx, capi.P32),
                         capi.ptr(req, capi.P64), capi.ptr(free, capi.P64))
    st = lib.sr_new_node_map(enc.ptr, ctypes.byref(params), ctypes.byref(m))
    if st == capi.SR_ERR_NIL_PRIORITY:
        raise NilPriorityPanic("nil Spec.Priority")
    if st != capi.SR_OK:
        raise PlannerError("sr_new_node_map failed with status %d" % st)

    def info(i):
        return NodeInfo(nodes[i], [pods[j] for j in idx[off[i]:off[i + 1]]], int(req[i]), int(free[i]))

    return {OnDemand: NodeInfoArray(info(i) for i in od[:nod[0]]),
            Spot: NodeInfoArray(info(i) for i in spot[:ns[0]])}
