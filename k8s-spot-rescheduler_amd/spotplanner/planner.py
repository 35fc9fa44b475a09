"""Device planner handle + cluster snapshot (ctypes over libsrplanner.so).

`PredicateChecker` owns an sr_ctx: it replaces the cluster-autoscaler
SchedulerBasedPredicateChecker the reference builds once per process
(rescheduler.go:149; tests: rescheduler_test.go:41,103).  `ClusterSnapshot`
owns an sr_snapshot (CA Basic/DeltaClusterSnapshot: AddNodeWithPods, AddPod,
Fork, Revert).  Every evaluation runs on the GPU through the C-ABI; there is
no CPU code path here.
"""
from __future__ import annotations

import ctypes
from typing import Dict, List, Optional

import numpy as np

from . import capi
from .model import EncodedCluster, Interner, Node, Pod, encode_cluster


class PlannerError(RuntimeError):
    pass


class FallbackRequired(RuntimeError):
    """The pods use predicates outside the encoded set: the caller must run the
    reference path (the Go drop-in calls the original canDrainNode)."""


def _check(lib, status, ctx=None, what="call"):
    if status != capi.SR_OK:
        msg = ""
        if ctx is not None:
            msg = lib.sr_last_error(ctx).decode(errors="replace")
        raise PlannerError("%s failed with status %d %s" % (what, status, msg))


class PredicateChecker:
    def __init__(self, device: int = 0):
        self.lib = capi.load_planner()
        h = ctypes.c_void_p()
        st = self.lib.sr_create(device, ctypes.byref(h))
        if st == capi.SR_ERR_NO_DEVICE:
            raise PlannerError("no HIP device: the drain planner runs only on the GPU")
        _check(self.lib, st, what="sr_create")
        self.handle = h

    def close(self):
        if getattr(self, "handle", None):
            self.lib.sr_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        return self.lib.sr_last_error(self.handle).decode(errors="replace")

    def set_timing(self, mask: int):
        """Bracket kernels with HIP events: 1 K0, 2 K2, 4 K3 (+collective)."""
        self.lib.sr_set_timing(self.handle, int(mask))

    def timing(self) -> capi.sr_timing:
        t = capi.sr_timing()
        self.lib.sr_get_timing(self.handle, ctypes.byref(t))
        return t

    def attach_collective(self, nranks: int, rank: int, allreduce_min):
        """sr_comm_init_host: the planner's allreduce(min) over the ranks is
        `allreduce_min(values: list[int]) -> list[int]` (e.g. torch.distributed
        over gloo), instead of RCCL."""
        def fn(_user, words, n):
            try:
                out = allreduce_min([int(words[i]) for i in range(n)])
                for i in range(n):
                    words[i] = int(out[i])
                return 0
            except Exception:  # noqa: BLE001 -- reported to the planner as a failed collective
                return 1
        self._collective = capi.ALLREDUCE_MIN_FN(fn)  # kept alive as long as the handle
        _check(self.lib, self.lib.sr_comm_init_host(self.handle, nranks, rank, self._collective, None), self.handle,
               "sr_comm_init_host")

    def attach_shared_memory(self, name: str, session: int, nranks: int, rank: int, max_cand: int):
        """sr_comm_init_shm: the ranks of one node reduce each tick through one
        shared-memory segment (`name`, identical on every rank): each rank's K2
        writes its outcomes there and each host walks them in global candidate
        order; shards must be interleaved (cand_global = (first + i) * nranks + rank)."""
        _check(self.lib, self.lib.sr_comm_init_shm(self.handle, name.encode(), session & 0xffffffff, nranks, rank,
                                                   max_cand), self.handle, "sr_comm_init_shm")


def NewTestPredicateChecker(device: int = 0):
    """simulator.NewTestPredicateChecker() -> (checker, err) (rescheduler_test.go:41)."""
    return PredicateChecker(device), None


def NewSchedulerBasedPredicateChecker(kube_client=None, stop=None, device: int = 0):
    """simulator.NewSchedulerBasedPredicateChecker (rescheduler.go:149)."""
    return PredicateChecker(device), None


class ClusterSnapshot:
    """Spot-node snapshot; nodes are scanned in the order they were added."""

    def __init__(self, interner: Optional[Interner] = None):
        self.lib = capi.load_planner()
        self.interner = interner or Interner()
        self._nodes: List[Node] = []
        self._pods: List[List[Pod]] = []
        self.handle = None
        self._pos: Dict[str, int] = {}

    # -- construction ----------------------------------------------------
    def AddNodeWithPods(self, node: Node, pods: List[Pod]):
        if self.handle is not None:
            raise PlannerError("AddNodeWithPods after the snapshot was materialised")
        self._pos[node.name] = len(self._nodes)
        self._nodes.append(node)
        self._pods.append(list(pods))

    def materialize(self):
        if self.handle is not None:
            return
        pods, pod_node = [], []
        for i, ps in enumerate(self._pods):
            pods.extend(ps)
            pod_node.extend([i] * len(ps))
        enc = encode_cluster(self._nodes, pods, self.interner, pod_node=pod_node)
        off = np.zeros(len(self._nodes) + 1, dtype=np.int32)
        for i, ps in enumerate(self._pods):
            off[i + 1] = off[i] + len(ps)
        idx = np.arange(len(pods), dtype=np.int32)
        spot = np.arange(len(self._nodes), dtype=np.int32)
        h = ctypes.c_void_p()
        st = self.lib.sr_snapshot_create(enc.ptr, capi.ptr(spot, capi.P32), len(self._nodes),
                                         capi.ptr(off, capi.P32), capi.ptr(idx, capi.P32), ctypes.byref(h))
        _check(self.lib, st, what="sr_snapshot_create")
        self.handle = h

    @classmethod
    def from_handle(cls, handle, interner: Interner, node_names: List[str]):
        s = cls(interner)
        s.handle = handle
        s._pos = {n: i for i, n in enumerate(node_names)}
        s._nodes = [None] * len(node_names)
        return s

    def close(self):
        if self.handle is not None:
            self.lib.sr_snapshot_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- ClusterSnapshot interface ----------------------------------------
    def node_names(self) -> List[str]:
        return sorted(self._pos, key=self._pos.get)

    def position(self, node_name: str) -> int:
        return self._pos[node_name]

    def encode_pods(self, pods: List[Pod]) -> EncodedCluster:
        return encode_cluster([], pods, self.interner, pod_node=[-1] * len(pods))

    def AddPod(self, pod: Pod, node_name: str):
        self.materialize()
        enc = self.encode_pods([pod])
        _check(self.lib, self.lib.sr_snapshot_add_pod(self.handle, enc.ptr, 0, self._pos[node_name]),
               what="sr_snapshot_add_pod")

    def Fork(self):
        self.materialize()
        return self.lib.sr_snapshot_fork(self.handle)

    def Revert(self):
        self.materialize()
        return self.lib.sr_snapshot_revert(self.handle)

    def node_state(self, node_name: str):
        """(requested cpu, memory, ephemeral), number of pods of a snapshot node."""
        self.materialize()
        req = np.zeros(3, dtype=np.int64)
        n = ctypes.c_int32()
        _check(self.lib, self.lib.sr_snapshot_node_state(self.handle, self._pos[node_name],
                                                         capi.ptr(req, capi.P64), ctypes.byref(n)))
        return tuple(int(x) for x in req), int(n.value)


def NewBasicClusterSnapshot(interner: Optional[Interner] = None) -> ClusterSnapshot:
    return ClusterSnapshot(interner)


def NewDeltaClusterSnapshot(interner: Optional[Interner] = None) -> ClusterSnapshot:
    return ClusterSnapshot(interner)
