"""Binding of libsrsynth.so (synthetic clusters for bench and tests) and the
tick builder used by bench.py and the parity tests: NewNodeMap ->
GetClusterSnapshot -> podsForDeletion per on-demand node."""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import capi


class sr_synth_params(ctypes.Structure):
    _fields_ = [("config", ctypes.c_int32), ("seed", ctypes.c_uint64), ("n_on_demand", ctypes.c_int32),
                ("n_spot", ctypes.c_int32), ("pinned_fraction", ctypes.c_double),
                ("stateful_fraction", ctypes.c_double), ("init_fraction", ctypes.c_double),
                ("gpu_fraction", ctypes.c_double), ("anti_fraction", ctypes.c_double),
                ("spread_fraction", ctypes.c_double)]


# The "realistic" variant of a config (bench --variant realistic): StatefulSet
# pods with zonal EBS CSI claims, init containers, GPU pods on GPU nodes.
REALISTIC = dict(stateful_fraction=0.15, init_fraction=0.2, gpu_fraction=0.3)
# The "affinity" variant (bench --variant affinity): every pod in a Deployment,
# 10 % of the Deployments with required hostname anti-affinity, 10 % with a
# zone DoNotSchedule topology spread constraint (their spot replicas included).
AFFINITY = dict(anti_fraction=0.10, spread_fraction=0.10)


_synth = None


def load_synth():
    global _synth
    if _synth is None:
        if not os.path.exists(capi.SYNTH_LIB):
            raise FileNotFoundError(capi.SYNTH_LIB + " missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(capi.SYNTH_LIB)
        lib.sr_synth_generate.argtypes = [ctypes.POINTER(sr_synth_params)]
        lib.sr_synth_generate.restype = ctypes.c_void_p
        lib.sr_synth_destroy.argtypes = [ctypes.c_void_p]
        lib.sr_synth_view.argtypes = [ctypes.c_void_p, ctypes.POINTER(capi.sr_cluster)]
        lib.sr_synth_labels.argtypes = [ctypes.c_void_p, ctypes.POINTER(capi.sr_node_label),
                                        ctypes.POINTER(capi.sr_node_label)]
        lib.sr_synth_drain.argtypes = [ctypes.c_void_p, ctypes.POINTER(capi.sr_pod_drain)]
        lib.sr_synth_string.argtypes = [ctypes.c_void_p, ctypes.c_int32]
        lib.sr_synth_string.restype = ctypes.c_char_p
        lib.sr_synth_num_strings.argtypes = [ctypes.c_void_p]
        lib.sr_synth_num_strings.restype = ctypes.c_int32
        lib.sr_synth_label_flags.argtypes = [ctypes.c_char_p]
        lib.sr_synth_label_flags.restype = ctypes.c_uint8
        _synth = lib
    return _synth


def synth_label_flags(s: str) -> int:
    """The generator's sr_cluster.str_label entry for `s` (its C++ validity functions)."""
    return int(load_synth().sr_synth_label_flags(s.encode()))


class SynthCluster:
    def __init__(self, config: int, seed: int = 0, n_on_demand: int = 0, n_spot: int = 0,
                 pinned_fraction: float = -1.0, stateful_fraction: float = 0.0, init_fraction: float = 0.0,
                 gpu_fraction: float = 0.0, anti_fraction: float = 0.0, spread_fraction: float = 0.0):
        self.lib = load_synth()
        p = sr_synth_params(config, seed, n_on_demand, n_spot, pinned_fraction, stateful_fraction, init_fraction,
                            gpu_fraction, anti_fraction, spread_fraction)
        self.handle = self.lib.sr_synth_generate(ctypes.byref(p))
        self.cluster = capi.sr_cluster()
        self.lib.sr_synth_view(self.handle, ctypes.byref(self.cluster))
        self.od_label = capi.sr_node_label()
        self.spot_label = capi.sr_node_label()
        self.lib.sr_synth_labels(self.handle, ctypes.byref(self.od_label), ctypes.byref(self.spot_label))
        self.drain = capi.sr_pod_drain()
        self.lib.sr_synth_drain(self.handle, ctypes.byref(self.drain))
        self.config = config

    @property
    def ptr(self):
        return ctypes.byref(self.cluster)

    @property
    def n_nodes(self):
        return self.cluster.nodes.n

    @property
    def n_pods(self):
        return self.cluster.pods.n

    def pod_flags(self) -> np.ndarray:
        return np.ctypeslib.as_array(self.cluster.pods.flags, shape=(self.n_pods,))

    def close(self):
        if self.handle:
            self.lib.sr_synth_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


@dataclass
class NodeMapArrays:
    spot: np.ndarray
    on_demand: np.ndarray
    node_pod_off: np.ndarray
    node_pod_idx: np.ndarray
    requested_cpu: np.ndarray
    free_cpu: np.ndarray

    def struct(self):
        ns = np.array([len(self.spot)], np.int32)
        nod = np.array([len(self.on_demand)], np.int32)
        self._keep = (ns, nod)
        return capi.sr_node_map(capi.ptr(self.spot, capi.P32), capi.ptr(ns, capi.P32),
                                capi.ptr(self.on_demand, capi.P32), capi.ptr(nod, capi.P32),
                                capi.ptr(self.node_pod_off, capi.P32), capi.ptr(self.node_pod_idx, capi.P32),
                                capi.ptr(self.requested_cpu, capi.P64), capi.ptr(self.free_cpu, capi.P64))


def new_node_map(fn, cluster_ptr, n_nodes: int, n_pods: int, od_label, spot_label, priority_threshold=0,
                 bufs: Optional[dict] = None):
    """Calls sr_new_node_map-shaped `fn` (the product's, or the oracle's in tests).
    `bufs`: output arrays kept across calls (a long-running planner's), filled
    on first use; the result's arrays are views of them."""
    def buf(name, n, dt):
        if bufs is None:
            return np.zeros(n, dt)
        a = bufs.get(name)
        if a is None or len(a) != n:
            a = bufs[name] = np.zeros(n, dt)
        return a
    spot = buf("spot", max(n_nodes, 1), np.int32)
    od = buf("od", max(n_nodes, 1), np.int32)
    ns, nod = buf("ns", 1, np.int32), buf("nod", 1, np.int32)
    off = buf("off", n_nodes + 1, np.int32)
    idx = buf("idx", max(n_pods, 1), np.int32)
    req = buf("req", max(n_nodes, 1), np.int64)
    free = buf("free", max(n_nodes, 1), np.int64)
    m = capi.sr_node_map(capi.ptr(spot, capi.P32), capi.ptr(ns, capi.P32), capi.ptr(od, capi.P32),
                         capi.ptr(nod, capi.P32), capi.ptr(off, capi.P32), capi.ptr(idx, capi.P32),
                         capi.ptr(req, capi.P64), capi.ptr(free, capi.P64))
    params = capi.sr_node_map_params(od_label, spot_label, priority_threshold)
    st = fn(cluster_ptr, ctypes.byref(params), ctypes.byref(m))
    if st != capi.SR_OK:
        raise RuntimeError("new_node_map status %d" % st)
    if bufs is not None:
        return NodeMapArrays(spot[: ns[0]], od[: nod[0]], off, idx[: int(off[-1])], req, free)
    return NodeMapArrays(spot[: ns[0]].copy(), od[: nod[0]].copy(), off, idx[: int(off[-1])], req, free)


def pods_for_deletion(fn, cluster_ptr, drain_ptr, nodes: np.ndarray, node_pod_off: np.ndarray,
                      node_pod_idx: np.ndarray, delete_non_replicated: bool = False, owner_filter: bool = True,
                      bufs: Optional[dict] = None):
    """sr_pods_for_deletion-shaped `fn` (the product's, or the oracle's in tests)
    over `nodes`: (cand_off, cand_pods, block_pod, block_reason, status).
    `bufs`: output arrays kept across calls (sized for every listed pod)."""
    nodes = np.ascontiguousarray(nodes, np.int32)
    n = len(nodes)
    npo = np.asarray(node_pod_off)
    if bufs is None:
        off = np.zeros(n + 1, np.int32)
        total = int(np.sum(npo[nodes + 1] - npo[nodes])) if n else 0
        pods = np.zeros(max(1, total), np.int32)
        bp = np.full(max(1, n), -1, np.int32)
        br = np.zeros(max(1, n), np.int32)
    else:  # the kept arrays: room for every pod of the node map (a list never holds more)
        def buf(name, k):
            a = bufs.get(name)
            if a is None or len(a) < k:
                a = bufs[name] = np.zeros(k, np.int32)
            return a
        off = buf("off", n + 1)[: n + 1]
        pods = buf("pods", max(1, int(npo[-1])))
        bp = buf("bp", max(1, n))[: max(1, n)]
        br = buf("br", max(1, n))[: max(1, n)]
    prm = capi.sr_drain_params(1 if delete_non_replicated else 0, 0,  # rescheduler.go:231 arguments 3, 4
                               1 if owner_filter else 0)
    st = fn(cluster_ptr, drain_ptr, ctypes.byref(prm), capi.ptr(nodes, capi.P32), n,
            capi.ptr(np.ascontiguousarray(node_pod_off, np.int32), capi.P32),
            capi.ptr(np.ascontiguousarray(node_pod_idx, np.int32), capi.P32), capi.ptr(off, capi.P32),
            capi.ptr(pods, capi.P32), capi.ptr(bp, capi.P32), capi.ptr(br, capi.P32))
    if bufs is not None:
        return off, pods[: int(off[-1])], bp[:n], br[:n], st
    return off, pods[: int(off[-1])].copy(), bp[:n], br[:n], st


def build_candidates(nm: NodeMapArrays, flags: np.ndarray):
    """podsForDeletion per on-demand node in NodeInfoArray order: NodeInfo.Pods
    minus mirror and DaemonSet-controlled pods (rescheduler.go:231-256)."""
    off = [0]
    pods = []
    drop = capi.SR_POD_MIRROR | capi.SR_POD_DAEMONSET_CONTROLLER
    for node in nm.on_demand:
        ps = nm.node_pod_idx[nm.node_pod_off[node]:nm.node_pod_off[node + 1]]
        keep = ps[(flags[ps] & drop) == 0]
        pods.append(keep)
        off.append(off[-1] + len(keep))
    cand_pods = np.concatenate(pods).astype(np.int32) if pods else np.zeros(0, np.int32)
    return np.asarray(off, np.int32), np.ascontiguousarray(cand_pods)


@dataclass
class Tick:
    synth: SynthCluster
    node_map: NodeMapArrays
    snapshot: object           # sr_snapshot* handle (product)
    cand_off: np.ndarray
    cand_pods: np.ndarray


def shard(cand_off: np.ndarray, cand_pods: np.ndarray, rank: int, world: int):
    """Candidates c with c % world == rank (interleaved, so every rank holds early candidates)."""
    n = len(cand_off) - 1
    idx = np.arange(rank, max(n, 0), world, dtype=np.int32)
    cand_off = np.asarray(cand_off)
    if world == 1:
        return np.ascontiguousarray(cand_off, np.int32), np.ascontiguousarray(cand_pods, np.int32), idx
    lens = (cand_off[idx + 1] - cand_off[idx]).astype(np.int64)
    off = np.zeros(len(idx) + 1, np.int64)
    np.cumsum(lens, out=off[1:])
    # positions of the kept candidates' pods: each range shifted to its new start
    pos = np.repeat(cand_off[idx].astype(np.int64) - off[:-1], lens) + np.arange(off[-1], dtype=np.int64)
    return off.astype(np.int32), np.ascontiguousarray(np.asarray(cand_pods)[pos], np.int32), idx
