"""ctypes binding of the CPU oracle (oracle/build/libsroracle.so).

Test infrastructure only: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker.  The product never imports this.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

from spotplanner import capi

REPO = capi.REPO_ROOT
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "build", "libsroracle.so")
NOT_EVALUATED = -4

_lib = None


def load_oracle():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(ORACLE_LIB):
        subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
    lib = ctypes.CDLL(ORACLE_LIB)
    VP = ctypes.c_void_p
    PC = ctypes.POINTER(capi.sr_cluster)
    P32, P64 = capi.P32, capi.P64
    lib.oracle_go_sort_by_key.argtypes = [P32, ctypes.c_int32, P64, ctypes.c_int32]
    lib.oracle_node_has_label.argtypes = [PC, ctypes.c_int32, ctypes.POINTER(capi.sr_node_label)]
    lib.oracle_node_has_label.restype = ctypes.c_int32
    lib.oracle_validate_label_flag.argtypes = [ctypes.c_int32]
    lib.oracle_validate_label_flag.restype = ctypes.c_int32
    lib.oracle_new_node_map.argtypes = [PC, ctypes.POINTER(capi.sr_node_map_params), ctypes.POINTER(capi.sr_node_map)]
    lib.oracle_new_node_map.restype = ctypes.c_int32
    lib.oracle_pods_for_deletion.argtypes = [PC, ctypes.POINTER(capi.sr_pod_drain), ctypes.POINTER(capi.sr_drain_params),
                                             P32, ctypes.c_int32, P32, P32, P32, P32, P32, P32]
    lib.oracle_pods_for_deletion.restype = ctypes.c_int32
    lib.oracle_snapshot_create.argtypes = [PC, P32, ctypes.c_int32, P32, P32]
    lib.oracle_snapshot_create.restype = VP
    lib.oracle_snapshot_destroy.argtypes = [VP]
    lib.oracle_snapshot_add_pod.argtypes = [VP, PC, ctypes.c_int32, ctypes.c_int32]
    lib.oracle_snapshot_fork.argtypes = [VP]
    lib.oracle_snapshot_fork.restype = ctypes.c_int32
    lib.oracle_snapshot_revert.argtypes = [VP]
    lib.oracle_snapshot_revert.restype = ctypes.c_int32
    lib.oracle_snapshot_node_state.argtypes = [VP, ctypes.c_int32, P64, P32]
    lib.oracle_check_predicates.argtypes = [VP, PC, ctypes.c_int32, ctypes.c_int32]
    lib.oracle_check_predicates.restype = ctypes.c_int32
    lib.oracle_pod_needs_fallback.argtypes = [VP, PC, ctypes.c_int32]
    lib.oracle_pod_needs_fallback.restype = ctypes.c_int32
    lib.oracle_find_spot_node_for_pod.argtypes = [VP, PC, ctypes.c_int32]
    lib.oracle_find_spot_node_for_pod.restype = ctypes.c_int32
    lib.oracle_can_drain_node.argtypes = [VP, PC, P32, ctypes.c_int32, P32]
    lib.oracle_can_drain_node.restype = ctypes.c_int32
    lib.oracle_plan.argtypes = [VP, PC, ctypes.POINTER(capi.sr_candidates), ctypes.c_int32, ctypes.c_int32,
                                ctypes.POINTER(capi.sr_plan_out)]
    lib.oracle_plan.restype = ctypes.c_int32
    _lib = lib
    return lib


class OracleSnapshot:
    def __init__(self, cluster_ptr, spot, node_pod_off, node_pod_idx):
        self.lib = load_oracle()
        self.spot = np.ascontiguousarray(spot, np.int32)
        self.h = self.lib.oracle_snapshot_create(cluster_ptr, capi.ptr(self.spot, capi.P32), len(self.spot),
                                                 capi.ptr(np.ascontiguousarray(node_pod_off, np.int32), capi.P32),
                                                 capi.ptr(np.ascontiguousarray(node_pod_idx, np.int32), capi.P32))

    def close(self):
        if self.h:
            self.lib.oracle_snapshot_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def node_state(self, pos):
        req = np.zeros(3, np.int64)
        n = ctypes.c_int32()
        self.lib.oracle_snapshot_node_state(self.h, pos, capi.ptr(req, capi.P64), ctypes.byref(n))
        return tuple(int(x) for x in req), int(n.value)


def oracle_plan(snap: OracleSnapshot, cluster_ptr, cand_off, cand_pods, mode=1, threads=1, cand_global=None):
    lib = load_oracle()
    cand_off = np.ascontiguousarray(cand_off, np.int32)
    cand_pods = np.ascontiguousarray(cand_pods, np.int32)
    n = len(cand_off) - 1
    c = capi.sr_candidates(n, capi.ptr(cand_off, capi.P32), capi.ptr(cand_pods, capi.P32),
                           capi.ptr(cand_global, capi.P32) if cand_global is not None else None)
    maxp = int(np.max(np.diff(cand_off))) if n > 0 else 0
    status = np.zeros(max(n, 1), np.int32)
    nodes = np.zeros(max(int(cand_off[-1]) if n else 0, 1), np.int32)
    wmap = np.full(max(maxp, 1), -1, np.int32)
    o = capi.sr_plan_out()
    o.status = capi.ptr(status, capi.P32)
    o.node_of_pod = capi.ptr(nodes, capi.P32)
    o.winner_map = capi.ptr(wmap, capi.P32)
    lib.oracle_plan(snap.h, cluster_ptr, ctypes.byref(c), mode, threads, ctypes.byref(o))
    return dict(winner=o.winner, first_ok=o.first_ok, first_fallback=o.first_fallback, status=status[:n],
                node_of_pod=nodes[: int(cand_off[-1]) if n else 0], winner_map=wmap[: o.winner_npods],
                checks=int(o.checks), fallback_pods=int(o.fallback_pods))


def oracle_new_node_map(cluster_ptr, n_nodes, n_pods, od_label, spot_label, thr=0):
    from spotplanner.synth import new_node_map
    return new_node_map(load_oracle().oracle_new_node_map, cluster_ptr, n_nodes, n_pods, od_label, spot_label, thr)
