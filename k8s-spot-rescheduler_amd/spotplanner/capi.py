"""ctypes view of include/sr_planner.h (constants, structs) and library loading.

The constants are parsed from the header itself so the Python side cannot drift
from the C-ABI.  `load_planner()` loads the in-tree libsrplanner.so and fails
loudly if it is missing: there is no CPU fallback for the planner.
"""
from __future__ import annotations

import ctypes
import os
import re

_PKG = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_PKG)                       # k8s-spot-rescheduler_amd/
REPO_ROOT = os.path.dirname(PKG_ROOT)
HEADER = os.path.join(REPO_ROOT, "include", "sr_planner.h")
LIB_DIR = os.path.join(PKG_ROOT, "lib")
PLANNER_LIB = os.path.join(LIB_DIR, "libsrplanner.so")
SYNTH_LIB = os.path.join(LIB_DIR, "libsrsynth.so")


def _parse_defines(path):
    """Integer #defines: decimal or hex literals, optionally `(x << n)` and a `u` suffix."""
    out = {}
    with open(path) as f:
        for line in f:
            m = re.match(r"#define\s+(SR_\w+)\s+\(?\s*(-?0x[0-9a-fA-F]+|-?\d+)u?\s*(?:<<\s*(\d+))?\s*\)?(\s|$)",
                         line)
            if m:
                v = int(m.group(2), 0)
                if m.group(3):
                    v <<= int(m.group(3))
                out[m.group(1)] = v
    return out


_DEF = _parse_defines(HEADER)
globals().update(_DEF)

P32 = ctypes.POINTER(ctypes.c_int32)
P64 = ctypes.POINTER(ctypes.c_int64)
PU8 = ctypes.POINTER(ctypes.c_uint8)
PU32 = ctypes.POINTER(ctypes.c_uint32)


class sr_nodes(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("name", P32), ("alloc_milli_cpu", P64), ("alloc_memory", P64),
                ("alloc_ephemeral", P64), ("alloc_pods", P64), ("unschedulable", PU8),
                ("label_off", P32), ("label_key", P32), ("label_val", P32),
                ("taint_off", P32), ("taint_key", P32), ("taint_val", P32), ("taint_effect", P32)]


class sr_pods(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("node", P32), ("cpu_sort_milli", P64), ("req_milli_cpu", P64),
                ("req_memory", P64), ("req_ephemeral", P64), ("priority", P32), ("has_priority", PU8),
                ("flags", PU32), ("sel_off", P32), ("sel_key", P32), ("sel_val", P32),
                ("aff_required", PU8), ("term_off", P32), ("term_expr_off", P32), ("term_field_off", P32),
                ("expr_key", P32), ("expr_op", P32), ("expr_val_off", P32), ("expr_vals", P32),
                ("field_key", P32), ("field_op", P32), ("field_val_off", P32), ("field_vals", P32),
                ("tol_off", P32), ("tol_key", P32), ("tol_op", P32), ("tol_val", P32), ("tol_effect", P32),
                ("port_off", P32), ("port_proto", P32), ("port_num", P32), ("port_ip", P32)]


class sr_pod_affinity(ctypes.Structure):
    _fields_ = [("ns", P32), ("label_off", P32), ("label_key", P32), ("label_val", P32), ("anti_off", P32),
                ("topology_key", P32), ("ns_off", P32), ("ns_ids", P32), ("selector_nil", PU8),
                ("ml_off", P32), ("ml_key", P32), ("ml_val", P32), ("me_off", P32), ("me_key", P32),
                ("me_op", P32), ("me_val_off", P32), ("me_vals", P32), ("aff_off", P32)]


class sr_spread(ctypes.Structure):
    _fields_ = [("off", P32), ("max_skew", P32), ("topology_key", P32), ("selector_nil", PU8),
                ("ml_off", P32), ("ml_key", P32), ("ml_val", P32), ("me_off", P32), ("me_key", P32),
                ("me_op", P32), ("me_val_off", P32), ("me_vals", P32), ("terminating", PU8)]


class sr_volumes(ctypes.Structure):
    _fields_ = [("prefilter_fail", PU8), ("disk_off", P32), ("disk_kind", P32), ("disk_id", P32), ("disk_ro", PU8),
                ("att_off", P32), ("att_key", P32), ("att_id", P32), ("att_noncsi", PU8),
                ("limit_off", P32), ("limit_key", P32), ("limit", P64),
                ("zone_off", P32), ("zone_key", P32), ("zone_val_off", P32), ("zone_vals", P32),
                ("zone_keys", ctypes.c_int32 * 4),
                ("pv_off", P32), ("pv_term_off", P32), ("term_expr_off", P32), ("term_field_off", P32),
                ("expr_key", P32), ("expr_op", P32), ("expr_val_off", P32), ("expr_vals", P32),
                ("field_key", P32), ("field_op", P32), ("field_val_off", P32), ("field_vals", P32)]


class sr_cluster(ctypes.Structure):
    _fields_ = [("nodes", sr_nodes), ("pods", sr_pods), ("id_empty", ctypes.c_int32),
                ("id_metadata_name", ctypes.c_int32), ("id_unschedulable_key", ctypes.c_int32),
                ("pod_affinity", ctypes.POINTER(sr_pod_affinity)), ("n_strings", ctypes.c_int32),
                ("str_int", ctypes.POINTER(ctypes.c_int64)), ("str_int_ok", ctypes.POINTER(ctypes.c_uint8)),
                ("str_label", ctypes.POINTER(ctypes.c_uint8)),
                ("pod_scalar_off", P32), ("pod_scalar_name", P32), ("pod_scalar_req", P64), ("pod_scalar_acc", P64),
                ("node_scalar_off", P32), ("node_scalar_name", P32), ("node_scalar_alloc", P64),
                ("acc_milli_cpu", P64), ("acc_memory", P64), ("acc_ephemeral", P64),
                ("spread", ctypes.POINTER(sr_spread)), ("volumes", ctypes.POINTER(sr_volumes)),
                ("pod_stamp", ctypes.POINTER(ctypes.c_uint64))]


class sr_node_label(ctypes.Structure):
    _fields_ = [("key", ctypes.c_int32), ("value", ctypes.c_int32), ("has_value", ctypes.c_int32)]


class sr_node_map_params(ctypes.Structure):
    _fields_ = [("on_demand", sr_node_label), ("spot", sr_node_label), ("priority_threshold", ctypes.c_int32)]


class sr_node_map(ctypes.Structure):
    _fields_ = [("spot", P32), ("n_spot", P32), ("on_demand", P32), ("n_on_demand", P32),
                ("node_pod_off", P32), ("node_pod_idx", P32), ("requested_cpu", P64), ("free_cpu", P64)]


class sr_pod_drain(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("flags", PU32), ("phase", PU8), ("restart_policy", PU8),
                ("deletion_age_ns", P64), ("grace_seconds", P64)]


class sr_drain_params(ctypes.Structure):
    _fields_ = [("skip_nodes_with_system_pods", ctypes.c_int32), ("skip_nodes_with_local_storage", ctypes.c_int32),
                ("owner_filter", ctypes.c_int32)]


class sr_candidates(ctypes.Structure):
    _fields_ = [("n_cand", ctypes.c_int32), ("cand_pod_off", P32), ("cand_pods", P32), ("cand_global", P32)]


class sr_plan_out(ctypes.Structure):
    _fields_ = [("winner", ctypes.c_int32), ("first_ok", ctypes.c_int32), ("first_fallback", ctypes.c_int32),
                ("winner_npods", ctypes.c_int32), ("checks", ctypes.c_uint64), ("fallback_pods", ctypes.c_uint64),
                ("status", P32), ("node_of_pod", P32), ("winner_map", P32), ("checks_dense", ctypes.c_uint64)]


# sr_allreduce_min_fn: int32 fn(void *user, uint64_t *words, int32_t n)
ALLREDUCE_MIN_FN = ctypes.CFUNCTYPE(ctypes.c_int32, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int32)


class sr_timing(ctypes.Structure):
    _fields_ = [("n_runs", ctypes.c_int32), ("ms_tables", ctypes.c_double),
                ("ms_placement", ctypes.c_double), ("ms_winner", ctypes.c_double),
                ("ms_pack_host", ctypes.c_double), ("ms_upload", ctypes.c_double),
                ("bytes_tables", ctypes.c_uint64), ("bytes_placement", ctypes.c_uint64),
                ("n_pods", ctypes.c_int32), ("n_spot", ctypes.c_int32), ("n_cand", ctypes.c_int32),
                ("n_words", ctypes.c_int32), ("n_rows_static", ctypes.c_int32), ("n_rows_threshold", ctypes.c_int32),
                ("n_classes", ctypes.c_int32), ("bytes_uploaded", ctypes.c_uint64), ("enc_new_specs", ctypes.c_int32),
                ("enc_static_rebuilt", ctypes.c_int32), ("enc_state_nodes", ctypes.c_int32),
                ("prefix_batches", ctypes.c_int32), ("enc_memo_pods", ctypes.c_int32),
                ("enc_reused", ctypes.c_int32), ("enc_pod_patches", ctypes.c_int32),
                ("k0_columns", ctypes.c_int32), ("k0_rows_moved", ctypes.c_int32), ("k0_dirty_nodes", ctypes.c_int32),
                ("ms_collective", ctypes.c_double), ("k2_launches", ctypes.c_int32),
                ("k2_list_by_cost", ctypes.c_int32), ("k2_coop", ctypes.c_int32)]


def ptr(arr, typ):
    """Pointer to a contiguous numpy array (None for an empty array is fine)."""
    if arr is None:
        return ctypes.cast(None, typ)
    return arr.ctypes.data_as(typ)


def make_cluster_struct(A) -> sr_cluster:
    c = sr_cluster()
    n = c.nodes
    n.n = A["n_nodes"]
    n.name = ptr(A["node_name"], P32)
    n.alloc_milli_cpu = ptr(A["alloc_cpu"], P64)
    n.alloc_memory = ptr(A["alloc_mem"], P64)
    n.alloc_ephemeral = ptr(A["alloc_eph"], P64)
    n.alloc_pods = ptr(A["alloc_pods"], P64)
    n.unschedulable = ptr(A["unsched"], PU8)
    n.label_off = ptr(A["label_off"], P32)
    n.label_key = ptr(A["label_key"], P32)
    n.label_val = ptr(A["label_val"], P32)
    n.taint_off = ptr(A["taint_off"], P32)
    n.taint_key = ptr(A["taint_key"], P32)
    n.taint_val = ptr(A["taint_val"], P32)
    n.taint_effect = ptr(A["taint_eff"], P32)
    p = c.pods
    p.n = A["n_pods"]
    p.node = ptr(A["pod_node"], P32)
    p.cpu_sort_milli = ptr(A["cpu_sort"], P64)
    p.req_milli_cpu = ptr(A["req_cpu"], P64)
    p.req_memory = ptr(A["req_mem"], P64)
    p.req_ephemeral = ptr(A["req_eph"], P64)
    p.priority = ptr(A["priority"], P32)
    p.has_priority = ptr(A["has_priority"], PU8)
    p.flags = ptr(A["flags"], PU32)
    for f in ("sel_off", "sel_key", "sel_val", "term_off", "term_expr_off", "term_field_off", "expr_key",
              "expr_op", "expr_val_off", "expr_vals", "field_key", "field_op", "field_val_off", "field_vals",
              "tol_off", "tol_key", "tol_op", "tol_val", "port_off", "port_proto", "port_num", "port_ip"):
        setattr(p, f, ptr(A[f], P32))
    p.tol_effect = ptr(A["tol_eff"], P32)
    p.aff_required = ptr(A["aff_required"], PU8)
    c.id_empty = A["id_empty"]
    c.id_metadata_name = A["id_metadata_name"]
    c.id_unschedulable_key = A["id_unschedulable_key"]
    if A.get("str_int") is not None:
        c.n_strings = len(A["str_int"])
        c.str_int = ptr(A["str_int"], P64)
        c.str_int_ok = ptr(A["str_int_ok"], PU8)
    if A.get("str_label") is not None:
        c.n_strings = len(A["str_label"])
        c.str_label = ptr(A["str_label"], PU8)
    if A.get("pod_scalar_off") is not None:
        c.pod_scalar_off = ptr(A["pod_scalar_off"], P32)
        c.pod_scalar_name = ptr(A["pod_scalar_name"], P32)
        c.pod_scalar_req = ptr(A["pod_scalar_req"], P64)
        c.pod_scalar_acc = ptr(A["pod_scalar_acc"], P64)
        c.node_scalar_off = ptr(A["node_scalar_off"], P32)
        c.node_scalar_name = ptr(A["node_scalar_name"], P32)
        c.node_scalar_alloc = ptr(A["node_scalar_alloc"], P64)
    if A.get("acc_cpu") is not None:
        c.acc_milli_cpu = ptr(A["acc_cpu"], P64)
        c.acc_memory = ptr(A["acc_mem"], P64)
        c.acc_ephemeral = ptr(A["acc_eph"], P64)
    if A.get("ts_off") is not None:
        ts = sr_spread()
        for f in ("off", "max_skew", "topology_key", "ml_off", "ml_key", "ml_val", "me_off", "me_key", "me_op",
                  "me_val_off", "me_vals"):
            setattr(ts, f, ptr(A["ts_" + f], P32))
        ts.selector_nil = ptr(A["ts_selector_nil"], PU8)
        ts.terminating = ptr(A["ts_terminating"], PU8)
        c._spread = ts  # keeps the struct alive as long as the cluster struct
        c.spread = ctypes.pointer(ts)
    if A.get("vol_prefilter_fail") is not None:
        v = sr_volumes()
        v.prefilter_fail = ptr(A["vol_prefilter_fail"], PU8)
        for f in ("disk_off", "disk_kind", "disk_id", "att_off", "att_key", "att_id", "limit_off", "limit_key",
                  "zone_off", "zone_key", "zone_val_off", "zone_vals", "pv_off", "pv_term_off", "term_expr_off",
                  "term_field_off", "expr_key", "expr_op", "expr_val_off", "expr_vals", "field_key", "field_op",
                  "field_val_off", "field_vals"):
            setattr(v, f, ptr(A["vol_" + f], P32))
        v.disk_ro = ptr(A["vol_disk_ro"], PU8)
        v.att_noncsi = ptr(A["vol_att_noncsi"], PU8)
        v.limit = ptr(A["vol_limit"], P64)
        for i in range(4):
            v.zone_keys[i] = int(A["vol_zone_keys"][i])
        c._volumes = v  # keeps the struct alive as long as the cluster struct
        c.volumes = ctypes.pointer(v)
    if A.get("pod_stamp") is not None:
        c.pod_stamp = ptr(A["pod_stamp"], ctypes.POINTER(ctypes.c_uint64))
    if A.get("pa_ns") is not None:
        pa = sr_pod_affinity()
        for f in ("ns", "label_off", "label_key", "label_val", "anti_off", "topology_key", "ns_off", "ns_ids",
                  "ml_off", "ml_key", "ml_val", "me_off", "me_key", "me_op", "me_val_off", "me_vals", "aff_off"):
            setattr(pa, f, ptr(A["pa_" + f], P32))
        pa.selector_nil = ptr(A["pa_selector_nil"], PU8)
        c._pod_affinity = pa  # keeps the struct alive as long as the cluster struct
        c.pod_affinity = ctypes.pointer(pa)
    return c


_planner = None


class PlannerLibraryMissing(RuntimeError):
    pass


def load_planner():
    """Load the in-tree HIP planner library; never substitutes anything for it."""
    global _planner
    if _planner is not None:
        return _planner
    path = PLANNER_LIB
    alt = os.environ.get("SR_PLANNER_LIB")  # same-box A/B of two builds (tools/gpu_ab.sh): an in-tree variant
    if alt:
        path = os.path.join(os.path.dirname(PLANNER_LIB), os.path.basename(alt))
    if not os.path.exists(path):
        raise PlannerLibraryMissing(
            "%s is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
            "(the planner has no CPU fallback)" % path)
    lib = ctypes.CDLL(path)
    _declare_planner(lib)
    check_abi(lib, path)
    _planner = lib
    return lib


class PlannerAbiMismatch(RuntimeError):
    pass


def check_abi(lib, path="libsrplanner.so"):
    """The shim contract: before the first planner call, the
    library's SR_ABI_VERSION must equal the header's this binding was built
    from -- sr_cluster grows at its end between versions, and a library fed a
    shorter struct would read past it."""
    have = int(lib.sr_abi_version())
    if have != SR_ABI_VERSION:  # noqa: F821 (parsed from the header)
        raise PlannerAbiMismatch("%s has SR_ABI_VERSION %d, this binding was built against %d"
                                 % (path, have, SR_ABI_VERSION))  # noqa: F821


def _declare_planner(lib):
    S = ctypes.c_int32
    VP = ctypes.c_void_p
    PC = ctypes.POINTER(sr_cluster)
    lib.sr_new_node_map.argtypes = [PC, ctypes.POINTER(sr_node_map_params), ctypes.POINTER(sr_node_map)]
    lib.sr_new_node_map.restype = S
    lib.sr_node_map_cache_create.argtypes = [ctypes.POINTER(VP)]
    lib.sr_node_map_cache_create.restype = S
    lib.sr_node_map_cache_destroy.argtypes = [VP]
    lib.sr_node_map_cache_destroy.restype = None
    lib.sr_new_node_map_cached.argtypes = [VP, PC, ctypes.POINTER(sr_node_map_params), ctypes.POINTER(sr_node_map),
                                           P32]
    lib.sr_new_node_map_cached.restype = S
    lib.sr_node_has_label.argtypes = [PC, ctypes.c_int32, ctypes.POINTER(sr_node_label)]
    lib.sr_node_has_label.restype = ctypes.c_int32
    lib.sr_pods_for_deletion.argtypes = [PC, ctypes.POINTER(sr_pod_drain), ctypes.POINTER(sr_drain_params), P32,
                                         ctypes.c_int32, P32, P32, P32, P32, P32, P32]
    lib.sr_pods_for_deletion.restype = S
    lib.sr_snapshot_create.argtypes = [PC, P32, ctypes.c_int32, P32, P32, ctypes.POINTER(VP)]
    lib.sr_snapshot_create.restype = S
    lib.sr_snapshot_refresh.argtypes = [VP, PC, P32, ctypes.c_int32, P32, P32, P32]
    lib.sr_snapshot_refresh.restype = S
    lib.sr_snapshot_refresh_cached.argtypes = [VP, VP, PC, P32, ctypes.c_int32, P32, P32, P32]
    lib.sr_snapshot_refresh_cached.restype = S
    lib.sr_snapshot_destroy.argtypes = [VP]
    lib.sr_snapshot_destroy.restype = None
    lib.sr_snapshot_add_pod.argtypes = [VP, PC, ctypes.c_int32, ctypes.c_int32]
    lib.sr_snapshot_add_pod.restype = S
    lib.sr_snapshot_fork.argtypes = [VP]
    lib.sr_snapshot_fork.restype = S
    lib.sr_snapshot_revert.argtypes = [VP]
    lib.sr_snapshot_revert.restype = S
    lib.sr_snapshot_node_state.argtypes = [VP, ctypes.c_int32, P64, P32]
    lib.sr_snapshot_node_state.restype = S
    lib.sr_snapshot_num_nodes.argtypes = [VP]
    lib.sr_snapshot_num_nodes.restype = ctypes.c_int32
    lib.sr_create.argtypes = [ctypes.c_int32, ctypes.POINTER(VP)]
    lib.sr_create.restype = S
    lib.sr_destroy.argtypes = [VP]
    lib.sr_destroy.restype = None
    lib.sr_last_error.argtypes = [VP]
    lib.sr_last_error.restype = ctypes.c_char_p
    lib.sr_build_info.argtypes = []
    lib.sr_build_info.restype = ctypes.c_char_p
    lib.sr_abi_version.argtypes = []
    lib.sr_abi_version.restype = ctypes.c_int32
    lib.sr_find_spot_nodes.argtypes = [VP, VP, PC, P32, ctypes.c_int32, P32, PU8]
    lib.sr_find_spot_nodes.restype = S
    lib.sr_can_drain_node.argtypes = [VP, VP, PC, P32, ctypes.c_int32, P32, P32, PU8]
    lib.sr_can_drain_node.restype = S
    lib.sr_plan.argtypes = [VP, VP, PC, ctypes.POINTER(sr_candidates), ctypes.POINTER(sr_plan_out)]
    lib.sr_plan.restype = S
    lib.sr_plan_first.argtypes = [VP, VP, PC, ctypes.POINTER(sr_candidates), ctypes.POINTER(sr_plan_out)]
    lib.sr_plan_first.restype = S
    lib.sr_plan_prepare.argtypes = [VP, VP, PC, ctypes.POINTER(sr_candidates)]
    lib.sr_plan_prepare.restype = S
    lib.sr_plan_run.argtypes = [VP, ctypes.POINTER(sr_plan_out)]
    lib.sr_plan_run.restype = S
    lib.sr_set_timing.argtypes = [VP, ctypes.c_int32]
    lib.sr_set_timing.restype = S
    lib.sr_get_timing.argtypes = [VP, ctypes.POINTER(sr_timing)]
    lib.sr_get_timing.restype = S
    lib.sr_comm_unique_id.argtypes = [ctypes.POINTER(ctypes.c_uint8)]
    lib.sr_comm_unique_id.restype = S
    lib.sr_comm_init.argtypes = [VP, ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32, ctypes.c_int32]
    lib.sr_comm_init.restype = S
    lib.sr_comm_init_host.argtypes = [VP, ctypes.c_int32, ctypes.c_int32, ALLREDUCE_MIN_FN, VP]
    lib.sr_comm_init_host.restype = S
    lib.sr_comm_init_shm.argtypes = [VP, ctypes.c_char_p, ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32]
    lib.sr_comm_init_shm.restype = S


# Every symbol include/sr_planner.h declares (checked by tests on CPU).
EXPORTED = ["sr_new_node_map", "sr_node_map_cache_create", "sr_node_map_cache_destroy", "sr_new_node_map_cached",
            "sr_node_has_label", "sr_pods_for_deletion", "sr_snapshot_create", "sr_snapshot_refresh", "sr_snapshot_refresh_cached",
            "sr_snapshot_destroy",
            "sr_snapshot_add_pod", "sr_snapshot_fork", "sr_snapshot_revert", "sr_snapshot_node_state",
            "sr_snapshot_num_nodes", "sr_create", "sr_destroy", "sr_last_error", "sr_build_info",
            "sr_abi_version", "sr_find_spot_nodes", "sr_can_drain_node", "sr_plan", "sr_plan_first", "sr_plan_prepare", "sr_plan_run",
            "sr_set_timing", "sr_get_timing", "sr_comm_unique_id", "sr_comm_init", "sr_comm_init_host",
            "sr_comm_init_shm"]
