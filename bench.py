#!/usr/bin/env python3
"""Drain-planner benchmark (BASELINE.json metric: drain-plan latency (ms) +
pod x node feasibility checks/s at 5k nodes / 150k pods).

One step = one housekeeping tick's planning segment on device-resident inputs:
K0 tables -> K2 feasibility rows + first-fit placement of every candidate
(each candidate's outcome and the first drainable mapping go straight to
mapped host memory; for N>1 into one shared-memory segment every rank's host
walks in global candidate order, or, with --transport rccl, an RCCL
allreduce(min) -> K3 winner mapping).
ms_per_step is the back-to-back tick with inputs in HBM (latency_ms: one tick
on an idle device, launch to the winner on the host); `value` is
reference-equivalent (pod, spot node) predicate checks per second over all
ranks: the CheckPredicates calls (rescheduler.go:344) the reference's loop
makes to reach the same plan of every candidate (findSpotNodeForPod stops at
the first fit).  The dense-equivalent rate (every candidate pod x every spot
node) is reported beside it, labelled as such.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 3]

N > 1 runs one process per GPU: under torch.distributed.run (RANK /
WORLD_SIZE / LOCAL_RANK / MASTER_* from the environment), or, when
WORLD_SIZE is not set, as N child processes this one starts and waits for
(it touches no GPU itself and exits non-zero if fewer than N devices are
visible or any rank fails).  Candidates are sharded c % N == rank: with
--scaling strong (the default, BASELINE's line) the config's own cluster is
split over the ranks, with --scaling weak the cluster has N x the config's
on-demand nodes over the same spot pool (every GPU holds one config-sized
candidate set); a strong line carries the weak-scaled measurement beside it
(weak_scaling).  The ranks reduce each tick's outcome through shared memory
(--transport shm, no collective) or one RCCL allreduce(min) (--transport rccl).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "k8s-spot-rescheduler_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from spotplanner import capi  # noqa: E402
from spotplanner.planner import PredicateChecker  # noqa: E402
from spotplanner.scaling import choose_scaling, predict  # noqa: E402
from spotplanner.synth import AFFINITY, REALISTIC, SynthCluster, new_node_map, pods_for_deletion, shard  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
DEFAULT_OD = {1: 10, 2: 300, 3: 1500, 4: 15000, 5: 300}
WORKLOAD_KIND = {1: "rescheduler_test-style, cpu/mem requests only",
                 2: "resource fit + PreferNoSchedule taints",
                 3: "nodeSelector + node affinity + tolerations",
                 4: "nodeSelector + node affinity + tolerations, all candidates per tick",
                 5: "host-port + DaemonSet heavy"}


def workload_name(config, n_nodes, n_od, n_spot, n_pods, world, scaling, variant="baseline"):
    """config.workload: the cluster this run actually planned (node, on-demand,
    spot and pod counts), and how its candidates were split over the ranks."""
    s = "C%d %d nodes (%d od / %d spot) / %d pods, %s" % (config, n_nodes, n_od, n_spot, n_pods,
                                                          WORKLOAD_KIND[config])
    if variant == "realistic":
        s += ("; realistic variant: %d%% StatefulSet pods with a zonal EBS CSI claim (CSINode limit 25), "
              "%d%% with an init container, %d%% of GPU-node pods asking for a GPU"
              % tuple(round(100 * REALISTIC[k]) for k in ("stateful_fraction", "init_fraction", "gpu_fraction")))
    elif variant == "affinity":
        s += ("; affinity variant: every pod in a Deployment (~5 replicas, 16 namespaces), %d%% of the Deployments "
              "with required hostname pod anti-affinity, %d%% with a zone DoNotSchedule topology spread constraint "
              "(maxSkew 1), their spot replicas included"
              % tuple(round(100 * AFFINITY[k]) for k in ("anti_fraction", "spread_fraction")))
    if world > 1:
        s += "; %s scaling: %d candidates sharded c %% %d" % (scaling, n_od, world)
    return s


def cluster_on_demand(config, world, scaling):
    """On-demand node count of the synthetic cluster: the config's own (strong
    scaling: a fixed cluster split over the ranks) or world x it (weak: each
    rank holds one config-sized candidate set over the same spot pool)."""
    return DEFAULT_OD[config] * (world if scaling == "weak" else 1)


def shard_sizes(n_cand, world):
    """Candidates per rank under the c % world split (shard())."""
    return [len(range(r, n_cand, world)) for r in range(world)]


E2E_IDLE = os.environ.get("SR_BENCH_E2E_IDLE", "1") != "0"


def latest_profile(name):
    """profiles/rNN/final/<name> or profiles/rNN/<name> of the newest round that has it, or None."""
    base = os.path.join(REPO, "profiles")
    rounds = sorted((d for d in os.listdir(base) if d.startswith("r") and d[1:].isdigit()), reverse=True) \
        if os.path.isdir(base) else []
    for d in rounds:
        for p in (os.path.join(base, d, "final", name), os.path.join(base, d, name)):
            if os.path.exists(p):
                return p
    return None


def k2_chain_summary(path):
    """K2's chain costs from the committed per-wave profile of this config
    (tools/k2_profile.py output, SR_K2_PROFILE run of the same build), or None."""
    if path is None or not os.path.exists(path):
        return None
    out = {"source": os.path.relpath(path, REPO)}
    lines = open(path).read().splitlines()
    for i, line in enumerate(lines):  # the longest node-order wave (older profiles: the latest-ending one)
        if line.startswith("longest waves") or (line.startswith("latest-ending waves") and "longest_wave" not in out):
            for row in lines[i + 1:i + 9]:
                f = row.split("|")[0].split()
                if len(f) == 5 and f[4] == "2":  # mode 2: node order (the chain model's kernel path)
                    out["longest_wave"] = {"columns": line.split(":", 1)[1].strip(), "values": row.strip()}
                    break
    for line in lines:
        if line.startswith("node order: cycles/visit"):
            nums = [float(x.strip(",")) for x in line.split() if x.strip(",").replace(".", "").isdigit()]
            if len(nums) >= 3:
                out.update({"cycles_per_visit_min_window": nums[0], "cycles_per_visit_placement": nums[1],
                            "cycles_per_visit_pointer_moves": nums[2]})
        elif line.startswith("node order: placement cycles per placed pod"):
            out["cycles_per_placed_pod"] = float(line.split()[-1])
        elif line.startswith("node order: visits"):
            out["visits_line"] = line.strip()
        elif line.startswith("wave dur us"):
            out["wave_us_p50_p90_p99_max"] = [float(x) for x in line.split(":")[1].split()]
        elif line.startswith("clock MHz"):
            out["clock_mhz"] = float(line.split(":")[1].split()[0])
    return out


# The chain's latency floor (roofline.latency): one dependent global load
# (tools/micro/dep_load.hip on one MI355X: 526 cycles for a first touch in a
# new kernel, 226 for an L2 hit) and one window step alone on a SIMD
# (tools/micro/place_chain.hip V13: 214 cycles per placed pod).
DEP_LOAD_CYCLES = 526
STEP_CYCLES = 214


def chain_latency(chain):
    """The longest wave of the committed K2 profile against its dependent-
    latency floor: every dependent memory round trip it cannot avoid (the
    work-list entry, its pod records with window 0, the F heads, each further
    window, each far-resolution chunk round) at DEP_LOAD_CYCLES, plus one
    STEP_CYCLES step per placed pod, over the cycles the wave took."""
    if not chain or "longest_wave" not in chain:
        return None
    parts = [p.split() for p in chain["longest_wave"]["values"].replace("(", " ").replace(")", " ")
             .replace(",", " ").split("|")]
    try:
        dur_us = float(parts[0][2])
        visits, placed, windows = (int(x) for x in parts[1][:3])
        cyc = [int(x) for x in parts[2][:5]]
        rounds = int(parts[4][1]) if len(parts) > 4 and len(parts[4]) > 1 else 0
    except (IndexError, ValueError):
        return None
    trips = 3 + max(0, windows - 1) + rounds
    floor = trips * DEP_LOAD_CYCLES + placed * STEP_CYCLES
    # the wave's whole duration in core cycles (a far resolution that ends the
    # wave falls outside the profile's section columns)
    measured = int(round(dur_us * chain["clock_mhz"])) if chain.get("clock_mhz") else sum(cyc)
    return {"bound": "latency", "floor_cycles": floor, "measured_cycles": measured,
            "frac": round(floor / measured, 4) if measured else None,
            "longest_wave": {"duration_us": dur_us, "dependent_round_trips": trips, "placements": placed,
                             "visits": visits,
                             "windows": windows, "chunk_rounds": rounds,
                             "cycles_entry_records_prologue_minwindow_placement_moves": cyc},
            "model": "floor = dependent round trips x %d cycles (tools/micro/dep_load.hip: a dependent load's first "
                     "touch in a new kernel) + placed pods x %d cycles (tools/micro/place_chain.hip V13: one window "
                     "step alone on a SIMD); measured = the longest K2 wave's cycles in the committed profile "
                     "(%s)" % (DEP_LOAD_CYCLES, STEP_CYCLES, chain.get("source"))}


def cpu_share():
    """Host threads the all-cores CPU baseline may use: the CPUs this process may
    run on (sched_getaffinity), capped by the job's CPU share when the host
    sets one (OMP_NUM_THREADS: 16 per GPU on the MI355X boxes, whose
    sched_getaffinity lists all 256 host CPUs of 8 GPUs' jobs), or --cpu-threads."""
    avail = len(os.sched_getaffinity(0))
    env = os.environ.get("SR_BENCH_CPU_THREADS") or os.environ.get("OMP_NUM_THREADS")
    return max(1, min(avail, int(env))) if env else avail


def host_threads():
    """The encoder pool's thread count (csrc/pool.hpp: SR_HOST_THREADS, else min(16, cores))."""
    env = os.environ.get("SR_HOST_THREADS")
    return max(1, int(env)) if env else min(16, os.cpu_count() or 1)


def plan_parity(o, gpu_status, gpu_nodes, cand_off):
    """Same rule as tests/test_gpu_parity.compare_plans: every candidate the
    device evaluates has the oracle's status and, pod by pod, the oracle's
    spot node; a candidate the device flags SR_CAND_FALLBACK goes to the
    reference path (rescheduler.go:357-370 on the host), so its oracle result
    is the tick's result.  Returns (identical, n_fallback, fallback pods)."""
    fb = gpu_status == capi.SR_CAND_FALLBACK
    ok = bool(np.all(fb | (gpu_status == o["status"])))
    for c in np.flatnonzero(~fb):
        seg = slice(int(cand_off[c]), int(cand_off[c + 1]))
        if not np.array_equal(gpu_nodes[seg], o["node_of_pod"][seg]):
            ok = False
            break
    n_fb_pods = int(np.sum(np.diff(cand_off)[fb])) if fb.any() else 0
    return ok, int(fb.sum()), n_fb_pods


def cpu_baseline(sc, nm, cand_off, cand_pods, n_spot, gpu_status, gpu_nodes, gpu_checks, seconds, mutation=None):
    """The oracle (C restatement of the reference planner) on this host, rank 0
    only; BASELINE.md's three modes: all candidates on 1 thread (`value`), the
    reference-faithful early exit on 1 thread (>= 10 runs), all candidates on
    the host's CPU share.  The whole tick on the CPU share runs first: its plan
    is the one compared with the GPU's.  Where the 1-thread whole tick would
    overrun `seconds` (C4, the affinity variant at C4), the 1-thread figure is
    a bounded sample: the first k candidates of the same tick, k x4 from 64
    until one run takes seconds / 5; `sample` says which."""
    from oracle_lib import OracleSnapshot, oracle_plan
    snap = OracleSnapshot(sc.ptr, nm.spot, nm.node_pod_off, nm.node_pod_idx)
    if mutation is not None:  # the steady-state tick's snapshot: one more pod on one spot node
        snap.lib.oracle_snapshot_add_pod(snap.h, sc.ptr, mutation[0], mutation[1])

    def timed(mode, threads, min_runs, budget_s, max_runs=500):
        for _ in range(2):  # warm-ups
            oracle_plan(snap, sc.ptr, cand_off, cand_pods, mode=mode, threads=threads)
        ts, r = [], None
        t_end = time.perf_counter() + budget_s
        while len(ts) < min_runs or (time.perf_counter() < t_end and len(ts) < max_runs):
            t0 = time.perf_counter()
            r = oracle_plan(snap, sc.ptr, cand_off, cand_pods, mode=mode, threads=threads)
            ts.append(time.perf_counter() - t0)
        return 1e3 * float(np.median(ts)), len(ts), sum(ts), r

    threads = cpu_share()
    n_cand = len(cand_off) - 1
    t0 = time.perf_counter()
    res = oracle_plan(snap, sc.ptr, cand_off, cand_pods, mode=1, threads=threads)  # the plan compared
    t_mt = time.perf_counter() - t0
    full_1core = t_mt * threads <= seconds
    if full_1core:
        ms_all, n_all, s_all, r1 = timed(1, 1, 3, seconds)
        checks_1 = float(r1["checks"])
        sample = ("full tick: all %d candidates / %d pods x %d spot nodes, median of %d runs (%.1f s) after 2 "
                  "warm-ups" % (n_cand, len(cand_pods), n_spot, n_all, s_all))
        dense_1 = float(len(cand_pods)) * n_spot
    else:
        k = 64
        while True:
            k = min(k, n_cand)
            off_k = np.ascontiguousarray(cand_off[:k + 1])
            pods_k = np.ascontiguousarray(cand_pods[:int(off_k[-1])])
            t0 = time.perf_counter()
            rk = oracle_plan(snap, sc.ptr, off_k, pods_k, mode=1, threads=1)
            dt = time.perf_counter() - t0
            if dt >= seconds / 5 or k == n_cand:
                break
            k *= 4
        ms_all, n_all, checks_1 = 1e3 * dt, 1, float(rk["checks"])
        sample = ("bounded sample: the first %d of the tick's %d candidates (%d pods x %d spot nodes), one 1-thread "
                  "run of %.1f s; the whole tick on %d threads took %.1f s" % (k, n_cand, len(pods_k), n_spot, dt,
                                                                                threads, t_mt))
        dense_1 = float(len(pods_k)) * n_spot
    ms_early, n_early, _, early = timed(0, 1, 10, min(2.0, seconds / 4))
    if t_mt > 1.0:  # a long whole tick: its one run is the CPU-share figure
        ms_mt, n_mt = 1e3 * t_mt, 1
    else:
        ms_mt, n_mt, _, _ = timed(1, threads, 10, min(3.0, seconds / 3))
    parity, n_fb, n_fb_pods = plan_parity(res, gpu_status, gpu_nodes, cand_off)
    return {"value": checks_1 / (ms_all / 1e3), "unit": "checks/s", "cores": 1, "kind": "port",
            "host_cpus": os.cpu_count(), "host_cpus_affinity": len(os.sched_getaffinity(0)),
            "host_cpu_share_threads": threads,
            "value_definition": "reference-equivalent checks (issued CheckPredicates calls) / 1-core all-candidates "
                                "time (the whole tick, or the bounded sample named in `sample`)",
            "dense_equivalent_per_s": dense_1 / (ms_all / 1e3),
            "sample": sample,
            "ms_per_tick_all_candidates_1core": round(ms_all, 3) if full_1core else None,
            "ms_1core_sample": None if full_1core else round(ms_all, 3),
            "ms_per_tick_reference_faithful_1core": round(ms_early, 4),
            "reference_faithful_runs": n_early,
            "reference_faithful_first_ok": int(early["first_ok"]),
            "ms_per_tick_all_candidates_%dthreads" % threads: round(ms_mt, 3),
            "all_candidates_threads_runs": n_mt,
            "threads_note": "all-candidates mode on the job's CPU share: min(sched_getaffinity, OMP_NUM_THREADS or "
                            "SR_BENCH_CPU_THREADS); a median after 2 warm-ups, or one run when it takes over 1 s",
            "issued_checks_per_tick": int(res["checks"]),
            "plans_identical_to_gpu": parity,
            "plans_compared": "the whole tick (%d candidates), planned by the oracle on %d threads" % (n_cand, threads),
            "reference_equivalent_checks_match_gpu": int(res["checks"]) == int(gpu_checks),
            "parity_rule": "device-evaluated candidates: status + every pod's node equal to the oracle; "
                           "fallback candidates take the reference path",
            "fallback_candidates": n_fb, "fallback_candidate_pods": n_fb_pods,
            "fallback_ratio": round(n_fb / max(1, len(cand_off) - 1), 4)}


def rank_record(rank, n_cand, n_pods, local_elapsed_s, steps, breakdown_ms):
    """One rank's own tick parts for the line's per_rank: its shard, its timed
    region's time per step before the max over ranks, and the calibration
    pass's K0 / K2 / collective / K3 per tick."""
    return {"rank": int(rank), "candidates": int(n_cand), "candidate_pods": int(n_pods),
            "ms_per_step_local": round(1e3 * local_elapsed_s / max(1, steps), 5),
            **{k + "_ms": round(float(v), 5) for k, v in breakdown_ms.items()}}


def gather_per_rank(rec, world):
    """Every rank's record on every rank, in rank order (gloo all_gather_object)."""
    if world <= 1:
        return [rec]
    import torch.distributed as dist
    out = [None] * world
    dist.all_gather_object(out, rec)
    return out


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"


def visible_devices(kfd_nodes=KFD_NODES, environ=None):
    """GPUs this process would see, counted without any HIP call (the launcher
    must not initialise the runtime in a parent that starts the ranks): the KFD
    topology nodes with SIMDs (GPU agents; CPU agents report simd_count 0),
    restricted by ROCR/HIP/CUDA_VISIBLE_DEVICES when one is set."""
    environ = os.environ if environ is None else environ
    n = 0
    try:
        entries = os.listdir(kfd_nodes)
    except OSError:
        entries = []
    for e in entries:
        try:
            with open(os.path.join(kfd_nodes, e, "properties")) as f:
                props = dict(line.split(None, 1) for line in f if len(line.split(None, 1)) == 2)
        except OSError:
            continue
        if int(props.get("simd_count", "0").strip() or 0) > 0:
            n += 1
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(n, argv, script=None, devices=None):
    """One child process per GPU (ranks 0..n-1, LOCAL_RANK = rank) running this
    script with the same arguments; rank 0 prints the JSON line.  This process
    never touches the GPU and never execs: it waits for the children, stops the
    others when one fails, and exits with the first failure's code.
    (`script` / `devices`: tests only.)"""
    have = visible_devices() if devices is None else devices
    if have < n:
        print("bench.py --gpus %d: only %d HIP device(s) visible; refusing to run %d ranks on fewer GPUs"
              % (n, have, n), file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)] + argv, env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # the other ranks would wait in a collective forever
                    q.terminate()
        time.sleep(0.05)
    return rc


def measure_ticks(lib, checker, sc, rank, world, args):
    """The timed region on one synthetic cluster: its node map and candidate
    lists (run()'s, rescheduler.go:228-264), this rank's shard (c % world), the
    steady-state tick prepared, one full run (K2's bytes, the reference-
    equivalent checks), the warm-up, the calibration pass, then EXACTLY
    args.steps sr_plan_run calls bracketed by barrier + synchronize (max over
    ranks), and the full run once more for the parity check."""
    import torch
    import torch.distributed as dist
    nm = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
    # run()'s candidate lists (rescheduler.go:228-264): GetPodsForDeletionOnNodeDrain + the
    # DaemonSet-owner filter, on the host (sr_pods_for_deletion)
    t0 = time.perf_counter()
    cand_off, cand_pods, _, _, st = pods_for_deletion(lib.sr_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain),
                                                      nm.on_demand, nm.node_pod_off, nm.node_pod_idx)
    pfd_ms = 1e3 * (time.perf_counter() - t0)
    assert st == capi.SR_OK, st
    loff, lpods, gidx = shard(cand_off, cand_pods, rank, world)

    snap = ctypes.c_void_p()
    st = lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                ctypes.byref(snap))
    assert st == capi.SR_OK
    cands = capi.sr_candidates(len(loff) - 1, capi.ptr(loff, capi.P32), capi.ptr(lpods, capi.P32),
                               capi.ptr(gidx, capi.P32))
    t0 = time.perf_counter()
    st = lib.sr_plan_prepare(checker.handle, snap, sc.ptr, ctypes.byref(cands))
    assert st == capi.SR_OK, checker.last_error()
    pack_ms = 1e3 * (time.perf_counter() - t0)

    maxp = int(np.max(np.diff(loff))) if len(loff) > 1 else 1
    wmap = np.zeros(max(1, maxp), np.int32)
    out = capi.sr_plan_out()
    out.winner_map = capi.ptr(wmap, capi.P32)
    mut_pod = int(cand_pods[0]) if len(cand_pods) else 0  # the same pod on every rank: one cluster state
    mut_pos = min(args.mut_pos, len(nm.spot) - 1)
    mutation = None
    steady = {"tick": "cold", "k0": "every row"}
    if args.tick == "steady" and mut_pos >= 0 and len(cand_pods):
        # The steady state of a planner between two housekeeping ticks: the
        # previous tick's candidate input on its snapshot (twice: the second
        # encode indexes the candidate side), then this tick, a fresh snapshot
        # with one more pod on one spot node.  The timed steps replay this
        # tick's device work: K0 on the changed word columns and moved
        # threshold rows (the rest of the tables is the previous tick's), K2, K3.
        for _ in range(2):
            assert lib.sr_plan_prepare(checker.handle, snap, sc.ptr, ctypes.byref(cands)) == capi.SR_OK
            assert lib.sr_plan_run(checker.handle, ctypes.byref(out)) == capi.SR_OK, checker.last_error()
        tick_snap = ctypes.c_void_p()
        assert lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                      capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                      ctypes.byref(tick_snap)) == capi.SR_OK
        assert lib.sr_snapshot_add_pod(tick_snap, sc.ptr, mut_pod, mut_pos) == capi.SR_OK
        lib.sr_snapshot_destroy(snap)
        snap = tick_snap
        assert lib.sr_plan_prepare(checker.handle, snap, sc.ptr, ctypes.byref(cands)) == capi.SR_OK
        tq = checker.timing()
        mutation = (mut_pod, mut_pos)
        k0 = ("none: the tables stand, K2 recomputes the changed node's bits (K0 runs once 16 nodes changed)"
              if tq.k0_columns == -2 else "every row" if tq.k0_columns == -1 else
              "incremental: %d word columns, %d moved threshold rows" % (tq.k0_columns, tq.k0_rows_moved))
        steady = {"tick": "steady: the previous tick's candidate input, one more pod on spot node %d" % mut_pos,
                  "candidate_side_reused": bool(tq.enc_reused), "pod_patches": int(tq.enc_pod_patches), "k0": k0,
                  "work_list_by_cost": bool(tq.k2_list_by_cost)}
    # one run with per-candidate outputs first: K2's byte counts and the
    # reference-equivalent check count of this workload's plan
    status = np.zeros(max(1, len(loff) - 1), np.int32)
    nodes_out = np.zeros(max(1, len(lpods)), np.int32)
    full = capi.sr_plan_out()
    full.status = capi.ptr(status, capi.P32)
    full.node_of_pod = capi.ptr(nodes_out, capi.P32)
    full.winner_map = capi.ptr(wmap, capi.P32)
    st = lib.sr_plan_run(checker.handle, ctypes.byref(full))
    assert st == capi.SR_OK, (st, checker.last_error())
    issued_local, dense_local = float(full.checks), float(full.checks_dense)
    for _ in range(args.warmup):
        assert lib.sr_plan_run(checker.handle, ctypes.byref(out)) == capi.SR_OK, checker.last_error()

    # Calibration (untimed): every kernel bracketed with events -> per-kernel
    # breakdown and the dominant kernel.
    names = ["k0_tables", "k2_placement", "k3_winner", "collective"]
    checker.set_timing(7)
    for _ in range(max(5, min(args.steps, 20))):
        st = lib.sr_plan_run(checker.handle, ctypes.byref(out))
        assert st == capi.SR_OK, (st, checker.last_error())
    tm = checker.timing()
    breakdown = dict(zip(names, [x / max(1, tm.n_runs) for x in
                                 (tm.ms_tables, tm.ms_placement, tm.ms_winner, tm.ms_collective)]))
    dom = max(names[:2], key=lambda x: breakdown[x])
    dom_bit = 1 << names.index(dom)

    # Timed region: K steps, only the dominant kernel bracketed with events.
    checker.set_timing(0 if args.no_events else dom_bit | (max(1, args.event_every) << 8))
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    bad = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bad |= lib.sr_plan_run(checker.handle, ctypes.byref(out))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    local_elapsed = elapsed
    assert bad == capi.SR_OK, (bad, checker.last_error())  # a failing run must not be timed as a fast step
    tm = checker.timing()
    dom_ms = ([tm.ms_tables, tm.ms_placement][names.index(dom)] / max(1, tm.n_runs) if not args.no_events
              else breakdown[dom])
    checker.set_timing(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        c = torch.tensor([issued_local, dense_local], dtype=torch.float64)
        dist.all_reduce(c, op=dist.ReduceOp.SUM)
        total_issued, total_dense = float(c[0].item()), float(c[1].item())
    else:
        total_issued, total_dense = issued_local, dense_local
    per_rank = gather_per_rank(rank_record(rank, len(loff) - 1, len(lpods), local_elapsed, args.steps, breakdown),
                               world)

    # per-candidate outputs once more (outside the timed region): the parity
    # check and K2's byte counts of the same plan
    st = lib.sr_plan_run(checker.handle, ctypes.byref(full))
    assert st == capi.SR_OK, (st, checker.last_error())
    tm = checker.timing()
    return dict(nm=nm, cand_off=cand_off, cand_pods=cand_pods, loff=loff, lpods=lpods, gidx=gidx, snap=snap,
                cands=cands, out=out, wmap=wmap, full=full, status=status, nodes_out=nodes_out, mutation=mutation, steady=steady,
                pfd_ms=pfd_ms, pack_ms=pack_ms, breakdown=breakdown, dom=dom, dom_ms=dom_ms, elapsed=elapsed,
                total_issued=total_issued, total_dense=total_dense, tm=tm, issued_local=issued_local,
                per_rank=per_rank, mut_pod=mut_pod, mut_pos=mut_pos)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", type=int, default=3, choices=[1, 2, 3, 4, 5])
    ap.add_argument("--variant", default="baseline", choices=["baseline", "realistic", "affinity"],
                    help="realistic: the config with StatefulSet volumes, init containers and GPU pods; affinity: "
                         "Deployments with hostname anti-affinity and zone topology spread (both report the "
                         "fallback ratio on them); baseline: BASELINE.json's config as specified")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (BASELINE's line): the config's own cluster, its candidates split over the ranks; "
                         "weak: N x its candidates over the same spot pool")
    ap.add_argument("--no-weak-beside", action="store_true",
                    help="N > 1 with --scaling strong: skip the weak-scaled measurement reported beside the line "
                         "(weak_scaling)")
    ap.add_argument("--transport", default="shm", choices=["shm", "rccl"],
                    help="N > 1: shm = the ranks reduce each tick through one shared-memory segment (no collective, "
                         "no K3; sr_comm_init_shm); rccl = one RCCL allreduce(min) + K3 (sr_comm_init)")
    ap.add_argument("--tick", default="steady", choices=["steady", "cold"],
                    help="steady: the timed step replays a steady-state tick (the previous tick's candidate input, "
                         "one spot node changed: incremental K0 + K2); cold: a first tick (every table row)")
    ap.add_argument("--mut-pos", type=int, default=7,
                    help="spot position of the steady tick's changed node (7: inside the 512-node F heads)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--e2e-reps", type=int, default=20, help="steady-state end-to-end ticks timed after the steps")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-events", action="store_true",
                    help="A/B only: no HIP events in the timed region (roofline from the calibration pass)")
    ap.add_argument("--event-every", type=int, default=16,
                    help="HIP events on every n-th step of the timed region (timestamped dispatches lengthen a tick)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    # SR_BENCH_DEVICE: every rank on that one GPU (rehearsing the N > 1 path on a one-GPU box, --transport shm)
    local = int(os.environ.get("SR_BENCH_DEVICE", os.environ.get("LOCAL_RANK", "0")))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(local)

    lib = capi.load_planner()
    checker = PredicateChecker(local)
    transport = "none"
    if world > 1 and args.transport == "shm":
        # one shared-memory segment per job: its name and session from rank 0
        box = [int.from_bytes(os.urandom(4), "little")]
        dist.broadcast_object_list(box, src=0)
        session = box[0]
        checker.attach_shared_memory("/srbench-%08x" % session, session, world, rank,
                                     max_cand=DEFAULT_OD[args.config] * world)
        dist.barrier()  # every rank attached before any plans (rank 0's planner removes the name when it closes)
        transport = "shm"
    elif world > 1:
        uid = (ctypes.c_uint8 * capi.SR_UNIQUE_ID_BYTES)()
        if rank == 0:
            assert lib.sr_comm_unique_id(uid) == capi.SR_OK
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0)
        uid = (ctypes.c_uint8 * capi.SR_UNIQUE_ID_BYTES).from_buffer_copy(box[0])
        st = lib.sr_comm_init(checker.handle, uid, world, rank)
        assert st == capi.SR_OK, checker.last_error()
        transport = "rccl"

    variant_kw = {"realistic": REALISTIC, "affinity": AFFINITY}.get(args.variant, {})
    sc = SynthCluster(args.config, n_on_demand=cluster_on_demand(args.config, world, args.scaling), **variant_kw)
    M = measure_ticks(lib, checker, sc, rank, world, args)
    # (loff / lpods / gidx stay referenced: `cands` points into them)
    nm, cand_off, cand_pods, loff, lpods = M["nm"], M["cand_off"], M["cand_pods"], M["loff"], M["lpods"]
    gidx = M["gidx"]  # noqa: F841
    snap, cands, out, wmap, full = M["snap"], M["cands"], M["out"], M["wmap"], M["full"]
    status, nodes_out, mutation, steady = M["status"], M["nodes_out"], M["mutation"], M["steady"]
    pfd_ms, pack_ms, breakdown, dom, dom_ms = M["pfd_ms"], M["pack_ms"], M["breakdown"], M["dom"], M["dom_ms"]
    elapsed, total_issued, total_dense, tm = M["elapsed"], M["total_issued"], M["total_dense"], M["tm"]
    issued_local, per_rank, mut_pod, mut_pos = M["issued_local"], M["per_rank"], M["mut_pod"], M["mut_pos"]
    ms_step = 1e3 * elapsed / args.steps

    # Result latency of one tick on an idle device: sr_plan_run from the launch
    # to the winner and its mapping in host memory.  On one rank the run returns
    # once the candidates up to the winner are planned (K2 writes each outcome
    # to the host) and the rest of the grid finishes behind it on the stream,
    # so back-to-back ticks (ms_per_step) are bounded by the whole K0 + K2.
    lat = []
    for _ in range(50):
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = lib.sr_plan_run(checker.handle, ctypes.byref(out))
        lat.append(1e3 * (time.perf_counter() - t1))
        assert st == capi.SR_OK, (st, checker.last_error())
        assert out.first_ok == full.first_ok and out.winner == full.winner
    torch.cuda.synchronize()
    if world == 1 and out.first_ok >= 0:  # the winner's mapping equals the full plan's
        k = int(out.first_ok)
        assert out.winner_npods == loff[k + 1] - loff[k]
        assert np.array_equal(wmap[:out.winner_npods], nodes_out[loff[k]:loff[k + 1]])

    # End-to-end ticks in the steady state (outside the contract's K steps).
    # Every tick gets a FRESH snapshot, as run() builds one per housekeeping
    # tick (rescheduler.go:195,215), and every other tick has one more pod on
    # one spot node: consecutive ticks differ in one node, the steady state of
    # a planner that keeps what it derived from the previous tick.  Snapshot
    # creation is host work of NewNodeMap / GetClusterSnapshot (in full_tick).
    first_ok_ref = out.first_ok

    def fresh_snapshot(r):
        h = ctypes.c_void_p()
        st_ = lib.sr_snapshot_create(sc.ptr, capi.ptr(nm.spot, capi.P32), len(nm.spot),
                                     capi.ptr(nm.node_pod_off, capi.P32), capi.ptr(nm.node_pod_idx, capi.P32),
                                     ctypes.byref(h))
        assert st_ == capi.SR_OK
        if r % 2 == 1 and mut_pos >= 0:
            assert lib.sr_snapshot_add_pod(h, sc.ptr, mut_pod, mut_pos) == capi.SR_OK
        return h

    def summary(xs):
        return {"median_ms": round(float(np.median(xs)), 4), "min_ms": round(float(np.min(xs)), 4)}

    ref_t, ref_batches, ref_enc, ref_state, ref_up, ref_upl = [], [], [], [], [], []
    all_t, all_enc, all_upl, all_state, all_reused, all_patches, all_bytes = [], [], [], [], [], [], []
    wmap2 = np.zeros_like(wmap)
    for r in range(args.e2e_reps + 2):  # two untimed ticks first: the planner's view of the pool settles
        h = fresh_snapshot(r)
        # reference-faithful tick: candidates in order until the first drainable one (sr_plan_first),
        # on an idle device as between two housekeeping ticks (the previous iteration's every-candidate
        # run may still be planning candidates past its winner)
        fo = capi.sr_plan_out()
        fo.winner_map = capi.ptr(wmap2, capi.P32)
        if E2E_IDLE:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = lib.sr_plan_first(checker.handle, h, sc.ptr, ctypes.byref(cands), ctypes.byref(fo))
        dt = 1e3 * (time.perf_counter() - t1)
        assert st == capi.SR_OK, checker.last_error()
        tq = checker.timing()
        if r >= 2:
            ref_t.append(dt)
            ref_batches.append(tq.prefix_batches)
            ref_enc.append(tq.ms_pack_host)
            ref_upl.append(tq.ms_upload)
            ref_state.append(tq.enc_state_nodes)
            ref_up.append(tq.bytes_uploaded)
        # all candidates planned: prepare + run
        if E2E_IDLE:
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        st = lib.sr_plan_prepare(checker.handle, h, sc.ptr, ctypes.byref(cands))
        assert st == capi.SR_OK, checker.last_error()
        st = lib.sr_plan_run(checker.handle, ctypes.byref(out))
        assert st == capi.SR_OK, checker.last_error()
        dt = 1e3 * (time.perf_counter() - t1)
        tq = checker.timing()
        if r >= 2:
            all_t.append(dt)
            all_enc.append(tq.ms_pack_host)
            all_upl.append(tq.ms_upload)
            all_state.append(tq.enc_state_nodes)
            all_reused.append(tq.enc_reused)
            all_patches.append(tq.enc_pod_patches)
            all_bytes.append(tq.bytes_uploaded)
        assert fo.first_ok == out.first_ok or world > 1
        lib.sr_snapshot_destroy(h)
    # The whole housekeeping tick from the cluster arrays: NewNodeMap (A1-A5),
    # the candidate lists (GetPodsForDeletionOnNodeDrain + owner filter),
    # GetClusterSnapshot (A6), then the reference-faithful planning.  Between
    # two ticks one pod on a spot node changes its cpu request (and stamp), so
    # that node's pod sort, RequestedCPU, place in the spot order and snapshot
    # state change.  "kept": a long-running planner that keeps the previous
    # tick's node map cache and snapshot (sr_new_node_map_cached,
    # sr_snapshot_refresh); "fresh": everything rebuilt every tick.
    cl = sc.cluster
    tick_pod = int(nm.node_pod_idx[nm.node_pod_off[nm.spot[mut_pos]]]) if mut_pos >= 0 and len(nm.spot) else -1
    if tick_pod >= 0 and nm.node_pod_off[nm.spot[mut_pos] + 1] == nm.node_pod_off[nm.spot[mut_pos]]:
        tick_pod = -1
    tick_arrays = [np.ctypeslib.as_array(a, shape=(sc.n_pods,)) for a in
                   (cl.pods.cpu_sort_milli, cl.pods.req_milli_cpu, cl.acc_milli_cpu) if a] if tick_pod >= 0 else []
    tick_base = [int(a[tick_pod]) for a in tick_arrays]
    stamps_v = np.ctypeslib.as_array(cl.pod_stamp, shape=(sc.n_pods,)) if cl.pod_stamp and tick_pod >= 0 else None
    stamp_base = int(stamps_v[tick_pod]) if stamps_v is not None else 0

    def set_tick_state(k):  # state k of the changing pod (0: as generated)
        for a, b in zip(tick_arrays, tick_base):
            a[tick_pod] = b + k
        if stamps_v is not None:
            stamps_v[tick_pod] = stamp_base ^ (0x5A5A5A5A00000000 * k)

    nm_bufs, pfd_bufs = {}, {}
    nm_cache = ctypes.c_void_p()
    assert lib.sr_node_map_cache_create(ctypes.byref(nm_cache)) == capi.SR_OK
    kept_snap = None
    stage_names = ("new_node_map", "pods_for_deletion", "snapshot", "plan_first")
    full_ticks = {"kept": ([], {k: [] for k in stage_names}), "fresh": ([], {k: [] for k in stage_names})}
    tick_first_ok = {}
    tick_rebuilt, tick_sorted, tick_plan = [], [], []
    for mode in ("kept", "fresh"):
        for r in range(args.e2e_reps + 1):  # the first tick untimed (the kept path fills its caches)
            set_tick_state(r % 2)
            sorted_n = ctypes.c_int32(0)
            rebuilt = ctypes.c_int32(0)
            t1 = time.perf_counter()
            if mode == "kept":  # the planner's buffers and caches from the previous tick
                nm2 = new_node_map(lambda cp, pp, mp: lib.sr_new_node_map_cached(nm_cache, cp, pp, mp,
                                                                                 ctypes.byref(sorted_n)),
                                   sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label, bufs=nm_bufs)
            else:
                nm2 = new_node_map(lib.sr_new_node_map, sc.ptr, sc.n_nodes, sc.n_pods, sc.od_label, sc.spot_label)
            t2 = time.perf_counter()
            co2, cp2, _, _, st = pods_for_deletion(lib.sr_pods_for_deletion, sc.ptr, ctypes.byref(sc.drain),
                                                   nm2.on_demand, nm2.node_pod_off, nm2.node_pod_idx,
                                                   bufs=pfd_bufs if mode == "kept" else None)
            assert st == capi.SR_OK, st
            lo2, lp2, gi2 = shard(co2, cp2, rank, world)
            t3 = time.perf_counter()
            args_snap = (sc.ptr, capi.ptr(nm2.spot, capi.P32), len(nm2.spot), capi.ptr(nm2.node_pod_off, capi.P32),
                         capi.ptr(nm2.node_pod_idx, capi.P32))
            if mode == "kept" and kept_snap is not None:  # linked to this tick's cached node map
                st = lib.sr_snapshot_refresh_cached(kept_snap, nm_cache, *args_snap, ctypes.byref(rebuilt))
                snap2 = kept_snap
            else:
                snap2 = ctypes.c_void_p()
                st = lib.sr_snapshot_create(*args_snap, ctypes.byref(snap2))
                if mode == "kept":
                    kept_snap = snap2
            assert st == capi.SR_OK
            t4 = time.perf_counter()
            c2 = capi.sr_candidates(len(lo2) - 1, capi.ptr(lo2, capi.P32), capi.ptr(lp2, capi.P32),
                                    capi.ptr(gi2, capi.P32))
            fo = capi.sr_plan_out()
            fo.winner_map = capi.ptr(wmap2, capi.P32)
            st = lib.sr_plan_first(checker.handle, snap2, sc.ptr, ctypes.byref(c2), ctypes.byref(fo))
            assert st == capi.SR_OK, checker.last_error()
            t5 = time.perf_counter()
            tq = checker.timing()
            if r and mode == "kept":
                tick_plan.append((tq.prefix_batches, tq.enc_reused, tq.enc_static_rebuilt, tq.enc_state_nodes,
                                  tq.ms_pack_host, tq.k0_columns))
            # both paths plan the same cluster state alike
            assert tick_first_ok.setdefault(r % 2, fo.first_ok) == fo.first_ok
            if mode == "fresh":
                lib.sr_snapshot_destroy(snap2)
            if r == 0:
                continue
            if mode == "kept":
                tick_rebuilt.append(rebuilt.value)
                tick_sorted.append(sorted_n.value)
            ft, stg = full_ticks[mode]
            ft.append(1e3 * (t5 - t1))
            for k, a, b in zip(stage_names, (t1, t2, t3, t4), (t2, t3, t4, t5)):
                stg[k].append(1e3 * (b - a))
    set_tick_state(0)
    if kept_snap is not None:
        lib.sr_snapshot_destroy(kept_snap)
    lib.sr_node_map_cache_destroy(nm_cache)
    end_to_end = None
    if ref_t:
        end_to_end = dict(summary(ref_t), **{
            "span": "sr_plan_first on a fresh snapshot with one spot node changed since the previous tick: "
                    "prefix-batched encode + H2D + kernels until the first drainable candidate, winner and "
                    "mapping on the host (run() stops there, rescheduler.go:286)",
            "prefix_batches": int(np.median(ref_batches)), "encode_ms_last_batch": round(float(np.median(ref_enc)), 4),
            "upload_issue_ms_last_batch": round(float(np.median(ref_upl)), 4),
            "state_nodes_reencoded": int(np.median(ref_state)), "upload_bytes": int(np.median(ref_up)),
            "all_candidates": dict(summary(all_t), **{
                "encode_ms": round(float(np.median(all_enc)), 3), "upload_ms": round(float(np.median(all_upl)), 3),
                "state_nodes_reencoded": int(np.median(all_state)),
                "candidate_side_reused": "%d of %d ticks" % (int(np.sum(all_reused)), len(all_reused)),
                "pod_patches_median": int(np.median(all_patches)), "upload_bytes": int(np.median(all_bytes)),
                "span": "sr_plan_prepare + sr_plan_run over every candidate, same fresh one-node-changed snapshots"}),
            "pods_for_deletion_ms": round(pfd_ms, 3), "reps": len(ref_t), "host_threads": host_threads(),
            "full_tick_median_ms": (round(float(np.median(full_ticks["kept"][0])), 3)
                                    if full_ticks["kept"][0] else None),
            "full_tick_stages_median_ms": {k: round(float(np.median(v)), 3) for k, v in full_ticks["kept"][1].items()}
            if full_ticks["kept"][0] else None,
            "full_tick_kept_state": {"nodes_sorted_median": int(np.median(tick_sorted)) if tick_sorted else None,
                                     "snapshot_nodes_rebuilt_median": int(np.median(tick_rebuilt))
                                     if tick_rebuilt else None,
                                     "plan_first_last": dict(zip(("prefix_batches", "enc_reused", "static_view",
                                                                  "state_nodes", "encode_ms_last_batch", "k0_columns"),
                                                                 tick_plan[-1])) if tick_plan else None},
            "full_tick_fresh_median_ms": (round(float(np.median(full_ticks["fresh"][0])), 3)
                                          if full_ticks["fresh"][0] else None),
            "full_tick_fresh_stages_median_ms": {k: round(float(np.median(v)), 3)
                                                 for k, v in full_ticks["fresh"][1].items()}
            if full_ticks["fresh"][0] else None,
            "full_tick_span": "cluster arrays (one spot pod's cpu request changed since the previous tick) -> "
                              "sr_new_node_map_cached -> sr_pods_for_deletion -> sr_snapshot_refresh_cached of the "
                              "previous tick's snapshot -> sr_plan_first; fresh: sr_new_node_map and "
                              "sr_snapshot_create every tick"})

    # N > 1, strong scaling (the line): the weak-scaled tick beside it, labelled
    # -- every rank one config-sized candidate set over the same spot pool (after
    # the latency and end-to-end sections, which plan the line's workload)
    weak_scaling = None
    if world > 1 and args.scaling == "strong" and not args.no_weak_beside:
        sw = SynthCluster(args.config, n_on_demand=cluster_on_demand(args.config, world, "weak"), **variant_kw)
        W = measure_ticks(lib, checker, sw, rank, world, args)
        weak_scaling = {
            "scaling": "weak", "value": W["total_issued"] / W["elapsed"] * args.steps if W["elapsed"] > 0 else 0.0,
            "unit": "checks/s", "ms_per_step": 1e3 * W["elapsed"] / args.steps,
            "plans_per_s": (len(W["cand_off"]) - 1) / (W["elapsed"] / args.steps),
            "workload": workload_name(args.config, sw.n_nodes, len(W["nm"].on_demand), len(W["nm"].spot), sw.n_pods,
                                      world, "weak", args.variant),
            "candidates_per_rank": shard_sizes(len(W["cand_off"]) - 1, world), "per_rank": W["per_rank"],
            "first_ok": int(W["out"].first_ok), "winner": int(W["out"].winner),
            "note": "not the line's value: N x the config's candidates over the same spot pool (weak scaling), "
                    "measured after the line in the same job"}
        lib.sr_snapshot_destroy(W["snap"])

    if rank == 0:
        alg = {"k2_placement": tm.bytes_placement, "k0_tables": tm.bytes_tables}[dom]
        achieved = alg / (dom_ms * 1e-3) / 1e9 if dom_ms > 0 else 0.0
        # PMC traffic of the same kernel on this config and variant, from the
        # committed rocprofv3 passes (not measured in this run), else null
        traffic, traffic_src, traffic_null = None, None, None
        pmc_name = "pmc_traffic_c%d%s.json" % (args.config, "" if args.variant == "baseline" else "_" + args.variant)
        pmc = os.path.join(REPO, "profiles", pmc_name)
        if world > 1:
            traffic_null = "no PMC pass of the multi-rank command"
        elif not os.path.exists(pmc):
            traffic_null = "no committed PMC pass for config %d, variant %s (profiles/%s)" % (args.config,
                                                                                          args.variant, pmc_name)
        else:
            with open(pmc) as f:
                pj = json.load(f)
            traffic = pj.get(dom)
            if traffic is None:
                traffic_null = "profiles/%s holds no %s entry" % (pmc_name, dom)
            traffic_src = {"file": os.path.relpath(pmc, REPO), "measured_at_head": pj.get("measured_at_head", "unknown"),
                           "how": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this bench command "
                                  "(tools/gpu_round.sh); not measured in this run"}
        chain = k2_chain_summary(latest_profile("c%d%s_k2_wave_profile.txt"
                                                % (args.config, "" if args.variant == "baseline" else "_" + args.variant)))
        line = {
            "metric": "reference-equivalent pod x spot-node feasibility checks/s (drain-plan latency: "
                      "drain_plan_latency_ms)",
            "value": total_issued / elapsed * args.steps if elapsed > 0 else 0.0,
            "unit": "checks/s",
            "checks_per_tick": {"reference_equivalent": int(total_issued), "dense_equivalent": int(total_dense),
                                "dense_equivalent_per_s": total_dense / elapsed * args.steps if elapsed > 0 else 0.0,
                                "note": "reference_equivalent = CheckPredicates calls the reference loop makes for "
                                        "the same plan of every candidate (value); dense_equivalent = candidate "
                                        "pods x spot nodes (notional, not work done)"},
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_step, "latency_ms": round(float(np.median(lat)), 5),
            "drain_plan_latency_ms": end_to_end["median_ms"] if end_to_end else None,
            "drain_plan_latency_span": "host to host, SURVEY 8(d): sr_plan_first on a fresh snapshot with one spot "
                                       "node changed (encode + H2D + kernels + winner and mapping on the host); "
                                       "end_to_end_tick has the every-candidate plan and the whole housekeeping "
                                       "tick; ms_per_step is the device tick (inputs resident, back to back)",
            "latency_span": "median of 50 single sr_plan_run calls on an idle device: launch to the winner and "
                            "its mapping in host memory (ms_per_step: back-to-back ticks, every candidate planned)",
            "plans_per_s": (len(cand_off) - 1) / (elapsed / args.steps),
            "higher_is_better": True, "scaling": args.scaling, "vs_baseline": None, "dtype": "int64",
            "data": "synthetic",
            "config": {"workload": workload_name(args.config, sc.n_nodes, len(nm.on_demand), len(nm.spot),
                                                 sc.n_pods, world, args.scaling, args.variant),
                       "variant": args.variant, **steady,
                       "nodes": sc.n_nodes, "pods": sc.n_pods, "on_demand_nodes": int(len(nm.on_demand)),
                       "spot_nodes": int(len(nm.spot)), "candidates": int(len(cand_off) - 1),
                       "candidate_pods": int(len(cand_pods)), "parallelism": "candidates c%%%d" % world,
                       "candidates_per_rank": shard_sizes(len(cand_off) - 1, world)},
            "collective": {"backend": transport, "ranks": world if world > 1 else 0,
                           "per_tick": {"shm": "no collective: every rank's K2 writes its outcomes into one "
                                               "shared-memory segment, each host walks them in global order "
                                               "(sr_comm_init_shm)",
                                        "rccl": "one allreduce(min) of 3 x u64 + K3",
                                        "none": "none (one GPU)"}[transport]},
            "per_rank": per_rank,
            "weak_scaling": weak_scaling,
            "scaling_model": {"prediction_us": predict(args.config, world, transport),
                              "model": "spotplanner/scaling.py: measured 1-GPU parts (round 6), ASSUMED RCCL "
                                       "allreduce latency, the shm transport's host walk bounded by the N=2 "
                                       "rehearsal on one GPU; per_rank holds the measured parts",
                              "strong_pays": choose_scaling(args.config, world, transport)[0] == "strong"}
            if world > 1 else None,
            "first_ok": int(out.first_ok), "winner": int(out.winner),
            "fallback_candidates": int(np.sum(status[:len(loff) - 1] == capi.SR_CAND_FALLBACK)),
            "kernels_ms": {kk: round(v, 5) for kk, v in breakdown.items()},
            "workload_rows": {"static_classes": tm.n_rows_static, "threshold_rows": tm.n_rows_threshold,
                              "words_per_row": tm.n_words},
            "host_pack_ms": round(pack_ms, 3),
            "end_to_end_tick": end_to_end,
            "host_pods_for_deletion_ms": round(pfd_ms, 3),
            "roofline": {"bound": "hbm", "kernel": dom, "kernel_ms": round(dom_ms, 5),
                         "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_ms_source": "HIP events of the timed region (every %d-th step, recorded by the "
                                             "kernel's own dispatch); they open at the dispatch, so they include "
                                             "the gap after the previous kernel" % max(1, args.event_every),
                         "kernel_ms_calibration": round(breakdown[dom], 5),
                         "frac_calibration": round(alg / (breakdown[dom] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                         if breakdown[dom] > 0 else None,
                         "calibration_source": "kernels_ms: the untimed calibration pass before the timed region, "
                                               "every kernel bracketed on every run",
                         "traffic_source": traffic_src, "traffic_null_reason": traffic_null,
                         "algorithmic_bytes": int(alg),
                         "bytes_definition": "bytes the kernel moves, counted by K2 per candidate (pod records, "
                                             "F-row heads and full-row scans, 64-node record windows, outputs; "
                                             "SURVEY 8(d) K2 formula over what is actually read)",
                         "limiter": "latency: one dependent placement chain per candidate (one wave each); the "
                                    "longest chain sets the kernel time, not bytes (DESIGN.md 4)",
                         "chain": chain,
                         "latency": chain_latency(chain)},
        }
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"] = cpu_baseline(sc, nm, cand_off, cand_pods, int(len(nm.spot)), status[:len(loff) - 1],
                                                nodes_out[:len(lpods)], issued_local, args.cpu_seconds, mutation)
        print(json.dumps(line), flush=True)
    lib.sr_snapshot_destroy(snap)
    checker.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
