"""Multi-GPU tick prediction and the sharding choice.

The reference plans a tick's candidates one after another (rescheduler.go:
228-287); the planner shards them c % N over N GPUs, each holding the whole
spot snapshot, and reduces the tick's outcome either through one shared-memory
segment every rank's K2 writes its outcomes to (transport "shm", bench.py's
default on one node: no collective, no K3) or with one RCCL allreduce(min) of
three u64 words followed by K3 (transport "rccl").  A rank's device tick is K2
over its shard plus, for N > 1 over RCCL, the collective and K3:

    tick(N) = max(chain, K2_1 * share(N)) + gap + [N > 1, rccl] (allreduce(N) + K3)

  chain   the longest candidate's dependent placement chain (one wave: no
          number of GPUs shortens it);
  K2_1    K2 over the whole candidate set on one GPU (throughput part);
  share   1/N under strong scaling (the config's candidates split), 1 under
          weak scaling (every rank holds a config-sized candidate set);
  gap     launch and kernel-boundary time of a back-to-back tick beyond K2;
  K3      the winner kernel after the collective (one GPU: K2 writes the
          result itself, no K3).

Sharding a fixed tick pays only when tick_strong(N) < tick(1): K2 must be
throughput-bound well above its chain.  Since round 6's cooperative blocks
C4 is again: its longest wave is 26.3 us in a 43.8 us K2 (15,000 candidates),
so over the shared-memory transport a 2-GPU tick is predicted at ~30 us.  C3
(1,500 candidates) is a 12.2 us chain in a 14.2 us K2, C5 a 36 us chain in a
35 us K2: a strong-scaled tick on 2-8 GPUs is no faster than on one.
bench.py reports the strong-scaled line (BASELINE's) with the weak-scaled tick
beside it; `choose_scaling` says which of the two the model expects to pay.
"""

# Measured on one MI355X in round 6 (profiles/r06/final/c*_bench.json:
# kernels_ms.k2_placement = K2, ms_per_step - K2 = gap (>= 0);
# c*_k2_wave_profile.txt: the longest wave = chain).  K3 4.5 us.
# Microseconds.  C4's longest wave is 28.8 us since the cooperative blocks
# (48.6 us before), so its 44 us K2 is throughput-bound again.
PARTS = {
    1: dict(k2=8.5, chain=5.2, gap=5.4, k3=4.5),
    2: dict(k2=18.5, chain=17.2, gap=0.5, k3=4.5),
    3: dict(k2=14.2, chain=12.2, gap=1.7, k3=4.5),   # profiles/r06/default_bench_c3.json
    4: dict(k2=43.8, chain=26.3, gap=0.0, k3=4.5),   # profiles/r06/final/c4_* (list head 512)
    5: dict(k2=35.2, chain=36.0, gap=0.6, k3=4.5),
}

# The shared-memory transport's cost per tick beyond one GPU's: each host
# waits for every rank's outcome words and walks them in global order.
# Measured only as an upper bound: two ranks sharing one GPU
# (profiles/r06/n2_shm_rehearsal.log: ms_per_step_local - K2 = 4.1-6.8 us,
# both ranks' kernels on one device).  Microseconds.
SHM_US = 4.0

# RCCL allreduce of 24 B over xGMI, per rank count.  ASSUMED, not measured:
# no multi-GPU box was available to this build; RCCL's
# small-message latency on one node, of the order of its LL protocol's few
# hops per ring step.  bench.py reports the measured value per rank when it
# runs on N GPUs (per_rank[].collective_ms).
ALLREDUCE_US = {1: 0.0, 2: 8.0, 4: 12.0, 8: 20.0}


def allreduce_us(n):
    if n in ALLREDUCE_US:
        return ALLREDUCE_US[n]
    lo = max(k for k in ALLREDUCE_US if k <= n)
    return ALLREDUCE_US[lo] * (n / lo) ** 0.5


def predict_tick_us(parts, n, scaling, transport="rccl"):
    """Predicted back-to-back device tick of one rank, us (transport "shm": the
    ranks' hosts walk the shared outcome words, no collective and no K3)."""
    share = 1.0 / n if scaling == "strong" else 1.0
    k2 = max(parts["chain"], parts["k2"] * share)
    if n <= 1:
        return k2 + parts["gap"]
    return k2 + parts["gap"] + (allreduce_us(n) + parts["k3"] if transport == "rccl" else SHM_US)


def predict(config, n, transport="rccl"):
    """Per-N prediction for a config: both scalings, the strong tick's speed-up
    over one GPU, and the predicted scaling efficiencies the driver would
    compute from the bench values (weak: N x the work in tick(N); strong: the
    same work in tick(N))."""
    p = PARTS[config]
    t1 = predict_tick_us(p, 1, "strong")
    ts = predict_tick_us(p, n, "strong", transport)
    tw = predict_tick_us(p, n, "weak", transport)
    return {"n": n, "transport": transport, "tick1_us": round(t1, 2), "strong_tick_us": round(ts, 2),
            "weak_tick_us": round(tw, 2),
            "strong_efficiency": round(t1 / (n * ts), 3), "weak_efficiency": round(t1 / tw, 3),
            "strong_pays": ts < t1}


def choose_scaling(config, n, transport="shm"):
    """Shard the config's own tick (strong) where that shortens it, else give
    every rank a config-sized candidate set (weak)."""
    if n <= 1:
        return "strong", "one GPU"
    r = predict(config, n, transport)
    if r["strong_pays"]:
        return "strong", "predicted strong tick %.1f us < 1-GPU tick %.1f us" % (r["strong_tick_us"], r["tick1_us"])
    return "weak", ("predicted strong tick %.1f us >= 1-GPU tick %.1f us (K2 chain-bound: the longest candidate's "
                    "chain %.1f us of %.1f us): sharding the config's tick does not pay"
                    % (r["strong_tick_us"], r["tick1_us"], PARTS[config]["chain"], PARTS[config]["k2"]))
