// planner.cpp — device context, resident buffers and the planning tick.
//
// sr_ctx plays the role of the reference's predicate checker (created once,
// rescheduler.go:149).  One tick (sr_plan_run) is three kernels on a single
// HIP stream; K3 writes the result straight into mapped host memory:
//   K0 tables -> K2 placement -> [RCCL allreduce(min)] -> K3 winner
// There is no CPU path: without a HIP device sr_create fails.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "host.hpp"
#include "kernels.hpp"

#include <dlfcn.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

namespace {

// RCCL is loaded on first use (sr_comm_unique_id / sr_comm_init): a
// single-GPU planner never maps it.  The calls keep their rccl.h signatures.
struct Rccl {
  decltype(&ncclGetUniqueId) get_unique_id = nullptr;
  decltype(&ncclCommInitRank) comm_init_rank = nullptr;
  decltype(&ncclAllReduce) all_reduce = nullptr;
  decltype(&ncclCommDestroy) comm_destroy = nullptr;
  decltype(&ncclGetErrorString) error_string = nullptr;
  bool ok = false;
};

const Rccl& rccl() {
  static const Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) return x;
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(h, "ncclGetUniqueId"));
    x.comm_init_rank = reinterpret_cast<decltype(x.comm_init_rank)>(dlsym(h, "ncclCommInitRank"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(h, "ncclAllReduce"));
    x.comm_destroy = reinterpret_cast<decltype(x.comm_destroy)>(dlsym(h, "ncclCommDestroy"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(h, "ncclGetErrorString"));
    x.ok = x.get_unique_id && x.comm_init_rank && x.all_reduce && x.comm_destroy && x.error_string;
    return x;
  }();
  return r;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};

struct HostBuf {
  void* p = nullptr;
  size_t cap = 0;
};

// One workload slot: an encoded candidate input with its device arena and
// pinned staging copy.  sr_plan_first's prefix batches and an every-candidate
// plan are different inputs; with a slot each, a tick whose inputs equal the
// previous tick's reuses each one's candidate side (CandReuse) and its
// device-resident records instead of re-encoding and re-uploading them.
struct Slot {
  sr::Workload wl;
  DevBuf arena;
  HostBuf h_arena;
  uint64_t dev_state_gen = ~0ull;   // encoder state whose node records the device arena holds
  uint64_t host_state_gen = ~0ull;  // ... and the pinned staging arena
  uint64_t dev_cand_gen = ~0ull;    // candidate generation (Workload::cand_gen) the device arena holds (its
                                    //   pod records as of the last K0 run plus none of the pending patches)
  uint64_t host_cand_gen = ~0ull;   // ... and the staging arena (every patch applied)
  DevBuf tables;                    // S and T rows (K0 writes, K2 reads)
  uint64_t tables_cand_gen = ~0ull; // candidate generation, encoder state, thresholds and atoms of the last K0
  uint64_t tables_state_gen = ~0ull;  //   run on `tables` (incremental K0 / K0-less runs: what changed since)
  std::vector<int64_t> tables_thr;
  uint64_t tables_atoms_ver = ~0ull;   // Workload::atoms_ver of the last K0 run
  std::vector<int32_t> atom_cols;      // inter-pod / spread atom words changed since (reuse encodes)
  // atom rows changed since version atoms_log_ver (reuse encodes of one
  // candidate generation): the staging and device copies of an older version
  // that is atoms_log_ver take only those rows
  uint64_t atoms_log_ver = ~0ull, last_atoms_ver = ~0ull;
  std::vector<int32_t> atoms_log;
  uint64_t host_atoms_ver = ~0ull, dev_atoms_ver = ~0ull;
  // the work list by cost (sr_ctx::list_cost): the candidate generation whose
  // K2 durations were copied back (h_cycles, complete at ev_cost), and the one
  // the list was reordered for
  uint64_t cost_gen = ~0ull, list_sorted_gen = ~0ull;
  HostBuf h_cycles;
  hipEvent_t ev_cost = nullptr;
  // spot nodes changed since tables_state_gen (valid: every state step since was one the encoder patched)
  std::vector<int32_t> dirty;
  bool dirty_valid = false;
  uint64_t seen_gen = ~0ull;        // encoder state at the slot's last prepare
  std::vector<int32_t> pending;     // pods re-pointed since the last K0 run (their device records are older)
  std::vector<uint8_t> pending_mark;
  bool class_flip = false;          // ... some of them to or from the empty class
  // what the next K0 launch of this slot brings the tables and the node section to (run() commits it)
  bool commit_k0 = false;
  bool need_k0 = true;              // the device records name rows no K0 run has written yet
  uint64_t key = 0;                 // fingerprint of the input it was last prepared for
  uint64_t used = 0;                // clock of its last prepare (least recently used is replaced)
};

}  // namespace

struct sr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string err;
  DevBuf out_node, out_status, out_bytes, dmin, prof, scratch;
  HostBuf h_result, h_status, h_node, h_bytes;
  HostBuf h_early;           // mapped: K2's per-candidate result words (single-rank runs)
  HostBuf h_comm;            // pinned: the reduced words of a caller-provided collective
  bool in_flight = false;    // a run returned with K2 still planning candidates past the winner
  uint64_t* d_early = nullptr;  // device address of h_early
  uint64_t issued_checks = 0;  // checks of the prepared workload's plan (known after a full run)
  bool issued_known = false;
  std::vector<std::unique_ptr<Slot>> slots;  // SR_PLAN_SLOTS (default 4), made on first use
  int32_t n_slots = 4;
  Slot* cur = nullptr;       // the slot of the last prepare
  uint64_t slot_clock = 0;
  std::vector<uint64_t> node_patch_words;  // this call's node patches (prepare)
  std::vector<int32_t> k0_cols, k0_rows;   // this call's incremental K0 (prepare)
  std::vector<uint64_t> pod_patch_words;   // this call's pod patches (prepare)
  int32_t k0_incremental = 1;  // SR_K0_INCREMENTAL=0: K0 always rewrites every row
  int32_t k0_skip = 1;         // SR_K0_SKIP=0: every run launches K0
  // SR_K2_SPLIT=0: one K2 launch.  Otherwise a work list the encoder split
  // (more entries than SR_K2_SPLIT_MIN, 4096: more waves than the chip holds
  // at once, with domain-path candidates) is planned by two kernels side by
  // side: the node-order candidates on the node-order kernel (fewer
  // registers, several waves per SIMD), the rest on the general kernel on a
  // second stream (C4's affinity variant, 15,000 entries: K2 142 -> 89 us; C3's,
  // 1,500, split too: 20 -> 39 us)
  int32_t k2_split = 1;
  // SR_LIST_COST=0: the work list stays longest-first by pod count.  Otherwise
  // the first run of a candidate generation records each candidate's K2 wave
  // duration, and the reused workloads of the next ticks dispatch the longest
  // waves first (a candidate whose pods scan far along their rows is short by
  // pod count but one of the longest waves: C4's last-starting waves)
  int32_t list_cost = 1;
  int32_t list_cost_min = 1024;  // SR_LIST_COST_MIN: only lists longer than this (C4 15,000 entries: K2 69 -> 45 us;
                                 // round 6, C3's 1,500: K2 -0.3 us, realistic C3 -0.7 us, affinity C3 16.3 -> 13.3 us;
                                 // C1 / C2 / C5's 300 entries keep the pod-count order)
  // SR_K2_COOP: a cost-ordered list's costliest entries planned by cooperative
  // blocks on the node-order kernel (four waves per block: the chain and
  // three waves scanning far resolutions with it); 0: none
  int32_t k2_coop = 64;
  // SR_K2_DISPATCH_EVENTS=0: the split launch's fork and join as marker
  // packets (hipEventRecord) instead of the completion signals of K0 and of
  // the general kernel's dispatch
  int32_t k2_dispatch_events = 1;
  DevBuf out_cycles;
  hipStream_t stream2 = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  uint64_t run_count = 0;      // runs of this context: d_min alternates between two buffers
  bool dmin_ready[2] = {false, false};  // buffer reset by the previous run's K2 (a K0-less run needs it)
  sr::EncoderCache enc;      // what the encoder keeps across calls (encode.cpp)
  hipEvent_t ev_upload = nullptr;  // the last upload (a staging buffer is reused after it)
  int32_t prefix_batch = 16;       // first batch of sr_plan_first (SR_PREFIX_BATCH; tools/gpu_prefix.sh)
  sr::DevWorkload dw{};
  bool prepared = false;
  int32_t timing = 0;        // SR_TIME_* kernel bits of the current setting
  int32_t timing_every = 1;  // sample every n-th run
  int64_t timing_runs = 0;   // runs since sr_set_timing
  int32_t timing_cur = 0;    // SR_TIME_* bits of the current run
  // HIP event pairs bracketing timed kernels, read back lazily (flush_timing)
  // so a timed run does not have to synchronise the stream.
  std::vector<hipEvent_t> ev_start, ev_end;
  std::vector<int8_t> ev_kernel;
  size_t ev_used = 0;
  uint32_t seq = 0;  // run sequence number (wraps: tags compare as uint32)
  sr_timing t{};
  ncclComm_t comm = nullptr;
  // sr_comm_init_shm: the ranks of one node reduce through host memory.  One
  // POSIX shared-memory segment holds, per rank and per tick parity, the
  // rank's published input words and the outcome words its K2 writes (mapped
  // into every rank's GPU); each rank's host walks them in global candidate
  // order up to the first drainable one (no collective, no K3: DESIGN.md §7).
  struct Shm {
    uint64_t* host = nullptr;  // the segment (every rank's regions)
    uint64_t* dev = nullptr;   // its device address in this process
    size_t bytes = 0;
    int32_t max_cand = 0;      // input candidates per rank and call
    uint32_t session = 0;
    uint64_t tick = 0;         // runs through the segment (identical on every rank)
    int32_t base = -1;         // the prepared call's first local candidate (cand_global[0] / nranks), -1: none
    std::string name;
    std::vector<int32_t> act_of;  // scratch: active candidate of each input candidate
  } shm;
  sr_allreduce_min_fn host_fn = nullptr;  // sr_comm_init_host: the caller's allreduce(min)
  void* host_user = nullptr;
  int nranks = 1, rank = 0;
  int64_t last_rank_next = -1;  // reduced smallest unplanned global index of the last collective run (-1: none)
  FILE* prof_file = nullptr;  // SR_K2_PROFILE: per-wave K2 records appended per run
  int32_t k2_mode = 0;        // SR_K2_MODE=1: pod-order K2 only (A/B measurement)
  int32_t node_patch = 1;     // SR_NODE_PATCH=0: a changed node section always goes up whole
  int32_t k2_narrow = 1;      // SR_K2_NARROW: 32-bit scaled window visits in node order (0: 64-bit only)
  int32_t k2_wpb = 0;         // SR_K2_WPB: K2 waves per block (1, 2, 4; 0 = by list length)
  int32_t k2_excl = 1;        // SR_K2_EXCL: exclusive candidates (one host port) with the taken-mask step
  int32_t k2_node_kernel = 1; // SR_K2_NODE_KERNEL: node-order-only K2 kernel when every candidate takes that path
  int32_t s_head_only = 1;    // SR_S_HEAD_ONLY: K0 writes S-row heads only on rows wider than 64 words (0: never)
};

namespace {

sr_status hip_fail(sr_ctx* ctx, hipError_t e, const char* what) {
  ctx->err = std::string(what) + ": " + hipGetErrorString(e);
  return SR_ERR_HIP;
}

#define HIP_TRY(ctx, expr)                                  \
  do {                                                      \
    hipError_t _e = (expr);                                 \
    if (_e != hipSuccess) return hip_fail((ctx), _e, #expr); \
  } while (0)

hipError_t dev_reserve(DevBuf& b, size_t bytes) {
  if (bytes <= b.cap) return hipSuccess;
  if (b.p) (void)hipFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max<size_t>(bytes + bytes / 4, 4096);
  hipError_t e = hipMalloc(&b.p, cap);
  if (e == hipSuccess) b.cap = cap;
  return e;
}

// Fresh pinned blocks are zeroed: the runtime may hand back memory an earlier
// context freed, and the tagged result words (mapped memory) must never carry
// a stale tag (run sequence numbers also come from one process-wide counter).
hipError_t host_reserve(HostBuf& b, size_t bytes) {
  if (bytes <= b.cap) return hipSuccess;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t cap = std::max<size_t>(bytes + bytes / 4, 4096);
  hipError_t e = hipHostMalloc(&b.p, cap, hipHostMallocMapped | hipHostMallocCoherent);
  if (e == hipSuccess) {
    b.cap = cap;
    std::memset(b.p, 0, cap);
  }
  return e;
}

// Run tags of every context of the process: a tag is never reused while the
// process lives (2^32 runs), so words a freed context left behind cannot match.
std::atomic<uint32_t> g_run_seq{0};

// Packs host vectors into one contiguous staging buffer (256-B aligned
// sections) so the whole workload goes up in a single copy.
class Packer {
 public:
  template <class T>
  size_t add(const std::vector<T>& v) {
    size_t off = (size_ + 255) & ~size_t(255);
    items_.push_back({off, v.data(), v.size() * sizeof(T)});
    size_ = off + v.size() * sizeof(T);
    return off;
  }
  size_t size() const { return (size_ + 255) & ~size_t(255); }
  void copy_to(char* dst, size_t from = 0) const {  // the sections at or after `from`
    for (const auto& it : items_)
      if (it.bytes && it.off >= from) std::memcpy(dst + it.off, it.src, it.bytes);
  }

 private:
  struct Item {
    size_t off;
    const void* src;
    size_t bytes;
  };
  std::vector<Item> items_;
  size_t size_ = 0;
};

// A run may return while K2 still plans the candidates after the winner (the
// stream keeps later work in order); host-side reallocation of its buffers
// waits for it here.
sr_status settle(sr_ctx* ctx) {
  if (!ctx->in_flight) return SR_OK;
  ctx->in_flight = false;
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  return SR_OK;
}

bool has_comm(const sr_ctx* ctx) { return ctx->comm != nullptr || ctx->host_fn != nullptr || ctx->shm.host != nullptr; }

// ---- the shared-memory transport (sr_comm_init_shm).  Per rank r and tick
// parity p a region of kShmHdr + 2 * max_cand words, each word tag << 32 |
// value (tag: the run's, identical on every rank):
//   hdr[0] input candidates of the call   hdr[1] its first local index + 1 (0: none)
//   hdr[2] first fallback (global) + 1    hdr[3] 1: the rank has finished this tick's walk
//   hdr[4] smallest global index the rank has not planned after this call + 1 (0: none)
//   in[i]  input candidate i: active candidate << 2 | 0, or 1 (no pods), 2 (fallback)
//   st[ci] written by K2: active candidate ci is drainable (1) or not (0)
constexpr size_t kShmHdr = 8;
size_t shm_region_words(const sr_ctx* ctx) { return kShmHdr + 2 * static_cast<size_t>(ctx->shm.max_cand); }
uint64_t* shm_region(sr_ctx* ctx, int32_t r, int p) {
  return ctx->shm.host + (static_cast<size_t>(r) * 2 + static_cast<size_t>(p)) * shm_region_words(ctx);
}
// tags of the shared words: the high bit set, so they never equal a
// single-rank run's (g_run_seq) in the context's private result words
uint32_t shm_tag(const sr_ctx* ctx, uint64_t tick) {
  return (ctx->shm.session + static_cast<uint32_t>(tick)) | 0x80000000u;
}

// Spins until ready().  A word of this rank's own K2 that has not arrived
// after 100 ms is waited for on the stream (which surfaces a kernel fault);
// another rank's after 60 s fails the run (that rank stopped planning).
template <class F>
sr_status shm_wait(sr_ctx* ctx, F ready, bool own, int32_t r) {
  if (ready()) return SR_OK;
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  bool synced = false;
  while (!ready()) {
    if ((++spins & 1023) != 0) continue;
    const auto dt = std::chrono::steady_clock::now() - t0;
    if (own && !synced && dt > std::chrono::milliseconds(100)) {
      HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
      synced = true;
      if (!ready()) {
        ctx->err = "K2 outcome word not written by this run";
        return SR_ERR_HIP;
      }
    } else if (!own && dt > std::chrono::seconds(60)) {
      ctx->err = "rank " + std::to_string(r) + " published no outcome for this tick within 60 s";
      return SR_ERR_RCCL;
    }
  }
  return SR_OK;
}

// Before K2: this rank's input words and header for the run's tick, into the
// region of the tick's parity once every rank has finished walking the tick
// that used it before; K2 then writes the outcome words there.
sr_status shm_publish(sr_ctx* ctx, int* par) {
  auto& S = ctx->shm;
  sr::DevWorkload& d = ctx->dw;
  const sr::Workload& w = ctx->cur->wl;
  const uint64_t tick = ++S.tick;
  const int p = static_cast<int>(tick & 1);
  if (tick > 2) {
    const uint64_t done = static_cast<uint64_t>(shm_tag(ctx, tick - 2)) << 32 | 1u;
    for (int32_t r = 0; r < ctx->nranks; ++r) {
      volatile uint64_t* hd = shm_region(ctx, r, p);
      sr_status st = shm_wait(ctx, [&] { return hd[3] == done; }, false, r);
      if (st != SR_OK) return st;
    }
  }
  const uint32_t tag = shm_tag(ctx, tick);
  ctx->seq = tag;
  d.seq = tag;
  const uint64_t T = static_cast<uint64_t>(tag) << 32;
  volatile uint64_t* reg = shm_region(ctx, ctx->rank, p);
  const int32_t n_in = w.n_input_cand;
  S.act_of.assign(static_cast<size_t>(std::max(0, n_in)), -1);
  for (int32_t ci = 0; ci < static_cast<int32_t>(w.cand_src.size()); ++ci) S.act_of[w.cand_src[ci]] = ci;
  for (int32_t i = 0; i < n_in; ++i) {
    const int32_t a = S.act_of[i];
    reg[kShmHdr + i] = T | static_cast<uint32_t>(a >= 0 ? a << 2 : w.status_host[i] == SR_CAND_FALLBACK ? 2 : 1);
  }
  std::atomic_thread_fence(std::memory_order_release);
  reg[0] = T | static_cast<uint32_t>(n_in);
  reg[1] = T | static_cast<uint32_t>(n_in > 0 ? S.base + 1 : 0);
  reg[2] = T | static_cast<uint32_t>(w.first_fallback + 1);
  reg[4] = T | static_cast<uint32_t>(d.rank_next == ~0ull ? 0 : d.rank_next + 1);
  d.res_stat = S.dev + (const_cast<uint64_t*>(reg) - S.host) + kShmHdr + S.max_cand;
  d.res_map = ctx->d_early + d.n_cand;
  *par = p;
  return SR_OK;
}

// After K2: the walk in global candidate order over every rank's words (rank
// g % N holds global index g), up to the first drainable candidate or the
// first index no rank planned in this call; the result words are written as
// K3 would (`result`, tagged), the owner's mapping from its K2 (rescheduler.go:
// 280-286 stops at the first drainable candidate, whichever rank planned it).
sr_status shm_reduce(sr_ctx* ctx, int p) {
  auto& S = ctx->shm;
  const sr::Workload& w = ctx->cur->wl;
  const uint32_t tag = ctx->dw.seq;
  const int32_t N = ctx->nranks;
  auto ready = [tag](volatile uint64_t* x) { return static_cast<uint32_t>(*x >> 32) == tag; };
  std::vector<int64_t> n_r(static_cast<size_t>(N)), b_r(static_cast<size_t>(N));
  int64_t ff = -1, nx = -1, g0 = INT64_MAX;
  for (int32_t r = 0; r < N; ++r) {
    volatile uint64_t* hd = shm_region(ctx, r, p);
    for (int i : {0, 1, 2, 4}) {
      sr_status st = shm_wait(ctx, [&] { return ready(hd + i); }, false, r);
      if (st != SR_OK) return st;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    n_r[r] = static_cast<uint32_t>(hd[0]);
    b_r[r] = static_cast<int64_t>(static_cast<uint32_t>(hd[1])) - 1;
    if (n_r[r] > 0) g0 = std::min(g0, b_r[r] * N + r);
    const int64_t f = static_cast<int64_t>(static_cast<uint32_t>(hd[2])) - 1;
    if (f >= 0) ff = ff < 0 ? f : std::min(ff, f);
    const int64_t x = static_cast<int64_t>(static_cast<uint32_t>(hd[4])) - 1;
    if (x >= 0) nx = nx < 0 ? x : std::min(nx, x);
  }
  int64_t first_ok = -1;
  int32_t owner = -1, oci = -1;
  for (int64_t g = g0; g0 != INT64_MAX; ++g) {
    const int32_t r = static_cast<int32_t>(g % N);
    const int64_t li = g / N;
    if (n_r[r] == 0 || li < b_r[r] || li >= b_r[r] + n_r[r]) break;  // no rank planned g in this call
    volatile uint64_t* reg = shm_region(ctx, r, p);
    volatile uint64_t* in = reg + kShmHdr + (li - b_r[r]);
    sr_status st = shm_wait(ctx, [&] { return ready(in); }, false, r);
    if (st != SR_OK) return st;
    const uint32_t v = static_cast<uint32_t>(*in);
    if ((v & 3u) != 0) continue;  // no pods to move, or the reference path
    const int32_t ci = static_cast<int32_t>(v >> 2);
    volatile uint64_t* sw = reg + kShmHdr + S.max_cand + ci;
    st = shm_wait(ctx, [&] { return ready(sw); }, r == ctx->rank, r);
    if (st != SR_OK) return st;
    if (static_cast<uint32_t>(*sw) & 1u) {
      first_ok = g;
      owner = r;
      oci = ci;
      break;
    }
  }
  shm_region(ctx, ctx->rank, p)[3] = static_cast<uint64_t>(tag) << 32 | 1u;  // this tick's words may be reused
  volatile uint64_t* res = static_cast<volatile uint64_t*>(ctx->h_result.p);
  const uint64_t T = static_cast<uint64_t>(tag) << 32;
  int32_t np = 0;
  if (owner == ctx->rank) {
    const int32_t off = w.cand_off[oci];
    np = w.cand_off[oci + 1] - off;
    volatile uint64_t* map = static_cast<volatile uint64_t*>(ctx->h_early.p) + ctx->dw.n_cand + off;
    for (int32_t q = 0; q < np; ++q) {
      sr_status st = shm_wait(ctx, [&] { return ready(map + q); }, true, ctx->rank);
      if (st != SR_OK) return st;
      res[sr::kResultHeader + q] = T | static_cast<uint32_t>(map[q]);
    }
  }
  res[0] = T | static_cast<uint32_t>(first_ok);
  res[1] = T | (owner == ctx->rank ? 1u : 0u);
  res[2] = T | static_cast<uint32_t>(np);
  res[3] = T | static_cast<uint32_t>(ff);
  res[4] = T | static_cast<uint32_t>(nx);
  return SR_OK;
}

// allreduce(min) of n <= 8 uint64 words in device memory, stream-ordered:
// RCCL in place, or the caller's collective on a pinned host copy.
sr_status allreduce_min_dev(sr_ctx* ctx, void* words, int32_t n) {
  if (ctx->comm) {
    ncclResult_t r = rccl().all_reduce(words, words, static_cast<size_t>(n), ncclUint64, ncclMin, ctx->comm,
                                       ctx->stream);
    if (r != ncclSuccess) {
      ctx->err = std::string("ncclAllReduce: ") + rccl().error_string(r);
      return SR_ERR_RCCL;
    }
    return SR_OK;
  }
  HIP_TRY(ctx, host_reserve(ctx->h_comm, 64));
  uint64_t* h = static_cast<uint64_t*>(ctx->h_comm.p);
  HIP_TRY(ctx, hipMemcpyAsync(h, words, sizeof(uint64_t) * n, hipMemcpyDeviceToHost, ctx->stream));
  HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
  if (ctx->host_fn(ctx->host_user, h, n) != 0) {
    ctx->err = "caller-provided allreduce(min) failed";
    return SR_ERR_RCCL;
  }
  HIP_TRY(ctx, hipMemcpyAsync(words, h, sizeof(uint64_t) * n, hipMemcpyHostToDevice, ctx->stream));
  return SR_OK;
}

// The slot for this input: the one last prepared for an input with the same
// fingerprint (the encoder then compares the input in full), else a new one
// while fewer than n_slots exist, else the least recently used.
Slot& pick_slot(sr_ctx* ctx, const sr_candidates* cands) {
  const int32_t n = cands->n_cand;
  uint64_t key = 0x5107ull + static_cast<uint64_t>(n);
  if (n > 0) {
    const int32_t b = cands->cand_pod_off[0], e = cands->cand_pod_off[n];
    auto mixin = [&](uint64_t x) { key = (key ^ x) * 0x100000001B3ull; };
    mixin(static_cast<uint32_t>(b));
    mixin(static_cast<uint32_t>(e));
    if (e > b) {
      mixin(static_cast<uint32_t>(cands->cand_pods[b]));
      mixin(static_cast<uint32_t>(cands->cand_pods[b + (e - b) / 2]));
      mixin(static_cast<uint32_t>(cands->cand_pods[e - 1]));
    }
    if (cands->cand_global) {
      mixin(static_cast<uint32_t>(cands->cand_global[0]));
      mixin(static_cast<uint32_t>(cands->cand_global[n - 1]));
    }
  }
  Slot* pick = nullptr;
  for (auto& sl : ctx->slots)
    if (sl->key == key) pick = sl.get();
  if (!pick && static_cast<int32_t>(ctx->slots.size()) < ctx->n_slots) {
    ctx->slots.push_back(std::make_unique<Slot>());
    pick = ctx->slots.back().get();
  }
  if (!pick) {
    pick = ctx->slots.front().get();
    for (auto& sl : ctx->slots)
      if (sl->used < pick->used) pick = sl.get();
  }
  pick->key = key;
  pick->used = ++ctx->slot_clock;
  return *pick;
}

sr_status prepare(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands) {
  auto t0 = std::chrono::steady_clock::now();
  ctx->prepared = false;
  if (ctx->shm.host) {  // the walk finds global index g on rank g % N: interleaved shards only
    const int32_t n = cands->n_cand, N = ctx->nranks;
    if (n > ctx->shm.max_cand) {
      ctx->err = "more candidates than sr_comm_init_shm's max_cand";
      return SR_ERR_CAPACITY;
    }
    const int32_t* G = cands->cand_global;
    if (n > 0 && !G && N > 1) {
      ctx->err = "the shared-memory transport needs cand_global (interleaved shards)";
      return SR_ERR_INVALID_ARG;
    }
    const int64_t b = n > 0 && G ? G[0] / N : 0;
    for (int32_t i = 0; i < n; ++i)
      if ((G ? G[i] : i) != (b + i) * N + ctx->rank) {
        ctx->err = "the shared-memory transport needs interleaved shards: cand_global[i] = (first + i) * nranks + rank";
        return SR_ERR_INVALID_ARG;
      }
    ctx->shm.base = n > 0 ? static_cast<int32_t>(b) : -1;
  }
  Slot& sl = pick_slot(ctx, cands);
  ctx->cur = &sl;
  sr::Workload& w = sl.wl;
  std::string err;
  sr_status st = sr::encode_workload(&ctx->enc, snap, c, cands, &w, &err);
  if (st != SR_OK) {
    ctx->err = err;
    sl.dev_state_gen = ~0ull;  // the encoder may have moved on: upload the node records again
    return st;
  }
  const int32_t na = static_cast<int32_t>(w.pod_src.size());
  const int32_t ncand = static_cast<int32_t>(w.cand_global.size());
  // Arena: the spot nodes' records and free values first (uploaded only when
  // the encoder's state view changed), then this call's sections.
  const sr::EncoderCache& E = ctx->enc;
  // Arena: the node section (spot nodes' records and free values), the
  // candidate section (class programs, pod records, candidate lists, domain
  // path and extension records: one candidate generation, w.cand_gen), then
  // this call's tick section (atoms, thresholds, patches).  Sections the
  // device already holds are not copied again.
  Packer pk;
  const size_t o_nr = pk.add(E.node_rec);
  const size_t o_nf = pk.add(E.node_free);
  const size_t node_bytes = pk.size();
  const size_t o_cpo = pk.add(w.cls_prog_off), o_cp = pk.add(w.cls_prog), o_cp8 = pk.add(w.cls_prog8);
  const size_t o_prec = pk.add(w.pod_rec);
  const size_t o_co = pk.add(w.cand_off), o_cg = pk.add(w.cand_global);
  const size_t o_ls = pk.add(w.list);
  const bool dyn = !w.dyn_cand.empty();
  const size_t o_dc = dyn ? pk.add(w.dyn_cand) : 0, o_dp = dyn ? pk.add(w.dyn_pod) : 0;
  const size_t o_di = dyn ? pk.add(w.ds_info) : 0;
  const bool ext = !w.ext_cand.empty();
  const size_t o_ec = ext ? pk.add(w.ext_cand) : 0, o_ep = ext ? pk.add(w.pod_ext) : 0;
  const size_t o_le = ext ? pk.add(w.list_ext) : 0;
  // the tick section: the atoms (rows a reuse encode changed go up alone),
  // then what follows the spot nodes' state every tick
  const size_t o_at = pk.add(w.atoms);
  const size_t tick_rest = pk.size();
  const size_t o_ns = ext ? pk.add(w.node_scal) : 0;  // the spot nodes' scalar usage
  const size_t o_st = dyn ? pk.add(w.sp_tab) : 0;     // the domain path's base counts
  const size_t o_dd = dyn ? pk.add(w.dk_dom) : 0;     // ... and node domains (the spot order may move)
  const size_t o_tt = pk.add(w.t_thr);
  // the atom-row log (see Slot)
  if (w.atoms_ver != sl.last_atoms_ver) {
    const bool follows = w.reused && !w.atom_rows_all && w.atoms_prev_ver == sl.last_atoms_ver;
    if (follows && sl.atoms_log_ver != ~0ull) {
      sl.atoms_log.insert(sl.atoms_log.end(), w.atom_rows.begin(), w.atom_rows.end());
    } else if (follows) {
      sl.atoms_log_ver = sl.last_atoms_ver;
      sl.atoms_log = w.atom_rows;
    } else {
      sl.atoms_log_ver = ~0ull;
      sl.atoms_log.clear();
    }
    if (sl.atoms_log.size() > 256) {
      sl.atoms_log_ver = ~0ull;
      sl.atoms_log.clear();
    }
    sl.last_atoms_ver = w.atoms_ver;
  }
  if (!w.reused || sl.dev_cand_gen != w.cand_gen) sl.atom_cols.clear();
  else sl.atom_cols.insert(sl.atom_cols.end(), w.atom_cols.begin(), w.atom_cols.end());
  // ---- the slot's device state against this call.  Spot nodes changed since
  // the slot's tables were written, accumulated over K0-less runs:
  if (w.state_gen != sl.seen_gen) {
    if (sl.dirty_valid && E.patched_from != ~0ull && E.patched_from == sl.seen_gen && E.state_gen == w.state_gen) {
      for (int32_t i : E.patched_nodes)
        if (std::find(sl.dirty.begin(), sl.dirty.end(), i) == sl.dirty.end()) sl.dirty.push_back(i);
    } else {
      sl.dirty_valid = false;
    }
    sl.seen_gen = w.state_gen;
  }
  constexpr size_t kDirtyMax = 64;
  if (sl.dirty.size() > kDirtyMax) sl.dirty_valid = false;
  // pods the encoder re-pointed since the last K0 run of this candidate generation
  if (!w.reused || sl.dev_cand_gen != w.cand_gen) {
    sl.pending.clear();
    sl.pending_mark.assign(static_cast<size_t>(na), 0);
    sl.class_flip = false;
  } else {
    if (sl.pending_mark.size() != static_cast<size_t>(na)) sl.pending_mark.assign(static_cast<size_t>(na), 0);
    for (size_t i = 0; i < w.pod_patch.size(); i += sr::kPodPatchWords) {
      const int32_t q = static_cast<int32_t>(w.pod_patch[i]);
      if (!sl.pending_mark[q]) {
        sl.pending_mark[q] = 1;
        sl.pending.push_back(q);
      }
    }
    sl.class_flip = sl.class_flip || w.class_flip;
  }
  const bool tables_cur = w.reused && sl.tables_cand_gen == w.cand_gen && sl.dev_cand_gen == w.cand_gen &&
                          sl.tables_thr.size() == w.t_thr.size() && sl.dirty_valid;
  // A K0-less run: the tables stand for every node but the changed ones, whose
  // records and T bits K2 takes from the node patches; the atoms (S rows) must
  // be the tables' and no pod may have left the empty class (K2's dead-pod
  // shortcut reads the device records).  Node-order candidates only.
  constexpr size_t kSkipDirty = 16;
  const bool k0_skip = ctx->k0_skip && ncand > 0 && tables_cur && sl.dirty.size() <= kSkipDirty && !sl.class_flip &&
                       w.dyn_cand.empty() && w.max_cand_pods <= 256 && ctx->k2_mode == 0 &&
                       sl.tables_atoms_ver == w.atoms_ver;
  // node patches {node, node_rec[8], node_free[3]}: the changed nodes' records
  // ride in the call's copy; K0 writes them into the node section (or K2 reads
  // them, K0-less)
  constexpr size_t kPatchNodes = 16;
  std::vector<uint64_t>& patch = ctx->node_patch_words;
  patch.clear();
  if (sl.dirty_valid && !sl.dirty.empty() && sl.dirty.size() <= kPatchNodes) {  // a superset of the nodes the
                                                                                 // device section lacks
    const size_t NP = static_cast<size_t>(w.n_pad);
    for (int32_t i : sl.dirty) {
      patch.push_back(static_cast<uint64_t>(i));
      for (size_t j = 0; j < 8; ++j) patch.push_back(E.node_rec[static_cast<size_t>(i) * 8 + j]);
      for (size_t dm = 0; dm < 3; ++dm) patch.push_back(static_cast<uint64_t>(E.node_free[dm * NP + i]));
    }
  }
  const size_t o_np = patch.empty() ? 0 : pk.add(patch);
  // pod patches of a K0 run: every pod re-pointed since the last one
  std::vector<uint64_t>& ppatch = ctx->pod_patch_words;
  ppatch.clear();
  if (w.reused && sl.dev_cand_gen == w.cand_gen)  // (unused if the run turns out K0-less)
    for (int32_t q : sl.pending)
      ppatch.insert(ppatch.end(), {static_cast<uint64_t>(q), w.pod_rec[static_cast<size_t>(q) * 6 + 4],
                                   w.pod_rec[static_cast<size_t>(q) * 6 + 5]});
  const size_t o_pp = ppatch.empty() ? 0 : pk.add(ppatch);
  // Incremental K0: the tables hold this candidate generation: the word
  // columns of the changed nodes and the T rows whose threshold moved are
  // rewritten; anything else rewrites every row.
  std::vector<int32_t>& kcols = ctx->k0_cols;
  std::vector<int32_t>& krows = ctx->k0_rows;
  kcols.clear();
  krows.clear();
  bool k0_inc = ctx->k0_incremental && tables_cur;  // (unused if the run turns out K0-less)
  if (k0_inc) {
    for (int32_t i : sl.dirty) kcols.push_back(i >> 6);
    kcols.insert(kcols.end(), sl.atom_cols.begin(), sl.atom_cols.end());
    std::sort(kcols.begin(), kcols.end());
    kcols.erase(std::unique(kcols.begin(), kcols.end()), kcols.end());
    for (size_t r = 0; r < w.t_thr.size(); ++r)
      if (w.t_thr[r] != sl.tables_thr[r] && w.t_thr[r] != sr::kTSpare) krows.push_back(static_cast<int32_t>(r));
    if (kcols.size() > 32 || krows.size() > 256) k0_inc = false;
  }
  if (!k0_inc) kcols.clear(), krows.clear();
  const size_t o_kc = kcols.empty() ? 0 : pk.add(kcols), o_kr = krows.empty() ? 0 : pk.add(krows);
  const size_t bytes = pk.size();

  HIP_TRY(ctx, hipSetDevice(ctx->device));
  st = settle(ctx);
  if (st != SR_OK) return st;
  // a reused workload's list in the order of its last run's K2 durations
  // (list_sorted_gen is set once the reordered list's copies are queued: a
  // prepare failing in between reorders and uploads it again next time)
  bool list_moved = false;
  if (ctx->list_cost && w.reused && sl.cost_gen == w.cand_gen && sl.list_sorted_gen != w.cand_gen) {
    HIP_TRY(ctx, hipEventSynchronize(sl.ev_cost));
    sr::reorder_list_by_cost(w, static_cast<const uint32_t*>(sl.h_cycles.p), ctx->enc.list_head, ctx->k2_coop);
    list_moved = true;
  }
  if (ctx->ev_upload) HIP_TRY(ctx, hipEventSynchronize(ctx->ev_upload));  // staging buffer free again
  const size_t h_cap = sl.h_arena.cap;
  HIP_TRY(ctx, host_reserve(sl.h_arena, bytes));
  if (sl.h_arena.cap != h_cap) sl.host_state_gen = sl.host_cand_gen = sl.host_atoms_ver = ~0ull;  // holds none
  const size_t arena_cap = sl.arena.cap;
  HIP_TRY(ctx, dev_reserve(sl.arena, bytes));  // a new allocation holds no node records
  const bool same_arena = sl.arena.cap == arena_cap;
  if (!same_arena) sl.dev_atoms_ver = ~0ull;
  const bool nodes_resident = same_arena && sl.dev_state_gen == w.state_gen;
  // a reuse encode's candidate section is on the device: K0 re-points the
  // records that moved (a K0-less run reads them as they are)
  const bool cand_resident = w.reused && same_arena && sl.dev_cand_gen == w.cand_gen;
  bool skip = k0_skip && cand_resident && same_arena && !sl.need_k0;
  // a few nodes changed since the generation on the device: K0 applies their
  // records from this call's copy (K0-less: K2 reads them there)
  const bool nodes_patch = !nodes_resident && same_arena && !patch.empty() && ctx->node_patch;
  const size_t n_rows = static_cast<size_t>(w.n_classes) + w.t_dim.size();
  const size_t row_bytes = static_cast<size_t>(w.Wp) * sizeof(uint64_t);
  const size_t t_cap = sl.tables.cap;
  HIP_TRY(ctx, dev_reserve(sl.tables, n_rows * row_bytes));
  if (sl.tables.cap != t_cap) {  // a new allocation holds no rows: every row below
    sl.tables_cand_gen = ~0ull;
    skip = false;
    k0_inc = false;
    kcols.clear();
    krows.clear();
  }
  HIP_TRY(ctx, dev_reserve(ctx->out_node, sizeof(int32_t) * std::max(1, na)));
  HIP_TRY(ctx, dev_reserve(ctx->out_status, sizeof(int32_t) * std::max(1, ncand)));
  HIP_TRY(ctx, dev_reserve(ctx->out_bytes, sizeof(uint32_t) * std::max(1, ncand)));
  HIP_TRY(ctx, dev_reserve(ctx->dmin, 64));
  const size_t res_bytes = sizeof(uint64_t) * (sr::kResultHeader + static_cast<size_t>(std::max(1, w.max_cand_pods)));
  HIP_TRY(ctx, host_reserve(ctx->h_result, res_bytes));  // mapped: K3 writes the result straight to the host
  HIP_TRY(ctx, host_reserve(ctx->h_early, sizeof(uint64_t) * (static_cast<size_t>(ncand) + na + 1)));
  auto t1 = std::chrono::steady_clock::now();
  const size_t from = nodes_resident || nodes_patch ? node_bytes : 0;
  // The staging arena keeps the node section of the generation it last held:
  // when that is the current one, or the one the encoder patched a few nodes
  // on, only those nodes' records are rewritten (no copy of the whole section).
  {
    char* hs = static_cast<char*>(sl.h_arena.p);
    const size_t NP = static_cast<size_t>(w.n_pad);
    if (sl.host_state_gen == w.state_gen) {
      // current
    } else if (E.patched_from != ~0ull && sl.host_state_gen == E.patched_from && E.state_gen == w.state_gen &&
               !E.patched_nodes.empty()) {
      for (int32_t i : E.patched_nodes) {
        std::memcpy(hs + o_nr + static_cast<size_t>(i) * 64, &E.node_rec[static_cast<size_t>(i) * 8], 64);
        for (size_t dm = 0; dm < 3; ++dm)
          std::memcpy(hs + o_nf + (dm * NP + static_cast<size_t>(i)) * 8, &E.node_free[dm * NP + i], 8);
      }
    } else {
      std::memcpy(hs + o_nr, E.node_rec.data(), E.node_rec.size() * sizeof(uint64_t));
      std::memcpy(hs + o_nf, E.node_free.data(), E.node_free.size() * sizeof(int64_t));
    }
    sl.host_state_gen = w.state_gen;
  }
  // the candidate section: kept in staging across a reuse encode (its pod
  // patches applied there too), packed again otherwise
  char* hs = static_cast<char*>(sl.h_arena.p);
  const size_t row_bytes8 = static_cast<size_t>(w.Wp) * sizeof(uint64_t);
  auto log_rows = [&](uint64_t have) {  // the rows a copy of version `have` lacks (null: every row)
    return have == w.atoms_ver ? &sl.atoms_log  // (unused)
           : sl.atoms_log_ver != ~0ull && have == sl.atoms_log_ver ? &sl.atoms_log : nullptr;
  };
  if (w.reused && sl.host_cand_gen == w.cand_gen) {
    for (size_t i = 0; i < w.pod_patch.size(); i += sr::kPodPatchWords)
      std::memcpy(hs + o_prec + (static_cast<size_t>(w.pod_patch[i]) * 6 + 4) * 8, &w.pod_patch[i + 1], 16);
    if (sl.host_atoms_ver != w.atoms_ver) {
      const std::vector<int32_t>* rows = log_rows(sl.host_atoms_ver);
      if (rows) {
        for (int32_t r : *rows)
          std::memcpy(hs + o_at + static_cast<size_t>(r) * row_bytes8, w.atoms.data() + static_cast<size_t>(r) * w.Wp, row_bytes8);
      } else {
        std::memcpy(hs + o_at, w.atoms.data(), w.atoms.size() * sizeof(uint64_t));
      }
    }
    if (list_moved) {
      std::memcpy(hs + o_ls, w.list.data(), w.list.size() * sizeof(int32_t));
      if (ext) std::memcpy(hs + o_le, w.list_ext.data(), w.list_ext.size() * sizeof(int32_t));
    }
    pk.copy_to(hs, tick_rest);
  } else {
    pk.copy_to(hs, node_bytes);
  }
  sl.host_cand_gen = w.cand_gen;
  sl.host_atoms_ver = w.atoms_ver;
  if (!cand_resident) {  // the records go up whole, current: nothing pending, but rows to write
    sl.pending.clear();
    std::fill(sl.pending_mark.begin(), sl.pending_mark.end(), 0);
    sl.class_flip = false;
    sl.need_k0 = true;
  }
  char* dv = static_cast<char*>(sl.arena.p);
  size_t atoms_up = tick_rest - o_at;  // atom bytes uploaded
  if (!cand_resident) {
    HIP_TRY(ctx, hipMemcpyAsync(dv + from, hs + from, bytes - from, hipMemcpyHostToDevice, ctx->stream));
  } else {
    if (from < node_bytes)
      HIP_TRY(ctx, hipMemcpyAsync(dv, hs, node_bytes, hipMemcpyHostToDevice, ctx->stream));
    // the atoms: current, a few rows behind (each row alone), or whole
    const std::vector<int32_t>* rows = sl.dev_atoms_ver == w.atoms_ver ? nullptr : log_rows(sl.dev_atoms_ver);
    if (sl.dev_atoms_ver == w.atoms_ver) {
      atoms_up = 0;
    } else if (rows && rows->size() <= 32) {
      for (int32_t r : *rows) {
        const size_t o = o_at + static_cast<size_t>(r) * row_bytes8;
        HIP_TRY(ctx, hipMemcpyAsync(dv + o, hs + o, row_bytes8, hipMemcpyHostToDevice, ctx->stream));
      }
      atoms_up = rows->size() * row_bytes8;
    } else {
      HIP_TRY(ctx, hipMemcpyAsync(dv + o_at, hs + o_at, tick_rest - o_at, hipMemcpyHostToDevice, ctx->stream));
    }
    HIP_TRY(ctx, hipMemcpyAsync(dv + tick_rest, hs + tick_rest, bytes - tick_rest, hipMemcpyHostToDevice, ctx->stream));
    if (list_moved) {  // the reordered work list into the resident candidate section
      HIP_TRY(ctx, hipMemcpyAsync(dv + o_ls, hs + o_ls, w.list.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                  ctx->stream));
      if (ext)
        HIP_TRY(ctx, hipMemcpyAsync(dv + o_le, hs + o_le, w.list_ext.size() * sizeof(int32_t), hipMemcpyHostToDevice,
                                    ctx->stream));
    }
  }
  sl.dev_atoms_ver = w.atoms_ver;
  if (sl.host_atoms_ver == w.atoms_ver) {  // both copies current: the log starts again here
    sl.atoms_log_ver = w.atoms_ver;
    sl.atoms_log.clear();
  }
  if (!ctx->ev_upload) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ev_upload, hipEventDisableTiming));
  HIP_TRY(ctx, hipEventRecord(ctx->ev_upload, ctx->stream));  // kernels queue behind the copy
  if (!nodes_patch) sl.dev_state_gen = w.state_gen;  // the section went up whole (or was current)
  sl.dev_cand_gen = w.cand_gen;
  if (list_moved) sl.list_sorted_gen = w.cand_gen;
  ctx->t.k2_list_by_cost = sl.list_sorted_gen == w.cand_gen ? 1 : 0;
  // run() commits what a K0 launch brings the slot to
  sl.commit_k0 = !skip;
  auto t2 = std::chrono::steady_clock::now();

  char* base = static_cast<char*>(sl.arena.p);
  auto at = [base](size_t off) { return static_cast<void*>(base + off); };
  sr::DevWorkload& d = ctx->dw;
  d = sr::DevWorkload{};
  d.n_spot = w.n_spot;
  d.n_pad = w.n_pad;
  d.Wp = w.Wp;
  d.node_rec = static_cast<const uint64_t*>(at(o_nr));
  d.node_free = static_cast<const int64_t*>(at(o_nf));
  d.n_atoms = w.n_atoms;
  d.atoms = static_cast<const uint64_t*>(at(o_at));
  d.cls_prog_off = static_cast<const int32_t*>(at(o_cpo));
  d.cls_prog = static_cast<const int32_t*>(at(o_cp));
  d.cls_prog8 = static_cast<const int32_t*>(at(o_cp8));
  d.n_classes = w.n_classes;
  d.s_empty_off = w.empty_class >= 0 ? static_cast<uint32_t>(w.empty_class) * static_cast<uint32_t>(w.Wp) : 0xffffffffu;
  d.n_t = static_cast<int32_t>(w.t_dim.size());
  for (int i = 0; i < 5; ++i) d.t_off[i] = w.t_off[i];
  d.t_thr = static_cast<const int64_t*>(at(o_tt));
  d.n_pods = na;
  d.pod_rec = static_cast<const uint64_t*>(at(o_prec));
  d.n_cand = ncand;
  d.cand_off = static_cast<const int32_t*>(at(o_co));
  d.cand_global = static_cast<const int32_t*>(at(o_cg));
  d.list = static_cast<const int4*>(at(o_ls));
  d.n_list = static_cast<int32_t>(w.list.size() / 4);
  d.n_list_head = std::min(d.n_list, sr::kListInline);
  for (int32_t i = 0; i < d.n_list_head; ++i)
    d.list_head[i] = int4{w.list[4 * i], w.list[4 * i + 1], w.list[4 * i + 2], w.list[4 * i + 3]};
  d.max_np = w.max_cand_pods;
  d.dyn_cand = dyn ? static_cast<const int32_t*>(at(o_dc)) : nullptr;
  d.dyn_pod = dyn ? static_cast<const uint64_t*>(at(o_dp)) : nullptr;
  d.dk_dom = dyn ? static_cast<const int32_t*>(at(o_dd)) : nullptr;
  d.ds_info = dyn ? static_cast<const int32_t*>(at(o_di)) : nullptr;
  d.sp_tab = dyn ? static_cast<const int32_t*>(at(o_st)) : nullptr;
  d.n_dk = w.n_dk;
  d.ext_cand = ext ? static_cast<const int32_t*>(at(o_ec)) : nullptr;
  d.pod_ext = ext ? static_cast<const uint64_t*>(at(o_ep)) : nullptr;
  d.list_ext = ext ? static_cast<const int4*>(at(o_le)) : nullptr;
  d.node_scal = ext ? static_cast<const int64_t*>(at(o_ns)) : nullptr;
  static_assert(sr::kDevExtU64 == sr::kExtU64, "extension record layout shared by encode.cpp and kernels.hip");
  static_assert(sr::kDevDynU64 == sr::kDynU64 && sr::kDevDomKeys == sr::kDomKeys && sr::kDevDynTerms == sr::kDynTerms &&
                    sr::kDevSpreadSlots == sr::kSpreadSlots,
                "domain-path layout shared by encode.cpp and kernels.hip");
  for (int k = 0; k < sr::kDomKeys; ++k) d.dk_row[k] = w.dk_row[k];
  d.S = static_cast<uint64_t*>(sl.tables.p);
  d.T = d.S + static_cast<size_t>(w.n_classes) * w.Wp;
  d.out_node = static_cast<int32_t*>(ctx->out_node.p);
  d.out_status = static_cast<int32_t*>(ctx->out_status.p);
  d.out_bytes = static_cast<uint32_t*>(ctx->out_bytes.p);
  d.d_min = static_cast<int32_t*>(ctx->dmin.p);
  d.k2_mode = ctx->k2_mode;
  d.k2_narrow = ctx->k2_narrow;
  d.k2_wpb = ctx->k2_wpb;
  d.k2_excl = ctx->k2_excl;
  d.k2_node_kernel = ctx->k2_node_kernel;
  // Wide rows, every candidate on the node-order kernel (launch_k2's condition)
  // and every class program in its 8-slot record: K0 writes only the S-row
  // heads, K2 evaluates S words beyond them from the programs.
  d.s_head_only = 0;
  if (ctx->s_head_only && w.Wp > 64 && w.dyn_cand.empty() && ctx->k2_mode == 0 && ctx->k2_node_kernel &&
      w.max_cand_pods >= 1 && w.max_cand_pods <= 256) {
    bool short_programs = true;
    for (int32_t k = 0; k < w.n_classes && short_programs; ++k)
      short_programs = w.cls_prog8[static_cast<size_t>(k) * 8] != -2;
    d.s_head_only = short_programs ? 1 : 0;
  }
  d.swap_mask = w.swap_mask;
  d.rank_next = ~0ull;  // sr_plan_first sets its batch's value
  d.prof = nullptr;
  if (ctx->prof_file) {
    const size_t pbytes = sizeof(uint64_t) * (16 * static_cast<size_t>(std::max(1, ncand)) + 2 * sr::kK0ProfWaves);
    HIP_TRY(ctx, dev_reserve(ctx->prof, pbytes));
    HIP_TRY(ctx, hipMemsetAsync(ctx->prof.p, 0, pbytes, ctx->stream));
    d.prof = static_cast<uint64_t*>(ctx->prof.p);
  }
  void* dres = nullptr;
  HIP_TRY(ctx, hipHostGetDevicePointer(&dres, ctx->h_result.p, 0));
  d.result = static_cast<uint64_t*>(dres);
  HIP_TRY(ctx, hipHostGetDevicePointer(&dres, ctx->h_early.p, 0));
  ctx->d_early = static_cast<uint64_t*>(dres);
  d.res_stat = d.res_map = nullptr;  // set per run
  ctx->t.bytes_uploaded = static_cast<uint64_t>(cand_resident ? (from < node_bytes ? node_bytes : 0) + atoms_up +
                                                                   bytes - tick_rest
                                                               : bytes - from);
  // K0 writes the patches into the node section; a K0-less run's K2 reads them
  // (every changed node, whether or not the section went up whole)
  const bool use_patch = skip ? !patch.empty() : nodes_patch;
  d.node_patch = use_patch ? static_cast<const uint64_t*>(at(o_np)) : nullptr;
  d.n_node_patch = use_patch ? static_cast<int32_t>(patch.size() / sr::kNodePatchU64) : 0;
  if (skip) k0_inc = false;
  d.k0_inc = k0_inc ? 1 : 0;
  d.n_k0_cols = static_cast<int32_t>(kcols.size());
  d.n_k0_rows = static_cast<int32_t>(krows.size());
  d.k0_cols = kcols.empty() ? nullptr : static_cast<const int32_t*>(at(o_kc));
  d.k0_rows = krows.empty() ? nullptr : static_cast<const int32_t*>(at(o_kr));
  const bool pods_patch = !skip && cand_resident && !ppatch.empty();
  d.pod_patch = pods_patch ? static_cast<const uint64_t*>(at(o_pp)) : nullptr;
  d.n_pod_patch = pods_patch ? static_cast<int32_t>(ppatch.size() / sr::kPodPatchU64) : 0;
  d.k0_skip = skip ? 1 : 0;
  d.n_dirty = 0;
  if (skip) {  // the changed nodes in the kernel arguments (<= 16: kSkipDirty)
    const size_t NP = static_cast<size_t>(w.n_pad);
    for (int32_t i : sl.dirty) {
      d.dirty_node[d.n_dirty] = i;
      for (size_t dm = 0; dm < 3; ++dm) d.dirty_free[d.n_dirty][dm] = E.node_free[dm * NP + static_cast<size_t>(i)];
      ++d.n_dirty;
    }
  }
  static_assert(sizeof(d.dirty_node) / sizeof(d.dirty_node[0]) == 16, "kSkipDirty nodes in the kernel arguments");
  d.first_fallback_local = w.first_fallback;
  static_assert(sr::kPodPatchU64 == sr::kPodPatchWords && sr::kTPad == sr::kTSpare, "patch layout shared with encode.cpp");

  const uint64_t row = static_cast<uint64_t>(w.Wp) * 8;
  // K0 algorithmic bytes: every table row written once; every atom row a class
  // program names, the nodes' free capacities and the thresholds read once.
  uint64_t atom_reads = w.cls_prog.size();
  const uint64_t s_row = d.s_head_only ? static_cast<uint64_t>(std::min(w.Wp, 8)) * 8 : row;  // S words K0 writes
  ctx->t.bytes_tables = static_cast<uint64_t>(w.n_classes) * s_row + w.t_dim.size() * row + atom_reads * s_row +
                        3ull * 8 * w.n_pad + 32ull * w.n_classes;
  if (k0_inc) {  // the changed columns of every row (S columns inside the written head), the moved rows whole
    const int32_t s_words = d.s_head_only ? std::min(w.Wp, 8) : w.Wp;
    uint64_t s_cols = 0;
    for (int32_t col : kcols) s_cols += col < s_words ? 1 : 0;
    ctx->t.bytes_tables = (static_cast<uint64_t>(w.n_classes) + atom_reads) * 8 * s_cols +
                          (32ull * w.n_classes) * (s_cols > 0 ? 1 : 0) + w.t_dim.size() * 8 * kcols.size() +
                          3ull * 64 * 8 * kcols.size() + krows.size() * (row + 8ull * w.n_pad);
  }
  // K2: counted by the kernel itself per candidate (out_bytes), read back by
  // the next run with status or node_of_pod outputs
  ctx->t.bytes_placement = 0;
  ctx->issued_known = false;
  ctx->issued_checks = 0;
  ctx->t.ms_pack_host = std::chrono::duration<double, std::milli>(t1 - t0).count();
  ctx->t.ms_upload = std::chrono::duration<double, std::milli>(t2 - t1).count();
  ctx->t.n_pods = na;
  ctx->t.n_spot = w.n_spot;
  ctx->t.n_cand = ncand;
  ctx->t.n_words = w.Wp;
  ctx->t.n_rows_static = d.n_classes;
  ctx->t.n_rows_threshold = d.n_t;
  ctx->t.n_classes = w.n_classes;
  ctx->t.enc_new_specs = ctx->enc.last_new_specs;
  ctx->t.enc_static_rebuilt = ctx->enc.last_static_changed;
  ctx->t.enc_state_nodes = ctx->enc.last_state_changed;
  ctx->t.enc_memo_pods = ctx->enc.last_memo_hits;
  ctx->t.enc_reused = ctx->enc.last_reused;
  ctx->t.enc_pod_patches = ctx->enc.last_pod_patches;
  ctx->t.k0_columns = skip ? -2 : k0_inc ? static_cast<int32_t>(kcols.size()) : -1;
  ctx->t.k0_rows_moved = k0_inc ? static_cast<int32_t>(krows.size()) : 0;
  ctx->t.k0_dirty_nodes = skip ? static_cast<int32_t>(patch.size() / sr::kNodePatchU64) : 0;
  if (skip) ctx->t.bytes_tables = 0;
  ctx->prepared = true;
  return SR_OK;
}

sr_status flush_timing(sr_ctx* ctx) {
  if (ctx->ev_used == 0) return SR_OK;
  HIP_TRY(ctx, hipEventSynchronize(ctx->ev_end[ctx->ev_used - 1]));
  double* sums[4] = {&ctx->t.ms_tables, &ctx->t.ms_placement, &ctx->t.ms_winner, &ctx->t.ms_collective};
  for (size_t i = 0; i < ctx->ev_used; ++i) {
    float ms = 0;
    HIP_TRY(ctx, hipEventElapsedTime(&ms, ctx->ev_start[i], ctx->ev_end[i]));
    *sums[ctx->ev_kernel[i]] += ms;
  }
  ctx->ev_used = 0;
  return SR_OK;
}

// The end of a single-rank winner-only run: walk K2's per-candidate words in
// candidate order up to the first drainable candidate, then read its mapping
// (rescheduler.go:280-286 stops there too).  A run whose words have not all
// arrived after 100 ms falls back to the stream, which also surfaces a kernel
// fault as an error.
sr_status finish_early(sr_ctx* ctx, sr_plan_out* out) {
  const sr::Workload& w = ctx->cur->wl;
  const sr::DevWorkload& d = ctx->dw;
  if (ctx->timing_cur) ctx->t.n_runs += 1;
  volatile uint64_t* stat = static_cast<volatile uint64_t*>(ctx->h_early.p);
  volatile uint64_t* map = stat + d.n_cand;
  const uint32_t tag = d.seq;
  auto ready = [&](volatile uint64_t* p) { return static_cast<uint32_t>(*p >> 32) == tag; };
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t spins = 0;
  bool synced = false;
  auto wait = [&](volatile uint64_t* p) -> sr_status {
    while (!ready(p)) {
      if (!synced && (++spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
        HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
        synced = true;
      }
      if (synced && !ready(p)) {
        ctx->err = "K2 result word not written by this run";
        return SR_ERR_HIP;
      }
    }
    return SR_OK;
  };
  int32_t k = 0;
  for (; k < d.n_cand; ++k) {
    sr_status st = wait(stat + k);
    if (st != SR_OK) return st;
    if (static_cast<uint32_t>(stat[k]) == 1) break;
  }
  ctx->in_flight = !synced;
  out->first_fallback = w.first_fallback;
  out->first_ok = k < d.n_cand ? w.cand_global[k] : -1;
  out->winner = (out->first_ok >= 0 && (w.first_fallback < 0 || w.first_fallback > out->first_ok)) ? out->first_ok : -1;
  out->winner_npods = 0;
  if (k < d.n_cand) {
    const int32_t o = w.cand_off[k], np = w.cand_off[k + 1] - o;
    for (int32_t q = 0; q < np; ++q) {
      sr_status st = wait(map + o + q);
      if (st != SR_OK) return st;
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    out->winner_npods = np;
    if (out->winner_map)
      for (int32_t q = 0; q < np; ++q) out->winner_map[q] = static_cast<int32_t>(static_cast<uint32_t>(map[o + q]));
  }
  out->checks_dense = static_cast<uint64_t>(d.n_pods) * static_cast<uint64_t>(w.n_spot);
  out->fallback_pods = w.fallback_pods;
  out->checks = ctx->issued_known ? ctx->issued_checks : 0;
  return SR_OK;
}

sr_status run(sr_ctx* ctx, sr_plan_out* out, bool full, bool use_comm) {
  if (!ctx->prepared) {
    ctx->err = "sr_plan_run before sr_plan_prepare";
    return SR_ERR_STATE;
  }
  const sr::Workload& w = ctx->cur->wl;
  sr::DevWorkload& d = ctx->dw;
  hipStream_t s = ctx->stream;
  HIP_TRY(ctx, hipSetDevice(ctx->device));
  const bool collective = has_comm(ctx) && use_comm;
  // Single rank, winner only: K2 writes each candidate's outcome to the host
  // and the run returns once the candidates up to the winner are known (no K3)
  const bool early = !collective && !full && !ctx->prof_file;
  const int32_t timing = (ctx->timing_runs++ % ctx->timing_every) == 0 ? ctx->timing : 0;
  ctx->timing_cur = timing;
  do ctx->seq = g_run_seq.fetch_add(1, std::memory_order_relaxed) + 1;
  while (ctx->seq == 0);  // tag 0 is never used: fresh result memory holds zeros
  d.seq = ctx->seq;
  volatile uint64_t* res = static_cast<volatile uint64_t*>(ctx->h_result.p);
  // Timed kernels get an event pair from the pool, recorded by their own
  // dispatch (hipExtLaunchKernelGGL); the collective is bracketed with
  // plain records.  Events are read back lazily (flush_timing).
  // k: 0 = K0, 1 = K2, 2 = K3, 3 = the collective (mask bit 2, with K3)
  auto pair_for = [&](int k, hipEvent_t* a, hipEvent_t* b) -> sr_status {
    *a = *b = nullptr;
    if (!(timing >> (k == 3 ? 2 : k) & 1)) return SR_OK;
    if (ctx->ev_used == ctx->ev_start.size()) {
      if (ctx->ev_used >= 3072) {  // bounded pool: read back what is pending
        sr_status st = flush_timing(ctx);
        if (st != SR_OK) return st;
      } else {
        hipEvent_t e0, e1;
        HIP_TRY(ctx, hipEventCreate(&e0));
        HIP_TRY(ctx, hipEventCreate(&e1));
        ctx->ev_start.push_back(e0);
        ctx->ev_end.push_back(e1);
        ctx->ev_kernel.push_back(0);
      }
    }
    const size_t i = ctx->ev_used++;
    ctx->ev_kernel[i] = static_cast<int8_t>(k);
    *a = ctx->ev_start[i];
    *b = ctx->ev_end[i];
    return SR_OK;
  };
#define PAIR(k, a, b)                         \
  hipEvent_t a, b;                            \
  do {                                        \
    sr_status _st = pair_for((k), &a, &b);    \
    if (_st != SR_OK) return _st;             \
  } while (0)
  hipEvent_t e0a = nullptr, e0b = nullptr;  // K0's pair only when it is launched (an unrecorded event fails)
  if (!d.k0_skip) {
    sr_status pst = pair_for(0, &e0a, &e0b);
    if (pst != SR_OK) return pst;
  }
  // the first run of a candidate generation records its K2 durations (list_cost)
  Slot& slc = *ctx->cur;
  const bool want_cost = ctx->list_cost && d.n_list > ctx->list_cost_min && slc.list_sorted_gen != w.cand_gen &&
                         slc.cost_gen != w.cand_gen;
  d.out_cycles = nullptr;
  if (want_cost) {
    HIP_TRY(ctx, dev_reserve(ctx->out_cycles, sizeof(uint32_t) * static_cast<size_t>(d.n_cand)));
    HIP_TRY(ctx, host_reserve(slc.h_cycles, sizeof(uint32_t) * static_cast<size_t>(d.n_cand)));
    if (!slc.ev_cost) HIP_TRY(ctx, hipEventCreateWithFlags(&slc.ev_cost, hipEventDisableTiming));
    d.out_cycles = static_cast<uint32_t*>(ctx->out_cycles.p);
  }
  // d_min alternates between two buffers: K0 resets this run's, K2 the next's
  const int par = static_cast<int>(ctx->run_count++ & 1);
  d.d_min = static_cast<int32_t*>(ctx->dmin.p) + 8 * par;
  d.d_min_next = static_cast<int32_t*>(ctx->dmin.p) + 8 * (1 - par);
  Slot& sl = *ctx->cur;
  // the split launch (see sr_ctx::k2_split): the node-order part on this
  // stream, the general one on stream2 between a fork and a join event
  const int32_t n_node = w.n_list_node;
  const bool split = ctx->k2_split && n_node > 0 && n_node < d.n_list && d.k2_mode == 0 && d.k2_node_kernel &&
                     w.max_np_node >= 1 && w.max_np_node <= 256;
  if (split && !ctx->stream2) {
    HIP_TRY(ctx, hipStreamCreateWithFlags(&ctx->stream2, hipStreamNonBlocking));
    HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming));
    HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming));
  }
  // the fork is K0's own completion signal when K0 runs untimed (no marker
  // packet between K0 and K2: ~5 us per marker on the split tick)
  bool forked = false;
  if (d.k0_skip) {
    if (!ctx->dmin_ready[par])  // no K2 of a previous run reset it: reset here
      HIP_TRY(ctx, hipMemsetAsync(d.d_min, 0xff, sizeof(uint64_t), s));
  } else {
    forked = split && !e0b && ctx->k2_dispatch_events;
    HIP_TRY(ctx, sr::launch_tables(d, w.first_fallback, s, e0a, forked ? ctx->ev_fork : e0b));
    if (sl.commit_k0) {  // K0 wrote the node and pod patches and brought the rows to this workload (a rerun:
      sl.commit_k0 = false;  // idempotent)
      sl.tables_cand_gen = w.cand_gen;
      sl.tables_state_gen = sl.dev_state_gen = w.state_gen;
      if (sl.tables_thr != w.t_thr) sl.tables_thr = w.t_thr;
      sl.tables_atoms_ver = w.atoms_ver;
      sl.atom_cols.clear();
      sl.dirty.clear();
      sl.dirty_valid = true;
      sl.seen_gen = w.state_gen;
      for (int32_t q : sl.pending) sl.pending_mark[q] = 0;
      sl.pending.clear();
      sl.class_flip = false;
      sl.need_k0 = false;
    }
  }
  ctx->dmin_ready[par] = false;
  ctx->dmin_ready[1 - par] = d.n_list > 0;  // K2's first candidate resets it
  PAIR(1, e1a, e1b);
  const bool shm = collective && ctx->shm.host;  // ranks reduce through host memory: no collective, no K3
  int shm_par = 0;
  if (early) {
    d.res_stat = ctx->d_early;
    d.res_map = ctx->d_early + d.n_cand;
  } else if (shm) {
    sr_status pst = shm_publish(ctx, &shm_par);
    if (pst != SR_OK) return pst;
  } else {
    d.res_stat = d.res_map = nullptr;
  }
  ctx->t.k2_launches = d.n_list > 0 ? (split ? 2 : 1) : 0;
  // cooperative blocks for the front of a cost-ordered list, on a node-order
  // launch of four waves per block without extension records
  d.n_coop = 0;
  {
    const bool node_launch = split || (!d.dyn_cand && d.k2_mode == 0 && d.max_np >= 1 && d.max_np <= 256 &&
                                       d.k2_node_kernel);
    const int32_t len = split ? n_node : d.n_list;
    const int32_t wpb = d.k2_wpb == 1 || d.k2_wpb == 2 || d.k2_wpb == 4 ? d.k2_wpb : (len <= 2048 ? 1 : 4);
    if (node_launch && wpb == 4 && !d.ext_cand && ctx->cur->list_sorted_gen == w.cand_gen)
      d.n_coop = std::min(w.n_coop_front, len);
  }
  ctx->t.k2_coop = d.n_coop;
  if (split) {
    sr::DevWorkload dp = d, dn = d;
    dp.list = d.list + n_node;
    dp.n_list = d.n_list - n_node;
    dp.n_list_head = 0;
    dp.n_coop = 0;  // (the general kernel)
    if (d.list_ext) dp.list_ext = d.list_ext + n_node;
    dn.n_list = n_node;
    dn.n_list_head = std::min(d.n_list_head, n_node);
    dn.max_np = w.max_np_node;
    dn.dyn_cand = nullptr;  // none of its candidates is on the domain path
    if (e1a) HIP_TRY(ctx, hipEventRecord(e1a, s));
    if (!forked) HIP_TRY(ctx, hipEventRecord(ctx->ev_fork, s));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
    // the join is the general kernel's own completion signal
    HIP_TRY(ctx, sr::launch_placement(dp, ctx->stream2, nullptr, ctx->k2_dispatch_events ? ctx->ev_join : nullptr));
    if (!ctx->k2_dispatch_events) HIP_TRY(ctx, hipEventRecord(ctx->ev_join, ctx->stream2));
    HIP_TRY(ctx, sr::launch_placement(dn, s, nullptr, nullptr));
    HIP_TRY(ctx, hipStreamWaitEvent(s, ctx->ev_join, 0));
    if (e1b) HIP_TRY(ctx, hipEventRecord(e1b, s));
  } else {
    HIP_TRY(ctx, sr::launch_placement(d, s, e1a, e1b));
  }
  if (want_cost) {  // after K2 in stream order: the next prepare waits for it (ev_cost)
    HIP_TRY(ctx, hipMemcpyAsync(slc.h_cycles.p, d.out_cycles, sizeof(uint32_t) * static_cast<size_t>(d.n_cand),
                                hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipEventRecord(slc.ev_cost, s));
    slc.cost_gen = w.cand_gen;
  }
  if (early) return finish_early(ctx, out);
  if (!shm) {  // the shared-memory transport has no collective and no K3 (shm_reduce below)
    PAIR(2, e2a, e2b);
    if (collective) {
      PAIR(3, eca, ecb);
      if (eca) HIP_TRY(ctx, hipEventRecord(eca, s));
      sr_status cst = allreduce_min_dev(ctx, d.d_min, 3);  // first ok, first fallback, rank_next
      if (cst != SR_OK) return cst;
      if (ecb) HIP_TRY(ctx, hipEventRecord(ecb, s));
    }
    HIP_TRY(ctx, sr::launch_winner(d, s, e2a, e2b));
  }
#undef PAIR
  if (timing) ctx->t.n_runs += 1;
  const int32_t na = d.n_pods, ncand = d.n_cand;
  if (full || ctx->prof_file) {
    if (full) {
      HIP_TRY(ctx, host_reserve(ctx->h_status, sizeof(int32_t) * std::max(1, ncand)));
      HIP_TRY(ctx, host_reserve(ctx->h_node, sizeof(int32_t) * std::max(1, na)));
      HIP_TRY(ctx, host_reserve(ctx->h_bytes, sizeof(uint32_t) * std::max(1, ncand)));
      if (ncand) {
        HIP_TRY(ctx, hipMemcpyAsync(ctx->h_status.p, d.out_status, sizeof(int32_t) * ncand, hipMemcpyDeviceToHost, s));
        HIP_TRY(ctx, hipMemcpyAsync(ctx->h_bytes.p, d.out_bytes, sizeof(uint32_t) * ncand, hipMemcpyDeviceToHost, s));
      }
      if (na) HIP_TRY(ctx, hipMemcpyAsync(ctx->h_node.p, d.out_node, sizeof(int32_t) * na, hipMemcpyDeviceToHost, s));
    }
    HIP_TRY(ctx, hipStreamSynchronize(s));
  } else if (shm) {
    // (the walk below waits for the outcome words it needs)
  } else {
    // Every result word carries this run's sequence number in its upper
    // half (K3 stores them without ordering): poll the header, then the
    // winner's mapping, instead of waking up on stream completion.  A run
    // that has not finished after 100 ms falls back to the stream (which
    // also surfaces a kernel fault as an error).
    const uint32_t tag = static_cast<uint32_t>(d.seq);
    auto ready = [&](size_t i) { return static_cast<uint32_t>(res[i] >> 32) == tag; };
    auto header_ready = [&] { return ready(0) && ready(1) && ready(2) && ready(3) && ready(4); };
    auto map_ready = [&] {
      if (!static_cast<uint32_t>(res[1])) return true;
      const size_t np = static_cast<uint32_t>(res[2]);
      for (size_t q = 0; q < np; ++q)
        if (!ready(sr::kResultHeader + q)) return false;
      return true;
    };
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t spins = 0;
    while (!(header_ready() && map_ready())) {
      if ((++spins & 1023) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(100)) {
        HIP_TRY(ctx, hipStreamSynchronize(s));
        break;
      }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  if (shm) {  // every rank's outcome words in global order (ms_collective: this host walk)
    const auto t0 = std::chrono::steady_clock::now();
    sr_status sst = shm_reduce(ctx, shm_par);
    if (sst != SR_OK) return sst;
    if (timing & 4) ctx->t.ms_collective += std::chrono::duration<double, std::milli>(
                                               std::chrono::steady_clock::now() - t0).count();
  }

  if (ctx->prof_file && ncand > 0) {  // diagnostics only (tools/k2_profile.py)
    std::vector<uint64_t> pr(static_cast<size_t>(ncand) * 16 + 2 * sr::kK0ProfWaves);
    HIP_TRY(ctx, hipMemcpy(pr.data(), d.prof, pr.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    const int64_t hdr[2] = {ncand, static_cast<int64_t>(sr::kK0ProfWaves)};
    std::fwrite(hdr, sizeof(hdr), 1, ctx->prof_file);
    std::fwrite(pr.data(), sizeof(uint64_t), pr.size(), ctx->prof_file);
    std::fflush(ctx->prof_file);
  }
  auto val = [&](size_t i) { return static_cast<int32_t>(static_cast<uint32_t>(res[i])); };
  const uint32_t tag = static_cast<uint32_t>(d.seq);
  for (size_t i = 0; i < 5; ++i)
    if (static_cast<uint32_t>(res[i] >> 32) != tag) {
      ctx->err = "result header not written by this run";
      return SR_ERR_HIP;
    }
  out->first_ok = val(0);
  out->first_fallback = val(3);
  ctx->last_rank_next = val(4);
  out->winner = (val(0) >= 0 && (val(3) < 0 || val(3) > val(0))) ? val(0) : -1;
  out->winner_npods = val(1) ? val(2) : 0;
  if (out->winner_map && val(1))
    for (int32_t q = 0; q < val(2); ++q) out->winner_map[q] = val(sr::kResultHeader + q);
  out->checks_dense = static_cast<uint64_t>(na) * static_cast<uint64_t>(w.n_spot);
  out->fallback_pods = w.fallback_pods;
  if (full) {
    const int32_t* hs = static_cast<const int32_t*>(ctx->h_status.p);
    const int32_t* hn = static_cast<const int32_t*>(ctx->h_node.p);
    const uint32_t* hb = static_cast<const uint32_t*>(ctx->h_bytes.p);
    if (out->status) {
      for (int32_t i = 0; i < w.n_input_cand; ++i) out->status[i] = w.status_host[i];
      for (int32_t k = 0; k < ncand; ++k) out->status[w.cand_src[k]] = hs[k];
    }
    // K2's own byte counts; the reference's CheckPredicates calls for the same
    // plan: findSpotNodeForPod stops at the first fit (position + 1 calls) and
    // scans every spot node for a pod that fits nowhere, where canDrainNode stops
    uint64_t bytes = 0, issued = 0;
    for (int32_t k = 0; k < ncand; ++k) {
      bytes += hb[k];
      const int32_t o = w.cand_off[k], np = w.cand_off[k + 1] - o;
      const int32_t done = hs[k] >= 0 ? std::min(np, hs[k]) : np;
      for (int32_t q = 0; q < done; ++q) issued += static_cast<uint64_t>(hn[o + q]) + 1;
      if (hs[k] >= 0) issued += static_cast<uint64_t>(w.n_spot);
    }
    ctx->t.bytes_placement = bytes;
    ctx->issued_checks = issued;
    ctx->issued_known = true;
    if (out->node_of_pod) {
      for (int32_t i = 0; i < w.n_input_pods; ++i) out->node_of_pod[i] = -1;
      for (int32_t q = 0; q < na; ++q) out->node_of_pod[w.pod_src[q] - w.pod_base] = hn[q];
    }
  }
  out->checks = ctx->issued_known ? ctx->issued_checks : 0;
  return SR_OK;
}

}  // namespace

static sr_status plan_first(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
                            sr_plan_out* out);

extern "C" {

#define SR_STR2(x) #x
#define SR_STR(x) SR_STR2(x)
const char* sr_build_info(void) {
  return "srplanner abi=" SR_STR(SR_ABI_VERSION) " target=gfx950 kernels=K0-tables,K2-placement(fused feasibility),K3-winner";
}

int32_t sr_abi_version(void) { return SR_ABI_VERSION; }

sr_status sr_create(int32_t device, sr_ctx** out) {
  if (!out) return SR_ERR_INVALID_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return SR_ERR_NO_DEVICE;
  if (device < 0 || device >= count) return SR_ERR_INVALID_ARG;
  auto* ctx = new sr_ctx();
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return SR_ERR_HIP;
  }
  if (const char* path = std::getenv("SR_K2_PROFILE")) ctx->prof_file = std::fopen(path, "ab");
  if (const char* m = std::getenv("SR_K2_MODE")) ctx->k2_mode = std::atoi(m) == 1 ? 1 : 0;
  if (const char* m = std::getenv("SR_NODE_PATCH")) ctx->node_patch = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_K2_NARROW")) ctx->k2_narrow = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_K2_NODE_KERNEL")) ctx->k2_node_kernel = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_S_HEAD_ONLY")) ctx->s_head_only = std::atoi(m) != 0;
  if (const char* b = std::getenv("SR_PREFIX_BATCH")) ctx->prefix_batch = std::max(1, std::atoi(b));
  if (const char* m = std::getenv("SR_K2_WPB")) ctx->k2_wpb = std::atoi(m);
  if (const char* m = std::getenv("SR_K2_EXCL")) ctx->k2_excl = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_PLAN_SLOTS")) ctx->n_slots = std::max(1, std::min(16, std::atoi(m)));
  if (const char* m = std::getenv("SR_K0_INCREMENTAL")) ctx->k0_incremental = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_K0_SKIP")) ctx->k0_skip = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_K2_SPLIT")) ctx->k2_split = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_LIST_COST")) ctx->list_cost = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_LIST_COST_MIN")) ctx->list_cost_min = std::max(0, std::atoi(m));
  if (const char* m = std::getenv("SR_K2_SPLIT_MIN")) ctx->enc.split_min = std::max(0, std::atoi(m));
  if (const char* m = std::getenv("SR_K2_DISPATCH_EVENTS")) ctx->k2_dispatch_events = std::atoi(m) != 0;
  if (const char* m = std::getenv("SR_LIST_HEAD")) ctx->enc.list_head = std::max(0, std::atoi(m));
  if (const char* m = std::getenv("SR_K2_COOP")) ctx->k2_coop = std::max(0, std::atoi(m));
  *out = ctx;
  return SR_OK;
}

void sr_destroy(sr_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  if (ctx->comm) (void)rccl().comm_destroy(ctx->comm);
  if (ctx->shm.host) {
    if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
    (void)hipHostUnregister(ctx->shm.host);
    munmap(ctx->shm.host, ctx->shm.bytes);
    if (ctx->rank == 0) shm_unlink(ctx->shm.name.c_str());  // the ranks keep their mappings
  }
  for (DevBuf* b : {&ctx->out_node, &ctx->out_status, &ctx->out_bytes, &ctx->dmin, &ctx->prof,
                    &ctx->scratch})
    if (b->p) (void)hipFree(b->p);
  if (ctx->ev_upload) (void)hipEventDestroy(ctx->ev_upload);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  for (hipEvent_t e : {ctx->ev_fork, ctx->ev_join})
    if (e) (void)hipEventDestroy(e);
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->out_cycles.p) (void)hipFree(ctx->out_cycles.p);
  for (HostBuf* b : {&ctx->h_result, &ctx->h_status, &ctx->h_node, &ctx->h_bytes, &ctx->h_early, &ctx->h_comm})
    if (b->p) (void)hipHostFree(b->p);
  for (auto& sl : ctx->slots) {
    if (sl->arena.p) (void)hipFree(sl->arena.p);
    if (sl->tables.p) (void)hipFree(sl->tables.p);
    if (sl->h_arena.p) (void)hipHostFree(sl->h_arena.p);
    if (sl->h_cycles.p) (void)hipHostFree(sl->h_cycles.p);
    if (sl->ev_cost) (void)hipEventDestroy(sl->ev_cost);
  }
  for (auto* v : {&ctx->ev_start, &ctx->ev_end})
    for (hipEvent_t e : *v) (void)hipEventDestroy(e);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->prof_file) std::fclose(ctx->prof_file);
  delete ctx;
}

const char* sr_last_error(const sr_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

sr_status sr_plan_first(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* cluster, const sr_candidates* cands,
                        sr_plan_out* out) {
  if (!ctx || !snap || !cluster || !cands || !out || cands->n_cand < 0) return SR_ERR_INVALID_ARG;
  return plan_first(ctx, snap, cluster, cands, out);
}

sr_status sr_plan_prepare(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* cluster, const sr_candidates* cands) {
  if (!ctx || !snap || !cluster || !cands || cands->n_cand < 0) return SR_ERR_INVALID_ARG;
  return prepare(ctx, snap, cluster, cands);
}

sr_status sr_plan_run(sr_ctx* ctx, sr_plan_out* out) {
  if (!ctx || !out) return SR_ERR_INVALID_ARG;
  return run(ctx, out, out->status != nullptr || out->node_of_pod != nullptr, true);
}

sr_status sr_plan(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* cluster, const sr_candidates* cands,
                  sr_plan_out* out) {
  if (!ctx || !snap || !cluster || !cands || !out || cands->n_cand < 0) return SR_ERR_INVALID_ARG;
  sr_status st = prepare(ctx, snap, cluster, cands);
  if (st != SR_OK) return st;
  return run(ctx, out, out->status != nullptr || out->node_of_pod != nullptr, true);
}

// run()'s loop with its break (rescheduler.go:228-287): prefix batches of
// candidates, each encoded and planned on its own, until the first drainable
// candidate is known.  Batch k covers local candidates [lo_k, hi_k) on every
// rank.  The run's collective also reduces the smallest global index some rank
// has not planned yet (rank_next): a drainable candidate below it is the first
// overall, whatever the partition of the global indices over the ranks (with
// contiguous shards, rank 1's early batches hold late indices, and batching
// goes on until rank 0 has planned everything below them).  Every rank sees the
// same reduced values, so all stop after the same batch.
static sr_status plan_first(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* c, const sr_candidates* cands,
                            sr_plan_out* out) {
  const int32_t n = cands->n_cand;
  const int32_t* off = cands->cand_pod_off;
  const bool full = out->status != nullptr || out->node_of_pod != nullptr;
  if (out->status)
    for (int32_t i = 0; i < n; ++i) out->status[i] = SR_CAND_SKIPPED;
  if (out->node_of_pod && n > 0)
    for (int32_t i = 0; i < off[n] - off[0]; ++i) out->node_of_pod[i] = -1;
  std::vector<int32_t> glob;
  if (!cands->cand_global) {
    glob.resize(static_cast<size_t>(std::max(0, n)));
    for (int32_t i = 0; i < n; ++i) glob[i] = i;
  }
  const int32_t* G = cands->cand_global ? cands->cand_global : glob.data();
  // suffix minima of the global indices: the smallest one not planned after a batch ending at l
  std::vector<int32_t> next(static_cast<size_t>(std::max(0, n)) + 1, INT32_MAX);
  int32_t maxp = 1;
  for (int32_t i = n - 1; i >= 0; --i) {
    if (G[i] < 0) {
      ctx->err = "cand_global holds a negative index";
      return SR_ERR_INVALID_ARG;
    }
    next[i] = std::min(next[i + 1], G[i]);
    maxp = std::max(maxp, off[i + 1] - off[i]);
  }
  out->winner = out->first_ok = out->first_fallback = -1;
  out->winner_npods = 0;
  out->checks = out->fallback_pods = out->checks_dense = 0;
  std::vector<int32_t> bst, bnode, bmap(out->winner_map ? static_cast<size_t>(maxp) : 0);
  const bool coll = has_comm(ctx);
  int32_t batches = 0;
  for (int32_t lo = 0, B = ctx->prefix_batch;; B = std::min(B * 2, 1 << 20)) {
    const int32_t hi = static_cast<int32_t>(std::min<int64_t>(INT32_MAX, static_cast<int64_t>(lo) + B));
    const int32_t l0 = std::min(lo, n), l1 = std::min(hi, n);
    sr_candidates sub{l1 - l0, off + l0, cands->cand_pods, G + l0};
    sr_plan_out o{};
    o.winner_map = out->winner_map ? bmap.data() : nullptr;
    if (full) {
      bst.assign(static_cast<size_t>(std::max(1, l1 - l0)), 0);
      bnode.assign(static_cast<size_t>(std::max(1, n > 0 ? off[l1] - off[l0] : 0)), -1);
      o.status = bst.data();
      o.node_of_pod = bnode.data();
    }
    sr_status st = prepare(ctx, snap, c, &sub);
    if (st != SR_OK) return st;
    ctx->dw.rank_next = next[l1] == INT32_MAX ? ~0ull : static_cast<uint64_t>(next[l1]);
    st = run(ctx, &o, full, true);
    if (st != SR_OK) return st;
    ++batches;
    if (full) {
      if (out->status) std::copy(bst.begin(), bst.begin() + (l1 - l0), out->status + l0);
      if (out->node_of_pod && n > 0) std::copy(bnode.begin(), bnode.begin() + (off[l1] - off[l0]), out->node_of_pod + (off[l0] - off[0]));
    }
    out->checks += o.checks;
    out->checks_dense += o.checks_dense;
    out->fallback_pods += o.fallback_pods;
    if (o.first_fallback >= 0 && (out->first_fallback < 0 || o.first_fallback < out->first_fallback))
      out->first_fallback = o.first_fallback;
    if (o.first_ok >= 0 && (out->first_ok < 0 || o.first_ok < out->first_ok)) {
      out->first_ok = o.first_ok;
      out->winner_npods = o.winner_npods;  // 0 on the ranks that do not own it
      if (out->winner_map)
        std::copy(bmap.begin(), bmap.begin() + o.winner_npods, out->winner_map);
    }
    // the smallest global index no rank has planned yet (reduced by the run's collective)
    const int64_t bound = coll ? (ctx->last_rank_next < 0 ? INT64_MAX : ctx->last_rank_next)
                               : (next[l1] == INT32_MAX ? INT64_MAX : next[l1]);
    if (bound == INT64_MAX || (out->first_ok >= 0 && out->first_ok < bound)) break;
    lo = hi;
  }
  out->winner = (out->first_ok >= 0 && (out->first_fallback < 0 || out->first_fallback > out->first_ok))
                    ? out->first_ok : -1;
  ctx->t.prefix_batches = batches;
  return SR_OK;
}

// Single-process helpers (no collective): findSpotNodeForPod / canDrainNode.
static sr_status plan_local(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* cluster,
                            const sr_candidates* cands, sr_plan_out* out) {
  sr_status st = prepare(ctx, snap, cluster, cands);
  if (st != SR_OK) return st;
  return run(ctx, out, true, false);
}

sr_status sr_find_spot_nodes(sr_ctx* ctx, const sr_snapshot* snap, const sr_cluster* cluster, const int32_t* pods,
                             int32_t n, int32_t* out_spot_pos, uint8_t* out_fallback) {
  if (!ctx || !snap || !cluster || n < 0 || (n > 0 && (!pods || !out_spot_pos))) return SR_ERR_INVALID_ARG;
  if (n == 0) return SR_OK;
  std::vector<int32_t> off(static_cast<size_t>(n) + 1), status(n);
  for (int32_t i = 0; i <= n; ++i) off[i] = i;
  sr_candidates c{n, off.data(), pods, nullptr};
  sr_plan_out o{};
  o.status = status.data();
  o.node_of_pod = out_spot_pos;
  sr_status st = plan_local(ctx, snap, cluster, &c, &o);
  if (st != SR_OK) return st;
  if (out_fallback)
    for (int32_t i = 0; i < n; ++i) out_fallback[i] = status[i] == SR_CAND_FALLBACK ? 1 : 0;
  return SR_OK;
}

sr_status sr_can_drain_node(sr_ctx* ctx, sr_snapshot* snap, const sr_cluster* cluster, const int32_t* pods,
                            int32_t n, int32_t* out_node_of_pod, int32_t* out_fail_pod, uint8_t* out_fallback) {
  if (!ctx || !snap || !cluster || n < 0 || (n > 0 && !pods) || !out_fail_pod) return SR_ERR_INVALID_ARG;
  std::vector<int32_t> map(static_cast<size_t>(std::max(1, n)), -1);
  int32_t off[2] = {0, n}, status = SR_CAND_EMPTY;
  if (out_fallback) *out_fallback = 0;
  *out_fail_pod = -1;
  if (n > 0) {
    sr_candidates c{1, off, pods, nullptr};
    sr_plan_out o{};
    o.status = &status;
    o.node_of_pod = map.data();
    sr_status st = plan_local(ctx, snap, cluster, &c, &o);
    if (st != SR_OK) return st;
    if (status == SR_CAND_FALLBACK) {
      if (out_fallback) *out_fallback = 1;
      if (out_node_of_pod)
        for (int32_t i = 0; i < n; ++i) out_node_of_pod[i] = -1;
      return SR_OK;
    }
    *out_fail_pod = status >= 0 ? status : -1;
    // Side effect of the reference: every placed pod is added to the snapshot
    // (rescheduler.go:366), also those before a failing pod.
    for (int32_t i = 0; i < n; ++i)
      if (map[i] >= 0) sr::snapshot_add_pod(snap, cluster, pods[i], map[i]);
  }
  if (out_node_of_pod)
    for (int32_t i = 0; i < n; ++i) out_node_of_pod[i] = map[i];
  return SR_OK;
}

sr_status sr_set_timing(sr_ctx* ctx, int32_t mask) {
  if (!ctx) return SR_ERR_INVALID_ARG;
  sr_status st = flush_timing(ctx);
  if (st != SR_OK) return st;
  ctx->timing = mask & 7;
  ctx->timing_every = std::max(1, (mask >> 8) & 0xffff);
  ctx->timing_runs = 0;
  ctx->t.n_runs = 0;
  ctx->t.ms_tables = ctx->t.ms_placement = ctx->t.ms_winner = ctx->t.ms_collective = 0;
  return SR_OK;
}

sr_status sr_get_timing(sr_ctx* ctx, sr_timing* out) {
  if (!ctx || !out) return SR_ERR_INVALID_ARG;
  sr_status st = flush_timing(ctx);
  if (st != SR_OK) return st;
  *out = ctx->t;
  return SR_OK;
}

sr_status sr_comm_unique_id(uint8_t out[SR_UNIQUE_ID_BYTES]) {
  if (!out) return SR_ERR_INVALID_ARG;
  ncclUniqueId id;
  static_assert(sizeof(id) == SR_UNIQUE_ID_BYTES, "ncclUniqueId size");
  if (!rccl().ok || rccl().get_unique_id(&id) != ncclSuccess) return SR_ERR_RCCL;
  std::memcpy(out, &id, sizeof(id));
  return SR_OK;
}

sr_status sr_comm_init_shm(sr_ctx* ctx, const char* name, uint32_t session, int32_t nranks, int32_t rank,
                           int32_t max_cand) {
  if (!ctx || !name || name[0] != '/' || nranks < 1 || rank < 0 || rank >= nranks || max_cand < 1 ||
      max_cand > (1 << 28) || has_comm(ctx))
    return SR_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return SR_ERR_HIP;
  const size_t words = static_cast<size_t>(nranks) * 2 * (kShmHdr + 2 * static_cast<size_t>(max_cand));
  const size_t bytes = (words * sizeof(uint64_t) + 4095) & ~size_t(4095);
  const int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
  if (fd < 0) {
    ctx->err = std::string("shm_open(") + name + "): " + std::strerror(errno);
    return SR_ERR_RCCL;
  }
  struct stat sb;
  if (fstat(fd, &sb) != 0 || (sb.st_size != 0 && static_cast<size_t>(sb.st_size) != bytes) ||
      (sb.st_size == 0 && ftruncate(fd, static_cast<off_t>(bytes)) != 0)) {  // every rank sizes it alike
    ctx->err = std::string("shared segment ") + name + ": size mismatch or " + std::strerror(errno) +
               " (every rank passes the same nranks and max_cand)";
    close(fd);
    return SR_ERR_RCCL;
  }
  void* p = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    ctx->err = std::string("mmap: ") + std::strerror(errno);
    return SR_ERR_RCCL;
  }
  void* dp = nullptr;
  hipError_t e = hipHostRegister(p, bytes, hipHostRegisterMapped);
  if (e == hipSuccess) e = hipHostGetDevicePointer(&dp, p, 0);
  if (e != hipSuccess) {
    munmap(p, bytes);
    return hip_fail(ctx, e, "hipHostRegister(shared segment)");
  }
  auto& S = ctx->shm;
  S.host = static_cast<uint64_t*>(p);
  S.dev = static_cast<uint64_t*>(dp);
  S.bytes = bytes;
  S.max_cand = max_cand;
  S.session = session;
  S.tick = 0;
  S.name = name;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return SR_OK;
}

sr_status sr_comm_init_host(sr_ctx* ctx, int32_t nranks, int32_t rank, sr_allreduce_min_fn fn, void* user) {
  if (!ctx || !fn || nranks < 1 || rank < 0 || rank >= nranks || has_comm(ctx)) return SR_ERR_INVALID_ARG;
  ctx->host_fn = fn;
  ctx->host_user = user;
  ctx->nranks = nranks;
  ctx->rank = rank;
  return SR_OK;
}

sr_status sr_comm_init(sr_ctx* ctx, const uint8_t id[SR_UNIQUE_ID_BYTES], int32_t nranks, int32_t rank) {
  if (!ctx || !id || nranks < 1 || rank < 0 || rank >= nranks || has_comm(ctx)) return SR_ERR_INVALID_ARG;
  if (hipSetDevice(ctx->device) != hipSuccess) return SR_ERR_HIP;
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  if (!rccl().ok) {
    ctx->err = "RCCL (librccl.so) could not be loaded";
    return SR_ERR_RCCL;
  }
  ncclResult_t r = rccl().comm_init_rank(&ctx->comm, nranks, uid, rank);
  if (r != ncclSuccess) {
    ctx->err = std::string("ncclCommInitRank: ") + rccl().error_string(r);
    ctx->comm = nullptr;
    return SR_ERR_RCCL;
  }
  ctx->nranks = nranks;
  ctx->rank = rank;
  return SR_OK;
}

}  // extern "C"
