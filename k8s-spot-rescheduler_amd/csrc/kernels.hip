// kernels.hip — gfx950 (CDNA4, wave64) kernels of the drain planner.
//
//  K0 tables      S (static class) and T (capacity threshold) bitmask rows over
//                 spot nodes (predicate factorisation: encode.cpp); S rows by
//                 lanes = words from the class programs over the atom rows, T
//                 rows by lanes = rows against the nodes' free values.
//  K2 placement   canDrainNode for every candidate at once (rescheduler.go:357-370),
//                 one wave per candidate, with feasibility F = S & T & T & T:
//                  - node order (k2_node_order; the k2_node kernel when every
//                    candidate takes it): windows of 64 spot nodes visited in
//                    NodeInfoArray order, each at most once, the candidate's
//                    pods placed in it in pod order (lanes = nodes) -- the
//                    same first fit as pod by pod;
//                  - pod order (k2_run): candidates of more than 256 pods;
//                  - the domain path (k2_domain): pods interacting through
//                    shared topology domains (inter-pod (anti-)affinity).
//                 On one GPU each wave writes its outcome (and the first
//                 drainable mapping) straight to mapped host memory.
//  K3 winner      N GPUs: after the RCCL allreduce(min), the owning rank's
//                 first drainable candidate's pod -> node mapping.
//
// No MFMA: there is no dense contraction anywhere on this path.
#include <algorithm>
#include <climits>

#include "kernels.hpp"

#include <hip/hip_ext.h>

namespace sr {
namespace {

// Lane mask of `p` (the compare feeds the mask directly, no 0/1 round trip).
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v & 0xffffffffu), lane));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), lane));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

// Minimum over the 64 lanes with DPP row shifts / broadcasts (no LDS round trips).
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ int dpp_min(int v) {
  return min(v, __builtin_amdgcn_update_dpp(INT_MAX, v, CTRL, ROW_MASK, 0xf, false));
}
__device__ __forceinline__ int wave_min(int v) {
  v = dpp_min<0x111>(v);       // row_shr:1
  v = dpp_min<0x112>(v);       // row_shr:2
  v = dpp_min<0x114>(v);       // row_shr:4
  v = dpp_min<0x118>(v);       // row_shr:8  -> lane 15 of each row holds the row minimum
  v = dpp_min<0x142, 0xa>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_min<0x143, 0xc>(v);  // row_bcast:31 into rows 2, 3
  return __builtin_amdgcn_readlane(v, 63);
}

// A 64-bit lane value shifted by a DPP row shift / row broadcast (zero where
// nothing is shifted in): the steps of wave-wide scans without LDS.
template <int CTRL, int ROW_MASK = 0xf>
__device__ __forceinline__ uint64_t dpp_shifted(uint64_t v) {
  const uint32_t lo = static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(v)), CTRL, ROW_MASK, 0xf, true));
  const uint32_t hi = static_cast<uint32_t>(
      __builtin_amdgcn_update_dpp(0, static_cast<int>(static_cast<uint32_t>(v >> 32)), CTRL, ROW_MASK, 0xf, true));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
// One word of an S row from its class's 8-slot program and the program's atom
// words v[u] (AND, AND NOT, terms ORed with their atoms ANDed).
__device__ __forceinline__ uint64_t eval_prog8(const int (&op)[8], const uint64_t (&v)[8]) {
  uint64_t acc = ~0ull, any = 0, cur = 0;
  bool has = false;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    if (op[u] < 0) break;  // wave-uniform in K0; per lane in K2
    switch (op[u] & 3) {
      case PROG_AND: acc &= v[u]; break;
      case PROG_ANDNOT: acc &= ~v[u]; break;
      case PROG_TERM_START:
        any |= has ? cur : 0;
        cur = v[u];
        has = true;
        break;
      default: cur &= v[u]; break;
    }
  }
  if (has) acc &= any | cur;
  return acc;
}

constexpr int kSHead = 8;  // S-row words K0 writes when s_head_only (= K2's F head, kNH)

// K0: bitmask rows.  Blocks [0, s_blocks): S rows, kSClasses classes per
// wave, lanes = words; blocks after: T rows, lanes = rows.
constexpr int kSClasses = 2;  // S rows per wave: their atom loads are in flight together
constexpr int kTWords = 2;    // T row words per wave

// One S row by the class's atom program read through cls_prog_off (any length):
// 64 words (lanes) at a time, the program loaded lane-parallel, its atom words
// fetched 8 at a time.
__device__ void s_row_general(const DevWorkload& w, int cls, int lane) {
  const int o0 = w.cls_prog_off[cls], n = w.cls_prog_off[cls + 1] - o0;
  const size_t Wp = static_cast<size_t>(w.Wp);
  for (int wb = 0; wb < w.Wp; wb += 64) {
    const int word = wb + lane;
    const bool wv = word < w.Wp;
    const uint64_t* __restrict__ at = w.atoms + (wv ? word : 0);
    uint64_t acc = ~0ull, any = 0, cur = 0;
    bool has = false;
    for (int base = 0; base < n; base += 64) {
      const int m = min(64, n - base);
      const int my = lane < m ? w.cls_prog[o0 + base + lane] : 0;
      for (int j0 = 0; j0 < m; j0 += 8) {
        uint64_t v[8];
        int op[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          op[u] = __builtin_amdgcn_readlane(my, j0 + u);
          v[u] = j0 + u < m ? at[static_cast<size_t>(op[u] >> 2) * Wp] : 0;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          if (j0 + u >= m) break;
          switch (op[u] & 3) {
            case PROG_AND: acc &= v[u]; break;
            case PROG_ANDNOT: acc &= ~v[u]; break;
            case PROG_TERM_START:
              any |= has ? cur : 0;
              cur = v[u];
              has = true;
              break;
            default: cur &= v[u]; break;
          }
        }
      }
    }
    if (has) acc &= any | cur;
    if (wv) w.S[static_cast<size_t>(cls) * Wp + word] = acc;
  }
}

// What every K0 launch does besides its rows: the node patches (the few spot
// nodes changed since the generation the node section holds: written for K2;
// T rows read them directly), the pod patches (records a candidate-side reuse
// encode re-pointed; K2 reads pod_rec after this kernel, every thread of the
// grid takes a share) and the reset of d_min.
__device__ __forceinline__ void k0_common(const DevWorkload& w, int local_first_fallback, int wave, int lane) {
  if (blockIdx.x == 0 && wave == 0 && w.n_node_patch > 0 && lane < 11) {
    for (int p = 0; p < w.n_node_patch; ++p) {
      const uint64_t* pr = w.node_patch + static_cast<size_t>(p) * kNodePatchU64;
      const size_t node = static_cast<size_t>(pr[0]);
      if (lane < 8) const_cast<uint64_t*>(w.node_rec)[node * 8 + lane] = pr[1 + lane];
      else const_cast<int64_t*>(w.node_free)[static_cast<size_t>(lane - 8) * w.n_pad + node] =
          static_cast<int64_t>(pr[1 + lane]);
    }
  }
  for (int i = static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x); i < w.n_pod_patch;
       i += static_cast<int>(gridDim.x * blockDim.x)) {
    const uint64_t* pp = w.pod_patch + static_cast<size_t>(i) * kPodPatchU64;
    uint64_t* rec = const_cast<uint64_t*>(w.pod_rec) + static_cast<size_t>(pp[0]) * 6;
    rec[4] = pp[1];
    rec[5] = pp[2];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    unsigned long long* dm = reinterpret_cast<unsigned long long*>(w.d_min);
    dm[0] = ~0ull;
    dm[1] = local_first_fallback < 0 ? ~0ull : static_cast<unsigned long long>(local_first_fallback) << 32;
    dm[2] = w.rank_next;
  }
}

// Free value of spot position n in dimension d (1..3) with this launch's node
// patches applied (block 0 writes them into node_free; other waves may run
// first, so they read the patch itself).
__device__ __forceinline__ int64_t free_of(const DevWorkload& w, int d, int n) {
  int64_t v = w.node_free[static_cast<size_t>(d - 1) * w.n_pad + n];
  for (int p = 0; p < w.n_node_patch; ++p) {
    const uint64_t* pr = w.node_patch + static_cast<size_t>(p) * kNodePatchU64;
    if (static_cast<uint64_t>(n) == pr[0]) v = static_cast<int64_t>(pr[8 + d]);
  }
  return v;
}

__global__ __launch_bounds__(256) void k0_tables(DevWorkload w, int s_blocks, int local_first_fallback) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  // diagnostics: per-wave {start, end} (s_memrealtime) after K2's records
  const size_t pw = static_cast<size_t>(blockIdx.x) * 4 + wave;
  uint64_t* const prof = w.prof && pw < kK0ProfWaves ? w.prof + static_cast<size_t>(w.n_cand) * 16 + 2 * pw : nullptr;
  if (prof && lane == 0)  // bit 63: an S-row wave
    prof[0] = __builtin_amdgcn_s_memrealtime() | (static_cast<int>(blockIdx.x) < s_blocks ? 1ull << 63 : 0ull);
  struct Stamp {
    uint64_t* p;
    int lane;
    __device__ ~Stamp() {
      if (p && lane == 0) p[1] = __builtin_amdgcn_s_memrealtime();
    }
  } stamp{prof, lane};
  k0_common(w, local_first_fallback, wave, lane);
  const size_t Wp = static_cast<size_t>(w.Wp);
  if (static_cast<int>(blockIdx.x) < s_blocks) {
    // S rows (NodeAffinity: nodeSelector pairs, required terms ORed with
    // their requirements ANDed; TaintToleration + NodeUnschedulable + pod
    // count: the composite atom; NodePorts: the class's ports against the
    // base UsedPorts).  A program of <= 8 operations is one scalar load; the
    // atom words of both classes are loaded before either is evaluated.
    const int c0 = __builtin_amdgcn_readfirstlane((static_cast<int>(blockIdx.x) * 4 + wave) * kSClasses);
    int op[kSClasses][8];
#pragma unroll
    for (int q = 0; q < kSClasses; ++q) {
      const int cls = c0 + q;
      if (cls < w.n_classes) {
        const int4* p8 = reinterpret_cast<const int4*>(w.cls_prog8 + static_cast<size_t>(cls) * 8);
        const int4 a = p8[0], b = p8[1];
        op[q][0] = a.x; op[q][1] = a.y; op[q][2] = a.z; op[q][3] = a.w;
        op[q][4] = b.x; op[q][5] = b.y; op[q][6] = b.z; op[q][7] = b.w;
      } else {
        op[q][0] = -3;  // no class
#pragma unroll
        for (int u = 1; u < 8; ++u) op[q][u] = -1;
      }
    }
    // rows wider than 64 words (C4: 548): two 64-word chunks per round, all
    // their atom loads in flight together; with s_head_only just the head
    const int s_words = w.s_head_only ? min(w.Wp, kSHead) : w.Wp;
    for (int wb = 0; wb < s_words; wb += 128) {
      const bool two = wb + 64 < s_words;  // wave-uniform
      uint64_t v[2][kSClasses][8];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        const int word = wb + 64 * h + lane;
        const size_t wi = word < s_words ? static_cast<size_t>(word) : 0;
#pragma unroll
        for (int q = 0; q < kSClasses; ++q)
#pragma unroll
          for (int u = 0; u < 8; ++u)
            v[h][q][u] = op[q][u] >= 0 ? w.atoms[static_cast<size_t>(op[q][u] >> 2) * Wp + wi] : 0;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !two) break;
        const int word = wb + 64 * h + lane;
        const bool wv = word < s_words;
#pragma unroll
        for (int q = 0; q < kSClasses; ++q) {
          if (op[q][0] < 0 && op[q][0] != -1) continue;  // no class, or a long program (below)
          const uint64_t acc = eval_prog8(op[q], v[h][q]);
          if (wv) w.S[static_cast<size_t>(c0 + q) * Wp + word] = acc;
        }
      }
    }
#pragma unroll
    for (int q = 0; q < kSClasses; ++q)
      if (op[q][0] == -2) s_row_general(w, c0 + q, lane);
    return;
  }
  // T rows: one wave per (dimension, group of 64 rows, kTWords words), lanes
  // = rows.  Bit i of lane r's word W is free[64 W + i] >= threshold[r]: the
  // word's 64 free values are one coalesced load, each broadcast by a
  // readlane pair, and a node costs a 64-bit compare and a shift-or -- no
  // cross-lane ballots.  Pad nodes hold INT64_MIN and never pass.
  int tw = (static_cast<int>(blockIdx.x) - s_blocks) * 4 + wave;
  const int wgroups = (w.Wp + kTWords - 1) / kTWords;
  int d = 0;
  for (; d < 4; ++d) {
    const int waves_d = (w.t_off[d + 1] - w.t_off[d] + 63) / 64 * wgroups;
    if (tw < waves_d) break;
    tw -= waves_d;
  }
  if (d == 4) return;  // wave-uniform
  const int g = tw / wgroups;
  const int W0 = (tw - g * wgroups) * kTWords;
  const int r0 = w.t_off[d] + 64 * g;
  const int nr = min(64, w.t_off[d + 1] - r0);
  const int64_t thr = lane < nr ? w.t_thr[r0 + lane] : INT64_MAX;
#pragma unroll
  for (int ww = 0; ww < kTWords; ++ww) {
    const int W = W0 + ww;
    if (W >= w.Wp) break;  // wave-uniform
    uint64_t word;
    if (d == 0) {  // row 0: every node
      const int nvalid = max(0, min(64, w.n_spot - 64 * W));
      word = nvalid >= 64 ? ~0ull : (1ull << nvalid) - 1;
    } else {
      const uint64_t fv = static_cast<uint64_t>(free_of(w, d, 64 * W + lane));
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i) lo |= static_cast<uint32_t>(static_cast<int64_t>(readlane64(fv, i)) >= thr) << i;
#pragma unroll
      for (int i = 0; i < 32; ++i)
        hi |= static_cast<uint32_t>(static_cast<int64_t>(readlane64(fv, 32 + i)) >= thr) << i;
      word = static_cast<uint64_t>(hi) << 32 | lo;
    }
    if (lane < nr && thr != kTPad) w.T[static_cast<size_t>(r0 + lane) * Wp + W] = word;  // spare rows: unread
  }
}


// K0, incremental (a candidate-side reuse tick whose tables this slot's last
// run wrote): the class programs, atoms outside the changed word columns and
// every unmoved threshold are those the tables were built from, so only the
// word columns holding changed spot nodes (k0_cols) are recomputed, in every
// S row (lanes = classes) and T row (lanes = rows), and the T rows whose
// threshold moved (k0_rows) whole (lanes = words).  Waves [0, s_waves): S
// columns; then t_waves (dimension, 64-row group) waves; then one wave per
// moved row.
__global__ __launch_bounds__(256) void k0_incremental(DevWorkload w, int s_waves, int t_waves,
                                                      int local_first_fallback) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
  k0_common(w, local_first_fallback, wave, lane);
  const int wv = static_cast<int>(blockIdx.x) * 4 + wave;
  const size_t Wp = static_cast<size_t>(w.Wp);
  if (wv < s_waves) {
    const int cls = wv * 64 + lane;
    if (cls >= w.n_classes) return;
    const int s_words = w.s_head_only ? min(w.Wp, kSHead) : w.Wp;
    const int4* p8 = reinterpret_cast<const int4*>(w.cls_prog8 + static_cast<size_t>(cls) * 8);
    const int4 a = p8[0], b = p8[1];
    const int op[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    for (int c = 0; c < w.n_k0_cols; ++c) {
      const int W = w.k0_cols[c];
      if (W >= s_words) continue;
      uint64_t acc;
      if (op[0] == -2) {  // a long program, read through cls_prog_off
        acc = ~0ull;
        uint64_t any = 0, cur = 0;
        bool has = false;
        for (int o = w.cls_prog_off[cls]; o < w.cls_prog_off[cls + 1]; ++o) {
          const int x = w.cls_prog[o];
          const uint64_t v = w.atoms[static_cast<size_t>(x >> 2) * Wp + W];
          switch (x & 3) {
            case PROG_AND: acc &= v; break;
            case PROG_ANDNOT: acc &= ~v; break;
            case PROG_TERM_START:
              any |= has ? cur : 0;
              cur = v;
              has = true;
              break;
            default: cur &= v; break;
          }
        }
        if (has) acc &= any | cur;
      } else {
        uint64_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = op[u] >= 0 ? w.atoms[static_cast<size_t>(op[u] >> 2) * Wp + W] : 0;
        acc = eval_prog8(op, v);
      }
      w.S[static_cast<size_t>(cls) * Wp + W] = acc;
    }
    return;
  }
  int tw = wv - s_waves;
  if (tw < t_waves) {
    int d = 1;  // row 0 (every node) never changes
    for (; d < 4; ++d) {
      const int waves_d = (w.t_off[d + 1] - w.t_off[d] + 63) / 64;
      if (tw < waves_d) break;
      tw -= waves_d;
    }
    if (d == 4) return;  // wave-uniform
    const int r0 = w.t_off[d] + 64 * tw;
    const int nr = min(64, w.t_off[d + 1] - r0);
    const int64_t thr = lane < nr ? w.t_thr[r0 + lane] : INT64_MAX;
    for (int c = 0; c < w.n_k0_cols; ++c) {
      const int W = w.k0_cols[c];
      const uint64_t fv = static_cast<uint64_t>(free_of(w, d, 64 * W + lane));
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int i = 0; i < 32; ++i) lo |= static_cast<uint32_t>(static_cast<int64_t>(readlane64(fv, i)) >= thr) << i;
#pragma unroll
      for (int i = 0; i < 32; ++i)
        hi |= static_cast<uint32_t>(static_cast<int64_t>(readlane64(fv, 32 + i)) >= thr) << i;
      if (lane < nr && thr != kTPad) w.T[static_cast<size_t>(r0 + lane) * Wp + W] = static_cast<uint64_t>(hi) << 32 | lo;
    }
    return;
  }
  const int mr = tw - t_waves;
  if (mr >= w.n_k0_rows) return;
  const int row = w.k0_rows[mr];
  const int d = row < w.t_off[2] ? 1 : row < w.t_off[3] ? 2 : 3;
  const int64_t thr = w.t_thr[row];
  for (int W = lane; W < w.Wp; W += 64) {
    uint64_t word = 0;
    for (int i = 0; i < 64; ++i) word |= static_cast<uint64_t>(free_of(w, d, 64 * W + i) >= thr) << i;
    w.T[static_cast<size_t>(row) * Wp + W] = word;
  }
}


// K2: one wave per candidate.  Touched-node slots live in registers, one per
// lane (64; a candidate touching more distinct nodes is rerun with 512), and
// CH*64 bitmask words per row are held as a register-resident touched mask
// (lane l owns words ch*64 + l).
//
// The feasibility of pod p against the base snapshot is evaluated here: F =
// S[class] & T[cpu] & T[mem] & T[eph] (encode.cpp), whose rows are small and
// L2-resident, so no dense P x N bitmask is ever written.  First fit almost
// always lands on the first few spot nodes, so only the head of a pod's rows
// (32 words = 2048 nodes, 1 KB for all four rows) is prefetched; a pod with no
// answer in the head scans whole 64-word chunks synchronously (rare, and
// once per failing candidate).
//
// It is one dependent chain per candidate, so it is built for latency: every
// load inside the pod loop is an LDS-DMA (global_load_lds) whose completion
// is waited for by hand with counted `s_waitcnt vmcnt(N)`:
//   - the heads of pods k+1..k+7 are in flight (8-slot LDS ring, one DMA per
//     pod);
//   - the base record of the next pod's first untouched feasible node is
//     fetched one pod ahead (speculative; used when the pod opens a new slot
//     on a node >= kNodeCache; nodes below that come from an LDS cache);
//   - the candidate's pod records are staged before the loop (128-pod window,
//     restaged per 64 pods for larger candidates).
// DMA issue order: prologue heads 0..6, spec(0), head 7; then per step k:
// spec(k+1), head(k+8).  vmcnt(N) waits for all but the N youngest, so the
// head of pod k+1 at the end of step k needs N <= min(k + 7, 12) and spec(k)
// in step k needs N <= 1.  Rare-path DMAs are always followed by vmcnt(0),
// which never weakens a later count.
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) void* gbl_vp;
#define SR_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// Winner: d_min[0] = packed first drainable candidate (possibly reduced over
// ranks), d_min[1] = packed first fallback; the winner's mapping is copied
// only by the rank that owns it.  `result` lives in mapped host memory, one
// 64-bit word per value tagged with the run's sequence number.
__device__ __forceinline__ void write_winner(const DevWorkload& w) {
  const int lane = threadIdx.x & 63;
  const unsigned long long* dm = reinterpret_cast<const unsigned long long*>(w.d_min);
  const unsigned long long ok = __hip_atomic_load(dm, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long fb = __hip_atomic_load(dm + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long nx = __hip_atomic_load(dm + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint64_t* r = w.result;
  const bool any = ok != ~0ull;
  const int g = any ? static_cast<int>(ok >> 32) : -1;
  const int li = any ? static_cast<int>(ok & 0xffffffffu) : -1;
  const bool local = any && li < w.n_cand && w.cand_global[li] == g;
  const int off = local ? w.cand_off[li] : 0;
  const int np = local ? w.cand_off[li + 1] - off : 0;
  // every word carries the run's sequence number in its upper half: the host
  // accepts each word on its own tag, so no store has to wait for another
  const uint64_t tag = static_cast<uint64_t>(static_cast<uint32_t>(w.seq)) << 32;
  auto put = [&](int i, int v) {
    __hip_atomic_store(r + i, tag | static_cast<uint32_t>(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  for (int q = lane; q < np; q += 64)
    put(kResultHeader + q, __hip_atomic_load(w.out_node + off + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  if (lane == 0) put(0, g);
  if (lane == 1) put(1, local ? 1 : 0);
  if (lane == 2) put(2, np);
  if (lane == 3) put(3, fb == ~0ull ? -1 : static_cast<int>(fb >> 32));
  if (lane == 4) put(4, nx == ~0ull ? -1 : static_cast<int>(nx));
}

// K3: one wave (after the collective on multi-GPU runs).
__global__ __launch_bounds__(64) void k3_winner(DevWorkload w) { write_winner(w); }

// The bits a pod conflicts with, from the state bits it sets: anti-affinity
// pairs (A: has the term, B: selected by it) swapped, host-port bits as they
// are (encode.cpp / antiaff.cpp).  An involution.
__device__ __forceinline__ uint64_t swap_pairs(uint64_t x, uint64_t m) {
  const uint64_t y = x & m, e = 0x5555555555555555ull;
  return (x & ~m) | ((y & e) << 1) | ((y >> 1) & e);
}

constexpr int kHead = 32;       // head of a pod's rows prefetched per step: words [0, 32) = nodes [0, 2048)
constexpr int kRing = 8;        // head ring: pods k..k+7 (rows of pod k+8 issued at the end of step k)
constexpr int kPodWin = 128;    // pod records staged per wave: two 64-pod halves
constexpr int kRecU64 = 6;      // {cpu, memory, ephemeral, ports, S | T cpu row offset, T mem | T eph row offset}
constexpr int kNodeCache = 16;  // base records of spot nodes [0, 16) kept in LDS
constexpr int kMaxPods = 512;   // pods per candidate on the device (encode.cpp: more -> fallback)

struct K2Lds {
  uint64_t ring[kRing][4 * kHead];  // head of the {S, T cpu, T mem, T eph} rows of pods k..k+7
  uint64_t chunk[256];              // rare: a full 64-word chunk of the current pod's rows
  uint64_t pods[kPodWin][kRecU64];  // pod record window
  uint64_t cache[kNodeCache][8];    // base node records
  uint64_t spec[8];                 // speculative node record
  uint64_t rec[8];                  // rare: reloaded node record
  int32_t omap[kMaxPods];           // spot position chosen for each pod
};

struct K2Stats {
  uint32_t n_spec_miss = 0, n_min = 0, n_far = 0;
  uint64_t cyc_a = 0, cyc_b = 0, cyc_c = 0, cyc_d = 0;
  uint64_t cyc_rec = 0;  // node order (profile builds): wave entry -> pod records in registers
  uint32_t narrow = 0;   // node order: the candidate's window visits use 32-bit scaled state
  uint64_t cyc_res = 0;  // node order: far-pointer resolution cycles (part of cyc_b) | chunk rounds << 40 | pods
                         // found dead << 56
  uint64_t cyc_win = 0;  // node order: window record loads waited for (part of cyc_b)
};

// One candidate's canDrainNode with 64 * SPL touched-node slots.  Returns the
// number of pods placed (np = all; status = failing pod or -1), or -1 when the
// candidate touches more distinct nodes than it has slots (the caller reruns
// it with more).
// EXT: the candidate has extension records at pod_ext[ebase ..] (the running
// state subtracts NodeInfo.AddPod's accounting instead of the fit request, and
// keeps up to two shared scalar resources per touched node).
template <int SPL, int CH, bool PROF, bool EXT = false>
__device__ __forceinline__ int k2_run(const DevWorkload& w, K2Lds& L, const int p0, const int np, int& status,
                                      K2Stats& st, uint32_t& nbytes, const int ebase = -1) {
  const int lane = threadIdx.x & 63;
  const int Wp = w.Wp;
  const uint64_t* __restrict__ tab = w.S;  // S rows then T rows: pod records hold word offsets

  // DMA helpers: 16 B per lane, LDS destination = base + 16 * lane
  auto dma = [&](const uint64_t* src, uint64_t* dst) {
    __builtin_amdgcn_global_load_lds((gbl_vp)src, (lds_vp)dst, 16, 0, 0);
  };
  // 64 words from word `base` of the four rows at offsets {r01.lo, r01.hi, r23.lo, r23.hi} -> dst[4][64]
  auto dma_rows = [&](uint64_t* dst, uint64_t r01, uint64_t r23, int base) {
    const uint32_t wi = static_cast<uint32_t>(min(base + 2 * (lane & 31), Wp - 2));
    const uint32_t ra = lane < 32 ? static_cast<uint32_t>(r01) : static_cast<uint32_t>(r01 >> 32);
    const uint32_t rb = lane < 32 ? static_cast<uint32_t>(r23) : static_cast<uint32_t>(r23 >> 32);
    dma(tab + (static_cast<uint64_t>(ra) + wi), dst);
    dma(tab + (static_cast<uint64_t>(rb) + wi), dst + 128);
  };
  auto dma_rows_of = [&](uint64_t* dst, int q, int base) {
    const uint64_t* pr = L.pods[q & (kPodWin - 1)];
    dma_rows(dst, pr[4], pr[5], base);
  };
  // head (kHead words) of the four rows: 16 lanes per row, one DMA -> dst[4][kHead]
  auto dma_head = [&](uint64_t* dst, uint64_t r01, uint64_t r23) {
    const int r = lane >> 4;
    const uint32_t wi = static_cast<uint32_t>(min(2 * (lane & 15), Wp - 2));
    const uint64_t rr = r < 2 ? r01 : r23;
    const uint32_t off = (r & 1) ? static_cast<uint32_t>(rr >> 32) : static_cast<uint32_t>(rr);
    dma(tab + (static_cast<uint64_t>(off) + wi), dst);
  };
  auto dma_head_of = [&](uint64_t* dst, int q) {
    const uint64_t* pr = L.pods[q & (kPodWin - 1)];
    dma_head(dst, pr[4], pr[5]);
  };
  auto dma_rec = [&](uint64_t* dst, int node) {
    if (lane < 4) dma(w.node_rec + static_cast<size_t>(node == INT_MAX ? 0 : node) * 8 + 2 * lane, dst);
  };
  // records of pods [64 m, 64 m + 64) into window half m & 1 (pod_rec is padded)
  auto dma_pods = [&](int m) {
    const uint64_t* src = w.pod_rec + static_cast<size_t>(p0 + 64 * m) * kRecU64 + 2 * lane;
    uint64_t* dst = L.pods[64 * (m & 1)];
#pragma unroll
    for (int j = 0; j < 3; ++j) dma(src + 128 * j, dst + 128 * j);
  };

  uint64_t touched[CH];
#pragma unroll
  for (int ch = 0; ch < CH; ++ch) touched[ch] = 0;
  int snode[SPL];
  int64_t scpu[SPL], smem[SPL], seph[SPL];
  int sleft[SPL];
  uint64_t sport[SPL];
  int64_t ss0[SPL], ss1[SPL];  // EXT: shared scalar resources' running free values
#pragma unroll
  for (int s = 0; s < SPL; ++s) {
    snode[s] = INT_MAX;
    scpu[s] = smem[s] = seph[s] = 0;
    sleft[s] = 0;
    sport[s] = 0;
    ss0[s] = ss1[s] = 0;
  }
  // EXT: the scalar slots' node_scal rows (uniform over the candidate's records)
  const uint64_t erow = EXT ? w.pod_ext[static_cast<size_t>(ebase) * kDevExtU64 + 7] : ~0ull;
  const int erow0 = static_cast<int32_t>(static_cast<uint32_t>(erow)), erow1 = static_cast<int32_t>(erow >> 32);
  int nslots = 0;
  uint64_t cyc_t = 0;
  auto cyc = [&]() -> uint64_t { return PROF ? __builtin_amdgcn_s_memtime() : 0ull; };
  const uint64_t lane_mask = lane < min(Wp, kHead) ? ~0ull : 0ull;

  // State of the next pod, gathered in one batch of LDS reads once its head
  // has landed: its head feasibility word, first untouched feasible node in
  // the head, request, and the S-row bit of every touched node in the head.
  uint64_t word_next = 0;
  int cnode0 = INT_MAX;
  int64_t nrc = 0, nrm = 0, nre = 0;
  uint64_t npm = 0;
  int64_t nac = 0, nam = 0, nae = 0, nsr0 = INT64_MIN, nsr1 = INT64_MIN, nsa0 = 0, nsa1 = 0;  // EXT record
  bool sbit[SPL];
  auto gather_next = [&](int kn) {
    if (EXT) {  // uniform: scalar loads, consumed by the next step
      const uint64_t* er = w.pod_ext + static_cast<size_t>(ebase + kn) * kDevExtU64;
      nac = static_cast<int64_t>(er[0]);
      nam = static_cast<int64_t>(er[1]);
      nae = static_cast<int64_t>(er[2]);
      nsr0 = static_cast<int64_t>(er[3]);
      nsr1 = static_cast<int64_t>(er[4]);
      nsa0 = static_cast<int64_t>(er[5]);
      nsa1 = static_cast<int64_t>(er[6]);
    }
    const uint64_t* img = L.ring[kn & (kRing - 1)];
    const uint64_t* pr = L.pods[kn & (kPodWin - 1)];
    uint64_t sw[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) sw[s] = img[snode[s] < 64 * kHead ? snode[s] >> 6 : 0];
    const int hl = lane & (kHead - 1);
    const uint64_t a = img[hl] & img[kHead + hl] & img[2 * kHead + hl] & img[3 * kHead + hl];
    nrc = static_cast<int64_t>(pr[0]);
    nrm = static_cast<int64_t>(pr[1]);
    nre = static_cast<int64_t>(pr[2]);
    npm = pr[3];
#pragma unroll
    for (int s = 0; s < SPL; ++s) sbit[s] = (sw[s] >> (snode[s] & 63)) & 1ull;
    word_next = a & lane_mask;
    const uint64_t clean0 = word_next & ~touched[0];
    const uint64_t mc0 = ballot(clean0 != 0);
    cnode0 = INT_MAX;
    if (mc0) {
      const int L0 = __builtin_ctzll(mc0);
      cnode0 = L0 * 64 + __builtin_ctzll(readlane64(clean0, L0));
    }
  };

  // prologue: node cache + pod window, then heads 0..6, (head 0 landed)
  // spec(0), head 7.  DMA order per step k afterwards: spec(k+1), head(k+8).
  static_assert(kRing == 8, "the vmcnt immediates below assume an 8-deep ring");
  dma(w.node_rec + 2 * lane, L.cache[0]);
  dma_pods(0);
  if (np > 64) dma_pods(1);
  // bytes moved (algorithmic, wave-uniform): node cache, pod records, per
  // step the head DMA (4 rows x kHead words) and the speculative record, rare
  // chunk scans and record reloads, the mapping and status writes
  nbytes += 64u * kNodeCache + (48u + 4u) * static_cast<uint32_t>(np) + 4u;
  SR_WAIT_VM(0);
#pragma unroll
  for (int j = 0; j < kRing - 1; ++j) dma_head_of(L.ring[j], min(j, np - 1));
  SR_WAIT_VM(6);  // head 0: heads 1..6 are younger
  gather_next(0);
  dma_rec(L.spec, cnode0);
  dma_head_of(L.ring[kRing - 1], min(kRing - 1, np - 1));

  status = -1;
  int k = 0;
  for (; k < np; ++k) {
    if (PROF) cyc_t = cyc();
    nbytes += 4u * kHead * 8u + 64u + (EXT ? 64u : 0u);  // this pod's head, speculative record (and extension)
    const int64_t rc = nrc, rm = nrm, re = nre;
    // what AddPod subtracts (EXT: calculateResource, else the fit request) and
    // the shared scalars' fit requests / accounting
    const int64_t ac = EXT ? nac : rc, am = EXT ? nam : rm, ae = EXT ? nae : re;
    const int64_t sr0 = nsr0, sr1 = nsr1, sa0 = nsa0, sa1 = nsa1;
    const uint64_t pm = npm;                          // state bits the pod sets
    const uint64_t pin = swap_pairs(pm, w.swap_mask);  // ... and those it conflicts with
    const bool zero = (rc | rm | re) == 0;  // fitsRequest skips the resource checks
    // Head (spot nodes [0, 2048)): touched nodes below the first untouched
    // feasible one, rechecked branch-free: class bit from the S row, capacity /
    // pod count / host ports from the candidate's own state (which implies the
    // base T rows, base pod count and base ports).
    int ans;
    {
      const int hi = min(cnode0, 64 * kHead);
      int best = INT_MAX;
#pragma unroll
      for (int s = 0; s < SPL; ++s) {
        const int nd = snode[s];
        const bool fit = (zero | ((rc <= scpu[s]) & (rm <= smem[s]) & (re <= seph[s]))) &  // NodeResourcesFit
                         (!EXT | ((sr0 <= ss0[s]) & (sr1 <= ss1[s])));
        const bool ok = (nd < hi) & sbit[s] & (sleft[s] >= 1) & ((sport[s] & pin) == 0) & fit;
        best = ok ? min(best, nd) : best;
      }
      const uint64_t hb = ballot(best != INT_MAX);
      int dnode = INT_MAX;
      if (hb) {
        dnode = (hb & (hb - 1)) ? wave_min(best) : __builtin_amdgcn_readlane(best, __builtin_ctzll(hb));
        if (PROF && (hb & (hb - 1))) ++st.n_min;
      }
      ans = min(cnode0, dnode);
    }
    // rare: nothing in the head; scan whole 64-word chunks (the head again
    // included, which cannot change the outcome)
    if (ans == INT_MAX && Wp > kHead) {
#pragma unroll
      for (int ch = 0; ch < CH; ++ch) {
        const int base = ch * 64;
        if (ans != INT_MAX || base >= Wp) continue;  // wave-uniform; keeps the loop unrollable
        if (PROF) ++st.n_far;
        nbytes += 4u * 64u * 8u;
        dma_rows_of(L.chunk, k, base);
        SR_WAIT_VM(0);
        const uint64_t* img = L.chunk;
        const uint64_t clean = (img[lane] & img[64 + lane] & img[128 + lane] & img[192 + lane]) &
                               ((base + lane < Wp) ? ~touched[ch] : 0ull);
        const uint64_t mc = ballot(clean != 0);
        int cnode = INT_MAX;
        if (mc) {
          const int L0 = __builtin_ctzll(mc);
          cnode = (base + L0) * 64 + __builtin_ctzll(readlane64(clean, L0));
        }
        const int lo = base * 64;
        const int hi = min(cnode, lo + 64 * 64);
        int best = INT_MAX;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          const int nd = snode[s];
          const bool in = (nd >= lo) & (nd < hi);
          const uint64_t sw = img[in ? (nd >> 6) - base : 0];
          const bool fit = (zero | ((rc <= scpu[s]) & (rm <= smem[s]) & (re <= seph[s]))) &
                           (!EXT | ((sr0 <= ss0[s]) & (sr1 <= ss1[s])));
          const bool ok =
              in & (((sw >> (nd & 63)) & 1ull) != 0) & (sleft[s] >= 1) & ((sport[s] & pin) == 0) & fit;
          best = ok ? min(best, nd) : best;
        }
        ans = min(cnode, wave_min(best));
      }
    }
    if (PROF) {
      const uint64_t t = cyc();
      st.cyc_a += t - cyc_t;
      cyc_t = t;
    }
    if (ans == INT_MAX) {  // "pod %s can't be rescheduled on any existing spot node"
      status = k;
      break;
    }
    if (lane == 0) L.omap[k] = ans;

    // ClusterSnapshot.AddPod(pod, node) on the candidate's private copy
    bool hit = false;
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
      if (snode[s] == ans) {
        scpu[s] -= ac;
        smem[s] -= am;
        seph[s] -= ae;
        sleft[s] -= 1;
        sport[s] |= pm;
        if (EXT) {
          ss0[s] -= sa0;
          ss1[s] -= sa1;
        }
        hit = true;
      }
    }
    if (!(ballot(hit) != 0)) {
      const int ns = nslots++;
      if (ns >= 64 * SPL) {  // slots exhausted: rerun with more
        SR_WAIT_VM(0);
        return -1;
      }
      // EXT: the node's base free value of each shared scalar (0: no slot)
      const int64_t b0 = EXT && erow0 >= 0 ? w.node_scal[static_cast<size_t>(erow0) * w.n_pad + ans] : 0;
      const int64_t b1 = EXT && erow1 >= 0 ? w.node_scal[static_cast<size_t>(erow1) * w.n_pad + ans] : 0;
      const uint64_t* rec;
      if (ans < kNodeCache) {
        rec = L.cache[ans];
      } else if (ans == cnode0) {
        SR_WAIT_VM(1);  // spec(k): only head(k+7) is younger
        rec = L.spec;
      } else {  // rare: not the speculated node
        if (PROF) ++st.n_spec_miss;
        nbytes += 64u;
        dma_rec(L.rec, ans);
        SR_WAIT_VM(0);
        rec = L.rec;
      }
      const int64_t fc = static_cast<int64_t>(rec[0]), fm = static_cast<int64_t>(rec[1]),
                    fe = static_cast<int64_t>(rec[2]);
      const uint64_t pb = rec[3];
      const int pl = static_cast<int>(static_cast<int64_t>(rec[4]));
#pragma unroll
      for (int s = 0; s < SPL; ++s) {
        if ((s == (ns >> 6)) & (lane == (ns & 63))) {
          snode[s] = ans;
          scpu[s] = fc - ac;
          smem[s] = fm - am;
          seph[s] = fe - ae;
          sleft[s] = pl - 1;
          sport[s] = pb | pm;
          if (EXT) {
            ss0[s] = b0 - sa0;
            ss1[s] = b1 - sa1;
          }
        }
      }
      const int tw = ans >> 6;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch)
        if (tw == ch * 64 + lane) touched[ch] |= 1ull << (ans & 63);
    }
    if (PROF) {
      const uint64_t t = cyc();
      st.cyc_b += t - cyc_t;
      cyc_t = t;
    }
    // next pod: its head (issued at the end of step k - 6: min(k + 7, 12)
    // younger DMAs), its state, its speculative record, head of pod k + 8
    if (k + 1 < np) {
      const int q = min(k + kRing, np - 1);
      const bool restage = q == k + kRing && (q & 63) == 0 && q >= kPodWin;
      if (restage) {  // window: records [q, q + 64) replace [q - 128, q - 64)
        dma_pods(q >> 6);
        SR_WAIT_VM(0);
      } else if (k >= 5) {
        SR_WAIT_VM(12);
      } else {
        SR_WAIT_VM(7);
      }
      if (PROF) {
        const uint64_t t = cyc();
        st.cyc_c += t - cyc_t;
        cyc_t = t;
      }
      const uint64_t* pq = L.pods[q & (kPodWin - 1)];
      const uint64_t r01 = pq[4], r23 = pq[5];
      gather_next(k + 1);
      dma_rec(L.spec, cnode0);  // L.spec's last reads (this step) have returned
      dma_head(L.ring[k & (kRing - 1)], r01, r23);
      if (PROF) st.cyc_d += cyc() - cyc_t;
    }
  }
  SR_WAIT_VM(0);  // no LDS-DMA may outlive the wave's LDS allocation
  return status >= 0 ? status : np;
}

// ------------------------------------------------------------ K2, node order
// First fit in pod order (canDrainNode) equals first fit in WINDOW order: visit
// the spot nodes 64 at a time (windows of NodeInfoArray order) and, in window
// W, place the candidate's pods not yet placed, in pod order, each on its first
// node of W that fits W's running state.  Every encoded predicate is
// node-local (a node's answer for pod k depends only on the candidate's pods
// already placed on that node), so by induction over k both orders place pod
// k on the same node: a pod placed in an earlier window never touched W, and
// inside W the pods meet W's nodes in pod order, as canDrainNode presents
// them.  Each window is therefore visited at most once, and only windows with
// base-feasible nodes (F = S & T & T & T) are worth visiting; a pod whose F
// row has no bit left can never be placed: it is the failing pod once every
// lower pod is placed, and pods above it are irrelevant (canDrainNode stops).
//
// One wave per candidate with <= 64 * G pods (G <= 4); lane l holds pods l,
// 64 + l, ... (group g = pod / 64):
//   prologue  pods whose S row is certainly empty (the encoder points them at
//             the all-zero class) bound the pods that matter; the F row head
//             (kNH words = 512 nodes) of each of those, 8 pods per load
//             instruction (lanes = pod x word), goes to LDS, the pod's lane
//             keeps its 8-bit mask of non-zero head words;
//   visits    n = min pointer over unplaced pods (DPP wave-min), W = n / 64;
//             the base records of W's 64 nodes in one register per field
//             (lanes = nodes), updated in place; the pods pointing into W one
//             by one (place_window: its F word of W & ballots of the compares
//             against the running state, the first set lane, the update of
//             that lane); pods that did not fit move their pointer to the
//             first set bit of their F row beyond W.  A pod whose head holds
//             no further bit points at kFar, the first chunk boundary: an
//             unresolved pointer.  When the minimum reaches an unresolved
//             pointer, its pods scan their rows from there, 64 words per round
//             (lanes = words), which leaves a mask of the chunk's non-zero
//             words for later moves; a mask that runs out makes the pointer
//             the next chunk boundary, unresolved.
// The chain is one step per pod plus one window load per visited window
// (C3: 1.06 windows per candidate); no step touches global memory unless the
// window moves or a pointer moves beyond the head.  Measured against visiting
// one node at a time (prefix-sum run passes over the pods pointing at it):
// C3 K2 17.7 -> 13.1 us, C5 61 -> 42 us.
// F head words per pod kept in LDS (8: nodes [0, 512); measured against 4 and 2: DESIGN §4)
constexpr int kNH = 8;
static_assert(kNH == 2 || kNH == 4 || kNH == 8, "head words per pod: a power of two up to 8 (8-bit head masks)");
constexpr int kNHS = kNH + 1;      // LDS stride per pod (odd number of words: conflict-free b64 reads)
constexpr int kFar = 64 * kNH;     // pointer sentinel: next feasible node lies at or beyond the head, unresolved

// Word `wd` of the lane's own F row, straight from the tables.
__device__ __forceinline__ uint64_t f_word_far(const uint64_t* __restrict__ tab, uint64_t r01, uint64_t r23, int wd) {
  return tab[static_cast<uint32_t>(r01) + wd] & tab[static_cast<uint32_t>(r01 >> 32) + wd] &
         tab[static_cast<uint32_t>(r23) + wd] & tab[static_cast<uint32_t>(r23 >> 32) + wd];
}

// The S part alone, from the lane's class program (s_head_only).
__device__ __forceinline__ uint64_t f_word_prog_s(const DevWorkload& w, const int32_t* pg, int wd) {
  int op[8];
  uint64_t v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) op[u] = pg[u];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = op[u] >= 0 ? w.atoms[static_cast<size_t>(op[u] >> 2) * w.Wp + wd] : 0ull;
  return eval_prog8(op, v);
}

// The same word with the S part evaluated from the lane's class program (in
// LDS) when K0 wrote only the heads of the S rows (s_head_only).
__device__ __forceinline__ uint64_t f_word_prog(const DevWorkload& w, const uint64_t* __restrict__ tab,
                                                const int32_t* pg, uint64_t r01, uint64_t r23, int wd) {
  int op[8];
  uint64_t v[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) op[u] = pg[u];
#pragma unroll
  for (int u = 0; u < 8; ++u) v[u] = op[u] >= 0 ? w.atoms[static_cast<size_t>(op[u] >> 2) * w.Wp + wd] : 0ull;
  return eval_prog8(op, v) & tab[static_cast<uint32_t>(r01 >> 32) + wd] & tab[static_cast<uint32_t>(r23) + wd] &
         tab[static_cast<uint32_t>(r23 >> 32) + wd];
}

// A K0-less run (k0_skip): the T rows predate the changes of the spot nodes
// in node_patch, so their bits of an F word (S & T rows) are recomputed from
// the S word and the nodes' current free values (fitsRequest per dimension;
// an all-zero request skips it).  Every other node's T bits stand: its free
// value is the one the rows were built from, and no node value then lay
// between a request and its row's threshold.
__device__ __forceinline__ uint64_t fix_dirty(const DevWorkload& w, uint64_t f, uint64_t s, int wd, int64_t rc,
                                              int64_t rm, int64_t re, bool zero) {
  for (int p = 0; p < w.n_dirty; ++p) {
    const int n = w.dirty_node[p];
    if ((n >> 6) != wd) continue;
    const uint64_t bit = 1ull << (n & 63);
    const bool fits = zero || (w.dirty_free[p][0] >= rc && w.dirty_free[p][1] >= rm && w.dirty_free[p][2] >= re);
    f = fits ? (f | (s & bit)) : (f & ~bit);
  }
  return f;
}

// A K0-less run: lane i's base record of window W from node_patch when node
// 64 W + i changed since the node section was written.
__device__ __forceinline__ void window_patch(const DevWorkload& w, int W, int lane, int64_t& ncpu, int64_t& nmem,
                                             int64_t& neph, uint64_t& nport, int& nleft) {
  for (int p = 0; p < w.n_node_patch; ++p) {
    const uint64_t* pr = w.node_patch + static_cast<size_t>(p) * kNodePatchU64;
    if (static_cast<int>(pr[0]) != 64 * W + lane) continue;
    ncpu = static_cast<int64_t>(pr[1]);
    nmem = static_cast<int64_t>(pr[2]);
    neph = static_cast<int64_t>(pr[3]);
    nport = pr[4];
    nleft = static_cast<int>(static_cast<int64_t>(pr[5]));
  }
}

// 32-bit value of lane `src` (per-lane source index), through the LDS crossbar.
__device__ __forceinline__ uint32_t from_lane(uint32_t v, int src) {
  return static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(src << 2, static_cast<int>(v)));
}

// Window visit (node order): the pods of `todo` (lanes of one
// pod group, in pod order; pods k >= kmax are irrelevant) placed one by one,
// each on its first node of window W (its F word `cur` there) that fits the
// running state of the window's nodes (lanes = nodes: NodeResourcesFit's
// compares, the pod-count limit, the NodePorts / anti-affinity state bits),
// which the placement then updates as ClusterSnapshot.AddPod would.  E: some
// pod of the candidate asks for ephemeral storage (otherwise the ephemeral
// check is the fixed `emask`); O: some pod sets or meets state bits.
// v_writelane_b32: lane k of v becomes the scalar x (two instructions where a
// compare-and-select per pod took three; the lane select goes through m0, as
// two SGPR operands exceed the constant bus); x and k wave-uniform
// (m0 is a reserved register: the clobber tells the compiler it changed but
// nothing preserves a value it held; no other instruction of these kernels
// reads m0 -- checked in the ISA of every part)
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ int writelane(int v, int x, int k) {
  asm("s_mov_b32 m0, %2\n\tv_writelane_b32 %0, %1, m0" : "+v"(v) : "s"(x), "s"(k) : "m0");
  return v;
}
#pragma clang diagnostic pop
// s_ff1_i32_b64: the lowest set bit of a scalar mask, -1 when it is zero (the
// compiler's ctz of a maybe-zero value adds a compare and a select)
__device__ __forceinline__ int ff1(uint64_t x) {
  int r;
  asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(x));
  return r;
}
// s_bitset0_b64: clear bit k of a scalar mask (one op for shift + andn2)
__device__ __forceinline__ uint64_t bitclear(uint64_t x, int k) {
  asm("s_bitset0_b64 %0, %1" : "+s"(x) : "s"(k));
  return x;
}

template <bool E, bool O>
__device__ __forceinline__ uint64_t place_window(uint64_t todo, int kmax, int W, int lane, int64_t rc, int64_t rm,
                                                 int64_t re, uint64_t pm, uint64_t cur, uint64_t zm,
                                                 uint64_t swap_mask, uint64_t emask, int64_t& ncpu, int64_t& nmem,
                                                 int64_t& neph, uint64_t& nport, int& nleft, int& node) {
  // jv: the lane each pod took (64: none), turned into node / placed once per
  // visit (measured: the bookkeeping in the step costs ~14% of a step)
  int jv = 64;
  if (kmax < 64) todo &= kmax <= 0 ? 0ull : (1ull << kmax) - 1;
  // without state bits one branch per pod: a pod that fits nowhere selects
  // lane -1 (no lane; jv keeps 64 for a pod not stepped)
  while (todo != 0) {
    const int k = __builtin_ctzll(todo);
    todo = bitclear(todo, k);  // s_bitset0: one scalar op (todo &= todo - 1 takes two)
    const int64_t c = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rc), k));
    const int64_t m = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rm), k));
    const int64_t e = E ? static_cast<int64_t>(readlane64(static_cast<uint64_t>(re), k)) : 0;
    const uint64_t q = O ? readlane64(pm, k) : 0ull;
    uint64_t fit = readlane64(cur, k) & ballot(nleft >= 1);
    const uint64_t res = ballot(ncpu >= c) & ballot(nmem >= m) & (E ? ballot(neph >= e) : emask);
    fit &= ((zm >> k) & 1) ? ~0ull : res;  // fitsRequest skips the resource checks
    if (O) fit &= ballot((nport & q) == 0);
    if (O) {  // measured: with state bits the update is cheaper behind a branch (C5)
      if (fit != 0) {
        const int j = __builtin_ctzll(fit);
        if (lane == j) {  // ClusterSnapshot.AddPod on the candidate's copy of node 64 W + j
          ncpu -= c;
          nmem -= m;
          if (E) neph -= e;
          nleft -= 1;
          nport |= swap_pairs(q, swap_mask);  // the bits it sets
        }
        jv = writelane(jv, j, k);  // pod k took lane j
      }
      continue;
    }
    const int j = ff1(fit);  // -1 when it fits nowhere (no lane)
    const bool hit = lane == j;  // ClusterSnapshot.AddPod on the candidate's copy of node 64 W + j
    ncpu -= hit ? c : 0;
    nmem -= hit ? m : 0;
    if (E) neph -= hit ? e : 0;
    nleft -= hit ? 1 : 0;
    jv = writelane(jv, j, k);  // pod k took lane j
  }
  const bool took = static_cast<unsigned>(jv) < 64u;  // -1 / 64: no lane
  node = took ? 64 * W + jv : node;
  return ballot(took);
}

// Extension-record values of a pod (XT candidates, lanes = pods): what
// NodeInfo.AddPod adds to Requested (calculateResource: no init containers),
// and per shared scalar slot the fit request (INT64_MIN / INT_MIN: the pod does
// not list the name) and the accounting.  64-bit, or scaled to 32 bits for
// narrow candidates (cpu / memory / ephemeral by the candidate's granularity,
// scalars unscaled).
template <typename T>
struct XVals {
  T ac, am, ae, r0, r1, a0, a1;
};

// place_window for an XT candidate.  The interaction stays node-local (AddPod
// changes only the chosen node: rescheduler.go:366), so window order still
// equals pod order; the running state of a window's node subtracts the
// accounting instead of the request and keeps the node's two shared scalar
// slots (ns0 / ns1: allocatable - requested, from node_scal), checked against
// the pod's scalar requests whatever its cpu / memory / ephemeral request
// (volume limits have no zero-request exemption; a zero-request pod listing
// an extended resource never reaches the device).
template <bool E, bool O>
__device__ __forceinline__ uint64_t place_window_x(uint64_t todo, int kmax, int W, int lane, int64_t rc, int64_t rm,
                                                   int64_t re, const XVals<int64_t>& x, uint64_t pm, uint64_t cur,
                                                   uint64_t zm, uint64_t swap_mask, uint64_t emask, int64_t& ncpu,
                                                   int64_t& nmem, int64_t& neph, uint64_t& nport, int& nleft,
                                                   int64_t& ns0, int64_t& ns1, int& node) {
  int jv = 64;
  if (kmax < 64) todo &= kmax <= 0 ? 0ull : (1ull << kmax) - 1;
  while (todo != 0) {
    const int k = __builtin_ctzll(todo);
    todo = bitclear(todo, k);
    const int64_t c = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rc), k));
    const int64_t m = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rm), k));
    const int64_t e = E ? static_cast<int64_t>(readlane64(static_cast<uint64_t>(re), k)) : 0;
    const int64_t r0 = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.r0), k));
    const int64_t r1 = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.r1), k));
    const uint64_t q = O ? readlane64(pm, k) : 0ull;
    uint64_t fit = readlane64(cur, k) & ballot(nleft >= 1) & ballot(ns0 >= r0) & ballot(ns1 >= r1);
    const uint64_t res = ballot(ncpu >= c) & ballot(nmem >= m) & (E ? ballot(neph >= e) : emask);
    fit &= ((zm >> k) & 1) ? ~0ull : res;  // fitsRequest skips the cpu / memory / ephemeral checks
    if (O) fit &= ballot((nport & q) == 0);
    if (fit != 0) {
      const int j = __builtin_ctzll(fit);
      const int64_t ac = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.ac), k));
      const int64_t am = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.am), k));
      const int64_t ae = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.ae), k));
      const int64_t a0 = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.a0), k));
      const int64_t a1 = static_cast<int64_t>(readlane64(static_cast<uint64_t>(x.a1), k));
      if (lane == j) {  // ClusterSnapshot.AddPod: Requested grows by calculateResource
        ncpu -= ac;
        nmem -= am;
        neph -= ae;
        nleft -= 1;
        ns0 -= a0;
        ns1 -= a1;
        if (O) nport |= swap_pairs(q, swap_mask);
      }
      jv = writelane(jv, j, k);  // pod k took lane j
    }
  }
  const bool took = static_cast<unsigned>(jv) < 64u;  // -1 / 64: no lane
  node = took ? 64 * W + jv : node;
  return ballot(took);
}

// The free value f of a node scaled to the candidate's request granularity
// 2^k (narrow candidates): f >> k, or -1 when f < 0 (no request fits, zero
// included, as with the 64-bit compare).  Values at or above 2^31 are
// clamped: every sum of the candidate's scaled requests stays below 2^31
// (Narrow), so a clamped node never refuses a pod it would have taken.
__device__ __forceinline__ int32_t scale32(int64_t f, int k) {
  const int64_t q = f >> k;
  return f < 0 ? -1 : (q > 0x7fffffffll ? 0x7fffffff : static_cast<int32_t>(q));
}

// The checks of one pod against the window's 32-bit state as one lane test:
// x - r saturated to 32 bits is >= 0 exactly when x >= r (the clamped
// difference keeps its sign), s | -s is negative exactly when s != 0 (the
// state bits the pod conflicts with), and the OR of such values is >= 0
// exactly when every test passes, so the pod-count, cpu, memory (ephemeral,
// state-bit) checks cost one ballot instead of three to five chained through
// VCC.
template <bool E, bool O>
__device__ __forceinline__ uint64_t fits32(int32_t c32, int32_t m32, int32_t e32, int nleft, uint64_t conflict,
                                           int32_t c, int32_t m, int32_t e) {
  int32_t t = __builtin_elementwise_sub_sat(c32, c) | __builtin_elementwise_sub_sat(m32, m) | (nleft - 1);
  if (E) t |= __builtin_elementwise_sub_sat(e32, e);
  if (O) {
    const uint32_t x = static_cast<uint32_t>(conflict) | static_cast<uint32_t>(conflict >> 32);
    t |= static_cast<int32_t>(x | (0u - x));
  }
  return ballot(t >= 0);
}

// place_window with the window's state and the pods' requests scaled to 32
// bits (narrow candidates: S <= f equals S >> k <= f >> k for the multiples
// S of 2^k the candidate's requests sum to): one compare and one select per
// field instead of 64-bit pairs.
// The bits a placed pod sets come from its lane (`ps`, read with the pod's
// request) rather than being recomputed from its conflict bits on the scalar
// unit every step (A/B on MI355X, r04: K2 -1.5% on C5, equal on C3; the
// predicated, branch-free form of the update measured 3% slower).
// X (exclusive candidate: every pod sets and conflicts with one state bit,
// e.g. one host port): a node takes at most one of its pods, and a node no
// pod took in this window still holds the window's entry state, so every
// pod's first fit is computed against that state with the nodes taken so far
// masked out (no update between steps: the chain is the scalar mask), and the
// nodes' updates follow in one permute of the placed pods' requests.
template <bool E, bool O, bool X = false>
__device__ __forceinline__ uint64_t place_window32(uint64_t todo, int kmax, int W, int lane, uint32_t nc, uint32_t nm,
                                                   uint32_t ne, uint64_t pm, uint64_t ps, uint64_t cur,
                                                   int32_t& c32, int32_t& m32, int32_t& e32,
                                                   uint64_t& nport, int& nleft, int& node) {
  if constexpr (X) {
    int jv = 64;
    if (kmax < 64) todo &= kmax <= 0 ? 0ull : (1ull << kmax) - 1;
    const uint64_t base = ballot(nleft >= 1);
    uint64_t taken = 0;
    while (todo != 0) {
      const int k = __builtin_ctzll(todo);
      todo = bitclear(todo, k);
      const int32_t c = __builtin_amdgcn_readlane(static_cast<int>(nc), k);
      const int32_t m = __builtin_amdgcn_readlane(static_cast<int>(nm), k);
      const int32_t e = E ? __builtin_amdgcn_readlane(static_cast<int>(ne), k) : 0;
      const uint64_t q = readlane64(pm, k);
      uint64_t fit = readlane64(cur, k) & base & ~taken & fits32<E, true>(c32, m32, e32, 1, nport & q, c, m, e);
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      taken |= fit & (0ull - fit);  // the lowest set bit: node j
      jv = writelane(jv, j, k);  // pod k took lane j
    }
    // node lane j receives the request and the set bits of the pod that took
    // it; the other pods send zeros to a node nobody took (one exists unless
    // all 64 did, and then every pod of the window placed)
    const int dst = jv < 64 ? jv : (taken == ~0ull ? lane : __builtin_ctzll(~taken));
    const bool snd = jv < 64;
    auto send = [&](uint32_t v) {
      return static_cast<uint32_t>(__builtin_amdgcn_ds_permute(dst << 2, static_cast<int>(snd ? v : 0u)));
    };
    const uint32_t rc = send(static_cast<uint32_t>(max(static_cast<int32_t>(nc), 0)));
    const uint32_t rm = send(static_cast<uint32_t>(max(static_cast<int32_t>(nm), 0)));
    const uint32_t re = E ? send(static_cast<uint32_t>(max(static_cast<int32_t>(ne), 0))) : 0u;
    const uint32_t rs_lo = send(static_cast<uint32_t>(ps)), rs_hi = send(static_cast<uint32_t>(ps >> 32));
    const bool got = (taken >> lane) & 1;
    c32 -= got ? static_cast<int32_t>(rc) : 0;
    m32 -= got ? static_cast<int32_t>(rm) : 0;
    if (E) e32 -= got ? static_cast<int32_t>(re) : 0;
    nleft -= got ? 1 : 0;
    nport |= got ? (static_cast<uint64_t>(rs_hi) << 32 | rs_lo) : 0ull;
    node = jv < 64 ? 64 * W + jv : node;
    return ballot(jv < 64);
  }
  // The zero-request exemption and the fixed ephemeral gate are in the
  // values, not in the step: an all-zero request is INT_MIN in nc / nm / ne
  // (it meets every state value), and without E a lane whose ephemeral free
  // value is negative holds INT_MIN as its cpu state (it refuses every other
  // request); the update subtracts max(request, 0).  Measured: the scalar
  // selects cost ~10% of a step.
  int jv = 64;  // as in place_window
  if (kmax < 64) todo &= kmax <= 0 ? 0ull : (1ull << kmax) - 1;
  while (todo != 0) {
    const int k = __builtin_ctzll(todo);
    todo = bitclear(todo, k);
    const int32_t c = __builtin_amdgcn_readlane(static_cast<int>(nc), k);
    const int32_t m = __builtin_amdgcn_readlane(static_cast<int>(nm), k);
    const int32_t e = E ? __builtin_amdgcn_readlane(static_cast<int>(ne), k) : 0;
    const uint64_t q = O ? readlane64(pm, k) : 0ull;
    uint64_t fit = readlane64(cur, k) & fits32<E, O>(c32, m32, e32, nleft, nport & q, c, m, e);
    const int32_t cu = max(c, 0), mu = max(m, 0), eu = max(e, 0);
    if (O) {  // as in place_window
      if (fit != 0) {
        const int j = __builtin_ctzll(fit);
        if (lane == j) {
          c32 -= cu;
          m32 -= mu;
          if (E) e32 -= eu;
          nleft -= 1;
          nport |= readlane64(ps, k);
        }
        jv = writelane(jv, j, k);  // pod k took lane j
      }
      continue;
    }
    const int j = ff1(fit);  // -1 when it fits nowhere (no lane)
    const bool hit = lane == j;  // ClusterSnapshot.AddPod on the candidate's copy of node 64 W + j
    c32 -= hit ? cu : 0;
    m32 -= hit ? mu : 0;
    if (E) e32 -= hit ? eu : 0;
    nleft -= hit ? 1 : 0;
    jv = writelane(jv, j, k);  // pod k took lane j
  }
  const bool took = static_cast<unsigned>(jv) < 64u;  // -1 / 64: no lane
  node = took ? 64 * W + jv : node;
  return ballot(took);
}

// place_window_x in 32-bit scaled form (narrow XT candidates): one lane test
// per pod as in fits32, the two scalar slots included (an unlisted name is
// INT_MIN: it meets every slot value); the update subtracts the scaled
// accounting.
template <bool E, bool O>
__device__ __forceinline__ uint64_t place_window32_x(uint64_t todo, int kmax, int W, int lane, uint32_t nc, uint32_t nm,
                                                     uint32_t ne, const XVals<uint32_t>& x, uint64_t pm, uint64_t ps,
                                                     uint64_t cur, int32_t& c32, int32_t& m32, int32_t& e32,
                                                     int32_t& s0, int32_t& s1, uint64_t& nport, int& nleft,
                                                     int& node) {
  int jv = 64;
  if (kmax < 64) todo &= kmax <= 0 ? 0ull : (1ull << kmax) - 1;
  while (todo != 0) {
    const int k = __builtin_ctzll(todo);
    todo = bitclear(todo, k);
    const int32_t c = __builtin_amdgcn_readlane(static_cast<int>(nc), k);
    const int32_t m = __builtin_amdgcn_readlane(static_cast<int>(nm), k);
    const int32_t e = E ? __builtin_amdgcn_readlane(static_cast<int>(ne), k) : 0;
    const int32_t r0 = __builtin_amdgcn_readlane(static_cast<int>(x.r0), k);
    const int32_t r1 = __builtin_amdgcn_readlane(static_cast<int>(x.r1), k);
    const uint64_t q = O ? readlane64(pm, k) : 0ull;
    int32_t t = __builtin_elementwise_sub_sat(c32, c) | __builtin_elementwise_sub_sat(m32, m) | (nleft - 1) |
                __builtin_elementwise_sub_sat(s0, r0) | __builtin_elementwise_sub_sat(s1, r1);
    if (E) t |= __builtin_elementwise_sub_sat(e32, e);
    if (O) {
      const uint64_t cf = nport & q;
      const uint32_t u = static_cast<uint32_t>(cf) | static_cast<uint32_t>(cf >> 32);
      t |= static_cast<int32_t>(u | (0u - u));
    }
    const uint64_t fit = readlane64(cur, k) & ballot(t >= 0);
    if (fit != 0) {
      const int j = __builtin_ctzll(fit);
      const int32_t ac = __builtin_amdgcn_readlane(static_cast<int>(x.ac), k);
      const int32_t am = __builtin_amdgcn_readlane(static_cast<int>(x.am), k);
      const int32_t ae = __builtin_amdgcn_readlane(static_cast<int>(x.ae), k);
      const int32_t a0 = __builtin_amdgcn_readlane(static_cast<int>(x.a0), k);
      const int32_t a1 = __builtin_amdgcn_readlane(static_cast<int>(x.a1), k);
      if (lane == j) {
        c32 -= ac;
        m32 -= am;
        e32 -= ae;
        s0 -= a0;
        s1 -= a1;
        nleft -= 1;
        if (O) nport |= readlane64(ps, k);
      }
      jv = writelane(jv, j, k);  // pod k took lane j
    }
  }
  const bool took = static_cast<unsigned>(jv) < 64u;  // -1 / 64: no lane
  node = took ? 64 * W + jv : node;
  return ballot(took);
}

// A narrow candidate's request granularity per dimension: every request is a
// multiple of 2^k (k = the smallest trailing-zero count among them).
struct Narrow {
  int kc, km, ke;
};

// ------------------------------------------------ K2, cooperative resolution
// The costliest candidates of a long work list get a block of kCoopWaves
// waves instead of one (C4: its longest wave spent ~60 % of its cycles in one
// far resolution -- several pods leaving the 512-node head together and
// scanning their 548-word rows 64 words per dependent round trip).  Wave 0
// keeps the candidate's placement chain; when pods need a far resolution it
// posts them in LDS and every wave of the block scans a share of the chunks
// (chunk k of the request to wave k % kCoopWaves, in order), so a resolution
// costs about chunks / kCoopWaves round trips instead of `chunks`.  Each wave
// records, per pod, the first chunk of its share with a non-zero word; the
// chain takes the lowest over the waves: the same first feasible node a
// sequential scan finds (findSpotNodeForPod's first fit, rescheduler.go:
// 339-352, the scan over spot nodes being a first-set-bit reduction).
constexpr int kCoopWaves = 4;
constexpr int kCoopPods = 64;
struct CoopArea {
  int32_t cmd, n, sw, pad;                 // cmd 0: a resolution request of n pods from word sw; 1: exit
  uint64_t r01[kCoopPods], r23[kCoopPods];  // the pods' row offsets
  int64_t rq[kCoopPods][3];                 // ... requests (K0-less corrections)
  int32_t op[kCoopPods][8];                 // ... class programs (head-only S rows)
  uint32_t best[kCoopPods];                 // lowest chunk found by any wave so far (skips higher ones)
  uint32_t rk[kCoopWaves][kCoopPods];       // per wave: first chunk of its share with a non-zero word (~0: none)
  uint64_t rm[kCoopWaves][kCoopPods];       //   its non-zero-word mask
  uint64_t rf[kCoopWaves][kCoopPods];       //   its first non-zero word
};

// Wave h's share of a request: chunks k = h, h + kCoopWaves, ... from the
// request's first chunk, each for every pod not resolved by a lower chunk
// yet, Q pods' loads in flight per round trip (as the chain's own resolve).
template <bool HO>
__device__ __forceinline__ void coop_scan(const DevWorkload& w, CoopArea& A, int h) {
  const int lane = threadIdx.x & 63;
  const int n = __builtin_amdgcn_readfirstlane(A.n), sw = __builtin_amdgcn_readfirstlane(A.sw);
  const int Wp = w.Wp;
  const uint64_t* __restrict__ tab = w.S;
  if (lane < n) A.rk[h][lane] = 0xffffffffu;
  const int cb0 = (sw >> 6) << 6;
  const int nch = (Wp - cb0 + 63) >> 6;
  const uint64_t all = n >= 64 ? ~0ull : (1ull << n) - 1;
  uint64_t found = 0;  // pods this wave resolved
  constexpr int Q = HO ? 2 : 4;
  for (int k = h; k < nch; k += kCoopWaves) {
    const int cb = cb0 + 64 * k;
    const int word = cb + lane;
    const bool wv = word >= sw && word < Wp;
    const uint32_t wi = wv ? static_cast<uint32_t>(word) : 0u;
    const uint64_t vw = ballot(wv);
    // pods open at chunk k: not resolved by this wave, no lower chunk found by another
    uint64_t open = all & ~found & ballot(lane < n && __hip_atomic_load(&A.best[lane], __ATOMIC_RELAXED,
                                                                           __HIP_MEMORY_SCOPE_WORKGROUP) >
                                                        static_cast<uint32_t>(k));
    while (open != 0) {
      int js[Q];
      uint64_t a01[Q], a23[Q];
      int op[Q][8];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        js[q] = open != 0 ? __builtin_ctzll(open) : -1;
        open &= open - 1;
        const int j = js[q] < 0 ? 0 : js[q];
        a01[q] = readlane64(A.r01[j], 0);
        a23[q] = readlane64(A.r23[j], 0);
        if constexpr (HO) {
#pragma unroll
          for (int u = 0; u < 8; ++u) op[q][u] = __builtin_amdgcn_readfirstlane(A.op[j][u]);
        }
      }
      uint64_t x[Q][HO ? 11 : 4];
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (js[q] < 0) continue;  // wave-uniform
        if constexpr (HO) {
#pragma unroll
          for (int u = 0; u < 8; ++u)
            x[q][u] = op[q][u] >= 0 ? w.atoms[static_cast<size_t>(op[q][u] >> 2) * Wp + wi] : 0ull;
          x[q][8] = tab[static_cast<uint32_t>(a01[q] >> 32) + wi];
          x[q][9] = tab[static_cast<uint32_t>(a23[q]) + wi];
          x[q][10] = tab[static_cast<uint32_t>(a23[q] >> 32) + wi];
        } else {
          x[q][0] = tab[static_cast<uint32_t>(a01[q]) + wi];
          x[q][1] = tab[static_cast<uint32_t>(a01[q] >> 32) + wi];
          x[q][2] = tab[static_cast<uint32_t>(a23[q]) + wi];
          x[q][3] = tab[static_cast<uint32_t>(a23[q] >> 32) + wi];
        }
      }
#pragma unroll
      for (int q = 0; q < Q; ++q) {
        if (js[q] < 0) continue;  // wave-uniform
        const int j = js[q];
        uint64_t f, sw0;
        if constexpr (HO) {
          uint64_t v8[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) v8[u] = x[q][u];
          sw0 = eval_prog8(op[q], v8);
          f = sw0 & x[q][8] & x[q][9] & x[q][10];
        } else {
          sw0 = x[q][0];
          f = x[q][0] & x[q][1] & x[q][2] & x[q][3];
        }
        if (w.k0_skip) {
          const int64_t rc = A.rq[j][0], rm = A.rq[j][1], re = A.rq[j][2];
          f = fix_dirty(w, f, sw0, word, rc, rm, re, (rc | rm | re) == 0);
        }
        const uint64_t m = ballot(wv && f != 0) & vw;
        if (m == 0) continue;
        found |= 1ull << j;
        if (lane == 0) {
          A.rk[h][j] = static_cast<uint32_t>(k);
          A.rm[h][j] = m;
          atomicMin(&A.best[j], static_cast<uint32_t>(k));
        }
        const uint64_t fw = readlane64(f, __builtin_ctzll(m));
        if (lane == 0) A.rf[h][j] = fw;
      }
    }
  }
}

// A helper wave of a cooperative block: scans its share of every request the
// chain wave posts until the chain posts the exit (the same number of block
// barriers on every wave).
__device__ __forceinline__ void coop_helper(const DevWorkload& w, CoopArea& A, int h) {
  for (;;) {
    __syncthreads();
    if (__hip_atomic_load(&A.cmd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 0) break;
    if (w.s_head_only) coop_scan<true>(w, A, h);
    else coop_scan<false>(w, A, h);
    __syncthreads();
  }
}

// Sum over the 64 lanes (DPP, as wave_min).
__device__ __forceinline__ int wave_sum(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);
  return __builtin_amdgcn_readlane(v, 63);
}

// WIDE: the F heads of 64 pods per memory round trip also for G > 1 (more
// registers: for launches whose waves fit the SIMDs at the lower occupancy)
// XT: the candidate has extension records at pod_ext[ebase ..] (init-container
// accounting, shared scalar / volume-limit slots: place_window_x).
// erow0_in / erow1_in: the slots' node_scal rows from the work-list entry's
// list_ext (k2_node), or -2: read them from the candidate's first record.
// COOP: the candidate's block cooperates on far resolutions (CoopArea A:
// this wave is the chain, the block's other waves scan with it).
template <int G, bool PROF, bool WIDE = false, bool XT = false, bool COOP = false>
__device__ __forceinline__ void k2_node_order(const DevWorkload& w, uint64_t* __restrict__ F, const int p0,
                                              const int np, int& status, K2Stats& st, uint32_t& nbytes,
                                              const int ebase = -1, const int erow0_in = -2,
                                              const int erow1_in = -2, CoopArea* A = nullptr) {
  static_assert(64 * G * kNHS * 8 <= sizeof(K2Lds), "node-order LDS exceeds the wave's K2 region");
  const int lane = threadIdx.x & 63;
  const int Wp = w.Wp;
  const uint64_t* __restrict__ tab = w.S;
  int64_t rc[G], rm[G], re[G];
  uint64_t pm[G], ps[G], r01[G], r23[G], fmask[G], act[G];
  int fbase[G];  // first word of the 64-word chunk fmask describes (rows wider than 64 words)
  bool unres[G]; // the pointer is a chunk boundary not yet scanned (kFar: the end of the head)
  uint64_t cur[G];  // F word holding the pod's pointer: moves inside a word need no LDS read
  uint32_t hmask[G];
  bool zero[G];
  int ptr[G], node[G];
  int dead = np;  // first pod with no feasible spot node left
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const uint64_t* pr = w.pod_rec + static_cast<size_t>(p0 + min(64 * g + lane, np - 1)) * kRecU64;
    rc[g] = static_cast<int64_t>(pr[0]);
    rm[g] = static_cast<int64_t>(pr[1]);
    re[g] = static_cast<int64_t>(pr[2]);
    pm[g] = swap_pairs(pr[3], w.swap_mask);  // the state bits the pod conflicts with
    ps[g] = pr[3];                            // ... and those it sets
    r01[g] = pr[4];
    r23[g] = pr[5];
    zero[g] = (rc[g] | rm[g] | re[g]) == 0;  // fitsRequest skips the resource checks
    fmask[g] = 0;
    fbase[g] = 0;
    unres[g] = false;
    hmask[g] = 0;
    cur[g] = 0;
    ptr[g] = INT_MAX;
    node[g] = -1;
    const uint64_t e = ballot(64 * g + lane < np && static_cast<uint32_t>(r01[g]) == w.s_empty_off);
    if (e != 0) dead = min(dead, 64 * g + __builtin_ctzll(e));
  }
  // XT: the pods' extension records and the slots' node_scal rows
  XVals<int64_t> xv[G];
  int erow0 = -1, erow1 = -1;
  if constexpr (XT) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint64_t* er = w.pod_ext + static_cast<size_t>(ebase + min(64 * g + lane, np - 1)) * kDevExtU64;
      xv[g] = {static_cast<int64_t>(er[0]), static_cast<int64_t>(er[1]), static_cast<int64_t>(er[2]),
               static_cast<int64_t>(er[3]), static_cast<int64_t>(er[4]), static_cast<int64_t>(er[5]),
               static_cast<int64_t>(er[6])};
    }
    if (erow0_in == -2) {
      const uint64_t erow = w.pod_ext[static_cast<size_t>(ebase) * kDevExtU64 + 7];
      erow0 = __builtin_amdgcn_readfirstlane(static_cast<int32_t>(static_cast<uint32_t>(erow)));
      erow1 = __builtin_amdgcn_readfirstlane(static_cast<int32_t>(erow >> 32));
    } else {
      erow0 = erow0_in;
      erow1 = erow1_in;
    }
    nbytes += 64u * static_cast<uint32_t>(np);
  }
  // Narrow (32-bit scaled) placement when every request of the candidate
  // allows it: the smallest trailing-zero count per dimension, then every
  // scaled request below 2^23 (place_window32: the <= 256 pods of the
  // candidate sum below 2^31).
  Narrow nk;
  bool narrow;
  uint32_t nc[G], nm[G], ne[G];
  XVals<uint32_t> nx[G];  // XT, narrow
  {
    auto tz = [](int64_t v) { return v == 0 ? 64 : __builtin_ctzll(static_cast<uint64_t>(v)); };
    int mc = 64, mm = 64, me = 64;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      mc = min(mc, tz(rc[g]));
      mm = min(mm, tz(rm[g]));
      me = min(me, tz(re[g]));
      if (XT && 64 * g + lane < np) {  // the accounting is subtracted at the same scale
        mc = min(mc, tz(xv[g].ac));
        mm = min(mm, tz(xv[g].am));
        me = min(me, tz(xv[g].ae));
      }
    }
    nk.kc = min(wave_min(mc), 62);
    nk.km = min(wave_min(mm), 62);
    nk.ke = min(wave_min(me), 62);
    bool ok = true;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const uint64_t a = static_cast<uint64_t>(rc[g]) >> nk.kc, b = static_cast<uint64_t>(rm[g]) >> nk.km,
                     c = static_cast<uint64_t>(re[g]) >> nk.ke;
      ok = ok && (a | b | c) < (1ull << 23);
      // an all-zero request (fitsRequest skips the resource checks) compares
      // as INT_MIN: every state value meets it (place_window32)
      nc[g] = zero[g] ? 0x80000000u : static_cast<uint32_t>(a);
      nm[g] = zero[g] ? 0x80000000u : static_cast<uint32_t>(b);
      ne[g] = zero[g] ? 0x80000000u : static_cast<uint32_t>(c);
      if constexpr (XT) {
        // accounting and scalar values below 2^23 (non-negative; a zero-request
        // pod accounts nothing, as it meets even the INT_MIN ephemeral gate),
        // scalars unscaled, an unlisted name INT_MIN
        const XVals<int64_t>& v = xv[g];
        const uint64_t lim = 1ull << 23;
        const bool in = 64 * g + lane < np;
        ok = ok && (!in || ((v.ac | v.am | v.ae | v.a0 | v.a1) >= 0 &&
                            ((static_cast<uint64_t>(v.ac) >> nk.kc) | (static_cast<uint64_t>(v.am) >> nk.km) |
                             (static_cast<uint64_t>(v.ae) >> nk.ke) | static_cast<uint64_t>(v.a0) |
                             static_cast<uint64_t>(v.a1)) < lim &&
                            (v.r0 == INT64_MIN || (v.r0 >= 0 && v.r0 < static_cast<int64_t>(lim))) &&
                            (v.r1 == INT64_MIN || (v.r1 >= 0 && v.r1 < static_cast<int64_t>(lim))) &&
                            (!zero[g] || (v.ac | v.am | v.ae) == 0)));
        nx[g] = {static_cast<uint32_t>(static_cast<uint64_t>(v.ac) >> nk.kc),
                 static_cast<uint32_t>(static_cast<uint64_t>(v.am) >> nk.km),
                 static_cast<uint32_t>(static_cast<uint64_t>(v.ae) >> nk.ke),
                 v.r0 == INT64_MIN ? 0x80000000u : static_cast<uint32_t>(v.r0),
                 v.r1 == INT64_MIN ? 0x80000000u : static_cast<uint32_t>(v.r1), static_cast<uint32_t>(v.a0),
                 static_cast<uint32_t>(v.a1)};
      }
    }
    narrow = w.k2_narrow && ballot(!ok) == 0;
  }
  // some pod asks for ephemeral storage (E) / sets or meets state bits (O):
  // without them those checks are uniform over the visit and never change
  bool E, O;
  {
    uint64_t e = 0, o = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      e |= ballot(64 * g + lane < np && (re[g] != 0 || (XT && xv[g].ae != 0)));
      o |= ballot(64 * g + lane < np && pm[g] != 0);
    }
    E = e != 0;
    O = o != 0;
  }
  // exclusive candidate (place_window32 X): a state bit every pod sets and
  // conflicts with -- pod 0's candidates checked against every pod
  bool X = false;
  if (O && !XT) {
    const uint64_t m0 = readlane64(ps[0] & pm[0], 0);
    for (uint64_t bits = m0; bits != 0 && !X; bits &= bits - 1) {
      const int b = __builtin_ctzll(bits);
      bool all = true;
#pragma unroll
      for (int g = 0; g < G; ++g) all = all && ballot(64 * g + lane < np && !(((ps[g] & pm[g]) >> b) & 1)) == 0;
      X = all && w.k2_excl;
    }
  }
  // node records of window 0 (spot nodes [0, 64)), where first fit usually
  // lands: in flight together with the F heads below
  int wcur = -1;  // register window: lane i holds the base record of node 64 * wcur + i
  int64_t ncpu = 0, nmem = 0, neph = 0;
  uint64_t nport = 0;
  int nleft = 0;
  int64_t ns0 = 0, ns1 = 0;  // XT: the node's shared scalar slots (allocatable - requested)
  auto load_scal = [&](int W) {
    if constexpr (XT) {
      const size_t n = static_cast<size_t>(64 * W + lane);
      ns0 = erow0 >= 0 ? w.node_scal[static_cast<size_t>(erow0) * w.n_pad + n] : 0;
      ns1 = erow1 >= 0 ? w.node_scal[static_cast<size_t>(erow1) * w.n_pad + n] : 0;
      nbytes += 64u * 16u;
    }
  };
  if (dead > 0) {
    const uint64_t* nr = w.node_rec + static_cast<size_t>(lane) * 8;
    ncpu = static_cast<int64_t>(nr[0]);
    nmem = static_cast<int64_t>(nr[1]);
    neph = static_cast<int64_t>(nr[2]);
    nport = nr[3];
    nleft = static_cast<int>(static_cast<int64_t>(nr[4]));
    if (w.k0_skip) window_patch(w, 0, lane, ncpu, nmem, neph, nport, nleft);
    load_scal(0);
    wcur = 0;
    nbytes += 64u * 40u;
  }
  if (PROF) {  // profile builds: wait for the pod records and window 0 here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    st.cyc_rec = __builtin_amdgcn_s_memtime();
  }
  // s_head_only: each pod's class program (8 slots) in LDS after the F heads,
  // for the S words beyond the head (k2_node sizes its LDS for it)
  // (pods from the first dead one on are never scanned: a candidate whose
  // first pod fits no node -- C4: 2,254 of 15,000 -- loads none)
  int32_t* PG = reinterpret_cast<int32_t*>(F + 64 * G * kNHS);
  if (w.s_head_only && dead > 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (64 * g >= dead) break;  // wave-uniform
      const uint32_t cls = static_cast<uint32_t>(r01[g]) / static_cast<uint32_t>(Wp);
      const int4* p8 = reinterpret_cast<const int4*>(w.cls_prog8 + static_cast<size_t>(cls) * 8);
      const int4 a = p8[0], b = p8[1];
      int4* dst = reinterpret_cast<int4*>(PG + (64 * g + lane) * 8);
      dst[0] = a;
      dst[1] = b;
    }
    nbytes += 32u * static_cast<uint32_t>(min(np, 64 * ((dead + 63) / 64)));
  }
  uint64_t cyc_t = PROF ? __builtin_amdgcn_s_memtime() : 0;
  // bytes moved (algorithmic, wave-uniform): pod records, F heads of pods
  // [0, dead) (4 rows x min(Wp, kNH) words), 64-node record windows (5 words
  // each), full-row scans and far words, the mapping and status writes
  nbytes += (48u + 4u) * static_cast<uint32_t>(np) + 4u + 32u * static_cast<uint32_t>(min(Wp, kNH)) * dead;

  // head words holding a node changed since the tables were written (K0-less
  // runs), and per pod (its lane) whether it fits each changed node: bit p for
  // node patch p (at most 16)
  uint32_t dirty_head = 0;
  uint32_t dfit[G];
  for (int p = 0; p < w.n_dirty; ++p) {  // kernel arguments
    const int wd0 = w.dirty_node[p] >> 6;
    dirty_head |= wd0 < kNH ? 1u << wd0 : 0u;
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    dfit[g] = 0;
    if (dirty_head != 0)
      for (int p = 0; p < w.n_dirty; ++p) {
        const bool fits = zero[g] || (w.dirty_free[p][0] >= rc[g] && w.dirty_free[p][1] >= rm[g] &&
                                      w.dirty_free[p][2] >= re[g]);
        dfit[g] |= fits ? 1u << p : 0u;
      }
  }
  // F heads of pods [0, dead): lanes = kPW pods x kNH words, kPB such batches
  // per step with all their loads in flight together (one memory round trip
  // per kPW * kPB pods)
  {
    constexpr int kPW = 64 / kNH;  // pods per load instruction
    // up to 64 pods in one round trip (G = 1 or WIDE), 32 per round beyond
    constexpr int kPB = (G == 1 || WIDE ? 64 : 32) / kPW;
    const int sub = lane / kNH, wd = lane % kNH;
    const bool wv = wd < Wp;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int lim = min(dead, 64 * g + 64);
      for (int b0 = 64 * g; b0 < lim; b0 += kPW * kPB) {
        uint64_t x[kPB][4];
        int kk[kPB];
        uint32_t fm[kPB];  // the pod's fit mask of the changed nodes (K0-less runs), with its row offsets
#pragma unroll
        for (int h = 0; h < kPB; ++h) {
          kk[h] = b0 + kPW * h + sub;
          x[h][0] = x[h][1] = x[h][2] = x[h][3] = 0;
          fm[h] = 0;
          if (b0 + kPW * h >= lim) continue;  // wave-uniform
          const int src = min(kk[h], np - 1) - 64 * g;  // lane of that pod in group g
          if (dirty_head != 0) fm[h] = from_lane(dfit[g], src);
          const uint32_t o0 = from_lane(static_cast<uint32_t>(r01[g]), src);
          const uint32_t o1 = from_lane(static_cast<uint32_t>(r01[g] >> 32), src);
          const uint32_t o2 = from_lane(static_cast<uint32_t>(r23[g]), src);
          const uint32_t o3 = from_lane(static_cast<uint32_t>(r23[g] >> 32), src);
          const uint32_t wi = wv ? wd : 0u;
          x[h][0] = tab[o0 + wi];
          x[h][1] = tab[o1 + wi];
          x[h][2] = tab[o2 + wi];
          x[h][3] = tab[o3 + wi];
        }
#pragma unroll
        for (int h = 0; h < kPB; ++h) {
          if (b0 + kPW * h >= lim) continue;  // wave-uniform
          uint64_t f = (wv && kk[h] < np) ? x[h][0] & x[h][1] & x[h][2] & x[h][3] : 0ull;
          if (dirty_head != 0) {  // the changed nodes' bits, from the pod's fit mask
            for (int p = 0; p < w.n_dirty; ++p) {
              const int n = w.dirty_node[p];
              if ((n >> 6) != wd) continue;
              const uint64_t bit = 1ull << (n & 63);
              f = (fm[h] >> p) & 1 ? (f | (x[h][0] & bit)) : (f & ~bit);
            }
            f = (wv && kk[h] < np) ? f : 0ull;
          }
          if (kk[h] < np) F[kk[h] * kNHS + wd] = f;
          const uint64_t m = ballot(f != 0);  // kNH bits per pod: bit kNH * i + word
          const int rel = 64 * g + lane - (b0 + kPW * h);
          if (rel >= 0 && rel < kPW) hmask[g] = static_cast<uint32_t>(m >> (kNH * rel)) & ((1u << kNH) - 1u);
        }
      }
    }
  }

  // pointers: first feasible head node of every pod below `dead`, else kFar
  // (beyond the head; resolved lazily) or none
  uint64_t any = 0;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int k = 64 * g + lane;
    if (k < dead) {
      if (hmask[g] != 0) {
        const int w0 = __builtin_ctz(hmask[g]);
        cur[g] = F[k * kNHS + w0];
        ptr[g] = w0 * 64 + __builtin_ctzll(cur[g]);
      } else {
        ptr[g] = Wp > kNH ? kFar : INT_MAX;
        unres[g] = Wp > kNH;
      }
    }
    const uint64_t gone = ballot(k < dead && ptr[g] == INT_MAX);
    if (gone != 0) dead = min(dead, 64 * g + __builtin_ctzll(gone));
  }
  uint64_t zm[G];  // pods with an all-zero request (fitsRequest skips the resource checks)
#pragma unroll
  for (int g = 0; g < G; ++g) {
    act[g] = ballot(64 * g + lane < dead);  // pods still to place
    any |= act[g];
    zm[g] = ballot(zero[g]);
  }
  if (PROF) {
    const uint64_t t = __builtin_amdgcn_s_memtime();
    st.cyc_a += t - cyc_t;
    cyc_t = t;
  }

  int visits = 0, placements = 0, windows = wcur + 1;
  while (any != 0) {
    int mine = INT_MAX;
#pragma unroll
    for (int g = 0; g < G; ++g) mine = ((act[g] >> lane) & 1) ? min(mine, ptr[g]) : mine;
    const int n = wave_min(mine);
    if (n == INT_MAX) break;  // unreachable: every pod still to place has a pointer
    // Unresolved pointers sit on chunk boundaries (kFar: the end of the head;
    // beyond it, the end of a 64-word chunk whose mask ran out).  When the
    // minimum reaches one, its pods scan their F rows from there, 64 words
    // per round (lanes = words), before node n is visited: a pod may resolve
    // to n itself.
    uint64_t unres_n = 0;
    if (n == kFar || (n & 4095) == 0) {  // wave-uniform
#pragma unroll
      for (int g = 0; g < G; ++g) unres_n |= ballot(((act[g] >> lane) & 1) && ptr[g] == n && unres[g]);
    }
    if (unres_n != 0) {
      const uint64_t cyc_r0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
      const int sw = n >> 6;  // first word to scan (every pending pod points at n)
      // Q pods per round, all their loads for one chunk in flight together:
      // 4 row words each, or (s_head_only) their programs' atom words and 3 T
      // row words each
      auto resolve = [&](auto qc, auto ho) {
        constexpr int Q = decltype(qc)::value;
        constexpr bool HO = decltype(ho)::value;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          uint64_t pend = ballot(((act[g] >> lane) & 1) && ptr[g] == n && unres[g]);
          while (pend != 0) {
            int js[Q];
            uint64_t a01[Q], a23[Q];
            int64_t qr[Q][3];
            int op[Q][8];
            uint32_t nops[Q];
#pragma unroll
            for (int q = 0; q < Q; ++q) {
              js[q] = pend != 0 ? __builtin_ctzll(pend) : -1;
              pend &= pend - 1;
              const int j = js[q] < 0 ? 0 : js[q];
              a01[q] = readlane64(r01[g], j);
              a23[q] = readlane64(r23[g], j);
              qr[q][0] = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rc[g]), j));
              qr[q][1] = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rm[g]), j));
              qr[q][2] = static_cast<int64_t>(readlane64(static_cast<uint64_t>(re[g]), j));
              nops[q] = 0;
              if constexpr (HO) {  // the pod's class program (LDS, broadcast)
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                  op[q][u] = __builtin_amdgcn_readfirstlane(PG[(64 * g + j) * 8 + u]);
                  nops[q] += op[q][u] >= 0 ? 1u : 0u;
                }
              }
            }
            int todo = 0;  // bit q: pod js[q] not resolved yet
#pragma unroll
            for (int q = 0; q < Q; ++q) todo |= js[q] >= 0 ? 1 << q : 0;
            for (int cb = (sw >> 6) << 6; todo != 0 && cb < Wp; cb += 64) {  // wave-uniform, <= Wp / 64 rounds
              const int word = cb + lane;
              const bool wv = word >= sw && word < Wp;
              const uint32_t wi = wv ? static_cast<uint32_t>(word) : 0u;
              if (PROF) st.cyc_res += 1ull << 40;  // chunk rounds
              uint64_t x[Q][HO ? 11 : 4];
#pragma unroll
              for (int q = 0; q < Q; ++q) {
                if (!((todo >> q) & 1)) continue;  // wave-uniform
                if constexpr (HO) {
#pragma unroll
                  for (int u = 0; u < 8; ++u)
                    x[q][u] = op[q][u] >= 0 ? w.atoms[static_cast<size_t>(op[q][u] >> 2) * Wp + wi] : 0ull;
                  x[q][8] = tab[static_cast<uint32_t>(a01[q] >> 32) + wi];
                  x[q][9] = tab[static_cast<uint32_t>(a23[q]) + wi];
                  x[q][10] = tab[static_cast<uint32_t>(a23[q] >> 32) + wi];
                } else {
                  x[q][0] = tab[static_cast<uint32_t>(a01[q]) + wi];
                  x[q][1] = tab[static_cast<uint32_t>(a01[q] >> 32) + wi];
                  x[q][2] = tab[static_cast<uint32_t>(a23[q]) + wi];
                  x[q][3] = tab[static_cast<uint32_t>(a23[q] >> 32) + wi];
                }
              }
              const uint64_t vw = ballot(wv);
#pragma unroll
              for (int q = 0; q < Q; ++q) {
                if (!((todo >> q) & 1)) continue;  // wave-uniform
                uint64_t f, sw0;
                if constexpr (HO) {
                  uint64_t v8[8];
#pragma unroll
                  for (int u = 0; u < 8; ++u) v8[u] = x[q][u];
                  sw0 = eval_prog8(op[q], v8);
                  f = sw0 & x[q][8] & x[q][9] & x[q][10];
                } else {
                  sw0 = x[q][0];
                  f = x[q][0] & x[q][1] & x[q][2] & x[q][3];
                }
                if (w.k0_skip)
                  f = fix_dirty(w, f, sw0, word, qr[q][0], qr[q][1], qr[q][2], (qr[q][0] | qr[q][1] | qr[q][2]) == 0);
                f = wv ? f : 0ull;
                const uint64_t m = ballot(f != 0);
                // algorithmic bytes: the words a sequential scan reads, up to the
                // first non-zero one (the rest of the chunk is speculative)
                const int upto = m != 0 ? __builtin_ctzll(m) : 63;
                const uint64_t need = upto == 63 ? vw : vw & ((2ull << upto) - 1);
                nbytes += (HO ? 8u * (nops[q] + 3u) : 32u) * static_cast<uint32_t>(__builtin_popcountll(need));
                if (m == 0 && cb + 64 < Wp) continue;  // nothing in this chunk: the next one
                todo &= ~(1 << q);
                int nx = INT_MAX;
                uint64_t fw = 0;
                if (m != 0) {
                  const int w2 = __builtin_ctzll(m);
                  fw = readlane64(f, w2);
                  nx = (cb + w2) * 64 + __builtin_ctzll(fw);
                }
                if (lane == js[q]) {
                  fmask[g] = m;
                  fbase[g] = cb;
                  ptr[g] = nx;
                  cur[g] = fw;
                  unres[g] = false;
                }
                if (nx == INT_MAX) dead = min(dead, 64 * g + js[q]);
                if (PROF && nx == INT_MAX) st.cyc_res += 1ull << 56;  // pods whose scan found no node
              }
            }
          }
        }
      };
      // Cooperative block: per pod group one request, every wave of the
      // block scans its share of the chunks (coop_scan), the chain takes per
      // pod the lowest chunk found
      auto coop_resolve = [&]() {
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const uint64_t pend = ballot(((act[g] >> lane) & 1) && ptr[g] == n && unres[g]);
          if (pend == 0) continue;  // wave-uniform
          const bool mine = (pend >> lane) & 1;
          const int slot = __builtin_popcountll(pend & ((1ull << lane) - 1));
          int nops = 0;
          if (mine) {
            A->r01[slot] = r01[g];
            A->r23[slot] = r23[g];
            A->rq[slot][0] = rc[g];
            A->rq[slot][1] = rm[g];
            A->rq[slot][2] = re[g];
            if (w.s_head_only)
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int o = PG[(64 * g + lane) * 8 + u];
                A->op[slot][u] = o;
                nops += o >= 0 ? 1 : 0;
              }
            A->best[slot] = 0xffffffffu;
          }
          if (lane == 0) {
            A->cmd = 0;
            A->n = __builtin_popcountll(pend);
            A->sw = sw;
          }
          __syncthreads();  // the request is posted: every wave scans its share
          if (w.s_head_only) coop_scan<true>(w, *A, 0);
          else coop_scan<false>(w, *A, 0);
          __syncthreads();  // every share scanned
          if (PROF) st.cyc_res += static_cast<uint64_t>((Wp - ((sw >> 6) << 6) + 64 * kCoopWaves - 1) /
                                                        (64 * kCoopWaves)) << 40;
          uint32_t bytes = 0;
          if (mine) {
            uint32_t kb = 0xffffffffu;
            int hb = 0;
#pragma unroll
            for (int h = 0; h < kCoopWaves; ++h) {
              const uint32_t k = A->rk[h][slot];
              hb = k < kb ? h : hb;
              kb = k < kb ? k : kb;
            }
            int nx = INT_MAX, words = Wp - sw;
            if (kb != 0xffffffffu) {
              const uint64_t m = A->rm[hb][slot], fw = A->rf[hb][slot];
              const int cb = ((sw >> 6) << 6) + 64 * static_cast<int>(kb);
              const int w2 = __builtin_ctzll(m);
              nx = (cb + w2) * 64 + __builtin_ctzll(fw);
              fmask[g] = m;
              fbase[g] = cb;
              cur[g] = fw;
              words = cb + w2 + 1 - sw;  // the words a sequential scan reads, up to the first non-zero one
            } else {
              fmask[g] = 0;
              cur[g] = 0;
            }
            ptr[g] = nx;
            unres[g] = false;
            bytes = static_cast<uint32_t>(words) * (w.s_head_only ? 8u * (static_cast<uint32_t>(nops) + 3u) : 32u);
          }
          nbytes += static_cast<uint32_t>(wave_sum(static_cast<int>(bytes)));
          const uint64_t gone = ballot(mine && ptr[g] == INT_MAX);
          if (gone != 0) dead = min(dead, 64 * g + __builtin_ctzll(gone));
          if (PROF) st.cyc_res += static_cast<uint64_t>(__builtin_popcountll(gone)) << 56;
        }
      };
      // pods per round (A/B: 8 or 16 pods per round made the realistic
      // variant's resolution slower, 21-28k cycles against 17.5k)
      constexpr int kResQ = 4;
      if constexpr (COOP) coop_resolve();
      else if (w.s_head_only) resolve(std::integral_constant<int, 2>{}, std::true_type{});
      else resolve(std::integral_constant<int, kResQ>{}, std::false_type{});
      if (PROF) st.cyc_res += __builtin_amdgcn_s_memtime() - cyc_r0;
      any = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        act[g] &= ballot(64 * g + lane < dead);
        any |= act[g];
      }
      continue;
    }
    ++visits;
    const int W = n >> 6;
    if (W != wcur) {  // wave-uniform
      const uint64_t cyc_w0 = PROF ? __builtin_amdgcn_s_memtime() : 0;
      const uint64_t* nr = w.node_rec + static_cast<size_t>(W * 64 + lane) * 8;
      ncpu = static_cast<int64_t>(nr[0]);
      nmem = static_cast<int64_t>(nr[1]);
      neph = static_cast<int64_t>(nr[2]);
      nport = nr[3];
      nleft = static_cast<int>(static_cast<int64_t>(nr[4]));
      if (w.k0_skip) window_patch(w, W, lane, ncpu, nmem, neph, nport, nleft);
      load_scal(W);
      wcur = W;
      ++windows;
      nbytes += 64u * 40u;
      if (PROF) {  // profile builds: the window's records (and node patches) waited for here
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st.cyc_win += __builtin_amdgcn_s_memtime() - cyc_w0;
      }
    }
    if (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      st.cyc_b += t - cyc_t;
      cyc_t = t;
    }
    uint64_t failed[G];
    // Window visit: every pod whose pointer lies in window W, in pod order,
    // goes to its first node of the window that fits the window's running
    // state (lanes = nodes; ncpu .. nleft are updated in place: the window
    // is never visited again).  The pod's F word of the window is `cur`.
    {
      const uint64_t emask = E ? 0ull : ballot(neph >= 0);  // no pod asks for ephemeral storage: fixed
      // narrow candidates: the window's free values scaled to 32 bits once
      // per visit (the 64-bit copies are not read again: the window is not)
      int32_t c32 = 0, m32 = 0, e32 = 0, s032 = 0, s132 = 0;
      st.narrow = narrow;
      if (narrow) {
        c32 = E || neph >= 0 ? scale32(ncpu, nk.kc) : INT_MIN;  // place_window32: the ephemeral gate
        m32 = scale32(nmem, nk.km);
        e32 = scale32(neph, nk.ke);
        if (XT) {
          s032 = scale32(ns0, 0);
          s132 = scale32(ns1, 0);
        }
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {  // groups in pod order: the state flows from one to the next
        const uint64_t cand = ballot(((act[g] >> lane) & 1) && (ptr[g] >> 6) == W);
        const uint64_t todo = 64 * g < dead ? cand : 0ull;  // wave-uniform
        uint64_t placed = 0;
        if (todo != 0) {
          const int kmax = dead - 64 * g;  // pods above the first dead one are irrelevant
#define SR_PW(e_, o_)                                                                                             \
  place_window<e_, o_>(todo, kmax, W, lane, rc[g], rm[g], re[g], pm[g], cur[g], zm[g], w.swap_mask, emask, ncpu, \
                       nmem, neph, nport, nleft, node[g])
#define SR_PW32(e_, o_)                                                                                           \
  place_window32<e_, o_>(todo, kmax, W, lane, nc[g], nm[g], ne[g], pm[g], ps[g], cur[g], c32, m32, e32, \
                         nport, nleft, node[g])
#define SR_PW32X(e_)                                                                                            \
  place_window32<e_, true, true>(todo, kmax, W, lane, nc[g], nm[g], ne[g], pm[g], ps[g], cur[g], c32, m32, e32, \
                                 nport, nleft, node[g])
#define SR_PWX(e_, o_)                                                                                          \
  place_window_x<e_, o_>(todo, kmax, W, lane, rc[g], rm[g], re[g], xv[g], pm[g], cur[g], zm[g], w.swap_mask, emask, \
                         ncpu, nmem, neph, nport, nleft, ns0, ns1, node[g])
#define SR_PW32XT(e_, o_)                                                                                       \
  place_window32_x<e_, o_>(todo, kmax, W, lane, nc[g], nm[g], ne[g], nx[g], pm[g], ps[g], cur[g], c32, m32, e32, \
                           s032, s132, nport, nleft, node[g])
          if (XT && narrow)
            placed = E ? (O ? SR_PW32XT(true, true) : SR_PW32XT(true, false))
                       : (O ? SR_PW32XT(false, true) : SR_PW32XT(false, false));
          else if (XT)
            placed = E ? (O ? SR_PWX(true, true) : SR_PWX(true, false)) : (O ? SR_PWX(false, true) : SR_PWX(false, false));
          else if (narrow && X)
            placed = E ? SR_PW32X(true) : SR_PW32X(false);
          else if (narrow)
            placed = E ? (O ? SR_PW32(true, true) : SR_PW32(true, false))
                       : (O ? SR_PW32(false, true) : SR_PW32(false, false));
          else
            placed = E ? (O ? SR_PW(true, true) : SR_PW(true, false)) : (O ? SR_PW(false, true) : SR_PW(false, false));
#undef SR_PW
#undef SR_PW32
#undef SR_PW32X
#undef SR_PWX
#undef SR_PW32XT
        }
        placements += __builtin_popcountll(placed);
        act[g] &= ~placed;
        failed[g] = cand & ~placed;
      }
    }
    if (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      st.cyc_c += t - cyc_t;
      cyc_t = t;
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (failed[g] == 0) continue;  // wave-uniform
      // pods that did not fit n: next set bit of their F row after n
      const int k = 64 * g + lane;
      bool far_word = false;
      if ((failed[g] >> lane) & 1) {
            // it left window W: no node of it fits
        int nx = INT_MAX;
        if (W < kNH) {
          const uint32_t rem = hmask[g] & (0xffu << (W + 1)) & 0xffu;
          if (rem != 0) {
            const int w2 = __builtin_ctz(rem);
            cur[g] = F[k * kNHS + w2];
            nx = w2 * 64 + __builtin_ctzll(cur[g]);
          } else if (Wp > kNH) {
            nx = kFar;
            unres[g] = true;
          }
        } else {
          const int lw = W - fbase[g];  // the pointer's word within the chunk fmask describes
          const uint64_t rem = lw >= 63 ? 0ull : fmask[g] & (~0ull << (lw + 1));
          if (rem != 0) {
            const int w2 = fbase[g] + __builtin_ctzll(rem);
            cur[g] = w.s_head_only ? f_word_prog(w, tab, PG + (64 * g + lane) * 8, r01[g], r23[g], w2)
                                   : f_word_far(tab, r01[g], r23[g], w2);
            if (w.k0_skip) {  // the S word again for the changed nodes' bits
              const uint64_t sw0 = w.s_head_only ? f_word_prog_s(w, PG + (64 * g + lane) * 8, w2)
                                                 : tab[static_cast<uint32_t>(r01[g]) + w2];
              cur[g] = fix_dirty(w, cur[g], sw0, w2, rc[g], rm[g], re[g], zero[g]);
            }
            nx = w2 * 64 + __builtin_ctzll(cur[g]);
            far_word = true;
          } else if (fbase[g] + 64 < Wp) {
            nx = (fbase[g] + 64) * 64;  // the next chunk, scanned when the minimum gets there
            unres[g] = true;
          }
        }
        ptr[g] = nx;
      }
      nbytes += 32u * static_cast<uint32_t>(__builtin_popcountll(ballot(far_word)));
      // a pod with no node left fails the candidate; pods above it are irrelevant
      const uint64_t gone = ballot((((failed[g] >> lane) & 1) != 0) & (ptr[g] == INT_MAX));
      if (gone != 0) dead = min(dead, 64 * g + __builtin_ctzll(gone));
    }
    any = 0;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      act[g] &= ballot(64 * g + lane < dead);
      any |= act[g];
    }
    if (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      st.cyc_d += t - cyc_t;
      cyc_t = t;
    }
  }
  if (PROF) {
    st.n_min = static_cast<uint32_t>(visits);
    st.n_far = static_cast<uint32_t>(windows);
    st.n_spec_miss = static_cast<uint32_t>(placements);
  }
  status = dead < np ? dead : -1;
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int k = 64 * g + lane;
    if (k < np) w.out_node[p0 + k] = k < dead ? node[g] : -1;
  }
}

// ------------------------------------------------------------ K2, domain path
// Candidates whose pods interact through a topology key with shared domains
// (InterPodAffinity across nodes: antiaff.cpp).  Placing a pod changes other
// nodes' answers -- every node of its domain -- so neither the node-order
// induction nor the static F rows hold.  Pods in order (canDrainNode), one
// wave, lanes = row words 64 at a time: F = S & T & T & T & the pod's
// dynamic row, where the dynamic row
//  - refuses, per key slot, the domains of the earlier pods it interacts with
//    through anti-affinity (satisfyExistingPodsAntiAffinity /
//    satisfyPodAntiAffinity against the pods AddPod put on the snapshot);
//  - with an affinity set whose terms an earlier pod matches, requires per
//    term a node in the base row or in the domain of such a pod's node, unless
//    the pair map is still empty and the pod matches its own terms
//    (satisfyPodAffinity); its class carries KEYS(S).
// Nodes the candidate already touched are rechecked against its own copy of
// their state (capacity, pod count, state bits), as in the pod order path.
// <= 64 pods: lane k keeps pod k's node and its domain per key slot, lane s
// the s-th touched node's state.
__device__ __forceinline__ uint64_t wave_or(uint64_t v) {
  v |= dpp_shifted<0x111>(v);
  v |= dpp_shifted<0x112>(v);
  v |= dpp_shifted<0x114>(v);
  v |= dpp_shifted<0x118>(v);
  v |= dpp_shifted<0x142, 0xa>(v);
  v |= dpp_shifted<0x143, 0xc>(v);
  return readlane64(v, 63);
}

__device__ __forceinline__ int dk_row_of(const DevWorkload& w, int k) {
  return k == 0 ? w.dk_row[0] : k == 1 ? w.dk_row[1] : k == 2 ? w.dk_row[2] : w.dk_row[3];
}

static_assert(64 * 32 * 8 <= sizeof(K2Lds), "domain path: touched bitmap of 2048 words in the wave's LDS");
// G groups of 64 pods (G = 1: <= 64 pods, G = 4: <= 256): lane l of group g
// keeps pod 64 g + l's node and domains, and the (64 g + l)-th touched node's
// state.  A pod record holds, per key slot, G mask words over the earlier
// pods, G affinity mask words and the set word (kDevDynU64 words, layout of
// encode.cpp).
template <int CH, int G, bool PROF>
__device__ __forceinline__ void k2_domain(const DevWorkload& w, uint64_t* __restrict__ tl, const int p0,
                                          const int np, const int dbase, int& status, uint32_t& nbytes,
                                          K2Stats& st, const int ebase = -1) {
  static_assert(kDevDomKeys == 4 && kDevDynTerms == 4, "the selects below unroll 4 key slots / terms");
  static_assert(G >= 1 && G <= kDevDynG, "pod groups of the domain-path record");
  const int lane = threadIdx.x & 63;
  const int Wp = w.Wp;
  const uint64_t* __restrict__ tab = w.S;
  const uint64_t* __restrict__ at = w.atoms;
  // touched nodes: slot 64 g + lane holds the running state of the slot's node
  int snode[G], sleft[G], nslots = 0;
  int64_t scpu[G], smem[G], seph[G];
  uint64_t sport[G];
  int64_t ss0[G], ss1[G];  // extension records: shared scalar resources' running free values
  const bool ext = ebase >= 0;
  const uint64_t erow = ext ? w.pod_ext[static_cast<size_t>(ebase) * kDevExtU64 + 7] : ~0ull;
  const int erow0 = static_cast<int32_t>(static_cast<uint32_t>(erow)), erow1 = static_cast<int32_t>(erow >> 32);
  // pod 64 g + lane: its node and its domain in every key slot
  int pnode[G];
  int pdom[G][kDevDomKeys];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    snode[g] = INT_MAX;
    sleft[g] = 0;
    scpu[g] = smem[g] = seph[g] = 0;
    sport[g] = 0;
    ss0[g] = ss1[g] = 0;
    pnode[g] = -1;
#pragma unroll
    for (int kk = 0; kk < kDevDomKeys; ++kk) pdom[g][kk] = -1;
  }
  for (int i = lane; i < 64 * CH; i += 64) tl[i] = 0;  // touched nodes (bitmap in the wave's LDS)
  nbytes += (48u + 8u * kDevDynU64 + 4u) * static_cast<uint32_t>(np) + 4u;
  status = -1;
  int k = 0;
  // A pod's records in two registers, loaded one pod ahead (every pod step
  // otherwise starts with a memory round trip for them): lanes [0,
  // kDevDynU64) of one its domain-path record; lanes [0, 6) of the other its
  // pod record, lanes [8, 16) its extension record
  static_assert(kDevDynU64 <= 64 && kRecU64 <= 8 && kDevExtU64 <= 8, "record lanes of the domain path");
  auto records = [&](int q) -> uint64_t {
    if (q >= np) return 0ull;
    if (lane < kDevDynU64) return w.dyn_pod[static_cast<size_t>(dbase + q) * kDevDynU64 + lane];
    return 0ull;
  };
  auto records_pod = [&](int q) -> uint64_t {
    if (q >= np) return 0ull;
    if (lane < kRecU64) return w.pod_rec[static_cast<size_t>(p0 + q) * kRecU64 + lane];
    if (ext && lane >= 8 && lane < 8 + kDevExtU64)
      return w.pod_ext[static_cast<size_t>(ebase + q) * kDevExtU64 + (lane - 8)];
    return 0ull;
  };
  if (ext) nbytes += 8u * kDevExtU64 * static_cast<uint32_t>(np);
  uint64_t rv = records(0), rvp = records_pod(0);
  uint64_t cyc_t = PROF ? __builtin_amdgcn_s_memtime() : 0;
  auto stamp = [&](uint64_t& acc) {
    if (PROF) {
      const uint64_t t = __builtin_amdgcn_s_memtime();
      acc += t - cyc_t;
      cyc_t = t;
    }
  };
  for (; k < np; ++k) {
    const uint64_t cur = rv, curp = rvp;
    rv = records(k + 1);
    rvp = records_pod(k + 1);
    auto D = [&](int i) { return readlane64(cur, i); };    // domain-path record word i
    auto PR = [&](int i) { return readlane64(curp, i); };  // pod record word i
    const int64_t rc = static_cast<int64_t>(PR(0)), rm = static_cast<int64_t>(PR(1)), re = static_cast<int64_t>(PR(2));
    const uint64_t pm = PR(3), r01 = PR(4), r23 = PR(5);
    const uint64_t pin = swap_pairs(pm, w.swap_mask);
    const bool zero = (rc | rm | re) == 0;
    // what AddPod subtracts and the shared scalars (extension record)
    auto EX = [&](int i) { return static_cast<int64_t>(readlane64(curp, 8 + i)); };
    const int64_t ac = ext ? EX(0) : rc, am = ext ? EX(1) : rm, ae = ext ? EX(2) : re;
    const int64_t sr0 = ext ? EX(3) : INT64_MIN, sr1 = ext ? EX(4) : INT64_MIN;
    const int64_t sa0 = ext ? EX(5) : 0, sa1 = ext ? EX(6) : 0;
    // anti-affinity: domains refused per key slot (earlier pods it interacts with)
    uint64_t fdom[kDevDomKeys];
#pragma unroll
    for (int kk = 0; kk < kDevDomKeys; ++kk) {
      uint64_t any = 0, bits = 0;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const uint64_t m = kk < w.n_dk ? D(kk * kDevDynG + g) : 0ull;
        any |= m;
        const bool in = 64 * g + lane < k && ((m >> lane) & 1) && pdom[g][kk] >= 0;
        bits |= in ? 1ull << pdom[g][kk] : 0ull;
      }
      fdom[kk] = any != 0 ? wave_or(bits) : 0ull;
    }
    stamp(st.cyc_a);
    // topology spread planned here (SpreadDyn, encode.cpp): the pair counts
    // with the earlier pods the constraint counts.  Table key: base count per
    // domain in lane d, plus those pods domain by domain, the minimum over the
    // pairs, the domains over maxSkew refused (into fdom).  Node-local key:
    // the nodes where those pods exceed the node's cap (lanes in nlref).
    uint64_t nlref[G];
#pragma unroll
    for (int g = 0; g < G; ++g) nlref[g] = 0;
#pragma unroll
    for (int s2 = 0; s2 < kDevSpreadSlots; ++s2) {
      const int sw = 5 * kDevDynG + 1 + s2 * (kDevDynG + 3);  // the slot's words in the record
      const uint64_t i0 = D(sw + kDevDynG);
      if (i0 == ~0ull) continue;  // wave-uniform
      const int kk = static_cast<int>(i0 & 3);
      const bool nl = ((i0 >> 2) & 1) != 0;
      const int self = static_cast<int>((i0 >> 3) & 1);
      const int64_t skew = static_cast<int32_t>(static_cast<uint32_t>(i0 >> 32));
      const uint32_t off = static_cast<uint32_t>(D(sw + kDevDynG + 1));
      uint64_t rem[G];
      int pd[G];  // the pod's domain of key slot kk
#pragma unroll
      for (int g = 0; g < G; ++g) {
        rem[g] = D(sw + g) & ballot(64 * g + lane < k);  // every earlier pod is placed
        int d = -1;
#pragma unroll
        for (int k2 = 0; k2 < kDevDomKeys; ++k2) d = k2 == kk ? pdom[g][k2] : d;
        pd[g] = d;
      }
      nbytes += 8u * (kDevDynG + 3) + 256u;
      if (!nl) {
        const int edom = static_cast<int32_t>(static_cast<uint32_t>(D(sw + kDevDynG + 1) >> 32));
        const uint64_t pm = D(sw + kDevDynG + 2);
#pragma unroll
        for (int g = 0; g < G; ++g) pd[g] = pd[g] >= 0 ? pd[g] : edom;  // a keyless node: the pair of ""
        int cv = w.sp_tab[off + lane];
        for (;;) {  // wave-uniform: one round per distinct domain of the counted pods
          int gs = -1;
#pragma unroll
          for (int g = G - 1; g >= 0; --g) gs = rem[g] != 0 ? g : gs;
          if (gs < 0) break;
          int d = 0;
#pragma unroll
          for (int g = 0; g < G; ++g)
            if (g == gs) d = __builtin_amdgcn_readlane(pd[g], __builtin_ctzll(rem[g]));
          int n = 0;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            const uint64_t same = rem[g] & ballot(pd[g] == d);
            rem[g] &= ~same;
            n += __builtin_popcountll(same);
          }
          if (d >= 0 && lane == d) cv += n;
        }
        const bool inp = ((pm >> lane) & 1) != 0;
        const int mn = wave_min(inp ? cv : INT_MAX);
        fdom[kk] |= ballot(inp && static_cast<int64_t>(cv) + self - mn > skew);
      } else {
        int capv[G];
#pragma unroll
        for (int g = 0; g < G; ++g) capv[g] = ((rem[g] >> lane) & 1) ? w.sp_tab[off + static_cast<uint32_t>(pnode[g])] : INT_MAX;
        for (;;) {  // wave-uniform: one round per distinct node of the counted pods
          int gs = -1;
#pragma unroll
          for (int g = G - 1; g >= 0; --g) gs = rem[g] != 0 ? g : gs;
          if (gs < 0) break;
          int y = 0, cap = 0;
#pragma unroll
          for (int g = 0; g < G; ++g)
            if (g == gs) {
              const int j = __builtin_ctzll(rem[g]);
              y = __builtin_amdgcn_readlane(pnode[g], j);
              cap = __builtin_amdgcn_readlane(capv[g], j);
            }
          uint64_t same[G];
          int n = 0;
#pragma unroll
          for (int g = 0; g < G; ++g) {
            same[g] = rem[g] & ballot(pnode[g] == y);
            rem[g] &= ~same[g];
            n += __builtin_popcountll(same[g]);
          }
          if (n > cap) {
#pragma unroll
            for (int g = 0; g < G; ++g) nlref[g] |= same[g];
          }
        }
      }
    }
    // affinity: per term its key slot, base row and the earlier matching pods'
    // domains (table key) or pods (node-local key: adom holds their lanes per group)
    const uint64_t meta = D(5 * kDevDynG);
    int nt = 0;
    int tslot[kDevDynTerms] = {0, 0, 0, 0}, tbase[kDevDynTerms] = {0, 0, 0, 0};
    uint64_t adom[kDevDynTerms][G];
#pragma unroll
    for (int i = 0; i < kDevDynTerms; ++i)
#pragma unroll
      for (int g = 0; g < G; ++g) adom[i][g] = 0;
    if (meta != ~0ull) {
      const int set = static_cast<int>(meta >> 1);
      const bool self = (meta & 1) != 0;
      const int32_t* si = w.ds_info + set * (2 + 2 * kDevDynTerms);
      nt = si[0];
      bool map_has = si[1] == 0;
#pragma unroll
      for (int i = 0; i < kDevDynTerms; ++i) {
        if (i >= nt) continue;
        tslot[i] = si[2 + 2 * i];
        tbase[i] = si[3 + 2 * i];
        const bool table = dk_row_of(w, tslot[i]) >= 0;
        uint64_t bits = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const uint64_t mm = D(4 * kDevDynG + g);
          int d = -1;
#pragma unroll
          for (int kk = 0; kk < kDevDomKeys; ++kk) d = kk == tslot[i] ? pdom[g][kk] : d;
          const bool in = 64 * g + lane < k && ((mm >> lane) & 1) && d >= 0;
          const uint64_t b = ballot(in);
          map_has = map_has || b != 0;
          bits |= in ? 1ull << d : 0ull;
          adom[i][g] = table ? 0ull : b;
        }
        if (table) adom[i][0] = wave_or(bits);
      }
      if (!map_has && self) nt = 0;  // first pod of a self-affine group: KEYS(S) (in its class) only
    }
    stamp(st.cyc_b);
    int ans = INT_MAX;
    for (int ch = 0; ch < CH && ans == INT_MAX && ch * 64 < Wp; ++ch) {
      const int wd = ch * 64 + lane;
      const bool wv = wd < Wp;
      const uint32_t wi = wv ? static_cast<uint32_t>(wd) : 0u;
      const uint64_t sv = tab[static_cast<uint32_t>(r01) + wi];
      const uint64_t tv = tab[static_cast<uint32_t>(r01 >> 32) + wi] & tab[static_cast<uint32_t>(r23) + wi] &
                          tab[static_cast<uint32_t>(r23 >> 32) + wi];
      nbytes += 64u * 32u;
      uint64_t dyn = ~0ull;
#pragma unroll
      for (int kk = 0; kk < kDevDomKeys; ++kk) {
        uint64_t m = fdom[kk];
        const int row0 = dk_row_of(w, kk);
        while (m != 0) {
          const int d = __builtin_ctzll(m);
          m &= m - 1;
          dyn &= ~at[static_cast<size_t>(row0 + d) * Wp + wi];
          nbytes += 64u * 8u;
        }
      }
#pragma unroll
      for (int i = 0; i < kDevDynTerms; ++i) {
        if (i >= nt) continue;
        uint64_t row = at[static_cast<size_t>(tbase[i]) * Wp + wi];
        nbytes += 64u * 8u;
        const int row0 = dk_row_of(w, tslot[i]);
        if (row0 >= 0) {  // domains of a table key
          uint64_t m = adom[i][0];
          while (m != 0) {
            const int x = __builtin_ctzll(m);
            m &= m - 1;
            row |= at[static_cast<size_t>(row0 + x) * Wp + wi];
            nbytes += 64u * 8u;
          }
        } else {  // the matching pods' nodes (node-local key)
#pragma unroll
          for (int g = 0; g < G; ++g) {
            uint64_t m = adom[i][g];
            while (m != 0) {
              const int x = __builtin_ctzll(m);
              m &= m - 1;
              const int y = __builtin_amdgcn_readlane(pnode[g], x);
              if ((y >> 6) == wd) row |= 1ull << (y & 63);
            }
          }
        }
        dyn &= row;
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {  // spread: nodes a node-local constraint refuses
        uint64_t m = nlref[g];
        while (m != 0) {
          const int x = __builtin_ctzll(m);
          m &= m - 1;
          const int y = __builtin_amdgcn_readlane(pnode[g], x);
          if ((y >> 6) == wd) dyn &= ~(1ull << (y & 63));
        }
      }
      const uint64_t sd = wv ? sv & dyn : 0ull;
      const uint64_t clean = sd & tv & ~tl[wd];
      const uint64_t mc = ballot(clean != 0);
      int cn = INT_MAX;
      if (mc != 0) {
        const int L0 = __builtin_ctzll(mc);
        cn = (ch * 64 + L0) * 64 + __builtin_ctzll(readlane64(clean, L0));
      }
      // touched nodes of this chunk below cn: S and dynamic bit from the word's
      // lane, the rest from the candidate's copy of the node
      int best = INT_MAX;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const bool in = snode[g] >= ch * 4096 && snode[g] < min(cn, (ch + 1) * 4096);
        const int src = in ? (snode[g] >> 6) - ch * 64 : 0;
        const uint64_t ws = (static_cast<uint64_t>(from_lane(static_cast<uint32_t>(sd >> 32), src)) << 32) |
                            from_lane(static_cast<uint32_t>(sd), src);
        const bool fit = (zero | ((rc <= scpu[g]) & (rm <= smem[g]) & (re <= seph[g]))) & (sr0 <= ss0[g]) &
                         (sr1 <= ss1[g]);
        const bool ok = in & (((ws >> (snode[g] & 63)) & 1ull) != 0) & (sleft[g] >= 1) & ((sport[g] & pin) == 0) & fit;
        best = ok ? min(best, snode[g]) : best;
      }
      ans = min(cn, wave_min(best));
    }
    stamp(st.cyc_c);
    if (ans == INT_MAX) {  // "pod %s can't be rescheduled on any existing spot node"
      status = k;
      break;
    }
    // ClusterSnapshot.AddPod on the candidate's copy
    bool hit = false;
#pragma unroll
    for (int g = 0; g < G; ++g) {
      if (ballot(snode[g] == ans) != 0) {
        hit = true;
        if (snode[g] == ans) {
          scpu[g] -= ac;
          smem[g] -= am;
          seph[g] -= ae;
          sleft[g] -= 1;
          sport[g] |= pm;
          ss0[g] -= sa0;
          ss1[g] -= sa1;
        }
      }
    }
    if (!hit) {
      const uint64_t* rec = w.node_rec + static_cast<size_t>(ans) * 8;
      const int64_t fc = static_cast<int64_t>(rec[0]), fm = static_cast<int64_t>(rec[1]),
                    fe = static_cast<int64_t>(rec[2]);
      const uint64_t pb = rec[3];
      const int pl = static_cast<int>(static_cast<int64_t>(rec[4]));
      const int64_t b0 = ext && erow0 >= 0 ? w.node_scal[static_cast<size_t>(erow0) * w.n_pad + ans] : 0;
      const int64_t b1 = ext && erow1 >= 0 ? w.node_scal[static_cast<size_t>(erow1) * w.n_pad + ans] : 0;
      nbytes += 40u;
#pragma unroll
      for (int g = 0; g < G; ++g)
        if (lane + 64 * g == nslots) {
          snode[g] = ans;
          scpu[g] = fc - ac;
          smem[g] = fm - am;
          seph[g] = fe - ae;
          sleft[g] = pl - 1;
          sport[g] = pb | pm;
          ss0[g] = b0 - sa0;
          ss1[g] = b1 - sa1;
        }
      ++nslots;
      if (lane == 0) tl[ans >> 6] |= 1ull << (ans & 63);
    }
    int dn[kDevDomKeys];
#pragma unroll
    for (int kk = 0; kk < kDevDomKeys; ++kk)
      dn[kk] = kk < w.n_dk ? w.dk_dom[static_cast<size_t>(kk) * w.n_spot + ans] : -1;
#pragma unroll
    for (int g = 0; g < G; ++g)
      if (lane + 64 * g == k) {
        pnode[g] = ans;
#pragma unroll
        for (int kk = 0; kk < kDevDomKeys; ++kk) pdom[g][kk] = dn[kk];
      }
    stamp(st.cyc_d);
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int kq = 64 * g + lane;
    if (kq < np) w.out_node[p0 + kq] = (status < 0 || kq < status) ? pnode[g] : -1;
  }
}

// K2: one wave per candidate (list entries {candidate, first pod, end pod,
// global index}, longest candidates first).
// A K2 wave's work-list entry (and profile stamps).
struct K2Entry {
  int ci, p0, np, g;
  uint64_t t_start, c_start, t_list;
};
template <bool PROF>
__device__ __forceinline__ K2Entry k2_entry(const DevWorkload& w, const int4* __restrict__ list, int li) {
  K2Entry x;
  x.t_start = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
  x.c_start = PROF || w.out_cycles ? __builtin_amdgcn_s_memtime() : 0;
  const int4 e = li < w.n_list_head ? w.list_head[li] : list[li];  // the head: with the kernel arguments
  x.ci = __builtin_amdgcn_readfirstlane(e.x);
  x.p0 = __builtin_amdgcn_readfirstlane(e.y);
  x.np = __builtin_amdgcn_readfirstlane(e.z) - x.p0;  // >= 1: empty candidates never reach the device
  x.g = __builtin_amdgcn_readfirstlane(e.w);
  if (PROF) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the work-list entry has arrived
  x.t_list = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
  return x;
}

// A K2 wave's outcome: status, bytes, the packed first-drainable minimum, the
// profile record and (single rank) the tagged words the host polls.
template <bool PROF>
__device__ __forceinline__ void k2_finish(const DevWorkload& w, const K2Entry& x, int status, int wide,
                                          uint32_t nbytes, const K2Stats& st) {
  const int lane = threadIdx.x & 63;
  const int ci = x.ci, p0 = x.p0, np = x.np;
  int best = 0;  // lane 0: this candidate is the first drainable one so far
  if (lane == 0 && ci == 0) {  // once per run: the next run's first word (K0 may not run then), this run's others
    unsigned long long* dn = reinterpret_cast<unsigned long long*>(w.d_min_next);
    unsigned long long* dm = reinterpret_cast<unsigned long long*>(w.d_min);
    dn[0] = ~0ull;
    dm[1] = w.first_fallback_local < 0 ? ~0ull : static_cast<unsigned long long>(w.first_fallback_local) << 32;
    dm[2] = w.rank_next;
  }
  if (lane == 0) {
    w.out_status[ci] = status;
    w.out_bytes[ci] = nbytes;
    if (w.out_cycles)
      w.out_cycles[ci] = static_cast<uint32_t>(min(__builtin_amdgcn_s_memtime() - x.c_start, 0xffffffffull));
    // packed (global candidate << 32 | local candidate): min = first drainable
    if (status < 0) {
      const unsigned long long key = (static_cast<unsigned long long>(x.g) << 32) | static_cast<unsigned>(ci);
      best = key < atomicMin(reinterpret_cast<unsigned long long*>(w.d_min), key);
    }
    if (PROF) {
      uint64_t* pr = w.prof + static_cast<size_t>(ci) * 16;
      pr[0] = x.t_start;
      pr[1] = x.t_list;  // the work-list entry has arrived
      pr[2] = __builtin_amdgcn_s_memrealtime();
      pr[3] = __builtin_amdgcn_s_memtime() - x.c_start;
      pr[4] = static_cast<uint64_t>(status >= 0 ? status + 1 : np);
      pr[5] = static_cast<uint64_t>(wide);
      pr[6] = st.n_spec_miss;
      pr[7] = static_cast<uint64_t>(st.n_min) | (static_cast<uint64_t>(st.n_far) << 32);
      pr[8] = st.cyc_a;
      pr[9] = st.cyc_b;
      pr[10] = st.cyc_c;
      pr[11] = st.cyc_d;
      if (wide == 2) {  // node order
        pr[12] = st.cyc_res;
        pr[13] = st.cyc_win;
        pr[14] = st.cyc_rec - x.c_start;
        pr[15] = st.narrow;
      }
    }
  }
  if (w.res_stat) {
    // Single rank: the host walks res_stat in candidate order and stops at the
    // first drainable candidate, whose mapping is in res_map -- its wave was
    // necessarily the first drainable one so far when it finished -- so the
    // result is in host memory as soon as the candidates up to the winner are
    // planned, not when the whole grid is.  Every word carries the run's tag
    // and is accepted on its own: no store waits for another.
    const uint64_t tag = static_cast<uint64_t>(w.seq) << 32;
    if (__builtin_amdgcn_readfirstlane(best)) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this wave's out_node stores, then read back
      for (int q = lane; q < np; q += 64)
        __hip_atomic_store(w.res_map + p0 + q,
                           tag | static_cast<uint32_t>(__hip_atomic_load(w.out_node + p0 + q, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT)),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (lane == 0)
      __hip_atomic_store(w.res_stat + ci, tag | (status < 0 ? 1u : 0u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int CH, bool PROF>
__global__ __launch_bounds__(256) void k2_place(DevWorkload w_arg, const int4* __restrict__ list, int n_list) {
  const DevWorkload& w = *(const DevWorkload*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)w_arg;  // as in k2_node
  extern __shared__ __attribute__((aligned(16))) uint64_t k2_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int li = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x * (blockDim.x >> 6)) + wave);
  if (li >= n_list) return;
  const K2Entry x = k2_entry<PROF>(w, list, li);
  const int ci = x.ci, p0 = x.p0, np = x.np;
  K2Lds& L = *reinterpret_cast<K2Lds*>(k2_lds + static_cast<size_t>(wave) * (sizeof(K2Lds) / 8));

  K2Stats st;
  int status = -1;
  int wide = 0;
  uint32_t nbytes = 0;
  const int dbase = w.dyn_cand ? __builtin_amdgcn_readfirstlane(w.dyn_cand[ci]) : -1;
  const int ebase = w.ext_cand ? __builtin_amdgcn_readfirstlane(w.ext_cand[ci]) : -1;
  const bool node_order = np <= 4 * 64 && w.k2_mode == 0;
  if (dbase >= 0) {  // writes out_node itself
    wide = 3;
    uint64_t* tl = reinterpret_cast<uint64_t*>(&L);
    if (np <= 64) k2_domain<CH, 1, PROF>(w, tl, p0, np, dbase, status, nbytes, st, ebase);
    else if (np <= 128) k2_domain<CH, 2, PROF>(w, tl, p0, np, dbase, status, nbytes, st, ebase);  // (4: +37 % per pod)
    else if (np <= 256) k2_domain<CH, 4, PROF>(w, tl, p0, np, dbase, status, nbytes, st, ebase);
    else k2_domain<CH, kDevDynG, PROF>(w, tl, p0, np, dbase, status, nbytes, st, ebase);
  } else if (node_order && ebase >= 0) {  // extension records, node order (place_window_x); writes out_node
    uint64_t* F = reinterpret_cast<uint64_t*>(&L);
    wide = 2;
    if (np <= 64) k2_node_order<1, PROF, false, true>(w, F, p0, np, status, st, nbytes, ebase);
    else if (np <= 128) k2_node_order<2, PROF, false, true>(w, F, p0, np, status, st, nbytes, ebase);
    else k2_node_order<4, PROF, false, true>(w, F, p0, np, status, st, nbytes, ebase);
  } else if (ebase >= 0) {  // extension records, pod order (SR_K2_MODE=1) with the extended running state
    int placed = k2_run<1, CH, PROF, true>(w, L, p0, np, status, st, nbytes, ebase);
    wide = placed < 0 ? 1 : 0;
    if (placed < 0) placed = k2_run<8, CH, PROF, true>(w, L, p0, np, status, st, nbytes, ebase);
    for (int i = lane; i < np; i += 64) w.out_node[p0 + i] = i < placed ? L.omap[i] : -1;
  } else if (node_order) {  // writes out_node itself
    uint64_t* F = reinterpret_cast<uint64_t*>(&L);
    wide = 2;
    if (np <= 64) k2_node_order<1, PROF>(w, F, p0, np, status, st, nbytes);
    else if (np <= 128) k2_node_order<2, PROF>(w, F, p0, np, status, st, nbytes);
    else k2_node_order<4, PROF>(w, F, p0, np, status, st, nbytes);
  } else {
    int placed = k2_run<1, CH, PROF>(w, L, p0, np, status, st, nbytes);
    wide = placed < 0 ? 1 : 0;
    if (placed < 0) placed = k2_run<8, CH, PROF>(w, L, p0, np, status, st, nbytes);  // > 64 distinct nodes
    for (int i = lane; i < np; i += 64) w.out_node[p0 + i] = i < placed ? L.omap[i] : -1;
  }
  k2_finish<PROF>(w, x, status, wide, nbytes, st);
}

// K2 when every candidate of the launch takes node order (no domain-path
// candidate, <= 64 * GMAX pods, default mode): only that path is compiled, so
// the kernel holds far fewer registers than k2_place (more waves per SIMD on
// the large configs), and a wave's LDS is just its F heads.
// XT: the launch holds candidates with extension records (ext_cand), which
// take place_window_x; the others the plain steps (a separate instance, so a
// launch without them keeps the lean kernel).
template <int GMAX, bool PROF, bool WIDE = false, bool XT = false>
__global__ __launch_bounds__(256) void k2_node(DevWorkload w_arg, const int4* __restrict__ list, int n_list) {
  // the workload read in place from the kernel-argument segment (w_arg is its
  // first argument): each field is a scalar load where it is used, instead of
  // values held (or spilled to scratch) across the kernel
  const DevWorkload& w = *(const DevWorkload*)__builtin_amdgcn_kernarg_segment_ptr();
  (void)w_arg;
  extern __shared__ __attribute__((aligned(16))) uint64_t k2_lds[];
  const int wave = threadIdx.x >> 6;
  const size_t region = 64 * GMAX * kNHS + (w.s_head_only ? 64 * GMAX * 4 : 0);  // LDS words per wave
  // the first n_coop blocks: one candidate each (the list's costliest), wave 0
  // its chain, the other waves scanning with it (launches of kCoopWaves waves
  // per block without extension records)
  const int nco = XT ? 0 : w.n_coop;
  if constexpr (!XT) {
    static_assert(sizeof(CoopArea) <= (kCoopWaves - 1) * 64 * kNHS * 8, "the cooperative area fits the helpers' LDS");
    if (static_cast<int>(blockIdx.x) < nco) {
      CoopArea* A = reinterpret_cast<CoopArea*>(k2_lds + region);
      if (wave != 0) {
        coop_helper(w, *A, wave);
        return;
      }
      const K2Entry x = k2_entry<PROF>(w, list, static_cast<int>(blockIdx.x));
      K2Stats st;
      int status = -1;
      uint32_t nbytes = 0;
      if (GMAX == 1 || x.np <= 64)
        k2_node_order<1, PROF, false, false, true>(w, k2_lds, x.p0, x.np, status, st, nbytes, -1, -2, -2, A);
      else if (GMAX == 2 || x.np <= 128)
        k2_node_order<(GMAX >= 2 ? 2 : 1), PROF, WIDE, false, true>(w, k2_lds, x.p0, x.np, status, st, nbytes, -1,
                                                                    -2, -2, A);
      else k2_node_order<GMAX, PROF, WIDE, false, true>(w, k2_lds, x.p0, x.np, status, st, nbytes, -1, -2, -2, A);
      if (threadIdx.x == 0) A->cmd = 1;  // the helpers leave
      __syncthreads();
      st.narrow |= 2;  // (profile: a cooperative block)
      k2_finish<PROF>(w, x, status, 2, nbytes, st);
      return;
    }
  }
  const int li = __builtin_amdgcn_readfirstlane(nco + static_cast<int>((blockIdx.x - nco) * (blockDim.x >> 6)) + wave);
  if (li >= n_list) return;
  int4 xe = {-1, -1, -1, 0};
  if (XT) xe = w.list_ext[li];  // issued with the entry: one round trip for both
  const K2Entry x = k2_entry<PROF>(w, list, li);
  uint64_t* F = k2_lds + static_cast<size_t>(wave) * region;
  K2Stats st;
  int status = -1;
  uint32_t nbytes = 0;
  if constexpr (XT) {
    const int ebase = __builtin_amdgcn_readfirstlane(xe.x);
    const int er0 = __builtin_amdgcn_readfirstlane(xe.y), er1 = __builtin_amdgcn_readfirstlane(xe.z);
    if (ebase >= 0) {
      if (GMAX == 1 || x.np <= 64)
        k2_node_order<1, PROF, false, true>(w, F, x.p0, x.np, status, st, nbytes, ebase, er0, er1);
      else if (GMAX == 2 || x.np <= 128)
        k2_node_order<(GMAX >= 2 ? 2 : 1), PROF, WIDE, true>(w, F, x.p0, x.np, status, st, nbytes, ebase, er0, er1);
      else k2_node_order<GMAX, PROF, WIDE, true>(w, F, x.p0, x.np, status, st, nbytes, ebase, er0, er1);
      k2_finish<PROF>(w, x, status, 2, nbytes, st);
      return;
    }
  }
  if (GMAX == 1 || x.np <= 64) k2_node_order<1, PROF>(w, F, x.p0, x.np, status, st, nbytes);
  else if (GMAX == 2 || x.np <= 128)
    k2_node_order<(GMAX >= 2 ? 2 : 1), PROF, WIDE>(w, F, x.p0, x.np, status, st, nbytes);
  else k2_node_order<GMAX, PROF, WIDE>(w, F, x.p0, x.np, status, st, nbytes);
  k2_finish<PROF>(w, x, status, 2, nbytes, st);
}

// K2 waves per block: SR_K2_WPB (1, 2, 4), else one wave per block for lists of
// at most 2,048 entries (the waves spread over every CU, so a long chain wave
// shares its CU with fewer others: C5 K2 38.2 -> 36.1 us, realistic C3 31.5 ->
// 30.5, C3 15.0 -> 14.4) and four above (C4: 15,000 waves)
static inline int k2_waves_per_block(const DevWorkload& w) {
  if (w.k2_wpb == 1 || w.k2_wpb == 2 || w.k2_wpb == 4) return w.k2_wpb;
  return w.n_list <= 2048 ? 1 : 4;
}

// Launch with optional HIP events recorded by the dispatch itself
// (hipExtLaunchKernelGGL: no event packets or host calls around the kernel).
template <typename K, typename... A>
void launch(K kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1, A... args) {
  if (ev0 || ev1) hipExtLaunchKernelGGL(kernel, grid, block, static_cast<uint32_t>(lds), s, ev0, ev1, 0, args...);
  else hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
}

}  // namespace

// The K2 launchers are compiled in parts (SR_KPART, Makefile: one object per
// part, built in parallel; -1 = everything in one translation unit): 0 = the
// dispatch, K0 and K3; 1 = the node-order kernels; 2..7 = the general kernel
// for rows of 1, 2, 4, 8, 16, 32 chunks of 64 words; 8 = the node-order
// kernels with extension records.
#ifndef SR_KPART
#define SR_KPART -1
#endif
// wide F-head rounds where the extra registers cost nothing: launches of at
// most two waves per SIMD (256 CUs x 4 SIMDs), and G = 4 (one wave per SIMD
// either way)
template <bool PROF>
hipError_t launch_k2_node_g(const DevWorkload& w, int G, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
template <bool PROF>
hipError_t launch_k2_node_xt_g(const DevWorkload& w, int G, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);
template <int CH, bool PROF>
hipError_t launch_k2_place_ch(const DevWorkload& w, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1);

#if SR_KPART == -1 || SR_KPART == 1
template <bool PROF>
hipError_t launch_k2_node_g(const DevWorkload& w, int G, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  const int n = w.n_list;
  const int wpb = k2_waves_per_block(w);  // waves per block
  // cooperative blocks first (one candidate each), then wpb candidates per block
  if (w.n_coop < 0 || w.n_coop > n || (w.n_coop > 0 && (wpb != kCoopWaves || w.ext_cand))) return hipErrorInvalidValue;
  const dim3 grid(w.n_coop + (n - w.n_coop + wpb - 1) / wpb), block(64 * wpb);
  const size_t lds = wpb * static_cast<size_t>(64 * G * kNHS + (w.s_head_only ? 64 * G * 4 : 0)) * 8;
  const bool wide = n <= 2048;
  if (w.ext_cand) return launch_k2_node_xt_g<PROF>(w, G, s, ev0, ev1);  // some candidate has extension records
  if (G == 1) launch(k2_node<1, PROF>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  else if (G == 2 && wide) launch(k2_node<2, PROF, true>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  else if (G == 2) launch(k2_node<2, PROF>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  else launch(k2_node<4, PROF, true>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  return hipGetLastError();
}
template hipError_t launch_k2_node_g<false>(const DevWorkload&, int, hipStream_t, hipEvent_t, hipEvent_t);
template hipError_t launch_k2_node_g<true>(const DevWorkload&, int, hipStream_t, hipEvent_t, hipEvent_t);
#endif

#if SR_KPART == -1 || SR_KPART == 8
// the node-order kernels of launches with extension-record candidates
template <bool PROF>
hipError_t launch_k2_node_xt_g(const DevWorkload& w, int G, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  const int n = w.n_list;
  const int wpb = k2_waves_per_block(w);
  const dim3 grid((n + wpb - 1) / wpb), block(64 * wpb);
  const size_t lds = wpb * static_cast<size_t>(64 * G * kNHS + (w.s_head_only ? 64 * G * 4 : 0)) * 8;
  const bool wide = n <= 2048;  // as launch_k2_node_g
  if (G == 1) launch(k2_node<1, PROF, false, true>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  else if (G == 2 && wide) launch(k2_node<2, PROF, true, true>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  else if (G == 2) launch(k2_node<2, PROF, false, true>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  else launch(k2_node<4, PROF, true, true>, grid, block, lds, s, ev0, ev1, w, w.list, n);
  return hipGetLastError();
}
template hipError_t launch_k2_node_xt_g<false>(const DevWorkload&, int, hipStream_t, hipEvent_t, hipEvent_t);
template hipError_t launch_k2_node_xt_g<true>(const DevWorkload&, int, hipStream_t, hipEvent_t, hipEvent_t);
#endif

#if SR_KPART == -1 || SR_KPART >= 2
template <int CH, bool PROF>
hipError_t launch_k2_place_ch(const DevWorkload& w, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  const int n = w.n_list;
  const int wpb = k2_waves_per_block(w);  // waves per block
  const dim3 grid((n + wpb - 1) / wpb), block(64 * wpb);
  launch(k2_place<CH, PROF>, grid, block, wpb * sizeof(K2Lds), s, ev0, ev1, w, w.list, n);
  return hipGetLastError();
}
#define SR_PLACE_INST(CH)                                                                                      \
  template hipError_t launch_k2_place_ch<CH, false>(const DevWorkload&, hipStream_t, hipEvent_t, hipEvent_t); \
  template hipError_t launch_k2_place_ch<CH, true>(const DevWorkload&, hipStream_t, hipEvent_t, hipEvent_t);
#endif
#if SR_KPART == -1 || SR_KPART == 2
SR_PLACE_INST(1)
#endif
#if SR_KPART == -1 || SR_KPART == 3
SR_PLACE_INST(2)
#endif
#if SR_KPART == -1 || SR_KPART == 4
SR_PLACE_INST(4)
#endif
#if SR_KPART == -1 || SR_KPART == 5
SR_PLACE_INST(8)
#endif
#if SR_KPART == -1 || SR_KPART == 6
SR_PLACE_INST(16)
#endif
#if SR_KPART == -1 || SR_KPART == 7
SR_PLACE_INST(32)
#endif

#if SR_KPART == -1 || SR_KPART == 0
template <bool PROF>
hipError_t launch_k2(const DevWorkload& w, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  const int n = w.n_list;
  if (n <= 0) return hipSuccess;
  if (!w.dyn_cand && w.k2_mode == 0 && w.max_np >= 1 && w.max_np <= 4 * 64 && w.k2_node_kernel)
    return launch_k2_node_g<PROF>(w, w.max_np <= 64 ? 1 : (w.max_np <= 128 ? 2 : 4), s, ev0, ev1);
  const int chunks = (w.Wp + 63) / 64;
  if (chunks <= 1) return launch_k2_place_ch<1, PROF>(w, s, ev0, ev1);
  if (chunks <= 2) return launch_k2_place_ch<2, PROF>(w, s, ev0, ev1);
  if (chunks <= 4) return launch_k2_place_ch<4, PROF>(w, s, ev0, ev1);
  if (chunks <= 8) return launch_k2_place_ch<8, PROF>(w, s, ev0, ev1);
  if (chunks <= 16) return launch_k2_place_ch<16, PROF>(w, s, ev0, ev1);
  return launch_k2_place_ch<32, PROF>(w, s, ev0, ev1);
}

hipError_t launch_tables(const DevWorkload& w, int32_t local_first_fallback, hipStream_t s, hipEvent_t ev0,
                         hipEvent_t ev1) {
  const int s_blocks = (w.n_classes + 4 * kSClasses - 1) / (4 * kSClasses);
  const int wgroups = (w.Wp + kTWords - 1) / kTWords;
  int t_waves = 0;
  for (int d = 0; d < 4; ++d) t_waves += (w.t_off[d + 1] - w.t_off[d] + 63) / 64 * wgroups;
  const unsigned blocks = static_cast<unsigned>(std::max(1, s_blocks + (t_waves + 3) / 4));
  if (w.k0_inc) {
    const int s_waves = w.n_k0_cols > 0 ? (w.n_classes + 63) / 64 : 0;
    int tw = 0;
    for (int d = 1; d < 4 && w.n_k0_cols > 0; ++d) tw += (w.t_off[d + 1] - w.t_off[d] + 63) / 64;
    const int waves = s_waves + tw + w.n_k0_rows;
    launch(k0_incremental, dim3(static_cast<unsigned>(std::max(1, (waves + 3) / 4))), dim3(256), 0, s, ev0, ev1, w,
           s_waves, tw, local_first_fallback);
    return hipGetLastError();
  }
  launch(k0_tables, dim3(blocks), dim3(256), 0, s, ev0, ev1, w, s_blocks, local_first_fallback);
  return hipGetLastError();
}

hipError_t launch_placement(const DevWorkload& w, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  return w.prof ? launch_k2<true>(w, s, ev0, ev1) : launch_k2<false>(w, s, ev0, ev1);
}

hipError_t launch_winner(const DevWorkload& w, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
  launch(k3_winner, dim3(1), dim3(64), 0, s, ev0, ev1, w);
  return hipGetLastError();
}
#endif  // SR_KPART 0

}  // namespace sr
