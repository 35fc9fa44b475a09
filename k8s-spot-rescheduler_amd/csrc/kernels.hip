// kernels.hip — gfx950 (CDNA4, wave64) kernels of the drain planner.
//
//  K0 tables      S (static class) and T (capacity threshold) bitmask rows over
//                 spot nodes: one lane per node, one 64-bit ballot per word
//                 (predicate factorisation: encode.cpp).
//  K1 feasibility dense pod x spot-node bitmask F = S & T & T & T per pod: the
//                 (pod, node) predicate of every pair against the base snapshot,
//                 16 B per lane, HBM-write bound.
//  K2 placement   canDrainNode for every candidate at once (rescheduler.go:357-370):
//                 one wave per candidate, pods in order, first fit in
//                 NodeInfoArray order = lowest set bit of F[p] among untouched
//                 nodes (ballot + ctz), touched nodes rechecked against the
//                 candidate's private capacity copy held in registers.
//  K3 winner      first drainable candidate's pod -> node mapping.
//
// No MFMA: there is no dense contraction anywhere on this path.
#include <algorithm>
#include <climits>

#include "kernels.hpp"

namespace sr {
namespace {

constexpr int kWave = 64;

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

// S row of one class for word w: its atom program evaluated 64 nodes at a time.
//   NodeAffinity (nodeSelector pairs; required terms ORed, requirements ANDed),
//   TaintToleration + NodeUnschedulable (untolerated taint atoms negated),
//   NodePorts (the class's ports against base UsedPorts), pod count (atom 0).
__device__ __forceinline__ uint64_t class_word(const DevWorkload& w, int cls, int word) {
  const size_t Wp = static_cast<size_t>(w.Wp);
  const uint64_t* __restrict__ at = w.atoms + word;
  uint64_t acc = ~0ull;
  for (int i = w.cls_and_off[cls]; i < w.cls_and_off[cls + 1]; ++i) acc &= at[w.cls_and[i] * Wp];
  for (int i = w.cls_not_off[cls]; i < w.cls_not_off[cls + 1]; ++i) acc &= ~at[w.cls_not[i] * Wp];
  const int flags = w.cls_flags[cls];
  if (flags & 1) {
    uint64_t any = 0;
    for (int t = w.cls_term_off[cls]; t < w.cls_term_off[cls + 1]; ++t) {
      uint64_t all = ~0ull;
      for (int i = w.term_atom_off[t]; i < w.term_atom_off[t + 1]; ++i) all &= at[w.term_atoms[i] * Wp];
      any |= all;
    }
    acc &= any;
  }
  return (flags & 2) ? 0 : acc;
}

// K0: bitmask rows.  Blocks [0, s_blocks): one wave per class, lanes = words
// (S rows, word-parallel atom programs).  Blocks after: T rows, grid over
// (row groups of 64) x (Wp / 4): each wave owns one 64-node word, loads its
// nodes' free capacity once and evaluates 64 thresholds (one ballot each),
// lane t keeping row r0 + t.
__global__ __launch_bounds__(256) void k0_tables(DevWorkload w, int s_blocks, int wblocks, int local_first_fallback) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    unsigned long long* dm = reinterpret_cast<unsigned long long*>(w.d_min);
    dm[0] = ~0ull;
    dm[1] = local_first_fallback < 0 ? ~0ull : static_cast<unsigned long long>(local_first_fallback) << 32;
  }
  if (static_cast<int>(blockIdx.x) < s_blocks) {
    const int cls = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + wave);
    if (cls >= w.n_classes) return;
    for (int word = lane; word < w.Wp; word += 64)
      w.S[static_cast<size_t>(cls) * w.Wp + word] = class_word(w, cls, word);
    return;
  }
  const int b = static_cast<int>(blockIdx.x) - s_blocks;
  const int g = b / wblocks;
  const int word = (b - g * wblocks) * 4 + wave;
  if (word >= w.Wp) return;  // wave-uniform
  const int n = word * 64 + lane;  // < n_pad: node arrays are padded
  const bool valid = n < w.n_spot;
  const int r0 = g * 64;
  const int nr = min(64, w.n_t - r0);
  const int64_t fc = w.free_cpu[n], fm = w.free_mem[n], fe = w.free_eph[n];
  const int my_dim = lane < nr ? w.t_dim[r0 + lane] : 3;
  const int64_t my_thr = lane < nr ? w.t_thr[r0 + lane] : 0;
  uint64_t acc = 0;
  for (int t = 0; t < nr; ++t) {
    const int dim = __builtin_amdgcn_readlane(my_dim, t);
    const int64_t thr = static_cast<int64_t>(readlane64(static_cast<uint64_t>(my_thr), t));
    const int64_t v = dim == 0 ? fc : (dim == 1 ? fm : fe);
    const uint64_t m = __ballot(valid && (dim == 3 || v >= thr));
    if (lane == t) acc = m;
  }
  if (lane < nr) w.T[static_cast<size_t>(r0 + lane) * w.Wp + word] = acc;
}

// K1: F[p] = S[s] & T[cpu] & T[mem] & T[eph]; one item = 16 B of one row, four
// independent items in flight per thread.
__device__ __forceinline__ ulonglong2 and4(ulonglong2 a, ulonglong2 b, ulonglong2 c, ulonglong2 d) {
  ulonglong2 f;
  f.x = a.x & b.x & c.x & d.x;
  f.y = a.y & b.y & c.y & d.y;
  return f;
}

__global__ __launch_bounds__(256) void k1_feasibility(const ulonglong2* __restrict__ S, const ulonglong2* __restrict__ T,
                                                      const int4* __restrict__ rows, ulonglong2* __restrict__ F,
                                                      uint32_t n_pods, uint32_t half) {
  const uint32_t total = n_pods * half;
  const uint32_t stride = gridDim.x * blockDim.x;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  constexpr int U = 4;
  for (; i + (U - 1) * stride < total; i += U * stride) {
    ulonglong2 a[U], b[U], c[U], d[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = i + u * stride;
      const uint32_t p = k / half;
      const uint32_t j = k - p * half;
      const int4 r = rows[p];
      a[u] = S[static_cast<size_t>(r.x) * half + j];
      b[u] = T[static_cast<size_t>(r.y) * half + j];
      c[u] = T[static_cast<size_t>(r.z) * half + j];
      d[u] = T[static_cast<size_t>(r.w) * half + j];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) F[i + u * stride] = and4(a[u], b[u], c[u], d[u]);
  }
  for (; i < total; i += stride) {
    const uint32_t p = i / half;
    const uint32_t j = i - p * half;
    const int4 r = rows[p];
    F[i] = and4(S[static_cast<size_t>(r.x) * half + j], T[static_cast<size_t>(r.y) * half + j],
                T[static_cast<size_t>(r.z) * half + j], T[static_cast<size_t>(r.w) * half + j]);
  }
}

// K2: one wave per candidate.  SPL touched-node slots per lane (64*SPL per
// candidate), CH*64 bitmask words per row held as a register-resident
// touched mask (lane l owns words ch*64 + l).
//
// It is one dependent chain per candidate, so it is built for latency: every
// load inside the pod loop is an LDS-DMA (global_load_lds) whose completion
// is waited for by hand with counted `s_waitcnt vmcnt(N)`:
//   - chunk 0 of rows p+1..p+3 is always in flight (4-slot LDS ring);
//   - the base record of the next pod's first untouched feasible node is
//     fetched one pod ahead (speculative; used when the pod opens a new slot);
//   - the candidate's pod records are staged once before the loop.
// DMA issue order per step k (fixed): ... spec(k+1), row(k+4).  At the end of
// step k-1, row k has >= 3 younger DMAs (spec(k-1)?, row(k+1), spec(k), row(k+2)
// for k >= 2; row(k+1), spec(k)... for k = 1) -> vmcnt(3); spec(k) has exactly
// one younger (row(k+3)) when step k consumes it -> vmcnt(1).  Extra DMAs
// (rare paths) are always followed by vmcnt(0), which never weakens a count.
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) void* gbl_vp;
#define SR_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

struct K2Lds {
  uint64_t row[4][64];  // row ring: chunk 0 of rows p..p+3
  uint64_t chunk[64];   // rare: chunks > 0
  uint64_t spec[8];     // speculative node record
  uint64_t rec[8];      // rare: reloaded node record
};

template <int SPL, int CH>
__global__ __launch_bounds__(256) void k2_place(DevWorkload w, const int32_t* __restrict__ list, int n_list) {
  extern __shared__ __attribute__((aligned(16))) uint64_t k2_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int li = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + wave);
  if (li >= n_list) return;
  const int ci = __builtin_amdgcn_readfirstlane(list[li]);
  const int p0 = __builtin_amdgcn_readfirstlane(w.cand_off[ci]);
  const int p1 = __builtin_amdgcn_readfirstlane(w.cand_off[ci + 1]);
  const int np = p1 - p0;
  const int Wp = w.Wp;
  // per-wave LDS: pod records [64*SPL][4] then the K2Lds block
  uint64_t* pods = k2_lds + static_cast<size_t>(wave) * (64 * SPL * 4 + sizeof(K2Lds) / 8);
  K2Lds& L = *reinterpret_cast<K2Lds*>(pods + 64 * SPL * 4);

  // DMA helpers: 16 B per lane, LDS destination = base + 16 * lane
  auto dma_row = [&](uint64_t* dst, int p, int base) {  // 64 words of row p from word `base`
    if (lane < 32) {
      const int wi = min(base + 2 * lane, Wp - 2);
      const uint64_t* src = w.F + static_cast<size_t>(min(p, p1 - 1)) * Wp + wi;
      __builtin_amdgcn_global_load_lds((gbl_vp)src, (lds_vp)dst, 16, 0, 0);
    }
  };
  auto dma_rec = [&](uint64_t* dst, int node) {
    if (lane < 4) {
      const uint64_t* src = w.node_rec + static_cast<size_t>(node == INT_MAX ? 0 : node) * 8 + 2 * lane;
      __builtin_amdgcn_global_load_lds((gbl_vp)src, (lds_vp)dst, 16, 0, 0);
    }
  };

  // pod records (AoS, 32 B per pod): 2 KB per 64 pods = 2 DMAs of 1 KB
#pragma unroll
  for (int b = 0; b < 2 * SPL; ++b)
    if (b * 32 < np) {
      const uint64_t* src = w.pod_rec + static_cast<size_t>(p0) * 4 + static_cast<size_t>(b) * 128 + 2 * lane;
      __builtin_amdgcn_global_load_lds((gbl_vp)src, (lds_vp)(pods + b * 128), 16, 0, 0);
    }

  uint64_t touched[CH];
#pragma unroll
  for (int ch = 0; ch < CH; ++ch) touched[ch] = 0;
  int snode[SPL];
  int64_t scpu[SPL], smem[SPL], seph[SPL];
  int sleft[SPL];
  uint64_t sport[SPL];
  int bnode[SPL];
#pragma unroll
  for (int s = 0; s < SPL; ++s) {
    snode[s] = INT_MAX;
    scpu[s] = smem[s] = seph[s] = 0;
    sleft[s] = 0;
    sport[s] = 0;
    bnode[s] = -1;
  }
  int nslots = 0;
  int status = -1;
  const uint64_t lane_mask = lane < Wp ? ~0ull : 0ull;

  auto first_clean0 = [&](uint64_t word) -> int {
    const uint64_t clean0 = word & ~touched[0];
    const uint64_t mc0 = __ballot(clean0 != 0);
    if (!mc0) return INT_MAX;
    const int L0 = __builtin_ctzll(mc0);
    return L0 * 64 + __builtin_ctzll(readlane64(clean0, L0));
  };

  // prologue: rows 0..2, then (row 0 landed) spec(0), row 3
  dma_row(L.row[0], p0, 0);
  dma_row(L.row[1], p0 + 1, 0);
  dma_row(L.row[2], p0 + 2, 0);
  SR_WAIT_VM(2);
  uint64_t word_next = L.row[0][lane] & lane_mask;
  int cnode0 = first_clean0(word_next);
  dma_rec(L.spec, cnode0);
  dma_row(L.row[3], p0 + 3, 0);

  for (int k = 0; k < np; ++k) {
    const int p = p0 + k;
    const uint64_t word0 = word_next;
    const uint64_t* prec = pods + static_cast<size_t>(k) * 4;
    const int64_t rc = static_cast<int64_t>(prec[0]), rm = static_cast<int64_t>(prec[1]),
                  re = static_cast<int64_t>(prec[2]);
    const uint64_t pm = prec[3];
    const bool zero = (rc | rm | re) == 0;  // fitsRequest skips the resource checks

    int ans = INT_MAX;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
      const int base = ch * 64;
      if (ans != INT_MAX || base >= Wp) continue;  // wave-uniform; keeps the loop unrollable
      uint64_t word = word0;
      int cnode = cnode0;
      if (ch > 0) {  // rare: the pod's first 4096 spot nodes hold no answer
        dma_row(L.chunk, p, base);
        SR_WAIT_VM(0);
        word = (base + lane < Wp) ? L.chunk[lane] : 0;
        const uint64_t clean = word & ~touched[ch];
        const uint64_t mc = __ballot(clean != 0);
        cnode = INT_MAX;
        if (mc) {
          const int L0 = __builtin_ctzll(mc);
          cnode = (base + L0) * 64 + __builtin_ctzll(readlane64(clean, L0));
        }
      }
      // touched base-feasible nodes below it: recheck with the candidate's own state
      int dnode = INT_MAX;
      if (__ballot((word & touched[ch]) != 0)) {
        const int lo = base * 64;
        const int hi = min(cnode, lo + 64 * 64);
        int best = INT_MAX;
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          const int nd = snode[s];
          const bool in = nd >= lo && nd < hi;
          const uint64_t ws = __shfl(word, in ? (nd >> 6) - base : lane, kWave);
          bool ok = in && ((ws >> (nd & 63)) & 1ull);
          ok = ok && sleft[s] >= 1 && (sport[s] & pm) == 0;                 // pod count, host ports
          ok = ok && (zero || (rc <= scpu[s] && rm <= smem[s] && re <= seph[s]));  // NodeResourcesFit
          if (ok) best = min(best, nd);
        }
        dnode = wave_min(best);
      }
      ans = min(cnode, dnode);
    }
    if (ans == INT_MAX) {  // "pod %s can't be rescheduled on any existing spot node"
      status = k;
      break;
    }
#pragma unroll
    for (int b = 0; b < SPL; ++b)
      if (b == (k >> 6) && lane == (k & 63)) bnode[b] = ans;

    // ClusterSnapshot.AddPod(pod, node) on the candidate's private copy
    bool hit = false;
#pragma unroll
    for (int s = 0; s < SPL; ++s) {
      if (snode[s] == ans) {
        scpu[s] -= rc;
        smem[s] -= rm;
        seph[s] -= re;
        sleft[s] -= 1;
        sport[s] |= pm;
        hit = true;
      }
    }
    if (!__any(hit)) {
      const int ns = nslots++;
      const uint64_t* rec = L.spec;
      SR_WAIT_VM(1);  // spec(k): only row(k+3) is younger
      if (ans != cnode0) {  // rare: not the speculated node
        dma_rec(L.rec, ans);
        SR_WAIT_VM(0);
        rec = L.rec;
      }
      const int64_t fc = static_cast<int64_t>(rec[0]), fm = static_cast<int64_t>(rec[1]),
                    fe = static_cast<int64_t>(rec[2]);
      const uint64_t pb = rec[3];
      const int pl = static_cast<int>(static_cast<int64_t>(rec[4]));
      if (lane == (ns & 63)) {
#pragma unroll
        for (int s = 0; s < SPL; ++s) {
          if (s == (ns >> 6)) {
            snode[s] = ans;
            scpu[s] = fc - rc;
            smem[s] = fm - rm;
            seph[s] = fe - re;
            sleft[s] = pl - 1;
            sport[s] = pb | pm;
          }
        }
      }
      const int tw = ans >> 6;
#pragma unroll
      for (int ch = 0; ch < CH; ++ch)
        if (tw == ch * 64 + lane) touched[ch] |= 1ull << (ans & 63);
    }
    // next pod: its row (>= 3 younger DMAs), its speculative record, row k + 4
    if (k + 1 < np) {
      SR_WAIT_VM(3);
      word_next = L.row[(k + 1) & 3][lane] & lane_mask;
      cnode0 = first_clean0(word_next);
      dma_rec(L.spec, cnode0);  // L.spec's last reads (this step) have returned
      dma_row(L.row[k & 3], p + 4, 0);
    }
  }

  SR_WAIT_VM(0);  // no LDS-DMA may outlive the wave's LDS allocation
#pragma unroll
  for (int b = 0; b < SPL; ++b) {
    const int q = p0 + 64 * b + lane;
    if (q < p1) w.out_node[q] = bnode[b];
  }
  if (lane == 0) {
    w.out_status[ci] = status;
    // packed (global candidate << 32 | local candidate): min = first drainable
    if (status < 0)
      atomicMin(reinterpret_cast<unsigned long long*>(w.d_min),
                (static_cast<unsigned long long>(w.cand_global[ci]) << 32) | static_cast<unsigned>(ci));
  }
}

// K3: one wave.  d_min[0] = packed first drainable candidate (possibly reduced
// over ranks), d_min[1] = packed first fallback; the winner's mapping is
// copied only by the rank that owns it.  `result` lives in mapped host memory.
__global__ __launch_bounds__(64) void k3_winner(DevWorkload w) {
  const unsigned long long* dm = reinterpret_cast<const unsigned long long*>(w.d_min);
  const unsigned long long ok = dm[0], fb = dm[1];
  int* r = w.result;
  const bool any = ok != ~0ull;
  const int g = any ? static_cast<int>(ok >> 32) : -1;
  const int li = any ? static_cast<int>(ok & 0xffffffffu) : -1;
  const bool local = any && li < w.n_cand && w.cand_global[li] == g;
  const int off = local ? w.cand_off[li] : 0;
  const int np = local ? w.cand_off[li + 1] - off : 0;
  for (int q = threadIdx.x; q < np; q += 64) r[4 + q] = w.out_node[off + q];
  if (threadIdx.x == 0) {
    r[0] = g;
    r[1] = local ? 1 : 0;
    r[2] = np;
    r[3] = fb == ~0ull ? -1 : static_cast<int>(fb >> 32);
  }
}

template <int SPL>
hipError_t launch_k2_variant(const DevWorkload& w, const int32_t* list, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4), block(256);
  const size_t lds = 4 * (64 * SPL * 4 * sizeof(uint64_t) + sizeof(K2Lds));
  const int chunks = (w.Wp + 63) / 64;
  if (chunks <= 1) hipLaunchKernelGGL((k2_place<SPL, 1>), grid, block, lds, s, w, list, n);
  else if (chunks <= 2) hipLaunchKernelGGL((k2_place<SPL, 2>), grid, block, lds, s, w, list, n);
  else if (chunks <= 4) hipLaunchKernelGGL((k2_place<SPL, 4>), grid, block, lds, s, w, list, n);
  else if (chunks <= 8) hipLaunchKernelGGL((k2_place<SPL, 8>), grid, block, lds, s, w, list, n);
  else if (chunks <= 16) hipLaunchKernelGGL((k2_place<SPL, 16>), grid, block, lds, s, w, list, n);
  else hipLaunchKernelGGL((k2_place<SPL, 32>), grid, block, lds, s, w, list, n);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_tables(const DevWorkload& w, int32_t local_first_fallback, hipStream_t s) {
  const int s_blocks = (w.n_classes + 3) / 4;
  const int t_groups = (w.n_t + 63) / 64;
  const int wblocks = (w.Wp + 3) / 4;
  const unsigned blocks = static_cast<unsigned>(std::max(1, s_blocks + t_groups * wblocks));
  hipLaunchKernelGGL(k0_tables, dim3(blocks), dim3(256), 0, s, w, s_blocks, wblocks, local_first_fallback);
  return hipGetLastError();
}

hipError_t launch_feasibility(const DevWorkload& w, hipStream_t s) {
  if (w.n_pods <= 0) return hipSuccess;
  const uint32_t half = static_cast<uint32_t>(w.Wp / 2);
  const uint64_t total = static_cast<uint64_t>(w.n_pods) * half;
  // ~4 items per thread, at least one wave of work per SIMD
  const uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((total + 1023) / 1024, 256 * 16));
  hipLaunchKernelGGL(k1_feasibility, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s,
                     reinterpret_cast<const ulonglong2*>(w.S), reinterpret_cast<const ulonglong2*>(w.T), w.pod_rows,
                     reinterpret_cast<ulonglong2*>(w.F), static_cast<uint32_t>(w.n_pods), half);
  return hipGetLastError();
}

hipError_t launch_placement(const DevWorkload& w, hipStream_t s) {
  hipError_t e = launch_k2_variant<2>(w, w.list_small, w.n_small, s);
  if (e != hipSuccess) return e;
  return launch_k2_variant<8>(w, w.list_large, w.n_large, s);
}

hipError_t launch_winner(const DevWorkload& w, hipStream_t s) {
  hipLaunchKernelGGL(k3_winner, dim3(1), dim3(64), 0, s, w);
  return hipGetLastError();
}

}  // namespace sr
