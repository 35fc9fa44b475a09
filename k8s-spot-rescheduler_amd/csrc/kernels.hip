// kernels.hip — gfx950 (CDNA4, wave64) kernels of the drain planner.
//
//  K0 tables      S (static class) and T (capacity threshold) bitmask rows over
//                 spot nodes: one lane per node, one 64-bit ballot per word
//                 (predicate factorisation: encode.cpp).
//  K2 placement   canDrainNode for every candidate at once (rescheduler.go:357-370):
//                 one wave per candidate, pods in order; the pod's feasibility
//                 row F = S & T & T & T is formed 64 words at a time from the
//                 tables and first fit in NodeInfoArray order = lowest set bit
//                 among untouched nodes (ballot + ctz), touched nodes rechecked
//                 against the candidate's private capacity copy in registers.
//  K3 winner      first drainable candidate's pod -> node mapping.
//
// No MFMA: there is no dense contraction anywhere on this path.
#include <algorithm>
#include <climits>

#include "kernels.hpp"

namespace sr {
namespace {

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

// K2: one wave per candidate.  Touched-node slots live in registers, one per
// lane (64; a candidate touching more distinct nodes is rerun with 512), and
// CH*64 bitmask words per row are held as a register-resident touched mask
// (lane l owns words ch*64 + l).
//
// The feasibility of pod p against the base snapshot is evaluated here, 64
// words (4096 spot nodes) at a time: F = S[class] & T[cpu] & T[mem] & T[eph]
// (encode.cpp).  The table rows are small and L2-resident, so no dense P x N
// bitmask is ever written: a pod's chunk costs four 512-B row reads.
//
// It is one dependent chain per candidate, so it is built for latency: every
// load inside the pod loop is an LDS-DMA (global_load_lds) whose completion
// is waited for by hand with counted `s_waitcnt vmcnt(N)`:
//   - chunk 0 of the four rows of pods p+1..p+3 is always in flight (4-slot
//     LDS ring, 2 DMAs per pod);
//   - the base record of the next pod's first untouched feasible node is
//     fetched one pod ahead (speculative; used when the pod opens a new slot
//     on a node >= kNodeCache; nodes below that come from an LDS cache);
//   - the candidate's pod records are staged before the loop (128-pod window,
//     restaged per 64 pods for larger candidates).
// DMA issue order per step k (fixed): ... spec(k+1), rows(k+4) x2.  At the end
// of step k, rows(k+1) has at most 6 younger DMAs (5 at k = 0) and every wait
// below is for "all but the N youngest" -> vmcnt(5) is safe for every k;
// spec(k) has exactly the two rows(k+3) DMAs younger when step k consumes it
// -> vmcnt(2).  Rare-path DMAs are always followed by vmcnt(0), which never
// weakens a later count.
typedef __attribute__((address_space(3))) void* lds_vp;
typedef __attribute__((address_space(1))) void* gbl_vp;
#define SR_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

constexpr int kPodWin = 128;    // pod records staged per wave: two 64-pod halves
constexpr int kRecU64 = 6;      // {cpu, memory, ephemeral, ports, S | T cpu row offset, T mem | T eph row offset}
constexpr int kNodeCache = 16;  // base records of spot nodes [0, 16) kept in LDS
constexpr int kMaxPods = 512;   // pods per candidate on the device (encode.cpp: more -> fallback)

struct K2Lds {
  uint64_t ring[4][256];            // chunk 0 of {S, T cpu, T mem, T eph} rows of pods k..k+3
  uint64_t chunk[256];              // rare: chunk > 0 of the current pod's rows
  uint64_t pods[kPodWin][kRecU64];  // pod record window
  uint64_t cache[kNodeCache][8];    // base node records
  uint64_t spec[8];                 // speculative node record
  uint64_t rec[8];                  // rare: reloaded node record
  int32_t omap[kMaxPods];           // spot position chosen for each pod
};

struct K2Stats {
  uint32_t n_spec_miss = 0, n_min = 0, n_far = 0;
  uint64_t cyc_a = 0, cyc_b = 0, cyc_c = 0, cyc_d = 0;
};

// One candidate's canDrainNode with 64 * SPL touched-node slots.  Returns the
// number of pods placed (np = all; status = failing pod or -1), or -1 when the
// candidate touches more distinct nodes than it has slots (the caller reruns
// it with more).
template <int SPL, int CH, bool PROF>
__device__ __forceinline__ int k2_run(const DevWorkload& w, K2Lds& L, const int p0, const int np, int& status,
                                      K2Stats& st) {
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
#pragma unroll
  for (int s = 0; s < SPL; ++s) {
    snode[s] = INT_MAX;
    scpu[s] = smem[s] = seph[s] = 0;
    sleft[s] = 0;
    sport[s] = 0;
  }
  int nslots = 0;
  uint64_t cyc_t = 0;
  auto cyc = [&]() -> uint64_t { return PROF ? __builtin_amdgcn_s_memtime() : 0ull; };
  const uint64_t lane_mask = lane < Wp ? ~0ull : 0ull;

  // State of the next pod, gathered in one batch of LDS reads once its rows
  // have landed: its chunk-0 feasibility word, first untouched feasible node,
  // request, and the S-row bit of every touched node.
  uint64_t word_next = 0;
  int cnode0 = INT_MAX;
  int64_t nrc = 0, nrm = 0, nre = 0;
  uint64_t npm = 0;
  bool sbit[SPL];
  auto gather_next = [&](int kn) {
    const uint64_t* img = L.ring[kn & 3];
    const uint64_t* pr = L.pods[kn & (kPodWin - 1)];
    uint64_t sw[SPL];
#pragma unroll
    for (int s = 0; s < SPL; ++s) sw[s] = img[snode[s] < 4096 ? snode[s] >> 6 : 0];
    const uint64_t a = img[lane] & img[64 + lane] & img[128 + lane] & img[192 + lane];
    nrc = static_cast<int64_t>(pr[0]);
    nrm = static_cast<int64_t>(pr[1]);
    nre = static_cast<int64_t>(pr[2]);
    npm = pr[3];
#pragma unroll
    for (int s = 0; s < SPL; ++s) sbit[s] = (sw[s] >> (snode[s] & 63)) & 1ull;
    word_next = a & lane_mask;
    const uint64_t clean0 = word_next & ~touched[0];
    const uint64_t mc0 = __ballot(clean0 != 0);
    cnode0 = INT_MAX;
    if (mc0) {
      const int L0 = __builtin_ctzll(mc0);
      cnode0 = L0 * 64 + __builtin_ctzll(readlane64(clean0, L0));
    }
  };

  // prologue: node cache + pod window, then rows 0..2, (row 0 landed) spec(0), row 3
  dma(w.node_rec + 2 * lane, L.cache[0]);
  dma_pods(0);
  if (np > 64) dma_pods(1);
  SR_WAIT_VM(0);
  dma_rows_of(L.ring[0], 0, 0);
  dma_rows_of(L.ring[1], min(1, np - 1), 0);
  dma_rows_of(L.ring[2], min(2, np - 1), 0);
  SR_WAIT_VM(4);
  gather_next(0);
  dma_rec(L.spec, cnode0);
  dma_rows_of(L.ring[3], min(3, np - 1), 0);

  status = -1;
  int k = 0;
  for (; k < np; ++k) {
    if (PROF) cyc_t = cyc();
    const int64_t rc = nrc, rm = nrm, re = nre;
    const uint64_t pm = npm;
    const bool zero = (rc | rm | re) == 0;  // fitsRequest skips the resource checks
    // Chunk 0 (spot nodes [0, 4096)): touched nodes below the first untouched
    // feasible one, rechecked branch-free: class bit from the S row, capacity /
    // pod count / host ports from the candidate's own state (which implies the
    // base T rows, base pod count and base ports).
    int ans;
    {
      const int hi = min(cnode0, 4096);
      int best = INT_MAX;
#pragma unroll
      for (int s = 0; s < SPL; ++s) {
        const int nd = snode[s];
        const bool fit = zero | ((rc <= scpu[s]) & (rm <= smem[s]) & (re <= seph[s]));  // NodeResourcesFit
        const bool ok = (nd < hi) & sbit[s] & (sleft[s] >= 1) & ((sport[s] & pm) == 0) & fit;
        best = ok ? min(best, nd) : best;
      }
      const uint64_t hb = __ballot(best != INT_MAX);
      int dnode = INT_MAX;
      if (hb) {
        dnode = (hb & (hb - 1)) ? wave_min(best) : __builtin_amdgcn_readlane(best, __builtin_ctzll(hb));
        if (PROF && (hb & (hb - 1))) ++st.n_min;
      }
      ans = min(cnode0, dnode);
    }
    // rare: the pod's first 4096 spot nodes hold no answer
#pragma unroll
    for (int ch = 1; ch < CH; ++ch) {
      const int base = ch * 64;
      if (ans != INT_MAX || base >= Wp) continue;  // wave-uniform; keeps the loop unrollable
      if (PROF) ++st.n_far;
      dma_rows_of(L.chunk, k, base);
      SR_WAIT_VM(0);
      const uint64_t* img = L.chunk;
      const uint64_t clean = (img[lane] & img[64 + lane] & img[128 + lane] & img[192 + lane]) &
                             ((base + lane < Wp) ? ~touched[ch] : 0ull);
      const uint64_t mc = __ballot(clean != 0);
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
        const bool fit = zero | ((rc <= scpu[s]) & (rm <= smem[s]) & (re <= seph[s]));
        const bool ok = in & (((sw >> (nd & 63)) & 1ull) != 0) & (sleft[s] >= 1) & ((sport[s] & pm) == 0) & fit;
        best = ok ? min(best, nd) : best;
      }
      ans = min(cnode, wave_min(best));
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
      if (ns >= 64 * SPL) {  // slots exhausted: rerun with more
        SR_WAIT_VM(0);
        return -1;
      }
      const uint64_t* rec;
      if (ans < kNodeCache) {
        rec = L.cache[ans];
      } else if (ans == cnode0) {
        SR_WAIT_VM(2);  // spec(k): only rows(k+3) are younger
        rec = L.spec;
      } else {  // rare: not the speculated node
        if (PROF) ++st.n_spec_miss;
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
          scpu[s] = fc - rc;
          smem[s] = fm - rm;
          seph[s] = fe - re;
          sleft[s] = pl - 1;
          sport[s] = pb | pm;
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
    // next pod: its rows (<= 6 younger DMAs), its state, its speculative
    // record, rows of pod k + 4
    if (k + 1 < np) {
      const int q = min(k + 4, np - 1);
      const bool restage = q == k + 4 && (q & 63) == 0 && q >= kPodWin;
      if (restage) dma_pods(q >> 6);  // window: records [q, q + 64) replace [q - 128, q - 64)
      SR_WAIT_VM(5);
      if (restage) SR_WAIT_VM(0);
      if (PROF) {
        const uint64_t t = cyc();
        st.cyc_c += t - cyc_t;
        cyc_t = t;
      }
      const uint64_t* pq = L.pods[q & (kPodWin - 1)];
      const uint64_t r01 = pq[4], r23 = pq[5];
      gather_next(k + 1);
      dma_rec(L.spec, cnode0);  // L.spec's last reads (this step) have returned
      dma_rows(L.ring[k & 3], r01, r23, 0);
      if (PROF) st.cyc_d += cyc() - cyc_t;
    }
  }
  SR_WAIT_VM(0);  // no LDS-DMA may outlive the wave's LDS allocation
  return status >= 0 ? status : np;
}

// K2: one wave per candidate (list entries {candidate, first pod, end pod,
// global index}, longest candidates first).
template <int CH, bool PROF>
__global__ __launch_bounds__(256) void k2_place(DevWorkload w, const int4* __restrict__ list, int n_list) {
  extern __shared__ __attribute__((aligned(16))) uint64_t k2_lds[];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int li = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + wave);
  if (li >= n_list) return;
  const uint64_t t_start = PROF ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint64_t c_start = PROF ? __builtin_amdgcn_s_memtime() : 0;
  const int4 e = list[li];
  const int ci = __builtin_amdgcn_readfirstlane(e.x);
  const int p0 = __builtin_amdgcn_readfirstlane(e.y);
  const int np = __builtin_amdgcn_readfirstlane(e.z) - p0;  // >= 1: empty candidates never reach the device
  const int g = __builtin_amdgcn_readfirstlane(e.w);
  K2Lds& L = *reinterpret_cast<K2Lds*>(k2_lds + static_cast<size_t>(wave) * (sizeof(K2Lds) / 8));

  K2Stats st;
  int status = -1;
  int placed = k2_run<1, CH, PROF>(w, L, p0, np, status, st);
  const int wide = placed < 0 ? 1 : 0;
  if (placed < 0) placed = k2_run<8, CH, PROF>(w, L, p0, np, status, st);  // > 64 distinct nodes

  for (int i = lane; i < np; i += 64) w.out_node[p0 + i] = i < placed ? L.omap[i] : -1;
  if (lane == 0) {
    w.out_status[ci] = status;
    // packed (global candidate << 32 | local candidate): min = first drainable
    if (status < 0)
      atomicMin(reinterpret_cast<unsigned long long*>(w.d_min),
                (static_cast<unsigned long long>(g) << 32) | static_cast<unsigned>(ci));
    if (PROF) {
      uint64_t* pr = w.prof + static_cast<size_t>(ci) * 16;
      pr[0] = t_start;
      pr[1] = t_start;
      pr[2] = __builtin_amdgcn_s_memrealtime();
      pr[3] = __builtin_amdgcn_s_memtime() - c_start;
      pr[4] = static_cast<uint64_t>(status >= 0 ? status + 1 : np);
      pr[5] = static_cast<uint64_t>(wide);
      pr[6] = st.n_spec_miss;
      pr[7] = static_cast<uint64_t>(st.n_min) | (static_cast<uint64_t>(st.n_far) << 32);
      pr[8] = st.cyc_a;
      pr[9] = st.cyc_b;
      pr[10] = st.cyc_c;
      pr[11] = st.cyc_d;
    }
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

template <bool PROF>
hipError_t launch_k2(const DevWorkload& w, hipStream_t s) {
  const int n = w.n_list;
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4), block(256);
  const size_t lds = 4 * sizeof(K2Lds);
  const int chunks = (w.Wp + 63) / 64;
  if (chunks <= 1) hipLaunchKernelGGL((k2_place<1, PROF>), grid, block, lds, s, w, w.list, n);
  else if (chunks <= 2) hipLaunchKernelGGL((k2_place<2, PROF>), grid, block, lds, s, w, w.list, n);
  else if (chunks <= 4) hipLaunchKernelGGL((k2_place<4, PROF>), grid, block, lds, s, w, w.list, n);
  else if (chunks <= 8) hipLaunchKernelGGL((k2_place<8, PROF>), grid, block, lds, s, w, w.list, n);
  else if (chunks <= 16) hipLaunchKernelGGL((k2_place<16, PROF>), grid, block, lds, s, w, w.list, n);
  else hipLaunchKernelGGL((k2_place<32, PROF>), grid, block, lds, s, w, w.list, n);
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

hipError_t launch_placement(const DevWorkload& w, hipStream_t s) {
  return w.prof ? launch_k2<true>(w, s) : launch_k2<false>(w, s);
}

hipError_t launch_winner(const DevWorkload& w, hipStream_t s) {
  hipLaunchKernelGGL(k3_winner, dim3(1), dim3(64), 0, s, w);
  return hipGetLastError();
}

}  // namespace sr
