// kernels.hip — gfx950 (CDNA4, wave64) kernels of the drain planner.
//
//  K0 tables      A/B bitmask rows over spot nodes: one lane per node, one
//                 64-bit ballot per word (predicate factorisation: encode.cpp).
//  K1 feasibility dense pod x spot-node bitmask F = A[a(p)] & B[b(p)]: the
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

__device__ __forceinline__ int wave_min(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, kWave));
  return v;
}

// Static part of the predicate for class `cls` on spot node n (bitset tests):
// NodeAffinity (nodeSelector + required terms), TaintToleration +
// NodeUnschedulable (pseudo-taint), NodePorts against the base UsedPorts.
__device__ __forceinline__ bool static_ok(const DevWorkload& w, int cls, int n) {
  const int flags = w.cls_flags[cls];
  if (flags & 2) return false;  // CLS_IMPOSSIBLE: required affinity without a satisfiable term
  const int WR = w.WR, WT = w.WT;
  const size_t NP = static_cast<size_t>(w.n_pad);
  for (int k = 0; k < WR; ++k) {
    const uint64_t s = w.cls_sel[cls * WR + k];
    if ((w.req_bits[k * NP + n] & s) != s) return false;
  }
  if (flags & 1) {  // CLS_AFF_REQUIRED: terms are ORed, requirements in a term ANDed
    bool any = false;
    for (int t = w.cls_term_off[cls]; t < w.cls_term_off[cls + 1] && !any; ++t) {
      bool all = true;
      for (int k = 0; k < WR; ++k) {
        const uint64_t m = w.term_mask[t * WR + k];
        all = all && (w.req_bits[k * NP + n] & m) == m;
      }
      any = all;
    }
    if (!any) return false;
  }
  for (int k = 0; k < WT; ++k)
    if (w.taint_bits[k * NP + n] & ~w.cls_tol[cls * WT + k]) return false;
  return (w.port_bits[n] & w.cls_port[cls]) == 0;
}

// K0: grid = (n_a + n_b) rows x ceil(Wp / 4) blocks; 4 waves per block, one word each.
__global__ __launch_bounds__(256) void k0_tables(DevWorkload w, int wblocks, int local_first_fallback) {
  const int row = blockIdx.x / wblocks;
  const int wb = blockIdx.x - row * wblocks;
  const int lane = threadIdx.x & 63;
  const int word = wb * 4 + (threadIdx.x >> 6);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    w.d_min[0] = INT_MAX;
    w.d_min[1] = local_first_fallback < 0 ? INT_MAX : local_first_fallback;
  }
  if (word >= w.Wp) return;  // wave-uniform
  const int n = word * 64 + lane;
  const bool valid = n < w.n_spot;
  bool ok = false;
  uint64_t* dst;
  if (row < w.n_a) {
    dst = w.A + static_cast<size_t>(row) * w.Wp + word;
    if (valid && w.pods_left[n] >= 1) {
      ok = w.a_zero[row] || (w.free_cpu[n] >= w.a_cpu[row] && w.free_eph[n] >= w.a_eph[row]);
      ok = ok && static_ok(w, w.a_class[row], n);
    }
  } else {
    const int r = row - w.n_a;
    dst = w.B + static_cast<size_t>(r) * w.Wp + word;
    ok = valid && (w.b_all[r] || w.free_mem[n] >= w.b_mem[r]);
  }
  const uint64_t m = __ballot(ok);
  if (lane == 0) *dst = m;
}

// K1: one thread = 16 B of F (two words of one row).
__global__ __launch_bounds__(256) void k1_feasibility(const uint64_t* __restrict__ A, const uint64_t* __restrict__ B,
                                                      const int32_t* __restrict__ pod_a,
                                                      const int32_t* __restrict__ pod_b, uint64_t* __restrict__ F,
                                                      uint32_t n_pods, uint32_t half) {
  const uint32_t total = n_pods * half;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += stride) {
    const uint32_t p = i / half;
    const uint32_t j = i - p * half;
    const ulonglong2 a = reinterpret_cast<const ulonglong2*>(A)[static_cast<size_t>(pod_a[p]) * half + j];
    const ulonglong2 b = reinterpret_cast<const ulonglong2*>(B)[static_cast<size_t>(pod_b[p]) * half + j];
    ulonglong2 f;
    f.x = a.x & b.x;
    f.y = a.y & b.y;
    reinterpret_cast<ulonglong2*>(F)[i] = f;
  }
}

// K2: one wave per candidate.  SPL touched-node slots per lane (64*SPL per
// candidate), CH*64 bitmask words per row held as a register-resident
// touched mask (lane l owns words ch*64 + l).
template <int SPL, int CH>
__global__ __launch_bounds__(256) void k2_place(DevWorkload w, const int32_t* __restrict__ list, int n_list) {
  const int lane = threadIdx.x & 63;
  const int li = __builtin_amdgcn_readfirstlane(static_cast<int>(blockIdx.x) * 4 + static_cast<int>(threadIdx.x >> 6));
  if (li >= n_list) return;
  const int ci = __builtin_amdgcn_readfirstlane(list[li]);
  const int p0 = __builtin_amdgcn_readfirstlane(w.cand_off[ci]);
  const int p1 = __builtin_amdgcn_readfirstlane(w.cand_off[ci + 1]);
  const int Wp = w.Wp;
  const uint64_t* __restrict__ F = w.F;

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
  int status = -1;

  uint64_t next = lane < Wp ? F[static_cast<size_t>(p0) * Wp + lane] : 0;
  for (int p = p0; p < p1; ++p) {
    const uint64_t word0 = next;
    if (p + 1 < p1) next = lane < Wp ? F[static_cast<size_t>(p + 1) * Wp + lane] : 0;
    const int64_t rc = w.pod_cpu[p], rm = w.pod_mem[p], re = w.pod_eph[p];
    const int zero = w.pod_zero[p];
    const uint64_t pm = w.pod_ports[p];

    int ans = INT_MAX;
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) {
      const int base = ch * 64;
      if (ans != INT_MAX || base >= Wp) continue;  // wave-uniform; keeps the loop unrollable
      const uint64_t word =
          ch == 0 ? word0 : (base + lane < Wp ? F[static_cast<size_t>(p) * Wp + base + lane] : 0);
      // untouched base-feasible nodes are final: the lowest one is a candidate answer
      const uint64_t clean = word & ~touched[ch];
      const uint64_t mc = __ballot(clean != 0);
      int cnode = INT_MAX;
      if (mc) {
        const int L = __builtin_ctzll(mc);
        cnode = (base + L) * 64 + __builtin_ctzll(readlane64(clean, L));
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
      status = p - p0;
      break;
    }
    if (lane == 0) w.out_node[p] = ans;

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
      const int64_t fc = w.free_cpu[ans], fm = w.free_mem[ans], fe = w.free_eph[ans];
      const int pl = w.pods_left[ans];
      const uint64_t pb = w.port_bits[ans];
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
  }
  if (status >= 0)
    for (int q = p0 + status + lane; q < p1; q += kWave) w.out_node[q] = -1;
  if (lane == 0) {
    w.out_status[ci] = status;
    if (status < 0) atomicMin(&w.d_min[0], w.cand_global[ci]);
  }
}

__global__ __launch_bounds__(256) void k3_winner(DevWorkload w) {
  __shared__ int loc;
  const int g = w.d_min[0];
  int* r = w.result;
  if (threadIdx.x == 0) loc = -1;
  __syncthreads();
  if (g != INT_MAX)
    for (int i = threadIdx.x; i < w.n_cand; i += blockDim.x)
      if (w.cand_global[i] == g) loc = i;  // global indices are unique
  __syncthreads();
  const int ci = loc;
  const int np = ci >= 0 ? w.cand_off[ci + 1] - w.cand_off[ci] : 0;
  if (threadIdx.x == 0) {
    r[0] = g == INT_MAX ? -1 : g;
    r[1] = ci >= 0 ? 1 : 0;
    r[2] = np;
    r[3] = w.d_min[1] == INT_MAX ? -1 : w.d_min[1];
  }
  if (ci >= 0)
    for (int q = threadIdx.x; q < np; q += blockDim.x) r[4 + q] = w.out_node[w.cand_off[ci] + q];
}

template <int SPL>
hipError_t launch_k2_variant(const DevWorkload& w, const int32_t* list, int n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const dim3 grid((n + 3) / 4), block(256);
  const int chunks = (w.Wp + 63) / 64;
  if (chunks <= 1) hipLaunchKernelGGL((k2_place<SPL, 1>), grid, block, 0, s, w, list, n);
  else if (chunks <= 2) hipLaunchKernelGGL((k2_place<SPL, 2>), grid, block, 0, s, w, list, n);
  else if (chunks <= 4) hipLaunchKernelGGL((k2_place<SPL, 4>), grid, block, 0, s, w, list, n);
  else if (chunks <= 8) hipLaunchKernelGGL((k2_place<SPL, 8>), grid, block, 0, s, w, list, n);
  else if (chunks <= 16) hipLaunchKernelGGL((k2_place<SPL, 16>), grid, block, 0, s, w, list, n);
  else hipLaunchKernelGGL((k2_place<SPL, 32>), grid, block, 0, s, w, list, n);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_tables(const DevWorkload& w, int32_t local_first_fallback, hipStream_t s) {
  const int wblocks = (w.Wp + 3) / 4;
  const int rows = w.n_a + w.n_b;
  hipLaunchKernelGGL(k0_tables, dim3(static_cast<unsigned>(rows * wblocks)), dim3(256), 0, s, w, wblocks,
                     local_first_fallback);
  return hipGetLastError();
}

hipError_t launch_feasibility(const DevWorkload& w, hipStream_t s) {
  if (w.n_pods <= 0) return hipSuccess;
  const uint32_t half = static_cast<uint32_t>(w.Wp / 2);
  const uint64_t total = static_cast<uint64_t>(w.n_pods) * half;
  const uint64_t blocks = std::min<uint64_t>((total + 255) / 256, 256 * 32);
  hipLaunchKernelGGL(k1_feasibility, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, s, w.A, w.B, w.pod_a,
                     w.pod_b, w.F, static_cast<uint32_t>(w.n_pods), half);
  return hipGetLastError();
}

hipError_t launch_placement(const DevWorkload& w, hipStream_t s) {
  hipError_t e = launch_k2_variant<2>(w, w.list_small, w.n_small, s);
  if (e != hipSuccess) return e;
  return launch_k2_variant<8>(w, w.list_large, w.n_large, s);
}

hipError_t launch_winner(const DevWorkload& w, hipStream_t s) {
  hipLaunchKernelGGL(k3_winner, dim3(1), dim3(256), 0, s, w);
  return hipGetLastError();
}

}  // namespace sr
