// Microbenchmark (tools only, not the product): cycles per pod step of K2's
// window placement (kernels.hip place_window) in isolation, one wave alone on
// the chip, for variants of where the pod's values come from and how wide the
// running state is.  A step: the pod's request, the fit mask over the 64
// window nodes (lanes), the first fitting lane, the running-state update.
//   V0  64-bit state, the pod's values by v_readlane from the pod lanes (the
//       product's form)
//   V1  32-bit state and values (v_readlane)
//   V2  64-bit state, the pod's values broadcast from LDS into VGPRs
//   V3  32-bit state, values from LDS
//   V4  V0 without the state update (fit mask + first lane only)
//   V5  V0's update chain only (first lane taken from the pod index)
//   V6  the product's whole step (F word, pod-count, zero-request and pod
//       bookkeeping: place_window<false, false>)
//   V7  V6 with 32-bit state and values
//   V8  V6 with cpu / memory packed in one 64-bit word (31-bit fields, guard
//       bit 31): one subtract, one mask compare, one select per step
//   V9  V7 with the differences computed beside the compares (one select per
//       field after the first lane is known) and the pod's node without the fit test
//   V10 V7 pipelined: pod k's fit mask is taken against the state without
//       pod k-1's update, and the bit of the node pod k-1 took is redone on the
//       scalar unit (that update reaches the vector state one step later)
//   V12 V7 with the per-lane checks folded into one compare: d = min3(cpu -
//       c', memory - m', pods left - 1) >= 0 (c', m' = -2^30 for an all-zero
//       request; the ephemeral gate folded into the cpu state), so the fit mask
//       is one ballot and the F word (no scalar select chain)
//   V13 V7 with the node and placed bookkeeping moved out of the step: the
//       first lane j is selected into pod k's lane of a VGPR, the
//       visit derives node / placed from it once
//   V11 V7 two pods per step (place_window32_pairs): pod b's mask against the
//       state before pod a and against it minus a, side by side (reported per pod)
// Build: hipcc -O3 --offload-arch=gfx950 -o place_chain place_chain.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }
__device__ __forceinline__ uint64_t readlane64(uint64_t v, int lane) {
  const uint32_t lo = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v & 0xffffffffu), lane));
  const uint32_t hi = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(v >> 32), lane));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

constexpr int kSteps = 4096;

template <int V>
__global__ __launch_bounds__(64) void k_chain(const int64_t* reqs, const int64_t* frees, uint64_t* out) {
  __shared__ int64_t lreq[2][64];
  const int lane = threadIdx.x;
  const int64_t rc = reqs[lane], rm = reqs[64 + lane];
  lreq[0][lane] = rc;
  lreq[1][lane] = rm;
  __syncthreads();
  int64_t ncpu = frees[lane], nmem = frees[64 + lane];
  uint32_t c32 = static_cast<uint32_t>(ncpu), m32 = static_cast<uint32_t>(nmem);
  const uint32_t rc32 = static_cast<uint32_t>(rc), rm32 = static_cast<uint32_t>(rm);
  uint64_t acc = 0, placed = 0;
  const uint64_t curw = ~0ull >> (lane & 7), zm = 0x1000100010001ull, emask = ballot(ncpu > 0);
  int nleft = 1000000 + lane, node = -1;
  uint64_t pk = (static_cast<uint64_t>(c32 & 0x3fffffffu) << 32) | 0x80000000ull | (m32 & 0x3fffffffu);
  const uint64_t rq = (static_cast<uint64_t>(rc32 & 0xffffu) << 32) | (rm32 >> 20);
  int32_t sc32 = static_cast<int32_t>(c32 & 0x3fffffff), sm32 = static_cast<int32_t>(m32 & 0x3fffffff), sleft = nleft;
  int pj = 64, qj = 64, jv = 64;
  const bool zr = (zm >> lane) & 1;
  const int32_t cq = zr ? -(1 << 30) : static_cast<int32_t>(rc32), mq = zr ? -(1 << 30) : static_cast<int32_t>(rm32);
  if constexpr (V == 12) {
    sc32 = ((emask >> lane) & 1) ? sc32 : -1;
    sleft -= 1;
  }
  int32_t pc = 0, pm_ = 0, qc = 0, qm = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int s = 0; s < kSteps; ++s) {
    const int k = __builtin_amdgcn_readfirstlane(s & 63);
    uint64_t fit;
    if constexpr (V == 0 || V == 4 || V == 5) {
      const int64_t c = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rc), k));
      const int64_t m = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rm), k));
      fit = V == 5 ? (1ull << k) : (ballot(ncpu >= c) & ballot(nmem >= m));
      if constexpr (V != 4) {
        const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
        const bool hit = lane == j;
        ncpu -= hit ? c : 0;
        nmem -= hit ? m : 0;
      }
    } else if constexpr (V == 1) {
      const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rc32), k));
      const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rm32), k));
      fit = ballot(c32 >= c) & ballot(m32 >= m);
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      c32 -= hit ? c : 0u;
      m32 -= hit ? m : 0u;
    } else if constexpr (V == 2) {
      const int64_t c = lreq[0][k], m = lreq[1][k];
      fit = ballot(ncpu >= c) & ballot(nmem >= m);
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      ncpu -= hit ? c : 0;
      nmem -= hit ? m : 0;
    } else if constexpr (V == 6) {
      const int64_t c = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rc), k));
      const int64_t m = static_cast<int64_t>(readlane64(static_cast<uint64_t>(rm), k));
      fit = readlane64(curw, k) & ballot(nleft >= 1);
      const uint64_t res = ballot(ncpu >= c) & ballot(nmem >= m) & emask;
      fit &= ((zm >> k) & 1) ? ~0ull : res;
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      ncpu -= hit ? c : 0;
      nmem -= hit ? m : 0;
      nleft -= hit ? 1 : 0;
      node = (lane == k && j < 64) ? 64 * 3 + j : node;
      placed |= fit != 0 ? 1ull << k : 0ull;
    } else if constexpr (V == 7) {
      const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rc32), k));
      const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rm32), k));
      fit = readlane64(curw, k) & ballot(nleft >= 1);
      const uint64_t res = ballot(c32 >= c) & ballot(m32 >= m) & emask;
      fit &= ((zm >> k) & 1) ? ~0ull : res;
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      c32 -= hit ? c : 0u;
      m32 -= hit ? m : 0u;
      nleft -= hit ? 1 : 0;
      node = (lane == k && j < 64) ? 64 * 3 + j : node;
      placed |= fit != 0 ? 1ull << k : 0ull;
    } else if constexpr (V == 8) {
      const uint64_t r = readlane64(rq, k);
      fit = readlane64(curw, k) & ballot(nleft >= 1);
      const uint64_t d = pk - r;
      const uint64_t res = ballot((d & 0x8000000080000000ull) == 0x80000000ull) & emask;
      fit &= ((zm >> k) & 1) ? ~0ull : res;
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      pk = hit ? d : pk;
      nleft -= hit ? 1 : 0;
      node = (lane == k && j < 64) ? 64 * 3 + j : node;
      placed |= fit != 0 ? 1ull << k : 0ull;
    } else if constexpr (V == 9) {
      const uint32_t c = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rc32), k));
      const uint32_t m = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(rm32), k));
      const uint32_t dc = c32 - c, dm = m32 - m;
      const int dl = nleft - 1;
      fit = readlane64(curw, k) & ballot(nleft >= 1);
      const uint64_t res = ballot(c32 >= c) & ballot(m32 >= m) & emask;
      fit &= ((zm >> k) & 1) ? ~0ull : res;
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      c32 = hit ? dc : c32;
      m32 = hit ? dm : m32;
      nleft = hit ? dl : nleft;
      node = lane == k ? 64 * 3 + j : node;
      placed |= fit != 0 ? 1ull << k : 0ull;
    } else if constexpr (V == 10) {
      const int32_t c = __builtin_amdgcn_readlane(static_cast<int>(rc32), k);
      const int32_t m = __builtin_amdgcn_readlane(static_cast<int>(rm32), k);
      // the update of the pod before last reaches the vector state
      const bool hp = lane == pj;
      sc32 -= hp ? pc : 0;
      sm32 -= hp ? pm_ : 0;
      sleft -= hp ? 1 : 0;
      // this pod against it (the last pod's node pj is redone below)
      uint64_t v = ballot(sleft >= 1) & ballot(sc32 >= c) & ballot(sm32 >= m);
      const bool zero = (zm >> k) & 1;
      if (zero) v = ballot(sleft >= 1);
      if (qj < 64) {
        const int32_t tc = __builtin_amdgcn_readlane(sc32, qj) - qc;
        const int32_t tm = __builtin_amdgcn_readlane(sm32, qj) - qm;
        const int32_t tl = __builtin_amdgcn_readlane(sleft, qj) - 1;
        const bool ok = tl >= 1 && (zero || (tc >= c && tm >= m));
        v = ok ? (v | (1ull << qj)) : (v & ~(1ull << qj));
      }
      fit = readlane64(curw, k) & v & (zero ? ~0ull : emask);
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      node = lane == k ? 64 * 3 + j : node;
      placed |= fit != 0 ? 1ull << k : 0ull;
      // pending: pod k-1's update moves to the "before last" slot, pod k's becomes pending
      pj = qj; pc = qc; pm_ = qm;
      qj = j; qc = c; qm = m;
    } else if constexpr (V == 11) {
      const int a = __builtin_amdgcn_readfirstlane((2 * s) & 63), b = a + 1;
      const int32_t ca = __builtin_amdgcn_readlane(static_cast<int>(rc32), a);
      const int32_t ma = __builtin_amdgcn_readlane(static_cast<int>(rm32), a);
      const int32_t cb = __builtin_amdgcn_readlane(static_cast<int>(rc32), b);
      const int32_t mb = __builtin_amdgcn_readlane(static_cast<int>(rm32), b);
      const uint64_t za = 0ull - ((zm >> a) & 1), zb = 0ull - ((zm >> b) & 1);
      const int32_t i32 = static_cast<int32_t>(c32), j32 = static_cast<int32_t>(m32);
      const uint64_t l1 = ballot(nleft >= 1);
      const uint64_t fa = readlane64(curw, a) & l1 & ((ballot(i32 >= ca) & ballot(j32 >= ma) & emask) | za);
      const uint64_t fwb = readlane64(curw, b);
      const uint64_t fold = fwb & l1 & ((ballot(i32 >= cb) & ballot(j32 >= mb) & emask) | zb);
      const uint64_t fnew =
          fwb & ballot(nleft >= 2) & ((ballot(i32 >= ca + cb) & ballot(j32 >= ma + mb) & emask) | zb);
      const int ja = fa != 0 ? __builtin_ctzll(fa) : 64;
      const uint64_t bit = ja < 64 ? 1ull << ja : 0ull;
      const uint64_t fb = (fold & ~bit) | (fnew & bit);
      const int jb = fb != 0 ? __builtin_ctzll(fb) : 64;
      const bool ha = lane == ja, hb = lane == jb;
      c32 -= (ha ? ca : 0) + (hb ? cb : 0);
      m32 -= (ha ? ma : 0) + (hb ? mb : 0);
      nleft -= (ha ? 1 : 0) + (hb ? 1 : 0);
      node = (lane == a && ja < 64) ? 64 * 3 + ja : node;
      node = (lane == b && jb < 64) ? 64 * 3 + jb : node;
      placed |= (fa != 0 ? 1ull << a : 0ull) | (fb != 0 ? 1ull << b : 0ull);
      fit = fa ^ fb;
    } else if constexpr (V == 12) {
      const int32_t c = __builtin_amdgcn_readlane(static_cast<int>(cq), k);
      const int32_t m = __builtin_amdgcn_readlane(static_cast<int>(mq), k);
      const int32_t cu = __builtin_amdgcn_readlane(static_cast<int>(rc32), k);
      const int32_t mu = __builtin_amdgcn_readlane(static_cast<int>(rm32), k);
      const int32_t d = min(min(sc32 - c, sm32 - m), sleft);
      fit = readlane64(curw, k) & ballot(d >= 0);
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      sc32 -= hit ? cu : 0;
      sm32 -= hit ? mu : 0;
      sleft -= hit ? 1 : 0;
      node = (lane == k && j < 64) ? 64 * 3 + j : node;
      placed |= fit != 0 ? 1ull << k : 0ull;
    } else if constexpr (V == 13) {
      const int32_t c = __builtin_amdgcn_readlane(static_cast<int>(rc32), k);
      const int32_t m = __builtin_amdgcn_readlane(static_cast<int>(rm32), k);
      const int32_t i32 = static_cast<int32_t>(c32), j32 = static_cast<int32_t>(m32);
      fit = readlane64(curw, k) & ballot(nleft >= 1);
      const uint64_t res = ballot(i32 >= c) & ballot(j32 >= m) & emask;
      fit &= ((zm >> k) & 1) ? ~0ull : res;
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      c32 -= hit ? c : 0u;
      m32 -= hit ? m : 0u;
      nleft -= hit ? 1 : 0;
      jv = lane == k ? j : jv;
    } else {
      const uint32_t c = static_cast<uint32_t>(lreq[0][k]), m = static_cast<uint32_t>(lreq[1][k]);
      fit = ballot(c32 >= c) & ballot(m32 >= m);
      const int j = fit != 0 ? __builtin_ctzll(fit) : 64;
      const bool hit = lane == j;
      c32 -= hit ? c : 0u;
      m32 -= hit ? m : 0u;
    }
    acc += fit;
  }
  if constexpr (V == 13) {
    placed = ballot(jv < 64);
    node = jv < 64 ? 64 * 3 + jv : node;
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    out[0] = t1 - t0;
    out[1] = acc;
  }
  out[2 + lane] = static_cast<uint64_t>(ncpu + nmem) + c32 + m32 + nleft + node + placed + pk + sc32 + sm32 + sleft + pj;
}

template <int V>
int run(const int64_t* dreq, const int64_t* dfree, uint64_t* dout, const char* name, int pods_per_step = 1) {
  std::vector<double> cyc;
  for (int r = 0; r < 21; ++r) {
    hipLaunchKernelGGL(k_chain<V>, dim3(1), dim3(64), 0, 0, dreq, dfree, dout);
    CK(hipDeviceSynchronize());
    uint64_t h[2];
    CK(hipMemcpy(h, dout, sizeof(h), hipMemcpyDeviceToHost));
    cyc.push_back(static_cast<double>(h[0]) / kSteps / pods_per_step);
  }
  std::sort(cyc.begin(), cyc.end());
  printf("%-58s %7.1f cycles/pod (median of 21)\n", name, cyc[10]);
  return 0;
}

int main() {
  std::vector<int64_t> req(128), fr(128);
  for (int i = 0; i < 64; ++i) {
    req[i] = 50 + (i * 37) % 200;             // milli-cpu
    req[64 + i] = (64 + (i * 53) % 512) << 20; // memory
    fr[i] = 4000000000ll + i;                  // plenty: every pod fits on lane 0 or near it
    fr[64 + i] = (1ll << 40) + i;
  }
  int64_t *dreq, *dfree;
  uint64_t* dout;
  CK(hipMalloc(&dreq, 128 * 8));
  CK(hipMalloc(&dfree, 128 * 8));
  CK(hipMalloc(&dout, 66 * 8));
  CK(hipMemcpy(dreq, req.data(), 128 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dfree, fr.data(), 128 * 8, hipMemcpyHostToDevice));
  run<0>(dreq, dfree, dout, "V0 64-bit state, values by v_readlane (product)");
  run<1>(dreq, dfree, dout, "V1 32-bit state, values by v_readlane");
  run<2>(dreq, dfree, dout, "V2 64-bit state, values from LDS");
  run<3>(dreq, dfree, dout, "V3 32-bit state, values from LDS");
  run<4>(dreq, dfree, dout, "V4 V0 fit mask + first lane only (no update)");
  run<5>(dreq, dfree, dout, "V5 V0 update chain only");
  run<6>(dreq, dfree, dout, "V6 product step (place_window<false, false>)");
  run<7>(dreq, dfree, dout, "V7 V6 with 32-bit state and values");
  run<8>(dreq, dfree, dout, "V8 V6 with cpu/memory packed in one word");
  run<9>(dreq, dfree, dout, "V9 V7, selects after the first lane, node unconditional");
  run<10>(dreq, dfree, dout, "V10 V7 pipelined (last pod's node redone on SALU)");
  run<11>(dreq, dfree, dout, "V11 V7 two pods per step", 2);
  run<12>(dreq, dfree, dout, "V12 V7 with the checks folded into one min3 compare");
  run<13>(dreq, dfree, dout, "V13 V7, node / placed once per visit");
  return 0;
}
