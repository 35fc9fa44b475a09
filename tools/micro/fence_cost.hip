// Microbenchmark (tools only, not the product): what a K0 -> K2 dependency
// costs inside one kernel versus across a kernel boundary on gfx950.
//   A: producer kernel (P blocks x 4 waves, each writing `bytes/P` of rows),
//      then a consumer kernel (C waves, each reading 8 words of the rows).
//   B: one kernel: producer blocks [0, P) store, __syncthreads, one agent
//      release fence + atomic add per block; consumer blocks poll the counter
//      (bounded), acquire, read.
//   C: as B, but the producer stores are nontemporal.
// Times are hipEvent pairs around each variant, medians of 200 runs.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int kWordsPerProducerWave = 56;  // one S row per wave (C3: Wp = 56)

__device__ __forceinline__ void produce(uint64_t* rows, int wave_id, bool nt) {
  const int lane = threadIdx.x & 63;
  if (lane < kWordsPerProducerWave) {
    uint64_t v = 0x9e3779b97f4a7c15ull * (wave_id + 1) ^ lane;
    uint64_t* p = rows + static_cast<size_t>(wave_id) * kWordsPerProducerWave + lane;
    if (nt) __builtin_nontemporal_store(v, p);
    else *p = v;
  }
}

__device__ __forceinline__ uint64_t consume(const uint64_t* rows, int nrows, int wave_id) {
  const int lane = threadIdx.x & 63;
  // 8 pods x 8 words of rows scattered like F heads
  const int r = (wave_id * 37 + (lane >> 3) * 101) % nrows;
  return rows[static_cast<size_t>(r) * kWordsPerProducerWave + (lane & 7)];
}

__global__ __launch_bounds__(256) void k_prod(uint64_t* rows) {
  produce(rows, blockIdx.x * 4 + (threadIdx.x >> 6), false);
}
__global__ __launch_bounds__(256) void k_cons(const uint64_t* rows, int nrows, uint64_t* out) {
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t x = consume(rows, nrows, wid);
  if (x == 0x1234) out[wid] = x;  // keep the load
}
// mode bits: 1 = per-block release fence, 2 = per-wave acquire, 4 = nontemporal
// stores, 8 = one elected write-back per XCD (consumers) instead of per block
__global__ __launch_bounds__(256) void k_fused(uint64_t* rows, int nrows, int P, unsigned* cnt, unsigned target,
                                               uint64_t* out, int mode) {
  if (static_cast<int>(blockIdx.x) < P) {
    produce(rows, blockIdx.x * 4 + (threadIdx.x >> 6), (mode & 4) != 0);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (mode & 1) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      else __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7;  // HW_REG_XCC_ID
      __hip_atomic_fetch_or(cnt + 9, 1u << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int wid = (blockIdx.x - P) * 4 + (threadIdx.x >> 6);
  unsigned spins = 0;
  while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target && ++spins < (1u << 16))
    __builtin_amdgcn_s_sleep(1);
  if (mode & 8) {
    unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 7;  // HW_REG_XCC_ID[3:0]
    unsigned* tick = cnt + 16 + xcc;
    unsigned* done = cnt + 8;
    if (__hip_atomic_fetch_add(tick, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_or(done, 1u << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned need = __hip_atomic_load(cnt + 9, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    while ((__hip_atomic_load(done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & need) != need && ++spins < (1u << 16))
      __builtin_amdgcn_s_sleep(1);
  }
  if (mode & 2) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  const uint64_t x = consume(rows, nrows, wid);
  if (x == 0x1234 || spins >= (1u << 16)) out[wid] = x | (1ull << 63);
}

int main() {
  const int P = 393 * 4 / 4;   // producer blocks (C3: ~1572 S waves + 308 T waves ~ 470 blocks)
  const int Pw = 470;
  const int C = 1500;          // consumer waves
  const int nrows = Pw * 4;
  uint64_t *rows, *out;
  unsigned* cnt;
  CK(hipMalloc(&rows, sizeof(uint64_t) * nrows * kWordsPerProducerWave));
  CK(hipMalloc(&out, sizeof(uint64_t) * 8192));
  CK(hipMalloc(&cnt, 256));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  (void)P;
  auto med = [](std::vector<float>& v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
  const int modes[] = {-1, 3, 1, 2, 0, 10, 8};
  const char* names[] = {"two kernels", "fused: release per block + acquire per wave", "fused: release per block only",
                         "fused: acquire per wave only", "fused: no fences (counter only)",
                         "fused: one write-back per XCD + acquire per wave", "fused: one write-back per XCD"};
  for (int vi = 0; vi < 7; ++vi) {
    std::vector<float> t;
    int bad = 0;
    for (int it = 0; it < 120; ++it) {
      CK(hipMemsetAsync(cnt, 0, 256, s));
      CK(hipEventRecord(a, s));
      if (modes[vi] < 0) {
        hipLaunchKernelGGL(k_prod, dim3(Pw), dim3(256), 0, s, rows);
        hipLaunchKernelGGL(k_cons, dim3((C + 3) / 4), dim3(256), 0, s, rows, nrows, out);
      } else {
        hipLaunchKernelGGL(k_fused, dim3(Pw + (C + 3) / 4), dim3(256), 0, s, rows, nrows, Pw, cnt, (unsigned)Pw, out,
                           modes[vi]);
      }
      CK(hipEventRecord(b, s));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (it >= 20) t.push_back(ms * 1000.0f);
    }
    (void)bad;
    printf("%-50s median %.2f us\n", names[vi], med(t));
    fflush(stdout);
  }
  // the cost of the fence alone: fused with target 0 (consumers never wait)
  std::vector<float> t;
  for (int it = 0; it < 220; ++it) {
    CK(hipEventRecord(a, s));
    hipLaunchKernelGGL(k_prod, dim3(Pw), dim3(256), 0, s, rows);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    if (it >= 20) t.push_back(ms * 1000.0f);
  }
  printf("producer kernel alone: median %.2f us\n", med(t));
  return 0;
}
