// dep_load.hip — latency of one dependent global load on gfx950, the unit of
// K2's chain floor (bench.py roofline.latency): a single wave chases pointers
// through a buffer, each address taken from the previous load's value, and
// times the chain with s_memtime.
//   warm_kernel: every wave of a full grid reads the buffer (it lands in the
//     MALL and the readers' L2s, as the previous tick's K2 leaves the tables);
//   chase_kernel (a new launch): the first pass over the buffer = a load that
//     misses the L2 the kernel boundary invalidated; the second pass over the
//     same lines = an L2 hit.
// Build: hipcc -O3 --offload-arch=gfx950 -o dep_load dep_load.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdint>
#include <numeric>
#include <random>
#include <vector>

constexpr int kSteps = 512;  // dependent loads per pass (one cache line each, 128 B apart or more)

__global__ void warm_kernel(const uint64_t* buf, size_t n, uint64_t* sink) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += static_cast<size_t>(gridDim.x) * blockDim.x)
    acc += buf[i];
  if (acc == 0x12345) sink[0] = acc;
}

// Vector loads, one word per lane (as K2's record and row loads): every word
// of a step's 64 holds the next step's offset.
__global__ void chase_kernel(const uint64_t* buf, uint64_t start, uint64_t* out) {
  const uint64_t lane = threadIdx.x & 63;
  uint64_t p = start;
  uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kSteps; ++i) p = buf[p + lane];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint64_t t1 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < kSteps; ++i) p = buf[p + lane];  // the same lines again: L2 hits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint64_t t2 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) {
    out[0] = t1 - t0;
    out[1] = t2 - t1;
    out[2] = p;
  }
}

int main() {
  const size_t n = size_t(1) << 22;  // 32 MB: beyond one XCD's L2, within the MALL
  std::vector<uint64_t> h(n, 0);
  // a random cycle over kSteps 512-B steps 4 KB apart
  std::vector<uint64_t> idx(kSteps);
  std::iota(idx.begin(), idx.end(), 0);
  std::shuffle(idx.begin() + 1, idx.end(), std::mt19937_64(7));
  for (int i = 0; i < kSteps; ++i)
    for (int l = 0; l < 64; ++l) h[idx[i] * 512 + l] = idx[(i + 1) % kSteps] * 512;
  uint64_t *d, *out, *sink;
  (void)hipMalloc(&d, n * 8);
  (void)hipMalloc(&out, 64);
  (void)hipMalloc(&sink, 64);
  (void)hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice);
  std::vector<double> cold, warm;
  for (int r = 0; r < 21; ++r) {
    warm_kernel<<<4096, 256>>>(d, n, sink);
    chase_kernel<<<1, 64>>>(d, 0, out);
    uint64_t o[3];
    (void)hipMemcpy(o, out, 24, hipMemcpyDeviceToHost);
    cold.push_back(double(o[0]) / kSteps);
    warm.push_back(double(o[1]) / kSteps);
  }
  std::sort(cold.begin(), cold.end());
  std::sort(warm.begin(), warm.end());
  printf("dependent load, first touch in a new kernel (MALL / HBM): %.0f cycles (median of 21)\n", cold[10]);
  printf("dependent load, L2 hit: %.0f cycles (median of 21)\n", warm[10]);
  return 0;
}
