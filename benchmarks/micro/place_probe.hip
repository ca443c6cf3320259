// Cost of the tiny server's all-wave "place" load burst (docs/DESIGN.md §2.1):
// W waves of one workgroup each issue K scattered 16-byte loads per lane into
// an L2-resident buffer (the packed adjacency of the 100k bench graph is
// ~2.6 MB), then the workgroup meets at a barrier.  Printed: cycles from the
// first issue to the barrier, per variant, median of 64 repetitions, with a
// fraction of the lanes masked off (a lane with no load: the back edge to a
// record's parent).  Tells whether the burst is bound by the number of lines
// the CU's address unit walks (cycles ~ lines) or by one load latency.
//
//   make micro && build/bin/place_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef unsigned long long u64x2 __attribute__((ext_vector_type(2), aligned(8)));

constexpr int kReps = 64;

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// K loads per lane (1 or 2, 16 B each: the X4 form's two halves), active
// lanes: lane % 10 < act10.  Lane addresses: a hash into `words` 8-byte words.
template <int K>
__global__ __launch_bounds__(1024) void k_place(const unsigned long long* __restrict__ adj, uint32_t words,
                                                uint32_t act10, unsigned long long* out, unsigned long long* sink) {
  const uint32_t tid = threadIdx.x, lane = tid & 63;
  unsigned long long acc = 0;
  for (int r = 0; r < kReps + 4; ++r) {
    __syncthreads();
    const unsigned long long t0 = clk();
    const uint32_t h = (tid * 2654435761u + (uint32_t)r * 40503u) % (words - 8);
    const uint32_t p = h & ~1u;
    if (lane % 10 < act10) {
      const u64x2 a = *reinterpret_cast<const u64x2*>(adj + p);
      acc += a.x ^ a.y;
      if (K == 2) {
        const u64x2 b = *reinterpret_cast<const u64x2*>(adj + p + 2);
        acc += b.x ^ b.y;
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const unsigned long long t1 = clk();
    if (tid == 0 && r >= 4) out[r - 4] = t1 - t0;
  }
  if (acc == 0x1234567) sink[tid] = acc;
}

int main() {
  const uint32_t words = (2600000 / 8) & ~15u;  // ~2.6 MB
  unsigned long long *adj, *out, *sink;
  CK(hipMalloc(&adj, (size_t)words * 8));
  CK(hipMalloc(&out, kReps * 8));
  CK(hipMalloc(&sink, 1024 * 8));
  std::vector<unsigned long long> h(words);
  for (uint32_t i = 0; i < words; ++i) h[i] = i * 0x9e3779b97f4a7c15ull;
  CK(hipMemcpy(adj, h.data(), (size_t)words * 8, hipMemcpyHostToDevice));
  std::printf("threads K act%% lines cycles(median) cycles/line\n");
  for (int threads : {64, 128, 256, 512, 1024})
    for (int k : {1, 2})
      for (uint32_t act : {10u, 7u}) {
        if (k == 1) k_place<1><<<1, threads>>>(adj, words, act, out, sink);
        else k_place<2><<<1, threads>>>(adj, words, act, out, sink);
        CK(hipGetLastError());
        CK(hipDeviceSynchronize());
        std::vector<unsigned long long> o(kReps);
        CK(hipMemcpy(o.data(), out, kReps * 8, hipMemcpyDeviceToHost));
        std::sort(o.begin(), o.end());
        const double lines = threads * k * (act / 10.0);
        std::printf("%5d %d %3u %6.0f %7llu %6.2f\n", threads, k, act * 10, lines, o[kReps / 2],
                    o[kReps / 2] / lines);
      }
  return 0;
}
