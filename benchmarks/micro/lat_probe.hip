// Latency probes for the single-workgroup search engine's inner loop
// (docs/DESIGN.md §2).  One workgroup; s_memtime (shader clock) around
// dependent chains of the operations a BFS level is made of.  Prints cycles
// per operation.  Build: make micro  (hipcc --offload-arch=gfx950).
#include <hip/hip_runtime.h>

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

constexpr int kIters = 256;
constexpr int kSlots = 8192;

__device__ __forceinline__ unsigned long long clk() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// out[k] = cycles per op of probe k (measured by lane 0 of wave 0)
__global__ __launch_bounds__(128) void k_probe(const uint32_t* __restrict__ gnext, uint32_t gmask,
                                               uint32_t* gstore, unsigned long long* out) {
  __shared__ uint32_t L[kSlots];
  __shared__ uint4 L4[kSlots / 4];
  __shared__ uint32_t flag;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int i = tid; i < kSlots; i += blockDim.x) L[i] = (uint32_t)((i * 2654435761u + 17) % kSlots);
  for (int i = tid; i < kSlots / 4; i += blockDim.x) L4[i] = make_uint4((i * 7 + 3) % (kSlots / 4), 0, 0, 0);
  if (tid == 0) flag = 0;
  __syncthreads();
  if (wid == 0) {
    uint32_t x = lane * 97 % kSlots;
    unsigned long long t0, t1;
    // 0: dependent ds_read_b32
    t0 = clk();
    for (int i = 0; i < kIters; ++i) x = L[x];
    asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(x));
    t1 = clk();
    if (lane == 0) out[0] = (t1 - t0) / kIters;
    // 1: dependent ds_read_b128
    uint32_t y = lane * 13 % (kSlots / 4);
    t0 = clk();
    for (int i = 0; i < kIters; ++i) y = L4[y].x;
    asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(y));
    t1 = clk();
    if (lane == 0) out[1] = (t1 - t0) / kIters;
    // 2: dependent ds_cmpst_rtn_b32 (fails: compares against a value never stored)
    x = lane * 31 % kSlots;
    t0 = clk();
    for (int i = 0; i < kIters; ++i) x = atomicCAS(&L[x], 0xfffffffeu, 0xfffffffdu) % kSlots;
    asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(x));
    t1 = clk();
    if (lane == 0) out[2] = (t1 - t0) / kIters;
    // 3: dependent ds_or_rtn_b32 (or 0: values unchanged)
    x = lane * 29 % kSlots;
    t0 = clk();
    for (int i = 0; i < kIters; ++i) x = atomicOr(&L[x], 0u) % kSlots;
    asm volatile("s_waitcnt lgkmcnt(0)" ::"v"(x));
    t1 = clk();
    if (lane == 0) out[3] = (t1 - t0) / kIters;
    // 4: dependent global load, scattered lanes (warm pass first)
    uint32_t g = (lane * 40503u) & gmask;
    for (int i = 0; i < kIters; ++i) g = gnext[g];
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(g));
    g = (lane * 40503u) & gmask;
    t0 = clk();
    for (int i = 0; i < kIters; ++i) g = gnext[g];
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(g));
    t1 = clk();
    if (lane == 0) out[4] = (t1 - t0) / kIters;
    // 5: dependent global load, all lanes same address (one line)
    uint32_t h = 0;
    t0 = clk();
    for (int i = 0; i < kIters; ++i) h = gnext[h & 0] + (h & 0);
    asm volatile("s_waitcnt vmcnt(0)" ::"v"(h));
    t1 = clk();
    if (lane == 0) out[5] = (t1 - t0) / kIters;
    // 6: issue cost of a scattered global store (no wait), 8 stores
    t0 = clk();
#pragma unroll
    for (int i = 0; i < 8; ++i) gstore[((lane * 4099u + i * 131071u) * 16) & gmask] = (uint32_t)i + g;
    t1 = clk();
    if (lane == 0) out[6] = (t1 - t0) / 8;
    // 7: drain of those stores
    t0 = clk();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    t1 = clk();
    if (lane == 0) out[7] = t1 - t0;
    // 8: store + vmcnt(0), dependent
    t0 = clk();
    for (int i = 0; i < 32; ++i) {
      gstore[((lane * 4099u + i * 7919u) * 16) & gmask] = (uint32_t)i;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    t1 = clk();
    if (lane == 0) out[8] = (t1 - t0) / 32;
    // 9: wave ballot + readlane + DPP-free prefix (mbcnt) in a loop
    unsigned long long acc = 0;
    t0 = clk();
    for (int i = 0; i < kIters; ++i) {
      unsigned long long m = __ballot((x + i) & 1);
      acc += __builtin_amdgcn_readfirstlane((uint32_t)m) + __popcll(m);
    }
    t1 = clk();
    if (lane == 0) out[9] = (t1 - t0) / kIters + (acc == 12345 ? 1 : 0);
    // 10: two-wave LDS ping-pong (round trip via flag), measured on wave 0
    t0 = clk();
    for (int r = 0; r < 64; ++r) {
      if (lane == 0) __hip_atomic_store(&flag, 2 * r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 2u * r + 2)
        __builtin_amdgcn_s_sleep(0);
    }
    t1 = clk();
    if (lane == 0) out[10] = (t1 - t0) / 64;
    // 11: same without s_sleep
    t0 = clk();
    for (int r = 64; r < 128; ++r) {
      if (lane == 0) __hip_atomic_store(&flag, 2 * r + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      while (__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 2u * r + 2) {
      }
    }
    t1 = clk();
    if (lane == 0) out[11] = (t1 - t0) / 64;
    // 12: __syncthreads-free: s_memtime overhead
    t0 = clk();
    t1 = clk();
    if (lane == 0) out[12] = t1 - t0;
  } else {
    // wave 1: echo the ping-pong
    for (int r = 0; r < 64; ++r) {
      while (__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 2u * r + 1)
        __builtin_amdgcn_s_sleep(0);
      if (lane == 0) __hip_atomic_store(&flag, 2 * r + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    for (int r = 64; r < 128; ++r) {
      while (__hip_atomic_load(&flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != 2u * r + 1) {
      }
      if (lane == 0) __hip_atomic_store(&flag, 2 * r + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
}

int main(int argc, char** argv) {
  const uint32_t mb = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 1;  // global working set, MiB (power of 2)
  const uint32_t n = mb * (1u << 20) / 4, mask = n - 1;
  std::vector<uint32_t> h(n);
  uint64_t s = 88172645463325252ull;
  for (uint32_t i = 0; i < n; ++i) {
    s ^= s << 13, s ^= s >> 7, s ^= s << 17;
    h[i] = (uint32_t)s & mask;
  }
  uint32_t *dn, *ds;
  unsigned long long* dout;
  CK(hipMalloc(&dn, n * 4));
  CK(hipMalloc(&ds, n * 4));
  CK(hipMalloc(&dout, 32 * 8));
  CK(hipMemcpy(dn, h.data(), n * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dout, 0, 32 * 8));
  for (int rep = 0; rep < 3; ++rep) k_probe<<<1, 128>>>(dn, mask, ds, dout);
  CK(hipDeviceSynchronize());
  unsigned long long o[32];
  CK(hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost));
  const char* names[] = {"ds_read_b32 (dependent)", "ds_read_b128 (dependent)", "ds_cmpst_rtn_b32 (dependent)",
                         "ds_or_rtn_b32 (dependent)", "global load scattered (dependent)",
                         "global load one line (dependent)", "scattered global store issue",
                         "drain 8 scattered stores (vmcnt0)", "store + vmcnt(0) round trip",
                         "ballot+readfirstlane+popc", "2-wave LDS ping-pong w/ s_sleep0 (round trip)",
                         "2-wave LDS ping-pong spin (round trip)", "s_memtime back-to-back"};
  std::printf("working set %u MiB\n", mb);
  for (int k = 0; k < 13; ++k) std::printf("%-48s %6llu cycles\n", names[k], o[k]);
  return 0;
}
