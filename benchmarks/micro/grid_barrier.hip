// Persistent multi-workgroup grid levels vs one launch per level (VERDICT r5
// item 4; docs/DESIGN.md §3).  A grid level of the 10M hand-off searches is a
// few thousand claims spread over the chip; between two levels the engine
// today pays a kernel boundary (device-gated levels) or a host round trip
// (host-planned levels).  A persistent loop would pay a grid barrier instead.
//
// Measured here, per level, G workgroups of 256 threads:
//   persist   one launch, `levels` levels, each = `work` claim atomics per
//             thread (atomicOr on a 10M-bit bitmap, agent scope) + an
//             XCD-hierarchical grid barrier (per-XCD arrival counter, the XCD's
//             last arriver releases and adds to a top counter, the last XCD
//             writes the generation; every workgroup polls it relaxed, then
//             acquires) -- the MI355X_MICROARCH.md "barrier-xcd" shape
//   launches  the same level as its own launch, back to back on one stream
//             (hipEvent wall time / levels): the kernel-boundary alternative
// Every spin is bounded (a timeout flag ends the kernel), and the grid is at
// most one workgroup per CU, so every workgroup is resident.
//
//   make micro && build/bin/grid_barrier
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

constexpr uint32_t kBits = 10000000u;
constexpr unsigned long long kSpinCap = 400000000ull;  // s_memrealtime ticks (100 MHz): 4 s

struct Sync {
  unsigned census[8 * 32];  // per XCD, one 128-byte line each
  unsigned xarrive[8 * 32];
  unsigned top[32];
  unsigned gen[32];
  unsigned start[32];
  unsigned timeout[32];
};

__device__ __forceinline__ unsigned xcc_id() {
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 7u;
}
__device__ __forceinline__ unsigned ld(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// one level's work: `work` claims per thread at hashed bit positions
__device__ __forceinline__ unsigned level_work(unsigned* bm, unsigned level, unsigned work) {
  unsigned acc = 0;
  const unsigned t = blockIdx.x * blockDim.x + threadIdx.x;
  for (unsigned k = 0; k < work; ++k) {
    const unsigned b = ((t * 2654435761u) ^ (level * 40503u + k * 97u)) % kBits;
    acc += atomicOr(&bm[b >> 5], 1u << (b & 31)) & 1u;
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_persist(unsigned levels, unsigned work, unsigned* bm, Sync* S,
                                                 unsigned long long* out, unsigned* sink) {
  __shared__ unsigned nx, nxcd, me, stop;
  const unsigned tid = threadIdx.x;
  if (tid == 0) {
    me = xcc_id();
    atomicAdd(&S->census[me * 32], 1u);
    atomicAdd(&S->start[0], 1u);
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    stop = 0;
    while (ld(&S->start[0]) < gridDim.x) {  // every workgroup has counted itself in
      __builtin_amdgcn_s_sleep(2);
      if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinCap) {
        stop = 1;
        atomicExch(&S->timeout[0], 1u);
        break;
      }
    }
    nx = ld(&S->census[me * 32]);
    unsigned k = 0;
    for (int x = 0; x < 8; ++x) k += ld(&S->census[x * 32]) ? 1u : 0u;
    nxcd = k;
  }
  __syncthreads();
  if (stop) return;
  unsigned acc = 0;
  const unsigned long long t_begin = __builtin_amdgcn_s_memrealtime();
  for (unsigned l = 0; l < levels; ++l) {
    acc += level_work(bm, l, work);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const unsigned a = atomicAdd(&S->xarrive[me * 32], 1u) + 1u;
      if (a == nx * (l + 1)) {  // the XCD's last arriver
        const unsigned b = atomicAdd(&S->top[0], 1u) + 1u;
        if (b == nxcd * (l + 1)) __hip_atomic_store(&S->gen[0], l + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      while (ld(&S->gen[0]) < l + 1) {
        __builtin_amdgcn_s_sleep(1);
        if (__builtin_amdgcn_s_memrealtime() - t0 > kSpinCap) {
          stop = 1;
          atomicExch(&S->timeout[0], 1u);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (stop) break;
  }
  if (tid == 0 && blockIdx.x == 0) out[0] = __builtin_amdgcn_s_memrealtime() - t_begin;
  if (acc == 0xdeadbeef) sink[0] = acc;
}

__global__ __launch_bounds__(256) void k_level(unsigned level, unsigned work, unsigned* bm, unsigned* sink) {
  const unsigned acc = level_work(bm, level, work);
  if (acc == 0xdeadbeef) sink[0] = acc;
}

int main() {
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  unsigned *bm, *sink;
  Sync* S;
  unsigned long long* out;
  CK(hipMalloc(&bm, kBits / 8 + 64));
  CK(hipMalloc(&S, sizeof(Sync)));
  CK(hipMalloc(&out, 64));
  CK(hipMalloc(&sink, 64));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned levels = 200;
  std::printf("# CUs %d; per-level cost in microseconds (median of 5 runs of %u levels)\n", cus, levels);
  std::printf("%-6s %-5s %-12s %-12s %-8s\n", "wgs", "work", "persist_us", "launch_us", "timeout");
  for (int g : {32, 64, 128, 256}) {
    if (g > cus) continue;
    for (unsigned work : {0u, 1u, 4u}) {
      std::vector<double> tp, tl;
      unsigned to = 0;
      for (int rep = 0; rep < 5; ++rep) {
        CK(hipMemsetAsync(bm, 0, kBits / 8 + 64, s));
        CK(hipMemsetAsync(S, 0, sizeof(Sync), s));
        k_persist<<<g, 256, 0, s>>>(levels, work, bm, S, out, sink);
        CK(hipGetLastError());
        CK(hipStreamSynchronize(s));
        unsigned long long ticks = 0;
        Sync h;
        CK(hipMemcpy(&ticks, out, 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&h, S, sizeof(Sync), hipMemcpyDeviceToHost));
        to |= h.timeout[0];
        tp.push_back(ticks * 1e-2 / levels);  // 100 MHz ticks -> us
        CK(hipMemsetAsync(bm, 0, kBits / 8 + 64, s));
        k_level<<<g, 256, 0, s>>>(0, work, bm, sink);  // warm
        CK(hipEventRecord(e0, s));
        for (unsigned l = 0; l < levels; ++l) k_level<<<g, 256, 0, s>>>(l, work, bm, sink);
        CK(hipEventRecord(e1, s));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        tl.push_back(ms * 1e3 / levels);
      }
      std::sort(tp.begin(), tp.end());
      std::sort(tl.begin(), tl.end());
      std::printf("%-6d %-5u %-12.2f %-12.2f %-8u\n", g, work, tp[2], tl[2], to);
    }
  }
  return 0;
}
