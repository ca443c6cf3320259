// Host <-> resident-kernel mailbox round trip, for the resident query server
// (csrc/hip/engine_kernels.hip, k_lds_server).  A one-wave kernel polls a
// request word; the host writes seq, the kernel echoes it into a pinned host
// word, the host spins on the echo.  Prints the median round trip per
// mailbox placement:
//   host     : request word in pinned host memory (GPU polls over PCIe)
//   devfine  : request word in fine-grained device memory written by the CPU
//              through the BAR (GPU polls its own HBM, bypassing L2)
//   hsa      : the same, allocated from the GPU's fine-grained HSA pool with
//              access granted to the CPU agent (hsa_amd_agents_allow_access)
// plus the kernel-launch round trip (empty kernel + host spin on a flag) for
// reference.  Build: make micro.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <x86intrin.h>

#include <setjmp.h>
#include <signal.h>

#include <algorithm>
#include <chrono>
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

// pipelined: keep several poll loads in flight (window 4) spaced by s_sleep
__global__ void k_echo(const uint32_t* req, uint32_t* resp, uint32_t n, int pipelined) {
  uint32_t last = 0;
  const unsigned long long t_end = __builtin_amdgcn_s_memrealtime() + 100000000ull;  // 1 s cap
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s = last;
    while (s == last) {
      if (pipelined) {
        const uint32_t a = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(16);
        const uint32_t b = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(16);
        const uint32_t c = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __builtin_amdgcn_s_sleep(16);
        const uint32_t d = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        s = a != last ? a : b != last ? b : c != last ? c : d;
      } else {
        s = __hip_atomic_load(req, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      if (__builtin_amdgcn_s_memrealtime() > t_end) return;
    }
    last = s;
    __hip_atomic_store(resp, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Ring of 4 poll loads kept in flight (a new one issued as each returns),
// spaced by s_sleep: a request is seen one PCIe read after it lands plus a
// fraction of the spacing, instead of up to two reads later.
__global__ void k_echo_ring(const uint32_t* req, uint32_t* resp, uint32_t n) {
  uint32_t last = 0;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t s, a, b, c, d, k = 0;
    asm volatile(
        "global_load_dword %[a], %[p], off sc0 sc1\n\t"
        "s_sleep 2\n\t"
        "global_load_dword %[b], %[p], off sc0 sc1\n\t"
        "s_sleep 2\n\t"
        "global_load_dword %[c], %[p], off sc0 sc1\n\t"
        "s_sleep 2\n\t"
        "global_load_dword %[d], %[p], off sc0 sc1\n"
        "1:\n\t"
        "s_waitcnt vmcnt(3)\n\t"
        "v_readfirstlane_b32 %[s], %[a]\n\t"
        "s_cmp_lg_u32 %[s], %[last]\n\t"
        "s_cbranch_scc1 2f\n\t"
        "global_load_dword %[a], %[p], off sc0 sc1\n\t"
        "s_waitcnt vmcnt(3)\n\t"
        "v_readfirstlane_b32 %[s], %[b]\n\t"
        "s_cmp_lg_u32 %[s], %[last]\n\t"
        "s_cbranch_scc1 2f\n\t"
        "global_load_dword %[b], %[p], off sc0 sc1\n\t"
        "s_waitcnt vmcnt(3)\n\t"
        "v_readfirstlane_b32 %[s], %[c]\n\t"
        "s_cmp_lg_u32 %[s], %[last]\n\t"
        "s_cbranch_scc1 2f\n\t"
        "global_load_dword %[c], %[p], off sc0 sc1\n\t"
        "s_waitcnt vmcnt(3)\n\t"
        "v_readfirstlane_b32 %[s], %[d]\n\t"
        "s_cmp_lg_u32 %[s], %[last]\n\t"
        "s_cbranch_scc1 2f\n\t"
        "global_load_dword %[d], %[p], off sc0 sc1\n\t"
        "s_add_u32 %[k], %[k], 1\n\t"
        "s_cmp_lt_u32 %[k], 0x800000\n\t"  // bounded: ~4 polls per pass, a few seconds
        "s_cbranch_scc1 1b\n\t"
        "s_mov_b32 %[s], %[last]\n"
        "2:\n\t"
        "s_waitcnt vmcnt(0)"
        : [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c), [d] "=&v"(d), [s] "=&s"(s), [k] "+s"(k)
        : [p] "v"(req), [last] "s"(last)
        : "scc", "memory");
    if (s == last) return;  // timed out
    last = s;
    __hip_atomic_store(resp, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void k_flag(uint32_t* resp, uint32_t v) {
  __hip_atomic_store(resp, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static sigjmp_buf g_jb;
static void on_segv(int) { siglongjmp(g_jb, 1); }
// Can the CPU store to this device pointer directly (large-BAR mapping)?
static bool cpu_writable(uint32_t* p) {
  struct sigaction sa{}, old{};
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  bool ok = false;
  if (sigsetjmp(g_jb, 1) == 0) {
    *(volatile uint32_t*)p = 0;
    ok = true;
  }
  sigaction(SIGSEGV, &old, nullptr);
  signal(SIGBUS, SIG_DFL);
  return ok;
}

// Fine-grained VRAM from the HSA pool, CPU access granted: nullptr if the
// runtime refuses (no large BAR, no such pool).
struct HsaFind {
  hsa_agent_t cpu{}, gpu{};
  bool have_cpu = false, have_gpu = false;
  hsa_amd_memory_pool_t pool{};
  bool have_pool = false;
};
static hsa_status_t find_agent(hsa_agent_t a, void* d) {
  auto* f = static_cast<HsaFind*>(d);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) f->cpu = a, f->have_cpu = true;
  if (t == HSA_DEVICE_TYPE_GPU && !f->have_gpu) f->gpu = a, f->have_gpu = true;
  return HSA_STATUS_SUCCESS;
}
static hsa_status_t find_pool(hsa_amd_memory_pool_t p, void* d) {
  auto* f = static_cast<HsaFind*>(d);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (seg == HSA_AMD_SEGMENT_GLOBAL && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) && !f->have_pool)
    f->pool = p, f->have_pool = true;
  return HSA_STATUS_SUCCESS;
}
static uint32_t* hsa_fine_vram(size_t bytes) {
  if (hsa_init() != HSA_STATUS_SUCCESS) return nullptr;
  HsaFind f;
  hsa_iterate_agents(find_agent, &f);
  if (!f.have_cpu || !f.have_gpu) return nullptr;
  hsa_amd_agent_iterate_memory_pools(f.gpu, find_pool, &f);
  if (!f.have_pool) {
    std::printf("hsa: no fine-grained global pool on the GPU agent\n");
    return nullptr;
  }
  void* p = nullptr;
  if (hsa_amd_memory_pool_allocate(f.pool, bytes, 0, &p) != HSA_STATUS_SUCCESS) return nullptr;
  const hsa_status_t s = hsa_amd_agents_allow_access(1, &f.cpu, nullptr, p);
  std::printf("hsa: fine-grained VRAM %p, allow_access(cpu) status %d\n", p, (int)s);
  if (s != HSA_STATUS_SUCCESS) return nullptr;
  return static_cast<uint32_t*>(p);
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

static double run_echo(uint32_t* req_host_view, const uint32_t* req_dev_view, uint32_t* resp, int pipelined) {
  const uint32_t n = 2000;
  *(volatile uint32_t*)req_host_view = 0;
  *(volatile uint32_t*)resp = 0;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  if (pipelined == 2)
    k_echo_ring<<<1, 64, 0, st>>>(req_dev_view, resp, n);
  else
    k_echo<<<1, 64, 0, st>>>(req_dev_view, resp, n, pipelined);
  CK(hipGetLastError());
  std::vector<double> rt;
  for (uint32_t i = 1; i <= n; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(req_host_view, i, __ATOMIC_RELEASE);
    const auto tmax = t0 + std::chrono::milliseconds(200);
    while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != i) {
      _mm_pause();
      if (std::chrono::steady_clock::now() > tmax) {
        std::printf("  timeout at %u\n", i);
        CK(hipStreamSynchronize(st));
        return -1;
      }
    }
    rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipStreamSynchronize(st));
  CK(hipStreamDestroy(st));
  return median(rt);
}

int main() {
  uint32_t *hreq, *resp;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hreq), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostMalloc(reinterpret_cast<void**>(&resp), 4096, hipHostMallocMapped | hipHostMallocCoherent));
  std::printf("host-pinned mailbox, serial polls    : %.2f us\n", run_echo(hreq, hreq, resp, 0));
  std::printf("host-pinned mailbox, pipelined polls : %.2f us\n", run_echo(hreq, hreq, resp, 1));
  std::printf("host-pinned mailbox, ring of 4 polls : %.2f us\n", run_echo(hreq, hreq, resp, 2));
  std::printf("host-pinned mailbox, serial polls    : %.2f us (again)\n", run_echo(hreq, hreq, resp, 0));
  std::printf("host-pinned mailbox, ring of 4 polls : %.2f us (again)\n", run_echo(hreq, hreq, resp, 2));

  uint32_t* dfine = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&dfine), 4096, hipDeviceMallocFinegrained) == hipSuccess) {
    hipPointerAttribute_t at{};
    CK(hipPointerGetAttributes(&at, dfine));
    std::printf("fine-grained device buffer: device ptr %p host ptr %p\n", at.devicePointer, at.hostPointer);
    if (at.hostPointer) {
      std::printf("device-fine mailbox, serial polls    : %.2f us\n",
                  run_echo(static_cast<uint32_t*>(at.hostPointer), dfine, resp, 0));
    } else if (cpu_writable(dfine)) {
      std::printf("device-fine mailbox (CPU stores through the device pointer), serial polls : %.2f us\n",
                  run_echo(dfine, dfine, resp, 0));
      std::printf("device-fine mailbox (CPU stores through the device pointer), ring of 4    : %.2f us\n",
                  run_echo(dfine, dfine, resp, 2));
    } else {
      std::printf("device-fine mailbox: not CPU-writable\n");
    }
  }
  uint32_t* dunc = nullptr;
  if (hipExtMallocWithFlags(reinterpret_cast<void**>(&dunc), 4096, hipDeviceMallocUncached) == hipSuccess) {
    if (cpu_writable(dunc))
      std::printf("device-uncached mailbox, serial polls : %.2f us\n", run_echo(dunc, dunc, resp, 0));
    else
      std::printf("device-uncached mailbox: not CPU-writable\n");
  }
  if (uint32_t* hf = hsa_fine_vram(4096)) {
    if (cpu_writable(hf)) {
      std::printf("hsa fine VRAM mailbox, serial polls   : %.2f us\n", run_echo(hf, hf, resp, 0));
      std::printf("hsa fine VRAM mailbox, ring of 4      : %.2f us\n", run_echo(hf, hf, resp, 2));
      std::printf("hsa fine VRAM mailbox, serial (again) : %.2f us\n", run_echo(hf, hf, resp, 0));
    } else {
      std::printf("hsa fine VRAM mailbox: not CPU-writable\n");
    }
  }
  uint32_t* dplain = nullptr;
  CK(hipMalloc(reinterpret_cast<void**>(&dplain), 4096));
  std::printf("plain hipMalloc: CPU-writable %d\n", (int)cpu_writable(dplain));
  // launch round trip
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<double> rt;
  for (uint32_t i = 1; i <= 2000; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    k_flag<<<1, 64, 0, st>>>(resp, 100000 + i);
    while (__atomic_load_n(resp, __ATOMIC_ACQUIRE) != 100000 + i) _mm_pause();
    rt.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  CK(hipStreamSynchronize(st));
  std::printf("kernel launch -> flag round trip     : %.2f us\n", median(rt));
  return 0;
}
