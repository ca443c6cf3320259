// Batched serving for searches that outgrow LDS (10M-vertex G(n,p), RMAT).
//
// k_lds_batch (engine_kernels.hip) answers a query per workgroup entirely in
// LDS; a query whose visited sets overflow the LDS hash used to be re-run on
// the host through the single-query grid engine, one at a time, so a batch on
// a 10M graph degenerated to sequential whole-GPU searches.  This kernel keeps
// those queries batched: one 1024-thread workgroup per query, visited sets as
// per-slot bitmaps in HBM, frontiers as slices of the per-slot BFS queue.
//
//   * Visited bitmaps are all-zero between launches.  They are allocated and
//     cleared once; at exit every workgroup clears exactly the words of the
//     vertices in its two queues (every set bit belongs to a queued vertex),
//     so a query costs O(visited), never O(n).
//   * A level expands the side whose frontier has fewer edges (A1 policy,
//     v1/main-v1.cpp:51), edge-balanced: the workgroup scans the degrees of
//     one frontier vertex per lane into LDS and each lane takes edges, finding its
//     vertex by binary search over the scan (no thread-per-vertex imbalance,
//     the reference's K1 shape, v3/bibfs_cuda_only.cu:13-43).
//   * Claim = test (cached) then atomicOr on the bitmap word; the winner of a
//     bit writes parent and appends to the queue.  The meet test is fused into
//     the claim (K2 check_intersect becomes one load of the other side's word).
//     All meets found in the first meeting level have the same length
//     d_s + 1 + d_t: a neighbour v of u (depth d_s) that the other side reached
//     at depth < d_t would have been expanded by it, so u would already be on
//     both sides.  Any meet vertex therefore gives a shortest path.  The
//     level stops at the first meet it sees, so WHICH shortest path a batch
//     returns depends on scheduling (it may differ between runs and from
//     search()); the hop count does not.  The contract is "any shortest path"
//     (tie-breaking is unspecified in every reference engine).
//   * A level whose frontier has more than `edge_cap` edges stops the query
//     with kHandoff; the host answers it with the single-query engine, whose
//     bottom-up levels suit hub-heavy frontiers better than one CU does.
#include <hip/hip_runtime.h>

#include "device.hpp"

namespace bibfs {
namespace {

using namespace dev;


struct BgArgs {
  const uint32_t* row_off;  // n + 1 (32-bit offsets)
  const uint32_t* col;
  uint32_t n;
  uint32_t words;           // bitmap words per side
  const uint32_t* qidx;     // K query indices into src/dst/slots/out
  const uint32_t* src;
  const uint32_t* dst;
  uint32_t* slots;          // per query: parent[2] + queue[2], n words each
  uint32_t* bits;           // per query: 2 * words, all-zero between launches
  BatchOut* out;
  uint32_t* path;           // per query: path_cap words
  uint32_t path_cap;
  unsigned long long edge_cap;
};

__device__ __forceinline__ uint32_t ld_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// kBgThreads: 1024 by default (16 waves: 4x fewer chunk trips per level for
// the same latency chain; measured 1.6-2.5x faster than 256 at 256 queries).
template <int kBgThreads>
__global__ __launch_bounds__(kBgThreads) void k_batch_global(BgArgs A) {
  __shared__ uint32_t pre[kBgThreads + 1];   // exclusive degree scan of the chunk
  __shared__ uint32_t rowb[kBgThreads];      // row start of each chunk vertex
  __shared__ uint32_t vtx[kBgThreads];       // the chunk's vertices
  __shared__ uint32_t wsum[kBgThreads / kWave];
  __shared__ uint32_t qtail, meet;
  __shared__ unsigned long long nedges;

  const uint32_t tid = threadIdx.x;
  const uint32_t q = A.qidx[blockIdx.x];
  const uint32_t n = A.n;
  const uint32_t src = A.src[q], dst = A.dst[q];
  uint32_t* base = A.slots + (size_t)q * 4 * n;
  // per-side pointers as selects, not arrays indexed by the side: a
  // dynamically indexed local array of pointers loses the global address
  // space, and every access through it became a flat operation
  uint32_t* const par0 = base;
  uint32_t* const par1 = base + n;
  uint32_t* const que0 = base + 2 * (size_t)n;
  uint32_t* const que1 = base + 3 * (size_t)n;
  uint32_t* const bit0 = A.bits + (size_t)q * 2 * A.words;
  uint32_t* const bit1 = bit0 + A.words;

  if (tid < 2) {
    const uint32_t r = tid ? dst : src;
    atomicOr(&(tid ? bit1 : bit0)[r >> 5], 1u << (r & 31));
    (tid ? par1 : par0)[r] = r;
    (tid ? que1 : que0)[0] = r;
  }
  if (tid == 0) meet = kEmpty;
  // every lane holds the same copy of the (small) search state
  uint32_t fbeg[2] = {0, 0}, fend[2] = {1, 1};
  int depth[2] = {0, 0};
  unsigned long long fedges[2] = {(unsigned long long)(A.row_off[src + 1] - A.row_off[src]),
                                  (unsigned long long)(A.row_off[dst + 1] - A.row_off[dst])};
  unsigned long long einsp = 0;
  uint32_t levels = 0, status = kRunning, side = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();

  while (status == kRunning) {
    if (fend[0] == fbeg[0] || fend[1] == fbeg[1]) {
      status = kNoPath;
      break;
    }
    const uint32_t s = fedges[0] <= fedges[1] ? 0u : 1u;
    if (fedges[s] > A.edge_cap) {
      status = kHandoff;
      break;
    }
    const uint32_t t = s ^ 1u;
    uint32_t* __restrict__ bs = s ? bit1 : bit0;
    const uint32_t* __restrict__ bt = t ? bit1 : bit0;
    uint32_t* __restrict__ ps = s ? par1 : par0;
    uint32_t* __restrict__ qs = s ? que1 : que0;
    if (tid == 0) {
      qtail = fend[s];
      nedges = 0;
    }
    __syncthreads();
    for (uint32_t c = fbeg[s]; c < fend[s]; c += kBgThreads) {
      const uint32_t i = c + tid;
      uint32_t u = 0, b = 0, deg = 0;
      if (i < fend[s]) {
        u = qs[i];
        b = A.row_off[u];
        deg = A.row_off[u + 1] - b;
      }
      // workgroup exclusive scan of deg: wave scan by DPP-free shuffles, then wave totals
      uint32_t x = deg;
      const uint32_t lane = tid & (kWave - 1), w = tid / kWave;
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t y = __shfl_up(x, d, kWave);
        if (lane >= (uint32_t)d) x += y;
      }
      if (lane == kWave - 1) wsum[w] = x;
      __syncthreads();
      uint32_t woff = 0, total = 0;
#pragma unroll
      for (uint32_t k = 0; k < kBgThreads / kWave; ++k) {
        woff += k < w ? wsum[k] : 0u;
        total += wsum[k];
      }
      pre[tid] = woff + x - deg;
      rowb[tid] = b;
      vtx[tid] = u;
      if (tid == 0) pre[kBgThreads] = total;
      __syncthreads();
      einsp += total;
      for (uint32_t e = tid; e < total; e += kBgThreads) {
        // every meet of this level has the same length (see above): the
        // first one ends the level (a Kronecker hub level would otherwise
        // walk all its edges on this one CU)
        if (__hip_atomic_load(&meet, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != kEmpty) break;
        // owner vertex: last j with pre[j] <= e
        uint32_t lo = 0, hi = kBgThreads;
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pre[mid] <= e) lo = mid;
          else hi = mid;
        }
        const uint32_t v = A.col[rowb[lo] + (e - pre[lo])];
        const uint32_t wi = v >> 5, bit = 1u << (v & 31);
        if (ld_agent(&bs[wi]) & bit) continue;
        const uint32_t old = atomicOr(&bs[wi], bit);
        if (old & bit) continue;
        ps[v] = vtx[lo];
        qs[atomicAdd(&qtail, 1u)] = v;
        atomicAdd(&nedges, (unsigned long long)(A.row_off[v + 1] - A.row_off[v]));
        if (ld_agent(&bt[wi]) & bit) atomicMin(&meet, v);
      }
      __syncthreads();  // pre/rowb/vtx are rewritten by the next chunk
      if (meet != kEmpty) break;  // block-uniform: read after the barrier
    }
    // plain stores of parent/queue become visible to every lane of the block
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    ++levels;
    side = s;
    fbeg[s] = fend[s];
    fend[s] = qtail;
    fedges[s] = nedges;
    depth[s] += 1;
    if (meet != kEmpty) status = kFound;
    __syncthreads();  // qtail/nedges/meet are reset by thread 0 next level
  }

  // result + path (thread 0 walks both parent chains)
  if (tid == 0) {
    BatchOut& o = A.out[q];
    o.status = status;
    o.levels = levels;
    o.einsp = einsp;
    o.visited = fend[0] + fend[1];
    o.meet = status == kFound ? meet : kEmpty;
    o.hops = -1;
    o.path_len = 0;
    if (status == kFound) {
      const uint32_t m = meet;
      const int d0 = depth[0], d1 = depth[1];
      (void)side;
      o.hops = d0 + d1;
      o.path_len = (uint32_t)(d0 + d1 + 1);
      if (o.path_len <= A.path_cap) {
        uint32_t* P = A.path + (size_t)q * A.path_cap;
        uint32_t x = m;
        for (int k = d0; k >= 0; --k) {
          P[k] = x;
          x = par0[x];
        }
        x = m;
        for (int k = d0; k <= d0 + d1; ++k) {
          P[k] = x;
          x = par1[x];
        }
      } else {
        o.status = kHandoff;  // path longer than the slot: the host re-runs it
      }
    }
  }
  // leave the bitmaps all-zero: clear the word of every queued vertex
  for (uint32_t i = tid; i < fend[0]; i += kBgThreads) bit0[que0[i] >> 5] = 0u;
  for (uint32_t i = tid; i < fend[1]; i += kBgThreads) bit1[que1[i] >> 5] = 0u;
  // vertices claimed in a level interrupted by nothing: fend already covers
  // every append (levels always run to completion before the loop exits)
}

}  // namespace

namespace launch {

void batch_global(const GraphView& g, uint32_t words, const uint32_t* d_qidx, uint32_t k, const uint32_t* d_src,
                  const uint32_t* d_dst, uint32_t* d_slots, uint32_t* d_bits, dev::BatchOut* d_out,
                  uint32_t* d_path, uint32_t path_cap, unsigned long long edge_cap, int threads, hipStream_t s) {
  BIBFS_REQUIRE(g.row_off32 != nullptr, "batched search: 32-bit row offsets required");
  BIBFS_REQUIRE((uint64_t)words >= (uint64_t)g.n / 32 + 1, "batch_global: bitmaps smaller than the graph");
  if (k == 0) return;
  BgArgs A{g.row_off32, g.col, g.n, words, d_qidx, d_src, d_dst, d_slots, d_bits, d_out, d_path, path_cap,
           edge_cap};
  if (threads == 1024)
    k_batch_global<1024><<<k, 1024, 0, s>>>(A);
  else
    k_batch_global<256><<<k, 256, 0, s>>>(A);
  HIP_CHECK(hipGetLastError());
}

}  // namespace launch
}  // namespace bibfs
