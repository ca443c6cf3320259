// Multi-GPU bidirectional BFS (see include/bibfs/dist_engine.hpp).
//
// Reference parity: v4/mpi_bas.cpp:79-132 (per-level loop), v4/comp.cu:20-38
// (expand kernel with a vertex-ownership filter that the reference disabled
// by launching with rank=0,size=1, v4/comp.cu:99), v2/main-v2.cpp:59-83 (the
// frontier-list exchange and the min-candidate meet rule) and the collective
// sites of SURVEY.md §2.5 (MPI_Allreduce BOR over N ints, LOR flags per level).
//
// A search runs in ROUNDS.  A round expands one side or -- when the two
// frontiers are comparable -- both sides in lockstep.  One side's level is
//   pre      (compute stream) top-down: expand the owned frontier, claim owned
//                             neighbours, emit (v, parent) candidates for
//                             remote owners (each remote vertex at most once
//                             per search and side); bottom-up: the owned slice
//                             of the frontier bitmap
//   exchange (comm stream)    ONE allgather: candidate blocks or bitmap slices
//   post     (comm stream)    owners claim the candidates addressed to them, or
//                             scan their unvisited vertices against the bitmap
// In a lockstep round the exchange + post of the source side run on the comm
// stream while the target side's pre runs on the compute stream: the
// opposite-direction expand overlaps the RCCL transfer.  The
// round ends with a meet check over the vertices claimed in it (exact lengths
// from per-vertex depths, so the minimum over a lockstep round is the
// distance) and ONE grouped allreduce -- {claimed counts, degree sums} (sum)
// and the meet key (min) -- read back with one host sync: the only host
// round trip of a round, except when a top-down candidate block cannot be
// sized from host-known bounds (then one allreduce(MAX) of the per-rank
// counts sizes it).
#include <algorithm>
#include <chrono>
#include <cstring>
#include <thread>

#include "bibfs/dist_engine.hpp"
#include "bibfs/io.hpp"
#include "comm.hpp"
#include "device.hpp"

namespace bibfs {

using namespace dev;
using dist::DType;
using dist::ROp;

namespace {

constexpr int kThreads = 256;
constexpr unsigned long long kNoKey = ~0ull;
constexpr uint64_t kCapMax = 1u << 20;          // candidate pairs per rank per level
constexpr uint64_t kNoSyncBytes = 1u << 20;     // candidate allgather sized from host bounds up to this many bytes
constexpr uint64_t kLockstepEdges = 1u << 16;   // both frontiers at most this many edges: always lockstep

struct DState {
  uint32_t fbeg[2], fend[2], qtail[2];  // queue[s][fbeg, fend) = frontier; qtail = append cursor
  uint32_t send_count[2];               // candidates this rank emitted for side s this level
  uint32_t pad[2];
  unsigned long long new_edges[2];      // degree sum of the vertices side s claimed this level
};

// Reduced across ranks (device words, read back into pinned memory).
struct Reduced {
  unsigned long long sums[4];  // [2s] vertices side s claimed this round, [2s+1] their degree sum (sum)
  unsigned long long meetkey;  // (path length << 32) | meet vertex (min)
  uint32_t maxsend[2];         // candidates of side s on this rank (max)
  uint32_t md[2];              // depth of the meet vertex from each root (owner contributes; min)
};

struct DView {
  uint32_t n, lo, hi, chunk;  // owned = [lo, hi); owner(v) = v / chunk
  const uint64_t* row_off;    // owned rows
  const uint32_t* col;        // global column ids
  uint32_t* vis[2];           // owned slices, chunk/32 words
  uint32_t* parent[2];        // chunk entries, valid where visited
  uint32_t* depth[2];         // chunk entries, valid where visited
  uint32_t* queue[2];         // owned vertices (global ids) in claim order
  uint32_t* sent[2];          // bitmaps over ALL vertices: remote vertices already offered this search
  uint32_t* obits[2];         // owned frontier slice (chunk/32 words)
  uint32_t* gbits[2];         // allgathered frontier bitmap (P * chunk/32 words: global index)
  uint32_t* send[2];          // {count, pad, (v, u) pairs}
  uint32_t* recv[2];          // P blocks
  uint32_t cap;               // candidate pairs per rank per level
  int P;
  DState* st;
  Reduced* red;
};

template <typename T>
__device__ __forceinline__ T* pick(T* const (&a)[2], int s) {
  return s ? a[1] : a[0];
}

// Claim owned vertex v for side s (parent u, depth dnew).  Wave-cooperative:
// every lane of the wave calls it, `want` masks lanes.  One queue append and
// one degree-sum atomic per wave.
__device__ __forceinline__ void wave_claim(const DView& V, int s, bool want, uint32_t v, uint32_t u,
                                           uint32_t dnew) {
  const uint32_t li = v - V.lo;
  uint32_t* vis = pick(V.vis, s);
  bool mine = false;
  if (want) {
    const uint32_t bit = 1u << (li & 31);
    if (!(vis[li >> 5] & bit)) mine = !(atomicOr(&vis[li >> 5], bit) & bit);
  }
  const unsigned long long mask = __ballot(mine);
  if (!mask) return;  // wave-uniform
  const uint32_t lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  unsigned long long deg = 0;
  if (mine) {
    pick(V.parent, s)[li] = u;
    pick(V.depth, s)[li] = dnew;
    deg = V.row_off[li + 1] - V.row_off[li];
  }
  uint32_t pos = 0;
  if (lane == (uint32_t)leader) pos = atomicAdd(&V.st->qtail[s], (uint32_t)__popcll(mask));
  pos = __shfl(pos, leader);
  if (mine) pick(V.queue, s)[pos + mbcnt64(mask)] = v;
  deg = wave_sum(deg);
  if (lane == (uint32_t)leader) atomicAdd(&V.st->new_edges[s], deg);
}

// Offer remote vertex v (parent u) to its owner -- at most once per search and
// side: after the level that offered it, v is visited by its owner (claimed
// from the exchange, or by the bottom-up fallback of an overflowing level).
__device__ __forceinline__ void wave_emit(const DView& V, int s, bool want, uint32_t v, uint32_t u) {
  uint32_t* sb = pick(V.sent, s);
  bool emit = false;
  if (want) {
    const uint32_t bit = 1u << (v & 31);
    if (!(sb[v >> 5] & bit)) emit = !(atomicOr(&sb[v >> 5], bit) & bit);
  }
  const unsigned long long mask = __ballot(emit);
  if (!mask) return;  // wave-uniform
  const uint32_t lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t pos = 0;
  if (lane == (uint32_t)leader) pos = atomicAdd(&V.st->send_count[s], (uint32_t)__popcll(mask));
  pos = __shfl(pos, leader) + mbcnt64(mask);
  if (emit && pos < V.cap) reinterpret_cast<uint2*>(pick(V.send, s))[1 + pos] = make_uint2(v, u);
}

// Top-down pre phase: edge-balanced expansion of the owned frontier.  A
// workgroup takes 256 frontier vertices, scans their degrees in LDS and walks
// the chunk's edges one per lane (binary search for the owning vertex), so a
// hub costs the same per edge as a leaf and no lane idles on a short row.
__global__ __launch_bounds__(kThreads) void k_td_expand(DView V, int s, uint32_t dnew, int first) {
  __shared__ uint32_t su[kThreads];
  __shared__ unsigned long long sb[kThreads], se[kThreads];
  __shared__ unsigned long long wsum[kThreads / kWave];
  if (first && blockIdx.x == 0 && threadIdx.x == 0) V.red->meetkey = kNoKey;  // new round
  const uint32_t fb = V.st->fbeg[s], F = V.st->fend[s] - fb;
  const uint32_t* q = pick(V.queue, s);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  for (uint64_t c0 = (uint64_t)blockIdx.x * kThreads; c0 < F; c0 += (uint64_t)gridDim.x * kThreads) {
    const uint64_t i = c0 + tid;
    unsigned long long deg = 0, b = 0;
    uint32_t u = 0;
    if (i < F) {
      u = q[fb + i];
      const uint32_t li = u - V.lo;
      b = V.row_off[li];
      deg = V.row_off[li + 1] - b;
    }
    su[tid] = u;
    sb[tid] = b;
    unsigned long long x = deg;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const unsigned long long y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == kWave - 1) wsum[wid] = x;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kThreads / kWave; ++k) {
      pre += k < wid ? wsum[k] : 0ull;
      tot += wsum[k];
    }
    se[tid] = pre + x - deg;
    __syncthreads();
    for (unsigned long long base = 0; base < tot; base += kThreads) {
      const unsigned long long e = base + tid;
      const bool valid = e < tot;
      uint32_t uu = 0, v = 0;
      if (valid) {
        uint32_t a = 0, z = kThreads;  // last slot whose edge range starts at or before e
        while (z - a > 1) {
          const uint32_t mid = (a + z) >> 1;
          if (se[mid] <= e) a = mid;
          else z = mid;
        }
        uu = su[a];
        v = V.col[sb[a] + (e - se[a])];
      }
      const bool own = valid && v >= V.lo && v < V.hi;
      wave_claim(V, s, own, v, uu, dnew);
      wave_emit(V, s, valid && !own, v, uu);
    }
    __syncthreads();
  }
}

__global__ void k_send_header(DView V, int s) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t c = V.st->send_count[s];
  pick(V.send, s)[0] = c;
  V.red->maxsend[s] = c;
}

// Top-down post phase: owners claim the candidates addressed to them (block r
// of the gathered buffer is rank r's {count, pad, pairs}).
__global__ __launch_bounds__(kThreads) void k_td_claim(DView V, int s, uint32_t per_rank, uint32_t dnew) {
  const uint64_t blk = 2 + 2 * (uint64_t)per_rank;
  const uint64_t total = (uint64_t)V.P * per_rank;
  const uint32_t* R = pick(V.recv, s);
  for (uint64_t base = (uint64_t)blockIdx.x * kThreads; base < total; base += (uint64_t)gridDim.x * kThreads) {
    const uint64_t t = base + threadIdx.x;
    bool want = false;
    uint32_t v = 0, u = 0;
    if (t < total) {
      const uint64_t r = t / per_rank, i = t % per_rank;
      const uint32_t* b = R + r * blk;
      if (i < min(b[0], per_rank)) {
        const uint2 p = reinterpret_cast<const uint2*>(b)[1 + i];
        v = p.x;
        u = p.y;
        want = v >= V.lo && v < V.hi;
      }
    }
    wave_claim(V, s, want, v, u, dnew);
  }
}

// Bottom-up pre phase: this rank's slice of the frontier bitmap.
__global__ void k_obits(DView V, int s, int first) {
  if (first && blockIdx.x == 0 && threadIdx.x == 0) V.red->meetkey = kNoKey;  // new round
  const uint32_t fb = V.st->fbeg[s], fe = V.st->fend[s];
  const uint32_t* q = pick(V.queue, s);
  uint32_t* ob = pick(V.obits, s);
  for (uint64_t i = fb + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < fe;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t li = q[i] - V.lo;
    atomicOr(&ob[li >> 5], 1u << (li & 31));
  }
}

// Bottom-up post phase: one wave owns 64 consecutive owned vertices (two
// whole visited words: the slice is 64-aligned); each unvisited one scans its
// row for a neighbour in the gathered frontier bitmap and stops at the first
// hit; the visited words are rebuilt from one ballot with plain stores.
__global__ __launch_bounds__(kThreads) void k_bu(DView V, int s, uint32_t dnew) {
  const uint32_t nloc = V.hi - V.lo;
  const uint32_t* __restrict__ gb = pick(V.gbits, s);
  uint32_t* __restrict__ vis = pick(V.vis, s);
  const uint32_t lane = __lane_id();
  const uint64_t nw = ((uint64_t)nloc + 63) / 64;
  const uint64_t w0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kWave;
  const uint64_t ws = (uint64_t)gridDim.x * blockDim.x / kWave;
  for (uint64_t gw = w0; gw < nw; gw += ws) {
    const uint32_t li = (uint32_t)(gw * 64 + lane);
    const uint32_t word = vis[gw * 2 + (lane >> 5)];
    const uint32_t bit = 1u << (lane & 31);
    bool found = false;
    uint32_t pu = 0;
    unsigned long long deg = 0;
    if (li < nloc && !(word & bit)) {
      const uint64_t b = V.row_off[li], e = V.row_off[li + 1];
      deg = e - b;
      uint64_t k = b;
      for (; k + 4 <= e && !found; k += 4) {
        const uint32_t c0 = V.col[k], c1 = V.col[k + 1], c2 = V.col[k + 2], c3 = V.col[k + 3];
        const bool h0 = (gb[c0 >> 5] >> (c0 & 31)) & 1u, h1 = (gb[c1 >> 5] >> (c1 & 31)) & 1u;
        const bool h2 = (gb[c2 >> 5] >> (c2 & 31)) & 1u, h3 = (gb[c3 >> 5] >> (c3 & 31)) & 1u;
        if (h0 | h1 | h2 | h3) {
          found = true;
          pu = h0 ? c0 : (h1 ? c1 : (h2 ? c2 : c3));
        }
      }
      for (; k < e && !found; ++k) {
        const uint32_t c0 = V.col[k];
        if ((gb[c0 >> 5] >> (c0 & 31)) & 1u) {
          found = true;
          pu = c0;
        }
      }
    }
    const unsigned long long mask = __ballot(found);
    if (!mask) continue;  // wave-uniform
    if (lane == 0) vis[gw * 2] = word | (uint32_t)mask;
    if (lane == 32) vis[gw * 2 + 1] = word | (uint32_t)(mask >> 32);
    const int leader = __ffsll((long long)mask) - 1;
    if (found) {
      pick(V.parent, s)[li] = pu;
      pick(V.depth, s)[li] = dnew;
    }
    uint32_t pos = 0;
    if (lane == (uint32_t)leader) pos = atomicAdd(&V.st->qtail[s], (uint32_t)__popcll(mask));
    pos = __shfl(pos, leader);
    if (found) pick(V.queue, s)[pos + mbcnt64(mask)] = V.lo + li;
    const unsigned long long ds = wave_sum(found ? deg : 0ull);
    if (lane == (uint32_t)leader) atomicAdd(&V.st->new_edges[s], ds);
  }
}

// Meet check for side s over the vertices it claimed this round: one the other
// side also holds closes a path of length dnew + depth_other(v).
__global__ __launch_bounds__(kThreads) void k_meet(DView V, int s, uint32_t dnew) {
  const uint32_t* q = pick(V.queue, s);
  const uint32_t* ov = pick(V.vis, s ^ 1);
  const uint32_t* od = pick(V.depth, s ^ 1);
  const uint32_t b = V.st->fend[s], e = V.st->qtail[s];
  unsigned long long best = kNoKey;
  for (uint64_t i = b + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < e;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = q[i], li = v - V.lo;
    if ((ov[li >> 5] >> (li & 31)) & 1u) {
      const unsigned long long key = ((unsigned long long)(dnew + od[li]) << 32) | v;
      best = key < best ? key : best;
    }
  }
#pragma unroll
  for (int o = kWave / 2; o >= 1; o >>= 1) {
    const unsigned long long y = __shfl_xor(best, o);
    best = y < best ? y : best;
  }
  if (__lane_id() == 0 && best != kNoKey) atomicMin(&V.red->meetkey, best);
}

// Round bookkeeping, identical on every rank: publish the per-side counts for
// the reduction and advance the frontiers of the sides that expanded.
__global__ void k_round_end(DView V, int sides) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DState* st = V.st;
  for (int s = 0; s < 2; ++s) {
    const bool on = (sides >> s) & 1;
    V.red->sums[2 * s] = on ? (unsigned long long)(st->qtail[s] - st->fend[s]) : 0ull;
    V.red->sums[2 * s + 1] = on ? st->new_edges[s] : 0ull;
    if (on) {
      st->fbeg[s] = st->fend[s];
      st->fend[s] = st->qtail[s];
    }
    st->send_count[s] = 0;
    st->new_edges[s] = 0;
  }
}

__global__ void k_seed(DView V, uint32_t src, uint32_t dst) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DState* st = V.st;
  for (int s = 0; s < 2; ++s) {
    st->fbeg[s] = st->fend[s] = st->qtail[s] = 0;
    st->send_count[s] = 0;
    st->new_edges[s] = 0;
    V.red->sums[2 * s] = V.red->sums[2 * s + 1] = 0;
    const uint32_t v = s ? dst : src;
    if (v >= V.lo && v < V.hi) {
      const uint32_t li = v - V.lo;
      pick(V.vis, s)[li >> 5] |= 1u << (li & 31);
      pick(V.parent, s)[li] = kEmpty;
      pick(V.depth, s)[li] = 0;
      pick(V.queue, s)[0] = v;
      st->fend[s] = st->qtail[s] = 1;
      V.red->sums[2 * s] = 1;
      V.red->sums[2 * s + 1] = V.row_off[li + 1] - V.row_off[li];
    }
  }
  V.red->meetkey = kNoKey;
  V.red->maxsend[0] = V.red->maxsend[1] = 0;
  V.red->md[0] = V.red->md[1] = kEmpty;
}

// The owner of the meet vertex contributes its two depths (others ~0, min-reduced).
__global__ void k_meet_depth(DView V, uint32_t meet) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool own = meet >= V.lo && meet < V.hi;
  V.red->md[0] = own ? V.depth[0][meet - V.lo] : kEmpty;
  V.red->md[1] = own ? V.depth[1][meet - V.lo] : kEmpty;
}

// Path reconstruction step: cur[q] -> its parent (only the owner knows it; the
// others contribute ~0 to the ncclMin that follows).
__global__ void k_path_step(DView V, uint32_t* cur, uint32_t* pathS, uint32_t* pathT, int i, int dS, int dT) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int q = 0; q < 2; ++q) {
    const int d = q ? dT : dS;
    const uint32_t c = cur[q];
    if (i <= d) (q ? pathT : pathS)[i] = c;
    uint32_t nxt = c;  // past the end: every rank keeps the same value
    if (i < d) {
      nxt = kEmpty;
      if (c >= V.lo && c < V.hi) nxt = (q ? V.parent[1] : V.parent[0])[c - V.lo];
    }
    cur[q] = nxt;
  }
}

// Reset the visited words of every vertex this search claimed (all of them are
// in the queues): no O(N) clear per search.
__global__ void k_cleanup(DView V) {
  for (int s = 0; s < 2; ++s) {
    const uint32_t qn = V.st->qtail[s];
    const uint32_t* q = pick(V.queue, s);
    uint32_t* vis = pick(V.vis, s);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < qn;
         i += (uint64_t)gridDim.x * blockDim.x)
      vis[(q[i] - V.lo) >> 5] = 0u;
  }
}

unsigned blocks_for(uint64_t work, int cus) {
  uint64_t b = (work + kThreads - 1) / kThreads;
  b = std::min<uint64_t>(b, (uint64_t)cus * 8);
  return (unsigned)std::max<uint64_t>(b, 1);
}

}  // namespace

std::vector<uint8_t> dist_unique_id() { return dist::rccl_unique_id(); }

struct DistBiBfs::Impl {
  int rank = 0, size = 1, device = 0, cus = 256;
  hipStream_t stream = nullptr;   // compute: pre phases, graph build
  hipStream_t cstream = nullptr;  // comm: exchanges, post phases, round end
  hipEvent_t ev_pre[2] = {nullptr, nullptr};
  hipEvent_t ev_round = nullptr;
  std::unique_ptr<dist::Comm> comm;
  uint32_t n = 0, lo = 0, hi = 0, chunk = 0, gwords = 0, cap = 0;
  uint64_t m_input = 0, nnz = 0;
  uint64_t* d_row_off = nullptr;
  uint32_t* d_col = nullptr;
  void* state = nullptr;
  uint32_t* sent_base = nullptr;  // both sides' sent bitmaps, contiguous (one memset)
  DView V{};
  uint32_t* d_cur = nullptr;
  uint32_t* d_pathS = nullptr;
  uint32_t* d_pathT = nullptr;
  Reduced* h_red = nullptr;  // pinned
  double* d_scalar = nullptr;
  DistLevelStats stats;

  void setup(int dev) {
    device = dev;
    rank = comm->rank();
    size = comm->size();
    HIP_CHECK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIP_CHECK(hipGetDeviceProperties(&prop, device));
    cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
    int lo_pri = 0, hi_pri = 0;
    HIP_CHECK(hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri));
    HIP_CHECK(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
    // the exchange path is the critical one: its stream gets the higher priority
    HIP_CHECK(hipStreamCreateWithPriority(&cstream, hipStreamNonBlocking, hi_pri));
    for (auto& e : ev_pre) HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&ev_round, hipEventDisableTiming));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red), sizeof(Reduced), hipHostMallocDefault));
  }

  void set_partition(uint32_t nn) {
    n = nn;
    const uint64_t per = ((uint64_t)nn + size - 1) / size;
    chunk = (uint32_t)std::max<uint64_t>(64, (per + 63) / 64 * 64);
    lo = (uint32_t)std::min<uint64_t>((uint64_t)rank * chunk, nn);
    hi = (uint32_t)std::min<uint64_t>((uint64_t)(rank + 1) * chunk, nn);
  }

  void free_all() {
    if (d_row_off) HIP_CHECK(hipFree(d_row_off));
    if (d_col) HIP_CHECK(hipFree(d_col));
    if (state) HIP_CHECK(hipFree(state));
    d_row_off = nullptr;
    d_col = nullptr;
    state = nullptr;
  }

  void alloc_state() {
    const uint64_t words = chunk / 32;
    gwords = (uint32_t)(((uint64_t)n + 31) / 32 + 1);
    cap = (uint32_t)std::min<uint64_t>(kCapMax, std::max<uint64_t>(n, 1));
    const uint64_t block = 2 + 2ULL * cap;
    size_t off = 0;
    auto take = [&](size_t bytes) {
      size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    size_t o_vis[2], o_par[2], o_dep[2], o_q[2], o_ob[2], o_gb[2], o_send[2], o_recv[2];
    for (int s = 0; s < 2; ++s) {
      o_vis[s] = take(words * 4);
      o_par[s] = take((size_t)chunk * 4);
      o_dep[s] = take((size_t)chunk * 4);
      o_q[s] = take((size_t)chunk * 4);
      o_ob[s] = take(words * 4);
      o_gb[s] = take(words * 4 * size);
      o_send[s] = take(block * 4);
      o_recv[s] = take(block * 4 * size);
    }
    const size_t o_sent = take((size_t)gwords * 4 * 2);
    const size_t o_st = take(sizeof(DState)), o_red = take(sizeof(Reduced)), o_cur = take(64),
                 o_ps = take(((size_t)n + 2) * 4), o_pt = take(((size_t)n + 2) * 4), o_sc = take(64);
    HIP_CHECK(hipMalloc(&state, off));
    char* b = static_cast<char*>(state);
    V.n = n;
    V.lo = lo;
    V.hi = hi;
    V.chunk = chunk;
    V.row_off = d_row_off;
    V.col = d_col;
    sent_base = reinterpret_cast<uint32_t*>(b + o_sent);
    for (int s = 0; s < 2; ++s) {
      V.vis[s] = reinterpret_cast<uint32_t*>(b + o_vis[s]);
      V.parent[s] = reinterpret_cast<uint32_t*>(b + o_par[s]);
      V.depth[s] = reinterpret_cast<uint32_t*>(b + o_dep[s]);
      V.queue[s] = reinterpret_cast<uint32_t*>(b + o_q[s]);
      V.obits[s] = reinterpret_cast<uint32_t*>(b + o_ob[s]);
      V.gbits[s] = reinterpret_cast<uint32_t*>(b + o_gb[s]);
      V.send[s] = reinterpret_cast<uint32_t*>(b + o_send[s]);
      V.recv[s] = reinterpret_cast<uint32_t*>(b + o_recv[s]);
      V.sent[s] = sent_base + (size_t)s * gwords;
      HIP_CHECK(hipMemsetAsync(V.vis[s], 0, words * 4, stream));
    }
    HIP_CHECK(hipMemsetAsync(sent_base, 0, (size_t)gwords * 4 * 2, stream));
    V.cap = cap;
    V.P = size;
    V.st = reinterpret_cast<DState*>(b + o_st);
    V.red = reinterpret_cast<Reduced*>(b + o_red);
    d_cur = reinterpret_cast<uint32_t*>(b + o_cur);
    d_pathS = reinterpret_cast<uint32_t*>(b + o_ps);
    d_pathT = reinterpret_cast<uint32_t*>(b + o_pt);
    d_scalar = reinterpret_cast<double*>(b + o_sc);
    HIP_CHECK(hipMemsetAsync(V.st, 0, sizeof(DState), stream));
    HIP_CHECK(hipMemsetAsync(d_scalar, 0, 64, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
  }

  void build_rows_from_device_edges(const uint32_t* d_uv, uint64_t m) {
    HIP_CHECK(hipMalloc(&d_row_off, ((size_t)(hi - lo) + 1) * 8));
    nnz = launch::count_csr_rows(d_uv, m, lo, hi, d_row_off, stream);
    HIP_CHECK(hipMalloc(&d_col, std::max<uint64_t>(nnz, 1) * 4));
    uint64_t* cursor = nullptr;
    HIP_CHECK(hipMalloc(&cursor, ((size_t)(hi - lo) + 1) * 8));
    launch::fill_csr_rows(d_uv, m, lo, hi, d_row_off, cursor, d_col, stream);
    HIP_CHECK(hipStreamSynchronize(stream));
    HIP_CHECK(hipFree(cursor));
  }

  void upload_rows(const Csr& rows) {
    HIP_CHECK(hipMalloc(&d_row_off, ((size_t)rows.n + 1) * 8));
    HIP_CHECK(hipMalloc(&d_col, std::max<uint64_t>(rows.nnz(), 1) * 4));
    HIP_CHECK(hipMemcpyAsync(d_row_off, rows.row_off.data(), ((size_t)rows.n + 1) * 8, hipMemcpyHostToDevice,
                             stream));
    if (rows.nnz())
      HIP_CHECK(hipMemcpyAsync(d_col, rows.col.data(), rows.nnz() * 4, hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    nnz = rows.nnz();
  }

  void read_back(hipStream_t s) {
    HIP_CHECK(hipMemcpyAsync(h_red, V.red, sizeof(Reduced), hipMemcpyDeviceToHost, s));
    HIP_CHECK(hipStreamSynchronize(s));
  }
};

DistBiBfs::DistBiBfs(int rank, int size, int device, const std::vector<uint8_t>& uid) : p_(new Impl) {
  HIP_CHECK(hipSetDevice(device));
  p_->comm = dist::make_rccl_comm(rank, size, uid);
  p_->setup(device);
}

DistBiBfs::DistBiBfs(std::unique_ptr<dist::Comm> comm, int device) : p_(new Impl) {
  HIP_CHECK(hipSetDevice(device));
  p_->comm = std::move(comm);
  p_->setup(device);
}

DistBiBfs::~DistBiBfs() {
  if (!p_) return;
  try {
    (void)hipSetDevice(p_->device);
    (void)hipStreamSynchronize(p_->stream);
    (void)hipStreamSynchronize(p_->cstream);
    p_->free_all();
  } catch (...) {
  }
  p_->comm.reset();
  (void)hipHostFree(p_->h_red);
  for (auto e : p_->ev_pre) (void)hipEventDestroy(e);
  (void)hipEventDestroy(p_->ev_round);
  (void)hipStreamDestroy(p_->cstream);
  (void)hipStreamDestroy(p_->stream);
}

void DistBiBfs::load_edges(const EdgeList& el) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.free_all();
  I.set_partition(el.n);
  I.m_input = el.m();
  Partition part;
  part.rank = I.rank;
  part.size = I.size;
  part.n = el.n;
  part.lo = I.lo;
  part.hi = I.hi;
  I.upload_rows(build_csr_rows(el, part));
  I.alloc_state();
}

void DistBiBfs::load_bin(const std::string& path) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.free_all();
  const BinHeader h = read_bin_header(path);
  I.set_partition(h.n);
  I.m_input = h.m;
  EdgeList shard = read_bin_shard(path, I.lo, I.hi);
  Partition part;
  part.rank = I.rank;
  part.size = I.size;
  part.n = h.n;
  part.lo = I.lo;
  part.hi = I.hi;
  I.upload_rows(build_csr_rows(shard, part));
  I.alloc_state();
}

void DistBiBfs::generate_gnp(uint32_t n, double p, uint64_t seed) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.free_all();
  I.set_partition(n);
  uint32_t* d_uv = nullptr;
  I.m_input = launch::gen_gnp_device(n, p, seed, &d_uv, I.stream);
  I.build_rows_from_device_edges(d_uv, I.m_input);
  HIP_CHECK(hipFree(d_uv));
  I.alloc_state();
}

void DistBiBfs::generate_rmat(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.free_all();
  I.set_partition(n);
  uint32_t* d_uv = nullptr;
  HIP_CHECK(hipMalloc(&d_uv, std::max<uint64_t>(2 * m, 2) * 4));
  launch::gen_rmat_device(n, m, seed, a, b, c, d_uv, I.stream);
  I.m_input = m;
  I.build_rows_from_device_edges(d_uv, m);
  HIP_CHECK(hipFree(d_uv));
  I.alloc_state();
}

SearchResult DistBiBfs::search(vid_t src, vid_t dst, const SearchOptions& opt) {
  auto& I = *p_;
  auto& V = I.V;
  const auto t0 = std::chrono::steady_clock::now();
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  BIBFS_REQUIRE(src < I.n && dst < I.n, "src/dst out of range");
  HIP_CHECK(hipSetDevice(I.device));
  I.stats = DistLevelStats{};
  SearchResult r;
  if (src == dst) {
    r.found = true;
    r.hops = 0;
    r.meet = src;
    r.path = {src};
    r.stats.visited = 1;
    r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return r;
  }
  const int cus = I.cus, P = I.size;
  hipStream_t ps = I.stream, cs = I.cstream;
  dist::Comm& comm = *I.comm;
  const uint32_t words = I.chunk / 32, nloc = I.hi - I.lo;

  k_seed<<<1, 64, 0, cs>>>(V, src, dst);
  comm.allreduce(V.red->sums, 4, DType::kU64, ROp::kSum, cs);
  HIP_CHECK(hipEventRecord(I.ev_round, cs));
  I.read_back(cs);
  // replicated host bookkeeping (identical on every rank)
  uint64_t cnt[2] = {1, 1}, fed[2] = {I.h_red->sums[1], I.h_red->sums[3]};
  uint64_t ved[2] = {fed[0], fed[1]};
  int depth[2] = {0, 0}, dir[2] = {1, 1}, turn = 0;
  const uint64_t nnz_total = 2 * I.m_input;
  unsigned long long key = kNoKey;
  bool dead = false;
  for (uint64_t guard = 0; guard <= 2ULL * I.n + 2 && key == kNoKey && !dead; ++guard) {
    const auto tr0 = std::chrono::steady_clock::now();
    // ---- which sides expand this round
    int sides[2] = {0, 1}, ns = 1;
    const uint64_t flo = std::min(fed[0], fed[1]), fhi = std::max(fed[0], fed[1]);
    if (opt.lockstep && opt.side != SidePolicy::kAlternate && (fhi <= kLockstepEdges || fhi <= 2 * flo)) {
      ns = 2;
    } else if (opt.side == SidePolicy::kAlternate) {
      sides[0] = turn;
      turn ^= 1;
    } else if (opt.side == SidePolicy::kSmallerFrontier) {
      sides[0] = cnt[0] <= cnt[1] ? 0 : 1;
    } else {
      sides[0] = fed[0] <= fed[1] ? 0 : 1;
    }
    int mode[2] = {1, 1};  // 1 top-down, 2 bottom-up
    for (int i = 0; i < ns; ++i) {
      const int s = sides[i];
      if (opt.direction == Direction::kTopDown) {
        mode[s] = 1;
      } else if (opt.direction == Direction::kBottomUp) {
        mode[s] = 2;
      } else {
        const double m_u = (double)nnz_total - (double)ved[s];
        if (dir[s] == 1 && (double)fed[s] > m_u / opt.alpha) dir[s] = 2;
        else if (dir[s] == 2 && (double)cnt[s] < (double)I.n / opt.beta) dir[s] = 1;
        mode[s] = dir[s];
      }
    }
    // ---- pre phases on the compute stream (behind the previous round)
    HIP_CHECK(hipStreamWaitEvent(ps, I.ev_round, 0));
    for (int i = 0; i < ns; ++i) {
      const int s = sides[i];
      const uint32_t dnew = (uint32_t)depth[s] + 1;
      const unsigned fblocks = blocks_for(cnt[s] / (uint64_t)P + kThreads, cus);
      if (mode[s] == 1) {
        k_td_expand<<<fblocks, kThreads, 0, ps>>>(V, s, dnew, i == 0);
        k_send_header<<<1, 64, 0, ps>>>(V, s);
      } else {
        HIP_CHECK(hipMemsetAsync(V.obits[s], 0, (size_t)words * 4, ps));
        k_obits<<<fblocks, kThreads, 0, ps>>>(V, s, i == 0);
      }
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipEventRecord(I.ev_pre[i], ps));
    }
    // ---- exchange + post phases on the comm stream: side 0's run while side
    // 1's pre phase is still computing on the other stream
    for (int i = 0; i < ns; ++i) {
      const int s = sides[i];
      const uint32_t dnew = (uint32_t)depth[s] + 1;
      HIP_CHECK(hipStreamWaitEvent(cs, I.ev_pre[i], 0));
      bool bottomup = mode[s] == 2;
      if (!bottomup) {
        uint64_t per;
        const uint64_t bound = std::min<uint64_t>(fed[s], I.cap);
        if (fed[s] <= I.cap && (2 + 2 * bound) * 4 * (uint64_t)P <= kNoSyncBytes) {
          per = bound;  // no rank emits more than the side's frontier edges: no count exchange
        } else {
          comm.allreduce(V.red->maxsend + s, 1, DType::kU32, ROp::kMax, cs);
          I.read_back(cs);
          per = I.h_red->maxsend[s];
          I.stats.count_syncs++;
          if (per > I.cap) {
            bottomup = true;  // finish the level bottom-up; the local claims made stay valid
            I.stats.overflow_levels++;
          }
        }
        if (!bottomup) {
          I.stats.sparse_levels++;
          if (per > 0) {
            const uint64_t blk = 2 + 2 * per;
            comm.allgather(V.send[s], V.recv[s], blk * 4, cs);
            k_td_claim<<<blocks_for((uint64_t)P * per, cus), kThreads, 0, cs>>>(V, s, (uint32_t)per, dnew);
            I.stats.exchanged_bytes += blk * 4 * (uint64_t)P;
          }
        } else {
          HIP_CHECK(hipMemsetAsync(V.obits[s], 0, (size_t)words * 4, cs));
          k_obits<<<blocks_for(cnt[s] / (uint64_t)P + kThreads, cus), kThreads, 0, cs>>>(V, s, 0);
        }
      }
      if (bottomup) {
        I.stats.dense_levels++;
        comm.allgather(V.obits[s], V.gbits[s], (size_t)words * 4, cs);
        k_bu<<<blocks_for(nloc, cus), kThreads, 0, cs>>>(V, s, dnew);
        I.stats.exchanged_bytes += (uint64_t)words * 4 * P;
        ++r.stats.bottomup_levels;
      }
      HIP_CHECK(hipGetLastError());
      r.stats.edges_inspected += fed[s];
      ++r.stats.levels;
    }
    int mask = 0;
    for (int i = 0; i < ns; ++i) {
      const int s = sides[i];
      k_meet<<<blocks_for(std::min<uint64_t>(fed[s], nloc), cus), kThreads, 0, cs>>>(V, s, (uint32_t)depth[s] + 1);
      mask |= 1 << s;
    }
    k_round_end<<<1, 64, 0, cs>>>(V, mask);
    HIP_CHECK(hipGetLastError());
    comm.group_begin();
    comm.allreduce(V.red->sums, 4, DType::kU64, ROp::kSum, cs);
    comm.allreduce(&V.red->meetkey, 1, DType::kU64, ROp::kMin, cs);
    comm.group_end();
    HIP_CHECK(hipEventRecord(I.ev_round, cs));
    I.read_back(cs);
    I.stats.rounds++;
    if (ns == 2) I.stats.lockstep_rounds++;
    I.stats.levels += ns;
    I.stats.comm_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tr0).count();
    for (int i = 0; i < ns; ++i) ++depth[sides[i]];
    key = I.h_red->meetkey;
    if (key != kNoKey) break;
    for (int i = 0; i < ns; ++i) {
      const int s = sides[i];
      cnt[s] = I.h_red->sums[2 * s];
      fed[s] = I.h_red->sums[2 * s + 1];
      ved[s] += fed[s];
      if (cnt[s] == 0) dead = true;  // that side's component is exhausted without a meet
    }
  }
  if (key != kNoKey) {
    const uint32_t meet = (uint32_t)(key & 0xffffffffull);
    r.found = true;
    r.meet = meet;
    r.hops = (int64_t)(key >> 32);
    if (opt.want_path) {
      k_meet_depth<<<1, 64, 0, cs>>>(V, meet);
      comm.allreduce(V.red->md, 2, DType::kU32, ROp::kMin, cs);
      I.read_back(cs);
      const int dS = (int)I.h_red->md[0], dT = (int)I.h_red->md[1];
      BIBFS_REQUIRE((int64_t)dS + dT == r.hops, "dist: meet depths disagree with the path length");
      const int K = std::max(dS, dT);
      const uint32_t init[2] = {meet, meet};
      HIP_CHECK(hipMemcpyAsync(I.d_cur, init, 8, hipMemcpyHostToDevice, cs));
      for (int i = 0; i <= K; ++i) {
        k_path_step<<<1, 64, 0, cs>>>(V, I.d_cur, I.d_pathS, I.d_pathT, i, dS, dT);
        if (i < K) comm.allreduce(I.d_cur, 2, DType::kU32, ROp::kMin, cs);
      }
      std::vector<uint32_t> pS((size_t)dS + 1), pT((size_t)dT + 1);
      HIP_CHECK(hipMemcpyAsync(pS.data(), I.d_pathS, pS.size() * 4, hipMemcpyDeviceToHost, cs));
      HIP_CHECK(hipMemcpyAsync(pT.data(), I.d_pathT, pT.size() * 4, hipMemcpyDeviceToHost, cs));
      HIP_CHECK(hipStreamSynchronize(cs));
      r.path.assign(pS.rbegin(), pS.rend());
      r.path.insert(r.path.end(), pT.begin() + 1, pT.end());
    }
  }
  k_cleanup<<<blocks_for(I.chunk, cus), kThreads, 0, cs>>>(V);
  HIP_CHECK(hipMemsetAsync(I.sent_base, 0, (size_t)I.gwords * 4 * 2, cs));
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipEventRecord(I.ev_round, cs));
  HIP_CHECK(hipStreamSynchronize(cs));
  r.stats.grid_levels = r.stats.levels;
  r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  r.search_ms = r.total_ms;
  return r;
}

void DistBiBfs::barrier() {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.comm->allreduce(I.d_scalar, 1, DType::kF64, ROp::kMax, I.cstream);
  HIP_CHECK(hipStreamSynchronize(I.cstream));
}

double DistBiBfs::allreduce_max(double x) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  double y = x;
  HIP_CHECK(hipMemcpyAsync(I.d_scalar, &y, 8, hipMemcpyHostToDevice, I.cstream));
  I.comm->allreduce(I.d_scalar, 1, DType::kF64, ROp::kMax, I.cstream);
  HIP_CHECK(hipMemcpyAsync(&y, I.d_scalar, 8, hipMemcpyDeviceToHost, I.cstream));
  HIP_CHECK(hipStreamSynchronize(I.cstream));
  return y;
}

int DistBiBfs::rank() const { return p_->rank; }
int DistBiBfs::size() const { return p_->size; }
uint32_t DistBiBfs::n() const { return p_->n; }
uint64_t DistBiBfs::m_input() const { return p_->m_input; }
uint64_t DistBiBfs::local_nnz() const { return p_->nnz; }
uint32_t DistBiBfs::lo() const { return p_->lo; }
uint32_t DistBiBfs::hi() const { return p_->hi; }
const DistLevelStats& DistBiBfs::last_stats() const { return p_->stats; }
const char* DistBiBfs::backend() const { return p_->comm->name(); }

namespace {

// Runs `body(engine, rank, results)` on `ranks` threads, each with a DistBiBfs
// on `device` over one in-process local group.  A failing rank aborts the
// group (so peers blocked in a collective return); its own message is thrown.
// Returns rank 0's results after checking that every rank agrees.
template <typename Body>
std::vector<SearchResult> run_local_ranks(const char* who, int ranks, int device, size_t nq, Body&& body) {
  BIBFS_REQUIRE(ranks >= 1 && ranks <= 16, std::string(who) + ": 1..16 ranks");
  auto group = dist::make_local_group(ranks);
  std::vector<std::vector<SearchResult>> out((size_t)ranks);
  std::vector<std::string> err((size_t)ranks);
  std::vector<std::thread> th;
  for (int r = 0; r < ranks; ++r)
    th.emplace_back([&, r] {
      try {
        DistBiBfs e(dist::make_local_comm(group, r), device);
        body(e, r, out[(size_t)r]);
      } catch (const std::exception& ex) {
        err[(size_t)r] = ex.what();
        dist::abort_local_group(*group);
      }
    });
  for (auto& t : th) t.join();
  for (int pass = 0; pass < 2; ++pass)  // the failing rank's own message before the others' "aborted"
    for (int r = 0; r < ranks; ++r)
      if (!err[(size_t)r].empty() && (pass == 1 || err[(size_t)r].find("aborted") == std::string::npos))
        throw Error(std::string(who) + " rank " + std::to_string(r) + ": " + err[(size_t)r]);
  for (int r = 1; r < ranks; ++r)
    for (size_t i = 0; i < nq; ++i)
      BIBFS_REQUIRE(out[(size_t)r][i].hops == out[0][i].hops && out[(size_t)r][i].path == out[0][i].path,
                    std::string(who) + ": ranks returned different results");
  return std::move(out[0]);
}

}  // namespace

std::vector<SearchResult> dist_local_run(int ranks, int device, const EdgeList& el,
                                         const std::vector<std::pair<vid_t, vid_t>>& queries,
                                         const SearchOptions& opt) {
  return run_local_ranks("dist_local_run", ranks, device, queries.size(),
                         [&](DistBiBfs& e, int, std::vector<SearchResult>& out) {
                           e.load_edges(el);
                           for (const auto& q : queries) out.push_back(e.search(q.first, q.second, opt));
                         });
}

std::vector<SearchResult> dist_local_generate_run(int ranks, int device, const std::string& kind, uint32_t n,
                                                  double arg, uint64_t seed,
                                                  const std::vector<std::pair<vid_t, vid_t>>& queries,
                                                  const SearchOptions& opt, DistLocalTiming* timing) {
  BIBFS_REQUIRE(kind == "gnp" || kind == "rmat", "dist_local_generate_run: kind must be gnp or rmat");
  std::vector<double> build_ms((size_t)std::max(ranks, 1), 0.0), qms;
  std::vector<uint64_t> nnz((size_t)std::max(ranks, 1), 0);
  std::vector<DistLevelStats> qstats;
  auto rs = run_local_ranks(
      "dist_local_generate_run", ranks, device, queries.size(),
      [&](DistBiBfs& e, int r, std::vector<SearchResult>& out) {
        const auto t0 = std::chrono::steady_clock::now();
        if (kind == "gnp")
          e.generate_gnp(n, arg, seed);
        else
          e.generate_rmat(n, (uint64_t)arg, seed);  // ends with hipFree of the edge list: synchronous
        build_ms[(size_t)r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        nnz[(size_t)r] = e.local_nnz();
        for (const auto& q : queries) {
          const auto q0 = std::chrono::steady_clock::now();
          out.push_back(e.search(q.first, q.second, opt));
          if (r == 0) {
            qms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - q0).count());
            qstats.push_back(e.last_stats());
          }
        }
      });
  if (timing) {
    timing->build_ms = *std::max_element(build_ms.begin(), build_ms.end());
    timing->query_ms = std::move(qms);
    timing->local_nnz = std::move(nnz);
    timing->stats = std::move(qstats);
  }
  return rs;
}

}  // namespace bibfs
