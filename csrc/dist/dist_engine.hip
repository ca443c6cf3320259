// Multi-GPU bidirectional BFS over RCCL (see include/bibfs/dist_engine.hpp).
//
// Reference parity: v4/mpi_bas.cpp:79-132 (per-level loop), v4/comp.cu:20-38
// (expand kernel with a vertex-ownership filter that the reference disabled
// by launching with rank=0,size=1, v4/comp.cu:99), and the collective sites
// of SURVEY.md §2.5 (MPI_Allreduce BOR over N ints per level, LOR flags).
// Here the ownership is real, the exchange is sparse when the frontier is
// small (allgather of candidates) and a bitmap when it is large (allgather of
// owned slices, N/8 bytes in total), and all state stays on the GPU.
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cstring>

#include "bibfs/dist_engine.hpp"
#include "bibfs/io.hpp"
#include "device.hpp"

namespace bibfs {

using namespace dev;

#define RCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess)                                                                \
      throw ::bibfs::Error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + \
                           __FILE__ + ":" + std::to_string(__LINE__));                    \
  } while (0)

namespace {

constexpr int kThreads = 256;

struct DState {
  uint32_t fbeg[2], fend[2], qtail[2];
  uint32_t send_count;
  uint32_t pad0;
  unsigned long long new_edges;  // degree sum of vertices claimed this level (owned)
  unsigned long long root_edges[2];
  uint32_t meet;                 // local meet candidate
  uint32_t pad1;
};

// reduced every level: [0] = new count (sum), [1] = new degree sum (sum)
struct Reduced {
  unsigned long long sums[2];
  uint32_t meet;  // min
  uint32_t maxsend;  // max
};

struct DView {
  uint32_t n, lo, hi, chunk;  // owned = [lo, hi), owner(v) = v / chunk
  const uint64_t* row_off;    // local rows
  const uint32_t* col;
  uint32_t* vis[2];           // owned slices (chunk/32 words)
  uint32_t* parent[2];        // chunk entries
  uint32_t* queue[2];         // chunk entries
  uint32_t* obits;            // owned frontier slice (chunk/32 words)
  const uint32_t* gbits;      // allgathered frontier bitmap (P * chunk/32 words)
  uint32_t* send;             // [count, pad, (v, u) pairs ...]
  const uint32_t* recv;       // P blocks of `block` u32
  uint32_t cap;               // candidate capacity per rank
  uint32_t block;             // u32 per rank block in recv
  int P;
  DState* st;
  Reduced* red;
};

__device__ __forceinline__ uint32_t* pick(uint32_t* const* a, int s) { return s ? a[1] : a[0]; }

// Claim owned vertex v (global id) for side s from parent u.  Returns true if new.
__device__ __forceinline__ bool claim_local(const DView& V, int s, uint32_t v, uint32_t u) {
  const uint32_t li = v - V.lo;
  uint32_t* vis = s ? V.vis[1] : V.vis[0];
  const uint32_t bit = 1u << (li & 31);
  if (vis[li >> 5] & bit) return false;
  if (atomicOr(&vis[li >> 5], bit) & bit) return false;
  (s ? V.parent[1] : V.parent[0])[li] = u;
  const uint32_t pos = atomicAdd(&V.st->qtail[s], 1u);
  (s ? V.queue[1] : V.queue[0])[pos] = v;
  atomicAdd(&V.st->new_edges, (unsigned long long)(V.row_off[li + 1] - V.row_off[li]));
  const uint32_t* ovis = s ? V.vis[0] : V.vis[1];
  if (ovis[li >> 5] & bit) atomicMin(&V.st->meet, v);
  return true;
}

// Sparse expansion: one wave per owned frontier vertex, lanes over neighbours.
__global__ __launch_bounds__(kThreads) void k_td_expand(DView V, int s) {
  const uint32_t fb = V.st->fbeg[s], fe = V.st->fend[s];
  const uint32_t* q = s ? V.queue[1] : V.queue[0];
  const int lane = __lane_id();
  const uint64_t w0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64;
  const uint64_t ws = (uint64_t)gridDim.x * blockDim.x / 64;
  for (uint64_t i = fb + w0; i < fe; i += ws) {
    const uint32_t u = q[i];
    const uint32_t li = u - V.lo;
    const uint64_t b = V.row_off[li], e = V.row_off[li + 1];
    for (uint64_t k = b + lane; k < e; k += 64) {
      const uint32_t v = V.col[k];
      if (v >= V.lo && v < V.hi) {
        claim_local(V, s, v, u);
      } else {
        const uint32_t pos = atomicAdd(&V.st->send_count, 1u);
        if (pos < V.cap) {
          V.send[2 + 2 * pos] = v;
          V.send[3 + 2 * pos] = u;
        }
      }
    }
  }
}

// Owners claim the candidates addressed to them.
__global__ __launch_bounds__(kThreads) void k_td_claim(DView V, int s, uint32_t per_rank, uint32_t blk) {
  const uint64_t total = (uint64_t)V.P * per_rank;
  for (uint64_t t = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; t < total;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = (uint32_t)(t / per_rank), i = (uint32_t)(t % per_rank);
    const uint32_t* b = V.recv + (uint64_t)r * blk;
    if (i >= min(b[0], V.cap)) continue;
    const uint32_t v = b[2 + 2 * i];
    if (v >= V.lo && v < V.hi) claim_local(V, s, v, b[3 + 2 * i]);
  }
}

__global__ void k_obits(DView V, int s) {
  const uint32_t fb = V.st->fbeg[s], fe = V.st->fend[s];
  const uint32_t* q = s ? V.queue[1] : V.queue[0];
  for (uint64_t i = fb + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < fe;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t li = q[i] - V.lo;
    atomicOr(&V.obits[li >> 5], 1u << (li & 31));
  }
}

// Dense expansion: owners scan their unvisited vertices for a frontier parent.
__global__ __launch_bounds__(kThreads) void k_bu(DView V, int s) {
  const uint32_t nloc = V.hi - V.lo;
  const uint32_t* vis = s ? V.vis[1] : V.vis[0];
  for (uint64_t li = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; li < nloc;
       li += (uint64_t)gridDim.x * blockDim.x) {
    if (vis[li >> 5] & (1u << (li & 31))) continue;
    const uint64_t b = V.row_off[li], e = V.row_off[li + 1];
    for (uint64_t k = b; k < e; ++k) {
      const uint32_t u = V.col[k];
      if (V.gbits[u >> 5] & (1u << (u & 31))) {
        claim_local(V, s, V.lo + (uint32_t)li, u);
        break;
      }
    }
  }
}

__global__ void k_seed(DView V, uint32_t src, uint32_t dst) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DState* st = V.st;
  const uint32_t r[2] = {src, dst};
  for (int s = 0; s < 2; ++s) {
    st->fbeg[s] = 0;
    st->fend[s] = 0;
    st->qtail[s] = 0;
    st->root_edges[s] = 0;
    const uint32_t v = r[s];
    if (v >= V.lo && v < V.hi) {
      const uint32_t li = v - V.lo;
      (s ? V.vis[1] : V.vis[0])[li >> 5] |= 1u << (li & 31);
      (s ? V.parent[1] : V.parent[0])[li] = kEmpty;
      (s ? V.queue[1] : V.queue[0])[0] = v;
      st->fend[s] = 1;
      st->qtail[s] = 1;
      st->root_edges[s] = V.row_off[li + 1] - V.row_off[li];
    }
  }
  st->send_count = 0;
  st->new_edges = 0;
  st->meet = kEmpty;
  V.red->sums[0] = st->root_edges[0];
  V.red->sums[1] = st->root_edges[1];
  V.red->meet = kEmpty;
  V.red->maxsend = 0;
}

// Before the stats reduction: publish this rank's contribution.
__global__ void k_stats(DView V, int s) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DState* st = V.st;
  V.red->sums[0] = st->qtail[s] - st->fend[s];
  V.red->sums[1] = st->new_edges;
  V.red->meet = st->meet;
}

__global__ void k_send_header(DView V) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  V.send[0] = V.st->send_count;
  V.red->maxsend = V.st->send_count;
}

// Level bookkeeping, identical on every rank.
__global__ void k_advance(DView V, int s) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DState* st = V.st;
  st->fbeg[s] = st->fend[s];
  st->fend[s] = st->qtail[s];
  st->send_count = 0;
  st->new_edges = 0;
}

// Path reconstruction step: cur[q] -> parent (only the owner knows it; the
// others contribute UINT_MAX to the ncclMin that follows).
__global__ void k_path_step(DView V, uint32_t* cur, uint32_t* pathS, uint32_t* pathT, int i, int dS,
                            int dT) {
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

__global__ void k_cleanup(DView V) {
  for (int s = 0; s < 2; ++s) {
    const uint32_t q = V.st->qtail[s];
    const uint32_t* qq = s ? V.queue[1] : V.queue[0];
    uint32_t* vis = s ? V.vis[1] : V.vis[0];
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < q;
         i += (uint64_t)gridDim.x * blockDim.x)
      vis[(qq[i] - V.lo) >> 5] = 0u;
  }
}

unsigned blocks_for(uint64_t work, int cus) {
  uint64_t b = (work + kThreads - 1) / kThreads;
  b = std::min<uint64_t>(b, (uint64_t)cus * 8);
  return (unsigned)std::max<uint64_t>(b, 1);
}

}  // namespace

std::vector<uint8_t> dist_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id));
}

struct DistBiBfs::Impl {
  int rank = 0, size = 1, device = 0, cus = 256;
  hipStream_t stream = nullptr;
  ncclComm_t comm = nullptr;
  uint32_t n = 0, lo = 0, hi = 0, chunk = 0;
  uint64_t m_input = 0, nnz = 0;
  uint64_t* d_row_off = nullptr;
  uint32_t* d_col = nullptr;
  void* state = nullptr;
  DView V{};
  uint32_t* d_cur = nullptr;
  uint32_t* d_pathS = nullptr;
  uint32_t* d_pathT = nullptr;
  Reduced* h_red = nullptr;  // pinned
  double* d_scalar = nullptr;
  DistLevelStats stats;
  uint32_t cap = 1u << 20;  // candidate pairs per rank per level

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
    const uint64_t block = 2 + 2ULL * cap;
    size_t off = 0;
    auto take = [&](size_t bytes) {
      size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    size_t o_vis[2], o_par[2], o_q[2];
    for (int s = 0; s < 2; ++s) {
      o_vis[s] = take(words * 4);
      o_par[s] = take((size_t)chunk * 4);
      o_q[s] = take((size_t)chunk * 4);
    }
    size_t o_ob = take(words * 4), o_gb = take(words * 4 * size), o_send = take(block * 4),
           o_recv = take(block * 4 * size), o_st = take(sizeof(DState)), o_red = take(sizeof(Reduced)),
           o_cur = take(64), o_ps = take(((size_t)n + 2) * 4), o_pt = take(((size_t)n + 2) * 4),
           o_sc = take(64);
    HIP_CHECK(hipMalloc(&state, off));
    char* b = static_cast<char*>(state);
    V.n = n;
    V.lo = lo;
    V.hi = hi;
    V.chunk = chunk;
    V.row_off = d_row_off;
    V.col = d_col;
    for (int s = 0; s < 2; ++s) {
      V.vis[s] = reinterpret_cast<uint32_t*>(b + o_vis[s]);
      V.parent[s] = reinterpret_cast<uint32_t*>(b + o_par[s]);
      V.queue[s] = reinterpret_cast<uint32_t*>(b + o_q[s]);
      HIP_CHECK(hipMemsetAsync(V.vis[s], 0, words * 4, stream));
    }
    V.obits = reinterpret_cast<uint32_t*>(b + o_ob);
    V.gbits = reinterpret_cast<uint32_t*>(b + o_gb);
    V.send = reinterpret_cast<uint32_t*>(b + o_send);
    V.recv = reinterpret_cast<uint32_t*>(b + o_recv);
    V.cap = cap;
    V.block = (uint32_t)block;
    V.P = size;
    V.st = reinterpret_cast<DState*>(b + o_st);
    V.red = reinterpret_cast<Reduced*>(b + o_red);
    d_cur = reinterpret_cast<uint32_t*>(b + o_cur);
    d_pathS = reinterpret_cast<uint32_t*>(b + o_ps);
    d_pathT = reinterpret_cast<uint32_t*>(b + o_pt);
    d_scalar = reinterpret_cast<double*>(b + o_sc);
    HIP_CHECK(hipMemsetAsync(V.st, 0, sizeof(DState), stream));
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

  // grouped allreduce of the level stats + host read-back
  void reduce_stats() {
    RCCL_CHECK(ncclGroupStart());
    RCCL_CHECK(ncclAllReduce(V.red->sums, V.red->sums, 2, ncclUint64, ncclSum, comm, stream));
    RCCL_CHECK(ncclAllReduce(&V.red->meet, &V.red->meet, 1, ncclUint32, ncclMin, comm, stream));
    RCCL_CHECK(ncclGroupEnd());
    HIP_CHECK(hipMemcpyAsync(h_red, V.red, sizeof(Reduced), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
  }
};

DistBiBfs::DistBiBfs(int rank, int size, int device, const std::vector<uint8_t>& uid) : p_(new Impl) {
  auto& I = *p_;
  I.rank = rank;
  I.size = size;
  I.device = device;
  BIBFS_REQUIRE(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
  HIP_CHECK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIP_CHECK(hipGetDeviceProperties(&prop, device));
  I.cus = prop.multiProcessorCount > 0 ? prop.multiProcessorCount : 256;
  HIP_CHECK(hipStreamCreateWithFlags(&I.stream, hipStreamNonBlocking));
  ncclUniqueId id;
  std::memcpy(&id, uid.data(), sizeof(id));
  RCCL_CHECK(ncclCommInitRank(&I.comm, size, id, rank));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&I.h_red), sizeof(Reduced), hipHostMallocDefault));
}

DistBiBfs::~DistBiBfs() {
  if (!p_) return;
  try {
    (void)hipSetDevice(p_->device);
    (void)hipStreamSynchronize(p_->stream);
    p_->free_all();
  } catch (...) {
  }
  if (p_->comm) (void)ncclCommDestroy(p_->comm);
  (void)hipHostFree(p_->h_red);
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
  const int cus = I.cus;
  k_seed<<<1, 64, 0, I.stream>>>(V, src, dst);
  RCCL_CHECK(ncclAllReduce(V.red->sums, V.red->sums, 2, ncclUint64, ncclSum, I.comm, I.stream));
  HIP_CHECK(hipMemcpyAsync(I.h_red, V.red, sizeof(Reduced), hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  // replicated host bookkeeping (identical on every rank)
  uint64_t cnt[2] = {1, 1}, fed[2] = {I.h_red->sums[0], I.h_red->sums[1]}, ved[2] = {fed[0], fed[1]};
  int depth[2] = {0, 0}, dir[2] = {1, 1}, turn = 0;
  const uint64_t nnz_total = 2 * I.m_input;
  uint32_t meet = kEmpty;
  bool found = false;
  const uint32_t words = I.chunk / 32;
  for (uint64_t guard = 0; guard <= 2ULL * I.n + 2; ++guard) {
    int s;
    if (opt.side == SidePolicy::kAlternate) {
      s = turn;
      turn ^= 1;
    } else if (opt.side == SidePolicy::kSmallerFrontier) {
      s = cnt[0] <= cnt[1] ? 0 : 1;
    } else {
      s = fed[0] <= fed[1] ? 0 : 1;
    }
    int mode;
    if (opt.direction == Direction::kTopDown) mode = 1;
    else if (opt.direction == Direction::kBottomUp) mode = 2;
    else {
      const double m_u = (double)nnz_total - (double)ved[s];
      if (dir[s] == 1 && (double)fed[s] > m_u / opt.alpha) dir[s] = 2;
      else if (dir[s] == 2 && (double)cnt[s] < (double)I.n / opt.beta) dir[s] = 1;
      mode = dir[s];
    }
    r.stats.edges_inspected += fed[s];
    const auto tc0 = std::chrono::steady_clock::now();
    if (mode == 1) {
      k_td_expand<<<blocks_for(cnt[s] * 64 / std::max(1, I.size) + 64, cus), kThreads, 0, I.stream>>>(V, s);
      k_send_header<<<1, 64, 0, I.stream>>>(V);
      RCCL_CHECK(ncclAllReduce(&V.red->maxsend, &V.red->maxsend, 1, ncclUint32, ncclMax, I.comm, I.stream));
      HIP_CHECK(hipMemcpyAsync(I.h_red, V.red, sizeof(Reduced), hipMemcpyDeviceToHost, I.stream));
      HIP_CHECK(hipStreamSynchronize(I.stream));
      const uint32_t maxc = I.h_red->maxsend;
      if (maxc > I.cap) {
        mode = 2;  // candidates overflowed: finish this level bottom-up (local claims already made stay valid)
        I.stats.overflow_levels++;
      } else {
        I.stats.sparse_levels++;
        if (maxc > 0) {
          // sized to the largest contribution, not to the capacity
          const uint32_t blk = 2 + 2 * maxc;
          RCCL_CHECK(ncclAllGather(V.send, const_cast<uint32_t*>(V.recv), blk, ncclUint32, I.comm, I.stream));
          k_td_claim<<<blocks_for((uint64_t)maxc * I.size, cus), kThreads, 0, I.stream>>>(V, s, maxc, blk);
          I.stats.candidates_sent += 0;
        }
      }
    }
    if (mode == 2) {
      I.stats.dense_levels++;
      HIP_CHECK(hipMemsetAsync(V.obits, 0, (size_t)words * 4, I.stream));
      k_obits<<<blocks_for(cnt[s], cus), kThreads, 0, I.stream>>>(V, s);
      RCCL_CHECK(ncclAllGather(V.obits, const_cast<uint32_t*>(V.gbits), words, ncclUint32, I.comm, I.stream));
      k_bu<<<blocks_for(I.hi - I.lo, cus), kThreads, 0, I.stream>>>(V, s);
    }
    k_stats<<<1, 64, 0, I.stream>>>(V, s);
    I.reduce_stats();
    I.stats.comm_ms += std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tc0).count();
    I.stats.levels++;
    r.stats.levels++;
    ++depth[s];
    const uint64_t ncnt = I.h_red->sums[0], nedg = I.h_red->sums[1];
    if (I.h_red->meet != kEmpty) {
      found = true;
      meet = I.h_red->meet;
      k_advance<<<1, 64, 0, I.stream>>>(V, s);
      break;
    }
    if (ncnt == 0) {
      k_advance<<<1, 64, 0, I.stream>>>(V, s);
      break;
    }
    k_advance<<<1, 64, 0, I.stream>>>(V, s);
    cnt[s] = ncnt;
    fed[s] = nedg;
    ved[s] += nedg;
  }
  if (found) {
    r.found = true;
    r.meet = meet;
    r.hops = depth[0] + depth[1];
    if (opt.want_path) {
      const int dS = depth[0], dT = depth[1], K = std::max(dS, dT);
      uint32_t init[2] = {meet, meet};
      HIP_CHECK(hipMemcpyAsync(I.d_cur, init, 8, hipMemcpyHostToDevice, I.stream));
      for (int i = 0; i <= K; ++i) {
        k_path_step<<<1, 64, 0, I.stream>>>(V, I.d_cur, I.d_pathS, I.d_pathT, i, dS, dT);
        if (i < K) RCCL_CHECK(ncclAllReduce(I.d_cur, I.d_cur, 2, ncclUint32, ncclMin, I.comm, I.stream));
      }
      std::vector<uint32_t> ps(dS + 1), pt(dT + 1);
      HIP_CHECK(hipMemcpyAsync(ps.data(), I.d_pathS, ps.size() * 4, hipMemcpyDeviceToHost, I.stream));
      HIP_CHECK(hipMemcpyAsync(pt.data(), I.d_pathT, pt.size() * 4, hipMemcpyDeviceToHost, I.stream));
      HIP_CHECK(hipStreamSynchronize(I.stream));
      r.path.assign(ps.rbegin(), ps.rend());
      r.path.insert(r.path.end(), pt.begin() + 1, pt.end());
    }
  }
  k_cleanup<<<blocks_for(I.chunk, cus), kThreads, 0, I.stream>>>(V);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(I.stream));
  r.stats.grid_levels = I.stats.levels;
  r.stats.bottomup_levels = I.stats.dense_levels;
  r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  r.search_ms = r.total_ms;
  return r;
}

void DistBiBfs::barrier() {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  RCCL_CHECK(ncclAllReduce(I.d_scalar, I.d_scalar, 1, ncclFloat64, ncclMax, I.comm, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
}

double DistBiBfs::allreduce_max(double x) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  double y = x;
  HIP_CHECK(hipMemcpyAsync(I.d_scalar, &y, 8, hipMemcpyHostToDevice, I.stream));
  RCCL_CHECK(ncclAllReduce(I.d_scalar, I.d_scalar, 1, ncclFloat64, ncclMax, I.comm, I.stream));
  HIP_CHECK(hipMemcpyAsync(&y, I.d_scalar, 8, hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
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

}  // namespace bibfs
