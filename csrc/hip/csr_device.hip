// Device-side graph ingest for MI355X: CSR build from an edge list
// (degree histogram -> exclusive scan -> scatter) and counter-based graph
// generators (G(n,p), R-MAT/Kronecker) whose output is bit-identical to the
// host generators in csrc/gen/gen.cpp (shared code in include/bibfs/rng.hpp).
//
// The reference builds its CSR on the host for every run
// (v3/bibfs_cuda_only.cu:89-99, v4/mpi_bas.cpp:45-57) with one fread per edge
// (v3:80-86); at 10M nodes that is ~3 s.  Here the edge list
// is copied once and the CSR is built by HBM-bandwidth kernels.
#include <vector>

#include "bibfs/rng.hpp"
#include "devmem.hpp"
#include "device.hpp"

namespace bibfs {
namespace {

constexpr int kScanThreads = 1024;
constexpr int kScanItems = 8;
constexpr uint64_t kScanTile = (uint64_t)kScanThreads * kScanItems;

// Rows [lo, hi) only (full graph: lo = 0, hi = n): the partitioned engine
// builds just its owned rows from the same edge stream.
__global__ void k_degree(const uint32_t* __restrict__ uv, uint64_t m, uint32_t lo, uint32_t hi,
                         uint64_t* __restrict__ deg) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 e = reinterpret_cast<const uint2*>(uv)[i];
    if (e.x == e.y) continue;  // self loops carry no BFS information
    if (e.x >= lo && e.x < hi) atomicAdd(reinterpret_cast<unsigned long long*>(&deg[e.x - lo]), 1ULL);
    if (e.y >= lo && e.y < hi) atomicAdd(reinterpret_cast<unsigned long long*>(&deg[e.y - lo]), 1ULL);
  }
}

// Block-wide inclusive scan of one value per thread (1024 threads = 16 waves).
__device__ uint64_t block_inclusive_scan(uint64_t x, uint64_t* wsum, uint64_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[wid] = x;
  __syncthreads();
  if (wid == 0) {
    uint64_t w = lane < (int)(blockDim.x >> 6) ? wsum[lane] : 0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint64_t y = __shfl_up(w, o);
      if (lane >= o) w += y;
    }
    if (lane < (int)(blockDim.x >> 6)) wsum[lane] = w;
  }
  __syncthreads();
  uint64_t r = x + (wid ? wsum[wid - 1] : 0);
  if (total) *total = wsum[(blockDim.x >> 6) - 1];
  __syncthreads();
  return r;
}

__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const uint64_t* __restrict__ d,
                                                              uint64_t count,
                                                              uint64_t* __restrict__ bsum) {
  __shared__ uint64_t wsum[16];
  const uint64_t base = blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k)
    if (base + k < count) s += d[base + k];
  uint64_t tot;
  block_inclusive_scan(s, wsum, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

// single block: exclusive scan of nb block sums (in place), any nb
__global__ __launch_bounds__(kScanThreads) void k_scan_bsums(uint64_t* __restrict__ bsum,
                                                             uint64_t nb) {
  __shared__ uint64_t wsum[16];
  uint64_t carry = 0;
  for (uint64_t base = 0; base < nb; base += kScanThreads) {
    const uint64_t i = base + threadIdx.x;
    uint64_t x = i < nb ? bsum[i] : 0;
    uint64_t tot;
    uint64_t inc = block_inclusive_scan(x, wsum, &tot);
    if (i < nb) bsum[i] = carry + inc - x;
    carry += tot;
  }
}

__global__ __launch_bounds__(kScanThreads) void k_scan_apply(uint64_t* __restrict__ d, uint64_t count,
                                                             const uint64_t* __restrict__ bsum) {
  __shared__ uint64_t wsum[16];
  const uint64_t base = blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanItems;
  uint64_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = (base + k < count) ? d[base + k] : 0;
    s += v[k];
  }
  uint64_t tot;
  uint64_t inc = block_inclusive_scan(s, wsum, &tot);
  uint64_t run = bsum[blockIdx.x] + inc - s;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    if (base + k < count) d[base + k] = run;
    run += v[k];
  }
}

// exclusive scan in place of count u64 values
void exclusive_scan_u64(uint64_t* d, uint64_t count, hipStream_t s) {
  const uint64_t nb = (count + kScanTile - 1) / kScanTile;
  uint64_t* bsum = nullptr;
  devmem::alloc(&bsum, (nb + 1) * sizeof(uint64_t));  // (counted by the partitioned build's tracker)
  k_scan_reduce<<<(unsigned)nb, kScanThreads, 0, s>>>(d, count, bsum);
  k_scan_bsums<<<1, kScanThreads, 0, s>>>(bsum, nb);
  k_scan_apply<<<(unsigned)nb, kScanThreads, 0, s>>>(d, count, bsum);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(s));
  devmem::release(bsum, (nb + 1) * sizeof(uint64_t));
}

__global__ void k_scatter(const uint32_t* __restrict__ uv, uint64_t m, uint32_t lo, uint32_t hi,
                          unsigned long long* __restrict__ cursor, uint32_t* __restrict__ col) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < m;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 e = reinterpret_cast<const uint2*>(uv)[i];
    if (e.x == e.y) continue;
    if (e.x >= lo && e.x < hi) col[atomicAdd(&cursor[e.x - lo], 1ULL)] = e.y;
    if (e.y >= lo && e.y < hi) col[atomicAdd(&cursor[e.y - lo], 1ULL)] = e.x;
  }
}

__global__ void k_copy_u64(const uint64_t* __restrict__ a, uint64_t cnt, uint64_t* __restrict__ b) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < cnt;
       i += (uint64_t)gridDim.x * blockDim.x)
    b[i] = a[i];
}

__global__ void k_row32(const uint64_t* __restrict__ r, uint32_t n1, uint32_t* __restrict__ r32) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n1;
       i += (uint64_t)gridDim.x * blockDim.x)
    r32[i] = (uint32_t)r[i];
}

// Packed adjacency for the latency-bound search: entry k carries everything
// the expansion of edge k needs -- the neighbour id, its degree and its row
// base -- so a BFS level costs ONE dependent global load per edge instead of
// col[k] followed by row_off[col[k]].
__global__ void k_padj(const uint64_t* __restrict__ r, const uint32_t* __restrict__ col, uint64_t nnz,
                       uint4* __restrict__ pa) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nnz;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = col[k];
    const uint64_t b = r[v], e = r[v + 1];
    const uint64_t d = e - b;
    pa[k] = make_uint4(v, d > 0xffffffffull ? 0xffffffffu : (uint32_t)d, (uint32_t)b, (uint32_t)(b >> 32));
  }
}

// The same in 8 bytes (launch::pack8; the caller checked the bounds).
__global__ void k_padj8(const uint64_t* __restrict__ r, const uint32_t* __restrict__ col, uint64_t nnz,
                        unsigned long long* __restrict__ pa) {
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nnz;
       k += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = col[k];
    const uint64_t b = r[v];
    pa[k] = launch::pack8(v, b, r[v + 1] - b);
  }
}

unsigned grid_for(uint64_t work, int threads) {
  uint64_t b = (work + threads - 1) / threads;
  if (b > 8192) b = 8192;  // 32 blocks per CU on 256 CUs, grid-stride beyond
  if (b < 1) b = 1;
  return (unsigned)b;
}

// ---------------------------------------------------------------- generators

__global__ void k_gnp_count(uint32_t n, double p, uint64_t seed, uint64_t nchunks,
                            uint64_t* __restrict__ cnt) {
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x)
    cnt[c] = gnp_walk_chunk(n, p, seed, nchunks, c, [](uint32_t, uint32_t) {});
}

__global__ void k_gnp_write(uint32_t n, double p, uint64_t seed, uint64_t nchunks,
                            const uint64_t* __restrict__ off, uint32_t* __restrict__ uv) {
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t pos = off[c];
    gnp_walk_chunk(n, p, seed, nchunks, c, [&](uint32_t v, uint32_t w) {
      uv[2 * pos] = w;
      uv[2 * pos + 1] = v;
      ++pos;
    });
  }
}

__global__ void k_rmat(RmatParams P, uint64_t m, uint32_t* __restrict__ uv) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < m;
       e += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u, v;
    rmat_edge(P, e, &u, &v);
    reinterpret_cast<uint2*>(uv)[e] = make_uint2(u, v);
  }
}

// ---- streamed generation of owned rows: the generators are pure functions of
// (seed, edge or chunk index), so a rank builds its CSR rows [lo, hi) in two
// passes over the stream -- degrees, then scatter -- and never materialises
// the edge list.  Peak memory is the shard itself (row offsets + columns) plus
// one cursor array, whatever the graph size (the reference broadcasts the
// whole edge list to every rank, v4/mpi_bas.cpp:29-64).
__device__ __forceinline__ void own_count(uint32_t x, uint32_t y, uint32_t lo, uint32_t hi, uint64_t* deg) {
  if (x == y) return;  // self loops carry no BFS information
  if (x >= lo && x < hi) atomicAdd(reinterpret_cast<unsigned long long*>(&deg[x - lo]), 1ULL);
  if (y >= lo && y < hi) atomicAdd(reinterpret_cast<unsigned long long*>(&deg[y - lo]), 1ULL);
}
__device__ __forceinline__ void own_scatter(uint32_t x, uint32_t y, uint32_t lo, uint32_t hi,
                                            unsigned long long* cursor, uint32_t* col) {
  if (x == y) return;
  if (x >= lo && x < hi) col[atomicAdd(&cursor[x - lo], 1ULL)] = y;
  if (y >= lo && y < hi) col[atomicAdd(&cursor[y - lo], 1ULL)] = x;
}

__global__ void k_rmat_degree(RmatParams P, uint64_t m, uint32_t lo, uint32_t hi, uint64_t* __restrict__ deg) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u, v;
    rmat_edge(P, e, &u, &v);
    own_count(u, v, lo, hi, deg);
  }
}
__global__ void k_rmat_scatter(RmatParams P, uint64_t m, uint32_t lo, uint32_t hi,
                               unsigned long long* __restrict__ cursor, uint32_t* __restrict__ col) {
  for (uint64_t e = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; e < m; e += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t u, v;
    rmat_edge(P, e, &u, &v);
    own_scatter(u, v, lo, hi, cursor, col);
  }
}
__global__ void k_gnp_degree(uint32_t n, double p, uint64_t seed, uint64_t nchunks, uint32_t lo, uint32_t hi,
                             uint64_t* __restrict__ deg, unsigned long long* __restrict__ medges) {
  unsigned long long mine = 0;
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x)
    mine += gnp_walk_chunk(n, p, seed, nchunks, c, [&](uint32_t v, uint32_t w) { own_count(w, v, lo, hi, deg); });
  if (mine) atomicAdd(medges, mine);
}
__global__ void k_gnp_scatter(uint32_t n, double p, uint64_t seed, uint64_t nchunks, uint32_t lo, uint32_t hi,
                              unsigned long long* __restrict__ cursor, uint32_t* __restrict__ col) {
  for (uint64_t c = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; c < nchunks;
       c += (uint64_t)gridDim.x * blockDim.x)
    gnp_walk_chunk(n, p, seed, nchunks, c, [&](uint32_t v, uint32_t w) { own_scatter(w, v, lo, hi, cursor, col); });
}

RmatParams rmat_params(uint32_t n, uint64_t seed, double a, double b, double c) {
  RmatParams P;
  P.n = n;
  P.scale = ceil_log2_u64(n);
  P.a = a;
  P.b = b;
  P.c = c;
  P.seed = seed;
  return P;
}

}  // namespace

namespace launch {

// Scan the degree array into row offsets, allocate the columns, run the
// scatter pass (`scatter(cursor, col)`); returns nnz.
template <class Scatter>
uint64_t finish_rows(uint32_t rows, uint64_t* d_row_off, uint32_t** d_col_out, hipStream_t s, Scatter scatter) {
  exclusive_scan_u64(d_row_off, rows + 1ULL, s);
  uint64_t nnz = 0;
  HIP_CHECK(hipMemcpyAsync(&nnz, d_row_off + rows, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  uint32_t* col = nullptr;
  devmem::alloc(&col, std::max<uint64_t>(nnz, 1) * 4);
  uint64_t* cursor = nullptr;
  devmem::alloc(&cursor, (rows + 1ULL) * 8);
  k_copy_u64<<<grid_for(rows + 1ULL, 256), 256, 0, s>>>(d_row_off, rows + 1ULL, cursor);
  scatter(reinterpret_cast<unsigned long long*>(cursor), col);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(s));
  devmem::release(cursor, (rows + 1ULL) * 8);
  *d_col_out = col;
  return nnz;
}

uint64_t gen_rows_rmat(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c, uint32_t lo, uint32_t hi,
                       uint64_t* d_row_off, uint32_t** d_col_out, hipStream_t s) {
  const RmatParams P = rmat_params(n, seed, a, b, c);
  const uint32_t rows = hi - lo;
  HIP_CHECK(hipMemsetAsync(d_row_off, 0, (rows + 1ULL) * 8, s));
  if (m) k_rmat_degree<<<grid_for(m, 256), 256, 0, s>>>(P, m, lo, hi, d_row_off);
  HIP_CHECK(hipGetLastError());
  return finish_rows(rows, d_row_off, d_col_out, s, [&](unsigned long long* cur, uint32_t* col) {
    if (m) k_rmat_scatter<<<grid_for(m, 256), 256, 0, s>>>(P, m, lo, hi, cur, col);
  });
}

uint64_t gen_rows_gnp(uint32_t n, double p, uint64_t seed, uint32_t lo, uint32_t hi, uint64_t* d_row_off,
                      uint32_t** d_col_out, uint64_t* m_out, hipStream_t s) {
  const uint64_t K = gnp_num_chunks(n, p);
  const uint32_t rows = hi - lo;
  unsigned long long* dm = nullptr;
  devmem::alloc(&dm, 8);
  HIP_CHECK(hipMemsetAsync(dm, 0, 8, s));
  HIP_CHECK(hipMemsetAsync(d_row_off, 0, (rows + 1ULL) * 8, s));
  k_gnp_degree<<<grid_for(K, 256), 256, 0, s>>>(n, p, seed, K, lo, hi, d_row_off, dm);
  HIP_CHECK(hipGetLastError());
  unsigned long long m = 0;
  HIP_CHECK(hipMemcpyAsync(&m, dm, 8, hipMemcpyDeviceToHost, s));
  const uint64_t nnz = finish_rows(rows, d_row_off, d_col_out, s, [&](unsigned long long* cur, uint32_t* col) {
    k_gnp_scatter<<<grid_for(K, 256), 256, 0, s>>>(n, p, seed, K, lo, hi, cur, col);
  });
  devmem::release(dm, 8);
  *m_out = m;
  return nnz;
}

uint64_t count_csr_rows(const uint32_t* d_uv, uint64_t m, uint32_t lo, uint32_t hi, uint64_t* d_row_off,
                        hipStream_t s) {
  const uint32_t n = hi - lo;
  HIP_CHECK(hipMemsetAsync(d_row_off, 0, (n + 1ULL) * sizeof(uint64_t), s));
  if (m) k_degree<<<grid_for(m, 256), 256, 0, s>>>(d_uv, m, lo, hi, d_row_off);
  HIP_CHECK(hipGetLastError());
  exclusive_scan_u64(d_row_off, n + 1ULL, s);
  uint64_t nnz = 0;
  HIP_CHECK(hipMemcpyAsync(&nnz, d_row_off + n, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return nnz;
}

uint64_t count_csr_entries(const uint32_t* d_uv, uint64_t m, uint32_t n, uint64_t* d_row_off,
                           hipStream_t s) {
  return count_csr_rows(d_uv, m, 0, n, d_row_off, s);
}

void fill_csr_rows(const uint32_t* d_uv, uint64_t m, uint32_t lo, uint32_t hi, const uint64_t* d_row_off,
                   uint64_t* d_cursor, uint32_t* d_col, hipStream_t s) {
  const uint32_t n = hi - lo;
  k_copy_u64<<<grid_for(n + 1ULL, 256), 256, 0, s>>>(d_row_off, n + 1ULL, d_cursor);
  if (m)
    k_scatter<<<grid_for(m, 256), 256, 0, s>>>(d_uv, m, lo, hi,
                                               reinterpret_cast<unsigned long long*>(d_cursor), d_col);
  HIP_CHECK(hipGetLastError());
}

void fill_csr(const uint32_t* d_uv, uint64_t m, uint32_t n, const uint64_t* d_row_off,
              uint64_t* d_cursor, uint32_t* d_col, hipStream_t s) {
  fill_csr_rows(d_uv, m, 0, n, d_row_off, d_cursor, d_col, s);
}

void build_padj8(const uint64_t* row_off, const uint32_t* col, uint64_t nnz, unsigned long long* padj8,
                 hipStream_t s) {
  if (nnz) k_padj8<<<grid_for(nnz, 256), 256, 0, s>>>(row_off, col, nnz, padj8);
  HIP_CHECK(hipGetLastError());
}

void build_padj(const uint64_t* row_off, const uint32_t* col, uint64_t nnz, uint4* padj, hipStream_t s) {
  if (nnz) k_padj<<<grid_for(nnz, 256), 256, 0, s>>>(row_off, col, nnz, padj);
  HIP_CHECK(hipGetLastError());
}

// Largest degree of the CSR (wave max, one atomic per wave).
__global__ void k_max_degree(const uint64_t* __restrict__ row_off, uint32_t n, unsigned long long* out) {
  unsigned long long m = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long d = row_off[i + 1] - row_off[i];
    m = d > m ? d : m;
  }
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long y = __shfl_xor(m, o);
    m = y > m ? y : m;
  }
  if (__lane_id() == 0 && m) atomicMax(out, m);
}

uint64_t max_degree(const uint64_t* d_row_off, uint32_t n, hipStream_t s) {
  unsigned long long* d = nullptr;
  devmem::alloc(&d, 8);
  HIP_CHECK(hipMemsetAsync(d, 0, 8, s));
  k_max_degree<<<(unsigned)std::min<uint64_t>(grid_for(n, 256), 2048), 256, 0, s>>>(d_row_off, n, d);
  HIP_CHECK(hipGetLastError());
  unsigned long long h = 0;
  HIP_CHECK(hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  devmem::release(d, 8);
  return h;
}

void make_row_off32(const uint64_t* d_row_off, uint32_t n, uint32_t* d_row_off32, hipStream_t s) {
  k_row32<<<grid_for(n + 1ULL, 256), 256, 0, s>>>(d_row_off, n + 1, d_row_off32);
  HIP_CHECK(hipGetLastError());
}

uint64_t gen_gnp_device(uint32_t n, double p, uint64_t seed, uint32_t** d_uv_out, hipStream_t s) {
  const uint64_t K = gnp_num_chunks(n, p);
  uint64_t* cnt = nullptr;
  HIP_CHECK(hipMalloc(&cnt, (K + 1) * sizeof(uint64_t)));
  HIP_CHECK(hipMemsetAsync(cnt, 0, (K + 1) * sizeof(uint64_t), s));
  k_gnp_count<<<grid_for(K, 256), 256, 0, s>>>(n, p, seed, K, cnt);
  HIP_CHECK(hipGetLastError());
  exclusive_scan_u64(cnt, K + 1, s);
  uint64_t total = 0;
  HIP_CHECK(hipMemcpyAsync(&total, cnt + K, sizeof(uint64_t), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  uint32_t* uv = nullptr;
  HIP_CHECK(hipMalloc(&uv, (2 * total + 2) * sizeof(uint32_t)));
  k_gnp_write<<<grid_for(K, 256), 256, 0, s>>>(n, p, seed, K, cnt, uv);
  HIP_CHECK(hipGetLastError());
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipFree(cnt));
  *d_uv_out = uv;
  return total;
}

void gen_rmat_device(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c,
                     uint32_t* d_uv, hipStream_t s) {
  const RmatParams P = rmat_params(n, seed, a, b, c);
  if (m) k_rmat<<<grid_for(m, 256), 256, 0, s>>>(P, m, d_uv);
  HIP_CHECK(hipGetLastError());
}

}  // namespace launch
}  // namespace bibfs
