// Internal header shared by the HIP translation units of the engine.
// gfx950 / CDNA4 only: wave64 everywhere, 64-bit ballots.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <string>

#include "bibfs/common.hpp"

namespace bibfs {
// Environment switches of the engines -- diagnostics and one memory budget.
// Every other setting is an API property (HipBiBfs setters, DistTuning).
namespace env {
// BIBFS_STAMP: cycle stamps (traced LDS / grid searches, the partitioned
// engine's solo workgroup); BIBFS_STAMP_SERVER: the resident LDS server's
// stamped build; BIBFS_TINY_STAMP: the tiny server's stamped build.
inline bool stamps() {
  static const bool on = std::getenv("BIBFS_STAMP") != nullptr;
  return on;
}
inline bool server_stamps() {
  static const bool on = std::getenv("BIBFS_STAMP_SERVER") != nullptr;
  return on;
}
inline bool tiny_stamps() {
  static const bool on = std::getenv("BIBFS_TINY_STAMP") != nullptr;
  return on;
}
// BIBFS_PADJ_MAX_MB: HBM budget of the packed adjacency (16 or 8 B per
// directed edge beside the CSR; default 4096 MiB, 0 = none).
inline uint64_t padj_budget_bytes() {
  static const uint64_t b = [] {
    const char* e = std::getenv("BIBFS_PADJ_MAX_MB");
    return (e ? std::strtoull(e, nullptr, 10) : 4096ull) << 20;
  }();
  return b;
}
}  // namespace env

namespace dev {

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess)                                                                 \
      throw ::bibfs::Error(std::string("HIP error ") + hipGetErrorString(_e) + " at " +   \
                           __FILE__ + ":" + std::to_string(__LINE__) + ": " #expr);        \
  } while (0)

constexpr int kWave = 64;
constexpr uint32_t kEmpty = 0xFFFFFFFFu;

// Last index a in [0, n) with pre[a] <= x, for ascending pre with pre[0] <= x,
// by binary lifting over a uniform trip count (`top`: the largest power of
// two below n, from a bound every lane shares).  A `while (hi - lo > 1)`
// search exits per lane, and the compiler drains every outstanding global
// load and store (s_waitcnt vmcnt(0)) at that divergent exit -- so loads
// issued for several items of a pass ran one after another.
__device__ __forceinline__ uint32_t lift_top(uint32_t n) { return n > 1 ? 1u << (31 - __clz(n - 1)) : 0u; }
template <typename T, typename X>
__device__ __forceinline__ uint32_t lift_search(const T* pre, uint32_t n, X x, uint32_t top) {
  uint32_t a = 0;
  for (uint32_t step = top; step; step >>= 1) {
    const uint32_t c = a + step;
    const T pc = pre[c < n ? c : n - 1];
    a = (c < n && pc <= x) ? c : a;
  }
  return a;
}

// Search status codes (DevState::status / HostResult::status)
enum : uint32_t { kRunning = 0, kFound = 1, kNoPath = 2, kHandoff = 3, kError = 4 };

// Search state shared by the LDS engine (on hand-off) and the grid engine.
// Lives in device memory; the host mirrors it with one small async copy.
struct DevState {
  uint32_t status;
  uint32_t meet;          // meet vertex (kEmpty = none yet)
  uint32_t meet_side;     // side whose expansion found the meet
  uint32_t levels;
  int32_t depth[2];       // depth of each side's current frontier
  uint32_t fbeg[2];       // current frontier = queue[s][fbeg, fend)
  uint32_t fend[2];
  uint32_t qtail[2];      // append cursor during a level (== fend between levels)
  uint32_t hub_count;     // grid top-down: number of hub vertices deferred
  uint32_t chunk;         // grid top-down: dynamic chunk counter
  unsigned long long hub_edge_cursor;
  unsigned long long fedges[2];   // sum of degrees of each current frontier
  unsigned long long vedges[2];   // sum of degrees of every vertex claimed by the side
  unsigned long long nedges;      // degrees of vertices claimed in the running level
  unsigned long long einsp;       // edges inspected
  uint32_t pad[4];
};

// Record the device writes straight into pinned host memory at the end of a
// query (no hipMemcpy on the critical path; the host spins on `seq`).
struct HostResult {
  uint32_t seq;           // written LAST, system-scope release
  uint32_t status;
  int32_t hops;
  uint32_t meet;
  uint32_t levels;
  uint32_t visited;
  unsigned long long einsp;
  int32_t depth[2];
  uint32_t path_len;      // hops + 1 when found
  uint32_t path_on_device;// 1 when the path did not fit the pinned buffer
  uint32_t lds_levels;
  uint32_t probe;         // LDS meet probe: frontier edges it read | 1 << 31 when it found the meet
  unsigned long long rt_begin, rt_end;  // s_memrealtime (100 MHz) around the LDS search
  unsigned long long rt_pickup;         // resident server: when the request was seen (0 otherwise)
  unsigned long long rt_walk;           // grid publish: when its path walk started (0: no grid walk)
};

// Pinned mailbox of the resident query server (k_lds_server).  The host
// writes src/dst/options, then `seq` (release); the server answers through
// HostResult with the same seq.
// The request is ONE 16-byte word, read by the server with a single PCIe
// load per poll (a poll of pinned host memory costs ~1 us): {seq, src, dst,
// tag} with tag = flags | (seq & 0xffffff) << 8, so a torn read is detected.
// The request owns the first 64-byte line and the server's status words the
// second: the server's per-query diagnostic stores then never invalidate the
// host's copy of the request line, and the host's post never has to re-fetch
// a line the GPU just wrote.
struct alignas(64) ServerBox {
  uint32_t seq, src, dst, tag;  // host -> server
  uint32_t req_pad[12];
  uint32_t alive;  // server -> host: its launch seq while running, ~launch seq after exit
  uint32_t stage;  // server -> host (diagnostics): 1 polling, 2 request taken, 3 answered
  uint32_t seen;   // last request seq the server took
  uint32_t pad[13];
};
static_assert(sizeof(ServerBox) == 128, "request line + status line");
constexpr uint32_t kReqStop = 1u, kReqLockstep = 2u;  // tag flags; side policy in bits 2..3
constexpr uint32_t kReqAltBuf = 16u;                   // tag flag: search in the server's second state set
__host__ __device__ inline uint32_t req_tag(uint32_t seq, uint32_t flags) { return (flags & 0xffu) | (seq << 8); }

// ---- small-graph resident server (tiny_engine.hip) --------------------------
// Graphs up to kTinyMaxN vertices keep both visited sets in LDS as bitmaps and
// read a packed adjacency: one 8-byte word per directed edge holding the
// neighbour id, its CSR base and its degree.  Word layout (52 bits):
// v[51:35] | base[34:9] | deg[8:0]; the server's records put the parent's
// queue index in [63:52].
constexpr uint32_t kTinyMaxN = 1u << 17;
constexpr uint64_t kTinyMaxNnz = 1ull << 26;
constexpr int kTinyB = 2;  // frontier edges per lane per round
// 9-bit degree field; per-wave record sums are scanned as two 16-bit halves
// (64 lanes x kTinyB x 511 < 2^16)
constexpr uint32_t kTinyMaxDeg = 511;
static_assert(64u * kTinyB * kTinyMaxDeg < 65536u, "per-wave record sums must fit 16 bits");
__host__ __device__ inline uint64_t tiny_pack(uint32_t v, uint64_t base, uint64_t deg) {
  return (uint64_t)v << 35 | base << 9 | deg;
}
// The answer: 16-byte packets, each carrying the query's seq in its first
// word and written by one 16-byte system-scope store, so the host checks every
// packet by itself and no release fence orders them (a packet is read whole
// by one 16-byte host load).
//   packet 0: {seq, status | levels << 8, hops, meet}
//   packet 1: {seq, device ticks (100 MHz, request seen -> answer), edges inspected, visited}
//   packet 2+: {seq, path[3j], path[3j+1], path[3j+2]}
struct alignas(16) TinyPkt {
  uint32_t seq, a, b, c;
};
enum : uint32_t { kTinyFound = 1, kTinyNoPath = 2, kTinyOverflow = 3 };
constexpr uint32_t kTinyQ = 4096;  // LDS queue capacity per side (12-bit queue indices)
// next-round records past the LDS buffer (all-wave rounds): global, per buffer and side
constexpr uint32_t kTinySpill = 2048;
constexpr uint32_t kTinyPktCap = 2 + (2 * kTinyQ + 2) / 3 + 1;

// Result of one query of the batched global-visited kernel (batch_global.hip).
struct BatchOut {
  uint32_t status;
  int32_t hops;
  uint32_t meet;
  uint32_t levels;
  uint32_t visited;
  uint32_t path_len;
  unsigned long long einsp;
};

struct LevelTraceDev {
  uint32_t side, depth, frontier, mode;
  unsigned long long edges, discovered;
};

template <typename T>
__device__ __forceinline__ T wave_sum(T x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// exclusive prefix count of set bits below this lane
__device__ __forceinline__ uint32_t mbcnt64(unsigned long long mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

__device__ __forceinline__ uint32_t load_agent(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace dev

// ----------------------------------------------------------------------------
// Host-side launchers (implemented in the .hip files)
// ----------------------------------------------------------------------------
namespace launch {

struct GraphView {
  uint32_t n;
  uint64_t nnz;
  const uint64_t* row_off;     // n + 1
  const uint32_t* row_off32;   // n + 1 copy when nnz < 2^32 (else nullptr)
  const uint32_t* col;
  const uint4* padj;           // nnz packed {v, deg(v), row_off[v] lo, hi}, or nullptr
  uint64_t max_deg = ~0ull;    // largest degree (unknown: ~0)
  // 8-byte packed adjacency (pack8): v[63:39] | base[38:10] | deg[9:0], for
  // graphs with n < 2^25, nnz < 2^29 and every degree < 1023 -- half the
  // bytes of padj, so a 10M-vertex graph's (176 MB) stays in the MALL
  const unsigned long long* padj8 = nullptr;
  // LDS meet probe before a hand-off: frontier edges it may read (hub graphs
  // only; HipBiBfs::set_lds_probe_edges, 0 = off)
  uint32_t probe_edges = 0;
};
__host__ __device__ inline unsigned long long pack8(uint32_t v, uint64_t base, uint64_t deg) {
  return (unsigned long long)v << 39 | base << 10 | deg;
}
__host__ __device__ inline uint32_t pack8_v(unsigned long long w) { return (uint32_t)(w >> 39); }
__host__ __device__ inline uint32_t pack8_base(unsigned long long w) { return (uint32_t)(w >> 10) & 0x1FFFFFFFu; }
__host__ __device__ inline uint32_t pack8_deg(unsigned long long w) { return (uint32_t)w & 0x3FFu; }
constexpr uint64_t kPack8MaxN = 1ull << 25, kPack8MaxNnz = 1ull << 29, kPack8MaxDeg = 1022;

struct SearchBuffers {
  uint32_t* vis[2];     // n/32 + 1 words each; all-zero between searches
  uint32_t* fbits[2];   // frontier bitmaps (bottom-up)
  uint32_t* nbits[2];   // next-frontier bitmaps (bottom-up)
  uint32_t* parent[2];  // n each, valid only where visited
  uint32_t* queue[2];   // n each, BFS order of claimed vertices
  uint32_t* hub_list;   // n (grid top-down deferred hubs)
  uint32_t* dpath;      // n + 1 (device path for long paths)
  dev::DevState* st;
  dev::LevelTraceDev* trace;
  uint32_t trace_cap;
  uint32_t words;       // n/32 + 1
  // Device hand-off words (resident searches, grid_auto): [0..1] gate = 64-bit
  // {handed off (0/1), seq} the LDS engine stores (agent scope, after its
  // release) when a search leaves it; [2..6] the auto level's plan (k_handoff)
  // for the kernels behind it.
  uint32_t* aux;
  uint32_t* hdump;      // raw LDS hash tables of a hash-set search's hand-off (handoff_dump_bytes())
  // stamped traces (BIBFS_STAMP): per grid level (levels % kGridStampLevels)
  // kGridStampWords s_memrealtime stamps of a top-down level -- block 0's
  // entry / chunk staged / chunk edges done / leaving, the finisher's start /
  // end -- so a level's time splits into its dependent phases
  unsigned long long* gstamp;
};
constexpr uint32_t kGridStampLevels = 64, kGridStampWords = 8;

struct HostSide {
  dev::HostResult* res;  // pinned, device-visible
  uint32_t* path;        // pinned
  uint32_t path_cap;
  dev::DevState* state = nullptr;  // pinned DevState mirror (the LDS hand-off publishes into it)
};

// csr_device.hip
void build_csr_from_edges(const uint32_t* d_uv, uint64_t m, uint32_t n, uint64_t* d_row_off,
                          uint32_t** d_col_out, uint64_t* nnz_out, uint32_t* d_row_off32_or_null,
                          hipStream_t s);
uint64_t count_csr_entries(const uint32_t* d_uv, uint64_t m, uint32_t n, uint64_t* d_row_off,
                           hipStream_t s);
void fill_csr(const uint32_t* d_uv, uint64_t m, uint32_t n, const uint64_t* d_row_off,
              uint64_t* d_cursor, uint32_t* d_col, hipStream_t s);
uint64_t count_csr_rows(const uint32_t* d_uv, uint64_t m, uint32_t lo, uint32_t hi, uint64_t* d_row_off,
                        hipStream_t s);
void fill_csr_rows(const uint32_t* d_uv, uint64_t m, uint32_t lo, uint32_t hi, const uint64_t* d_row_off,
                   uint64_t* d_cursor, uint32_t* d_col, hipStream_t s);
void build_padj(const uint64_t* row_off, const uint32_t* col, uint64_t nnz, uint4* padj, hipStream_t s);
void build_padj8(const uint64_t* row_off, const uint32_t* col, uint64_t nnz, unsigned long long* padj8, hipStream_t s);
void make_row_off32(const uint64_t* d_row_off, uint32_t n, uint32_t* d_row_off32, hipStream_t s);
uint64_t max_degree(const uint64_t* d_row_off, uint32_t n, hipStream_t s);  // synchronous
uint64_t gen_gnp_device(uint32_t n, double p, uint64_t seed, uint32_t** d_uv_out, hipStream_t s);
void gen_rmat_device(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c,
                     uint32_t* d_uv, hipStream_t s);
// Owned rows [lo, hi) of a device-generated graph straight from the generator
// (two passes, no edge list): fills d_row_off (hi - lo + 1), allocates the
// columns, returns nnz.  gen_rows_gnp also returns the undirected edge count.
uint64_t gen_rows_rmat(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c, uint32_t lo, uint32_t hi,
                       uint64_t* d_row_off, uint32_t** d_col_out, hipStream_t s);
uint64_t gen_rows_gnp(uint32_t n, double p, uint64_t seed, uint32_t lo, uint32_t hi, uint64_t* d_row_off,
                      uint32_t** d_col_out, uint64_t* m_out, hipStream_t s);

// tiny_engine.hip
struct TinyArgs {
  const unsigned long long* tadj;   // nnz packed words
  const unsigned long long* tinfo;  // n packed words (the vertex's own)
  uint32_t n;
  dev::ServerBox* box;               // pinned: alive word (and the request, unless `req` is elsewhere)
  const void* req;                  // the 16-byte request the server polls (the pinned box)
  dev::TinyPkt* pkts;               // pinned, kTinyPktCap packets
  uint32_t launch_seq, last_seq;
  int pin_xcc;
  uint32_t* ticket;
  unsigned long long idle_ticks;
  unsigned long long* stamps;       // device, 16 words (stamp build only)
  unsigned long long* spill;        // device, [2 buffers][2 sides][kTinySpill] records
};
bool tiny_supported(uint32_t n, uint64_t nnz, uint64_t max_deg);
void build_tiny_adj(const uint64_t* row_off, const uint32_t* col, uint32_t n, uint64_t nnz,
                    unsigned long long* tadj, unsigned long long* tinfo, hipStream_t s);
void tiny_server(const TinyArgs& a, bool stamp, hipStream_t s);

// engine_kernels.hip
void lds_search(const GraphView& g, const SearchBuffers& b, const HostSide& h, uint32_t src,
                uint32_t dst, uint32_t seq, int side_policy, int trace, int pin_xcc, uint32_t* ticket,
                int lockstep, hipStream_t s);
int lds_threads();
uint32_t lds_probe_budget();  // BIBFS_LDS_PROBE_EDGES (default 16384; 0 = no meet probe before a hand-off)
size_t lds_bytes(bool wide);
void lds_server(const GraphView& g, const SearchBuffers& b, const SearchBuffers& b_alt, const HostSide& h,
                dev::ServerBox* box, uint32_t launch_seq, uint32_t last_seq, int pin_xcc, uint32_t* ticket,
                unsigned long long idle_ticks, bool stamp_server, hipStream_t s);
void lds_batch(const GraphView& g, const SearchBuffers& b, uint32_t* h_src, uint32_t* h_dst,
               uint32_t k, uint32_t* d_slots, dev::HostResult* h_res, uint32_t* h_path, uint32_t path_cap,
               uint32_t seq, hipStream_t s);
void seed_state(const GraphView& g, const SearchBuffers& b, uint32_t src, uint32_t dst,
                hipStream_t s);
// batch_global.hip: one workgroup per query, bitmaps in HBM (queries that outgrow LDS)
void batch_global(const GraphView& g, uint32_t words, const uint32_t* qidx, uint32_t k, const uint32_t* src,
                  const uint32_t* dst, uint32_t* slots, uint32_t* bits, dev::BatchOut* out, uint32_t* path,
                  uint32_t path_cap, unsigned long long edge_cap, int threads, hipStream_t s);
// One top-down level; the LAST workgroup finishes it, publishes the mirror
// (seq) and, when the search ended, walks the path and publishes the result
// (res_seq).  hub_deg != ~0u: frontier vertices above that degree are deferred
// to the edge-parallel hub pass enqueued behind, which then finishes the level.
void grid_topdown(const GraphView& g, const SearchBuffers& b, int side, int cus, uint64_t frontier,
                  uint64_t frontier_edges, dev::DevState* mirror, uint32_t seq, int trace, const HostSide& h, uint32_t res_seq,
                  uint32_t hub_deg, hipStream_t s);
void grid_bottomup(const GraphView& g, const SearchBuffers& b, int side, int cus, hipStream_t s);
// Behind a hash-set LDS search's hand-off (n > 2^17): scatter the dumped hash
// tables into the global visited bitmaps, grid-wide (grid_auto does it itself).
void handoff_scatter(const GraphView& g, const SearchBuffers& b, hipStream_t s);
size_t handoff_dump_bytes();
void build_frontier_bits(const GraphView& g, const SearchBuffers& b, int side, hipStream_t s);
void finish_level(const SearchBuffers& b, int side, int mode, int trace, dev::DevState* mirror, uint32_t seq,
                  const HostSide& h, uint32_t res_seq, uint32_t n, hipStream_t s);
uint32_t grid_hub_degree();
void bitmap_meet(const SearchBuffers& b, uint32_t* d_flag, hipStream_t s);
void walk_path(const SearchBuffers& b, const HostSide& h, uint32_t src, uint32_t dst, uint32_t seq,
               uint32_t n, hipStream_t s);
// if_done: 0 = always; 1 = only once a grid level ended the search; 2 = and
// only behind an auto chain that took the hand-off (aux[2] bit 0)
void cleanup(const SearchBuffers& b, uint32_t n, uint32_t* done_ctr, uint32_t* host_tag, uint32_t tag,
             int if_done, hipStream_t s);
// Device hand-off: one top-down level enqueued BEFORE the resident LDS search
// it continues.  Its workgroups wait on the gate (aux) for search `gate_seq`
// to leave LDS, plan the level on the device (side, hub degree, chunk size:
// the host rules of grid_level), run it and finish it like grid_topdown
// (mirror `seq`, result `res_seq`); a search that ended in LDS, or a first
// level the Beamer rule sends bottom-up, makes it a no-op (the latter
// publishes the mirror unchanged, so the host loop takes that level).
// levels > 1 chains that many device-planned levels: the finisher of each
// plans the next one into aux (or ends the chain: search over, or a level the
// Beamer rule declines, which publishes the mirror `seq` for the host).
void grid_auto(const GraphView& g, const SearchBuffers& b, int cus, uint64_t max_deg, double alpha,
               dev::DevState* mirror, uint32_t seq, const HostSide& h, uint32_t res_seq, uint32_t gate_seq,
               unsigned long long gate_ticks, int levels, hipStream_t s);

}  // namespace launch
}  // namespace bibfs
