// Bidirectional-BFS search kernels for MI355X (gfx950, wave64).
//
// Reference kernels replaced:
//   K1 expand_frontier      v3/bibfs_cuda_only.cu:13-43  thread-per-vertex over ALL N every level
//   K2 check_intersect      v3/bibfs_cuda_only.cu:45-62  O(N) scan per level
//   K3 expand_frontier_kernel v4/comp.cu:20-38           same + dead partition filter
//   K4 check_intersect_kernel v4/comp.cu:40-47
// The reference pays ~8 host<->device operations plus 3 launches per level
// (v3:176-199).  Here:
//   * k_lds_bibfs: the whole search in ONE launch of ONE 1024-thread workgroup.
//     Visited sets are LDS hash tables (claim = LDS CAS, ~100 cycles, instead
//     of a returning global atomic at ~1,700 cycles measured on gfx950), both
//     frontiers are LDS-resident together with their CSR row offsets, which are
//     prefetched speculatively the moment a neighbour id arrives, so each level
//     costs two dependent global loads (column id, then row offsets) plus LDS
//     work and one barrier.  The meet test is fused into the claim.  No global
//     atomics, no O(N) pass, no host round trip per level; the result and the
//     path are written straight into pinned host memory.
//   * k_grid_topdown / k_grid_hubs / k_grid_bottomup: device-wide levels for
//     frontiers that outgrow LDS (RMAT/Kronecker), with dynamic chunking,
//     hub deferral, wave-aggregated queue appends, early exit on meet and a
//     Beamer direction switch driven by the host.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstddef>
#include <cstdlib>

#include <type_traits>

#include "device.hpp"

namespace bibfs {
namespace {

using namespace dev;

// ============================================================================
// LDS engine
// ============================================================================
// One persistent 1024-thread workgroup runs the whole search; no global
// atomics, no per-level host round trip.  LDS holds
//   * H[2][8192]  open-addressing hash sets of every vertex each side claimed.
//                 Keys carry the parity of the claim depth in bit 31, which is
//                 all the meet rule needs (below).
//   * R[4][CAP]   per-edge work records {parent u, CSR index k} of the two
//                 current frontiers and two frontiers being built.  Records are
//                 written at claim time for every edge of the new vertex (its
//                 row offsets are prefetched the moment its id arrives), so a
//                 level needs no degree scan and no edge->vertex search.
// A level costs two dependent global loads (column id, then row offsets of
// the new vertex) plus LDS work.  Two schedules hide that chain:
//   * lockstep rounds -- while both frontiers are small, wave 0 expands the
//     source side and wave 1 the target side CONCURRENTLY (one round = two
//     levels in the time of one); they sync through an LDS counter.
//   * big levels -- a frontier above kSmallEdges edges is expanded by all 16
//     waves (one edge per lane, 4 in flight), appends placed by one packed LDS
//     atomic per wave + a DPP prefix sum; waves 2-15 are parked at the
//     workgroup barrier otherwise.
// Meet rule.  At the first round in which any vertex becomes visited by both
// sides (S expanding depth a -> a+1, T expanding b -> b+1 or idle), every hit
// of a newly claimed vertex in the other side's set has the other depth in
// {b, b+1} (a shallower one would have met a round earlier), so the stored
// depth parity identifies it and each candidate's exact length is known; the
// answer is the minimum candidate of that round.  Two concurrent claims of the
// same vertex are always seen by at least one side: each side completes its
// own insert (LDS CAS) before reading the other set.
// Tuning constants (each was A/B-measured; the files are named beside it).
// Variants measured slower and removed from the code (results and the A/B
// files: docs/DESIGN.md §8): a readfirstlane'd wave id, ballot-driven record
// appends, hash-set all-wave rounds with an LDS queue (profiles/r2_wave_hash_ab.txt)
// and 4-slot hash buckets (profiles/r4_lds_hash_bucket_ab.jsonl).
// 1 = lockstep rounds of up to kLdsThreads frontier edges run on EVERY wave
// with one LDS-only barrier per round (wave_rounds); 0 = the wave-0 rounds.
constexpr bool kWaveRounds = true;
// 1 = an all-wave round that cannot carry both frontiers expands the smaller
// side alone (while it fits) instead of leaving the all-wave rounds.
constexpr bool kWaveSingle = true;
// batches of 64 edges per wave in those rounds (1: frontiers up to 1024 edges, 2: 2048)
constexpr uint32_t kWaveB = 2;
static_assert(kWaveB == 1 || kWaveB == 2 || kWaveB == 4, "batches per wave: 1, 2 or 4");
// 1 = the all-wave rounds also run with LDS hash visited sets, claiming into
// the GLOBAL queue and parent arrays (records carry parent ids, as in the
// wave-0 schedule): no LDS queue, so the record buffers keep their full size
// and the search hands off no earlier than without the all-wave rounds.  Only
// on graphs whose largest degree is at most kWaveHashMaxDeg (LdsParams::
// wave_hash): a hub's edge records are appended by one lane.  Measured
// (profiles/r4_lds_wave_hash_global_ab.jsonl, mean search): 10M G(n, p)
// 67.5 -> 63.5-64.0 us, 3M 38.3 -> 34.2, 1M 30.2 -> 26.0; ungated it cost
// Kronecker 22 +4 us (profiles/r4_lds_wave_hash_global_ungated.jsonl).
constexpr bool kWaveHashG = true;
// (lifting the gate once cooperative appends existed changed nothing:
// profiles/r5_wave_hash_gate_ab.jsonl)
constexpr uint64_t kWaveHashMaxDeg = 255;
// Resident server: the mailbox diagnostics (stage / seen / poll latency) are
// system-scope stores to host memory.  vmcnt counts stores too, so if wave 0
// issued them, its first global load of the search would wait for their PCIe
// acks.  1 = the last wave issues them (it is parked during small rounds).
constexpr bool kDiagOffWave0 = true;

// Workgroup size of the LDS engine.  1024 threads = 4 waves per SIMD caps a
// wave at 128 VGPRs (the kernel sits at that limit; 2-4 spills); 512 threads
// lift the cap to 256 but halve the lanes of the all-wave levels.  A/B on
// 100k / 1M G(n,p) (profiles/r2_lds_ab.txt): 1024 is 0.5-0.9 us faster.
constexpr int kLdsThreads = 1024;
constexpr int kHashBits = 13;
constexpr uint32_t kHashSize = 1u << kHashBits;  // slots per side
constexpr uint32_t kHashMask = kHashSize - 1;
constexpr uint32_t kHashLimit = kHashSize * 3 / 4;  // max visited per side in LDS
constexpr int kBatch = 4;                           // edges per thread per round (big levels)
constexpr uint32_t kSmallEdges = 128;  // a level this small runs on one wave
constexpr uint32_t kDualEdges = 256;    // both sides together this small: one lockstep round
constexpr uint32_t kDualBigEdges = 4096;                  // balanced sides up to this many edges: lockstep big level
constexpr uint32_t kDegClamp = 65535;               // per-lane edge contribution to the packed counter
// Bitmap mode with the all-wave rounds: smaller record buffers make room for
// the LDS queue (vertex + parent's queue index per side) the path is walked on.
constexpr uint32_t kCapBm = 1900;
constexpr uint32_t kQCap = 2048;
constexpr uint32_t kParity = 0x80000000u;           // depth-parity bit of a hash key
constexpr uint32_t kIdMask = 0x7fffffffu;

template <typename OffT>
struct LdsRec;
template <>
struct LdsRec<uint32_t> {
  using type = uint2;  // {parent, k}
  static constexpr uint32_t cap = 2976;
};
template <>
struct LdsRec<uint64_t> {
  using type = uint4;  // {parent, k_lo, k_hi, pad}
  static constexpr uint32_t cap = 1488;
};

__device__ __forceinline__ void rec_set(uint2& r, uint32_t u, uint32_t k) { r = make_uint2(u, k); }
__device__ __forceinline__ void rec_set(uint4& r, uint32_t u, uint64_t k) {
  r = make_uint4(u, (uint32_t)k, (uint32_t)(k >> 32), 0u);
}
__device__ __forceinline__ uint32_t rec_k(const uint2& r) { return r.y; }
__device__ __forceinline__ uint64_t rec_k(const uint4& r) { return (uint64_t)r.y | ((uint64_t)r.z << 32); }

template <typename OffT>
struct LdsParams {
  const OffT* row_off;
  const uint32_t* col;
  const uint4* padj;  // packed {v, deg, base lo, base hi} per edge, or nullptr
  const unsigned long long* padj8;  // or its 8-byte form (launch::pack8), or nullptr
  uint32_t n;
  uint32_t src, dst, seq;
  int side_policy;
  int trace;
  int pin_xcc;        // >= 0: only a block on this XCD may run the search
  uint32_t* ticket;   // monotonic election word (atomicMax with seq)
  int lockstep;       // allow concurrent two-sided rounds
  OffT nnz_m1;        // last valid CSR index (clamp for record-driven loads)
  int batch;          // batched search: no hand-off state / device path (the host re-runs those queries)
  launch::SearchBuffers b;
  launch::HostSide h;
  // 0: fresh LDS (one-shot / batch kernels); resident server: 1 = its first
  // search, 2 = a later one (LDS kept from the previous search in this launch)
  int resident = 0;
  // resident server: the second search-state set (request flag kReqAltBuf);
  // the host alternates sets so a search never shares its global state with
  // the previous search's still-running cleanup
  launch::SearchBuffers b_alt{};
  // hash-set searches (kWaveHashG): run the all-wave rounds (graphs without
  // hubs; a hub's records are written by one lane)
  int wave_hash = 0;
  // meet probe before a hand-off: frontier edges it may read (0 = off; see
  // lds_meet_probe)
  uint32_t probe = 0;
};

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

__device__ __forceinline__ uint32_t hslot(uint32_t v) {
  return (v * 0x9E3779B1u) >> (32 - kHashBits);
}

// Insert vertex v with the given key (v | parity); true when v was absent.
__device__ __forceinline__ bool hash_insert(uint32_t* H, uint32_t v, uint32_t key) {
  uint32_t h = hslot(v);
  for (uint32_t probe = 0; probe < kHashSize; ++probe) {  // bounded: the load limit keeps it short
    const uint32_t old = atomicCAS(&H[h], kEmpty, key);
    if (old == kEmpty) return true;
    if ((old & kIdMask) == v) return false;
    h = (h + 1) & kHashMask;
  }
  return false;
}

// Stored key of v (kEmpty when absent).
__device__ __forceinline__ uint32_t hash_find(const uint32_t* H, uint32_t v) {
  uint32_t h = hslot(v);
  for (uint32_t probe = 0; probe < kHashSize; ++probe) {
    const uint32_t k = H[h];
    if (k == kEmpty || (k & kIdMask) == v) return k;
    h = (h + 1) & kHashMask;
  }
  return kEmpty;
}

// ---- bitmap visited sets (graphs with n <= kBmMaxN): the hash area holds,
// per side, one u64 per 32 vertices -- low half = claimed at an even depth,
// high half = claimed at an odd depth.  A claim is one ds_or_rtn_b64: the
// returned word says whether the vertex was already held at either parity.
// A losing claim still sets its parity bit ("pollution"); a vertex with both
// bits therefore has the OLDER depth, which for a first meet is b (see the
// lockstep rule above), so the readers below map both-bits to b.
constexpr uint32_t kBmMaxN = kHashSize * 16;  // 4096 u64 words per side = 131072 vertices

__device__ __forceinline__ bool bm_claim(unsigned long long* W, uint32_t v, uint32_t parity) {
  const uint32_t b = v & 31;
  const unsigned long long old = atomicOr(&W[v >> 5], 1ull << (b + 32 * parity));
  return ((old >> b) & 1ull) == 0 && ((old >> (32 + b)) & 1ull) == 0;
}

// 0 = absent, 1 = even depth, 2 = odd depth, 3 = both (the older claim)
__device__ __forceinline__ uint32_t bm_state(const unsigned long long* W, uint32_t v) {
  const uint32_t b = v & 31;
  const unsigned long long w = W[v >> 5];
  return (uint32_t)((w >> b) & 1ull) | ((uint32_t)((w >> (32 + b)) & 1ull) << 1);
}

// Walk one side's parent chain from the meet vertex: side 0 writes path
// positions d0 .. 0, side 1 writes d0 .. d0 + d1.  One loop shape for both
// sides so two lanes of one wave walk the two chains concurrently.
__device__ void walk_side(const uint32_t* parent, uint32_t n, uint32_t meet, int side, int d0, int d1,
                          uint32_t* out) {
  uint32_t v = meet;
  int pos = d0;
  const int step = side ? 1 : -1;
  for (int remain = side ? d1 : d0;; --remain) {
    out[pos] = v;
    if (remain == 0 || v >= n) break;  // v >= n only if the chain were inconsistent: never read past it
    v = load_agent(&parent[v]);
    pos += step;
  }
}

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }

// Inclusive wave64 prefix sum on the VALU via DPP (row_shr 1/2/4/8 inside
// each 16-lane row, then row_bcast15 / row_bcast31 across rows) -- no LDS
// permutes, ~6 instructions.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}


// Published by wave 0 for the parked waves: the big level to run (or the end).
// E[q] = records of side q to expand (0 = side q idle this level).
struct LevelPlan {
  uint32_t status;
  uint32_t E[2], cur[2], off[2], nxt[2], qbase[2], depth[2];
  uint32_t pside, pfb, pcnt;  // kProbing: the side that does not fit, its frontier in the global queue
  uint32_t prec;              // ... its level's records in LDS (R[cur[side]][off[side] ..]), or 0
};

// Internal plan status: probe the level that does not fit LDS for a meet
// before handing it to the grid (never published).
constexpr uint32_t kProbing = 7;
constexpr uint32_t kProbeU = 4;  // frontier edges per thread per probe pass

// Meet probe (all waves of the LDS engine, read-only).  The next level of
// side q does not fit LDS, so the search would hand off to the grid engine.
// No meet has been found yet, so every vertex of the other side adjacent to
// q's frontier sits at that side's frontier depth (a shallower one would
// have claimed -- or been claimed from -- the frontier vertex already, and
// the claim would have seen the meet): EVERY such edge ends the search with
// the same, shortest, length dq + 1 + do.  The CPU engine stops at the first
// one, after a few thousand edges on hub graphs; the grid level reads them
// all.  So before handing off, the frontier's edges are read in passes of
// kLdsThreads * kProbeU and tested against the other side's LDS visited set
// -- no claims, no state written -- until an edge hits or `budget` edges
// were read.  The edges come from the level's records when they are in LDS
// (`recs`: a level that leaves LDS because a visited set is full -- one
// dependent load per pass), else from the queue (a level whose records did
// not fit: chunks of 1024 frontier vertices, block scan of their degrees,
// binary search per edge -- three dependent loads per chunk).
// Returns (u << 32) | v of a hit (u in q's frontier, v visited by the other
// side), or ~0; *walked = edges read.  Every wave calls it (barriers inside).
template <typename OffT, bool kBm, typename Rec>
__device__ unsigned long long lds_meet_probe(const LdsParams<OffT>& P, int q, uint32_t fb, uint32_t F,
                                             const Rec* recs, uint32_t nrec, uint32_t budget, const uint32_t* Ho,
                                             const unsigned long long* Wo, void* scratch, uint32_t* walked_out) {
  __shared__ unsigned long long pr_hit;
  __shared__ uint32_t pr_wsum[kLdsThreads / kWave], pr_total;
  const int tid = threadIdx.x, wid = tid >> 6;
  const uint32_t lane = __lane_id();
  uint32_t* su = static_cast<uint32_t*>(scratch);                 // [kLdsThreads] frontier vertex
  OffT* sbp = reinterpret_cast<OffT*>(su + kLdsThreads);           // its row base
  uint32_t* sEb = reinterpret_cast<uint32_t*>(sbp + kLdsThreads);  // exclusive prefix of the (clamped) degrees
  const uint32_t* qu = q ? P.b.queue[1] : P.b.queue[0];
  if (tid == 0) pr_hit = ~0ull;
  // every wave's queue stores complete before any wave reads the queue with
  // L2 loads (__syncthreads() alone waits for no store on gfx950)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  uint32_t walked = 0;
  bool stop = false;
  // one pass's test: the other side's visited set, the smallest hit kept; true
  // (uniform) once any wave hit
  auto test_pass = [&](const uint32_t (&uu)[kProbeU], const uint32_t (&v)[kProbeU], const bool (&ok)[kProbeU]) {
    unsigned long long best = ~0ull;
#pragma unroll
    for (uint32_t j = 0; j < kProbeU; ++j) {
      bool hit;
      if constexpr (kBm) hit = ok[j] && bm_state(Wo, v[j]) != 0u;
      else hit = ok[j] && hash_find(Ho, v[j]) != kEmpty;
      const unsigned long long key = ((unsigned long long)uu[j] << 32) | v[j];
      if (hit && key < best) best = key;
    }
    if (__ballot(best != ~0ull)) {
      unsigned long long m = best;
      for (int off = 32; off >= 1; off >>= 1) {
        const unsigned long long y = __shfl_xor(m, off);
        m = y < m ? y : m;
      }
      if (lane == 0) atomicMin(&pr_hit, m);
    }
    __syncthreads();
    return uni((uint32_t)(pr_hit >> 32)) != 0xffffffffu;
  };
  if (recs) {
    for (uint32_t base = 0; base < nrec; base += kLdsThreads * kProbeU) {
      const uint32_t pass = min(kLdsThreads * kProbeU, nrec - base);
      if (walked + pass > budget) break;  // (uniform)
      walked += pass;
      uint32_t v[kProbeU], uu[kProbeU];
      bool ok[kProbeU];
#pragma unroll
      for (uint32_t j = 0; j < kProbeU; ++j) {
        const uint32_t i = base + j * kLdsThreads + (uint32_t)tid;
        ok[j] = i < nrec;
        const Rec r = recs[ok[j] ? i : 0u];
        uu[j] = r.x;
        const OffT k = min((OffT)rec_k(r), P.nnz_m1);
        v[j] = 0u;
        if (ok[j]) v[j] = P.padj8 ? launch::pack8_v(P.padj8[k]) : P.padj ? P.padj[k].x : P.col[k];
      }
      if (test_pass(uu, v, ok)) break;
    }
    F = 0;  // (no queue chunks)
  }
  for (uint32_t c0 = 0; c0 < F && !stop; c0 += kLdsThreads) {
    const uint32_t i = c0 + (uint32_t)tid;
    uint32_t u = 0, d = 0;
    OffT b = 0;
    if (i < F) {
      u = load_agent(&qu[fb + i]);  // queue entries were written by this search (L2)
      b = P.row_off[u];
      d = (uint32_t)min((OffT)(P.row_off[u + 1] - b), (OffT)(1u << 20));  // sums stay < 2^31
    }
    su[tid] = u;
    sbp[tid] = b;
    const uint32_t incl = wave_incl_scan(d);
    if (lane == kWave - 1) pr_wsum[wid] = incl;
    __syncthreads();
    if (tid == 0) {
      uint32_t a = 0;
      for (int k = 0; k < kLdsThreads / kWave; ++k) {
        const uint32_t t = pr_wsum[k];
        pr_wsum[k] = a;
        a += t;
      }
      pr_total = a;
    }
    __syncthreads();
    sEb[tid] = incl - d + pr_wsum[wid];
    const uint32_t Ec = uni(pr_total);
    __syncthreads();
    for (uint32_t base = 0; base < Ec; base += kLdsThreads * kProbeU) {
      const uint32_t pass = min(kLdsThreads * kProbeU, Ec - base);
      if (walked + pass > budget) {  // (uniform)
        stop = true;
        break;
      }
      walked += pass;
      uint32_t v[kProbeU], uu[kProbeU];
      bool ok[kProbeU];
#pragma unroll
      for (uint32_t j = 0; j < kProbeU; ++j) {
        const uint32_t e = base + j * kLdsThreads + (uint32_t)tid;
        ok[j] = e < Ec;
        const uint32_t lo = lift_search(sEb, kLdsThreads, e, kLdsThreads / 2);
        uu[j] = su[lo];
        v[j] = ok[j] ? P.col[sbp[lo] + (OffT)(e - sEb[lo])] : 0u;  // every pass's loads in flight together
      }
      if (test_pass(uu, v, ok)) {
        stop = true;
        break;
      }
    }
    __syncthreads();  // the chunk's LDS arrays are read until here
  }
  *walked_out = walked;
  const unsigned long long r = pr_hit;
  return ((unsigned long long)uni((uint32_t)(r >> 32)) << 32) | uni((uint32_t)r);
}

// One whole search by one workgroup.  `elected`: the caller already owns the
// search (the resident server); otherwise the block runs the XCD election.
template <typename OffT, bool kStamp, bool kBm>
__device__ __forceinline__ void lds_search_body(const LdsParams<OffT>& P, bool elected) {
  using Rec = typename LdsRec<OffT>::type;
  constexpr bool kLq = kBm && kWaveRounds && std::is_same<OffT, uint32_t>::value;  // LDS queue + walk
  // all-wave rounds: with the LDS queue (kLq), or on hash sets with the global queue
  constexpr bool kWr = kLq || (kWaveHashG && !kBm && kWaveRounds && std::is_same<OffT, uint32_t>::value);
  constexpr uint32_t CAP = kLq ? kCapBm : LdsRec<OffT>::cap;
  __shared__ __attribute__((aligned(16))) uint32_t H[2][kHashSize];  // (16-byte bucket reads)
  __shared__ Rec R[4][CAP];
  // kLq: per side, the vertices in claim (queue) order and each one's parent's
  // queue index; a search that ends inside the all-wave rounds walks its path
  // here instead of along the global parent arrays
  __shared__ uint32_t LQ[kLq ? 2 : 1][kLq ? kQCap : 1];
  __shared__ uint32_t LP[kLq ? 2 : 1][kLq ? kQCap : 1];
  __shared__ uint32_t lq_meet[2];
  __shared__ unsigned long long ctr[2][2];  // big levels [slot][side]: (count << 32) | clamped edge sum
  __shared__ unsigned long long meetk[2];   // big levels [slot]: min (len << 32 | side << 31 | vertex)
  __shared__ LevelPlan plan;
  __shared__ uint32_t won;
  __shared__ __attribute__((aligned(16))) uint32_t pub_img[64];  // hand-off DevState [0, 32) / HostResult [32, 64) images

  // The thread index goes through an opaque copy: in the resident server this
  // body sits inside the query loop, and without it the compiler hoists every
  // tid-derived LDS address out of that loop and keeps them live across it --
  // at the 128-VGPR cap of a 1024-thread workgroup, as scratch spills reloaded
  // on every query.
  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int wid = tid >> 6;
  const uint32_t lane = __lane_id();
  // XCD affinity: the search is latency-bound on dependent CSR loads, so it
  // always runs on the same XCD, whose L2 keeps the graph's hot lines across
  // queries.  Several blocks are launched; the first one on the chosen XCD
  // wins the ticket and every other block exits at once (the host relaunches
  // with pin_xcc = -1 if no block reached that XCD).  The ticket atomic
  // (~1.6k cycles) is only resolved after the block-private initialisation
  // below; a losing candidate's few global writes there are idempotent.
  unsigned long long e0 = 0, e1 = 0, e3 = 0, e4 = 0;  // kStamp: entry / elected / loop end / walked
  unsigned long long e5 = 0, e6 = 0, e7 = 0, e8 = 0;  // kStamp: publish split
  if (kStamp && tid == 0) e0 = __builtin_amdgcn_s_memtime();
  const bool cand = elected || (P.pin_xcc < 0 ? blockIdx.x == 0 : xcc_id() == (uint32_t)P.pin_xcc);
  if (!cand) return;  // block-uniform
  uint32_t ticket_old = 0;
  if (tid == 0 && !elected) ticket_old = atomicMax(P.ticket, P.seq);

  // Each lane's vertex gets its dl edge records Rn[eb .. eb+dl).  Short runs
  // are written by their own lane (exec-masked loop); a run longer than
  // kCoopRun -- a hub's neighbour on a power-law graph, thousands of records
  // -- by the whole wave, 64 records per store, one run after another: one
  // lane writing 2k records serially held a Kronecker 22 lockstep round for
  // ~18k cycles (profiles/r5_kron22_probe_stamps.txt).  Every lane of the
  // wave calls it (ballot inside).
  auto append_records = [&](Rec* Rn, uint32_t dl, uint32_t eb, uint32_t v, OffT base) {
    constexpr uint32_t kCoopRun = 32;
    const bool coop = dl > kCoopRun;
    for (uint32_t j = 0; j < (coop ? 0u : dl); ++j) rec_set(Rn[eb + j], v, base + j);
    for (unsigned long long m = __ballot(coop); m; m &= m - 1) {
      const int l = __ffsll((long long)m) - 1;
      const uint32_t d = __builtin_amdgcn_readlane(dl, l), e = __builtin_amdgcn_readlane(eb, l);
      const uint32_t vl = __builtin_amdgcn_readlane(v, l);
      // (readlane returns int: widen through uint32_t, or a row base at or
      // above 2^31 -- Kronecker 27 -- is sign-extended into garbage)
      OffT bl;
      if constexpr (sizeof(OffT) == 8)
        bl = (OffT)(uint32_t)__builtin_amdgcn_readlane((uint32_t)base, l) |
             ((OffT)(uint32_t)__builtin_amdgcn_readlane((uint32_t)((uint64_t)base >> 32), l) << 32);
      else
        bl = (OffT)(uint32_t)__builtin_amdgcn_readlane((uint32_t)base, l);
      for (uint32_t j = lane; j < d; j += kWave) rec_set(Rn[e + j], vl, bl + j);
    }
  };
  // Edge k -> (neighbour v, its row [ob, oe)): one packed load, or col[k] then
  // the row offsets (a second dependent load) when no packed adjacency exists.
  // The branch is on a kernel argument: wave-uniform.
  auto fetch_edges = [&](auto bc, const OffT* kk, uint32_t* vv, OffT* ob, OffT* oe) {
    constexpr int B = decltype(bc)::value;
    if (P.padj8) {
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const unsigned long long w = P.padj8[kk[k]];
        vv[k] = launch::pack8_v(w);
        ob[k] = (OffT)launch::pack8_base(w);
        oe[k] = ob[k] + (OffT)launch::pack8_deg(w);
      }
    } else if (P.padj) {
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const uint4 q = P.padj[kk[k]];
        vv[k] = q.x;
        ob[k] = (OffT)((uint64_t)q.z | ((uint64_t)q.w << 32));
        oe[k] = ob[k] + (OffT)q.y;
      }
    } else {
#pragma unroll
      for (int k = 0; k < B; ++k) vv[k] = P.col[kk[k]];
#pragma unroll
      for (int k = 0; k < B; ++k) {  // row offsets, in flight during the claims
        ob[k] = P.row_off[vv[k]];
        oe[k] = P.row_off[vv[k] + 1];
      }
    }
  };
  uint32_t* Hflat = &H[0][0];
  // Visited sets start empty.  A resident search that ended inside the
  // all-wave rounds cleared the bitmap words it set after publishing (sparse,
  // off the critical path), so the 64 KB clear -- >= 512 cycles of LDS write
  // bandwidth -- is skipped when the previous search left it clean.
  __shared__ uint32_t bm_dirty;
  if (!kBm || P.resident < 2 || bm_dirty) {
    const uint32_t fill = kBm ? 0u : kEmpty;
    uint4* H4 = reinterpret_cast<uint4*>(Hflat);
    for (uint32_t i = tid; i < 2 * kHashSize / 4; i += kLdsThreads) H4[i] = make_uint4(fill, fill, fill, fill);
  }
  // side q's bitmap view of the same LDS (kBm)
  auto W = [&](int q) { return reinterpret_cast<unsigned long long*>(q ? H[1] : H[0]); };
  if (tid < 4) ctr[tid >> 1][tid & 1] = 0;
  if (tid < 2) meetk[tid] = ~0ull;

  // ---- replicated search state: identical in waves 0 and 1 (the workers);
  // two structs selected field-wise (a struct-level `?:` or an array indexed
  // by the runtime side is lowered through scratch memory).
  struct SideState {
    uint32_t cur, off, cnt, hcnt, qend, fbeg, ovf;  // records: R[cur][off .. off + fed)
    int depth;
    unsigned long long fed, ved;
  };
  auto sel = [](bool one, const SideState& a, const SideState& b) {
    SideState x;
    x.cur = one ? b.cur : a.cur;
    x.off = one ? b.off : a.off;
    x.cnt = one ? b.cnt : a.cnt;
    x.hcnt = one ? b.hcnt : a.hcnt;
    x.qend = one ? b.qend : a.qend;
    x.fbeg = one ? b.fbeg : a.fbeg;
    x.ovf = one ? b.ovf : a.ovf;
    x.depth = one ? b.depth : a.depth;
    x.fed = one ? b.fed : a.fed;
    x.ved = one ? b.ved : a.ved;
    return x;
  };
  // both endpoints' row offsets in flight together (the stores below would
  // otherwise order side 1's loads after side 0's)
  const OffT rb0 = P.row_off[P.src], re0 = P.row_off[P.src + 1];
  const OffT rb1 = P.row_off[P.dst], re1 = P.row_off[P.dst + 1];
  auto init_side = [&](int q) {
    SideState x;
    const uint32_t r = q ? P.dst : P.src;
    const OffT b = q ? rb1 : rb0, e = q ? re1 : re0;
    x.cur = (uint32_t)q;
    x.off = 0;
    x.cnt = 1;
    x.hcnt = 1;
    x.qend = 1;
    x.fbeg = 0;
    x.depth = 0;
    x.fed = (unsigned long long)(e - b);
    x.ved = x.fed;
    x.ovf = (e - b) > (OffT)CAP ? 1u : 0u;
    if (!x.ovf)
      for (uint32_t j = tid; j < (uint32_t)(e - b); j += kLdsThreads) rec_set(R[q][j], r, b + j);
    if (tid == q) {
      (q ? P.b.parent[1] : P.b.parent[0])[r] = kEmpty;
      (q ? P.b.queue[1] : P.b.queue[0])[0] = r;
    }
    return x;
  };
  SideState s0 = init_side(0), s1 = init_side(1);
  // a record buffer that holds neither side's current frontier (4 buffers, <= 2 in use)
  auto free_buf = [&]() -> uint32_t {
    const uint32_t used = (1u << s0.cur) | (1u << s1.cur);
    return (uint32_t)__builtin_ctz(~used & 0xfu);
  };
  uint32_t levels = 0, status = kRunning, meet = kEmpty, md0 = 0, md1 = 0, rounds = 0, bigs = 0;
  unsigned long long einsp = 0;
  int turn = 0;
  if (tid == 0) won = elected || ticket_old < P.seq;
  // LDS-only barrier: the two global stores above are never read back in LDS
  // mode before the final drain (a full __syncthreads waits for their acks)
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (!uni(won)) return;  // uniform: a divergent-looking exit around barriers can be mis-structurized
  if (kStamp && tid == 0) e1 = __builtin_amdgcn_s_memtime();
  if (tid < 2) {  // depth 0: parity 0
    if constexpr (kBm) bm_claim(W(tid), tid ? P.dst : P.src, 0);
    else hash_insert(H[tid], tid ? P.dst : P.src, tid ? P.dst : P.src);
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");

  auto fits = [&](const SideState& x) {
    return !x.ovf && (kBm || (unsigned long long)x.hcnt + x.fed <= kHashLimit);
  };
  auto record_trace = [&](int q, const SideState& x, uint32_t E, uint32_t ncnt, uint32_t mode) {
    if (lane == 0 && wid == 0 && P.trace && levels < P.b.trace_cap) {
      LevelTraceDev& t = P.b.trace[levels];
      t.side = (uint32_t)q;
      t.depth = (uint32_t)x.depth;
      t.frontier = x.cnt;
      t.mode = mode;
      t.edges = E;
      t.discovered = ncnt;
    }
  };
  // apply a finished level of side q to the replicated state
  auto apply = [&](int q, uint32_t E, uint32_t nxt, uint32_t noff, uint32_t ncnt, uint32_t necl, uint32_t mode) {
    SideState x = sel(q, s0, s1);
    record_trace(q, x, E, ncnt, mode);
    ++levels;
    einsp += E;
    const uint32_t qbase = x.qend;
    ++x.depth;
    x.hcnt += ncnt;
    x.qend += ncnt;
    if (ncnt) {
      x.fbeg = qbase;
      x.cur = nxt;
      x.off = noff;
    }
    x.cnt = ncnt;
    x.fed = necl;
    x.ved += necl;
    x.ovf = (unsigned long long)noff + necl > CAP ? 1u : 0u;  // records live at [noff, noff + necl)
    s0 = sel(q, x, s0);
    s1 = sel(q, s1, x);
  };

  // ---- wave 0 expands one level of side 0 (E0 records) and/or side 1 (E1
  // records) in the same instructions: lanes [0, E0) of the virtual edge list
  // are side 0, [E0, E0 + E1) side 1.  With both sides active this is a
  // lockstep round; the meet rule is the parity rule above (a claim and the
  // opposite read are ordered per lane, and one wave's LDS ops execute in
  // order, so two same-round claims of one vertex always see each other).
  // Returns the round's best meet candidate through mlen/mv/m0/m1.
  struct Dual {
    uint32_t ncnt[2], necl[2];
    uint32_t mlen, mv, m0, m1;
    uint32_t pad[2];  // kStamp: phase split
  };
  // New records of both sides go to ONE buffer: all side-0 lanes precede the
  // side-1 lanes in (batch, lane) order, so one running prefix puts side 0's
  // records at [0, necl[0]) and side 1's right after -- one scan and one
  // append per batch, and the next round reads the two runs back-to-back.
  auto dual_level = [&](uint32_t E0, uint32_t E1, uint32_t nxt) -> Dual {
    Dual out;
    out.ncnt[0] = out.ncnt[1] = out.necl[0] = out.necl[1] = 0;
    out.mlen = kEmpty;
    out.mv = kEmpty;
    out.m0 = out.m1 = 0;
    out.pad[0] = out.pad[1] = 0;
    const uint32_t ET = E0 + E1;
    if (ET == 0) return out;
    const bool both = E0 != 0 && E1 != 0;
    const uint32_t b0 = (uint32_t)s0.depth, b1 = (uint32_t)s1.depth;  // current frontier depths
    const Rec* R0 = &R[s0.cur][s0.off];
    const Rec* R1 = &R[s1.cur][s1.off];
    Rec* Nb = R[nxt];
    auto run = [&](auto bc, uint32_t base) {
      constexpr int B = decltype(bc)::value;
      uint32_t vv[B], uu[B];
      OffT ob[B], oe[B], kk[B];
      bool ok[B], sd[B], isnew[B];
      unsigned long long sp0 = 0, sp1 = 0, sp2 = 0;
      if constexpr (kStamp) sp0 = stamp();
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const uint32_t e = base + k * kWave + lane;
        ok[k] = e < ET;
        sd[k] = e >= E0;
        const uint32_t i = ok[k] ? (sd[k] ? e - E0 : e) : 0u;  // invalid lanes re-read record 0
        const Rec r = sd[k] ? R1[i] : R0[i];
        uu[k] = r.x;
        kk[k] = min(rec_k(r), P.nnz_m1);  // clamp: a bad record can never fault
      }
      fetch_edges(bc, kk, vv, ob, oe);
      if constexpr (kStamp) {
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        sp1 = stamp();
      }
      uint32_t hl = kEmpty, hv = 0, hd = 0;  // this lane's best meet: length, vertex, own claim depth
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const uint32_t a = (sd[k] ? b1 : b0) + 1;  // claim depth on this lane's side
        const uint32_t bo = sd[k] ? b0 : b1;       // opposite side's frontier depth
        uint32_t f;  // opposite state: 0 absent, else 1 + parity (3 = an older claim)
        if constexpr (kBm) {
          isnew[k] = ok[k] && bm_claim(W(sd[k]), vv[k], a & 1);
          f = isnew[k] ? bm_state(W(!sd[k]), vv[k]) : 0u;
        } else {
          isnew[k] = ok[k] && hash_insert(sd[k] ? H[1] : H[0], vv[k], vv[k] | ((a & 1) ? kParity : 0u));
          const uint32_t key = isnew[k] ? hash_find(sd[k] ? H[0] : H[1], vv[k]) : kEmpty;
          f = key == kEmpty ? 0u : 1u + (key >> 31);
        }
        if (f != 0) {
          // opposite side idle: the hit has its frontier depth; in lockstep
          // its parity says frontier depth or the one being claimed now
          const uint32_t dob = (!both || f == 3 || (f - 1) == (bo & 1)) ? bo : bo + 1;
          if (a + dob < hl) {
            hl = a + dob;
            hv = vv[k];
            hd = sd[k] ? dob | (a << 16) : a | (dob << 16);  // (side-0 depth, side-1 depth)
          }
        }
      }
      if constexpr (kStamp) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        sp2 = stamp();
      }
      unsigned long long hm = __ballot(hl != kEmpty);
      while (hm) {  // rare: only in the meeting round
        const int l = __ffsll((long long)hm) - 1;
        hm &= hm - 1;
        const uint32_t len = __builtin_amdgcn_readlane(hl, l);
        if (len < out.mlen) {
          out.mlen = len;
          out.mv = __builtin_amdgcn_readlane(hv, l);
          const uint32_t dd = __builtin_amdgcn_readlane(hd, l);
          out.m0 = dd & 0xffffu;
          out.m1 = dd >> 16;
        }
      }
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const unsigned long long mask = __ballot(isnew[k]);
        if (!mask) continue;  // wave-uniform
        const unsigned long long m1 = __ballot(isnew[k] && sd[k]);  // side-1 lanes: the upper ones
        const OffT d = isnew[k] ? oe[k] - ob[k] : (OffT)0;
        const uint32_t dc = (uint32_t)min(d, (OffT)kDegClamp);
        const uint32_t incl = wave_incl_scan(dc);
        const uint32_t eb = out.necl[0] + out.necl[1] + incl - dc;  // one running prefix
        if (isnew[k]) {
          // queue rank within the lane's own side
          const uint32_t idx = sd[k] ? out.ncnt[1] + mbcnt64(m1) : out.ncnt[0] + mbcnt64(mask);
          const uint32_t qe = sd[k] ? s1.qend : s0.qend;
          (sd[k] ? P.b.parent[1] : P.b.parent[0])[vv[k]] = uu[k];
          if (qe + idx < P.n) (sd[k] ? P.b.queue[1] : P.b.queue[0])[qe + idx] = vv[k];
        }
        append_records(Nb, isnew[k] && (OffT)eb + d <= (OffT)CAP ? (uint32_t)d : 0u, eb, vv[k], ob[k]);
        // per-side totals: side 0's part of the scan ends at its last lane
        const uint32_t n1 = (uint32_t)__popcll(m1);
        const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
        const uint32_t e1 = __ballot(sd[k]) ? tot - __builtin_amdgcn_readlane(incl, __ffsll((long long)__ballot(sd[k])) - 1) +
                                                  __builtin_amdgcn_readlane(dc, __ffsll((long long)__ballot(sd[k])) - 1)
                                            : 0u;
        out.ncnt[0] += (uint32_t)__popcll(mask) - n1;
        out.ncnt[1] += n1;
        out.necl[0] += tot - e1;
        out.necl[1] += e1;
      }
      if constexpr (kStamp) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        const unsigned long long sp3 = stamp();
        auto c16 = [](unsigned long long d) { return (uint32_t)(d > 0xffff ? 0xffff : d); };
        out.pad[0] = c16(sp1 - sp0);
        out.pad[1] = c16(sp2 - sp1) | (c16(sp3 - sp2) << 16);
      }
    };
    if (ET <= (uint32_t)kWave) {
      run(std::integral_constant<int, 1>{}, 0u);
    } else if (ET <= 2u * kWave) {
      run(std::integral_constant<int, 2>{}, 0u);
    } else {
      for (uint32_t base = 0; base < ET; base += kWave * 4) run(std::integral_constant<int, 4>{}, base);
    }
    return out;
  };

  // ---- all-wave lockstep rounds (bitmap mode, 32-bit offsets, packed
  // adjacency; both frontiers together <= 2 x kLdsThreads edges).  The edges
  // are cut into batches of 64, side 0's batches first; wave w takes batches
  // w and w + 16, so every batch serves ONE side and the side is a scalar.
  // Per batch: one packed-adjacency load, the bitmap claim with the
  // opposite-side word read in flight beside it, then a DPP degree scan and
  // ONE packed LDS atomic that places the batch's new vertices and their edge
  // records.  One barrier per round, LDS-only.  The round
  // counters rotate over three slots, so the barrier that publishes slot r
  // also orders the reset of slot r + 2 after every read of it (round r - 1's).
  // The search state is replicated: every thread reads the same counters and
  // applies the same update.
  // Records carry the PARENT'S QUEUE INDEX (not its id) and a claim lands only
  // in the LDS queue (LQ: vertex, LP: parent's queue index) -- no global store
  // at all -- so a search that ends here walks its path in LDS.  A phase that
  // ends with the search still running (a round above 2 x kLdsThreads edges, a
  // record or LDS-queue bound) writes the global queue and parent arrays from
  // the LDS queue, rewrites the current records to vertex ids and hands the
  // state to the wave-0 schedule through s0/s1.
  __shared__ unsigned long long wctr[3][2];  // [slot][side]: (count << 32) | edge sum
  __shared__ unsigned long long wmeet[3];    // [slot]: min (len << 32 | side << 31 | vertex)
  bool lq_done = false;                      // replicated: the search ended inside wave_rounds
  auto wave_rounds = [&]() {
    if constexpr (!kWr) {
      return;
    } else {
      if ((!P.padj && !P.padj8) || !P.lockstep || (P.trace && !kStamp) || s0.ovf || s1.ovf) return;  // uniform
      if (!kLq && !P.wave_hash) return;
      uint32_t E0 = (uint32_t)s0.fed, E1 = (uint32_t)s1.fed;
      uint32_t d0 = (uint32_t)s0.depth, d1 = (uint32_t)s1.depth;
      uint32_t qe0 = s0.qend, qe1 = s1.qend, c0 = s0.cnt, c1 = s1.cnt, h0 = s0.hcnt, h1 = s1.hcnt;
      unsigned long long v0 = s0.ved, v1 = s1.ved;
      uint32_t a0 = s0.cur, o0 = s0.off, a1 = s1.cur, o1 = s1.off;  // current records
      uint32_t* const par0 = P.b.parent[0];
      uint32_t* const par1 = P.b.parent[1];
      uint32_t* const que0 = P.b.queue[0];
      uint32_t* const que1 = P.b.queue[1];
      unsigned long long* const W0 = W(0);
      unsigned long long* const W1 = W(1);
      const uint4* const padj = P.padj;
      if (tid < 6) wctr[tid >> 1][tid & 1] = 0;
      if (tid < 3) wmeet[tid] = ~0ull;
      if constexpr (kLq) {
        if (tid < 2) {  // depth 0: the endpoints at queue index 0
          LQ[tid][0] = tid ? P.dst : P.src;
          LP[tid][0] = kEmpty;
        }
        for (uint32_t i = tid; i < E0 + E1; i += kLdsThreads) {  // seed records: parent = queue index 0
          if (i < E0) R[a0][o0 + i].x = 0u;
          else R[a1][o1 + i - E0].x = 0u;
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      uint32_t slot = 0, rounds_done = 0;
      uint32_t X0 = 0, X1 = 0;  // edges each side expands this round (0: the side idles)
      auto round = [&](auto bc, uint32_t nb0, uint32_t nbt, uint32_t x0, uint32_t x1) {
        constexpr int B = decltype(bc)::value;
        unsigned long long lt0 = 0, lt1 = 0, lsub = 0;  // kStamp: round start / work done / sub-phases
        if constexpr (kStamp) lt0 = stamp();
        auto sub = [&](int k) {  // kStamp: cycles since the previous mark into 16-bit field k
          if constexpr (kStamp) {
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            const unsigned long long t = stamp();
            lsub |= min(t - (k ? lt1 : lt0), 0xffffull) << (16 * k);
            lt1 = t;
          }
        };
        const uint32_t wv = uni((uint32_t)tid >> 6);
        if (wv >= nbt) return lsub;  // wave-uniform: no batch this round, only the barrier
        bool act[B], sd[B], ok[B], isnew[B];
        uint32_t u[B], v[B], dg[B], ob[B];
        unsigned long long old[B], w[B];
#pragma unroll
        for (int k = 0; k < B; ++k) {  // records -> packed adjacency loads, all in flight
          const uint32_t bt = wv + (uint32_t)k * (kLdsThreads / kWave);
          act[k] = bt < nbt;  // scalar
          sd[k] = bt >= nb0;  // scalar
          const uint32_t e = (bt - (sd[k] ? nb0 : 0u)) * kWave + lane;
          ok[k] = act[k] && e < (sd[k] ? X1 : X0);
          const Rec r = (sd[k] ? &R[a1][o1] : &R[a0][o0])[ok[k] ? e : 0u];
          u[k] = r.x;
          if (P.padj8) {  // kernel argument: uniform
            const unsigned long long w = P.padj8[min(r.y, P.nnz_m1)];
            v[k] = launch::pack8_v(w);
            dg[k] = launch::pack8_deg(w);
            ob[k] = launch::pack8_base(w);
          } else {
            const uint4 pq = padj[min(r.y, P.nnz_m1)];
            v[k] = pq.x;
            dg[k] = pq.y;
            ob[k] = pq.z;
          }
        }
        sub(0);
#pragma unroll
        for (int k = 0; k < B; ++k) {  // claims, the opposite words beside them
          const uint32_t a = (sd[k] ? d1 : d0) + 1;
          old[k] = ~0ull;
          if constexpr (kBm) {
            const uint32_t bit = v[k] & 31u;
            if (ok[k]) old[k] = atomicOr(&(sd[k] ? W1 : W0)[v[k] >> 5], 1ull << (bit + ((a & 1u) << 5)));
            w[k] = (sd[k] ? W0 : W1)[v[k] >> 5];
          } else {
            // hash sets: insert (key = id | parity of the claim depth), then
            // the opposite table's key; old/w carry "new" and that key
            const bool ins = ok[k] && hash_insert(sd[k] ? H[1] : H[0], v[k], v[k] | ((a & 1u) ? kParity : 0u));
            old[k] = ins ? 0ull : ~0ull;
            w[k] = ins ? hash_find(sd[k] ? H[0] : H[1], v[k]) : kEmpty;
          }
        }
        unsigned long long best = ~0ull;
#pragma unroll
        for (int k = 0; k < B; ++k) {
          const uint32_t a = (sd[k] ? d1 : d0) + 1;
          const uint32_t bo = sd[k] ? d0 : d1;  // opposite frontier depth (lockstep: parity rule)
          uint32_t f;  // opposite state: 0 absent, else 1 + parity (3 = an older claim)
          if constexpr (kBm) {
            const uint32_t bit = v[k] & 31u;
            isnew[k] = ((old[k] >> bit) & 0x100000001ull) == 0;
            f = (uint32_t)((w[k] >> bit) & 1ull) | ((uint32_t)((w[k] >> (32 + bit)) & 1ull) << 1);
          } else {
            isnew[k] = old[k] == 0ull;
            f = w[k] == kEmpty ? 0u : 1u + (uint32_t)(w[k] >> 31);
          }
          if (isnew[k] && f != 0) {
            const uint32_t dob = (f == 3 || (f - 1) == (bo & 1u)) ? bo : bo + 1;
            const unsigned long long key = ((unsigned long long)(a + dob) << 32) | ((sd[k] ? 1ull : 0ull) << 31) | v[k];
            best = key < best ? key : best;
          }
        }
        sub(1);
        if (__ballot(best != ~0ull)) {  // the meeting round only
          unsigned long long m = best;
          for (int off = 32; off >= 1; off >>= 1) {
            const unsigned long long y = __shfl_xor(m, off);
            m = y < m ? y : m;
          }
          if (lane == 0) atomicMin(&wmeet[slot], m);
        }
#pragma unroll
        for (int k = 0; k < B; ++k) {
          const unsigned long long mask = __ballot(isnew[k]);
          if (!mask) continue;  // wave-uniform
          const uint32_t dc = isnew[k] ? min(dg[k], kDegClamp) : 0u;
          const uint32_t incl = wave_incl_scan(dc);
          const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
          // a side served by one batch owns its counter: a plain store, no atomic round trip
          const bool alone = sd[k] ? nbt - nb0 == 1 : nb0 == 1;  // scalar
          const unsigned long long add = ((unsigned long long)__popcll(mask) << 32) | tot;
          unsigned long long pos = 0;
          if (alone) {
            if (lane == 0) wctr[slot][sd[k] ? 1 : 0] = add;
          } else if (lane == 0) {
            pos = atomicAdd(&wctr[slot][sd[k] ? 1 : 0], add);
          }
          const uint32_t be = alone ? 0u : __builtin_amdgcn_readlane((uint32_t)pos, 0);
          const uint32_t bn = alone ? 0u : __builtin_amdgcn_readlane((uint32_t)(pos >> 32), 0);
          const uint32_t eb = be + incl - dc;
          const uint32_t qi = (sd[k] ? qe1 : qe0) + bn + mbcnt64(mask);  // kLq: < kQCap (round bound)
          if constexpr (kLq) {
            if (isnew[k]) {
              (sd[k] ? LP[1] : LP[0])[qi] = u[k];
              (sd[k] ? LQ[1] : LQ[0])[qi] = v[k];
            }
          } else if (isnew[k]) {  // global queue and parents; records carry the parent's id
            (sd[k] ? par1 : par0)[v[k]] = u[k];
            if (qi < P.n) (sd[k] ? que1 : que0)[qi] = v[k];
          }
          if (k == 0) sub(2);
          append_records(sd[k] ? R[x1] : R[x0], isnew[k] && eb + dg[k] <= CAP ? dg[k] : 0u, eb, kLq ? qi : v[k],
                         ob[k]);
        }
        sub(3);
        return lsub;
      };
      constexpr uint32_t kMaxBatches = kWaveB * (kLdsThreads / kWave);
      for (;;) {
        if (status != kRunning || E0 == 0 || E1 == 0) break;
        // A side can expand here when its records are all in LDS (E <= CAP),
        // its batches fit the waves and every claim fits the LDS queue (a side
        // claims at most E new vertices).  Both sides when both fit together
        // (lockstep: one round per two levels); otherwise the side with fewer
        // edges alone while it fits -- an unbalanced pair (one frontier past the
        // queue or record bound) then still ends in LDS instead of handing the
        // search to the wave-0 schedule.  The meet rule covers an idle side.
        const uint32_t nb0e = (E0 + kWave - 1) / kWave, nb1e = (E1 + kWave - 1) / kWave;
        const bool f0 = E0 <= CAP && nb0e <= kMaxBatches && (!kLq || qe0 + E0 <= kQCap) && (kBm || h0 + E0 <= kHashLimit);
        const bool f1 = E1 <= CAP && nb1e <= kMaxBatches && (!kLq || qe1 + E1 <= kQCap) && (kBm || h1 + E1 <= kHashLimit);
        bool run0 = f0, run1 = f1;
        if (!(f0 && f1 && nb0e + nb1e <= kMaxBatches)) {
          if (!kWaveSingle || !(f0 || f1)) break;
          run0 = f0 && (!f1 || E0 <= E1);
          run1 = !run0;
        }
        X0 = run0 ? E0 : 0u;
        X1 = run1 ? E1 : 0u;
        const uint32_t ET = X0 + X1;
        const uint32_t nb0 = run0 ? nb0e : 0u, nbt = nb0 + (run1 ? nb1e : 0u);
        const uint32_t used = (1u << a0) | (1u << a1);
        const uint32_t x0 = (uint32_t)__builtin_ctz(~used & 0xfu);
        const uint32_t x1 = (uint32_t)__builtin_ctz(~(used | (1u << x0)) & 0xfu);
        unsigned long long rt0r = 0, lsub = 0;
        if constexpr (kStamp) rt0r = stamp();
        if (kWaveB == 1 || nbt <= (uint32_t)(kLdsThreads / kWave))
          lsub = round(std::integral_constant<int, 1>{}, nb0, nbt, x0, x1);
        else if (kWaveB == 2 || nbt <= 2u * (kLdsThreads / kWave))
          lsub = round(std::integral_constant<int, (kWaveB > 1 ? 2 : 1)>{}, nb0, nbt, x0, x1);
        else
          lsub = round(std::integral_constant<int, (kWaveB > 2 ? 4 : 1)>{}, nb0, nbt, x0, x1);
        unsigned long long rt1r = 0;
        if constexpr (kStamp) rt1r = stamp();
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // LDS-only: stores stay in flight
        const unsigned long long p0 = wctr[slot][0], p1 = wctr[slot][1], mk = wmeet[slot];
        const uint32_t sn = slot == 2 ? 0u : slot + 1, sr = sn == 2 ? 0u : sn + 1;
        if (tid < 2) wctr[sr][tid] = 0;
        if (tid == 2) wmeet[sr] = ~0ull;
        const uint32_t n0 = uni((uint32_t)(p0 >> 32)), l0 = uni((uint32_t)p0);
        const uint32_t n1 = uni((uint32_t)(p1 >> 32)), l1 = uni((uint32_t)p1);
        const uint32_t mk_hi = uni((uint32_t)(mk >> 32)), mk_lo = uni((uint32_t)mk);
        if (mk_hi != 0xffffffffu && (meet == kEmpty || mk_hi < md0 + md1)) {
          const uint32_t side = mk_lo >> 31;
          const uint32_t a = (side ? d1 : d0) + 1;
          meet = mk_lo & kIdMask;
          md0 = side ? mk_hi - a : a;
          md1 = side ? a : mk_hi - a;
        }
        if constexpr (kStamp) {
          const uint32_t lv = levels + (run0 && run1 ? 1u : 0u);
          if (tid == 0 && lv < P.b.trace_cap) {
            LevelTraceDev& t = P.b.trace[lv];
            const unsigned long long rt2r = stamp();
            t.side = (uint32_t)(rt2r - rt0r);
            t.depth = (uint32_t)(rt1r - rt0r);
            t.frontier = (uint32_t)(rt2r - rt1r);
            t.mode = 8;
            t.edges = ET;
            t.discovered = lsub;
          }
        }
        levels += (run0 ? 1u : 0u) + (run1 ? 1u : 0u);
        einsp += ET;
        ++rounds_done;
        if (run0) {  // an idle side keeps its frontier, records and counts
          ++d0, qe0 += n0, h0 += n0, c0 = n0, v0 += l0, E0 = l0, a0 = x0, o0 = 0;
        }
        if (run1) {
          ++d1, qe1 += n1, h1 += n1, c1 = n1, v1 += l1, E1 = l1, a1 = x1, o1 = 0;
        }
        if (meet != kEmpty) status = kFound;
        else if ((run0 && n0 == 0) || (run1 && n1 == 0)) status = kNoPath;
        slot = sn;
      }
      if (!kLq) {
        // global queue and parents all along: nothing to materialise, the path
        // is walked along the global parent arrays.  The wave-0 schedule may
        // read queue entries other waves wrote (rebuild, meet probe: L2
        // loads), so every wave's stores complete before it goes on alone --
        // __syncthreads() alone waits for no store on gfx950.
        if (status == kRunning && rounds_done) asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      } else if (status != kRunning) {
        lq_done = true;  // the path is walked in LDS
      } else {
        // the wave-0 schedule continues: it needs the global queue and parent
        // arrays (the hand-off, the global path walk) and records that carry
        // parent ids -- both materialised here from the LDS queue
        for (uint32_t i = tid; i < qe0 + qe1; i += kLdsThreads) {
          const int q = i >= qe0;
          const uint32_t j = q ? i - qe0 : i;
          if (j == 0) continue;  // the endpoints: written by init_side
          const uint32_t x = LQ[q][j];
          (q ? par1 : par0)[x] = LQ[q][LP[q][j]];
          if (j < P.n) (q ? que1 : que0)[j] = x;
        }
        for (uint32_t i = tid; i < E0 + E1; i += kLdsThreads) {
          if (i < E0) {
            if (o0 + i < CAP) R[a0][o0 + i].x = LQ[0][R[a0][o0 + i].x];
          } else if (o1 + i - E0 < CAP) {
            R[a1][o1 + i - E0].x = LQ[1][R[a1][o1 + i - E0].x];
          }
        }
        // (the queue / parent stores complete too: see the !kLq case)
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
      }
      if (rounds_done == 0) return;
      s0.cur = a0, s0.off = o0, s0.fed = E0, s0.depth = (int)d0, s0.fbeg = qe0 - c0, s0.qend = qe0;
      s0.cnt = c0, s0.hcnt = h0, s0.ved = v0, s0.ovf = E0 > CAP ? 1u : 0u;
      s1.cur = a1, s1.off = o1, s1.fed = E1, s1.depth = (int)d1, s1.fbeg = qe1 - c1, s1.qend = qe1;
      s1.cnt = c1, s1.hcnt = h1, s1.ved = v1, s1.ovf = E1 > CAP ? 1u : 0u;
    }
  };

  // Wave 0: side q's level records were lost -- a lockstep round puts side
  // 1's records after side 0's in one buffer, so a big side 0 overflowed a
  // small side 1 with it -- but the level itself is small: rebuild them from
  // the global queue into a free buffer (queue entry -> row, one wave-wide
  // degree scan, cooperative appends), so the search stays in LDS instead of
  // handing a level of a few dozen edges to the grid.  At most kRebuildMax
  // frontier vertices (their loads all in flight at once).  true = rebuilt.
  auto rebuild = [&](int q) -> bool {
    constexpr uint32_t kRebuildMax = 4 * kWave;
    SideState x = sel(q, s0, s1);
    if (!x.ovf || x.cnt > kRebuildMax || x.fed > CAP || !(kBm || x.hcnt + x.fed <= kHashLimit)) return false;
    const uint32_t buf = free_buf();
    const uint32_t* qu = q ? P.b.queue[1] : P.b.queue[0];
    // wave 0's own queue stores complete (other waves drained theirs before
    // the barrier that left wave 0 alone)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t u[4], d[4];
    OffT b[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = (uint32_t)j * kWave + lane;
      u[j] = i < x.cnt ? load_agent(&qu[x.fbeg + i]) : 0u;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = (uint32_t)j * kWave + lane;
      b[j] = 0;
      d[j] = 0;
      if (i < x.cnt) {
        b[j] = P.row_off[u[j]];
        d[j] = (uint32_t)min((OffT)(P.row_off[u[j] + 1] - b[j]), (OffT)CAP + 1);
      }
    }
    uint32_t run = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t incl = wave_incl_scan(d[j]);
      const uint32_t eb = run + incl - d[j];
      append_records(R[buf], eb + d[j] <= CAP ? d[j] : 0u, eb, u[j], b[j]);
      run += __builtin_amdgcn_readlane(incl, 63);
    }
    if (uni(run) != (uint32_t)x.fed) return false;  // (never: fed is this frontier's degree sum)
    x.cur = buf;
    x.off = 0;
    x.ovf = 0;
    s0 = sel(q, x, s0);
    s1 = sel(q, s1, x);
    return true;
  };

  unsigned long long clk0 = 0;
  // the search's start stamp waits in LDS for the publish (held in registers
  // across the search it was the kernel's one VGPR spill)
  __shared__ unsigned long long rt0_lds;
  if (tid == 0) rt0_lds = __builtin_amdgcn_s_memrealtime();
  if (kStamp && tid == 0) clk0 = __builtin_amdgcn_s_memtime();
  wave_rounds();  // every wave; the replicated state continues below
  uint32_t fstatus = kRunning;
  bool probed = false, probe_hit = false;
  uint32_t probe_walked = 0;
  for (;;) {
    if (wid == 0) {
      // ---- wave 0 alone: dual-side (lockstep) and single-side rounds while
      // the frontiers are small; no barrier, the other waves stay parked
      for (;;) {
        if (status != kRunning) break;
        const bool f0 = fits(s0), f1 = fits(s1);
        int q;
        if (P.side_policy == 2) q = turn;
        else if (P.side_policy == 1) q = s0.cnt <= s1.cnt ? 0 : 1;
        else q = s0.fed <= s1.fed ? 0 : 1;
        const bool dual = P.lockstep && f0 && f1 && s0.fed + s1.fed <= kDualEdges;
        const bool fq = q ? f1 : f0;
        const unsigned long long eq = q ? s1.fed : s0.fed;
        if (!dual && (!fq || eq > kSmallEdges)) {
          if (!fq && rebuild(q)) continue;  // a small level whose records were lost: rebuilt, stays in LDS
          // a level that does not fit: probe it for a meet first (hub graphs)
          if (!fq) status = (P.probe && !P.batch && !probed) ? kProbing : kHandoff;
          break;  // big level (all waves), probe or hand-off
        }
        unsigned long long ts0 = 0;
        if (kStamp && tid == 0) ts0 = stamp();
        const uint32_t E0 = dual || q == 0 ? (uint32_t)s0.fed : 0u;
        const uint32_t E1 = dual || q == 1 ? (uint32_t)s1.fed : 0u;
        const uint32_t nb = free_buf();
        const Dual w = dual_level(E0, E1, nb);
        if (w.mlen != kEmpty && (meet == kEmpty || w.mlen < md0 + md1)) {
          meet = w.mv;
          md0 = w.m0;
          md1 = w.m1;
        }
        if (dual) {
          apply(0, E0, nb, 0u, w.ncnt[0], w.necl[0], 1);
          apply(1, E1, nb, w.necl[0], w.ncnt[1], w.necl[1], 1);
          if (meet != kEmpty) status = kFound;
          else if (s0.cnt == 0 || s1.cnt == 0) status = kNoPath;
        } else {
          apply(q, q ? E1 : E0, nb, 0u, q ? w.ncnt[1] : w.ncnt[0], q ? w.necl[1] : w.necl[0], 2);  // no runtime index
          if (P.side_policy == 2) turn ^= 1;
          if (meet != kEmpty) status = kFound;
          else if ((q ? s1.cnt : s0.cnt) == 0) status = kNoPath;
        }
        if (kStamp && tid == 0 && levels - 1 < P.b.trace_cap) {
          LevelTraceDev& t = P.b.trace[levels - 1];
          t.side = (uint32_t)(stamp() - ts0);
          t.depth = 0;
          t.frontier = 0;
          t.mode = dual ? 1 : 2;
          t.edges = (unsigned long long)w.pad[0] | ((unsigned long long)w.pad[1] << 32);
        }
      }
      // publish the plan for a big level (or the end): both sides in lockstep
      // while both fit and are balanced (one pass of 1024 lanes, or within 2x),
      // else the policy's side
      if (lane == 0) {
        int q;
        if (P.side_policy == 2) q = turn;
        else if (P.side_policy == 1) q = s0.cnt <= s1.cnt ? 0 : 1;
        else q = s0.fed <= s1.fed ? 0 : 1;
        const unsigned long long lo = min(s0.fed, s1.fed), hi = max(s0.fed, s1.fed);
        const bool both = P.lockstep && fits(s0) && fits(s1) &&
                          (lo + hi <= (unsigned long long)kLdsThreads || (hi <= 2 * lo && lo + hi <= kDualBigEdges));
        LevelPlan p;
        p.status = status;
        const uint32_t fa = free_buf();
        const uint32_t fb = (uint32_t)__builtin_ctz(~((1u << s0.cur) | (1u << s1.cur) | (1u << fa)) & 0xfu);
        p.E[0] = both || q == 0 ? (uint32_t)s0.fed : 0u;
        p.E[1] = both || q == 1 ? (uint32_t)s1.fed : 0u;
        p.cur[0] = s0.cur, p.cur[1] = s1.cur;
        p.off[0] = s0.off, p.off[1] = s1.off;
        p.nxt[0] = fa;
        p.nxt[1] = both ? fb : fa;
        p.qbase[0] = s0.qend, p.qbase[1] = s1.qend;
        p.depth[0] = (uint32_t)s0.depth, p.depth[1] = (uint32_t)s1.depth;
        p.pside = (uint32_t)q;
        p.pfb = q ? s1.fbeg : s0.fbeg;
        p.pcnt = q ? s1.cnt : s0.cnt;
        p.prec = (q ? s1.ovf : s0.ovf) ? 0u : (uint32_t)(q ? s1.fed : s0.fed);  // records in LDS: their count
        plan = p;
      }
    }
    __syncthreads();  // B1: parked waves released for a big level, or for the exit
    unsigned long long ts0 = 0, ts1 = 0, ts2 = 0;
    if (kStamp && tid == 0) ts0 = stamp();
    fstatus = uni(plan.status);
    if (fstatus == kProbing) {
      const int pq = (int)uni(plan.pside);
      uint32_t walked = 0;
      const uint32_t nrec = uni(plan.prec);
      const Rec* recs = nrec ? &R[uni(plan.cur[pq])][uni(plan.off[pq])] : nullptr;
      // the chunk path's scratch: a record buffer the level's records are not in
      const uint32_t sbuf = (uint32_t)__builtin_ctz(~(1u << uni(plan.cur[pq])) & 0xfu);
      const unsigned long long hit =
          lds_meet_probe<OffT, kBm, Rec>(P, pq, uni(plan.pfb), uni(plan.pcnt), recs, nrec, P.probe,
                                         pq ? H[0] : H[1], W(pq ^ 1), &R[sbuf][0], &walked);
      probed = true;
      probe_walked = walked;
      if (wid == 0) {
        if (hit != ~0ull) {
          const uint32_t u = (uint32_t)(hit >> 32), v = (uint32_t)hit;
          const uint32_t dq = pq ? (uint32_t)s1.depth : (uint32_t)s0.depth;
          const uint32_t dob = pq ? (uint32_t)s0.depth : (uint32_t)s1.depth;
          if (lane == 0) (pq ? P.b.parent[1] : P.b.parent[0])[v] = u;  // the claim the probe did not make
          meet = v;
          md0 = pq ? dob : dq + 1;
          md1 = pq ? dq + 1 : dob;
          record_trace(pq, sel(pq, s0, s1), walked, 1u, 9u);  // mode 9: a level the probe ended
          ++levels;
          einsp += walked;
          status = kFound;
          probe_hit = true;
        } else {
          status = kHandoff;
        }
      }
      continue;  // wave 0 publishes the final plan at the top of the loop
    }
    if (fstatus != kRunning) break;
    // ---- big level: every wave, one edge per lane; side 0's records then side
    // 1's (virtual list as in dual_level); per-side LDS counters place the
    // appends, one packed atomicMin keeps the shortest meet candidate
    const uint32_t E0 = uni(plan.E[0]), E1 = uni(plan.E[1]);
    const uint32_t ET = E0 + E1;
    const bool bboth = E0 != 0 && E1 != 0;
    const uint32_t bd0 = uni(plan.depth[0]), bd1 = uni(plan.depth[1]);
    const uint32_t qb0 = uni(plan.qbase[0]), qb1 = uni(plan.qbase[1]);
    const Rec* Rc0 = &R[uni(plan.cur[0])][uni(plan.off[0])];
    const Rec* Rc1 = &R[uni(plan.cur[1])][uni(plan.off[1])];
    Rec* Rn0 = R[uni(plan.nxt[0])];
    Rec* Rn1 = R[uni(plan.nxt[1])];
    const uint32_t slot = bigs & 1;  // double-buffered: wave 0 reads it after B2
    auto batch = [&](auto bc, uint32_t base) {
      constexpr int B = decltype(bc)::value;
      uint32_t vv[B], uu[B];
      OffT ob[B], oe[B];
      bool ok[B], sd[B];
      OffT kk[B];
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const uint32_t e = base + k * kLdsThreads + tid;
        ok[k] = e < ET;
        sd[k] = e >= E0;
        const uint32_t i = ok[k] ? (sd[k] ? e - E0 : e) : 0u;
        const Rec r = sd[k] ? Rc1[i] : Rc0[i];
        uu[k] = r.x;
        kk[k] = min(rec_k(r), P.nnz_m1);
      }
      fetch_edges(bc, kk, vv, ob, oe);
      bool isnew[B];
      unsigned long long best = ~0ull;
#pragma unroll
      for (int k = 0; k < B; ++k) {
        const uint32_t a = (sd[k] ? bd1 : bd0) + 1;
        const uint32_t bo = sd[k] ? bd0 : bd1;
        uint32_t f;
        if constexpr (kBm) {
          isnew[k] = ok[k] && bm_claim(W(sd[k]), vv[k], a & 1);
          f = isnew[k] ? bm_state(W(!sd[k]), vv[k]) : 0u;
        } else {
          isnew[k] = ok[k] && hash_insert(sd[k] ? H[1] : H[0], vv[k], vv[k] | ((a & 1) ? kParity : 0u));
          const uint32_t key = isnew[k] ? hash_find(sd[k] ? H[0] : H[1], vv[k]) : kEmpty;
          f = key == kEmpty ? 0u : 1u + (key >> 31);
        }
        if (f != 0) {
          const uint32_t dob = (!bboth || f == 3 || (f - 1) == (bo & 1)) ? bo : bo + 1;
          const unsigned long long key = ((unsigned long long)(a + dob) << 32) | ((sd[k] ? 1ull : 0ull) << 31) | vv[k];
          best = key < best ? key : best;
        }
      }
      if (__ballot(best != ~0ull)) {  // rare: the meeting level
        unsigned long long m = best;
        for (int off = 32; off >= 1; off >>= 1) {
          const unsigned long long y = __shfl_xor(m, off);
          m = y < m ? y : m;
        }
        if (lane == 0) atomicMin(&meetk[slot], m);
      }
#pragma unroll
      for (int k = 0; k < B; ++k) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bool mine = isnew[k] && sd[k] == (q == 1);
          const unsigned long long mask = __ballot(mine);
          if (!mask) continue;  // wave-uniform
          const OffT d = mine ? oe[k] - ob[k] : (OffT)0;
          const uint32_t dc = (uint32_t)min(d, (OffT)kDegClamp);
          const uint32_t incl = wave_incl_scan(dc);
          const uint32_t wtot = __builtin_amdgcn_readlane(incl, 63);
          const int leader = __ffsll((long long)mask) - 1;
          unsigned long long old = 0;
          if (lane == (uint32_t)leader)
            old = atomicAdd(&ctr[slot][q], ((unsigned long long)__popcll(mask) << 32) | wtot);
          const uint32_t olo = __builtin_amdgcn_readlane((uint32_t)old, leader);
          const uint32_t ohi = __builtin_amdgcn_readlane((uint32_t)(old >> 32), leader);
          const uint32_t eb = olo + incl - dc;
          if (mine) {
            const uint32_t idx = ohi + mbcnt64(mask);
            const uint32_t qb = q ? qb1 : qb0;
            (q ? P.b.parent[1] : P.b.parent[0])[vv[k]] = uu[k];
            if (qb + idx < P.n) (q ? P.b.queue[1] : P.b.queue[0])[qb + idx] = vv[k];
          }
          append_records(q ? Rn1 : Rn0, mine && (OffT)eb + d <= (OffT)CAP ? (uint32_t)d : 0u, eb, vv[k], ob[k]);
        }
      }
    };
    if (ET <= (uint32_t)kLdsThreads) {
      if ((uint32_t)wid * kWave < ET) batch(std::integral_constant<int, 1>{}, 0u);
    } else {
      for (uint32_t base = 0; base < ET; base += kLdsThreads * kBatch)
        if (base + (uint32_t)wid * kWave < ET) batch(std::integral_constant<int, kBatch>{}, base);
    }
    if (kStamp && tid == 0) ts1 = stamp();
    // B2: every claim of the big level is in LDS, and its queue / parent
    // stores are complete (wave 0 may read queue entries next: rebuild, probe)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kStamp && tid == 0) ts2 = stamp();
    if (wid == 0) {
      const unsigned long long p0 = ctr[slot][0], p1 = ctr[slot][1];
      const unsigned long long mk = meetk[slot];
      // the other slot is used by the next big level (wave 0 read it one big
      // level ago)
      // (the lane index re-read: an address derived from `lane` was kept live
      // across the search, a spill in the 64-bit-offset kernel)
      uint32_t l = __lane_id();
      asm volatile("" : "+v"(l));
      if (l < 2) ctr[slot ^ 1][l] = 0;
      if (lane == 0) meetk[slot ^ 1] = ~0ull;
      const uint32_t mk_hi = uni((uint32_t)(mk >> 32)), mk_lo = uni((uint32_t)mk);
      if (mk != ~0ull && (meet == kEmpty || mk_hi < md0 + md1)) {
        const uint32_t side = mk_lo >> 31;
        const uint32_t a = (side ? bd1 : bd0) + 1;
        meet = mk_lo & kIdMask;
        md0 = side ? mk_hi - a : a;
        md1 = side ? a : mk_hi - a;
      }
      const uint32_t n0 = uni((uint32_t)(p0 >> 32)), l0 = uni((uint32_t)p0);
      const uint32_t n1 = uni((uint32_t)(p1 >> 32)), l1 = uni((uint32_t)p1);
      const uint32_t nb0 = uni(plan.nxt[0]), nb1 = uni(plan.nxt[1]);
      if (E0) apply(0, E0, nb0, 0u, n0, l0, 3);
      if (E1) apply(1, E1, nb1, 0u, n1, l1, 3);
      if (!bboth && P.side_policy == 2) turn ^= 1;
      if (meet != kEmpty) status = kFound;
      else if ((E0 && n0 == 0) || (E1 && n1 == 0)) status = kNoPath;
      if (kStamp && tid == 0 && levels - 1 < P.b.trace_cap) {
        LevelTraceDev& t = P.b.trace[levels - 1];
        t.side = (uint32_t)(ts1 - ts0);
        t.depth = (uint32_t)(ts2 - ts1);
        t.frontier = (uint32_t)(stamp() - ts2);
        t.mode = 3;
      }
    }
    ++bigs;  // every wave: the slot parity must agree across the workgroup
  }
  if (kStamp && tid == 0 && P.b.trace_cap > 1) {
    LevelTraceDev& t = P.b.trace[P.b.trace_cap - 1];
    e3 = __builtin_amdgcn_s_memtime();
    t.edges = e3 - clk0;
    t.discovered = __builtin_amdgcn_s_memrealtime() - rt0_lds;
  }

  // search state is valid in wave 0; fstatus (from the final plan) in every wave
  HostResult* Rr = P.h.res;
  if (kLq && lq_done && status == kFound) {
    // the meet vertex's queue index on each side: one parallel LDS search
    for (uint32_t i = tid; i < s0.qend + s1.qend; i += kLdsThreads) {
      const int q = i >= s0.qend;
      const uint32_t j = q ? i - s0.qend : i;
      if (j < kQCap && LQ[q][j] == meet) lq_meet[q] = j;
    }
  } else {
    // Parent stores of every wave must have reached L2 before the walkers'
    // L1-bypassing loads read them.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (wid == 0) {
    const uint32_t hops = md0 + md1;
    const uint32_t path_len = status == kFound ? hops + 1 : 0u;
    const bool path_dev = status == kFound && path_len > P.h.path_cap && !P.batch;
    const bool path_skip = status == kFound && path_len > P.h.path_cap && P.batch;  // host re-runs it
    // Two lanes walk the two parent chains side by side into LDS (the record
    // buffers are free now); then the whole wave streams the path to the
    // pinned host buffer with write-through stores, 64 entries per instruction.
    uint32_t* pbuf = reinterpret_cast<uint32_t*>(&R[0][0]);
    constexpr uint32_t kPbufCap = sizeof(R) / sizeof(uint32_t);
    const bool staged = !path_dev && !path_skip && path_len <= kPbufCap;
    // (staged and unstaged walks are separate calls: one pointer selected
    // between LDS and global memory would make every path store a flat store)
    auto walk = [&](uint32_t* out) {
      if (kLq && lq_done) {
        // LDS walk: lane 0 from the meet back to the source (positions md0 .. 0),
        // lane 1 on to the target (md0 .. md0 + md1), one LDS load per hop
        uint32_t i = lq_meet[tid];
        int pos = (int)md0;
        for (int remain = tid ? (int)md1 : (int)md0;; --remain) {
          out[pos] = LQ[tid][i];
          if (remain == 0) break;
          i = LP[tid][i];
          if (i >= kQCap) break;  // never: every claim's parent index is in the queue
          pos += tid ? 1 : -1;
        }
      } else {
        walk_side(tid ? P.b.parent[1] : P.b.parent[0], P.n, meet, tid, (int)md0, (int)md1, out);
      }
    };
    if (status == kFound && !path_skip && tid < 2) {
      if (staged) walk(pbuf);
      else walk(path_dev ? P.b.dpath : P.h.path);
    }
    if (staged) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (uint32_t i = lane; i < path_len; i += kWave)
        __hip_atomic_store(&P.h.path[i], pbuf[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (kStamp && tid == 0) e4 = __builtin_amdgcn_s_memtime();
    // Hand-off state and result record: lane 0 builds both images in LDS, then
    // every lane stores one word -- one store instruction per record instead of
    // ~30 serial single-lane stores (~4k cycles of a 10M hand-off).
    const bool hand = status == kHandoff && !P.batch;
    constexpr uint32_t kStW = (uint32_t)(sizeof(DevState) / 4), kMirW = (uint32_t)(offsetof(DevState, pad) / 4);
    constexpr uint32_t kResW = (uint32_t)(offsetof(HostResult, rt_pickup) / 4);
    static_assert(kStW <= 32 && kResW <= 32, "one lane per word");
    if (lane == 0) {
      DevState& sv = *reinterpret_cast<DevState*>(&pub_img[0]);
      if (hand) {
        sv = DevState{};
        sv.status = kRunning;
        sv.meet = kEmpty;
        sv.levels = levels;
        sv.einsp = einsp;
        for (int q = 0; q < 2; ++q) {
          const SideState x = sel(q, s0, s1);
          sv.depth[q] = x.depth;
          sv.fbeg[q] = x.fbeg;
          sv.fend[q] = x.qend;
          sv.qtail[q] = x.qend;
          sv.fedges[q] = x.fed;
          sv.vedges[q] = x.ved;
        }
      }
      HostResult& rv = *reinterpret_cast<HostResult*>(&pub_img[32]);
      rv.status = status;
      rv.hops = status == kFound ? (int32_t)hops : -1;
      rv.meet = meet;
      rv.levels = levels;
      rv.lds_levels = levels;
      rv.visited = s0.hcnt + s1.hcnt;
      rv.einsp = einsp;
      rv.depth[0] = status == kFound ? (int32_t)md0 : s0.depth;
      rv.depth[1] = status == kFound ? (int32_t)md1 : s1.depth;
      rv.path_len = path_len;
      rv.path_on_device = path_dev ? 1u : path_skip ? 2u : 0u;
      rv.probe = min(probe_walked, 0x7fffffffu) | (probe_hit ? 0x80000000u : 0u);
      rv.rt_begin = rt0_lds;
      rv.rt_end = __builtin_amdgcn_s_memrealtime();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // same wave: lane 0's LDS writes precede the reads
    if (hand && lane < kStW) {
      const uint32_t w = pub_img[lane];
      reinterpret_cast<uint32_t*>(P.b.st)[lane] = w;  // pad included: zero (done counter, gate words elsewhere)
      // the host continues from this mirror (no copy + sync); pad[0] is the
      // mirror's seq and stays, pad[1] (the level done counter) is cleared
      if (DevState* m = P.h.state; m && (lane < kMirW || lane == kMirW + 1))
        __hip_atomic_store(reinterpret_cast<uint32_t*>(m) + lane, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (kStamp && tid == 0) e5 = __builtin_amdgcn_s_memtime();
    // write-through (system-scope) stores: no L2 writeback needed for the host;
    // seq (word 0) is written last, below
    if (lane >= 1 && lane < kResW)
      __hip_atomic_store(reinterpret_cast<uint32_t*>(Rr) + lane, pub_img[32 + lane], __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (kStamp && tid == 0) e6 = __builtin_amdgcn_s_memtime();
  if (fstatus == kHandoff && !P.batch) {
    // Materialise the LDS visited sets as global bitmaps for the grid engine.
    if constexpr (kBm) {
      const uint32_t words = (P.n + 31) >> 5;  // <= kHashSize / 2 per side
      for (uint32_t i = tid; i < 2 * words; i += kLdsThreads) {
        const int q = i >= words;
        const uint32_t wi = q ? i - words : i;
        const unsigned long long w = W(q)[wi];
        (q ? P.b.vis[1] : P.b.vis[0])[wi] = (uint32_t)w | (uint32_t)(w >> 32);
      }
    } else {
      // The raw hash tables, coalesced; the whole grid scatters them into the
      // bitmaps (k_handoff_scatter).  Scattering them here -- ~10^4 atomics on
      // distinct lines from ONE CU at ~1 line per cycle -- cost ~7 us of a 10M
      // hand-off.
      const uint4* h4 = reinterpret_cast<const uint4*>(Hflat);
      uint4* d4 = reinterpret_cast<uint4*>(P.b.hdump);
      for (uint32_t i = tid; i < 2 * kHashSize / 4; i += kLdsThreads) d4[i] = h4[i];
    }
  }
  if (kStamp && tid == 0) e7 = __builtin_amdgcn_s_memtime();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // every wave's path / state / bitmap stores drained before publishing
  if (kStamp && tid == 0) e8 = __builtin_amdgcn_s_memtime();
  if (tid == 0) {
    // Device-memory results (hand-off state and bitmaps, an over-long path)
    // are read next by kernels / copies that may run on other XCDs: write
    // this XCD's L2 back first.  The host-visible fields went write-through.
    // (an unstaged path written with plain stores to host memory also needs the
    // system-scope release)
    if (status == kFound && md0 + md1 + 1 > sizeof(R) / sizeof(uint32_t)) __threadfence_system();
    else if (fstatus == kHandoff) __threadfence();
    if (kStamp && P.b.trace_cap > 2) {  // phase split: election / init / (loop) / walk / publish
      LevelTraceDev& t = P.b.trace[P.b.trace_cap - 2];
      t.side = (uint32_t)(e1 - e0);  // entry -> election resolved (init overlapped)
      t.depth = (uint32_t)(clk0 - e1);
      t.frontier = (uint32_t)(e4 - e3);
      t.mode = (uint32_t)(__builtin_amdgcn_s_memtime() - e4);
      if (P.b.trace_cap > 3) {  // publish split: state / result puts / bitmaps issued / drained / fence
        LevelTraceDev& u = P.b.trace[P.b.trace_cap - 3];
        u.side = (uint32_t)(e5 - e4);
        u.depth = (uint32_t)(e6 - e5);
        u.frontier = (uint32_t)(e7 - e6);
        u.mode = (uint32_t)(e8 - e7);
        u.edges = __builtin_amdgcn_s_memtime() - e8;
      }
    }
    __hip_atomic_store(&Rr->seq, P.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (!P.batch) {
      // the gate of an auto level enqueued behind this search (grid_auto):
      // {handed off, seq}, behind the hand-off state's release above
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(reinterpret_cast<unsigned long long*>(P.b.aux),
                         ((unsigned long long)P.seq << 32) | (fstatus == kHandoff ? 1ull : 0ull), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (kLq && kBm) {
    if (P.resident) {
      // after the publish: leave the bitmaps clean for the next search.  Every
      // set bit belongs to a vertex of a side's LDS queue (a losing claim only
      // re-marks a vertex that side already holds), so zeroing those words
      // clears everything; otherwise the next search clears it all.
      if (lq_done) {
        for (uint32_t i = tid; i < s0.qend + s1.qend; i += kLdsThreads) {
          const int q = i >= s0.qend;
          const uint32_t j = q ? i - s0.qend : i;
          W(q)[LQ[q][j] >> 5] = 0ull;
        }
      }
      if (tid == 0) bm_dirty = lq_done ? 0u : 1u;  // read after the server loop's barriers
    }
  }
}

template <typename OffT, bool kStamp, bool kBm>
__global__ __launch_bounds__(kLdsThreads, 1) void k_lds_bibfs(LdsParams<OffT> P) {
  lds_search_body<OffT, kStamp, kBm>(P, false);
}

// ---- batched search: block b answers query b with its own parent/queue slot,
// result slot and pinned path slot (throughput serving: one CU per query,
// 256 queries in flight on a full MI355X).
struct BatchArgs {
  uint32_t* src;             // K (pinned host)
  uint32_t* dst;             // K (pinned host)
  uint32_t* slots;           // per slot: parent[2] + queue[2], n words each
  HostResult* res;           // K pinned results
  uint32_t* path;            // K pinned path slots of path_cap words
  uint32_t path_cap;
  uint32_t seq;
};

template <typename OffT, bool kBm>
__global__ __launch_bounds__(kLdsThreads, 1) void k_lds_batch(LdsParams<OffT> P, BatchArgs A) {
  const uint32_t b = blockIdx.x;
  LdsParams<OffT> Q = P;
  // src/dst come straight from the pinned host array (no staging copy)
  Q.src = min(__hip_atomic_load(&A.src[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), P.n - 1);
  Q.dst = min(__hip_atomic_load(&A.dst[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), P.n - 1);
  Q.seq = A.seq;
  uint32_t* base = A.slots + (size_t)b * 4 * P.n;
  Q.b.parent[0] = base;
  Q.b.parent[1] = base + P.n;
  Q.b.queue[0] = base + 2 * (size_t)P.n;
  Q.b.queue[1] = base + 3 * (size_t)P.n;
  Q.h.res = A.res + b;
  Q.h.path = A.path + (size_t)b * A.path_cap;
  Q.h.path_cap = A.path_cap;
  Q.batch = 1;
  Q.trace = 0;
  lds_search_body<OffT, false, kBm>(Q, true);
}

// ---- resident query server -------------------------------------------------
// One elected workgroup stays on the GPU and serves queries posted by the
// host in a pinned mailbox: no kernel launch per query (~5 us saved of a
// ~30 us query).  Thread 0 polls the mailbox over PCIe with system-scope
// loads; the search itself is the same body as the one-shot kernel, and the
// result is published through the same pinned HostResult.  Exit: the host's
// stop word, or `idle_ticks` of s_memrealtime (100 MHz) without a request --
// every wave reaches the exit through the same barrier, so the grid drains
// even if the host process is gone.
template <typename OffT, bool kBm, bool kStamp = false>
__global__ __launch_bounds__(kLdsThreads, 1) void k_lds_server(LdsParams<OffT> P, ServerBox* box,
                                                              uint32_t last_seq, unsigned long long idle_ticks) {
  // Every branch that encloses a barrier is made provably wave-uniform
  // (readfirstlane): with a lane-divergent-looking loop exit the structurizer
  // may keep lanes 1..63 of wave 0 looping over the barriers while lane 0
  // waits to poll -- a deadlock.  So the whole of wave 0 polls, uniformly.
  __shared__ uint32_t cmd[7];  // stop, seq, src, dst, side_policy, lockstep, state set
  __shared__ uint32_t srv_won;
  const int tid = threadIdx.x;
  const uint32_t wid = __builtin_amdgcn_readfirstlane((uint32_t)tid >> 6);
  const bool cand = P.pin_xcc < 0 ? blockIdx.x == 0 : xcc_id() == (uint32_t)P.pin_xcc;
  if (!cand) return;
  if (tid == 0) srv_won = atomicMax(P.ticket, P.seq) < P.seq;
  __syncthreads();
  if (!uni(srv_won)) return;
  if (tid == 0) __hip_atomic_store(&box->alive, P.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __shared__ uint32_t diag[3];  // seen, poll latency, polls
  bool first = true;           // the first search of this launch: LDS holds nothing of ours
  __shared__ unsigned long long diag_t;
  constexpr int kDiagTid = kDiagOffWave0 ? kLdsThreads - kWave : 0;  // lane 0 of the last wave
  for (;;) {
    if (tid == kDiagTid) __hip_atomic_store(&box->stage, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (wid == 0) {
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t stop = 0, polls = 0;
      uint4 rq;
      unsigned long long tl = t0, lat = 0;
      for (;;) {
        ++polls;
        // One 16-byte system-scope load (bypasses the caches; relaxed: an
        // acquire would invalidate this XCD's L2 -- the hot graph -- per poll).
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 r4;
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)"
                     : "=v"(r4)
                     : "v"(box)
                     : "memory");
        rq.x = uni(r4.x), rq.y = uni(r4.y), rq.z = uni(r4.z), rq.w = uni(r4.w);
        const unsigned long long tn = __builtin_amdgcn_s_memrealtime();
        lat = tn - tl;  // one poll round trip (100 MHz ticks)
        tl = tn;
        const bool whole = (rq.w >> 8) == (rq.x & 0xffffffu);  // not torn
        if (whole && rq.x != last_seq) {
          stop = rq.w & kReqStop;
          break;
        }
        if (tn - t0 > idle_ticks) {
          stop = 1;
          break;
        }
      }
      if (tid == 0) {
        diag[0] = rq.x;
        diag[1] = (uint32_t)lat;
        diag[2] = polls;
        diag_t = tl;
        cmd[0] = stop;
        cmd[1] = rq.x;
        cmd[2] = rq.y;
        cmd[3] = rq.z;
        cmd[4] = (rq.w >> 2) & 3u;
        cmd[5] = (rq.w & kReqLockstep) ? 1u : 0u;
        cmd[6] = (rq.w & kReqAltBuf) ? 1u : 0u;
      }
    }
    // LDS-only barriers around the request: the diagnostic stores to host
    // memory (last wave) drain during the search instead of holding it
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (tid == kDiagTid) {
      __hip_atomic_store(&box->stage, 2u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&box->seen, diag[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&box->pad[0], diag[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&box->pad[1], diag[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&P.h.res->rt_pickup, diag_t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (uni(cmd[0])) break;
    LdsParams<OffT> Q = P;
    Q.seq = uni(cmd[1]);
    // the host validated src/dst against n; clamp anyway so a torn mailbox can never fault
    Q.src = min(uni(cmd[2]), P.n - 1);
    Q.dst = min(uni(cmd[3]), P.n - 1);
    Q.side_policy = (int)uni(cmd[4]);
    Q.lockstep = (int)uni(cmd[5]);
    Q.trace = kStamp ? 2 : 0;  // kStamp: BIBFS_STAMP_SERVER profiling build of the server
    if (uni(cmd[6])) Q.b = P.b_alt;
    Q.resident = first ? 1 : 2;
    first = false;
    last_seq = Q.seq;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");  // every wave has read cmd
    lds_search_body<OffT, kStamp, kBm>(Q, true);
    if (tid == kDiagTid) __hip_atomic_store(&box->stage, 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid == 0) {
    __threadfence_system();
    __hip_atomic_store(&box->alive, ~P.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // exited
  }
}

// ============================================================================
// Grid engine
// ============================================================================
constexpr int kGridThreads = 256;
constexpr uint32_t kHubDegree = 4096;  // deferred to k_grid_hubs
constexpr uint64_t kGridChunkMin = 32;  // smallest chunk (vertices) of k_grid_topdown
// A chunk holds this percentage of one 256-edge batch at the frontier's mean
// degree.  At 100 about half the chunks of a G(n, p) level went just past
// 256 edges and walked a second serial batch, and the level waits for its
// slowest block (stamped 10M levels: block claims at ~4.5 or ~9 us,
// profiles/r5_grid_stamps_10m.txt).
constexpr uint64_t kGridChunkFill = 75;
constexpr int kHubTile = 1024;  // k_grid_hubs: hubs staged in LDS per pass
// a hub-free level of at most one hub tile runs as one edge-parallel pass when
// its top-down pass would walk more than this many 256-edge batches per block
// (1 vs 2: Kronecker 25 44.1-45.1 -> 43.4-43.8 us, Kronecker 22 37.5-37.9 ->
// 36.9-37.3 us mean search, 10M unchanged; profiles/r4_grid_direct_batches_ab.jsonl)
constexpr uint64_t kGridDirectBatches = 1;
// Single-side grid levels stop at their first meet (every meet of such a level
// has the same length).  The edge loops of k_grid_topdown / k_grid_hubs read
// the meet word every (mask + 1) batches of 256 edges per workgroup: a
// Kronecker hub level spans only a few grid-stride iterations, so a sparse
// check never fires before the level has walked every hub edge.
constexpr uint32_t kMeetCheckMask = 0;
// 1 = k_grid_topdown's dependent round trips trimmed: each workgroup's first
// chunk is its block index (no ticket), the ticket and the meet word are read
// side by side, and a claim reads its visited word before the atomicOr only
// on levels of more than kGridPrecheckEdges frontier edges (small levels
// claim mostly unvisited vertices: the read only adds a round trip).
constexpr bool kGridFast = true;
constexpr uint64_t kGridPrecheckEdges = 1ull << 16;
// 1 = small top-down levels read the packed adjacency (GridParams::padj):
// 10M 61.9-62.2 -> 61.3-61.6 us, Kronecker 22 37.5-38.2 -> 36.5-37.8 us mean
// search (profiles/r4_grid_padj_ab.jsonl)
constexpr bool kGridPadj = true;

template <typename OffT>
struct GridParams {
  const OffT* row_off;
  const uint32_t* col;
  uint32_t n;
  int side;
  launch::SearchBuffers b;
  DevState* mirror;  // fused level end: pinned state mirror (nullptr = separate finish kernel)
  uint32_t seq;
  int trace;
  launch::HostSide h;  // fused publish of a finished search (path + result)
  uint32_t res_seq;
  uint32_t hub_deg;    // frontier vertices above this degree go to k_grid_hubs (~0u: never)
  uint32_t chunk_v;    // k_grid_topdown: frontier vertices per chunk ticket (<= kGridThreads)
  // auto level (grid_auto): the gate's search seq, the CU count and the graph
  // facts the device-side plan needs
  uint32_t gate_seq;
  unsigned long long gate_ticks;  // k_handoff gives up on the gate after this many s_memrealtime ticks
  uint32_t cus;
  unsigned long long max_deg;
  unsigned long long nnz;
  float alpha;
  uint32_t nparts;     // workgroups taking part in the level (0 = gridDim.x); the rest exit at once
  uint32_t fbase, fcount;  // auto level: the frontier, from the plan (0/0 = read DevState)
  int chain;           // auto level with another auto level enqueued behind it: its finisher plans that one
  int hub_direct;      // k_grid_hubs: the whole frontier is the hub list (no top-down pass before it)
  int precheck;        // claims read the visited word before the atomicOr (big levels)
  // packed adjacency {v, deg, base}: on small levels (!precheck) an edge's one
  // 16-byte load brings the neighbour's degree with its id (no row-offset
  // round trip after the claim); nullptr = col + row_off
  const uint4* padj;
  const unsigned long long* padj8;  // its 8-byte form (preferred when set)
};

// aux[2], the auto chain's word: bit 0 = the chain took the hand-off (its
// levels dirtied the global state: the predicated cleanup runs), bit 1 = the
// side of the planned level, bit 2 = it runs as one edge-parallel hub pass
// over the whole frontier (hub_direct), bit 3 = a planned level is to run.
constexpr uint32_t kAuxTook = 1u, kAuxDirect = 4u, kAuxActive = 8u, kAuxPrecheck = 16u;

// The auto level's plan from the frontier facts, with the host's rules
// (grid_level / choose_side / choose_mode): the side with fewer frontier
// edges; declined when the Beamer rule wants bottom-up; hub degree; chunk size.
struct AutoPlan {
  uint32_t active, side, F, hub, cv, fb;
  bool declined, direct, precheck;
};
template <typename OffT>
__device__ __forceinline__ AutoPlan plan_auto_level(const GridParams<OffT>& P, unsigned long long fe0,
                                                    unsigned long long fe1, unsigned long long ve0,
                                                    unsigned long long ve1, uint32_t fb0, uint32_t fb1, uint32_t fd0,
                                                    uint32_t fd1) {
  AutoPlan a{1u, 0u, 0u, ~0u, (uint32_t)kGridThreads, 0u, false, false, true};
  a.side = fe0 <= fe1 ? 0u : 1u;
  const unsigned long long fe = a.side ? fe1 : fe0;
  const double m_u = (double)P.nnz - (double)(a.side ? ve1 : ve0);
  a.fb = a.side ? fb1 : fb0;
  a.F = (a.side ? fd1 : fd0) - a.fb;
  if ((double)fe > m_u / (double)P.alpha) {
    a.active = 0;
    a.declined = true;
    return a;
  }
  if (P.max_deg > kHubDegree && fe > kHubDegree) a.hub = kHubDegree;
  if (a.F <= 4096 && fe > 16384 && P.max_deg > 64) a.hub = 64;
  if ((a.F + kGridThreads - 1) / kGridThreads < P.cus * 4u && fe > 0)
    a.cv = (uint32_t)min<uint64_t>(kGridThreads,
                                   max<uint64_t>(kGridChunkMin, kGridThreads * kGridChunkFill * (uint64_t)a.F / (100 * fe)));
  // grid_topdown's rule: a hub level of at most one hub tile is one
  // edge-parallel pass (P.hub_direct: allowed on this chain)
  {
    const uint64_t chunks = ((uint64_t)a.F + a.cv - 1) / a.cv;
    const uint64_t blocks = min<uint64_t>((uint64_t)P.cus * 4, max<uint64_t>(1, chunks));
    a.direct = P.hub_direct && a.F <= (uint32_t)kHubTile &&
               (a.hub != ~0u || fe > kGridDirectBatches * kGridThreads * blocks);
  }
  a.precheck = !kGridFast || fe > kGridPrecheckEdges;
  return a;
}

// The plan for the kernels behind: [2] the chain word; [3] frontier size;
// [4] hub degree; [5] chunk size; [6] frontier base
__device__ __forceinline__ void write_auto_plan(uint32_t* aux, const AutoPlan& a, bool took) {
  aux[2] = (took ? kAuxTook : 0u) |
           (a.active ? kAuxActive | a.side << 1 | (a.direct ? kAuxDirect : 0u) | (a.precheck ? kAuxPrecheck : 0u)
                     : 0u);
  aux[3] = a.F;
  aux[4] = a.hub;
  aux[5] = a.cv;
  aux[6] = a.fb;
}

// The per-level values a grid kernel reads: the host's (GridParams) for a
// host-planned level, the plan in aux for an auto level.  Kept apart from
// GridParams so that no kernel writes its kernel-argument struct: the auto
// kernels did, which put a copy of it in scratch (320 B per thread), and every
// pointer read through the copy became a scratch load plus a flat access
// (flat operations also count in lgkmcnt, so each LDS wait waited for them).
struct GridLv {
  int side, precheck, hub_direct;
  uint32_t hub_deg, chunk_v, fbase, fcount, nparts;
  bool packed;  // the level may read the packed adjacency (an auto big level: 4-byte column loads)
};
template <typename OffT>
__device__ __forceinline__ GridLv grid_lv(const GridParams<OffT>& P) {
  return GridLv{P.side, P.precheck, P.hub_direct, P.hub_deg, P.chunk_v, P.fbase, P.fcount, P.nparts, true};
}

template <typename OffT>
__device__ void fused_finish(const GridParams<OffT>& P, const GridLv& L, int mode, bool hub_pass);

// Claim v for side s from parent u; wave-uniform call (every lane calls it,
// `valid` masks lanes with no edge).  Appends claimed vertices to the queue
// with one atomic per wave and checks the other side's bitmap (fused meet).
template <typename OffT>
__device__ __forceinline__ void grid_claim(const GridParams<OffT>& P, const GridLv& L, bool valid, uint32_t u,
                                           uint32_t v, uint32_t vdeg = ~0u) {
  const int s = L.side, o = s ^ 1;
  DevState* st = P.b.st;
  const uint32_t w = v >> 5, bit = 1u << (v & 31);
  bool mine = false;
  if (valid && (!L.precheck || !(P.b.vis[s][w] & bit))) mine = !(atomicOr(&P.b.vis[s][w], bit) & bit);
  const unsigned long long mask = __ballot(mine);
  if (!mask) return;
  const int lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t deg = 0;
  if (mine) {
    // write-through (sc1): the level's last workgroup may walk this parent
    // chain in the same kernel, from another XCD, with sc1 loads
    __hip_atomic_store(&P.b.parent[s][v], u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    deg = vdeg != ~0u ? vdeg : (uint32_t)(P.row_off[v + 1] - P.row_off[v]);
    if (P.b.vis[o][w] & bit) {
      if (atomicCAS(&st->meet, kEmpty, v) == kEmpty) st->meet_side = (uint32_t)s;
    }
  }
  uint32_t pos = 0;
  if (lane == leader) pos = atomicAdd(&st->qtail[s], (uint32_t)__popcll(mask));
  pos = __shfl(pos, leader);
  if (mine) P.b.queue[s][pos + mbcnt64(mask)] = v;
  const unsigned long long dsum = wave_sum((unsigned long long)deg);
  if (lane == leader) atomicAdd(&st->nedges, dsum);
}

// Hand-off kernel: the first kernel behind an LDS search that left LDS.
//  * gated (grid_auto: enqueued before the search started): wave 0 of every
//    workgroup waits for the gate -- search `gate_seq` has left LDS -- with
//    relaxed agent-scope polls and s_sleep, then one agent acquire (the
//    hand-off state was released by the LDS engine before the gate); block 0
//    plans the auto level from DevState with the host's rules (grid_level /
//    choose_side / choose_mode: the side with fewer frontier edges, declined
//    when the Beamer rule wants bottom-up, hub degree, chunk size) into aux
//    for the kernels behind it; a declined level publishes the host mirror
//    unchanged, so the host loop takes it over.
//  * hash-set searches (n > kBmMaxN): the LDS engine dumped its raw hash
//    tables (coalesced); every thread scatters one slot into the global
//    visited bitmaps (a single CU issuing them cost ~7 us on 10M G(n, p)).
// A gate already holding a later search's seq ends the wait at once (that
// search ran after ours: ours stayed in LDS; a chain delayed behind earlier
// launches on the stream used to wait out the whole timeout there).
// The gate wait gives up after GridParams::gate_ticks (default 6 s of
// s_memrealtime, 100 MHz -- longer than the host's 5 s server wait).  A wait
// that gives up runs no level and publishes nothing (aux[2] = 0); the host
// sees the auto chain drain unpublished and continues the search itself from
// the hand-off mirror (HipBiBfs::Impl::wait_auto, fallback path).
constexpr int kHandoffBlocks = 64;  // x kGridThreads = 2 * kHashSize: one slot per thread
static_assert(kHandoffBlocks * kGridThreads == 2 * kHashSize, "one hash slot per thread");
template <typename OffT>
__global__ __launch_bounds__(kGridThreads) void k_handoff(GridParams<OffT> P, int gated, int scatter) {
  __shared__ uint32_t shand;
  DevState* st = P.b.st;
  if (gated) {
    if (threadIdx.x < kWave) {  // wave 0, uniformly
      const uint32_t lane = threadIdx.x;
      const unsigned long long* gate = reinterpret_cast<const unsigned long long*>(P.b.aux);
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      unsigned long long g = 0;
      bool seen = false;
      for (;;) {
        g = __hip_atomic_load(gate, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        g = ((unsigned long long)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(g >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)g);
        const uint32_t gs = (uint32_t)(g >> 32);
        if (gs == P.gate_seq) {
          seen = true;
          break;
        }
        // A LATER search already answered on this state set (the gate word is
        // per set; sets alternate): ours ended in LDS -- a search that hands
        // off holds the host in wait_auto until this chain publishes, so no
        // later search can start -- and this chain was only late behind the
        // stream's earlier launches.  Nothing to run.
        if ((int32_t)(gs - P.gate_seq) > 0) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > P.gate_ticks) break;
        __builtin_amdgcn_s_sleep(8);  // ~0.2 us: the pollers must not crowd the LDS search's memory
      }
      const bool hand = seen && (uint32_t)g == 1u;
      if (hand) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      if (blockIdx.x == 0) {
        AutoPlan ap{0u, 0u, 0u, ~0u, (uint32_t)kGridThreads, 0u, false, false, true};
        if (hand) {
          // the whole DevState in one round trip: lane i loads word i
          constexpr uint32_t kW = (uint32_t)(sizeof(DevState) / sizeof(uint32_t));
          const uint32_t w = lane < kW ? load_agent(reinterpret_cast<const uint32_t*>(st) + lane) : 0u;
          auto word = [&](const void* field) {
            return (uint32_t)__builtin_amdgcn_readlane(
                (int)w, (int)((reinterpret_cast<const char*>(field) - reinterpret_cast<const char*>(st)) / 4));
          };
          auto dword = [&](const unsigned long long* field) {
            return (unsigned long long)word(field) |
                   (unsigned long long)word(reinterpret_cast<const uint32_t*>(field) + 1) << 32;
          };
          ap = plan_auto_level(P, dword(&st->fedges[0]), dword(&st->fedges[1]), dword(&st->vedges[0]),
                               dword(&st->vedges[1]), word(&st->fbeg[0]), word(&st->fbeg[1]), word(&st->fend[0]),
                               word(&st->fend[1]));
        }
        if (lane == 0) {
          write_auto_plan(P.b.aux, ap, ap.active != 0);  // a declined level: the chain takes nothing
          if (ap.declined && P.mirror)
            __hip_atomic_store(&P.mirror->pad[0], P.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
      if (lane == 0) shand = hand;
    }
    __syncthreads();
    if (!__builtin_amdgcn_readfirstlane(shand)) return;
  }
  if (scatter) {
    const uint32_t i = blockIdx.x * kGridThreads + threadIdx.x;
    const uint32_t k = P.b.hdump[i];
    if (k != kEmpty) {
      const uint32_t v = k & kIdMask;
      atomicOr(&(i >= kHashSize ? P.b.vis[1] : P.b.vis[0])[v >> 5], 1u << (v & 31));
    }
  }
}

// Auto level (grid_auto): the plan k_handoff left in aux (written by the
// kernel before: plain loads).  false = no level to run, or this workgroup is
// beyond the level's chunk count (the host's launch size) -- it leaves before
// any ticket or done-counter atomic.
template <typename OffT>
__device__ bool auto_plan(const GridParams<OffT>& P, GridLv& L) {
  const uint32_t xp = __builtin_amdgcn_readfirstlane(P.b.aux[2]);
  if (!(xp & kAuxActive) || (xp & kAuxDirect)) return false;  // direct: the hub pass runs the level
  L.side = (int)((xp >> 1) & 1u);
  L.precheck = (xp & kAuxPrecheck) ? 1 : 0;
  L.packed = !L.precheck;  // big level: 4-byte column loads
  L.fcount = __builtin_amdgcn_readfirstlane(P.b.aux[3]);
  L.hub_deg = __builtin_amdgcn_readfirstlane(P.b.aux[4]);
  L.chunk_v = __builtin_amdgcn_readfirstlane(P.b.aux[5]);
  L.fbase = __builtin_amdgcn_readfirstlane(P.b.aux[6]);
  const uint32_t chunks = (L.fcount + L.chunk_v - 1) / L.chunk_v;
  L.nparts = max(1u, min(gridDim.x, chunks));
  return blockIdx.x < L.nparts;
}

template <typename OffT, bool kAuto = false>
__global__ __launch_bounds__(kGridThreads) void k_grid_topdown(GridParams<OffT> P) {
  GridLv L = grid_lv(P);
  if constexpr (kAuto) {
    if (!auto_plan(P, L)) return;
  }
  __shared__ uint32_t sv[kGridThreads];
  __shared__ OffT sb[kGridThreads];
  __shared__ uint32_t sEb[kGridThreads];
  __shared__ uint32_t wsum[kGridThreads / kWave];
  __shared__ uint32_t schunk, stotal;
  const int s = L.side;
  DevState* st = P.b.st;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  // stamped trace (BIBFS_STAMP): block 0's phases, kGridStampWords per level
  unsigned long long* gst = nullptr;
  if (!kAuto && P.trace == 2 && blockIdx.x == 0 && tid == 0 && P.b.gstamp) {
    gst = P.b.gstamp + (size_t)(st->levels % launch::kGridStampLevels) * launch::kGridStampWords;
    gst[0] = __builtin_amdgcn_s_memrealtime();
  }
  const uint32_t fbase = kAuto ? L.fbase : st->fbeg[s];
  const uint32_t F = kAuto ? L.fcount : st->fend[s] - fbase;
  const uint32_t parts = L.nparts ? L.nparts : gridDim.x;
  const unsigned long long* const padj8 = L.packed ? P.padj8 : nullptr;
  const uint4* const padj = L.packed ? P.padj : nullptr;
  for (uint32_t round = 0;; ++round) {
    if (kGridFast) {
      // chunk b first (no ticket); then tickets, numbered after the blocks'
      // own chunks, with the meet word read beside the ticket
      if (tid == 0) {
        if (round == 0) {
          schunk = blockIdx.x;
        } else if ((uint64_t)parts * L.chunk_v >= F) {
          schunk = kEmpty;  // every chunk went to a block of its own: no ticket to take
        } else {
          const uint32_t t = atomicAdd(&st->chunk, 1u);
          schunk = load_agent(&st->meet) != kEmpty ? kEmpty : parts + t;
        }
      }
    } else if (tid == 0) {
      schunk = (load_agent(&st->meet) != kEmpty) ? kEmpty : atomicAdd(&st->chunk, 1u);
    }
    __syncthreads();
    const uint32_t c = schunk;
    const uint32_t cv = L.chunk_v;
    if (c == kEmpty || (uint64_t)c * cv >= F) break;
    const uint32_t i = c * cv + tid;
    uint32_t deg = 0, u = 0;
    OffT b = 0;
    if ((uint32_t)tid < cv && i < F) {
      u = P.b.queue[s][fbase + i];
      b = P.row_off[u];
      deg = (uint32_t)(P.row_off[u + 1] - b);
      if (deg > L.hub_deg) {
        P.b.hub_list[atomicAdd(&st->hub_count, 1u)] = u;
        deg = 0;
      }
    }
    sv[tid] = u;
    sb[tid] = b;
    uint32_t x = deg;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const uint32_t y = __shfl_up(x, off);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wid] = x;
    __syncthreads();
    if (tid == 0) {
      uint32_t a = 0;
      for (int k = 0; k < kGridThreads / kWave; ++k) {
        const uint32_t t = wsum[k];
        wsum[k] = a;
        a += t;
      }
      stotal = a;
    }
    __syncthreads();
    sEb[tid] = x - deg + wsum[wid];
    __syncthreads();
    if (gst && round == 0) gst[1] = __builtin_amdgcn_s_memrealtime();  // first chunk staged
    const uint32_t Ec = stotal;
    for (uint32_t base = 0, it = 0; base < Ec; base += kGridThreads, ++it) {
      // a meet ends the level (single-side level: every meet has the same
      // length): check it every 16 batches, wave-uniformly
      if (it > 0 && (it & kMeetCheckMask) == kMeetCheckMask &&
          __builtin_amdgcn_readfirstlane(load_agent(&st->meet)) != kEmpty)
        break;
      const uint32_t e = base + tid;
      const bool valid = e < Ec;
      uint32_t uu = 0, v = 0, vdeg = ~0u;
      if (valid) {
        const uint32_t lo = lift_search(sEb, kGridThreads, e, kGridThreads / 2);
        uu = sv[lo];
        const OffT k = sb[lo] + (OffT)(e - sEb[lo]);
        if (padj8) {  // small level: the neighbour's degree with its id
          const unsigned long long w = padj8[k];
          v = launch::pack8_v(w);
          vdeg = launch::pack8_deg(w);
        } else if (padj) {
          const uint4 q = padj[k];
          v = q.x;
          vdeg = q.y;
        } else {
          v = P.col[k];
        }
      }
      grid_claim(P, L, valid, uu, v, vdeg);
    }
    if (gst && round == 0) {  // first chunk's claims and appends issued ...
      gst[2] = __builtin_amdgcn_s_memrealtime();
    }
    __syncthreads();
  }
  if (gst) gst[3] = __builtin_amdgcn_s_memrealtime();  // block 0 leaves its chunks
  if (P.mirror) fused_finish(P, L, 1, false);
}

// Hub vertices (degree > hub_deg) deferred by k_grid_topdown, expanded
// edge-parallel: every workgroup stages a tile of up to 1024 hubs with the
// exclusive prefix of their degrees in LDS and walks the tile's flattened edge
// range with a grid stride (binary search for the hub of an edge), so each
// hub's edges spread over every CU (the previous kernel walked the hub list
// in order in every workgroup).  Enqueued right behind the top-down kernel;
// a no-op when that level deferred nothing (its finisher reset hub_count),
// otherwise its last workgroup finishes the level.
template <typename OffT, bool kAuto = false>
__global__ __launch_bounds__(kGridThreads) void k_grid_hubs(GridParams<OffT> P) {
  __shared__ uint32_t hu[kHubTile];
  __shared__ OffT hb[kHubTile];
  __shared__ unsigned long long hp[kHubTile + 1];
  __shared__ unsigned long long wsum[kGridThreads / kWave];
  DevState* st = P.b.st;
  GridLv L = grid_lv(P);
  if constexpr (kAuto) {  // behind an auto level: its plan (written by the kernel before)
    const uint32_t xp = __builtin_amdgcn_readfirstlane(P.b.aux[2]);
    if (!(xp & kAuxActive)) return;
    L.side = (int)((xp >> 1) & 1u);
    L.hub_direct = (xp & kAuxDirect) ? 1 : 0;
    L.precheck = (xp & kAuxPrecheck) ? 1 : 0;
    L.hub_deg = __builtin_amdgcn_readfirstlane(P.b.aux[4]);
    // the host's hub launch size: 4 workgroups per frontier vertex
    L.nparts = max(1u, min(gridDim.x, 4u * __builtin_amdgcn_readfirstlane(P.b.aux[3])));
    if (blockIdx.x >= L.nparts) return;
  }
  // the hub list: the vertices k_grid_topdown deferred, or (hub_direct) the
  // whole frontier -- a small frontier of heavy vertices skips the top-down
  // pass, which ran it on a handful of workgroups
  const uint32_t* const hl = L.hub_direct ? P.b.queue[L.side] + st->fbeg[L.side] : P.b.hub_list;
  const uint32_t H = L.hub_direct ? st->fend[L.side] - st->fbeg[L.side] : st->hub_count;
  if (H == 0) return;  // grid-uniform: the top-down finisher completed the level
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (uint32_t t0 = 0; t0 < H; t0 += kHubTile) {
    const uint32_t nt = min((uint32_t)kHubTile, H - t0);
    constexpr int kPer = kHubTile / kGridThreads;
    unsigned long long d[kPer], run = 0;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t j = tid * kPer + k;
      d[k] = 0;
      if (j < nt) {
        const uint32_t u = hl[t0 + j];
        const OffT b = P.row_off[u];
        d[k] = (unsigned long long)(P.row_off[u + 1] - b);
        hu[j] = u;
        hb[j] = b;
      }
      run += d[k];
    }
    unsigned long long x = run;  // inclusive wave scan of per-thread sums
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
      const unsigned long long y = __shfl_up(x, o);
      if (lane >= o) x += y;
    }
    if (lane == kWave - 1) wsum[wid] = x;
    __syncthreads();
    unsigned long long pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < kGridThreads / kWave; ++k) {
      pre += k < wid ? wsum[k] : 0ull;
      tot += wsum[k];
    }
    unsigned long long e0 = pre + x - run;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      hp[tid * kPer + k] = e0;
      e0 += d[k];
    }
    __syncthreads();
    uint32_t it = 0;
    for (unsigned long long base = (unsigned long long)blockIdx.x * kGridThreads; base < tot;
         base += (unsigned long long)(L.nparts ? L.nparts : gridDim.x) * kGridThreads, ++it) {
      if (it > 0 && (it & kMeetCheckMask) == kMeetCheckMask &&
          __builtin_amdgcn_readfirstlane(load_agent(&st->meet)) != kEmpty)
        break;
      const unsigned long long e = base + tid;
      const bool valid = e < tot;
      uint32_t uu = 0, v = 0;
      if (valid) {
        const uint32_t a = lift_search(hp, nt, e, lift_top(nt));  // last hub whose edge range starts at or before e
        uu = hu[a];
        v = P.col[hb[a] + (OffT)(e - hp[a])];
      }
      grid_claim(P, L, valid, uu, v);
    }
    __syncthreads();
  }
  fused_finish(P, L, 1, true);
}

// Bottom-up level for side s: every unvisited vertex looks for a parent in the
// frontier bitmap, stopping at the first hit.  One wave owns 64 consecutive
// vertices = two whole bitmap words, so visited / next-frontier words are
// written with plain stores built from one ballot (no atomics).
template <typename OffT>
__global__ __launch_bounds__(kGridThreads) void k_grid_bottomup(GridParams<OffT> P) {
  const int s = P.side, o = s ^ 1;
  DevState* st = P.b.st;
  const uint32_t* __restrict__ fb = P.b.fbits[s];
  uint32_t* __restrict__ vis = P.b.vis[s];
  uint32_t* __restrict__ nb = P.b.nbits[s];
  const int lane = __lane_id();
  const uint64_t nw = ((uint64_t)P.n + 63) / 64;
  const uint64_t wave0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / 64;
  const uint64_t wstride = (uint64_t)gridDim.x * blockDim.x / 64;
  unsigned long long insp_acc = 0;
  for (uint64_t gw = wave0; gw < nw; gw += wstride) {
    const uint32_t mt = __shfl(load_agent(&st->meet), 0);  // wave-uniform early exit
    if (mt != kEmpty) break;
    const uint64_t v64 = gw * 64 + lane;
    const uint32_t v = (uint32_t)v64;
    const bool inr = v64 < P.n;
    const uint32_t word = vis[gw * 2 + (lane >> 5)];
    const uint32_t bit = 1u << (lane & 31);
    bool found = false;
    uint32_t pu = 0;
    OffT rb = 0, re = 0;
    if (inr && !(word & bit)) {
      rb = P.row_off[v];
      re = P.row_off[v + 1];
      OffT k = rb;
      for (; k + 4 <= re && !found; k += 4) {
        uint32_t c0 = P.col[k], c1 = P.col[k + 1], c2 = P.col[k + 2], c3 = P.col[k + 3];
        const bool h0 = fb[c0 >> 5] & (1u << (c0 & 31));
        const bool h1 = fb[c1 >> 5] & (1u << (c1 & 31));
        const bool h2 = fb[c2 >> 5] & (1u << (c2 & 31));
        const bool h3 = fb[c3 >> 5] & (1u << (c3 & 31));
        if (h0 | h1 | h2 | h3) {
          found = true;
          pu = h0 ? c0 : (h1 ? c1 : (h2 ? c2 : c3));
          insp_acc += (unsigned long long)(h0 ? 1 : (h1 ? 2 : (h2 ? 3 : 4)));
        } else {
          insp_acc += 4;
        }
      }
      for (; k < re && !found; ++k) {
        const uint32_t c0 = P.col[k];
        ++insp_acc;
        if (fb[c0 >> 5] & (1u << (c0 & 31))) {
          found = true;
          pu = c0;
        }
      }
    }
    const unsigned long long mask = __ballot(found);
    if (lane == 0) nb[gw * 2] = (uint32_t)mask;
    if (lane == 32) nb[gw * 2 + 1] = (uint32_t)(mask >> 32);
    if (!mask) continue;
    if (lane == 0) vis[gw * 2] = word | (uint32_t)mask;
    if (lane == 32) vis[gw * 2 + 1] = word | (uint32_t)(mask >> 32);
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t deg = 0;
    if (found) {
      P.b.parent[s][v] = pu;
      deg = (uint32_t)(re - rb);
      if (P.b.vis[o][v >> 5] & bit) {
        if (atomicCAS(&st->meet, kEmpty, v) == kEmpty) st->meet_side = (uint32_t)s;
      }
    }
    uint32_t pos = 0;
    if (lane == leader) pos = atomicAdd(&st->qtail[s], (uint32_t)__popcll(mask));
    pos = __shfl(pos, leader);
    if (found) P.b.queue[s][pos + mbcnt64(mask)] = v;
    const unsigned long long dsum = wave_sum((unsigned long long)deg);
    if (lane == leader) atomicAdd(&st->nedges, dsum);
  }
  const unsigned long long isum = wave_sum(insp_acc);
  if (lane == 0 && isum) atomicAdd(&st->einsp, isum);
}

__global__ void k_frontier_bits(launch::SearchBuffers b, int s) {
  const DevState* st = b.st;
  const uint32_t fb0 = st->fbeg[s], fe = st->fend[s];
  for (uint64_t i = fb0 + blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < fe;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = b.queue[s][i];
    atomicOr(&b.fbits[s][v >> 5], 1u << (v & 31));
  }
}

// Single-thread level bookkeeping (avoids a host round trip for state updates).
__device__ void finish_state(DevState& st, const launch::SearchBuffers& b, int s, int mode, int trace);

// Copy a DevState into the pinned host mirror: one write-through store per
// lane (one wide PCIe write instead of ~30 serial ones), drained, then `seq`.
__device__ void publish_state(const DevState& v, DevState* mirror, uint32_t seq, uint32_t lane) {
  constexpr uint32_t kWords = (uint32_t)(offsetof(DevState, pad) / sizeof(uint32_t));
  static_assert(kWords <= 64, "one lane per word");
  if (lane < kWords)
    __hip_atomic_store(&reinterpret_cast<uint32_t*>(mirror)[lane], reinterpret_cast<const uint32_t*>(&v)[lane],
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) __hip_atomic_store(&mirror->pad[0], seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ void publish_result(const launch::SearchBuffers& b, const launch::HostSide& h, const DevState& sv,
                               uint32_t res_seq, uint32_t n);

__global__ void k_finish_level(launch::SearchBuffers b, int s, int mode, int trace, DevState* mirror,
                               uint32_t seq, launch::HostSide h, uint32_t res_seq, uint32_t n) {
  __shared__ DevState sv;
  if (blockIdx.x != 0) return;
  if (threadIdx.x == 0) {
    finish_state(*b.st, b, s, mode, trace);
    sv = *b.st;
  }
  __syncthreads();
  if (res_seq && sv.status != kRunning) publish_result(b, h, sv, res_seq, n);
  if (mirror && threadIdx.x < 64) publish_state(sv, mirror, seq, threadIdx.x);
}

// A finished search, published by the workgroup that finished its last level:
// two waves walk the two parent chains (sc1 loads) into pinned host memory,
// then one lane writes the result record, `seq` last (system-scope release).
// Needs >= 2 waves.
__device__ void publish_result(const launch::SearchBuffers& b, const launch::HostSide& h, const DevState& sv,
                               uint32_t res_seq, uint32_t n) {
  const int tid = threadIdx.x;
  const uint32_t status = sv.status == kFound ? kFound : kNoPath;
  const int d0 = sv.depth[0], d1 = sv.depth[1];
  const uint32_t hops = (uint32_t)(d0 + d1);
  uint32_t* out = (hops + 1 <= h.path_cap) ? h.path : b.dpath;
  const unsigned long long t_walk = __builtin_amdgcn_s_memrealtime();
  if (status == kFound && (tid == 0 || tid == kWave)) {
    walk_side(b.parent[tid ? 1 : 0], n, sv.meet, tid ? 1 : 0, d0, d1, out);
    __threadfence_system();
  }
  __syncthreads();
  if (tid == 0) {
    HostResult* Rr = h.res;
    Rr->rt_walk = t_walk;
    Rr->status = status;
    Rr->hops = status == kFound ? (int32_t)hops : -1;
    Rr->meet = sv.meet;
    Rr->levels = sv.levels;
    Rr->visited = sv.qtail[0] + sv.qtail[1];
    Rr->einsp = sv.einsp;
    Rr->depth[0] = d0;
    Rr->depth[1] = d1;
    Rr->path_len = status == kFound ? hops + 1 : 0u;
    Rr->path_on_device = (status == kFound && hops + 1 > h.path_cap) ? 1u : 0u;
    // end of a search that left LDS: rt_begin is the LDS kernel's stamp, so
    // rt_end - rt_begin is the device-side span of the whole search
    Rr->rt_end = __builtin_amdgcn_s_memrealtime();
    __threadfence_system();
    __hip_atomic_store(&Rr->seq, res_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// End-of-level bookkeeping of the grid engine on a DevState (device memory
// or a workgroup's LDS copy).
__device__ void finish_state(DevState& sref, const launch::SearchBuffers& b, int s, int mode, int trace) {
  DevState* st = &sref;
  const uint32_t ncnt = st->qtail[s] - st->fend[s];
  if (trace && st->levels < b.trace_cap) {
    LevelTraceDev& t = b.trace[st->levels];
    t.side = s;
    t.depth = st->depth[s];
    t.frontier = st->fend[s] - st->fbeg[s];
    t.mode = (uint32_t)mode + 3;  // 4 = grid top-down, 5 = grid bottom-up
    t.edges = mode == 1 ? st->fedges[s] : 0;
    t.discovered = ncnt;
  }
  if (mode == 1) st->einsp += st->fedges[s];
  st->levels++;
  st->depth[s]++;
  if (st->meet != kEmpty) {
    st->status = kFound;
  } else if (ncnt == 0) {
    st->status = kNoPath;
  } else {
    st->fbeg[s] = st->fend[s];
    st->fend[s] = st->qtail[s];
    st->fedges[s] = st->nedges;
    st->vedges[s] += st->nedges;
  }
  st->nedges = 0;
  st->chunk = 0;
  st->hub_count = 0;
  st->hub_edge_cursor = 0;
}

// Fused end of a grid level: the LAST workgroup of the level's kernel (told by
// a done counter) finishes the level itself -- no extra kernel launch.  Every
// DevState word is read with a device-scope atomic (the counters were updated
// by atomics from every XCD; a plain load could see a stale L2 line), the
// bookkeeping runs on an LDS copy, the words go back with plain stores (the
// next level is a new launch), and the pinned mirror is published; when the
// level ended the search, the same workgroup walks the path (the parents
// were stored write-through) and publishes the result.  A top-down level that
// deferred hubs leaves the finish to k_grid_hubs (hub_pass), which runs next.
template <typename OffT>
__device__ void fused_finish(const GridParams<OffT>& P, const GridLv& L, int mode, bool hub_pass) {
  __shared__ DevState sv;
  __shared__ uint32_t slast;
  constexpr uint32_t kWords = (uint32_t)(sizeof(DevState) / sizeof(uint32_t));
  static_assert(kWords <= 64, "one lane per word");
  const launch::SearchBuffers& b = P.b;
  const uint32_t tid = threadIdx.x;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this workgroup's atomics and sc1 stores have completed
  __syncthreads();
  const uint32_t parts = L.nparts ? L.nparts : gridDim.x;
  if (tid == 0) slast = atomicAdd(&b.st->pad[1], 1u) == parts - 1;
  __syncthreads();
  if (!__builtin_amdgcn_readfirstlane(slast)) return;
  uint32_t* w = reinterpret_cast<uint32_t*>(b.st);
  unsigned long long* gst = nullptr;  // stamped trace: the finisher's start / end
  if (P.trace == 2 && tid == 0 && b.gstamp) {
    gst = b.gstamp + (size_t)(b.st->levels % launch::kGridStampLevels) * launch::kGridStampWords;
    gst[4] = __builtin_amdgcn_s_memrealtime();
  }
  if (tid < kWords) reinterpret_cast<uint32_t*>(&sv)[tid] = atomicAdd(&w[tid], 0u);
  __syncthreads();
  const bool defer = !hub_pass && sv.hub_count != 0;  // the hub pass finishes this level
  if (tid == 0) {
    sv.pad[1] = 0;  // done counter, for the next kernel
    if (!defer) finish_state(sv, b, L.side, mode, P.trace);
  }
  __syncthreads();
  if (defer) {
    if (tid == 0) atomicExch(&b.st->pad[1], 0u);
    return;
  }
  if (tid < kWords) w[tid] = reinterpret_cast<const uint32_t*>(&sv)[tid];
  if (P.res_seq && sv.status != kRunning) publish_result(b, P.h, sv, P.res_seq, P.n);
  // an auto level with another one chained behind it plans that level (the
  // next launch reads aux); the host hears nothing until the chain ends
  bool next = false;
  if (P.chain) {
    __shared__ uint32_t snext;
    if (tid == 0) {
      AutoPlan ap{0u, 0u, 0u, ~0u, (uint32_t)kGridThreads, 0u, false, false, true};
      if (sv.status == kRunning)
        ap = plan_auto_level(P, sv.fedges[0], sv.fedges[1], sv.vedges[0], sv.vedges[1], sv.fbeg[0], sv.fbeg[1],
                             sv.fend[0], sv.fend[1]);
      write_auto_plan(b.aux, ap, true);
      snext = ap.active;
    }
    __syncthreads();
    next = snext != 0;
  }
  if (P.mirror && !next && tid < 64) publish_state(sv, P.mirror, P.seq, tid);
  if (gst) gst[5] = __builtin_amdgcn_s_memrealtime();
}

// Seed a search for the grid engine / step-wise API.
template <typename OffT>
__global__ void k_seed(const OffT* row_off, launch::SearchBuffers b, uint32_t src, uint32_t dst) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DevState* st = b.st;
  const uint32_t r[2] = {src, dst};
  for (int s = 0; s < 2; ++s) {
    const uint32_t v = r[s];
    b.queue[s][0] = v;
    b.parent[s][v] = kEmpty;
    atomicOr(&b.vis[s][v >> 5], 1u << (v & 31));
    st->depth[s] = 0;
    st->fbeg[s] = 0;
    st->fend[s] = 1;
    st->qtail[s] = 1;
    st->fedges[s] = row_off[v + 1] - row_off[v];
    st->vedges[s] = st->fedges[s];
  }
  st->status = kRunning;
  st->meet = (src == dst) ? src : kEmpty;
  st->meet_side = 0;
  st->levels = 0;
  st->hub_count = 0;
  st->chunk = 0;
  st->hub_edge_cursor = 0;
  st->nedges = 0;
  st->einsp = 0;
}

// Publish a finished grid search: walk both parent chains (two waves in
// parallel) into pinned host memory, then release the result record.
__global__ void k_publish(launch::SearchBuffers b, launch::HostSide h, uint32_t seq, uint32_t n) {
  const DevState* st = b.st;
  const int tid = threadIdx.x;
  const uint32_t status = st->status == kFound ? kFound : kNoPath;
  const int d0 = st->depth[0], d1 = st->depth[1];
  const uint32_t hops = (uint32_t)(d0 + d1);
  uint32_t* out = (hops + 1 <= h.path_cap) ? h.path : b.dpath;
  if (status == kFound && (tid == 0 || tid == kWave)) {
    walk_side(b.parent[tid ? 1 : 0], n, st->meet, tid ? 1 : 0, d0, d1, out);
    __threadfence_system();
  }
  __syncthreads();
  if (tid == 0) {
    HostResult* R = h.res;
    R->rt_walk = 0;  // (no rt_end stamp here: the host times this path with events)
    R->status = status;
    R->hops = status == kFound ? (int32_t)hops : -1;
    R->meet = st->meet;
    R->levels = st->levels;
    R->visited = st->qtail[0] + st->qtail[1];
    R->einsp = st->einsp;
    R->depth[0] = d0;
    R->depth[1] = d1;
    R->path_len = status == kFound ? hops + 1 : 0u;
    R->path_on_device = (status == kFound && hops + 1 > h.path_cap) ? 1u : 0u;
    __threadfence_system();
    __hip_atomic_store(&R->seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Reset the visited words of every vertex a grid search claimed (all of them
// are in the queues), so the next search starts from all-zero bitmaps without
// an O(N) memset.
// Clears the visited words of every queued vertex.  The last workgroup then
// writes `tag` to pinned host memory: the resident server runs on another
// stream, so the host checks the tag before a new search may hand off into
// these bitmaps.
// if_done: enqueued behind every grid level, it only runs once a level has
// ended the search (then right behind that level, with no launch latency).
__global__ void k_cleanup(launch::SearchBuffers b, uint32_t* done_ctr, uint32_t* host_tag, uint32_t tag,
                          int if_done) {
  const DevState* st = b.st;
  if (if_done == 2 && !(load_agent(&b.aux[2]) & kAuxTook)) return;  // no auto level ran (grid-uniform)
  if (if_done && load_agent(&st->status) == kRunning) return;  // grid-uniform
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x, t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  if (((uint64_t)st->qtail[0] + st->qtail[1]) * 32 > b.words) {
    // a large visited set (a hub level): streaming every word beats one
    // dependent queue load per cleared word
    for (int s = 0; s < 2; ++s) {
      uint4* w4 = reinterpret_cast<uint4*>(b.vis[s]);
      const uint64_t n4 = b.words / 4;
      for (uint64_t i = t0; i < n4; i += stride) w4[i] = make_uint4(0u, 0u, 0u, 0u);
      for (uint64_t i = n4 * 4 + t0; i < b.words; i += stride) b.vis[s][i] = 0u;
    }
  } else {
    for (int s = 0; s < 2; ++s) {
      const uint32_t q = st->qtail[s];
      for (uint64_t i = t0; i < q; i += stride) b.vis[s][b.queue[s][i] >> 5] = 0u;
    }
  }
  // every wave's clears drained, then ONE agent release per workgroup (a
  // __threadfence() in every thread was a write-back + invalidate per lane:
  // ~20 us of a 10M cleanup) before the block counts itself done
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (threadIdx.x == 0 && atomicAdd(done_ctr, 1u) == gridDim.x - 1) {
    *done_ctr = 0;
    __threadfence_system();
    __hip_atomic_store(host_tag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// K2/K4 parity: any vertex visited by both sides (bitmap AND + wave any).
__global__ void k_bitmap_meet(launch::SearchBuffers b, uint32_t* flag) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < b.words;
       i += (uint64_t)gridDim.x * blockDim.x)
    acc |= b.vis[0][i] & b.vis[1][i];
  if (__any(acc != 0) && __lane_id() == 0) atomicOr(flag, 1u);
}

template <typename OffT>
GridParams<OffT> gp(const launch::GraphView& g, const launch::SearchBuffers& b, int side) {
  GridParams<OffT> P;
  P.row_off = reinterpret_cast<const OffT*>(g.row_off32 ? (const void*)g.row_off32 : (const void*)g.row_off);
  P.col = g.col;
  P.n = g.n;
  P.side = side;
  P.b = b;
  P.mirror = nullptr;
  P.seq = 0;
  P.trace = 0;
  P.h = launch::HostSide{nullptr, nullptr, 0, nullptr};
  P.res_seq = 0;
  P.hub_deg = kHubDegree;
  P.chunk_v = kGridThreads;
  P.gate_seq = 0;
  P.gate_ticks = 0;
  P.cus = 0;
  P.max_deg = 0;
  P.nnz = g.nnz;
  P.alpha = 14.0f;
  P.nparts = 0;
  P.fbase = P.fcount = 0;
  P.chain = 0;
  P.hub_direct = 0;
  P.precheck = 1;
  P.padj = kGridPadj ? g.padj : nullptr;
  P.padj8 = kGridPadj ? g.padj8 : nullptr;
  return P;
}

}  // namespace

namespace launch {

int lds_threads() { return kLdsThreads; }

// frontier edges the meet probe may read before a hand-off (default of
// HipBiBfs::set_lds_probe_edges; 0 = off)
uint32_t lds_probe_budget() { return 16384u; }

// The probe runs on graphs whose largest degree is above 64 (hub graphs): on
// G(n, p) it hit a quarter of the 10M hand-offs but a miss costs ~9 us on a
// near-full hash set, a wash (profiles/r5_lds_coop_append_probe_ab.jsonl).
constexpr uint64_t kProbeMinDeg = 64;
static uint32_t probe_for(const GraphView& g) { return g.max_deg > kProbeMinDeg ? g.probe_edges : 0u; }

size_t lds_bytes(bool wide) {
  return 2 * kHashSize * 4 + 4 * (wide ? LdsRec<uint64_t>::cap * 16 : LdsRec<uint32_t>::cap * 8) + 128;
}

void lds_search(const GraphView& g, const SearchBuffers& b, const HostSide& h, uint32_t src,
                uint32_t dst, uint32_t seq, int side_policy, int trace, int pin_xcc, uint32_t* ticket,
                int lockstep, hipStream_t s) {
  // 16 blocks = 2 per XCD under round-robin dispatch; only the elected one works
  const unsigned blocks = pin_xcc >= 0 ? 16 : 1;
  if (g.row_off32) {
    LdsParams<uint32_t> P{g.row_off32, g.col, g.padj, g.padj8, g.n, src, dst, seq, side_policy, trace, pin_xcc, ticket,
                           lockstep, (uint32_t)(g.nnz ? g.nnz - 1 : 0), 0, b, h};
    P.wave_hash = g.max_deg <= kWaveHashMaxDeg ? 1 : 0;
    P.probe = probe_for(g);
    const bool bm = g.n <= kBmMaxN;  // whole visited sets fit LDS as bitmaps
    if (trace == 2) {
      if (bm) k_lds_bibfs<uint32_t, true, true><<<blocks, kLdsThreads, 0, s>>>(P);
      else k_lds_bibfs<uint32_t, true, false><<<blocks, kLdsThreads, 0, s>>>(P);
    } else {
      if (bm) k_lds_bibfs<uint32_t, false, true><<<blocks, kLdsThreads, 0, s>>>(P);
      else k_lds_bibfs<uint32_t, false, false><<<blocks, kLdsThreads, 0, s>>>(P);
    }
  } else {
    LdsParams<uint64_t> P{g.row_off, g.col, g.padj, nullptr, g.n, src, dst, seq, side_policy, trace, pin_xcc, ticket,
                           lockstep, (uint64_t)(g.nnz ? g.nnz - 1 : 0), 0, b, h};
    P.probe = probe_for(g);
    if (trace == 2)
      k_lds_bibfs<uint64_t, true, false><<<blocks, kLdsThreads, 0, s>>>(P);
    else
      k_lds_bibfs<uint64_t, false, false><<<blocks, kLdsThreads, 0, s>>>(P);
  }
  HIP_CHECK(hipGetLastError());
}

void lds_server(const GraphView& g, const SearchBuffers& b, const SearchBuffers& b_alt, const HostSide& h,
                dev::ServerBox* box, uint32_t launch_seq, uint32_t last_seq, int pin_xcc, uint32_t* ticket,
                unsigned long long idle_ticks, bool stamp_server, hipStream_t s) {
  const unsigned blocks = pin_xcc >= 0 ? 16 : 1;
  if (!g.row_off32) {  // nnz >= 2^32 (Kronecker 27+): 64-bit offsets, hash-set mode
    LdsParams<uint64_t> P{g.row_off, g.col, g.padj, nullptr, g.n, 0, 0, launch_seq, 0, 0, pin_xcc, ticket, 1,
                          (uint64_t)(g.nnz ? g.nnz - 1 : 0), 0, b, h};
    P.b_alt = b_alt;
    P.probe = probe_for(g);
    k_lds_server<uint64_t, false><<<blocks, kLdsThreads, 0, s>>>(P, box, last_seq, idle_ticks);
    HIP_CHECK(hipGetLastError());
    return;
  }
  LdsParams<uint32_t> P{g.row_off32, g.col, g.padj, g.padj8, g.n, 0, 0, launch_seq, 0, 0, pin_xcc, ticket, 1,
                         (uint32_t)(g.nnz ? g.nnz - 1 : 0), 0, b, h};
  P.b_alt = b_alt;
  P.wave_hash = g.max_deg <= kWaveHashMaxDeg ? 1 : 0;
  P.probe = probe_for(g);
  if (g.n <= kBmMaxN && stamp_server)  // cycle stamps of the server's phases
    k_lds_server<uint32_t, true, true><<<blocks, kLdsThreads, 0, s>>>(P, box, last_seq, idle_ticks);
  else if (g.n <= kBmMaxN)
    k_lds_server<uint32_t, true><<<blocks, kLdsThreads, 0, s>>>(P, box, last_seq, idle_ticks);
  else
    k_lds_server<uint32_t, false><<<blocks, kLdsThreads, 0, s>>>(P, box, last_seq, idle_ticks);
  HIP_CHECK(hipGetLastError());
}

void lds_batch(const GraphView& g, const SearchBuffers& b, uint32_t* d_src, uint32_t* d_dst,
               uint32_t k, uint32_t* d_slots, dev::HostResult* h_res, uint32_t* h_path, uint32_t path_cap,
               uint32_t seq, hipStream_t s) {
  BIBFS_REQUIRE(g.row_off32 != nullptr, "batched search: 32-bit row offsets required");
  LdsParams<uint32_t> P{g.row_off32, g.col, g.padj, g.padj8, g.n, 0, 0, seq, 0, 0, -1, nullptr, 1,
                         (uint32_t)(g.nnz ? g.nnz - 1 : 0), 1, b, HostSide{h_res, h_path, path_cap}};
  BatchArgs A{d_src, d_dst, d_slots, h_res, h_path, path_cap, seq};
  if (g.n <= kBmMaxN)
    k_lds_batch<uint32_t, true><<<k, kLdsThreads, 0, s>>>(P, A);
  else
    k_lds_batch<uint32_t, false><<<k, kLdsThreads, 0, s>>>(P, A);
  HIP_CHECK(hipGetLastError());
}

void seed_state(const GraphView& g, const SearchBuffers& b, uint32_t src, uint32_t dst,
                hipStream_t s) {
  if (g.row_off32)
    k_seed<uint32_t><<<1, 64, 0, s>>>(g.row_off32, b, src, dst);
  else
    k_seed<uint64_t><<<1, 64, 0, s>>>(g.row_off, b, src, dst);
  HIP_CHECK(hipGetLastError());
}

uint32_t grid_hub_degree() { return kHubDegree; }


void grid_topdown(const GraphView& g, const SearchBuffers& b, int side, int cus, uint64_t frontier,
                  uint64_t frontier_edges, dev::DevState* mirror, uint32_t seq, int trace, const HostSide& h, uint32_t res_seq,
                  uint32_t hub_deg, hipStream_t s) {
  // Dynamic chunks of frontier vertices; never more blocks than chunks:
  // every block takes at least one ticket from ONE counter, and 1024 blocks
  // contending on it cost ~12 us even for a 3-vertex frontier.  A chunk is
  // sized to about one 256-edge batch of the frontier's mean degree (64..256
  // vertices): a block walks its chunk's edges in serial batches, each a chain
  // of dependent loads and atomics, so a mid-size frontier (10^3-10^5
  // vertices, degree ~2) spreads over 4x the blocks instead of running ~3
  // batches back to back on a few CUs.  Frontiers that fill every block keep
  // 256-vertex chunks (fewer ticket atomics).
  uint64_t cv = kGridThreads;
  if ((frontier + kGridThreads - 1) / kGridThreads < (uint64_t)cus * 4 && frontier_edges > 0)
    cv = std::min<uint64_t>(kGridThreads, std::max<uint64_t>(kGridChunkMin, kGridThreads * kGridChunkFill * frontier /
                                                                               (100 * frontier_edges)));
  const uint64_t chunks = (frontier + cv - 1) / cv;
  const unsigned blocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus * 4, chunks));
  const unsigned hblocks = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)cus * 4, frontier * 4));
  // A hub level whose whole frontier fits one hub tile runs as ONE edge-parallel
  // pass over every frontier edge (k_grid_hubs, hub_direct): the top-down pass
  // would walk its light vertices on frontier/cv workgroups (one, for a
  // Kronecker hub level of ~40 vertices: ~10 us) before the hub pass starts.
  // Measured (profiles/r4_grid_hub_direct_ab.jsonl, mean search): Kronecker 22
  // 47.4-48.5 -> 40.6-42.1 us, Kronecker 25 60.8 -> 48.7 us.  Sizing that
  // pass by edges instead (mode 2: up to 1024 workgroups) lost: 57.1 us.
  // With the hub-free small heavy levels too (profiles/r4_grid_direct_levels_ab.jsonl):
  // Kronecker 22 46.9-48.1 -> 38.0-38.3 us, Kronecker 25 56.2-57.9 -> 44.0-44.2
  // us against no direct levels; 10M G(n, p) unchanged.
  // (also a level without hubs whose top-down pass would walk more than
  // kGridDirectBatches 256-edge batches per workgroup: a few heavy-ish
  // vertices on one block)
  const bool direct = frontier <= (uint64_t)kHubTile &&
                      (hub_deg != ~0u || frontier_edges > kGridDirectBatches * kGridThreads * blocks);
  auto launch_one = [&](auto P) {
    using OffT = std::remove_const_t<std::remove_pointer_t<decltype(P.row_off)>>;
    P.mirror = mirror, P.seq = seq, P.trace = trace, P.h = h, P.res_seq = res_seq;
    P.hub_deg = hub_deg;  // ~0u: no hub pass
    P.chunk_v = (uint32_t)cv;
    P.precheck = (!kGridFast || frontier_edges > kGridPrecheckEdges) ? 1 : 0;
    if (P.precheck || !kGridPadj) P.padj = nullptr, P.padj8 = nullptr;
    if (direct) {
      P.hub_direct = 1;
      k_grid_hubs<OffT><<<hblocks, kGridThreads, 0, s>>>(P);
      return;
    }
    k_grid_topdown<OffT><<<blocks, kGridThreads, 0, s>>>(P);
    if (hub_deg != ~0u) k_grid_hubs<OffT><<<hblocks, kGridThreads, 0, s>>>(P);
  };
  if (g.row_off32) launch_one(gp<uint32_t>(g, b, side));
  else launch_one(gp<uint64_t>(g, b, side));
  HIP_CHECK(hipGetLastError());
}

void grid_auto(const GraphView& g, const SearchBuffers& b, int cus, uint64_t max_deg, double alpha,
               dev::DevState* mirror, uint32_t seq, const HostSide& h, uint32_t res_seq, uint32_t gate_seq,
               unsigned long long gate_ticks, int levels, hipStream_t s) {
  // The grid size is fixed before the frontier exists: cus / 4 workgroups
  // for the first level (a 10M G(n, p) hand-off level is ~17 chunks; every
  // workgroup takes chunk tickets, and fewer blocks keep the ticket and done
  // counters cheap), one per CU for a chained level (a frontier ~2x larger:
  // the blocks beyond its chunk count leave at once).  The hub pass behind a
  // level is enqueued only when the graph has a vertex above 64.
  const unsigned blocks = (unsigned)std::max(8, cus / 4);
  const unsigned cblocks = (unsigned)std::max(8, cus);
  // the hub pass: the host's grid size for a hub level (4 blocks per frontier
  // vertex up to 4 per CU; k_grid_hubs<auto> leaves the blocks beyond it)
  const unsigned hblocks = (unsigned)std::max(8, cus * 4);
  const int scatter = g.n > kBmMaxN ? 1 : 0;
  auto launch_one = [&](auto P) {
    using OffT = std::remove_const_t<std::remove_pointer_t<decltype(P.row_off)>>;
    P.mirror = mirror, P.seq = seq, P.trace = 0, P.h = h, P.res_seq = res_seq;
    P.gate_seq = gate_seq;
    P.gate_ticks = gate_ticks;
    P.cus = (uint32_t)cus;
    P.max_deg = max_deg;
    P.nnz = g.nnz;
    P.alpha = (float)alpha;
    P.chain = 0;
    // the planners may choose direct hub levels (only with the hub pass enqueued)
    P.hub_direct = max_deg > 64 ? 1 : 0;
    k_handoff<OffT><<<kHandoffBlocks, kGridThreads, 0, s>>>(P, 1, scatter);
    for (int l = 0; l < std::max(1, levels); ++l) {
      P.chain = l + 1 < levels ? 1 : 0;
      k_grid_topdown<OffT, true><<<l ? cblocks : blocks, kGridThreads, 0, s>>>(P);
      if (max_deg > 64) k_grid_hubs<OffT, true><<<hblocks, kGridThreads, 0, s>>>(P);
    }
  };
  if (g.row_off32) launch_one(gp<uint32_t>(g, b, 0));
  else launch_one(gp<uint64_t>(g, b, 0));
  HIP_CHECK(hipGetLastError());
}


void handoff_scatter(const GraphView& g, const SearchBuffers& b, hipStream_t s) {
  if (g.n <= kBmMaxN) return;  // bitmap-mode searches copied their bitmaps themselves
  if (g.row_off32) k_handoff<uint32_t><<<kHandoffBlocks, kGridThreads, 0, s>>>(gp<uint32_t>(g, b, 0), 0, 1);
  else k_handoff<uint64_t><<<kHandoffBlocks, kGridThreads, 0, s>>>(gp<uint64_t>(g, b, 0), 0, 1);
  HIP_CHECK(hipGetLastError());
}

size_t handoff_dump_bytes() { return 2 * kHashSize * sizeof(uint32_t); }

void grid_bottomup(const GraphView& g, const SearchBuffers& b, int side, int cus, hipStream_t s) {
  const uint64_t waves = ((uint64_t)g.n + 63) / 64;
  uint64_t blocks = (waves + 3) / 4;
  const uint64_t cap = (uint64_t)cus * 8;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  if (g.row_off32) {
    auto P = gp<uint32_t>(g, b, side);
    k_grid_bottomup<uint32_t><<<(unsigned)blocks, kGridThreads, 0, s>>>(P);
  } else {
    auto P = gp<uint64_t>(g, b, side);
    k_grid_bottomup<uint64_t><<<(unsigned)blocks, kGridThreads, 0, s>>>(P);
  }
  HIP_CHECK(hipGetLastError());
}

void build_frontier_bits(const GraphView& g, const SearchBuffers& b, int side, hipStream_t s) {
  (void)g;
  HIP_CHECK(hipMemsetAsync(b.fbits[side], 0, (size_t)b.words * 4, s));
  k_frontier_bits<<<1024, 256, 0, s>>>(b, side);
  HIP_CHECK(hipGetLastError());
}

void finish_level(const SearchBuffers& b, int side, int mode, int trace, DevState* mirror, uint32_t seq,
                  const HostSide& h, uint32_t res_seq, uint32_t n, hipStream_t s) {
  k_finish_level<<<1, 128, 0, s>>>(b, side, mode, trace, mirror, seq, h, res_seq, n);
  HIP_CHECK(hipGetLastError());
}

void bitmap_meet(const SearchBuffers& b, uint32_t* d_flag, hipStream_t s) {
  HIP_CHECK(hipMemsetAsync(d_flag, 0, 4, s));
  k_bitmap_meet<<<1024, 256, 0, s>>>(b, d_flag);
  HIP_CHECK(hipGetLastError());
}

void walk_path(const SearchBuffers& b, const HostSide& h, uint32_t src, uint32_t dst, uint32_t seq,
               uint32_t n, hipStream_t s) {
  (void)src;
  (void)dst;
  k_publish<<<1, 128, 0, s>>>(b, h, seq, n);
  HIP_CHECK(hipGetLastError());
}

void cleanup(const SearchBuffers& b, uint32_t n, uint32_t* done_ctr, uint32_t* host_tag, uint32_t tag,
             int if_done, hipStream_t s) {
  (void)n;
  k_cleanup<<<64, 1024, 0, s>>>(b, done_ctr, host_tag, tag, if_done);  // few blocks: one done-counter atomic each
  HIP_CHECK(hipGetLastError());
}

}  // namespace launch
}  // namespace bibfs
