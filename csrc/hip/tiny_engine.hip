// Small-graph resident query server: the latency path of the headline config
// (G(n, 2.2/n), 100k vertices, one query at a time, path returned to the host).
//
// What the reference does per level (v3/bibfs_cuda_only.cu:173-203): three
// launches over all N vertices, ~8 host<->device copies and a printf.  Here a
// whole query is a few hundred nanoseconds of LDS work per level inside ONE
// persistent workgroup that never leaves the GPU:
//   * the graph is read through a packed adjacency (8 B per directed edge:
//     neighbour id, its CSR base, its degree -- device.hpp tiny_pack), so a
//     level costs exactly one dependent global load (the neighbour word,
//     L2-resident: the server is pinned to one XCD) and everything after it
//     is LDS;
//   * both visited sets are LDS bitmaps with two bits per vertex (claimed at
//     an even / odd depth), so a claim is one ds_or_rtn_b64 and the other
//     side's bits are read right behind it -- the meet test is fused into the
//     claim, and the depth parity of a hit gives the candidate's exact length
//     (the first-meet rule, docs/DESIGN.md §2);
//   * both frontiers are expanded in the same round ("lockstep") by all 16
//     waves, one frontier edge per lane, with ONE LDS-only barrier per round;
//     new vertices go to per-side LDS queues (vertex | parent's queue index)
//     and their edges straight into the next round's per-edge records, so a
//     round needs no degree scan and no edge -> vertex search;
//   * the path is walked in LDS (one LDS load per hop, both chains at once);
//   * the answer goes to pinned host memory as self-tagged 16-byte packets
//     (TinyPkt): no release fence, no flag store behind the payload.
// Records that do not fit the LDS buffers spill to global memory (all-wave
// rounds, L2-resident; a round of up to ~4k items runs in two passes), so a
// long-path query's big last level still ends here.  Queries that still do
// not fit (a round above 4095 items, a queue above kTinyQ without a meet)
// answer kTinyOverflow and the host re-runs them on the general engine
// (engine_kernels.hip), which has the grid hand-off.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "device.hpp"

namespace bibfs {
namespace {

using namespace dev;

#ifndef BIBFS_TINY_THREADS
#define BIBFS_TINY_THREADS 1024
#endif
constexpr int kTT = BIBFS_TINY_THREADS;
constexpr uint32_t kTW = kTinyMaxN / 32;  // u64 visited words per side (low half even, high half odd)
constexpr uint32_t kTRC = 2008;           // per-edge records per side per buffer
constexpr uint32_t kQBits = 12;
constexpr uint32_t kTinyUnroll = 4;  // record stores per new vertex without a loop
// Rounds whose two frontiers together exceed this many edges expand the side
// with fewer edges alone (lockstep below it).  1024 measured best on
// G(100k, 6/n): 14.7 us mean query vs 17.2 at 2048 (fewer queue overflows,
// 31 vs 218 in 1920 queries) and 15.4 at 512 -- profiles/r3_tiny_ab.jsonl.
#ifndef BIBFS_TINY_LOCK_MAX
#define BIBFS_TINY_LOCK_MAX 1024
#endif
constexpr uint32_t kLockMax = BIBFS_TINY_LOCK_MAX;
// All-wave rounds: 1 = fetch each neighbour's first edges speculatively at the
// round's start (beside the claim), 0 = only for the vertices claimed, after
// the claim.  With one 8-byte load per edge word 16 waves of speculative
// scattered loads queued on the address unit (17.6 vs 17.2 us,
// profiles/r3_tiny_ab.jsonl); with the two 16-byte loads of BIBFS_TINY_X4 the
// speculation wins: 14.15-14.19 vs 14.42-14.52 us mean query
// (profiles/r3_tiny_specall_ab.jsonl).
#ifndef BIBFS_TINY_SPEC_ALL
#define BIBFS_TINY_SPEC_ALL 1
#endif
constexpr bool kSpecAll = BIBFS_TINY_SPEC_ALL;
// 1 = a neighbour's first kTinyUnroll edge words come in with two 16-byte
// loads under one exec mask (tadj is padded by kTinyUnroll words), 0 = one
// 8-byte load per word, each under its own degree mask.
// 1 measured 14.5 vs 14.8 us mean query, device 11.45 vs 11.77 us
// (profiles/r3_tiny_x4_ab.jsonl).
#ifndef BIBFS_TINY_X4
#define BIBFS_TINY_X4 1
#endif
constexpr bool kX4 = BIBFS_TINY_X4;
// 1 = single-wave rounds of at most 64 edges run a one-item body (see the loop)
#ifndef BIBFS_TINY_SW_SPLIT
#define BIBFS_TINY_SW_SPLIT 1
#endif
constexpr bool kSwSplit = BIBFS_TINY_SW_SPLIT;
// Items per lane of the widest single-wave round (2 or 4): with 4, rounds of
// 129-256 edges stay on wave 0 (no barrier, SGPR state) instead of starting
// the all-wave phase.  Measured slower: device 11.61-11.75 vs 10.55-10.63 us
// mean per 100k query (profiles/r4_tiny_sw4_ab.jsonl) -- a 4-item wave-0
// round costs more than the 16-wave round it replaces.  Off (2).
#ifndef BIBFS_TINY_SW_NB
#define BIBFS_TINY_SW_NB 2
#endif
constexpr int kSwNB = BIBFS_TINY_SW_NB;
static_assert(kSwNB == 2 || kSwNB == 4, "single-wave items per lane");
// 1 = all-wave rounds of at most kTT edges run a one-item body
#ifndef BIBFS_TINY_AW_SPLIT
#define BIBFS_TINY_AW_SPLIT 1
#endif
constexpr bool kAwSplit = BIBFS_TINY_AW_SPLIT;
typedef unsigned long long u64x2a8 __attribute__((ext_vector_type(2), aligned(8)));
static_assert(kTinyUnroll == 4, "two 16-byte loads per neighbour");
// 1 = the second 16-byte load (edge words 2, 3) only for a neighbour with
// more than two edges (at G(n, 2.2/n) ~60% of the vertices have at most
// two).  Measured no gain: 14.50-14.56 vs 14.38-14.48 us mean query, device
// 11.48-11.54 vs 11.41-11.47 us (profiles/r4_tiny_lazy2_ab.jsonl, 2 x 1920
// queries each) -- the masked lines are not what bounds a round.  Off.
#ifndef BIBFS_TINY_LAZY2
#define BIBFS_TINY_LAZY2 0
#endif
constexpr bool kLazy2 = BIBFS_TINY_LAZY2;
// 1 = all-wave rounds spill next-round records past the LDS buffers to global
// memory (TinyArgs::spill) instead of answering kTinyOverflow
#ifndef BIBFS_TINY_SPILL
#define BIBFS_TINY_SPILL 1
#endif
constexpr bool kSpillOn = BIBFS_TINY_SPILL;
__device__ __forceinline__ void load_first4(unsigned long long (&w)[kTinyUnroll],
                                            const unsigned long long* __restrict__ p, uint32_t deg) {
  if (deg) {  // (exec-masked per lane)
    const u64x2a8 a = *reinterpret_cast<const u64x2a8*>(p);
    w[0] = a.x, w[1] = a.y;
  }
  if (kLazy2 ? deg > 2 : deg > 0) {
    const u64x2a8 b = *reinterpret_cast<const u64x2a8*>(p + 2);
    w[2] = b.x, w[3] = b.y;
  }
}
static_assert(kTinyQ == 1u << kQBits, "queue index width");

// Per-round counter (three slots, rotated): new records of side 0 [19:0] and
// side 1 [39:20], new queue entries of side 0 [51:40] and side 1 [63:52].
// Field bounds: a round has at most kMaxRound = 4095 items, so at most 4095
// new vertices per side (< 2^12); the record fields take 20 bits, so each
// wave's record count is clamped to kTRC + kTinySpill + 1 when it is added
// (past that the records overflow anyway, caught per lane).
struct TinyCtl {
  unsigned long long cnt[3];
  unsigned long long meet;   // min over candidates of len << 32 | side << 31 | queue index; 0 = overflow
  uint32_t other_q;          // the meet vertex's queue index on the other side
  uint32_t rovf;             // a record buffer overflowed (fatal only without a meet)
  uint32_t won;
  uint32_t cmd[4];           // stop, seq, src, dst
};

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ unsigned long long uni64(unsigned long long x) {
  return (unsigned long long)uni((uint32_t)x) | (unsigned long long)uni((uint32_t)(x >> 32)) << 32;
}
__device__ __forceinline__ uint32_t lane0(uint32_t x) { return __builtin_amdgcn_readlane(x, 0); }
__device__ __forceinline__ uint32_t lane63(uint32_t x) { return __builtin_amdgcn_readlane(x, 63); }

__device__ __forceinline__ uint32_t xcc_id() {
  uint32_t x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & 0xf;
}

// LDS-only workgroup barrier: the rounds issue no global stores, so there is
// nothing in vmcnt to drain (the global loads were consumed before it).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Inclusive wave64 prefix sum on the VALU via DPP (row shifts, then row
// broadcasts 15 / 31): no LDS permutes.
__device__ __forceinline__ uint32_t wave_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// One 16-byte system-scope store (write-through to pinned host memory).
__device__ __forceinline__ void store_sys16(TinyPkt* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
}

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// Per-round state every wave holds identically (SGPRs), handed from the
// single-wave phase to the all-wave phase through LDS.
struct TinyState {
  uint32_t status, E0, E1, cb0, cb1, d0, d1, ql0, ql1, levels, x0, x1;
  unsigned long long einsp, meet;
};

// tiny word fields (device.hpp tiny_pack) and the record's parent index
__device__ __forceinline__ uint32_t tw_v(unsigned long long w) { return (uint32_t)(w >> 35) & 0x1FFFFu; }
__device__ __forceinline__ uint32_t tw_base(unsigned long long w) { return (uint32_t)(w >> 9) & 0x3FFFFFFu; }
__device__ __forceinline__ uint32_t tw_deg(unsigned long long w) { return (uint32_t)w & 0x1FFu; }
__device__ __forceinline__ uint32_t tw_pq(unsigned long long w) { return (uint32_t)(w >> 52); }

// Uniform description of one round.
struct RoundCtx {
  uint32_t x0, tot;                  // items [0, x0) are side 0's records, [x0, tot) side 1's
  const unsigned long long* rb0;     // side 0's current records
  const unsigned long long* rb1x;    // side 1's current records, minus x0 (indexed by the item)
  unsigned long long* nb[2];         // next-round record buffers
  // records past the LDS buffers (slot >= kTRC) live in global memory
  // (TinyArgs::spill, [buffer][side][kTinySpill]); the slices are computed
  // only on the rare paths that touch them, to keep this context small
  unsigned long long* spill;
  uint32_t cb;                       // current record buffer per side: bit 0 side 0, bit 1 side 1
  bool spilled;                      // a side's current records pass kTRC (uniform)
  uint32_t par[2];                   // depth parity bit of this round's claims per side
  uint32_t dep[2];                   // frontier depth per side before the round
  bool exp[2];                       // the side expands this round
};

// One lane's NB items (frontier edges) of a round.
template <int NB>
struct Work {
  unsigned long long rec[NB];        // the record: the neighbour's tiny word | parent queue index << 52
  unsigned long long nbw[NB][kTinyUnroll];  // the neighbour's first edges' words (speculative)
  unsigned long long oth[NB];        // the other side's visited word of the neighbour
  bool act[NB], s1[NB], nw[NB];
  uint32_t deg[NB];                  // degree of the neighbour when this lane claimed it (else 0)
};

// Round step 1: read the records, and at once issue the loads of each
// neighbour's first edges (the NEXT round's records, fetched speculatively
// so their latency overlaps the claim) and the claims.  Branch-free: an idle
// lane reads a harmless word and claims with an empty mask.
template <int NB, bool kSpec, bool kSpill>
__device__ __forceinline__ void round_issue(Work<NB>& W, const RoundCtx& R, uint32_t i0, uint32_t stride, int nb,
                                            const unsigned long long* __restrict__ tadj,
                                            unsigned long long (*VIS)[kTW]) {
  unsigned long long old[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint32_t i = i0 + (uint32_t)b * stride;
    W.act[b] = i < R.tot;
    W.s1[b] = i >= R.x0;
    W.rec[b] = 1ull;  // an idle lane: vertex 0, base 0, degree 1
    if (b < nb && W.act[b]) {
      const uint32_t li = W.s1[b] ? i - R.x0 : i;  // the record's slot in its side's buffer
      if (!kSpill || !R.spilled || li < kTRC) W.rec[b] = (W.s1[b] ? R.rb1x : R.rb0)[i];
      else  // a spilled record (written by another wave last round: L2, past this CU's L1)
        W.rec[b] = __hip_atomic_load(R.spill + (size_t)(((R.cb >> (W.s1[b] ? 1 : 0)) & 1u) * 2 + (W.s1[b] ? 1 : 0)) *
                                                  kTinySpill + (li - kTRC), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (kSpec) {
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (b >= nb) continue;
      const uint32_t base = tw_base(W.rec[b]), deg = W.act[b] ? tw_deg(W.rec[b]) : 0u;
      if (kX4) {
        load_first4(W.nbw[b], tadj + base, deg);
        continue;
      }
#pragma unroll
      for (uint32_t j = 0; j < kTinyUnroll; ++j)
        if (j < deg) W.nbw[b][j] = tadj[base + j];  // exec-masked: no address for a missing edge
    }
  }
  // claim, then read the other side's word: the LDS executes one wave's DS
  // instructions in order, so of two same-round claims of a vertex by the two
  // sides at least one sees the other.  That needs every claim ISSUED before
  // the other-side reads; the two are relaxed atomics on different words,
  // which the C++ model would let the compiler reorder (a store-buffer /
  // Dekker pattern), so a compiler-only fence pins the order (no instruction:
  // the hardware order then comes from in-order DS issue).
  // (word indices, not pointers: a pointer select here lost the LDS address
  // space, and the other-side read became a flat load -- whose lgkmcnt wait
  // then also waited for the speculative global loads issued just above)
  uint32_t wi[NB];
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    old[b] = W.oth[b] = 0ull;
    wi[b] = (W.s1[b] ? kTW : 0u) + (tw_v(W.rec[b]) >> 5);  // own word in the flat [2][kTW] set
    if (b >= nb) continue;
    const uint32_t v = tw_v(W.rec[b]);
    const uint32_t par = W.s1[b] ? R.par[1] : R.par[0];
    const unsigned long long m = W.act[b] ? 1ull << ((v & 31) + (par << 5)) : 0ull;
    old[b] = __hip_atomic_fetch_or(&VIS[0][0] + wi[b], m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b >= nb) continue;
    W.oth[b] = __hip_atomic_load(&VIS[0][0] + (wi[b] ^ kTW), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint32_t bt = tw_v(W.rec[b]) & 31;
    W.nw[b] = b < nb && W.act[b] && ((((uint32_t)old[b] | (uint32_t)(old[b] >> 32)) >> bt) & 1u) == 0;
    W.deg[b] = W.nw[b] ? tw_deg(W.rec[b]) : 0u;
  }
}

// The claimed vertices' first edges (the next round's records), fetched as
// soon as the claims are known -- their latency overlaps the counts and the
// round counter's atomic instead of stalling the place step.
template <int NB>
__device__ __forceinline__ void round_fetch(Work<NB>& W, int nb, const unsigned long long* __restrict__ tadj) {
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b >= nb) continue;
    const uint32_t base = tw_base(W.rec[b]);
    if (kX4) {
      load_first4(W.nbw[b], tadj + base, W.deg[b]);
      continue;
    }
#pragma unroll
    for (uint32_t j = 0; j < kTinyUnroll; ++j)
      if (j < W.deg[b]) W.nbw[b][j] = tadj[base + j];
  }
}

// Per-lane and per-wave counts of the new vertices: queue slots from ballots,
// record slots from ONE DPP scan of the degrees (side 0 [15:0], side 1
// [31:16]) while a wave's sum fits 16 bits (NB <= 2), else one scan per side.
template <int NB>
struct Counts {
  uint32_t qpre[NB];  // new vertices of this lane's side below this lane (in batches < b, then lanes < lane)
  uint32_t qt[2];     // the wave's new vertices per side (uniform)
  uint32_t ex[2], et[2];  // exclusive / total (uniform) record counts per side
};
template <int NB>
__device__ __forceinline__ void round_count(Counts<NB>& K, const Work<NB>& W) {
  uint32_t ep = 0, ep1 = 0;
  constexpr bool kPacked = 64u * NB * kTinyMaxDeg < 65536u;
  K.qt[0] = K.qt[1] = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const unsigned long long m0 = __ballot(W.nw[b] && !W.s1[b]), m1 = __ballot(W.nw[b] && W.s1[b]);
    K.qpre[b] = W.s1[b] ? K.qt[1] + mbcnt64(m1) : K.qt[0] + mbcnt64(m0);
    K.qt[0] += (uint32_t)__popcll(m0);
    K.qt[1] += (uint32_t)__popcll(m1);
    if (kPacked) {
      ep += W.deg[b] << (W.s1[b] ? 16 : 0);
    } else {
      ep += W.s1[b] ? 0u : W.deg[b];
      ep1 += W.s1[b] ? W.deg[b] : 0u;
    }
  }
  const uint32_t ei = wave_scan(ep);
  if (kPacked) {
    K.ex[0] = (ei - ep) & 0xffffu;
    K.ex[1] = (ei - ep) >> 16;
    const uint32_t t = lane63(ei);
    K.et[0] = t & 0xffffu;
    K.et[1] = t >> 16;
  } else {
    const uint32_t ei1 = wave_scan(ep1);
    K.ex[0] = ei - ep;
    K.ex[1] = ei1 - ep1;
    K.et[0] = lane63(ei);
    K.et[1] = lane63(ei1);
  }
}

// Round step 2: queue entries, next-round records (the speculatively loaded
// words, tagged with the new vertex's queue index) and meet candidates.
// q0b/q1b: queue index of the wave's first new vertex per side; e0b/e1b: its
// first record slot per side.  Returns kOvfQueue when a queue would overflow
// (fatal: the path walk needs every entry) and kOvfRec when a record buffer
// would (fatal only if the round finds no meet: records feed the NEXT round).
// A lane with nothing to store writes its own junk slot (no branch).
// kCand (every lane, wave-uniform): the wave stored a meet candidate this round
constexpr uint32_t kOvfQueue = 1, kOvfRec = 2, kCand = 4;
template <int NB, bool kSpec, bool kSpill>
__device__ __forceinline__ uint32_t round_place(Work<NB>& W, const Counts<NB>& K, const RoundCtx& R, int nb,
                                                uint32_t q0b, uint32_t q1b, uint32_t e0b, uint32_t e1b, bool wspill, uint32_t lane,
                                                const unsigned long long* __restrict__ tadj, uint32_t (*QU)[kTinyQ],
                                                uint32_t* JQ, unsigned long long* JR, unsigned long long* meet) {
  uint32_t ovf = 0;
  uint32_t e0 = e0b + K.ex[0], e1 = e1b + K.ex[1];
  // (!kSpec: the claimed vertices' first edges were fetched by round_fetch,
  // right after the claims, so their latency overlaps the counting)
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b >= nb) continue;
    const bool s1 = W.s1[b], nw = W.nw[b];
    const uint32_t v = tw_v(W.rec[b]);
    const uint32_t deg = W.deg[b];
    const uint32_t q = (s1 ? q1b : q0b) + K.qpre[b];
    const uint32_t e = s1 ? e1 : e0;
    if (s1) e1 += deg;
    else e0 += deg;
    const bool qok = nw && q < kTinyQ;
    const bool rok = qok && e + deg <= (kSpill ? kTRC + kTinySpill : kTRC);
    if (nw && !qok) ovf |= kOvfQueue;
    if (qok && !rok) ovf |= kOvfRec;
    *(qok ? &QU[s1 ? 1 : 0][q] : JQ + lane) = v << kQBits | tw_pq(W.rec[b]);
    unsigned long long* out = R.nb[s1 ? 1 : 0] + e;
    unsigned long long* junk = JR + lane;
    const uint32_t dd = rok ? deg : 0u;
    const unsigned long long tag = (unsigned long long)q << 52;
    if (!kSpill || !wspill) {
      // past the degree (or with nothing to store) a store goes to the lane's junk slot
#pragma unroll
      for (uint32_t j = 0; j < kTinyUnroll; ++j) *(j < dd ? out + j : junk) = W.nbw[b][j] | tag;
      if (__ballot(rok && deg > kTinyUnroll)) {  // rare: a vertex of degree > 4
        const uint32_t base = tw_base(W.rec[b]);
        for (uint32_t j = kTinyUnroll; rok && j < deg; ++j) out[j] = tadj[base + j] | tag;
      }
    } else {  // rare: some of the wave's records go past the LDS buffer (global spill)
      const uint32_t side = s1 ? 1u : 0u;
      unsigned long long* sp = R.spill + (size_t)((((R.cb >> side) & 1u) ^ 1u) * 2 + side) * kTinySpill;
      const uint32_t base = tw_base(W.rec[b]);
      for (uint32_t j = 0; j < dd; ++j) {
        const unsigned long long w = (j < kTinyUnroll ? W.nbw[b][j] : tadj[base + j]) | tag;
        if (e + j < kTRC) out[j] = w;
        else sp[e + j - kTRC] = w;
      }
    }
    const uint32_t bt = v & 31;
    const uint32_t ost = (uint32_t)((W.oth[b] >> bt) & 1ull) | (uint32_t)((W.oth[b] >> (bt + 32)) & 1ull) << 1;
    const bool cand = qok && ost;
    const bool anyc = __ballot(cand) != 0;
    if (anyc) ovf |= kCand;
    if (anyc && cand) {  // a meet: the other side holds v at depth bo, or bo + 1 if it claimed v now
      const uint32_t bo = s1 ? R.dep[0] : R.dep[1];
      const bool oexp = s1 ? R.exp[0] : R.exp[1];
      const uint32_t dov = (oexp && ost == (1u << ((bo + 1) & 1))) ? bo + 1 : bo;
      const uint32_t ds = s1 ? R.dep[1] : R.dep[0];
      atomicMin(meet, (unsigned long long)(ds + 1 + dov) << 32 | (unsigned long long)(s1 ? 1u : 0u) << 31 | q);
    }
  }
  return ovf;
}

template <bool kStamp>
__global__ __launch_bounds__(kTT, 1) void k_tiny_server(launch::TinyArgs P) {
  static_assert(kTinyB == 2, "two items per lane");
  constexpr uint32_t kCapR = (uint32_t)kTT * kTinyB;  // frontier edges one all-wave pass expands
  // A single-side round may take two passes (the queue-count fields are 12
  // bits): a long-path query's last level is often just above one pass, and
  // it usually holds the meet -- run on instead of falling back to the
  // general engine (a host round trip and a launch).
  constexpr uint32_t kMaxRound = 2 * kCapR - 1;
  constexpr uint32_t kCapW = 64u * kSwNB;              // ... one single-wave round
  __shared__ unsigned long long VIS[2][kTW];
  __shared__ uint32_t QU[2][kTinyQ];
  __shared__ unsigned long long R[2][2][kTRC];  // [buffer][side][record]
  __shared__ TinyCtl C;
  __shared__ TinyState S;
  __shared__ uint32_t JQ[64];  // junk slots of the branch-free stores
  __shared__ unsigned long long JR[64];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63;
  const uint32_t wid = uni(tid >> 6);

  // ---- election: one block on the pinned XCD keeps the graph in its L2
  const bool cand = P.pin_xcc < 0 ? blockIdx.x == 0 : xcc_id() == (uint32_t)P.pin_xcc;
  if (!cand) return;
  if (tid == 0) C.won = atomicMax(P.ticket, P.launch_seq) < P.launch_seq;
  __syncthreads();
  if (!uni(C.won)) return;
  if (tid == 0) __hip_atomic_store(&P.box->alive, P.launch_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);


  auto zero_state = [&]() {
    unsigned long long* V = &VIS[0][0];
#pragma unroll 4
    for (uint32_t i = tid; i < 2 * kTW; i += kTT) V[i] = 0ull;
    if (tid < 3) C.cnt[tid] = 0ull;
    if (tid == 0) {
      C.meet = ~0ull;
      C.rovf = 0u;
    }
  };
  zero_state();
  lds_barrier();

  auto make_ctx = [&](uint32_t x0, uint32_t x1, uint32_t cb0, uint32_t cb1, uint32_t d0, uint32_t d1) {
    RoundCtx X;
    X.x0 = x0;
    X.tot = x0 + x1;
    X.rb0 = &R[cb0][0][0];
    X.rb1x = &R[cb1][1][0] - x0;
    X.nb[0] = &R[cb0 ^ 1][0][0];
    X.nb[1] = &R[cb1 ^ 1][1][0];
    X.spill = P.spill;
    X.cb = cb0 | cb1 << 1;
    X.par[0] = (d0 + 1) & 1;
    X.par[1] = (d1 + 1) & 1;
    X.dep[0] = d0;
    X.dep[1] = d1;
    X.exp[0] = x0 != 0;
    X.exp[1] = x1 != 0;
    X.spilled = x0 > kTRC || x1 > kTRC;
    return X;
  };

  uint32_t last_seq = P.last_seq;
  for (;;) {
    unsigned long long rt0 = 0;
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long sw[6] = {0, 0, 0, 0, 0, 0};  // stamp build: single-wave rounds, issue, count, place, meet read, edges
    uint32_t seq = 0;
    // ======== wave 0 alone: poll, seed, and the rounds small enough for one
    // wave -- no barrier, the round state in SGPRs, the counters from the
    // wave's own ballots and scan.  The other waves sleep in the barrier below.
    if (wid == 0) {
      // wait for a request: one 16-byte system-scope load of the pinned
      // mailbox per poll (relaxed: the XCD's L2 -- the graph -- is never
      // invalidated).  A CPU-written VRAM slot was measured instead and not
      // kept (no faster; benchmarks/micro/mailbox_rtt.hip)
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t stop = 0;
      u32x4 rq;
      for (;;) {
        u32x4 r4;
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r4) : "v"(P.req) : "memory");
        rq.x = uni(r4.x), rq.y = uni(r4.y), rq.z = uni(r4.z), rq.w = uni(r4.w);
        rt0 = __builtin_amdgcn_s_memrealtime();
        const bool whole = (rq.w >> 8) == (rq.x & 0xffffffu);  // not torn
        if (whole && rq.x != last_seq) {
          stop = rq.w & kReqStop;
          break;
        }
        if (rt0 - t0 > P.idle_ticks) {
          stop = 1;
          break;
        }
      }
      seq = rq.x;
      if (lane == 0) {
        C.cmd[0] = stop;
        C.cmd[1] = seq;
      }
      if (!stop) {
        if (kStamp) st[0] = stamp();
        // the host checked src/dst < n and src != dst; clamp anyway (a torn request never faults)
        const uint32_t src = min(rq.y, P.n - 1), dst = min(rq.z, P.n - 1);
        // ---- seed: both roots at depth 0; their records are their
        // neighbours' words (parent queue index 0 = the root)
        const unsigned long long fs = P.tinfo[src], fd = P.tinfo[dst];
        TinyState T{};
        T.E0 = tw_deg(fs);
        T.E1 = tw_deg(fd);
        T.ql0 = T.ql1 = 1;
        T.meet = ~0ull;
        {
          const uint32_t b0 = tw_base(fs), b1 = tw_base(fd);
          for (uint32_t j = lane; j < T.E0; j += 64) R[0][0][j] = P.tadj[b0 + j];
          for (uint32_t j = lane; j < T.E1; j += 64) R[0][1][j] = P.tadj[b1 + j];
          if (lane == 0) {
            QU[0][0] = src << kQBits;
            QU[1][0] = dst << kQBits;
            VIS[0][src >> 5] = 1ull << (src & 31);
            VIS[1][dst >> 5] = 1ull << (dst & 31);
          }
        }
        if (T.E0 == 0 || T.E1 == 0) T.status = kTinyNoPath;  // an isolated endpoint
        if (kStamp) st[1] = stamp();
        // ---- single-wave rounds: both frontiers together up to 128 edges.
        // Compiled twice: one item per lane for rounds of at most 64 edges
        // (the first rounds of a query), two otherwise -- the one-item body
        // carries none of the second item's selects, ballots and stores.
        // (Every exit sets T.status, which ends the loop.)
        auto sw_round = [&](auto nbc) {
          constexpr int NB = decltype(nbc)::value;
          const uint32_t x0 = T.E0, x1 = T.E1;
          const RoundCtx X = make_ctx(x0, x1, T.cb0, T.cb1, T.d0, T.d1);
          Work<NB> W;
          unsigned long long t_ = kStamp ? stamp() : 0;
          auto mark = [&](int k) {
            if (kStamp) {
              const unsigned long long u_ = stamp();
              sw[k] += u_ - t_;
              t_ = u_;
            }
          };
          round_issue<NB, true, false>(W, X, lane, 64, NB, P.tadj, VIS);
          mark(1);
          Counts<NB> K;
          round_count<NB>(K, W);
          mark(2);
          const uint32_t ovf =
              round_place<NB, true, false>(W, K, X, NB, T.ql0, T.ql1, 0u, 0u, false, lane, P.tadj, QU, JQ, JR, &C.meet);
          const bool qovf = __ballot(ovf & kOvfQueue) != 0, rovf = __ballot(ovf & kOvfRec) != 0;
          mark(3);
          if (kStamp) {
            ++sw[0];
            sw[5] += x0 + x1;
          }
          T.x0 = x0;
          T.x1 = x1;
          T.einsp += x0 + x1;
          T.levels += 2;
          T.ql0 += K.qt[0];
          T.ql1 += K.qt[1];
          if (qovf) {
            T.status = kTinyOverflow;
            return;
          }
          // the wave's own ds_min_u64 precede this read (one wave's LDS ops are
          // in order); read only when this round stored a candidate (C.meet is
          // otherwise still ~0: a meet ends the search in the round that finds it)
          const unsigned long long m =
              (uni(ovf) & kCand) ? uni64(__hip_atomic_load(&C.meet, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
                                 : ~0ull;
          mark(4);
          if (m != ~0ull) {
            T.meet = m;
            T.status = kTinyFound;
            return;
          }
          if (rovf) {  // the next round's records do not fit
            T.status = kTinyOverflow;
            return;
          }
          T.E0 = K.et[0];
          T.E1 = K.et[1];
          T.cb0 ^= 1;
          T.cb1 ^= 1;
          ++T.d0;
          ++T.d1;
          if (!T.E0 || !T.E1) T.status = kTinyNoPath;  // a side claimed nothing: its component is exhausted
        };
        while (T.status == 0 && T.E0 + T.E1 <= kCapW) {
          if (kSwSplit && T.E0 + T.E1 <= 64) sw_round(std::integral_constant<int, 1>{});
          else if (kSwNB == 2 || T.E0 + T.E1 <= 128) sw_round(std::integral_constant<int, 2>{});
          else sw_round(std::integral_constant<int, kSwNB>{});
        }
        if (lane == 0) S = T;
      }
    }
    lds_barrier();
    if (uni(C.cmd[0])) break;
    seq = uni(C.cmd[1]);
    last_seq = seq;
    if (kStamp) st[2] = stamp();

    // ======== all-wave rounds (uniform state, identical in every wave)
    uint32_t status = uni(S.status), E0 = uni(S.E0), E1 = uni(S.E1), cb0 = uni(S.cb0), cb1 = uni(S.cb1);
    uint32_t d0 = uni(S.d0), d1 = uni(S.d1), ql0 = uni(S.ql0), ql1 = uni(S.ql1), levels = uni(S.levels);
    uint32_t x0 = uni(S.x0), x1 = uni(S.x1), slot = 0;
    unsigned long long einsp = uni64(S.einsp), meet = uni64(S.meet);
    // stamp build: wave 0's cycles per round phase (s_memtime, waits at each mark)
    unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0}, tp = kStamp ? stamp() : 0;
    uint32_t rnd = 0;
#define TINY_PH(k)                         \
  if (kStamp && wid == 0) {                \
    const unsigned long long t_ = stamp(); \
    ph[k] += t_ - tp;                      \
    tp = t_;                               \
  }
    while (status == 0) {
      x0 = E0;
      x1 = E1;
      if (x0 + x1 > kCapR || x0 + x1 > kLockMax) {  // the side with fewer edges alone
        if (x0 <= x1) x1 = 0;
        else x0 = 0;
        if (x0 + x1 > kMaxRound) {
          status = kTinyOverflow;
          break;
        }
      }
      // the counter slot of the NEXT round was last read two barriers ago; the
      // last wave (idle in small rounds) clears it
      if (tid == kTT - 64) C.cnt[slot == 2 ? 0 : slot + 1] = 0ull;
      const RoundCtx X = make_ctx(x0, x1, cb0, cb1, d0, d1);
      TINY_PH(0)
      // one item per lane when the round has at most kTT edges (every round
      // under the lockstep cap), two otherwise: as in the single-wave phase
      // the one-item body carries none of the second item's instructions
      bool wsp = false;  // (uniform) this wave stored spilled records this round
      // c0: first item of this pass (a two-pass round: 0, then kCapR)
      auto aw_round = [&](auto nbc, uint32_t c0) {
        constexpr int NB = decltype(nbc)::value;
        const int nb = (NB == 2 && c0 + wid * 64 + kTT < X.tot) ? 2 : 1;  // uniform
        Work<NB> W;
        round_issue<NB, kSpecAll, kSpillOn>(W, X, c0 + tid, kTT, nb, P.tadj, VIS);
        if (!kSpecAll) round_fetch<NB>(W, nb, P.tadj);
        Counts<NB> K;
        round_count<NB>(K, W);
        TINY_PH(3)
        if (K.qt[0] | K.qt[1]) {  // uniform
          // ONE ds_add_rtn_u64 on the packed round counter (TinyCtl layout).
          // A wave's record count is clamped to kTRC + kTinySpill + 1: past
          // that its lanes overflow anyway (kOvfRec), and the clamp keeps 32
          // wave passes below 2^20, so a field never carries into the next.
          unsigned long long base = 0;
          if (lane == 0)
            base = atomicAdd(&C.cnt[slot], (unsigned long long)min(K.et[0], kTRC + kTinySpill + 1) |
                                               (unsigned long long)min(K.et[1], kTRC + kTinySpill + 1) << 20 |
                                               (unsigned long long)K.qt[0] << 40 | (unsigned long long)K.qt[1] << 52);
          const uint32_t blo = lane0((uint32_t)base), bhi = lane0((uint32_t)(base >> 32));
          TINY_PH(4)
          const uint32_t e0b = blo & 0xFFFFFu, e1b = ((blo >> 20) | (bhi << 12)) & 0xFFFFFu;
          // (uniform) does any of this wave's records land past the LDS buffer?
          const bool wspill = e0b + K.et[0] > kTRC || e1b + K.et[1] > kTRC;
          wsp = wsp || wspill;
          const uint32_t ovf = round_place<NB, kSpecAll, kSpillOn>(W, K, X, nb, ql0 + ((bhi >> 8) & 0xFFFu),
                                                                   ql1 + (bhi >> 20), e0b, e1b, wspill, lane, P.tadj,
                                                                   QU, JQ, JR, &C.meet);
          // a full queue: fatal in a lockstep round (a dropped candidate may be
          // the shorter one -- key 0 = overflow, a meet has length >= 1); in a
          // single-side round every candidate has the same length, so like a
          // record overflow it is fatal only if the round finds no meet
          if (ovf & kOvfQueue) {
            if (X.x0 != 0 && X.x0 != X.tot) atomicMin(&C.meet, 0ull);
            else C.rovf = 1u;
          }
          if (ovf & kOvfRec) C.rovf = 1u;
        }
      };
      for (uint32_t c0 = 0; c0 < X.tot; c0 += kCapR) {  // one pass, two for a big single-side round
        if (c0 + wid * 64 < X.tot) {
          if (kAwSplit && X.tot - c0 <= (uint32_t)kTT) aw_round(std::integral_constant<int, 1>{}, c0);
          else aw_round(std::integral_constant<int, 2>{}, c0);
        }
      }
      TINY_PH(5)
      // LDS barrier; a wave that spilled records (global stores, rare) drains
      // them first for the next round's readers -- the others leave their
      // unused speculative loads in flight
      if (kSpillOn && wsp) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lds_barrier();
      TINY_PH(6)
      einsp += X.tot;
      levels += (x0 != 0) + (x1 != 0);
      const unsigned long long cnt = uni64(C.cnt[slot]);
      meet = uni64(C.meet);
      slot = slot == 2 ? 0 : slot + 1;
      if (x0) ql0 += (uint32_t)(cnt >> 40) & 0xFFFu;
      if (x1) ql1 += (uint32_t)(cnt >> 52);
      if (meet != ~0ull) {
        status = meet == 0 ? kTinyOverflow : kTinyFound;
        break;
      }
      if (uni(C.rovf)) {  // no meet, and the next round's records do not fit
        status = kTinyOverflow;
        break;
      }
      if (x0) {
        E0 = (uint32_t)cnt & 0xFFFFFu;
        cb0 ^= 1;
        ++d0;
        if (!E0) status = kTinyNoPath;  // side 0 claimed nothing: its component is exhausted
      }
      if (x1) {
        E1 = (uint32_t)(cnt >> 20) & 0xFFFFFu;
        cb1 ^= 1;
        ++d1;
        if (!E1) status = kTinyNoPath;
      }
      ++rnd;
      TINY_PH(7)
    }
#undef TINY_PH
    if (kStamp) st[3] = stamp();

    // ---- the path: find the meet vertex on the other side, walk both chains
    uint32_t len = 0, mv = ~0u;
    const uint32_t visited = ql0 + ql1;
    uint32_t* PATH = reinterpret_cast<uint32_t*>(&R[0][0][0]);
    if (status == kTinyFound) {
      len = (uint32_t)(meet >> 32);
      const uint32_t s = (uint32_t)(meet >> 31) & 1u, qs = (uint32_t)meet & 0x7fffffffu;
      mv = QU[s][qs] >> kQBits;
      const uint32_t o = s ^ 1, nqo = o ? ql1 : ql0;
      for (uint32_t i = tid; i < nqo; i += kTT)
        if ((QU[o][i] >> kQBits) == mv) C.other_q = i;
      lds_barrier();
      if (kStamp) st[4] = stamp();
      if (wid == 0 && lane < 2) {
        const uint32_t qo = C.other_q;
        const uint32_t dsv = (s ? d1 : d0) + 1;    // depth of the meet vertex on the claiming side
        const uint32_t d0v = s ? len - dsv : dsv;  // its distance from src = its path position
        const uint32_t side = lane;
        uint32_t idx = side == s ? qs : qo;
        const uint32_t hops = side ? len - d0v : d0v;
        uint32_t pos = d0v;
        for (uint32_t t = 0; t <= hops; ++t) {
          const uint32_t e = QU[side][idx];
          PATH[pos] = e >> kQBits;
          idx = e & (kTinyQ - 1);
          pos = side ? pos + 1 : pos - 1;
        }
      }
    }
    // ---- publish: self-tagged packets, one 16-byte store each
    if (wid == 0) {
      if (kStamp) st[5] = stamp();
      const unsigned long long rt1 = __builtin_amdgcn_s_memrealtime();
      const uint32_t plen = status == kTinyFound ? len + 1 : 0u;
      const uint32_t npk = 2 + (plen + 2) / 3;
      for (uint32_t j = lane; j < npk; j += 64) {
        u32x4 pk;
        pk.x = seq;
        if (j == 0) {
          pk.y = status | levels << 8;
          pk.z = status == kTinyFound ? len : ~0u;
          pk.w = mv;
        } else if (j == 1) {
          pk.y = (uint32_t)(rt1 - rt0);
          pk.z = (uint32_t)min(einsp, 0xffffffffull);
          pk.w = visited;
        } else {
          const uint32_t t = 3 * (j - 2);
          pk.y = PATH[t];
          pk.z = t + 1 < plen ? PATH[t + 1] : 0u;
          pk.w = t + 2 < plen ? PATH[t + 2] : 0u;
        }
        store_sys16(P.pkts + j, pk);
      }
      if (kStamp && lane == 0) {
        st[6] = stamp();
        st[7] = rnd;
        for (int k = 0; k < 8; ++k) P.stamps[k] = st[k];
        for (int k = 0; k < 8; ++k) P.stamps[8 + k] = ph[k];
        for (int k = 0; k < 6; ++k) P.stamps[16 + k] = sw[k];
      }
    }
    zero_state();
    lds_barrier();
  }
  if (tid == 0) {
    __threadfence_system();
    __hip_atomic_store(&P.box->alive, ~P.launch_seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // exited
  }
}

__global__ void k_tiny_adj(const uint64_t* __restrict__ row_off, const uint32_t* __restrict__ col, uint32_t n,
                           uint64_t nnz, unsigned long long* __restrict__ tadj, unsigned long long* __restrict__ tinfo) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t k = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; k < nnz; k += stride) {
    const uint32_t v = col[k];
    const uint64_t b = row_off[v];
    tadj[k] = tiny_pack(v, b, row_off[v + 1] - b);
  }
  for (uint64_t v = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; v < n; v += stride) {
    const uint64_t b = row_off[v];
    tinfo[v] = tiny_pack((uint32_t)v, b, row_off[v + 1] - b);
  }
}

}  // namespace

namespace launch {

bool tiny_supported(uint32_t n, uint64_t nnz, uint64_t max_deg) {
  return n >= 2 && n <= kTinyMaxN && nnz < kTinyMaxNnz && max_deg <= kTinyMaxDeg;
}

void build_tiny_adj(const uint64_t* row_off, const uint32_t* col, uint32_t n, uint64_t nnz,
                    unsigned long long* tadj, unsigned long long* tinfo, hipStream_t s) {
  const uint64_t work = nnz > n ? nnz : n;
  const unsigned blocks = (unsigned)((work + 255) / 256 < 4096 ? (work + 255) / 256 : 4096);
  k_tiny_adj<<<blocks ? blocks : 1, 256, 0, s>>>(row_off, col, n, nnz, tadj, tinfo);
  HIP_CHECK(hipGetLastError());
}

void tiny_server(const TinyArgs& a, bool stamp, hipStream_t s) {
  BIBFS_REQUIRE(a.n >= 2 && a.n <= kTinyMaxN, "tiny server: graph too large");
  const unsigned blocks = a.pin_xcc >= 0 ? 16 : 1;  // 2 per XCD under round-robin dispatch; one is elected
  if (stamp) k_tiny_server<true><<<blocks, kTT, 0, s>>>(a);
  else k_tiny_server<false><<<blocks, kTT, 0, s>>>(a);
  HIP_CHECK(hipGetLastError());
}

}  // namespace launch
}  // namespace bibfs
