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
// Queries that do not fit (a round above 2048 frontier edges, a queue above
// kTinyQ) answer kTinyOverflow and the host re-runs them on the general
// engine (engine_kernels.hip), which has the grid hand-off.
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "device.hpp"

namespace bibfs {
namespace {

using namespace dev;

#ifndef BIBFS_TINY_THREADS
#define BIBFS_TINY_THREADS 1024
#endif
constexpr int kTT = BIBFS_TINY_THREADS;
constexpr uint32_t kTW = kTinyMaxN / 32;  // u64 visited words per side (low half even, high half odd)
constexpr uint32_t kTRC = 2040;           // per-edge records per side per buffer
constexpr uint32_t kQBits = 12;
constexpr uint32_t kTinyUnroll = 4;  // record stores per new vertex without a loop
static_assert(kTinyQ == 1u << kQBits, "queue index width");

// Per-round counter (three slots, rotated): new records of side 0 [19:0] and
// side 1 [39:20], new queue entries of side 0 [51:40] and side 1 [63:52].
// Field bounds: a round has at most kCapR = 2048 new vertices per side
// (< 2^12 with the queue capped at kTinyQ = 4096 -- a larger sum is an overflow
// anyway) and 2048 x kTinyMaxDeg < 2^20 new records.
struct TinyCtl {
  unsigned long long cnt[3];
  unsigned long long meet;   // min over candidates of len << 32 | side << 31 | queue index; 0 = overflow
  uint32_t other_q;          // the meet vertex's queue index on the other side
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

// One lane's share of a round: its NB frontier edges (items i0 + b * stride),
// loaded, claimed and checked against the other side.
template <int NB>
struct LaneWork {
  unsigned long long rec[NB], fat[NB], oth[NB];
  bool act[NB], s1[NB], nw[NB];
  uint32_t deg[NB], qpre[NB];
  uint32_t ep;        // degrees of the new vertices, side 0 | side 1 << 16
  uint32_t qt0, qt1;  // the wave's new vertices per side (uniform)
};

template <int NB>
__device__ __forceinline__ void expand_claim(LaneWork<NB>& W, int nb, uint32_t i0, uint32_t stride, uint32_t x0,
                                             uint32_t tot, uint32_t par0, uint32_t par1,
                                             const unsigned long long* rb0, const unsigned long long* rb1,
                                             const unsigned long long* __restrict__ tadj,
                                             unsigned long long (*VIS)[kTW]) {
  unsigned long long old[NB];
  // Branch-free: an idle lane reads record 0, loads word 0 and claims with an
  // empty mask, so each step is ONE wave instruction per batch and the loads /
  // claims of all batches stay in flight together.
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint32_t i = i0 + (uint32_t)b * stride;
    W.act[b] = i < tot;
    W.s1[b] = i >= x0;
    W.rec[b] = W.fat[b] = W.oth[b] = old[b] = 0ull;
    if (b < nb) W.rec[b] = *((W.s1[b] ? rb1 : rb0) + (W.act[b] ? i : 0u));
  }
#pragma unroll
  for (int b = 0; b < NB; ++b)
    if (b < nb) W.fat[b] = tadj[W.act[b] ? (uint32_t)W.rec[b] : 0u];
  // claim, then read the other side's word: the LDS executes one wave's DS
  // instructions in order, so of two same-round claims of a vertex by the two
  // sides at least one sees the other
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (b < nb) {
      const uint32_t v = (uint32_t)(W.fat[b] >> 47);
      const uint32_t sh = (v & 31) + ((W.s1[b] ? par1 : par0) << 5);
      const unsigned long long m = W.act[b] ? 1ull << sh : 0ull;
      unsigned long long* w = &VIS[W.s1[b] ? 1 : 0][v >> 5];
      old[b] = __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      W.oth[b] = __hip_atomic_load(W.s1[b] ? w - kTW : w + kTW, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  }
  // new vertices: queue slots from ballots (no scan)
  W.ep = 0;
  W.qt0 = W.qt1 = 0;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    const uint32_t bt = (uint32_t)(W.fat[b] >> 47) & 31;
    W.nw[b] = W.act[b] && ((old[b] >> bt) & 0x100000001ull) == 0;
    W.deg[b] = W.nw[b] ? (uint32_t)(W.fat[b] & 0xFFFFFu) : 0u;
    W.ep += W.s1[b] ? W.deg[b] << 16 : W.deg[b];
    const unsigned long long m0 = __ballot(W.nw[b] && !W.s1[b]), m1 = __ballot(W.nw[b] && W.s1[b]);
    W.qpre[b] = W.s1[b] ? W.qt1 + mbcnt64(m1) : W.qt0 + mbcnt64(m0);
    W.qt0 += (uint32_t)__popcll(m0);
    W.qt1 += (uint32_t)__popcll(m1);
  }
}

// Queue entries and next-round records of the lane's new vertices; meet
// candidates go to C.meet.  q0b/q1b: queue index of the wave's first new
// vertex per side; e0p/e1p: the lane's first record slot per side.  Returns
// true when a queue or record buffer would overflow.
template <int NB>
__device__ __forceinline__ bool place(const LaneWork<NB>& W, uint32_t q0b, uint32_t q1b, uint32_t e0p, uint32_t e1p,
                                      uint32_t cb0, uint32_t cb1, uint32_t d0, uint32_t d1, uint32_t x0, uint32_t x1,
                                      uint32_t (*QU)[kTinyQ], unsigned long long (*R)[2][kTRC],
                                      unsigned long long* meet) {
  bool ovf = false;
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    if (!W.nw[b]) continue;
    const bool s1 = W.s1[b];
    const uint32_t v = (uint32_t)(W.fat[b] >> 47);
    const uint32_t base_v = (uint32_t)((W.fat[b] >> 20) & 0x7FFFFFFu);
    const uint32_t deg = W.deg[b];
    const uint32_t q = (s1 ? q1b : q0b) + W.qpre[b];
    const uint32_t e = s1 ? e1p : e0p;
    if (s1) e1p += deg;
    else e0p += deg;
    if (q >= kTinyQ || e + deg > kTRC) {
      ovf = true;
      continue;
    }
    QU[s1 ? 1 : 0][q] = v << kQBits | (uint32_t)(W.rec[b] >> 32);
    unsigned long long* out = &R[(s1 ? cb1 : cb0) ^ 1][s1 ? 1 : 0][e];
    const unsigned long long hi = (unsigned long long)q << 32;
    // the first kTinyUnroll records straight-line: past the degree a store
    // rewrites the last record with its own value (deg >= 1: the edge back to
    // the parent) instead of branching
#pragma unroll
    for (uint32_t j = 0; j < kTinyUnroll; ++j) {
      const uint32_t jj = min(j, deg - 1);
      out[jj] = hi | (base_v + jj);
    }
    for (uint32_t j = kTinyUnroll; j < deg; ++j) out[j] = hi | (base_v + j);
    const uint32_t bt = v & 31;
    const uint32_t ost = (uint32_t)((W.oth[b] >> bt) & 1ull) | (uint32_t)((W.oth[b] >> (bt + 32)) & 1ull) << 1;
    if (ost) {  // a meet: the other side holds v at depth bo, or bo + 1 if it claimed v this round
      const uint32_t bo = s1 ? d0 : d1;
      const bool oexp = (s1 ? x0 : x1) != 0;
      const uint32_t dov = (oexp && ost == (1u << ((bo + 1) & 1))) ? bo + 1 : bo;
      const uint32_t len = (s1 ? d1 : d0) + 1 + dov;
      atomicMin(meet, (unsigned long long)len << 32 | (unsigned long long)(s1 ? 1u : 0u) << 31 | q);
    }
  }
  return ovf;
}

template <bool kStamp>
__global__ __launch_bounds__(kTT, 1) void k_tiny_server(launch::TinyArgs P) {
  constexpr int B = kTinyB;
  constexpr uint32_t kCapR = (uint32_t)kTT * B;  // frontier edges one all-wave round expands
  constexpr int SB = 2;                          // batches per lane in the single-wave rounds
  constexpr uint32_t kCapW = 64u * SB;           // frontier edges one single-wave round expands
  __shared__ unsigned long long VIS[2][kTW];
  __shared__ uint32_t QU[2][kTinyQ];
  __shared__ unsigned long long R[2][2][kTRC];  // [buffer][side][record]: parent queue index << 32 | CSR index
  __shared__ TinyCtl C;
  __shared__ TinyState S;
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
    if (tid == 0) C.meet = ~0ull;
  };
  zero_state();
  lds_barrier();

  uint32_t last_seq = P.last_seq;
  for (;;) {
    unsigned long long rt0 = 0;
    unsigned long long st[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t seq = 0;
    // ======== wave 0 alone: poll, seed, and the rounds small enough for one
    // wave -- no barrier, the round state in SGPRs, the counters from the
    // wave's own scan.  The other waves sleep in the barrier below.
    if (wid == 0) {
      // wait for a request: one 16-byte system-scope load of the pinned
      // mailbox per poll (relaxed: the XCD's L2 -- the graph -- is never
      // invalidated)
      const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
      uint32_t stop = 0;
      u32x4 rq;
      for (;;) {
        u32x4 r4;
        asm volatile("global_load_dwordx4 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(r4) : "v"(P.box) : "memory");
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
        // ---- seed: both roots at depth 0, their edges as the first records
        const unsigned long long fs = P.tinfo[src], fd = P.tinfo[dst];
        TinyState T{};
        T.E0 = (uint32_t)(fs & 0xFFFFFu);
        T.E1 = (uint32_t)(fd & 0xFFFFFu);
        T.ql0 = T.ql1 = 1;
        T.meet = ~0ull;
        {
          const uint32_t b0 = (uint32_t)((fs >> 20) & 0x7FFFFFFu), b1 = (uint32_t)((fd >> 20) & 0x7FFFFFFu);
          for (uint32_t j = lane; j < min(T.E0, kTRC); j += 64) R[0][0][j] = b0 + j;
          for (uint32_t j = lane; j < min(T.E1, kTRC); j += 64) R[0][1][j] = b1 + j;
          if (lane == 0) {
            QU[0][0] = src << kQBits;
            QU[1][0] = dst << kQBits;
            VIS[0][src >> 5] = 1ull << (src & 31);
            VIS[1][dst >> 5] = 1ull << (dst & 31);
          }
        }
        if (T.E0 == 0 || T.E1 == 0) T.status = kTinyNoPath;  // an isolated endpoint
        else if (T.E0 > kTRC || T.E1 > kTRC) T.status = kTinyOverflow;
        if (kStamp) st[1] = stamp();
        // ---- single-wave rounds
        while (T.status == 0 && T.E0 + T.E1 <= kCapW) {
          const uint32_t x0 = T.E0, x1 = T.E1, tot = x0 + x1;
          const int nb = tot > 64 ? SB : 1;
          LaneWork<SB> W;
          expand_claim<SB>(W, nb, lane, 64, x0, tot, (T.d0 + 1) & 1, (T.d1 + 1) & 1, &R[T.cb0][0][0],
                           &R[T.cb1][1][0] - x0, P.tadj, VIS);
          const uint32_t ei = wave_scan(W.ep);
          const uint32_t et = lane63(ei);
          const uint32_t ex = ei - W.ep;
          const bool ovf = place<SB>(W, T.ql0, T.ql1, ex & 0xffffu, ex >> 16, T.cb0, T.cb1, T.d0, T.d1, x0, x1, QU,
                                     R, &C.meet);
          const bool ovf_any = __ballot(ovf) != 0;
          T.x0 = x0;
          T.x1 = x1;
          T.einsp += tot;
          T.levels += (x0 != 0) + (x1 != 0);
          if (ovf_any) {
            T.status = kTinyOverflow;
            break;
          }
          if (x0) T.ql0 += W.qt0;
          if (x1) T.ql1 += W.qt1;
          // the wave's own ds_min_u64 precede this read (one wave's LDS ops are in order)
          const unsigned long long m = uni64(__hip_atomic_load(&C.meet, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
          if (m != ~0ull) {
            T.meet = m;
            T.status = kTinyFound;
            break;
          }
          if (x0) {
            T.E0 = et & 0xffffu;
            T.cb0 ^= 1;
            ++T.d0;
            if (!T.E0) T.status = kTinyNoPath;  // side 0 claimed nothing: its component is exhausted
          }
          if (x1) {
            T.E1 = et >> 16;
            T.cb1 ^= 1;
            ++T.d1;
            if (!T.E1) T.status = kTinyNoPath;
          }
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
      if (x0 + x1 > kCapR) {  // both do not fit one round: the side with fewer edges alone
        if (x0 <= x1) x1 = 0;
        else x0 = 0;
        if (x0 + x1 > kCapR) {
          status = kTinyOverflow;
          break;
        }
      }
      // the counter slot of the NEXT round was last read two barriers ago; the
      // last wave (idle in small rounds) clears it
      if (tid == kTT - 64) C.cnt[slot == 2 ? 0 : slot + 1] = 0ull;
      const uint32_t tot = x0 + x1;
      TINY_PH(0)
      if (wid * 64 < tot) {
        // batches this wave holds at all (uniform): batch b covers lanes tid + b * kTT
        const int nb = (wid * 64 + kTT < tot) ? B : 1;
        LaneWork<B> W;
        expand_claim<B>(W, nb, tid, kTT, x0, tot, (d0 + 1) & 1, (d1 + 1) & 1, &R[cb0][0][0], &R[cb1][1][0] - x0,
                        P.tadj, VIS);
        TINY_PH(3)
        if (W.qt0 | W.qt1) {  // uniform
          // record slots from one DPP scan of the degrees (both sides as 16-bit
          // halves), both counters in ONE ds_add_rtn_u64 (TinyCtl field layout)
          const uint32_t ei = wave_scan(W.ep);
          const uint32_t et = lane63(ei);
          unsigned long long base = 0;
          if (lane == 0)
            base = atomicAdd(&C.cnt[slot], (unsigned long long)(et & 0xffffu) | (unsigned long long)(et >> 16) << 20 |
                                               (unsigned long long)W.qt0 << 40 | (unsigned long long)W.qt1 << 52);
          const uint32_t blo = lane0((uint32_t)base), bhi = lane0((uint32_t)(base >> 32));
          TINY_PH(4)
          const uint32_t ex = ei - W.ep;  // exclusive, per 16-bit half
          const bool ovf = place<B>(W, ql0 + ((bhi >> 8) & 0xFFFu), ql1 + (bhi >> 20), (blo & 0xFFFFFu) + (ex & 0xffffu),
                                    ((blo >> 20) | (bhi << 12)) + (ex >> 16), cb0, cb1, d0, d1, x0, x1, QU, R, &C.meet);
          if (ovf) atomicMin(&C.meet, 0ull);  // key 0 = overflow (a meet has length >= 1)
        }
      }
      TINY_PH(5)
      lds_barrier();
      TINY_PH(6)
      einsp += tot;
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
