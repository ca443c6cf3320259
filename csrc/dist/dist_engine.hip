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
//   pre      top-down: expand the owned frontier, claim owned neighbours, emit
//            (v, parent) candidates for remote owners (each remote vertex at
//            most once per search and side); bottom-up: the owned slice of
//            the frontier bitmap
//   exchange ONE allgather: candidate blocks or bitmap slices
//   post     owners claim the candidates addressed to them, or scan their
//            unvisited vertices against the gathered bitmap
// and every round ends with a meet check over the vertices claimed in it
// (exact lengths from per-vertex depths, so the minimum over a lockstep round
// is the distance) and ONE grouped allreduce {claimed counts, degree sums
// (sum); meet key (min)}.
//
// Where the reference (and this engine's first version) went back to the host
// after every level (v4/mpi_bas.cpp:85,107,124: three blocking collectives and
// host scans per level), the round POLICY now lives on the device: `Ctl` is
// recomputed at the start of each round from the previous round's reduced
// values -- the same bytes on every rank, so every rank plans the same round
// -- and the host enqueues `spec_rounds` sparse rounds back to back, each
// with a fixed-capacity candidate exchange:
//   k_spec_expand (plan + both sides' pre) -> allgather -> k_spec_claim (both
//   sides' post) -> k_meet_end (meet + round end) -> grouped allreduce
// A round whose plan says "done", "no path" or "stalled" runs as no-ops; the
// host reads `Ctl` once per batch.  A round the speculative shape cannot
// carry (bottom-up, or a frontier with more edges than the enqueued block
// capacity, so a rank could overflow it) stalls the batch, and the host plans
// that one round itself with exact sizing (and, in lockstep, the comm-stream
// overlap of one side's exchange with the other side's expand).
// In a host-planned lockstep round side S's exchange + post run on the comm
// stream while side T's pre runs on the compute stream.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <csignal>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "bibfs/dist_engine.hpp"
#include "bibfs/hip_engine.hpp"
#include "bibfs/io.hpp"
#include "bibfs/trace.hpp"
#include "comm.hpp"
#include "device.hpp"
#include "devmem.hpp"

namespace bibfs {

using namespace dev;
using dist::DType;
using dist::ROp;

namespace {

constexpr int kThreads = 256;
constexpr unsigned long long kNoKey = ~0ull;
constexpr uint64_t kCapMax = 1u << 20;          // host-planned round: candidate pairs per rank per level
constexpr uint64_t kLockstepEdges = 1u << 16;   // both frontiers at most this many edges: always lockstep
// Balanced frontiers (within 2x) go lockstep only up to this size: beyond it a
// lockstep round doubles the work of the meeting level (Kronecker hub levels,
// 10^7 edges a side), while a single-side level does the smaller half and
// stops at its first meet (every meet of a single-side level has one length).
constexpr uint64_t kLockstepMaxEdges = 1u << 20;
constexpr uint32_t kSpecCapMin = 1024;          // smallest speculative candidate block (pairs)
// A frontier vertex with more edges than this is not expanded by the block
// that holds it: it is deferred to a hub list whose edges the whole grid then
// walks edge-parallel (a degree-10^6 hub would otherwise serialise on one CU).
constexpr uint64_t kHubDeg = 512;
// 1 = a frontier of at most one 256-vertex chunk is expanded by every block of
// the launch, each walking a stride of its edges (td_expand_side)
#ifndef BIBFS_DIST_SPREAD
#define BIBFS_DIST_SPREAD 1
#endif
constexpr bool kDistSpread = BIBFS_DIST_SPREAD;
// Levels with more frontier edges than this read the visited word before the
// claim's atomicOr (ClaimMeet::precheck).
constexpr uint64_t kPrecheckEdges = 1u << 16;
constexpr uint64_t kNoHubs = ~0ull;
constexpr int kHubTile = 1024;                  // hubs staged in LDS per pass
constexpr uint32_t kSpecHubCap = 4096;          // speculative blocks up to this size skip the hub pass
constexpr uint32_t kTraceCap = 4096;            // rounds recorded with SearchOptions::trace
constexpr uint32_t kPlanRing = 64;              // pinned per-round plan words (lookahead < this)
constexpr int kStageRanks = 16;                 // gathered reductions staged in LDS up to this many ranks
constexpr uint32_t kOwnerCapMin = 256;          // smallest owner-addressed candidate block (pairs)
// Small rounds at P > 1 (one workgroup per rank, see small_expand):
constexpr uint32_t kSmallE = 1024;              // frontier edges per side (any rank)
constexpr uint32_t kSmallV = 512;               // frontier vertices per side (all ranks) staged in LDS
constexpr uint32_t kSmallClaim = 2048;          // candidates (all senders, both sides) one block claims
constexpr int kSmallU = 4;                      // items per thread in flight per pass

// Search control state: identical on every rank (computed from reduced
// values only).  Double-buffered by round parity: round `it` reads
// ctl[(it-1)&1] and writes ctl[it&1].
enum : uint32_t { kRun = 0, kDone = 1, kDead = 2, kStall = 3 };
enum : uint32_t { kStallNone = 0, kStallDense = 1, kStallCap = 2, kStallHost = 3, kStallPipe = 4 };
constexpr uint32_t kSeedBit = 4;                       // Ctl::sides of the seeding pseudo-round
// plan_round flags: account only / run the stalled plan speculatively / run it
// as a host-planned round / plan, then stall for the host (host-only mode)
// ... / a pipelined plan (accounts the pending round psides, stalls on any
// spill) / a drain (account the pending round exactly, then leave the pipeline)
enum : int { kPlanAccountOnly = 1, kPlanResume = 2, kPlanForce = 4, kPlanStall = 8, kPlanPipe = 16, kPlanDrain = 32 };
// A pipelined plan stalls (and the search continues with exact plans) once a
// rank's frontier share passes this many edges: the next round's frontier,
// which it cannot see yet, must stay far below the spill lists.
constexpr uint64_t kPipeMaxEdges = 1u << 14;
// ... and only on graphs without hubs: a round whose frontier the plan cannot
// see yet is at most (its input's vertices) x (max degree) edges.  On a
// Kronecker graph the roots' neighbourhoods hold hubs of degree 10^5: the
// blind round expands them into tiny owner blocks, spills and drains on every
// query (Kronecker 22, P = 2: 1.57 ms pipelined vs 0.63 ms exact,
// profiles/r6_dist_rounds_local.jsonl).
constexpr uint64_t kPipeMaxDeg = 64;

struct Ctl {
  unsigned long long cnt[2];   // current frontier sizes (vertices)
  unsigned long long fed[2];   // current frontier degree sums
  unsigned long long fmax[2];  // the largest share of fed[s] on one rank (bounds a rank's candidate block)
  unsigned long long ved[2];   // degree sum of everything side s claimed
  unsigned long long vis[2];   // vertices side s claimed (incl. the root)
  unsigned long long key;      // (length << 32) | meet vertex, once found
  unsigned long long einsp;    // edges inspected by the expanded levels
  unsigned long long ticks;    // device time of the search (s_memrealtime, 100 MHz): seed -> this plan
  unsigned long long pkey;     // meet key found while a continuation round is still due (min so far)
  uint32_t depth[2];           // depth of the current frontier
  uint32_t dir[2];             // 1 top-down, 2 bottom-up (Beamer state)
  uint32_t turn;               // alternate policy
  uint32_t state;              // kRun / kDone / kDead / kStall
  uint32_t sides;              // sides THIS round expands (0 = no-op round)
  uint32_t modes;              // bit s: side s bottom-up this round
  uint32_t want, want_modes;   // the planned round (kept when it stalls)
  uint32_t stall;              // kStall* reason
  uint32_t rounds, lockstep_rounds, levels, sparse_levels;
  uint32_t next_it;            // k_spec_solo's exit: the round the host continues with
  uint32_t cont;               // sides THIS round continues: re-offer their spilled candidates (no expansion)
  uint32_t cont_due;           // sides whose level is incomplete (spilled candidates wait to be offered)
  uint32_t cont_rounds;        // continuation rounds run
  uint32_t lost;               // a rank's spill list overflowed (candidates dropped): the search failed
  // Pipelined rounds (DistTuning::pipeline): the plan of round it is made
  // before round it-1's claims are reduced, so it accounts round it-2.  The
  // round planned last time, not accounted yet, is psides / pcont; xdepth is
  // the depth of the frontier THIS round expands (= depth when nothing is
  // pending) -- every expansion / claim kernel takes its depths from xdepth.
  uint32_t psides, pcont;
  uint32_t xdepth[2];
};

struct Policy {
  double alpha, beta;
  // alpha, beta in 1/256 steps: the planner's Beamer tests in integer
  // arithmetic (one lane's f64 conversions and compares cost it ~1k cycles a
  // round; 14 and 24, the defaults, are exact)
  unsigned long long alpha_q, beta_q;
  unsigned long long nnz_total;
  uint32_t n;
  int lockstep, side, direction;
  uint32_t epoch;     // search number: tags the plan words (a late no-op round of the previous search never matches)
  uint32_t walk_cap;  // words of the pinned path buffer (one rank: the round that ends the search walks the path)
  uint32_t spill_cap; // candidates a rank's spill list holds per side (DView::spill_cap)
  int source_only;    // unidirectional BFS from src (DistBiBfs::search_unidirectional): side 0 expands alone
  int want_path;
};

// Reduced across ranks (device words), double-buffered like Ctl.
struct Reduced {
  unsigned long long sums[4];  // [2s] vertices side s claimed this round, [2s+1] their degree sum (sum)
  unsigned long long meetkey;  // (path length << 32) | meet vertex (min)
  unsigned long long nfmax[2]; // ~(this rank's degree sum of side s's new frontier): min = ~max over ranks
  uint32_t maxsend[2];         // candidates of side s on this rank (max; host-planned rounds)
  uint32_t md[2];              // depth of the meet vertex from each root (owner contributes; min)
  // candidates of side s one rank tried to spill this round (max): above the
  // spill list's capacity some were DROPPED and the level would be incomplete,
  // so the plan ends the search as an error (Ctl::lost) instead of going on
  uint32_t spillmax[2];
  unsigned long long spill[2]; // candidates of side s that did not fit their owner's block (sum)
  unsigned long long nocmax;   // ~(largest candidate count this rank addressed to one owner): min = ~max
  // pipelined rounds: candidates of side s that did not fit their owner's
  // block in the round whose exchange carried this record (max) -- the level
  // that round expanded is incomplete, so the next plan stalls and drains
  uint32_t nsp[2];
};
// Pipelined rounds: every owner-addressed exchange carries, in front of each
// peer's candidate blocks, the sender's reduction of the round before (its
// `red` with nsp of this round): the round's ONE collective is the exchange.
constexpr uint32_t kHdrWords = 32;
static_assert(sizeof(Reduced) <= kHdrWords * 4, "reduction header");

// One accounted round (SearchOptions::trace): the frontiers it expanded and
// what they discovered -- the same record on every rank.
struct RoundRec {
  uint32_t sides, modes, depth[2];
  unsigned long long cnt[2], fed[2];  // expanded frontiers (vertices, degree sum)
  unsigned long long sums[4];         // discovered: [2s] vertices, [2s+1] their degree sum
  unsigned long long meetkey;
};

// Per-round device stamps (DistTuning::stamps): s_memrealtime (100 MHz) at
// the entry of the round's expansion launch(es) and of its claim launch, and
// when their last workgroup finishes -- so the host can split a round into
// kernel time and the gaps the exchanges (and launch latencies) leave between
// the kernels.
struct RoundStamp {
  unsigned long long eb, ee, cb, ce;
  // small rounds (block 0): expansion planned, frontier staged + scanned,
  // edges done; claim: candidates claimed
  unsigned long long ep, es, ex, cx;
  unsigned long long sg;  // block (0, 0): the previous plan and the reductions staged (before planning)
  uint32_t tag, small;  // small: bit 0 expansion, bit 1 claim ran the one-workgroup path
};

struct DState {
  uint32_t fbeg[2], fend[2], qtail[2];  // queue[s][fbeg, fend) = frontier; qtail = append cursor
  uint32_t send_count[2];               // candidates this rank emitted for side s this level
  uint32_t done_blocks[3];              // last-block detection (expand, meet, hubs)
  uint32_t hub_count[2];                // deferred hubs of side s this level
  uint32_t pad;
  unsigned long long new_edges[2];      // degree sum of the vertices side s claimed this level
  uint32_t meet_found;                  // a single-side level claimed a vertex the other side holds
  unsigned long long t0;                // s_memrealtime at the seed
  uint32_t spill_n[2][2];               // [side][list] spilled candidates held (owner-addressed rounds)
  uint32_t spill_cur[2];                // [side] the list holding the candidates still to be offered
  uint32_t ocmax;                       // largest per-owner candidate count of this round (the header writer)
  uint32_t pad2[3];
};

struct DView {
  uint32_t n, lo, hi, chunk;  // owned = [lo, hi); owner(v) = v / chunk
  const uint64_t* row_off;    // owned rows
  const uint32_t* col;        // global column ids
  // One rank: packed adjacency {v, deg(v), row_off[v] lo, hi} per edge (16 B;
  // when it fits DistTuning's budget), so a solo round's claims need no
  // dependent row-offset load; nullptr = col + row_off.
  const uint4* padj;
  // Visited bits of both sides interleaved: owned word w of side s is
  // vis[s][2 * w] (vis[1] = vis[0] + 1), so the 64-bit word w of vis[0]
  // holds side 0 in its low and side 1 in its high half -- a claim's one
  // 64-bit atomicOr returns the other side's bit with its own.
  uint32_t* vis[2];
  uint32_t* parent[2];        // chunk entries, valid where visited
  uint32_t* depth[2];         // chunk entries, valid where visited
  uint32_t* queue[2];         // owned vertices (global ids) in claim order
  uint32_t* hubs[2];          // deferred high-degree frontier vertices (this level)
  uint32_t* sent[2];          // bitmaps over ALL vertices: remote vertices already offered this search
  uint32_t* obits[2];         // owned frontier slice (chunk/32 words)
  uint32_t* gbits[2];         // allgathered frontier bitmap (P * chunk/32 words: global index)
  uint32_t* sendbuf;          // candidate blocks {count, pad, (v, u) pairs}: 2 sides (x P owners in
                              // owner-addressed rounds: block (o, s) at (2 o + s) * block_words)
  uint32_t* ocount;           // [2][P] candidates addressed to each owner this round
  uint2* spill[2][2];         // [side][list] candidates that did not fit their owner's block
  uint32_t spill_cap;
  uint32_t* recvbuf;          // P ranks x 2 sides of blocks
  uint32_t cap;               // host-planned round: candidate pairs per rank per level
  int P;
  DState* st;
  Ctl* ctl;                   // [2]
  uint64_t* plan_ring;        // pinned [kPlanRing]: slot it % kPlanRing = fed_max << 32 | (it + 1) << 8 | state << 2 | sides
  uint64_t* plan_aux;         // pinned [kPlanRing]: largest per-owner candidate count of the round before it
  Ctl* host_ctl;              // pinned: the accounted Ctl, written by the round whose plan ends the search
  uint32_t* host_walk;        // pinned: {status, dS, dT, epoch, path[]} (one rank, the same round)
  struct RoundRec* trace;     // per-round record (SearchOptions::trace), or nullptr
  uint32_t trace_cap;
  RoundStamp* rstamp;         // [kTraceCap] per-round stamps (DistTuning::stamps), or nullptr
  Reduced* red;               // [2] this rank's values of a round (claims min the meet key here)
  // [2] x P: every rank's `red` of a round, allgathered (ONE collective per
  // round's reduction); readers reduce them (reduce_gathered).  One rank:
  // redg[p] = &red[p], nothing is gathered.
  Reduced* redg[2];
};

template <typename T>
__device__ __forceinline__ T* pick(T* const (&a)[2], int s) {
  return s ? a[1] : a[0];
}

__host__ __device__ inline uint64_t block_words(uint32_t cap) { return 2 + 2 * (uint64_t)cap; }
// Owner-addressed exchange (speculative rounds with more than one rank): one
// region per peer o -- the reduction header, then o's side-0 and side-1
// blocks of `ocap` pairs -- so ONE alltoall moves both sides and the header.
__host__ __device__ inline uint64_t peer_words(uint32_t ocap) { return kHdrWords + 2 * block_words(ocap); }
__host__ __device__ inline uint64_t oblock(int s, uint32_t o, uint32_t ocap) {
  return (uint64_t)o * peer_words(ocap) + kHdrWords + (uint64_t)s * block_words(ocap);
}

// Copy a small struct into LDS, one 32-bit word per thread (the block's
// threads issue the loads together).
__device__ __forceinline__ void stage_words(void* dst, const void* src, size_t bytes) {
  for (uint32_t k = threadIdx.x; k < bytes / 4; k += blockDim.x)
    static_cast<uint32_t*>(dst)[k] = static_cast<const uint32_t*>(src)[k];
}

// The reduction of a round from every rank's gathered values: counts and
// degree sums add, the meet key / frontier-max complements / meet depths
// take the min, send counts the max.
__device__ void reduce_gathered(const Reduced* g, int P, Reduced& out) {
  Reduced r = g[0];
  for (int k = 1; k < P; ++k) {
    const Reduced& x = g[k];
    for (int i = 0; i < 4; ++i) r.sums[i] += x.sums[i];
    r.meetkey = min(r.meetkey, x.meetkey);
    r.nocmax = min(r.nocmax, x.nocmax);
    for (int s = 0; s < 2; ++s) {
      r.spill[s] += x.spill[s];
      r.nfmax[s] = min(r.nfmax[s], x.nfmax[s]);
      r.maxsend[s] = max(r.maxsend[s], x.maxsend[s]);
      r.md[s] = min(r.md[s], x.md[s]);
      r.spillmax[s] = max(r.spillmax[s], x.spillmax[s]);
      r.nsp[s] = max(r.nsp[s], x.nsp[s]);
    }
  }
  out = r;
}

// ---------------------------------------------------------------------------
// Round policy (device).  Accounts the previous round, then plans this one.
// Every input is a reduced value, so every rank computes the same plan.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void plan_round_regs(const Ctl& p, const Reduced& rd, const Policy& pol,
                                                uint64_t spec_cap, int flags, Ctl& c);

// The planner runs on one thread with every operand in registers: its inputs
// are copied in once (one round of independent loads, LDS or global) and the
// plan copied out once -- on references into LDS or global memory its ~50
// dependent field accesses cost ~8k cycles per round (measured, k_spec_solo).
__device__ __forceinline__ void plan_round(const Ctl& p, const Reduced& rd, const Policy& pol, uint64_t spec_cap,
                                           int flags, Ctl& out) {
  const Ctl pl = p;
  const Reduced rl = rd;
  Ctl cl;
  plan_round_regs(pl, rl, pol, spec_cap, flags, cl);
  out = cl;
}


__device__ __forceinline__ void plan_round_regs(const Ctl& p0, const Reduced& rd, const Policy& pol,
                                                uint64_t spec_cap, int flags, Ctl& c) {
  // A pipelined plan (and the drain that leaves the pipeline) accounts the
  // PENDING round -- planned last time, its reduction arrived with the round
  // planned after it -- not the round planned last time.  Terminal plans
  // (no-op rounds past the end) account nothing.
  const bool pipe = (flags & kPlanPipe) != 0;
  Ctl p = p0;
  if ((pipe && p0.state == kRun) || (flags & kPlanDrain)) {
    p.sides = p0.psides;
    p.cont = p0.pcont;
    if (flags & kPlanDrain) p.state = kRun;  // the pipelined stall this drain answers
  }
  c = p;
  c.sides = 0;
  c.modes = 0;
  c.cont = 0;
  // the round planned now becomes the pending one (pipelined), or nothing is pending
  c.psides = pipe ? p0.sides : 0u;
  c.pcont = pipe ? p0.cont : 0u;
  uint32_t want = 0, wm = 0;
  if (p.state == kStall) {
    if (!(flags & (kPlanResume | kPlanForce))) return;  // stays stalled until the host acts
    want = p.want;
    wm = p.want_modes;
  } else {
    if (p.sides & kSeedBit) {  // the roots: frontier sizes of the seeding pseudo-round
      for (int s = 0; s < 2; ++s) {
        c.cnt[s] = rd.sums[2 * s];
        c.fed[s] = rd.sums[2 * s + 1];
        c.fmax[s] = c.fed[s];  // one owner per root
        c.ved[s] = c.fed[s];
        c.vis[s] = c.cnt[s];
      }
    } else if (p.sides | p.cont) {
      int ns = 0;
      for (int s = 0; s < 2; ++s) {
        if ((p.sides >> s) & 1) {
          ++ns;
          c.depth[s] += 1;
          c.levels += 1;
          c.cnt[s] = rd.sums[2 * s];
          c.fed[s] = rd.sums[2 * s + 1];
          c.fmax[s] = ~rd.nfmax[s];
          c.ved[s] += c.fed[s];
          c.vis[s] += c.cnt[s];
        } else if ((p.cont >> s) & 1) {  // more of the same level (depth unchanged)
          c.cnt[s] += rd.sums[2 * s];
          c.fed[s] += rd.sums[2 * s + 1];
          c.fmax[s] += ~rd.nfmax[s];  // per-rank maxima added: an upper bound
          c.ved[s] += rd.sums[2 * s + 1];
          c.vis[s] += rd.sums[2 * s];
        }
      }
      if (p.sides) {  // a continuation completes its round's levels: not a round of its own
        c.rounds += 1;
        if (ns == 2) c.lockstep_rounds += 1;
      }
      // Candidates that did not fit their owner's block (owner-addressed
      // exchange) leave their side's level incomplete: a continuation round
      // offers them before anything else is decided -- the level's meets
      // are only complete (and its minimum exact) once they are claimed.
      c.pkey = min(p.pkey, rd.meetkey);
      if (rd.spillmax[0] > pol.spill_cap || rd.spillmax[1] > pol.spill_cap) {
        // candidates were dropped (emit_owned_pair): the level is incomplete,
        // so neither a meet nor "no path" from here on would be exact
        c.lost = 1;
        c.state = kDead;
        return;
      }
      c.cont_due = (rd.spill[0] ? 1u : 0u) | (rd.spill[1] ? 2u : 0u);
      // (pipelined: a spilling round stalls the plan after it before any
      // round is accounted with cont_due, so it is never set here)
      if (!c.cont_due) {
        if (c.pkey != kNoKey) {
          c.state = kDone;
          c.key = c.pkey;
          return;
        }
        // an empty frontier: that side's component is exhausted (checked for
        // both sides: a side that emptied while the other one's level was
        // still being completed by continuation rounds is caught here too)
        for (int s = 0; s < 2; ++s)
          if (c.cnt[s] == 0) c.state = kDead;
      }
    }
    c.xdepth[0] = c.depth[0];
    c.xdepth[1] = c.depth[1];
    if (c.state != kRun || (flags & kPlanAccountOnly)) return;
    // Pipelined: the round planned last time left candidates unsent (its
    // level is incomplete) -- stall; the host drains the pipeline (accounts
    // that round exactly) and the search goes on with exact plans, which run
    // the continuation round.
    if (pipe && ((((p0.sides & 3u) | p0.cont) && (rd.nsp[0] | rd.nsp[1])) || c.cont_due)) {
      c.state = kStall;
      c.stall = kStallPipe;
      return;
    }
    if (c.cont_due) {  // the continuation round: no expansion, the spilled candidates offered again
      c.cont = c.cont_due;
      c.cont_due = 0;
      c.cont_rounds += 1;
      c.state = kRun;
      c.stall = kStallNone;
      return;
    }
    if ((uint64_t)c.rounds > 2ull * pol.n + 2) {  // safety net (v3 parity: iteration cap N)
      c.state = kDead;
      return;
    }
    const unsigned long long flo = min(c.fed[0], c.fed[1]), fhi = max(c.fed[0], c.fed[1]);
    if (pol.source_only) {
      want = 1;  // a plain BFS from src: it ends when it claims dst (held by side 1 at depth 0)
    } else if (pol.lockstep && pol.side != (int)SidePolicy::kAlternate &&
        (fhi <= kLockstepEdges || (fhi <= 2 * flo && fhi <= kLockstepMaxEdges))) {
      want = 3;
    } else if (pol.side == (int)SidePolicy::kAlternate) {
      want = 1u << c.turn;
      c.turn ^= 1u;
    } else if (pol.side == (int)SidePolicy::kSmallerFrontier) {
      want = c.cnt[0] <= c.cnt[1] ? 1u : 2u;
    } else {
      want = c.fed[0] <= c.fed[1] ? 1u : 2u;
    }
    for (int s = 0; s < 2; ++s) {
      if (!((want >> s) & 1)) continue;
      uint32_t mode;
      if (pol.direction == (int)Direction::kTopDown) {
        mode = 1;
      } else if (pol.direction == (int)Direction::kBottomUp) {
        mode = 2;
      } else {
        // Beamer: m_f > m_u / alpha and n_f < n / beta, multiplied out, in
        // 1/256 fixed point (fed, m_u < 2^40 and alpha_q, beta_q <= 2^20 --
        // alpha and beta clamped to [0, 4096] by policy(): no u64 overflow)
        const unsigned long long m_u = pol.nnz_total > c.ved[s] ? pol.nnz_total - c.ved[s] : 0ull;
        if (c.dir[s] == 1 && c.fed[s] * pol.alpha_q > m_u * 256ull) c.dir[s] = 2;
        else if (c.dir[s] == 2 && c.cnt[s] * pol.beta_q < (unsigned long long)pol.n * 256ull) c.dir[s] = 1;
        mode = c.dir[s];
      }
      if (mode == 2) wm |= 1u << s;
    }
    c.want = want;
    c.want_modes = wm;
  }
  if (!(flags & kPlanForce)) {
    bool fits = wm == 0;
    for (int s = 0; s < 2; ++s)
      if (((want >> s) & 1) && (c.fmax[s] > spec_cap || (pipe && c.fmax[s] > kPipeMaxEdges)))
        fits = false;  // a rank's block holds its share
    if (!fits || (flags & kPlanStall)) {
      c.state = kStall;
      c.stall = pipe ? kStallPipe : (flags & kPlanStall) ? kStallHost : (wm ? kStallDense : kStallCap);
      return;
    }
  }
  c.state = kRun;
  c.stall = kStallNone;
  c.sides = want;
  c.modes = wm;
  if (pipe)  // the pending round's output is this round's frontier
    for (int s = 0; s < 2; ++s) c.xdepth[s] = c.depth[s] + ((p0.sides >> s) & 1u);
  for (int s = 0; s < 2; ++s)
    if ((want >> s) & 1) {
      c.einsp += c.fed[s];
      if (!((wm >> s) & 1)) c.sparse_levels += 1;
    }
}

// Publish round `p`'s plan; with tracing on, also record the round it
// accounted (pend 1, pipelined plans: the pending round psides / pcont of a
// running plan; pend 2, a drain: that of the stalled plan it answers; always
// top-down).
__device__ void publish(const DView& V, int p, const Ctl& prev, const Reduced& rd, const Ctl& c, int pend = 0) {
  V.ctl[p] = c;
  const bool live = prev.state == kRun || (pend == 2 && prev.state == kStall);
  const uint32_t asides = pend ? (live ? prev.psides : 0u) : prev.sides;
  const uint32_t acont = pend ? (live ? prev.pcont : 0u) : prev.cont;
  if (V.trace && asides && !(asides & kSeedBit) && c.rounds >= 1 && c.rounds <= V.trace_cap) {
    RoundRec& t = V.trace[c.rounds - 1];
    t.sides = asides;
    t.modes = pend ? 0u : prev.modes;
    for (int s = 0; s < 2; ++s) {
      t.depth[s] = prev.depth[s];
      t.cnt[s] = prev.cnt[s];
      t.fed[s] = prev.fed[s];
    }
    for (int k = 0; k < 4; ++k) t.sums[k] = rd.sums[k];
    t.meetkey = rd.meetkey;
  } else if (V.trace && acont && c.rounds >= 1 && c.rounds <= V.trace_cap) {
    RoundRec& t = V.trace[c.rounds - 1];  // a continuation adds to its round's record
    for (int k = 0; k < 4; ++k) t.sums[k] += rd.sums[k];
    t.meetkey = min(t.meetkey, rd.meetkey);
  }
}

// Meet detection at claim time (speculative rounds): `meetkey` non-null.
// Every vertex that becomes held by both sides in a round is seen by at least
// one of its two claims: each claim's atomicOr completes (its result decides
// `mine`) before the same thread's device-scope load of the other side's
// word, and device-scope atomics are coherent across XCDs -- so of two
// same-round claims the later one sees the earlier.  The other side's depth
// of v is read the same way; kEmpty there (depth arrays are kEmpty outside a
// search) means that side claimed v in THIS round and its store is not
// visible yet, so the depth is its frontier depth + 1.  single: a
// single-side level, where every meet has the same length, so the first one
// also raises DState::meet_found and the expansion loops stop early.
// (edge searches: dev::lift_search, device.hpp -- uniform trip count, no
// divergent loop exit for the compiler to drain outstanding loads at)
struct ClaimMeet {
  unsigned long long* meetkey = nullptr;
  uint32_t dclaim = 0;  // the depth the other side's claims of this round get (its kEmpty depth reads)
  bool single = false;
  // read the visited word before the atomicOr (skips the atomic for a vertex
  // already held): pays on big levels, where most edges lead to visited
  // vertices and the atomics' throughput counts; a small level's latency
  // chain is one round trip shorter without it
  bool precheck = true;
};

// Claim owned vertex v for side s (parent u, depth dnew).  Wave-cooperative:
// every lane of the wave calls it, `want` masks lanes.  One queue append and
// one degree-sum atomic per wave.
// have_row: the caller read v's row [prb, pre_) with v itself (packed adjacency).
__device__ __forceinline__ void wave_claim(const DView& V, int s, bool want, uint32_t v, uint32_t u,
                                           uint32_t dnew, const ClaimMeet& cm = ClaimMeet{}, bool have_row = false,
                                           unsigned long long prb = 0, unsigned long long pre_ = 0) {
  const uint32_t li = v - V.lo;
  bool mine = false, other = false;
  unsigned long long best = kNoKey;
  unsigned long long rb = 0, re = 0;
  if (want) {
    unsigned long long* w = reinterpret_cast<unsigned long long*>(V.vis[0]) + (li >> 5);
    const unsigned long long m = 1ull << ((li & 31) + 32 * s);
    if (!cm.precheck || !(*w & m)) {
      // both sides' bits in one word: the claim returns the other side's too;
      // of two same-round claims of v the later atomic sees the earlier
      const unsigned long long old = atomicOr(w, m);
      rb = have_row ? prb : V.row_off[li];  // the degree, fetched beside the claim (independent of its result)
      re = have_row ? pre_ : V.row_off[li + 1];
      mine = !(old & m);
      other = (old >> ((li & 31) + 32 * (s ^ 1))) & 1ull;
    }
    if ((cm.meetkey || cm.single) && mine && other) {
      if (cm.meetkey) {
        uint32_t dd = __hip_atomic_load(&pick(V.depth, s ^ 1)[li], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (dd == kEmpty) dd = cm.dclaim;
        best = ((unsigned long long)(dnew + dd) << 32) | v;
      }
      if (cm.single) __hip_atomic_store(&V.st->meet_found, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (cm.meetkey && __ballot(best != kNoKey)) {  // rare: the meeting round
#pragma unroll
    for (int o = kWave / 2; o >= 1; o >>= 1) {
      const unsigned long long y = __shfl_xor(best, o);
      best = y < best ? y : best;
    }
    if (__lane_id() == 0) atomicMin(cm.meetkey, best);
  }
  const unsigned long long mask = __ballot(mine);
  if (!mask) return;  // wave-uniform
  const uint32_t lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  unsigned long long deg = 0;
  if (mine) {
    pick(V.parent, s)[li] = u;
    pick(V.depth, s)[li] = dnew;
    deg = re - rb;
  }
  uint32_t pos = 0;
  if (lane == (uint32_t)leader) pos = atomicAdd(&V.st->qtail[s], (uint32_t)__popcll(mask));
  pos = __shfl(pos, leader);
  if (mine) pick(V.queue, s)[pos + mbcnt64(mask)] = v;
  deg = wave_sum(deg);
  if (lane == (uint32_t)leader) (void)__hip_atomic_fetch_add(&V.st->new_edges[s], deg, __ATOMIC_RELAXED,
                                                             __HIP_MEMORY_SCOPE_AGENT);
}

// Offer remote vertex v (parent u) to its owner -- at most once per search and
// side: after the level that offered it, v is visited by its owner (claimed
// from the exchange, or by the bottom-up fallback of an overflowing level).
// Owner-addressed emission (speculative rounds with more than one rank): one
// block of `cap` pairs per owner rank; a candidate that does not fit goes to
// the round's spill list and is offered by a continuation round.
struct OwnerEmit {
  uint32_t cap = 0;           // pairs per owner block; 0 = one block per side (host-planned rounds)
  uint32_t bw = 0;            // words per block
  uint2* spill = nullptr;     // this round's overflow list of the side
  uint32_t* spill_n = nullptr;
};

__device__ __forceinline__ void emit_owned_pair(const DView& V, int s, uint32_t v, uint32_t u, const OwnerEmit& oe) {
  const uint32_t o = v / V.chunk;
  const uint32_t pos = atomicAdd(&V.ocount[s * V.P + o], 1u);
  if (pos < oe.cap) {
    reinterpret_cast<uint2*>(V.sendbuf + oblock(s, o, oe.cap))[1 + pos] = make_uint2(v, u);
  } else {
    // (a rank's candidates of a level never exceed the list while its frontier
    // edges stay within round_edge_cap(); if they ever do, the count still
    // grows past the cap and the next plan fails the search: Ctl::lost)
    const uint32_t q = atomicAdd(oe.spill_n, 1u);
    if (q < V.spill_cap) oe.spill[q] = make_uint2(v, u);
  }
}

// Pipelined rounds: the reduction header in front of every peer's blocks --
// this rank's `red` of round it - 1 (final since that round's claim kernel)
// with nsp = the candidates of round `it` that went to the spill lists.
__device__ void write_peer_headers(const DView& V, uint32_t cap, uint32_t it, uint32_t nsp0, uint32_t nsp1) {
  constexpr uint32_t kRedW = sizeof(Reduced) / 4, kNspW = offsetof(Reduced, nsp) / 4;
  const uint32_t* red = reinterpret_cast<const uint32_t*>(&V.red[(it - 1u) & 1u]);
  for (uint32_t t = threadIdx.x; t < (uint32_t)V.P * kHdrWords; t += blockDim.x) {
    const uint32_t o = t / kHdrWords, w = t % kHdrWords;
    const uint32_t x = w == kNspW ? nsp0 : w == kNspW + 1 ? nsp1 : w < kRedW ? red[w] : 0u;
    V.sendbuf[(uint64_t)o * peer_words(cap) + w] = x;
  }
}

// The last workgroup of a round's emitting kernel: every owner block's count
// into its header, the counters reset, the largest per-owner count kept for
// the host's sizing of the next blocks; pipelined rounds also write the
// reduction headers.
__device__ void write_owner_headers(const DView& V, uint32_t cap, uint32_t it, int pipe) {
  for (uint32_t t = threadIdx.x; t < 2u * V.P; t += blockDim.x) {
    const uint32_t ss = t / V.P, o = t % V.P, k = ss * V.P + o;
    const uint32_t cnt = atomicExch(&V.ocount[k], 0u);
    V.sendbuf[oblock((int)ss, o, cap)] = min(cnt, cap);
    if (cnt) atomicMax(&V.st->ocmax, cnt);
  }
  if (pipe) {
    // the other blocks' spills are atomics completed before they counted in
    const DState* st = V.st;
    const uint32_t n0 = __hip_atomic_load(&st->spill_n[0][st->spill_cur[0]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t n1 = __hip_atomic_load(&st->spill_n[1][st->spill_cur[1]], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    write_peer_headers(V, cap, it, n0, n1);
  }
}

// Where a claim kernel reads the exchange: rank r's block for this rank (its
// header, then both sides' candidate blocks).  direct: the transport's
// in-place view (Comm::alltoall_view -- the local group points into the
// peers' send buffers, nothing is copied); else the copy in recvbuf.
struct PeerTab {
  const uint32_t* p[kStageRanks];
  int direct;
};
__device__ __forceinline__ const uint32_t* peer_at(const DView& V, const PeerTab& pt, uint32_t r, uint32_t cap) {
  return pt.direct ? pt.p[r] : V.recvbuf + (uint64_t)r * peer_words(cap);
}
// side s's candidate block inside a peer's block
__device__ __forceinline__ uint64_t pblock(int s, uint32_t cap) { return kHdrWords + (uint64_t)s * block_words(cap); }

// Device-ordered exchange (DistTuning::dev_sync over Comm::dev_window): the
// round's expansion writes this rank's window half (epoch & 1) and the claim
// kernel reads the peers' halves in place once every peer's flag reached the
// round's epoch -- no host rendezvous and no cross-stream event between the
// two kernels.  A rank's flag is raised by its claim kernel, so it also says
// that rank's claims of the epoch before are complete: the half a rank
// rewrites two epochs later is no longer read by anyone.  The data were
// written by the peers' previous kernels (the kernel boundary writes the
// XCD L2s back); the waiter polls with agent-scope loads and then acquires
// (L1 invalidate) before any load of them.  epoch 0 = off.
constexpr unsigned kDevSyncBlocks = 8;  // widest claim grid (per side) that waits on the device
struct DevSync {
  const unsigned long long* peer_flag[kStageRanks];
  unsigned long long* flag;       // this rank's (its window's first word)
  unsigned long long epoch;
  unsigned long long limit;       // s_memrealtime ticks a wait may take (the host's timeout)
  const uint32_t* h_abort;        // pinned: set when the host gave up on the search
  int P;
};

// Thread 0 of a block: raise this rank's flag (block (0, 0) only), wait for
// every peer's, acquire.  False: the wait ran out or the host aborted (the
// block must leave without reading the exchange; the host throws).
__device__ bool dev_sync_wait(const DevSync& ds) {
  if (blockIdx.x == 0 && blockIdx.y == 0) __hip_atomic_store(ds.flag, ds.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  bool ok = true;
  for (int r = 0; r < ds.P && ok; ++r) {
    for (uint32_t k = 1; __hip_atomic_load(ds.peer_flag[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < ds.epoch; ++k) {
      __builtin_amdgcn_s_sleep(1);
      if ((k & 255) == 0 && (__builtin_amdgcn_s_memrealtime() - t0 > ds.limit ||
                             __hip_atomic_load(ds.h_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0)) {
        ok = false;
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  return ok;
}

// Every block: the wait above on thread 0, shared through LDS.
__device__ __forceinline__ bool dev_sync_block(const DevSync& ds) {
  __shared__ int sok;
  if (threadIdx.x == 0) sok = dev_sync_wait(ds) ? 1 : 0;
  __syncthreads();
  return sok != 0;
}

// The end of a search that exchanged through the window: after this kernel
// every peer's claims of the search are complete (their windows may be
// released or rewritten), one epoch of its own.
__global__ void k_dev_barrier(DevSync ds) {
  if (threadIdx.x == 0) (void)dev_sync_wait(ds);
}

// Pipelined rounds, claim kernel: every peer's header -- its reduction of
// round it - 1 -- into the gathered slot of that round (what the round's
// separate allgather delivers in exact mode), read by the plan of round it + 1.
__device__ void scatter_peer_headers(const DView& V, uint32_t cap, uint32_t it, const PeerTab& pt) {
  constexpr uint32_t kRedW = sizeof(Reduced) / 4;
  uint32_t* g = reinterpret_cast<uint32_t*>(V.redg[(it - 1u) & 1u]);
  for (uint32_t t = threadIdx.x; t < (uint32_t)V.P * kRedW; t += blockDim.x) {
    const uint32_t r = t / kRedW, w = t % kRedW;
    g[t] = peer_at(V, pt, r, cap)[w];
  }
}

__device__ __forceinline__ void wave_emit(const DView& V, int s, bool want, uint32_t v, uint32_t u, uint2* pairs,
                                          uint32_t cap, const OwnerEmit& oe) {
  uint32_t* sb = pick(V.sent, s);
  bool emit = false;
  if (want) {
    const uint32_t bit = 1u << (v & 31);
    if (!(sb[v >> 5] & bit)) emit = !(atomicOr(&sb[v >> 5], bit) & bit);
  }
  if (oe.cap) {
    if (emit) emit_owned_pair(V, s, v, u, oe);
    return;
  }
  const unsigned long long mask = __ballot(emit);
  if (!mask) return;  // wave-uniform
  const uint32_t lane = __lane_id();
  const int leader = __ffsll((long long)mask) - 1;
  uint32_t pos = 0;
  if (lane == (uint32_t)leader) pos = atomicAdd(&V.st->send_count[s], (uint32_t)__popcll(mask));
  pos = __shfl(pos, leader) + mbcnt64(mask);
  if (emit && pos < cap) pairs[pos] = make_uint2(v, u);
}

// Top-down pre phase of side s: edge-balanced expansion of the owned
// frontier.  A workgroup takes 256 frontier vertices, scans their degrees in
// LDS and walks the chunk's edges one per lane (binary search for the owning
// vertex), so a hub costs the same per edge as a leaf and no lane idles on a
// short row.  Block-uniform control flow (it contains barriers).
__device__ __forceinline__ bool meet_seen(const DView& V) {
  return __hip_atomic_load(&V.st->meet_found, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
}

// exit_on_meet: a single-side level, which stops once a meet is claimed.
__device__ void td_expand_side(const DView& V, int s, uint32_t dnew, uint2* pairs, uint32_t cap, uint32_t b0,
                               uint32_t nb, uint64_t hub_deg, bool exit_on_meet, const ClaimMeet& cm, uint32_t fb,
                               uint32_t F, const OwnerEmit& oe) {
  __shared__ uint32_t su[kThreads];
  __shared__ unsigned long long sb[kThreads], se[kThreads];
  __shared__ unsigned long long wsum[kThreads / kWave];
  __shared__ uint32_t sstop;
  const uint32_t* q = pick(V.queue, s);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  // A frontier of at most one chunk (a Kronecker hub round's few heavy-ish
  // vertices) would run on block 0 alone, its edges in serial 256-edge
  // steps: instead EVERY block stages that chunk and walks a stride of its
  // edges (block 0 alone defers the hubs).
  const bool spread = kDistSpread && F <= (uint32_t)kThreads && nb > 1;
  for (uint64_t c0 = spread ? 0 : (uint64_t)b0 * kThreads; c0 < F;
       c0 += spread ? (uint64_t)F : (uint64_t)nb * kThreads) {
    if (exit_on_meet && c0 != (uint64_t)b0 * kThreads) {  // block-uniform: the flag goes through LDS between barriers
      if (tid == 0) sstop = meet_seen(V) ? 1u : 0u;
      __syncthreads();
      if (sstop) break;
    }
    const uint64_t i = c0 + tid;
    unsigned long long deg = 0, b = 0;
    uint32_t u = 0;
    if (i < F) {
      u = q[fb + i];
      const uint32_t li = u - V.lo;
      b = V.row_off[li];
      deg = V.row_off[li + 1] - b;
    }
    const bool hub = deg > hub_deg;  // expanded by k_td_hubs instead
    const unsigned long long hm = __ballot(hub);
    if (hm && spread && b0 != 0) {
      deg = hub ? 0ull : deg;  // block 0 lists them
    } else if (hm) {
      uint32_t pos = 0;
      const int leader = __ffsll((long long)hm) - 1;
      if (lane == leader) pos = atomicAdd(&V.st->hub_count[s], (uint32_t)__popcll(hm));
      pos = __shfl(pos, leader);
      if (hub) pick(V.hubs, s)[pos + mbcnt64(hm)] = u;
      if (hub) deg = 0;
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
    uint32_t iter = 0;
    const unsigned long long ebase = spread ? (unsigned long long)b0 * kThreads : 0ull;
    const unsigned long long estep = spread ? (unsigned long long)nb * kThreads : (unsigned long long)kThreads;
    for (unsigned long long base = ebase; base < tot; base += estep, ++iter) {
      // wave-uniform exit (no barrier in this loop)
      if (exit_on_meet && iter > 0 && __builtin_amdgcn_readfirstlane(meet_seen(V) ? 1u : 0u)) break;
      const unsigned long long e = base + tid;
      const bool valid = e < tot;
      uint32_t uu = 0, v = 0;
      unsigned long long prb = 0, pre_ = 0;
      if (valid) {
        const uint32_t a = lift_search(se, kThreads, e, kThreads / 2);  // last slot whose edge range starts at or before e
        uu = su[a];
        const unsigned long long k = sb[a] + (e - se[a]);
        if (V.padj) {  // one rank: the neighbour's row comes with its id
          const uint4 q = V.padj[k];
          v = q.x;
          prb = (unsigned long long)q.z | (unsigned long long)q.w << 32;
          pre_ = prb + q.y;
        } else {
          v = V.col[k];
        }
      }
      const bool own = valid && v >= V.lo && v < V.hi;
      wave_claim(V, s, own, v, uu, dnew, cm, V.padj != nullptr, prb, pre_);
      wave_emit(V, s, valid && !own, v, uu, pairs, cap, oe);
    }
    __syncthreads();
  }
}

// End of a speculative round on this rank, by the last workgroup of the
// round's last claiming kernel: the per-side counts for the reduction, the
// frontiers advanced, and the NEXT round's meet key reset (this round's plan
// -- every workgroup of its first kernel -- has read that buffer).  `sides`
// comes from the caller's own copy of the plan: inside the planning kernel
// ctl[p] is block 0's plain store, not yet visible to the other workgroups.
// A continuation side (`cont`) extends its current frontier with what it
// claimed (same level) instead of advancing it, and its spill lists swap:
// the candidates still unsent are the ones this round could not place.
__device__ void spec_round_end(const DView& V, uint32_t it, uint32_t sides, uint32_t cont) {
  const int p = it & 1;
  DState* st = V.st;
  for (int s = 0; s < 2; ++s) {
    const bool on = (sides >> s) & 1, co = (cont >> s) & 1;
    const uint32_t qt = atomicAdd(&st->qtail[s], 0u);
    const unsigned long long ne = atomicExch(&st->new_edges[s], 0ull);
    V.red[p].sums[2 * s] = (on || co) ? (unsigned long long)(qt - st->fend[s]) : 0ull;
    V.red[p].sums[2 * s + 1] = (on || co) ? ne : 0ull;
    V.red[p].nfmax[s] = (on || co) ? ~ne : ~0ull;
    if (on) st->fbeg[s] = st->fend[s];
    if (on || co) st->fend[s] = qt;
    const uint32_t cur = st->spill_cur[s];
    if (co) {
      V.red[p].spill[s] = st->spill_n[s][cur ^ 1];
      st->spill_n[s][cur] = 0;
      st->spill_cur[s] = cur ^ 1;
    } else {
      V.red[p].spill[s] = on ? st->spill_n[s][cur] : 0ull;
    }
    V.red[p].spillmax[s] = (uint32_t)min(V.red[p].spill[s], 0xffffffffull);
    st->hub_count[s] = 0;
  }
  V.red[p].nocmax = ~(unsigned long long)atomicExch(&st->ocmax, 0u);
  V.red[p ^ 1].meetkey = kNoKey;
}

// A block's claims (returning and non-returning atomics) complete before it
// counts itself in for the last-block test of a round-ending kernel.
__device__ __forceinline__ void drain_atomics() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// Last-block detection: true in exactly one block, after every block of the
// grid has passed this point.  No fence: the last block reads only words the
// other blocks updated with returning atomics (completed before their waves
// reached the barrier, so before their arrival was counted) and reads them
// with atomics; plain stores of other blocks are consumed only by the next
// stream operation (kernel boundary).  A __threadfence here would cost
// ~3.5 us per block (buffer_wbl2 + buffer_inv, MI355X_MICROARCH.md price list).
__device__ __forceinline__ bool last_block(uint32_t* counter, uint32_t nblocks) {
  __shared__ int last;
  __syncthreads();
  if (threadIdx.x == 0) last = atomicAdd(counter, 1u) == nblocks - 1;
  __syncthreads();
  return last != 0;
}

// Plan-word tag: the search's epoch (8 bits) and the round number + 1 (16 bits;
// the host waits for a round at most kPlanRing - 1 behind the newest).
__host__ __device__ inline uint32_t plan_tag(uint32_t epoch, uint32_t it) {
  return (epoch & 0xffu) << 16 | ((it + 1u) & 0xffffu);
}

// One rank, the round whose plan ends the search: the two parent chains from
// the meet vertex into the pinned path buffer {status, dS, dT, epoch, path}
// (status 0 = walked, 1 = inconsistent, 2 = longer than the buffer: the host
// launches k_walk_local).  Called by a whole wave: lanes 0 and 1 walk one
// side each (one dependent load per hop).
__device__ void terminal_walk(const DView& V, unsigned long long key, const Policy& pol) {
  const uint32_t lane = threadIdx.x & 63;
  uint32_t* out = V.host_walk;
  const uint32_t meet = (uint32_t)key, hops = (uint32_t)(key >> 32);
  const bool fits = 4 + (uint64_t)hops + 1 <= pol.walk_cap && meet >= V.lo && meet < V.hi;
  uint32_t d0 = 0, d1 = 0;
  if (fits) {
    d0 = V.depth[0][meet - V.lo];
    d1 = V.depth[1][meet - V.lo];
  }
  bool ok = fits && d0 != kEmpty && d1 != kEmpty && d0 + d1 == hops;
  if (lane < 2 && ok) {
    const int sd = (int)lane;
    const uint32_t len = sd ? d1 : d0;
    uint32_t v = meet;
    for (uint32_t k = 0; k <= len && ok; ++k) {
      __hip_atomic_store(out + 4 + (sd ? d0 + k : d0 - k), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (k < len) {
        v = V.parent[sd][v - V.lo];
        ok = v >= V.lo && v < V.hi;
      }
    }
  }
  const bool both = __shfl(ok ? 1 : 0, 0) && __shfl(ok ? 1 : 0, 1);
  if (lane == 0) {
    __hip_atomic_store(out + 1, d0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out + 2, d1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out + 3, pol.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out, !fits ? 2u : both ? 0u : 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __threadfence_system();
}

// ---- speculative round kernels ---------------------------------------------

// Small rounds (P > 1): the whole rank's expansion / claims by one workgroup
// (defined with the solo kernel's helpers below).  The tests are grid-uniform:
// every block computed the same plan.
// Block (0, 0)'s LDS staging of both frontiers for a small round: filled by
// waves 1-3 while lane 0 plans the round (small_prefetch), so the frontier's
// queue and row-offset loads overlap the planner instead of following it.
struct SmallStage {
  uint32_t su[2 * kSmallV];            // frontier vertices: side 0's, then side 1's
  unsigned long long sb[2 * kSmallV];  // their row begins
  uint32_t se[2 * kSmallV + 1];        // degrees -> exclusive edge prefix
  uint32_t n0, nv, valid;              // side 0's count, both, staged (both frontiers fit)
  uint32_t qbase[2], spbase[2], lst[2];
};
__device__ void small_prefetch(const DView& V, const uint32_t* fr, SmallStage& S, uint32_t t, uint32_t nt);
__device__ void small_expand(const DView& V, const Ctl& c, uint32_t it, uint32_t ocap, const uint32_t* fr,
                             SmallStage& S, RoundStamp* rs, int pipe);
__device__ void small_claim_round(const DView& V, const Ctl& c, uint32_t it, uint32_t cap, RoundStamp* rs, int pipe,
                                  const PeerTab& pt);
__device__ __forceinline__ bool small_expand_ok(const Ctl& c, int P) {
  if (c.cont || !c.sides || P > kStageRanks) return false;
  for (int s = 0; s < 2; ++s)
    if (((c.sides >> s) & 1) && (c.fmax[s] > kSmallE || c.cnt[s] > kSmallV)) return false;
  return true;
}
__device__ __forceinline__ bool small_claim_ok(const Ctl& c, int P) {
  if (c.cont || !c.sides || P > kStageRanks) return false;
  unsigned long long most = 0;  // a sender's block of side s holds at most its frontier edges of s
  for (int s = 0; s < 2; ++s)
    if ((c.sides >> s) & 1) most += c.fmax[s];
  return most * (unsigned long long)P <= kSmallClaim;
}

__device__ __forceinline__ RoundStamp* round_stamp(const DView& V, uint32_t it) {
  return V.rstamp ? V.rstamp + (it % kTraceCap) : nullptr;
}

// Publish the plan `c` of round `it` (one wave calls it; lane 0 stores): the
// Ctl (and, tracing, the record of the round it accounted), the accounted
// Ctl to the host when this plan ends the search (one rank: the path walked
// into pinned memory first), the largest per-owner count of the round
// before, then the plan word the host paces its enqueueing on.
__device__ void publish_plan(const DView& V, uint32_t it, const Policy& pol, const Ctl& prev, const Reduced& rd,
                             Ctl& c, int pend) {
  const bool terminal = c.state == kDone || c.state == kDead;
  if (threadIdx.x == 0) publish(V, it & 1, prev, rd, c, pend);
  // the round that ends the search hands the host its accounted Ctl directly
  // (no k_final launch + wait after the batch); later no-op rounds repeat it
  const bool first_end = terminal && prev.state == kRun;
  // one rank holds every parent: walk the path now, into pinned memory
  if (first_end && V.P == 1 && c.state == kDone && pol.want_path) terminal_walk(V, c.key, pol);
  if (threadIdx.x != 0) return;
  if (first_end) {
    c.ticks = __builtin_amdgcn_s_memrealtime() - V.st->t0;
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&c);
    uint64_t* dst = reinterpret_cast<uint64_t*>(V.host_ctl);
    for (uint32_t k = 0; k < sizeof(Ctl) / 8; ++k)
      __hip_atomic_store(dst + k, src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __threadfence_system();
  }
  // the largest per-owner candidate count of the round before (sizes the
  // host's owner blocks), then the plan word behind it
  __hip_atomic_store(&V.plan_aux[it % kPlanRing], ~rd.nocmax, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __threadfence_system();
  // one 8-byte write-through store per round: the host paces its enqueueing
  // on the plan and sizes the rounds it enqueues from the frontier (larger
  // side's edge count, clamped to 32 bits)
  const unsigned long long fm = min(max(c.fmax[0], c.fmax[1]), 0xffffffffull);
  __hip_atomic_store(&V.plan_ring[it % kPlanRing],
                     (uint64_t)fm << 32 | ((uint64_t)plan_tag(pol.epoch, it) << 8) | (c.state << 2) | (c.sides & 3u),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Plan (every block computes the same plan; block 0 publishes it) + top-down
// pre phase of both sides (blockIdx.y = side) into blocks of `cap` pairs.
// header = 0: k_td_hubs runs next (it writes the headers); finish: this
// kernel ends the round's claims on this rank (one rank, no hub pass).
// pipe: a pipelined round (more than one rank, DistTuning::pipeline) -- the
// plan accounts the pending round from the reductions the last exchange
// carried (gathered slot it & 1; round 0 plans exactly from the seed), and
// the exchange of this round carries this rank's reduction of the last one.
__global__ __launch_bounds__(kThreads) void k_spec_expand(DView V, uint32_t it, Policy pol, uint32_t cap,
                                                          int flags, uint64_t hub_deg, int header, int finish,
                                                          uint32_t ocap, uint32_t plan_cap, int pipe) {
  const unsigned long long t_in = __builtin_amdgcn_s_memrealtime();
  const int p = it & 1;
  // a pipelined plan; round 0's accounts nothing (the seed is pending: its
  // reduction rides round 0's exchange, no seed gather) and plans both roots.
  // Every later pipelined round was planned by the previous round's claim
  // kernel (pre): this kernel only loads the plan.
  const bool pplan = pipe != 0;
  const bool pre = pipe && it > 0;
  __shared__ Ctl c, prev;
  __shared__ Reduced rd;
  __shared__ uint32_t fr[4];  // frontier bounds: fbeg[2], fend[2]
  // the previous plan and reduction (and the frontier bounds) staged into LDS
  // with one round of parallel loads (thread 0 alone would chain them
  // through plan_round's branches)
  if (pre) {
    stage_words(&c, &V.ctl[p], sizeof(Ctl));
  } else {
    stage_words(&prev, &V.ctl[p ^ 1], sizeof(Ctl));
  }
  const Reduced* const gsrc = V.redg[pplan ? p : p ^ 1];  // (round 0, pipelined: read, unused)
  __shared__ Reduced gst[kStageRanks];
  if (!pre && V.P <= kStageRanks) stage_words(gst, gsrc, (size_t)V.P * sizeof(Reduced));
  if (threadIdx.x >= kThreads - 4) {
    const uint32_t k = threadIdx.x - (kThreads - 4);
    fr[k] = k < 2 ? V.st->fbeg[k] : V.st->fend[k - 2];
  }
  __syncthreads();
  const unsigned long long t_staged = __builtin_amdgcn_s_memrealtime();
  __shared__ SmallStage sm;
  if (threadIdx.x < kWave) {  // wave 0 plans, on wave-uniform (scalar) registers
    if (threadIdx.x == 0 && !pre) {
      // (two call sites, not one through a conditional pointer: that made every
      // load of the planner's inputs a flat load)
      if (V.P <= kStageRanks) reduce_gathered(gst, V.P, rd);
      else reduce_gathered(gsrc, V.P, rd);
      if (pplan) rd.nocmax = ~0ull;  // (round 0 planned blind: no owner counts yet, the host's sizing reads 0)
      plan_round(prev, rd, pol, plan_cap, flags | (pplan ? kPlanPipe : 0), c);
    }
  } else if (threadIdx.x >= kWave && ocap && header && V.P <= kStageRanks && blockIdx.x == 0 && blockIdx.y == 0) {
    small_prefetch(V, fr, sm, threadIdx.x - kWave, kThreads - kWave);  // (a no-op unless the round is small)
  }
  __syncthreads();
  const bool terminal = c.state == kDone || c.state == kDead;
  // One block publishes the plan: block (0, 1) when the launch has a second
  // row, so the plan publication (its system-scope stores and fence, several
  // microseconds on one lane) never delays block (0, 0), which runs a small
  // round's whole expansion (small_expand).  (A pipelined round after the
  // first was planned and published by the previous round's claim kernel.)
  const bool planner = !pre && blockIdx.x == 0 && blockIdx.y == (gridDim.y > 1 ? 1u : 0u);
  if (planner && threadIdx.x < kWave) publish_plan(V, it, pol, prev, rd, c, pplan ? 1 : 0);
  // a round enqueued past the end of the search: nothing to expand, no round
  // end (every block sees the same plan, so no block counts itself in)
  if (terminal) return;
  if (RoundStamp* rs = round_stamp(V, it); rs && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {
    rs->eb = t_in;
    rs->tag = plan_tag(pol.epoch, it);
    rs->small = 0;
  }
  // small round: one workgroup.  The frontiers it stages must fit its LDS
  // arrays: checked on the frontier bounds every block read (a pipelined
  // plan's sizes are a round old and only steer the choice).
  const bool fits_stage = (!(c.sides & 1u) || fr[2] - fr[0] <= kSmallV) && (!(c.sides & 2u) || fr[3] - fr[1] <= kSmallV);
  if (ocap && header && fits_stage && small_expand_ok(c, V.P)) {
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      if (RoundStamp* rs = round_stamp(V, it); rs && threadIdx.x == 0) {
        rs->ep = __builtin_amdgcn_s_memrealtime();
        rs->sg = t_staged;
        rs->small = 1;
      }
      small_expand(V, c, it, ocap, fr, sm, round_stamp(V, it), pipe);
      if (RoundStamp* rs = round_stamp(V, it)) {
        __syncthreads();
        if (threadIdx.x == 0) rs->ee = __builtin_amdgcn_s_memrealtime();
      }
    }
    return;
  }
  const int s = (int)blockIdx.y;
  OwnerEmit oe;
  if (ocap) {
    const uint32_t cur = V.st->spill_cur[s], tgt = ((c.cont >> s) & 1) ? cur ^ 1 : cur;
    oe.cap = ocap;
    oe.bw = (uint32_t)block_words(ocap);
    oe.spill = V.spill[s][tgt];
    oe.spill_n = &V.st->spill_n[s][tgt];
  }
  if ((c.sides >> s) & 1) {
    ClaimMeet cm;
    cm.meetkey = &V.red[p].meetkey;
    cm.dclaim = c.xdepth[s ^ 1] + 1;  // (only a claim of the other side this round reads kEmpty)
    cm.single = c.sides != 3u;
    cm.precheck = c.fed[s] > kPrecheckEdges;
    td_expand_side(V, s, c.xdepth[s] + 1, reinterpret_cast<uint2*>(V.sendbuf + s * block_words(cap)) + 1, cap,
                   blockIdx.x, gridDim.x, hub_deg, c.sides != 3u, cm, fr[s], fr[2 + s] - fr[s], oe);
  } else if (ocap && ((c.cont >> s) & 1)) {
    // a continuation: the candidates of this side's level that did not fit
    // their owner's block last time, offered again (their `sent` bits stay set)
    const uint32_t cur = V.st->spill_cur[s];
    const uint32_t nsp = min(V.st->spill_n[s][cur], V.spill_cap);
    const uint2* sp = V.spill[s][cur];
    for (uint64_t i = blockIdx.x * (uint64_t)kThreads + threadIdx.x; i < nsp; i += (uint64_t)gridDim.x * kThreads) {
      const uint2 x = sp[i];
      emit_owned_pair(V, s, x.x, x.y, oe);
    }
  }
  if (!header) return;  // k_td_hubs runs next and writes the headers
  if (finish) drain_atomics();
  uint32_t* done = &V.st->done_blocks[0];
  if (last_block(done, gridDim.x * gridDim.y)) {
    if (ocap) {
      write_owner_headers(V, ocap, it, pipe);
      if (threadIdx.x == 0) atomicExch(done, 0u);
    } else if (threadIdx.x < 2) {
      const int ss = threadIdx.x;
      const uint32_t cnt = atomicExch(&V.st->send_count[ss], 0u);
      V.sendbuf[ss * block_words(cap)] = ((c.sides >> ss) & 1) ? min(cnt, cap) : 0u;
      if (ss == 0) atomicExch(&V.st->done_blocks[0], 0u);
    }
    if (finish && threadIdx.x == kWave) spec_round_end(V, it, c.sides, c.cont);  // another wave: the header atomics are independent
    if (RoundStamp* rs = round_stamp(V, it)) {
      __syncthreads();
      if (threadIdx.x == 0) rs->ee = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// ---- one-rank solo rounds -----------------------------------------------------
// With one rank there is no exchange, so the sparse rounds need no kernel
// boundary at all: ONE workgroup runs round after round with the frontiers,
// their row offsets and degree prefixes in LDS, the round's counters in LDS
// and the visited bitmaps claimed with L2 atomics (one CU: no device-scope
// round trip, no last-block detection, no plan word per round).  It stops at
// the first round it cannot hold -- a side above kSoloV vertices or kSoloE
// edges, or a bottom-up plan -- and leaves the state exactly as a stalled
// speculative round does (ctl/red/st), so the multi-workgroup rounds or a
// host-planned round take over; a plan that ends the search walks the path
// (terminal_walk) and publishes like k_spec_expand.
constexpr int kSoloT = 512;  // 2 waves per SIMD: 256 VGPRs (the unrolled claims need them)
constexpr uint32_t kSoloV = 2048;  // frontier vertices per side held in LDS
constexpr uint32_t kSoloE = 8192;  // frontier edges per side one solo round expands
constexpr uint32_t kSoloRounds = 1u << 16;
constexpr int kSoloU = 4;          // edges per thread in flight per pass

// Workgroup barrier that waits for LDS traffic only (no vmcnt drain).
__device__ __forceinline__ void solo_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Exclusive prefix of ND[0, cnt) into FP[0, cnt], FP[cnt] = total; half the
// workgroup per side (t = thread index within the half).
__device__ void solo_scan(const uint32_t* ND, uint32_t* FP, uint32_t cnt, uint32_t t, uint32_t* wtot) {
  constexpr uint32_t kHalf = kSoloT / 2, kPer = kSoloV / kHalf, kWaves = kHalf / 64;
  uint32_t v[kPer], run = 0;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = t * kPer + k;
    v[k] = i < cnt ? ND[i] : 0u;
    run += v[k];
  }
  uint32_t x = run;  // inclusive wave scan of the per-thread sums
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const uint32_t y = __shfl_up(x, o);
    if ((t & 63) >= (uint32_t)o) x += y;
  }
  if ((t & 63) == 63) wtot[t >> 6] = x;
  solo_lds_barrier();
  uint32_t base = 0, tot = 0;
#pragma unroll
  for (uint32_t w = 0; w < kWaves; ++w) {
    base += w < (t >> 6) ? wtot[w] : 0u;
    tot += wtot[w];
  }
  uint32_t e = base + x - run;
#pragma unroll
  for (uint32_t k = 0; k < kPer; ++k) {
    const uint32_t i = t * kPer + k;
    if (i < cnt) FP[i] = e;
    e += v[k];
  }
  if (t == 0) FP[cnt < kSoloV ? cnt : kSoloV] = tot;
}

// kStamp (BIBFS_DIST_STAMP=1): thread 0's cycles per phase summed over the
// rounds into stamps[0..7] = {plan, edges, end, scan, rounds, edges expanded, setup, exit}.
__device__ __forceinline__ unsigned long long solo_clock() {
  unsigned long long t;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  return t;
}

// The same prefix by ONE wave (32 entries per lane, one wave scan): no barrier.
// Inclusive wave64 prefix sum on the VALU via DPP (row shifts, then the
// row-15 / row-31 broadcasts): no LDS permutes.
__device__ __forceinline__ uint32_t dpp_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
  return x;
}

// Exclusive degree prefix FP[0..cnt] of ND[0..cnt) by one wave (cnt uniform,
// <= kSoloV): 64 consecutive entries per step -- conflict-free LDS accesses,
// one DPP scan, the running total carried in an SGPR -- so a round pays
// ceil(cnt / 64) steps.  (It was 32 fixed steps of lane-blocked entries, each
// LDS access a 32-word-stride bank conflict: ~5.4k cycles per G(1M) round,
// profiles/r3_dist_solo_stamps.txt.)
__device__ void solo_wave_scan(const uint32_t* ND, uint32_t* FP, uint32_t cnt, uint32_t lane) {
  uint32_t carry = 0;
  for (uint32_t c0 = 0; c0 < cnt; c0 += kWave) {
    const uint32_t i = c0 + lane;
    const uint32_t v = i < cnt ? ND[i] : 0u;
    const uint32_t x = dpp_scan(v);
    if (i < cnt) FP[i] = carry + x - v;
    carry += (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
  }
  if (lane == 0) FP[cnt] = carry;
}

template <bool kStamp>
__global__ __launch_bounds__(kSoloT, 1) void k_spec_solo(DView V, uint32_t it0, Policy pol, uint32_t emax,
                                                         int seed, uint32_t seed_src, uint32_t seed_dst,
                                                         uint32_t* fin, uint32_t tag, unsigned long long* stamps) {
  unsigned long long ph[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, tp = kStamp ? solo_clock() : 0;
#define SOLO_PH(k)                                \
  if (kStamp && threadIdx.x == 0) {               \
    const unsigned long long t_ = solo_clock();   \
    ph[k] += t_ - tp;                             \
    tp = t_;                                      \
  }
  __shared__ Ctl c, pc;  // this round's plan / the executed previous plan
  __shared__ Reduced rd;  // the previous round's reduction (one rank: local)
  __shared__ uint32_t FV[2][2][kSoloV];             // [buffer][side] frontier vertices
  __shared__ unsigned long long FB[2][2][kSoloV];   // their row begins
  __shared__ uint32_t FP[2][kSoloV + 1];             // [side] exclusive degree prefix of the current frontier
  __shared__ uint32_t ND[2][kSoloV];                 // [side] degrees of the vertices claimed this round
  __shared__ uint32_t wtot[2][kSoloT / 128];
  __shared__ uint32_t nf[2], qt[2], fbg[2], fnd[2], cb[2], go;
  __shared__ unsigned long long ne[2], best;
  const uint32_t tid = threadIdx.x;
  // the arrays in registers: selected per lane by side (an indexed DView
  // member would be a vector load from the kernel arguments per use)
  const uint32_t* const col = V.col;
  const uint64_t* const row_off = V.row_off;
  const uint4* const padj = V.padj;
  unsigned long long* const visw = reinterpret_cast<unsigned long long*>(V.vis[0]);  // both sides per word
  uint32_t* const par0 = V.parent[0];
  uint32_t* const par1 = V.parent[1];
  uint32_t* const dep0 = V.depth[0];
  uint32_t* const dep1 = V.depth[1];
  uint32_t* const que0 = V.queue[0];
  uint32_t* const que1 = V.queue[1];
  const uint32_t lo = V.lo;
  const uint32_t half = tid / (kSoloT / 2);  // the side a thread scans for
  if (seed & 1) {
    // the seeding pseudo-round (k_seed) done here: one launch fewer, and the
    // state goes straight into LDS (round it0 = 0 accounts it)
    if (tid < 2) {
      const uint32_t v = tid ? seed_dst : seed_src, li = v - lo;
      const unsigned long long b = row_off[li], d = row_off[li + 1] - b;
      __hip_atomic_fetch_or(visw + (li >> 5), 1ull << ((li & 31) + 32 * tid), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_WORKGROUP);
      (tid ? par1 : par0)[li] = kEmpty;
      __hip_atomic_store((tid ? dep1 : dep0) + li, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      (tid ? que1 : que0)[0] = v;
      fbg[tid] = 0;
      fnd[tid] = qt[tid] = 1;
      cb[tid] = 0;
      FV[0][tid][0] = v;
      FB[0][tid][0] = b;
      ND[tid][0] = (uint32_t)min(d, (unsigned long long)kSoloE + 1);
      rd.sums[2 * tid] = 1;
      rd.sums[2 * tid + 1] = d;
    }
    if (tid == 0) {
      V.st->t0 = __builtin_amdgcn_s_memrealtime();
      rd.meetkey = kNoKey;
      Ctl z = {};
      z.dir[0] = z.dir[1] = 1;
      z.state = kRun;
      z.sides = kSeedBit;
      z.key = z.pkey = kNoKey;
      pc = z;
      rd.spill[0] = rd.spill[1] = 0;
      rd.spillmax[0] = rd.spillmax[1] = 0;
      rd.nocmax = ~0ull;
    }
    __syncthreads();
  } else {
    const int pp = (it0 + 1) & 1;  // buffers of round it0 - 1
    stage_words(&pc, &V.ctl[pp], sizeof(Ctl));
    stage_words(&rd, &V.red[pp], sizeof(Reduced));
    if (tid < 2) {
      fbg[tid] = V.st->fbeg[tid];
      fnd[tid] = V.st->fend[tid];
      qt[tid] = V.st->qtail[tid];
      cb[tid] = 0;
    }
    __syncthreads();
    // the current frontiers (at most kSoloV each, or the first plan stops)
    for (uint32_t i = tid; i < 2 * kSoloV; i += kSoloT) {
      const uint32_t sd = i / kSoloV, k = i % kSoloV;
      if (fbg[sd] + k < fnd[sd]) {
        const uint32_t v = V.queue[sd][fbg[sd] + k];
        const unsigned long long b = V.row_off[v - V.lo];
        FV[0][sd][k] = v;
        FB[0][sd][k] = b;
        ND[sd][k] = (uint32_t)min(V.row_off[v - V.lo + 1] - b, (unsigned long long)kSoloE + 1);
      }
    }
    __syncthreads();
  }
  solo_scan(ND[half], FP[half], min(fnd[half] - fbg[half], kSoloV), tid % (kSoloT / 2), wtot[half]);
  __syncthreads();

  uint32_t it = it0;
  SOLO_PH(6)
  // One lane plans round `it` (from pc / rd); stalls a round the solo
  // workgroup cannot hold, and resets the round's LDS counters.
  auto plan_next = [&](uint32_t it_) {
    plan_round(pc, rd, pol, emax, 0, c);  // a side above emax frontier edges: kStallCap
    bool fits = true;
    for (int sd = 0; sd < 2; ++sd)
      if (((c.want >> sd) & 1) && (c.cnt[sd] > kSoloV || fnd[sd] - fbg[sd] > kSoloV)) fits = false;
    if (c.state == kRun && !fits) {  // the multi-workgroup rounds take it from here
      c.state = kStall;
      c.stall = kStallCap;
      c.sides = c.modes = 0;
      c.einsp = pc.einsp;
      c.sparse_levels = pc.sparse_levels;
    }
    go = c.state == kRun;
    if (go) {
      publish(V, it_ & 1, pc, rd, c);
      nf[0] = nf[1] = 0;
      ne[0] = ne[1] = 0;
      best = kNoKey;
    }
  };
  constexpr uint32_t kPlanner = 2 * kWave;  // lane 0 of wave 2: plans while waves 0-1 scan
  if (tid == kPlanner) plan_next(it);
  solo_lds_barrier();
  for (uint32_t r = 0; r < kSoloRounds; ++r, ++it) {
    SOLO_PH(0)
    if (!go) break;
    const uint32_t sides = c.sides;
    const uint32_t F0 = (sides & 1) ? fnd[0] - fbg[0] : 0u, F1 = (sides & 2) ? fnd[1] - fbg[1] : 0u;
    const uint32_t E0 = (sides & 1) ? FP[0][F0] : 0u, E1 = (sides & 2) ? FP[1][F1] : 0u;
    const bool pre = c.fed[0] + c.fed[1] > kPrecheckEdges;
    const uint32_t dn0 = c.depth[0] + 1, dn1 = c.depth[1] + 1;  // depth of this round's claims per side
    // kSoloU edges per thread per pass, every load of a pass in flight together;
    // the pass loop is wave-uniform (appends are aggregated per wave)
    const uint32_t E = E0 + E1, lane = tid & 63;
    for (uint32_t base = 0; base + (tid & ~63u) < E; base += kSoloT * kSoloU) {
      uint32_t uu[kSoloU], vv[kSoloU], oth[kSoloU];
      unsigned long long old[kSoloU];
      unsigned long long ad[kSoloU], rb[kSoloU], re[kSoloU];
      int ss[kSoloU];
      bool ok[kSoloU], mine[kSoloU];
#pragma unroll
      for (int j = 0; j < kSoloU; ++j) {
        const uint32_t e = base + (uint32_t)j * kSoloT + tid;
        ok[j] = e < E;
        const int sd = e >= E0;
        ss[j] = sd;
        const uint32_t k = ok[j] ? (sd ? e - E0 : e) : 0u, b = cb[sd];
        // last slot whose edge range starts at or before k
        const uint32_t a = lift_search(FP[sd], ok[j] ? (sd ? F1 : F0) : 1u, k, lift_top(max(F0, F1)));
        uu[j] = FV[b][sd][a];
        ad[j] = FB[b][sd][a] + (k - FP[sd][a]);
      }
      unsigned long long pb[kSoloU];
      uint32_t pd[kSoloU];
      if (padj) {  // kernel argument: uniform
#pragma unroll
        for (int j = 0; j < kSoloU; ++j) {
          const uint4 q = padj[ok[j] ? ad[j] : 0ull];  // an idle slot reads a valid entry
          vv[j] = q.x;
          pd[j] = q.y;
          pb[j] = (unsigned long long)q.z | (unsigned long long)q.w << 32;
        }
      } else {
#pragma unroll
        for (int j = 0; j < kSoloU; ++j) vv[j] = col[ok[j] ? ad[j] : 0ull];  // an idle slot reads a valid word
      }
#pragma unroll
      for (int j = 0; j < kSoloU; ++j) vv[j] = ok[j] ? vv[j] : lo;
      // claims: one CU, so the atomics are performed in its L2 (workgroup
      // scope); one 64-bit atomicOr returns both sides' bits (of two
      // same-round claims of a vertex the later sees the earlier); the
      // degree is fetched beside the claim
#pragma unroll
      for (int j = 0; j < kSoloU; ++j) {
        const uint32_t li = vv[j] - lo;
        const unsigned long long m = 1ull << ((li & 31) + 32 * ss[j]);
        unsigned long long* w = visw + (li >> 5);
        const bool claim = ok[j] && (!pre || !(*w & m));  // a stale L1 word only misses bits: safe
        old[j] = claim ? __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) : m;
        if (padj) {  // the row came with the neighbour id
          rb[j] = claim ? pb[j] : 0ull;
          re[j] = claim ? pb[j] + pd[j] : 0ull;
        } else {
          rb[j] = claim ? row_off[li] : 0ull;
          re[j] = claim ? row_off[li + 1] : 0ull;
        }
      }
#pragma unroll
      for (int j = 0; j < kSoloU; ++j) {
        const uint32_t li = vv[j] - lo;
        mine[j] = !((old[j] >> ((li & 31) + 32 * ss[j])) & 1ull);
        oth[j] = (uint32_t)(old[j] >> (32 * (ss[j] ^ 1)));  // the other side's half
      }
#pragma unroll
      for (int j = 0; j < kSoloU; ++j) {
        const uint32_t li = vv[j] - lo, bit = 1u << (li & 31);
        const int sd = ss[j];
        const uint32_t dnew = sd ? dn1 : dn0;
        if (mine[j] && (oth[j] & bit)) {  // rare: a meet
          uint32_t dd = __hip_atomic_fetch_add((sd ? dep0 : dep1) + li, 0u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
          if (dd == kEmpty) dd = (sd ? dn0 : dn1);  // claimed this round, its store not performed yet
          atomicMin(&best, ((unsigned long long)(dnew + dd) << 32) | vv[j]);
        }
        if (mine[j]) {
          (sd ? par1 : par0)[li] = uu[j];
          __hip_atomic_store((sd ? dep1 : dep0) + li, dnew, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
#pragma unroll
        for (int side = 0; side < 2; ++side) {  // appends: one LDS atomic per wave and side
          const bool here = mine[j] && sd == side;
          const unsigned long long m = __ballot(here);
          if (!m) continue;  // wave-uniform
          uint32_t pos = 0;
          if (lane == 0) pos = atomicAdd(&nf[side], (uint32_t)__popcll(m));
          pos = __shfl(pos, 0) + mbcnt64(m);
          const unsigned long long dg = here ? re[j] - rb[j] : 0ull;
          const unsigned long long dsum = wave_sum(dg);
          if (lane == 0) atomicAdd(&ne[side], dsum);
          if (here) {
            (side ? que1 : que0)[qt[side] + pos] = vv[j];
            if (pos < kSoloV) {
              FV[cb[side] ^ 1][side][pos] = vv[j];
              FB[cb[side] ^ 1][side][pos] = rb[j];
              ND[side][pos] = (uint32_t)min(dg, (unsigned long long)kSoloE + 1);
            }
          }
        }
      }
    }
    __syncthreads();  // (with vmcnt(0)): this round's depth stores are in L2 before a later round reads them
    SOLO_PH(1)
    if (kStamp && tid == 0) {
      ph[4] += 1;
      ph[5] += E;
    }
    // The next frontiers' degree prefix -- wave 0 side 0, wave 1 side 1, no
    // barrier inside (an idle side's prefix is rebuilt unchanged) -- while
    // lane 0 of wave 2 does the round's bookkeeping and plans the next
    // round; ONE LDS barrier orders all of it for everyone.
    const uint32_t wid = tid / kWave;
    if (wid < 2) {
      const uint32_t cnt_next = ((sides >> wid) & 1) ? nf[wid] : fnd[wid] - fbg[wid];
      solo_wave_scan(ND[wid], FP[wid], min(cnt_next, kSoloV), lane);
    } else if (tid == kPlanner) {
      for (int sd = 0; sd < 2; ++sd) {
        const bool on = (sides >> sd) & 1;
        rd.sums[2 * sd] = on ? (unsigned long long)nf[sd] : 0ull;
        rd.sums[2 * sd + 1] = on ? ne[sd] : 0ull;
        rd.nfmax[sd] = on ? ~ne[sd] : ~0ull;
        if (on) {
          fbg[sd] = fnd[sd];
          fnd[sd] = qt[sd] + nf[sd];
          qt[sd] = fnd[sd];
          cb[sd] ^= 1u;
        }
      }
      rd.meetkey = best;
      rd.spill[0] = rd.spill[1] = 0;
      rd.spillmax[0] = rd.spillmax[1] = 0;
      rd.nocmax = ~0ull;
      pc = c;
      plan_next(it + 1);
    }
    solo_lds_barrier();
    SOLO_PH(3)
  }
  // ---- exit: the state a stalled speculative round leaves, or the end of the search
  const bool ended = c.state == kDone || c.state == kDead;
  if (tid < kWave) {
  if (V.P == 1 && c.state == kDone && pol.want_path) terminal_walk(V, c.key, pol);  // wave 0
  if (tid == 0) {
  const int p = it & 1;
  DState* st = V.st;
  for (int sd = 0; sd < 2; ++sd) {
    st->fbeg[sd] = fbg[sd];
    st->fend[sd] = fnd[sd];
    st->qtail[sd] = qt[sd];
    st->send_count[sd] = 0;
    st->hub_count[sd] = 0;
    st->new_edges[sd] = 0;
  }
  st->done_blocks[0] = st->done_blocks[1] = st->done_blocks[2] = 0;
  st->meet_found = 0;
  V.ctl[p ^ 1] = pc;  // round it - 1, executed, and its reduction
  V.red[p ^ 1] = rd;
  publish(V, p, pc, rd, c);  // this round's plan (and the trace record of round it - 1)
  Ctl h = c;
  if (c.state == kDone || c.state == kDead) {
    h.ticks = __builtin_amdgcn_s_memrealtime() - st->t0;
    h.next_it = it + 1;
  } else {
    // as k_spec_expand(it) publishing the stall, then k_final(it + 1)
    h.sides = h.modes = 0;
    V.ctl[p ^ 1] = h;
    V.red[p].meetkey = kNoKey;  // the buffer of round it + 2
    h.next_it = it + 2;
  }
  const uint64_t* src = reinterpret_cast<const uint64_t*>(&h);
  uint64_t* dst = reinterpret_cast<uint64_t*>(V.host_ctl);
  for (uint32_t k = 0; k < sizeof(Ctl) / 8; ++k)
    __hip_atomic_store(dst + k, src[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  SOLO_PH(7)
  if (kStamp)
    for (int k = 0; k < 10; ++k) stamps[k] = ph[k];
#undef SOLO_PH
  __threadfence_system();
  __hip_atomic_store(fin, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }  // tid == 0
  }  // wave 0
  // The reset below must not start before wave 0's terminal walk has read the
  // meet vertex's depths and parent chains: without this barrier waves 1..15
  // cleared them under it (an intermittent "parent chains do not add up" at
  // world 1, GPU suite, round 3).
  __syncthreads();
  // A search that ended here resets its own state after the host has its
  // answer (no k_cleanup launch; the next search's launch queues behind this
  // one): every vertex it claimed is in the queues.
  // (not when the path outgrew the pinned buffer: k_walk_local still reads the depths)
  if (!ended || (seed & 2) || (c.state == kDone && pol.want_path && 4 + (c.key >> 32) + 1 > pol.walk_cap)) return;
  for (int sd = 0; sd < 2; ++sd) {
    uint32_t* vis = pick(V.vis, sd);
    uint32_t* dep = sd ? dep1 : dep0;
    const uint32_t* q = sd ? que1 : que0;
    for (uint32_t i = tid; i < qt[sd]; i += kSoloT) {
      const uint32_t li = __hip_atomic_load(q + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - lo;
      vis[2 * (li >> 5)] = 0u;
      dep[li] = kEmpty;
    }
  }
}

// ---- small rounds with more than one rank: ONE workgroup per rank ---------------
// A sparse round's per-rank work at P > 1 is often a few hundred edges, yet
// the multi-workgroup kernels pay a chain of device-scope round trips for it
// (stamped, benchmarks/dist_rounds.py: G(1M) at P = 2 13 us of expansion and
// 6 us of claims per round): queue / degree / candidate counters as global
// atomics, last-block detection, owner headers by atomicExch.  When the plan
// says the round is small (every expanding side at most kSmallE frontier
// edges on any rank and kSmallV frontier vertices), block (0, 0) does the
// whole rank's round alone: counters in LDS, claims and the `sent` test as
// workgroup-scope atomics (performed in the CU's L2 -- no other workgroup
// touches these words during the launch, and the kernel boundary publishes
// them), the owner headers and the round state written once at the end.
// Every block computes the same plan, so the choice is grid-uniform; the
// other blocks return before touching any counter.

struct SmallCtr {
  uint32_t q[2];                 // queue entries this launch appended per side
  unsigned long long ne[2];      // their degree sums
  uint32_t oc[2][kStageRanks];   // candidates per (side, owner)
  uint32_t sp[2];                // candidates per side that went to the spill list
  unsigned long long best;       // meet key (min)
  uint32_t found;                // a meet was claimed
};

__device__ __forceinline__ unsigned long long wg_fetch_or(unsigned long long* w, unsigned long long m) {
  return __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ uint32_t wg_fetch_or32(uint32_t* w, uint32_t m) {
  return __hip_atomic_fetch_or(w, m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// Exclusive prefix of X[0, cnt) in place, X[cnt] = total (cnt <= 4 * kThreads,
// whole block, values < 2^32): 4 consecutive entries per thread, one DPP
// wave scan, the wave totals through LDS.
__device__ void small_scan(uint32_t* X, uint32_t cnt) {
  __shared__ uint32_t wt[kThreads / kWave];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  uint32_t v[4], run = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = 4 * tid + k;
    v[k] = i < cnt ? X[i] : 0u;
    run += v[k];
  }
  const uint32_t inc = dpp_scan(run);
  if (lane == 63) wt[wid] = inc;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kThreads / kWave; ++w) {
    pre += w < (int)wid ? wt[w] : 0u;
    tot += wt[w];
  }
  uint32_t e = pre + inc - run;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint32_t i = 4 * tid + k;
    if (i < cnt) X[i] = e;
    e += v[k];
  }
  if (tid == 0) X[cnt] = tot;
  __syncthreads();
}

// Claim owned vertex v for side s (parent u, depth dn[s]) inside a small
// round: the visited word by a workgroup-scope atomicOr (both sides' bits in
// it), the meet by the other side's bit, queue appends and degree sums into
// LDS.  Wave-cooperative (every lane calls it); the side is per lane, so one
// call serves both sides of a lockstep round.  dcl[s]: the depth a claim of
// the other side made in THIS round has (its depth store may not be visible).
// One workgroup alone claims in these words during the launch: workgroup
// scope (its L2) is enough, the kernel boundary publishes them.
// Split in two so a pass's items overlap: small_claim_issue sends the claim
// atomic and the row-bound loads of one item (nothing reads them), and the
// caller issues every item's (and every offer's) atomics before the first
// small_claim reads a result -- one round trip per pass, not one per item.
// (the row bounds are loaded beside the claim, independent of its result; a
// loser's load is wasted)
struct ClaimIn {
  unsigned long long old = 0, rb = 0, re = 0;
};
__device__ __forceinline__ void small_claim_issue(const DView& V, bool want, int s, uint32_t v, ClaimIn& in) {
  if (!want) return;
  const uint32_t li = v - V.lo;
  unsigned long long* const visw = reinterpret_cast<unsigned long long*>(V.vis[0]);
  in.old = wg_fetch_or(visw + (li >> 5), 1ull << ((li & 31) + 32 * s));
  in.rb = V.row_off[li];
  in.re = V.row_off[li + 1];
}
__device__ __forceinline__ void small_claim(const DView& V, SmallCtr& K, const uint32_t* qbase, bool want, int s,
                                            uint32_t v, uint32_t u, const uint32_t* dn, const uint32_t* dcl,
                                            bool single, const ClaimIn& in) {
  const uint32_t li = v - V.lo;
  bool mine = false;
  unsigned long long rb = 0, re = 0, best = kNoKey;
  if (want) {
    const unsigned long long m = 1ull << ((li & 31) + 32 * s);
    const unsigned long long old = in.old;
    rb = in.rb;
    re = in.re;
    mine = !(old & m);
    const bool other = (old >> ((li & 31) + 32 * (s ^ 1))) & 1ull;
    if (mine) {
      if (other) {
        uint32_t dd = __hip_atomic_load(&pick(V.depth, s ^ 1)[li], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (dd == kEmpty) dd = s ? dcl[1] : dcl[0];
        best = ((unsigned long long)((s ? dn[1] : dn[0]) + dd) << 32) | v;
      }
    }
  }
  if (__ballot(best != kNoKey)) {  // rare: the meeting round
#pragma unroll
    for (int o = kWave / 2; o >= 1; o >>= 1) {
      const unsigned long long y = __shfl_xor(best, o);
      best = y < best ? y : best;
    }
    if (__lane_id() == 0) {
      atomicMin(&K.best, best);
      if (single) K.found = 1;
    }
  }
  if (!__ballot(mine)) return;  // wave-uniform
  if (mine) {
    pick(V.parent, s)[li] = u;
    __hip_atomic_store(&pick(V.depth, s)[li], s ? dn[1] : dn[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  }
  const uint32_t lane = __lane_id();
#pragma unroll
  for (int sd = 0; sd < 2; ++sd) {
    const bool m = mine && s == sd;
    const unsigned long long mask = __ballot(m);
    if (!mask) continue;  // wave-uniform
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t pos = 0;
    if (lane == (uint32_t)leader) pos = atomicAdd(&K.q[sd], (uint32_t)__popcll(mask));
    pos = __shfl(pos, leader);
    if (m) pick(V.queue, sd)[qbase[sd] + pos + mbcnt64(mask)] = v;
    const unsigned long long deg = wave_sum(m ? re - rb : 0ull);
    if (lane == (uint32_t)leader) atomicAdd(&K.ne[sd], deg);
  }
}

// Offer remote vertex v (parent u) of side s to its owner: once per search
// (the `sent` bit, workgroup scope), into the owner's block or the spill list.
// (issued with the claims: small_emit_issue returns the old `sent` word)
__device__ __forceinline__ uint32_t small_emit_issue(const DView& V, bool want, int s, uint32_t v) {
  return want ? wg_fetch_or32(&pick(V.sent, s)[v >> 5], 1u << (v & 31)) : 0u;
}
__device__ __forceinline__ void small_emit(const DView& V, SmallCtr& K, const uint32_t* spbase, const uint32_t* lst,
                                           bool want, int s, uint32_t v, uint32_t u, uint32_t ocap, uint32_t old) {
  if (!want) return;
  if (old & (1u << (v & 31))) return;
  const uint32_t o = v / V.chunk;
  const uint32_t pos = atomicAdd(&K.oc[s][o], 1u);
  if (pos < ocap) {
    reinterpret_cast<uint2*>(V.sendbuf + oblock(s, o, ocap))[1 + pos] = make_uint2(v, u);
  } else {
    const uint32_t q = (s ? spbase[1] : spbase[0]) + atomicAdd(&K.sp[s], 1u);
    if (q < V.spill_cap) V.spill[s][s ? lst[1] : lst[0]][q] = make_uint2(v, u);  // past it: Ctl::lost (plan_round)
  }
}

// The expansion of a small round by block (0, 0): both sides' frontiers
// staged in LDS (side 0's vertices, then side 1's), one degree prefix, and
// passes of kSmallU edges per thread (all their loads in flight together).
// Stage both sides' frontiers (and the round's state words) into S, threads
// t of nt.  valid = 0 when a frontier is above kSmallV on this rank (possible
// for a side that does not expand this round): small_expand then stages the
// expanding sides itself.
__device__ void small_prefetch(const DView& V, const uint32_t* fr, SmallStage& S, uint32_t t, uint32_t nt) {
  const uint32_t n0 = fr[2] - fr[0], n1 = fr[3] - fr[1];
  const uint32_t valid = n0 <= kSmallV && n1 <= kSmallV;
  if (t == 0) {
    S.n0 = n0;
    S.nv = n0 + n1;
    S.valid = valid;
  }
  if (!valid) return;
  const DState* st = V.st;
  if (t < 2) {
    const uint32_t cur = st->spill_cur[t];
    S.qbase[t] = st->qtail[t];
    S.lst[t] = cur;
    S.spbase[t] = st->spill_n[t][cur];
  }
  for (uint32_t i = t; i < n0 + n1; i += nt) {
    const int s = i >= n0;
    const uint32_t u = pick(V.queue, s)[fr[s] + (s ? i - n0 : i)];
    const uint32_t li = u - V.lo;
    const unsigned long long b = V.row_off[li];
    S.su[i] = u;
    S.sb[i] = b;
    S.se[i] = (uint32_t)(V.row_off[li + 1] - b);
  }
}

// pipe: the round's exchange also carries this rank's reduction header.
__device__ void small_expand(const DView& V, const Ctl& c, uint32_t it, uint32_t ocap, const uint32_t* fr,
                             SmallStage& S, RoundStamp* rs, int pipe) {
  __shared__ SmallCtr K;
  uint32_t* const su = S.su;
  unsigned long long* const sb = S.sb;
  uint32_t* const se = S.se;
  const uint32_t tid = threadIdx.x;
  const int p = it & 1;
  DState* st = V.st;
  const uint32_t mine_sides = c.sides;
  if (!S.valid) {  // (a big idle side): stage the expanding sides only
    const uint32_t F0 = (mine_sides & 1) ? fr[2] - fr[0] : 0u, F1 = (mine_sides & 2) ? fr[3] - fr[1] : 0u;
    if (tid == 0) {
      S.n0 = F0;
      S.nv = F0 + F1;  // <= 2 kSmallV (the plan's vertex bound)
    }
    if (tid < 2) {
      const uint32_t cur = st->spill_cur[tid];
      S.qbase[tid] = st->qtail[tid];
      S.lst[tid] = cur;
      S.spbase[tid] = st->spill_n[tid][cur];
    }
    for (uint32_t i = tid; i < F0 + F1; i += kThreads) {
      const int s = i >= F0;
      const uint32_t u = pick(V.queue, s)[fr[s] + (s ? i - F0 : i)];
      const uint32_t li = u - V.lo;
      const unsigned long long b = V.row_off[li];
      su[i] = u;
      sb[i] = b;
      se[i] = (uint32_t)(V.row_off[li + 1] - b);
    }
    __syncthreads();
  } else {
    // staged during the plan: a side that does not expand keeps its entries
    // with degree 0 (the edge search skips them)
    for (uint32_t i = tid; i < S.nv; i += kThreads)
      if (!((c.sides >> (i >= S.n0 ? 1 : 0)) & 1)) se[i] = 0;
  }
  if (tid < 2) {
    K.q[tid] = 0;
    K.ne[tid] = 0;
    K.sp[tid] = 0;
  }
  if (tid < 2 * kStageRanks) K.oc[tid / kStageRanks][tid % kStageRanks] = 0;
  if (tid == 0) {
    K.best = kNoKey;
    K.found = 0;
  }
  __syncthreads();
  const uint32_t nv = S.nv, F0 = S.n0;
  const uint32_t* const qbase = S.qbase;
  const uint32_t* const spbase = S.spbase;
  const uint32_t* const lst = S.lst;
  small_scan(se, nv);
  if (rs && tid == 0) rs->es = __builtin_amdgcn_s_memrealtime();
  const uint32_t E = se[nv];
  const uint32_t dn[2] = {c.xdepth[0] + 1, c.xdepth[1] + 1};
  const uint32_t dcl[2] = {c.xdepth[1] + 1, c.xdepth[0] + 1};  // (only this round's claims of the other side read kEmpty)
  const bool single = c.sides != 3u;
  for (uint32_t base = 0; base < E; base += kThreads * kSmallU) {  // block-uniform trip count
    uint32_t vv[kSmallU], uu[kSmallU];
    int ss[kSmallU];
    bool ok[kSmallU];
#pragma unroll
    for (int k = 0; k < kSmallU; ++k) {
      const uint32_t e = base + k * kThreads + tid;
      ok[k] = e < E;
      vv[k] = uu[k] = 0;
      ss[k] = 0;
      if (ok[k]) {
        const uint32_t a = lift_search(se, nv, e, lift_top(nv));  // last vertex whose edge range starts at or before e
        ss[k] = a >= F0;
        uu[k] = su[a];
        vv[k] = V.col[sb[a] + (e - se[a])];
      }
    }
    bool own[kSmallU];
    ClaimIn ci[kSmallU];
    uint32_t so[kSmallU];
#pragma unroll
    for (int k = 0; k < kSmallU; ++k) {  // every item's claim / offer atomic in flight together
      own[k] = ok[k] && vv[k] >= V.lo && vv[k] < V.hi;
      small_claim_issue(V, own[k], ss[k], vv[k], ci[k]);
      so[k] = small_emit_issue(V, ok[k] && !own[k], ss[k], vv[k]);
    }
#pragma unroll
    for (int k = 0; k < kSmallU; ++k) {
      small_claim(V, K, qbase, own[k], ss[k], vv[k], uu[k], dn, dcl, single, ci[k]);
      small_emit(V, K, spbase, lst, ok[k] && !own[k], ss[k], vv[k], uu[k], ocap, so[k]);
    }
  }
  __syncthreads();
  if (rs && tid == 0) rs->ex = __builtin_amdgcn_s_memrealtime();
  // owner headers (count capped to the block), the reduction headers of a
  // pipelined round, the round's state
  for (uint32_t t = tid; t < 2u * V.P; t += kThreads) {
    const uint32_t s = t / V.P, o = t % V.P;
    const uint32_t cnt = K.oc[s][o];
    V.sendbuf[oblock((int)s, o, ocap)] = min(cnt, ocap);
    if (cnt) atomicMax(&st->ocmax, cnt);
  }
  if (pipe) write_peer_headers(V, ocap, it, spbase[0] + K.sp[0], spbase[1] + K.sp[1]);
  if (tid == 0) {
    for (int s = 0; s < 2; ++s) {
      st->qtail[s] = qbase[s] + K.q[s];
      st->new_edges[s] += K.ne[s];
      st->spill_n[s][lst[s]] = spbase[s] + K.sp[s];
    }
    if (K.found) st->meet_found = 1;
    if (K.best != kNoKey) atomicMin(&V.red[p].meetkey, K.best);
  }
}

// The claims of a small round by block (0, 0) of k_spec_claim: every sender's
// block of both sides, then the round's end (spec_round_end's bookkeeping,
// from the LDS counters -- one thread, plain accesses).
__device__ void small_claim_round(const DView& V, const Ctl& c, uint32_t it, uint32_t cap, RoundStamp* rs, int pipe,
                                  const PeerTab& pt) {
  __shared__ uint32_t cnt[2 * kStageRanks + 1];
  __shared__ SmallCtr K;
  __shared__ uint32_t qbase[2], fend0[2], spn[2], ocm;
  __shared__ unsigned long long ne0[2];
  const uint32_t tid = threadIdx.x;
  const int p = it & 1;
  const int P = V.P;
  DState* st = V.st;
  if (pipe) scatter_peer_headers(V, cap, it, pt);
  if (tid < 2) {
    qbase[tid] = st->qtail[tid];
    K.q[tid] = 0;
    K.ne[tid] = 0;
  } else if (tid >= kWave && tid < kWave + 2) {  // the round end's inputs, loaded up front
    const uint32_t s = tid - kWave;
    ne0[s] = st->new_edges[s];
    fend0[s] = st->fend[s];
    spn[s] = st->spill_n[s][st->spill_cur[s]];
  } else if (tid == kWave + 2) {
    ocm = st->ocmax;
  }
  if (tid == 0) {
    K.best = kNoKey;
    K.found = 0;
  }
  // item space: side 0's P blocks, then side 1's (a side that did not expand: 0)
  if (tid < 2u * P) {
    const uint32_t s = tid / P;
    cnt[tid] = ((c.sides >> s) & 1) ? min(peer_at(V, pt, tid % P, cap)[pblock((int)s, cap)], cap) : 0u;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t run = 0;
    for (int k = 0; k < 2 * P; ++k) {
      const uint32_t x = cnt[k];
      cnt[k] = run;
      run += x;
    }
    cnt[2 * P] = run;
  }
  __syncthreads();
  const uint32_t tot = cnt[2 * P];
  const uint32_t dn[2] = {c.xdepth[0] + 1, c.xdepth[1] + 1};
  const uint32_t dcl[2] = {((c.sides >> 1) & 1) ? c.xdepth[1] + 1 : c.xdepth[1],
                           (c.sides & 1) ? c.xdepth[0] + 1 : c.xdepth[0]};
  const bool single = c.sides != 3u;
  for (uint32_t base = 0; base < tot; base += kThreads * kSmallU) {
    uint2 x[kSmallU];
    int ss[kSmallU];
    bool ok[kSmallU];
#pragma unroll
    for (int k = 0; k < kSmallU; ++k) {
      const uint32_t i = base + k * kThreads + tid;
      ok[k] = i < tot;
      ss[k] = 0;
      x[k] = make_uint2(0, 0);
      if (ok[k]) {
        const uint32_t a = lift_search(cnt, 2 * P, i, lift_top(2 * P));  // the block holding item i
        ss[k] = (int)(a / P);
        x[k] = reinterpret_cast<const uint2*>(peer_at(V, pt, a % P, cap) + pblock((int)(a / P), cap))[1 + (i - cnt[a])];
      }
    }
    bool want[kSmallU];
    ClaimIn ci[kSmallU];
#pragma unroll
    for (int k = 0; k < kSmallU; ++k) {  // every item's claim atomic in flight together
      want[k] = ok[k] && x[k].x >= V.lo && x[k].x < V.hi;
      small_claim_issue(V, want[k], ss[k], x[k].x, ci[k]);
    }
#pragma unroll
    for (int k = 0; k < kSmallU; ++k) small_claim(V, K, qbase, want[k], ss[k], x[k].x, x[k].y, dn, dcl, single, ci[k]);
  }
  __syncthreads();
  if (rs && tid == 0) rs->cx = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {  // spec_round_end from the LDS counters (no continuation in a small round)
    for (int s = 0; s < 2; ++s) {
      const bool on = (c.sides >> s) & 1;
      const uint32_t qt = qbase[s] + K.q[s];
      const unsigned long long ne = ne0[s] + K.ne[s];
      st->qtail[s] = qt;
      st->new_edges[s] = 0;
      V.red[p].sums[2 * s] = on ? (unsigned long long)(qt - fend0[s]) : 0ull;
      V.red[p].sums[2 * s + 1] = on ? ne : 0ull;
      V.red[p].nfmax[s] = on ? ~ne : ~0ull;
      if (on) {
        st->fbeg[s] = fend0[s];
        st->fend[s] = qt;
      }
      const unsigned long long sp = on ? spn[s] : 0ull;
      V.red[p].spill[s] = sp;
      V.red[p].spillmax[s] = (uint32_t)min(sp, 0xffffffffull);
      st->hub_count[s] = 0;
    }
    if (K.found) st->meet_found = 1;
    V.red[p].nocmax = ~(unsigned long long)ocm;
    st->ocmax = 0;
    V.red[p].meetkey = min(V.red[p].meetkey, K.best);
    V.red[p ^ 1].meetkey = kNoKey;
  }
}

// Edge-parallel expansion of the deferred hubs.  side >= 0: that side (a
// host-planned round, depth dnew, blocks of V.cap pairs); side < 0: both
// sides of speculative round `it` (blockIdx.y = side, blocks of `cap` pairs)
// and the last block writes the candidate headers.  Every block stages a tile
// of hubs with their degree prefix in LDS and walks the tile's flattened edge
// range with a grid stride, so each hub's edges spread over all CUs.
__global__ __launch_bounds__(kThreads) void k_td_hubs(DView V, uint32_t it, int side, uint32_t dnew_fixed,
                                                      uint32_t cap, int single, int finish, uint32_t ocap, int pipe) {
  __shared__ uint32_t hu[kHubTile];
  __shared__ unsigned long long hb[kHubTile], hp[kHubTile + 1];
  __shared__ unsigned long long wsum[kThreads / kWave];
  const int s = side >= 0 ? side : (int)blockIdx.y;
  uint32_t sides = 1u << s, dnew = dnew_fixed;
  if (side < 0) {
    const Ctl& c = V.ctl[it & 1];
    if (c.state == kDone || c.state == kDead) return;  // past the end of the search (k_spec_expand)
    sides = c.sides;
    dnew = c.xdepth[s] + 1;
  }
  const uint32_t H = V.st->hub_count[s];
  uint2* pairs = reinterpret_cast<uint2*>(V.sendbuf + s * block_words(cap)) + 1;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wid = tid / kWave;
  const bool exit_on_meet = side < 0 ? sides != 3u : single != 0;
  ClaimMeet cm;  // speculative rounds detect meets at claim time; host rounds in k_meet_end
  cm.single = exit_on_meet;
  OwnerEmit oe;
  if (side < 0) {
    cm.meetkey = &V.red[it & 1].meetkey;
    cm.dclaim = V.ctl[it & 1].xdepth[s ^ 1] + 1;
    if (ocap) {  // (a continuation round has no hubs: the expanding side's list)
      const uint32_t cur = V.st->spill_cur[s];
      oe.cap = ocap;
      oe.bw = (uint32_t)block_words(ocap);
      oe.spill = V.spill[s][cur];
      oe.spill_n = &V.st->spill_n[s][cur];
    }
  }
  __shared__ uint32_t sstop;
  if ((sides >> s) & 1) {
    for (uint32_t t0 = 0; t0 < H; t0 += kHubTile) {
      if (exit_on_meet) {  // block-uniform
        if (tid == 0) sstop = meet_seen(V) ? 1u : 0u;
        __syncthreads();
        if (sstop) break;
      }
      const uint32_t nt = min((uint32_t)kHubTile, H - t0);
      constexpr int kPer = kHubTile / kThreads;  // hubs per thread for the scan
      unsigned long long d[kPer], run = 0;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t j = tid * kPer + k;
        d[k] = 0;
        if (j < nt) {
          const uint32_t u = pick(V.hubs, s)[t0 + j], li = u - V.lo;
          const unsigned long long b = V.row_off[li];
          d[k] = V.row_off[li + 1] - b;
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
      for (int k = 0; k < kThreads / kWave; ++k) {
        pre += k < wid ? wsum[k] : 0ull;
        tot += wsum[k];
      }
      unsigned long long e0 = pre + x - run;
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        hp[tid * kPer + k] = e0;
        e0 += d[k];
      }
      if (tid == 0) hp[kHubTile] = tot;
      __syncthreads();
      uint32_t iter = 0;
      for (unsigned long long base = (unsigned long long)blockIdx.x * kThreads; base < tot;
           base += (unsigned long long)gridDim.x * kThreads, ++iter) {
        if (exit_on_meet && iter > 0 && __builtin_amdgcn_readfirstlane(meet_seen(V) ? 1u : 0u)) break;
        const unsigned long long e = base + tid;
        const bool valid = e < tot;
        uint32_t uu = 0, v = 0;
        if (valid) {
          const uint32_t a = lift_search(hp, nt, e, lift_top(nt));  // last hub whose edge range starts at or before e
          uu = hu[a];
          v = V.col[hb[a] + (e - hp[a])];
        }
        const bool own = valid && v >= V.lo && v < V.hi;
        wave_claim(V, s, own, v, uu, dnew, cm);
        wave_emit(V, s, valid && !own, v, uu, pairs, cap, oe);
      }
      __syncthreads();
    }
  }
  if (side >= 0) return;
  if (finish) drain_atomics();
  if (last_block(&V.st->done_blocks[2], gridDim.x * gridDim.y)) {
    if (ocap) {
      write_owner_headers(V, ocap, it, pipe);
      if (threadIdx.x == 0) atomicExch(&V.st->done_blocks[2], 0u);
    } else if (threadIdx.x < 2) {
      const int ss = threadIdx.x;
      const uint32_t cnt = atomicExch(&V.st->send_count[ss], 0u);
      V.sendbuf[ss * block_words(cap)] = ((sides >> ss) & 1) ? min(cnt, cap) : 0u;
      if (ss == 0) atomicExch(&V.st->done_blocks[2], 0u);
    }
    if (finish && threadIdx.x == kWave) spec_round_end(V, it, sides, V.ctl[it & 1].cont);
    if (RoundStamp* rs = round_stamp(V, it)) {  // the hub pass ends the round's expansion
      __syncthreads();
      if (threadIdx.x == 0) rs->ee = __builtin_amdgcn_s_memrealtime();
    }
  }
}

// Pipelined rounds: plan round it + 1 in the claim kernel of round it (one
// block; see k_spec_claim) and publish it as k_spec_expand would.
__device__ void plan_next_round(const DView& V, uint32_t it, uint32_t cap, const Policy& pol, uint32_t plan_cap,
                                const PeerTab& pt) {
  constexpr uint32_t kRedW = sizeof(Reduced) / 4;
  __shared__ Ctl prev, c;
  __shared__ Reduced rd;
  __shared__ uint32_t gw[kStageRanks * kRedW];
  stage_words(&prev, &V.ctl[it & 1], sizeof(Ctl));
  for (uint32_t t = threadIdx.x; t < (uint32_t)V.P * kRedW; t += blockDim.x)
    gw[t] = peer_at(V, pt, t / kRedW, cap)[t % kRedW];
  __syncthreads();
  if (threadIdx.x == 0) {
    reduce_gathered(reinterpret_cast<const Reduced*>(gw), V.P, rd);
    plan_round(prev, rd, pol, plan_cap, kPlanPipe, c);
  }
  __syncthreads();
  if (threadIdx.x < kWave) publish_plan(V, it + 1, pol, prev, rd, c, 1);
}

// Post phase of both sides: owners claim the candidates addressed to them
// (rank r's side-s block at recvbuf + oblock(s, r, cap)).
// (more than one rank: this kernel ends the round's claims; its last
// workgroup closes the round.  pipe: block (0, 0) also moves the reduction
// headers the exchange carried into the gathered slot of round it - 1.)
__global__ __launch_bounds__(kThreads) void k_spec_claim(DView V, uint32_t it, uint32_t cap, int pipe, Policy pol,
                                                         uint32_t plan_cap, PeerTab pt, DevSync ds) {
  unsigned long long t_in = __builtin_amdgcn_s_memrealtime();
  if (ds.epoch) {  // (the stamps count the wait as exchange)
    if (!dev_sync_block(ds)) return;  // a wait that ran out: the host throws
    t_in = __builtin_amdgcn_s_memrealtime();
  }
  if (pipe && blockIdx.x == gridDim.x - 1) {
    // Pipelined rounds: the extra block plans round it + 1 while the others
    // claim round it -- its inputs (this round's plan, every rank's reduction
    // of round it - 1 in the exchange's headers) are all here, and the claims
    // do not change them -- so the next expansion starts with its plan ready.
    if (blockIdx.y == 0) plan_next_round(V, it, cap, pol, plan_cap, pt);
    return;
  }
  const Ctl& c = V.ctl[it & 1];
  if (c.state == kDone || c.state == kDead) return;  // past the end of the search (k_spec_expand)
  RoundStamp* rs = round_stamp(V, it);
  if (rs && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) rs->cb = t_in;
  if (small_claim_ok(c, V.P)) {  // small round: one workgroup claims and closes it
    if (blockIdx.x == 0 && blockIdx.y == 0) {
      if (rs && threadIdx.x == 0) rs->small |= 2u;
      small_claim_round(V, c, it, cap, rs, pipe, pt);
      if (rs) {
        __syncthreads();
        if (threadIdx.x == 0) rs->ce = __builtin_amdgcn_s_memrealtime();
      }
    }
    return;
  }
  const int s = blockIdx.y;
  if (pipe && blockIdx.x == 0 && s == 0) scatter_peer_headers(V, cap, it, pt);
  const uint32_t nbx = gridDim.x - (pipe ? 1u : 0u);  // the claiming blocks (pipelined: not the planner's column)
  // a continuation side claims at the depth its level already has
  const uint32_t dnew = ((c.sides >> s) & 1) ? c.xdepth[s] + 1 : c.xdepth[s];
  ClaimMeet cm;
  cm.meetkey = &V.red[it & 1].meetkey;
  cm.dclaim = ((c.sides >> (s ^ 1)) & 1) ? c.xdepth[s ^ 1] + 1 : c.xdepth[s ^ 1];
  cm.single = c.sides != 3u;
  for (int r = 0; (((c.sides | c.cont) >> s) & 1) && r < V.P; ++r) {  // block-uniform
    const uint32_t* b = peer_at(V, pt, (uint32_t)r, cap) + pblock(s, cap);
    const uint32_t cnt = min(b[0], cap);
    const uint2* pr = reinterpret_cast<const uint2*>(b) + 1;
    for (uint64_t base = (uint64_t)blockIdx.x * kThreads; base < cnt; base += (uint64_t)nbx * kThreads) {
      const uint64_t i = base + threadIdx.x;
      bool want = false;
      uint32_t v = 0, u = 0;
      if (i < cnt) {
        const uint2 x = pr[i];
        v = x.x;
        u = x.y;
        want = v >= V.lo && v < V.hi;
      }
      wave_claim(V, s, want, v, u, dnew, cm);
    }
  }
  drain_atomics();
  if (last_block(&V.st->done_blocks[1], nbx * gridDim.y) && threadIdx.x == 0) {
    spec_round_end(V, it, c.sides, c.cont);
    atomicExch(&V.st->done_blocks[1], 0u);
    if (rs) rs->ce = __builtin_amdgcn_s_memrealtime();
  }
}

// Meet check over the vertices each expanded side claimed this round (one the
// other side also holds closes a path of length dnew + depth_other(v)), then
// -- last block -- the round's bookkeeping: publish the per-side counts for
// the reduction and advance the frontiers.
__global__ __launch_bounds__(kThreads) void k_meet_end(DView V, uint32_t it) {
  const int p = it & 1;
  const uint32_t sides = V.ctl[p].sides;
  DState* st = V.st;
  const uint32_t f0 = st->fend[0], f1 = st->fend[1];
  const uint32_t n0 = (sides & 1) ? st->qtail[0] - f0 : 0u;
  const uint32_t n1 = (sides & 2) ? st->qtail[1] - f1 : 0u;
  unsigned long long best = kNoKey;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (uint64_t)n0 + n1;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const int s = i < n0 ? 0 : 1;
    const uint32_t v = pick(V.queue, s)[s ? f1 + (uint32_t)(i - n0) : f0 + (uint32_t)i];
    const uint32_t li = v - V.lo;
    if ((pick(V.vis, s ^ 1)[2 * (li >> 5)] >> (li & 31)) & 1u) {
      const unsigned long long key =
          ((unsigned long long)(V.ctl[p].depth[s] + 1 + pick(V.depth, s ^ 1)[li]) << 32) | v;
      best = key < best ? key : best;
    }
  }
#pragma unroll
  for (int o = kWave / 2; o >= 1; o >>= 1) {
    const unsigned long long y = __shfl_xor(best, o);
    best = y < best ? y : best;
  }
  if (__lane_id() == 0 && best != kNoKey) atomicMin(&V.red[p].meetkey, best);
  if (last_block(&st->done_blocks[1], gridDim.x) && threadIdx.x == 0) {
    for (int s = 0; s < 2; ++s) {
      const bool on = (sides >> s) & 1;
      const uint32_t qt = atomicAdd(&st->qtail[s], 0u);
      const unsigned long long ne = atomicExch(&st->new_edges[s], 0ull);
      V.red[p].sums[2 * s] = on ? (unsigned long long)(qt - st->fend[s]) : 0ull;
      V.red[p].sums[2 * s + 1] = on ? ne : 0ull;
      V.red[p].nfmax[s] = on ? ~ne : ~0ull;
      if (on) {
        st->fbeg[s] = st->fend[s];
        st->fend[s] = qt;
      }
      st->hub_count[s] = 0;
      V.red[p].spill[s] = 0;  // host-planned exchanges are sized exactly: nothing spills
      V.red[p].spillmax[s] = 0;
    }
    V.red[p].nocmax = ~0ull;
    atomicExch(&st->done_blocks[1], 0u);
  }
}

// Account the last enqueued round and publish Ctl to the host (pinned).
// flags = kPlanAccountOnly, or kPlanStall to also plan the next round for the host.
// Writes the accounted Ctl to pinned host memory, then `tag` into the pinned
// word the host spins on (no stream query on the host side).
__global__ void k_final(DView V, uint32_t it, Policy pol, Ctl* host, int flags, uint32_t* fin, uint32_t tag) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int p = it & 1;
  Ctl c;
  Reduced rd;
  // (a drain: the pending round's reduction came with the stalled round's
  // exchange, into the gathered slot of round it - 2)
  const bool drain = (flags & kPlanDrain) != 0;
  reduce_gathered(drain ? V.redg[p] : V.redg[p ^ 1], V.P, rd);
  plan_round(V.ctl[p ^ 1], rd, pol, 0, flags, c);
  c.ticks = __builtin_amdgcn_s_memrealtime() - V.st->t0;
  publish(V, p, V.ctl[p ^ 1], rd, c, drain ? 2 : 0);
  V.red[p ^ 1].meetkey = kNoKey;  // read; it is the buffer of the next round (it + 1)
  *host = c;
  __threadfence_system();
  __hip_atomic_store(fin, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// End-of-stream marker for DistBiBfs::Impl::wait: everything before it in the
// stream has completed (and its writes are visible) once the host sees `tag`.
__global__ void k_host_tag(uint32_t* fin, uint32_t tag) {
  if (threadIdx.x != 0) return;
  __threadfence_system();
  __hip_atomic_store(fin, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ---- host-planned round kernels ---------------------------------------------

// Execute the stalled plan (sizes were chosen by the host from exact bounds).
__global__ void k_plan_force(DView V, uint32_t it, Policy pol) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int p = it & 1;
  Ctl c;
  Reduced rd;
  reduce_gathered(V.redg[p ^ 1], V.P, rd);
  plan_round(V.ctl[p ^ 1], rd, pol, 0, kPlanForce, c);
  publish(V, p, V.ctl[p ^ 1], rd, c);
  V.red[p].meetkey = kNoKey;
}

__global__ __launch_bounds__(kThreads) void k_td_expand(DView V, int s, uint32_t dnew, uint64_t hub_deg,
                                                        int single) {
  ClaimMeet cm;  // host rounds: keys from k_meet_end; the flag only stops a single-side level early
  cm.single = single != 0;
  const uint32_t fb = V.st->fbeg[s];
  td_expand_side(V, s, dnew, reinterpret_cast<uint2*>(V.sendbuf + s * block_words(V.cap)) + 1, V.cap, blockIdx.x,
                 gridDim.x, hub_deg, single != 0, cm, fb, V.st->fend[s] - fb, OwnerEmit{});
}

__global__ void k_send_header(DView V, int s, uint32_t it) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const uint32_t c = V.st->send_count[s];
  V.st->send_count[s] = 0;
  V.sendbuf[s * block_words(V.cap)] = c;
  V.red[it & 1].maxsend[s] = c;
}

// Host-planned post phase: owners claim the candidates addressed to them
// (rank r's block of `per` pairs at recvbuf + s * P * block_words(cap) + r * block_words(per)).
__global__ __launch_bounds__(kThreads) void k_td_claim(DView V, int s, uint32_t per, uint32_t dnew) {
  const uint64_t blk = block_words(per);
  const uint64_t total = (uint64_t)V.P * per;
  const uint32_t* R = V.recvbuf + (uint64_t)s * V.P * block_words(V.cap);
  for (uint64_t base = (uint64_t)blockIdx.x * kThreads; base < total; base += (uint64_t)gridDim.x * kThreads) {
    const uint64_t t = base + threadIdx.x;
    bool want = false;
    uint32_t v = 0, u = 0;
    if (t < total) {
      const uint64_t r = t / per, i = t % per;
      const uint32_t* b = R + r * blk;
      if (i < min(b[0], per)) {
        const uint2 x = reinterpret_cast<const uint2*>(b)[1 + i];
        v = x.x;
        u = x.y;
        want = v >= V.lo && v < V.hi;
      }
    }
    wave_claim(V, s, want, v, u, dnew);
  }
}

// Bottom-up pre phase: this rank's slice of the frontier bitmap.
__global__ void k_obits(DView V, int s) {
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
    const uint32_t word = vis[2 * (gw * 2 + (lane >> 5))];
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
    if (lane == 0) vis[2 * (gw * 2)] = word | (uint32_t)mask;  // this side's half only
    if (lane == 32) vis[2 * (gw * 2 + 1)] = word | (uint32_t)(mask >> 32);
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

// Seeding pseudo-round: roots claimed by their owners; ctl[1] / red[1] hold
// the state round 0 reads.
__global__ void k_seed(DView V, uint32_t src, uint32_t dst) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  DState* st = V.st;
  Reduced& r = V.red[1];
  for (int s = 0; s < 2; ++s) {
    st->fbeg[s] = st->fend[s] = st->qtail[s] = 0;
    st->send_count[s] = 0;
    st->done_blocks[s] = 0;
    st->done_blocks[2] = 0;
    st->hub_count[s] = 0;
    st->new_edges[s] = 0;
    st->meet_found = 0;
    st->spill_n[s][0] = st->spill_n[s][1] = 0;
    st->spill_cur[s] = 0;
    r.spill[s] = 0;
    r.spillmax[s] = 0;
    r.nsp[s] = 0;
    V.red[0].nsp[s] = 0;  // (only exchange headers carry nsp: a gathered copy of red must read 0)
    r.sums[2 * s] = r.sums[2 * s + 1] = 0;
    const uint32_t v = s ? dst : src;
    if (v >= V.lo && v < V.hi) {
      const uint32_t li = v - V.lo;
      pick(V.vis, s)[2 * (li >> 5)] |= 1u << (li & 31);
      pick(V.parent, s)[li] = kEmpty;
      pick(V.depth, s)[li] = 0;
      pick(V.queue, s)[0] = v;
      st->fend[s] = st->qtail[s] = 1;
      r.sums[2 * s] = 1;
      r.sums[2 * s + 1] = V.row_off[li + 1] - V.row_off[li];
    }
  }
  st->t0 = __builtin_amdgcn_s_memrealtime();
  st->ocmax = 0;
  r.nocmax = ~0ull;
  r.meetkey = kNoKey;
  V.red[0].meetkey = kNoKey;  // round 0 detects its meets into red[0]
  Ctl c = {};
  c.dir[0] = c.dir[1] = 1;
  c.state = kRun;
  c.sides = kSeedBit;
  c.key = c.pkey = kNoKey;
  V.ctl[1] = c;
}

// ---- path reconstruction ----------------------------------------------------

// Distributed path check: block b takes the b-th path edge (path[i], path[i+1])
// whose first vertex this rank owns (idx[b] = i) and scans that vertex's row
// for the second one; found[b] = 1 if it is there.
__global__ __launch_bounds__(kThreads) void k_path_edges(DView V, const uint32_t* __restrict__ path,
                                                         const uint32_t* __restrict__ idx, uint32_t* found) {
  const uint32_t i = idx[blockIdx.x];
  const uint32_t u = path[i], v = path[i + 1];
  const uint32_t li = u - V.lo;
  const unsigned long long b = V.row_off[li], e = V.row_off[li + 1];
  int hit = 0;
  for (unsigned long long base = b; base < e; base += kThreads) {  // block-uniform trip count
    const unsigned long long k = base + threadIdx.x;
    const int mine = k < e && V.col[k] == v;
    hit = __syncthreads_or(mine);
    if (hit) break;
  }
  if (threadIdx.x == 0) found[blockIdx.x] = hit ? 1u : 0u;
}

// Pack this rank's claimed (vertex, parent) pairs of both sides: one block of
// {count_S, count_T, S pairs[capS], T pairs[capT]} (the queues hold exactly
// the claimed owned vertices).  Only vertices up to the accounted depths dS /
// dT: a pipelined search ends one round before its last executed round, whose
// claims the final plan has not counted (capS / capT); they sit at the queue's
// end (queues are in level order) and go out as empty pairs the walk skips.
__global__ void k_pack_parents(DView V, uint32_t capS, uint32_t capT, uint32_t dS, uint32_t dT) {
  uint32_t* out = V.sendbuf;
  const uint32_t qn0 = V.st->qtail[0], qn1 = V.st->qtail[1];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    out[0] = min(qn0, capS);
    out[1] = min(qn1, capT);
  }
  uint2* pr = reinterpret_cast<uint2*>(out + 2);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (uint64_t)qn0 + qn1;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const int s = i < qn0 ? 0 : 1;
    const uint32_t k = s ? (uint32_t)(i - qn0) : (uint32_t)i;
    if (k >= (s ? capT : capS)) continue;
    const uint32_t v = pick(V.queue, s)[k];
    const bool acc = pick(V.depth, s)[v - V.lo] <= (s ? dT : dS);
    pr[(s ? capS : 0) + k] = acc ? make_uint2(v, pick(V.parent, s)[v - V.lo]) : make_uint2(kEmpty, kEmpty);
  }
}

// One workgroup: every rank's gathered pairs into two LDS hash tables
// (vertex -> parent, one per side), then the two parent chains from the meet
// vertex.  out (pinned host memory) = {status, dS, dT, stamps, path[hops + 1]};
// status 0 = ok.  Then `tag` into fin, after a system-scope release: the host
// reads the path where the kernel wrote it (no copy, no tag kernel behind).
// k_walk's LDS tables: the CU's 160 KB less its static words (the DevSync flag word)
constexpr uint64_t kWalkSlots = (160 * 1024 - 256) / 8;
__global__ __launch_bounds__(1024) void k_walk(const uint32_t* __restrict__ recv, PeerTab pt, DevSync ds, int P,
                                               uint32_t capS, uint32_t capT, uint32_t slotsS, uint32_t slotsT,
                                               uint32_t meet, uint32_t hops, uint32_t* out, uint32_t* fin,
                                               uint32_t tag) {
  extern __shared__ uint32_t lds[];
  // the device-ordered gather: every rank packed its pairs into its window
  // half of the epoch; wait for the peers' flags, then read them in place
  if (ds.epoch && !dev_sync_block(ds)) return;  // (a wait that ran out: the host throws)
  const unsigned long long t_in = __builtin_amdgcn_s_memrealtime();
  // per-side table base and size as selects, not local arrays indexed by the
  // side (those went to scratch, and the table accesses became flat)
  auto keys = [&](int s) { return s ? lds + 2 * slotsS : lds; };
  auto nslot = [&](int s) { return s ? slotsT : slotsS; };
  // multiply-shift range reduction: any table size, so a ~0.77 load factor
  // fits ~15k (vertex, parent) pairs in 160 KB of LDS
  auto home = [&](int s, uint32_t v) { return (uint32_t)(((uint64_t)(v * 2654435761u) * nslot(s)) >> 32); };
  auto next = [&](int s, uint32_t h) { return h + 1 == nslot(s) ? 0u : h + 1; };
  for (uint32_t i = threadIdx.x; i < slotsS + slotsT; i += blockDim.x) {
    const uint32_t s = i < slotsS ? 0 : 1, k = s ? i - slotsS : i;
    keys(s)[2 * k] = kEmpty;
  }
  __syncthreads();
  const uint64_t blk = 2 + 2 * ((uint64_t)capS + capT);
  // kU pairs per thread loaded before any is inserted: the loads of a pass
  // are in flight together (one pair per iteration left every iteration a
  // dependent global round trip: ~50 us for a G(1M) path at P = 2)
  constexpr int kU = 8;
  for (int r = 0; r < P; ++r) {
    const uint32_t* b = pt.direct ? pt.p[r] : recv + (uint64_t)r * blk;
    const uint32_t c0 = b[0], c1 = b[1];
    const uint2* pr = reinterpret_cast<const uint2*>(b + 2);
    for (uint32_t base = 0; base < c0 + c1; base += kU * blockDim.x) {
      uint2 xs[kU];
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const uint32_t i = base + k * blockDim.x + threadIdx.x;
        xs[k] = i < c0 + c1 ? pr[i < c0 ? i : capS + (i - c0)] : make_uint2(kEmpty, kEmpty);
      }
#pragma unroll
      for (int k = 0; k < kU; ++k) {
        const uint32_t i = base + k * blockDim.x + threadIdx.x;
        const uint2 x = xs[k];
        if (x.x == kEmpty) continue;  // past the count, or claimed after the accounted depth (k_pack_parents)
        const int s = i < c0 ? 0 : 1;
        uint32_t h = home(s, x.x);
        bool placed = false;
        for (uint32_t probe = 0; probe < nslot(s); ++probe) {  // (bounded: a full table ends the walk as not found)
          const uint32_t prev = atomicCAS(&keys(s)[2 * h], kEmpty, x.x);
          if (prev == kEmpty || prev == x.x) {
            placed = true;
            break;
          }
          h = next(s, h);
        }
        if (placed) keys(s)[2 * h + 1] = x.y;
      }
    }
  }
  __syncthreads();
  const unsigned long long t_built = __builtin_amdgcn_s_memrealtime();
  // lanes 0 and 1 of wave 0 walk one side each: the chain lengths, then (with
  // the meet's position known) each side's half of the path
  if (threadIdx.x >= 2) return;
  // out[3]: the phases' 10 ns ticks (tables built | chains walked << 16), for
  // stamped searches; then the release and the tag (lane 0, after both lanes'
  // stores: the fence is the wave's)
  auto stamp = [&] {
    const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
    out[3] = (uint32_t)min(t_built - t_in, 0xffffull) | (uint32_t)min(t_end - t_built, 0xffffull) << 16;
  };
  auto release = [&] {
    __threadfence_system();
    if (threadIdx.x == 0) __hip_atomic_store(fin, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  };
  const int s = (int)threadIdx.x;
  auto parent_of = [&](uint32_t v, bool& ok) -> uint32_t {
    uint32_t h = home(s, v);
    for (uint32_t probe = 0; probe < nslot(s); ++probe) {
      const uint2 kv = reinterpret_cast<const uint2*>(keys(s))[h];  // key and parent in one LDS load
      if (kv.x == v) return kv.y;
      if (kv.x == kEmpty) break;
      h = next(s, h);
    }
    ok = false;
    return kEmpty;
  };
  bool ok = true;
  uint32_t d = 0;
  for (uint32_t v = meet, u; ok && (u = parent_of(v, ok)) != kEmpty && d <= hops; v = u) ++d;
  const uint32_t dx = (uint32_t)__shfl_xor((int)d, 1), okx = (uint32_t)__shfl_xor(ok ? 1 : 0, 1);
  const uint32_t d0 = s ? dx : d, d1 = s ? d : dx;
  if (!ok || !okx || d0 + d1 != hops) {
    if (s == 0) {
      out[0] = 1;
      out[1] = d0;
      out[2] = d1;
      stamp();
    }
    release();
    return;
  }
  uint32_t* path = out + 4;  // src .. meet .. dst; both lanes write the meet at d0
  uint32_t v = meet;
  if (s == 0) {
    for (int i = (int)d0; i >= 0; --i) {
      path[i] = v;
      v = parent_of(v, ok);
    }
    out[0] = 0;
    out[1] = d0;
    out[2] = d1;
    stamp();
  } else {
    for (uint32_t i = d0; i <= hops; ++i) {
      path[i] = v;
      v = parent_of(v, ok);
    }
  }
  release();
}

// One rank owns every vertex: the two parent chains are walked straight from
// the local parent arrays (two lanes, one dependent load per hop) and the
// result goes to pinned host memory, then `tag` -- no pack, gather or copy.
// out = {status, dS, dT, pad, path[hops + 1]} as k_walk.
__global__ void k_walk_local(DView V, uint32_t meet, uint32_t hops, uint32_t* out, uint32_t* fin, uint32_t tag) {
  const uint32_t s = threadIdx.x;
  if (s < 2) {
    const uint32_t li = meet - V.lo;
    const uint32_t d0 = V.depth[0][li], d1 = V.depth[1][li];
    bool ok = d0 != kEmpty && d1 != kEmpty && d0 + d1 == hops;
    if (ok) {  // a parent outside the owned range (never, on a consistent state) stops the walk
      uint32_t v = meet;
      if (s == 0) {
        for (int i = (int)d0; i >= 0 && ok; --i) {
          out[4 + i] = v;
          if (i) v = V.parent[0][v - V.lo];
          ok = !i || (v >= V.lo && v < V.hi);
        }
      } else {
        for (uint32_t i = d0; i <= hops && ok; ++i) {
          out[4 + i] = v;
          if (i < hops) v = V.parent[1][v - V.lo];
          ok = i == hops || (v >= V.lo && v < V.hi);
        }
      }
    }
    const bool okx = __shfl_xor(ok ? 1 : 0, 1) != 0;
    if (s == 0) {
      out[0] = ok && okx ? 0u : 1u;
      out[1] = d0;
      out[2] = d1;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(fin, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Fallback for very large visited sets: the owner of the meet vertex
// contributes its two depths (others ~0, min-reduced) ...
__global__ void k_meet_depth(DView V, uint32_t meet, uint32_t it) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const bool own = meet >= V.lo && meet < V.hi;
  V.red[it & 1].md[0] = own ? V.depth[0][meet - V.lo] : kEmpty;
  V.red[it & 1].md[1] = own ? V.depth[1][meet - V.lo] : kEmpty;
}

// ... and one step per hop: cur[q] -> its parent (only the owner knows it; the
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
// in the queues: no O(N) clear of the owned slices) and the `sent` bitmaps
// (2 x N/8 bytes, streamed as 16-byte stores), in one launch.
__global__ void k_cleanup(DView V, uint64_t sent_words) {
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, nth = (uint64_t)gridDim.x * blockDim.x;
  for (int s = 0; s < 2; ++s) {
    const uint32_t qn = V.st->qtail[s];
    const uint32_t* q = pick(V.queue, s);
    uint32_t* vis = pick(V.vis, s);
    uint32_t* dep = pick(V.depth, s);
    for (uint64_t i = tid; i < qn; i += nth) {
      const uint32_t li = q[i] - V.lo;
      vis[2 * (li >> 5)] = 0u;
      dep[li] = kEmpty;  // claim-time meet detection reads kEmpty as "not visible yet"
    }
  }
  uint4* sw = reinterpret_cast<uint4*>(V.sent[0]);  // both sides, contiguous, 256-B aligned
  for (uint64_t i = tid; i < sent_words / 4; i += nth) sw[i] = make_uint4(0, 0, 0, 0);
  for (uint64_t i = sent_words / 4 * 4 + tid; i < sent_words; i += nth) V.sent[0][i] = 0u;
}

unsigned blocks_for(uint64_t work, int cus) {
  uint64_t b = (work + kThreads - 1) / kThreads;
  b = std::min<uint64_t>(b, (uint64_t)cus * 8);
  return (unsigned)std::max<uint64_t>(b, 1);
}

uint32_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x && p < (1ull << 31)) p <<= 1;
  return (uint32_t)p;
}

}  // namespace

std::vector<uint8_t> dist_unique_id(const std::string& backend) {
  if (backend == "ipc") return dist::ipc_unique_id();
  BIBFS_REQUIRE(backend == "rccl", "dist: backend must be rccl or ipc, got " + backend);
  return dist::rccl_unique_id();
}

int gpu_count() {
  int n = 0;
  return hipGetDeviceCount(&n) == hipSuccess ? n : 0;
}

// An error every rank raises at the same point of the same search (decided
// from reduced values), with no collective outstanding: it does not abort
// the communicator, and the next search runs normally.
struct ConsistentError : Error {
  using Error::Error;
};

struct DistBiBfs::Impl {
  int rank = 0, size = 1, device = 0, cus = 256;
  hipStream_t stream = nullptr;   // compute: pre phases of host-planned rounds, graph build
  hipStream_t cstream = nullptr;  // comm: everything of speculative rounds, exchanges, post phases
  hipEvent_t ev_pre[2] = {nullptr, nullptr};
  hipEvent_t ev_round = nullptr;
  hipEvent_t ev_t0 = nullptr, ev_t1 = nullptr;  // timing events around a search
  std::unique_ptr<dist::Comm> comm;
  uint32_t n = 0, lo = 0, hi = 0, chunk = 0, gwords = 0, cap_alloc = 0;
  uint32_t block_cap = 0;  // pairs per candidate block the send buffer holds (per side)
  uint64_t m_input = 0, nnz = 0;
  uint64_t* d_row_off = nullptr;
  uint32_t* d_col = nullptr;
  uint4* d_padj = nullptr;  // one rank: packed adjacency (DView::padj)
  void* state = nullptr;
  size_t state_bytes = 0, padj_bytes = 0;
  // Everything this rank holds on the device goes through `mem` (devmem.hpp):
  // exact current / peak bytes of the build (temporaries included), the
  // device's free-memory low-water mark beside it, and DistTuning::hbm_cap_bytes.
  devmem::Tracker mem;
  size_t gen_hbm_peak_bytes = 0;  // hipMemGetInfo: free before the build - least free during it
  // path reconstruction buffers: O(path length), grown on demand (never O(n))
  uint32_t* d_pathbuf = nullptr;
  size_t path_cap = 0;            // entries per path array (pathS, pathT, and a third behind them)
  uint32_t* sent_base = nullptr;  // both sides' sent bitmaps, contiguous (one memset)
  DView V{};
  uint32_t* d_cur = nullptr;
  uint32_t* d_pathS = nullptr;
  uint32_t* d_pathT = nullptr;
  RoundRec* d_trace = nullptr;
  RoundStamp* d_rstamp = nullptr;
  Reduced* h_red = nullptr;    // pinned
  Ctl* h_ctl = nullptr;        // pinned, written by k_final
  uint32_t* h_fin = nullptr;   // pinned, k_final's tag (written after h_ctl)
  uint32_t* h_abort = nullptr; // pinned: 1 = the host gave up (DevSync waits leave)
  // the device-ordered exchange (DistTuning::dev_sync): the window, the size
  // of one half, and the epoch of the last round / barrier that used it
  dist::Comm::Window win{};
  bool win_ok = false;
  size_t win_half = 0;
  unsigned long long dev_epoch = 0;
  DevSync dev_sync(unsigned long long e) const {
    DevSync d{};
    for (int r = 0; r < size; ++r)
      d.peer_flag[r] = static_cast<const unsigned long long*>(win.peer[r]);
    d.flag = static_cast<unsigned long long*>(win.mine);
    d.epoch = e;
    d.limit = (unsigned long long)(std::max(0.1, tune.timeout_s) * 1e8);  // (s_memrealtime: 100 MHz)
    d.h_abort = h_abort;
    d.P = size;
    return d;
  }
  // a host wait that gives up releases the device waits too
  void give_up() {
    if (h_abort) __atomic_store_n(h_abort, 1u, __ATOMIC_RELEASE);
  }
  uint32_t fin_seq = 0;
  uint64_t* h_plan = nullptr;  // pinned plan ring (k_spec_expand)
  uint64_t* h_aux = nullptr;   // pinned: per-round largest per-owner candidate count
  uint32_t* h_walk = nullptr;  // pinned
  size_t h_walk_cap = 0;
  uint32_t epoch = 0;          // searches run (Policy::epoch)
  double* d_scalar = nullptr;
  unsigned long long* d_stamps = nullptr;  // k_spec_solo<true> phase cycles
  bool solo_stamp = false;
  DistLevelStats stats;
  DistTuning tune;
  bool source_only = false;  // the search in progress is search_unidirectional's
  bool pipe_off = false;     // the search in progress runs exact plans (a pipelined attempt overflowed)
  // World size 1 (DistTuning::world1_single): the rank's shard is the whole
  // graph, so queries go to the single-GPU engine over the same device CSR
  // (adopted, not copied) with its resident server; the partitioned rounds
  // (solo workgroup, speculative rounds) serve search_unidirectional and
  // world1_single = false.
  std::unique_ptr<HipBiBfs> single;
  void ensure_single() {
    if (single || !d_row_off) return;
    auto eng = std::make_unique<HipBiBfs>(device);
    eng->adopt_device_csr(n, nnz, m_input, d_row_off, d_col);
    // the cap is checked before the resident server starts and before the
    // engine is kept: a caller that catches the error holds no engine over it
    check_single_cap(*eng);
    eng->set_resident(true);
    single = std::move(eng);
  }
  int fault_at = 0, fault_mode = 0;

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
    HIP_CHECK(hipEventCreate(&ev_t0));
    HIP_CHECK(hipEventCreate(&ev_t1));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_red), sizeof(Reduced), hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_ctl), sizeof(Ctl), hipHostMallocDefault));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_fin), 64, hipHostMallocDefault));
    std::memset(h_fin, 0, 64);
    h_abort = h_fin + 8;  // (the DevSync abort word shares h_fin's 64 bytes)
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_plan), kPlanRing * 8, hipHostMallocDefault));
    std::memset(h_plan, 0, kPlanRing * 8);
    V.plan_ring = h_plan;
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_aux), kPlanRing * 8, hipHostMallocDefault));
    std::memset(h_aux, 0, kPlanRing * 8);
    V.plan_aux = h_aux;
    V.host_ctl = h_ctl;
    ensure_walk_buf(1u << 14);
    HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(&k_walk),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)(kWalkSlots * 8)));
    if (const char* t = std::getenv("BIBFS_DIST_TIMEOUT_S")) tune.timeout_s = std::max(0.1, std::atof(t));
    comm->set_timeout(tune.timeout_s);
    solo_stamp = env::stamps();  // BIBFS_STAMP: the solo workgroup's phase cycles
    HIP_CHECK(hipMalloc(&d_stamps, 16 * sizeof(unsigned long long)));
  }

  void set_partition(uint32_t nn) {
    n = nn;
    const uint64_t per = ((uint64_t)nn + size - 1) / size;
    chunk = (uint32_t)std::max<uint64_t>(64, (per + 63) / 64 * 64);
    lo = (uint32_t)std::min<uint64_t>((uint64_t)rank * chunk, nn);
    hi = (uint32_t)std::min<uint64_t>((uint64_t)(rank + 1) * chunk, nn);
  }

  size_t row_off_bytes() const { return ((size_t)(hi - lo) + 1) * 8; }
  size_t col_bytes() const { return std::max<uint64_t>(nnz, 1) * 4; }

  void free_all() {
    single.reset();  // (stops its resident server; the CSR it borrowed is freed below)
    devmem::Scope scope(&mem);
    devmem::release(d_row_off, row_off_bytes());
    devmem::release(d_col, col_bytes());
    devmem::release(d_padj, padj_bytes);
    devmem::release(state, state_bytes);
    devmem::release(d_pathbuf, path_cap * 3 * 4 + 64);
    d_row_off = nullptr;
    d_col = nullptr;
    d_padj = nullptr;
    state = nullptr;
    d_pathbuf = nullptr;
    path_cap = 0;
    state_bytes = padj_bytes = 0;
    n = 0;
    nnz = 0;
  }

  // Path buffers for at least `entries` vertices per chain: pathS / pathT of
  // the per-hop walk and k_walk's {status, dS, dT, epoch, path} output.
  void ensure_path_dev(size_t entries) {
    entries += 8;
    if (entries <= path_cap) return;
    devmem::Scope scope(&mem);
    if (d_pathbuf) {
      HIP_CHECK(hipStreamSynchronize(cstream));  // an earlier walk may still read it
      devmem::release(d_pathbuf, path_cap * 3 * 4 + 64);
    }
    path_cap = std::max<size_t>(entries, 1u << 14);
    // three arrays: pathS, pathT, and room behind pathT (validate_path keeps
    // its found flags after the indices there)
    devmem::alloc(&d_pathbuf, path_cap * 3 * 4 + 64);
    d_pathS = d_pathbuf;
    d_pathT = d_pathbuf + path_cap;
  }

  // effective host-planned block capacity (tuning may shrink it for tests)
  uint32_t cap() const {
    return tune.cap ? std::min<uint32_t>(tune.cap, cap_alloc) : cap_alloc;
  }

  void alloc_state() {
    const uint64_t words = chunk / 32;
    gwords = (uint32_t)(((uint64_t)n + 31) / 32 + 1);
    cap_alloc = (uint32_t)std::min<uint64_t>(kCapMax, std::max<uint64_t>(n, 1));
    // blocks must also hold a speculative round's two blocks and the path gather
    block_cap = std::max<uint32_t>(cap_alloc, std::max<uint32_t>(tune.walk_max, kSpecCapMin));
    const uint64_t block = block_words(block_cap);
    size_t off = 0;
    auto take = [&](size_t bytes) {
      size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    size_t o_vis[2], o_par[2], o_dep[2], o_q[2], o_ob[2], o_gb[2], o_hub[2];
    for (int s = 0; s < 2; ++s) {
      o_hub[s] = take((size_t)chunk * 4);
      o_vis[s] = s ? o_vis[0] : take(words * 8);  // interleaved: one allocation for both sides
      o_par[s] = take((size_t)chunk * 4);
      o_dep[s] = take((size_t)chunk * 4);
      o_q[s] = take((size_t)chunk * 4);
      o_ob[s] = take(words * 4);
      o_gb[s] = take(words * 4 * size);
    }
    // send: one block per side, or (owner-addressed rounds) one per side and owner
    // (owner-addressed rounds: per peer a reduction header and two blocks)
    const size_t o_send = take((kHdrWords + 2 * block) * 4 * size), o_recv = take((kHdrWords + 2 * block) * 4 * size);
    const size_t o_ocount = take(2 * (size_t)size * 4);
    size_t o_spill[2][2];
    for (int s = 0; s < 2; ++s)
      for (int l = 0; l < 2; ++l) o_spill[s][l] = take(size > 1 ? (size_t)block_cap * 8 : 8);
    const size_t o_sent = take((size_t)gwords * 4 * 2);
    const size_t o_st = take(sizeof(DState)), o_ctl = take(2 * sizeof(Ctl)), o_red = take(2 * sizeof(Reduced)),
                 o_redg = take(2 * (size_t)size * sizeof(Reduced)),
                 o_cur = take(64), o_sc = take(64),
                 o_tr = take((size_t)kTraceCap * sizeof(RoundRec)),
                 o_rs = take((size_t)kTraceCap * sizeof(RoundStamp));
    {
      devmem::Scope scope(&mem);
      devmem::alloc(&state, off);
      state_bytes = off;
    }
    char* b = static_cast<char*>(state);
    V.n = n;
    V.lo = lo;
    V.hi = hi;
    V.chunk = chunk;
    V.row_off = d_row_off;
    V.col = d_col;
    sent_base = reinterpret_cast<uint32_t*>(b + o_sent);
    for (int s = 0; s < 2; ++s) {
      V.vis[s] = reinterpret_cast<uint32_t*>(b + o_vis[0]) + s;
      V.parent[s] = reinterpret_cast<uint32_t*>(b + o_par[s]);
      V.depth[s] = reinterpret_cast<uint32_t*>(b + o_dep[s]);
      V.queue[s] = reinterpret_cast<uint32_t*>(b + o_q[s]);
      V.hubs[s] = reinterpret_cast<uint32_t*>(b + o_hub[s]);
      V.obits[s] = reinterpret_cast<uint32_t*>(b + o_ob[s]);
      V.gbits[s] = reinterpret_cast<uint32_t*>(b + o_gb[s]);
      V.sent[s] = sent_base + (size_t)s * gwords;
      if (!s) HIP_CHECK(hipMemsetAsync(V.vis[0], 0, words * 8, stream));
      HIP_CHECK(hipMemsetAsync(V.depth[s], 0xff, (size_t)chunk * 4, stream));  // kEmpty
    }
    V.sendbuf = reinterpret_cast<uint32_t*>(b + o_send);
    V.ocount = reinterpret_cast<uint32_t*>(b + o_ocount);
    HIP_CHECK(hipMemsetAsync(V.ocount, 0, 2 * (size_t)size * 4, stream));
    for (int s = 0; s < 2; ++s)
      for (int l = 0; l < 2; ++l) V.spill[s][l] = reinterpret_cast<uint2*>(b + o_spill[s][l]);
    V.spill_cap = size > 1 ? block_cap : 1;
    V.recvbuf = reinterpret_cast<uint32_t*>(b + o_recv);
    HIP_CHECK(hipMemsetAsync(sent_base, 0, (size_t)gwords * 4 * 2, stream));
    V.cap = cap();
    V.P = size;
    V.st = reinterpret_cast<DState*>(b + o_st);
    V.ctl = reinterpret_cast<Ctl*>(b + o_ctl);
    V.red = reinterpret_cast<Reduced*>(b + o_red);
    for (int q = 0; q < 2; ++q)
      V.redg[q] = size == 1 ? V.red + q : reinterpret_cast<Reduced*>(b + o_redg) + (size_t)q * size;
    d_cur = reinterpret_cast<uint32_t*>(b + o_cur);
    ensure_path_dev(1u << 14);
    d_scalar = reinterpret_cast<double*>(b + o_sc);
    d_trace = reinterpret_cast<RoundRec*>(b + o_tr);
    d_rstamp = reinterpret_cast<RoundStamp*>(b + o_rs);
    HIP_CHECK(hipMemsetAsync(d_rstamp, 0, (size_t)kTraceCap * sizeof(RoundStamp), stream));
    V.rstamp = nullptr;
    V.trace = nullptr;
    V.trace_cap = kTraceCap;
    HIP_CHECK(hipMemsetAsync(V.st, 0, sizeof(DState), stream));
    HIP_CHECK(hipMemsetAsync(d_scalar, 0, 64, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    // the device-ordered exchange's window (collective: every rank decides
    // alike): two halves of P owner blocks at the largest speculative block
    if (!win_ok && size > 1 && size <= kStageRanks && tune.dev_sync) {
      const uint32_t smax = std::max<uint32_t>(kSpecCapMin, std::min<uint32_t>(tune.spec_cap_max, block_cap));
      const size_t half = (size_t)peer_words(smax) * 4 * (size_t)size;
      dist::Comm::Window w;
      if (comm->dev_window(dist::Comm::kWinFlagBytes + 2 * half, w)) {
        win = w;
        win_half = half;
        win_ok = true;
      }
    }
  }

  // bytes of the owned CSR shard (row offsets + columns) and the generator's
  // peak allocation while building it (streamed generation: shard + cursor)
  // Largest degree of the whole graph (max over the shards).  No vertex above
  // kHubDeg: no hub is ever deferred, so no speculative round launches the hub pass.
  uint64_t max_deg = 0;
  // One rank owns every row: the packed adjacency of the single-GPU engine
  // (16 B per edge) within BIBFS_PADJ_MAX_MB (default 4096 MiB, 0 = off).
  // G(1M) world-1 query 0.108 -> 0.103 ms (profiles/r3_dist_padj_ab.jsonl).
  bool padj_tried = false;
  void ensure_padj() {
    if (padj_tried) return;
    padj_tried = true;
    if (!(size == 1 && lo == 0 && nnz)) return;
    const uint64_t budget = env::padj_budget_bytes();
    if (nnz * 16 > budget) return;
    devmem::Scope scope(&mem);
    devmem::alloc(&d_padj, nnz * 16);
    padj_bytes = nnz * 16;
    launch::build_padj(d_row_off, d_col, nnz, d_padj, stream);
    HIP_CHECK(hipStreamSynchronize(stream));
    V.padj = d_padj;
  }
  void finish_build() {
    devmem::Scope scope(&mem);
    alloc_state();
    V.padj = nullptr;
    padj_tried = false;
    // world1_single serves the queries from the single-GPU engine, which
    // builds its own packed adjacency: the rounds' one is made only if the
    // partitioned rounds ever run at world size 1 (no duplicate)
    if (!(size == 1 && tune.world1_single)) ensure_padj();
    double y = (double)launch::max_degree(d_row_off, hi - lo, stream);
    if (size > 1) {
      HIP_CHECK(hipMemcpyAsync(d_scalar, &y, 8, hipMemcpyHostToDevice, cstream));
      comm->allreduce(d_scalar, 1, DType::kF64, ROp::kMax, cstream);
      HIP_CHECK(hipMemcpyAsync(&y, d_scalar, 8, hipMemcpyDeviceToHost, cstream));
      wait(cstream);
    }
    max_deg = (uint64_t)y;
    if (size == 1 && tune.world1_single) ensure_single();
  }
  // The adopted single-GPU engine allocates outside devmem (its own arrays;
  // the CSR is this rank's): hold DistTuning::hbm_cap_bytes against
  // everything this rank holds once it exists.
  void check_single_cap(const HipBiBfs& eng) const {
    if (!mem.cap) return;
    const size_t all = eng.device_bytes(), csr = row_off_bytes() + col_bytes();
    const size_t held = mem.cur + (all > csr ? all - csr : 0);
    if (held > mem.cap)
      throw Error("dist: HBM cap exceeded: this rank would hold " + std::to_string(held) + " bytes with the " +
                  "single-GPU engine's arrays (cap " + std::to_string(mem.cap) + ")");
  }
  // Measured, not a formula: the most this rank held at once while its CSR
  // shard was built (generator / scan temporaries included), and the
  // device's free-memory drop over the same span.  Called when the shard is
  // complete, before the search state is allocated (resident_bytes covers
  // everything held afterwards).
  void record_build_peak() {
    gen_peak_bytes = mem.peak;
    gen_hbm_peak_bytes = mem.hbm_peak();
  }

  size_t gen_peak_bytes = 0;
  size_t shard_bytes() const { return ((size_t)(hi - lo) + 1) * 8 + (size_t)nnz * 4; }

  void upload_rows(const Csr& rows) {
    devmem::Scope scope(&mem);
    mem.reset_peak();
    devmem::alloc(&d_row_off, ((size_t)rows.n + 1) * 8);
    devmem::alloc(&d_col, std::max<uint64_t>(rows.nnz(), 1) * 4);
    HIP_CHECK(hipMemcpyAsync(d_row_off, rows.row_off.data(), ((size_t)rows.n + 1) * 8, hipMemcpyHostToDevice,
                             stream));
    if (rows.nnz())
      HIP_CHECK(hipMemcpyAsync(d_col, rows.col.data(), rows.nnz() * 4, hipMemcpyHostToDevice, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    nnz = rows.nnz();
    record_build_peak();
  }

  // Host wait with a watchdog.  A one-lane kernel at the end of the stream
  // writes a tag into pinned memory and the host spins on it: it sees the
  // stream drain one PCIe write after the last kernel instead of at the next
  // hipStreamQuery poll (~10-20 us later on this stack; A/B in
  // profiles/r2_dist_fintag_ab.txt).  An RCCL error reported by the
  // communicator, or no progress within timeout_s (a dead or hung peer leaves
  // our collective waiting forever), aborts the communicator and throws.
  // Largest per-rank frontier (edges) a speculative round may expand before
  // the plan stalls it for the host: one rank exchanges nothing, so nothing
  // bounds it; more ranks' candidates (at most their frontier edges) must fit
  // the spill lists.  DistTuning::spec_stall_edges lowers it (tests force
  // host-planned rounds with it).
  // (from the spill lists' allocation, not V.spill_cap: DistTuning::spill_cap
  // shrinks the lists below what this guard assumes, which is how the tests
  // make a round overflow them)
  uint32_t round_edge_cap() const {
    const uint32_t hard = size == 1 ? 0xFFFFFFFFu : block_cap;
    return tune.spec_stall_edges ? std::min<uint32_t>(tune.spec_stall_edges, hard) : hard;
  }

  uint32_t next_tag() {
    fin_seq = fin_seq + 1 == 0 ? 1 : fin_seq + 1;
    return fin_seq;
  }

  void ensure_walk_buf(size_t words) {
    if (h_walk_cap >= words) return;
    if (h_walk) {  // a round still in flight may write the old buffer
      HIP_CHECK(hipStreamSynchronize(cstream));
      HIP_CHECK(hipHostFree(h_walk));
    }
    h_walk_cap = std::max<size_t>(words, 1u << 14);
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_walk), h_walk_cap * 4, hipHostMallocDefault));
    V.host_walk = h_walk;
  }

  void wait(hipStream_t s) {
    const uint32_t tag = next_tag();
    k_host_tag<<<1, 64, 0, s>>>(h_fin, tag);
    HIP_CHECK(hipGetLastError());
    stats.host_syncs++;
    spin_tag(tag, s);
  }

  void spin_tag(uint32_t tag, hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    const auto deadline = t0 + std::chrono::duration<double>(tune.timeout_s);
    for (uint64_t spin = 0;; ++spin) {
      if (__atomic_load_n(h_fin, __ATOMIC_ACQUIRE) == tag) return;
      if ((spin & 1023) == 1023) {
        const hipError_t e = hipStreamQuery(s);
        if (e != hipSuccess && e != hipErrorNotReady) HIP_CHECK(e);
        if (e == hipSuccess && __atomic_load_n(h_fin, __ATOMIC_ACQUIRE) != tag)
          throw Error("dist: stream drained without its host tag");
        try {
          comm->check();
        } catch (...) {
          give_up();
          throw;
        }
        const auto now = std::chrono::steady_clock::now();
        if (now > deadline) {
          give_up();
          comm->abort();
          throw Error("dist: rank " + std::to_string(rank) + " waited " + std::to_string(tune.timeout_s) +
                      " s for a round (peer failure or hang); communicator aborted");
        }
        if (now - t0 > std::chrono::milliseconds(2)) std::this_thread::sleep_for(std::chrono::microseconds(50));
      }
    }
  }

  // Enqueue k_final and wait for it through its pinned tag: the host sees the
  // accounted Ctl one PCIe write after the kernel ends instead of at the next
  // hipStreamQuery poll.  k_final is the last work in the stream here, so
  // this is a full host sync.  Same watchdog as wait().
  void final_and_wait(uint32_t it, const Policy& pol, int flags, hipStream_t s) {
    const uint32_t tag = next_tag();
    k_final<<<1, 64, 0, s>>>(V, it, pol, h_ctl, flags, h_fin, tag);
    HIP_CHECK(hipGetLastError());
    stats.host_syncs++;
    spin_tag(tag, s);
  }

  // Spin until the device has planned round `need` and return ITS plan word
  // (the per-round ring slot, so every rank stops enqueueing after the same
  // round however far its GPU has progressed).  Same watchdog as wait().
  uint64_t wait_plan(uint32_t need, hipStream_t s) {
    const auto t0 = std::chrono::steady_clock::now();
    const auto deadline = t0 + std::chrono::duration<double>(tune.timeout_s);
    const uint64_t* slot = &h_plan[need % kPlanRing];
    const uint64_t tag = plan_tag(epoch, need);
    for (uint64_t spin = 0;; ++spin) {
      const uint64_t w = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
      if (((w >> 8) & 0xffffffu) == tag) return w;
      if ((spin & 1023) == 1023) {
        const hipError_t e = hipStreamQuery(s);
        if (e == hipSuccess) {  // drained without planning that round: it was never enqueued
          const uint64_t w2 = __atomic_load_n(slot, __ATOMIC_ACQUIRE);
          if (((w2 >> 8) & 0xffffffu) == tag) return w2;
          throw Error("dist: stream drained before round " + std::to_string(need) + " was planned");
        }
        if (e != hipErrorNotReady) HIP_CHECK(e);
        try {
          comm->check();
        } catch (...) {
          give_up();
          throw;
        }
        const auto now = std::chrono::steady_clock::now();
        if (now > deadline) {
          give_up();
          comm->abort();
          throw Error("dist: rank " + std::to_string(rank) + " waited " + std::to_string(tune.timeout_s) +
                      " s for round " + std::to_string(need) + " (peer failure or hang); communicator aborted");
        }
      }
    }
  }

  Policy policy(const SearchOptions& opt) const {
    Policy p;
    p.alpha = opt.alpha;
    p.beta = opt.beta;
    // alpha / beta in 1/256 fixed point, clamped to [0, 4096] (the device
    // products above stay below 2^60).  The single-GPU engine compares in
    // floating point: an alpha or beta that is not a multiple of 1/256 can
    // flip a borderline direction decision between the two engines (never the
    // hop count -- both directions find the same levels).
    auto q8 = [](double x) {
      return (unsigned long long)std::llround(std::min(std::max(x, 0.0), 4096.0) * 256.0);
    };
    p.alpha_q = q8(opt.alpha);
    p.beta_q = q8(opt.beta);
    p.nnz_total = 2 * m_input;
    p.n = n;
    p.lockstep = opt.lockstep ? 1 : 0;
    p.side = (int)opt.side;
    p.direction = (int)opt.direction;
    p.epoch = epoch;
    p.walk_cap = (uint32_t)std::min<size_t>(h_walk_cap, 0xffffffffu);
    p.want_path = opt.want_path ? 1 : 0;
    p.spill_cap = V.spill_cap;
    p.source_only = source_only ? 1 : 0;
    return p;
  }

  void maybe_fault(int it) {
    if (!fault_mode || it < fault_at) return;
    const int mode = fault_mode;
    fault_mode = 0;
    if (mode == 2) std::this_thread::sleep_for(std::chrono::duration<double>(2 * tune.timeout_s));
    if (mode == 3) ::raise(SIGKILL);  // a rank process dies mid-search (multi-process transports)
    throw Error("dist: injected fault on rank " + std::to_string(rank) + " at round " + std::to_string(it));
  }

  SearchResult search(vid_t src, vid_t dst, const SearchOptions& opt);
  void host_round(uint32_t it, const Policy& pol, SearchResult& r);

  // DistTuning::stamps: split the search's speculative rounds (those stamped
  // with this search's tags among rounds [0, it_end)) into kernel time and
  // the gaps between the kernels (exchange + launch latency), in microseconds.
  void collect_stamps(uint32_t it_end) {
    std::vector<RoundStamp> ring(kTraceCap);
    HIP_CHECK(hipMemcpy(ring.data(), d_rstamp, ring.size() * sizeof(RoundStamp), hipMemcpyDeviceToHost));
    const uint32_t lo_it = it_end > kTraceCap ? it_end - kTraceCap : 0;
    const RoundStamp* prev = nullptr;
    uint32_t prev_it = 0;
    auto us = [](unsigned long long a, unsigned long long b) { return b > a ? (double)(b - a) * 1e-2 : 0.0; };
    for (uint32_t i = lo_it; i < it_end; ++i) {
      const RoundStamp& x = ring[i % kTraceCap];
      if (x.tag != plan_tag(epoch, i) || !x.eb || !x.ee) continue;
      stats.stamped_rounds++;
      const unsigned long long ee = x.ee;
      stats.expand_us += us(x.eb, x.ee);
      if (x.cb && x.ce && x.cb >= x.eb) {
        stats.claim_us += us(x.cb, x.ce);
        stats.exchange_us += us(ee, x.cb);
      }
      if (prev && prev_it + 1 == i) stats.status_us += us(prev->ce ? prev->ce : prev->ee, x.eb);
      if (x.small & 1) {
        stats.small_expand_rounds++;
        stats.sx_plan_us += us(x.eb, x.ep);
        stats.sx_staging_us += us(x.eb, x.sg);
        stats.sx_stage_us += us(x.ep, x.es);
        stats.sx_edges_us += us(x.es, x.ex);
        stats.sx_end_us += us(x.ex, x.ee);
      }
      if (x.small & 2) {
        stats.small_claim_rounds++;
        stats.sc_claims_us += us(x.cb, x.cx);
        stats.sc_end_us += us(x.cx, x.ce);
      }
      prev = &x;
      prev_it = i;
    }
  }
  bool walk_path(uint64_t key, SearchResult& r, uint32_t tag);
  bool path_dsync = false;  // the search's path gather went through the device window
  void finish_walk(SearchResult& r);
  void cleanup_enqueue(const Ctl& h);
  void walk_path_per_hop(uint64_t key, uint32_t it, SearchResult& r);
};

// One round planned by the host (a stalled speculative plan: a bottom-up
// level, or a sparse level too big for the speculative block).  Sizes come
// from the read-back Ctl; one host wait at the end (k_final).
void DistBiBfs::Impl::host_round(uint32_t it, const Policy& pol, SearchResult& r) {
  TraceRange range("dist:host_round");
  const Ctl h = *h_ctl;
  hipStream_t ps = stream, cs = cstream;
  const int P = size;
  const uint32_t words = chunk / 32, nloc = hi - lo;
  const uint32_t capr = cap();
  V.cap = capr;
  stats.host_rounds++;
  k_plan_force<<<1, 64, 0, cs>>>(V, it, pol);
  HIP_CHECK(hipGetLastError());
  int sides[2], ns = 0;
  for (int s = 0; s < 2; ++s)
    if ((h.want >> s) & 1) sides[ns++] = s;
  // ---- pre phases on the compute stream
  HIP_CHECK(hipEventRecord(ev_round, cs));
  HIP_CHECK(hipStreamWaitEvent(ps, ev_round, 0));
  for (int i = 0; i < ns; ++i) {
    const int s = sides[i];
    const uint32_t dnew = h.depth[s] + 1;
    const unsigned fblocks = blocks_for(h.cnt[s] / (uint64_t)P + kThreads, cus);
    if (!((h.want_modes >> s) & 1)) {
      const bool hubs = h.fed[s] > kHubDeg;
      k_td_expand<<<fblocks, kThreads, 0, ps>>>(V, s, dnew, hubs ? kHubDeg : kNoHubs, ns == 1);
      if (hubs)
        k_td_hubs<<<blocks_for(std::min<uint64_t>(h.fed[s], (uint64_t)cus * 8 * kThreads), cus), kThreads, 0, ps>>>(
            V, it, s, dnew, capr, ns == 1, 0, 0, 0);
      k_send_header<<<1, 64, 0, ps>>>(V, s, it);
    } else {
      HIP_CHECK(hipMemsetAsync(V.obits[s], 0, (size_t)words * 4, ps));
      k_obits<<<fblocks, kThreads, 0, ps>>>(V, s);
    }
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipEventRecord(ev_pre[i], ps));
  }
  // ---- exchange + post phases on the comm stream: side 0's run while side
  // 1's pre phase is still computing on the other stream
  for (int i = 0; i < ns; ++i) {
    const int s = sides[i];
    const uint32_t dnew = h.depth[s] + 1;
    HIP_CHECK(hipStreamWaitEvent(cs, ev_pre[i], 0));
    bool bottomup = (h.want_modes >> s) & 1;
    if (!bottomup) {
      uint64_t per;
      const uint64_t bound = std::min<uint64_t>(h.fed[s], capr);
      if (h.fed[s] <= capr && block_words(bound) * 4 * (uint64_t)P <= tune.nosync_bytes) {
        per = bound;  // no rank emits more than the side's frontier edges: no count exchange
      } else {
        comm->allreduce(V.red[it & 1].maxsend + s, 1, DType::kU32, ROp::kMax, cs);
        stats.collectives++;
        HIP_CHECK(hipMemcpyAsync(h_red, V.red + (it & 1), sizeof(Reduced), hipMemcpyDeviceToHost, cs));
        wait(cs);
        per = h_red->maxsend[s];
        stats.count_syncs++;
        if (per > capr) {
          bottomup = true;  // finish the level bottom-up; the local claims made stay valid
          stats.overflow_levels++;
        }
      }
      if (!bottomup) {
        if (per > 0) {
          // this side's exchange lands at recvbuf + s * P * block_words(per); a
          // rank's send block is at sendbuf + s * block_words(capr)
          uint32_t* recv = V.recvbuf + (uint64_t)s * P * block_words(capr);
          comm->allgather(V.sendbuf + s * block_words(capr), recv, block_words(per) * 4, cs);
          stats.collectives++;
          k_td_claim<<<blocks_for((uint64_t)P * per, cus), kThreads, 0, cs>>>(V, s, (uint32_t)per, dnew);
          stats.exchanged_bytes += block_words(per) * 4 * (uint64_t)P;
        }
      } else {
        HIP_CHECK(hipMemsetAsync(V.obits[s], 0, (size_t)words * 4, cs));
        k_obits<<<blocks_for(h.cnt[s] / (uint64_t)P + kThreads, cus), kThreads, 0, cs>>>(V, s);
      }
    }
    if (bottomup) {
      stats.dense_levels++;
      comm->allgather(V.obits[s], V.gbits[s], (size_t)words * 4, cs);
      stats.collectives++;
      k_bu<<<blocks_for(nloc, cus), kThreads, 0, cs>>>(V, s, dnew);
      stats.exchanged_bytes += (uint64_t)words * 4 * P;
      ++r.stats.bottomup_levels;
    }
    HIP_CHECK(hipGetLastError());
  }
  const uint64_t claimed_bound = std::min<uint64_t>((uint64_t)nloc, h.fed[0] + h.fed[1] + 1);
  k_meet_end<<<blocks_for(claimed_bound, cus), kThreads, 0, cs>>>(V, it);
  HIP_CHECK(hipGetLastError());
  if (P > 1) {
    comm->allgather(&V.red[it & 1], V.redg[it & 1], sizeof(Reduced), cs);
    stats.collectives++;
  }
}

SearchResult DistBiBfs::Impl::search(vid_t src, vid_t dst, const SearchOptions& opt) {
  TraceRange range("dist:search");
  const auto t0 = std::chrono::steady_clock::now();
  BIBFS_REQUIRE(n > 0, "no graph loaded");
  BIBFS_REQUIRE(src < n && dst < n, "src/dst out of range");
  if (comm->aborted()) throw Error("dist: the communicator was aborted by an earlier failure");
  HIP_CHECK(hipSetDevice(device));
  stats = DistLevelStats{};
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
  if (size == 1 && tune.world1_single && !source_only) {
    ensure_single();
    SearchResult rs = single->search(src, dst, opt);
    stats.single_engine = 1;
    stats.levels = rs.stats.levels;
    stats.device_ms = rs.search_ms;
    stats.comm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rs;
  }
  const int P = size;
  hipStream_t cs = cstream;
  if (P == 1) ensure_padj();  // (the partitioned rounds at world size 1: built on first use)
  ++epoch;
  // (before policy(): the plan's overflow test and the kernels' spill bound
  // must be the same number)
  V.spill_cap = size > 1 ? (tune.spill_cap ? std::min(block_cap, tune.spill_cap) : block_cap) : 1;
  const Policy pol = policy(opt);
  V.cap = cap();
  V.trace = opt.trace ? d_trace : nullptr;
  V.rstamp = tune.stamps ? d_rstamp : nullptr;

  // Plan words of older searches must not match this one's tags.  Only the
  // previous search's trailing no-op rounds can still be running (its
  // terminal round ran after its own seed, behind everything before it);
  // they carry the previous epoch.
  std::memset(h_plan, 0, kPlanRing * 8);
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const bool solo = P == 1 && tune.solo && tune.spec_rounds > 0;
  if (!solo) k_seed<<<1, 64, 0, cs>>>(V, src, dst);  // (the solo workgroup seeds itself)
  // (the pipelined planner reduces every rank's header in LDS: up to kStageRanks ranks)
  // (a lookahead of one round only: the drain accounts the round the first
  // stalled plan left pending, which deeper no-op tails would overwrite)
  const bool pipe_start =
      P > 1 && P <= kStageRanks && tune.pipeline && tune.spec_rounds == 1 && max_deg <= kPipeMaxDeg && !pipe_off;
  if (P > 1 && !pipe_start) {  // (pipelined: the seed's reduction rides round 0's exchange)
    comm->allgather(&V.red[1], V.redg[1], sizeof(Reduced), cs);
    stats.collectives++;
  }
  uint32_t it = 0;
  uint32_t spec_cap = kSpecCapMin;
  uint32_t ocap_last = 0;  // owner block capacity of the last speculative round
  bool solo_cleaned = false;
  int flags = 0;
  bool have_ctl = false;  // h_ctl describes the current device state
  const int K = std::min<int>(std::max(0, tune.spec_rounds), (int)kPlanRing - 1);
  const bool host_only = K == 0;  // A/B mode: every round planned on the host
  // Pipelined rounds (DistTuning::pipeline, more than one rank): the round's
  // reduction travels with the next round's candidate exchange -- ONE
  // collective per round -- and each plan accounts the round before the last
  // one.  The first stall (a spill, a big or dense frontier) drains the
  // pipeline and the search continues with exact plans.
  bool pipe = pipe_start;
  bool pipe_used = pipe;
  bool dsync_used = false;  // a round exchanged through the window (DevSync): a barrier closes the search
  stats.pipelined = pipe ? 1 : 0;
  const uint32_t spec_max = std::max<uint32_t>(kSpecCapMin, std::min<uint32_t>(tune.spec_cap_max, block_cap));
  if (host_only) {
    final_and_wait(it++, pol, kPlanStall, cs);
    have_ctl = true;
  } else if (solo) {
    // one launch for every round the solo workgroup can hold; it leaves the
    // state of a stalled round (or the finished search) and its Ctl in h_ctl
    const uint32_t tag = next_tag();
    const uint32_t emax = std::min<uint32_t>(std::max<uint32_t>(tune.solo_edges, 1), kSoloE);
    // bit 0: the workgroup seeds the search; bit 1: no self-cleanup (k_cleanup after the search instead)
    const int sflags = 1;  // the search that ends in the solo workgroup resets its own state
    if (solo_stamp) k_spec_solo<true><<<1, kSoloT, 0, cs>>>(V, it, pol, emax, sflags, src, dst, h_fin, tag, d_stamps);
    else k_spec_solo<false><<<1, kSoloT, 0, cs>>>(V, it, pol, emax, sflags, src, dst, h_fin, tag, nullptr);
    HIP_CHECK(hipGetLastError());
    stats.host_syncs++;
    spin_tag(tag, cs);
    if (solo_stamp) {
      unsigned long long st8[10];
      HIP_CHECK(hipMemcpy(st8, d_stamps, sizeof st8, hipMemcpyDeviceToHost));
      std::fprintf(stderr,
                   "[solo] rounds %llu edges %llu | cycles: setup %llu plan %llu (planner %llu publish %llu) edges %llu "
                   "end %llu scan %llu exit %llu\n",
                   st8[4], st8[5], st8[6], st8[0], st8[8], st8[9], st8[1], st8[2], st8[3], st8[7]);
    }
    have_ctl = true;
    stats.solo_rounds = (int)(h_ctl->rounds);
    solo_cleaned = (h_ctl->state == kDead ||
                   (h_ctl->state == kDone && !(pol.want_path && 4 + (h_ctl->key >> 32) + 1 > pol.walk_cap)));
    it = h_ctl->next_it;
    const uint64_t fm = std::max(h_ctl->fmax[0], h_ctl->fmax[1]);
    spec_cap = std::min(spec_max, std::max<uint32_t>(kSpecCapMin, next_pow2(4 * fm)));
  }
  for (uint64_t guard = 0;; ++guard) {
    BIBFS_REQUIRE(guard <= 4ull * n + 16, "dist: search did not terminate");
    if (have_ctl && h_ctl->state != kRun && h_ctl->state != kStall) break;
    if (have_ctl && h_ctl->state == kStall) {
      const Ctl& h = *h_ctl;
      uint64_t need = 0;
      for (int s = 0; s < 2; ++s)
        if ((h.want >> s) & 1) need = std::max<uint64_t>(need, h.fmax[s]);
      if (!host_only && h.stall == kStallCap && need <= round_edge_cap()) {
        spec_cap = std::min<uint32_t>(spec_max, std::max<uint32_t>(spec_cap, next_pow2(need)));
        flags = kPlanResume;  // re-run the stalled plan speculatively with a bigger block
      } else {
        maybe_fault((int)it);
        host_round(it, pol, r);
        final_and_wait(it + 1, pol, host_only ? kPlanStall : kPlanAccountOnly, cs);
        it += 2;
        const uint64_t fm = std::max(h_ctl->fmax[0], h_ctl->fmax[1]);
        spec_cap = std::min(spec_max, std::max<uint32_t>(kSpecCapMin, next_pow2(4 * fm)));
        continue;
      }
    }
    // ---- speculative sparse rounds with a rolling lookahead
    TraceRange batch_range("dist:speculative_batch");
    // Rolling lookahead: round `it` is enqueued once the plan of round it - K
    // is visible in pinned memory (no stream sync); enqueueing stops at the
    // first such plan that is not "run" (done, no path or stalled), so about K
    // no-op rounds trail the end of a search.  Each round's block capacity is
    // predicted from the frontier sizes of the plans seen so far (growth per
    // round, extrapolated K rounds), so a growing frontier rarely stalls the
    // lookahead.  Plans and frontier sizes are reduced values, identical on
    // every rank: every rank enqueues the same rounds with the same sizes.
    const uint32_t first = it;
    uint32_t cap_it = spec_cap;
    uint32_t ocap = ocap_last;
    uint64_t f_prev = 0;
    uint32_t seen_state = kRun;  // state of the last plan word read
    for (int k = 0;; ++k) {
      if (k >= K) {
        const uint32_t need = it - (uint32_t)K;
        const uint64_t w = wait_plan(need, cs);
        stats.plan_polls++;
        seen_state = (uint32_t)(w >> 2) & 3u;
        if (seen_state != kRun) break;
        const uint64_t f = w >> 32;
        uint64_t g = 2;  // growth per round; x2 until two plans are seen
        if (f_prev) g = std::min<uint64_t>(8, std::max<uint64_t>(1, (f + f_prev - 1) / f_prev));
        // (a pipelined plan's frontier is one round older: one more round of growth)
        const int lag = pipe ? 1 : 0;
        uint64_t pred = f;
        for (int j = 0; j < K + lag && pred < spec_max; ++j) pred *= g;
        cap_it = std::max<uint32_t>(cap_it, std::min<uint32_t>(spec_max, next_pow2(std::min<uint64_t>(pred + pred / 2, spec_max))));
        f_prev = f;
        // owner blocks: the largest per-owner count of round need - 1, grown
        // over the K + 1 rounds since, with half again as slack; too small
        // costs a continuation round, too big only bytes
        const uint64_t om = std::min<uint64_t>(__atomic_load_n(&h_aux[need % kPlanRing], __ATOMIC_ACQUIRE), spec_max);
        uint64_t op = om;
        for (int j = 0; j <= K + lag && op < cap_it; ++j) op *= g;
        ocap = std::min<uint32_t>(cap_it, std::max<uint32_t>(kOwnerCapMin, next_pow2(op + op / 2 + 16)));
      }
      if (P == 1) ocap = 0;  // nothing is ever offered
      else if (tune.owner_cap) ocap = tune.owner_cap;
      else if (!ocap) ocap = kOwnerCapMin;
      ocap = std::min(std::min(ocap, cap_it), spec_max);  // (the buffers hold blocks of spec_max pairs)
      if ((uint64_t)(it - first) > 4ull * n + 16) break;  // safety net
      const unsigned bx = std::min<unsigned>((unsigned)cus * 2, cap_it / kThreads + 1);  // ~ this rank's edges
      const unsigned cx = std::min<unsigned>((unsigned)cus * 2,
                                             std::max<unsigned>(1, (uint32_t)P * ocap / kThreads / 4 + 1));
      const uint64_t peer_bytes = peer_words(ocap) * 4;  // header + both sides' blocks for one owner
      // With blocks of at most kSpecHubCap pairs a frontier vertex has at most
      // that many edges: one workgroup walks them in <= 16 steps, no hub pass.
      const bool hubs = cap_it > kSpecHubCap && max_deg > kHubDeg;
      const unsigned hx = std::min<unsigned>((unsigned)cus, cap_it / kThreads + 1);
      maybe_fault((int)it);
      // The round's last claiming kernel closes it (meets were detected at
      // claim time): the claim kernel with more than one rank, else the hub
      // pass or the expansion itself -- no separate meet / round-end kernel.
      const int end_in_expand = (P == 1 && !hubs) ? 1 : 0;
      // The plan stalls a round whose per-rank frontier edges exceed this:
      // with one rank nothing is exchanged, so nothing bounds a round; with
      // more, a rank's candidates (at most its frontier edges) must fit the
      // spill lists (owner blocks overflow into them).
      const uint32_t plan_cap = round_edge_cap();
      const int pp = pipe ? 1 : 0;
      // the device-ordered exchange: this round's candidates go to the
      // window half of its epoch, which the peers' claim kernels read once
      // this rank's flag says so (no host rendezvous; see DevSync)
      // (small claim grids only: every waiting workgroup holds a CU slot, and
      // the peers' expansions it waits for must still find room -- a wide claim
      // grid per rank on one GPU starved them)
      const bool dsync = P > 1 && win_ok && tune.dev_sync && peer_bytes * (uint64_t)P <= win_half && cx + 1u <= kDevSyncBlocks;
      DView VR = V;
      unsigned long long ep = 0;
      if (dsync) {
        ep = ++dev_epoch;
        VR.sendbuf = reinterpret_cast<uint32_t*>(static_cast<char*>(win.mine) + dist::Comm::kWinFlagBytes +
                                                 (ep & 1) * win_half);
        dsync_used = true;
        stats.dev_sync_rounds++;
      }
      k_spec_expand<<<dim3(bx, 2), kThreads, 0, cs>>>(VR, it, pol, cap_it, k == 0 ? flags : 0,
                                                      hubs ? kHubDeg : kNoHubs, hubs ? 0 : 1, end_in_expand, ocap,
                                                      plan_cap, pp);
      if (hubs) k_td_hubs<<<dim3(hx, 2), kThreads, 0, cs>>>(VR, it, -1, 0, cap_it, 0, P == 1 ? 1 : 0, ocap, pp);
      HIP_CHECK(hipGetLastError());
      if (P > 1) {
        // Owner-addressed exchange: ONE alltoall moves, per peer, the
        // reduction header and both sides' candidate blocks (oblock); each
        // rank receives only what is addressed to it.  Pipelined, the header
        // is the round's status too: no second collective.
        // (read in place where the transport allows: no copy on the local group)
        PeerTab pt{};
        DevSync ds{};
        if (dsync) {
          for (int r = 0; r < P; ++r)
            pt.p[r] = reinterpret_cast<const uint32_t*>(static_cast<const char*>(win.peer[r]) + dist::Comm::kWinFlagBytes +
                                                        (ep & 1) * win_half + (size_t)rank * peer_bytes);
          pt.direct = 1;
          ds = dev_sync(ep);
        } else if (P <= kStageRanks) {
          const void* pv[kStageRanks];
          comm->alltoall_view(V.sendbuf, V.recvbuf, peer_bytes, cs, pv);
          for (int r = 0; r < P; ++r) pt.p[r] = static_cast<const uint32_t*>(pv[r]);
          pt.direct = 1;
        } else {
          comm->alltoall(V.sendbuf, V.recvbuf, peer_bytes, cs);
        }
        // (pipelined: one extra block plans the next round beside the claims)
        k_spec_claim<<<dim3(cx + (pipe ? 1u : 0u), 2), kThreads, 0, cs>>>(VR, it, ocap, pp, pol, plan_cap, pt, ds);
        HIP_CHECK(hipGetLastError());
        if (!dsync && P <= kStageRanks) comm->alltoall_release(cs);
        stats.collectives++;
        stats.exchanged_bytes += peer_bytes * (P - 1);
        if (!pipe) {  // exact plans: the round's reduction, every rank's values gathered, reduced by the reader
          comm->allgather(&V.red[it & 1], V.redg[it & 1], sizeof(Reduced), cs);
          stats.collectives++;
          stats.exchanged_bytes += sizeof(Reduced) * (P - 1);
        }
      }
      stats.spec_rounds++;
      ++it;
    }
    spec_cap = cap_it;
    ocap_last = ocap;
    flags = 0;
    have_ctl = true;
    if (seen_state == kDone || seen_state == kDead) {
      // the round that ended the search wrote its accounted Ctl to h_ctl
      // before its plan word: no k_final + wait (the no-op rounds behind it
      // drain before the search's last tag)
      ++it;
      break;
    }
    if (pipe && seen_state == kStall) {
      // drain: the stalled pipelined plan is replaced by the exact account of
      // the round it left pending (its reduction arrived with the stalled
      // round's exchange); from here on every plan is exact
      final_and_wait(it++, pol, kPlanAccountOnly | kPlanDrain, cs);
      pipe = false;
      stats.pipe_drains++;
    } else {
      final_and_wait(it++, pol, kPlanAccountOnly, cs);
    }
    if (h_ctl->state == kRun) {  // size the next batch for the frontier we have now
      const uint64_t fm = std::max(h_ctl->fmax[0], h_ctl->fmax[1]);
      spec_cap = std::min(spec_max, std::max<uint32_t>(spec_cap, next_pow2(4 * fm)));
    }
  }
  // every peer's reads of this rank's window during this search complete
  // before this rank's stream goes on (the window may be released): one
  // barrier epoch at the search's end -- after the path gather, or here on
  // the paths that end the search now
  auto window_barrier = [&] {
    k_dev_barrier<<<1, 64, 0, cs>>>(dev_sync(++dev_epoch));
    HIP_CHECK(hipGetLastError());
    dsync_used = false;
  };
  path_dsync = false;
  const Ctl h = *h_ctl;
  if (dsync_used && h.lost) window_barrier();
  if (h.lost && pipe_used) {
    // a pipelined round ran on a frontier its plan could not see yet and
    // overflowed the spill lists: every rank saw it (reduced values), so
    // every rank answers the query again with exact plans
    cleanup_enqueue(h);
    pipe_off = true;
    SearchResult again;
    try {
      again = search(src, dst, opt);
    } catch (...) {
      pipe_off = false;
      throw;
    }
    pipe_off = false;
    stats.pipe_retries++;
    return again;
  }
  if (h.lost) {
    // every rank decided `lost` from the same reduced values, so every rank
    // throws here, after the same collectives: the communicator stays usable
    cleanup_enqueue(h);
    throw ConsistentError("dist: a rank's candidate spill list overflowed (" + std::to_string(V.spill_cap) +
                " pairs): candidates were dropped, the search result would not be exact");
  }
  stats.rounds = (int)h.rounds;
  stats.lockstep_rounds = (int)h.lockstep_rounds;
  stats.levels = (int)h.levels;
  stats.sparse_levels = (int)h.sparse_levels;
  stats.cont_rounds = (int)h.cont_rounds;
  r.stats.levels = (int)h.levels;
  r.stats.edges_inspected = h.einsp;
  r.stats.visited = h.vis[0] + h.vis[1];
  stats.comm_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  // The search's result is complete on the host when the walk (if any) is:
  // with one rank the round that ended the search walked the path into
  // pinned memory before its plan word (terminal_walk); otherwise a gathered
  // walk, or k_walk_local when the path outgrew the pinned buffer.  The host
  // waits on a tag only for those, and never for the reset of the search
  // state: k_cleanup trails in cstream, where everything the next search
  // enqueues is ordered behind it (the compute stream waits on an event of
  // cstream before it is used).
  bool path_pending = false;  // a walk result lands in h_walk behind `tag`
  uint32_t tag = 0;
  if (h.state == kDone) {
    const uint64_t key = h.key;
    r.found = true;
    r.meet = (uint32_t)(key & 0xffffffffull);
    r.hops = (int64_t)(key >> 32);
    if (opt.want_path && P == 1) {
      const bool walked = h_walk[3] == pol.epoch && h_walk[0] != 2u;
      if (!walked) {
        ensure_walk_buf(4 + (size_t)r.hops + 1);
        tag = next_tag();
        k_walk_local<<<1, 64, 0, cs>>>(V, r.meet, (uint32_t)r.hops, h_walk, h_fin, tag);
        HIP_CHECK(hipGetLastError());
      }
      path_pending = true;
    } else if (opt.want_path) {
      const uint32_t wt = next_tag();  // k_walk releases the path with it
      if ((path_pending = walk_path(key, r, wt))) tag = wt;
      else walk_path_per_hop(key, it, r);
    }
  }
  if (dsync_used || path_dsync) window_barrier();
  if ((opt.trace || tune.stamps) && !tag) {  // trace records / stamps are plain device stores: drain the rounds first
    tag = next_tag();
    k_host_tag<<<1, 64, 0, cs>>>(h_fin, tag);
    HIP_CHECK(hipGetLastError());
  }
  if (!solo_cleaned) cleanup_enqueue(h);
  if (tag) {
    stats.host_syncs++;
    spin_tag(tag, cs);
  }
  if (path_pending) finish_walk(r);
  if (tune.stamps) collect_stamps(it);
  if (opt.trace && h.rounds) {
    std::vector<RoundRec> tr(std::min<uint32_t>(h.rounds, kTraceCap));
    HIP_CHECK(hipMemcpy(tr.data(), d_trace, tr.size() * sizeof(RoundRec), hipMemcpyDeviceToHost));
    for (const RoundRec& t : tr)
      for (int s = 0; s < 2; ++s) {
        if (!((t.sides >> s) & 1)) continue;
        LevelTrace lt;
        lt.side = s;
        lt.depth = (int)t.depth[s];
        lt.frontier = t.cnt[s];
        lt.edges = t.fed[s];
        lt.discovered = t.sums[2 * s];
        lt.mode = ((t.modes >> s) & 1) ? 5 : 4;
        r.stats.trace.push_back(lt);
      }
  }
  const double dms = (double)h.ticks / 1e5;  // s_memrealtime: 100 MHz
  stats.device_ms = dms;
  r.stats.grid_levels = r.stats.levels;
  r.search_ms = dms;
  r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return r;
}

// Path in O(1) collectives: every rank packs the (vertex, parent) pairs it
// claimed, ONE allgather, and a one-workgroup kernel walks both parent chains
// from LDS tables.  False when the visited sets are too large for that.
bool DistBiBfs::Impl::walk_path(uint64_t key, SearchResult& r, uint32_t tag) {
  TraceRange range("dist:path_gather");
  const Ctl& h = *h_ctl;
  const uint64_t vS = h.vis[0], vT = h.vis[1];
  if (vS + vT > tune.walk_max) return false;
  const uint32_t capS = (uint32_t)std::max<uint64_t>(vS, 1), capT = (uint32_t)std::max<uint64_t>(vT, 1);
  // Linear probing: as sparse as the LDS allows, down to a 0.75 load factor.
  // At 0.75 the tables' clusters made the walk's inserts and lookups ~1,000
  // cycles each (G(1M), ~3k pairs: 17 + 14 us of a 33 us walk kernel).
  const uint64_t need = (uint64_t)capS + capS / 3 + 1 + capT + capT / 3 + 1;
  if (need > kWalkSlots) return false;
  const uint64_t f = std::min<uint64_t>(4, kWalkSlots / ((uint64_t)capS + capT + 2));  // slots per pair (1 = 0.75 fill)
  const uint32_t slotsS = (uint32_t)(f > 1 ? f * capS + 1 : capS + capS / 3 + 1),
                 slotsT = (uint32_t)(f > 1 ? f * capT + 1 : capT + capT / 3 + 1);
  const size_t lds = (size_t)(slotsS + slotsT) * 8;
  if (lds > kWalkSlots * 8) return false;
  const uint32_t meet = (uint32_t)(key & 0xffffffffull), hops = (uint32_t)(key >> 32);
  hipStream_t cs = cstream;
  // sized before the collective (every rank knows `hops`): a failing
  // allocation aborts the communicator before, not between, collectives
  ensure_path_dev((size_t)hops + 5);
  ensure_walk_buf(4 + (size_t)hops + 1);  // (k_walk writes the path there)
  const uint64_t blk = 2 + 2 * ((uint64_t)capS + capT);
  // the gather through the device window where the round exchange uses it
  // (the same epoch protocol: pack into this epoch's half, raise, wait, read)
  const bool dsync = win_ok && tune.dev_sync && size <= kStageRanks && blk * 4 <= win_half;
  DView VR = V;
  PeerTab pt{};
  DevSync ds{};
  if (dsync) {
    const unsigned long long ep = ++dev_epoch;
    VR.sendbuf = reinterpret_cast<uint32_t*>(static_cast<char*>(win.mine) + dist::Comm::kWinFlagBytes +
                                             (ep & 1) * win_half);
    for (int r = 0; r < size; ++r)
      pt.p[r] = reinterpret_cast<const uint32_t*>(static_cast<const char*>(win.peer[r]) + dist::Comm::kWinFlagBytes +
                                                  (ep & 1) * win_half);
    pt.direct = 1;
    ds = dev_sync(ep);
    path_dsync = true;
  }
  k_pack_parents<<<blocks_for(vS + vT, cus), kThreads, 0, cs>>>(VR, capS, capT, h.depth[0], h.depth[1]);
  if (!dsync) comm->allgather(V.sendbuf, V.recvbuf, blk * 4, cs);
  stats.collectives++;
  stats.path_collectives++;
  stats.exchanged_bytes += blk * 4 * size;
  k_walk<<<1, 1024, lds, cs>>>(V.recvbuf, pt, ds, size, capS, capT, slotsS, slotsT, meet, hops, h_walk, h_fin, tag);
  HIP_CHECK(hipGetLastError());
  return true;  // read by finish_walk after the search's last wait (its tag)
}

void DistBiBfs::Impl::finish_walk(SearchResult& r) {
  const uint32_t hops = (uint32_t)r.hops;
  BIBFS_REQUIRE(h_walk[0] == 0, "dist: parent chains from the meet vertex do not add up to the path length (" +
                                    std::to_string(h_walk[1]) + " + " + std::to_string(h_walk[2]) +
                                    " != " + std::to_string(hops) + ")");
  r.path.assign(h_walk + 4, h_walk + 4 + hops + 1);
  if (tune.stamps) {
    stats.walk_insert_us += (h_walk[3] & 0xffffu) * 0.01;
    stats.walk_chain_us += (h_walk[3] >> 16) * 0.01;
  }
}

void DistBiBfs::Impl::cleanup_enqueue(const Ctl& h) {
  const uint64_t sent_words = (uint64_t)gwords * 2;
  const uint64_t work = std::max<uint64_t>(h.vis[0] + h.vis[1], sent_words / 4);
  k_cleanup<<<blocks_for(std::max<uint64_t>(work, 1), cus), kThreads, 0, cstream>>>(V, sent_words);
  HIP_CHECK(hipGetLastError());
}

// Fallback: one allreduce per hop (visited sets too large to gather).
void DistBiBfs::Impl::walk_path_per_hop(uint64_t key, uint32_t it, SearchResult& r) {
  TraceRange range("dist:path_per_hop");
  hipStream_t cs = cstream;
  const uint32_t meet = (uint32_t)(key & 0xffffffffull);
  ensure_path_dev((size_t)std::max<int64_t>(r.hops, 0) + 1);  // (K <= hops; sized before any collective)
  k_meet_depth<<<1, 64, 0, cs>>>(V, meet, it);
  comm->allreduce(V.red[it & 1].md, 2, DType::kU32, ROp::kMin, cs);
  stats.collectives++;
  stats.path_collectives++;
  HIP_CHECK(hipMemcpyAsync(h_red, V.red + (it & 1), sizeof(Reduced), hipMemcpyDeviceToHost, cs));
  wait(cs);
  const int dS = (int)h_red->md[0], dT = (int)h_red->md[1];
  BIBFS_REQUIRE((int64_t)dS + dT == r.hops, "dist: meet depths disagree with the path length");
  const int K = std::max(dS, dT);
  const uint32_t init[2] = {meet, meet};
  HIP_CHECK(hipMemcpyAsync(d_cur, init, 8, hipMemcpyHostToDevice, cs));
  for (int i = 0; i <= K; ++i) {
    k_path_step<<<1, 64, 0, cs>>>(V, d_cur, d_pathS, d_pathT, i, dS, dT);
    if (i < K) {
      comm->allreduce(d_cur, 2, DType::kU32, ROp::kMin, cs);
      stats.collectives++;
      stats.path_collectives++;
    }
  }
  std::vector<uint32_t> pS((size_t)dS + 1), pT((size_t)dT + 1);
  HIP_CHECK(hipMemcpyAsync(pS.data(), d_pathS, pS.size() * 4, hipMemcpyDeviceToHost, cs));
  HIP_CHECK(hipMemcpyAsync(pT.data(), d_pathT, pT.size() * 4, hipMemcpyDeviceToHost, cs));
  wait(cs);
  r.path.assign(pS.rbegin(), pS.rend());
  r.path.insert(r.path.end(), pT.begin() + 1, pT.end());
}

DistBiBfs::DistBiBfs(int rank, int size, int device, const std::vector<uint8_t>& uid, const std::string& backend)
    : p_(new Impl) {
  HIP_CHECK(hipSetDevice(device));
  const char* w1 = std::getenv("BIBFS_WORLD1_COMM");  // "rccl" / "ipc": keep that backend at one rank (tests)
  if (size == 1 && (backend == "ipc" || backend == "rccl") && !(w1 && backend == w1))
    // one rank: every collective is a copy to itself -- the in-process group
    // of one does that without RCCL's ~3.4 s communicator bootstrap
    p_->comm = dist::make_local_comm(dist::make_local_group(1, p_->tune.timeout_s), 0);
  else if (backend == "ipc")
    p_->comm = dist::make_ipc_comm(rank, size, uid, p_->tune.timeout_s);
  else if (backend == "rccl")
    p_->comm = dist::make_rccl_comm(rank, size, uid);
  else
    throw Error("dist: backend must be rccl or ipc, got " + backend);
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
    if (!p_->comm->aborted()) {
      (void)hipStreamSynchronize(p_->stream);
      (void)hipStreamSynchronize(p_->cstream);
    }
    p_->free_all();
  } catch (...) {
  }
  p_->comm.reset();
  (void)hipFree(p_->d_stamps);
  (void)hipHostFree(p_->h_red);
  (void)hipHostFree(p_->h_ctl);
  (void)hipHostFree(p_->h_fin);
  (void)hipHostFree(p_->h_plan);
  (void)hipHostFree(p_->h_aux);
  if (p_->h_walk) (void)hipHostFree(p_->h_walk);
  for (auto e : p_->ev_pre) (void)hipEventDestroy(e);
  (void)hipEventDestroy(p_->ev_round);
  (void)hipEventDestroy(p_->ev_t0);
  (void)hipEventDestroy(p_->ev_t1);
  (void)hipStreamDestroy(p_->cstream);
  (void)hipStreamDestroy(p_->stream);
}

void DistBiBfs::load_edges(const EdgeList& el) {
  TraceRange range("dist:build");
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
  I.finish_build();
}

void DistBiBfs::load_bin(const std::string& path) {
  TraceRange range("dist:build");
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
  I.finish_build();
}

void DistBiBfs::generate_gnp(uint32_t n, double p, uint64_t seed) {
  TraceRange range("dist:build");
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.free_all();
  I.set_partition(n);
  // owned rows straight from the generator (no edge list on any rank)
  {
    devmem::Scope scope(&I.mem);
    I.mem.reset_peak();
    devmem::alloc(&I.d_row_off, I.row_off_bytes());
    uint64_t m = 0;
    I.nnz = launch::gen_rows_gnp(n, p, seed, I.lo, I.hi, I.d_row_off, &I.d_col, &m, I.stream);
    I.m_input = m;
    I.record_build_peak();
  }
  I.finish_build();
}

void DistBiBfs::generate_rmat(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c) {
  TraceRange range("dist:build");
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.free_all();
  I.set_partition(n);
  // owned rows straight from the generator (no edge list on any rank)
  {
    devmem::Scope scope(&I.mem);
    I.mem.reset_peak();
    devmem::alloc(&I.d_row_off, I.row_off_bytes());
    I.nnz = launch::gen_rows_rmat(n, m, seed, a, b, c, I.lo, I.hi, I.d_row_off, &I.d_col, I.stream);
    I.m_input = m;
    I.record_build_peak();
  }
  I.finish_build();
}

SearchResult DistBiBfs::search(vid_t src, vid_t dst, const SearchOptions& opt) {
  auto& I = *p_;
  // Input errors fail identically on every rank before any collective is
  // enqueued: they must not abort the communicator (a bad query would
  // otherwise poison every later search).
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  BIBFS_REQUIRE(src < I.n && dst < I.n, "src/dst out of range");
  try {
    return I.search(src, dst, opt);
  } catch (const ConsistentError&) {
    throw;  // every rank raised it at the same point: no peer is left in a collective
  } catch (...) {
    // A rank that fails mid-search would leave its peers blocked in a
    // collective forever: tear the communicator down so they return too.
    I.give_up();
    I.comm->abort();
    throw;
  }
}

bool DistBiBfs::query_is_local() const {
  const auto& I = *p_;
  return I.size == 1 && I.tune.world1_single && I.single != nullptr;
}

int64_t DistBiBfs::query(vid_t src, vid_t dst, std::vector<vid_t>* path) {
  auto& I = *p_;
  if (query_is_local()) {
    // world size 1: the rank's shard is the whole graph and the adopted
    // single-GPU engine answers through its resident server (tiny / LDS),
    // exactly as HipBiBfs::query -- the partitioned wrapper adds nothing
    if (I.comm->aborted()) throw Error("dist: the communicator was aborted by an earlier failure");
    I.stats = DistLevelStats{};
    I.stats.single_engine = 1;
    return I.single->query(src, dst, path);
  }
  SearchResult r = search(src, dst);
  if (path) *path = std::move(r.path);
  return r.found ? (int64_t)r.hops : -1;
}

void DistBiBfs::barrier() {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  I.comm->allreduce(I.d_scalar, 1, DType::kF64, ROp::kMax, I.cstream);
  I.wait(I.cstream);
}

bool DistBiBfs::validate_path(vid_t src, vid_t dst, int64_t hops, const std::vector<vid_t>& path) {
  auto& I = *p_;
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  HIP_CHECK(hipSetDevice(I.device));
  // Shape checks first: every rank holds the same path, so they all decide
  // alike and either all reach the collective below or none does.
  if (hops < 0 || path.size() != (size_t)hops + 1 || path.front() != src || path.back() != dst) return false;
  for (vid_t v : path)
    if (v >= I.n) return false;
  if (hops == 0) return src == dst;
  std::vector<uint32_t> idx;
  for (size_t i = 0; i + 1 < path.size(); ++i)
    if (path[i] >= I.lo && path[i] < I.hi) idx.push_back((uint32_t)i);
  double found = 0;
  if (!idx.empty()) {
    I.ensure_path_dev(path.size() + idx.size() + 1);
    uint32_t* d_path = I.d_pathS;
    uint32_t* d_idx = I.d_pathT;
    uint32_t* d_found = I.d_pathT + idx.size();
    HIP_CHECK(hipMemcpyAsync(d_path, path.data(), path.size() * 4, hipMemcpyHostToDevice, I.cstream));
    HIP_CHECK(hipMemcpyAsync(d_idx, idx.data(), idx.size() * 4, hipMemcpyHostToDevice, I.cstream));
    k_path_edges<<<(unsigned)idx.size(), kThreads, 0, I.cstream>>>(I.V, d_path, d_idx, d_found);
    HIP_CHECK(hipGetLastError());
    std::vector<uint32_t> f(idx.size());
    HIP_CHECK(hipMemcpyAsync(f.data(), d_found, f.size() * 4, hipMemcpyDeviceToHost, I.cstream));
    I.wait(I.cstream);
    for (uint32_t x : f) found += x;
  }
  // every edge's first vertex has exactly one owner: the edges found over all
  // ranks must be all `hops` of them
  double y = found;
  HIP_CHECK(hipMemcpyAsync(I.d_scalar, &y, 8, hipMemcpyHostToDevice, I.cstream));
  I.comm->allreduce(I.d_scalar, 1, DType::kF64, ROp::kSum, I.cstream);
  HIP_CHECK(hipMemcpyAsync(&y, I.d_scalar, 8, hipMemcpyDeviceToHost, I.cstream));
  I.wait(I.cstream);
  return (int64_t)(y + 0.5) == hops;
}

SearchResult DistBiBfs::search_unidirectional(vid_t src, vid_t dst) {
  auto& I = *p_;
  SearchOptions opt;
  opt.lockstep = false;
  opt.want_path = false;
  I.source_only = true;
  struct Reset {
    Impl& I;
    ~Reset() { I.source_only = false; }
  } reset{I};
  return search(src, dst, opt);
}

double DistBiBfs::allreduce_max(double x) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  double y = x;
  HIP_CHECK(hipMemcpyAsync(I.d_scalar, &y, 8, hipMemcpyHostToDevice, I.cstream));
  I.comm->allreduce(I.d_scalar, 1, DType::kF64, ROp::kMax, I.cstream);
  HIP_CHECK(hipMemcpyAsync(&y, I.d_scalar, 8, hipMemcpyDeviceToHost, I.cstream));
  I.wait(I.cstream);
  return y;
}

void DistBiBfs::release() {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  HIP_CHECK(hipStreamSynchronize(I.cstream));
  I.free_all();
}

void DistBiBfs::set_tuning(const DistTuning& t) {
  BIBFS_REQUIRE(t.spec_rounds >= 0 && t.timeout_s > 0 && t.walk_max >= 1, "bad DistTuning");
  const bool realloc = p_->state && t.walk_max > p_->tune.walk_max;
  p_->tune = t;
  p_->mem.cap = t.hbm_cap_bytes;
  p_->comm->set_timeout(t.timeout_s);
  if (realloc) {  // path-gather blocks are sized from walk_max
    HIP_CHECK(hipSetDevice(p_->device));
    devmem::Scope scope(&p_->mem);
    devmem::release(p_->state, p_->state_bytes);
    p_->state = nullptr;
    p_->alloc_state();
  }
}
const DistTuning& DistBiBfs::tuning() const { return p_->tune; }
void DistBiBfs::inject_fault(int at, int mode) {
  p_->fault_at = at;
  p_->fault_mode = mode;
}

int DistBiBfs::rank() const { return p_->rank; }
int DistBiBfs::size() const { return p_->size; }
uint32_t DistBiBfs::n() const { return p_->n; }
uint64_t DistBiBfs::m_input() const { return p_->m_input; }
uint64_t DistBiBfs::local_nnz() const { return p_->nnz; }
size_t DistBiBfs::shard_bytes() const { return p_->shard_bytes(); }
size_t DistBiBfs::gen_peak_bytes() const { return p_->gen_peak_bytes; }
size_t DistBiBfs::gen_hbm_peak_bytes() const { return p_->gen_hbm_peak_bytes; }
size_t DistBiBfs::resident_bytes() const {
  // (+ the world-1 single-GPU engine's own arrays; its CSR is this rank's)
  const auto& I = *p_;
  size_t extra = 0;
  if (I.single) {
    const size_t all = I.single->device_bytes(), csr = I.row_off_bytes() + I.col_bytes();
    extra = all > csr ? all - csr : 0;
  }
  return I.mem.cur + extra;
}
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
std::vector<SearchResult> run_local_ranks(const char* who, int ranks, int device, size_t nq, const DistTuning& tune,
                                          const DistLocalFault& fault, Body&& body) {
  BIBFS_REQUIRE(ranks >= 1 && ranks <= 16, std::string(who) + ": 1..16 ranks");
  auto group = dist::make_local_group(ranks, tune.timeout_s);
  std::vector<std::vector<SearchResult>> out((size_t)ranks);
  std::vector<std::string> err((size_t)ranks);
  std::vector<std::thread> th;
  for (int r = 0; r < ranks; ++r)
    th.emplace_back([&, r] {
      try {
        DistBiBfs e(dist::make_local_comm(group, r), device);
        e.set_tuning(tune);
        if (fault.rank == r) e.inject_fault(fault.at, fault.mode);
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
                                         const SearchOptions& opt, const DistTuning& tuning,
                                         const DistLocalFault& fault, std::vector<DistLevelStats>* stats) {
  return run_local_ranks("dist_local_run", ranks, device, queries.size(), tuning, fault,
                         [&](DistBiBfs& e, int r, std::vector<SearchResult>& out) {
                           e.load_edges(el);
                           for (const auto& q : queries) {
                             // an out-of-range query fails on every rank before any
                             // collective: reported as hops -2, the group keeps serving
                             if (q.first >= el.n || q.second >= el.n) {
                               bool threw = false;
                               try {
                                 e.search(q.first, q.second, opt);
                               } catch (const Error&) {
                                 threw = true;
                               }
                               BIBFS_REQUIRE(threw, "dist: an out-of-range query did not raise");
                               SearchResult bad;
                               bad.hops = -2;
                               out.push_back(bad);
                               if (r == 0 && stats) stats->push_back(DistLevelStats{});
                               continue;
                             }
                             out.push_back(e.search(q.first, q.second, opt));
                             if (r == 0 && stats) stats->push_back(e.last_stats());
                           }
                         });
}

std::vector<SearchResult> dist_local_generate_run(int ranks, int device, const std::string& kind, uint32_t n,
                                                  double arg, uint64_t seed,
                                                  const std::vector<std::pair<vid_t, vid_t>>& queries,
                                                  const SearchOptions& opt, DistLocalTiming* timing,
                                                  const DistTuning& tuning, int verify) {
  BIBFS_REQUIRE(kind == "gnp" || kind == "rmat", "dist_local_generate_run: kind must be gnp or rmat");
  const size_t R = (size_t)std::max(ranks, 1);
  std::vector<double> build_ms(R, 0.0), qms;
  std::vector<uint64_t> nnz(R, 0), shard(R, 0), peak(R, 0), hpeak(R, 0), resident(R, 0);
  std::vector<DistLevelStats> qstats;
  std::vector<int> valid;
  std::vector<int64_t> uni;
  auto rs = run_local_ranks(
      "dist_local_generate_run", ranks, device, queries.size(), tuning, DistLocalFault{},
      [&](DistBiBfs& e, int r, std::vector<SearchResult>& out) {
        const auto t0 = std::chrono::steady_clock::now();
        if (kind == "gnp")
          e.generate_gnp(n, arg, seed);
        else
          e.generate_rmat(n, (uint64_t)arg, seed);  // synchronous (ends with the cursor's hipFree)
        build_ms[(size_t)r] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        nnz[(size_t)r] = e.local_nnz();
        shard[(size_t)r] = e.shard_bytes();
        peak[(size_t)r] = e.gen_peak_bytes();
        hpeak[(size_t)r] = e.gen_hbm_peak_bytes();
        resident[(size_t)r] = e.resident_bytes();
        for (size_t qi = 0; qi < queries.size(); ++qi) {
          const auto& q = queries[qi];
          const auto q0 = std::chrono::steady_clock::now();
          out.push_back(e.search(q.first, q.second, opt));
          if (r == 0) {
            qms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - q0).count());
            qstats.push_back(e.last_stats());
          }
          if (verify > 0) {  // collective checks (every rank), no graph copy anywhere
            const SearchResult& x = out.back();
            const int ok = x.found ? (e.validate_path(q.first, q.second, x.hops, x.path) ? 1 : 0) : -1;
            const int64_t uh = (int)qi < verify ? e.search_unidirectional(q.first, q.second).hops : -2;
            if (r == 0) {
              valid.push_back(ok);
              uni.push_back(uh);
            }
          }
        }
      });
  if (timing) {
    timing->build_ms = *std::max_element(build_ms.begin(), build_ms.end());
    timing->query_ms = std::move(qms);
    timing->local_nnz = std::move(nnz);
    timing->shard_bytes = std::move(shard);
    timing->gen_peak_bytes = std::move(peak);
    timing->gen_hbm_peak_bytes = std::move(hpeak);
    timing->resident_bytes = std::move(resident);
    timing->stats = std::move(qstats);
    timing->path_valid = std::move(valid);
    timing->uni_hops = std::move(uni);
  }
  return rs;
}

}  // namespace bibfs
