// Multi-GPU bidirectional BFS (v4 capability, C10/C11/C12 + P1-P4 in
// SURVEY.md), re-designed for MI355X nodes: one process per GPU, RCCL over
// xGMI for every per-level exchange, device-resident state.
//
// Partition: 1-D block over vertices, block size rounded up to 64 so every
// rank's slice of a frontier bitmap is a whole number of words and the
// allgathered bitmap is directly indexable by global vertex id.  Rank r holds
// only its own CSR rows (column ids global), its slice of both visited
// bitmaps, and parents / BFS queues of its own vertices; the reference
// replicated the whole graph and all state on every rank
// (v2/second_try.cpp:44-50, v4/mpi_bas.cpp:42-64, v4/comp.cu:99).
//
// Per round (one side, or both in lockstep), each expanding side runs one level:
//   sparse (top-down): owners expand their frontier vertices; neighbours they
//     own are claimed on the spot, the rest become (v, parent) candidates
//     (each remote vertex offered once per search) exchanged with ONE
//     ncclAllGather; owners then claim the candidates addressed to them.
//   dense (bottom-up): the owned frontier bitmap slices are allgathered into a
//     full bitmap and every owner scans its unvisited vertices for a parent.
// The owner of a vertex holds both sides' visited bits and depths, so the
// meet test is local and exact; claimed counts / degree sums (ncclSum) and
// the meet key (ncclMin over length << 32 | vertex) are reduced in one
// grouped call per round.
// No host round trip per round: the round policy (sides, direction,
// termination) is computed ON THE DEVICE from the reduced values, identically
// on every rank, and the host enqueues K sparse rounds at a time with a
// fixed-capacity exchange; kernels of a round that is not needed become
// no-ops, and the host waits once per K rounds.  A round the speculative
// shape cannot carry (a dense level, or a frontier larger than the enqueued
// capacity) stalls the batch; the host then plans that round itself, sized
// exactly.  The path comes back with ONE allgather of the
// claimed (vertex, parent) pairs, walked on the device from an LDS table.
// MPI is not needed at runtime: the communicator is bootstrapped from a
// unique id distributed by MPI (mpi_bibfs), torch.distributed (bench.py) or
// any other channel.
#pragma once

#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "bibfs/graph.hpp"
#include "bibfs/result.hpp"

namespace bibfs {

// Group id of a collective backend, made on rank 0 and handed to every rank:
// "rccl" -> ncclGetUniqueId bytes; "ipc" -> the name of the IPC group's
// shared-memory control segment (comm.hpp: P processes on one GPU or several).
std::vector<uint8_t> dist_unique_id(const std::string& backend = "rccl");
int gpu_count();                         // visible HIP devices (0 when none / no driver)

namespace dist {
class Comm;  // collective backend (RCCL, or the in-process test group): csrc/dist/comm.hpp
}

struct DistLevelStats {
  int levels = 0;                  // side-levels expanded
  int rounds = 0, lockstep_rounds = 0;
  int sparse_levels = 0, dense_levels = 0, overflow_levels = 0;
  int count_syncs = 0;             // extra host round trips to size a candidate exchange
  int host_syncs = 0;              // host waits on the device in this search (all causes)
  int spec_rounds = 0;             // rounds enqueued speculatively (incl. no-op tails after the end)
  int plan_polls = 0;              // lookahead waits on the pinned plan word (no stream sync)
  int host_rounds = 0;             // rounds planned on the host (dense levels, oversized exchanges)
  int collectives = 0;             // RCCL calls issued (allgather + allreduce)
  uint64_t exchanged_bytes = 0;    // bytes this rank received from allgathers
  double comm_ms = 0.0;            // host wall time of the round loop (this rank)
  double device_ms = 0.0;          // device time from the first to the last op of the search (events)
  int path_collectives = 0;        // collectives spent reconstructing the path
  int solo_rounds = 0;             // rounds run by the one-workgroup solo kernel (one rank)
  int cont_rounds = 0;             // continuation rounds: candidates that overflowed an owner block re-offered
  int pipelined = 0;               // 1: the search started with pipelined plans (DistTuning::pipeline, no hubs)
  int pipe_drains = 0;             // pipelined searches that stalled and continued with exact plans
  int pipe_retries = 0;            // pipelined searches answered again with exact plans (a spill list overflowed)
  int dev_sync_rounds = 0;         // speculative rounds whose exchange was ordered on the device (DistTuning::dev_sync)
  int single_engine = 0;           // world size 1: answered by the single-GPU engine (DistTuning::world1_single)
  // DistTuning::stamps: the speculative rounds split by device stamps (sums
  // over the stamped rounds, microseconds): expansion kernel(s), claim kernel,
  // expansion end -> claim start (candidate exchange + launch gap), claim end
  // -> next expansion start (status allgather + launch gap)
  int stamped_rounds = 0;
  double expand_us = 0.0, claim_us = 0.0, exchange_us = 0.0, status_us = 0.0;
  // the path gather's walk kernel (stamped searches): LDS tables built / both chains walked
  double walk_insert_us = 0.0, walk_chain_us = 0.0;
  // ... of them, the rounds that took the one-workgroup small paths, by phase:
  // expansion = plan (entry -> planned) + stage (frontier staged, degree
  // prefix) + edges + end (headers, state); claim = claims + end
  int small_expand_rounds = 0, small_claim_rounds = 0;
  double sx_plan_us = 0.0, sx_stage_us = 0.0, sx_edges_us = 0.0, sx_end_us = 0.0;
  double sx_staging_us = 0.0;      // ... of sx_plan_us: entry -> previous plan + reductions staged in LDS
  double sc_claims_us = 0.0, sc_end_us = 0.0;
};

// Knobs of the partitioned engine (defaults are the production settings; the
// small-capacity ones exist so tests can force every exchange branch).
struct DistTuning {
  int spec_rounds = 1;             // lookahead: rounds enqueued ahead of the last plan the host saw (0 = host plans every round)
  uint32_t spec_cap_max = 1u << 16;  // largest per-rank candidate block of a speculative round (pairs)
  uint32_t cap = 0;                // per-rank candidate block of a host-planned round (0 = min(2^20, n))
  uint64_t nosync_bytes = 1u << 20;  // host-planned round: size the exchange from host bounds up to this
  double timeout_s = 120.0;        // a host wait longer than this aborts the communicator and throws
  uint32_t walk_max = 15000;       // path from one gathered parent table when both sides claimed <= this
  bool solo = true;                // one rank: small rounds in one persistent workgroup (k_spec_solo)
  uint32_t solo_edges = 2048;      // ... while every expanding side has at most this many frontier edges (<= 8192)
  uint32_t owner_cap = 0;          // > 1 rank: pairs per owner-addressed block (0 = predicted per round)
  uint32_t spec_stall_edges = 0;   // a speculative round above this many per-rank frontier edges stalls for a
                                   // host-planned round (0 = only when the spill lists could overflow)
  bool pipeline = true;            // > 1 rank: ONE collective per speculative round -- each round's reduction
                                   // travels with the next round's candidate exchange and every plan accounts
                                   // the round before the last (with spec_rounds == 1 only);
                                   // false = exact plans, a status allgather per round
  bool dev_sync = true;            // 2..16 IPC ranks (processes) sharing one GPU: a round's claim kernel waits on
                                   // the peers' flags in a device window instead of a host rendezvous
                                   // (other transports ignore it)
  size_t hbm_cap_bytes = 0;        // > 0: a build that would make this rank hold more device memory throws
                                   // (tests: rehearse "does not fit one GPU" at small scale)
  bool world1_single = true;       // one rank: answer queries with the single-GPU engine over this rank's device
                                   // CSR (the whole graph; no copy), resident server included; false = the
                                   // partitioned rounds (solo workgroup + speculative rounds) at world size 1 too
  uint32_t spill_cap = 0;          // test hook: > 0 caps the candidate spill lists below their allocation while
                                   // the round-size guard keeps assuming the allocation -- a round can then
                                   // overflow them, which fails the search on every rank (the group lives on)
  bool stamps = false;             // per-round device stamps -> DistLevelStats::{expand,claim,exchange,status}_us
                                   // (adds one host wait + a copy per search: diagnostics, not serving)
};

class DistBiBfs {
 public:
  // backend "rccl" (one process per GPU) or "ipc" (processes may share a GPU)
  DistBiBfs(int rank, int size, int device, const std::vector<uint8_t>& unique_id,
            const std::string& backend = "rccl");
  DistBiBfs(std::unique_ptr<dist::Comm> comm, int device);                          // any backend
  ~DistBiBfs();
  DistBiBfs(const DistBiBfs&) = delete;
  DistBiBfs& operator=(const DistBiBfs&) = delete;

  void load_edges(const EdgeList& el);          // every rank passes the same edge list
  void load_bin(const std::string& path);       // each rank streams the file, keeps its rows
  void generate_gnp(uint32_t n, double p, uint64_t seed);   // on device, owned rows only
  void generate_rmat(uint32_t n, uint64_t m, uint64_t seed, double a = 0.57, double b = 0.19,
                     double c = 0.19);

  // Collective: every rank calls it with the same arguments; every rank gets
  // the full result (hops + path).
  SearchResult search(vid_t src, vid_t dst, const SearchOptions& opt = {});
  // Lean serving call (collective like search): the hop count (-1 = no path)
  // and the path.  At world size 1 with world1_single it is the single-GPU
  // engine's own query() -- no SearchResult, no stats, no device switch -- so
  // a one-rank job serves at the single engine's latency.
  int64_t query(vid_t src, vid_t dst, std::vector<vid_t>* path);
  // true when query() is answered by the single-GPU engine without a
  // collective (bindings keep the GIL for it, like HipBiBfs.query)
  bool query_is_local() const;

  // Collective checks that need no copy of the whole graph anywhere:
  // validate_path -- every edge (path[i], path[i+1]) is looked up in the row
  // of path[i] by the rank that owns it, one sum-allreduce of the edges found
  // (plus endpoints and length); search_unidirectional -- a plain
  // level-synchronous BFS from src over the same partition (side 0 expands
  // alone, so its hop count is independent of the bidirectional meet rule).
  bool validate_path(vid_t src, vid_t dst, int64_t hops, const std::vector<vid_t>& path);
  SearchResult search_unidirectional(vid_t src, vid_t dst);

  void barrier();
  double allreduce_max(double x);
  void release();  // free the graph shard and search state (the communicator stays)

  void set_tuning(const DistTuning& t);
  const DistTuning& tuning() const;
  // Fault injection (tests): from the `at`-th enqueued round of a search on,
  // this rank throws (mode 1), stalls for 2 x timeout_s before throwing
  // (mode 2), or kills its own process (mode 3: multi-process backends).
  // mode 0 disarms.
  void inject_fault(int at, int mode);

  int rank() const;
  int size() const;
  uint32_t n() const;
  uint64_t m_input() const;
  uint64_t local_nnz() const;
  size_t shard_bytes() const;     // owned CSR rows: row offsets + columns
  // Measured device memory of the last build (devmem.hpp): the most this rank
  // held at once while building its CSR shard (generator / scan temporaries
  // included), the device's free-memory drop over that span (hipMemGetInfo
  // low-water mark: equal up to allocator granularity with one rank per GPU),
  // and what it holds now (shard + search state).
  size_t gen_peak_bytes() const;
  size_t gen_hbm_peak_bytes() const;
  size_t resident_bytes() const;
  uint32_t lo() const;
  uint32_t hi() const;
  const DistLevelStats& last_stats() const;
  const char* backend() const;  // "rccl", "ipc" or "local"

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

// Test harness: `ranks` ranks as threads of this process
// sharing `device`, exchanging through the in-process local group instead of
// RCCL.  Every rank loads `el` and answers `queries`; returns rank 0's results
// after checking that every rank returned the same hop counts and paths.
// `fault_rank` >= 0 arms inject_fault(fault_at, fault_mode) on that rank.
struct DistLocalFault {
  int rank = -1, at = 0, mode = 0;
};
std::vector<SearchResult> dist_local_run(int ranks, int device, const EdgeList& el,
                                         const std::vector<std::pair<vid_t, vid_t>>& queries,
                                         const SearchOptions& opt = {}, const DistTuning& tuning = {},
                                         const DistLocalFault& fault = {},
                                         std::vector<DistLevelStats>* stats = nullptr);

// Same harness, but every rank generates the graph on the device itself
// (kind "gnp": arg = p; kind "rmat": arg = edge count) and keeps only its
// vertex block's CSR rows -- the path the multi-GPU bench takes, so a
// CSR-sharded Kronecker graph can be rehearsed on one GPU.  Fills rank 0's
// wall time per query and the slowest rank's build time.
struct DistLocalTiming {
  double build_ms = 0.0;
  std::vector<double> query_ms;
  std::vector<uint64_t> local_nnz;  // per rank
  std::vector<uint64_t> shard_bytes, gen_peak_bytes;  // per rank
  std::vector<uint64_t> gen_hbm_peak_bytes, resident_bytes;  // per rank (devmem.hpp)
  std::vector<DistLevelStats> stats;  // rank 0, per query
  // verify > 0: per query, the distributed path check (1 valid, 0 invalid,
  // -1 no path), and for the first `verify` queries the hop count of a
  // unidirectional partitioned BFS (-2 = not run)
  std::vector<int> path_valid;
  std::vector<int64_t> uni_hops;
};
std::vector<SearchResult> dist_local_generate_run(int ranks, int device, const std::string& kind, uint32_t n,
                                                  double arg, uint64_t seed,
                                                  const std::vector<std::pair<vid_t, vid_t>>& queries,
                                                  const SearchOptions& opt, DistLocalTiming* timing,
                                                  const DistTuning& tuning = {}, int verify = 0);

}  // namespace bibfs
