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
// Per level (side s, chosen identically on every rank from allreduced stats):
//   sparse (top-down): owners expand their frontier vertices; neighbours they
//     own are claimed on the spot, the rest become (v, parent) candidates that
//     are exchanged with ONE ncclAllGather sized to the largest contribution;
//     owners then claim the candidates addressed to them.
//   dense (bottom-up): the owned frontier bitmap slices are allgathered into a
//     full bitmap and every owner scans its unvisited vertices for a parent.
//   The owner of a vertex holds both sides' visited bits, so the meet test is
//   local; {claimed count, claimed degree sum} (ncclSum) and the meet vertex
//   (ncclMin) are reduced in one grouped call.
// MPI is not needed at runtime: the communicator is bootstrapped from a
// unique id distributed by MPI (mpi_bibfs), torch.distributed (bench.py) or
// any other channel.
#pragma once

#include <memory>
#include <string>
#include <vector>

#include "bibfs/graph.hpp"
#include "bibfs/result.hpp"

namespace bibfs {

std::vector<uint8_t> dist_unique_id();  // ncclGetUniqueId as bytes

struct DistLevelStats {
  int levels = 0, sparse_levels = 0, dense_levels = 0, overflow_levels = 0;
  uint64_t candidates_sent = 0;   // this rank
  double comm_ms = 0.0;           // host-visible time in collectives (this rank)
};

class DistBiBfs {
 public:
  DistBiBfs(int rank, int size, int device, const std::vector<uint8_t>& unique_id);
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

  void barrier();
  double allreduce_max(double x);

  int rank() const;
  int size() const;
  uint32_t n() const;
  uint64_t m_input() const;
  uint64_t local_nnz() const;
  uint32_t lo() const;
  uint32_t hi() const;
  const DistLevelStats& last_stats() const;

 private:
  struct Impl;
  std::unique_ptr<Impl> p_;
};

}  // namespace bibfs
