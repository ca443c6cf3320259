// CPU engines: the serial bidirectional BFS (v1 capability, C1 in SURVEY.md)
// and a plain single-source BFS oracle used by tests and by the CLIs'
// --verify flag.
#pragma once

#include <vector>

#include "bibfs/graph.hpp"
#include "bibfs/result.hpp"

namespace bibfs {

// Serial level-synchronous bi-BFS over a CSR.  Same algorithm family as
// v1/main-v1.cpp:50-81 (expand one side per level, stop at the first vertex
// claimed by both sides, reconstruct through both parent chains) with the
// reference's src == dst bug fixed (v1 prints 2 hops) and
// no O(N) re-initialisation between queries: only the vertices a query
// touched are reset (their ids are already in the per-side queues).
class SerialBiBfs {
 public:
  explicit SerialBiBfs(const Csr& g);
  SearchResult search(vid_t src, vid_t dst, const SearchOptions& opt = {});

 private:
  const Csr& g_;
  std::vector<uint8_t> vis_[2];
  std::vector<vid_t> parent_[2];
  std::vector<vid_t> queue_[2];  // all claimed vertices, BFS order (frontier = tail segment)
};

// Plain BFS from src (early exit at dst); the independent oracle of the tests.
SearchResult bfs_oracle(const Csr& g, vid_t src, vid_t dst);

// Full single-source distances (-1 = unreachable).
std::vector<int64_t> bfs_distances(const Csr& g, vid_t src);

// True when `path` is a valid src->dst walk of `hops` edges in g.
bool validate_path(const Csr& g, vid_t src, vid_t dst, int64_t hops, const std::vector<vid_t>& path,
                   std::string* why = nullptr);

}  // namespace bibfs
