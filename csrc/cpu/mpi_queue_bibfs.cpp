// MPI frontier-list bidirectional BFS (C4 capability).  See include/bibfs/mpi_engines.hpp.
#include <algorithm>
#include <vector>

#include "bibfs/mpi_engines.hpp"

namespace bibfs {

SearchResult mpi_queue_bibfs(MPI_Comm comm, const Csr& g, vid_t src, vid_t dst, const SearchOptions& opt) {
  const double t0 = MPI_Wtime();
  int rank, size;
  MPI_Comm_rank(comm, &rank);
  MPI_Comm_size(comm, &size);
  SearchResult r;
  BIBFS_REQUIRE(src < g.n && dst < g.n, "src/dst out of range");
  if (src == dst) {  // main-v2.cpp:27-31
    r.found = true;
    r.hops = 0;
    r.meet = src;
    r.path = {src};
    r.total_ms = r.search_ms = (MPI_Wtime() - t0) * 1e3;
    return r;
  }
  std::vector<int32_t> dist[2];
  std::vector<vid_t> parent[2], front[2];
  for (int s = 0; s < 2; ++s) {
    dist[s].assign(g.n, -1);
    parent[s].assign(g.n, kNoVertex);
  }
  const vid_t root[2] = {src, dst};
  for (int s = 0; s < 2; ++s) {
    dist[s][root[s]] = 0;
    front[s].push_back(root[s]);
  }
  int64_t best = -1;
  vid_t best_v = kNoVertex;
  int turn = 0;
  std::vector<uint32_t> mine, all;
  std::vector<int> counts(size), displs(size);
  while (!front[0].empty() && !front[1].empty()) {
    int s;
    if (opt.side == SidePolicy::kAlternate) {
      s = turn;
      turn ^= 1;
    } else {
      s = front[0].size() <= front[1].size() ? 0 : 1;
    }
    const int o = s ^ 1;
    // cyclic split of the replicated frontier list (main-v2.cpp:47,89)
    mine.clear();
    uint64_t insp = 0;
    for (size_t i = (size_t)rank; i < front[s].size(); i += (size_t)size) {
      const vid_t u = front[s][i];
      for (uint64_t k = g.row_off[u]; k < g.row_off[u + 1]; ++k) {
        const vid_t v = g.col[k];
        ++insp;
        if (dist[s][v] >= 0) continue;
        mine.push_back(v);
        mine.push_back(u);
      }
    }
    int c = (int)mine.size();
    MPI_Allgather(&c, 1, MPI_INT, counts.data(), 1, MPI_INT, comm);  // main-v2.cpp:59
    int tot = 0;
    for (int q = 0; q < size; ++q) {
      displs[q] = tot;
      tot += counts[q];
    }
    all.resize((size_t)tot);
    MPI_Allgatherv(mine.data(), c, MPI_UINT32_T, all.data(), counts.data(), displs.data(), MPI_UINT32_T,
                   comm);  // main-v2.cpp:67-68
    uint64_t ginsp = 0;
    MPI_Allreduce(&insp, &ginsp, 1, MPI_UINT64_T, MPI_SUM, comm);
    r.stats.edges_inspected += ginsp;
    r.stats.levels++;
    // deterministic merge in rank order: every rank ends with identical state
    std::vector<vid_t> nf;
    for (int i = 0; i + 1 < tot; i += 2) {
      const vid_t v = all[(size_t)i], u = all[(size_t)i + 1];
      if (dist[s][v] >= 0) continue;
      dist[s][v] = dist[s][u] + 1;
      parent[s][v] = u;
      nf.push_back(v);
      if (dist[o][v] >= 0) {  // candidate-min meet rule (main-v2.cpp:73-79)
        const int64_t cand = (int64_t)dist[s][v] + dist[o][v];
        if (best < 0 || cand < best) {
          best = cand;
          best_v = v;
        }
      }
    }
    front[s].swap(nf);
    if (best >= 0) break;
  }
  // found flag + candidate agree on every rank (main-v2.cpp:82-83 reduce them with LOR / MIN)
  int64_t gbest;
  MPI_Allreduce(&best, &gbest, 1, MPI_INT64_T, MPI_MAX, comm);
  if (gbest >= 0) {
    r.found = true;
    r.hops = best;
    r.meet = best_v;
    if (opt.want_path) {
      std::vector<vid_t> a, b;
      for (vid_t x = best_v; x != kNoVertex; x = parent[0][x]) a.push_back(x);
      for (vid_t x = best_v; x != kNoVertex; x = parent[1][x]) b.push_back(x);
      r.path.assign(a.rbegin(), a.rend());
      r.path.insert(r.path.end(), b.begin() + 1, b.end());
    }
  }
  uint64_t v = 0;
  for (int s = 0; s < 2; ++s)
    for (vid_t x = 0; x < g.n; ++x) v += dist[s][x] >= 0;
  r.stats.visited = v;
  r.total_ms = r.search_ms = (MPI_Wtime() - t0) * 1e3;
  return r;
}

}  // namespace bibfs
