// MPI bitmap bidirectional BFS (C3 capability).  See include/bibfs/mpi_engines.hpp.
#include <algorithm>
#include <chrono>
#include <cstring>
#include <vector>

#include "bibfs/io.hpp"
#include "bibfs/mpi_engines.hpp"

namespace bibfs {

EdgeList mpi_bcast_edges(MPI_Comm comm, const std::string& path) {
  int rank;
  MPI_Comm_rank(comm, &rank);
  EdgeList el;
  uint64_t hdr[2] = {0, 0};
  int ok = 1;
  std::string err;
  if (rank == 0) {
    try {
      el = read_bin(path);
      hdr[0] = el.n;
      hdr[1] = el.m();
    } catch (const std::exception& e) {
      ok = 0;
      err = e.what();
    }
  }
  MPI_Bcast(&ok, 1, MPI_INT, 0, comm);
  if (!ok) throw Error(rank == 0 ? err : "rank 0 failed to read " + path);
  MPI_Bcast(hdr, 2, MPI_UINT64_T, 0, comm);
  el.n = (uint32_t)hdr[0];
  el.uv.resize(2 * hdr[1]);
  // chunked broadcast (MPI counts are int)
  const uint64_t total = el.uv.size();
  const uint64_t step = 1ULL << 28;
  for (uint64_t off = 0; off < total; off += step)
    MPI_Bcast(el.uv.data() + off, (int)std::min(step, total - off), MPI_UINT32_T, 0, comm);
  return el;
}

SearchResult mpi_bitmap_bibfs(MPI_Comm comm, const Csr& rows, const Partition& part, vid_t src, vid_t dst,
                              const SearchOptions& opt) {
  const double t0 = MPI_Wtime();
  SearchResult r;
  const uint32_t n = part.n;
  BIBFS_REQUIRE(src < n && dst < n, "src/dst out of range");
  if (src == dst) {
    r.found = true;
    r.hops = 0;
    r.meet = src;
    r.path = {src};
    r.total_ms = r.search_ms = (MPI_Wtime() - t0) * 1e3;
    return r;
  }
  const uint64_t L = ((uint64_t)n + 63) / 64;
  std::vector<uint64_t> front[2], vis[2], next(L);
  std::vector<vid_t> parent[2];
  for (int s = 0; s < 2; ++s) {
    front[s].assign(L, 0);
    vis[s].assign(L, 0);
    parent[s].assign(n, kNoVertex);
  }
  const vid_t root[2] = {src, dst};
  for (int s = 0; s < 2; ++s) {
    front[s][root[s] >> 6] |= 1ULL << (root[s] & 63);
    vis[s][root[s] >> 6] |= 1ULL << (root[s] & 63);
  }
  // owned word range for the scans (block partition, rounded to words)
  const uint64_t wlo = part.lo / 64, whi = std::min<uint64_t>(L, ((uint64_t)part.hi + 63) / 64);
  uint64_t cnt[2] = {1, 1};
  int depth[2] = {0, 0}, turn = 0;
  vid_t meet = kNoVertex;
  for (;;) {
    int s;
    if (opt.side == SidePolicy::kAlternate) {
      s = turn;
      turn ^= 1;
    } else {
      s = cnt[0] <= cnt[1] ? 0 : 1;  // frontier vertex counts are what the bitmaps give cheaply
    }
    const int o = s ^ 1;
    std::fill(next.begin(), next.end(), 0ULL);
    uint64_t insp = 0;
    for (uint64_t w = wlo; w < whi; ++w) {
      uint64_t bits = front[s][w];
      while (bits) {
        const int b = __builtin_ctzll(bits);
        bits &= bits - 1;
        const vid_t u = (vid_t)(w * 64 + b);
        if (!part.owns(u)) continue;
        const uint32_t lu = u - part.lo;
        for (uint64_t k = rows.row_off[lu]; k < rows.row_off[lu + 1]; ++k) {
          const vid_t v = rows.col[k];
          const uint64_t m = 1ULL << (v & 63);
          ++insp;
          if ((vis[s][v >> 6] | next[v >> 6]) & m) continue;
          next[v >> 6] |= m;
          parent[s][v] = u;
        }
      }
    }
    // merge: every rank gets the union of discoveries (v2/second_try.cpp:82-85)
    MPI_Allreduce(MPI_IN_PLACE, next.data(), (int)L, MPI_UINT64_T, MPI_BOR, comm);
    uint64_t local[2] = {0, insp};
    vid_t lmeet = kNoVertex;
    for (uint64_t w = 0; w < L; ++w) {
      const uint64_t nw = next[w] & ~vis[s][w];
      front[s][w] = nw;
      vis[s][w] |= nw;
      if (w >= wlo && w < whi) {
        local[0] += (uint64_t)__builtin_popcountll(nw);
        const uint64_t hit = nw & vis[o][w];
        if (hit && lmeet == kNoVertex) lmeet = (vid_t)(w * 64 + __builtin_ctzll(hit));
      }
    }
    uint64_t glob[2];
    MPI_Allreduce(local, glob, 2, MPI_UINT64_T, MPI_SUM, comm);
    vid_t gmeet;
    MPI_Allreduce(&lmeet, &gmeet, 1, MPI_UINT32_T, MPI_MIN, comm);
    ++depth[s];
    r.stats.levels++;
    r.stats.edges_inspected += glob[1];
    cnt[s] = glob[0];
    if (gmeet != kNoVertex) {
      meet = gmeet;
      break;
    }
    if (glob[0] == 0) break;  // either frontier empty => unreachable ('||', not v2's '&&')
  }
  if (meet != kNoVertex) {
    r.found = true;
    r.meet = meet;
    r.hops = depth[0] + depth[1];
    if (opt.want_path) {
      // walk both chains; any rank that recorded a parent supplies it (MIN)
      std::vector<vid_t> a{meet}, b{meet};
      vid_t cur[2] = {meet, meet};
      for (int i = 0; i < std::max(depth[0], depth[1]); ++i) {
        vid_t cand[2];
        for (int q = 0; q < 2; ++q) cand[q] = (i < depth[q] && cur[q] != root[q]) ? parent[q][cur[q]] : cur[q];
        vid_t red[2];
        MPI_Allreduce(cand, red, 2, MPI_UINT32_T, MPI_MIN, comm);
        for (int q = 0; q < 2; ++q)
          if (i < depth[q]) {
            cur[q] = red[q];
            (q ? b : a).push_back(red[q]);
          }
      }
      r.path.assign(a.rbegin(), a.rend());
      r.path.insert(r.path.end(), b.begin() + 1, b.end());
    }
  }
  uint64_t vis_cnt = 0;
  for (int s = 0; s < 2; ++s)
    for (uint64_t w = wlo; w < whi; ++w) vis_cnt += (uint64_t)__builtin_popcountll(vis[s][w]);
  MPI_Allreduce(MPI_IN_PLACE, &vis_cnt, 1, MPI_UINT64_T, MPI_SUM, comm);
  r.stats.visited = vis_cnt;
  r.total_ms = r.search_ms = (MPI_Wtime() - t0) * 1e3;
  return r;
}

}  // namespace bibfs
