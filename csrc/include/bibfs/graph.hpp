// Graph containers: edge list (the .bin on-disk format), CSR, 1-D partition.
//
// Reference parity: every reference engine builds its adjacency inline from the
// .bin edge list (v1/main-v1.cpp:35-40, v2/second_try.cpp:45-50,
// v3/bibfs_cuda_only.cu:89-99, v4/mpi_bas.cpp:45-57).  Here there is ONE
// builder (csrc/csr/csr.cpp on the host, csrc/hip/csr_device.hip on the GPU).
#pragma once

#include <cstdint>
#include <vector>

#include "bibfs/common.hpp"

namespace bibfs {

// Undirected edge list, exactly the payload of a .bin file:
// u32 N, u32 M, then M x (u32 u, u32 v)   (graphs/generate_graph.py:35-39).
struct EdgeList {
  uint32_t n = 0;
  std::vector<uint32_t> uv;  // 2*M entries: u0 v0 u1 v1 ...
  uint64_t m() const { return uv.size() / 2; }
};

// Symmetric CSR with 64-bit row offsets (so 2M may exceed 2^32).
struct Csr {
  uint32_t n = 0;
  uint64_t m_input = 0;            // undirected edges of the input (for GTEPS = M/t)
  std::vector<uint64_t> row_off;   // n + 1
  std::vector<uint32_t> col;       // row_off[n] directed entries
  uint64_t nnz() const { return col.size(); }
  uint64_t degree(vid_t v) const { return row_off[v + 1] - row_off[v]; }
};

struct CsrOptions {
  bool drop_self_loops = true;
  bool dedup = false;     // sort + unique each row (needed only for multigraph inputs)
  bool sort_rows = false; // deterministic neighbour order
  int threads = 0;        // 0 = hardware concurrency
};

// 1-D block vertex partition: rank r owns [lo, hi) with lo = floor(r*n/P).
// The reference partitions cyclically (u % size == rank, v2/second_try.cpp:71,
// v4/comp.cu:27); a block partition keeps owned rows contiguous so a rank can
// hold only its own CSR rows and its own bitmap segment.
struct Partition {
  int rank = 0, size = 1;
  uint32_t n = 0, lo = 0, hi = 0;
  static Partition block(uint32_t n, int rank, int size) {
    Partition p;
    p.rank = rank;
    p.size = size;
    p.n = n;
    p.lo = (uint32_t)((uint64_t)n * rank / size);
    p.hi = (uint32_t)((uint64_t)n * (rank + 1) / size);
    return p;
  }
  uint32_t lo_of(int r) const { return (uint32_t)((uint64_t)n * r / size); }
  int owner(vid_t v) const {
    // smallest r with lo_of(r+1) > v
    int r = (int)(((uint64_t)v * size) / (n ? n : 1));
    while (r > 0 && lo_of(r) > v) --r;
    while (r + 1 < size && lo_of(r + 1) <= v) ++r;
    return r;
  }
  uint32_t count() const { return hi - lo; }
  bool owns(vid_t v) const { return v >= lo && v < hi; }
};

// Build the full symmetric CSR (each input edge stored in both directions).
Csr build_csr(const EdgeList& el, const CsrOptions& opt = {});

// Build only the rows owned by `part` (row i of the result is vertex part.lo+i;
// column ids stay global).
Csr build_csr_rows(const EdgeList& el, const Partition& part, const CsrOptions& opt = {});

// Edge list back from a CSR (each undirected edge once, u < v order not kept).
EdgeList csr_to_edges(const Csr& g);

}  // namespace bibfs
