// On-disk formats (API surface preserved from the reference):
//  * .bin edge list: little-endian u32 N, u32 M, M x (u32 u, u32 v)
//    writer graphs/generate_graph.py:35-39, readers v1/main-v1.cpp:26-30 etc.
//  * .json sidecar: {"source", "target", "hop_count" (int|null), "nodes"}
//    graphs/generate_graph.py:53-62.
//  * legacy dense matrix: u32 N + N*N u8 (v2/read_in.cpp:7-24).
//  * .csr cache (new): magic "BBFSCSR1", u32 n, u64 m_input, u64 nnz,
//    (n+1) x u64 row_off, nnz x u32 col -- lets end-to-end runs skip the
//    edge-list -> CSR step (SURVEY.md §5 checkpoint row).
#pragma once

#include <optional>
#include <string>
#include <vector>

#include "bibfs/graph.hpp"

namespace bibfs {

struct BinHeader {
  uint32_t n = 0, m = 0;
};

BinHeader read_bin_header(const std::string& path);
// Validates header against the file size ("Unexpected EOF", v1/main-v1.cpp:31-34)
// and every endpoint against N (the reference does not: out-of-range ids are UB there).
EdgeList read_bin(const std::string& path);
void write_bin(const std::string& path, const EdgeList& el);

// Stream the file and keep only edges with at least one endpoint in [lo, hi):
// the per-rank shard read of the partitioned engines (no rank-0 broadcast of
// the whole edge list, unlike v2/second_try.cpp:44 and v4/mpi_bas.cpp:42).
EdgeList read_bin_shard(const std::string& path, uint32_t lo, uint32_t hi);

struct PathJson {
  int64_t source = 0, target = 0;
  std::optional<int64_t> hop_count;  // null when unreachable
  std::vector<int64_t> nodes;
};
void write_path_json(const std::string& path, const PathJson& pj);
PathJson read_path_json(const std::string& path);
// "<stem>.json" next to "<stem>.bin" (graphs/generate_graph.py:54-55 splits on the first '.').
std::string sidecar_path(const std::string& bin_path);

struct DenseMatrix {
  uint32_t n = 0;
  std::vector<uint8_t> a;  // n*n row-major
};
DenseMatrix read_dense(const std::string& path);
void write_dense(const std::string& path, const DenseMatrix& m);

void write_csr_cache(const std::string& path, const Csr& g);
Csr read_csr_cache(const std::string& path);

}  // namespace bibfs
