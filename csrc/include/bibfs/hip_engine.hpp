// Single-GPU bidirectional BFS engine for MI355X (v3 capability, C7/K1/K2 in
// SURVEY.md, re-designed for CDNA4; see docs/DESIGN.md).
//
// Two tiers, chosen per level on the device:
//  * LDS engine: ONE persistent 1024-thread workgroup runs the whole search in
//    a single launch.  Both visited sets live in LDS hash tables, both
//    frontiers (with their CSR row offsets prefetched) live in LDS, the meet
//    test is fused into the claim, and no global atomics are issued (a global
//    atomic with return costs ~1,700 cycles on gfx950, an LDS CAS ~100).  On
//    reference-shape graphs (G(n, 2.2/n)) the entire search runs here.
//  * Grid engine: when a frontier outgrows LDS, state is handed off to
//    device-wide top-down (load-balanced, wave-aggregated queue appends) and
//    bottom-up (bitmap, early exit, ballot-built words) kernels with a Beamer
//    direction switch.  This serves RMAT/Kronecker graphs.
// Header is HIP-free (pimpl) so g++-built tools and bindings can include it.
#pragma once

#include <memory>

#include "bibfs/graph.hpp"
#include "bibfs/result.hpp"

namespace bibfs {

struct DeviceInfo {
  std::string name;
  std::string arch;
  int cus = 0;
  size_t hbm_bytes = 0;
  int lds_bytes = 0;
};

class HipBiBfs {
 public:
  explicit HipBiBfs(int device = 0);
  ~HipBiBfs();
  HipBiBfs(const HipBiBfs&) = delete;
  HipBiBfs& operator=(const HipBiBfs&) = delete;

  // --- graph ingest -------------------------------------------------------
  void load_csr(const Csr& g);                 // upload a host CSR
  // Serve a CSR that already lives on this device (u64 row offsets, u32
  // columns, both directions): no copy; the caller keeps ownership and must
  // keep it alive until release() / destruction (the partitioned engine at
  // world size 1 hands its shard -- the whole graph -- to this engine).
  void adopt_device_csr(uint32_t n, uint64_t nnz, uint64_t m_input, uint64_t* d_row_off, uint32_t* d_col);
  void load_edges(const EdgeList& el);         // upload edges, build CSR on device
  void generate_gnp(uint32_t n, double p, uint64_t seed);                // on device
  void generate_rmat(uint32_t n, uint64_t m, uint64_t seed, double a = 0.57, double b = 0.19,
                     double c = 0.19);                                     // on device
  void release();                              // free the graph and all search state (HBM)
  uint32_t n() const;
  uint64_t nnz() const;
  uint64_t m_input() const;
  double last_build_ms() const;                // device time of the last ingest
  size_t device_bytes() const;                 // HBM held by graph + search state

  // --- search ---------------------------------------------------------------
  SearchResult search(vid_t src, vid_t dst, const SearchOptions& opt = {});
  // Serving entry point: hop count (-1 = no path) and, when path != nullptr,
  // the path src .. dst.  Small graphs (n <= 2^17) are answered by the
  // resident tiny server (csrc/hip/tiny_engine.hip) when resident serving is
  // on; everything else, and queries that outgrow it, by search().
  int64_t query(vid_t src, vid_t dst, std::vector<vid_t>* path);
  double last_search_ms() const;         // device time of the last query()
  uint64_t last_edges_inspected() const;
  bool tiny_engine() const;              // the loaded graph has the tiny server's packed adjacency
  uint64_t tiny_overflows() const;       // queries the tiny server handed back to the general engine (cumulative)
  // Host-path stamps of query() on the tiny server (diagnostics): on = reset
  // and start; host_stamps() = {queries, then mean microseconds of: entry ->
  // request posted, posted -> first answer packet seen, -> every packet
  // read, -> return}.
  void set_host_stamps(bool on);
  std::vector<double> host_stamps() const;

  // Throughput serving: answer K queries with one launch, one workgroup (one
  // CU) per query, up to 256 in flight.  Same results as K search() calls.
  // Queries whose visited sets outgrow LDS get a second batched pass with
  // HBM bitmaps (one 256-thread workgroup each); a query with a level above
  // `batch_edge_cap` edges, or a path longer than the batch path slot, is
  // re-run through search().
  std::vector<SearchResult> search_batch(const std::vector<vid_t>& src, const std::vector<vid_t>& dst,
                                         const SearchOptions& opt = {});
  void set_batch_edge_cap(uint64_t edges);
  uint64_t batch_edge_cap() const;
  // Queries of the last search_batch call that fell back to search() (a level
  // above batch_edge_cap, a path longer than the slot, or a failed pass).
  uint64_t last_batch_fallbacks() const;
  // lds_first: 1 = LDS pass first, 0 = HBM-bitmap pass only, -1 = auto (by n);
  // threads: HBM-pass workgroup size 256 / 1024, 0 = auto (by query count)
  void set_batch_tuning(int lds_first, int threads);

  // Resident query server: one workgroup stays on the GPU and takes queries
  // from a pinned mailbox, so a query costs no kernel launch.  It exits by
  // itself after `idle_ms` without a query (and is relaunched on demand),
  // and is stopped before any graph change or destruction.
  void set_resident(bool on, double idle_ms = 200.0);
  bool resident() const;
  // Device hand-off (default on; env BIBFS_AUTO_HANDOFF=0 sets the default
  // off): a resident search enqueues its first grid level before the search
  // starts, gated on the device, so a search that outgrows LDS continues
  // without a host round trip (docs/DESIGN.md §3).
  void set_auto_handoff(bool on);
  bool auto_handoff() const;
  // How long the device-gated first grid level waits for its search to leave
  // LDS (default 6 s); hand-offs it missed continue on the host (counted).
  void set_auto_gate_timeout_us(double us);
  double auto_gate_timeout_us() const;
  uint64_t auto_gate_misses() const;
  // Device-planned grid levels chained behind the hand-off (1-8, default 1):
  // each level's finisher plans the next one, so a
  // search that needs that many grid levels never waits for the host.
  void set_auto_levels(int levels);
  int auto_levels() const;
  // The device hand-off runs on graphs whose largest degree is at most this
  // (default 64: hub graphs keep host-planned levels).
  void set_auto_max_degree(uint64_t deg);
  uint64_t auto_max_degree() const;
  // Meet probe of the LDS engine (hub graphs, largest degree > 64): before a
  // level that does not fit LDS is handed to the grid engine, up to this many
  // of its frontier edges are tested against the other side's visited set;
  // any hit ends the search with the shortest length (default 16384; 0 = off).
  void set_lds_probe_edges(uint32_t edges);
  uint32_t lds_probe_edges() const;
  // Build-time flags, applied by the next load / generate: wide_offsets keeps
  // no 32-bit row-offset copy (a small graph then runs the nnz >= 2^32
  // kernels; tests), stream_gen generates even small graphs straight into the
  // CSR (the large-graph path; tests), tiny = false keeps the tiny server off
  // (the general resident server answers every graph; benchmarks).
  void set_build_flags(bool wide_offsets, bool stream_gen, bool tiny = true);

  // --- step-wise API (parity with the reference's per-level C API,
  //     v4/comp.h:8-36: init frontiers, expand one side, check intersection)
  void begin(vid_t src, vid_t dst);
  // Expands one level of `side` with the grid engine; returns number of newly
  // claimed vertices (0 = frontier died).  *met set when the sides met.
  uint64_t expand(int side, bool* met, Direction dir = Direction::kTopDown);
  bool check_meet();                    // bitmap AND over all words (K2/K4 parity)
  SearchResult finish();                // path reconstruction + cleanup

  // --- introspection for tests --------------------------------------------
  Csr download_csr() const;
  std::vector<vid_t> neighbors(vid_t u) const;  // one CSR row, copied from the device
  EdgeList download_edges() const;      // edges of the last generate_* call
  int device() const;
  DeviceInfo info() const;
  void* stream() const;                 // hipStream_t
  void synchronize() const;

 private:
  SearchResult search_general(vid_t src, vid_t dst, const SearchOptions& opt);
  struct Impl;
  std::unique_ptr<Impl> p_;
};

}  // namespace bibfs
