// Host side of the single-GPU engine: graph residency, search dispatch
// (LDS persistent engine -> optional hand-off to the grid engine), pinned
// result delivery, and the step-wise C-API-style interface.
//
// Reference parity: v3/bibfs_cuda_only.cu:128-234 (allocation, per-level
// host loop, cudaEvent timing) and v4/comp.cu:49-133 (device runtime API).
// Differences by design: device state is allocated once per graph and kept
// clean between queries, the per-level loop runs on the device, and the host
// learns the result by polling a pinned word instead of a memcpy + sync chain.
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "bibfs/hip_engine.hpp"
#include "bibfs/trace.hpp"
#include "device.hpp"

namespace bibfs {

using namespace dev;

struct HipBiBfs::Impl {
  int device = 0;
  hipStream_t stream = nullptr;
  hipDeviceProp_t prop{};
  int cus = 256;

  // graph
  uint32_t n = 0;
  uint64_t nnz = 0, m_input = 0;
  uint64_t* d_row_off = nullptr;
  uint32_t* d_row_off32 = nullptr;
  uint32_t* d_col = nullptr;
  uint4* d_padj = nullptr;   // packed adjacency (LDS engine), when it fits the budget
  unsigned long long* d_padj8 = nullptr;  // its 8-byte form (launch::pack8), instead of it where it fits
  uint64_t max_deg = 0;      // largest degree: no hub pass when it is below the hub degree
  uint32_t* d_uv = nullptr;  // last generated edge list (kept for small graphs / tests)
  uint64_t uv_m = 0;
  // graphs above this many undirected edges are generated straight into the
  // CSR (two passes over the counter-based generator, no edge list in HBM)
  static constexpr uint64_t kKeepEdges = 1ull << 26;
  bool force_stream_gen = false;  // (tests) stream-generate small graphs too: HipBiBfs::set_build_flags
  bool wide_offsets = false;      // (tests) no 32-bit row-offset copy: the nnz >= 2^32 kernels
  bool tiny_enabled = true;       // the tiny server for graphs it supports
  double build_ms = 0.0;

  // search state
  launch::SearchBuffers buf{};
  void* state_block = nullptr;  // one allocation holding every per-search array (state set 0)
  void* state_block_alt = nullptr;  // state set 1 (resident queries alternate)
  size_t state_bytes_alt = 0;
  size_t state_bytes = 0;
  uint32_t* d_flag = nullptr;     // [0] bitmap-meet flag, [4] election ticket, [8] cleanup done counter
  uint32_t* h_clean = nullptr;    // pinned: tag of the last finished k_cleanup
  uint32_t clean_seq = 0;
  // two search-state sets: resident queries alternate between them, so a
  // search never shares global state with the previous search's cleanup
  launch::SearchBuffers bufs[2]{};
  int cur = 0;
  uint32_t clean_tag[2] = {0, 0};  // last cleanup enqueued on each set
  bool grid_cleaned = false;  // the search's last grid level enqueued the cleanup that ran

  // Device hand-off (grid_auto): on by default for resident searches of
  // graphs the general server takes, with the default level policy, when no
  // vertex has more than auto_max_deg edges; HipBiBfs::set_auto_handoff(false) turns it off
  // (A/B).  Hub graphs keep the host-planned first level: on Kronecker 22 the
  // auto level lost in three A/Bs (0.058-0.060 vs 0.054-0.057 ms) while
  // 10M G(n, p) gains ~1% (profiles/r3_auto_handoff_ab2.jsonl).
  // (set_auto_max_degree overrides the bound, for A/B on hub graphs: with the
  // hub pass sized like the host's it still lost on Kronecker 22, 71.6-72.2 vs
  // 47.2-49.8 us mean search, profiles/r4_auto_chain_ab.jsonl; with direct hub
  // levels planned on the device too, 50.8-52.6 vs 44.5-44.7 and Kronecker 25
  // 60.6 vs 51.0, profiles/r4_auto_hub_direct_ab.jsonl -- a gated chain of
  // k_handoff + top-down + 1024-block hub launches behind EVERY query costs
  // ~30 us of stream time, which the next query's hand-off queues behind)
  uint64_t auto_max_deg = 64;
  uint32_t probe_edges = launch::lds_probe_budget();  // LDS meet probe (HipBiBfs::set_lds_probe_edges)
  bool auto_on = true;
  // Device-planned grid levels chained behind the hand-off (the first one
  // planned by k_handoff, each further one by the finisher of the level before):
  // set_auto_levels, default 1.  Chains of 2 / 3 measured slower on 10M
  // G(n, p): 69.3-70.1 / 71.4 vs 67.1-67.2 us mean search -- the LDS phase
  // itself slows by ~2 us per chained level (the extra launches behind every
  // query) and the second level saves less than that
  // (profiles/r4_auto_chain_ab.jsonl).
  int auto_levels = 1;
  // (A lazy chain -- the host enqueuing the planned next level only after the
  // search handed off -- measured slower too: 10M 61.3 -> 64.0 us mean search,
  // profiles/r4_auto_lazy_ab.jsonl; removed.)
  bool auto_usable(const SearchOptions& opt) const {
    return auto_on && nnz > 0 && max_deg <= auto_max_deg && !opt.trace && !opt.force_grid &&
           opt.direction == Direction::kAuto && opt.side == SidePolicy::kSmallerEdges;
  }
  // k_handoff's gate wait limit (microseconds; set_auto_gate_timeout_us).
  // Longer than the host's 5 s server wait, so a late server does not strand
  // the auto chain; a wait that gives up anyway is recovered on the host.
  double auto_gate_us = 6e6;
  uint64_t auto_gate_misses = 0;  // hand-offs the auto chain missed (host fallback ran)
  // After an auto level's search handed off: wait for the auto level's result
  // (kAutoFinal), its mirror publish (kAutoMirror: the search continues on the
  // host), or the chain draining with neither (kAutoMissed: the gate wait gave
  // up before the search handed off -- no level ran, no scatter, no publish;
  // the caller continues from the LDS engine's own hand-off mirror).
  enum AutoOutcome { kAutoFinal, kAutoMirror, kAutoMissed };
  AutoOutcome wait_auto(uint32_t pub, uint32_t ls) {
    for (uint64_t it = 1;; ++it) {
      if (__atomic_load_n(&h_gres->seq, __ATOMIC_ACQUIRE) == pub) return kAutoFinal;
      if (__atomic_load_n(&h_state->pad[0], __ATOMIC_ACQUIRE) == ls) {
        return __atomic_load_n(&h_gres->seq, __ATOMIC_ACQUIRE) == pub ? kAutoFinal : kAutoMirror;
      }
      if ((it & 8191) == 0) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess && __atomic_load_n(&h_gres->seq, __ATOMIC_ACQUIRE) != pub &&
            __atomic_load_n(&h_state->pad[0], __ATOMIC_ACQUIRE) != ls)
          return kAutoMissed;
        if (e != hipSuccess && e != hipErrorNotReady)
          throw Error(std::string("bibfs: auto grid level failed: ") + hipGetErrorString(e));
      } else {
        _mm_pause();
      }
    }
  }
  uint32_t next_clean_tag() {
    clean_seq = clean_seq + 1 == 0 ? 1 : clean_seq + 1;
    return clean_seq;
  }

  // async cleanup of the global visited words; its tag lets the host order
  // the resident server's next hand-off (another stream) after it
  // tags increase and cleanups finish in stream order, so "done" is h_clean >= tag
  void cleanup_async(bool if_done = false) {
    clean_tag[cur] = next_clean_tag();
    launch::cleanup(buf, n, d_flag + 8, h_clean, clean_seq, if_done, stream);
  }
  void wait_tag(uint32_t tag) {
    if (!tag) return;
    for (uint64_t it = 1; (int32_t)(__atomic_load_n(h_clean, __ATOMIC_ACQUIRE) - tag) < 0; ++it) {
      if ((it & 8191) == 0) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess && (int32_t)(__atomic_load_n(h_clean, __ATOMIC_ACQUIRE) - tag) < 0)
          throw Error("bibfs: cleanup finished without its tag");
        if (e != hipSuccess && e != hipErrorNotReady)
          throw Error(std::string("bibfs: cleanup failed: ") + hipGetErrorString(e));
      } else {
        _mm_pause();
      }
    }
  }
  // Resident query: switch to the other state set and wait only for the
  // cleanup last enqueued on THAT set (two searches ago: normally long done).
  void flip_state_set() {
    ensure_alt_set();
    cur ^= 1;
    buf = bufs[cur];
    wait_tag(clean_tag[cur]);
    clean_tag[cur] = 0;
  }

  // pinned host memory
  HostResult* h_res = nullptr;
  // The grid levels of a search publish into `gres`: h_res, or for a search
  // with an auto level behind it h_gres -- a record of its own, so the auto
  // level never writes over the LDS answer the host is reading.
  HostResult* h_gres = nullptr;
  HostResult* gres = nullptr;
  uint32_t* h_path = nullptr;
  uint32_t h_path_cap = 1u << 20;
  DevState* h_state = nullptr;
  uint32_t seq = 0;
  int pin_xcc = 0;  // XCD that runs the LDS engine (-1 = wherever block 0 lands)

  hipEvent_t ev0 = nullptr, ev1 = nullptr;

  // batched search (k_lds_batch)
  uint32_t* d_bslots = nullptr;   // per slot parent[2] + queue[2]
  uint32_t* d_bq = nullptr;       // src[K], dst[K]
  HostResult* h_bres = nullptr;   // pinned
  uint32_t* h_bpath = nullptr;    // pinned, K * kBatchPath
  uint32_t* h_bq = nullptr;       // pinned staging for src/dst
  uint32_t bcap = 0;              // slots allocated
  uint64_t bedge_cap = 1ull << 20;  // batch_global: larger levels go to search()
  uint64_t batch_fallbacks = 0;     // last search_batch: queries re-run through search()
  int blds = -1;                    // batch: LDS pass first (1), never (0), auto (-1)
  int bthreads = 0;                 // batch_global workgroup size (256 / 1024), 0 = auto
  uint32_t* d_bbits = nullptr;    // per slot 2 visited bitmaps (batch_global), all-zero between launches
  uint32_t* h_bqidx = nullptr;    // pinned: queries handed to batch_global
  BatchOut* h_bout = nullptr;     // pinned: batch_global results
  static constexpr uint32_t kBatchPath = 4096;

  void free_batch() {
    if (d_bslots) HIP_CHECK(hipFree(d_bslots));
    if (d_bq) HIP_CHECK(hipFree(d_bq));
    if (h_bres) HIP_CHECK(hipHostFree(h_bres));
    if (h_bpath) HIP_CHECK(hipHostFree(h_bpath));
    if (h_bq) HIP_CHECK(hipHostFree(h_bq));
    if (d_bbits) HIP_CHECK(hipFree(d_bbits));
    if (h_bqidx) HIP_CHECK(hipHostFree(h_bqidx));
    if (h_bout) HIP_CHECK(hipHostFree(h_bout));
    d_bbits = h_bqidx = nullptr;
    h_bout = nullptr;
    d_bslots = d_bq = nullptr;
    h_bres = nullptr;
    h_bpath = h_bq = nullptr;
    bcap = 0;
  }

  void ensure_batch(uint32_t k) {
    if (k <= bcap) return;
    free_batch();
    HIP_CHECK(hipMalloc(&d_bslots, (size_t)k * 4 * n * sizeof(uint32_t)));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_bres), (size_t)k * sizeof(HostResult),
                            hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_bpath), (size_t)k * kBatchPath * sizeof(uint32_t),
                            hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_bq), (size_t)k * 2 * sizeof(uint32_t),
                            hipHostMallocMapped | hipHostMallocCoherent));  // read by the kernel directly
    std::memset(h_bres, 0, (size_t)k * sizeof(HostResult));
    HIP_CHECK(hipMalloc(&d_bbits, (size_t)k * 2 * buf.words * sizeof(uint32_t)));
    HIP_CHECK(hipMemsetAsync(d_bbits, 0, (size_t)k * 2 * buf.words * sizeof(uint32_t), stream));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_bqidx), (size_t)k * sizeof(uint32_t),
                            hipHostMallocMapped | hipHostMallocCoherent));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_bout), (size_t)k * sizeof(BatchOut),
                            hipHostMallocMapped | hipHostMallocCoherent));
    bcap = k;
  }

  // resident server (k_lds_server, or k_tiny_server for small graphs)
  hipStream_t sstream = nullptr;
  ServerBox* h_box = nullptr;
  bool resident = false;         // user setting
  bool srv_running = false;      // a server kernel was launched and has not been seen to exit
  int srv_kind = 0;              // kSrvLds / kSrvTiny: which server kernel is running
  uint32_t srv_launch_seq = 0;
  unsigned long long srv_idle_ticks = 20000000ull;  // 200 ms of s_memrealtime
  static constexpr int kSrvLds = 1, kSrvTiny = 2;

  // small-graph server (tiny_engine.hip): packed adjacency + self-tagged result packets
  unsigned long long* d_tadj = nullptr;
  unsigned long long* d_tinfo = nullptr;
  unsigned long long* d_tspill = nullptr;  // tiny server: records past its LDS buffers
  unsigned long long* d_stamps = nullptr;
  TinyPkt* h_pkts = nullptr;
  bool tiny_ok = false;
  // the last query answered (query() API)
  uint64_t tiny_overflows = 0;  // queries the tiny server handed back (re-run on the general engine)
  double last_ms = 0.0;
  uint64_t last_einsp = 0;
  static bool tiny_stamp() { return env::tiny_stamps(); }
  bool tiny_usable(const SearchOptions& opt) const {
    return tiny_ok && resident && !opt.trace && !opt.force_grid && opt.lockstep &&
           opt.direction == Direction::kAuto && opt.side == SidePolicy::kSmallerEdges;
  }

  // step-wise API
  int dir[2] = {1, 1};
  bool fbits_valid[2] = {false, false};
  vid_t step_src = 0, step_dst = 0;

  launch::GraphView view() const {
    return launch::GraphView{n, nnz, d_row_off, d_row_off32, d_col, d_padj, max_deg, d_padj8, probe_edges};
  }

  bool server_usable() const { return d_row_off32 != nullptr && n > 0 && n <= 0x7fffffffu; }  // batch kernel
  // the resident LDS server runs with 32- or 64-bit row offsets
  bool lds_server_usable() const { return n > 0 && n <= 0x7fffffffu; }

  // one aligned 16-byte store: the server reads the request with one load
  void post(uint32_t s, uint32_t src, uint32_t dst, uint32_t flags) {
    const __m128i v = _mm_set_epi32((int)req_tag(s, flags), (int)dst, (int)src, (int)s);
    _mm_store_si128(reinterpret_cast<__m128i*>(h_box), v);
    std::atomic_thread_fence(std::memory_order_seq_cst);
  }

  // Launch a server kernel of `kind`; it serves requests whose seq != last.
  void launch_kind(int kind, int pin, uint32_t last) {
    srv_launch_seq = ++seq == 0 ? ++seq : seq;
    HIP_CHECK(hipSetDevice(device));
    __atomic_store_n(&h_box->alive, 0u, __ATOMIC_RELEASE);
    if (kind == kSrvTiny) {
      launch::TinyArgs a{d_tadj, d_tinfo, n, h_box, h_box, h_pkts,
                         srv_launch_seq, last, pin, d_flag + 4, srv_idle_ticks, d_stamps, d_tspill};
      launch::tiny_server(a, tiny_stamp(), sstream);
    } else {
      launch::lds_server(view(), bufs[0], bufs[1], launch::HostSide{h_res, h_path, h_path_cap, h_state}, h_box,
                         srv_launch_seq, last, pin, d_flag + 4, srv_idle_ticks, env::server_stamps(), sstream);
    }
    srv_kind = kind;
    srv_running = true;
  }
  void launch_server(int pin) { launch_kind(kSrvLds, pin, __atomic_load_n(&h_box->seq, __ATOMIC_ACQUIRE)); }

  // Make a server of `kind` run (stopping the other kind first).
  void ensure_server(int kind) {
    if (srv_running && srv_kind != kind) stop_server();
    if (srv_running && __atomic_load_n(&h_box->alive, __ATOMIC_ACQUIRE) == ~srv_launch_seq)
      srv_running = false;  // idled out (a relaunch queues behind its last instructions)
    if (!srv_running) launch_kind(kind, pin_xcc, __atomic_load_n(&h_box->seq, __ATOMIC_ACQUIRE));
  }

  // Spin until done(); every 8192 spins check the deadline and that the
  // server still runs -- relaunching it (unpinned if no block reached the
  // pinned XCD) so the pending request qseq is served.
  template <class Done>
  void wait_server(int kind, uint32_t qseq, Done done) {
    const auto t0 = std::chrono::steady_clock::now();
    for (uint64_t it = 1;; ++it) {
      if (done()) return;
      if ((it & 8191) == 0) {
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
          char msg[512];
          std::snprintf(msg, sizeof msg,
                        "bibfs: resident server (kind %d) did not answer query %u in 5 s (alive %u launch %u)", kind,
                        qseq, h_box->alive, srv_launch_seq);
          std::fprintf(stderr, "%s\n", msg);
          post(++seq == 0 ? ++seq : seq, 0, 0, kReqStop);
          throw Error(msg);
        }
        const hipError_t e = hipStreamQuery(sstream);
        if (e == hipSuccess) {  // server gone: idle exit raced this query, or no block won the election
          if (done()) return;
          if (__atomic_load_n(&h_box->alive, __ATOMIC_ACQUIRE) != ~srv_launch_seq) pin_xcc = -1;
          srv_running = false;
          launch_kind(kind, pin_xcc, qseq - 1);
        } else if (e != hipErrorNotReady) {
          throw Error(std::string("bibfs: resident server failed: ") + hipGetErrorString(e));
        }
      } else {
        _mm_pause();
      }
    }
  }

  // One query through the small-graph server.  Returns kTinyFound /
  // kTinyNoPath / kTinyOverflow (the caller re-runs those on the general
  // engine); fills hops, meet, stats and, when path != nullptr, the path.
  struct TinyAnswer {
    uint32_t status = 0, levels = 0, hops = 0, meet = 0, ticks = 0, einsp = 0, visited = 0;
  };
  static bool read_pkt(const TinyPkt* p, uint32_t want, TinyPkt& out) {
    asm volatile("" ::: "memory");
    const __m128i v = _mm_load_si128(reinterpret_cast<const __m128i*>(p));  // one 16-byte load: a whole packet
    _mm_storeu_si128(reinterpret_cast<__m128i*>(&out), v);
    return out.seq == want;
  }
  void spin_pkt(const TinyPkt* p, uint32_t want, TinyPkt& out) {
    for (uint64_t it = 1; !read_pkt(p, want, out); ++it) {
      if ((it & 65535) == 0 && hipStreamQuery(sstream) == hipSuccess && !read_pkt(p, want, out))
        throw Error("bibfs: tiny server exited with an answer half written");
      _mm_pause();
    }
  }
  // Host-path stamps of the serving call (set_host_stamps(true)): steady-clock
  // nanoseconds summed over queries -- entry -> request posted, posted -> first
  // answer packet seen, -> all packets read, -> return to the binding.
  bool host_stamps_on = false;
  uint64_t hs_n = 0, hs_post = 0, hs_wait = 0, hs_read = 0, hs_tail = 0;
  std::chrono::steady_clock::time_point hs_t0, hs_t1, hs_t2, hs_t3;
  static uint64_t ns(std::chrono::steady_clock::duration d) {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(d).count();
  }
  uint32_t tiny_search(uint32_t src, uint32_t dst, std::vector<vid_t>* path, TinyAnswer& a) {
    ensure_server(kSrvTiny);
    const uint32_t qseq = ++seq == 0 ? ++seq : seq;
    post(qseq, src, dst, 0u);
    if (host_stamps_on) hs_t1 = std::chrono::steady_clock::now();
    TinyPkt p0, p1;
    wait_server(kSrvTiny, qseq, [&] { return read_pkt(h_pkts, qseq, p0); });
    if (host_stamps_on) hs_t2 = std::chrono::steady_clock::now();
    spin_pkt(h_pkts + 1, qseq, p1);
    a.status = p0.a & 0xffu;
    a.levels = p0.a >> 8;
    a.hops = p0.b;
    a.meet = p0.c;
    a.ticks = p1.a;
    a.einsp = p1.b;
    a.visited = p1.c;
    if (a.status == kTinyOverflow) ++tiny_overflows;
    if (a.status == kTinyFound && path) {
      const uint32_t plen = a.hops + 1;
      path->resize(plen);
      vid_t* out = path->data();
      for (uint32_t j = 0; 3 * j < plen; ++j) {
        TinyPkt pk;
        spin_pkt(h_pkts + 2 + j, qseq, pk);
        out[3 * j] = pk.a;
        if (3 * j + 1 < plen) out[3 * j + 1] = pk.b;
        if (3 * j + 2 < plen) out[3 * j + 2] = pk.c;
      }
    }
    if (host_stamps_on) hs_t3 = std::chrono::steady_clock::now();
    if (tiny_stamp()) {
      unsigned long long s[22];
      HIP_CHECK(hipMemcpy(s, d_stamps, sizeof s, hipMemcpyDeviceToHost));
      std::fprintf(stderr,
                   "[tiny] cycles: seed %llu single-wave %llu all-wave %llu (%llu rounds, %.0f/round) meet-scan %llu "
                   "walk %llu publish %llu | device %.2f us, %u levels, status %u\n",
                   s[1] - s[0], s[2] - s[1], s[3] - s[2], s[7], s[7] ? (double)(s[3] - s[2]) / (double)s[7] : 0.0,
                   s[4] ? s[4] - s[3] : 0ull, s[4] ? s[5] - s[4] : 0ull, s[6] - s[5], a.ticks * 0.01, a.levels, a.status);
      const double r = s[7] ? (double)s[7] : 1.0;
      std::fprintf(stderr,
                   "[tiny] per all-wave round (wave 0): plan %.0f claim %.0f scan+atomic %.0f place %.0f barrier %.0f "
                   "book %.0f\n",
                   s[8] / r, s[11] / r, s[12] / r, s[13] / r, s[14] / r, s[15] / r);
      const double w = s[16] ? (double)s[16] : 1.0;
      std::fprintf(stderr,
                   "[tiny] per single-wave round (%llu rounds, %.1f edges each): issue+claim %.0f count %.0f "
                   "place %.0f meet-read %.0f\n",
                   s[16], s[21] / w, s[17] / w, s[18] / w, s[19] / w, s[20] / w);
    }
    return a.status;
  }

  void stop_server() {
    if (!srv_running) return;
    const uint32_t s = ++seq == 0 ? ++seq : seq;
    post(s, 0, 0, kReqStop);
    HIP_CHECK(hipStreamSynchronize(sstream));
    srv_running = false;
  }

  // Post one query to the server; server_wait then waits for its answer (the
  // LDS engine answers every search, a hand-off included).
  void server_post(uint32_t src, uint32_t dst, const SearchOptions& opt, uint32_t qseq) {
    ensure_server(kSrvLds);
    post(qseq, src, dst, (opt.lockstep ? kReqLockstep : 0u) | ((uint32_t)opt.side & 3u) << 2 | (cur ? kReqAltBuf : 0u));
  }
  void server_wait(uint32_t qseq) {
    wait_server(kSrvLds, qseq, [&] { return __atomic_load_n(&h_res->seq, __ATOMIC_ACQUIRE) == qseq; });
  }

  bool borrowed_csr = false;  // d_row_off / d_col belong to the caller (adopt_device_csr)
  void free_graph() {
    stop_server();
    free_batch();
    if (borrowed_csr) {
      d_row_off = nullptr;
      d_col = nullptr;
      borrowed_csr = false;
    }
    if (d_row_off) HIP_CHECK(hipFree(d_row_off));
    if (d_row_off32) HIP_CHECK(hipFree(d_row_off32));
    if (d_col) HIP_CHECK(hipFree(d_col));
    if (d_padj) HIP_CHECK(hipFree(d_padj));
    if (d_padj8) HIP_CHECK(hipFree(d_padj8));
    if (d_tadj) HIP_CHECK(hipFree(d_tadj));
    if (d_tinfo) HIP_CHECK(hipFree(d_tinfo));
    if (d_tspill) HIP_CHECK(hipFree(d_tspill));
    d_tadj = d_tinfo = d_tspill = nullptr;
    tiny_ok = false;
    if (d_uv) HIP_CHECK(hipFree(d_uv));
    if (state_block) HIP_CHECK(hipFree(state_block));
    if (state_block_alt) HIP_CHECK(hipFree(state_block_alt));
    state_block_alt = nullptr;
    state_bytes_alt = 0;
    d_row_off = nullptr;
    d_row_off32 = nullptr;
    d_col = nullptr;
    d_padj = nullptr;
    d_padj8 = nullptr;
    d_uv = nullptr;
    state_block = nullptr;
    n = 0;
    nnz = m_input = uv_m = 0;
  }

  // One allocation for every per-search array, sized for the 288 GB HBM of
  // the part: 3 bitmaps pairs (n/8 B each) + parent/queue (4n B each) per side.
  void alloc_state() {
    alloc_state_set();
    bufs[0] = buf;
    bufs[1] = launch::SearchBuffers{};  // allocated by the first resident query
    cur = 0;
    clean_tag[0] = clean_tag[1] = 0;
  }

  // State set 1 (same layout, its own block), on the first resident query:
  // graph loads and one-shot use pay nothing for it.  The server takes both
  // sets at launch, so a running server is stopped first (it relaunches on
  // the query being posted).
  void ensure_alt_set() {
    if (state_block_alt) return;
    stop_server();
    void* const blk0 = state_block;
    const size_t bytes0 = state_bytes;
    uint32_t* const flag0 = d_flag;
    const launch::SearchBuffers set0 = buf;
    alloc_state_set();  // into buf / state_block / state_bytes / d_flag
    bufs[1] = buf;
    state_block_alt = state_block;
    state_bytes_alt = state_bytes;
    state_block = blk0;
    state_bytes = bytes0;
    d_flag = flag0;
    buf = set0;
  }

  void alloc_state_set() {
    const uint64_t words = ((uint64_t)n + 63) / 64 * 2 + 2;
    const uint64_t trace_cap = 4096;
    size_t off = 0;
    auto take = [&](size_t bytes) {
      size_t o = off;
      off += (bytes + 255) & ~(size_t)255;
      return o;
    };
    size_t o_vis[2], o_fb[2], o_nb[2], o_par[2], o_q[2];
    for (int s = 0; s < 2; ++s) {
      o_vis[s] = take(words * 4);
      o_fb[s] = take(words * 4);
      o_nb[s] = take(words * 4);
    }
    for (int s = 0; s < 2; ++s) {
      o_par[s] = take((size_t)n * 4 + 4);
      o_q[s] = take((size_t)n * 4 + 4);
    }
    size_t o_hub = take((size_t)n * 4 + 4);
    size_t o_path = take((size_t)n * 4 + 8);
    size_t o_st = take(sizeof(DevState));
    size_t o_tr = take(trace_cap * sizeof(LevelTraceDev));
    size_t o_flag = take(64);
    size_t o_aux = take(64);
    size_t o_hdump = take(launch::handoff_dump_bytes());
    size_t o_gst = take((size_t)launch::kGridStampLevels * launch::kGridStampWords * 8);
    state_bytes = off;
    HIP_CHECK(hipMalloc(&state_block, state_bytes));
    char* base = static_cast<char*>(state_block);
    for (int s = 0; s < 2; ++s) {
      buf.vis[s] = reinterpret_cast<uint32_t*>(base + o_vis[s]);
      buf.fbits[s] = reinterpret_cast<uint32_t*>(base + o_fb[s]);
      buf.nbits[s] = reinterpret_cast<uint32_t*>(base + o_nb[s]);
      buf.parent[s] = reinterpret_cast<uint32_t*>(base + o_par[s]);
      buf.queue[s] = reinterpret_cast<uint32_t*>(base + o_q[s]);
    }
    buf.hub_list = reinterpret_cast<uint32_t*>(base + o_hub);
    buf.dpath = reinterpret_cast<uint32_t*>(base + o_path);
    buf.st = reinterpret_cast<DevState*>(base + o_st);
    buf.trace = reinterpret_cast<LevelTraceDev*>(base + o_tr);
    buf.trace_cap = (uint32_t)trace_cap;
    buf.words = (uint32_t)words;
    d_flag = reinterpret_cast<uint32_t*>(base + o_flag);
    buf.aux = reinterpret_cast<uint32_t*>(base + o_aux);
    buf.gstamp = reinterpret_cast<unsigned long long*>(base + o_gst);
    buf.hdump = reinterpret_cast<uint32_t*>(base + o_hdump);
    // visited bitmaps must start (and stay) all-zero
    for (int s = 0; s < 2; ++s) HIP_CHECK(hipMemsetAsync(buf.vis[s], 0, words * 4, stream));
    HIP_CHECK(hipMemsetAsync(buf.st, 0, sizeof(DevState), stream));
    HIP_CHECK(hipMemsetAsync(d_flag, 0, 64, stream));  // bitmap-meet flag + LDS-engine election ticket
    HIP_CHECK(hipMemsetAsync(buf.aux, 0, 64, stream));  // gate / auto plan
    HIP_CHECK(hipStreamSynchronize(stream));
  }

  void finish_graph(double ms) {
    // wide_offsets (tests, set_build_flags): no 32-bit copy of the row
    // offsets, so a small graph takes the 64-bit-offset kernels of an
    // nnz >= 2^32 graph
    if (nnz < 0xFFFFFFFFULL && !wide_offsets) {
      HIP_CHECK(hipMalloc(&d_row_off32, ((size_t)n + 1) * 4));
      launch::make_row_off32(d_row_off, n, d_row_off32, stream);
    }
    // Packed adjacency: 16 B per directed edge next to the 4 B CSR column.
    // Budget BIBFS_PADJ_MAX_MB (default 4096 MiB; 0 disables) -- a 10M-vertex
    // G(n, 2.2/n) needs 352 MB, a scale-27 Kronecker graph would need ~69 GB,
    // where the plain CSR path is used instead.
    const uint64_t budget = env::padj_budget_bytes();
    max_deg = launch::max_degree(d_row_off, n, stream);
    // 8 B per edge (launch::pack8) where ids, bases and degrees fit: half the
    // bytes (10M G(n, p): 176 instead of 352 MB).  The hope was a MALL-resident
    // adjacency and shorter dependent loads; measured the same search times
    // (10M 62.8-63.1 vs 62.8-63.2 us, profiles/r4_padj8_ab.jsonl), so what it
    // buys is the memory.
    if (nnz && n < launch::kPack8MaxN && nnz < launch::kPack8MaxNnz && max_deg <= launch::kPack8MaxDeg &&
        nnz * 8 <= budget) {
      HIP_CHECK(hipMalloc(&d_padj8, nnz * 8));
      launch::build_padj8(d_row_off, d_col, nnz, d_padj8, stream);
    } else if (nnz && nnz * 16 <= budget) {
      HIP_CHECK(hipMalloc(&d_padj, nnz * 16));
      launch::build_padj(d_row_off, d_col, nnz, d_padj, stream);
    }
    // small graphs: the packed 8-byte adjacency of the tiny server (8 (nnz + n) B)
    if (tiny_enabled && launch::tiny_supported(n, nnz, max_deg)) {
      HIP_CHECK(hipMalloc(&d_tadj, (std::max<uint64_t>(nnz, 1) + 4) * 8));  // +4: 16-byte first-edge loads
      HIP_CHECK(hipMalloc(&d_tinfo, (size_t)n * 8));
      HIP_CHECK(hipMalloc(&d_tspill, (size_t)4 * kTinySpill * 8));
      launch::build_tiny_adj(d_row_off, d_col, n, nnz, d_tadj, d_tinfo, stream);
      tiny_ok = true;
    }
    alloc_state();
    build_ms = ms;
  }

  void build_from_device_edges(const uint32_t* uv, uint64_t m) {
    nnz = launch::count_csr_entries(uv, m, n, d_row_off, stream);
    HIP_CHECK(hipMalloc(&d_col, std::max<uint64_t>(nnz, 1) * 4));
    uint64_t* cursor = nullptr;
    HIP_CHECK(hipMalloc(&cursor, ((size_t)n + 1) * 8));
    launch::fill_csr(uv, m, n, d_row_off, cursor, d_col, stream);
    HIP_CHECK(hipStreamSynchronize(stream));
    HIP_CHECK(hipFree(cursor));
  }

  void wait_seq(uint32_t want, const HostResult* rec = nullptr) {
    const HostResult* R = rec ? rec : h_res;
    for (uint64_t it = 1;; ++it) {
      if (__atomic_load_n(&R->seq, __ATOMIC_ACQUIRE) == want) return;
      if ((it & 4095) == 0) {
        hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess) {
          if (__atomic_load_n(&R->seq, __ATOMIC_ACQUIRE) == want) return;
          throw Error("bibfs: search kernel finished without publishing a result");
        }
        if (e != hipErrorNotReady)
          throw Error(std::string("bibfs: search kernel failed: ") + hipGetErrorString(e));
      } else {
        _mm_pause();
      }
    }
  }

  // like wait_seq, but returns false when the kernel completed without publishing
  bool wait_seq_or_done(uint32_t want) {
    for (uint64_t it = 1;; ++it) {
      if (__atomic_load_n(&h_res->seq, __ATOMIC_ACQUIRE) == want) return true;
      if ((it & 4095) == 0) {
        hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess) return __atomic_load_n(&h_res->seq, __ATOMIC_ACQUIRE) == want;
        if (e != hipErrorNotReady)
          throw Error(std::string("bibfs: search kernel failed: ") + hipGetErrorString(e));
      } else {
        _mm_pause();
      }
    }
  }

  uint32_t level_seq = 0;  // k_finish_level publishes DevState into pinned h_state with this seq

  // wait for the pinned DevState mirror of the last finished level
  void wait_level() {
    for (uint64_t it = 1; __atomic_load_n(&h_state->pad[0], __ATOMIC_ACQUIRE) != level_seq; ++it) {
      if ((it & 8191) == 0) {
        const hipError_t e = hipStreamQuery(stream);
        if (e == hipSuccess && __atomic_load_n(&h_state->pad[0], __ATOMIC_ACQUIRE) != level_seq)
          throw Error("bibfs: grid level finished without publishing its state");
        if (e != hipSuccess && e != hipErrorNotReady)
          throw Error(std::string("bibfs: grid level failed: ") + hipGetErrorString(e));
      } else {
        _mm_pause();
      }
    }
  }

  void sync_state() {
    HIP_CHECK(hipMemcpyAsync(h_state, buf.st, sizeof(DevState), hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
  }

  // one grid level of side s; mode 1 = top-down, 2 = bottom-up.  The level's
  // last workgroup finishes it and publishes the pinned mirror; when the level
  // ends the search it also walks the path and publishes the result with
  // res_seq (0 = leave that to the caller: step-wise API).
  uint32_t res_seq = 0;
  void grid_level(int s, int mode, int trace) {
    const auto g = view();
    const launch::HostSide hs{gres, h_path, h_path_cap, h_state};
    const uint32_t ls = ++level_seq == 0 ? ++level_seq : level_seq;
    if (mode == 2) {
      if (!fbits_valid[s]) launch::build_frontier_bits(g, buf, s, stream);
      launch::grid_bottomup(g, buf, s, cus, stream);
      std::swap(buf.fbits[s], buf.nbits[s]);
      fbits_valid[s] = true;
      launch::finish_level(buf, s, mode, trace, h_state, ls, hs, res_seq, n, stream);
    } else {
      // Vertices above the hub degree go to the edge-parallel hub pass (a
      // vertex that big can only be in a frontier with that many edges).  The
      // top-down kernel gives each workgroup 256 frontier VERTICES, so a small
      // frontier of heavy vertices (Kronecker levels after the hand-off: a few
      // hundred vertices, 10^5 edges) would run on a handful of workgroups:
      // then every vertex above 64 edges goes edge-parallel over all CUs (at
      // most a few hub tiles: every workgroup stages each tile, so a frontier
      // of tens of thousands of vertices stays with the chunked kernel).
      const uint64_t F = h_state->fend[s] - h_state->fbeg[s], fe = h_state->fedges[s];
      uint32_t hub_deg = ~0u;
      if (max_deg > launch::grid_hub_degree() && fe > launch::grid_hub_degree()) hub_deg = launch::grid_hub_degree();
      if (F <= 4096 && fe > 16384 && max_deg > 64) hub_deg = 64;
      launch::grid_topdown(g, buf, s, cus, F, fe, h_state, ls, trace, hs, res_seq, hub_deg, stream);
      fbits_valid[s] = false;
    }
    // the cleanup rides behind every level and runs behind the one that ends
    // the search, so it is done about when the host has read the answer
    if (res_seq) cleanup_async(true);
    wait_level();
  }

  int choose_mode(int s, const SearchOptions& opt) {
    if (opt.direction == Direction::kTopDown) return 1;
    if (opt.direction == Direction::kBottomUp) return 2;
    const DevState& st = *h_state;
    const double m_f = (double)st.fedges[s];
    const double m_u = (double)nnz - (double)st.vedges[s];
    const double n_f = (double)(st.fend[s] - st.fbeg[s]);
    if (dir[s] == 1 && m_f > m_u / opt.alpha) dir[s] = 2;
    else if (dir[s] == 2 && n_f < (double)n / opt.beta) dir[s] = 1;
    return dir[s];
  }

  int choose_side(const SearchOptions& opt, int& turn) {
    const DevState& st = *h_state;
    if (opt.side == SidePolicy::kAlternate) {
      int s = turn;
      turn ^= 1;
      return s;
    }
    if (opt.side == SidePolicy::kSmallerFrontier)
      return (st.fend[0] - st.fbeg[0]) <= (st.fend[1] - st.fbeg[1]) ? 0 : 1;
    return st.fedges[0] <= st.fedges[1] ? 0 : 1;
  }

  // Runs grid levels until the search ends; returns #grid levels and #bottom-up levels.
  // mirror_valid: the LDS hand-off already published DevState into h_state.
  bool mirror_valid = false;
  void grid_loop(const SearchOptions& opt, SearchStats& stats) {
    dir[0] = dir[1] = 1;
    fbits_valid[0] = fbits_valid[1] = false;
    int turn = 0;
    // 2 = stamped (BIBFS_STAMP): the level kernels also write their phase stamps
    const int trace = opt.trace ? (env::stamps() ? 2 : 1) : 0;
    for (uint32_t guard = 0; guard <= 2 * (uint64_t)n + 2; ++guard) {
      if (guard == 0 && !mirror_valid) sync_state();  // state left by the seed
      if (h_state->status != kRunning || h_state->meet != kEmpty) break;
      const int s = choose_side(opt, turn);
      const int mode = choose_mode(s, opt);
      grid_level(s, mode, trace);
      stats.grid_levels++;
      if (mode == 2) stats.bottomup_levels++;
    }
  }

  SearchResult collect(const HostResult& R, const SearchOptions& opt, SearchStats stats) {
    SearchResult r;
    r.stats = std::move(stats);
    r.found = R.status == kFound;
    r.hops = r.found ? R.hops : -1;
    r.meet = r.found ? R.meet : kNoVertex;
    r.stats.levels = (int)R.levels;
    r.stats.edges_inspected = R.einsp;
    r.stats.visited = R.visited;
    if (r.found && opt.want_path) {
      r.path.resize(R.path_len);
      if (R.path_on_device) {
        HIP_CHECK(hipMemcpyAsync(r.path.data(), buf.dpath, (size_t)R.path_len * 4,
                                 hipMemcpyDeviceToHost, stream));
        HIP_CHECK(hipStreamSynchronize(stream));
      } else {
        std::memcpy(r.path.data(), h_path, (size_t)R.path_len * 4);
      }
    }
    return r;
  }

  void fetch_clock(SearchResult& r) {
    LevelTraceDev t{};
    HIP_CHECK(hipMemcpyAsync(&t, buf.trace + buf.trace_cap - 1, sizeof t, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    if (t.discovered)
      std::fprintf(stderr, "[stamp] shader clock %.0f MHz over %.2f us\n", (double)t.edges / (double)t.discovered * 100.0,
                   (double)t.discovered / 100.0);
    LevelTraceDev u{};
    HIP_CHECK(hipMemcpyAsync(&u, buf.trace + buf.trace_cap - 2, sizeof u, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    std::fprintf(stderr, "[stamp] cycles: election %u init %u search-loop %llu path-walk %u publish %u\n", u.side,
                 u.depth, (unsigned long long)t.edges, u.frontier, u.mode);
    LevelTraceDev w{};
    HIP_CHECK(hipMemcpyAsync(&w, buf.trace + buf.trace_cap - 3, sizeof w, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    std::fprintf(stderr, "[stamp] publish: hand-off state %u result puts %u bitmaps issued %u drained %u fence %llu\n",
                 w.side, w.depth, w.frontier, w.mode, (unsigned long long)w.edges);
  }

  // Stamped grid levels (BIBFS_STAMP + trace): block 0's phases and the
  // finisher's, in us from block 0's entry (s_memrealtime, 100 MHz).
  void fetch_grid_stamps(const SearchResult& r) {
    std::vector<unsigned long long> g((size_t)launch::kGridStampLevels * launch::kGridStampWords);
    HIP_CHECK(hipMemcpyAsync(g.data(), buf.gstamp, g.size() * 8, hipMemcpyDeviceToHost, stream));
    HIP_CHECK(hipStreamSynchronize(stream));
    for (size_t l = 0; l < r.stats.trace.size() && l < launch::kGridStampLevels; ++l) {
      if (r.stats.trace[l].mode != 4) continue;  // grid top-down levels
      const unsigned long long* t = &g[l * launch::kGridStampWords];
      if (!t[0] || t[5] < t[0]) continue;
      auto us = [&](int k) { return t[k] >= t[0] ? (double)(t[k] - t[0]) * 0.01 : -1.0; };
      std::fprintf(stderr,
                   "[grid stamp] level %zu (frontier %llu, edges %llu): block 0 staged %.2f us, claims issued %.2f, "
                   "left %.2f; finisher start %.2f, end %.2f\n",
                   l, (unsigned long long)r.stats.trace[l].frontier, (unsigned long long)r.stats.trace[l].edges, us(1),
                   us(2), us(3), us(4), us(5));
    }
  }

  void fetch_trace(SearchResult& r) {
    const uint32_t L = std::min<uint32_t>((uint32_t)r.stats.levels, buf.trace_cap);
    std::vector<LevelTraceDev> t(L);
    if (L) {
      HIP_CHECK(hipMemcpyAsync(t.data(), buf.trace, L * sizeof(LevelTraceDev), hipMemcpyDeviceToHost,
                               stream));
      HIP_CHECK(hipStreamSynchronize(stream));
    }
    r.stats.trace.clear();
    for (auto& x : t) {
      LevelTrace lt;
      lt.side = (int)x.side;
      lt.depth = (int)x.depth;
      lt.frontier = x.frontier;
      lt.edges = x.edges;
      lt.discovered = x.discovered;
      lt.mode = (int)x.mode;
      r.stats.trace.push_back(lt);
    }
  }
};

HipBiBfs::HipBiBfs(int device) : p_(new Impl) {
  p_->device = device;
  HIP_CHECK(hipSetDevice(device));
  HIP_CHECK(hipGetDeviceProperties(&p_->prop, device));
  p_->cus = p_->prop.multiProcessorCount > 0 ? p_->prop.multiProcessorCount : 256;
  HIP_CHECK(hipStreamCreateWithFlags(&p_->stream, hipStreamNonBlocking));
  HIP_CHECK(hipStreamCreateWithFlags(&p_->sstream, hipStreamNonBlocking));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_box), sizeof(ServerBox),
                          hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(p_->h_box, 0, sizeof(ServerBox));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_res), sizeof(HostResult),
                          hipHostMallocMapped | hipHostMallocCoherent));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_path), (size_t)p_->h_path_cap * 4,
                          hipHostMallocMapped | hipHostMallocCoherent));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_state), sizeof(DevState),
                          hipHostMallocMapped | hipHostMallocCoherent));  // k_finish_level writes it
  std::memset(p_->h_res, 0, sizeof(HostResult));
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_gres), sizeof(HostResult),
                          hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(p_->h_gres, 0, sizeof(HostResult));
  p_->gres = p_->h_res;
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_clean), 64, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(p_->h_clean, 0, 64);
  HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&p_->h_pkts), kTinyPktCap * sizeof(TinyPkt),
                          hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(p_->h_pkts, 0, kTinyPktCap * sizeof(TinyPkt));
  HIP_CHECK(hipMalloc(&p_->d_stamps, 32 * sizeof(unsigned long long)));
  HIP_CHECK(hipEventCreate(&p_->ev0));
  HIP_CHECK(hipEventCreate(&p_->ev1));
}

HipBiBfs::~HipBiBfs() {
  if (!p_) return;
  try {
    (void)hipSetDevice(p_->device);
    (void)hipStreamSynchronize(p_->stream);
    p_->free_graph();
  } catch (...) {
  }
  (void)hipStreamDestroy(p_->sstream);
  (void)hipHostFree(p_->h_box);
  (void)hipHostFree(p_->h_res);
  (void)hipHostFree(p_->h_gres);
  (void)hipHostFree(p_->h_clean);
  (void)hipHostFree(p_->h_pkts);
  (void)hipFree(p_->d_stamps);
  (void)hipHostFree(p_->h_path);
  (void)hipHostFree(p_->h_state);
  (void)hipEventDestroy(p_->ev0);
  (void)hipEventDestroy(p_->ev1);
  (void)hipStreamDestroy(p_->stream);
}

void HipBiBfs::load_csr(const Csr& g) {
  TraceRange range("bibfs:build");
  HIP_CHECK(hipSetDevice(p_->device));
  p_->free_graph();
  auto& I = *p_;
  I.n = g.n;
  I.nnz = g.nnz();
  I.m_input = g.m_input;
  HIP_CHECK(hipEventRecord(I.ev0, I.stream));
  HIP_CHECK(hipMalloc(&I.d_row_off, ((size_t)g.n + 1) * 8));
  HIP_CHECK(hipMalloc(&I.d_col, std::max<size_t>(g.nnz(), 1) * 4));
  HIP_CHECK(hipMemcpyAsync(I.d_row_off, g.row_off.data(), ((size_t)g.n + 1) * 8,
                           hipMemcpyHostToDevice, I.stream));
  if (g.nnz())
    HIP_CHECK(hipMemcpyAsync(I.d_col, g.col.data(), g.nnz() * 4, hipMemcpyHostToDevice, I.stream));
  HIP_CHECK(hipEventRecord(I.ev1, I.stream));
  HIP_CHECK(hipEventSynchronize(I.ev1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, I.ev0, I.ev1));
  I.finish_graph(ms);
}


void HipBiBfs::adopt_device_csr(uint32_t n, uint64_t nnz, uint64_t m_input, uint64_t* d_row_off,
                                uint32_t* d_col) {
  TraceRange range("bibfs:build");
  HIP_CHECK(hipSetDevice(p_->device));
  p_->free_graph();
  auto& I = *p_;
  I.n = n;
  I.nnz = nnz;
  I.m_input = m_input;
  I.d_row_off = d_row_off;
  I.d_col = d_col;
  I.borrowed_csr = true;
  I.finish_graph(0.0);
}

void HipBiBfs::load_edges(const EdgeList& el) {
  TraceRange range("bibfs:build");
  HIP_CHECK(hipSetDevice(p_->device));
  p_->free_graph();
  auto& I = *p_;
  I.n = el.n;
  I.m_input = el.m();
  HIP_CHECK(hipEventRecord(I.ev0, I.stream));
  uint32_t* d_uv = nullptr;
  HIP_CHECK(hipMalloc(&d_uv, std::max<size_t>(el.uv.size(), 2) * 4));
  if (!el.uv.empty())
    HIP_CHECK(hipMemcpyAsync(d_uv, el.uv.data(), el.uv.size() * 4, hipMemcpyHostToDevice, I.stream));
  HIP_CHECK(hipMalloc(&I.d_row_off, ((size_t)I.n + 1) * 8));
  I.build_from_device_edges(d_uv, el.m());
  HIP_CHECK(hipEventRecord(I.ev1, I.stream));
  HIP_CHECK(hipEventSynchronize(I.ev1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, I.ev0, I.ev1));
  HIP_CHECK(hipFree(d_uv));
  I.finish_graph(ms);
}

void HipBiBfs::generate_gnp(uint32_t n, double p, uint64_t seed) {
  TraceRange range("bibfs:build");
  HIP_CHECK(hipSetDevice(p_->device));
  p_->free_graph();
  auto& I = *p_;
  I.n = n;
  HIP_CHECK(hipEventRecord(I.ev0, I.stream));
  HIP_CHECK(hipMalloc(&I.d_row_off, ((size_t)n + 1) * 8));
  const double expect_m = p * 0.5 * (double)n * (double)(n - 1);
  if (expect_m > (double)Impl::kKeepEdges || p_->force_stream_gen) {
    // large graph: CSR straight from the generator, no edge list in HBM
    uint64_t m = 0;
    I.nnz = launch::gen_rows_gnp(n, p, seed, 0, n, I.d_row_off, &I.d_col, &m, I.stream);
    I.m_input = m;
  } else {
    uint32_t* d_uv = nullptr;
    const uint64_t m = launch::gen_gnp_device(n, p, seed, &d_uv, I.stream);
    I.m_input = m;
    I.build_from_device_edges(d_uv, m);
    I.d_uv = d_uv;  // kept for download_edges()
    I.uv_m = m;
  }
  HIP_CHECK(hipEventRecord(I.ev1, I.stream));
  HIP_CHECK(hipEventSynchronize(I.ev1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, I.ev0, I.ev1));
  I.finish_graph(ms);
}

void HipBiBfs::generate_rmat(uint32_t n, uint64_t m, uint64_t seed, double a, double b, double c) {
  TraceRange range("bibfs:build");
  HIP_CHECK(hipSetDevice(p_->device));
  p_->free_graph();
  auto& I = *p_;
  BIBFS_REQUIRE(n >= 2, "R-MAT needs n >= 2");
  I.n = n;
  I.m_input = m;
  HIP_CHECK(hipEventRecord(I.ev0, I.stream));
  HIP_CHECK(hipMalloc(&I.d_row_off, ((size_t)n + 1) * 8));
  if (m > Impl::kKeepEdges || p_->force_stream_gen) {
    // large graph: CSR straight from the generator, no edge list in HBM
    I.nnz = launch::gen_rows_rmat(n, m, seed, a, b, c, 0, n, I.d_row_off, &I.d_col, I.stream);
  } else {
    uint32_t* d_uv = nullptr;
    HIP_CHECK(hipMalloc(&d_uv, std::max<uint64_t>(2 * m, 2) * 4));
    launch::gen_rmat_device(n, m, seed, a, b, c, d_uv, I.stream);
    I.build_from_device_edges(d_uv, m);
    I.d_uv = d_uv;  // kept for download_edges()
    I.uv_m = m;
  }
  HIP_CHECK(hipEventRecord(I.ev1, I.stream));
  HIP_CHECK(hipEventSynchronize(I.ev1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, I.ev0, I.ev1));
  I.finish_graph(ms);
}

void HipBiBfs::set_resident(bool on, double idle_ms) {
  auto& I = *p_;
  HIP_CHECK(hipSetDevice(I.device));
  if (!on) I.stop_server();
  I.resident = on;
  I.srv_idle_ticks = (unsigned long long)(idle_ms * 1e5);  // s_memrealtime: 100 MHz
}
bool HipBiBfs::resident() const { return p_->resident; }
void HipBiBfs::set_batch_edge_cap(uint64_t edges) { p_->bedge_cap = edges; }
void HipBiBfs::set_batch_tuning(int lds_first, int threads) {
  BIBFS_REQUIRE(threads == 0 || threads == 256 || threads == 1024, "batch threads must be 0, 256 or 1024");
  p_->blds = lds_first;
  p_->bthreads = threads;
}
uint64_t HipBiBfs::batch_edge_cap() const { return p_->bedge_cap; }
uint64_t HipBiBfs::last_batch_fallbacks() const { return p_->batch_fallbacks; }

std::vector<SearchResult> HipBiBfs::search_batch(const std::vector<vid_t>& src, const std::vector<vid_t>& dst,
                                                 const SearchOptions& opt) {
  auto& I = *p_;
  BIBFS_REQUIRE(src.size() == dst.size(), "search_batch: src and dst sizes differ");
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  HIP_CHECK(hipSetDevice(I.device));
  const size_t K = src.size();
  std::vector<SearchResult> out(K);
  I.batch_fallbacks = 0;
  if (K == 0) return out;
  for (size_t i = 0; i < K; ++i) BIBFS_REQUIRE(src[i] < I.n && dst[i] < I.n, "src/dst out of range");
  if (opt.force_grid || opt.trace || !I.server_usable()) {  // the batch kernel is the LDS engine only
    for (size_t i = 0; i < K; ++i) out[i] = search(src[i], dst[i], opt);
    I.batch_fallbacks = K;
    return out;
  }
  // slots: up to 1024 per launch.  Per-slot state (parent + queue, 16n B) is
  // touched sparsely, so the budget is generous: up to 40 GiB or half the free
  // HBM -- enough for 256 concurrent 10M-vertex queries on one MI355X.
  size_t hbm_free = 0, hbm_total = 0;
  HIP_CHECK(hipMemGetInfo(&hbm_free, &hbm_total));
  const uint64_t budget = std::min<uint64_t>(40ull << 30, (uint64_t)hbm_free / 2 + (uint64_t)I.bcap * (16ull * I.n));
  const uint64_t per_slot = 16ull * I.n + 8ull * I.buf.words;
  const uint32_t kmax = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(1024, budget / per_slot));
  for (size_t c0 = 0; c0 < K; c0 += kmax) {
    const uint32_t k = (uint32_t)std::min<size_t>(kmax, K - c0);
    const auto t0 = std::chrono::steady_clock::now();
    I.ensure_batch(k);
    std::memcpy(I.h_bq, src.data() + c0, k * 4);
    std::memcpy(I.h_bq + k, dst.data() + c0, k * 4);
    const uint32_t seq = ++I.seq == 0 ? ++I.seq : I.seq;
    // auto: the HBM-bitmap pass alone.  Measured at 256 queries
    // (benchmarks/batch_serving.py, profiles/r1_batch_serving.jsonl) it beats
    // LDS-pass-first at every size: 100k G(n,p) 1.12 -> 0.56 us/query, 1M
    // 2.00 -> 1.01, 10M 3.43 -> 2.37, Kronecker-22 13.1 -> 12.4.  The LDS
    // engine stays the single-query (latency) path.
    const bool lds_first = I.blds >= 0 ? I.blds != 0 : false;
    if (lds_first) {
      launch::lds_batch(I.view(), I.buf, I.h_bq, I.h_bq + k, k, I.d_bslots, I.h_bres, I.h_bpath, Impl::kBatchPath,
                        seq, I.stream);
    } else {
      for (uint32_t i = 0; i < k; ++i) {
        I.h_bres[i].status = kHandoff;
        I.h_bres[i].path_on_device = 0;
        __atomic_store_n(&I.h_bres[i].seq, seq, __ATOMIC_RELEASE);
      }
    }
    for (uint32_t i = 0; i < k; ++i) {
      for (uint64_t it = 1; __atomic_load_n(&I.h_bres[i].seq, __ATOMIC_ACQUIRE) != seq; ++it) {
        if ((it & 8191) == 0) {
          const hipError_t e = hipStreamQuery(I.stream);
          if (e == hipSuccess && __atomic_load_n(&I.h_bres[i].seq, __ATOMIC_ACQUIRE) != seq)
            throw Error("bibfs: batched search finished without publishing every result");
          if (e != hipSuccess && e != hipErrorNotReady)
            throw Error(std::string("bibfs: batched search failed: ") + hipGetErrorString(e));
        } else {
          _mm_pause();
        }
      }
    }
    // queries whose visited sets outgrew LDS: one more batched pass with the
    // visited bitmaps in HBM (batch_global.hip) instead of one-by-one re-runs
    uint32_t nglobal = 0;
    for (uint32_t i = 0; i < k; ++i) {
      const HostResult& R = I.h_bres[i];
      if (src[c0 + i] != dst[c0 + i] && R.status == kHandoff) I.h_bqidx[nglobal++] = i;
    }
    if (nglobal) {
      launch::batch_global(I.view(), I.buf.words, I.h_bqidx, nglobal, I.h_bq, I.h_bq + k, I.d_bslots, I.d_bbits,
                           I.h_bout, I.h_bpath, Impl::kBatchPath, I.bedge_cap,
                           I.bthreads ? I.bthreads : 1024,
                           I.stream);
      HIP_CHECK(hipStreamSynchronize(I.stream));
    }
    std::vector<char> via_global(k, 0);
    for (uint32_t j = 0; j < nglobal; ++j) via_global[I.h_bqidx[j]] = 1;
    const double wall = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    for (uint32_t i = 0; i < k; ++i) {
      const HostResult& R = I.h_bres[i];
      SearchResult& r = out[c0 + i];
      const vid_t s = src[c0 + i], d = dst[c0 + i];
      if (s == d) {
        r = search(s, d, opt);
        continue;
      }
      if (via_global[i]) {
        const BatchOut& G = I.h_bout[i];
        if (G.status != kFound && G.status != kNoPath) {
          r = search(s, d, opt);  // a level above the edge cap / path longer than the slot
          ++I.batch_fallbacks;
          continue;
        }
        r.found = G.status == kFound;
        r.hops = r.found ? G.hops : -1;
        r.meet = r.found ? G.meet : kNoVertex;
        r.stats.levels = (int)G.levels;
        r.stats.edges_inspected = G.einsp;
        r.stats.visited = G.visited;
        r.stats.handoff = true;
        if (r.found && opt.want_path) r.path.assign(I.h_bpath + (size_t)i * Impl::kBatchPath,
                                                    I.h_bpath + (size_t)i * Impl::kBatchPath + G.path_len);
        r.search_ms = wall;
        r.total_ms = wall;
        continue;
      }
      if (R.status == kHandoff || R.path_on_device == 2 || (R.status != kFound && R.status != kNoPath)) {
        r = search(s, d, opt);  // path longer than the slot: single-query engines
        ++I.batch_fallbacks;
        continue;
      }
      r.found = R.status == kFound;
      r.hops = r.found ? R.hops : -1;
      r.meet = r.found ? R.meet : kNoVertex;
      r.stats.levels = (int)R.levels;
      r.stats.edges_inspected = R.einsp;
      r.stats.visited = R.visited;
      if (r.found && opt.want_path) r.path.assign(I.h_bpath + (size_t)i * Impl::kBatchPath,
                                                  I.h_bpath + (size_t)i * Impl::kBatchPath + R.path_len);
      r.search_ms = (double)(R.rt_end - R.rt_begin) * 1e-5;
      r.total_ms = wall;  // the whole batch's wall time
    }
  }
  HIP_CHECK(hipStreamSynchronize(I.stream));
  return out;
}

void HipBiBfs::release() {
  HIP_CHECK(hipSetDevice(p_->device));
  HIP_CHECK(hipStreamSynchronize(p_->stream));
  p_->free_graph();
}

uint32_t HipBiBfs::n() const { return p_->n; }
uint64_t HipBiBfs::nnz() const { return p_->nnz; }
uint64_t HipBiBfs::m_input() const { return p_->m_input; }
double HipBiBfs::last_build_ms() const { return p_->build_ms; }
size_t HipBiBfs::device_bytes() const {
  const auto& I = *p_;
  return ((size_t)I.n + 1) * 8 + (I.d_row_off32 ? ((size_t)I.n + 1) * 4 : 0) + I.nnz * 4 +
         (I.d_padj ? I.nnz * 16 : 0) + (I.d_padj8 ? I.nnz * 8 : 0) +
         (I.d_uv ? I.uv_m * 8 : 0) + I.state_bytes + I.state_bytes_alt;
}
int HipBiBfs::device() const { return p_->device; }
void* HipBiBfs::stream() const { return p_->stream; }
void HipBiBfs::synchronize() const { HIP_CHECK(hipStreamSynchronize(p_->stream)); }

DeviceInfo HipBiBfs::info() const {
  DeviceInfo d;
  d.name = p_->prop.name;
  d.arch = p_->prop.gcnArchName;
  d.cus = p_->prop.multiProcessorCount;
  d.hbm_bytes = p_->prop.totalGlobalMem;
  d.lds_bytes = (int)p_->prop.sharedMemPerBlock;
  return d;
}

int64_t HipBiBfs::query(vid_t src, vid_t dst, std::vector<vid_t>* path) {
  auto& I = *p_;
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  BIBFS_REQUIRE(src < I.n && dst < I.n, "src/dst out of range");
  if (src == dst) {
    if (path) path->assign(1, src);
    I.last_ms = 0.0;
    I.last_einsp = 0;
    return 0;
  }
  static const SearchOptions kDefault{};
  if (I.tiny_usable(kDefault)) {
    if (I.host_stamps_on) I.hs_t0 = std::chrono::steady_clock::now();
    Impl::TinyAnswer a;
    const uint32_t st = I.tiny_search(src, dst, path, a);
    if (st != kTinyOverflow) {
      I.last_ms = a.ticks * 1e-5;
      I.last_einsp = a.einsp;
      if (I.host_stamps_on) {
        ++I.hs_n;
        I.hs_post += Impl::ns(I.hs_t1 - I.hs_t0);
        I.hs_wait += Impl::ns(I.hs_t2 - I.hs_t1);
        I.hs_read += Impl::ns(I.hs_t3 - I.hs_t2);
        I.hs_tail += Impl::ns(std::chrono::steady_clock::now() - I.hs_t3);
      }
      if (st == kTinyFound) return a.hops;
      if (path) path->clear();
      return -1;
    }
  }
  SearchResult r = search_general(src, dst, kDefault);
  I.last_ms = r.search_ms;
  I.last_einsp = r.stats.edges_inspected;
  if (path) *path = std::move(r.path);
  return r.found ? r.hops : -1;
}

double HipBiBfs::last_search_ms() const { return p_->last_ms; }
uint64_t HipBiBfs::last_edges_inspected() const { return p_->last_einsp; }
bool HipBiBfs::tiny_engine() const { return p_->tiny_ok; }
void HipBiBfs::set_auto_handoff(bool on) { p_->auto_on = on; }
void HipBiBfs::set_build_flags(bool wide_offsets, bool stream_gen, bool tiny) {
  p_->wide_offsets = wide_offsets;
  p_->force_stream_gen = stream_gen;
  p_->tiny_enabled = tiny;
}
void HipBiBfs::set_auto_gate_timeout_us(double us) { p_->auto_gate_us = us; }
double HipBiBfs::auto_gate_timeout_us() const { return p_->auto_gate_us; }
uint64_t HipBiBfs::auto_gate_misses() const { return p_->auto_gate_misses; }
void HipBiBfs::set_auto_levels(int levels) {
  BIBFS_REQUIRE(levels >= 1 && levels <= 8, "auto_levels must be in [1, 8]");
  p_->auto_levels = levels;
}
int HipBiBfs::auto_levels() const { return p_->auto_levels; }
void HipBiBfs::set_auto_max_degree(uint64_t deg) { p_->auto_max_deg = deg; }
uint64_t HipBiBfs::auto_max_degree() const { return p_->auto_max_deg; }
bool HipBiBfs::auto_handoff() const { return p_->auto_on; }
void HipBiBfs::set_lds_probe_edges(uint32_t edges) {
  if (edges == p_->probe_edges) return;
  p_->probe_edges = edges;
  p_->stop_server();  // a running LDS server holds the old budget: relaunched by the next search
}
uint32_t HipBiBfs::lds_probe_edges() const { return p_->probe_edges; }
uint64_t HipBiBfs::tiny_overflows() const { return p_->tiny_overflows; }
void HipBiBfs::set_host_stamps(bool on) {
  p_->host_stamps_on = on;
  p_->hs_n = p_->hs_post = p_->hs_wait = p_->hs_read = p_->hs_tail = 0;
}
std::vector<double> HipBiBfs::host_stamps() const {
  const double n = p_->hs_n ? (double)p_->hs_n : 1.0;
  return {(double)p_->hs_n, p_->hs_post / n * 1e-3, p_->hs_wait / n * 1e-3, p_->hs_read / n * 1e-3,
          p_->hs_tail / n * 1e-3};
}

SearchResult HipBiBfs::search(vid_t src, vid_t dst, const SearchOptions& opt) {
  auto& I = *p_;
  if (src != dst && I.n > 0 && src < I.n && dst < I.n && I.tiny_usable(opt)) {
    const auto t0 = std::chrono::steady_clock::now();
    SearchResult r;
    Impl::TinyAnswer a;
    const uint32_t st = I.tiny_search(src, dst, opt.want_path ? &r.path : nullptr, a);
    if (st != kTinyOverflow) {
      r.found = st == kTinyFound;
      r.hops = r.found ? (int64_t)a.hops : -1;
      r.meet = r.found ? a.meet : kNoVertex;
      r.stats.levels = (int)a.levels;
      r.stats.edges_inspected = a.einsp;
      r.stats.visited = a.visited;
      r.search_ms = a.ticks * 1e-5;
      r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
      return r;
    }
  }
  return search_general(src, dst, opt);
}

SearchResult HipBiBfs::search_general(vid_t src, vid_t dst, const SearchOptions& opt) {
  TraceRange range("bibfs:search");
  auto& I = *p_;
  const auto t0 = std::chrono::steady_clock::now();
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  BIBFS_REQUIRE(src < I.n && dst < I.n, "src/dst out of range");
  if (src == dst) {
    SearchResult r;
    r.found = true;
    r.hops = 0;
    r.meet = src;
    r.path = {src};
    r.stats.visited = 1;
    r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return r;
  }
  HIP_CHECK(hipSetDevice(I.device));
  const uint32_t seq = ++I.seq == 0 ? ++I.seq : I.seq;
  const auto g = I.view();
  launch::HostSide hs{I.h_res, I.h_path, I.h_path_cap, I.h_state};
  // the grid levels' record (h_gres behind an auto level, else h_res)
  I.gres = I.h_res;
  struct GresReset {
    Impl& I;
    ~GresReset() { I.gres = I.h_res; }
  } gres_reset{I};
  auto hsg = [&I] { return launch::HostSide{I.gres, I.h_path, I.h_path_cap, I.h_state}; };
  SearchStats stats;
  bool grid = opt.force_grid;
  double lds_ms = 0.0;
  int stats_handoff_levels = -1;  // levels the LDS phase ran before a hand-off
  uint32_t lds_probe = 0;         // HostResult::probe of the LDS phase
  bool use_auto = false, auto_final = false;  // device hand-off (grid_auto) behind a resident search
  uint32_t pub_auto = 0, auto_ls = 0, auto_tag = 0;
  grid = grid || I.n > 0x7fffffffu;
  // device time: the LDS kernel stamps itself (s_memrealtime); events only
  // around grid levels, where their ~µs cost is noise
  if (grid) HIP_CHECK(hipEventRecord(I.ev0, I.stream));  // LDS hash keys carry a parity bit: ids < 2^31
  if (!grid) {
    const int tr = opt.trace ? (env::stamps() ? 2 : 1) : 0;
    const int lock = (opt.lockstep && I.n <= 0x7fffffffu) ? 1 : 0;
    // BIBFS_STAMP_SERVER: the server's profiling build answers traced queries too
    const bool stamp_srv = env::server_stamps();
    // with the tiny server resident for this graph, the queries it cannot take
    // (non-default options, overflow) run one-shot beside it
    if (I.resident && !I.tiny_ok && (!opt.trace || stamp_srv) && I.lds_server_usable()) {
      I.flip_state_set();  // the server (own stream) must not share state with a running cleanup
      use_auto = I.auto_usable(opt);
      I.gres = use_auto ? I.h_gres : I.h_res;
      if (use_auto) {
        // device hand-off: the first grid level is enqueued before the search
        // starts and waits on the device for it to leave LDS (grid_auto)
        pub_auto = ++I.seq == 0 ? ++I.seq : I.seq;
        auto_ls = ++I.level_seq == 0 ? ++I.level_seq : I.level_seq;
      }
      I.server_post(src, dst, opt, seq);
      if (use_auto) {
        launch::grid_auto(g, I.buf, I.cus, I.max_deg, opt.alpha, I.h_state, auto_ls, hsg(), pub_auto, seq,
                          (unsigned long long)(std::max(0.0, I.auto_gate_us) * 100.0), I.auto_levels,
                          I.stream);
        auto_tag = I.next_clean_tag();
        launch::cleanup(I.buf, I.n, I.d_flag + 8, I.h_clean, auto_tag, 2, I.stream);
      }
      I.server_wait(seq);
    } else {
      launch::lds_search(g, I.buf, hs, src, dst, seq, (int)opt.side, tr, I.pin_xcc, I.d_flag + 4, lock,
                         I.stream);
    }
    if (use_auto) {
      // every resident search answers through h_res (a hand-off too); the
      // auto level behind it publishes into its own record, h_gres
      lds_ms = (double)(I.h_res->rt_end - I.h_res->rt_begin) * 1e-5;
      lds_probe = I.h_res->probe;
      if (I.h_res->status == kHandoff) {
        grid = true;
        stats.handoff = true;
        const uint32_t lv1 = I.h_res->levels;
        stats_handoff_levels = (int)lv1;
        const auto outcome = I.wait_auto(pub_auto, auto_ls);
        auto_final = outcome == Impl::kAutoFinal;
        if (auto_final) {
          stats.grid_levels = (int)(I.gres->levels - lv1);
          I.clean_tag[I.cur] = auto_tag;  // the cleanup behind the auto level ran (its tag)
        } else if (outcome == Impl::kAutoMissed) {
          // the gate wait gave up before this search handed off: nothing ran
          // behind it (no scatter, no level, no cleanup), so continue exactly
          // like a non-auto hand-off -- scatter the dumped hash tables and run
          // the host loop from the mirror the LDS engine published
          ++I.auto_gate_misses;
          I.mirror_valid = true;
          I.gres = I.h_res;
          pub_auto = 0;
          launch::handoff_scatter(g, I.buf, I.stream);
        } else {
          // the auto level finished without ending the search, or declined
          // (bottom-up): the host loop continues from its mirror
          if (I.h_state->levels > lv1) stats.grid_levels = (int)(I.h_state->levels - lv1);
          I.mirror_valid = true;
        }
      }
    } else {
      if (I.h_res->seq != seq && !I.wait_seq_or_done(seq)) {
        // no block reached the pinned XCD: relaunch unpinned, and stop pinning
        I.pin_xcc = -1;
        launch::lds_search(g, I.buf, hs, src, dst, seq, (int)opt.side, tr, -1, I.d_flag + 4, lock, I.stream);
        I.wait_seq(seq);
      }
      lds_ms = (double)(I.h_res->rt_end - I.h_res->rt_begin) * 1e-5;  // 100 MHz
      lds_probe = I.h_res->probe;
      if (I.h_res->status == kHandoff) {
        grid = true;
        stats.handoff = true;
        stats_handoff_levels = (int)I.h_res->levels;
        I.mirror_valid = true;  // the LDS kernel published the hand-off state
        launch::handoff_scatter(g, I.buf, I.stream);
      }
    }
  } else {
    launch::seed_state(g, I.buf, src, dst, I.stream);
  }
  uint32_t pub_seq = seq;
  if (auto_final) {
    pub_seq = pub_auto;
    I.grid_cleaned = true;
  } else if (grid) {
    TraceRange grange("bibfs:grid_levels");
    pub_seq = (use_auto && pub_auto) ? pub_auto : (++I.seq == 0 ? ++I.seq : I.seq);
    I.res_seq = pub_seq;  // the level that ends the search publishes the path + result
    try {
      I.grid_loop(opt, stats);
    } catch (...) {
      // unwind: a failed level must not leave the set's visited words dirty or
      // a stale predicated-cleanup tag that later flips would wait for forever
      I.res_seq = 0;
      I.mirror_valid = false;
      try {
        I.cleanup_async(false);
      } catch (...) {
      }
      throw;
    }
    I.res_seq = 0;
    I.mirror_valid = false;
    I.grid_cleaned = stats.grid_levels > 0;
    if (I.gres->seq != pub_seq) {  // ended before any grid level ran (meet at hand-off / seed)
      launch::walk_path(I.buf, hsg(), src, dst, pub_seq, I.n, I.stream);
      I.wait_seq(pub_seq, I.gres);
      I.grid_cleaned = false;
    }
  }
  // device time of a hand-off search: the grid publish stamps rt_end on the
  // same 100 MHz clock as the LDS kernel's rt_begin (no events, no event sync
  // on the query path); a search that never ran in LDS is timed with events
  const bool timed_by_events = grid && !stats.handoff;
  if (timed_by_events) HIP_CHECK(hipEventRecord(I.ev1, I.stream));
  if (!timed_by_events) {  // the LDS engine ran: its meet probe's record
    stats.probe_edges = lds_probe & 0x7fffffffu;
    stats.probe_hit = (lds_probe >> 31) != 0;
  }
  SearchResult r = I.collect(grid ? *I.gres : *I.h_res, opt, std::move(stats));
  r.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  r.search_ms = lds_ms;
  r.stats.lds_ms = lds_ms;
  if (!grid || stats_handoff_levels >= 0) r.stats.lds_levels = grid ? stats_handoff_levels : r.stats.levels;
  if (grid && !timed_by_events && I.gres->seq == pub_seq) {
    r.search_ms = (double)(I.gres->rt_end - I.h_res->rt_begin) * 1e-5;
    if (I.gres->rt_walk && I.gres->rt_end > I.gres->rt_walk)
      r.stats.walk_ms = (double)(I.gres->rt_end - I.gres->rt_walk) * 1e-5;
  }
  // the last grid level's predicated cleanup did the work (its tag is the
  // pending one); a search that ended before any grid level cleans up here
  if (grid && !I.grid_cleaned) I.cleanup_async();
  if (timed_by_events) {
    HIP_CHECK(hipEventSynchronize(I.ev1));
    float ms = 0;
    HIP_CHECK(hipEventElapsedTime(&ms, I.ev0, I.ev1));
    r.search_ms += ms;
  }
  if (opt.trace) I.fetch_trace(r);
  if (opt.trace && env::stamps()) {
    I.fetch_clock(r);
    I.fetch_grid_stamps(r);
  }
  return r;
}

// ---------------------------------------------------------------- step-wise API

void HipBiBfs::begin(vid_t src, vid_t dst) {
  auto& I = *p_;
  BIBFS_REQUIRE(I.n > 0, "no graph loaded");
  BIBFS_REQUIRE(src < I.n && dst < I.n, "src/dst out of range");
  HIP_CHECK(hipSetDevice(I.device));
  I.step_src = src;
  I.step_dst = dst;
  I.fbits_valid[0] = I.fbits_valid[1] = false;
  I.dir[0] = I.dir[1] = 1;
  launch::seed_state(I.view(), I.buf, src, dst, I.stream);
  I.sync_state();
}

uint64_t HipBiBfs::expand(int side, bool* met, Direction dir) {
  auto& I = *p_;
  BIBFS_REQUIRE(side == 0 || side == 1, "side must be 0 or 1");
  const uint32_t before = I.h_state->qtail[side];
  if (I.h_state->status != kRunning) {
    if (met) *met = I.h_state->meet != kEmpty;
    return 0;
  }
  I.grid_level(side, dir == Direction::kBottomUp ? 2 : 1, 0);
  if (met) *met = I.h_state->meet != kEmpty;
  return I.h_state->qtail[side] - before;
}

bool HipBiBfs::check_meet() {
  auto& I = *p_;
  launch::bitmap_meet(I.buf, I.d_flag, I.stream);
  uint32_t f = 0;
  HIP_CHECK(hipMemcpyAsync(&f, I.d_flag, 4, hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  return f != 0;
}

SearchResult HipBiBfs::finish() {
  auto& I = *p_;
  SearchResult r;
  if (I.step_src == I.step_dst) {
    r.found = true;
    r.hops = 0;
    r.meet = I.step_src;
    r.path = {I.step_src};
  } else {
    const uint32_t seq = ++I.seq == 0 ? ++I.seq : I.seq;
    launch::HostSide hs{I.h_res, I.h_path, I.h_path_cap, I.h_state};
    launch::walk_path(I.buf, hs, I.step_src, I.step_dst, seq, I.n, I.stream);
    I.wait_seq(seq);
    SearchOptions opt;
    r = I.collect(*I.h_res, opt, SearchStats{});
  }
  I.cleanup_async();
  HIP_CHECK(hipStreamSynchronize(I.stream));
  return r;
}

// ---------------------------------------------------------------- test helpers

Csr HipBiBfs::download_csr() const {
  const auto& I = *p_;
  Csr g;
  g.n = I.n;
  g.m_input = I.m_input;
  g.row_off.resize((size_t)I.n + 1);
  g.col.resize(I.nnz);
  HIP_CHECK(hipMemcpyAsync(g.row_off.data(), I.d_row_off, ((size_t)I.n + 1) * 8, hipMemcpyDeviceToHost,
                           I.stream));
  if (I.nnz)
    HIP_CHECK(hipMemcpyAsync(g.col.data(), I.d_col, I.nnz * 4, hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  return g;
}

// Row u of the device CSR (for checking paths on graphs too large to copy to
// the host: one row per call).
std::vector<vid_t> HipBiBfs::neighbors(vid_t u) const {
  const auto& I = *p_;
  BIBFS_REQUIRE(u < I.n, "neighbors: vertex out of range");
  uint64_t r[2];
  HIP_CHECK(hipMemcpyAsync(r, I.d_row_off + u, 16, hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  std::vector<vid_t> out(r[1] - r[0]);
  if (!out.empty())
    HIP_CHECK(hipMemcpyAsync(out.data(), I.d_col + r[0], out.size() * 4, hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  return out;
}

EdgeList HipBiBfs::download_edges() const {
  const auto& I = *p_;
  EdgeList el;
  el.n = I.n;
  BIBFS_REQUIRE(I.d_uv != nullptr, "no device-generated edge list resident");
  el.uv.resize(2 * I.uv_m);
  if (I.uv_m)
    HIP_CHECK(hipMemcpyAsync(el.uv.data(), I.d_uv, I.uv_m * 8, hipMemcpyDeviceToHost, I.stream));
  HIP_CHECK(hipStreamSynchronize(I.stream));
  return el;
}

}  // namespace bibfs
