// bibfs_selftest [spec...] : device-vs-host consistency checks for the HIP engine
// (CSR build, generators, LDS engine, grid engine) against the CPU oracle.
// Used for bring-up on the GPU box; the pytest GPU suite covers the same
// ground through the Python bindings.
#include <algorithm>
#include <random>

#include "bibfs/hip_engine.hpp"
#include "cli_common.hpp"

using namespace bibfs;

static int failures = 0;
#define CHECK(c, ...)                      \
  do {                                     \
    if (!(c)) {                            \
      std::printf("FAIL: " __VA_ARGS__);   \
      std::printf("\n");                   \
      ++failures;                          \
    }                                      \
  } while (0)

static bool same_csr(const Csr& a, const Csr& b) {
  if (a.n != b.n || a.nnz() != b.nnz()) {
    std::printf("  csr size mismatch n %u/%u nnz %llu/%llu\n", a.n, b.n, (unsigned long long)a.nnz(),
                (unsigned long long)b.nnz());
    return false;
  }
  for (uint32_t v = 0; v < a.n; ++v) {
    if (a.row_off[v] != b.row_off[v]) {
      std::printf("  row_off[%u] %llu vs %llu\n", v, (unsigned long long)a.row_off[v], (unsigned long long)b.row_off[v]);
      return false;
    }
    std::vector<uint32_t> x(a.col.begin() + a.row_off[v], a.col.begin() + a.row_off[v + 1]);
    std::vector<uint32_t> y(b.col.begin() + b.row_off[v], b.col.begin() + b.row_off[v + 1]);
    std::sort(x.begin(), x.end());
    std::sort(y.begin(), y.end());
    if (x != y) {
      std::printf("  row %u differs: host [", v);
      for (auto t : x) std::printf(" %u", t);
      std::printf(" ] dev [");
      for (auto t : y) std::printf(" %u", t);
      std::printf(" ] row_off host %llu..%llu dev %llu..%llu\n", (unsigned long long)a.row_off[v],
                  (unsigned long long)a.row_off[v + 1], (unsigned long long)b.row_off[v],
                  (unsigned long long)b.row_off[v + 1]);
      std::printf("  dev row_off[0..16]:");
      for (int i = 0; i < 16 && i <= (int)b.n; ++i) std::printf(" %llu", (unsigned long long)b.row_off[i]);
      std::printf("\n  host row_off[0..16]:");
      for (int i = 0; i < 16 && i <= (int)a.n; ++i) std::printf(" %llu", (unsigned long long)a.row_off[i]);
      std::printf("\n  dev col[0..16]:");
      for (int i = 0; i < 16 && i < (int)b.nnz(); ++i) std::printf(" %u", b.col[i]);
      std::printf("\n");
      return false;
    }
  }
  return true;
}

static void check_searches(HipBiBfs& eng, const Csr& g, int nq, uint64_t seed, const SearchOptions& opt,
                           const char* tag) {
  std::mt19937_64 rng(seed);
  int bad = 0;
  double tsum = 0;
  for (int q = 0; q < nq; ++q) {
    vid_t s = q == 0 ? 0 : (vid_t)(rng() % g.n), d = q == 0 ? g.n - 1 : (vid_t)(rng() % g.n);
    auto o = bfs_oracle(g, s, d);
    auto r = eng.search(s, d, opt);
    tsum += r.total_ms;
    std::string why;
    bool ok = (o.hops == r.hops) && (!r.found || validate_path(g, s, d, r.hops, r.path, &why));
    if (!ok && bad < 5)
      std::printf("  [%s] query %u->%u: oracle %lld got %lld %s levels=%d handoff=%d\n", tag, s, d,
                  (long long)o.hops, (long long)r.hops, why.c_str(), r.stats.levels, (int)r.stats.handoff);
    bad += !ok;
  }
  std::printf("  [%s] %d/%d queries correct, mean query %.3f ms\n", tag, nq - bad, nq, tsum / nq);
  CHECK(bad == 0, "%s: %d wrong answers", tag, bad);
}

int main(int argc, char** argv) {
  std::setvbuf(stdout, nullptr, _IOLBF, 0);  // line-buffered: a killed run still shows how far it got
  std::vector<std::string> specs;
  for (int i = 1; i < argc; ++i) specs.push_back(argv[i]);
  if (specs.empty()) specs = {"gnp:1000::1", "gnp:100000::6", "rmat:65536:1048576:3"};
  try {
    HipBiBfs eng(0);
    auto inf = eng.info();
    std::printf("device %s arch %s cus %d hbm %.1f GB lds/block %d\n", inf.name.c_str(), inf.arch.c_str(),
                inf.cus, inf.hbm_bytes / 1e9, inf.lds_bytes);
    for (const auto& sp : specs) {
      std::printf("== %s\n", sp.c_str());
      EdgeList el = cli::edges_from_spec(sp);
      Csr host = build_csr(el);
      // 1. device CSR build from an uploaded edge list
      eng.load_edges(el);
      Csr dev = eng.download_csr();
      CHECK(same_csr(host, dev), "%s: device CSR differs from host CSR", sp.c_str());
      if (failures) { std::printf("stopping before searches\n"); return 1; }
      SearchOptions o;
      check_searches(eng, host, 40, 11, o, "lds");
      SearchOptions nl;
      nl.lockstep = false;
      check_searches(eng, host, 20, 16, nl, "lds-nolock");
      SearchOptions al;
      al.side = SidePolicy::kAlternate;
      check_searches(eng, host, 10, 17, al, "lds-alt");
      // resident server: queries through the pinned mailbox, interleaved with
      // one-shot and grid queries (the server must stay consistent)
      eng.set_resident(true);
      check_searches(eng, host, 40, 18, o, "lds-resident");
      check_searches(eng, host, 5, 19, nl, "lds-resident-nolock");
      eng.set_resident(false);
      {  // batched: one workgroup per query
        std::mt19937_64 rng(23);
        std::vector<vid_t> bs, bd;
        for (int q = 0; q < 300; ++q) {
          bs.push_back(q == 0 ? 0 : (vid_t)(rng() % host.n));
          bd.push_back(q == 0 ? host.n - 1 : (vid_t)(rng() % host.n));
        }
        const double tb = cli::now_s();
        auto rs = eng.search_batch(bs, bd, o);
        const double dt = (cli::now_s() - tb) * 1e3;
        int bad = 0;
        for (size_t q = 0; q < rs.size(); ++q) {
          auto orc = bfs_oracle(host, bs[q], bd[q]);
          std::string why;
          bool ok = orc.hops == rs[q].hops &&
                    (!rs[q].found || validate_path(host, bs[q], bd[q], rs[q].hops, rs[q].path, &why));
          if (!ok && bad < 5)
            std::printf("  [lds-batch] query %u->%u: oracle %lld got %lld %s\n", bs[q], bd[q],
                        (long long)orc.hops, (long long)rs[q].hops, why.c_str());
          bad += !ok;
        }
        std::printf("  [lds-batch] %d/%zu queries correct, %.3f ms for the batch (%.1f us/query)\n",
                    (int)rs.size() - bad, rs.size(), dt, dt * 1e3 / rs.size());
        CHECK(bad == 0, "lds-batch: %d wrong answers", bad);
      }
      SearchOptions g;
      g.force_grid = true;
      check_searches(eng, host, 20, 12, g, "grid-auto");
      g.direction = Direction::kTopDown;
      check_searches(eng, host, 10, 13, g, "grid-td");
      g.direction = Direction::kBottomUp;
      check_searches(eng, host, 10, 14, g, "grid-bu");
      // 2. uploaded host CSR
      eng.load_csr(host);
      check_searches(eng, host, 10, 15, o, "lds-hostcsr");
    }
    // 3. device generators == host generators
    {
      eng.generate_gnp(20000, 3.0 / 20000, 9);
      EdgeList d = eng.download_edges(), h = gen_gnp(20000, 3.0 / 20000, 9);
      CHECK(d.uv == h.uv, "device G(n,p) != host G(n,p) (m %llu vs %llu)", (unsigned long long)d.m(),
            (unsigned long long)h.m());
      eng.generate_rmat(30000, 200000, 5);
      EdgeList d2 = eng.download_edges(), h2 = gen_rmat(30000, 200000, 5);
      CHECK(d2.uv == h2.uv, "device R-MAT != host R-MAT");
      std::printf("  generators: device == host checked\n");
    }
  } catch (const std::exception& e) {
    std::printf("EXCEPTION: %s\n", e.what());
    return 3;
  }
  std::printf(failures ? "SELFTEST FAILED (%d)\n" : "SELFTEST PASSED\n", failures);
  return failures ? 1 : 0;
}
