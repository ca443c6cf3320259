// bibfs_bench <graph.bin | spec> [--queries Q] [--warmup W] [--seed S] [--src S --dst D]
//             [--engine hip|serial] [--json] [--force-grid]
//
// Native benchmark driver (the reference's harness, benchmark_test.sh, ran
// every binary once per graph with no warm-up).  Runs W warm-up queries then
// Q timed queries -- (src, dst) = (0, N-1) first, then seeded random pairs --
// and reports median / p10 / p90 query latency, search-only device time,
// load + CSR build time and GTEPS = M / t (input edges over query time, the
// BASELINE.md normalisation) plus GTEPS over inspected edges.
#include <random>

#include "bibfs/hip_engine.hpp"
#include "cli_common.hpp"

int main(int argc, char** argv) {
  auto a = cli::parse(argc, argv, {"queries", "warmup", "seed", "src", "dst", "engine", "side", "direction"});
  if (a.pos.size() != 1) {
    std::fprintf(stderr, "Usage: %s <graph.bin|spec> [--queries Q] [--warmup W] [--json]\n", argv[0]);
    return 1;
  }
  try {
    const std::string graph = a.pos[0];
    const int Q = (int)a.geti("queries", 100), W = (int)a.geti("warmup", 10);
    const std::string engine = a.get("engine", "hip");
    double t0 = cli::now_s();
    bibfs::EdgeList el = cli::edges_from_spec(graph);
    const double load_ms = (cli::now_s() - t0) * 1e3;
    const uint32_t n = el.n;
    const uint64_t m = el.m();
    std::mt19937_64 rng((uint64_t)a.geti("seed", 7));
    std::vector<std::pair<uint32_t, uint32_t>> pairs;
    if (a.has("src")) pairs.emplace_back((uint32_t)a.geti("src", 0), (uint32_t)a.geti("dst", (long long)n - 1));
    else pairs.emplace_back(0u, n - 1);
    while ((int)pairs.size() < Q + W) pairs.emplace_back((uint32_t)(rng() % n), (uint32_t)(rng() % n));
    auto opt = cli::options_from(a);
    std::vector<double> tq, ts;
    uint64_t insp = 0, found = 0;
    double build_ms = 0;
    auto run = [&](auto&& search) {
      for (int i = 0; i < W; ++i) search(pairs[(size_t)(i + 1) % pairs.size()]);
      for (int i = 0; i < Q; ++i) {
        auto r = search(pairs[(size_t)i]);
        tq.push_back(r.total_ms);
        ts.push_back(r.search_ms);
        insp += r.stats.edges_inspected;
        found += r.found;
      }
    };
    if (engine == "serial") {
      double tb = cli::now_s();
      bibfs::Csr g = bibfs::build_csr(el);
      build_ms = (cli::now_s() - tb) * 1e3;
      bibfs::SerialBiBfs eng(g);
      run([&](std::pair<uint32_t, uint32_t> p) { return eng.search(p.first, p.second, opt); });
    } else {
      bibfs::HipBiBfs eng(0);
      eng.load_edges(el);
      build_ms = eng.last_build_ms();
      run([&](std::pair<uint32_t, uint32_t> p) { return eng.search(p.first, p.second, opt); });
    }
    std::vector<double> sq = tq;
    std::sort(sq.begin(), sq.end());
    auto pct = [&](double f) { return sq[(size_t)std::min<double>(sq.size() - 1, f * (sq.size() - 1))]; };
    const double med = cli::median(tq), meds = cli::median(ts);
    double mean = 0;
    for (double x : tq) mean += x;
    mean /= std::max<size_t>(1, tq.size());
    const double gteps = (double)m / (med * 1e-3) / 1e9;
    const double gteps_insp = (double)insp / Q / (mean * 1e-3) / 1e9;
    std::printf(
        "{\"engine\": \"%s\", \"graph\": \"%s\", \"n\": %u, \"m\": %llu, \"queries\": %d, \"found\": %llu, "
        "\"first_query_ms\": %.6f, \"median_query_ms\": %.6f, \"p10_ms\": %.6f, \"p90_ms\": %.6f, "
        "\"mean_query_ms\": %.6f, \"median_search_ms\": %.6f, \"load_ms\": %.3f, \"build_ms\": %.3f, "
        "\"gteps\": %.4f, \"gteps_inspected\": %.6f, \"queries_per_s\": %.1f}\n",
        engine.c_str(), graph.c_str(), n, (unsigned long long)m, Q, (unsigned long long)found, tq[0], med,
        pct(0.1), pct(0.9), mean, meds, load_ms, build_ms, gteps, gteps_insp, 1e3 / mean);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
