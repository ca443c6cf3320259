// bibfs_serial <graph_file> <src> <dst> [--repeat R] [--json] [--verify] [--side edges|frontier]
//
// v1 capability (reference v1/main-v1.cpp): serial bidirectional BFS on the CPU.
// Same argv and stdout lines; times the search only, like v1 (:49,82,100),
// and additionally reports load / CSR-build time with --json.
#include "cli_common.hpp"

int main(int argc, char** argv) {
  auto a = cli::parse(argc, argv, {"repeat", "side", "direction"});
  if (a.pos.size() != 3) {
    std::fprintf(stderr, "Usage: %s <graph_file> <src> <dst> [--repeat R] [--json] [--verify]\n", argv[0]);
    return 1;
  }
  try {
    const std::string graph = a.pos[0];
    const bibfs::vid_t src = (bibfs::vid_t)std::atoll(a.pos[1].c_str());
    const bibfs::vid_t dst = (bibfs::vid_t)std::atoll(a.pos[2].c_str());
    double t0 = cli::now_s();
    bibfs::EdgeList el = cli::edges_from_spec(graph);
    double t1 = cli::now_s();
    bibfs::Csr g = bibfs::build_csr(el);
    double t2 = cli::now_s();
    if (src >= g.n || dst >= g.n) {
      std::fprintf(stderr, "src/dst must be < N = %u\n", g.n);
      return 1;
    }
    bibfs::SerialBiBfs eng(g);
    auto opt = cli::options_from(a);
    const int repeat = (int)std::max(1LL, a.geti("repeat", 1));
    std::vector<double> ts;
    bibfs::SearchResult r;
    for (int i = 0; i < repeat; ++i) {
      r = eng.search(src, dst, opt);
      ts.push_back(r.search_ms);
    }
    const double med = cli::median(ts);
    if (a.has("json")) {
      cli::print_json(r, "serial", graph, g.n, g.m_input, src, dst, (t1 - t0) * 1e3, (t2 - t1) * 1e3, med, med,
                      repeat, 0);
      return 0;
    }
    cli::print_result(r, src, dst);
    for (auto& t : r.stats.trace)
      std::printf("Level side=%d depth=%d frontier=%llu edges=%llu new=%llu mode=cpu\n", t.side, t.depth,
                  (unsigned long long)t.frontier, (unsigned long long)t.edges,
                  (unsigned long long)t.discovered);
    std::printf("Serial bidirectional BFS took %.9g seconds\n", med * 1e-3);
    if (a.has("verify")) {
      auto o = bibfs::bfs_oracle(g, src, dst);
      std::string why;
      bool ok = o.hops == r.hops && (!r.found || bibfs::validate_path(g, src, dst, r.hops, r.path, &why));
      std::printf("Verify: %s (oracle hops = %lld)%s%s\n", ok ? "OK" : "MISMATCH", (long long)o.hops,
                  why.empty() ? "" : " ", why.c_str());
      if (!ok) return 2;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
