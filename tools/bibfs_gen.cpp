// bibfs_gen --type gnp|rmat|kron --n N [--p P | --avg-deg D] [--m M] [--scale S --edgefactor EF]
//           [--seed S] [--src S] [--dst D] --out FILE.bin [--no-json] [--csr-cache FILE.csr]
//
// Native counterpart of graphs/generate_graph.py (C16): writes the same .bin
// edge list and .json sidecar ({"source","target","hop_count","nodes"}), but
// seeded, multi-threaded and without the O(N^2) dense matrix of
// generate_graph.py:32.  The sidecar's ground truth comes from an independent
// single-source BFS (bfs_oracle), not from the bidirectional engines.
#include "cli_common.hpp"

int main(int argc, char** argv) {
  auto a = cli::parse(argc, argv, {"type", "n", "p", "avg-deg", "m", "scale", "edgefactor", "seed", "src", "dst",
                                   "out", "csr-cache"});
  const std::string out = a.get("out", "");
  if (out.empty()) {
    std::fprintf(stderr,
                 "Usage: %s --type gnp|rmat|kron --n N [--p P|--avg-deg D] [--m M] [--scale S] [--seed S] "
                 "[--src S] [--dst D] --out FILE.bin\n",
                 argv[0]);
    return 1;
  }
  try {
    const std::string type = a.get("type", "gnp");
    const uint64_t seed = (uint64_t)a.geti("seed", 1);
    bibfs::EdgeList el;
    double t0 = cli::now_s();
    if (type == "gnp") {
      uint32_t n = (uint32_t)a.geti("n", 50000);
      double p = a.has("p") ? a.getd("p", 0) : (a.has("avg-deg") ? a.getd("avg-deg", 2.2) / n : bibfs::reference_p(n));
      std::printf("Generating G(%u, p=%.12g) seed=%llu\n", n, p, (unsigned long long)seed);
      el = bibfs::gen_gnp(n, p, seed);
    } else if (type == "rmat") {
      uint32_t n = (uint32_t)a.geti("n", 1 << 20);
      uint64_t m = (uint64_t)a.geti("m", 16LL * n);
      std::printf("Generating R-MAT(n=%u, m=%llu) seed=%llu\n", n, (unsigned long long)m, (unsigned long long)seed);
      el = bibfs::gen_rmat(n, m, seed);
    } else if (type == "kron") {
      int scale = (int)a.geti("scale", 20), ef = (int)a.geti("edgefactor", 16);
      std::printf("Generating Kronecker(scale=%d, edgefactor=%d) seed=%llu\n", scale, ef, (unsigned long long)seed);
      el = bibfs::gen_kronecker(scale, ef, seed);
    } else {
      std::fprintf(stderr, "unknown --type %s\n", type.c_str());
      return 1;
    }
    std::printf("  n=%u m=%llu (%.3f s)\n", el.n, (unsigned long long)el.m(), cli::now_s() - t0);
    bibfs::write_bin(out, el);
    std::printf("Wrote %s\n", out.c_str());
    if (!a.has("no-json") || a.has("csr-cache")) {
      bibfs::Csr g = bibfs::build_csr(el);
      if (a.has("csr-cache")) {
        bibfs::write_csr_cache(a.get("csr-cache"), g);
        std::printf("Wrote %s\n", a.get("csr-cache").c_str());
      }
      if (!a.has("no-json")) {
        bibfs::vid_t src = (bibfs::vid_t)a.geti("src", 0);
        bibfs::vid_t dst = (bibfs::vid_t)a.geti("dst", (long long)el.n - 1);
        std::printf("Computing shortest path from %u to %u\n", src, dst);
        auto r = bibfs::bfs_oracle(g, src, dst);
        bibfs::PathJson pj;
        pj.source = src;
        pj.target = dst;
        if (r.found) {
          pj.hop_count = r.hops;
          for (auto v : r.path) pj.nodes.push_back(v);
          std::printf("  -> hop count = %lld\n", (long long)r.hops);
        } else {
          std::printf("  -> no path found\n");
        }
        const std::string js = bibfs::sidecar_path(out);
        bibfs::write_path_json(js, pj);
        std::printf("Wrote path info to %s\n", js.c_str());
      }
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
