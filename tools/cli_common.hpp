// Shared CLI helpers: the reference's positional argv (<graph.bin> <src> <dst>,
// SURVEY.md §2.7) plus optional flags, and the reference-compatible stdout
// lines that benchmark_test.sh:61-69 parses (first number on the first line
// matching /search time|^\[time\]|took[[:space:]]+[0-9]|gpu bfs time/, in
// SECONDS -- the reference's v3 printed milliseconds there).
#pragma once

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "bibfs/cpu_engine.hpp"
#include "bibfs/gen.hpp"
#include "bibfs/io.hpp"

namespace cli {

struct Args {
  std::vector<std::string> pos;
  std::vector<std::pair<std::string, std::string>> kv;
  bool has(const std::string& k) const {
    for (auto& p : kv)
      if (p.first == k) return true;
    return false;
  }
  std::string get(const std::string& k, const std::string& def = "") const {
    for (auto& p : kv)
      if (p.first == k) return p.second;
    return def;
  }
  long long geti(const std::string& k, long long def) const {
    std::string v = get(k, "");
    return v.empty() ? def : std::atoll(v.c_str());
  }
  double getd(const std::string& k, double def) const {
    std::string v = get(k, "");
    return v.empty() ? def : std::atof(v.c_str());
  }
};

// --flag, --key=value, --key value (value-taking keys listed in `valued`)
inline Args parse(int argc, char** argv, const std::vector<std::string>& valued) {
  Args a;
  for (int i = 1; i < argc; ++i) {
    std::string s = argv[i];
    if (s.rfind("--", 0) == 0) {
      std::string k = s.substr(2), v;
      size_t eq = k.find('=');
      if (eq != std::string::npos) {
        v = k.substr(eq + 1);
        k = k.substr(0, eq);
      } else {
        for (auto& x : valued)
          if (x == k && i + 1 < argc) {
            v = argv[++i];
            break;
          }
      }
      a.kv.emplace_back(k, v);
    } else {
      a.pos.push_back(s);
    }
  }
  return a;
}

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline bibfs::SearchOptions options_from(const Args& a) {
  bibfs::SearchOptions o;
  std::string side = a.get("side", "edges");
  if (side == "frontier") o.side = bibfs::SidePolicy::kSmallerFrontier;
  else if (side == "alternate") o.side = bibfs::SidePolicy::kAlternate;
  std::string d = a.get("direction", "auto");
  if (d == "topdown") o.direction = bibfs::Direction::kTopDown;
  else if (d == "bottomup") o.direction = bibfs::Direction::kBottomUp;
  o.alpha = a.getd("alpha", o.alpha);
  o.beta = a.getd("beta", o.beta);
  o.force_grid = a.has("force-grid");
  o.trace = a.has("trace");
  o.lockstep = !a.has("no-lockstep");
  return o;
}

// Reference stdout contract (v1/main-v1.cpp:84-101, v4/mpi_bas.cpp:137-163).
inline void print_result(const bibfs::SearchResult& r, bibfs::vid_t src, bibfs::vid_t dst,
                         bool print_path = true) {
  if (!r.found) {
    std::printf("No path found between %u and %u\n", src, dst);
    return;
  }
  std::printf("Shortest path length = %lld\n", (long long)r.hops);
  if (print_path && !r.path.empty()) {
    std::string line = "Path:";
    char buf[16];
    for (auto v : r.path) {
      std::snprintf(buf, sizeof buf, " %u", v);
      line += buf;
    }
    std::printf("%s\n", line.c_str());
  }
}

inline void print_path(const bibfs::SearchResult& r) {
  if (!r.found || r.path.empty()) return;
  std::string line = "Path:";
  char buf[16];
  for (auto v : r.path) {
    std::snprintf(buf, sizeof buf, " %u", v);
    line += buf;
  }
  std::printf("%s\n", line.c_str());
}

inline void print_json(const bibfs::SearchResult& r, const std::string& engine, const std::string& graph,
                       uint32_t n, uint64_t m, bibfs::vid_t src, bibfs::vid_t dst, double load_ms,
                       double build_ms, double median_search_ms, double median_total_ms, int repeat,
                       int gpus) {
  const double gteps = median_total_ms > 0 ? (double)m / (median_total_ms * 1e-3) / 1e9 : 0.0;
  const double gteps_insp =
      median_total_ms > 0 ? (double)r.stats.edges_inspected / (median_total_ms * 1e-3) / 1e9 : 0.0;
  std::printf(
      "{\"engine\": \"%s\", \"graph\": \"%s\", \"n\": %u, \"m\": %llu, \"src\": %u, \"dst\": %u, "
      "\"found\": %s, \"hops\": %lld, \"levels\": %d, \"edges_inspected\": %llu, \"visited\": %llu, "
      "\"load_ms\": %.6f, \"build_ms\": %.6f, \"search_ms\": %.6f, \"query_ms\": %.6f, "
      "\"end_to_end_ms\": %.6f, \"gteps\": %.6f, \"gteps_inspected\": %.6f, \"repeat\": %d, "
      "\"gpus\": %d, \"handoff\": %s, \"grid_levels\": %d}\n",
      engine.c_str(), graph.c_str(), n, (unsigned long long)m, src, dst, r.found ? "true" : "false",
      (long long)r.hops, r.stats.levels, (unsigned long long)r.stats.edges_inspected,
      (unsigned long long)r.stats.visited, load_ms, build_ms, median_search_ms, median_total_ms,
      load_ms + build_ms + median_total_ms, gteps, gteps_insp, repeat, gpus,
      r.stats.handoff ? "true" : "false", r.stats.grid_levels);
}

inline double median(std::vector<double> v) {
  if (v.empty()) return 0.0;
  std::sort(v.begin(), v.end());
  return v.size() % 2 ? v[v.size() / 2] : 0.5 * (v[v.size() / 2 - 1] + v[v.size() / 2]);
}

// Accepts "<graph.bin>" or a generator spec "gnp:N[:p[:seed]]", "rmat:N:M[:seed]",
// "kron:SCALE[:EF[:seed]]" so large configs need no file on disk.
inline bool is_spec(const std::string& g) {
  return g.rfind("gnp:", 0) == 0 || g.rfind("rmat:", 0) == 0 || g.rfind("kron:", 0) == 0;
}

inline std::vector<std::string> split(const std::string& s, char c) {
  std::vector<std::string> out;
  size_t b = 0;
  for (;;) {
    size_t e = s.find(c, b);
    out.push_back(s.substr(b, e == std::string::npos ? std::string::npos : e - b));
    if (e == std::string::npos) break;
    b = e + 1;
  }
  return out;
}

inline bibfs::EdgeList edges_from_spec(const std::string& g) {
  auto f = split(g, ':');
  if (f[0] == "gnp") {
    uint32_t n = (uint32_t)std::atoll(f.at(1).c_str());
    double p = f.size() > 2 && !f[2].empty() ? std::atof(f[2].c_str()) : bibfs::reference_p(n);
    uint64_t seed = f.size() > 3 ? std::strtoull(f[3].c_str(), nullptr, 10) : 1;
    return bibfs::gen_gnp(n, p, seed);
  }
  if (f[0] == "rmat") {
    uint32_t n = (uint32_t)std::atoll(f.at(1).c_str());
    uint64_t m = std::strtoull(f.at(2).c_str(), nullptr, 10);
    uint64_t seed = f.size() > 3 ? std::strtoull(f[3].c_str(), nullptr, 10) : 1;
    return bibfs::gen_rmat(n, m, seed);
  }
  if (f[0] == "kron") {
    int scale = std::atoi(f.at(1).c_str());
    int ef = f.size() > 2 ? std::atoi(f[2].c_str()) : 16;
    uint64_t seed = f.size() > 3 ? std::strtoull(f[3].c_str(), nullptr, 10) : 1;
    return bibfs::gen_kronecker(scale, ef, seed);
  }
  return bibfs::read_bin(g);
}

}  // namespace cli
