// Seeded graph generators (host side).  Device twins live in
// csrc/hip/gen_device.hip and produce bit-identical edge lists (rng.hpp).
//
// Reference: graphs/generate_graph.py:31 (networkx fast_gnp_random_graph,
// unseeded) and graphs/make_graphs:8-13 (p = 2.2000000001 / N).  The native
// generator adds a seed, avoids the O(N^2) dense matrix the reference builds
// (generate_graph.py:32, the "900 GBs" complaint of README.md:19) and adds
// R-MAT / Kronecker for the BASELINE.json RMAT-22 and scale-27 configs.
#pragma once

#include "bibfs/graph.hpp"
#include "bibfs/rng.hpp"

namespace bibfs {

EdgeList gen_gnp(uint32_t n, double p, uint64_t seed, int threads = 0);
// R-MAT with `m` edges on n vertices (n need not be a power of two).
EdgeList gen_rmat(uint32_t n, uint64_t m, uint64_t seed, double a = 0.57, double b = 0.19,
                  double c = 0.19, int threads = 0);
// Graph500-style Kronecker: n = 2^scale, m = edgefactor * n.
EdgeList gen_kronecker(int scale, int edgefactor, uint64_t seed, int threads = 0);

// Reference suite density (graphs/make_graphs:8): p = 2.2000000001 / N.
inline double reference_p(uint32_t n) { return 2.2000000001 / (double)n; }

}  // namespace bibfs
