// Search result returned by every engine (CPU serial, CPU MPI, HIP single-GPU,
// HIP multi-GPU).  The reference engines each print a different subset
// (v3 prints no hop count, v2 a wrong one); here every
// engine returns the same record and the CLIs print the reference lines from it.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "bibfs/common.hpp"

namespace bibfs {

enum class Direction : int { kAuto = 0, kTopDown = 1, kBottomUp = 2 };

// Which frontier expands next.  kSmallerEdges is the default for every engine;
// kSmallerFrontier is v1's rule (v1/main-v1.cpp:51), kAlternate the strict
// S-then-T order of v2/main-v2.cpp:45-131.
enum class SidePolicy : int { kSmallerEdges = 0, kSmallerFrontier = 1, kAlternate = 2 };

struct SearchOptions {
  SidePolicy side = SidePolicy::kSmallerEdges;
  Direction direction = Direction::kAuto;
  double alpha = 14.0;   // Beamer top-down -> bottom-up switch: m_f > m_u / alpha
  double beta = 24.0;    // bottom-up -> top-down switch: n_f < n / beta
  bool want_path = true;
  bool force_grid = false;     // GPU: skip the single-workgroup LDS engine
  bool lockstep = true;        // GPU LDS engine: expand both small frontiers concurrently
  bool trace = false;          // record per-level trace
};

struct LevelTrace {
  int side = 0;             // 0 = source side, 1 = target side
  int depth = 0;            // depth of the frontier that was expanded
  uint64_t frontier = 0;    // vertices expanded
  uint64_t edges = 0;       // edges inspected
  uint64_t discovered = 0;  // newly claimed vertices
  int mode = 0;  // 0 CPU, 1 LDS lockstep round, 2 LDS single wave, 3 LDS all waves, 4 grid top-down,
                 // 5 grid bottom-up, 9 LDS meet probe (a level ended at its first meet, edges = edges read)
};

struct SearchStats {
  int levels = 0;              // half-steps performed
  uint64_t edges_inspected = 0;
  uint64_t visited = 0;        // vertices claimed by both sides (incl. src/dst)
  int grid_levels = 0;         // GPU: levels run by the grid engine
  int bottomup_levels = 0;
  bool handoff = false;        // GPU: persistent engine handed off to the grid engine
  double lds_ms = 0.0;         // GPU: device time of the one-workgroup (LDS / tiny) phase
  int lds_levels = 0;          // GPU: levels that phase ran (before a hand-off)
  double walk_ms = 0.0;        // GPU: the grid publish's path walk + result record (hand-off searches)
  uint64_t probe_edges = 0;    // GPU: frontier edges the LDS engine's meet probe read before a hand-off
  bool probe_hit = false;      // GPU: ... and it found the meet (no hand-off)
  std::vector<LevelTrace> trace;
};

struct SearchResult {
  bool found = false;
  int64_t hops = -1;            // BFS distance; -1 when unreachable
  std::vector<vid_t> path;      // src .. dst, hops + 1 vertices (empty when !found)
  vid_t meet = kNoVertex;       // vertex where the two searches met
  SearchStats stats;
  double search_ms = 0.0;       // engine-internal search time (device time for GPU)
  double total_ms = 0.0;        // wall time of the search call (query -> path on host)
};

}  // namespace bibfs
