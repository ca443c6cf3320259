// Common definitions shared by every translation unit of the bibfs native core.
//
// The reference (Tomaszbrauntsch/Bidirectional-BFS) uses int32 everywhere
// (v3/bibfs_cuda_only.cu:89-99, v4/mpi_bas.cpp:45-57), which caps the graph at
// 2^31 directed CSR entries.  This core uses 32-bit vertex ids and 64-bit edge
// offsets so a scale-27 Kronecker graph (2^32 directed entries) is addressable.
#pragma once

#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>

#if defined(__HIPCC__)
#define BIBFS_HD __host__ __device__
#else
#define BIBFS_HD
#endif

namespace bibfs {

using vid_t = uint32_t;   // vertex id
using eoff_t = uint64_t;  // edge offset into CSR column array

constexpr vid_t kNoVertex = 0xFFFFFFFFu;

// Error type used by the whole core; the CLI tools print e.what() and exit 1,
// matching the reference's "print + exit" error style (v1/main-v1.cpp:23-34).
struct Error : std::runtime_error {
  explicit Error(const std::string& m) : std::runtime_error(m) {}
};

#define BIBFS_REQUIRE(cond, msg)                                              \
  do {                                                                        \
    if (!(cond)) throw ::bibfs::Error(std::string(msg));                      \
  } while (0)

}  // namespace bibfs
