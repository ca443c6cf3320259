// Device-memory accounting for one rank's graph build and search state.
//
// A Tracker counts the bytes a rank holds through devmem::alloc (current and
// peak, exact: temporaries of the CSR build -- scan partials, the scatter
// cursor -- included) and can enforce a per-rank cap.  It also samples
// hipMemGetInfo at every tracked allocation, so the device's own low-water
// mark (free memory before the build minus the least seen during it) is
// reported beside the count; with one rank per GPU the two agree up to the
// allocator's granularity, with several ranks on one GPU only the count is
// per rank.
//
// The tracker is installed per thread (devmem::Scope), so the local-group
// test ranks (threads of one process) each count their own allocations.
// Code that runs with no tracker installed allocates as plain hipMalloc.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

#include "bibfs/common.hpp"

namespace bibfs {
namespace devmem {

struct Tracker {
  size_t cur = 0;        // bytes held now
  size_t peak = 0;       // most bytes held at once since reset_peak()
  size_t cap = 0;        // 0 = no cap; else alloc() past it throws
  size_t free_start = 0; // hipMemGetInfo free bytes at reset_peak()
  size_t free_low = 0;   // least free bytes seen since reset_peak()
  void reset_peak() {
    peak = cur;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess) free_start = free_low = fr;
  }
  size_t hbm_peak() const { return free_start > free_low ? free_start - free_low : 0; }
};

inline Tracker*& current() {
  static thread_local Tracker* t = nullptr;
  return t;
}

// RAII: install `t` as this thread's tracker for the scope.
struct Scope {
  Tracker* prev;
  explicit Scope(Tracker* t) : prev(current()) { current() = t; }
  ~Scope() { current() = prev; }
  Scope(const Scope&) = delete;
  Scope& operator=(const Scope&) = delete;
};

template <typename T>
inline void alloc(T** p, size_t bytes) {
  Tracker* t = current();
  if (t && t->cap && t->cur + bytes > t->cap)
    throw Error("devmem: this rank would hold " + std::to_string(t->cur + bytes) + " bytes, above its HBM cap of " +
                std::to_string(t->cap) + " bytes (DistTuning::hbm_cap_bytes)");
  void* q = nullptr;
  const hipError_t e = hipMalloc(&q, bytes);
  if (e != hipSuccess)
    throw Error(std::string("devmem: hipMalloc(") + std::to_string(bytes) + ") failed: " + hipGetErrorString(e));
  *p = static_cast<T*>(q);
  if (t) {
    t->cur += bytes;
    if (t->cur > t->peak) t->peak = t->cur;
    size_t fr = 0, tot = 0;
    if (hipMemGetInfo(&fr, &tot) == hipSuccess && fr < t->free_low) t->free_low = fr;
  }
}

inline void release(void* p, size_t bytes) {
  if (!p) return;
  const hipError_t e = hipFree(p);
  if (e != hipSuccess) throw Error(std::string("devmem: hipFree failed: ") + hipGetErrorString(e));
  if (Tracker* t = current()) t->cur = t->cur > bytes ? t->cur - bytes : 0;
}

}  // namespace devmem
}  // namespace bibfs
