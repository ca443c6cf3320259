// roctx ranges around the engines' host-side phases (graph build, LDS search,
// grid levels, speculative / host-planned rounds, path walk), so a
// `rocprofv3 --marker-trace --kernel-trace` timeline shows which phase each
// kernel and copy belongs to.  With no profiler attached a push/pop is a few
// ns.  (SURVEY.md §5 tracing row: "rocprofv3 kernel counters + roctx ranges".)
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace bibfs {

class TraceRange {
 public:
  explicit TraceRange(const char* name) { roctxRangePush(name); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace bibfs
