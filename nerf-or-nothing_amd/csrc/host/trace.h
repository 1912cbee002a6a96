// roctx phase ranges (SURVEY.md §5 "Tracing": the reference has no tracing at all, MNcpp:97-133
// prints after a device sync).  Host-side ranges around each enqueued phase of a training step; a
// profiler that collects them (`rocprofv3 --marker-trace`) lines them up with the kernel trace.
// Without a tool attached each push/pop is a call into librocprofiler-sdk-roctx that returns at once.
#pragma once
#include <rocprofiler-sdk-roctx/roctx.h>

namespace AcceleratedNeRFUtils {

struct TraceRange {
  explicit TraceRange(const char* msg) { roctxRangePushA(msg); }
  ~TraceRange() { roctxRangePop(); }
  TraceRange(const TraceRange&) = delete;
  TraceRange& operator=(const TraceRange&) = delete;
};

// one name per KernelTimer id (accelerated.h TimerId, nof.h NOF_NUM_TIMERS)
inline const char* timer_range_name(int id) {
  static const char* const kNames[] = {"nof:pack_weights", "nof:sample",     "nof:mlp_fwd",
                                       "nof:render_fwd",   "nof:render_bwd", "nof:mlp_bwd",
                                       "nof:wgrad",        "nof:wgrad_reduce"};
  return id >= 0 && id < (int)(sizeof(kNames) / sizeof(kNames[0])) ? kNames[id] : "nof:?";
}

}  // namespace AcceleratedNeRFUtils
