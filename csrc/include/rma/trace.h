// Host-side tracing ranges (ROCTX) for rocprofv3 --marker-trace.
//
// The reference profiles with Julia's sampling profiler around its time loop
// (scripts/diffusion_2D_perf_hide_prof.jl:32-63,110-121). Here the executor
// and the Python layer mark step / boundary / halo / interior ranges; the
// ROCTX library is dlopen'ed lazily so nothing is linked when tracing is off.
#pragma once

#include <string>

namespace rma {

void trace_enable(bool on);
bool trace_enabled();
void trace_push(const char* name);
void trace_pop();
void trace_mark(const char* name);

struct TraceRange {
  explicit TraceRange(const char* name) : on_(trace_enabled()) {
    if (on_) trace_push(name);
  }
  ~TraceRange() {
    if (on_) trace_pop();
  }
  bool on_;
};

}  // namespace rma
