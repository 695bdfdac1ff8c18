#include "rma/trace.h"

#include <dlfcn.h>

#include <atomic>
#include <mutex>

namespace rma {

namespace {
using push_fn = int (*)(const char*);
using pop_fn = int (*)();
using mark_fn = void (*)(const char*);

std::atomic<bool> g_on{false};
std::once_flag g_once;
push_fn g_push = nullptr;
pop_fn g_pop = nullptr;
mark_fn g_mark = nullptr;

void load() {
  const char* libs[] = {"librocprofiler-sdk-roctx.so.1", "librocprofiler-sdk-roctx.so",
                        "libroctx64.so.4", "libroctx64.so"};
  for (const char* l : libs) {
    void* h = dlopen(l, RTLD_NOW | RTLD_GLOBAL);
    if (!h) continue;
    g_push = reinterpret_cast<push_fn>(dlsym(h, "roctxRangePushA"));
    g_pop = reinterpret_cast<pop_fn>(dlsym(h, "roctxRangePop"));
    g_mark = reinterpret_cast<mark_fn>(dlsym(h, "roctxMarkA"));
    if (g_push && g_pop) return;
  }
  g_push = nullptr;
  g_pop = nullptr;
  g_mark = nullptr;
}
}  // namespace

void trace_enable(bool on) {
  if (on) std::call_once(g_once, load);
  g_on.store(on && g_push != nullptr);
}
bool trace_enabled() { return g_on.load(std::memory_order_relaxed); }
void trace_push(const char* name) {
  if (g_push) g_push(name);
}
void trace_pop() {
  if (g_pop) g_pop();
}
void trace_mark(const char* name) {
  if (g_mark) g_mark(name);
}

}  // namespace rma
