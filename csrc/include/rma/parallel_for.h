// Minimal host thread pool-free parallel loop for the CPU twins (no OpenMP:
// the process already hosts torch's OpenMP runtime and we do not want a second
// one next to it).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

namespace rma {

// Worker count: hardware threads, capped at 16 and at OMP_NUM_THREADS /
// RMA_NUM_THREADS when set (several ranks share one host in the CPU tests).
inline int64_t host_threads() {
  int64_t nt = std::min<int64_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  for (const char* var : {"RMA_NUM_THREADS", "OMP_NUM_THREADS"}) {
    if (const char* s = std::getenv(var)) {
      const long v = std::strtol(s, nullptr, 10);
      if (v > 0) return std::min<int64_t>(nt, v);
    }
  }
  return nt;
}

// f(i) for i in [begin, end) over up to host_threads() threads. Exceptions
// thrown by f (on a worker or on the calling thread) are caught, every
// spawned thread is joined on every path, and the first exception is
// rethrown to the caller (a joinable std::thread destroyed by unwinding would
// otherwise call std::terminate).
template <typename F>
void parallel_for(int64_t begin, int64_t end, int64_t min_chunk, F&& f) {
  const int64_t n = end - begin;
  if (n <= 0) return;
  int64_t nt = host_threads();
  nt = std::min(nt, std::max<int64_t>(1, n / std::max<int64_t>(1, min_chunk)));
  if (nt <= 1) {
    for (int64_t i = begin; i < end; ++i) f(i);
    return;
  }
  std::mutex mu;
  std::exception_ptr first;
  auto run = [&](int64_t a, int64_t b) {
    try {
      for (int64_t i = a; i < b; ++i) f(i);
    } catch (...) {
      std::lock_guard<std::mutex> lk(mu);
      if (!first) first = std::current_exception();
    }
  };
  std::vector<std::thread> th;
  th.reserve(nt);
  struct Joiner {  // joins on every exit path, unwinding included
    std::vector<std::thread>& t;
    ~Joiner() {
      for (auto& x : t)
        if (x.joinable()) x.join();
    }
  } joiner{th};
  int64_t t = 0;
  for (; t < nt; ++t) {
    const int64_t a = begin + n * t / nt, b = begin + n * (t + 1) / nt;
    try {
      th.emplace_back(run, a, b);
    } catch (const std::system_error&) {
      break;  // out of threads (loaded host): the caller runs the rest itself
    }
  }
  for (; t < nt; ++t) run(begin + n * t / nt, begin + n * (t + 1) / nt);
  for (auto& x : th) x.join();
  if (first) std::rethrow_exception(first);
}

}  // namespace rma
