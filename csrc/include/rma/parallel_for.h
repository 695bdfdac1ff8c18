// Minimal host thread pool-free parallel loop for the CPU twins (no OpenMP:
// the process already hosts torch's OpenMP runtime and we do not want a second
// one next to it).
#pragma once

#include <algorithm>
#include <cstdint>
#include <thread>
#include <vector>

namespace rma {

template <typename F>
void parallel_for(int64_t begin, int64_t end, int64_t min_chunk, F&& f) {
  const int64_t n = end - begin;
  if (n <= 0) return;
  int64_t nt = std::max<int64_t>(1, std::min<int64_t>(std::thread::hardware_concurrency(), 16));
  nt = std::min(nt, std::max<int64_t>(1, n / std::max<int64_t>(1, min_chunk)));
  if (nt <= 1) {
    for (int64_t i = begin; i < end; ++i) f(i);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt);
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t a = begin + n * t / nt, b = begin + n * (t + 1) / nt;
    th.emplace_back([a, b, &f] {
      for (int64_t i = a; i < b; ++i) f(i);
    });
  }
  for (auto& x : th) x.join();
}

}  // namespace rma
