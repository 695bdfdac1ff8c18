// Threaded host self test of the device loopback transport and the halo
// engine (csrc/runtime/loopback.cpp, csrc/runtime/halo.cpp) against the host
// HIP stand-in of tests/native/hip_stub/hip/hip_runtime.h, built once with
// ThreadSanitizer and once with AddressSanitizer + UBSan
// (tests/test_native_host_threads.py).
//
// This is the code where logical-rank threads meet: mailboxes, "ready" /
// "consumed" events shared across threads, pack buffers a peer copies out
// of, and endpoints torn down while peers are still finishing their last
// group. Cases:
//   1. teardown_while_peer_waits: rank A finishes and destroys its endpoint
//      while rank B is still blocked on a third rank before it waits on the
//      "consumed" event A recorded. Deterministic; the round-4 GPU-suite
//      SIGSEGV (the event died with A's endpoint) fails it under both builds.
//   2. halo_stress: P rank threads run the real HaloExchanger over
//      LoopbackEndpoints (per-dimension, cross and merged groups; open and
//      periodic grids incl. two messages per pair), with growing tiles so
//      the plan cache misses and pack buffers are reallocated, alternating
//      fields so it also hits; every tile is checked against the global
//      field after every exchange. Ranks then tear down in a random order.
//   3. random_groups: P threads, random message patterns (several messages
//      per pair, sizes, nesting), random teardown delays.
//   4. ipc_ring: the HIP IPC transport (csrc/runtime/ipc.cpp) between P rank
//      threads standing in for processes (shared-memory flag blocks, handle
//      export / connect, shm unlink), in host and stream mode: ring groups of
//      two messages per pair with random sizes, a mailbox overflow of a LATER
//      peer that must leave the transport in step, and a stream-mode wait
//      that times out and must surface through check_error().
#include <array>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <future>
#include <memory>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>  // the host stub (tests/native/hip_stub)

#include <condition_variable>
#include <map>
#include <mutex>
#include <unistd.h>

#include "rma/halo.h"
#include "rma/ipc.h"
#include "rma/kernels.h"
#include "rma/loopback.h"
#include "rma/topology.h"

namespace rma {
// the stub "stream" runs everything at enqueue time: the pack / unpack
// kernels become their CPU twins
void copy2d_batch_gpu(const Copy2d* copies, int n, int elem_bytes, stream_t) {
  copy2d_batch_cpu(copies, n, elem_bytes);
}
// ... and the IPC flag kernels (csrc/kernels/flags.hip) a bounded host spin
void flag_wait_gpu(const uint64_t* flag, uint64_t want, double timeout_s, uint32_t* err,
                   uint32_t code, stream_t) {
  auto* f = reinterpret_cast<const std::atomic<uint64_t>*>(flag);
  const auto t0 = std::chrono::steady_clock::now();
  while (f->load(std::memory_order_acquire) != want) {
    if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s) {
      __atomic_store_n(err, code, __ATOMIC_RELEASE);
      return;
    }
    std::this_thread::yield();
  }
}
void flag_write_gpu(uint64_t* flag, uint64_t value, stream_t) {
  reinterpret_cast<std::atomic<uint64_t>*>(flag)->store(value, std::memory_order_release);
}
}  // namespace rma

namespace {
using namespace rma;

std::atomic<int> g_fail{0};
std::atomic<long long> g_hits{0}, g_misses{0};  // halo plan cache, all stress cases

#define CHECK(c, ...)                                                        \
  do {                                                                       \
    if (!(c)) {                                                              \
      std::fprintf(stderr, "FAILED %s at line %d: ", #c, __LINE__);          \
      std::fprintf(stderr, __VA_ARGS__);                                     \
      std::fprintf(stderr, "\n");                                            \
      ++g_fail;                                                              \
    }                                                                        \
  } while (0)

template <typename F>
std::thread guarded(F f, const char* what, int rank) {
  return std::thread([f, what, rank]() mutable {
    try {
      f();
    } catch (const std::exception& e) {
      std::fprintf(stderr, "FAILED %s rank %d: %s\n", what, rank, e.what());
      ++g_fail;
    }
  });
}

void sleep_us(int us) { std::this_thread::sleep_for(std::chrono::microseconds(us)); }

// ---------------------------------------------------------------------------
int teardown_while_peer_waits() {
  auto hub = std::make_shared<LoopbackHub>(3, 30.0);
  double src[4] = {1, 2, 3, 4}, ra[4] = {}, rc[4] = {};
  std::promise<void> a_gone;
  std::shared_future<void> a_gone_f = a_gone.get_future().share();
  std::vector<std::thread> th;
  th.push_back(guarded(
      [&] {  // B: sends to C first (blocks there), then to A
        LoopbackEndpoint B(hub, 0);
        B.group_start();
        B.send(src, sizeof src, 2, nullptr);
        B.send(src, sizeof src, 1, nullptr);
        B.group_end();
      },
      "teardown B", 0));
  th.push_back(guarded(
      [&] {  // A: receives, returns, and is destroyed before B looks at A's event
        {
          LoopbackEndpoint A(hub, 1);
          A.group_start();
          A.recv(ra, sizeof ra, 0, nullptr);
          A.group_end();
        }
        a_gone.set_value();
      },
      "teardown A", 1));
  th.push_back(guarded(
      [&] {  // C: takes B's message only after A is gone
        a_gone_f.wait();
        LoopbackEndpoint C(hub, 2);
        C.group_start();
        C.recv(rc, sizeof rc, 0, nullptr);
        C.group_end();
      },
      "teardown C", 2));
  for (auto& t : th) t.join();
  CHECK(std::memcmp(ra, src, sizeof src) == 0, "A received wrong data");
  CHECK(std::memcmp(rc, src, sizeof src) == 0, "C received wrong data");
  return g_fail.load();
}

// ---------------------------------------------------------------------------
struct StressCase {
  std::array<int, 3> dims, periods;
  int iters;
  unsigned seed;
};

int halo_stress(const StressCase& sc) {
  const int P = sc.dims[0] * sc.dims[1] * sc.dims[2];
  CartTopology topo(P, sc.dims, sc.periods);
  auto hub = std::make_shared<LoopbackHub>(P, 30.0);
  std::atomic<long> checked{0};
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r) {
    th.push_back(guarded(
        [&, r] {
          std::mt19937 rng(sc.seed * 977u + (unsigned)r);
          auto ep = std::make_unique<LoopbackEndpoint>(hub, r);
          auto hx = std::make_unique<HaloExchanger>(ep.get(), r, topo.neighbors(r));
          hx->set_diagonals(topo.diagonals(r));
          const auto nb = topo.neighbors(r);
          const auto c = topo.coords(r);
          std::array<std::vector<double>, 2> buf;
          for (int it = 0; it < sc.iters; ++it) {
            // all ranks derive the same sizes / widths / mode from (seed, it)
            const int phase = it / 4;
            const int hw = 1 + (int)((sc.seed + (unsigned)phase) % 3);
            const int ol = 2 * hw;
            const int64_t n[2] = {ol + hw + 3 + 3 * phase, ol + hw + 2 + 2 * phase};
            const int mode = (int)((sc.seed + 7u * (unsigned)it) % 3);  // 0 dims, 1 cross, 2 merged
            std::vector<double>& a = buf[it % 2];
            if (it % 4 < 2) a.assign((size_t)(n[0] * n[1]), 0.0);  // new tiles: plan miss
            int64_t ng[2];
            for (int d = 0; d < 2; ++d)
              ng[d] = sc.periods[d] ? (int64_t)sc.dims[d] * (n[d] - ol)
                                    : (int64_t)sc.dims[d] * (n[d] - ol) + ol;
            auto gidx = [&](int d, int64_t i) {
              int64_t g = (int64_t)c[d] * (n[d] - ol) + i;
              if (sc.periods[d]) g = ((g % ng[d]) + ng[d]) % ng[d];
              return g;
            };
            auto gval = [&](int64_t x, int64_t y) {
              return (double)gidx(0, x) + 1000.0 * (double)(gidx(1, y) + 1) + 1e7 * it;
            };
            auto in_halo = [&](int d, int64_t i) {
              return (nb[d][0] >= 0 && i < hw) || (nb[d][1] >= 0 && i >= n[d] - hw);
            };
            for (int64_t y = 0; y < n[1]; ++y)
              for (int64_t x = 0; x < n[0]; ++x)
                a[(size_t)(y * n[0] + x)] = (in_halo(0, x) || in_halo(1, y)) ? -1.0 : gval(x, y);
            HaloField f;
            f.ptr = a.data();
            f.size = {n[0], n[1], 1};
            f.ol = {ol, ol, 2};
            f.hw = {hw, hw, 1};
            if (rng() % 4 == 0) sleep_us((int)(rng() % 200));  // shuffle thread timing
            if (mode == 0)
              hx->exchange({f}, nullptr, 7);
            else if (mode == 1)
              hx->exchange_cross({f}, nullptr, 7);
            else
              hx->exchange_merged({f}, nullptr);
            for (int64_t y = 0; y < n[1]; ++y)
              for (int64_t x = 0; x < n[0]; ++x) {
                if (mode == 1 && in_halo(0, x) && in_halo(1, y)) continue;  // cross: corners stale
                const double v = a[(size_t)(y * n[0] + x)];
                if (v != gval(x, y)) {
                  CHECK(false, "dims %dx%d periods %d%d rank %d it %d mode %d cell (%lld,%lld): %g != %g",
                        sc.dims[0], sc.dims[1], sc.periods[0], sc.periods[1], r, it, mode,
                        (long long)x, (long long)y, v, gval(x, y));
                  return;
                }
              }
            ++checked;
          }
          g_hits += hx->plan_hits();
          g_misses += hx->plan_misses();
          // random teardown order: an endpoint / exchanger may go while peers
          // are still inside their last group
          sleep_us((int)(rng() % 300));
          if (rng() % 2) {
            hx.reset();
            ep.reset();
          } else {
            ep.reset();  // the exchanger no longer talks to it
            hx.reset();
          }
        },
        "halo_stress", r));
  }
  for (auto& t : th) t.join();
  CHECK(checked.load() == (long)P * sc.iters, "checked %ld of %ld", checked.load(),
        (long)P * sc.iters);
  return g_fail.load();
}

// ---------------------------------------------------------------------------
int random_groups(int P, int rounds, unsigned seed) {
  auto hub = std::make_shared<LoopbackHub>(P, 30.0);
  // the message pattern of every round is known to all ranks (same seed)
  struct M {
    int src, dst, elems;
  };
  std::vector<std::vector<M>> pattern(rounds);
  std::mt19937 g(seed);
  for (int k = 0; k < rounds; ++k) {
    const int nm = 1 + (int)(g() % (unsigned)(2 * P));
    for (int i = 0; i < nm; ++i) {
      M m{(int)(g() % (unsigned)P), (int)(g() % (unsigned)P), 1 + (int)(g() % 64)};
      pattern[k].push_back(m);
    }
  }
  auto val = [](int k, int i, int e) { return 1e6 * k + 1e3 * i + e; };
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r) {
    th.push_back(guarded(
        [&, r] {
          std::mt19937 rng(seed + 31u * (unsigned)r);
          LoopbackEndpoint ep(hub, r);
          for (int k = 0; k < rounds; ++k) {
            const auto& pat = pattern[(size_t)k];
            std::vector<std::vector<double>> sb(pat.size()), rb(pat.size());
            const bool nested = (k % 3) == 1;
            ep.group_start();
            if (nested) ep.group_start();
            for (size_t i = 0; i < pat.size(); ++i) {
              const M& m = pat[i];
              if (m.src == r) {
                sb[i].resize((size_t)m.elems);
                for (int e = 0; e < m.elems; ++e) sb[i][(size_t)e] = val(k, (int)i, e);
                ep.send(sb[i].data(), sb[i].size() * 8, m.dst, nullptr);
              }
            }
            for (size_t i = 0; i < pat.size(); ++i) {
              const M& m = pat[i];
              if (m.dst == r) {
                rb[i].assign((size_t)m.elems, -1.0);
                ep.recv(rb[i].data(), rb[i].size() * 8, m.src, nullptr);
              }
            }
            if (nested) ep.group_end();
            ep.group_end();
            for (size_t i = 0; i < pat.size(); ++i)
              if (pat[i].dst == r)
                for (int e = 0; e < pat[i].elems; ++e)
                  if (rb[i][(size_t)e] != val(k, (int)i, e)) {
                    CHECK(false, "round %d msg %zu elem %d on rank %d", k, i, e, r);
                    return;
                  }
            if (rng() % 8 == 0) sleep_us((int)(rng() % 100));
          }
          sleep_us((int)(rng() % 300));
        },
        "random_groups", r));
  }
  for (auto& t : th) t.join();
  return g_fail.load();
}

// ---------------------------------------------------------------------------
class Barrier {  // C++17: no std::barrier
 public:
  explicit Barrier(int n) : n_(n) {}
  void wait() {
    std::unique_lock<std::mutex> lk(mu_);
    const int gen = gen_;
    if (++count_ == n_) {
      count_ = 0;
      ++gen_;
      cv_.notify_all();
      return;
    }
    cv_.wait(lk, [&] { return gen_ != gen; });
  }

 private:
  std::mutex mu_;
  std::condition_variable cv_;
  int n_, count_ = 0, gen_ = 0;
};

int ipc_ring(int P, int mode, int groups, unsigned seed) {
  const size_t cap = 4096;  // bytes of one mailbox slot
  const std::string token = "tsel" + std::to_string(getpid()) + "m" + std::to_string(mode) + "p" +
                            std::to_string(P);
  Barrier bar(P);
  std::mutex mu;
  std::map<std::pair<int, int>, std::string> blobs;
  std::vector<std::thread> th;
  for (int r = 0; r < P; ++r) {
    th.push_back(guarded(
        [&, r] {
          const int nxt = (r + 1) % P, prv = (r + P - 1) % P;
          IpcTransport t(r, P, 0, {nxt, prv}, cap, token, 30.0, mode);
          {
            std::lock_guard<std::mutex> lk(mu);
            for (int p : {nxt, prv})
              if (p != r) blobs[{r, p}] = t.export_for(p);
          }
          bar.wait();
          for (int p : {nxt, prv}) {
            if (p == r) continue;
            std::string b;
            {
              std::lock_guard<std::mutex> lk(mu);
              b = blobs.at({p, r});
            }
            t.connect(p, b);
          }
          bar.wait();
          t.unlink_shm();
          std::mt19937 g(seed);  // every rank draws the same sizes
          for (int k = 0; k < groups; ++k) {
            const size_t n0 = 1 + g() % 200, n1 = 1 + g() % 200;  // doubles (2 msgs <= cap)
            const bool overflow = k == groups / 2;
            std::vector<double> s0(n0), s1(n1), r0(n0, -1), r1(n1, -1);
            for (size_t i = 0; i < n0; ++i) s0[i] = 1e6 * k + 1e3 * r + (double)i;
            for (size_t i = 0; i < n1; ++i) s1[i] = -(1e6 * k + 1e3 * r + (double)i);
            if (overflow) {  // 8 B to the next rank, cap + 8 B to the previous one
              std::vector<double> big(cap / 8 + 1, 0.0), rb(cap / 8 + 1);
              bool threw = false;
              try {
                t.group_start();
                t.send(s0.data(), 8, nxt, nullptr);
                t.send(big.data(), big.size() * 8, prv, nullptr);
                t.recv(r0.data(), 8, prv, nullptr);
                t.recv(rb.data(), rb.size() * 8, nxt, nullptr);
                t.group_end();
              } catch (const Error&) {
                threw = true;
              }
              CHECK(threw && !t.poisoned(), "rank %d: overflow must throw, unpoisoned", r);
              continue;
            }
            t.group_start();
            t.send(s0.data(), n0 * 8, nxt, nullptr);
            t.send(s1.data(), n1 * 8, nxt, nullptr);
            t.recv(r0.data(), n0 * 8, prv, nullptr);
            t.recv(r1.data(), n1 * 8, prv, nullptr);
            t.group_end();
            for (size_t i = 0; i < n0; ++i)
              if (r0[i] != 1e6 * k + 1e3 * prv + (double)i) {
                CHECK(false, "ipc mode %d rank %d group %d msg 0 elem %zu", mode, r, k, i);
                return;
              }
            for (size_t i = 0; i < n1; ++i)
              if (r1[i] != -(1e6 * k + 1e3 * prv + (double)i)) {
                CHECK(false, "ipc mode %d rank %d group %d msg 1 elem %zu", mode, r, k, i);
                return;
              }
          }
          CHECK(mode == 1 ? t.host_waits() == 0 : t.host_waits() > 0, "rank %d host waits %llu", r,
                (unsigned long long)t.host_waits());
          bar.wait();  // nobody unmaps while a peer still copies out of its mailbox
        },
        "ipc_ring", r));
  }
  for (auto& x : th) x.join();
  return g_fail.load();
}

// stream mode: a receive whose sender never sends times out (bounded) and
// surfaces at the next group / check_error
int ipc_stream_timeout() {
  const std::string token = "tselto" + std::to_string(getpid());
  Barrier bar(2);
  std::mutex mu;
  std::map<std::pair<int, int>, std::string> blobs;
  std::vector<std::thread> th;
  for (int r = 0; r < 2; ++r) {
    th.push_back(guarded(
        [&, r] {
          const int p = 1 - r;
          IpcTransport t(r, 2, 0, {p}, 64, token, 0.05, 1);
          {
            std::lock_guard<std::mutex> lk(mu);
            blobs[{r, p}] = t.export_for(p);
          }
          bar.wait();
          std::string b;
          {
            std::lock_guard<std::mutex> lk(mu);
            b = blobs.at({p, r});
          }
          t.connect(p, b);
          bar.wait();
          if (r == 1) {
            double x = -1;
            t.recv(&x, 8, 0, nullptr);  // rank 0 never sends: the wait gives up
            bool threw = false;
            try {
              t.check_error();
            } catch (const Error& e) {
              threw = std::string(e.what()).find("timed out") != std::string::npos;
            }
            CHECK(threw && t.poisoned(), "stream wait timeout not reported");
          }
          bar.wait();
        },
        "ipc_stream_timeout", r));
  }
  for (auto& x : th) x.join();
  return g_fail.load();
}

}  // namespace

int main() {
  if (teardown_while_peer_waits()) return 1;
  std::printf("teardown_while_peer_waits OK (stub waits %ld)\n", rma_stub::waits().load());
  const StressCase cases[] = {
      {{2, 1, 1}, {0, 0, 0}, 12, 1u}, {{2, 1, 1}, {1, 0, 0}, 12, 2u},
      {{1, 2, 1}, {1, 1, 0}, 12, 3u}, {{2, 2, 1}, {0, 0, 0}, 12, 4u},
      {{2, 2, 1}, {1, 1, 0}, 16, 5u}, {{3, 2, 1}, {1, 0, 0}, 12, 6u},
      {{4, 2, 1}, {0, 1, 0}, 12, 7u}, {{1, 1, 1}, {1, 1, 0}, 8, 8u},
  };
  for (const StressCase& sc : cases) {
    if (halo_stress(sc)) return 1;
    std::printf("halo_stress dims %dx%d periods %d%d OK\n", sc.dims[0], sc.dims[1], sc.periods[0],
                sc.periods[1]);
  }
  if (g_hits.load() == 0 || g_misses.load() == 0) {
    std::fprintf(stderr, "FAILED plan cache: %lld hits, %lld misses\n", g_hits.load(), g_misses.load());
    return 1;
  }
  std::printf("halo plan cache: %lld hits, %lld misses\n", g_hits.load(), g_misses.load());
  for (int P : {2, 3, 5, 8})
    if (random_groups(P, 60, 100u + (unsigned)P)) return 1;
  std::printf("random_groups OK\n");
  for (int mode : {0, 1})
    for (int P : {2, 3, 5})
      if (ipc_ring(P, mode, 40, 7u + (unsigned)P)) return 1;
  std::printf("ipc_ring OK (host and stream mode, 2/3/5 ranks)\n");
  if (ipc_stream_timeout()) return 1;
  std::printf("ipc_stream_timeout OK\n");
  if (rma_stub::live_events() != 0 || rma_stub::live_allocs() != 0) {
    std::fprintf(stderr, "FAILED leak: %ld events, %ld allocations alive\n",
                 rma_stub::live_events().load(), rma_stub::live_allocs().load());
    return 1;
  }
  std::printf("threaded selftest OK\n");
  return 0;
}
