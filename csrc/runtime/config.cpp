// RMA_DIAG parsing and validated tuning knobs (rma/config.h).
#include "rma/config.h"

#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <sstream>
#include <vector>

#include "rma/common.h"

namespace rma {

const char* const kDiagKeys[] = {
    // executor / planner (C++)
    "skip_exchange",     // every halo exchange skipped (WRONG multi-rank results)
    "exec_streams",      // pool | lofirst | hifirst | plain: executor stream creation
    "exec_verbose",      // print the executor's stream priorities
    "no_prime",          // no kernel priming at executor construction
    "no_lag",            // every pass waits for the previous exchange
    "no_halo_cross",     // one-step passes: one group per dimension
    "no_halo_merged",    // x+y neighbours: one group per dimension (also Python)
    "no_halo_batch",     // one pack / unpack launch per plane
    "frame_sides",       // all: frame rects on every side once any neighbour exists
    "frame_chunk_div",   // N: aligned frame tasks of 1/N the interior's rows
    "frame_aligned",     // 0 | 1: force the frame layout
    "frame_bands",       // task | ol: force the aligned y-band height
    "no_frame_fill",     // frame bands not filled into the interior
    "pipe_fast",         // pipe | pipe5: the LDS-ring fast kernel at every depth
    "pass_costs",        // K:cost/K:cost/...: planner cost overrides
    // communication (C++)
    "rccl_data_blocking",  // blocking RCCL data path of a non-blocking communicator
    "rccl_graph",          // allow hipGraph capture over RCCL
    "no_ipc_graph",        // refuse hipGraph capture over the IPC transport
    // Python side (rocm_mpi_amd/config.py)
    "hostname",             // node name for the local-rank exchange (tests)
    "rccl_fallback",        // RCCL init failure falls back to the staged transport
    "bench_rc_dir",         // bench.py: every rank writes its exit status there
    "bench_n1_cache",       // bench.py: path of the N = 1 record
    "bench_check_raise",    // bench.py: before | after: injected halo-check failure
    "bench_check_corrupt",  // bench.py: corrupt one halo-check cell
    "bench_window_corrupt", // bench.py: corrupt one window cell
    "bench_field_corrupt",  // bench.py: nan | hot | cold: one bad timed-field cell
    "bench_rccl_log_dir",   // bench.py: RCCL log directory of the link probe
    nullptr};

namespace {

bool known(const std::string& k) {
  for (const char* const* p = kDiagKeys; *p; ++p)
    if (k == *p) return true;
  return false;
}

// (key, value) entries of RMA_DIAG, validated
std::vector<std::pair<std::string, std::string>> entries() {
  std::vector<std::pair<std::string, std::string>> out;
  const char* e = std::getenv("RMA_DIAG");
  if (!e || !*e) return out;
  std::stringstream ss(e);
  std::string item;
  while (std::getline(ss, item, ',')) {
    if (item.empty()) continue;
    const size_t eq = item.find('=');
    std::string k = item.substr(0, eq), v = eq == std::string::npos ? "1" : item.substr(eq + 1);
    if (!known(k)) {
      std::string all;
      for (const char* const* p = kDiagKeys; *p; ++p) all += std::string(all.empty() ? "" : " ") + *p;
      throw_error("RMA_DIAG: unknown key", __FILE__, __LINE__, k + " (known: " + all + ")");
    }
    out.emplace_back(std::move(k), std::move(v));
  }
  return out;
}

}  // namespace

std::string diag_string() {
  (void)entries();
  const char* e = std::getenv("RMA_DIAG");
  return e ? e : "";
}

bool diag_flag(const char* key) {
  for (const auto& kv : entries())
    if (kv.first == key) return kv.second != "0";
  return false;
}

std::string diag_value(const char* key, const std::string& dflt) {
  for (const auto& kv : entries())
    if (kv.first == key) return kv.second;
  return dflt;
}

double env_double(const char* name, double dflt, double lo, double hi) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  errno = 0;
  char* end = nullptr;
  const double v = std::strtod(e, &end);
  if (errno || end == e || *end != '\0' || !std::isfinite(v) || v < lo || v > hi) {
    std::ostringstream m;
    m << e << " (expected a number in [" << lo << ", " << hi << "])";
    throw_error((std::string(name) + ": bad value").c_str(), __FILE__, __LINE__, m.str());
  }
  return v;
}

std::string env_choice(const char* name, const char* choices, const char* dflt) {
  const char* e = std::getenv(name);
  if (!e || !*e) return dflt;
  std::stringstream ss(choices);
  std::string c;
  while (std::getline(ss, c, '|'))
    if (c == e) return c;
  throw_error((std::string(name) + ": bad value").c_str(), __FILE__, __LINE__,
              std::string(e) + " (one of " + choices + ")");
}

}  // namespace rma
