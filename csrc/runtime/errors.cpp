#include <atomic>
#include <sstream>

#include "rma/common.h"

namespace rma {

namespace {
std::atomic<int> g_rank{-1};
}

int current_rank_for_errors() { return g_rank.load(); }
void set_rank_for_errors(int rank) { g_rank.store(rank); }

void throw_error(const char* what, const char* file, int line, const std::string& detail) {
  std::ostringstream oss;
  const int r = g_rank.load();
  oss << "[rocm_mpi_amd";
  if (r >= 0) oss << " rank " << r;
  oss << "] " << what << " (" << file << ":" << line << ")";
  if (!detail.empty()) oss << ": " << detail;
  throw Error(oss.str());
}

}  // namespace rma
