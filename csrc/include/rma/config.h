// Runtime configuration from the environment.
//
// Two kinds of variables (docs/TUNING.md):
//  * tuning knobs, each its own documented variable (RMA_TRANSPORT,
//    RMA_EXEC_FUSED, RMA_EXEC_FUSED_TIMEOUT, RMA_RCCL_LIB, ...), read where they
//    apply and validated (a malformed value is an error, not a silent default);
//  * diagnostics and A/B switches, all in ONE variable:
//        RMA_DIAG="key[=value],key[=value],..."
//    e.g. RMA_DIAG=no_lag,exec_streams=hifirst,pass_costs=20:1.9/24:2.2.
//    Keys are checked against kDiagKeys (C++ and Python keys: the Python side,
//    rocm_mpi_amd/config.py, reads the same variable); an unknown key is an
//    error. Values may not contain ',' (pass_costs uses '/' between entries).
//
// The reference's whole configuration surface is 8 constants per script
// (scripts/diffusion_2D_perf.jl:15-25) plus IGG_ROCMAWARE_MPI
// (scripts/setenv.sh:13); this keeps the production surface that small.
#pragma once

#include <string>

namespace rma {

// every RMA_DIAG key, C++ and Python (rocm_mpi_amd/config.py DIAG_KEYS mirrors it)
extern const char* const kDiagKeys[];

// "key" or "key=<anything but 0>" present in RMA_DIAG (re-read on every call)
bool diag_flag(const char* key);
// value of "key=value" in RMA_DIAG, or dflt when absent ("key" alone: "1")
std::string diag_value(const char* key, const std::string& dflt = "");
// the RMA_DIAG string (empty when unset), after validating every key
std::string diag_string();

// a tuning knob: the variable's value as a double in [lo, hi], dflt when unset;
// anything else (not a number, out of range) is an error naming the variable
double env_double(const char* name, double dflt, double lo, double hi);
// a tuning knob with a fixed set of values ("a|b|c"); dflt when unset
std::string env_choice(const char* name, const char* choices, const char* dflt);

}  // namespace rma
