// RCCL point-to-point inside hipGraph stream capture, without torch: the
// system RCCL and HIP runtime of /opt/rocm only, one rank, send/recv to self.
// Every stage prints before it runs, and a SIGSEGV handler prints a host
// backtrace, so a crash says where it happened (bench/rccl_graph_probe.py
// found RCCL P2P under capture segfaulting inside the framework's process).
//
//   build/bench/rccl_capture_probe [bytes] [mode]
//     mode 0: group(send, recv) to self; 1: two groups (send, then recv)
#include <execinfo.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__,  \
              __LINE__);                                                          \
      exit(2);                                                                    \
    }                                                                             \
  } while (0)
#define NK(x)                                                                     \
  do {                                                                            \
    ncclResult_t r = (x);                                                         \
    if (r != ncclSuccess) {                                                       \
      fprintf(stderr, "RCCL error %s at %s:%d\n", ncclGetErrorString(r), __FILE__, \
              __LINE__);                                                          \
      exit(3);                                                                    \
    }                                                                             \
  } while (0)

static void on_segv(int sig) {
  void* bt[64];
  const int n = backtrace(bt, 64);
  fprintf(stderr, "signal %d, host backtrace:\n", sig);
  backtrace_symbols_fd(bt, n, 2);
  _exit(128 + sig);
}

static void stage(const char* s) {
  printf("stage: %s\n", s);
  fflush(stdout);
}

int main(int argc, char** argv) {
  signal(SIGSEGV, on_segv);
  signal(SIGABRT, on_segv);
  const size_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1 << 20);
  const int mode = argc > 2 ? atoi(argv[2]) : 0;
  int v = 0;
  ncclGetVersion(&v);
  printf("rccl %d bytes %zu mode %d\n", v, bytes, mode);
  CK(hipSetDevice(0));
  ncclUniqueId id;
  NK(ncclGetUniqueId(&id));
  ncclComm_t comm;
  stage("ncclCommInitRank");
  NK(ncclCommInitRank(&comm, 1, id, 0));
  char *sb, *rb;
  CK(hipMalloc(&sb, bytes));
  CK(hipMalloc(&rb, bytes));
  CK(hipMemset(sb, 7, bytes));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto enqueue = [&] {
    if (mode == 0) {
      NK(ncclGroupStart());
      NK(ncclSend(sb, bytes, ncclUint8, 0, comm, s));
      NK(ncclRecv(rb, bytes, ncclUint8, 0, comm, s));
      NK(ncclGroupEnd());
    } else {
      NK(ncclGroupStart());
      NK(ncclSend(sb, bytes, ncclUint8, 0, comm, s));
      NK(ncclRecv(rb, bytes, ncclUint8, 0, comm, s));
      NK(ncclGroupEnd());
      NK(ncclGroupStart());
      NK(ncclSend(rb, bytes, ncclUint8, 0, comm, s));
      NK(ncclRecv(sb, bytes, ncclUint8, 0, comm, s));
      NK(ncclGroupEnd());
    }
  };
  auto verify = [&](const char* what) {
    std::vector<char> h(bytes);
    CK(hipMemcpy(h.data(), rb, bytes, hipMemcpyDeviceToHost));
    size_t bad = 0;
    for (char c : h) bad += c != 7;
    printf("%s: %zu bad bytes\n", what, bad);
    fflush(stdout);
    return bad == 0;
  };
  stage("eager group");
  enqueue();
  CK(hipStreamSynchronize(s));
  if (!verify("eager")) return 4;
  CK(hipMemset(rb, 0, bytes));
  stage("begin capture");
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  stage("group under capture");
  enqueue();
  hipGraph_t g;
  stage("end capture");
  CK(hipStreamEndCapture(s, &g));
  size_t nn = 0;
  CK(hipGraphGetNodes(g, nullptr, &nn));
  printf("graph nodes: %zu\n", nn);
  hipGraphExec_t ge;
  stage("instantiate");
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  stage("launch x10");
  for (int i = 0; i < 10; ++i) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  if (!verify("graph")) return 5;
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  NK(ncclCommDestroy(comm));
  printf("OK\n");
  return 0;
}
