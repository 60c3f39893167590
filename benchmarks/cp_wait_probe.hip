// Probe: can a stream wait on a memory value (hipStreamWaitValue64, executed by the command
// processor, no CU spinning) and write one (hipStreamWriteValue64) inside a captured hipGraph?
// If so, the device p2p transport's wait kernels (parallel/devp2p.py) could become CP waits.
// Prints what capture / instantiation / replay returned and whether two replays waited.
// Measured on MI355X / ROCm 7.2: both replays wait, yet the graph holds ONE node (the memory
// operations ride on the kernel node), and a whole device-transport step built from them
// (a set / wait-equal / reset handshake per edge) produced wrong numbers in the loopback
// harness: mid-graph ordering of captured stream memory operations is not what the transport needs.
//
//   hipcc -O2 -std=c++17 --offload-arch=gfx950 benchmarks/cp_wait_probe.hip -o gpubin/cp_wait_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <thread>

__global__ void mark(int* out, int v) {
  if (threadIdx.x == 0) out[0] = v;
}

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    printf("%-70s -> %s\n", #x, hipGetErrorString(e_));                         \
    if (e_ != hipSuccess) ok = false;                                           \
  } while (0)

int main() {
  bool ok = true;
  uint64_t* flag = nullptr;  // host-pinned, device-visible: the host plays the remote producer
  uint64_t* wflag = nullptr;
  int* out = nullptr;
  CK(hipHostMalloc((void**)&flag, 8, hipHostMallocCoherent));
  CK(hipHostMalloc((void**)&wflag, 8, hipHostMallocCoherent));
  CK(hipMalloc((void**)&out, 4));
  *flag = 0;
  *wflag = 0;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipMemsetAsync(out, 0, 4, s));
  CK(hipStreamSynchronize(s));
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  CK(hipStreamWaitValue64(s, flag, 1, hipStreamWaitValueGte, ~0ull));
  hipLaunchKernelGGL(mark, dim3(1), dim3(64), 0, s, out, 7);
  CK(hipGetLastError());
  CK(hipStreamWriteValue64(s, wflag, 5, 0));
  CK(hipStreamEndCapture(s, &g));
  if (!g) {
    printf("RESULT: capture produced no graph\n");
    return 1;
  }
  size_t n = 0;
  CK(hipGraphGetNodes(g, nullptr, &n));
  printf("graph nodes: %zu\n", n);
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  if (!ge) {
    printf("RESULT: not instantiable\n");
    return 1;
  }
  CK(hipGraphLaunch(ge, s));
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  int early = -1;
  hipError_t q = hipStreamQuery(s);
  printf("after 200 ms without the flag: stream %s, wflag %llu\n", q == hipSuccess ? "DONE (did not wait)" : "busy (waiting)",
         (unsigned long long)*wflag);
  *flag = 1;  // release
  auto t0 = std::chrono::steady_clock::now();
  while (hipStreamQuery(s) != hipSuccess && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  CK(hipMemcpy(&early, out, 4, hipMemcpyDeviceToHost));
  printf("after release: out %d (want 7), wflag %llu (want 5)\n", early, (unsigned long long)*wflag);
  (void)q;
  // second replay with the flag reset: a wait that is part of the graph must block again
  *flag = 0;
  *wflag = 0;
  CK(hipMemsetAsync(out, 0, 4, s));
  CK(hipStreamSynchronize(s));
  CK(hipGraphLaunch(ge, s));
  std::this_thread::sleep_for(std::chrono::milliseconds(200));
  const hipError_t q2 = hipStreamQuery(s);
  printf("second replay, flag reset: stream %s, wflag %llu\n", q2 == hipSuccess ? "DONE (did not wait)" : "busy (waiting)",
         (unsigned long long)*wflag);
  *flag = 1;
  CK(hipStreamSynchronize(s));
  printf("RESULT: %s (%zu graph node(s) for kernel + wait + write)\n",
         q2 != hipSuccess ? "replays wait for the value" : "replays do NOT wait (the operations ran at capture only)", n);
  return 0;
}
