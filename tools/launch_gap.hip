// Back-to-back launch cost of a tiny kernel on one stream, with 0, 1 or 2
// hipEventRecord calls (timing disabled) after each launch, eager and in a
// captured graph: what the eager path of a device-engine run() pays per call
// beyond its kernel (small-message latency).
//
//   hipcc --offload-arch=gfx950 -O2 tools/launch_gap.hip -o tools/launch_gap
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                             \
    }                                                                           \
  } while (0)

__global__ void tiny(float* x, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] += 1.0f;
}

int main() {
  const int iters = 2000, n = 256;
  float* x;
  CK(hipMalloc(&x, n * sizeof(float)));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t ev[2];
  for (auto& e : ev) CK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  auto issue = [&](int events) {
    hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, x, n);
    for (int k = 0; k < events; k++) CK(hipEventRecord(ev[k], s));
  };
  for (int events = 0; events <= 2; events++) {
    for (int i = 0; i < 50; i++) issue(events);
    CK(hipStreamSynchronize(s));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < iters; i++) issue(events);
    auto t1 = std::chrono::steady_clock::now();
    CK(hipStreamSynchronize(s));
    auto t2 = std::chrono::steady_clock::now();
    const double us = std::chrono::duration<double, std::micro>(t2 - t0).count() / iters;
    const double is = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
    std::printf("{\"mode\": \"eager\", \"events_per_launch\": %d, \"us_per_launch\": %.2f, "
                "\"issue_us\": %.2f}\n", events, us, is);
  }
  hipGraph_t g;
  hipGraphExec_t ge;
  const int per = 20;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < per; i++) hipLaunchKernelGGL(tiny, dim3(1), dim3(256), 0, s, x, n);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int i = 0; i < 5; i++) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters / per; i++) CK(hipGraphLaunch(ge, s));
  CK(hipStreamSynchronize(s));
  auto t1 = std::chrono::steady_clock::now();
  std::printf("{\"mode\": \"graph\", \"per_graph\": %d, \"us_per_launch\": %.2f}\n", per,
              std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  for (auto& e : ev) CK(hipEventDestroy(e));
  CK(hipStreamDestroy(s));
  CK(hipFree(x));
  return 0;
}
