// hip_api_cost.cc -- host cost of the HIP calls one executor hop makes, and
// the completion latency the host progress loop sees (1-GPU box).
//   hipcc --offload-arch=gfx950 -O2 tools/hip_api_cost.cc -o /tmp/hip_api_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));            \
      return 1;                                                            \
    }                                                                      \
  } while (0)

__global__ void empty_kernel() {}

__global__ void add_kernel(float* d, const float* a, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) d[i] += a[i];
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) {
  return std::chrono::duration<double, std::micro>(b - a).count();
}

int main() {
  const int N = 2000;
  float *a, *b;
  CK(hipMalloc(&a, 1 << 20));
  CK(hipMalloc(&b, 1 << 20));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev[N];
  for (int i = 0; i < N; i++) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  // warm
  for (int i = 0; i < 100; i++) {
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s1);
    CK(hipMemcpyAsync(b, a, 4096, hipMemcpyDeviceToDevice, s2));
  }
  CK(hipDeviceSynchronize());

  auto t0 = clk::now();
  for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s1);
  auto t1 = clk::now();
  CK(hipDeviceSynchronize());
  std::printf("kernel launch (empty)          %7.2f us/call\n", us(t0, t1) / N);

  t0 = clk::now();
  for (int i = 0; i < N; i++) hipLaunchKernelGGL(add_kernel, dim3(4), dim3(256), 0, s1, a, b, 1024);
  t1 = clk::now();
  CK(hipDeviceSynchronize());
  std::printf("kernel launch (add 1024)       %7.2f us/call\n", us(t0, t1) / N);

  t0 = clk::now();
  for (int i = 0; i < N; i++) CK(hipMemcpyAsync(b, a, 4096, hipMemcpyDeviceToDevice, s2));
  t1 = clk::now();
  CK(hipDeviceSynchronize());
  std::printf("hipMemcpyAsync D2D 4 KiB       %7.2f us/call\n", us(t0, t1) / N);

  t0 = clk::now();
  for (int i = 0; i < N; i++) CK(hipMemcpyPeerAsync(b, 0, a, 0, 4096, s2));
  t1 = clk::now();
  CK(hipDeviceSynchronize());
  std::printf("hipMemcpyPeerAsync 4 KiB       %7.2f us/call\n", us(t0, t1) / N);

  t0 = clk::now();
  for (int i = 0; i < N; i++) CK(hipEventRecord(ev[i], s1));
  t1 = clk::now();
  CK(hipDeviceSynchronize());
  std::printf("hipEventRecord                 %7.2f us/call\n", us(t0, t1) / N);

  t0 = clk::now();
  for (int i = 0; i < N; i++) (void)hipEventQuery(ev[i]);
  t1 = clk::now();
  std::printf("hipEventQuery (complete)       %7.2f us/call\n", us(t0, t1) / N);

  t0 = clk::now();
  for (int i = 0; i < N; i++) CK(hipStreamWaitEvent(s2, ev[i], 0));
  t1 = clk::now();
  CK(hipDeviceSynchronize());
  std::printf("hipStreamWaitEvent (complete)  %7.2f us/call\n", us(t0, t1) / N);

  // round trip: enqueue small copy + record, poll until the event completes
  double tot = 0;
  for (int i = 0; i < 200; i++) {
    auto a0 = clk::now();
    CK(hipMemcpyAsync(b, a, 4096, hipMemcpyDeviceToDevice, s2));
    CK(hipEventRecord(ev[i], s2));
    while (hipEventQuery(ev[i]) == hipErrorNotReady) {
    }
    tot += us(a0, clk::now());
  }
  std::printf("copy 4 KiB + record + poll     %7.2f us round trip\n", tot / 200);
  tot = 0;
  for (int i = 0; i < 200; i++) {
    auto a0 = clk::now();
    hipLaunchKernelGGL(add_kernel, dim3(4), dim3(256), 0, s1, a, b, 1024);
    CK(hipEventRecord(ev[i], s1));
    while (hipEventQuery(ev[i]) == hipErrorNotReady) {
    }
    tot += us(a0, clk::now());
  }
  std::printf("kernel + record + poll         %7.2f us round trip\n", tot / 200);
  // cross-stream chain: copy on s2, s1 waits, kernel on s1, poll
  tot = 0;
  for (int i = 0; i < 200; i++) {
    auto a0 = clk::now();
    CK(hipMemcpyAsync(b, a, 4096, hipMemcpyDeviceToDevice, s2));
    CK(hipEventRecord(ev[2 * i], s2));
    CK(hipStreamWaitEvent(s1, ev[2 * i], 0));
    hipLaunchKernelGGL(add_kernel, dim3(4), dim3(256), 0, s1, a, b, 1024);
    CK(hipEventRecord(ev[2 * i + 1], s1));
    while (hipEventQuery(ev[2 * i + 1]) == hipErrorNotReady) {
    }
    tot += us(a0, clk::now());
  }
  std::printf("copy->wait->kernel->poll       %7.2f us round trip\n", tot / 200);
  // hipStreamWriteValue64 into host-pinned memory: GPU-side signal latency
  uint64_t* flag = nullptr;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocCoherent));
  *flag = 0;
  uint64_t* dflag = nullptr;
  CK(hipHostGetDevicePointer((void**)&dflag, flag, 0));
  tot = 0;
  for (int i = 1; i <= 200; i++) {
    auto a0 = clk::now();
    CK(hipMemcpyAsync(b, a, 4096, hipMemcpyDeviceToDevice, s2));
    CK(hipStreamWriteValue64(s2, dflag, (uint64_t)i, 0));
    while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) < (uint64_t)i) {
    }
    tot += us(a0, clk::now());
  }
  std::printf("copy + streamWriteValue64 poll %7.2f us round trip\n", tot / 200);
  std::printf("done\n");
  return 0;
}
