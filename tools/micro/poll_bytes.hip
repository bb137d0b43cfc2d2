// poll_bytes.hip -- what one flag poll of the device engines costs in HBM
// counters (attribute the plan kernel's read excess).
//
// G workgroups; lane 0 of each polls its own flag word K times with the
// product's poll (xgmi_kernels.hip get_flag: a system-scope compare-exchange
// that never matches, on uncached device memory, s_sleep(2) between polls).
// Run under rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE with K = 0 and K > 0:
// (FETCH(K) - FETCH(0)) / (G * K) = the counter's bytes per poll.
//
//   hipcc --offload-arch=gfx950 -O3 -o poll_bytes poll_bytes.hip
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d D -o fetch -- ./poll_bytes 1000 512
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kStride = 16;  // one flag per 128-byte line, as kFlagStride

__global__ void poll_kernel(const unsigned long long* flags, int K, unsigned long long* sink) {
  if (threadIdx.x == 0) {
    unsigned long long* word =
        const_cast<unsigned long long*>(flags) + (size_t)blockIdx.x * kStride + threadIdx.x;
    unsigned long long acc = 0;
    for (int k = 0; k < K; k++) {
      unsigned long long v = ~0ull;
      __hip_atomic_compare_exchange_strong(word, &v, ~0ull, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_SYSTEM);
      acc += v;
      __builtin_amdgcn_s_sleep(2);
    }
    // keeps the loop; never true (flags are 0); a per-lane (vector) address
    if (acc == 12345) sink[blockIdx.x + threadIdx.x] = acc;
  }
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 1000;
  const int G = argc > 2 ? std::atoi(argv[2]) : 512;
  const int launches = 5;
  unsigned long long* flags = nullptr;
  unsigned long long* sink = nullptr;
  const size_t bytes = (size_t)G * kStride * sizeof(unsigned long long);
  if (hipExtMallocWithFlags((void**)&flags, bytes, hipDeviceMallocUncached) != hipSuccess ||
      hipMalloc((void**)&sink, G * sizeof(unsigned long long)) != hipSuccess) {
    std::fprintf(stderr, "allocation failed\n");
    return 1;
  }
  (void)hipMemset(flags, 0, bytes);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  poll_kernel<<<G, 256>>>(flags, K, sink);  // warm-up
  (void)hipEventRecord(e0, nullptr);
  for (int i = 0; i < launches; i++) poll_kernel<<<G, 256>>>(flags, K, sink);
  (void)hipEventRecord(e1, nullptr);
  if (hipEventSynchronize(e1) != hipSuccess) {
    std::fprintf(stderr, "kernel failed\n");
    return 1;
  }
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::printf("{\"K\": %d, \"G\": %d, \"us_per_launch\": %.2f, \"ns_per_poll\": %.1f}\n", K, G,
              ms * 1e3 / launches, K > 0 ? ms * 1e6 / launches / K : 0.0);
  (void)hipFree(flags);
  (void)hipFree(sink);
  return 0;
}
