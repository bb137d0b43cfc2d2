// stream_handoff.hip -- what one dependent round of a DMA-driven ring costs
// when the hand-off between the copy and the reduce is made (a) by the host
// (the host-issued steps engine: the host sees the copy's event, then
// launches the reduce), (b) on the device with cross-stream events, (c) on
// the device with small bounded wait / signal kernels on flag words (the
// device engines' flag protocol), (d) with HIP's stream memory operations
// (hipStreamWaitValue64 / hipStreamWriteValue64) on host-coherent words.
//
// One GPU, one process, two streams: a copy stream and a compute stream.
// Round i: copy  land <- acc  (hipMemcpyAsync, once the reduce of round i-1
// is done), then  acc = land + 1  (once copy i is done).  Every round depends
// on the previous one, so K rounds take K hand-off pairs; after K rounds every
// element of acc is K exactly when every round saw the previous one's result.
// Modes (b)-(d) enqueue all K rounds behind a gate kernel first, so the host's
// enqueue cost is not on the chain; the time is gate open -> both streams idle.
//
//   hipcc --offload-arch=gfx950 -O3 -o stream_handoff stream_handoff.hip
//   ./stream_handoff [K] [floats...]      (one JSON line per mode and size)
//   GPU_STREAMOPS_CP_WAIT=1 ./stream_handoff   (memops waits on the CP)
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int kStride = 16;                          // one flag per 128-byte line
constexpr uint64_t kTimeoutTicks = 500000000ull;    // 5 s of s_memrealtime (100 MHz)

__device__ __forceinline__ uint64_t get_flag(uint64_t* word) {
  uint64_t v = ~uint64_t(0);
  __hip_atomic_compare_exchange_strong(word, &v, ~uint64_t(0), __ATOMIC_RELAXED,
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  return v;
}

// lane 0 waits (bounded) until *word >= want; a timeout sets *status
__device__ __forceinline__ void wait_ge(uint64_t* word, uint64_t want, int* status) {
  if (threadIdx.x == 0) {
    const uint64_t start = __builtin_amdgcn_s_memrealtime();
    while (get_flag(word) < want) {
      if (__builtin_amdgcn_s_memrealtime() - start > kTimeoutTicks) {
        __hip_atomic_store(status, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

__global__ void wait_kernel(uint64_t* word, uint64_t want, int* status) {
  wait_ge(word, want, status);
}

__global__ void signal_kernel(uint64_t* word, uint64_t v) {
  if (threadIdx.x == 0) {
    (void)__hip_atomic_exchange(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// acc = land + 1 over a grid-stride range
__global__ void step_kernel(float* acc, const float* land, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    acc[i] = land[i] + 1.0f;
  }
}

// the same, after waiting for `deliver` >= round; the last workgroup to
// finish writes `credit` = round
__global__ void step_wait_kernel(float* acc, const float* land, size_t n, uint64_t* deliver,
                                 uint64_t* credit, unsigned* ticket, uint64_t round,
                                 int* status) {
  wait_ge(deliver, round, status);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    acc[i] = land[i] + 1.0f;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_ACQ_REL,
                                              __HIP_MEMORY_SCOPE_AGENT);
    if ((t + 1) % gridDim.x == 0) {
      (void)__hip_atomic_exchange(credit, round, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

struct Bufs {
  size_t n = 0;
  float* acc = nullptr;
  float* land = nullptr;  // uncached, as the product's landing regions
  uint64_t* dflags = nullptr;  // uncached device flags: deliver, credit
  unsigned* ticket = nullptr;
  uint64_t* hwords = nullptr;  // host-coherent: gate, deliver, credit
  int* status = nullptr;       // host-coherent
  hipStream_t copy = nullptr, comp = nullptr;
};

static int grid_for(size_t n) {
  size_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > 64 ? 64 : g));
}

static void reset(Bufs& b) {
  CK(hipMemset(b.acc, 0, b.n * sizeof(float)));
  CK(hipMemset(b.land, 0, b.n * sizeof(float)));
  CK(hipMemset(b.dflags, 0, 4 * kStride * sizeof(uint64_t)));
  CK(hipMemset(b.ticket, 0, sizeof(unsigned)));
  CK(hipDeviceSynchronize());
  for (int i = 0; i < 4 * kStride; i++) b.hwords[i] = 0;
  *b.status = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
}

static bool check(const Bufs& b, int K) {
  std::vector<float> h(b.n);
  CK(hipMemcpy(h.data(), b.acc, b.n * sizeof(float), hipMemcpyDeviceToHost));
  for (size_t i = 0; i < b.n; i++) {
    if (h[i] != (float)K) return false;
  }
  return true;
}

// releases every wait of a gated run that has not finished by the deadline
struct Watchdog {
  std::atomic<bool> done{false};
  std::thread t;
  Watchdog(Bufs& b, double seconds) {
    t = std::thread([&b, this, seconds] {
      const auto end = std::chrono::steady_clock::now() + std::chrono::duration<double>(seconds);
      while (!done.load()) {
        if (std::chrono::steady_clock::now() > end) {
          std::fprintf(stderr, "watchdog: releasing the waits\n");
          for (int i = 0; i < 4 * kStride; i++) {
            __atomic_store_n(&b.hwords[i], (uint64_t)1 << 62, __ATOMIC_SEQ_CST);
          }
          __atomic_store_n(b.status, 2, __ATOMIC_SEQ_CST);
          return;
        }
        std::this_thread::sleep_for(std::chrono::milliseconds(5));
      }
    });
  }
  ~Watchdog() {
    done.store(true);
    t.join();
  }
};

static double gated_run(Bufs& b, int K, const std::string& mode) {
  reset(b);
  uint64_t* gate = &b.hwords[0];
  uint64_t* hdeliver = &b.hwords[kStride];
  uint64_t* hcredit = &b.hwords[2 * kStride];
  uint64_t* ddeliver = &b.dflags[0];
  uint64_t* dcredit = &b.dflags[kStride];
  const int G = grid_for(b.n);
  std::vector<hipEvent_t> evc(K + 1), evr(K + 1);
  if (mode == "events") {
    for (int i = 0; i <= K; i++) {
      CK(hipEventCreateWithFlags(&evc[i], hipEventDisableTiming));
      CK(hipEventCreateWithFlags(&evr[i], hipEventDisableTiming));
    }
  }
  Watchdog wd(b, 20.0);
  wait_kernel<<<1, 64, 0, b.copy>>>(gate, 1, b.status);
  wait_kernel<<<1, 64, 0, b.comp>>>(gate, 1, b.status);
  for (int i = 1; i <= K; i++) {
    // copy stream: after the reduce of round i-1, land <- acc, then deliver i
    if (mode == "events") {
      if (i > 1) CK(hipStreamWaitEvent(b.copy, evr[i - 1], 0));
    } else if (mode == "kernels") {
      wait_kernel<<<1, 64, 0, b.copy>>>(dcredit, (uint64_t)(i - 1), b.status);
    } else {
      CK(hipStreamWaitValue64(b.copy, hcredit, (uint64_t)(i - 1), hipStreamWaitValueGte));
    }
    CK(hipMemcpyAsync(b.land, b.acc, b.n * sizeof(float), hipMemcpyDeviceToDevice, b.copy));
    if (mode == "events") {
      CK(hipEventRecord(evc[i], b.copy));
    } else if (mode == "kernels") {
      signal_kernel<<<1, 64, 0, b.copy>>>(ddeliver, (uint64_t)i);
    } else {
      CK(hipStreamWriteValue64(b.copy, hdeliver, (uint64_t)i, 0));
    }
    // compute stream: after copy i, acc = land + 1, then credit i
    if (mode == "events") {
      CK(hipStreamWaitEvent(b.comp, evc[i], 0));
      step_kernel<<<G, 256, 0, b.comp>>>(b.acc, b.land, b.n);
      CK(hipEventRecord(evr[i], b.comp));
    } else if (mode == "kernels") {
      step_wait_kernel<<<G, 256, 0, b.comp>>>(b.acc, b.land, b.n, ddeliver, dcredit, b.ticket,
                                              (uint64_t)i, b.status);
    } else {
      CK(hipStreamWaitValue64(b.comp, hdeliver, (uint64_t)i, hipStreamWaitValueGte));
      step_kernel<<<G, 256, 0, b.comp>>>(b.acc, b.land, b.n);
      CK(hipStreamWriteValue64(b.comp, hcredit, (uint64_t)i, 0));
    }
  }
  CK(hipGetLastError());
  const auto t0 = std::chrono::steady_clock::now();
  __atomic_store_n(gate, (uint64_t)1, __ATOMIC_SEQ_CST);
  CK(hipStreamSynchronize(b.comp));
  CK(hipStreamSynchronize(b.copy));
  const auto t1 = std::chrono::steady_clock::now();
  if (mode == "events") {
    for (int i = 0; i <= K; i++) {
      CK(hipEventDestroy(evc[i]));
      CK(hipEventDestroy(evr[i]));
    }
  }
  return std::chrono::duration<double>(t1 - t0).count();
}

// the host-issued steps engine's hand-off: the host sees copy i's event,
// then launches the reduce of round i
static double host_run(Bufs& b, int K) {
  reset(b);
  const int G = grid_for(b.n);
  std::vector<hipEvent_t> evc(K + 1), evr(K + 1);
  for (int i = 0; i <= K; i++) {
    CK(hipEventCreateWithFlags(&evc[i], hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&evr[i], hipEventDisableTiming));
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 1; i <= K; i++) {
    if (i > 1) CK(hipStreamWaitEvent(b.copy, evr[i - 1], 0));
    CK(hipMemcpyAsync(b.land, b.acc, b.n * sizeof(float), hipMemcpyDeviceToDevice, b.copy));
    CK(hipEventRecord(evc[i], b.copy));
    for (;;) {
      const hipError_t e = hipEventQuery(evc[i]);
      if (e == hipSuccess) break;
      if (e != hipErrorNotReady) CK(e);
      _mm_pause();
    }
    step_kernel<<<G, 256, 0, b.comp>>>(b.acc, b.land, b.n);
    CK(hipEventRecord(evr[i], b.comp));
  }
  CK(hipStreamSynchronize(b.comp));
  const auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i <= K; i++) {
    CK(hipEventDestroy(evc[i]));
    CK(hipEventDestroy(evr[i]));
  }
  return std::chrono::duration<double>(t1 - t0).count();
}

int main(int argc, char** argv) {
  const int K = argc > 1 ? std::atoi(argv[1]) : 200;
  std::vector<size_t> sizes;
  for (int i = 2; i < argc; i++) sizes.push_back((size_t)std::atoll(argv[i]));
  if (sizes.empty()) sizes = {1024, 262144};
  int canWait = 0;
  CK(hipDeviceGetAttribute(&canWait, hipDeviceAttributeCanUseStreamWaitValue, 0));
  const char* cp = std::getenv("GPU_STREAMOPS_CP_WAIT");
  Bufs b;
  CK(hipStreamCreateWithFlags(&b.copy, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&b.comp, hipStreamNonBlocking));
  CK(hipExtMallocWithFlags((void**)&b.dflags, 4 * kStride * sizeof(uint64_t),
                           hipDeviceMallocUncached));
  CK(hipMalloc((void**)&b.ticket, sizeof(unsigned)));
  CK(hipHostMalloc((void**)&b.hwords, 4 * kStride * sizeof(uint64_t),
                   hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc((void**)&b.status, sizeof(int), hipHostMallocCoherent | hipHostMallocMapped));
  for (size_t n : sizes) {
    b.n = n;
    CK(hipMalloc((void**)&b.acc, n * sizeof(float)));
    CK(hipExtMallocWithFlags((void**)&b.land, n * sizeof(float), hipDeviceMallocUncached));
    std::vector<std::string> modes = {"host", "events", "kernels"};
    if (canWait) modes.push_back("memops");
    for (const auto& m : modes) {
      // one untimed pass, then the timed one
      double s = m == "host" ? host_run(b, 20) : gated_run(b, 20, m);
      s = m == "host" ? host_run(b, K) : gated_run(b, K, m);
      const bool ok = check(b, K) && *b.status == 0;
      std::printf(
          "{\"mode\": \"%s\", \"floats\": %zu, \"rounds\": %d, \"us_per_round\": %.2f, "
          "\"exact\": %s, \"status\": %d, \"cp_wait\": \"%s\", \"can_wait_value\": %d}\n",
          m.c_str(), n, K, s * 1e6 / K, ok ? "true" : "false", *b.status, cp ? cp : "",
          canWait);
      std::fflush(stdout);
      if (*b.status != 0) return 2;
    }
    CK(hipFree(b.acc));
    CK(hipFree(b.land));
  }
  return 0;
}
