// executor_internal.h -- helpers shared by the executor's translation units
// (executor.cc: construction, rendezvous of scratch, the host-issued steps
// engine; executor_host.cc: host-memory endpoints; executor_device.cc: the
// device-driven engines).
#pragma once

#include <immintrin.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime_api.h>

namespace gloo {
namespace exec {

// A SEND is split only when every part is at least this big.
constexpr size_t kMinSplitBytes = 1 << 20;

// GLOO_AMD_TRACE=1: one stderr line per executor step / runtime call.
inline bool traceOn() {
  static const bool on = [] {
    const char* e = std::getenv("GLOO_AMD_TRACE");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

#define GLX_TRACE(...)                                   \
  do {                                                   \
    if (::gloo::exec::traceOn()) {                       \
      std::fprintf(stderr, "[glx-trace] " __VA_ARGS__);  \
      std::fputc('\n', stderr);                          \
    }                                                    \
  } while (0)

// GLOO_AMD_TRACE_MEM=1: one stderr line per allocation, free, host
// registration and unregistration the library makes (diagnostics).
inline bool traceMemOn() {
  static const bool on = [] {
    const char* e = std::getenv("GLOO_AMD_TRACE_MEM");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

#define GLX_TRACE_MEM(...)                                   \
  do {                                                       \
    if (::gloo::exec::traceMemOn()) {                        \
      std::fprintf(stderr, "[glx-mem] " __VA_ARGS__);        \
      std::fputc('\n', stderr);                              \
    }                                                        \
  } while (0)

// Host memory (pageable or pinned) as opposed to device/managed memory.
inline bool isHostPointer(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return true;  // unknown to HIP: plain pageable host memory
  }
  return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeUnregistered;
}

inline bool isPinnedHost(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Blocking wait for a stream with a short wake-up: poll for up to 200 us
// (a device-driven small allreduce finishes in a few us; the runtime's
// blocking wait adds several us of wake-up), then block.
inline hipError_t spinSync(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
    _mm_pause();
  }
  return hipStreamSynchronize(s);
}

// H2D pieces of host-mode staging: small enough that the schedule starts
// early, large enough to run the PCIe link at full rate.
constexpr int64_t kStagePieceBytes = int64_t(8) << 20;
// bounce block of a pageable buffer that has no whole pinned mirror
constexpr size_t kBounceBytes = size_t(8) << 20;
// free pinned blocks the process-wide cache keeps for later algorithms; the
// rest go back to the runtime (hipHostFree)
constexpr size_t kPinnedCacheCap = size_t(1) << 30;
// glx_set_pinned_mirror_limit: pageable buffers above it use a bounce block
// (0: no limit)
size_t pinnedMirrorLimit();
void setPinnedMirrorLimit(size_t bytes);

}  // namespace exec
}  // namespace gloo
