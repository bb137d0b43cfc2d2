// Microbench: in-place fp32 a += b over 256 MiB, launch-shape variants.
// hipcc --offload-arch=gfx950 -O3 -o reduce_variants reduce_variants.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

template <bool NT>
__device__ __forceinline__ v4u ld(const v4u* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(v4u* p, v4u v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
__device__ __forceinline__ v4u add(v4u x, v4u y) {
  v4f a = __builtin_bit_cast(v4f, x), b = __builtin_bit_cast(v4f, y);
  return __builtin_bit_cast(v4u, a + b);
}

// 0: grid-stride (the product's shape)
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_gs(v4u* a, const v4u* b, size_t n) {
  const size_t step = (size_t)gridDim.x * kBlock * U;
  for (size_t base = (size_t)blockIdx.x * kBlock * U + threadIdx.x; base < n; base += step) {
    v4u x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) { x[u] = ld<NT>(a + i); y[u] = ld<NT>(b + i); }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) st<NT>(a + i, add(x[u], y[u]));
    }
  }
}

// 1: contiguous span per workgroup
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_span(v4u* a, const v4u* b, size_t n) {
  const size_t tile = (size_t)kBlock * U;
  const size_t tiles = (n + tile - 1) / tile;
  const size_t per = (tiles + gridDim.x - 1) / gridDim.x;
  const size_t t0 = blockIdx.x * per, t1 = std::min(tiles, t0 + per);
  for (size_t t = t0; t < t1; t++) {
    const size_t base = t * tile + threadIdx.x;
    v4u x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) { x[u] = ld<NT>(a + i); y[u] = ld<NT>(b + i); }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) st<NT>(a + i, add(x[u], y[u]));
    }
  }
}

// 2: one tile per workgroup (grid = tiles); XCD: tiles of consecutive
// workgroups on one XCD are adjacent
template <int U, bool NT, bool XCD>
__global__ __launch_bounds__(kBlock) void k_flat(v4u* a, const v4u* b, size_t n) {
  size_t t = blockIdx.x;
  if (XCD) {
    const size_t G = gridDim.x;  // multiple of 8 by construction
    t = (t % 8) * (G / 8) + t / 8;
  }
  const size_t base = t * kBlock * U + threadIdx.x;
  v4u x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + (size_t)u * kBlock;
    if (i < n) { x[u] = ld<NT>(a + i); y[u] = ld<NT>(b + i); }
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + (size_t)u * kBlock;
    if (i < n) st<NT>(a + i, add(x[u], y[u]));
  }
}

// 3: grid-stride, loads of the next iteration issued before this one's stores
template <int U, bool NT>
__global__ __launch_bounds__(kBlock) void k_pipe(v4u* a, const v4u* b, size_t n) {
  const size_t step = (size_t)gridDim.x * kBlock * U;
  size_t base = (size_t)blockIdx.x * kBlock * U + threadIdx.x;
  v4u x[U], y[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + (size_t)u * kBlock;
    if (i < n) { x[u] = ld<NT>(a + i); y[u] = ld<NT>(b + i); }
  }
  for (; base < n; base += step) {
    v4u r[U];
#pragma unroll
    for (int u = 0; u < U; u++) r[u] = add(x[u], y[u]);
    const size_t nb = base + step;
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = nb + (size_t)u * kBlock;
      if (i < n) { x[u] = ld<NT>(a + i); y[u] = ld<NT>(b + i); }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) st<NT>(a + i, r[u]);
    }
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

int main() {
  const size_t bytes = size_t(256) << 20, n = bytes / 16;
  v4u *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 0, bytes));
  CK(hipMemset(b, 0, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, int U, int bpc, auto launch) {
    for (int i = 0; i < 5; i++) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 30; r++) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    const double us = ts[ts.size() / 2] * 1e3, best = ts[0] * 1e3;
    printf("{\"kernel\": \"%s\", \"unroll\": %d, \"bpc\": %d, \"us_med\": %.2f, \"us_min\": %.2f, \"TBps_med\": %.3f}\n",
           name, U, bpc, us, best, 3.0 * bytes / us / 1e6);
    fflush(stdout);
  };
#define GS(U, NT, BPC) timeit(NT ? "gs_nt" : "gs", U, BPC, [&] { hipLaunchKernelGGL((k_gs<U, NT>), dim3(cus * BPC), dim3(kBlock), 0, 0, a, b, n); })
#define SP(U, NT, BPC) timeit(NT ? "span_nt" : "span", U, BPC, [&] { hipLaunchKernelGGL((k_span<U, NT>), dim3(cus * BPC), dim3(kBlock), 0, 0, a, b, n); })
#define PI(U, NT, BPC) timeit(NT ? "pipe_nt" : "pipe", U, BPC, [&] { hipLaunchKernelGGL((k_pipe<U, NT>), dim3(cus * BPC), dim3(kBlock), 0, 0, a, b, n); })
#define FL(U, NT, X) timeit(X ? (NT ? "flat_xcd_nt" : "flat_xcd") : (NT ? "flat_nt" : "flat"), U, 0, [&] { \
    size_t G = (n + kBlock * U - 1) / (kBlock * U); G = (G + 7) / 8 * 8; \
    hipLaunchKernelGGL((k_flat<U, NT, X>), dim3((unsigned)G), dim3(kBlock), 0, 0, a, b, n); })
  for (int pass = 0; pass < 2; pass++) {
    GS(4, true, 64); GS(4, true, 8); GS(4, true, 4); GS(8, true, 8); GS(2, true, 16);
    GS(4, false, 64);
    SP(4, true, 4); SP(4, true, 8); SP(8, true, 4); SP(4, false, 8); SP(2, true, 16);
    PI(4, true, 4); PI(4, true, 8); PI(2, true, 8); PI(2, true, 16);
    FL(1, true, false); FL(2, true, false); FL(4, true, false); FL(4, false, false);
    FL(2, true, true); FL(4, true, true); FL(8, true, true);
  }
  return 0;
}
