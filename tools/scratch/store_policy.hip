// Microbench: in-place fp32 a += b over 256 MiB with the product's
// grid-stride shape (unroll 4, 64 workgroups per CU), varying the cache
// policy of the loads and of the stores; plus the same with `a` in uncached
// memory (hipDeviceMallocUncached).  Question: the copy kernel stores into
// uncached memory faster than into plain memory (tools/scratch/uc_store_bw.py,
// profiles/r4h_*); does a write-through store policy give the reduce the same?
// hipcc --offload-arch=gfx950 -O3 -o store_policy store_policy.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));
constexpr int kBlock = 256;

template <int LP>
__device__ __forceinline__ v4u ld(const v4u* p) {
  if (LP == 1) return __builtin_nontemporal_load(p);
  return *p;
}
// SP: 0 plain, 1 nt (builtin), 2 sc1, 3 sc0 sc1, 4 nt sc0 sc1, 5 sc0
template <int SP>
__device__ __forceinline__ void st(v4u* p, v4u v) {
  if (SP == 0) {
    *p = v;
  } else if (SP == 1) {
    __builtin_nontemporal_store(v, p);
  } else if (SP == 2) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
  } else if (SP == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(p), "v"(v) : "memory");
  } else if (SP == 4) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  } else {
    asm volatile("global_store_dwordx4 %0, %1, off sc0" ::"v"(p), "v"(v) : "memory");
  }
}
__device__ __forceinline__ v4u add(v4u x, v4u y) {
  v4f a = __builtin_bit_cast(v4f, x), b = __builtin_bit_cast(v4f, y);
  return __builtin_bit_cast(v4u, a + b);
}

template <int U, int LP, int SP>
__global__ __launch_bounds__(kBlock) void k_gs(v4u* c, const v4u* a, const v4u* b, size_t n) {
  const size_t step = (size_t)gridDim.x * kBlock * U;
  for (size_t base = (size_t)blockIdx.x * kBlock * U + threadIdx.x; base < n; base += step) {
    v4u x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) { x[u] = ld<LP>(a + i); y[u] = ld<LP>(b + i); }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < n) st<SP>(c + i, add(x[u], y[u]));
    }
  }
}

__global__ void fill_random(v4u* p, size_t n, unsigned seed) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    v4u v;
    for (int k = 0; k < 4; k++) {
      unsigned long long x = (i * 4 + k) ^ ((unsigned long long)seed << 40);
      x += 0x9e3779b97f4a7c15ull;
      x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
      x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
      x ^= x >> 31;
      // a float in [-1, 1): sums never overflow over the runs
      v[k] = __float_as_uint(((float)(x >> 40) - 8388608.0f) / 8388608.0f);
    }
    p[i] = v;
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1);} } while (0)

int main(int argc, char** argv) {
  const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 256;
  const bool random = argc > 2 && argv[2][0] == 'r';
  const size_t bytes = mib << 20, n = bytes / 16;
  v4u *a, *b, *auc;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipExtMallocWithFlags((void**)&auc, bytes, hipDeviceMallocUncached));
  if (random) {
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, a, n, 1u);
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, b, n, 2u);
    hipLaunchKernelGGL(fill_random, dim3(4096), dim3(256), 0, 0, auc, n, 3u);
  } else {
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    CK(hipMemset(auc, 0, bytes));
  }
  CK(hipDeviceSynchronize());
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; i++) launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ts;
    for (int r = 0; r < 20; r++) {
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
    printf("{\"MiB\": %zu, \"data\": \"%s\", \"variant\": \"%s\", \"us_med\": %.2f, \"us_min\": %.2f, \"TBps_med\": %.3f}\n",
           mib, random ? "random" : "zeros", name, us, best, 3.0 * bytes / us / 1e6);
    fflush(stdout);
  };
  const dim3 grid(cus * 64), blk(kBlock);
#define V(NAME, LP, SP, C, A) \
  timeit(NAME, [&] { hipLaunchKernelGGL((k_gs<4, LP, SP>), grid, blk, 0, 0, C, A, b, n); })
  V("ld_nt st_nt (product)", 1, 1, a, a);
  V("ld_nt st_plain", 1, 0, a, a);
  V("ld_nt st_sc1", 1, 2, a, a);
  V("ld_nt st_sc0sc1", 1, 3, a, a);
  V("ld_nt st_sc0sc1nt", 1, 4, a, a);
  V("ld_nt st_sc0", 1, 5, a, a);
  V("ld_plain st_sc0sc1", 0, 3, a, a);
  V("ld_plain st_plain", 0, 0, a, a);
  V("uncached a: ld_nt st_plain", 1, 0, auc, auc);
  V("ld_nt st_nt (product)", 1, 1, a, a);
  return 0;
}
