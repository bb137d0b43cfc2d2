// copy_bw.hip -- microbenchmark: how fast does a grid of G workgroups copy
// when each workgroup streams its own contiguous slice (the device engines'
// slicing, xgmi_kernels.hip) vs a grid-stride loop over the whole buffer?
// Built and driven by tools/micro/copy_bw.py (one GPU).
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint32_t v4u __attribute__((ext_vector_type(4)));

template <int U, bool SLICED>
__global__ __launch_bounds__(256, 2) void copy_kernel(v4u* dst, const v4u* src, size_t nv,
                                                      size_t slice) {
  size_t a = 0, b = nv, stride = 256;
  size_t i;
  if (SLICED) {
    a = (size_t)blockIdx.x * slice;
    b = a + slice < nv ? a + slice : nv;
    i = a + threadIdx.x;
  } else {
    stride = (size_t)gridDim.x * 256;
    i = (size_t)blockIdx.x * 256 + threadIdx.x;
  }
  for (; i + (U - 1) * stride < b; i += U * stride) {
    v4u x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = src[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; u++) dst[i + u * stride] = x[u];
  }
  for (; i < b; i += stride) dst[i] = src[i];
}

extern "C" int copy_bw_launch(void* dst, const void* src, size_t bytes, int G, int U, int sliced,
                              hipStream_t s) {
  const size_t nv = bytes / 16;
  const size_t slice = (nv + G - 1) / G;
  v4u* d = (v4u*)dst;
  const v4u* x = (const v4u*)src;
#define L(UU, SS) hipLaunchKernelGGL((copy_kernel<UU, SS>), dim3(G), dim3(256), 0, s, d, x, nv, slice)
  if (sliced) {
    if (U == 4) L(4, true); else if (U == 8) L(8, true); else L(16, true);
  } else {
    if (U == 4) L(4, false); else if (U == 8) L(8, false); else L(16, false);
  }
#undef L
  return (int)hipGetLastError();
}
