// oneshot_kernels.hip -- the replicated ring_chunked schedule (plan.h,
// planRingChunkedReplicated / planFnRingReplicated) as ONE device-driven
// kernel per rank, for small buffers where the host-mediated executor's
// per-hop latency (event polling + control-block counters, ~40 us) would
// dominate.
//
// Every rank runs the same grid over the same element slices (a function
// of count, dtype and P only).  Workgroup w of rank r:
//   1. push  -- stores slice w of r's buffer into its landing region in
//               every peer (IPC-mapped, uncached device memory) over xGMI,
//               then system-scope release and one flag word per peer:
//               flag[peer][r][w] = epoch;
//   2. wait  -- one lane polls flag[r][k][w] >= epoch for every peer k
//               (bounded: a peer that never arrives sets *status and the
//               workgroup exits -- every wave reaches the end);
//   3. fold  -- slice w of the result, each chunk's elements folded along
//               that chunk's ring chain (the same operand order as the
//               ring: acc = op(newer rank's value, acc)), written in place.
// Landing regions are double-buffered by epoch parity: a rank writes epoch
// e into region[e & 1] of a peer only after its epoch e-1 kernel saw every
// peer's epoch e-1 flags, i.e. after every peer finished epoch e-2, the last
// reader of that region.
//
// Bit-exact with the host-mediated replicated plan and hence with the
// reference's ring (same chains; tests/test_allreduce_gpu.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "elem_ops.h"
#include "kernels.h"

namespace glx {
namespace {

template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void oneshot_kernel(OneShotParams p) {
  using E = Elem<T, OP>;
  using S = typename E::S;
  constexpr int V = 16 / sizeof(S);
  const int w = blockIdx.x;
  const size_t e0 = (size_t)w * p.slice;
  const size_t e1 = e0 + p.slice < p.count ? e0 + p.slice : p.count;
  S* buf = reinterpret_cast<S*>(p.buf);
  const bool aligned = ((uintptr_t)p.buf % 16) == 0;
  // vectors [v0, v1) and scalar tail [t0, e1) of this slice (e0 % V == 0)
  const size_t v0 = e0 / V, v1 = e1 / V, t0 = v1 * V > e0 ? v1 * V : e0;

  // ---- 1. push -------------------------------------------------------------
  // each vector is loaded once and stored to every peer (ring order from rank+1)
  char* to[kOsMaxRanks - 1];
#pragma unroll
  for (int d = 1; d < kOsMaxRanks; d++) {
    int j = p.rank + d;
    if (j >= p.P) j -= p.P;
    to[d - 1] = d < p.P ? p.push[j] : nullptr;
  }
  if (aligned) {
    for (size_t i = v0 + threadIdx.x; i < v1; i += kBlock) {
      const v4u x = reinterpret_cast<const v4u*>(buf)[i];
#pragma unroll
      for (int d = 1; d < kOsMaxRanks; d++) {
        if (d < p.P) reinterpret_cast<v4u*>(to[d - 1])[i] = x;
      }
    }
  }
  for (size_t i = (aligned ? t0 : e0) + threadIdx.x; i < e1; i += kBlock) {
    const S x = buf[i];
#pragma unroll
    for (int d = 1; d < kOsMaxRanks; d++) {
      if (d < p.P) reinterpret_cast<S*>(to[d - 1])[i] = x;
    }
  }
  // every wave's stores complete and visible system-wide before the flags
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __syncthreads();
  if ((int)threadIdx.x < p.P && (int)threadIdx.x != p.rank) {
    __hip_atomic_store(p.flagOut[threadIdx.x] + w, p.epoch, __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }

  // ---- 2. wait ---------------------------------------------------------------
  __shared__ int s_ok;
  if (threadIdx.x == 0) {
    int ok = 1;
    const uint64_t start = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < p.P && ok; k++) {
      if (k == p.rank) continue;
      const uint64_t* f = p.flagIn + (size_t)k * p.G + w;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < p.epoch) {
        if (__builtin_amdgcn_s_memrealtime() - start > p.timeoutTicks) {
          ok = 0;
          __hip_atomic_store(p.status, 1 + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    // drop any stale copy of the landing lines before anyone reads them
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    s_ok = ok;
  }
  __syncthreads();
  if (!s_ok) return;

  // ---- 3. fold ---------------------------------------------------------------
  for (int q = 0; q < p.njobs; q++) {
    const size_t jb = p.jobOff[q], je = p.jobOff[q] + p.jobLen[q];
    const size_t a = jb > e0 ? jb : e0, b = je < e1 ? je : e1;
    if (a >= b) continue;
    const S* src[kOsMaxRanks];
#pragma unroll
    for (int i = 0; i < kOsMaxRanks; i++) {
      const int r = p.chain[q][i];
      src[i] = i < p.P ? (r == p.rank ? buf : reinterpret_cast<const S*>(p.land[r])) : nullptr;
    }
    size_t sa = a, sb = b;  // vector body [sa, sb) when aligned
    if (aligned) {
      sa = (a + V - 1) / V * V;
      sb = b / V * V;
      if (sa > sb) sa = sb = b;
    } else {
      sa = sb = b;
    }
    // scalar head [a, sa) and tail [sb, b) (everything when unaligned)
    for (size_t t = threadIdx.x; t < (sa - a) + (b - sb); t += kBlock) {
      const size_t i = t < sa - a ? a + t : sb + (t - (sa - a));
      S acc = src[0][i];
#pragma unroll
      for (int k = 1; k < kOsMaxRanks; k++) {
        if (k < p.P) acc = E::apply(src[k][i], acc);
      }
      buf[i] = acc;
    }
    for (size_t v = sa / V + threadIdx.x; v < sb / V; v += kBlock) {
      v4u y[kOsMaxRanks];  // all P loads in flight before the chain
#pragma unroll
      for (int k = 0; k < kOsMaxRanks; k++) {
        if (k < p.P) y[k] = reinterpret_cast<const v4u*>(src[k])[v];
      }
      v4u acc = y[0];
#pragma unroll
      for (int k = 1; k < kOsMaxRanks; k++) {
        if (k < p.P) acc = vec_apply<T, OP>(y[k], acc);
      }
      reinterpret_cast<v4u*>(buf)[v] = acc;
    }
  }
}

template <typename T>
hipError_t launch_os_op(int op, const OneShotParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.G), block(kBlock);
  switch (op) {
    case GLX_SUM: hipLaunchKernelGGL((oneshot_kernel<T, GLX_SUM>), grid, block, 0, s, p); break;
    case GLX_PRODUCT:
      hipLaunchKernelGGL((oneshot_kernel<T, GLX_PRODUCT>), grid, block, 0, s, p);
      break;
    case GLX_MAX: hipLaunchKernelGGL((oneshot_kernel<T, GLX_MAX>), grid, block, 0, s, p); break;
    case GLX_MIN: hipLaunchKernelGGL((oneshot_kernel<T, GLX_MIN>), grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t launch_oneshot(int op, int dtype, const OneShotParams& p, hipStream_t s) {
  if (p.P < 2 || p.P > kOsMaxRanks || p.G < 1 || p.G > kOsMaxSlices || p.njobs < 0 ||
      p.njobs > kOsMaxRanks || p.count == 0 || p.slice == 0 ||
      (size_t)p.G * p.slice < p.count || (size_t)(p.G - 1) * p.slice >= p.count) {
    return hipErrorInvalidValue;  // the grid must cover the buffer exactly
  }
  switch (dtype) {
    case GLX_INT8: return launch_os_op<int8_t>(op, p, s);
    case GLX_UINT8: return launch_os_op<uint8_t>(op, p, s);
    case GLX_INT32: return launch_os_op<int32_t>(op, p, s);
    case GLX_INT64: return launch_os_op<int64_t>(op, p, s);
    case GLX_UINT64: return launch_os_op<uint64_t>(op, p, s);
    case GLX_FLOAT32: return launch_os_op<float>(op, p, s);
    case GLX_FLOAT64: return launch_os_op<double>(op, p, s);
    case GLX_FLOAT16: return launch_os_op<f16_t>(op, p, s);
    case GLX_BFLOAT16: return launch_os_op<bf16_t>(op, p, s);
  }
  return hipErrorInvalidValue;
}

}  // namespace glx
