// reduce_kernels.hip -- the per-chunk elementwise reduction of the gloo
// allreduce hot path, hand-written for CDNA4 (gfx950).
//
// Replaces gloo::sum/product/max/min<T> (gloo/math.h:15-73) and the CUDA
// analog cudaSum/... (gloo/cuda.cu:307-434).  Memory-bound: 3 streams of
// n*sizeof(T) bytes (two reads, one write) per call, no reuse -> the roofline
// is HBM (8 TB/s spec, ~6.3 TB/s achievable float4 copy on MI355X).  No MFMA,
// no LDS: each lane moves 16-byte vectors (global_load/store_dwordx4), UNROLL
// independent vectors in flight per lane, 256-thread (4-wave) workgroups,
// grid-stride over a grid capped at a few workgroups per CU.
//
// Semantics are the reference CPU path's, bit for bit:
//   sum / product : a + b, a * b (integers wrap, IEEE fp32/fp64 RNE)
//   max           : (a < b) ? b : a     == std::max(a, b)  (gloo/math.h:51)
//   min           : (b < a) ? b : a     == std::min(a, b)  (gloo/math.h:66)
//   float16       : widen (exact), op in fp32, round-to-nearest-even once,
//                   NaN -> 0x7fff          (gloo/types.h:181-204, 248-305)
//                   max/min compare in fp32, return the raw 16-bit operand
//                   (gloo/types.h:318-336 + std::max on float16 objects)
//   bfloat16      : as float16 with bf16 rounding (no reference: unpinned)
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <cstdlib>
#include <type_traits>
#include <vector>

#include "common.h"
#include "elem_ops.h"
#include "kernels.h"

namespace glx {
namespace {

// ---- kernels --------------------------------------------------------------

// Elements [0, head) and [head + nvec*V, head + nvec*V + tail) are done one
// per thread by the first threads of the grid; [head, head + nvec*V) is the
// 16-byte-aligned body, UNROLL vectors per lane per grid-stride step.
// dst may alias a or b: every lane reads its vectors before writing them.
// LOADC: dst is not a, and its prior value matters (float16 assignment
// semantics) -- read it as a third stream.
template <typename T, int OP, int UNROLL, bool LOADC, int POL>
__global__ __launch_bounds__(kBlock) void reduce_kernel(
    typename Elem<T, OP>::S* dst, const typename Elem<T, OP>::S* a,
    const typename Elem<T, OP>::S* b, size_t head, size_t nvec, size_t tail) {
  using E = Elem<T, OP>;
  using S = typename E::S;
  constexpr int V = 16 / sizeof(S);
  const size_t gtid = (size_t)blockIdx.x * kBlock + threadIdx.x;

  if (gtid < head) dst[gtid] = LOADC ? E::apply3(dst[gtid], a[gtid], b[gtid]) : E::apply(a[gtid], b[gtid]);
  if (gtid < tail) {
    size_t i = head + nvec * V + gtid;
    dst[i] = LOADC ? E::apply3(dst[i], a[i], b[i]) : E::apply(a[i], b[i]);
  }

  v4u* vd = reinterpret_cast<v4u*>(dst + head);
  const v4u* va = reinterpret_cast<const v4u*>(a + head);
  const v4u* vb = reinterpret_cast<const v4u*>(b + head);
  const WtStream wt(vd);
  const size_t step = (size_t)gridDim.x * kBlock * UNROLL;
  for (size_t base = (size_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
       base < nvec; base += step) {
    v4u x[UNROLL], y[UNROLL], z[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec) {
        x[u] = ld16p<POL>(va + i);
        y[u] = ld16p<POL>(vb + i);
        if (LOADC) z[u] = vd[i];
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec) {
        const v4u r = LOADC ? vec_apply3<T, OP>(z[u], x[u], y[u]) : vec_apply<T, OP>(x[u], y[u]);
        if (POL == kPolNtWt) {
          wt.put(i, r);
        } else {
          st16<POL == kPolNt>(vd + i, r);
        }
      }
    }
  }
}

// Fallback when a, b and dst do not share one 16-byte phase: element-wise,
// still coalesced across lanes.
template <typename T, int OP>
__global__ __launch_bounds__(kBlock) void reduce_scalar_kernel(
    typename Elem<T, OP>::S* dst, const typename Elem<T, OP>::S* a,
    const typename Elem<T, OP>::S* b, size_t n) {
  using E = Elem<T, OP>;
  const size_t step = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += step)
    dst[i] = E::apply3(dst[i], a[i], b[i]);
}

// Fold over k <= kMaxSrc sources, one pass:
//   REV = false: acc = s0; acc = op(acc, s_j)   -- left fold, the reference's
//                local multi-pointer reduce (gloo/allreduce_ring_chunked.h:89-91)
//   REV = true : acc = s0; acc = op(s_j, acc)   -- the ring's per-chunk chain,
//                where each rank applies op(own value, incoming partial)
//                (gloo/allreduce_ring_chunked.h:145)
// Same 16-byte phase requirement as reduce_kernel (else the scalar kernel).
constexpr int kMaxSrc = 16;
struct SrcPtrs { const void* p[kMaxSrc]; };

template <typename T, int OP, bool REV>
__device__ __forceinline__ typename Elem<T, OP>::S fold_step(typename Elem<T, OP>::S acc,
                                                             typename Elem<T, OP>::S y) {
  return REV ? Elem<T, OP>::apply(y, acc) : Elem<T, OP>::apply(acc, y);
}

template <typename T, int OP, int UNROLL, bool REV, bool WT>
__global__ __launch_bounds__(kBlock) void reduce_n_kernel(
    typename Elem<T, OP>::S* dst, SrcPtrs srcs, int k, size_t head, size_t nvec,
    size_t tail) {
  using E = Elem<T, OP>;
  using S = typename E::S;
  constexpr int V = 16 / sizeof(S);
  const size_t gtid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  auto src = [&](int j) { return reinterpret_cast<const S*>(srcs.p[j]); };
  for (int side = 0; side < 2; side++) {
    size_t lim = side == 0 ? head : tail;
    if (gtid >= lim) continue;
    size_t i = side == 0 ? gtid : head + nvec * V + gtid;
    S acc = src(0)[i];
    for (int j = 1; j < k; j++) acc = fold_step<T, OP, REV>(acc, src(j)[i]);
    dst[i] = acc;
  }
  v4u* vd = reinterpret_cast<v4u*>(dst + head);
  const WtStream wt(vd);
  const size_t step = (size_t)gridDim.x * kBlock * UNROLL;
  for (size_t base = (size_t)blockIdx.x * kBlock * UNROLL + threadIdx.x;
       base < nvec; base += step) {
    v4u acc[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec) acc[u] = ld16<true>(reinterpret_cast<const v4u*>(src(0) + head) + i);
    }
    for (int j = 1; j < k; j++) {
      v4u y[UNROLL];
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        size_t i = base + (size_t)u * kBlock;
        if (i < nvec) y[u] = ld16<true>(reinterpret_cast<const v4u*>(src(j) + head) + i);
      }
#pragma unroll
      for (int u = 0; u < UNROLL; u++) {
        size_t i = base + (size_t)u * kBlock;
        if (i < nvec) acc[u] = REV ? vec_apply<T, OP>(y[u], acc[u]) : vec_apply<T, OP>(acc[u], y[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec) {
        if (WT) {
          wt.put(i, acc[u]);
        } else {
          st16<true>(vd + i, acc[u]);
        }
      }
    }
  }
}

// Several independent folds in one launch (blockIdx.y = job): the
// replicated schedule folds every chunk of the buffer, each in its own
// operand order, and one launch costs less than P back-to-back ones.
constexpr int kMaxJobs = 8;
struct FoldJob {
  void* dst;
  const void* p[kMaxSrc];
  int k;
  size_t head, nvec, tail;  // head/tail elements done scalar (head = n: all scalar)
};
struct FoldJobs { FoldJob j[kMaxJobs]; };

template <typename T, int OP, bool REV>
__global__ __launch_bounds__(kBlock) void reduce_n_batch_kernel(FoldJobs jobs) {
  using E = Elem<T, OP>;
  using S = typename E::S;
  constexpr int V = 16 / sizeof(S);
  const FoldJob& jb = jobs.j[blockIdx.y];
  S* dst = reinterpret_cast<S*>(jb.dst);
  auto src = [&](int j) { return reinterpret_cast<const S*>(jb.p[j]); };
  const size_t gstep = (size_t)gridDim.x * kBlock;
  const size_t gtid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  const size_t tail_at = jb.head + jb.nvec * V;
  for (size_t t = gtid; t < jb.head + jb.tail; t += gstep) {
    const size_t i = t < jb.head ? t : tail_at + (t - jb.head);
    S acc = src(0)[i];
    for (int j = 1; j < jb.k; j++) acc = fold_step<T, OP, REV>(acc, src(j)[i]);
    dst[i] = acc;
  }
  v4u* vd = reinterpret_cast<v4u*>(dst + jb.head);
  for (size_t i = gtid; i < jb.nvec; i += gstep) {
    v4u acc = ld16<true>(reinterpret_cast<const v4u*>(src(0) + jb.head) + i);
    for (int j = 1; j < jb.k; j++) {
      v4u y = ld16<true>(reinterpret_cast<const v4u*>(src(j) + jb.head) + i);
      acc = REV ? vec_apply<T, OP>(y, acc) : vec_apply<T, OP>(acc, y);
    }
    st16<true>(vd + i, acc);
  }
}

template <typename T, int OP, bool REV>
__global__ __launch_bounds__(kBlock) void reduce_n_scalar_kernel(
    typename Elem<T, OP>::S* dst, SrcPtrs srcs, int k, size_t n) {
  using S = typename Elem<T, OP>::S;
  const size_t step = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += step) {
    S acc = reinterpret_cast<const S*>(srcs.p[0])[i];
    for (int j = 1; j < k; j++)
      acc = fold_step<T, OP, REV>(acc, reinterpret_cast<const S*>(srcs.p[j])[i]);
    dst[i] = acc;
  }
}

// ---- peer copy ------------------------------------------------------------
// The chunk exchange as a kernel instead of a DMA (SDMA) copy: the lanes of
// the sending GPU store 16-byte vectors straight into the peer's receive
// region through its IPC-mapped address, so the copy runs over xGMI at the
// rate of the compute units' remote stores rather than one copy engine's.
// Nontemporal loads (the source is read once); write-through or plain
// stores by the stream policy (policy_for).  The first lanes move the
// unaligned head and tail bytes.
template <int UNROLL, bool WT>
__global__ __launch_bounds__(kBlock) void copy_kernel(char* __restrict__ dst,
                                                      const char* __restrict__ src,
                                                      size_t head, size_t nvec, size_t tail) {
  const size_t gtid = (size_t)blockIdx.x * kBlock + threadIdx.x;
  if (gtid < head) dst[gtid] = src[gtid];
  const size_t tail_at = head + nvec * 16;
  if (gtid < tail) dst[tail_at + gtid] = src[tail_at + gtid];
  const v4u* vs = reinterpret_cast<const v4u*>(src + head);
  v4u* vd = reinterpret_cast<v4u*>(dst + head);
  const WtStream wt(vd);
  const size_t stride = (size_t)gridDim.x * kBlock * UNROLL;
  for (size_t base = (size_t)blockIdx.x * kBlock * UNROLL + threadIdx.x; base < nvec;
       base += stride) {
    v4u x[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec) x[u] = ld16<true>(vs + i);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec) {
        if (WT) {
          wt.put(i, x[u]);
        } else {
          st16<false>(vd + i, x[u]);
        }
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void copy_bytes_kernel(char* __restrict__ dst,
                                                            const char* __restrict__ src,
                                                            size_t n) {
  const size_t step = (size_t)gridDim.x * kBlock;
  for (size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += step) dst[i] = src[i];
}

// ---- launch ---------------------------------------------------------------

// Process-wide launch settings.  Rank threads of one process launch
// concurrently while glx_tune_reduce / glx_set_copy_blocks may write them, so
// every setting is atomic (relaxed: each is read once per launch and any
// value written is a valid one), and the CU count is read once
// (executor*.cc keeps its settings the same way).
std::atomic<int> g_copy_blocks{64};  // grid of the copy kernel (workgroups)
std::atomic<int> g_unroll{4};  // tuned on MI355X: tools/tune_reduce.py, profiles/r1_tune_reduce_nt.log
std::atomic<int> g_blocks_per_cu{64};  // grid cap = CUs * this (256 MiB fp32: one vector pass per lane)
std::once_flag g_num_cus_once;
int g_num_cus = 256;  // written once under g_num_cus_once
// Cache policy of the reduce kernel's streams (StreamPolicy, or kPolAuto).
// Measured on MI355X with uniform random fp32 (tools/tune_policy.py,
// profiles/r4j_*, r4k_*): nontemporal loads always win; for the stores,
// write-through (sc1) is fastest while the written stream fits the 256 MB
// Infinity Cache (64 MiB: 28.0 vs 31.5 us; 256 MiB: 110.5 vs 123.7 us), and
// nontemporal stores are fastest beyond it (320 MiB: 161.9 vs 163.7 us;
// 1 GiB: 527 vs 543 us).
constexpr int kPolAuto = 4;
std::atomic<int> g_policy{kPolAuto};
constexpr size_t kWtMaxBytes = size_t(256) << 20;  // per stream, write-through up to here

int policy_for(size_t stream_bytes) {
  const int pol = g_policy.load(std::memory_order_relaxed);
  if (pol != kPolAuto) {
    // write-through streams are addressed by 32-bit buffer offsets
    return pol == kPolNtWt && stream_bytes > kWtMaxStream ? kPolNt : pol;
  }
  return stream_bytes <= kWtMaxBytes ? kPolNtWt : kPolNt;
}

// Write-through stores for the fold (reduce_n) and copy kernels: the
// reduce kernel's policy (policy_for) for the stream's size.
bool use_wt(size_t stream_bytes) {
  if (stream_bytes > kWtMaxStream) return false;
  return policy_for(stream_bytes) == kPolNtWt;
}

int num_cus() {
  std::call_once(g_num_cus_once, [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) ==
            hipSuccess &&
        n > 0) {
      g_num_cus = n;
    } else {
      (void)hipGetLastError();
    }
  });
  return g_num_cus;
}

size_t grid_for(size_t work_items, int unroll) {
  size_t per_block = (size_t)kBlock * unroll;
  size_t blocks = (work_items + per_block - 1) / per_block;
  size_t cap = (size_t)num_cus() * (size_t)g_blocks_per_cu.load(std::memory_order_relaxed);
  if (blocks > cap) blocks = cap;
  if (blocks == 0) blocks = 1;
  return blocks;
}

// Streams longer than this go out as consecutive launches over equal
// segments of at most this many bytes each (the policy still chosen for the
// whole stream).  One grid-stride launch over 1 GiB fp32 on the HBM-only loop
// took 526 us, four launches over 256 MiB segments 497 us (6.12 vs 6.48
// TB/s; 128 MiB: 502, 512 MiB: 505; at 256 MiB one launch stays best:
// tools/seg_1GiB.py, profiles/r10/reduce_segments.jsonl).
constexpr size_t kSegBytes = size_t(256) << 20;

template <typename T, int OP, int UNROLL>
hipError_t launch_vec(void* dst, const void* a, const void* b, size_t head,
                      size_t nvec, size_t tail, hipStream_t s, int pol) {
  using S = typename Elem<T, OP>::S;
  size_t blocks = grid_for(nvec, UNROLL);
  size_t edge_blocks = (std::max(head, tail) + kBlock - 1) / kBlock;
  if (blocks < edge_blocks) blocks = edge_blocks;
  const dim3 grid((unsigned)blocks), block(kBlock);
  if (std::is_same<T, f16_t>::value && dst != a) {
    hipLaunchKernelGGL((reduce_kernel<T, OP, UNROLL, true, kPolPlain>), grid, block, 0, s,
                       (S*)dst, (const S*)a, (const S*)b, head, nvec, tail);
    return hipGetLastError();
  }
  switch (pol) {
    case kPolPlain:
      hipLaunchKernelGGL((reduce_kernel<T, OP, UNROLL, false, kPolPlain>), grid, block, 0, s,
                         (S*)dst, (const S*)a, (const S*)b, head, nvec, tail);
      break;
    case kPolNtWt:
      hipLaunchKernelGGL((reduce_kernel<T, OP, UNROLL, false, kPolNtWt>), grid, block, 0, s,
                         (S*)dst, (const S*)a, (const S*)b, head, nvec, tail);
      break;
    case kPolNtPlain:
      hipLaunchKernelGGL((reduce_kernel<T, OP, UNROLL, false, kPolNtPlain>), grid, block, 0, s,
                         (S*)dst, (const S*)a, (const S*)b, head, nvec, tail);
      break;
    default:
      hipLaunchKernelGGL((reduce_kernel<T, OP, UNROLL, false, kPolNt>), grid, block, 0, s,
                         (S*)dst, (const S*)a, (const S*)b, head, nvec, tail);
  }
  return hipGetLastError();
}

template <typename T, int OP>
hipError_t launch_typed(void* dst, const void* a, const void* b, size_t n,
                        hipStream_t s) {
  using S = typename Elem<T, OP>::S;
  constexpr size_t es = sizeof(S);
  constexpr size_t V = 16 / es;
  uintptr_t pd = (uintptr_t)dst, pa = (uintptr_t)a, pb = (uintptr_t)b;
  if ((pd % 16) == (pa % 16) && (pd % 16) == (pb % 16) && (pd % es) == 0) {
    size_t head = ((16 - (pd % 16)) % 16) / es;
    if (head > n) head = n;
    size_t nvec = (n - head) / V;
    size_t tail = n - head - nvec * V;
    const int pol = policy_for(nvec * 16);  // the whole stream's
    // equal segments of at most kSegBytes (kSegBytes above): the head goes
    // with the first, the tail with the last
    const size_t nseg = (nvec * 16 + kSegBytes - 1) / kSegBytes;
    const size_t segVec = nseg > 1 ? (nvec + nseg - 1) / nseg : nvec;
    size_t at = 0;  // elements before this segment's first
    for (size_t v0 = 0; v0 < nvec || v0 == 0; v0 += segVec) {
      const size_t nv = std::min(segVec, nvec - v0);
      const size_t h = v0 == 0 ? head : 0;
      const size_t t = v0 + nv >= nvec ? tail : 0;
      S* d = static_cast<S*>(dst) + at;
      const S* x = static_cast<const S*>(a) + at;
      const S* y = static_cast<const S*>(b) + at;
      hipError_t e;
      switch (g_unroll.load(std::memory_order_relaxed)) {
        case 1: e = launch_vec<T, OP, 1>(d, x, y, h, nv, t, s, pol); break;
        case 2: e = launch_vec<T, OP, 2>(d, x, y, h, nv, t, s, pol); break;
        case 8: e = launch_vec<T, OP, 8>(d, x, y, h, nv, t, s, pol); break;
        default: e = launch_vec<T, OP, 4>(d, x, y, h, nv, t, s, pol);
      }
      if (e != hipSuccess) return e;
      at += h + nv * V;
      if (nv == 0) break;  // nvec == 0: the one launch did head and tail
    }
    return hipSuccess;
  }
  size_t blocks = grid_for(n, 4);
  hipLaunchKernelGGL((reduce_scalar_kernel<T, OP>), dim3((unsigned)blocks),
                     dim3(kBlock), 0, s, (S*)dst, (const S*)a, (const S*)b, n);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_op(int op, void* dst, const void* a, const void* b, size_t n,
                     hipStream_t s) {
  switch (op) {
    case GLX_SUM: return launch_typed<T, GLX_SUM>(dst, a, b, n, s);
    case GLX_PRODUCT: return launch_typed<T, GLX_PRODUCT>(dst, a, b, n, s);
    case GLX_MAX: return launch_typed<T, GLX_MAX>(dst, a, b, n, s);
    case GLX_MIN: return launch_typed<T, GLX_MIN>(dst, a, b, n, s);
  }
  return hipErrorInvalidValue;
}

template <typename T, int OP, bool REV>
hipError_t launch_n_pass(void* dst, const void* const* srcs, int k, size_t n,
                         hipStream_t s) {
  using S = typename Elem<T, OP>::S;
  constexpr size_t es = sizeof(S);
  constexpr size_t V = 16 / es;
  SrcPtrs sp{};
  for (int j = 0; j < k; j++) sp.p[j] = srcs[j];
  uintptr_t phase = (uintptr_t)dst % 16;
  bool same = ((uintptr_t)dst % es) == 0;
  for (int j = 0; j < k; j++) same = same && ((uintptr_t)srcs[j] % 16) == phase;
  if (!same) {
    size_t blocks = grid_for(n, 4);
    hipLaunchKernelGGL((reduce_n_scalar_kernel<T, OP, REV>), dim3((unsigned)blocks),
                       dim3(kBlock), 0, s, (S*)dst, sp, k, n);
    return hipGetLastError();
  }
  size_t head = ((16 - phase) % 16) / es;
  if (head > n) head = n;
  size_t nvec = (n - head) / V;
  size_t tail = n - head - nvec * V;
  const bool wt = use_wt(nvec * 16);  // the whole stream's policy
  // equal segments of at most kSegBytes, as launch_typed (1 GiB fp32, two
  // sources: 532 -> 500 us; four: 919 -> 886 us -- tools/seg_fold.py,
  // profiles/r10/fold_segments.jsonl)
  const size_t nseg = (nvec * 16 + kSegBytes - 1) / kSegBytes;
  const size_t segVec = nseg > 1 ? (nvec + nseg - 1) / nseg : nvec;
  size_t at = 0;  // elements before this segment's first
  for (size_t v0 = 0; v0 < nvec || v0 == 0; v0 += segVec) {
    const size_t nv = std::min(segVec, nvec - v0);
    const size_t h = v0 == 0 ? head : 0;
    const size_t t = v0 + nv >= nvec ? tail : 0;
    SrcPtrs q{};
    for (int j = 0; j < k; j++) q.p[j] = static_cast<const S*>(srcs[j]) + at;
    S* d = static_cast<S*>(dst) + at;
    size_t blocks = grid_for(nv, 4);
    size_t edge_blocks = (std::max(h, t) + kBlock - 1) / kBlock;
    if (blocks < edge_blocks) blocks = edge_blocks;
    if (wt) {
      hipLaunchKernelGGL((reduce_n_kernel<T, OP, 4, REV, true>), dim3((unsigned)blocks),
                         dim3(kBlock), 0, s, d, q, k, h, nv, t);
    } else {
      hipLaunchKernelGGL((reduce_n_kernel<T, OP, 4, REV, false>), dim3((unsigned)blocks),
                         dim3(kBlock), 0, s, d, q, k, h, nv, t);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    at += h + nv * V;
    if (nv == 0) break;  // nvec == 0: the one launch did head and tail
  }
  return hipSuccess;
}

// Folds of more than kMaxSrc sources continue from dst in further passes.
template <typename T, int OP>
hipError_t launch_n_typed(void* dst, const void* const* srcs, int k, size_t n,
                          hipStream_t s, bool rev) {
  std::vector<const void*> v(srcs, srcs + k);
  int at = 0;
  hipError_t e = hipSuccess;
  bool first = true;
  while (e == hipSuccess && (first || at < k)) {
    std::vector<const void*> pass;
    if (!first) pass.push_back(dst);
    while (at < k && (int)pass.size() < kMaxSrc) pass.push_back(v[at++]);
    if (pass.size() >= 2 || first) {
      e = rev ? launch_n_pass<T, OP, true>(dst, pass.data(), (int)pass.size(), n, s)
              : launch_n_pass<T, OP, false>(dst, pass.data(), (int)pass.size(), n, s);
    }
    first = false;
  }
  return e;
}

template <typename T, int OP>
hipError_t launch_batch_typed(const FoldJobs& jobs, int njobs, size_t max_work, bool rev,
                              hipStream_t s) {
  size_t bx = (max_work + kBlock - 1) / kBlock;
  size_t cap = (size_t)num_cus() * 8;
  if (bx > cap) bx = cap;
  if (bx == 0) bx = 1;
  dim3 grid((unsigned)bx, (unsigned)njobs);
  if (rev) {
    hipLaunchKernelGGL((reduce_n_batch_kernel<T, OP, true>), grid, dim3(kBlock), 0, s, jobs);
  } else {
    hipLaunchKernelGGL((reduce_n_batch_kernel<T, OP, false>), grid, dim3(kBlock), 0, s, jobs);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_batch_op(int op, const std::vector<FoldSpec>& specs, bool rev,
                           hipStream_t s) {
  using S = typename Elem<T, GLX_SUM>::S;
  constexpr size_t es = sizeof(S);
  constexpr size_t V = 16 / es;
  for (size_t at = 0; at < specs.size(); at += kMaxJobs) {
    FoldJobs jobs{};
    int nj = 0;
    size_t max_work = 1;
    for (size_t q = at; q < specs.size() && q < at + kMaxJobs; q++) {
      const FoldSpec& f = specs[q];
      if (f.n == 0) continue;
      if (f.k < 1 || f.k > kMaxSrc) return hipErrorInvalidValue;
      FoldJob& jb = jobs.j[nj++];
      jb.dst = f.dst;
      jb.k = f.k;
      uintptr_t phase = (uintptr_t)f.dst % 16;
      bool same = ((uintptr_t)f.dst % es) == 0;
      for (int j = 0; j < f.k; j++) {
        jb.p[j] = f.srcs[j];
        same = same && ((uintptr_t)f.srcs[j] % 16) == phase;
      }
      if (same) {
        jb.head = ((16 - phase) % 16) / es;
        if (jb.head > f.n) jb.head = f.n;
        jb.nvec = (f.n - jb.head) / V;
        jb.tail = f.n - jb.head - jb.nvec * V;
      } else {
        jb.head = f.n;
        jb.nvec = 0;
        jb.tail = 0;
      }
      max_work = std::max(max_work, std::max(jb.nvec, jb.head + jb.tail));
    }
    if (nj == 0) continue;
    hipError_t e = hipErrorInvalidValue;
    switch (op) {
      case GLX_SUM: e = launch_batch_typed<T, GLX_SUM>(jobs, nj, max_work, rev, s); break;
      case GLX_PRODUCT: e = launch_batch_typed<T, GLX_PRODUCT>(jobs, nj, max_work, rev, s); break;
      case GLX_MAX: e = launch_batch_typed<T, GLX_MAX>(jobs, nj, max_work, rev, s); break;
      case GLX_MIN: e = launch_batch_typed<T, GLX_MIN>(jobs, nj, max_work, rev, s); break;
    }
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <typename T>
hipError_t launch_n_op(int op, void* dst, const void* const* srcs, int k,
                       size_t n, hipStream_t s, bool rev) {
  switch (op) {
    case GLX_SUM: return launch_n_typed<T, GLX_SUM>(dst, srcs, k, n, s, rev);
    case GLX_PRODUCT: return launch_n_typed<T, GLX_PRODUCT>(dst, srcs, k, n, s, rev);
    case GLX_MAX: return launch_n_typed<T, GLX_MAX>(dst, srcs, k, n, s, rev);
    case GLX_MIN: return launch_n_typed<T, GLX_MIN>(dst, srcs, k, n, s, rev);
  }
  return hipErrorInvalidValue;
}

}  // namespace

hipError_t launch_copy(void* dst, const void* src, size_t bytes, hipStream_t s) {
  return launch_copy_blocks(dst, src, bytes, 0, s);
}

hipError_t launch_copy_blocks(void* dst, const void* src, size_t bytes, int grid,
                              hipStream_t s) {
  if (bytes == 0) return hipSuccess;
  const uintptr_t pd = (uintptr_t)dst, ps = (uintptr_t)src;
  const unsigned blocks =
      (unsigned)std::max(1, grid > 0 ? grid : g_copy_blocks.load(std::memory_order_relaxed));
  if (pd % 16 != ps % 16) {
    hipLaunchKernelGGL(copy_bytes_kernel, dim3(blocks), dim3(kBlock), 0, s, (char*)dst,
                       (const char*)src, bytes);
    return hipGetLastError();
  }
  size_t head = (16 - pd % 16) % 16;
  if (head > bytes) head = bytes;
  const size_t nvec = (bytes - head) / 16;
  const size_t tail = bytes - head - nvec * 16;
  if (use_wt(nvec * 16)) {
    hipLaunchKernelGGL((copy_kernel<4, true>), dim3(blocks), dim3(kBlock), 0, s, (char*)dst,
                       (const char*)src, head, nvec, tail);
  } else {
    hipLaunchKernelGGL((copy_kernel<4, false>), dim3(blocks), dim3(kBlock), 0, s, (char*)dst,
                       (const char*)src, head, nvec, tail);
  }
  return hipGetLastError();
}

void set_copy_blocks(int blocks) {
  if (blocks > 0) g_copy_blocks.store(blocks, std::memory_order_relaxed);
}

int copy_blocks() { return g_copy_blocks.load(std::memory_order_relaxed); }

hipError_t launch_reduce(int op, int dtype, void* dst, const void* a,
                         const void* b, size_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  switch (dtype) {
    case GLX_INT8: return launch_op<int8_t>(op, dst, a, b, n, s);
    case GLX_UINT8: return launch_op<uint8_t>(op, dst, a, b, n, s);
    case GLX_INT32: return launch_op<int32_t>(op, dst, a, b, n, s);
    case GLX_INT64: return launch_op<int64_t>(op, dst, a, b, n, s);
    case GLX_UINT64: return launch_op<uint64_t>(op, dst, a, b, n, s);
    case GLX_FLOAT32: return launch_op<float>(op, dst, a, b, n, s);
    case GLX_FLOAT64: return launch_op<double>(op, dst, a, b, n, s);
    case GLX_FLOAT16: return launch_op<f16_t>(op, dst, a, b, n, s);
    case GLX_BFLOAT16: return launch_op<bf16_t>(op, dst, a, b, n, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_reduce_n_batch(int op, int dtype, const std::vector<FoldSpec>& specs,
                                 hipStream_t s, bool rev) {
  for (const FoldSpec& f : specs) {
    if (f.k > kMaxSrc) {  // rare: fall back to one multi-pass fold each
      for (const FoldSpec& g : specs) {
        hipError_t e = launch_reduce_n(op, dtype, g.dst, g.srcs.data(), g.k, g.n, s, rev);
        if (e != hipSuccess) return e;
      }
      return hipSuccess;
    }
  }
  switch (dtype) {
    case GLX_INT8: return launch_batch_op<int8_t>(op, specs, rev, s);
    case GLX_UINT8: return launch_batch_op<uint8_t>(op, specs, rev, s);
    case GLX_INT32: return launch_batch_op<int32_t>(op, specs, rev, s);
    case GLX_INT64: return launch_batch_op<int64_t>(op, specs, rev, s);
    case GLX_UINT64: return launch_batch_op<uint64_t>(op, specs, rev, s);
    case GLX_FLOAT32: return launch_batch_op<float>(op, specs, rev, s);
    case GLX_FLOAT64: return launch_batch_op<double>(op, specs, rev, s);
    case GLX_FLOAT16: return launch_batch_op<f16_t>(op, specs, rev, s);
    case GLX_BFLOAT16: return launch_batch_op<bf16_t>(op, specs, rev, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_reduce_n(int op, int dtype, void* dst, const void* const* srcs,
                           int k, size_t n, hipStream_t s, bool rev) {
  if (n == 0) return hipSuccess;
  switch (dtype) {
    case GLX_INT8: return launch_n_op<int8_t>(op, dst, srcs, k, n, s, rev);
    case GLX_UINT8: return launch_n_op<uint8_t>(op, dst, srcs, k, n, s, rev);
    case GLX_INT32: return launch_n_op<int32_t>(op, dst, srcs, k, n, s, rev);
    case GLX_INT64: return launch_n_op<int64_t>(op, dst, srcs, k, n, s, rev);
    case GLX_UINT64: return launch_n_op<uint64_t>(op, dst, srcs, k, n, s, rev);
    case GLX_FLOAT32: return launch_n_op<float>(op, dst, srcs, k, n, s, rev);
    case GLX_FLOAT64: return launch_n_op<double>(op, dst, srcs, k, n, s, rev);
    case GLX_FLOAT16: return launch_n_op<f16_t>(op, dst, srcs, k, n, s, rev);
    case GLX_BFLOAT16: return launch_n_op<bf16_t>(op, dst, srcs, k, n, s, rev);
  }
  return hipErrorInvalidValue;
}

size_t reduce_segment_bytes() { return kSegBytes; }

void set_reduce_tuning(int unroll, int blocks_per_cu, int nontemporal) {
  if (unroll == 1 || unroll == 2 || unroll == 4 || unroll == 8) {
    g_unroll.store(unroll, std::memory_order_relaxed);
  }
  if (blocks_per_cu > 0) g_blocks_per_cu.store(blocks_per_cu, std::memory_order_relaxed);
  if (nontemporal >= 0 && nontemporal <= kPolAuto) {
    g_policy.store(nontemporal, std::memory_order_relaxed);
  }
}

void reduce_tuning(int* unroll, int* blocks_per_cu, int* policy) {
  *unroll = g_unroll.load(std::memory_order_relaxed);
  *blocks_per_cu = g_blocks_per_cu.load(std::memory_order_relaxed);
  *policy = g_policy.load(std::memory_order_relaxed);
}

}  // namespace glx
