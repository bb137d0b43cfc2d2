// kernels.h -- host-side launchers of the HIP kernels (reduce_kernels.hip).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>

#include <vector>

namespace glx {

// dst = op(a, b), n elements of dtype, on stream s.  Never synchronises.
hipError_t launch_reduce(int op, int dtype, void* dst, const void* a,
                         const void* b, size_t n, hipStream_t s);

// Fold of op over srcs[0..k-1] (k >= 1): acc = srcs[0], then
// acc = op(acc, srcs[j]) (rev = false, left fold) or acc = op(srcs[j], acc)
// (rev = true, the ring's chain order).  dst may alias srcs[0].
hipError_t launch_reduce_n(int op, int dtype, void* dst, const void* const* srcs,
                           int k, size_t n, hipStream_t s, bool rev = false);

// Several independent folds (same op/dtype/order) in one launch.
struct FoldSpec {
  void* dst;
  std::vector<const void*> srcs;
  int k;
  size_t n;
};
hipError_t launch_reduce_n_batch(int op, int dtype, const std::vector<FoldSpec>& specs,
                                 hipStream_t s, bool rev);

// Byte copy dst <- src as a kernel on stream s (dst may be a peer GPU's
// IPC-mapped memory: the stores then travel over xGMI).  Never synchronises.
hipError_t launch_copy(void* dst, const void* src, size_t bytes, hipStream_t s);
// Grid (workgroups) of the copy kernel.
void set_copy_blocks(int blocks);
int copy_blocks();

// Tuning knobs of the vector kernel (lanes' unroll depth, grid cap per CU,
// nontemporal loads/stores: 0/1, -1 = keep).
void set_reduce_tuning(int unroll, int blocks_per_cu, int nontemporal);

}  // namespace glx
