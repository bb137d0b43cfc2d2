// host_ops.h -- the local multi-pointer reduce and broadcast on HOST memory:
// the analog of the reference's cudaHostReduce / cudaHostBroadcast, which its
// GPU algorithms use instead of the device ops below kOnDeviceThreshold
// (gloo/algorithm.cc:16; gloo/cuda_allreduce_halving_doubling.cc:478,538,585).
// Here: algorithms whose buffers are in host memory, with several pointers,
// fold them on the host when the buffer is smaller than kOnDeviceThreshold
// and stage ONE buffer through the device (instead of one H2D per pointer
// plus a fold kernel), then broadcast the result to the pointers on the host.
//
// Semantics are the reference's gloo/math.h in place, bit for bit, as the
// device kernels' (elem_ops.h): sum(T* a, const T* b, n) with its float16
// rounding and assignment rule (gloo/types.h:129-147, 181-204, 251-305).
#pragma once

#include <stddef.h>

namespace glx {

// gloo/algorithm.cc:16
constexpr size_t kOnDeviceThreshold = 256 * 1024;

// dst = ((srcs[0] op srcs[1]) op srcs[2]) ... over n elements (the local
// left fold, gloo/allreduce_ring_chunked.h:89-91); dst may be srcs[0].
void host_reduce_n(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n);

}  // namespace glx
