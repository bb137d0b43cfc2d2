// elem_ops.h -- device-side element operations shared by the HIP kernels
// (reduce_kernels.hip, xgmi_kernels.hip): the reference CPU path's
// semantics, bit for bit (see reduce_kernels.hip's header for the rules).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "common.h"
#include "kernels.h"

namespace glx {
namespace {

constexpr int kBlock = 256;

// 16-byte vector as a native clang vector (one global_load/store_dwordx4).
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// Streaming loads/stores; NT = nontemporal hint (the data is touched once).
template <bool NT>
__device__ __forceinline__ v4u ld16(const v4u* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st16(v4u* p, v4u v) {
  if (NT) {
    __builtin_nontemporal_store(v, p);
  } else {
    *p = v;
  }
}

// Write-through stores (`sc1`): the line leaves this XCD's L2 with the store
// instead of staying dirty there until an eviction writes it back; for a
// stream written once that fits the Infinity Cache this is the fastest store
// (tools/tune_policy.py; profiles/r4j_*, r4k_*).  HIP has no global
// store builtin with that cache policy, so the stream is written through a
// buffer resource over its base (a compiler builtin, not inline asm: the
// compiler then tracks the store for waitcnts and register hazards).
// Offsets are 32-bit: a stream must stay below 2 GiB (kWtMaxStream,
// kernels.h; the executors enforce it for every workgroup span).
// p as the compiler can prove wave-uniform (callers pass one value to every
// lane), so a buffer resource over it stays in SGPRs.
__device__ __forceinline__ void* uniform_ptr(void* p) {
  const uint64_t u = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
}
struct WtStream {
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ explicit WtStream(void* base)
      // raw buffer, no stride, every byte below 2 GiB in range; dword3 of
      // the descriptor as every gfx9-family part takes it
      : r(__builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000)) {}
  // 16-byte vector i of the stream; cache policy 16 = sc1 (gfx940 family)
  __device__ __forceinline__ void put(size_t i, v4u v) const {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(i * 16), 0, 16);
  }
};

// Cache policy of a streaming kernel's loads and stores.
enum StreamPolicy : int {
  kPolPlain = 0,    // plain loads, plain stores
  kPolNt = 1,       // nontemporal loads and stores
  kPolNtWt = 2,     // nontemporal loads, write-through stores
  kPolNtPlain = 3,  // nontemporal loads, plain stores
};

template <int POL>
__device__ __forceinline__ v4u ld16p(const v4u* p) {
  return ld16<POL != kPolPlain>(p);
}


// ---- scalar element ops on storage types ---------------------------------

__device__ __forceinline__ float h2f(uint16_t h) {
  return __half2float(__ushort_as_half(h));  // v_cvt_f32_f16: exact
}

__device__ __forceinline__ uint16_t f2h(float f) {
  // v_cvt_f16_f32 rounds to nearest even (default mode) with IEEE
  // subnormals and overflow to inf; only the NaN encoding needs fixing.
  // Issued as inline asm so the compiler cannot fold widen->op->narrow into
  // a mixed-precision FMA (it lowers fptrunc(a*b) to v_fma_mixlo_f16 a,b,+0,
  // which turns a -0 product into +0).
  uint32_t r;
  asm("v_cvt_f16_f32_e32 %0, %1" : "=v"(r) : "v"(f));
  return (f != f) ? (uint16_t)0x7fff : (uint16_t)(r & 0xffffu);
}

__device__ __forceinline__ float b2f(uint16_t h) {
  return __uint_as_float((uint32_t)h << 16);
}

__device__ __forceinline__ uint16_t f2b(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fff;
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

template <typename T, int OP>
struct Op;

// Integers: sum/product computed in the unsigned type of the same width so
// wrap-around is defined (the reference's signed overflow is UB; gcc wraps).
template <typename T> struct UnsignedOf { using type = T; };
template <> struct UnsignedOf<int8_t> { using type = uint8_t; };
template <> struct UnsignedOf<int32_t> { using type = uint32_t; };
template <> struct UnsignedOf<int64_t> { using type = uint64_t; };

template <typename T>
struct Op<T, GLX_SUM> {
  static __device__ __forceinline__ T apply(T a, T b) {
    using U = typename UnsignedOf<T>::type;
    return (T)((U)a + (U)b);
  }
};
template <typename T>
struct Op<T, GLX_PRODUCT> {
  static __device__ __forceinline__ T apply(T a, T b) {
    using U = typename UnsignedOf<T>::type;
    return (T)((U)a * (U)b);
  }
};
template <typename T>
struct Op<T, GLX_MAX> {
  static __device__ __forceinline__ T apply(T a, T b) { return (a < b) ? b : a; }
};
template <typename T>
struct Op<T, GLX_MIN> {
  static __device__ __forceinline__ T apply(T a, T b) { return (b < a) ? b : a; }
};

template <>
struct Op<float, GLX_SUM> {
  static __device__ __forceinline__ float apply(float a, float b) {
    return __fadd_rn(a, b);  // never contracted into an fma
  }
};
template <>
struct Op<float, GLX_PRODUCT> {
  static __device__ __forceinline__ float apply(float a, float b) {
    return __fmul_rn(a, b);
  }
};
template <>
struct Op<double, GLX_SUM> {
  static __device__ __forceinline__ double apply(double a, double b) {
    return __dadd_rn(a, b);
  }
};
template <>
struct Op<double, GLX_PRODUCT> {
  static __device__ __forceinline__ double apply(double a, double b) {
    return __dmul_rn(a, b);
  }
};

// 16-bit floats are carried as their raw bits in these tag types.
struct f16_t { uint16_t x; };
struct bf16_t { uint16_t x; };

template <typename H> struct HalfTraits;
template <> struct HalfTraits<f16_t> {
  static __device__ __forceinline__ float widen(uint16_t h) { return h2f(h); }
  static __device__ __forceinline__ uint16_t narrow(float f) { return f2h(f); }
};
template <> struct HalfTraits<bf16_t> {
  static __device__ __forceinline__ float widen(uint16_t h) { return b2f(h); }
  static __device__ __forceinline__ uint16_t narrow(float f) { return f2b(f); }
};

template <typename H, int OP>
struct HalfOp {
  static __device__ __forceinline__ uint16_t apply(uint16_t a, uint16_t b) {
    using Tr = HalfTraits<H>;
    float x = Tr::widen(a), y = Tr::widen(b);
    if (OP == GLX_SUM) return Tr::narrow(__fadd_rn(x, y));
    if (OP == GLX_PRODUCT) return Tr::narrow(__fmul_rn(x, y));
    if (OP == GLX_MAX) return (x < y) ? b : a;
    return (y < x) ? b : a;  // GLX_MIN
  }
};

// The reference's float16 assignment (gloo/types.h:129-147): `old = v` is
// skipped when v.x == half((float)old.x) -- operator!= compares against the
// old bits read as an integer.  Restated so fp16 results stay bit-exact.
__device__ __forceinline__ uint16_t f16_assign(uint16_t old, uint16_t v) {
  // (float)old is an integer 0..65535, never NaN: the bare conversion suffices
  uint32_t g;
  asm("v_cvt_f16_f32_e32 %0, %1" : "=v"(g) : "v"((float)(uint32_t)old));
  return (v == (uint16_t)(g & 0xffffu)) ? old : v;
}

// Storage type and element op for a tag type.  apply3(old, a, b) is the value
// c[i] ends up with when c[i] held `old` (c == a in place: old == a).
template <typename T, int OP> struct Elem {
  using S = T;
  static __device__ __forceinline__ S apply(S a, S b) { return Op<T, OP>::apply(a, b); }
  static __device__ __forceinline__ S apply3(S, S a, S b) { return apply(a, b); }
};
template <int OP> struct Elem<f16_t, OP> {
  using S = uint16_t;
  static __device__ __forceinline__ S apply3(S old, S a, S b) {
    S v = HalfOp<f16_t, OP>::apply(a, b);
    if (OP == GLX_SUM || OP == GLX_PRODUCT) v = f16_assign(a, v);  // inside operator+=
    return f16_assign(old, v);                                        // c[i] = ...
  }
  // In place (c == a): the assignment at `c[i] = ...` repeats the one inside
  // operator+=/*= with the same old value, which cannot change the result
  // (if the first kept `a`, the second keeps it too), so one suffices.
  static __device__ __forceinline__ S apply(S a, S b) {
    return f16_assign(a, HalfOp<f16_t, OP>::apply(a, b));
  }
};
template <int OP> struct Elem<bf16_t, OP> {
  using S = uint16_t;
  static __device__ __forceinline__ S apply(S a, S b) { return HalfOp<bf16_t, OP>::apply(a, b); }
  static __device__ __forceinline__ S apply3(S, S a, S b) { return apply(a, b); }
};

// ---- 16-byte vector op ----------------------------------------------------

template <typename T, int OP>
__device__ __forceinline__ v4u vec_apply3(v4u vo, v4u va, v4u vb) {
  using E = Elem<T, OP>;
  using S = typename E::S;
  constexpr int V = 16 / sizeof(S);
  union U { v4u v; S s[V]; };
  U o, a, b, c;
  o.v = vo;
  a.v = va;
  b.v = vb;
#pragma unroll
  for (int i = 0; i < V; i++) c.s[i] = E::apply3(o.s[i], a.s[i], b.s[i]);
  return c.v;
}

template <typename T, int OP>
__device__ __forceinline__ v4u vec_apply(v4u va, v4u vb) {
  using E = Elem<T, OP>;
  using S = typename E::S;
  constexpr int V = 16 / sizeof(S);
  union U { v4u v; S s[V]; };
  U a, b, c;
  a.v = va;
  b.v = vb;
#pragma unroll
  for (int i = 0; i < V; i++) c.s[i] = E::apply(a.s[i], b.s[i]);
  return c.v;
}

}  // namespace
}  // namespace glx
