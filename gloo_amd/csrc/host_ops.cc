// host_ops.cc -- see host_ops.h.
#include "host_ops.h"

#include <stdint.h>

#include <cstring>
#include <type_traits>

#include "common.h"

namespace glx {
namespace {

float bitsToFloat(uint32_t u) {
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

uint32_t floatToBits(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return u;
}

// IEEE binary16 -> binary32, exact (NaN payloads do not matter: every NaN
// narrows back to 0x7fff and compares unordered).
float halfToFloat(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  uint32_t exp = (h >> 10) & 0x1fu, man = h & 0x3ffu;
  if (exp == 0x1fu) return bitsToFloat(sign | 0x7f800000u | (man << 13));
  if (exp == 0) {
    if (man == 0) return bitsToFloat(sign);
    // subnormal: value = man * 2^-24
    const float v = (float)man * 5.9604644775390625e-8f;
    return sign ? -v : v;
  }
  return bitsToFloat(sign | ((exp + 112u) << 23) | (man << 13));
}

// binary32 -> binary16, round to nearest even, overflow to inf, NaN -> 0x7fff
// (cpu_float2half_rn, gloo/types.h:251-305).
uint16_t floatToHalf(float f) {
  const uint32_t x = floatToBits(f);
  const uint32_t u = x & 0x7fffffffu, sign = (x >> 16) & 0x8000u;
  if (u > 0x7f800000u) return 0x7fff;
  if (u >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds past 65504
  if (u < 0x33000001u) return (uint16_t)sign;               // below half the least subnormal
  uint32_t exp = u >> 23, man = u & 0x7fffffu, shift;
  if (exp > 112) {  // normal half
    shift = 13;
    exp -= 112;
  } else {          // subnormal half: the implicit bit joins the mantissa
    shift = 126 - exp;
    exp = 0;
    man |= 0x800000u;
  }
  const uint32_t half = 1u << (shift - 1), rest = man & ((1u << shift) - 1);
  man >>= shift;
  if (rest > half || (rest == half && (man & 1u))) {
    if ((++man & 0x3ffu) == 0 && exp != 0) {  // mantissa carried into the exponent
      exp++;
      man = 0;
    }
  }
  return (uint16_t)(sign | (exp << 10) | man);
}

float bf16ToFloat(uint16_t h) { return bitsToFloat((uint32_t)h << 16); }

uint16_t floatToBf16(float f) {
  const uint32_t u = floatToBits(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return 0x7fff;
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

// float16 assignment: the store is skipped when the new bits equal
// half((float)old_bits) (gloo/types.h:129-142: operator!= converts the old
// bits, read as an integer, to a half).
uint16_t f16Assign(uint16_t old, uint16_t v) {
  return v == floatToHalf((float)old) ? old : v;
}

template <typename T>
struct Wide {
  using U = typename std::make_unsigned<T>::type;
};

template <typename T>
T intOp(int op, T a, T b) {
  using U = typename std::make_unsigned<T>::type;
  switch (op) {
    case GLX_SUM: return (T)((U)a + (U)b);
    case GLX_PRODUCT: return (T)((U)a * (U)b);
    case GLX_MAX: return (a < b) ? b : a;
    default: return (b < a) ? b : a;
  }
}

template <typename T>
T floatOp(int op, T a, T b) {
  switch (op) {
    case GLX_SUM: return a + b;
    case GLX_PRODUCT: return a * b;
    case GLX_MAX: return (a < b) ? b : a;
    default: return (b < a) ? b : a;
  }
}

// a = a op b for 16-bit floats carried as bits (max/min return an operand)
template <bool BF16>
uint16_t halfOp(int op, uint16_t a, uint16_t b) {
  const float x = BF16 ? bf16ToFloat(a) : halfToFloat(a);
  const float y = BF16 ? bf16ToFloat(b) : halfToFloat(b);
  uint16_t v;
  switch (op) {
    case GLX_SUM: v = BF16 ? floatToBf16(x + y) : floatToHalf(x + y); break;
    case GLX_PRODUCT: v = BF16 ? floatToBf16(x * y) : floatToHalf(x * y); break;
    case GLX_MAX: v = (x < y) ? b : a; break;
    default: v = (y < x) ? b : a; break;
  }
  return BF16 ? v : f16Assign(a, v);  // in place: a is the old value
}

template <typename S, typename F>
void fold(S* dst, const void* const* srcs, int k, size_t n, F f) {
  const S* s0 = static_cast<const S*>(srcs[0]);
  if (dst != s0) std::memcpy(dst, s0, n * sizeof(S));
  for (int j = 1; j < k; j++) {
    const S* b = static_cast<const S*>(srcs[j]);
    for (size_t i = 0; i < n; i++) dst[i] = f(dst[i], b[i]);
  }
}

}  // namespace

void host_reduce_n(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n) {
  GLX_ENFORCE(k >= 1 && srcs != nullptr && dst != nullptr, "host_reduce_n: bad arguments");
  GLX_ENFORCE(op >= GLX_SUM && op <= GLX_MIN, "host_reduce_n: unknown op ", op);
  switch (dtype) {
#define GLX_HOST_INT(CODE, T) \
  case CODE: fold<T>(static_cast<T*>(dst), srcs, k, n, [op](T a, T b) { return intOp<T>(op, a, b); }); return;
    GLX_HOST_INT(GLX_INT8, int8_t)
    GLX_HOST_INT(GLX_UINT8, uint8_t)
    GLX_HOST_INT(GLX_INT32, int32_t)
    GLX_HOST_INT(GLX_INT64, int64_t)
    GLX_HOST_INT(GLX_UINT64, uint64_t)
#undef GLX_HOST_INT
    case GLX_FLOAT32:
      fold<float>(static_cast<float*>(dst), srcs, k, n,
                  [op](float a, float b) { return floatOp<float>(op, a, b); });
      return;
    case GLX_FLOAT64:
      fold<double>(static_cast<double*>(dst), srcs, k, n,
                   [op](double a, double b) { return floatOp<double>(op, a, b); });
      return;
    case GLX_FLOAT16:
      fold<uint16_t>(static_cast<uint16_t*>(dst), srcs, k, n,
                     [op](uint16_t a, uint16_t b) { return halfOp<false>(op, a, b); });
      return;
    case GLX_BFLOAT16:
      fold<uint16_t>(static_cast<uint16_t*>(dst), srcs, k, n,
                     [op](uint16_t a, uint16_t b) { return halfOp<true>(op, a, b); });
      return;
  }
  GLX_ENFORCE(false, "host_reduce_n: unknown dtype ", dtype);
}

}  // namespace glx
