// common.h -- error conventions of gloo_amd.
//
// Inside the library errors are C++ exceptions carrying gloo's own names:
//   EnforceNotMet  -- GLOO_ENFORCE* failures   (gloo/common/logging.h:21-52)
//   IoException    -- timeouts, peer loss       (gloo/common/error.h:45)
//   HipError       -- a failed HIP call (the CUDA_CHECK analog,
//                     gloo/cuda_private.h:25-37)
// The C ABI (capi.cc) catches them and returns GLX_ERR_* codes plus a
// thread-local message; Python re-raises the same exception names.
#pragma once

#include <hip/hip_runtime_api.h>

#include <sstream>
#include <stdexcept>
#include <string>

#include "../../include/gloo_amd/glx.h"

namespace gloo {

struct Exception : public std::runtime_error {
  explicit Exception(const std::string& msg) : std::runtime_error(msg) {}
};

struct EnforceNotMet : public Exception {
  explicit EnforceNotMet(const std::string& msg) : Exception(msg) {}
};

struct IoException : public Exception {
  explicit IoException(const std::string& msg) : Exception(msg) {}
};

struct TimeoutException : public IoException {
  explicit TimeoutException(const std::string& msg) : IoException(msg) {}
};

struct HipError : public Exception {
  HipError(const std::string& msg, hipError_t e) : Exception(msg), err(e) {}
  hipError_t err;
};

namespace detail {
inline void cat(std::ostringstream&) {}
template <typename T, typename... Rest>
void cat(std::ostringstream& os, const T& v, const Rest&... rest) {
  os << v;
  cat(os, rest...);
}
}  // namespace detail

template <typename... Args>
std::string MakeString(const Args&... args) {
  std::ostringstream os;
  detail::cat(os, args...);
  return os.str();
}

}  // namespace gloo

#define GLX_ENFORCE(cond, ...)                                              \
  do {                                                                      \
    if (!(cond)) {                                                          \
      throw ::gloo::EnforceNotMet(::gloo::MakeString(                       \
          __FILE__, ":", __LINE__, ": enforce fail: ", #cond, ". ",         \
          ##__VA_ARGS__));                                                  \
    }                                                                       \
  } while (0)

#define GLX_HIP_CHECK(expr)                                                 \
  do {                                                                      \
    hipError_t glx_e_ = (expr);                                             \
    if (glx_e_ != hipSuccess) {                                             \
      throw ::gloo::HipError(                                               \
          ::gloo::MakeString(__FILE__, ":", __LINE__, ": ", #expr, " -> ",  \
                             hipGetErrorName(glx_e_), ": ",                 \
                             hipGetErrorString(glx_e_)),                    \
          glx_e_);                                                          \
    }                                                                       \
  } while (0)

#define GLX_THROW_IO(...) \
  throw ::gloo::IoException(::gloo::MakeString(__VA_ARGS__))

#define GLX_THROW_TIMEOUT(...) \
  throw ::gloo::TimeoutException(::gloo::MakeString(__VA_ARGS__))
