// gloo/hip_allreduce.h -- gloo_amd's MI355X allreduce behind the reference's
// own Algorithm surface.  A gloo maintainer drops this header into the gloo
// tree (next to gloo/cuda_allreduce_ring_chunked.h) and links
// -lgloo_amd -lamdhip64; callers keep gloo's types, macros and exceptions.
//
//   HipAllreduceRingChunked<T>     ~ CudaAllreduceRingChunked<T>
//                                    (gloo/cuda_allreduce_ring_chunked.h:22-26)
//   HipAllreduceHalvingDoubling<T> ~ CudaAllreduceHalvingDoubling<T>
//                                    (gloo/cuda_allreduce_halving_doubling.h:25-30)
//
// Both take the reference's gloo::Context, the device pointers of this rank,
// the element count, optional streams (outputs valid once streams[0] reaches
// the end of run(); without streams, when run() returns -- docs/cuda.md:9-11)
// and a gloo::ReductionFunction<T> accepted by its type() (SUM, PRODUCT, MAX,
// MIN; the reference's accelerated paths do the same, gloo/algorithm.h:40-48:
// a CUSTOM function cannot run on the device and is refused).
//
// The one addition to the CUDA constructors is the rendezvous::Store the
// gloo context was connected with: the xGMI transport publishes its device
// endpoints (IPC handles of receive regions, flag rows) through it.  It must
// outlive the algorithms' first run().  The first algorithm created on a gloo
// context sets up one xGMI context for it (all ranks create algorithms in the
// same order, as gloo requires); later ones share it.
//
// Failures map onto gloo's own exceptions: timeouts and lost peers throw
// gloo::IoException (GLOO_THROW_IO_EXCEPTION, gloo/common/error.h:50),
// everything else gloo::EnforceNotMet (GLOO_ENFORCE_EQ,
// gloo/common/logging.h:149).
#pragma once

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "gloo/algorithm.h"
#include "gloo/common/error.h"
#include "gloo/common/logging.h"
#include "gloo/context.h"
#include "gloo/rendezvous/store.h"
#include "gloo/types.h"
#include "gloo_amd/glx.h"

namespace gloo {
namespace hip {

template <typename T> struct GlxType;
template <> struct GlxType<int8_t> { static constexpr int value = GLX_INT8; };
template <> struct GlxType<uint8_t> { static constexpr int value = GLX_UINT8; };
template <> struct GlxType<int32_t> { static constexpr int value = GLX_INT32; };
template <> struct GlxType<int64_t> { static constexpr int value = GLX_INT64; };
template <> struct GlxType<uint64_t> { static constexpr int value = GLX_UINT64; };
template <> struct GlxType<float> { static constexpr int value = GLX_FLOAT32; };
template <> struct GlxType<double> { static constexpr int value = GLX_FLOAT64; };
template <> struct GlxType<float16> { static constexpr int value = GLX_FLOAT16; };

// gloo::ReductionType -> glx_op (the codes are the same by construction)
template <typename T>
int glxOp(const ReductionFunction<T>* fn) {
  GLOO_ENFORCE(fn != nullptr, "null reduction function");
  const ReductionType t = fn->type();
  GLOO_ENFORCE(t == SUM || t == PRODUCT || t == MAX || t == MIN,
               "HIP allreduce: reduction type ", (int)t,
               " has no device implementation (SUM, PRODUCT, MAX and MIN do)");
  return (int)t;
}

inline void check(int rc, const char* what) {
  if (rc == GLX_OK) return;
  if (rc == GLX_ERR_TIMEOUT || rc == GLX_ERR_IO) {
    GLOO_THROW_IO_EXCEPTION(what, ": ", glx_last_error());
  }
  GLOO_ENFORCE_EQ(rc, GLX_OK, what, ": ", glx_last_error());
}

// A gloo rendezvous::Store seen through the glx callback store, keys under
// `prefix`.  get is a non-blocking probe (-1 if the key is absent): the
// Store interface has no probe, so a 1 ms wait stands in for one.
class StoreBridge {
 public:
  StoreBridge(rendezvous::Store& store, std::string prefix)
      : store_(store), prefix_(std::move(prefix)) {
    handle_ = glx_callback_store_create(&StoreBridge::set, &StoreBridge::get, this);
    GLOO_ENFORCE(handle_ != nullptr, "glx_callback_store_create failed");
  }
  ~StoreBridge() { glx_store_destroy(handle_); }
  StoreBridge(const StoreBridge&) = delete;
  StoreBridge& operator=(const StoreBridge&) = delete;
  glx_store* handle() const { return handle_; }

 private:
  static int set(void* user, const char* key, const void* data, size_t len) {
    auto* self = static_cast<StoreBridge*>(user);
    try {
      const char* d = static_cast<const char*>(data);
      self->store_.set(self->prefix_ + key, std::vector<char>(d, d + len));
      return 0;
    } catch (const std::exception&) {
      return 1;
    }
  }
  static int64_t get(void* user, const char* key, void* buf, size_t cap) {
    auto* self = static_cast<StoreBridge*>(user);
    const std::string k = self->prefix_ + key;
    try {
      self->store_.wait({k}, std::chrono::milliseconds(1));
    } catch (const std::exception&) {
      return -1;  // not there yet
    }
    try {
      const std::vector<char> v = self->store_.get(k);
      std::memcpy(buf, v.data(), std::min(cap, v.size()));
      return (int64_t)v.size();
    } catch (const std::exception&) {
      return -1;
    }
  }

  rendezvous::Store& store_;
  const std::string prefix_;
  glx_store* handle_ = nullptr;
};

// One xGMI context per gloo context, shared by the algorithms made on it.
class XgmiContext {
 public:
  static std::shared_ptr<XgmiContext> of(const std::shared_ptr<Context>& ctx,
                                         rendezvous::Store& store, int device) {
    static std::mutex m;
    static std::map<const Context*, std::weak_ptr<XgmiContext>> all;
    {
      std::lock_guard<std::mutex> g(m);
      auto it = all.find(ctx.get());
      if (it != all.end()) {
        if (auto live = it->second.lock()) return live;
      }
    }
    // Connect without the registry lock: connecting waits for the peers,
    // which may be threads of this process making their own contexts (a gloo
    // context is used by one thread at a time, so nobody races for this key).
    // The slot is the same on every rank: gloo contexts hand them out in
    // algorithm-creation order (gloo/context.cc:49-54).
    const int slot = ctx->nextSlot();
    std::shared_ptr<XgmiContext> x(
        new XgmiContext(ctx, store, device, "gloo_amd/" + std::to_string(slot) + "/"));
    std::lock_guard<std::mutex> g(m);
    all[ctx.get()] = x;
    return x;
  }
  ~XgmiContext() { glx_context_destroy(glx_); }
  glx_context* get() const { return glx_; }

 private:
  XgmiContext(const std::shared_ptr<Context>& ctx, rendezvous::Store& store, int device,
              const std::string& prefix)
      : bridge_(store, prefix) {
    glx_ = glx_context_create(ctx->rank, ctx->size, device);
    GLOO_ENFORCE(glx_ != nullptr, "glx_context_create: ", glx_last_error());
    check(glx_context_set_timeout(glx_, (int64_t)ctx->getTimeout().count()),
          "glx_context_set_timeout");
    check(glx_context_connect_full_mesh(glx_, bridge_.handle()),
          "glx_context_connect_full_mesh");
  }
  StoreBridge bridge_;
  glx_context* glx_ = nullptr;
};

// The HIP device of a device pointer (the CUDA algorithms infer it likewise).
inline int deviceOf(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) == hipSuccess && a.type == hipMemoryTypeDevice) {
    return a.device;
  }
  (void)hipGetLastError();
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

template <typename T>
class Allreduce : public Algorithm {
 public:
  void run() override { check(glx_algorithm_run(alg_), "run"); }
  ~Allreduce() override { glx_algorithm_destroy(alg_); }
  // bytes moved over the peer links per run (introspection)
  int64_t bytesSent() const { return glx_algorithm_bytes_sent(alg_); }

 protected:
  Allreduce(int algo, const std::shared_ptr<Context>& context, rendezvous::Store& store,
            const std::vector<T*>& ptrs, int count, const std::vector<hipStream_t>& streams,
            const ReductionFunction<T>* fn)
      : Algorithm(context) {
    GLOO_ENFORCE(!ptrs.empty(), "at least one pointer is required");
    xgmi_ = XgmiContext::of(context, store, deviceOf(ptrs[0]));
    std::vector<void*> p(ptrs.begin(), ptrs.end());
    std::vector<glx_stream_t> s(streams.begin(), streams.end());
    alg_ = glx_allreduce_create(xgmi_->get(), algo, p.data(), (int)p.size(), count,
                                GlxType<T>::value, glxOp(fn), s.empty() ? nullptr : s.data(),
                                (int)s.size());
    GLOO_ENFORCE(alg_ != nullptr, "glx_allreduce_create: ", glx_last_error());
  }

 private:
  std::shared_ptr<XgmiContext> xgmi_;
  glx_algorithm* alg_ = nullptr;
};

}  // namespace hip

template <typename T>
class HipAllreduceRingChunked : public hip::Allreduce<T> {
 public:
  HipAllreduceRingChunked(const std::shared_ptr<Context>& context, rendezvous::Store& store,
                          const std::vector<T*>& ptrs, int count,
                          const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                          const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_RING_CHUNKED, context, store, ptrs, count, streams, fn) {}
};

template <typename T>
class HipAllreduceHalvingDoubling : public hip::Allreduce<T> {
 public:
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& context, rendezvous::Store& store,
                              const std::vector<T*>& ptrs, int count,
                              const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                              const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_HALVING_DOUBLING, context, store, ptrs, count, streams,
                          fn) {}
};

}  // namespace gloo
