// gloo_amd.hpp -- header-only C++ surface of the MI355X allreduce path, over
// the C ABI in glx.h.  It mirrors the reference's operator interface so C++
// callers of gloo's allreduce switch by changing the namespace:
//
//   gloo::rendezvous::HashStore / FileStore / PrefixStore  (gloo/rendezvous/*.h)
//   gloo::rendezvous::Context(rank, size) + connectFullMesh (gloo/rendezvous/context.h:25-35)
//   gloo::ReductionFunction<T>::sum/product/min/max         (gloo/algorithm.h:59-96)
//   gloo::Algorithm::run()                                  (gloo/algorithm.h:20-38)
//   gloo::CudaAllreduceRingChunked<T>(ctx, ptrs, count, streams)
//                                      (gloo/cuda_allreduce_ring_chunked.h:22-26)
//   gloo::CudaAllreduceHalvingDoubling<T>(ctx, ptrs, count, streams)
//                                      (gloo/cuda_allreduce_halving_doubling.h:25-30)
//   gloo::AllreduceOptions + gloo::allreduce(opts)          (gloo/allreduce.h:89-195)
//   gloo::EnforceNotMet, gloo::IoException                  (gloo/common/logging.h:21,
//                                                            gloo/common/error.h:45)
// become gloo_amd::<same name> (device algorithms: HipAllreduceRingChunked<T>,
// HipAllreduceHalvingDoubling<T>).  Link with -lgloo_amd.
#pragma once

#include <chrono>
#include <cstdint>
#include <algorithm>
#include <exception>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "glx.h"

namespace gloo_amd {

struct Exception : public std::runtime_error {
  explicit Exception(const std::string& m) : std::runtime_error(m) {}
};
struct EnforceNotMet : public Exception {
  explicit EnforceNotMet(const std::string& m) : Exception(m) {}
};
struct IoException : public Exception {
  explicit IoException(const std::string& m) : Exception(m) {}
};
struct HipError : public Exception {
  explicit HipError(const std::string& m) : Exception(m) {}
};

inline void check(int rc, const char* what) {
  if (rc == GLX_OK) return;
  std::string m = std::string(what) + ": " + glx_last_error();
  switch (rc) {
    case GLX_ERR_TIMEOUT:
    case GLX_ERR_IO:
      throw IoException(m);
    case GLX_ERR_HIP:
      throw HipError(m);
    case GLX_ERR_INVALID:
    case GLX_ERR_ENFORCE:
      throw EnforceNotMet(m);
    default:
      throw Exception(m);
  }
}

template <typename P>
P* checkHandle(P* p, const char* what) {
  if (p == nullptr) {
    std::string m = std::string(what) + ": " + glx_last_error();
    if (m.find("Timed out") != std::string::npos) throw IoException(m);
    throw EnforceNotMet(m);
  }
  return p;
}

// 16-bit float element types (raw bits), layout-compatible with gloo::float16.
struct float16 {
  uint16_t x;
};
struct bfloat16 {
  uint16_t x;
};

template <typename T>
struct DType;
template <> struct DType<int8_t> { static constexpr int value = GLX_INT8; };
template <> struct DType<uint8_t> { static constexpr int value = GLX_UINT8; };
template <> struct DType<int32_t> { static constexpr int value = GLX_INT32; };
template <> struct DType<int64_t> { static constexpr int value = GLX_INT64; };
template <> struct DType<uint64_t> { static constexpr int value = GLX_UINT64; };
template <> struct DType<float> { static constexpr int value = GLX_FLOAT32; };
template <> struct DType<double> { static constexpr int value = GLX_FLOAT64; };
template <> struct DType<float16> { static constexpr int value = GLX_FLOAT16; };
template <> struct DType<bfloat16> { static constexpr int value = GLX_BFLOAT16; };

// The glx dtype of T, or -1 for an element type the device ops do not have
// (a caller's host Func takes any T, as the reference's does).
template <typename T, typename = void>
struct DTypeOrNone {
  static constexpr int value = -1;
};
template <typename T>
struct DTypeOrNone<T, std::void_t<decltype(DType<T>::value)>> {
  static constexpr int value = DType<T>::value;
};

enum ReductionType {
  SUM = GLX_SUM,
  PRODUCT = GLX_PRODUCT,
  MAX = GLX_MAX,
  MIN = GLX_MIN,
  CUSTOM = 1000  // gloo/algorithm.h:56
};

// gloo::ReductionFunction<T> (gloo/algorithm.h:58-83): the device kernel is
// selected by type(); a CUSTOM one carries the caller's fn(x, y, n), x =
// f(x, y), which runs on the host -- the ring-chunked and halving-doubling
// classes then need host buffers (glx_allreduce_create_host_fn).
template <typename T>
class ReductionFunction {
 public:
  using Function = void(T*, const T*, size_t n);
  explicit ReductionFunction(ReductionType t, Function* fn = nullptr) : type_(t), fn_(fn) {
    if ((t == CUSTOM) != (fn != nullptr)) {
      throw EnforceNotMet("ReductionFunction: a function goes with CUSTOM, and only there");
    }
  }
  ReductionType type() const { return type_; }
  void call(T* x, const T* y, size_t n) const { fn_(x, y, n); }
  static const ReductionFunction<T>* sum;
  static const ReductionFunction<T>* product;
  static const ReductionFunction<T>* min;
  static const ReductionFunction<T>* max;

 private:
  ReductionType type_;
  Function* fn_;
};
template <typename T>
const ReductionFunction<T>* ReductionFunction<T>::sum = new ReductionFunction<T>(SUM);
template <typename T>
const ReductionFunction<T>* ReductionFunction<T>::product = new ReductionFunction<T>(PRODUCT);
template <typename T>
const ReductionFunction<T>* ReductionFunction<T>::min = new ReductionFunction<T>(MIN);
template <typename T>
const ReductionFunction<T>* ReductionFunction<T>::max = new ReductionFunction<T>(MAX);

namespace rendezvous {

class Store {
 public:
  explicit Store(glx_store* s) : s_(checkHandle(s, "Store")) {}
  virtual ~Store() { glx_store_destroy(s_); }
  Store(const Store&) = delete;
  Store& operator=(const Store&) = delete;
  void set(const std::string& key, const std::vector<char>& data) {
    check(glx_store_set(s_, key.c_str(), data.data(), data.size()), "Store::set");
  }
  std::vector<char> get(const std::string& key,
                        std::chrono::milliseconds timeout = std::chrono::seconds(30)) {
    size_t n = 0;
    check(glx_store_get(s_, key.c_str(), nullptr, 0, &n, timeout.count()), "Store::get");
    std::vector<char> v(n);
    check(glx_store_get(s_, key.c_str(), v.data(), v.size(), &n, timeout.count()),
          "Store::get");
    return v;
  }
  glx_store* handle() const { return s_; }

 private:
  glx_store* s_;
};

class HashStore : public Store {
 public:
  HashStore() : Store(glx_hash_store_create()) {}
};

class FileStore : public Store {
 public:
  explicit FileStore(const std::string& path) : Store(glx_file_store_create(path.c_str())) {}
};

class PrefixStore : public Store {
 public:
  PrefixStore(const std::string& prefix, Store& base)
      : Store(glx_prefix_store_create(prefix.c_str(), base.handle())) {}
};

// gloo::rendezvous::Context bound to one HIP device.
class Context {
 public:
  Context(int rank, int size, int device = -1)
      : c_(checkHandle(glx_context_create(rank, size, device), "Context")),
        rank(rank),
        size(size) {}
  ~Context() { glx_context_destroy(c_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;

  void connectFullMesh(Store& store) {
    check(glx_context_connect_full_mesh(c_, store.handle()), "connectFullMesh");
  }
  void setTimeout(std::chrono::milliseconds t) {
    check(glx_context_set_timeout(c_, t.count()), "setTimeout");
  }
  std::chrono::milliseconds getTimeout() const {
    return std::chrono::milliseconds(glx_context_get_timeout(c_));
  }
  int nextSlot(int numToSkip = 1) { return glx_context_next_slot(c_, numToSkip); }
  // gloo::Context::base (gloo/context.h:33): HipAllreduceBcube's group size
  void setBase(int b) {
    check(glx_context_set_base(c_, b), "setBase");
    base_ = b;
  }
  int base() const { return base_; }
  glx_context* handle() const { return c_; }

 private:
  glx_context* c_;
  int base_ = 2;

 public:
  const int rank;
  const int size;
};

}  // namespace rendezvous

using Context = rendezvous::Context;

// gloo::Algorithm (gloo/algorithm.h:19-38): the algorithm keeps its context
// and the caller's rank/size.  There are no transport pairs (peers are
// reached through their IPC-mapped memory), so the ring helpers
// getLeftPair()/getRightPair() become the ranks they would connect to.
class Algorithm {
 public:
  explicit Algorithm(const std::shared_ptr<Context>& context)
      : context_(context), contextRank_(context->rank), contextSize_(context->size) {}
  virtual ~Algorithm() = default;
  virtual void run() = 0;

 protected:
  std::shared_ptr<Context> context_;
  const int contextRank_;
  const int contextSize_;

  int getLeftRank() const { return (contextSize_ + contextRank_ - 1) % contextSize_; }
  int getRightRank() const { return (contextRank_ + 1) % contextSize_; }
};

// A HIP event (gloo::CudaStream's record / wait, gloo/cuda.h:40-120).
class Event {
 public:
  Event() { check(glx_event_create(&e_), "Event"); }
  ~Event() { glx_event_destroy(e_); }
  Event(const Event&) = delete;
  Event& operator=(const Event&) = delete;
  void record(glx_stream_t stream) { check(glx_event_record(e_, stream), "Event::record"); }
  // true once everything recorded before it has completed
  bool query() {
    const int rc = glx_event_query(e_);
    if (rc == GLX_NOT_READY) return false;
    check(rc, "Event::query");
    return true;
  }
  // stream waits on the device; nullptr: the calling thread blocks
  void wait(glx_stream_t stream = nullptr) { check(glx_event_wait(e_, stream), "Event::wait"); }
  glx_event_t handle() const { return e_; }

 private:
  glx_event_t e_ = nullptr;
};

// How an algorithm's messages moved (glx_algorithm_transport_stats).
struct TransportStats {
  int64_t peerCopies, deviceCopies, kernelCopies, deviceKernels, bytes, hostFolds, doneEvents,
      flagKernels;
};

namespace detail {
template <typename T>
class DeviceAllreduce : public Algorithm {
 protected:
  using Create = glx_algorithm* (*)(glx_context*, void* const*, int, int, int, int,
                                    const glx_stream_t*, int);
  // customAlgo: the glx algorithm a CUSTOM function runs as on host buffers
  // (GLX_ALGO_RING_CHUNKED / _HALVING_DOUBLING; -1: refused)
  DeviceAllreduce(Create create, const std::shared_ptr<Context>& ctx,
                  const std::vector<T*>& ptrs, int count,
                  const std::vector<glx_stream_t>& streams, const ReductionFunction<T>* fn,
                  int customAlgo = -1)
      : Algorithm(ctx) {
    std::vector<void*> p(ptrs.begin(), ptrs.end());
    if (fn == nullptr) throw EnforceNotMet("allreduce: null reduction function");
    if (fn->type() == CUSTOM) {
      if (customAlgo < 0) {
        throw EnforceNotMet("a CUSTOM reduction function runs with HipAllreduceRingChunked or "
                            "HipAllreduceHalvingDoubling on host buffers");
      }
      if (!streams.empty()) {
        throw EnforceNotMet("a CUSTOM reduction function runs on the host: no streams");
      }
      custom_.reset(new CustomCall{fn, nullptr});
      a_ = checkHandle(glx_allreduce_create_host_fn(ctx->handle(), customAlgo, p.data(),
                                                    (int)p.size(), count, sizeof(T),
                                                    &CustomCall::trampoline, custom_.get()),
                       "allreduce");
      return;
    }
    a_ = checkHandle(create(ctx->handle(), p.data(), (int)p.size(), count, DType<T>::value,
                            fn->type(), streams.empty() ? nullptr : streams.data(),
                            (int)streams.size()),
                     "allreduce");
  }

 public:
  ~DeviceAllreduce() override { glx_algorithm_destroy(a_); }
  void run() override {
    const int rc = glx_algorithm_run(a_);
    if (custom_ && custom_->error) {  // the function's own exception, not a glx error
      std::exception_ptr e = custom_->error;
      custom_->error = nullptr;
      std::rethrow_exception(e);
    }
    check(rc, "run");
  }
  int64_t bytesSentPerRun() const { return glx_algorithm_bytes_sent(a_); }
  // GLX_ENGINE_STEPS / _ONESHOT / _TWOSHOT / _DEVSTEPS / _DMASTEPS (glx.h)
  int engine() const { return glx_algorithm_engine(a_); }
  // Host buffer fed from a transport: runFed() runs while feed() (any
  // thread) reports which elements have arrived; doneRanges() lists the
  // {off, len} ranges already back in host memory.
  void runFed() { check(glx_algorithm_run_fed(a_), "runFed"); }
  void feed(int64_t off, int64_t len) { check(glx_algorithm_feed(a_, off, len), "feed"); }
  std::vector<std::pair<int64_t, int64_t>> doneRanges() const {
    int64_t cap = 0;
    for (;;) {  // ranges keep completing while a run is in flight
      std::vector<int64_t> v((size_t)std::max<int64_t>(2 * cap, 2));
      const int64_t k = glx_algorithm_done_ranges(a_, v.data(), cap);
      check(k < 0 ? GLX_ERR_INVALID : GLX_OK, "doneRanges");
      if (k <= cap) {
        std::vector<std::pair<int64_t, int64_t>> out;
        for (int64_t i = 0; i < k; i++) out.emplace_back(v[2 * i], v[2 * i + 1]);
        return out;
      }
      cap = 2 * k;
    }
  }
  // record `ev` at the end of the last run's work (streams[0] with streams)
  void record(Event& ev) { check(glx_algorithm_record(a_, ev.handle()), "record"); }
  TransportStats transportStats() const {
    int64_t o[8] = {0};
    glx_algorithm_transport_stats(a_, o, 8);
    return TransportStats{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]};
  }

 private:
  // glx_reduce_fn -> the CUSTOM function: x = f(x, y) is the host program's
  // c = f(a = c, b); the first exception it throws is kept and rethrown by
  // run() (never unwound through the C ABI)
  struct CustomCall {
    const ReductionFunction<T>* fn;
    std::exception_ptr error;
    static int trampoline(void* user, void* c, const void*, const void* b, size_t n) {
      CustomCall* call = static_cast<CustomCall*>(user);
      if (call->error) return 1;
      try {
        call->fn->call(static_cast<T*>(c), static_cast<const T*>(b), n);
      } catch (...) {
        call->error = std::current_exception();
        return 1;
      }
      return 0;
    }
  };
  glx_algorithm* a_ = nullptr;
  std::unique_ptr<CustomCall> custom_;
};
}  // namespace detail

// Data movement of HipAllreduceRingChunked (results are bit-identical):
// RING = the reference's ring (one link per direction); MESH = each rank
// folds its chunk pair from every peer directly (all links at once);
// REPLICATED = one round, every rank folds everything (small buffers);
// AUTO = REPLICATED up to a threshold per rank (with the device-driven
// engines 16 MiB at P = 2, 2 MiB at P <= 4, 1 MiB above; 256 KiB without),
// MESH above.  With the ranks on distinct devices
// or processes REPLICATED and MESH run as one device-driven kernel per rank
// (one-shot / two-shot; see setMeshEngine / setDeviceEngines).
enum class Schedule { RING, MESH, REPLICATED, AUTO };

// Engine knobs for algorithms created afterwards (process-wide; every rank
// must set them alike).  mode: GLX_DEVICE_ENGINES_AUTO (one rank per GPU),
// _OFF, _ON, _SHARED (also processes sharing a GPU within the queue budget).
inline void setDeviceEngines(int mode) { check(glx_set_device_engines(mode), "setDeviceEngines"); }
inline int deviceEngines() { return glx_get_device_engines(); }
// GLX_ENGINE_TWOSHOT (default) or GLX_ENGINE_STEPS for the MESH schedule.
inline void setMeshEngine(int engine) { check(glx_set_mesh_engine(engine), "setMeshEngine"); }
// -1 (automatic, default), GLX_ENGINE_DEVSTEPS, GLX_ENGINE_STEPS or
// GLX_ENGINE_DMASTEPS for RING, halving-doubling, bcube and the
// function-style ring.
inline void setStepsEngine(int engine) { check(glx_set_steps_engine(engine), "setStepsEngine"); }

namespace detail {
inline glx_algorithm* createRing(glx_context* c, void* const* p, int n, int count, int dt,
                                 int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_RING_CHUNKED, p, n, count, dt, op, s, ns);
}
inline glx_algorithm* createMesh(glx_context* c, void* const* p, int n, int count, int dt,
                                 int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_RING_CHUNKED_MESH, p, n, count, dt, op, s, ns);
}
inline glx_algorithm* createRepl(glx_context* c, void* const* p, int n, int count, int dt,
                                 int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_RING_CHUNKED_REPL, p, n, count, dt, op, s, ns);
}
inline glx_algorithm* createAuto(glx_context* c, void* const* p, int n, int count, int dt,
                                 int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_RING_CHUNKED_AUTO, p, n, count, dt, op, s, ns);
}
inline glx_algorithm* createRingWhole(glx_context* c, void* const* p, int n, int count, int dt,
                                      int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_RING, p, n, count, dt, op, s, ns);
}
inline glx_algorithm* createBcube(glx_context* c, void* const* p, int n, int count, int dt,
                                  int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_BCUBE, p, n, count, dt, op, s, ns);
}
inline glx_algorithm* createLocal(glx_context* c, void* const* p, int n, int count, int dt,
                                  int op, const glx_stream_t* s, int ns) {
  return glx_allreduce_create(c, GLX_ALGO_LOCAL, p, n, count, dt, op, s, ns);
}
}  // namespace detail

// gloo::CudaHostWorkspace<T> / CudaDeviceWorkspace<T> analogs
// (gloo/cuda_workspace.h:20-30), the algorithms' optional second template
// argument.  Over xGMI the inter-rank scratch is always the receiver's device
// memory, so both tags run the same schedule with the same result bits.
template <typename T>
struct HipHostWorkspace {
  using Pointer = T*;
  static constexpr const char* kName = "host";
};
template <typename T>
struct HipDeviceWorkspace {
  using Pointer = T*;
  static constexpr const char* kName = "device";
};

// gloo::CudaAllreduceRingChunked<T, W> analog (gloo/cuda_allreduce_ring_chunked.h:19-26).
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceRingChunked : public detail::DeviceAllreduce<T> {
 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceRingChunked(const std::shared_ptr<Context>& ctx, const std::vector<T*>& ptrs,
                          int count, const std::vector<glx_stream_t>& streams = {},
                          const ReductionFunction<T>* fn = ReductionFunction<T>::sum,
                          Schedule schedule = Schedule::AUTO)
      : detail::DeviceAllreduce<T>(schedule == Schedule::MESH         ? &detail::createMesh
                                   : schedule == Schedule::REPLICATED ? &detail::createRepl
                                   : schedule == Schedule::RING       ? &detail::createRing
                                                                      : &detail::createAuto,
                                   ctx, ptrs, count, streams, fn, GLX_ALGO_RING_CHUNKED) {}
};

// gloo::CudaAllreduceHalvingDoubling<T, W> analog (gloo/cuda_allreduce_halving_doubling.h:22-30).
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceHalvingDoubling : public detail::DeviceAllreduce<T> {
 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& ctx,
                              const std::vector<T*>& ptrs, int count,
                              const std::vector<glx_stream_t>& streams = {},
                              const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : detail::DeviceAllreduce<T>(&glx_allreduce_halving_doubling_create, ctx, ptrs, count,
                                   streams, fn, GLX_ALGO_HALVING_DOUBLING) {}
  // the CUDA constructor's pipelineBroadcastAndReduce: recorded, same result
  // (the device-driven schedule overlaps its steps either way)
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& ctx,
                              const std::vector<T*>& ptrs, int count,
                              const std::vector<glx_stream_t>& streams,
                              bool pipelineBroadcastAndReduce)
      : detail::DeviceAllreduce<T>(&glx_allreduce_halving_doubling_create, ctx, ptrs, count,
                                   streams, ReductionFunction<T>::sum),
        pipelined_(pipelineBroadcastAndReduce) {}
  bool pipelined() const { return pipelined_; }

 private:
  bool pipelined_ = false;
};

// gloo::CudaAllreduceRing<T, W> / AllreduceRing<T> analog
// (gloo/cuda_allreduce_ring.h:17-24, gloo/allreduce_ring.h:20): each rank's
// own left fold x[r] op x[r-1] op ... (float results may differ between
// ranks, as in the reference).
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceRing : public detail::DeviceAllreduce<T> {
 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceRing(const std::shared_ptr<Context>& ctx, const std::vector<T*>& ptrs, int count,
                   const std::vector<glx_stream_t>& streams = {},
                   const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : detail::DeviceAllreduce<T>(&detail::createRingWhole, ctx, ptrs, count, streams, fn) {}
};

// gloo::CudaAllreduceBcube<T, W> / AllreduceBcube<T> analog
// (gloo/cuda_allreduce_bcube.h, gloo/allreduce_bcube.h:256): groups of the
// context's base() ranks (Context::setBase, default 2).
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceBcube : public detail::DeviceAllreduce<T> {
 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceBcube(const std::shared_ptr<Context>& ctx, const std::vector<T*>& ptrs, int count,
                    const std::vector<glx_stream_t>& streams = {},
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : detail::DeviceAllreduce<T>(&detail::createBcube, ctx, ptrs, count, streams, fn) {}
};

// gloo::CudaAllreduceLocal<T> / AllreduceLocal<T> analog
// (gloo/cuda_allreduce_local.h:21-27, gloo/allreduce_local.h:17-22): this
// rank's pointers folded into ptrs[0] and copied back to the others; no peer
// is involved, whatever the context's size (the context gives the device's
// timeout only).
template <typename T>
class HipAllreduceLocal : public detail::DeviceAllreduce<T> {
 public:
  HipAllreduceLocal(const std::shared_ptr<Context>& ctx, const std::vector<T*>& ptrs, int count,
                    const std::vector<glx_stream_t>& streams = {},
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : detail::DeviceAllreduce<T>(&detail::createLocal, ctx, ptrs, count, streams, fn) {}
};

// gloo::CudaAllreduceHalvingDoublingPipelined<T, W> analog
// (gloo/cuda_allreduce_halving_doubling_pipelined.h:13-27).
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceHalvingDoublingPipelined : public HipAllreduceHalvingDoubling<T, W> {
 public:
  HipAllreduceHalvingDoublingPipelined(const std::shared_ptr<Context>& ctx,
                                       const std::vector<T*>& ptrs, int count,
                                       const std::vector<glx_stream_t>& streams = {})
      : HipAllreduceHalvingDoubling<T, W>(ctx, ptrs, count, streams, true) {}
};

// gloo::sum<T>(c, a, b, n) on the device (gloo/math.h:15-28).
template <typename T>
void sum(T* c, const T* a, const T* b, size_t n, glx_stream_t stream = nullptr) {
  check(glx_reduce(GLX_SUM, DType<T>::value, c, a, b, n, stream), "sum");
}
template <typename T>
void product(T* c, const T* a, const T* b, size_t n, glx_stream_t stream = nullptr) {
  check(glx_reduce(GLX_PRODUCT, DType<T>::value, c, a, b, n, stream), "product");
}
template <typename T>
void max(T* c, const T* a, const T* b, size_t n, glx_stream_t stream = nullptr) {
  check(glx_reduce(GLX_MAX, DType<T>::value, c, a, b, n, stream), "max");
}
template <typename T>
void min(T* c, const T* a, const T* b, size_t n, glx_stream_t stream = nullptr) {
  check(glx_reduce(GLX_MIN, DType<T>::value, c, a, b, n, stream), "min");
}

// gloo::sum<T>(void*, const void*, const void*, size_t) and friends with the
// reference's untyped signature (gloo/math.h:15-73), on device pointers:
// these are what AllreduceOptions::setReduceFunction recognises.
template <typename T>
void sum(void* c, const void* a, const void* b, size_t n) {
  check(glx_reduce(GLX_SUM, DType<T>::value, c, a, b, n, nullptr), "sum");
}
template <typename T>
void product(void* c, const void* a, const void* b, size_t n) {
  check(glx_reduce(GLX_PRODUCT, DType<T>::value, c, a, b, n, nullptr), "product");
}
template <typename T>
void max(void* c, const void* a, const void* b, size_t n) {
  check(glx_reduce(GLX_MAX, DType<T>::value, c, a, b, n, nullptr), "max");
}
template <typename T>
void min(void* c, const void* a, const void* b, size_t n) {
  check(glx_reduce(GLX_MIN, DType<T>::value, c, a, b, n, nullptr), "min");
}

// gloo::AllreduceOptions (gloo/allreduce.h:89-193).  The reduction is one of
// the gloo/math.h ops -- pass &gloo_amd::sum<T> (the reference's idiom,
// allreduce_test.cc:380-383), a ReductionFunction<T>, or a ReductionType --
// on device (or staged host) buffers; or, as the reference's Func
// (gloo/allreduce.h:36,69), any other c = f(a, b) callable on HOST buffers,
// run on the host in the reference's order (glx_allreduce_host_fn).
// setStream() is an addition: without it allreduce() returns with the
// outputs complete, like the reference.
class AllreduceOptions {
 public:
  using Func = std::function<void(void*, const void*, const void*, size_t)>;
  using MathFn = void (*)(void*, const void*, const void*, size_t);
  enum Algorithm {
    UNSPECIFIED = GLX_ALLREDUCE_UNSPECIFIED,
    RING = GLX_ALLREDUCE_RING,
    BCUBE = GLX_ALLREDUCE_BCUBE,
    RING_MESH = GLX_ALLREDUCE_RING_MESH,  // RING's result over all links
    RING_REPLICATED = GLX_ALLREDUCE_RING_REPLICATED,  // RING's result in one round
  };

  explicit AllreduceOptions(const std::shared_ptr<Context>& context) : context_(context) {}

  void setAlgorithm(Algorithm algorithm) { algorithm_ = algorithm; }

  template <typename T>
  void setInput(T* ptr, size_t elements) {
    setInputs(&ptr, 1, elements);
  }
  template <typename T>
  void setInputs(std::vector<T*> ptrs, size_t elements) {
    setInputs(ptrs.data(), ptrs.size(), elements);
  }
  template <typename T>
  void setInputs(T** ptrs, size_t len, size_t elements) {
    setType<T>(elements);
    in_.assign(ptrs, ptrs + len);
  }
  template <typename T>
  void setOutput(T* ptr, size_t elements) {
    setOutputs(&ptr, 1, elements);
  }
  template <typename T>
  void setOutputs(std::vector<T*> ptrs, size_t elements) {
    setOutputs(ptrs.data(), ptrs.size(), elements);
  }
  template <typename T>
  void setOutputs(T** ptrs, size_t len, size_t elements) {
    setType<T>(elements);
    out_.assign(ptrs, ptrs + len);
  }

  void setReduceFunction(Func fn) {
    fn_ = fn;
    op_ = -1;
  }
  void setReduceFunction(ReductionType t) {
    op_ = t;
    fn_ = nullptr;
  }
  template <typename T>
  void setReduceFunction(const ReductionFunction<T>* fn) {
    setReduceFunction(fn->type());
  }
  void setTag(uint32_t tag) { tag_ = tag; }
  void setMaxSegmentSize(size_t maxSegmentSize) { maxSegmentSize_ = maxSegmentSize; }
  void setTimeout(std::chrono::milliseconds timeout) { timeout_ = timeout; }
  void setStream(glx_stream_t stream) { stream_ = stream; }

 private:
  template <typename T>
  void setType(size_t elements) {
    dtype_ = DTypeOrNone<T>::value;
    elementSize_ = sizeof(T);
    elements_ = elements;
  }
  template <typename T>
  static int opOf(MathFn f) {
    if (f == static_cast<MathFn>(&sum<T>)) return GLX_SUM;
    if (f == static_cast<MathFn>(&product<T>)) return GLX_PRODUCT;
    if (f == static_cast<MathFn>(&max<T>)) return GLX_MAX;
    if (f == static_cast<MathFn>(&min<T>)) return GLX_MIN;
    return -1;
  }
  // the device op of a gloo/math.h function of the buffers' type; -1 for any
  // other function (a host Func)
  int resolveOp() const {
    if (!fn_) return op_ < 0 ? GLX_SUM : op_;
    const MathFn* t = fn_.target<MathFn>();
    if (t == nullptr || *t == nullptr) return -1;
    switch (dtype_) {
      case GLX_INT8: return opOf<int8_t>(*t);
      case GLX_UINT8: return opOf<uint8_t>(*t);
      case GLX_INT32: return opOf<int32_t>(*t);
      case GLX_INT64: return opOf<int64_t>(*t);
      case GLX_UINT64: return opOf<uint64_t>(*t);
      case GLX_FLOAT32: return opOf<float>(*t);
      case GLX_FLOAT64: return opOf<double>(*t);
      case GLX_FLOAT16: return opOf<float16>(*t);
      case GLX_BFLOAT16: return opOf<bfloat16>(*t);
    }
    return -1;
  }
  // glx_reduce_fn -> the caller's Func; the first exception it throws is
  // kept (never unwound through the C ABI) and rethrown by allreduce()
  struct HostCall {
    const Func* fn;
    std::exception_ptr error;
    static int trampoline(void* user, void* c, const void* a, const void* b, size_t n) {
      HostCall* call = static_cast<HostCall*>(user);
      if (call->error) return 1;
      try {
        (*call->fn)(c, a, b, n);
      } catch (...) {
        call->error = std::current_exception();
        return 1;
      }
      return 0;
    }
  };

  std::shared_ptr<Context> context_;
  int algorithm_ = UNSPECIFIED;
  std::vector<void*> in_, out_;
  size_t elements_ = 0;
  size_t elementSize_ = 0;
  int dtype_ = -1;
  Func fn_ = nullptr;
  int op_ = -1;
  uint32_t tag_ = 0;
  size_t maxSegmentSize_ = 0;
  std::chrono::milliseconds timeout_{0};
  glx_stream_t stream_ = nullptr;

  friend void allreduce(const AllreduceOptions& opts);
};

// gloo::allreduce (gloo/allreduce.h:195, gloo/allreduce.cc:97-146)
inline void allreduce(const AllreduceOptions& opts) {
  const int op = opts.resolveOp();
  if (op < 0) {
    // a host Func: host buffers, no stream (glx_allreduce_host_fn refuses
    // device buffers with a message)
    if (opts.stream_ != nullptr) {
      throw EnforceNotMet("allreduce: a caller's reduce function runs on the host, with "
                          "host buffers; there is no stream to order it on");
    }
    AllreduceOptions::HostCall call{&opts.fn_, nullptr};
    const int rc = glx_allreduce_host_fn(
        opts.context_->handle(), opts.algorithm_, opts.elementSize_,
        &AllreduceOptions::HostCall::trampoline, &call,
        opts.in_.empty() ? nullptr : opts.in_.data(), (int)opts.in_.size(), opts.out_.data(),
        (int)opts.out_.size(), opts.elements_, opts.tag_, opts.maxSegmentSize_,
        (int64_t)opts.timeout_.count());
    if (call.error) std::rethrow_exception(call.error);
    check(rc, "allreduce");
    return;
  }
  check(glx_allreduce(opts.context_->handle(), opts.algorithm_, opts.dtype_, op,
                      opts.in_.data(), (int)opts.in_.size(), opts.out_.data(),
                      (int)opts.out_.size(), opts.elements_, opts.tag_, opts.maxSegmentSize_,
                      (int64_t)opts.timeout_.count(), opts.stream_),
        "allreduce");
}

}  // namespace gloo_amd
