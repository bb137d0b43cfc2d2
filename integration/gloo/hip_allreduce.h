// gloo/hip_allreduce.h -- gloo_amd's MI355X allreduce behind the reference's
// own Algorithm surface.  A gloo maintainer drops this header into the gloo
// tree (next to gloo/cuda_allreduce_ring_chunked.h) and links
// -lgloo_amd -lamdhip64; callers keep gloo's types, macros and exceptions.
//
//   HipAllreduceRingChunked<T, W>     ~ CudaAllreduceRingChunked<T, W>
//                                       (gloo/cuda_allreduce_ring_chunked.h:19-26)
//   HipAllreduceHalvingDoubling<T, W> ~ CudaAllreduceHalvingDoubling<T, W>
//                                       (gloo/cuda_allreduce_halving_doubling.h:22-30)
//   HipAllreduceRing<T, W>            ~ CudaAllreduceRing<T, W>
//                                       (gloo/cuda_allreduce_ring.h:17-24)
//   HipAllreduceBcube<T, W>           ~ CudaAllreduceBcube<T, W>
//                                       (gloo/cuda_allreduce_bcube.h), groups
//                                       of the gloo context's `base` ranks
//   HipAllreduceLocal<T>              ~ CudaAllreduceLocal<T>
//                                       (gloo/cuda_allreduce_local.h:21-27), this
//                                       rank's pointers only, no exchange
//   HipAllreduceHalvingDoublingPipelined<T, W>
//                                     ~ CudaAllreduceHalvingDoublingPipelined<T, W>
//                                       (gloo/cuda_allreduce_halving_doubling_pipelined.h:13-27)
//   HipHostWorkspace<T>, HipDeviceWorkspace<T>
//                                     ~ CudaHostWorkspace<T>, CudaDeviceWorkspace<T>
//                                       (gloo/cuda_workspace.h:20-30)
//
// W defaults to the host workspace as in the reference, so every CUDA call
// site (gloo/test/cuda_allreduce_test.cc:85-144, gloo/benchmark/
// cuda_main.cc:184-197) switches by renaming the type.  The workspace only
// says where the CUDA algorithms keep their inter-rank scratch (host memory
// for a TCP pair, device memory for a GPUDirect one); over xGMI the scratch is
// always the receiver's device memory, so both tags run the same schedule
// with the same result bits (workspace() reports the tag).
//
// Both take the reference's gloo::Context, the device pointers of this rank,
// the element count, optional streams (outputs valid once streams[0] reaches
// the end of run(); without streams, when run() returns -- docs/cuda.md:9-11)
// and a gloo::ReductionFunction<T> accepted by its type() (SUM, PRODUCT, MAX,
// MIN run on the device; the reference's accelerated paths do the same,
// gloo/algorithm.h:40-48).  A CUSTOM function cannot run on the device: with
// HOST buffers the ring-chunked and halving-doubling classes run their
// program on the host, calling it exactly where the reference's CPU classes
// do (glx_allreduce_create_host_fn); with device buffers it is refused.
//
// The constructors are the CUDA ones, argument for argument (plus the
// optional ReductionFunction of the CPU algorithms).  The xGMI transport
// exchanges its device endpoints (IPC handles of receive regions, flag rows)
// over the gloo context's own pairs with gloo::allgather (ContextStore
// below), so nothing beyond the connected context is needed: at connect (the
// first HIP algorithm created on a context) and at each algorithm's first
// run(), every rank, whatever else it did in between.  An overload
// taking the rendezvous::Store the context was connected with is kept: it
// publishes the endpoints there instead (no collective at first run).  The
// first algorithm created on a gloo context sets up one xGMI context for it
// (all ranks create algorithms in the same order, as gloo requires); later
// ones share it.
//
// gloo::hip::allreduce(opts[, stream]) is gloo::allreduce(const
// AllreduceOptions&) (gloo/allreduce.h:193) for device buffers: the same
// options object (inputs, outputs, algorithm, tag, segment size, timeout);
// the reduce function must be one of the gloo/math.h templates (&gloo::sum<T>
// ...), which also names the element type.
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
#include <exception>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "gloo/algorithm.h"
#include "gloo/allgather.h"
#include "gloo/allreduce.h"
#include "gloo/math.h"
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

// The xGMI layer's rendezvous keys carried by the gloo context itself.
// Every key is set by the rank that owns it and read by its peers.  An
// exchange is ONE collective: every rank contributes the keys it set since
// the previous one, gathered with gloo::allgather (gloo/allgather.h:71) over
// the context's pairs.  Exchanges happen at program points every rank passes
// in the same order, never because one rank happens to lack a key:
//   * connect (the first HIP algorithm created on the context) and
//     gloo::hip::allreduce calls: the rank sets its own keys and then reads
//     its peers' ones, which no earlier exchange can have carried (a peer
//     sets them in the same call) -- so every rank misses and exchanges;
//   * each class algorithm's first run(): one exchange, unconditionally
//     (sync()), after which the algorithm's records must all be here.  gloo
//     constructors are local, so ranks may interleave creating and running
//     algorithms differently (create A, create B, run A, run B on one rank;
//     create A, run A, create B, run B on another); runs are collective and
//     come in the same order everywhere, so the exchanges line up.  (Round 3
//     exchanged on a missed read only; with that interleaving the second rank
//     already held B's record from A's exchange, skipped the one the first
//     rank started at B's run, and both waited out the timeout.)
// A key still missing after its exchange will never arrive (the ranks'
// programs differ): the read fails at once (-2) instead of waiting out the
// timeout, and a strict read (inside a first run) never exchanges at all.
class ContextStore {
 public:
  // the allgather tag of the exchanges: any value user collectives on this
  // context do not run under concurrently (they run on the same thread)
  static constexpr uint32_t kTag = 0x676c7800u;  // "glx"

  explicit ContextStore(std::shared_ptr<Context> ctx) : ctx_(std::move(ctx)) {
    handle_ = glx_callback_store_create(&ContextStore::set, &ContextStore::get, this);
    GLOO_ENFORCE(handle_ != nullptr, "glx_callback_store_create failed");
  }
  ~ContextStore() { glx_store_destroy(handle_); }
  ContextStore(const ContextStore&) = delete;
  ContextStore& operator=(const ContextStore&) = delete;
  glx_store* handle() const { return handle_; }
  int exchanges() const { return exchanges_; }
  const std::string& lastError() const { return error_; }

  // one collective exchange now, whatever this rank already knows
  void sync() { exchange(); }
  // strict: a missed read fails at once instead of exchanging
  void setStrict(bool strict) { strict_ = strict; }

 private:
  static int set(void* user, const char* key, const void* data, size_t len) {
    auto* self = static_cast<ContextStore*>(user);
    const char* d = static_cast<const char*>(data);
    self->known_[key] = std::vector<char>(d, d + len);
    self->pending_.push_back(key);
    return 0;
  }

  static int64_t get(void* user, const char* key, void* buf, size_t cap) {
    auto* self = static_cast<ContextStore*>(user);
    auto it = self->known_.find(key);
    if (it == self->known_.end() && self->strict_) {
      self->error_ = std::string("no rank published '") + key +
                     "' before this algorithm's first run (the ranks created their "
                     "algorithms in different orders)";
      return -2;
    }
    if (it == self->known_.end()) {
      try {
        self->exchange();
      } catch (const std::exception& e) {
        self->error_ = e.what();
        return -2;
      }
      it = self->known_.find(key);
      if (it == self->known_.end()) {
        self->error_ = std::string("no rank published '") + key + "'";
        return -2;
      }
    }
    std::memcpy(buf, it->second.data(), std::min(cap, it->second.size()));
    return (int64_t)it->second.size();
  }

  template <typename U>
  static void put(std::vector<char>& b, const U& v) {
    const char* p = reinterpret_cast<const char*>(&v);
    b.insert(b.end(), p, p + sizeof(U));
  }

  // keys set since the last exchange: [u32 key length, key, u64 value
  // length, value]...; two allgathers: every rank's byte count, then the
  // records padded to the longest
  void exchange() {
    std::vector<char> mine;
    for (const auto& k : pending_) {
      const std::vector<char>& v = known_[k];
      put<uint32_t>(mine, (uint32_t)k.size());
      mine.insert(mine.end(), k.begin(), k.end());
      put<uint64_t>(mine, (uint64_t)v.size());
      mine.insert(mine.end(), v.begin(), v.end());
    }
    const int P = ctx_->size;
    int64_t len = (int64_t)mine.size();
    std::vector<int64_t> lens((size_t)P, 0);
    {
      AllgatherOptions o(ctx_);
      o.setInput(&len, 1);
      o.setOutput(lens.data(), (size_t)P);
      o.setTag(kTag);
      allgather(o);
    }
    const size_t mx = (size_t)*std::max_element(lens.begin(), lens.end());
    std::vector<char> all(mx * (size_t)P);
    if (mx > 0) {
      mine.resize(mx);
      AllgatherOptions o(ctx_);
      o.setInput(mine.data(), mx);
      o.setOutput(all.data(), mx * (size_t)P);
      o.setTag(kTag);
      allgather(o);
    }
    for (int r = 0; r < P; r++) {
      const char* p = all.data() + (size_t)r * mx;
      const char* end = p + lens[(size_t)r];
      while (p < end) {
        uint32_t kl;
        std::memcpy(&kl, p, sizeof(kl));
        p += sizeof(kl);
        std::string k(p, kl);
        p += kl;
        uint64_t vl;
        std::memcpy(&vl, p, sizeof(vl));
        p += sizeof(vl);
        known_[k] = std::vector<char>(p, p + vl);
        p += vl;
      }
    }
    pending_.clear();
    exchanges_++;
  }

  std::shared_ptr<Context> ctx_;
  glx_store* handle_ = nullptr;
  std::map<std::string, std::vector<char>> known_;
  std::vector<std::string> pending_;
  int exchanges_ = 0;
  bool strict_ = false;
  std::string error_;
};

// One xGMI context per gloo context, shared by the algorithms made on it.
class XgmiContext {
 public:
  // store == nullptr: the endpoints travel over the gloo context (ContextStore)
  static std::shared_ptr<XgmiContext> of(const std::shared_ptr<Context>& ctx,
                                         rendezvous::Store* store, int device) {
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
  // exchanges over the gloo context so far (0 with a rendezvous store)
  int exchanges() const { return viaContext_ ? viaContext_->exchanges() : 0; }
  // an algorithm's first run: one exchange on every rank, then `fn` with
  // strict reads (nothing to do with a rendezvous store: its reads wait)
  template <typename F>
  void firstRun(F&& fn) {
    if (!viaContext_) {
      fn();
      return;
    }
    viaContext_->sync();
    viaContext_->setStrict(true);
    try {
      fn();
    } catch (...) {
      viaContext_->setStrict(false);
      throw;
    }
    viaContext_->setStrict(false);
  }

 private:
  XgmiContext(const std::shared_ptr<Context>& ctx, rendezvous::Store* store, int device,
              const std::string& prefix) {
    glx_store* st = nullptr;
    if (store != nullptr) {
      bridge_.reset(new StoreBridge(*store, prefix));
      st = bridge_->handle();
    } else {
      viaContext_.reset(new ContextStore(ctx));
      st = viaContext_->handle();
    }
    glx_ = glx_context_create(ctx->rank, ctx->size, device);
    GLOO_ENFORCE(glx_ != nullptr, "glx_context_create: ", glx_last_error());
    check(glx_context_set_timeout(glx_, (int64_t)ctx->getTimeout().count()),
          "glx_context_set_timeout");
    check(glx_context_connect_full_mesh(glx_, st), "glx_context_connect_full_mesh");
  }
  std::unique_ptr<StoreBridge> bridge_;
  std::unique_ptr<ContextStore> viaContext_;
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

// A class algorithm's ReductionFunction<T> of type CUSTOM through
// glx_reduce_fn: the reference calls fn_->call(x, y, n), x = f(x, y); the
// host-run program calls (c = x, a = x, b = y).  The first exception the
// function throws is kept (never unwound through the C ABI) and rethrown
// by run().
template <typename T>
struct ClassFnCall {
  const ReductionFunction<T>* fn;
  std::exception_ptr error;
  static int trampoline(void* user, void* c, const void* /*a == c*/, const void* b, size_t n) {
    ClassFnCall* call = static_cast<ClassFnCall*>(user);
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

template <typename T>
class Allreduce : public Algorithm {
 public:
  void run() override {
    if (ran_) {
      runOnce();
      return;
    }
    xgmi_->firstRun([&] { runOnce(); });
    ran_ = true;
  }
  ~Allreduce() override { glx_algorithm_destroy(alg_); }
  // bytes moved over the peer links per run (introspection)
  int64_t bytesSent() const { return glx_algorithm_bytes_sent(alg_); }
  // endpoint exchanges over the gloo context so far (introspection)
  int exchanges() const { return xgmi_->exchanges(); }

 protected:
  Allreduce(int algo, const std::shared_ptr<Context>& context, rendezvous::Store* store,
            const std::vector<T*>& ptrs, int count, const std::vector<hipStream_t>& streams,
            const ReductionFunction<T>* fn)
      : Algorithm(context) {
    GLOO_ENFORCE(!ptrs.empty(), "at least one pointer is required");
    xgmi_ = XgmiContext::of(context, store, deviceOf(ptrs[0]));
    // gloo::Context::base (gloo/context.h:33): AllreduceBcube's group size
    check(glx_context_set_base(xgmi_->get(), std::max(2, context->base)), "base");
    std::vector<void*> p(ptrs.begin(), ptrs.end());
    std::vector<glx_stream_t> s(streams.begin(), streams.end());
    GLOO_ENFORCE(fn != nullptr, "null reduction function");
    if (fn->type() == CUSTOM) {
      // a host function: host buffers, the algorithm's program run on the
      // host (glx_allreduce_create_host_fn; device buffers are refused there)
      GLOO_ENFORCE(s.empty(), "HIP allreduce: a CUSTOM reduction function runs on the host, "
                   "with host buffers; there are no streams to order it on");
      custom_.reset(new ClassFnCall<T>{fn, nullptr});
      alg_ = glx_allreduce_create_host_fn(xgmi_->get(), algo, p.data(), (int)p.size(), count,
                                          sizeof(T), &ClassFnCall<T>::trampoline, custom_.get());
      GLOO_ENFORCE(alg_ != nullptr, "glx_allreduce_create_host_fn: ", glx_last_error());
      return;
    }
    alg_ = glx_allreduce_create(xgmi_->get(), algo, p.data(), (int)p.size(), count,
                                GlxType<T>::value, glxOp(fn), s.empty() ? nullptr : s.data(),
                                (int)s.size());
    GLOO_ENFORCE(alg_ != nullptr, "glx_allreduce_create: ", glx_last_error());
  }

 private:
  void runOnce() {
    const int rc = glx_algorithm_run(alg_);
    if (custom_ && custom_->error) {
      std::exception_ptr e = custom_->error;
      custom_->error = nullptr;
      std::rethrow_exception(e);
    }
    check(rc, "run");
  }

  std::shared_ptr<XgmiContext> xgmi_;
  glx_algorithm* alg_ = nullptr;
  std::unique_ptr<ClassFnCall<T>> custom_;
  bool ran_ = false;
};

// AllreduceOptions keeps its settings in a protected member that only
// gloo::allreduce may read (gloo/allreduce.h:187-190); a pointer to that
// member, formed inside a derived class, reads it from any options object.
struct OptionsAccess : AllreduceOptions {
  static const detail::AllreduceOptionsImpl& of(const AllreduceOptions& o) {
    return o.*(&OptionsAccess::impl_);
  }
};

// The glx element type and op of a reduce function that is one of the
// gloo/math.h templates (&gloo::sum<T>, &gloo::product<T>, &gloo::max<T>,
// &gloo::min<T>); false for anything else (a host-only std::function).
using MathFn = void (*)(void*, const void*, const void*, size_t);

template <typename T>
bool matchMath(MathFn f, int* dtype, int* op) {
  const MathFn fns[4] = {&gloo::sum<T>, &gloo::product<T>, &gloo::max<T>, &gloo::min<T>};
  const int ops[4] = {GLX_SUM, GLX_PRODUCT, GLX_MAX, GLX_MIN};
  for (int i = 0; i < 4; i++) {
    if (f == fns[i]) {
      *dtype = GlxType<T>::value;
      *op = ops[i];
      return true;
    }
  }
  return false;
}

inline bool mathFunction(const AllreduceOptions::Func& fn, int* dtype, int* op) {
  const MathFn* f = fn.target<MathFn>();
  if (f == nullptr || *f == nullptr) return false;
  return matchMath<float>(*f, dtype, op) || matchMath<double>(*f, dtype, op) ||
         matchMath<float16>(*f, dtype, op) || matchMath<int32_t>(*f, dtype, op) ||
         matchMath<int64_t>(*f, dtype, op) || matchMath<uint64_t>(*f, dtype, op) ||
         matchMath<int8_t>(*f, dtype, op) || matchMath<uint8_t>(*f, dtype, op);
}

inline size_t glxElementSize(int dtype) {
  switch (dtype) {
    case GLX_INT8:
    case GLX_UINT8: return 1;
    case GLX_FLOAT16: return 2;
    case GLX_INT32:
    case GLX_FLOAT32: return 4;
    default: return 8;
  }
}

// A caller's AllreduceOptions::Func through glx_reduce_fn: the call's
// function, and the first exception it threw (never unwound through the C
// ABI; rethrown after the call).
struct HostFnCall {
  const AllreduceOptions::Func* fn;
  std::exception_ptr error;
  static int trampoline(void* user, void* c, const void* a, const void* b, size_t n) {
    HostFnCall* call = static_cast<HostFnCall*>(user);
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

// gloo::allreduce(const AllreduceOptions&) (gloo/allreduce.h:193,
// gloo/allreduce.cc:97-146).  Same options, same checks (gloo/allreduce.cc:
// 113-119), same result bits; opts.setAlgorithm picks the reference's
// schedule (RING, BCUBE; UNSPECIFIED = RING's result with the data movement
// chosen by size).  With gloo/math.h's sum/product/max/min<T> the buffers
// may be device memory (the xGMI path); stream == nullptr: the outputs are
// complete on return, else the work is ordered on `stream`.  With any other
// Func (gloo/allreduce.h:36,69,171) the buffers must be host memory: the
// same step program runs on the host, calling the function in the
// reference's order (glx_allreduce_host_fn).
inline void allreduce(const AllreduceOptions& opts, hipStream_t stream = nullptr) {
  const detail::AllreduceOptionsImpl& o = OptionsAccess::of(opts);
  GLOO_ENFORCE(o.context, "allreduce: no context");
  GLOO_ENFORCE(!o.out.empty(), "allreduce: no output buffer");
  GLOO_ENFORCE(o.elementSize > 0);
  GLOO_ENFORCE(o.reduce, "allreduce: no reduce function");
  int dtype = -1, op = -1;
  if (!mathFunction(o.reduce, &dtype, &op)) {
    GLOO_ENFORCE(stream == nullptr,
                 "HIP allreduce: a caller's reduce function runs on the host, with host "
                 "buffers; there is no stream to order it on");
    const size_t bytes = o.elements * o.elementSize;
    std::vector<void*> in, out;
    for (const auto& b : o.in) {
      GLOO_ENFORCE_EQ(b->size, bytes, "input buffers must all hold the element count");
      in.push_back(b->ptr);
    }
    for (const auto& b : o.out) {
      GLOO_ENFORCE_EQ(b->size, bytes, "output buffers must all hold the element count");
      out.push_back(b->ptr);
    }
    int algorithm = GLX_ALLREDUCE_UNSPECIFIED;
    if (o.algorithm == detail::AllreduceOptionsImpl::RING) algorithm = GLX_ALLREDUCE_RING;
    if (o.algorithm == detail::AllreduceOptionsImpl::BCUBE) algorithm = GLX_ALLREDUCE_BCUBE;
    auto x = XgmiContext::of(o.context, nullptr, deviceOf(out[0]));
    HostFnCall call{&o.reduce, nullptr};
    const int rc = glx_allreduce_host_fn(
        x->get(), algorithm, o.elementSize, &HostFnCall::trampoline, &call,
        in.empty() ? nullptr : in.data(), (int)in.size(), out.data(), (int)out.size(),
        o.elements, o.tag, o.maxSegmentSize, (int64_t)o.timeout.count());
    if (call.error) std::rethrow_exception(call.error);
    check(rc, "allreduce");
    return;
  }
  GLOO_ENFORCE_EQ(glxElementSize(dtype), o.elementSize,
                  "reduce function's element type differs from the buffers'");
  const size_t bytes = o.elements * o.elementSize;
  std::vector<void*> in, out;  // device buffers (or host ones, staged per call)
  for (const auto& b : o.in) {
    GLOO_ENFORCE_EQ(b->size, bytes, "input buffers must all hold the element count");
    in.push_back(b->ptr);
  }
  for (const auto& b : o.out) {
    GLOO_ENFORCE_EQ(b->size, bytes, "output buffers must all hold the element count");
    out.push_back(b->ptr);
  }
  int algorithm = GLX_ALLREDUCE_UNSPECIFIED;
  switch (o.algorithm) {
    case detail::AllreduceOptionsImpl::RING: algorithm = GLX_ALLREDUCE_RING; break;
    case detail::AllreduceOptionsImpl::BCUBE: algorithm = GLX_ALLREDUCE_BCUBE; break;
    default: break;
  }
  auto x = XgmiContext::of(o.context, nullptr, deviceOf(out[0]));
  check(glx_allreduce(x->get(), algorithm, dtype, op, in.empty() ? nullptr : in.data(),
                      (int)in.size(), out.data(), (int)out.size(), o.elements, o.tag,
                      o.maxSegmentSize, (int64_t)o.timeout.count(), stream),
        "allreduce");
}

}  // namespace hip

// ~ CudaHostWorkspace<T> / CudaDeviceWorkspace<T> (gloo/cuda_workspace.h:20-30):
// the algorithms' second template argument.  Pointer is what the scratch of
// that workspace would be; over xGMI both run the same device schedule.
template <typename T>
class HipHostWorkspace {
 public:
  using Pointer = T*;
  static constexpr const char* kName = "host";
};

template <typename T>
class HipDeviceWorkspace {
 public:
  using Pointer = T*;
  static constexpr const char* kName = "device";
};

namespace hip {
template <typename T, typename W>
struct IsWorkspace {
  static constexpr bool value = std::is_same<W, HipHostWorkspace<T>>::value ||
                                std::is_same<W, HipDeviceWorkspace<T>>::value;
};
}  // namespace hip

// ~ CudaAllreduceRingChunked<T, W> (gloo/cuda_allreduce_ring_chunked.h:19-26)
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceRingChunked : public hip::Allreduce<T> {
  static_assert(hip::IsWorkspace<T, W>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");

 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceRingChunked(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                          const int count,
                          const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                          const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_RING_CHUNKED, context, nullptr, ptrs, count, streams, fn) {}
  // endpoints published through the store the context was connected with
  HipAllreduceRingChunked(const std::shared_ptr<Context>& context, rendezvous::Store& store,
                          const std::vector<T*>& ptrs, const int count,
                          const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                          const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_RING_CHUNKED, context, &store, ptrs, count, streams, fn) {}
};

// ~ CudaAllreduceHalvingDoubling<T, W> (gloo/cuda_allreduce_halving_doubling.h:22-30)
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceHalvingDoubling : public hip::Allreduce<T> {
  static_assert(hip::IsWorkspace<T, W>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");

 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& context,
                              const std::vector<T*>& ptrs, const int count,
                              const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                              const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_HALVING_DOUBLING, context, nullptr, ptrs, count, streams,
                          fn) {}
  // the CUDA constructor's last argument: whether to pipeline the local
  // broadcast with the reduce (gloo/cuda_allreduce_halving_doubling.h:30;
  // gloo/cuda_allreduce_halving_doubling.cc:252-279,374-392: with several
  // local pointers, fold only the first send's range before sending, the rest
  // while the first receive is in flight, and broadcast each allgather step's
  // block to the other pointers as soon as it lands).  The result is the
  // same either way; the device-driven schedule overlaps its steps
  // regardless, so the flag is recorded (pipelined()) and changes nothing.
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& context,
                              const std::vector<T*>& ptrs, const int count,
                              const std::vector<hipStream_t>& streams,
                              bool pipelineBroadcastAndReduce)
      : hip::Allreduce<T>(GLX_ALGO_HALVING_DOUBLING, context, nullptr, ptrs, count, streams,
                          ReductionFunction<T>::sum),
        pipelined_(pipelineBroadcastAndReduce) {}
  HipAllreduceHalvingDoubling(const std::shared_ptr<Context>& context, rendezvous::Store& store,
                              const std::vector<T*>& ptrs, const int count,
                              const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                              const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_HALVING_DOUBLING, context, &store, ptrs, count, streams,
                          fn) {}
  bool pipelined() const { return pipelined_; }

 private:
  bool pipelined_ = false;
};

// ~ CudaAllreduceRing<T, W> (gloo/cuda_allreduce_ring.h:17-24) and the CPU
// AllreduceRing<T> (gloo/allreduce_ring.h:20): each rank's own left fold
// x[r] op x[r-1] op ... op x[r-P+1] (float results may differ between ranks,
// as in the reference); whole buffers, one round over every link.
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceRing : public hip::Allreduce<T> {
  static_assert(hip::IsWorkspace<T, W>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");

 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceRing(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                   const int count,
                   const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                   const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_RING, context, nullptr, ptrs, count, streams, fn) {}
  HipAllreduceRing(const std::shared_ptr<Context>& context, rendezvous::Store& store,
                   const std::vector<T*>& ptrs, const int count,
                   const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                   const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_RING, context, &store, ptrs, count, streams, fn) {}
};

// ~ CudaAllreduceBcube<T, W> (gloo/cuda_allreduce_bcube.h) and the CPU
// AllreduceBcube<T> (gloo/allreduce_bcube.h:256): groups of context->base
// ranks, the reference's ranges and reduction order.
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceBcube : public hip::Allreduce<T> {
  static_assert(hip::IsWorkspace<T, W>::value,
                "W must be HipHostWorkspace<T> or HipDeviceWorkspace<T>");

 public:
  static const char* workspace() { return W::kName; }
  HipAllreduceBcube(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                    const int count,
                    const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_BCUBE, context, nullptr, ptrs, count, streams, fn) {}
  HipAllreduceBcube(const std::shared_ptr<Context>& context, rendezvous::Store& store,
                    const std::vector<T*>& ptrs, const int count,
                    const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : hip::Allreduce<T>(GLX_ALGO_BCUBE, context, &store, ptrs, count, streams, fn) {}
};

// ~ CudaAllreduceLocal<T> (gloo/cuda_allreduce_local.h:21-27) and the CPU
// AllreduceLocal<T> (gloo/allreduce_local.h:17-22, allreduce_local.cc:21-31):
// this rank's pointers folded left into ptrs[0], then copied to the others.
// Nothing is exchanged, so unlike the classes above it takes no part in the
// xGMI context's exchanges: it runs on a one-rank glx context of its own (a
// rank may create and run it alone, as with the reference's).
template <typename T>
class HipAllreduceLocal : public Algorithm {
 public:
  HipAllreduceLocal(const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs,
                    const int count,
                    const std::vector<hipStream_t>& streams = std::vector<hipStream_t>(),
                    const ReductionFunction<T>* fn = ReductionFunction<T>::sum)
      : Algorithm(context) {
    GLOO_ENFORCE(!ptrs.empty(), "at least one pointer is required");
    local_ = glx_context_create(0, 1, hip::deviceOf(ptrs[0]));
    GLOO_ENFORCE(local_ != nullptr, "glx_context_create: ", glx_last_error());
    std::vector<void*> p(ptrs.begin(), ptrs.end());
    std::vector<glx_stream_t> s(streams.begin(), streams.end());
    if (glx_context_set_timeout(local_, (int64_t)context->getTimeout().count()) == GLX_OK) {
      alg_ = glx_allreduce_create(local_, GLX_ALGO_LOCAL, p.data(), (int)p.size(), count,
                                  hip::GlxType<T>::value, hip::glxOp(fn),
                                  s.empty() ? nullptr : s.data(), (int)s.size());
    }
    if (alg_ == nullptr) {
      const std::string err = glx_last_error();
      glx_context_destroy(local_);
      GLOO_ENFORCE(false, "glx_allreduce_create: ", err);
    }
  }
  ~HipAllreduceLocal() override {
    glx_algorithm_destroy(alg_);
    glx_context_destroy(local_);
  }
  void run() override { hip::check(glx_algorithm_run(alg_), "run"); }

 private:
  glx_context* local_ = nullptr;
  glx_algorithm* alg_ = nullptr;
};

// ~ CudaAllreduceHalvingDoublingPipelined<T, W>
// (gloo/cuda_allreduce_halving_doubling_pipelined.h:13-27): halving-doubling
// with pipelineBroadcastAndReduce = true, the same four arguments.
template <typename T, typename W = HipHostWorkspace<T>>
class HipAllreduceHalvingDoublingPipelined : public HipAllreduceHalvingDoubling<T, W> {
 public:
  HipAllreduceHalvingDoublingPipelined(
      const std::shared_ptr<Context>& context, const std::vector<T*>& ptrs, const int count,
      const std::vector<hipStream_t>& streams = std::vector<hipStream_t>())
      : HipAllreduceHalvingDoubling<T, W>(context, ptrs, count, streams, true) {}
};

}  // namespace gloo
