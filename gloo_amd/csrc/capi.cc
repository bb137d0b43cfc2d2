// capi.cc -- the extern "C" boundary (include/gloo_amd/glx.h).
// Every entry point catches, records the message for glx_last_error() and
// returns a GLX_ERR_* code; nothing throws across the ABI.
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <memory>
#include <string>

#include "../../include/gloo_amd/glx.h"
#include "collectives.h"
#include "common.h"
#include "context.h"
#include "executor.h"
#include "executor_internal.h"
#include "host_fn.h"
#include "host_ops.h"
#include "kernels.h"
#include "linkprobe.h"
#include "plan.h"
#include "store.h"

struct glx_store {
  std::shared_ptr<gloo::rendezvous::Store> s;
};
struct glx_context {
  std::shared_ptr<gloo::Context> c;
};
struct glx_algorithm {
  std::unique_ptr<gloo::HipPlanExecutor> a;
  // or a class algorithm with a caller's function on host buffers
  // (glx_allreduce_create_host_fn): the executor, its buffers and function
  std::shared_ptr<gloo::HostFnExecutor> hostFn;
  std::vector<void*> ptrs;
  glx_reduce_fn fn = nullptr;
  void* user = nullptr;
};
struct glx_link_probe {
  std::unique_ptr<gloo::LinkProbe> p;
};

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

template <typename F>
int guarded(F&& f) {
  try {
    g_last_error.clear();
    return f();
  } catch (const gloo::TimeoutException& e) {
    return fail(GLX_ERR_TIMEOUT, e.what());
  } catch (const gloo::IoException& e) {
    return fail(GLX_ERR_IO, e.what());
  } catch (const gloo::HipError& e) {
    return fail(GLX_ERR_HIP, e.what());
  } catch (const gloo::EnforceNotMet& e) {
    return fail(GLX_ERR_ENFORCE, e.what());
  } catch (const std::logic_error& e) {
    return fail(GLX_ERR_INVALID, e.what());
  } catch (const std::exception& e) {
    return fail(GLX_ERR_INTERNAL, e.what());
  } catch (...) {
    return fail(GLX_ERR_INTERNAL, "unknown exception");
  }
}

int hipStatus(hipError_t e, const char* what) {
  if (e == hipSuccess) return GLX_OK;
  return fail(GLX_ERR_HIP, std::string(what) + ": " + hipGetErrorName(e) + ": " +
                               hipGetErrorString(e));
}

bool validDtype(int d) { return d >= GLX_INT8 && d <= GLX_BFLOAT16; }
bool validOp(int o) { return o >= GLX_SUM && o <= GLX_MIN; }

glx_algorithm* makeAlgorithm(int algo, glx_context* ctx, void* const* ptrs, int nptrs,
                             int count, int dtype, int op, const glx_stream_t* streams,
                             int nstreams) {
  glx_algorithm* out = nullptr;
  guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    GLX_ENFORCE(ptrs != nullptr && nptrs > 0, "need at least one pointer");
    GLX_ENFORCE(count >= 0, "negative element count");
    GLX_ENFORCE(nstreams == 0 || streams != nullptr, "null streams array");
    std::vector<void*> p(ptrs, ptrs + nptrs);
    std::vector<hipStream_t> s;
    for (int i = 0; i < nstreams; i++) s.push_back((hipStream_t)streams[i]);
    std::unique_ptr<gloo::HipPlanExecutor> a(
        new gloo::HipPlanExecutor(ctx->c, algo, p, count, dtype, op, s));
    out = new glx_algorithm{std::move(a)};
    return GLX_OK;
  });
  return out;
}

glx::PlanParams planParams(int esize, int64_t maxSegmentBytes, int64_t minPieceBytes) {
  glx::PlanParams p;
  p.esize = esize;
  if (maxSegmentBytes > 0) p.maxSegmentBytes = maxSegmentBytes;
  p.minPieceBytes = minPieceBytes < 0 ? 0 : minPieceBytes;
  // the programs the host-issued / DMA steps engines run under
  // glx_set_pipeline_bytes (the CPU tests replay them)
  p.pipelineBytes = glx::pipelineBytes();
  return p;
}

}  // namespace

extern "C" {

const char* glx_last_error(void) { return g_last_error.c_str(); }

const char* glx_version(void) { return "0.1.0"; }

size_t glx_dtype_size(int dtype) {
  static const size_t sz[] = {1, 1, 4, 8, 8, 4, 8, 2, 2};
  return validDtype(dtype) ? sz[dtype] : 0;
}

int glx_reduce(int op, int dtype, void* dst, const void* a, const void* b, size_t n,
               glx_stream_t stream) {
  if (!validOp(op)) return fail(GLX_ERR_INVALID, "glx_reduce: unknown op");
  if (!validDtype(dtype)) return fail(GLX_ERR_INVALID, "glx_reduce: unknown dtype");
  if (n > 0 && (dst == nullptr || a == nullptr || b == nullptr)) {
    return fail(GLX_ERR_INVALID, "glx_reduce: null pointer");
  }
  return hipStatus(glx::launch_reduce(op, dtype, dst, a, b, n, (hipStream_t)stream),
                   "glx_reduce");
}

int glx_reduce_n(int op, int dtype, void* dst, const void* const* srcs, int k, size_t n,
                 glx_stream_t stream) {
  if (!validOp(op)) return fail(GLX_ERR_INVALID, "glx_reduce_n: unknown op");
  if (!validDtype(dtype)) return fail(GLX_ERR_INVALID, "glx_reduce_n: unknown dtype");
  if (k < 2 || k > 8 || srcs == nullptr) {
    return fail(GLX_ERR_INVALID, "glx_reduce_n: need 2..8 sources");
  }
  return hipStatus(glx::launch_reduce_n(op, dtype, dst, srcs, k, n, (hipStream_t)stream),
                   "glx_reduce_n");
}

int glx_host_reduce_n(int op, int dtype, void* dst, const void* const* srcs, int k,
                      size_t n) {
  return guarded([&]() -> int {
    GLX_ENFORCE(validOp(op) && validDtype(dtype), "glx_host_reduce_n: unknown op/dtype");
    GLX_ENFORCE(k >= 1 && srcs != nullptr && (n == 0 || dst != nullptr),
                "glx_host_reduce_n: need k >= 1 sources and a destination");
    if (n > 0) glx::host_reduce_n(op, dtype, dst, srcs, k, n);
    return GLX_OK;
  });
}

int glx_peer_copy(void* dst, int dst_dev, const void* src, int src_dev, size_t bytes,
                  glx_stream_t stream) {
  if (bytes == 0) return GLX_OK;
  if (dst == nullptr || src == nullptr) return fail(GLX_ERR_INVALID, "glx_peer_copy: null");
  return hipStatus(hipMemcpyPeerAsync(dst, dst_dev, src, src_dev, bytes, (hipStream_t)stream),
                   "hipMemcpyPeerAsync");
}

int glx_copy(void* dst, const void* src, size_t bytes, int blocks, glx_stream_t stream) {
  if (bytes == 0) return GLX_OK;
  if (dst == nullptr || src == nullptr) return fail(GLX_ERR_INVALID, "glx_copy: null");
  return hipStatus(glx::launch_copy_blocks(dst, src, bytes, blocks, (hipStream_t)stream),
                   "glx_copy");
}

int glx_enable_peer(int a, int b) {
  if (a == b) return GLX_OK;
  int cur = 0;
  hipGetDevice(&cur);
  for (int pass = 0; pass < 2; pass++) {
    int from = pass == 0 ? a : b, to = pass == 0 ? b : a;
    hipError_t e = hipSetDevice(from);
    if (e == hipSuccess) e = hipDeviceEnablePeerAccess(to, 0);
    if (e == hipErrorPeerAccessAlreadyEnabled) {
      (void)hipGetLastError();
      e = hipSuccess;
    }
    if (e != hipSuccess) {
      hipSetDevice(cur);
      return hipStatus(e, "hipDeviceEnablePeerAccess");
    }
  }
  hipSetDevice(cur);
  return GLX_OK;
}

size_t glx_reduce_segment_bytes(void) { return glx::reduce_segment_bytes(); }

int glx_tune_reduce(int unroll, int blocks_per_cu, int nontemporal) {
  if (unroll != 1 && unroll != 2 && unroll != 4 && unroll != 8) {
    return fail(GLX_ERR_INVALID, "glx_tune_reduce: unroll must be 1, 2, 4 or 8");
  }
  if (blocks_per_cu < 0) return fail(GLX_ERR_INVALID, "glx_tune_reduce: blocks_per_cu < 0");
  glx::set_reduce_tuning(unroll, blocks_per_cu, nontemporal);
  return GLX_OK;
}

int glx_set_max_message_bytes(int64_t bytes) {
  if (bytes < 0 || (bytes > 0 && bytes < 4096)) {
    return fail(GLX_ERR_INVALID, "glx_set_max_message_bytes: 0 (default) or at least 4096");
  }
  glx::setMaxMessageBytes(bytes);
  return GLX_OK;
}

int64_t glx_max_message_bytes(void) { return glx::maxMessageBytes(); }

int glx_set_pipeline_bytes(int64_t bytes) {
  if (bytes < 0 || (bytes > 0 && bytes < 4096)) {
    return fail(GLX_ERR_INVALID, "glx_set_pipeline_bytes: 0 (off) or at least 4096");
  }
  glx::setPipelineBytes(bytes);
  return GLX_OK;
}

int64_t glx_pipeline_bytes(void) { return glx::pipelineBytes(); }

int glx_reduce_tuning(int* unroll, int* blocks_per_cu, int* policy) {
  if (unroll == nullptr || blocks_per_cu == nullptr || policy == nullptr) {
    return fail(GLX_ERR_INVALID, "glx_reduce_tuning: null argument");
  }
  glx::reduce_tuning(unroll, blocks_per_cu, policy);
  return GLX_OK;
}

int glx_set_copy_engine(int engine, int blocks) {
  if (engine != 0 && engine != 1) return fail(GLX_ERR_INVALID, "copy engine must be 0 or 1");
  gloo::HipPlanExecutor::setCopyEngine(engine);
  glx::set_copy_blocks(blocks);
  return GLX_OK;
}

int glx_set_mesh_engine(int engine) {
  if (engine != GLX_ENGINE_STEPS && engine != GLX_ENGINE_TWOSHOT) {
    return fail(GLX_ERR_INVALID, "mesh engine must be GLX_ENGINE_STEPS or GLX_ENGINE_TWOSHOT");
  }
  gloo::HipPlanExecutor::setMeshEngine(engine);
  return GLX_OK;
}

int glx_set_engine_streams(int fast) {
  if (fast != 0 && fast != 1 && fast != -1) {
    return fail(GLX_ERR_INVALID, "engine streams must be -1, 0 or 1");
  }
  gloo::HipPlanExecutor::setEngineStreams(fast);
  return GLX_OK;
}

int glx_set_steps_engine(int engine) {
  if (engine != GLX_ENGINE_STEPS && engine != GLX_ENGINE_DEVSTEPS &&
      engine != GLX_ENGINE_DMASTEPS && engine != -1) {
    return fail(GLX_ERR_INVALID,
                "steps engine must be GLX_ENGINE_STEPS, GLX_ENGINE_DEVSTEPS, "
                "GLX_ENGINE_DMASTEPS or -1 (by size)");
  }
  gloo::HipPlanExecutor::setStepsEngine(engine);
  return GLX_OK;
}

int glx_set_device_engines(int mode) {
  if (mode < GLX_DEVICE_ENGINES_AUTO || mode > GLX_DEVICE_ENGINES_SHARED) {
    return fail(GLX_ERR_INVALID, "device engine mode must be -1 (auto), 0 (off), 1 (on) or 2 (shared)");
  }
  gloo::HipPlanExecutor::setDeviceEngines(mode);
  return GLX_OK;
}

int glx_get_device_engines(void) { return gloo::HipPlanExecutor::deviceEngines(); }

int glx_device_engines_rule(int mode, int ranks, int ranks_per_device, int threads_share_device,
                            int max_hw_queues) {
  if (mode < GLX_DEVICE_ENGINES_AUTO || mode > GLX_DEVICE_ENGINES_SHARED || ranks < 1 ||
      ranks_per_device < 1 || ranks_per_device > ranks) {
    (void)fail(GLX_ERR_INVALID, "glx_device_engines_rule: invalid argument");
    return -1;
  }
  return gloo::HipPlanExecutor::deviceEnginesRule(mode, ranks, ranks_per_device,
                                                  threads_share_device != 0, max_hw_queues)
             ? 1
             : 0;
}

int glx_set_copy_split(int k) {
  if (k < 1 || k > 8) return fail(GLX_ERR_INVALID, "glx_set_copy_split: k must be in [1, 8]");
  gloo::HipPlanExecutor::setCopySplit(k);
  return GLX_OK;
}

int glx_set_pinned_mirror_limit(size_t bytes) {
  gloo::exec::setPinnedMirrorLimit(bytes);
  return GLX_OK;
}

int glx_device_count(int* count) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  if (count) *count = n;
  return GLX_OK;
}

// ---- stores ----------------------------------------------------------------

glx_store* glx_hash_store_create(void) {
  return new glx_store{std::make_shared<gloo::rendezvous::HashStore>()};
}

glx_store* glx_file_store_create(const char* path) {
  glx_store* out = nullptr;
  guarded([&]() -> int {
    GLX_ENFORCE(path != nullptr, "null path");
    out = new glx_store{std::make_shared<gloo::rendezvous::FileStore>(path)};
    return GLX_OK;
  });
  return out;
}

glx_store* glx_prefix_store_create(const char* prefix, glx_store* base) {
  if (prefix == nullptr || base == nullptr) return nullptr;
  return new glx_store{std::make_shared<gloo::rendezvous::PrefixStore>(prefix, base->s)};
}

glx_store* glx_callback_store_create(glx_store_set_fn set_fn, glx_store_get_fn get_fn,
                                     void* user) {
  if (set_fn == nullptr || get_fn == nullptr) return nullptr;
  return new glx_store{std::make_shared<gloo::rendezvous::CallbackStore>(set_fn, get_fn, user)};
}

void glx_store_destroy(glx_store* store) { delete store; }

int glx_store_set(glx_store* store, const char* key, const void* data, size_t len) {
  return guarded([&]() -> int {
    GLX_ENFORCE(store != nullptr && key != nullptr, "null store/key");
    const char* d = static_cast<const char*>(data);
    store->s->set(key, std::vector<char>(d, d + (d ? len : 0)));
    return GLX_OK;
  });
}

int glx_store_get(glx_store* store, const char* key, void* buf, size_t cap,
                  size_t* len_out, int64_t timeout_ms) {
  return guarded([&]() -> int {
    GLX_ENFORCE(store != nullptr && key != nullptr, "null store/key");
    auto v = store->s->get(key, std::chrono::milliseconds(timeout_ms));
    if (buf != nullptr && cap > 0) memcpy(buf, v.data(), std::min(cap, v.size()));
    if (len_out) *len_out = v.size();
    return GLX_OK;
  });
}

// ---- context -----------------------------------------------------------------

glx_context* glx_context_create(int rank, int size, int device) {
  glx_context* out = nullptr;
  guarded([&]() -> int {
    out = new glx_context{std::make_shared<gloo::Context>(rank, size, device)};
    return GLX_OK;
  });
  return out;
}

void glx_context_destroy(glx_context* ctx) {
  if (ctx == nullptr) return;
  guarded([&]() -> int {
    ctx->c->clearOps();
    return GLX_OK;
  });
  delete ctx;
}

int glx_context_connect_full_mesh(glx_context* ctx, glx_store* store) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr && store != nullptr, "null context/store");
    ctx->c->connectFullMesh(store->s);
    return GLX_OK;
  });
}

int glx_context_rank(glx_context* ctx) { return ctx ? ctx->c->rank : -1; }
int glx_context_size(glx_context* ctx) { return ctx ? ctx->c->size : -1; }
int glx_context_device(glx_context* ctx) { return ctx ? ctx->c->device() : -1; }

int glx_context_set_base(glx_context* ctx, int base) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    GLX_ENFORCE(base >= 2, "base must be at least 2");
    ctx->c->setBase(base);
    return GLX_OK;
  });
}

int64_t glx_plan_bcube(int rank, int size, int64_t count, int base, int64_t* steps, int64_t cap,
                       int64_t* scratch_elems) {
  glx::PlanParams prm;
  prm.base = base;
  int64_t n = -1;
  guarded([&]() -> int {
    glx::Plan p = glx::makePlan(glx::ALGO_BCUBE, rank, size, count, prm);
    n = (int64_t)p.steps.size();
    if (scratch_elems) *scratch_elems = p.scratch_elems;
    for (int64_t i = 0; i < n && i < cap && steps != nullptr; i++) {
      const glx::Step& s = p.steps[(size_t)i];
      int64_t* o = steps + 8 * i;
      o[0] = s.kind;
      o[1] = s.peer;
      o[2] = s.channel;
      o[3] = s.off;
      o[4] = s.len;
      o[5] = s.boff;
      o[6] = s.dst_off;
      o[7] = s.flags;
    }
    return GLX_OK;
  });
  return n;
}

int glx_context_set_timeout(glx_context* ctx, int64_t timeout_ms) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    GLX_ENFORCE(timeout_ms >= 0, "negative timeout");
    ctx->c->setTimeout(std::chrono::milliseconds(timeout_ms));
    return GLX_OK;
  });
}

int64_t glx_context_get_timeout(glx_context* ctx) {
  return ctx ? (int64_t)ctx->c->getTimeout().count() : -1;
}

int glx_context_next_slot(glx_context* ctx, int num_to_skip) {
  int slot = -1;
  int rc = guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    slot = ctx->c->nextSlot(num_to_skip);
    return GLX_OK;
  });
  return rc == GLX_OK ? slot : -1;
}

// ---- algorithms --------------------------------------------------------------

glx_algorithm* glx_allreduce_ring_chunked_create(glx_context* ctx, void* const* ptrs,
                                                 int nptrs, int count, int dtype, int op,
                                                 const glx_stream_t* streams,
                                                 int nstreams) {
  return makeAlgorithm(glx::ALGO_RING_CHUNKED, ctx, ptrs, nptrs, count, dtype, op,
                       streams, nstreams);
}

glx_algorithm* glx_allreduce_halving_doubling_create(glx_context* ctx, void* const* ptrs,
                                                     int nptrs, int count, int dtype,
                                                     int op, const glx_stream_t* streams,
                                                     int nstreams) {
  return makeAlgorithm(glx::ALGO_HALVING_DOUBLING, ctx, ptrs, nptrs, count, dtype, op,
                       streams, nstreams);
}

glx_algorithm* glx_allreduce_create(glx_context* ctx, int algo, void* const* ptrs, int nptrs,
                                    int count, int dtype, int op, const glx_stream_t* streams,
                                    int nstreams) {
  if (algo == GLX_ALGO_RING_CHUNKED_AUTO && ctx != nullptr && count >= 0) {
    algo = glx::autoRingSchedule(ctx->c->size, (int64_t)count * (int64_t)glx_dtype_size(dtype),
                                 /*fn=*/false, gloo::HipPlanExecutor::deviceEnginesAvailable(*ctx->c));
  }
  if (algo == GLX_ALGO_LOCAL && ctx != nullptr) {
    // gloo::AllreduceLocal<T> (gloo/allreduce_local.cc:21-31): this rank's
    // pointers folded into ptrs[0] and copied back, nothing exchanged.  The
    // P = 1 case of every class algorithm is exactly that fold and broadcast,
    // so it runs on a private one-rank context on the same device (staging of
    // host buffers, pointers on other GPUs of this rank, streams: as for the
    // others) -- no peer is involved, whatever the caller's context size.
    glx_context local{std::make_shared<gloo::Context>(0, 1, ctx->c->device())};
    local.c->setTimeout(ctx->c->getTimeout());
    return makeAlgorithm(glx::ALGO_RING_CHUNKED, &local, ptrs, nptrs, count, dtype, op, streams,
                         nstreams);
  }
  if (algo != GLX_ALGO_RING_CHUNKED && algo != GLX_ALGO_HALVING_DOUBLING &&
      algo != GLX_ALGO_RING_CHUNKED_MESH && algo != GLX_ALGO_RING_CHUNKED_REPL &&
      algo != GLX_ALGO_RING && algo != GLX_ALGO_BCUBE) {
    fail(GLX_ERR_INVALID, "glx_allreduce_create: unknown algorithm");
    return nullptr;
  }
  return makeAlgorithm(algo, ctx, ptrs, nptrs, count, dtype, op, streams, nstreams);
}

int glx_allreduce(glx_context* ctx, int algorithm, int dtype, int op, void* const* inputs,
                  int num_inputs, void* const* outputs, int num_outputs, size_t elements,
                  uint32_t tag, size_t max_segment_size, int64_t timeout_ms,
                  glx_stream_t stream) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    GLX_ENFORCE(num_inputs >= 0 && (num_inputs == 0 || inputs != nullptr), "bad inputs");
    GLX_ENFORCE(num_outputs >= 0 && (num_outputs == 0 || outputs != nullptr), "bad outputs");
    gloo::AllreduceOptions o(ctx->c);
    o.algorithm = algorithm;
    o.dtype = dtype;
    o.op = op;
    o.in.assign(inputs, inputs + num_inputs);
    o.out.assign(outputs, outputs + num_outputs);
    o.elements = elements;
    o.tag = tag;
    o.maxSegmentSize = max_segment_size;
    o.timeout = std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 0);
    o.stream = (hipStream_t)stream;
    gloo::allreduce(o);
    return GLX_OK;
  });
}

int glx_allreduce_host_fn(glx_context* ctx, int algorithm, size_t element_size,
                          glx_reduce_fn fn, void* user, void* const* inputs, int num_inputs,
                          void* const* outputs, int num_outputs, size_t elements, uint32_t tag,
                          size_t max_segment_size, int64_t timeout_ms) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    GLX_ENFORCE(fn != nullptr, "allreduce: null reduction function");
    GLX_ENFORCE(num_inputs >= 0 && (num_inputs == 0 || inputs != nullptr), "bad inputs");
    GLX_ENFORCE(num_outputs > 0 && outputs != nullptr, "allreduce: at least one output");
    GLX_ENFORCE(element_size > 0, "allreduce: element size must be positive");
    GLX_ENFORCE(algorithm == GLX_ALLREDUCE_UNSPECIFIED || algorithm == GLX_ALLREDUCE_RING ||
                    algorithm == GLX_ALLREDUCE_BCUBE,
                "allreduce with a host reduction function: RING or BCUBE");
    GLX_ENFORCE(elements <= ((size_t)1 << 40), "allreduce: too many elements");
    std::vector<const void*> in(inputs, inputs + num_inputs);
    std::vector<void*> out(outputs, outputs + num_outputs);
    for (const void* p : in) {
      GLX_ENFORCE(gloo::exec::isHostPointer(p),
                  "allreduce: a host reduction function needs host buffers (a device cannot "
                  "run it); device buffers take gloo::sum/product/max/min");
    }
    for (const void* p : out) {
      GLX_ENFORCE(gloo::exec::isHostPointer(p),
                  "allreduce: a host reduction function needs host buffers (a device cannot "
                  "run it); device buffers take gloo::sum/product/max/min");
    }
    if (elements == 0) return GLX_OK;  // gloo/allreduce.cc:98-100
    auto& c = *ctx->c;
    GLX_ENFORCE(c.size == 1 || c.connected(),
                "allreduce: context must be connected (connectFullMesh)");
    const int algo = algorithm == GLX_ALLREDUCE_BCUBE ? glx::ALGO_FN_BCUBE : glx::ALGO_FN_RING;
    const size_t maxSeg = max_segment_size == 0 ? (size_t)glx::kMaxSegmentBytes
                                                : max_segment_size;
    const std::string key = "hostfn/" + std::to_string(algo) + "/" +
                            std::to_string(element_size) + "/" + std::to_string(elements) +
                            "/" + std::to_string(tag) + "/" + std::to_string(maxSeg);
    std::shared_ptr<gloo::Algorithm> alg;
    {
      std::lock_guard<std::mutex> g(c.opsMutex);
      auto it = c.ops.find(key);
      if (it != c.ops.end()) {
        alg = it->second;
      } else {
        alg = std::make_shared<gloo::HostFnExecutor>(ctx->c, algo, element_size, elements,
                                                     maxSeg);
        c.ops.emplace(key, alg);
      }
    }
    static_cast<gloo::HostFnExecutor&>(*alg).call(
        fn, user, in, out, std::chrono::milliseconds(timeout_ms > 0 ? timeout_ms : 0));
    return GLX_OK;
  });
}

glx_algorithm* glx_allreduce_create_host_fn(glx_context* ctx, int algo, void* const* ptrs,
                                            int nptrs, int count, size_t element_size,
                                            glx_reduce_fn fn, void* user) {
  glx_algorithm* out = nullptr;
  guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    GLX_ENFORCE(ptrs != nullptr && nptrs > 0, "need at least one pointer");
    GLX_ENFORCE(count >= 0, "negative element count");
    GLX_ENFORCE(fn != nullptr, "null reduction function");
    GLX_ENFORCE(element_size > 0 && element_size <= ((size_t)1 << 20), "bad element size");
    // every ring_chunked schedule computes the reference ring's bits: the
    // host runs the ring's own program
    int a = -1;
    if (algo == GLX_ALGO_RING_CHUNKED || algo == GLX_ALGO_RING_CHUNKED_MESH ||
        algo == GLX_ALGO_RING_CHUNKED_REPL || algo == GLX_ALGO_RING_CHUNKED_AUTO) {
      a = glx::ALGO_RING_CHUNKED;
    } else if (algo == GLX_ALGO_HALVING_DOUBLING) {
      a = glx::ALGO_HALVING_DOUBLING;
    }
    GLX_ENFORCE(a >= 0,
                "a CUSTOM reduction function runs with AllreduceRingChunked or "
                "AllreduceHalvingDoubling (algorithm ", algo, ")");
    std::vector<void*> p(ptrs, ptrs + nptrs);
    for (const void* q : p) {
      GLX_ENFORCE(q != nullptr, "null pointer");
      GLX_ENFORCE(gloo::exec::isHostPointer(q),
                  "a CUSTOM reduction function needs host buffers (a device cannot run "
                  "it); device buffers take SUM, PRODUCT, MAX or MIN");
    }
    auto& c = *ctx->c;
    GLX_ENFORCE(c.size == 1 || c.connected(),
                "allreduce: context must be connected (connectFullMesh)");
    auto h = std::make_unique<glx_algorithm>();
    h->hostFn = std::make_shared<gloo::HostFnExecutor>(ctx->c, a, element_size,
                                                       (size_t)count, 0);
    h->ptrs = std::move(p);
    h->fn = fn;
    h->user = user;
    out = h.release();
    return GLX_OK;
  });
  return out;
}

int glx_algorithm_run(glx_algorithm* alg) {
  return guarded([&]() -> int {
    GLX_ENFORCE(alg != nullptr, "null algorithm");
    if (alg->hostFn) {
      alg->hostFn->call(alg->fn, alg->user, {}, alg->ptrs, std::chrono::milliseconds(0));
      return GLX_OK;
    }
    alg->a->run();
    return GLX_OK;
  });
}

namespace {
gloo::HipPlanExecutor& planExecutor(glx_algorithm* alg, const char* what) {
  GLX_ENFORCE(alg != nullptr, "null algorithm");
  GLX_ENFORCE(alg->a != nullptr, what, ": not available for an algorithm with a CUSTOM "
              "reduction function (it runs on the host)");
  return *alg->a;
}
}  // namespace

int glx_algorithm_run_fed(glx_algorithm* alg) {
  return guarded([&]() -> int {
    planExecutor(alg, "run_fed").runFed();
    return GLX_OK;
  });
}

int glx_algorithm_feed(glx_algorithm* alg, int64_t off, int64_t len) {
  return guarded([&]() -> int {
    planExecutor(alg, "feed").feed(off, len);
    return GLX_OK;
  });
}

int64_t glx_algorithm_done_ranges(glx_algorithm* alg, int64_t* out, int64_t cap) {
  int64_t n = -1;
  guarded([&]() -> int {
    const std::vector<glx::Range> r = planExecutor(alg, "done_ranges").doneRanges();
    n = (int64_t)r.size();
    for (int64_t i = 0; i < n && i < cap && out != nullptr; i++) {
      out[2 * i] = r[(size_t)i].off;
      out[2 * i + 1] = r[(size_t)i].len;
    }
    return GLX_OK;
  });
  return n;
}

int64_t glx_algorithm_bytes_sent(glx_algorithm* alg) {
  return alg && alg->a ? alg->a->bytesSentPerRun() : -1;
}

int glx_algorithm_engine(glx_algorithm* alg) {
  if (alg == nullptr) return -1;
  return alg->a ? alg->a->engine() : GLX_ENGINE_HOSTFN;
}

int glx_set_device_sync(int mode) {
  if (mode < -1 || mode > 5) return fail(GLX_ERR_INVALID, "glx_set_device_sync: -1 .. 5");
  gloo::HipPlanExecutor::setDeviceSync(mode);
  return GLX_OK;
}

int glx_algorithm_sync(glx_algorithm* alg) {
  return alg != nullptr && alg->a ? alg->a->syncMode() : -1;
}

int glx_algorithm_fast_streams(glx_algorithm* alg) {
  return alg != nullptr && alg->a && alg->a->fastStreams() ? 1 : 0;
}

int glx_algorithm_transport_stats(glx_algorithm* alg, int64_t* out, int cap) {
  if (alg == nullptr || out == nullptr || cap < 6) {
    fail(GLX_ERR_INVALID, "glx_algorithm_transport_stats: null algorithm/output or cap < 6");
    return -1;
  }
  if (!alg->a) {  // a host-function algorithm moves nothing over the links
    for (int i = 0; i < cap && i < 8; i++) out[i] = 0;
    return cap < 8 ? cap : 8;
  }
  const auto& t = alg->a->transportStats();
  out[0] = t.peerCopies;
  out[1] = t.deviceCopies;
  out[2] = t.kernelCopies;
  out[3] = t.deviceKernels;
  out[4] = t.bytes;
  out[5] = t.hostFolds;
  if (cap < 7) return 6;
  out[6] = t.doneEvents;
  if (cap < 8) return 7;
  out[7] = t.flagKernels;
  return 8;
}

int glx_algorithm_record(glx_algorithm* alg, glx_event_t ev) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ev != nullptr, "null event");
    planExecutor(alg, "record").recordDone((hipEvent_t)ev);
    return GLX_OK;
  });
}

int glx_context_peer_info(glx_context* ctx, int peer, int* info) {
  return guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr && info != nullptr, "null argument");
    GLX_ENFORCE(ctx->c->connected(), "context not connected");
    GLX_ENFORCE(peer >= 0 && peer < ctx->c->size, "peer ", peer, " out of range");
    const gloo::PeerEndpoint& p = ctx->c->peer(peer);
    const gloo::PeerEndpoint& me = ctx->c->peer(ctx->c->rank);
    info[0] = p.localDevice;
    info[1] = (!p.busId.empty() && p.busId == me.busId) ||
                      (p.busId.empty() && p.pid == me.pid && p.device == me.device)
                  ? 1
                  : 0;
    info[2] = p.canAccessPeer;
    info[3] = p.nativeAtomics;
    info[4] = ctx->c->flagStores() ? 1 : 0;
    return GLX_OK;
  });
}

glx_link_probe* glx_link_probe_create(glx_context* ctx, size_t bytes) {
  glx_link_probe* out = nullptr;
  guarded([&]() -> int {
    GLX_ENFORCE(ctx != nullptr, "null context");
    out = new glx_link_probe{std::unique_ptr<gloo::LinkProbe>(new gloo::LinkProbe(ctx->c, bytes))};
    return GLX_OK;
  });
  return out;
}

int glx_link_probe_run(glx_link_probe* probe, int pattern, int engine, int blocks, int reps,
                       double* seconds, size_t* link_bytes) {
  return guarded([&]() -> int {
    GLX_ENFORCE(probe != nullptr && seconds != nullptr, "null argument");
    *seconds = probe->p->run(pattern, engine, blocks, reps);
    if (link_bytes != nullptr) *link_bytes = probe->p->busiestLinkBytes(pattern);
    return GLX_OK;
  });
}

void glx_link_probe_destroy(glx_link_probe* probe) {
  guarded([&]() -> int {
    delete probe;
    return GLX_OK;
  });
}

int glx_context_ipc_stats(glx_context* ctx, int64_t* imports, int64_t* base_fixups) {
  if (ctx == nullptr) return fail(GLX_ERR_INVALID, "null context");
  if (imports) *imports = ctx->c->ipcImports();
  if (base_fixups) *base_fixups = ctx->c->ipcBaseFixups();
  return GLX_OK;
}

int glx_event_create(glx_event_t* ev) {
  if (ev == nullptr) return fail(GLX_ERR_INVALID, "glx_event_create: null output");
  hipEvent_t e = nullptr;
  const int rc = hipStatus(hipEventCreateWithFlags(&e, hipEventDisableTiming),
                           "hipEventCreateWithFlags");
  *ev = rc == GLX_OK ? (glx_event_t)e : nullptr;
  return rc;
}

int glx_event_destroy(glx_event_t ev) {
  if (ev == nullptr) return GLX_OK;
  return hipStatus(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy");
}

int glx_event_record(glx_event_t ev, glx_stream_t stream) {
  if (ev == nullptr) return fail(GLX_ERR_INVALID, "glx_event_record: null event");
  return hipStatus(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream), "hipEventRecord");
}

int glx_event_query(glx_event_t ev) {
  if (ev == nullptr) return fail(GLX_ERR_INVALID, "glx_event_query: null event");
  const hipError_t e = hipEventQuery((hipEvent_t)ev);
  if (e == hipErrorNotReady) {
    (void)hipGetLastError();
    return GLX_NOT_READY;
  }
  return hipStatus(e, "hipEventQuery");
}

int glx_event_wait(glx_event_t ev, glx_stream_t stream) {
  if (ev == nullptr) return fail(GLX_ERR_INVALID, "glx_event_wait: null event");
  if (stream == nullptr) {
    return hipStatus(hipEventSynchronize((hipEvent_t)ev), "hipEventSynchronize");
  }
  return hipStatus(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0),
                   "hipStreamWaitEvent");
}

void glx_algorithm_destroy(glx_algorithm* alg) {
  guarded([&]() -> int {
    delete alg;
    return GLX_OK;
  });
}

// ---- plan introspection --------------------------------------------------------

int64_t glx_plan(int algo, int rank, int size, int64_t count, int64_t* steps, int64_t cap,
                 int64_t* scratch_elems) {
  return glx_plan_ex(algo, rank, size, count, 4, 0, glx::PlanParams().minPieceBytes, steps,
                     cap, scratch_elems);
}

int64_t glx_plan_ex(int algo, int rank, int size, int64_t count, int esize,
                    int64_t max_segment_bytes, int64_t min_piece_bytes, int64_t* steps,
                    int64_t cap, int64_t* scratch_elems) {
  int64_t n = -1;
  guarded([&]() -> int {
    glx::Plan p = glx::makePlan(algo, rank, size, count,
                                planParams(esize, max_segment_bytes, min_piece_bytes));
    n = (int64_t)p.steps.size();
    if (scratch_elems) *scratch_elems = p.scratch_elems;
    for (int64_t i = 0; i < n && i < cap && steps != nullptr; i++) {
      const glx::Step& s = p.steps[(size_t)i];
      int64_t* o = steps + 8 * i;
      o[0] = s.kind;
      o[1] = s.peer;
      o[2] = s.channel;
      o[3] = s.off;
      o[4] = s.len;
      o[5] = s.boff;
      o[6] = s.dst_off;
      o[7] = s.flags;
    }
    return GLX_OK;
  });
  return n;
}

int64_t glx_plan_stage(int algo, int rank, int size, int64_t count, int esize,
                       int64_t max_piece, int64_t* h2d, int64_t h2d_cap, int64_t* d2h,
                       int64_t d2h_cap, int64_t* n_d2h) {
  int64_t n = -1;
  guarded([&]() -> int {
    glx::Plan p = glx::makePlan(algo, rank, size, count,
                                planParams(esize, 0, glx::PlanParams().minPieceBytes));
    glx::StagePlan sp = glx::stagePlan(p, count, max_piece);
    n = (int64_t)sp.h2d.size();
    for (int64_t i = 0; i < n && i < h2d_cap && h2d != nullptr; i++) {
      h2d[2 * i] = sp.h2d[(size_t)i].off;
      h2d[2 * i + 1] = sp.h2d[(size_t)i].len;
    }
    int64_t k = 0;
    auto put = [&](int64_t step, const glx::Range& r) {
      if (k < d2h_cap && d2h != nullptr) {
        d2h[3 * k] = step;
        d2h[3 * k + 1] = r.off;
        d2h[3 * k + 2] = r.len;
      }
      k++;
    };
    for (size_t i = 0; i < sp.d2h.size(); i++) {
      for (const auto& r : sp.d2h[i]) put((int64_t)i, r);
    }
    for (const auto& r : sp.d2hRest) put(-1, r);
    if (n_d2h) *n_d2h = k;
    return GLX_OK;
  });
  return n;
}

int64_t glx_plan_sync(int algo, int rank, int size, int64_t count, int esize,
                      int64_t max_segment_bytes, int64_t min_piece_bytes, int G,
                      int64_t* bounds, int64_t bounds_cap, int64_t* nbounds, int64_t* info,
                      int64_t* steps, int64_t cap) {
  int64_t n = -1;
  guarded([&]() -> int {
    const glx::SyncTable t = glx::syncTable(
        algo, rank, size, count, planParams(esize, max_segment_bytes, min_piece_bytes), G);
    n = (int64_t)t.steps.size();
    if (info) {
      info[0] = t.slice;
      info[1] = t.safe ? 1 : 0;
      info[2] = t.slots;
    }
    if (nbounds) *nbounds = (int64_t)t.bounds.size();
    for (int64_t i = 0; i < (int64_t)t.bounds.size() && i < bounds_cap && bounds != nullptr;
         i++) {
      bounds[i] = t.bounds[(size_t)i];
    }
    // cap counts int64 slots: step i is written only when all of
    // its GLX_PLAN_SYNC_WIDTH words fit
    for (int64_t i = 0; i < n && (i + 1) * GLX_PLAN_SYNC_WIDTH <= cap && steps != nullptr; i++) {
      const glx::StepSync& y = t.steps[(size_t)i];
      int64_t* o = steps + GLX_PLAN_SYNC_WIDTH * i;
      o[0] = y.chan;
      o[1] = y.seg0;
      o[2] = y.seg1;
      o[3] = (int64_t)y.seq;
      o[4] = (int64_t)y.perRun;
      o[5] = y.fuse;
      o[6] = (int64_t)y.rseq;
      o[7] = (int64_t)y.rperRun;
      o[8] = y.keep;
      o[9] = y.pre;
      o[10] = y.pre0;
      o[11] = y.pre1;
    }
    return GLX_OK;
  });
  return n;
}

int64_t glx_device_layout(int algo, int rank, int size, int64_t count, int esize,
                          int64_t max_slices, int64_t* out, int64_t cap) {
  int64_t n = -1;
  guarded([&]() -> int {
    const bool oneShot = algo == GLX_ALGO_RING_CHUNKED_REPL || algo == glx::ALGO_FN_RING_REPL;
    const bool twoShot = algo == GLX_ALGO_RING_CHUNKED_MESH || algo == glx::ALGO_FN_RING_MESH;
    GLX_ENFORCE(oneShot || twoShot, "glx_device_layout: not a replicated or mesh schedule");
    GLX_ENFORCE(esize == 1 || esize == 2 || esize == 4 || esize == 8, "bad element size");
    glx::Plan p = glx::makePlan(algo, rank, size, count,
                                planParams(esize, 0, glx::PlanParams().minPieceBytes));
    const glx::DeviceLayout d =
        oneShot ? glx::oneShotLayout(p, rank, size, count, esize, max_slices)
                : glx::twoShotLayout(p, rank, size, count, esize, max_slices);
    std::vector<int64_t> v = {d.G, d.slice, d.maxLen, d.njobs};
    const int K = glx::kDevMaxRanks;
    for (int q = 0; q < K; q++) v.push_back(d.jobOff[q]);
    for (int q = 0; q < K; q++) v.push_back(d.jobLen[q]);
    for (int q = 0; q < K; q++)
      for (int i = 0; i < K; i++) v.push_back(d.chain[q][i]);
    for (int c = 0; c < K; c++) v.push_back(d.rangeOff[c]);
    for (int c = 0; c < K; c++) v.push_back(d.rangeLen[c]);
    for (int i = 0; i < K; i++) v.push_back(d.myChain[i]);
    n = (int64_t)v.size();
    for (int64_t i = 0; i < n && i < cap && out != nullptr; i++) out[i] = v[(size_t)i];
    return GLX_OK;
  });
  return n;
}

int64_t glx_plan_fold(int algo, int rank, int size, int64_t count, int64_t fold,
                      int64_t* srcs, int64_t cap) {
  return glx_plan_fold_ex(algo, rank, size, count, 4, 0, glx::PlanParams().minPieceBytes,
                          fold, srcs, cap);
}

int64_t glx_plan_fold_ex(int algo, int rank, int size, int64_t count, int esize,
                         int64_t max_segment_bytes, int64_t min_piece_bytes, int64_t fold,
                         int64_t* srcs, int64_t cap) {
  int64_t n = -1;
  guarded([&]() -> int {
    glx::Plan p = glx::makePlan(algo, rank, size, count,
                                planParams(esize, max_segment_bytes, min_piece_bytes));
    GLX_ENFORCE(fold >= 0 && fold < (int64_t)p.folds.size(), "fold index out of range");
    const auto& f = p.folds[(size_t)fold];
    n = (int64_t)f.size();
    for (int64_t i = 0; i < n && i < cap && srcs != nullptr; i++) srcs[i] = f[(size_t)i];
    return GLX_OK;
  });
  return n;
}

}  // extern "C"
