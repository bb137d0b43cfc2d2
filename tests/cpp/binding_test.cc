// binding_test.cc -- TEST INFRASTRUCTURE: integration/gloo/hip_allreduce.h
// (the header a gloo maintainer adds) compiled against the REFERENCE's own
// headers (/root/reference) and linked with the reference's objects
// (oracle/_ref/obj: its Context, rendezvous stores, tcp transport,
// AllreduceRingChunked) plus libgloo_amd.so.  Built by `make -C oracle
// binding` into oracle/_ref/binding_test.
//
//   binding_test cpu   no GPU: type / reduction-type mapping, CUSTOM refused
//                      on the device with gloo::EnforceNotMet and run on
//                      host buffers against the reference's own classes and
//                      gloo::allreduce, the store bridge both ways
//                      the endpoint exchange over the gloo context itself
//                      (ContextStore: gloo::allgather on the tcp pairs)
//   binding_test gpu   P thread-ranks on one GPU bootstrapped exactly like
//                      the reference's tests (HashStore + tcp loopback +
//                      rendezvous::Context::connectFullMesh, gloo/test/
//                      base_test.h:91-166); HipAllreduceRingChunked<float>,
//                      HipAllreduceHalvingDoubling<float16|int32>,
//                      HipAllreduceHalvingDoublingPipelined<float|float16>
//                      and the HipDeviceWorkspace instantiations built with
//                      the CUDA constructors' exact arguments (ctx, ptrs,
//                      count[, streams]) on device buffers; algorithms
//                      created and run in different interleavings per rank;
//                      gloo::hip::allreduce(AllreduceOptions) on the same
//                      options the reference's gloo::allreduce takes,
//                      compared bit for bit with the reference's own CPU
//                      algorithms run on host copies of the same inputs in
//                      the same process.
#include <execinfo.h>
#include <hip/hip_runtime_api.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <chrono>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "gloo/allreduce.h"
#include "gloo/allreduce_bcube.h"
#include "gloo/allreduce_halving_doubling.h"
#include "gloo/allreduce_local.h"
#include "gloo/allreduce_ring.h"
#include "gloo/allreduce_ring_chunked.h"
#include "gloo/hip_allreduce.h"
#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"

namespace {

int failures = 0;
int g_base = 2;  // gloo::Context::base of the contexts spawn() creates

#define EXPECT(cond, ...)                                 \
  do {                                                    \
    if (!(cond)) {                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s ", __FILE__, __LINE__, #cond); \
      std::fprintf(stderr, __VA_ARGS__);                  \
      std::fprintf(stderr, "\n");                         \
      failures++;                                         \
    }                                                     \
  } while (0)

uint64_t mix(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

template <typename T> T value(int r, size_t i);
template <> float value<float>(int r, size_t i) {
  return (float)((int64_t)(mix(((uint64_t)r << 40) ^ i) >> 40) - (1 << 23)) / (float)(1 << 23);
}
template <> int32_t value<int32_t>(int r, size_t i) {
  return (int32_t)(mix(((uint64_t)r << 40) ^ i) >> 44) - (1 << 19);
}
template <> uint64_t value<uint64_t>(int r, size_t i) {
  return mix(((uint64_t)r << 40) ^ i);
}
template <> gloo::float16 value<gloo::float16>(int r, size_t i) {
  return gloo::cpu_float2half_rn(value<float>(r, i));
}

void spawn(int P, const std::function<void(std::shared_ptr<gloo::Context>,
                                           gloo::rendezvous::Store&, int)>& fn);

void compareCustom(int P, int count, int nin, int nout, gloo::AllreduceOptions::Algorithm algo,
                   size_t maxSeg);
void compareClassCustom(int P, int count, int nptrs, bool hd);

void spawnCpu2(const std::function<void(std::shared_ptr<gloo::Context>,
                                        gloo::rendezvous::Store&, int)>& fn) {
  spawn(2, fn);
}

int cpuMode() {
  using namespace gloo;
  EXPECT(hip::GlxType<float>::value == GLX_FLOAT32, "float");
  EXPECT(hip::GlxType<float16>::value == GLX_FLOAT16, "float16");
  EXPECT(hip::GlxType<int32_t>::value == GLX_INT32, "int32");
  EXPECT(hip::glxOp(ReductionFunction<float>::sum) == GLX_SUM, "sum");
  EXPECT(hip::glxOp(ReductionFunction<float>::product) == GLX_PRODUCT, "product");
  EXPECT(hip::glxOp(ReductionFunction<float>::max) == GLX_MAX, "max");
  EXPECT(hip::glxOp(ReductionFunction<float>::min) == GLX_MIN, "min");
  ReductionFunction<float> custom(CUSTOM, [](float*, const float*, size_t) {});
  bool refused = false;
  try {
    hip::glxOp(&custom);
  } catch (const EnforceNotMet&) {
    refused = true;
  }
  EXPECT(refused, "CUSTOM must be refused with gloo::EnforceNotMet");
  // glx_* errors surface as gloo's exceptions
  bool io = false, enforce = false;
  try {
    hip::check(GLX_ERR_TIMEOUT, "probe");
  } catch (const IoException&) {
    io = true;
  }
  try {
    hip::check(GLX_ERR_INVALID, "probe");
  } catch (const EnforceNotMet&) {
    enforce = true;
  }
  EXPECT(io && enforce, "error mapping");
  // the store bridge, both ways, with a prefix
  rendezvous::HashStore hs;
  hip::StoreBridge bridge(hs, "pfx/");
  const char msg[] = "endpoint";
  EXPECT(glx_store_set(bridge.handle(), "a", msg, sizeof(msg)) == GLX_OK, "%s", glx_last_error());
  const auto got = hs.get("pfx/a");
  EXPECT(got.size() == sizeof(msg) && std::memcmp(got.data(), msg, sizeof(msg)) == 0, "set");
  hs.set("pfx/b", std::vector<char>(70000, 'x'));
  std::vector<char> buf(70000);
  size_t len = 0;
  EXPECT(glx_store_get(bridge.handle(), "b", buf.data(), buf.size(), &len, 1000) == GLX_OK,
         "%s", glx_last_error());
  EXPECT(len == 70000 && buf[69999] == 'x', "get");
  EXPECT(glx_store_get(bridge.handle(), "missing", buf.data(), buf.size(), &len, 30) ==
             GLX_ERR_TIMEOUT,
         "a missing key must time out");
  // two thread-ranks' gloo contexts get their xGMI contexts through the
  // shared registry at once (it must not serialise their connects)
  spawnCpu2([&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store& st, int) {
    auto x = hip::XgmiContext::of(ctx, &st, -1);
    EXPECT(x && x->get() != nullptr, "registry");
    EXPECT(hip::XgmiContext::of(ctx, &st, -1) == x, "one xGMI context per gloo context");
    EXPECT(hip::XgmiContext::of(ctx, nullptr, -1) == x, "the store does not split the registry");
  });
  // the drop-in's endpoint exchange over the gloo context alone (no store):
  // two thread-ranks connect their xGMI contexts through gloo::allgather
  spawnCpu2([&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int) {
    auto x = hip::XgmiContext::of(ctx, nullptr, -1);
    EXPECT(x && x->get() != nullptr, "connect over the gloo context");
    EXPECT(x->exchanges() == 2, "connect takes two exchanges (endpoints, mapped): %d",
           x->exchanges());
  });
  // the exchange store on its own: keys set by each rank are read by the
  // other after one collective exchange; a key nobody set fails at once
  // (one more exchange), not after the timeout
  spawnCpu2([&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
    hip::ContextStore cs(ctx);
    const std::string mine = "k/" + std::to_string(r), theirs = "k/" + std::to_string(1 - r);
    std::vector<char> val(3000 + (size_t)r, (char)('a' + r));
    EXPECT(glx_store_set(cs.handle(), mine.c_str(), val.data(), val.size()) == GLX_OK, "set");
    std::vector<char> buf(4096);
    size_t len = 0;
    EXPECT(glx_store_get(cs.handle(), theirs.c_str(), buf.data(), buf.size(), &len, 10000) ==
               GLX_OK, "get: %s", glx_last_error());
    EXPECT(len == 3000 + (size_t)(1 - r) && buf[0] == (char)('a' + 1 - r), "value");
    EXPECT(cs.exchanges() == 1, "one exchange: %d", cs.exchanges());
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = glx_store_get(cs.handle(), "never", buf.data(), buf.size(), &len, 20000);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    EXPECT(rc == GLX_ERR_IO && s < 5.0, "a key nobody set: rc %d after %.1f s", rc, s);
  });
  // exchange points that do not depend on what a rank already knows (ADVICE
  // r3): rank 0 creates A and B before running A, rank 1 creates B only after
  // running A.  Each first run is one exchange on every rank (sync()), its
  // reads strict; exchanging on a missed read instead, rank 1 would hold B0
  // from A's exchange, skip the one rank 0 starts at B's run, and both would
  // wait out the timeout.
  spawnCpu2([&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
    hip::ContextStore cs(ctx);
    std::vector<char> buf(64);
    size_t len = 0;
    auto set = [&](const std::string& k) {
      EXPECT(glx_store_set(cs.handle(), k.c_str(), k.data(), k.size()) == GLX_OK, "set");
    };
    auto firstRun = [&](const std::string& k) {  // what XgmiContext::firstRun does
      cs.sync();
      cs.setStrict(true);
      const int rc = glx_store_get(cs.handle(), k.c_str(), buf.data(), buf.size(), &len, 20000);
      cs.setStrict(false);
      EXPECT(rc == GLX_OK && len == k.size() && std::memcmp(buf.data(), k.data(), len) == 0,
             "rank %d reads %s: rc %d (%s)", r, k.c_str(), rc, glx_last_error());
    };
    const std::string peer = std::to_string(1 - r), me = std::to_string(r);
    if (r == 0) {
      set("A/" + me);
      set("B/" + me);
      firstRun("A/" + peer);
      firstRun("B/" + peer);
    } else {
      set("A/" + me);
      firstRun("A/" + peer);
      set("B/" + me);
      firstRun("B/" + peer);
    }
    EXPECT(cs.exchanges() == 2, "rank %d: two exchanges, one per first run: %d", r,
           cs.exchanges());
    // a strict read of a key nobody set fails at once, without an exchange
    cs.setStrict(true);
    EXPECT(glx_store_get(cs.handle(), "never", buf.data(), buf.size(), &len, 20000) ==
               GLX_ERR_IO && cs.exchanges() == 2,
           "strict miss");
    cs.setStrict(false);
  });
  // the CUDA type surface compiles with the type renamed
  static_assert(std::is_same<HipAllreduceRingChunked<float>,
                             HipAllreduceRingChunked<float, HipHostWorkspace<float>>>::value,
                "the host workspace is the default, as in the reference");
  static_assert(std::is_base_of<HipAllreduceHalvingDoubling<float16>,
                                HipAllreduceHalvingDoublingPipelined<float16>>::value,
                "Pipelined derives from HalvingDoubling, as in the reference");
  EXPECT(std::string(HipAllreduceRingChunked<float, HipDeviceWorkspace<float>>::workspace()) ==
             "device", "workspace tag");
  // two ranks' xGMI contexts connect through the bridge over one gloo store
  // (the endpoint exchange needs no GPU)
  {
    rendezvous::HashStore shared;
    std::vector<std::thread> ts;
    int rcs[2] = {-1, -1};
    for (int r = 0; r < 2; r++) {
      ts.emplace_back([&, r] {
        hip::StoreBridge b(shared, "cx/");
        glx_context* c = glx_context_create(r, 2, -1);
        rcs[r] = c ? glx_context_connect_full_mesh(c, b.handle()) : -2;
        glx_context_destroy(c);
      });
    }
    for (auto& t : ts) t.join();
    EXPECT(rcs[0] == GLX_OK && rcs[1] == GLX_OK, "connect through the bridge: %d %d (%s)",
           rcs[0], rcs[1], glx_last_error());
  }
  // a caller's Func on host buffers needs no GPU (glx_allreduce_host_fn)
  for (auto algo : {AllreduceOptions::Algorithm::RING, AllreduceOptions::Algorithm::BCUBE}) {
    compareCustom(2, 1000, 0, 1, algo, 0);
    compareCustom(3, 4099, 2, 1, algo, 1024);
    compareCustom(4, 65537, 1, 2, algo, 0);
  }
  // the class algorithms with a CUSTOM ReductionFunction on host buffers
  for (bool hd : {false, true}) {
    compareClassCustom(2, 1000, 1, hd);
    compareClassCustom(3, 4099, 2, hd);
    compareClassCustom(5, 65537, 1, hd);
  }
  std::printf("binding_test cpu: %s\n", failures ? "FAILED" : "OK");
  return failures ? 1 : 0;
}

// P thread-ranks as in gloo/test/base_test.h:91-166
void spawn(int P, const std::function<void(std::shared_ptr<gloo::Context>,
                                           gloo::rendezvous::Store&, int)>& fn) {
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  std::vector<std::thread> ts;
  std::vector<std::string> errs(P);
  for (int r = 0; r < P; r++) {
    ts.emplace_back([&, r] {
      try {
        gloo::transport::tcp::attr attr("127.0.0.1");
        auto dev = gloo::transport::tcp::CreateDevice(attr);
        auto ctx = std::make_shared<gloo::rendezvous::Context>(r, P, g_base);
        ctx->setTimeout(std::chrono::seconds(60));
        ctx->connectFullMesh(*store, dev);
        fn(ctx, *store, r);
      } catch (const std::exception& e) {
        errs[r] = e.what();
      }
    });
  }
  for (auto& t : ts) t.join();
  for (int r = 0; r < P; r++) EXPECT(errs[r].empty(), "rank %d: %s", r, errs[r].c_str());
}

enum Ctor { kDefault, kStreams, kViaStore };

template <typename T, template <typename> class Hip, template <typename> class Ref>
void compare(const char* name, int P, int count, int nptrs, const gloo::ReductionFunction<T>* fn,
             Ctor how = kDefault) {
  const bool viaStore = how == kViaStore;
  // inputs, and the reference's own CPU algorithm on host copies of them
  std::vector<std::vector<std::vector<T>>> in(P), ref(P), got(P);
  for (int r = 0; r < P; r++) {
    for (int k = 0; k < nptrs; k++) {
      std::vector<T> v((size_t)count);
      for (int i = 0; i < count; i++) v[(size_t)i] = value<T>(r * nptrs + k, (size_t)i);
      in[r].push_back(v);
    }
    ref[r] = in[r];
    got[r] = in[r];
  }
  std::printf("%s: reference CPU run\n", name);
  spawn(P, [&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
    std::vector<T*> ptrs;
    for (auto& v : ref[r]) ptrs.push_back(v.data());
    Ref<T> alg(ctx, ptrs, count, fn);
    alg.run();
  });
  std::printf("%s: HIP run\n", name);
  spawn(P, [&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store& store, int r) {
    std::vector<T*> dev;
    for (int k = 0; k < nptrs; k++) {
      T* d = nullptr;
      if (hipMalloc((void**)&d, sizeof(T) * (size_t)std::max(count, 1)) != hipSuccess) {
        throw std::runtime_error("hipMalloc");
      }
      hipMemcpy(d, in[r][(size_t)k].data(), sizeof(T) * (size_t)count, hipMemcpyHostToDevice);
      dev.push_back(d);
    }
    std::vector<hipStream_t> streams;
    if (how == kStreams) {  // one stream per pointer, as cuda_allreduce_test.cc passes them
      for (int k = 0; k < nptrs; k++) {
        hipStream_t st = nullptr;
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
          throw std::runtime_error("hipStreamCreate");
        }
        streams.push_back(st);
      }
    }
    {
      // the CUDA constructors' arguments; SUM needs no function at all
      std::unique_ptr<Hip<T>> a;
      // the Pipelined class has the CUDA one's four arguments only
      constexpr bool withFn =
          std::is_constructible<Hip<T>, std::shared_ptr<gloo::Context>, std::vector<T*>, int,
                                std::vector<hipStream_t>, const gloo::ReductionFunction<T>*>::value;
      // HipAllreduceLocal exchanges nothing, so it has no store overload
      constexpr bool withStore =
          std::is_constructible<Hip<T>, std::shared_ptr<gloo::Context>, gloo::rendezvous::Store&,
                                std::vector<T*>, int, std::vector<hipStream_t>,
                                const gloo::ReductionFunction<T>*>::value;
      if (how == kStreams) {
        a.reset(new Hip<T>(ctx, dev, count, streams));  // gloo/test/cuda_allreduce_test.cc:85-144
      } else if (fn == gloo::ReductionFunction<T>::sum && !viaStore) {
        a.reset(new Hip<T>(ctx, dev, count));
      } else if constexpr (withFn) {
        if (viaStore) {
          if constexpr (withStore) {
            a.reset(new Hip<T>(ctx, store, dev, count, {}, fn));
          } else {
            throw std::runtime_error("this class takes no store");
          }
        } else {
          a.reset(new Hip<T>(ctx, dev, count, {}, fn));
        }
      } else {
        throw std::runtime_error("this class takes no reduction function");
      }
      Hip<T>& alg = *a;
      for (int it = 0; it < 2; it++) {  // repeated runs on one instance
        for (int k = 0; k < nptrs && it > 0; k++) {
          hipMemcpy(dev[(size_t)k], in[r][(size_t)k].data(), sizeof(T) * (size_t)count,
                    hipMemcpyHostToDevice);
        }
        alg.run();
        // with streams the outputs are valid once the streams reach the end
        // of run() (docs/cuda.md:9-11)
        for (hipStream_t st : streams) hipStreamSynchronize(st);
      }
    }
    for (hipStream_t st : streams) hipStreamDestroy(st);
    for (int k = 0; k < nptrs; k++) {
      hipMemcpy(got[r][(size_t)k].data(), dev[(size_t)k], sizeof(T) * (size_t)count,
                hipMemcpyDeviceToHost);
      hipFree(dev[(size_t)k]);
    }
  });
  size_t bad = 0;
  for (int r = 0; r < P; r++) {
    for (int k = 0; k < nptrs; k++) {
      bad += std::memcmp(got[r][(size_t)k].data(), ref[r][(size_t)k].data(),
                         sizeof(T) * (size_t)count) != 0;
    }
  }
  EXPECT(bad == 0, "%s: %zu buffers differ from the reference", name, bad);
  std::printf("%s P=%d count=%d ptrs=%d%s: %s\n", name, P, count, nptrs,
              viaStore ? " (store)" : how == kStreams ? " (streams)" : "",
              bad ? "MISMATCH" : "ok");
}

// gloo::hip::allreduce(opts) against the reference's gloo::allreduce(opts):
// the same options (inputs or in-place outputs, algorithm, segment size, tag)
// built on each side, device buffers for the HIP call, host copies for the
// reference's.
template <typename T>
void compareFn(const char* name, int P, int count, int nin, int nout,
               gloo::AllreduceOptions::Algorithm algo, size_t maxSeg,
               void (*fn)(void*, const void*, const void*, size_t)) {
  std::vector<std::vector<std::vector<T>>> in(P), out0(P), ref(P), got(P);
  for (int r = 0; r < P; r++) {
    for (int k = 0; k < nin; k++) {
      std::vector<T> v((size_t)count);
      for (int i = 0; i < count; i++) v[(size_t)i] = value<T>(r * 8 + k, (size_t)i);
      in[r].push_back(v);
    }
    for (int k = 0; k < nout; k++) {
      std::vector<T> v((size_t)count);
      for (int i = 0; i < count; i++) v[(size_t)i] = value<T>(r * 8 + 4 + k, (size_t)i);
      out0[r].push_back(v);
    }
    ref[r] = out0[r];
    got[r] = out0[r];
  }
  auto setup = [&](gloo::AllreduceOptions& o, std::vector<T*>& ins, std::vector<T*>& outs) {
    o.setAlgorithm(algo);
    if (!ins.empty()) o.setInputs(ins, (size_t)count);
    o.setOutputs(outs, (size_t)count);
    o.setReduceFunction(fn);
    o.setTag(7);
    if (maxSeg > 0) o.setMaxSegmentSize(maxSeg);
  };
  spawn(P, [&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
    std::vector<std::vector<T>> hin = in[r];
    std::vector<T*> ins, outs;
    for (auto& v : hin) ins.push_back(v.data());
    for (auto& v : ref[r]) outs.push_back(v.data());
    gloo::AllreduceOptions o(ctx);
    setup(o, ins, outs);
    gloo::allreduce(o);
  });
  spawn(P, [&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
    std::vector<T*> ins, outs;
    auto upload = [&](const std::vector<T>& v) {
      T* d = nullptr;
      if (hipMalloc((void**)&d, sizeof(T) * (size_t)std::max(count, 1)) != hipSuccess) {
        throw std::runtime_error("hipMalloc");
      }
      hipMemcpy(d, v.data(), sizeof(T) * (size_t)count, hipMemcpyHostToDevice);
      return d;
    };
    for (auto& v : in[r]) ins.push_back(upload(v));
    for (auto& v : out0[r]) outs.push_back(upload(v));
    for (int it = 0; it < 2; it++) {  // the second call reuses the exchanged buffers
      for (int k = 0; k < nout && it > 0; k++) {
        hipMemcpy(outs[(size_t)k], out0[r][(size_t)k].data(), sizeof(T) * (size_t)count,
                  hipMemcpyHostToDevice);
      }
      gloo::AllreduceOptions o(ctx);
      setup(o, ins, outs);
      gloo::hip::allreduce(o);
    }
    for (int k = 0; k < nout; k++) {
      hipMemcpy(got[r][(size_t)k].data(), outs[(size_t)k], sizeof(T) * (size_t)count,
                hipMemcpyDeviceToHost);
    }
    for (T* d : ins) hipFree(d);
    for (T* d : outs) hipFree(d);
  });
  size_t bad = 0;
  for (int r = 0; r < P; r++) {
    for (int k = 0; k < nout; k++) {
      bad += std::memcmp(got[r][(size_t)k].data(), ref[r][(size_t)k].data(),
                         sizeof(T) * (size_t)count) != 0;
    }
  }
  EXPECT(bad == 0, "%s: %zu buffers differ from the reference", name, bad);
  std::printf("%s P=%d count=%d in=%d out=%d: %s\n", name, P, count, nin, nout,
              bad ? "MISMATCH" : "ok");
}

// A caller's AllreduceOptions::Func (gloo/allreduce.h:36,69,171) on HOST
// buffers: gloo::hip::allreduce runs it on the host in the reference's
// order; the reference's gloo::allreduce with the same std::function (a
// capturing closure, c = k*a + b over 32-bit words, neither commutative nor
// associative) on host copies gives the bits to match.  Two calls per rank,
// the second reusing the cached executor.
void compareCustom(int P, int count, int nin, int nout, gloo::AllreduceOptions::Algorithm algo,
                   size_t maxSeg) {
  const uint32_t k = 3;
  gloo::AllreduceOptions::Func f = [k](void* c, const void* a, const void* b, size_t n) {
    const uint32_t* x = static_cast<const uint32_t*>(a);
    const uint32_t* y = static_cast<const uint32_t*>(b);
    uint32_t* z = static_cast<uint32_t*>(c);
    for (size_t i = 0; i < n; i++) z[i] = k * x[i] + y[i];
  };
  using T = int32_t;
  std::vector<std::vector<std::vector<T>>> in(P), out0(P), ref(P), got(P);
  for (int r = 0; r < P; r++) {
    for (int j = 0; j < nin; j++) {
      std::vector<T> v((size_t)count);
      for (int i = 0; i < count; i++) v[(size_t)i] = value<T>(r * 8 + j, (size_t)i);
      in[r].push_back(v);
    }
    for (int j = 0; j < nout; j++) {
      std::vector<T> v((size_t)count);
      for (int i = 0; i < count; i++) v[(size_t)i] = value<T>(r * 8 + 4 + j, (size_t)i);
      out0[r].push_back(v);
    }
    ref[r] = out0[r];
  }
  auto run = [&](bool hip, std::vector<std::vector<std::vector<T>>>& outs) {
    spawn(P, [&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
      for (int it = 0; it < (hip ? 2 : 1); it++) {
        std::vector<std::vector<T>> hin = in[r];
        outs[r] = out0[r];
        std::vector<T*> ins, os;
        for (auto& v : hin) ins.push_back(v.data());
        for (auto& v : outs[r]) os.push_back(v.data());
        gloo::AllreduceOptions o(ctx);
        o.setAlgorithm(algo);
        if (!ins.empty()) o.setInputs(ins, (size_t)count);
        o.setOutputs(os, (size_t)count);
        o.setReduceFunction(f);
        if (maxSeg > 0) o.setMaxSegmentSize(maxSeg);
        if (hip) {
          gloo::hip::allreduce(o);
        } else {
          gloo::allreduce(o);
        }
      }
    });
  };
  run(false, ref);
  run(true, got);
  size_t bad = 0;
  for (int r = 0; r < P; r++) {
    for (int j = 0; j < nout; j++) {
      bad += std::memcmp(got[r][(size_t)j].data(), ref[r][(size_t)j].data(),
                         sizeof(T) * (size_t)count) != 0;
    }
  }
  EXPECT(bad == 0, "custom Func: %zu buffers differ from the reference", bad);
  std::printf("custom Func (host) %s P=%d count=%d in=%d out=%d seg=%zu: %s\n",
              algo == gloo::AllreduceOptions::Algorithm::BCUBE ? "bcube" : "ring", P, count,
              nin, nout, maxSeg, bad ? "MISMATCH" : "ok");
}

// HipAllreduceRingChunked / HipAllreduceHalvingDoubling with a CUSTOM
// ReductionFunction<int32_t> (gloo/algorithm.h:56,58-83; x = 3x + y over
// 32-bit words, neither commutative nor associative) on HOST buffers,
// against the reference's own AllreduceRingChunked / AllreduceHalvingDoubling
// with the same function on copies of the same inputs.  Two runs of the
// HIP instance.
void classTimes3Plus(int32_t* x, const int32_t* y, size_t n) {
  for (size_t i = 0; i < n; i++) x[i] = (int32_t)(3u * (uint32_t)x[i] + (uint32_t)y[i]);
}

void compareClassCustom(int P, int count, int nptrs, bool hd) {
  using T = int32_t;
  static const gloo::ReductionFunction<T> fn(gloo::CUSTOM, &classTimes3Plus);
  std::vector<std::vector<std::vector<T>>> init(P), ref(P), got(P);
  for (int r = 0; r < P; r++) {
    for (int j = 0; j < nptrs; j++) {
      std::vector<T> v((size_t)count);
      for (int i = 0; i < count; i++) v[(size_t)i] = value<T>(r * 8 + j, (size_t)i);
      init[r].push_back(v);
    }
  }
  auto run = [&](bool hip, std::vector<std::vector<std::vector<T>>>& outs) {
    spawn(P, [&](std::shared_ptr<gloo::Context> ctx, gloo::rendezvous::Store&, int r) {
      std::vector<T*> ptrs;
      outs[r] = init[r];
      for (auto& v : outs[r]) ptrs.push_back(v.data());
      std::unique_ptr<gloo::Algorithm> a;
      if (hip && hd) {
        a.reset(new gloo::HipAllreduceHalvingDoubling<T>(ctx, ptrs, count, {}, &fn));
      } else if (hip) {
        a.reset(new gloo::HipAllreduceRingChunked<T>(ctx, ptrs, count, {}, &fn));
      } else if (hd) {
        a.reset(new gloo::AllreduceHalvingDoubling<T>(ctx, ptrs, count, &fn));
      } else {
        a.reset(new gloo::AllreduceRingChunked<T>(ctx, ptrs, count, &fn));
      }
      for (int it = 0; it < (hip ? 2 : 1); it++) {
        if (it > 0) {
          for (int j = 0; j < nptrs; j++) outs[r][(size_t)j] = init[r][(size_t)j];
        }
        a->run();
      }
    });
  };
  run(false, ref);
  run(true, got);
  size_t bad = 0;
  for (int r = 0; r < P; r++) {
    for (int j = 0; j < nptrs; j++) {
      bad += std::memcmp(got[r][(size_t)j].data(), ref[r][(size_t)j].data(),
                         sizeof(T) * (size_t)count) != 0;
    }
  }
  EXPECT(bad == 0, "CUSTOM ReductionFunction: %zu buffers differ from the reference", bad);
  std::printf("CUSTOM ReductionFunction (host) %s P=%d count=%d ptrs=%d: %s\n",
              hd ? "halving_doubling" : "ring_chunked", P, count, nptrs,
              bad ? "MISMATCH" : "ok");
}

template <typename T>
using RingDeviceWs = gloo::HipAllreduceRingChunked<T, gloo::HipDeviceWorkspace<T>>;
template <typename T>
using HdDeviceWs = gloo::HipAllreduceHalvingDoubling<T, gloo::HipDeviceWorkspace<T>>;

// Algorithms created and run in different interleavings on different ranks
// (legal: gloo constructors are local, runs are collective in one order).
// Rank 0: create A, create B, run A, run B; the others: create A, run A,
// create B, run B.  The endpoint exchanges over the gloo context must line up
// (ADVICE r3); both results against the reference's CPU algorithms.
void interleaved() {
  using namespace gloo;
  const int P = 3, count = 50001;
  std::vector<std::vector<float>> in(P), refA(P), refB(P), gotA(P), gotB(P);
  for (int r = 0; r < P; r++) {
    in[r].resize((size_t)count);
    for (int i = 0; i < count; i++) in[r][(size_t)i] = value<float>(r, (size_t)i);
    refA[r] = refB[r] = gotA[r] = gotB[r] = in[r];
  }
  spawn(P, [&](std::shared_ptr<Context> ctx, rendezvous::Store&, int r) {
    std::vector<float*> a{refA[r].data()}, b{refB[r].data()};
    AllreduceRingChunked<float>(ctx, a, count).run();
    AllreduceHalvingDoubling<float>(ctx, b, count).run();
  });
  spawn(P, [&](std::shared_ptr<Context> ctx, rendezvous::Store&, int r) {
    float *da = nullptr, *db = nullptr;
    if (hipMalloc((void**)&da, sizeof(float) * count) != hipSuccess ||
        hipMalloc((void**)&db, sizeof(float) * count) != hipSuccess) {
      throw std::runtime_error("hipMalloc");
    }
    hipMemcpy(da, in[r].data(), sizeof(float) * count, hipMemcpyHostToDevice);
    hipMemcpy(db, in[r].data(), sizeof(float) * count, hipMemcpyHostToDevice);
    std::vector<float*> pa{da}, pb{db};
    std::unique_ptr<HipAllreduceRingChunked<float>> A(
        new HipAllreduceRingChunked<float>(ctx, pa, count));
    std::unique_ptr<HipAllreduceHalvingDoublingPipelined<float>> B;
    if (r == 0) B.reset(new HipAllreduceHalvingDoublingPipelined<float>(ctx, pb, count));
    A->run();
    if (r != 0) B.reset(new HipAllreduceHalvingDoublingPipelined<float>(ctx, pb, count));
    B->run();
    EXPECT(A->exchanges() == 4, "rank %d: connect (2) + one per first run (2): %d", r,
           A->exchanges());
    hipMemcpy(gotA[r].data(), da, sizeof(float) * count, hipMemcpyDeviceToHost);
    hipMemcpy(gotB[r].data(), db, sizeof(float) * count, hipMemcpyDeviceToHost);
    A.reset();
    B.reset();
    hipFree(da);
    hipFree(db);
  });
  size_t bad = 0;
  for (int r = 0; r < P; r++) {
    bad += gotA[r] != refA[r];
    bad += gotB[r] != refB[r];
  }
  EXPECT(bad == 0, "interleaved creation: %zu buffers differ from the reference", bad);
  std::printf("interleaved creation/run (rank 0: A, B, run A, run B) P=%d: %s\n", P,
              bad ? "MISMATCH" : "ok");
}

// AllreduceLocal exchanges nothing: one rank creates and runs it while its
// peer does no gloo work at all (a collective inside would wait out the
// timeout), then the pair still runs a ring together.
void localAlone() {
  using namespace gloo;
  const int count = 70001;
  std::vector<float> a(count), b(count), want(count), got(count);
  for (int i = 0; i < count; i++) {
    a[(size_t)i] = value<float>(0, (size_t)i);
    b[(size_t)i] = value<float>(1, (size_t)i);
  }
  {
    std::vector<float> x = a, y = b;
    std::vector<float*> ptrs = {x.data(), y.data()};
    auto solo = std::make_shared<rendezvous::HashStore>();
    // the CPU AllreduceLocal on a one-rank context as the expected value
    auto ctx1 = std::make_shared<rendezvous::Context>(0, 1);
    transport::tcp::attr attr("127.0.0.1");
    auto dev = transport::tcp::CreateDevice(attr);
    ctx1->connectFullMesh(*solo, dev);
    AllreduceLocal<float>(ctx1, ptrs, count).run();
    want = x;
  }
  const auto t0 = std::chrono::steady_clock::now();
  spawn(2, [&](std::shared_ptr<Context> ctx, rendezvous::Store&, int r) {
    ctx->setTimeout(std::chrono::seconds(5));
    if (r == 0) {
      float* d[2];
      for (int k = 0; k < 2; k++) {
        if (hipMalloc((void**)&d[k], sizeof(float) * count) != hipSuccess) {
          throw std::runtime_error("hipMalloc");
        }
        hipMemcpy(d[k], (k ? b : a).data(), sizeof(float) * count, hipMemcpyHostToDevice);
      }
      HipAllreduceLocal<float> l(ctx, {d[0], d[1]}, count);
      l.run();
      hipMemcpy(got.data(), d[1], sizeof(float) * count, hipMemcpyDeviceToHost);
      for (float* p : d) hipFree(p);
    }
  });
  const double secs =
      std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  const bool same = std::memcmp(got.data(), want.data(), sizeof(float) * count) == 0;
  EXPECT(same, "local alone: result differs from the reference");
  EXPECT(secs < 4.0, "local alone took %.1f s (waited for the idle peer?)", secs);
  std::printf("local<float> on one rank of two, peer idle: %s (%.2f s)\n",
              same && secs < 4.0 ? "ok" : "FAILED", secs);
}

int gpuMode() {
  using namespace gloo;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n < 1) {
    std::printf("binding_test gpu: no GPU\n");
    return 2;
  }
  compare<float, HipAllreduceRingChunked, AllreduceRingChunked>(
      "ring_chunked<float> sum", 2, 100003, 1, ReductionFunction<float>::sum);
  compare<float, HipAllreduceRingChunked, AllreduceRingChunked>(
      "ring_chunked<float> max", 3, 4099, 2, ReductionFunction<float>::max);
  compare<float16, HipAllreduceHalvingDoubling, AllreduceHalvingDoubling>(
      "halving_doubling<float16> sum", 4, 65539, 1, ReductionFunction<float16>::sum);
  compare<int32_t, HipAllreduceHalvingDoubling, AllreduceHalvingDoubling>(
      "halving_doubling<int32> product", 3, 1000, 1, ReductionFunction<int32_t>::product);
  compare<float, HipAllreduceRingChunked, AllreduceRingChunked>(
      "ring_chunked<float> sum", 2, 4099, 1, ReductionFunction<float>::sum, kViaStore);
  // the reference CUDA test's factories (gloo/test/cuda_allreduce_test.cc:
  // 85-144) with the type renamed: <T> with (ctx, ptrs, count, streams), the
  // pipelined halving-doubling, and the device-workspace instantiations
  // (cuda_allreduce_ring_chunked.cc:361, cuda_allreduce_halving_doubling.cc:647)
  compare<float, HipAllreduceRingChunked, AllreduceRingChunked>(
      "ring_chunked<float> (ctx, ptrs, count, streams)", 3, 70001, 2,
      ReductionFunction<float>::sum, kStreams);
  compare<float16, HipAllreduceHalvingDoubling, AllreduceHalvingDoubling>(
      "halving_doubling<float16> (ctx, ptrs, count, streams)", 3, 40961, 2,
      ReductionFunction<float16>::sum, kStreams);
  compare<float, HipAllreduceHalvingDoublingPipelined, AllreduceHalvingDoubling>(
      "halving_doubling_pipelined<float>", 4, 100003, 2, ReductionFunction<float>::sum, kStreams);
  compare<float16, HipAllreduceHalvingDoublingPipelined, AllreduceHalvingDoubling>(
      "halving_doubling_pipelined<float16>", 5, 65539, 1, ReductionFunction<float16>::sum);
  compare<float, RingDeviceWs, AllreduceRingChunked>(
      "ring_chunked<float, HipDeviceWorkspace>", 2, 100003, 1, ReductionFunction<float>::sum,
      kStreams);
  compare<float, HdDeviceWs, AllreduceHalvingDoubling>(
      "halving_doubling<float, HipDeviceWorkspace>", 3, 100003, 1, ReductionFunction<float>::sum);
  // CudaAllreduceRing<T>(context, ptrs, count, streams) (cuda_allreduce_test.cc:75-91)
  // against the CPU AllreduceRing<T>: every rank's own fold order
  compare<float, HipAllreduceRing, AllreduceRing>(
      "ring<float> (ctx, ptrs, count, streams)", 5, 100003, 2, ReductionFunction<float>::sum,
      kStreams);
  compare<float16, HipAllreduceRing, AllreduceRing>(
      "ring<float16>", 3, 65539, 1, ReductionFunction<float16>::sum);
  compare<float, HipAllreduceRing, AllreduceRing>(
      "ring<float> max", 4, 4099, 1, ReductionFunction<float>::max);
  // CudaAllreduceBcube<T>(context, ptrs, count, streams) (cuda_allreduce_test.cc:
  // 93-110) against the CPU AllreduceBcube<T>, contexts with base 2 and 3
  compare<float, HipAllreduceBcube, AllreduceBcube>(
      "bcube<float> base 2 (ctx, ptrs, count, streams)", 4, 100003, 2,
      ReductionFunction<float>::sum, kStreams);
  g_base = 3;
  compare<float16, HipAllreduceBcube, AllreduceBcube>(
      "bcube<float16> base 3", 9, 4099, 1, ReductionFunction<float16>::sum);
  compare<float, HipAllreduceBcube, AllreduceBcube>(
      "bcube<float> base 3, P = 5", 5, 1000, 1, ReductionFunction<float>::max);
  g_base = 2;
  // CudaAllreduceLocal<T>(context, ptrs, count, streams) (cuda_allreduce_local.h:21-27)
  // against the CPU AllreduceLocal<T> (allreduce_local.cc:21-31)
  compare<float, HipAllreduceLocal, AllreduceLocal>(
      "local<float> (ctx, ptrs, count, streams)", 2, 100003, 3, ReductionFunction<float>::sum,
      kStreams);
  compare<float16, HipAllreduceLocal, AllreduceLocal>(
      "local<float16> max", 3, 65539, 4, ReductionFunction<float16>::max);
  compare<int32_t, HipAllreduceLocal, AllreduceLocal>(
      "local<int32> product", 1, 4099, 2, ReductionFunction<int32_t>::product);
  localAlone();
  interleaved();
  using MathFn = void (*)(void*, const void*, const void*, size_t);
  compareFn<float>("allreduce(opts) RING float sum", 3, 100003, 0, 1,
                   AllreduceOptions::Algorithm::RING, 0, (MathFn)&gloo::sum<float>);
  compareFn<float>("allreduce(opts) RING float sum, 2 in, 2 out, 128 B segments", 4, 10000, 2, 2,
                   AllreduceOptions::Algorithm::RING, 128, (MathFn)&gloo::sum<float>);
  compareFn<float16>("allreduce(opts) BCUBE float16 max", 4, 65539, 1, 1,
                     AllreduceOptions::Algorithm::BCUBE, 0, (MathFn)&gloo::max<float16>);
  compareFn<uint64_t>("allreduce(opts) RING uint64 sum", 7, 1000, 0, 3,
                      AllreduceOptions::Algorithm::RING, 128, (MathFn)&gloo::sum<uint64_t>);
  compareFn<int32_t>("allreduce(opts) UNSPECIFIED int32 min", 2, 5000, 1, 1,
                     AllreduceOptions::Algorithm::UNSPECIFIED, 0, (MathFn)&gloo::min<int32_t>);
  std::printf("binding_test gpu: %s\n", failures ? "FAILED" : "OK");
  return failures ? 1 : 0;
}

}  // namespace

void onFault(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  dprintf(2, "binding_test: signal %d, backtrace:\n", sig);
  backtrace_symbols_fd(frames, n, 2);
  _exit(128 + sig);
}

int main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IONBF, 0);
  signal(SIGSEGV, onFault);
  signal(SIGABRT, onFault);
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  return mode == "gpu" ? gpuMode() : cpuMode();
}
