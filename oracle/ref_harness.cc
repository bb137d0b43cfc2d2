// ref_harness.cc -- TEST INFRASTRUCTURE ONLY (built into oracle/_ref/).
//
// A thin extern "C" shim over the REFERENCE implementation itself: it
// includes the reference headers from /root/reference and is linked against
// the reference's own tcp/rendezvous/core sources (compiled verbatim from
// /root/reference by oracle/Makefile -- nothing is copied into this repo).
// It lets the Python test-suite (and bench.py's cpu_baseline leg) run
//   * gloo::sum/product/max/min<T>            (gloo/math.h:15-73)
//   * gloo::AllreduceRingChunked<T>           (gloo/allreduce_ring_chunked.h:19)
//   * gloo::AllreduceHalvingDoubling<T>       (gloo/allreduce_halving_doubling.h:37)
//   * gloo::AllreduceRing<T>                  (gloo/allreduce_ring.h:20)
//   * gloo::AllreduceBcube<T>                 (gloo/allreduce_bcube.h:256)
//   * gloo::allreduce(AllreduceOptions)       (gloo/allreduce.cc:97-146, RING/BCUBE)
// exactly the way the reference's tests do: P threads in one process, one
// HashStore, tcp devices on loopback (gloo/test/base_test.h:91-166).
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <exception>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "gloo/allreduce.h"
#include "gloo/allreduce_halving_doubling.h"
#include "gloo/allreduce_bcube.h"
#include "gloo/allreduce_ring.h"
#include "gloo/allreduce_ring_chunked.h"
#include "gloo/math.h"
#include "gloo/rendezvous/context.h"
#include "gloo/rendezvous/hash_store.h"
#include "gloo/transport/tcp/device.h"
#include "gloo/types.h"

namespace {

int g_bcube_base = 2;  // gloo::Context::base for AllreduceBcube (ref_set_bcube_base)

enum { R_INT8 = 0, R_UINT8, R_INT32, R_INT64, R_UINT64, R_FLOAT32, R_FLOAT64,
       R_FLOAT16, R_BFLOAT16 };
enum { R_SUM = 1, R_PRODUCT = 2, R_MAX = 3, R_MIN = 4 };
// Caller-supplied reduction functions (AllreduceOptions::Func,
// gloo/allreduce.h:36,69,171) for the custom-function fixtures, over 32-bit
// words: a bitwise or, and c = 3a + b (mod 2^32) -- neither commutative nor
// associative, so the output bits pin the order and operands of every call.
enum { R_CUSTOM_OR = 100, R_CUSTOM_3A_PLUS_B = 101 };

void customOr(void* c, const void* a, const void* b, size_t n) {
  const uint32_t* x = static_cast<const uint32_t*>(a);
  const uint32_t* y = static_cast<const uint32_t*>(b);
  uint32_t* z = static_cast<uint32_t*>(c);
  for (size_t i = 0; i < n; i++) z[i] = x[i] | y[i];
}

void custom3aPlusB(void* c, const void* a, const void* b, size_t n) {
  const uint32_t* x = static_cast<const uint32_t*>(a);
  const uint32_t* y = static_cast<const uint32_t*>(b);
  uint32_t* z = static_cast<uint32_t*>(c);
  for (size_t i = 0; i < n; i++) z[i] = 3u * x[i] + y[i];
}

// The same two functions as ReductionFunction<T>s of type CUSTOM for the
// class algorithms (gloo/algorithm.h:58-83: Function(T* x, const T* y, n),
// x = f(x, y) in place), over 4-byte T.
template <typename T>
void classOr(T* x, const T* y, size_t n) { customOr(x, x, y, n); }
template <typename T>
void class3aPlusB(T* x, const T* y, size_t n) { custom3aPlusB(x, x, y, n); }

thread_local std::string g_err;

template <typename T>
int reduceT(int op, void* c, const void* a, const void* b, size_t n) {
  switch (op) {
    case R_SUM: gloo::sum<T>(c, a, b, n); return 0;
    case R_PRODUCT: gloo::product<T>(c, a, b, n); return 0;
    case R_MAX: gloo::max<T>(c, a, b, n); return 0;
    case R_MIN: gloo::min<T>(c, a, b, n); return 0;
  }
  return -1;
}

template <typename T>
const gloo::ReductionFunction<T>* fnFor(int op) {
  switch (op) {
    case R_SUM: return gloo::ReductionFunction<T>::sum;
    case R_PRODUCT: return gloo::ReductionFunction<T>::product;
    case R_MAX: return gloo::ReductionFunction<T>::max;
    case R_MIN: return gloo::ReductionFunction<T>::min;
  }
  if constexpr (sizeof(T) == 4) {
    static const gloo::ReductionFunction<T> orFn(gloo::CUSTOM, &classOr<T>);
    static const gloo::ReductionFunction<T> threeAPlusBFn(gloo::CUSTOM, &class3aPlusB<T>);
    if (op == R_CUSTOM_OR) return &orFn;
    if (op == R_CUSTOM_3A_PLUS_B) return &threeAPlusBFn;
  }
  return nullptr;
}

// Runs `iters` back-to-back run() calls of one algorithm instance on every
// rank (after `warmup` untimed calls).  Rank 0 reports the wall time of the
// timed calls.  bufs[r * nptrs + i] is rank r's i-th buffer.
template <typename T>
int allreduceT(int algo, int op, int P, int nptrs, int count, void** bufs,
               int warmup, int iters, double* seconds) {
  auto fn = fnFor<T>(op);
  if (fn == nullptr) return -1;
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  std::vector<std::thread> threads;
  std::vector<std::string> errors(P);
  std::mutex doneMu;
  std::condition_variable doneCv;
  int done = 0;
  for (int r = 0; r < P; r++) {
    threads.emplace_back([&, r]() {
      try {
        gloo::transport::tcp::attr attr("127.0.0.1");
        auto dev = gloo::transport::tcp::CreateDevice(attr);
        auto ctx = std::make_shared<gloo::rendezvous::Context>(r, P, g_bcube_base);
        ctx->connectFullMesh(*store, dev);
        std::vector<T*> ptrs;
        for (int i = 0; i < nptrs; i++) {
          ptrs.push_back(static_cast<T*>(bufs[r * nptrs + i]));
        }
        std::unique_ptr<gloo::Algorithm> alg;
        if (algo == 0) {
          alg.reset(new gloo::AllreduceRingChunked<T>(ctx, ptrs, count, fn));
        } else if (algo == 9) {
          alg.reset(new gloo::AllreduceRing<T>(ctx, ptrs, count, fn));
        } else if (algo == 10) {
          alg.reset(new gloo::AllreduceBcube<T>(ctx, ptrs, count, fn));
        } else {
          alg.reset(new gloo::AllreduceHalvingDoubling<T>(ctx, ptrs, count, fn));
        }
        for (int i = 0; i < warmup; i++) alg->run();
        auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < iters; i++) alg->run();
        auto t1 = std::chrono::steady_clock::now();
        if (r == 0 && seconds != nullptr) {
          *seconds = std::chrono::duration<double>(t1 - t0).count();
        }
        // every rank's run() has returned before any tears its pairs down:
        // AllreduceRing's last notification (allreduce_ring.h:104-108) may
        // still be in flight when a neighbour is done
        {
          std::unique_lock<std::mutex> lk(doneMu);
          if (++done >= P) doneCv.notify_all();
          doneCv.wait(lk, [&] { return done >= P; });
        }
      } catch (const std::exception& e) {
        errors[r] = e.what();
        std::lock_guard<std::mutex> lk(doneMu);  // count this rank for the barrier
        if (++done >= P) doneCv.notify_all();
      }
    });
  }
  for (auto& t : threads) t.join();
  for (int r = 0; r < P; r++) {
    if (!errors[r].empty()) {
      g_err = "rank " + std::to_string(r) + ": " + errors[r];
      return -2;
    }
  }
  return 0;
}

template <typename T>
gloo::AllreduceOptions::Func mathFn(int op) {
  void (*f)(void*, const void*, const void*, size_t) = nullptr;
  switch (op) {
    case R_CUSTOM_OR: f = &customOr; break;
    case R_CUSTOM_3A_PLUS_B: f = &custom3aPlusB; break;
    case R_SUM: f = &gloo::sum<T>; break;
    case R_PRODUCT: f = &gloo::product<T>; break;
    case R_MAX: f = &gloo::max<T>; break;
    case R_MIN: f = &gloo::min<T>; break;
  }
  return gloo::AllreduceOptions::Func(f);
}

// One gloo::allreduce(opts) call on every rank (gloo/test/allreduce_test.cc:
// 306-356 shows the options the reference's own tests use).
template <typename T>
int allreduceFnT(int algo, int op, int P, int nin, int nout, size_t count, size_t maxSeg,
                 void** ins, void** outs) {
  const bool custom = op == R_CUSTOM_OR || op == R_CUSTOM_3A_PLUS_B;
  if (custom ? sizeof(T) != 4 : (op < R_SUM || op > R_MIN)) return -1;
  auto store = std::make_shared<gloo::rendezvous::HashStore>();
  std::vector<std::thread> threads;
  std::vector<std::string> errors(P);
  for (int r = 0; r < P; r++) {
    threads.emplace_back([&, r]() {
      try {
        gloo::transport::tcp::attr attr("127.0.0.1");
        auto dev = gloo::transport::tcp::CreateDevice(attr);
        auto ctx = std::make_shared<gloo::rendezvous::Context>(r, P);
        ctx->connectFullMesh(*store, dev);
        gloo::AllreduceOptions opts(ctx);
        opts.setAlgorithm(algo == 2 ? gloo::AllreduceOptions::Algorithm::BCUBE
                                    : gloo::AllreduceOptions::Algorithm::RING);
        std::vector<T*> in, out;
        for (int i = 0; i < nin; i++) in.push_back(static_cast<T*>(ins[r * nin + i]));
        for (int i = 0; i < nout; i++) out.push_back(static_cast<T*>(outs[r * nout + i]));
        if (nin > 0) opts.setInputs(in, count);
        opts.setOutputs(out, count);
        opts.setReduceFunction(mathFn<T>(op));
        if (maxSeg > 0) opts.setMaxSegmentSize(maxSeg);
        gloo::allreduce(opts);
      } catch (const std::exception& e) {
        errors[r] = e.what();
      }
    });
  }
  for (auto& t : threads) t.join();
  for (int r = 0; r < P; r++) {
    if (!errors[r].empty()) {
      g_err = "rank " + std::to_string(r) + ": " + errors[r];
      return -2;
    }
  }
  return 0;
}

template <typename T>
int reduceSlices(int op, char* c, const char* a, const char* b, size_t n, int threads,
                 int iters, double* seconds) {
  if (threads < 1 || iters < 1) return -1;
  std::atomic<int> ready{0};
  std::atomic<bool> go{false};
  std::vector<std::thread> ts;
  const size_t per = (n + (size_t)threads - 1) / (size_t)threads;
  for (int t = 0; t < threads; t++) {
    ts.emplace_back([&, t]() {
      const size_t lo = std::min(n, (size_t)t * per), hi = std::min(n, lo + per);
      ready.fetch_add(1);
      while (!go.load()) std::this_thread::yield();
      for (int i = 0; i < iters; i++) {
        reduceT<T>(op, c + lo * sizeof(T), a + lo * sizeof(T), b + lo * sizeof(T), hi - lo);
      }
    });
  }
  while (ready.load() < threads) std::this_thread::yield();
  const auto t0 = std::chrono::steady_clock::now();
  go.store(true);
  for (auto& th : ts) th.join();
  const auto t1 = std::chrono::steady_clock::now();
  if (seconds != nullptr) *seconds = std::chrono::duration<double>(t1 - t0).count();
  return 0;
}

}  // namespace

extern "C" {

// The reference's gloo::sum/product/max/min<T> split over `threads` host
// threads (contiguous slices), each running its slice `iters` times; wall
// time of the whole in *seconds (the CPU baseline's N-thread leg).
int ref_reduce_mt(int op, int dtype, void* c, const void* a, const void* b, size_t n,
                  int threads, int iters, double* seconds) {
  char* cc = static_cast<char*>(c);
  const char* ca = static_cast<const char*>(a);
  const char* cb = static_cast<const char*>(b);
  switch (dtype) {
    case R_FLOAT32: return reduceSlices<float>(op, cc, ca, cb, n, threads, iters, seconds);
    case R_FLOAT16:
      return reduceSlices<gloo::float16>(op, cc, ca, cb, n, threads, iters, seconds);
    case R_INT32: return reduceSlices<int32_t>(op, cc, ca, cb, n, threads, iters, seconds);
    case R_FLOAT64: return reduceSlices<double>(op, cc, ca, cb, n, threads, iters, seconds);
  }
  return -1;
}

const char* ref_last_error() { return g_err.c_str(); }

// c = op(a, b) through the reference's own gloo/math.h templates.
int ref_reduce(int op, int dtype, void* c, const void* a, const void* b,
               size_t n) {
  switch (dtype) {
    case R_INT8: return reduceT<int8_t>(op, c, a, b, n);
    case R_UINT8: return reduceT<uint8_t>(op, c, a, b, n);
    case R_INT32: return reduceT<int32_t>(op, c, a, b, n);
    case R_INT64: return reduceT<int64_t>(op, c, a, b, n);
    case R_UINT64: return reduceT<uint64_t>(op, c, a, b, n);
    case R_FLOAT32: return reduceT<float>(op, c, a, b, n);
    case R_FLOAT64: return reduceT<double>(op, c, a, b, n);
    case R_FLOAT16: return reduceT<gloo::float16>(op, c, a, b, n);
  }
  return -1;  // bf16: the reference has no such type
}

// Reference fp16 conversions (gloo/types.h:248-339) for conversion sweeps.
void ref_f32_to_f16(const float* in, uint16_t* out, size_t n) {
  for (size_t i = 0; i < n; i++) out[i] = gloo::cpu_float2half_rn(in[i]).x;
}

void ref_f16_to_f32(const uint16_t* in, float* out, size_t n) {
  for (size_t i = 0; i < n; i++) {
    gloo::float16 h;
    h.x = in[i];
    out[i] = gloo::cpu_half2float(h);
  }
}

// gloo::Context::base of the contexts ref_allreduce creates (AllreduceBcube's
// group size; the other algorithms ignore it)
void ref_set_bcube_base(int base) { g_bcube_base = base; }

// algo: 0 = AllreduceRingChunked, 1 = AllreduceHalvingDoubling, 9 = AllreduceRing,
// 10 = AllreduceBcube (base: ref_set_bcube_base).  op: R_SUM..R_MIN, or the
// CUSTOM functions R_CUSTOM_OR / R_CUSTOM_3A_PLUS_B for 4-byte types.

int ref_allreduce(int algo, int op, int dtype, int P, int nptrs, int count,
                  void** bufs, int warmup, int iters, double* seconds) {
  switch (dtype) {
    case R_INT8: return allreduceT<int8_t>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_UINT8: return allreduceT<uint8_t>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_INT32: return allreduceT<int32_t>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_INT64: return allreduceT<int64_t>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_UINT64: return allreduceT<uint64_t>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_FLOAT32: return allreduceT<float>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_FLOAT64: return allreduceT<double>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
    case R_FLOAT16: return allreduceT<gloo::float16>(algo, op, P, nptrs, count, bufs, warmup, iters, seconds);
  }
  return -1;
}

// algo: 1 = Algorithm::RING, 2 = Algorithm::BCUBE.  ins[r * nin + i],
// outs[r * nout + i]; max_seg 0 = the default segment size.
int ref_allreduce_fn(int algo, int op, int dtype, int P, int nin, int nout, size_t count,
                     size_t max_seg, void** ins, void** outs) {
  switch (dtype) {
    case R_INT8: return allreduceFnT<int8_t>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_UINT8: return allreduceFnT<uint8_t>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_INT32: return allreduceFnT<int32_t>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_INT64: return allreduceFnT<int64_t>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_UINT64: return allreduceFnT<uint64_t>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_FLOAT32: return allreduceFnT<float>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_FLOAT64: return allreduceFnT<double>(algo, op, P, nin, nout, count, max_seg, ins, outs);
    case R_FLOAT16: return allreduceFnT<gloo::float16>(algo, op, P, nin, nout, count, max_seg, ins, outs);
  }
  return -1;
}

}  // extern "C"
