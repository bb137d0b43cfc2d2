// host_fn.h -- gloo::allreduce(opts) with a caller-supplied reduction function
// on host buffers.
//
// The reference's AllreduceOptions::Func (gloo/allreduce.h:36,69,171) is any
// host std::function c = f(a, b) over n elements; its RING and BCUBE
// schedules call it in a fixed order (gloo/allreduce.cc:44-95 local
// reduction of several inputs, :286-297 the ring's out = f(out, tmp), :580-596
// bcube's left fold over the group's peers).  A device cannot run such a
// function, so for host buffers the same step program the device path runs
// (plan.h planFnRing / planFnBcube: the reference's segments, ownership and
// order) is executed on the host: SEND = memcpy into the receiver's landing
// region (POSIX shared memory every peer maps), RECV / RELEASE = the
// context's shared-memory delivery and credit counters, REDUCE / FOLD = the
// caller's function, COPY = memcpy.  Bits equal the reference's for any
// function (tests/golden/allreduce_custom_golden.*, made by the reference
// itself).  Device buffers with such a function are refused (glx.h).
//
// The class algorithms AllreduceRingChunked<T> / AllreduceHalvingDoubling<T>
// with a ReductionFunction<T> of type CUSTOM (gloo/algorithm.h:58-83) run the
// same way over their own programs (plan.h planRingChunked /
// planHalvingDoubling): their function is x = f(x, y) in place
// (allreduce_ring_chunked.h:89-99,141-157; allreduce_halving_doubling.h:
// 231-273), which is this executor's call with c == a -- the local
// multi-pointer fold, every REDUCE step, and no FOLD step in those programs
// (tests/golden/allreduce_class_custom_golden.*).
#pragma once

#include <chrono>
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "context.h"
#include "executor.h"
#include "plan.h"

namespace gloo {

// c = f(a, b) over n elements, as the reference's Func; `user` passed through;
// nonzero = the function failed (glx.h glx_reduce_fn): the call stops.
using HostReduceFn = int (*)(void* user, void* c, const void* a, const void* b, size_t n);

class HostFnExecutor : public Algorithm {
 public:
  // algo: glx::ALGO_FN_RING or glx::ALGO_FN_BCUBE (built on the first call
  // ...), or glx::ALGO_RING_CHUNKED / ALGO_HALVING_DOUBLING (a class
  // algorithm: built by its constructor, capi.cc glx_allreduce_create_host_fn,
  // maxSegmentBytes unused).  Function-style: built on the first call
  // of a (schedule, element size, elements, tag, maxSegmentSize) and kept in
  // the context (collectives.cc's rule: every rank makes the same calls).
  HostFnExecutor(const std::shared_ptr<Context>& ctx, int algo, size_t elementSize,
                 size_t elements, size_t maxSegmentBytes);
  ~HostFnExecutor() noexcept(false) override;
  void run() override;  // refused: needs the call's buffers and function

  // One call: inputs (maybe none) reduced into out[0] (:44-82), the
  // allreduce, out[0] broadcast to the other outputs (:87-96).
  void call(HostReduceFn fn, void* user, const std::vector<const void*>& in,
            const std::vector<void*>& out, std::chrono::milliseconds timeout);

 private:
  struct Chan {
    int peer = -1;
    int64_t tag = -1;
    uint32_t word = 0;                         // our counter word
    std::atomic<uint64_t>* peerWord = nullptr;  // out: peer's delivery; in: peer's credit
    uint64_t count = 0;                        // sent / received
    uint64_t consumed = 0;                     // in: released
  };
  void publish();
  void resolve();
  int chanIndex(std::vector<Chan>& v, int peer, int64_t tag);
  template <typename Pred>
  void waitFor(Pred done, const char* what, int peer, std::chrono::milliseconds timeout);

  int algo_;
  size_t es_, elements_;
  glx::Plan plan_;
  int slot_ = 0;
  std::string shmName_;
  char* region_ = nullptr;
  size_t regionBytes_ = 0;
  bool unlinked_ = false;
  bool resolved_ = false;
  bool broken_ = false;  // the last call failed part-way (no credit drain at destruction)
  uint64_t calls_ = 0;
  std::vector<Chan> out_, in_;
  std::vector<int> stepChan_;
  std::vector<char*> peerRegion_;  // by rank (mapped receive regions of our out-peers)
  std::vector<size_t> peerBytes_;
};

}  // namespace gloo
