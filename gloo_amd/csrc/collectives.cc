// collectives.cc -- gloo::allreduce(opts) on the xGMI executor.
//
// The reference builds its scratch and transport buffers inside every call
// (gloo/allreduce.cc:220-225).  On the device that would put a hipMalloc and
// an IPC handle exchange with every peer into each call, so the executor for
// a given (algorithm, dtype, op, elements, tag, maxSegmentSize) is built on
// the first call and kept in the context; the user buffers themselves are
// per call and never published (receive regions are ours, and a message's
// landing phase depends only on its element offset).  All ranks must make the
// same sequence of calls (as in the reference), so their executors are
// created in the same order and draw matching slots from Context::nextSlot.
#include "collectives.h"

#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/gloo_amd/glx.h"
#include "common.h"
#include "executor.h"

namespace gloo {

namespace {

int64_t envBytes(const char* name, int64_t dflt) {
  const char* e = std::getenv(name);
  if (e == nullptr || *e == 0) return dflt;
  char* end = nullptr;
  long long v = std::strtoll(e, &end, 10);
  return (end != e && v >= 0) ? (int64_t)v : dflt;
}

int scheduleFor(int algorithm, const Context& ctx, int64_t bytes) {
  switch (algorithm) {
    case AllreduceOptions::UNSPECIFIED:
      // RING's result (gloo/allreduce.cc:134-137) moved the fastest way
      return glx::autoRingSchedule(ctx.size, bytes, /*fn=*/true,
                                   HipPlanExecutor::deviceEnginesAvailable(ctx));
    case AllreduceOptions::RING: return glx::ALGO_FN_RING;
    case AllreduceOptions::RING_MESH: return glx::ALGO_FN_RING_MESH;
    case AllreduceOptions::RING_REPLICATED: return glx::ALGO_FN_RING_REPL;
    case AllreduceOptions::BCUBE: return glx::ALGO_FN_BCUBE;
  }
  GLX_ENFORCE(false, "Algorithm not handled.");  // :141-142
  return -1;
}

}  // namespace

void allreduce(const AllreduceOptions& opts) {
  GLX_ENFORCE(opts.context != nullptr, "allreduce: null context");
  GLX_ENFORCE(opts.algorithm >= AllreduceOptions::UNSPECIFIED &&
                  opts.algorithm <= AllreduceOptions::RING_REPLICATED,
              "Algorithm not handled.");  // :141-142
  if (opts.elements == 0) return;  // :98-100
  // sanity checks (:107-122)
  GLX_ENFORCE(!opts.out.empty(), "allreduce: at least one output is required");
  const size_t es = glx_dtype_size(opts.dtype);
  GLX_ENFORCE(es > 0, "allreduce: unknown dtype ", opts.dtype);
  GLX_ENFORCE(opts.op >= GLX_SUM && opts.op <= GLX_MIN, "allreduce: unknown reduction ",
              opts.op);
  GLX_ENFORCE(opts.elements <= ((size_t)1 << 40), "allreduce: too many elements");
  auto& ctx = *opts.context;
  GLX_ENFORCE(ctx.size == 1 || ctx.connected(),
              "allreduce: context must be connected (connectFullMesh)");

  const int schedule = scheduleFor(opts.algorithm, ctx, (int64_t)(opts.elements * es));
  const size_t maxSeg = opts.maxSegmentSize == 0 ? (size_t)glx::kMaxSegmentBytes
                                                 : opts.maxSegmentSize;
  const std::string key = std::to_string(schedule) + "/" + std::to_string(opts.dtype) + "/" +
                          std::to_string(opts.op) + "/" + std::to_string(opts.elements) + "/" +
                          std::to_string(opts.tag) + "/" + std::to_string(maxSeg);
  std::shared_ptr<Algorithm> alg;
  {
    std::lock_guard<std::mutex> g(ctx.opsMutex);
    auto it = ctx.ops.find(key);
    if (it != ctx.ops.end()) {
      alg = it->second;
    } else {
      glx::PlanParams prm;
      prm.esize = (int)es;
      prm.maxSegmentBytes = (int64_t)maxSeg;
      prm.minPieceBytes = envBytes("GLOO_AMD_MIN_PIECE_BYTES", prm.minPieceBytes);
      alg = std::make_shared<HipPlanExecutor>(opts.context, schedule,
                                              std::vector<void*>{opts.out[0]},
                                              (int64_t)opts.elements, opts.dtype, opts.op,
                                              std::vector<hipStream_t>(), prm,
                                              /*perCallBuffers=*/true);
      ctx.ops.emplace(key, alg);
    }
  }
  HipPlanExecutor::FnCall call;
  call.in = opts.in;
  call.out = opts.out;
  call.stream = opts.stream;
  call.timeout = opts.timeout;
  static_cast<HipPlanExecutor&>(*alg).runFn(call);
}

}  // namespace gloo
