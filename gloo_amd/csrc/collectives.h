// collectives.h -- the function-style collective surface, gloo::allreduce
// (gloo/allreduce.h:89-193, gloo/allreduce.cc:97-146), on device buffers.
#pragma once

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <cstdint>
#include <memory>
#include <vector>

#include "context.h"
#include "plan.h"

namespace gloo {

// detail::AllreduceOptionsImpl (gloo/allreduce.h:22-84) with the reduce
// function named by (dtype, op) instead of a host std::function.
struct AllreduceOptions {
  enum Algorithm { UNSPECIFIED = 0, RING = 1, BCUBE = 2, RING_MESH = 3, RING_REPLICATED = 4 };

  explicit AllreduceOptions(const std::shared_ptr<Context>& c) : context(c) {}

  std::shared_ptr<Context> context;
  std::chrono::milliseconds timeout{0};  // 0: the context's (:45-48)
  int algorithm = UNSPECIFIED;
  std::vector<void*> in, out;
  size_t elements = 0;
  int dtype = -1;
  int op = -1;
  uint32_t tag = 0;
  size_t maxSegmentSize = (size_t)glx::kMaxSegmentBytes;
  hipStream_t stream = nullptr;  // null: complete on return
};

void allreduce(const AllreduceOptions& opts);

}  // namespace gloo
