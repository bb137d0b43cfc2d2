// linkprobe.h -- measured xGMI link ceilings between a context's ranks (see
// linkprobe.cc).  Collective construction; run() is per rank: callers
// barrier before it (so every rank sends at once) and take the max time over
// ranks; they barrier again before destroying a probe (a peer may still be
// writing into this rank's block until then).
#pragma once

#include <hip/hip_runtime_api.h>

#include <memory>
#include <string>
#include <vector>

#include "context.h"

namespace gloo {

class LinkProbe {
 public:
  enum Pattern { kRing = 0, kMesh = 1 };
  enum Engine { kDma = 0, kKernel = 1 };

  LinkProbe(std::shared_ptr<Context> ctx, size_t bytes);
  ~LinkProbe();
  LinkProbe(const LinkProbe&) = delete;
  LinkProbe& operator=(const LinkProbe&) = delete;

  // `reps` rounds of the pattern back to back; seconds on this rank
  double run(int pattern, int engine, int blocks, int reps);
  // bytes one round puts on this rank's busiest outgoing link
  size_t busiestLinkBytes(int pattern) const;

 private:
  void issue(int pattern, int engine, int blocks);

  std::shared_ptr<Context> ctx_;
  size_t bytes_;
  SharedBlock recv_;
  char* src_ = nullptr;
  std::string key_;
  std::vector<char*> peers_;  // each peer's receive block as mapped here
  std::vector<int> devs_;     // each peer's device ordinal in this process
  std::vector<hipStream_t> streams_;
};

}  // namespace gloo
