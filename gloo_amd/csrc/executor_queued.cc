// executor_queued.cc -- the queued steps engine of HipPlanExecutor (host-issued
// steps enqueued at once, stream-ordered flag waits).  See executor.h.
#include "executor.h"

#include <immintrin.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>

#include "common.h"
#include "executor_internal.h"
#include "host_ops.h"
#include "kernels.h"

namespace gloo {

using namespace exec;  // NOLINT: the executor's own helpers

// ---------------------------------------------------------------------------
// Queued steps engine
// ---------------------------------------------------------------------------

// Flag rows (one flag per 128-B line, the plan kernel's layout with G = 1):
// [in_.size()] delivery flags, [out_.size()] credit flags, then one local copy
// counter per out-channel (never published).
void HipPlanExecutor::setupQueued() {
  pk_.G = 1;
  for (size_t k = 0; k < in_.size(); k++) in_[k].deliveryWord = (uint32_t)k;
  for (size_t k = 0; k < out_.size(); k++) out_[k].creditWord = (uint32_t)(in_.size() + k);
  const size_t rows = std::max<size_t>(1, in_.size() + 2 * out_.size());
  ddAlloc(rows * glx::kFlagBytes);
  for (size_t k = 0; k < out_.size(); k++) {
    out_[k].devCounter = flagRow((uint32_t)(in_.size() + out_.size() + k));
  }
}

uint64_t* HipPlanExecutor::flagRow(uint32_t row) const {
  return reinterpret_cast<uint64_t*>(ddBlocks_.at(0)) + (size_t)row * glx::kFlagStride;
}

// The host engine's loop (exchange) with its two blocking waits and its
// completion polling replaced by launches: a SEND's credit wait is a
// flag_wait on its copy stream(s), the delivery that ends it a flag_put after
// its copies (or the copy kernel's own last workgroup); a RECV is a flag_wait
// on the compute stream, a RELEASE a flag_put after the reduce that read the
// region.  The streams carry the program order the host loop used to
// enforce, so the same deadlock-freedom holds: each wait blocks only work
// issued after it in that order, and every signal is issued before any later
// wait of its stream.  Message numbers are cumulative over runs (out_.sent,
// in_.received / consumed), so no device state needs resetting.
void HipPlanExecutor::exchangeQueued(char* ptr0) {
  if (!resolved_) resolvePeers();
  checkDevice();  // an earlier asynchronous call that timed out
  devRuns_++;
  const uint64_t ticks = (uint64_t)effectiveTimeout().count() * (uint64_t)clockKhz_;
  const int store = context_->flagStores() ? 1 : 0;
  auto code = [&](size_t step, int peer) { return 1 + peer + 256 * (1 + (int)step); };
  bool computeSinceMark = true;  // the caller's writes to ptr0 count as compute
  for (auto& c : copies_) c.last = nullptr;
  const auto& steps = plan_.steps;
  for (size_t i = 0; i < steps.size(); i++) {
    const glx::Step& s = steps[i];
    switch (s.kind) {
      case glx::SEND: {
        OutChan& oc = out_[stepChan_[i]];
        const uint64_t n = ++oc.sent;
        const size_t nbytes = (size_t)s.len * esize_;
        CopyStream& c0 = copies_[oc.stream];
        // message n may land once the receiver has consumed message n-1
        auto creditWait = [&](hipStream_t st) {
          if (n > 1) {
            GLX_HIP_CHECK(glx::launch_flag_wait(flagRow(oc.creditWord), n - 1, ticks,
                                                ddStatusDev_, ddClaim_, code(i, oc.peer), st));
          }
        };
        if (nbytes == 0) {
          creditWait(c0.s);
          GLX_HIP_CHECK(glx::launch_flag_put(oc.devDelivery, n, store, c0.s));
          // the run ends only after this delivery too
          GLX_HIP_CHECK(hipEventRecord(events_[i * (size_t)split_], c0.s));
          c0.last = events_[i * (size_t)split_];
          break;
        }
        if (computeSinceMark) {
          GLX_HIP_CHECK(hipEventRecord(computeMark_, compute_));
          markEpoch_++;
          computeSinceMark = false;
        }
        char* dst = landing(peerBlocks_[oc.peer], s.dst_off, s.off, s.len);
        const char* src = ptr0 + (size_t)s.off * esize_;
        auto prepare = [&](CopyStream& cs) {
          creditWait(cs.s);
          if (cs.waitedMark != markEpoch_) {
            GLX_HIP_CHECK(hipStreamWaitEvent(cs.s, computeMark_, 0));
            cs.waitedMark = markEpoch_;
          }
          if (staged_) waitH2D(cs.s, cs.h2dWaited, s.off, s.len);
        };
        hipEvent_t done = events_[i * (size_t)split_];
        if (copyEngine_ == kCopyKernel) {
          prepare(c0);
          const int blocks = std::max(1, glx::copy_blocks());
          oc.counterTarget += (uint64_t)blocks;
          GLX_HIP_CHECK(glx::launch_copy_signal(dst, src, nbytes, blocks, oc.devCounter,
                                                oc.counterTarget, oc.devDelivery, n, store,
                                                c0.s));
          transport_.kernelCopies++;
        } else {
          int parts = split_;
          while (parts > 1 && nbytes / (size_t)parts < kMinSplitBytes) parts--;
          const size_t per = ((nbytes / (size_t)parts) + 255) & ~(size_t)255;
          for (int j = 0; j < parts; j++) {
            const size_t at = (size_t)j * per;
            if (at >= nbytes) break;
            const size_t len = std::min(per, nbytes - at);
            CopyStream& cs = copies_[oc.stream + j];
            prepare(cs);
            hipError_t ce = hipErrorUnknown;
            if (peerCopyOk_ && oc.peerDevice >= 0 && oc.peerDevice != device_) {
              ce = hipMemcpyPeerAsync(dst + at, oc.peerDevice, src + at, device_, len, cs.s);
              if (ce == hipSuccess) {
                transport_.peerCopies++;
              } else {
                (void)hipGetLastError();
                peerCopyOk_ = false;
                std::fprintf(stderr,
                             "[gloo_amd] rank %d: hipMemcpyPeerAsync to device %d refused "
                             "(%s: %s); peer copies of this algorithm use hipMemcpyAsync\n",
                             contextRank_, oc.peerDevice, hipGetErrorName(ce),
                             hipGetErrorString(ce));
              }
            }
            if (ce != hipSuccess) {
              GLX_HIP_CHECK(hipMemcpyAsync(dst + at, src + at, len, hipMemcpyDeviceToDevice,
                                           cs.s));
              transport_.deviceCopies++;
            }
            if (j > 0) {  // part j done -> the delivery on part 0's stream waits for it
              hipEvent_t ev = events_[i * (size_t)split_ + (size_t)j];
              GLX_HIP_CHECK(hipEventRecord(ev, cs.s));
              GLX_HIP_CHECK(hipStreamWaitEvent(c0.s, ev, 0));
              cs.last = ev;
            }
          }
          GLX_HIP_CHECK(glx::launch_flag_put(oc.devDelivery, n, store, c0.s));
        }
        transport_.bytes += (int64_t)nbytes;
        GLX_HIP_CHECK(hipEventRecord(done, c0.s));
        c0.last = done;
        inflight_.push_back({s.off, s.len, done});
        break;
      }
      case glx::RECV: {
        InChan& ic = in_[stepChan_[i]];
        const uint64_t n = ++ic.received;
        GLX_HIP_CHECK(glx::launch_flag_wait(flagRow(ic.deliveryWord), n, ticks, ddStatusDev_,
                                            ddClaim_, code(i, ic.peer), compute_));
        break;
      }
      case glx::REDUCE:
      case glx::COPY: {
        waitWar(s.off, s.len);
        if (staged_) waitH2D(compute_, computeH2dWaited_, s.off, s.len);
        char* dst = ptr0 + (size_t)s.off * esize_;
        const char* src = landing(blocks_, s.boff, s.off, s.len);
        if (s.kind == glx::REDUCE) {
          GLX_HIP_CHECK(
              glx::launch_reduce(op_, dtype_, dst, dst, src, (size_t)s.len, compute_));
        } else {  // our copy kernel: see exchange()
          GLX_HIP_CHECK(glx::launch_copy(dst, src, (size_t)s.len * esize_, compute_));
        }
        computeSinceMark = true;
        if (staged_ && !stage_.d2h[i].empty()) {  // final values: copy back now
          GLX_HIP_CHECK(hipEventRecord(d2hEvents_[i], compute_));
          GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, d2hEvents_[i], 0));
          copyBack(stage_.d2h[i]);
        }
        break;
      }
      case glx::FOLD: {
        size_t last = i;
        while (last + 1 < steps.size() && steps[last + 1].kind == glx::FOLD &&
               steps[last + 1].flags == s.flags) {
          last++;
        }
        const bool rev = (s.flags & glx::kFoldLeft) == 0;
        const bool whole = (s.flags & glx::kFoldWhole) != 0;
        std::vector<glx::FoldSpec> specs;
        for (size_t q = i; q <= last; q++) {
          const glx::Step& f = steps[q];
          waitWar(f.off, f.len);
          if (staged_) waitH2D(compute_, computeH2dWaited_, f.off, f.len);
          glx::FoldSpec spec;
          spec.dst = ptr0 + (size_t)f.off * esize_;
          spec.n = (size_t)f.len;
          for (int64_t r : plan_.folds[(size_t)f.boff]) {
            if (r < 0) {
              spec.srcs.push_back(spec.dst);
            } else if (whole) {
              spec.srcs.push_back(landing(blocks_, r, 0) + (size_t)f.off * esize_);
            } else {
              spec.srcs.push_back(landing(blocks_, r, f.off, f.len));
            }
          }
          spec.k = (int)spec.srcs.size();
          specs.push_back(std::move(spec));
        }
        if (specs.size() == 1) {
          const glx::FoldSpec& f = specs[0];
          GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, f.dst, f.srcs.data(), f.k, f.n,
                                             compute_, rev));
        } else {
          GLX_HIP_CHECK(glx::launch_reduce_n_batch(op_, dtype_, specs, compute_, rev));
        }
        computeSinceMark = true;
        for (size_t q = i; q <= last; q++) {
          if (staged_ && !stage_.d2h[q].empty()) {
            GLX_HIP_CHECK(hipEventRecord(d2hEvents_[q], compute_));
            GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, d2hEvents_[q], 0));
            copyBack(stage_.d2h[q]);
          }
        }
        i = last;
        break;
      }
      case glx::RELEASE: {
        InChan& ic = in_[stepChan_[i]];
        GLX_HIP_CHECK(glx::launch_flag_put(ic.devCredit, ++ic.consumed, store, compute_));
        break;
      }
      default:
        GLX_ENFORCE(false, "bad plan step kind ", s.kind);
    }
  }
  // the caller's stream must not run ahead of copies still reading ptr0
  for (auto& c : copies_) {
    if (c.last != nullptr) GLX_HIP_CHECK(hipStreamWaitEvent(compute_, c.last, 0));
  }
  inflight_.clear();
}

}  // namespace gloo
