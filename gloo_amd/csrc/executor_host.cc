// executor_host.cc -- host-memory endpoints of HipPlanExecutor:
// staged, transport-fed and function-style host buffers.  See executor.h.
#include "executor.h"

#include <immintrin.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <mutex>
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

// gloo::allreduce(opts) on host buffers (the reference's own calling
// convention, e.g. CPU tensors): the buffers change from call to call, so
// they are not pinned; they are copied into device staging buffers owned by
// this executor, the device path runs there, and the result is copied back
// to every output.  Blocking, like the reference.
// Staging of host memory for the function-style op (created at its first
// overlapped host call): the class algorithms' machinery (setupHostMode)
// with one device buffer and per-call host sources / destinations.
void HipPlanExecutor::setupCallStaging() {
  if (!devBufs_.empty()) return;
  const size_t bytes = (size_t)count_ * esize_;
  char* d = nullptr;
  GLX_HIP_CHECK(hipMalloc((void**)&d, bytes));
  devBufs_.push_back(d);
  GLX_HIP_CHECK(hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking));
  GLX_HIP_CHECK(hipStreamCreateWithFlags(&d2h_, hipStreamNonBlocking));
  stage_ = glx::stagePlan(plan_, count_, std::max<int64_t>(1, kStagePieceBytes / (int64_t)esize_));
  h2dEvents_.resize(stage_.h2d.size(), nullptr);
  for (auto& e : h2dEvents_) GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (contextSize_ == 1 && ptrs_.size() > 1) {  // runHost's per-piece fold
    pieceDone_.resize(stage_.h2d.size(), nullptr);
    for (auto& e : pieceDone_) GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  d2hEvents_.assign(plan_.steps.size(), nullptr);
  for (size_t i = 0; i < plan_.steps.size(); i++) {
    if (!stage_.d2h[i].empty()) {
      GLX_HIP_CHECK(hipEventCreateWithFlags(&d2hEvents_[i], hipEventDisableTiming));
    }
  }
  GLX_HIP_CHECK(hipEventCreateWithFlags(&hostDone_, hipEventDisableTiming));
}

// gloo::allreduce(opts) on ONE host input (or in place on the output) and
// ONE host output: staged like the class algorithms -- H2D pieces in the
// order the schedule first touches them, every step waiting only for its
// own, each range copied back to the output right after its final write --
// instead of copying everything in, running, and copying everything out.
void HipPlanExecutor::runFnHostStaged(const FnCall& call) {
  setupCallStaging();
  void* src = call.in.empty() ? call.out[0] : call.in[0];
  callSrc_ = {src};
  callDst_ = {call.out[0]};
  for (int i = 0; i < 2; i++) {  // pageable source / destination: through a mirror
    void* u = i == 0 ? src : call.out[0];
    callMirrored_[i] = !isPinnedHost(u);
    if (callMirrored_[i] && callMirror_[i].p == nullptr) {
      takeMirror(callMirror_[i], std::max<size_t>((size_t)count_ * esize_, 16));
    }
  }
  staged_ = true;
  timeout_ = call.timeout;
  struct Restore {
    HipPlanExecutor* e;
    ~Restore() {
      e->callSrc_.clear();
      e->callDst_.clear();
      e->staged_ = e->hostMode_;
      e->timeout_ = std::chrono::milliseconds(0);
    }
  } restore{this};
  computeH2dWaited_ = -1;
  for (auto& c : copies_) c.h2dWaited = -1;
  {
    std::lock_guard<std::mutex> g(doneMutex_);
    doneQueue_.clear();
    doneUsed_ = 0;
  }
  pieceIssued_.assign(stage_.h2d.size(), 0);
  for (size_t j = 0; j < stage_.h2d.size(); j++) issuePiece(j);
  if (contextSize_ > 1) exchange(devBufs_[0]);
  // ranges no step wrote hold the input: the output needs them too when it
  // is another buffer (one input: genLocalReduceFunction copies,
  // gloo/allreduce.cc:50-56)
  if (src != call.out[0]) {
    waitH2D(compute_, computeH2dWaited_, 0, count_);
    GLX_HIP_CHECK(hipEventRecord(hostDone_, compute_));
    GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, hostDone_, 0));
    copyBack(contextSize_ > 1 ? stage_.d2hRest : std::vector<glx::Range>{{0, count_}});
  }
  waitDevice(compute_);
  GLX_HIP_CHECK(hipStreamSynchronize(d2h_));
  GLX_HIP_CHECK(hipStreamSynchronize(h2d_));
  noteDone(d2h_);
  checkDevice();
  flushMirrors();
}

void HipPlanExecutor::runFnHost(const FnCall& call) {
  GLX_ENFORCE(call.stream == nullptr, "a stream cannot be used with host-memory buffers");
  if (call.in.size() <= 1 && call.out.size() == 1) {
    runFnHostStaged(call);
    return;
  }
  const size_t bytes = (size_t)count_ * esize_;
  // device staging: out[0], and the inputs (or, with no inputs, the outputs,
  // which are then folded into out[0])
  const std::vector<void*>& srcs = call.in.empty() ? call.out : call.in;
  const size_t need = 1 + srcs.size();
  while (fnStage_.size() < need) {
    char* d = nullptr;
    GLX_HIP_CHECK(hipMalloc((void**)&d, bytes));
    fnStage_.push_back(d);
  }
  timeout_ = call.timeout;
  struct Restore {
    HipPlanExecutor* e;
    ~Restore() { e->timeout_ = std::chrono::milliseconds(0); }
  } restore{this};
  // pageable buffers through pinned mirrors: slots 0..srcs-1 the sources,
  // then out[0]'s old value (float16), then the outputs
  while (fnMirror_.size() < srcs.size() + 1 + call.out.size()) fnMirror_.emplace_back();
  // a whole host buffer to the device: directly when pinned, else through its
  // mirror (or bounce block)
  auto stageIn = [&](char* dev, void* user, PinnedBlock& m) {
    char* src = mirrorFor(user, m);
    if (m.bounce && src == m.p) {
      bounceIn(dev, static_cast<const char*>(user), bytes, m, compute_);
    } else {
      GLX_HIP_CHECK(hipMemcpyAsync(dev, src, bytes, hipMemcpyHostToDevice, compute_));
    }
  };
  for (size_t i = 0; i < srcs.size(); i++) stageIn(fnStage_[1 + i], srcs[i], fnMirror_[i]);
  std::vector<void*> din, dout;
  char* out0;
  if (call.in.empty()) {  // the staged outputs are the data; out[0]'s copy gets the result
    dout.assign(fnStage_.begin() + 1, fnStage_.begin() + 1 + (long)srcs.size());
    out0 = fnStage_[1];
  } else {
    din.assign(fnStage_.begin() + 1, fnStage_.begin() + 1 + (long)srcs.size());
    dout.push_back(fnStage_[0]);
    out0 = fnStage_[0];
    if (dtype_ == GLX_FLOAT16 && din.size() >= 2) {
      // float16's assignment reads out[0]'s old value
      stageIn(out0, call.out[0], fnMirror_[srcs.size()]);
    }
  }
  localReduce(din, dout);
  if (contextSize_ > 1) exchange(out0);
  std::vector<char*> outDma(call.out.size());
  for (size_t i = 0; i < call.out.size(); i++) {
    PinnedBlock& m = fnMirror_[srcs.size() + 1 + i];
    outDma[i] = isPinnedHost(call.out[i]) ? static_cast<char*>(call.out[i])
                                          : mirrorFor(nullptr, m);
    if (m.bounce && outDma[i] == m.p) continue;  // after the run, piece by piece
    GLX_HIP_CHECK(hipMemcpyAsync(outDma[i], out0, bytes, hipMemcpyDeviceToHost, compute_));
  }
  noteDone(compute_);
  waitDevice(compute_);
  checkDevice();
  for (size_t i = 0; i < call.out.size(); i++) {
    PinnedBlock& m = fnMirror_[srcs.size() + 1 + i];
    if (outDma[i] == call.out[i]) continue;
    if (m.bounce) {
      bounceOut(static_cast<char*>(call.out[i]), out0, bytes, m, compute_);
    } else {
      std::memcpy(call.out[i], outDma[i], bytes);
    }
  }
}

namespace {
// Pinned host staging blocks (hipHostMalloc) are not handed back to the
// runtime while the process lives: they wait here for the next algorithm,
// the policy context.cc applies to uncached device blocks after freed ones
// were seen breaking later allocations of the same process.
// Cached blocks are our own hipHostMalloc allocations; none of them ever
// shares a page with a caller's memory (the round-3 illegal address came from
// registering callers' pages), so handing the ones beyond the
// cap back to the runtime is safe.
struct PinnedCache {
  std::mutex mu;
  std::vector<std::pair<size_t, char*>> free;  // oldest first
  size_t total = 0;                            // bytes in `free`
};

PinnedCache& pinnedCache() {
  static PinnedCache* c = new PinnedCache();  // never destroyed
  return *c;
}

// A cached block of at least *bytes (at most about twice that), else a new
// one; null when the runtime cannot pin that much even after the cache gave
// its blocks back.
char* tryTakePinned(size_t* bytes) {
  PinnedCache& c = pinnedCache();
  {
    std::lock_guard<std::mutex> g(c.mu);
    const size_t most = std::max(2 * *bytes, *bytes + (size_t(4) << 20));
    size_t best = c.free.size();
    for (size_t i = 0; i < c.free.size(); i++) {
      const size_t b = c.free[i].first;
      if (b >= *bytes && b <= most && (best == c.free.size() || b < c.free[best].first)) best = i;
    }
    if (best != c.free.size()) {
      char* p = c.free[best].second;
      *bytes = c.free[best].first;
      c.total -= *bytes;
      c.free.erase(c.free.begin() + (long)best);
      return p;
    }
  }
  for (int attempt = 0; attempt < 2; attempt++) {
    char* p = nullptr;
    if (hipHostMalloc((void**)&p, *bytes, hipHostMallocDefault) == hipSuccess) return p;
    (void)hipGetLastError();
    if (attempt == 0) {  // give the cached blocks back and try once more
      std::lock_guard<std::mutex> g(c.mu);
      for (auto& b : c.free) (void)hipHostFree(b.second);
      c.free.clear();
      c.total = 0;
    }
  }
  return nullptr;
}

char* takePinned(size_t* bytes) {
  char* p = tryTakePinned(bytes);
  GLX_ENFORCE(p != nullptr, "cannot pin ", *bytes, " bytes of host memory");
  return p;
}

std::atomic<size_t> g_mirrorLimit{0};  // glx_set_pinned_mirror_limit
}  // namespace

namespace exec {
size_t pinnedMirrorLimit() { return g_mirrorLimit.load(); }
void setPinnedMirrorLimit(size_t bytes) { g_mirrorLimit.store(bytes); }
}  // namespace exec

void HipPlanExecutor::givePinned(char* p, size_t bytes) {
  if (p == nullptr) return;
  PinnedCache& c = pinnedCache();
  std::lock_guard<std::mutex> g(c.mu);
  c.free.emplace_back(bytes, p);
  c.total += bytes;
  while (c.total > kPinnedCacheCap && !c.free.empty()) {
    (void)hipHostFree(c.free.front().second);
    c.total -= c.free.front().first;
    c.free.erase(c.free.begin());
  }
}

void HipPlanExecutor::takeMirror(PinnedBlock& m, size_t bytes) {
  m.bounce = false;
  m.bytes = bytes;
  const size_t limit = pinnedMirrorLimit();
  m.p = (limit == 0 || bytes <= limit) ? tryTakePinned(&m.bytes) : nullptr;
  if (m.p == nullptr) {
    // two halves: H2D pieces read the first while D2H ranges land in the
    // second (a class algorithm's buffer is both source and destination,
    // and its last H2D piece may still be in flight when the first range
    // comes back)
    m.bytes = 2 * std::min(bytes, kBounceBytes);
    m.p = takePinned(&m.bytes);
    m.bounce = true;
  }
  GLX_TRACE_MEM("r%d %s %p (%zu) for a pageable buffer of %zu", contextRank_,
                m.bounce ? "bounce" : "mirror", (void*)m.p, m.bytes, bytes);
}

void HipPlanExecutor::bounceIn(char* dev, const char* user, size_t n, PinnedBlock& b,
                               hipStream_t s) {
  const size_t half = b.bytes / 2;  // the block's H2D half
  for (size_t at = 0; at < n; at += half) {
    const size_t len = std::min(half, n - at);
    GLX_HIP_CHECK(hipStreamSynchronize(s));  // the half's previous piece has been read
    std::memcpy(b.p, user + at, len);
    GLX_HIP_CHECK(hipMemcpyAsync(dev + at, b.p, len, hipMemcpyHostToDevice, s));
  }
}

void HipPlanExecutor::bounceOut(char* user, const char* dev, size_t n, PinnedBlock& b,
                                hipStream_t s) {
  const size_t half = b.bytes / 2;
  char* out = b.p + half;  // the block's D2H half
  for (size_t at = 0; at < n; at += half) {
    const size_t len = std::min(half, n - at);
    GLX_HIP_CHECK(hipMemcpyAsync(out, dev + at, len, hipMemcpyDeviceToHost, s));
    GLX_HIP_CHECK(hipStreamSynchronize(s));
    std::memcpy(user + at, out, len);
  }
}

// `user` when it is pinned (or null: a destination-only mirror is wanted);
// else the pinned block m, taken on first use, with `user`'s bytes copied
// in when `user` is a source and m is a whole mirror (a bounce block is
// filled piece by piece by bounceIn).
char* HipPlanExecutor::mirrorFor(void* user, PinnedBlock& m) {
  if (user != nullptr && isPinnedHost(user)) return static_cast<char*>(user);
  if (m.p == nullptr) takeMirror(m, std::max<size_t>((size_t)count_ * esize_, 16));
  if (user != nullptr && !m.bounce) std::memcpy(m.p, user, (size_t)count_ * esize_);
  return m.p;
}

void HipPlanExecutor::setupHostMode() {
  const size_t bytes = (size_t)count_ * esize_;
  // Several host pointers under kOnDeviceThreshold: fold them on the host
  // into one pinned staging buffer and stage only that through the device
  // (the reference's cudaHostReduce / cudaHostBroadcast below the threshold,
  // gloo/cuda_allreduce_halving_doubling.cc:478-484)
  hostFold_ = ptrs_.size() > 1 && bytes < glx::kOnDeviceThreshold;
  if (hostFold_) {
    hostStageBytes_ = std::max<size_t>(bytes, 16);
    hostStage_ = takePinned(&hostStageBytes_);
  }
  // pageable buffers get their pinned mirrors (a host fold's single source
  // is the pinned hostStage_ itself)
  ptrMirror_.assign(ptrs_.size(), PinnedBlock{});
  if (!hostFold_) {
    for (size_t k = 0; k < ptrs_.size(); k++) {
      if (isPinnedHost(ptrs_[k])) continue;
      takeMirror(ptrMirror_[k], std::max<size_t>(bytes, 16));
    }
  }
  for (size_t k = 0; k < hostSources().size(); k++) {
    char* d = nullptr;
    GLX_HIP_CHECK(hipMalloc((void**)&d, bytes));
    GLX_TRACE_MEM("r%d hipMalloc devBuf %p (%zu)", contextRank_, (void*)d, bytes);
    devBufs_.push_back(d);
  }
  GLX_HIP_CHECK(hipStreamCreateWithFlags(&h2d_, hipStreamNonBlocking));
  GLX_HIP_CHECK(hipStreamCreateWithFlags(&d2h_, hipStreamNonBlocking));
  stage_ = glx::stagePlan(plan_, count_, std::max<int64_t>(1, kStagePieceBytes / (int64_t)esize_));
  h2dEvents_.resize(stage_.h2d.size(), nullptr);
  for (auto& e : h2dEvents_) GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  if (contextSize_ == 1 && ptrs_.size() > 1) {  // runHost's per-piece fold
    pieceDone_.resize(stage_.h2d.size(), nullptr);
    for (auto& e : pieceDone_) GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  d2hEvents_.assign(plan_.steps.size(), nullptr);
  for (size_t i = 0; i < plan_.steps.size(); i++) {
    if (!stage_.d2h[i].empty()) {
      GLX_HIP_CHECK(hipEventCreateWithFlags(&d2hEvents_[i], hipEventDisableTiming));
    }
  }
  GLX_HIP_CHECK(hipEventCreateWithFlags(&hostDone_, hipEventDisableTiming));
}

// Make `s` wait for the H2D pieces overlapping [off, off+len).  h2d_ is one
// in-order stream, so waiting for the latest such piece covers the others.
void HipPlanExecutor::waitH2D(hipStream_t s, int& waited, int64_t off, int64_t len) {
  if (fedRun_) {
    // pieces are issued as they are fed, in any order: wait (bounded) until
    // every piece of the range has been issued, then for each one's copy
    std::vector<size_t> need;
    for (size_t j = 0; j < stage_.h2d.size(); j++) {
      const glx::Range& r = stage_.h2d[j];
      if (r.off < off + len && off < r.off + r.len) need.push_back(j);
    }
    std::unique_lock<std::mutex> lk(feedMutex_);
    const auto deadline = std::chrono::steady_clock::now() + effectiveTimeout();
    for (size_t j : need) {
      while (!pieceIssued_[j]) {
        if (feedCv_.wait_until(lk, deadline) == std::cv_status::timeout && !pieceIssued_[j]) {
          broken_ = true;
          GLX_THROW_TIMEOUT("Timed out waiting for host data: elements [", stage_.h2d[j].off,
                            ", ", stage_.h2d[j].off + stage_.h2d[j].len,
                            ") were never fed (rank ", contextRank_, ", timeout ",
                            effectiveTimeout().count(), " ms)");
        }
      }
      GLX_HIP_CHECK(hipStreamWaitEvent(s, h2dEvents_[j], 0));
    }
    return;
  }
  int last = -1;
  for (size_t j = 0; j < stage_.h2d.size(); j++) {
    const glx::Range& r = stage_.h2d[j];
    if (r.off < off + len && off < r.off + r.len) last = (int)j;
  }
  if (last > waited) {
    GLX_HIP_CHECK(hipStreamWaitEvent(s, h2dEvents_[(size_t)last], 0));
    waited = last;
  }
}

// The host buffers the device copies are staged from and back to: the
// user's pointers, or the one pinned buffer they were folded into.
// user buffer `u` as the copies see it, given its block (null: pinned)
HipPlanExecutor::HostSide HipPlanExecutor::sideOf(char* u, const PinnedBlock* m) {
  if (m == nullptr || m->p == nullptr) return {u, u, nullptr};
  if (m->bounce) return {u, nullptr, const_cast<PinnedBlock*>(m)};
  return {u, m->p, nullptr};
}

std::vector<HipPlanExecutor::HostSide> HipPlanExecutor::hostSources() const {
  if (!callSrc_.empty()) {
    char* u = static_cast<char*>(callSrc_[0]);
    return {sideOf(u, callMirrored_[0] ? &callMirror_[0] : nullptr)};
  }
  if (hostFold_) return {HostSide{hostStage_, hostStage_, nullptr}};
  std::vector<HostSide> v;
  for (size_t k = 0; k < ptrs_.size(); k++) {
    v.push_back(sideOf(static_cast<char*>(ptrs_[k]), &ptrMirror_[k]));
  }
  return v;
}

std::vector<HipPlanExecutor::HostSide> HipPlanExecutor::hostDests() const {
  if (!callDst_.empty()) {
    char* u = static_cast<char*>(callDst_[0]);
    return {sideOf(u, callMirrored_[1] ? &callMirror_[1] : nullptr)};
  }
  return hostSources();
}

void HipPlanExecutor::copyOut(const std::vector<glx::Range>& ranges) {
  for (const HostSide& h : hostDests()) {
    if (h.dma == h.user || h.dma == nullptr) continue;  // pinned, or bounced already
    for (const glx::Range& r : ranges) {
      const size_t at = (size_t)r.off * esize_, n = (size_t)r.len * esize_;
      std::memcpy(h.user + at, h.dma + at, n);
    }
  }
}

// After the run's streams are synchronised: every batch not yet copied out.
void HipPlanExecutor::flushMirrors() {
  std::lock_guard<std::mutex> g(doneMutex_);
  for (DoneBatch& b : doneQueue_) {
    if (!b.pendingOut) continue;
    copyOut(b.ranges);
    b.pendingOut = false;
  }
}

// Final values of `ranges` (in devBufs_[0]) to every user pointer, on d2h_
// (the caller has made d2h_ wait for the writes).
void HipPlanExecutor::copyBack(const std::vector<glx::Range>& ranges) {
  const std::vector<HostSide> dsts = hostDests();
  bool mirrored = false;
  for (const HostSide& h : dsts) mirrored = mirrored || (h.dma != h.user && h.dma != nullptr);
  for (const glx::Range& r : ranges) {
    const size_t at = (size_t)r.off * esize_, n = (size_t)r.len * esize_;
    for (const HostSide& h : dsts) {
      if (h.bounce != nullptr) {  // no mirror: through the bounce block, now
        bounceOut(h.user + at, devBufs_[0] + at, n, *h.bounce, d2h_);
        continue;
      }
      GLX_HIP_CHECK(hipMemcpyAsync(h.dma + at, devBufs_[0] + at, n, hipMemcpyDeviceToHost, d2h_));
    }
  }
  if (ranges.empty() || hostFold_) return;  // host-folded results return at the end
  // completion marker for doneRanges()
  std::lock_guard<std::mutex> g(doneMutex_);
  if (doneUsed_ == doneEvents_.size()) {
    hipEvent_t e = nullptr;
    GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    doneEvents_.push_back(e);
  }
  hipEvent_t e = doneEvents_[doneUsed_++];
  GLX_HIP_CHECK(hipEventRecord(e, d2h_));
  doneQueue_.push_back(DoneBatch{e, ranges, mirrored});
}

std::vector<glx::Range> HipPlanExecutor::doneRanges() {
  std::lock_guard<std::mutex> g(doneMutex_);
  std::vector<glx::Range> out;
  for (auto& b : doneQueue_) {
    const hipError_t e = b.ev != nullptr ? hipEventQuery(b.ev) : hipSuccess;
    if (e == hipErrorNotReady) {
      (void)hipGetLastError();
      continue;
    }
    GLX_HIP_CHECK(e);
    if (b.pendingOut) {  // landed in the mirror: out to the caller's buffer first
      copyOut(b.ranges);
      b.pendingOut = false;
    }
    out.insert(out.end(), b.ranges.begin(), b.ranges.end());
  }
  return out;
}

// Issue piece j's H2D copy (the caller holds feedMutex_ or runs alone).
void HipPlanExecutor::issuePiece(size_t j) {
  const glx::Range& r = stage_.h2d[j];
  const size_t at = (size_t)r.off * esize_, n = (size_t)r.len * esize_;
  const std::vector<HostSide> hsrc = hostSources();
  for (size_t k = 0; k < hsrc.size(); k++) {
    if (hsrc[k].bounce != nullptr) {
      bounceIn(devBufs_[k] + at, hsrc[k].user + at, n, *hsrc[k].bounce, h2d_);
      continue;
    }
    // pageable: into the mirror on the host first (the copy below then
    // reads pinned memory only)
    if (hsrc[k].dma != hsrc[k].user) std::memcpy(hsrc[k].dma + at, hsrc[k].user + at, n);
    GLX_HIP_CHECK(hipMemcpyAsync(devBufs_[k] + at, hsrc[k].dma + at, n, hipMemcpyHostToDevice,
                                 h2d_));
  }
  GLX_HIP_CHECK(hipEventRecord(h2dEvents_[j], h2d_));
  pieceIssued_[j] = 1;
}

// Issue every piece the feeds now cover (feedMutex_ held, a fed run active).
void HipPlanExecutor::issueFedPiecesLocked() {
  for (size_t j = 0; j < stage_.h2d.size(); j++) {
    if (pieceIssued_[j]) continue;
    const glx::Range& r = stage_.h2d[j];
    bool covered = false;
    for (const glx::Range& f : fed_) {
      if (f.off <= r.off && r.off + r.len <= f.off + f.len) covered = true;
    }
    if (covered) issuePiece(j);
  }
  feedCv_.notify_all();
}

void HipPlanExecutor::feed(int64_t off, int64_t len) {
  GLX_ENFORCE(hostMode_, "feed() needs an algorithm on host-memory buffers");
  GLX_ENFORCE(off >= 0 && len >= 0 && off + len <= count_, "feed range [", off, ", ",
              off + len, ") outside the buffer of ", count_, " elements");
  if (len == 0) return;
  GLX_HIP_CHECK(hipSetDevice(device_));  // this may be the transport's thread
  std::lock_guard<std::mutex> g(feedMutex_);
  // merge into the fed set
  int64_t lo = off, hi = off + len;
  std::vector<glx::Range> merged;
  for (const glx::Range& f : fed_) {
    if (f.off + f.len < lo || f.off > hi) {
      merged.push_back(f);
    } else {
      lo = std::min(lo, f.off);
      hi = std::max(hi, f.off + f.len);
    }
  }
  merged.push_back({lo, hi - lo});
  fed_.swap(merged);
  if (fedRun_) issueFedPiecesLocked();
}

void HipPlanExecutor::runFed() {
  GLX_ENFORCE(hostMode_, "runFed() needs an algorithm on host-memory buffers");
  GLX_ENFORCE(ptrs_.size() == 1, "runFed() takes one host buffer (the transport's)");
  GLX_HIP_CHECK(hipSetDevice(device_));
  {
    std::lock_guard<std::mutex> g(doneMutex_);
    doneQueue_.clear();
    doneUsed_ = 0;
  }
  {
    std::lock_guard<std::mutex> g(feedMutex_);
    fedRun_ = true;
    pieceIssued_.assign(stage_.h2d.size(), 0);
    issueFedPiecesLocked();  // what arrived before the run
  }
  struct End {
    HipPlanExecutor* e;
    ~End() {
      std::lock_guard<std::mutex> g(e->feedMutex_);
      e->fedRun_ = false;
      e->fed_.clear();
    }
  } end{this};
  if (contextSize_ == 1) {
    // nothing to exchange: the result is the input once it has all arrived
    waitH2D(compute_, computeH2dWaited_, 0, count_);
    GLX_HIP_CHECK(hipStreamSynchronize(h2d_));
    std::lock_guard<std::mutex> g(doneMutex_);
    // in place: the caller's buffer already holds the result, and h2d_ is
    // synchronised -- the batch is complete now (no event: doneRanges()
    // right after runFed() returns must report it)
    doneQueue_.push_back(DoneBatch{nullptr, {glx::Range{0, count_}}, false});
    return;
  }
  runHost();
}

void HipPlanExecutor::runHost() {
  if (contextSize_ == 1 && ptrs_.size() == 1) return;  // the result is the input
  const size_t bytes = (size_t)count_ * esize_;
  if (hostFold_) {  // local reduce on the host (below kOnDeviceThreshold)
    std::vector<const void*> srcs(ptrs_.begin(), ptrs_.end());
    glx::host_reduce_n(op_, dtype_, hostStage_, srcs.data(), (int)srcs.size(), (size_t)count_);
    transport_.hostFolds++;
    if (contextSize_ == 1) {
      for (void* p : ptrs_) std::memcpy(p, hostStage_, bytes);
      return;
    }
  }
  const size_t nsrc = hostSources().size();
  computeH2dWaited_ = -1;
  for (auto& c : copies_) c.h2dWaited = -1;
  if (!fedRun_) {
    {
      std::lock_guard<std::mutex> g(doneMutex_);
      doneQueue_.clear();
      doneUsed_ = 0;
    }
    pieceIssued_.assign(stage_.h2d.size(), 0);
    for (size_t j = 0; j < stage_.h2d.size(); j++) issuePiece(j);
  }
  if (contextSize_ == 1 && nsrc > 1 && !fedRun_) {
    // One rank, several host pointers: the allreduce is the local fold and
    // broadcast.  Pipelined per H2D piece: the fold of piece j runs once its
    // copies have landed, and its result goes back to every host pointer
    // while later pieces are still coming in (H2D and D2H overlap on the
    // full-duplex link).
    for (size_t j = 0; j < stage_.h2d.size(); j++) {
      const glx::Range& r = stage_.h2d[j];
      GLX_HIP_CHECK(hipStreamWaitEvent(compute_, h2dEvents_[j], 0));
      std::vector<const void*> srcs;
      for (char* d : devBufs_) srcs.push_back(d + (size_t)r.off * esize_);
      GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, devBufs_[0] + (size_t)r.off * esize_,
                                         srcs.data(), (int)srcs.size(), (size_t)r.len,
                                         compute_));
      GLX_HIP_CHECK(hipEventRecord(pieceDone_[j], compute_));
      GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, pieceDone_[j], 0));
      copyBack({r});
    }
    waitDevice(compute_);
    GLX_HIP_CHECK(hipStreamSynchronize(d2h_));
    GLX_HIP_CHECK(hipStreamSynchronize(h2d_));
    noteDone(d2h_);
    flushMirrors();
    return;
  }
  if (nsrc > 1) {  // local fold needs every buffer whole
    waitH2D(compute_, computeH2dWaited_, 0, count_);
    std::vector<const void*> srcs(devBufs_.begin(), devBufs_.end());
    GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, devBufs_[0], srcs.data(), (int)srcs.size(),
                                       (size_t)count_, compute_));
  }
  if (contextSize_ > 1) exchange(devBufs_[0]);
  // ranges no step wrote: their value is the local fold (a no-op for one
  // pointer, whose host copy already holds it)
  if (nsrc > 1 && !stage_.d2hRest.empty()) {
    GLX_HIP_CHECK(hipEventRecord(hostDone_, compute_));
    GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, hostDone_, 0));
    copyBack(stage_.d2hRest);
  }
  waitDevice(compute_);
  GLX_HIP_CHECK(hipStreamSynchronize(d2h_));
  GLX_HIP_CHECK(hipStreamSynchronize(h2d_));
  noteDone(d2h_);
  checkDevice();
  flushMirrors();
  if (hostFold_) {  // local broadcast on the host
    for (void* p : ptrs_) std::memcpy(p, hostStage_, bytes);
  }
}

}  // namespace gloo
