// executor.cc -- see executor.h.
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
#include "host_ops.h"
#include "kernels.h"

namespace gloo {

namespace {

constexpr uint32_t kAlgMagic = 0x474c5841u;  // "GLXA"

template <typename T>
void putPod(std::vector<char>& b, const T& v) {
  b.insert(b.end(), (const char*)&v, (const char*)&v + sizeof(T));
}

template <typename T>
T getPod(const std::vector<char>& b, size_t& at) {
  GLX_ENFORCE(at + sizeof(T) <= b.size(), "truncated algorithm record");
  T v;
  memcpy(&v, b.data() + at, sizeof(T));
  at += sizeof(T);
  return v;
}

void putRef(std::vector<char>& b, const SharedRef& r) {
  putPod(b, r.ptr);
  putPod(b, r.id);
  putPod(b, r.ipcStatus);
  putPod(b, r.ipc);
  putPod(b, r.canaryOff);
  putPod(b, r.canary);
  putPod(b, r.baseOff);
}

SharedRef getRef(const std::vector<char>& b, size_t& at) {
  SharedRef r;
  r.ptr = getPod<uint64_t>(b, at);
  r.id = getPod<int64_t>(b, at);
  r.ipcStatus = getPod<int32_t>(b, at);
  r.ipc = getPod<hipIpcMemHandle_t>(b, at);
  r.canaryOff = getPod<uint64_t>(b, at);
  r.canary = getPod<uint64_t>(b, at);
  r.baseOff = getPod<uint64_t>(b, at);
  return r;
}

enum { DIR_IN = 0, DIR_OUT = 1 };

// A SEND is split only when every part is at least this big.
constexpr size_t kMinSplitBytes = 1 << 20;

int initialSplit() {
  const char* e = std::getenv("GLOO_AMD_COPY_SPLIT");
  int k = e ? std::atoi(e) : 1;
  return k < 1 ? 1 : k;
}

std::atomic<int> g_copy_split{initialSplit()};

// Default: hipMemcpyPeerAsync (the DMA engines); GLOO_AMD_COPY_ENGINE=kernel
// selects the copy kernel (the sending GPU's compute units store into the
// receiver's region over xGMI).
int initialEngine() {
  const char* e = std::getenv("GLOO_AMD_COPY_ENGINE");
  return (e != nullptr && std::strcmp(e, "kernel") == 0) ? 1 : 0;
}

std::atomic<int> g_copy_engine{initialEngine()};

// GLOO_AMD_TRACE=1: one stderr line per executor step / runtime call.
const bool g_trace = [] {
  const char* e = std::getenv("GLOO_AMD_TRACE");
  return e != nullptr && e[0] == '1';
}();

#define GLX_TRACE(...)                        \
  do {                                        \
    if (g_trace) {                            \
      std::fprintf(stderr, "[glx-trace] " __VA_ARGS__); \
      std::fputc('\n', stderr);              \
    }                                         \
  } while (0)

// Host memory (pageable or pinned) as opposed to device/managed memory.
bool isHostPointer(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return true;  // unknown to HIP: plain pageable host memory
  }
  return a.type == hipMemoryTypeHost || a.type == hipMemoryTypeUnregistered;
}

bool isPinnedHost(const void* p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

// Blocking wait for a stream with a short wake-up: poll for up to 200 us
// (a device-driven small allreduce finishes in a few us; the runtime's
// blocking wait adds several us of wake-up), then block.
hipError_t spinSync(hipStream_t s) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    if (std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(200)) break;
    _mm_pause();
  }
  return hipStreamSynchronize(s);
}

// H2D pieces of host-mode staging: small enough that the schedule starts
// early, large enough to run the PCIe link at full rate.
constexpr int64_t kStagePieceBytes = int64_t(8) << 20;

}  // namespace

void HipPlanExecutor::setCopySplit(int k) {
  g_copy_split.store(std::max(1, std::min(k, (int)kMaxSplit)));
}

int HipPlanExecutor::copySplit() { return g_copy_split.load(); }

void HipPlanExecutor::setCopyEngine(int engine) { g_copy_engine.store(engine == 1 ? 1 : 0); }

int HipPlanExecutor::copyEngine() { return g_copy_engine.load(); }

HipPlanExecutor::HipPlanExecutor(const std::shared_ptr<Context>& ctx, int algo,
                                 const std::vector<void*>& ptrs, int64_t count,
                                 int dtype, int op,
                                 const std::vector<hipStream_t>& streams,
                                 const glx::PlanParams& prm, bool perCallBuffers)
    : Algorithm(ctx), algo_(algo), ptrs_(ptrs), count_(count), dtype_(dtype), op_(op) {
  try {
    construct(ctx, ptrs, streams, prm, perCallBuffers);
  } catch (...) {
    release();
    throw;
  }
}

void HipPlanExecutor::construct(const std::shared_ptr<Context>& ctx,
                                const std::vector<void*>& ptrs,
                                const std::vector<hipStream_t>& streams,
                                const glx::PlanParams& prm, bool perCallBuffers) {
  const int algo = algo_, dtype = dtype_, op = op_;
  const int64_t count = count_;
  GLX_ENFORCE(!ptrs.empty(), "at least one buffer pointer is required");
  GLX_ENFORCE(count >= 0 && count <= (int64_t(1) << 40), "count out of range: ", count);
  esize_ = glx_dtype_size(dtype);
  GLX_ENFORCE(esize_ > 0, "unknown dtype ", dtype);
  GLX_ENFORCE(op >= GLX_SUM && op <= GLX_MIN, "unknown reduction op ", op);
  GLX_ENFORCE(streams.empty() || streams.size() == ptrs.size(),
              "streams must be empty or one per pointer (got ", streams.size(),
              " for ", ptrs.size(), " pointers)");
  GLX_ENFORCE(ptrs.size() <= 8, "at most 8 local pointers are supported");
  for (void* p : ptrs) GLX_ENFORCE(p != nullptr || count == 0, "null buffer pointer");
  GLX_ENFORCE(contextSize_ == 1 || ctx->connected(),
              "context must be connected (connectFullMesh) before creating algorithms");
  device_ = ctx->device();
  GLX_HIP_CHECK(hipSetDevice(device_));
  slot_ = ctx->nextSlot();
  GLX_TRACE("r%d new algorithm: slot %d, algo %d, count %ld, dtype %d, op %d", contextRank_,
            slot_, algo_, (long)count_, dtype_, op_);
  glx::PlanParams pp = prm;
  pp.esize = (int)esize_;
  plan_ = glx::makePlan(algo, contextRank_, contextSize_, count, pp);
  prm_ = pp;

  userStream_ = !streams.empty();
  if (userStream_) {
    GLX_ENFORCE(perCallBuffers || streams.size() == 1 || streams.size() == ptrs.size(),
                "streams: pass one per pointer (", ptrs.size(), "), or one; got ",
                streams.size());
    compute_ = streams[0];
    for (size_t i = 1; i < streams.size(); i++) {
      if (streams[i] == compute_) continue;
      sideStreams_.push_back(streams[i]);
      sideIn_.push_back(nullptr);
      GLX_HIP_CHECK(hipEventCreateWithFlags(&sideIn_.back(), hipEventDisableTiming));
    }
    if (!sideStreams_.empty()) {
      GLX_HIP_CHECK(hipEventCreateWithFlags(&sideOut_, hipEventDisableTiming));
    }
  } else {
    GLX_HIP_CHECK(hipStreamCreateWithFlags(&compute_, hipStreamNonBlocking));
    ownCompute_ = true;
  }
  split_ = std::max(1, std::min(copySplit(), (int)kMaxSplit));
  copyEngine_ = copyEngine();

  // perCallBuffers (function style): ptrs only describe the first call; the
  // buffers of every call come with runFn, host ones staged per call there
  hostMode_ = !perCallBuffers && count_ > 0 && isHostPointer(ptrs[0]);
  for (void* p : ptrs) {
    GLX_ENFORCE(perCallBuffers || count_ == 0 || isHostPointer(p) == hostMode_,
                "buffers must be all device memory or all host memory");
  }
  GLX_ENFORCE(!hostMode_ || !userStream_, "streams cannot be used with host-memory buffers");
  if (hostMode_) setupHostMode();
  staged_ = hostMode_;
  if (!hostMode_ && !perCallBuffers && count_ > 0) {
    // pointers on other GPUs of this rank (the reference's multi-device
    // ranks, gloo/cuda_allreduce_ring_chunked.cc): the fold kernel reads them
    // and the broadcast writes them over xGMI from this rank's device
    for (void* p : ptrs) {
      hipPointerAttribute_t a;
      if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();
        continue;
      }
      if (a.type == hipMemoryTypeDevice && a.device >= 0 && a.device != device_) {
        int can = 0;
        GLX_HIP_CHECK(hipDeviceCanAccessPeer(&can, device_, a.device));
        GLX_ENFORCE(can, "buffer on device ", a.device, " is not reachable from device ",
                    device_, " (no peer access)");
        hipError_t e = hipDeviceEnablePeerAccess(a.device, 0);
        if (e == hipErrorPeerAccessAlreadyEnabled) {
          (void)hipGetLastError();
        } else {
          GLX_HIP_CHECK(e);
        }
      }
    }
  }

  engine_ = engineFor(*ctx, algo, count_, (int)esize_);
  if (engine_ == kEngineDevSteps) {
    // the plan kernel's grid and bookkeeping; when a landing region would be
    // shared by two workgroups across messages, keep the host-issued steps
    // (every rank computes the same from every rank's program)
    const size_t minSlice = 4096 / esize_;
    const glx::SyncTable probe = glx::syncTable(algo, contextRank_, contextSize_, count_, pp, 1);
    int64_t maxSeg = 1;
    for (size_t k = 0; k + 1 < probe.bounds.size(); k++) {
      maxSeg = std::max(maxSeg, probe.bounds[k + 1] - probe.bounds[k]);
    }
    const size_t G = std::max<size_t>(
        1, std::min(maxSlices(2), ((size_t)maxSeg + minSlice - 1) / minSlice));
    // programs without FOLD steps run the 2-source variant (81 instead of 145
    // VGPRs).  The grid stays sized by the 8-source variant's residency: with
    // 8 ranks sharing one GPU, 160 instead of 96 workgroups per rank made the
    // 256 MiB ring 30 % slower (stores through the IPC mappings contend;
    // profiles/r2k_*); one rank per GPU gets 512 either way.
    pk_.maxSrc = probe.anyFold ? glx::kOsMaxRanks : 2;
    sync_ = glx::syncTable(algo, contextRank_, contextSize_, count_, pp, (int)G);
    pk_.G = (int)G;
    // GLOO_AMD_FUSE=0: one landing slot per channel and no reduce-and-forward
    // (the round-1 protocol; every rank must agree, which resolvePeers checks)
    static const bool fuse = [] {
      const char* e = std::getenv("GLOO_AMD_FUSE");
      return !(e != nullptr && e[0] == '0');
    }();
    slots_ = fuse ? sync_.slots : 1;
    if (!sync_.safe) engine_ = kEngineSteps;
  }
  if (engine_ == kEngineOneShot || engine_ == kEngineTwoShot) {
    setupDevice();
  } else {
    // Receive regions are uncached for every engine: peers' stores (their
    // kernels' or DMA) land behind this GPU's L2, and a region is reused
    // every run, so no stale line of an earlier message may be cached.  (The
    // plan kernel reads its `slots_` landing slots inside the launch right
    // after an in-kernel flag wait, where nothing else could drop such a
    // line.)  GLOO_AMD_STEPS_SCRATCH=cached gives the host-issued and queued
    // engines hipMalloc'd regions instead (diagnostics).
    static const bool stepsCached = [] {
      const char* e = std::getenv("GLOO_AMD_STEPS_SCRATCH");
      return e != nullptr && std::strcmp(e, "cached") == 0;
    }();
    const bool uncached = engine_ == kEngineDevSteps || !stepsCached;
    allocScratch(uncached, engine_ == kEngineDevSteps ? slots_ : 1);
  }

  // Channels named by the plan; allocate our counter words.
  auto& ctl = ctx->localControl();
  stepChan_.assign(plan_.steps.size(), -1);
  const bool hostSteps = engine_ == kEngineSteps;
  const bool copyStreams = hostSteps || engine_ == kEngineQueued;
  for (size_t i = 0; i < plan_.steps.size() &&
                     (copyStreams || engine_ == kEngineDevSteps);
       i++) {
    const auto& s = plan_.steps[i];
    if (s.kind == glx::SEND) {
      int idx = outIndex((int)s.peer, (int)s.channel);
      if (idx < 0) {
        OutChan oc;
        oc.peer = (int)s.peer;
        oc.tag = (int)s.channel;
        // plan kernel: no control-block words or copy streams; queued: copy
        // streams, no words (flag rows are assigned in setupDevSteps /
        // setupQueued)
        oc.creditWord = hostSteps ? ctl.allocWord() : 0;
        oc.credit = hostSteps ? ctl.word(oc.creditWord) : nullptr;
        // one copy stream per destination peer: copies to different peers
        // run concurrently on different xGMI links
        oc.stream = copyStreams ? -1 : 0;
        for (const auto& o : out_) {
          if (copyStreams && o.peer == oc.peer) oc.stream = o.stream;
        }
        if (oc.stream < 0) {
          oc.stream = (int)copies_.size();
          for (int j = 0; j < split_; j++) {
            CopyStream cs;
            GLX_HIP_CHECK(hipStreamCreateWithFlags(&cs.s, hipStreamNonBlocking));
            copies_.push_back(cs);
          }
        }
        out_.push_back(oc);
        idx = (int)out_.size() - 1;
      }
      stepChan_[i] = idx;
    } else if (s.kind == glx::RECV || s.kind == glx::RELEASE) {
      int idx = inIndex((int)s.peer, (int)s.channel);
      if (idx < 0) {
        InChan ic;
        ic.peer = (int)s.peer;
        ic.tag = (int)s.channel;
        ic.deliveryWord = hostSteps ? ctl.allocWord() : 0;
        ic.delivery = hostSteps ? ctl.word(ic.deliveryWord) : nullptr;
        in_.push_back(ic);
        idx = (int)in_.size() - 1;
      }
      stepChan_[i] = idx;
    }
  }
  if (engine_ == kEngineDevSteps || engine_ == kEngineQueued) setupDevice();
  events_.resize(plan_.steps.size() * (size_t)split_, nullptr);
  for (auto& e : events_) GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  GLX_HIP_CHECK(hipEventCreateWithFlags(&computeMark_, hipEventDisableTiming));
  GLX_HIP_CHECK(hipEventCreateWithFlags(&lastDone_, hipEventDisableTiming));
  if (contextSize_ > 1 && count_ > 0) publish();
}

HipPlanExecutor::~HipPlanExecutor() noexcept(false) { release(); }

void HipPlanExecutor::drainCredits() noexcept {
  if (broken_) return;  // a peer timed out or exited: nothing more will come
  const auto deadline = std::chrono::steady_clock::now() + effectiveTimeout();
  auto pause = [] { std::this_thread::sleep_for(std::chrono::microseconds(50)); };
  try {
    if (engine_ == kEngineSteps) {
      for (auto& oc : out_) {
        while (oc.credit != nullptr && oc.credit->load(std::memory_order_acquire) < oc.sent &&
               std::chrono::steady_clock::now() < deadline) {
          context_->checkPeersAlive();
          pause();
        }
      }
    } else if (engine_ == kEngineDevSteps && devRuns_ > 0 && !ddBlocks_.empty()) {
      // final credit of out-channel c on every workgroup: devRuns_ * perRun
      std::vector<uint64_t> want(out_.size(), 0);
      for (size_t i = 0; i < plan_.steps.size() && i < sync_.steps.size(); i++) {
        if (plan_.steps[i].kind == glx::SEND) {
          const size_t c = (size_t)sync_.steps[i].chan;
          if (c < want.size()) want[c] = devRuns_ * sync_.steps[i].perRun;
        }
      }
      const size_t G = (size_t)pk_.G;
      std::vector<uint64_t> row(G * glx::kFlagStride);
      for (size_t c = 0; c < out_.size(); c++) {
        const uint64_t* dev = reinterpret_cast<const uint64_t*>(ddBlocks_[0]) +
                              (size_t)out_[c].creditWord * G * glx::kFlagStride;
        for (;;) {
          if (hipMemcpy(row.data(), dev, G * glx::kFlagBytes, hipMemcpyDeviceToHost) !=
              hipSuccess) {
            (void)hipGetLastError();
            break;
          }
          bool done = true;
          for (size_t w = 0; w < G && done; w++) done = row[w * glx::kFlagStride] >= want[c];
          if (done || std::chrono::steady_clock::now() >= deadline) break;
          context_->checkPeersAlive();  // throws if a peer exited: stop waiting
          pause();
        }
      }
    }
    if (engine_ == kEngineQueued && !ddBlocks_.empty()) {
      for (const auto& oc : out_) {
        for (;;) {
          uint64_t v = 0;
          if (hipMemcpy(&v, flagRow(oc.creditWord), sizeof(v), hipMemcpyDeviceToHost) !=
              hipSuccess) {
            (void)hipGetLastError();
            break;
          }
          if (v >= oc.sent || std::chrono::steady_clock::now() >= deadline) break;
          context_->checkPeersAlive();
          pause();
        }
      }
    }
  } catch (...) {
  }
}

void HipPlanExecutor::release() noexcept {
  if (device_ < 0) return;  // nothing was acquired
  hipSetDevice(device_);
  drainCredits();
  // the last call's work may sit on a caller's stream (runFn with a stream):
  // it reads our scratch until it completes
  if (lastDone_ != nullptr && lastStream_ != nullptr) hipEventSynchronize(lastDone_);
  if (compute_ != nullptr) hipStreamSynchronize(compute_);
  for (auto& c : copies_) hipStreamSynchronize(c.s);
  for (hipStream_t st : {h2d_, d2h_}) {
    if (st != nullptr) {
      hipStreamSynchronize(st);
      hipStreamDestroy(st);
    }
  }
  for (auto& e : h2dEvents_) {
    if (e != nullptr) hipEventDestroy(e);
  }
  for (auto& e : pieceDone_) {
    if (e != nullptr) hipEventDestroy(e);
  }
  for (auto& e : d2hEvents_) {
    if (e != nullptr) hipEventDestroy(e);
  }
  if (hostDone_) hipEventDestroy(hostDone_);
  for (auto& e : doneEvents_) {
    if (e != nullptr) hipEventDestroy(e);
  }
  for (char* d : devBufs_) hipFree(d);
  if (hostStage_) hipHostFree(hostStage_);
  for (char* d : fnStage_) hipFree(d);
  for (void* p : registered_) hipHostUnregister(p);
  for (auto& e : events_) {
    if (e != nullptr) hipEventDestroy(e);
  }
  if (computeMark_) hipEventDestroy(computeMark_);
  if (lastDone_) hipEventDestroy(lastDone_);
  for (auto& e : sideIn_) {
    if (e != nullptr) hipEventDestroy(e);
  }
  sideIn_.clear();
  if (sideOut_) hipEventDestroy(sideOut_);
  sideOut_ = nullptr;
  for (auto& b : blocks_) {
    if (b.ref.id > 0) context_->releaseShared(b.ref.id);
  }
  for (const SharedRef& r : ddRefs_) context_->releaseShared(r.id);
  if (ddStatus_) hipHostFree(ddStatus_);
  if (ddClaim_) hipFree(ddClaim_);
  if (trace_) hipHostFree(trace_);
  if (ddDone_) hipEventDestroy(ddDone_);
  for (auto& c : copies_) hipStreamDestroy(c.s);
  if (ownCompute_ && compute_) hipStreamDestroy(compute_);
  if (devSteps_) hipFree(devSteps_);
  if (devSegs_) hipFree(devSegs_);
  if (devFoldSrc_) hipFree(devFoldSrc_);
  if (engine_ == kEngineSteps) {
    auto& ctl = context_->localControl();
    for (auto& oc : out_) ctl.freeWord(oc.creditWord);
    for (auto& ic : in_) ctl.freeWord(ic.deliveryWord);
  }
}

int HipPlanExecutor::outIndex(int peer, int tag) {
  for (size_t i = 0; i < out_.size(); i++)
    if (out_[i].peer == peer && out_[i].tag == tag) return (int)i;
  return -1;
}

int HipPlanExecutor::inIndex(int peer, int tag) {
  for (size_t i = 0; i < in_.size(); i++)
    if (in_[i].peer == peer && in_[i].tag == tag) return (int)i;
  return -1;
}


// Our record for this algorithm instance: where peers land their messages
// (scratch pointer / IPC handle) and which counter words they bump (our
// delivery words) or watch (our credit words).
void HipPlanExecutor::publish() {
  std::vector<char> b;
  putPod<uint32_t>(b, kAlgMagic);
  putPod<int64_t>(b, (int64_t)::getpid());
  // what this slot holds: peers check it against their own algorithm
  putPod<int32_t>(b, (int32_t)algo_);
  putPod<int64_t>(b, count_);
  putPod<int32_t>(b, (int32_t)dtype_);
  putPod<int32_t>(b, (int32_t)op_);
  putPod<int32_t>(b, (int32_t)blocks_.size());
  for (const auto& blk : blocks_) {
    putPod<int64_t>(b, blk.start);
    putPod<int64_t>(b, blk.elems);
    putRef(b, blk.ref);
  }
  putPod<int32_t>(b, (int32_t)(in_.size() + out_.size()));
  for (auto& ic : in_) {
    putPod<int32_t>(b, ic.peer);
    putPod<int32_t>(b, ic.tag);
    putPod<int32_t>(b, DIR_IN);
    putPod<int32_t>(b, (int32_t)ic.deliveryWord);
  }
  for (auto& oc : out_) {
    putPod<int32_t>(b, oc.peer);
    putPod<int32_t>(b, oc.tag);
    putPod<int32_t>(b, DIR_OUT);
    putPod<int32_t>(b, (int32_t)oc.creditWord);
  }
  putPod<int32_t>(b, engine_);
  putPod<int32_t>(b, (int32_t)slots_);
  putPod<int32_t>(b, (int32_t)copyEngine_);
  putPod<int32_t>(b, (int32_t)ddBlocks_.size());
  for (size_t k = 0; k < ddBlocks_.size(); k++) putRef(b, ddRefs_[k]);
  const std::vector<int64_t> retired = context_->retiredShared();
  putPod<int32_t>(b, (int32_t)retired.size());
  for (int64_t id : retired) putPod<int64_t>(b, id);
  context_->store().set(
      "glx/alg/" + std::to_string(slot_) + "/" + std::to_string(contextRank_), b);
}

// The retired shared-block ids at the end of an algorithm record (publish).
std::vector<int64_t> HipPlanExecutor::retiredIn(const std::vector<char>& rec) const {
  // walk the record's fixed parts to its tail
  size_t at = 0;
  getPod<uint32_t>(rec, at);
  getPod<int64_t>(rec, at);
  getPod<int32_t>(rec, at);
  getPod<int64_t>(rec, at);
  getPod<int32_t>(rec, at);
  getPod<int32_t>(rec, at);
  const int32_t nblocks = getPod<int32_t>(rec, at);
  for (int32_t k = 0; k < nblocks; k++) {
    getPod<int64_t>(rec, at);
    getPod<int64_t>(rec, at);
    getRef(rec, at);
  }
  const int32_t nchan = getPod<int32_t>(rec, at);
  at += (size_t)nchan * 4 * sizeof(int32_t);
  getPod<int32_t>(rec, at);  // engine
  getPod<int32_t>(rec, at);  // slots
  getPod<int32_t>(rec, at);  // copy engine
  const int32_t nb = getPod<int32_t>(rec, at);
  for (int32_t k = 0; k < nb; k++) getRef(rec, at);
  const int32_t n = getPod<int32_t>(rec, at);
  std::vector<int64_t> ids;
  for (int32_t i = 0; i < n; i++) ids.push_back(getPod<int64_t>(rec, at));
  return ids;
}

void HipPlanExecutor::resolvePeers() {
  std::map<int, bool> peers;
  for (auto& oc : out_) peers[oc.peer] = true;
  for (auto& ic : in_) peers[ic.peer] = true;
  for (int r = 0; r < contextSize_ && engine_ != kEngineSteps; r++) {
    if (r != contextRank_) peers[r] = true;
  }
  for (auto& kv : peers) {
    const int r = kv.first;
    PeerEndpoint& pe = context_->peer(r);
    GLX_TRACE("r%d resolve: get record of rank %d", contextRank_, r);
    auto b = context_->store().get(
        "glx/alg/" + std::to_string(slot_) + "/" + std::to_string(r),
        effectiveTimeout());
    size_t at = 0;
    GLX_ENFORCE(getPod<uint32_t>(b, at) == kAlgMagic, "bad algorithm record from rank ", r);
    getPod<int64_t>(b, at);  // pid (already known from the endpoint)
    const int32_t ralgo = getPod<int32_t>(b, at);
    const int64_t rcount = getPod<int64_t>(b, at);
    const int32_t rdtype = getPod<int32_t>(b, at);
    const int32_t rop = getPod<int32_t>(b, at);
    GLX_ENFORCE(ralgo == algo_ && rcount == count_ && rdtype == dtype_ && rop == op_,
                "rank ", r, "'s algorithm in slot ", slot_, " (algorithm ", ralgo, ", count ",
                rcount, ", dtype ", rdtype, ", op ", rop, ") differs from rank ", contextRank_,
                "'s (algorithm ", algo_, ", count ", count_, ", dtype ", dtype_, ", op ", op_,
                "): the ranks created their algorithms in different orders");
    // the peer's retired blocks sit at the end of its record: close our
    // mappings of them before mapping anything new
    if (!pe.sameProcess) context_->dropImported(r, retiredIn(b));
    const int32_t nblocks = getPod<int32_t>(b, at);
    bool needScratch = false;
    for (auto& oc : out_) needScratch = needScratch || oc.peer == r;
    std::vector<ScratchBlock> pb;
    for (int32_t k = 0; k < nblocks; k++) {
      ScratchBlock blk;
      blk.start = getPod<int64_t>(b, at);
      blk.elems = getPod<int64_t>(b, at);
      blk.ref = getRef(b, at);
      if (!needScratch) continue;
      if (pe.sameProcess) {
        blk.ptr = reinterpret_cast<char*>((uintptr_t)blk.ref.ptr);
      } else {
        blk.ptr = context_->importShared(r, blk.ref);
        GLX_TRACE("r%d resolve: rank %d block %d (shared %ld, %ld elems) at %p", contextRank_,
                  r, k, (long)blk.ref.id, (long)blk.elems, (void*)blk.ptr);
      }
      pb.push_back(blk);
    }
    if (needScratch) peerBlocks_[r] = pb;
    int32_t n = getPod<int32_t>(b, at);
    for (int32_t i = 0; i < n; i++) {
      int32_t peer = getPod<int32_t>(b, at);
      int32_t tag = getPod<int32_t>(b, at);
      int32_t dir = getPod<int32_t>(b, at);
      int32_t word = getPod<int32_t>(b, at);
      if (peer != contextRank_) continue;
      if (dir == DIR_IN) {  // peer receives from us on `tag`
        int idx = outIndex(r, tag);
        if (idx >= 0) {
          if (engine_ == kEngineSteps) out_[idx].delivery = pe.ctl->word((uint32_t)word);
          out_[idx].peerRow = word;
          out_[idx].peerDevice = pe.localDevice;
        }
      } else {  // peer sends to us on `tag`: its credit word
        int idx = inIndex(r, tag);
        if (idx >= 0) {
          if (engine_ == kEngineSteps) in_[idx].credit = pe.ctl->word((uint32_t)word);
          in_[idx].peerRow = word;
        }
      }
    }
    const int32_t peerEngine = getPod<int32_t>(b, at);
    GLX_ENFORCE(peerEngine == engine_, "rank ", r, " runs engine ", peerEngine, ", rank ",
                contextRank_, " engine ", engine_, " (schedules disagree)");
    const int32_t peerSlots = getPod<int32_t>(b, at);
    GLX_ENFORCE(engine_ != kEngineDevSteps || peerSlots == slots_, "rank ", r, " keeps ",
                peerSlots, " landing slot(s) per channel, rank ", contextRank_, " ", slots_,
                " (GLOO_AMD_FUSE must be the same on every rank)");
    getPod<int32_t>(b, at);  // the peer's copy engine (recorded for diagnostics)
    const int32_t nb = getPod<int32_t>(b, at);
    std::vector<char*> blocks;
    for (int32_t k = 0; k < nb; k++) {
      const SharedRef ref = getRef(b, at);
      if (pe.sameProcess) {
        blocks.push_back(reinterpret_cast<char*>((uintptr_t)ref.ptr));
      } else {
        blocks.push_back(context_->importShared(r, ref));
      }
    }
    if (engine_ != kEngineSteps) ddPeer_[r] = blocks;
    if (engine_ == kEngineDevSteps || engine_ == kEngineQueued) {  // the peer's flag rows
      GLX_ENFORCE(!blocks.empty(), "rank ", r, " published no flag rows");
      uint64_t* rows = reinterpret_cast<uint64_t*>(blocks[0]);
      const size_t G = (size_t)pk_.G;
      for (auto& oc : out_) {
        if (oc.peer == r && oc.peerRow >= 0) {
          oc.devDelivery = rows + (size_t)oc.peerRow * G * glx::kFlagStride;
        }
      }
      for (auto& ic : in_) {
        if (ic.peer == r && ic.peerRow >= 0) {
          ic.devCredit = rows + (size_t)ic.peerRow * G * glx::kFlagStride;
        }
      }
    }
  }
  const bool dev = engine_ == kEngineDevSteps || engine_ == kEngineQueued;
  for (auto& oc : out_) {
    GLX_ENFORCE(dev ? oc.devDelivery != nullptr : oc.delivery != nullptr, "rank ", oc.peer,
                " has no receive channel ", oc.tag, " from rank ", contextRank_,
                " (schedules disagree)");
  }
  for (auto& ic : in_) {
    GLX_ENFORCE(dev ? ic.devCredit != nullptr : ic.credit != nullptr, "rank ", ic.peer,
                " has no send channel ", ic.tag, " to rank ", contextRank_,
                " (schedules disagree)");
  }
  resolved_ = true;
}

// A message for ptr0[off, ...) lands at the 16-byte phase that offset has in
// a 16-byte aligned buffer, so the reduce kernel reading it next to ptr0 stays
// on its 16-byte vector path (an unaligned ptr0 still works: the kernel then
// takes its scalar path).  Both sides compute it from `off` alone.
char* HipPlanExecutor::landing(const std::vector<ScratchBlock>& blocks, int64_t boff,
                               int64_t off, int64_t len) const {
  const ScratchBlock* blk = nullptr;
  for (const auto& b : blocks) {
    if (b.start <= boff && boff < b.start + b.elems) {
      blk = &b;
      break;
    }
  }
  GLX_ENFORCE(blk != nullptr && blk->ptr != nullptr, "no receive block holds region ", boff);
  uintptr_t at = ((uintptr_t)(boff - blk->start) * esize_ + 15) & ~(uintptr_t)15;
  at += ((uintptr_t)off * esize_) % 16;
  if (len >= 0) {  // a copy or reduce of len elements stays inside the block (slot 0)
    const size_t cap = slots_ > 1 ? slotBytes(*blk) : (size_t)blk->elems * esize_ + 64;
    GLX_ENFORCE(at + (size_t)len * esize_ <= cap, "receive region ", boff, " (+", len,
                " elements at byte ", at, ") overruns its block of ", cap, " bytes");
    GLX_ENFORCE(off >= 0 && off + len <= count_, "step range [", off, ", ", off + len,
                ") outside the buffer of ", count_, " elements");
  }
  return blk->ptr + at;
}

// Shared blocks are exported as soon as they are allocated; the handle goes
// into the algorithm record (publish).
char* HipPlanExecutor::allocShared(size_t bytes, unsigned flags, SharedRef* ref) {
  const SharedBlock b = context_->acquireShared(bytes, flags);
  *ref = b.ref;
  GLX_TRACE("r%d shared block %ld (%zu bytes) at %p, base offset %lu", contextRank_,
            (long)b.ref.id, b.bytes, (void*)b.ptr, (unsigned long)b.ref.baseOff);
  return b.ptr;
}

// Bytes from one landing slot of a scratch block to the next.
size_t HipPlanExecutor::slotBytes(const ScratchBlock& b) const {
  return ((size_t)b.elems * esize_ + 64 + 255) & ~(size_t)255;
}

const HipPlanExecutor::ScratchBlock& HipPlanExecutor::blockOf(
    const std::vector<ScratchBlock>& blocks, int64_t boff) const {
  for (const auto& b : blocks) {
    if (b.start <= boff && boff < b.start + b.elems) return b;
  }
  GLX_ENFORCE(false, "no receive block holds region ", boff);
  return blocks.front();
}

void HipPlanExecutor::allocScratch(bool uncached, int slots) {
  if (plan_.scratch_elems <= 0) return;
  // region starts = where messages land
  std::vector<int64_t> starts;
  for (const auto& s : plan_.steps) {
    if (s.kind == glx::RECV) starts.push_back(s.boff);
  }
  starts.push_back(0);
  std::sort(starts.begin(), starts.end());
  starts.erase(std::unique(starts.begin(), starts.end()), starts.end());
  starts.push_back(plan_.scratch_elems);  // sentinel
  ScratchBlock cur;
  cur.start = 0;
  for (size_t i = 0; i + 1 < starts.size(); i++) {
    const int64_t regionElems = starts[i + 1] - starts[i];
    const size_t curBytes = (size_t)cur.elems * esize_;
    if (cur.elems > 0 && curBytes + (size_t)regionElems * esize_ > kMaxBlockBytes) {
      blocks_.push_back(cur);
      cur = ScratchBlock();
      cur.start = starts[i];
    }
    cur.elems += regionElems;
  }
  if (cur.elems > 0) blocks_.push_back(cur);
  for (auto& b : blocks_) {
    const size_t bytes = slots > 1 ? (size_t)slots * slotBytes(b) : (size_t)b.elems * esize_ + 64;
    b.ptr = allocShared(bytes, uncached ? hipDeviceMallocUncached : 0u, &b.ref);
    GLX_HIP_CHECK(hipMemset(b.ptr, 0, bytes));
  }
  GLX_HIP_CHECK(hipDeviceSynchronize());
}

void HipPlanExecutor::pollPending() {
  for (size_t i = 0; i < pending_.size();) {
    Pending& p = pending_[i];
    bool blocked = false;  // never overtake an earlier signal to the same word
    for (size_t j = 0; j < i && !blocked; j++) blocked = pending_[j].word == p.word;
    bool done = false;
    if (!blocked) {
      done = true;
      for (int k = 0; k < p.nev && done; k++) {
        hipError_t e = hipEventQuery(p.ev[k]);
        if (e == hipErrorNotReady) {
          done = false;
        } else if (e != hipSuccess) {
          GLX_HIP_CHECK(e);
        }
      }
    }
    if (done) {
      p.word->store(p.value, std::memory_order_release);
      pending_.erase(pending_.begin() + (long)i);
    } else {
      i++;
    }
  }
}

template <typename Pred>
void HipPlanExecutor::waitFor(Pred done, const char* what, int peer) {
  if (done()) return;
  const auto timeout = effectiveTimeout();
  const auto start = std::chrono::steady_clock::now();
  auto lastAlive = start;
  bool warned = false;
  for (uint64_t spin = 1;; spin++) {
    pollPending();
    if (done()) return;
    if ((spin & 255) == 0) {
      auto now = std::chrono::steady_clock::now();
      if (!warned && now - start > std::chrono::seconds(10)) {
        // a stuck collective should say where it is stuck long before the timeout
        std::fprintf(stderr,
                     "[gloo_amd] rank %d still waiting for %s from rank %d after 10 s "
                     "(%zu completions pending)\n",
                     contextRank_, what, peer, pending_.size());
        warned = true;
      }
      if (now - start > timeout) {
        broken_ = true;
        GLX_THROW_TIMEOUT(
            "Timed out waiting for ", what, " from rank ", peer, " (rank ",
            contextRank_, ", after ",
            std::chrono::duration_cast<std::chrono::milliseconds>(now - start).count(),
            " ms, timeout ", timeout.count(), " ms)");
      }
      if (now - lastAlive > std::chrono::milliseconds(200)) {
        try {
          context_->checkPeersAlive();
        } catch (...) {
          broken_ = true;
          throw;
        }
        lastAlive = now;
      }
    }
    if (spin > 4096) {
      sched_yield();
    } else {
      _mm_pause();
    }
  }
}

void HipPlanExecutor::waitWar(int64_t off, int64_t len) {
  for (size_t i = 0; i < inflight_.size();) {
    const InflightSend& s = inflight_[i];
    const bool overlap = s.off < off + len && off < s.off + s.len;
    if (overlap) {
      if (hipEventQuery(s.event) != hipSuccess) {
        GLX_HIP_CHECK(hipStreamWaitEvent(compute_, s.event, 0));
      }
      inflight_.erase(inflight_.begin() + (long)i);
    } else {
      i++;
    }
  }
}

void HipPlanExecutor::drain() {
  waitFor([&] { return pending_.empty(); }, "local completions", contextRank_);
}

void HipPlanExecutor::run() {
  if (count_ == 0) return;  // gloo/allreduce_ring_chunked.h:84-86
  GLX_HIP_CHECK(hipSetDevice(device_));
  if (hostMode_) {
    runHost();
    return;
  }
  char* ptr0 = static_cast<char*>(ptrs_[0]);
  const size_t bytes = (size_t)count_ * esize_;
  // the caller's pending work on every pointer's stream comes first
  for (size_t i = 0; i < sideStreams_.size(); i++) {
    GLX_HIP_CHECK(hipEventRecord(sideIn_[i], sideStreams_[i]));
    GLX_HIP_CHECK(hipStreamWaitEvent(compute_, sideIn_[i], 0));
  }

  // Local multi-pointer reduce into ptrs_[0] (left fold, :89-91).
  if (ptrs_.size() > 1) {
    std::vector<const void*> srcs(ptrs_.begin(), ptrs_.end());
    GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, ptr0, srcs.data(), (int)srcs.size(),
                                       (size_t)count_, compute_));
  }
  if (contextSize_ > 1) exchange(ptr0);
  // Local broadcast of ptrs_[0] (:209-211).
  for (size_t i = 1; i < ptrs_.size(); i++) {
    GLX_HIP_CHECK(hipMemcpyAsync(ptrs_[i], ptr0, bytes, hipMemcpyDeviceToDevice, compute_));
  }
  if (sideOut_ != nullptr) {  // results valid on every pointer's stream
    GLX_HIP_CHECK(hipEventRecord(sideOut_, compute_));
    for (hipStream_t st : sideStreams_) GLX_HIP_CHECK(hipStreamWaitEvent(st, sideOut_, 0));
  }
  noteDone(compute_);
  GLX_TRACE("r%d sync", contextRank_);
  if (!userStream_) {
    waitDevice(compute_);
    checkDevice();
  }
  GLX_TRACE("r%d done", contextRank_);
}

// genLocalReduceFunction (gloo/allreduce.cc:44-82) over the whole buffer at
// once: each segment's local reduction happens exactly once in the
// reference, before the segment is first sent or reduced into, and it is
// elementwise, so doing it up front gives the same bits.
void HipPlanExecutor::localReduce(const std::vector<void*>& in,
                                  const std::vector<void*>& out) {
  const size_t n = (size_t)count_;
  void* out0 = out[0];
  if (in.size() == 1) {  // :50-56
    if (in[0] != out0) {
      GLX_HIP_CHECK(hipMemcpyAsync(out0, in[0], n * esize_, hipMemcpyDeviceToDevice, compute_));
    }
  } else if (in.size() >= 2) {  // :58-71
    std::vector<const void*> rest;
    if (dtype_ == GLX_FLOAT16) {
      // out0 = fn(in0, in1) writes a buffer other than its first operand,
      // and float16's assignment reads the destination's old value
      // (gloo/types.h operator=): the two-operand kernel reproduces that
      GLX_HIP_CHECK(glx::launch_reduce(op_, dtype_, out0, in[0], in[1], n, compute_));
      rest.push_back(out0);
      for (size_t i = 2; i < in.size(); i++) rest.push_back(in[i]);
    } else {
      rest.assign(in.begin(), in.end());
    }
    if (rest.size() >= 2) {
      GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, out0, rest.data(), (int)rest.size(), n,
                                         compute_));
    }
  } else if (out.size() >= 2) {  // :72-81, no inputs: fold the outputs
    std::vector<const void*> srcs(out.begin(), out.end());
    GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, out0, srcs.data(), (int)srcs.size(), n,
                                       compute_));
  }
}

void HipPlanExecutor::runFn(const FnCall& call) {
  GLX_ENFORCE(!call.out.empty(), "allreduce needs at least one output");
  for (void* p : call.out) GLX_ENFORCE(p != nullptr || count_ == 0, "null output pointer");
  for (void* p : call.in) GLX_ENFORCE(p != nullptr || count_ == 0, "null input pointer");
  if (count_ == 0) return;  // gloo/allreduce.cc:98-100
  const bool host = isHostPointer(call.out[0]);
  for (void* p : call.out) {
    GLX_ENFORCE(isHostPointer(p) == host, "buffers must be all device or all host memory");
  }
  for (void* p : call.in) {
    GLX_ENFORCE(isHostPointer(p) == host, "buffers must be all device or all host memory");
  }
  GLX_HIP_CHECK(hipSetDevice(device_));
  if (host) {
    runFnHost(call);
    return;
  }
  // per-call stream and timeout (opts.timeout, gloo/allreduce.h:50)
  struct Restore {
    HipPlanExecutor* e;
    hipStream_t s;
    ~Restore() {
      e->compute_ = s;
      e->timeout_ = std::chrono::milliseconds(0);
    }
  } restore{this, compute_};
  if (call.stream != nullptr) compute_ = call.stream;
  timeout_ = call.timeout;
  localReduce(call.in, call.out);
  char* out0 = static_cast<char*>(call.out[0]);
  if (contextSize_ > 1) exchange(out0);  // :129-146
  for (size_t i = 1; i < call.out.size(); i++) {  // broadcastOutputs
    GLX_HIP_CHECK(hipMemcpyAsync(call.out[i], out0, (size_t)count_ * esize_,
                                 hipMemcpyDeviceToDevice, compute_));
  }
  noteDone(compute_);
  if (call.stream == nullptr) {
    waitDevice(compute_);
    checkDevice();
  }
}

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
  for (size_t i = 0; i < srcs.size(); i++) {
    GLX_HIP_CHECK(hipMemcpyAsync(fnStage_[1 + i], srcs[i], bytes, hipMemcpyHostToDevice,
                                 compute_));
  }
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
      GLX_HIP_CHECK(hipMemcpyAsync(out0, call.out[0], bytes, hipMemcpyHostToDevice, compute_));
    }
  }
  localReduce(din, dout);
  if (contextSize_ > 1) exchange(out0);
  for (void* p : call.out) {
    GLX_HIP_CHECK(hipMemcpyAsync(p, out0, bytes, hipMemcpyDeviceToHost, compute_));
  }
  noteDone(compute_);
  waitDevice(compute_);
  checkDevice();
}

void HipPlanExecutor::setupHostMode() {
  const size_t bytes = (size_t)count_ * esize_;
  // Several host pointers under kOnDeviceThreshold: fold them on the host
  // into one pinned staging buffer and stage only that through the device
  // (the reference's cudaHostReduce / cudaHostBroadcast below the threshold,
  // gloo/cuda_allreduce_halving_doubling.cc:478-484)
  hostFold_ = ptrs_.size() > 1 && bytes < glx::kOnDeviceThreshold;
  if (hostFold_) {
    GLX_HIP_CHECK(hipHostMalloc((void**)&hostStage_, std::max<size_t>(bytes, 16),
                                hipHostMallocDefault));
  }
  for (void* p : hostSources()) {
    if (!isPinnedHost(p)) {
      // pin the caller's buffer for the algorithm's lifetime (the reference's
      // algorithms also bind their buffers at construction); if the runtime
      // refuses, pageable copies are still correct, only slower
      if (hipHostRegister(p, bytes, hipHostRegisterPortable) == hipSuccess) {
        registered_.push_back(p);
      } else {
        (void)hipGetLastError();
      }
    }
    char* d = nullptr;
    GLX_HIP_CHECK(hipMalloc((void**)&d, bytes));
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
std::vector<void*> HipPlanExecutor::hostSources() const {
  if (!callSrc_.empty()) return callSrc_;
  if (hostFold_) return {hostStage_};
  return ptrs_;
}

std::vector<void*> HipPlanExecutor::hostDests() const {
  if (!callDst_.empty()) return callDst_;
  return hostSources();
}

// Final values of `ranges` (in devBufs_[0]) to every user pointer, on d2h_
// (the caller has made d2h_ wait for the writes).
void HipPlanExecutor::copyBack(const std::vector<glx::Range>& ranges) {
  for (const glx::Range& r : ranges) {
    const size_t at = (size_t)r.off * esize_, n = (size_t)r.len * esize_;
    for (void* p : hostDests()) {
      GLX_HIP_CHECK(hipMemcpyAsync(static_cast<char*>(p) + at, devBufs_[0] + at, n,
                                   hipMemcpyDeviceToHost, d2h_));
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
  doneQueue_.push_back(DoneBatch{e, ranges});
}

std::vector<glx::Range> HipPlanExecutor::doneRanges() {
  std::lock_guard<std::mutex> g(doneMutex_);
  std::vector<glx::Range> out;
  for (const auto& b : doneQueue_) {
    const hipError_t e = hipEventQuery(b.ev);
    if (e == hipErrorNotReady) {
      (void)hipGetLastError();
      continue;
    }
    GLX_HIP_CHECK(e);
    out.insert(out.end(), b.ranges.begin(), b.ranges.end());
  }
  return out;
}

// Issue piece j's H2D copy (the caller holds feedMutex_ or runs alone).
void HipPlanExecutor::issuePiece(size_t j) {
  const glx::Range& r = stage_.h2d[j];
  const size_t at = (size_t)r.off * esize_, n = (size_t)r.len * esize_;
  const std::vector<void*> hsrc = hostSources();
  for (size_t k = 0; k < hsrc.size(); k++) {
    GLX_HIP_CHECK(hipMemcpyAsync(devBufs_[k] + at, static_cast<const char*>(hsrc[k]) + at, n,
                                 hipMemcpyHostToDevice, h2d_));
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
    copyBack({});
    std::lock_guard<std::mutex> g(doneMutex_);
    if (doneEvents_.empty()) {
      hipEvent_t e = nullptr;
      GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      doneEvents_.push_back(e);
    }
    GLX_HIP_CHECK(hipEventRecord(doneEvents_[0], h2d_));
    doneQueue_.push_back(DoneBatch{doneEvents_[0], {glx::Range{0, count_}}});
    doneUsed_ = 1;
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
  const std::vector<void*> hsrc = hostSources();
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
  if (contextSize_ == 1 && hsrc.size() > 1 && !fedRun_) {
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
    return;
  }
  if (hsrc.size() > 1) {  // local fold needs every buffer whole
    waitH2D(compute_, computeH2dWaited_, 0, count_);
    std::vector<const void*> srcs(devBufs_.begin(), devBufs_.end());
    GLX_HIP_CHECK(glx::launch_reduce_n(op_, dtype_, devBufs_[0], srcs.data(), (int)srcs.size(),
                                       (size_t)count_, compute_));
  }
  if (contextSize_ > 1) exchange(devBufs_[0]);
  // ranges no step wrote: their value is the local fold (a no-op for one
  // pointer, whose host copy already holds it)
  if (hsrc.size() > 1 && !stage_.d2hRest.empty()) {
    GLX_HIP_CHECK(hipEventRecord(hostDone_, compute_));
    GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, hostDone_, 0));
    copyBack(stage_.d2hRest);
  }
  waitDevice(compute_);
  GLX_HIP_CHECK(hipStreamSynchronize(d2h_));
  GLX_HIP_CHECK(hipStreamSynchronize(h2d_));
  noteDone(d2h_);
  checkDevice();
  if (hostFold_) {  // local broadcast on the host
    for (void* p : ptrs_) std::memcpy(p, hostStage_, bytes);
  }
}

void HipPlanExecutor::noteDone(hipStream_t s) {
  GLX_HIP_CHECK(hipEventRecord(lastDone_, s));
  lastStream_ = s;
}

void HipPlanExecutor::recordDone(hipEvent_t ev) {
  GLX_HIP_CHECK(hipSetDevice(device_));
  GLX_HIP_CHECK(hipEventRecord(ev, lastStream_ != nullptr ? lastStream_ : compute_));
}

void HipPlanExecutor::exchange(char* ptr0) {
  if (engine_ == kEngineQueued) {
    exchangeQueued(ptr0);
    return;
  }
  if (engine_ != kEngineSteps) {
    runDevice(ptr0);
    return;
  }
  if (!resolved_) resolvePeers();
  bool computeSinceMark = true;  // the caller's writes to ptr0 count as compute
  for (auto& c : copies_) c.last = nullptr;
  const auto& steps = plan_.steps;
  for (size_t i = 0; i < steps.size(); i++) {
    const glx::Step& s = steps[i];
    GLX_TRACE("r%d step %zu kind %d peer %d chan %d off %ld len %ld", contextRank_, i,
              (int)s.kind, (int)s.peer, (int)s.channel, (long)s.off, (long)s.len);
    switch (s.kind) {
      case glx::SEND: {
        OutChan& oc = out_[stepChan_[i]];
        const uint64_t n = ++oc.sent;
        // one receive region per channel: message n may only land once the
        // receiver has consumed message n-1
        waitFor([&] { return oc.credit->load(std::memory_order_acquire) + 1 >= n; },
                "receive-region credit", oc.peer);
        const size_t nbytes = (size_t)s.len * esize_;
        Pending pd{};
        pd.word = oc.delivery;
        pd.value = n;
        if (nbytes > 0) {
          if (computeSinceMark) {
            GLX_HIP_CHECK(hipEventRecord(computeMark_, compute_));
            markEpoch_++;
            computeSinceMark = false;
          }
          char* dst = landing(peerBlocks_[oc.peer], s.dst_off, s.off, s.len);
          const char* src = ptr0 + (size_t)s.off * esize_;
          int parts = split_;
          while (parts > 1 && nbytes / (size_t)parts < kMinSplitBytes) parts--;
          const size_t per = ((nbytes / (size_t)parts) + 255) & ~(size_t)255;
          for (int j = 0; j < parts; j++) {
            const size_t at = (size_t)j * per;
            if (at >= nbytes) break;
            const size_t len = std::min(per, nbytes - at);
            CopyStream& cs = copies_[oc.stream + j];
            if (cs.waitedMark != markEpoch_) {
              // the chunk may have been produced by compute work: order after it
              GLX_HIP_CHECK(hipStreamWaitEvent(cs.s, computeMark_, 0));
              cs.waitedMark = markEpoch_;
            }
            if (staged_) waitH2D(cs.s, cs.h2dWaited, s.off, s.len);
            hipError_t ce = hipErrorUnknown;
            if (copyEngine_ == kCopyKernel) {
              ce = glx::launch_copy(dst + at, src + at, len, cs.s);
              GLX_HIP_CHECK(ce);
              transport_.kernelCopies++;
            } else if (peerCopyOk_ && oc.peerDevice >= 0 && oc.peerDevice != device_) {
              ce = hipMemcpyPeerAsync(dst + at, oc.peerDevice, src + at, device_, len, cs.s);
              if (ce == hipSuccess) {
                transport_.peerCopies++;
              } else {
                (void)hipGetLastError();
                // e.g. an IPC mapping the peer API rejects: the copy still
                // crosses xGMI (the destination is the peer's memory), now as
                // a plain device copy; say so once and count every one
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
            transport_.bytes += (int64_t)len;
            GLX_TRACE("r%d   copy part %d issued (%zu bytes)", contextRank_, j, len);
            hipEvent_t ev = events_[i * (size_t)split_ + (size_t)j];
            GLX_HIP_CHECK(hipEventRecord(ev, cs.s));
            cs.last = ev;
            inflight_.push_back({s.off, s.len, ev});
            pd.ev[pd.nev++] = ev;
          }
        }
        pending_.push_back(pd);
        break;
      }
      case glx::RECV: {
        InChan& ic = in_[stepChan_[i]];
        const uint64_t n = ++ic.received;
        waitFor([&] { return ic.delivery->load(std::memory_order_acquire) >= n; },
                "data", ic.peer);
        break;
      }
      case glx::REDUCE: {
        waitWar(s.off, s.len);
        if (staged_) waitH2D(compute_, computeH2dWaited_, s.off, s.len);
        char* dst = ptr0 + (size_t)s.off * esize_;
        const char* src = landing(blocks_, s.boff, s.off, s.len);
        GLX_HIP_CHECK(glx::launch_reduce(op_, dtype_, dst, dst, src, (size_t)s.len, compute_));
        computeSinceMark = true;
        if (staged_ && !stage_.d2h[i].empty()) {  // final values: copy back now
          GLX_HIP_CHECK(hipEventRecord(d2hEvents_[i], compute_));
          GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, d2hEvents_[i], 0));
          copyBack(stage_.d2h[i]);
        }
        break;
      }
      case glx::FOLD: {
        // consecutive FOLD steps of the same kind go out as one batched launch
        size_t last = i;
        while (last + 1 < steps.size() && steps[last + 1].kind == glx::FOLD &&
               steps[last + 1].flags == s.flags) {
          last++;
        }
        const bool rev = (s.flags & glx::kFoldLeft) == 0;  // ring chain vs left fold
        const bool whole = (s.flags & glx::kFoldWhole) != 0;
        std::vector<glx::FoldSpec> specs;
        for (size_t q = i; q <= last; q++) {
          const glx::Step& f = steps[q];
          waitWar(f.off, f.len);
          if (staged_) waitH2D(compute_, computeH2dWaited_, f.off, f.len);
          char* dst = ptr0 + (size_t)f.off * esize_;
          glx::FoldSpec spec;
          spec.dst = dst;
          spec.n = (size_t)f.len;
          for (int64_t r : plan_.folds[(size_t)f.boff]) {
            if (r < 0) {
              spec.srcs.push_back(dst);
            } else if (whole) {  // whole-buffer message: element off is off into it
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
          if (staged_ && !stage_.d2h[q].empty()) {  // final values: copy back now
            GLX_HIP_CHECK(hipEventRecord(d2hEvents_[q], compute_));
            GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, d2hEvents_[q], 0));
            copyBack(stage_.d2h[q]);
          }
        }
        i = last;
        break;
      }
      case glx::COPY: {
        waitWar(s.off, s.len);
        if (staged_) waitH2D(compute_, computeH2dWaited_, s.off, s.len);
        char* dst = ptr0 + (size_t)s.off * esize_;
        const char* src = landing(blocks_, s.boff, s.off, s.len);
        // our copy kernel, not hipMemcpyAsync: the region may be uncached
        // memory, which the runtime's copies do not keep in stream order
        // 
        GLX_HIP_CHECK(glx::launch_copy(dst, src, (size_t)s.len * esize_, compute_));
        computeSinceMark = true;
        if (staged_ && !stage_.d2h[i].empty()) {  // final values: copy back now
          GLX_HIP_CHECK(hipEventRecord(d2hEvents_[i], compute_));
          GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, d2hEvents_[i], 0));
          copyBack(stage_.d2h[i]);
        }
        break;
      }
      case glx::RELEASE: {
        InChan& ic = in_[stepChan_[i]];
        const uint64_t v = ++ic.consumed;
        hipEvent_t ev = events_[i * (size_t)split_];
        GLX_HIP_CHECK(hipEventRecord(ev, compute_));
        Pending pd{};
        pd.ev[0] = ev;
        pd.nev = 1;
        pd.word = ic.credit;
        pd.value = v;
        pending_.push_back(pd);
        break;
      }
      default:
        GLX_ENFORCE(false, "bad plan step kind ", s.kind);
    }
    pollPending();
  }
  GLX_TRACE("r%d drain (%zu pending)", contextRank_, pending_.size());
  drain();
  GLX_TRACE("r%d drained", contextRank_);
  // the caller's stream must not run ahead of copies still reading ptr0
  for (auto& c : copies_) {
    if (c.last != nullptr) GLX_HIP_CHECK(hipStreamWaitEvent(compute_, c.last, 0));
  }
  inflight_.clear();
}

// ---------------------------------------------------------------------------
// Device-driven engines (xgmi_kernels.hip)
// ---------------------------------------------------------------------------

namespace {

int initialMeshEngine() {
  const char* e = std::getenv("GLOO_AMD_MESH_ENGINE");
  if (e != nullptr && std::strcmp(e, "steps") == 0) return HipPlanExecutor::kEngineSteps;
  if (e != nullptr && std::strcmp(e, "queued") == 0) return HipPlanExecutor::kEngineQueued;
  return HipPlanExecutor::kEngineTwoShot;
}

std::atomic<int> g_mesh_engine{initialMeshEngine()};

// -1 = by size (the plan kernel up to kDevStepsMaxBytes per rank, where its
// per-step flag round trips beat host-issued steps; host-issued steps with
// their wide copy and reduce launches above), else a fixed engine.
int initialStepsEngine() {
  const char* e = std::getenv("GLOO_AMD_STEPS_ENGINE");
  if (e != nullptr && std::strcmp(e, "host") == 0) return HipPlanExecutor::kEngineSteps;
  if (e != nullptr && std::strcmp(e, "device") == 0) return HipPlanExecutor::kEngineDevSteps;
  if (e != nullptr && std::strcmp(e, "queued") == 0) return HipPlanExecutor::kEngineQueued;
  return -1;
}

int64_t devStepsMaxBytes() {
  const char* e = std::getenv("GLOO_AMD_DEVSTEPS_MAX_BYTES");
  return e != nullptr ? std::atoll(e) : (int64_t(32) << 20);
}

std::atomic<int> g_steps_engine{initialStepsEngine()};

}  // namespace

void HipPlanExecutor::setMeshEngine(int engine) {
  g_mesh_engine.store(engine == kEngineSteps || engine == kEngineQueued ? engine
                                                                       : kEngineTwoShot);
}

int HipPlanExecutor::meshEngine() { return g_mesh_engine.load(); }

void HipPlanExecutor::setStepsEngine(int engine) {
  g_steps_engine.store(engine < 0 ? -1
                                  : (engine == kEngineSteps || engine == kEngineQueued
                                         ? engine
                                         : kEngineDevSteps));
}

int HipPlanExecutor::stepsEngine() { return g_steps_engine.load(); }

namespace {

int initialDeviceEngines() {
  const char* e = std::getenv("GLOO_AMD_ONESHOT");
  if (e != nullptr && e[0] == '0') return 0;
  if (e != nullptr && e[0] == '1') return 1;
  return -1;
}

std::atomic<int> g_device_engines{initialDeviceEngines()};

}  // namespace

void HipPlanExecutor::setDeviceEngines(int mode) {
  g_device_engines.store(mode < 0 ? -1 : (mode > 0 ? 1 : 0));
}

bool HipPlanExecutor::deviceEnginesAvailable(const Context& ctx) {
  if (ctx.size < 2 || ctx.size > glx::kOsMaxRanks) return false;
  const int mode = g_device_engines.load();
  if (mode >= 0) return mode == 1;
  return !ctx.ranksShareDevice();
}

// The inputs are the same on every rank, so every rank makes the same choice
// (and publish/resolve checks that they did).
int HipPlanExecutor::engineFor(const Context& ctx, int algo, int64_t count, int esize) {
  if (count <= 0 || !deviceEnginesAvailable(ctx)) return kEngineSteps;
  if (algo == glx::ALGO_RING_CHUNKED_REPL || algo == glx::ALGO_FN_RING_REPL) {
    return kEngineOneShot;
  }
  if (algo == glx::ALGO_RING_CHUNKED_MESH || algo == glx::ALGO_FN_RING_MESH) {
    return meshEngine();
  }
  if (algo == glx::ALGO_RING_CHUNKED || algo == glx::ALGO_HALVING_DOUBLING ||
      algo == glx::ALGO_FN_RING || algo == glx::ALGO_FN_BCUBE) {
    const int e = stepsEngine();
    if (e >= 0) return e;
    // auto: the plan kernel for small and medium buffers
    return count * esize <= devStepsMaxBytes() ? kEngineDevSteps : kEngineSteps;
  }
  return kEngineSteps;
}

// Peers' stores land in our HBM behind our caches' back: uncached memory
// (default), or fine-grained memory (GLOO_AMD_DD_MEM=finegrained: cached
// non-coherently, the kernels' system-scope acquire drops stale lines).
char* HipPlanExecutor::ddAlloc(size_t bytes) {
  static const unsigned flags = [] {
    const char* e = std::getenv("GLOO_AMD_DD_MEM");
    return (e != nullptr && std::strcmp(e, "finegrained") == 0) ? hipDeviceMallocFinegrained
                                                                 : hipDeviceMallocUncached;
  }();
  SharedRef ref;
  char* d = allocShared(bytes, flags, &ref);
  ddRefs_.push_back(ref);
  GLX_TRACE("r%d ddAlloc %zu bytes at %p", contextRank_, bytes, (void*)d);
  ddBlocks_.push_back(d);
  GLX_HIP_CHECK(hipMemset(d, 0, bytes));
  return d;
}

void HipPlanExecutor::setupDevice() {
  if (engine_ == kEngineOneShot) {
    setupOneShot();
  } else if (engine_ == kEngineTwoShot) {
    setupTwoShot();
  } else if (engine_ == kEngineQueued) {
    setupQueued();
  } else {
    setupDevSteps();
  }
  // status int, then (as 64-bit words 1..3) the flag value seen, the value
  // awaited and the workgroup of a timed-out wait
  GLX_HIP_CHECK(hipHostMalloc((void**)&ddStatus_, 4 * sizeof(uint64_t),
                              hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(ddStatus_, 0, 4 * sizeof(uint64_t));
  GLX_HIP_CHECK(hipHostGetDevicePointer((void**)&ddStatusDev_, ddStatus_, 0));
  os_.status = ddStatusDev_;
  ts_.status = ddStatusDev_;
  pk_.status = ddStatusDev_;
  GLX_HIP_CHECK(hipMalloc((void**)&ddClaim_, sizeof(int)));
  GLX_HIP_CHECK(hipMemset(ddClaim_, 0, sizeof(int)));
  os_.claim = ddClaim_;
  ts_.claim = ddClaim_;
  pk_.claim = ddClaim_;
  const int fs = context_->flagStores() ? 1 : 0;
  os_.flagStore = fs;
  ts_.flagStore = fs;
  pk_.flagStore = fs;
  GLX_HIP_CHECK(hipEventCreateWithFlags(&ddDone_, hipEventDisableTiming));
  int khz = 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device_) == hipSuccess &&
      khz > 0) {
    clockKhz_ = khz;
  }
  GLX_HIP_CHECK(hipDeviceSynchronize());
}

// Workgroups (= slices) per launch: kOsMaxSlices, fewer if the kernel's
// resident capacity shared by the ranks on the busiest GPU is smaller (ranks
// spin on each other's workgroups, so every grid must be resident at once).
// Same inputs on every rank -> same grid.
size_t HipPlanExecutor::maxSlices(int kernel) const {
  const int cap = glx::device_engine_resident_blocks(kernel, op_, dtype_);
  const int share = context_->maxRanksPerDevice();
  size_t g = glx::kOsMaxSlices;
  if (cap > 0) g = std::min(g, (size_t)std::max(1, cap / std::max(1, share)));
  return g;
}

void HipPlanExecutor::setupOneShot() {
  const int P = contextSize_;
  const glx::DeviceLayout d =
      glx::oneShotLayout(plan_, contextRank_, P, count_, (int)esize_, (int64_t)maxSlices(0));
  glx::OneShotParams& p = os_;
  p.P = P;
  p.rank = contextRank_;
  p.count = (size_t)count_;
  p.slice = (size_t)d.slice;
  p.G = d.G;
  p.njobs = d.njobs;
  for (int q = 0; q < d.njobs; q++) {
    p.jobOff[q] = (size_t)d.jobOff[q];
    p.jobLen[q] = (size_t)d.jobLen[q];
    for (int i = 0; i < P; i++) p.chain[q][i] = (uint8_t)d.chain[q][i];
  }
  ddSlot_ = ((size_t)count_ * esize_ + 255) & ~(size_t)255;
  ddAlloc((size_t)P * ddSlot_);
  ddAlloc((size_t)P * ddSlot_);
  p.flagIn = reinterpret_cast<const uint64_t*>(
      ddAlloc((size_t)P * (size_t)p.G * glx::kFlagBytes));
}

void HipPlanExecutor::setupTwoShot() {
  const int P = contextSize_;
  const glx::DeviceLayout d =
      glx::twoShotLayout(plan_, contextRank_, P, count_, (int)esize_, (int64_t)maxSlices(1));
  glx::TwoShotParams& p = ts_;
  p.P = P;
  p.rank = contextRank_;
  p.trace = nullptr;
  for (int c = 0; c < glx::kOsMaxRanks; c++) {
    p.rangeOff[c] = (size_t)d.rangeOff[c];
    p.rangeLen[c] = (size_t)d.rangeLen[c];
    p.chain[c] = (uint8_t)d.myChain[c];
  }
  p.slice = (size_t)d.slice;
  p.G = d.G;
  if (devTrace()) {
    const size_t n = (size_t)std::max<int64_t>(1, maxSlices(1)) * glx::kTsTrace;
    GLX_HIP_CHECK(hipHostMalloc((void**)&trace_, n * sizeof(uint64_t), hipHostMallocDefault));
    std::memset(trace_, 0, n * sizeof(uint64_t));
    p.trace = trace_;
  }
  ddSlot_ = ((size_t)d.maxLen * esize_ + 16 + 255) & ~(size_t)255;
  for (int k = 0; k < 4; k++) ddAlloc((size_t)P * ddSlot_);  // RS 0/1, AG 0/1
  char* flags = ddAlloc(2 * (size_t)P * (size_t)p.G * glx::kFlagBytes);
  p.flagAIn = reinterpret_cast<const uint64_t*>(flags);
  p.flagBIn = reinterpret_cast<const uint64_t*>(flags) + (size_t)P * (size_t)p.G * glx::kFlagStride;
}

// The plan kernel: segments from every rank's program (plan.cc syncTable),
// G workgroups, flag rows [our in-channels' deliveries, then our
// out-channels' credits][G] in one uncached block.
void HipPlanExecutor::setupDevSteps() {
  GLX_ENFORCE(sync_.outChans.size() == out_.size() && sync_.inChans.size() == in_.size(),
              "plan kernel: channel tables disagree");
  const size_t G = (size_t)pk_.G;
  std::vector<glx::DevSegment> segs;
  for (size_t k = 0; k + 1 < sync_.bounds.size(); k++) {
    glx::DevSegment sg;
    sg.off = sync_.bounds[k];
    sg.len = sync_.bounds[k + 1] - sync_.bounds[k];
    sg.slice = sync_.slice;  // one slice size for every segment (SyncTable::safe)
    segs.push_back(sg);
  }
  if (segs.empty()) segs.push_back(glx::DevSegment{0, 0, (int64_t)(16 / esize_)});
  GLX_HIP_CHECK(hipMalloc((void**)&devSegs_, segs.size() * sizeof(glx::DevSegment)));
  GLX_HIP_CHECK(hipMemcpy(devSegs_, segs.data(), segs.size() * sizeof(glx::DevSegment),
                          hipMemcpyHostToDevice));
  pk_.segs = devSegs_;
  for (size_t k = 0; k < in_.size(); k++) in_[k].deliveryWord = (uint32_t)k;
  for (size_t k = 0; k < out_.size(); k++) out_[k].creditWord = (uint32_t)(in_.size() + k);
  const size_t rows = std::max<size_t>(1, in_.size() + out_.size());
  ddAlloc(rows * G * glx::kFlagBytes);
  static const int pollLoad = [] {
    const char* e = std::getenv("GLOO_AMD_FLAG_POLL");
    return (e != nullptr && std::strcmp(e, "load") == 0) ? 1 : 0;
  }();
  pk_.pollLoad = pollLoad;
  pk_.trace = nullptr;
  if (devTrace()) {
    const size_t n = G * (2 * plan_.steps.size() + 1);
    GLX_HIP_CHECK(hipHostMalloc((void**)&trace_, n * sizeof(uint64_t), hipHostMallocDefault));
    std::memset(trace_, 0, n * sizeof(uint64_t));
    pk_.trace = trace_;
  }
}

// After resolvePeers: the step table with every address the kernel needs.
void HipPlanExecutor::buildDevSteps() {
  const size_t G = (size_t)pk_.G;
  uint64_t* rows = reinterpret_cast<uint64_t*>(ddBlocks_[0]);
  // element i of a message for ptr0[off...] sits at landing + (i - off)*es
  auto vbase = [&](char* at, int64_t off) {
    return reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(at) -
                                   (uintptr_t)off * (uintptr_t)esize_);
  };
  std::vector<glx::DevStep> ds;
  std::vector<const char*> fs;
  for (size_t i = 0; i < plan_.steps.size(); i++) {
    const glx::Step& s = plan_.steps[i];
    const glx::StepSync& y = sync_.steps[i];
    glx::DevStep d{};
    d.kind = (int32_t)s.kind;
    d.peer = (int32_t)s.peer;
    d.seg0 = y.seg0;
    d.seg1 = y.seg1;
    d.seq = y.seq;
    d.perRun = y.perRun;
    d.rseq = y.rseq;
    d.rperRun = y.rperRun;
    const bool fused = slots_ == 2 && y.fuse >= 0;
    switch (s.kind) {
      case glx::SEND: {
        GLX_ENFORCE(y.chan == stepChan_[i], "plan kernel: channel numbering disagrees");
        const OutChan& oc = out_[(size_t)y.chan];
        d.dst = s.len > 0 ? vbase(landing(peerBlocks_[oc.peer], s.dst_off, s.off), s.off)
                          : nullptr;
        d.dstSlot = s.len > 0 ? (int64_t)slotBytes(blockOf(peerBlocks_[oc.peer], s.dst_off)) : 0;
        d.flag = oc.devDelivery;
        d.credit = rows + (size_t)oc.creditWord * G * glx::kFlagStride;
        if (fused) d.kind = glx::kStepNop;  // done inside step y.fuse
        break;
      }
      case glx::RECV:
      case glx::RELEASE: {
        GLX_ENFORCE(y.chan == stepChan_[i], "plan kernel: channel numbering disagrees");
        const InChan& ic = in_[(size_t)y.chan];
        d.flag = s.kind == glx::RECV ? rows + (size_t)ic.deliveryWord * G * glx::kFlagStride
                                     : ic.devCredit;
        break;
      }
      case glx::REDUCE:
      case glx::COPY: {
        d.src = vbase(landing(blocks_, s.boff, s.off), s.off);
        d.srcSlot = (int64_t)slotBytes(blockOf(blocks_, s.boff));
        if (fused) {  // and the SEND of the result: its peer, slot, flags, numbers
          const glx::Step& t = plan_.steps[(size_t)y.fuse];
          const glx::StepSync& ty = sync_.steps[(size_t)y.fuse];
          const OutChan& oc = out_[(size_t)ty.chan];
          d.kind = s.kind == glx::REDUCE ? glx::kStepReduceSend : glx::kStepCopySend;
          d.peer = (int32_t)t.peer;
          d.seq = ty.seq;
          d.perRun = ty.perRun;
          d.dst = vbase(landing(peerBlocks_[oc.peer], t.dst_off, t.off), t.off);
          d.dstSlot = (int64_t)slotBytes(blockOf(peerBlocks_[oc.peer], t.dst_off));
          d.flag = oc.devDelivery;
          d.credit = rows + (size_t)oc.creditWord * G * glx::kFlagStride;
        }
        break;
      }
      case glx::FOLD: {
        const auto& f = plan_.folds[(size_t)s.boff];
        GLX_ENFORCE(f.size() <= (size_t)glx::kOsMaxRanks, "plan kernel: fold of ", f.size(),
                    " sources");
        d.nsrc = (int32_t)f.size();
        d.left = (s.flags & glx::kFoldLeft) != 0 ? 1 : 0;
        d.srcIndex = (int64_t)fs.size();
        const bool whole = (s.flags & glx::kFoldWhole) != 0;
        for (int64_t r : f) {
          if (r < 0) {
            fs.push_back(nullptr);
          } else if (whole) {  // whole-buffer message: element i at landing(r, 0) + i*es
            fs.push_back(landing(blocks_, r, 0));
          } else {
            fs.push_back(vbase(landing(blocks_, r, s.off), s.off));
          }
        }
        break;
      }
      default:
        GLX_ENFORCE(false, "bad plan step kind ", s.kind);
    }
    ds.push_back(d);
  }
  if (fs.empty()) fs.push_back(nullptr);
  if (ds.empty()) ds.push_back(glx::DevStep{});  // never walked (nsteps = 0)
  hostSteps_ = ds;
  GLX_HIP_CHECK(hipMalloc((void**)&devSteps_, ds.size() * sizeof(glx::DevStep)));
  GLX_HIP_CHECK(hipMemcpy(devSteps_, ds.data(), ds.size() * sizeof(glx::DevStep),
                          hipMemcpyHostToDevice));
  GLX_HIP_CHECK(hipMalloc((void**)&devFoldSrc_, fs.size() * sizeof(char*)));
  GLX_HIP_CHECK(hipMemcpy(devFoldSrc_, fs.data(), fs.size() * sizeof(char*),
                          hipMemcpyHostToDevice));
  pk_.steps = devSteps_;
  pk_.foldSrc = devFoldSrc_;
  pk_.nsteps = (int)plan_.steps.size();
  pk_.slots = slots_;
}

void HipPlanExecutor::waitDevice(hipStream_t s) {
  if (engine_ == kEngineSteps || ddStatus_ == nullptr || contextSize_ == 1) {
    GLX_HIP_CHECK(spinSync(s));
    return;
  }
  const auto t0 = std::chrono::steady_clock::now();
  auto lastAlive = t0;
  for (uint64_t spin = 1;; spin++) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) {
      GLX_HIP_CHECK(e);
      return;
    }
    if ((spin & 63) == 0) {
      const auto now = std::chrono::steady_clock::now();
      if (now - lastAlive > std::chrono::milliseconds(100)) {
        lastAlive = now;
        const int dead = context_->deadPeer();
        if (dead >= 0) {
          // every kernel wait polls this word and gives up; the launch drains
          *reinterpret_cast<volatile int*>(ddStatus_) = 1 + dead;
          (void)hipStreamSynchronize(s);
          broken_ = true;
          context_->checkPeersAlive();  // throws IoException naming the rank
        }
      }
    }
    if (spin > 4096) {
      sched_yield();
    } else {
      _mm_pause();
    }
  }
}

void HipPlanExecutor::checkDevice() {
  if (engine_ == kEngineSteps) return;
  const int st = *reinterpret_cast<volatile int*>(ddStatus_);
  if (st != 0) {
    broken_ = true;
    const int peer = (st & 255) - 1, step = (st >> 8) - 1;
    std::string where;
    if (step >= 0 && (size_t)step < plan_.steps.size()) {
      const glx::Step& s = plan_.steps[(size_t)step];
      where = std::string(", ") + (s.kind == glx::SEND ? "credit for send" : "receive") +
              " step " + std::to_string(step) + " of run " + std::to_string(devRuns_ - 1);
    }
    const volatile uint64_t* d = reinterpret_cast<const volatile uint64_t*>(ddStatus_);
    // The flag words as the host reads them now (the kernel has finished):
    // ours, and the peer's through our IPC mapping of its memory.  A receiver
    // whose flag still holds the old value while its sender reads the new
    // one through its mapping would mean the two views are not one memory.
    std::string flags;
    const size_t w = (size_t)d[3];
    auto readFlag = [&](const uint64_t* row) -> std::string {
      uint64_t v = 0;
      if (row == nullptr || w >= (size_t)pk_.G) return "?";
      if (hipMemcpy(&v, row + w * glx::kFlagStride, sizeof(v), hipMemcpyDeviceToHost) !=
          hipSuccess) {
        (void)hipGetLastError();
        return "?";
      }
      return std::to_string(v);
    };
    if (engine_ == kEngineDevSteps && step >= 0 && (size_t)step < hostSteps_.size()) {
      const glx::DevStep& ds = hostSteps_[(size_t)step];
      if (ds.kind == glx::SEND) {
        flags = "; now: our credit flag " + readFlag(ds.credit) +
                ", the receiver's delivery flag through our mapping " + readFlag(ds.flag);
      } else if (ds.kind == glx::RECV) {
        flags = "; now: our delivery flag " + readFlag(ds.flag);
      }
    }
    GLX_THROW_TIMEOUT("Timed out waiting for data from rank ", peer, " (rank ", contextRank_,
                      ", device-driven allreduce", where, ": workgroup ", d[3], " saw ", d[1],
                      ", awaited ", d[2], ", timeout ", effectiveTimeout().count(), " ms",
                      flags, ")");
  }
}

bool HipPlanExecutor::devTrace() {
  static const bool on = [] {
    const char* e = std::getenv("GLOO_AMD_DEVTRACE");
    return e != nullptr && e[0] == '1';
  }();
  return on;
}

// Diagnostics (GLOO_AMD_DEVTRACE=1): wait for the launch just issued and
// print, per phase, the mean and max over workgroups of the time since the
// workgroup started (s_memrealtime), plus the grid's span.
void HipPlanExecutor::traceTwoShot(const glx::TwoShotParams& launched) {
  (void)launched;
  GLX_HIP_CHECK(hipStreamSynchronize(compute_));
  const int G = ts_.G;
  const uint64_t* t = trace_;
  const double us = 1e3 / (double)clockKhz_;
  uint64_t t0min = ~uint64_t(0), t5max = 0;
  double mean[glx::kTsTrace] = {0}, mx[glx::kTsTrace] = {0};
  for (int w = 0; w < G; w++) {
    const uint64_t* r = t + (size_t)w * glx::kTsTrace;
    t0min = std::min(t0min, r[0]);
    t5max = std::max(t5max, r[5]);
    for (int k = 1; k < glx::kTsTrace; k++) {
      const double d = r[k] >= r[0] ? (double)(r[k] - r[0]) * us : 0.0;
      mean[k] += d / G;
      mx[k] = std::max(mx[k], d);
    }
  }
  double st = 0, stmax = 0;  // start skew within the grid
  for (int w = 0; w < G; w++) {
    const double d = (double)(t[(size_t)w * glx::kTsTrace] - t0min) * us;
    st += d / G;
    stmax = std::max(stmax, d);
  }
  std::fprintf(stderr, "[devtrace r%d] resident capacity %d, ranks on the busiest device %d\n",
               contextRank_, glx::device_engine_resident_blocks(1, op_, dtype_),
               context_->maxRanksPerDevice());
  std::fprintf(stderr,
               "[devtrace r%d two-shot G=%d slice=%zu] span %.1f us | start skew mean %.1f max "
               "%.1f | since start (mean/max): pushed %.1f/%.1f  copies-in %.1f/%.1f  "
               "folded %.1f/%.1f  results-in %.1f/%.1f  end %.1f/%.1f\n",
               contextRank_, G, ts_.slice, (double)(t5max - t0min) * us, st, stmax, mean[1],
               mx[1], mean[2], mx[2], mean[3], mx[3], mean[4], mx[4], mean[5], mx[5]);
}

// Diagnostics (GLOO_AMD_DEVTRACE=1): wait for the plan kernel just launched
// and print, per step, the mean over workgroups of the time spent waiting
// (credit for a SEND, delivery for a RECV) and working, plus totals.
void HipPlanExecutor::traceDevSteps(const glx::PlanKernelParams& launched) {
  GLX_HIP_CHECK(hipStreamSynchronize(compute_));
  const int G = launched.G, n = launched.nsteps;
  const size_t row = 2 * (size_t)n + 1;
  const double us = 1e3 / (double)clockKhz_;
  static const char* kinds[] = {"SEND", "RECV", "REDUCE", "COPY", "RELEASE", "FOLD"};
  uint64_t t0 = ~uint64_t(0), t1 = 0;
  double waitTot[6] = {0}, workTot[6] = {0};
  std::string lines;
  for (int i = 0; i < n; i++) {
    double wsum = 0, ksum = 0, kmax = 0;
    for (int w = 0; w < G; w++) {
      const uint64_t* t = trace_ + (size_t)w * row;
      if (i == 0) t0 = std::min(t0, t[0]);
      if (i == n - 1) t1 = std::max(t1, t[2 * (size_t)n]);
      const uint64_t after = t[2 * i + 1] != 0 ? t[2 * i + 1] : t[2 * i];
      const double wt = (double)(after - t[2 * i]) * us;
      const double kt = (double)(t[2 * i + 2] - after) * us;
      wsum += wt / G;
      ksum += kt / G;
      kmax = std::max(kmax, kt);
    }
    const int k = plan_.steps[(size_t)i].kind;
    waitTot[k] += wsum;
    workTot[k] += ksum;
    char b[160];
    std::snprintf(b, sizeof(b), "  step %2d %-7s len %9ld  wait %8.1f  work %8.1f (max %8.1f) us\n",
                  i, kinds[k], (long)plan_.steps[(size_t)i].len, wsum, ksum, kmax);
    lines += b;
  }
  std::fprintf(stderr, "[devtrace r%d plan kernel G=%d, %d steps, run %lu] span %.1f us\n%s",
               contextRank_, G, n, (unsigned long)launched.run, (double)(t1 - t0) * us,
               lines.c_str());
  for (int k = 0; k < 6; k++) {
    if (waitTot[k] + workTot[k] > 0) {
      std::fprintf(stderr, "[devtrace r%d]   %-7s wait %9.1f us  work %9.1f us (sums of means)\n",
                   contextRank_, kinds[k], waitTot[k], workTot[k]);
    }
  }
}

void HipPlanExecutor::runDevice(char* ptr0) {
  if (!resolved_) resolvePeers();
  checkDevice();  // an earlier asynchronous call that timed out
  const int P = contextSize_;
  const uint64_t e = ++ddEpoch_;
  const int par = (int)(e & 1);
  const uint64_t ticks = (uint64_t)effectiveTimeout().count() * (uint64_t)clockKhz_;
  // epochs stay ordered even when calls come on different streams
  if (ddLaunched_) GLX_HIP_CHECK(hipStreamWaitEvent(compute_, ddDone_, 0));
  if (staged_) waitH2D(compute_, computeH2dWaited_, 0, count_);
  if (engine_ == kEngineOneShot) {
    glx::OneShotParams p = os_;
    p.buf = ptr0;
    p.epoch = e;
    p.timeoutTicks = ticks;
    for (int j = 0; j < P; j++) {
      if (j == contextRank_) {
        p.push[j] = nullptr;
        p.land[j] = ptr0;
        p.flagOut[j] = nullptr;
        continue;
      }
      const auto& pb = ddPeer_.at(j);
      p.push[j] = pb[(size_t)par] + (size_t)contextRank_ * ddSlot_;
      p.land[j] = ddBlocks_[(size_t)par] + (size_t)j * ddSlot_;
      p.flagOut[j] = reinterpret_cast<uint64_t*>(pb[2]) +
                     (size_t)contextRank_ * (size_t)p.G * glx::kFlagStride;
    }
    GLX_TRACE("r%d one-shot epoch %lu (G=%d slice=%zu)", contextRank_, (unsigned long)e, p.G,
              p.slice);
    GLX_HIP_CHECK(glx::launch_oneshot(op_, dtype_, p, compute_));
    transport_.deviceKernels++;
  } else if (engine_ == kEngineDevSteps) {
    if (devSteps_ == nullptr) buildDevSteps();
    glx::PlanKernelParams p = pk_;
    p.buf = ptr0;
    p.run = devRuns_++;
    p.timeoutTicks = ticks;
    GLX_TRACE("r%d plan kernel run %lu (G=%d, %d steps)", contextRank_, (unsigned long)p.run,
              p.G, p.nsteps);
    if (p.trace != nullptr) {
      std::memset(trace_, 0, (size_t)p.G * (2 * (size_t)p.nsteps + 1) * sizeof(uint64_t));
    }
    GLX_HIP_CHECK(glx::launch_plan_kernel(op_, dtype_, p, compute_));
    transport_.deviceKernels++;
    if (p.trace != nullptr) traceDevSteps(p);
  } else {
    glx::TwoShotParams p = ts_;
    p.buf = ptr0;
    p.epoch = e;
    p.timeoutTicks = ticks;
    const size_t G = (size_t)p.G;
    // element i of range c at vbase + i*es: the 16-byte phase of a 16-byte
    // aligned buffer (see xgmi_kernels.hip)
    auto vbase = [&](char* slot, int c) {
      const size_t off = p.rangeOff[c] * esize_;
      return slot + (off % 16) - off;
    };
    for (int j = 0; j < P; j++) {
      if (j == contextRank_) {
        p.rsPush[j] = p.agPush[j] = nullptr;
        p.rsLand[j] = p.agLand[j] = nullptr;
        p.flagAOut[j] = p.flagBOut[j] = nullptr;
        continue;
      }
      const auto& pb = ddPeer_.at(j);
      const size_t mine = (size_t)contextRank_ * ddSlot_, theirs = (size_t)j * ddSlot_;
      p.rsPush[j] = vbase(pb[(size_t)par] + mine, j);             // my copy of range j
      p.rsLand[j] = vbase(ddBlocks_[(size_t)par] + theirs, contextRank_);  // j's copy of mine
      p.agPush[j] = vbase(pb[2 + (size_t)par] + mine, contextRank_);       // my result
      p.agLand[j] = vbase(ddBlocks_[2 + (size_t)par] + theirs, j);         // j's result
      uint64_t* pf = reinterpret_cast<uint64_t*>(pb[4]);
      p.flagAOut[j] = pf + (size_t)contextRank_ * G * glx::kFlagStride;
      p.flagBOut[j] = pf + ((size_t)P * G + (size_t)contextRank_ * G) * glx::kFlagStride;
    }
    GLX_TRACE("r%d two-shot epoch %lu (G=%d slice=%zu)", contextRank_, (unsigned long)e, p.G,
              p.slice);
    GLX_HIP_CHECK(glx::launch_twoshot(op_, dtype_, p, compute_));
    transport_.deviceKernels++;
    if (devTrace()) traceTwoShot(p);
  }
  GLX_HIP_CHECK(hipEventRecord(ddDone_, compute_));
  ddLaunched_ = true;
  if (staged_) {
    GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, ddDone_, 0));
    copyBack({glx::Range{0, count_}});
  }
}

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
