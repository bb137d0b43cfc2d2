// executor.cc -- HipPlanExecutor: construction, rendezvous of scratch between
// ranks, the host-issued steps engine and run()/runFn().  The host-memory
// endpoints and device-driven engines live in executor_{host,device}.cc.  See executor.h.
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

std::atomic<int> g_copy_split{1};  // glx_set_copy_split

// Default: hipMemcpyPeerAsync (the DMA engines); glx_set_copy_engine(1, ...)
// selects the copy kernel (the sending GPU's compute units store into the
// receiver's region over xGMI).
std::atomic<int> g_copy_engine{0};

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
  pp.base = ctx->base();
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
  if ((engine_ == kEngineOneShot || engine_ == kEngineTwoShot) && count_ > 0) {
    // Their layouts read whole ranges off the plan (no split messages), and
    // each of their slot arrays holds P ranges (two-shot) or P whole buffers
    // (one-shot) in one block, which must stay shareable between processes
    // (Context::kIpcMaxBlockBytes).  Otherwise the same schedule runs as
    // host-issued steps -- from every rank's unsplit program, so all agree.
    glx::PlanParams whole = prm_;
    whole.maxMessageBytes = INT64_MAX;
    int64_t maxMsg = 0;
    for (int q = 0; q < contextSize_; q++) {
      for (const auto& s : glx::makePlan(algo, q, contextSize_, count_, whole).steps) {
        if (s.kind == glx::SEND) maxMsg = std::max(maxMsg, s.len);
      }
    }
    const size_t arr = (size_t)contextSize_ * ((size_t)maxMsg * esize_ + 512) + 4096;
    if (maxMsg * (int64_t)esize_ > prm_.maxMessageBytes ||
        (ctx->sharesAcrossProcesses() && arr >= Context::ipcMaxBlockBytes())) {
      engine_ = kEngineSteps;
    }
  }
  if (engine_ == kEngineDmaSteps) split_ = 1;  // one copy (one done word) per SEND
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
    // two landing slots per region must stay shareable (Context::
    // kIpcMaxBlockBytes): a larger region runs with one slot and no
    // reduce-and-forward, which every rank derives alike from the geometry
    if (slots_ > 1 && ctx->sharesAcrossProcesses()) {
      // from the largest region of EVERY rank's program, so all ranks agree
      const ScratchBlock whole{0, sync_.maxRegionElems, nullptr, {}};
      if ((size_t)slots_ * slotBytes(whole) + 4096 >= Context::ipcMaxBlockBytes()) slots_ = 1;
    }
    if (!sync_.safe) engine_ = kEngineSteps;
  }
  // Pipelining below chunk granularity (glx_set_pipeline_bytes): the
  // host-issued and DMA steps engines on device buffers run the program with
  // its messages cut into pieces and reduce-and-forward per piece (plan.h
  // splitMessages); every rank reaches the same engine, hence the same plan
  if ((engine_ == kEngineSteps || engine_ == kEngineDmaSteps) && !hostMode_ &&
      contextSize_ > 1 && count_ > 0 && glx::pipelineBytes() > 0) {
    prm_.pipelineBytes = glx::pipelineBytes();
    plan_ = glx::makePlan(algo, contextRank_, contextSize_, count_, prm_);
  }
  if (engine_ == kEngineOneShot || engine_ == kEngineTwoShot) {
    setupDevice();
  } else {
    // Receive regions are uncached for every engine: peers' stores (their
    // kernels' or DMA) land behind this GPU's L2, and a region is reused
    // every run, so no stale line of an earlier message may be cached.  (The
    // plan kernel reads its `slots_` landing slots inside the launch right
    // after an in-kernel flag wait, where nothing else could drop such a
    // line.)
    allocScratch(!cachedSlotsForTest(), engine_ == kEngineDevSteps ? slots_ : 1);
  }

  // Channels named by the plan; allocate our counter words.
  auto& ctl = ctx->localControl();
  stepChan_.assign(plan_.steps.size(), -1);
  const bool hostSteps = engine_ == kEngineSteps;
  const bool copyStreams = hostSteps || engine_ == kEngineDmaSteps;
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
        // device engines: no control-block words (their flag rows are
        // assigned in setupDevSteps / setupDmaSteps); the plan kernel has no
        // copy streams
        oc.creditWord = hostSteps ? ctl.allocWord() : 0;
        oc.credit = hostSteps ? ctl.word(oc.creditWord) : nullptr;
        // one copy stream per destination peer: copies to different peers
        // run concurrently on different xGMI links.  The DMA steps engine
        // gives every channel its own (its copies wait on the GPU, so the
        // ring's two channels to one peer overlap their copies' fixed
        // start-up costs instead of queueing behind each other)
        oc.stream = copyStreams ? -1 : 0;
        for (const auto& o : out_) {
          if (copyStreams && o.peer == oc.peer && engine_ != kEngineDmaSteps) oc.stream = o.stream;
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
  if (engine_ == kEngineDevSteps || engine_ == kEngineDmaSteps) setupDevice();
  events_.resize(plan_.steps.size() * (size_t)split_, nullptr);
  for (auto& e : events_) GLX_HIP_CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  GLX_HIP_CHECK(hipEventCreateWithFlags(&computeMark_, hipEventDisableTiming));
  GLX_HIP_CHECK(hipEventCreateWithFlags(&lastDone_, hipEventDisableTiming));
  if (contextSize_ > 1 && count_ > 0) publish();
}

HipPlanExecutor::~HipPlanExecutor() noexcept(false) { release(); }

void HipPlanExecutor::drainCredits() noexcept {
  if (broken_) return;  // a peer timed out or exited: nothing more will come
  // a device launch reported a timeout or an overlap that no call has
  // raised yet: its grid stopped early, so its counts will never settle
  if (deviceReported()) return;
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
    } else if (engine_ == kEngineDmaSteps) {
      // our last run's work (its copies and signals included: the compute
      // stream waits for them), then every receiver's credit for our last
      // message into our flag words
      if (hipStreamSynchronize(compute_) != hipSuccess) {
        (void)hipGetLastError();
        return;
      }
      for (auto& oc : out_) {
        for (;;) {
          uint64_t v = 0;
          if (hipMemcpy(&v, dmaWord(oc.creditWord), sizeof(v), hipMemcpyDeviceToHost) !=
              hipSuccess) {
            (void)hipGetLastError();
            break;
          }
          if (v >= oc.sent || deviceReported() || std::chrono::steady_clock::now() >= deadline) {
            break;
          }
          context_->checkPeersAlive();  // throws if a peer exited: stop waiting
          pause();
        }
      }
    } else {
      // the launches the GPU completed, graph replays on other streams
      // included: wait until every started launch finished
      const uint64_t settled = settleLaunches(deadline);
      if (engine_ != kEngineDevSteps || devRuns_ == 0 || ddBlocks_.empty()) return;
      const uint64_t runs = std::max<uint64_t>(devRuns_, settled);
      // final credit of out-channel c on every workgroup: runs * perRun
      std::vector<uint64_t> want(out_.size(), 0);
      for (size_t i = 0; i < plan_.steps.size() && i < sync_.steps.size(); i++) {
        if (plan_.steps[i].kind == glx::SEND) {
          const size_t c = (size_t)sync_.steps[i].chan;
          if (c < want.size()) want[c] = runs * sync_.steps[i].perRun;
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
  } catch (...) {
  }
}

uint64_t HipPlanExecutor::settleLaunches(std::chrono::steady_clock::time_point deadline) noexcept {
  if (launchCtr_ == nullptr) return 0;
  if (hipStreamSynchronize(compute_) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  const int G = engine_ == kEngineOneShot ? os_.G : (engine_ == kEngineTwoShot ? ts_.G : pk_.G);
  std::vector<uint64_t> ctr(glx::kLaunchStartsOffset + (size_t)G);
  for (;;) {
    if (hipMemcpy(ctr.data(), launchCtr_, ctr.size() * sizeof(uint64_t),
                  hipMemcpyDeviceToHost) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    const uint64_t done = ctr[0];
    uint64_t started = 0;  // workgroup starts, every index
    for (int w = 0; w < G; w++) started += ctr[glx::kLaunchStartsOffset + (size_t)w];
    if (started <= done * (uint64_t)G || std::chrono::steady_clock::now() >= deadline ||
        deviceReported()) {
      return done;
    }
    // a peer that exited ends the wait (this function must not throw: it
    // runs from the destructor's drain)
    if (context_->deadPeer() >= 0) return done;
    std::this_thread::sleep_for(std::chrono::microseconds(50));
  }
}

void HipPlanExecutor::reportPolls() noexcept {
  if (polls_ == nullptr) return;
  const size_t G = (size_t)pk_.G;
  std::vector<uint64_t> v(G, 0);
  uint64_t ctr = 0;
  if (hipMemcpy(v.data(), polls_, G * sizeof(uint64_t), hipMemcpyDeviceToHost) == hipSuccess &&
      (runCtr_ == nullptr ||
       hipMemcpy(&ctr, runCtr_, sizeof(ctr), hipMemcpyDeviceToHost) == hipSuccess)) {
    uint64_t sum = 0, mx = 0;
    for (uint64_t x : v) {
      sum += x;
      mx = std::max(mx, x);
    }
    std::fprintf(stderr,
                 "[polls r%d] plan kernel G=%zu steps=%zu launches=%lu flag_reads=%lu "
                 "per_launch=%.1f max_per_workgroup=%lu\n",
                 contextRank_, G, plan_.steps.size(), (unsigned long)ctr, (unsigned long)sum,
                 ctr > 0 ? (double)sum / (double)ctr : 0.0, (unsigned long)mx);
  }
  (void)hipGetLastError();
  hipFree(polls_);
  polls_ = nullptr;
}

void HipPlanExecutor::release() noexcept {
  if (device_ < 0) return;  // nothing was acquired
  hipSetDevice(device_);
  // DMA steps engine after a failed run: flag waits of it may still be queued
  // for messages that will never come; stop them at once
  if (engine_ == kEngineDmaSteps && broken_ && ddStatus_ != nullptr &&
      *reinterpret_cast<volatile int*>(ddStatus_) == 0) {
    *reinterpret_cast<volatile int*>(ddStatus_) = 1 + contextRank_;
  }
  drainCredits();
  reportPolls();
  // the last call's work may sit on a caller's stream (runFn with a stream):
  // it reads our scratch until it completes
  if (lastDone_ != nullptr && lastStream_ != nullptr) hipEventSynchronize(lastDone_);
  if (ddDone_ != nullptr && fnCalls_) hipEventSynchronize(ddDone_);
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
  for (char* d : devBufs_) {
    GLX_TRACE_MEM("r%d hipFree devBuf %p", contextRank_, (void*)d);
    hipFree(d);
  }
  givePinned(hostStage_, hostStageBytes_);
  hostStage_ = nullptr;
  for (char* d : fnStage_) hipFree(d);
  for (PinnedBlock& m : ptrMirror_) givePinned(m.p, m.bytes);
  ptrMirror_.clear();
  for (PinnedBlock& m : callMirror_) givePinned(m.p, m.bytes);
  for (PinnedBlock& m : fnMirror_) givePinned(m.p, m.bytes);
  fnMirror_.clear();
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
  putPod<int64_t>(b, prm_.maxMessageBytes);  // how this rank's program cut its messages
  putPod<int64_t>(b, prm_.pipelineBytes);
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
  getPod<int64_t>(rec, at);  // max message bytes
  getPod<int64_t>(rec, at);  // pipeline bytes
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
  std::map<int, uint64_t*> abortWords;  // DMA steps engine: peer -> its abort word
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
                " (GLOO_AMD_FUSE must be the same on every rank; two slots are kept only "
                "while two of the largest region stay below the 2 GiB IPC block limit)");
    const int64_t peerMaxMsg = getPod<int64_t>(b, at);
    const int64_t peerPipe = getPod<int64_t>(b, at);
    GLX_ENFORCE(peerPipe == prm_.pipelineBytes, "rank ", r, " pipelines in pieces of ",
                peerPipe, " bytes, rank ", contextRank_, " in ", prm_.pipelineBytes,
                " (glx_set_pipeline_bytes must be the same on every rank)");
    GLX_ENFORCE(peerMaxMsg == prm_.maxMessageBytes, "rank ", r, " cuts messages above ",
                peerMaxMsg, " bytes, rank ", contextRank_, " above ", prm_.maxMessageBytes,
                " (glx_set_max_message_bytes must be the same on every rank)");
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
    if (engine_ == kEngineDevSteps || engine_ == kEngineDmaSteps) {  // the peer's flag rows
      GLX_ENFORCE(!blocks.empty(), "rank ", r, " published no flag rows");
      uint64_t* rows = reinterpret_cast<uint64_t*>(blocks[0]);
      const size_t G = engine_ == kEngineDevSteps ? (size_t)pk_.G : 1;  // DMA steps: one word
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
      if (engine_ == kEngineDmaSteps) abortWords[r] = rows;  // word 0: its abort word
    }
  }
  if (engine_ == kEngineDmaSteps) {
    // every peer's abort word; with more peers than a flag kernel carries,
    // those our copies land in (the ones a stray copy could overwrite)
    dmaAbortOut_.clear();
    for (const auto& kv : abortWords) {
      bool out = false;
      for (const auto& oc : out_) out = out || oc.peer == kv.first;
      if (abortWords.size() <= (size_t)glx::kFlagAbortMax || out) {
        dmaAbortOut_.push_back(kv.second);
      }
    }
    GLX_ENFORCE(dmaAbortOut_.size() <= (size_t)glx::kFlagAbortMax, "DMA steps engine: ",
                dmaAbortOut_.size(), " receiving peers (at most ", glx::kFlagAbortMax, ")");
  }
  const bool dev = engine_ == kEngineDevSteps || engine_ == kEngineDmaSteps;
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

// The largest receive region of the plan (elements): RECV steps land at
// their region's start, regions run to the next start (allocScratch).

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
  // Only what messages land in gets memory: a region runs from a RECV's
  // landing start to the next start, but no further than its longest
  // message plus the landing pad -- a layout slot no message lands in (a mesh
  // rank's own range) gets none (at 2 GiB it crossed the IPC limit).
  // Consecutive regions share a block up to kMaxBlockBytes.
  ScratchBlock cur;
  cur.start = 0;
  for (size_t i = 0; i + 1 < starts.size(); i++) {
    const int64_t regionElems = glx::landedRegionElems(plan_, starts[i], starts[i + 1]);
    if (regionElems == 0) continue;  // nothing lands here
    const size_t curBytes = (size_t)cur.elems * esize_;
    if (cur.elems > 0 && (cur.start + cur.elems != starts[i] ||
                          curBytes + (size_t)regionElems * esize_ > kMaxBlockBytes)) {
      blocks_.push_back(cur);
      cur = ScratchBlock();
    }
    if (cur.elems == 0) cur.start = starts[i];
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
  if (engine_ == kEngineSteps || staged_ || ptrs_.size() > 1 || sideOut_ != nullptr ||
      contextSize_ == 1) {
    noteDone(compute_);
  } else {
    // nothing follows the device launch on compute_, which is this
    // algorithm's stream for its life: release() synchronizes it, and an
    // event record here would cost every call several microseconds
    lastStream_ = compute_;
  }
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
  if (!fnCalls_ && ddLaunched_) {  // run() launches recorded no done event
    GLX_HIP_CHECK(hipEventRecord(ddDone_, ddLastStream_));
    transport_.doneEvents++;
  }
  fnCalls_ = true;
  if (call.stream != nullptr) compute_ = call.stream;
  timeout_ = call.timeout;
  localReduce(call.in, call.out);
  char* out0 = static_cast<char*>(call.out[0]);
  if (contextSize_ > 1) exchange(out0);  // :129-146
  for (size_t i = 1; i < call.out.size(); i++) {  // broadcastOutputs
    GLX_HIP_CHECK(hipMemcpyAsync(call.out[i], out0, (size_t)count_ * esize_,
                                 hipMemcpyDeviceToDevice, compute_));
  }
  if (engine_ == kEngineSteps || staged_ || call.out.size() > 1 || contextSize_ == 1) {
    noteDone(compute_);
  } else {
    lastStream_ = compute_;  // the launch's ddDone_ is the last thing on it
  }
  if (call.stream == nullptr) {
    waitDevice(compute_);
    checkDevice();
  }
}

void HipPlanExecutor::noteDone(hipStream_t s) {
  GLX_HIP_CHECK(hipEventRecord(lastDone_, s));
  transport_.doneEvents++;
  lastStream_ = s;
}

void HipPlanExecutor::recordDone(hipEvent_t ev) {
  GLX_HIP_CHECK(hipSetDevice(device_));
  GLX_HIP_CHECK(hipEventRecord(ev, lastStream_ != nullptr ? lastStream_ : compute_));
}

void HipPlanExecutor::issueCopy(char* dst, const char* src, size_t len, OutChan& oc,
                                hipStream_t s) {
  hipError_t ce = hipErrorUnknown;
  if (copyEngine_ == kCopyKernel) {
    ce = glx::launch_copy(dst, src, len, s);
    GLX_HIP_CHECK(ce);
    transport_.kernelCopies++;
  } else if (peerCopyOk_ && oc.peerDevice >= 0 && oc.peerDevice != device_) {
    ce = hipMemcpyPeerAsync(dst, oc.peerDevice, src, device_, len, s);
    if (ce == hipSuccess) {
      transport_.peerCopies++;
    } else {
      (void)hipGetLastError();
      // e.g. an IPC mapping the peer API rejects: the copy still crosses
      // xGMI (the destination is the peer's memory), now as a plain device
      // copy; say so once and count every one
      peerCopyOk_ = false;
      std::fprintf(stderr,
                   "[gloo_amd] rank %d: hipMemcpyPeerAsync to device %d refused "
                   "(%s: %s); peer copies of this algorithm use hipMemcpyAsync\n",
                   contextRank_, oc.peerDevice, hipGetErrorName(ce), hipGetErrorString(ce));
    }
  }
  if (ce != hipSuccess) {
    GLX_HIP_CHECK(hipMemcpyAsync(dst, src, len, hipMemcpyDeviceToDevice, s));
    transport_.deviceCopies++;
  }
  transport_.bytes += (int64_t)len;
}

void HipPlanExecutor::setupDmaSteps() {
  // word 0: the abort word (kernels.h abort marks), at the same place on every rank
  for (size_t k = 0; k < in_.size(); k++) in_[k].deliveryWord = (uint32_t)(1 + k);
  for (size_t k = 0; k < out_.size(); k++) out_[k].creditWord = (uint32_t)(1 + in_.size() + k);
  markWord_ = (uint32_t)(1 + in_.size() + out_.size());
  for (size_t j = 0; j < copies_.size(); j++) copies_[j].doneWord = markWord_ + 1 + (uint32_t)j;
  ddAlloc(((size_t)markWord_ + 1 + copies_.size()) * glx::kFlagBytes);
}

void HipPlanExecutor::dmaOp(hipStream_t s, int32_t kind, uint64_t* word, uint64_t value,
                            int32_t code) {
  if (!dmaOps_.empty() && (dmaOpsStream_ != s || dmaOps_.size() == (size_t)glx::kFlagOpsMax)) {
    dmaFlush();
  }
  dmaOpsStream_ = s;
  dmaOps_.push_back(glx::FlagOp{word, value, kind, code});
}

void HipPlanExecutor::dmaFlush() {
  if (dmaOps_.empty()) return;
  glx::FlagOpsParams p{};
  for (size_t k = 0; k < dmaOps_.size(); k++) p.ops[k] = dmaOps_[k];
  p.n = (int)dmaOps_.size();
  p.flagStore = context_->flagStores() ? 1 : 0;
  p.timeoutTicks = dmaTicks_;
  p.status = ddStatusDev_;
  p.claim = ddClaim_;
  p.abortIn = dmaWord(0);
  p.nAbort = (int)dmaAbortOut_.size();
  for (size_t k = 0; k < dmaAbortOut_.size(); k++) p.abortOut[k] = dmaAbortOut_[k];
  p.abortValue = 1 + (uint64_t)contextRank_;
  dmaOps_.clear();
  GLX_HIP_CHECK(glx::launch_flag_ops(p, dmaOpsStream_));
  transport_.flagKernels++;
}

// exchange() with its hand-offs on the GPU (executor.h, DMA steps engine).
// Each wait of the host-issued steps becomes a flag wait on the stream whose
// next work needs it, each counter the host would bump a flag signal on the
// stream whose work it announces:
//   SEND     copy stream: wait for the compute mark (the chunk's producer)
//            and for the receiver's credit of the previous message; the copy;
//            signal the receiver's delivery word and our done word
//   RECV     compute stream: wait for our delivery word
//   REDUCE / FOLD / COPY  compute stream: wait for the done words of sends
//            still reading the range it overwrites; the launch
//   RELEASE  compute stream: signal the sender's credit word
// Consecutive ops of one stream go out as one kernel, before anything else
// is enqueued (dmaOp / dmaFlush), so the rank enqueues everything in program
// order; at the end the compute stream also waits for every copy.  Each
// stream runs in program order and every wait is for an earlier step of this
// rank or for a peer's signal the host-issued steps wait for at the same
// point, so this engine cannot deadlock where those cannot (they, with copies
// that complete at once, are the program run in order); streams that share a
// hardware queue -- with each other or with the staging streams -- merely run
// closer to that order.  (A first version queued a copy's signals until that
// stream's next copy: in a hardware queue shared with the compute stream they
// then sat behind a later wait whose peer waited for them -- a cycle the
// staged host-buffer runs hit, tests/mp_worker.py dmasteps.)
void HipPlanExecutor::exchangeDma(char* ptr0) {
  // the message numbers are the host's: a captured run would replay stale
  // ones (checked first: resolving the peers makes synchronous copies)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  GLX_HIP_CHECK(hipStreamIsCapturing(compute_, &cap));
  GLX_ENFORCE(cap == hipStreamCaptureStatusNone,
              "the DMA steps engine cannot be captured into a HIP graph (its message numbers "
              "are counted on the host); capture an algorithm on a one-kernel engine");
  // a failure part way leaves peers waiting for messages this run will never
  // send: the algorithm is unusable, and release() stops its queued waits
  struct Broken {
    HipPlanExecutor* e;
    bool done = false;
    ~Broken() {
      if (!done) e->broken_ = true;
    }
  } broken{this};
  if (!resolved_) resolvePeers();
  checkDevice();  // an earlier asynchronous call that timed out
  dmaTicks_ = (uint64_t)effectiveTimeout().count() * (uint64_t)clockKhz_;
  // calls on different streams (function style) stay in call order
  if (ddLaunched_ && ddLastStream_ != compute_) {
    GLX_HIP_CHECK(hipStreamWaitEvent(compute_, ddDone_, 0));
  }
  auto code = [](int peer, size_t step) { return (int32_t)(1 + peer + 256 * (1 + (int)step)); };
  const int self = contextRank_;
  bool computeSinceMark = true;  // the caller's writes to ptr0 count as compute
  auto waitSends = [&](int64_t off, int64_t len, size_t step) {
    for (size_t k = 0; k < inflight_.size();) {
      const InflightSend& f = inflight_[k];
      if (f.off < off + len && off < f.off + f.len) {
        dmaOp(compute_, glx::kFlagWait, dmaWord(copies_[(size_t)f.stream].doneWord), f.done,
              code(self, step));
        inflight_.erase(inflight_.begin() + (long)k);
      } else {
        k++;
      }
    }
  };
  auto finalValues = [&](size_t step) {  // host mode: copy the step's final ranges back
    if (staged_ && !stage_.d2h[step].empty()) {
      dmaFlush();
      GLX_HIP_CHECK(hipEventRecord(d2hEvents_[step], compute_));
      GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, d2hEvents_[step], 0));
      copyBack(stage_.d2h[step]);
    }
  };
  auto h2d = [&](hipStream_t st, int& waited, int64_t off, int64_t len) {
    dmaFlush();  // (a fed run may block here until the range is fed)
    waitH2D(st, waited, off, len);
  };
  const auto& steps = plan_.steps;
  for (size_t i = 0; i < steps.size(); i++) {
    const glx::Step& s = steps[i];
    switch (s.kind) {
      case glx::SEND: {
        OutChan& oc = out_[stepChan_[i]];
        const uint64_t n = ++oc.sent;
        CopyStream& cs = copies_[(size_t)oc.stream];
        if (computeSinceMark) {  // the chunk may have been produced by compute work
          dmaOp(compute_, glx::kFlagSignal, dmaWord(markWord_), ++marks_);
          computeSinceMark = false;
        }
        if (cs.waitedMark != marks_) {
          dmaOp(cs.s, glx::kFlagWait, dmaWord(markWord_), marks_, code(self, i));
          cs.waitedMark = marks_;
        }
        // one receive region per channel: message n lands once the receiver
        // has consumed message n - 1
        if (n > 1) {
          dmaOp(cs.s, glx::kFlagWait, dmaWord(oc.creditWord), n - 1, code(oc.peer, i));
        }
        if (staged_) h2d(cs.s, cs.h2dWaited, s.off, s.len);
        dmaFlush();
        const size_t nbytes = (size_t)s.len * esize_;
        if (nbytes > 0) {
          issueCopy(landing(peerBlocks_[oc.peer], s.dst_off, s.off, s.len),
                    ptr0 + (size_t)s.off * esize_, nbytes, oc, cs.s);
        }
        // (the runtime's hipStreamWriteValue64 in place of these two signals:
        // two blit kernels, 0.79 instead of 0.83 ms for the 256 MiB ring at
        // P = 2 on one GPU -- not worth a beta API)
        dmaOp(cs.s, glx::kFlagSignal, oc.devDelivery, n);
        dmaOp(cs.s, glx::kFlagSignal, dmaWord(cs.doneWord), ++cs.copies);
        InflightSend f{s.off, s.len, nullptr};
        f.stream = oc.stream;
        f.done = cs.copies;
        inflight_.push_back(f);
        break;
      }
      case glx::RECV: {
        InChan& ic = in_[stepChan_[i]];
        dmaOp(compute_, glx::kFlagWait, dmaWord(ic.deliveryWord), ++ic.received,
              code(ic.peer, i));
        break;
      }
      case glx::REDUCE:
      case glx::COPY: {
        waitSends(s.off, s.len, i);
        if (staged_) h2d(compute_, computeH2dWaited_, s.off, s.len);
        dmaFlush();
        char* dst = ptr0 + (size_t)s.off * esize_;
        const char* src = landing(blocks_, s.boff, s.off, s.len);
        if (s.kind == glx::REDUCE) {
          GLX_HIP_CHECK(
              glx::launch_reduce(op_, dtype_, dst, dst, src, (size_t)s.len, compute_));
        } else {  // the landing region is uncached: our copy kernel (exchange())
          GLX_HIP_CHECK(glx::launch_copy(dst, src, (size_t)s.len * esize_, compute_));
        }
        computeSinceMark = true;
        finalValues(i);
        break;
      }
      case glx::FOLD: {
        size_t last = i;  // consecutive FOLDs of one kind: one batched launch
        while (last + 1 < steps.size() && steps[last + 1].kind == glx::FOLD &&
               steps[last + 1].flags == s.flags) {
          last++;
        }
        const bool rev = (s.flags & glx::kFoldLeft) == 0;
        const bool whole = (s.flags & glx::kFoldWhole) != 0;
        std::vector<glx::FoldSpec> specs;
        for (size_t q = i; q <= last; q++) {
          const glx::Step& f = steps[q];
          waitSends(f.off, f.len, q);
          if (staged_) h2d(compute_, computeH2dWaited_, f.off, f.len);
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
        dmaFlush();
        if (specs.size() == 1) {
          const glx::FoldSpec& f = specs[0];
          GLX_HIP_CHECK(
              glx::launch_reduce_n(op_, dtype_, f.dst, f.srcs.data(), f.k, f.n, compute_, rev));
        } else {
          GLX_HIP_CHECK(glx::launch_reduce_n_batch(op_, dtype_, specs, compute_, rev));
        }
        computeSinceMark = true;
        for (size_t q = i; q <= last; q++) finalValues(q);
        i = last;
        break;
      }
      case glx::RELEASE: {
        InChan& ic = in_[stepChan_[i]];
        dmaOp(compute_, glx::kFlagSignal, ic.devCredit, ++ic.consumed);
        break;
      }
      default:
        GLX_ENFORCE(false, "bad plan step kind ", s.kind);
    }
  }
  // the caller's stream must not run ahead of copies still reading ptr0
  for (auto& cs : copies_) {
    if (cs.copies > 0) {
      dmaOp(compute_, glx::kFlagWait, dmaWord(cs.doneWord), cs.copies, code(self, steps.size()));
    }
  }
  dmaFlush();
  inflight_.clear();
  if (staged_ || fnCalls_) {  // for a later call on another stream
    GLX_HIP_CHECK(hipEventRecord(ddDone_, compute_));
    transport_.doneEvents++;
  }
  ddLaunched_ = true;
  ddLastStream_ = compute_;
  broken.done = true;
}

void HipPlanExecutor::exchange(char* ptr0) {
  if (engine_ == kEngineDmaSteps) {
    exchangeDma(ptr0);
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
            issueCopy(dst + at, src + at, len, oc, cs.s);
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

}  // namespace gloo
