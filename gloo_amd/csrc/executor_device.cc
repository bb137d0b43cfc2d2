// executor_device.cc -- the device-driven engines of HipPlanExecutor (one-shot,
// two-shot, plan kernel; kernels in xgmi_kernels.hip).  See executor.h.
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
// Device-driven engines (xgmi_kernels.hip)
// ---------------------------------------------------------------------------

namespace {

// Process-wide engine choices (glx_set_mesh_engine / glx_set_steps_engine;
// no environment overrides: every rank's process must choose alike).
std::atomic<int> g_mesh_engine{HipPlanExecutor::kEngineTwoShot};

// -1 = by size (the plan kernel up to kDevStepsMaxBytes per rank when ranks
// share a GPU, where its per-step flag round trips beat host-issued steps;
// host-issued steps with their wide copy and reduce launches above), else a
// fixed engine.
std::atomic<int> g_steps_engine{-1};

constexpr int64_t kDevStepsMaxBytes = int64_t(32) << 20;

}  // namespace

void HipPlanExecutor::setMeshEngine(int engine) {
  g_mesh_engine.store(engine == kEngineSteps ? engine : kEngineTwoShot);
}

int HipPlanExecutor::meshEngine() { return g_mesh_engine.load(); }

void HipPlanExecutor::setStepsEngine(int engine) {
  g_steps_engine.store(engine < 0 ? -1
                                  : (engine == kEngineSteps || engine == kEngineDmaSteps
                                         ? engine
                                         : kEngineDevSteps));
}

int HipPlanExecutor::stepsEngine() { return g_steps_engine.load(); }

namespace {
// -1 auto (default: fast for the ring's programs), 0 plain, 1 fast.
// GLOO_AMD_ENGINE_STREAMS=fast|plain|auto.
std::atomic<int> g_engine_streams{[] {
  const char* e = std::getenv("GLOO_AMD_ENGINE_STREAMS");
  if (e != nullptr && std::strcmp(e, "fast") == 0) return 1;
  if (e != nullptr && std::strcmp(e, "plain") == 0) return 0;
  return -1;
}()};
}  // namespace

namespace {
// -1 auto, 0 system-scope release / acquire around the device engines' flags,
// 1 narrow, 2-4 the test-only broken modes (kernels.h kSync*).
// GLOO_AMD_SYNC=system|narrow|unsafe_noacquire|unsafe_norelease|unsafe_test.
std::atomic<int> g_device_sync{[] {
  const char* e = std::getenv("GLOO_AMD_SYNC");
  if (e == nullptr) return -1;
  if (std::strcmp(e, "narrow") == 0) return glx::kSyncNarrow;
  if (std::strcmp(e, "system") == 0) return glx::kSyncSystem;
  if (std::strcmp(e, "unsafe_noacquire") == 0) return glx::kSyncNoAcquire;
  if (std::strcmp(e, "unsafe_norelease") == 0) return glx::kSyncNoRelease;
  if (std::strcmp(e, "unsafe_test") == 0) return glx::kSyncUnsafe;
  if (std::strcmp(e, "unsafe_cached") == 0) return glx::kSyncCachedSlots;
  return -1;
}()};
}  // namespace

void HipPlanExecutor::setDeviceSync(int mode) {
  g_device_sync.store(mode < 0 || mode > glx::kSyncCachedSlots ? -1 : mode);
}

bool HipPlanExecutor::cachedSlotsForTest() {
  return g_device_sync.load() == glx::kSyncCachedSlots;
}

int HipPlanExecutor::deviceSync() { return g_device_sync.load(); }

void HipPlanExecutor::setEngineStreams(int fast) {
  g_engine_streams.store(fast < 0 ? -1 : (fast != 0 ? 1 : 0));
}

int HipPlanExecutor::engineStreams() { return g_engine_streams.load(); }

namespace {

// glx_set_device_engines; GLOO_AMD_DEVICE_ENGINES=auto|off|on|shared
std::atomic<int> g_device_engines{[] {
  const char* e = std::getenv("GLOO_AMD_DEVICE_ENGINES");
  if (e != nullptr && std::strcmp(e, "off") == 0) return HipPlanExecutor::kDevEnginesOff;
  if (e != nullptr && std::strcmp(e, "on") == 0) return HipPlanExecutor::kDevEnginesOn;
  if (e != nullptr && std::strcmp(e, "shared") == 0) return HipPlanExecutor::kDevEnginesShared;
  return HipPlanExecutor::kDevEnginesAuto;
}()};

}  // namespace

void HipPlanExecutor::setDeviceEngines(int mode) {
  g_device_engines.store(mode < kDevEnginesAuto || mode > kDevEnginesShared ? kDevEnginesAuto
                                                                            : mode);
}

int HipPlanExecutor::deviceEngines() { return g_device_engines.load(); }

// Hardware queues one process opens (HIP's GPU_MAX_HW_QUEUES, default 4).
int HipPlanExecutor::hwQueuesPerProcess() { return hwQueuesOfProcess(); }

bool HipPlanExecutor::deviceEnginesRule(int mode, int size, int ranksPerDevice,
                                        bool threadsShareDevice, int maxQueues) {
  if (size < 2 || size > glx::kOsMaxRanks) return false;
  if (mode == kDevEnginesOff) return false;
  if (mode == kDevEnginesOn) return true;
  // The device engines' kernels wait on each other, so every rank's kernel
  // must be running at once.  One rank per GPU: always.
  if (ranksPerDevice <= 1) return true;
  // Ranks sharing a GPU: not by default (executor.h: work queued ahead of a
  // rank's collective can be starved by its peers' spinning grids).
  if (mode != kDevEnginesShared) return false;
  // Threads of one process sharing a GPU: never (their launches may
  // serialise).  Processes sharing a GPU: only while all their hardware
  // queues fit what the GPU's scheduler maps at once; beyond that it
  // time-slices the queues and every dependent step waits for a rotation
  // (8 processes x 4 queues on one MI355X: ~170 ms per 1-element allreduce,
  // 8 x 2: ~60 ms, 8 x 1 and 4 x 4: < 1 ms; DESIGN.md 9, profiles/r7e_*,
  // r7g_queue_sweep.txt).
  if (threadsShareDevice) return false;
  // each process: its hardware queues plus an allowance of one (the
  // measurements need it; 8 x 2 time-slices although 4 x 4 does not).  The
  // largest queue count any rank published, so ranks launched with
  // different GPU_MAX_HW_QUEUES still choose alike.
  return ranksPerDevice * (std::max(1, maxQueues) + 1) <= kSharedQueueBudget;
}

bool HipPlanExecutor::deviceEnginesAvailable(const Context& ctx) {
  return deviceEnginesRule(g_device_engines.load(), ctx.size, ctx.maxRanksPerDevice(),
                           ctx.ranksShareDevice(), ctx.maxHwQueues());
}

bool HipPlanExecutor::dmaStepsAvailable(const Context& ctx) {
  return ctx.size >= 2 && g_device_engines.load() != kDevEnginesOff && !ctx.ranksShareDevice();
}

// The inputs are the same on every rank, so every rank makes the same choice
// (and publish/resolve checks that they did).
int HipPlanExecutor::engineFor(const Context& ctx, int algo, int64_t count, int esize) {
  const bool stepsAlgo = algo == glx::ALGO_RING_CHUNKED || algo == glx::ALGO_HALVING_DOUBLING ||
                         algo == glx::ALGO_FN_RING || algo == glx::ALGO_FN_BCUBE ||
                         algo == glx::ALGO_RING || algo == glx::ALGO_BCUBE;
  // the DMA steps engine only when asked for (glx_set_steps_engine)
  if (count > 0 && stepsAlgo && stepsEngine() == kEngineDmaSteps) {
    return dmaStepsAvailable(ctx) ? kEngineDmaSteps : kEngineSteps;
  }
  if (count <= 0 || !deviceEnginesAvailable(ctx)) return kEngineSteps;
  if (algo == glx::ALGO_RING_CHUNKED_REPL || algo == glx::ALGO_FN_RING_REPL) {
    return kEngineOneShot;
  }
  if (algo == glx::ALGO_RING_CHUNKED_MESH || algo == glx::ALGO_FN_RING_MESH) {
    return meshEngine();
  }
  if (algo == glx::ALGO_RING_CHUNKED || algo == glx::ALGO_HALVING_DOUBLING ||
      algo == glx::ALGO_FN_RING || algo == glx::ALGO_FN_BCUBE || algo == glx::ALGO_RING ||
      algo == glx::ALGO_BCUBE) {
    const int e = stepsEngine();
    if (e >= 0) return e;
    // auto: the plan kernel, at every size when every rank has a GPU of its
    // own (it takes the host's round trip out of each of the ring's 4P-4
    // dependent hops); with ranks sharing a GPU (rehearsals)
    // only up to kDevStepsMaxBytes, where it was measured faster there.
    // Every rank sees every endpoint, so all choose alike.
    if (ctx.maxRanksPerDevice() == 1) return kEngineDevSteps;
    return count * esize <= kDevStepsMaxBytes ? kEngineDevSteps : kEngineSteps;
  }
  return kEngineSteps;
}

// Peers' stores land in our HBM behind our caches' back: uncached memory,
// which no L2 holds -- the narrow flag sync relies on it (kernels.h).
char* HipPlanExecutor::ddAlloc(size_t bytes, bool slots) {
  SharedRef ref;
  if (slots && cachedSlotsForTest()) cachedSlots_ = true;
  char* d = allocShared(bytes, slots && cachedSlots_ ? 0u : hipDeviceMallocUncached, &ref);
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
  } else if (engine_ == kEngineDmaSteps) {
    setupDmaSteps();
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
  // The plan kernel's streams (setEngineStreams): nontemporal loads and
  // write-through stores, or plain.  The one-shot and two-shot kernels are
  // always plain.
  // release / acquire around the flags (kernels.h): automatic = kAutoNarrow
  int sync = deviceSync();
  if (sync == glx::kSyncCachedSlots) {
    cachedSlots_ = true;  // allocScratch / ddAlloc took cached slots; narrow kernels
    sync = glx::kSyncNarrow;
    std::fprintf(stderr,
                 "[gloo_amd] rank %d: TEST-ONLY cached landing slots (GLOO_AMD_SYNC="
                 "unsafe_cached): results may be stale\n",
                 contextRank_);
  }
  const int narrow = sync < 0 ? (kAutoNarrow ? glx::kSyncNarrow : glx::kSyncSystem) : sync;
  if (narrow >= glx::kSyncNoAcquire) {
    std::fprintf(stderr,
                 "[gloo_amd] rank %d: TEST-ONLY broken flag sync %d (GLOO_AMD_SYNC=unsafe_*): "
                 "results may be stale\n",
                 contextRank_, narrow);
  }
  os_.narrow = narrow;
  ts_.narrow = narrow;
  pk_.narrow = narrow;
  // the plan kernel's stream policy, automatic: write-through only where a
  // system-scope release would otherwise write back the ring's freshly
  // reduced lines; with the narrow release nothing is written back and plain
  // stores measured faster
  const int pol = engineStreams();
  const bool ring = algo_ == glx::ALGO_RING_CHUNKED || algo_ == glx::ALGO_FN_RING;
  pk_.fast = (pol > 0 || (pol < 0 && ring && !narrow)) ? 1 : 0;
  if (narrow == glx::kSyncUnsafe) pk_.fast = 0;  // its build has plain streams only
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
//
// When several ranks share a GPU (the one-GPU rehearsals and tests) their
// grids together would fill exactly the occupancy the runtime reports, and
// every workgroup of every grid must be resident at once: if the dispatcher
// packs the CUs even slightly unevenly (waves of a workgroup sharing a SIMD,
// another kernel briefly holding a slot) a workgroup waits for a slot that
// only a spinning workgroup could free -- a deadlock that ends at the
// timeout.  So shared GPUs keep a quarter of the reported capacity free.
size_t HipPlanExecutor::maxSlices(int kernel) const {
  const int cap = glx::device_engine_resident_blocks(kernel, op_, dtype_);
  const int share = std::max(1, context_->maxRanksPerDevice());
  size_t g = glx::kOsMaxSlices;
  if (cap > 0) {
    const int usable = share > 1 ? cap * 3 / 4 : cap;
    g = std::min(g, (size_t)std::max(1, usable / share));
  }
  return g;
}

// A workgroup's span of one segment: its stores into a peer's slot go through
// a write-through buffer resource with 32-bit offsets (xgmi_kernels.hip
// VecOut), so the span must stay below kWtMaxStream.  Spans are
// slice elements; a slice over 2 GiB would need a buffer over 1 TiB per rank.
void HipPlanExecutor::enforceSpan(size_t sliceElems) const {
  GLX_ENFORCE(sliceElems * esize_ <= glx::kWtMaxStream, "device engine: a workgroup span of ",
              sliceElems * esize_, " bytes exceeds the write-through stores' 2 GiB offsets");
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
  enforceSpan((size_t)d.slice);
  for (int q = 0; q < d.njobs; q++) {
    p.jobOff[q] = (size_t)d.jobOff[q];
    p.jobLen[q] = (size_t)d.jobLen[q];
    for (int i = 0; i < P; i++) p.chain[q][i] = (uint8_t)d.chain[q][i];
  }
  ddSlot_ = ((size_t)count_ * esize_ + 255) & ~(size_t)255;
  ddAlloc((size_t)P * ddSlot_, true);
  ddAlloc((size_t)P * ddSlot_, true);
  // the flag rows, then the launch counters on lines of their own (kernels.h)
  const size_t rows = (size_t)P * (size_t)p.G * glx::kFlagBytes;
  char* flags = ddAlloc(rows + glx::launchCtrBytes(p.G));
  p.flagIn = reinterpret_cast<const uint64_t*>(flags);
  p.epochCtr = reinterpret_cast<uint64_t*>(flags + rows);
  launchCtr_ = p.epochCtr;
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
  enforceSpan((size_t)d.slice);
  if (devTrace()) {
    const size_t n = (size_t)std::max<int64_t>(1, maxSlices(1)) * glx::kTsTrace;
    GLX_HIP_CHECK(hipHostMalloc((void**)&trace_, n * sizeof(uint64_t), hipHostMallocDefault));
    std::memset(trace_, 0, n * sizeof(uint64_t));
    p.trace = trace_;
  }
  ddSlot_ = ((size_t)d.maxLen * esize_ + 16 + 255) & ~(size_t)255;
  for (int k = 0; k < 4; k++) ddAlloc((size_t)P * ddSlot_, true);  // RS 0/1, AG 0/1
  // the A and B flag rows, then the launch counters on lines of their own
  const size_t rows = 2 * (size_t)P * (size_t)p.G * glx::kFlagBytes;
  char* flags = ddAlloc(rows + glx::launchCtrBytes(p.G));
  p.flagAIn = reinterpret_cast<const uint64_t*>(flags);
  p.flagBIn = reinterpret_cast<const uint64_t*>(flags) + (size_t)P * (size_t)p.G * glx::kFlagStride;
  p.epochCtr = reinterpret_cast<uint64_t*>(flags + rows);
  launchCtr_ = p.epochCtr;
}

// The plan kernel: segments from every rank's program (plan.cc syncTable),
// G workgroups, flag rows [our in-channels' deliveries, then our
// out-channels' credits][G] in one uncached block.
void HipPlanExecutor::setupDevSteps() {
  GLX_ENFORCE(sync_.outChans.size() == out_.size() && sync_.inChans.size() == in_.size(),
              "plan kernel: channel tables disagree");
  enforceSpan((size_t)sync_.slice);
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
  // the flag rows, then the run count on lines of its own, uncached like the
  // flags: the 8 XCDs' L2s are not coherent with each other, and the
  // workgroup that advances the count and the ones that read it in the next
  // launch may sit on different XCDs -- in memory no L2 holds, every read
  // sees the last advance without relying on the cache maintenance at
  // kernel boundaries
  char* block = ddAlloc(rows * G * glx::kFlagBytes + glx::launchCtrBytes((int)G));
  runCtr_ = reinterpret_cast<uint64_t*>(block + rows * G * glx::kFlagBytes);
  pk_.runCtr = runCtr_;
  launchCtr_ = runCtr_;

  pk_.polls = nullptr;
  if (const char* e = std::getenv("GLOO_AMD_COUNT_POLLS"); e != nullptr && e[0] == '1') {
    GLX_HIP_CHECK(hipMalloc((void**)&polls_, G * sizeof(uint64_t)));
    GLX_HIP_CHECK(hipMemset(polls_, 0, G * sizeof(uint64_t)));
    pk_.polls = polls_;
  }
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
    const bool pre = slots_ == 2 && y.pre >= 0;  // partial reduce-and-forward
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
        if (pre) {  // segments [pre0, pre1) were stored by step y.pre
          d.pre0 = y.pre0;
          d.pre1 = y.pre1;
        }
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
          d.kind = s.kind == glx::COPY ? glx::kStepCopySend
                   : y.keep != 0     ? glx::kStepReduceSend
                                     : glx::kStepReduceForward;
          d.peer = (int32_t)t.peer;
          d.seq = ty.seq;
          d.perRun = ty.perRun;
          d.dst = vbase(landing(peerBlocks_[oc.peer], t.dst_off, t.off), t.off);
          d.dstSlot = (int64_t)slotBytes(blockOf(peerBlocks_[oc.peer], t.dst_off));
          d.flag = oc.devDelivery;
          d.credit = rows + (size_t)oc.creditWord * G * glx::kFlagStride;
        } else if (pre) {  // the overlap into the next SEND's slot, after its credit
          const glx::Step& t = plan_.steps[(size_t)y.pre];
          const glx::StepSync& ty = sync_.steps[(size_t)y.pre];
          const OutChan& oc = out_[(size_t)ty.chan];
          d.kind = s.kind == glx::COPY ? glx::kStepCopyPre
                   : y.keep != 0     ? glx::kStepReducePre
                                     : glx::kStepReducePreForward;
          d.peer = (int32_t)t.peer;
          d.seq = ty.seq;
          d.perRun = ty.perRun;
          d.dst = vbase(landing(peerBlocks_[oc.peer], t.dst_off, t.off), t.off);
          d.dstSlot = (int64_t)slotBytes(blockOf(peerBlocks_[oc.peer], t.dst_off));
          d.credit = rows + (size_t)oc.creditWord * G * glx::kFlagStride;
          d.pre0 = y.pre0;
          d.pre1 = y.pre1;
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
  if (st == glx::kStatusOverlap) {
    broken_ = true;
    const volatile uint64_t* d = reinterpret_cast<const volatile uint64_t*>(ddStatus_);
    GLX_ENFORCE(false, "device-driven allreduce (rank ", contextRank_, "): launch ", d[2],
                " started while launch ", d[1],
                " of the same algorithm was still running -- its runs and graph replays "
                "must be stream-ordered (issue them on the algorithm's stream, or make "
                "the other stream wait for it); the algorithm is unusable now");
  }
  if ((st & ~0xffff) == glx::kStatusPeerAbort) {
    broken_ = true;
    GLX_THROW_IO("Rank ", st & 0xffff, " gave up on its DMA steps run (a wait of its timed "
                      "out, or it saw a peer exit), so its copies to rank ", contextRank_,
                      " may have landed without their credit; rank ", contextRank_,
                      " stopped its run rather than return that data (DMA steps engine, abort "
                      "mark)");
  }
  if (st != 0) {
    broken_ = true;
    const int peer = (st & 255) - 1, step = (st >> 8) - 1;
    std::string where;
    if (step >= 0 && (size_t)step < plan_.steps.size()) {
      const glx::Step& s = plan_.steps[(size_t)step];
      where = std::string(", ") + (s.kind == glx::SEND ? "credit for send" : "receive") +
              " step " + std::to_string(step) +
              (engine_ == kEngineDmaSteps ? std::string(" (DMA steps engine)")
                                          : " of run " + std::to_string(devRuns_ - 1));
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
  const uint64_t e = ++ddEpoch_;  // the host's count (diagnostics); the kernels count on the GPU
  const uint64_t ticks = (uint64_t)effectiveTimeout().count() * (uint64_t)clockKhz_;
  // epochs stay ordered even when calls come on different streams (on the
  // same stream the order is the stream's -- and a launch being captured
  // into a graph must not wait on an event recorded outside the capture)
  if (ddLaunched_ && ddLastStream_ != compute_) {
    GLX_HIP_CHECK(hipStreamWaitEvent(compute_, ddDone_, 0));
  }
  if (staged_) waitH2D(compute_, computeH2dWaited_, 0, count_);
  if (engine_ == kEngineOneShot) {
    glx::OneShotParams p = os_;
    p.buf = ptr0;
    p.epoch = e;
    p.timeoutTicks = ticks;
    for (int j = 0; j < P; j++) {
      if (j == contextRank_) {
        for (int par = 0; par < 2; par++) {
          p.push[par][j] = nullptr;
          p.land[par][j] = ptr0;
        }
        p.flagOut[j] = nullptr;
        continue;
      }
      const auto& pb = ddPeer_.at(j);
      for (int par = 0; par < 2; par++) {  // the kernel picks by its epoch's parity
        p.push[par][j] = pb[(size_t)par] + (size_t)contextRank_ * ddSlot_;
        p.land[par][j] = ddBlocks_[(size_t)par] + (size_t)j * ddSlot_;
      }
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
        for (int par = 0; par < 2; par++) {
          p.rsPush[par][j] = p.agPush[par][j] = nullptr;
          p.rsLand[par][j] = p.agLand[par][j] = nullptr;
        }
        p.flagAOut[j] = p.flagBOut[j] = nullptr;
        continue;
      }
      const auto& pb = ddPeer_.at(j);
      const size_t mine = (size_t)contextRank_ * ddSlot_, theirs = (size_t)j * ddSlot_;
      for (int par = 0; par < 2; par++) {  // the kernel picks by its epoch's parity
        const size_t q = (size_t)par;
        p.rsPush[par][j] = vbase(pb[q] + mine, j);                      // my copy of range j
        p.rsLand[par][j] = vbase(ddBlocks_[q] + theirs, contextRank_);  // j's copy of mine
        p.agPush[par][j] = vbase(pb[2 + q] + mine, contextRank_);       // my result
        p.agLand[par][j] = vbase(ddBlocks_[2 + q] + theirs, j);         // j's result
      }
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
  // The done event serves a later call on another stream (function-style
  // calls) and the staged copy-back; run() keeps one stream for its life,
  // and each event record costs the stream several microseconds per call.
  if (staged_ || fnCalls_) {
    GLX_HIP_CHECK(hipEventRecord(ddDone_, compute_));
    transport_.doneEvents++;
  }
  ddLaunched_ = true;
  ddLastStream_ = compute_;
  if (staged_) {
    GLX_HIP_CHECK(hipStreamWaitEvent(d2h_, ddDone_, 0));
    copyBack({glx::Range{0, count_}});
  }
}

}  // namespace gloo
