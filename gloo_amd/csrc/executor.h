// executor.h -- runs a compiled schedule (plan.h) on this rank's GPU.
//
// This is the device-side Algorithm: HipAllreduceRingChunked and
// HipAllreduceHalvingDoubling are an Executor over the corresponding plan.
//   * payload: hipMemcpyPeerAsync ptr0 -> peer receive region, on a
//     dedicated copy stream (side stream, as gloo's CUDA path keeps copies
//     off the compute stream, gloo/cuda_allreduce_ring_chunked.cc:322-356);
//   * reduction: glx reduce kernel on the compute stream (the user's
//     stream when one is given);
//   * copy/compute overlap: a SEND waits (GPU side, hipStreamWaitEvent) only
//     for the compute work that produced its source; a REDUCE/COPY waits only
//     for in-flight SENDs whose source range it overwrites;
//   * completion signalling: host progress loop polls hipEventQuery and
//     bumps peers' counters (see context.h), never blocking on one stream.
#pragma once

#include <hip/hip_runtime_api.h>

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <cstdint>
#include <map>
#include <memory>
#include <vector>

#include "context.h"
#include "kernels.h"
#include "plan.h"

namespace gloo {

class Algorithm {  // gloo/algorithm.h:20-38
 public:
  explicit Algorithm(const std::shared_ptr<Context>& ctx)
      : context_(ctx), contextRank_(ctx->rank), contextSize_(ctx->size) {}
  virtual ~Algorithm() noexcept(false) {}
  virtual void run() = 0;

 protected:
  std::shared_ptr<Context> context_;
  const int contextRank_;
  const int contextSize_;
};

class HipPlanExecutor : public Algorithm {
 public:
  HipPlanExecutor(const std::shared_ptr<Context>& ctx, int algo,
                  const std::vector<void*>& ptrs, int64_t count, int dtype,
                  int op, const std::vector<hipStream_t>& streams,
                  const glx::PlanParams& prm = glx::PlanParams(), bool perCallBuffers = false);
  ~HipPlanExecutor() noexcept(false) override;

  // Class-style run (gloo/allreduce_ring_chunked.h:83-212): fold ptrs into
  // ptrs[0], run the schedule on it, copy it to the other pointers.
  void run() override;

  // Host-memory endpoint fed from a transport (the reference
  // receives socket bytes into a registered host buffer,
  // gloo/transport/tcp/pair.cc:385-451): runFed() is run() on a host buffer
  // whose bytes are NOT all there yet -- each H2D piece is issued when
  // feed() has covered it, and every step waits only for the pieces of its
  // own range, so the schedule starts on the first bytes to arrive.  feed()
  // may be called from another thread, before or during runFed() (feeds
  // count for the next runFed).  doneRanges() lists the element ranges whose
  // final values are back in host memory (in completion order; the ring
  // returns chunk after chunk), for a caller streaming results out.
  void runFed();
  void feed(int64_t off, int64_t len);
  std::vector<glx::Range> doneRanges();

  // Function-style run (gloo/allreduce.cc:97-146) on buffers given per call:
  // inputs reduced into out[0] (genLocalReduceFunction, :44-82), the schedule
  // on out[0], out[0] copied to out[1..] (genLocalBroadcastFunction, :87-95).
  // The buffers may differ from call to call; nothing about them is
  // published to peers.
  struct FnCall {
    std::vector<void*> in, out;
    hipStream_t stream = nullptr;  // null: own stream, complete on return
    std::chrono::milliseconds timeout{0};  // 0: the context's
  };
  void runFn(const FnCall& call);

  int64_t bytesSentPerRun() const { return plan_.bytes_sent * (int64_t)esize_; }

  // How this algorithm's messages actually moved, counted since
  // construction (SENDs of the host-issued steps engine, by mechanism, and
  // launches of a device-driven engine, whose kernels store into the peers'
  // memory themselves).
  struct TransportStats {
    int64_t peerCopies = 0;     // hipMemcpyPeerAsync (DMA engines over xGMI)
    int64_t deviceCopies = 0;   // hipMemcpyAsync: same-device peers, or after
                                // hipMemcpyPeerAsync refused an IPC mapping
    int64_t kernelCopies = 0;   // copy kernel storing into the peer's memory
    int64_t deviceKernels = 0;  // one-shot / two-shot / plan kernel launches
    int64_t bytes = 0;          // bytes of the copies above
    int64_t hostFolds = 0;      // local reduces done on the host (kOnDeviceThreshold)
    int64_t doneEvents = 0;     // hipEventRecords after a run's work (each costs
                                // the stream several microseconds)
    int64_t flagKernels = 0;    // DMA steps engine: flag-op launches (hand-offs)
  };
  const TransportStats& transportStats() const { return transport_; }
  // Record `ev` after this algorithm's last enqueued work: the compute
  // stream of the last run (the caller's stream when one was given).
  void recordDone(hipEvent_t ev);

  // Copies of one SEND are split over this many streams per destination
  // (several DMA engines feeding one link).  Read at construction.
  static void setCopySplit(int k);
  static int copySplit();
  // How a SEND moves its bytes: kCopyDma = hipMemcpyPeerAsync (copy
  // engines), kCopyKernel = a copy kernel storing into the peer's memory
  // over xGMI.  Read at construction.
  static constexpr int kCopyDma = 0, kCopyKernel = 1;
  static void setCopyEngine(int engine);
  static int copyEngine();
  const glx::Plan& plan() const { return plan_; }
  // How run() executes: kEngineSteps (host-issued schedule steps),
  // kEngineOneShot / kEngineTwoShot (one device-driven kernel per rank).
  int engine() const { return engine_; }
  // the plan kernel runs nontemporal loads and write-through stores
  bool fastStreams() const { return engine_ == kEngineDevSteps && pk_.fast != 0; }

 private:
  struct OutChan {  // this rank -> peer
    int peer, tag;
    uint32_t creditWord;            // in our control block, written by peer
    std::atomic<uint64_t>* credit;  // = our word
    std::atomic<uint64_t>* delivery = nullptr;  // in peer's block
    uint64_t sent = 0;
    int peerDevice = -1;
    int stream = 0;
    int peerRow = -1;                 // plan kernel: the receiver's delivery row
    uint64_t* devDelivery = nullptr;  // plan kernel: that row (peer memory)
  };
  struct CopyStream {
    hipStream_t s = nullptr;
    uint64_t waitedMark = 0;      // last compute mark this stream waited on
    hipEvent_t last = nullptr;    // last copy recorded in the current run
    int h2dWaited = -1;           // host mode: last H2D piece waited on this run
    // DMA steps engine: this stream's done word (copies completed, counted
    // across runs)
    uint32_t doneWord = 0;
    uint64_t copies = 0;
  };
  struct InChan {  // peer -> this rank
    int peer, tag;
    uint32_t deliveryWord;
    std::atomic<uint64_t>* delivery;  // our word, written by peer
    std::atomic<uint64_t>* credit = nullptr;  // in peer's block
    uint64_t received = 0, consumed = 0;
    int peerRow = -1;               // plan kernel: the sender's credit row
    uint64_t* devCredit = nullptr;  // plan kernel: that row (peer memory)
  };
  static constexpr int kMaxSplit = 8;
  struct Pending {  // fire `value` into `word` once all `ev` (maybe none) complete
    hipEvent_t ev[kMaxSplit];
    int nev;
    std::atomic<uint64_t>* word;
    uint64_t value;
  };
  // Receive scratch is allocated in blocks (each region whole in one block,
  // blocks <= kMaxBlockBytes unless one region is larger), each exported with
  // its own IPC handle.
  struct ScratchBlock {
    int64_t start = 0;  // first element (in plan region coordinates)
    int64_t elems = 0;
    char* ptr = nullptr;
    SharedRef ref;  // the context's shared block (allocShared), as peers map it
  };
  static constexpr size_t kMaxBlockBytes = size_t(256) << 20;
  struct InflightSend {
    int64_t off, len;
    hipEvent_t event;
    int stream = -1;    // DMA steps engine: the copy stream and its done count
    uint64_t done = 0;  // once this send's copy completed
  };

  void publish();
  void resolvePeers();
  std::vector<int64_t> retiredIn(const std::vector<char>& rec) const;
  int outIndex(int peer, int tag);
  int inIndex(int peer, int tag);
  void pollPending();
  template <typename Pred>
  void waitFor(Pred done, const char* what, int peer);
  void drain();
  // len >= 0: throw unless len elements from there stay inside the block
  char* landing(const std::vector<ScratchBlock>& blocks, int64_t boff, int64_t off,
                int64_t len = -1) const;
  void exchange(char* ptr0);
  // One SEND's bytes (or one split part of them) to oc's peer on stream s:
  // the copy kernel, hipMemcpyPeerAsync, or hipMemcpyAsync (same device, or
  // after the peer API refused a mapping)
  void issueCopy(char* dst, const char* src, size_t len, OutChan& oc, hipStream_t s);
  // DMA steps engine (kEngineDmaSteps): the host-issued program -- the same
  // copies on the copy streams, the same reduce launches on the compute
  // stream -- with every hand-off made on the GPU by flag-op kernels
  // (kernels.h FlagOpsParams) instead of by the host, so run() only enqueues.
  // Flag words, one per 128-byte line, in one uncached block peers map
  // (ddBlocks_[0]): our abort word (word 0, kernels.h abort marks), our
  // in-channels' delivery words, our out-channels' credit words, the compute
  // mark, each copy stream's done word; all but the abort word count across
  // runs.
  void setupDmaSteps();
  void exchangeDma(char* ptr0);
  uint64_t* dmaWord(uint32_t w) const {
    return reinterpret_cast<uint64_t*>(ddBlocks_[0]) + (size_t)w * glx::kFlagStride;
  }
  // Flag ops wait in ONE list, for one stream at a time, and go out as a
  // kernel before anything else is enqueued: on any stream, or by the host
  // (a flush whenever the next op or enqueue is for another stream).  So every
  // rank enqueues its ops in program order, and streams that share a hardware
  // queue run them in that order -- a signal queued behind a later wait of
  // another stream could hold up a peer that this wait is for.
  void dmaOp(hipStream_t s, int32_t kind, uint64_t* word, uint64_t value, int32_t code = 0);
  void dmaFlush();
  std::vector<glx::FlagOp> dmaOps_;
  hipStream_t dmaOpsStream_ = nullptr;
  uint32_t markWord_ = 0;
  uint64_t marks_ = 0;     // compute marks signalled
  std::vector<uint64_t*> dmaAbortOut_;  // peers' abort words (their flag blocks' word 0)
  uint64_t dmaTicks_ = 0;  // the current run's wait timeout in s_memrealtime ticks
  std::chrono::milliseconds effectiveTimeout() const {
    return timeout_.count() > 0 ? timeout_ : context_->getTimeout();
  }  // the plan's steps on ptr0 (contextSize_ > 1)
  void localReduce(const std::vector<void*>& in, const std::vector<void*>& out);
  // Receive scratch blocks; `slots` copies of each (the plan kernel's
  // landing slots, plan.h SyncTable::slots), slotBytes() apart.
  void allocScratch(bool uncached = false, int slots = 1);
  size_t slotBytes(const ScratchBlock& b) const;
  const ScratchBlock& blockOf(const std::vector<ScratchBlock>& blocks, int64_t boff) const;
  int slots_ = 1;  // plan kernel: landing slots per channel
  void waitWar(int64_t off, int64_t len);
  // The constructor's work; on a throw the constructor releases whatever it
  // had acquired (the destructor never runs for a half-built object).
  void construct(const std::shared_ptr<Context>& ctx, const std::vector<void*>& ptrs,
                 const std::vector<hipStream_t>& streams, const glx::PlanParams& prm,
                 bool perCallBuffers);
  void release() noexcept;
  static void givePinned(char* p, size_t bytes);
  // Before our memory is freed: wait (bounded by the context timeout) until
  // every receiver has credited our last message.  Those credit stores are
  // the only writes a peer can still make into our memory (shm counters or,
  // for the plan kernel, device flag rows) after our last run returned.
  void drainCredits() noexcept;
  bool broken_ = false;  // a wait timed out or a peer exited

  glx::Plan plan_;
  int algo_;
  std::vector<void*> ptrs_;
  int64_t count_;
  int dtype_, op_;
  size_t esize_;
  int device_ = -1;
  int slot_ = 0;
  bool userStream_ = false;
  hipStream_t compute_ = nullptr;
  // the caller's streams of ptrs[1..] (CudaAllreduceRingChunked's one stream
  // per pointer, gloo/cuda_allreduce_ring_chunked.cc:53-66): run() orders
  // itself after their pending work and their later work after its results
  std::vector<hipStream_t> sideStreams_;
  std::vector<hipEvent_t> sideIn_;
  hipEvent_t sideOut_ = nullptr;
  std::vector<CopyStream> copies_;
  uint64_t markEpoch_ = 0;
  int split_ = 1;
  int copyEngine_ = kCopyDma;
  bool peerCopyOk_ = true;  // hipMemcpyPeerAsync accepted for IPC-mapped peers
  TransportStats transport_;
  bool ownCompute_ = false;
  std::vector<ScratchBlock> blocks_;                  // ours
  std::map<int, std::vector<ScratchBlock>> peerBlocks_;  // by destination rank
  std::chrono::milliseconds timeout_{0};  // per-call override (0: context's)

  // Host-memory endpoints (host mode): the user's pointers are
  // host memory; the schedule runs on device copies.  H2D pieces go out in
  // first-use order on h2d_ and every step waits only for the pieces of its
  // own range; each range is copied back on d2h_ right after its final write.
  // Pinned user memory is copied directly.  Pageable user memory is never
  // handed to the runtime (no hipHostRegister of the caller's pages, no
  // pageable hipMemcpy): it is mirrored by a pinned workspace block, as the
  // reference's CUDA algorithms stage host data through a pinned host
  // workspace (gloo/cuda_workspace.h, CudaHostWorkspace); a piece is copied
  // into the mirror on the host when it is issued, and a range comes back
  // out of it once its D2H copy has completed (doneRanges / end of run).
  bool hostMode_ = false;
  std::vector<char*> devBufs_;     // device copy of each user pointer (or of hostStage_)
  bool hostFold_ = false;          // several pointers < kOnDeviceThreshold: fold on the host
  char* hostStage_ = nullptr;      // pinned: the host fold's result, staged and returned
  size_t hostStageBytes_ = 0;      // its size (from and back to a process-wide cache)
  // A pinned block of the process-wide cache: a whole-buffer mirror, or --
  // when no mirror of the buffer's size could be pinned (or it exceeds
  // glx_set_pinned_mirror_limit) -- a bounce block of two halves of at
  // most kBounceBytes (H2D pieces through the first, D2H ranges through the
  // second) that every copy goes through piece by piece, waiting for each
  // piece (a failed pinned allocation must not fail the op)
  struct PinnedBlock {
    char* p = nullptr;
    size_t bytes = 0;
    bool bounce = false;
  };
  // A host buffer as the copies see it: `user` (the caller's) and `dma`
  // (what the DMA reads / writes: `user` itself when pinned, else its
  // mirror; null when the copies go through the bounce block `bounce`)
  struct HostSide {
    char* user;
    char* dma;
    PinnedBlock* bounce;
  };
  std::vector<HostSide> hostSources() const;  // H2D sources of the staged buffer
  std::vector<HostSide> hostDests() const;    // where its final values go back to
  static HostSide sideOf(char* u, const PinnedBlock* m);
  // m's mirror for a pageable buffer of `bytes` (or its bounce block)
  void takeMirror(PinnedBlock& m, size_t bytes);
  // copies through a bounce block: H2D returns with the last piece in flight
  // on `s`; D2H returns with every byte in `user`
  void bounceIn(char* dev, const char* user, size_t n, PinnedBlock& b, hipStream_t s);
  void bounceOut(char* user, const char* dev, size_t n, PinnedBlock& b, hipStream_t s);
  std::vector<PinnedBlock> ptrMirror_;  // per ptrs_ entry (p == nullptr: pinned)
  PinnedBlock callMirror_[2];           // a function-style call: source, destination
  bool callMirrored_[2] = {false, false};  // the current call uses them
  std::vector<PinnedBlock> fnMirror_;   // runFnHost's whole-buffer copies
  // The pinned block `m` (taken from the process-wide cache on first use)
  // when `user` is pageable, else `user`.
  char* mirrorFor(void* user, PinnedBlock& m);
  // Mirrored destinations: ranges [at, at+n) from the mirror to the user.
  void copyOut(const std::vector<glx::Range>& ranges);
  void flushMirrors();  // every completed batch's copy-out (end of a run)
  // staged_: the current run stages host memory (class host mode, or a
  // function-style call on host buffers); callSrc_/callDst_: that call's
  // host buffers
  bool staged_ = false;
  std::vector<void*> callSrc_, callDst_;
  void setupCallStaging();
  void runFnHostStaged(const FnCall& call);
  hipStream_t h2d_ = nullptr, d2h_ = nullptr;
  glx::StagePlan stage_;
  std::vector<hipEvent_t> h2dEvents_;  // one per stage_.h2d piece
  std::vector<hipEvent_t> pieceDone_;  // one rank, several pointers: piece j folded
  std::vector<hipEvent_t> d2hEvents_;  // one per step (recorded where d2h is non-empty)
  hipEvent_t hostDone_ = nullptr;
  int computeH2dWaited_ = -1;
  void setupHostMode();
  void waitH2D(hipStream_t s, int& waited, int64_t off, int64_t len);
  void copyBack(const std::vector<glx::Range>& ranges);
  void runHost();
  // fed runs (runFed / feed): feeds of the current run, merged; which H2D
  // pieces have been issued; completed copy-backs (event, ranges)
  std::mutex feedMutex_;
  std::condition_variable feedCv_;
  bool fedRun_ = false;
  std::vector<glx::Range> fed_;
  std::vector<uint8_t> pieceIssued_;
  void issueFedPiecesLocked();
  void issuePiece(size_t j);
  std::mutex doneMutex_;
  struct DoneBatch {
    hipEvent_t ev;
    std::vector<glx::Range> ranges;
    bool pendingOut;  // the ranges still sit in mirrors only
  };
  std::vector<DoneBatch> doneQueue_;
  std::vector<hipEvent_t> doneEvents_;  // pool
  size_t doneUsed_ = 0;
  std::vector<char*> fnStage_;  // device staging of function-style host buffers
  void runFnHost(const FnCall& call);
  std::vector<OutChan> out_;
  std::vector<InChan> in_;
  std::vector<int> stepChan_;        // channel index per step
  std::vector<hipEvent_t> events_;   // split_ per step
  hipEvent_t computeMark_ = nullptr;
  // end of the last call's work and the stream it ran on (the caller's, for
  // runFn with a stream): release() waits for it, recordDone() orders after it
  hipEvent_t lastDone_ = nullptr;
  hipStream_t lastStream_ = nullptr;
  void noteDone(hipStream_t s);
  bool resolved_ = false;
  std::vector<Pending> pending_;
  std::vector<InflightSend> inflight_;

  // Device-driven engines (xgmi_kernels.hip): the replicated schedule as the
  // one-shot kernel, the mesh schedule as the two-shot kernel.  No channels,
  // no scratch blocks; uncached blocks (IPC-exported, each its own handle):
  //   one-shot: [0],[1] landing slots [P][ddSlot_] of parity 0/1; [2] flags [P][G]
  //   two-shot: [0],[1] RS slots, [2],[3] AG slots of parity 0/1;
  //             [4] flags: A [P][G], then B [P][G]
  int engine_ = kEngineSteps;
  std::vector<char*> ddBlocks_;
  std::vector<SharedRef> ddRefs_;  // ddBlocks_' shared blocks, as peers map them
  // Device memory peers will map, from the context's pool of exported blocks
  // (flags 0: hipMalloc, else hipExtMallocWithFlags); back to the pool in
  // release().
  char* allocShared(size_t bytes, unsigned flags, SharedRef* ref);
  std::map<int, std::vector<char*>> ddPeer_;  // peers' blocks (IPC-mapped)
  size_t ddSlot_ = 0;                         // bytes per landing slot
  glx::OneShotParams os_{};                   // fixed parts of the kernels' parameters
  glx::TwoShotParams ts_{};
  // plan kernel (engine devsteps): step table, segments and fold sources in
  // device memory, built at the first run (they hold peers' addresses)
  glx::PlanKernelParams pk_{};
  glx::PlanParams prm_;
  glx::SyncTable sync_;
  glx::DevStep* devSteps_ = nullptr;
  std::vector<glx::DevStep> hostSteps_;  // host copy (timeout diagnostics)
  glx::DevSegment* devSegs_ = nullptr;
  uint64_t* runCtr_ = nullptr;  // the plan kernel's run count (kernels.h), in the flag block
  // the device engine's launch counters (kernels.h launchCtrBytes), any engine
  uint64_t* launchCtr_ = nullptr;
  // GLOO_AMD_COUNT_POLLS=1: the plan kernel's flag reads per workgroup
  // (PlanKernelParams::polls), reported on stderr when the algorithm is freed
  uint64_t* polls_ = nullptr;
  void reportPolls() noexcept;
  // Wait (bounded by the deadline) until every launch of the device engine
  // that has started -- graph replays on any stream included -- completed;
  // returns the launches completed (0 if unknown).
  uint64_t settleLaunches(std::chrono::steady_clock::time_point deadline) noexcept;
  // A device-engine launch wrote the status word (a timed-out wait or an
  // overlapping launch): its workgroups stopped early.
  bool deviceReported() const noexcept {
    return ddStatus_ != nullptr && *reinterpret_cast<const volatile int*>(ddStatus_) != 0;
  }
  const char** devFoldSrc_ = nullptr;
  uint64_t devRuns_ = 0;
  uint64_t ddEpoch_ = 0;
  int* ddStatus_ = nullptr;  // pinned host word the kernels flag timeouts in
  int* ddStatusDev_ = nullptr;
  int* ddClaim_ = nullptr;  // device word: the first timed-out workgroup claims the report
  hipEvent_t ddDone_ = nullptr;
  bool ddLaunched_ = false;
  // a function-style call came (runFn): the stream may change from call to
  // call, so every device launch records ddDone_ for the next one to wait on
  bool fnCalls_ = false;
  hipStream_t ddLastStream_ = nullptr;  // the stream of the last device-engine launch
  int clockKhz_ = 100000;  // s_memrealtime rate
  uint64_t* trace_ = nullptr;  // GLOO_AMD_DEVTRACE=1: two-shot phase stamps (pinned host)
  static bool devTrace();
  void traceTwoShot(const glx::TwoShotParams& launched);
  void traceDevSteps(const glx::PlanKernelParams& launched);
  static int engineFor(const Context& ctx, int algo, int64_t count, int esize);
  // uncached device memory from the context's pool (flag rows; landing slots
  // when `slots`, which the test-only kSyncCachedSlots allocates cached)
  char* ddAlloc(size_t bytes, bool slots = false);
  // the test-only kSyncCachedSlots mode is in force (kernels.h)
  static bool cachedSlotsForTest();
  void setupDevice();
  size_t maxSlices(int kernel) const;
  void setupOneShot();
  void setupTwoShot();
  void setupDevSteps();
  void buildDevSteps();
  void runDevice(char* ptr0);
  void checkDevice();
  // Wait for stream s after a device-engine launch.  While waiting, watch
  // the peers' processes: if one exits, stop every kernel wait at once
  // (status word) and throw IoException instead of running into the timeout.
  void waitDevice(hipStream_t s);

 public:
  static constexpr int kEngineSteps = 0, kEngineOneShot = 1, kEngineTwoShot = 2,
                       kEngineDevSteps = 3, kEngineDmaSteps = 4;
  // Whether the DMA steps engine can run on this context: not for rank
  // threads sharing a device (their streams share the process's hardware
  // queues, where one rank's flag wait would hold up a peer's copy it waits
  // for), not under the device-engine mode "off".  Processes sharing a GPU
  // may: a flag wait holds one wave, not the GPU's CUs.
  static bool dmaStepsAvailable(const Context& ctx);
  // Whether device-driven engines can run on this context:
  // deviceEnginesRule over the context's endpoints and setDeviceEngines.
  static bool deviceEnginesAvailable(const Context& ctx);
  // The rule itself (glx_device_engines_rule), a pure function so every rank
  // derives the same answer from the same endpoints and the CPU tests can
  // walk it.  mode: kDevEnginesAuto / Off / On / Shared.
  //  * auto (default): only when every rank has a GPU of its own.  Ranks
  //    sharing a GPU wait for each other's kernels while holding its CUs, so
  //    any other work queued ahead of one rank's collective -- on its stream
  //    or in a hardware queue its stream shares -- can be starved by the
  //    peers' resident grids until the timeout (8 x 1 queue,
  //    a GEMM ahead of rank 0's collective, profiles/r9j_*, r9l_*).  No
  //    queue count rules that out (a GEMM on the collective's own stream
  //    forms the same cycle), so the default keeps such ranks on the
  //    host-issued steps, which hold no CUs while they wait.
  //  * shared: also processes sharing a GPU, while ranks-on-the-GPU x
  //    (queues + 1) <= kSharedQueueBudget -- for rehearsals and callers that
  //    run nothing else on the shared GPU while a collective is in flight.
  //    Never threads of one process (their launches may serialise).
  //  * on: always (the caller guarantees co-residency); off: never.
  static bool deviceEnginesRule(int mode, int size, int ranksPerDevice, bool threadsShareDevice,
                                int maxQueues);
  static constexpr int kDevEnginesAuto = -1, kDevEnginesOff = 0, kDevEnginesOn = 1,
                       kDevEnginesShared = 2;
  // Processes sharing one GPU (shared mode) get the device engines only while
  // ranks-on-the-GPU x (hwQueuesPerProcess() + 1) stays within this many
  // hardware queues, leaving room for one more process's (measured on one
  // MI355X with a busy parent process: 2x4, 3x4, 4x4, 5x2, 6x2, 8x1
  // co-schedule; 8x2 and 8x4 time-slice: profiles/r7g_queue_sweep.txt).
  static constexpr int kSharedQueueBudget = 20;
  static int hwQueuesPerProcess();
  void enforceSpan(size_t sliceElems) const;
  // Mode for algorithms created afterwards (kDevEngines*); the initial value
  // comes from GLOO_AMD_DEVICE_ENGINES=auto|off|on|shared.
  static void setDeviceEngines(int mode);
  static int deviceEngines();
  // Engine of the mesh schedule when available: kEngineTwoShot (default)
  // or kEngineSteps.  Read at construction.
  static void setMeshEngine(int engine);
  static int meshEngine();
  // Engine of the ring, halving-doubling, bcube and function-style ring
  // schedules when available: -1 = automatic (default: the plan kernel with
  // one rank per GPU; ranks sharing a GPU: up to 32 MiB per rank, host-issued
  // steps above), kEngineDevSteps or kEngineSteps.
  static void setStepsEngine(int engine);
  static int stepsEngine();
  // Streams of the device-driven kernels for algorithms created afterwards:
  // 0 plain loads and stores (default), 1 nontemporal loads and write-through
  // stores (glx_set_engine_streams).
  static void setEngineStreams(int fast);
  // release / acquire around the device engines' flags: -1 auto, 0 system
  // scope, 1 narrow, 2-4 the test-only broken modes (kernels.h kSync*); for
  // algorithms created afterwards
  static void setDeviceSync(int mode);
  static int deviceSync();
  static constexpr bool kAutoNarrow = true;
  // the device engine's kernels.h kSync* mode (1 narrow, 0 system scope,
  // 2-4 test-only), -1 host-issued steps (and the DMA steps engine: its flags follow
  // completed stream work, no fences)
  int syncMode() const {
    if (engine_ == kEngineSteps || engine_ == kEngineDmaSteps) return -1;
    if (cachedSlots_) return glx::kSyncCachedSlots;
    return engine_ == kEngineDevSteps ? pk_.narrow
                                      : (engine_ == kEngineOneShot ? os_.narrow : ts_.narrow);
  }
  bool cachedSlots_ = false;  // landing slots allocated cached (test-only mode)
  static int engineStreams();
};

}  // namespace gloo
