// kernels.h -- host-side launchers of the HIP kernels (reduce_kernels.hip).
#pragma once

#include <hip/hip_runtime_api.h>
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace glx {

// dst = op(a, b), n elements of dtype, on stream s.  Never synchronises.
hipError_t launch_reduce(int op, int dtype, void* dst, const void* a,
                         const void* b, size_t n, hipStream_t s);

// Fold of op over srcs[0..k-1] (k >= 1): acc = srcs[0], then
// acc = op(acc, srcs[j]) (rev = false, left fold) or acc = op(srcs[j], acc)
// (rev = true, the ring's chain order).  dst may alias srcs[0].
hipError_t launch_reduce_n(int op, int dtype, void* dst, const void* const* srcs,
                           int k, size_t n, hipStream_t s, bool rev = false);

// Several independent folds (same op/dtype/order) in one launch.
struct FoldSpec {
  void* dst;
  std::vector<const void*> srcs;
  int k;
  size_t n;
};
hipError_t launch_reduce_n_batch(int op, int dtype, const std::vector<FoldSpec>& specs,
                                 hipStream_t s, bool rev);

// Byte copy dst <- src as a kernel on stream s (dst may be a peer GPU's
// IPC-mapped memory: the stores then travel over xGMI).  Never synchronises.
hipError_t launch_copy(void* dst, const void* src, size_t bytes, hipStream_t s);
// The same with an explicit grid (<= 0: the configured copy_blocks()).
hipError_t launch_copy_blocks(void* dst, const void* src, size_t bytes, int grid,
                              hipStream_t s);
// Grid (workgroups) of the copy kernel.
void set_copy_blocks(int blocks);
int copy_blocks();

// One-shot replicated allreduce (xgmi_kernels.hip): one kernel per rank
// pushes the buffer to every peer, waits on per-slice flags and folds every
// chunk along its ring chain.  All pointers are device-accessible; push/land
// regions and flags are uncached device memory (peers' via IPC).
constexpr int kOsMaxRanks = 8;
constexpr int kOsMaxSlices = 512;  // workgroups (= slices) per launch
// Write-through stores address their stream through a buffer resource with
// 32-bit offsets (elem_ops.h): one stream -- a reduce launch's destination,
// or one workgroup's span of a device engine -- must stay below 2 GiB.
constexpr size_t kWtMaxStream = (size_t(1) << 31) - 16;
// Flags are 8-byte words, each alone in its 128-byte L2 line: flag f of a
// row starts at row + f * kFlagStride (no line holds flags of two writers).
constexpr int kFlagStride = 16;
// Release / acquire around the device engines' flags.  Everything a flag
// publishes lives in the receiver's landing slots: uncached device memory
// (MTYPE UC), never held by an L2.  System scope (narrow = 0) still writes
// back every dirty line of the XCD's L2 before each flag (buffer_wbl2 sc0
// sc1) and invalidates the L2 after each wait (buffer_inv sc0 sc1); narrow
// (1) only completes the stores (s_waitcnt vmcnt(0)) before a flag and
// invalidates the CU's L1 after a wait (agent scope).
//
// The `narrow` field of the engines' parameters holds one of these modes.
// Modes 2-4 are TEST ONLY positive controls (GLOO_AMD_SYNC=unsafe_*): each
// breaks one premise of the narrow form, so the GPU suite can show that its
// checks catch a stale hand-off (tests/test_sync_control_gpu.py).
constexpr int kSyncSystem = 0;
constexpr int kSyncNarrow = 1;
constexpr int kSyncNoAcquire = 2;  // narrow without the consumer's L1 invalidate
constexpr int kSyncNoRelease = 3;  // narrow without the producer's store-completion wait and
                                   // the workgroup barrier before its flag
constexpr int kSyncUnsafe = 4;     // neither, and plain (write-back) stores into peers' slots
// narrow, with every engine's landing slots in CACHED memory (hipMalloc): the
// narrow form's premise (no L2 holds a slot line) broken on the host side;
// the kernels run kSyncNarrow
constexpr int kSyncCachedSlots = 5;
constexpr size_t kFlagBytes = kFlagStride * sizeof(uint64_t);
// A device engine's launch counters (xgmi_kernels.hip launch_number), uncached,
// after its flag rows: a line with the launches completed, a line with the
// workgroups finished in the current launch, then one word per workgroup
// index: the launches that index has started.
constexpr size_t kLaunchStartsOffset = 2 * kFlagStride;  // in uint64 words
inline size_t launchCtrBytes(int G) {
  return kLaunchStartsOffset * sizeof(uint64_t) +
         (((size_t)G * sizeof(uint64_t) + kFlagBytes - 1) / kFlagBytes) * kFlagBytes;
}
// status code of a launch that started while the previous launch of the same
// algorithm was still running (words 1, 2: launches completed, its number)
constexpr int kStatusOverlap = 0x7fff0000;
struct OneShotParams {
  char* buf;                        // this rank's buffer: input and result
  // by the epoch's parity (the two slot sets alternate between launches):
  char* push[2][kOsMaxRanks];       // this rank's landing region in peer j (j != rank)
  const char* land[2][kOsMaxRanks];  // rank k's landing region here (k != rank)
  uint64_t* flagOut[kOsMaxRanks];   // peer j's flag row for this rank ([G] flags)
  const uint64_t* flagIn;           // this rank's flags: [P][G] flags
  int* status;                      // host-visible: 1 + rank that never arrived
  int* claim;                       // device word: the first timed-out workgroup reports
  int flagStore;                    // 1: write peers' flags with stores (Context::flagStores)
  int narrow;                       // 1: narrow release / acquire around flags (below)
  uint64_t epoch;                   // host's count of its launches (diagnostics only)
  // uncached device memory, launchCtrBytes(G): the launch's epoch is its
  // launch number + 1 (>= 1, +1 per launch, equal on all ranks) --
  // graph-capturable, as PlanKernelParams::runCtr
  uint64_t* epochCtr;
  uint64_t timeoutTicks;            // s_memrealtime ticks
  size_t count;                     // elements
  size_t slice;                     // elements per workgroup, multiple of 16 / esize
  int P, rank, G;
  int njobs;                        // chunk ranges with their own chain
  size_t jobOff[kOsMaxRanks], jobLen[kOsMaxRanks];
  uint8_t chain[kOsMaxRanks][kOsMaxRanks];  // fold order: acc = op(x[chain[i]], acc)
};
hipError_t launch_oneshot(int op, int dtype, const OneShotParams& p, hipStream_t s);

// Two-shot mesh allreduce (xgmi_kernels.hip): rank j owns range j; every
// rank pushes its copy of range j to owner j, the owner folds it along its
// chain and pushes the result to everyone.  Slot pointers are "virtual
// buffers": element i of range c at ptr + i * esize.
struct TwoShotParams {
  char* buf;
  // by the epoch's parity (the two slot sets alternate between launches):
  char* rsPush[2][kOsMaxRanks];        // owner j's RS slot for this rank's copy of range j
  const char* rsLand[2][kOsMaxRanks];  // this rank's RS slot holding rank k's copy of range rank
  char* agPush[2][kOsMaxRanks];        // peer j's AG slot for this rank's finished range
  const char* agLand[2][kOsMaxRanks];  // this rank's AG slot holding owner j's finished range
  uint64_t* flagAOut[kOsMaxRanks];  // owner j's A-flag row for this rank ([G] flags)
  const uint64_t* flagAIn;          // [P][G]: rank k's copy of my range slice landed
  uint64_t* flagBOut[kOsMaxRanks];  // peer j's B-flag row for this rank as owner
  const uint64_t* flagBIn;          // [P][G]: owner j's finished slice landed
  int* status;
  int* claim;
  int flagStore;
  int narrow;                       // 1: narrow release / acquire around flags (below)
  uint64_t epoch, timeoutTicks;     // epoch: the host's count (diagnostics only)
  uint64_t* epochCtr;               // as OneShotParams::epochCtr
  size_t rangeOff[kOsMaxRanks], rangeLen[kOsMaxRanks];  // by owner
  uint8_t chain[kOsMaxRanks];       // this rank's fold order
  size_t slice;                     // elements per workgroup per range, multiple of 16 / esize
  int P, rank, G;
  // diagnostics (GLOO_AMD_DEVTRACE=1): per workgroup [G][kTsTrace] s_memrealtime
  // stamps: start, pushed, peers' copies landed, folded, results landed, end
  uint64_t* trace;
};
constexpr int kTsTrace = 6;
hipError_t launch_twoshot(int op, int dtype, const TwoShotParams& p, hipStream_t s);
// Plan kernel (xgmi_kernels.hip): ANY compiled schedule (a plan.h step
// program) as one device-driven kernel per rank.  The buffer is cut into
// segments at every step boundary of every rank's program and every segment
// into G slices; workgroup w owns slice w of every segment on every rank, so
// each step gives every workgroup a share and an element is always handled
// by the same workgroup index: workgroups of one rank never wait for each
// other, workgroup w only for workgroup w of its peers.  Per (channel,
// workgroup) flag rows carry the host executor's delivery / credit counts.
struct DevSegment {
  int64_t off, len, slice;  // slice: elements per workgroup, whole 16-byte vectors
};
// Step kinds of the plan kernel: glx::StepKind (0 SEND, 1 RECV, 2 REDUCE,
// 3 COPY, 4 RELEASE, 5 FOLD) plus the reduce-and-forward forms (plan.h
// StepSync::fuse): REDUCE or COPY and the SEND of the same range in one
// pass, and the SEND they absorbed, which is then skipped; ReduceForward is
// a ReduceSend whose result goes to the peer's slot only (StepSync::keep 0:
// the buffer's copy would be overwritten unread).
constexpr int32_t kStepReduceSend = 6, kStepCopySend = 7, kStepNop = 8, kStepReduceForward = 9;
// Partial reduce-and-forward (plan.h StepSync::pre): a REDUCE / COPY whose
// segments [pre0, pre1) also go into the next SEND's slot (ReducePreForward:
// into that slot only), and that SEND (kind 0 with pre0 < pre1) storing only
// its other segments before it signals.
constexpr int32_t kStepReducePre = 10, kStepReducePreForward = 11, kStepCopyPre = 12;
struct DevStep {
  int32_t kind;            // glx::StepKind or kStep* above
  int32_t peer;            // reported on timeout
  int32_t seg0, seg1;      // the step's element range = segments [seg0, seg1)
  int32_t nsrc;            // FOLD: number of sources, first at foldSrc[srcIndex]
  int32_t left;            // FOLD: 1 = left fold (plan.h kFoldLeft), 0 = the ring's chain
  int32_t pre0, pre1;      // partial reduce-and-forward: the overlap's segments
  int64_t srcIndex;
  const char* src;         // REDUCE / COPY: landing region (slot 0) as a virtual buffer
  char* dst;               // SEND: the peer's landing region (slot 0) as a virtual buffer
  uint64_t* flag;          // SEND: peer's delivery row; RECV: my delivery row;
                           // RELEASE: peer's credit row
  const uint64_t* credit;  // SEND: my credit row
  uint64_t seq, perRun;    // SEND/RECV/RELEASE: message number within a run (1-based),
                           // messages per run
  uint64_t rseq, rperRun;  // REDUCE / COPY: the same for the message they read
  int64_t srcSlot;         // REDUCE / COPY: bytes from one landing slot to the next
  int64_t dstSlot;         // SEND: the same in the peer's region
};
struct PlanKernelParams {
  char* buf;
  const DevStep* steps;        // device memory
  const DevSegment* segs;      // device memory
  const char* const* foldSrc;  // device memory; nullptr = buf
  int nsteps, G;
  int slots;                   // landing slots per channel (1 or 2, plan.h SyncTable)
  int maxSrc;                  // most sources of a FOLD step (2 when there is none)
  uint64_t run;                // host's count of its launches (diagnostics only)
  // uncached device memory, per algorithm, launchCtrBytes(G): [0] runs
  // completed, advanced by the last workgroup to finish a launch; a
  // workgroup's run number is the launches its index started before -- so the message
  // numbers follow the launches the GPU actually ran, a launch captured in a
  // graph and replayed numbers its messages like an eager one, and a launch
  // overlapping the previous one reports kStatusOverlap (xgmi_kernels.hip
  // launch_number)
  uint64_t* runCtr;
  uint64_t timeoutTicks;
  int* status;
  int* claim;
  int narrow;                  // 1: narrow release / acquire around flags (below)
  int flagStore;               // 1: write peers' flags with stores (Context::flagStores)
  int fast;                    // 1: nontemporal loads, write-through stores (plan kernel only;
                               // every span's stores stay below kWtMaxStream: setupDevSteps)
  // diagnostics (GLOO_AMD_DEVTRACE=1): [G][2 * nsteps + 1] s_memrealtime
  // stamps per workgroup: step i started (2i), its wait was satisfied
  // (2i + 1; RECV / SEND only), the kernel ended (2 nsteps)
  uint64_t* trace;
  // diagnostics (GLOO_AMD_COUNT_POLLS=1): [G] device words, += the flag reads
  // (memory-side compare-exchanges) each workgroup's waits made per launch
  uint64_t* polls;
};
hipError_t launch_plan_kernel(int op, int dtype, const PlanKernelParams& p, hipStream_t s);

// kSyncUnsafe's kernels: the same engines compiled with plain stores into
// peers' slots (xgmi_kernels.hip built a second time with
// GLX_XGMI_UNSAFE_TU; the launchers above dispatch to them).
hipError_t launch_oneshot_unsafe_stores(int op, int dtype, const OneShotParams& p,
                                        hipStream_t s);
hipError_t launch_twoshot_unsafe_stores(int op, int dtype, const TwoShotParams& p,
                                        hipStream_t s);
hipError_t launch_plan_kernel_unsafe_stores(int op, int dtype, const PlanKernelParams& p,
                                            hipStream_t s);

// Stream-ordered flag operations of the DMA steps engine (engine dmasteps,
// executor.cc exchange): the host-issued program's copies (hipMemcpyPeerAsync
// on the copy streams) and reduce launches, with every hand-off between them
// -- a copy waiting for the receiver's credit or for the reduce that produced
// its chunk, a reduce waiting for its message, the credit back to the sender
// -- made on the GPU by this one-wave kernel on the stream it orders, instead
// of by the host.  Lane 0 performs the ops in order: kFlagWait waits (bounded)
// until *word >= value, kFlagSignal writes value into word (a flag word in
// this rank's or a peer's uncached flag block).  The stream's earlier work
// has completed when the kernel starts (stream order); before its first
// signal the kernel also releases at system scope (buffer_wbl2 sc0 sc1), so
// the signal publishes that work to SDMA engines and peers whatever scope the
// runtime's release between kernels had.
//
// Abort marks: a copy waits for its receiver's credit in the flag
// kernel before it, but HIP runs the copy whatever that kernel found.  So a
// flag kernel that gives up -- a wait timed out, the status word was set (a
// peer exited, another wait gave up, release() of a broken algorithm) or a
// peer's abort mark arrived -- first writes 1 + rank into the abort word of
// every peer (abortOut) and completes that write before it ends, i.e. before
// the copy queued behind it can start.  Every flag kernel reads its own abort
// word (abortIn) at its start and while it waits: a receiver whose landing
// region such a copy may have overwritten reaches the RELEASE of that region
// only after the reduce reading it has finished, so if the copy landed during
// the reduce the mark was already there, and the run fails with
// kStatusPeerAbort + sender instead of returning the overwritten data.
constexpr int kFlagOpsMax = 8;
constexpr int kFlagAbortMax = 32;
constexpr int kStatusPeerAbort = 0x7ffe0000;  // | the aborting peer's rank
constexpr int32_t kFlagWait = 0, kFlagSignal = 1;
struct FlagOp {
  uint64_t* word;
  uint64_t value;
  int32_t kind;  // kFlagWait / kFlagSignal
  int32_t code;  // wait: status code on timeout, 1 + peer + 256 * (1 + step)
};
struct FlagOpsParams {
  FlagOp ops[kFlagOpsMax];
  int n;
  int flagStore;          // 1: signals are stores (Context::flagStores), else exchanges
  uint64_t timeoutTicks;  // s_memrealtime ticks, each wait from the kernel's start
  int* status;            // host-visible: a timeout's code; nonzero stops every wait
  int* claim;             // device word: the first timed-out wait reports
  const uint64_t* abortIn;              // this rank's abort word (nonzero: a peer gave up)
  uint64_t* abortOut[kFlagAbortMax];    // peers' abort words, written when this rank gives up
  int nAbort;
  uint64_t abortValue;                  // 1 + this rank
};
hipError_t launch_flag_ops(const FlagOpsParams& p, hipStream_t s);

// Workgroups of a device-engine kernel (kernel 0 = one-shot, 1 = two-shot,
// 2 = plan kernel, 3 = plan kernel for programs without FOLD steps) for
// (op, dtype) that fit on the current device at once
// (occupancy x CUs).  A grid of peers waiting on each other must be
// resident as a whole.
int device_engine_resident_blocks(int kernel, int op, int dtype);

// Streams longer than this go out as consecutive launches of the reduce
// kernel over equal segments of at most this many bytes (reduce_kernels.hip
// kSegBytes).
size_t reduce_segment_bytes();

// Tuning knobs of the vector kernel (lanes' unroll depth, grid cap per CU,
// nontemporal loads/stores: 0/1, -1 = keep).
void set_reduce_tuning(int unroll, int blocks_per_cu, int nontemporal);
// The settings now in force (policy: 0..3 a fixed one, 4 automatic).
void reduce_tuning(int* unroll, int* blocks_per_cu, int* policy);

}  // namespace glx
