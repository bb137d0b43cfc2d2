// plan.h -- per-rank step programs of the allreduce schedules (host logic).
//
// A schedule is compiled, once per algorithm instance, into a straight-line
// program of steps that the xGMI executor (executor.cc) runs on every
// run().  The same programs are exported through glx_plan() so the CPU test
// suite can replay them against the oracle without a GPU.
//
//   SEND    copy ptr0[off, off+len) into peer's receive region `dst_off`
//           of channel `channel` (one hipMemcpyPeerAsync), then bump the
//           channel's delivery counter in the peer's control block.
//   RECV    wait until the next message on (peer, channel) has landed.
//   REDUCE  ptr0[off, off+len) = op(ptr0[off, off+len), region(boff))
//   COPY    ptr0[off, off+len) = region(boff)
//   RELEASE the last message of (peer, channel) is consumed: once the GPU
//           work reading it completes, credit the sender.
//   FOLD    ptr0[off, off+len) = op(s[k-1], ... op(s[2], op(s[1], s[0]))),
//           s[i] = region(folds[boff][i]), or ptr0[off, off+len) itself for
//           an entry of -1 -- a ring's per-chunk reduction chain evaluated in
//           one pass (the operand order of every op is the ring's: the newer
//           rank's value first, the running partial second).  With flags &
//           kFoldLeft the order is the left fold op(...op(op(s0, s1), s2)...),
//           i.e. bcube's "out = op(out, peer)" for peers in group order.
//
// Region offsets are in elements; each region is padded by kPadElems so a
// message can land at the 16-byte phase of the receiver's ptr0 (keeps the
// reduce kernel on its dwordx4 path for any chunk offset).
#pragma once

#include <cstdint>
#include <utility>
#include <vector>

namespace glx {

enum StepKind : int64_t { SEND = 0, RECV = 1, REDUCE = 2, COPY = 3, RELEASE = 4, FOLD = 5 };

struct Step {
  int64_t kind;
  int64_t peer;     // SEND: destination rank; RECV/RELEASE: source rank
  int64_t channel;  // channel tag (per ordered rank pair)
  int64_t off;      // SEND: source offset; REDUCE/COPY: destination offset (elements of ptr0)
  int64_t len;      // elements (0 allowed for SEND/RECV: a signal only)
  int64_t boff;     // RECV/REDUCE/COPY: region base in this rank's scratch
  int64_t dst_off;  // SEND: region base in the peer's scratch
  int64_t flags;
};

struct Plan {
  std::vector<Step> steps;
  std::vector<std::vector<int64_t>> folds;  // FOLD sources (region offsets; -1 = ptr0)
  int64_t scratch_elems = 0;  // receive-region space (incl. padding), elements
  int64_t bytes_sent = 0;     // payload bytes this rank sends per run (for metrics)
};

enum Algo {
  ALGO_RING_CHUNKED = 0,       // class AllreduceRingChunked
  ALGO_HALVING_DOUBLING = 1,   // class AllreduceHalvingDoubling
  ALGO_RING_CHUNKED_MESH = 2,  // ring_chunked's result over all links
  ALGO_FN_RING = 3,            // gloo::allreduce(opts), Algorithm::RING
  ALGO_FN_RING_MESH = 4,       // its result over all links
  ALGO_FN_BCUBE = 5,           // gloo::allreduce(opts), Algorithm::BCUBE
  ALGO_RING_CHUNKED_REPL = 6,  // ring_chunked's result in one round (small buffers)
  ALGO_FN_RING_REPL = 7,       // RING's result in one round (small buffers)
  ALGO_RING = 9,               // class AllreduceRing (whole buffers, per-rank order)
  ALGO_BCUBE = 10,             // class AllreduceBcube (groups of `base` ranks)
};

constexpr int64_t kFoldLeft = 1;  // FOLD flag, see above
// FOLD flag: the source regions hold whole-buffer messages (sent from
// element 0), so s[i] for ptr0[off...] sits `off` elements into region i.
constexpr int64_t kFoldWhole = 2;

// gloo/allreduce.h:80 (AllreduceOptionsImpl::kMaxSegmentSize)
constexpr int64_t kMaxSegmentBytes = 1 << 20;

// Messages longer than this go as consecutive pieces (splitMessages below),
// so no receive region -- hence no shared block another process imports --
// reaches the 2 GiB at which the HIP runtime's IPC import hangs
// (Context::kIpcMaxBlockBytes), whatever count the reference accepts
// (VERDICT r5 #3); two landing slots of a piece still fit below it.
constexpr int64_t kMaxMessageBytes = int64_t(512) << 20;
// The process-wide setting (glx_set_max_message_bytes; every rank must use
// the same): kMaxMessageBytes unless changed -- tests lower it to run split
// programs at small sizes.
int64_t maxMessageBytes();
void setMaxMessageBytes(int64_t bytes);

// Inputs of the function-style schedules besides (rank, size, count).
struct PlanParams {
  int esize = 4;                                // bytes per element
  int64_t maxSegmentBytes = kMaxSegmentBytes;   // opts.maxSegmentSize
  // Device pipelining granularity of the function-style ring: a chunk's
  // segments are moved in pieces of at least this many bytes (results are
  // unchanged: they depend only on which rank owns which element, which
  // maxSegmentBytes fixes exactly as the reference does).
  int64_t minPieceBytes = 4 << 20;
  // class AllreduceBcube: ranks per group (gloo::Context::base, default 2)
  int base = 2;
  // messages above this many bytes are split (kMaxMessageBytes)
  int64_t maxMessageBytes = glx::maxMessageBytes();
  // > 0: pipelining below chunk granularity (the executor sets it for the
  // host-issued and DMA steps engines, glx_set_pipeline_bytes): messages are
  // cut into pieces of about this many bytes, and a reduce-and-forward is
  // done per piece (splitMessages' `forward`)
  int64_t pipelineBytes = 0;
};

// Cut every message whose landing spans more than maxElems elements into
// consecutive pieces.  A message for ptr0[off, off + len) lands at its
// region's 16-byte base plus the phase off mod V (V = 16 / esize elements);
// sub-region q of a region is [q * maxElems, (q + 1) * maxElems) past that
// base (maxElems a multiple of V), and piece q is the part of the message
// landing there -- so every piece after the first starts at phase 0 at its
// sub-region's base, and the sub-regions are the same for every message of
// the region.  The sender's SEND becomes one SEND per piece (dst + q *
// maxElems); on the receiver, each group of RECVs, the REDUCE / COPY / FOLD
// steps reading their regions and their RELEASEs (every schedule's shape) is
// repeated per piece, every step narrowed to piece q (the offset of each
// message is taken from the steps reading it).  Piece q travels on channel
// tag + q * kPieceChannelStride: one channel per sub-region, so each credit
// protects exactly the bytes it guards, and a piece never waits for an
// earlier piece of its own message, which the receiver may release only after
// its own sends (halving-doubling's exchanges would deadlock).  The
// per-element reduction chains are untouched: results are bit-identical.
// Plans folding whole-buffer messages (kFoldWhole: AllreduceRing, the
// replicated schedules) are left whole.
//
// forward: the SENDs right after a receive group that send one of its
// REDUCE / COPY results on (the ring's "reduce, notify, forward",
// gloo/allreduce_ring_chunked.h:141-157; the mesh's result to every peer)
// go out per piece too, right after that piece's RELEASE -- the next rank
// starts on piece 0 while this one reduces piece 1 (the reference's own
// segmented ring keeps two segments in flight, gloo/allreduce.cc:279-321).
// Each piece index is its own ring of messages, so this adds no credit cycle.
constexpr int64_t kPieceChannelStride = int64_t(1) << 16;
void splitMessages(Plan& p, int64_t maxElems, int64_t V, bool forward = false);

// glx_set_pipeline_bytes / GLOO_AMD_PIPELINE_BYTES: 0 (default) = off.
int64_t pipelineBytes();
void setPipelineBytes(int64_t bytes);

// Region padding: room to land a message at any 16-byte phase after
// rounding its region base up to 16 bytes (<= 30 bytes for 1-byte elements).
constexpr int64_t kPadElems = 32;

// gloo/allreduce_ring_chunked.h:22-236
Plan planRingChunked(int rank, int size, int64_t count);
// gloo/allreduce_halving_doubling.h:37-361
Plan planHalvingDoubling(int rank, int size, int64_t count);

// ring_chunked's chunking and exact reduction order, moved over all links:
// every rank folds its own chunk pair from the other ranks' copies (one
// xGMI link per peer), then sends the result to everyone.
Plan planRingChunkedMesh(int rank, int size, int64_t count);

// gloo/allreduce.cc:148-393 (ring) with the reference's segment ownership;
// pieces of >= minPieceBytes move two at a time per direction.
Plan planFnRing(int rank, int size, int64_t count, const PlanParams& prm);
// The same chunks and reduction chains, each owner folding its chunk from
// all peers at once.
Plan planFnRingMesh(int rank, int size, int64_t count, const PlanParams& prm);
// One-round ("replicated") variants for small buffers: every rank sends its
// whole buffer to every peer and evaluates every chunk's reduction chain
// itself (one batched fold launch).  Same chains as the ring, so the same
// bits; (P-1)·S bytes out per rank, one dependent round instead of 4P-4.
Plan planRingChunkedReplicated(int rank, int size, int64_t count);
Plan planFnRingReplicated(int rank, int size, int64_t count, const PlanParams& prm);

// gloo/allreduce.cc:395-669 (bcube, n = 2)
Plan planFnBcube(int rank, int size, int64_t count);
// AllreduceRing (gloo/allreduce_ring.h:72-114): every rank ends with its own
// left fold x[r] op x[r-1] op ... op x[r-P+1] of the locally reduced buffers
// (ranks' float results may differ, as in the reference).  The reference
// forwards whole buffers around the ring in P-1 dependent rounds; here every
// rank sends its buffer to every peer in one round (P-1 links, S each) and
// folds in the reference's order.
Plan planRing(int rank, int size, int64_t count);
// AllreduceBcube (gloo/allreduce_bcube.h:256-695): log_base(P) steps; in
// step s each rank exchanges with the other members of its group (ranks
// base^s apart) and reduces its own range, peers in group order; then the
// all-gather retraces the steps.  Ranges, counts and the groups follow the
// reference's Node / Group setup (:620-695, :60-240) exactly, including its
// wrap-around offsets when there are fewer elements than group members.
Plan planBcube(int rank, int size, int64_t count, int base);

Plan makePlan(int algo, int rank, int size, int64_t count,
              const PlanParams& prm = PlanParams());

// Automatic data movement for the ring's result (all bit-identical): the
// one-round replicated schedule up to a threshold per rank, the all-links
// mesh above, the ring itself from kMeshMaxBytes.  fn: the function-style RING family instead of the class
// ring_chunked one.  deviceDriven: the replicated schedule will run as the
// one-shot kernel (no host round trips), which moves the threshold from
// 256 KiB to 16 MiB (P = 2), 2 MiB (P <= 4) or 1 MiB (P <= 8).  (An
// explicit schedule -- "ring", "mesh", "replicated" -- forces one.)
// Largest buffer (bytes per rank) the automatic choice gives the mesh.
constexpr int64_t kMeshMaxBytes = (int64_t(2) << 30) - (int64_t(64) << 20);
int autoRingSchedule(int size, int64_t bytes, bool fn, bool deviceDriven = false);

// Geometry of the device-driven engines (xgmi_kernels.hip), read off a
// compiled replicated plan (one-shot) or mesh plan (two-shot): the same
// ranges and chains as the plan's FOLD steps, so the kernels compute exactly
// what the steps engine computes.  One workgroup per slice index; slices are
// >= 4 KiB, whole 16-byte vectors, at most maxSlices of them.
constexpr int kDevMaxRanks = 8;
struct DeviceLayout {
  int G = 0;            // workgroups = slices
  int64_t slice = 0;    // elements per slice (one-shot: of the buffer;
                        // two-shot: of every owner's range)
  // one-shot: chunk ranges and each one's chain (fold order of ranks)
  int njobs = 0;
  int64_t jobOff[kDevMaxRanks] = {}, jobLen[kDevMaxRanks] = {};
  int chain[kDevMaxRanks][kDevMaxRanks] = {};
  // two-shot: owner j's range, and this rank's own chain
  int64_t rangeOff[kDevMaxRanks] = {}, rangeLen[kDevMaxRanks] = {};
  int myChain[kDevMaxRanks] = {};
  int64_t maxLen = 0;   // largest range (two-shot slot size)
};
DeviceLayout oneShotLayout(const Plan& plan, int rank, int size, int64_t count, int esize,
                           int64_t maxSlices);
DeviceLayout twoShotLayout(const Plan& plan, int rank, int size, int64_t count, int esize,
                           int64_t maxSlices);

// The plan kernel's bookkeeping for one rank's program: segment bounds (0,
// count and both ends of every data step of EVERY rank's program, so all
// ranks cut alike and every step range is a union of segments), the slice
// (every segment is cut into G slices of this many elements, a whole number
// of 16-byte vectors; workgroup w owns slice w of every segment), and per
// step its channel (out-channel index for SEND, in-channel index for RECV /
// RELEASE, numbered by first use -- the executor's numbering), its segments
// and its message number within a run (1-based) out of perRun.
//
// safe: the kernel's credits are per (channel, workgroup), so a landing
// region is protected only if every two messages landing in it give every
// byte they both cover to the same workgroup (a workgroup may run several
// messages ahead of another).  Checked over every region of every rank;
// when it fails the executor keeps the host-issued steps.
//
// fuse: a REDUCE or COPY whose result the program sends on next (the SEND of
// the same range follows it with only RELEASEs in between -- the ring's
// "reduce, notify, forward", gloo/allreduce_ring_chunked.h:141-157) names
// that SEND; the plan kernel does both in one pass (the result goes to the
// buffer and into the receiver's landing region together, so the link is
// busy while the chunk is reduced) and waits for the SEND's credit before
// the pass.  Moving that wait earlier cannot deadlock: the credit is for the
// previous message on the channel, whose release depends only on older
// messages.  The SEND itself then names the step it was fused into.
//
// slots: landing slots per channel.  The kernel keeps 2 when it can (no FOLD
// in any rank's program, every landing region fed by one channel): message
// n of a channel lands in slot (n-1) % 2, so a SEND waits for the release of
// message n-2 instead of n-1.  That is what makes the fused wait above
// deadlock-free: with one slot, rank r's fused pass would wait for rank
// r+1's release of message k, which r+1 gives only after its own fused pass
// waits for r+2's release of k ... around the ring; with two, each wait is
// for an older message, down to the first two, which need none.  Fusion is
// therefore used only with 2 slots.
//
// rseq/rperRun: for a REDUCE or COPY, the message number of the RECV whose
// landing region it reads (its slot).
//
// keep: for a fused REDUCE, whether its result must also stay in the
// buffer.  In the ring's reduce-scatter a rank forwards each partial sum and
// never reads it again: the allgather's COPY overwrites the range with the
// final value first (gloo/allreduce_ring_chunked.h:141-157 then :173-200).
// keep = 0 when, scanning this rank's program past the fused SEND, the first
// step touching any element of the range is a COPY covering all of it; any
// read (REDUCE, SEND, FOLD) or partial overwrite first, or none at all (the
// value is final), keeps it.  The plan kernel then stores the partial only
// into the peer's slot: 0.75 S fewer HBM writes per rank at P = 8.
//
// pre: partial reduce-and-forward, where the SEND after a REDUCE / COPY (past
// RELEASEs only) covers part of its range, or more: halving-doubling's
// reduce-scatter reduces a block and sends half of it on in the next step,
// its allgather copies a block in and sends it on together with the rest.
// The REDUCE / COPY names that SEND (pre) and stores the overlap's segments
// [pre0, pre1) into the receiver's slot in the same pass, after the SEND's
// credit; the SEND (pre = that step, same pre0 / pre1) stores only its other
// segments and then signals the message.  keep applies to the overlap of a
// REDUCE (0: the overlap's values go to the peer only).
struct StepSync {
  int32_t chan = -1;
  int32_t seg0 = 0, seg1 = 0;
  uint64_t seq = 0, perRun = 0;
  int32_t fuse = -1;  // REDUCE/COPY: the SEND fused into it; SEND: the step it is in
  uint64_t rseq = 0, rperRun = 0;
  int32_t keep = 1;
  int32_t pre = -1;           // see above
  int32_t pre0 = 0, pre1 = 0;  // the overlap, in segments
};
struct SyncTable {
  std::vector<int64_t> bounds;
  int64_t slice = 0;
  bool safe = true;
  int slots = 1;
  bool anyFold = false;  // some rank's program has a FOLD step
  // the largest receive region (elements) of ANY rank's program: every rank
  // derives the plan kernel's landing-slot count from it alike
  int64_t maxRegionElems = 0;
  std::vector<std::pair<int, int>> outChans, inChans;  // (peer, tag)
  std::vector<StepSync> steps;
};
SyncTable syncTable(int algo, int rank, int size, int64_t count, const PlanParams& prm,
                    int G);
// The receive region some message lands in at `start` (RECV steps land at
// their region's start): up to the next start, but no further than its
// longest message plus the landing pad; 0 if nothing lands there.  The
// executor allocates exactly these (allocScratch).
int64_t landedRegionElems(const Plan& plan, int64_t start, int64_t next);
// The largest of them in one program.
int64_t maxRegionOf(const Plan& plan);

// Host-memory endpoints: when the user's buffer is in host
// memory the executor stages it through a device buffer.  This derives from
// a plan (1) the order to copy the buffer in: pieces in the order the steps
// first touch them, so the schedule starts after the first piece instead of
// the whole buffer; (2) for every step, the ranges whose final value it
// writes (copied back right after it), and the ranges no step writes
// (copied back at the end).  Pieces are at most maxPiece elements.
struct Range {
  int64_t off, len;
};
struct StagePlan {
  std::vector<Range> h2d;                 // issue order
  std::vector<std::vector<Range>> d2h;    // per step index
  std::vector<Range> d2hRest;
};
StagePlan stagePlan(const Plan& plan, int64_t count, int64_t maxPiece);

}  // namespace glx
