/*
 * glx.h -- the C-ABI drop-in boundary of gloo_amd (MI355X-native gloo
 * allreduce hot path).  Plain pointers, sizes and ints only: no C++ and no
 * torch types cross this line.  Implemented by gloo_amd/libgloo_amd.so
 * (sources under gloo_amd/csrc).
 *
 * Every entry point names the reference interface it replaces
 * (liuxiaotiao/gloo, paths relative to the reference root).
 *
 * Conventions
 *   - Return value: GLX_OK (0) or a GLX_ERR_* code.  Functions never throw.
 *     glx_last_error() returns the message of the calling thread's last
 *     failure (mirrors GLOO_ENFORCE -> EnforceNotMet, gloo/common/logging.h:21-52,
 *     and IoException, gloo/common/error.h:45).
 *   - Streams are hipStream_t passed as void*; NULL = the internal stream of
 *     the object (or the legacy default stream for glx_reduce).
 *   - dtype / op codes below; op values equal gloo::ReductionType
 *     (gloo/algorithm.h:49-57).
 */
#ifndef GLOO_AMD_GLX_H_
#define GLOO_AMD_GLX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* libgloo_amd.so exports exactly these entry points: everything else in it
 * is built with hidden visibility, so it links beside the reference's own
 * libgloo (whose C++ symbols share the namespace `gloo`) without clashing. */
#if defined(__GNUC__)
#pragma GCC visibility push(default)
#endif

/* ---- codes ------------------------------------------------------------ */
enum glx_dtype {
  GLX_INT8 = 0,
  GLX_UINT8 = 1,
  GLX_INT32 = 2,
  GLX_INT64 = 3,
  GLX_UINT64 = 4,
  GLX_FLOAT32 = 5,
  GLX_FLOAT64 = 6,
  GLX_FLOAT16 = 7,  /* gloo::float16, gloo/types.h:96 */
  GLX_BFLOAT16 = 8  /* no reference counterpart (parity unpinned) */
};

enum glx_op { /* == gloo::ReductionType, gloo/algorithm.h:49-57 */
  GLX_SUM = 1,
  GLX_PRODUCT = 2,
  GLX_MAX = 3,
  GLX_MIN = 4
};

enum glx_status {
  GLX_OK = 0,
  GLX_ERR_INVALID = 1,  /* bad argument -> EnforceNotMet */
  GLX_ERR_HIP = 2,      /* HIP runtime error (CUDA_CHECK analog, gloo/cuda_private.h:25-37) */
  GLX_ERR_TIMEOUT = 3,  /* IoException("Timed out ..."), gloo/common/error.h:45 */
  GLX_ERR_IO = 4,       /* IoException (peer gone / closed) */
  GLX_ERR_ENFORCE = 5,  /* EnforceNotMet, gloo/common/logging.h:21 */
  GLX_ERR_INTERNAL = 6
};

typedef void* glx_stream_t; /* a hipStream_t */

/* Message of this thread's last failed call ("" if none). */
const char* glx_last_error(void);
/* Library version, e.g. "0.1.0". */
const char* glx_version(void);
/* Size in bytes of one element of dtype (0 if unknown). */
size_t glx_dtype_size(int dtype);

/* ---- device kernels ---------------------------------------------------- */

/* dst[i] = op(a[i], b[i]) for i < n, enqueued on `stream` (device pointers;
 * dst may alias a or b).  Replaces the per-chunk reduction
 *   gloo::sum/product/max/min<T>(void* c, const void* a, const void* b, size_t n)
 *     -- gloo/math.h:15-73
 * and its device analog cudaSum/cudaProduct/cudaMax/cudaMin(T*, const T*,
 * size_t, cudaStream_t) -- gloo/cuda.h:274-284, gloo/cuda.cu:307-434.
 * Semantics are the CPU path's: max(a,b) = (a < b) ? b : a (operand order
 * matters for NaN / signed zero); 16-bit floats widen to fp32, op, and round
 * to nearest even once (float16 NaN -> 0x7fff, gloo/types.h:181-204,248-305).
 * Integer sum/product wrap. */
int glx_reduce(int op, int dtype, void* dst, const void* a, const void* b,
               size_t n, glx_stream_t stream);

/* dst[i] = op(...op(op(srcs[0][i], srcs[1][i]), srcs[2][i])..., srcs[k-1][i])
 * -- the left fold the reference performs for ptrs.size() > 1
 * (gloo/allreduce_ring_chunked.h:89-91, gloo/allreduce_halving_doubling.h:232-234),
 * fused into one pass.  2 <= k <= 8. */
int glx_reduce_n(int op, int dtype, void* dst, const void* const* srcs, int k,
                 size_t n, glx_stream_t stream);

/* The same left fold on HOST memory (host pointers; dst may be srcs[0]),
 * 1 <= k.  The analog of the reference's cudaHostReduce, which its GPU
 * algorithms use below kOnDeviceThreshold = 256 KiB (gloo/algorithm.cc:16,
 * gloo/cuda_allreduce_halving_doubling.cc:478-484); the algorithms here use
 * it for multi-pointer host buffers under that size.  Same bits as
 * glx_reduce_n. */
int glx_host_reduce_n(int op, int dtype, void* dst, const void* const* srcs, int k,
                      size_t n);

/* Device->device copy of `bytes` from (src on srcDev) to (dst on dstDev) over
 * xGMI with hipMemcpyPeerAsync.  Replaces the D2D copy of CudaStream::copyAsync
 * (gloo/cuda.cu:91-149) and the transport's Buffer::send for device buffers
 * (gloo/transport/buffer.h:26-34). */
int glx_peer_copy(void* dst, int dst_dev, const void* src, int src_dev,
                  size_t bytes, glx_stream_t stream);

/* The same copy made by the copy kernel the kernel transport uses
 * (glx_set_copy_engine(1, blocks)): 16-byte vector stores from this GPU's
 * compute units straight into `dst`, which may be a peer GPU's memory mapped
 * into this process (IPC) -- the CU-driven counterpart of glx_peer_copy, for
 * measuring what stores over one xGMI link reach.  `blocks` workgroups
 * (<= 0: the transport's current setting). */
int glx_copy(void* dst, const void* src, size_t bytes, int blocks, glx_stream_t stream);

/* hipDeviceEnablePeerAccess both ways between devices a and b (idempotent).
 * Analog of cudaDeviceEnablePeerAccess in gloo/cuda_collectives_native.h:216-276. */
int glx_enable_peer(int dev_a, int dev_b);

/* Tuning hook of the reduce kernel: lanes' unroll depth (1, 2, 4 or 8 16-byte
 * vectors in flight per lane), grid cap in workgroups per CU (0 = keep) and
 * the cache policy of its streams (`nontemporal`; -1 keep): 0 plain loads and
 * stores, 1 nontemporal loads and stores, 2 nontemporal loads and
 * write-through (sc1) stores, 3 nontemporal loads and plain stores, 4 auto
 * (default: 2 while one stream is at most 256 MiB -- the Infinity Cache's
 * size -- and 1 above). */
int glx_tune_reduce(int unroll, int blocks_per_cu, int nontemporal);
/* The reduce kernel's settings now in force (policy 4 = automatic).  The
 * settings are process-wide and atomic: rank threads may launch while
 * another thread tunes. */
int glx_reduce_tuning(int* unroll, int* blocks_per_cu, int* policy);
/* Messages above this many bytes go as consecutive pieces, each a message of
 * its own landing in a receive region of its own (plan.h splitMessages), so
 * no block another process must import reaches 2 GiB whatever the count
 * (default 512 MiB; 0 restores it; at least 4096).  Process-wide, for
 * algorithms created afterwards; every rank must use the same value (checked
 * when the algorithm's peers resolve).  Results are unchanged. */
int glx_set_max_message_bytes(int64_t bytes);
int64_t glx_max_message_bytes(void);
/* Pipelining below chunk granularity for the host-issued and DMA steps
 * engines on device buffers: each message goes as pieces of about this many
 * bytes, each reduced and forwarded on its own (plan.h splitMessages with
 * forward; the reference's segmented ring keeps two segments in flight,
 * gloo/allreduce.cc:279-321).  0 = off (default; GLOO_AMD_PIPELINE_BYTES).
 * Process-wide, for algorithms created afterwards; every rank must use the
 * same value (checked).  Results are unchanged. */
int glx_set_pipeline_bytes(int64_t bytes);
int64_t glx_pipeline_bytes(void);
/* glx_reduce on more than this many bytes per stream goes out as consecutive
 * kernel launches over equal segments of at most this size (one grid-stride
 * launch over 1 GiB streams ran 6 % slower on MI355X): a
 * profiler sees that many dispatches per call. */
size_t glx_reduce_segment_bytes(void);

/* Split every peer copy of algorithms created afterwards over k streams per
 * destination (k DMA engines feeding one link; parts >= 1 MiB).  Default 1,
 * (every rank's process alike). */
int glx_set_copy_split(int k);
/* Host-memory endpoints: a pageable buffer is staged through a pinned mirror
 * of its size (the reference's CudaHostWorkspace, gloo/cuda_workspace.h:20);
 * above `bytes` (0: no limit, the default), or when the runtime cannot pin a
 * mirror that large, through an 8 MiB pinned bounce block instead, piece by
 * piece (slower, same result).  For algorithms created afterwards. */
int glx_set_pinned_mirror_limit(size_t bytes);
/* How peer copies are made by algorithms created afterwards: engine 0 =
 * hipMemcpyPeerAsync (DMA copy engines, default), 1 = a copy kernel storing
 * into the peer's memory over xGMI, with `blocks` workgroups (<= 0: keep).
 * Default 0. */
int glx_set_copy_engine(int engine, int blocks);
/* Engine of the mesh schedule (ring_chunked's result over all links) for
 * algorithms created afterwards, when device-driven engines are available
 * (ranks on distinct devices or processes, P <= 8): GLX_ENGINE_TWOSHOT (one
 * device-driven kernel per rank, default) or GLX_ENGINE_STEPS (host-issued
 * copies and fold kernels). */
int glx_set_mesh_engine(int engine);
/* Device-driven engines for algorithms created afterwards (initially from
 * GLOO_AMD_DEVICE_ENGINES=auto|off|on|shared):
 *   GLX_DEVICE_ENGINES_AUTO (default): when every rank has a GPU of its own.
 *     Ranks sharing a GPU run host-issued steps: their device engines wait
 *     for each other while holding the GPU's CUs, so other work queued ahead
 *     of one rank's collective can be starved until the timeout.
 *   GLX_DEVICE_ENGINES_SHARED: also processes sharing a GPU while
 *     ranks x (queues + 1) <= 20, queues = the largest GPU_MAX_HW_QUEUES any
 *     rank published (never threads sharing one device) -- for callers that
 *     queue no other GPU work ahead of a collective on the shared GPU.
 *   GLX_DEVICE_ENGINES_ON: always (the caller guarantees the ranks' kernels
 *     run concurrently).  GLX_DEVICE_ENGINES_OFF: never.
 * Every rank must use the same mode (a mismatch fails at the first run with
 * "schedules disagree"). */
#define GLX_DEVICE_ENGINES_AUTO (-1)
#define GLX_DEVICE_ENGINES_OFF 0
#define GLX_DEVICE_ENGINES_ON 1
#define GLX_DEVICE_ENGINES_SHARED 2
int glx_set_device_engines(int mode);
/* The current mode (GLX_DEVICE_ENGINES_*). */
int glx_get_device_engines(void);
/* The rule glx_set_device_engines' modes apply, for `ranks` ranks of which
 * at most `ranks_per_device` share one GPU (`threads_share_device`: two
 * ranks of one process on one GPU), with the largest GPU_MAX_HW_QUEUES any
 * rank's process uses: 1 = device engines, 0 = host-issued steps, -1 =
 * invalid argument.  No GPU needed. */
int glx_device_engines_rule(int mode, int ranks, int ranks_per_device, int threads_share_device,
                            int max_hw_queues);
/* Engine of the ring, halving-doubling, bcube and function-style ring
 * schedules for algorithms created afterwards, when device-driven engines
 * are available: -1 = automatic (default: the plan kernel -- at every size
 * with one rank per GPU, up to 32 MiB per rank when ranks share a GPU,
 * host-issued steps above), GLX_ENGINE_DEVSTEPS (the plan kernel),
 * GLX_ENGINE_STEPS (host-issued steps) or GLX_ENGINE_DMASTEPS (the
 * host-issued program -- hipMemcpyPeerAsync on side streams, reduce kernels --
 * with its hand-offs made on the GPU; chosen whenever it can run: not for rank
 * threads sharing a device, not under device-engine mode "off"). */
int glx_set_steps_engine(int engine);
/* Cache policy of the plan kernel's own loads and stores for algorithms
 * created afterwards: -1 automatic (default: plain, except nontemporal loads
 * and write-through (sc1) stores -- the reduce kernel's policy -- for the
 * ring's programs under the system-scope flag sync, whose per-step release
 * then finds nothing dirty to write back), 0 plain, 1 nontemporal and
 * write-through for every program.  The one-shot and two-shot kernels are
 * always plain.  Env GLOO_AMD_ENGINE_STREAMS=fast|plain. */
int glx_set_engine_streams(int fast);

/* Release / acquire around the device engines' flag words (one-shot,
 * two-shot, plan kernel) for algorithms created afterwards.  Everything a
 * flag publishes is stored into the receiver's landing slot, uncached device
 * memory that no L2 holds.  0 = system scope: before every flag the XCD's
 * whole L2 is written back (buffer_wbl2 sc0 sc1), after every wait it is
 * invalidated (buffer_inv sc0 sc1); 1 = narrow: the stores are completed
 * (s_waitcnt vmcnt(0)) before a flag and the CU's L1 invalidated after a wait
 * (agent scope); -1 = automatic (default: narrow).  Env
 * GLOO_AMD_SYNC=system|narrow.
 * Every rank may choose independently (the protocol is the same).
 * TEST ONLY, deliberately broken positive controls for the suite's stale-data
 * checks (results may be wrong; never for use): 2 = narrow without the
 * consumer's acquire, 3 = narrow without the producer's store-completion
 * wait, 4 = neither, with plain (write-back) stores into peers' slots, 5 =
 * narrow with every engine's landing slots in cached memory.  Env
 * GLOO_AMD_SYNC=unsafe_noacquire|unsafe_norelease|unsafe_test|unsafe_cached. */
int glx_set_device_sync(int mode);

/* Number of visible HIP devices (0 when no GPU). */
int glx_device_count(int* count);

/* ---- rendezvous stores (gloo/rendezvous/store.h) ----------------------- */
typedef struct glx_store glx_store;

/* In-process store shared by thread-ranks: gloo/rendezvous/hash_store.h:20. */
glx_store* glx_hash_store_create(void);
/* Directory-backed store for ranks in separate processes on one node:
 * gloo/rendezvous/file_store.h:19. */
glx_store* glx_file_store_create(const char* path);
/* Key prefixing wrapper: gloo/rendezvous/prefix_store.h. */
glx_store* glx_prefix_store_create(const char* prefix, glx_store* base);
/* Store implemented by the caller (e.g. a torch.distributed TCPStore from
 * Python, or gloo's own context in integration/gloo/hip_allreduce.h).  set:
 * store value.  get: copy the value of an EXISTING key into buf (cap bytes),
 * return its full length, -1 if the key is absent (the caller polls again
 * until its timeout), or -2 if it is absent and never will be (the wait fails
 * at once with GLX_ERR_IO). */
typedef int (*glx_store_set_fn)(void* user, const char* key, const void* data,
                                size_t len);
typedef int64_t (*glx_store_get_fn)(void* user, const char* key, void* buf,
                                    size_t cap);
glx_store* glx_callback_store_create(glx_store_set_fn set_fn,
                                     glx_store_get_fn get_fn, void* user);
void glx_store_destroy(glx_store* store);
int glx_store_set(glx_store* store, const char* key, const void* data,
                  size_t len);
/* Blocks until key exists (or timeout_ms elapses -> GLX_ERR_TIMEOUT).
 * Writes min(len, cap) bytes to buf and the full length to *len_out. */
int glx_store_get(glx_store* store, const char* key, void* buf, size_t cap,
                  size_t* len_out, int64_t timeout_ms);

/* ---- context (gloo/context.h:26-58, gloo/rendezvous/context.h:25-35) --- */
typedef struct glx_context glx_context;

/* A rank of `size` ranks bound to HIP device `device` (-1 = current).
 * Replaces gloo::rendezvous::Context(rank, size) + transport::Device. */
glx_context* glx_context_create(int rank, int size, int device);
void glx_context_destroy(glx_context* ctx);
/* Publish this rank's xGMI endpoint, wait for every peer's, map the peers'
 * control blocks.  Replaces rendezvous::Context::connectFullMesh(Store&,
 * shared_ptr<Device>&) -- gloo/rendezvous/context.cc:43-113. */
int glx_context_connect_full_mesh(glx_context* ctx, glx_store* store);
int glx_context_rank(glx_context* ctx);
int glx_context_size(glx_context* ctx);
int glx_context_device(glx_context* ctx);
/* gloo::Context::setTimeout/getTimeout (gloo/context.h:50-53); default 30 s
 * (gloo/context.cc:18). */
int glx_context_set_timeout(glx_context* ctx, int64_t timeout_ms);
/* gloo::Context::base (gloo/context.h:33): ranks per group of the
 * GLX_ALGO_BCUBE algorithms created afterwards (default 2, >= 2). */
int glx_context_set_base(glx_context* ctx, int base);
int64_t glx_context_get_timeout(glx_context* ctx);
/* gloo::Context::nextSlot(numToSkip), gloo/context.cc:49-54. */
int glx_context_next_slot(glx_context* ctx, int num_to_skip);

/* ---- allreduce algorithms (gloo/algorithm.h:20-38) ---------------------- */
typedef struct glx_algorithm glx_algorithm;

/* HipAllreduceRingChunked: gloo::AllreduceRingChunked<T>
 * (gloo/allreduce_ring_chunked.h:22-26) on device buffers, constructor shaped
 * like CudaAllreduceRingChunked<T>(context, ptrs, count, streams)
 * (gloo/cuda_allreduce_ring_chunked.h:22-26).  ptrs: nptrs device pointers of
 * this rank (same device), count elements each.  streams: 0 or nptrs
 * hipStream_t; with streams the op is asynchronous w.r.t. the host beyond
 * the last exchange and the outputs are valid once streams[0] completes;
 * without, outputs are valid when run() returns (docs/cuda.md:9-11). */
glx_algorithm* glx_allreduce_ring_chunked_create(glx_context* ctx,
                                                 void* const* ptrs, int nptrs,
                                                 int count, int dtype, int op,
                                                 const glx_stream_t* streams,
                                                 int nstreams);
/* HipAllreduceHalvingDoubling: gloo::AllreduceHalvingDoubling<T>
 * (gloo/allreduce_halving_doubling.h:67-71); ctor shaped like
 * CudaAllreduceHalvingDoubling (gloo/cuda_allreduce_halving_doubling.h:25-30). */
glx_algorithm* glx_allreduce_halving_doubling_create(
    glx_context* ctx, void* const* ptrs, int nptrs, int count, int dtype, int op,
    const glx_stream_t* streams, int nstreams);
/* Schedules.  GLX_ALGO_RING_CHUNKED_MESH computes exactly what
 * AllreduceRingChunked computes -- same chunking, same per-chunk reduction
 * chain and operand order, bit-identical results -- but moves the data over
 * every peer link at once: each rank receives its chunk pair's operands from
 * all peers (one xGMI link each), evaluates the ring's chain in one fold
 * kernel, and sends the result to every peer. */
enum glx_algo {
  GLX_ALGO_RING_CHUNKED = 0,
  GLX_ALGO_HALVING_DOUBLING = 1,
  GLX_ALGO_RING_CHUNKED_MESH = 2,
  /* schedules of glx_allreduce (plan introspection only) */
  GLX_ALGO_FN_RING = 3,
  GLX_ALGO_FN_RING_MESH = 4,
  GLX_ALGO_FN_BCUBE = 5,
  /* one round for small buffers: every rank receives every peer's whole
   * buffer and folds every chunk in the ring's own order (bit-identical) */
  GLX_ALGO_RING_CHUNKED_REPL = 6,
  GLX_ALGO_FN_RING_REPL = 7,
  /* AllreduceRingChunked's result, data movement chosen at creation:
   * replicated up to 256 KiB per rank (16 / 2 / 1 MiB at P = 2 / <= 4 / <= 8
   * on the device-driven engines), mesh above */
  GLX_ALGO_RING_CHUNKED_AUTO = 8,
  /* gloo::AllreduceRing<T> (gloo/allreduce_ring.h:20): each rank's left fold
   * of the ranks' buffers starting from its own, r, r-1, ..., r-P+1 (float
   * results may differ between ranks, as in the reference); whole buffers,
   * one round over every link instead of P-1 forwarding rounds */
  GLX_ALGO_RING = 9,
  /* gloo::AllreduceBcube<T> (gloo/allreduce_bcube.h:256): groups of the
   * context's base ranks (glx_context_set_base, gloo::Context::base) */
  GLX_ALGO_BCUBE = 10,
  /* gloo::AllreduceLocal<T> (gloo/allreduce_local.h:17): this rank's
   * pointers folded into ptrs[0] and broadcast back; no exchange */
  GLX_ALGO_LOCAL = 11
};
glx_algorithm* glx_allreduce_create(glx_context* ctx, int algo, void* const* ptrs,
                                    int nptrs, int count, int dtype, int op,
                                    const glx_stream_t* streams, int nstreams);

/* Buffers may be device memory or host memory (pageable or pinned; all
 * pointers of one algorithm alike).  Host buffers are staged through device
 * copies: H2D in the order the schedule first touches each piece, every step
 * waiting only for its own range, and each range copied back as soon as its
 * final value is written.  Pinned buffers are copied
 * directly; pageable ones through a pinned workspace mirror (the caller's
 * pages are never registered with the runtime). */

/* ---- function-style collective ---------------------------------------- */
/* gloo::AllreduceOptions::Algorithm (gloo/allreduce.h:38-42), plus
 * GLX_ALLREDUCE_RING_MESH: RING's exact result (same chunk ownership, same
 * reduction chain and operand order) with every owner folding its chunk from
 * all peers at once over all xGMI links. */
enum glx_allreduce_algorithm {
  GLX_ALLREDUCE_UNSPECIFIED = 0,
  GLX_ALLREDUCE_RING = 1,
  GLX_ALLREDUCE_BCUBE = 2,
  GLX_ALLREDUCE_RING_MESH = 3,
  GLX_ALLREDUCE_RING_REPLICATED = 4  /* RING's result in one round (small buffers) */
};
/* gloo::allreduce(const AllreduceOptions&) (gloo/allreduce.cc:97-146,
 * gloo/allreduce.h:89-193) on device buffers.  The reduce function is one of
 * the gloo/math.h templates for `dtype`, selected by `op` (the device cannot
 * run a host std::function).
 *   inputs/num_inputs   opts.setInputs (may be 0: out[0] is the input and
 *                       out[1..] are folded into it)
 *   outputs/num_outputs opts.setOutputs (>= 1; all get the result)
 *   elements            element count of every buffer
 *   tag                 opts.setTag: concurrent operations need distinct tags
 *   max_segment_size    opts.setMaxSegmentSize in bytes (0: 1 MiB default);
 *                       it fixes which rank reduces which elements, hence
 *                       the result bits, exactly as in the reference
 *   timeout_ms          opts.setTimeout (<= 0: the context's timeout)
 *   stream              NULL: the call returns with the outputs complete;
 *                       else the work is ordered on `stream`.
 * Every rank calls with the same algorithm/dtype/op/elements/tag/
 * max_segment_size.  The first call with a given combination sets up and
 * exchanges receive buffers with the peers (once; later calls reuse them).
 * UNSPECIFIED computes RING's result with the data movement chosen per
 * size (replicated up to 256 KiB per rank -- 16 / 2 / 1 MiB at P = 2 /
 * <= 4 / <= 8 on the device-driven engines -- mesh above). */
int glx_allreduce(glx_context* ctx, int algorithm, int dtype, int op,
                  void* const* inputs, int num_inputs, void* const* outputs,
                  int num_outputs, size_t elements, uint32_t tag,
                  size_t max_segment_size, int64_t timeout_ms, glx_stream_t stream);

/* A caller's reduction function c = f(a, b) over n elements -- the
 * reference's AllreduceOptions::Func (gloo/allreduce.h:36,69,171), which may
 * be any host std::function (bitwise ops, user types, non-commutative ops);
 * `user` is passed through. */
typedef int (*glx_reduce_fn)(void* user, void* c, const void* a, const void* b, size_t n);
/* It returns 0, or nonzero when it failed (a C++ wrapper caught an exception
 * it must not unwind through this ABI): the call then stops at once with
 * GLX_ERR_INVALID on that rank and reduces nothing more -- its peers wait
 * for messages that never come and fail with GLX_ERR_TIMEOUT, as the
 * reference's ranks do when one rank's Func throws. */
/* gloo::allreduce(opts) with such a function, on HOST buffers: the same step
 * program as glx_allreduce (RING, or BCUBE; UNSPECIFIED = RING) run on the
 * host -- messages through shared memory, every reduction a call of `fn` in
 * the reference's order and operand order (gloo/allreduce.cc:44-95,
 * :286-297, :580-596), so the result bits are the reference's for any
 * function.  element_size: bytes per element (any, as opts.elementSize).
 * Device buffers are refused (GLX_ERR_INVALID): a device cannot run a host
 * function; use glx_allreduce with sum/product/max/min there.  Every rank
 * must make the same sequence of calls (as in the reference). */
int glx_allreduce_host_fn(glx_context* ctx, int algorithm, size_t element_size,
                          glx_reduce_fn fn, void* user, void* const* inputs, int num_inputs,
                          void* const* outputs, int num_outputs, size_t elements, uint32_t tag,
                          size_t max_segment_size, int64_t timeout_ms);

/* The class algorithms with a ReductionFunction<T> of type CUSTOM
 * (gloo/algorithm.h:56,58-83: Function(T* x, const T* y, n), x = f(x, y) in
 * place) -- replaces gloo::AllreduceRingChunked<T>(context, ptrs, count, fn)
 * (gloo/allreduce_ring_chunked.h:22-26) and gloo::AllreduceHalvingDoubling<T>
 * (gloo/allreduce_halving_doubling.h:67-81) with such an fn.  A device cannot
 * run a host function, so the buffers must be HOST memory: the algorithm's
 * program runs on the host (shared-memory messages, the context's counters),
 * calling fn(user, x, x, y, n) exactly where the reference calls fn_->call(x,
 * y, n) -- the local fold of ptrs[1..] into ptrs[0], every reduce-scatter
 * step -- so the result bits are the reference's for any function.  algo:
 * GLX_ALGO_RING_CHUNKED (any of its schedules: the ring's program) or
 * GLX_ALGO_HALVING_DOUBLING.  Created in the same order on every rank (it
 * takes a context slot, like the others); glx_algorithm_run runs it;
 * run_fed / feed / done_ranges / record are not available (GLX_ERR_ENFORCE),
 * glx_algorithm_engine returns GLX_ENGINE_HOSTFN.  NULL on error. */
glx_algorithm* glx_allreduce_create_host_fn(glx_context* ctx, int algo, void* const* ptrs,
                                            int nptrs, int count, size_t element_size,
                                            glx_reduce_fn fn, void* user);

/* Algorithm::run() (gloo/algorithm.h:26).  With streams and the
 * GLX_ENGINE_DMASTEPS engine the call only enqueues (copies, reduce and flag
 * kernels on streams[0] and the algorithm's copy streams; message numbers
 * are the host's, so it is not graph-capturable).  With streams and a
 * one-kernel device engine (GLX_ENGINE_ONESHOT, _TWOSHOT, _DEVSTEPS) the
 * call only enqueues one kernel on streams[0] and can be captured into a HIP graph
 * (hipStreamBeginCapture on streams[0]) after one eager run: the kernels
 * keep their run count / epoch on the device, so every replay is one more
 * run on that rank, in sequence with eager runs.  Runs and replays of one
 * algorithm must be stream-ordered (replay on streams[0], or make the
 * replay's stream wait for the previous run): a launch that starts while
 * the previous one is still running is detected on the device, does
 * nothing, and the next call returns GLX_ERR_ENFORCE ("... still running");
 * the algorithm is unusable afterwards.  Every replay must have been issued
 * before the algorithm is destroyed (its destructor waits for every
 * started launch). */
int glx_algorithm_run(glx_algorithm* alg);

/* Host-memory endpoint fed from a transport.  The reference receives socket
 * bytes into a registered host buffer (gloo/transport/tcp/pair.cc:385-451)
 * and reduces once a message is whole; here the algorithm (created on ONE
 * host buffer) is run while that buffer is still filling:
 *   glx_algorithm_run_fed  -- run() whose H2D copies wait for feeds: each
 *                             8 MiB piece is copied as soon as feeds cover
 *                             it, every step waits only for the pieces of
 *                             its own range.  Blocks until the result is
 *                             back in host memory; GLX_ERR_TIMEOUT if some
 *                             piece is never fed within the timeout.
 *   glx_algorithm_feed     -- elements [off, off+len) of the buffer hold
 *                             their data now.  Any thread, before (counts
 *                             for the next run) or during run_fed.
 *   glx_algorithm_done_ranges -- element ranges {off, len} whose results are
 *                             in host memory already, in completion order
 *                             (the ring returns chunk after chunk), for a
 *                             caller that streams results back out; writes at
 *                             most cap pairs and returns how many ranges are
 *                             done (more than cap when more completed; call
 *                             again with a larger buffer), or -1.
 */
int glx_algorithm_run_fed(glx_algorithm* alg);
int glx_algorithm_feed(glx_algorithm* alg, int64_t off, int64_t len);
int64_t glx_algorithm_done_ranges(glx_algorithm* alg, int64_t* out, int64_t cap);
/* Number of bytes moved over the peer links by this rank in one run(). */
int64_t glx_algorithm_bytes_sent(glx_algorithm* alg);
/* How run() executes: GLX_ENGINE_STEPS = the schedule's steps issued by the
 * host (copies, reduce kernels, control-block counters); GLX_ENGINE_ONESHOT =
 * the replicated schedule as one device-driven kernel per rank (small
 * buffers); GLX_ENGINE_TWOSHOT = the mesh schedule as one device-driven
 * kernel per rank.  Device-driven engines need the ranks on distinct devices
 * or processes.  Results are identical. */
#define GLX_ENGINE_STEPS 0
#define GLX_ENGINE_ONESHOT 1
#define GLX_ENGINE_TWOSHOT 2
/* GLX_ENGINE_DEVSTEPS = any other schedule (ring, halving-doubling, bcube,
 * function-style ring) run as ONE device-driven kernel per rank that walks
 * the schedule's step program (the plan kernel). */
#define GLX_ENGINE_DEVSTEPS 3
/* GLX_ENGINE_DMASTEPS = the host-issued steps' copies (hipMemcpyPeerAsync on
 * per-peer side streams) and reduce launches, enqueued by run() in one pass:
 * every wait between them -- a copy for the receiver's credit and for the
 * reduce that produced its chunk, a reduce for its message -- is a one-wave
 * flag kernel on the waiting stream, every counter a flag word written by
 * one, instead of the host's progress loop (glx_set_steps_engine). */
#define GLX_ENGINE_DMASTEPS 4
/* GLX_ENGINE_HOSTFN = a class algorithm with a CUSTOM reduction function on
 * host buffers (glx_allreduce_create_host_fn): its program run on the host. */
#define GLX_ENGINE_HOSTFN 5
int glx_algorithm_engine(glx_algorithm* alg);
/* 1 when the algorithm's plan kernel runs nontemporal loads and write-through
 * stores (glx_set_engine_streams), else 0. */
int glx_algorithm_fast_streams(glx_algorithm* alg);
/* Release / acquire its device engine runs around flag words: 1 narrow, 0
 * system scope, -1 host-issued steps (glx_set_device_sync). */
int glx_algorithm_sync(glx_algorithm* alg);
/* How this algorithm's messages actually moved since it was created, as 6
 * int64 written to out (cap >= 6): {peer_copies (hipMemcpyPeerAsync, the DMA
 * engines over xGMI), device_copies (hipMemcpyAsync: peers on the same device,
 * or a peer whose IPC mapping hipMemcpyPeerAsync refused -- logged once),
 * kernel_copies (copy kernel storing into the peer's memory),
 * device_kernels (launches of a device-driven engine, whose kernels store into
 * the peers' memory themselves), bytes (of the copies), host_folds (local
 * multi-pointer reduces done on the host: host buffers below
 * kOnDeviceThreshold = 256 KiB, gloo/algorithm.cc:16), done_events (event
 * records after a run's work: none for run() on a device engine, whose stream
 * is fixed -- each record costs the stream microseconds per call),
 * flag_kernels (GLX_ENGINE_DMASTEPS: flag-op launches, the hand-offs)}.  The
 * peer-copy analog of the reference's transport byte counters and of its
 * intra-process peer copies (gloo/cuda_collectives_native.h:205-276).  Fills
 * min(cap, 8) fields (cap >= 6); returns that count, or -1. */
int glx_algorithm_transport_stats(glx_algorithm* alg, int64_t* out, int cap);
void glx_algorithm_destroy(glx_algorithm* alg);

/* IPC imports this context has made and checked (every imported shared
 * block's canary word is verified before use), and how many of them the
 * runtime mapped at the base of the exporter's allocation rather than at the
 * exported pointer (corrected with the published offset).  Returns GLX_OK. */
int glx_context_ipc_stats(glx_context* ctx, int64_t* imports, int64_t* base_fixups);

/* What this rank learnt about peer `peer`'s GPU at connect (the link the
 * transport will use; the reference's analog is the PCI distance it reads,
 * gloo/common/linux.cc:126).  info[5] =
 *   {device ordinal of the peer's GPU in this process (-1 unknown),
 *    1 if it is this rank's own GPU,
 *    hipDeviceCanAccessPeer (-1: same GPU / not asked),
 *    hipDevP2PAttrNativeAtomicSupported of the link (-1: same GPU / not asked),
 *    1 if this rank's kernels write peers' flags with stores (some link lacks
 *      atomics, or GLOO_AMD_FLAG_WRITE=store)}. */
int glx_context_peer_info(glx_context* ctx, int peer, int* info);

/* ---- measured link ceilings ----------------------------------
 * A receive block of (P-1) x `bytes` per rank, exported and imported
 * through the context's own canary-checked IPC path (the one every engine
 * uses) and uncached like the engines' landing regions.  create is
 * collective (every rank, same bytes, in the same order as its other
 * creations).  run writes `reps` rounds, pattern 0 = ring (`bytes` to
 * rank+1) or 1 = mesh (`bytes` to every peer: the same volume on each of the
 * P-1 links), engine 0 = hipMemcpyPeerAsync (one stream per
 * destination) or 1 = the copy kernel (`blocks` workgroups shared by the
 * destinations), and returns this rank's seconds and the bytes one round
 * puts on its busiest link.  run is NOT synchronising: callers barrier
 * before it (so every rank sends at once) and take the max over ranks;
 * destroy only after a barrier that follows every rank's last run. */
typedef struct glx_link_probe glx_link_probe;
glx_link_probe* glx_link_probe_create(glx_context* ctx, size_t bytes);
int glx_link_probe_run(glx_link_probe* probe, int pattern, int engine, int blocks, int reps,
                       double* seconds, size_t* link_bytes);
void glx_link_probe_destroy(glx_link_probe* probe);

/* ---- events (gloo::CudaStream's record / wait, gloo/cuda.h:40-120) -------
 * A caller that gives an algorithm streams gets its outputs valid once
 * streams[0] reaches the end of run(); these order other streams (or the
 * host) after that point without synchronising the device. */
typedef void* glx_event_t; /* a hipEvent_t */
/* hipEventCreateWithFlags(hipEventDisableTiming). */
int glx_event_create(glx_event_t* ev);
int glx_event_destroy(glx_event_t ev);
/* Record on `stream` (NULL = the legacy default stream). */
int glx_event_record(glx_event_t ev, glx_stream_t stream);
/* GLX_OK when everything recorded before it has completed, GLX_NOT_READY
 * while it is pending, else an error code. */
#define GLX_NOT_READY 7
int glx_event_query(glx_event_t ev);
/* Make `stream` wait for the event on the device (hipStreamWaitEvent); with
 * stream NULL the calling thread blocks until it completes. */
int glx_event_wait(glx_event_t ev, glx_stream_t stream);
/* Record `ev` where run() left the algorithm's work: the end of its last
 * call on its compute stream (streams[0] when given, else the internal
 * stream, on which a run without streams has already completed). */
int glx_algorithm_record(glx_algorithm* alg, glx_event_t ev);

/* ---- schedule introspection (host logic; no GPU needed) ----------------- */
/* The per-rank step program an algorithm executes.  Each step is 8 int64:
 * {kind, peer, channel, off, len, boff, dst_off, flags}; kinds: 0 SEND,
 * 1 RECV, 2 REDUCE, 3 COPY, 4 RELEASE, 5 FOLD.  algo: glx_algo.  Returns the
 * number of steps (writes at most cap) or -1.  *scratch_elems receives the
 * per-rank receive-buffer size. */
int64_t glx_plan(int algo, int rank, int size, int64_t count, int64_t* steps,
                 int64_t cap, int64_t* scratch_elems);
/* Geometry the device-driven engines derive from a replicated (one-shot)
 * or mesh (two-shot) schedule, for host-side replay in tests: writes
 * [G, slice, maxLen, njobs, jobOff[8], jobLen[8], chain[8][8], rangeOff[8],
 * rangeLen[8], myChain[8]] (up to cap values) and returns their number, or
 * -1 (glx_last_error()).  max_slices bounds G (the launch uses the kernel's
 * resident capacity per rank). */
int64_t glx_device_layout(int algo, int rank, int size, int64_t count, int esize,
                          int64_t max_slices, int64_t* out, int64_t cap);
/* The plan kernel's bookkeeping for one rank's step program with G
 * workgroups (host logic): segment bounds (written to bounds, *nbounds =
 * their number), info = {slice, safe, slots} (3 int64: elements per
 * workgroup slice; 1 if no landing region is shared by two workgroups across
 * messages, else the executor keeps host-issued steps; landing slots per
 * channel, 1 or 2: message n lands in slot (n-1) % slots), and per step 12
 * int64 {channel, seg0, seg1, seq, perRun, fuse, rseq, rperRun, keep, pre,
 * pre0, pre1} (channel =
 * out-channel index for SEND, in-channel index for RECV/RELEASE, -1
 * otherwise; seq = message number within a run, 1-based; fuse = for a
 * REDUCE/COPY the index of the SEND of the same range the kernel does in the
 * same pass (reduce-and-forward, with 2 slots only), for that SEND the index
 * of the step it is done in, else -1; rseq/rperRun = for a REDUCE/COPY the
 * number of the message it reads; keep = 0 for a fused REDUCE whose result
 * is overwritten whole by a later COPY before anything reads it -- the
 * kernel then stores it only into the peer's slot -- else 1; for a partial
 * one, of its overlap; pre / pre0 / pre1 = partial reduce-and-forward, where
 * the SEND after a REDUCE / COPY overlaps its range without equalling it: the
 * REDUCE / COPY names the SEND and stores the overlap's segments [pre0, pre1)
 * into its slot, the SEND names the step and stores only its other segments;
 * -1 / 0 / 0 otherwise, plan.h StepSync).  `cap` counts int64 slots of
 * `steps` (GLX_PLAN_SYNC_WIDTH per step; a step is written only if it fits
 * whole).  Returns the number of steps or -1. */
#define GLX_PLAN_SYNC_WIDTH 12
int64_t glx_plan_sync(int algo, int rank, int size, int64_t count, int esize,
                      int64_t max_segment_bytes, int64_t min_piece_bytes, int G,
                      int64_t* bounds, int64_t bounds_cap, int64_t* nbounds, int64_t* info,
                      int64_t* steps, int64_t cap);
/* Sources of FOLD step number `fold` (its boff field): region offsets, -1 =
 * the rank's own buffer.  Returns the count (writes at most cap) or -1. */
int64_t glx_plan_fold(int algo, int rank, int size, int64_t count, int64_t fold,
                      int64_t* srcs, int64_t cap);
/* The same for the function-style schedules, whose geometry also depends on
 * the element size, opts.maxSegmentSize (0: default) and the device piece
 * size of the ring (min_piece_bytes; 0: the reference's own segments). */
int64_t glx_plan_ex(int algo, int rank, int size, int64_t count, int esize,
                    int64_t max_segment_bytes, int64_t min_piece_bytes, int64_t* steps,
                    int64_t cap, int64_t* scratch_elems);
/* AllreduceBcube's step program for a given base (glx_plan's layout). */
int64_t glx_plan_bcube(int rank, int size, int64_t count, int base, int64_t* steps, int64_t cap,
                       int64_t* scratch_elems);
int64_t glx_plan_fold_ex(int algo, int rank, int size, int64_t count, int esize,
                         int64_t max_segment_bytes, int64_t min_piece_bytes, int64_t fold,
                         int64_t* srcs, int64_t cap);
/* Host-memory staging derived from a plan (the algorithm's buffers are in
 * host memory): h2d receives {off, len} pairs in issue order (returns their
 * number, writes at most h2d_cap); d2h receives {step, off, len} triples --
 * a range copied back right after step `step` writes its final value, step
 * -1 for ranges no step writes -- (*n_d2h = their number, writes at most
 * d2h_cap).  Pieces are at most max_piece elements. */
int64_t glx_plan_stage(int algo, int rank, int size, int64_t count, int esize,
                       int64_t max_piece, int64_t* h2d, int64_t h2d_cap, int64_t* d2h,
                       int64_t d2h_cap, int64_t* n_d2h);

#if defined(__GNUC__)
#pragma GCC visibility pop
#endif

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* GLOO_AMD_GLX_H_ */
