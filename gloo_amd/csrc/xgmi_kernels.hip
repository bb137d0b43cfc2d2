// xgmi_kernels.hip -- device-driven allreduce engines: a whole schedule as
// ONE kernel per rank, the ranks' kernels handing data to each other through
// IPC-mapped uncached device memory over xGMI and synchronising on flag
// words, with no host round trip between steps.  Two engines, both
// bit-identical to the reference's ring (same chunks, same per-element
// reduction chains, acc = op(newer rank's value, acc)):
//
//  one-shot (the replicated schedule, plan.h planRingChunkedReplicated /
//  planFnRingReplicated; small buffers).  Workgroup w of rank r:
//    1. push  slice w of r's buffer to every peer's landing slot [r];
//             system-scope release; flagOut[peer][r][w] = epoch
//    2. wait  one lane polls flagIn[k][w] >= epoch for every peer k
//    3. fold  slice w of every chunk along that chunk's chain, in place.
//
//  two-shot (the all-links mesh, plan.h planRingChunkedMesh /
//  planFnRingMesh; medium and large buffers).  Rank j owns range j.
//  Workgroup w of rank r:
//    1. push  slice w of every range j != r to owner j's RS slot [r]; flag A
//    2. fold  slice w of range r once every peer's A flag is up, along the
//             range's chain; the result goes to r's buffer AND to every
//             peer's AG slot [r] in the same pass; flag B
//    3. take  slice w of every range j != r from AG slot [j] once owner j's
//             B flag is up.
//
// Waits are bounded: a peer that never arrives sets *status (1 + its rank)
// and the workgroup exits, so every wave reaches the end.  Landing slots are
// double-buffered by epoch parity: a rank writes epoch e into a peer's slot
// only after its epoch e-1 kernel saw that peer's epoch e-1 flags, i.e. after
// the peer finished epoch e-2, the last reader of that parity.
//
// Slots use a "virtual buffer" layout: element i of range c lives at
// vbase + i*es with vbase = slot + (off_c*es mod 16) - off_c*es, so it has
// the 16-byte phase it has in a 16-byte-aligned user buffer and the body of
// every span runs on 16-byte vectors (an unaligned user buffer takes the
// scalar path on its own side; the slot layout never depends on it).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"
#include "elem_ops.h"
#include "kernels.h"

namespace glx {
namespace {

// [a, b) as scalar head [a, hs), 16-byte vectors [va, vb) (elements
// [hs, ts)) and scalar tail [ts, b); all scalar when the buffer is not
// 16-byte aligned or the span holds no whole vector.
struct Span {
  size_t a, b, hs, ts, va, vb;
  __device__ __forceinline__ size_t nedge() const { return (hs - a) + (b - ts); }
  __device__ __forceinline__ size_t edge(size_t t) const {
    return t < hs - a ? a + t : ts + (t - (hs - a));
  }
};

template <int V>
__device__ __forceinline__ Span split_span(size_t a, size_t b, bool aligned) {
  Span s{a, b, b, b, 0, 0};
  if (aligned) {
    const size_t va = (a + V - 1) / V, vb = b / V;
    if (va < vb) {
      s.va = va;
      s.vb = vb;
      s.hs = va * V;
      s.ts = vb * V;
    }
  }
  return s;
}

// Vector loads of the plan kernel's streams: FAST = nontemporal.  Stores:
// FAST = write-through through a buffer resource (WtStream, compiler-tracked).
// The one-shot and two-shot kernels always run plain.
template <bool FAST>
__device__ __forceinline__ v4u ldv(const v4u* p) {
  return ld16<FAST>(p);
}

// Store policies of a span's destination: plain, write-through at device
// scope (sc1: the plan kernel's fast streams into this rank's buffer), or
// write-through at system scope (sc0 sc1) -- every store into ANOTHER rank's
// landing slot.  Those slots are uncached memory, so even a plain store
// reaches it, but the narrow flag sync (kernels.h) relies on nothing of a
// handed-off message waiting in this XCD's L2: the system write-through makes
// that hold whatever memory type a peer's mapping gets.
enum StorePol : int { kStPlain = 0, kStLocalWt = 1, kStRemote = 2 };

template <int SP>
struct WtCache {
  static constexpr int aux = SP == kStRemote ? 17 : 16;  // sc0 sc1 | sc1 (gfx940 family)
};

// Stores of vectors [va, vb) of one workgroup's span.  The write-through
// resource is built at the span's first vector, not at the (virtual) buffer
// base: its 32-bit offsets then stay below the span's size whatever the
// buffer's, and the base is made wave-uniform (readfirstlane) so the resource
// lives in SGPRs instead of a per-store waterfall loop.
template <int SP>
struct VecOut {
  v4u* base;
  size_t origin;
  __amdgpu_buffer_rsrc_t r;
  __device__ __forceinline__ VecOut(void* b, size_t va)
      : base(reinterpret_cast<v4u*>(b)),
        origin(va),
        r(__builtin_amdgcn_make_buffer_rsrc(
            SP != kStPlain ? uniform_ptr(reinterpret_cast<v4u*>(b) + va) : b, 0, 0x7fffffff,
            0x00020000)) {}
  __device__ __forceinline__ void put(size_t i, v4u v) const {
    if (SP != kStPlain) {
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)((i - origin) * 16), 0,
                                             WtCache<SP>::aux);
    } else {
      base[i] = v;
    }
  }
};

template <int N> struct BitsOf;
template <> struct BitsOf<1> { using type = uint8_t; };
template <> struct BitsOf<2> { using type = uint16_t; };
template <> struct BitsOf<4> { using type = uint32_t; };
template <> struct BitsOf<8> { using type = uint64_t; };

// One element store with policy SP (the unaligned head / tail of a span):
// write-through stores are relaxed atomic stores at the matching scope,
// i.e. global_store_{byte,short,dword,dwordx2} sc1 / sc0 sc1.
template <int SP, typename S>
__device__ __forceinline__ void put1(S* p, S v) {
  if (SP == kStPlain) {
    *p = v;
  } else {
    using U = typename BitsOf<sizeof(S)>::type;
    U u;
    __builtin_memcpy(&u, &v, sizeof(S));
    if (SP == kStRemote) {
      __hip_atomic_store(reinterpret_cast<U*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      __hip_atomic_store(reinterpret_cast<U*>(p), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Copy [a, b) of src to dst (virtual-buffer pointers with equal phases):
// loads as FAST says, stores with policy SP.
template <typename S, bool FAST, int SP>
__device__ __forceinline__ void copy_span(S* dst, const S* src, size_t a, size_t b,
                                          bool aligned) {
  const Span sp = split_span<16 / sizeof(S)>(a, b, aligned);
  const size_t va = sp.va, vb = sp.vb;
  for (size_t t = threadIdx.x; t < sp.nedge(); t += kBlock) {
    const size_t i = sp.edge(t);
    put1<SP>(dst + i, src[i]);
  }
  const v4u* vs = reinterpret_cast<const v4u*>(src);
  const VecOut<SP> vd(dst, va);
  constexpr int U = 8;  // vectors in flight per lane
  size_t i = va + threadIdx.x;
  for (; i + (U - 1) * kBlock < vb; i += U * kBlock) {
    v4u x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = ldv<FAST>(vs + i + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; u++) vd.put(i + u * kBlock, x[u]);
  }
  for (; i < vb; i += kBlock) vd.put(i, ldv<FAST>(vs + i));
}

// Copy [a, b) of src to every dsts[d] for d < n (one load, n stores):
// dsts[0 .. FIRST_REMOTE-1] are this rank's (policy LSP), the rest other
// ranks' landing slots (system write-through).
template <typename S, bool FAST, int LSP, int FIRST_REMOTE, int MAXD = kOsMaxRanks - 1,
          int RSP = kStRemote>
__device__ __forceinline__ void scatter_span(char* const* dsts, int n, const S* src, size_t a,
                                             size_t b, bool aligned) {
  const Span sp = split_span<16 / sizeof(S)>(a, b, aligned);
  const size_t va = sp.va, vb = sp.vb;
  for (size_t t = threadIdx.x; t < sp.nedge(); t += kBlock) {
    const size_t i = sp.edge(t);
    const S x = src[i];
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < n) {
        if (d >= FIRST_REMOTE) {
          put1<RSP>(reinterpret_cast<S*>(dsts[d]) + i, x);
        } else {
          put1<LSP>(reinterpret_cast<S*>(dsts[d]) + i, x);
        }
      }
    }
  }
  const v4u* vs = reinterpret_cast<const v4u*>(src);
  constexpr int U = MAXD <= 2 ? 4 : 2;  // vectors in flight per lane
  size_t i = va + threadIdx.x;
  for (; i + (U - 1) * kBlock < vb; i += U * kBlock) {
    v4u x[U];
#pragma unroll
    for (int u = 0; u < U; u++) x[u] = ldv<FAST>(vs + i + u * kBlock);
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < n) {
        if (d >= FIRST_REMOTE) {
          const VecOut<RSP> o(dsts[d], va);
#pragma unroll
          for (int u = 0; u < U; u++) o.put(i + u * kBlock, x[u]);
        } else {
          const VecOut<LSP> o(dsts[d], va);
#pragma unroll
          for (int u = 0; u < U; u++) o.put(i + u * kBlock, x[u]);
        }
      }
    }
  }
  for (; i < vb; i += kBlock) {
    const v4u x = ldv<FAST>(vs + i);
#pragma unroll
    for (int d = 0; d < MAXD; d++) {
      if (d < n) {
        if (d >= FIRST_REMOTE) {
          VecOut<RSP>(dsts[d], va).put(i, x);
        } else {
          VecOut<LSP>(dsts[d], va).put(i, x);
        }
      }
    }
  }
}

// [a, b) of dst = fold of srcs[0..P-1]: acc = s0, then acc = op(s_k, acc)
// (the ring's chain: the newer rank's value is the in-place destination)
// or, LEFT, acc = op(acc, s_k) (a left fold, out = op(out, peer)).
// The result also goes to every outs[d], d < nout.
// dst is this rank's buffer (stores as FAST says; none when !KEEP: the
// result goes to the outs only); outs are other ranks' landing slots
// (system write-through).
template <typename T, int OP, bool FAST, bool LEFT = false, int MAXK = kOsMaxRanks,
          bool KEEP = true, int RSP = kStRemote>
__device__ __forceinline__ void fold_span(typename Elem<T, OP>::S* dst,
                                          const typename Elem<T, OP>::S* const* srcs, int P,
                                          char* const* outs, int nout, size_t a, size_t b,
                                          bool aligned) {
  constexpr int LSP = FAST ? kStLocalWt : kStPlain;
  using E = Elem<T, OP>;
  using S = typename E::S;
  const Span sp = split_span<16 / sizeof(S)>(a, b, aligned);
  const size_t va = sp.va, vb = sp.vb;
  for (size_t t = threadIdx.x; t < sp.nedge(); t += kBlock) {
    const size_t i = sp.edge(t);
    S y[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; k++) {
      if (k < P) y[k] = srcs[k][i];
    }
    S acc = y[0];
#pragma unroll
    for (int k = 1; k < MAXK; k++) {
      if (k < P) acc = LEFT ? E::apply(acc, y[k]) : E::apply(y[k], acc);
    }
    if (KEEP) put1<LSP>(dst + i, acc);
#pragma unroll
    for (int d = 0; d < MAXK - 1; d++) {
      if (d < nout) put1<RSP>(reinterpret_cast<S*>(outs[d]) + i, acc);
    }
  }
  // U vectors per lane, all U*P loads in flight before the chains: 4 for
  // the 2-source folds (the ring's reduce-and-forward), 2 for wider ones
  // (registers); none for 1-byte types (16 lanes of byte ops per vector
  // already fill the registers)
  constexpr int U = MAXK <= 2 ? 4 : 2;
  size_t v = va + threadIdx.x;
  for (; sizeof(S) > 1 && v + (U - 1) * kBlock < vb; v += U * kBlock) {
    v4u y[U][MAXK];
#pragma unroll
    for (int u = 0; u < U; u++) {
#pragma unroll
      for (int k = 0; k < MAXK; k++) {
        if (k < P) y[u][k] = ldv<FAST>(reinterpret_cast<const v4u*>(srcs[k]) + v + u * kBlock);
      }
    }
    v4u acc[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      acc[u] = y[u][0];
#pragma unroll
      for (int k = 1; k < MAXK; k++) {
        if (k < P) {
          acc[u] = LEFT ? vec_apply<T, OP>(acc[u], y[u][k]) : vec_apply<T, OP>(y[u][k], acc[u]);
        }
      }
    }
    if (KEEP) {
      const VecOut<LSP> od(dst, va);
#pragma unroll
      for (int u = 0; u < U; u++) od.put(v + u * kBlock, acc[u]);
    }
#pragma unroll
    for (int d = 0; d < MAXK - 1; d++) {
      if (d < nout) {
        const VecOut<RSP> o(outs[d], va);
#pragma unroll
        for (int u = 0; u < U; u++) o.put(v + u * kBlock, acc[u]);
      }
    }
  }
  for (; v < vb; v += kBlock) {
    v4u y[MAXK];
#pragma unroll
    for (int k = 0; k < MAXK; k++) {
      if (k < P) y[k] = ldv<FAST>(reinterpret_cast<const v4u*>(srcs[k]) + v);
    }
    v4u acc = y[0];
#pragma unroll
    for (int k = 1; k < MAXK; k++) {
      if (k < P) acc = LEFT ? vec_apply<T, OP>(acc, y[k]) : vec_apply<T, OP>(y[k], acc);
    }
    if (KEEP) VecOut<LSP>(dst, va).put(v, acc);
#pragma unroll
    for (int d = 0; d < MAXK - 1; d++) {
      if (d < nout) VecOut<RSP>(outs[d], va).put(v, acc);
    }
  }
}

// Flag words are written by other agents (peers over xGMI, other processes
// on this GPU, workgroups on other XCDs) and polled by their owner.  Writes
// are atomic exchanges and polls atomic compare-exchanges, at system scope:
// both execute at the memory side, so no L2 -- the writer's, the reader's or
// that of another XCD -- ever holds a copy of a flag line that could be read
// stale or written back over a newer value.  Each flag has a 128-byte line
// of its own (kFlagStride words): one writer per line.  Where the link to a
// peer's GPU carries no atomics (Context::flagStores) the write is a
// system-scope store instead: it goes through to the uncached flag block all
// the same, and the owner's polls stay memory-side.
__device__ __forceinline__ void put_flag(uint64_t* word, uint64_t v, bool store = false) {
  if (store) {
    __hip_atomic_store(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    (void)__hip_atomic_exchange(word, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A compare-exchange that never matches (flags never reach ~0): a real
// memory-side read (an idempotent add or or would be turned into a load).
__device__ __forceinline__ uint64_t get_flag(const uint64_t* word) {
  uint64_t v = ~uint64_t(0);
  __hip_atomic_compare_exchange_strong(const_cast<uint64_t*>(word), &v, ~uint64_t(0),
                                       __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
  return v;
}

__device__ __forceinline__ uint64_t* flag_at(uint64_t* row, int w) {
  return row + (size_t)w * kFlagStride;
}

__device__ __forceinline__ const uint64_t* flag_at(const uint64_t* row, int w) {
  return row + (size_t)w * kFlagStride;
}

// Every wave's stores complete and visible system-wide, then (by lanes
// 0..P-1, lane r excluded, where want(lane)) flag words set to epoch.
// Release before a flag.  system: every dirty line of this XCD's L2 written
// back (buffer_wbl2 sc0 sc1) and the stores completed.  narrow: the stores
// completed only -- enough when everything the flag publishes was stored into
// the receiver's landing slot, uncached memory (MTYPE UC) that no L2 holds
// (the device engines' protocol); the workgroup fence keeps
// the compiler from moving the stores past the flag.  (sync: kernels.h
// kSync*; the test-only modes kSyncNoRelease / kSyncUnsafe keep only a
// compiler barrier, and their flag skips the workgroup barrier too
// (flag_barrier): it may overtake the other waves' stores.)
__device__ __forceinline__ void release_stores(int sync) {
  if (sync == kSyncNoRelease || sync == kSyncUnsafe) {
    asm volatile("" ::: "memory");
    return;
  }
  if (sync == kSyncSystem) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  } else {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  }
  // the compiler may drop the wait after the write-back when it can prove no
  // store is outstanding (MI355X_MICROARCH.md, compiler hazard): keep it
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// Acquire after a flag.  system: this CU's L1 and this XCD's L2 invalidated
// (buffer_inv sc0 sc1).  narrow: the L1 only (agent scope, buffer_inv sc1):
// the landing slots are uncached, so no L2 line of them can be stale.  The
// test-only kSyncNoAcquire / kSyncUnsafe keep a compiler barrier only.
__device__ __forceinline__ void acquire_loads(int sync) {
  if (sync == kSyncNoAcquire || sync == kSyncUnsafe) {
    asm volatile("" ::: "memory");
  } else if (sync == kSyncSystem) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  } else {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
}

// The workgroup barrier between every wave's stores and the flag lane.  The
// test-only kSyncNoRelease / kSyncUnsafe skip it: lane 0's flag then goes out
// as soon as ITS wave has issued its stores -- the hazard of a flag that
// overtakes the data, amplified so a one-GPU run can show the checks see it.
__device__ __forceinline__ void flag_barrier(int sync) {
  if (sync != kSyncNoRelease && sync != kSyncUnsafe) __syncthreads();
}

template <typename Want>
__device__ __forceinline__ void release_flags(uint64_t* const* rows, int P, int rank, int w,
                                              uint64_t epoch, bool store, Want want,
                                              int sync) {
  release_stores(sync);
  flag_barrier(sync);
  const int t = (int)threadIdx.x;
  if (t < P && t != rank && want(t)) put_flag(flag_at(rows[t], w), epoch, store);
}

// Every wave's stores complete and visible system-wide, then lane 0 stores
// `value` into `word` (a flag in a peer's memory).
__device__ __forceinline__ void signal_flag(uint64_t* word, uint64_t value, bool store,
                                            int sync) {
  release_stores(sync);
  flag_barrier(sync);
  if (threadIdx.x == 0) put_flag(word, value, store);
}

// The first workgroup of the launch whose wait times out reports it: status
// = 1 + peer (+ 256 * (1 + step) when the plan kernel says where), then as
// 64-bit words 1..3 the value seen, the value awaited and the workgroup.
// `claim` (device memory, zero until a timeout) keeps the report of one
// workgroup whole.
__device__ __forceinline__ void report_timeout(int* status, int* claim, int code,
                                               uint64_t seen, uint64_t awaited) {
  int expected = 0;
  if (!__hip_atomic_compare_exchange_strong(claim, &expected, 1, __ATOMIC_RELAXED,
                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
    return;
  }
  uint64_t* detail = reinterpret_cast<uint64_t*>(status);
  __hip_atomic_store(detail + 1, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(detail + 2, awaited, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(detail + 3, (uint64_t)blockIdx.x, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Lane 0 waits until word >= epoch (bounded); the whole workgroup learns
// the outcome.  Returns false after a timeout (reported).

// `polls` (lane 0's, may be null): += the flag reads this wait made
// (diagnostics: PlanKernelParams::polls).
__device__ __forceinline__ bool wait_flag(const uint64_t* word, uint64_t epoch, int peer,
                                          uint64_t start, uint64_t timeoutTicks, int* status,
                                          int* claim, int* s_ok, int sync, bool acquire = true,
                                          int where = 0, uint32_t* polls = nullptr) {
  if (threadIdx.x == 0) {
    int ok = 1;
    uint64_t v;
    uint32_t spin = 1;
    for (; (v = get_flag(word)) < epoch; spin++) {
      if (__builtin_amdgcn_s_memrealtime() - start > timeoutTicks) {
        ok = 0;
        report_timeout(status, claim, 1 + peer + 256 * where, v, epoch);
        break;
      }
      // the status word is host memory: nonzero once another wait gave up or
      // the host saw a peer process exit (it then stops every wait at once)
      if ((spin & 127) == 0 && *reinterpret_cast<const volatile int*>(status) != 0) {
        ok = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (polls != nullptr) *polls += spin;
    // drop any stale copy of the landing lines before anyone reads them
    if (acquire) acquire_loads(sync);
    *s_ok = ok;
  }
  __syncthreads();
  return *s_ok != 0;
}

// ---- launch counts kept on the device ------------------------------------------

// The launch's number: launches of this algorithm before it.  Uncached
// counters after the flag rows (the workgroup advancing one and those
// reading it next may sit on different XCDs, whose L2s are not coherent):
// ctr[0] launches completed, advanced by finish_launch once the last
// workgroup is done; ctr[kFlagStride] workgroups finished in the current
// launch; ctr[kLaunchStartsOffset + w] the launches workgroup index w has
// started.  A workgroup takes its index's count as its launch number, so the
// numbers come from the GPU and a captured launch replays correctly.
// Launches of one algorithm must not overlap (a graph replayed on another
// stream than eager runs): in stream order every workgroup starts
// after the previous launch completed, so the completed count equals its
// number.  Otherwise either the two launches' workgroups happen to form runs
// one after the other -- each number taken by one workgroup per index, a run
// starting only once the one before completed: a valid serialisation of the
// same algorithm on the same buffer -- or some workgroup sees fewer completed
// launches than its number: it reports kStatusOverlap and its launch does
// nothing more (returns false).  (tests/test_plan_kernel_sim.py models it.)
__device__ __forceinline__ bool launch_number(uint64_t* ctr, int* status, int* claim,
                                              uint64_t* number) {
  __shared__ uint64_t s_n;
  __shared__ int s_in_order;
  if (threadIdx.x == 0) {
    const uint64_t n = __hip_atomic_fetch_add(ctr + kLaunchStartsOffset + blockIdx.x,
                                              (uint64_t)1, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
    const uint64_t done = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_n = n;
    s_in_order = done == n ? 1 : 0;
    if (done != n) report_timeout(status, claim, kStatusOverlap, done, n);
  }
  __syncthreads();
  *number = s_n;
  return s_in_order != 0;
}

__device__ __forceinline__ void finish_launch(uint64_t* ctr, int G) {
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t* done = ctr + kFlagStride;  // a line of its own
    const uint64_t n =
        __hip_atomic_fetch_add(done, (uint64_t)1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (n == (uint64_t)G - 1) {
      __hip_atomic_store(done, (uint64_t)0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_fetch_add(ctr, (uint64_t)1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ---- one-shot ---------------------------------------------------------------

template <typename T, int OP, bool FAST, int RSP>
__device__ __forceinline__ void oneshot_body(const OneShotParams& p) {
  using S = typename Elem<T, OP>::S;
  __shared__ int s_ok;
  const int w = blockIdx.x;
  const size_t e0 = (size_t)w * p.slice;
  const size_t e1 = e0 + p.slice < p.count ? e0 + p.slice : p.count;
  S* buf = reinterpret_cast<S*>(p.buf);
  const bool aligned = ((uintptr_t)p.buf % 16) == 0;
  uint64_t launched;
  if (!launch_number(p.epochCtr, p.status, p.claim, &launched)) return;
  const uint64_t epoch = launched + 1;
  const int par = (int)(epoch & 1);

  // 1. push (peers in ring order from rank+1)
  char* to[kOsMaxRanks - 1];
#pragma unroll
  for (int d = 1; d < kOsMaxRanks; d++) {
    int j = p.rank + d;
    if (j >= p.P) j -= p.P;
    to[d - 1] = d < p.P ? p.push[par][j] : nullptr;
  }
  scatter_span<S, FAST, kStPlain, 0, kOsMaxRanks - 1, RSP>(to, p.P - 1, buf, e0, e1, aligned);
  release_flags(p.flagOut, p.P, p.rank, w, epoch, p.flagStore != 0, [](int) { return true; },
                p.narrow);

  // 2. wait
  const uint64_t start = __builtin_amdgcn_s_memrealtime();
  for (int k = 0; k < p.P; k++) {
    if (k == p.rank) continue;
    if (!wait_flag(flag_at(p.flagIn, k * p.G + w), epoch, k, start, p.timeoutTicks,
                   p.status, p.claim, &s_ok, p.narrow)) {
      return;
    }
  }

  // 3. fold every chunk's part of this slice along its chain
  for (int q = 0; q < p.njobs; q++) {
    const size_t jb = p.jobOff[q], je = p.jobOff[q] + p.jobLen[q];
    const size_t a = jb > e0 ? jb : e0, b = je < e1 ? je : e1;
    if (a >= b) continue;
    const S* src[kOsMaxRanks];
#pragma unroll
    for (int i = 0; i < kOsMaxRanks; i++) {
      const int r = p.chain[q][i];
      src[i] = i < p.P ? (r == p.rank ? buf : reinterpret_cast<const S*>(p.land[par][r]))
                       : nullptr;
    }
    fold_span<T, OP, FAST>(buf, src, p.P, nullptr, 0, a, b, aligned);
  }
  finish_launch(p.epochCtr, p.G);
}

// >= 2 waves per SIMD: every rank's grid (<= kOsMaxSlices workgroups) stays
// resident even when a few ranks share one GPU
template <typename T, int OP, int RSP>
__global__ __launch_bounds__(kBlock, 2) void oneshot_kernel(OneShotParams p) {
  oneshot_body<T, OP, false, RSP>(p);
}

// ---- two-shot ---------------------------------------------------------------

template <typename T, int OP, bool FAST, int RSP>
__device__ __forceinline__ void twoshot_body(const TwoShotParams& p) {
  using S = typename Elem<T, OP>::S;
  __shared__ int s_ok;
  const int w = blockIdx.x;
  auto stamp = [&](int k) {  // diagnostics only (p.trace is null otherwise)
    if (p.trace != nullptr && threadIdx.x == 0) {
      p.trace[(size_t)w * kTsTrace + k] = __builtin_amdgcn_s_memrealtime();
    }
  };
  stamp(0);
  S* buf = reinterpret_cast<S*>(p.buf);
  const bool aligned = ((uintptr_t)p.buf % 16) == 0;
  uint64_t launched;
  if (!launch_number(p.epochCtr, p.status, p.claim, &launched)) return;
  const uint64_t epoch = launched + 1;
  const int par = (int)(epoch & 1);
  auto span = [&](int c, size_t& a, size_t& b) {  // slice w of range c
    const size_t off = p.rangeOff[c], len = p.rangeLen[c];
    const size_t s0 = (size_t)w * p.slice;
    a = off + (s0 < len ? s0 : len);
    b = off + (s0 + p.slice < len ? s0 + p.slice : len);
    return a < b;
  };

  // 1. push my copy of every other range's slice to its owner.  Workgroups
  //    start at different owners (w mod P-1) so that at any moment the
  //    grid's stores spread over all P-1 links instead of queueing on one.
  for (int q = 0; q < p.P - 1; q++) {
    int j = p.rank + 1 + (q + w) % (p.P - 1);
    if (j >= p.P) j -= p.P;
    size_t a, b;
    if (span(j, a, b)) {
      copy_span<S, FAST, RSP>(reinterpret_cast<S*>(p.rsPush[par][j]), buf, a, b, aligned);
    }
  }
  release_flags(p.flagAOut, p.P, p.rank, w, epoch, p.flagStore != 0, [&](int j) {
    size_t a, b;
    return span(j, a, b);
  }, p.narrow);
  stamp(1);

  // 2. fold my range's slice from every peer's copy; result to my buffer
  //    and to every peer's AG slot in the same pass
  const uint64_t start = __builtin_amdgcn_s_memrealtime();
  size_t a, b;
  if (span(p.rank, a, b)) {
    for (int k = 0; k < p.P; k++) {
      if (k == p.rank) continue;
      if (!wait_flag(flag_at(p.flagAIn, k * p.G + w), epoch, k, start, p.timeoutTicks,
                     p.status, p.claim, &s_ok, p.narrow)) {
        return;
      }
    }
    stamp(2);
    const S* src[kOsMaxRanks];
#pragma unroll
    for (int i = 0; i < kOsMaxRanks; i++) {
      const int r = p.chain[i];
      src[i] = i < p.P ? (r == p.rank ? buf : reinterpret_cast<const S*>(p.rsLand[par][r]))
                       : nullptr;
    }
    char* outs[kOsMaxRanks - 1];
#pragma unroll
    for (int d = 1; d < kOsMaxRanks; d++) {
      int j = p.rank + d;
      if (j >= p.P) j -= p.P;
      outs[d - 1] = d < p.P ? p.agPush[par][j] : nullptr;
    }
    fold_span<T, OP, FAST, false, kOsMaxRanks, true, RSP>(buf, src, p.P, outs, p.P - 1, a, b, aligned);
    release_flags(p.flagBOut, p.P, p.rank, w, epoch, p.flagStore != 0,
                  [](int) { return true; }, p.narrow);
  }
  stamp(3);

  // 3. take every other owner's finished slice
  for (int d = 1; d < p.P; d++) {
    int j = p.rank - d;
    if (j < 0) j += p.P;
    if (!span(j, a, b)) continue;
    if (!wait_flag(flag_at(p.flagBIn, j * p.G + w), epoch, j, start, p.timeoutTicks,
                   p.status, p.claim, &s_ok, p.narrow)) {
      return;
    }
    if (d == 1) stamp(4);
    copy_span<S, FAST, kStPlain>(buf, reinterpret_cast<const S*>(p.agLand[par][j]), a, b,
                                 aligned);
  }
  stamp(5);
  finish_launch(p.epochCtr, p.G);
}

template <typename T, int OP, int RSP>
__global__ __launch_bounds__(kBlock, 2) void twoshot_kernel(TwoShotParams p) {
  twoshot_body<T, OP, false, RSP>(p);
}

// ---- plan kernel --------------------------------------------------------------

// Workgroup w's part [a, b) of a segment.
__device__ __forceinline__ bool seg_part(const DevSegment& sg, int w, size_t& a, size_t& b) {
  const size_t off = (size_t)sg.off, len = (size_t)sg.len, sl = (size_t)sg.slice;
  const size_t s0 = (size_t)w * sl;
  a = off + (s0 < len ? s0 : len);
  b = off + (s0 + sl < len ? s0 + sl : len);
  return a < b;
}

// MAXSRC: the most sources a FOLD step of the program has (8), or 2 for the
// programs without FOLD steps (ring, halving-doubling, function-style ring):
// the 8-way fold's registers would cut the resident workgroups per CU from
// the 2-source variant's count (kernel-resource-usage) to 3.
template <typename T, int OP, int MAXSRC, bool FAST, int RSP>
__device__ __forceinline__ void plan_body(const PlanKernelParams& p) {
  using S = typename Elem<T, OP>::S;
  __shared__ int s_ok;
  const int w = blockIdx.x;
  S* buf = reinterpret_cast<S*>(p.buf);
  const bool aligned = ((uintptr_t)p.buf % 16) == 0;
  const int sync = p.narrow;  // kernels.h kSync*
  // diagnostics (GLOO_AMD_DEVTRACE=1): per workgroup and step, when the step
  // started and when its wait (if any) was satisfied
  uint64_t* tr = p.trace != nullptr ? p.trace + (size_t)w * (2 * (size_t)p.nsteps + 1) : nullptr;
  auto stamp = [&](int k) {
    if (tr != nullptr && threadIdx.x == 0) tr[k] = __builtin_amdgcn_s_memrealtime();
  };
  // message m of a channel lands in slot (m - 1) % slots
  auto slotOf = [&](uint64_t m) -> uint64_t { return p.slots == 2 ? ((m - 1) & 1) : 0; };
  // the runs completed before this launch (kernels.h PlanKernelParams::runCtr)
  uint64_t run;
  if (!launch_number(p.runCtr, p.status, p.claim, &run)) return;
  uint32_t polls = 0;  // lane 0's flag reads (diagnostics: p.polls)
  for (int i = 0; i < p.nsteps; i++) {
    const DevStep st = p.steps[i];
    const uint64_t seq = run * st.perRun + st.seq;
    stamp(2 * i);
    switch (st.kind) {
      case kStepReducePre:          // REDUCE, the overlap also into the next SEND's slot
      case kStepReducePreForward:   // the same, the overlap into that slot only
      case kStepCopyPre: {          // COPY, the overlap also into the next SEND's slot
        if (seq > (uint64_t)p.slots &&
            !wait_flag(flag_at(st.credit, w), seq - p.slots, st.peer,
                       __builtin_amdgcn_s_memrealtime(), p.timeoutTicks, p.status, p.claim,
                       &s_ok, sync, /*acquire=*/false, 1 + i, &polls)) {
          return;
        }
        stamp(2 * i + 1);
        char* dst = st.dst + slotOf(seq) * (uint64_t)st.dstSlot;
        const S* src = reinterpret_cast<const S*>(
            st.src + slotOf(run * st.rperRun + st.rseq) * (uint64_t)st.srcSlot);
        char* outs[2] = {reinterpret_cast<char*>(buf), dst};
        const S* srcs[2] = {buf, src};
        for (int g = st.seg0; g < st.seg1; g++) {
          size_t a, b;
          if (!seg_part(p.segs[g], w, a, b)) continue;
          const bool over = g >= st.pre0 && g < st.pre1;
          if (st.kind == kStepCopyPre) {
            if (over) {
              scatter_span<S, FAST, FAST ? kStLocalWt : kStPlain, 1, 2, RSP>(outs, 2, src, a, b,
                                                                        aligned);
            } else {
              copy_span<S, FAST, FAST ? kStLocalWt : kStPlain>(buf, src, a, b, aligned);
            }
          } else if (!over) {
            fold_span<T, OP, FAST, true, 2>(buf, srcs, 2, nullptr, 0, a, b, aligned);
          } else if (st.kind == kStepReducePreForward) {
            fold_span<T, OP, FAST, true, 2, false, RSP>(buf, srcs, 2, outs + 1, 1, a, b, aligned);
          } else {
            fold_span<T, OP, FAST, true, 2, true, RSP>(buf, srcs, 2, outs + 1, 1, a, b, aligned);
          }
        }
        break;  // the SEND signals the message once its other segments are stored
      }
      case 0:                    // SEND, once the receiver has consumed message seq-slots
      case kStepReduceSend:      // REDUCE + SEND of its result in one pass
      case kStepReduceForward:   // the same, result to the peer only
      case kStepCopySend: {      // COPY + SEND of its result in one pass
        if (seq > (uint64_t)p.slots &&
            !wait_flag(flag_at(st.credit, w), seq - p.slots, st.peer,
                       __builtin_amdgcn_s_memrealtime(), p.timeoutTicks, p.status, p.claim,
                       &s_ok, sync, /*acquire=*/false, 1 + i, &polls)) {
          return;
        }
        stamp(2 * i + 1);
        char* dst = st.dst + slotOf(seq) * (uint64_t)st.dstSlot;
        if (st.kind == 0) {
          for (int g = st.seg0; g < st.seg1; g++) {
            size_t a, b;
            if (g >= st.pre0 && g < st.pre1) continue;  // stored by the step before
            if (seg_part(p.segs[g], w, a, b)) {
              copy_span<S, FAST, RSP>(reinterpret_cast<S*>(dst), buf, a, b, aligned);
            }
          }
        } else {
          const S* src = reinterpret_cast<const S*>(
              st.src + slotOf(run * st.rperRun + st.rseq) * (uint64_t)st.srcSlot);
          char* outs[2] = {reinterpret_cast<char*>(buf), dst};
          const S* srcs[2] = {buf, src};
          for (int g = st.seg0; g < st.seg1; g++) {
            size_t a, b;
            if (!seg_part(p.segs[g], w, a, b)) continue;
            if (st.kind == kStepCopySend) {
              scatter_span<S, FAST, FAST ? kStLocalWt : kStPlain, 1, 2, RSP>(outs, 2, src, a, b,
                                                                        aligned);
            } else if (st.kind == kStepReduceForward) {
              fold_span<T, OP, FAST, true, 2, false, RSP>(buf, srcs, 2, outs + 1, 1, a, b, aligned);
            } else {
              fold_span<T, OP, FAST, true, 2, true, RSP>(buf, srcs, 2, outs + 1, 1, a, b, aligned);
            }
          }
        }
        signal_flag(flag_at(st.flag, w), seq, p.flagStore != 0, sync);
        break;
      }
      case 1:  // RECV
        if (!wait_flag(flag_at(st.flag, w), seq, st.peer, __builtin_amdgcn_s_memrealtime(),
                       p.timeoutTicks, p.status, p.claim, &s_ok, sync, true, 1 + i, &polls)) {
          return;
        }
        stamp(2 * i + 1);
        break;
      case 2:    // REDUCE: buf = op(buf, region), in place
      case 3:    // COPY:   buf = region
      case 5: {  // FOLD
        const S* srcs[MAXSRC];
#pragma unroll
        for (int k = 0; k < MAXSRC; k++) srcs[k] = buf;
        int n = 2;
        if (st.kind == 5) {
          n = st.nsrc;
          for (int k = 0; k < n && k < MAXSRC; k++) {
            const char* q = p.foldSrc[st.srcIndex + k];
            if (q != nullptr) srcs[k] = reinterpret_cast<const S*>(q);
          }
        } else {
          srcs[1] = reinterpret_cast<const S*>(
              st.src + slotOf(run * st.rperRun + st.rseq) * (uint64_t)st.srcSlot);
        }
        for (int g = st.seg0; g < st.seg1; g++) {
          size_t a, b;
          if (!seg_part(p.segs[g], w, a, b)) continue;
          if (st.kind == 3) {
            copy_span<S, FAST, FAST ? kStLocalWt : kStPlain>(buf, srcs[1], a, b, aligned);
          } else if (st.kind == 2 || st.left) {
            fold_span<T, OP, FAST, true, MAXSRC>(buf, srcs, n, nullptr, 0, a, b, aligned);
          } else {
            fold_span<T, OP, FAST, false, MAXSRC>(buf, srcs, n, nullptr, 0, a, b, aligned);
          }
        }
        break;
      }
      case 4:  // RELEASE: every wave is done reading the region
        __syncthreads();
        if (threadIdx.x == 0) put_flag(flag_at(st.flag, w), seq, p.flagStore != 0);
        break;
      default:  // kStepNop: a SEND done inside the step it was fused into
        break;
    }
  }
  stamp(2 * p.nsteps);
  if (p.polls != nullptr && threadIdx.x == 0) {
    __hip_atomic_fetch_add(p.polls + w, (uint64_t)polls, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  }
  // the last workgroup to finish advances the run count for the next launch
  // (every workgroup read it at its start, before it could finish)
  finish_launch(p.runCtr, p.G);
}

template <typename T, int OP, int MAXSRC, int RSP>
__global__ __launch_bounds__(kBlock, 2) void plan_kernel(PlanKernelParams p) {
  if constexpr (RSP == kStRemote) {  // the test-only plain-store build runs plain streams
    if (p.fast) {
      plan_body<T, OP, MAXSRC, true, RSP>(p);
      return;
    }
  }
  plan_body<T, OP, MAXSRC, false, RSP>(p);
}

#ifndef GLX_XGMI_UNSAFE_TU
// ---- flag operations of the DMA steps engine (kernels.h FlagOpsParams) ------

// One wave; lane 0 walks the ops in order.  A wait polls memory-side
// (get_flag) with a short sleep, gives up after the timeout (reported like
// the device engines' waits) or as soon as the status word is nonzero (another
// wait gave up, or the host saw a peer exit): the ops after it are skipped, so
// no signal claims work that did not happen, and the stream drains.
//
// Giving up also posts this rank's abort mark to every peer, completed before
// the kernel ends -- before a copy queued behind it on the stream can start
// (kernels.h, abort marks); a peer's mark makes this kernel give up too.
__device__ __forceinline__ void post_aborts(const FlagOpsParams& p) {
  for (int k = 0; k < p.nAbort; k++) put_flag(p.abortOut[k], p.abortValue, p.flagStore != 0);
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// A peer's abort mark (0: none): a system-scope load of our own uncached word.
__device__ __forceinline__ uint64_t peer_abort(const FlagOpsParams& p) {
  return p.abortIn != nullptr
             ? __hip_atomic_load(p.abortIn, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
             : 0;
}

__global__ __launch_bounds__(64) void flag_ops_kernel(FlagOpsParams p) {
  if (threadIdx.x != 0) return;
  const uint64_t start = __builtin_amdgcn_s_memrealtime();
  const volatile int* status = reinterpret_cast<const volatile int*>(p.status);
  auto abandoned = [&]() {  // a peer's mark: report it, pass it on
    const uint64_t a = peer_abort(p);
    if (a == 0) return false;
    report_timeout(p.status, p.claim, kStatusPeerAbort | (int)((a - 1) & 0xffff), a, 0);
    post_aborts(p);
    return true;
  };
  if (*status != 0) {
    post_aborts(p);
    return;
  }
  if (abandoned()) return;
  bool released = false;
  for (int i = 0; i < p.n; i++) {
    const FlagOp& o = p.ops[i];
    if (o.kind == kFlagSignal) {
      if (!released) {
        // once per kernel, before its first signal: the stream's earlier
        // work (a reduce writing the chunk an SDMA copy on another stream
        // reads next, which no L2 sees) written back system-wide; HIP's own
        // release between same-stream kernels may be agent scope
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        released = true;
      }
      put_flag(o.word, o.value, p.flagStore != 0);
      continue;
    }
    uint64_t v;
    for (uint32_t spin = 1; (v = get_flag(o.word)) < o.value; spin++) {
      if (__builtin_amdgcn_s_memrealtime() - start > p.timeoutTicks) {
        report_timeout(p.status, p.claim, o.code, v, o.value);
        post_aborts(p);
        return;
      }
      if ((spin & 127) == 0) {
        if (*status != 0) {
          post_aborts(p);
          return;
        }
        if (abandoned()) return;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
}
#endif

// ---- launch -------------------------------------------------------------------

// This file is compiled twice (Makefile): as the product's engines, whose
// stores into peers' slots are system-scope write-through (kStRemote), and
// with GLX_XGMI_UNSAFE_TU as the TEST-ONLY kSyncUnsafe build of the same
// engines with plain stores there (kernels.h, tests/test_sync_control_gpu.py);
// the product launchers hand kSyncUnsafe launches to the second build.
#ifdef GLX_XGMI_UNSAFE_TU
constexpr int kTuRsp = kStPlain;
#define GLX_TU_NAME(f) f##_unsafe_stores
#else
constexpr int kTuRsp = kStRemote;
#define GLX_TU_NAME(f) f
#endif

template <typename T>
hipError_t launch_os_op(int op, const OneShotParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.G), block(kBlock);
  switch (op) {
    case GLX_SUM: hipLaunchKernelGGL((oneshot_kernel<T, GLX_SUM, kTuRsp>), grid, block, 0, s, p); break;
    case GLX_PRODUCT:
      hipLaunchKernelGGL((oneshot_kernel<T, GLX_PRODUCT, kTuRsp>), grid, block, 0, s, p);
      break;
    case GLX_MAX: hipLaunchKernelGGL((oneshot_kernel<T, GLX_MAX, kTuRsp>), grid, block, 0, s, p); break;
    case GLX_MIN: hipLaunchKernelGGL((oneshot_kernel<T, GLX_MIN, kTuRsp>), grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_ts_op(int op, const TwoShotParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.G), block(kBlock);
  switch (op) {
    case GLX_SUM: hipLaunchKernelGGL((twoshot_kernel<T, GLX_SUM, kTuRsp>), grid, block, 0, s, p); break;
    case GLX_PRODUCT:
      hipLaunchKernelGGL((twoshot_kernel<T, GLX_PRODUCT, kTuRsp>), grid, block, 0, s, p);
      break;
    case GLX_MAX: hipLaunchKernelGGL((twoshot_kernel<T, GLX_MAX, kTuRsp>), grid, block, 0, s, p); break;
    case GLX_MIN: hipLaunchKernelGGL((twoshot_kernel<T, GLX_MIN, kTuRsp>), grid, block, 0, s, p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

#ifndef GLX_XGMI_UNSAFE_TU
template <typename T, int OP>
const void* engine_kernel(int kernel) {
  if (kernel == 0) return (const void*)oneshot_kernel<T, OP, kStRemote>;
  if (kernel == 1) return (const void*)twoshot_kernel<T, OP, kStRemote>;
  if (kernel == 3) return (const void*)plan_kernel<T, OP, 2, kStRemote>;
  return (const void*)plan_kernel<T, OP, kOsMaxRanks, kStRemote>;
}

template <typename T>
int resident_typed(int kernel, int op) {
  const void* k = nullptr;
  switch (op) {
    case GLX_SUM: k = engine_kernel<T, GLX_SUM>(kernel); break;
    case GLX_PRODUCT: k = engine_kernel<T, GLX_PRODUCT>(kernel); break;
    case GLX_MAX: k = engine_kernel<T, GLX_MAX>(kernel); break;
    case GLX_MIN: k = engine_kernel<T, GLX_MIN>(kernel); break;
    default: return 0;
  }
  int perCu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCu, k, kBlock, 0) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return perCu * cus;
}

#endif

template <typename T, int MAXSRC>
hipError_t launch_pk_src(int op, const PlanKernelParams& p, hipStream_t s) {
  const dim3 grid((unsigned)p.G), block(kBlock);
  switch (op) {
    case GLX_SUM:
      hipLaunchKernelGGL((plan_kernel<T, GLX_SUM, MAXSRC, kTuRsp>), grid, block, 0, s, p);
      break;
    case GLX_PRODUCT:
      hipLaunchKernelGGL((plan_kernel<T, GLX_PRODUCT, MAXSRC, kTuRsp>), grid, block, 0, s, p);
      break;
    case GLX_MAX:
      hipLaunchKernelGGL((plan_kernel<T, GLX_MAX, MAXSRC, kTuRsp>), grid, block, 0, s, p);
      break;
    case GLX_MIN:
      hipLaunchKernelGGL((plan_kernel<T, GLX_MIN, MAXSRC, kTuRsp>), grid, block, 0, s, p);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_pk_op(int op, const PlanKernelParams& p, hipStream_t s) {
  return p.maxSrc <= 2 ? launch_pk_src<T, 2>(op, p, s) : launch_pk_src<T, kOsMaxRanks>(op, p, s);
}

}  // namespace

#ifndef GLX_XGMI_UNSAFE_TU
int device_engine_resident_blocks(int kernel, int op, int dtype) {
  switch (dtype) {
    case GLX_INT8: return resident_typed<int8_t>(kernel, op);
    case GLX_UINT8: return resident_typed<uint8_t>(kernel, op);
    case GLX_INT32: return resident_typed<int32_t>(kernel, op);
    case GLX_INT64: return resident_typed<int64_t>(kernel, op);
    case GLX_UINT64: return resident_typed<uint64_t>(kernel, op);
    case GLX_FLOAT32: return resident_typed<float>(kernel, op);
    case GLX_FLOAT64: return resident_typed<double>(kernel, op);
    case GLX_FLOAT16: return resident_typed<f16_t>(kernel, op);
    case GLX_BFLOAT16: return resident_typed<bf16_t>(kernel, op);
  }
  return 0;
}

#endif

hipError_t GLX_TU_NAME(launch_oneshot)(int op, int dtype, const OneShotParams& p, hipStream_t s) {
#ifndef GLX_XGMI_UNSAFE_TU
  if (p.narrow == kSyncUnsafe) return launch_oneshot_unsafe_stores(op, dtype, p, s);
#endif
  if (p.status == nullptr || p.claim == nullptr || p.epochCtr == nullptr) {
    return hipErrorInvalidValue;
  }
  if (p.P < 2 || p.P > kOsMaxRanks || p.G < 1 || p.G > kOsMaxSlices || p.njobs < 0 ||
      p.njobs > kOsMaxRanks || p.count == 0 || p.slice == 0 ||
      (size_t)p.G * p.slice < p.count || (size_t)(p.G - 1) * p.slice >= p.count) {
    return hipErrorInvalidValue;  // the grid must cover the buffer exactly
  }
  switch (dtype) {
    case GLX_INT8: return launch_os_op<int8_t>(op, p, s);
    case GLX_UINT8: return launch_os_op<uint8_t>(op, p, s);
    case GLX_INT32: return launch_os_op<int32_t>(op, p, s);
    case GLX_INT64: return launch_os_op<int64_t>(op, p, s);
    case GLX_UINT64: return launch_os_op<uint64_t>(op, p, s);
    case GLX_FLOAT32: return launch_os_op<float>(op, p, s);
    case GLX_FLOAT64: return launch_os_op<double>(op, p, s);
    case GLX_FLOAT16: return launch_os_op<f16_t>(op, p, s);
    case GLX_BFLOAT16: return launch_os_op<bf16_t>(op, p, s);
  }
  return hipErrorInvalidValue;
}

hipError_t GLX_TU_NAME(launch_plan_kernel)(int op, int dtype, const PlanKernelParams& p,
                                           hipStream_t s) {
#ifndef GLX_XGMI_UNSAFE_TU
  if (p.narrow == kSyncUnsafe) return launch_plan_kernel_unsafe_stores(op, dtype, p, s);
#endif
  if (p.G < 1 || p.G > kOsMaxSlices || p.nsteps < 0 || p.steps == nullptr ||
      p.segs == nullptr || p.foldSrc == nullptr || p.status == nullptr || p.claim == nullptr ||
      p.runCtr == nullptr ||
      (p.slots != 1 && p.slots != 2) || p.maxSrc < 2 || p.maxSrc > kOsMaxRanks) {
    return hipErrorInvalidValue;
  }
  switch (dtype) {
    case GLX_INT8: return launch_pk_op<int8_t>(op, p, s);
    case GLX_UINT8: return launch_pk_op<uint8_t>(op, p, s);
    case GLX_INT32: return launch_pk_op<int32_t>(op, p, s);
    case GLX_INT64: return launch_pk_op<int64_t>(op, p, s);
    case GLX_UINT64: return launch_pk_op<uint64_t>(op, p, s);
    case GLX_FLOAT32: return launch_pk_op<float>(op, p, s);
    case GLX_FLOAT64: return launch_pk_op<double>(op, p, s);
    case GLX_FLOAT16: return launch_pk_op<f16_t>(op, p, s);
    case GLX_BFLOAT16: return launch_pk_op<bf16_t>(op, p, s);
  }
  return hipErrorInvalidValue;
}

hipError_t GLX_TU_NAME(launch_twoshot)(int op, int dtype, const TwoShotParams& p, hipStream_t s) {
#ifndef GLX_XGMI_UNSAFE_TU
  if (p.narrow == kSyncUnsafe) return launch_twoshot_unsafe_stores(op, dtype, p, s);
#endif
  size_t maxLen = 0;
  for (int c = 0; c < p.P && c < kOsMaxRanks; c++) {
    maxLen = p.rangeLen[c] > maxLen ? p.rangeLen[c] : maxLen;
  }
  if (p.P < 2 || p.P > kOsMaxRanks || p.G < 1 || p.G > kOsMaxSlices || p.slice == 0 ||
      (size_t)p.G * p.slice < maxLen || p.status == nullptr || p.claim == nullptr ||
      p.epochCtr == nullptr) {
    return hipErrorInvalidValue;  // the slices must cover every range
  }
  switch (dtype) {
    case GLX_INT8: return launch_ts_op<int8_t>(op, p, s);
    case GLX_UINT8: return launch_ts_op<uint8_t>(op, p, s);
    case GLX_INT32: return launch_ts_op<int32_t>(op, p, s);
    case GLX_INT64: return launch_ts_op<int64_t>(op, p, s);
    case GLX_UINT64: return launch_ts_op<uint64_t>(op, p, s);
    case GLX_FLOAT32: return launch_ts_op<float>(op, p, s);
    case GLX_FLOAT64: return launch_ts_op<double>(op, p, s);
    case GLX_FLOAT16: return launch_ts_op<f16_t>(op, p, s);
    case GLX_BFLOAT16: return launch_ts_op<bf16_t>(op, p, s);
  }
  return hipErrorInvalidValue;
}

#ifndef GLX_XGMI_UNSAFE_TU
hipError_t launch_flag_ops(const FlagOpsParams& p, hipStream_t s) {
  if (p.n < 1 || p.n > kFlagOpsMax || p.status == nullptr || p.claim == nullptr ||
      p.nAbort < 0 || p.nAbort > kFlagAbortMax) {
    return hipErrorInvalidValue;
  }
  for (int k = 0; k < p.nAbort; k++) {
    if (p.abortOut[k] == nullptr) return hipErrorInvalidValue;
  }
  for (int i = 0; i < p.n; i++) {
    if (p.ops[i].word == nullptr ||
        (p.ops[i].kind != kFlagWait && p.ops[i].kind != kFlagSignal)) {
      return hipErrorInvalidValue;
    }
  }
  hipLaunchKernelGGL(flag_ops_kernel, dim3(1), dim3(64), 0, s, p);
  return hipGetLastError();
}
#endif

}  // namespace glx
