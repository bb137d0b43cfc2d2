#!/usr/bin/env python3
"""The reference's benchmark runner (gloo/benchmark/{main,cuda_main,runner,
options}.cc) for its allreduce benchmarks, on gloo_amd: the same command
line, the same inputs and verification, the same sampling loop and the same
table, so a user of `gloo/benchmark/benchmark` or `benchmark_cuda` gets
comparable numbers from the MI355X path.  One process per rank:

    python tools/gloo_benchmark.py -s 8 -r $R --shared-path /tmp/rdv \\
        [--elements N] [--inputs K] [--iteration-count N | --iteration-time 2s] \\
        [--warmup-iters 5] [--no-verify] [--halfprecision] [--base B] [--nanos] \\
        cuda_allreduce_ring_chunked

(-s / -r default to WORLD_SIZE / RANK, so torchrun works too.)  Benchmarks:
allreduce_{ring,ring_chunked,halving_doubling,bcube,local} and the cuda_
names of the same classes (cuda_allreduce_halving_doubling_pipelined too);
all run on the GPU (rank r on device r % GPUs, or --device) -- the CPU names
are accepted because a switching user's scripts use them.

What matches the reference:
* inputs: input i of rank r holds x[j] = j * (P * inputs) + r * inputs + i
  (gloo/benchmark/benchmark.h:54-73);
* verify (default on, first run of every size): every output equals
  T(j * size^2 + size(size-1)/2), size = P * inputs (cuda_main.cc:112-129,
  main.cc:262-296); allreduce_local: the sum of this rank's inputs only.  Like
  the reference the check is exact; where the expected values exceed the
  type's exact integer range (2^24 fp32, 2^11 fp16) the sums round, so the
  check there allows the rounding (relative 1e-6 * size fp32, max(1e-3,
  size * 2^-11) fp16; infinities where the expectation overflows fp16).
  fp16 outputs of 15360 and more are not verified: there the reference's own
  float16 assignment can keep a stale operand (gloo/types.h:129-134), and
  this path reproduces the reference's bits, not the arithmetic sum;
* sampling (runner.cc:270-357): warmup runs, then an iteration count from
  --iteration-count or from --iteration-time (default 2 s) over the warmup
  median, raised 1.2x until the samples cover the time (rank 0 decides
  both and every rank follows);
  each sample is one run() (results complete on return), between barriers;
* output (runner.cc:400-520, rank 0): size (B), elements, min / p50 / p99 /
  max latency (us, or ns with --nanos), bandwidth = bytes * samples / total
  time / 2^30 ("GB/s" as the reference labels it), iterations;
* without --elements, the sweep 100, 200, 500, ..., 1M, 2M, 5M elements.
--json also prints one JSON line per size.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

K_COL_S, K_COL_M, K_COL_L = 11, 13, 19
K_TOTAL = 6 * K_COL_S + K_COL_M + K_COL_L
K_HEADER = K_TOTAL // 2
K_ITERS_MULTIPLIER = 1.2
K_MAX_ITERATIONS = 1000000000

CLASSES = {
    "allreduce_ring": "AllreduceRing",
    "allreduce_ring_chunked": "AllreduceRingChunked",
    "allreduce_halving_doubling": "AllreduceHalvingDoubling",
    "allreduce_bcube": "AllreduceBcube",
    "allreduce_local": "AllreduceLocal",
    "cuda_allreduce_ring": "HipAllreduceRing",
    "cuda_allreduce_ring_chunked": "HipAllreduceRingChunked",
    "cuda_allreduce_halving_doubling": "HipAllreduceHalvingDoubling",
    "cuda_allreduce_halving_doubling_pipelined": "HipAllreduceHalvingDoublingPipelined",
    "cuda_allreduce_bcube": "HipAllreduceBcube",
    "cuda_allreduce_local": "HipAllreduceLocal",
}


def parse_time(s):
    """--iteration-time: '2s', '500ms', '100us' or nanoseconds (options.cc)."""
    for suf, mul in (("ms", 1e6), ("us", 1e3), ("ns", 1.0), ("s", 1e9)):
        if s.endswith(suf):
            return int(float(s[:-len(suf)]) * mul)
    return int(s)


def parse_args(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0],
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("-s", "--size", type=int, default=int(os.environ.get("WORLD_SIZE", "1")))
    ap.add_argument("-r", "--rank", type=int, default=int(os.environ.get("RANK", "0")))
    ap.add_argument("-x", "--prefix", default="gloo_amd_benchmark")
    ap.add_argument("--shared-path", default=None,
                    help="file-system rendezvous directory (required for -s > 1)")
    ap.add_argument("-t", "--transport", default="xgmi",
                    help="accepted for the reference's scripts; the transport is xGMI")
    ap.add_argument("--no-verify", dest="verify", action="store_false", default=True)
    ap.add_argument("--show-all-errors", action="store_true")
    ap.add_argument("--elements", type=int, default=-1)
    ap.add_argument("--inputs", type=int, default=1)
    ap.add_argument("--warmup-iters", type=int, default=5)
    ap.add_argument("--iteration-count", type=int, default=-1)
    ap.add_argument("--iteration-time", type=parse_time, default=2 * 10**9)
    ap.add_argument("--nanos", action="store_true")
    ap.add_argument("--halfprecision", action="store_true")
    ap.add_argument("--base", type=int, default=2)
    ap.add_argument("--threads", type=int, default=1, help="1 (one context per process)")
    ap.add_argument("--device", type=int, default=None, help="GPU (default rank %% GPUs)")
    ap.add_argument("--json", action="store_true", help="also one JSON line per size")
    ap.add_argument("benchmark", choices=sorted(CLASSES))
    a = ap.parse_args(argv)
    if a.threads != 1:
        ap.error("--threads: one context per process here (start more ranks instead)")
    if a.size > 1 and not a.shared_path:
        ap.error("--shared-path is required with more than one process")
    return a


def inputs_for(np, dtype, P, rank, inputs, n):
    """gloo/benchmark/benchmark.h:54-73."""
    stride = P * inputs
    j = np.arange(n, dtype=np.float64)
    return [(j * stride + (rank * inputs + i)).astype(dtype) for i in range(inputs)]


def expected_for(np, dtype, bench, P, rank, inputs, n):
    """The value every output must hold (main.cc:262-296, cuda_main.cc:112-129)."""
    j = np.arange(n, dtype=np.float64)
    if bench.endswith("allreduce_local"):
        stride = P * inputs
        exp = inputs * (j * stride + rank * inputs) + inputs * (inputs - 1) / 2.0
    else:
        size = P * inputs
        exp = j * size * size + size * (size - 1) / 2.0
    with np.errstate(over="ignore"):  # fp16 overflows to inf, as the sums do
        return exp, exp.astype(dtype)


# float16: at or above this value the reference's own sums can keep a stale
# operand.  float16::operator= (gloo/types.h:129-134) skips the store when the
# destination equals float16(int(rhs.x)), the bit pattern read as an integer
# (>= 15360 for any value >= 1); this path reproduces the reference's bits
# (DESIGN.md 2), not the arithmetic sum, so such outputs are not verified.
F16_UNCHECKED_FROM = 15360.0


def check(np, dtype, got, exp64, exp, size):
    """Exact like the reference where the type holds the values exactly;
    within the sums' rounding beyond.  Returns the mismatching indices."""
    exact_max = 2.0 ** (11 if dtype == np.float16 else 24)
    g = got.astype(np.float64)
    e = exp.astype(np.float64)
    bad = g != e
    if dtype == np.float16:
        bad &= np.abs(exp64) < F16_UNCHECKED_FROM
    big = np.abs(exp64) > exact_max
    if big.any():
        # one rounding per hop: fp16 2^-11 relative each (at least the
        # reference tests' 1e-3, base_test.h), fp32 1e-6 per rank
        rel = max(1e-3, size * 2.0 ** -11) if dtype == np.float16 else 1e-6 * max(1, size)
        both_inf = np.isinf(g) & np.isinf(e) & (np.sign(g) == np.sign(e))
        ok = both_inf | (np.abs(g - exp64) <= rel * np.abs(exp64))
        bad = np.where(big, ~ok, bad)
        if dtype == np.float16:
            bad &= np.abs(exp64) < F16_UNCHECKED_FROM
    return np.nonzero(bad)[0]


class Rendezvous:
    """The runner's barrier and broadcast (runner.cc:360-395) over the store."""

    def __init__(self, gloo_amd, a):
        self.rank, self.size = a.rank, a.size
        self.store = (gloo_amd.rendezvous.PrefixStore(a.prefix + "/",
                                                      gloo_amd.rendezvous.FileStore(a.shared_path))
                      if a.size > 1 else gloo_amd.rendezvous.HashStore())
        self.n = 0

    def barrier(self):
        self.n += 1
        if self.size == 1:
            return
        self.store.set("barrier/%d/%d" % (self.n, self.rank), b"1")
        for r in range(self.size):
            self.store.get("barrier/%d/%d" % (self.n, r), timeout_ms=600000)

    def broadcast(self, value):
        self.n += 1
        if self.size == 1:
            return value
        key = "bcast/%d" % self.n
        if self.rank == 0:
            self.store.set(key, str(int(value)).encode())
        return int(self.store.get(key, timeout_ms=600000).decode())


def percentile(sorted_ns, pct):
    return sorted_ns[int(pct * len(sorted_ns))]  # timer.h:96-98


def main(argv=None):
    a = parse_args(argv)
    import numpy as np
    import torch

    import gloo_amd

    dev = a.device if a.device is not None else a.rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(dev)
    rdv = Rendezvous(gloo_amd, a)
    ctx = gloo_amd.rendezvous.Context(a.rank, a.size, dev)
    ctx.base = a.base
    ctx.connectFullMesh(rdv.store)
    cls = getattr(gloo_amd, CLASSES[a.benchmark])
    np_t = np.float16 if a.halfprecision else np.float32
    t_t = torch.float16 if a.halfprecision else torch.float32
    es = 2 if a.halfprecision else 4
    div = 1 if a.nanos else 1000
    unit = "(ns)" if a.nanos else "(us)"

    if a.rank == 0:
        line = "=" * (K_TOTAL + 2)
        name = a.benchmark.upper()
        print(line)
        print(name.rjust(K_HEADER + len(name) // 2))
        print()
        print("Device:".ljust(K_COL_M) + "xGMI, %s (device %d of %d)"
              % (torch.cuda.get_device_name(dev), dev, torch.cuda.device_count()))
        opts = "processes=%d, inputs=%d, threads=1" % (a.size, a.inputs)
        if a.benchmark.endswith("allreduce_bcube"):
            opts += ", base=%d" % a.base
        if a.benchmark.startswith("cuda_"):
            opts += ", gpudirect=no"
        opts += ", verify=%s" % ("true" if a.verify else "false")
        print("Options:".ljust(K_COL_M) + opts)
        print()
        print(line)
        title = "BENCHMARK RESULTS"
        print(title.rjust(K_HEADER + len(title) // 2))
        print()
        print("size (B)".rjust(K_COL_S) + "elements".rjust(K_COL_S)
              + ("min " + unit).rjust(K_COL_S) + ("p50 " + unit).rjust(K_COL_S)
              + ("p99 " + unit).rjust(K_COL_S) + ("max " + unit).rjust(K_COL_S)
              + "bandwidth (GB/s)".rjust(K_COL_L) + "iterations".rjust(K_COL_M))
        sys.stdout.flush()

    sizes = [a.elements] if a.elements > 0 else [
        i * m for i in (100, 1000, 10000, 100000, 1000000) for m in (1, 2, 5)]
    failures = 0
    for n in sizes:
        host = inputs_for(np, np_t, a.size, a.rank, a.inputs, n)
        bufs = [torch.from_numpy(h).to(device="cuda:%d" % dev, dtype=t_t) for h in host]
        torch.cuda.synchronize()
        alg = cls(ctx, bufs, n)
        if a.verify:
            alg.run()
            torch.cuda.synchronize()
            exp64, exp = expected_for(np, np_t, a.benchmark, a.size, a.rank, a.inputs, n)
            errs = []
            for k, b in enumerate(bufs):
                idx = check(np, np_t, b.cpu().numpy(), exp64, exp, a.size * a.inputs)
                for i in (idx if a.show_all_errors else idx[:1]):
                    errs.append("[rank %d] input %d: Mismatch at index: %d (got %r, expected %r)"
                                % (a.rank, k, i, float(b[i].item()), float(exp[i])))
            if errs:
                failures += 1
                for e in errs:
                    print(e, file=sys.stderr)
            rdv.barrier()

        def sample(iters):
            rdv.barrier()
            out = []
            for _ in range(iters):
                t0 = time.perf_counter_ns()
                alg.run()  # results complete on return (no streams)
                out.append(time.perf_counter_ns() - t0)
            rdv.barrier()
            return out

        warm = sorted(sample(a.warmup_iters)) if a.warmup_iters > 0 else []
        iters = a.iteration_count
        if iters <= 0:
            med = percentile(warm, 0.5) if warm else 1
            iters = rdv.broadcast(max(1, a.iteration_time // max(1, med)))
        while True:
            res = sample(iters)
            if a.iteration_count > 0:
                break
            # rank 0 decides whether the samples cover the time and every rank
            # follows (each rank judging its own samples could split them: one
            # stops while another waits for the next round)
            nxt = 0
            if sum(res) <= a.iteration_time and iters < K_MAX_ITERATIONS:
                nxt = max(int(K_ITERS_MULTIPLIER * iters), iters + 1)
            iters = rdv.broadcast(min(nxt, K_MAX_ITERATIONS))
            if iters == 0:
                break
        alg.close()
        if a.rank == 0:
            lat = sorted(res)
            nbytes = n * es
            secs = sum(lat) / 1e9
            gbps = nbytes * len(lat) / secs / (1024 ** 3)
            print(str(nbytes).rjust(K_COL_S) + str(n).rjust(K_COL_S)
                  + str(lat[0] // div).rjust(K_COL_S)
                  + str(percentile(lat, 0.5) // div).rjust(K_COL_S)
                  + str(percentile(lat, 0.99) // div).rjust(K_COL_S)
                  + str(lat[-1] // div).rjust(K_COL_S)
                  + ("%.3f" % gbps).rjust(K_COL_L) + str(len(lat)).rjust(K_COL_M))
            if a.json:
                print(json.dumps({"benchmark": a.benchmark, "processes": a.size,
                                  "inputs": a.inputs, "bytes": nbytes, "elements": n,
                                  "min_ns": lat[0], "p50_ns": percentile(lat, 0.5),
                                  "p99_ns": percentile(lat, 0.99), "max_ns": lat[-1],
                                  "GiBps": round(gbps, 3), "iterations": len(lat),
                                  "dtype": "f16" if a.halfprecision else "f32",
                                  "verified": a.verify and failures == 0}))
            sys.stdout.flush()
        del bufs
    if a.rank == 0:
        print()
        print("=" * (K_TOTAL + 2))
    rdv.barrier()
    ctx.close()
    return 1 if failures else 0


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    sys.exit(main())
