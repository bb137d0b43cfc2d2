"""Host<->device copy engines for the H<->D-inclusive path:
can H2D and D2H overlap over one PCIe link if one direction is done by the
DMA engine (hipMemcpyAsync) and the other by CUs (the product's copy kernel
storing into / loading from pinned host memory)?  256 MiB each way, pinned
host blocks from hipHostMalloc (torch pin_memory), one GPU.

    python tools/micro/pcie_duplex.py > gpurun_out/pcie_duplex.json
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import gloo_amd  # noqa: E402

MiB = 1 << 20


def main():
    n = 256 * MiB
    hs = torch.empty(n, dtype=torch.uint8).pin_memory()   # H2D source
    hd = torch.empty(n, dtype=torch.uint8).pin_memory()   # D2H destination
    hs.fill_(7)
    ds = torch.full((n,), 3, dtype=torch.uint8, device="cuda")  # D2H source
    dd = torch.empty(n, dtype=torch.uint8, device="cuda")       # H2D destination
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def dma_h2d(s):
        with torch.cuda.stream(s):
            dd.copy_(hs, non_blocking=True)

    def dma_d2h(s):
        with torch.cuda.stream(s):
            hd.copy_(ds, non_blocking=True)

    def cu_h2d(s, blocks):
        gloo_amd.kernel_copy(dd.data_ptr(), hs.data_ptr(), n, blocks, s)

    def cu_d2h(s, blocks):
        gloo_amd.kernel_copy(hd.data_ptr(), ds.data_ptr(), n, blocks, s)

    def timed(fns, reps=5):
        for f in fns:
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            for f in fns:
                f()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    out = {}

    def rec(name, fns, nbytes):
        t = timed(fns)
        out[name] = {"ms": round(t * 1e3, 3), "GBps_total": round(nbytes / t / 1e9, 1)}
        print(name, out[name], flush=True)

    rec("dma_h2d", [lambda: dma_h2d(sa)], n)
    rec("dma_d2h", [lambda: dma_d2h(sa)], n)
    for blocks in (32, 64, 128, 256, 512):
        rec("cu_h2d_%dwg" % blocks, [lambda b=blocks: cu_h2d(sa, b)], n)
        rec("cu_d2h_%dwg" % blocks, [lambda b=blocks: cu_d2h(sa, b)], n)
    rec("duplex_dma_dma", [lambda: dma_h2d(sa), lambda: dma_d2h(sb)], 2 * n)
    for blocks in (64, 128, 256):
        rec("duplex_dma_h2d_cu_d2h_%dwg" % blocks,
            [lambda: dma_h2d(sa), lambda b=blocks: cu_d2h(sb, b)], 2 * n)
        rec("duplex_cu_h2d_%dwg_dma_d2h" % blocks,
            [lambda b=blocks: cu_h2d(sa, b), lambda: dma_d2h(sb)], 2 * n)
        rec("duplex_cu_cu_%dwg" % blocks,
            [lambda b=blocks: cu_h2d(sa, b), lambda b=blocks: cu_d2h(sb, b)], 2 * n)
    torch.cuda.synchronize()
    assert bool((dd == 7).all()) and bool((hd == 3).all())
    print(json.dumps(out))


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
