#!/usr/bin/env python3
"""PCIe copy rates between pinned host memory and the GPU (torch copies on
dedicated streams): one direction alone, both at once, and each direction
split over 2 streams -- what bounds the host-staged (H<->D-inclusive) path of
DESIGN.md 7, whose N = 1 run moves 512 MiB in and 512 MiB out."""
import json
import time

import torch


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    nb = 256 << 20
    h = [torch.empty(nb, dtype=torch.uint8).pin_memory() for _ in range(4)]
    d = [torch.empty(nb, dtype=torch.uint8, device="cuda") for _ in range(4)]
    s = [torch.cuda.Stream() for _ in range(4)]

    def run(jobs):  # jobs: (stream index, dst, src)
        for k, dst, src in jobs:
            with torch.cuda.stream(s[k]):
                dst.copy_(src, non_blocking=True)

    out = {}
    cases = {
        "h2d_1x256MiB": [(0, d[0], h[0])],
        "d2h_1x256MiB": [(0, h[0], d[0])],
        "h2d_2x256MiB_one_stream": [(0, d[0], h[0]), (0, d[1], h[1])],
        "h2d_2x256MiB_two_streams": [(0, d[0], h[0]), (1, d[1], h[1])],
        "d2h_2x256MiB_two_streams": [(0, h[0], d[0]), (1, h[1], d[1])],
        "duplex_1+1_two_streams": [(0, d[0], h[0]), (1, h[1], d[1])],
        "duplex_2+2_one_stream_each_way": [(0, d[0], h[0]), (0, d[1], h[1]),
                                           (1, h[2], d[2]), (1, h[3], d[3])],
        "duplex_2+2_four_streams": [(0, d[0], h[0]), (1, d[1], h[1]),
                                    (2, h[2], d[2]), (3, h[3], d[3])],
    }
    for name, jobs in cases.items():
        t = timed(lambda: run(jobs))
        out[name] = {"ms": round(t * 1e3, 3), "GBps_total": round(len(jobs) * nb / t / 1e9, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
