"""Copy bandwidth of G workgroups, contiguous slices vs grid-stride (see
copy_bw.hip).  Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC
tools/micro/copy_bw.hip -o tools/micro/libcopy_bw.so; run on one GPU."""
import ctypes
import os

import torch


def main():
    lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcopy_bw.so"))
    lib.copy_bw_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    for mib in (4, 64, 256):
        nbytes = mib << 20
        src = torch.ones(nbytes // 4, device="cuda")
        dst = torch.zeros_like(src)
        s = torch.cuda.current_stream()
        for G in (256, 512, 1024, 4096):
            for U in (4, 8, 16):
                for sliced in (1, 0):
                    def go():
                        rc = lib.copy_bw_launch(dst.data_ptr(), src.data_ptr(), nbytes, G, U,
                                                sliced, ctypes.c_void_p(s.cuda_stream))
                        assert rc == 0
                    for _ in range(3):
                        go()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = torch.cuda.Event(enable_timing=True)
                    reps = 20
                    e0.record(s)
                    for _ in range(reps):
                        go()
                    e1.record(s)
                    torch.cuda.synchronize()
                    us = e0.elapsed_time(e1) / reps * 1e3
                    print("copy %4d MiB G %5d U %2d %-7s %8.1f us %7.0f GB/s"
                          % (mib, G, U, "sliced" if sliced else "stride", us,
                             2 * nbytes / us / 1e3), flush=True)
        assert bool((dst == 1).all())


if __name__ == "__main__":
    import faulthandler
    faulthandler.enable()  # a crash prints every thread's stack
    main()
