"""GPU checks of the raw copy entry points (glx_copy: the kernel transport's
copy kernel; glx_peer_copy: hipMemcpyPeerAsync).  The bench's link probe
and callers holding foreign buffers use them; byte-exact for any length and
alignment (the kernel has a 16-byte vector body and byte head/tail paths)."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.mark.parametrize("nbytes", [1, 15, 16, 17, 4096, 1000003, 64 << 20])
@pytest.mark.parametrize("dst_off,src_off", [(0, 0), (3, 3), (1, 5), (16, 0)])
@pytest.mark.parametrize("engine", ["kernel", "dma"])
def test_copy_bytes_exact(nbytes, dst_off, src_off, engine):
    import gloo_amd
    g = torch.Generator(device="cuda").manual_seed(nbytes + dst_off)
    src = torch.randint(0, 256, (nbytes + 64,), dtype=torch.uint8, device="cuda", generator=g)
    dst = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    if engine == "kernel":
        gloo_amd.kernel_copy(dst.data_ptr() + dst_off, src.data_ptr() + src_off, nbytes, 64, s)
    else:
        dev = torch.cuda.current_device()
        gloo_amd.peer_copy(dst.data_ptr() + dst_off, dev, src.data_ptr() + src_off, dev,
                           nbytes, s)
    torch.cuda.synchronize()
    assert torch.equal(dst[dst_off:dst_off + nbytes], src[src_off:src_off + nbytes])
    assert int(dst[:dst_off].sum()) == 0 and int(dst[dst_off + nbytes:].sum()) == 0


def test_copy_zero_bytes_and_null():
    import gloo_amd
    s = torch.cuda.current_stream()
    gloo_amd.kernel_copy(0, 0, 0, 64, s)  # nothing to do: OK
    with pytest.raises(gloo_amd.EnforceNotMet):
        gloo_amd.kernel_copy(0, 0, 16, 64, s)
