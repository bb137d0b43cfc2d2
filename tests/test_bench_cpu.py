"""bench.py's host-side logic on CPU: the per-candidate result check (a
world_size-2 gloo process group, as the N>1 bench runs it), candidate
naming, and the algorithmic byte counts the roofline fields are built from."""
import os
import socket
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

torch = pytest.importorskip("torch")

import bench  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _check_worker(rank, world, port, dtype, corrupt, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 16
    srcs = [bench.synthetic(torch, n, dtype, torch.device("cpu"), 1234 + r) for r in range(world)]
    # the allreduce result every rank holds: the sum in fp32, rounded to the type
    total = srcs[0].float()
    for x in srcs[1:]:
        total = total + x.float()
    result = total.to(srcs[0].dtype)
    if corrupt == "stale_chunk":
        # one 1/16 chunk holds this rank's own input instead of the sum
        c = n // 16
        result[3 * c:4 * c] = srcs[rank][3 * c:4 * c]
    elif corrupt == "one_element":
        result[777] = result[777] + 1
    ok, rel = bench.result_check(torch, dist, srcs[rank], result)
    q.put((rank, ok, rel))
    dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["f32", "f16", "bf16"])
@pytest.mark.parametrize("corrupt", [None, "stale_chunk", "one_element"])
def test_result_check_world2(dtype, corrupt):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_check_worker, args=(r, 2, port, dtype, corrupt, q))
             for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    oks = {r: ok for r, ok, _ in out}
    if corrupt is None:
        assert all(oks.values()), out
    elif corrupt == "stale_chunk":
        assert not any(oks.values()), out
    else:
        # one element off by 1 in 65536: below the check's resolution for
        # 16-bit types, caught for fp32 only when it exceeds the tolerance;
        # the check is for whole stale or missing chunks, not single ulps
        assert all(isinstance(ok, bool) for ok in oks.values())


def test_plan_names():
    assert bench.plan_name("ring_chunked_host") == "ring_chunked"
    assert bench.plan_name("ring_chunked_queued") == "ring_chunked"
    assert bench.plan_name("ring_chunked_mesh_steps") == "ring_chunked_mesh"
    assert bench.plan_name("ring_chunked_mesh_queued") == "ring_chunked_mesh"
    assert bench.plan_name("halving_doubling_queued") == "halving_doubling"


def test_roofline_byte_counts_ring_p8():
    """The ring at P=8 sends 1.75 S on its one link (28 chunks of S/16) and
    the mesh 2S/P per link: the figures DESIGN.md 5 quotes."""
    gloo_amd = pytest.importorskip("gloo_amd")
    n, es = 1 << 20, 4
    S = n * es
    ring = bench.busiest_link_bytes(gloo_amd, "ring_chunked", 0, 8, n, es)
    assert ring == 7 * S // 4
    mesh = bench.busiest_link_bytes(gloo_amd, "ring_chunked_mesh_steps", 0, 8, n, es)
    assert mesh == 2 * S // 8
    hbm = bench.plan_hbm_bytes(gloo_amd, "ring_chunked", 0, 8, n, es)
    assert hbm == 63 * S // 8  # 7.875 S: sends 2 x 1.75 S, reduces 3 x 0.875 S, copies 2 x 0.875 S
