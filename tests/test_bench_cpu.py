"""bench.py's host-side logic on CPU: the per-candidate result check (a
world_size-2 gloo process group, as the N>1 bench runs it), candidate
naming, and the algorithmic byte counts the roofline fields are built from."""
import json
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
    assert bench.plan_name("ring_chunked_plain_narrow") == "ring_chunked"
    assert bench.plan_name("ring_chunked_mesh_steps") == "ring_chunked_mesh"
    assert bench.plan_name("ring_chunked_mesh_system") == "ring_chunked_mesh"
    assert bench.plan_name("halving_doubling_host") == "halving_doubling"
    assert bench.plan_name("ring_chunked_dma") == "ring_chunked"
    assert bench.plan_name("halving_doubling_dma") == "halving_doubling"
    assert bench.golden_plan("ring_chunked_dma") == "ring_chunked"
    # every default and opt-in candidate names a schedule the planner knows
    for c in bench.DEFAULT_CANDIDATES + bench.EXTRA_CANDIDATES + bench.EXTRA_ALTS:
        assert bench.plan_name(c) in ("ring_chunked", "ring_chunked_mesh",
                                      "halving_doubling"), c


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


def test_fused_hbm_bytes_ring_p8():
    """The plan kernel's reduce-and-forward: 26 of the ring's 28 sends at P=8
    re-use the pass that wrote their range, so they only write the receiver's
    copy (7.875 S - 26/16 S = 6.25 S), and 12 of its 14 partial sums are not
    stored in the buffer at all (plan.h StepSync::keep): 6.25 S - 12/16 S =
    5.5 S per step."""
    gloo_amd = pytest.importorskip("gloo_amd")
    n, es = 1 << 20, 4
    S = n * es
    hbm = bench.plan_hbm_bytes(gloo_amd, "ring_chunked", 0, 8, n, es, fused=True)
    assert hbm == 88 * S // 16


def test_fused_hbm_bytes_halving_doubling_p8():
    """Halving-doubling's partial reduce-and-forward (plan.h StepSync::pre):
    a reduce-scatter step's reduction stores the half sent on next straight
    into that peer's slot (and not into the buffer: the allgather overwrites
    it), an allgather COPY also stores into the next peer's slot: 7.875 S -
    1/16 S (the one exact fusion) - 1.125 S (reads and dead writes the
    partial ones save) = 6.625 S at P = 8 (configs[3])."""
    gloo_amd = pytest.importorskip("gloo_amd")
    n, es = 1 << 20, 4
    S = n * es
    hbm = bench.plan_hbm_bytes(gloo_amd, "halving_doubling", 0, 8, n, es, fused=True)
    assert hbm == 106 * S // 16
    sy = gloo_amd.plan_sync("halving_doubling", 0, 8, n, 1)["steps"]
    steps = gloo_amd.plan("halving_doubling", 0, 8, n)[0]
    partial = [(i, y[9]) for i, y in enumerate(sy) if steps[i][0] in (2, 3) and y[9] >= 0]
    assert len(partial) == 4
    for i, j in partial:
        assert steps[j][0] == 0 and sy[j][9] == i and sy[j][10:12] == sy[i][10:12]


def test_north_star_block_p8():
    S = 256 << 20
    ns = bench.north_star_block(S, 8, 3.5e-3, 3.4e-3, "devsteps", 100 * S // 16)
    # 1.75 S on the one link at 153 GB/s = 3.07 ms; the 80 % target 3.84 ms
    assert ns["link_bytes_per_step"] == 7 * S // 4
    assert abs(ns["link_bound_ms"] - 3.0704) < 1e-3
    assert abs(ns["target_ms"] - 3.838) < 1e-3
    assert abs(ns["link_frac"] - 3.0704 / 3.5) < 1e-3
    assert ns["meets_target"] is True  # 3.5 ms <= 3.84 ms
    assert bench.north_star_block(S, 8, 4.0e-3, 4.0e-3, "devsteps", 0)["meets_target"] is False


def _ring_run(t, engine, tr):
    return {"t": t, "p50": t, "engine": engine, "hbm": 100 * (256 << 20) // 16,
            "transport": "x", "tr": tr, "fast": False, "sync": "narrow"}


def test_north_star_section_carries_every_ring():
    """the plan kernel (CU stores), the host-issued DMA ring
    and the DMA ring with on-GPU hand-offs all appear, each with its own link
    fraction, measured-link fraction against the probe of ITS transport, and
    reference-digest match; the top level repeats the fastest one."""
    S = 256 << 20
    links = {"ring_dma_GBps": 140.0, "ring_kernel_GBps": 120.0}
    runs = {"ring_chunked": _ring_run(3.5e-3, "devsteps", ("dma", 1, 0)),
            "ring_chunked_host": _ring_run(3.4e-3, "steps", ("dma", 1, 0)),
            "ring_chunked_dma": _ring_run(3.3e-3, "dmasteps", ("dma", 1, 0))}
    ns = bench.north_star_section(S, 8, runs, links, {a: True for a in runs}, {})
    pk, host = ns["rings"]["ring_chunked"], ns["rings"]["ring_chunked_host"]
    dma = ns["rings"]["ring_chunked_dma"]
    for b in (pk, host, dma):
        for k in ("ms_per_step", "link_frac", "measured_link_frac", "reference_digest_match"):
            assert k in b, (k, b)
    assert pk["measured_link"] == "ring_kernel_GBps" and host["measured_link"] == "ring_dma_GBps"
    assert dma["measured_link"] == "ring_dma_GBps"
    assert abs(pk["measured_link_frac"] - pk["link_GBps"] / 120.0) < 1e-3
    assert ns["candidate"] == "ring_chunked_dma"  # the fastest one
    # one of them failed: it still appears, with its error
    ns = bench.north_star_section(S, 8, {"ring_chunked": runs["ring_chunked"]}, None, {},
                                  {"ring_chunked_host": "IoException: boom"})
    assert ns["rings"]["ring_chunked_host"] == {"error": "IoException: boom"}
    assert ns["candidate"] == "ring_chunked" and "measured_link_frac" not in ns
    ns = bench.north_star_section(S, 8, {}, None, {}, {})
    assert "error" in ns and set(ns["rings"]) == set(bench.NS_RINGS)
    # the opt-in DMA-steps ring appears only when it was timed (or failed)
    ns = bench.north_star_section(S, 8, {"ring_chunked": runs["ring_chunked"]}, None, {}, {})
    assert set(ns["rings"]) == set(bench.NS_RINGS)


@pytest.mark.parametrize("world", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("mib", [4, 256, 1024])
def test_link_probe_moves_at_least_the_candidates_per_link_volume(world, mib):
    """the probe's ceiling for a pattern must come from at
    least the per-link volume the candidates move in one run -- the mesh's
    2S/P per link, a ring chunk S/2P per step -- and never from a
    latency-bound size (>= 64 MiB), on every link the pattern uses."""
    gloo_amd = pytest.importorskip("gloo_amd")
    S = mib << 20
    b = bench.probe_link_bytes(S, world)
    n = S // 4
    mesh = bench.busiest_link_bytes(gloo_amd, "ring_chunked_mesh_steps", 0, world, n, 4)
    ring_chunk = S // (2 * world)
    assert b >= mesh and b >= ring_chunk and b >= 64 << 20 and b % 4096 == 0
    assert bench.PROBE_REPS >= 10 and bench.PROBE_BLOCKS >= 512


def test_twoshot_hbm_bytes_p8():
    assert bench.twoshot_hbm_bytes(256 << 20, 8) == int(5.5 * (256 << 20))


def test_n_gt_1_traffic_record_is_keyed_by_candidate():
    rec = bench.load_traffic("ring_chunked:f32:256MiB:P8", record=True)
    # 5.5 S since the dead-write elision (6.25 S before, kept under "previous")
    assert rec and 0.98 < rec["hbm_bytes_per_launch"] / (5.5 * (256 << 20)) < 1.1
    rec = bench.load_traffic("ring_chunked_mesh:f32:256MiB:P8", record=True)
    assert rec and 0.98 < rec["hbm_bytes_per_launch"] / bench.twoshot_hbm_bytes(256 << 20, 8) < 1.1


def test_candidate_lists_default_is_small():
    class A:
        algo, schedule, candidates, no_alt = "ring_chunked", "auto", "default", False
    c, alts = bench.candidate_lists(A)
    assert c[0] == "ring_chunked" and len(c) + len(alts) <= 6
    assert not any(x.endswith(("_fast", "_system")) for x in c + alts)
    # the ring and the mesh both by CU stores and by DMA (the node run's open question)
    assert {"ring_chunked", "ring_chunked_mesh", "ring_chunked_host", "ring_chunked_dma",
            "ring_chunked_mesh_steps"} <= set(c)
    assert {d for d in bench.DMA_CANDIDATES if not d.endswith("_pipe")} <= set(c)
    A.candidates = "all"
    c, alts = bench.candidate_lists(A)
    assert "ring_chunked_fast" in c and "ring_chunked_system" in c
    assert "halving_doubling_host" in alts


def test_metric_name_follows_dtype():
    assert bench.metric_name("f32") == (
        "allreduce GB/s (device-resident, fp32) at 1/2/4/8 MI355X; % HBM|xGMI roofline")
    assert "f16" in bench.metric_name("f16")


def _info(same, atomics=True, access=True, stores=False):
    return {"device": 1, "same_gpu": same, "can_access_peer": None if same else access,
            "native_atomics": None if same else atomics, "flag_stores": stores}


def test_transport_health_distinct_gpus():
    ok = {"ring_chunked": {"peer_copies": 0, "device_copies": 0, "kernel_copies": 0,
                           "device_kernels": 3, "bytes": 0, "host_folds": 0}}
    infos = [[_info(False)], [_info(False)]]
    st, err = bench.transport_health(infos, [ok, ok])
    assert err is None and st["ranks_on_distinct_gpus"]
    # a hipMemcpyAsync fallback on one rank is an error on the node
    bad = {"ring_chunked_host": dict(ok["ring_chunked"], device_copies=28)}
    st, err = bench.transport_health(infos, [ok, bad])
    assert err is not None and "hipMemcpyAsync" in err and "rank 1" in err
    # a link without native atomics (flag words written with stores)
    infos2 = [[_info(False, atomics=False, stores=True)], [_info(False)]]
    st, err = bench.transport_health(infos2, [ok, ok])
    assert err is not None and "atomics" in err and st["flag_stores"] == [True, False]


def test_transport_health_shared_gpu_rehearsal_is_not_an_error():
    """Ranks sharing one GPU (the one-GPU rehearsal) copy with hipMemcpyAsync
    by design; that is reported, not an error."""
    st = {"ring_chunked_host": {"peer_copies": 0, "device_copies": 28, "kernel_copies": 0,
                                "device_kernels": 0, "bytes": 1, "host_folds": 0}}
    status, err = bench.transport_health([[_info(True)], [_info(True)]], [st, st])
    assert err is None and not status["ranks_on_distinct_gpus"]


@pytest.mark.parametrize("dtype", ["f32", "f16", "bf16"])
def test_splitmix_fill_matches_oracle_generator(dtype):
    """bench.py regenerates SURVEY 8d's inputs in torch (int64 with masked
    shifts); they must be the oracle generator's bits, or the reference
    digests in tests/golden/bench_golden.json could never match."""
    import numpy as np
    from oracle import oracle as O
    code = {"f32": O.FLOAT32, "f16": O.FLOAT16, "bf16": O.BFLOAT16}[dtype]
    for rank in (0, 1, 5):
        n = 70001
        t = bench.splitmix_fill(torch, n, dtype, "cpu", bench.SEED, rank, chunk=20000)
        got = t.view(torch.int16 if t.element_size() == 2 else torch.int32).numpy()
        exp = O.fill(code, n, 0, seed=bench.SEED, rank=rank)
        assert np.array_equal(got.view(np.uint8), exp.view(np.uint8))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_reference_cases_for_the_bench_workload(world):
    """The N > 1 default workload (256 MiB fp32 per rank) has the reference's
    digests for both plans, and their recorded input digests are those of
    the generator bench.py uses (checked on a prefix-independent basis: the
    full 256 MiB input of rank 1)."""
    n = (256 << 20) // 4
    cases = bench.reference_cases(world, n, "f32")
    assert set(cases) == {"ring_chunked", "halving_doubling"}
    x = bench.splitmix_fill(torch, n, "f32", "cpu", bench.SEED, 1)
    assert bench.sha256_of(x) == cases["ring_chunked"]["input_sha256"][1]
    assert bench.golden_plan("ring_chunked_mesh") == "ring_chunked"
    assert bench.golden_plan("halving_doubling_system") == "halving_doubling"
    assert bench.reference_cases(3, n, "f32") == {}


def test_reference_cases_cfg5():
    cases = bench.reference_cases(8, 1 << 29, "f16")
    assert set(cases) == {"ring_chunked"}


def test_failure_line_is_one_json_line_with_the_error():
    import argparse
    import json
    ns = argparse.Namespace(dtype="f32", steps=None, warmup=5, algo="ring_chunked", size_mib=256)
    line = bench.failure_line(ns, 8, RuntimeError("every candidate failed: {...}"))
    s = json.dumps(line)
    assert "\n" not in s
    d = json.loads(s)
    assert d["value"] is None and d["n_gpus"] == 8 and "every candidate failed" in d["error"]
    assert d["metric"] == bench.metric_name("f32")


def test_live_pmc_traffic_off_and_failure_paths(monkeypatch):
    """N = 1 roofline.traffic is measured in the run by rocprofv3 --pmc child
    passes; --no-pmc (the children themselves) and a missing rocprofv3 fall
    back to the stored pass."""
    class A:
        no_pmc, dtype, size_mib = True, "f32", 256
    assert bench.live_pmc_traffic(A) is None
    A.no_pmc = False
    import shutil
    monkeypatch.setattr(shutil, "which", lambda name: None)
    assert bench.live_pmc_traffic(A) is None


# ---------------------------------------------------------------------------
# The N > 1 line's claims: what a rehearsal and a
# degraded node transport may say.
# ---------------------------------------------------------------------------
def _stats(peer=0, device=0, kernel=0, kernels=0, nbytes=0):
    return {"peer_copies": peer, "device_copies": device, "kernel_copies": kernel,
            "device_kernels": kernels, "bytes": nbytes, "host_folds": 0, "done_events": 0}


def _line(world=8):
    """The N > 1 line's north-star and roofline parts, as bench_multi builds
    them, for a healthy-looking 3.5 ms plan-kernel ring and 3.3 ms DMA rings."""
    S = 256 << 20
    links = {"ring_dma_GBps": 140.0, "ring_kernel_GBps": 120.0}
    runs = {"ring_chunked": _ring_run(3.5e-3, "devsteps", ("dma", 1, 0)),
            "ring_chunked_host": _ring_run(3.3e-3, "steps", ("dma", 1, 0)),
            "ring_chunked_dma": _ring_run(3.3e-3, "dmasteps", ("dma", 1, 0))}
    ns = bench.north_star_section(S, world, runs, links, {a: True for a in runs}, {})
    return {"value": S / 3.3e-3 / 1e9, "north_star": ns,
            "roofline": {"frac": 0.93, "link_measured": dict(links, frac=0.97)}}


def _node_stats(host_stats):
    return {"ring_chunked": _stats(kernels=24, nbytes=7 << 28),
            "ring_chunked_mesh": _stats(kernels=24, nbytes=7 << 28),
            "ring_chunked_host": host_stats,
            "ring_chunked_dma": _stats(peer=28 * 24, nbytes=7 << 28),
            "ring_chunked_mesh_steps": _stats(peer=14 * 24, nbytes=7 << 28)}


def _meets(res):
    ns = res["north_star"]
    return [b.get("meets_target") for b in [ns] + list(ns["rings"].values())]


def _infos(world, **kw):
    return [[_info(False, **kw) for _ in range(world - 1)] for _ in range(world)]


def test_node_line_healthy_transport_keeps_its_claims():
    """8 ranks on 8 distinct GPUs, every DMA candidate made peer copies,
    native atomics everywhere: no error, the north-star verdict stands."""
    world = 8
    health, err = bench.transport_health(
        _infos(world), [_node_stats(_stats(peer=28 * 24, nbytes=7 << 28))] * world)
    res = bench.apply_transport_verdict(_line(world), health, err)
    assert err is None and "error" not in res and "rehearsal" not in res
    assert all(m is True for m in _meets(res))
    assert res["roofline"]["frac"] == 0.93
    assert res["north_star"]["link_frac"] is not None


@pytest.mark.parametrize("case", ["device_copies", "no_atomics", "no_peer_copies", "no_access"])
def test_node_line_degraded_transport_carries_an_error_and_no_verdict(case):
    """a synthetic 8-distinct-GPU record whose transport is
    degraded -- a hipMemcpyAsync fallback in the DMA ring, a link without
    native atomics, a DMA ring that made no peer copies, a peer GPU that
    cannot be accessed -- puts an error in the line and never a
    meets_target."""
    world = 8
    host = _stats(peer=28 * 24, nbytes=7 << 28)
    kw = {}
    if case == "device_copies":
        host = _stats(peer=20, device=8, nbytes=7 << 28)
    elif case == "no_peer_copies":
        host = _stats(nbytes=7 << 28)
    elif case == "no_atomics":
        kw = {"atomics": False, "stores": True}
    else:
        kw = {"access": False}
    stats = [_node_stats(_stats(peer=28 * 24, nbytes=7 << 28))] * (world - 1) + [_node_stats(host)]
    health, err = bench.transport_health(_infos(world, **kw), stats)
    assert health["ranks_on_distinct_gpus"] and err is not None
    res = bench.apply_transport_verdict(_line(world), health, err)
    assert res["error"] == err
    assert all(m is None for m in _meets(res)), _meets(res)
    assert res["north_star"]["error"] == err
    line = json.loads(json.dumps(res))
    assert "meets_target\": true" not in json.dumps(line)


def test_rehearsal_line_makes_no_link_claims():
    """ranks sharing one GPU moved no byte over a link, so
    link_frac, meets_target, measured_link_frac and roofline.frac are null
    and the line says it is a rehearsal (the shared-GPU copies are not an
    error)."""
    world = 8
    same = [[_info(True) for _ in range(world - 1)] for _ in range(world)]
    health, err = bench.transport_health(
        same, [_node_stats(_stats(device=28 * 24, nbytes=7 << 28))] * world)
    assert err is None and not health["ranks_on_distinct_gpus"]
    res = bench.apply_transport_verdict(_line(world), health, err)
    assert res["rehearsal"] == bench.REHEARSAL_NOTE
    assert res["roofline"]["frac"] is None and res["roofline"]["link_measured"]["frac"] is None
    for b in [res["north_star"]] + list(res["north_star"]["rings"].values()):
        for k in bench.LINK_CLAIMS:
            assert b[k] is None, (k, b)
    assert res["value"] > 0  # the measured time itself stands


def test_multi_line_value_is_algbw_and_workload_names_the_schedule():
    """value = algbw = S / t (gloo/benchmark/runner.cc:488-496);
    the mesh headline is named as such in config.workload."""
    import inspect
    src = inspect.getsource(bench.bench_multi)
    assert '"value": round(algbw, 3)' in src and "world * S / t" in src  # aggregate kept aside
    assert '"aggregate_GBps"' in src
    assert bench.multi_workload("ring_chunked", "ring_chunked", "f32", 256) == \
        "allreduce_ring_chunked_fp32_256MiB_per_rank"
    assert bench.multi_workload("ring_chunked", "ring_chunked_mesh", "f32", 256) == \
        "allreduce_ring_chunked_mesh_schedule_fp32_256MiB_per_rank"
    assert bench.multi_workload("halving_doubling", "halving_doubling", "f16", 1024) == \
        "allreduce_halving_doubling_f16_1024MiB_per_rank"


def test_reduce_segments_follow_the_library():
    """bench.py scales the per-dispatch PMC bytes by the dispatches one
    glx_reduce call makes: equal segments of at most
    glx_reduce_segment_bytes() (256 MiB) per stream."""
    assert bench.reduce_segments(256 << 20) == 1
    assert bench.reduce_segments((256 << 20) + 16) == 2
    assert bench.reduce_segments(1 << 30) == 4


def _refill_worker(rank, world, port, fault, use_digest, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n = 1 << 14
    srcs = [bench.synthetic(torch, n, "f32", torch.device("cpu"), 77 + r) for r in range(world)]
    total = srcs[0].clone()
    for x in srcs[1:]:
        total = total + x
    golden = bench.sha256_of(total) if use_digest else None
    buf = torch.empty_like(total)
    calls = [0]

    def run_once():
        k = calls[0]
        calls[0] += 1
        buf.copy_(total)
        if fault == "stale_run" and k == 3 and rank == 1:
            # one rank's run 3 kept a chunk of its own input (a stale hand-off)
            buf[:n // 8] = srcs[rank][:n // 8]
        elif fault == "one_ulp" and k == 1 and rank == 0:
            # one element one ulp off: below result_check's tolerance, but the
            # ranks' bits now differ (and the reference digest, if any)
            buf[5] = torch.nextafter(buf[5], torch.tensor(2.0))
        return buf

    ok, detail, last = bench.refill_checks(torch, dist, srcs[rank], run_once, runs=5,
                                           golden_sha=golden)
    q.put((rank, ok, detail, calls[0]))
    dist.destroy_process_group()


@pytest.mark.parametrize("fault,use_digest", [(None, True), (None, False),
                                              ("stale_run", True), ("stale_run", False),
                                              ("one_ulp", True), ("one_ulp", False)])
def test_refill_checks_catch_a_wrong_run_on_any_rank(fault, use_digest):
    """after a candidate's timing, K >= 5 refilled runs are
    checked on EVERY rank (bench.refill_checks) -- a stale hand-off on one
    rank in one run fails the candidate on all ranks alike, and says which
    run and rank; a one-ulp difference below result_check's tolerance is
    still caught by the cross-rank checksum (and the digest)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_refill_worker, args=(r, 2, port, fault, use_digest, q))
             for r in range(2)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [o[3] for o in out] == [bench.REFILL_RUNS] * 2 and bench.REFILL_RUNS >= 5
    oks = [o[1] for o in out]
    details = [o[2] for o in out]
    assert details[0]["bad"] == details[1]["bad"]  # every rank reaches the same verdict
    if fault is None:
        assert oks == [True, True] and details[0]["bad_count"] == 0
        assert details[0]["digest_checked"] is use_digest
    elif fault == "stale_run":
        assert oks == [False, False]
        b = details[0]["bad"]
        assert {(e["run"], e["rank"]) for e in b} >= {(3, 1)}
        assert not [e for e in b if e["run"] != 3]
        assert any(e["result_check"] is False for e in b if e["rank"] == 1)
        if use_digest:
            assert any(e["digest"] is False for e in b if e["rank"] == 1)
    else:
        assert oks == [False, False]
        b = details[0]["bad"]
        assert b and all(e["run"] == 1 and not e["ranks_agree"] for e in b)
        assert all(e["result_check"] for e in b)  # below the weighted sum's resolution
        if use_digest:
            assert [e["digest"] for e in b if e["rank"] == 0] == [False]
