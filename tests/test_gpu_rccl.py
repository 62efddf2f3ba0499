"""The multi-GPU code paths that a one-GPU box can execute (round-5 verdict
item 4).  The reference has no multi-GPU path (cuSrc/path_tracer.cu:256-306 renders on one
device, default stream); these are this build's own row-tiling obligations:

* multigpu.TileGather through a real RCCL process group ("nccl" backend, world size 1 on
  cuda:0, `device_id` bound): init_process_group, all_gather_into_tensor and the on-device
  stitch run, and the frame equals the plain render and the oracle bit for bit;
* bench.py under torch.distributed.run with WORLD_SIZE=1: the same process group, collective and
  barriers inside the timed loop, on the bench's own code path;
* cpt_gather_rows' three branches: same device (stitch reads in place), staged peer copy
  (forced through cpt_set_debug_gather, so it runs on one GPU), and the xGMI peer-access read
  between two devices -- skipped when the box has fewer than two GPUs (the pool's boxes have
  one; the driver's 8-GPU SCALE run is where it executes).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from cpppathtracer_amd import Renderer, camera_get_copy, scenes, tiling

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_rank(port, q, W, H, SPP, DEPTH, seed):
    import torch
    import torch.distributed as dist
    from cpppathtracer_amd import Renderer, camera_get_copy, multigpu, scenes, texture_io
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    backend = dist.get_backend()
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as r:
        stream = torch.cuda.Stream()        # the bench's arrangement: one non-default stream
        torch.cuda.set_stream(stream)
        r.set_stream(stream.cuda_stream)
        r.set_scene(scenes.SCENES["s1000"]())
        r.set_env(texture_io.load_cptex())
        g = multigpu.TileGather(W, H, 1, 0, dev, backend="nccl")
        r.set_frame(W, H, g.rows)
        r.init_rng(seed)
        r.render(cam, SPP, DEPTH, ordered=True, schedule="cost")
        fb = g(r)                            # RCCL all_gather_into_tensor + stitch
        torch.cuda.synchronize()
        plain = r.read_accum()
        q.put((backend, fb.cpu().numpy().reshape(H * W, 4), plain))
    dist.barrier()
    dist.destroy_process_group()


def test_tilegather_rccl_world1(oracle_mod, sky):
    import torch.multiprocessing as mp
    W, H, SPP, DEPTH, seed = 96, 52, 2, 16, 77
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_rank, args=(_free_port(), q, W, H, SPP, DEPTH, seed))
    p.start()
    backend, fb, plain = q.get(timeout=240)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl"
    np.testing.assert_array_equal(fb.view(np.uint32), plain.view(np.uint32))
    rows = np.array([0, 7, 8, 25, 51], dtype=np.int32)
    cam = camera_get_copy(scenes.camera_for(W, H))
    orng = oracle_mod.init_rng(seed, W, rows, threads=8)
    oacc, _, _, _ = oracle_mod.render(scenes.SCENES["s1000"](), cam, sky, rows, SPP, DEPTH, orng, threads=8)
    np.testing.assert_array_equal(fb.reshape(H, W, 4)[rows].reshape(-1, 4).view(np.uint32), oacc.view(np.uint32))


def test_bench_under_torchrun_world1():
    """bench.py's own N-rank code path at WORLD_SIZE=1: process group, RCCL all-gather + stitch
    inside the timed steps, barriers, max-over-ranks all-reduce, walk parity count."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "1", "--config", "c4", "--width", "128", "--height", "64", "--spp", "4",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-hbm-probe"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    out = json.loads(line)
    assert out["n_gpus"] == 1
    assert "RCCL all-gather" in out["config"]["parallelism"]
    assert out["roofline"]["walk_vs_reference_pixels_differing"] == 0
    assert out["value"] > 0


def _tiles_and_mono(objs, sky, W, H, spp, depth, seed, world, devices):
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as m:
        m.set_scene(objs)
        m.set_env(sky)
        m.set_frame(W, H)
        m.init_rng(seed)
        m.render(cam, spp, depth, aux=True, ordered=True, schedule="cost", sync=True)
        mono = m.read_accum(), m.read_aux()
    tiles = []
    for rank in range(world):
        t = Renderer(devices[rank % len(devices)])
        tiles.append(t)
        t.set_scene(objs)
        t.set_env(sky)
        t.set_frame(W, H, tiling.partition_rows(H, world, rank))
        t.init_rng(seed)
        t.render(cam, spp, depth, aux=True, ordered=True, schedule="cost")   # asynchronous
    return tiles, mono


def _gather_check(frame, tiles, mono, want_modes):
    try:
        for t in tiles:
            frame.gather_rows(t)
        acc, (nrm, dep) = frame.read_accum(), frame.read_aux()
        modes = [frame.last_gather_mode(t) for t in tiles]
    finally:
        for t in tiles:
            t.close()
    assert modes == want_modes
    np.testing.assert_array_equal(acc.view(np.uint32), mono[0].view(np.uint32))
    np.testing.assert_array_equal(nrm.view(np.uint32), mono[1][0].view(np.uint32))
    np.testing.assert_array_equal(dep, mono[1][1])


@pytest.mark.parametrize("staged", [False, True])
def test_gather_rows_branches_one_device(sky, staged):
    objs = scenes.scene_s1000(n=200)
    W, H, spp, depth, seed, world = 72, 40, 2, 12, 5, 3
    tiles, mono = _tiles_and_mono(objs, sky, W, H, spp, depth, seed, world, [0])
    with Renderer(0) as frame:
        frame.set_frame(W, H)
        frame.set_debug_gather(staged)
        assert frame.last_gather_mode(tiles[0]) is None
        _gather_check(frame, tiles, mono, ["staged" if staged else "same_device"] * world)


def test_gather_rows_peer_two_devices(sky):
    from cpppathtracer_amd.renderer import device_count
    if device_count() < 2:
        pytest.skip("one GPU on this box: the xGMI peer branch runs on multi-GPU nodes only")
    objs = scenes.scene_s1000(n=200)
    W, H, spp, depth, seed, world = 72, 40, 2, 12, 5, 2
    tiles, mono = _tiles_and_mono(objs, sky, W, H, spp, depth, seed, world, [1])
    with Renderer(0) as frame:
        frame.set_frame(W, H)
        _gather_check(frame, tiles, mono, ["peer"] * world)


def test_tilegather_copy_ordered_against_torch_stream(sky):
    """cpt_copy_accum_device orders the tile copy against torch's stream with no host wait
    (round 6; round 5 found one 8-rank stitched frame with pass counts of 0 where a late zero
    fill of TileGather's send buffer on torch's stream landed after the copy on the context's own
    stream).  Torch's stream is held busy by a long sleep right before each write of `send` it
    queues -- the buffers' zero fill, then a NaN fill standing for a collective still using the
    buffer -- while the context (on its own non-blocking stream) is idle: an unordered copy would
    run first and be overwritten.  The frame must equal the render bit for bit both times."""
    import torch
    from cpppathtracer_amd import multigpu
    W, H, spp, depth, seed = 96, 52, 2, 16, 41
    dev = torch.device("cuda", 0)
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as r:   # its own stream: nothing orders it with torch's
        r.set_scene(scenes.scene_s1000(n=200))
        r.set_env(sky)
        r.set_frame(W, H, tiling.partition_rows(H, 1, 0))
        r.init_rng(seed)
        r.render(cam, spp, depth, ordered=True, sync=True)
        want = r.read_accum()
        torch.cuda._sleep(300_000_000)                 # ~0.1 s of torch's stream
        g = multigpu.TileGather(W, H, 1, 0, dev, backend="gloo")   # its zero fills: behind the sleep
        got = g(r).reshape(H * W, 4).cpu().numpy()
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
        torch.cuda._sleep(300_000_000)
        g.send.fill_(float("nan"))                     # a late writer of `send` on torch's stream
        got = g(r).reshape(H * W, 4).cpu().numpy()
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def test_bench_two_ranks_balanced_partition():
    """bench.py --gpus 2 --partition balanced, the two ranks sharing this box's GPU (gloo host
    copies): every rank deals the 8-row blocks by the same whole-frame pilot (tiling.lpt_owner),
    the stitched frame's walk parity count is 0 and the line names the partition."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--config", "c4", "--width", "256",
           "--height", "120", "--spp", "8", "--steps", "1", "--warmup", "1", "--partition", "balanced",
           "--no-cpu-baseline", "--no-hbm-probe", "--no-strong-check"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CPT_BENCH_BACKEND="gloo")
    r = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["n_gpus"] == 2
    assert "pilot's cost" in out["config"]["parallelism"]
    assert out["roofline"]["walk_vs_reference_pixels_differing"] == 0
    assert out["partition_pilot_ms"] > 0
