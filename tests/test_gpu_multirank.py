"""bench.py's N-rank path through libcpt.so on one GPU: N ranks (gloo, all on cuda:0) each
render their interleaved 8-row blocks with the HIP megakernel (timed instantiation, cost
schedule), the fp32 tiles are all-gathered and stitched on the device (multigpu.TileGather),
and the stitched frame must equal the single-rank render and the oracle bit for bit.  The
second case is C5's frame (3840x2160) in C5's 8-way partition, with the tail-consolidating
kernel forced (the one an 8-GPU C5 run uses), at 2 spp."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DEPTH = 16
CASES = [(96, 52, 3, 2, None, None), (3840, 2160, 2, 8, True, [0, 7, 8, 1079, 1080, 2151, 2159])]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, W, H, SPP, consolidate):
    import torch
    import torch.distributed as dist
    from cpppathtracer_amd import Renderer, camera_get_copy, multigpu, scenes, texture_io
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as r:
        r.set_scene(scenes.SCENES["s1000"]())
        r.set_env(texture_io.load_cptex())
        g = multigpu.TileGather(W, H, world, rank, dev, backend="gloo")
        r.set_frame(W, H, g.rows)
        r.init_rng(scenes.DEFAULT_SEED)
        r.render(cam, SPP, DEPTH, ordered=True, schedule="cost", sync=True, consolidate=consolidate)
        fb = g(r)
        torch.cuda.synchronize()
        if rank == 0:
            q.put(fb.cpu().numpy().reshape(H * W, 4))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("W,H,SPP,world,consolidate,oracle_rows", CASES)
def test_ranks_stitch_equals_monolithic_and_oracle(oracle_mod, sky, W, H, SPP, world, consolidate, oracle_rows):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q, W, H, SPP, consolidate)) for r in range(world)]
    for p in procs:
        p.start()
    fb = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    from cpppathtracer_amd import Renderer, camera_get_copy, scenes
    cam = camera_get_copy(scenes.camera_for(W, H))
    with Renderer(0) as r:
        r.set_scene(scenes.SCENES["s1000"]())
        r.set_env(sky)
        r.set_frame(W, H)
        r.init_rng(scenes.DEFAULT_SEED)
        r.render(cam, SPP, DEPTH, ordered=True, schedule="cost", sync=True)
        mono = r.read_accum()
    bad = np.any(fb.view(np.uint32) != mono.view(np.uint32), axis=1)
    if bad.any():   # which side is wrong: rows, pass counts, and the stitched frame vs the oracle
        ys = np.unique(np.nonzero(bad)[0] // W)
        print(f"{bad.sum()} pixels differ in {ys.size} rows (first {ys[:16].tolist()}); pass counts "
              f"stitched {np.unique(fb[bad, 3])[:8].tolist()} monolithic {np.unique(mono[bad, 3])[:8].tolist()}")
    np.testing.assert_array_equal(fb.view(np.uint32), mono.view(np.uint32))
    rows = np.arange(H, dtype=np.int32) if oracle_rows is None else np.array(oracle_rows, dtype=np.int32)
    orng = oracle_mod.init_rng(scenes.DEFAULT_SEED, W, rows, threads=8)
    oacc, _, _, _ = oracle_mod.render(scenes.SCENES["s1000"](), cam, sky, rows, SPP, DEPTH, orng, threads=8)
    got = fb.reshape(H, W, 4)[rows].reshape(-1, 4)
    np.testing.assert_array_equal(got.view(np.uint32), oacc.view(np.uint32))
