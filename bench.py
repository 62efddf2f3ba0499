"""Benchmark of the integrator hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4] [--spp S]

One step = one full render of the configured workload (all `spp` SamplePixel passes for
every pixel of the image; each pass continues the pixel's XORWOW stream, exactly like the
reference's progressive passes) with inputs already resident in HBM, plus — for N > 1 — the
RCCL gather of the fp32 framebuffer tiles.  Multi-GPU: one process per GPU (torchrun), the
image rows are dealt in interleaved 8-row blocks (row tiling).  Scaling (DESIGN.md
§Multi-GPU): "weak" (default) keeps the pixels per GPU fixed — at N GPUs the image is the
configuration's resolution scaled by sqrt(N) per axis (same aspect and framing; N = 4 is
3840x2160) — and "strong" renders the configuration's image at every N.

Rank 0 prints one JSON line with `roofline` (algorithmic bytes of SURVEY.md §8(d) ÷ the
kernel's HIP-event time) and `cpu_baseline` (the scalar oracle on a bounded sample of the
same workload on the host cores).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mpaths/sec (pixels×spp/s) at 1920×1080; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)


def byte_model(st, paths, node_bytes=32):
    """B_read = sum_segments[76 + 32 n_node + 32 n_prim + (hit ? 40 : 16)] + 16 P.
    node_bytes = 128 for the ordered walk's 4-wide nodes (four child boxes + refs per visit)."""
    return (76 * st["segments"] + node_bytes * st["nodes"] + 32 * st["prims"] + 40 * st["hits"]
            + 16 * st["misses"] + 16 * paths)


def cpu_baseline(cfg, objs, sky, cam, seconds_hint=15.0, threads=None):
    """The oracle (scalar C++ restatement, test infrastructure) on a bounded sample: 16 rows
    spread over the image, full width, `spp_sample` passes (a pixel's passes are sequential, so
    the sample takes the first passes of every sampled pixel)."""
    import oracle
    threads = threads or max(1, min(16, os.cpu_count() or 1))
    W, H = cfg["width"], cfg["height"]
    rows = np.linspace(0, H - 1, 16).astype(np.int32)
    # calibrate with a short run, then size the sample to ~seconds_hint
    spp_probe = 2
    rng = oracle.init_rng(cfg["seed"], W, rows, threads=threads)
    t = time.perf_counter()
    oracle.render(objs, cam, sky, rows, spp_probe, cfg["depth"], rng, threads=threads)
    dt = max(time.perf_counter() - t, 1e-3)
    spp_sample = int(max(2, min(cfg["spp"], spp_probe * seconds_hint / dt)))
    rng = oracle.init_rng(cfg["seed"], W, rows, threads=threads)
    t = time.perf_counter()
    oracle.render(objs, cam, sky, rows, spp_sample, cfg["depth"], rng, threads=threads)
    dt = time.perf_counter() - t
    paths = rows.size * W * spp_sample
    return {
        "value": round(paths / dt / 1e6, 4),
        "unit": "Mpaths/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{rows.size} rows evenly spaced x {W} px x first {spp_sample} of {cfg['spp']} spp of "
                  f"{cfg['name']} ({paths} paths, {dt:.1f} s, std::thread over rows)",
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--spp", type=int, default=None, help="override the config's spp")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--path", default="megakernel", choices=["megakernel", "wavefront"])
    ap.add_argument("--walk", default="ordered", choices=["reference", "ordered"],
                    help="BVH node order: the reference's right-first DFS, or near-first per ray octant "
                         "(CPT_TRAVERSAL_ORDERED, same closest hits; DESIGN.md §Ordered walk)")
    ap.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                    help="weak: pixels per GPU fixed (image grows by sqrt(N) per axis); strong: fixed image")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hbm-probe", action="store_true", help="skip the streaming-read ceiling probe")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--traffic-json", default=None,
                    help="per-launch HBM traffic measured by rocprofv3 PMC (profiles/*.json) for this config")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io, tiling

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # CPT_BENCH_BACKEND=gloo: rehearsal of the N-rank path on a box with fewer GPUs (ranks share
    # devices round-robin, collectives go through host copies).  Never used for reported runs.
    backend = os.environ.get("CPT_BENCH_BACKEND", "nccl")
    if world > 1:
        local_dev = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local_dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    cfg = dict(scenes.CONFIGS[args.config])
    cfg["name"] = args.config
    if args.spp:
        cfg["spp"] = args.spp
    if args.width:
        cfg["width"] = args.width
    if args.height:
        cfg["height"] = args.height
    cfg["seed"] = args.seed
    if args.scaling == "weak" and world > 1 and not (args.width or args.height):
        cfg["width"], cfg["height"] = tiling.weak_scaled_size(cfg["width"], cfg["height"], world)
    W, H, spp, depth = cfg["width"], cfg["height"], cfg["spp"], cfg["depth"]
    objs = scenes.SCENES[cfg["scene"]]()
    sky = texture_io.load_cptex()
    cam = camera_get_copy(scenes.camera_for(W, H))
    rows = tiling.partition_rows(H, world, rank)

    def _all_reduce(x, op=dist.ReduceOp.SUM):
        if backend == "nccl":
            dist.all_reduce(x, op=op)
            return x
        h = x.cpu()
        dist.all_reduce(h, op=op)
        return h.to(x.device)

    r = Renderer(torch.cuda.current_device())
    # One non-default HIP stream for everything: the render kernels (via cpt_set_stream), the
    # RCCL all-gather and the timing events.  (The default stream's handle is 0, which the
    # C-ABI reads as "use the context's own stream".)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    r.set_stream(stream.cuda_stream)
    r.set_scene(objs)
    r.set_env(sky)
    r.set_frame(W, H, rows)
    t_init = time.perf_counter()
    r.init_rng(cfg["seed"])
    torch.cuda.synchronize()
    t_init = time.perf_counter() - t_init

    npix_local = rows.size * W
    max_rows = tiling.max_rows(H, world)
    send = torch.zeros((max_rows * W, 4), dtype=torch.float32, device=dev)
    gathered = torch.zeros((world * max_rows * W, 4), dtype=torch.float32, device=dev) if world > 1 else None
    stitch_idx = torch.from_numpy(tiling.stitch_index(H, W, world)).to(dev) if world > 1 else None
    kernel_events = []
    ordered = args.walk == "ordered"

    def step(timed=False):
        if timed:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
        r.render(cam, spp, depth, path=args.path, ordered=ordered)
        if timed:
            e1.record(stream)
            kernel_events.append((e0, e1))
        if world > 1:
            # RCCL all-gather of the fp32 tiles over xGMI, then the on-device stitch into the
            # full framebuffer (rank 0 keeps it; every rank holds a copy after all-gather)
            r.copy_accum_device(send.data_ptr(), npix_local * 16)
            if backend == "nccl":
                dist.all_gather_into_tensor(gathered, send)
            else:
                g_host = gathered.cpu()
                dist.all_gather_into_tensor(g_host, send.cpu())
                gathered.copy_(g_host)
            fb = gathered.view(world * max_rows, W, 4).index_select(0, stitch_idx)
            return fb
        return None

    # Counting pass (same config, same pixels) for the algorithmic byte model; not timed.  It
    # always walks the reference order: the byte model prices the reference algorithm's node
    # and primitive fetches, whatever walk the timed steps use.
    KEYS = ("segments", "nodes", "prims", "hits", "misses")

    def count_pass(walk_ordered):
        r.init_rng(cfg["seed"])     # both counting passes trace the same paths
        r.reset_stats()
        r.render(cam, spp, depth, stats=True, path=args.path, ordered=walk_ordered)
        torch.cuda.synchronize()
        loc = r.stats()
        v = torch.tensor([loc[k] for k in KEYS], dtype=torch.float64, device=dev)
        if world > 1:
            v = _all_reduce(v)
        return dict(zip(KEYS, (int(x) for x in v.tolist())))

    walk_info = r.walk_info()
    # the box's measured HBM streaming-read ceiling (4 GiB, 10 passes), reported beside the spec peak
    hbm_read_measured = r.measure_read_bandwidth(4 << 30, 10) if not args.no_hbm_probe else None
    walk_node_bytes = 128 if ordered and walk_info["n_wide"] > 0 else 32   # 4-wide walk nodes
    st = count_pass(False)
    walk_counts, walk_diff = None, None
    if ordered:
        # full-size parity of the ordered walk against the reference walk: the two counting
        # passes trace the same paths, so their framebuffers must be bit-identical
        fb_ref = torch.empty((npix_local, 4), dtype=torch.float32, device=dev)
        r.copy_accum_device(fb_ref.data_ptr(), npix_local * 16)
        walk_counts = count_pass(True)
        fb_ord = torch.empty_like(fb_ref)
        r.copy_accum_device(fb_ord.data_ptr(), npix_local * 16)
        torch.cuda.synchronize()
        nd = (fb_ref.view(torch.int32) != fb_ord.view(torch.int32)).any(dim=1).sum().to(torch.float64)
        if world > 1:
            nd = _all_reduce(nd)
        walk_diff = int(nd.item())
        del fb_ref, fb_ord
    r.init_rng(cfg["seed"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # k_megakernel's device time per launch: HIP events recorded around each render on the
    # launch stream (the context launches on torch's current stream, set above)
    avg_kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in kernel_events]))

    t = torch.tensor([elapsed, avg_kernel_ms], dtype=torch.float64, device=dev)
    if world > 1:
        t = _all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, avg_kernel_ms_max = t.tolist()

    if rank == 0:
        paths_total = W * H * spp
        value = paths_total * args.steps / elapsed / 1e6
        # algorithmic bytes of one launch on rank 0's pixels: scale whole-image counts by the
        # pixel share (interleaved blocks keep the shares statistically equal)
        share = npix_local / float(W * H)
        # Algorithmic bytes of one launch (SURVEY.md 8(d) per-unit model x the units the launch
        # processes): the executed walk's own segment/node/primitive counts.  The same model on
        # the reference algorithm's counts (its right-first DFS over its median tree, which
        # visits more nodes for the same closest hits) is reported beside it.
        bytes_ref = byte_model(st, paths_total) * share
        bytes_launch = byte_model(walk_counts, paths_total, walk_node_bytes) * share if walk_counts else bytes_ref
        achieved = bytes_launch / (avg_kernel_ms / 1e3) / 1e9
        achieved_ref_model = bytes_ref / (avg_kernel_ms / 1e3) / 1e9
        # HBM traffic per launch from rocprofv3 PMC passes of this same workload (committed under
        # profiles/, made by tools/profile.sh + tools/pmc_traffic.py); null when none matches.
        traffic = None
        tpath = args.traffic_json or os.path.join(REPO, "profiles", f"traffic_{args.config}_{args.path}_{args.walk}.json")
        if os.path.exists(tpath):
            with open(tpath) as f:
                tj = json.load(f)
            if (tj.get("config") == args.config and tj.get("n_rows") == int(rows.size) and tj.get("spp") == spp
                    and tj.get("path") == args.path and tj.get("walk", "reference") == args.walk):
                traffic = tj.get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mpaths/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (deterministic procedural scene, sky.png fixture)",
            "config": {
                "workload": f"{args.config}: {cfg['scene']} {W}x{H} {spp}spp depth {depth}",
                "width": W, "height": H, "spp": spp, "max_depth": depth, "seed": cfg["seed"],
                "rows_rendered": H, "path": args.path, "walk": args.walk,
                "parallelism": f"row-tiled x{world} (interleaved {tiling.BLOCK_ROWS}-row blocks)" + (
                    ", RCCL all-gather" if world > 1 else ""),
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "hbm_read_measured_gbs": round(hbm_read_measured, 1) if hbm_read_measured else None,
                "achieved_reference_model": round(achieved_ref_model, 2),
                "kernel": "k_megakernel" if args.path == "megakernel" else "wavefront (k_wf_extend+k_wf_shade per bounce)",
                "kernel_avg_ms": round(avg_kernel_ms, 3),
                "bytes_per_launch": int(bytes_launch),
                "byte_model": f"SURVEY.md 8(d): 76 S + {walk_node_bytes if walk_counts else 32} nodes + 32 prims + 40 hits "
                              f"+ 16 misses + 16 P, on walk_counts ({walk_node_bytes}-B nodes: "
                              f"{'4-wide' if walk_node_bytes == 128 else 'binary'} walk tree)",
                "walk_info": walk_info,
                "walk_counts": walk_counts,
                "reference_counts": st,
                "walk_vs_reference_pixels_differing": walk_diff,
            },
            "rng_init_ms": round(t_init * 1e3, 2),
        }
        if not args.no_cpu_baseline:
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, objs, sky, cam, seconds_hint=args.cpu_seconds)
            except Exception as e:  # the baseline must never sink the GPU measurement
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
