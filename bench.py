"""Benchmark of the integrator hot path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c4|c5|...] [--spp S]
                    [--scaling strong|weak] [--schedule cost|tiles] [--consolidate auto|on|off]

One step = one full render of the configured workload (all `spp` SamplePixel passes for
every pixel of the image; each pass continues the pixel's XORWOW stream, exactly like the
reference's progressive passes) with inputs already resident in HBM, plus — for N > 1 — the
gather of the fp32 framebuffer tiles.

Multi-GPU: one process per GPU.  Run under torchrun (WORLD_SIZE set; it must equal --gpus),
or give `--gpus N` without a launcher: the parent then starts N ranks through
`torch.distributed.run` before it touches the GPU, relays rank 0's line and exits with the
launcher's status.  The image rows are dealt to the ranks in interleaved 8-row blocks (row
tiling).  Scaling: "strong" (default) renders the
configuration's image (C4: 1920x1080, the metric's resolution; the north star's "1920x1080 at
1, 2, 4 and 8 GPUs") at every N -- its ceiling is the longest pixel chain, DESIGN.md
§Multi-GPU; "weak" keeps the pixels per GPU fixed by scaling each axis by sqrt(N) (N = 4:
3840x2160, C5's frame).  With N > 1 the other mode is timed too over the same ranks and
reported as a side field (`weak_scaling` / `strong_scaling`).

--dispatch K times the reference's own per-pass loop instead (DispatchRay: 1-spp render +
Denoising + Mix + BGRA8 to the host, path_tracer.cu:256-306) with one and with several row-tile
contexts, and prints a separate JSON line (not the headline metric).

Rank 0 prints one JSON line with `roofline` (SURVEY.md §8(d) algorithmic bytes ÷ the kernel's
HIP-event time, beside the rocprof-measured HBM bytes and VALU issue of a committed profile of
the same workload) and `cpu_baseline` (the scalar oracle on a bounded sample of the same
workload on the host cores, 1 thread and all usable cores).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "Mpaths/sec (pixels×spp/s) at 1920×1080; achieved HBM GB/s vs peak"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)
WIDE_NODE_BYTES = 112   # a 4-wide walk node visit reads 7 x 16 B of the compact image (cpt_path.hpp)
LDS_TREE_NODES = 512    # the LDS kernels stage the image's first 512 nodes (cpt_path.hpp lds_tree_nodes)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks (GPUs); without a launcher N > 1 spawns N ranks via torch.distributed.run")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c4", choices=["c1", "c2", "c3", "c4", "c5"])
    ap.add_argument("--spp", type=int, default=None, help="override the config's spp")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--objects", type=int, default=None,
                    help="S1000 generator with this many primitives instead of 1000 (BVH-size scaling runs)")
    ap.add_argument("--path", default="megakernel", choices=["megakernel", "wavefront"])
    ap.add_argument("--walk", default="ordered", choices=["reference", "ordered"],
                    help="BVH node order: the reference's right-first DFS, or near-first per ray octant "
                         "(CPT_TRAVERSAL_ORDERED, same closest hits; DESIGN.md §Ordered walk)")
    ap.add_argument("--consolidate", default="auto", choices=["auto", "on", "off"],
                    help="megakernel tail consolidation (auto: on for ranks of more than 1 and at most 4 pixels per lane, spp >= 512)")
    ap.add_argument("--schedule", default="auto", choices=["auto", "cost", "tiles"],
                    help="megakernel pixel dequeue order: 8x8 tiles heaviest first from a pilot pass "
                         "(CPT_SCHEDULE_COST), or tiles in row-major order; auto: cost from 64 passes up "
                         "(the pilot is one pass: a quarter of C1's 4-pass frame, C1 1043 vs 1556 Mpaths/s)")
    ap.add_argument("--partition", default="interleaved", choices=["interleaved", "balanced"],
                    help="N > 1: each rank's rows -- interleaved 8-row blocks (block b to rank b mod N), or the "
                         "blocks dealt by a 4-pass pilot of the whole frame, heaviest first to the least-loaded "
                         "rank (tiling.lpt_owner; every rank computes the same partition at setup)")
    ap.add_argument("--scaling", default="strong", choices=["strong", "weak"],
                    help="strong (default): the config's image (C4: 1920x1080, the metric's resolution) at every N; "
                         "weak: pixels per GPU fixed (image grows by sqrt(N))")
    ap.add_argument("--no-strong-check", action="store_true",
                    help="N > 1: skip the extra timing in the other scaling mode (weak-scaled frame, or with "
                         "--scaling weak the config's own frame strong-scaled)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-hbm-probe", action="store_true", help="skip the streaming-read ceiling probe")
    ap.add_argument("--no-count", action="store_true",
                    help="skip the counting passes (roofline byte counts and walk parity): profiling runs only")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target seconds per CPU baseline leg")
    ap.add_argument("--dispatch", type=int, default=0,
                    help="K > 0: time K passes of the reference's per-pass DispatchRay loop instead (1 spp + "
                         "Denoising + Mix + BGRA8 copy; one JSON line, not the headline)")
    ap.add_argument("--dispatch-contexts", type=int, default=8,
                    help="--dispatch: also time the loop with this many row-tile contexts + gather (1: skip)")
    ap.add_argument("--dispatch-schedule", default="previous", choices=["previous", "tiles"],
                    help="--dispatch: the per-pass render's tile order (previous: heaviest first by the last pass's "
                         "draws, as PathTracer::DispatchRay does; tiles: row-major)")
    ap.add_argument("--profile-json", default=None,
                    help="rocprof summary of this workload (profiles/rocprof_*.json, tools/rocprof_summary.py)")
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------
# launcher: N ranks without torchrun
# ---------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(args, argv) -> list:
    """The torch.distributed.run command that starts `args.gpus` ranks of this script."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]


def check_world(args, env) -> int:
    """World size this rank runs at; raises SystemExit(2) when --gpus disagrees with the launcher."""
    world = int(env.get("WORLD_SIZE", "1"))
    if args.gpus is not None and args.gpus != world:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        raise SystemExit(2)
    return world


# ---------------------------------------------------------------------------------------
# measurement helpers
# ---------------------------------------------------------------------------------------
def byte_model(st, paths, node_bytes=32):
    """B_read = sum_segments[76 + 32 n_node + 32 n_prim + (hit ? 40 : 16)] + 16 P.
    node_bytes = 112 for the ordered walk's 4-wide nodes (a visit loads four child boxes in
    octant form + four refs: 7 x 16 B)."""
    return (76 * st["segments"] + node_bytes * st["nodes"] + 32 * st["prims"] + 40 * st["hits"]
            + 16 * st["misses"] + 16 * paths)


def usable_cores() -> dict:
    """nproc, the affinity mask, and the cgroup CPU quota (the box grants a CPU share below nproc)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    usable = min(aff, quota) if quota else aff
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "usable": usable}


def cpu_baseline(cfg, objs, sky, cam, seconds_hint=10.0):
    """The oracle (scalar C++ restatement, test infrastructure) on a bounded sample: every 16th
    row (at least as many rows as threads), full width, the first `spp_sample` passes of every
    sampled pixel (a pixel's passes are sequential).  Two legs: 1 thread, and all usable cores
    (std::thread over rows)."""
    import numpy as np
    import oracle
    cores = usable_cores()
    W, H = cfg["width"], cfg["height"]

    def leg(threads, rows):
        spp_probe = 1
        rng = oracle.init_rng(cfg["seed"], W, rows, threads=threads)
        t = time.perf_counter()
        oracle.render(objs, cam, sky, rows, spp_probe, cfg["depth"], rng, threads=threads)
        dt = max(time.perf_counter() - t, 1e-3)
        spp_sample = int(max(1, min(cfg["spp"], spp_probe * seconds_hint / dt)))
        rng = oracle.init_rng(cfg["seed"], W, rows, threads=threads)
        t = time.perf_counter()
        oracle.render(objs, cam, sky, rows, spp_sample, cfg["depth"], rng, threads=threads)
        dt = time.perf_counter() - t
        paths = rows.size * W * spp_sample
        return paths / dt / 1e6, f"{rows.size} rows x {W} px x first {spp_sample} of {cfg['spp']} spp ({paths} paths, {dt:.1f} s)"

    n_all = cores["usable"]
    step = 16
    while step > 1 and (H + step - 1) // step < n_all:
        step //= 2
    rows_all = np.arange(0, H, step, dtype=np.int32)
    v1, s1 = leg(1, rows_all[:: max(1, rows_all.size // 4)])     # 1 thread: 4 of the sampled rows
    va, sa = leg(n_all, rows_all)
    return {
        "value": round(va, 4),
        "unit": "Mpaths/s",
        "cores": n_all,
        "kind": "port",
        "sample": f"{cfg['name']}: every {step}th row; all cores: {sa}; 1 thread: {s1}",
        "threads_1": round(v1, 4),
        "threads_all": round(va, 4),
        "nproc": cores["nproc"],
        "cgroup_quota": cores["cgroup_quota"],
        "affinity": cores["affinity"],
    }


def load_profile(path, config, n_rows, spp, gpu_path, walk, schedule):
    """A committed rocprof summary (tools/rocprof_summary.py) of exactly this workload, or None."""
    if not path or not os.path.exists(path):
        return None
    with open(path) as f:
        pj = json.load(f)
    want = {"config": config, "n_rows": n_rows, "spp": spp, "path": gpu_path, "walk": walk, "schedule": schedule}
    return pj if all(pj.get(k) == v for k, v in want.items()) else None


# ---------------------------------------------------------------------------------------
# one rank
# ---------------------------------------------------------------------------------------
def run(args):
    import numpy as np
    import torch
    import torch.distributed as dist

    from cpppathtracer_amd import Renderer, camera_get_copy, multigpu, scenes, texture_io, tiling

    world = check_world(args, os.environ)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # CPT_BENCH_BACKEND=gloo: rehearsal of the N-rank path on a box with fewer GPUs (ranks share
    # devices round-robin, collectives go through host copies).  Labelled as such in the line.
    backend = os.environ.get("CPT_BENCH_BACKEND", "nccl")
    # Under a launcher (torch.distributed.run sets RANK and MASTER_ADDR) the process group, the
    # all-gather and the stitch run at every world size, 1 included, so the RCCL path executes on
    # a one-GPU box (tests/test_gpu_rccl.py); a plain `python bench.py` at N = 1 has none.
    use_pg = world > 1 or ("RANK" in os.environ and "MASTER_ADDR" in os.environ)
    if use_pg:
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
    W0, H0 = cfg["width"], cfg["height"]   # the configuration's own frame (strong-scaling check)
    if args.scaling == "weak" and world > 1 and not (args.width or args.height):
        cfg["width"], cfg["height"] = tiling.weak_scaled_size(cfg["width"], cfg["height"], world)
    W, H, spp, depth = cfg["width"], cfg["height"], cfg["spp"], cfg["depth"]
    if args.objects and cfg["scene"] == "s1000":
        objs = scenes.scene_s1000(n=args.objects)
        cfg["scene"] = f"s1000(n={args.objects})"
    else:
        objs = scenes.SCENES[cfg["scene"]]()
    sky = texture_io.load_cptex()
    cam = camera_get_copy(scenes.camera_for(W, H))
    rows = tiling.partition_rows(H, world, rank)
    parts = None
    partition_pilot_ms = None

    def _all_reduce(x, op=dist.ReduceOp.SUM):
        if backend == "nccl":
            dist.all_reduce(x, op=op)
            return x
        h = x.cpu()
        dist.all_reduce(h, op=op)
        return h.to(x.device)

    r = Renderer(torch.cuda.current_device())
    # One non-default HIP stream for everything: the render kernels (via cpt_set_stream), the
    # all-gather and the timing events.  (The default stream's handle is 0, which the C-ABI
    # reads as "use the context's own stream".)
    stream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)
    assert stream.cuda_stream != 0
    r.set_stream(stream.cuda_stream)
    r.set_scene(objs)
    r.set_env(sky)
    if args.partition == "balanced" and world > 1:
        # setup, not timed: a pilot of the whole frame, identical on every rank (same scene, camera,
        # seed), gives each 8-row block's work; every rank deals the blocks the same way
        t_p = time.perf_counter()
        r.set_frame(W, H)
        r.init_rng(cfg["seed"])
        owner = tiling.lpt_owner(tiling.block_costs_from_tiles(r.tile_costs(cam, 4, depth, ordered=args.walk == "ordered")),
                                 world)
        parts = [tiling.rows_of_owner(H, owner, k) for k in range(world)]
        rows = parts[rank]
        partition_pilot_ms = round((time.perf_counter() - t_p) * 1e3, 2)
    r.set_frame(W, H, rows)
    t_init = time.perf_counter()
    r.init_rng(cfg["seed"])
    torch.cuda.synchronize()
    t_init = time.perf_counter() - t_init

    npix_local = rows.size * W
    gather = multigpu.TileGather(W, H, world, rank, dev, backend, parts=parts) if use_pg else None
    kernel_events = []
    ordered = args.walk == "ordered"
    schedule = args.schedule if args.path == "megakernel" else "tiles"
    if schedule == "auto":
        schedule = "cost" if spp >= 64 else "tiles"
    consolidate = {"auto": None, "on": True, "off": False}[args.consolidate]
    # the library's rule (cpt_capi.cpp): the LDS-walk megakernel consolidates its tail when the
    # rank holds more than 1 and at most 4 pixels per lane of the persistent grid (1024 lanes per
    # CU) and the chains have at least 512 passes
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    consolidating = (args.path == "megakernel" and ordered and spp > 1 and
                     (consolidate if consolidate is not None else spp >= 512 and 1024 * cus < npix_local <= 4 * 1024 * cus))

    def step(timed=False):
        r.render(cam, spp, depth, path=args.path, ordered=ordered, schedule=schedule, consolidate=consolidate)
        if timed:
            # the dominant kernel's device time: HIP events the context records on its launch
            # stream around the megakernel (after the cost schedule's pilot); waits for it
            kernel_events.append(r.last_kernel_stats())
        if gather is not None:
            # all-gather of the fp32 tiles (RCCL over xGMI), then the on-device stitch into the
            # full framebuffer (every rank holds a copy after the all-gather)
            return gather(r)
        return None

    # Counting passes (same pixels, same seed; not timed) for the algorithmic byte model: the
    # reference walk's counts, and the executed walk's counts and framebuffer, which must equal
    # the reference walk's bit for bit.
    KEYS = ("segments", "nodes", "prims", "hits", "misses")

    def count_pass(walk_ordered):
        r.init_rng(cfg["seed"])
        r.reset_stats()
        r.render(cam, spp, depth, stats=True, path=args.path, ordered=walk_ordered)
        torch.cuda.synchronize()
        loc = r.stats()
        loc["global_nodes"] = r.raw_counters()[6]   # wide-node visits past the LDS image
        v = torch.tensor([loc[k] for k in KEYS + ("global_nodes",)], dtype=torch.float64, device=dev)
        if use_pg:
            v = _all_reduce(v)
        return dict(zip(KEYS + ("global_nodes",), (int(x) for x in v.tolist())))

    walk_info = r.walk_info()
    hbm_ceiling = r.measure_read_bandwidth(4 << 30, 10) if not args.no_hbm_probe else None
    wide = ordered and walk_info["n_wide"] > 0
    # Global-memory bytes per node visit of the executed walk: the wide walk reads the top
    # LDS_TREE_NODES nodes from the workgroup's LDS image (loaded once per workgroup per launch,
    # priced below), so those visits move no global-memory bytes; visits past the image read
    # 112 B from global memory (counted separately); a binary visit reads 32 B.
    lds_image = wide
    n_lds = min(walk_info["n_wide"], LDS_TREE_NODES)
    walk_node_bytes = 0 if lds_image else 32
    st = walk_counts = walk_diff = None
    if not args.no_count:
        st = count_pass(False)
        walk_counts = st
        if ordered:
            fb_ref = torch.empty((npix_local, 4), dtype=torch.float32, device=dev)
            r.copy_accum_device(fb_ref.data_ptr(), npix_local * 16, torch.cuda.current_stream().cuda_stream)
            walk_counts = count_pass(True)
            fb_ord = torch.empty_like(fb_ref)
            r.copy_accum_device(fb_ord.data_ptr(), npix_local * 16, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            nd = (fb_ref.view(torch.int32) != fb_ord.view(torch.int32)).any(dim=1).sum().to(torch.float64)
            if use_pg:
                nd = _all_reduce(nd)
            walk_diff = int(nd.item())
            del fb_ref, fb_ord
    r.init_rng(cfg["seed"])

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    if use_pg:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    if use_pg:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # average device time of one launch of the dominant kernel over the timed steps
    avg_kernel_ms = float(np.mean([ms for ms, _ in kernel_events])) if kernel_events else float("nan")
    launches = kernel_events[-1][1] if kernel_events else 0
    t = torch.tensor([elapsed, avg_kernel_ms], dtype=torch.float64, device=dev)
    if use_pg:
        t = _all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, avg_kernel_ms_max = t.tolist()

    # N > 1: the other scaling mode over the same ranks, 1 untimed + 2 timed frames with the
    # gather -- strong (the default): the weak-scaled frame (pixels per GPU fixed); weak: the
    # configuration's own frame strong-scaled (the north star's 1920x1080 at N GPUs, whose
    # ceiling is the longest pixel chain).
    other = None
    if world > 1 and not args.no_strong_check:
        if args.scaling == "weak":
            Wx, Hx, mode = W0, H0, "strong"
        else:
            (Wx, Hx), mode = tiling.weak_scaled_size(W0, H0, world), "weak"
        if (Wx, Hx) != (W, H):
            rows_x = tiling.partition_rows(Hx, world, rank)
            cam_x = camera_get_copy(scenes.camera_for(Wx, Hx))
            r.set_frame(Wx, Hx, rows_x)
            r.init_rng(cfg["seed"])
            gather_x = multigpu.TileGather(Wx, Hx, world, rank, dev, backend)
            n_other = 2
            for k in range(n_other + 1):
                if k == 1:
                    dist.barrier()
                    torch.cuda.synchronize()
                    ts = time.perf_counter()
                r.render(cam_x, spp, depth, path=args.path, ordered=ordered, schedule=schedule,
                         consolidate=consolidate)
                gather_x(r)
            torch.cuda.synchronize()
            dist.barrier()
            ts = torch.tensor([time.perf_counter() - ts], dtype=torch.float64, device=dev)
            ts = _all_reduce(ts, op=dist.ReduceOp.MAX).item()
            other = {
                "mode": mode,
                "workload": f"{args.config}: {cfg['scene']} {Wx}x{Hx} {spp}spp depth {depth}",
                "n_gpus": world, "steps": n_other, "ms_per_step": round(ts / n_other * 1e3, 3),
                "value": round(Wx * Hx * spp * n_other / ts / 1e6, 3), "unit": "Mpaths/s",
                "note": ("the configuration's own frame row-tiled over the same ranks (strong scaling); its ceiling "
                         "is the longest pixel chain (DESIGN.md §Multi-GPU)" if mode == "strong" else
                         "the frame scaled by sqrt(N) per axis, so every rank holds the N = 1 pixel count (weak "
                         "scaling: the path shards into independent row tiles)"),
            }

    if rank == 0:
        paths_total = W * H * spp
        value = paths_total * args.steps / elapsed / 1e6
        if not use_pg:
            collective = ""
        elif backend == "nccl":
            collective = ", RCCL all-gather of the fp32 tiles"
        else:
            collective = f", {backend} all-gather via host copies (rehearsal, ranks share GPUs)"
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
                "rows_rendered": H, "path": args.path, "walk": args.walk, "schedule": schedule,
                "tail_consolidation": bool(consolidating),
                # strong (default since round 4): the config's own frame at every N; weak: pixels per
                # GPU fixed.  N > 1 values of rounds 1-3 were weak-scaled
                "scaling": args.scaling,
                "parallelism": (f"row-tiled x{world} (interleaved {tiling.BLOCK_ROWS}-row blocks){collective}"
                                if parts is None else
                                f"row-tiled x{world} ({tiling.BLOCK_ROWS}-row blocks dealt by a pilot's cost){collective}"),
            },
            "rng_init_ms": round(t_init * 1e3, 2),
        }
        if partition_pilot_ms is not None:
            out["partition_pilot_ms"] = partition_pilot_ms   # setup, outside the timed steps
        if other:
            out[f"{other.pop('mode')}_scaling"] = other
        if st is not None:
            # Algorithmic bytes of one launch: SURVEY.md 8(d)'s per-unit model x the units the
            # launch processes (the executed walk's own counts; a 4-wide node visit = 112 B),
            # rank 0's share of them (interleaved blocks keep the shares statistically equal),
            # over the max-over-ranks render time.
            share = npix_local / float(W * H)
            bytes_launch = byte_model(walk_counts, paths_total, walk_node_bytes) * share
            if lds_image:   # every workgroup stages the image once (one workgroup per CU)
                bytes_launch += n_lds * WIDE_NODE_BYTES * torch.cuda.get_device_properties(dev).multi_processor_count
                bytes_launch += walk_counts["global_nodes"] * WIDE_NODE_BYTES * share
            bytes_ref = byte_model(st, paths_total) * share
            kms = avg_kernel_ms_max if world > 1 else avg_kernel_ms
            t_render = kms * max(1, launches) / 1e3   # the byte counts cover every launch of the render
            achieved = bytes_launch / t_render / 1e9
            roof = {
                # The roofline the north star prices the kernel against: the
                # algorithmic HBM bytes of the executed walk over the kernel's time.  It is NOT
                # what bounds the kernel: its working set is cache-resident (measured HBM read
                # below) and the SQ counters show divergent VALU issue + latency (`limiter`).
                "bound": "issue/latency (divergent traversal; algorithmic-byte HBM roofline reported)",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "kernel": "k_megakernel" if args.path == "megakernel" else "wavefront (k_wf_extend+k_wf_shade per bounce)",
                "kernel_avg_ms": round(kms, 3),
                "launches_per_step": launches,
                "bytes_per_launch": int(bytes_launch),
                "byte_model": (f"SURVEY.md 8(d): 76 S + {walk_node_bytes} nodes + 32 prims + 40 hits + 16 misses + 16 P "
                               "on the executed walk's counts" +
                               (" (4-wide nodes read from the workgroup's LDS image: no global-memory bytes per "
                                "visit, + the image's 112 B x min(n_wide, 512) once per workgroup, + 112 B per "
                                "visit of a node past the LDS image)" if lds_image else " (binary nodes)")),
                "lds_node_bytes_per_launch": int((walk_counts["nodes"] - walk_counts["global_nodes"]) *
                                                 WIDE_NODE_BYTES * share) if lds_image else 0,
                "walk_info": walk_info,
                "walk_counts": walk_counts,
                "reference_counts": st,
                "achieved_reference_model": round(bytes_ref / t_render / 1e9, 2),
                "frac_reference_model": round(bytes_ref / t_render / 1e9 / HBM_PEAK_GBS, 4),
                "reference_model_note": "SURVEY.md 8(d)'s literal figure: the same model on the reference algorithm's "
                                        "counts (right-first DFS over its median tree, 32-B nodes) for the same paths. "
                                        "It prices node visits and primitive tests the ordered walk does not make "
                                        "(7.1x the nodes), so it exceeds the HBM peak: not a roofline",
                "walk_vs_reference_pixels_differing": walk_diff,
                "hbm_stream_ceiling_gbs": round(hbm_ceiling, 1) if hbm_ceiling else None,
            }
            prof = load_profile(args.profile_json or os.path.join(
                REPO, "profiles", f"rocprof_{args.config}_{args.path}_{args.walk}.json"),
                args.config, int(rows.size), spp, args.path, args.walk, schedule) if world == 1 else None
            if prof:
                # rocprofv3 passes of this same workload (profiles/, tools/profile.sh +
                # tools/rocprof_summary.py): measured HBM bytes and the VALU-issue roofline
                roof["traffic"] = prof["hbm_bytes_per_launch"]
                roof["hbm_read_gbs_rocprof"] = prof["hbm_read_gbs"]
                roof["hbm_read_frac_rocprof"] = round(prof["hbm_read_gbs"] / HBM_PEAK_GBS, 6)
                roof["kernel_avg_ms_rocprof"] = prof["kernel_avg_ms_rocprof"]
                roof["l2_hit_rate_rocprof"] = prof.get("l2_hit_rate")
                roof["valu_issue_roofline"] = {
                    "achieved_frac": prof["issue"].get("valu_issue_frac"),
                    "note": "wave64 VALU instructions x 2 cycles / (1024 SIMDs x clock x time), MI355X_MICROARCH.md "
                            "wave scheduling; lanes_per_valu = active lanes per VALU instruction",
                    **{k: prof["issue"][k] for k in ("lanes_per_valu", "wait_frac", "clock_ghz") if k in prof["issue"]},
                }
                # the binding roof: VALU issue x the share of a wave's 64 lanes each VALU
                # instruction does useful work on
                iss, lanes = prof["issue"].get("valu_issue_frac"), prof["issue"].get("lanes_per_valu")
                if iss is not None and lanes is not None:
                    roof["useful_lane_issue_frac"] = round(iss * lanes / 64.0, 4)
                    roof["useful_lane_issue_note"] = ("valu_issue_roofline.achieved_frac x lanes_per_valu / 64: the "
                                                      "fraction of the SIMDs' lane-issue capacity doing useful work")
                roof["limiter"] = prof["limiter"]
                roof["profile"] = prof["source"]
            out["roofline"] = roof
        if not args.no_cpu_baseline and world == 1:
            try:
                out["cpu_baseline"] = cpu_baseline(cfg, objs, sky, cam, seconds_hint=args.cpu_seconds)
            except Exception as e:  # the baseline must never sink the GPU measurement
                out["cpu_baseline"] = {"value": None, "error": repr(e)}
        print(json.dumps(out), flush=True)
    r.close()
    if use_pg:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------------------
# --dispatch K: the reference's own per-pass loop (PipelineLoop, path_tracer.cu:256-306)
# ---------------------------------------------------------------------------------------
DISPLAY_BYTES_PER_PIXEL = 60   # k_denoise_rows: accum 16 + normal 12 + depth 4 + mix 12 read + 12 written + BGRA 4


def dispatch_bench(args):
    """ms per DispatchRay pass: a 1-spp SamplePixel render (radiance + first-hit normal/depth, not
    accumulated), Denoising + Mix into BGRA8, and the W x H x 4 B copy to the host that the
    reference's callback receives -- per pass, with each kernel's HIP-event time.  Once with one
    context (SetDevices(1)), once with `--dispatch-contexts` row-tile contexts gathered into a
    frame context (SetDevices(n): the contexts share this box's GPU), whose per-pass gather is
    also timed on its own.  One JSON line; not the headline metric."""
    import numpy as np
    import torch

    from cpppathtracer_amd import Renderer, camera_get_copy, scenes, texture_io, tiling

    torch.cuda.set_device(0)
    cfg = dict(scenes.CONFIGS[args.config])
    W, H, depth = args.width or cfg["width"], args.height or cfg["height"], cfg["depth"]
    objs = scenes.SCENES[cfg["scene"]]()
    sky = texture_io.load_cptex()
    cam0 = camera_get_copy(scenes.camera_for(W, H))
    K, warm = args.dispatch, 3
    host = torch.empty((H, W, 4), dtype=torch.uint8, pin_memory=True).numpy()   # the callback's frame
    h_eff, w_eff = 16 * (H // 16), 16 * (W // 16)

    def cam_at(idx):   # GetCopy's cur_sample_idx of pass idx (motional_camera.cu:195)
        c = np.array(cam0, copy=True)
        c["cur_sample_idx"] = idx
        return c

    def make(dev_rows=None):
        r = Renderer(0)
        r.set_scene(objs)
        r.set_env(sky)
        r.set_frame(W, H, dev_rows)
        r.init_rng(args.seed)
        return r

    def summary(samples):
        a = np.array(samples)
        return {"median": round(float(np.median(a)), 3), "mean": round(float(a.mean()), 3),
                "min": round(float(a.min()), 3), "max": round(float(a.max()), 3)}

    # ---- one context -------------------------------------------------------------------
    r = make()
    wall, rend, disp = [], [], []
    for k in range(warm + K):
        idx = k + 1
        t0 = time.perf_counter()
        r.render(cam_at(idx), 1, depth, aux=True, ordered=args.walk == "ordered", schedule=args.dispatch_schedule)
        r.denoise_mix(idx, out=host)   # waits for the frame on the host
        t1 = time.perf_counter()
        if k >= warm:
            wall.append((t1 - t0) * 1e3)
            rend.append(r.last_render_ms())
            disp.append(r.last_display_ms())
    # the display kernel alone, device frame only (no pinned host frame written over PCIe): the
    # same accumulator re-displayed K times (each call advances the Mix mean, as a pass does)
    dev_only = []
    for k in range(warm + K):
        r.denoise_mix(warm + K + 1 + k, host=False)
        if k >= warm:
            dev_only.append(r.last_display_ms())
    r.close()
    d_ms = float(np.median(dev_only))
    display_bytes = DISPLAY_BYTES_PER_PIXEL * w_eff * h_eff
    one = {
        "contexts": 1,
        "pass_ms": summary(wall),
        "render_ms": summary(rend),
        "display_ms": summary(disp),
        "display_device_only_ms": summary(dev_only),
        "display_host_frame_ms": round(float(np.median(disp)) - d_ms, 4),
        "copy_and_host_ms": round(float(np.median(wall)) - float(np.median(rend)) - float(np.median(disp)), 3),
        "display_roofline": {
            "kernel": "k_denoise_rows", "bound": "hbm", "bytes_per_launch": display_bytes,
            "achieved": round(display_bytes / (d_ms * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(display_bytes / (d_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "byte_model": f"{DISPLAY_BYTES_PER_PIXEL} B x W'H' ({w_eff}x{h_eff}): accumulator 16 + normal 12 + "
                          "depth 4 + mix 12 read + 12 written + BGRA8 4",
            "time": "display_device_only_ms (device frame only; the pinned host frame's PCIe write is "
                    "display_host_frame_ms on top, in display_ms)",
        },
    }
    # ---- n row-tile contexts + the frame context (SetDevices(n) on this GPU) -------------
    n = args.dispatch_contexts
    multi = None
    if n > 1:
        tiles = [make(tiling.partition_rows(H, n, t)) for t in range(n)]
        frame = make()
        wall, gath = [], []
        for k in range(warm + K):
            idx = k + 1
            t0 = time.perf_counter()
            for t in tiles:
                t.render(cam_at(idx), 1, depth, aux=True, ordered=args.walk == "ordered",
                         schedule=args.dispatch_schedule)
            for t in tiles:
                frame.gather_rows(t)
            frame.denoise_mix(idx, out=host)
            t1 = time.perf_counter()
            for t in tiles:   # (their errors; their work is done)
                t.synchronize()
            # the gather alone: every tile's render finished, then the n gathers and one wait
            tg = time.perf_counter()
            for t in tiles:
                frame.gather_rows(t)
            frame.synchronize()
            tg = time.perf_counter() - tg
            if k >= warm:
                wall.append((t1 - t0) * 1e3)
                gath.append(tg * 1e3)
        multi = {"contexts": n, "pass_ms": summary(wall), "gather_ms": summary(gath),
                 "note": f"{n} row-tile contexts (interleaved {tiling.BLOCK_ROWS}-row blocks) on one GPU, gathered "
                         "into a frame context by cpt_gather_rows (events, no host wait), then one display pass"}
        for t in tiles:
            t.close()
        frame.close()
    out = {
        "metric": "ms per DispatchRay pass (1 spp SamplePixel + Denoising + Mix + BGRA8 to the host)",
        "config": {"workload": f"{args.config}: {cfg['scene']} {W}x{H} 1spp depth {depth} per pass",
                   "width": W, "height": H, "walk": args.walk, "schedule": args.dispatch_schedule, "passes": K,
                   "warmup": warm,
                   "host_buffer": "pinned"},
        "higher_is_better": False,
        "single": one,
    }
    if multi:
        out["multi"] = multi
    print(json.dumps(out), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.dispatch:
        dispatch_bench(args)
        return
    if args.gpus is not None and args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the ranks before anything here touches the GPU
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        rc = subprocess.call(launcher_command(args, argv), env=env)
        sys.exit(rc)
    run(args)


if __name__ == "__main__":
    main()
