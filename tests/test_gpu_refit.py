"""Device refit of cpt_update_objects (SceneBVH::UpdateObject, bvh.cu:122-157) against the
oracle's refit BVH (oracle.render_edited), bit for bit.

The reference refits the updated leaf's ancestors and keeps the topology; libcpt does the
same on the GPU for every device copy (reference order, the walk tree's octant orders, its
4-wide image in LDS and HBM, its leaf array).  `rebuild=True` is cpt_update_objects_rebuild:
the ordered walk's SAH tree is rebuilt on the host instead; the images must not change.
"""
import numpy as np
import pytest

from cpppathtracer_amd import camera_get_copy, scenes

from test_gpu_parity import _check_stats, _kw, _timed

pytestmark = pytest.mark.gpu


def _edits(objs, n_moves, seed, swap_material=True):
    """Random moves/resizes of n_moves bounded objects, one material swap, one repeated index
    (the last object of a batch wins)."""
    rng = np.random.default_rng(seed)
    bounded = np.flatnonzero(objs["type"] != 1)
    pick = rng.choice(bounded, size=min(n_moves, bounded.size), replace=False)
    edits = []
    for i in pick:
        o = objs[int(i)].copy()
        o["center"][0] += np.float32(rng.uniform(-60, 60))
        o["center"][2] += np.float32(rng.uniform(-40, 40))
        o["radius"] *= np.float32(rng.uniform(0.5, 1.6))
        if o["type"] == 2:
            o["height"] *= np.float32(rng.uniform(0.6, 1.5))
        edits.append((int(i), o))
    if swap_material:
        o = objs[int(bounded[1])].copy()
        o["material"] = objs[int(bounded[2])]["material"]
        edits.append((int(bounded[1]), o))
    i, o = edits[0]
    o2 = o.copy()
    o2["center"][1] += np.float32(7.5)
    edits.append((i, o2))          # the same index again: this one wins
    return edits


def _render_edited(gpu, oracle_mod, sky, objs, edits, W, H, spp, depth, path, rebuild, batch=True):
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    if batch:
        gpu.update_objects([i for i, _ in edits], np.array([o for _, o in edits]), rebuild=rebuild)
    else:
        for i, o in edits:
            gpu.update_objects([i], np.array([o]), rebuild=rebuild)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    gpu.init_rng(5)
    gpu.reset_stats()
    stats = not _timed(path)
    gpu.render(cam, spp, depth, stats=stats, sync=True, **_kw(path))
    ga, gs = gpu.read_accum(), (gpu.stats() if stats else None)
    if stats and _kw(path)["ordered"]:
        gs["fallbacks"] = gpu.raw_counters()[5]
    rows = np.arange(H, dtype=np.int32)
    rng = oracle_mod.init_rng(5, W, rows, threads=8)
    oa, os_ = oracle_mod.render_edited(objs, edits, cam, sky, rows, spp, depth, rng, threads=8, walk_rebuild=rebuild)
    if _kw(path)["ordered"] and stats:
        oracle_mod.set_walk(True)
        try:
            _, w_st = oracle_mod.render_edited(objs, edits, cam, sky, rows, spp, depth,
                                               oracle_mod.init_rng(5, W, rows, threads=8), threads=8,
                                               walk_rebuild=rebuild)
            w_st["fallbacks"] = oracle_mod.last_fallbacks()
        finally:
            oracle_mod.set_walk(False)
        os_ = dict(os_, walk=w_st)
    np.testing.assert_array_equal(gpu.read_rng(), rng)
    _check_stats(gs, os_, path)
    np.testing.assert_array_equal(ga.view(np.uint32), oa.view(np.uint32))
    return ga


@pytest.mark.parametrize("path", ["megakernel", "megakernel:ordered", "megakernel:plain", "wavefront:ordered",
                                  "megakernel:ordered+timed", "megakernel:ordered+timed+cons"])
def test_device_refit_s1000(gpu, oracle_mod, sky, path):
    """40 moved / resized objects, a material swap and a repeated index in one batch, on the
    S1000 generator (470 wide nodes: the whole image in LDS)."""
    objs = scenes.scene_s1000()
    _render_edited(gpu, oracle_mod, sky, objs, _edits(objs, 40, 1), 64, 36, 2, 16, path, rebuild=False)


@pytest.mark.parametrize("path", ["megakernel:ordered", "megakernel:plain", "megakernel:ordered+timed"])
def test_device_refit_beyond_lds_image(gpu, oracle_mod, sky, path):
    """A 3000-primitive tree (> LDS_TREE_NODES wide nodes: the image's lower part is read from
    HBM), 300 edits: both parts of the image and the leaf array are refit."""
    objs = scenes.scene_s1000(n=3000)
    gpu.set_scene(objs)
    assert gpu.walk_info()["n_wide"] > 512
    _render_edited(gpu, oracle_mod, sky, objs, _edits(objs, 300, 2), 64, 36, 2, 16, path, rebuild=False)
    if path.startswith("megakernel:ordered"):   # the plain walk uses the binary orders, not the image
        from test_gpu_parity import assert_hbm_part_walked
        assert_hbm_part_walked(gpu, path, 64, 36, 16)


def _new_material(base, k):
    """A material no object of the scene uses: its own colour and emission."""
    m = base.copy()
    m["kd"] = np.array([0.11 + 0.07 * k, 0.83 - 0.05 * k, 0.37], np.float32)
    m["emit_intensity"] = np.float32(0.25 + k)
    return m


@pytest.mark.parametrize("path", ["megakernel:ordered", "megakernel", "megakernel:ordered+timed"])
def test_device_refit_new_materials(gpu, oracle_mod, sky, path):
    """An update batch (device refit, no rebuild) that gives objects materials no object had
    before: the material array grows past its allocation.  Two batches, the second growing it
    again, each against the oracle bit for bit."""
    objs = scenes.scene_s1000(n=120)
    bounded = np.flatnonzero(objs["type"] != 1)
    edits = []
    for k, i in enumerate(bounded[:6]):
        o = objs[int(i)].copy()
        o["material"] = _new_material(o["material"], k)
        o["center"][1] += np.float32(2.0)
        edits.append((int(i), o))
    _render_edited(gpu, oracle_mod, sky, objs, edits, 48, 32, 2, 8, path, rebuild=False)
    more = list(edits)
    for k, i in enumerate(bounded[6:40]):
        o = objs[int(i)].copy()
        o["material"] = _new_material(o["material"], 10 + k)
        more.append((int(i), o))
    _render_edited(gpu, oracle_mod, sky, objs, more, 48, 32, 2, 8, path, rebuild=False, batch=False)


def test_device_refit_material_table_bounded(gpu, oracle_mod, sky):
    """Advisor r04: an object whose material changes every frame (a device refit per frame) must
    not grow the material table without bound -- unreferenced slots are dropped with a rebuild
    once the table holds more than 2x the referenced slots + 16 -- and the image after 100 such
    frames is still the oracle's."""
    objs = scenes.scene_s1000(n=120)
    W, H = 48, 32
    cam = camera_get_copy(scenes.camera_for(W, H))
    gpu.set_scene(objs)
    gpu.set_env(sky)
    gpu.set_frame(W, H)
    n0 = gpu.material_count()
    i = int(np.flatnonzero(objs["type"] == 0)[3])
    cur = objs.copy()
    peak = 0
    for f in range(100):
        o = cur[i].copy()
        o["material"] = _new_material(objs[i]["material"], 100 + f)
        cur[i] = o
        gpu.update_objects([i], o.reshape(1))
        peak = max(peak, gpu.material_count())
    assert peak <= 2 * (n0 + 1) + 17, (n0, peak)
    gpu.init_rng(3)
    gpu.render(cam, 2, 8, ordered=True, sync=True)
    rows = np.arange(H, dtype=np.int32)
    orng = oracle_mod.init_rng(3, W, rows, threads=8)
    # (only the material changed: the refit tree's boxes are the original ones)
    oacc, _ = oracle_mod.render_edited(objs, [(i, cur[i])], cam, sky, rows, 2, 8, orng, threads=8, walk_rebuild=False)
    np.testing.assert_array_equal(gpu.read_accum().view(np.uint32), oacc.view(np.uint32))


@pytest.mark.parametrize("path", ["megakernel:ordered", "megakernel", "megakernel:plain"])
def test_device_refit_platform_height(gpu, oracle_mod, sky, path):
    """A platform that stays a platform with a new y_pos (and a new material): its copies at the
    head of every octant order and of the wide tree's leaf array are rewritten by the device
    refit alone (no rebuild), and the image is the oracle's."""
    objs = scenes.scene_s1000(n=80)
    floor = int(np.flatnonzero(objs["type"] == 1)[0])
    o = objs[floor].copy()
    o["y_pos"] = np.float32(4.5)
    o["material"] = _new_material(o["material"], 3)
    sph = int(np.flatnonzero(objs["type"] == 0)[1])
    o2 = objs[sph].copy()
    o2["center"][1] += np.float32(3.0)
    _render_edited(gpu, oracle_mod, sky, objs, [(floor, o), (sph, o2)], 48, 32, 2, 8, path, rebuild=False)


@pytest.mark.parametrize("path", ["megakernel:ordered", "megakernel:plain"])
def test_rebuild_matches_refit(gpu, oracle_mod, sky, path):
    """cpt_update_objects_rebuild (new SAH walk tree) and the device refit give the oracle's
    image; single-object calls equal the batch."""
    objs = scenes.scene_s1000(n=200)
    edits = _edits(objs, 25, 3)
    a = _render_edited(gpu, oracle_mod, sky, objs, edits, 48, 32, 2, 8, path, rebuild=True)
    b = _render_edited(gpu, oracle_mod, sky, objs, edits, 48, 32, 2, 8, path, rebuild=False)
    c = _render_edited(gpu, oracle_mod, sky, objs, edits, 48, 32, 2, 8, path, rebuild=False, batch=False)
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
    np.testing.assert_array_equal(b.view(np.uint32), c.view(np.uint32))


def test_platform_edit_rebuilds(gpu, oracle_mod, sky):
    """A sphere becoming a platform (and the floor a sphere) changes the walk tree's leaf set:
    the update rebuilds it; the image still equals the oracle's."""
    objs = scenes.scene_s1000(n=60)
    floor = int(np.flatnonzero(objs["type"] == 1)[0])
    sph = int(np.flatnonzero(objs["type"] == 0)[2])
    o1 = objs[sph].copy()
    o1["type"] = 1
    o1["y_pos"] = np.float32(-3.0)
    o2 = objs[floor].copy()
    o2["type"] = 0
    o2["radius"] = np.float32(20.0)
    o2["center"] = np.array([0.0, 10.0, -100.0], np.float32)
    for path in ("megakernel:ordered", "megakernel"):
        _render_edited(gpu, oracle_mod, sky, objs, [(sph, o1), (floor, o2)], 48, 32, 2, 8, path, rebuild=False)


def test_bvh_export_after_device_refit(gpu):
    """The host's reference tree follows the device refit (cpt_scene_bvh_export): same boxes as
    a fresh build of the oracle-style refit on the host (cpt_update_objects_rebuild)."""
    objs = scenes.scene_s1000(n=100)
    edits = _edits(objs, 10, 4)
    idx, new = [i for i, _ in edits], np.array([o for _, o in edits])
    gpu.set_scene(objs)
    gpu.update_objects(idx, new)
    b1, l1 = gpu.bvh_export()
    gpu.set_scene(objs)
    gpu.update_objects(idx, new, rebuild=True)
    b2, l2 = gpu.bvh_export()
    np.testing.assert_array_equal(l1, l2)
    np.testing.assert_array_equal(b1.view(np.uint32), b2.view(np.uint32))
