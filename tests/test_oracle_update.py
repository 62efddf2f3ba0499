"""Oracle restatement of SceneBVH::UpdateObject (bvh.cu:122-157), host only."""
import numpy as np

from cpppathtracer_amd import camera_get_copy, scenes


def _setup(oracle_mod, W=24, H=16):
    objs = scenes.scene_s1000(n=30)
    cam = camera_get_copy(scenes.camera_for(W, H))
    rows = np.arange(H, dtype=np.int32)
    return objs, cam, rows


def test_no_edits_is_plain_render(oracle_mod, sky):
    objs, cam, rows = _setup(oracle_mod)
    W = int(cam["width"])
    r1 = oracle_mod.init_rng(3, W, rows, threads=4)
    a1, s1 = oracle_mod.render_edited(objs, [], cam, sky, rows, 2, 6, r1, threads=4)
    r2 = oracle_mod.init_rng(3, W, rows, threads=4)
    a2, s2, _, _ = oracle_mod.render(objs, cam, sky, rows, 2, 6, r2, threads=4)
    np.testing.assert_array_equal(a1.view(np.uint32), a2.view(np.uint32))
    assert s1 == s2


def test_edit_and_restore_is_identity(oracle_mod, sky):
    """Moving an object away and back refits every ancestor box to its original value."""
    objs, cam, rows = _setup(oracle_mod)
    W = int(cam["width"])
    moved = objs[4].copy()
    moved["center"][0] += 100.0
    r1 = oracle_mod.init_rng(3, W, rows, threads=4)
    a1, s1 = oracle_mod.render_edited(objs, [(4, moved), (4, objs[4].copy())], cam, sky, rows, 2, 6, r1, threads=4)
    r2 = oracle_mod.init_rng(3, W, rows, threads=4)
    a2, s2, _, _ = oracle_mod.render(objs, cam, sky, rows, 2, 6, r2, threads=4)
    np.testing.assert_array_equal(a1.view(np.uint32), a2.view(np.uint32))
    assert s1 == s2


def test_edit_keeps_topology(oracle_mod, sky):
    """After a large move the refit tree keeps the original topology (a fresh build of the
    edited scene has another one), and closest hits agree with the fresh build whenever no
    exact ties are involved (same image here)."""
    objs, cam, rows = _setup(oracle_mod)
    W = int(cam["width"])
    moved = objs[4].copy()
    moved["center"][0] -= 60.0
    edited = objs.copy()
    edited[4] = moved
    r1 = oracle_mod.init_rng(3, W, rows, threads=4)
    a1, s1 = oracle_mod.render_edited(objs, [(4, moved)], cam, sky, rows, 2, 6, r1, threads=4)
    r2 = oracle_mod.init_rng(3, W, rows, threads=4)
    a2, s2, _, _ = oracle_mod.render(edited, cam, sky, rows, 2, 6, r2, threads=4)
    assert s1["segments"] == s2["segments"] and s1["hits"] == s2["hits"]
    assert (oracle_mod.build_bvh(objs)[1] != oracle_mod.build_bvh(edited)[1]).any()   # a fresh build differs
    np.testing.assert_array_equal(a1.view(np.uint32), a2.view(np.uint32))


def test_diagnostic_ordered_walk_same_image(oracle_mod, sky):
    """The oracle's diagnostic restatement of the ordered walk (oracle.set_walk) finds the same
    closest hits as the reference DFS: same image and RNG end state, its own node counts."""
    _, cam, rows = _setup(oracle_mod, 40, 24)
    objs = scenes.scene_s1000()
    W = int(cam["width"])
    r1 = oracle_mod.init_rng(9, W, rows, threads=4)
    a1, s1, _, _ = oracle_mod.render(objs, cam, sky, rows, 3, 8, r1, threads=4)
    oracle_mod.set_walk(True)
    try:
        r2 = oracle_mod.init_rng(9, W, rows, threads=4)
        a2, s2, _, _ = oracle_mod.render(objs, cam, sky, rows, 3, 8, r2, threads=4)
    finally:
        oracle_mod.set_walk(False)
    np.testing.assert_array_equal(a1.view(np.uint32), a2.view(np.uint32))
    np.testing.assert_array_equal(r1, r2)
    assert s1["segments"] == s2["segments"] and s1["nodes"] != s2["nodes"]


def test_refit_walk_tree_same_image_as_rebuilt(oracle_mod, sky):
    """The ordered walk on a refit walk tree (libcpt's device refit, cpt_update_objects) and on
    one rebuilt from the edited objects (cpt_update_objects_rebuild) find the same closest hits
    as the reference walk: same image and RNG end states; the refit tree's node counts are its
    own (a worse tree after large moves, never a different hit)."""
    _, cam, rows = _setup(oracle_mod, 40, 24)
    objs = scenes.scene_s1000()
    W = int(cam["width"])
    rng = np.random.default_rng(5)
    edits = []
    for i in rng.choice(np.flatnonzero(objs["type"] != 1), size=200, replace=False):
        o = objs[int(i)].copy()
        o["center"][0] += np.float32(rng.uniform(-80, 80))
        o["radius"] *= np.float32(rng.uniform(0.5, 1.5))
        edits.append((int(i), o))
    r0 = oracle_mod.init_rng(4, W, rows, threads=4)
    a0, s0 = oracle_mod.render_edited(objs, edits, cam, sky, rows, 2, 8, r0, threads=4)
    out = []
    oracle_mod.set_walk(True)
    try:
        for rebuild in (False, True):
            r = oracle_mod.init_rng(4, W, rows, threads=4)
            a, s = oracle_mod.render_edited(objs, edits, cam, sky, rows, 2, 8, r, threads=4, walk_rebuild=rebuild)
            np.testing.assert_array_equal(a.view(np.uint32), a0.view(np.uint32))
            np.testing.assert_array_equal(r, r0)
            assert s["segments"] == s0["segments"] and s["hits"] == s0["hits"]
            out.append(s)
    finally:
        oracle_mod.set_walk(False)
    assert out[0]["nodes"] != out[1]["nodes"]   # two different walk trees
