"""Deterministic synthetic scenes for the benchmark configs.

* S3    — 3 diffuse spheres + sky (configs 1, 2)
* S4    — Platform + Glass / "Metal" / "Mirror" spheres + sky (config 3; all BSDF branches)
* S1000 — floor + 1000 random spheres/cylinders with 20 random materials (configs 4, 5)

S1000 follows the distributions of the reference's scene script
(cppSrc/video_renderer.cpp:41-117) but replaces ``srand(time(0))``/``rand()``
(ray_tracing_math.hpp:30-37) with an MSVC-compatible LCG at a fixed seed so every run,
on every machine, builds the same scene.  Float arithmetic is done in float32 exactly as
the C++ expressions do.
"""
import numpy as np

from .types import (CYLINDER, DIFFUSE, GLASS, METAL, MIRROR, OBJECT_DTYPE, PLATFORM, SPHERE,
                    make_camera, make_material, make_object)

F = np.float32

# Camera used by the reference app (video_renderer.cpp:34-38)
CAMERA_ORIGIN = (130.0, 103.0, 130.0)
CAMERA_LOOK_AT = (0.0, 0.0, 0.0)


class MsvcRand:
    """MSVC ``rand()``: x = x*214013 + 2531011 (mod 2^32); return (x >> 16) & 0x7FFF."""

    RAND_MAX = 32767

    def __init__(self, seed):
        self.x = seed & 0xFFFFFFFF

    def rand(self):
        self.x = (self.x * 214013 + 2531011) & 0xFFFFFFFF
        return (self.x >> 16) & 0x7FFF

    def random(self):
        # ray_tracing_math.hpp:35  static_cast<float>(rand()) / static_cast<float>(RAND_MAX)
        return F(self.rand()) / F(self.RAND_MAX)

    def random3(self):
        a = self.random()
        b = self.random()
        c = self.random()
        return np.array([a, b, c], dtype=np.float32)


def _floor(material):
    # video_renderer.cpp:73-81
    return make_object(PLATFORM, material, center=(0.0, -10000.0, 0.0), radius=10000.0, y_pos=0.0)


def scene_s3():
    """Three diffuse spheres, no floor."""
    objs = np.zeros(3, dtype=OBJECT_DTYPE)
    kds = [(0.8, 0.3, 0.3), (0.3, 0.8, 0.3), (0.3, 0.3, 0.8)]
    for i, (cx, kd) in enumerate(zip((-35.0, 0.0, 35.0), kds)):
        objs[i] = make_object(SPHERE, make_material(DIFFUSE, kd=kd), center=(cx, 15.0, 0.0), radius=15.0)
    return objs


def scene_s4():
    """Floor + Glass, MaterialType::Metal (-> MirrorHitShader), MaterialType::Mirror
    (-> MetalHitShader) spheres."""
    objs = np.zeros(4, dtype=OBJECT_DTYPE)
    objs[0] = _floor(make_material(DIFFUSE, kd=(0.95, 0.95, 0.95)))
    objs[1] = make_object(SPHERE, make_material(GLASS, kd=(1.0, 1.0, 1.0), refractive_index=1.5, smoothness=4.0),
                          center=(-35.0, 15.0, 0.0), radius=15.0)
    objs[2] = make_object(SPHERE, make_material(METAL, kd=(0.8, 0.6, 0.2), smoothness=2.5),
                          center=(0.0, 15.0, 0.0), radius=15.0)
    objs[3] = make_object(SPHERE, make_material(MIRROR, kd=(0.9, 0.9, 0.9), smoothness=3.0, reflectivity=0.6),
                          center=(35.0, 15.0, 0.0), radius=15.0)
    return objs


def scene_s4_textured(handles=(1, 2, 3)):
    """scene_s4 with textured materials (§8(f) rank 4): the floor (Diffuse), the Metal and the
    Glass sphere take their kd from the textures bound to `handles`."""
    from .types import set_material_texture
    objs = scene_s4()
    for i, h in zip((0, 2, 1), handles):
        m = objs[i]["material"].copy()
        objs[i]["material"] = set_material_texture(m, h)
    return objs


def synthetic_texture(seed, width=16, height=8, full=False):
    """A random RGBA8 texture; `full` keeps all columns, else the AddTexByFile upload quirk
    (width/4 valid columns, textures.cu:32-33)."""
    from .texture_io import EnvTexture
    rng = np.random.default_rng(seed)
    cols = width if full else width // 4
    return EnvTexture(rng.integers(0, 256, size=(height, cols, 4), dtype=np.uint8), width, height)


def scene_s1000(seed=20250124, n=1000):
    """Floor + n random spheres / cylinders (video_renderer.cpp:41-117 distributions)."""
    rng = MsvcRand(seed)
    mats = [make_material(DIFFUSE, kd=(0.95, 0.95, 0.95))]
    for _ in range(1, 20):
        kd = rng.random3()
        rnd = int(rng.random() * F(2048)) % 5
        if rnd == 1:
            m = make_material(METAL, kd=kd, smoothness=rng.random() * F(4) + F(1.0),
                              reflectivity=rng.random() * F(0.8))
        elif rnd == 2:
            kd2 = F(0.5) + F(0.5) * rng.random3()
            m = make_material(MIRROR, kd=kd2, smoothness=rng.random() * F(4) + F(0.5))
        elif rnd == 3:
            sm = rng.random() * F(4) + F(2.0)
            ior = rng.random() * F(2) + F(1.2)
            m = make_material(GLASS, kd=(1.0, 1.0, 1.0), smoothness=sm, refractive_index=ior)
        else:
            m = make_material(DIFFUSE, kd=kd)
        mats.append(m)
    objs = np.zeros(n + 1, dtype=OBJECT_DTYPE)
    objs[0] = _floor(mats[0])
    for k in range(n):
        z = F(-550.0) + F(1.1) * F(k)
        rnd = int(rng.random() * F(2048)) % 2
        mat = mats[rng.rand() % 20]
        r = rng.random() * F(15.0) + F(1.0)
        if rnd == 0:
            x = rng.random() * F(300.0) - F(150.0)
            objs[k + 1] = make_object(SPHERE, mat, center=(x, r, z), radius=r)
        else:
            h = r / F(2) + rng.random() * F(20.0)
            x = rng.random() * F(300.0) - F(150.0)
            objs[k + 1] = make_object(CYLINDER, mat, center=(x, h / F(2), z), radius=r, height=h)
    return objs


SCENES = {"s3": scene_s3, "s4": scene_s4, "s1000": scene_s1000}


# BASELINE.json configs.  rows = H unless a caller subsamples.
CONFIGS = {
    "c1": dict(scene="s3", width=256, height=256, spp=4, depth=4),
    "c2": dict(scene="s3", width=1280, height=720, spp=256, depth=8),
    "c3": dict(scene="s4", width=1920, height=1080, spp=1024, depth=16),
    "c4": dict(scene="s1000", width=1920, height=1080, spp=1024, depth=16),
    "c5": dict(scene="s1000", width=3840, height=2160, spp=4096, depth=16),
}

DEFAULT_SEED = 1234


def camera_for(width, height):
    return make_camera(width, height, origin=CAMERA_ORIGIN, look_at=CAMERA_LOOK_AT)
