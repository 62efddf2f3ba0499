"""Reference-layout POD types as numpy dtypes (the drop-in data formats).

These mirror, byte for byte, the structs the reference passes around, so arrays built
here can cross the C-ABI (include/cpt.h) unchanged:

* ``MATERIAL_DTYPE`` — ``Material`` (include/material.h:17-35 in the reference), 40 B:
  type @0, have_tex @4, union{float3 kd; cudaTextureObject_t tex} @8, refractive_index @24,
  emit_intensity @28, smoothness @32, reflectivity @36.
* ``OBJECT_DTYPE`` — ``Object`` (include/object.h:17-32), 72 B: type @0, material @8,
  center @48, radius @60, y_pos @64, height @68.
* ``CAMERA_DTYPE`` — ``MotionalCamera`` (include/motional_camera.h:8-24), 136 B.
"""
import numpy as np

# PrimitiveType::Enum (object.h:7-15)
SPHERE, PLATFORM, CYLINDER = 0, 1, 2
# MaterialType::Enum (material.h:5-15)
DIFFUSE, METAL, MIRROR, GLASS, TEST = 0, 1, 2, 3, 4

DEFAULT_RAY_TMAX = np.float32(1e30)   # ray_tracing_common.h:11
BOUNCE_RAY_TMIN = np.float32(2e-5)    # ray_tracing_common.h:12
MAX_RECURSION_DEPTH_SET = 32          # path_tracer.h:13

MATERIAL_DTYPE = np.dtype(
    {
        "names": ["type", "have_tex", "kd", "refractive_index", "emit_intensity", "smoothness", "reflectivity"],
        "formats": ["<i4", "u1", ("<f4", 3), "<f4", "<f4", "<f4", "<f4"],
        "offsets": [0, 4, 8, 24, 28, 32, 36],
        "itemsize": 40,
    }
)

OBJECT_DTYPE = np.dtype(
    {
        "names": ["type", "material", "center", "radius", "y_pos", "height"],
        "formats": ["<i4", MATERIAL_DTYPE, ("<f4", 3), "<f4", "<f4", "<f4"],
        "offsets": [0, 8, 48, 60, 64, 68],
        "itemsize": 72,
    }
)

CAMERA_DTYPE = np.dtype(
    {
        "names": [
            "vup", "width", "height", "cur_sample_idx", "origin", "look_at", "view_fov",
            "dist_to_focus", "lens_radius", "move_speed", "u", "v", "w", "top_left_corner",
            "horizontal", "vertical",
        ],
        "formats": [
            ("<f4", 3), "<i4", "<i4", "<u4", ("<f4", 3), ("<f4", 3), "<f4", "<f4", "<f4", "<f4",
            ("<f4", 3), ("<f4", 3), ("<f4", 3), ("<f4", 3), ("<f4", 3), ("<f4", 3),
        ],
        "offsets": [0, 12, 16, 20, 24, 36, 48, 52, 56, 60, 64, 76, 88, 100, 112, 124],
        "itemsize": 136,
    }
)

assert MATERIAL_DTYPE.itemsize == 40 and OBJECT_DTYPE.itemsize == 72 and CAMERA_DTYPE.itemsize == 136


def make_material(mtype=DIFFUSE, kd=(0.0, 0.0, 0.0), refractive_index=0.0, emit_intensity=0.0,
                  smoothness=0.0, reflectivity=0.0):
    """A zero-initialised Material (the reference memsets before filling, video_renderer.cpp:43)."""
    m = np.zeros((), dtype=MATERIAL_DTYPE)
    m["type"] = mtype
    m["have_tex"] = 0
    m["kd"] = np.asarray(kd, dtype=np.float32)
    m["refractive_index"] = np.float32(refractive_index)
    m["emit_intensity"] = np.float32(emit_intensity)
    m["smoothness"] = np.float32(smoothness)
    m["reflectivity"] = np.float32(reflectivity)
    return m


# cudaTextureAddressMode / cudaTextureFilterMode values (cpt.h CPT_ADDRESS_*, CPT_FILTER_*)
ADDRESS_WRAP, ADDRESS_CLAMP, ADDRESS_MIRROR, ADDRESS_BORDER = 0, 1, 2, 3
FILTER_POINT, FILTER_LINEAR = 0, 1


def set_material_texture(m, handle):
    """Make a Material textured (have_tex_ = true, tex_ = handle).  tex_ shares bytes 8..15
    with kd_ (material.h:21-25), so kd.x/kd.y become the handle's low/high 32 bits as floats
    (the emission colour the reference computes from kd_); kd.z is left as it was."""
    m["have_tex"] = 1
    bits = np.array([handle & 0xFFFFFFFF, (handle >> 32) & 0xFFFFFFFF], dtype=np.uint32).view(np.float32)
    kd = np.array(m["kd"], dtype=np.float32)
    kd[0], kd[1] = bits[0], bits[1]
    m["kd"] = kd
    return m


def make_object(ptype, material, center=(0.0, 0.0, 0.0), radius=0.0, y_pos=0.0, height=0.0):
    o = np.zeros((), dtype=OBJECT_DTYPE)
    o["type"] = ptype
    o["material"] = material
    o["center"] = np.asarray(center, dtype=np.float32)
    o["radius"] = np.float32(radius)
    o["y_pos"] = np.float32(y_pos)
    o["height"] = np.float32(height)
    return o


def make_camera(width, height, origin=(0.0, 0.0, 0.0), look_at=(0.0, 0.0, 1.0)):
    """MotionalCamera(width, height, ori, at) with the header's default members
    (motional_camera.h:8-19, motional_camera.cu:14-39): vup (0,1,0), fov 30,
    dist_to_focus 100, lens_radius 0.0005, move_speed 50, cur_sample_idx 0."""
    c = np.zeros((), dtype=CAMERA_DTYPE)
    c["vup"] = np.array([0.0, 1.0, 0.0], dtype=np.float32)
    c["width"] = width
    c["height"] = height
    c["cur_sample_idx"] = 0
    c["origin"] = np.asarray(origin, dtype=np.float32)
    c["look_at"] = np.asarray(look_at, dtype=np.float32)
    c["view_fov"] = np.float32(30)
    c["dist_to_focus"] = np.float32(100)
    c["lens_radius"] = np.float32(0.0005)
    c["move_speed"] = np.float32(50.0)
    return c
