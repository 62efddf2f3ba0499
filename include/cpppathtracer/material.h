// material.h — Material POD of the drop-in API (reference include/material.h:5-35).
#pragma once

#include "ray_tracing_common.h"
#include "textures.h"

namespace MaterialType {
enum Enum {
    Diffuse = 0,
    Metal,    // shaded by the reference's MirrorHitShader (material.cu:151-153)
    Mirror,   // shaded by the reference's MetalHitShader  (material.cu:154-156)
    Glass,
    Test,     // falls through to Diffuse
    Count
};
}  // namespace MaterialType

// 40 bytes, byte-identical to the reference Material and to cpt_material.
class Material {
public:
    MaterialType::Enum type_;
    bool have_tex_;
    union {
        float3 kd_;
        PocaTexture tex_;     // have_tex_: kd = the texture sampled at (0, 0) (material.cu:11-18)
    };
    float refractive_index_;
    float emit_intensity_;
    float smoothness_;
    float reflectivity_;
};
static_assert(sizeof(Material) == 40, "Material layout");
static_assert(sizeof(Material) == sizeof(cpt_material), "Material == cpt_material");
