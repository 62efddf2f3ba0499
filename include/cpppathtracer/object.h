// object.h — Object POD of the drop-in API (reference include/object.h:7-32).
#pragma once

#include "material.h"
#include "ray_tracing_common.h"

namespace PrimitiveType {
enum Enum { Sphere, Platform, Cylinder, Count };
}  // namespace PrimitiveType

// 72 bytes, byte-identical to the reference Object and to cpt_object.  IntersectionTest /
// ClosetHit are device code in the reference (object.cu:114-132); here they run inside the
// HIP kernels, so only the host AABB helpers remain as members.
class Object {
public:
    float3 GetAABBMin();   // object.cu:153-170
    float3 GetAABBMax();   // object.cu:134-151

    PrimitiveType::Enum type_;
    Material material_;

    float3 center_;
    float radius_;   // for Sphere and Cylinder
    float y_pos_;    // for Platform
    float height_;   // for Cylinder
};
static_assert(sizeof(Object) == 72, "Object layout");
static_assert(sizeof(Object) == sizeof(cpt_object), "Object == cpt_object");
