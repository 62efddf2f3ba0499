// ray_tracing_common.h — host-side POD types of the drop-in C++ API.
//
// Mirrors the reference's include/ray_tracing_common.h (constants :11-12, DispatchRayArgs
// :37-40) and the float3 helpers its scene code uses (Common/helper_math.h host path), with
// no CUDA or HIP types: float3 here is a 12-byte POD layout-identical to CUDA's float3 and
// to cpt_float3 in include/cpt.h.  Device-only types (Ray, RayPayload, IntersectionAttributes)
// live inside the HIP kernels and are not part of the host API.
#pragma once

#include <stdint.h>

#include <cmath>
#include <cstdlib>
#include <ctime>

#include "../cpt.h"

#define DEFAULT_RAY_TMAX 1e30f
#define BOUNCE_RAY_TMIN 2e-5f

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#ifndef MAX
#define MAX(a, b) ((a) > (b) ? (a) : (b))
#endif
#ifndef MIN
#define MIN(a, b) ((a) < (b) ? (a) : (b))
#endif
#ifndef ABS
#define ABS(a) ((a) >= 0 ? (a) : -(a))
#endif

typedef uint32_t uint;

#ifndef CPT_HAVE_FLOAT3
typedef cpt_float3 float3;
static_assert(sizeof(float3) == 12, "float3 must be 12 bytes");

inline float3 make_float3(float x, float y, float z) { return float3{x, y, z}; }
inline float3 make_float3(float s) { return float3{s, s, s}; }
inline float3 operator+(float3 a, float3 b) { return make_float3(a.x + b.x, a.y + b.y, a.z + b.z); }
inline float3 operator-(float3 a, float3 b) { return make_float3(a.x - b.x, a.y - b.y, a.z - b.z); }
inline float3 operator-(float3 a) { return make_float3(-a.x, -a.y, -a.z); }
inline float3 operator*(float3 a, float3 b) { return make_float3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline float3 operator*(float s, float3 a) { return make_float3(s * a.x, s * a.y, s * a.z); }
inline float3 operator*(float3 a, float s) { return make_float3(a.x * s, a.y * s, a.z * s); }
inline float3 operator+(float s, float3 a) { return make_float3(s + a.x, s + a.y, s + a.z); }
inline float3 operator+(float3 a, float s) { return make_float3(a.x + s, a.y + s, a.z + s); }
inline float3 operator/(float3 a, float s) { return make_float3(a.x / s, a.y / s, a.z / s); }
inline void operator+=(float3& a, float3 b) { a = a + b; }
inline void operator-=(float3& a, float3 b) { a = a - b; }
inline void operator*=(float3& a, float3 b) { a = a * b; }
inline float dot(float3 a, float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float length(float3 v) { return sqrtf(dot(v, v)); }
inline float3 normalize(float3 v) { float inv = 1.0f / sqrtf(dot(v, v)); return v * inv; }
inline float3 cross(float3 a, float3 b) {
    return make_float3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
#endif

// Host random helpers of the reference scene script (ray_tracing_math.hpp:30-41).  The
// reference's `float random()` collides with POSIX `long random(void)` on Linux, so it is
// spelled cpt_random() here.
inline float cpt_random() {
    static bool init = false;
    if (!init) {
        srand(static_cast<unsigned>(time(0)));
        init = true;
    }
    return static_cast<float>(rand()) / static_cast<float>(RAND_MAX);
}
inline float3 create_random_float3() {
    float a = cpt_random(), b = cpt_random(), c = cpt_random();
    return make_float3(a, b, c);
}

// ray_tracing_common.h:37-40 — the callback receives the BGRA8 frame of one pass.
struct DispatchRayArgs {
    void* cbParam;
    void (*Callback)(uint8_t* data, int width, int height, void* cbParam);
};
