// cpt_path.hpp — device functions of the integrator shared by the megakernel
// (cpt_kernels.hip) and the wavefront kernels (cpt_wavefront.hip): environment fetch,
// intersectors, BVH walk, BSDF sampling, miss, camera ray generation.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpt_device.hpp"
#include "cpt_internal.hpp"
#include "cpt_stamps.hpp"
#include "cpt_tuning.hpp"

namespace cpt {

// ======================================================================================
// Environment texture (textures.cu:14-71): uchar4 cudaArray, normalized coordinates,
// Mirror addressing, Linear filter, NormalizedFloat read.  Texels live as packed RGBA8
// words, `cols` valid columns per row (the reference uploads width/4 texels per row,
// textures.cu:32-33); texels at x >= cols read as 0.  Bilinear weights are rounded to
// 1/256 (9-bit fixed point, 8 fractional bits), computed and blended in f32 in a fixed
// order.
// ======================================================================================
__device__ __forceinline__ int mirror_index(int i, int n) {
    if (i >= -n && i < 2 * n) {   // the range every sky fetch lands in: no integer division
        const int m = i < 0 ? -1 - i : i;
        return m >= n ? 2 * n - 1 - m : m;
    }
    int period = 2 * n;
    int m = i % period;
    if (m < 0) m += period;
    if (m >= n) m = period - 1 - m;
    return m;
}

// Texel index after addressing (cudaTextureAddressMode values, cpt.h); -1 = outside the
// texture under Border (border colour 0).
template <int ADDR>
__device__ __forceinline__ int address_index(int i, int n) {
    if (ADDR == 0) { int m = i % n; return m < 0 ? m + n : m; }         // wrap
    if (ADDR == 1) return i < 0 ? 0 : (i >= n ? n - 1 : i);           // clamp
    if (ADDR == 3) return (i < 0 || i >= n) ? -1 : i;                 // border
    return mirror_index(i, n);                                        // mirror
}

struct TexView { const uint32_t* texels; int w, h, cols; };

template <int ADDR>
__device__ __forceinline__ void texel(const TexView& t, int i, int j, float out[3]) {
    int x = address_index<ADDR>(i, t.w), y = address_index<ADDR>(j, t.h);
    if (x < 0 || y < 0 || x >= t.cols) { out[0] = out[1] = out[2] = 0.0f; return; }
    uint32_t v = t.texels[(size_t)y * t.cols + x];
    out[0] = dm::div255(v & 0xffu);          // (float)c / 255.0f, exactly
    out[1] = dm::div255((v >> 8) & 0xffu);
    out[2] = dm::div255((v >> 16) & 0xffu);
}

// tex2D<float4> at normalized (u, v), rgb (textures.cu:68-71).  Linear: taps at
// floor(u*w - 0.5) and +1, weights rounded to 1/256; point: the texel at floor(u*w).
template <int ADDR, bool LINEAR>
__device__ inline v3 tex_fetch(const TexView& t, float u, float v) {
    if (t.cols <= 0) return mk1(0.0f);
    if (!LINEAR) {
        float x = u * (float)t.w, y = v * (float)t.h;
        if (!(x > -1e7f && x < 1e7f && y > -1e7f && y < 1e7f)) return mk1(0.0f);
        float c[3];
        texel<ADDR>(t, (int)__builtin_floorf(x), (int)__builtin_floorf(y), c);
        return mk(c[0], c[1], c[2]);
    }
    float x = u * (float)t.w - 0.5f;
    float y = v * (float)t.h - 0.5f;
    if (!(x > -1e7f && x < 1e7f && y > -1e7f && y < 1e7f)) return mk1(0.0f);
    float fx = __builtin_floorf(x), fy = __builtin_floorf(y);
    float a = __builtin_floorf((x - fx) * 256.0f + 0.5f) * 0.00390625f;
    float b = __builtin_floorf((y - fy) * 256.0f + 0.5f) * 0.00390625f;
    int i0 = (int)fx, j0 = (int)fy;
    float t00[3], t10[3], t01[3], t11[3];
    texel<ADDR>(t, i0, j0, t00);
    texel<ADDR>(t, i0 + 1, j0, t10);
    texel<ADDR>(t, i0, j0 + 1, t01);
    texel<ADDR>(t, i0 + 1, j0 + 1, t11);
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    float r[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) r[c] = ((w00 * t00[c] + w10 * t10[c]) + w01 * t01[c]) + w11 * t11[c];
    return mk(r[0], r[1], r[2]);
}

__device__ inline v3 tex_fetch_dyn(const TexView& t, int addr, int filter, float u, float v) {
    const bool lin = filter != 0;
    switch (addr) {
        case 0: return lin ? tex_fetch<0, true>(t, u, v) : tex_fetch<0, false>(t, u, v);
        case 1: return lin ? tex_fetch<1, true>(t, u, v) : tex_fetch<1, false>(t, u, v);
        case 3: return lin ? tex_fetch<3, true>(t, u, v) : tex_fetch<3, false>(t, u, v);
        default: return lin ? tex_fetch<2, true>(t, u, v) : tex_fetch<2, false>(t, u, v);
    }
}

// The sky: AddTexByFile's defaults, mirror + linear (textures.h:9-11).
__device__ inline v3 tex2d(const KParams& p, float u, float v) {
    return tex_fetch<2, true>(TexView{p.env, p.env_w, p.env_h, p.env_cols}, u, v);
}

// ======================================================================================
// Per-segment ray with its exact reciprocals (see qdiv in cpt_device.hpp).
// ======================================================================================
typedef float f2v __attribute__((ext_vector_type(2)));

// Margins of the ordered walk's conservative slab test (slab_pass below): relative to the
// plane distances (folded into the per-ray reciprocals, RayK::inx ...) and absolute (the exit
// offsets carry 2 x WALK_MARGIN_ABS, rounded up, and 1e-6 for the relative margin's rounding).
constexpr float WALK_MARGIN_REL = 1e-3f, WALK_MARGIN_ABS = 1e-4f;
constexpr float SLAB_SHRINK = 1.0f - WALK_MARGIN_REL, SLAB_GROW = 1.0f + WALK_MARGIN_REL;
constexpr float SLAB_ABS = 2.0f * WALK_MARGIN_ABS * (1.0f + 2.0f * WALK_MARGIN_REL) * SLAB_GROW + 1e-6f;

struct RayK {
    v3 o, d;
    float tmin;
    double yx, yy, yz;   // 1/d.x, 1/d.y, 1/d.z   (exact slab planes; d.y also for caps / platform);
                         // yx and yz are filled by with_slab() where an exact slab test runs
    double ya;           // 1/dot(d,d)            (sphere roots, object.cu:15-20)
    double yc;           // 1/(dx*dx + dz*dz)     (cylinder side roots, object.cu:69-79)
    float aa, ac;        // dot(d,d) and dx*dx + dz*dz themselves: the quadratics' `a` (per ray)
    // The ordered walk's conservative slabs (slab_reject<*, true>, wide_pair, slab_pass): a plane
    // p of axis a is entered at t = fma(p, in_a, cn_a) and left at fma(p, if_a, cf_a), with
    // in_a = i (1 - 1e-3), if_a = i (1 + 1e-3) for the f32 i = 1/d_a (the relative margin: an
    // entry distance shrinks toward 0 and an exit distance grows by 1e-3 of itself) and
    // c_a = -(o_a * i_a) -+ beta_a; beta_a = 2^-20 |o_a * i_a| covers the rounding of the product
    // and the sum, so an entry plane's t is never above (p - o_a) * in_a before its own rounding
    // (DESIGN.md §Ordered walk).  The exit offsets also carry the absolute margin.  A skipped
    // axis (|d| < 1e-30) has i = 0 and c = -+2e30: no constraint, which only widens.
    float inx, iny, inz, ifx, ify, ifz;
    float nx, ny, nz;    // entry offsets
    float fx, fy, fz;    // exit offsets (+ SLAB_ABS)
    float t3;            // conservative tmin limit: t3 - 1e-3 |t3|, t3 = (tmin - 1e-4) * (1 + 2e-3)
};

// Entry / exit reciprocals and offsets of one axis of the conservative slabs (RayK::inx ...).
__device__ __forceinline__ void slab_axis(float o, float d, float& in, float& if_, float& cn, float& cf) {
    const float i = __builtin_fabsf(d) >= 1e-30f ? rcp_f(d) : 0.0f;
    in = i * SLAB_SHRINK;
    if_ = i * SLAB_GROW;
    const float pn = o * in, pf = o * if_;
    cn = i != 0.0f ? -pn - __builtin_fabsf(pn) * 0x1p-20f : -DEFAULT_RAY_TMAX * 2;
    cf = i != 0.0f ? (-pf + __builtin_fabsf(pf) * 0x1p-20f) + SLAB_ABS : DEFAULT_RAY_TMAX * 2;
}

__device__ __forceinline__ RayK make_rayk(const Ray& r) {
    RayK k;
    k.o = r.o;
    k.d = r.d;
    k.tmin = r.tmin;
    k.yx = 0.0;   // with_slab()
    k.yy = rcp_d(r.d.y);
    k.yz = 0.0;
    k.aa = dot(r.d, r.d);
    k.ac = r.d.x * r.d.x + r.d.z * r.d.z;
    k.ya = rcp_d(k.aa);
    k.yc = rcp_d(k.ac);
    slab_axis(r.o.x, r.d.x, k.inx, k.ifx, k.nx, k.fx);
    slab_axis(r.o.y, r.d.y, k.iny, k.ify, k.ny, k.fy);
    slab_axis(r.o.z, r.d.z, k.inz, k.ifz, k.nz, k.fz);
    const float t3 = (r.tmin - 1e-4f) * (1.0f + 2e-3f);
    k.t3 = t3 - WALK_MARGIN_REL * __builtin_fabsf(t3);
    return k;
}

// The exact slab test's reciprocals, computed where one runs (the winner certificate and the
// reference walk), so the ordered walk does not carry them.
__device__ __forceinline__ RayK with_slab(const RayK& k0) {
    RayK k = k0;
    k.yx = rcp_d(k0.d.x);
    k.yz = rcp_d(k0.d.z);
    return k;
}

// ======================================================================================
// Intersectors (object.cu:10-128) on an inline leaf.  `tmax` is the traversal's shrinking
// closest distance (TraceRay's by-value ray, bvh.cu:167).
// ======================================================================================
struct Hit { v3 normal, pos; };

// Deferred hit attributes: a leaf test only decides whether the primitive replaces the
// current closest hit (and shrinks tmax); the hit position and normal of the WINNER are
// computed once after the walk from (t, node, kind), with the reference's own formulas.
// The position is ray.origin + temp * ray.dir in every intersector (object.cu:21,29,44,...),
// and the normal depends only on which case accepted:
enum : int {
    HK_SPHERE_ROOT1 = 0,   // (p - c) / radius           (object.cu:23-24, signed radius)
    HK_SPHERE_ROOT2 = 1,   // normalize(p - c)            (object.cu:30)
    HK_CYL_SIDE = 2,       // normalize(p.x-cx, 0, p.z-cz) (object.cu:97-99,105-107)
    HK_FACING_Y = 3        // normalize(0, -d.y, 0): caps and platform (object.cu:43,62,75)
};

// Sphere (object.cu:10-35)
__device__ __forceinline__ bool sphere_test(const Node& s, const RayK& ray, float& tmax, int& kind) {
    const v3 c = mk(s.a0, s.a1, s.a2);
    const float radius = s.b0;
    const v3 A_C = ray.o - c;
    const float b = dot(A_C, ray.d);
    const float cc = dot(A_C, A_C) - radius * radius;
    const float a = dot(ray.d, ray.d);
    const float disc = b * b - a * cc;
    if (!(disc > 0)) return false;
    const float sq = __builtin_sqrtf(disc);
    float temp = qdiv(-b - sq, a, ray.ya);
    if (temp < tmax && temp > ray.tmin) {
        tmax = temp;
        kind = HK_SPHERE_ROOT1;
        return true;
    }
    temp = qdiv(-b + sq, a, ray.ya);
    if (temp < tmax && temp > ray.tmin) {
        tmax = temp;
        kind = HK_SPHERE_ROOT2;
        return true;
    }
    return false;
}

// Platform: the plane y = y_pos, only when the ray approaches it (object.cu:37-48)
__device__ __forceinline__ bool platform_test(const Node& pl, const RayK& ray, float& tmax, int& kind) {
    const float y_pos = pl.b1;
    if ((ray.o.y < y_pos && ray.d.y > 0.f) || (ray.o.y > y_pos && ray.d.y < 0.f)) {
        const float temp = qdiv(y_pos - ray.o.y, ray.d.y, ray.yy);
        if (temp < tmax && temp > ray.tmin) {
            tmax = temp;
            kind = HK_FACING_Y;
            return true;
        }
    }
    return false;
}

// One cylinder cap disk (object.cu:52-77).  The reference's `sqrtf(q) < radius` is decided as
// `q <= bound` with the leaf's precomputed bound (Node::b1 of a cylinder leaf, cpt_capi.cpp
// cap_disk_bound): the same decision for every float q, without the correctly rounded square
// root.
__device__ __forceinline__ bool cap_test(float cx, float cz, float bound, const RayK& ray, float& tmax, int& kind,
                                         float ypos) {
    if ((ray.o.y < ypos && ray.d.y > 0.f) || (ray.o.y > ypos && ray.d.y < 0.f)) {
        const float temp = qdiv(ypos - ray.o.y, ray.d.y, ray.yy);
        if (temp < tmax && temp > ray.tmin) {
            const float hx = ray.o.x + temp * ray.d.x, hz = ray.o.z + temp * ray.d.z;
            if ((hx - cx) * (hx - cx) + (hz - cz) * (hz - cz) <= bound) {
                tmax = temp;
                    kind = HK_FACING_Y;
                return true;
            }
        }
    }
    return false;
}

// Cylinder: caps, then the side quadratic with the y-range check (object.cu:50-112).  The
// second root can never replace an accepted first root (temp2 >= temp1 under monotone
// rounding), so the side returns after the first accepted root.
__device__ __forceinline__ bool cylinder_test(const Node& cy, const RayK& ray, float& tmax, int& kind) {
    const float ccx = cy.a0, ccy = cy.a1, ccz = cy.a2, r = cy.b0, height = cy.b2;
    bool ret = false;
    const float upper = ccy + height / 2;
    if (cap_test(ccx, ccz, cy.b1, ray, tmax, kind, upper)) ret = true;
    const float lower = ccy - height / 2;
    if (cap_test(ccx, ccz, cy.b1, ray, tmax, kind, lower)) ret = true;
    const float dx = ray.d.x, dz = ray.d.z;
    const float cx = ray.o.x - ccx, cz = ray.o.z - ccz;
    const float a = dx * dx + dz * dz;
    const float b = cx * dx + cz * dz;
    const float c = cx * cx + cz * cz - r * r;
    const float disc = b * b - a * c;
    if (disc > 0.f) {
        const float sq = __builtin_sqrtf(disc);
        float temp = qdiv(-b - sq, a, ray.yc);
        float hy = ray.o.y + temp * ray.d.y;
        if (temp < tmax && temp > ray.tmin && hy > lower && hy < upper) {
            tmax = temp;
            kind = HK_CYL_SIDE;
            return true;
        }
        temp = qdiv(-b + sq, a, ray.yc);
        hy = ray.o.y + temp * ray.d.y;
        if (temp < tmax && temp > ray.tmin && hy > lower && hy < upper) {
            tmax = temp;
            kind = HK_CYL_SIDE;
            return true;
        }
    }
    return ret;
}

__device__ __forceinline__ bool leaf_test(const Node& nd, const RayK& ray, float& tmax, int& kind) {
    const int type = nd.code & 3;
    if (type == 0) return sphere_test(nd, ray, tmax, kind);
    if (type == 2) return cylinder_test(nd, ray, tmax, kind);
    if (type == 1) return platform_test(nd, ray, tmax, kind);
    return false;                        // unknown PrimitiveType: IntersectionTest -> false
}

// Attributes of the winning primitive (see HK_*).
__device__ __forceinline__ Hit hit_attributes(const Node& nd, const RayK& ray, float t, int kind) {
    Hit h;
    h.pos = ray.o + t * ray.d;
    const v3 c = mk(nd.a0, nd.a1, nd.a2);
    const v3 pc = h.pos - c;
    if (kind == HK_SPHERE_ROOT1) {
        // (p - c) / radius, each component the IEEE quotient: qdiv with the sphere leaf's double
        // reciprocal of its radius (Node::b1/b2, cpt_capi.cpp make_node)
        const double y = __hiloint2double(__float_as_int(nd.b2), __float_as_int(nd.b1));
        h.normal = mk(qdiv(pc.x, nd.b0, y), qdiv(pc.y, nd.b0, y), qdiv(pc.z, nd.b0, y));
    } else {
        // the other three cases normalize a vector of their own: one normalize for the wave
        const bool cyl = kind == HK_CYL_SIDE, root2 = kind == HK_SPHERE_ROOT2;
        const v3 v = mk(root2 || cyl ? pc.x : 0.f, root2 ? pc.y : (cyl ? 0.f : -ray.d.y), root2 || cyl ? pc.z : 0.f);
        h.normal = normalize(v);
    }
    return h;
}

// ======================================================================================
// SceneBVH::TraceRay (bvh.cu:167-205) as a stackless skip-link walk.  The nodes are stored
// in the exact order the reference's stack DFS pops them (right child first), so visiting
// n, then n+1 on a box hit or node.miss on a box miss / after a leaf, reproduces the
// reference's visit sequence, leaf-before-box order and pruning against the shrinking tmax
// one for one — no stack, no scratch memory.
// ======================================================================================

struct Counters {
    uint32_t segments, nodes, prims, hits, misses, fallbacks;
    uint32_t gnodes;   // wide-node visits read from the image in global memory (not the LDS copy)
};

// Slab test of one internal node (bvh.cu:181-200).  The six plane distances use the exact
// quotient; if any of them is zero/subnormal the node is redone with the IEEE divide.
// FAST (rays without NaN): the plane distances of the axes that are used are never NaN
// (finite box coordinate minus finite origin, times a finite reciprocal), so the ternary
// MIN/MAX of the reference equal v_min/v_max_f32 up to the sign of a zero, which none of
// the three comparisons can see.  Rays carrying a NaN take the exact ternary form.
// CONS (the ordered walk's tree): the interval from f32 reciprocals (no exactness needed),
// widened by a relative margin before the three comparisons, so that a primitive whose
// computed hit lies slightly outside its box by rounding is still tested (DESIGN.md
// §Ordered walk).  The margin dwarfs the reciprocal's few-ulp error.
// The conservative walk's tmax limit (slab_reject<*, true>'s `tmax` argument).
__device__ __forceinline__ float walk_limit(float tmax) {
    return ((tmax + WALK_MARGIN_ABS) * (1.0f + 2.0f * WALK_MARGIN_REL)) * SLAB_GROW;
}

// The conservative pass test on a box's entry / exit distances: lo = max over axes of the
// entry planes' fma(p, in, cn), hi = min of the exit planes' fma(p, if, cf) (RayK::inx ...,
// which carry the relative and absolute margins); the box passes iff
//     max(lo, t3') <= min(hi, limit')
// with t3' = t3 - 1e-3 |t3| and limit' = walk_limit(tmax) (both widened the same way).  It
// passes every box the round-2 test passed (reject iff lo - hi > 1e-3 (|lo| + |hi|) + 2e-4, or
// lo > (tmax + 1e-4) * 1.002, or hi < (tmin - 1e-4) * 1.002, on unscaled distances): for the
// distances >= 0 the scaled ones are the old ones times (1 -+ 1e-3), and the few in (t3, 0)
// differ from that by less than the 1e-6 the exit offsets add (DESIGN.md §Ordered walk).
// lo' = max(lo, t3') is also the child's sort key.
__device__ __forceinline__ bool slab_pass(float& lo, float hi, float t3, float limit) {
    lo = __builtin_fmaxf(lo, t3);
    return lo <= __builtin_fminf(hi, limit);
}

template <bool FAST, bool CONS = false>
__device__ __forceinline__ bool slab_reject(const Node& nd, const RayK& ray, float tmax) {
    if (CONS) {
        // The entry plane of an axis is its min plane when 1/d >= 0 (also on a skipped axis).
        const bool px = ray.inx >= 0.0f, py = ray.iny >= 0.0f, pz = ray.inz >= 0.0f;
        float lo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(px ? nd.a0 : nd.b0, ray.inx, ray.nx),
                                                   __builtin_fmaf(py ? nd.a1 : nd.b1, ray.iny, ray.ny)),
                                   __builtin_fmaf(pz ? nd.a2 : nd.b2, ray.inz, ray.nz));
        const float hi = __builtin_fminf(__builtin_fminf(__builtin_fmaf(px ? nd.b0 : nd.a0, ray.ifx, ray.fx),
                                                         __builtin_fmaf(py ? nd.b1 : nd.a1, ray.ify, ray.fy)),
                                         __builtin_fmaf(pz ? nd.b2 : nd.a2, ray.ifz, ray.fz));
        return !slab_pass(lo, hi, ray.t3, tmax);
    }
    float t0x = qdiv_raw(nd.a0 - ray.o.x, ray.yx), t1x = qdiv_raw(nd.b0 - ray.o.x, ray.yx);
    float t0y = qdiv_raw(nd.a1 - ray.o.y, ray.yy), t1y = qdiv_raw(nd.b1 - ray.o.y, ray.yy);
    float t0z = qdiv_raw(nd.a2 - ray.o.z, ray.yz), t1z = qdiv_raw(nd.b2 - ray.o.z, ray.yz);
    float mn = __builtin_fminf(__builtin_fminf(__builtin_fminf(__builtin_fabsf(t0x), __builtin_fabsf(t1x)),
                                               __builtin_fminf(__builtin_fabsf(t0y), __builtin_fabsf(t1y))),
                               __builtin_fminf(__builtin_fabsf(t0z), __builtin_fabsf(t1z)));
    if (__builtin_expect(mn < FLT_MIN_NORMAL, 0)) {
        t0x = (nd.a0 - ray.o.x) / ray.d.x; t1x = (nd.b0 - ray.o.x) / ray.d.x;
        t0y = (nd.a1 - ray.o.y) / ray.d.y; t1y = (nd.b1 - ray.o.y) / ray.d.y;
        t0z = (nd.a2 - ray.o.z) / ray.d.z; t1z = (nd.b2 - ray.o.z) / ray.d.z;
    }
    // axes with d == 0 are skipped (bvh.cu:182,188,194): selects, not branches
    float lo = -DEFAULT_RAY_TMAX * 2, hi = DEFAULT_RAY_TMAX * 2;
    float lx, hx, ly, hy, lz, hz;
    if (FAST) {
        lx = __builtin_fmaxf(lo, __builtin_fminf(t0x, t1x));
        hx = __builtin_fminf(hi, __builtin_fmaxf(t0x, t1x));
    } else {
        lx = tmax_(lo, tmin_(t0x, t1x));
        hx = tmin_(hi, tmax_(t0x, t1x));
    }
    lo = ray.d.x != 0.f ? lx : lo;
    hi = ray.d.x != 0.f ? hx : hi;
    if (FAST) {
        ly = __builtin_fmaxf(lo, __builtin_fminf(t0y, t1y));
        hy = __builtin_fminf(hi, __builtin_fmaxf(t0y, t1y));
    } else {
        ly = tmax_(lo, tmin_(t0y, t1y));
        hy = tmin_(hi, tmax_(t0y, t1y));
    }
    lo = ray.d.y != 0.f ? ly : lo;
    hi = ray.d.y != 0.f ? hy : hi;
    if (FAST) {
        lz = __builtin_fmaxf(lo, __builtin_fminf(t0z, t1z));
        hz = __builtin_fminf(hi, __builtin_fmaxf(t0z, t1z));
    } else {
        lz = tmax_(lo, tmin_(t0z, t1z));
        hz = tmin_(hi, tmax_(t0z, t1z));
    }
    lo = ray.d.z != 0.f ? lz : lo;
    hi = ray.d.z != 0.f ? hz : hi;
    return lo > hi || lo > tmax || hi < ray.tmin;
}

// slab_reject<FAST, true> on a walk-tree inner node stored in octant form (cpt_capi.cpp
// linearise): a.xyz are the planes a ray of the node's octant enters through, b.xyz the ones
// it leaves through.  For an axis with i != 0 the sign of i is the octant's, so the entry
// plane's distance is the min of the pair and the exit plane's the max (the subtraction, the
// product and the fma are monotone); a skipped axis gives -2e30 / +2e30 in that order.  So
// lo and hi are bit for bit those of the min/max form and the decision is the same.

__device__ __forceinline__ bool slab_reject_octant(const Node& nd, const RayK& ray, float limit) {
    float lo = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(nd.a0, ray.inx, ray.nx), __builtin_fmaf(nd.a1, ray.iny, ray.ny)),
                               __builtin_fmaf(nd.a2, ray.inz, ray.nz));
    const float hi = __builtin_fminf(__builtin_fminf(__builtin_fmaf(nd.b0, ray.ifx, ray.fx), __builtin_fmaf(nd.b1, ray.ify, ray.fy)),
                                     __builtin_fmaf(nd.b2, ray.ifz, ray.fz));
    return !slab_pass(lo, hi, ray.t3, limit);
}

// Node fetch.  BufSrc reads through a buffer descriptor over the whole node array (built from
// kernel arguments, so it is wave-uniform and lives in SGPRs): a 32-bit per-lane byte offset
// instead of 64-bit address arithmetic, and out-of-range offsets read 0 instead of needing a
// clamp (the walk never uses a node past its order's end).
typedef unsigned int v4u32 __attribute__((ext_vector_type(4)));

struct BufSrc {
    __amdgpu_buffer_rsrc_t rsrc;
    uint32_t base;   // byte offset of the order's node 0
    __device__ __forceinline__ Node operator()(uint32_t i) const {
        const uint32_t off = base + (i << 5);
        const v4u32 a = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off, 0, 0);
        const v4u32 b = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 16, 0, 0);
        Node n;
        n.a0 = __uint_as_float(a.x); n.a1 = __uint_as_float(a.y); n.a2 = __uint_as_float(a.z); n.miss = (int32_t)a.w;
        n.b0 = __uint_as_float(b.x); n.b1 = __uint_as_float(b.y); n.b2 = __uint_as_float(b.z); n.code = (int32_t)b.w;
        return n;
    }
};

// The wide tree's compact image (cpt_capi.cpp linearise_wide): 7 x 16 B per node, after the
// eight binary octant orders; padded to whole 32-B Nodes.
__host__ __device__ __forceinline__ int wide_compact_nodes(int n_wide) { return (7 * n_wide + 1) / 2; }
// Node index of the compact image, and of the wide tree's leaf array after it (the image's
// leaf refs index that array).
__host__ __device__ __forceinline__ int wide_image_base(const KParams& p) { return p.n_nodes + 8 * p.n_walk; }
__host__ __device__ __forceinline__ int wide_leaves_base(const KParams& p) {
    return wide_image_base(p) + wide_compact_nodes(p.n_wide);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t node_rsrc(const KParams& p) {
    const uint32_t bytes = (uint32_t)(wide_leaves_base(p) + p.n_leaves) * (uint32_t)sizeof(Node);
    return __builtin_amdgcn_make_buffer_rsrc((void*)p.nodes, (short)0, (int)bytes, 0x00020000);
}

// The node order a ray walks: the reference order, or with CPT_TRAVERSAL_ORDERED the walk
// tree's order for its direction octant (near child of every split first, DESIGN.md
// §Ordered walk).  Returns the first node and sets the order's length.
__device__ __forceinline__ uint32_t walk_order(const KParams& p, v3 d, int& n) {
    const int oct = (d.x < 0.f ? 1 : 0) | (d.y < 0.f ? 2 : 0) | (d.z < 0.f ? 4 : 0);
    n = p.n_walk;
    return (uint32_t)(p.n_nodes + oct * p.n_walk);   // first node of the octant's order
}

// Leaf test with the reference's first-found rule for equal distances.  `rank` is the leaf's
// position in the reference order, best_rank the current closest primitive's.  A primitive the
// reference meets earlier (rank < best_rank; only possible in the ordered walk) must win a
// tie, so it is tested against next_up(tmax): "temp < next_up(tmax)" == "temp <= tmax".  Its
// first accepted case sets tmax = temp, so its later cases compare strictly, as in the
// reference.  tmax > 0 always (hits need temp > tmin >= 0), so next_up is the bit pattern + 1.
// Object::GetAABBMin/Max (object.cu:134-170) of a leaf's primitive, as the host computes it.
__device__ __forceinline__ void leaf_aabb(const Node& nd, Node& box) {
    const float tol = 2e-5f * 5.f;
    const int type = nd.code & 3;
    const float r = nd.b0 >= 0 ? nd.b0 : -nd.b0;
    if (type == 0) {
        box.a0 = nd.a0 - r; box.a1 = nd.a1 - r; box.a2 = nd.a2 - r;
        box.b0 = nd.a0 + r; box.b1 = nd.a1 + r; box.b2 = nd.a2 + r;
    } else if (type == 1) {
        box.a0 = -1e30f * 5; box.a1 = nd.b1 - tol; box.a2 = -1e30f * 5;
        box.b0 = 1e30f * 5; box.b1 = nd.b1 + tol; box.b2 = 1e30f * 5;
    } else if (type == 2) {
        box.a0 = nd.a0 - r; box.a1 = nd.a1 - nd.b2 / 2 - tol; box.a2 = nd.a2 - r;
        box.b0 = nd.a0 + r; box.b1 = nd.a1 + nd.b2 / 2 + tol; box.b2 = nd.a2 + r;
    } else {
        box.a0 = box.a1 = box.a2 = box.b0 = box.b1 = box.b2 = 0.f;
    }
}

// The winner certificate without quotients.  The certificate asks whether the exact slab test
// (slab_reject<FAST> with exact quotients, bvh.cu:181-200) passes the winner's box at
// tmax = t (the winner's distance).  On an axis with d != 0, with s_a = RN(a - o) and
// s_b = RN(b - o) the reference's own differences for the box planes a <= b, the box passes if
// every such axis has RN(s_a / d) and RN(s_b / d) on either side of t (then lo <= t <= hi, and
// hi >= t > tmin).  For d > 0 that follows from s_a <= t d <= s_b (RN is monotone and t is a
// float); for d < 0 the quotients swap roles and the inequalities flip, which is the same
// condition.  So: s_a <= T and s_b >= U with T = RN(P - 2^-21 |P|), U = RN(P + 2^-21 |P|), P =
// RN(t d): for a normal P, |P - t d| <= 2^-24 |P|, and the single rounding of the fma keeps T
// below and U above t d.  Axes with d == 0 are skipped, as in the reference; a subnormal or zero
// P, an infinite one and NaNs give no certificate.  When this is inconclusive (the hit lies
// within ~2^-21 of a box plane) the exact test decides.  One product and two fmas per axis
// instead of two double reciprocals and six double quotients: C4 2233-2241 vs 2169-2183
// Mpaths/s, VALU instructions -2.7% (profiles/r06/cert/).  Checked against the exact test in
// numpy (tests/test_certificate.py).
__device__ __forceinline__ bool cert_inside_axis(float a, float b, float o, float d, float t) {
    const float s_a = a - o, s_b = b - o;
    const float P = t * d;
    const float T = __builtin_fmaf(__builtin_fabsf(P), -0x1p-21f, P);
    const float U = __builtin_fmaf(__builtin_fabsf(P), 0x1p-21f, P);
    return d == 0.0f || (s_a <= T && s_b >= U && __builtin_fabsf(P) >= 0x1p-100f);
}
__device__ __forceinline__ bool cert_inside(const Node& box, const RayK& ray, float t) {
    return cert_inside_axis(box.a0, box.b0, ray.o.x, ray.d.x, t) && cert_inside_axis(box.a1, box.b1, ray.o.y, ray.d.y, t) &&
           cert_inside_axis(box.a2, box.b2, ray.o.z, ray.d.z, t);
}

// Sphere (object.cu:10-35) and cylinder (object.cu:50-112) in one code path for a wave that
// holds both.  Each lane computes exactly its own type's expressions in the reference's
// operation order: dot(A_C, d) = (x + y) + z for a sphere, cx*dx + cz*dz for a cylinder side
// (the y term is selected in or out, never multiplied by 0), likewise for a and c; the root
// quotients use that type's own reciprocal (ya or yc).  The cylinder's caps run first (only on
// cylinder lanes), then the shared roots with the cylinder's y-range check.
__device__ __forceinline__ bool sphere_cyl_test(const Node& nd, const RayK& ray, float& tmax, int& kind) {
    const bool sph = (nd.code & 3) == 0;
    const float r = nd.b0;
    bool ret = false;
    float lower = 0.f, upper = 0.f;
    if (!sph) {
        upper = nd.a1 + nd.b2 / 2;
        if (cap_test(nd.a0, nd.a2, nd.b1, ray, tmax, kind, upper)) ret = true;
        lower = nd.a1 - nd.b2 / 2;
        if (cap_test(nd.a0, nd.a2, nd.b1, ray, tmax, kind, lower)) ret = true;
    }
    const float cx = ray.o.x - nd.a0, cy = ray.o.y - nd.a1, cz = ray.o.z - nd.a2;
    const float dx = ray.d.x, dy = ray.d.y, dz = ray.d.z;
    const float bx = cx * dx, ax = dx * dx, qx = cx * cx;
    const float b = (sph ? bx + cy * dy : bx) + cz * dz;
    // (dx*dx + dy*dy) + dz*dz or dx*dx + dz*dz: the ray's own, computed once (RayK::aa / ac)
    const float a = sph ? ray.aa : ray.ac;
    (void)ax;
    const float c = ((sph ? qx + cy * cy : qx) + cz * cz) - r * r;
    const float disc = b * b - a * c;
    if (!(disc > 0.f)) return ret;
    const double y = sph ? ray.ya : ray.yc;
    const float sq = __builtin_sqrtf(disc);
    float temp = qdiv(-b - sq, a, y);
    float hy = ray.o.y + temp * dy;
    if (temp < tmax && temp > ray.tmin && (sph || (hy > lower && hy < upper))) {
        tmax = temp;
        kind = sph ? HK_SPHERE_ROOT1 : HK_CYL_SIDE;
        return true;
    }
    temp = qdiv(-b + sq, a, y);
    hy = ray.o.y + temp * dy;
    if (temp < tmax && temp > ray.tmin && (sph || (hy > lower && hy < upper))) {
        tmax = temp;
        kind = sph ? HK_SPHERE_ROOT2 : HK_CYL_SIDE;
        return true;
    }
    return ret;
}

// The ordered walk (CONS) pretests a cylinder's own box with the conservative slab before its
// exact test (PRETEST; the wide walk's parent already tested it), and runs spheres and
// cylinder sides through one quadratic (sphere_cyl_test).
template <bool FAST, bool CONS, bool PRETEST = true>
__device__ __forceinline__ bool ranked_leaf_test(const Node& nd, const RayK& ray, float& tmax, int& kind, int& best_rank) {
    float tm = nd.miss < best_rank ? __int_as_float(__float_as_int(tmax) + 1) : tmax;
    if (CONS && PRETEST && (nd.code & 3) == 2) {
        Node box;
        leaf_aabb(nd, box);
        if (slab_reject<FAST, true>(box, ray, walk_limit(tm))) return false;
    }
    if (CONS && ((nd.code & 1) == 0)) {   // sphere (0) or cylinder (2)
        if (!sphere_cyl_test(nd, ray, tm, kind)) return false;
    } else if (!leaf_test(nd, ray, tm, kind)) {
        return false;
    }
    tmax = tm;
    best_rank = nd.miss;
    return true;
}

// Returns 1 on a hit, 0 on a miss, and -1 (CONS only) when the winner's certificate fails:
// the caller then walks the reference order instead.
template <bool STATS, bool FAST, bool CONS = false, typename SRC>
__device__ __forceinline__ int trace(const SRC& nodes, int n_nodes, const RayK& ray, Hit& h, int& code_out,
                                     Counters& cnt) {
    float tmax = DEFAULT_RAY_TMAX;
    int best = -1, kind = 0;
    int best_rank = 0x7fffffff;   // reference-order position of the current closest primitive
    int ni = 0;
    Node nd{};
    if (n_nodes > 0) nd = nodes(0);
    // The successor of node ni is ni + 1 (box hit: its first child; after a leaf) or nd.miss
    // (box miss); the chosen one is loaded after the node's test (the other waves of the SIMD
    // hide the latency).
    while (ni < n_nodes) {
        const bool leaf = nd.code >= 0;
        if (STATS) cnt.nodes++;
        bool take_a = false;
        if (leaf) {
            // IntersectionTest first (bvh.cu:175-180); the leaf's own box test is moot
            if (STATS) cnt.prims++;
            int k;
            if (ranked_leaf_test<FAST, CONS>(nd, ray, tmax, k, best_rank)) { best = ni; kind = k; }
        } else {
            take_a = CONS ? !slab_reject_octant(nd, ray, walk_limit(tmax)) : !slab_reject<FAST>(nd, ray, tmax);
        }
        ni = take_a || leaf ? ni + 1 : nd.miss;
        nd = nodes(ni);
    }
    if (best < 0) return 0;
    const Node w = nodes(best);
    if (CONS) {
        // Certificate: the winner's own box passes the exact slab test at tmax = t_win.  Its
        // reference ancestors contain that box, so (slab distances are monotone in the box
        // planes) they pass at any tmax >= t_win: the reference walk reaches the winner, and
        // with every primitive it tests also tested here, it keeps the same one.
        Node box;
        leaf_aabb(w, box);
        if (!cert_inside(box, ray, tmax) && slab_reject<FAST>(box, with_slab(ray), tmax)) return -1;
    }
    h = hit_attributes(w, ray, tmax, kind);
    code_out = w.code;
    return 1;
}

// Leaf rounds of the wide walk run when SPEC_LEAF_ROUND 64ths of the wave's working lanes are
// stopped at a parked leaf (cpt_tuning.hpp).

// ======================================================================================
// The ordered walk on the 4-wide walk tree (DESIGN.md §Ordered walk, Execution).  One iteration reads a
// 112-B node of the tree's compact image (cpt_capi.cpp linearise_wide) and tests its four
// children's boxes with the conservative octant-form slab; the nearest hit child is taken
// next, the other hits go onto a per-lane stack in LDS (far ones first).  Leaves are parked
// and tested in wave-wide rounds: a lane that meets a leaf parks it and walks on; it stops at
// a second leaf or when its stack is empty, and once enough lanes are stopped every lane
// with a parked leaf tests it (Aila & Laine's speculative traversal).  The boxes tested are
// the binary walk tree's, so the superset argument holds: every primitive the plain walk
// tests, whose box passes the conservative test, is tested here too, under a limit that is
// never below the final tmax; the rank rule and the certificate are unchanged.
// ======================================================================================
constexpr int WIDE_LANES = 256;   // block size of the kernels without the LDS image

// Number of set bits of a wave-uniform mask as a 32-bit value (two 32-bit popcounts: the
// compiler then compares it with SALU s_cmp_*_u32; a 64-bit popcount it compares with VALU
// v_cmp_*_u64).  (Not inline asm: s_bcnt1 writes SCC, which an asm statement cannot declare.)
__device__ __forceinline__ uint32_t wave_count(uint64_t m) {
    return (uint32_t)__builtin_popcount((uint32_t)m) + (uint32_t)__builtin_popcount((uint32_t)(m >> 32));
}

typedef __attribute__((address_space(3))) int16_t lds_i16;

// The compact image's first LDS_TREE_NODES nodes are staged in LDS (k_megakernel<..., LDST>,
// k_wf_extend<..., LDST>); a larger tree's remaining nodes are read from the image in global
// memory (L2-resident).  The host numbers the wide nodes largest box first, parents before
// children (cpt_capi.cpp linearise_wide), so the LDS part is the top of the tree, the part
// every ray walks.
// (LDS_TREE_NODES, lds_tree_nodes: cpt_internal.hpp)

struct WideNode {
    f2v e[3][2], x[3][2];   // entry / exit planes per axis, children (0,1) and (2,3)
    int ref[4];
    uint32_t r01, r23;      // the refs as stored: slots 0 | 1 << 16, 2 | 3 << 16
};

// A node of the compact image for a ray whose direction signs are (sx, sy, sz): the entry
// planes of an axis are the slots' max planes when the ray runs toward -axis, else the min
// planes, i.e. the planes the ray enters through; quad(k) reads the node's k-th 16 B.
template <typename QUAD>
__device__ __forceinline__ WideNode wide_node(const QUAD& quad, int sx, int sy, int sz) {
    WideNode n;
    const uint4 ex = quad(sx), xx = quad(1 - sx), ey = quad(2 + sy), xy = quad(3 - sy), ez = quad(4 + sz),
                xz = quad(5 - sz);
    const uint4 r = quad(6);
    auto lo = [](uint4 v) { return f2v{__uint_as_float(v.x), __uint_as_float(v.y)}; };
    auto hi = [](uint4 v) { return f2v{__uint_as_float(v.z), __uint_as_float(v.w)}; };
    n.e[0][0] = lo(ex); n.e[0][1] = hi(ex); n.x[0][0] = lo(xx); n.x[0][1] = hi(xx);
    n.e[1][0] = lo(ey); n.e[1][1] = hi(ey); n.x[1][0] = lo(xy); n.x[1][1] = hi(xy);
    n.e[2][0] = lo(ez); n.e[2][1] = hi(ez); n.x[2][0] = lo(xz); n.x[2][1] = hi(xz);
    n.ref[0] = (int)(int16_t)(r.x & 0xffffu); n.ref[1] = (int)(int16_t)(r.x >> 16);
    n.ref[2] = (int)(int16_t)(r.y & 0xffffu); n.ref[3] = (int)(int16_t)(r.y >> 16);
    n.r01 = r.x;
    n.r23 = r.y;
    return n;
}

// Node `cur` from the LDS image (cur < n_lds: ds_read_b128) or from the image in global memory
// (buffer loads at per-lane offsets).  Both hold the same bits, so the walk's decisions do not
// depend on where a node was read.  HYB = false: the whole tree is in LDS (no per-node check).
template <bool HYB>
__device__ __forceinline__ WideNode load_wide_node(const uint4* tree, int n_lds, __amdgpu_buffer_rsrc_t rsrc,
                                                   uint32_t image_off, int cur, int sx, int sy, int sz) {
    if (!HYB || __builtin_expect(cur < n_lds, 1)) {
        // cur < 2^15: a 24-bit multiply-add (full rate; v_mul_lo_u32 is quarter rate, and the
        // compiler turns __umul24 of a value it cannot bound back into one)
        // (`tree` is the block's LDS copy: its LDS address is 32 bits)
        typedef unsigned int v4u_t __attribute__((ext_vector_type(4)));
        typedef __attribute__((address_space(3))) const v4u_t lds_v4u;
        typedef __attribute__((address_space(3))) const uint4 lds_u4;
        uint32_t a;
        asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(a) : "v"(cur), "s"(112u), "v"((uint32_t)(uintptr_t)(lds_u4*)tree));
        lds_v4u* const q = (lds_v4u*)(uintptr_t)a;
        return wide_node([&](int k) { const v4u_t v = q[k]; return make_uint4(v.x, v.y, v.z, v.w); }, sx, sy, sz);
    }
    const uint32_t off = image_off + (uint32_t)cur * 112u;
    return wide_node(
        [&](int k) {
            const v4u32 v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, off + 16u * (uint32_t)k, 0, 0);
            return make_uint4(v.x, v.y, v.z, v.w);
        },
        sx, sy, sz);
}

// Hit mask of children (a, b) of a pair: slab_reject_octant for each; lo_a / lo_b get their
// sort keys (slab_pass's lo').
__device__ __forceinline__ uint32_t wide_pair(const f2v e[3], const f2v x[3], const RayK& ray, float limit,
                                              float& lo_a, float& lo_b) {
    lo_a = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(e[0].x, ray.inx, ray.nx), __builtin_fmaf(e[1].x, ray.iny, ray.ny)),
                           __builtin_fmaf(e[2].x, ray.inz, ray.nz));
    lo_b = __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaf(e[0].y, ray.inx, ray.nx), __builtin_fmaf(e[1].y, ray.iny, ray.ny)),
                           __builtin_fmaf(e[2].y, ray.inz, ray.nz));
    const float hi_a = __builtin_fminf(__builtin_fminf(__builtin_fmaf(x[0].x, ray.ifx, ray.fx), __builtin_fmaf(x[1].x, ray.ify, ray.fy)),
                                       __builtin_fmaf(x[2].x, ray.ifz, ray.fz));
    const float hi_b = __builtin_fminf(__builtin_fminf(__builtin_fmaf(x[0].y, ray.ifx, ray.fx), __builtin_fmaf(x[1].y, ray.ify, ray.fy)),
                                       __builtin_fmaf(x[2].y, ray.ifz, ray.fz));
    const bool pa = slab_pass(lo_a, hi_a, ray.t3, limit), pb = slab_pass(lo_b, hi_b, ray.t3, limit);
    return (pa ? 1u : 0u) | (pb ? 2u : 0u);
}

// Child refs (the image's int16 words, cpt_capi.cpp linearise_wide): >= 0 a wide node, -1 none,
// <= -2 leaf i of the leaf array as ~(i + 1).  The host keeps the ranges within 15 bits, so the
// LDS stack holds 16-bit entries (BLK lanes x CPT_WSTACK x 2 B per block).
// A lane's wide walk in progress, kept across rounds of the megakernel when the walk is
// suspended (trace_wide's `suspend_at`): the stack itself stays in LDS.
struct WalkState {
    lds_i16* top;
    int cur, parked, best, kind, best_rank;
    float tmax, limit;
    bool active;   // a walk is in progress (suspended in an earlier round)
};

// Suspension (the megakernel): once at most `suspend_at` lanes of the wave still walk and at
// least SUSPEND_MIN_DONE lanes of this call have finished theirs, the call returns 2 for the
// lanes still walking (their state in `ws`) and the finished lanes go on to shade and start
// their next segment; the suspended lanes resume in the next round, beside them.  The walk's
// tail -- iterations with a few working lanes -- then overlaps other lanes' work.  At least
// one iteration runs per call, so every walk progresses.  The result does not depend on
// where a walk is suspended: it is the closest hit over a superset of the primitives the
// reference tests, whatever the culling limit was at each node (DESIGN.md §Ordered walk).

// `tree` is the block's LDS copy of the image's first lds_tree_nodes(n_wide) nodes; HYB: the
// tree is larger (n_wide > LDS_TREE_NODES), so some nodes come from global memory.
template <bool STATS, int BLK, bool HYB>
__device__ __forceinline__ int trace_wide(const KParams& p, __amdgpu_buffer_rsrc_t rsrc, int oct, const RayK& ray,
                                          Hit& h, int& code_out, Counters& cnt, const uint4* tree, WalkState& ws,
                                          int suspend_at) {
    __shared__ int16_t wstack[CPT_WSTACK * BLK];
    // an LDS-typed pointer: 32-bit ds_read/ds_write addressing (a generic pointer costs a
    // 64-bit multiply-add per push and pop)
    lds_i16* const stk = (lds_i16*)wstack + threadIdx.x;
    // Leaves by index into the wide tree's leaf array (platforms first, 32 B each, contiguous in
    // HBM; staging it in LDS as well needs the pending sky fetches' LDS and measured 1.5% slower
    // than keeping those).
    constexpr int leaf0 = 0;
    auto leaf_of = [&](int ref) { return ~ref - 1; };
    const BufSrc leaf_src{rsrc, (uint32_t)wide_leaves_base(p) * (uint32_t)sizeof(Node)};
    auto leaf = [&](int i) -> Node { return leaf_src(i); };
    const int n_lds = lds_tree_nodes(p.n_wide);
    const uint32_t image_off = (uint32_t)wide_image_base(p) * (uint32_t)sizeof(Node);
    constexpr int NONE = -1;
    const uint64_t participants = __ballot(1);
    stamps::lap(6);
#ifdef CPT_POOLDIAG
    pooldiag::resumed(wave_count(__builtin_amdgcn_ballot_w64(ws.active)));
#endif
    if (!ws.active) {
        // a new walk: the platforms (every ray tests them) first, by the whole wave at once,
        // so the walk starts with their tmax; same rank rule, so the order does not matter
        ws.tmax = DEFAULT_RAY_TMAX;
        ws.best = -1;
        ws.kind = 0;
        ws.best_rank = 0x7fffffff;
        for (int k = 0; k < p.n_unb; ++k) {
            if (STATS) cnt.prims++;
            const Node pl = leaf(leaf0 + k);
            int kk;
            if (ranked_leaf_test<true, true, false>(pl, ray, ws.tmax, kk, ws.best_rank)) {
                ws.best = leaf0 + k;
                ws.kind = kk;
            }
        }
        ws.limit = walk_limit(ws.tmax);   // changes only in leaf rounds
        ws.top = stk;
        ws.cur = 0;        // the root
        ws.parked = -1;    // leaf-array index of the parked leaf
    }
    stamps::lap(7);
    // the walk runs on the lane's WalkState itself (one copy of it lives across the round)
    float& tmax = ws.tmax;
    float& limit = ws.limit;
    int& best = ws.best;
    int& kind = ws.kind;
    int& best_rank = ws.best_rank;
    lds_i16*& top = ws.top;   // the next free stack entry (entries are BLK apart)
    int& cur = ws.cur;
    int& parked = ws.parked;
    const int sx = oct & 1, sy = (oct >> 1) & 1, sz = oct >> 2;
    auto pop = [&]() -> int {
        if (top == stk) return NONE;
        top -= BLK;
        return (int)*top;
    };
    // Invariant at the top of every iteration: a lane whose next ref is a leaf has a parked leaf
    // (cur <= -2 implies parked >= 0); the node visit and the leaf round below keep it.
    // The node visits run in an inner loop that leaves for a leaf round (or ends the walk), so
    // the walk's tmax / limit / best are invariant in it: the compiler then keeps them in place
    // instead of copying them around the leaf round's branch in every node iteration.
    int it = 0;
    for (;;) {
        bool leaf_round = false;
        for (;; ++it) {
            stamps::count(9);
            if (cur >= 0) {
                execdiag::lanes(p.stats + 64, 1);
                if (STATS) {
                    cnt.nodes++;
                    cnt.gnodes += HYB && cur >= n_lds ? 1u : 0u;
                }
                const WideNode n = load_wide_node<HYB>(tree, n_lds, rsrc, image_off, cur, sx, sy, sz);
                const f2v e01[3] = {n.e[0][0], n.e[1][0], n.e[2][0]}, x01[3] = {n.x[0][0], n.x[1][0], n.x[2][0]};
                const f2v e23[3] = {n.e[0][1], n.e[1][1], n.e[2][1]}, x23[3] = {n.x[0][1], n.x[1][1], n.x[2][1]};
                float lo[4];
                const uint32_t m = wide_pair(e01, x01, ray, limit, lo[0], lo[1]) |
                                   (wide_pair(e23, x23, ray, limit, lo[2], lo[3]) << 2);
                // The hit child walked next is the one with the nearest entry distance (first
                // slot on ties): the minimum of sort keys made of the distance's bits with the
                // slot in the two low bits (integer order is the float order for the distances
                // >= 0; the few negative ones, of boxes the ray starts in, come first, and ties
                // within 4 ulps go to the first slot -- the order only steers the walk, the hits
                // do not depend on it).  The other hits are pushed (slot 3 first) without
                // branches: every slot is written at the top, and the top moves past it only
                // when it is pushed (the host bounds the depth, so a write at an unmoved top
                // stays inside the lane's stack).
                int key = 0x7fffffff;
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const int kk = (__float_as_int(lo[k]) & ~3) | k;
                    key = ((m >> k) & 1u) && kk < key ? kk : key;
                }
                const int bk = key & 3;
                const uint32_t pm = m & ~(1u << bk);   // the hits pushed
#pragma unroll
                for (int k = 3; k >= 0; --k) {
                    *top = (int16_t)n.ref[k];
                    top += __builtin_amdgcn_ubfe(pm, (uint32_t)k, 1u) * BLK;
                }
                const uint32_t word = (bk & 2) ? n.r23 : n.r01;
                cur = m == 0 ? pop() : (int)(int16_t)(word >> ((bk & 1) << 4));
                if (cur <= -2 && parked < 0) {   // park the nearest leaf at once
                    parked = leaf_of(cur);
                    cur = pop();
                }
            }
            // (one ballot per compare, combined as masks: a ballot of anything but a single
            // compare -- __ballot's int argument, a named bool, an || -- is materialised in a
            // VGPR and compared back into a mask)
            const uint64_t has_parked = __builtin_amdgcn_ballot_w64(parked >= 0);
            const uint64_t w = has_parked | __builtin_amdgcn_ballot_w64(cur != NONE);
            const uint64_t stopped = has_parked & __builtin_amdgcn_ballot_w64(cur < 0);   // at a second leaf or out of nodes
            // wave-uniform counts as 32-bit SGPR values: SALU compares (the compiler otherwise
            // compares the 64-bit popcount with VALU v_cmp_*_u64)
            const uint32_t n_w = wave_count(w);
#ifdef CPT_POOLDIAG
            pooldiag::iteration(wave_count(participants & ~w), n_w);
#endif
            const bool tail = n_w <= 8u;   // stamps only: the walk's tail (few lanes left)
            stamps::lap(tail ? 11 : 1);
            if (tail) stamps::count(13);
            if (!w) break;
            if (n_w <= (uint32_t)suspend_at && wave_count(participants & ~w) >= (uint32_t)SUSPEND_MIN_DONE && it > 0)
                break;
            if (wave_count(stopped) * 64u >= (uint32_t)SPEC_LEAF_ROUND * n_w) {
                leaf_round = true;
                ++it;
                break;
            }
        }
        if (!leaf_round) break;   // the walk ended or is suspended
        if (parked >= 0) {
            stamps::count(10);
            execdiag::lanes(p.stats + 64, 2);
            if (STATS) cnt.prims++;
            const Node lf = leaf(parked);
            int k;
            // no pretest: the parent's slab test already tested this leaf's own box
            if (ranked_leaf_test<true, true, false>(lf, ray, tmax, k, best_rank)) {
                best = parked;
                kind = k;
                limit = walk_limit(tmax);
            }
            parked = -1;
            if (cur <= -2) {   // the lane stopped at a second leaf: park it
                parked = leaf_of(cur);
                cur = pop();
            }
        }
        stamps::lap(2);
    }
    const bool working = parked >= 0 || cur != NONE;
#ifdef CPT_POOLDIAG
    pooldiag::suspended(wave_count(__builtin_amdgcn_ballot_w64(working)));
#endif
    ws.active = working;
    if (working) return 2;   // suspended
    if (best < 0) return 0;
    execdiag::lanes(p.stats + 64, 3);
    const Node wn = leaf(best);
    Node box;
    leaf_aabb(wn, box);
    if (!cert_inside(box, ray, tmax) && slab_reject<true>(box, with_slab(ray), tmax)) return -1;
    h = hit_attributes(wn, ray, tmax, kind);
    code_out = wn.code;
    return 1;
}

// TraceRay for one segment: the reference order, or the ordered walk with its certificate
// and the reference-order fallback (CPT_TRAVERSAL_ORDERED): the 4-wide walk with parked
// leaves (ordered == 1, a wide tree, and a kernel that staged its image in LDS: LDST), else
// the binary octant orders testing each leaf where the walk meets it.
// Returns 1 hit, 0 miss, or 2 when the walk was suspended (only with suspend_at > 0; the
// lane calls again in a later round with the same ray and `ws`).
template <bool STATS, bool FAST, bool CONS = false>
__device__ __forceinline__ int trace_any(__amdgpu_buffer_rsrc_t rsrc, uint32_t base, int n, const RayK& ray, Hit& h,
                                         int& code, Counters& cnt) {
    return trace<STATS, FAST, CONS>(BufSrc{rsrc, base}, n, ray, h, code, cnt);
}

template <bool STATS, int BLK = WIDE_LANES, bool LDST = false, bool HYB = true>
__device__ __forceinline__ int trace_segment(const KParams& p, const RayK& rk, bool finite, Hit& h, int& code,
                                             Counters& cnt, const uint4* tree, WalkState& ws, int suspend_at) {
    const __amdgpu_buffer_rsrc_t rsrc = node_rsrc(p);
    if (p.ordered && __builtin_expect(finite, 1)) {
        int n, r = -1;
        bool wide = false;
        if constexpr (LDST) {
            if (p.ordered == 1 && p.n_wide > 0) {
                const int oct = (rk.d.x < 0.f ? 1 : 0) | (rk.d.y < 0.f ? 2 : 0) | (rk.d.z < 0.f ? 4 : 0);
                r = trace_wide<STATS, BLK, HYB>(p, rsrc, oct, rk, h, code, cnt, tree, ws, suspend_at);
                wide = true;
            }
        }
        if (!wide) {
            const uint32_t base = walk_order(p, rk.d, n) * (uint32_t)sizeof(Node);
            r = trace_any<STATS, true, true>(rsrc, base, n, rk, h, code, cnt);
        }
        if (__builtin_expect(r >= 0, 1)) return r;
        if (STATS) cnt.fallbacks++;
    }
    const RayK rs = with_slab(rk);
    if (__builtin_expect(finite, 1)) return trace_any<STATS, true>(rsrc, 0u, p.n_nodes, rs, h, code, cnt) > 0 ? 1 : 0;
    return trace_any<STATS, false>(rsrc, 0u, p.n_nodes, rs, h, code, cnt) > 0 ? 1 : 0;
}

// The same without suspension (a walk always completes).
template <bool STATS, int BLK = WIDE_LANES, bool LDST = false>
__device__ __forceinline__ bool trace_segment(const KParams& p, const RayK& rk, bool finite, Hit& h, int& code,
                                              Counters& cnt, const uint4* tree = nullptr) {
    WalkState ws;
    ws.active = false;
    return trace_segment<STATS, BLK, LDST>(p, rk, finite, h, code, cnt, tree, ws, 0) == 1;
}

// ======================================================================================
// BSDF sampling (material.cu:20-163).
// ======================================================================================
struct Shade { v3 radiance, attenuation, bounce; };

// to_world (ray_tracing_math.hpp:51-63)
__device__ __forceinline__ v3 to_world(v3 a, v3 N) {
    v3 B, C;
    if (__builtin_fabsf(N.x) > __builtin_fabsf(N.y)) {
        float invLen = rcp_f(sqrt_nn(N.x * N.x + N.z * N.z));
        C = mk(N.z * invLen, 0.0f, -N.x * invLen);
    } else {
        float invLen = rcp_f(sqrt_nn(N.y * N.y + N.z * N.z));
        C = mk(0.f, N.z * invLen, -N.y * invLen);
    }
    B = cross(C, N);
    return (a.x * B + a.y * C) + a.z * N;
}

// z = pow(x1, inv_alpha) (double pow), r = sqrtf(1 - z^2), phi = (float)(2*M_PI*x2); pow, sinf
// and cosf through their short forms (cpt_device.hpp lobe_pow, lobe_sincos: the same floats).
__device__ __forceinline__ v3 lobe(float x_1, float x_2, double inv_alpha) {
    float z = lobe_pow(x_1, inv_alpha);
    float r = sqrt_nn(1.0f - z * z);
    float phi = (float)(2 * REF_PI * (double)x_2);
    float sp, cp;
    lobe_sincos(phi, &sp, &cp);
    return mk(r * cp, r * sp, z);
}

// schlick (ray_tracing_math.hpp:65-69), pow(float,int) -> float overload in device code, as
// dm::pow5f; r0 = ((1 - ref_idx) / (1 + ref_idx))^2 is the material's, prepared once
// (Mat::schlick_r0).
__device__ __forceinline__ float schlick(float cosine, float r0) {
    return r0 + (1 - r0) * dm::pow5f(1 - cosine);
}

// refract (ray_tracing_math.hpp:71-80), discriminant through double (1.0 literal).
__device__ __forceinline__ bool refract(v3 v, v3 n, float ni_over_nt, v3& refracted) {
    v3 uv = normalize_u(v);
    float dt = dot(uv, n);
    float discriminant = (float)(1.0 - (double)(ni_over_nt * ni_over_nt * (1 - dt * dt)));
    if (discriminant > 0) {
        refracted = normalize_u(ni_over_nt * (uv - n * dt) - n * sqrt_nn(discriminant));
        return true;
    }
    return false;
}

// Material::EvalAttenuationAndCreateRay (material.cu:145-163) with the Metal/Mirror swap.
// The four shaders share their expensive tail: every one draws x_1, x_2, builds a lobe
// direction (pow + sincos in double) and rotates it onto an axis with to_world.  Only the
// lobe exponent, the axis and the extra draws differ, so those are selected per lane first
// and lobe()/to_world() run once for the whole wave instead of once per material type
// present in it.  Per lane, the operations and the RNG draw order are exactly the shaders':
//   Diffuse (material.cu:20-38):  x1 x2;      lobe(1/2) about N
//   Metal -> MirrorHitShader (:40-64):  x1 x2;  lobe(1/alpha) about reflect(dir, N)
//   Mirror -> MetalHitShader (:66-99):  x1 x2 u;  u < reflectivity ? lobe(1/alpha) about
//                                       reflect(dir, N) : lobe(1/2) about N
//   Glass (:101-143):  x1 x2; refract/schlick; u;  lobe(1/alpha) about reflect(in, N) or
//                      the refracted direction
__device__ inline void eval_material(const Mat& m, v3 normal, v3 in_dir, Xorwow& rng, Shade& out,
                                     unsigned long long* diag = nullptr) {
    const v3 kd = mk(m.att_x, m.att_y, m.att_z);   // GetKd(0, 0)
    const v3 zero = mk(0.0f, 0.0f, 0.0f);
    const int type = (m.type >= 1 && m.type <= 3) ? m.type : 0;   // Test / unknown: Diffuse (:161)
    const float x_1 = uniform(rng), x_2 = uniform(rng);
    double ia = type == 0 ? 1.0 / 2 : m.inv_alpha;
    v3 axis = normal;
    if (type == 1) {
        axis = reflect(in_dir, normal);
    } else if (type == 2) {
        if (diag) execdiag::lanes(diag, 15);
        if (uniform(rng) < m.reflectivity) axis = reflect(in_dir, normal);
        else ia = 1.0 / 2.0;
    } else if (type == 3) {
        if (diag) execdiag::lanes(diag, 5);
        v3 outward, refracted = mk1(0.0f);
        float ni_over_nt, reflect_prob, cosine;
        const v3 in = normalize_u(in_dir);
        if (dot(in, normal) > 0) {
            outward = -normal;
            ni_over_nt = m.ior;
            cosine = dot(in, normal);
            cosine = sqrt_nn(1 - m.ior * m.ior * (1 - cosine * cosine));
        } else {
            outward = normal;
            ni_over_nt = m.inv_ior;   // 1.f / ior, prepared once
            cosine = -dot(in, normal);
        }
        if (refract(in, outward, ni_over_nt, refracted)) reflect_prob = schlick(cosine, m.schlick_r0);
        else reflect_prob = 1.0f;
        axis = uniform(rng) < reflect_prob ? reflect(in, normal) : refracted;
    }
    const v3 local = lobe(x_1, x_2, ia);
    out.bounce = to_world(local, axis);
    const float c = dot(normal, out.bounce);
    // per component: a struct-valued select here became an indexed scratch load
    const bool keep = type == 3 || (type == 2 ? !(c < 0) : c > 0.0f);
    out.attenuation = mk(keep ? kd.x : zero.x, keep ? kd.y : zero.y, keep ? kd.z : zero.z);
    out.radiance = mk(m.rad_x, m.rad_y, m.rad_z);   // emit_intensity_ * kd_
}

// Miss (path_tracer.cu:117-122)
__device__ __forceinline__ v3 miss_radiance(const KParams& p, v3 dir) {
    v3 d = normalize_u(dir);
    // asinf / atanf through their short forms (cpt_device.hpp miss_asinf, miss_atanf: the same floats)
    float v = (float)(dm::div_pi(miss_asinf(d.z)) + 0.5);     // (double)asinf / REF_PI + 0.5
    float u = (float)dm::div_pi(miss_atanf(d.y / d.x) / 2);    // (double)(atanf / 2) / REF_PI
    return tex2d(p, u, v);
}

// MotionalCamera::RayGen (motional_camera.cu:202-213)
__device__ __forceinline__ Ray ray_gen(const CamK& c, int x, int y, Xorwow& rng) {
    float r1 = uniform(rng), r2 = uniform(rng), r3 = uniform(rng);
    v3 rd = c.lens_radius * mk(r1, r2, r3);
    v3 u = mk(c.u[0], c.u[1], c.u[2]), v = mk(c.v[0], c.v[1], c.v[2]);
    v3 origin = mk(c.origin[0], c.origin[1], c.origin[2]);
    v3 offset = u * rd.x + v * rd.y;
    // float(x) / float(width): for 1 <= x < width <= 2^24 the quotient is a normal float, which
    // qdiv_raw with the double reciprocal gets exactly (cpt_device.hpp); x = 0 gives +0
    float dx = x > 0 ? qdiv_raw(float(x), c.inv_w) : 0.f;
    float dy = y > 0 ? qdiv_raw(float(y), c.inv_h) : 0.f;
    Ray ray;
    ray.o = origin + offset;
    v3 tl = mk(c.top_left[0], c.top_left[1], c.top_left[2]);
    v3 hz = mk(c.horizontal[0], c.horizontal[1], c.horizontal[2]);
    v3 vt = mk(c.vertical[0], c.vertical[1], c.vertical[2]);
    ray.d = normalize((((tl + dx * hz) + dy * vt) - origin) - offset);
    ray.tmin = 0.f;
    ray.tmax = DEFAULT_RAY_TMAX;
    return ray;
}
__device__ __forceinline__ Ray ray_gen(const KParams& p, int x, int y, Xorwow& rng) { return ray_gen(p.cam, x, y, rng); }

// A kernel-argument field read where it is used: a scalar load from the kernarg segment through
// a pointer the compiler cannot hoist (the empty asm redefines it), instead of a value held in
// SGPRs across a persistent kernel's whole loop (whose SGPR spills to VGPR lanes cost v_readlane
// / v_writelane pairs inside the hot loop).  Only for kernels whose single argument is KParams.
__device__ __forceinline__ const KParams& kernarg_params() {
    typedef __attribute__((address_space(4))) const KParams kparams4;
    kparams4* base = (kparams4*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(base));
    return *(const KParams*)base;
}
template <typename T>
__device__ __forceinline__ T kernarg_field(size_t offset) {
    typedef __attribute__((address_space(4))) const char kchar;
    kchar* base = (kchar*)__builtin_amdgcn_kernarg_segment_ptr();
    asm volatile("" : "+s"(base));
    return *(const T*)(base + offset);   // a generic pointer: the AS4 origin is inferred
}

__device__ __forceinline__ uint64_t wave_sum(uint32_t v) {
    uint64_t s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

}  // namespace cpt
