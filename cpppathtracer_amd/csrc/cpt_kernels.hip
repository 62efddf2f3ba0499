// cpt_kernels.hip — HIP kernels of the MI355X integrator (gfx950, wave64).
//
//   k_prepare_materials  per-material constants (alpha, 1/alpha) — material.cu:43,69,103
//   k_rng_*              InitCuRand (path_tracer.cu:36-42) as three GF(2) kernels
//   k_megakernel         SamplePixel (path_tracer.cu:124-175), all spp passes per launch,
//                        per-lane path regeneration, state in registers
//   k_math_batch         device-math KAT surface for the parity tests
//
// Reference semantics per function are cited inline; DESIGN.md has the data layout and the
// roofline of each kernel.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpt_device.hpp"
#include "cpt_internal.hpp"

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
    int period = 2 * n;
    int m = i % period;
    if (m < 0) m += period;
    if (m >= n) m = period - 1 - m;
    return m;
}

__device__ __forceinline__ void texel(const KParams& p, int i, int j, float out[3]) {
    int x = mirror_index(i, p.env_w), y = mirror_index(j, p.env_h);
    if (x >= p.env_cols) { out[0] = out[1] = out[2] = 0.0f; return; }
    uint32_t t = p.env[(size_t)y * p.env_cols + x];
    out[0] = (float)(t & 0xffu) / 255.0f;
    out[1] = (float)((t >> 8) & 0xffu) / 255.0f;
    out[2] = (float)((t >> 16) & 0xffu) / 255.0f;
}

__device__ inline v3 tex2d(const KParams& p, float u, float v) {
    float x = u * (float)p.env_w - 0.5f;
    float y = v * (float)p.env_h - 0.5f;
    if (!(x > -1e7f && x < 1e7f && y > -1e7f && y < 1e7f) || p.env_cols <= 0) return mk1(0.0f);
    float fx = __builtin_floorf(x), fy = __builtin_floorf(y);
    float a = __builtin_floorf((x - fx) * 256.0f + 0.5f) * 0.00390625f;
    float b = __builtin_floorf((y - fy) * 256.0f + 0.5f) * 0.00390625f;
    int i0 = (int)fx, j0 = (int)fy;
    float t00[3], t10[3], t01[3], t11[3];
    texel(p, i0, j0, t00);
    texel(p, i0 + 1, j0, t10);
    texel(p, i0, j0 + 1, t01);
    texel(p, i0 + 1, j0 + 1, t11);
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    float r[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) r[c] = ((w00 * t00[c] + w10 * t10[c]) + w01 * t01[c]) + w11 * t11[c];
    return mk(r[0], r[1], r[2]);
}

// ======================================================================================
// Intersectors (object.cu:10-128).  `tmax` is the traversal's shrinking closest distance.
// ======================================================================================
struct Hit { v3 normal, pos; };

__device__ __forceinline__ bool sphere_test(const Prim& s, const Ray& ray, float& tmax, Hit& h) {
    v3 c = mk(s.cx, s.cy, s.cz);
    v3 A_C = ray.o - c;
    v3 B = ray.d;
    float a = dot(B, B);
    float b = dot(A_C, B);
    float cc = dot(A_C, A_C) - s.radius * s.radius;
    float disc = b * b - a * cc;
    if (disc > 0) {
        float sq = __builtin_sqrtf(disc);
        float temp = (-b - sq) / a;
        if (temp < tmax && temp > ray.tmin) {
            tmax = temp;
            h.pos = ray.o + temp * ray.d;
            h.normal = (h.pos - c) / s.radius;       // first root: divided by the signed radius
            return true;
        }
        temp = (-b + sq) / a;
        if (temp < tmax && temp > ray.tmin) {
            tmax = temp;
            h.pos = ray.o + temp * ray.d;
            h.normal = normalize(h.pos - c);
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ bool platform_test(const Prim& pl, const Ray& ray, float& tmax, Hit& h) {
    if ((ray.o.y < pl.y_pos && ray.d.y > 0.f) || (ray.o.y > pl.y_pos && ray.d.y < 0.f)) {
        float temp = (pl.y_pos - ray.o.y) / ray.d.y;
        if (temp < tmax && temp > ray.tmin) {
            tmax = temp;
            h.pos = ray.o + temp * ray.d;
            h.normal = normalize(mk(0, -ray.d.y, 0));  // faces the ray
            return true;
        }
    }
    return false;
}

__device__ __forceinline__ bool cap_test(const Prim& cy, const Ray& ray, float& tmax, Hit& h, float ypos) {
    if ((ray.o.y < ypos && ray.d.y > 0.f) || (ray.o.y > ypos && ray.d.y < 0.f)) {
        float temp = (ypos - ray.o.y) / ray.d.y;
        v3 hp = ray.o + temp * ray.d;
        if (temp < tmax && temp > ray.tmin &&
            __builtin_sqrtf((hp.x - cy.cx) * (hp.x - cy.cx) + (hp.z - cy.cz) * (hp.z - cy.cz)) < cy.radius) {
            tmax = temp;
            h.pos = hp;
            h.normal = normalize(mk(0, -ray.d.y, 0));
            return true;
        }
    }
    return false;
}

__device__ inline bool cylinder_test(const Prim& cy, const Ray& ray, float& tmax, Hit& h) {
    bool ret = false;
    float upper = cy.cy + cy.height / 2;
    if (cap_test(cy, ray, tmax, h, upper)) ret = true;
    float lower = cy.cy - cy.height / 2;
    if (cap_test(cy, ray, tmax, h, lower)) ret = true;
    float dx = ray.d.x, dz = ray.d.z, r = cy.radius;
    float cx = ray.o.x - cy.cx;
    float cz = ray.o.z - cy.cz;
    float a = dx * dx + dz * dz;
    float b = cx * dx + cz * dz;
    float c = cx * cx + cz * cz - r * r;
    float disc = b * b - a * c;
    if (disc > 0.f) {
        float sq = __builtin_sqrtf(disc);
        float temp = (-b - sq) / a;
        v3 hp = ray.o + temp * ray.d;
        if (temp < tmax && temp > ray.tmin && hp.y > lower && hp.y < upper) {
            tmax = temp;
            h.pos = hp;
            h.normal = normalize(mk(hp.x - cy.cx, 0.f, hp.z - cy.cz));
            ret = true;
        }
        temp = (-b + sq) / a;
        hp = ray.o + temp * ray.d;
        if (temp < tmax && temp > ray.tmin && hp.y > lower && hp.y < upper) {
            tmax = temp;
            h.pos = hp;
            h.normal = normalize(mk(hp.x - cy.cx, 0.f, hp.z - cy.cz));
            ret = true;
        }
    }
    return ret;
}

// ======================================================================================
// SceneBVH::TraceRay (bvh.cu:167-205) as a stackless skip-link walk.  The nodes are stored
// in the exact order the reference's stack DFS pops them (right child first), so visiting
// n, then n+1 on a box hit or node.miss on a box miss / after a leaf, reproduces the
// reference's visit sequence, leaf-before-box order and pruning against the shrinking tmax
// one for one — no stack, no scratch memory.
// ======================================================================================
struct Counters { uint32_t segments, nodes, prims, hits, misses; };

template <bool STATS>
__device__ inline bool trace(const KParams& p, const Ray& ray, Hit& h, int& prim_out, Counters& cnt) {
    float tmax = ray.tmax;
    bool hit = false;
    int ni = 0;
    const int n_nodes = p.n_nodes;
    while (ni < n_nodes) {
        const Node nd = p.nodes[ni];
        if (STATS) cnt.nodes++;
        if (nd.prim >= 0) {
            if (STATS) cnt.prims++;
            const Prim pr = p.prims[nd.prim];
            bool r;
            if (pr.type == 0) r = sphere_test(pr, ray, tmax, h);
            else if (pr.type == 1) r = platform_test(pr, ray, tmax, h);
            else if (pr.type == 2) r = cylinder_test(pr, ray, tmax, h);
            else r = false;
            if (r) { hit = true; prim_out = nd.prim; }
            ni = nd.miss;   // the leaf's own slab test only decides whether to push (-1,-1)
        } else {
            float lo = -DEFAULT_RAY_TMAX * 2, hi = DEFAULT_RAY_TMAX * 2;
            if (ray.d.x != 0.f) {
                float t0 = (nd.bmin_x - ray.o.x) / ray.d.x;
                float t1 = (nd.bmax_x - ray.o.x) / ray.d.x;
                lo = tmax_(lo, tmin_(t0, t1));
                hi = tmin_(hi, tmax_(t0, t1));
            }
            if (ray.d.y != 0.f) {
                float t0 = (nd.bmin_y - ray.o.y) / ray.d.y;
                float t1 = (nd.bmax_y - ray.o.y) / ray.d.y;
                lo = tmax_(lo, tmin_(t0, t1));
                hi = tmin_(hi, tmax_(t0, t1));
            }
            if (ray.d.z != 0.f) {
                float t0 = (nd.bmin_z - ray.o.z) / ray.d.z;
                float t1 = (nd.bmax_z - ray.o.z) / ray.d.z;
                lo = tmax_(lo, tmin_(t0, t1));
                hi = tmin_(hi, tmax_(t0, t1));
            }
            bool reject = lo > hi || lo > tmax || hi < ray.tmin;
            ni = reject ? nd.miss : ni + 1;
        }
    }
    return hit;
}

// ======================================================================================
// BSDF sampling (material.cu:20-163).
// ======================================================================================
struct Shade { v3 radiance, attenuation, bounce; };

// to_world (ray_tracing_math.hpp:51-63)
__device__ __forceinline__ v3 to_world(v3 a, v3 N) {
    v3 B, C;
    if (__builtin_fabsf(N.x) > __builtin_fabsf(N.y)) {
        float invLen = 1.0f / __builtin_sqrtf(N.x * N.x + N.z * N.z);
        C = mk(N.z * invLen, 0.0f, -N.x * invLen);
    } else {
        float invLen = 1.0f / __builtin_sqrtf(N.y * N.y + N.z * N.z);
        C = mk(0.f, N.z * invLen, -N.y * invLen);
    }
    B = cross(C, N);
    return (a.x * B + a.y * C) + a.z * N;
}

// z = pow(x1, inv_alpha) (double pow), r = sqrtf(1 - z^2), phi = (float)(2*M_PI*x2).
__device__ __forceinline__ v3 lobe(float x_1, float x_2, double inv_alpha) {
    float z = (float)dm::pow((double)x_1, inv_alpha);
    float r = __builtin_sqrtf(1.0f - z * z);
    float phi = (float)(2 * REF_PI * (double)x_2);
    float sp, cp;
    dm::sincosf_(phi, &sp, &cp);
    return mk(r * cp, r * sp, z);
}

// schlick (ray_tracing_math.hpp:65-69), pow(float,int) -> float overload in device code.
__device__ __forceinline__ float schlick(float cosine, float ref_idx) {
    float r0 = (1 - ref_idx) / (1 + ref_idx);
    r0 *= r0;
    return r0 + (1 - r0) * dm::powf_(1 - cosine, 5.0f);
}

// refract (ray_tracing_math.hpp:71-80), discriminant through double (1.0 literal).
__device__ __forceinline__ bool refract(v3 v, v3 n, float ni_over_nt, v3& refracted) {
    v3 uv = normalize(v);
    float dt = dot(uv, n);
    float discriminant = (float)(1.0 - (double)(ni_over_nt * ni_over_nt * (1 - dt * dt)));
    if (discriminant > 0) {
        refracted = normalize(ni_over_nt * (uv - n * dt) - n * __builtin_sqrtf(discriminant));
        return true;
    }
    return false;
}

// Material::EvalAttenuationAndCreateRay (material.cu:145-163) with the Metal/Mirror swap.
__device__ inline void eval_material(const Mat& m, v3 normal, v3 in_dir, Xorwow& rng, Shade& out) {
    const v3 kd = mk(m.kd_x, m.kd_y, m.kd_z);
    const v3 zero = mk(0.0f, 0.0f, 0.0f);
    if (m.type == 1) {
        // MaterialType::Metal -> MirrorHitShader (material.cu:40-64)
        float x_1 = uniform(rng), x_2 = uniform(rng);
        v3 local = lobe(x_1, x_2, m.inv_alpha);
        v3 wo = to_world(local, reflect(in_dir, normal));
        out.attenuation = dot(normal, wo) > 0.0f ? kd : zero;
        out.bounce = wo;
    } else if (m.type == 2) {
        // MaterialType::Mirror -> MetalHitShader (material.cu:66-99)
        float x_1 = uniform(rng), x_2 = uniform(rng);
        if (uniform(rng) < m.reflectivity) {
            v3 local = lobe(x_1, x_2, m.inv_alpha);
            out.bounce = to_world(local, reflect(in_dir, normal));
        } else {
            v3 local = lobe(x_1, x_2, 1.0 / 2.0);
            out.bounce = to_world(local, normal);
        }
        out.attenuation = dot(out.bounce, normal) < 0 ? zero : kd;
    } else if (m.type == 3) {
        // GlassHitShader (material.cu:101-143)
        float x_1 = uniform(rng), x_2 = uniform(rng);
        v3 local = lobe(x_1, x_2, m.inv_alpha);
        v3 outward, refracted = mk1(0.0f);
        float ni_over_nt, reflect_prob, cosine;
        v3 in = normalize(in_dir);
        if (dot(in, normal) > 0) {
            outward = -normal;
            ni_over_nt = m.ior;
            cosine = dot(in, normal);
            cosine = __builtin_sqrtf(1 - m.ior * m.ior * (1 - cosine * cosine));
        } else {
            outward = normal;
            ni_over_nt = 1.f / m.ior;
            cosine = -dot(in, normal);
        }
        if (refract(in, outward, ni_over_nt, refracted)) reflect_prob = schlick(cosine, m.ior);
        else reflect_prob = 1.0f;
        if (uniform(rng) < reflect_prob) out.bounce = to_world(local, reflect(in, normal));
        else out.bounce = to_world(local, refracted);
        out.attenuation = kd;
    } else {
        // Diffuse (and Test / unknown: default branch) -> DiffuseHitShader (material.cu:20-38)
        float x_1 = uniform(rng), x_2 = uniform(rng);
        v3 local = lobe(x_1, x_2, 1.0 / 2);
        out.bounce = to_world(local, normal);
        out.attenuation = dot(normal, out.bounce) > 0.0f ? kd : zero;
    }
    out.radiance = m.emit * kd;
}

// Miss (path_tracer.cu:117-122)
__device__ __forceinline__ v3 miss_radiance(const KParams& p, v3 dir) {
    v3 d = normalize(dir);
    float v = (float)((double)dm::asinf_(d.z) / REF_PI + 0.5);
    float u = (float)((double)(dm::atanf_(d.y / d.x) / 2) / REF_PI);
    return tex2d(p, u, v);
}

// MotionalCamera::RayGen (motional_camera.cu:202-213)
__device__ __forceinline__ Ray ray_gen(const KParams& p, int x, int y, Xorwow& rng) {
    const CamK& c = p.cam;
    float r1 = uniform(rng), r2 = uniform(rng), r3 = uniform(rng);
    v3 rd = c.lens_radius * mk(r1, r2, r3);
    v3 u = mk(c.u[0], c.u[1], c.u[2]), v = mk(c.v[0], c.v[1], c.v[2]);
    v3 origin = mk(c.origin[0], c.origin[1], c.origin[2]);
    v3 offset = u * rd.x + v * rd.y;
    float dx = float(x) / float(c.width);
    float dy = float(y) / float(c.height);
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

__device__ __forceinline__ uint64_t wave_sum(uint32_t v) {
    uint64_t s = v;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    return s;
}

// ======================================================================================
// k_megakernel — SamplePixel (path_tracer.cu:124-175) for `spp` consecutive passes.
//
// One lane owns one pixel for the whole launch: the XORWOW state, the path state and the
// pass accumulator stay in VGPRs; HBM is touched once per pixel on entry (24 B rng + 16 B
// accumulator) and once on exit.  When a lane's path ends it immediately starts the
// pixel's next pass (per-lane path regeneration), so a wave stays full until its lanes run
// out of passes — the pixel's passes are sequential anyway (the RNG stream persists across
// passes, a16).  Waves cover 8x8 pixel tiles so first-bounce rays of a wave are coherent.
// ======================================================================================
template <bool STATS, bool AUX>
__global__ void __launch_bounds__(256) k_megakernel(const KParams p) {
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int tiles_x = (p.width + 7) >> 3;
    const int tx = wave % tiles_x, ty = wave / tiles_x;
    const int x = tx * 8 + (lane & 7);
    const int ri = ty * 8 + (lane >> 3);
    Counters cnt{0, 0, 0, 0, 0};
    const bool active = x < p.width && ri < p.n_rows;
    if (active) {
        const int y = p.rows[ri];
        const size_t npix = (size_t)p.n_rows * p.width;
        const size_t pix = (size_t)ri * p.width + x;
        Xorwow s;
        s.v0 = p.rng[pix];
        s.v1 = p.rng[npix + pix];
        s.v2 = p.rng[2 * npix + pix];
        s.v3 = p.rng[3 * npix + pix];
        s.v4 = p.rng[4 * npix + pix];
        s.d = p.rng[5 * npix + pix];
        float4 acc = p.accumulate ? p.accum[pix] : make_float4(0.f, 0.f, 0.f, 0.f);
        v3 sum = mk(acc.x, acc.y, acc.z);
        float passes = acc.w;
        v3 first_normal = mk1(0.f);
        float first_depth = 0.f;
        const uint32_t max_depth = (uint32_t)p.max_depth;
        int left = p.spp;
        if (left > 0 && max_depth == 0) {
            // while (0 < 0) never runs: each pass is RayGen's three draws and zero radiance.
            for (; left > 0; --left) {
                (void)ray_gen(p, x, y, s);
                sum = sum + mk1(0.f);
                passes += 1.0f;
            }
            first_normal = mk1(0.f);
            first_depth = 0.f;
        }
        if (left > 0) {
            Ray ray = ray_gen(p, x, y, s);
            v3 att = mk1(1.f), rad = mk1(0.f);
            uint32_t depth = 0;
            bool first = true;
            v3 nrm_acc = mk1(0.f);
            float dep_acc = 0.f;
            for (;;) {
                Hit h;
                int prim = -1;
                if (STATS) cnt.segments++;
                bool hit = trace<STATS>(p, ray, h, prim, cnt);
                Shade sh;
                v3 attr_normal;
                if (hit) {
                    if (STATS) cnt.hits++;
                    const Mat m = p.mats[p.prims[prim].material];
                    eval_material(m, h.normal, ray.d, s, sh);
                    attr_normal = h.normal;
                    ray.o = h.pos;                         // payload.hit_pos = position
                } else {
                    if (STATS) cnt.misses++;
                    sh.radiance = miss_radiance(p, ray.d);
                    sh.attenuation = mk1(0.f);             // never read: the path ends here
                    sh.bounce = ray.d;
                    attr_normal = -ray.d;
                    depth = MAX_RECURSION_DEPTH_SET;       // termination sentinel (path_tracer.cu:121)
                }
                rad = rad + att * sh.radiance;
                att = att * sh.attenuation;
                if (AUX && first) {
                    nrm_acc = nrm_acc + attr_normal;
                    dep_acc += DEFAULT_RAY_TMAX;           // TraceRay took the ray by value (a18)
                }
                first = false;
                ray.d = normalize(sh.bounce);
                ray.tmin = BOUNCE_RAY_TMIN;
                ray.tmax = DEFAULT_RAY_TMAX;
                depth++;
                if (!(depth < max_depth)) {
                    sum = sum + rad;
                    passes += 1.0f;
                    if (AUX) { first_normal = nrm_acc; first_depth = dep_acc; }
                    if (--left == 0) break;
                    ray = ray_gen(p, x, y, s);
                    att = mk1(1.f);
                    rad = mk1(0.f);
                    depth = 0;
                    first = true;
                    nrm_acc = mk1(0.f);
                    dep_acc = 0.f;
                }
            }
        }
        p.accum[pix] = make_float4(sum.x, sum.y, sum.z, passes);
        if (AUX && p.spp > 0) {
            p.normal[3 * pix + 0] = first_normal.x;
            p.normal[3 * pix + 1] = first_normal.y;
            p.normal[3 * pix + 2] = first_normal.z;
            p.depth[pix] = first_depth;
        }
        p.rng[pix] = s.v0;
        p.rng[npix + pix] = s.v1;
        p.rng[2 * npix + pix] = s.v2;
        p.rng[3 * npix + pix] = s.v3;
        p.rng[4 * npix + pix] = s.v4;
        p.rng[5 * npix + pix] = s.d;
    }
    if (STATS) {
        uint64_t a = wave_sum(cnt.segments), b = wave_sum(cnt.nodes), c = wave_sum(cnt.prims);
        uint64_t d = wave_sum(cnt.hits), e = wave_sum(cnt.misses);
        if (lane == 0) {
            atomicAdd((unsigned long long*)&p.stats[0], (unsigned long long)a);
            atomicAdd((unsigned long long*)&p.stats[1], (unsigned long long)b);
            atomicAdd((unsigned long long*)&p.stats[2], (unsigned long long)c);
            atomicAdd((unsigned long long*)&p.stats[3], (unsigned long long)d);
            atomicAdd((unsigned long long*)&p.stats[4], (unsigned long long)e);
        }
    }
}

// ======================================================================================
// Per-material constants: alpha = pow(1000.0f, s) (float pow), 1.0 / alpha in double
// (material.cu:43-45, 69-70, 103-104).
// ======================================================================================
__global__ void k_prepare_materials(Mat* mats, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float alpha = dm::powf_(1000.0f, mats[i].smoothness);
    mats[i].inv_alpha = 1.0 / (double)alpha;
}

// ======================================================================================
// InitCuRand (path_tracer.cu:36-42): curand_init(seed, (x<<32)|y, 0) per pixel, i.e.
// v = A^(2^67 * ((x<<32)|y)) v_seed.  Factored as v = M_y (N_x v_seed) with
// M_y = A^(2^67 y), N_x = A^(2^99 x) — GF(2) linear, exact.  jumps[t] = A^(2^67 * 2^t)
// (160x160 bits, column-major: column c = 5 words at [t][c*5..c*5+4]).
// All loops over matrix columns are wave-uniform, so the column loads are uniform too.
// ======================================================================================
__device__ __forceinline__ void matvec_uniform(const uint32_t* __restrict__ M, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0;
    for (int c = 0; c < 160; ++c) {
        uint32_t mask = 0u - ((in[c >> 5] >> (c & 31)) & 1u);
        const uint32_t* col = M + c * 5;
        r0 ^= mask & col[0];
        r1 ^= mask & col[1];
        r2 ^= mask & col[2];
        r3 ^= mask & col[3];
        r4 ^= mask & col[4];
    }
    out[0] = r0; out[1] = r1; out[2] = r2; out[3] = r3; out[4] = r4;
}

// w[x] = N_x v_seed for every column x of the frame (one thread per x).
__global__ void k_rng_columns(const uint32_t* __restrict__ jumps, uint32_t seed_v0, uint32_t seed_v1, uint32_t seed_v2,
                              uint32_t seed_v3, uint32_t seed_v4, int width, uint32_t* __restrict__ w) {
    int x = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t v[5] = {seed_v0, seed_v1, seed_v2, seed_v3, seed_v4};
    for (int t = 0; t < 31; ++t) {              // bits 32..62 of the subsequence
        uint32_t out[5];
        matvec_uniform(jumps + (size_t)(32 + t) * 800, v, out);
        bool take = x < width && ((x >> t) & 1);
        if (take) { v[0] = out[0]; v[1] = out[1]; v[2] = out[2]; v[3] = out[3]; v[4] = out[4]; }
        if (!__any(x < width && (x >> (t + 1)) != 0)) break;
    }
    if (x < width) for (int k = 0; k < 5; ++k) w[(size_t)k * width + x] = v[k];
}

// M_y for every distinct row: block = one row, 160 threads = the 160 columns.
__global__ void k_rng_rowmats(const uint32_t* __restrict__ jumps, const int32_t* __restrict__ rows,
                              uint32_t* __restrict__ mats) {
    const int ri = blockIdx.x;
    const int c = threadIdx.x;
    const uint32_t y = (uint32_t)rows[ri];
    uint32_t v[5] = {0, 0, 0, 0, 0};
    if (c < 160) v[c >> 5] = 1u << (c & 31);
    for (int t = 0; t < 32 && (y >> t) != 0; ++t) {
        if ((y >> t) & 1u) {
            uint32_t out[5];
            matvec_uniform(jumps + (size_t)t * 800, v, out);
            for (int k = 0; k < 5; ++k) v[k] = out[k];
        }
    }
    if (c < 160)
        for (int k = 0; k < 5; ++k) mats[(size_t)ri * 800 + c * 5 + k] = v[k];
}

// v_pixel = M_y w_x; d = the seed's d (2^67 k Weyl steps are 0 mod 2^32).  Grid: (x blocks, rows).
__global__ void k_rng_pixels(const uint32_t* __restrict__ rowmats, const uint32_t* __restrict__ w, int width,
                             int n_rows, uint32_t seed_d, uint32_t* __restrict__ rng) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int ri = blockIdx.y;
    const uint32_t* M = rowmats + (size_t)ri * 800;
    uint32_t in[5];
    const int xx = x < width ? x : width - 1;
    for (int k = 0; k < 5; ++k) in[k] = w[(size_t)k * width + xx];
    uint32_t out[5];
    matvec_uniform(M, in, out);
    if (x < width) {
        const size_t npix = (size_t)n_rows * width;
        const size_t pix = (size_t)ri * width + x;
        for (int k = 0; k < 5; ++k) rng[k * npix + pix] = out[k];
        rng[5 * npix + pix] = seed_d;
    }
}

// ======================================================================================
// Device-math KAT (see cpt.h cpt_math_batch).
// ======================================================================================
__global__ void k_math_batch(int op, const float* a, const float* b, float* out, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float x = a[i], y = b[i], r;
    switch (op) {
        case 0: r = dm::powf_(x, y); break;
        case 1: { float s, c; dm::sincosf_(x, &s, &c); r = s; break; }
        case 2: { float s, c; dm::sincosf_(x, &s, &c); r = c; break; }
        case 3: r = dm::asinf_(x); break;
        case 4: r = dm::atanf_(x); break;
        case 5: r = (float)dm::pow((double)x, 1.0 / (double)y); break;
        case 6: r = (float)((double)x / (double)y); break;
        case 7: r = x / y; break;
        case 8: r = __builtin_sqrtf(x); break;
        default: r = __builtin_nanf("");
    }
    out[i] = r;
}

// ======================================================================================
// Host-side launchers (called from cpt_capi.cpp).
// ======================================================================================
hipError_t launch_megakernel(const KParams& p, bool stats, bool aux, hipStream_t stream) {
    const int tiles = ((p.width + 7) / 8) * ((p.n_rows + 7) / 8);
    const int blocks = (tiles + 3) / 4;
    if (blocks == 0) return hipSuccess;
    if (stats && aux) hipLaunchKernelGGL((k_megakernel<true, true>), dim3(blocks), dim3(256), 0, stream, p);
    else if (stats) hipLaunchKernelGGL((k_megakernel<true, false>), dim3(blocks), dim3(256), 0, stream, p);
    else if (aux) hipLaunchKernelGGL((k_megakernel<false, true>), dim3(blocks), dim3(256), 0, stream, p);
    else hipLaunchKernelGGL((k_megakernel<false, false>), dim3(blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

hipError_t launch_prepare_materials(Mat* mats, int n, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_prepare_materials, dim3((n + 63) / 64), dim3(64), 0, stream, mats, n);
    return hipGetLastError();
}

hipError_t launch_init_rng(const uint32_t* jumps, const uint32_t seed_state[6], int width, const int32_t* rows, int n_rows,
                           uint32_t* scratch_w, uint32_t* scratch_mats, uint32_t* rng, hipStream_t stream) {
    if (width <= 0 || n_rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_rng_columns, dim3((width + 63) / 64), dim3(64), 0, stream, jumps, seed_state[0], seed_state[1],
                       seed_state[2], seed_state[3], seed_state[4], width, scratch_w);
    hipLaunchKernelGGL(k_rng_rowmats, dim3(n_rows), dim3(192), 0, stream, jumps, rows, scratch_mats);
    hipLaunchKernelGGL(k_rng_pixels, dim3((width + 255) / 256, n_rows), dim3(256), 0, stream, scratch_mats, scratch_w,
                       width, n_rows, seed_state[5], rng);
    return hipGetLastError();
}

hipError_t launch_math_batch(int op, const float* a, const float* b, float* out, size_t n, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_math_batch, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, op, a, b, out, n);
    return hipGetLastError();
}

}  // namespace cpt
