// cpt_capi.cpp — implementation of the C-ABI in include/cpt.h: contexts, frames, the RNG init,
// render launches, the row-tile gather, counters and the display path.  The scene half
// (upload, material slots, walk trees, device refit) is cpt_scene.cpp; the host BVH builds and
// the XORWOW tables are cpt_host_bvh.cpp / cpt_host_rng.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "cpt_context.hpp"

// CPT_SCHEDULE_PREVIOUS: renders between rebuilds of the heaviest-first tile order.  Round 5,
// C4 DispatchRay loop, three interleaved rounds (profiles/r05/ab_dispatch_order_every.log): every
// render 1.71-1.72 ms per pass, every 4th 1.66-1.68, every 8th 1.65-1.66; the 1-spp render itself
// is unchanged (1.42-1.43), so the staler order costs nothing measurable.
constexpr int PREV_ORDER_EVERY = 8;

static_assert(sizeof(cpt_material) == 40, "cpt_material must match Material (40 B)");
static_assert(sizeof(cpt_object) == 72, "cpt_object must match Object (72 B)");
static_assert(sizeof(cpt_camera) == 136, "cpt_camera must match MotionalCamera (136 B)");
static_assert(offsetof(cpt_object, center) == 48, "Object::center_ offset");
static_assert(offsetof(cpt_material, refractive_index) == 24, "Material::refractive_index_ offset");

using namespace cpt::host;
using namespace cpt::ctx;

namespace {
std::string g_create_error;
}  // namespace

namespace cpt {
namespace ctx {

int fail(cpt_ctx* c, int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    if (c) c->err = buf;
    else g_create_error = buf;
    return code;
}

void free_frame(cpt_ctx* c) {
    (void)hipFree(c->d_rows); c->d_rows = nullptr;
    (void)hipFree(c->d_rng); c->d_rng = nullptr;
    (void)hipFree(c->d_accum); c->d_accum = nullptr;
    (void)hipFree(c->d_normal); c->d_normal = nullptr;
    (void)hipFree(c->d_depth); c->d_depth = nullptr;
    (void)hipFree(c->d_mix); c->d_mix = nullptr;
    for (float4** a : {&c->wf.ray_o[0], &c->wf.ray_d[0], &c->wf.att[0], &c->wf.rad[0], &c->wf.aux[0], &c->wf.ray_o[1],
                       &c->wf.ray_d[1], &c->wf.att[1], &c->wf.rad[1], &c->wf.aux[1], &c->wf.hit_p, &c->wf.hit_n}) {
        (void)hipFree(*a);
        *a = nullptr;
    }
    for (int b = 0; b < 2; ++b) {
        (void)hipFree(c->wf.rng_a[b]); c->wf.rng_a[b] = nullptr;
        (void)hipFree(c->wf.rng_b[b]); c->wf.rng_b[b] = nullptr;
    }
    (void)hipFree(c->wf.queue[0]); c->wf.queue[0] = nullptr;
    (void)hipFree(c->wf.queue[1]); c->wf.queue[1] = nullptr;
    (void)hipFree(c->wf.ident); c->wf.ident = nullptr;
    (void)hipFree(c->wf.counts); c->wf.counts = nullptr;
    c->wf_ready = false;
    (void)hipFree(c->d_bgra); c->d_bgra = nullptr;
    (void)hipFree(c->d_dn_sink); c->d_dn_sink = nullptr;
    c->band_y0 = c->band_y1 = -1;
    (void)hipFree(c->d_scratch_w); c->d_scratch_w = nullptr;
    (void)hipFree(c->d_scratch_m); c->d_scratch_m = nullptr;
    (void)hipFree(c->d_sched); c->d_sched = nullptr; c->cap_sched = 0;
    (void)hipFree(c->d_tile_order); c->d_tile_order = nullptr; c->cap_tile_order = 0;
    (void)hipFree(c->d_prev_d); c->d_prev_d = nullptr;
    (void)hipFree(c->d_prev_order); c->d_prev_order = nullptr;
    c->prev_d_valid = c->prev_order_valid = false;
    c->frame_set = c->rng_set = false;
}

// The kernels' sticky error word (KParams::error, CPT_DEVERR_*): read after the context's
// stream has drained; a set word is cleared and reported once, like a sticky HIP error.
// Both the read and the clear run on the context's own stream (a blocking hipMemcpy would
// synchronise with the legacy default stream and so with other streams' work, e.g. collectives).
int check_device_error(cpt_ctx* c) {
    uint32_t v = 0;
    hipStream_t s = c->stream();
    HIP_TRY(c, hipMemcpyAsync(&v, c->d_work + 4, sizeof(v), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    if (v == 0) return CPT_OK;
    HIP_TRY(c, hipMemsetAsync(c->d_work + 4, 0, sizeof(v), s));
    return fail(c, CPT_ERR_DEVICE, "device error 0x%x:%s%s%s", v,
                (v & cpt::CPT_DEVERR_KEEPER_TIMEOUT) ? " a keeper wave gave up with chains still live (pixels left unfinished);" : "",
                (v & cpt::CPT_DEVERR_PUBLISH_TIMEOUT) ? " a handed-over chain was never published (its pixel was not written);" : "",
                (v & cpt::CPT_DEVERR_RESUME_CAP) ? " the consolidation slab is too small for the grid;" : "");
}

// Drain the context's stream, then report a device-side error of the work it ran.
int sync_checked(cpt_ctx* c) {
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    return check_device_error(c);
}

}  // namespace ctx
}  // namespace cpt

extern "C" {

int cpt_abi_version(void) { return CPT_ABI_VERSION; }

const char* cpt_status_string(int status) {
    switch (status) {
        case CPT_OK: return "ok";
        case CPT_ERR_INVALID_ARG: return "invalid argument";
        case CPT_ERR_NO_DEVICE: return "no HIP device";
        case CPT_ERR_HIP: return "HIP runtime error";
        case CPT_ERR_OUT_OF_MEMORY: return "out of device memory";
        case CPT_ERR_STATE: return "invalid state";
        case CPT_ERR_UNSUPPORTED: return "unsupported";
        case CPT_ERR_DEVICE: return "device-side error";
        default: return "unknown status";
    }
}

int cpt_get_device_count(int* count) {
    if (!count) return CPT_ERR_INVALID_ARG;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = (e == hipSuccess) ? n : 0;
    return CPT_OK;
}

int cpt_create(int device, cpt_ctx** out) {
    if (!out) return fail(nullptr, CPT_ERR_INVALID_ARG, "cpt_create: out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
        return fail(nullptr, CPT_ERR_NO_DEVICE, "cpt_create: no HIP device visible");
    if (device < 0 || device >= n) return fail(nullptr, CPT_ERR_INVALID_ARG, "cpt_create: device %d of %d", device, n);
    cpt_ctx* c = new (std::nothrow) cpt_ctx;
    if (!c) return fail(nullptr, CPT_ERR_OUT_OF_MEMORY, "cpt_create: host allocation failed");
    c->device = device;
    hipError_t e = hipSetDevice(device);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_start);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_stop);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_main);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_dn0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev_dn1);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_ready, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_gathered, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_caller, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_copied, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_stats, 128 * sizeof(unsigned long long));   // [64..128) execdiag
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_work, 64);   // [0] dequeue counter, [4] error word
    if (e == hipSuccess) e = hipMemset(c->d_work, 0, 64);
    if (e == hipSuccess) e = hipMemset(c->d_stats, 0, 128 * sizeof(unsigned long long));
    if (e == hipSuccess) {
        const std::vector<uint32_t>& J = jump_tables();
        e = hipMalloc((void**)&c->d_jumps, J.size() * sizeof(uint32_t));
        if (e == hipSuccess) e = hipMemcpy(c->d_jumps, J.data(), J.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    }
    if (e != hipSuccess) {
        int rc = fail(nullptr, CPT_ERR_HIP, "cpt_create: %s", hipGetErrorString(e));
        cpt_destroy(c);
        return rc;
    }
    *out = c;
    return CPT_OK;
}

int cpt_destroy(cpt_ctx* c) {
    if (!c) return CPT_OK;
    (void)hipSetDevice(c->device);
    if (c->own_stream) (void)hipStreamSynchronize(c->own_stream);
    if (c->user_stream) (void)hipStreamSynchronize(c->user_stream);
    free_frame(c);
    (void)hipFree(c->d_nodes);
    (void)hipFree(c->d_mats);
    (void)hipFree(c->d_refit_plan);
    (void)hipFree(c->d_refit_boxes);
    (void)hipFree(c->d_refit_work);
    (void)hipFree(c->d_env);
    for (auto& t : c->textures) (void)hipFree(t.d_texels);
    (void)hipFree(c->d_texdescs);
    (void)hipFree(c->d_tex_of_mat);
    (void)hipFree(c->d_jumps);
    (void)hipFree(c->d_stats);
    (void)hipFree(c->d_work);
    (void)hipFree(c->d_resume);
    (void)hipFree(c->d_gather);
    for (auto& g : c->gather_maps) (void)hipFree(g.d_map);
    if (c->ev_dn0) (void)hipEventDestroy(c->ev_dn0);
    if (c->ev_dn1) (void)hipEventDestroy(c->ev_dn1);
    if (c->ev_ready) (void)hipEventDestroy(c->ev_ready);
    if (c->ev_gathered) (void)hipEventDestroy(c->ev_gathered);
    if (c->ev_caller) (void)hipEventDestroy(c->ev_caller);
    if (c->ev_copied) (void)hipEventDestroy(c->ev_copied);
    if (c->ev_start) (void)hipEventDestroy(c->ev_start);
    if (c->ev_stop) (void)hipEventDestroy(c->ev_stop);
    if (c->ev_main) (void)hipEventDestroy(c->ev_main);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    delete c;
    return CPT_OK;
}

const char* cpt_last_error(const cpt_ctx* c) { return c ? c->err.c_str() : g_create_error.c_str(); }

int cpt_set_stream(cpt_ctx* c, void* s) {
    if (!c) return CPT_ERR_INVALID_ARG;
    c->user_stream = (hipStream_t)s;
    return CPT_OK;
}

// MotionalCamera::GetCopy (motional_camera.cu:177-200)
int cpt_camera_get_copy(cpt_camera* cam) {
    if (!cam || cam->width <= 0 || cam->height <= 0) return CPT_ERR_INVALID_ARG;
    auto sub = [](cpt_float3 a, cpt_float3 b) { return cpt_float3{a.x - b.x, a.y - b.y, a.z - b.z}; };
    auto add = [](cpt_float3 a, cpt_float3 b) { return cpt_float3{a.x + b.x, a.y + b.y, a.z + b.z}; };
    auto scale = [](float s, cpt_float3 a) { return cpt_float3{s * a.x, s * a.y, s * a.z}; };
    auto dot = [](cpt_float3 a, cpt_float3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
    auto normalize = [&](cpt_float3 v) {
        float inv = 1.0f / sqrtf(dot(v, v));
        return cpt_float3{v.x * inv, v.y * inv, v.z * inv};
    };
    auto cross = [](cpt_float3 a, cpt_float3 b) {
        return cpt_float3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    };
    float theta = (float)((double)cam->view_fov * 3.14159265358979323846 / 180);
    float aspect = float(cam->width) / float(cam->height);
    float half_height = tanf(theta / 2);
    float half_width = aspect * half_height;
    cam->w = normalize(sub(cam->origin, cam->look_at));
    cam->u = normalize(cross(cam->vup, cam->w));
    cam->v = cross(cam->w, cam->u);
    cpt_float3 ol = sub(cam->origin, cam->look_at);
    cam->dist_to_focus = sqrtf(dot(ol, ol));
    float d = cam->dist_to_focus;
    cam->top_left_corner = sub(add(sub(cam->origin, scale(half_width * d, cam->u)), scale(half_height * d, cam->v)),
                               scale(d, cam->w));
    cam->horizontal = scale(2 * half_width * d, cam->u);
    cam->vertical = scale(-2 * half_height * d, cam->v);
    cam->cur_sample_idx++;
    return CPT_OK;
}

int cpt_set_frame(cpt_ctx* c, int width, int height, const int32_t* rows, int n_rows) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (width <= 0 || height <= 0) return fail(c, CPT_ERR_INVALID_ARG, "cpt_set_frame: %dx%d", width, height);
    // the megakernel keeps a lane's pixel as 16-bit x / y and a 32-bit index
    if (width > 65535 || height > 65535)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_set_frame: %dx%d exceeds 65535 pixels per axis", width, height);
    std::vector<int32_t> r;
    if (rows) {
        if (n_rows < 0) return fail(c, CPT_ERR_INVALID_ARG, "cpt_set_frame: n_rows %d", n_rows);
        r.assign(rows, rows + n_rows);
        for (int32_t y : r)
            if (y < 0 || y >= height) return fail(c, CPT_ERR_INVALID_ARG, "cpt_set_frame: row %d outside [0,%d)", y, height);
    } else {
        r.resize(height);
        for (int y = 0; y < height; ++y) r[y] = y;
    }
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    free_frame(c);
    static std::atomic<uint64_t> frame_gens{0};
    c->frame_gen = ++frame_gens;
    c->width = width;
    c->height = height;
    c->n_rows = (int)r.size();
    c->rows_h = r;
    size_t npix = (size_t)c->n_rows * width;
    if (c->n_rows > 0) {
        HIP_TRY(c, hipMalloc((void**)&c->d_rows, r.size() * sizeof(int32_t)));
        HIP_TRY(c, hipMemcpy(c->d_rows, r.data(), r.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        HIP_TRY(c, hipMalloc((void**)&c->d_rng, 6 * npix * sizeof(uint32_t)));
        HIP_TRY(c, hipMalloc((void**)&c->d_accum, npix * sizeof(float4)));
        HIP_TRY(c, hipMemset(c->d_accum, 0, npix * sizeof(float4)));
        HIP_TRY(c, hipMemset(c->d_rng, 0, 6 * npix * sizeof(uint32_t)));
    }
    c->frame_set = true;
    c->rng_set = false;
    return CPT_OK;
}

int cpt_init_rng(cpt_ctx* c, uint64_t seed) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_init_rng: cpt_set_frame first");
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->n_rows == 0) { c->rng_set = true; return CPT_OK; }
    if (!c->d_scratch_w) HIP_TRY(c, hipMalloc((void**)&c->d_scratch_w, 5 * (size_t)c->width * sizeof(uint32_t)));
    if (!c->d_scratch_m) HIP_TRY(c, hipMalloc((void**)&c->d_scratch_m, (size_t)c->n_rows * 800 * sizeof(uint32_t)));
    c->prev_d_valid = false;   // CPT_SCHEDULE_PREVIOUS counts draws from the next render on
    uint32_t st[6];
    curand_seed_state(seed, st);
    HIP_TRY(c, cpt::launch_init_rng(c->d_jumps, st, c->width, c->d_rows, c->n_rows, c->d_scratch_w, c->d_scratch_m,
                                   c->d_rng, c->stream()));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    // the scratch matrices are n_rows * 3.2 KB; release them (one-time init)
    (void)hipFree(c->d_scratch_m); c->d_scratch_m = nullptr;
    (void)hipFree(c->d_scratch_w); c->d_scratch_w = nullptr;
    c->rng_set = true;
    return CPT_OK;
}

int cpt_read_rng(cpt_ctx* c, uint32_t* planar6) {
    if (!c || !planar6) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_read_rng: no frame");
    if (int rc = sync_checked(c)) return rc;
    size_t n = 6 * (size_t)c->n_rows * c->width;
    if (n) HIP_TRY(c, hipMemcpy(planar6, c->d_rng, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return CPT_OK;
}

int cpt_write_rng(cpt_ctx* c, const uint32_t* planar6) {
    if (!c || !planar6) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_write_rng: no frame");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    size_t n = 6 * (size_t)c->n_rows * c->width;
    if (n) HIP_TRY(c, hipMemcpy(c->d_rng, planar6, n * sizeof(uint32_t), hipMemcpyHostToDevice));
    c->rng_set = true;
    c->prev_d_valid = false;
    return CPT_OK;
}

// The megakernel's parameters for a render of the context's frame (cpt_render, cpt_tile_costs).
static void fill_params(cpt_ctx* c, const cpt_camera* cam, int spp, int max_depth, uint32_t flags, cpt::KParams& p) {
    std::memset(&p, 0, sizeof(p));
    p.nodes = c->d_nodes;
    p.mats = c->d_mats;
    p.n_nodes = c->n_bvh;
    p.n_walk = c->n_walk;
    p.n_wide = c->n_wide;
    p.n_unb = c->n_unb;
    p.n_leaves = c->n_wide > 0 ? c->n_leaves : 0;
    p.ordered = (flags & CPT_TRAVERSAL_ORDERED) ? ((flags & CPT_TRAVERSAL_PLAIN_LEAVES) ? 2 : 1) : 0;
    p.env = c->d_env;
    p.env_w = c->env_w;
    p.env_h = c->env_h;
    p.env_cols = c->d_env ? c->env_cols : 0;
    for (int k = 0; k < 3; ++k) {
        p.cam.origin[k] = (&cam->origin.x)[k];
        p.cam.u[k] = (&cam->u.x)[k];
        p.cam.v[k] = (&cam->v.x)[k];
        p.cam.top_left[k] = (&cam->top_left_corner.x)[k];
        p.cam.horizontal[k] = (&cam->horizontal.x)[k];
        p.cam.vertical[k] = (&cam->vertical.x)[k];
    }
    p.cam.lens_radius = cam->lens_radius;
    p.cam.width = cam->width;
    p.cam.height = cam->height;
    p.cam.inv_w = 1.0 / (double)(float)cam->width;
    p.cam.inv_h = 1.0 / (double)(float)cam->height;
    p.rows = c->d_rows;
    p.n_rows = c->n_rows;
    p.width = c->width;
    p.rng = c->d_rng;
    p.accum = c->d_accum;
    p.normal = c->d_normal;
    p.depth = c->d_depth;
    p.stats = c->d_stats;
    p.work = c->d_work;
    p.spp = spp;
    p.max_depth = max_depth;
    p.accumulate = (flags & CPT_RENDER_ACCUMULATE) ? 1 : 0;
    p.lanes = 64;
#ifdef CPT_DIAGNOSTIC_LANES
    // lane-latency experiments (tools/lane_latency.py builds with -DCPT_DIAGNOSTIC_LANES)
    if (const char* e = getenv("CPT_LANES_PER_WAVE")) p.lanes = std::max(1, std::min(64, atoi(e)));
    if (const char* e = getenv("CPT_REPLICATE")) p.replicate = std::max(1, std::min(64, atoi(e)));
#endif
    if (p.replicate < 1) p.replicate = 1;
    p.error = c->d_work + 4;
    p.dbg = c->dbg;
    p.keeper_spin_log2 = c->keeper_spin_log2;
    p.publish_wait_log2 = c->publish_wait_log2;
}

// The cost schedule's pilot: min(PILOT_MAX, max(1, spp / PILOT_DIV)) passes, ranking the 8x8
// tiles by their heaviest pixel.  Round 6 (interleaved, profiles/r06/keymax/): with the max key,
// up to 16 passes at one per 128 spp against round 5's 4 at one per 512: C4 2182-2198 vs 2065-2072
// Mpaths/s (8 passes at one per 256: 2159-2175), C5 N = 8 slowest rank 2101 vs 2388 ms; C2 / C3
// unchanged.
constexpr int PILOT_MAX = 16, PILOT_DIV = 128;
int cpt_render(cpt_ctx* c, const cpt_camera* cam, int spp, int max_depth, uint32_t flags) {
    if (!c || !cam) return CPT_ERR_INVALID_ARG;
    if (spp < 0 || max_depth < 0 || max_depth > (int)cpt::MAX_RECURSION_DEPTH_SET)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_render: spp %d, max_depth %d (must be 0..32)", spp, max_depth);
    if (!c->scene_set) return fail(c, CPT_ERR_STATE, "cpt_render: cpt_set_scene first");
    if (!c->frame_set || !c->rng_set) return fail(c, CPT_ERR_STATE, "cpt_render: cpt_set_frame + cpt_init_rng first");
    if (cam->width != c->width || cam->height != c->height)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_render: camera %dx%d vs frame %dx%d", cam->width, cam->height, c->width, c->height);
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = c->stream();
    const bool aux = (flags & CPT_RENDER_AUX) != 0;
    if (aux) {
        size_t npix = (size_t)c->n_rows * c->width;
        if (!c->d_normal && npix) HIP_TRY(c, hipMalloc((void**)&c->d_normal, npix * 3 * sizeof(float)));
        if (!c->d_depth && npix) HIP_TRY(c, hipMalloc((void**)&c->d_depth, npix * sizeof(float)));
    }
    cpt::KParams p;
    fill_params(c, cam, spp, max_depth, flags, p);
    const bool wavefront = (flags & CPT_PATH_WAVEFRONT) != 0;
    if (wavefront && !c->wf_ready && c->n_rows > 0) {
        const size_t npix = (size_t)c->n_rows * c->width;
        for (float4** a : {&c->wf.ray_o[0], &c->wf.ray_d[0], &c->wf.att[0], &c->wf.rad[0], &c->wf.aux[0],
                           &c->wf.ray_o[1], &c->wf.ray_d[1], &c->wf.att[1], &c->wf.rad[1], &c->wf.aux[1], &c->wf.hit_p,
                           &c->wf.hit_n})
            HIP_TRY(c, hipMalloc((void**)a, npix * sizeof(float4)));
        for (int b = 0; b < 2; ++b) {
            HIP_TRY(c, hipMalloc((void**)&c->wf.rng_a[b], npix * sizeof(uint4)));
            HIP_TRY(c, hipMalloc((void**)&c->wf.rng_b[b], npix * sizeof(uint2)));
        }
        HIP_TRY(c, hipMalloc((void**)&c->wf.queue[0], npix * sizeof(int32_t)));
        HIP_TRY(c, hipMalloc((void**)&c->wf.queue[1], npix * sizeof(int32_t)));
        HIP_TRY(c, hipMalloc((void**)&c->wf.ident, npix * sizeof(int32_t)));
        HIP_TRY(c, hipMalloc((void**)&c->wf.counts, 8 * sizeof(uint32_t)));
        HIP_TRY(c, cpt::wavefront_build_ident(p, c->wf, s));
        c->wf_ready = true;
    }
    HIP_TRY(c, hipEventRecord(c->ev_start, s));
    if (wavefront) {
        if (!p.accumulate && c->n_rows > 0)
            HIP_TRY(c, hipMemsetAsync(c->d_accum, 0, (size_t)c->n_rows * c->width * sizeof(float4), s));
        int launches = 0;
        HIP_TRY(c, hipEventRecord(c->ev_main, s));
        HIP_TRY(c, cpt::launch_wavefront(p, c->wf, (flags & CPT_RENDER_STATS) != 0, aux, s, &launches));
        c->last_launches = launches;
    } else {
        c->last_launches = 1;
        bool prev_schedule = false;
        if (!(flags & CPT_SCHEDULE_COST) && (flags & CPT_SCHEDULE_PREVIOUS) && spp > 0 && c->n_rows > 0) {
            // the order the previous render's draws gave; the draws of this one from here
            const size_t npix = (size_t)c->n_rows * c->width;
            if (c->prev_order_valid) p.tile_order = c->d_prev_order;
            if (!c->d_prev_d) HIP_TRY(c, hipMalloc((void**)&c->d_prev_d, npix * sizeof(uint32_t)));
            if (!c->prev_d_valid) {
                HIP_TRY(c, hipMemcpyAsync(c->d_prev_d, c->d_rng + 5 * npix, npix * sizeof(uint32_t),
                                          hipMemcpyDeviceToDevice, s));
                c->prev_d_valid = true;   // the draws are counted from here
            }
            prev_schedule = true;
        }
        if ((flags & CPT_SCHEDULE_COST) && spp > 0 && c->n_rows > 0) {
            // pilot: 1 pass per 128 (1..16), then the tiles sorted by their heaviest pixel, first
            const int passes = std::min(PILOT_MAX, std::max(1, spp / PILOT_DIV));
            const size_t n_tiles = (size_t)((c->width + 7) / 8) * ((c->n_rows + 7) / 8);
            const size_t bytes = cpt::tile_schedule_scratch_bytes(c->width, c->n_rows);
            if (c->cap_sched < bytes) {
                (void)hipFree(c->d_sched);
                c->d_sched = nullptr;
                c->cap_sched = 0;
                HIP_TRY(c, hipMalloc(&c->d_sched, bytes));
                c->cap_sched = bytes;
            }
            int rc;
            if ((rc = ensure(c, &c->d_tile_order, &c->cap_tile_order, n_tiles)) != CPT_OK) return rc;
            HIP_TRY(c, cpt::launch_tile_schedule(p, passes, c->d_sched, c->cap_sched, c->d_tile_order, s));
            p.tile_order = c->d_tile_order;
        }
        // Tail consolidation (cpt_kernels.hip): one slab of hand-over slots per workgroup of the
        // persistent grid (one LDS workgroup of 1024 lanes per CU), 3 x 256 chains each.  By
        // default for frames of more than 1 and at most 4 pixels per lane and chains of at least
        // 512 passes: with more pixels the tail is a small part of the render, with short chains
        // the hand-overs do not pay, and the plain kernel's tighter code wins (DESIGN.md
        // §Multi-GPU; C2 at 0.9 pixels per lane and 256 spp: 23.2 vs 21.9 Gpaths/s without).  At
        // one pixel per lane no lane takes a second chain and the plain kernel wins too (C4 at
        // N = 8, slowest rank: 309 vs 322 ms in r06, 314-318 vs 322 in r05, 304 vs 325 with
        // this rule; profiles/r06/reh_cons_r06z.log, r06/cert/reh_c4_cons_rule.log,
        // profiles/r05/reh_cons_off_vs_auto.log).
        int cus = 0;
        HIP_TRY(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        cus = std::max(cus, 1);
        const size_t frame_px = (size_t)c->n_rows * c->width, grid_lanes = 1024u * (size_t)cus;
        const bool cons = (flags & CPT_SCHEDULE_CONSOLIDATE) ||
                          (!(flags & CPT_SCHEDULE_NO_CONSOLIDATE) && spp >= 512 && frame_px > grid_lanes &&
                           frame_px <= 4u * grid_lanes);
        if (cons && spp > 1) {
            const size_t cap = 3u * 256u * (size_t)cus;
            int rc;
            if ((rc = ensure(c, &c->d_resume, &c->cap_resume, 5 * cap)) != CPT_OK) return rc;
            p.resume = c->d_resume;
            p.resume_cap = cap;
        }
        HIP_TRY(c, hipEventRecord(c->ev_main, s));
        HIP_TRY(c, cpt::launch_megakernel(p, (flags & CPT_RENDER_STATS) != 0, aux, s));
        HIP_TRY(c, hipEventRecord(c->ev_stop, s));
        if (prev_schedule && (!c->prev_order_valid || ++c->prev_since_order >= PREV_ORDER_EVERY)) {
            // the next render's order from this one's draws (after the timed events: the render's
            // own time is the kernel's; the stream runs this before the caller's next work).
            // Refreshed every PREV_ORDER_EVERY renders: the draws then span those renders (the
            // RNG's d word counts them all), and the order, a heuristic, costs ~65 us to rebuild
            const size_t n_tiles = (size_t)((c->width + 7) / 8) * ((c->n_rows + 7) / 8);
            const size_t bytes = cpt::tile_schedule_scratch_bytes(c->width, c->n_rows);
            if (c->cap_sched < bytes) {
                (void)hipFree(c->d_sched);
                c->d_sched = nullptr;
                c->cap_sched = 0;
                HIP_TRY(c, hipMalloc(&c->d_sched, bytes));
                c->cap_sched = bytes;
            }
            if (!c->d_prev_order) HIP_TRY(c, hipMalloc((void**)&c->d_prev_order, n_tiles * sizeof(uint32_t)));
            HIP_TRY(c, cpt::launch_tile_order_from_draws(p, c->d_prev_d, c->d_sched, c->cap_sched, c->d_prev_order, s));
            c->prev_d_valid = true;
            c->prev_order_valid = true;
            c->prev_since_order = 0;
        }
    }
    if (flags & CPT_PATH_WAVEFRONT) HIP_TRY(c, hipEventRecord(c->ev_stop, s));
    c->have_timing = true;
    if (flags & CPT_RENDER_SYNC) return sync_checked(c);
    return CPT_OK;
}

// The cost schedule's pilot on its own (cost-balanced row partitions, tiling.py): `passes` passes
// from the context's current RNG states, nothing written back, each 8x8 tile's work (segments +
// node visits + primitive tests) into `out`.
int cpt_tile_costs(cpt_ctx* c, const cpt_camera* cam, int passes, int max_depth, uint32_t flags, uint32_t* out,
                   size_t n_out) {
    if (!c || !cam || !out || passes < 1 || max_depth < 0 || max_depth > (int)cpt::MAX_RECURSION_DEPTH_SET)
        return CPT_ERR_INVALID_ARG;
    if (!c->scene_set) return fail(c, CPT_ERR_STATE, "cpt_tile_costs: cpt_set_scene first");
    if (!c->frame_set || !c->rng_set) return fail(c, CPT_ERR_STATE, "cpt_tile_costs: cpt_set_frame + cpt_init_rng first");
    if (cam->width != c->width || cam->height != c->height)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_tile_costs: camera %dx%d vs frame %dx%d", cam->width, cam->height, c->width,
                    c->height);
    const size_t n_tiles = (size_t)((c->width + 7) / 8) * ((c->n_rows + 7) / 8);
    if (n_out < n_tiles) return fail(c, CPT_ERR_INVALID_ARG, "cpt_tile_costs: %zu < %zu tiles", n_out, n_tiles);
    if (n_tiles == 0) return CPT_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = c->stream();
    cpt::KParams p;
    fill_params(c, cam, passes, max_depth, flags & (CPT_TRAVERSAL_ORDERED | CPT_TRAVERSAL_PLAIN_LEAVES), p);
    const size_t bytes = cpt::tile_schedule_scratch_bytes(c->width, c->n_rows);
    if (c->cap_sched < bytes) {
        (void)hipFree(c->d_sched);
        c->d_sched = nullptr;
        c->cap_sched = 0;
        HIP_TRY(c, hipMalloc(&c->d_sched, bytes));
        c->cap_sched = bytes;
    }
    int rc;
    if ((rc = ensure(c, &c->d_tile_order, &c->cap_tile_order, n_tiles)) != CPT_OK) return rc;
    HIP_TRY(c, cpt::launch_tile_schedule(p, passes, c->d_sched, c->cap_sched, c->d_tile_order, s));
    // the unsorted costs are the scratch's first n_tiles words (the sort writes elsewhere)
    HIP_TRY(c, hipMemcpyAsync(out, c->d_sched, n_tiles * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    return sync_checked(c);
}

// Row-tile gather: the rows `src` rendered, placed into `dst`'s frame at the
// same global rows by one stitch kernel on dst's stream, ordered by events (no host wait; see
// cpt_gather_rows below for the three ways the stitch reaches src's buffers).
namespace {
// Peer access from `dev` to `peer`'s memory, enabled once per ordered pair for the process.
// Returns false when the pair has no peer path (the gather then stages through a peer copy).
bool ensure_peer_access(int dev, int peer) {
    static std::mutex mu;
    static std::vector<std::pair<std::pair<int, int>, bool>> known;
    std::lock_guard<std::mutex> lk(mu);
    for (const auto& k : known)
        if (k.first == std::make_pair(dev, peer)) return k.second;
    int can = 0;
    bool ok = hipDeviceCanAccessPeer(&can, dev, peer) == hipSuccess && can;
    if (ok) {
        int cur = 0;
        (void)hipGetDevice(&cur);
        ok = hipSetDevice(dev) == hipSuccess;
        if (ok) {
            const hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
            ok = e == hipSuccess || e == hipErrorPeerAccessAlreadyEnabled;
            if (!ok) (void)hipGetLastError();   // clear the sticky error
        }
        (void)hipSetDevice(cur);
    }
    known.emplace_back(std::make_pair(dev, peer), ok);
    return ok;
}
}  // namespace

// The row map of a (dst, src) frame pair lives in a device buffer of dst, uploaded when either
// frame changes (cpt_set_frame bumps frame_gen).  src's work is ordered before the stitch by an
// event (no host wait), and src's later work after it by another, so N gathers queue back to
// back on dst's stream and one synchronisation of dst covers them all.  On two devices the
// stitch kernel reads src's buffers directly over xGMI (peer access, enabled once per pair);
// without a peer path it stages them through hipMemcpyPeerAsync.
int cpt_gather_rows(cpt_ctx* dst, cpt_ctx* src) {
    if (!dst || !src || dst == src) return dst ? fail(dst, CPT_ERR_INVALID_ARG, "cpt_gather_rows: bad contexts") : CPT_ERR_INVALID_ARG;
    if (!dst->frame_set || !src->frame_set) return fail(dst, CPT_ERR_STATE, "cpt_gather_rows: both contexts need a frame");
    if (dst->width != src->width || dst->height != src->height)
        return fail(dst, CPT_ERR_INVALID_ARG, "cpt_gather_rows: frame %dx%d vs %dx%d", dst->width, dst->height, src->width,
                    src->height);
    cpt_ctx::GatherMap* gm = nullptr;
    for (auto& g : dst->gather_maps)
        if (g.src == src) gm = &g;
    if (!gm) {
        dst->gather_maps.push_back(cpt_ctx::GatherMap{});
        gm = &dst->gather_maps.back();
        gm->src = src;
    }
    if (gm->src_gen != src->frame_gen || gm->dst_gen != dst->frame_gen || gm->src_device != src->device) {
        std::vector<int32_t> at(dst->height, -1);   // dst row index of each global row (first occurrence)
        for (int j = dst->n_rows - 1; j >= 0; --j) at[dst->rows_h[j]] = j;
        std::vector<int32_t> map(src->n_rows);
        for (int i = 0; i < src->n_rows; ++i) {
            const int32_t j = at[src->rows_h[i]];
            if (j < 0)
                return fail(dst, CPT_ERR_INVALID_ARG, "cpt_gather_rows: row %d is not in the destination frame", src->rows_h[i]);
            map[i] = j;
        }
        HIP_TRY(dst, hipSetDevice(dst->device));
        if (gm->d_map) { (void)hipFree(gm->d_map); gm->d_map = nullptr; }
        if (!map.empty()) {
            HIP_TRY(dst, hipMalloc((void**)&gm->d_map, map.size() * sizeof(int32_t)));
            HIP_TRY(dst, hipMemcpy(gm->d_map, map.data(), map.size() * sizeof(int32_t), hipMemcpyHostToDevice));
        }
        gm->src_gen = src->frame_gen;
        gm->dst_gen = dst->frame_gen;
        gm->src_device = src->device;
        gm->peer = src->device == dst->device || ensure_peer_access(dst->device, src->device);
    }
    const bool staged = !gm->peer || dst->force_staged_gather;
    gm->mode = staged ? CPT_GATHER_STAGED : src->device == dst->device ? CPT_GATHER_SAME_DEVICE : CPT_GATHER_PEER;
    if (src->n_rows == 0) return CPT_OK;
    const size_t npix = (size_t)src->n_rows * src->width;
    const bool aux = src->d_normal && src->d_depth;
    // src's queued work (its render) before the stitch
    HIP_TRY(src, hipSetDevice(src->device));
    HIP_TRY(src, hipEventRecord(src->ev_ready, src->stream()));
    HIP_TRY(dst, hipSetDevice(dst->device));
    hipStream_t s = dst->stream();
    HIP_TRY(dst, hipStreamWaitEvent(s, src->ev_ready, 0));
    const size_t dst_npix = (size_t)dst->n_rows * dst->width;
    if (aux) {
        // rows no source covers read as zero normals and depths
        if (!dst->d_normal) {
            HIP_TRY(dst, hipMalloc((void**)&dst->d_normal, dst_npix * 3 * sizeof(float)));
            HIP_TRY(dst, hipMemsetAsync(dst->d_normal, 0, dst_npix * 3 * sizeof(float), s));
        }
        if (!dst->d_depth) {
            HIP_TRY(dst, hipMalloc((void**)&dst->d_depth, dst_npix * sizeof(float)));
            HIP_TRY(dst, hipMemsetAsync(dst->d_depth, 0, dst_npix * sizeof(float), s));
        }
    }
    const float4* s_acc = src->d_accum;
    const float* s_nrm = aux ? src->d_normal : nullptr;
    const float* s_dep = aux ? src->d_depth : nullptr;
    if (staged) {
        // staging: accumulator (npix float4), then normals (3 npix floats) and depths (npix floats)
        int rc;
        if ((rc = ensure(dst, &dst->d_gather, &dst->cap_gather, aux ? 2 * npix : npix)) != CPT_OK) return rc;
        float* st_nrm = reinterpret_cast<float*>(dst->d_gather + npix);
        float* st_dep = st_nrm + 3 * npix;
        HIP_TRY(dst, hipMemcpyPeerAsync(dst->d_gather, dst->device, src->d_accum, src->device, npix * sizeof(float4), s));
        if (aux) {
            HIP_TRY(dst, hipMemcpyPeerAsync(st_nrm, dst->device, src->d_normal, src->device, npix * 3 * sizeof(float), s));
            HIP_TRY(dst, hipMemcpyPeerAsync(st_dep, dst->device, src->d_depth, src->device, npix * sizeof(float), s));
        }
        s_acc = dst->d_gather;
        s_nrm = aux ? st_nrm : nullptr;
        s_dep = aux ? st_dep : nullptr;
    }
    HIP_TRY(dst, cpt::launch_stitch_rows(s_acc, s_nrm, s_dep, gm->d_map, dst->width, src->n_rows, dst->d_accum,
                                         dst->d_normal, dst->d_depth, s));
    // src's later work (a next render into the buffers just read) after the stitch
    HIP_TRY(dst, hipEventRecord(dst->ev_gathered, s));
    HIP_TRY(src, hipSetDevice(src->device));
    HIP_TRY(src, hipStreamWaitEvent(src->stream(), dst->ev_gathered, 0));
    HIP_TRY(dst, hipSetDevice(dst->device));
    return CPT_OK;
}

int cpt_last_gather_mode(cpt_ctx* dst, cpt_ctx* src, int* mode) {
    if (!dst || !src || !mode) return dst ? fail(dst, CPT_ERR_INVALID_ARG, "cpt_last_gather_mode: null argument") : CPT_ERR_INVALID_ARG;
    *mode = -1;
    for (const auto& g : dst->gather_maps)
        if (g.src == src) *mode = g.mode;
    return CPT_OK;
}

int cpt_set_debug_gather(cpt_ctx* c, int force_staged) {
    if (!c) return CPT_ERR_INVALID_ARG;
    c->force_staged_gather = force_staged != 0;
    return CPT_OK;
}

int cpt_set_debug_consolidation(cpt_ctx* c, uint32_t flags, int keeper_spin_log2, int publish_wait_log2) {
    if (!c || keeper_spin_log2 < 0 || keeper_spin_log2 > 30 || publish_wait_log2 < 0 || publish_wait_log2 > 30 ||
        (flags & ~3u))
        return c ? fail(c, CPT_ERR_INVALID_ARG, "cpt_set_debug_consolidation: bad arguments") : CPT_ERR_INVALID_ARG;
    c->dbg = flags;
    c->keeper_spin_log2 = keeper_spin_log2;
    c->publish_wait_log2 = publish_wait_log2;
    return CPT_OK;
}

int cpt_synchronize(cpt_ctx* c) {
    if (!c) return CPT_ERR_INVALID_ARG;
    return sync_checked(c);
}

int cpt_read_accum(cpt_ctx* c, float* rgba) {
    if (!c || !rgba) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_read_accum: no frame");
    if (int rc = sync_checked(c)) return rc;
    size_t n = (size_t)c->n_rows * c->width;
    if (n) HIP_TRY(c, hipMemcpy(rgba, c->d_accum, n * sizeof(float4), hipMemcpyDeviceToHost));
    return CPT_OK;
}

int cpt_clear_accum(cpt_ctx* c) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_clear_accum: no frame");
    HIP_TRY(c, hipSetDevice(c->device));
    size_t n = (size_t)c->n_rows * c->width;
    if (n) HIP_TRY(c, hipMemsetAsync(c->d_accum, 0, n * sizeof(float4), c->stream()));
    return CPT_OK;
}

int cpt_read_aux(cpt_ctx* c, float* normal3, float* depth) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (!c->d_normal || !c->d_depth) return fail(c, CPT_ERR_STATE, "cpt_read_aux: render with CPT_RENDER_AUX first");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    size_t n = (size_t)c->n_rows * c->width;
    if (normal3 && n) HIP_TRY(c, hipMemcpy(normal3, c->d_normal, n * 3 * sizeof(float), hipMemcpyDeviceToHost));
    if (depth && n) HIP_TRY(c, hipMemcpy(depth, c->d_depth, n * sizeof(float), hipMemcpyDeviceToHost));
    return CPT_OK;
}

// Checkpoint / resume: the accumulator and the first-hit aux buffers restored
// from host copies (with cpt_write_rng, a render resumes bit for bit where it stopped).
int cpt_write_accum(cpt_ctx* c, const float* rgba) {
    if (!c || !rgba) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_write_accum: no frame");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    const size_t n = (size_t)c->n_rows * c->width;
    if (n) HIP_TRY(c, hipMemcpy(c->d_accum, rgba, n * sizeof(float4), hipMemcpyHostToDevice));
    return CPT_OK;
}

int cpt_write_aux(cpt_ctx* c, const float* normal3, const float* depth) {
    if (!c || !normal3 || !depth) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_write_aux: no frame");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    const size_t n = (size_t)c->n_rows * c->width;
    if (!c->d_normal && n) HIP_TRY(c, hipMalloc((void**)&c->d_normal, n * 3 * sizeof(float)));
    if (!c->d_depth && n) HIP_TRY(c, hipMalloc((void**)&c->d_depth, n * sizeof(float)));
    if (n) {
        HIP_TRY(c, hipMemcpy(c->d_normal, normal3, n * 3 * sizeof(float), hipMemcpyHostToDevice));
        HIP_TRY(c, hipMemcpy(c->d_depth, depth, n * sizeof(float), hipMemcpyHostToDevice));
    }
    return CPT_OK;
}

// A device-to-device copy from one of the context's buffers, ordered against the caller's stream
// without a host wait: the context's stream waits for the work queued on `caller` so far (a fill
// of dst, a collective still reading it), copies, and `caller` waits for the copy (the collective
// queued next reads the copied bytes).  Nothing to order when caller is the context's stream.
static int copy_ordered(cpt_ctx* c, void* dst, const void* src, size_t bytes, hipStream_t caller) {
    HIP_TRY(c, hipSetDevice(c->device));
    const bool other = caller != c->stream();
    if (other) {
        HIP_TRY(c, hipEventRecord(c->ev_caller, caller));
        HIP_TRY(c, hipStreamWaitEvent(c->stream(), c->ev_caller, 0));
    }
    if (bytes) HIP_TRY(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, c->stream()));
    if (other) {
        HIP_TRY(c, hipEventRecord(c->ev_copied, c->stream()));
        HIP_TRY(c, hipStreamWaitEvent(caller, c->ev_copied, 0));
    }
    return CPT_OK;
}

int cpt_copy_accum_device(cpt_ctx* c, void* dst, size_t bytes, void* caller_stream) {
    if (!c || (!dst && bytes)) return CPT_ERR_INVALID_ARG;
    size_t have = (size_t)c->n_rows * c->width * sizeof(float4);
    if (bytes > have) return fail(c, CPT_ERR_INVALID_ARG, "cpt_copy_accum_device: %zu > %zu bytes", bytes, have);
    return copy_ordered(c, dst, c->d_accum, bytes, (hipStream_t)caller_stream);
}

int cpt_get_stats(cpt_ctx* c, cpt_stats* out) {
    if (!c || !out) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    unsigned long long h[8];
    HIP_TRY(c, hipMemcpy(h, c->d_stats, sizeof(h), hipMemcpyDeviceToHost));
    out->segments = h[0];
    out->node_visits = h[1];
    out->prim_tests = h[2];
    out->hits = h[3];
    out->misses = h[4];
    return CPT_OK;
}

int cpt_debug_timeline(cpt_ctx* c, uint64_t* out, int n) {
    if (!c || !out || n <= 0) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const hipError_t e = cpt::timeline_read(reinterpret_cast<unsigned long long*>(out), n, c->stream());
    if (e == hipErrorNotSupported) return fail(c, CPT_ERR_STATE, "cpt_debug_timeline: not a CPT_TIMELINE build");
    if (e != hipSuccess) return fail(c, CPT_ERR_HIP, "cpt_debug_timeline: %s", hipGetErrorString(e));
    return CPT_OK;
}

int cpt_get_raw_counters(cpt_ctx* c, uint64_t* out8) {
    if (!c || !out8) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    HIP_TRY(c, hipMemcpy(out8, c->d_stats, 8 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return CPT_OK;
}

int cpt_get_diag_counters(cpt_ctx* c, uint64_t* out16) {
    if (!c || !out16) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    HIP_TRY(c, hipMemcpy(out16, c->d_stats + 16, 16 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return CPT_OK;
}

int cpt_get_execdiag_counters(cpt_ctx* c, uint64_t* out64) {
    if (!c || !out64) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipStreamSynchronize(c->stream()));
    HIP_TRY(c, hipMemcpy(out64, c->d_stats + 64, 64 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return CPT_OK;
}

int cpt_get_walk_info(cpt_ctx* c, int32_t* out4) {
    if (!c || !out4) return CPT_ERR_INVALID_ARG;
    out4[0] = c->n_bvh;
    out4[1] = c->n_walk;
    out4[2] = c->n_wide;
    out4[3] = c->n_unb;
    return CPT_OK;
}

int cpt_reset_stats(cpt_ctx* c) {
    if (!c) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemsetAsync(c->d_stats, 0, 128 * sizeof(unsigned long long), c->stream()));
    return CPT_OK;
}

int cpt_last_render_ms(cpt_ctx* c, float* ms) {
    if (!c || !ms) return CPT_ERR_INVALID_ARG;
    if (!c->have_timing) return fail(c, CPT_ERR_STATE, "cpt_last_render_ms: nothing rendered");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipEventSynchronize(c->ev_stop));
    HIP_TRY(c, hipEventElapsedTime(ms, c->ev_start, c->ev_stop));
    c->last_kernel_ms = *ms;
    return CPT_OK;
}

int cpt_last_kernel_stats(cpt_ctx* c, float* avg_ms, int* launches) {
    if (!c || !avg_ms || !launches) return CPT_ERR_INVALID_ARG;
    float ms = 0.f;
    int rc = cpt_last_render_ms(c, &ms);
    if (rc != CPT_OK) return rc;
    HIP_TRY(c, hipEventElapsedTime(&ms, c->ev_main, c->ev_stop));   // without the pilot
    *launches = c->last_launches;
    *avg_ms = c->last_launches > 0 ? ms / (float)c->last_launches : 0.f;
    return CPT_OK;
}

// Display path on output rows [y0, y1) of the 16-aligned launch (path_tracer.cu:177-254).
// The context's frame rows must be one ascending run that covers the band and its 3-row halo
// (clipped to [0, H')): every neighbour the linear-offset stencil reaches.  The running mean
// and the BGRA8 rows belong to the band; a different band starts a fresh mean.
static int denoise_band(cpt_ctx* c, uint32_t cur_sample_idx, int y0, int y1, uint8_t* bgra_host, size_t out_rows) {
    if (!c->frame_set) return fail(c, CPT_ERR_STATE, "cpt_denoise_mix: cpt_set_frame first");
    if (!c->d_normal || !c->d_depth) return fail(c, CPT_ERR_STATE, "cpt_denoise_mix: render with CPT_RENDER_AUX first");
    if (cur_sample_idx == 0) return fail(c, CPT_ERR_INVALID_ARG, "cpt_denoise_mix: cur_sample_idx must be >= 1");
    const int h_eff = 16 * (c->height / 16);
    if (y0 < 0 || y1 > h_eff || y0 >= y1)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_denoise_mix_band: band [%d, %d) outside [0, %d)", y0, y1, h_eff);
    const int row0 = c->rows_h.empty() ? 0 : c->rows_h[0];
    for (int i = 0; i < c->n_rows; ++i)
        if (c->rows_h[i] != row0 + i)
            return fail(c, CPT_ERR_STATE, "cpt_denoise_mix: the frame rows must be one ascending run");
    const int need0 = std::max(0, y0 - 3), need1 = std::min(h_eff, y1 + 3);
    if (row0 > need0 || row0 + c->n_rows < need1)
        return fail(c, CPT_ERR_STATE, "cpt_denoise_mix_band: rows [%d, %d) rendered, band [%d, %d) needs [%d, %d)", row0,
                    row0 + c->n_rows, y0, y1, need0, need1);
    HIP_TRY(c, hipSetDevice(c->device));
    hipStream_t s = c->stream();
    const size_t cap_rows = std::max<size_t>(out_rows, (size_t)(y1 - y0));
    if (c->band_y0 != y0 || c->band_y1 != y1) {
        (void)hipFree(c->d_mix); c->d_mix = nullptr;
        (void)hipFree(c->d_bgra); c->d_bgra = nullptr;
        const size_t n = cap_rows * c->width;
        HIP_TRY(c, hipMalloc((void**)&c->d_mix, n * 3 * sizeof(float)));
        HIP_TRY(c, hipMemsetAsync(c->d_mix, 0, n * 3 * sizeof(float), s));
        HIP_TRY(c, hipMalloc((void**)&c->d_bgra, n * 4));
        HIP_TRY(c, hipMemsetAsync(c->d_bgra, 0, n * 4, s));
        c->band_y0 = y0;
        c->band_y1 = y1;
    }
    // A pinned host frame (hipHostMalloc / hipHostRegister, e.g. torch's pin_memory) is written by
    // the kernel itself through its device alias, so the PCIe transfer overlaps the stencil
    // instead of following it; pageable memory takes the copy after the kernel.
    uint8_t* host_alias = nullptr;
    if (bgra_host && c->width % 16 == 0) {   // (columns past 16*(W/16) are never written by the kernel)
        hipPointerAttribute_t attr;
        if (hipPointerGetAttributes(&attr, bgra_host) == hipSuccess && attr.type == hipMemoryTypeHost &&
            attr.devicePointer != nullptr)
            host_alias = static_cast<uint8_t*>(attr.devicePointer);
        else
            (void)hipGetLastError();   // pageable: not an error
    }
    if (!c->d_dn_sink) HIP_TRY(c, hipMalloc((void**)&c->d_dn_sink, cpt::DN_SINK_SLOTS * sizeof(float4)));
    HIP_TRY(c, hipEventRecord(c->ev_dn0, s));
    HIP_TRY(c, cpt::launch_denoise_mix(c->d_accum, c->d_normal, c->d_depth, c->d_mix, c->d_bgra, host_alias, c->d_dn_sink, c->width,
                                      c->height, row0, c->n_rows, y0, y1, cur_sample_idx, s));
    HIP_TRY(c, hipEventRecord(c->ev_dn1, s));
    c->have_dn_timing = true;
    if (bgra_host && host_alias) {
        // the kernel writes the band's rows; the rest of the frame is zero, as the copy gives
        const size_t band = (size_t)(y1 - y0) * c->width * 4;
        std::memset(bgra_host + band, 0, cap_rows * c->width * 4 - band);
        HIP_TRY(c, hipStreamSynchronize(s));
    } else if (bgra_host) {
        HIP_TRY(c, hipMemcpyAsync(bgra_host, c->d_bgra, cap_rows * c->width * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipStreamSynchronize(s));
    }
    return CPT_OK;
}

int cpt_last_display_ms(cpt_ctx* c, float* ms) {
    if (!c || !ms) return CPT_ERR_INVALID_ARG;
    if (!c->have_dn_timing) return fail(c, CPT_ERR_STATE, "cpt_last_display_ms: no display frame yet");
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipEventSynchronize(c->ev_dn1));
    HIP_TRY(c, hipEventElapsedTime(ms, c->ev_dn0, c->ev_dn1));
    return CPT_OK;
}

int cpt_denoise_mix(cpt_ctx* c, uint32_t cur_sample_idx, uint8_t* bgra_host) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (!c->frame_set || c->n_rows != c->height) return fail(c, CPT_ERR_STATE, "cpt_denoise_mix: needs a full frame");
    for (int y = 0; y < c->height; ++y)
        if (c->rows_h[y] != y) return fail(c, CPT_ERR_STATE, "cpt_denoise_mix: needs rows 0..height-1 in order");
    const int h_eff = 16 * (c->height / 16);
    if (16 * (c->width / 16) == 0 || h_eff == 0) {   // nothing is launched; the frame stays 0
        if (bgra_host) std::memset(bgra_host, 0, (size_t)c->width * c->height * 4);
        return CPT_OK;
    }
    // the whole frame's rows (those past H' are never written and stay 0)
    return denoise_band(c, cur_sample_idx, 0, h_eff, bgra_host, (size_t)c->height);
}

int cpt_host_register(void* ptr, size_t bytes) {
    if (!ptr || bytes == 0) return fail(nullptr, CPT_ERR_INVALID_ARG, "cpt_host_register: empty buffer");
    const hipError_t e = hipHostRegister(ptr, bytes, hipHostRegisterMapped);
    if (e != hipSuccess) return fail(nullptr, CPT_ERR_HIP, "cpt_host_register: %s", hipGetErrorString(e));
    return CPT_OK;
}

int cpt_host_unregister(void* ptr) {
    if (!ptr) return fail(nullptr, CPT_ERR_INVALID_ARG, "cpt_host_unregister: null buffer");
    const hipError_t e = hipHostUnregister(ptr);
    if (e != hipSuccess) return fail(nullptr, CPT_ERR_HIP, "cpt_host_unregister: %s", hipGetErrorString(e));
    return CPT_OK;
}

int cpt_denoise_mix_band(cpt_ctx* c, uint32_t cur_sample_idx, int y0, int y1, uint8_t* bgra_host) {
    if (!c) return CPT_ERR_INVALID_ARG;
    return denoise_band(c, cur_sample_idx, y0, y1, bgra_host, 0);
}

int cpt_copy_bgra_device(cpt_ctx* c, void* device_dst, size_t bytes, void* caller_stream) {
    if (!c || !device_dst) return CPT_ERR_INVALID_ARG;
    if (!c->d_bgra) return fail(c, CPT_ERR_STATE, "cpt_copy_bgra_device: no display frame yet");
    const size_t have = (size_t)(c->band_y1 - c->band_y0) * c->width * 4;
    if (bytes > have) return fail(c, CPT_ERR_INVALID_ARG, "cpt_copy_bgra_device: %zu bytes requested, band holds %zu", bytes, have);
    return copy_ordered(c, device_dst, c->d_bgra, bytes, (hipStream_t)caller_stream);
}

int cpt_display_band(const cpt_ctx* c, int* y0, int* y1) {
    if (!c || !y0 || !y1) return CPT_ERR_INVALID_ARG;
    *y0 = c->d_mix ? c->band_y0 : 0;
    *y1 = c->d_mix ? c->band_y1 : 0;
    return CPT_OK;
}

int cpt_read_mix(cpt_ctx* c, float* rgb, size_t capacity) {
    if (!c || !rgb) return CPT_ERR_INVALID_ARG;
    if (!c->d_mix) return fail(c, CPT_ERR_STATE, "cpt_read_mix: no display frame yet");
    const size_t rows = (size_t)(c->band_y1 - c->band_y0);
    if (capacity < rows * c->width * 3)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_read_mix: %zu floats given, the band [%d, %d) holds %zu", capacity,
                    c->band_y0, c->band_y1, rows * c->width * 3);
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(rgb, c->d_mix, rows * c->width * 3 * sizeof(float), hipMemcpyDeviceToHost, c->stream()));
    return sync_checked(c);
}

int cpt_reset_display(cpt_ctx* c) {
    if (!c) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    if (c->d_mix) {
        const int h_eff = 16 * (c->height / 16);
        const size_t rows = c->band_y0 == 0 && c->band_y1 == h_eff ? (size_t)c->height : (size_t)(c->band_y1 - c->band_y0);
        HIP_TRY(c, hipMemsetAsync(c->d_mix, 0, rows * c->width * 3 * sizeof(float), c->stream()));
    }
    return CPT_OK;
}

int cpt_math_batch(cpt_ctx* c, int op, const float* a, const float* b, float* out, size_t n) {
    if (!c || !a || !b || !out) return CPT_ERR_INVALID_ARG;
    if (n == 0) return CPT_OK;
    HIP_TRY(c, hipSetDevice(c->device));
    float *da = nullptr, *db = nullptr, *dout = nullptr;
    hipError_t e = hipMalloc((void**)&da, n * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&db, n * 4);
    if (e == hipSuccess) e = hipMalloc((void**)&dout, n * 4);
    if (e == hipSuccess) e = hipMemcpy(da, a, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(db, b, n * 4, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = cpt::launch_math_batch(op, da, db, dout, n, c->stream());
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream());
    if (e == hipSuccess) e = hipMemcpy(out, dout, n * 4, hipMemcpyDeviceToHost);
    (void)hipFree(da);
    (void)hipFree(db);
    (void)hipFree(dout);
    if (e != hipSuccess) return fail(c, CPT_ERR_HIP, "cpt_math_batch: %s", hipGetErrorString(e));
    return CPT_OK;
}

int cpt_cap_disk_bound(float radius, float* out) {
    if (!out) return CPT_ERR_INVALID_ARG;
    *out = cap_disk_bound(radius);
    return CPT_OK;
}

int cpt_measure_read_bandwidth(cpt_ctx* c, size_t bytes, int iters, float* gbps) {
    if (!c || !gbps || bytes < 16 || iters < 1) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t n = bytes / 16;
    float4* d = nullptr;
    float* o = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int dev = 0, cus = 0;
    hipError_t e = hipMalloc((void**)&d, n * 16);
    if (e == hipSuccess) e = hipMalloc((void**)&o, sizeof(float));
    if (e == hipSuccess) e = hipMemsetAsync(d, 0, n * 16, c->stream());
    if (e == hipSuccess) e = hipGetDevice(&dev);
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    const int grid = 8 * std::max(cus, 1);   // 8 blocks of 256 lanes per CU, grid-stride
    if (e == hipSuccess) e = cpt::launch_stream_read(d, n, o, grid, c->stream());   // warm-up
    if (e == hipSuccess) e = hipEventRecord(e0, c->stream());
    for (int i = 0; e == hipSuccess && i < iters; ++i) e = cpt::launch_stream_read(d, n, o, grid, c->stream());
    if (e == hipSuccess) e = hipEventRecord(e1, c->stream());
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d);
    (void)hipFree(o);
    if (e != hipSuccess) return fail(c, CPT_ERR_HIP, "cpt_measure_read_bandwidth: %s", hipGetErrorString(e));
    *gbps = (float)((double)n * 16.0 * iters / (ms * 1e-3) / 1e9);
    return CPT_OK;
}

int cpt_measure_read_pattern(cpt_ctx* c, int bytes_per_lane, size_t bytes, int iters, float* gbps) {
    if (!c || !gbps || bytes < 64 || iters < 1 || (bytes_per_lane != 4 && bytes_per_lane != 12 && bytes_per_lane != 16))
        return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t n_lanes = bytes / (size_t)bytes_per_lane;
    float* d = nullptr;
    float* o = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int cus = 0;
    hipError_t e = hipMalloc((void**)&d, n_lanes * bytes_per_lane);
    if (e == hipSuccess) e = hipMalloc((void**)&o, sizeof(float));
    if (e == hipSuccess) e = hipMemsetAsync(d, 0, n_lanes * bytes_per_lane, c->stream());
    if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
    if (e == hipSuccess) e = hipEventCreate(&e0);
    if (e == hipSuccess) e = hipEventCreate(&e1);
    const int grid = 8 * std::max(cus, 1);
    if (e == hipSuccess) e = hipEventRecord(e0, c->stream());
    for (int i = 0; e == hipSuccess && i < iters; ++i) e = cpt::launch_read_pattern(bytes_per_lane, d, n_lanes, o, grid, c->stream());
    if (e == hipSuccess) e = hipEventRecord(e1, c->stream());
    if (e == hipSuccess) e = hipEventSynchronize(e1);
    float ms = 0.f;
    if (e == hipSuccess) e = hipEventElapsedTime(&ms, e0, e1);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    (void)hipFree(d);
    (void)hipFree(o);
    if (e != hipSuccess) return fail(c, CPT_ERR_HIP, "cpt_measure_read_pattern: %s", hipGetErrorString(e));
    *gbps = (float)((double)n_lanes * bytes_per_lane * iters / (ms * 1e-3) / 1e9);
    return CPT_OK;
}

int cpt_selftest_qdiv(cpt_ctx* c, int which, uint64_t n, uint64_t seed, uint64_t* out, int out_len) {
    if (!c || !out || out_len < 1 || which < 0 || which > 16) return CPT_ERR_INVALID_ARG;
    HIP_TRY(c, hipSetDevice(c->device));
    unsigned long long* d = nullptr;
    HIP_TRY(c, hipMalloc((void**)&d, out_len * sizeof(unsigned long long)));
    hipError_t e = hipMemsetAsync(d, 0, out_len * sizeof(unsigned long long), c->stream());
    if (e == hipSuccess) e = cpt::launch_selftest_qdiv(which, n, seed, d, out_len, c->stream());
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream());
    if (e == hipSuccess) e = hipMemcpy(out, d, out_len * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (e != hipSuccess) return fail(c, CPT_ERR_HIP, "cpt_selftest_qdiv: %s", hipGetErrorString(e));
    return CPT_OK;
}

}  // extern "C"
