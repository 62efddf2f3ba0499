// cpt_capi.cpp — implementation of the C-ABI in include/cpt.h.
//
// Owns the per-context device memory, builds the reference's median-split BVH on the host
// (bvh.cu:31-120) and linearises it into the skip-link order the kernels walk, computes the
// XORWOW jump tables (GF(2) matrix powers), and launches the kernels on one HIP stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <new>
#include <queue>
#include <string>
#include <functional>
#include <vector>

#include "../../include/cpt.h"
#include "cpt_internal.hpp"

static_assert(sizeof(cpt_material) == 40, "cpt_material must match Material (40 B)");
static_assert(sizeof(cpt_object) == 72, "cpt_object must match Object (72 B)");
static_assert(sizeof(cpt_camera) == 136, "cpt_camera must match MotionalCamera (136 B)");
static_assert(offsetof(cpt_object, center) == 48, "Object::center_ offset");
static_assert(offsetof(cpt_material, refractive_index) == 24, "Material::refractive_index_ offset");

namespace {

using cpt::Mat;
using cpt::Node;
using cpt::TexDesc;

std::string g_create_error;

// ------------------------------------------------------------------------------------
// Host BVH: SceneBVH::Divide (bvh.cu:31-90) and the skip-link linearisation.
// ------------------------------------------------------------------------------------
struct F3 { float x, y, z; };

inline float MIN_(float a, float b) { return a < b ? a : b; }   // ray_tracing_math.hpp:19-21
inline float MAX_(float a, float b) { return a > b ? a : b; }   // ray_tracing_math.hpp:15-17
inline float ABS_(float a) { return a >= 0 ? a : -a; }          // ray_tracing_math.hpp:23-25

// Object::GetAABBMax / GetAABBMin (object.cu:134-170)
F3 aabb_max(const cpt_object& o) {
    const float tol = 2e-5f * 5.f;
    switch (o.type) {
        case CPT_PRIM_SPHERE: {
            float r = ABS_(o.radius);
            return F3{o.center.x + r, o.center.y + r, o.center.z + r};
        }
        case CPT_PRIM_PLATFORM: return F3{1e30f * 5, o.y_pos + tol, 1e30f * 5};
        case CPT_PRIM_CYLINDER:
            return F3{o.center.x + ABS_(o.radius), o.center.y + o.height / 2 + tol, o.center.z + ABS_(o.radius)};
        default: return F3{0, 0, 0};
    }
}

F3 aabb_min(const cpt_object& o) {
    const float tol = 2e-5f * 5.f;
    switch (o.type) {
        case CPT_PRIM_SPHERE: {
            float r = ABS_(o.radius);
            return F3{o.center.x - r, o.center.y - r, o.center.z - r};
        }
        case CPT_PRIM_PLATFORM: return F3{-1e30f * 5, o.y_pos - tol, -1e30f * 5};
        case CPT_PRIM_CYLINDER:
            return F3{o.center.x - ABS_(o.radius), o.center.y - o.height / 2 - tol, o.center.z - ABS_(o.radius)};
        default: return F3{0, 0, 0};
    }
}

struct BNode {            // bvh.h:32-38, object stored as an index
    F3 bmin, bmax;
    bool is_object;
    int left, right, obj, parent;
    int axis;              // split axis of an internal node (its children's centroid order)
};

struct HostBvh {
    std::vector<BNode> nodes;          // Divide creation order (reference order)
    std::vector<int> leaf_of_object;   // object index -> node
};

int divide(HostBvh& b, const std::vector<cpt_object>& objs, std::vector<int>& idx, int l, int r) {
    if (l >= r) return -1;
    int ret = (int)b.nodes.size();
    b.nodes.push_back(BNode{});
    F3 lmin = aabb_min(objs[idx[l]]), lmax = aabb_max(objs[idx[l]]);
    if (l == r - 1) {
        BNode& n = b.nodes[ret];
        n.left = n.right = -1;
        n.bmin = lmin; n.bmax = lmax;
        n.is_object = true;
        n.obj = idx[l];
        b.leaf_of_object[idx[l]] = ret;
        return ret;
    }
    float minx = lmin.x, miny = lmin.y, minz = lmin.z, maxx = lmax.x, maxy = lmax.y, maxz = lmax.z;
    for (int i = l + 1; i < r; ++i) {
        F3 a = aabb_min(objs[idx[i]]), c = aabb_max(objs[idx[i]]);
        minx = MIN_(minx, a.x); miny = MIN_(miny, a.y); minz = MIN_(minz, a.z);
        maxx = MAX_(maxx, c.x); maxy = MAX_(maxy, c.y); maxz = MAX_(maxz, c.z);
    }
    float sx = maxx - minx, sy = maxy - miny, sz = maxz - minz;
    int axis = (sx >= sy && sx >= sz) ? 0 : (sy >= sz ? 1 : 2);
    // Centroids precomputed once per split (the reference recomputes them in the comparator);
    // stable order for equal centroids (std::sort's tie order is implementation-defined).
    std::vector<std::pair<float, int>> keyed;
    keyed.reserve(r - l);
    for (int i = l; i < r; ++i) {
        F3 a = aabb_min(objs[idx[i]]), c = aabb_max(objs[idx[i]]);
        float lo = axis == 0 ? a.x : axis == 1 ? a.y : a.z;
        float hi = axis == 0 ? c.x : axis == 1 ? c.y : c.z;
        keyed.emplace_back((lo + hi) / 2, idx[i]);
    }
    std::stable_sort(keyed.begin(), keyed.end(),
                     [](const std::pair<float, int>& p, const std::pair<float, int>& q) { return p.first < q.first; });
    for (int i = l; i < r; ++i) idx[i] = keyed[i - l].second;
    int mid = (l + r) / 2;
    int left = divide(b, objs, idx, l, mid);
    int right = divide(b, objs, idx, mid, r);
    BNode& n = b.nodes[ret];
    n.left = left; n.right = right;
    n.bmin = F3{minx, miny, minz};
    n.bmax = F3{maxx, maxy, maxz};
    n.is_object = false;
    n.obj = -1;
    n.axis = axis;
    b.nodes[left].parent = ret;
    b.nodes[right].parent = ret;
    return ret;
}

void build_host_bvh(HostBvh& b, const std::vector<cpt_object>& objs) {
    b.nodes.clear();
    b.leaf_of_object.assign(objs.size(), -1);
    if (objs.empty()) return;
    b.nodes.reserve(2 * objs.size());
    std::vector<int> idx(objs.size());
    for (size_t i = 0; i < objs.size(); ++i) idx[i] = (int)i;
    divide(b, objs, idx, 0, (int)objs.size());
    b.nodes[0].parent = -1;
}

// The cap-disk bound of a cylinder leaf (Node::b1, cpt_path.hpp cap_test): the largest float c
// with  sqrtf(q) < radius  <=>  q <= c  for every float q.  sqrtf is correctly rounded, so
// sqrtf(q) < r  <=>  sqrtf(q) <= pred(r)  <=>  sqrt(q) < m, m = (pred(r) + r) / 2 (a tie at m
// is impossible: m has 25 significant bits, so m^2 has at least 49 and is no float)  <=>
// q < m^2 (exact in double)  <=>  q <= RD(m^2).  radius <= 0 or NaN: never (c = -1).
float cap_disk_bound(float r) {
    if (!(r > 0.0f)) return -1.0f;
    if (r == INFINITY) return FLT_MAX;
    const double m = ((double)std::nextafter(r, 0.0f) + (double)r) * 0.5;
    const double x = m * m;
    float c = (float)x;
    if ((double)c > x) c = std::nextafter(c, -INFINITY);
    return c;
}

// Node contents: internal -> its box; leaf -> the primitive inline (cpt_device.hpp Node).
Node make_node(const BNode& n, const std::vector<cpt_object>& objs, const std::vector<int>& mat_of_obj) {
    Node g;
    if (n.is_object) {
        const cpt_object& o = objs[n.obj];
        g.a0 = o.center.x; g.a1 = o.center.y; g.a2 = o.center.z;
        g.b0 = o.radius; g.b1 = o.y_pos; g.b2 = o.height;
        int type = (o.type >= 0 && o.type <= 2) ? o.type : 3;
        if (type == CPT_PRIM_CYLINDER) g.b1 = cap_disk_bound(o.radius);   // y_pos is a platform's
        if (type == CPT_PRIM_SPHERE) {
            // the root-1 normal's exact quotients (cpt_path.hpp hit_attributes): the correctly
            // rounded double reciprocal of the radius, its low word in b1 and high word in b2
            const double inv_r = 1.0 / (double)o.radius;
            uint32_t w[2];
            std::memcpy(w, &inv_r, 8);
            std::memcpy(&g.b1, &w[0], 4);
            std::memcpy(&g.b2, &w[1], 4);
        }
        g.code = (mat_of_obj[n.obj] << 2) | type;
    } else {
        g.a0 = n.bmin.x; g.a1 = n.bmin.y; g.a2 = n.bmin.z;
        g.b0 = n.bmax.x; g.b1 = n.bmax.y; g.b2 = n.bmax.z;
        g.code = -1;
    }
    g.miss = -1;
    return g;
}

// Right-first preorder = the order the reference's stack DFS pops nodes (left pushed first,
// bvh.cu:201-202).  Internal nodes: miss = position after the node's subtree.  Leaves: the
// walk always continues at position + 1, so `miss` carries the leaf's position in this
// reference order instead (the tie rank of the ordered walk, cpt_path.hpp trace).
//
// octant >= 0 builds the near-first order for rays whose direction signs are the octant's
// bits (bit a set = negative along axis a): at each internal node the child on the near side
// of its split axis comes first.  ref_pos gives the leaves' reference positions.
void linearise(const HostBvh& b, const std::vector<cpt_object>& objs, const std::vector<int>& mat_of_obj,
               std::vector<Node>& out, std::vector<int>& pos_of_node, int octant, const std::vector<int>* ref_pos,
               int root = 0, const std::vector<int>& prefix = {}) {
    const size_t base = out.size();
    pos_of_node.assign(b.nodes.size(), -1);
    for (int leaf : prefix) {            // unbounded leaves, tested before the tree
        pos_of_node[leaf] = (int)(out.size() - base);
        out.push_back(make_node(b.nodes[leaf], objs, mat_of_obj));
        out.back().miss = (*ref_pos)[leaf];
    }
    if (b.nodes.empty() || root < 0) return;
    struct Frame { int node; int stage; };
    std::vector<Frame> st;
    st.push_back({root, 0});
    while (!st.empty()) {
        Frame& f = st.back();
        const BNode& n = b.nodes[f.node];
        if (f.stage == 0) {
            pos_of_node[f.node] = (int)(out.size() - base);
            out.push_back(make_node(n, objs, mat_of_obj));
            if (n.is_object) {
                out.back().miss = ref_pos ? (*ref_pos)[f.node] : pos_of_node[f.node];
                st.pop_back();
                continue;
            }
            if (octant >= 0) {
                // octant form (cpt_path.hpp slab_reject_octant): a = the planes a ray of this
                // octant enters through, b = the ones it leaves through (bmax first on an
                // axis the ray runs down)
                Node& q = out.back();
                if (octant & 1) std::swap(q.a0, q.b0);
                if (octant & 2) std::swap(q.a1, q.b1);
                if (octant & 4) std::swap(q.a2, q.b2);
            }
            f.stage = 1;
            // the reference pops the right child first; a ray moving +axis meets the left
            // (lower-centroid) child first
            const bool right_first = octant < 0 || ((octant >> n.axis) & 1);
            st.push_back({right_first ? n.right : n.left, 0});
        } else if (f.stage == 1) {
            f.stage = 2;
            const bool right_first = octant < 0 || ((octant >> n.axis) & 1);
            st.push_back({right_first ? n.left : n.right, 0});
        } else {
            out[base + pos_of_node[f.node]].miss = (int)(out.size() - base);
            st.pop_back();
        }
    }
}

// ------------------------------------------------------------------------------------
// XORWOW jump tables: jumps[t] = A^(2^67 * 2^t), 160x160 over GF(2), column-major
// (column c = A^k e_c as 5 words), the layout rocRAND uses (rocrand_xorwow.h:51-65).
// ------------------------------------------------------------------------------------
struct BitMat { uint32_t m[800]; };

void xorshift_step(uint32_t v[5]) {   // linear part of curand() (d excluded)
    uint32_t t = v[0] ^ (v[0] >> 2);
    v[0] = v[1]; v[1] = v[2]; v[2] = v[3]; v[3] = v[4];
    v[4] = (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1));
}

void bm_apply(const BitMat& M, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int c = 0; c < 160; ++c)
        if ((in[c >> 5] >> (c & 31)) & 1u)
            for (int k = 0; k < 5; ++k) r[k] ^= M.m[c * 5 + k];
    std::memcpy(out, r, sizeof(r));
}

BitMat bm_square(const BitMat& M) {
    BitMat R;
    for (int c = 0; c < 160; ++c) bm_apply(M, &M.m[c * 5], &R.m[c * 5]);
    return R;
}

const std::vector<uint32_t>& jump_tables() {
    static std::vector<uint32_t> tbl;
    static std::once_flag once;
    std::call_once(once, [] {
        BitMat A;
        for (int c = 0; c < 160; ++c) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[c >> 5] = 1u << (c & 31);
            xorshift_step(v);
            std::memcpy(&A.m[c * 5], v, 20);
        }
        for (int i = 0; i < 67; ++i) A = bm_square(A);
        tbl.resize(64 * 800);
        for (int t = 0; t < 64; ++t) {
            std::memcpy(&tbl[(size_t)t * 800], A.m, sizeof(A.m));
            A = bm_square(A);
        }
    });
    return tbl;
}

// curand_init's seed scrambling (curand_kernel.h, CUDA 11.7).
void curand_seed_state(uint64_t seed, uint32_t out[6]) {
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0;
    uint32_t t1 = 2591861531u * s1;
    out[0] = 123456789u + t0;
    out[1] = 362436069u ^ t0;
    out[2] = 521288629u + t1;
    out[3] = 88675123u ^ t1;
    out[4] = 5783321u + t0;
    out[5] = 6615241u + t1 + t0;
}

}  // namespace

// ======================================================================================
// Context
// ======================================================================================
struct cpt_ctx {
    int device = 0;
    hipStream_t own_stream = nullptr;
    hipStream_t user_stream = nullptr;
    hipEvent_t ev_start = nullptr, ev_stop = nullptr;
    hipEvent_t ev_main = nullptr;   // after the cost schedule's pilot: the dominant kernel(s) only
    bool have_timing = false;
    std::string err;

    // scene
    std::vector<cpt_object> objs;
    HostBvh bvh;
    std::vector<Node> lin;             // 9 orders of n_bvh nodes: reference, then octants 0..7
    std::vector<int> pos_of_node;      // BNode -> position in the reference order
    int n_bvh = 0;                     // nodes of the reference order
    int n_walk = 0;                    // nodes of each octant order (walk tree + unbounded leaves)
    int n_wide = 0;                    // 4-wide walk-tree nodes per octant (0: none, binary walk)
    int n_unb = 0;                     // unbounded (platform) leaves at the head of each octant order
    int n_leaves = 0;                  // the wide tree's leaf array (after its compact image)
    std::vector<Mat> mats_h;           // deduplicated materials (host-staged, see Mat)
    std::vector<int> mat_have_tex;     // per material slot: textured?
    std::vector<uint64_t> mat_tex;     // per material slot: texture handle (textured slots)
    std::vector<int> mat_of_obj;       // object index -> material index
    Node* d_nodes = nullptr;
    Mat* d_mats = nullptr;
    size_t cap_nodes = 0, cap_mats = 0;
    bool scene_set = false;
    // device refit (cpt_update_objects): the plan of both trees (ids: reference tree, then walk
    // tree), parents, heights, each object's walk-tree leaf, the boxes as built
    std::vector<cpt::RefitNode> refit_plan;
    std::vector<int32_t> refit_parent, refit_height, refit_walk_leaf;
    std::vector<cpt::Box6> refit_boxes;
    std::vector<uint8_t> refit_mark;   // scratch of an update batch (all zero between batches)
    int refit_n_ref = 0;
    cpt::RefitNode* d_refit_plan = nullptr;
    cpt::Box6* d_refit_boxes = nullptr;
    uint8_t* d_refit_work = nullptr;   // an update batch: RefitLeaf records, then the dirty node ids
    size_t cap_refit_plan = 0, cap_refit_boxes = 0, cap_refit_work = 0;
    float last_update_ms = 0.f;     // host wall time of the last cpt_update_objects[_rebuild]

    // material textures (cpt_bind_texture)
    struct Texture { uint64_t handle; uint32_t* d_texels; int w, h, cols, addr, filter; };
    std::vector<Texture> textures;
    TexDesc* d_texdescs = nullptr;
    int32_t* d_tex_of_mat = nullptr;
    size_t cap_texdescs = 0, cap_tex_of_mat = 0;

    // environment
    uint32_t* d_env = nullptr;
    int env_w = 1, env_h = 1, env_cols = 0;
    size_t cap_env = 0;

    // frame
    int width = 0, height = 0, n_rows = 0;
    std::vector<int32_t> rows_h;
    int32_t* d_rows = nullptr;
    uint32_t* d_rng = nullptr;
    float4* d_accum = nullptr;
    float* d_normal = nullptr;
    float* d_depth = nullptr;
    bool frame_set = false, rng_set = false;

    // rng init
    uint32_t* d_jumps = nullptr;
    uint32_t* d_scratch_w = nullptr;
    uint32_t* d_scratch_m = nullptr;

    unsigned long long* d_stats = nullptr;
    uint32_t* d_work = nullptr;
    void* d_sched = nullptr;     // cost schedule: pilot tile costs + sort scratch
    size_t cap_sched = 0;
    uint32_t* d_tile_order = nullptr;
    size_t cap_tile_order = 0;
    uint4* d_resume = nullptr;          // tail consolidation: handed-over chains (5 x uint4 each)
    size_t cap_resume = 0;
    cpt::WfState wf{};           // wavefront path state (allocated on first use)
    bool wf_ready = false;
    float* d_mix = nullptr;      // display running mean (Mix), rgb per pixel of the display band
    uint8_t* d_bgra = nullptr;   // display frame (band rows)
    int band_y0 = -1, band_y1 = -1;   // display band the buffers hold
    float last_kernel_ms = 0.f;
    int last_launches = 0;
    // row-tile gather (cpt_gather_rows): a source's rows staged on this device, and the frame
    // row each goes to
    float4* d_gather = nullptr;
    size_t cap_gather = 0;
    int32_t* d_gather_map = nullptr;
    size_t cap_gather_map = 0;
    std::vector<int32_t> gather_map_h;
    // consolidation test hooks (cpt_set_debug_consolidation)
    uint32_t dbg = 0;
    int keeper_spin_log2 = 0, publish_wait_log2 = 0;

    hipStream_t stream() const { return user_stream ? user_stream : own_stream; }
};

namespace {

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

#define HIP_TRY(ctx, expr)                                                                             \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return fail((ctx), e_ == hipErrorOutOfMemory ? CPT_ERR_OUT_OF_MEMORY : CPT_ERR_HIP,        \
                        "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);           \
    } while (0)

template <typename T>
int ensure(cpt_ctx* c, T** ptr, size_t* cap, size_t count) {
    if (*ptr && *cap >= count) return CPT_OK;
    if (*ptr) { (void)hipFree(*ptr); *ptr = nullptr; *cap = 0; }
    if (count == 0) return CPT_OK;
    HIP_TRY(c, hipMalloc((void**)ptr, count * sizeof(T)));
    *cap = count;
    return CPT_OK;
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
    c->band_y0 = c->band_y1 = -1;
    (void)hipFree(c->d_scratch_w); c->d_scratch_w = nullptr;
    (void)hipFree(c->d_scratch_m); c->d_scratch_m = nullptr;
    (void)hipFree(c->d_sched); c->d_sched = nullptr; c->cap_sched = 0;
    (void)hipFree(c->d_tile_order); c->d_tile_order = nullptr; c->cap_tile_order = 0;
    c->frame_set = c->rng_set = false;
}

// Host staging of a Mat (cpt_device.hpp): att = kd_ (the union's bits: the handle's for a
// textured material), rad.x = emit_intensity_; k_prepare_materials completes it.
Mat to_mat(const cpt_material& m) {
    Mat g;
    std::memset(&g, 0, sizeof(g));
    g.att_x = m.u.kd.x; g.att_y = m.u.kd.y; g.att_z = m.u.kd.z;
    g.type = m.type;
    g.rad_x = m.emit_intensity;
    g.ior = m.refractive_index;
    g.reflectivity = m.reflectivity;
    g.smoothness = m.smoothness;
    g.inv_alpha = 0.0;
    return g;
}

int material_slot(cpt_ctx* c, const cpt_material& m) {
    Mat g = to_mat(m);
    const int tex = m.have_tex ? 1 : 0;
    for (size_t i = 0; i < c->mats_h.size(); ++i)
        if (std::memcmp(&c->mats_h[i], &g, sizeof(Mat)) == 0 && c->mat_have_tex[i] == tex &&
            (!tex || c->mat_tex[i] == m.u.tex))
            return (int)i;
    c->mats_h.push_back(g);
    c->mat_have_tex.push_back(tex);
    c->mat_tex.push_back(tex ? m.u.tex : 0);
    return (int)c->mats_h.size() - 1;
}

// Walk tree of the ordered walk (CPT_TRAVERSAL_ORDERED, DESIGN.md §Ordered walk): a binned
// SAH tree over the bounded primitives, one primitive per leaf.  Platforms (+-5e30 boxes) stay
// out of it: the walk tests them first.  The tree only decides which primitives a ray tests;
// the closest hit is the reference's (rank tie rule, conservative slab test, winner
// certificate in cpt_path.hpp).
namespace sah {
constexpr int NB = 16;
inline float comp(const F3& v, int a) { return a == 0 ? v.x : (a == 1 ? v.y : v.z); }
inline F3 fmin3(const F3& a, const F3& b) { return F3{MIN_(a.x, b.x), MIN_(a.y, b.y), MIN_(a.z, b.z)}; }
inline F3 fmax3(const F3& a, const F3& b) { return F3{MAX_(a.x, b.x), MAX_(a.y, b.y), MAX_(a.z, b.z)}; }
inline float area(const F3& lo, const F3& hi) {
    const float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return 2.f * (dx * dy + dy * dz + dz * dx);
}
inline int bin_of(float c, float e0, float e1) { return std::min(NB - 1, (int)((c - e0) / (e1 - e0) * NB)); }

int leaf(HostBvh& t, const std::vector<cpt_object>& O, int o) {
    BNode n{};
    n.bmin = aabb_min(O[o]);
    n.bmax = aabb_max(O[o]);
    n.is_object = true;
    n.left = n.right = -1;
    n.obj = o;
    n.parent = -1;
    t.nodes.push_back(n);
    return (int)t.nodes.size() - 1;
}

int build(HostBvh& t, const std::vector<cpt_object>& O, std::vector<int>& idx, int l, int r) {
    if (r - l == 1) return leaf(t, O, idx[l]);
    F3 lo = aabb_min(O[idx[l]]), hi = aabb_max(O[idx[l]]);
    F3 clo{1e30f, 1e30f, 1e30f}, chi{-1e30f, -1e30f, -1e30f};
    std::vector<float> cen(3 * (r - l));
    for (int i = l; i < r; ++i) {
        const F3 a = aabb_min(O[idx[i]]), b = aabb_max(O[idx[i]]);
        lo = fmin3(lo, a);
        hi = fmax3(hi, b);
        const F3 c{(a.x + b.x) * .5f, (a.y + b.y) * .5f, (a.z + b.z) * .5f};
        cen[3 * (i - l)] = c.x; cen[3 * (i - l) + 1] = c.y; cen[3 * (i - l) + 2] = c.z;
        clo = fmin3(clo, c);
        chi = fmax3(chi, c);
    }
    float best = 3.0e38f;
    int best_axis = -1, best_bin = -1;
    for (int axis = 0; axis < 3; ++axis) {
        const float e0 = comp(clo, axis), e1 = comp(chi, axis);
        if (!(e1 > e0)) continue;
        int cnt[NB] = {0};
        F3 blo[NB], bhi[NB];
        for (int b = 0; b < NB; ++b) { blo[b] = F3{1e30f, 1e30f, 1e30f}; bhi[b] = F3{-1e30f, -1e30f, -1e30f}; }
        for (int i = l; i < r; ++i) {
            const int b = bin_of(cen[3 * (i - l) + axis], e0, e1);
            cnt[b]++;
            blo[b] = fmin3(blo[b], aabb_min(O[idx[i]]));
            bhi[b] = fmax3(bhi[b], aabb_max(O[idx[i]]));
        }
        for (int sp = 1; sp < NB; ++sp) {
            int nl = 0, nr = 0;
            F3 llo{1e30f, 1e30f, 1e30f}, lhi{-1e30f, -1e30f, -1e30f}, rlo = llo, rhi = lhi;
            for (int b = 0; b < sp; ++b) if (cnt[b]) { nl += cnt[b]; llo = fmin3(llo, blo[b]); lhi = fmax3(lhi, bhi[b]); }
            for (int b = sp; b < NB; ++b) if (cnt[b]) { nr += cnt[b]; rlo = fmin3(rlo, blo[b]); rhi = fmax3(rhi, bhi[b]); }
            if (!nl || !nr) continue;
            const float cost = area(llo, lhi) * nl + area(rlo, rhi) * nr;
            if (cost < best) { best = cost; best_axis = axis; best_bin = sp; }
        }
    }
    int axis, mid;
    if (best_axis < 0) {
        // all centroids coincide: split the list in half (stable order)
        axis = 0;
        mid = (l + r) / 2;
    } else {
        axis = best_axis;
        const float e0 = comp(clo, axis), e1 = comp(chi, axis);
        std::vector<int> lhs, rhs;
        for (int i = l; i < r; ++i)
            (bin_of(cen[3 * (i - l) + axis], e0, e1) < best_bin ? lhs : rhs).push_back(idx[i]);
        std::copy(lhs.begin(), lhs.end(), idx.begin() + l);
        std::copy(rhs.begin(), rhs.end(), idx.begin() + l + (int)lhs.size());
        mid = l + (int)lhs.size();
    }
    const int me = (int)t.nodes.size();
    t.nodes.push_back(BNode{});
    const int L = build(t, O, idx, l, mid), R = build(t, O, idx, mid, r);
    BNode& n = t.nodes[me];
    n.bmin = lo; n.bmax = hi;
    n.is_object = false;
    n.left = L; n.right = R; n.obj = -1; n.parent = -1; n.axis = axis;
    t.nodes[L].parent = me;
    t.nodes[R].parent = me;
    return me;
}
}  // namespace sah

// ------------------------------------------------------------------------------------
// 4-wide walk tree (DESIGN.md §Wide walk).  The binary SAH walk tree is collapsed into
// nodes of up to four children: starting from a node's two children, the internal child
// with the largest box is replaced by its own two children until there are four (or only
// leaves).  Appended to `out` (after the eight binary octant orders): the compact image,
// 7 x 16 B per node (layout below), then the leaf array.  Nodes are numbered largest box
// first (root 0).  Returns n_wide, or 0 when the device walk's stack (WIDE_STACK entries per
// lane, cpt_path.hpp) could overflow on this tree or a ref would not fit 15 bits.
// ------------------------------------------------------------------------------------
constexpr int WIDE_STACK = CPT_WSTACK;

int linearise_wide(const HostBvh& w, int root, const std::vector<int>& pos0, int n_bvh, int n_unb,
                   std::vector<Node>& out, int* n_leaves_out, std::vector<int>& slot_of, std::vector<int>& leaf_of) {
    std::vector<int> wbin;                      // binary node of each wide node
    std::vector<std::vector<int>> kids;         // its children (binary node ids)
    std::vector<int> wide_of(w.nodes.size(), -1);
    auto area = [&](int b) {
        const BNode& n = w.nodes[b];
        const float dx = n.bmax.x - n.bmin.x, dy = n.bmax.y - n.bmin.y, dz = n.bmax.z - n.bmin.z;
        return dx * dy + dy * dz + dz * dx;
    };
    int max_push = 0;
    std::function<void(int, int)> make = [&](int b, int pushed) {
        const int id = (int)wbin.size();
        wbin.push_back(b);
        wide_of[b] = id;
        std::vector<int> ch = {w.nodes[b].left, w.nodes[b].right};
        while (ch.size() < 4) {
            int best = -1;
            float ba = -1.f;
            for (size_t k = 0; k < ch.size(); ++k)
                if (!w.nodes[ch[k]].is_object && area(ch[k]) > ba) { ba = area(ch[k]); best = (int)k; }
            if (best < 0) break;
            const int x = ch[best];
            ch.erase(ch.begin() + best);
            ch.insert(ch.begin() + best, {w.nodes[x].left, w.nodes[x].right});
        }
        kids.push_back(ch);
        // a lane entering this node keeps one hit child and pushes the others
        pushed += (int)ch.size() - 1;
        max_push = std::max(max_push, pushed);
        for (int x : ch)
            if (!w.nodes[x].is_object) make(x, pushed);
    };
    make(root, n_unb);   // the walk starts with the root and the platforms on the stack
    if (max_push + 1 > WIDE_STACK) return 0;
    const int n_wide = (int)wbin.size();
    // The leaf array after the compact image: the platforms (the head of every octant order),
    // then the walk tree's leaves in the order the wide nodes, in preorder, first reference
    // them (a subtree's leaves share cache lines); Node copies of octant 0's inline leaves.
    // The compact image refers to leaf i as ~(i + 1) (<= -2, apart from the empty slot's -1).
    std::vector<int> li_of(w.nodes.size(), -1), leaf_pos;
    for (int k = 0; k < n_unb; ++k) leaf_pos.push_back(k);
    for (int id = 0; id < n_wide; ++id)
        for (int x : kids[id])
            if (w.nodes[x].is_object && li_of[x] < 0) {
                li_of[x] = (int)leaf_pos.size();
                leaf_pos.push_back(pos0[x]);
            }
    if ((int)leaf_pos.size() > 32765) return 0;
    // The ids are preorder (make's recursion order), which keeps a subtree's nodes and leaves
    // together in memory.  A tree larger than the LDS image is renumbered so that its first
    // LDS_TREE_NODES ids -- the part the device stages in LDS -- are its top: the nodes a
    // best-first expansion from the root by surface area (which a random ray hits in
    // proportion to) reaches first, each after its parent; those first, then the rest, each
    // part in preorder.
    if (n_wide > cpt::LDS_TREE_NODES) {
        std::vector<char> top(n_wide, 0);
        std::priority_queue<std::pair<float, int>, std::vector<std::pair<float, int>>, std::greater<>> pq;
        pq.emplace(-area(wbin[0]), 0);
        for (int taken = 0; !pq.empty() && taken < cpt::LDS_TREE_NODES; ++taken) {
            const int id = pq.top().second;
            pq.pop();
            top[id] = 1;
            for (int x : kids[id])
                if (!w.nodes[x].is_object) pq.emplace(-area(x), wide_of[x]);
        }
        std::vector<int> order;   // new id -> old id: the top in preorder, then the rest
        order.reserve(n_wide);
        for (int part = 1; part >= 0; --part)
            for (int id = 0; id < n_wide; ++id)
                if (top[id] == part) order.push_back(id);
        std::vector<int> new_id(n_wide);
        for (int k = 0; k < n_wide; ++k) new_id[order[k]] = k;
        std::vector<int> wbin2(n_wide);
        std::vector<std::vector<int>> kids2(n_wide);
        for (int k = 0; k < n_wide; ++k) {
            wbin2[k] = wbin[order[k]];
            kids2[k] = kids[order[k]];
        }
        wbin.swap(wbin2);
        kids.swap(kids2);
        for (int& x : wide_of)
            if (x >= 0) x = new_id[x];
    }
    // the device stack holds 16-bit refs: wide node ids and ~(leaf position) within 15 bits
    if (n_wide > 32767) return 0;
    for (int p : pos0)
        if (p > 32766) return 0;
    const size_t base = out.size();
    const size_t n_compact = (size_t)(n_wide * 7 + 1) / 2;
    out.resize(base + n_compact + leaf_pos.size());
    for (size_t i = 0; i < leaf_pos.size(); ++i) out[base + n_compact + i] = out[(size_t)n_bvh + leaf_pos[i]];
    *n_leaves_out = (int)leaf_pos.size();
    // The compact image (cpt_path.hpp trace_wide; its first LDS_TREE_NODES nodes are staged in
    // LDS): 7 x 16 B per node, one copy for every direction octant --
    //   [min x][max x][min y][max y][min z][max z] of the four slots, then
    //   {refs of slots 0..3 as int16, 8 B zero}.
    // A lane reads its entry planes at min or max by the sign of its direction, i.e. the planes
    // its octant enters through, and orders the hit children by their entry distances.  The
    // slots are in the order of the binary splits between the node and its children (left
    // first); an empty slot has an inverted box that every ray rejects.
    uint32_t* compact = reinterpret_cast<uint32_t*>(&out[base]);
    std::memset(compact, 0, n_compact * sizeof(Node));
    for (int id = 0; id < n_wide; ++id) {
        const std::vector<int>& ch = kids[id];
        std::vector<int> ord;
        std::function<void(int)> rec = [&](int x) {
            if (std::find(ch.begin(), ch.end(), x) != ch.end()) { ord.push_back(x); return; }
            rec(w.nodes[x].left);
            rec(w.nodes[x].right);
        };
        rec(wbin[id]);
        uint32_t* q = compact + (size_t)id * 28;
        for (int k = 0; k < 4; ++k) {
            F3 lo{1e30f, 1e30f, 1e30f}, hi{-1e30f, -1e30f, -1e30f};
            int32_t r = -1;
            if (k < (int)ord.size()) {
                const BNode& n = w.nodes[ord[k]];
                lo = n.bmin;
                hi = n.bmax;
                r = n.is_object ? ~(li_of[ord[k]] + 1) : wide_of[ord[k]];
            }
            const float l3[3] = {lo.x, lo.y, lo.z}, h3[3] = {hi.x, hi.y, hi.z};
            for (int a = 0; a < 3; ++a) {
                std::memcpy(&q[(2 * a) * 4 + k], &l3[a], 4);
                std::memcpy(&q[(2 * a + 1) * 4 + k], &h3[a], 4);
            }
            q[24 + (k >> 1)] |= (uint32_t)(uint16_t)(int16_t)r << (16 * (k & 1));
            if (k < (int)ord.size()) slot_of[ord[k]] = id * 4 + k;
        }
    }
    // the device refit's map (binary walk node -> leaf array index; the platforms are its head)
    leaf_of = li_of;
    for (size_t b = 0; b < w.nodes.size(); ++b)
        if (w.nodes[b].is_object && leaf_of[b] < 0 && pos0[b] >= 0 && pos0[b] < n_unb) leaf_of[b] = pos0[b];
    return n_wide;
}

// Returns the walk tree's root (-1: no bounded primitive); `unbounded` = its platform leaves
// by reference rank; `rank` = the reference rank of every walk-tree leaf.
int build_walk_tree(const cpt_ctx* c, HostBvh& w, std::vector<int>& unbounded, std::vector<int>& rank);

// The reference order followed by the eight octant orders of the walk tree (one array,
// n_walk nodes each: the unbounded leaves, then the tree).
void build_refit_plan(cpt_ctx* c, const HostBvh& w, const std::vector<int> (&pos)[8], const std::vector<int>& slot_of,
                      const std::vector<int>& leaf_of);

void linearise_all(cpt_ctx* c) {
    c->lin.clear();
    c->n_walk = 0;
    c->n_wide = 0;
    c->n_unb = 0;
    c->refit_plan.clear();
    c->lin.reserve(9 * c->bvh.nodes.size());
    linearise(c->bvh, c->objs, c->mat_of_obj, c->lin, c->pos_of_node, -1, nullptr);
    c->n_bvh = (int)c->lin.size();
    if (c->n_bvh == 0) return;
    HostBvh w;
    std::vector<int> unbounded, rank, pos[8];
    const int root = build_walk_tree(c, w, unbounded, rank);
    for (int o = 0; o < 8; ++o) linearise(w, c->objs, c->mat_of_obj, c->lin, pos[o], o, &rank, root, unbounded);
    c->n_walk = (int)(c->lin.size() - c->n_bvh) / 8;
    c->n_unb = (int)unbounded.size();
    c->n_leaves = 0;
    std::vector<int> slot_of(w.nodes.size(), -1), leaf_of(w.nodes.size(), -1);
    if (root >= 0 && !w.nodes[root].is_object)
        c->n_wide = linearise_wide(w, root, pos[0], c->n_bvh, c->n_unb, c->lin, &c->n_leaves, slot_of, leaf_of);
    build_refit_plan(c, w, pos, slot_of, leaf_of);
}

// The device refit's plan (cpt_internal.hpp RefitNode): every node of both trees with the
// positions of its copies, its parent and its height (leaves 0), and each object's two leaves.
void build_refit_plan(cpt_ctx* c, const HostBvh& w, const std::vector<int> (&pos)[8], const std::vector<int>& slot_of,
                      const std::vector<int>& leaf_of) {
    const int nr = (int)c->bvh.nodes.size(), nw = (int)w.nodes.size();
    c->refit_n_ref = nr;
    c->refit_plan.assign(nr + nw, cpt::RefitNode{});
    c->refit_parent.assign(nr + nw, -1);
    c->refit_height.assign(nr + nw, 0);
    c->refit_boxes.assign(nr + nw, cpt::Box6{});
    c->refit_walk_leaf.assign(c->objs.size(), -1);
    c->refit_mark.assign(nr + nw, 0);
    for (int i = 0; i < nr + nw; ++i) {
        const bool ref = i < nr;
        const BNode& n = ref ? c->bvh.nodes[i] : w.nodes[i - nr];
        cpt::RefitNode& r = c->refit_plan[i];
        const int off = ref ? 0 : nr;
        r.left = n.is_object ? -1 : n.left + off;
        r.right = n.is_object ? -1 : n.right + off;
        r.slot = ref ? -1 : slot_of[i - nr];
        r.leaf = ref || c->n_wide == 0 ? -1 : leaf_of[i - nr];
        for (int o = 0; o < 8; ++o) r.pos[o] = -1;
        if (ref) r.pos[0] = c->pos_of_node[i];
        else
            for (int o = 0; o < 8; ++o)
                r.pos[o] = pos[o][i - nr] < 0 ? -1 : c->n_bvh + o * c->n_walk + pos[o][i - nr];
        c->refit_boxes[i] = cpt::Box6{{n.bmin.x, n.bmin.y, n.bmin.z}, {n.bmax.x, n.bmax.y, n.bmax.z}};
        if (!n.is_object) {
            c->refit_parent[r.left] = i;
            c->refit_parent[r.right] = i;
        } else if (!ref) {
            c->refit_walk_leaf[n.obj] = i;
        }
    }
    // heights, children first: both builders number a parent before its children (bvh.cu:31-90
    // divide, sah::build)
    for (int i = nr + nw - 1; i >= 0; --i) {
        const cpt::RefitNode& r = c->refit_plan[i];
        if (r.left >= 0)
            c->refit_height[i] = 1 + std::max(c->refit_height[r.left], c->refit_height[r.right]);
    }
}

int build_walk_tree(const cpt_ctx* c, HostBvh& w, std::vector<int>& unbounded, std::vector<int>& rank) {
    const std::vector<cpt_object>& O = c->objs;
    w.nodes.clear();
    w.leaf_of_object.assign(O.size(), -1);
    unbounded.clear();
    std::vector<int> idx;
    std::vector<std::pair<int, int>> flat;   // (reference rank, object) of the platforms
    for (size_t o = 0; o < O.size(); ++o) {
        const int ref_rank = c->pos_of_node[c->bvh.leaf_of_object[o]];
        if (O[o].type == CPT_PRIM_PLATFORM) flat.emplace_back(ref_rank, (int)o);
        else idx.push_back((int)o);
    }
    std::sort(flat.begin(), flat.end());
    for (const auto& f : flat) unbounded.push_back(sah::leaf(w, O, f.second));
    const int root = idx.empty() ? -1 : sah::build(w, O, idx, 0, (int)idx.size());
    rank.assign(w.nodes.size(), -1);
    for (size_t i = 0; i < w.nodes.size(); ++i)
        if (w.nodes[i].is_object) rank[i] = c->pos_of_node[c->bvh.leaf_of_object[w.nodes[i].obj]];
    return root;
}

// The kernels' sticky error word (KParams::error, CPT_DEVERR_*): read after the context's
// stream has drained; a set word is cleared and reported once, like a sticky HIP error.
int check_device_error(cpt_ctx* c) {
    uint32_t v = 0;
    HIP_TRY(c, hipMemcpy(&v, c->d_work + 4, sizeof(v), hipMemcpyDeviceToHost));
    if (v == 0) return CPT_OK;
    HIP_TRY(c, hipMemset(c->d_work + 4, 0, sizeof(v)));
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

int upload_materials(cpt_ctx* c);

int upload_scene(cpt_ctx* c) {
    if (c->lin.size() * sizeof(Node) > (size_t)INT32_MAX)   // the walk's buffer descriptor range
        return fail(c, CPT_ERR_UNSUPPORTED, "scene too large: %zu BVH nodes in all orders (max %zu)", c->lin.size(),
                    (size_t)INT32_MAX / sizeof(Node));
    HIP_TRY(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c, &c->d_nodes, &c->cap_nodes, std::max<size_t>(1, c->lin.size()))) != CPT_OK) return rc;
    if ((rc = ensure(c, &c->d_mats, &c->cap_mats, std::max<size_t>(1, c->mats_h.size()))) != CPT_OK) return rc;
    hipStream_t s = c->stream();
    if (!c->lin.empty())
        HIP_TRY(c, hipMemcpyAsync(c->d_nodes, c->lin.data(), c->lin.size() * sizeof(Node), hipMemcpyHostToDevice, s));
    if (!c->refit_plan.empty()) {   // the device refit's plan and the boxes as built
        if ((rc = ensure(c, &c->d_refit_plan, &c->cap_refit_plan, c->refit_plan.size())) != CPT_OK) return rc;
        if ((rc = ensure(c, &c->d_refit_boxes, &c->cap_refit_boxes, c->refit_boxes.size())) != CPT_OK) return rc;
        HIP_TRY(c, hipMemcpyAsync(c->d_refit_plan, c->refit_plan.data(), c->refit_plan.size() * sizeof(cpt::RefitNode),
                                  hipMemcpyHostToDevice, s));
        HIP_TRY(c, hipMemcpyAsync(c->d_refit_boxes, c->refit_boxes.data(), c->refit_boxes.size() * sizeof(cpt::Box6),
                                  hipMemcpyHostToDevice, s));
    }
    if ((rc = upload_materials(c)) != CPT_OK) return rc;
    HIP_TRY(c, hipStreamSynchronize(s));
    c->scene_set = true;
    return CPT_OK;
}

// The deduplicated materials (and the descriptors of the textures they use), completed on the
// device by k_prepare_materials.
int upload_materials(cpt_ctx* c) {
    int rc;
    hipStream_t s = c->stream();
    if (!c->mats_h.empty()) {
        // textured materials: resolve their handles against the bound textures
        std::vector<int32_t> tex_of_mat(c->mats_h.size(), -1);
        bool any = false;
        for (size_t i = 0; i < c->mats_h.size(); ++i) {
            if (!c->mat_have_tex[i]) continue;
            for (size_t t = 0; t < c->textures.size(); ++t)
                if (c->textures[t].handle == c->mat_tex[i]) tex_of_mat[i] = (int32_t)t;
            if (tex_of_mat[i] < 0)
                return fail(c, CPT_ERR_INVALID_ARG, "textured material uses handle %llu, which is not bound (cpt_bind_texture)",
                            (unsigned long long)c->mat_tex[i]);
            any = true;
        }
        if (any) {
            std::vector<TexDesc> descs(c->textures.size());
            for (size_t t = 0; t < descs.size(); ++t) {
                const auto& x = c->textures[t];
                descs[t] = TexDesc{x.d_texels, x.w, x.h, x.cols, x.addr, x.filter, 0};
            }
            if ((rc = ensure(c, &c->d_texdescs, &c->cap_texdescs, descs.size())) != CPT_OK) return rc;
            if ((rc = ensure(c, &c->d_tex_of_mat, &c->cap_tex_of_mat, tex_of_mat.size())) != CPT_OK) return rc;
            HIP_TRY(c, hipMemcpyAsync(c->d_texdescs, descs.data(), descs.size() * sizeof(TexDesc), hipMemcpyHostToDevice, s));
            HIP_TRY(c, hipMemcpyAsync(c->d_tex_of_mat, tex_of_mat.data(), tex_of_mat.size() * sizeof(int32_t),
                                      hipMemcpyHostToDevice, s));
            // the staging vectors must outlive the async copies
            HIP_TRY(c, hipStreamSynchronize(s));
        }
        HIP_TRY(c, hipMemcpyAsync(c->d_mats, c->mats_h.data(), c->mats_h.size() * sizeof(Mat), hipMemcpyHostToDevice, s));
        HIP_TRY(c, cpt::launch_prepare_materials(c->d_mats, any ? c->d_tex_of_mat : nullptr, any ? c->d_texdescs : nullptr,
                                                 (int)c->mats_h.size(), s));
    }
    return CPT_OK;
}

// SceneBVH::UpdateObject for a batch, on the device (cpt_kernels.hip k_refit_*): the updated
// objects are already in c->objs (and the host's reference tree is refit, for
// cpt_scene_bvh_export).  The host names the updated leaves and the union of their ancestors in
// both trees, height by height -- O(updates x depth), independent of the scene size -- and the
// device rewrites every copy: the reference order, the eight octant orders, the 4-wide image and
// leaf array.  Same topology as built (the reference never rebuilds either); the walk tree keeps
// its SAH structure, so the ordered walk stays exact (any tree of conservative boxes is) while
// its efficiency may drift after large motions (cpt_update_objects_rebuild re-optimises).
int device_refit(cpt_ctx* c, int n, const int* indices, bool mats_changed) {
    std::vector<int> uniq(indices, indices + n);
    std::sort(uniq.begin(), uniq.end());
    uniq.erase(std::unique(uniq.begin(), uniq.end()), uniq.end());
    const int nr = c->refit_n_ref;
    std::vector<cpt::RefitLeaf> recs(uniq.size());
    std::vector<int32_t> dirty;
    std::vector<uint8_t>& mark = c->refit_mark;
    mark.resize(c->refit_plan.size(), 0);
    for (size_t k = 0; k < uniq.size(); ++k) {
        const int o = uniq[k];
        cpt::RefitLeaf& r = recs[k];
        r.ref_id = c->bvh.leaf_of_object[o];
        r.walk_id = c->refit_walk_leaf[o];
        r.prim = make_node(c->bvh.nodes[r.ref_id], c->objs, c->mat_of_obj);
        const F3 lo = aabb_min(c->objs[o]), hi = aabb_max(c->objs[o]);
        r.box = cpt::Box6{{lo.x, lo.y, lo.z}, {hi.x, hi.y, hi.z}};
        for (int id : {r.ref_id, r.walk_id})
            for (int p = id < 0 ? -1 : c->refit_parent[id]; p >= 0 && !mark[p]; p = c->refit_parent[p]) {
                mark[p] = 1;
                dirty.push_back(p);
            }
    }
    for (int32_t d : dirty) mark[d] = 0;
    std::stable_sort(dirty.begin(), dirty.end(),
                     [&](int32_t a, int32_t b) { return c->refit_height[a] < c->refit_height[b]; });
    std::vector<int32_t> level_end;
    for (size_t i = 0; i < dirty.size(); ++i)
        if (i + 1 == dirty.size() || c->refit_height[dirty[i + 1]] != c->refit_height[dirty[i]])
            level_end.push_back((int32_t)(i + 1));
    const size_t rec_bytes = recs.size() * sizeof(cpt::RefitLeaf);
    std::vector<uint8_t> work(rec_bytes + dirty.size() * sizeof(int32_t));
    std::memcpy(work.data(), recs.data(), rec_bytes);
    if (!dirty.empty()) std::memcpy(work.data() + rec_bytes, dirty.data(), dirty.size() * sizeof(int32_t));
    HIP_TRY(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c, &c->d_refit_work, &c->cap_refit_work, work.size())) != CPT_OK) return rc;
    uint8_t* const d_work = c->d_refit_work;
    hipStream_t s = c->stream();
    HIP_TRY(c, hipMemcpyAsync(d_work, work.data(), work.size(), hipMemcpyHostToDevice, s));
    const size_t image_base = (size_t)c->n_bvh + 8 * (size_t)c->n_walk;
    uint32_t* image = c->n_wide > 0 ? reinterpret_cast<uint32_t*>(c->d_nodes + image_base) : nullptr;
    Node* leaves = c->n_wide > 0 ? c->d_nodes + image_base + ((size_t)c->n_wide * 7 + 1) / 2 : nullptr;
    HIP_TRY(c, cpt::launch_refit(reinterpret_cast<const cpt::RefitLeaf*>(d_work), (int)recs.size(),
                                 reinterpret_cast<const int32_t*>(d_work + rec_bytes), level_end.data(),
                                 (int)level_end.size(), nr, c->d_refit_plan, c->d_refit_boxes, c->d_nodes, image, leaves,
                                 s));
    if (mats_changed && (rc = upload_materials(c)) != CPT_OK) return rc;
    // the staging vector must outlive the copy; the render after an update sees the new scene
    return sync_checked(c);
}

}  // namespace

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
    (void)hipFree(c->d_gather_map);
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

int cpt_set_scene(cpt_ctx* c, const cpt_object* objs, int n) {
    if (!c || n < 0 || (n > 0 && !objs)) return c ? fail(c, CPT_ERR_INVALID_ARG, "cpt_set_scene: bad arguments") : CPT_ERR_INVALID_ARG;
    c->scene_set = false;   // until the new scene is uploaded
    try {
        c->objs.assign(objs, objs + n);
        build_host_bvh(c->bvh, c->objs);
        // Objects carry their Material by value (bvh.cu:43); identical materials share one slot.
        c->mats_h.clear();
        c->mat_have_tex.clear();
        c->mat_tex.clear();
        c->mat_of_obj.assign(n, 0);
        for (int i = 0; i < n; ++i) c->mat_of_obj[i] = material_slot(c, c->objs[i].material);
        linearise_all(c);
    } catch (const std::bad_alloc&) {
        return fail(c, CPT_ERR_OUT_OF_MEMORY, "cpt_set_scene: host allocation failed");
    }
    return upload_scene(c);
}

// SceneBVH::UpdateObject (bvh.cu:122-157): replace the leaf's object, refit the ancestors
// (MIN/MAX of the two children per axis), re-upload.
static int update_objects(cpt_ctx* c, int n, const int* indices, const cpt_object* objs, bool rebuild) {
    if (!c || n < 0 || (n > 0 && (!indices || !objs))) return CPT_ERR_INVALID_ARG;
    if (!c->scene_set) return fail(c, CPT_ERR_STATE, "cpt_update_objects: cpt_set_scene first");
    for (int k = 0; k < n; ++k)
        if (indices[k] < 0 || indices[k] >= (int)c->objs.size())
            return fail(c, CPT_ERR_INVALID_ARG, "cpt_update_objects: index %d out of range", indices[k]);
    if (n == 0) return CPT_OK;
    const auto t0 = std::chrono::steady_clock::now();
    // a primitive becoming or ceasing to be a platform changes the walk tree's leaf set: rebuild
    for (int k = 0; k < n && !rebuild; ++k)
        if ((c->objs[indices[k]].type == CPT_PRIM_PLATFORM) != (objs[k].type == CPT_PRIM_PLATFORM)) rebuild = true;
    if (c->refit_plan.empty()) rebuild = true;
    const size_t n_mats = c->mats_h.size();
    // SceneBVH::UpdateObject (bvh.cu:144-157) on the host's reference tree (cpt_scene_bvh_export
    // reads it): the leaf takes the object, its ancestors' boxes become the union of their
    // children's.  The refit is a function of the leaves only, so the device copies are refit
    // once per batch below (device_refit), or rebuilt and uploaded once.
    for (int k = 0; k < n; ++k) {
        const int index = indices[k];
        c->objs[index] = objs[k];
        c->mat_of_obj[index] = material_slot(c, objs[k].material);
        int ni = c->bvh.leaf_of_object[index];
        while (ni != -1) {
            BNode& nd = c->bvh.nodes[ni];
            if (nd.is_object) {
                nd.bmax = aabb_max(c->objs[nd.obj]);
                nd.bmin = aabb_min(c->objs[nd.obj]);
            } else {
                const BNode& L = c->bvh.nodes[nd.left];
                const BNode& R = c->bvh.nodes[nd.right];
                nd.bmax = F3{MAX_(L.bmax.x, R.bmax.x), MAX_(L.bmax.y, R.bmax.y), MAX_(L.bmax.z, R.bmax.z)};
                nd.bmin = F3{MIN_(L.bmin.x, R.bmin.x), MIN_(L.bmin.y, R.bmin.y), MIN_(L.bmin.z, R.bmin.z)};
            }
            ni = nd.parent;
        }
    }
    int rc;
    if (rebuild) {
        // the reference tree keeps its topology (refit above); the walk tree is rebuilt from the
        // current objects, then all nine orders are re-linearised and uploaded
        linearise_all(c);
        rc = upload_scene(c);
    } else {
        rc = device_refit(c, n, indices, c->mats_h.size() != n_mats);
    }
    c->last_update_ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return rc;
}

int cpt_update_objects(cpt_ctx* c, int n, const int* indices, const cpt_object* objs) {
    return update_objects(c, n, indices, objs, false);
}

int cpt_update_objects_rebuild(cpt_ctx* c, int n, const int* indices, const cpt_object* objs) {
    return update_objects(c, n, indices, objs, true);
}

int cpt_last_update_ms(cpt_ctx* c, float* ms) {
    if (!c || !ms) return CPT_ERR_INVALID_ARG;
    *ms = c->last_update_ms;
    return CPT_OK;
}

int cpt_update_object(cpt_ctx* c, int index, const cpt_object* obj) {
    if (!c || !obj) return CPT_ERR_INVALID_ARG;
    return cpt_update_objects(c, 1, &index, obj);
}

int cpt_scene_bvh_export(cpt_ctx* c, float* boxes, int32_t* links, int capacity, int* n_nodes) {
    if (!c || !n_nodes) return CPT_ERR_INVALID_ARG;
    int m = (int)c->bvh.nodes.size();
    *n_nodes = m;
    for (int i = 0; i < m && i < capacity; ++i) {
        const BNode& n = c->bvh.nodes[i];
        if (boxes) {
            float* b = boxes + 6 * i;
            b[0] = n.bmin.x; b[1] = n.bmin.y; b[2] = n.bmin.z; b[3] = n.bmax.x; b[4] = n.bmax.y; b[5] = n.bmax.z;
        }
        if (links) {
            int32_t* l = links + 4 * i;
            l[0] = n.is_object; l[1] = n.left; l[2] = n.right; l[3] = n.obj;
        }
    }
    return CPT_OK;
}

int cpt_bvh_build_host(const cpt_object* objs, int n, float* boxes, int32_t* links, int capacity, int* n_nodes) {
    if (n < 0 || (n > 0 && !objs) || !n_nodes) return CPT_ERR_INVALID_ARG;
    try {
        std::vector<cpt_object> v(objs, objs + n);
        HostBvh b;
        build_host_bvh(b, v);
        int m = (int)b.nodes.size();
        *n_nodes = m;
        for (int i = 0; i < m && i < capacity; ++i) {
            const BNode& nd = b.nodes[i];
            if (boxes) {
                float* x = boxes + 6 * i;
                x[0] = nd.bmin.x; x[1] = nd.bmin.y; x[2] = nd.bmin.z; x[3] = nd.bmax.x; x[4] = nd.bmax.y; x[5] = nd.bmax.z;
            }
            if (links) {
                int32_t* l = links + 4 * i;
                l[0] = nd.is_object; l[1] = nd.left; l[2] = nd.right; l[3] = nd.obj;
            }
        }
    } catch (const std::bad_alloc&) {
        return CPT_ERR_OUT_OF_MEMORY;
    }
    return CPT_OK;
}

int cpt_set_env_texture(cpt_ctx* c, const uint8_t* rgba, int logical_width, int height, int valid_cols) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (logical_width <= 0 || height <= 0 || valid_cols < 0 || valid_cols > logical_width || (valid_cols > 0 && !rgba))
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_set_env_texture: bad geometry %dx%d cols %d", logical_width, height, valid_cols);
    HIP_TRY(c, hipSetDevice(c->device));
    size_t n = (size_t)valid_cols * height;
    int rc = ensure(c, &c->d_env, &c->cap_env, std::max<size_t>(1, n));
    if (rc != CPT_OK) return rc;
    if (n) HIP_TRY(c, hipMemcpy(c->d_env, rgba, n * 4, hipMemcpyHostToDevice));
    c->env_w = logical_width;
    c->env_h = height;
    c->env_cols = valid_cols;
    return CPT_OK;
}

int cpt_bind_texture(cpt_ctx* c, uint64_t handle, const uint8_t* rgba, int logical_width, int height, int valid_cols,
                     int address_mode, int filter_mode) {
    if (!c) return CPT_ERR_INVALID_ARG;
    if (logical_width <= 0 || height <= 0 || valid_cols < 0 || valid_cols > logical_width || (valid_cols > 0 && !rgba) ||
        address_mode < CPT_ADDRESS_WRAP || address_mode > CPT_ADDRESS_BORDER || filter_mode < CPT_FILTER_POINT ||
        filter_mode > CPT_FILTER_LINEAR)
        return fail(c, CPT_ERR_INVALID_ARG, "cpt_bind_texture: bad geometry %dx%d cols %d or mode %d/%d", logical_width,
                    height, valid_cols, address_mode, filter_mode);
    HIP_TRY(c, hipSetDevice(c->device));
    const size_t n = (size_t)valid_cols * height;
    uint32_t* d = nullptr;
    HIP_TRY(c, hipMalloc((void**)&d, std::max<size_t>(1, n) * 4));
    if (n) {
        hipError_t e = hipMemcpy(d, rgba, n * 4, hipMemcpyHostToDevice);
        if (e != hipSuccess) { (void)hipFree(d); return fail(c, CPT_ERR_HIP, "cpt_bind_texture: %s", hipGetErrorString(e)); }
    }
    cpt_ctx::Texture t{handle, d, logical_width, height, valid_cols, address_mode, filter_mode};
    bool replaced = false;
    for (auto& x : c->textures)
        if (x.handle == handle) { (void)hipFree(x.d_texels); x = t; replaced = true; }
    if (!replaced) c->textures.push_back(t);
    return c->scene_set ? upload_scene(c) : CPT_OK;   // re-prepare the materials
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
    return CPT_OK;
}

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
        if ((flags & CPT_SCHEDULE_COST) && spp > 0 && c->n_rows > 0) {
            // pilot: 1 pass per 512 (1..4), then the tiles sorted heaviest first
            const int passes = std::min(4, std::max(1, spp / 512));
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
        // default for frames of at most 4 pixels per lane and chains of at least 512 passes:
        // with more pixels the tail is a small part of the render, with short chains the
        // hand-overs do not pay, and the plain kernel's tighter code wins (DESIGN.md §Multi-GPU;
        // C2 at 0.9 pixels per lane and 256 spp: 23.2 vs 21.9 Gpaths/s without).
        int cus = 0;
        HIP_TRY(c, hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device));
        cus = std::max(cus, 1);
        const bool cons = (flags & CPT_SCHEDULE_CONSOLIDATE) ||
                          (!(flags & CPT_SCHEDULE_NO_CONSOLIDATE) && spp >= 512 &&
                           (size_t)c->n_rows * c->width <= 4u * 1024u * (size_t)cus);
        if (cons && spp > 1) {
            const size_t cap = 3u * 256u * (size_t)cus;
            int rc;
            if ((rc = ensure(c, &c->d_resume, &c->cap_resume, 5 * cap)) != CPT_OK) return rc;
            p.resume = c->d_resume;
            p.resume_cap = cap;
        }
        HIP_TRY(c, hipEventRecord(c->ev_main, s));
        HIP_TRY(c, cpt::launch_megakernel(p, (flags & CPT_RENDER_STATS) != 0, aux, s));
    }
    HIP_TRY(c, hipEventRecord(c->ev_stop, s));
    c->have_timing = true;
    if (flags & CPT_RENDER_SYNC) return sync_checked(c);
    return CPT_OK;
}

// Row-tile gather: the rows `src` rendered, placed into `dst`'s frame at the
// same global rows.  One peer copy of src's buffers to dst's device (hipMemcpyPeerAsync: xGMI
// between two MI355X, a plain device copy when both contexts share a GPU), then one stitch
// kernel on dst's stream.  Waits for src; asynchronous with respect to dst.
int cpt_gather_rows(cpt_ctx* dst, cpt_ctx* src) {
    if (!dst || !src || dst == src) return dst ? fail(dst, CPT_ERR_INVALID_ARG, "cpt_gather_rows: bad contexts") : CPT_ERR_INVALID_ARG;
    if (!dst->frame_set || !src->frame_set) return fail(dst, CPT_ERR_STATE, "cpt_gather_rows: both contexts need a frame");
    if (dst->width != src->width || dst->height != src->height)
        return fail(dst, CPT_ERR_INVALID_ARG, "cpt_gather_rows: frame %dx%d vs %dx%d", dst->width, dst->height, src->width,
                    src->height);
    std::vector<int32_t> at(dst->height, -1);   // dst row index of each global row (first occurrence)
    for (int j = dst->n_rows - 1; j >= 0; --j) at[dst->rows_h[j]] = j;
    dst->gather_map_h.resize(src->n_rows);
    for (int i = 0; i < src->n_rows; ++i) {
        const int32_t j = at[src->rows_h[i]];
        if (j < 0) return fail(dst, CPT_ERR_INVALID_ARG, "cpt_gather_rows: row %d is not in the destination frame", src->rows_h[i]);
        dst->gather_map_h[i] = j;
    }
    if (src->n_rows == 0) return CPT_OK;
    if (int rc = sync_checked(src)) return fail(dst, rc, "cpt_gather_rows: source: %s", src->err.c_str());
    const size_t npix = (size_t)src->n_rows * src->width;
    const bool aux = src->d_normal && src->d_depth;
    HIP_TRY(dst, hipSetDevice(dst->device));
    hipStream_t s = dst->stream();
    const size_t dst_npix = (size_t)dst->n_rows * dst->width;
    if (aux) {
        if (!dst->d_normal) HIP_TRY(dst, hipMalloc((void**)&dst->d_normal, dst_npix * 3 * sizeof(float)));
        if (!dst->d_depth) HIP_TRY(dst, hipMalloc((void**)&dst->d_depth, dst_npix * sizeof(float)));
    }
    int rc;
    // staging: accumulator (npix float4), then normals (3 npix floats) and depths (npix floats)
    if ((rc = ensure(dst, &dst->d_gather, &dst->cap_gather, aux ? 2 * npix : npix)) != CPT_OK) return rc;
    if ((rc = ensure(dst, &dst->d_gather_map, &dst->cap_gather_map, (size_t)src->n_rows)) != CPT_OK) return rc;
    float* st_nrm = reinterpret_cast<float*>(dst->d_gather + npix);
    float* st_dep = st_nrm + 3 * npix;
    HIP_TRY(dst, hipMemcpyAsync(dst->d_gather_map, dst->gather_map_h.data(), src->n_rows * sizeof(int32_t),
                                hipMemcpyHostToDevice, s));
    HIP_TRY(dst, hipMemcpyPeerAsync(dst->d_gather, dst->device, src->d_accum, src->device, npix * sizeof(float4), s));
    if (aux) {
        HIP_TRY(dst, hipMemcpyPeerAsync(st_nrm, dst->device, src->d_normal, src->device, npix * 3 * sizeof(float), s));
        HIP_TRY(dst, hipMemcpyPeerAsync(st_dep, dst->device, src->d_depth, src->device, npix * sizeof(float), s));
    }
    HIP_TRY(dst, cpt::launch_stitch_rows(dst->d_gather, aux ? st_nrm : nullptr, aux ? st_dep : nullptr, dst->d_gather_map,
                                         dst->width, src->n_rows, dst->d_accum, dst->d_normal, dst->d_depth, s));
    // the host row map is read by the async upload: keep it until the stream passes the copy
    HIP_TRY(dst, hipStreamSynchronize(s));
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

int cpt_copy_accum_device(cpt_ctx* c, void* dst, size_t bytes) {
    if (!c || (!dst && bytes)) return CPT_ERR_INVALID_ARG;
    size_t have = (size_t)c->n_rows * c->width * sizeof(float4);
    if (bytes > have) return fail(c, CPT_ERR_INVALID_ARG, "cpt_copy_accum_device: %zu > %zu bytes", bytes, have);
    HIP_TRY(c, hipSetDevice(c->device));
    if (bytes) HIP_TRY(c, hipMemcpyAsync(dst, c->d_accum, bytes, hipMemcpyDeviceToDevice, c->stream()));
    return CPT_OK;
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
    HIP_TRY(c, cpt::launch_denoise_mix(c->d_accum, c->d_normal, c->d_depth, c->d_mix, c->d_bgra, c->width, c->height,
                                      row0, y0, y1, cur_sample_idx, s));
    if (bgra_host) {
        HIP_TRY(c, hipMemcpyAsync(bgra_host, c->d_bgra, cap_rows * c->width * 4, hipMemcpyDeviceToHost, s));
        HIP_TRY(c, hipStreamSynchronize(s));
    }
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

int cpt_denoise_mix_band(cpt_ctx* c, uint32_t cur_sample_idx, int y0, int y1, uint8_t* bgra_host) {
    if (!c) return CPT_ERR_INVALID_ARG;
    return denoise_band(c, cur_sample_idx, y0, y1, bgra_host, 0);
}

int cpt_copy_bgra_device(cpt_ctx* c, void* device_dst, size_t bytes) {
    if (!c || !device_dst) return CPT_ERR_INVALID_ARG;
    if (!c->d_bgra) return fail(c, CPT_ERR_STATE, "cpt_copy_bgra_device: no display frame yet");
    const size_t have = (size_t)(c->band_y1 - c->band_y0) * c->width * 4;
    if (bytes > have) return fail(c, CPT_ERR_INVALID_ARG, "cpt_copy_bgra_device: %zu bytes requested, band holds %zu", bytes, have);
    HIP_TRY(c, hipSetDevice(c->device));
    HIP_TRY(c, hipMemcpyAsync(device_dst, c->d_bgra, bytes, hipMemcpyDeviceToDevice, c->stream()));
    return CPT_OK;
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

int cpt_selftest_qdiv(cpt_ctx* c, int which, uint64_t n, uint64_t seed, uint64_t* out, int out_len) {
    if (!c || !out || out_len < 1 || which < 0 || which > 5) return CPT_ERR_INVALID_ARG;
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
