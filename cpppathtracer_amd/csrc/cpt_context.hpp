// cpt_context.hpp — the C-ABI's context (struct cpt_ctx of include/cpt.h) and the helpers its
// implementation files share: cpt_capi.cpp (context, frame, RNG, render, gather, display) and
// cpt_scene.cpp (scene upload, material slots, walk trees, device refit).  Host code only.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

#include "../../include/cpt.h"
#include "cpt_host.hpp"
#include "cpt_internal.hpp"

using cpt::Mat;
using cpt::Node;
using cpt::TexDesc;
using cpt::host::HostBvh;

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
    hipEvent_t ev_dn0 = nullptr, ev_dn1 = nullptr;   // around the last display kernel (k_denoise_rows)
    bool have_dn_timing = false;
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
    // CPT_SCHEDULE_PREVIOUS: the Weyl plane after the last such render, and the tile order
    // its draws gave (the next render's dequeue order)
    uint32_t* d_prev_d = nullptr;
    uint32_t* d_prev_order = nullptr;
    bool prev_d_valid = false, prev_order_valid = false;
    int prev_since_order = 0;   // renders since the CPT_SCHEDULE_PREVIOUS order was rebuilt
    uint4* d_resume = nullptr;          // tail consolidation: handed-over chains (5 x uint4 each)
    size_t cap_resume = 0;
    cpt::WfState wf{};           // wavefront path state (allocated on first use)
    bool wf_ready = false;
    float* d_mix = nullptr;      // display running mean (Mix), rgb per pixel of the display band
    uint8_t* d_bgra = nullptr;   // display frame (band rows)
    float4* d_dn_sink = nullptr; // k_denoise_strip: where lanes without an output pixel store (DN_SINK_SLOTS)
    int band_y0 = -1, band_y1 = -1;   // display band the buffers hold
    float last_kernel_ms = 0.f;
    int last_launches = 0;
    // row-tile gather (cpt_gather_rows): per source context, the frame row each of its rows goes
    // to (a device buffer, rebuilt when either frame changes); a source's rows staged on this
    // device when the pair has no peer path
    struct GatherMap {
        const cpt_ctx* src = nullptr;
        uint64_t src_gen = 0, dst_gen = 0;
        int src_device = -1;
        bool peer = false;
        int mode = -1;   // last gather: CPT_GATHER_SAME_DEVICE / _PEER / _STAGED
        int32_t* d_map = nullptr;
    };
    std::vector<GatherMap> gather_maps;
    float4* d_gather = nullptr;
    size_t cap_gather = 0;
    uint64_t frame_gen = 0;           // process-unique id of the current frame layout (cpt_set_frame)
    hipEvent_t ev_ready = nullptr;    // a gather's source: its queued work
    hipEvent_t ev_gathered = nullptr; // a gather's destination: the stitch done
    hipEvent_t ev_caller = nullptr;   // a device copy's caller stream: its queued work
    hipEvent_t ev_copied = nullptr;   // a device copy: done on the context's stream
    // consolidation test hooks (cpt_set_debug_consolidation)
    uint32_t dbg = 0;
    bool force_staged_gather = false;   // gather test hook (cpt_set_debug_gather)
    int keeper_spin_log2 = 0, publish_wait_log2 = 0;

    hipStream_t stream() const { return user_stream ? user_stream : own_stream; }
};

namespace cpt {
namespace ctx {

// Records a formatted message on the context (or, without one, for cpt_last_error(NULL)) and
// returns `code`.
int fail(cpt_ctx* c, int code, const char* fmt, ...);

#define HIP_TRY(ctx, expr)                                                                             \
    do {                                                                                               \
        hipError_t e_ = (expr);                                                                        \
        if (e_ != hipSuccess)                                                                          \
            return fail((ctx), e_ == hipErrorOutOfMemory ? CPT_ERR_OUT_OF_MEMORY : CPT_ERR_HIP,        \
                        "%s: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);           \
    } while (0)

template <typename T>
inline int ensure(cpt_ctx* c, T** ptr, size_t* cap, size_t count) {
    if (*ptr && *cap >= count) return CPT_OK;
    if (*ptr) { (void)hipFree(*ptr); *ptr = nullptr; *cap = 0; }
    if (count == 0) return CPT_OK;
    HIP_TRY(c, hipMalloc((void**)ptr, count * sizeof(T)));
    *cap = count;
    return CPT_OK;
}

void free_frame(cpt_ctx* c);
// Drain the context's stream, then report a device-side error of the work it ran.
int check_device_error(cpt_ctx* c);
int sync_checked(cpt_ctx* c);

// cpt_scene.cpp
int material_slot(cpt_ctx* c, const cpt_material& m);
void linearise_all(cpt_ctx* c);
int upload_scene(cpt_ctx* c);
int upload_materials(cpt_ctx* c);
int device_refit(cpt_ctx* c, int n, const int* indices, bool mats_changed);

}  // namespace ctx
}  // namespace cpt
