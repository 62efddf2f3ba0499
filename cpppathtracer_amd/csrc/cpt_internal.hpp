// cpt_internal.hpp — shared between the HIP kernels and the C-ABI implementation.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "cpt_device.hpp"

// Per-lane LDS stack entries of the wide walk; the host keeps the binary walk for a tree that
// could need more (cpt_capi.cpp linearise_wide).
#define CPT_WSTACK 32

namespace cpt {

// Wide-tree nodes staged in LDS by the LDS kernels (cpt_path.hpp trace_wide); the host numbers
// a larger tree so that these are its top (cpt_capi.cpp linearise_wide).
constexpr int LDS_TREE_NODES = 512;
__host__ __device__ __forceinline__ int lds_tree_nodes(int n_wide) { return n_wide < LDS_TREE_NODES ? n_wide : LDS_TREE_NODES; }

// Camera snapshot as the kernel needs it (the reference passes the whole MotionalCamera by
// value in PathTracerParams, path_tracer.cu:14-27; only these fields are read by RayGen).
struct CamK {
    float origin[3];
    float u[3], v[3];
    float top_left[3], horizontal[3], vertical[3];
    float lens_radius;
    int width, height;
    double inv_w, inv_h;   // 1.0 / (double)(float)width, height: RayGen's x / width, y / height as
                           // exact quotients (cpt_path.hpp ray_gen)
};

// Kernel arguments (passed by value: they land in the kernarg segment and are read with
// scalar loads).
struct KParams {
    const Node* nodes;      // skip-link orders, leaves inline: the reference order (n_nodes), then
                            // the walk tree's eight octant orders (n_walk each)
    const Mat* mats;        // deduplicated materials, indexed by Node::code >> 2
    int n_nodes, n_walk;
    int n_wide;             // 4-wide walk-tree nodes: their compact image follows the eight octant
                            // orders (0: the ordered walk uses the binary octant orders)
    int n_unb;              // unbounded leaves at the head of every octant order
    int n_leaves;           // the wide tree's leaf array (platforms first), after its compact image
    int ordered;            // CPT_TRAVERSAL_ORDERED: walk the ray's octant order (2: plain leaves)
    const uint32_t* env;    // packed RGBA8, env_cols x env_h
    int env_w, env_h, env_cols;
    CamK cam;
    const int32_t* rows;    // global row index per context row
    int n_rows, width;
    uint32_t* rng;          // planar [6][n_rows*width]
    float4* accum;          // [n_rows*width] rgb sums + pass count
    float* normal;          // [n_rows*width][3] (AUX)
    float* depth;           // [n_rows*width]    (AUX)
    unsigned long long* stats;  // [5]           (STATS)
    uint32_t* work;         // pixel dequeue counter (zeroed before each launch)
    const uint32_t* tile_order;  // megakernel dequeue order of the 8x8 tiles (nullptr: row-major)
    uint32_t* tile_cost;    // pilot launch only: per-tile work (cost schedule)
    int spp, max_depth, accumulate;
    int lanes;              // lanes per wave that take pixels (64; fewer: DIAGNOSTIC CPT_LANES_PER_WAVE)
    int replicate;          // lanes per taken pixel (1; more: DIAGNOSTIC CPT_REPLICATE, identical copies)
    // Tail consolidation (LDS walk only; nullptr: off): slabs of chains handed over at a pass
    // boundary by retiring waves, 5 x uint4 per chain, ho_slots chains per workgroup.
    uint4* resume;
    size_t resume_cap;      // chains (all workgroups)
    // Sticky device error word (CPT_DEVERR_*), or-ed by a kernel that had to abandon work; the
    // host reads and clears it at its next synchronising call (cpt_capi.cpp check_device_error).
    uint32_t* error;
    // Test hooks of the consolidation's error paths (cpt_set_debug_consolidation; 0 in normal
    // use): dbg bit 0 = a phantom live chain in every workgroup (a lost count), bit 1 = hand-overs
    // never publish their slot; the keeper's idle-spin limit and the hand-over wait as log2
    // (0 = the defaults, 2^26 and 2^22).
    uint32_t dbg;
    int keeper_spin_log2, publish_wait_log2;
};

// Device error bits (KParams::error).
enum : uint32_t {
    CPT_DEVERR_KEEPER_TIMEOUT = 1u,    // a keeper wave gave up waiting while chains were live
    CPT_DEVERR_PUBLISH_TIMEOUT = 2u,   // a taken hand-over slot was never published (chain lost)
    CPT_DEVERR_RESUME_CAP = 4u,        // consolidation slab too small for the grid
};

// Cost schedule (cpt_kernels.hip, DESIGN.md §Cost schedule): a `passes`-pass pilot of the
// megakernel sums each 8x8 tile's work, then `order` (one u32 per tile) gets the tiles
// heaviest first.  `scratch` holds tile_schedule_scratch_bytes() bytes.
size_t tile_schedule_scratch_bytes(int width, int n_rows);
// CPT_SCHEDULE_PREVIOUS: each 8x8 tile's RNG draws since `d_prev` (the Weyl plane d of the
// states, planar [5] of p.rng), then d_prev := d; the tiles sorted heaviest first into `order`.
hipError_t launch_tile_order_from_draws(const KParams& p, uint32_t* d_prev, void* scratch, size_t scratch_bytes,
                                        uint32_t* order, hipStream_t stream);
hipError_t launch_tile_schedule(const KParams& p, int passes, void* scratch, size_t scratch_bytes, uint32_t* order,
                                hipStream_t stream);

// Wavefront path state (cpt_wavefront.hip): SoA float4 arrays indexed by QUEUE SLOT + queues.
// The carried state is double-buffered: bounce b reads buffer b & 1 at its queue slot and shade
// writes each surviving path into buffer (b + 1) & 1 at the slot the compaction gave it, so
// every state access is coalesced.  Hit records are per slot of the current bounce.
struct WfState {
    float4 *ray_o[2], *ray_d[2], *att[2], *rad[2], *aux[2];
    float4 *hit_p, *hit_n;
    uint4* rng_a[2];      // a live path's XORWOW state by slot: (v0, v1, v2, v3) ...
    uint2* rng_b[2];      // ... and (v4, d); back in the per-pixel planes when the path ends
    int32_t* queue[2];
    int32_t* ident;       // tile-ordered identity queue (first bounce)
    uint32_t* counts;     // [0], [1]: queue sizes; [3]: ident size
};

// Device refit of cpt_update_objects (SceneBVH::UpdateObject, bvh.cu:122-157, on the GPU).  The
// reference tree's nodes and the walk tree's nodes are numbered together ("refit ids": the
// reference tree's BNodes first, then the walk tree's); each records where its copies live in
// the node buffer.  The topology is fixed until the next cpt_set_scene.
struct RefitNode {
    int32_t left, right;    // children (refit ids); a leaf has left = -1
    int32_t slot;           // 4-wide image slot holding this node's box (wide id * 4 + k), or -1
    int32_t leaf;           // index in the wide tree's leaf array (walk-tree leaves), or -1
    int32_t pos[8];         // node-buffer index of each copy: the reference order (pos[0]) or the
                            // octant orders 0..7 of the walk tree (octant form); -1: none
};
struct Box6 { float lo[3], hi[3]; };
// One updated object: its inline primitive (Node::miss is not written: each copy keeps its own)
// and its box (Object::GetAABBMin/Max), for its leaf in each tree.
struct RefitLeaf {
    Node prim;
    Box6 box;
    int32_t ref_id, walk_id;
};
// The leaves, then the dirty internal nodes height by height (children before parents): one
// launch of k_refit_leaves, one of k_refit_nodes per height.  n_ref: reference-tree ids are
// [0, n_ref); `image` / `leaves` are the wide tree's compact image and leaf array (nullptr: none).
hipError_t launch_refit(const RefitLeaf* leaves_in, int n_leaves, const int32_t* dirty, const int32_t* level_end,
                        int n_levels, int n_ref, const RefitNode* nodes_plan, Box6* boxes, Node* nodes, uint32_t* image,
                        Node* leaves, hipStream_t stream);

hipError_t launch_megakernel(const KParams& p, bool stats, bool aux, hipStream_t stream);
hipError_t launch_wavefront(const KParams& p, WfState& w, bool stats, bool aux, hipStream_t stream, int* launches);
hipError_t wavefront_build_ident(const KParams& p, WfState& w, hipStream_t stream);
hipError_t launch_prepare_materials(Mat* mats, const int32_t* tex_of_mat, const TexDesc* texs, int n,
                                    hipStream_t stream);
hipError_t launch_init_rng(const uint32_t* jumps, const uint32_t seed_state[6], int width, const int32_t* rows,
                           int n_rows, uint32_t* scratch_w, uint32_t* scratch_mats, uint32_t* rng, hipStream_t stream);
hipError_t launch_math_batch(int op, const float* a, const float* b, float* out, size_t n, hipStream_t stream);
hipError_t launch_stream_read(const float4* p, size_t n, float* out, int grid, hipStream_t stream);
hipError_t launch_read_pattern(int bpl, const float* p, size_t n_lanes, float* out, int grid, hipStream_t stream);
hipError_t timeline_read(unsigned long long* out, int n, hipStream_t stream);
hipError_t launch_selftest_qdiv(int which, uint64_t n, uint64_t seed, unsigned long long* out, int out_len,
                                hipStream_t stream);
hipError_t launch_stitch_rows(const float4* src_acc, const float* src_nrm, const float* src_dep, const int32_t* dst_row,
                              int width, int n_rows, float4* acc, float* nrm, float* dep, hipStream_t stream);
// out_host (nullable): the device alias of a pinned host frame, written beside `out`; accum /
// normal / depth hold the context's ctx_rows rows from row0; sink: a
// device buffer of DN_SINK_SLOTS float4s the strip kernel's lanes without an output pixel store to
constexpr int DN_SINK_SLOTS = 1024 * 64;
hipError_t launch_denoise_mix(const float4* accum, const float* normal, const float* depth, float* mix, uint8_t* out,
                              uint8_t* out_host, float4* sink, int width, int height, int row0, int ctx_rows, int y0, int y1,
                              uint32_t cur_sample_idx, hipStream_t stream);

}  // namespace cpt
