/*
 * cpt.h — C-ABI of the MI355X path-tracing integrator (libcpt.so).
 *
 * This is the drop-in boundary for the reference's hot path (DearPoca/CppPathTracer,
 * cuSrc/path_tracer.cu:124-175 `SamplePixel` and everything it reaches).  Plain C types
 * only: no HIP, CUDA or torch types cross it.  Every function returns an int status
 * (0 = CPT_OK); no exception crosses the ABI.  The reference logs CUDA errors and
 * continues (path_tracer.cu:54-57, 279-283); here the status is returned and the message
 * is kept in cpt_last_error().
 *
 * Which reference interface each entry point replaces (file:line under the reference):
 *
 *   cpt_create / cpt_destroy        PathTracer construction + InitBuffers' cudaMallocs
 *                                   (path_tracer.cu:44-115); the reference never frees.
 *   cpt_set_scene                   SceneBVH::AddObject + BuildBVH + BuildBVHInGpu
 *                                   (bvh.cu:22-29, 116-120, 97-114), reached from
 *                                   PathTracer::AddObject / InitPipeline (path_tracer.cu:29-34, 308-314).
 *   cpt_update_object(s)            SceneBVH::UpdateObject (bvh.cu:144-157).
 *   cpt_set_env_texture             PocaTextureUtils::AddTexByFile (textures.cu:14-62) +
 *                                   the sky load in InitBuffers (path_tracer.cu:47).
 *   cpt_bind_texture                AddTexByFile for a material texture: the handle the app
 *                                   stores in Material::tex_ (material.h:21-25), sampled by
 *                                   Material::GetKd (material.cu:11-18).
 *   cpt_set_frame                   InitBuffers' per-pixel buffers (path_tracer.cu:44-115),
 *                                   plus a row window/list for multi-GPU row tiling.
 *   cpt_init_rng                    InitCuRand kernel (path_tracer.cu:36-42, 99-107).
 *   cpt_camera_get_copy             MotionalCamera::GetCopy (motional_camera.cu:177-200).
 *   cpt_render                      The SamplePixel launch in PipelineLoop
 *                                   (path_tracer.cu:264-283), `spp` passes at once.
 *   cpt_read_accum / cpt_read_aux   The per-pixel render_target / normal / depth buffers
 *                                   written by SamplePixel (path_tracer.cu:172-174).
 *   cpt_denoise_mix                 Denoising + Mix + BGRA8 readback (path_tracer.cu:177-254,
 *                                   285-303).
 *   cpt_denoise_mix_band            The same for one row band of a multi-GPU display (the
 *                                   Denoising/Mix launch restricted to rows y0..y1-1; the
 *                                   band's renderer also renders a 3-row halo).
 */
#ifndef CPT_H_
#define CPT_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CPT_ABI_VERSION 1

enum cpt_status {
    CPT_OK = 0,
    CPT_ERR_INVALID_ARG = 1,
    CPT_ERR_NO_DEVICE = 2,
    CPT_ERR_HIP = 3,
    CPT_ERR_OUT_OF_MEMORY = 4,
    CPT_ERR_STATE = 5,       /* e.g. render before scene/frame/rng were set */
    CPT_ERR_UNSUPPORTED = 6,
    /* A kernel had to abandon work (e.g. a tail-consolidation hand-over timed out, so some
     * pixels were not finished); reported by the next synchronising call on the context
     * (cpt_synchronize, cpt_read_accum, cpt_read_rng, cpt_render with CPT_RENDER_SYNC, ...),
     * like the reference's logged CUDA errors (path_tracer.cu:279-283).  Sticky until read. */
    CPT_ERR_DEVICE = 7
};

/* PrimitiveType::Enum (object.h:7-15) and MaterialType::Enum (material.h:5-15). */
enum cpt_primitive_type { CPT_PRIM_SPHERE = 0, CPT_PRIM_PLATFORM = 1, CPT_PRIM_CYLINDER = 2 };
enum cpt_material_type {
    CPT_MAT_DIFFUSE = 0,
    CPT_MAT_METAL = 1,   /* shaded by MirrorHitShader (material.cu:151-153 swap, kept) */
    CPT_MAT_MIRROR = 2,  /* shaded by MetalHitShader  (material.cu:154-156 swap, kept) */
    CPT_MAT_GLASS = 3,
    CPT_MAT_TEST = 4     /* falls through to Diffuse (material.cu:160-161) */
};

/* Layout-identical to CUDA float3 (12 bytes, 4-byte aligned). */
typedef struct cpt_float3 { float x, y, z; } cpt_float3;

/* Material (material.h:17-35), 40 bytes. */
typedef struct cpt_material {
    int32_t type;              /* @0  cpt_material_type */
    uint8_t have_tex;          /* @4  nonzero: kd = the texture bound to u.tex (cpt_bind_texture) */
    uint8_t pad_[3];
    union {                    /* @8  union { float3 kd_; cudaTextureObject_t tex_; } */
        cpt_float3 kd;
        uint64_t tex;
    } u;
    float refractive_index;    /* @24 */
    float emit_intensity;      /* @28 */
    float smoothness;          /* @32 */
    float reflectivity;        /* @36 */
} cpt_material;

/* Object (object.h:17-32), 72 bytes. */
typedef struct cpt_object {
    int32_t type;              /* @0  cpt_primitive_type */
    int32_t pad_;
    cpt_material material;     /* @8  */
    cpt_float3 center;         /* @48 */
    float radius;              /* @60 sphere, cylinder */
    float y_pos;               /* @64 platform */
    float height;              /* @68 cylinder */
} cpt_object;

/* MotionalCamera (motional_camera.h:8-24), 136 bytes.  u/v/w/top_left/horizontal/vertical
 * are the GetCopy() outputs; cpt_camera_get_copy() fills them. */
typedef struct cpt_camera {
    cpt_float3 vup;            /* @0   */
    int32_t width, height;     /* @12, @16 */
    uint32_t cur_sample_idx;   /* @20  */
    cpt_float3 origin;         /* @24  */
    cpt_float3 look_at;        /* @36  */
    float view_fov;            /* @48  degrees */
    float dist_to_focus;       /* @52  */
    float lens_radius;         /* @56  */
    float move_speed;          /* @60  */
    cpt_float3 u, v, w;        /* @64, @76, @88 */
    cpt_float3 top_left_corner;/* @100 */
    cpt_float3 horizontal;     /* @112 */
    cpt_float3 vertical;       /* @124 */
} cpt_camera;

/* Per-render counters for the algorithmic byte model. */
typedef struct cpt_stats {
    uint64_t segments;     /* TraceRay calls                          */
    uint64_t node_visits;  /* non-sentinel nodes popped (bvh.cu:173)  */
    uint64_t prim_tests;   /* IntersectionTest calls (bvh.cu:176)     */
    uint64_t hits;
    uint64_t misses;
} cpt_stats;

typedef struct cpt_ctx cpt_ctx;

/* cpt_render flags */
#define CPT_RENDER_ACCUMULATE 0x1u   /* add into the accumulator instead of overwriting it   */
#define CPT_RENDER_AUX        0x2u   /* write first-hit normal + depth of the last pass       */
#define CPT_RENDER_STATS      0x4u   /* count segments/nodes/prims/hits/misses (slower)       */
#define CPT_RENDER_SYNC       0x8u   /* block until the render finished                        */
#define CPT_PATH_MEGAKERNEL   0x000u /* per-lane path regeneration megakernel (default)        */
#define CPT_PATH_WAVEFRONT    0x100u /* SoA wavefront: extend / shade / compact per bounce      */
/* Near-first BVH walk: each ray walks the node order of its direction octant (near child of
 * every split first), and equal distances go to the primitive the reference order meets
 * first.  It finds the same closest hit as the reference's right-first DFS
 * (bvh.cu:167-205) unless a primitive's computed hit distance lies outside its own box's
 * computed slab interval by rounding (DESIGN.md §Ordered walk).  Node/prim counts
 * (CPT_RENDER_STATS) are then this walk's counts, not the reference's. */
#define CPT_TRAVERSAL_ORDERED 0x200u
/* With CPT_TRAVERSAL_ORDERED: test each leaf where the walk meets it.  By default the ordered
 * walk parks a leaf and runs the parked leaves of a wave together (DESIGN.md §Ordered walk,
 * parked leaves); the closest hits are the same, but the node/prim counts then depend on which rays
 * share a wave.  This flag makes them a per-ray property (the oracle's diagnostic walk). */
#define CPT_TRAVERSAL_PLAIN_LEAVES 0x400u
/* Megakernel pixel schedule: a short pilot render (1..4 passes from the current RNG states,
 * nothing written back) measures each 8x8 tile's work, and the render then dequeues the tiles
 * heaviest first (longest processing time first).  Results are identical to the row-major
 * tile order (a pixel's stream depends only on (seed, x, y)); the heaviest pixel chains start
 * at once, which shortens the tail when the image has few pixels per lane (row tiles on many
 * GPUs, DESIGN.md §Cost schedule).  Ignored by CPT_PATH_WAVEFRONT. */
#define CPT_SCHEDULE_COST 0x800u
/* Megakernel tail consolidation: once the pixel queue is drained, the
 * waves of a workgroup hand their chains over at pass boundaries so that each SIMD runs fewer,
 * fuller waves while chains finish.  Identical results.  By default it runs when spp >= 512 and
 * the frame holds more than 1 and at most 4 pixels per lane of the persistent grid (a
 * strong-scaled row tile on 2-7 GPUs at 1080p);
 * these flags force it on or off (on needs spp > 1).  Only the 4-wide walk consolidates
 * (CPT_TRAVERSAL_ORDERED with a 4-wide walk tree, cpt_get_walk_info [2] > 0).  A hand-over that
 * cannot complete ends the render with CPT_ERR_DEVICE, never with silently missing pixels. */
#define CPT_SCHEDULE_CONSOLIDATE    0x1000u
#define CPT_SCHEDULE_NO_CONSOLIDATE 0x2000u
/* Megakernel pixel schedule without a pilot, for renders of few passes that repeat over the
 * same frame (the DispatchRay loop, path_tracer.cu:256-306): the tiles are dequeued heaviest
 * first by the work of the context's PREVIOUS render with this flag -- each tile's RNG draws,
 * read off the XORWOW Weyl counters (d advances by 362437 per draw), which follow the path
 * lengths -- and the first render in a frame uses the row-major order.  Identical results;
 * ignored with CPT_SCHEDULE_COST and by CPT_PATH_WAVEFRONT. */
#define CPT_SCHEDULE_PREVIOUS       0x4000u

int cpt_abi_version(void);
const char* cpt_status_string(int status);
int cpt_get_device_count(int* count);

int cpt_create(int device, cpt_ctx** out);
int cpt_destroy(cpt_ctx* ctx);
/* Last error message of ctx (or of the last failed cpt_create when ctx is NULL). */
const char* cpt_last_error(const cpt_ctx* ctx);
/* Launch on `hip_stream` (a hipStream_t) instead of the context's own stream; NULL restores it. */
int cpt_set_stream(cpt_ctx* ctx, void* hip_stream);

/* Host-side MotionalCamera::GetCopy: computes the basis and corner vectors, increments
 * cur_sample_idx (motional_camera.cu:177-200). */
int cpt_camera_get_copy(cpt_camera* cam);

/* Builds the reference's median-split BVH over `objs` (objects copied by value, like
 * bvh.cu:43) and uploads it.  n_objs may be 0 (every ray misses). */
int cpt_set_scene(cpt_ctx* ctx, const cpt_object* objs, int n_objs);
/* Replace object `index` (AddObject order) and refit the ancestors' boxes. */
int cpt_update_object(cpt_ctx* ctx, int index, const cpt_object* obj);
/* The same for n objects at once (SceneBVH::UpdateObject, bvh.cu:122-157), refit on the GPU:
 * the host names the updated leaves and their ancestors (O(n x depth)), kernels rewrite the
 * boxes bottom-up in every device copy of both trees (reference order, walk orders, 4-wide
 * image); topology as built.  The refit is a function of the leaves only, so the result equals
 * n single updates in any order (a repeated index: the last object wins).  Returns after the
 * device copies are updated.  An edit that turns an object into a platform or back rebuilds
 * like cpt_update_objects_rebuild. */
int cpt_update_objects(cpt_ctx* ctx, int n, const int* indices, const cpt_object* objs);
/* The same edits, with the ordered walk's SAH tree rebuilt from the edited objects on the host
 * and all orders re-linearised and uploaded (the reference order is refit either way): restores
 * the walk tree's quality after large motions.  Same images. */
int cpt_update_objects_rebuild(cpt_ctx* ctx, int n, const int* indices, const cpt_object* objs);
/* Material slots the scene holds (deduplicated per value, cpt_set_scene; a device refit that
 * gives objects new materials appends slots, and once more than twice the referenced ones
 * (+ 16) are held, the unreferenced slots are dropped with a rebuild). */
int cpt_get_material_count(cpt_ctx* ctx, int* n);
/* Host wall time of the last cpt_update_objects[_rebuild] call, ms. */
int cpt_last_update_ms(cpt_ctx* ctx, float* ms);
/* Exports the BVH in the reference's node order (Divide creation order): per node
 * boxes[6] = {min xyz, max xyz}, links[4] = {is_object, left, right, object index}. */
int cpt_scene_bvh_export(cpt_ctx* ctx, float* boxes, int32_t* links, int capacity, int* n_nodes);
/* Same BVH build without a context or a GPU (host only), same export format. */
int cpt_bvh_build_host(const cpt_object* objs, int n_objs, float* boxes, int32_t* links, int capacity, int* n_nodes);

/* Environment map, RGBA8 rows of `valid_cols` texels (the reference uploads only
 * logical_width/4 texels per row, textures.cu:32-33; texels at x >= valid_cols read 0).
 * Sampler: normalized coords, mirror addressing, bilinear, c/255 (textures.cu:36-44). */
int cpt_set_env_texture(cpt_ctx* ctx, const uint8_t* rgba, int logical_width, int height, int valid_cols);

/* cudaTextureAddressMode / cudaTextureFilterMode values of AddTexByFile's arguments. */
#define CPT_ADDRESS_WRAP   0
#define CPT_ADDRESS_CLAMP  1
#define CPT_ADDRESS_MIRROR 2   /* AddTexByFile's default */
#define CPT_ADDRESS_BORDER 3   /* border colour 0 */
#define CPT_FILTER_POINT   0
#define CPT_FILTER_LINEAR  1   /* AddTexByFile's default */

/* Binds texels to a material texture handle (replacing an earlier binding).  A textured
 * material (have_tex != 0) takes its diffuse colour from the texture bound to u.tex:
 * GetKd is always called at normalized (0, 0) (material.cu:31,56,95,140 pass no uv), so
 * the colour is that one sample, taken once per material when the scene is prepared.
 * Emission keeps reading kd_, i.e. the bits of the handle, as the reference's union does
 * (material.cu:36).  Layout as cpt_set_env_texture; a material whose handle is unbound
 * makes cpt_set_scene / cpt_render fail with CPT_ERR_INVALID_ARG.  Binding after
 * cpt_set_scene re-prepares the materials. */
int cpt_bind_texture(cpt_ctx* ctx, uint64_t handle, const uint8_t* rgba, int logical_width, int height,
                     int valid_cols, int address_mode, int filter_mode);

/* Per-pixel buffers for a width x height frame; the context renders the global image rows
 * listed in `rows` (n_rows of them; rows == NULL means 0..height-1).  Pixel i of the
 * context's buffers is (x = i % width, y = rows[i / width]). */
int cpt_set_frame(cpt_ctx* ctx, int width, int height, const int32_t* rows, int n_rows);
/* curand_init(seed, (x << 32) | y, 0) for every pixel of the context (InitCuRand). */
int cpt_init_rng(cpt_ctx* ctx, uint64_t seed);
int cpt_read_rng(cpt_ctx* ctx, uint32_t* planar6);          /* [6][n_rows*width]: v0..v4, d */
int cpt_write_rng(cpt_ctx* ctx, const uint32_t* planar6);

/* `spp` SamplePixel passes for every pixel of the context, each pass continuing the
 * pixel's XORWOW stream; the accumulator holds rgb sums + pass count per pixel.
 * max_depth in [0, 32] (MAX_RECURSION_DEPTH_SET, path_tracer.h:13).  Asynchronous unless
 * CPT_RENDER_SYNC. */
int cpt_render(cpt_ctx* ctx, const cpt_camera* cam, int spp, int max_depth, uint32_t flags);
int cpt_synchronize(cpt_ctx* ctx);
int cpt_read_accum(cpt_ctx* ctx, float* rgba);               /* [n_rows*width][4] */
int cpt_clear_accum(cpt_ctx* ctx);
int cpt_read_aux(cpt_ctx* ctx, float* normal3, float* depth); /* either may be NULL */
/* Checkpoint / resume (the reference keeps its running state only in device memory,
 * path_tracer.cu:91-99): restore the accumulator ([rows*W][4]: rgb sums + pass count) and the
 * first-hit normal / depth buffers from host copies made with cpt_read_accum / cpt_read_aux.
 * With cpt_write_rng, a render (and the display path) resumes bit for bit. */
int cpt_write_accum(cpt_ctx* ctx, const float* rgba);
int cpt_write_aux(cpt_ctx* ctx, const float* normal3, const float* depth);
/* The cost schedule's pilot alone (for cost-balanced row partitions across ranks, tiling.py):
 * `passes` passes from the context's current RNG states (nothing is written back), each 8x8 tile's
 * work -- segments + node visits + primitive tests, the walk of `flags`' CPT_TRAVERSAL_* bits --
 * into out[tile] (tiles row-major over the context's rows: ((n_rows+7)/8) x ((width+7)/8);
 * n_out at least that).  Synchronous. */
int cpt_tile_costs(cpt_ctx* ctx, const cpt_camera* cam, int passes, int max_depth, uint32_t flags, uint32_t* out,
                   size_t n_out);
/* Device-to-device copy of the accumulator (e.g. into an RCCL send buffer), ordered against the
 * caller's HIP stream `caller_stream` (NULL: the null stream) without blocking the host: the
 * context's stream first waits for the work queued on caller_stream so far (a fill of dst, a
 * collective still reading it), then copies, and caller_stream waits for the copy (work queued on
 * it next, e.g. the all-gather, reads the copied bytes).  When caller_stream is the context's own
 * launch stream (cpt_set_stream) the copy is simply queued there.  Device errors of the render
 * surface at the next synchronising call. */
int cpt_copy_accum_device(cpt_ctx* ctx, void* device_dst, size_t bytes, void* caller_stream);
/* Row-tile gather (multi-GPU row tiling; the single-GPU reference writes the
 * whole frame from SamplePixel, path_tracer.cu:172-174): places the rows `src` rendered -- its
 * accumulator, and its first-hit normals and depths when it rendered with CPT_RENDER_AUX --
 * into `dst`'s frame at the same global rows (dst must hold every one of them, e.g. a full
 * frame).  src and dst may live on different devices (the stitch reads src over xGMI with peer
 * access, enabled once per device pair; a staged peer copy where no peer path exists) or on the
 * same one.  Asynchronous: ordered after src's queued work and before src's later work by
 * events, with no host wait, so several gathers queue back to back; dst then holds the stitched
 * frame for its next call (cpt_synchronize, cpt_read_accum, cpt_read_aux, cpt_denoise_mix).
 * src's device errors are reported by src's own next synchronising call. */
int cpt_gather_rows(cpt_ctx* dst, cpt_ctx* src);
/* How the last cpt_gather_rows(dst, src) reached src's buffers (-1: no gather of the pair yet):
 * the stitch read them in place on the same device, read them over xGMI with peer access
 * (contexts on two devices), or read a staged hipMemcpyPeerAsync copy (no peer path, or
 * forced by cpt_set_debug_gather).  No reference counterpart: a test hook for §8(e). */
#define CPT_GATHER_SAME_DEVICE 0
#define CPT_GATHER_PEER 1
#define CPT_GATHER_STAGED 2
int cpt_last_gather_mode(cpt_ctx* dst, cpt_ctx* src, int* mode);
/* TEST HOOK: force dst's gathers through the staged peer copy (the fallback for device pairs
 * without peer access), so that branch runs on a one-GPU box too. */
int cpt_set_debug_gather(cpt_ctx* dst, int force_staged);
int cpt_get_stats(cpt_ctx* ctx, cpt_stats* out);
int cpt_reset_stats(cpt_ctx* ctx);
/* All 8 raw device counters (0-4 = cpt_stats; 5 = ordered-walk segments that failed the
 * winner certificate and took the reference walk (CPT_RENDER_STATS | CPT_TRAVERSAL_ORDERED);
 * 6 = 4-wide node visits read from global memory, i.e. past the LDS image's first 512 nodes). */
int cpt_get_raw_counters(cpt_ctx* ctx, uint64_t* out8);
/* DIAGNOSTIC (a library built with CPT_TIMELINE; CPT_ERR_STATE otherwise): the megakernel's
 * lane-occupancy timeline since the last call, n words (<= 4 x 4096 + 4): per 1.31 ms bin of
 * the device's 100 MHz clock (a ring of 4096 bins) busy-lane x ticks, wave x 64 x ticks, busy-lane
 * x ticks after the pixel queue ran dry, of level-0 waves; then the first tick a wave saw the
 * queue dry.  Clears it (tools/timeline.py). */
int cpt_debug_timeline(cpt_ctx* ctx, uint64_t* out, int n);
/* DIAGNOSTIC: the 16 wave-time stamp slots of a CPT_STAMPS build (cpt_stamps.hpp; all zero in
 * the shipped library), summed over the renders since the last cpt_reset_stats. */
int cpt_get_diag_counters(cpt_ctx* ctx, uint64_t* out16);
/* DIAGNOSTIC: the exec-mask census of a CPT_EXECDIAG build (cpt_stamps.hpp execdiag; all zero in
 * the shipped library): per code region r < 16, [r] entries, [16 + r] entries with <= 16 active
 * lanes, [32 + r] with <= 8, [48 + r] the sum of active lanes, since the last cpt_reset_stats. */
int cpt_get_execdiag_counters(cpt_ctx* ctx, uint64_t* out64);
/* Node counts of the scene's walk structures (host-side, no GPU work): [0] the reference
 * order (bvh.cu's tree, 32-B nodes), [1] each octant order of the binary walk tree, [2] the
 * 4-wide walk tree's nodes (112 B each in its compact image, the first 512 staged in LDS; 0 =
 * the ordered walk uses the binary orders), [3] the unbounded (platform) leaves tested before
 * the walk tree.  With [2] > 0, the `nodes` counter of an ordered render counts 4-wide node
 * visits. */
int cpt_get_walk_info(cpt_ctx* ctx, int32_t* out4);
/* Device time of the last cpt_render (HIP events on the launch stream); waits for it. */
int cpt_last_render_ms(cpt_ctx* ctx, float* ms);
/* Average device time of one launch of the last cpt_render's dominant kernel: the megakernel
 * (launches = 1; the cost schedule's pilot and sort are not included) or the wavefront's
 * extend/shade launches (their total / launches).  Waits for the render. */
int cpt_last_kernel_stats(cpt_ctx* ctx, float* avg_ms, int* launches);

/* Display path (path_tracer.cu:177-254): 5x5 edge-aware denoise of the current 1-spp
 * radiance (accumulator / pass count), running-mean Mix with weight 1/cur_sample_idx,
 * BGRA8 out (alpha byte untouched).  Needs a full frame (rows == NULL).  A pinned bgra_host
 * (cpt_host_register, hipHostMalloc, torch pin_memory) of a 16-aligned width is written by the
 * display kernel itself over PCIe; other memory gets a copy after it (the reference's
 * cudaMemcpy, path_tracer.cu:303). */
int cpt_denoise_mix(cpt_ctx* ctx, uint32_t cur_sample_idx, uint8_t* bgra_host);
/* Pin / unpin a host buffer (hipHostRegister, mapped) so display frames reach it without a
 * staging copy -- e.g. the BGRA8 buffer the reference hands to its per-pass callback
 * (path_tracer.cu:303-304).  Unregister before freeing it. */
int cpt_host_register(void* ptr, size_t bytes);
int cpt_host_unregister(void* ptr);
/* Display path for output rows [y0, y1) of the 16-aligned launch (0 <= y0 < y1 <= 16*(H/16)),
 * for row-banded multi-GPU display: the context's frame rows (cpt_set_frame) must be one
 * ascending run covering [max(0, y0-3), min(16*(H/16), y1+3)) -- the band and the rows its
 * linear-offset stencil reaches (x +- 2 wraps into the next row).  The Mix running mean and the
 * BGRA8 output hold the band's rows only ((y1-y0) x W x 4 bytes to bgra_host, may be NULL); a
 * new band starts a fresh (zeroed) mean.  Byte-identical to rows y0..y1-1 of cpt_denoise_mix. */
int cpt_denoise_mix_band(cpt_ctx* ctx, uint32_t cur_sample_idx, int y0, int y1, uint8_t* bgra_host);
/* Device-to-device copy of the current display band's BGRA8 rows (for an RCCL gather), ordered
 * against caller_stream as cpt_copy_accum_device. */
int cpt_copy_bgra_device(cpt_ctx* ctx, void* device_dst, size_t bytes, void* caller_stream);
/* The output rows [y0, y1) the display buffers currently hold (cpt_denoise_mix: the whole
 * 16-aligned launch; cpt_denoise_mix_band: the band); 0, 0 before the first display pass. */
int cpt_display_band(const cpt_ctx* ctx, int* y0, int* y1);
/* The Mix running mean of the current display band ([(y1-y0)*W][3] floats: rows y0..y1-1; the
 * whole 16-aligned launch's rows for cpt_denoise_mix), read back for checking and checkpoints.
 * `capacity` is rgb's size in floats: CPT_ERR_INVALID_ARG (nothing written) when it is smaller
 * than the band (size it from cpt_display_band). */
int cpt_read_mix(cpt_ctx* ctx, float* rgb, size_t capacity);
/* Device time of the last display kernel (Denoising + Mix, the reference's per-pass log of
 * path_tracer.cu:261,300 split by kernel), from HIP events on the context's stream; waits
 * for it. */
int cpt_last_display_ms(cpt_ctx* ctx, float* ms);
/* Zero the Mix running mean (the reference's buffer starts uninitialised; here it is zeroed
 * when the frame is created and by this call). */
int cpt_reset_display(cpt_ctx* ctx);

/* HBM streaming-read ceiling of the device (the roofline peak, measured on
 * the box): `iters` grid-stride 16-B-per-lane read passes over a fresh `bytes`-byte buffer
 * (use >> 256 MiB so the Infinity Cache cannot serve it), GB/s from HIP events. */
int cpt_measure_read_bandwidth(cpt_ctx* ctx, size_t bytes, int iters, float* gbps);
/* DIAGNOSTIC: the same streaming read in the display kernel's access shapes, bytes_per_lane 4 (one
 * float per lane), 12 (three consecutive floats per lane) or 16 (one float4), one kernel
 * (k_read_pattern<bpl>) per shape: the known byte counts a rocprofv3 FETCH_SIZE pass is calibrated
 * against (tools/fetch_calibration.py). */
int cpt_measure_read_pattern(cpt_ctx* ctx, int bytes_per_lane, size_t bytes, int iters, float* gbps);
/* Host-only test hook (no GPU): the cap-disk bound a cylinder leaf carries (cpt_capi.cpp
 * cap_disk_bound), the largest float c with  sqrtf(q) < radius  <=>  q <= c  for every float
 * q; the kernels decide the reference's cap test (object.cu:52-77) with it. */
int cpt_cap_disk_bound(float radius, float* out);
/* Device-math known-answer surface used by the parity tests: op 0 powf(a,b), 1 sinf(a),
 * 2 cosf(a), 3 asinf(a), 4 atanf(a), 5 (float)pow((double)a, 1.0/(double)b),
 * 6 (float)((double)a / (double)b) [IEEE f64 division], 7 a / b [f32 division],
 * 8 sqrtf(a), 9 pow(a, 5) as schlick computes it (dm::pow5f). */
int cpt_math_batch(cpt_ctx* ctx, int op, const float* a, const float* b, float* out, size_t n);
/* Device self-test of the exact-quotient kernel helper against the hardware IEEE f32 divide
 * over n hashed operand pairs (which: 0 all bit patterns, 1 slab-like ranges, 2 mid ranges).
 * which = 3: the f64 reciprocal helper rcp_d(d) against the IEEE 1.0 / (double)d for the first
 * n float bit patterns d (n = 2^32: all of them); which = 4: the f32 reciprocal helper rcp_f on
 * its domain (2^-126 <= |d| < 2^126, 0, inf, NaN) and rcp_f(sqrtf(d)) for every pattern.
 * which = 5: the f32 square-root helper sqrt_nn against sqrtf on its domain (+-0,
 * |x| >= 2^-96, inf, NaN).
 * which = 6: the display weight dn_weight (short exp + rounding guard) against its slow form
 * dn_weight_slow for the float bit patterns [0, n) (n = 2^31: every non-negative float, inf and
 * NaN); which = 7: counts the patterns whose guard sends them to the slow form (not an error).
 * which = 8: the BSDF lobe's short pow (lobe_pow) against (float)pow(x, y) of the full double
 * sequence for the float bit patterns x in [0, n), y = the double whose bits are `seed`;
 * which = 9: counts the x whose guard sends them to the full pow; which = 10: the lobe's short
 * sinf/cosf (lobe_sincos) against the full sequence for the float patterns [0, n); which = 11:
 * counts the guard's fallbacks there; which = 12: the sky fetch's short atanf and asinf
 * (miss_atanf, miss_asinf) against the full sequences for the float patterns [0, n); which = 13:
 * counts the patterns where either guard falls back (asinf: on [-1, 1]).
 * which = 14: the ordered walk's quotient-free winner certificate (cert_inside) against the exact
 * slab test on n hashed cases from `seed` (boxes, rays, distances within 16 ulps of a plane):
 * out[0] counts the cases it certifies and the exact test rejects (0 expected); which = 15 counts
 * the certified cases and which = 16 the cases the exact test passes.
 * out[0] receives the mismatch count (0 expected), out[1..out_len) up to out_len-1 failing
 * pairs as (a bits << 32 | d bits). */
int cpt_selftest_qdiv(cpt_ctx* ctx, int which, uint64_t n, uint64_t seed, uint64_t* out, int out_len);
/* TEST HOOK for the tail consolidation's error paths (all zero = normal operation): flags bit 0
 * starts every workgroup with a phantom live chain (a lost count: the keeper waves can never
 * see the workgroup drained), bit 1 makes hand-overs never publish their slot; the keeper's
 * idle-spin limit and the hand-over wait as log2 (0 = the defaults, 26 and 22).  A render that
 * trips either limit must end with CPT_ERR_DEVICE. */
int cpt_set_debug_consolidation(cpt_ctx* ctx, uint32_t flags, int keeper_spin_log2, int publish_wait_log2);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* CPT_H_ */
