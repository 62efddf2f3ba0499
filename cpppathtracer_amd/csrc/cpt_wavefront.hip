// cpt_wavefront.hip — the SoA wavefront integrator (CPT_PATH_WAVEFRONT).
//
// The same SamplePixel semantics as k_megakernel (path_tracer.cu:124-175), split into
// kernels that each do one uniform thing over a queue of live paths:
//
//   k_wf_raygen   pass start: RayGen for every pixel (motional_camera.cu:202-213)
//   k_wf_extend   TraceRay for every queued ray (bvh.cu:167-205) -> hit record
//   k_wf_shade    ClosetHit/Miss + path bookkeeping (path_tracer.cu:141-169); live paths are
//                 re-compacted into the next queue with a wave64 ballot + mbcnt prefix and ONE
//                 atomic per wave; finished paths add their radiance to the pixel accumulator
//
// Path state lives in HBM as SoA float4 arrays indexed by queue slot, double-buffered across
// bounces: shade writes a surviving path at the slot the compaction gives it, so extend and the
// next shade read it coalesced.  Queues map slot -> pixel, for the per-pixel XORWOW state and
// the accumulator only.  A pixel's
// passes run in order (pass p for all pixels, then p+1), so every pixel consumes its XORWOW
// stream exactly as in the megakernel and the results are bit-identical to it.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "cpt_path.hpp"

namespace cpt {

// Packed per-slot path state (all float4, 16-B aligned, SoA).
//   ray_o  = (o.xyz, tmin)         ray_d = (d.xyz, depth as uint bits)
//   att    = (attenuation.xyz, first-segment flag bits)
//   rad    = (radiance.xyz, unused)
//   hit_p  = (hit pos.xyz, code bits: material << 2 | type, or -1 = miss)
//   hit_n  = (normal.xyz, unused)
//   aux    = (first-hit normal sum.xyz, depth sum)          (AUX only)

__device__ __forceinline__ uint32_t wave_append(bool alive, uint32_t* counter) {
    const uint64_t m = __ballot(alive);
    if (m == 0) return 0;
    const int leader = __ffsll((unsigned long long)m) - 1;
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == leader) base = atomicAdd(counter, (uint32_t)__popcll(m));
    base = __shfl(base, leader);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ void load_rng(const KParams& p, size_t npix, size_t pix, Xorwow& s) {
    s.v0 = p.rng[pix];
    s.v1 = p.rng[npix + pix];
    s.v2 = p.rng[2 * npix + pix];
    s.v3 = p.rng[3 * npix + pix];
    s.v4 = p.rng[4 * npix + pix];
    s.d = p.rng[5 * npix + pix];
}

__device__ __forceinline__ void load_rng_slot(const WfState& w, int b, uint32_t i, Xorwow& s) {
    const uint4 a = w.rng_a[b][i];
    const uint2 c = w.rng_b[b][i];
    s.v0 = a.x; s.v1 = a.y; s.v2 = a.z; s.v3 = a.w;
    s.v4 = c.x; s.d = c.y;
}

__device__ __forceinline__ void store_rng_slot(const WfState& w, int b, uint32_t i, const Xorwow& s) {
    w.rng_a[b][i] = make_uint4(s.v0, s.v1, s.v2, s.v3);
    w.rng_b[b][i] = make_uint2(s.v4, s.d);
}

__device__ __forceinline__ void store_rng(const KParams& p, size_t npix, size_t pix, const Xorwow& s) {
    p.rng[pix] = s.v0;
    p.rng[npix + pix] = s.v1;
    p.rng[2 * npix + pix] = s.v2;
    p.rng[3 * npix + pix] = s.v3;
    p.rng[4 * npix + pix] = s.v4;
    p.rng[5 * npix + pix] = s.d;
}

// Pass start.  The first queue is the tile-ordered identity (k_wf_ident, exactly npix
// entries), so nothing is appended here: slot i of state buffer 0 is the path of pixel
// ident[i].  max_depth == 0: the pass is RayGen's draws and a zero radiance.
template <bool AUX>
__global__ void __launch_bounds__(256) k_wf_raygen(const KParams p, WfState w) {
    const size_t npix = (size_t)p.n_rows * p.width;
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < npix; i += stride) {
        const size_t pix = (size_t)w.ident[i];
        const int x = (int)(pix % p.width), ri = (int)(pix / p.width);
        Xorwow s;
        load_rng(p, npix, pix, s);
        const Ray ray = ray_gen(p, x, p.rows[ri], s);
        if (p.max_depth == 0) {
            store_rng(p, npix, pix, s);
            float4 a = p.accum[pix];
            p.accum[pix] = make_float4(a.x + 0.f, a.y + 0.f, a.z + 0.f, a.w + 1.0f);
            if (AUX) {
                p.normal[3 * pix] = 0.f;
                p.normal[3 * pix + 1] = 0.f;
                p.normal[3 * pix + 2] = 0.f;
                p.depth[pix] = 0.f;
            }
            continue;
        }
        w.ray_o[0][i] = make_float4(ray.o.x, ray.o.y, ray.o.z, ray.tmin);
        w.ray_d[0][i] = make_float4(ray.d.x, ray.d.y, ray.d.z, __uint_as_float(0u));
        w.att[0][i] = make_float4(1.f, 1.f, 1.f, __uint_as_float(1u));
        w.rad[0][i] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (AUX) w.aux[0][i] = make_float4(0.f, 0.f, 0.f, 0.f);
        store_rng_slot(w, 0, (uint32_t)i, s);   // the path carries its stream until it ends
    }
}

// LDST: the megakernel's wide walk on the workgroup's LDS image of the tree (1024-lane blocks,
// one per CU; the image is staged only by blocks that have rays), else the binary walks.
constexpr int WF_LDS_BLOCK = 1024;
template <bool LDST> constexpr int wf_extend_block() { return LDST ? WF_LDS_BLOCK : 256; }

template <bool STATS, bool LDST>
__global__ void __launch_bounds__(wf_extend_block<LDST>()) k_wf_extend(const KParams p, WfState w,
                                                                       const uint32_t* __restrict__ nin,
                                                                       const int sb) {
    constexpr int BLK = wf_extend_block<LDST>();
    const uint32_t n = *nin;
    __shared__ uint4 s_tree[LDST ? LDS_TREE_NODES * 7 : 1];
    if (LDST) {
        if ((uint32_t)blockIdx.x * BLK >= n) return;   // no ray for this block in this bounce
        const uint4* src = reinterpret_cast<const uint4*>(p.nodes + wide_image_base(p));
        for (int i = threadIdx.x; i < 7 * lds_tree_nodes(p.n_wide); i += BLK) s_tree[i] = src[i];
        __syncthreads();
    }
    Counters cnt{};
    const uint32_t stride = gridDim.x * blockDim.x;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const float4 o = w.ray_o[sb][i], d = w.ray_d[sb][i];
        Ray ray;
        ray.o = mk(o.x, o.y, o.z);
        ray.d = mk(d.x, d.y, d.z);
        ray.tmin = o.w;
        ray.tmax = DEFAULT_RAY_TMAX;
        const RayK rk = make_rayk(ray);
        const bool finite = !(ray.o.x != ray.o.x || ray.o.y != ray.o.y || ray.o.z != ray.o.z || ray.d.x != ray.d.x ||
                              ray.d.y != ray.d.y || ray.d.z != ray.d.z);
        Hit h;
        int code = -1;
        if (STATS) cnt.segments++;
        bool hit;
        if (LDST) hit = trace_segment<STATS, BLK, true>(p, rk, finite, h, code, cnt, s_tree);
        else hit = trace_segment<STATS>(p, rk, finite, h, code, cnt);
        w.hit_p[i] = make_float4(h.pos.x, h.pos.y, h.pos.z, __int_as_float(hit ? code : -1));
        if (hit) w.hit_n[i] = make_float4(h.normal.x, h.normal.y, h.normal.z, 0.f);
    }
    if (STATS) {
        const uint64_t a = wave_sum(cnt.segments), b = wave_sum(cnt.nodes), c = wave_sum(cnt.prims);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd((unsigned long long*)&p.stats[0], (unsigned long long)a);
            atomicAdd((unsigned long long*)&p.stats[1], (unsigned long long)b);
            atomicAdd((unsigned long long*)&p.stats[2], (unsigned long long)c);
        }
        const uint64_t f = wave_sum(cnt.fallbacks);   // ordered walk: certificate fallbacks
        if ((threadIdx.x & 63) == 0 && f) atomicAdd((unsigned long long*)&p.stats[5], (unsigned long long)f);
        const uint64_t g = wave_sum(cnt.gnodes);      // wide nodes read from global memory
        if ((threadIdx.x & 63) == 0 && g) atomicAdd((unsigned long long*)&p.stats[6], (unsigned long long)g);
    }
}

template <bool STATS, bool AUX>
__global__ void __launch_bounds__(256) k_wf_shade(const KParams p, WfState w, const int32_t* __restrict__ qin,
                                                 const uint32_t* __restrict__ nin, int32_t* __restrict__ qout,
                                                 uint32_t* __restrict__ nout, const int sb) {
    const uint32_t n = *nin;
    const size_t npix = (size_t)p.n_rows * p.width;
    const uint32_t max_depth = (uint32_t)p.max_depth;
    uint32_t hits = 0, misses = 0;
    const uint32_t stride = gridDim.x * blockDim.x;
    // all lanes run the same trip count so the wave-level append sees the whole wave
    const uint32_t trips = (n + stride - 1) / stride;
    // The block's 256 slots are regrouped misses-first through LDS (a counting sort on
    // miss / hit / past-the-queue), so a wave runs the sky path or the material path, rarely both.
    __shared__ uint32_t s_cnt[3][4];
    __shared__ uint32_t s_slot[256];
    __shared__ uint32_t s_app[5];   // the block's survivors per wave, then the block's first slot
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (uint32_t t = 0, i0 = blockIdx.x * blockDim.x + threadIdx.x; t < trips; ++t, i0 += stride) {
        const int key = i0 < n ? (__float_as_int(w.hit_p[i0].w) >= 0 ? 1 : 0) : 2;
        uint64_t mk_[3];
        for (int k = 0; k < 3; ++k) mk_[k] = __ballot(key == k);
        if (lane == 0)
            for (int k = 0; k < 3; ++k) s_cnt[k][wv] = (uint32_t)__popcll(mk_[k]);
        __syncthreads();
        uint32_t pos = 0;
        for (int k = 0; k < 3; ++k)
            for (int v = 0; v < 4; ++v)
                if (k < key || (k == key && v < wv)) pos += s_cnt[k][v];
        const uint64_t mine = mk_[key];
        pos += __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
        s_slot[pos] = i0;
        __syncthreads();
        const uint32_t i = s_slot[threadIdx.x];
        bool alive = false;
        int pix = 0;
        float4 no4, nd4, na4, nr4, nx4;   // the surviving path's state for buffer sb ^ 1
        Xorwow s;
        if (i < n) {
            pix = qin[i];
            load_rng_slot(w, sb, i, s);
            const float4 o4 = w.ray_o[sb][i], d4 = w.ray_d[sb][i], a4 = w.att[sb][i], r4 = w.rad[sb][i];
            const float4 hp = w.hit_p[i];
            v3 dir = mk(d4.x, d4.y, d4.z);
            v3 att = mk(a4.x, a4.y, a4.z), rad = mk(r4.x, r4.y, r4.z);
            uint32_t depth = __float_as_uint(d4.w);
            const bool first = __float_as_uint(a4.w) != 0u;
            const int code = __float_as_int(hp.w);
            Shade sh;
            v3 attr_normal;
            v3 org = mk(o4.x, o4.y, o4.z);
            if (code >= 0) {
                hits++;
                const float4 hn = w.hit_n[i];
                const v3 normal = mk(hn.x, hn.y, hn.z);
                const Mat m = p.mats[code >> 2];
                eval_material(m, normal, dir, s, sh);
                attr_normal = normal;
                org = mk(hp.x, hp.y, hp.z);              // payload.hit_pos = position
            } else {
                misses++;
                sh.radiance = miss_radiance(p, dir);
                sh.attenuation = mk1(0.f);
                sh.bounce = dir;
                attr_normal = -dir;
                depth = MAX_RECURSION_DEPTH_SET;          // termination sentinel (path_tracer.cu:121)
            }
            rad = rad + att * sh.radiance;
            att = att * sh.attenuation;
            float4 aux4 = make_float4(0.f, 0.f, 0.f, 0.f);
            if (AUX) {
                aux4 = w.aux[sb][i];
                if (first) {
                    const v3 nn = mk(aux4.x, aux4.y, aux4.z) + attr_normal;
                    aux4 = make_float4(nn.x, nn.y, nn.z, aux4.w + DEFAULT_RAY_TMAX);
                }
            }
            dir = normalize(sh.bounce);
            depth++;
            if (!(depth < max_depth)) {
                // path done: the pass's radiance joins the pixel's sum (passes in order)
                const float4 a = p.accum[pix];
                p.accum[pix] = make_float4(a.x + rad.x, a.y + rad.y, a.z + rad.z, a.w + 1.0f);
                if (AUX) {
                    p.normal[3 * (size_t)pix] = aux4.x;
                    p.normal[3 * (size_t)pix + 1] = aux4.y;
                    p.normal[3 * (size_t)pix + 2] = aux4.z;
                    p.depth[pix] = aux4.w;
                }
                store_rng(p, npix, pix, s);
            } else {
                alive = true;
                no4 = make_float4(org.x, org.y, org.z, BOUNCE_RAY_TMIN);
                nd4 = make_float4(dir.x, dir.y, dir.z, __uint_as_float(depth));
                na4 = make_float4(att.x, att.y, att.z, __uint_as_float(0u));
                nr4 = make_float4(rad.x, rad.y, rad.z, 0.f);
                nx4 = aux4;
            }
        }
        // the survivors' queue slots: one counter atomic per block and trip (the block's four
        // waves' counts summed in LDS) rather than one per wave -- every wave of the grid appends
        // to this one counter, and one atomic per wave contended for it; the order of the queue
        // does not change any pixel's result
        const uint64_t am = __ballot(alive);
        if (lane == 0) s_app[wv] = (uint32_t)__popcll(am);
        __syncthreads();
        if (threadIdx.x == 0) {
            const uint32_t tot = s_app[0] + s_app[1] + s_app[2] + s_app[3];
            s_app[4] = tot ? atomicAdd(nout, tot) : 0u;
        }
        __syncthreads();
        uint32_t slot = s_app[4];
        for (int v = 0; v < wv; ++v) slot += s_app[v];
        slot += __builtin_amdgcn_mbcnt_hi((uint32_t)(am >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)am, 0u));
        if (alive) {
            const int ob = sb ^ 1;
            qout[slot] = pix;
            w.ray_o[ob][slot] = no4;
            w.ray_d[ob][slot] = nd4;
            w.att[ob][slot] = na4;
            w.rad[ob][slot] = nr4;
            if (AUX) w.aux[ob][slot] = nx4;
            store_rng_slot(w, ob, slot, s);
        }
    }
    if (STATS) {
        const uint64_t a = wave_sum(hits), b = wave_sum(misses);
        if ((threadIdx.x & 63) == 0) {
            atomicAdd((unsigned long long*)&p.stats[3], (unsigned long long)a);
            atomicAdd((unsigned long long*)&p.stats[4], (unsigned long long)b);
        }
    }
}

// Tile-ordered identity queue: the frame's pixels walked in 8x8 tiles (a wave's 64 consecutive
// ids are one tile), so each wave's first-bounce rays are coherent.
__global__ void k_wf_ident(int width, int n_rows, int32_t* q, uint32_t* count) {
    const int tiles_x = (width + 7) / 8;
    const uint32_t n_work = (uint32_t)tiles_x * ((n_rows + 7) / 8) * 64u;
    for (uint32_t id = blockIdx.x * blockDim.x + threadIdx.x; id < n_work; id += gridDim.x * blockDim.x) {
        const uint32_t tile = id >> 6, k = id & 63;
        const int x = (int)(tile % tiles_x) * 8 + (int)(k & 7);
        const int ri = (int)(tile / tiles_x) * 8 + (int)(k >> 3);
        // the valid pixels of a wave's 64 consecutive ids (one tile) get consecutive slots, one
        // counter atomic per wave (the queue's order only steers coherence, not any result)
        const bool valid = x < width && ri < n_rows;
        const uint32_t slot = wave_append(valid, count);
        if (valid) q[slot] = ri * width + x;
    }
}

// ======================================================================================
// Host driver: spp passes x (raygen, max_depth x (extend, shade)).
// ======================================================================================
static int persistent_grid(const void* fn, int block, size_t items) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        if (cus <= 0) cus = 256;
    }
    int per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, 0) != hipSuccess || per_cu < 1) per_cu = 1;
    const long long want = (long long)((items + block - 1) / block);
    return (int)std::max<long long>(1, std::min<long long>(want, (long long)per_cu * cus));
}

hipError_t wavefront_build_ident(const KParams& p, WfState& w, hipStream_t stream) {
    hipError_t e = hipMemsetAsync(w.counts + 3, 0, sizeof(uint32_t), stream);
    if (e != hipSuccess) return e;
    const size_t npix = (size_t)p.n_rows * p.width;
    hipLaunchKernelGGL(k_wf_ident, dim3((unsigned)std::min<size_t>(4096, (npix + 255) / 256 + 1)), dim3(256), 0, stream,
                       p.width, p.n_rows, w.ident, w.counts + 3);
    return hipGetLastError();
}

template <bool S, bool A, bool T>
static hipError_t wf_render_t(const KParams& p, WfState& w, hipStream_t stream, int* launches) {
    const size_t npix = (size_t)p.n_rows * p.width;
    constexpr int eb = wf_extend_block<T>();
    const int gr = persistent_grid((const void*)k_wf_raygen<A>, 256, npix);
    const int ge = persistent_grid((const void*)k_wf_extend<S, T>, eb, npix);
    const int gs = persistent_grid((const void*)k_wf_shade<S, A>, 256, npix);
    hipError_t e = hipSuccess;
    int n = 0;
    for (int pass = 0; pass < p.spp && e == hipSuccess; ++pass) {
        hipLaunchKernelGGL(k_wf_raygen<A>, dim3(gr), dim3(256), 0, stream, p, w);
        ++n;
        const int32_t* cur = w.ident;
        const uint32_t* cur_n = w.counts + 3;
        for (int b = 0; b < p.max_depth; ++b) {
            int32_t* nxt = w.queue[b & 1];
            uint32_t* nxt_n = w.counts + (b & 1);
            e = hipMemsetAsync(nxt_n, 0, sizeof(uint32_t), stream);
            if (e != hipSuccess) break;
            hipLaunchKernelGGL((k_wf_extend<S, T>), dim3(ge), dim3(eb), 0, stream, p, w, cur_n, b & 1);
            hipLaunchKernelGGL((k_wf_shade<S, A>), dim3(gs), dim3(256), 0, stream, p, w, cur, cur_n, nxt, nxt_n, b & 1);
            n += 2;
            cur = nxt;
            cur_n = nxt_n;
        }
        if (e == hipSuccess) e = hipGetLastError();
    }
    if (launches) *launches = n;
    return e;
}

template <bool T>
static hipError_t wf_render_any(const KParams& p, WfState& w, bool stats, bool aux, hipStream_t stream, int* launches) {
    if (stats && aux) return wf_render_t<true, true, T>(p, w, stream, launches);
    if (stats) return wf_render_t<true, false, T>(p, w, stream, launches);
    if (aux) return wf_render_t<false, true, T>(p, w, stream, launches);
    return wf_render_t<false, false, T>(p, w, stream, launches);
}

hipError_t launch_wavefront(const KParams& p, WfState& w, bool stats, bool aux, hipStream_t stream, int* launches) {
    if (p.width <= 0 || p.n_rows <= 0) return hipSuccess;
    // the wide walk runs on the LDS image (+ global memory past LDS_TREE_NODES), as in the
    // megakernel (cpt_kernels.hip use_lds_tree)
    const bool lds = p.ordered == 1 && p.n_wide > 0;
    return lds ? wf_render_any<true>(p, w, stats, aux, stream, launches)
               : wf_render_any<false>(p, w, stats, aux, stream, launches);
}

}  // namespace cpt
