// cpt_scene.cpp — the scene half of the C-ABI (include/cpt.h): objects to device nodes
// (SceneBVH::AddObject + BuildBVH + BuildBVHInGpu, bvh.cu:22-29, 97-120), material slots,
// the ordered walk's trees, and SceneBVH::UpdateObject (bvh.cu:122-157) as a device refit.
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

using namespace cpt::host;
using namespace cpt::ctx;

namespace cpt {
namespace ctx {

// Host staging of a Mat (cpt_device.hpp): att = kd_ (the union's bits: the handle's for a
// textured material), rad.x = emit_intensity_; k_prepare_materials completes it.
static Mat to_mat(const cpt_material& m) {
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

// Drops the material slots no object references any more and renumbers the rest (order kept).
// Leaves carry their slot in `code`, so the caller re-linearises and uploads the scene after it.
static void compact_materials(cpt_ctx* c) {
    std::vector<int> remap(c->mats_h.size(), -1);
    for (int m : c->mat_of_obj) remap[m] = 0;
    std::vector<Mat> mats;
    std::vector<int> have;
    std::vector<uint64_t> tex;
    for (size_t i = 0; i < remap.size(); ++i) {
        if (remap[i] < 0) continue;
        remap[i] = (int)mats.size();
        mats.push_back(c->mats_h[i]);
        have.push_back(c->mat_have_tex[i]);
        tex.push_back(c->mat_tex[i]);
    }
    for (int& m : c->mat_of_obj) m = remap[m];
    c->mats_h.swap(mats);
    c->mat_have_tex.swap(have);
    c->mat_tex.swap(tex);
}

// Returns the walk tree's root (-1: no bounded primitive); `unbounded` = its platform leaves
// by reference rank; `rank` = the reference rank of every walk-tree leaf.
static int build_walk_tree(const cpt_ctx* c, HostBvh& w, std::vector<int>& unbounded, std::vector<int>& rank);

// The reference order followed by the eight octant orders of the walk tree (one array,
// n_walk nodes each: the unbounded leaves, then the tree).
static void build_refit_plan(cpt_ctx* c, const HostBvh& w, const std::vector<int> (&pos)[8], const std::vector<int>& slot_of,
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

int upload_scene(cpt_ctx* c) {
    if (c->lin.size() * sizeof(Node) > (size_t)INT32_MAX)   // the walk's buffer descriptor range
        return fail(c, CPT_ERR_UNSUPPORTED, "scene too large: %zu BVH nodes in all orders (max %zu)", c->lin.size(),
                    (size_t)INT32_MAX / sizeof(Node));
    HIP_TRY(c, hipSetDevice(c->device));
    int rc;
    if ((rc = ensure(c, &c->d_nodes, &c->cap_nodes, std::max<size_t>(1, c->lin.size()))) != CPT_OK) return rc;
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
// device by k_prepare_materials.  The device array is sized here: an update batch can add
// material slots (material_slot) and reaches this without upload_scene (device_refit).
int upload_materials(cpt_ctx* c) {
    int rc;
    hipStream_t s = c->stream();
    if (c->d_mats && c->cap_mats < c->mats_h.size()) {
        // a grown array: the kernels of earlier renders may still read the old one
        HIP_TRY(c, hipStreamSynchronize(s));
    }
    if ((rc = ensure(c, &c->d_mats, &c->cap_mats, std::max<size_t>(1, c->mats_h.size()))) != CPT_OK) return rc;
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

}  // namespace ctx
}  // namespace cpt

extern "C" {

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
    // The device refit appends a slot per new material and never frees one, so a scene that edits
    // a material every frame would grow the table (and its per-batch dedup scan and upload)
    // without bound.  Once the table holds more than twice the slots the objects reference (+ 16),
    // the unreferenced ones are dropped and the scene is re-linearised with the new numbering (a
    // rebuild, amortised over the batches that grew the table).
    if (c->mats_h.size() > n_mats) {
        std::vector<char> used(c->mats_h.size(), 0);
        size_t n_used = 0;
        for (int m : c->mat_of_obj)
            if (!used[m]) { used[m] = 1; ++n_used; }
        if (c->mats_h.size() > 2 * n_used + 16) {
            compact_materials(c);
            rebuild = true;
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

int cpt_get_material_count(cpt_ctx* c, int* n) {
    if (!c || !n) return CPT_ERR_INVALID_ARG;
    *n = (int)c->mats_h.size();
    return CPT_OK;
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

}  // extern "C"
