// cpt_host.hpp — host-side scene preparation of libcpt (no device code): the reference's
// median-split BVH (SceneBVH::Divide, bvh.cu:31-90), the ordered walk's SAH tree, their
// linearisations into the node orders and the 4-wide image the kernels walk
// (cpt_host_bvh.cpp), and the XORWOW jump tables of InitCuRand (cpt_host_rng.cpp).
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/cpt.h"
#include "cpt_internal.hpp"

namespace cpt {
namespace host {

struct F3 { float x, y, z; };

inline float MIN_(float a, float b) { return a < b ? a : b; }   // ray_tracing_math.hpp:19-21
inline float MAX_(float a, float b) { return a > b ? a : b; }   // ray_tracing_math.hpp:15-17
inline float ABS_(float a) { return a >= 0 ? a : -a; }          // ray_tracing_math.hpp:23-25

// Object::GetAABBMax / GetAABBMin (object.cu:134-170)
F3 aabb_max(const cpt_object& o);
F3 aabb_min(const cpt_object& o);

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

// SceneBVH::Divide over all objects (bvh.cu:31-120): node 0 is the root.
void build_host_bvh(HostBvh& b, const std::vector<cpt_object>& objs);
// The cap-disk bound of a cylinder leaf (Node::b1): sqrtf(q) < r  <=>  q <= bound.
float cap_disk_bound(float r);
// A leaf's or internal node's device Node (cpt_device.hpp).
Node make_node(const BNode& n, const std::vector<cpt_object>& objs, const std::vector<int>& mat_of_obj);
// Skip-link preorder of a tree (octant < 0: the reference's right-first order; else the
// near-first order of a direction octant), appended to `out`.
void linearise(const HostBvh& b, const std::vector<cpt_object>& objs, const std::vector<int>& mat_of_obj,
               std::vector<Node>& out, std::vector<int>& pos_of_node, int octant, const std::vector<int>* ref_pos,
               int root = 0, const std::vector<int>& prefix = {});

namespace sah {
int leaf(HostBvh& t, const std::vector<cpt_object>& O, int o);
int build(HostBvh& t, const std::vector<cpt_object>& O, std::vector<int>& idx, int l, int r);
}  // namespace sah

constexpr int WIDE_STACK = CPT_WSTACK;
// The 4-wide walk tree's compact image + leaf array, appended to `out`; returns n_wide (0: the
// binary walk is used instead).
int linearise_wide(const HostBvh& w, int root, const std::vector<int>& pos0, int n_bvh, int n_unb,
                   std::vector<Node>& out, int* n_leaves_out, std::vector<int>& slot_of, std::vector<int>& leaf_of);

// jumps[t] = A^(2^67 * 2^t), 64 matrices of 160x160 bits (column-major, rocRAND's layout).
const std::vector<uint32_t>& jump_tables();
// curand_init's seed scrambling: v[0..4], d.
void curand_seed_state(uint64_t seed, uint32_t out[6]);

}  // namespace host
}  // namespace cpt
