// cpt_host_bvh.cpp — host BVH builds and linearisations (cpt_host.hpp): the reference's
// median split (bvh.cu:31-120), the ordered walk's binned SAH tree, the skip-link orders and
// the 4-wide compact image the kernels walk.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <functional>
#include <mutex>
#include <queue>
#include <vector>

#include "cpt_host.hpp"

namespace cpt {
namespace host {

// ------------------------------------------------------------------------------------
// Host BVH: SceneBVH::Divide (bvh.cu:31-90) and the skip-link linearisation.
// ------------------------------------------------------------------------------------

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


static int divide(HostBvh& b, const std::vector<cpt_object>& objs, std::vector<int>& idx, int l, int r) {
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
               int root, const std::vector<int>& prefix) {
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
// 4-wide walk tree (DESIGN.md §Ordered walk, Execution).  The binary SAH walk tree is collapsed into
// nodes of up to four children: starting from a node's two children, the internal child
// with the largest box is replaced by its own two children until there are four (or only
// leaves).  Appended to `out` (after the eight binary octant orders): the compact image,
// 7 x 16 B per node (layout below), then the leaf array.  Nodes are numbered largest box
// first (root 0).  Returns n_wide, or 0 when the device walk's stack (WIDE_STACK entries per
// lane, cpt_path.hpp) could overflow on this tree or a ref would not fit 15 bits.
// ------------------------------------------------------------------------------------

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

}  // namespace host
}  // namespace cpt
