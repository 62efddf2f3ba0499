// walk_lab.cpp — BVH walk experiments on the oracle (design tool; not part of the product).
//
// Compiled together with oracle/cpt_oracle.cpp into a stand-in oracle library
// (tools/walk_lab.py).  Every traced segment still takes the reference DFS result, so paths
// are the reference's; next to it the experimental walk runs on the same ray, and the lab
// counts its node visits / primitive tests and every segment whose closest hit (object, t,
// normal, position) differs from the reference's.
//
// Modes:
//   1  ordered walk on the reference tree (near child by split-axis sign, rank tie rule)
//   2  as 1, but unbounded primitives (platforms) are tested before the walk, outside the tree
//   3  as 2 on a binned-SAH tree over the bounded primitives (1 primitive per leaf)
//   4  the reference tree with the unbounded leaves spliced out (sibling promoted, the
//      ancestors' boxes refit); every other node keeps the reference's box
//   5  as 3 (SAH), with a conservative slab test (relative margin LAB_MARGIN) and a winner
//      certificate: the winner's own AABB must pass the exact slab test at t = t_win, else
//      the segment falls back to the reference walk (counted)
//   6  as 4, with the margin and the certificate of mode 5
//   7  as 5, on the 4-wide collapse of the SAH tree (cpt_capi.cpp linearise_wide) with a
//      stack walk; LAB_WIDTH=8 collapses to 8 children, LAB_SORT orders the hit children by
//      entry distance, LAB_CULL re-tests popped entries at the current tmax
// LAB_NB sets the SAH bin count (default 16), LAB_MARGIN the conservative margin.
#include "../oracle/cpt_oracle.cpp"
#include <cstdlib>
#include <functional>

namespace lab {

struct ANode {
    f3 bmin, bmax;
    int left = -1, right = -1, obj = -1, axis = 0;
};

struct WNode {               // mode 7: 4-wide node, children per octant in near-first order
    int child[8][8];
    int n = 0;
};

struct Tree {
    std::vector<WNode> wide;
    std::vector<ANode> wbox;   // box of each wide node
    int wroot = -1;
    std::vector<ANode> nodes;
    std::vector<int> unbounded;      // objects tested before the walk
    std::vector<int> rank_of_obj;    // reference right-first preorder rank of each object's leaf
    int root = -1;
};

int g_mode = 0;
float g_margin = 1e-3f;
std::atomic<uint64_t> g_fallback{0}, g_pretest_miss{0};
Tree g_tree;
std::atomic<uint64_t> g_nodes{0}, g_prims{0}, g_segments{0}, g_diff{0}, g_diff_obj{0};
std::mutex g_mu;
const Bvh* volatile g_src = nullptr;

f3 fmin3(f3 a, f3 b) { return mk(MIN_(a.x, b.x), MIN_(a.y, b.y), MIN_(a.z, b.z)); }
f3 fmax3(f3 a, f3 b) { return mk(MAX_(a.x, b.x), MAX_(a.y, b.y), MAX_(a.z, b.z)); }
float comp(f3 v, int a) { return a == 0 ? v.x : a == 1 ? v.y : v.z; }
float area(f3 lo, f3 hi) {
    float dx = hi.x - lo.x, dy = hi.y - lo.y, dz = hi.z - lo.z;
    return 2.f * (dx * dy + dy * dz + dz * dx);
}

int build_median(Tree& t, const Object* O, std::vector<int>& idx, int l, int r);
int build_sah(Tree& t, const Object* O, std::vector<int>& idx, int l, int r);

int make_leaf(Tree& t, const Object* O, int o) {
    ANode n;
    n.bmin = aabb_min(O[o]);
    n.bmax = aabb_max(O[o]);
    n.obj = o;
    t.nodes.push_back(n);
    return (int)t.nodes.size() - 1;
}

int build_median(Tree& t, const Object* O, std::vector<int>& idx, int l, int r) {
    if (r - l == 1) return make_leaf(t, O, idx[l]);
    f3 lo = aabb_min(O[idx[l]]), hi = aabb_max(O[idx[l]]);
    for (int i = l + 1; i < r; ++i) { lo = fmin3(lo, aabb_min(O[idx[i]])); hi = fmax3(hi, aabb_max(O[idx[i]])); }
    float sx = hi.x - lo.x, sy = hi.y - lo.y, sz = hi.z - lo.z;
    int axis = (sx >= sy && sx >= sz) ? 0 : (sy >= sz ? 1 : 2);
    std::stable_sort(idx.begin() + l, idx.begin() + r, [&](int a, int b) {
        return comp(aabb_min(O[a]), axis) + comp(aabb_max(O[a]), axis) < comp(aabb_min(O[b]), axis) + comp(aabb_max(O[b]), axis);
    });
    int me = (int)t.nodes.size();
    t.nodes.push_back(ANode{});
    int mid = (l + r) / 2;
    int L = build_median(t, O, idx, l, mid), R = build_median(t, O, idx, mid, r);
    ANode& n = t.nodes[me];
    n.left = L; n.right = R; n.axis = axis; n.bmin = lo; n.bmax = hi;
    return me;
}

// Binned SAH (16 bins per axis over centroids); falls back to the median split when no
// binned split beats the leaf-less cost.
int build_sah(Tree& t, const Object* O, std::vector<int>& idx, int l, int r) {
    if (r - l == 1) return make_leaf(t, O, idx[l]);
    f3 lo = aabb_min(O[idx[l]]), hi = aabb_max(O[idx[l]]);
    f3 clo = mk(1e30f, 1e30f, 1e30f), chi = mk(-1e30f, -1e30f, -1e30f);
    for (int i = l; i < r; ++i) {
        f3 a = aabb_min(O[idx[i]]), b = aabb_max(O[idx[i]]);
        lo = fmin3(lo, a); hi = fmax3(hi, b);
        f3 c = mk((a.x + b.x) * .5f, (a.y + b.y) * .5f, (a.z + b.z) * .5f);
        clo = fmin3(clo, c); chi = fmax3(chi, c);
    }
    static const int NB = std::getenv("LAB_NB") ? std::max(2, std::min(256, std::atoi(std::getenv("LAB_NB")))) : 16;
    float best = 1e38f;
    int best_axis = -1, best_bin = -1;
    for (int axis = 0; axis < 3; ++axis) {
        float e0 = comp(clo, axis), e1 = comp(chi, axis);
        if (!(e1 > e0)) continue;
        int cnt[256] = {0};
        f3 blo[256], bhi[256];
        for (int b = 0; b < NB; ++b) { blo[b] = mk(1e30f, 1e30f, 1e30f); bhi[b] = mk(-1e30f, -1e30f, -1e30f); }
        for (int i = l; i < r; ++i) {
            f3 a = aabb_min(O[idx[i]]), bb = aabb_max(O[idx[i]]);
            float c = (comp(a, axis) + comp(bb, axis)) * .5f;
            int b = std::min(NB - 1, (int)((c - e0) / (e1 - e0) * NB));
            cnt[b]++; blo[b] = fmin3(blo[b], a); bhi[b] = fmax3(bhi[b], bb);
        }
        for (int s = 1; s < NB; ++s) {
            int nl = 0, nr = 0;
            f3 llo = mk(1e30f, 1e30f, 1e30f), lhi = mk(-1e30f, -1e30f, -1e30f), rlo = llo, rhi = lhi;
            for (int b = 0; b < s; ++b) if (cnt[b]) { nl += cnt[b]; llo = fmin3(llo, blo[b]); lhi = fmax3(lhi, bhi[b]); }
            for (int b = s; b < NB; ++b) if (cnt[b]) { nr += cnt[b]; rlo = fmin3(rlo, blo[b]); rhi = fmax3(rhi, bhi[b]); }
            if (!nl || !nr) continue;
            float cost = area(llo, lhi) * nl + area(rlo, rhi) * nr;
            if (cost < best) { best = cost; best_axis = axis; best_bin = s; }
        }
    }
    int me = (int)t.nodes.size();
    t.nodes.push_back(ANode{});
    int mid, axis;
    if (best_axis < 0) {
        return t.nodes.pop_back(), build_median(t, O, idx, l, r);
    } else {
        axis = best_axis;
        float e0 = comp(clo, axis), e1 = comp(chi, axis);
        auto it = std::stable_partition(idx.begin() + l, idx.begin() + r, [&](int o) {
            float c = (comp(aabb_min(O[o]), axis) + comp(aabb_max(O[o]), axis)) * .5f;
            return std::min(NB - 1, (int)((c - e0) / (e1 - e0) * NB)) < best_bin;
        });
        mid = (int)(it - idx.begin());
    }
    int L = build_sah(t, O, idx, l, mid), R = build_sah(t, O, idx, mid, r);
    ANode& n = t.nodes[me];
    n.left = L; n.right = R; n.axis = axis; n.bmin = lo; n.bmax = hi;
    return me;
}

void prepare(const Bvh& bvh) {
    std::lock_guard<std::mutex> g(g_mu);
    if (g_src == &bvh) return;
    Tree t;
    int n_obj = 0;
    for (const Node& n : bvh.nodes) if (n.is_object) n_obj = std::max(n_obj, n.obj + 1);
    t.rank_of_obj.assign(n_obj, 0);
    for (size_t i = 0; i < bvh.nodes.size(); ++i) if (bvh.nodes[i].is_object) t.rank_of_obj[bvh.nodes[i].obj] = bvh.rank[i];
    if (g_mode == 1 || g_mode == 4 || g_mode == 6) {
        for (const Node& n : bvh.nodes) {
            ANode a;
            a.bmin = n.bmin; a.bmax = n.bmax; a.left = n.left; a.right = n.right;
            a.obj = n.is_object ? n.obj : -1;
            t.nodes.push_back(a);
        }
        for (size_t i = 0; i < bvh.nodes.size(); ++i) t.nodes[i].axis = bvh.axis[i];
        t.root = 0;
        if (g_mode == 4 || g_mode == 6) {
            std::vector<int> parent(t.nodes.size(), -1);
            for (size_t i = 0; i < t.nodes.size(); ++i)
                if (t.nodes[i].obj < 0) { parent[t.nodes[i].left] = (int)i; parent[t.nodes[i].right] = (int)i; }
            for (size_t i = 0; i < t.nodes.size(); ++i) {
                if (t.nodes[i].obj < 0 || bvh.objs[t.nodes[i].obj].type != PRIM_PLATFORM) continue;
                t.unbounded.push_back(t.nodes[i].obj);
                int p = parent[i];
                if (p < 0) { t.root = -1; continue; }
                int sib = t.nodes[p].left == (int)i ? t.nodes[p].right : t.nodes[p].left;
                int gp = parent[p];
                parent[sib] = gp;
                if (gp < 0) t.root = sib;
                else if (t.nodes[gp].left == p) t.nodes[gp].left = sib;
                else t.nodes[gp].right = sib;
                for (int a = gp; a >= 0; a = parent[a]) {
                    const ANode &L = t.nodes[t.nodes[a].left], &R = t.nodes[t.nodes[a].right];
                    t.nodes[a].bmin = fmin3(L.bmin, R.bmin);
                    t.nodes[a].bmax = fmax3(L.bmax, R.bmax);
                }
            }
        }
    } else {
        std::vector<int> idx;
        for (int o = 0; o < n_obj; ++o) {
            if (bvh.objs[o].type == PRIM_PLATFORM) t.unbounded.push_back(o);
            else idx.push_back(o);
        }
        if (!idx.empty())
            t.root = g_mode == 2 ? build_median(t, bvh.objs, idx, 0, (int)idx.size())
                                 : build_sah(t, bvh.objs, idx, 0, (int)idx.size());
    }
    if (g_mode == 7 && t.root >= 0 && t.nodes[t.root].obj < 0) {
        // collapse: replace the largest-area internal child by its two children until 4
        std::function<int(int)> collapse = [&](int b) -> int {
            std::vector<int> ch = {t.nodes[b].left, t.nodes[b].right};
            while ((int)ch.size() < (std::getenv("LAB_WIDTH") ? std::atoi(std::getenv("LAB_WIDTH")) : 4)) {
                int best = -1; float ba = -1.f;
                for (size_t k = 0; k < ch.size(); ++k) {
                    const ANode& c = t.nodes[ch[k]];
                    if (c.obj >= 0) continue;
                    const float dx = c.bmax.x - c.bmin.x, dy = c.bmax.y - c.bmin.y, dz = c.bmax.z - c.bmin.z;
                    const float a = dx * dy + dy * dz + dz * dx;
                    if (a > ba) { ba = a; best = (int)k; }
                }
                if (best < 0) break;
                const int c = ch[best];
                ch.erase(ch.begin() + best);
                ch.insert(ch.begin() + best, {t.nodes[c].left, t.nodes[c].right});
            }
            // octant orders: near-first by the binary subtree's split axes, via a recursive
            // order over the binary nodes between b and its wide children
            const int me = (int)t.wide.size();
            t.wide.push_back(WNode{});
            t.wbox.push_back(t.nodes[b]);
            std::vector<int> wch(ch.size());
            for (size_t k = 0; k < ch.size(); ++k) wch[k] = t.nodes[ch[k]].obj >= 0 ? -1 - ch[k] : collapse(ch[k]);
            WNode& w = t.wide[me];
            w.n = (int)ch.size();
            for (int o = 0; o < 8; ++o) {
                std::vector<int> ord;
                std::function<void(int)> rec = [&](int x) {
                    for (size_t k = 0; k < ch.size(); ++k) if (ch[k] == x) { ord.push_back(wch[k]); return; }
                    const ANode& n = t.nodes[x];
                    const bool neg = (o >> n.axis) & 1;
                    rec(neg ? n.right : n.left);
                    rec(neg ? n.left : n.right);
                };
                rec(b);
                for (int k = 0; k < w.n; ++k) t.wide[me].child[o][k] = ord[k];
            }
            return me;
        };
        t.wroot = collapse(t.root);
    }
    g_tree = std::move(t);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    g_src = &bvh;
}

bool slab_ok(const ANode& n, const Ray& ray) {
    Node m;
    m.bmin = n.bmin; m.bmax = n.bmax;
    if (g_mode < 5) return slab_pass(m, ray);
    // conservative: the product's slab (f32 reciprocals, cpt_path.hpp slab_reject<FAST, true>)
    const float BIG = DEFAULT_RAY_TMAX * 2;
    const float o[3] = {ray.origin.x, ray.origin.y, ray.origin.z}, d[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
    const float a[3] = {n.bmin.x, n.bmin.y, n.bmin.z}, b[3] = {n.bmax.x, n.bmax.y, n.bmax.z};
    float l[3], h[3];
    for (int k = 0; k < 3; ++k) {
        const float inv = fabsf(d[k]) >= 1e-30f ? 1.0f / d[k] : 0.0f;
        const float t0 = (a[k] - o[k]) * inv, t1 = (b[k] - o[k]) * inv;
        l[k] = inv != 0.f ? fminf(t0, t1) : -BIG;
        h[k] = inv != 0.f ? fmaxf(t0, t1) : BIG;
    }
    float lo = fmaxf(fmaxf(l[0], l[1]), l[2]);
    float hi = fminf(fminf(h[0], h[1]), h[2]);
    lo = lo - (g_margin * fabsf(lo) + 1e-4f);
    hi = hi + (g_margin * fabsf(hi) + 1e-4f);
    return !(lo > hi || lo > ray.tmax || hi < ray.tmin);
}

std::atomic<uint64_t> g_boxes{0}, g_stale{0};

bool alt_trace(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, uint64_t& nodes, uint64_t& prims) {
    const Tree& t = g_tree;
    bool ret = false;
    int best_rank = 0x7fffffff;
    auto test = [&](int o) {
        prims++;
        Ray r2 = ray;
        if (t.rank_of_obj[o] < best_rank) {
            uint32_t u;
            std::memcpy(&u, &r2.tmax, 4);
            u += 1;
            std::memcpy(&r2.tmax, &u, 4);
        }
        if (g_mode >= 5 && bvh.objs[o].type != PRIM_PLATFORM) {
            ANode box;
            box.bmin = aabb_min(bvh.objs[o]);
            box.bmax = aabb_max(bvh.objs[o]);
            if (!slab_ok(box, r2)) {
                Ray r3 = r2;
                Attr a3 = attr;
                if (intersection_test(bvh.objs[o], r3, a3)) {
                    g_pretest_miss++;
                    std::lock_guard<std::mutex> g(g_mu);
                    if (g_pretest_miss <= 5)
                        fprintf(stderr, "pretest-miss: type=%d o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) tmin=%g t=%.9g tmax=%.9g c=(%.9g %.9g %.9g) r=%.9g h=%.9g\n",
                                bvh.objs[o].type, ray.origin.x, ray.origin.y, ray.origin.z, ray.dir.x, ray.dir.y, ray.dir.z,
                                ray.tmin, r3.tmax, r2.tmax, bvh.objs[o].center.x, bvh.objs[o].center.y, bvh.objs[o].center.z,
                                bvh.objs[o].radius, bvh.objs[o].height);
                }
                return;
            }
        }
        if (intersection_test(bvh.objs[o], r2, attr)) {
            ray.tmax = r2.tmax;
            hit_obj = o;
            best_rank = t.rank_of_obj[o];
            ret = true;
        }
    };
    for (int o : t.unbounded) test(o);
    if (t.root < 0) return ret;
    if (g_mode == 7 && t.wroot >= 0) {
        const int oct = (ray.dir.x < 0.f ? 1 : 0) | (ray.dir.y < 0.f ? 2 : 0) | (ray.dir.z < 0.f ? 4 : 0);
        int st[512], tp = 0;
        st[tp++] = t.wroot;
        while (tp > 0) {
            const int x = st[--tp];
            if (std::getenv("LAB_CULL")) {   // re-test the popped entry's box at the current tmax
                ANode box;
                if (x < 0) box = t.nodes[-1 - x];
                else { box.bmin = t.wbox[x].bmin; box.bmax = t.wbox[x].bmax; }
                if (x != t.wroot && !slab_ok(box, ray)) { g_stale++; continue; }
            }
            nodes++;                       // iterations (pops)
            if (x < 0) { test(t.nodes[-1 - x].obj); continue; }
            const WNode& w = t.wide[x];
            int hit[8], nh = 0;
            float ent[8];
            for (int k = 0; k < w.n; ++k) {
                const int c = w.child[oct][k];
                g_boxes++;
                const ANode& cn = c < 0 ? t.nodes[-1 - c] : t.nodes[0];
                ANode box;
                if (c < 0) box = cn;
                else { box.bmin = t.wbox[c].bmin; box.bmax = t.wbox[c].bmax; }
                if (slab_ok(box, ray)) {
                    const float o3[3] = {ray.origin.x, ray.origin.y, ray.origin.z}, d3[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
                    const float a3[3] = {box.bmin.x, box.bmin.y, box.bmin.z}, b3[3] = {box.bmax.x, box.bmax.y, box.bmax.z};
                    float e = -1e30f;
                    for (int q = 0; q < 3; ++q)
                        if (d3[q] != 0.f) e = std::max(e, std::min((a3[q] - o3[q]) / d3[q], (b3[q] - o3[q]) / d3[q]));
                    ent[nh] = e;
                    hit[nh++] = c;
                }
            }
            if (std::getenv("LAB_SORT"))   // nearest entry distance first (dynamic order)
                for (int i = 1; i < nh; ++i)
                    for (int j = i; j > 0 && ent[j] < ent[j - 1]; --j) { std::swap(ent[j], ent[j - 1]); std::swap(hit[j], hit[j - 1]); }
            for (int k = nh - 1; k >= 0; --k) st[tp++] = hit[k];
        }
        return ret;
    }
    int stack[512], top = 0;
    stack[top++] = t.root;
    const float d[3] = {ray.dir.x, ray.dir.y, ray.dir.z};
    while (top > 0) {
        const ANode& n = t.nodes[stack[--top]];
        nodes++;
        if (n.obj >= 0) { test(n.obj); continue; }
        if (!slab_ok(n, ray)) continue;
        const bool right_first = d[n.axis] < 0.f;
        stack[top++] = right_first ? n.left : n.right;
        stack[top++] = right_first ? n.right : n.left;
    }
    return ret;
}

bool hook(const Bvh& bvh, Ray ray, Attr& attr, int& hit_obj, Stats& st) {
    if (g_src != &bvh) prepare(bvh);
    Attr a2 = attr;
    int h2 = -1;
    uint64_t nodes = 0, prims = 0;
    bool r2 = alt_trace(bvh, ray, a2, h2, nodes, prims);
    const Attr a_in = attr;
    bool r = trace_ray_ref(bvh, ray, attr, hit_obj, st);
    if (g_mode >= 5 && r2) {
        // certificate: the winner's own AABB passes the exact slab test at tmax = t_win
        Node m;
        m.bmin = aabb_min(bvh.objs[h2]);
        m.bmax = aabb_max(bvh.objs[h2]);
        Ray rc = ray;
        // t_win from the hit position is not exact; recompute by re-testing the winner alone
        Attr tmp = a_in;
        rc.tmax = DEFAULT_RAY_TMAX;
        Ray rw = ray;
        rw.tmax = DEFAULT_RAY_TMAX;
        intersection_test(bvh.objs[h2], rw, tmp);
        rc.tmax = rw.tmax;
        if (!slab_pass(m, rc)) {
            g_fallback++;
            r2 = r; h2 = hit_obj; a2 = attr;   // fallback: the reference walk's result
        }
    }
    g_nodes += nodes;
    g_prims += prims;
    g_segments++;
    if (r != r2 || (r && (h2 != hit_obj || std::memcmp(&a2, &attr, sizeof(Attr)) != 0))) {
        g_diff++;
        if (r != r2 || h2 != hit_obj) g_diff_obj++;
        std::lock_guard<std::mutex> g(g_mu);
        if (g_diff <= 8)
            fprintf(stderr, "diff: o=(%.9g %.9g %.9g) d=(%.9g %.9g %.9g) tmin=%g | ref hit=%d obj=%d t=%.9g type=%d | alt hit=%d obj=%d type=%d pos=(%.9g %.9g %.9g)\n",
                    ray.origin.x, ray.origin.y, ray.origin.z, ray.dir.x, ray.dir.y, ray.dir.z, ray.tmin, (int)r, hit_obj,
                    r ? attr.hit_pos.x : 0.f, r ? bvh.objs[hit_obj].type : -1, (int)r2, h2, r2 ? bvh.objs[h2].type : -1,
                    a2.hit_pos.x, a2.hit_pos.y, a2.hit_pos.z);
    }
    return r;
}

}  // namespace lab

extern "C" {
void lab_set_margin(float m) { lab::g_margin = m; }
void lab_set_mode(int m) {
    lab::g_mode = m;
    lab::g_src = nullptr;
    g_trace_hook = m ? lab::hook : nullptr;
}
void lab_counts(uint64_t out[6]) {
    out[0] = lab::g_segments; out[1] = lab::g_nodes; out[2] = lab::g_prims; out[3] = lab::g_diff; out[4] = lab::g_diff_obj;
    out[5] = lab::g_fallback;
    fprintf(stderr, "pretest misses: %llu, wide box tests/seg %.2f\n", (unsigned long long)lab::g_pretest_miss.load(),
            lab::g_segments ? (double)lab::g_boxes.load() / lab::g_segments : 0.0);
    fprintf(stderr, "stale pops/seg %.3f\n", lab::g_segments ? (double)lab::g_stale.load() / lab::g_segments : 0.0);
    lab::g_boxes = 0;
    lab::g_stale = 0;
    lab::g_pretest_miss = 0;
    lab::g_segments = lab::g_nodes = lab::g_prims = lab::g_diff = lab::g_diff_obj = lab::g_fallback = 0;
}
}
