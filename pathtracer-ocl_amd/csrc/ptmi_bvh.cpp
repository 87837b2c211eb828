// ptmi_bvh.cpp -- traversal structure for the triangles of one reference BVH root.
//
// The reference walks its own BVH (CLGroup preorder array, tracer.cl:617-719):
// a triangle of node g is a candidate of a ray iff the ray's LINE passes the
// reference box test (intersectRayWithBox, tracer.cl:270-280) of every node on
// the path root -> g.  That tree keeps 46 % of the teapot's triangles on inner
// nodes (up to 305 per node, bvh.go:92-119), so walking it costs hundreds of
// triangle tests per ray.
//
// Here each root's triangles get a second, independent index: a 4-wide SAH BVH
// with conservatively widened boxes.  The kernel uses it to FIND the triangles
// a ray hits, then admits a hit as a candidate only after checking the
// reference gate above for that triangle (its "chain": the boxes of the
// reference nodes strictly below the root down to g, tested with the
// reference's exact arithmetic).  Candidate set and tie-break order are the
// reference's, so the winner is too; see DESIGN.md "Parity contract".
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ptmi.h"
#include "ptmi_bvh.h"
#include "ptmi_f16.h"

namespace ptmi {
namespace {

template <typename T>
T rd(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    return v;
}

struct Prim {
    double mn[3], mx[3], c[3];
    int32_t tri;    // reference triangle index
    int32_t chain;  // (chain offset << 5) | chain length
};

struct BNode {  // binary build node
    double mn[3], mx[3];
    int left = -1, right = -1;  // inner: children; leaf: left = -1
    int first = 0, count = 0;   // leaf: prims [first, first + count)
};

constexpr int kLeafMax = 7;         // 3-bit count in the leaf entry code
constexpr int kMaxBinaryDepth = 14; // binary leaves at depth <= 14, so BVH4 chains of <= 7 nodes
constexpr int kMaxNode4Depth = 7;   // 3 pushes per Node4 level: the kernel's stack needs 21 entries
constexpr int kBins = 32;

double area(const double* mn, const double* mx) {
    const double dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
    return (dx < 0 || dy < 0 || dz < 0) ? 0.0 : 2.0 * (dx * dy + dy * dz + dz * dx);
}

void grow(double* mn, double* mx, const double* a, const double* b) {
    for (int k = 0; k < 3; k++) {
        mn[k] = std::min(mn[k], a[k]);
        mx[k] = std::max(mx[k], b[k]);
    }
}

struct Builder {
    std::vector<Prim>& prims;
    std::vector<BNode> nodes;
    double c_tri = 2.0;        // SAH cost of a triangle test relative to a node visit
    int leaf_max = kLeafMax;   // triangles per leaf (<= kLeafMax)
    explicit Builder(std::vector<Prim>& p) : prims(p) {
#if defined(PTMI_STUDY) && PTMI_STUDY  // study build only: the SAH / leaf-size sweeps (tools/bvh_sweep.sh)
        if (const char* e = std::getenv("PTMI_BVH_CTRI")) c_tri = std::atof(e);
        if (const char* e = std::getenv("PTMI_BVH_LEAF")) leaf_max = std::max(1, std::min(kLeafMax, std::atoi(e)));
#endif
    }

    int make_leaf(int lo, int hi, const double* mn, const double* mx) {
        BNode n;
        std::memcpy(n.mn, mn, 24);
        std::memcpy(n.mx, mx, 24);
        n.first = lo;
        n.count = hi - lo;
        nodes.push_back(n);
        return (int)nodes.size() - 1;
    }

    int build(int lo, int hi, int depth) {
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        double cmn[3] = {INFINITY, INFINITY, INFINITY}, cmx[3] = {-INFINITY, -INFINITY, -INFINITY};
        for (int i = lo; i < hi; i++) {
            grow(mn, mx, prims[i].mn, prims[i].mx);
            grow(cmn, cmx, prims[i].c, prims[i].c);
        }
        const int n = hi - lo;
        if (n <= 2) return make_leaf(lo, hi, mn, mx);
        // Depth budget: when the remaining levels barely suffice for a balanced
        // tree, split at the median (guarantees depth <= kMaxBinaryDepth).
        int need = 0;
        while ((leaf_max << need) < n) need++;
        int axis = 0;
        for (int k = 1; k < 3; k++)
            if (cmx[k] - cmn[k] > cmx[axis] - cmn[axis]) axis = k;
        int mid = -1;
        if (need + 1 >= kMaxBinaryDepth - depth || cmx[axis] - cmn[axis] <= 0.0) {
            if (n <= leaf_max) return make_leaf(lo, hi, mn, mx);
            mid = (lo + hi) / 2;
            std::nth_element(prims.begin() + lo, prims.begin() + mid, prims.begin() + hi,
                             [axis](const Prim& a, const Prim& b) {
                                 return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.tri < b.tri);
                             });
        } else {
            // Binned SAH over all three axes.
            double best = INFINITY;
            int best_axis = -1, best_bin = -1;
            for (int k = 0; k < 3; k++) {
                const double ext = cmx[k] - cmn[k];
                if (ext <= 0.0) continue;
                double bmn[kBins][3], bmx[kBins][3];
                int bc[kBins] = {0};
                for (int b = 0; b < kBins; b++)
                    for (int q = 0; q < 3; q++) bmn[b][q] = INFINITY, bmx[b][q] = -INFINITY;
                const double s = kBins / ext;
                for (int i = lo; i < hi; i++) {
                    int b = std::min(kBins - 1, (int)((prims[i].c[k] - cmn[k]) * s));
                    bc[b]++;
                    grow(bmn[b], bmx[b], prims[i].mn, prims[i].mx);
                }
                double rmn[3] = {INFINITY, INFINITY, INFINITY}, rmx[3] = {-INFINITY, -INFINITY, -INFINITY};
                double ra[kBins];
                int rc[kBins];
                int cnt = 0;
                for (int b = kBins - 1; b > 0; b--) {
                    grow(rmn, rmx, bmn[b], bmx[b]);
                    cnt += bc[b];
                    ra[b] = area(rmn, rmx) * cnt;
                    rc[b] = cnt;
                }
                double lmn[3] = {INFINITY, INFINITY, INFINITY}, lmx[3] = {-INFINITY, -INFINITY, -INFINITY};
                cnt = 0;
                for (int b = 0; b < kBins - 1; b++) {
                    grow(lmn, lmx, bmn[b], bmx[b]);
                    cnt += bc[b];
                    if (cnt == 0 || rc[b + 1] == 0) continue;
                    const double cost = area(lmn, lmx) * cnt + ra[b + 1];
                    if (cost < best) {
                        best = cost;
                        best_axis = k;
                        best_bin = b;
                    }
                }
            }
            // SAH: a node visit costs 1 (four FP32 slab tests), a triangle test
            // c_tri (FP64 Moller-Trumbore), in units of the parent's area.
            const double leaf_cost = area(mn, mx) * n * c_tri;
            if (n <= leaf_max && (best_axis < 0 || leaf_cost <= area(mn, mx) + c_tri * best))
                return make_leaf(lo, hi, mn, mx);
            if (best_axis < 0) {
                mid = (lo + hi) / 2;
                std::nth_element(prims.begin() + lo, prims.begin() + mid, prims.begin() + hi,
                                 [axis](const Prim& a, const Prim& b) {
                                     return a.c[axis] < b.c[axis] || (a.c[axis] == b.c[axis] && a.tri < b.tri);
                                 });
            } else {
                const double s = kBins / (cmx[best_axis] - cmn[best_axis]);
                const double c0 = cmn[best_axis];
                auto it = std::partition(prims.begin() + lo, prims.begin() + hi, [&](const Prim& p) {
                    return std::min(kBins - 1, (int)((p.c[best_axis] - c0) * s)) <= best_bin;
                });
                mid = (int)(it - prims.begin());
                if (mid == lo || mid == hi) mid = (lo + hi) / 2;
            }
        }
        const int me = (int)nodes.size();
        nodes.emplace_back();
        const int l = build(lo, mid, depth + 1);
        const int r = build(mid, hi, depth + 1);
        BNode& nd = nodes[me];
        std::memcpy(nd.mn, mn, 24);
        std::memcpy(nd.mx, mx, 24);
        nd.left = l;
        nd.right = r;
        return me;
    }
};

// The builder's leaf code (ptmi_device.h Node4): the leaf's first triangle behind the wide
// leaf bit; its last triangle carries kLastTri.  finalize_index_codes re-codes the whole
// scene's index once every object is built.
int32_t leaf_code(int32_t first) { return kLeafWide | first; }


}  // namespace

int build_object_index(const uint8_t* tris, const std::vector<DevNode>& nodes, const std::vector<int32_t>& tri_off,
                       const std::vector<int32_t>& tri_cnt, const int32_t* roots, int n_roots, const double* gate_mn,
                       const double* gate_mx, RootIndex& out, RootRec* rec, char* err, size_t err_len) {
    *rec = RootRec{};
    rec->sc = 1.0f;
    int32_t* entry = &rec->entry;
    const int32_t root = n_roots > 0 ? roots[0] : -1;  // for messages
    // Reference subtrees of the object's roots (children > 0 are present,
    // tracer.cl:683/704), each node with its gate chain: the path from its root.
    // A triangle reachable from two roots appears twice, each with its own chain
    // (the reference tests it once per root walk).
    std::vector<Prim> prims;
    std::vector<std::pair<int32_t, std::vector<int32_t>>> todo;
    for (int i = n_roots - 1; i >= 0; i--) todo.push_back({roots[i], {roots[i]}});
    while (!todo.empty()) {
        auto [g, path] = todo.back();
        todo.pop_back();
        if (path.size() > 30) {
            std::snprintf(err, err_len, "reference BVH deeper than 29 levels below root %d", root);
            return PTMI_ERR_UNSUPPORTED;
        }
        // The chain: the group object's own gate box (tracer.cl:609), then the
        // boxes of the reference nodes from the root down to this node (617-719).
        const int32_t off = (int32_t)out.chain_boxes.size();
        ChainBox core;  // the intersection of the chain's boxes, stored after them
        for (int k = 0; k < 3; k++) core.mn[k] = -HUGE_VAL, core.mx[k] = HUGE_VAL;
        for (size_t i = 0; i <= path.size(); i++) {
            ChainBox b;
            if (i == 0) {
                std::memcpy(b.mn, gate_mn, 24);
                std::memcpy(b.mx, gate_mx, 24);
            } else {
                std::memcpy(b.mn, nodes[path[i - 1]].bb_min, 24);
                std::memcpy(b.mx, nodes[path[i - 1]].bb_max, 24);
            }
            out.chain_boxes.push_back(b);
            for (int a = 0; a < 3; a++) {
                core.mn[a] = std::max(core.mn[a], b.mn[a]);  // NaN bounds leave the core unbounded
                core.mx[a] = std::min(core.mx[a], b.mx[a]);  // there: no certificate is issued (NaN test)
                if (b.mn[a] != b.mn[a] || b.mx[a] != b.mx[a]) core.mn[a] = core.mx[a] = NAN;
            }
        }
        out.chain_boxes.push_back(core);
        const int32_t chain = (off << 5) | (int32_t)(path.size() + 1);
        for (int32_t t = tri_off[g]; t < tri_off[g] + tri_cnt[g]; t++) {
            const uint8_t* b = tris + (size_t)PTMI_TRIANGLE_BYTES * t;
            Prim p;
            double v[5][3];
            for (int k = 0; k < 3; k++) {
                v[0][k] = rd<double>(b + 0 + 8 * k);
                v[1][k] = rd<double>(b + 32 + 8 * k);
                v[2][k] = rd<double>(b + 64 + 8 * k);
                v[3][k] = v[0][k] + rd<double>(b + 96 + 8 * k);   // the p1 + e1, p1 + e2 that
                v[4][k] = v[0][k] + rd<double>(b + 128 + 8 * k);  // Moller-Trumbore spans
            }
            for (int k = 0; k < 3; k++) {
                p.mn[k] = p.mx[k] = v[0][k];
                for (int i = 1; i < 5; i++) {
                    p.mn[k] = std::min(p.mn[k], v[i][k]);
                    p.mx[k] = std::max(p.mx[k], v[i][k]);
                }
                p.c[k] = 0.5 * (p.mn[k] + p.mx[k]);
            }
            p.tri = t;
            p.chain = chain;
            prims.push_back(p);
        }
        for (int32_t c : {nodes[g].child1, nodes[g].child0})
            if (c > 0) {
                auto q = path;
                q.push_back(c);
                todo.push_back({c, q});
            }
    }
    if (prims.empty()) {  // nothing to intersect: an empty hull no slab test passes
        *entry = kEmptyChild;
        for (int k = 0; k < 3; k++) rec->hull_mn[k] = 1.0, rec->hull_mx[k] = -1.0;
        return PTMI_OK;
    }
    if (prims.size() > ((size_t)kLeafMax << kMaxBinaryDepth)) {
        std::snprintf(err, err_len, "BVH root %d holds %zu triangles (max %d per root)", root, prims.size(),
                      kLeafMax << kMaxBinaryDepth);
        return PTMI_ERR_UNSUPPORTED;
    }
    // Non-finite vertices would void the conservative box argument.
    for (const Prim& p : prims)
        for (int k = 0; k < 3; k++)
            if (!std::isfinite(p.mn[k]) || !std::isfinite(p.mx[k])) {
                std::snprintf(err, err_len, "triangle %d has non-finite vertices", p.tri);
                return PTMI_ERR_UNSUPPORTED;
            }
    Builder B(prims);
    const int broot = B.build(0, (int)prims.size(), 0);

    // Conservative widening: far beyond the ~1e-15 relative error of a computed
    // Moller-Trumbore hit point and of the slab arithmetic in the kernel.
    double scale = 0.0;
    for (const Prim& p : prims)
        for (int k = 0; k < 3; k++) scale = std::max({scale, std::fabs(p.mn[k]), std::fabs(p.mx[k])});
    const double m = 1e-7 * scale + 1e-300;
    // The root's frame (RootRec): Node4 bounds are stored as (bound - ctr) / 2^s, ctr
    // the hull centre rounded to float (an exact double, so the kernel's o - ctr is one
    // double rounding), 2^s the smallest power of two (s in [0, 28]) that brings the
    // root's extent under 2^15.  A mesh far from the origin keeps binary16's 11
    // significant bits on its own extent instead of on its distance from the origin,
    // and one larger than binary16's range keeps finite bounds.  The double subtraction
    // rounds by <= 2^-52 scale, far inside the widening m.
    double ext = 0.0;
    for (int k = 0; k < 3; k++) {
        const BNode& hb = B.nodes[broot];
        rec->hull_mn[k] = hb.mn[k] - m;
        rec->hull_mx[k] = hb.mx[k] + m;
        const float c = (float)(0.5 * hb.mn[k] + 0.5 * hb.mx[k]);
        rec->ctr[k] = std::isfinite(c) ? (double)c : 0.0;
        ext = std::max({ext, std::fabs(rec->hull_mn[k] - rec->ctr[k]), std::fabs(rec->hull_mx[k] - rec->ctr[k])});
    }
    int s = 0;
    while (s < 28 && ext > std::ldexp(32768.0, s)) s++;
    const double inv_sc = std::ldexp(1.0, -s), sc = std::ldexp(1.0, s);
    rec->sc = (float)sc;
    // Node4 bounds: binary16, rounded outward from the widened doubles in the root's
    // frame (+-infinity past the binary16 range: still conservative, and exact in the
    // kernel's slab arithmetic; bmax, its error bound, runs over the finite bounds, in
    // object-space units relative to ctr).
    auto bound_abs = [sc](uint16_t h) {
        const double v = std::fabs(f16_value(h)) * sc;
        return std::isfinite(v) ? (float)v : 0.0f;
    };
    float bmax = 0.0f;

    // Triangles in leaf order.
    const int32_t tri_base = (int32_t)out.tris.size();
    std::vector<int32_t> leaf_first(B.nodes.size(), 0);
    for (size_t i = 0; i < B.nodes.size(); i++) {
        const BNode& n = B.nodes[i];
        if (n.left >= 0) continue;
        leaf_first[i] = (int32_t)out.tris.size();
        std::vector<Prim> lp(prims.begin() + n.first, prims.begin() + n.first + n.count);
        std::sort(lp.begin(), lp.end(), [](const Prim& a, const Prim& b) { return a.tri < b.tri; });
        for (const Prim& p : lp) {
            const uint8_t* b = tris + (size_t)PTMI_TRIANGLE_BYTES * p.tri;
            DevTri t{};
            std::memcpy(t.p1, b + 0, 24);
            std::memcpy(t.e1, b + 96, 24);
            std::memcpy(t.e2, b + 128, 24);
            t.n = p.tri;
            t.chain = p.chain;
            out.tris.push_back(t);
        }
        out.tris.back().chain |= kLastTri;  // the leaf ends here (ptmi_kernels.hip leaf_visit)
    }
    (void)tri_base;
    auto code_of = [&](int bi) -> int32_t {
        const BNode& n = B.nodes[bi];
        return n.left < 0 ? leaf_code(leaf_first[bi]) : -2;  // -2: inner, resolved below
    };
    // Collapse the binary tree to 4-wide nodes (children = grandchildren of
    // inner children), emitted breadth first: the top levels of the first
    // object's index are the first Node4s, which the kernel stages in LDS.
    std::vector<std::pair<int, int>> work;  // (binary node, Node4 slot), a FIFO
    std::vector<int> level;                 // 1-based Node4 level of work[i]
    size_t work_head = 0;
    int cur_level = 0;
    auto emit = [&](int bi) -> int32_t {
        if (B.nodes[bi].left < 0) return code_of(bi);
        const int32_t slot = (int32_t)out.nodes.size();
        out.nodes.emplace_back();
        work.push_back({bi, slot});
        level.push_back(cur_level + 1);
        return slot;
    };
    *entry = emit(broot);
    while (work_head < work.size()) {
        cur_level = level[work_head];
        // The kernel's traversal stack holds 3 entries per Node4 level (kStack >= 21).
        if (cur_level > kMaxNode4Depth) {
            std::snprintf(err, err_len, "BVH4 of root %d deeper than %d levels", root, kMaxNode4Depth);
            return PTMI_ERR_UNSUPPORTED;
        }
        auto [bi, slot] = work[work_head++];
        int kids[4], nk = 0;
        for (int c : {B.nodes[bi].left, B.nodes[bi].right}) {
            if (B.nodes[c].left >= 0) {
                kids[nk++] = B.nodes[c].left;
                kids[nk++] = B.nodes[c].right;
            } else {
                kids[nk++] = c;
            }
        }
        Node4 nd{};
        for (int i = 0; i < 4; i++) {
            if (i < nk) {
                const BNode& c = B.nodes[kids[i]];
                for (int k = 0; k < 3; k++) {
                    nd.bnd[k][0][i] = f16_down(((c.mn[k] - m) - rec->ctr[k]) * inv_sc);
                    nd.bnd[k][1][i] = f16_up(((c.mx[k] + m) - rec->ctr[k]) * inv_sc);
                    bmax = std::max({bmax, bound_abs(nd.bnd[k][0][i]), bound_abs(nd.bnd[k][1][i])});
                }
                nd.child[i] = 0;  // patched after emit (emit may grow out.nodes)
            } else {
                // an empty slot: a point box at +infinity, culled by the kernel's slab
                // test for every ray (ptmi_kernels.hip node_children)
                for (int k = 0; k < 3; k++) nd.bnd[k][0][i] = nd.bnd[k][1][i] = kF16Inf;
                nd.child[i] = kEmptyChild;
            }
        }
        for (int i = 0; i < nk; i++) nd.child[i] = emit(kids[i]);
        out.nodes[slot] = nd;
    }
    rec->bmax = bmax;
    return PTMI_OK;
}

int32_t finalize_index_codes(RootIndex& idx, std::vector<RootRec>& recs) {
    // The sentinel: one degenerate triangle (zero edges: |det| = 0 < EPSILON for every finite
    // ray, and NaN comparisons for a NaN ray), the target of every empty slot.
    DevTri z{};
    z.n = 0;
    z.chain = kLastTri;
    idx.tris.push_back(z);
    const int32_t sentinel = (int32_t)idx.tris.size() - 1;
    const bool narrow = idx.nodes.size() < (size_t)kLeafNarrow && sentinel < kLeafNarrow;
    const int32_t lb = narrow ? kLeafNarrow : kLeafWide;
    auto recode = [&](int32_t c) -> int32_t {
        if (c == kEmptyChild) return lb | sentinel;
        if (c >= kLeafWide) return lb | (c - kLeafWide);
        return c;  // a Node4 index
    };
    for (Node4& nd : idx.nodes)
        for (int i = 0; i < 4; i++) nd.child[i] = recode(nd.child[i]);
    for (RootRec& r : recs) r.entry = recode(r.entry);
#if defined(PTMI_STACKLESS) && PTMI_STACKLESS
    // DIAGNOSTIC stackless walk (ptmi_kernels.hip walk_index_stackless): each Node4's parent in
    // the high half of its child[0] (16-bit codes leave it free; 0xFFFF at a root).
    if (narrow) {
        std::vector<uint32_t> parent(idx.nodes.size(), 0xFFFFu);
        for (size_t n = 0; n < idx.nodes.size(); n++)
            for (int i = 0; i < 4; i++)
                if (idx.nodes[n].child[i] < lb) parent[idx.nodes[n].child[i]] = (uint32_t)n;
        for (size_t n = 0; n < idx.nodes.size(); n++)
            idx.nodes[n].child[0] = (int32_t)(((uint32_t)idx.nodes[n].child[0] & 0xFFFFu) | (parent[n] << 16));
    }
#endif
    return lb;
}

}  // namespace ptmi
