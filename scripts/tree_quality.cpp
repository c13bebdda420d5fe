// CPU study: how many four-wide node visits and leaf gates does a bounce ray
// of the BASELINE scenes cost on (A) the four-wide tree the library derives
// from the reference's own tree (render.hip build_hnodes: live_node chain
// collapse, greedy four-slot cut) against (B) a four-wide tree built afresh
// over the same live leaves by a binned SAH?
//
// Exactness does not depend on the inner structure: the reference reaches a
// leaf iff the ray passes the leaf's own box (boxes nest and the slab test is
// monotone under containment), so any tree over the live
// leaves whose inner boxes contain their leaves', gated by the exact leaf box
// and the sphere test, finds the same closest hit. This program only counts
// work; the walk is the kernel's (nearest slot first, entry-beyond-best
// pruning), in plain float.
//
//   g++ -O2 -std=c++17 -Iinclude scripts/tree_quality.cpp \
//       -Lcs201_sah-bvh_ray_tracer_amd -lmirt -Wl,-rpath,$PWD/cs201_sah-bvh_ray_tracer_amd -o /tmp/tq
//   /tmp/tq [n_spheres] [scene: render|bench] [pixel stride] [bins] [leaf_max]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <tuple>
#include <vector>

#include "mirt.h"

namespace {

struct Box {
    float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
    void grow(const Box& b)
    {
        for (int k = 0; k < 3; k++) {
            lo[k] = std::min(lo[k], b.lo[k]);
            hi[k] = std::max(hi[k], b.hi[k]);
        }
    }
    float area() const
    {
        const float dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
        return dx < 0 ? 0.0f : dx * dy + dy * dz + dz * dx;
    }
};

struct Leaf {
    Box box;
    int sphere;
};

// four-wide node: slot >= 0 inner node, slot < 0 leaf ~slot, INT32_MIN none
constexpr int kMaxWide = 8;
int g_quant = 0;  // argv[10]: 1 = 8-bit slot boxes in the node's frame (fp32 origin), 2 = fp16 origin
int g_wide = 4;  // slots per node of tree A (argv[9]: 4 as the library, 8 to price an eight-wide layout)
struct W4 {
    Box box[kMaxWide];
    int ref[kMaxWide];
    int pos[kMaxWide];  // octant position of each slot (g_order 1)
    int n = 0;
};
int g_order = 0;  // argv[11]: 0 = passing slots sorted by entry; 1 = fixed octant order (no sort)
int g_popcheck = 1;  // argv[12]: 1 = a popped entry beyond best is dropped unvisited; 0 = visited (the kernel)

// Slots to octant positions 0..7 (bit a set: the slot's centre lies on the
// + side of the node's centre on axis a), greedily by how far each slot lies
// along each position's diagonal; a ray then takes its passing slots in the
// order p ^ s (s: the sign bits of its direction), near side first.
void assign_positions(W4& w)
{
    Box all;
    for (int k = 0; k < w.n; k++) all.grow(w.box[k]);
    float cen[3];
    for (int a = 0; a < 3; a++) cen[a] = 0.5f * (all.lo[a] + all.hi[a]);
    std::vector<std::tuple<float, int, int>> cand;
    for (int k = 0; k < w.n; k++) {
        float c[3];
        for (int a = 0; a < 3; a++)
            c[a] = (w.box[k].lo[a] <= w.box[k].hi[a]) ? 0.5f * (w.box[k].lo[a] + w.box[k].hi[a]) - cen[a] : 0.0f;
        for (int p = 0; p < 8; p++) {
            float d = 0;
            for (int a = 0; a < 3; a++) d += ((p >> a) & 1) ? c[a] : -c[a];
            cand.emplace_back(-d, k, p);
        }
    }
    std::sort(cand.begin(), cand.end());
    bool used_k[kMaxWide] = {}, used_p[8] = {};
    for (auto& [cost, k, p] : cand) {
        if (used_k[k] || used_p[p]) continue;
        used_k[k] = used_p[p] = true;
        w.pos[k] = p;
    }
}

struct Tree {
    std::vector<W4> nodes;
    int root_ref;
    Box root_box;
};

// ---------------------------------------------------------------- tree A
const mirt_node* g_nd;
int g_ns;
std::vector<int> g_leaf_of;  // flat node -> leaf index

bool dead(uint32_t i) { return g_nd[i].sphere >= 0 && ((g_nd[i].skip & MIRT_NODE_EMPTY) || g_nd[i].sphere >= g_ns); }
uint32_t live(uint32_t ci)
{
    for (;;) {
        if (g_nd[ci].sphere >= 0) return dead(ci) ? 0xffffffffu : ci;
        const uint32_t l = ci + 1, r = g_nd[ci + 1].skip & MIRT_SKIP_MASK;
        const bool dl = dead(l), dr = dead(r);
        if (dl && dr) return 0xffffffffu;
        if (!dl && !dr) return ci;
        ci = dl ? r : l;
    }
}
Box nbox(uint32_t i)
{
    Box b;
    std::memcpy(b.lo, g_nd[i].bmin, 12);
    std::memcpy(b.hi, g_nd[i].bmax, 12);
    return b;
}

int build_a(Tree& t, uint32_t y)  // HNode of inner node y (its greedy four-slot cut)
{
    uint32_t cut[kMaxWide + 1];
    int m = 0;
    auto add = [&](uint32_t c) {
        const uint32_t ci = live(c);
        if (ci != 0xffffffffu) cut[m++] = ci;
    };
    add(y + 1);
    add(g_nd[y + 1].skip & MIRT_SKIP_MASK);
    while (m < g_wide) {
        int best = -1;
        float ba = -1;
        for (int j = 0; j < m; j++) {
            if (g_nd[cut[j]].sphere >= 0) continue;
            const float a = nbox(cut[j]).area();
            if (a > ba || best < 0) {
                best = j;
                ba = a;
            }
        }
        if (best < 0) break;
        const uint32_t c = cut[best];
        cut[best] = cut[--m];
        add(c + 1);
        add(g_nd[c + 1].skip & MIRT_SKIP_MASK);
    }
    const int me = (int)t.nodes.size();
    t.nodes.emplace_back();
    // g_quant: slot boxes stored as 8-bit codes in the node's own frame
    // (origin = the slots' min corner, per axis a power-of-two step >=
    // extent / 255), rounded outward: the looseness a 64-B eight-wide node costs
    Box frame;
    for (int k = 0; k < m; k++) frame.grow(nbox(cut[k]));
    double step[3];
    if (g_quant == 2)  // origin stored in fp16, rounded down (the 64-B eight-wide unit's header)
        for (int a = 0; a < 3; a++) {
            int e;
            std::frexp(frame.lo[a], &e);
            const double ulp = std::ldexp(1.0, std::max(e - 11, -24));
            frame.lo[a] = (float)(std::floor((double)frame.lo[a] / ulp) * ulp);
        }
    for (int a = 0; a < 3; a++) {
        const double ext = (double)frame.hi[a] - frame.lo[a];
        step[a] = ext > 0 ? std::ldexp(1.0, (int)std::ceil(std::log2(ext / 255.0))) : 1.0;
    }
    for (int k = 0; k < m; k++) {
        const uint32_t c = cut[k];
        Box b = nbox(c);
        if (g_quant)
            for (int a = 0; a < 3; a++) {
                if (!(b.lo[a] <= b.hi[a])) continue;  // an inverted (empty) box stays as is
                const double ql = std::floor(((double)b.lo[a] - frame.lo[a]) / step[a]);
                const double qh = std::ceil(((double)b.hi[a] - frame.lo[a]) / step[a]);
                b.lo[a] = std::nextafter((float)(frame.lo[a] + ql * step[a]), -INFINITY);
                b.hi[a] = std::nextafter((float)(frame.lo[a] + qh * step[a]), INFINITY);
            }
        int ref;
        if (g_nd[c].sphere >= 0)
            ref = ~g_leaf_of[c];
        else
            ref = build_a(t, c);
        t.nodes[me].box[k] = b;
        t.nodes[me].ref[k] = ref;
    }
    t.nodes[me].n = m;
    assign_positions(t.nodes[me]);
    return me;
}

// ---------------------------------------------------------------- tree B
const std::vector<Leaf>* g_leaves;
int g_bins = 16, g_leaf_max = 1;

struct BNode {  // binary build node
    Box box;
    int l = -1, r = -1;      // children (binary) or -1
    std::vector<int> prims;  // leaf: leaf indices
};

int sah_build(std::vector<BNode>& bn, std::vector<int>& idx, int lo, int hi)
{
    const std::vector<Leaf>& L = *g_leaves;
    BNode node;
    Box cb;  // centroid bounds
    for (int i = lo; i < hi; i++) {
        node.box.grow(L[idx[i]].box);
        Box c;
        for (int k = 0; k < 3; k++) c.lo[k] = c.hi[k] = 0.5f * (L[idx[i]].box.lo[k] + L[idx[i]].box.hi[k]);
        cb.grow(c);
    }
    const int me = (int)bn.size();
    bn.push_back(node);
    const int n = hi - lo;
    float best_cost = INFINITY;
    int best_axis = -1, best_split = -1;
    if (n > g_leaf_max) {
        for (int a = 0; a < 3; a++) {
            const float ext = cb.hi[a] - cb.lo[a];
            if (!(ext > 0)) continue;
            std::vector<Box> bb(g_bins);
            std::vector<int> bc(g_bins, 0);
            for (int i = lo; i < hi; i++) {
                const float c = 0.5f * (L[idx[i]].box.lo[a] + L[idx[i]].box.hi[a]);
                int b = (int)((c - cb.lo[a]) / ext * g_bins);
                b = std::min(std::max(b, 0), g_bins - 1);
                bb[b].grow(L[idx[i]].box);
                bc[b]++;
            }
            for (int s = 1; s < g_bins; s++) {
                Box lb, rb;
                int ln = 0, rn = 0;
                for (int b = 0; b < s; b++) {
                    if (bc[b]) lb.grow(bb[b]);
                    ln += bc[b];
                }
                for (int b = s; b < g_bins; b++) {
                    if (bc[b]) rb.grow(bb[b]);
                    rn += bc[b];
                }
                if (!ln || !rn) continue;
                const float cost = ln * lb.area() + rn * rb.area();
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = a;
                    best_split = s;
                }
            }
        }
    }
    if (best_axis < 0) {
        if (n > g_leaf_max) {  // no plane: median split by index
            const int mid = lo + n / 2;
            const int l = sah_build(bn, idx, lo, mid), r = sah_build(bn, idx, mid, hi);
            bn[me].l = l;
            bn[me].r = r;
            return me;
        }
        for (int i = lo; i < hi; i++) bn[me].prims.push_back(idx[i]);
        return me;
    }
    const float ext = cb.hi[best_axis] - cb.lo[best_axis];
    auto pred = [&](int p) {
        const float c = 0.5f * (L[p].box.lo[best_axis] + L[p].box.hi[best_axis]);
        int b = (int)((c - cb.lo[best_axis]) / ext * g_bins);
        b = std::min(std::max(b, 0), g_bins - 1);
        return b < best_split;
    };
    const int mid = (int)(std::partition(idx.begin() + lo, idx.begin() + hi, pred) - idx.begin());
    const int l = sah_build(bn, idx, lo, mid), r = sah_build(bn, idx, mid, hi);
    bn[me].l = l;
    bn[me].r = r;
    return me;
}

// a binary node's slot reference in the four-wide tree
int wide_from(Tree& t, const std::vector<BNode>& bn, int b);
int slot_ref(Tree& t, const std::vector<BNode>& bn, int b)
{
    if (bn[b].l < 0 && bn[b].prims.size() == 1) return ~bn[b].prims[0];
    return wide_from(t, bn, b);
}
int wide_from(Tree& t, const std::vector<BNode>& bn, int b)
{
    std::vector<int> cut;
    if (bn[b].l < 0) {  // multi-prim leaf: its prims as slots (leaf_max <= 4)
        const int me = (int)t.nodes.size();
        t.nodes.emplace_back();
        for (size_t k = 0; k < bn[b].prims.size(); k++) {
            t.nodes[me].box[k] = (*g_leaves)[bn[b].prims[k]].box;
            t.nodes[me].ref[k] = ~bn[b].prims[k];
        }
        t.nodes[me].n = (int)bn[b].prims.size();
        return me;
    }
    cut = {bn[b].l, bn[b].r};
    while (cut.size() < 4) {
        int best = -1;
        float ba = -1;
        for (size_t j = 0; j < cut.size(); j++) {
            if (bn[cut[j]].l < 0) continue;
            if (bn[cut[j]].box.area() > ba) {
                best = (int)j;
                ba = bn[cut[j]].box.area();
            }
        }
        if (best < 0) break;
        const int c = cut[best];
        cut.erase(cut.begin() + best);
        cut.push_back(bn[c].l);
        cut.push_back(bn[c].r);
    }
    const int me = (int)t.nodes.size();
    t.nodes.emplace_back();
    t.nodes[me].n = (int)cut.size();
    for (size_t k = 0; k < cut.size(); k++) {
        const int ref = slot_ref(t, bn, cut[k]);
        t.nodes[me].box[k] = bn[cut[k]].box;
        t.nodes[me].ref[k] = ref;
    }
    return me;
}

// ---------------------------------------------------------------- walk
struct Ray {
    float o[3], d[3], inv[3];
};
bool slab(const Ray& r, const Box& b, float& tmin)
{
    float t0 = -INFINITY, t1 = INFINITY;
    for (int k = 0; k < 3; k++) {
        float a = (b.lo[k] - r.o[k]) * r.inv[k], c = (b.hi[k] - r.o[k]) * r.inv[k];
        if (std::isnan(a) || std::isnan(c)) {
            a = -INFINITY;
            c = INFINITY;
        }
        t0 = std::max(t0, std::min(a, c));
        t1 = std::min(t1, std::max(a, c));
    }
    tmin = t0;
    return t1 >= t0 && t1 > 1e-6f;
}
float sphere_t(const Ray& r, const mirt_sphere& s)
{
    const float ox = r.o[0] - s.center.x, oy = r.o[1] - s.center.y, oz = r.o[2] - s.center.z;
    const float a = r.d[0] * r.d[0] + r.d[1] * r.d[1] + r.d[2] * r.d[2];
    const float b = 2.0f * (ox * r.d[0] + oy * r.d[1] + oz * r.d[2]);
    const float c = ox * ox + oy * oy + oz * oz - s.radius * s.radius;
    const float disc = b * b - 4 * a * c;
    if (!(disc > 0)) return -1;
    const float t = (float)((-(double)b - std::sqrt((double)disc)) / (2.0 * a));
    return t > 1e-6f ? t : -1;
}

struct Stats {
    double visits = 0, gates = 0, rays = 0, pushes = 0;
    double over = 0;  // steps whose pushes would overflow a 20-entry stack (the kernel's kWideStack)
    double slots = 0;  // live slots of the visited nodes (a visit that loads only those)
    int max_stack = 0;
};

int walk(const Tree& t, const std::vector<Leaf>& L, const mirt_sphere* sp, const Ray& r, float& best, Stats& st,
         std::vector<int>* trace = nullptr)
{
    best = INFINITY;
    int bs = -1;
    std::vector<int> stack;
    std::vector<float> sentry;
    float e;
    if (!slab(r, t.root_box, e)) return -1;
    stack.push_back(t.root_ref);
    sentry.push_back(e);
    st.rays++;
    while (!stack.empty()) {
        const int n = stack.back();
        const float en = sentry.back();
        stack.pop_back();
        sentry.pop_back();
        if (g_popcheck && en > best) continue;
        st.visits++;
        if (trace) trace->push_back(n);
        const W4& w = t.nodes[n];
        for (int k = 0; k < w.n; k++) st.slots += w.ref[k] != INT32_MIN;
        std::pair<float, int> in[kMaxWide];
        int m = 0;
        for (int k = 0; k < w.n; k++) {
            float ek;
            if (!slab(r, w.box[k], ek) || ek > best) continue;
            if (w.ref[k] < 0) {
                st.gates++;
                const int li = ~w.ref[k];
                const float tt = sphere_t(r, sp[L[li].sphere]);
                if (tt > 0 && (tt < best || (tt == best && L[li].sphere > bs))) {
                    best = tt;
                    bs = L[li].sphere;
                }
            } else {
                in[m++] = {g_order ? (float)(w.pos[k] ^ ((r.d[0] < 0) | (r.d[1] < 0) << 1 | (r.d[2] < 0) << 2))
                                   : ek,
                           w.ref[k]};
            }
        }
        std::sort(in, in + m, [](auto& a, auto& b) { return a.first > b.first; });  // far first: near on top
        if (m > 0 && (int)stack.size() + m - 1 > 20) st.over++;
        for (int k = 0; k < m; k++) {
            if (!g_order && in[k].first > best) continue;
            stack.push_back(in[k].second);
            sentry.push_back(g_order ? -INFINITY : in[k].first);
            st.pushes++;
        }
        st.max_stack = std::max(st.max_stack, (int)stack.size());
    }
    return bs;
}

Ray make_ray(float ox, float oy, float oz, float dx, float dy, float dz)
{
    Ray r{{ox, oy, oz}, {dx, dy, dz}, {}};
    for (int k = 0; k < 3; k++) r.inv[k] = 1.0f / r.d[k];
    return r;
}

}  // namespace

uint32_t spread3(uint32_t v)
{
    v &= 0x3ff;
    v = (v | (v << 16)) & 0x030000ff;
    v = (v | (v << 8)) & 0x0300f00f;
    v = (v | (v << 4)) & 0x030c30c3;
    v = (v | (v << 2)) & 0x09249249;
    return v;
}

// Lockstep model of a wave of 64 bounce walks: at step s every lane still
// walking reads its s-th node; the texture path's cost follows the DISTINCT
// nodes (64-B lines) a load instruction touches. Reports distinct nodes per
// lane-step for the first-bounce records taken 64 at a time in the queue's
// order (8x8 camera tiles) and after sorting them by other keys.
void coherence_study(const Tree& A, const std::vector<Leaf>& leaves, const mirt_sphere* sp, const mirt_camera& cam,
                     int crop)
{
    const int Wd = 1920, Hd = 1080;
    const float aspect = (float)Wd / Hd;
    const float fov = (float)((double)cam.fov * (M_PI / 180.0));
    const float hh = (float)std::tan((double)(fov / 2.0f)), hw = aspect * hh;
    std::mt19937 rng(9);
    std::uniform_real_distribution<float> U(-1, 1);
    struct Rec {
        Ray r;
        uint64_t tile, key_oct, key_morton, key_both;
    };
    std::vector<Rec> recs;
    Box sb;
    for (int i = 0; i < (int)leaves.size(); i++) sb.grow(leaves[i].box);
    const int x0 = Wd / 2 - crop / 2, y0 = Hd / 2 - crop / 2;
    Stats dummy;
    for (int ty = 0; ty < crop / 8; ty++)
        for (int tx = 0; tx < crop / 8; tx++)
            for (int ly = 0; ly < 8; ly++)
                for (int lx = 0; lx < 8; lx++) {
                    const int x = x0 + tx * 8 + lx, y = y0 + ty * 8 + ly;
                    const float u = ((float)x / Wd - 0.5f) * aspect, v = -((float)y / Hd - 0.5f);
                    float d[3];
                    for (int k = 0; k < 3; k++) {
                        const float f = (&cam.forward.x)[k], rr = (&cam.right.x)[k], up = (&cam.up.x)[k];
                        d[k] = f + rr * (2 * hw) * u + up * (2 * hh) * v;
                    }
                    const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                    Ray r = make_ray(cam.position.x, cam.position.y, cam.position.z, d[0] / l, d[1] / l, d[2] / l);
                    float t;
                    const int h = walk(A, leaves, sp, r, t, dummy);
                    if (h < 0) continue;
                    const mirt_sphere& s = sp[h];
                    float p[3] = {r.o[0] + r.d[0] * t, r.o[1] + r.d[1] * t, r.o[2] + r.d[2] * t};
                    float nrm[3] = {p[0] - s.center.x, p[1] - s.center.y, p[2] - s.center.z};
                    float q[3];
                    for (;;) {
                        q[0] = U(rng);
                        q[1] = U(rng);
                        q[2] = U(rng);
                        const float qq = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
                        if (qq > 0 && qq < 1) break;
                    }
                    const float ql = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
                    const float dd = q[0] * nrm[0] + q[1] * nrm[1] + q[2] * nrm[2];
                    for (int k = 0; k < 3; k++) q[k] = (dd > 0 ? 1 : -1) * q[k] / ql;
                    Rec rc;
                    rc.r = make_ray(p[0], p[1], p[2], q[0], q[1], q[2]);
                    rc.tile = recs.size();
                    const uint32_t oct = (q[0] < 0) | (q[1] < 0) << 1 | (q[2] < 0) << 2;
                    uint32_t m[3];
                    for (int k = 0; k < 3; k++)
                        m[k] = (uint32_t)std::min(1023.0f, std::max(0.0f, (p[k] - sb.lo[k]) / (sb.hi[k] - sb.lo[k]) * 1024));
                    const uint64_t mort = spread3(m[0]) | spread3(m[1]) << 1 | spread3(m[2]) << 2;
                    rc.key_oct = (uint64_t)oct << 40 | rc.tile;
                    rc.key_morton = mort;
                    rc.key_both = (uint64_t)oct << 32 | mort;
                    recs.push_back(rc);
                }
    std::vector<std::vector<int>> traces(recs.size());
    for (size_t i = 0; i < recs.size(); i++) {
        float t;
        walk(A, leaves, sp, recs[i].r, t, dummy, &traces[i]);
    }
    auto score = [&](const char* name, std::vector<size_t> order) {
        double distinct = 0, lanes = 0, steps = 0, gdistinct = 0, glanes = 0;
        for (size_t w = 0; w + 64 <= order.size(); w += 64) {
            size_t longest = 0;
            for (int l = 0; l < 64; l++) longest = std::max(longest, traces[order[w + l]].size());
            for (size_t st = 0; st < longest; st++) {
                std::vector<int> ids;
                for (int l = 0; l < 64; l++) {
                    const auto& tr = traces[order[w + l]];
                    if (st < tr.size()) ids.push_back(tr[st]);
                }
                std::sort(ids.begin(), ids.end());
                lanes += ids.size();
                for (int id : ids) glanes += id >= 16;  // the first 16 nodes sit in LDS (MIRT_HCACHE)
                ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
                distinct += ids.size();
                for (int id : ids) gdistinct += id >= 16;
                steps++;
            }
        }
        printf("  %-34s distinct nodes per lane-step %.3f (global loads only %.3f)  active lanes per step %.1f\n",
               name, distinct / lanes, gdistinct / glanes, lanes / steps);
    };
    std::vector<size_t> o(recs.size());
    for (size_t i = 0; i < o.size(); i++) o[i] = i;
    printf("coherence (lockstep model), %zu first-bounce records of a %dx%d centre crop\n", recs.size(), crop, crop);
    score("queue order (8x8 camera tiles)", o);
    auto by = [&](uint64_t Rec::*k) {
        std::vector<size_t> v = o;
        std::stable_sort(v.begin(), v.end(), [&](size_t a, size_t b) { return recs[a].*k < recs[b].*k; });
        return v;
    };
    score("octant, then queue order", by(&Rec::key_oct));
    score("Morton(hit point)", by(&Rec::key_morton));
    score("octant, then Morton(hit point)", by(&Rec::key_both));
    for (int g : {64, 128, 256, 1024}) {
        std::vector<size_t> v = o;
        auto oct = [&](size_t i) { return recs[i].key_oct >> 40; };
        std::stable_sort(v.begin(), v.end(), [&](size_t a, size_t b) {
            return a / g != b / g ? a / g < b / g : oct(a) < oct(b);
        });
        char name[64];
        snprintf(name, sizeof name, "octant within %d-record groups", g);
        score(name, v);
        v = o;
        std::stable_sort(v.begin(), v.end(), [&](size_t a, size_t b) {
            return a / g != b / g ? a / g < b / g : recs[a].key_both < recs[b].key_both;
        });
        snprintf(name, sizeof name, "oct+Morton within %d-record groups", g);
        score(name, v);
    }
    std::vector<size_t> sh = o;
    std::shuffle(sh.begin(), sh.end(), rng);
    score("random order", sh);
}

// Screen-space binning of the camera rays (all share the camera origin):
// per 8x8 tile, the live leaves whose sphere's projected disc (conservative
// bounding square, +2 px) overlaps the tile, sorted by the sphere's nearest
// distance; walk them front to back until every lane's best hit is nearer
// than the next candidate. Reports candidates walked per tile (each a
// wave-uniform step: one sphere test per lane) and pairs binned.
void binning_study(const std::vector<Leaf>& leaves, const mirt_sphere* sp, const mirt_camera& cam, int Wd, int Hd)
{
    const float aspect = (float)Wd / Hd;
    const float fov = (float)((double)cam.fov * (M_PI / 180.0));
    const float hh = (float)std::tan((double)(fov / 2.0f)), hw = aspect * hh;
    const int tx = (Wd + 7) / 8, ty = (Hd + 7) / 8;
    std::vector<std::vector<std::pair<float, int>>> bins((size_t)tx * ty);
    const float* o = &cam.position.x;
    const float* F = &cam.forward.x;
    const float* R = &cam.right.x;
    const float* U = &cam.up.x;
    long pairs = 0, full = 0;
    for (int li = 0; li < (int)leaves.size(); li++) {
        const mirt_sphere& s = sp[leaves[li].sphere];
        const float c[3] = {s.center.x - o[0], s.center.y - o[1], s.center.z - o[2]};
        const float r = std::fabs(s.radius);
        const float z = c[0] * F[0] + c[1] * F[1] + c[2] * F[2];
        const float x = c[0] * R[0] + c[1] * R[1] + c[2] * R[2];
        const float y = c[0] * U[0] + c[1] * U[1] + c[2] * U[2];
        const float dist = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]);
        int x0 = 0, x1 = tx - 1, y0 = 0, y1 = ty - 1;
        if (z - r > 1e-3f) {  // wholly in front: bound the disc by its tangent cone
            const float sa = r / std::sqrt(std::max(z * z - r * r, 1e-12f));  // tan of the half-angle, ~
            // screen coords: u = x / (z * 2hw) + 0.5 (in W units), v = -y / (z * 2hh) + 0.5
            const float ux = x / z, uy = y / z;
            const float ext = sa * (1.0f + std::fabs(ux) + std::fabs(uy)) * 1.5f;  // generous
            const float px0 = ((ux - ext) / (2 * hw) + 0.5f) * Wd - 2, px1 = ((ux + ext) / (2 * hw) + 0.5f) * Wd + 2;
            const float py0 = (-(uy + ext) / (2 * hh) + 0.5f) * Hd - 2, py1 = (-(uy - ext) / (2 * hh) + 0.5f) * Hd + 2;
            x0 = std::max(0, (int)std::floor(px0) / 8);
            x1 = std::min(tx - 1, (int)std::floor(px1) / 8);
            y0 = std::max(0, (int)std::floor(py0) / 8);
            y1 = std::min(ty - 1, (int)std::floor(py1) / 8);
            if (px1 < 0 || py1 < 0 || px0 >= Wd || py0 >= Hd) continue;
        } else if (z + r < 0) {
            continue;  // wholly behind
        } else {
            full++;
        }
        for (int b = y0; b <= y1; b++)
            for (int a = x0; a <= x1; a++) {
                bins[(size_t)b * tx + a].push_back({dist - r, li});
                pairs++;
            }
    }
    double walked = 0, tiles = 0, listed = 0;
    Stats dummy;
    for (int b = 0; b < ty; b++)
        for (int a = 0; a < tx; a++) {
            auto& L = bins[(size_t)b * tx + a];
            std::sort(L.begin(), L.end());
            listed += L.size();
            float best[64];
            bool any = false;
            for (int l = 0; l < 64; l++) best[l] = INFINITY;
            size_t k = 0;
            for (; k < L.size(); k++) {
                bool need = false;
                for (int l = 0; l < 64; l++)
                    if (best[l] >= L[k].first) need = true;
                if (!need) break;
                for (int l = 0; l < 64; l++) {
                    const int x = a * 8 + (l & 7), y = b * 8 + (l >> 3);
                    if (x >= Wd || y >= Hd) continue;
                    const float u = ((float)x / Wd - 0.5f) * aspect, v = -((float)y / Hd - 0.5f);
                    float d[3];
                    for (int q = 0; q < 3; q++) d[q] = F[q] + R[q] * (2 * hw) * u + U[q] * (2 * hh) * v;
                    const float len = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
                    Ray ray = make_ray(o[0], o[1], o[2], d[0] / len, d[1] / len, d[2] / len);
                    const float t = sphere_t(ray, sp[leaves[L[k].second].sphere]);
                    if (t > 0 && t < best[l]) best[l] = t;
                    any = true;
                }
            }
            (void)any;
            walked += k;
            tiles++;
        }
    printf("binning %dx%d: %ld tile-leaf pairs (%.1f per tile, %ld leaves cover the screen), candidates walked per "
           "tile %.2f\n", Wd, Hd, pairs, listed / tiles, full, walked / tiles);
}

int main(int argc, char** argv)
{
    const int n = argc > 1 ? atoi(argv[1]) : 10000;
    const std::string scene = argc > 2 ? argv[2] : "render";
    const int stride = argc > 3 ? atoi(argv[3]) : 4;
    g_bins = argc > 4 ? atoi(argv[4]) : 16;
    g_leaf_max = argc > 5 ? atoi(argv[5]) : 1;
    g_wide = argc > 9 ? atoi(argv[9]) : 4;
    g_quant = argc > 10 ? atoi(argv[10]) : 0;
    g_order = argc > 11 ? atoi(argv[11]) : 0;
    g_popcheck = argc > 12 ? atoi(argv[12]) : 1;
    mirt_rand_state st;
    mirt_srand(&st, 1);
    std::vector<mirt_sphere> sp(n);
    if (scene == "render")
        mirt_scene_random(&st, sp.data(), n);
    else
        mirt_scene_benchmark(&st, sp.data(), n, 1000.0f);
    mirt_node* nd = nullptr;
    int nn = 0;
    mirt_bvh_build_flat(sp.data(), 0, n, 0, &nd, &nn);
    g_nd = nd;
    g_ns = n;
    std::vector<Leaf> leaves;
    g_leaf_of.assign(nn, -1);
    for (int i = 0; i < nn; i++)
        if (nd[i].sphere >= 0 && !dead(i)) {
            g_leaf_of[i] = (int)leaves.size();
            leaves.push_back(Leaf{nbox(i), nd[i].sphere});
        }
    g_leaves = &leaves;
    Tree A;  // the root's HNode is the four-slot cut of flat node 0
    A.root_box = nbox(0);
    A.root_ref = build_a(A, 0);
    if (argc > 6 && std::string(argv[6]) == "binning") {
        mirt_camera cam;
        mirt_camera_default(&cam);
        binning_study(leaves, sp.data(), cam, argc > 7 ? atoi(argv[7]) : 1920, argc > 8 ? atoi(argv[8]) : 1080);
        return 0;
    }
    if (argc > 6 && std::string(argv[6]) == "coherence") {
        mirt_camera cam;
        mirt_camera_default(&cam);
        coherence_study(A, leaves, sp.data(), cam, argc > 7 ? atoi(argv[7]) : 512);
        return 0;
    }
    Tree B;
    std::vector<BNode> bn;
    std::vector<int> idx(leaves.size());
    for (size_t i = 0; i < idx.size(); i++) idx[i] = (int)i;
    const int broot = sah_build(bn, idx, 0, (int)idx.size());
    B.root_box = bn[broot].box;
    B.root_ref = wide_from(B, bn, broot);
    // rays: camera rays of the default camera at 1920x1080 (every stride-th
    // pixel each way), then up to 4 diffuse bounces each (uniform hemisphere)
    mirt_camera cam;
    mirt_camera_default(&cam);
    const int Wd = 1920, Hd = 1080;
    const float aspect = (float)Wd / Hd;
    const float fov = (float)((double)cam.fov * (M_PI / 180.0));
    const float hh = (float)std::tan((double)(fov / 2.0f)), hw = aspect * hh;
    std::mt19937 rng(5);
    std::uniform_real_distribution<float> U(-1, 1);
    Stats sa[2], sb[2];  // [0] camera rays, [1] bounces
    long mism = 0;
    for (int y = 0; y < Hd; y += stride)
        for (int x = 0; x < Wd; x += stride) {
            const float u = ((float)x / Wd - 0.5f) * aspect, v = -((float)y / Hd - 0.5f);
            float d[3];
            for (int k = 0; k < 3; k++) {
                const float f = (&cam.forward.x)[k], rr = (&cam.right.x)[k], up = (&cam.up.x)[k];
                d[k] = f + rr * (2 * hw) * u + up * (2 * hh) * v;
            }
            const float l = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            Ray r = make_ray(cam.position.x, cam.position.y, cam.position.z, d[0] / l, d[1] / l, d[2] / l);
            for (int level = 0; level < 5; level++) {
                float ta, tb;
                const int ha = walk(A, leaves, sp.data(), r, ta, sa[level > 0]);
                const int hb = walk(B, leaves, sp.data(), r, tb, sb[level > 0]);
                if (ha != hb) mism++;
                if (ha < 0) break;
                const mirt_sphere& s = sp[ha];
                float p[3] = {r.o[0] + r.d[0] * ta, r.o[1] + r.d[1] * ta, r.o[2] + r.d[2] * ta};
                float nrm[3] = {p[0] - s.center.x, p[1] - s.center.y, p[2] - s.center.z};
                float q[3];
                for (;;) {
                    q[0] = U(rng);
                    q[1] = U(rng);
                    q[2] = U(rng);
                    const float qq = q[0] * q[0] + q[1] * q[1] + q[2] * q[2];
                    if (qq > 0 && qq < 1) break;
                }
                const float ql = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
                float dd = q[0] * nrm[0] + q[1] * nrm[1] + q[2] * nrm[2];
                for (int k = 0; k < 3; k++) q[k] = (dd > 0 ? 1 : -1) * q[k] / ql;
                r = make_ray(p[0], p[1], p[2], q[0], q[1], q[2]);
            }
        }
    auto pr = [](const char* name, const Stats& s, size_t nodes) {
        printf("  %-28s nodes %7zu  rays %8.0f  visits/ray %7.2f  gates/ray %6.2f  pushes/ray %6.2f  max stack %d  overflow/ray %.4f  live slots/visit %.2f\n",
               name, nodes, s.rays, s.visits / s.rays, s.gates / s.rays, s.pushes / s.rays, s.max_stack, s.over / s.rays,
               s.slots / s.visits);
    };
    printf("%s %d spheres, %zu live leaves, %d flat nodes, pixel stride %d, SAH bins %d, leaf max %d\n",
           scene.c_str(), n, leaves.size(), nn, stride, g_bins, g_leaf_max);
    pr("A camera (reference-derived)", sa[0], A.nodes.size());
    pr("B camera (SAH over leaves)", sb[0], B.nodes.size());
    pr("A bounces", sa[1], A.nodes.size());
    pr("B bounces", sb[1], B.nodes.size());
    printf("  closest-hit mismatches A vs B: %ld\n", mism);
    mirt_bvh_free_flat(nd);
    return 0;
}
