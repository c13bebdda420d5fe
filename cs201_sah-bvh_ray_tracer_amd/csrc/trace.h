// Device side of the render path: exact-semantics restatements of the
// reference's per-ray functions, written for wave64 / gfx950.
//
// Floating point follows the reference operation by operation (the .hip is
// compiled with -ffp-contract=off; divisions and square roots are the IEEE
// correctly rounded HIP defaults; the double-precision segments of
// hit.c:28 and vec3.c:22 are computed in double). Where a cheaper estimate
// is used (slab_fast, sphere_t), it only ever DECIDES an outcome when a
// proven error bound shows the reference computation would decide the same
// way, and falls back to the reference arithmetic otherwise.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mirt.h"
#include "rng.h"

namespace mirt {

constexpr float kEps = 0.000001f;  // constants.h:6
constexpr int kMaxDepth = 8;       // bounce levels kept in registers

// Device copy of a flattened node (mirt_node, include/mirt.h) padded to 64 B,
// with the leaf's sphere (centre, radius) inline so a leaf step needs no
// second, dependent load. Inner nodes and the &spheres[N] sentinel carry NaN
// geometry (never hits).
struct __attribute__((aligned(64))) DNode {
    float bmin[3];
    float bmax[3];
    int32_t sphere;   // leaf: sphere index; inner: -1
    uint32_t skip;    // next node after this subtree | MIRT_NODE_EMPTY
    float4 geo;       // leaf sphere centre.xyz, radius
    uint32_t pad[4];
};
static_assert(sizeof(DNode) == 64, "device node is 64 B");

// The same tree re-laid for ordered walks: one node per inner node of the
// reference tree holding BOTH children, so one load tests both and the walk
// can enter the nearer child first. PNode 0 is a virtual parent whose only
// child is the root. A child reference is an inner PNode index, kPLeaf |
// sphere index (a leaf that can hit), or kPNone (no child that can ever hit:
// a 0-sphere leaf or the &spheres[N] sentinel of hit.c). A child slot holds
// the child's box (lo.xyz, hi.xyz) -- for a leaf that is the box of the
// node's whole sphere range, not of its one sphere (a depth-40 leaf keeps
// the range's bounds but tests only node->sphere, bvh.c:122-136), so the
// sphere itself is fetched when the box passes.
// `flat` and `end` locate the node in the flat pre-order tree, [flat + 1,
// end) being its children's subtrees, which a walk can take in DFS order
// without a stack.
constexpr uint32_t kPLeaf = 0x80000000u;
constexpr uint32_t kPNone = 0xffffffffu;
constexpr uint32_t kPIndex = 0x7fffffffu;
struct __attribute__((aligned(64))) PNode {
    float c0[6];
    float c1[6];
    uint32_t ref0, ref1;
    uint32_t flat, end;
};
static_assert(sizeof(PNode) == 64, "ordered node is 64 B");

// Four-wide layout for per-lane walks: HNode(Y), for an inner node Y of the
// reference tree, holds Y's grandchildren (a child that is a leaf stands in
// for its own slot), so a walk takes half the dependent steps. The skipped
// children's boxes need no test: the tree's boxes nest (checked at upload)
// and hit.c's slab test is monotone under containment (correctly rounded
// subtraction and division are monotone, so a box inside another gets a
// later entry and an earlier exit), so a ray that passes a box passes every
// enclosing one -- the leaves reached are exactly those hit.c:91-109
// reaches. The same argument lets slot boxes be CONSERVATIVE: each is
// stored in fp16 rounded outward (a superset) and tested with a fast test
// that passes when undecided -- entering an inner node too eagerly costs
// work, never a result, because every leaf is still gated by its exact box.
// A leaf slot's sphere and its exact box live in two arrays (structure of
// arrays, round 6): the gate reads the 16-B sphere first and the 32-B box only
// for a hit that could win, so the spheres the walks read are packed eight to
// a 128-B line (a 48-B record per leaf held 2.7) and the hot part of a large
// tree -- HNodes + spheres -- is two thirds of the bytes it was. 64 B per node = the bytes of two fp32 boxes: divergent
// per-lane loads are bound by the bytes the texture path returns.
// HNode 0 is a virtual node whose only slot is the root; slot references: an
// inner HNode index, kPLeaf | leaf index, or kPNone. HAux holds the
// node's flat DFS segment [flat + 1, end), read only when the stack is full.
struct __attribute__((aligned(64))) HNode {
    struct Slot {
        uint32_t box[3];  // per axis: fp16 lo (bits 0-15) | fp16 hi (bits 16-31)
        uint32_t ref;
    } slot[4];            // 16 B per slot: one dwordx4 each
};
static_assert(sizeof(HNode) == 64, "wide node is 64 B");
struct HAux {
    uint32_t flat, end;
};
struct __attribute__((aligned(32))) LeafBox {
    float lo[3], hi[3];  // the leaf's exact box (bvh.c bounds)
    int32_t sphere;
    uint32_t pad;
};
static_assert(sizeof(LeafBox) == 32, "leaf box is 32 B");

// Read-only scene in HBM (L2 / Infinity-Cache resident at the BASELINE sizes).
struct DevScene {
    const DNode* nodes;     // 64 B, leaf sphere inline: scalar (wave-uniform) walks
    const mirt_node* nodes32;  // the same tree in 32 B (mirt_node): per-lane walks (twice the nodes per L1 line)
    const float4* geo;      // centre.xyz, radius per sphere; [num_spheres] = NaN sentinel
    const uint32_t* color;  // packed RGBA8
    uint32_t num_nodes;
    int num_spheres;
    // closest-hit pruning (Prune below): enabled only for a tree whose boxes
    // enclose their subtrees (checked at upload)
    int prune;
    float r_max;   // largest sphere radius
    float c_max;   // largest |centre|_inf + radius
    // ordered walks (PNode): set when leaves hold increasing sphere indices
    // in DFS order (so the index is the DFS tie key) and the tree is shallow
    // enough for the 64-entry walk stack
    const PNode* pnodes;
    int ordered;
    // four-wide per-lane walks (HNode): ordered trees whose boxes nest
    const HNode* hnodes;
    const HAux* haux;
    const float4* leaf_geo;   // per leaf: its sphere (centre, radius)
    const LeafBox* leaf_box;  // per leaf: its exact box and sphere index
    int wide;
    uint32_t num_hnodes;  // HNodes, numbered breadth-first: the first ones are the top levels
    // where a four-wide walk starts: the root's own HNode (1) -- HNode 0's
    // single slot is the root box, which every ray that can hit a leaf passes
    // (boxes nest), so its step is skipped -- or 0 when the root is a leaf
    uint32_t wide_root;
    // |coordinate| bound C of every box and of the bounce
    // rays' origins the HNode slot boxes were grown for (2^-19 C)
    float o_bound;
};

// LDS-resident node data (address space 3: ds_read, never a flat load)
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const u32x4 lds_uint4;
__device__ __forceinline__ uint4 lds_load(lds_uint4* p)
{
    const u32x4 v = *p;
    return make_uint4(v.x, v.y, v.z, v.w);
}

struct Ray {
    float ox, oy, oz, dx, dy, dz;
};

struct Counters {
    uint32_t rays, nodes, spheres, hits;
    uint32_t steps;  // traversal loop iterations executed (every lane counts; /64 = wave steps)
    // the camera-ray level alone (the wavefront schedule's primary pass);
    // the rest of nodes/spheres/hits is the bounce pass
    uint32_t nodes0, spheres0, hits0;
};

// A node in registers (12 dwords).
struct NodeV {
    float b0, b1, b2, b3, b4, b5;
    int32_t sphere;
    uint32_t skip;
    float4 g;
};

typedef const __attribute__((address_space(4))) uint32_t cu32_t;
typedef const __attribute__((address_space(4))) float cf32_t;

// Wave-uniform index -> read through the constant address space, which the
// backend lowers to scalar loads (s_load_dwordx8 + x4 for a node).
__device__ __forceinline__ NodeV load_node_uniform(const DNode* base, uint32_t i)
{
    const cu32_t* p = (const cu32_t*)base + 16u * i;
    NodeV n;
    n.b0 = __uint_as_float(p[0]);
    n.b1 = __uint_as_float(p[1]);
    n.b2 = __uint_as_float(p[2]);
    n.b3 = __uint_as_float(p[3]);
    n.b4 = __uint_as_float(p[4]);
    n.b5 = __uint_as_float(p[5]);
    n.sphere = (int32_t)p[6];
    n.skip = p[7];
    n.g = make_float4(__uint_as_float(p[8]), __uint_as_float(p[9]), __uint_as_float(p[10]), __uint_as_float(p[11]));
    return n;
}

__device__ __forceinline__ float4 load_geo_uniform(const float4* base, int i)
{
    const cf32_t* p = (const cf32_t*)base + 4 * i;
    return make_float4(p[0], p[1], p[2], p[3]);
}

// Divergent index -> three 16-B vector loads per node.
__device__ __forceinline__ NodeV load_node_lane(const DNode* base, uint32_t i)
{
    const float4* p = (const float4*)(base + i);
    const float4 a = p[0], b = p[1], g = p[2];
    NodeV n;
    n.b0 = a.x;
    n.b1 = a.y;
    n.b2 = a.z;
    n.b3 = a.w;
    n.b4 = b.x;
    n.b5 = b.y;
    n.sphere = __float_as_int(b.z);
    n.skip = __float_as_uint(b.w);
    n.g = g;
    return n;
}

// vec3.c:21-24: len = (float)sqrt((double)(x*x + y*y + z*z)); divide by len.
__device__ __forceinline__ void normalize3(float& x, float& y, float& z)
{
    float sq = x * x;
    sq = sq + y * y;
    sq = sq + z * z;
    const float len = (float)__dsqrt_rn((double)sq);
    if (len != 0.0f) {
        x = x / len;
        y = y / len;
        z = z / len;
    } else {
        x = y = z = 0.0f;
    }
}

__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz)
{
    float s = ax * bx;  // vec3.c:26, left to right
    s = s + ay * by;
    return s + az * bz;
}

// Per-ray constants of the slab test (hit.c:54-76): the per-axis d == 0
// branch does not depend on the box, nor do the reciprocals of slab_fast.
struct SlabRay {
    float ox, oy, oz, dx, dy, dz;
    float ix, iy, iz;  // correctly rounded 1/d
    bool zx, zy, zz;
    bool generic;      // a zero or tiny (< 2^-40) direction component: exact test only
};

__device__ __forceinline__ SlabRay slab_ray(const Ray& r)
{
    SlabRay s;
    s.ox = r.ox;
    s.oy = r.oy;
    s.oz = r.oz;
    s.dx = r.dx;
    s.dy = r.dy;
    s.dz = r.dz;
    s.zx = r.dx == 0.0f;
    s.zy = r.dy == 0.0f;
    s.zz = r.dz == 0.0f;
    const float tiny = 0x1p-40f;
    s.generic = !(fabsf(r.dx) >= tiny && fabsf(r.dy) >= tiny && fabsf(r.dz) >= tiny);
    s.ix = 1.0f / r.dx;
    s.iy = 1.0f / r.dy;
    s.iz = 1.0f / r.dz;
    return s;
}

// hit.c:49-82: true IEEE division per axis (no reciprocal: SURVEY §8.H3),
// d == 0 -> (-inf, +inf), min/max exact, accept tmax >= tmin && tmax > EPS.
__device__ __forceinline__ bool slab_test(const SlabRay& r, float x0, float y0, float z0, float x1, float y1,
                                          float z1)
{
    float tx1 = -INFINITY, tx2 = INFINITY, ty1 = -INFINITY, ty2 = INFINITY, tz1 = -INFINITY, tz2 = INFINITY;
    if (!r.zx) {
        tx1 = (x0 - r.ox) / r.dx;
        tx2 = (x1 - r.ox) / r.dx;
    }
    if (!r.zy) {
        ty1 = (y0 - r.oy) / r.dy;
        ty2 = (y1 - r.oy) / r.dy;
    }
    if (!r.zz) {
        tz1 = (z0 - r.oz) / r.dz;
        tz2 = (z1 - r.oz) / r.dz;
    }
    const float tmin = fmaxf(fminf(tx1, tx2), fmaxf(fminf(ty1, ty2), fminf(tz1, tz2)));
    const float tmax = fminf(fmaxf(tx1, tx2), fminf(fmaxf(ty1, ty2), fmaxf(tz1, tz2)));
    return tmax >= tmin && tmax > kEps;
}

// Closest-hit pruning: a walk may skip a subtree whose box the ray can only
// enter beyond the best hit so far, because no sphere inside can then record
// t <= best (the reference's DFS, hit.c:91-109, tests everything; the result
// is the same closest hit with the same later-leaf-wins tie rule, since the
// walk still visits leaves in DFS order and only drops losers).
//
// Bound: let sphere S (centre c, radius r) lie in box B and let its
// hit.c:19-39 arithmetic return t' with t' <= best. The point p = o + t' d
// (exact) then lies within D of S's surface: with the computed quadratic,
// |p - c|^2 - r^2 equals the rounding error of the discriminant over 4a plus
// the a/b roundings times t'^2 / t', all below 35 u M^2 (u = 2^-24,
// M = max(|o - c|, r)), so D <= sqrt(35 u) M < 2^-9.3 M; and M <= t'|d| + r + D
// <= best |d| + r_max + D. The reference's leaf boxes fl(c -+ r) and the
// computed fl(o - c) move S by below 2^-22 (|o|_inf + c_max). Hence p lies in
// B grown by m = 2^-8 (best |d| + r_max) + 2^-20 (|o|_inf + c_max) (>2x over
// both terms; a float32 sweep of grazing rays peaks at 2^-10.5 M), so t' is at
// least the entry t of the grown box, max_k (near_k - m |1/d_k|). slab_fast's
// near_k is within 2^-21 of the exact (b_k - o_k) / d_k (its 2^-22 plus the
// rounding of b_k - o_k), so
// fma(near_k, 1 - 2^-20, -m |1/d_k|), when positive, is at most (1 + u) times
// the exact grown near plane whatever the cancellation; the box is pruned only
// when that computed entry exceeds lim = best (1 + 2^-18).
struct Prune {
    float m;    // growth of the box (world units)
    float lim;  // prune when the grown box's entry t exceeds this; +inf = off
};

__device__ __forceinline__ Prune prune_off() { return {INFINITY, INFINITY}; }

// Without any hit, M <= |o - c| + r <= sqrt(3) (|o|_inf + c_max) bounds every
// sphere, so m0 = (2^-7 + 2^-20)(|o|_inf + c_max) is a valid growth from the
// start (used by the zero-component test of pruned_any; the entry test also
// needs a best).
__device__ __forceinline__ float prune_m0(const DevScene& sc, float ox, float oy, float oz)
{
    const float oi = fmaxf(fabsf(ox), fmaxf(fabsf(oy), fabsf(oz)));
    return (oi + sc.c_max) * (0x1p-7f + 0x1p-20f);
}

__device__ __forceinline__ Prune prune_start(const DevScene& sc, float ox, float oy, float oz)
{
    return sc.prune ? Prune{prune_m0(sc, ox, oy, oz), INFINITY} : prune_off();
}

// After a hit at t = best (finite). a4 = 4 d.d (SphRay). Both growths bound
// the same error, so the smaller one is used.
__device__ __forceinline__ void prune_update(Prune& p, const DevScene& sc, float ox, float oy, float oz, float a4,
                                             float best)
{
    const float dl = __builtin_amdgcn_sqrtf(a4) * (0.5f + 0x1p-20f);  // >= |d|
    const float oi = fmaxf(fabsf(ox), fmaxf(fabsf(oy), fabsf(oz)));
    p.m = fminf((best * dl + sc.r_max) * 0x1p-8f + (oi + sc.c_max) * 0x1p-20f, prune_m0(sc, ox, oy, oz));
    p.lim = best + best * 0x1p-18f;
}

// The same predicate, decided from reciprocal-multiply estimates whenever
// that is provably safe, else by slab_test (same result, bit for bit).
//
// For a = RN(b - o) (computed identically in both), Q = RN(a / d) is the
// reference's slab value and q = RN(a * RN(1/d)) ours: |q - Q| <= 3u|a/d|,
// u = 2^-24 (one rounding in 1/d, one in the product, Q's own half ulp), so
// every t value moves by < 2^-22 |t|; max/min select from values that moved
// that little, so |tmin' - tmin| and |tmax' - tmax| stay < 2^-22 of their
// magnitudes, and the two subtractions below add < 2^-24 (|tmin|+|tmax|).
// m = 2^-20 (|tmin'| + |tmax'|) therefore bounds every perturbation with a
// 2x margin: when a comparison clears m it has the reference's outcome;
// otherwise (near-tangent boxes) the exact division path decides.
// Requires finite, normal-range reciprocals: rays with a zero or tiny
// component take slab_test (`generic`), whose +-inf handling is exact.
// A box beyond the pruning limit (Prune) fails before any of this.
__device__ __forceinline__ bool slab_fast(const SlabRay& r, const Prune& p, float x0, float y0, float z0, float x1,
                                          float y1, float z1, float& near)
{
    // one fma per plane, as slab_cons_fast (its error bound below): the
    // margins cover it, so a decided comparison is still the reference's
    const float oix = r.ox * r.ix, oiy = r.oy * r.iy, oiz = r.oz * r.iz;
    const float mo = fmaxf(fabsf(oix), fmaxf(fabsf(oiy), fabsf(oiz))) * 0x1p-22f;
    const float tx1 = fmaf(x0, r.ix, -oix), tx2 = fmaf(x1, r.ix, -oix);
    const float ty1 = fmaf(y0, r.iy, -oiy), ty2 = fmaf(y1, r.iy, -oiy);
    const float tz1 = fmaf(z0, r.iz, -oiz), tz2 = fmaf(z1, r.iz, -oiz);
    const float nx = fminf(tx1, tx2), ny = fminf(ty1, ty2), nz = fminf(tz1, tz2);
    constexpr float c = 1.0f - 0x1p-20f;
    const float entry = fmaxf(fmaf(nx, c, -fmaf(p.m, fabsf(r.ix), mo)),
                              fmaxf(fmaf(ny, c, -fmaf(p.m, fabsf(r.iy), mo)), fmaf(nz, c, -fmaf(p.m, fabsf(r.iz), mo))));
    if (entry > p.lim) return false;
    const float tmin = fmaxf(nx, fmaxf(ny, nz));
    near = tmin;
    const float tmax = fminf(fmaxf(tx1, tx2), fminf(fmaxf(ty1, ty2), fmaxf(tz1, tz2)));
    const float m = fmaf(fabsf(tmin) + fabsf(tmax), 0x1p-20f, 2.0f * mo);
    const float gap = tmax - tmin, above = tmax - kEps;
    if (gap > m && above > m) return true;
    if (gap < -m || above < -m) return false;
    return slab_test(r, x0, y0, z0, x1, y1, z1);
}

// The Prune test for any ray, including those slab_fast leaves to slab_test:
// an axis whose direction component is zero or tiny (|d| < 2^-40) is left
// out of the max, which only lowers the entry bound; the other axes use the
// same normal-range reciprocals and margins as slab_fast. An axis with d == 0
// exactly prunes on its own when o lies outside the grown slab: every point
// o + t d has that coordinate, and a recordable hit lies within the grown box
// (Prune), although hit.c:54-57 passes such boxes by ignoring the slab.
// (lo - m, hi + m are rounded, but m carries a 2x margin far above 2^-24
// (c_max + m).)
__device__ __forceinline__ bool pruned_any(const SlabRay& r, const Prune& p, float x0, float y0, float z0, float x1,
                                           float y1, float z1)
{
    if (r.zx && (r.ox < x0 - p.m || r.ox > x1 + p.m)) return true;
    if (r.zy && (r.oy < y0 - p.m || r.oy > y1 + p.m)) return true;
    if (r.zz && (r.oz < z0 - p.m || r.oz > z1 + p.m)) return true;
    constexpr float c = 1.0f - 0x1p-20f;
    const float tiny = 0x1p-40f;
    float e = -INFINITY;
    if (fabsf(r.dx) >= tiny) e = fmaxf(e, fmaf(fminf((x0 - r.ox) * r.ix, (x1 - r.ox) * r.ix), c, -(p.m * fabsf(r.ix))));
    if (fabsf(r.dy) >= tiny) e = fmaxf(e, fmaf(fminf((y0 - r.oy) * r.iy, (y1 - r.oy) * r.iy), c, -(p.m * fabsf(r.iy))));
    if (fabsf(r.dz) >= tiny) e = fmaxf(e, fmaf(fminf((z0 - r.oz) * r.iz, (z1 - r.oz) * r.iz), c, -(p.m * fabsf(r.iz))));
    return e > p.lim;
}
__device__ __forceinline__ bool pruned_any(const SlabRay& r, const Prune& p, const NodeV& n)
{
    return pruned_any(r, p, n.b0, n.b1, n.b2, n.b3, n.b4, n.b5);
}

template <bool FAST>
__device__ __forceinline__ bool slab(const SlabRay& r, const Prune& p, const NodeV& n)
{
    float near;
    if (FAST && !r.generic) return slab_fast(r, p, n.b0, n.b1, n.b2, n.b3, n.b4, n.b5, near);
    return slab_test(r, n.b0, n.b1, n.b2, n.b3, n.b4, n.b5);
}

// The slab predicate of one box plus an entry estimate for ordering the
// walk (any value is correct there; only the visiting order changes).
template <bool FAST>
__device__ __forceinline__ bool slab_box(const SlabRay& r, const Prune& p, float x0, float y0, float z0, float x1,
                                         float y1, float z1, float& near)
{
    if (FAST && !r.generic) return slab_fast(r, p, x0, y0, z0, x1, y1, z1, near);
    near = 0.0f;
    if (FAST && pruned_any(r, p, x0, y0, z0, x1, y1, z1)) return false;
    return slab_test(r, x0, y0, z0, x1, y1, z1);
}

// Conservative box test: passes whenever hit.c's slab test on this box
// would (slab_fast's margins, with "undecided" counted as a pass), and also
// applies the pruning bound, which holds for any box containing the subtree.
// Branch-free, valid for rays without a zero/tiny direction component
// (slab_cons handles those with the exact division test).
//
// A plane's t is one fma, t = fl(b ix - fl(o ix)) (ix = fl(1/d)): against
// the exact T = (b - o) / d it is off by at most 2.01 u |T| (ix and the
// fma's rounding) plus 1.01 u |o ix| (the rounding of o ix), and hit.c's
// Q = fl(fl(b - o) / d) is within 2.01 u |T| of T. The relative part is
// covered by slab_fast's margin 2^-20 (|tmin| + |tmax|) (16 u against the
// 4.1 u needed), the absolute part by mo = 2^-22 max_k |o_k ix_k| (4 u, twice
// the 2.02 u of two values), added to the margin and to the pruning growth.
//
// BND (the bounce kernel's walks over HNodes): no margin.
// Every HNode slot box is stored grown by delta = 2^-19 C (DevScene::o_bound
// = C bounds every box coordinate and every bounce-ray origin; a ray whose
// origin lies outside takes the exact test, `generic`). In world units along
// axis k, a plane's computed t misses the exact (b - o)/d by at most
// (2.01 u |b - o| + 1.01 u |o|) / |d_k| <= 5.03 u C / |d_k| and hit.c's Q by
// 2.01 u |b_e - o| / |d_k| <= 4.02 u C / |d_k| of its exact box's plane b_e;
// the grown plane lies delta / |d_k| further out in t, 3.5x their sum. So
// every axis's computed entry is <= hit.c's and its exit >= hit.c's, hence
// tmin' <= tmin and tmax' >= tmax: a box hit.c passes passes here, and the
// comparison needs no margin. An origin within 4C (the camera rays of the
// packet walk over PNodes, whose inner-child boxes are grown the same way)
// still fits: (2.01 u 5C + 1.01 u 4C) + 2.01 u 5C = 24.1 u C < 32 u C.
template <bool BND = false>
__device__ __forceinline__ bool slab_cons_fast(const SlabRay& r, const Prune& p, float x0, float y0, float z0,
                                               float x1, float y1, float z1, float& near)
{
    const float oix = r.ox * r.ix, oiy = r.oy * r.iy, oiz = r.oz * r.iz;  // shared by a step's boxes (CSE)
    const float mo = fmaxf(fabsf(oix), fmaxf(fabsf(oiy), fabsf(oiz))) * 0x1p-22f;
    const float tx1 = fmaf(x0, r.ix, -oix), tx2 = fmaf(x1, r.ix, -oix);
    const float ty1 = fmaf(y0, r.iy, -oiy), ty2 = fmaf(y1, r.iy, -oiy);
    const float tz1 = fmaf(z0, r.iz, -oiz), tz2 = fmaf(z1, r.iz, -oiz);
    const float nx = fminf(tx1, tx2), ny = fminf(ty1, ty2), nz = fminf(tz1, tz2);
    constexpr float c = 1.0f - 0x1p-20f;
    const float entry = fmaxf(fmaf(nx, c, -fmaf(p.m, fabsf(r.ix), mo)),
                              fmaxf(fmaf(ny, c, -fmaf(p.m, fabsf(r.iy), mo)), fmaf(nz, c, -fmaf(p.m, fabsf(r.iz), mo))));
    const float tmin = fmaxf(nx, fmaxf(ny, nz));
    const float tmax = fminf(fmaxf(tx1, tx2), fminf(fmaxf(ty1, ty2), fmaxf(tz1, tz2)));
    near = tmin;
    if (BND) {
        // the pruning entry without slab_fast's guards either: entry'_k =
        // fl(nx'_k - m |ix_k|) is below the exact entry of the exact box
        // grown by m (Prune) by the growth delta / |d_k| = 32 u C / |d_k| less
        // at most 5.03 u C (the plane) + 2.1 u C (the fma's rounding of a
        // value within 2.1 C / |d_k|) + u m (|ix|'s): a box pruned here is
        // one the guarded test prunes
        const float ent = fmaxf(fmaf(-p.m, fabsf(r.ix), nx), fmaxf(fmaf(-p.m, fabsf(r.iy), ny), fmaf(-p.m, fabsf(r.iz), nz)));
        return !(ent > p.lim) & !(tmax < fmaxf(tmin, kEps));
    }
    const float m = fmaf(fabsf(tmin) + fabsf(tmax), 0x1p-20f, 2.0f * mo);
    // tmax - tmin >= -m and tmax - eps >= -m as one comparison (m has 4x slack
    // over the rounding of either form; a NaN passes, as before)
    return !(entry > p.lim) & !(tmax + m < fmaxf(tmin, kEps));
}

template <bool BND = false>
__device__ __forceinline__ bool slab_cons(const SlabRay& r, const Prune& p, float x0, float y0, float z0, float x1,
                                          float y1, float z1, float& near)
{
    bool pass = slab_cons_fast<BND>(r, p, x0, y0, z0, x1, y1, z1, near);
    if (r.generic) {  // a lane branch taken only by rays with a zero/tiny component
        near = 0.0f;
        pass = !pruned_any(r, p, x0, y0, z0, x1, y1, z1) && slab_test(r, x0, y0, z0, x1, y1, z1);
    }
    return pass;
}

// Per-ray constants of ray_sphere_intersect: a = d.d, 4a and 2a (hit.c:22-28).
// Recomputed from d at each sphere test (eight VALU) instead of held for the
// whole walk (round 3: four VGPRs fewer in every walk loop -- registers, not
// VALU, limit the walks); the same IEEE expressions, so the same bits; 1/(2a)
// -- only the estimate's scale -- from v_rcp_f32 (1 ulp, well inside
// sphere_t's 2^-18 margin).
struct SphRay {
    float ox, oy, oz, dx, dy, dz;
    __device__ __forceinline__ float a() const { return dot3(dx, dy, dz, dx, dy, dz); }
    __device__ __forceinline__ float a4() const { return 4.0f * a(); }  // hit.c:25: (4 * a) * c
    __device__ __forceinline__ float inv2a() const { return __builtin_amdgcn_rcpf(2.0f * a()); }
    __device__ __forceinline__ double a2() const { return (double)(2.0f * a()); }
};

__device__ __forceinline__ SphRay sph_ray(const Ray& r) { return {r.ox, r.oy, r.oz, r.dx, r.dy, r.dz}; }

// hit.c:19-39 without point/normal (computed once for the winner): the t a
// hit would record if it could still become the closest (t <= best, the
// later-DFS-leaf-wins tie rule), else -1.
//
// The discriminant is the reference's float expression (it alone decides
// hit vs miss). t itself is hit.c:28 in double, rounded to float, which costs
// a chain of f64 sqrt/div; it is only evaluated when a float estimate cannot
// rule the hit out. Estimate: s' = sqrt(disc) to ~1 ulp, t' = RN(-b - s') *
// RN(1/(2a)); every step is within a few u = 2^-24 relative of its operands,
// so |t' - t| < 8u (|b| + s') / 2a, and M = 2^-18 (|b| + s') |1/(2a)| bounds
// that 8x over. If t' - M > best the recorded t would exceed best (cannot
// win); if t' + M <= EPS it would fail t > EPS. Otherwise the exact path runs.
template <bool FAST>
__device__ __forceinline__ float sphere_t(const SphRay& r, float4 s, float best)
{
    const float ocx = r.ox - s.x, ocy = r.oy - s.y, ocz = r.oz - s.z;
    const float b = 2.0f * dot3(ocx, ocy, ocz, r.dx, r.dy, r.dz);
    const float c = dot3(ocx, ocy, ocz, ocx, ocy, ocz) - s.w * s.w;
    const float disc = b * b - r.a4() * c;
    if (!(disc > 0.0f)) return -1.0f;
    if (FAST) {
        const float sq = __builtin_amdgcn_sqrtf(disc);
        const float te = (-b - sq) * r.inv2a();
        const float m = (fabsf(b) + sq) * fabsf(r.inv2a()) * 0x1p-18f;
        if (te - m > best || te + m <= kEps) return -1.0f;
    }
    // hit.c:28 in double: (-b - sqrt(disc)) / (2a), rounded to float
    const double num = (double)(-b) - __dsqrt_rn((double)disc);
    const float t = (float)__ddiv_rn(num, r.a2());
    return (t > kEps && t <= best) ? t : -1.0f;
}

// One step of the per-lane DFS walk with on-demand loads (the body of
// closest_bvh's per-lane loop), for kernels that interleave walking with
// other per-lane work.
// TIEKEY: inside an ordered walk the best so far may come from a later DFS
// leaf, so a tie replaces it only for a larger sphere index (the DFS key).
template <bool FAST, bool COUNT, bool TIEKEY = false>
__device__ __forceinline__ void lane_step(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                          uint32_t& next, float& best_t, int& best_s, Counters& cnt)
{
    const float4* p = (const float4*)(sc.nodes32 + next);
    const float4 a = p[0], b = p[1];
    NodeV nd;
    nd.b0 = a.x; nd.b1 = a.y; nd.b2 = a.z; nd.b3 = a.w; nd.b4 = b.x; nd.b5 = b.y;
    nd.sphere = __float_as_int(b.z);
    nd.skip = __float_as_uint(b.w);
    const bool inner = nd.sphere < 0;
    const bool pass = (nd.skip & MIRT_NODE_EMPTY) || slab<FAST>(sr, pr, nd);
    if (COUNT) cnt.nodes++;
    if (pass && inner) {
        next = next + 1;
    } else {
        if (pass) {
            if (COUNT) cnt.spheres++;
            const float t = sphere_t<FAST>(sp, sc.geo[nd.sphere], best_t);
            if (t > 0.0f && (!TIEKEY || t < best_t || nd.sphere > best_s)) {
                best_t = t;
                best_s = nd.sphere;
                if (sc.prune) prune_update(pr, sc, sr.ox, sr.oy, sr.oz, sp.a4(), t);
            }
        }
        next = nd.skip & MIRT_SKIP_MASK;
    }
}

// Closest hit over the flattened tree in the reference's DFS order
// (hit.c:91-109: left before right; the later leaf wins a tie on t, so the
// scan keeps `t <= best`). Each lane keeps only `next`, the index of the
// next node of its own pre-order walk: inner node passed -> i + 1, else
// skip(i). Empty (count 0) leaves always pass the slab test.
//
// UNIFORM: the wave walks the union of its lanes' walks in index order with
// a wave-uniform cursor; at node i only lanes whose next == i act. Lanes
// that did not reach i have next >= skip(i) (no walk can enter a subtree
// without visiting its root), so the cursor advances to i + 1 if any lane
// descended and to skip(i) otherwise -- no stack, no reduction, and every
// node load is a scalar load.
// Otherwise every lane walks its own sequence with vector loads (lane_step).
//
// The uniform walk is a latency-bound chain (load -> test -> next index), so
// each step issues the loads of BOTH possible successors (i + 1 and skip(i))
// before testing node i; the test then overlaps the load latency.
template <bool UNIFORM, bool FAST, bool COUNT>
__device__ __forceinline__ void closest_bvh(const DevScene& sc, const Ray& ray, bool active, float& best_t,
                                            int& best_s, Counters& cnt)
{
    const SlabRay sr = slab_ray(ray);
    const SphRay sp = sph_ray(ray);
    Prune pr = prune_off();
    const uint32_t end = sc.num_nodes;
    const uint32_t last = end - 1;
    uint32_t next = active ? 0u : end;
    best_t = INFINITY;
    best_s = -1;
    if constexpr (UNIFORM) {
        uint32_t cur = __builtin_amdgcn_readfirstlane(__ballot(active) ? 0u : end);
        if (cur >= end) return;
        NodeV nd = load_node_uniform(sc.nodes, cur);
        while (cur < end) {
            if (COUNT) cnt.steps++;
            const uint32_t skip = nd.skip & MIRT_SKIP_MASK;
            const bool inner = nd.sphere < 0;
            // both loads always issue (a leaf's skip is i + 1: the second is a
            // scalar-cache hit); nothing reads them until the step is decided
            const NodeV na = load_node_uniform(sc.nodes, min(cur + 1, last));
            const NodeV nb = load_node_uniform(sc.nodes, min(skip, last));
            bool descend = false;
            if (next == cur) {
                const bool pass = (nd.skip & MIRT_NODE_EMPTY) || slab<FAST>(sr, pr, nd);
                if (COUNT) cnt.nodes++;
                if (pass && inner) {
                    next = cur + 1;
                    descend = true;
                } else {
                    next = skip;
                    if (pass) {
                        if (COUNT) cnt.spheres++;
                        const float t = sphere_t<FAST>(sp, nd.g, best_t);
                        if (t > 0.0f) {
                            best_t = t;
                            best_s = nd.sphere;
                            if (sc.prune) prune_update(pr, sc, ray.ox, ray.oy, ray.oz, sp.a4(), t);
                        }
                    }
                }
            }
            if (__builtin_amdgcn_readfirstlane(__ballot(descend) != 0)) {  // wave-uniform branch
                cur = cur + 1;
                nd = na;
            } else {
                cur = skip;
                nd = nb;
            }
        }
    } else {
        // per lane: 32 B of box/links per step, the leaf sphere only when the
        // leaf's box passes
        while (__ballot(next < end)) {
            if (COUNT) cnt.steps++;
            if (next < end) lane_step<FAST, COUNT>(sc, sr, sp, pr, next, best_t, best_s, cnt);
        }
    }
}

__device__ __forceinline__ float wave_min(float v)
{
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v = fminf(v, __shfl_xor(v, off));
    return v;
}

// Node-parallel walk of ONE (wave-uniform) ray by the whole wave. Rays with
// an exactly zero direction component (the image's centre row and column
// under an axis-aligned camera) ignore that slab entirely (hit.c:54-57), so
// they pass most boxes and walk a large part of the tree -- the centre
// pixel of the default camera visits all 29,399 nodes at 10k spheres. Walked
// one node per step they set the frame time; here every step tests the 64
// consecutive pre-order nodes [cur, cur + 64) in parallel (coalesced loads,
// sphere tests for every passing leaf), then replays the DFS over the
// chunk's pass/leaf masks on the scalar unit: a run of passed inner nodes
// advances one by one, any other node jumps to its skip. Hit candidates are
// the visited passing leaves; the chunk's winner (min t, later DFS index on
// a tie) replaces the running best when t <= best -- the sequential rule of
// hit.c:105-108 applied chunk by chunk.
template <bool FAST, bool COUNT>
__device__ __forceinline__ void closest_bvh_chunked(const DevScene& sc, const Ray& ray, float& best_t, int& best_s,
                                                    Counters& cnt)
{
    const SlabRay sr = slab_ray(ray);
    const SphRay sp = sph_ray(ray);
    const uint32_t end = sc.num_nodes;
    const uint32_t lane = threadIdx.x & 63;
    uint32_t cur = 0;
    float bt = INFINITY;
    int bs = -1;
    Prune pr = prune_start(sc, ray.ox, ray.oy, ray.oz);  // wave-uniform: one ray
    while (cur < end) {
        if (COUNT) cnt.steps++;
        const uint32_t base = cur;
        const uint32_t i = base + lane;
        bool pass = false, leaf = false;
        uint32_t skip = end;
        int sph = -1;
        float t = -1.0f;
        if (i < end) {
            const NodeV nd = load_node_lane(sc.nodes, i);
            skip = nd.skip & MIRT_SKIP_MASK;
            leaf = nd.sphere >= 0;
            sph = nd.sphere;
            // pruned against the best at the chunk's start: a box beyond it
            // is beyond every later best too
            pass = (nd.skip & MIRT_NODE_EMPTY) || (!(FAST && pruned_any(sr, pr, nd)) && slab<FAST>(sr, prune_off(), nd));
            if (pass && leaf) t = sphere_t<FAST>(sp, nd.g, bt);
        }
        const uint64_t descend = __ballot(pass && !leaf);
        uint64_t visited = 0;
        uint32_t c = cur;
        const uint32_t lim = min(base + 64, end);
        while (c < lim) {
            uint32_t k = c - base;
            // consume the run of passed inner nodes starting at k
            const uint64_t run = ~(descend >> k);
            const uint32_t n = run ? (uint32_t)__builtin_ctzll(run) : 64u - k;
            const uint32_t stop = min(k + n, lim - base);
            if (stop > k) visited |= (stop - k >= 64 ? ~0ull : ((1ull << (stop - k)) - 1)) << k;
            c = base + stop;
            if (c >= lim) break;
            k = stop;
            visited |= 1ull << k;  // a leaf or a failed node: jump past its subtree
            c = __builtin_amdgcn_readlane(skip, k);
        }
        cur = c;
        const bool cand = ((visited >> lane) & 1) && t > 0.0f;
        const float tmin = wave_min(cand ? t : INFINITY);
        if (tmin <= bt && tmin < INFINITY) {
            const uint64_t eq = __ballot(cand && t == tmin);
            const int last = 63 - __builtin_clzll(eq);
            bt = tmin;
            bs = __builtin_amdgcn_readlane(sph, last);
            if (FAST && sc.prune) prune_update(pr, sc, ray.ox, ray.oy, ray.oz, sp.a4(), bt);
        }
        const uint64_t passed_leaves = __ballot(pass && leaf);
        if (COUNT) {  // uniform values: every lane holds the ray's totals
            cnt.nodes += __popcll(visited);
            cnt.spheres += __popcll(visited & passed_leaves);
        }
    }
    best_t = bt;
    best_s = bs;
}

__device__ __forceinline__ float readlane_f(float v, int l)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

struct PNodeV {
    float a0, a1, a2, a3, a4, a5;  // child 0 slot
    float b0, b1, b2, b3, b4, b5;  // child 1 slot
    uint32_t r0, r1, flat, end;
};

__device__ __forceinline__ PNodeV load_pnode_uniform(const PNode* base, uint32_t i)
{
    const cu32_t* p = (const cu32_t*)base + 16u * i;
    PNodeV n;
    n.a0 = __uint_as_float(p[0]);
    n.a1 = __uint_as_float(p[1]);
    n.a2 = __uint_as_float(p[2]);
    n.a3 = __uint_as_float(p[3]);
    n.a4 = __uint_as_float(p[4]);
    n.a5 = __uint_as_float(p[5]);
    n.b0 = __uint_as_float(p[6]);
    n.b1 = __uint_as_float(p[7]);
    n.b2 = __uint_as_float(p[8]);
    n.b3 = __uint_as_float(p[9]);
    n.b4 = __uint_as_float(p[10]);
    n.b5 = __uint_as_float(p[11]);
    n.r0 = p[12];
    n.r1 = p[13];
    n.flat = p[14];
    n.end = p[15];
    return n;
}

__device__ __forceinline__ PNodeV load_pnode_lane(const PNode* base, uint32_t i)
{
    const float4* p = (const float4*)(base + i);
    const float4 q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3];
    PNodeV n;
    n.a0 = q0.x;
    n.a1 = q0.y;
    n.a2 = q0.z;
    n.a3 = q0.w;
    n.a4 = q1.x;
    n.a5 = q1.y;
    n.b0 = q1.z;
    n.b1 = q1.w;
    n.b2 = q2.x;
    n.b3 = q2.y;
    n.b4 = q2.z;
    n.b5 = q2.w;
    n.r0 = __float_as_uint(q3.x);
    n.r1 = __float_as_uint(q3.y);
    n.flat = __float_as_uint(q3.z);
    n.end = __float_as_uint(q3.w);
    return n;
}

__device__ __forceinline__ bool pref_leaf(uint32_t r) { return r != kPNone && (r & kPLeaf); }
__device__ __forceinline__ bool pref_inner(uint32_t r) { return !(r & kPLeaf); }

// A leaf's sphere (hit.c:94-99) as a candidate of an ORDERED walk: the
// closest hit is the least t, a tie going to the later DFS leaf (hit.c:108),
// which is the larger sphere index for the trees `DevScene::ordered` admits
// -- so the result does not depend on the visiting order.
template <bool FAST>
__device__ __forceinline__ void consider_sphere(const DevScene& sc, const SphRay& sp, Prune& pr, float ox, float oy,
                                                float oz, int si, float4 g, float& best_t, int& best_s)
{
    const float t = sphere_t<FAST>(sp, g, best_t);
    if (t > 0.0f && (t < best_t || si > best_s)) {
        best_t = t;
        best_s = si;
        if (sc.prune) prune_update(pr, sc, ox, oy, oz, sp.a4(), t);
    }
}

// One child slot of a PNode for one lane: a leaf's box then its sphere; an
// inner child's box. Returns whether the walk should enter the child (inner
// and passed), with its entry estimate.
template <bool FAST, bool COUNT, bool BND = false, bool SFIRST = false>
__device__ __forceinline__ bool visit_child(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                            uint32_t ref, float s0, float s1, float s2, float s3, float s4, float s5,
                                            float& near, float& best_t, int& best_s, Counters& cnt)
{
    if (ref == kPNone) return false;
    if (ref & kPLeaf) {
        if (COUNT) cnt.nodes++;
        const int si = (int)(ref & kPIndex);
        if constexpr (SFIRST && FAST && !COUNT) {
            // (the camera packets: the sphere is a wave-uniform load) the
            // sphere first, the leaf's exact box only for a hit that can
            // win (the bounce walk's gate order, wide_leaf): the outcome is
            // (box passes) AND (a hit that wins), and a box beyond the best
            // hit (pruned) cannot hold one. Round 6: the camera pass 0.32 ->
            // 0.29 ms, depth 1 +6%, 1080p/100k +6% (MEASUREMENTS.md §D)
            const float t = sphere_t<FAST>(sp, sc.geo[si], best_t);
            if (t > 0.0f && (t < best_t || si > best_s) && slab_box<FAST>(sr, pr, s0, s1, s2, s3, s4, s5, near)) {
                best_t = t;
                best_s = si;
                if (sc.prune) prune_update(pr, sc, sr.ox, sr.oy, sr.oz, sp.a4(), t);
            }
            return false;
        }
        if (slab_box<FAST>(sr, pr, s0, s1, s2, s3, s4, s5, near)) {
            if (COUNT) cnt.spheres++;
            consider_sphere<FAST>(sc, sp, pr, sr.ox, sr.oy, sr.oz, si, sc.geo[si], best_t, best_s);
        }
        return false;
    }
    if (COUNT) cnt.nodes++;
    // an inner box needs only a conservative test: the reference's test is
    // monotone under containment, so a ray that passes any leaf box below
    // passes this one too, and every leaf is still gated exactly
    if (FAST) return slab_cons<BND>(sr, pr, s0, s1, s2, s3, s4, s5, near);
    return slab_box<FAST>(sr, pr, s0, s1, s2, s3, s4, s5, near);
}

// Ordered closest hit of a wave of rays walked as one packet (camera rays),
// over PNodes with scalar loads. `mask` holds the lanes that passed every
// box on the path to the current node, so a lane tests a child only when
// hit.c:91-109 would (the reference gates each subtree by all its
// ancestors' boxes); a node's two children are tested together, leaf
// children's spheres at once, and the walk enters the child that the lanes
// passing both see nearer (a vote), pushing the other (node, lane mask) on
// a stack kept one entry per lane (entry k in lane k). Pruning (Prune)
// drops boxes beyond each lane's best hit. Stack depth <= tree depth + 1 <=
// 64 (checked at upload).
template <bool FAST, bool COUNT, bool BND = false>
__device__ __forceinline__ void closest_packet_ordered(const DevScene& sc, const Ray& ray, bool active, float& best_t,
                                                       int& best_s, Counters& cnt)
{
    const SlabRay sr = slab_ray(ray);
    const SphRay sp = sph_ray(ray);
    Prune pr = prune_start(sc, ray.ox, ray.oy, ray.oz);  // m0: zero-component lanes prune from the start
    best_t = INFINITY;
    best_s = -1;
    const uint32_t lane = threadIdx.x & 63;
    uint64_t mask = __ballot(active);
    uint32_t cur = 0;
    uint32_t top = 0;
    uint32_t st_node = 0, st_lo = 0, st_hi = 0;
    while (mask) {
        if (COUNT) cnt.steps++;
        const PNodeV nd = load_pnode_uniform(sc.pnodes, cur);
        const bool in = (mask >> lane) & 1;
        float e0 = 0.0f, e1 = 0.0f;
        bool h0 = false, h1 = false;
        if (in) {
            h0 = visit_child<FAST, COUNT, BND, true>(sc, sr, sp, pr, nd.r0, nd.a0, nd.a1, nd.a2, nd.a3, nd.a4, nd.a5,
                                                     e0, best_t, best_s, cnt);
            h1 = visit_child<FAST, COUNT, BND, true>(sc, sr, sp, pr, nd.r1, nd.b0, nd.b1, nd.b2, nd.b3, nd.b4, nd.b5,
                                                     e1, best_t, best_s, cnt);
        }
        const uint64_t m0 = __ballot(h0), m1 = __ballot(h1);
        if (m0 && m1) {
            const uint64_t both = m0 & m1;
            const uint64_t v = __ballot(((both >> lane) & 1) && e1 < e0);
            const bool swap = 2 * __popcll(v) > __popcll(both);
            const uint32_t second = swap ? nd.r0 : nd.r1;
            const uint64_t sm = swap ? m0 : m1;
            if (lane == top) {
                st_node = second;
                st_lo = (uint32_t)sm;
                st_hi = (uint32_t)(sm >> 32);
            }
            top++;
            cur = swap ? nd.r1 : nd.r0;
            mask = swap ? m1 : m0;
        } else if (m0 | m1) {
            cur = m0 ? nd.r0 : nd.r1;
            mask = m0 | m1;
        } else if (top > 0) {
            top--;
            cur = (uint32_t)__builtin_amdgcn_readlane(st_node, top);
            // readlane returns int: zero-extend both halves
            mask = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(st_hi, top) << 32) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane(st_lo, top);
        } else {
            break;
        }
    }
}

// Per-lane DFS walk (any tree, the reference order): `cur` is the next flat
// node, the walk ends at `end` (kPNone: done).
struct DfsWalk {
    uint32_t cur, end;
};

// Per-lane four-wide walk (bounce rays): `cur` is the HNode to visit (kPNone:
// done) or, while `end` != 0, the next node of a flat DFS segment ending at
// `end`. Subtrees still to visit wait on a per-lane stack in LDS (`stk`:
// entry k at stk[k * kWideStride]); a step pushes all passing inner slots but
// the nearest, farthest first. When that would overflow kWideStack, the
// node's whole subtree is walked as a DFS segment instead.
#ifndef MIRT_WIDE_STACK
#define MIRT_WIDE_STACK 20
#endif
constexpr int kWideStack = MIRT_WIDE_STACK;
constexpr int kWideStride = 256;  // threads per workgroup of the bounce kernel
struct WideWalk {
    uint32_t cur, end, top;
};

__device__ __forceinline__ WideWalk wide_walk_start(const DevScene& sc, bool active)
{
    return WideWalk{active ? sc.wide_root : kPNone, 0u, 0u};
}
__device__ __forceinline__ bool wide_walking(const WideWalk& w) { return w.cur != kPNone; }

__device__ __forceinline__ void wide_walk_pop(WideWalk& w, const uint32_t* stk)
{
    if (w.top == 0) {
        w.cur = kPNone;
        return;
    }
    w.top--;
    w.cur = stk[w.top * kWideStride];
}

// Compare-exchange of (entry, ref) pairs: ascending entry.
__device__ __forceinline__ void cx(float& ka, uint32_t& ra, float& kb, uint32_t& rb)
{
    const bool sw = kb < ka;
    const float k = sw ? kb : ka;
    const uint32_t r = sw ? rb : ra;
    kb = sw ? ka : kb;
    rb = sw ? ra : rb;
    ka = k;
    ra = r;
}

__device__ __forceinline__ float h_lo(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v & 0xffffu)); }
__device__ __forceinline__ float h_hi(uint32_t v) { return (float)__builtin_bit_cast(_Float16, (uint16_t)(v >> 16)); }

// The leaf gate of a leaf slot whose fp16 box passed: its exact box under
// hit.c's test, then its sphere. COUNT: the sphere test counts.
//
// The gate's outcome is (box passes) AND (sphere hit that wins), so the
// timed build tests the sphere first and reads the exact box (32 of the
// record's 48 B) only for a winning hit -- rare: most gates end at the
// sphere. Same box test, same prune state, same result; COUNT keeps the
// reference's order so the box-gated sphere tests are what it counts.
template <bool FAST, bool COUNT>
__device__ __forceinline__ void wide_leaf(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                          uint32_t ref, float& best_t, int& best_s, Counters& cnt)
{
    const uint32_t li = ref & ~kPLeaf;
    const float4* lp = (const float4*)(sc.leaf_box + li);
    float e;
    if constexpr (COUNT) {
        const float4 l0 = lp[0], l1 = lp[1], g = sc.leaf_geo[li];
        if (slab_box<FAST>(sr, pr, l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, e)) {
            cnt.spheres++;
            consider_sphere<FAST>(sc, sp, pr, sr.ox, sr.oy, sr.oz, __float_as_int(l1.z), g, best_t, best_s);
        }
    } else {
        const float t = sphere_t<FAST>(sp, sc.leaf_geo[li], best_t);
        if (t > 0.0f) {
            const float4 l0 = lp[0], l1 = lp[1];
            const int si = __float_as_int(l1.z);
            if ((t < best_t || si > best_s) && slab_box<FAST>(sr, pr, l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, e)) {
                best_t = t;
                best_s = si;
                if (sc.prune) prune_update(pr, sc, sr.ox, sr.oy, sr.oz, sp.a4(), t);
            }
        }
    }
}

// The timed gate of wide_leaf with its sphere already loaded: the sphere,
// then (for a hit that could win) the exact box.
__device__ __forceinline__ void leaf_gate(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                          uint32_t ref, float4 g, float& best_t, int& best_s)
{
    const float t = sphere_t<true>(sp, g, best_t);
    if (t > 0.0f) {
        const float4* lp = (const float4*)(sc.leaf_box + (ref & ~kPLeaf));
        const float4 l0 = lp[0], l1 = lp[1];
        const int si = __float_as_int(l1.z);
        float e;
        if ((t < best_t || si > best_s) && slab_box<true>(sr, pr, l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, e)) {
            best_t = t;
            best_s = si;
            if (sc.prune) prune_update(pr, sc, sr.ox, sr.oy, sr.oz, sp.a4(), t);
        }
    }
}

// hc / hc_n: the first hc_n HNodes (the tree's top levels, visited by
// every ray) staged in LDS by the caller; a node there is read from LDS
// instead of through the vector-memory path (the bounce kernel's busiest
// unit, TD: its cost is the bytes returned per lane, however coalesced).
template <bool FAST, bool COUNT, bool BATCH = false, bool BND = false>
__device__ __forceinline__ void wide_lane_step(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                               WideWalk& w, uint32_t* stk, float& best_t, int& best_s, Counters& cnt,
                                               lds_uint4* hc = nullptr, uint32_t hc_n = 0)
{
    if (COUNT) cnt.steps++;
    if (w.end) {
        lane_step<FAST, COUNT, true>(sc, sr, sp, pr, w.cur, best_t, best_s, cnt);
        if (w.cur >= w.end) {
            w.end = 0;
            wide_walk_pop(w, stk);
        }
        return;
    }
    // 1. the four conservative slot tests, computed for every slot (no branch
    // for the compiler to sink a load into); COUNT: a slot test is a node test
    float e0 = 0.0f, e1 = 0.0f, e2 = 0.0f, e3 = 0.0f;
    bool h0, h1, h2, h3;
    uint4 q3;  // the slots' references
    {
        uint4 s0, s1, s2, s3;
        if (w.cur < hc_n) {
            lds_uint4* p = hc + 4 * w.cur;
            s0 = lds_load(p);
            s1 = lds_load(p + 1);
            s2 = lds_load(p + 2);
            s3 = lds_load(p + 3);
        } else {
            const uint4* p = (const uint4*)(sc.hnodes + w.cur);
            s0 = p[0];
            s1 = p[1];
            s2 = p[2];
            s3 = p[3];
        }
        auto test = [&](const uint4& q, float& e) {
            if (COUNT && q.w != kPNone) cnt.nodes++;
            const bool pass =
                slab_cons<BND>(sr, pr, h_lo(q.x), h_lo(q.y), h_lo(q.z), h_hi(q.x), h_hi(q.y), h_hi(q.z), e);
            return pass & (q.w != kPNone);
        };
        h0 = test(s0, e0);
        h1 = test(s1, e1);
        h2 = test(s2, e2);
        h3 = test(s3, e3);
        q3 = make_uint4(s0.w, s1.w, s2.w, s3.w);
    }
    uint32_t lm = (uint32_t)(h0 && (q3.x & kPLeaf)) | (uint32_t)(h1 && (q3.y & kPLeaf)) << 1 |
                  (uint32_t)(h2 && (q3.z & kPLeaf)) << 2 | (uint32_t)(h3 && (q3.w & kPLeaf)) << 3;
    h0 = h0 && !(lm & 1);
    h1 = h1 && !(lm & 2);
    h2 = h2 && !(lm & 4);
    h3 = h3 && !(lm & 8);
    // 2. passing inner slots: nearest next, the others pushed farthest first.
    // Before the leaf gates, so the slots' keys and flags are dead while the
    // gates run (the gates' outcome does not depend on the order)
    const uint32_t n = (uint32_t)h0 + (uint32_t)h1 + (uint32_t)h2 + (uint32_t)h3;
    if (n == 0) {
        wide_walk_pop(w, stk);
    } else if (w.top + n - 1 > (uint32_t)kWideStack) {
        // the node's whole subtree as a flat DFS segment, its leaf slots included
        const HAux ax = sc.haux[w.cur];
        w.cur = ax.flat + 1;
        w.end = ax.end;
        lm = 0;
    } else {
        // failing slots get +inf keys and passing ones a finite key, so the n
        // passing slots sort first
        constexpr float big = 3.0e38f;
        float k0 = h0 ? fminf(e0, big) : INFINITY, k1 = h1 ? fminf(e1, big) : INFINITY;
        float k2 = h2 ? fminf(e2, big) : INFINITY, k3 = h3 ? fminf(e3, big) : INFINITY;
        uint32_t a0 = q3.x, a1 = q3.y, a2 = q3.z, a3 = q3.w;
        cx(k0, a0, k1, a1);
        cx(k2, a2, k3, a3);
        cx(k0, a0, k2, a2);
        cx(k1, a1, k3, a3);
        cx(k1, a1, k2, a2);
        if (n >= 2) stk[(w.top + n - 2) * kWideStride] = a1;
        if (n >= 3) stk[(w.top + n - 3) * kWideStride] = a2;
        if (n >= 4) stk[(w.top + n - 4) * kWideStride] = a3;
        w.top += n - 1;
        w.cur = a0;
    }
    // 3. passing leaf slots (the node's boxes are dead here): each lane works
    // through its own list, so the gate code runs max-over-lanes times
    // instead of once per slot that any lane passes
    if constexpr (BATCH && FAST && !COUNT) {
        // every passing leaf's sphere requested at once (one dependent round
        // trip for the step instead of one per leaf), then the gates in slot
        // order against the best so far (least t, a tie to the larger index:
        // order-free). Pays where the leaf records miss L2 (a 1M-sphere
        // scene); on an L2-resident tree the extra live registers cost more
        // than the round trips they save
        if (__ballot(lm != 0)) {
            float4 g0, g1, g2, g3;
            if (lm & 1) g0 = sc.leaf_geo[q3.x & ~kPLeaf];
            if (lm & 2) g1 = sc.leaf_geo[q3.y & ~kPLeaf];
            if (lm & 4) g2 = sc.leaf_geo[q3.z & ~kPLeaf];
            if (lm & 8) g3 = sc.leaf_geo[q3.w & ~kPLeaf];
            if (lm & 1) leaf_gate(sc, sr, sp, pr, q3.x, g0, best_t, best_s);
            if (lm & 2) leaf_gate(sc, sr, sp, pr, q3.y, g1, best_t, best_s);
            if (lm & 4) leaf_gate(sc, sr, sp, pr, q3.z, g2, best_t, best_s);
            if (lm & 8) leaf_gate(sc, sr, sp, pr, q3.w, g3, best_t, best_s);
        }
    } else {
        while (__ballot(lm != 0)) {
            if (lm) {
                const uint32_t i = __builtin_ctz(lm);
                lm &= lm - 1;
                const uint32_t ref = i == 0 ? q3.x : i == 1 ? q3.y : i == 2 ? q3.z : q3.w;
                wide_leaf<FAST, COUNT>(sc, sr, sp, pr, ref, best_t, best_s, cnt);
            }
        }
    }
}

// ---------------------------------------------------------------- quad walk
// The four-wide walk with one ray per QUAD of lanes (lane j of a quad owns
// slot j of every HNode): the four slot tests of a step run side by side,
// and the quad reads its node as one 64-B line (four lanes x one dwordx4)
// instead of one lane issuing four. The ray and the walk state are
// replicated in the quad's lanes and change only through quad-uniform
// values; candidates and the order of the passing children are reduced
// across the quad with DPP. The result is the same closest hit: least t,
// a tie to the larger sphere index -- an order-free rule.

template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int kQuadXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kQuadXor2 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int kQuadXor3 = 0x1B;  // quad_perm [3,2,1,0]

struct QuadWalk {
    uint32_t cur, end, top;
};

// a better than b: least t, a tie to the larger sphere index
__device__ __forceinline__ bool cand_better(float ta, int sa, float tb, int sb)
{
    return ta < tb || (ta == tb && sa > sb);
}

template <int CTRL>
__device__ __forceinline__ void cand_merge(float& t, int& si)
{
    const float ot = __uint_as_float(quad_perm<CTRL>(__float_as_uint(t)));
    const int os = (int)quad_perm<CTRL>((uint32_t)si);
    if (cand_better(ot, os, t, si)) {
        t = ot;
        si = os;
    }
}

// `stk`: this ray's LDS stack column (entry k at stk[k * STRIDE], CAP entries).
template <bool FAST, int STRIDE, int CAP, bool BND = false>
__device__ __forceinline__ void quad_step(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                          QuadWalk& w, uint32_t* stk, float& best_t, int& best_s,
                                          lds_uint4* hc = nullptr, uint32_t hc_n = 0)
{
    Counters cnt{0, 0, 0, 0, 0};
    if (w.end) {  // DFS segment (the stack was full): every lane of the quad walks it alike
        lane_step<FAST, false, true>(sc, sr, sp, pr, w.cur, best_t, best_s, cnt);
        if (w.cur >= w.end) {
            w.end = 0;
            if (w.top == 0) {
                w.cur = kPNone;
            } else {
                w.top--;
                w.cur = stk[w.top * STRIDE];
            }
        }
        return;
    }
    const uint32_t j = threadIdx.x & 3;
    uint4 q;
    if (w.cur < hc_n)
        q = lds_load(hc + 4 * w.cur + j);
    else
        q = ((const uint4*)(sc.hnodes + w.cur))[j];
    float e = 0.0f;
    const bool pass = slab_cons<BND>(sr, pr, h_lo(q.x), h_lo(q.y), h_lo(q.z), h_hi(q.x), h_hi(q.y), h_hi(q.z), e) &
                      (q.w != kPNone);
    // a passing leaf: its exact gate and sphere give this lane's candidate
    float ct = INFINITY;
    int cs = -1;
    if (pass && (q.w & kPLeaf)) {  // sphere first, the exact box only for a hit (wide_leaf)
        const float4* lp = (const float4*)(sc.leaf_box + (q.w & ~kPLeaf));
        const float t = sphere_t<FAST>(sp, sc.leaf_geo[q.w & ~kPLeaf], best_t);
        if (t > 0.0f) {
            const float4 l0 = lp[0], l1 = lp[1];
            float ee;
            if (slab_box<FAST>(sr, pr, l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, ee)) {
                ct = t;
                cs = __float_as_int(l1.z);
            }
        }
    }
    cand_merge<kQuadXor1>(ct, cs);
    cand_merge<kQuadXor2>(ct, cs);
    if (cs >= 0 && cand_better(ct, cs, best_t, best_s)) {
        best_t = ct;
        best_s = cs;
        if (sc.prune) prune_update(pr, sc, sr.ox, sr.oy, sr.oz, sp.a4(), ct);
    }
    // the passing inner slots: rank by entry (ties by slot), nearest next
    const bool inner = pass && !(q.w & kPLeaf);
    const float key = inner ? fminf(e, 3.0e38f) : INFINITY;
    const float k1 = __uint_as_float(quad_perm<kQuadXor1>(__float_as_uint(key)));
    const float k2 = __uint_as_float(quad_perm<kQuadXor2>(__float_as_uint(key)));
    const float k3 = __uint_as_float(quad_perm<kQuadXor3>(__float_as_uint(key)));
    const uint32_t rank = (uint32_t)(k1 < key || (k1 == key && (j ^ 1) < j)) +
                          (uint32_t)(k2 < key || (k2 == key && (j ^ 2) < j)) +
                          (uint32_t)(k3 < key || (k3 == key && (j ^ 3) < j));
    const uint32_t n = (uint32_t)__popcll((__ballot(inner) >> (threadIdx.x & 60)) & 0xF);
    uint32_t nx = inner && rank == 0 ? q.w + 1 : 0u;  // + 1: 0 means none
    nx |= quad_perm<kQuadXor1>(nx);
    nx |= quad_perm<kQuadXor2>(nx);
    if (n == 0) {
        if (w.top == 0) {
            w.cur = kPNone;
        } else {
            w.top--;
            w.cur = stk[w.top * STRIDE];
        }
        return;
    }
    if (w.top + n - 1 > (uint32_t)CAP) {
        const HAux ax = sc.haux[w.cur];
        w.cur = ax.flat + 1;
        w.end = ax.end;
        return;
    }
    if (inner && rank > 0) stk[(w.top + n - 1 - rank) * STRIDE] = q.w;
    w.top += n - 1;
    w.cur = nx - 1;
}

// ---------------------------------------------------------------- solo walk
// The last ray of a bounce wave (the queue is dry and the quad drain has one
// ray left): all 16 quads of the wave walk its four-wide tree at once. Each
// quad visits one node per step (slot j in lane j, as quad_step) and goes on
// with its nearest passing child; the other passing children wait on ONE
// stack spread over the wave's 64 LDS columns (entry k at row k / 64, column
// k % 64: the wave's other chains are done, so their columns are free), and
// idle quads take the stack's top entries. A step thus covers up to 16 nodes
// instead of one, so the launch's longest chains -- which set when a
// persistent launch ends -- take far fewer dependent round trips. The best
// hit is reduced over the wave after every step (min t, a tie to the larger
// sphere index: order-free, so the same closest hit as any other walk). A
// node whose children would overflow the stack is walked as its flat DFS
// segment by its quad (lane_step), as quad_step does.
struct SoloWalk {
    uint32_t cur, end;  // this quad's node (kPNone: idle) or flat DFS segment (end != 0)
    uint32_t top;       // stack depth (wave-uniform)
};

__device__ __forceinline__ uint32_t* solo_slot(uint32_t* wst, uint32_t k)
{
    return wst + (k >> 6) * kWideStride + (k & 63u);
}

// One step of the solo walk; false once every quad is idle and the stack is
// empty. wst: the wave's LDS stack (column 0 of its 64), CAP entries.
template <bool FAST, int CAP, bool BND = false>
__device__ __forceinline__ bool solo_step(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr,
                                          SoloWalk& w, uint32_t* wst, float& best_t, int& best_s, lds_uint4* hc,
                                          uint32_t hc_n)
{
    const uint32_t lane = threadIdx.x & 63, j = lane & 3;
    // 1. idle quads take the stack's top entries (quad of idle rank r: entry top - 1 - r)
    const uint64_t idle = __ballot(w.cur == kPNone && j == 0);
    const uint32_t take = min((uint32_t)__popcll(idle), w.top);
    if (w.cur == kPNone) {
        const uint32_t qb = lane & ~3u;
        const uint32_t r = (uint32_t)__popcll(qb ? idle & ((1ull << qb) - 1) : 0ull);
        if (r < take) w.cur = *solo_slot(wst, w.top - 1 - r);
    }
    w.top -= take;
    if (!__ballot(w.cur != kPNone)) return false;
    float ct = INFINITY;   // this lane's candidate
    int cs = -1;
    bool push = false;
    Counters cnt{0, 0, 0, 0, 0};
    if (w.cur != kPNone && w.end) {
        // a flat DFS segment: the quad's four lanes walk it alike
        float bt = best_t;
        int bs = best_s;
        lane_step<FAST, false, true>(sc, sr, sp, pr, w.cur, bt, bs, cnt);
        if (bs != best_s || bt != best_t) {
            ct = bt;
            cs = bs;
        }
        if (w.cur >= w.end) {
            w.end = 0;
            w.cur = kPNone;
        }
    }
    bool seg_fallback = false;
    uint32_t nx = 0;
    bool inner = false;
    uint32_t rank = 0, n_in = 0, qref = kPNone;
    if (w.cur != kPNone && !w.end) {
        uint4 q;
        if (w.cur < hc_n)
            q = lds_load(hc + 4 * w.cur + j);
        else
            q = ((const uint4*)(sc.hnodes + w.cur))[j];
        qref = q.w;
        float e = 0.0f;
        const bool pass =
            slab_cons<BND>(sr, pr, h_lo(q.x), h_lo(q.y), h_lo(q.z), h_hi(q.x), h_hi(q.y), h_hi(q.z), e) &
            (q.w != kPNone);
        if (pass && (q.w & kPLeaf)) {  // sphere first, the exact box only for a hit (wide_leaf)
            const float4* lp = (const float4*)(sc.leaf_box + (q.w & ~kPLeaf));
            const float t = sphere_t<FAST>(sp, sc.leaf_geo[q.w & ~kPLeaf], best_t);
            if (t > 0.0f) {
                const float4 l0 = lp[0], l1 = lp[1];
                float ee;
                if (slab_box<FAST>(sr, pr, l0.x, l0.y, l0.z, l0.w, l1.x, l1.y, ee)) {
                    ct = t;
                    cs = __float_as_int(l1.z);
                }
            }
        }
        inner = pass && !(q.w & kPLeaf);
        const float key = inner ? fminf(e, 3.0e38f) : INFINITY;
        const float k1 = __uint_as_float(quad_perm<kQuadXor1>(__float_as_uint(key)));
        const float k2 = __uint_as_float(quad_perm<kQuadXor2>(__float_as_uint(key)));
        const float k3 = __uint_as_float(quad_perm<kQuadXor3>(__float_as_uint(key)));
        rank = (uint32_t)(k1 < key || (k1 == key && (j ^ 1) < j)) + (uint32_t)(k2 < key || (k2 == key && (j ^ 2) < j)) +
               (uint32_t)(k3 < key || (k3 == key && (j ^ 3) < j));
        n_in = (uint32_t)__popcll((__ballot(inner) >> (lane & 60)) & 0xF);
        nx = inner && rank == 0 ? q.w + 1 : 0u;  // + 1: 0 means none
        nx |= quad_perm<kQuadXor1>(nx);
        nx |= quad_perm<kQuadXor2>(nx);
        push = inner && rank > 0;
    }
    // 2. the pushes of every quad, or -- if they would overflow the stack --
    // each pushing quad walks its node's subtree as a flat DFS segment
    const uint64_t pm = __ballot(push);
    const uint32_t np = (uint32_t)__popcll(pm);
    if (w.top + np > (uint32_t)CAP) seg_fallback = true;   // wave-uniform
    if (w.cur != kPNone && !w.end) {
        if (seg_fallback && n_in > 1) {
            const HAux ax = sc.haux[w.cur];
            w.cur = ax.flat + 1;
            w.end = ax.end;
        } else {
            w.cur = n_in ? nx - 1 : kPNone;
        }
    }
    if (!seg_fallback) {
        if (push) *solo_slot(wst, w.top + __builtin_amdgcn_mbcnt_hi((uint32_t)(pm >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)pm, 0u))) = qref;
        w.top += np;
    }
    // 3. the best hit over the wave (every lane then holds it)
    if (!cand_better(ct, cs, best_t, best_s) || cs < 0) {
        ct = best_t;
        cs = best_s;
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
        const float ot = __shfl_xor(ct, off);
        const int os = __shfl_xor(cs, off);
        if (cand_better(ot, os, ct, cs)) {
            ct = ot;
            cs = os;
        }
    }
    if (cs >= 0 && cand_better(ct, cs, best_t, best_s)) {
        best_t = ct;
        best_s = cs;
    }
    // the prune state follows the (now wave-uniform) best
    if (best_s >= 0 && sc.prune) prune_update(pr, sc, sr.ox, sr.oy, sr.oz, sp.a4(), best_t);
    return true;
}

// Closest hit for every active lane: degenerate rays (a zero or tiny
// direction component, `SlabRay::generic`) one at a time with the whole
// wave (closest_bvh_chunked), the rest with the lane-parallel walk (or the
// ordered packet walk, for UNIFORM on a tree that admits it).
template <bool UNIFORM, bool FAST, bool COUNT>
__device__ __forceinline__ void closest_hit(const DevScene& sc, const Ray& ray, bool active, float& best_t,
                                            int& best_s, Counters& cnt, uint32_t* wstk = nullptr)
{
    bool gen = active && slab_ray(ray).generic;
    if (UNIFORM && FAST && sc.ordered) {
        // with pruning (sc.ordered implies it), a zero-component ray is held
        // to boxes around its own coordinate (pruned_any) and walks in the
        // packet like any other
        closest_packet_ordered<FAST, COUNT>(sc, ray, active, best_t, best_s, cnt);
        gen = false;
    } else if (!UNIFORM && FAST && sc.wide && wstk) {
        // the bounce kernel's walk (wstk: a kWideStack-entry LDS column)
        const SlabRay sr = slab_ray(ray);
        const SphRay sp = sph_ray(ray);
        Prune pr = prune_off();
        best_t = INFINITY;
        best_s = -1;
        WideWalk w = wide_walk_start(sc, active && !gen);
        while (__ballot(wide_walking(w))) {
            if (!wide_walking(w)) continue;
            wide_lane_step<FAST, COUNT>(sc, sr, sp, pr, w, wstk, best_t, best_s, cnt);
        }
    } else {
        closest_bvh<UNIFORM, FAST, COUNT>(sc, ray, active && !gen, best_t, best_s, cnt);
    }
    uint64_t gm = __ballot(gen);
    const int lane = threadIdx.x & 63;
    while (gm) {
        const int l = __builtin_ctzll(gm);
        gm &= gm - 1;
        const Ray rr{readlane_f(ray.ox, l), readlane_f(ray.oy, l), readlane_f(ray.oz, l),
                     readlane_f(ray.dx, l), readlane_f(ray.dy, l), readlane_f(ray.dz, l)};
        float t;
        int s;
        Counters c2{0, 0, 0, 0, 0};
        closest_bvh_chunked<FAST, COUNT>(sc, rr, t, s, c2);
        if (COUNT) cnt.steps += c2.steps;
        if (lane == l) {
            best_t = t;
            best_s = s;
            if (COUNT) {
                cnt.nodes += c2.nodes;
                cnt.spheres += c2.spheres;
            }
        }
    }
}

// Spheres [s0, s1) against this lane's ray, in array order (the first of
// equal t wins: renderer.c:39's strict `<`), into best_t / best_s.
__device__ __forceinline__ void brute_range_packed(const DevScene& sc, const SphRay& sp, bool active, int s0, int s1,
                                                   float& best_t, int& best_s)
{
    constexpr bool FAST = true;
    // eight spheres per iteration, two per instruction (packed fp32:
    // v_pk_mul/v_pk_add, the same IEEE roundings as hit.c:22-26's scalar
    // expressions, no contraction): the discriminants decide nearly every
    // pair at once, and only a batch with some disc > 0 walks its spheres
    // through sphere_t (which recomputes that disc) in array order
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 ox = sp.ox, oy = sp.oy, oz = sp.oz, dx = sp.dx, dy = sp.dy, dz = sp.dz;
    const f2 a4 = sp.a4();
    auto disc2 = [&](const float4& p, const float4& q) {
        const f2 ocx = ox - f2{p.x, q.x}, ocy = oy - f2{p.y, q.y}, ocz = oz - f2{p.z, q.z};
        const f2 r = f2{p.w, q.w};
        const f2 b = 2.0f * ((ocx * dx + ocy * dy) + ocz * dz);
        const f2 c = ((ocx * ocx + ocy * ocy) + ocz * ocz) - r * r;
        return b * b - a4 * c;
    };
    int k = s0;
    // one base pointer per batch, constant offsets: two s_load_dwordx16;
    // the next batch is requested before this one is tested
    auto batch = [&](int k0, float4* g) {
        const cf32_t* p = (const cf32_t*)sc.geo + 4 * k0;
#pragma unroll
        for (int j = 0; j < 8; j++) g[j] = make_float4(p[4 * j], p[4 * j + 1], p[4 * j + 2], p[4 * j + 3]);
    };
    float4 g[8], gn[8];
    if (k + 8 <= s1) batch(k, g);
    for (; k + 8 <= s1; k += 8) {
        if (k + 16 <= s1) batch(k + 8, gn);
        if (active) {
            const f2 d0 = disc2(g[0], g[1]), d1 = disc2(g[2], g[3]), d2 = disc2(g[4], g[5]), d3 = disc2(g[6], g[7]);
            const f2 m01 = __builtin_elementwise_max(d0, d1), m23 = __builtin_elementwise_max(d2, d3);
            const f2 m = __builtin_elementwise_max(m01, m23);
            // NaN discs (the padding sentinel never enters here) compare false either way
            if (m.x > 0.0f || m.y > 0.0f || !(m.x == m.x) || !(m.y == m.y)) {
#pragma unroll
                for (int j = 0; j < 8; j++) {
                    const float t = sphere_t<FAST>(sp, g[j], best_t);
                    if (t > 0.0f && t < best_t) {
                        best_t = t;
                        best_s = k + j;
                    }
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 8; j++) g[j] = gn[j];
    }
    for (; k < s1; k++) {
        const float4 g = load_geo_uniform(sc.geo, k);
        if (active) {
            const float t = sphere_t<FAST>(sp, g, best_t);
            if (t > 0.0f && t < best_t) {
                best_t = t;
                best_s = k;
            }
        }
    }
}

// renderer.c:36-43: every sphere in array order, the first wins a tie (so
// the estimate may discard t >= best, not just t > best).
template <bool FAST, bool COUNT>
__device__ __forceinline__ void closest_brute(const DevScene& sc, const Ray& ray, bool active, float& best_t,
                                              int& best_s, Counters& cnt)
{
    const SphRay sp = sph_ray(ray);
    best_t = INFINITY;
    best_s = -1;
    if (!__ballot(active) || sc.num_spheres == 0) return;
    if (FAST && !COUNT) {
        brute_range_packed(sc, sp, active, 0, sc.num_spheres, best_t, best_s);
        return;
    }
    float4 g = load_geo_uniform(sc.geo, 0);
    for (int i = 0; i < sc.num_spheres; i++) {
        const float4 gn = load_geo_uniform(sc.geo, i + 1);  // [num_spheres] is the sentinel: in bounds
        if (active) {
            if (COUNT) cnt.spheres++;
            const float t = sphere_t<FAST>(sp, g, best_t);
            if (t > 0.0f && t < best_t) {
                best_t = t;
                best_s = i;
            }
        }
        g = gn;
    }
}

// hit.c:32-33 for the winning sphere: point = o + d t, normal = |point - c|.
__device__ __forceinline__ void hit_point_normal(const Ray& r, float t, float4 s, float* p, float* n)
{
    p[0] = r.ox + r.dx * t;
    p[1] = r.oy + r.dy * t;
    p[2] = r.oz + r.dz * t;
    n[0] = p[0] - s.x;
    n[1] = p[1] - s.y;
    n[2] = p[2] - s.z;
    normalize3(n[0], n[1], n[2]);
}

// sphere.c:19-32 with vec3.c:64-69 on the per-pixel stream: rejection-sample
// p in the unit ball (x, y, z drawn in that order), normalise, flip into the
// hemisphere of n.
__device__ __forceinline__ void hemisphere(uint64_t key, uint32_t& k, const float* n, float& x, float& y,
                                           float& z)
{
    // The reference loops until a draw is accepted (acceptance pi/6 per try);
    // the cap only guarantees every wave terminates.
    for (int tries = 0; tries < 4096; tries++) {
        x = -1.0f + ((float)draw(key, k++) / 2147483648.0f) * 2.0f;
        y = -1.0f + ((float)draw(key, k++) / 2147483648.0f) * 2.0f;
        z = -1.0f + ((float)draw(key, k++) / 2147483648.0f) * 2.0f;
        const float l2 = dot3(x, y, z, x, y, z);
        if (l2 < 1.0f && l2 != 0.0f) break;
    }
    normalize3(x, y, z);
    if (!(dot3(x, y, z, n[0], n[1], n[2]) > 0.0f)) {
        x = x * -1.0f;
        y = y * -1.0f;
        z = z * -1.0f;
    }
}

// renderer.c:65-70 sky gradient (float, truncated to Uint8).
__device__ __forceinline__ uint32_t sky_rgba(float dy)
{
    const float t = 0.5f * (dy + 1.0f);
    const float omt = 1.0f - t;
    const float r = omt * 255.0f + t * 128.0f;
    const float g = omt * 255.0f + t * 178.0f;
    return (uint32_t)((int)r & 0xff) | ((uint32_t)((int)g & 0xff) << 8) | (255u << 16) | (255u << 24);
}

// renderer.c:56-58: (Uint8)(base + 0.5 * refl) computed in double and
// truncated through int32 (x86 keeps the low byte). base and
// refl are integers <= 255, so base + 0.5 refl is exact and its truncation
// is (2 base + refl) >> 1.
__device__ __forceinline__ uint32_t blend_rgba(uint32_t base, uint32_t refl)
{
    uint32_t out = 255u << 24;
    for (int c = 0; c < 3; c++) {
        const uint32_t b = (base >> (8 * c)) & 0xff, f = (refl >> (8 * c)) & 0xff;
        out |= (((2u * b + f) >> 1) & 0xffu) << (8 * c);
    }
    return out;
}

// Frame schedules (mirt_set_option MIRT_OPT_TRAVERSAL). TILE: one kernel,
// each wave traces the whole paths of an 8x8 tile (trace_path: camera rays
// as a packet, bounces per lane). WAVEFRONT (default, depth >= 2): camera
// rays as packets, then persistent per-lane bounce chains fed by a queue
// (render.hip primary_kernel / bounce_kernel).
// (ids as in include/mirt.h: 5 is the round-1 value of WAVEFRONT, kept so
// that the retired ids 1-4 are rejected rather than silently remapped)
enum Trav { kTravTile = 0, kTravWavefront = 5 };

// trace_ray (renderer.c:21-77) with the recursion turned into a loop over
// bounce levels that the whole wave executes together (the traversal needs
// convergent lanes). Returns packed RGBA8. `key` is the pixel's RNG stream.
// The base colours of the hit levels (folded innermost-first at the end,
// renderer.c:55-58) live in LDS, `cstack[level * cstride]`, one column per
// thread, to keep them out of the register budget.
template <bool FAST, bool COUNT>
__device__ __forceinline__ uint32_t trace_path(const DevScene& sc, Ray ray, bool alive, int depth, bool use_bvh,
                                               uint64_t key, Counters& cnt, uint32_t* cstack, int cstride,
                                               uint32_t* wstk = nullptr)
{
    int levels = 0;
    uint32_t tail = 255u << 24;  // renderer.c:23-24 depth exhausted -> (0,0,0,255)
    uint32_t k = 0;
    for (int level = 0; level < depth; level++) {
        if (!__ballot(alive)) break;
        float t;
        int s;
        if (use_bvh) {
            // primary rays of an 8x8 tile are coherent: walk them as one
            // packet; bounce rays scatter: each lane walks alone
            if (level == 0)
                closest_hit<true, FAST, COUNT>(sc, ray, alive, t, s, cnt);
            else
                closest_hit<false, FAST, COUNT>(sc, ray, alive, t, s, cnt, wstk);
        } else {
            closest_brute<FAST, COUNT>(sc, ray, alive, t, s, cnt);
        }
        if (alive) {
            if (COUNT) cnt.rays++;
            if (s < 0) {
                tail = sky_rgba(ray.dy);
                alive = false;
            } else {
                if (COUNT) cnt.hits++;
                cstack[levels * cstride] = sc.color[s];
                levels++;
                if (level + 1 < depth) {
                    // the bounce of renderer.c:51-55; at the last level it would
                    // be traced with depth 0 and return black, so it is skipped
                    const float4 g = sc.geo[s];
                    float p[3], n[3];
                    hit_point_normal(ray, t, g, p, n);
                    float bx, by, bz;
                    hemisphere(key, k, n, bx, by, bz);
                    ray = {p[0], p[1], p[2], bx, by, bz};
                } else {
                    alive = false;
                }
            }
        }
        if (COUNT && level == 0) {
            cnt.nodes0 = cnt.nodes;
            cnt.spheres0 = cnt.spheres;
            cnt.hits0 = cnt.hits;
        }
    }
    for (int l = levels - 1; l >= 0; l--) tail = blend_rgba(cstack[l * cstride], tail);
    return tail;
}

}  // namespace mirt
