// Device side of the render path: exact-semantics restatements of the
// reference's per-ray functions, written for wave64 / gfx950.
//
// Floating point follows the reference operation by operation (the .hip is
// compiled with -ffp-contract=off; divisions and square roots are the IEEE
// correctly rounded HIP defaults; the double-precision segments of
// hit.c:28 and vec3.c:22 are computed in double). Anything else would move
// the framebuffer away from the reference's bytes.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/mirt.h"
#include "rng.h"

namespace mirt {

constexpr float kEps = 0.000001f;  // constants.h:6
constexpr int kMaxDepth = 8;       // bounce levels kept in registers

// Read-only scene in HBM. Loads whose index is wave-uniform go through the
// constant address space so they become scalar (s_load) loads.
struct DevScene {
    const mirt_node* nodes;
    const float4* geo;      // centre.xyz, radius; [num_spheres] = NaN sentinel (never hits)
    const uint32_t* color;  // packed RGBA8
    uint32_t num_nodes;
    int num_spheres;
};

struct Ray {
    float ox, oy, oz, dx, dy, dz;
};

struct Counters {
    uint32_t rays, nodes, spheres, hits;
};

typedef const __attribute__((address_space(4))) uint32_t cu32_t;
typedef const __attribute__((address_space(4))) float cf32_t;

// Wave-uniform index -> read through the constant address space, which the
// backend lowers to scalar loads (s_load_dwordx8 for a node, x4 for a sphere).
__device__ __forceinline__ mirt_node load_node_uniform(const mirt_node* base, uint32_t i)
{
    const cu32_t* p = (const cu32_t*)base + 8u * i;
    mirt_node n;
    n.bmin[0] = __uint_as_float(p[0]);
    n.bmin[1] = __uint_as_float(p[1]);
    n.bmin[2] = __uint_as_float(p[2]);
    n.bmax[0] = __uint_as_float(p[3]);
    n.bmax[1] = __uint_as_float(p[4]);
    n.bmax[2] = __uint_as_float(p[5]);
    n.sphere = (int32_t)p[6];
    n.skip = p[7];
    return n;
}
__device__ __forceinline__ float4 load_geo_uniform(const float4* base, int i)
{
    const cf32_t* p = (const cf32_t*)base + 4 * i;
    return make_float4(p[0], p[1], p[2], p[3]);
}

// Divergent index -> two 16-B vector loads per node.
__device__ __forceinline__ mirt_node load_node_lane(const mirt_node* base, uint32_t i)
{
    const float4* p = (const float4*)(base + i);
    const float4 a = p[0], b = p[1];
    mirt_node n;
    n.bmin[0] = a.x;
    n.bmin[1] = a.y;
    n.bmin[2] = a.z;
    n.bmax[0] = a.w;
    n.bmax[1] = b.x;
    n.bmax[2] = b.y;
    n.sphere = __float_as_int(b.z);
    n.skip = __float_as_uint(b.w);
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
// branch does not depend on the box.
struct SlabRay {
    float ox, oy, oz, dx, dy, dz;
    bool zx, zy, zz;
};

__device__ __forceinline__ SlabRay slab_ray(const Ray& r)
{
    return {r.ox, r.oy, r.oz, r.dx, r.dy, r.dz, r.dx == 0.0f, r.dy == 0.0f, r.dz == 0.0f};
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

// Per-ray constants of ray_sphere_intersect: a = d.d, 4a and 2a (hit.c:22-28).
struct SphRay {
    float ox, oy, oz, dx, dy, dz;
    float a4;     // 4 * a  (hit.c:25: 4 * a * c evaluates (4 * a) * c)
    double a2;    // (double)(2.0f * a)
};

__device__ __forceinline__ SphRay sph_ray(const Ray& r)
{
    const float a = dot3(r.dx, r.dy, r.dz, r.dx, r.dy, r.dz);
    return {r.ox, r.oy, r.oz, r.dx, r.dy, r.dz, 4.0f * a, (double)(2.0f * a)};
}

// hit.c:19-39 without the point/normal (computed once for the winner).
// Returns t > EPS on a hit, else -1.
__device__ __forceinline__ float sphere_t(const SphRay& r, float4 s)
{
    const float ocx = r.ox - s.x, ocy = r.oy - s.y, ocz = r.oz - s.z;
    const float b = 2.0f * dot3(ocx, ocy, ocz, r.dx, r.dy, r.dz);
    const float c = dot3(ocx, ocy, ocz, ocx, ocy, ocz) - s.w * s.w;
    const float disc = b * b - r.a4 * c;
    if (disc > 0.0f) {
        // hit.c:28 in double: (-b - sqrt(disc)) / (2a), rounded to float
        const double num = (double)(-b) - __dsqrt_rn((double)disc);
        const float t = (float)__ddiv_rn(num, r.a2);
        if (t > kEps) return t;
    }
    return -1.0f;
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
// node / sphere load is a scalar load.
// Otherwise (LANE): every lane walks its own sequence with vector loads.
template <bool UNIFORM, bool COUNT>
__device__ __forceinline__ void closest_bvh(const DevScene& sc, const Ray& ray, bool active, float& best_t,
                                            int& best_s, Counters& cnt)
{
    const SlabRay sr = slab_ray(ray);
    const SphRay sp = sph_ray(ray);
    const uint32_t end = sc.num_nodes;
    uint32_t next = active ? 0u : end;
    best_t = INFINITY;
    best_s = -1;
    if constexpr (UNIFORM) {
        uint32_t cur = __builtin_amdgcn_readfirstlane(__ballot(active) ? 0u : end);
        while (cur < end) {
            const mirt_node nd = load_node_uniform(sc.nodes, cur);
            const uint32_t skip = nd.skip & MIRT_SKIP_MASK;
            bool descend = false;
            if (next == cur) {
                const bool pass = (nd.skip & MIRT_NODE_EMPTY) ||
                                  slab_test(sr, nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2]);
                if (COUNT) cnt.nodes++;
                if (pass && nd.sphere < 0) {
                    next = cur + 1;
                    descend = true;
                } else {
                    next = skip;
                    if (pass) {
                        if (COUNT) cnt.spheres++;
                        const float t = sphere_t(sp, load_geo_uniform(sc.geo, nd.sphere));
                        if (t > 0.0f && t <= best_t) {
                            best_t = t;
                            best_s = nd.sphere;
                        }
                    }
                }
            }
            cur = __builtin_amdgcn_readfirstlane(__ballot(descend) ? cur + 1 : skip);
        }
    } else {
        while (__ballot(next < end)) {
            if (next < end) {
                const mirt_node nd = load_node_lane(sc.nodes, next);
                const bool pass = (nd.skip & MIRT_NODE_EMPTY) ||
                                  slab_test(sr, nd.bmin[0], nd.bmin[1], nd.bmin[2], nd.bmax[0], nd.bmax[1], nd.bmax[2]);
                if (COUNT) cnt.nodes++;
                if (pass && nd.sphere < 0) {
                    next = next + 1;
                } else {
                    next = nd.skip & MIRT_SKIP_MASK;
                    if (pass) {
                        if (COUNT) cnt.spheres++;
                        const float t = sphere_t(sp, sc.geo[nd.sphere]);
                        if (t > 0.0f && t <= best_t) {
                            best_t = t;
                            best_s = nd.sphere;
                        }
                    }
                }
            }
        }
    }
}

// renderer.c:36-43: every sphere in array order, the first wins a tie.
template <bool COUNT>
__device__ __forceinline__ void closest_brute(const DevScene& sc, const Ray& ray, bool active, float& best_t,
                                              int& best_s, Counters& cnt)
{
    const SphRay sp = sph_ray(ray);
    best_t = INFINITY;
    best_s = -1;
    if (!__ballot(active)) return;
    for (int i = 0; i < sc.num_spheres; i++) {
        const float4 g = load_geo_uniform(sc.geo, i);
        if (active) {
            if (COUNT) cnt.spheres++;
            const float t = sphere_t(sp, g);
            if (t > 0.0f && t < best_t) {
                best_t = t;
                best_s = i;
            }
        }
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

// trace_ray (renderer.c:21-77) with the recursion turned into a loop over
// bounce levels that the whole wave executes together (the traversal needs
// convergent lanes). Returns packed RGBA8. `key` is the pixel's RNG stream.
template <bool UNIFORM, bool COUNT>
__device__ __forceinline__ uint32_t trace_path(const DevScene& sc, Ray ray, bool alive, int depth, bool use_bvh,
                                               uint64_t key, Counters& cnt)
{
    uint32_t base[kMaxDepth];
    int levels = 0;
    uint32_t tail = 255u << 24;  // renderer.c:23-24 depth exhausted -> (0,0,0,255)
    uint32_t k = 0;
    for (int level = 0; level < depth; level++) {
        if (!__ballot(alive)) break;
        float t;
        int s;
        if (use_bvh)
            closest_bvh<UNIFORM, COUNT>(sc, ray, alive, t, s, cnt);
        else
            closest_brute<COUNT>(sc, ray, alive, t, s, cnt);
        if (alive) {
            if (COUNT) cnt.rays++;
            if (s < 0) {
                tail = sky_rgba(ray.dy);
                alive = false;
            } else {
                if (COUNT) cnt.hits++;
#pragma unroll
                for (int l = 0; l < kMaxDepth; l++)
                    if (l == levels) base[l] = sc.color[s];
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
    }
#pragma unroll
    for (int l = kMaxDepth - 1; l >= 0; l--)
        if (l < levels) tail = blend_rgba(base[l], tail);
    return tail;
}

}  // namespace mirt
