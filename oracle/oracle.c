/*
 * oracle/oracle.c -- TEST INFRASTRUCTURE ONLY: CPU restatement of the
 * reference's primary-ray render path, used as the parity checker.
 *
 *   Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 *   load this library. The product (cs201_sah-bvh_ray_tracer_amd/) never links
 *   or calls it.
 *
 * It restates, function by function, the reference algorithm under
 * /root/reference (file:line cited at each function), written independently
 * (no reference source is copied). It is pinned against the reference itself:
 * tests/golden/ holds vectors produced by the unmodified reference sources
 * compiled by oracle/Makefile into oracle/_ref/ (tests/golden/make_golden.py),
 * and tests/test_oracle_golden.py checks this file against every one of them.
 *
 * Floating point: compiled with -O2 -ffp-contract=off and no -march (SURVEY.md
 * §8.H1: FMA contraction changes the BVH). Float/double promotion is written
 * out explicitly wherever the reference mixes them (hit.c:28, ray.c:19-20,
 * renderer.c:56-58, vec3.c:22).
 *
 * Random numbers: mode 0 draws from glibc's serial rand() exactly like the
 * reference (single-threaded; bit-exact vs the unmodified reference at
 * depth 1, where draws are consumed but never used, renderer.c:51-55 with
 * renderer.c:23-24). Mode 1 uses the per-pixel counter contract of
 * oracle/rng_contract.h so rows can run on many threads.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#include "../include/mirt.h"
#include "rng_contract.h"

#define O_EPS 0.000001f /* constants.h:6 */

/* ------------------------------------------------------------------ RNG */

static int o_mode;                   /* 0: glibc stream, 1: per-pixel contract */
static __thread uint64_t o_key;      /* contract key of the pixel being traced */
static __thread uint32_t o_draws;    /* rand() calls made for that pixel so far */

static int o_rand(void)
{
    if (o_mode == 1) return oc_draw(o_key, o_draws++);
    return rand();
}

void o_srand(unsigned seed) { srand(seed); }
int o_libc_rand(void) { return rand(); }
int o_contract_draw(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t k)
{
    return oc_draw(oc_pixel_key(seed, pixel, sample), k);
}

/* ------------------------------------------------------------ vec math */

typedef mirt_vec3 V3;

static V3 v3(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
static V3 vsub(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }   /* vec3.c:17 */
static V3 vadd(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }   /* vec3.c:30 */
static V3 vscale(V3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }   /* vec3.c:34 */
static float vdot(V3 a, V3 b)                                                /* vec3.c:26 */
{
    float s = a.x * b.x;
    s = s + a.y * b.y;
    return s + a.z * b.z;
}
static V3 vnorm(V3 a)                                                        /* vec3.c:21-24 */
{
    float sq = vdot(a, a);
    float len = (float)sqrt((double)sq);
    if (len == 0.0f) return v3(0.0f, 0.0f, 0.0f);
    return v3(a.x / len, a.y / len, a.z / len);
}

/* sphere.c:14-16 random_float and vec3.c:64-69 vec3_random share one form */
static float o_unit_draw(float lo, float hi)
{
    float f = (float)o_rand() / (float)RAND_MAX;
    return lo + f * (hi - lo);
}

/* sphere.c:19-24 + sphere.c:26-32 */
static V3 o_hemisphere(V3 n)
{
    V3 p;
    for (;;) {
        float x = o_unit_draw(-1.0f, 1.0f);
        float y = o_unit_draw(-1.0f, 1.0f);
        float z = o_unit_draw(-1.0f, 1.0f);
        p = v3(x, y, z);
        float l2 = vdot(p, p);
        if (l2 < 1.0f && l2 != 0.0f) break;
    }
    p = vnorm(p);
    if ((double)vdot(p, n) > 0.0) return p;
    return vscale(p, -1.0f);
}

/* --------------------------------------------------------- scene inputs */

/* sphere.c:52-59, drawn in the order x, y, z, r, R, G, B */
void o_gen_render_scene(unsigned seed, int n, mirt_sphere *out)
{
    int saved = o_mode;
    o_mode = 0;
    srand(seed);
    for (int i = 0; i < n; i++) {
        mirt_sphere s;
        s.center.x = o_unit_draw(-40.0f, 40.0f);
        s.center.y = o_unit_draw(-20.0f, 20.0f);
        s.center.z = o_unit_draw(-10.0f, 5.0f);
        s.radius = o_unit_draw(0.5f, 5.0f);
        s.color.r = (uint8_t)(o_rand() % 256);
        s.color.g = (uint8_t)(o_rand() % 256);
        s.color.b = (uint8_t)(o_rand() % 256);
        s.color.a = 255;
        out[i] = s;
    }
    o_mode = saved;
}

/* benchmark.c:307-314 centre draws + sphere.c:34-41 create_benchmark_sphere */
void o_gen_bench_scene(unsigned seed, int n, float world, mirt_sphere *out)
{
    int saved = o_mode;
    o_mode = 0;
    srand(seed);
    for (int i = 0; i < n; i++) {
        mirt_sphere s;
        float half = world / 2;
        s.center.x = (float)rand() / (float)RAND_MAX * world - half;
        s.center.y = (float)rand() / (float)RAND_MAX * world - half;
        s.center.z = (float)rand() / (float)RAND_MAX * world - half;
        s.radius = 0.5f;
        s.color.r = (uint8_t)(rand() % 256);
        s.color.g = (uint8_t)(rand() % 256);
        s.color.b = (uint8_t)(rand() % 256);
        s.color.a = 255;
        out[i] = s;
    }
    o_mode = saved;
}

/* ------------------------------------------------------------ BVH build */

typedef struct ONode {
    mirt_aabb box;
    struct ONode *kid[2];
    int first;   /* index of node->sphere in the array (leaf), -1 inner */
    int count;   /* sphere_count */
} ONode;

static mirt_aabb box_empty(void)                                   /* bvh.c:19-24 */
{
    mirt_aabb b;
    b.min = v3(INFINITY, INFINITY, INFINITY);
    b.max = v3(-INFINITY, -INFINITY, -INFINITY);
    return b;
}
static void box_grow(mirt_aabb *b, const mirt_sphere *s)           /* bvh.c:26-46 */
{
    float r = s->radius;
    float lo[3] = {s->center.x - r, s->center.y - r, s->center.z - r};
    float hi[3] = {s->center.x + r, s->center.y + r, s->center.z + r};
    b->min.x = fminf(b->min.x, lo[0]);
    b->min.y = fminf(b->min.y, lo[1]);
    b->min.z = fminf(b->min.z, lo[2]);
    b->max.x = fmaxf(b->max.x, hi[0]);
    b->max.y = fmaxf(b->max.y, hi[1]);
    b->max.z = fmaxf(b->max.z, hi[2]);
}
static float box_area(const mirt_aabb *b)                          /* bvh.c:48-57 */
{
    float dx = b->max.x - b->min.x, dy = b->max.y - b->min.y, dz = b->max.z - b->min.z;
    float s = dx * dy;
    s = s + dy * dz;
    s = s + dz * dx;
    return 2.0f * s;
}
static float axis_of(const mirt_sphere *s, int axis)
{
    return axis == 0 ? s->center.x : (axis == 1 ? s->center.y : s->center.z);
}
static float box_lo(const mirt_aabb *b, int a) { return a == 0 ? b->min.x : (a == 1 ? b->min.y : b->min.z); }
static float box_hi(const mirt_aabb *b, int a) { return a == 0 ? b->max.x : (a == 1 ? b->max.y : b->max.z); }

/* bvh.c:59-97: one full pass per candidate plane, exactly as the reference */
static float sah_cost(const mirt_sphere *s, int lo, int hi, int axis, float plane)
{
    mirt_aabb L = box_empty(), R = box_empty();
    int nl = 0, nr = 0;
    for (int i = lo; i < hi; i++) {
        if (axis_of(&s[i], axis) < plane) { nl++; box_grow(&L, &s[i]); }
        else { nr++; box_grow(&R, &s[i]); }
    }
    float al = box_area(&L), ar = box_area(&R);
    float sum = (float)nl * al;
    sum = sum + (float)nr * ar;
    return 0.125f + sum;
}

/* bvh.c:117-209 */
static ONode *o_build_rec(mirt_sphere *s, int lo, int hi, int depth)
{
    ONode *nd = (ONode *)malloc(sizeof(ONode));
    nd->box = box_empty();
    for (int i = lo; i < hi; i++) box_grow(&nd->box, &s[i]);
    int n = hi - lo;
    if (n <= 1 || depth >= 40) {
        nd->kid[0] = nd->kid[1] = NULL;
        nd->first = lo;
        nd->count = n;
        return nd;
    }
    float best = INFINITY, best_plane = 0.0f;
    int best_axis = 0;
    for (int axis = 0; axis < 3; axis++) {
        float b0 = box_lo(&nd->box, axis), b1 = box_hi(&nd->box, axis);
        for (int k = 1; k < 8; k++) {
            float plane = b0 + ((float)k / 8.0f) * (b1 - b0);
            float c = sah_cost(s, lo, hi, axis, plane);
            if (c < best) { best = c; best_axis = axis; best_plane = plane; }
        }
    }
    int mid = lo;
    for (int i = lo; i < hi; i++) {
        if (axis_of(&s[i], best_axis) < best_plane) {
            mirt_sphere t = s[i]; s[i] = s[mid]; s[mid] = t;
            mid++;
        }
    }
    nd->kid[0] = o_build_rec(s, lo, mid, depth + 1);
    nd->kid[1] = o_build_rec(s, mid, hi, depth + 1);
    nd->first = -1;
    nd->count = 0;
    return nd;
}

void *o_build(mirt_sphere *s, int start, int end, int depth) { return o_build_rec(s, start, end, depth); }

void o_free(void *root)                                            /* benchmark.c:81-88 */
{
    ONode *nd = (ONode *)root;
    if (!nd) return;
    o_free(nd->kid[0]);
    o_free(nd->kid[1]);
    free(nd);
}

static int o_flatten_rec(const ONode *nd, mirt_node *out, int at)
{
    int me = at++;
    mirt_node *f = &out[me];
    f->bmin[0] = nd->box.min.x; f->bmin[1] = nd->box.min.y; f->bmin[2] = nd->box.min.z;
    f->bmax[0] = nd->box.max.x; f->bmax[1] = nd->box.max.y; f->bmax[2] = nd->box.max.z;
    if (nd->first >= 0) {
        f->sphere = nd->first;
    } else {
        f->sphere = -1;
        at = o_flatten_rec(nd->kid[0], out, at);
        at = o_flatten_rec(nd->kid[1], out, at);
    }
    f->skip = (uint32_t)at | (nd->first >= 0 && nd->count == 0 ? MIRT_NODE_EMPTY : 0u);
    return at;
}

static int o_count_nodes(const ONode *nd)
{
    return nd ? 1 + o_count_nodes(nd->kid[0]) + o_count_nodes(nd->kid[1]) : 0;
}

int o_node_count(void *root) { return o_count_nodes((const ONode *)root); }

/* pre-order with left = i+1 and a skip (escape) index; mirt.h documents it */
int o_flatten(void *root, mirt_node *out, int cap)
{
    int n = o_count_nodes((const ONode *)root);
    if (n > cap) return -n;
    return o_flatten_rec((const ONode *)root, out, 0);
}

/* ---------------------------------------------------------- intersect */

typedef struct { float t; V3 p, n; int hit; int sphere; } OHit;

/* hit.c:19-39 */
static OHit o_sphere_hit(const mirt_ray *r, const mirt_sphere *sp, int idx)
{
    OHit h;
    memset(&h, 0, sizeof h);
    h.sphere = -1;
    V3 oc = vsub(r->origin, sp->center);
    float a = vdot(r->direction, r->direction);
    float b = 2.0f * vdot(oc, r->direction);
    float c = vdot(oc, oc) - sp->radius * sp->radius;
    float disc = b * b - (4.0f * a) * c;
    if (disc > 0.0f) {
        double num = (double)(-b) - sqrt((double)disc);
        float t = (float)(num / (double)(2.0f * a));
        if (t > O_EPS) {
            h.hit = 1;
            h.t = t;
            h.p = vadd(r->origin, vscale(r->direction, t));
            h.n = vnorm(vsub(h.p, sp->center));
            h.sphere = idx;
        }
    }
    return h;
}

/* hit.c:49-82 */
static int o_slab(const mirt_ray *r, const mirt_aabb *b)
{
    const float o[3] = {r->origin.x, r->origin.y, r->origin.z};
    const float d[3] = {r->direction.x, r->direction.y, r->direction.z};
    const float lo[3] = {b->min.x, b->min.y, b->min.z};
    const float hi[3] = {b->max.x, b->max.y, b->max.z};
    float near_[3], far_[3];
    for (int a = 0; a < 3; a++) {
        float t1, t2;
        if (d[a] == 0.0f) { t1 = -INFINITY; t2 = INFINITY; }
        else { t1 = (lo[a] - o[a]) / d[a]; t2 = (hi[a] - o[a]) / d[a]; }
        near_[a] = fminf(t1, t2);
        far_[a] = fmaxf(t1, t2);
    }
    float tmin = fmaxf(near_[0], fmaxf(near_[1], near_[2]));
    float tmax = fminf(far_[0], fminf(far_[1], far_[2]));
    return tmax >= tmin && tmax > O_EPS;
}

typedef struct { long long nodes, spheres; } OCount;

/* hit.c:91-109: recursive DFS; ties resolve to the right subtree */
static OHit o_bvh_hit(const mirt_ray *r, const ONode *nd, const mirt_sphere *s, int ns, OCount *cnt)
{
    OHit none;
    memset(&none, 0, sizeof none);
    none.sphere = -1;
    if (cnt) cnt->nodes++;
    if (!o_slab(r, &nd->box)) return none;
    if (nd->first >= 0) {
        if (cnt) cnt->spheres++;
        if (nd->first >= ns) return none; /* &spheres[N]: never-hit sentinel */
        return o_sphere_hit(r, &s[nd->first], nd->first);
    }
    OHit L = o_bvh_hit(r, nd->kid[0], s, ns, cnt);
    OHit R = o_bvh_hit(r, nd->kid[1], s, ns, cnt);
    if (!L.hit) return R;
    if (!R.hit) return L;
    return L.t < R.t ? L : R;
}

/* hit.c:91-109 over a FLAT pre-order tree (include/mirt.h mirt_node: left
   child i + 1, right child = the left subtree's skip): the same recursion,
   for trees too large for this file's own build (the 10M / 100M benchmark
   sweep points, whose trees are pinned by their SHA tests) */
static OHit o_flat_hit(const mirt_ray *r, const mirt_node *nd, uint32_t i, const mirt_sphere *s, int ns)
{
    OHit none;
    memset(&none, 0, sizeof none);
    none.sphere = -1;
    mirt_aabb box;
    memcpy(&box.min, nd[i].bmin, sizeof box.min);
    memcpy(&box.max, nd[i].bmax, sizeof box.max);
    if (!o_slab(r, &box)) return none;
    if (nd[i].sphere >= 0) {
        if (nd[i].sphere >= ns) return none;
        return o_sphere_hit(r, &s[nd[i].sphere], nd[i].sphere);
    }
    OHit L = o_flat_hit(r, nd, i + 1, s, ns);
    OHit R = o_flat_hit(r, nd, nd[i + 1].skip & MIRT_SKIP_MASK, s, ns);
    if (!L.hit) return R;
    if (!R.hit) return L;
    return L.t < R.t ? L : R;
}

/* renderer.c:36-43: brute force, first sphere wins ties */
static OHit o_brute_hit(const mirt_ray *r, const mirt_sphere *s, int ns)
{
    OHit best;
    memset(&best, 0, sizeof best);
    best.t = INFINITY;
    best.sphere = -1;
    for (int i = 0; i < ns; i++) {
        OHit h = o_sphere_hit(r, &s[i], i);
        if (h.hit && h.t < best.t) best = h;
    }
    return best;
}

static void o_store_hit(const OHit *h, mirt_hit *out)
{
    out->t = h->t;
    out->point = h->p;
    out->normal = h->n;
    out->hit = h->hit;
    out->sphere = h->hit ? h->sphere : -1;
    out->pad = 0;
}

void o_intersect(void *root, const mirt_sphere *s, int ns, const mirt_ray *rays, int n, int use_bvh,
                 mirt_hit *out)
{
    for (int i = 0; i < n; i++) {
        OHit h = use_bvh ? o_bvh_hit(&rays[i], (const ONode *)root, s, ns, NULL) : o_brute_hit(&rays[i], s, ns);
        if (!use_bvh && !h.hit) h.t = 0.0f; /* report like a fresh HitRecord */
        o_store_hit(&h, &out[i]);
    }
}

void o_intersect_flat(const mirt_node *nodes, int nn, const mirt_sphere *s, int ns, const mirt_ray *rays, int n,
                      mirt_hit *out)
{
    for (int i = 0; i < n; i++) {
        OHit h;
        if (nn > 0) {
            h = o_flat_hit(&rays[i], nodes, 0, s, ns);
        } else {
            memset(&h, 0, sizeof h);
            h.sphere = -1;
        }
        o_store_hit(&h, &out[i]);
    }
}

void o_sphere_pairs(const mirt_ray *rays, const mirt_sphere *s, int n, mirt_hit *out)
{
    for (int i = 0; i < n; i++) {
        OHit h = o_sphere_hit(&rays[i], &s[i], i);
        o_store_hit(&h, &out[i]);
    }
}

void o_aabb_pairs(const mirt_ray *rays, const mirt_aabb *b, int n, int32_t *out)
{
    for (int i = 0; i < n; i++) out[i] = o_slab(&rays[i], &b[i]);
}

/* ------------------------------------------------------------- shading */

/* renderer.c:21-77, recursion unrolled into a loop over bounce levels */
static mirt_rgba8 o_trace(mirt_ray ray, const mirt_sphere *s, int ns, int depth, const ONode *root,
                          OCount *cnt, long long *rays_traced)
{
    uint8_t base[3 * 64];
    int levels = 0;
    mirt_rgba8 tail;
    tail.r = tail.g = tail.b = 0;
    tail.a = 255;
    for (int d = depth; d > 0; d--) {
        if (rays_traced) (*rays_traced)++;
        OHit h = root ? o_bvh_hit(&ray, root, s, ns, cnt) : o_brute_hit(&ray, s, ns);
        if (!h.hit) {
            float t = 0.5f * (ray.direction.y + 1.0f);
            float omt = 1.0f - t;
            float r = omt * 255.0f + t * 128.0f;
            float g = omt * 255.0f + t * 178.0f;
            tail.r = (uint8_t)(int)r;
            tail.g = (uint8_t)(int)g;
            tail.b = 255;
            break;
        }
        const mirt_rgba8 c = s[h.sphere].color;
        base[3 * levels + 0] = c.r;
        base[3 * levels + 1] = c.g;
        base[3 * levels + 2] = c.b;
        levels++;
        V3 dir = o_hemisphere(h.n);   /* drawn even when the bounce is never traced */
        ray.origin = h.p;
        ray.direction = dir;
    }
    /* renderer.c:56-58: (Uint8)(base + 0.5*refl) in double; x86 cvttsd2si keeps
       the low byte, so values above 255 wrap */
    for (int l = levels - 1; l >= 0; l--) {
        double r = (double)base[3 * l + 0] + 0.5 * (double)tail.r;
        double g = (double)base[3 * l + 1] + 0.5 * (double)tail.g;
        double b = (double)base[3 * l + 2] + 0.5 * (double)tail.b;
        tail.r = (uint8_t)(int32_t)r;
        tail.g = (uint8_t)(int32_t)g;
        tail.b = (uint8_t)(int32_t)b;
        tail.a = 255;
    }
    return tail;
}

/* ray.c:17-32; ray.c:18 uses the compile-time WIDTH/HEIGHT, here runtime */
static mirt_ray o_camera_ray(const mirt_camera *cam, int W, int H, float u, float v)
{
    float aspect = (float)W / (float)H;
    float fov_rad = (float)((double)cam->fov * (M_PI / 180.0));
    float half_h = (float)tan((double)(fov_rad / 2.0f));
    float half_w = aspect * half_h;
    V3 horiz = vscale(cam->right, 2.0f * half_w);
    V3 vert = vscale(cam->up, 2.0f * half_h);
    V3 d = vadd(cam->forward, vscale(horiz, u));
    d = vadd(d, vscale(vert, v));
    mirt_ray r;
    r.origin = cam->position;
    r.direction = vnorm(d);
    return r;
}

void o_camera_ray_px(const mirt_camera *cam, int W, int H, int x, int y, mirt_ray *out)
{
    float aspect = (float)W / (float)H;                    /* main.c:356 */
    float u = ((float)x / (float)W - 0.5f) * aspect;       /* main.c:362 */
    float v = (float)y / (float)H - 0.5f;                  /* main.c:363 */
    *out = o_camera_ray(cam, W, H, u, -v);                 /* main.c:365 */
}

/* main.c:362-365 with the build's jitter (rng_contract.h OC_JITTER_*): the
   sample point (x + jx, y + jy) of the pixel's contract stream */
static void o_camera_ray_jittered(const mirt_camera *cam, int W, int H, int x, int y, uint64_t key, mirt_ray *out)
{
    float aspect = (float)W / (float)H;
    float xf = (float)x + (float)oc_draw(key, OC_JITTER_X) / 2147483648.0f;
    float yf = (float)y + (float)oc_draw(key, OC_JITTER_Y) / 2147483648.0f;
    float u = (xf / (float)W - 0.5f) * aspect;
    float v = yf / (float)H - 0.5f;
    *out = o_camera_ray(cam, W, H, u, -v);
}

/* main.c:358-374 (fresh frame) over a list of rows. mode 0 must run with one
   thread (serial glibc stream in pixel order); mode 1 is thread-count
   independent; jitter (mode 1 only) moves each camera ray's sample point.
   counts (nullable) receives {rays traced, node tests, sphere tests}. */
void o_render_rows(const mirt_camera *cam, int W, int H, const mirt_sphere *s, int ns, void *root,
                   int depth, int use_bvh, int mode, uint64_t seed, uint32_t sample,
                   const int *rows, int nrows, mirt_rgba8 *out, int nthreads, long long *counts, int jitter)
{
    o_mode = mode;
    long long c_rays = 0, c_nodes = 0, c_sph = 0;
#ifdef _OPENMP
    if (mode == 0 || nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : c_rays, c_nodes, c_sph)
#endif
    for (int ri = 0; ri < nrows; ri++) {
        int y = rows[ri];
        OCount cnt = {0, 0};
        long long nr = 0;
        for (int x = 0; x < W; x++) {
            mirt_ray r;
            if (mode == 1) { o_key = oc_pixel_key(seed, (uint32_t)(y * W + x), sample); o_draws = 0; }
            if (mode == 1 && jitter)
                o_camera_ray_jittered(cam, W, H, x, y, o_key, &r);
            else
                o_camera_ray_px(cam, W, H, x, y, &r);
            out[(size_t)ri * W + x] = o_trace(r, s, ns, depth, use_bvh ? (const ONode *)root : NULL,
                                              counts ? &cnt : NULL, counts ? &nr : NULL);
        }
        c_rays += nr;
        c_nodes += cnt.nodes;
        c_sph += cnt.spheres;
    }
    if (counts) { counts[0] = c_rays; counts[1] = c_nodes; counts[2] = c_sph; }
    o_mode = 0;
}

/* trace_ray over arbitrary rays; ray i uses contract pixel index i (mode 1) */
void o_trace_rays(const mirt_ray *rays, int n, const mirt_sphere *s, int ns, void *root, int depth,
                  int use_bvh, int mode, uint64_t seed, uint32_t sample, mirt_rgba8 *out)
{
    o_mode = mode;
    for (int i = 0; i < n; i++) {
        if (mode == 1) { o_key = oc_pixel_key(seed, (uint32_t)i, sample); o_draws = 0; }
        out[i] = o_trace(rays[i], s, ns, depth, use_bvh ? (const ONode *)root : NULL, NULL, NULL);
    }
    o_mode = 0;
}

/* main.c:368-370 (fresh) and main.c:394-401 (accumulate) on a row-major
   float3 buffer; returns the displayed colour. */
void o_accumulate(const mirt_rgba8 *color, int n, float *acc, int fresh, int frames, mirt_rgba8 *shown)
{
    for (int i = 0; i < n; i++) {
        float c[3] = {(float)color[i].r / 255.0f, (float)color[i].g / 255.0f, (float)color[i].b / 255.0f};
        if (fresh) {
            for (int k = 0; k < 3; k++) acc[3 * i + k] = c[k];
            shown[i] = color[i];
        } else {
            uint8_t o[3];
            for (int k = 0; k < 3; k++) {
                acc[3 * i + k] = acc[3 * i + k] + c[k];
                float v = acc[3 * i + k] / (float)frames * 255.0f;
                o[k] = (uint8_t)(int32_t)fmin((double)v, 255.0);
            }
            shown[i].r = o[0]; shown[i].g = o[1]; shown[i].b = o[2]; shown[i].a = 255;
        }
    }
}

/* ------------------------------------------------------- BVH debug overlay */
/* bvh_visualiser.c:16-126 restated on a W x H RGBA8 canvas cleared to
   (0, 0, 0, 255) (main.c:342-343): draw_bvh_recursive's pre-order, draw_aabb's
   12 edges, draw_debug_line's 5 offset lines, each a Bresenham line between
   the integer endpoints (both inclusive, off-screen pixels skipped -- the
   build's definition of SDL_RenderDrawLine), later lines overwriting
   earlier ones. Nodes at depth >= max_levels are skipped (max_levels < 0:
   none). */
typedef struct { int x, y; } OPoint;

static int o_x86_trunc(float x) { return (x > -2147483648.0f && x < 2147483648.0f) ? (int)x : INT32_MIN; }

static OPoint o_world_to_screen(V3 p, const mirt_camera *cam, int W, int H, float half_w, float half_h)
{                                                                   /* bvh_visualiser.c:16-41 */
    OPoint none = {-1, -1};
    V3 t = vsub(p, cam->position);
    float z = vdot(t, cam->forward);
    if (z <= 0.1f) return none;
    float x = vdot(t, cam->right);
    float y = vdot(t, cam->up);
    float sx = (x / (z * half_w * 2.0f) + 0.5f) * (float)W;
    float sy = (-y / (z * half_h * 2.0f) + 0.5f) * (float)H;
    if (sx < (float)-W || sx > (float)(W * 2) || sy < (float)-H || sy > (float)(H * 2)) return none;
    OPoint r = {o_x86_trunc(sx), o_x86_trunc(sy)};
    return r;
}

static void o_plot_line(mirt_rgba8 *img, int W, int H, int x0, int y0, int x1, int y1, mirt_rgba8 c)
{
    int dx = abs(x1 - x0), dy = -abs(y1 - y0), sx = x0 < x1 ? 1 : -1, sy = y0 < y1 ? 1 : -1, err = dx + dy;
    for (;;) {
        if (x0 >= 0 && x0 < W && y0 >= 0 && y0 < H) img[(size_t)y0 * W + x0] = c;
        if (x0 == x1 && y0 == y1) break;
        int e2 = 2 * err;
        if (e2 >= dy) { err += dy; x0 += sx; }
        if (e2 <= dx) { err += dx; y0 += sy; }
    }
}

static void o_overlay_rec(const ONode *nd, const mirt_camera *cam, int W, int H, float hw, float hh, int depth,
                          int max_levels, mirt_rgba8 *img)
{
    static const int edge[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6},
                                    {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
    static const int off[5][2] = {{0, 0}, {1, 0}, {0, 1}, {-1, 0}, {0, -1}};
    if (!nd) return;
    if (max_levels < 0 || depth < max_levels) {
        mirt_rgba8 c;                                               /* bvh_visualiser.c:107-110 */
        c.r = (uint8_t)(255 - (depth * 40) % 200);
        c.g = (uint8_t)((depth * 80) % 200);
        c.b = (uint8_t)((depth * 120) % 200);
        c.a = 180;
        const mirt_aabb *b = &nd->box;
        V3 k[8] = {v3(b->min.x, b->min.y, b->min.z), v3(b->max.x, b->min.y, b->min.z),
                   v3(b->max.x, b->max.y, b->min.z), v3(b->min.x, b->max.y, b->min.z),
                   v3(b->min.x, b->min.y, b->max.z), v3(b->max.x, b->min.y, b->max.z),
                   v3(b->max.x, b->max.y, b->max.z), v3(b->min.x, b->max.y, b->max.z)};
        for (int e = 0; e < 12; e++) {                              /* draw_aabb :84-98 */
            OPoint s = o_world_to_screen(k[edge[e][0]], cam, W, H, hw, hh);
            OPoint t = o_world_to_screen(k[edge[e][1]], cam, W, H, hw, hh);
            if (s.x == -1 || t.x == -1) continue;                   /* draw_debug_line :49 */
            if (!(s.x >= -W && s.x <= W * 2 && s.y >= -H && s.y <= H * 2 && t.x >= -W && t.x <= W * 2 &&
                  t.y >= -H && t.y <= H * 2))
                continue;
            for (int o = 0; o < 5; o++)                             /* :56-67 */
                o_plot_line(img, W, H, s.x + off[o][0], s.y + off[o][1], t.x + off[o][0], t.y + off[o][1], c);
        }
    }
    if (nd->first < 0) {                                            /* :115-116 */
        o_overlay_rec(nd->kid[0], cam, W, H, hw, hh, depth + 1, max_levels, img);
        o_overlay_rec(nd->kid[1], cam, W, H, hw, hh, depth + 1, max_levels, img);
    }
}

void o_bvh_overlay(void *root, const mirt_camera *cam, int W, int H, int max_levels, mirt_rgba8 *img)
{
    for (size_t i = 0; i < (size_t)W * H; i++) { img[i].r = img[i].g = img[i].b = 0; img[i].a = 255; }
    float fov_rad = (float)((double)cam->fov * (M_PI / 180.0));    /* bvh_visualiser.c:26-29 */
    float hh = tanf(fov_rad / 2.0f);
    float hw = (float)W / (float)H * hh;
    o_overlay_rec((const ONode *)root, cam, W, H, hw, hh, 0, max_levels, img);
}
