/*
 * oracle/ref_harness.c -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/).
 *
 * A headless driver around the UNMODIFIED reference sources
 * /root/reference/src/{vec3,camera,sphere,ray,bvh,hit,renderer}.c, compiled
 * by oracle/Makefile. Nothing from the reference is copied here: this file
 * only calls the reference's own functions, in the way its drivers do
 * (main.c:203-225 + main.c:356-374, benchmark.c:306-317), so the outputs it
 * produces ARE the reference's outputs. tests/golden/make_golden.py turns
 * them into committed fixtures.
 *
 * rand() is interposed (the .so links with -Bsymbolic so the reference's
 * calls bind here): mode 0 forwards to glibc's rand() (the unmodified
 * behaviour), mode 1 applies the per-pixel contract of rng_contract.h.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "Custom/constants.h"
#include "Custom/bvh.h"
#include "Custom/camera.h"
#include "Custom/hit.h"
#include "Custom/ray.h"
#include "Custom/renderer.h"
#include "Custom/sphere.h"

#include "../include/mirt.h"
#include "rng_contract.h"

static int (*g_libc_rand)(void);
static int g_mode;
static __thread uint64_t g_key;
static __thread uint32_t g_k;

int rand(void)
{
    if (g_mode == 1) return oc_draw(g_key, g_k++);
    if (!g_libc_rand) g_libc_rand = (int (*)(void))dlsym(RTLD_NEXT, "rand");
    return g_libc_rand();
}

int h_width(void) { return WIDTH; }
int h_height(void) { return HEIGHT; }
int h_sizeof_sphere(void) { return (int)sizeof(Sphere); }
int h_sizeof_node(void) { return (int)sizeof(BVHNode); }
int h_sizeof_hit(void) { return (int)sizeof(HitRecord); }
int h_sizeof_camera(void) { return (int)sizeof(Camera); }
void h_srand(unsigned s) { srand(s); }
int h_rand(void) { return rand(); }

/* main.c:218-221 */
void h_gen_render_scene(unsigned seed, int n, Sphere *out)
{
    g_mode = 0;
    srand(seed);
    for (int i = 0; i < n; i++) out[i] = create_random_sphere();
}

/* benchmark.c:307-314 (the centre expression is the driver's, the sphere
   comes from the reference's create_benchmark_sphere) */
void h_gen_bench_scene(unsigned seed, int n, float world_size, Sphere *out)
{
    g_mode = 0;
    srand(seed);
    for (int j = 0; j < n; j++) {
        Vec3 c;
        c.x = (float)rand() / RAND_MAX * world_size - world_size / 2;
        c.y = (float)rand() / RAND_MAX * world_size - world_size / 2;
        c.z = (float)rand() / RAND_MAX * world_size - world_size / 2;
        out[j] = create_benchmark_sphere(c);
    }
}

void *h_build(Sphere *s, int start, int end, int depth) { return build_bvh_node(s, start, end, depth); }

static void free_tree(BVHNode *n)
{
    if (!n) return;
    free_tree(n->left);
    free_tree(n->right);
    free(n);
}
void h_free(void *root) { free_tree((BVHNode *)root); }

static int count_tree(const BVHNode *n) { return n ? 1 + count_tree(n->left) + count_tree(n->right) : 0; }
int h_node_count(void *root) { return count_tree((const BVHNode *)root); }

static int flat_rec(const BVHNode *n, const Sphere *base, mirt_node *out, int at)
{
    int me = at++;
    out[me].bmin[0] = n->bounds.min.x; out[me].bmin[1] = n->bounds.min.y; out[me].bmin[2] = n->bounds.min.z;
    out[me].bmax[0] = n->bounds.max.x; out[me].bmax[1] = n->bounds.max.y; out[me].bmax[2] = n->bounds.max.z;
    if (n->sphere) {
        out[me].sphere = (int32_t)(n->sphere - base);
    } else {
        out[me].sphere = -1;
        at = flat_rec(n->left, base, out, at);
        at = flat_rec(n->right, base, out, at);
    }
    out[me].skip = (uint32_t)at | ((n->sphere && n->sphere_count == 0) ? MIRT_NODE_EMPTY : 0u);
    return at;
}
int h_flatten(void *root, const Sphere *base, mirt_node *out, int cap)
{
    int n = count_tree((const BVHNode *)root);
    if (n > cap) return -n;
    return flat_rec((const BVHNode *)root, base, out, 0);
}

/* leaf sphere_count of every leaf in DFS order (stats) */
static int leafcounts_rec(const BVHNode *n, int32_t *out, int at)
{
    if (n->sphere) { out[at] = n->sphere_count; return at + 1; }
    at = leafcounts_rec(n->left, out, at);
    return leafcounts_rec(n->right, out, at);
}
int h_leaf_counts(void *root, int32_t *out) { return leafcounts_rec((const BVHNode *)root, out, 0); }

static void put_hit(const HitRecord *h, const Sphere *base, mirt_hit *o)
{
    o->t = h->t;
    o->point.x = h->point.x; o->point.y = h->point.y; o->point.z = h->point.z;
    o->normal.x = h->normal.x; o->normal.y = h->normal.y; o->normal.z = h->normal.z;
    o->hit = h->hit_something;
    o->sphere = (h->hit_something && h->object) ? (int32_t)(h->object - base) : -1;
    o->pad = 0;
}

void h_intersect_bvh(void *root, const Sphere *base, const Ray *rays, int n, mirt_hit *out)
{
    for (int i = 0; i < n; i++) {
        HitRecord h = ray_bvh_intersect(rays[i], (BVHNode *)root);
        put_hit(&h, base, &out[i]);
    }
}

/* One point of run_benchmark_with_plotting (benchmark.c:283-332) on the
   CURRENT rand() stream (h_srand once, then the points in sweep order):
   n spheres (benchmark.c:307-314), build_bvh_node(s, 0, n - 1, 20)
   (benchmark.c:317), then the loops of benchmark_no_bvh (benchmark.c:
   172-222) and benchmark_with_bvh (benchmark.c:224-255) around the
   reference's own vec3_normalize / ray_sphere_intersect / ray_bvh_intersect,
   timed with clock() as there. Out: the spheres (post-build order), the two
   ray sets, per-ray hit flags, seconds of each loop. */
void h_bench_point(int n, int num_rays, float world_size, Sphere *s_out, Ray *rays_a, Ray *rays_b,
                   int32_t *hit_a, int32_t *hit_b, double *secs)
{
    g_mode = 0;
    Sphere *s = malloc((size_t)n * sizeof(Sphere));
    for (int j = 0; j < n; j++) {
        Vec3 c = {
            (float)rand() / RAND_MAX * world_size - world_size / 2,
            (float)rand() / RAND_MAX * world_size - world_size / 2,
            (float)rand() / RAND_MAX * world_size - world_size / 2};
        s[j] = create_benchmark_sphere(c);
    }
    BVHNode *root = build_bvh_node(s, 0, n - 1, 20);
    clock_t t0 = clock();
    for (int i = 0; i < num_rays; i++) {
        Vec3 dir = {
            (float)rand() / RAND_MAX * 2 - 1,
            (float)rand() / RAND_MAX * 2 - 1,
            (float)rand() / RAND_MAX * 2 - 1};
        dir = vec3_normalize(dir);
        Ray ray = {{0, 0, 0}, dir};
        int found = 0;
        for (int j = 0; j < n; j++) {
            HitRecord h = ray_sphere_intersect(ray, &s[j]);
            if (h.hit_something) found = 1;
        }
        rays_a[i] = ray;
        hit_a[i] = found;
    }
    clock_t t1 = clock();
    for (int i = 0; i < num_rays; i++) {
        Vec3 dir = {
            (float)rand() / RAND_MAX * 2 - 1,
            (float)rand() / RAND_MAX * 2 - 1,
            (float)rand() / RAND_MAX * 2 - 1};
        dir = vec3_normalize(dir);
        Ray ray = {{0, 0, 0}, dir};
        HitRecord h = ray_bvh_intersect(ray, root);
        rays_b[i] = ray;
        hit_b[i] = h.hit_something;
    }
    clock_t t2 = clock();
    secs[0] = (double)(t1 - t0) / CLOCKS_PER_SEC;
    secs[1] = (double)(t2 - t1) / CLOCKS_PER_SEC;
    memcpy(s_out, s, (size_t)n * sizeof(Sphere));
    free_tree(root);
    free(s);
}

void h_sphere_pairs(const Ray *rays, Sphere *s, int n, mirt_hit *out)
{
    for (int i = 0; i < n; i++) {
        HitRecord h = ray_sphere_intersect(rays[i], &s[i]);
        put_hit(&h, &s[i], &out[i]);
        if (out[i].hit) out[i].sphere = i;
    }
}

void h_aabb_pairs(const Ray *rays, const AABB *b, int n, int32_t *out)
{
    for (int i = 0; i < n; i++) out[i] = ray_aabb_intersect(rays[i], b[i]);
}

/* main.c:356-366 for one pixel */
void h_camera_ray(Camera *cam, int x, int y, Ray *out)
{
    float aspect_ratio = (float)WIDTH / (float)HEIGHT;
    float u = ((float)x / WIDTH - 0.5f) * aspect_ratio;
    float v = (float)y / HEIGHT - 0.5f;
    *out = get_camera_ray(cam, u, -v);
}

/* main.c:358-374 over the rows [row0, row0 + nrows*step) with stride step.
   mode 0 = the unmodified glibc stream (call h_srand first), single thread;
   mode 1 = rng contract, any thread count. */
void h_render(const Camera *cam_in, Sphere *spheres, int n, void *root, int depth, int use_bvh, int mode,
              uint64_t seed, uint32_t sample, int row0, int step, int nrows, uint8_t *rgba, int nthreads,
              int jitter)
{
    g_mode = mode;
    if (mode == 0) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
    for (int ri = 0; ri < nrows; ri++) {
        Camera cam = *cam_in;
        int y = row0 + ri * step;
        float aspect_ratio = (float)WIDTH / (float)HEIGHT;
        for (int x = 0; x < WIDTH; x++) {
            float u = ((float)x / WIDTH - 0.5f) * aspect_ratio;
            float v = (float)y / HEIGHT - 0.5f;
            if (mode == 1) { g_key = oc_pixel_key(seed, (uint32_t)(y * WIDTH + x), sample); g_k = 0; }
            if (mode == 1 && jitter) {  /* the build's jitter (rng_contract.h), not main.c */
                float xf = (float)x + (float)oc_draw(g_key, OC_JITTER_X) / 2147483648.0f;
                float yf = (float)y + (float)oc_draw(g_key, OC_JITTER_Y) / 2147483648.0f;
                u = (xf / WIDTH - 0.5f) * aspect_ratio;
                v = yf / HEIGHT - 0.5f;
            }
            Ray ray = get_camera_ray(&cam, u, -v);
            SDL_Color c = trace_ray(ray, spheres, n, depth, use_bvh ? (BVHNode *)root : NULL);
            uint8_t *p = rgba + ((size_t)ri * WIDTH + x) * 4;
            p[0] = c.r; p[1] = c.g; p[2] = c.b; p[3] = c.a;
        }
    }
    g_mode = 0;
}

/* trace_ray on explicit rays; ray i uses contract pixel i in mode 1 */
void h_trace_rays(const Ray *rays, int n, Sphere *spheres, int ns, void *root, int depth, int use_bvh, int mode,
                  uint64_t seed, uint32_t sample, uint8_t *rgba)
{
    g_mode = mode;
    for (int i = 0; i < n; i++) {
        if (mode == 1) { g_key = oc_pixel_key(seed, (uint32_t)i, sample); g_k = 0; }
        SDL_Color c = trace_ray(rays[i], spheres, ns, depth, use_bvh ? (BVHNode *)root : NULL);
        rgba[4 * i + 0] = c.r; rgba[4 * i + 1] = c.g; rgba[4 * i + 2] = c.b; rgba[4 * i + 3] = c.a;
    }
    g_mode = 0;
}

void h_camera_update(Camera *cam) { camera_update(cam); }
