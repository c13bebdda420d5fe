/*
 * A C caller of the drop-in boundary replaying the reference's benchmark mode
 * (run_benchmark_with_plotting, benchmark.c:283-332) with its two timed loops
 * (benchmark_no_bvh benchmark.c:172-220, benchmark_with_bvh benchmark.c:
 * 222-255) as batch calls: one glibc rand() stream (srand once, a fixed seed
 * in place of time(NULL)), per sweep point n spheres at uniform centres
 * (benchmark.c:307-314), build_bvh_node(spheres, 0, n - 1, 20)
 * (benchmark.c:317), num_rays rays for the brute-force loop, num_rays more for
 * the BVH loop.
 *
 *   dropin_bench SEED NUM_RAYS OUT n1 [n2 ...] [--per-ray K]
 *
 * Prints the reference's report per point and appends save_benchmark_data's
 * "n time_no_bvh time_with_bvh" line (benchmark.c:160-170; device seconds of
 * the batch launches) to OUT.txt; OUT.bin gets, per point, the int32 hit flags
 * of the brute-force loop and of the BVH loop (num_rays each).
 * --per-ray K: the first K rays of both loops again through the per-ray
 * surface (mirt_ray_sphere_intersect over every sphere / mirt_ray_bvh_intersect
 * on the pointer tree, the calls benchmark.c:196 and :242 make) -- must agree.
 * --per-ray-bvh K: the BVH loop's first K rays only (one launch per ray, so it
 * runs at every point of the reference sweep, whose arrays of 10k spheres and
 * up glibc munmaps on free: the drop-in must never read a freed array).
 * Each point declares its whole array (mirt_dropin_scene: the tree covers
 * [0, n - 1) of it, benchmark.c:317) and clears the declaration before
 * freeing it -- the documented recipe for benchmark.c.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mirt.h"
#include "mirt_dropin.h"

static int fail(const char *what, int rc)
{
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, mirt_last_error());
    return 1;
}

int main(int argc, char **argv)
{
    if (argc < 5) {
        fprintf(stderr, "usage: %s SEED NUM_RAYS OUT n1 [n2 ...] [--per-ray K]\n", argv[0]);
        return 2;
    }
    const unsigned seed = (unsigned)strtoul(argv[1], NULL, 10);
    const int num_rays = atoi(argv[2]);
    const char *out = argv[3];
    int per_ray = 0, per_ray_bvh = 0, npts = 0;
    int counts[64];
    for (int i = 4; i < argc; i++) {
        if (!strcmp(argv[i], "--per-ray") && i + 1 < argc) per_ray = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--per-ray-bvh") && i + 1 < argc) per_ray_bvh = atoi(argv[++i]);
        else if (npts < 64) counts[npts++] = atoi(argv[i]);
    }
    const float world_size = 1000.0f; /* benchmark.c:299 */

    char path[4096];
    snprintf(path, sizeof path, "%s.txt", out);
    FILE *fdat = fopen(path, "w"); /* remove("benchmark_data.txt") + append, benchmark.c:285 */
    snprintf(path, sizeof path, "%s.bin", out);
    FILE *fbin = fopen(path, "wb");
    if (!fdat || !fbin) return fail("fopen", -1);

    mirt_ctx *ctx;
    int rc = mirt_create(0, &ctx);
    if (rc) return fail("mirt_create", rc);
    mirt_rand_state st;
    mirt_srand(&st, seed); /* benchmark.c:286 */
    mirt_ray *rays_a = malloc(sizeof(mirt_ray) * (size_t)num_rays);
    mirt_ray *rays_b = malloc(sizeof(mirt_ray) * (size_t)num_rays);
    int32_t *hit_a = malloc(sizeof(int32_t) * (size_t)num_rays);
    int32_t *hit_b = malloc(sizeof(int32_t) * (size_t)num_rays);
    mirt_hit *rec_b = malloc(sizeof(mirt_hit) * (size_t)num_rays);
    if (!rays_a || !rays_b || !hit_a || !hit_b || !rec_b) return 1;
    int mismatches = 0;

    for (int i = 0; i < npts; i++) {
        const int n = counts[i];
        printf("Testing with %d spheres:\n", n);
        mirt_sphere *spheres = malloc(sizeof(mirt_sphere) * (size_t)n);
        if (!spheres) return 1;
        if ((rc = mirt_scene_benchmark(&st, spheres, n, world_size))) return fail("mirt_scene_benchmark", rc);
        mirt_bvh_node *root = mirt_build_bvh_node(spheres, 0, n - 1, 20); /* benchmark.c:317 */
        if (!root) return fail("mirt_build_bvh_node", -1);
        /* the rays each loop draws from the same stream (benchmark.c:176-185, 228-237) */
        if ((rc = mirt_bench_rays(&st, rays_a, num_rays))) return fail("mirt_bench_rays", rc);
        if ((rc = mirt_bench_rays(&st, rays_b, num_rays))) return fail("mirt_bench_rays", rc);
        if ((rc = mirt_scene_upload(ctx, spheres, n, root))) return fail("mirt_scene_upload", rc);
        if ((rc = mirt_dropin_scene(spheres, n))) return fail("mirt_dropin_scene", rc);

        if ((rc = mirt_any_hit_rays(ctx, rays_a, num_rays, 0, hit_a))) return fail("mirt_any_hit_rays", rc);
        const double t_no = mirt_last_kernel_ms(ctx) / 1e3;
        int inter_a = 0;
        for (int k = 0; k < num_rays; k++) inter_a += hit_a[k];
        printf("No BVH:\nTime: %f seconds\nIntersection tests: %lld\nIntersections found: %d\n\n", t_no,
               (long long)n * num_rays, inter_a);

        if ((rc = mirt_intersect_rays(ctx, rays_b, num_rays, 1, rec_b))) return fail("mirt_intersect_rays", rc);
        const double t_bvh = mirt_last_kernel_ms(ctx) / 1e3;
        int inter_b = 0;
        for (int k = 0; k < num_rays; k++) inter_b += (hit_b[k] = rec_b[k].hit);
        printf("With BVH:\nTime: %f seconds\nIntersections found: %d\n\n", t_bvh, inter_b);

        if (per_ray > 0) {
            /* benchmark.c:190-199 and :239-241, one ray at a time */
            const int K = per_ray < num_rays ? per_ray : num_rays;
            for (int k = 0; k < K; k++) {
                int found = 0;
                for (int j = 0; j < n && !found; j++)
                    found = mirt_ray_sphere_intersect(rays_a[k], &spheres[j]).hit_something;
                if (mirt_dropin_status()) return fail("mirt_ray_sphere_intersect", mirt_dropin_status());
                if (found != hit_a[k]) mismatches++;
                mirt_hit_record h = mirt_ray_bvh_intersect(rays_b[k], root);
                if (mirt_dropin_status()) return fail("mirt_ray_bvh_intersect", mirt_dropin_status());
                if (h.hit_something != hit_b[k] ||
                    (h.hit_something && (h.object != &spheres[rec_b[k].sphere] || h.t != rec_b[k].t)))
                    mismatches++;
            }
            printf("per-ray surface, first %d rays of both loops: %d mismatches\n", K, mismatches);
        }
        if (per_ray_bvh > 0) {
            const int K = per_ray_bvh < num_rays ? per_ray_bvh : num_rays;
            int bad = 0;
            for (int k = 0; k < K; k++) {
                mirt_hit_record h = mirt_ray_bvh_intersect(rays_b[k], root);
                if (mirt_dropin_status()) return fail("mirt_ray_bvh_intersect", mirt_dropin_status());
                if (h.hit_something != hit_b[k] ||
                    (h.hit_something && (h.object != &spheres[rec_b[k].sphere] || h.t != rec_b[k].t)))
                    bad++;
            }
            mismatches += bad;
            printf("per-ray BVH surface, first %d rays: %d mismatches\n", K, bad);
        }

        fprintf(fdat, "%d %f %f\n", n, t_no, t_bvh); /* save_benchmark_data */
        fwrite(hit_a, sizeof(int32_t), (size_t)num_rays, fbin);
        fwrite(hit_b, sizeof(int32_t), (size_t)num_rays, fbin);
        /* benchmark.c:323-324 exactly: no invalidate -- the next size's tree
           and array usually come back at these addresses, and the drop-in's
           content fingerprint has to notice (the per-ray check above runs at
           every sweep point) */
        mirt_dropin_scene(NULL, 0);
        mirt_free_bvh(root);
        free(spheres);
        printf("----------------------------------------\n");
    }
    fclose(fdat);
    fclose(fbin);
    mirt_dropin_release();
    mirt_destroy(ctx);
    free(rays_a);
    free(rays_b);
    free(hit_a);
    free(hit_b);
    free(rec_b);
    return mismatches ? 3 : 0;
}
