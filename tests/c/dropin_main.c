/*
 * A C caller of the drop-in boundary (include/mirt.h, include/mirt_dropin.h)
 * that replays the reference's interactive loop headless: main.c:203-225
 * (camera, scene, build_bvh_node) and the frame loop of main.c:274-421 --
 * the SDL event handling (camera moves -> fresh frame, camera_update on mouse
 * motion, 'b' toggles the BVH) driven by a script instead of SDL, each frame
 * ONE mirt_render_frame call in place of the per-pixel loop of main.c:356-407.
 *
 *   dropin_main W H NSPH SEED SCRIPT OUT [--ref-build LIBREF] [--per-ray] [--gpus N [--same-device]]
 *
 * SCRIPT: frames separated by ',', each listing the events polled before it:
 *   w s a d   move along forward / right (main.c:291-310)
 *   u l       SPACE / LSHIFT: up / down (main.c:311-318)
 *   b         toggle use_bvh (main.c:319-322)
 *   mX:Y;     mouse motion with the left button, xrel X, yrel Y (main.c:329-336)
 *   R         redraw: camera.move = 1 without moving (not in main.c; starts a
 *             fresh frame, e.g. the first)
 * OUT: OUT.rgba gets every displayed frame (H*W*4 bytes each, row-major) and
 * OUT.txt one line per frame: "frame sample accumulate frames use_bvh
 * <camera as 16 hex words>".
 * --ref-build LIBREF: build the tree with the REFERENCE's build_bvh_node
 * (dlsym from an oracle/_ref library) and upload that pointer tree.
 * --per-ray: also render the first frame through the per-ray surface
 * (mirt_get_camera_ray + mirt_trace_ray per pixel, the loop of
 * main.c:358-374; two launches per pixel, so for small frames) and check it
 * against mirt_render_frame's.
 * --gpus N: the same loop over N GPUs from this one thread (include/mirt_multi.h:
 * interleaved 8-row blocks per GPU, the slabs gathered to GPU 0 over RCCL, one
 * mirt_multi_render_frame per frame); --same-device puts the N ranks on GPU 0
 * (copy-mode gather: the N-GPU frame geometry on a one-GPU box).
 * Exit status 0 = ran (and the per-ray check matched).
 */
#include <dlfcn.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mirt.h"
#include "mirt_dropin.h"
#include "mirt_multi.h"

#define MOVE_SPEED 0.5f      /* constants.h:3 */
#define ROTATE_SPEED 0.002f  /* constants.h:4 */
#define MAX_DEPTH 5          /* constants.h:5 */

static mirt_vec3 v_add(mirt_vec3 a, mirt_vec3 b) { return (mirt_vec3){a.x + b.x, a.y + b.y, a.z + b.z}; }
static mirt_vec3 v_sub(mirt_vec3 a, mirt_vec3 b) { return (mirt_vec3){a.x - b.x, a.y - b.y, a.z - b.z}; }
static mirt_vec3 v_mul(mirt_vec3 v, float t) { return (mirt_vec3){v.x * t, v.y * t, v.z * t}; }

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static int fail(const char *what, int rc)
{
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, mirt_last_error());
    return 1;
}

int main(int argc, char **argv)
{
    if (argc < 7) {
        fprintf(stderr, "usage: %s W H NSPH SEED SCRIPT OUT [--ref-build LIBREF] [--per-ray]\n", argv[0]);
        return 2;
    }
    const int W = atoi(argv[1]), H = atoi(argv[2]), N = atoi(argv[3]);
    const unsigned seed = (unsigned)strtoul(argv[4], NULL, 10);
    const char *script = argv[5], *out = argv[6];
    const char *libref = NULL;
    int per_ray = 0, gpus = 0, same_device = 0;
    for (int i = 7; i < argc; i++) {
        if (!strcmp(argv[i], "--ref-build") && i + 1 < argc) libref = argv[++i];
        else if (!strcmp(argv[i], "--per-ray")) per_ray = 1;
        else if (!strcmp(argv[i], "--gpus") && i + 1 < argc) gpus = atoi(argv[++i]);
        else if (!strcmp(argv[i], "--same-device")) same_device = 1;
    }

    /* main.c:203-221: camera, srand, N x create_random_sphere */
    mirt_camera camera;
    mirt_camera_default(&camera);
    mirt_rand_state st;
    mirt_srand(&st, seed);
    mirt_sphere *spheres = malloc(sizeof(mirt_sphere) * (size_t)N);
    if (!spheres) return 1;
    int rc = mirt_scene_random(&st, spheres, N);
    if (rc) return fail("mirt_scene_random", rc);

    /* main.c:224-228: build_bvh_node(spheres, 0, N, 0), timed */
    double t0 = now();
    mirt_bvh_node *root;
    if (libref) {
        void *h = dlopen(libref, RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            fprintf(stderr, "dlopen %s: %s\n", libref, dlerror());
            return 1;
        }
        /* the reference's own builder (bvh.c:117-209): same struct bytes */
        mirt_bvh_node *(*ref_build)(mirt_sphere *, int, int, int) =
            (mirt_bvh_node * (*)(mirt_sphere *, int, int, int)) dlsym(h, "build_bvh_node");
        if (!ref_build) return fail("dlsym build_bvh_node", -1);
        root = ref_build(spheres, 0, N, 0);
        printf("BVH built by the reference's build_bvh_node\n");
    } else {
        root = mirt_build_bvh_node(spheres, 0, N, 0);
    }
    if (!root) return fail("build_bvh_node", -1);
    printf("BVH built in %f seconds (%d nodes)\n", now() - t0, mirt_bvh_count(root));

    mirt_ctx *ctx = NULL;
    mirt_multi *multi = NULL;
    if (gpus > 0) {
        /* mirt_init(num_gpus) of SURVEY 8(b): one renderer over the node's GPUs */
        int devs[64];
        if (gpus > 64) return fail("--gpus", -1);
        for (int g = 0; g < gpus; g++) devs[g] = same_device ? 0 : g;
        if ((rc = mirt_multi_create(devs, gpus, 1, 0, &multi))) return fail("mirt_multi_create", rc);
        printf("%d ranks, gather over %s\n", mirt_multi_size(multi), mirt_multi_backend(multi));
        if ((rc = mirt_multi_scene_upload(multi, spheres, N, root))) return fail("mirt_multi_scene_upload", rc);
        ctx = mirt_multi_ctx(multi, 0, 0);
    } else {
        if ((rc = mirt_create(0, &ctx))) return fail("mirt_create", rc);
        /* the reference's pointer tree and the (reordered) spheres, copied once */
        if ((rc = mirt_scene_upload(ctx, spheres, N, root))) return fail("mirt_scene_upload", rc);
    }

    char path[4096];
    snprintf(path, sizeof path, "%s.rgba", out);
    FILE *fimg = fopen(path, "wb");
    snprintf(path, sizeof path, "%s.txt", out);
    FILE *flog = fopen(path, "w");
    if (!fimg || !flog) return fail("fopen", -1);
    mirt_rgba8 *frame = malloc(sizeof(mirt_rgba8) * (size_t)W * H);
    if (!frame) return 1;

    int use_bvh = 1, accumulated_frames = 1, frame_count = 0; /* main.c:233-240 */
    double total_render_time = 0;
    const char *p = script;
    for (;;) {
        double frame_start = now();
        /* main.c:277-338: the events of this frame */
        while (*p && *p != ',') {
            switch (*p++) {
            case 'w': camera.position = v_add(camera.position, v_mul(camera.forward, MOVE_SPEED)); camera.move = 1; break;
            case 's': camera.position = v_sub(camera.position, v_mul(camera.forward, MOVE_SPEED)); camera.move = 1; break;
            case 'a': camera.position = v_sub(camera.position, v_mul(camera.right, MOVE_SPEED)); camera.move = 1; break;
            case 'd': camera.position = v_add(camera.position, v_mul(camera.right, MOVE_SPEED)); camera.move = 1; break;
            case 'u': camera.position.y += MOVE_SPEED; camera.move = 1; break;
            case 'l': camera.position.y -= MOVE_SPEED; camera.move = 1; break;
            case 'b': use_bvh = !use_bvh; printf("BVH %s\n", use_bvh ? "enabled" : "disabled"); break;
            case 'R': camera.move = 1; break;
            case 'm': {
                int xrel = 0, yrel = 0, used = 0;
                if (sscanf(p, "%d:%d;%n", &xrel, &yrel, &used) < 2 || !used) return fail("script", -1);
                p += used;
                camera.yaw += xrel * ROTATE_SPEED;
                camera.pitch -= yrel * ROTATE_SPEED;
                camera.pitch = fmax(fmin(camera.pitch, M_PI / 2 - 0.1f), -M_PI / 2 + 0.1f);
                mirt_camera_update(&camera);
                camera.move = 1;
                break;
            }
            default: break;
            }
        }
        /* main.c:349-408: fresh frame after a move, else accumulate */
        mirt_frame_desc fd;
        memset(&fd, 0, sizeof fd);
        fd.width = W;
        fd.height = H;
        fd.max_depth = MAX_DEPTH;
        fd.use_bvh = use_bvh;
        fd.seed = seed;
        fd.sample = (uint32_t)frame_count;
        fd.row_block = 8;
        fd.num_shards = 1;
        if (camera.move) {
            fd.accumulate = 0;
            fd.frames = 1;
            accumulated_frames = 1;
            camera.move = 0;
        } else {
            accumulated_frames++;
            fd.accumulate = 1;
            fd.frames = accumulated_frames;
        }
        if (multi) {
            fd.num_shards = 1; /* the whole frame: mirt_multi shards it */
            if ((rc = mirt_multi_render_frame(multi, &camera, &fd, frame))) return fail("mirt_multi_render_frame", rc);
        } else if ((rc = mirt_render_frame(ctx, &camera, &fd, frame))) {
            return fail("mirt_render_frame", rc);
        }
        fwrite(frame, sizeof(mirt_rgba8), (size_t)W * H, fimg);
        uint32_t cw[16];
        memcpy(cw, &camera, sizeof cw);
        fprintf(flog, "%d %u %d %d %d", frame_count, fd.sample, fd.accumulate, fd.frames, use_bvh);
        for (int k = 0; k < 16; k++) fprintf(flog, " %08x", cw[k]);
        fprintf(flog, "\n");

        if (per_ray && frame_count == 0) {
            /* main.c:358-374 through the per-ray surface: one get_camera_ray
               and one trace_ray per pixel, in the reference's loop order (the
               RNG contract's pixel index is the call order, y*W+x); the
               fresh frame just displayed is what it must reproduce */
            if (fd.accumulate) return fail("--per-ray needs a fresh first frame (start the script with R)", -1);
            if ((rc = mirt_dropin_init(0, W, H))) return fail("mirt_dropin_init", rc);
            mirt_dropin_rng(seed, fd.sample);
            const float aspect_ratio = (float)W / (float)H;
            int bad = 0;
            for (int y = 0; y < H; y++) {
                for (int x = 0; x < W; x++) {
                    float u = ((float)x / W - 0.5f) * aspect_ratio;
                    float v = (float)y / H - 0.5f;
                    mirt_ray ray = mirt_get_camera_ray(&camera, u, -v);
                    mirt_rgba8 c = mirt_trace_ray(ray, spheres, N, MAX_DEPTH, use_bvh ? root : NULL);
                    if (mirt_dropin_status()) return fail("mirt_trace_ray", mirt_dropin_status());
                    if (memcmp(&c, &frame[(size_t)y * W + x], 4)) bad++;
                }
            }
            printf("per-ray loop (%dx%d pixels): %d differ from mirt_render_frame\n", W, H, bad);
            mirt_dropin_release();
            if (bad) return 3;
        }

        double frame_time = now() - frame_start; /* main.c:410-420 */
        total_render_time += frame_time;
        frame_count++;
        if (frame_count % 10 == 0)
            printf("Average frame time: %f seconds (%.2f FPS)\n", total_render_time / frame_count,
                   frame_count / total_render_time);
        if (!*p) break;
        p++; /* ',' */
    }
    printf("\nFinal Performance Report:\nframes %d, average %f ms, kernel %f ms (last)\n", frame_count,
           total_render_time / frame_count * 1e3, mirt_last_kernel_ms(ctx));
    fclose(fimg);
    fclose(flog);
    if (multi) mirt_multi_destroy(multi);
    else mirt_destroy(ctx);
    mirt_free_bvh(root);
    free(frame);
    free(spheres);
    return 0;
}
