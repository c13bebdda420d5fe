/*
 * include/mirt.h -- C ABI of the MI355X-native primary-ray render path
 * (camera rays -> BVH traversal + ray/sphere intersection -> closest-hit
 * diffuse shading -> RGBA framebuffer) of ShivangNagta/CS201_SAH-BVH_Ray_Tracer.
 *
 * Every entry point is plain C: POD structs, pointers and sizes, int status.
 * Structs are layout-compatible with the reference's own types (sizes are
 * asserted in csrc/host_scene.cpp), so a caller can pass its arrays through
 * unchanged. The reference interface each entry point replaces is cited as
 * file:line under /root/reference/ (see also INTEGRATION.md).
 *
 * Threading: one host thread per mirt_ctx. Blocking calls return with the
 * result in host memory; *_device calls enqueue on the given HIP stream.
 * Errors: negative status, message in mirt_last_error(); the library never
 * aborts and never falls back to a CPU path.
 */
#ifndef MIRT_H
#define MIRT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ types */

typedef struct mirt_vec3 { float x, y, z; } mirt_vec3;            /* vec3.h:3-7 (12 B)   */
typedef struct mirt_rgba8 { uint8_t r, g, b, a; } mirt_rgba8;     /* SDL_Color (4 B)     */
typedef struct mirt_sphere {                                      /* sphere.h:7-11 (20 B) */
    mirt_vec3 center;
    float radius;
    mirt_rgba8 color;
} mirt_sphere;
typedef struct mirt_ray { mirt_vec3 origin, direction; } mirt_ray; /* ray.h:5-8 (24 B)   */
typedef struct mirt_camera {                                      /* camera.h:5-14 (64 B) */
    mirt_vec3 position, forward, right, up;
    float yaw, pitch, fov;
    int move;
} mirt_camera;
typedef struct mirt_aabb { mirt_vec3 min, max; } mirt_aabb;       /* bvh.h:7-10 (24 B)   */
typedef struct mirt_bvh_node {                                    /* bvh.h:12-18 (56 B)  */
    mirt_aabb bounds;
    struct mirt_bvh_node *left, *right;
    mirt_sphere *sphere;
    int sphere_count;
} mirt_bvh_node;
typedef struct mirt_hit_record {                                  /* hit.h:8-14 (40 B)   */
    float t;
    mirt_vec3 point, normal;
    int hit_something;
    mirt_sphere *object;
} mirt_hit_record;

/* HitRecord for batch calls: the object pointer becomes an index into the
   uploaded sphere array (-1: no hit). 40 B. */
typedef struct mirt_hit {
    float t;
    mirt_vec3 point, normal;
    int32_t hit;
    int32_t sphere;
    int32_t pad;
} mirt_hit;

/* Flattened BVH node, the layout the kernel walks (32 B, 32-B aligned).
   Depth-first pre-order of the reference tree (bvh.c:203-204: left subtree,
   then right): the left child of inner node i is i+1 and `skip` is the index
   that follows i's subtree, so the reference DFS order (hit.c:102-103) is a
   forward scan that jumps to `skip` when a box is missed or a leaf is done.
   sphere  >= 0: leaf testing spheres[sphere] (bvh.c:133; == num_spheres is the
            never-hit sentinel of SURVEY §8.H7); -1: inner node.
   skip bit 31 (MIRT_NODE_EMPTY): the leaf holds 0 spheres; its box is the
            inverted create_empty_aabb() box (bvh.c:19-24), which always passes
            ray_aabb_intersect (hit.c:49-82). */
typedef struct mirt_node {
    float bmin[3];
    float bmax[3];
    int32_t sphere;
    uint32_t skip;
} mirt_node;
#define MIRT_NODE_EMPTY 0x80000000u
#define MIRT_SKIP_MASK 0x7fffffffu

/* glibc TYPE_3 rand() state (the reference seeds glibc with srand(),
   main.c:90, benchmark.c:287). */
typedef struct mirt_rand_state {
    int32_t r[34];
    int32_t f, b;
} mirt_rand_state;

/* One frame (or one shard of one frame). */
typedef struct mirt_frame_desc {
    int32_t width, height;   /* the reference's compile-time WIDTH/HEIGHT (constants.h:7-8) */
    int32_t max_depth;       /* trace_ray depth argument (main.c:366, MAX_DEPTH = 5) */
    int32_t use_bvh;         /* main.c:366 `use_bvh ? root : NULL`; 0 = brute force */
    uint64_t seed;           /* RNG contract seed */
    uint32_t sample;         /* RNG contract sample index (frame number) */
    int32_t accumulate;      /* 0: fresh frame main.c:358-374; 1: accumulate main.c:379-408 */
    int32_t frames;          /* accumulate: divisor accumulated_frames (main.c:380) */
    int32_t row_block;       /* rows per interleave block (default 8) */
    int32_t shard;           /* this shard renders row blocks b with b % num_shards == shard */
    int32_t num_shards;
    int32_t samples;         /* frames rendered by this call, samples sample .. sample+samples-1 of the
                                RNG contract (0 or 1: one). One launch covers all of them, so the
                                bounce pass's tail (its longest chains) is paid once, not per frame.
                                Output: `samples` consecutive slabs, one per frame; with an
                                accumulation buffer, the frames are folded into it in order (as
                                `samples` successive calls would: frame j has divisor frames + j)
                                and slab j holds the display main.c:379-408 shows after frame j
                                (the blocking / async calls return the last one) */
    int32_t jitter;          /* 1: camera rays through (x + jx, y + jy), j in [0, 1)^2 from the pixel's
                                RNG contract stream (rng.h; BASELINE configs[4] "4 spp jittered" --
                                the reference samples pixel corners only); 0: main.c:362-363 */
    int32_t lead_skip;       /* shard weighting (mirt 0.6; 0 = none): blocks are dealt in periods of 8
                                rounds, one block per shard per round, and shard 0 sits out the first
                                lead_skip (0..7) rounds of every period -- so shard 0 renders
                                (8 - lead_skip) / (8 num_shards - lead_skip) of the frame
                                (csrc/shard.h). 0 = block b to shard b % num_shards. num_shards >= 2 */
} mirt_frame_desc;

/* Work counters of the walk as configured; with MIRT_OPT_PRUNE = 0 they are
   exactly the reference DFS (hit.c:91-109) node and sphere tests. */
typedef struct mirt_counts {
    uint64_t rays;       /* rays traced (primary + bounces) */
    uint64_t nodes;      /* ray_aabb_intersect calls */
    uint64_t spheres;    /* ray_sphere_intersect calls from leaves (or brute force) */
    uint64_t hits;       /* rays that found a closest hit */
    uint64_t lane_steps; /* traversal loop iterations x 64 lanes executed by the
                            default schedule; nodes / lane_steps = SIMD efficiency */
    /* the camera-ray level alone (depth level 0 = the wavefront schedule's
       primary pass); nodes - nodes_primary etc. is the bounce pass */
    uint64_t nodes_primary;
    uint64_t spheres_primary;
    uint64_t hits_primary;
} mirt_counts;

enum {
    MIRT_OK = 0,
    MIRT_E_INVALID = -1,
    MIRT_E_NOMEM = -2,
    MIRT_E_NOSCENE = -3,
    MIRT_E_DEVICE = -4   /* HIP runtime error; see mirt_last_error() */
};

typedef struct mirt_ctx mirt_ctx;

const char *mirt_version(void);
const char *mirt_last_error(void);

/* ------------------------------------------------- host: scene inputs */

/* glibc srand()/rand() restated (TYPE_3 additive feedback), so scenes are
   reproducible from a seed on any host. */
void mirt_srand(mirt_rand_state *st, unsigned int seed);
int mirt_rand(mirt_rand_state *st);

/* n x create_random_sphere() (sphere.c:52-59) as main.c:218-221. */
int mirt_scene_random(mirt_rand_state *st, mirt_sphere *out, int n);
/* n x benchmark centre + create_benchmark_sphere() (benchmark.c:307-314, sphere.c:34-41). */
int mirt_scene_benchmark(mirt_rand_state *st, mirt_sphere *out, int n, float world_size);
/* n benchmark rays (benchmark.c:176-185, 228-237): origin 0, direction
   vec3_normalize of three (float)rand()/RAND_MAX*2-1 draws. */
int mirt_bench_rays(mirt_rand_state *st, mirt_ray *out, int n);
/* The default camera of main.c:203-211. */
void mirt_camera_default(mirt_camera *cam);
/* camera_update (camera.c:10-18): basis from yaw/pitch. */
void mirt_camera_update(mirt_camera *cam);

/* --------------------------------------------- host: BVH (bit-identical) */

/* build_bvh_node (bvh.c:117-209): same signature, same pointer tree, same
   in-place reordering of `spheres`. Free with mirt_free_bvh. */
mirt_bvh_node *mirt_build_bvh_node(mirt_sphere *spheres, int start, int end, int depth);
/* free_bvh (benchmark.c:81-88) */
void mirt_free_bvh(mirt_bvh_node *node);
/* Number of nodes in a pointer tree. */
int mirt_bvh_count(const mirt_bvh_node *root);
/* Flatten a pointer tree (built by the reference's build_bvh_node or by
   mirt_build_bvh_node) whose leaf pointers index `base`. Returns the node
   count, or -needed if cap is too small. */
int mirt_bvh_flatten(const mirt_bvh_node *root, const mirt_sphere *base, mirt_node *out, int cap);
/* Build straight into the flat layout: same tree as
   mirt_bvh_flatten(build_bvh_node(spheres, start, end, depth)) bit for bit,
   with the SAH planes of bvh.c:143-170 evaluated by one binned pass per axis.
   *out_nodes is malloc'd; release with mirt_bvh_free_flat. */
int mirt_bvh_build_flat(mirt_sphere *spheres, int start, int end, int depth,
                        mirt_node **out_nodes, int *out_count);
void mirt_bvh_free_flat(mirt_node *nodes);
/* Check that nodes[0, num_nodes) is a well-formed flat pre-order tree over
   num_spheres spheres: root skip == num_nodes, every skip in (i, num_nodes],
   leaves skip to i + 1 and index spheres in [0, num_spheres] (num_spheres =
   the never-hit sentinel), MIRT_NODE_EMPTY only on leaves, and every inner
   node's two subtrees [i+1, r) and [r, skip) nest exactly inside it.
   MIRT_OK or MIRT_E_INVALID (mirt_last_error names the first bad node). The
   uploads run this check; it never touches the GPU. */
int mirt_bvh_validate_flat(const mirt_node *nodes, int num_nodes, int num_spheres);
/* mirt_bvh_build_flat through a flattened-tree cache file (SURVEY.md §8(f)
   rank 3; replaces the build_bvh_node call at main.c:225 / benchmark.c:317 on
   a rerun). If `path` holds the tree of exactly these input spheres
   (FNV-1a 64 of spheres[start,end) + start, end, depth; payload hash checked)
   the reordered spheres are copied into spheres[start,end), the nodes are
   returned and *out_cached = 1. Otherwise the tree is built, written to
   `path` (temp file + rename) and *out_cached = 0, or -1 if the file could
   not be written (the build result is still returned; mirt_last_error says
   why). Same outputs as mirt_bvh_build_flat, bit for bit. */
int mirt_bvh_build_flat_cached(const char *path, mirt_sphere *spheres, int start, int end, int depth,
                               mirt_node **out_nodes, int *out_count, int *out_cached);

/* ------------------------------------------------------ device context */

int mirt_create(int device, mirt_ctx **out);
void mirt_destroy(mirt_ctx *ctx);

/* Copy the (already built, hence reordered) spheres and the caller's tree to
   the device. The library keeps no pointer into caller memory. */
int mirt_scene_upload(mirt_ctx *ctx, const mirt_sphere *spheres, int num_spheres, const mirt_bvh_node *root);
int mirt_scene_upload_flat(mirt_ctx *ctx, const mirt_sphere *spheres, int num_spheres,
                           const mirt_node *nodes, int num_nodes);

/* ---------------------------------------------------------- rendering */

/* Number of rows (and the row indices, if rows != NULL) a shard renders. */
int mirt_shard_rows(const mirt_frame_desc *fd, int32_t *rows);

/* The pixel loop of main.c:356-374 (fresh) / main.c:382-407 (accumulate) for
   the shard described by fd: writes the displayed RGBA8 colour of every pixel
   of the shard's rows, compacted in shard row order, to host memory `out`
   (num_rows * width). Accumulation state lives on the device (per ctx); with
   fd->samples > 1 the frames are accumulated in order and `out` receives the
   display after the last one. */
int mirt_render_frame(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd, mirt_rgba8 *out);

/* Same, asynchronously on `stream` (a hipStream_t; NULL = the default stream),
   into device memory: d_out = samples * num_rows * width packed RGBA8 (frame
   j's slab at j * num_rows * width). d_accum is a device float buffer of
   num_rows * width * 3 (may be NULL when fd->accumulate == 0); given with
   samples > 1, the frames are folded into it and slab j receives the display
   after frame j. Given by ctxs that share their accumulation buffer
   (mirt_ctx_share_accum), the folds into d_accum follow call order across
   those ctxs' streams. Inputs are already resident in HBM. The ctx's frame scratch
   (bounce queue, deferral list) is one per ctx: a launch on a different
   stream than the ctx's previous launch first waits for that launch (an
   event), so frames of one ctx never overlap; use one ctx per stream for
   frames in flight. */
int mirt_render_frame_device(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd,
                             uint32_t *d_out, float *d_accum, void *stream);

/* Frames in flight to host memory (SURVEY §8(d) t_frame: call -> RGBA8 on
   the host). mirt_render_frame_async enqueues what mirt_render_frame does --
   the frame's kernels and the D2H copy of its display into `out` -- on the
   ctx's own stream and returns at once; `out` holds the frame once
   mirt_ctx_wait(ctx) returns (or after the next blocking call on the ctx).
   `out` should be page-locked memory from mirt_host_alloc: then the copy is a
   DMA that overlaps the next frame's kernels on another ctx; pageable memory
   works too but the runtime stages it. Rotating two or three ctxs (each with
   the scene uploaded) keeps the GPU busy while earlier frames drain and
   copy: for frame k use ctx k % n, mirt_ctx_wait it first (its buffer from
   frame k - n is then complete), then mirt_render_frame_async. For the
   accumulating loop (main.c:379-408) the rotated ctxs must share ONE
   accumulation buffer: mirt_ctx_share_accum(ctx[i], ctx[0]). */
int mirt_render_frame_async(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd, mirt_rgba8 *out);
/* Block until every call enqueued on the ctx's stream has finished. */
int mirt_ctx_wait(mirt_ctx *ctx);
/* Page-locked host memory (hipHostMalloc) for frame outputs; mirt_host_free
   releases it (NULL is ignored). */
int mirt_host_alloc(size_t bytes, void **out);
void mirt_host_free(void *p);
/* Page-lock a caller-owned buffer in place (hipHostRegister) -- the frame
   buffer main.c:241-273's loop mallocs once and reuses every frame: the
   blocking mirt_render_frame's D2H into it is then one DMA instead of the
   runtime's staged pageable copy -- or none at all: with MIRT_OPT_ZERO_COPY
   (default) the frame kernels write the pixels straight into it. The
   registration pins the pages until mirt_host_unregister, which must come
   before the buffer is freed. */
int mirt_host_register(void *p, size_t bytes);
int mirt_host_unregister(void *p);

/* Download the ctx's accumulation buffer (row-major float3 of the shard),
   after every fold enqueued into it so far. */
int mirt_accum_download(mirt_ctx *ctx, float *out, size_t count);

/* Frames in flight of ONE accumulating display loop (main.c:379-408) on
   several ctxs: ctx uses owner's accumulation buffer from now on (owner NULL
   or ctx itself: a private buffer again). Each frame's colours then go to
   the ctx's own slab and a fold kernel adds them to the shared buffer; the
   folds run in call order across the ctxs' streams (events), the tracing
   still overlaps. Without it every ctx accumulates only its own frames, so a
   rotation of n ctxs would average 1/n of the frames. Both ctxs must be on
   the same device; waits for ctx's enqueued frames first. Ctxs that share a
   buffer must be driven from ONE host thread (the call order is the fold
   order). */
int mirt_ctx_share_accum(mirt_ctx *ctx, mirt_ctx *owner);

/* trace_ray (renderer.c:21-77) on n arbitrary rays; ray i uses RNG contract
   pixel index i. */
int mirt_trace_rays(mirt_ctx *ctx, const mirt_ray *rays, int n, int depth, int use_bvh,
                    uint64_t seed, uint32_t sample, mirt_rgba8 *out);
/* Same, ray i using RNG contract pixel index pixel0 + i (a caller's own pixel
   loop in chunks: pixel0 = y * width + x of the chunk's first pixel). */
int mirt_trace_rays_at(mirt_ctx *ctx, const mirt_ray *rays, int n, int depth, int use_bvh,
                       uint64_t seed, uint32_t sample, uint32_t pixel0, mirt_rgba8 *out);

/* Closest hit: ray_bvh_intersect (hit.c:91-109) when use_bvh, else the brute
   force loop of renderer.c:36-43. */
int mirt_intersect_rays(mirt_ctx *ctx, const mirt_ray *rays, int n, int use_bvh, mirt_hit *out);

/* benchmark.c:172-255 as batches. Any hit: out[i] = 1 if ray i hits some
   sphere (benchmark_no_bvh's hit_found, benchmark.c:190-199, when use_bvh =
   0; ray_bvh_intersect(...).hit_something, benchmark.c:239-241, when 1).
   Both intersect calls split the brute-force loop over sphere chunks across
   the chip (64-bit atomicMin of (t, index): the first sphere wins ties as in
   renderer.c:39; every sphere is tested, as the reference does). The device
   time of the call's kernels is mirt_last_kernel_ms(). */
int mirt_any_hit_rays(mirt_ctx *ctx, const mirt_ray *rays, int n, int use_bvh, int32_t *out);

/* Element-wise ray_sphere_intersect (hit.c:19-39) / ray_aabb_intersect
   (hit.c:49-82) on pairs; need no scene. */
int mirt_sphere_pairs(mirt_ctx *ctx, const mirt_ray *rays, const mirt_sphere *spheres, int n, mirt_hit *out);
int mirt_aabb_pairs(mirt_ctx *ctx, const mirt_ray *rays, const mirt_aabb *boxes, int n, int32_t *out);

/* The camera ray of every pixel of the shard (ray.c:17-32 with the pixel
   mapping of main.c:356-365). */
int mirt_camera_rays(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd, mirt_ray *out);
/* The BVH debug overlay (bvh_visualiser.c:16-126, 'o' in main.c:323-327):
   every node of the uploaded tree with depth < max_levels (all: -1) drawn as
   its box's 12 projected edges, 5 one-pixel-offset lines each, coloured by
   depth, over black; a pixel shows the last line drawn over it in the
   reference's order (pre-order nodes, draw_aabb's edge order). Lines are
   rasterised by Bresenham between the integer endpoints of world_to_screen
   (the reference leaves that to SDL's backend). Writes width * height RGBA8. */
int mirt_bvh_overlay(mirt_ctx *ctx, const mirt_camera *cam, int width, int height, int max_levels,
                     mirt_rgba8 *out);
/* get_camera_ray (ray.c:17-32) at n caller-given (u, v) pairs (uv[2i],
   uv[2i+1]), for a frame of width x height (the reference's compile-time
   WIDTH/HEIGHT, ray.c:18). */
int mirt_camera_rays_uv(mirt_ctx *ctx, const mirt_camera *cam, int width, int height, const float *uv, int n,
                        mirt_ray *out);

/* Reference-DFS work counters of one frame (instrumented kernel build,
   untimed): the algorithmic-bytes numerator of SURVEY §8(d). */
int mirt_count_frame(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd, mirt_counts *out);

/* Diagnostic: renders the frame with the instrumented kernel and writes, per
   8x8 tile (= wave), {tile, traversal loop steps, start, end} with start/end
   read from the 100 MHz s_memrealtime clock. Returns the number of waves
   (or -waves if cap is too small). */
int mirt_wave_stats(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd, uint32_t *out, int cap);

/* Diagnostic: renders the frame (depth >= 2, BVH, wavefront schedule) with the
   instrumented bounce kernel and writes 12 uint64 per bounce wave: loop
   iterations, walking lanes summed over them, the same two after the bounce
   queue ran dry, start / queue-dry / end time (100 MHz clock), longest
   chain << 32 | longest walk (steps) of the lane loop, quad-drain loop
   iterations, the time the quad drain began (0: none), lane-steps of the
   lane loop spent in DFS-segment fallbacks (a four-wide step whose pushes
   would overflow the LDS lane stack walks the node's subtree in DFS order)
   and the fallbacks entered. Returns the number of waves (or -waves if cap
   is too small). */
int mirt_bounce_stats(mirt_ctx *ctx, const mirt_camera *cam, const mirt_frame_desc *fd, uint64_t *out, int cap);

/* The ctx's own stream (a hipStream_t, non-blocking): the blocking calls run
   on it; a caller may pass it to mirt_render_frame_device. */
void *mirt_ctx_stream(mirt_ctx *ctx);

/* Device time (ms) of the last render kernel launched by a blocking call. */
float mirt_last_kernel_ms(mirt_ctx *ctx);

/* Device time (ms) of the two passes of the last frame this ctx launched
   with the wavefront schedule (blocking or _device call; waits for it):
   phase[0] = deferral mark + primary kernel (camera rays), phase[1] = the
   bounce kernel. Returns MIRT_E_INVALID if no wavefront frame was launched. */
int mirt_last_phase_ms(mirt_ctx *ctx, float *phase);
/* The same two times for each of the ctx's last min(max, 64) wavefront
   frames, oldest first (out[2j], out[2j + 1]), recorded by HIP events on the
   frame's own stream -- so frames that ran while other ctxs' frames shared
   the chip report their passes' durations under that overlap. Waits for
   them; returns the number of frames written. */
int mirt_phase_log(mirt_ctx *ctx, float *out, int max);

/* Kernel schedule knobs (results are identical under every setting; only
   speed changes). MIRT_OPT_TRAVERSAL: MIRT_TRAV_WAVEFRONT (default: camera-ray
   packets, then persistent per-lane bounce chains fed by a queue, for BVH
   frames of depth >= 2) or MIRT_TRAV_TILE (one kernel: each wave traces the
   whole paths of an 8x8 tile; always used for depth 1 and brute force).
   MIRT_OPT_FAST_SLAB: 1 (default) = reciprocal-multiply slab test with an
   exact-division fallback for undecidable boxes; 0 = the division-only slab
   test of hit.c:49-82 (and the reference DFS order everywhere).
   MIRT_OPT_BLOCK_WAVES: 8x8 pixel tiles (waves) per workgroup of the tile
   kernel: 1, 2, 4 (default) or 8. MIRT_OPT_DEFER: 1 (default) = on a tree
   that does not admit ordered walks, camera rays with a zero/tiny direction
   component are traced first, one per wave (node-parallel walk).
   MIRT_OPT_PRUNE: 1 (default) = with the fast slab test, skip subtrees whose
   box the ray provably enters beyond the best hit so far (the closest hit and
   its tie rule are unchanged; active only for a tree whose boxes enclose
   their subtrees, checked at upload); 0 = the reference's exhaustive DFS.
   MIRT_OPT_ORDERED: 1 (default) = with pruning, walks enter the nearer child
   first -- camera rays as packets over both-children nodes, bounce rays over
   a four-wide re-layout of the same tree (exact because the reference slab
   test is monotone under box containment); same closest hit, ties still go
   to the later DFS leaf; active only for a tree whose leaves hold increasing
   sphere indices in DFS order, as the reference's builds do, and depth < 63;
   0 = DFS order. */
enum { MIRT_OPT_TRAVERSAL = 1, MIRT_OPT_FAST_SLAB = 2, MIRT_OPT_BLOCK_WAVES = 3, MIRT_OPT_DEFER = 4,
       MIRT_OPT_BOUNCE_THRESHOLD = 5, /* wavefront: shade finished bounce rays once fewer than
                                         this many lanes of a wave still walk (0..64, default 20) */
       MIRT_OPT_PRUNE = 6, MIRT_OPT_ORDERED = 7,
       MIRT_OPT_BOUNCE_BLOCKS = 9,  /* wavefront: persistent bounce workgroups, 0 = occupancy x CUs
                                       (default: best for one frame at a time); with several contexts
                                       keeping frames in flight, ~1.5 per CU (384 on MI355X) */
       MIRT_OPT_QUAD_DRAIN = 11,    /* four-wide bounce walk: 1 (default) = once the queue is dry
                                       and <= 16 lanes of a wave are busy, finish them as quads */
       MIRT_OPT_LEAF_BATCH = 14,    /* four-wide bounce walk: load a step's passing leaf spheres
                                       together: 0 never, 1 always, 2 (default) when the tree's
                                       four-wide layout exceeds the chip's 32 MiB of L2;
                                       mirt_get_option reads back 0/1: in effect for the scene) */
       MIRT_OPT_QUAD_BATCH = 15,    /* mirt_intersect_rays / mirt_any_hit_rays with the BVH: 1
                                       (default) = a batch too small to fill the chip one ray per
                                       lane walks one ray per four lanes (benchmark.c's 10k rays) */
       MIRT_OPT_ZERO_COPY = 17,     /* frames of one sample into PAGE-LOCKED memory
                                       (mirt_host_alloc / mirt_host_register; the ctx's own
                                       accumulation): the frame kernels store every pixel
                                       straight into it instead of a DMA copy after them --
                                       1 (default) for the blocking mirt_render_frame, 2 for
                                       mirt_render_frame_async too, 0 never. Pageable memory:
                                       a copy. */
       MIRT_OPT_QUEUE_ORDER = 18,   /* wavefront: order of a frame's first bounces in the bounce
                                       queue -- 0 (default) = tile order for the blocking
                                       mirt_render_frame (a frame alone on the chip), grouped by
                                       direction octant per workgroup for frames in flight;
                                       1 = always grouped; 2 = always tile order. Speed only. */
       MIRT_OPT_DEBUG_STALL_MS = 19, /* test hook: every frame of this context starts behind a
                                       kernel that waits this many ms (0..10000, default 0), then
                                       exits -- a frame that overruns a caller's deadline
                                       (mirt_multi's MIRT_MULTI_OPT_TIMEOUT_MS) without a hang */ };
/* Traversal ids keep their first-release values (mirt 0.1: TILE 0, WAVEFRONT 5).
   ABI note: the mirt 0.2 header numbered WAVEFRONT 1; mirt_set_option accepts
   1 as a deprecated alias of MIRT_TRAV_WAVEFRONT (mirt_get_option reads back
   5), to be dropped in 1.0. The retired ids 2-4 (chunked / DFS-only schedules
   of mirt 0.1) and the retired option ids 8, 10, 12, 13, 20 (20: the bounce
   pass's continuation queue of mirt 0.5, measured slower and removed) return
   MIRT_E_INVALID. */
enum { MIRT_TRAV_TILE = 0, MIRT_TRAV_WAVEFRONT = 5, MIRT_TRAV_WAVEFRONT_V02 = 1 /* deprecated alias */ };
int mirt_set_option(mirt_ctx *ctx, int option, int value);
int mirt_get_option(mirt_ctx *ctx, int option);

#ifdef __cplusplus
}
#endif
#endif /* MIRT_H */
