/*
 * include/mirt_multi.h -- one renderer over several GPUs of a node, driven from
 * ONE host thread ("int mirt_init(int num_gpus)"; §8(e):
 * "shard by pixel-row tiles across the 8 GPUs ... RCCL gather").
 *
 * The reference renders a frame with one pixel loop on one core
 * (main.c:356-374 fresh, main.c:379-408 accumulating). Here every frame is
 * split by interleaved row blocks: block b (fd->row_block rows, default 8) goes
 * to rank b % n, so the dense centre rows spread over all GPUs. Each rank
 * renders its blocks into a compact slab in its own HBM with the single-GPU
 * kernels (scene replicated per device). Then, by default (gather), the slabs
 * go to rank 0 -- over RCCL (ncclGroupStart + ncclSend/ncclRecv, one
 * communicator per device from ncclCommInitAll) when the ranks are distinct
 * devices, or by device copies in "copy" mode -- a kernel on rank 0
 * de-interleaves them into the row-major frame, and one D2H copy delivers it.
 * With MIRT_MULTI_HOST_DIRECT every rank instead copies its row blocks
 * straight into the caller's host frame over its own host link (no exchange
 * between GPUs, no single link carrying the whole frame). Frames are
 * byte-identical to mirt_render_frame on one GPU whatever n and the delivery
 * are (the RNG contract keys on the full-frame pixel index).
 *
 * Frames in flight: `lanes` independent sets of per-rank contexts, slabs and
 * gather buffers. A launch (mirt_multi_render_frames_async) goes to lane
 * k % lanes after that lane's previous launch is waited for, so launch k + 1's
 * kernels start while launch k drains, gathers and copies; one launch may
 * carry several successive frames (each delivered to its own buffer), so the
 * bounce pass's latency tail is paid once per launch. With lanes > 1 every
 * context's persistent bounce pass takes 1.5 workgroups per CU
 * (MIRT_OPT_BOUNCE_BLOCKS) so the launches in flight share the chip;
 * MIRT_MULTI_FULL_GRID gives a launch that nothing follows the whole chip.
 * The lanes of a rank share ONE accumulation buffer (mirt_ctx_share_accum),
 * so the accumulating loop of main.c:379-408 stays exact in flight. Each
 * context has its own stream: set GPU_MAX_HW_QUEUES (e.g. 16) in the
 * environment before the HIP runtime starts so they get hardware queues.
 *
 * Errors: negative MIRT_E_* status, message in mirt_last_error(); an RCCL
 * failure is MIRT_E_DEVICE with ncclGetErrorString's text. No CPU path. No
 * call waits unboundedly: a lane whose work is not done after
 * MIRT_MULTI_OPT_TIMEOUT_MS fails the object (MIRT_E_DEVICE, the stuck
 * ranks named, every communicator aborted with ncclCommAbort); from then on
 * every call returns MIRT_E_DEVICE and mirt_multi_destroy releases only host
 * memory (device buffers of a possibly stuck GPU are left to process exit).
 *
 * Verification status: on one GPU the RCCL gather runs end to end with
 * MIRT_MULTI_OPT_GATHER_SELF (rank 0's slabs sent to itself) and in the
 * per-shard emulation (rank k > 0's send, rank 0's receives, as self
 * send/receive groups); tests/test_multi.py checks the received slabs and the
 * frames against the reference's golden frame and mirt_multi_get_stats'
 * counters. The n-GPU gather (sends from n devices' streams into rank 0) has
 * not run on a multi-GPU node yet. Copy mode with n same-device ranks
 * exercises the same geometry, strides and de-interleave.
 */
#ifndef MIRT_MULTI_H
#define MIRT_MULTI_H

#include "mirt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mirt_multi mirt_multi;

/* mirt_multi_create flags */
enum {
    MIRT_MULTI_COPY = 1,        /* gather by device copies (hipMemcpyPeerAsync) even when the devices are
                                   distinct; implied when a device repeats (RCCL refuses two ranks on one
                                   device): n ranks on one GPU render the same shards, so the frame geometry
                                   of an n-GPU node is testable on one */
    MIRT_MULTI_HOST_DIRECT = 2, /* frames delivered to host memory by every rank: rank r copies its row
                                   blocks of each frame straight into the caller's buffer (one strided DMA
                                   per frame from its own device); no gather to device 0 */
    MIRT_MULTI_QUEUE_AHEAD = 4  /* 2 x `lanes` launch slots over `lanes` context sets: slot l + lanes queues
                                   its kernels behind slot l's on the same contexts' streams (so a context
                                   starts its next launch the moment its last one's kernels end, with no
                                   host turnaround), renders into its own slabs, and delivers them on its
                                   context's copy stream (2 streams per context:
                                   give the process GPU_MAX_HW_QUEUES >= 2 x lanes); mirt_multi_lanes()
                                   then returns 2 x lanes */
};

/* mirt_multi_render_frames_async flags */
enum {
    MIRT_MULTI_FULL_GRID = 1    /* this launch's bounce passes take the full persistent grid (nothing will
                                   share the chip with them: the last launches of a known sequence) */
};

/* mirt_multi_set_option / mirt_multi_get_option: these, or any MIRT_OPT_* of
   mirt.h (applied to every context). */
enum {
    MIRT_MULTI_OPT_TIMEOUT_MS = 256,     /* bound of every wait, ms (default 60000; 0 = unbounded) */
    MIRT_MULTI_OPT_EMULATE_WORLD = 257,  /* measurement only, n == 1: the one rank plays shard
                                            EMULATE_RANK of a frame split EMULATE_WORLD ways -- its own
                                            render, its send, and as rank 0 also the other shards'
                                            receives, the de-interleave and the frame's D2H; the frames
                                            delivered are NOT complete. 0 or 1 = off (default) */
    MIRT_MULTI_OPT_EMULATE_RANK = 258,
    MIRT_MULTI_OPT_DIRECT_COPY = 259,    /* MIRT_MULTI_HOST_DIRECT: each rank's blocks of a frame as one strided
                                            copy (hipMemcpy2DAsync, 0, default), one copy per row block (1), or
                                            a kernel storing them into the mapped page-locked frame (2) */
    MIRT_MULTI_OPT_COPY_STREAM = 260,    /* MIRT_MULTI_QUEUE_AHEAD: a launch's copies on its context's stream
                                            behind its kernels (0, default) or on the context's copy stream (1);
                                            2: on the copy stream, and a launch is enqueued only once the
                                            kernels of the launch in its contexts' other slot have finished
                                            (one launch's kernels per context at a time; its copies still
                                            running). DESIGN §8 has the measurements */
    MIRT_MULTI_OPT_GATHER_SELF = 261,    /* gather delivery: 1 = rank 0's own slabs travel through the gather
                                            too (an RCCL send to itself, or a device copy in copy mode) instead
                                            of being read in place, so every slab of the frame takes one path
                                            -- with one GPU, the RCCL gather path end to end. 0 = off (default) */
    MIRT_MULTI_OPT_LEAD_SKIP = 262       /* 0..7: rank 0 renders a lighter share of every frame (it also
                                            receives, de-interleaves and delivers it in the gather): row blocks
                                            are dealt 8 rounds at a time, one per rank per round, and rank 0
                                            sits out this many rounds of every 8 (mirt_frame_desc.lead_skip);
                                            0 = block b to rank b % n; 8 (default) = automatic: the gather
                                            at n = 2 / 3-4 / 5-6 / 7+ ranks 0 / 1 / 2 / 3, host-direct 0.
                                            Frames are the same bytes whatever the value */
};

/* Counters of what the object issued since it was created (mirt_multi_get_stats). */
typedef struct mirt_multi_stats {
    uint64_t launches;      /* launches enqueued (mirt_multi_render_frames_async calls that succeeded) */
    uint64_t comm_inits;    /* ncclCommInitAll calls that succeeded (0 or 1) */
    uint64_t rccl_groups;   /* ncclGroupStart / ncclGroupEnd groups issued on rank 0 (one per gathered launch) */
    uint64_t rccl_sends;    /* ncclSend calls issued (every rank) */
    uint64_t rccl_recvs;    /* ncclRecv calls issued (rank 0) */
    uint64_t rccl_bytes;    /* bytes those receives carry */
    uint64_t device_copies; /* copy-mode gather copies (hipMemcpyAsync / hipMemcpyPeerAsync) */
} mirt_multi_stats;

/* n ranks on devices[0..n-1] (NULL: devices 0..n-1; n <= 64), `lanes` launches in
   flight (>= 1), flags MIRT_MULTI_*. With distinct devices and no
   MIRT_MULTI_COPY the gather runs over RCCL (ncclCommInitAll over the devices).
   mirt_init(n) of SURVEY §8(b) is mirt_multi_create(NULL, n, 1, 0, &m). */
int mirt_multi_create(const int *devices, int n, int lanes, int flags, mirt_multi **out);
void mirt_multi_destroy(mirt_multi *m);
/* Ranks (GPUs, or same-device shards), launch slots (lanes; 2 x lanes with
   MIRT_MULTI_QUEUE_AHEAD), the gather path ("rccl" or
   "copy"), the delivery ("gather" or "host-direct"), and 1 once the object has
   failed (0 otherwise). */
int mirt_multi_size(const mirt_multi *m);
int mirt_multi_lanes(const mirt_multi *m);
const char *mirt_multi_backend(const mirt_multi *m);
const char *mirt_multi_delivery(const mirt_multi *m);
int mirt_multi_failed(const mirt_multi *m);
/* The context of (lane, rank), e.g. for mirt_last_phase_ms; owned by m. */
mirt_ctx *mirt_multi_ctx(mirt_multi *m, int lane, int rank);
/* MIRT_MULTI_OPT_*, or mirt_set_option on every context. */
int mirt_multi_set_option(mirt_multi *m, int option, int value);
int mirt_multi_get_option(mirt_multi *m, int option);

/* mirt_scene_upload / mirt_scene_upload_flat to every context (the scene is
   replicated on every device; call after the build reordered the spheres). */
int mirt_multi_scene_upload(mirt_multi *m, const mirt_sphere *spheres, int num_spheres, const mirt_bvh_node *root);
int mirt_multi_scene_upload_flat(mirt_multi *m, const mirt_sphere *spheres, int num_spheres, const mirt_node *nodes,
                                 int num_nodes);

/* One launch of `nframes` successive frames (RNG samples fd->sample ..
   fd->sample + nframes - 1; accumulating: divisors fd->frames + j, as nframes
   successive calls) over all ranks, enqueued on the next lane after waiting for
   that lane's previous launch (whose outputs are then complete); returns at
   once. Frame j (width x height RGBA8, row-major) goes to outs[j], host memory
   (page-locked from mirt_host_alloc / mirt_host_register makes the copies DMA);
   outs NULL: the frames stay on the devices (gathered on device 0; with
   MIRT_MULTI_HOST_DIRECT, each rank's slabs). fd describes the whole frame:
   shard 0, num_shards 0 or 1; fd->row_block is the interleave block (0: 8);
   several frames need fd->samples <= 1. flags: MIRT_MULTI_FULL_GRID. The
   buffers must stay valid until mirt_multi_wait (or the lane's next launch)
   returns. */
int mirt_multi_render_frames_async(mirt_multi *m, const mirt_camera *cam, const mirt_frame_desc *fd, int nframes,
                                   int flags, mirt_rgba8 *const *outs);
/* The pixel loop of main.c:356-374 (fd->accumulate 0) / main.c:379-408
   (accumulate) over all ranks: one frame into `out`. Blocking. */
int mirt_multi_render_frame(mirt_multi *m, const mirt_camera *cam, const mirt_frame_desc *fd, mirt_rgba8 *out);
/* One frame, enqueued (mirt_multi_render_frames_async with nframes 1). */
int mirt_multi_render_frame_async(mirt_multi *m, const mirt_camera *cam, const mirt_frame_desc *fd,
                                  mirt_rgba8 *out);
/* Block until every launch on every lane has delivered its frames (bounded
   by MIRT_MULTI_OPT_TIMEOUT_MS). */
int mirt_multi_wait(mirt_multi *m);

/* The object's counters (struct above). */
int mirt_multi_get_stats(const mirt_multi *m, mirt_multi_stats *out);
/* Test hook (gather delivery, a frame split over > 1 shards or
   MIRT_MULTI_OPT_GATHER_SELF): after waiting for lane `lane` (-1: the lane of
   the last launch), copy shard `shard`'s display slab of frame `frame` of that
   launch, as it arrived in device 0's gather buffer -- the shard's compact rows
   (its row blocks in image order, width pixels each) -- into host `out`
   (`bytes` at least rows x width x 4). Blocking. */
int mirt_multi_read_gathered(mirt_multi *m, int lane, int shard, int frame, mirt_rgba8 *out, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* MIRT_MULTI_H */
