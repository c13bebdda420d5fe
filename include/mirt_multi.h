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
 * kernels (scene replicated per device), the slabs are gathered to rank 0 --
 * over RCCL (ncclGroupStart + ncclSend/ncclRecv, one communicator per device
 * from ncclCommInitAll) when the ranks are distinct devices, or by device
 * copies in "copy" mode -- a kernel on rank 0 de-interleaves them into the
 * row-major frame, and one D2H copy delivers it. Frames are byte-identical
 * to mirt_render_frame on one GPU whatever n is (the RNG contract keys on the
 * full-frame pixel index).
 *
 * Frames in flight: `lanes` independent sets of per-rank contexts, slabs and
 * gather buffers. mirt_multi_render_frame_async enqueues frame k on lane
 * k % lanes (after waiting for that lane's previous frame), so frame k + 1's
 * kernels start while frame k drains, gathers and copies. The lanes of a rank
 * share ONE accumulation buffer (mirt_ctx_share_accum), so the accumulating
 * loop of main.c:379-408 stays exact with frames in flight.
 *
 * Errors: negative MIRT_E_* status, message in mirt_last_error(); an RCCL
 * failure is MIRT_E_DEVICE with ncclGetErrorString's text. No CPU path.
 */
#ifndef MIRT_MULTI_H
#define MIRT_MULTI_H

#include "mirt.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct mirt_multi mirt_multi;

enum {
    MIRT_MULTI_COPY = 1  /* gather by device copies (hipMemcpyPeerAsync) even when the devices are
                            distinct; implied when a device repeats (RCCL refuses two ranks on one
                            device): n ranks on one GPU render the same shards, so the frame geometry
                            of an n-GPU node is testable on one */
};

/* n ranks on devices[0..n-1] (NULL: devices 0..n-1), `lanes` frames in flight
   (>= 1), flags MIRT_MULTI_*. With distinct devices and no MIRT_MULTI_COPY the
   gather runs over RCCL (ncclCommInitAll over the devices). mirt_init(n) of
   SURVEY §8(b) is mirt_multi_create(NULL, n, 1, 0, &m). */
int mirt_multi_create(const int *devices, int n, int lanes, int flags, mirt_multi **out);
void mirt_multi_destroy(mirt_multi *m);
/* Ranks (GPUs, or same-device shards), lanes, and the gather path: "rccl" or "copy". */
int mirt_multi_size(const mirt_multi *m);
int mirt_multi_lanes(const mirt_multi *m);
const char *mirt_multi_backend(const mirt_multi *m);
/* The context of (lane, rank), e.g. for mirt_last_phase_ms; owned by m. */
mirt_ctx *mirt_multi_ctx(mirt_multi *m, int lane, int rank);
/* mirt_set_option on every context. */
int mirt_multi_set_option(mirt_multi *m, int option, int value);

/* mirt_scene_upload / mirt_scene_upload_flat to every context (the scene is
   replicated on every device; call after the build reordered the spheres). */
int mirt_multi_scene_upload(mirt_multi *m, const mirt_sphere *spheres, int num_spheres, const mirt_bvh_node *root);
int mirt_multi_scene_upload_flat(mirt_multi *m, const mirt_sphere *spheres, int num_spheres, const mirt_node *nodes,
                                 int num_nodes);

/* The pixel loop of main.c:356-374 (fd->accumulate 0) / main.c:379-408
   (accumulate) over all ranks: writes the whole width x height RGBA8 frame,
   row-major, to host memory `out` (page-locked memory from mirt_host_alloc
   makes the copy a DMA). fd describes the whole frame: shard 0, num_shards 0
   or 1; fd->row_block is the interleave block (0: 8). Blocking. */
int mirt_multi_render_frame(mirt_multi *m, const mirt_camera *cam, const mirt_frame_desc *fd, mirt_rgba8 *out);
/* The same enqueued on the next lane (waiting first for that lane's previous
   frame, whose `out` is then complete); returns at once. `out` must stay
   valid until mirt_multi_wait (or the lane's next frame) returns. */
int mirt_multi_render_frame_async(mirt_multi *m, const mirt_camera *cam, const mirt_frame_desc *fd,
                                  mirt_rgba8 *out);
/* Block until every frame enqueued on every lane has reached host memory. */
int mirt_multi_wait(mirt_multi *m);

#ifdef __cplusplus
}
#endif
#endif /* MIRT_MULTI_H */
