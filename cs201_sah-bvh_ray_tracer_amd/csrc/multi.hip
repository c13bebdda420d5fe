// include/mirt_multi.h: one frame loop over the GPUs of a node from one host
// thread (SURVEY.md §8(b) mirt_init(num_gpus), §8(e) row-tile shard + RCCL
// gather). The reference's pixel loop (main.c:356-374 / 379-408) becomes, per
// frame: every rank renders its interleaved row blocks with the single-GPU
// kernels into a compact slab (render.hip, mirt::enqueue_frame_device), the
// slabs go to rank 0 -- one RCCL group of ncclSend / ncclRecv over
// communicators from ncclCommInitAll, or device copies in "copy" mode --
// deinterleave_kernel writes the row-major frame, and one D2H copy delivers it.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <new>
#include <vector>

#include "../../include/mirt_multi.h"
#include "internal.h"

using namespace mirt;

namespace {

// The gathered slabs (rank r's compact rows at gathered + r * slab_elems) ->
// the row-major frame. Image row y lies in row block b = y / rb, which rank
// b % n rendered as its compact row (b / n) * rb + y % rb (host_scene.cpp
// shard_row_count's geometry). One thread per pixel, rows across blockIdx.y:
// both sides are coalesced row segments.
__global__ void __launch_bounds__(256) deinterleave_kernel(const uint32_t* __restrict__ gathered,
                                                           uint32_t* __restrict__ frame, int width, int height,
                                                           int rb, int n, size_t slab_elems)
{
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    if (x >= width || y >= height) return;
    const int b = y / rb;
    const size_t row = (size_t)(b / n) * rb + y % rb;
    frame[(size_t)y * width + x] = gathered[(size_t)(b % n) * slab_elems + row * width + x];
}

int hip_err(hipError_t e, const char* what)
{
    set_error("%s: %s", what, hipGetErrorString(e));
    return MIRT_E_DEVICE;
}

int nccl_err(ncclResult_t r, const char* what)
{
    set_error("%s: %s", what, ncclGetErrorString(r));
    return MIRT_E_DEVICE;
}

#define MHIP(expr)                                        \
    do {                                                  \
        hipError_t e_ = (expr);                           \
        if (e_ != hipSuccess) return hip_err(e_, #expr);  \
    } while (0)
#define MNCCL(expr)                                       \
    do {                                                  \
        ncclResult_t r_ = (expr);                         \
        if (r_ != ncclSuccess) return nccl_err(r_, #expr); \
    } while (0)

// Device buffer on `dev` of at least `bytes` (grown, never shrunk).
int grow(int dev, uint32_t** p, size_t* cap, size_t bytes)
{
    if (bytes <= *cap) return MIRT_OK;
    MHIP(hipSetDevice(dev));
    if (*p) MHIP(hipFree(*p));
    *p = nullptr;
    *cap = 0;
    MHIP(hipMalloc((void**)p, bytes));
    *cap = bytes;
    return MIRT_OK;
}

// One frame in flight: a context per rank, the gather buffer and the frame
// on rank 0, and the copy-mode events.
struct Lane {
    std::vector<mirt_ctx*> ctx;       // rank r's context (device dev[r], its own stream)
    std::vector<hipEvent_t> rendered; // copy mode: rank r's slab is complete
    uint32_t* gathered = nullptr;     // rank 0: n slabs of slab_elems
    size_t gathered_cap = 0;
    uint32_t* frame = nullptr;        // rank 0: the de-interleaved frame
    size_t frame_cap = 0;
    bool pending = false;             // a frame was enqueued and not yet waited for
};

}  // namespace

struct mirt_multi {
    int n = 0;
    std::vector<int> dev;
    bool rccl = false;
    std::vector<ncclComm_t> comm;
    std::vector<Lane> lanes;
    int next = 0;
};

namespace {

hipStream_t stream_of(mirt_ctx* c) { return (hipStream_t)mirt_ctx_stream(c); }

int wait_lane(mirt_multi* m, Lane& L)
{
    if (!L.pending) return MIRT_OK;
    L.pending = false;
    for (int r = 0; r < m->n; r++) {
        MHIP(hipSetDevice(m->dev[r]));
        MHIP(hipStreamSynchronize(stream_of(L.ctx[r])));
    }
    return MIRT_OK;
}

// Frame k on lane L: every rank's shard, the gather to rank 0, the
// de-interleave and the D2H copy into `out`, all enqueued.
int enqueue(mirt_multi* m, Lane& L, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out)
{
    const int n = m->n;
    mirt_frame_desc sd = *fd;
    sd.row_block = fd->row_block > 0 ? fd->row_block : 8;
    sd.num_shards = n;
    // the widest shard (rank 0's: it holds the first block) sets the slab stride
    sd.shard = 0;
    const size_t slab_elems = (size_t)shard_row_count(&sd) * fd->width;
    const int dev0 = m->dev[0];
    int rc = grow(dev0, &L.gathered, &L.gathered_cap, 4 * slab_elems * n + 4);
    if (!rc && n > 1) rc = grow(dev0, &L.frame, &L.frame_cap, 4 * (size_t)fd->width * fd->height + 4);
    if (rc) return rc;
    // rank r renders its row blocks: its `samples` slabs in the ctx's own
    // buffer (the display is the last), with its (lane-shared) accumulation
    std::vector<uint32_t*> disp(n, nullptr);
    std::vector<size_t> elems(n, 0);
    for (int r = 0; r < n; r++) {
        sd.shard = r;
        elems[r] = (size_t)shard_row_count(&sd) * fd->width;
        rc = enqueue_frame_device(L.ctx[r], cam, &sd, nullptr, &disp[r], "mirt_multi_render_frame");
        if (rc) return rc;
    }
    hipStream_t s0 = stream_of(L.ctx[0]);
    if (m->rccl) {
        // one group: every rank (rank 0 included, a self send/recv, so every
        // slab takes one path) sends its display slab to rank 0, which
        // receives slab r at gathered + r * slab_elems; each op on the stream
        // that rendered it, so it starts when that rank's frame is done
        MNCCL(ncclGroupStart());
        for (int r = 0; r < n; r++) {
            ncclResult_t e = ncclSend(disp[r], elems[r], ncclUint32, 0, m->comm[r], stream_of(L.ctx[r]));
            if (e == ncclSuccess)
                e = ncclRecv(L.gathered + (size_t)r * slab_elems, elems[r], ncclUint32, r, m->comm[0], s0);
            if (e != ncclSuccess) {
                (void)ncclGroupEnd();
                return nccl_err(e, "mirt_multi_render_frame: ncclSend/ncclRecv");
            }
        }
        MNCCL(ncclGroupEnd());
    } else {
        // copy mode: rank 0's stream waits for each rank's frame, then copies
        // its slab (peer-to-peer across devices, device-local otherwise)
        for (int r = 0; r < n; r++) {
            if (r > 0) {
                MHIP(hipSetDevice(m->dev[r]));
                MHIP(hipEventRecord(L.rendered[r], stream_of(L.ctx[r])));
                MHIP(hipSetDevice(dev0));
                MHIP(hipStreamWaitEvent(s0, L.rendered[r], 0));
            }
            MHIP(hipSetDevice(dev0));
            uint32_t* dst = L.gathered + (size_t)r * slab_elems;
            if (m->dev[r] == dev0)
                MHIP(hipMemcpyAsync(dst, disp[r], 4 * elems[r], hipMemcpyDeviceToDevice, s0));
            else
                MHIP(hipMemcpyPeerAsync(dst, dev0, disp[r], m->dev[r], 4 * elems[r], s0));
        }
    }
    MHIP(hipSetDevice(dev0));
    const uint32_t* src = L.gathered;   // n == 1: the one slab is the frame
    if (n > 1) {
        const dim3 grid((fd->width + 255) / 256, fd->height);
        deinterleave_kernel<<<grid, 256, 0, s0>>>(L.gathered, L.frame, fd->width, fd->height, sd.row_block, n,
                                                  slab_elems);
        MHIP(hipGetLastError());
        src = L.frame;
    }
    MHIP(hipMemcpyAsync(out, src, 4 * (size_t)fd->width * fd->height, hipMemcpyDeviceToHost, s0));
    L.pending = true;
    return MIRT_OK;
}

bool multi_ok(mirt_multi* m, const char* fn)
{
    if (!m) set_error("%s: null mirt_multi", fn);
    return m != nullptr;
}

int check_frame(const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out, const char* fn)
{
    if (!cam || !fd || !out || fd->shard != 0 || fd->num_shards > 1 || fd->num_shards < 0 || fd->row_block < 0) {
        set_error("%s: invalid arguments (fd describes the whole frame: shard 0, num_shards 0 or 1)", fn);
        return MIRT_E_INVALID;
    }
    mirt_frame_desc whole = *fd;
    whole.num_shards = 1;
    whole.row_block = fd->row_block > 0 ? fd->row_block : 8;
    if (!frame_desc_valid(&whole)) {
        set_error("%s: invalid frame descriptor", fn);
        return MIRT_E_INVALID;
    }
    return MIRT_OK;
}

}  // namespace

extern "C" {

int mirt_multi_create(const int* devices, int n, int lanes, int flags, mirt_multi** out)
try {
    if (!out || n <= 0 || lanes <= 0 || (flags & ~MIRT_MULTI_COPY)) {
        set_error("mirt_multi_create: invalid arguments");
        return MIRT_E_INVALID;
    }
    *out = nullptr;
    int have = 0;
    MHIP(hipGetDeviceCount(&have));
    mirt_multi* m = new mirt_multi();
    m->n = n;
    for (int r = 0; r < n; r++) m->dev.push_back(devices ? devices[r] : r);
    bool distinct = true;
    for (int r = 0; r < n; r++) {
        if (m->dev[r] < 0 || m->dev[r] >= have) {
            set_error("mirt_multi_create: device %d not present (%d visible)", m->dev[r], have);
            delete m;
            return MIRT_E_INVALID;
        }
        for (int q = 0; q < r; q++) distinct = distinct && m->dev[q] != m->dev[r];
    }
    m->rccl = distinct && !(flags & MIRT_MULTI_COPY);
    auto fail = [&](int rc) {
        mirt_multi_destroy(m);
        return rc;
    };
    if (m->rccl) {
        m->comm.assign(n, nullptr);
        ncclResult_t e = ncclCommInitAll(m->comm.data(), n, m->dev.data());
        if (e != ncclSuccess) {
            m->comm.clear();
            return fail(nccl_err(e, "mirt_multi_create: ncclCommInitAll"));
        }
    } else {
        // copy mode across distinct devices: direct peer copies where the
        // link allows (the runtime stages them otherwise)
        for (int r = 1; r < n; r++) {
            if (m->dev[r] == m->dev[0]) continue;
            int can = 0;
            if (hipDeviceCanAccessPeer(&can, m->dev[0], m->dev[r]) == hipSuccess && can) {
                (void)hipSetDevice(m->dev[0]);
                (void)hipDeviceEnablePeerAccess(m->dev[r], 0);   // already enabled is fine
                (void)hipGetLastError();
            }
        }
    }
    m->lanes.resize(lanes);
    for (int l = 0; l < lanes; l++) {
        Lane& L = m->lanes[l];
        L.ctx.assign(n, nullptr);
        L.rendered.assign(n, nullptr);
        for (int r = 0; r < n; r++) {
            int rc = mirt_create(m->dev[r], &L.ctx[r]);
            if (rc) return fail(rc);
            (void)hipSetDevice(m->dev[r]);
            hipError_t e = hipEventCreateWithFlags(&L.rendered[r], hipEventDisableTiming);
            if (e != hipSuccess) return fail(hip_err(e, "mirt_multi_create: hipEventCreate"));
            // the lanes of a rank keep ONE accumulation buffer: frames in
            // flight of the accumulating loop (main.c:379-408) fold in order
            if (l > 0) {
                rc = mirt_ctx_share_accum(L.ctx[r], m->lanes[0].ctx[r]);
                if (rc) return fail(rc);
            }
        }
    }
    *out = m;
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    set_error("mirt_multi_create: out of host memory");
    return MIRT_E_NOMEM;
}

void mirt_multi_destroy(mirt_multi* m)
{
    if (!m) return;
    for (Lane& L : m->lanes) (void)wait_lane(m, L);
    for (Lane& L : m->lanes) {
        for (int r = 0; r < (int)L.ctx.size(); r++) {
            if (L.rendered[r]) {
                (void)hipSetDevice(m->dev[r]);
                (void)hipEventDestroy(L.rendered[r]);
            }
            mirt_destroy(L.ctx[r]);
        }
        (void)hipSetDevice(m->dev[0]);
        if (L.gathered) (void)hipFree(L.gathered);
        if (L.frame) (void)hipFree(L.frame);
    }
    for (ncclComm_t c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    delete m;
}

int mirt_multi_size(const mirt_multi* m) { return m ? m->n : MIRT_E_INVALID; }
int mirt_multi_lanes(const mirt_multi* m) { return m ? (int)m->lanes.size() : MIRT_E_INVALID; }
const char* mirt_multi_backend(const mirt_multi* m) { return !m ? "" : m->rccl ? "rccl" : "copy"; }

mirt_ctx* mirt_multi_ctx(mirt_multi* m, int lane, int rank)
{
    if (!m || lane < 0 || lane >= (int)m->lanes.size() || rank < 0 || rank >= m->n) return nullptr;
    return m->lanes[lane].ctx[rank];
}

int mirt_multi_set_option(mirt_multi* m, int option, int value)
{
    if (!multi_ok(m, "mirt_multi_set_option")) return MIRT_E_INVALID;
    for (Lane& L : m->lanes)
        for (mirt_ctx* c : L.ctx)
            if (int rc = mirt_set_option(c, option, value)) return rc;
    return MIRT_OK;
}

int mirt_multi_scene_upload(mirt_multi* m, const mirt_sphere* spheres, int num_spheres, const mirt_bvh_node* root)
{
    if (!multi_ok(m, "mirt_multi_scene_upload")) return MIRT_E_INVALID;
    for (Lane& L : m->lanes)
        if (int rc = wait_lane(m, L)) return rc;
    for (Lane& L : m->lanes)
        for (mirt_ctx* c : L.ctx)
            if (int rc = mirt_scene_upload(c, spheres, num_spheres, root)) return rc;
    return MIRT_OK;
}

int mirt_multi_scene_upload_flat(mirt_multi* m, const mirt_sphere* spheres, int num_spheres, const mirt_node* nodes,
                                 int num_nodes)
{
    if (!multi_ok(m, "mirt_multi_scene_upload_flat")) return MIRT_E_INVALID;
    for (Lane& L : m->lanes)
        if (int rc = wait_lane(m, L)) return rc;
    for (Lane& L : m->lanes)
        for (mirt_ctx* c : L.ctx)
            if (int rc = mirt_scene_upload_flat(c, spheres, num_spheres, nodes, num_nodes)) return rc;
    return MIRT_OK;
}

int mirt_multi_render_frame_async(mirt_multi* m, const mirt_camera* cam, const mirt_frame_desc* fd,
                                  mirt_rgba8* out)
{
    if (!multi_ok(m, "mirt_multi_render_frame_async")) return MIRT_E_INVALID;
    if (int rc = check_frame(cam, fd, out, "mirt_multi_render_frame_async")) return rc;
    Lane& L = m->lanes[m->next];
    if (int rc = wait_lane(m, L)) return rc;
    m->next = (m->next + 1) % (int)m->lanes.size();
    return enqueue(m, L, cam, fd, out);
}

int mirt_multi_render_frame(mirt_multi* m, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out)
{
    if (!multi_ok(m, "mirt_multi_render_frame")) return MIRT_E_INVALID;
    if (int rc = check_frame(cam, fd, out, "mirt_multi_render_frame")) return rc;
    Lane& L = m->lanes[m->next];
    if (int rc = wait_lane(m, L)) return rc;
    m->next = (m->next + 1) % (int)m->lanes.size();
    if (int rc = enqueue(m, L, cam, fd, out)) return rc;
    return wait_lane(m, L);
}

int mirt_multi_wait(mirt_multi* m)
{
    if (!multi_ok(m, "mirt_multi_wait")) return MIRT_E_INVALID;
    for (Lane& L : m->lanes)
        if (int rc = wait_lane(m, L)) return rc;
    return MIRT_OK;
}

}  // extern "C"
