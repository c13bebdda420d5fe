// include/mirt_multi.h: one frame loop over the GPUs of a node from one host
// thread (SURVEY.md §8(b) mirt_init(num_gpus), §8(e) row-tile shard + RCCL
// gather). The reference's pixel loop (main.c:356-374 / 379-408) becomes, per
// launch of `nframes` successive frames: every rank renders its interleaved
// row blocks of all of them with the single-GPU kernels into compact slabs
// (render.hip, mirt::enqueue_frame_device), then either
//   gather (default): the slabs go to rank 0 -- one RCCL group of ncclSend /
//     ncclRecv over communicators from ncclCommInitAll, or device copies in
//     "copy" mode -- deinterleave_kernel writes the row-major frames and one
//     D2H copy per frame delivers them; or
//   host-direct (MIRT_MULTI_HOST_DIRECT): every rank copies its row blocks
//     straight into the host frames (one strided DMA per frame over its own
//     host link), no exchange between GPUs.
// `lanes` sets of contexts keep launches in flight. Every wait is bounded
// (MIRT_MULTI_OPT_TIMEOUT_MS): a lane that does not finish fails the object
// with the stuck rank named and the communicators aborted, never a hang.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <memory>
#include <mutex>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mirt_multi.h"
#include "internal.h"
#include "shard.h"

using namespace mirt;

namespace {

constexpr int kMaxShards = 64;  // shards of one frame (ranks, or the emulated world)
// The frame's D2H is issued as a 2D copy (H rows of W pixels, the path the
// host-direct copies take): the runtime runs it on a DMA engine, where a 1D
// copy of the same bytes ran as a blit kernel on the context's compute queue
// for most frames (14 of 20 in the timed loop's trace), taking CU time from
// the frames in flight. Measured (profiles/r05_logs/r05av/): N = 1
// host-inclusive 2,477-2,525 -> 2,543-2,572 Mrays/s, depth 1 6,775-6,930 ->
// 8,431-8,455.

// Where every shard's displays are (kernel argument of deinterleave_kernel):
// shard s's `nframes` displays at p[s], frame j at + j * rows[s] * width --
// rank 0's own slabs in place, the other shards' in the gather buffer.
struct ShardSrc {
    const uint32_t* p[kMaxShards];
    int rows[kMaxShards];
};

// The shards' slabs -> the row-major frames. Image row y lies in row block
// b = y / rb, which its owner shard s rendered as compact row c * rb + y % rb
// (shard.h block_owner: b % n, or the lead-skip weighting). One thread per
// pixel, rows across blockIdx.y, frames across blockIdx.z: both sides are
// coalesced row segments.
__global__ void __launch_bounds__(256) deinterleave_kernel(ShardSrc src, uint32_t* __restrict__ frames, int width,
                                                           int height, int rb, int n, int lead_skip)
{
    const int x = blockIdx.x * 256 + threadIdx.x;
    const int y = blockIdx.y;
    const int j = blockIdx.z;
    if (x >= width || y >= height) return;
    int s, c;
    block_owner(y / rb, n, lead_skip, s, c);
    const size_t row = (size_t)c * rb + y % rb;
    frames[((size_t)j * height + y) * width + x] = src.p[s][((size_t)j * src.rows[s] + row) * width + x];
}

// MIRT_MULTI_OPT_DIRECT_COPY 2: shard s's compact rows straight into the
// row-major host frame (device-visible address of page-locked memory) by a
// kernel, 16 B per thread, instead of a strided DMA: compact row r is image
// row shard_block(s, r / rb) * rb + r % rb (shard.h; the image's short last
// block lies at the slab's end).
__global__ void __launch_bounds__(256) scatter_rows_kernel(const uint32_t* __restrict__ slab,
                                                           uint32_t* __restrict__ frame, int width, int rows,
                                                           int rb, int world, int s, int lead_skip)
{
    const int r = blockIdx.y;
    const int x = (int)(blockIdx.x * 256 + threadIdx.x) * 4;
    if (r >= rows || x >= width) return;
    const int y = shard_block(s, r / rb, world, lead_skip) * rb + r % rb;
    const uint32_t* src = slab + (size_t)r * width + x;
    uint32_t* dst = frame + (size_t)y * width + x;
    if (x + 4 <= width && (((uintptr_t)src | (uintptr_t)dst) & 15) == 0) {
        *(uint4*)dst = *(const uint4*)src;
    } else {
        for (int i = 0; i < 4 && x + i < width; i++) dst[i] = src[i];
    }
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

// What one launch asks of every rank (set by the caller's thread before the
// ranks issue it; read-only while they do).
struct Launch {
    mirt_camera cam;
    mirt_frame_desc sd;             // shard geometry of the frame (num_shards = world), samples = spp * nframes
    int nframes = 1, flags = 0, world = 1, W = 0, H = 0, rb = 8;
    bool emu = false, gather = false, rank0_assembles = false, deliver = false;
    bool self = false;              // MIRT_MULTI_OPT_GATHER_SELF: rank 0's own slabs into its slot too
    ShardSrc sr{};                  // rows of every shard (p[] filled by rank 0)
    size_t shard_stride = 0, frame_elems = 0;
    std::vector<mirt_rgba8*> dst;   // frame j's host destination (page-locked: the caller's or the staging)
};

// One launch in flight: a context per rank, the gather buffer and the frames
// on rank 0, the copy-mode events and each rank's completion event.
struct Lane {
    std::vector<mirt_ctx*> ctx;       // rank r's context (device dev[r], its own stream)
    bool owns_ctx = true;             // MIRT_MULTI_QUEUE_AHEAD: lanes l and l + contexts share lane l's contexts
    std::vector<hipEvent_t> rendered; // copy mode: rank r's slabs are complete
    std::vector<hipEvent_t> done;     // rank r: the launch's last operation (on the copy stream with QUEUE_AHEAD)
    // MIRT_MULTI_QUEUE_AHEAD: this lane's own display slabs per rank (the
    // context's stream renders the next lane's launch into ITS slabs while
    // this one's copies run), the copy stream and the event it waits on
    std::vector<uint32_t*> slab;
    std::vector<size_t> slab_cap;
    std::vector<hipStream_t> cstream;
    std::vector<hipEvent_t> kdone;
    std::vector<char> kdone_set;      // rank r's copy stream already waits for this launch (rank r's thread only)
    uint32_t* gathered = nullptr;     // rank 0: every shard's displays
    size_t gathered_cap = 0;
    uint32_t* frame = nullptr;        // rank 0: the de-interleaved frames
    size_t frame_cap = 0;
    // a launch was (possibly partly) enqueued and not yet waited for: set
    // before the first enqueue, cleared only once every rank's work is done
    bool pending = false;
    // outputs in pageable memory: a copy into them would block the enqueuing
    // thread behind the frame (no bounded wait), so the frames land in this
    // page-locked staging area and are copied out once the lane is waited for
    uint8_t* stage = nullptr;
    size_t stage_cap = 0;
    struct Deferred {
        void* dst;
        const void* src;
        size_t bytes;
    };
    std::vector<Deferred> deferred;
    Launch job;
    // the ranks' issue of the current launch (rank threads): ranks done issuing,
    // and copy mode's hand-over of each rank's slabs to rank 0
    std::unique_ptr<std::atomic<int>> issued{new std::atomic<int>(0)};
    std::vector<std::unique_ptr<std::atomic<uint64_t>>> slabs_ready;   // launch number whose `rendered[r]` is recorded
    std::vector<uint32_t*> src;       // rank r's first display slab of the current launch
    uint64_t seq = 0;                 // launch number on this lane
    std::unique_ptr<std::mutex> err_mu{new std::mutex};
    int err = MIRT_OK;                // first issue error of the current launch
    std::string err_msg;
};

// One host thread per rank (n > 1): the caller's thread prepares a launch and
// hands it to every rank's thread, which issues that rank's part on its own
// device -- so N GPUs are fed by N threads, not one, and rank r's first
// launch does not wait behind ranks 0 .. r - 1's (one host
// thread calls; inside, one stream per GPU).
struct RankThread {
    std::thread th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<int> q;                // lanes to issue, in launch order
    bool stop = false;
};

}  // namespace

struct mirt_multi {
    int n = 0;
    int nctx = 0;                     // context sets (the `lanes` argument)
    bool ahead = false;               // MIRT_MULTI_QUEUE_AHEAD: 2 x nctx lanes, two launches per context
    int ahead_copy_stream = 0;        // MIRT_MULTI_OPT_COPY_STREAM: the copies on the context's copy stream
    std::vector<int> dev;
    bool rccl = false;
    bool direct = false;              // MIRT_MULTI_HOST_DIRECT
    std::vector<ncclComm_t> comm;
    std::vector<Lane> lanes;
    std::vector<std::unique_ptr<RankThread>> workers;   // n > 1
    int next = 0;
    int timeout_ms = 60000;           // MIRT_MULTI_OPT_TIMEOUT_MS (0: unbounded)
    int emu_world = 0, emu_rank = 0;  // MIRT_MULTI_OPT_EMULATE_*: this one rank plays shard emu_rank of emu_world
    int direct_copy = 0;              // MIRT_MULTI_OPT_DIRECT_COPY: 0 one strided copy per frame, 1 one per row block
    int lead_skip = kLeadRounds;      // MIRT_MULTI_OPT_LEAD_SKIP: shard 0's lighter share (shard.h); 8 automatic
    bool gather_self = false;         // MIRT_MULTI_OPT_GATHER_SELF: rank 0's own slabs travel through the gather too
    int last_lane = -1;               // lane of the last launch enqueued
    // a wait timed out or a device call failed: every call returns fail_msg;
    // read by the rank threads before every issue and every RCCL call
    std::atomic<bool> failed{false};
    std::string fail_msg;
    // rank r's RCCL calls hold comm_mu[r]; fail_multi takes it before aborting
    // the communicator, so no rank thread is between its `failed` check and
    // its call when the communicator goes
    std::vector<std::unique_ptr<std::timed_mutex>> comm_mu;
    // mirt_multi_get_stats
    std::atomic<uint64_t> st_launches{0}, st_comm_inits{0}, st_groups{0}, st_sends{0}, st_recvs{0}, st_bytes{0},
        st_copies{0};
};

namespace {

hipStream_t stream_of(mirt_ctx* c) { return (hipStream_t)mirt_ctx_stream(c); }

// The lead-skip weighting of a frame split `world` ways (shard.h): the
// option's value, or by default (kLeadRounds: automatic) a lighter share for
// rank 0 in the gather only -- it also receives, de-interleaves and delivers
// the frame. Measured (per-shard emulation, frames gathered on GPU 0,
// MEASUREMENTS.md §D): N = 8 lead skip 0 / 2 / 3 / 4 -> 10.3 / 12.4 / 15.7 /
// 13.8-15.1 G rays/s (at 3 rank 0 0.10 ms per frame, ranks 1-7 0.126-0.132);
// N = 4: skip 1 8.0 G (rank 0 0.240 vs 0.25-0.26 ms), skip 2 7.9 G; N = 2:
// skip 0 4.3 G, skip 1 4.2 G. Rank 0's exchange costs about the same per
// frame at any N while the render share shrinks with N, so the skip grows
// with N.
int lead_skip_for(const mirt_multi* m, int world, bool gather)
{
    if (world <= 1) return 0;
    if (m->lead_skip < kLeadRounds) return m->lead_skip;
    if (!gather) return 0;
    return world <= 2 ? 0 : world <= 4 ? 1 : world <= 6 ? 2 : 3;
}

int failed_status(const mirt_multi* m, const char* fn)
{
    set_error("%s: %s", fn, m->fail_msg.c_str());
    return MIRT_E_DEVICE;
}

// The object cannot go on: abort the communicators (an RCCL kernel stuck on a
// peer polls the abort flag and exits), remember why, and fail from now on.
// Called on the caller's thread only (the waits). The rank threads see
// `failed` before their next issue and before every RCCL call, and stop
// issuing; a rank thread still inside an RCCL call (holding comm_mu[r] past
// the grace period: stuck on a peer) is released by the abort itself. The
// communicator handles stay set (never used again; a failed object's destroy
// does not destroy them).
int fail_multi(mirt_multi* m, const std::string& why)
{
    m->fail_msg = why;
    m->failed.store(true, std::memory_order_seq_cst);
    for (Lane& L : m->lanes) L.deferred.clear();
    for (size_t r = 0; r < m->comm.size(); r++) {
        if (!m->comm[r]) continue;
        std::unique_lock<std::timed_mutex> lk(*m->comm_mu[r], std::defer_lock);
        (void)lk.try_lock_for(std::chrono::milliseconds(200));
        (void)ncclCommAbort(m->comm[r]);
    }
    set_error("%s", why.c_str());
    return MIRT_E_DEVICE;
}

// Wait for lane `li`'s launch on every rank: every rank thread has issued
// it, then each rank's completion event, polled against the deadline (no
// unbounded hipStreamSynchronize). An issue error is returned once the work
// that did reach the streams has finished.
int wait_lane(mirt_multi* m, int li)
{
    if (m->failed) return failed_status(m, "mirt_multi");
    Lane& L = m->lanes[li];
    if (!L.pending) return MIRT_OK;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto over = [&]() {
        return m->timeout_ms > 0 && std::chrono::duration<double, std::milli>(clk::now() - t0).count() > m->timeout_ms;
    };
    for (long polls = 0; L.issued->load(std::memory_order_acquire) < m->n; polls++) {
        if (over())
            return fail_multi(m, "lane " + std::to_string(li) + ": the rank threads did not issue the launch within " +
                                     std::to_string(m->timeout_ms) + " ms (MIRT_MULTI_OPT_TIMEOUT_MS); communicators "
                                     "aborted, the object is unusable");
        if (polls < 2000)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    for (int r = 0; r < m->n; r++) {
        for (long polls = 0;; polls++) {
            const hipError_t e = hipEventQuery(L.done[r]);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) {
                (void)hipGetLastError();
                return fail_multi(m, std::string("rank ") + std::to_string(r) + " (device " +
                                         std::to_string(m->dev[r]) + "): " + hipGetErrorString(e));
            }
            if (over()) {
                std::string stuck;
                for (int q = r; q < m->n; q++)
                    if (hipEventQuery(L.done[q]) == hipErrorNotReady)
                        stuck += (stuck.empty() ? "" : ", ") + std::to_string(q) + " (device " +
                                 std::to_string(m->dev[q]) + ")";
                (void)hipGetLastError();
                return fail_multi(m, "lane " + std::to_string(li) + " not done after " +
                                         std::to_string(m->timeout_ms) + " ms (MIRT_MULTI_OPT_TIMEOUT_MS); stuck rank(s) " +
                                         stuck + "; communicators aborted, the object is unusable");
            }
            // spin briefly (a frame in flight is usually about to end), then
            // give the core back between polls
            if (polls < 2000)
                std::this_thread::yield();
            else
                std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    L.pending = false;
    if (L.err) {
        const int rc = L.err;
        set_error("%s", L.err_msg.c_str());
        L.err = MIRT_OK;
        L.deferred.clear();
        return rc;
    }
    for (const Lane::Deferred& d : L.deferred) std::memcpy(d.dst, d.src, d.bytes);
    L.deferred.clear();
    return MIRT_OK;
}

// MIRT_MULTI_OPT_COPY_STREAM 2: before a launch on lane li, the KERNELS of
// the launch in the same contexts' other slot must have finished (its copies
// may still run on the copy streams): one launch's kernels per context at a
// time, as without QUEUE_AHEAD, but a frame's D2H no longer holds its context.
int wait_sibling_kernels(mirt_multi* m, int li)
{
    const int sib = li < m->nctx ? li + m->nctx : li - m->nctx;
    Lane& S = m->lanes[sib];
    if (!S.pending) return MIRT_OK;
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    auto over = [&]() {
        return m->timeout_ms > 0 && std::chrono::duration<double, std::milli>(clk::now() - t0).count() > m->timeout_ms;
    };
    for (long polls = 0; S.issued->load(std::memory_order_acquire) < m->n; polls++) {
        if (over()) return fail_multi(m, "lane " + std::to_string(sib) + ": the rank threads did not issue the launch");
        if (polls < 2000)
            std::this_thread::yield();
        else
            std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
    for (int r = 0; r < m->n; r++) {
        if (!S.kdone_set[r]) continue;
        for (long polls = 0;; polls++) {
            const hipError_t e = hipEventQuery(S.kdone[r]);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) {
                (void)hipGetLastError();
                return fail_multi(m, std::string("rank ") + std::to_string(r) + ": " + hipGetErrorString(e));
            }
            if (over())
                return fail_multi(m, "lane " + std::to_string(sib) + " kernels not done after " +
                                         std::to_string(m->timeout_ms) + " ms (MIRT_MULTI_OPT_TIMEOUT_MS)");
            if (polls < 2000)
                std::this_thread::yield();
            else
                std::this_thread::sleep_for(std::chrono::microseconds(50));
        }
    }
    return MIRT_OK;
}

int communicators(mirt_multi* m)
{
    if (!m->comm.empty()) return MIRT_OK;
    m->comm.assign(m->n, nullptr);
    const ncclResult_t e = ncclCommInitAll(m->comm.data(), m->n, m->dev.data());
    if (e != ncclSuccess) {
        m->comm.clear();
        return nccl_err(e, "mirt_multi: ncclCommInitAll");
    }
    m->st_comm_inits.fetch_add(1);
    return MIRT_OK;
}

// The caller's part of a launch on lane L: the geometry, rank 0's buffers,
// where every frame lands. Then the ranks issue it (issue_rank).
int prepare(mirt_multi* m, Lane& L, const mirt_camera* cam, const mirt_frame_desc* fd, int nframes, int flags,
            mirt_rgba8* const* outs)
{
    Launch& J = L.job;
    J.cam = *cam;
    J.nframes = nframes;
    J.flags = flags;
    J.emu = m->emu_world > 1;
    J.world = J.emu ? m->emu_world : m->n;   // shards of the frame
    J.W = fd->width;
    J.H = fd->height;
    const int spp = std::max(1, fd->samples);
    J.sd = *fd;
    J.sd.row_block = fd->row_block > 0 ? fd->row_block : 8;
    J.sd.num_shards = J.world;
    J.sd.samples = spp * nframes;
    J.sd.lead_skip = lead_skip_for(m, J.world, !m->direct);
    J.rb = J.sd.row_block;
    J.sr = ShardSrc{};
    mirt_frame_desc g = J.sd;
    int most = 0;
    for (int s = 0; s < J.world; s++) {
        g.shard = s;
        J.sr.rows[s] = shard_row_count(&g);
        most = std::max(most, J.sr.rows[s]);
    }
    J.shard_stride = (size_t)most * J.W * nframes;   // every shard's slot in the gather buffer
    J.frame_elems = (size_t)J.W * J.H;
    J.gather = !m->direct;                                     // frames to device 0
    J.rank0_assembles = J.gather && (!J.emu || m->emu_rank == 0);
    J.deliver = outs != nullptr;
    J.self = J.gather && m->gather_self;
    if (J.gather && (J.world > 1 || J.self)) {
        int rc = grow(m->dev[0], &L.gathered, &L.gathered_cap, 4 * J.shard_stride * J.world + 4);
        if (!rc && J.rank0_assembles) rc = grow(m->dev[0], &L.frame, &L.frame_cap, 4 * J.frame_elems * nframes + 4);
        if (rc) return rc;
    }
    if (m->rccl && J.gather && (m->n > 1 || J.emu || m->gather_self))
        if (int rc = communicators(m)) return rc;
    // where frame j lands: the caller's buffer if it is page-locked, else
    // the lane's staging area (copied out by wait_lane)
    J.dst.assign(nframes, nullptr);
    L.deferred.clear();
    if (outs) {
        const size_t fb = 4 * J.frame_elems;
        for (int j = 0; j < nframes; j++) {
            if (host_page_locked(outs[j], fb)) {
                J.dst[j] = outs[j];
                continue;
            }
            if (L.stage_cap < fb * nframes) {
                if (L.stage) MHIP(hipHostFree(L.stage));
                L.stage = nullptr;
                L.stage_cap = 0;
                MHIP(hipHostMalloc((void**)&L.stage, fb * nframes, hipHostMallocPortable));
                L.stage_cap = fb * nframes;
            }
            J.dst[j] = (mirt_rgba8*)(L.stage + fb * j);
            L.deferred.push_back({outs[j], J.dst[j], fb});
        }
    }
    return MIRT_OK;
}

// Where rank r's delivery copies of lane L go: the context's stream, or with
// MIRT_MULTI_QUEUE_AHEAD the lane's copy stream, made to wait (once per
// launch) for everything the context's stream has been given so far -- so the
// next lane's launch on the same context starts its kernels while these
// copies run.
hipStream_t copy_stream(mirt_multi* m, Lane& L, int r)
{
    const hipStream_t st = stream_of(L.ctx[r]);
    if (!m->ahead || !m->ahead_copy_stream) return st;
    if (!L.kdone_set[r]) {
        (void)hipEventRecord(L.kdone[r], st);
        (void)hipStreamWaitEvent(L.cstream[r], L.kdone[r], 0);
        L.kdone_set[r] = 1;
    }
    return L.cstream[r];
}

// Rank r's part of lane L's current launch, on its own device and stream:
// its row blocks of every frame, then its share of the delivery, then the
// completion event. Called by rank r's thread (or, for one rank, the
// caller's).
int issue_rank_body(mirt_multi* m, Lane& L, int r)
{
    const Launch& J = L.job;
    const int n = m->n;
    const int s = J.emu ? m->emu_rank : r;    // the shard rank r renders
    const size_t elems = (size_t)J.sr.rows[s] * J.W;
    mirt_frame_desc sd = J.sd;
    sd.shard = s;
    mirt_ctx* c = L.ctx[r];
    hipStream_t st = stream_of(c);
    if (m->ahead) L.kdone_set[r] = 0;
    int keep = 0;
    if (J.flags & MIRT_MULTI_FULL_GRID) {
        keep = mirt_get_option(c, MIRT_OPT_BOUNCE_BLOCKS);
        (void)mirt_set_option(c, MIRT_OPT_BOUNCE_BLOCKS, 0);
    }
    uint32_t* disp = nullptr;
    uint32_t* out = nullptr;
    if (m->ahead) {
        // the lane's own slabs: every frame of the launch (spp * nframes samples)
        const size_t need = 4 * elems * (size_t)std::max(1, sd.samples) + 4;
        if (need > L.slab_cap[r])   // a pending fold of the old slab (the lazy fold) is taken first
            if (int g = accum_settle(c)) return g;
        if (int g = grow(m->dev[r], &L.slab[r], &L.slab_cap[r], need)) return g;
        out = L.slab[r];
    }
    int rc = enqueue_frame_device(c, &J.cam, &sd, out, &disp, "mirt_multi_render_frames_async", J.nframes > 1);
    if (J.flags & MIRT_MULTI_FULL_GRID) (void)mirt_set_option(c, MIRT_OPT_BOUNCE_BLOCKS, keep);
    if (rc) return rc;
    uint32_t* src = disp - (size_t)(J.nframes - 1) * elems;   // spp == 1 when nframes > 1: slab j = frame j
    const size_t cnt = elems * J.nframes;
    L.src[r] = src;
    MHIP(hipSetDevice(m->dev[r]));
    if (J.gather) {
        // slabs that travel: every rank's but rank 0's own (read in place,
        // unless MIRT_MULTI_OPT_GATHER_SELF sends it to itself too); one
        // emulated rank sends its own to itself, as rank k > 0 its shard, as
        // rank 0 a stand-in for each other shard's receive
        const bool self = J.self;
        const bool exchange = n > 1 || J.emu || self;
        if (!m->rccl && r > 0) {
            // copy mode: rank 0's stream copies this rank's slabs once they are done
            MHIP(hipEventRecord(L.rendered[r], st));
            L.slabs_ready[r]->store(L.seq, std::memory_order_release);
        } else if (m->rccl && exchange && r > 0) {
            // RCCL: this rank's displays to rank 0, on the stream that rendered them
            std::lock_guard<std::timed_mutex> lk(*m->comm_mu[r]);
            if (m->failed.load()) return failed_status(m, "mirt_multi_render_frames_async");
            MNCCL(ncclSend(src, cnt, ncclUint32, 0, m->comm[r], st));
            m->st_sends.fetch_add(1);
        }
        if (r == 0) {
            ShardSrc sr = J.sr;
            // the shards' displays in the gather buffer; rank 0's own where it
            // rendered them (or, sent to itself, in its slot too)
            for (int q = 0; q < J.world; q++) sr.p[q] = L.gathered + (size_t)q * J.shard_stride;
            if (!self) sr.p[s] = src;
            if (m->rccl && exchange) {
                // one group on rank 0's stream: shard q arrives at gathered + q * stride
                struct P2p {
                    const uint32_t* from;   // null: a receive from rank `peer` only
                    size_t count;
                    int slot, peer;
                };
                std::vector<P2p> ops;
                if (self || (J.emu && m->emu_rank > 0)) ops.push_back({src, cnt, s, 0});
                if (J.emu && m->emu_rank == 0)   // the other shards' receives, its own slab standing in
                    for (int q = 1; q < J.world; q++)
                        ops.push_back({src, std::min(cnt, (size_t)J.sr.rows[q] * J.W * J.nframes), q, 0});
                for (int q = 1; q < n; q++) ops.push_back({nullptr, (size_t)J.sr.rows[q] * J.W * J.nframes, q, q});
                std::lock_guard<std::timed_mutex> lk(*m->comm_mu[0]);
                if (m->failed.load()) return failed_status(m, "mirt_multi_render_frames_async");
                MNCCL(ncclGroupStart());
                ncclResult_t e = ncclSuccess;
                for (const P2p& o : ops) {
                    if (o.count == 0) continue;
                    if (o.from) {
                        e = ncclSend(o.from, o.count, ncclUint32, 0, m->comm[0], st);
                        if (e != ncclSuccess) break;
                        m->st_sends.fetch_add(1);
                    }
                    e = ncclRecv(L.gathered + (size_t)o.slot * J.shard_stride, o.count, ncclUint32, o.peer,
                                 m->comm[0], st);
                    if (e != ncclSuccess) break;
                    m->st_recvs.fetch_add(1);
                    m->st_bytes.fetch_add(4 * o.count);
                }
                if (e != ncclSuccess) {
                    (void)ncclGroupEnd();
                    return nccl_err(e, "mirt_multi_render_frames_async: ncclSend/ncclRecv");
                }
                MNCCL(ncclGroupEnd());
                m->st_groups.fetch_add(1);
            } else if (!m->rccl) {
                if (self) {   // rank 0's own slabs into its slot, as the other ranks' are copied
                    MHIP(hipMemcpyAsync(L.gathered + (size_t)s * J.shard_stride, src, 4 * cnt, hipMemcpyDeviceToDevice,
                                        st));
                    m->st_copies.fetch_add(1);
                }
                // copy mode: wait for each rank's slabs, then copy them
                // (peer-to-peer across devices, device-local otherwise)
                using clk = std::chrono::steady_clock;
                const auto t0 = clk::now();
                for (int q = 1; q < n; q++) {
                    while (L.slabs_ready[q]->load(std::memory_order_acquire) != L.seq) {
                        if (m->timeout_ms > 0 &&
                            std::chrono::duration<double, std::milli>(clk::now() - t0).count() > m->timeout_ms) {
                            set_error("mirt_multi: rank %d never handed its slabs over", q);
                            return MIRT_E_DEVICE;
                        }
                        std::this_thread::yield();
                    }
                    MHIP(hipStreamWaitEvent(st, L.rendered[q], 0));
                    uint32_t* to = L.gathered + (size_t)q * J.shard_stride;
                    const size_t cq = (size_t)J.sr.rows[q] * J.W * J.nframes;
                    if (m->dev[q] == m->dev[0])
                        MHIP(hipMemcpyAsync(to, L.src[q], 4 * cq, hipMemcpyDeviceToDevice, st));
                    else
                        MHIP(hipMemcpyPeerAsync(to, m->dev[0], L.src[q], m->dev[q], 4 * cq, st));
                    m->st_copies.fetch_add(1);
                }
                if (J.emu && m->emu_rank == 0) {
                    // emulated rank 0 of a `world`-rank job in copy mode: the
                    // other shards' slabs arrive as device copies of its own
                    // (HBM writes of the receives; no wire time, no receive kernels)
                    for (int q = 1; q < J.world; q++) {
                        MHIP(hipMemcpyAsync(L.gathered + (size_t)q * J.shard_stride, src,
                                            4 * std::min(cnt, (size_t)J.sr.rows[q] * J.W * J.nframes),
                                            hipMemcpyDeviceToDevice, st));
                        m->st_copies.fetch_add(1);
                    }
                }
            }
            if (J.rank0_assembles) {
                // one shard: its displays are the frames (in its slot when sent to itself)
                const uint32_t* frames = self ? L.gathered + (size_t)s * J.shard_stride : src;
                if (J.world > 1) {
                    const dim3 grid((J.W + 255) / 256, J.H, J.nframes);
                    deinterleave_kernel<<<grid, 256, 0, st>>>(sr, L.frame, J.W, J.H, J.rb, J.world, J.sd.lead_skip);
                    MHIP(hipGetLastError());
                    frames = L.frame;
                }
                if (J.deliver) {
                    const hipStream_t cs = copy_stream(m, L, r);
                    for (int j = 0; j < J.nframes; j++)   // as a 2D copy (H rows of W pixels): a DMA engine
                        MHIP(hipMemcpy2DAsync(J.dst[j], 4 * (size_t)J.W, frames + (size_t)j * J.frame_elems,
                                              4 * (size_t)J.W, 4 * (size_t)J.W, J.H, hipMemcpyDeviceToHost, cs));
                }
            }
        }
    } else if (J.deliver) {
        // host-direct: this rank's row blocks of frame j straight into its
        // host frame as strided copies (rows of rb * W pixels): with plain
        // interleaving (lead_skip 0) its full blocks b = s, s + world, ... are
        // ONE copy (destination pitch world * rb rows); with the lead-skip
        // weighting one copy per position k of a period (destination pitch
        // P * rb rows, source pitch w * rb rows); the image's short last block
        // (if it is this shard's) after them
        const int W = J.W, H = J.H, rb = J.rb, world = J.world, d = J.sd.lead_skip;
        const int blocks = (H + rb - 1) / rb;
        const int last = blocks - 1;
        const int nb = shard_block_count(s, blocks, world, d);     // this shard's blocks
        int owner_last = 0, c_last = 0;
        block_owner(last, world, d, owner_last, c_last);
        const bool has_short = H % rb != 0 && owner_last == s;
        const int nfull = nb - (has_short ? 1 : 0);
        const int P = shard_period(world, d), w = shard_period_blocks(s, d);
        const int last_full = H % rb != 0 ? last - 1 : last;        // the image's last full block
        st = copy_stream(m, L, r);   // the copies (with QUEUE_AHEAD on the lane's copy stream)
        for (int j = 0; j < J.nframes; j++) {
            const uint32_t* sj = src + (size_t)j * elems;
            uint32_t* dj = (uint32_t*)J.dst[j];
            if (m->direct_copy == 2 && J.sr.rows[s] > 0) {
                // a copy kernel storing into the mapped frame (staged outputs too: page-locked)
                uint32_t* dd = host_device_ptr(dj, 4 * (size_t)W * H);
                if (!dd) {
                    set_error("mirt_multi: the frame is not one mapped page-locked range (DIRECT_COPY 2)");
                    return MIRT_E_INVALID;
                }
                const dim3 grid((unsigned)((W + 1023) / 1024), (unsigned)J.sr.rows[s]);
                scatter_rows_kernel<<<grid, 256, 0, st>>>(sj, dd, W, J.sr.rows[s], rb, world, s, d);
                MHIP(hipGetLastError());
                continue;
            }
            if (m->direct_copy == 1) {   // one copy per row block
                for (int i = 0; i < nfull; i++)
                    MHIP(hipMemcpyAsync(dj + (size_t)shard_block(s, i, world, d) * rb * W, sj + (size_t)i * rb * W,
                                        (size_t)rb * W * 4, hipMemcpyDeviceToHost, st));
            } else if (d == 0) {
                if (nfull > 0)
                    MHIP(hipMemcpy2DAsync(dj + (size_t)s * rb * W, (size_t)world * rb * W * 4, sj, (size_t)rb * W * 4,
                                          (size_t)rb * W * 4, nfull, hipMemcpyDeviceToHost, st));
            } else {
                for (int k = 0; k < w; k++) {
                    const int pos = shard_block_pos(s, k, world, d);
                    const int cnt = last_full >= pos ? (last_full - pos) / P + 1 : 0;   // full blocks at pos
                    if (cnt > 0)
                        MHIP(hipMemcpy2DAsync(dj + (size_t)pos * rb * W, (size_t)P * rb * W * 4,
                                              sj + (size_t)k * rb * W, (size_t)w * rb * W * 4, (size_t)rb * W * 4,
                                              cnt, hipMemcpyDeviceToHost, st));
                }
            }
            // the short block as a one-row 2D copy too: a 1D copy after the strided one on the
            // same stream cost a rank ~0.5 ms per frame (N = 2, 16-row blocks: profiles/r05_logs/r05at/),
            // the runtime moving between its copy paths
            if (has_short) {
                const size_t sb = (size_t)(H - last * rb) * W * 4;
                MHIP(hipMemcpy2DAsync(dj + (size_t)last * rb * W, sb, sj + (size_t)c_last * rb * W, sb, sb, 1,
                                      hipMemcpyDeviceToHost, st));
            }
        }
    }
    // the launch's last operation on this rank: its copy stream when the
    // lane has one (it waited for everything the context's stream did)
    MHIP(hipEventRecord(L.done[r], copy_stream(m, L, r)));
    return MIRT_OK;
}

// issue_rank_body with its outcome recorded on the lane: the first error
// (with its message, which lives in this thread's error slot) and, on an
// error, the completion event over whatever did reach the stream.
void issue_rank(mirt_multi* m, Lane& L, int r)
{
    // a failed object issues nothing more (its lanes are never waited for again)
    const int rc = m->failed.load() ? failed_status(m, "mirt_multi_render_frames_async") : issue_rank_body(m, L, r);
    if (rc) {
        (void)hipSetDevice(m->dev[r]);
        (void)hipEventRecord(L.done[r], stream_of(L.ctx[r]));
        (void)hipGetLastError();
        if (!m->rccl && r > 0) L.slabs_ready[r]->store(L.seq, std::memory_order_release);   // rank 0 must not wait
        std::lock_guard<std::mutex> lk(*L.err_mu);
        if (!L.err) {
            L.err = rc;
            L.err_msg = mirt_last_error();
        }
    }
    L.issued->fetch_add(1, std::memory_order_acq_rel);
}

// `w` is passed in, not read from m->workers: the caller's thread is still
// appending the later ranks' workers (reallocating that vector) while the
// first threads start.
void rank_thread_main(mirt_multi* m, int r, RankThread* wp)
{
    RankThread& w = *wp;
    (void)hipSetDevice(m->dev[r]);
    for (;;) {
        int li;
        {
            std::unique_lock<std::mutex> lk(w.mu);
            w.cv.wait(lk, [&] { return w.stop || !w.q.empty(); });
            if (w.q.empty()) return;   // stop, nothing left
            li = w.q.front();
            w.q.pop_front();
        }
        issue_rank(m, m->lanes[li], r);
    }
}

// Launch on lane li: prepared here, issued by every rank (its own thread
// when n > 1).
int enqueue(mirt_multi* m, int li, const mirt_camera* cam, const mirt_frame_desc* fd, int nframes, int flags,
            mirt_rgba8* const* outs)
{
    Lane& L = m->lanes[li];
    if (int rc = prepare(m, L, cam, fd, nframes, flags, outs)) return rc;
    L.seq++;
    L.err = MIRT_OK;
    L.issued->store(0, std::memory_order_relaxed);
    L.pending = true;
    if (m->workers.empty()) {
        for (int r = m->n - 1; r >= 0; r--) issue_rank(m, L, r);
        return MIRT_OK;
    }
    for (int r = 0; r < m->n; r++) {
        RankThread& w = *m->workers[r];
        {
            std::lock_guard<std::mutex> lk(w.mu);
            w.q.push_back(li);
        }
        w.cv.notify_one();
    }
    return MIRT_OK;
}

bool multi_ok(mirt_multi* m, const char* fn)
{
    if (!m) set_error("%s: null mirt_multi", fn);
    return m != nullptr;
}

int check_frame(const mirt_multi* m, const mirt_camera* cam, const mirt_frame_desc* fd, int nframes,
                mirt_rgba8* const* outs, const char* fn)
{
    if (!cam || !fd || fd->shard != 0 || fd->num_shards > 1 || fd->num_shards < 0 || fd->row_block < 0 ||
        fd->lead_skip != 0 || nframes < 1) {
        set_error("%s: invalid arguments (fd describes the whole frame: shard 0, num_shards 0 or 1, lead_skip 0 "
                  "-- the weighting is MIRT_MULTI_OPT_LEAD_SKIP)", fn);
        return MIRT_E_INVALID;
    }
    if (nframes > 1 && fd->samples > 1) {
        set_error("%s: several frames per launch need one sample per frame (fd->samples <= 1)", fn);
        return MIRT_E_INVALID;
    }
    if (outs)
        for (int j = 0; j < nframes; j++)
            if (!outs[j]) {
                set_error("%s: outs[%d] is null", fn, j);
                return MIRT_E_INVALID;
            }
    mirt_frame_desc whole = *fd;
    whole.num_shards = m->emu_world > 1 ? m->emu_world : m->n;
    whole.row_block = fd->row_block > 0 ? fd->row_block : 8;
    whole.samples = std::max(1, fd->samples) * nframes;
    whole.lead_skip = lead_skip_for(m, whole.num_shards, !m->direct);
    if (!frame_desc_valid(&whole) || whole.num_shards > kMaxShards) {
        set_error("%s: invalid frame descriptor (or more than 64 frames / samples per launch)", fn);
        return MIRT_E_INVALID;
    }
    return MIRT_OK;
}

}  // namespace

extern "C" {

int mirt_multi_create(const int* devices, int n, int lanes, int flags, mirt_multi** out)
try {
    if (!out || n <= 0 || n > kMaxShards || lanes <= 0 ||
        (flags & ~(MIRT_MULTI_COPY | MIRT_MULTI_HOST_DIRECT | MIRT_MULTI_QUEUE_AHEAD))) {
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
    m->direct = (flags & MIRT_MULTI_HOST_DIRECT) != 0;
    m->ahead = (flags & MIRT_MULTI_QUEUE_AHEAD) != 0;
    m->nctx = lanes;
    m->rccl = distinct && !(flags & MIRT_MULTI_COPY);
    for (int r = 0; r < n; r++) m->comm_mu.emplace_back(new std::timed_mutex);
    auto fail = [&](int rc) {
        mirt_multi_destroy(m);
        return rc;
    };
    if (m->rccl) {
        // communicators: at the first launch that exchanges anything (never
        // for one rank, whose slab is its frame), after the contexts' streams
        // exist -- RCCL's own streams created first would share the lanes'
        // hardware queues (GPU_MAX_HW_QUEUES is 4 by default)
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
    const int slots = m->ahead ? 2 * lanes : lanes;
    m->lanes.resize(slots);
    for (int l = 0; l < slots; l++) {
        Lane& L = m->lanes[l];
        L.ctx.assign(n, nullptr);
        L.rendered.assign(n, nullptr);
        L.done.assign(n, nullptr);
        L.src.assign(n, nullptr);
        L.slab.assign(n, nullptr);
        L.slab_cap.assign(n, 0);
        L.cstream.assign(n, nullptr);
        L.kdone.assign(n, nullptr);
        L.kdone_set.assign(n, 0);
        L.owns_ctx = l < lanes;
        for (int r = 0; r < n; r++) L.slabs_ready.emplace_back(new std::atomic<uint64_t>(0));
        for (int r = 0; r < n; r++) {
            (void)hipSetDevice(m->dev[r]);
            hipError_t e = hipEventCreateWithFlags(&L.rendered[r], hipEventDisableTiming);
            if (e == hipSuccess) e = hipEventCreateWithFlags(&L.done[r], hipEventDisableTiming);
            if (e == hipSuccess && m->ahead) e = hipEventCreateWithFlags(&L.kdone[r], hipEventDisableTiming);
            // one copy stream per context, shared by its two launch slots (a
            // stream beyond the process's hardware queues shares one with
            // another stream, whose waits then block it)
            if (e == hipSuccess && m->ahead && L.owns_ctx)
                e = hipStreamCreateWithFlags(&L.cstream[r], hipStreamNonBlocking);
            if (e != hipSuccess) return fail(hip_err(e, "mirt_multi_create: hipEventCreate / hipStreamCreate"));
            if (!L.owns_ctx) {
                // the second launch slot of context set l - lanes: its kernels
                // queue behind that lane's on the same stream
                L.ctx[r] = m->lanes[l - lanes].ctx[r];
                L.cstream[r] = m->lanes[l - lanes].cstream[r];
                continue;
            }
            int rc = mirt_create(m->dev[r], &L.ctx[r]);
            if (rc) return fail(rc);
            if (lanes > 1) {
                // launches in flight share the chip: each bounce pass at 1.5
                // persistent workgroups per CU instead of the full grid
                // (2,400 -> 2,648 Mrays/s at four in flight)
                int cus = 0;
                e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, m->dev[r]);
                if (e != hipSuccess) return fail(hip_err(e, "mirt_multi_create: hipDeviceGetAttribute"));
                rc = mirt_set_option(L.ctx[r], MIRT_OPT_BOUNCE_BLOCKS, std::max(1, 3 * cus / 2));
                if (rc) return fail(rc);
            }
            // the lanes of a rank keep ONE accumulation buffer: frames in
            // flight of the accumulating loop (main.c:379-408) fold in order
            if (l > 0) {
                rc = mirt_ctx_share_accum(L.ctx[r], m->lanes[0].ctx[r]);
                if (rc) return fail(rc);
            }
        }
    }
    // one issuing thread per rank (n > 1)
    if (n > 1) {
        m->workers.reserve(n);
        for (int r = 0; r < n; r++) {
            m->workers.emplace_back(new RankThread());
            RankThread* w = m->workers.back().get();
            w->th = std::thread(rank_thread_main, m, r, w);
        }
    }
    *out = m;
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    set_error("mirt_multi_create: out of host memory");
    return MIRT_E_NOMEM;
} catch (const std::system_error&) {
    set_error("mirt_multi_create: could not start the rank threads");
    return MIRT_E_NOMEM;
}

void mirt_multi_destroy(mirt_multi* m)
{
    if (!m) return;
    for (int l = 0; l < (int)m->lanes.size() && !m->failed; l++) (void)wait_lane(m, l);
    for (auto& w : m->workers) {
        {
            std::lock_guard<std::mutex> lk(w->mu);
            w->stop = true;
        }
        w->cv.notify_one();
    }
    if (m->failed) {
        // work may still be queued on a stuck device, and a rank thread may be
        // inside a call that waits for it: freeing the buffers, destroying the
        // streams or joining that thread would wait too, so they are left to
        // the process's exit (the communicators were aborted when it failed)
        // (the object itself stays allocated: a detached rank thread may
        // still touch its lane and its queue)
        for (auto& w : m->workers) w->th.detach();
        return;
    }
    for (auto& w : m->workers) w->th.join();
    m->workers.clear();
    // a fresh frame's display left pending on a rank's shared accumulation
    // buffer (the lazy fold) may lie in a lane's own slab (QUEUE_AHEAD):
    // fold it, and let every read of the slabs end, before any slab is freed
    for (Lane& L : m->lanes)
        if (L.owns_ctx)
            for (mirt_ctx* c : L.ctx)
                if (c) (void)accum_settle(c);
    for (Lane& L : m->lanes) {
        for (int r = 0; r < (int)L.ctx.size(); r++) {
            (void)hipSetDevice(m->dev[r]);
            if (L.rendered[r]) (void)hipEventDestroy(L.rendered[r]);
            if (L.done[r]) (void)hipEventDestroy(L.done[r]);
            if (r < (int)L.kdone.size() && L.kdone[r]) (void)hipEventDestroy(L.kdone[r]);
            if (L.owns_ctx && r < (int)L.cstream.size() && L.cstream[r]) (void)hipStreamDestroy(L.cstream[r]);
            if (r < (int)L.slab.size() && L.slab[r]) (void)hipFree(L.slab[r]);
            if (L.owns_ctx) mirt_destroy(L.ctx[r]);
        }
        (void)hipSetDevice(m->dev[0]);
        if (L.gathered) (void)hipFree(L.gathered);
        if (L.frame) (void)hipFree(L.frame);
        if (L.stage) (void)hipHostFree(L.stage);
    }
    for (ncclComm_t c : m->comm)
        if (c) (void)ncclCommDestroy(c);
    delete m;
}

int mirt_multi_size(const mirt_multi* m) { return m ? m->n : MIRT_E_INVALID; }
int mirt_multi_lanes(const mirt_multi* m) { return m ? (int)m->lanes.size() : MIRT_E_INVALID; }
const char* mirt_multi_backend(const mirt_multi* m) { return !m ? "" : m->rccl ? "rccl" : "copy"; }
const char* mirt_multi_delivery(const mirt_multi* m) { return !m ? "" : m->direct ? "host-direct" : "gather"; }
int mirt_multi_failed(const mirt_multi* m) { return !m ? MIRT_E_INVALID : m->failed ? 1 : 0; }

mirt_ctx* mirt_multi_ctx(mirt_multi* m, int lane, int rank)
{
    if (!m || lane < 0 || lane >= (int)m->lanes.size() || rank < 0 || rank >= m->n) return nullptr;
    return m->lanes[lane].ctx[rank];
}

int mirt_multi_set_option(mirt_multi* m, int option, int value)
{
    if (!multi_ok(m, "mirt_multi_set_option")) return MIRT_E_INVALID;
    if (m->failed) return failed_status(m, "mirt_multi_set_option");
    // the rank threads read the options and the contexts while they issue a
    // launch: change them only with no launch in flight
    if (option != MIRT_MULTI_OPT_TIMEOUT_MS)
        for (int l = 0; l < (int)m->lanes.size(); l++)
            if (int rc = wait_lane(m, l)) return rc;
    switch (option) {
    case MIRT_MULTI_OPT_TIMEOUT_MS:
        if (value < 0) break;
        m->timeout_ms = value;
        return MIRT_OK;
    case MIRT_MULTI_OPT_EMULATE_WORLD:
        // launches in flight would mix shard geometries: only between frames
        if (value < 0 || value > kMaxShards || (value > 1 && m->n != 1)) break;
        m->emu_world = value;
        if (m->emu_rank >= std::max(1, value)) m->emu_rank = 0;
        return MIRT_OK;
    case MIRT_MULTI_OPT_DIRECT_COPY:
        if (value < 0 || value > 2) break;
        m->direct_copy = value;
        return MIRT_OK;
    case MIRT_MULTI_OPT_COPY_STREAM:
        if (value < 0 || value > 2) break;
        m->ahead_copy_stream = value;
        return MIRT_OK;
    case MIRT_MULTI_OPT_EMULATE_RANK:
        if (value < 0 || value >= std::max(1, m->emu_world)) break;
        m->emu_rank = value;
        return MIRT_OK;
    case MIRT_MULTI_OPT_GATHER_SELF:
        if (value < 0 || value > 1) break;
        m->gather_self = value == 1;
        return MIRT_OK;
    case MIRT_MULTI_OPT_LEAD_SKIP:
        if (value < 0 || value > kLeadRounds) break;   // kLeadRounds: automatic
        m->lead_skip = value;
        return MIRT_OK;
    default:
        for (Lane& L : m->lanes)
            if (L.owns_ctx)
                for (mirt_ctx* c : L.ctx)
                    if (int rc = mirt_set_option(c, option, value)) return rc;
        return MIRT_OK;
    }
    set_error("mirt_multi_set_option: invalid option %d / value %d", option, value);
    return MIRT_E_INVALID;
}

int mirt_multi_get_option(mirt_multi* m, int option)
{
    if (!multi_ok(m, "mirt_multi_get_option")) return MIRT_E_INVALID;
    if (option == MIRT_MULTI_OPT_TIMEOUT_MS) return m->timeout_ms;
    if (option == MIRT_MULTI_OPT_EMULATE_WORLD) return m->emu_world;
    if (option == MIRT_MULTI_OPT_EMULATE_RANK) return m->emu_rank;
    if (option == MIRT_MULTI_OPT_DIRECT_COPY) return m->direct_copy;
    if (option == MIRT_MULTI_OPT_COPY_STREAM) return m->ahead_copy_stream;
    if (option == MIRT_MULTI_OPT_GATHER_SELF) return m->gather_self ? 1 : 0;
    if (option == MIRT_MULTI_OPT_LEAD_SKIP) return m->lead_skip;
    return mirt_get_option(m->lanes[0].ctx[0], option);
}

int mirt_multi_scene_upload(mirt_multi* m, const mirt_sphere* spheres, int num_spheres, const mirt_bvh_node* root)
{
    if (!multi_ok(m, "mirt_multi_scene_upload")) return MIRT_E_INVALID;
    for (int l = 0; l < (int)m->lanes.size(); l++)
        if (int rc = wait_lane(m, l)) return rc;
    for (Lane& L : m->lanes)
        if (L.owns_ctx)
            for (mirt_ctx* c : L.ctx)
                if (int rc = mirt_scene_upload(c, spheres, num_spheres, root)) return rc;
    return MIRT_OK;
}

int mirt_multi_scene_upload_flat(mirt_multi* m, const mirt_sphere* spheres, int num_spheres, const mirt_node* nodes,
                                 int num_nodes)
{
    if (!multi_ok(m, "mirt_multi_scene_upload_flat")) return MIRT_E_INVALID;
    for (int l = 0; l < (int)m->lanes.size(); l++)
        if (int rc = wait_lane(m, l)) return rc;
    for (Lane& L : m->lanes)
        if (L.owns_ctx)
            for (mirt_ctx* c : L.ctx)
                if (int rc = mirt_scene_upload_flat(c, spheres, num_spheres, nodes, num_nodes)) return rc;
    return MIRT_OK;
}

int mirt_multi_render_frames_async(mirt_multi* m, const mirt_camera* cam, const mirt_frame_desc* fd, int nframes,
                                   int flags, mirt_rgba8* const* outs)
try {
    const char* fn = "mirt_multi_render_frames_async";
    if (!multi_ok(m, fn)) return MIRT_E_INVALID;
    if (m->failed) return failed_status(m, fn);
    if (int rc = check_frame(m, cam, fd, nframes, outs, fn)) return rc;
    const int li = m->next;
    if (int rc = wait_lane(m, li)) return rc;
    if (m->ahead && m->ahead_copy_stream == 2)
        if (int rc = wait_sibling_kernels(m, li)) return rc;
    // an error here (before any rank issued) leaves the lane and the rotation
    // as they were; the ranks' own issue errors come back from the lane's wait
    if (int rc = enqueue(m, li, cam, fd, nframes, flags, outs)) return rc;
    m->next = (m->next + 1) % (int)m->lanes.size();
    m->last_lane = li;
    m->st_launches.fetch_add(1);
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    set_error("mirt_multi_render_frames_async: out of host memory");
    return MIRT_E_NOMEM;
}

int mirt_multi_render_frame_async(mirt_multi* m, const mirt_camera* cam, const mirt_frame_desc* fd,
                                  mirt_rgba8* out)
{
    if (!out) {
        set_error("mirt_multi_render_frame_async: null output");
        return MIRT_E_INVALID;
    }
    return mirt_multi_render_frames_async(m, cam, fd, 1, 0, &out);
}

int mirt_multi_render_frame(mirt_multi* m, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out)
{
    if (!multi_ok(m, "mirt_multi_render_frame")) return MIRT_E_INVALID;
    const int li = m->next;
    if (int rc = mirt_multi_render_frame_async(m, cam, fd, out)) return rc;
    return wait_lane(m, li);
}

int mirt_multi_wait(mirt_multi* m)
{
    if (!multi_ok(m, "mirt_multi_wait")) return MIRT_E_INVALID;
    for (int l = 0; l < (int)m->lanes.size(); l++)
        if (int rc = wait_lane(m, l)) return rc;
    return MIRT_OK;
}

int mirt_multi_get_stats(const mirt_multi* m, mirt_multi_stats* out)
{
    if (!m || !out) {
        set_error("mirt_multi_get_stats: invalid arguments");
        return MIRT_E_INVALID;
    }
    out->launches = m->st_launches.load();
    out->comm_inits = m->st_comm_inits.load();
    out->rccl_groups = m->st_groups.load();
    out->rccl_sends = m->st_sends.load();
    out->rccl_recvs = m->st_recvs.load();
    out->rccl_bytes = m->st_bytes.load();
    out->device_copies = m->st_copies.load();
    return MIRT_OK;
}

int mirt_multi_read_gathered(mirt_multi* m, int lane, int shard, int frame, mirt_rgba8* out, size_t bytes)
try {
    const char* fn = "mirt_multi_read_gathered";
    if (!multi_ok(m, fn)) return MIRT_E_INVALID;
    if (m->failed) return failed_status(m, fn);
    if (lane < 0) lane = m->last_lane;
    if (lane < 0 || lane >= (int)m->lanes.size() || !out) {
        set_error("%s: no such lane (or no launch yet), or null output", fn);
        return MIRT_E_INVALID;
    }
    if (int rc = wait_lane(m, lane)) return rc;
    Lane& L = m->lanes[lane];
    const Launch& J = L.job;
    if (!J.gather || (J.world <= 1 && !J.self) || !L.gathered || shard < 0 || shard >= J.world || frame < 0 ||
        frame >= J.nframes) {
        set_error("%s: the lane's last launch gathered no such shard / frame (gather delivery, world > 1)", fn);
        return MIRT_E_INVALID;
    }
    const size_t n = (size_t)J.sr.rows[shard] * J.W;
    if (bytes < 4 * n) {
        set_error("%s: output holds %zu bytes, the shard's slab %zu", fn, bytes, 4 * n);
        return MIRT_E_INVALID;
    }
    MHIP(hipSetDevice(m->dev[0]));
    MHIP(hipMemcpy(out, L.gathered + (size_t)shard * J.shard_stride + (size_t)frame * n, 4 * n, hipMemcpyDeviceToHost));
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    set_error("mirt_multi_read_gathered: out of host memory");
    return MIRT_E_NOMEM;
}

}  // extern "C"
