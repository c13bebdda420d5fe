// HIP kernels and the device half of the C ABI (include/mirt.h).
//
// Frame kernel: one wave64 per 8x8 pixel tile (coherent primary rays share
// their BVH walk), 4 waves per 256-thread workgroup. Each lane traces one
// pixel through trace_path (trace.h); the wave walks the skip-threaded tree
// with a wave-uniform cursor, so node and sphere reads are scalar loads of
// an L2-resident array. Output is packed RGBA8 (one dword per pixel).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <algorithm>
#include <map>
#include <mutex>
#include <cstring>
#include <new>
#include <vector>

#include "internal.h"
#include "shard.h"
#include "trace.h"

using namespace mirt;

namespace {

// Per-frame constants computed on the host with the reference's expressions
// (ray.c:18-24, main.c:356) -- libm tan stays on the host.
struct FrameConst {
    float px, py, pz;  // camera position (ray origin)
    float fx, fy, fz;  // forward
    float hx, hy, hz;  // horizontal = right * (2 half_width)
    float vx, vy, vz;  // vertical = up * (2 half_height)
    float aspect, wf, hf;
    int width, height, depth, use_bvh;
    uint64_t seed;
    uint32_t sample;
    int accumulate;
    float frames;
    int row_block, shard, num_shards, lead_skip;
    int jitter;        // sub-pixel jitter of camera rays from the RNG contract (camera_ray)
    int num_rows;      // rows of this launch: shard_rows x samples (frame j's rows follow frame j-1's)
    int shard_rows;    // rows of one frame of this shard
    int samples;       // frames in this launch (RNG samples sample .. sample + samples - 1)
};

FrameConst make_frame_const(const mirt_camera* cam, const mirt_frame_desc* fd)
{
    FrameConst f{};
    const float aspect = (float)fd->width / (float)fd->height;                    // ray.c:18
    const float fov_rad = (float)((double)cam->fov * (M_PI / 180.0));             // ray.c:19
    const float half_h = (float)std::tan((double)(fov_rad / 2.0f));               // ray.c:20
    const float half_w = aspect * half_h;                                         // ray.c:21
    const float sw = 2.0f * half_w, sh = 2.0f * half_h;
    f.px = cam->position.x; f.py = cam->position.y; f.pz = cam->position.z;
    f.fx = cam->forward.x; f.fy = cam->forward.y; f.fz = cam->forward.z;
    f.hx = cam->right.x * sw; f.hy = cam->right.y * sw; f.hz = cam->right.z * sw;  // ray.c:23
    f.vx = cam->up.x * sh; f.vy = cam->up.y * sh; f.vz = cam->up.z * sh;          // ray.c:24
    f.aspect = aspect;                                                            // main.c:356
    f.wf = (float)fd->width;
    f.hf = (float)fd->height;
    f.width = fd->width;
    f.height = fd->height;
    f.depth = fd->max_depth;
    f.use_bvh = fd->use_bvh;
    f.seed = fd->seed;
    f.sample = fd->sample;
    f.accumulate = fd->accumulate;
    f.frames = (float)fd->frames;
    f.row_block = fd->row_block;
    f.shard = fd->shard;
    f.num_shards = fd->num_shards;
    f.lead_skip = fd->lead_skip;
    f.shard_rows = shard_row_count(fd);
    f.samples = fd->samples > 1 ? fd->samples : 1;
    f.jitter = fd->jitter != 0;
    f.num_rows = f.shard_rows * f.samples;
    return f;
}

// Image row of launch row r (compacted shard row r % shard_rows of frame r / shard_rows).
__device__ __forceinline__ int shard_row_to_y(const FrameConst& f, int r)
{
    if (f.samples > 1) r %= f.shard_rows;
    const int blk = r / f.row_block;
    return shard_block(f.shard, blk, f.num_shards, f.lead_skip) * f.row_block + (r - blk * f.row_block);
}

// RNG contract sample of launch row r (one sample per frame).
__device__ __forceinline__ uint32_t row_sample(const FrameConst& f, int r)
{
    return f.samples > 1 ? f.sample + (uint32_t)(r / f.shard_rows) : f.sample;
}

// main.c:362-365 + ray.c:26-31 for pixel (x, y) of RNG sample `sample`.
// Jittered frames (mirt_frame_desc.jitter; BASELINE configs[4] "4 spp
// jittered" -- the reference has no jitter, so the build defines it): the
// sample point moves by (jx, jy) in [0, 1)^2, two draws of the pixel's RNG
// contract stream at indices its bounce sampling never reaches (rng.h).
__device__ __forceinline__ Ray camera_ray(const FrameConst& f, int x, int y, uint32_t sample)
{
    float xf = (float)x, yf = (float)y;
    if (f.jitter) {
        const uint64_t key = pixel_key(f.seed, (uint32_t)(y * f.width + x), sample);
        xf = xf + (float)draw(key, kJitterDrawX) / 2147483648.0f;
        yf = yf + (float)draw(key, kJitterDrawY) / 2147483648.0f;
    }
    const float u = (xf / f.wf - 0.5f) * f.aspect;
    const float v = -(yf / f.hf - 0.5f);
    float dx = f.fx + f.hx * u, dy = f.fy + f.hy * u, dz = f.fz + f.hz * u;
    dx = dx + f.vx * v;
    dy = dy + f.vy * v;
    dz = dz + f.vz * v;
    normalize3(dx, dy, dz);
    return {f.px, f.py, f.pz, dx, dy, dz};
}

__device__ __forceinline__ void add_counts(mirt_counts* out, const Counters& c)
{
    atomicAdd((unsigned long long*)&out->rays, (unsigned long long)c.rays);
    atomicAdd((unsigned long long*)&out->nodes, (unsigned long long)c.nodes);
    atomicAdd((unsigned long long*)&out->spheres, (unsigned long long)c.spheres);
    atomicAdd((unsigned long long*)&out->hits, (unsigned long long)c.hits);
    atomicAdd((unsigned long long*)&out->lane_steps, (unsigned long long)c.steps);
    atomicAdd((unsigned long long*)&out->nodes_primary, (unsigned long long)c.nodes0);
    atomicAdd((unsigned long long*)&out->spheres_primary, (unsigned long long)c.spheres0);
    atomicAdd((unsigned long long*)&out->hits_primary, (unsigned long long)c.hits0);
}

// Pixels whose camera ray has a zero or tiny direction component (the image
// centre row / column under an axis-aligned camera) ignore a slab
// (hit.c:54-57) and walk a large part of the tree. A pre-pass lists them
// (mark_deferred_kernel); the first `blocks` workgroups of the frame kernel
// trace them one pixel per wave (the node-parallel walk of trace.h) while
// the other workgroups trace the 8x8 tiles and skip them, so the long walks
// start first and overlap the bulk instead of trailing it.
struct Deferred {
    const uint32_t* list;   // r * width + x
    const uint32_t* count;
    int blocks;
};

// One pixel of the pixel loop: main.c:362-366 ray, trace_ray, then the
// display/accumulation of main.c:368-372 (fresh) or main.c:394-405.
template <bool FAST, bool COUNT>
__device__ __forceinline__ void render_pixel(const DevScene& sc, const FrameConst& f, int x, int r, bool alive,
                                             bool skip_generic, uint32_t* __restrict__ out, float* __restrict__ acc,
                                             Counters& cnt, uint32_t* cstack, int cstride,
                                             uint32_t* wstk = nullptr)
{
    const int y = alive ? shard_row_to_y(f, r) : 0;
    const Ray ray = camera_ray(f, alive ? x : 0, y, row_sample(f, r));
    if (skip_generic && alive && slab_ray(ray).generic) alive = false;  // a deferred wave traces it
    const uint64_t key = pixel_key(f.seed, (uint32_t)(y * f.width + x), row_sample(f, r));
    const uint32_t c = trace_path<FAST, COUNT>(sc, ray, alive, f.depth, f.use_bvh != 0, key, cnt, cstack,
                                                     cstride, wstk);
    if (!alive) return;
    const size_t i = (size_t)r * f.width + x;
    uint32_t shown = c;
    if (acc) {
        float* a = acc + 3 * i;
        for (int ch = 0; ch < 3; ch++) {
            const float v = (float)((c >> (8 * ch)) & 0xff) / 255.0f;  // main.c:368-370 / 394-396
            if (f.accumulate) {
                a[ch] = a[ch] + v;
                const float avg = a[ch] / f.frames * 255.0f;           // main.c:398-400
                const uint32_t q = (uint32_t)(int)fminf(avg, 255.0f);
                shown = (shown & ~(0xffu << (8 * ch))) | ((q & 0xffu) << (8 * ch));
            } else {
                a[ch] = v;
            }
        }
    }
    out[i] = shown;
}

// The pixel loop of main.c:358-374 (fresh) / main.c:382-407 (accumulate).
template <bool FAST, bool COUNT>
__global__ __launch_bounds__(512) void render_kernel(DevScene sc, FrameConst f, uint32_t* __restrict__ out,
                                                      float* __restrict__ acc, mirt_counts* counts,
                                                      uint32_t* wave_stats, Deferred dfr)
{
    uint64_t t0 = 0;
    if (COUNT) t0 = __builtin_amdgcn_s_memrealtime();
    __shared__ uint32_t cstack[kMaxDepth * 512];
    // the four-wide walk's stack (stride kWideStride: workgroups of up to 256)
    __shared__ uint32_t wstack[kWideStack * kWideStride];
    uint32_t* wstk = blockDim.x <= kWideStride ? wstack + threadIdx.x : nullptr;
    Counters cnt{0, 0, 0, 0, 0};
    const int bw = blockDim.x >> 6;
    const int wave = threadIdx.x >> 6;
    if ((int)blockIdx.x < dfr.blocks) {
        const uint32_t n = __builtin_amdgcn_readfirstlane(*dfr.count);
        const uint32_t stride = (uint32_t)(dfr.blocks * bw);
        for (uint32_t j = blockIdx.x * bw + wave; j < n; j += stride) {
            const uint32_t p = __builtin_amdgcn_readfirstlane(dfr.list[j]);
            render_pixel<FAST, COUNT>(sc, f, (int)(p % f.width), (int)(p / f.width), (threadIdx.x & 63) == 0,
                                            false, out, acc, cnt, cstack + threadIdx.x, blockDim.x, wstk);
        }
        if (COUNT) add_counts(counts, cnt);
        return;
    }
    const int tile = (blockIdx.x - dfr.blocks) * bw + wave;
    const int lane = threadIdx.x & 63;
    const int tiles_x = (f.width + 7) >> 3;
    const int x = (tile % tiles_x) * 8 + (lane & 7);
    const int r = (tile / tiles_x) * 8 + (lane >> 3);
    render_pixel<FAST, COUNT>(sc, f, x, r, x < f.width && r < f.num_rows, dfr.blocks > 0, out, acc, cnt,
                                    cstack + threadIdx.x, blockDim.x, wstk);
    if (COUNT) {
        add_counts(counts, cnt);
        if (wave_stats && lane == 0) {
            // diagnostic: {tile, traversal steps of this wave, start, end} (100 MHz clock)
            const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
            uint32_t* w = wave_stats + 4 * (size_t)tile;
            w[0] = tile;
            w[1] = cnt.steps;
            w[2] = (uint32_t)t0;
            w[3] = (uint32_t)t1;
        }
    }
}

// MIRT_OPT_DEBUG_STALL_MS (test hook): one wave that waits `ticks` of the
// 100 MHz real-time clock, then exits -- a frame that cannot finish within a
// caller's deadline, bounded so the grid always drains.
__global__ void stall_kernel(uint64_t ticks)
{
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

__global__ void mark_deferred_kernel(FrameConst f, uint32_t* __restrict__ list, uint32_t* __restrict__ count)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (x >= f.width || r >= f.num_rows) return;
    const Ray ray = camera_ray(f, x, shard_row_to_y(f, r), row_sample(f, r));
    if (slab_ray(ray).generic) list[atomicAdd(count, 1u)] = (uint32_t)(r * f.width + x);
}

// main.c:368-372 / 394-405 for one finished pixel i of the shard.
__device__ __forceinline__ void store_pixel(const FrameConst& f, uint32_t* __restrict__ out, float* __restrict__ acc,
                                            size_t i, uint32_t c)
{
    uint32_t shown = c;
    if (acc) {
        float* a = acc + 3 * i;
        for (int ch = 0; ch < 3; ch++) {
            const float v = (float)((c >> (8 * ch)) & 0xff) / 255.0f;
            if (f.accumulate) {
                a[ch] = a[ch] + v;
                const float avg = a[ch] / f.frames * 255.0f;
                const uint32_t q = (uint32_t)(int)fminf(avg, 255.0f);
                shown = (shown & ~(0xffu << (8 * ch))) | ((q & 0xffu) << (8 * ch));
            } else {
                a[ch] = v;
            }
        }
    }
    out[i] = shown;
}

// A launch of f.samples > 1 frames with an accumulation buffer (or any frame
// of a ctx whose accumulation buffer is shared, mirt_ctx_share_accum): the
// kernels wrote each frame's colours to its own slab of `out`; fold them
// into `acc` in frame order, exactly as f.samples successive store_pixel
// calls would (frame j: fresh if j == 0 and !f.accumulate, else divisor
// f.frames + j), leaving in slab j the display main.c:394-405 shows after
// frame j.
__global__ void fold_samples_kernel(FrameConst f, uint32_t* __restrict__ out, float* __restrict__ acc)
{
    const size_t n = (size_t)f.shard_rows * f.width;
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float* a = acc + 3 * i;
    float a0 = a[0], a1 = a[1], a2 = a[2];
    for (int j = 0; j < f.samples; j++) {
        const uint32_t c = out[(size_t)j * n + i];
        uint32_t shown = c;
        float* ch[3] = {&a0, &a1, &a2};
        for (int k = 0; k < 3; k++) {
            const float v = (float)((c >> (8 * k)) & 0xff) / 255.0f;       // main.c:368-370 / 394-396
            if (j == 0 && !f.accumulate) {
                *ch[k] = v;
            } else {
                *ch[k] = *ch[k] + v;
                const float avg = *ch[k] / (f.frames + (float)j) * 255.0f;  // main.c:398-400
                const uint32_t q = (uint32_t)(int)fminf(avg, 255.0f);
                shown = (shown & ~(0xffu << (8 * k))) | ((q & 0xffu) << (8 * k));
            }
        }
        out[(size_t)j * n + i] = shown;
    }
    a[0] = a0;
    a[1] = a1;
    a[2] = a2;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t mask)
{
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// ------------------------------------------------------------------------
// Wavefront schedule (depth >= 2): the camera rays of 8x8 tiles are walked
// as packets (wave-uniform cursor); the bounce chains that follow are
// scattered, so they go through a queue to persistent waves in which every
// lane owns one pixel's chain and refills from the queue when it ends.

// Measured (scripts/ab_libs.py, 1080p/10k/depth 5, profiles/r02*_ab*.log): 192
// nodes at 4 waves/SIMD 1659 Mrays/s; 96 nodes at 5 waves/SIMD (the LDS of
// five workgroups then fits 160 KB) 1772; 6 waves/SIMD spills: 1587.
#ifndef MIRT_HCACHE
#define MIRT_HCACHE 16
#endif
constexpr uint32_t kHCache = MIRT_HCACHE;
constexpr int kBounceDiag = 12;  // mirt_bounce_stats words per wave  // HNodes staged in LDS per bounce workgroup (64 B each)

// The bounce queue's control words: {records written} in the first 128-B
// line, then one read head per queue SEGMENT, each in its own line. The
// bounce waves read the queue as kQSeg contiguous segments (the primary
// pass fills it in roughly tile order, so a segment is roughly a band of the
// image): the waves of workgroup b start on segment b % kQSeg -- the
// workgroups that share an XCD (dealt round-robin over the 8), so a
// segment's rays, and the nodes near their origins, stay in one XCD's L2 --
// and move on to the next segment when theirs runs dry. Eight heads also
// split the refill atomics that one word would serialise.
#ifndef MIRT_QSEG
#define MIRT_QSEG 8
#endif
constexpr uint32_t kQSeg = MIRT_QSEG;
constexpr uint32_t kQLine = 32;                        // dwords per 128-B line
constexpr size_t kQCtlBytes = 4 * kQLine * (1 + kQSeg);

// First bounce of one pixel, produced by primary_kernel.
struct BounceRec {
    float ox, oy, oz, dx, dy, dz;
    uint32_t pixel;  // r * width + x (shard-compacted row r)
    uint32_t k;      // RNG contract draws consumed so far
    uint32_t base0;  // colour of the camera ray's hit (renderer.c:49)
    uint32_t pad;
};


// ORD: the tree admits the ordered packet walk (DevScene::ordered), which
// also takes zero-component rays -- that build has no deferred waves and no
// other walk, so it keeps the register budget of the packet walk alone.
// BND (ORD only): the camera is within 4C of the origin (DevScene::o_bound):
// the packet walk tests the grown inner-child boxes without margins (trace.h).
template <bool FAST, bool ORD, bool BND = false>
// Register budget of the ordered camera-packet kernel (ORD): 8 waves per SIMD (64 VGPRs, no
// scratch; 67 and 7 waves without the attribute). With four frames in flight
// its waves share the CUs with the bounce passes, and the eighth wave hides
// more of the packet walk's scalar-load latency (1080p/10k +0.3-1.1%,
// 1080p/100k +3.7%, profiles/r02_ab/r02ax_primary_waves8_*).
#ifndef MIRT_BOUNCE_WAVES
#define MIRT_BOUNCE_WAVES 5
#endif
#ifndef MIRT_PRIMARY_WAVES
#define MIRT_PRIMARY_WAVES 8
#endif
// (Round 3: the ordered kernel groups each workgroup's first bounces by
// direction octant in the queue -- scripts/tree_quality.cpp's lockstep model:
// distinct nodes per lane-step -9%, busy lanes per step +13%; measured +1.8%.)
#define MIRT_PRIMARY_ATTR __attribute__((amdgpu_waves_per_eu(ORD ? MIRT_PRIMARY_WAVES : 1)))
__global__ __launch_bounds__(256) MIRT_PRIMARY_ATTR void primary_kernel(DevScene sc, FrameConst f, uint32_t* __restrict__ out,
                                                      float* __restrict__ acc, Deferred dfr,
                                                      BounceRec* __restrict__ queue, uint32_t* __restrict__ qctl,
                                                      int octants = 1)
{
    __shared__ uint32_t cstack[ORD ? 1 : kMaxDepth * 256];
    Counters cnt{0, 0, 0, 0, 0};
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    // the workgroup's first bounces, grouped by direction octant before they
    // enter the queue (the last of the four waves to finish writes them)
    __shared__ BounceRec grec[ORD ? 256 : 1];
    __shared__ uint32_t gcount[4], gdone;
    if (ORD) {
        if (threadIdx.x == 0) gdone = 0;
        __syncthreads();
    }
    if (!ORD && (int)blockIdx.x < dfr.blocks) {  // zero-component camera rays: whole path in this wave
        const uint32_t n = __builtin_amdgcn_readfirstlane(*dfr.count);
        const uint32_t stride = (uint32_t)(dfr.blocks * 4);
        for (uint32_t j = blockIdx.x * 4 + wave; j < n; j += stride) {
            const uint32_t p = __builtin_amdgcn_readfirstlane(dfr.list[j]);
            render_pixel<FAST, false>(sc, f, (int)(p % f.width), (int)(p / f.width), lane == 0, false,
                                                     out, acc, cnt, cstack + threadIdx.x, 256);
        }
        return;
    }
    const int tile = (blockIdx.x - dfr.blocks) * 4 + wave;
    int x, r;
    bool alive;
    if (ORD && f.samples >= 4) {
        // four frames in flight or more (frames of one camera, or jittered
        // samples of one pixel): a packet is 4x4 pixels x 4 successive frames,
        // whose camera rays are the same or nearly so -- a quarter of an 8x8
        // tile's footprint, so the packet's walk is the union of fewer paths
        // (launch_render_body's ptiles counts these tiles)
        const int txs = (f.width + 3) >> 2, tys = (f.shard_rows + 3) >> 2;
        const int g = tile / (txs * tys), rem = tile - g * (txs * tys);
        x = (rem % txs) * 4 + (lane & 3);
        const int yr = (rem / txs) * 4 + ((lane >> 2) & 3);
        const int j = g * 4 + (lane >> 4);
        alive = x < f.width && yr < f.shard_rows && j < f.samples;
        r = j * f.shard_rows + yr;
    } else {
        const int tiles_x = (f.width + 7) >> 3;
        x = (tile % tiles_x) * 8 + (lane & 7);
        r = (tile / tiles_x) * 8 + (lane >> 3);
        alive = x < f.width && r < f.num_rows;
    }
    const int y = alive ? shard_row_to_y(f, r) : 0;
    const Ray ray = camera_ray(f, alive ? x : 0, y, row_sample(f, r));
    if (!ORD && dfr.blocks > 0 && alive && slab_ray(ray).generic) alive = false;  // traced by a deferred wave
    float t;
    int s;
    if constexpr (ORD) {
        closest_packet_ordered<FAST, false, BND>(sc, ray, alive, t, s, cnt);
    } else
        closest_hit<true, FAST, false>(sc, ray, alive, t, s, cnt);
    const size_t i = (size_t)r * f.width + x;
    bool push = false;
    BounceRec rec;
    if (alive) {
        if (s < 0) {
            store_pixel(f, out, acc, i, sky_rgba(ray.dy));      // renderer.c:65-70
        } else if (f.depth < 2) {
            // depth 1: the bounce would be traced with depth 0 and return
            // black (renderer.c:23-24), so the pixel is base + 0.5 * black
            store_pixel(f, out, acc, i, blend_rgba(sc.color[s], 255u << 24));
        } else {
            // renderer.c:49-55: base colour, then the bounce (depth >= 2 here)
            const float4 g = sc.geo[s];
            float p[3], n[3];
            hit_point_normal(ray, t, g, p, n);
            uint32_t k = 0;
            float bx, by, bz;
            hemisphere(pixel_key(f.seed, (uint32_t)(y * f.width + x), row_sample(f, r)), k, n, bx, by, bz);
            rec = BounceRec{p[0], p[1], p[2], bx, by, bz, (uint32_t)i, k, sc.color[s], 0u};
            push = true;
        }
    }
    const uint64_t pm = __ballot(push);
    if constexpr (ORD) {
        if (push) grec[wave * 64 + lanes_below(pm)] = rec;
        if (lane == 0) gcount[wave] = (uint32_t)__popcll(pm);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        uint32_t prev = 0;
        if (lane == 0) prev = __hip_atomic_fetch_add(&gdone, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        if (__builtin_amdgcn_readfirstlane(prev) != (blockDim.x >> 6) - 1) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // the last wave: octant of each record's direction, counts per
        // (wave, octant), then every record to base + its octant's offset.
        // octants == 0 (a frame alone on its ctx: the blocking call): tile
        // order, still one queue atomic per workgroup -- measured (DESIGN
        // §8): the lone frame's bounce pass is 2-4% shorter in tile order,
        // frames in flight are 1% faster grouped
        const int nw = blockDim.x >> 6;
        uint32_t oct[4], tot[8] = {0, 0, 0, 0, 0, 0, 0, 0}, total = 0;
        bool has[4];
        for (int w = 0; w < nw; w++) {
            const uint32_t n = gcount[w];
            has[w] = (uint32_t)lane < n;
            const BounceRec& r = grec[w * 64 + (has[w] ? lane : 0)];
            oct[w] = octants ? (r.dx < 0.0f ? 1u : 0u) | (r.dy < 0.0f ? 2u : 0u) | (r.dz < 0.0f ? 4u : 0u) : 0u;
            for (uint32_t o = 0; o < 8; o++) tot[o] += (uint32_t)__popcll(__ballot(has[w] && oct[w] == o));
            total += n;
        }
        if (!total) return;
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&qctl[0], total);
        base = __builtin_amdgcn_readfirstlane(base);
        uint32_t run[8];
        for (uint32_t o = 0, acc = 0; o < 8; o++) {
            run[o] = base + acc;
            acc += tot[o];
        }
        for (int w = 0; w < nw; w++) {
            uint32_t pos = 0;
            for (uint32_t o = 0; o < 8; o++) {
                const uint64_t m = __ballot(has[w] && oct[w] == o);
                if (has[w] && oct[w] == o) pos = run[o] + lanes_below(m);
                run[o] += (uint32_t)__popcll(m);
            }
            if (has[w]) queue[pos] = grec[w * 64 + lane];
        }
        return;
    }
    if (pm) {  // one atomic per wave; records stay in tile order
        const int leader = __builtin_ctzll(pm);
        uint32_t base = 0;
        if (lane == leader) base = atomicAdd(&qctl[0], (uint32_t)__popcll(pm));
        base = __builtin_amdgcn_readlane(base, leader);
        if (push) queue[base + lanes_below(pm)] = rec;
    }
}

// The bounce kernel's walks test the HNode slot boxes without
// slab_cons_fast's margins (trace.h, BND): the boxes are grown by 2^-19
// DevScene::o_bound at upload, and a bounce ray whose origin lies within that
// bound -- a hit point in the scene -- needs no more; an origin beyond it (or
// NaN) takes the exact test. Round 6: serial bounce pass 0.84-0.86 ->
// 0.83 ms, 1080p/10k +1.5-3%, 1080p/100k +3.5% (MEASUREMENTS.md §D).
constexpr bool kBoundedSlab = true;
__device__ __forceinline__ SlabRay bounce_slab_ray(const DevScene& sc, const Ray& ray)
{
    SlabRay s = slab_ray(ray);
    s.generic = s.generic || !(fmaxf(fabsf(ray.ox), fmaxf(fabsf(ray.oy), fabsf(ray.oz))) <= sc.o_bound);
    return s;
}

// The walk of one bounce ray: WALK 0 = reference DFS order (any tree),
// 2 = ordered four-wide (HNode, LDS stack).
template <int WALK>
struct BounceWalk;
template <>
struct BounceWalk<0> {
    DfsWalk w;
    __device__ void start(const DevScene& sc) { w = DfsWalk{0u, sc.num_nodes}; }
    __device__ void stop() { w = DfsWalk{kPNone, 0u}; }
    __device__ bool walking() const { return w.cur != kPNone; }
    template <bool FAST>
    __device__ void step(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr, uint32_t*, float& bt,
                         int& bs, Counters& cnt)
    {
        lane_step<FAST, false>(sc, sr, sp, pr, w.cur, bt, bs, cnt);
        if (w.cur >= w.end) w.cur = kPNone;
    }
};
template <int WALK>
struct WideBounceWalk {  // WALK 2: four-wide; 4: four-wide, a step's leaf spheres loaded together
    WideWalk w;
    lds_uint4* hc = nullptr;  // the top HNodes staged in LDS (bounce_kernel)
    uint32_t hc_n = 0;
    __device__ void start(const DevScene& sc) { w = wide_walk_start(sc, true); }
    __device__ void stop() { w = WideWalk{kPNone, 0u, 0u}; }
    __device__ bool walking() const { return wide_walking(w); }
    template <bool FAST>
    __device__ void step(const DevScene& sc, const SlabRay& sr, const SphRay& sp, Prune& pr, uint32_t* stk,
                         float& bt, int& bs, Counters& cnt)
    {
        // the bounded test in WALK 2; WALK 4 (trees past the L2) keeps the
        // margins: with its batched leaf loads the bounded form spills more
        // (4K/1M: -8%, MEASUREMENTS.md §D)
        wide_lane_step<FAST, false, WALK == 4, kBoundedSlab && WALK != 4>(sc, sr, sp, pr, w, stk, bt, bs, cnt, hc,
                                                                          hc_n);
    }
};
template <>
struct BounceWalk<2> : WideBounceWalk<2> {};
template <>
struct BounceWalk<4> : WideBounceWalk<4> {};

// DIAG (mirt_bounce_stats): per wave {loop iterations, walking lanes summed
// over them, the same two after the queue ran dry, start / queue-dry / end
// time (100 MHz clock), longest chain << 32 | longest walk (in steps)}.

// Dynamic LDS of a bounce launch: the colour stack's rows for a frame of
// `depth` levels (bounce levels 1 .. depth - 1 store a colour each).
inline size_t bounce_lds_bytes(int depth) { return sizeof(uint32_t) * 256 * (size_t)std::max(depth - 1, 1); }

// The RNG key of the pixel a bounce chain belongs to (rng.h: the per-pixel
// stream of its full-frame index and sample), recomputed where a level is
// shaded rather than held in two registers for the whole walk.
__device__ __forceinline__ uint64_t chain_key(const FrameConst& f, uint32_t pixel)
{
    const int r = (int)(pixel / (uint32_t)f.width), x = (int)(pixel - (uint32_t)r * (uint32_t)f.width);
    return pixel_key(f.seed, (uint32_t)(shard_row_to_y(f, r) * f.width + x), row_sample(f, r));
}

// The shading of one lane whose walk for this level is done (renderer.c:46-77
// for that level): returns true if the chain goes on (ray re-aimed); else the
// pixel's colour is folded from the colour stack and stored (if `store`).
__device__ __forceinline__ bool shade_level(const DevScene& sc, const FrameConst& f, Ray& ray, float best_t,
                                            int best_s, int& level, uint32_t& k, uint64_t key, uint32_t* cs,
                                            int cstride, uint32_t base0, uint32_t pixel, uint32_t* __restrict__ out,
                                            float* __restrict__ acc, bool store)
{
    uint32_t tail = 255u << 24;  // depth exhausted: black (renderer.c:23-24)
    int stored = level - 1;
    if (best_s < 0) {
        tail = sky_rgba(ray.dy);
    } else {
        cs[(level - 1) * cstride] = sc.color[best_s];
        stored = level;
        if (level + 1 < f.depth) {  // trace_ray(bounce, depth - 1) still has depth
            const float4 g = sc.geo[best_s];
            float p[3], nn[3];
            hit_point_normal(ray, best_t, g, p, nn);
            float bx, by, bz;
            hemisphere(key, k, nn, bx, by, bz);
            ray = Ray{p[0], p[1], p[2], bx, by, bz};
            level++;
            return true;
        }
    }
    uint32_t c = tail;
    for (int l = stored - 1; l >= 0; l--) c = blend_rgba(cs[l * cstride], c);
    if (store) store_pixel(f, out, acc, pixel, blend_rgba(base0, c));
    return false;
}


// The rest of the chain of the wave's one remaining ray (held by the quad of
// lane l0), every lane of the wave taking part: its state broadcast from l0,
// its stack moved from its source lane's column to the wave layout of
// solo_step, each level walked with solo_step and shaded as shade_level
// (lane 0 stores the pixel).
template <bool FAST, bool BND>
__device__ __forceinline__ void solo_chain(const DevScene& sc, const FrameConst& f, int l0, Ray ray, float best_t,
                                        int best_s, Prune pr, QuadWalk qw, int level, uint32_t k, uint32_t pixel,
                                        uint32_t base0, uint32_t src, uint32_t* wst, uint32_t* wcs,
                                        uint32_t* __restrict__ out, float* __restrict__ acc, lds_uint4* hc,
                                        uint32_t hc_n)
{
    const uint32_t lane = threadIdx.x & 63;
    auto bu = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_readlane((int)v, l0); };
    auto bf = [&](float v) { return __uint_as_float(bu(__float_as_uint(v))); };
    ray = Ray{bf(ray.ox), bf(ray.oy), bf(ray.oz), bf(ray.dx), bf(ray.dy), bf(ray.dz)};
    best_t = bf(best_t);
    best_s = (int)bu((uint32_t)best_s);
    pr = Prune{bf(pr.m), bf(pr.lim)};
    level = (int)bu((uint32_t)level);
    k = bu(k);
    pixel = bu(pixel);
    base0 = bu(base0);
    src = bu(src);
    const uint32_t cur = bu(qw.cur), end = bu(qw.end), top = bu(qw.top);
    // the stack (top <= kWideStack entries, column src) to the wave layout
    uint32_t v = 0;
    if (lane < top) v = wst[lane * kWideStride + src];
    __builtin_amdgcn_wave_barrier();
    if (lane < top) *solo_slot(wst, lane) = v;
    uint32_t* cs = wcs + src;  // the colour stack stays in the source column
    SlabRay sr = bounce_slab_ray(sc, ray);
    SphRay sp = sph_ray(ray);
    SoloWalk w{lane < 4 ? cur : kPNone, lane < 4 ? end : 0u, top};
    for (;;) {
        while (solo_step<FAST, kWideStack * 64, BND>(sc, sr, sp, pr, w, wst, best_t, best_s, hc, hc_n)) {
        }
        if (!shade_level(sc, f, ray, best_t, best_s, level, k, chain_key(f, pixel), cs, kWideStride, base0, pixel, out,
                         acc, lane == 0))
            return;
        sr = bounce_slab_ray(sc, ray);
        sp = sph_ray(ray);
        w = SoloWalk{lane < 4 ? sc.wide_root : kPNone, 0u, 0u};
        best_t = INFINITY;
        best_s = -1;
        pr = prune_off();
    }
}

// Persistent bounce pass: each lane owns one pixel's chain of bounces,
// refilled from the primary pass's queue. WALK 2 (default) ends with a QUAD
// DRAIN: once the queue is dry and at most 16 of
// a wave's lanes are still busy, their chains move to quads (registers by
// ds_bpermute; the LDS stacks stay in the source lane's columns) and are
// finished four lanes per ray -- a sparse wave costs full issue slots per
// step, so four lanes per ray make the drain's steps about four times
// shorter at no extra cost.
// Register budget of the bounce kernel: 5 waves per SIMD (<= 96 VGPRs; 4
// without the attribute, at 114). The pipelined frames gain most: the
// co-running primary pass gets the issue slots the fifth wave hides.
#define MIRT_BOUNCE_ATTR __attribute__((amdgpu_waves_per_eu(MIRT_BOUNCE_WAVES)))
template <bool FAST, int WALK, bool DIAG = false>
__global__ __launch_bounds__(256) MIRT_BOUNCE_ATTR void bounce_kernel(DevScene sc, FrameConst f, uint32_t* __restrict__ out,
                                                     float* __restrict__ acc, const BounceRec* __restrict__ queue,
                                                     uint32_t* __restrict__ qctl, int threshold, int quad_drain,
                                                     uint64_t* __restrict__ diag = nullptr)
{
    uint64_t dg_it = 0, dg_lanes = 0, dg_it_x = 0, dg_lanes_x = 0, dg_tx = 0, dg_qit = 0, dg_tq = 0;
    const uint64_t dg_t0 = DIAG ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t dg_steps = 0, dg_chain = 0, dg_walk_max = 0, dg_chain_max = 0;
    uint64_t dg_seg = 0, dg_fb = 0;
    constexpr bool LANE4 = WALK == 2 || WALK == 4;  // four-wide, one ray per lane
    constexpr int cstride = 256;
    // the colour stack: one row per bounce level that can store a colour
    // (levels 1 .. depth - 1), sized at launch (bounce_lds_bytes): a depth-5
    // frame needs 4 of kMaxDepth's 8 rows, and the 4 KB it leaves free per
    // workgroup is room for the co-running frames' workgroups
    extern __shared__ uint32_t cstack[];
    __shared__ uint32_t wstack[LANE4 ? kWideStack * kWideStride : 1];
    __shared__ uint32_t qsrc[LANE4 ? 4 * 16 : 1];  // quad drain: source lane of each quad, per wave
    // the tree's top levels (the first kHCache HNodes, breadth-first) in LDS:
    // every bounce walk starts there, so those steps skip the vector-memory
    // path (TD, the kernel's busiest unit)
    __shared__ uint4 hcache[LANE4 ? 4 * kHCache : 1];
    uint32_t hc_n = 0;
    if constexpr (LANE4) {
        hc_n = min((uint32_t)kHCache, sc.num_hnodes);
        const uint4* src = (const uint4*)sc.hnodes;
        for (uint32_t i = threadIdx.x; i < 4 * hc_n; i += blockDim.x) hcache[i] = src[i];
        __syncthreads();
    }
    uint32_t* cs = cstack + threadIdx.x;
    uint32_t* stk = wstack + (LANE4 ? threadIdx.x : 0);
    Counters cnt{0, 0, 0, 0, 0};
    const uint32_t n = __builtin_amdgcn_readfirstlane(qctl[0]);
    uint32_t seg = blockIdx.x % kQSeg, segs_left = kQSeg;  // wave-uniform
    bool has = false, exhausted = false;
    Ray ray{0, 0, 0, 0, 0, 0};
    SlabRay sr = bounce_slab_ray(sc, ray);
    SphRay sp = sph_ray(ray);
    Prune pr = prune_off();
    BounceWalk<WALK> w;
    if constexpr (LANE4) {
        w.hc = (lds_uint4*)hcache;
        w.hc_n = hc_n;
    }
    w.stop();
    uint32_t pixel = 0, k = 0, base0 = 0;
    int level = 0, best_s = -1;
    float best_t = INFINITY;
    for (;;) {
        // refill lanes that own no chain (one atomic per wave, tile order
        // kept), from the next segment while the current one is dry
        const uint64_t need = __ballot(!has);
        while (need && !exhausted) {
            const int leader = __builtin_ctzll(need);
            const uint32_t lo = (uint32_t)((uint64_t)n * seg / kQSeg);
            const uint32_t sz = (uint32_t)((uint64_t)n * (seg + 1) / kQSeg) - lo;
            uint32_t b = 0;
            if ((threadIdx.x & 63) == leader) b = atomicAdd(&qctl[kQLine * (1 + seg)], (uint32_t)__popcll(need));
            b = __builtin_amdgcn_readlane(b, leader);
            if (b + (uint32_t)__popcll(need) >= sz) {  // this segment is dry: the next one
                seg = seg + 1 == kQSeg ? 0 : seg + 1;
                if (--segs_left == 0) exhausted = true;
            }
            if (!has) {
                const uint32_t lane0 = threadIdx.x & 63;
                const uint32_t idx = b + (uint32_t)__popcll(need & ((1ull << lane0) - 1));
                if (idx < sz) {
                    const BounceRec rec = queue[lo + idx];
                    ray = Ray{rec.ox, rec.oy, rec.oz, rec.dx, rec.dy, rec.dz};
                    sr = bounce_slab_ray(sc, ray);
                    sp = sph_ray(ray);
                    pixel = rec.pixel;
                    k = rec.k;
                    base0 = rec.base0;
                    level = 1;
                    w.start(sc);
                    best_t = INFINITY;
                    best_s = -1;
                    pr = prune_off();
                    has = true;
                }
            }
            if (b < sz) break;
        }
        if (!__ballot(has)) break;
        if (DIAG && exhausted && !dg_tx) dg_tx = __builtin_amdgcn_s_memrealtime();
        if (LANE4 && quad_drain && exhausted && __popcll(__ballot(has)) <= 16) break;  // -> quad drain
        // walk until few lanes are still walking and the others can make progress
        for (;;) {
            const uint64_t walking = __ballot(has && w.walking());
            if (!walking) break;
            if (__popcll(walking) < threshold &&
                (__ballot(has && !w.walking()) || (!exhausted && __ballot(!has))))
                break;
            if (DIAG) {
                dg_it++;
                dg_lanes += __popcll(walking);
                if (exhausted) {
                    dg_it_x++;
                    dg_lanes_x += __popcll(walking);
                }
                if (has && w.walking()) dg_steps++;
            }
            if constexpr (DIAG && LANE4) {
                // lane-steps spent in a DFS-segment fallback (the lane stack
                // would have overflowed), and the fallbacks entered
                const bool seg0 = has && w.walking() && w.w.end != 0;
                if (has && w.walking()) w.template step<FAST>(sc, sr, sp, pr, stk, best_t, best_s, cnt);
                dg_seg += seg0 ? 1u : 0u;
                dg_fb += (!seg0 && has && w.w.end != 0) ? 1u : 0u;
            } else {
                if (has && w.walking()) w.template step<FAST>(sc, sr, sp, pr, stk, best_t, best_s, cnt);
            }
        }
        // shade every lane whose ray is done
        if (has && !w.walking()) {
            if (DIAG) {
                dg_walk_max = max(dg_walk_max, dg_steps);
                dg_chain += dg_steps;
                dg_steps = 0;
            }
            if (shade_level(sc, f, ray, best_t, best_s, level, k, chain_key(f, pixel), cs, cstride, base0, pixel, out,
                            acc, true)) {
                sr = bounce_slab_ray(sc, ray);
                sp = sph_ray(ray);
                w.start(sc);
                best_t = INFINITY;
                best_s = -1;
                pr = prune_off();
            } else {
                has = false;
                if (DIAG) {
                    dg_chain_max = max(dg_chain_max, dg_chain);
                    dg_chain = 0;
                }
            }
        }
    }
    if constexpr (LANE4) {
        // quad drain (uniform control flow here: every lane is active)
        const uint64_t busy = __ballot(has);
        if (busy) {
            const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
            if (has) qsrc[wv * 16 + lanes_below(busy)] = lane;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t q = lane >> 2;
            const bool qhas = q < (uint32_t)__popcll(busy);
            const uint32_t src = qsrc[wv * 16 + (qhas ? q : 0)];
            auto pull = [&](uint32_t v) { return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)v); };
            auto pullf = [&](float v) { return __uint_as_float(pull(__float_as_uint(v))); };
            ray = Ray{pullf(ray.ox), pullf(ray.oy), pullf(ray.oz), pullf(ray.dx), pullf(ray.dy), pullf(ray.dz)};
            pixel = pull(pixel);
            k = pull(k);
            level = (int)pull((uint32_t)level);
            base0 = pull(base0);
            best_t = pullf(best_t);
            best_s = (int)pull((uint32_t)best_s);
            pr = Prune{pullf(pr.m), pullf(pr.lim)};
            const WideWalk& lw = w.w;
            QuadWalk qw{pull(lw.cur), pull(lw.end), pull(lw.top)};
            has = qhas;
            if (!qhas) qw.cur = kPNone;
            sr = bounce_slab_ray(sc, ray);
            sp = sph_ray(ray);
            // the ray's LDS stacks stay in its source lane's columns
            uint32_t* qstk = wstack + (threadIdx.x & ~63u) + src;
            uint32_t* qcs = cstack + (threadIdx.x & ~63u) + src;
            if (DIAG) dg_tq = __builtin_amdgcn_s_memrealtime();
            while (__ballot(has)) {
                if (DIAG) dg_qit++;
                if (!DIAG) {
                    // one ray left in the wave: every quad of the wave walks it
                    const uint64_t rays = __ballot(has && (lane & 3) == 0);
                    if (__popcll(rays) == 1) {
                        solo_chain<FAST, kBoundedSlab && WALK != 4>(sc, f, __builtin_ctzll(rays), ray, best_t, best_s, pr,
                                                                    qw, level, k, pixel,
                                         base0, src, wstack + (threadIdx.x & ~63u), cstack + (threadIdx.x & ~63u),
                                         out, acc, (lds_uint4*)hcache, hc_n);
                        break;
                    }
                }
                if (has && qw.cur != kPNone)
                    quad_step<FAST, kWideStride, kWideStack, kBoundedSlab && WALK != 4>(sc, sr, sp, pr, qw, qstk, best_t,
                                                                                        best_s,
                                                             (lds_uint4*)hcache, hc_n);
                if (has && qw.cur == kPNone) {
                    if (shade_level(sc, f, ray, best_t, best_s, level, k, chain_key(f, pixel), qcs, kWideStride, base0, pixel, out,
                                    acc, (lane & 3) == 0)) {
                        sr = bounce_slab_ray(sc, ray);
                        sp = sph_ray(ray);
                        qw = QuadWalk{sc.wide_root, 0u, 0u};
                        best_t = INFINITY;
                        best_s = -1;
                        pr = prune_off();
                    } else {
                        has = false;
                    }
                }
            }
        }
    }
    if (DIAG) {
        for (int o = 32; o; o >>= 1) {
            dg_walk_max = max(dg_walk_max, (uint32_t)__shfl_xor((int)dg_walk_max, o));
            dg_chain_max = max(dg_chain_max, (uint32_t)__shfl_xor((int)dg_chain_max, o));
        }
        if ((threadIdx.x & 63) == 0) {
            uint64_t* d = diag + kBounceDiag * (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
            d[0] = dg_it;
            d[1] = dg_lanes;
            d[2] = dg_it_x;
            d[3] = dg_lanes_x;
            d[4] = dg_t0;
            d[5] = dg_tx;
            d[6] = __builtin_amdgcn_s_memrealtime();
            d[7] = ((uint64_t)dg_chain_max << 32) | dg_walk_max;
            d[8] = dg_qit;
            d[9] = dg_tq;
        }
        // per-lane sums reduced over the wave
        for (int o = 32; o; o >>= 1) {
            dg_seg += (uint64_t)__shfl_xor((long long)dg_seg, o);
            dg_fb += (uint64_t)__shfl_xor((long long)dg_fb, o);
        }
        if ((threadIdx.x & 63) == 0) {
            uint64_t* d = diag + kBounceDiag * (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
            d[10] = dg_seg;
            d[11] = dg_fb;
        }
    }
}

// trace_ray on explicit rays (renderer.c:21); ray i uses contract pixel i.
template <bool FAST>
__global__ __launch_bounds__(256) void trace_rays_kernel(DevScene sc, const mirt_ray* __restrict__ rays, int n,
                                                         int depth, int use_bvh, uint64_t seed, uint32_t sample,
                                                         uint32_t pixel0, uint32_t* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool alive = i < n;
    const mirt_ray& rr = rays[alive ? i : 0];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    Counters cnt{0, 0, 0, 0, 0};
    __shared__ uint32_t cstack[kMaxDepth * 256];
    __shared__ uint32_t wstack[kWideStack * kWideStride];
    const uint32_t c = trace_path<FAST, false>(sc, ray, alive, depth, use_bvh != 0,
                                                  pixel_key(seed, pixel0 + (uint32_t)i, sample), cnt, cstack + threadIdx.x, 256,
                                                  wstack + threadIdx.x);
    if (alive) out[i] = c;
}

__device__ __forceinline__ void store_hit(const Ray& ray, float t, int s, const DevScene& sc, mirt_hit* o)
{
    mirt_hit h;
    memset(&h, 0, sizeof h);
    h.sphere = -1;
    if (s >= 0) {
        float p[3], nn[3];
        hit_point_normal(ray, t, sc.geo[s], p, nn);
        h.t = t;
        h.point = {p[0], p[1], p[2]};
        h.normal = {nn[0], nn[1], nn[2]};
        h.hit = 1;
        h.sphere = s;
    }
    *o = h;
}

// Brute force (renderer.c:36-43, benchmark.c:190-199) split over sphere
// chunks so that a few thousand rays still fill the chip: workgroup (bx, by)
// runs rays [256 bx, 256 bx + 256) against spheres [chunk by, chunk (by + 1)),
// every lane reading the same sphere (scalar loads, one fetch per wave).
// The chunk's best (t, index) joins keys[ray] by a 64-bit atomicMin of
// (bits(t) << 32 | index) -- t > 0 orders as its bit pattern, and on equal t
// the smaller index (the first sphere in array order) wins, as the loop's
// strict `<` does. Any-hit flags are keys != ~0: every sphere is still
// tested, as benchmark.c:190-199 does (an early exit measured slower: the
// per-sphere vote costs more than the rare hit saves).
template <bool FAST>
__global__ __launch_bounds__(256) void brute_chunk_kernel(DevScene sc, const mirt_ray* __restrict__ rays, int n,
                                                          int chunk, unsigned long long* __restrict__ keys)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    bool active = i < n;
    const mirt_ray& rr = rays[active ? i : 0];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    const SphRay sp = sph_ray(ray);
    const int s0 = (int)blockIdx.y * chunk;
    const int s1 = min(s0 + chunk, sc.num_spheres);
    float best_t = INFINITY;
    int best_s = -1;
    if (FAST && s0 < s1 && __ballot(active)) {
        brute_range_packed(sc, sp, active, s0, s1, best_t, best_s);
    } else if (s0 < s1 && __ballot(active)) {
        float4 g = load_geo_uniform(sc.geo, s0);
        for (int k = s0; k < s1; k++) {
            const float4 gn = load_geo_uniform(sc.geo, k + 1);  // [num_spheres] is the sentinel: in bounds
            if (active) {
                const float t = sphere_t<FAST>(sp, g, best_t);
                if (t > 0.0f && t < best_t) {
                    best_t = t;
                    best_s = k;
                }
            }
            g = gn;
        }
    }
    if (best_s >= 0) atomicMin(&keys[i], ((unsigned long long)__float_as_uint(best_t) << 32) | (unsigned)best_s);
}

// The hit records of brute_chunk_kernel (hit.c:32-33 for the winner).
__global__ __launch_bounds__(256) void brute_finish_kernel(DevScene sc, const mirt_ray* __restrict__ rays, int n,
                                                           const unsigned long long* __restrict__ keys,
                                                           mirt_hit* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const mirt_ray& rr = rays[i];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    const unsigned long long k = keys[i];
    const bool hit = k != ~0ull;
    store_hit(ray, hit ? __uint_as_float((uint32_t)(k >> 32)) : INFINITY, hit ? (int)(uint32_t)k : -1, sc, &out[i]);
}

// ray_bvh_intersect(...).hit_something per ray (benchmark.c:239-241).
template <bool FAST>
__global__ __launch_bounds__(256) void bvh_any_kernel(DevScene sc, const mirt_ray* __restrict__ rays, int n,
                                                      int32_t* __restrict__ out)
{
    __shared__ uint32_t wstack[kWideStack * kWideStride];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool alive = i < n;
    const mirt_ray& rr = rays[alive ? i : 0];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    Counters cnt{0, 0, 0, 0, 0};
    float t;
    int s;
    closest_hit<false, FAST, false>(sc, ray, alive, t, s, cnt, wstack + threadIdx.x);
    if (alive) out[i] = s >= 0 ? 1 : 0;
}

__global__ void keys_to_flags_kernel(const unsigned long long* __restrict__ keys, int n, int32_t* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = keys[i] != ~0ull ? 1 : 0;
}

// ray_bvh_intersect (hit.c:91) / brute-force closest hit (renderer.c:36-43)
template <bool FAST>
__global__ __launch_bounds__(256) void intersect_kernel(DevScene sc, const mirt_ray* __restrict__ rays, int n,
                                                        int use_bvh, mirt_hit* __restrict__ out)
{
    __shared__ uint32_t wstack[kWideStack * kWideStride];
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool alive = i < n;
    const mirt_ray& rr = rays[alive ? i : 0];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    Counters cnt{0, 0, 0, 0, 0};
    float t;
    int s;
    // arbitrary rays are incoherent: per-lane walks (four-wide where the
    // tree admits it, each lane with its LDS stack column), not packets
    if (use_bvh)
        closest_hit<false, FAST, false>(sc, ray, alive, t, s, cnt, wstack + threadIdx.x);
    else
        closest_brute<FAST, false>(sc, ray, alive, t, s, cnt);
    if (alive) store_hit(ray, t, s, sc, &out[i]);
}

// ray_bvh_intersect (hit.c:91-109) for a batch too small to fill the chip
// one ray per lane (benchmark.c's 10,000 rays): one ray per QUAD of lanes,
// lane j testing slot j of every four-wide node (quad_step, the bounce
// kernel's drain walk), so each ray's dependent chain of node fetches is
// walked by four lanes and the batch occupies four times the lanes. The
// tree's top HNodes are staged in LDS; rays with a zero/tiny direction
// component take the exact wave-cooperative walk afterwards (closest_hit).
// ANY: the hit flag (benchmark.c:239-241), else the hit record.
constexpr int kQuadBatchThreads = 64;  // 16 rays per workgroup: a small batch spreads over the CUs
template <bool ANY>
__global__ __launch_bounds__(kQuadBatchThreads) void intersect_quad_kernel(DevScene sc, const mirt_ray* __restrict__ rays,
                                                                          int n, mirt_hit* __restrict__ out,
                                                                          int32_t* __restrict__ flags)
{
    constexpr int kRays = kQuadBatchThreads / 4;
    __shared__ uint32_t qstack[kWideStack * kRays];
    __shared__ uint4 hcache[4 * kHCache];
    const uint32_t hc_n = min((uint32_t)kHCache, sc.num_hnodes);
    for (uint32_t i = threadIdx.x; i < 4 * hc_n; i += blockDim.x) hcache[i] = ((const uint4*)sc.hnodes)[i];
    __syncthreads();
    const int q = (int)(threadIdx.x >> 2);
    const int i = (int)blockIdx.x * kRays + q;
    const bool alive = i < n;
    const mirt_ray& rr = rays[alive ? i : 0];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    const SlabRay sr = slab_ray(ray);
    const SphRay sp = sph_ray(ray);
    Prune pr = prune_off();
    const bool gen = alive && sr.generic;
    float best_t = INFINITY;
    int best_s = -1;
    QuadWalk qw{alive && !gen ? sc.wide_root : kPNone, 0u, 0u};
    while (__ballot(qw.cur != kPNone)) {
        if (qw.cur != kPNone)
            quad_step<true, kRays, kWideStack>(sc, sr, sp, pr, qw, qstack + q, best_t, best_s, (lds_uint4*)hcache, hc_n);
    }
    uint64_t gm = __ballot(gen && (threadIdx.x & 3) == 0);
    while (gm) {  // zero-component rays: the exact chunked walk, one ray per wave pass
        const int l = __builtin_ctzll(gm);
        gm &= gm - 1;
        const Ray g{readlane_f(ray.ox, l), readlane_f(ray.oy, l), readlane_f(ray.oz, l),
                    readlane_f(ray.dx, l), readlane_f(ray.dy, l), readlane_f(ray.dz, l)};
        float t;
        int s2;
        Counters c2{0, 0, 0, 0, 0};
        closest_bvh_chunked<true, false>(sc, g, t, s2, c2);
        if ((int)(threadIdx.x & 63) >> 2 == l >> 2) {
            best_t = t;
            best_s = s2;
        }
    }
    if (alive && (threadIdx.x & 3) == 0) {
        if (ANY)
            flags[i] = best_s >= 0 ? 1 : 0;
        else
            store_hit(ray, best_t, best_s, sc, &out[i]);
    }
}

// element-wise ray_sphere_intersect (hit.c:19-39)
__global__ void sphere_pairs_kernel(const mirt_ray* __restrict__ rays, const mirt_sphere* __restrict__ sph, int n,
                                    mirt_hit* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const mirt_ray rr = rays[i];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    const float4 g = make_float4(sph[i].center.x, sph[i].center.y, sph[i].center.z, sph[i].radius);
    const float t = sphere_t<false>(sph_ray(ray), g, INFINITY);
    mirt_hit h;
    memset(&h, 0, sizeof h);
    h.sphere = -1;
    if (t > 0.0f) {
        float p[3], nn[3];
        hit_point_normal(ray, t, g, p, nn);
        h.t = t;
        h.point = {p[0], p[1], p[2]};
        h.normal = {nn[0], nn[1], nn[2]};
        h.hit = 1;
        h.sphere = i;
    }
    out[i] = h;
}

// element-wise ray_aabb_intersect (hit.c:49-82)
__global__ void aabb_pairs_kernel(const mirt_ray* __restrict__ rays, const mirt_aabb* __restrict__ boxes, int n,
                                  int32_t* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const mirt_ray rr = rays[i];
    const Ray ray{rr.origin.x, rr.origin.y, rr.origin.z, rr.direction.x, rr.direction.y, rr.direction.z};
    const mirt_aabb b = boxes[i];
    out[i] = slab_test(slab_ray(ray), b.min.x, b.min.y, b.min.z, b.max.x, b.max.y, b.max.z) ? 1 : 0;
}

__global__ void camera_rays_kernel(FrameConst f, mirt_ray* __restrict__ out)
{
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int r = blockIdx.y;
    if (x >= f.width || r >= f.num_rows) return;
    const Ray ray = camera_ray(f, x, shard_row_to_y(f, r), row_sample(f, r));
    out[(size_t)r * f.width + x] = {{ray.ox, ray.oy, ray.oz}, {ray.dx, ray.dy, ray.dz}};
}

// get_camera_ray (ray.c:17-32) at caller-given (u, v): the batched form of
// the per-ray call, for callers that build their own pixel loop.
__global__ void camera_uv_kernel(FrameConst f, const float2* __restrict__ uv, int n, mirt_ray* __restrict__ out)
{
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float u = uv[i].x, v = uv[i].y;
    float dx = f.fx + f.hx * u, dy = f.fy + f.hy * u, dz = f.fz + f.hz * u;
    dx = dx + f.vx * v;
    dy = dy + f.vy * v;
    dz = dz + f.vz * v;
    normalize3(dx, dy, dz);
    out[i] = {{f.px, f.py, f.pz}, {dx, dy, dz}};
}

// ---------------------------------------------------------------- BVH overlay
// The debug view of bvh_visualiser.c:16-126 ('o' in main.c:323-327): every
// node's box (pre-order, bvh_visualiser.c:110-116) as 12 projected edges
// (draw_aabb :71-99), each drawn 5 times offset by one pixel (draw_debug_line
// :45-68), coloured by depth (:107-110) over a cleared black screen. Later
// lines overwrite earlier ones, so a pixel shows the LAST line (in draw
// order) that covers it: pass 1 rasterises every line and keeps the largest
// draw index per pixel (atomicMax), pass 2 colours. Rasterisation (SDL's
// depends on the backend; the reference marks the view "NOT WORKING") is the
// build's definition: Bresenham over integer endpoints, both inclusive,
// pixels off screen skipped.
struct OverlayConst {
    float px, py, pz, fx, fy, fz, rx, ry, rz, ux, uy, uz;
    float half_w, half_h;  // host: tanf (glibc) as bvh_visualiser.c:27-30
    int width, height, max_levels;
};

// (int)x of x86 (cvttss2si): NaN and out-of-range values give INT_MIN.
__device__ __forceinline__ int x86_trunc(float x)
{
    return (x > -2147483648.0f && x < 2147483648.0f) ? (int)x : INT_MIN;
}

// world_to_screen, bvh_visualiser.c:16-41 (float arithmetic, no contraction)
__device__ __forceinline__ int2 world_to_screen(const OverlayConst& o, float x, float y, float z)
{
    const float tx = x - o.px, ty = y - o.py, tz = z - o.pz;
    const float zz = tx * o.fx + ty * o.fy + tz * o.fz;
    if (zz <= 0.1f) return make_int2(-1, -1);
    const float xx = tx * o.rx + ty * o.ry + tz * o.rz;
    const float yy = tx * o.ux + ty * o.uy + tz * o.uz;
    const float sx = (xx / (zz * o.half_w * 2.0f) + 0.5f) * (float)o.width;
    const float sy = (-yy / (zz * o.half_h * 2.0f) + 0.5f) * (float)o.height;
    if (sx < (float)-o.width || sx > (float)(o.width * 2) || sy < (float)-o.height || sy > (float)(o.height * 2))
        return make_int2(-1, -1);
    return make_int2(x86_trunc(sx), x86_trunc(sy));
}

__constant__ int kBoxEdge[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6},
                                    {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
__constant__ int kLineOffset[5][2] = {{0, 0}, {1, 0}, {0, 1}, {-1, 0}, {0, -1}};

// one thread per (node, edge, offset): draw index (node * 12 + edge) * 5 + offset
__global__ void overlay_lines_kernel(OverlayConst o, const mirt_node* __restrict__ nodes,
                                     const uint8_t* __restrict__ ndepth, uint32_t count, uint32_t* __restrict__ last)
{
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    if (id >= count) return;
    const uint32_t node = id / 60, edge = (id / 5) % 12, off = id % 5;
    if (o.max_levels >= 0 && ndepth[node] >= o.max_levels) return;
    const mirt_node nd = nodes[node];
    auto corner = [&](int k) {  // draw_aabb's corner order (:73-82)
        const int hx = (k == 1 || k == 2 || k == 5 || k == 6), hy = (k == 2 || k == 3 || k == 6 || k == 7), hz = k >= 4;
        return world_to_screen(o, hx ? nd.bmax[0] : nd.bmin[0], hy ? nd.bmax[1] : nd.bmin[1],
                               hz ? nd.bmax[2] : nd.bmin[2]);
    };
    const int2 a = corner(kBoxEdge[edge][0]), b = corner(kBoxEdge[edge][1]);
    if (a.x == -1 || b.x == -1) return;  // :49 (tests x only)
    const int W = o.width, H = o.height;
    if (!(a.x >= -W && a.x <= W * 2 && a.y >= -H && a.y <= H * 2 && b.x >= -W && b.x <= W * 2 && b.y >= -H &&
          b.y <= H * 2))
        return;  // :51-54
    int x0 = a.x + kLineOffset[off][0], y0 = a.y + kLineOffset[off][1];
    const int x1 = b.x + kLineOffset[off][0], y1 = b.y + kLineOffset[off][1];
    const uint32_t tag = id + 1;
    const int dx = abs(x1 - x0), dy = -abs(y1 - y0), sx = x0 < x1 ? 1 : -1, sy = y0 < y1 ? 1 : -1;
    int err = dx + dy;
    for (;;) {
        if (x0 >= 0 && x0 < W && y0 >= 0 && y0 < H) atomicMax(&last[(size_t)y0 * W + x0], tag);
        if (x0 == x1 && y0 == y1) break;
        const int e2 = 2 * err;
        if (e2 >= dy) {
            err += dy;
            x0 += sx;
        }
        if (e2 <= dx) {
            err += dx;
            y0 += sy;
        }
    }
}

__global__ void overlay_colour_kernel(const uint32_t* __restrict__ last, const uint8_t* __restrict__ ndepth,
                                      size_t n, uint32_t* __restrict__ out)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t v = last[i];
    uint32_t c = 0xff000000u;  // SDL_RenderClear with (0, 0, 0, 255), main.c:342-343
    if (v) {
        const uint32_t d = ndepth[(v - 1) / 60];
        const uint32_t r = 255 - (d * 40) % 200, g = (d * 80) % 200, b = (d * 120) % 200;  // :107-110
        c = r | g << 8 | b << 16 | 180u << 24;
    }
    out[i] = c;
}

}  // namespace

// ------------------------------------------------------------------ context

constexpr int kPhaseRing = 64;  // frames of pass timings kept per ctx (mirt_phase_log)

// The float accumulation buffer of main.c:241-273 (x-major there, row-major
// float3 here). One per ctx by default; mirt_ctx_share_accum lets the ctxs
// that keep frames of one display loop in flight (main.c:379-408, one ctx
// per hardware queue) use ONE buffer: every frame's colours then go to its
// own slab and a fold kernel adds them to the buffer, the folds of
// successive calls ordered across the ctxs' streams by `folded` (the event
// of the last fold enqueued, on whichever stream) -- the tracing overlaps,
// only the folds (a few microseconds each) run in call order.
struct AccumShare {
    int refs = 1;
    int device = 0;
    float* d_acc = nullptr;
    size_t cap = 0;          // bytes allocated
    size_t pixels = 0;       // pixels of the running accumulation (0: none yet)
    hipEvent_t folded = nullptr;
    bool has_fold = false;   // `folded` was recorded at least once
    // Lazy fold (round 5): the display slab of the last FRESH
    // frame issued on the share and not yet folded into d_acc. A fresh
    // frame's accumulation state is its colours / 255 (main.c:368-370), which
    // its slab holds exactly, so it is folded only when a frame or a read
    // needs d_acc (accum_materialize) -- fresh frames in flight no longer wait
    // for each other's folds, and a fresh frame superseded by a later one is
    // never folded at all.
    const uint32_t* pend = nullptr;
    mirt_ctx* pend_ctx = nullptr;   // the ctx that rendered it (its slab must outlive the read)
    hipEvent_t pend_ev = nullptr;   // recorded after that frame's render
};
// (A launch of several fresh frames, mirt_multi at N >= 4, keeps its ordered
// fold: the lanes then finish in the order the caller rotates through them;
// its last display left pending ran the slowest shard of an 8-way split 2-4%
// slower, profiles/r05_logs/r05bc/.)



struct mirt_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    bool timed_recorded = false;  // ev0/ev1 bracket a launch (mirt_last_kernel_ms)
    float last_ms = 0.0f;
    // wavefront phase boundaries of the last frame (any API)
    // (a ring of kPhaseRing frames: mirt_phase_log reads back the passes of
    // frames that ran overlapped with other ctxs' frames, without a sync
    // between them)
    hipEvent_t ph0[kPhaseRing] = {}, ph1[kPhaseRing] = {}, ph2[kPhaseRing] = {};
    uint32_t ph_next = 0;   // ring slot of the next wavefront frame
    uint32_t ph_count = 0;  // wavefront frames recorded (saturates at kPhaseRing)
    bool phases_valid = false;
    // the frame scratch (queue, deferral list, phase events) is per ctx: a
    // launch on another stream than the previous one waits for it
    hipEvent_t done = nullptr;
    // Lazy fold: another stream read this ctx's display slab for the
    // share's pending fold; the ctx's next write to it waits for `slab_free`
    hipEvent_t slab_free = nullptr;
    bool slab_guard = false;
    hipStream_t last_stream = nullptr;
    bool launched = false;
    // scene (replicated per device, uploaded once)
    DNode* d_nodes = nullptr;
    mirt_node* d_nodes32 = nullptr;
    float4* d_geo = nullptr;
    uint32_t* d_color = nullptr;
    int num_nodes = 0, num_spheres = -1;
    // frame buffers owned by the ctx (blocking API)
    uint32_t* d_out = nullptr;
    size_t out_cap = 0;
    AccumShare* acc = nullptr;  // accumulation buffer (own, or shared: mirt_ctx_share_accum)
    // staging for batch calls
    void* d_in = nullptr;
    void* d_res = nullptr;
    size_t in_cap = 0, res_cap = 0;
    mirt_counts* d_counts = nullptr;
    // kernel schedule (mirt_set_option)
    int trav = kTravWavefront;
    int fast_slab = 1;
    int block_waves = 4;  // waves (8x8 tiles) per workgroup
    int defer = 1;        // trace zero-component camera rays in leading waves
    int prune = 1;              // closest-hit pruning (trace.h Prune), FAST slab only
    bool prune_ok = false;      // the uploaded tree's boxes enclose their subtrees
    PNode* d_pnodes = nullptr;  // ordered-walk layout of the tree
    bool ordered_ok = false;    // leaves in DFS order hold increasing sphere indices, depth < 63
    int ordered = 1;            // ordered (nearer-child-first) walks where the tree admits them
    HNode* d_hnodes = nullptr;  // four-wide layout (per-lane walks)
    HAux* d_haux = nullptr;
    char* d_leaves = nullptr;   // leaf spheres (float4 each), then at leaf_box_off the leaf boxes (LeafBox each)
    size_t leaf_box_off = 0;
    uint32_t num_hnodes = 0;
    uint32_t wide_root = 0;     // HNode a four-wide walk starts at (DevScene::wide_root)
    uint8_t* d_ndepth = nullptr;  // depth of every flat node (BVH overlay colours)
    uint32_t* d_overlay = nullptr;  // BVH overlay: per-pixel last line in draw order
    size_t overlay_cap = 0;
    float r_max = 0.0f, c_max = 0.0f;
    float o_bound = 0.0f;       // the bounce walks' origin bound the HNode boxes were grown for
    int bounce_threshold = 20;  // wavefront: shade finished rays once fewer lanes walk (swept: profiles/r02thr_threshold_sweep.txt)
    int bounce_blocks = 0;      // wavefront: persistent workgroups (set in mirt_create)
    int bounce_blocks_opt = 0;  // MIRT_OPT_BOUNCE_BLOCKS override (0: occupancy x CUs)
    int quad_drain = 1;         // four-wide bounce walk: finish the drain four lanes per ray
    int quad_batch = 1;                          // small BVH batches one ray per quad (intersect_quad_kernel)
    int leaf_batch_opt = 2;                        // MIRT_OPT_LEAF_BATCH: 0 off, 1 on, 2 auto (leaf_big)
    int zero_copy = 1;          // MIRT_OPT_ZERO_COPY: blocking frames into page-locked memory written in place
    bool leaf_big = false;      // the four-wide tree (HNodes + leaves) exceeds the chip's L2
    void* d_queue = nullptr;    // wavefront: {count, head} + bounce records
    size_t queue_cap = 0;
    bool lone_frame = false;    // mirt_render_frame's frame: the first bounces queued in tile order
    int queue_order = 0;        // MIRT_OPT_QUEUE_ORDER: 0 auto (tile order for lone_frame), 1 octants, 2 tile order
    uint32_t* d_defer = nullptr;  // [count, list...]
    size_t defer_cap = 0;
    unsigned long long* d_keys = nullptr;  // chunked brute force: per-ray (t, index) keys
    size_t keys_cap = 0;
    int num_cus = 0;
    int debug_stall_ms = 0;     // MIRT_OPT_DEBUG_STALL_MS: test hook, each frame starts behind a bounded wait
};

namespace {

int hip_fail(hipError_t e, const char* what)
{
    set_error("%s: %s", what, hipGetErrorString(e));
    return MIRT_E_DEVICE;
}

#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return hip_fail(e_, #expr); \
    } while (0)

int ensure(void** p, size_t* cap, size_t bytes)
{
    if (bytes <= *cap) return MIRT_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    HIP_TRY(hipMalloc(p, bytes));
    *cap = bytes;
    return MIRT_OK;
}

// The pruning bound (trace.h Prune) holds for a tree in which every leaf box
// holds its sphere's box as bvh.c:26-46 computes it, fl(c -+ r), and every
// inner box holds both children's boxes; the reference's own trees are built
// that way. Also returns the scene constants of the bound. A NaN anywhere,
// a non-finite sphere or a tree that does not nest turns pruning off.
// A 0-sphere leaf whose sphere (hit.c:96-97 tests it) is no non-empty leaf's
// tested sphere: a tree built over part of an array (benchmark.c:317 builds
// over [0, n - 1)) whose SAH fallback left a last leaf empty points at the
// element after the range, which only that leaf tests. The pruned and
// ordered walks drop 0-sphere leaves (dead_leaf), so such a tree is walked
// in the reference's DFS order instead.
bool orphan_phantoms(const mirt_node* nd, int nn, int ns)
{
    std::vector<char> tested((size_t)ns + 1, 0);
    for (int i = 0; i < nn; i++)
        if (nd[i].sphere >= 0 && nd[i].sphere < ns && !(nd[i].skip & MIRT_NODE_EMPTY)) tested[nd[i].sphere] = 1;
    for (int i = 0; i < nn; i++)
        if (nd[i].sphere >= 0 && nd[i].sphere < ns && (nd[i].skip & MIRT_NODE_EMPTY) && !tested[nd[i].sphere])
            return true;
    return false;
}

bool tree_encloses(const mirt_sphere* sp, int ns, const mirt_node* nd, int nn, float* r_max, float* c_max)
{
    float rm = 0.0f, cm = 0.0f;
    for (int i = 0; i < ns; i++) {
        const float c[3] = {sp[i].center.x, sp[i].center.y, sp[i].center.z};
        const float r = std::fabs(sp[i].radius);
        if (!std::isfinite(c[0]) || !std::isfinite(c[1]) || !std::isfinite(c[2]) || !std::isfinite(r)) return false;
        rm = std::max(rm, r);
        cm = std::max(cm, std::max(std::fabs(c[0]), std::max(std::fabs(c[1]), std::fabs(c[2]))) + r);
    }
    auto holds = [](const mirt_node& outer, const mirt_node& inner) {
        if (inner.skip & MIRT_NODE_EMPTY) return true;  // +inf/-inf box, no sphere
        for (int k = 0; k < 3; k++)
            if (!(outer.bmin[k] <= inner.bmin[k] && outer.bmax[k] >= inner.bmax[k])) return false;
        return true;
    };
    for (int i = 0; i < nn; i++) {
        const mirt_node& n = nd[i];
        if (n.skip & MIRT_NODE_EMPTY) continue;
        if (n.sphere >= 0) {
            if (n.sphere >= ns) continue;  // the never-hit sentinel
            const mirt_sphere& s = sp[n.sphere];
            const float c[3] = {s.center.x, s.center.y, s.center.z};
            const float r = std::fabs(s.radius);
            for (int k = 0; k < 3; k++)
                if (!(n.bmin[k] <= c[k] - r && n.bmax[k] >= c[k] + r)) return false;
        } else {
            const uint32_t left = (uint32_t)i + 1, right = nd[left].skip & MIRT_SKIP_MASK;
            if (!holds(n, nd[left]) || (right < (uint32_t)nn && right < (n.skip & MIRT_SKIP_MASK) && !holds(n, nd[right])))
                return false;
        }
    }
    *r_max = rm;
    *c_max = cm;
    return true;
}

// A leaf the fast walks may drop: the &spheres[N] sentinel (never hits), or
// a 0-sphere leaf. hit.c:96-97 does test a 0-sphere leaf's sphere (its box,
// create_empty_aabb's, always passes): spheres[start] of its range when the
// SAH fallback split left it empty (mid == start: the first sphere of its
// sibling's range), spheres[end] when it split right (mid == end: a sphere
// of some LATER subtree). Dropping it is exact when that sphere is the
// tested sphere of a non-empty leaf (upload checks this, `orphan_phantoms`;
// otherwise only the reference-order DFS walk runs) and the ray reaches that
// leaf whenever it hits the sphere: the leaf's box holds the sphere's box
// fl(c -+ r) (checked, tree_encloses), the reference slab test is monotone
// under containment, so this rests on ONE assumption -- hit.c:49-82's
// division slab test passes the box fl(c -+ r) of every sphere that
// hit.c:19-39 reports hit. Both are exact-rounding computations of the same
// chord; tests/test_gpu_parity.py test_phantom_grazing_rays aims grazing rays
// at the spheres of both kinds of 0-sphere leaf and compares the fast walks
// with the DFS walk and the oracle.
bool dead_leaf(const mirt_node* nd, uint32_t i, int ns)
{
    return nd[i].sphere >= 0 && ((nd[i].skip & MIRT_NODE_EMPTY) || nd[i].sphere >= ns);
}

// The node a walk may take in place of flat node ci: an inner node one of
// whose children is dead adds nothing but its box test, which its live
// child's (nested, hence stricter) box test implies -- so the chains of
// one-sided splits the reference's SAH fallback builds (bvh.c:139-141,
// runs of nodes each with a 0-sphere leaf beside the rest of the range)
// collapse to the subtree that can hit. kPNone: nothing below can hit.
uint32_t live_node(const mirt_node* nd, uint32_t ci, int ns)
{
    for (;;) {
        if (nd[ci].sphere >= 0) return dead_leaf(nd, ci, ns) ? kPNone : ci;
        const uint32_t l = ci + 1, r = nd[ci + 1].skip & MIRT_SKIP_MASK;
        const bool dl = dead_leaf(nd, l, ns), dr = dead_leaf(nd, r, ns);
        if (dl && dr) return kPNone;
        if (!dl && !dr) return ci;
        ci = dl ? r : l;
    }
}

// PNode layout (trace.h) of a validated flat tree. Returns whether ordered
// walks may use it: hit-able leaves must carry strictly increasing sphere
// indices in DFS order (then the index is hit.c:108's tie key -- true of the
// reference's trees, whose build partitions the array in place) and the
// inner depth must leave the packet walk's stack (one entry per level)
// within 64.
// grow > 0: an inner child's box grown by `grow` on each face (rounded
// outward): the camera packets' margin-free test (trace.h); leaf children keep
// their exact boxes, which gate every sphere.
bool build_pnodes(const mirt_node* nd, int nn, const mirt_sphere* sp, int ns, std::vector<PNode>& pn, double grow)
{
    std::vector<uint32_t> pidx((size_t)nn, kPNone);
    uint32_t np = 1;
    for (int i = 0; i < nn; i++)
        if (nd[i].sphere < 0) pidx[i] = np++;
    pn.assign(np, PNode{});
    auto set_child = [&](PNode& p, int k, uint32_t c) {
        const uint32_t ci = live_node(nd, c, ns);
        if (ci == kPNone) {  // nothing below can hit: an empty slot
            float* slot = k ? p.c1 : p.c0;
            std::memcpy(slot, nd[c].bmin, sizeof nd[c].bmin);
            std::memcpy(slot + 3, nd[c].bmax, sizeof nd[c].bmax);
            (k ? p.ref1 : p.ref0) = kPNone;
            return;
        }
        const mirt_node& n = nd[ci];
        float* slot = k ? p.c1 : p.c0;
        uint32_t ref = pidx[ci];
        std::memcpy(slot, n.bmin, sizeof n.bmin);
        std::memcpy(slot + 3, n.bmax, sizeof n.bmax);
        if (n.skip & MIRT_NODE_EMPTY) {
            ref = kPNone;  // a 0-sphere leaf: passes, never hits
        } else if (n.sphere >= 0) {
            if (n.sphere >= ns || (uint32_t)n.sphere > kPIndex) {
                ref = kPNone;
            } else {
                ref = kPLeaf | (uint32_t)n.sphere;
            }
        }
        if (grow > 0.0 && ref != kPNone && !(ref & kPLeaf))
            for (int a = 0; a < 3; a++) {
                slot[a] = std::nextafter((float)((double)slot[a] - grow), -INFINITY);
                slot[3 + a] = std::nextafter((float)((double)slot[3 + a] + grow), INFINITY);
            }
        (k ? p.ref1 : p.ref0) = ref;
    };
    pn[0].ref0 = pn[0].ref1 = kPNone;
    pn[0].flat = 0xffffffffu;  // flat + 1 == 0: the whole tree
    pn[0].end = (uint32_t)nn;
    if (nn > 0) set_child(pn[0], 0, 0);
    bool mono = nn > 0;
    int last = -1;
    std::vector<uint32_t> ends;  // subtree ends of the open inner nodes
    size_t depth = 0;
    for (int i = 0; i < nn; i++) {
        while (!ends.empty() && ends.back() <= (uint32_t)i) ends.pop_back();
        if (nd[i].sphere < 0) {
            PNode& p = pn[pidx[i]];
            set_child(p, 0, (uint32_t)i + 1);
            set_child(p, 1, nd[i + 1].skip & MIRT_SKIP_MASK);
            p.flat = (uint32_t)i;
            p.end = nd[i].skip & MIRT_SKIP_MASK;
            ends.push_back(nd[i].skip & MIRT_SKIP_MASK);
            depth = std::max(depth, ends.size());
        } else if (!(nd[i].skip & MIRT_NODE_EMPTY) && nd[i].sphere < ns) {
            if (nd[i].sphere <= last) mono = false;
            last = nd[i].sphere;
        }
    }
    return mono && depth + 2 <= 64;
}

// fp16 bits of the largest half <= v / the smallest half >= v (a value
// beyond the fp16 range rounds out to -inf / +inf: still a superset).
uint16_t half_bits(float v)
{
    const _Float16 h = (_Float16)v;
    uint16_t b;
    std::memcpy(&b, &h, 2);
    return b;
}
float half_value(uint16_t b)
{
    _Float16 h;
    std::memcpy(&h, &b, 2);
    return (float)h;
}
uint16_t half_down(float v)
{
    uint16_t b = half_bits(v);
    while (half_value(b) > v) b = b == 0x0000 ? 0x8001 : (b & 0x8000) ? b + 1 : b - 1;
    return b;
}
uint16_t half_up(float v)
{
    uint16_t b = half_bits(v);
    while (half_value(b) < v) b = b == 0x8000 ? 0x0001 : (b & 0x8000) ? b - 1 : b + 1;
    return b;
}

// HNode layout (trace.h) of a validated flat tree: HNode 0 holds the root;
// an HNode for each inner node that is some HNode's slot holds that node's
// grandchildren (a leaf child standing in for its own); one leaf (sphere +
// exact box) per leaf slot. Used only when the PNode conditions hold and the boxes nest.
// grow > 0 (the bounce walks' bounded slab test): every slot box grown by `grow` on each face
// before the outward fp16 rounding.
void build_hnodes(const mirt_node* nd, int nn, const mirt_sphere* sp, int ns, std::vector<HNode>& hn,
                  std::vector<HAux>& aux, std::vector<float4>& lgeo, std::vector<LeafBox>& lbox, double grow)
{
    hn.assign(1, HNode{});
    aux.assign(1, HAux{0xffffffffu, (uint32_t)nn});  // flat + 1 == 0: the whole tree
    lgeo.clear();
    lbox.clear();
    std::vector<uint32_t> todo;  // inner nodes waiting for their HNode: HNode 1 + i is todo[i]
    auto fill = [&](size_t hi, int k, uint32_t c) {
        HNode& h = hn[hi];
        const uint32_t ci = live_node(nd, c, ns);
        if (ci == kPNone) {
            h.slot[k].ref = kPNone;
            return;
        }
        const mirt_node& n = nd[ci];
        for (int a = 0; a < 3; a++) {
            float lo = n.bmin[a], hi = n.bmax[a];
            if (grow > 0.0) {   // rounded outward again: the float of lo - grow may lie above it
                lo = std::nextafter((float)((double)lo - grow), -INFINITY);
                hi = std::nextafter((float)((double)hi + grow), INFINITY);
            }
            h.slot[k].box[a] = (uint32_t)half_down(lo) | ((uint32_t)half_up(hi) << 16);
        }
        uint32_t ref;
        if (n.skip & MIRT_NODE_EMPTY) {
            ref = kPNone;
        } else if (n.sphere >= 0) {
            if (n.sphere >= ns) {
                ref = kPNone;
            } else {
                LeafBox l{};
                std::memcpy(l.lo, n.bmin, sizeof l.lo);
                std::memcpy(l.hi, n.bmax, sizeof l.hi);
                l.sphere = n.sphere;
                const mirt_sphere& s = sp[n.sphere];
                ref = kPLeaf | (uint32_t)lbox.size();
                lbox.push_back(l);
                lgeo.push_back(make_float4(s.center.x, s.center.y, s.center.z, s.radius));
            }
        } else {
            todo.push_back(ci);
            ref = (uint32_t)todo.size();
        }
        h.slot[k].ref = ref;
    };
    for (int k = 0; k < 4; k++) hn[0].slot[k].ref = kPNone;
    if (nn == 0) return;
    fill(0, 0, 0);
    for (size_t next = 0; next < todo.size(); next++) {
        const uint32_t y = todo[next];
        HNode h{};
        for (int k = 0; k < 4; k++) h.slot[k].ref = kPNone;
        hn.push_back(h);
        aux.push_back(HAux{y, nd[y].skip & MIRT_SKIP_MASK});
        // the four slots: y's live children, then the inner slot with the
        // largest box replaced by its two live children while a slot is
        // free (every slot stays inside y's flat subtree, which HAux walks)
        uint32_t cut[4];
        int m = 0;
        auto add = [&](uint32_t c) {
            const uint32_t ci = live_node(nd, c, ns);
            if (ci != kPNone) cut[m++] = ci;
        };
        add(y + 1);
        add(nd[y + 1].skip & MIRT_SKIP_MASK);
        while (m < 4) {
            int best = -1;
            float best_area = -1.0f;
            for (int j = 0; j < m; j++) {
                const mirt_node& n = nd[cut[j]];
                if (n.sphere >= 0) continue;
                const float dx = n.bmax[0] - n.bmin[0], dy = n.bmax[1] - n.bmin[1], dz = n.bmax[2] - n.bmin[2];
                const float area = dx * dy + dy * dz + dz * dx;
                if (area > best_area || best < 0) {
                    best = j;
                    best_area = area;
                }
            }
            if (best < 0) break;
            const uint32_t c = cut[best];
            cut[best] = cut[--m];
            add(c + 1);
            add(nd[c + 1].skip & MIRT_SKIP_MASK);
        }
        for (int k = 0; k < m; k++) fill(hn.size() - 1, k, cut[k]);
    }
}

// MIRT_OPT_LEAF_BATCH: the bounce walk loads a step's passing leaf spheres
// together (bounce_kernel WALK 4) -- by default when the four-wide tree is
// larger than the chip's L2 (32 MiB over the 8 XCDs), where the leaf loads
// miss: 4K/1M +9%, 1080p/10k and 100k -9% / -6%
bool leaf_batch(const mirt_ctx* c)
{
    return c->leaf_batch_opt == 1 || (c->leaf_batch_opt == 2 && c->leaf_big);
}

DevScene dev_scene(const mirt_ctx* c)
{
    const bool prune = c->prune && c->prune_ok;
    const bool ordered = prune && c->ordered && c->ordered_ok && c->fast_slab;
    return DevScene{c->d_nodes, c->d_nodes32, c->d_geo, c->d_color, (uint32_t)c->num_nodes, c->num_spheres,
                    prune, c->r_max, c->c_max, c->d_pnodes, ordered, c->d_hnodes, c->d_haux,
                    (const float4*)c->d_leaves, (const LeafBox*)(c->d_leaves + c->leaf_box_off), ordered,
                    ordered ? c->num_hnodes : 0u, c->wide_root, c->o_bound};
}

AccumShare* accum_new(int device)
{
    AccumShare* a = new (std::nothrow) AccumShare();
    if (!a) return nullptr;
    a->device = device;
    if (hipEventCreateWithFlags(&a->folded, hipEventDisableTiming) != hipSuccess) {
        delete a;
        return nullptr;
    }
    if (hipEventCreateWithFlags(&a->pend_ev, hipEventDisableTiming) != hipSuccess) {
        (void)hipEventDestroy(a->folded);
        delete a;
        return nullptr;
    }
    return a;
}

void accum_release(AccumShare* a)
{
    if (!a || --a->refs > 0) return;
    if (a->d_acc) (void)hipFree(a->d_acc);
    if (a->folded) (void)hipEventDestroy(a->folded);
    if (a->pend_ev) (void)hipEventDestroy(a->pend_ev);
    delete a;
}

// A fresh frame's accumulation state from its display: acc = c / 255 per
// channel, exactly store_pixel's fresh branch (main.c:368-370).
__global__ void acc_from_display_kernel(const uint32_t* __restrict__ disp, float* __restrict__ acc, size_t n)
{
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = disp[i];
    for (int ch = 0; ch < 3; ch++) acc[3 * i + ch] = (float)((c >> (8 * ch)) & 0xff) / 255.0f;
}

// The share's pending fresh frame folded into d_acc on stream s, behind the
// share's last fold and that frame's render; the slab's ctx then waits for
// this read before writing its slab again.
int accum_materialize(AccumShare* a, hipStream_t s)
{
    if (!a || !a->pend) return MIRT_OK;
    if (a->has_fold) HIP_TRY(hipStreamWaitEvent(s, a->folded, 0));
    HIP_TRY(hipStreamWaitEvent(s, a->pend_ev, 0));
    const size_t n = a->pixels;
    acc_from_display_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(a->pend, a->d_acc, n);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(a->folded, s));
    a->has_fold = true;
    mirt_ctx* pc = a->pend_ctx;
    HIP_TRY(hipEventRecord(pc->slab_free, s));
    pc->slab_guard = true;
    a->pend = nullptr;
    a->pend_ctx = nullptr;
    return MIRT_OK;
}

// A fresh frame's display left pending on its share (the lazy fold): the
// newest fresh frame supersedes any earlier one.
int accum_set_pending(AccumShare* a, mirt_ctx* c, const uint32_t* disp, hipStream_t s)
{
    HIP_TRY(hipEventRecord(a->pend_ev, s));
    a->pend = disp;
    a->pend_ctx = c;
    return MIRT_OK;
}

// The accumulation buffer for frames of `pixels` pixels, enqueued on stream
// s: (re)allocated if too small, cleared when the frame geometry changes
// (a new accumulation starts). Ordered behind the share's last fold.
int accum_prepare(AccumShare* a, size_t pixels, hipStream_t s)
{
    if (a->cap < pixels * 12 + 4) {
        // other ctxs' streams may still fold into the old buffer
        if (a->d_acc) HIP_TRY(hipDeviceSynchronize());
        int rc = ensure((void**)&a->d_acc, &a->cap, pixels * 12 + 4);
        if (rc) return rc;
        a->pixels = 0;
    }
    if (a->pixels != pixels) {
        a->pend = nullptr;   // a frame of the old geometry: a new accumulation starts
        a->pend_ctx = nullptr;
        if (a->has_fold) HIP_TRY(hipStreamWaitEvent(s, a->folded, 0));
        HIP_TRY(hipMemsetAsync(a->d_acc, 0, pixels * 12, s));
        HIP_TRY(hipEventRecord(a->folded, s));
        a->has_fold = true;
        a->pixels = pixels;
    }
    return MIRT_OK;
}

bool ctx_ok(mirt_ctx* c, bool need_scene, const char* fn)
{
    if (!c) {
        set_error("%s: null context", fn);
        return false;
    }
    if (need_scene && c->num_spheres < 0) {
        set_error("%s: no scene uploaded", fn);
        return false;
    }
    return hipSetDevice(c->device) == hipSuccess;
}

template <bool COUNT>
void dispatch_render(bool fast, const DevScene& sc, const FrameConst& f, uint32_t* d_out, float* d_acc, hipStream_t s,
                     int blocks, int bw, mirt_counts* d_counts, uint32_t* d_ws, Deferred dfr)
{
    if (fast)
        render_kernel<true, COUNT><<<blocks + dfr.blocks, 64 * bw, 0, s>>>(sc, f, d_out, d_acc, d_counts, d_ws, dfr);
    else
        render_kernel<false, COUNT><<<blocks + dfr.blocks, 64 * bw, 0, s>>>(sc, f, d_out, d_acc, d_counts, d_ws, dfr);
}

int launch_render_body(mirt_ctx* c, const FrameConst& f, uint32_t* d_out, float* d_acc, hipStream_t s, bool timed,
                       mirt_counts* d_counts, uint32_t* d_wave_stats, uint64_t* d_bdiag, AccumShare* chain);

// The accumulation chain of a frame of ctx c: its share when other ctxs hold
// it too (their folds must be ordered), else none.
AccumShare* accum_chain(const mirt_ctx* c)
{
    return c->acc && c->acc->refs > 1 ? c->acc : nullptr;
}

// The first bounces grouped by direction octant in the queue (frames in
// flight) or in tile order (a frame alone: the blocking call), or as
// MIRT_OPT_QUEUE_ORDER forces.
int octant_queue(const mirt_ctx* c)
{
    return c->queue_order == 1 || (c->queue_order == 0 && !c->lone_frame) ? 1 : 0;
}

int launch_render(mirt_ctx* c, const FrameConst& f, uint32_t* d_out, float* d_acc, hipStream_t s, bool timed,
                  mirt_counts* d_counts, uint32_t* d_wave_stats = nullptr, uint64_t* d_bdiag = nullptr)
{
    if (c->launched && c->last_stream != s) HIP_TRY(hipStreamWaitEvent(s, c->done, 0));
    if (c->slab_guard) {   // another stream still reads this ctx's slab (a pending fold)
        HIP_TRY(hipStreamWaitEvent(s, c->slab_free, 0));
        c->slab_guard = false;
    }
    const int rc = launch_render_body(c, f, d_out, d_acc, s, timed, d_counts, d_wave_stats, d_bdiag,
                                      d_counts ? nullptr : accum_chain(c));
    if (rc) return rc;
    HIP_TRY(hipEventRecord(c->done, s));
    c->last_stream = s;
    c->launched = true;
    return MIRT_OK;
}

// The frame's camera rays may test the grown PNode inner-child boxes without
// margins (trace.h slab_cons_fast<BND>): the camera within 4C.
bool camera_bounded(const mirt_ctx* c, const FrameConst& f)
{
    const float o = std::max(std::fabs(f.px), std::max(std::fabs(f.py), std::fabs(f.pz)));
    return c->o_bound > 0.0f && o <= 4.0f * c->o_bound;
}

int launch_render_body(mirt_ctx* c, const FrameConst& f, uint32_t* d_out, float* d_acc, hipStream_t s, bool timed,
                       mirt_counts* d_counts, uint32_t* d_wave_stats, uint64_t* d_bdiag, AccumShare* chain)
{
    const int tiles = ((f.width + 7) / 8) * ((f.num_rows + 7) / 8);
    const int bw = c->block_waves;
    const int blocks = (tiles + bw - 1) / bw;
    if (blocks == 0) return MIRT_OK;
    if (c->debug_stall_ms > 0) {
        stall_kernel<<<1, 64, 0, s>>>((uint64_t)c->debug_stall_ms * 100000u);
        HIP_TRY(hipGetLastError());
    }
    if (timed) {
        HIP_TRY(hipEventRecord(c->ev0, s));
        c->timed_recorded = true;
    }
    // several frames, or a buffer shared with other ctxs' frames in flight,
    // and an accumulation buffer: raw colours per frame, then
    // fold_samples_kernel accumulates them in order (behind the previous
    // fold into a shared buffer, whichever stream enqueued it)
    float* const d_fold = f.samples > 1 || chain ? d_acc : nullptr;
    if (d_fold) d_acc = nullptr;
    // Lazy fold: a fresh one-sample frame on a share leaves its display
    // pending instead of folding it; any other frame that folds first takes
    // the pending one (an accumulating frame needs it in d_acc) or drops it (a
    // fresh multi-sample fold overwrites d_acc whole)
    const bool lazy = chain && d_fold && !f.accumulate && f.samples == 1;
    if (chain && d_fold && !lazy) {
        if (f.accumulate) {
            if (int rc = accum_materialize(chain, s)) return rc;   // before this frame's render can touch a slab
        } else {
            chain->pend = nullptr;
            chain->pend_ctx = nullptr;
        }
    }
    auto fold = [&]() -> int {
        if (!d_fold) return MIRT_OK;
        if (lazy) return accum_set_pending(chain, c, d_out, s);
        const size_t n = (size_t)f.shard_rows * f.width;
        if (chain && chain->has_fold) HIP_TRY(hipStreamWaitEvent(s, chain->folded, 0));
        fold_samples_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(f, d_out, d_fold);
        HIP_TRY(hipGetLastError());
        if (chain) {
            HIP_TRY(hipEventRecord(chain->folded, s));
            chain->has_fold = true;
        }
        return MIRT_OK;
    };
    const bool wavefront = c->trav == kTravWavefront && f.use_bvh && f.depth >= 2 && !d_counts;
    // depth 1 (camera rays and their shading only): the camera-packet kernel
    // alone, at its 8 waves per SIMD, where the tree admits the ordered walk
    const bool primary_only = c->trav == kTravWavefront && f.use_bvh && f.depth == 1 && !d_counts && c->fast_slab &&
                              dev_scene(c).ordered;
    const int dbw = wavefront || primary_only ? 4 : bw;  // the wavefront kernels use 256-thread workgroups
    Deferred dfr{nullptr, nullptr, 0};
    c->phases_valid = wavefront;
    const uint32_t ps = c->ph_next;
    if (wavefront) {
        HIP_TRY(hipEventRecord(c->ph0[ps], s));
        c->ph_next = (ps + 1) % kPhaseRing;
        c->ph_count = std::min<uint32_t>(c->ph_count + 1, kPhaseRing);
    }
    const DevScene sc = dev_scene(c);
    // the ordered packet walk takes zero-component camera rays itself
    if (f.use_bvh && c->defer && !sc.ordered) {
        const size_t pixels = (size_t)f.num_rows * f.width;
        int rc = ensure((void**)&c->d_defer, &c->defer_cap, 4 * (pixels + 1));
        if (rc) return rc;
        HIP_TRY(hipMemsetAsync(c->d_defer, 0, 4, s));
        mark_deferred_kernel<<<dim3((f.width + 255) / 256, f.num_rows), 256, 0, s>>>(f, c->d_defer + 1, c->d_defer);
        HIP_TRY(hipGetLastError());
        // enough waves for the centre row and column of an axis-aligned
        // camera; a longer list is strided over the same waves
        const size_t want = std::min(pixels, (size_t)(f.width + f.num_rows + 64));
        dfr = Deferred{c->d_defer + 1, c->d_defer, (int)((want + dbw - 1) / dbw)};
    }
    if (primary_only) {
        // no bounce records: the queue is never written (its control words
        // are read only by a bounce pass)
        int rc = ensure(&c->d_queue, &c->queue_cap, sizeof(BounceRec) + kQCtlBytes);
        if (rc) return rc;
        uint32_t* qctl = (uint32_t*)c->d_queue;
        BounceRec* queue = (BounceRec*)((char*)c->d_queue + kQCtlBytes);
        const int ptiles = f.samples >= 4 ? ((f.width + 3) / 4) * ((f.shard_rows + 3) / 4) * ((f.samples + 3) / 4)
                                          : tiles;
        if (camera_bounded(c, f))
            primary_kernel<true, true, true><<<(ptiles + 3) / 4, 256, 0, s>>>(sc, f, d_out, d_acc, dfr, queue, qctl);
        else
            primary_kernel<true, true><<<(ptiles + 3) / 4, 256, 0, s>>>(sc, f, d_out, d_acc, dfr, queue, qctl);
        HIP_TRY(hipGetLastError());
        if (int rc2 = fold()) return rc2;
        if (timed) HIP_TRY(hipEventRecord(c->ev1, s));
        return MIRT_OK;
    }
    if (wavefront) {
        const size_t pixels = (size_t)f.num_rows * f.width;
        int rc = ensure(&c->d_queue, &c->queue_cap, sizeof(BounceRec) * pixels + kQCtlBytes);
        if (rc) return rc;
        uint32_t* qctl = (uint32_t*)c->d_queue;                          // {count}, segment heads
        BounceRec* queue = (BounceRec*)((char*)c->d_queue + kQCtlBytes);
        HIP_TRY(hipMemsetAsync(qctl, 0, kQCtlBytes, s));
        // primary_kernel's packets: 8x8 pixel tiles, or 4x4 pixels x 4 frames
        // for an ordered walk over four frames or more
        const int ptiles = c->fast_slab && sc.ordered && f.samples >= 4
                               ? ((f.width + 3) / 4) * ((f.shard_rows + 3) / 4) * ((f.samples + 3) / 4)
                               : tiles;
        const int pblocks = (ptiles + 3) / 4 + dfr.blocks;
        const int bblocks = c->bounce_blocks_opt ? c->bounce_blocks_opt : c->bounce_blocks;
        const size_t blds = bounce_lds_bytes(f.depth);
        if (c->fast_slab && sc.ordered && camera_bounded(c, f))
            primary_kernel<true, true, true><<<pblocks, 256, 0, s>>>(sc, f, d_out, d_acc, dfr, queue, qctl,
                                                                     octant_queue(c));
        else if (c->fast_slab && sc.ordered)
            primary_kernel<true, true><<<pblocks, 256, 0, s>>>(sc, f, d_out, d_acc, dfr, queue, qctl, octant_queue(c));
        else if (c->fast_slab)
            primary_kernel<true, false><<<pblocks, 256, 0, s>>>(sc, f, d_out, d_acc, dfr, queue, qctl, octant_queue(c));
        else
            primary_kernel<false, false><<<pblocks, 256, 0, s>>>(sc, f, d_out, d_acc, dfr, queue, qctl, octant_queue(c));
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ph1[ps], s));
        if (d_bdiag && sc.wide)
            bounce_kernel<true, 2, true><<<bblocks, 256, blds, s>>>(sc, f, d_out, d_acc, queue, qctl, c->bounce_threshold, c->quad_drain, d_bdiag);
        else if (d_bdiag)
            bounce_kernel<true, 0, true><<<bblocks, 256, blds, s>>>(sc, f, d_out, d_acc, queue, qctl, c->bounce_threshold, c->quad_drain, d_bdiag);
        else if (sc.wide && leaf_batch(c))
            bounce_kernel<true, 4><<<bblocks, 256, blds, s>>>(sc, f, d_out, d_acc, queue, qctl, c->bounce_threshold, c->quad_drain);
        else if (sc.wide)
            bounce_kernel<true, 2><<<bblocks, 256, blds, s>>>(sc, f, d_out, d_acc, queue, qctl, c->bounce_threshold, c->quad_drain);
        else if (c->fast_slab)
            bounce_kernel<true, 0><<<bblocks, 256, blds, s>>>(sc, f, d_out, d_acc, queue, qctl, c->bounce_threshold, c->quad_drain);
        else
            bounce_kernel<false, 0><<<bblocks, 256, blds, s>>>(sc, f, d_out, d_acc, queue, qctl, c->bounce_threshold, c->quad_drain);
        HIP_TRY(hipGetLastError());
        HIP_TRY(hipEventRecord(c->ph2[ps], s));
        if (int rc = fold()) return rc;
        if (timed) HIP_TRY(hipEventRecord(c->ev1, s));
        return MIRT_OK;
    }
    if (d_counts)
        dispatch_render<true>(true, sc, f, d_out, d_acc, s, blocks, bw, d_counts, d_wave_stats, dfr);
    else
        dispatch_render<false>(c->fast_slab != 0, sc, f, d_out, d_acc, s, blocks, bw, nullptr, nullptr, dfr);
    HIP_TRY(hipGetLastError());
    if (int rc = fold()) return rc;
    if (timed) HIP_TRY(hipEventRecord(c->ev1, s));
    return MIRT_OK;
}

// Workgroup size of a per-ray batch kernel: one wave per workgroup while the
// batch is too small to give every CU a few waves (each walk is a chain of
// dependent loads, so spreading the waves over CUs is what shortens it).
int batch_threads(const mirt_ctx* c, int n)
{
    return n < 256 * 4 * std::max(1, c->num_cus) ? 64 : 256;
}

// intersect_quad_kernel for a BVH batch: the four-wide tree, the fast slab
// filter, and fewer rays than give every CU four waves of one ray per lane
// (MIRT_OPT_QUAD_BATCH 0 turns it off)
bool quad_batch(const mirt_ctx* c, int n)
{
    const DevScene sc = dev_scene(c);
    return c->quad_batch && c->fast_slab && sc.wide && n <= 64 * 4 * std::max(1, c->num_cus);
}

// brute_chunk_kernel over the rays in c->d_in: enough sphere chunks that the
// grid has ~8 workgroups per CU whatever the ray count.
int launch_brute(mirt_ctx* c, int n)
{
    int rc = ensure((void**)&c->d_keys, &c->keys_cap, sizeof(unsigned long long) * (size_t)n);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_keys, 0xff, sizeof(unsigned long long) * (size_t)n, c->stream));
    const int ns = c->num_spheres;
    if (ns <= 0) return MIRT_OK;
    const int bx = (n + 255) / 256;
    const int want = std::max(1, 8 * std::max(1, c->num_cus) / bx);
    const int chunks = std::min(std::min(want, (ns + 63) / 64), 65535);
    const int chunk = (ns + chunks - 1) / chunks;
    const dim3 grid(bx, (ns + chunk - 1) / chunk);
    const DevScene sc = dev_scene(c);
    const mirt_ray* d_rays = (const mirt_ray*)c->d_in;
    if (c->fast_slab)
        brute_chunk_kernel<true><<<grid, 256, 0, c->stream>>>(sc, d_rays, n, chunk, c->d_keys);
    else
        brute_chunk_kernel<false><<<grid, 256, 0, c->stream>>>(sc, d_rays, n, chunk, c->d_keys);
    HIP_TRY(hipGetLastError());
    return MIRT_OK;
}

}  // namespace

extern "C" {

int mirt_create(int device, mirt_ctx** out)
{
    if (!out) return MIRT_E_INVALID;
    *out = nullptr;
    int n = 0;
    HIP_TRY(hipGetDeviceCount(&n));
    if (device < 0 || device >= n) {
        set_error("mirt_create: device %d not present (%d visible)", device, n);
        return MIRT_E_INVALID;
    }
    HIP_TRY(hipSetDevice(device));
    mirt_ctx* c = new (std::nothrow) mirt_ctx();
    if (!c) {
        set_error("mirt_create: out of host memory");
        return MIRT_E_NOMEM;
    }
    c->device = device;
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipEventCreate(&c->ev0);
    if (e == hipSuccess) e = hipEventCreate(&c->ev1);
    for (int k = 0; k < kPhaseRing && e == hipSuccess; k++) {
        e = hipEventCreate(&c->ph0[k]);
        if (e == hipSuccess) e = hipEventCreate(&c->ph1[k]);
        if (e == hipSuccess) e = hipEventCreate(&c->ph2[k]);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->slab_free, hipEventDisableTiming);
    if (e == hipSuccess) e = hipMalloc((void**)&c->d_counts, sizeof(mirt_counts));
    if (e == hipSuccess) {
        c->acc = accum_new(device);
        if (!c->acc) e = hipErrorOutOfMemory;
    }
    if (e == hipSuccess) {
        int cus = 0, per_cu = 0;
        e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
        if (e == hipSuccess)
            e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, bounce_kernel<true, 2>, 256,
                                                             bounce_lds_bytes(kMaxDepth));
        c->bounce_blocks = std::max(1, cus) * std::max(1, per_cu);
        c->num_cus = cus;
    }
    if (e != hipSuccess) {
        mirt_destroy(c);
        return hip_fail(e, "mirt_create");
    }
    *out = c;
    return MIRT_OK;
}

void mirt_destroy(mirt_ctx* c)
{
    if (!c) return;
    (void)hipSetDevice(c->device);
    // a share that lives on must not keep a pending fold of this ctx's slab
    if (c->acc && c->acc->refs > 1 && c->acc->pend_ctx == c) (void)accum_materialize(c->acc, c->stream);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->slab_guard) (void)hipEventSynchronize(c->slab_free);   // another stream's read of the slab
    accum_release(c->acc);
    for (void* p : {(void*)c->d_nodes, (void*)c->d_nodes32, (void*)c->d_geo, (void*)c->d_color, (void*)c->d_out,
                    c->d_in, c->d_res, (void*)c->d_counts, (void*)c->d_defer, c->d_queue, (void*)c->d_keys, (void*)c->d_pnodes,
                    (void*)c->d_hnodes, (void*)c->d_haux, (void*)c->d_leaves, (void*)c->d_ndepth,
                    (void*)c->d_overlay})
        if (p) (void)hipFree(p);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (int k = 0; k < kPhaseRing; k++)
        for (hipEvent_t ev : {c->ph0[k], c->ph1[k], c->ph2[k]})
            if (ev) (void)hipEventDestroy(ev);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->slab_free) (void)hipEventDestroy(c->slab_free);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int mirt_scene_upload_flat(mirt_ctx* c, const mirt_sphere* spheres, int ns, const mirt_node* nodes, int nn)
try {
    if (!ctx_ok(c, false, "mirt_scene_upload_flat")) return MIRT_E_INVALID;
    if (ns < 0 || nn < 0 || (ns > 0 && !spheres) || (nn > 0 && !nodes)) {
        set_error("mirt_scene_upload_flat: invalid arguments");
        return MIRT_E_INVALID;
    }
    // a malformed tree must not send the host layout builders or the kernels
    // out of bounds
    if (int rc = validate_flat(nodes, nn, ns, 0, "mirt_scene_upload_flat")) return rc;
    float r_max = 0.0f, c_max = 0.0f;
    const bool encloses = tree_encloses(spheres, ns, nodes, nn, &r_max, &c_max) && !orphan_phantoms(nodes, nn, ns);
    std::vector<float4> geo((size_t)ns + 1);
    std::vector<uint32_t> col((size_t)ns + 1);
    for (int i = 0; i < ns; i++) {
        geo[i] = make_float4(spheres[i].center.x, spheres[i].center.y, spheres[i].center.z, spheres[i].radius);
        std::memcpy(&col[i], &spheres[i].color, 4);
    }
    geo[ns] = make_float4(NAN, NAN, NAN, NAN);  // &spheres[N] sentinel: never hits
    col[ns] = 0xff000000u;
    for (void* p : {(void*)c->d_nodes, (void*)c->d_nodes32, (void*)c->d_geo, (void*)c->d_color, (void*)c->d_pnodes,
                    (void*)c->d_hnodes, (void*)c->d_haux, (void*)c->d_leaves, (void*)c->d_ndepth})
        if (p) (void)hipFree(p);
    c->d_ndepth = nullptr;
    c->d_pnodes = nullptr;
    c->d_hnodes = nullptr;
    c->d_haux = nullptr;
    c->d_leaves = nullptr;
    c->d_nodes = nullptr;
    c->d_nodes32 = nullptr;
    c->d_geo = nullptr;
    c->d_color = nullptr;
    c->num_spheres = -1;
    // device layout: 64-B nodes with each leaf's sphere inline (trace.h DNode)
    std::vector<DNode> dn((size_t)nn);
    for (int i = 0; i < nn; i++) {
        DNode& d = dn[i];
        std::memset(&d, 0, sizeof d);
        std::memcpy(d.bmin, nodes[i].bmin, sizeof d.bmin);
        std::memcpy(d.bmax, nodes[i].bmax, sizeof d.bmax);
        d.sphere = nodes[i].sphere;
        d.skip = nodes[i].skip;
        d.geo = nodes[i].sphere >= 0 ? geo[nodes[i].sphere] : geo[ns];
    }
    HIP_TRY(hipMalloc((void**)&c->d_nodes, sizeof(DNode) * (size_t)(nn > 0 ? nn : 1)));
    HIP_TRY(hipMalloc((void**)&c->d_geo, sizeof(float4) * geo.size()));
    HIP_TRY(hipMalloc((void**)&c->d_color, sizeof(uint32_t) * col.size()));
    HIP_TRY(hipMalloc((void**)&c->d_nodes32, sizeof(mirt_node) * (size_t)(nn > 0 ? nn : 1)));
    if (nn > 0) HIP_TRY(hipMemcpy(c->d_nodes, dn.data(), sizeof(DNode) * (size_t)nn, hipMemcpyHostToDevice));
    if (nn > 0) HIP_TRY(hipMemcpy(c->d_nodes32, nodes, sizeof(mirt_node) * (size_t)nn, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_geo, geo.data(), sizeof(float4) * geo.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_color, col.data(), sizeof(uint32_t) * col.size(), hipMemcpyHostToDevice));
    // the margin-free box tests (bounce walks, camera packets): C bounds every box coordinate and every sphere point
    // (so every bounce-ray origin, up to rounding: the margin 2^-10 C + 2^-10),
    // and the slot boxes grow by 2^-19 C (trace.h slab_cons_fast<BND>)
    double cb = c_max;
    for (int i = 0; i < nn; i++) {
        if (nodes[i].skip & MIRT_NODE_EMPTY) continue;
        for (int a = 0; a < 3; a++)
            for (float v : {nodes[i].bmin[a], nodes[i].bmax[a]})
                if (std::isfinite(v)) cb = std::max(cb, (double)std::fabs(v));
    }
    cb = cb * (1.0 + 0x1p-10) + 0x1p-10;
    const bool bounded = encloses && cb < 6.0e4;   // fp16 range: the grown boxes stay finite
    c->o_bound = bounded ? (float)cb : 0.0f;   // 0: every bounce ray takes the exact test
    std::vector<PNode> pn;
    const bool ordered = build_pnodes(nodes, nn, spheres, ns, pn, bounded ? cb * 0x1p-19 : 0.0);
    HIP_TRY(hipMalloc((void**)&c->d_pnodes, sizeof(PNode) * pn.size()));
    HIP_TRY(hipMemcpy(c->d_pnodes, pn.data(), sizeof(PNode) * pn.size(), hipMemcpyHostToDevice));
    std::vector<HNode> hn;
    std::vector<HAux> hx;
    std::vector<float4> lgeo;
    std::vector<LeafBox> lbox;
    build_hnodes(nodes, nn, spheres, ns, hn, hx, lgeo, lbox, bounded ? cb * 0x1p-19 : 0.0);
    const size_t nl = lbox.size();
    const size_t box_off = (sizeof(float4) * nl + 255) & ~(size_t)255;
    HIP_TRY(hipMalloc((void**)&c->d_hnodes, sizeof(HNode) * hn.size()));
    HIP_TRY(hipMalloc((void**)&c->d_haux, sizeof(HAux) * hx.size()));
    HIP_TRY(hipMalloc((void**)&c->d_leaves, box_off + sizeof(LeafBox) * std::max<size_t>(nl, 1)));
    HIP_TRY(hipMemcpy(c->d_hnodes, hn.data(), sizeof(HNode) * hn.size(), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->d_haux, hx.data(), sizeof(HAux) * hx.size(), hipMemcpyHostToDevice));
    if (nl) {
        HIP_TRY(hipMemcpy(c->d_leaves, lgeo.data(), sizeof(float4) * nl, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(c->d_leaves + box_off, lbox.data(), sizeof(LeafBox) * nl, hipMemcpyHostToDevice));
    }
    // node depths (pre-order: the children of inner node i are i + 1 and the
    // left subtree's skip), clamped to 255 -- the overlay's colour key
    std::vector<uint8_t> ndepth((size_t)std::max(nn, 1), 0);
    for (int i = 0; i < nn; i++) {
        if (nodes[i].sphere >= 0) continue;
        const uint8_t d = ndepth[i] == 255 ? 255 : (uint8_t)(ndepth[i] + 1);
        ndepth[i + 1] = d;
        ndepth[nodes[i + 1].skip & MIRT_SKIP_MASK] = d;
    }
    HIP_TRY(hipMalloc((void**)&c->d_ndepth, ndepth.size()));
    HIP_TRY(hipMemcpy(c->d_ndepth, ndepth.data(), ndepth.size(), hipMemcpyHostToDevice));
    c->num_nodes = nn;
    c->num_spheres = ns;
    c->num_hnodes = (uint32_t)hn.size();
    c->leaf_box_off = box_off;
    c->leaf_big = sizeof(HNode) * hn.size() + (sizeof(float4) + sizeof(LeafBox)) * nl > ((size_t)32 << 20);
    {
        const uint32_t r = hn[0].slot[0].ref;
        c->wide_root = (r != kPNone && !(r & kPLeaf)) ? r : 0u;
    }
    c->ordered_ok = ordered;
    c->prune_ok = encloses;
    c->r_max = r_max;
    c->c_max = c_max;
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    set_error("mirt_scene_upload_flat: out of host memory");
    return MIRT_E_NOMEM;
}

int mirt_scene_upload(mirt_ctx* c, const mirt_sphere* spheres, int ns, const mirt_bvh_node* root)
try {
    if (!root) return mirt_scene_upload_flat(c, spheres, ns, nullptr, 0);
    const int nn = mirt_bvh_count(root);
    std::vector<mirt_node> flat((size_t)nn);
    if (mirt_bvh_flatten(root, spheres, flat.data(), nn) != nn) {
        set_error("mirt_scene_upload: flatten failed");
        return MIRT_E_INVALID;
    }
    return mirt_scene_upload_flat(c, spheres, ns, flat.data(), nn);
} catch (const std::bad_alloc&) {
    set_error("mirt_scene_upload: out of host memory");
    return MIRT_E_NOMEM;
}

int mirt_render_frame_device(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, uint32_t* d_out,
                             float* d_acc, void* stream)
{
    if (!ctx_ok(c, true, "mirt_render_frame_device")) return MIRT_E_NOSCENE;
    if (!cam || !frame_desc_valid(fd) || !d_out || (fd->accumulate && !d_acc)) {
        set_error("mirt_render_frame_device: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (fd->use_bvh && c->num_nodes == 0) {
        set_error("mirt_render_frame_device: use_bvh set but no tree uploaded");
        return MIRT_E_NOSCENE;
    }
    const FrameConst f = make_frame_const(cam, fd);
    return launch_render(c, f, d_out, d_acc, (hipStream_t)stream, false, nullptr);
}

}  // extern "C"

namespace {

// The frame of mirt_render_frame up to its D2H copy, enqueued on the ctx's
// stream: `samples` slabs into d_out (the ctx's own buffer when null),
// accumulation in the ctx's (possibly shared) buffer. *d_display = the slab
// that holds the display after the last frame.
int enqueue_frame(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, uint32_t* d_out,
                  uint32_t** d_display, const char* fn, bool independent = false)
{
    if (!ctx_ok(c, true, fn)) return MIRT_E_NOSCENE;
    if (!cam || !frame_desc_valid(fd)) {
        set_error("%s: invalid arguments", fn);
        return MIRT_E_INVALID;
    }
    if (fd->use_bvh && c->num_nodes == 0) {
        set_error("%s: use_bvh set but no tree uploaded", fn);
        return MIRT_E_NOSCENE;
    }
    const FrameConst f = make_frame_const(cam, fd);
    const size_t pixels = (size_t)f.shard_rows * f.width;  // one frame (several: slab j = display after frame j)
    if (!d_out && c->out_cap < pixels * f.samples * 4 + 4) {
        // the slab is reallocated: a pending fold of it is taken first, and
        // any other stream's read of it has ended
        if (c->acc->pend_ctx == c) {
            if (int rc = accum_materialize(c->acc, c->stream)) return rc;
        }
        if (c->slab_guard) {
            HIP_TRY(hipEventSynchronize(c->slab_free));
            c->slab_guard = false;
        }
        HIP_TRY(hipStreamSynchronize(c->stream));
    }
    if (!d_out) {
        int rc = ensure((void**)&c->d_out, &c->out_cap, pixels * f.samples * 4 + 4);
        if (rc) return rc;
        d_out = c->d_out;
    }
    // a new frame geometry starts a fresh accumulation buffer
    int rc = accum_prepare(c->acc, pixels, c->stream);
    if (rc) return rc;
    // independent fresh frames (mirt_multi's launches of several frames): raw
    // slabs, then the last one folded as a fresh frame, so the (possibly
    // shared) accumulation buffer holds what a sequence of fresh frames leaves
    const bool raw = independent && f.samples > 1 && !f.accumulate;
    rc = launch_render(c, f, d_out, raw ? nullptr : c->acc->d_acc, c->stream, true, nullptr);
    if (rc) return rc;
    *d_display = d_out + (size_t)(f.samples - 1) * pixels;
    if (raw) {
        FrameConst f1 = f;
        f1.samples = 1;
        f1.accumulate = 0;
        AccumShare* chain = accum_chain(c);
        if (chain) {   // this fold is newer than a pending fresh display: that one is dropped
            chain->pend = nullptr;
            chain->pend_ctx = nullptr;
        }
        if (chain && chain->has_fold) HIP_TRY(hipStreamWaitEvent(c->stream, chain->folded, 0));
        fold_samples_kernel<<<(unsigned)((pixels + 255) / 256), 256, 0, c->stream>>>(f1, *d_display, c->acc->d_acc);
        HIP_TRY(hipGetLastError());
        if (chain) {
            HIP_TRY(hipEventRecord(chain->folded, c->stream));
            chain->has_fold = true;
        }
        HIP_TRY(hipEventRecord(c->done, c->stream));
    }
    return MIRT_OK;
}

// The frame of mirt_render_frame up to and including its D2H copy, enqueued
// on the ctx's stream.
int enqueue_host_frame(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out,
                       const char* fn)
{
    if (!out) {
        set_error("%s: invalid arguments", fn);
        return MIRT_E_INVALID;
    }
    uint32_t* disp = nullptr;
    if (int rc = enqueue_frame(c, cam, fd, nullptr, &disp, fn)) return rc;
    // as a 2D copy (rows x width): the runtime takes a DMA engine for it, where a
    // 1D copy of the same bytes often runs as a blit kernel on this stream's
    // compute queue (as multi.hip does)
    const size_t row = (size_t)fd->width * 4;
    HIP_TRY(hipMemcpy2DAsync(out, row, disp, row, row, (size_t)shard_row_count(fd), hipMemcpyDeviceToHost, c->stream));
    return MIRT_OK;
}

}  // namespace

namespace mirt {
int enqueue_frame_device(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, uint32_t* d_out,
                         uint32_t** d_display, const char* fn, bool independent)
{
    return enqueue_frame(c, cam, fd, d_out, d_display, fn, independent);
}
int ctx_device(const mirt_ctx* c) { return c->device; }
}  // namespace mirt

extern "C" {

namespace {

// The device-visible address of a page-locked host range (mirt_host_alloc /
// mirt_host_register memory), or null for pageable memory -- and for a range
// that spans separately registered pieces: the device mapping must be ONE
// contiguous range (the last byte's device address = the first's + bytes - 1),
// else the kernels' stores would land elsewhere (the copy path takes it).
uint32_t* host_mapped(const void* p, size_t bytes)
{
    hipPointerAttribute_t a, b;
    if (hipPointerGetAttributes(&a, p) != hipSuccess || a.type != hipMemoryTypeHost || !a.devicePointer ||
        hipPointerGetAttributes(&b, (const char*)p + bytes - 1) != hipSuccess || b.type != hipMemoryTypeHost ||
        (const char*)b.devicePointer != (const char*)a.devicePointer + bytes - 1) {
        (void)hipGetLastError();   // a pageable pointer is an error to the query, not to the caller
        return nullptr;
    }
    return (uint32_t*)a.devicePointer;
}

}  // namespace

extern "C++" {
namespace mirt {
// The device-visible address of a page-locked host range (null if it is not
// one contiguous mapping): mirt_multi's copy kernels store into it.
uint32_t* host_device_ptr(const void* p, size_t bytes) { return host_mapped(p, bytes); }
// Before a caller frees or reallocates an external slab ctx c rendered into:
// a pending fold of it is taken now and every read of it has ended.
int accum_settle(mirt_ctx* c)
{
    if (c->acc && c->acc->pend_ctx == c) {
        if (int rc = accum_materialize(c->acc, c->stream)) return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->slab_guard) {
        HIP_TRY(hipEventSynchronize(c->slab_free));
        c->slab_guard = false;
    }
    return MIRT_OK;
}
// Page-locked ranges this library handed out or registered (mirt_host_alloc /
// mirt_host_register): checked without a HIP call, which the frame loops of
// mirt_multi make for every output of every launch.
static std::mutex g_pin_mu;
static std::map<uintptr_t, size_t> g_pinned;   // start -> bytes
void pinned_add(const void* p, size_t bytes)
{
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pinned[(uintptr_t)p] = bytes;
}
void pinned_remove(const void* p)
{
    std::lock_guard<std::mutex> lk(g_pin_mu);
    g_pinned.erase((uintptr_t)p);
}
bool host_page_locked(const void* p, size_t bytes)
{
    {
        std::lock_guard<std::mutex> lk(g_pin_mu);
        auto it = g_pinned.upper_bound((uintptr_t)p);
        if (it != g_pinned.begin()) {
            --it;
            if ((uintptr_t)p + bytes <= it->first + it->second) return true;
        }
    }
    return host_mapped(p, bytes) != nullptr;   // pinned by other means (e.g. the caller's hipHostMalloc)
}
}  // namespace mirt
}

static int render_frame_blocking(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out);

// The blocking call renders one frame with nothing after it on the ctx: its
// first bounces go to the queue in tile order (lone_frame), which the
// bounce pass walks 2-4% faster when no other frame shares the chip.
int mirt_render_frame(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out)
{
    if (c) c->lone_frame = true;
    const int rc = render_frame_blocking(c, cam, fd, out);
    if (c) c->lone_frame = false;
    return rc;
}

static int render_frame_blocking(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out)
{
    // a page-locked destination (the recipe for main.c's reused frame buffer:
    // mirt_host_register): the frame kernels store each pixel straight into
    // it, so the frame is in host memory when they end -- no copy after them
    // (one frame, the ctx's own accumulation: nothing reads the output back)
    if (c && c->zero_copy && out && frame_desc_valid(fd) && fd->samples <= 1 && !accum_chain(c)) {
        if (uint32_t* d = host_mapped(out, (size_t)shard_row_count(fd) * fd->width * 4)) {
            uint32_t* disp = nullptr;
            if (int rc = enqueue_frame(c, cam, fd, d, &disp, "mirt_render_frame")) return rc;
            HIP_TRY(hipStreamSynchronize(c->stream));
            HIP_TRY(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
            return MIRT_OK;
        }
    }
    if (int rc = enqueue_host_frame(c, cam, fd, out, "mirt_render_frame")) return rc;
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    return MIRT_OK;
}

int mirt_render_frame_async(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_rgba8* out)
{
    // MIRT_OPT_ZERO_COPY 2: frames in flight into page-locked memory are
    // written in place too (no DMA behind each frame's kernels)
    if (c && c->zero_copy == 2 && out && frame_desc_valid(fd) && fd->samples <= 1 && !accum_chain(c)) {
        if (uint32_t* d = host_mapped(out, (size_t)shard_row_count(fd) * fd->width * 4)) {
            uint32_t* disp = nullptr;
            return enqueue_frame(c, cam, fd, d, &disp, "mirt_render_frame_async");
        }
    }
    return enqueue_host_frame(c, cam, fd, out, "mirt_render_frame_async");
}

int mirt_ctx_wait(mirt_ctx* c)
{
    if (!ctx_ok(c, false, "mirt_ctx_wait")) return MIRT_E_INVALID;
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->timed_recorded) HIP_TRY(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    return MIRT_OK;
}

int mirt_host_alloc(size_t bytes, void** out)
{
    if (!out) return MIRT_E_INVALID;
    *out = nullptr;
    HIP_TRY(hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocPortable));   // pinned for every device (mirt_multi host-direct)
    mirt::pinned_add(*out, bytes ? bytes : 1);
    return MIRT_OK;
}

void mirt_host_free(void* p)
{
    if (!p) return;
    mirt::pinned_remove(p);
    (void)hipHostFree(p);
}

int mirt_host_register(void* p, size_t bytes)
{
    if (!p || !bytes) {
        set_error("mirt_host_register: invalid arguments");
        return MIRT_E_INVALID;
    }
    HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterPortable));
    mirt::pinned_add(p, bytes);
    return MIRT_OK;
}

int mirt_host_unregister(void* p)
{
    if (!p) {
        set_error("mirt_host_unregister: null pointer");
        return MIRT_E_INVALID;
    }
    mirt::pinned_remove(p);
    HIP_TRY(hipHostUnregister(p));
    return MIRT_OK;
}

int mirt_accum_download(mirt_ctx* c, float* out, size_t count)
{
    if (!ctx_ok(c, false, "mirt_accum_download") || !out) return MIRT_E_INVALID;
    AccumShare* a = c->acc;
    if (count > a->pixels * 3) {
        set_error("mirt_accum_download: %zu floats requested, %zu held", count, a->pixels * 3);
        return MIRT_E_INVALID;
    }
    // after every fold enqueued so far, whichever ctx's stream carries it
    if (int rc = accum_materialize(a, c->stream)) return rc;
    if (a->has_fold) HIP_TRY(hipStreamWaitEvent(c->stream, a->folded, 0));
    HIP_TRY(hipMemcpyAsync(out, a->d_acc, count * sizeof(float), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

int mirt_ctx_share_accum(mirt_ctx* c, mirt_ctx* owner)
{
    if (!ctx_ok(c, false, "mirt_ctx_share_accum")) return MIRT_E_INVALID;
    if (owner && owner->device != c->device) {
        set_error("mirt_ctx_share_accum: ctxs on devices %d and %d", c->device, owner->device);
        return MIRT_E_INVALID;
    }
    AccumShare* next = owner && owner != c ? owner->acc : nullptr;
    if (next == c->acc || (!next && c->acc->refs == 1)) return MIRT_OK;  // already so / already private
    if (!next) {
        next = accum_new(c->device);
        if (!next) {
            set_error("mirt_ctx_share_accum: out of host memory");
            return MIRT_E_NOMEM;
        }
    } else {
        if (next->refs == 1) {
            // the owner's frames enqueued while its buffer was private wrote
            // it directly (store_pixel) and recorded no fold event: from now
            // on every fold, on any stream, must follow them
            if (next->has_fold) HIP_TRY(hipStreamWaitEvent(owner->stream, next->folded, 0));
            HIP_TRY(hipEventRecord(next->folded, owner->stream));
            next->has_fold = true;
        }
        next->refs++;
    }
    // c's frames enqueued so far still use its old buffer (and a pending
    // fold of c's slab is taken into it before c leaves)
    if (c->acc->pend_ctx == c) {
        if (int rc = accum_materialize(c->acc, c->stream)) return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (c->slab_guard) {
        HIP_TRY(hipEventSynchronize(c->slab_free));
        c->slab_guard = false;
    }
    accum_release(c->acc);
    c->acc = next;
    return MIRT_OK;
}

int mirt_count_frame(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_counts* out)
{
    if (!ctx_ok(c, true, "mirt_count_frame")) return MIRT_E_NOSCENE;
    if (!cam || !frame_desc_valid(fd) || !out) {
        set_error("mirt_count_frame: invalid arguments");
        return MIRT_E_INVALID;
    }
    const FrameConst f = make_frame_const(cam, fd);
    const size_t pixels = (size_t)f.num_rows * f.width;
    int rc = ensure((void**)&c->d_out, &c->out_cap, pixels * 4 + 4);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_counts, 0, sizeof(mirt_counts), c->stream));
    FrameConst f2 = f;
    f2.accumulate = 0;
    rc = launch_render(c, f2, c->d_out, nullptr, c->stream, false, c->d_counts);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, c->d_counts, sizeof(mirt_counts), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

int mirt_wave_stats(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, uint32_t* out, int cap)
{
    if (!ctx_ok(c, true, "mirt_wave_stats")) return MIRT_E_NOSCENE;
    if (!cam || !frame_desc_valid(fd)) {
        set_error("mirt_wave_stats: invalid arguments");
        return MIRT_E_INVALID;
    }
    FrameConst f = make_frame_const(cam, fd);
    f.accumulate = 0;
    const int waves = ((f.width + 7) / 8) * ((f.num_rows + 7) / 8);
    if (!out || cap < waves) return -waves;
    const size_t pixels = (size_t)f.num_rows * f.width;
    int rc = ensure((void**)&c->d_out, &c->out_cap, pixels * 4 + 4);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, 16 * (size_t)waves + 64);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_counts, 0, sizeof(mirt_counts), c->stream));
    rc = launch_render(c, f, c->d_out, nullptr, c->stream, false, c->d_counts, (uint32_t*)c->d_res);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, c->d_res, 16 * (size_t)waves, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return waves;
}

int mirt_bounce_stats(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, uint64_t* out, int cap)
{
    if (!ctx_ok(c, true, "mirt_bounce_stats")) return MIRT_E_NOSCENE;
    if (!cam || !frame_desc_valid(fd) || !fd->use_bvh || fd->max_depth < 2 || c->trav != kTravWavefront) {
        set_error("mirt_bounce_stats: needs a BVH frame of depth >= 2 under the wavefront schedule");
        return MIRT_E_INVALID;
    }
    const int waves = (c->bounce_blocks_opt ? c->bounce_blocks_opt : c->bounce_blocks) * 4;
    if (!out || cap < waves) return -waves;
    static_assert(kBounceDiag == 12, "mirt.h documents 12 words per wave");
    FrameConst f = make_frame_const(cam, fd);
    f.accumulate = 0;
    const size_t pixels = (size_t)f.num_rows * f.width;
    int rc = ensure((void**)&c->d_out, &c->out_cap, pixels * 4 + 4);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, 8 * kBounceDiag * (size_t)waves + 64);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_res, 0, 8 * kBounceDiag * (size_t)waves, c->stream));
    rc = launch_render(c, f, c->d_out, nullptr, c->stream, false, nullptr, nullptr, (uint64_t*)c->d_res);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(out, c->d_res, 8 * kBounceDiag * (size_t)waves, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return waves;
}

int mirt_camera_rays(mirt_ctx* c, const mirt_camera* cam, const mirt_frame_desc* fd, mirt_ray* out)
{
    if (!ctx_ok(c, false, "mirt_camera_rays")) return MIRT_E_INVALID;
    if (!cam || !frame_desc_valid(fd) || !out) {
        set_error("mirt_camera_rays: invalid arguments");
        return MIRT_E_INVALID;
    }
    const FrameConst f = make_frame_const(cam, fd);
    const size_t bytes = (size_t)f.num_rows * f.width * sizeof(mirt_ray);
    int rc = ensure(&c->d_res, &c->res_cap, bytes + 4);
    if (rc) return rc;
    if (f.num_rows > 0) {
        camera_rays_kernel<<<dim3((f.width + 255) / 256, f.num_rows), 256, 0, c->stream>>>(f, (mirt_ray*)c->d_res);
        HIP_TRY(hipGetLastError());
    }
    HIP_TRY(hipMemcpyAsync(out, c->d_res, bytes, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

int mirt_trace_rays(mirt_ctx* c, const mirt_ray* rays, int n, int depth, int use_bvh, uint64_t seed,
                    uint32_t sample, mirt_rgba8* out)
{
    return mirt_trace_rays_at(c, rays, n, depth, use_bvh, seed, sample, 0, out);
}

int mirt_trace_rays_at(mirt_ctx* c, const mirt_ray* rays, int n, int depth, int use_bvh, uint64_t seed,
                       uint32_t sample, uint32_t pixel0, mirt_rgba8* out)
{
    if (!ctx_ok(c, true, "mirt_trace_rays")) return MIRT_E_NOSCENE;
    if (n < 0 || (n > 0 && (!rays || !out)) || depth < 0 || depth > kMaxDepth) {
        set_error("mirt_trace_rays: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (use_bvh && c->num_nodes == 0) {
        set_error("mirt_trace_rays: use_bvh set but no tree uploaded");
        return MIRT_E_NOSCENE;
    }
    if (n == 0) return MIRT_OK;
    int rc = ensure(&c->d_in, &c->in_cap, sizeof(mirt_ray) * (size_t)n);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, 4 * (size_t)n);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_in, rays, sizeof(mirt_ray) * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    {
        const dim3 g((n + 255) / 256), b(256);
        const DevScene sc = dev_scene(c);
        const mirt_ray* in = (const mirt_ray*)c->d_in;
        uint32_t* res = (uint32_t*)c->d_res;
        if (c->fast_slab)
            trace_rays_kernel<true><<<g, b, 0, c->stream>>>(sc, in, n, depth, use_bvh, seed, sample, pixel0, res);
        else
            trace_rays_kernel<false><<<g, b, 0, c->stream>>>(sc, in, n, depth, use_bvh, seed, sample, pixel0, res);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->d_res, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    return MIRT_OK;
}

int mirt_intersect_rays(mirt_ctx* c, const mirt_ray* rays, int n, int use_bvh, mirt_hit* out)
{
    if (!ctx_ok(c, true, "mirt_intersect_rays")) return MIRT_E_NOSCENE;
    if (n < 0 || (n > 0 && (!rays || !out))) {
        set_error("mirt_intersect_rays: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (use_bvh && c->num_nodes == 0) {
        set_error("mirt_intersect_rays: use_bvh set but no tree uploaded");
        return MIRT_E_NOSCENE;
    }
    if (n == 0) return MIRT_OK;
    int rc = ensure(&c->d_in, &c->in_cap, sizeof(mirt_ray) * (size_t)n);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, sizeof(mirt_hit) * (size_t)n);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_in, rays, sizeof(mirt_ray) * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    const int bt = batch_threads(c, n);
    if (!use_bvh) {
        rc = launch_brute(c, n);
        if (rc) return rc;
        brute_finish_kernel<<<(n + 255) / 256, 256, 0, c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n,
                                                                    c->d_keys, (mirt_hit*)c->d_res);
    } else if (quad_batch(c, n)) {
        intersect_quad_kernel<false><<<(n + kQuadBatchThreads / 4 - 1) / (kQuadBatchThreads / 4), kQuadBatchThreads, 0,
                                        c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n, (mirt_hit*)c->d_res,
                                                     nullptr);
    } else if (c->fast_slab) {
        intersect_kernel<true><<<(n + bt - 1) / bt, bt, 0, c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n,
                                                                      use_bvh, (mirt_hit*)c->d_res);
    } else {
        intersect_kernel<false><<<(n + bt - 1) / bt, bt, 0, c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n,
                                                                       use_bvh, (mirt_hit*)c->d_res);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->d_res, sizeof(mirt_hit) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    return MIRT_OK;
}

int mirt_any_hit_rays(mirt_ctx* c, const mirt_ray* rays, int n, int use_bvh, int32_t* out)
{
    if (!ctx_ok(c, true, "mirt_any_hit_rays")) return MIRT_E_NOSCENE;
    if (n < 0 || (n > 0 && (!rays || !out))) {
        set_error("mirt_any_hit_rays: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (use_bvh && c->num_nodes == 0) {
        set_error("mirt_any_hit_rays: use_bvh set but no tree uploaded");
        return MIRT_E_NOSCENE;
    }
    if (n == 0) return MIRT_OK;
    int rc = ensure(&c->d_in, &c->in_cap, sizeof(mirt_ray) * (size_t)n);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, sizeof(int32_t) * (size_t)n);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_in, rays, sizeof(mirt_ray) * (size_t)n, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipEventRecord(c->ev0, c->stream));
    const int bt = batch_threads(c, n);
    if (!use_bvh) {
        rc = launch_brute(c, n);
        if (rc) return rc;
        keys_to_flags_kernel<<<(n + 255) / 256, 256, 0, c->stream>>>(c->d_keys, n, (int32_t*)c->d_res);
    } else if (quad_batch(c, n)) {
        intersect_quad_kernel<true><<<(n + kQuadBatchThreads / 4 - 1) / (kQuadBatchThreads / 4), kQuadBatchThreads, 0,
                                       c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n, nullptr,
                                                    (int32_t*)c->d_res);
    } else if (c->fast_slab) {
        bvh_any_kernel<true><<<(n + bt - 1) / bt, bt, 0, c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n,
                                                                    (int32_t*)c->d_res);
    } else {
        bvh_any_kernel<false><<<(n + bt - 1) / bt, bt, 0, c->stream>>>(dev_scene(c), (const mirt_ray*)c->d_in, n,
                                                                     (int32_t*)c->d_res);
    }
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(c->ev1, c->stream));
    HIP_TRY(hipMemcpyAsync(out, c->d_res, sizeof(int32_t) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipEventElapsedTime(&c->last_ms, c->ev0, c->ev1));
    return MIRT_OK;
}

int mirt_bvh_overlay(mirt_ctx* c, const mirt_camera* cam, int width, int height, int max_levels, mirt_rgba8* out)
{
    if (!ctx_ok(c, true, "mirt_bvh_overlay")) return MIRT_E_NOSCENE;
    if (!cam || width <= 0 || height <= 0 || !out || (size_t)width * height > ((size_t)1 << 31)) {
        set_error("mirt_bvh_overlay: invalid arguments");
        return MIRT_E_INVALID;
    }
    OverlayConst o{};
    o.px = cam->position.x; o.py = cam->position.y; o.pz = cam->position.z;
    o.fx = cam->forward.x; o.fy = cam->forward.y; o.fz = cam->forward.z;
    o.rx = cam->right.x; o.ry = cam->right.y; o.rz = cam->right.z;
    o.ux = cam->up.x; o.uy = cam->up.y; o.uz = cam->up.z;
    const float fov_rad = (float)((double)cam->fov * (M_PI / 180.0));  // bvh_visualiser.c:26
    o.half_h = tanf(fov_rad / 2.0f);                                    // :27 (float tanf)
    o.half_w = (float)width / (float)height * o.half_h;                 // :28-29
    o.width = width;
    o.height = height;
    o.max_levels = max_levels;
    const size_t pixels = (size_t)width * height;
    int rc = ensure((void**)&c->d_overlay, &c->overlay_cap, 4 * pixels);
    if (!rc) rc = ensure((void**)&c->d_out, &c->out_cap, 4 * pixels + 4);
    if (rc) return rc;
    HIP_TRY(hipMemsetAsync(c->d_overlay, 0, 4 * pixels, c->stream));
    const uint64_t lines = (uint64_t)c->num_nodes * 60;
    if (lines > 0xffffffffull) {
        set_error("mirt_bvh_overlay: too many nodes");
        return MIRT_E_INVALID;
    }
    if (lines) {
        overlay_lines_kernel<<<(unsigned)((lines + 255) / 256), 256, 0, c->stream>>>(o, c->d_nodes32, c->d_ndepth,
                                                                                     (uint32_t)lines, c->d_overlay);
        HIP_TRY(hipGetLastError());
    }
    overlay_colour_kernel<<<(unsigned)((pixels + 255) / 256), 256, 0, c->stream>>>(c->d_overlay, c->d_ndepth, pixels,
                                                                                 c->d_out);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, c->d_out, 4 * pixels, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

int mirt_camera_rays_uv(mirt_ctx* c, const mirt_camera* cam, int width, int height, const float* uv, int n,
                        mirt_ray* out)
{
    if (!ctx_ok(c, false, "mirt_camera_rays_uv")) return MIRT_E_INVALID;
    if (!cam || width <= 0 || height <= 0 || n < 0 || (n > 0 && (!uv || !out))) {
        set_error("mirt_camera_rays_uv: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (n == 0) return MIRT_OK;
    mirt_frame_desc fd{};
    fd.width = width;
    fd.height = height;
    fd.row_block = 8;
    fd.num_shards = 1;
    const FrameConst f = make_frame_const(cam, &fd);
    int rc = ensure(&c->d_in, &c->in_cap, 8 * (size_t)n);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, sizeof(mirt_ray) * (size_t)n);
    if (rc) return rc;
    HIP_TRY(hipMemcpyAsync(c->d_in, uv, 8 * (size_t)n, hipMemcpyHostToDevice, c->stream));
    camera_uv_kernel<<<(n + 255) / 256, 256, 0, c->stream>>>(f, (const float2*)c->d_in, n, (mirt_ray*)c->d_res);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, c->d_res, sizeof(mirt_ray) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

int mirt_sphere_pairs(mirt_ctx* c, const mirt_ray* rays, const mirt_sphere* spheres, int n, mirt_hit* out)
{
    if (!ctx_ok(c, false, "mirt_sphere_pairs")) return MIRT_E_INVALID;
    if (n < 0 || (n > 0 && (!rays || !spheres || !out))) {
        set_error("mirt_sphere_pairs: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (n == 0) return MIRT_OK;
    const size_t rb = sizeof(mirt_ray) * (size_t)n, sb = sizeof(mirt_sphere) * (size_t)n;
    int rc = ensure(&c->d_in, &c->in_cap, rb + sb + 16);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, sizeof(mirt_hit) * (size_t)n);
    if (rc) return rc;
    char* din = (char*)c->d_in;
    HIP_TRY(hipMemcpyAsync(din, rays, rb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(din + rb, spheres, sb, hipMemcpyHostToDevice, c->stream));
    sphere_pairs_kernel<<<(n + 255) / 256, 256, 0, c->stream>>>((const mirt_ray*)din, (const mirt_sphere*)(din + rb),
                                                               n, (mirt_hit*)c->d_res);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, c->d_res, sizeof(mirt_hit) * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

int mirt_aabb_pairs(mirt_ctx* c, const mirt_ray* rays, const mirt_aabb* boxes, int n, int32_t* out)
{
    if (!ctx_ok(c, false, "mirt_aabb_pairs")) return MIRT_E_INVALID;
    if (n < 0 || (n > 0 && (!rays || !boxes || !out))) {
        set_error("mirt_aabb_pairs: invalid arguments");
        return MIRT_E_INVALID;
    }
    if (n == 0) return MIRT_OK;
    const size_t rb = sizeof(mirt_ray) * (size_t)n, bb = sizeof(mirt_aabb) * (size_t)n;
    int rc = ensure(&c->d_in, &c->in_cap, rb + bb + 16);
    if (!rc) rc = ensure(&c->d_res, &c->res_cap, 4 * (size_t)n);
    if (rc) return rc;
    char* din = (char*)c->d_in;
    HIP_TRY(hipMemcpyAsync(din, rays, rb, hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(din + rb, boxes, bb, hipMemcpyHostToDevice, c->stream));
    aabb_pairs_kernel<<<(n + 255) / 256, 256, 0, c->stream>>>((const mirt_ray*)din, (const mirt_aabb*)(din + rb), n,
                                                             (int32_t*)c->d_res);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipMemcpyAsync(out, c->d_res, 4 * (size_t)n, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return MIRT_OK;
}

float mirt_last_kernel_ms(mirt_ctx* c) { return c ? c->last_ms : 0.0f; }

void* mirt_ctx_stream(mirt_ctx* c)
{
    return c ? (void*)c->stream : nullptr;
}

int mirt_last_phase_ms(mirt_ctx* c, float* phase)
{
    if (!c || !phase) return MIRT_E_INVALID;
    if (!c->phases_valid) {
        set_error("mirt_last_phase_ms: the last frame did not use the wavefront schedule");
        return MIRT_E_INVALID;
    }
    HIP_TRY(hipSetDevice(c->device));
    const uint32_t k = (c->ph_next + kPhaseRing - 1) % kPhaseRing;
    HIP_TRY(hipEventSynchronize(c->ph2[k]));
    HIP_TRY(hipEventElapsedTime(&phase[0], c->ph0[k], c->ph1[k]));
    HIP_TRY(hipEventElapsedTime(&phase[1], c->ph1[k], c->ph2[k]));
    return MIRT_OK;
}

int mirt_phase_log(mirt_ctx* c, float* out, int max)
{
    if (!c || max < 0 || (max > 0 && !out)) return MIRT_E_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    const int n = std::min<int>(max, (int)c->ph_count);
    for (int j = 0; j < n; j++) {  // oldest first
        const uint32_t k = (c->ph_next + kPhaseRing - (uint32_t)(n - j)) % kPhaseRing;
        HIP_TRY(hipEventSynchronize(c->ph2[k]));
        HIP_TRY(hipEventElapsedTime(&out[2 * j], c->ph0[k], c->ph1[k]));
        HIP_TRY(hipEventElapsedTime(&out[2 * j + 1], c->ph1[k], c->ph2[k]));
    }
    return n;
}

int mirt_set_option(mirt_ctx* c, int option, int value)
{
    if (!c) return MIRT_E_INVALID;
    switch (option) {
    case MIRT_OPT_TRAVERSAL:
        // mirt 0.2 numbered WAVEFRONT 1 (0.1 and 0.3+: 5); 1 stays a
        // deprecated alias so binaries built against the 0.2 header keep working
        if (value == MIRT_TRAV_WAVEFRONT_V02) value = MIRT_TRAV_WAVEFRONT;
        if (value != MIRT_TRAV_TILE && value != MIRT_TRAV_WAVEFRONT) break;
        c->trav = value;
        return MIRT_OK;
    case MIRT_OPT_FAST_SLAB:
        c->fast_slab = value != 0;
        return MIRT_OK;
    case MIRT_OPT_BOUNCE_THRESHOLD:
        if (value < 0 || value > 64) break;
        c->bounce_threshold = value;
        return MIRT_OK;
    case MIRT_OPT_DEFER:
        c->defer = value != 0;
        return MIRT_OK;
    case MIRT_OPT_PRUNE:
        c->prune = value != 0;
        return MIRT_OK;
    case MIRT_OPT_ORDERED:
        c->ordered = value != 0;
        return MIRT_OK;
    case MIRT_OPT_BOUNCE_BLOCKS:
        if (value < 0) break;
        c->bounce_blocks_opt = value;
        return MIRT_OK;
    case MIRT_OPT_QUAD_DRAIN:
        c->quad_drain = value != 0;
        return MIRT_OK;
    case MIRT_OPT_QUAD_BATCH:
        c->quad_batch = value != 0;
        return MIRT_OK;
    case MIRT_OPT_ZERO_COPY:
        if (value < 0 || value > 2) break;
        c->zero_copy = value;
        return MIRT_OK;
    case MIRT_OPT_DEBUG_STALL_MS:
        if (value < 0 || value > 10000) break;
        c->debug_stall_ms = value;
        return MIRT_OK;
    case MIRT_OPT_QUEUE_ORDER:
        if (value < 0 || value > 2) break;
        c->queue_order = value;
        return MIRT_OK;
    case MIRT_OPT_LEAF_BATCH:
        if (value < 0 || value > 2) break;
        c->leaf_batch_opt = value;
        return MIRT_OK;
    case MIRT_OPT_BLOCK_WAVES:
        if (value != 1 && value != 2 && value != 4 && value != 8) break;
        c->block_waves = value;
        return MIRT_OK;
    default:
        break;
    }
    set_error("mirt_set_option: bad option %d / value %d", option, value);
    return MIRT_E_INVALID;
}

int mirt_get_option(mirt_ctx* c, int option)
{
    if (!c) return MIRT_E_INVALID;
    if (option == MIRT_OPT_TRAVERSAL) return c->trav;
    if (option == MIRT_OPT_FAST_SLAB) return c->fast_slab;
    if (option == MIRT_OPT_BLOCK_WAVES) return c->block_waves;
    if (option == MIRT_OPT_DEFER) return c->defer;
    if (option == MIRT_OPT_BOUNCE_THRESHOLD) return c->bounce_threshold;
    if (option == MIRT_OPT_PRUNE) return c->prune;
    if (option == MIRT_OPT_ORDERED) return c->ordered;
    if (option == MIRT_OPT_BOUNCE_BLOCKS) return c->bounce_blocks_opt;
    if (option == MIRT_OPT_QUAD_DRAIN) return c->quad_drain;
    if (option == MIRT_OPT_QUAD_BATCH) return c->quad_batch;
    if (option == MIRT_OPT_ZERO_COPY) return c->zero_copy;
    if (option == MIRT_OPT_QUEUE_ORDER) return c->queue_order;
    if (option == MIRT_OPT_DEBUG_STALL_MS) return c->debug_stall_ms;
    if (option == MIRT_OPT_LEAF_BATCH) return leaf_batch(c) ? 1 : 0;  // in effect for the uploaded scene
    set_error("mirt_get_option: bad option %d", option);
    return MIRT_E_INVALID;
}

}  // extern "C"
