// Host-side inputs of the render path: glibc rand() restated, the two
// synthetic sphere-scene generators and the camera, plus error/shard helpers.
//
// These run once per scene / per frame on the host; the per-pixel work is in
// render.hip. Compiled with -ffp-contract=off and no -march.
#include <cmath>
#include <cstdint>
#include <cstring>

#include <algorithm>

#include "internal.h"
#include "shard.h"

static_assert(sizeof(mirt_vec3) == 12, "Vec3 is 12 B (vec3.h:3-7)");
static_assert(sizeof(mirt_sphere) == 20, "Sphere is 20 B (sphere.h:7-11)");
static_assert(sizeof(mirt_ray) == 24, "Ray is 24 B (ray.h:5-8)");
static_assert(sizeof(mirt_camera) == 64, "Camera is 64 B (camera.h:5-14)");
static_assert(sizeof(mirt_aabb) == 24, "AABB is 24 B (bvh.h:7-10)");
static_assert(sizeof(mirt_bvh_node) == 56, "BVHNode is 56 B (bvh.h:12-18)");
static_assert(sizeof(mirt_hit_record) == 40, "HitRecord is 40 B (hit.h:8-14)");
static_assert(sizeof(mirt_hit) == 40, "mirt_hit is 40 B");
static_assert(sizeof(mirt_node) == 32, "flat node is 32 B");
static_assert(offsetof(mirt_bvh_node, left) == 24 && offsetof(mirt_bvh_node, sphere) == 40 &&
                  offsetof(mirt_bvh_node, sphere_count) == 48,
              "BVHNode field offsets");
static_assert(offsetof(mirt_hit_record, object) == 32, "HitRecord.object at 32");

namespace mirt {

static thread_local char g_err[512];

void set_error(const char* fmt, ...)
{
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
}

bool frame_desc_valid(const mirt_frame_desc* fd)
{
    if (!fd) return false;
    if (fd->width <= 0 || fd->height <= 0 || fd->max_depth < 0 || fd->max_depth > 8) return false;
    if (fd->row_block <= 0 || fd->num_shards <= 0 || fd->shard < 0 || fd->shard >= fd->num_shards) return false;
    if (fd->accumulate && fd->frames <= 0) return false;
    if (fd->samples < 0 || fd->samples > 64) return false;
    if (fd->lead_skip < 0 || fd->lead_skip >= kLeadRounds || (fd->lead_skip > 0 && fd->num_shards < 2)) return false;
    const int64_t samples = fd->samples > 1 ? fd->samples : 1;
    return (int64_t)fd->width * fd->height * samples <= (int64_t)1 << 31;
}

int shard_row_count(const mirt_frame_desc* fd)
{
    const int rb = fd->row_block, n = fd->num_shards, d = fd->lead_skip;
    const int blocks = (fd->height + rb - 1) / rb;
    const int c = shard_block_count(fd->shard, blocks, n, d);
    if (c == 0) return 0;
    // every block is full but the image's last one, if it is this shard's
    const int last = shard_block(fd->shard, c - 1, n, d);
    return (c - 1) * rb + std::min(rb, fd->height - last * rb);
}

}  // namespace mirt

extern "C" {

const char* mirt_version(void) { return "mirt 0.6 (gfx950)"; }
const char* mirt_last_error(void) { return mirt::g_err; }

// ------------------------------------------------------------------ rand
// glibc srandom_r/random_r, TYPE_3: x[i] = x[i-3] + x[i-31] (mod 2^32), the
// output drops the low bit. Seeding runs the Park-Miller LCG (16807) through
// Schrage's decomposition, then discards 310 outputs.
static const int kDeg = 31, kSep = 3;

void mirt_srand(mirt_rand_state* st, unsigned int seed)
{
    if (seed == 0) seed = 1;
    int32_t w = (int32_t)seed;
    st->r[0] = w;
    for (int i = 1; i < kDeg; i++) {
        const int64_t hi = w / 127773, lo = w % 127773;
        int64_t nx = 16807 * lo - 2836 * hi;
        w = (int32_t)nx;
        if (w < 0) w += 2147483647;
        st->r[i] = w;
    }
    st->f = kSep;
    st->b = 0;
    for (int i = 0; i < 10 * kDeg; i++) (void)mirt_rand(st);
}

int mirt_rand(mirt_rand_state* st)
{
    const uint32_t v = (uint32_t)st->r[st->f] + (uint32_t)st->r[st->b];
    st->r[st->f] = (int32_t)v;
    if (++st->f >= kDeg) {
        st->f = 0;
        ++st->b;
    } else if (++st->b >= kDeg) {
        st->b = 0;
    }
    return (int)(v >> 1);
}

// sphere.c:14-16 random_float: lo + ((float)rand() / RAND_MAX) * (hi - lo)
static float uniform_draw(mirt_rand_state* st, float lo, float hi)
{
    const float f = (float)mirt_rand(st) / 2147483648.0f;  // (float)RAND_MAX == 2^31
    return lo + f * (hi - lo);
}

// sphere.c:52-59 create_random_sphere, called n times as main.c:218-221.
// Designated initialisers evaluate in order under gcc: x, y, z, r, R, G, B.
int mirt_scene_random(mirt_rand_state* st, mirt_sphere* out, int n)
{
    if (!st || (!out && n > 0) || n < 0) return MIRT_E_INVALID;
    for (int i = 0; i < n; i++) {
        mirt_sphere s;
        s.center.x = uniform_draw(st, -40.0f, 40.0f);
        s.center.y = uniform_draw(st, -20.0f, 20.0f);
        s.center.z = uniform_draw(st, -10.0f, 5.0f);
        s.radius = uniform_draw(st, 0.5f, 5.0f);
        s.color.r = (uint8_t)(mirt_rand(st) % 256);
        s.color.g = (uint8_t)(mirt_rand(st) % 256);
        s.color.b = (uint8_t)(mirt_rand(st) % 256);
        s.color.a = 255;
        out[i] = s;
    }
    return MIRT_OK;
}

// benchmark.c:307-314 centre = (float)rand()/RAND_MAX*world - world/2 per
// axis, then create_benchmark_sphere (sphere.c:34-41): r = 0.5, 3 colour draws.
int mirt_scene_benchmark(mirt_rand_state* st, mirt_sphere* out, int n, float world)
{
    if (!st || (!out && n > 0) || n < 0) return MIRT_E_INVALID;
    const float half = world / 2;
    for (int i = 0; i < n; i++) {
        mirt_sphere s;
        s.center.x = (float)mirt_rand(st) / 2147483648.0f * world - half;
        s.center.y = (float)mirt_rand(st) / 2147483648.0f * world - half;
        s.center.z = (float)mirt_rand(st) / 2147483648.0f * world - half;
        s.radius = 0.5f;
        s.color.r = (uint8_t)(mirt_rand(st) % 256);
        s.color.g = (uint8_t)(mirt_rand(st) % 256);
        s.color.b = (uint8_t)(mirt_rand(st) % 256);
        s.color.a = 255;
        out[i] = s;
    }
    return MIRT_OK;
}

// ---------------------------------------------------------------- camera
void mirt_camera_default(mirt_camera* c)  // main.c:203-211
{
    std::memset(c, 0, sizeof *c);
    c->position = {0.0f, 4.0f, 50.0f};
    c->forward = {0.0f, 0.0f, -1.0f};
    c->right = {1.0f, 0.0f, 0.0f};
    c->up = {0.0f, 1.0f, 0.0f};
    c->yaw = (float)-M_PI;
    c->pitch = 0.0f;
    c->fov = 45.0f;
    c->move = 0;
}

static mirt_vec3 v_norm(mirt_vec3 a)  // vec3.c:21-24 (double sqrt of the float sum)
{
    float sq = a.x * a.x;
    sq = sq + a.y * a.y;
    sq = sq + a.z * a.z;
    const float len = (float)std::sqrt((double)sq);
    if (len == 0.0f) return {0.0f, 0.0f, 0.0f};
    return {a.x / len, a.y / len, a.z / len};
}

static mirt_vec3 v_cross(mirt_vec3 a, mirt_vec3 b)  // vec3.c:38-44
{
    return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

void mirt_camera_update(mirt_camera* c)  // camera.c:10-18 (libm in double)
{
    const double cp = std::cos((double)c->pitch), sp = std::sin((double)c->pitch);
    const double sy = std::sin((double)c->yaw), cy = std::cos((double)c->yaw);
    c->forward.x = (float)(cp * sy);
    c->forward.y = (float)sp;
    c->forward.z = (float)(cp * cy);
    c->forward = v_norm(c->forward);
    c->right = v_norm(v_cross(c->forward, {0.0f, 1.0f, 0.0f}));
    c->up = v_norm(v_cross(c->right, c->forward));
}

// benchmark.c:176-185 / 228-237: direction = normalize((float)rand()/RAND_MAX
// * 2 - 1 per axis, x then y then z), origin (0,0,0); n rays off the stream.
int mirt_bench_rays(mirt_rand_state* st, mirt_ray* out, int n)
{
    if (!st || (!out && n > 0) || n < 0) return MIRT_E_INVALID;
    for (int i = 0; i < n; i++) {
        mirt_vec3 d;
        d.x = (float)mirt_rand(st) / 2147483648.0f * 2 - 1;
        d.y = (float)mirt_rand(st) / 2147483648.0f * 2 - 1;
        d.z = (float)mirt_rand(st) / 2147483648.0f * 2 - 1;
        out[i].origin = {0.0f, 0.0f, 0.0f};
        out[i].direction = v_norm(d);
    }
    return MIRT_OK;
}

int mirt_shard_rows(const mirt_frame_desc* fd, int32_t* rows)
{
    if (!mirt::frame_desc_valid(fd)) {
        mirt::set_error("mirt_shard_rows: invalid frame descriptor");
        return MIRT_E_INVALID;
    }
    const int n = mirt::shard_row_count(fd);
    if (rows) {
        const int rb = fd->row_block;
        for (int r = 0; r < n; r++)
            rows[r] = mirt::shard_block(fd->shard, r / rb, fd->num_shards, fd->lead_skip) * rb + r % rb;
    }
    return n;
}

}  // extern "C"
