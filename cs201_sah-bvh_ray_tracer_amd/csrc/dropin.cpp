// The reference's per-ray call surface (include/mirt_dropin.h) over the batch
// C ABI: one launch per call on a process-wide context, the caller's scene
// uploaded once per (sphere array, count, tree root) key.
//
//   mirt_get_camera_ray        ray.c:17-32      -> mirt_camera_rays_uv, n = 1
//   mirt_trace_ray             renderer.c:21-77 -> mirt_trace_rays_at, pixel = call counter
//   mirt_ray_sphere_intersect  hit.c:19-39      -> mirt_sphere_pairs, n = 1
//   mirt_ray_aabb_intersect    hit.c:49-82      -> mirt_aabb_pairs, n = 1
//   mirt_ray_bvh_intersect     hit.c:91-109     -> mirt_intersect_rays (BVH), n = 1
#include <cstring>
#include <mutex>
#include <new>
#include <vector>

#include "../../include/mirt_dropin.h"
#include "internal.h"

namespace {

struct DropinState {
    std::mutex mu;
    mirt_ctx* ctx = nullptr;
    int device = 0, width = 800, height = 600;  // constants.h:7-8 defaults
    // the uploaded scene's key (caller memory is never kept beyond the key)
    const mirt_sphere* spheres = nullptr;
    int num_spheres = -1;
    const mirt_bvh_node* root = nullptr;
    bool bound = false;
    uint64_t seed = 1;
    uint32_t sample = 0, pixel = 0;
    int status = MIRT_OK;
};

DropinState& state()
{
    static DropinState s;
    return s;
}

int ensure_ctx(DropinState& s)
{
    if (s.ctx) return MIRT_OK;
    return mirt_create(s.device, &s.ctx);
}

int bind(DropinState& s, const mirt_sphere* sp, int ns, const mirt_bvh_node* root)
{
    if (s.bound && s.spheres == sp && s.num_spheres == ns && s.root == root) return MIRT_OK;
    s.bound = false;
    const int rc = mirt_scene_upload(s.ctx, sp, ns, root);
    if (rc) return rc;
    s.spheres = sp;
    s.num_spheres = ns;
    s.root = root;
    s.bound = true;
    return MIRT_OK;
}

// Lowest and highest leaf sphere pointer of a pointer tree (bvh.c:131-137:
// every leaf, empty ones included, points into the build's array).
void leaf_range(const mirt_bvh_node* root, const mirt_sphere** lo, const mirt_sphere** hi)
{
    std::vector<const mirt_bvh_node*> todo{root};  // explicit stack: any tree depth
    while (!todo.empty()) {
        const mirt_bvh_node* n = todo.back();
        todo.pop_back();
        if (!n) continue;
        if (n->sphere) {
            if (!*lo || n->sphere < *lo) *lo = n->sphere;
            if (!*hi || n->sphere > *hi) *hi = n->sphere;
            continue;
        }
        todo.push_back(n->right);
        todo.push_back(n->left);
    }
}

mirt_hit_record to_record(const mirt_hit& h, mirt_sphere* base)
{
    mirt_hit_record r;
    std::memset(&r, 0, sizeof r);  // hit.c:20: a miss is the zero record
    if (h.hit) {
        r.t = h.t;
        r.point = h.point;
        r.normal = h.normal;
        r.hit_something = 1;
        r.object = base + h.sphere;
    }
    return r;
}

template <class F>
int guarded(DropinState& s, F&& body)
{
    int rc;
    try {
        rc = ensure_ctx(s);
        if (!rc) rc = body();
    } catch (const std::bad_alloc&) {
        mirt::set_error("mirt drop-in: out of host memory");
        rc = MIRT_E_NOMEM;
    } catch (...) {
        mirt::set_error("mirt drop-in: unexpected exception");
        rc = MIRT_E_INVALID;
    }
    s.status = rc;
    return rc;
}

}  // namespace

extern "C" {

int mirt_dropin_init(int device, int width, int height)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    if (width <= 0 || height <= 0) {
        mirt::set_error("mirt_dropin_init: invalid frame size %dx%d", width, height);
        return s.status = MIRT_E_INVALID;
    }
    if (s.ctx && s.device != device) {
        mirt_destroy(s.ctx);
        s.ctx = nullptr;
        s.bound = false;
    }
    s.device = device;
    s.width = width;
    s.height = height;
    return guarded(s, [] { return MIRT_OK; });
}

void mirt_dropin_release(void)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.ctx) mirt_destroy(s.ctx);
    s.ctx = nullptr;
    s.bound = false;
}

void mirt_dropin_rng(uint64_t seed, uint32_t sample)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    s.seed = seed;
    s.sample = sample;
    s.pixel = 0;
}

void mirt_dropin_invalidate(void)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    s.bound = false;
}

int mirt_dropin_status(void)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    return s.status;
}

mirt_ray mirt_get_camera_ray(mirt_camera* camera, float u, float v)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    mirt_ray out;
    std::memset(&out, 0, sizeof out);
    const float uv[2] = {u, v};
    guarded(s, [&] { return mirt_camera_rays_uv(s.ctx, camera, s.width, s.height, uv, 1, &out); });
    return out;
}

mirt_rgba8 mirt_trace_ray(mirt_ray ray, mirt_sphere* spheres, int num_spheres, int depth, mirt_bvh_node* bvh)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    mirt_rgba8 out{0, 0, 0, 255};  // renderer.c:23-24's value for depth <= 0
    if (depth <= 0) {
        s.pixel++;
        s.status = MIRT_OK;
        return out;
    }
    guarded(s, [&] {
        int rc = bind(s, spheres, num_spheres, bvh);
        if (!rc) rc = mirt_trace_rays_at(s.ctx, &ray, 1, depth, bvh != nullptr, s.seed, s.sample, s.pixel, &out);
        return rc;
    });
    s.pixel++;
    return out;
}

mirt_hit_record mirt_ray_sphere_intersect(mirt_ray ray, mirt_sphere* sphere)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    mirt_hit h;
    std::memset(&h, 0, sizeof h);
    if (guarded(s, [&] { return mirt_sphere_pairs(s.ctx, &ray, sphere, 1, &h); })) std::memset(&h, 0, sizeof h);
    h.sphere = 0;  // the pair's own sphere
    return to_record(h, sphere);
}

int mirt_ray_aabb_intersect(mirt_ray ray, mirt_aabb box)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    int32_t hit = 0;
    guarded(s, [&] { return mirt_aabb_pairs(s.ctx, &ray, &box, 1, &hit); });
    return hit;
}

mirt_hit_record mirt_ray_bvh_intersect(mirt_ray ray, mirt_bvh_node* node)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    mirt_hit h;
    std::memset(&h, 0, sizeof h);
    const mirt_sphere* base = nullptr;
    const int rc = guarded(s, [&] {
        if (!node) {
            mirt::set_error("mirt_ray_bvh_intersect: null tree");
            return (int)MIRT_E_INVALID;
        }
        if (!(s.bound && s.root == node)) {
            // a tree seen without its sphere array: the leaves span it
            const mirt_sphere *lo = nullptr, *hi = nullptr;
            leaf_range(node, &lo, &hi);
            if (!lo) {
                mirt::set_error("mirt_ray_bvh_intersect: tree without leaves");
                return (int)MIRT_E_INVALID;
            }
            if (int r = bind(s, lo, (int)(hi - lo) + 1, node)) return r;
        }
        base = s.spheres;
        return mirt_intersect_rays(s.ctx, &ray, 1, 1, &h);
    });
    if (rc) std::memset(&h, 0, sizeof h);
    return to_record(h, const_cast<mirt_sphere*>(base));
}

}  // extern "C"
