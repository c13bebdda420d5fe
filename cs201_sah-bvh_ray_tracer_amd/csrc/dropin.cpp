// The reference's per-ray call surface (include/mirt_dropin.h) over the batch
// C ABI: one launch per call on a process-wide context, the caller's scene
// uploaded once per (sphere array, count, tree root, content fingerprint)
// key. The fingerprint matters because benchmark.c:306-324 frees the tree and
// the spheres and mallocs the next size's: the allocator hands the same
// addresses back (glibc's tcache is LIFO and the root is freed last), so the
// pointers alone would keep walking the previous, freed scene.
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
    uint64_t fingerprint = 0;       // scene_fingerprint at bind (sphere samples from that call's arguments)
    uint64_t tree_fp = 0;           // tree_fingerprint at bind (what ray_bvh_intersect re-checks)
    bool bound = false;
    // mirt_dropin_scene: the caller's whole sphere array, for trees built over
    // part of it (benchmark.c:317 builds over [0, n - 1) of n spheres)
    const mirt_sphere* decl = nullptr;
    int decl_n = 0;
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

// FNV-1a 64 over a byte range.
uint64_t fnv(uint64_t h, const void* p, size_t n)
{
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

// A cheap content fingerprint of a tree, read only through the caller's
// CURRENT tree pointer: the first 31 nodes in breadth-first order (bounds,
// sphere count, and the sphere a non-empty leaf tests, read through that
// leaf's own pointer). Never through a sphere pointer kept from an earlier
// call: benchmark.c:323-324 frees the previous point's array, and at 10k
// spheres and up glibc returns it to the kernel (munmap), so a stored pointer
// may point at unmapped memory. ~60 small loads, against a GPU launch per call.
uint64_t tree_fingerprint(const mirt_bvh_node* root)
{
    uint64_t h = 0xcbf29ce484222325ull;
    const mirt_bvh_node* q[31];
    int head = 0, tail = 0;
    if (root) q[tail++] = root;
    while (head < tail) {
        const mirt_bvh_node* n = q[head++];
        h = fnv(h, &n->bounds, sizeof n->bounds);
        h = fnv(h, &n->sphere_count, sizeof n->sphere_count);
        if (n->sphere) {
            if (n->sphere_count > 0) h = fnv(h, n->sphere, sizeof(mirt_sphere));
            continue;
        }
        for (const mirt_bvh_node* c : {n->left, n->right})
            if (c && tail < 31) q[tail++] = c;
    }
    return h;
}

// The same plus up to 32 spheres strided over the array the caller passes IN
// THIS CALL (sp, ns are current arguments, so reading them is the caller's
// own contract, as trace_ray reading spheres[] is).
uint64_t scene_fingerprint(const mirt_sphere* sp, int ns, const mirt_bvh_node* root)
{
    uint64_t h = fnv(tree_fingerprint(root), &ns, sizeof ns);
    if (sp && ns > 0) {
        const int step = ns > 32 ? ns / 32 : 1;
        for (int i = 0; i < ns; i += step) h = fnv(h, &sp[i], sizeof(mirt_sphere));
        h = fnv(h, &sp[ns - 1], sizeof(mirt_sphere));
    }
    return h;
}

int bind(DropinState& s, const mirt_sphere* sp, int ns, const mirt_bvh_node* root)
{
    const uint64_t fp = scene_fingerprint(sp, ns, root);
    if (s.bound && s.spheres == sp && s.num_spheres == ns && s.root == root && s.fingerprint == fp) return MIRT_OK;
    s.bound = false;
    const int rc = mirt_scene_upload(s.ctx, sp, ns, root);
    if (rc) return rc;
    s.spheres = sp;
    s.num_spheres = ns;
    s.root = root;
    s.fingerprint = fp;
    s.tree_fp = tree_fingerprint(root);
    s.bound = true;
    return MIRT_OK;
}

// The sphere array a pointer tree seen without one spans (bvh.c:131-137):
// *lo = the lowest leaf sphere pointer (empty leaves included: a 0-sphere
// leaf points at spheres[start] of its range), *count = up to the end of the
// highest NON-empty leaf's range. A 0-sphere leaf at the very end of the
// build range points one past it (&spheres[end]): that element
// is not read -- its index is the never-hit sentinel (count) -- unless the
// caller declared a longer array with mirt_dropin_scene.
bool leaf_range(const mirt_bvh_node* root, const mirt_sphere** lo, int* count)
{
    const mirt_sphere *low = nullptr, *end = nullptr;
    std::vector<const mirt_bvh_node*> todo{root};  // explicit stack: any tree depth
    while (!todo.empty()) {
        const mirt_bvh_node* n = todo.back();
        todo.pop_back();
        if (!n) continue;
        if (n->sphere) {
            if (!low || n->sphere < low) low = n->sphere;
            if (n->sphere_count > 0 && (!end || n->sphere + n->sphere_count > end)) end = n->sphere + n->sphere_count;
            continue;
        }
        todo.push_back(n->right);
        todo.push_back(n->left);
    }
    if (!low) return false;
    *lo = low;
    *count = end && end > low ? (int)(end - low) : 0;
    return true;
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

int mirt_dropin_scene(const mirt_sphere* spheres, int num_spheres)
{
    DropinState& s = state();
    std::lock_guard<std::mutex> lk(s.mu);
    if (num_spheres < 0 || (num_spheres > 0 && !spheres)) {
        mirt::set_error("mirt_dropin_scene: invalid arguments");
        return s.status = MIRT_E_INVALID;
    }
    s.decl = num_spheres > 0 ? spheres : nullptr;
    s.decl_n = num_spheres;
    return s.status = MIRT_OK;
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
        // the scene bound by the last trace_ray (or this call), if the tree
        // is still the same (pointer and content, read through `node` only:
        // the stored sphere pointer may belong to a freed array)
        // (and its leaves still point into the bound array: a tree rebuilt
        // at the same address with the same content over a RELOCATED array
        // fingerprints the same, but its hit records must point into the
        // new array -- one leaf, reached through the current tree, tells)
        const mirt_bvh_node* leaf = node;
        while (leaf && !leaf->sphere) leaf = leaf->left ? leaf->left : leaf->right;
        const bool same_array = leaf && leaf->sphere >= s.spheres && leaf->sphere < s.spheres + s.num_spheres;
        if (!(s.bound && s.root == node && same_array && s.tree_fp == tree_fingerprint(node))) {
            // a tree seen without its sphere array: the leaves span it, or
            // the array the caller declared (mirt_dropin_scene) holds them
            const mirt_sphere* lo = nullptr;
            int count = 0;
            if (!leaf_range(node, &lo, &count)) {
                mirt::set_error("mirt_ray_bvh_intersect: tree without leaves");
                return (int)MIRT_E_INVALID;
            }
            if (s.decl && lo >= s.decl && lo + count <= s.decl + s.decl_n) {
                lo = s.decl;
                count = s.decl_n;
            }
            if (int r = bind(s, lo, count, node)) return r;
        }
        base = s.spheres;
        return mirt_intersect_rays(s.ctx, &ray, 1, 1, &h);
    });
    if (rc) std::memset(&h, 0, sizeof h);
    return to_record(h, const_cast<mirt_sphere*>(base));
}

}  // extern "C"
