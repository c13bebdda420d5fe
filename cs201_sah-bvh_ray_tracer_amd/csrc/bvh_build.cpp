// Host BVH construction, bit-identical to the reference's build_bvh_node
// (bvh.c:117-209), emitted straight into the flat layout the kernel walks
// (mirt_node, include/mirt.h), plus conversions to/from the reference's
// pointer tree (bvh.h:12-18).
//
// Bit-exactness argument (checked against tests/golden/ tree hashes):
//  * node bounds are fmin/fmax of sphere boxes (bvh.c:37-46): exact, so the
//    combine order is irrelevant;
//  * the 21 SAH candidates (bvh.c:143-170) are evaluated from 8 per-axis bins
//    instead of 21 passes (bvh.c:59-97). Plane i puts a sphere left iff its
//    centre < split_i, and split_1 <= ... <= split_7 (monotone float ops), so
//    a sphere is left of plane i iff its bin b (first plane it is left of) is
//    <= i. Bin boxes/counts are exact; the left/right boxes and counts of
//    every plane are therefore identical to the reference's, and the cost is
//    then evaluated with the reference's exact operation sequence;
//  * the in-place partition (bvh.c:172-201) is the reference's swap loop.
// No FMA contraction (-ffp-contract=off): bvh.c:54-56,96,150-158 are
// contraction-sensitive.
//
// Threads: after a node's partition its two children own disjoint ranges of
// the sphere array and their builds are independent, so above kParMin
// spheres (and up to kParDepth levels deep: at most 2^kParDepth tasks) both
// children are built concurrently by child builders. The parent keeps a
// marker node per child and counts the child's nodes in its own indices, so
// every skip is final relative to the builder's origin; emit() then writes
// the pre-order array once, each node copied once, skips offset by the
// builder's position. Every node is computed by the same sequence of
// operations as in one thread: the tree is the same bits.
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <future>
#include <memory>
#include <new>
#include <system_error>
#include <vector>

#include "internal.h"

namespace {

struct Box {
    float lo[3], hi[3];
};

inline Box box_empty()  // bvh.c:19-24
{
    Box b;
    for (int a = 0; a < 3; a++) {
        b.lo[a] = INFINITY;
        b.hi[a] = -INFINITY;
    }
    return b;
}

inline void box_add(Box& b, const mirt_sphere& s)  // bvh.c:26-46
{
    const float c[3] = {s.center.x, s.center.y, s.center.z};
    for (int a = 0; a < 3; a++) {
        b.lo[a] = std::fmin(b.lo[a], c[a] - s.radius);
        b.hi[a] = std::fmax(b.hi[a], c[a] + s.radius);
    }
}

inline void box_merge(Box& b, const Box& o)
{
    for (int a = 0; a < 3; a++) {
        b.lo[a] = std::fmin(b.lo[a], o.lo[a]);
        b.hi[a] = std::fmax(b.hi[a], o.hi[a]);
    }
}

inline float box_area(const Box& b)  // bvh.c:48-57
{
    const float dx = b.hi[0] - b.lo[0], dy = b.hi[1] - b.lo[1], dz = b.hi[2] - b.lo[2];
    float s = dx * dy;
    s = s + dy * dz;
    s = s + dz * dx;
    return 2.0f * s;
}

inline float centre(const mirt_sphere& s, int axis)
{
    return axis == 0 ? s.center.x : (axis == 1 ? s.center.y : s.center.z);
}

constexpr int kParMin = 32768;  // spheres below which a subtree is built on one thread
constexpr int kParDepth = 4;    // levels that may fork (<= 16 concurrent builds)

// MIRT_BVH_FORK_LEVELS overrides kParDepth (0 = one thread)
int fork_levels()
{
    const char* e = std::getenv("MIRT_BVH_FORK_LEVELS");
    return e ? std::atoi(e) : kParDepth;
}

struct FlatBuilder {
    mirt_sphere* s;
    std::vector<mirt_node> nodes;  // own nodes, plus one marker (sphere = -2 - k) per child builder k
    std::vector<int32_t> counts;   // sphere_count of leaves (bvh.c:134), 0 for inner nodes
    int par = 0;                   // fork levels left
    uint32_t total = 0;            // nodes of the finished subtree (children's included)
    std::vector<std::unique_ptr<FlatBuilder>> kids;

    // the pre-order array of this subtree at out[base..base + total)
    void emit(mirt_node* out, int32_t* cnt, uint32_t base) const
    {
        uint32_t pos = base;
        for (size_t i = 0; i < nodes.size(); i++) {
            const mirt_node& n = nodes[i];
            if (n.sphere <= -2) {
                const FlatBuilder& k = *kids[(size_t)(-2 - n.sphere)];
                k.emit(out, cnt, pos);
                pos += k.total;
                continue;
            }
            mirt_node o = n;
            o.skip = ((n.skip & ~MIRT_NODE_EMPTY) + base) | (n.skip & MIRT_NODE_EMPTY);
            out[pos] = o;
            if (cnt) cnt[pos] = counts[i];
            pos++;
        }
    }

    std::vector<mirt_node> flat(std::vector<int32_t>* cnt) const
    {
        std::vector<mirt_node> out(total);
        if (cnt) cnt->assign(total, 0);
        emit(out.data(), cnt ? cnt->data() : nullptr, 0);
        return out;
    }

    void run(int lo, int hi, int depth)
    {
        build(lo, hi, depth);
        total = cur;
    }

    uint32_t cur = 0;  // final-array index (relative to this builder) of the next node

    void emit_box(mirt_node& n, const Box& b)
    {
        for (int a = 0; a < 3; a++) {
            n.bmin[a] = b.lo[a];
            n.bmax[a] = b.hi[a];
        }
    }

    void build(int lo, int hi, int depth)
    {
        const int me = (int)nodes.size();  // slot in `nodes`
        const uint32_t at = cur++;         // index in the final array (relative)
        nodes.push_back(mirt_node{});
        counts.push_back(0);
        Box bounds = box_empty();
        for (int i = lo; i < hi; i++) box_add(bounds, s[i]);
        emit_box(nodes[me], bounds);
        const int n = hi - lo;
        if (n <= 1 || depth >= 40) {  // bvh.c:131-137 (n == 0 leaves too)
            nodes[me].sphere = lo;
            nodes[me].skip = (at + 1) | (n == 0 ? MIRT_NODE_EMPTY : 0u);
            counts[me] = n;
            return;
        }

        float best_cost = INFINITY, best_split = 0.0f;  // bvh.c:139-141
        int best_axis = 0;
        for (int axis = 0; axis < 3; axis++) {
            float split[8];
            for (int i = 1; i < 8; i++)  // bvh.c:150/154/158
                split[i] = bounds.lo[axis] + ((float)i / 8.0f) * (bounds.hi[axis] - bounds.lo[axis]);
            Box bin_box[9];
            int bin_n[9] = {0};
            for (int k = 1; k <= 8; k++) bin_box[k] = box_empty();
            for (int i = lo; i < hi; i++) {
                const float c = centre(s[i], axis);
                int b = 1;
                while (b < 8 && !(c < split[b])) b++;  // first plane this sphere is left of (8: none)
                bin_n[b]++;
                box_add(bin_box[b], s[i]);
            }
            // prefix (left of plane i = bins 1..i) and suffix (right = bins i+1..8)
            Box left[8], right[9];
            int nl[8], nr[9];
            Box acc = box_empty();
            int cnt = 0;
            for (int i = 1; i < 8; i++) {
                box_merge(acc, bin_box[i]);
                cnt += bin_n[i];
                left[i] = acc;
                nl[i] = cnt;
            }
            acc = box_empty();
            cnt = 0;
            for (int i = 8; i >= 2; i--) {
                box_merge(acc, bin_box[i]);
                cnt += bin_n[i];
                right[i - 1] = acc;
                nr[i - 1] = cnt;
            }
            for (int i = 1; i < 8; i++) {
                const float la = box_area(left[i]), ra = box_area(right[i]);
                float sum = (float)nl[i] * la;  // bvh.c:96
                sum = sum + (float)nr[i] * ra;
                const float cost = 0.125f + sum;
                if (cost < best_cost) {
                    best_cost = cost;
                    best_axis = axis;
                    best_split = split[i];
                }
            }
        }

        int mid = lo;  // bvh.c:172-201
        for (int i = lo; i < hi; i++) {
            if (centre(s[i], best_axis) < best_split) {
                const mirt_sphere t = s[i];
                s[i] = s[mid];
                s[mid] = t;
                mid++;
            }
        }
        if (par > 0 && n >= kParMin) {
            auto l = std::make_unique<FlatBuilder>(), r = std::make_unique<FlatBuilder>();
            l->s = r->s = s;
            l->par = r->par = par - 1;
            FlatBuilder *lp = l.get(), *rp = r.get();
            std::future<void> fl;
            try {
                fl = std::async(std::launch::async, [=] { lp->run(lo, mid, depth + 1); });
            } catch (const std::system_error&) {  // no thread to be had: build it here, same bits
                lp->run(lo, mid, depth + 1);
            }
            rp->run(mid, hi, depth + 1);
            if (fl.valid()) fl.get();
            for (auto* k : {&l, &r}) {
                mirt_node mk{};
                mk.sphere = -2 - (int32_t)kids.size();
                cur += (*k)->total;
                kids.push_back(std::move(*k));
                nodes.push_back(mk);
                counts.push_back(0);
            }
        } else {
            build(lo, mid, depth + 1);
            build(mid, hi, depth + 1);
        }
        nodes[me].sphere = -1;
        nodes[me].skip = cur;
    }
};

void free_tree(mirt_bvh_node* node)  // benchmark.c:81-88
{
    if (!node) return;
    free_tree(node->left);
    free_tree(node->right);
    std::free(node);
}

// nullptr if a malloc failed (every node allocated so far is freed)
mirt_bvh_node* to_pointer_tree(const std::vector<mirt_node>& f, const std::vector<int32_t>& counts,
                               mirt_sphere* base, int& i)
{
    const int me = i++;
    mirt_bvh_node* n = (mirt_bvh_node*)std::malloc(sizeof(mirt_bvh_node));
    if (!n) return nullptr;
    n->bounds.min = {f[me].bmin[0], f[me].bmin[1], f[me].bmin[2]};
    n->bounds.max = {f[me].bmax[0], f[me].bmax[1], f[me].bmax[2]};
    n->left = n->right = nullptr;
    n->sphere = nullptr;
    n->sphere_count = 0;
    if (f[me].sphere >= 0) {
        n->sphere = base + f[me].sphere;
        n->sphere_count = counts[me];
    } else {
        n->left = to_pointer_tree(f, counts, base, i);
        n->right = n->left ? to_pointer_tree(f, counts, base, i) : nullptr;
        if (!n->right) {
            free_tree(n);
            return nullptr;
        }
    }
    return n;
}

int count_tree(const mirt_bvh_node* n) { return n ? 1 + count_tree(n->left) + count_tree(n->right) : 0; }

int flatten_rec(const mirt_bvh_node* n, const mirt_sphere* base, mirt_node* out, int at)
{
    const int me = at++;
    out[me].bmin[0] = n->bounds.min.x;
    out[me].bmin[1] = n->bounds.min.y;
    out[me].bmin[2] = n->bounds.min.z;
    out[me].bmax[0] = n->bounds.max.x;
    out[me].bmax[1] = n->bounds.max.y;
    out[me].bmax[2] = n->bounds.max.z;
    if (n->sphere) {
        out[me].sphere = (int32_t)(n->sphere - base);
    } else {
        out[me].sphere = -1;
        at = flatten_rec(n->left, base, out, at);
        at = flatten_rec(n->right, base, out, at);
    }
    const bool empty = n->sphere && n->sphere_count == 0;
    out[me].skip = (uint32_t)at | (empty ? MIRT_NODE_EMPTY : 0u);
    return at;
}

int set_nomem(const char* fn)
{
    mirt::set_error("%s: out of host memory", fn);
    return MIRT_E_NOMEM;
}

}  // namespace

namespace mirt {

int validate_flat(const mirt_node* nd, int nn, int num_spheres, int sphere_lo, const char* fn)
{
    if (nn < 0 || (nn > 0 && !nd)) {
        set_error("%s: invalid node array", fn);
        return MIRT_E_INVALID;
    }
    if (nn == 0) return MIRT_OK;
    if ((nd[0].skip & MIRT_SKIP_MASK) != (uint32_t)nn) {
        set_error("%s: root skip %u != node count %d", fn, nd[0].skip & MIRT_SKIP_MASK, nn);
        return MIRT_E_INVALID;
    }
    for (int i = 0; i < nn; i++) {
        const uint32_t skip = nd[i].skip & MIRT_SKIP_MASK;
        const bool leaf = nd[i].sphere >= 0;
        const bool empty = (nd[i].skip & MIRT_NODE_EMPTY) != 0;
        bool ok = skip > (uint32_t)i && skip <= (uint32_t)nn && nd[i].sphere >= -1 && nd[i].sphere <= num_spheres &&
                  (!leaf || nd[i].sphere >= sphere_lo) && (!empty || leaf);
        if (ok && leaf) {
            ok = skip == (uint32_t)i + 1;
        } else if (ok) {
            // inner: left child i+1, right child r = the left subtree's end;
            // both subtrees nest exactly inside (i, skip)
            const uint32_t r = (uint32_t)i + 1 < skip ? nd[i + 1].skip & MIRT_SKIP_MASK : 0u;
            ok = (uint32_t)i + 1 < skip && r > (uint32_t)i + 1 && r < skip && (nd[r].skip & MIRT_SKIP_MASK) == skip;
        }
        if (!ok) {
            set_error("%s: malformed node %d (sphere %d, skip %u)", fn, i, nd[i].sphere, skip);
            return MIRT_E_INVALID;
        }
    }
    return MIRT_OK;
}

}  // namespace mirt

extern "C" {

int mirt_bvh_validate_flat(const mirt_node* nodes, int num_nodes, int num_spheres)
{
    return mirt::validate_flat(nodes, num_nodes, num_spheres, 0, "mirt_bvh_validate_flat");
}

int mirt_bvh_build_flat(mirt_sphere* spheres, int start, int end, int depth, mirt_node** out_nodes,
                        int* out_count)
try {
    if (!spheres || !out_nodes || !out_count || start < 0 || end < start) {
        mirt::set_error("mirt_bvh_build_flat: invalid arguments");
        return MIRT_E_INVALID;
    }
    FlatBuilder b;
    b.s = spheres;
    b.par = fork_levels();
    b.run(start, end, depth);
    mirt_node* out = (mirt_node*)std::malloc((size_t)b.total * sizeof(mirt_node));
    if (!out) {
        mirt::set_error("mirt_bvh_build_flat: out of host memory");
        return MIRT_E_NOMEM;
    }
    b.emit(out, nullptr, 0);
    *out_nodes = out;
    *out_count = (int)b.total;
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    return set_nomem("mirt_bvh_build_flat");
}

void mirt_bvh_free_flat(mirt_node* nodes) { std::free(nodes); }

mirt_bvh_node* mirt_build_bvh_node(mirt_sphere* spheres, int start, int end, int depth)
try {
    if (!spheres || start < 0 || end < start) {
        mirt::set_error("mirt_build_bvh_node: invalid arguments");
        return nullptr;
    }
    FlatBuilder b;
    b.s = spheres;
    b.par = fork_levels();
    b.run(start, end, depth);
    std::vector<int32_t> counts;
    const std::vector<mirt_node> flat = b.flat(&counts);
    int i = 0;
    mirt_bvh_node* root = to_pointer_tree(flat, counts, spheres, i);
    if (!root) set_nomem("mirt_build_bvh_node");
    return root;
} catch (const std::bad_alloc&) {
    set_nomem("mirt_build_bvh_node");
    return nullptr;
}

void mirt_free_bvh(mirt_bvh_node* node) { free_tree(node); }

int mirt_bvh_count(const mirt_bvh_node* root) { return count_tree(root); }

int mirt_bvh_flatten(const mirt_bvh_node* root, const mirt_sphere* base, mirt_node* out, int cap)
{
    if (!root || !base) {
        mirt::set_error("mirt_bvh_flatten: null tree or sphere base");
        return MIRT_E_INVALID;
    }
    const int n = count_tree(root);
    if (!out || n > cap) return -n;
    return flatten_rec(root, base, out, 0);
}

}  // extern "C"
