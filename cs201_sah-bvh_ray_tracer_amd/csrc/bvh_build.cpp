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
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
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

struct FlatBuilder {
    mirt_sphere* s;
    std::vector<mirt_node> nodes;
    std::vector<int32_t> counts;  // sphere_count of leaves (bvh.c:134), 0 for inner nodes

    void emit_box(mirt_node& n, const Box& b)
    {
        for (int a = 0; a < 3; a++) {
            n.bmin[a] = b.lo[a];
            n.bmax[a] = b.hi[a];
        }
    }

    void build(int lo, int hi, int depth)
    {
        const int me = (int)nodes.size();
        nodes.push_back(mirt_node{});
        counts.push_back(0);
        Box bounds = box_empty();
        for (int i = lo; i < hi; i++) box_add(bounds, s[i]);
        emit_box(nodes[me], bounds);
        const int n = hi - lo;
        if (n <= 1 || depth >= 40) {  // bvh.c:131-137 (n == 0 leaves too)
            nodes[me].sphere = lo;
            nodes[me].skip = (uint32_t)(me + 1) | (n == 0 ? MIRT_NODE_EMPTY : 0u);
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
        build(lo, mid, depth + 1);
        build(mid, hi, depth + 1);
        nodes[me].sphere = -1;
        nodes[me].skip = (uint32_t)nodes.size();
    }
};

mirt_bvh_node* to_pointer_tree(const std::vector<mirt_node>& f, const std::vector<int32_t>& counts,
                               mirt_sphere* base, int& i)
{
    const int me = i++;
    mirt_bvh_node* n = (mirt_bvh_node*)std::malloc(sizeof(mirt_bvh_node));
    if (!n) return nullptr;
    n->bounds.min = {f[me].bmin[0], f[me].bmin[1], f[me].bmin[2]};
    n->bounds.max = {f[me].bmax[0], f[me].bmax[1], f[me].bmax[2]};
    if (f[me].sphere >= 0) {
        n->left = n->right = nullptr;
        n->sphere = base + f[me].sphere;
        n->sphere_count = counts[me];
    } else {
        n->left = to_pointer_tree(f, counts, base, i);
        n->right = to_pointer_tree(f, counts, base, i);
        n->sphere = nullptr;
        n->sphere_count = 0;
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

}  // namespace

extern "C" {

int mirt_bvh_build_flat(mirt_sphere* spheres, int start, int end, int depth, mirt_node** out_nodes,
                        int* out_count)
{
    if (!spheres || !out_nodes || !out_count || start < 0 || end < start) {
        mirt::set_error("mirt_bvh_build_flat: invalid arguments");
        return MIRT_E_INVALID;
    }
    FlatBuilder b{spheres, {}, {}};
    b.nodes.reserve((size_t)(end - start) * 3 + 1);
    b.build(start, end, depth);
    mirt_node* out = (mirt_node*)std::malloc(b.nodes.size() * sizeof(mirt_node));
    if (!out) {
        mirt::set_error("mirt_bvh_build_flat: out of host memory");
        return MIRT_E_NOMEM;
    }
    std::memcpy(out, b.nodes.data(), b.nodes.size() * sizeof(mirt_node));
    *out_nodes = out;
    *out_count = (int)b.nodes.size();
    return MIRT_OK;
}

void mirt_bvh_free_flat(mirt_node* nodes) { std::free(nodes); }

mirt_bvh_node* mirt_build_bvh_node(mirt_sphere* spheres, int start, int end, int depth)
{
    if (!spheres || start < 0 || end < start) {
        mirt::set_error("mirt_build_bvh_node: invalid arguments");
        return nullptr;
    }
    FlatBuilder b{spheres, {}, {}};
    b.build(start, end, depth);
    int i = 0;
    return to_pointer_tree(b.nodes, b.counts, spheres, i);
}

void mirt_free_bvh(mirt_bvh_node* node)  // benchmark.c:81-88
{
    if (!node) return;
    mirt_free_bvh(node->left);
    mirt_free_bvh(node->right);
    std::free(node);
}

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
