// Flattened-tree cache file: the host build of
// build_bvh_node (bvh.c:117-209) reorders the sphere array in place and is
// the only O(n log n) host step before a frame (S_bench(1M): 19.5 s in the
// reference, ~1 s in bvh_build.cpp). A rerun on the same spheres can load the
// result instead: the reordered spheres and the pre-order mirt_node array.
//
// File layout (little-endian, native struct layout — the file is a cache,
// not an interchange format):
//   char     magic[8]     "MIRTBVH1"
//   uint32_t sphere_size  sizeof(mirt_sphere) = 20
//   uint32_t node_size    sizeof(mirt_node)   = 32
//   int32_t  start, end, depth, num_nodes      the build_bvh_node arguments
//   uint64_t key          FNV-1a 64 (word-wise, Fnv below) over the INPUT
//                         spheres[start,end) bytes, then start, end, depth
//   uint64_t payload      the same hash over the stored spheres and nodes
//   mirt_sphere[end-start]  spheres[start,end) as the build left them
//   mirt_node[num_nodes]
// A file whose header, key or payload hash does not match, whose tree is not
// well formed (mirt_bvh_validate_flat) or whose spheres are not a permutation
// of the input is ignored and rewritten; writes go to "<path>.tmp.<pid>" and are renamed into place, so a
// reader never sees a half-written file.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include <unistd.h>

#include "internal.h"

namespace {

constexpr char kMagic[8] = {'M', 'I', 'R', 'T', 'B', 'V', 'H', '1'};

struct Header {
    char magic[8];
    uint32_t sphere_size, node_size;
    int32_t start, end, depth, num_nodes;
    uint64_t key, payload;
};
static_assert(sizeof(Header) == 48, "cache header layout");

// FNV-1a 64 taken over 64-bit words (then the tail bytes): one multiply per
// 8 bytes, so hashing the 1M-sphere file (215 MB) costs ~30 ms, not the
// ~0.3 s of the byte-wise form.
struct Fnv {
    uint64_t h = 1469598103934665603ull;
    void add(const void* p, size_t n)
    {
        const unsigned char* b = (const unsigned char*)p;
        size_t i = 0;
        for (; i + 8 <= n; i += 8) {
            uint64_t w;
            std::memcpy(&w, b + i, 8);
            h = (h ^ w) * 1099511628211ull;
        }
        for (; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    }
};

uint64_t input_key(const mirt_sphere* s, int start, int end, int depth)
{
    Fnv f;
    f.add(s + start, (size_t)(end - start) * sizeof(mirt_sphere));
    f.add(&start, sizeof start);
    f.add(&end, sizeof end);
    f.add(&depth, sizeof depth);
    return f.h;
}

// Order-independent hash of a sphere array (sum of a 64-bit mix of each
// record): equal for a permutation, so a cached array must hold exactly the
// input's spheres.
uint64_t multiset_hash(const mirt_sphere* s, size_t n)
{
    uint64_t sum = 0;
    for (size_t i = 0; i < n; i++) {
        Fnv f;
        f.add(s + i, sizeof(mirt_sphere));
        uint64_t z = f.h + 0x9e3779b97f4a7c15ull;  // splitmix64 finaliser
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        sum += z ^ (z >> 31);
    }
    return sum;
}

// Loads the file into `sph` (end-start spheres) and a malloc'd node array if
// it is a valid cache entry for `key`; returns false otherwise, touching
// nothing the caller owns.
bool try_load(const char* path, const mirt_sphere* input, uint64_t key, int start, int end, int depth,
              std::vector<mirt_sphere>& sph, mirt_node** nodes, int* count)
{
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    Header h;
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, kMagic, 8) == 0 &&
              h.sphere_size == sizeof(mirt_sphere) && h.node_size == sizeof(mirt_node) && h.key == key &&
              h.start == start && h.end == end && h.depth == depth && h.num_nodes > 0;
    mirt_node* nd = nullptr;
    if (ok) {
        sph.resize((size_t)(end - start));
        nd = (mirt_node*)std::malloc((size_t)h.num_nodes * sizeof(mirt_node));
        ok = nd && std::fread(sph.data(), sizeof(mirt_sphere), sph.size(), f) == sph.size() &&
             std::fread(nd, sizeof(mirt_node), (size_t)h.num_nodes, f) == (size_t)h.num_nodes &&
             std::fgetc(f) == EOF;
    }
    std::fclose(f);
    if (ok) {
        Fnv p;
        p.add(sph.data(), sph.size() * sizeof(mirt_sphere));
        p.add(nd, (size_t)h.num_nodes * sizeof(mirt_node));
        ok = p.h == h.payload;
    }
    // the payload hash has no secret: also require a tree the uploads accept
    // (leaves index spheres[start, end]) over a permutation of the input
    ok = ok && mirt::validate_flat(nd, h.num_nodes, end, start, "cache") == MIRT_OK &&
         multiset_hash(sph.data(), sph.size()) == multiset_hash(input + start, (size_t)(end - start));
    if (!ok) {
        std::free(nd);
        return false;
    }
    *nodes = nd;
    *count = h.num_nodes;
    return true;
}

bool save(const char* path, uint64_t key, int start, int end, int depth, const mirt_sphere* sph,
          const mirt_node* nodes, int num_nodes)
{
    Header h;
    std::memcpy(h.magic, kMagic, 8);
    h.sphere_size = sizeof(mirt_sphere);
    h.node_size = sizeof(mirt_node);
    h.start = start;
    h.end = end;
    h.depth = depth;
    h.num_nodes = num_nodes;
    h.key = key;
    Fnv p;
    p.add(sph, (size_t)(end - start) * sizeof(mirt_sphere));
    p.add(nodes, (size_t)num_nodes * sizeof(mirt_node));
    h.payload = p.h;

    const std::string tmp = std::string(path) + ".tmp." + std::to_string((long)getpid());
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) {
        mirt::set_error("mirt_bvh_build_flat_cached: cannot write %s", tmp.c_str());
        return false;
    }
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 &&
              std::fwrite(sph, sizeof(mirt_sphere), (size_t)(end - start), f) == (size_t)(end - start) &&
              std::fwrite(nodes, sizeof(mirt_node), (size_t)num_nodes, f) == (size_t)num_nodes;
    ok = (std::fclose(f) == 0) && ok;
    if (ok && std::rename(tmp.c_str(), path) == 0) return true;
    std::remove(tmp.c_str());
    mirt::set_error("mirt_bvh_build_flat_cached: cannot write %s", path);
    return false;
}

}  // namespace

extern "C" {

int mirt_bvh_build_flat_cached(const char* path, mirt_sphere* spheres, int start, int end, int depth,
                               mirt_node** out_nodes, int* out_count, int* out_cached)
try {
    if (!path || !spheres || !out_nodes || !out_count || start < 0 || end < start) {
        mirt::set_error("mirt_bvh_build_flat_cached: invalid arguments");
        return MIRT_E_INVALID;
    }
    const uint64_t key = input_key(spheres, start, end, depth);
    std::vector<mirt_sphere> sph;
    if (try_load(path, spheres, key, start, end, depth, sph, out_nodes, out_count)) {
        std::memcpy(spheres + start, sph.data(), sph.size() * sizeof(mirt_sphere));
        if (out_cached) *out_cached = 1;
        return MIRT_OK;
    }
    const int rc = mirt_bvh_build_flat(spheres, start, end, depth, out_nodes, out_count);
    if (rc != MIRT_OK) return rc;
    const bool saved = save(path, key, start, end, depth, spheres + start, *out_nodes, *out_count);
    if (out_cached) *out_cached = saved ? 0 : -1;
    return MIRT_OK;
} catch (const std::bad_alloc&) {
    mirt::set_error("mirt_bvh_build_flat_cached: out of host memory");
    return MIRT_E_NOMEM;
}

}  // extern "C"
