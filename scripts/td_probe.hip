// Texture-path probe (not part of the library): cost of per-lane 16-B loads
// from an L1/L2-resident table as a function of how many 64-B nodes the
// lanes of one wave touch per instruction -- the bounce walk's node loads
// are four dwordx4 per lane-visit.
//   hipcc -O3 --offload-arch=gfx950 scripts/td_probe.hip -o scripts/td_probe
//   ./td_probe   (prints ns per wave-instruction for each lane grouping)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

// group: lanes per node (1 = every lane its own node, 4 = a quad shares one
// node, each lane its own 16 B of it, 64 = the wave shares one node).
// words: 4 loads per lane-visit (the whole 64-B node per lane) when
// `whole`, else 1 (the lane's 16-B piece).
__global__ void probe(const uint4* __restrict__ tab, uint32_t mask, int group, int whole, int iters,
                      uint32_t* __restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t seed = blockIdx.x * 977u + (threadIdx.x / group) * 131u;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t node = ((seed + (uint32_t)i * 7919u) * 2654435761u >> 8) & mask;  // independent loads
        const uint4* p = tab + 4 * node;
        if (whole) {
            const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
            acc += a.x ^ b.y ^ c.z ^ d.w;
        } else {
            const uint4 a = p[lane & 3];
            acc += a.x ^ a.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main()
{
    const uint32_t nodes = 1u << 14;  // 1 MB: L2-resident
    uint4* tab;
    uint32_t* out;
    (void)hipMalloc(&tab, sizeof(uint4) * 4 * nodes);
    (void)hipMalloc(&out, 4);
    (void)hipMemset(tab, 1, sizeof(uint4) * 4 * nodes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int blocks = 256 * 8, threads = 256, iters = 256;
    for (int whole = 1; whole >= 0; whole--)
        for (int group : {1, 4, 16, 64}) {
            probe<<<blocks, threads>>>(tab, nodes - 1, group, whole, iters, out);
            (void)hipEventRecord(e0);
            probe<<<blocks, threads>>>(tab, nodes - 1, group, whole, iters, out);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double inst = (double)blocks * (threads / 64) * iters * (whole ? 4 : 1);
            printf("whole=%d lanes_per_node=%2d  %.3f ms  %.3f ns per wave-load-instruction (chip)\n", whole, group,
                   ms, ms * 1e6 / inst);
        }
    (void)hipFree(tab);
    (void)hipFree(out);
    return 0;
}
