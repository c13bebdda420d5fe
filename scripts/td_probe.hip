// Vector-memory gather probe (not part of the library): the chip's peak rate
// of wave-level 16-B-per-lane loads (global_load_dwordx4) from an
// L2-resident table, as a function of how many distinct 64-B nodes one
// instruction touches -- the denominator of bench.py's `roofline` (the
// bounce walk's node, leaf and sphere loads are per-lane dwordx4 gathers over
// an L2-resident tree).
//   hipcc -O3 --offload-arch=gfx950 scripts/td_probe.hip -o scripts/td_probe
//   ./scripts/td_probe > profiles/r04_td_probe.json   (one JSON object)
//   ./scripts/td_probe --mix                          (the walk's access mix, below)
// Shapes:
//   lines L (1..64): L lanes of each wave active, each reading its own
//     64-B node as four dwordx4 (the bounce walk's HNode visit) -> L distinct
//     nodes per load instruction. The walk's waves run with a varying number
//     of active lanes (queue refill at 20, quad drain below 16), so its mean
//     distinct lines per instruction (TCP accesses / VMEM instructions in
//     the counter pass) selects the peak it is priced against.
//   shared G: all 64 lanes active, G lanes per node (quads, whole wave).
// Every case: 8 waves per SIMD (2048 workgroups x 256), 256 independent
// node visits per lane, timed after a warm-up launch; chip rate = wave-load
// instructions / s.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void __launch_bounds__(256) probe(const uint4* __restrict__ tab, uint32_t mask, int active, int group,
                                             int iters, uint32_t* __restrict__ out)
{
    const uint32_t lane = threadIdx.x & 63;
    if ((int)lane >= active) return;
    const uint32_t seed = blockIdx.x * 977u + (threadIdx.x / group) * 131u;
    uint32_t acc = 0;
    for (int i = 0; i < iters; i++) {
        const uint32_t node = ((seed + (uint32_t)i * 7919u) * 2654435761u >> 8) & mask;  // independent visits
        const uint4* p = tab + 4 * node;
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        // every word used, so each load stays one global_load_dwordx4
        acc += (a.x ^ a.y ^ a.z ^ a.w) + (b.x ^ b.y ^ b.z ^ b.w) + (c.x ^ c.y ^ c.z ^ c.w) + (d.x ^ d.y ^ d.z ^ d.w);
    }
    if (acc == 0x12345678u) out[0] = acc;   // keeps the loads; never true for the table's contents
}

// Round 5: the bounce walk's access MIX, to explain why
// its TD is 44% busy at 19% of the independent-gather peak. Each lane walks
// `iters` nodes; a visit is the same four dwordx4 as above, but
//   dep = 1: the next node index is computed from the loaded data (a chain of
//            dependent gathers, as a walk's next node comes from its node),
//   cold:   a fraction cold/256 of the visits go to a 256 MB table (L2 and
//            MALL misses, as the 13% of the kernel's requests that miss L2),
//   waves:  occupancy forced down by dynamic LDS (5 per SIMD as the kernel).
__global__ void __launch_bounds__(256) probe_mix(const uint4* __restrict__ hot, const uint4* __restrict__ cold,
                                                 uint32_t hot_mask, uint32_t cold_mask, int active, int dep,
                                                 uint32_t cold256, int valu, int ldsr, int narrow, int iters,
                                                 uint32_t* __restrict__ out)
{
    extern __shared__ uint4 pad[];
    const uint32_t lane = threadIdx.x & 63;
    if ((int)lane >= active) return;
    uint32_t x = blockIdx.x * 977u + threadIdx.x * 131u + 1u;
    uint32_t acc = 0;
    float f = (float)lane;
    const uint32_t* hot32 = reinterpret_cast<const uint32_t*>(hot);
    for (int i = 0; i < iters; i++) {
        const uint32_t h = (x + (uint32_t)i * 7919u) * 2654435761u;
        const bool is_cold = ((h >> 24) & 0xffu) < cold256;
        const uint4* p = is_cold ? cold + 4 * ((h >> 4) & cold_mask) : hot + 4 * ((h >> 8) & hot_mask);
        const uint4 a = p[0], b = p[1], c = p[2], d = p[3];
        uint32_t v = (a.x ^ a.y ^ a.z ^ a.w) + (b.x ^ b.y ^ b.z ^ b.w) + (c.x ^ c.y ^ c.z ^ c.w) +
                     (d.x ^ d.y ^ d.z ^ d.w);
        for (int k = 0; k < narrow; k++) v += hot32[(h >> (3 + k)) & (hot_mask * 16u + 15u)];   // dword gathers
        for (int k = 0; k < ldsr; k++) {   // LDS-resident node reads (the walk's top levels)
            const uint4 q = pad[(h >> (2 * k + 5)) & 1023u];
            acc += q.x ^ q.w;
        }
        for (int k = 0; k < valu; k++) f = __builtin_fmaf(f, 1.0001f, (float)(v + k));   // slab-test ALU work
        acc += v;
        if (dep) x ^= v;   // the next address depends on this node's data
    }
    if (acc == 0x12345678u || f == 1.2345f) out[0] = acc;
}

int mix_main()
{
    const uint32_t hot_nodes = 1u << 14, cold_nodes = 1u << 22;   // 1 MB / 256 MB
    uint4 *hot = nullptr, *cold = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&hot, sizeof(uint4) * 4 * hot_nodes) != hipSuccess ||
        hipMalloc(&cold, sizeof(uint4) * 4 * (size_t)cold_nodes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess)
        return 1;
    (void)hipMemset(hot, 0, sizeof(uint4) * 4 * hot_nodes);     // zero data: a dependent chain stays a hash walk
    (void)hipMemset(cold, 0, sizeof(uint4) * 4 * (size_t)cold_nodes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 0, clk_khz = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const int threads = 256;
    printf("{\"probe\": \"scripts/td_probe.hip --mix\", \"cus\": %d, \"clock_khz\": %d, \"cases\": [", cus, clk_khz);
    struct Case { int active, dep, cold256, waves, valu, ldsr, narrow, blocks = 2048, iters = 256; };
    const Case cases[] = {{20, 0, 0, 8, 0, 0, 0},  {20, 1, 0, 8, 0, 0, 0},  {20, 1, 0, 5, 0, 0, 0},
                          {20, 0, 33, 8, 0, 0, 0}, {20, 1, 33, 5, 0, 0, 0}, {20, 1, 33, 8, 0, 0, 0},
                          {64, 1, 0, 5, 0, 0, 0},  {64, 0, 0, 8, 0, 0, 0},
                          // round 5, session n: the walk's other work beside its gathers
                          {20, 1, 33, 5, 48, 0, 0}, {20, 1, 33, 5, 0, 4, 0}, {20, 1, 33, 5, 0, 0, 2},
                          {20, 1, 33, 5, 48, 4, 2}, {20, 0, 0, 8, 48, 0, 0}, {20, 0, 0, 5, 0, 4, 0},
                          // the bounce kernel's own mix per visit (counter pass of the 1080p/10k timed
                          // launch: 50.7 VALU and 1 LDS instruction per vector load) at its occupancy
                          // in one launch (384 workgroups of 256 = 1.5 waves per SIMD), then fuller
                          {20, 1, 33, 8, 200, 4, 0, 384, 1024}, {20, 1, 33, 8, 200, 4, 0, 768, 512},
                          {20, 1, 33, 5, 200, 4, 0, 2048, 256}, {20, 1, 33, 8, 200, 0, 0, 384, 1024}};
    bool first = true;
    for (const Case& c : cases) {
        // dynamic LDS sized so that only c.waves waves (workgroups / 4 x 4 SIMDs) fit a CU's 160 KB
        size_t lds = c.waves >= 8 ? 0 : (160 * 1024) / (size_t)c.waves - 256;
        if (c.ldsr && lds < 16384) lds = 16384;   // the reads' 1024 x 16 B
        const int blocks = c.blocks, iters = c.iters;
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            probe_mix<<<blocks, threads, lds>>>(hot, cold, hot_nodes - 1, cold_nodes - 1, c.active, c.dep, c.cold256,
                                                c.valu, c.ldsr, c.narrow, iters, out);
            (void)hipEventRecord(e0);
            probe_mix<<<blocks, threads, lds>>>(hot, cold, hot_nodes - 1, cold_nodes - 1, c.active, c.dep, c.cold256,
                                                c.valu, c.ldsr, c.narrow, iters, out);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double inst = (double)blocks * (threads / 64) * iters * (4 + c.narrow);
        printf("%s\n  {\"active_lanes\": %d, \"dependent\": %d, \"cold_frac\": %.3f, \"waves_per_simd\": %d, "
               "\"valu_fma_per_visit\": %d, \"lds_reads_per_visit\": %d, \"dword_loads_per_visit\": %d, "
               "\"workgroups\": %d, \"visits_per_lane\": %d, "
               "\"lds_bytes\": %zu, \"ms\": %.4f, \"wave_load_instructions\": %.0f, \"ginst_per_s\": %.3f}",
               first ? "" : ",", c.active, c.dep, c.cold256 / 256.0, c.waves, c.valu, c.ldsr, c.narrow, blocks, iters,
               lds, best, inst,
               inst / (best * 1e-3) / 1e9);
        first = false;
    }
    printf("\n]}\n");
    (void)hipFree(hot);
    (void)hipFree(cold);
    (void)hipFree(out);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc > 1 && argv[1][0] == '-' && argv[1][1] == '-' && argv[1][2] == 'm') return mix_main();
    const uint32_t nodes = 1u << 14;  // 16k x 64 B = 1 MB: L2-resident (the 10k scene's four-wide tree: 0.7 MB)
    uint4* tab = nullptr;
    uint32_t* out = nullptr;
    if (hipMalloc(&tab, sizeof(uint4) * 4 * nodes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
    (void)hipMemset(tab, 1, sizeof(uint4) * 4 * nodes);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    int cus = 0, clk_khz = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
    const int blocks = 2048, threads = 256, iters = 256;
    printf("{\"probe\": \"scripts/td_probe.hip\", \"cus\": %d, \"clock_khz\": %d, \"table_bytes\": %u, "
           "\"waves\": %d, \"visits_per_lane\": %d, \"loads_per_visit\": 4, \"cases\": [",
           cus, clk_khz, (unsigned)(64u * nodes), blocks * threads / 64, iters);
    const int lines[] = {64, 48, 32, 24, 20, 16, 12, 8, 4, 1};
    const int shared[] = {4, 16, 64};
    bool first = true;
    for (int k = 0; k < (int)(sizeof lines / sizeof lines[0]) + (int)(sizeof shared / sizeof shared[0]); k++) {
        const bool sh = k >= (int)(sizeof lines / sizeof lines[0]);
        const int active = sh ? 64 : lines[k];
        const int group = sh ? shared[k - sizeof lines / sizeof lines[0]] : 1;
        float best = 1e30f;
        for (int rep = 0; rep < 3; rep++) {
            probe<<<blocks, threads>>>(tab, nodes - 1, active, group, iters, out);   // warm
            (void)hipEventRecord(e0);
            probe<<<blocks, threads>>>(tab, nodes - 1, active, group, iters, out);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        const double inst = (double)blocks * (threads / 64) * iters * 4;   // wave-level load instructions
        const int distinct = sh ? 64 / group : active;
        printf("%s\n  {\"active_lanes\": %d, \"lanes_per_node\": %d, \"nodes_per_instruction\": %d, \"ms\": %.4f, "
               "\"wave_load_instructions\": %.0f, \"ginst_per_s\": %.3f, \"cycles_per_instruction_per_cu\": %.2f}",
               first ? "" : ",", active, group, distinct, best, inst, inst / (best * 1e-3) / 1e9,
               (best * 1e-3) * clk_khz * 1e3 * cus / inst);
        first = false;
    }
    printf("\n]}\n");
    (void)hipFree(tab);
    (void)hipFree(out);
    return 0;
}
