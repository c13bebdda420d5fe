// Why trace.h normalize3 keeps the binary64 square root: over all 2^32
// binary32 bit patterns, the binary32 spellings of sqrt (__fsqrt_rn, sqrtf,
// __builtin_sqrtf) against the binary64 root rounded to binary32 (vec3.c:22's
// (float)sqrt((double)x), which equals the correctly rounded binary32 root),
// compiled with the product's flags. Prints the mismatch count of each
// binary32 spelling and up to 8 mismatching inputs; exit status 0 iff the
// spelling named by argv[1] has none.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

// hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 scripts/sqrt_exhaustive.hip -o scripts/sqrt_exhaustive

// VARIANT 0: __fsqrt_rn, 1: sqrtf, 2: __builtin_sqrtf
template <int VARIANT>
__device__ __forceinline__ float sqrt32(float x)
{
    if constexpr (VARIANT == 0) return __fsqrt_rn(x);
    else if constexpr (VARIANT == 1) return sqrtf(x);
    else return __builtin_sqrtf(x);
}

template <int VARIANT>
__global__ void check(unsigned long long* bad, uint32_t* first)
{
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
        const float x = __uint_as_float((uint32_t)i);
        const float a = sqrt32<VARIANT>(x);
        const float b = (float)__dsqrt_rn((double)x);
        const bool same = (a != a && b != b) || __float_as_uint(a) == __float_as_uint(b);
        if (!same) {
            // [0]: all, [1]: subnormal inputs
            const unsigned long long k = atomicAdd(&bad[0], 1ull);
            if ((((uint32_t)i >> 23) & 0xff) == 0) atomicAdd(&bad[1], 1ull);
            if (k < 8) first[k] = (uint32_t)i;
        }
    }
}

int main(int argc, char** argv)
{
    // argv[1]: the variant the product uses (default 0); every variant is
    // reported, the exit status is that one's
    const int want = argc > 1 ? argv[1][0] - '0' : 0;
    unsigned long long* d_bad = nullptr;
    uint32_t* d_first = nullptr;
    if (hipMalloc(&d_bad, 2 * sizeof(unsigned long long)) != hipSuccess ||
        hipMalloc(&d_first, 8 * sizeof(uint32_t)) != hipSuccess)
        return 2;
    int rc = 0;
    for (int v = 0; v < 3; v++) {
        (void)hipMemset(d_bad, 0, 2 * sizeof(unsigned long long));
        (void)hipMemset(d_first, 0, 8 * sizeof(uint32_t));
        if (v == 0) check<0><<<4096, 256>>>(d_bad, d_first);
        if (v == 1) check<1><<<4096, 256>>>(d_bad, d_first);
        if (v == 2) check<2><<<4096, 256>>>(d_bad, d_first);
        unsigned long long bad[2] = {0, 0};
        uint32_t first[8] = {0};
        if (hipMemcpy(bad, d_bad, sizeof(bad), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(first, d_first, sizeof(first), hipMemcpyDeviceToHost) != hipSuccess)
            return 2;
        printf("variant %d mismatches %llu (subnormal inputs %llu)", v, bad[0], bad[1]);
        for (unsigned long long k = 0; k < bad[0] && k < 8; k++) printf(" 0x%08x", first[k]);
        printf("\n");
        if (v == want && bad[0]) rc = 1;
    }
    (void)hipFree(d_bad);
    (void)hipFree(d_first);
    return rc;
}
