// Per-pixel counter-based RNG that replaces the reference's serial glibc
// rand() stream on the render path. Contract:
//
//   key(seed, pixel, sample) = mix(seed ^ mix((sample << 32) | pixel))
//   draw(key, k)             = mix(key + (k + 1) * 0x9E3779B97F4A7C15) >> 33
//
// mix = splitmix64 finaliser; pixel = y * W + x of the full frame (so a shard
// draws exactly what the full frame draws); k counts the rand() calls made
// while tracing that pixel. draw() is in [0, 2^31 - 1] = [0, RAND_MAX].
// tests/golden/golden.json "contract" pins the values.
#pragma once
#include <cstdint>

#if defined(__HIP__)
#include <hip/hip_runtime.h>
#define MIRT_HD __host__ __device__ __forceinline__
#else
#define MIRT_HD inline
#endif

namespace mirt {

MIRT_HD uint64_t mix64(uint64_t z)
{
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBull;
    z ^= z >> 31;
    return z;
}

MIRT_HD uint64_t pixel_key(uint64_t seed, uint32_t pixel, uint32_t sample)
{
    return mix64(seed ^ mix64(((uint64_t)sample << 32) | (uint64_t)pixel));
}

MIRT_HD int draw(uint64_t key, uint32_t k)
{
    return (int)(mix64(key + (uint64_t)(k + 1u) * 0x9E3779B97F4A7C15ull) >> 33);
}

// Jittered frames: the camera ray's sample point is (x + jx, y + jy) with
// j = (float)draw(key, kJitterDraw*) / 2^31 in [0, 1) -- draws at indices the
// bounce sampling (k = 0, 1, ...; a few dozen per pixel) never reaches.
constexpr uint32_t kJitterDrawX = 0x7ffffff0u, kJitterDrawY = 0x7ffffff1u;

}  // namespace mirt
