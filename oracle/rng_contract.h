/*
 * oracle/rng_contract.h -- TEST INFRASTRUCTURE (checker side). Never linked into
 * the product library.
 *
 * The reference draws every random number from glibc's single serial rand()
 * stream (vec3.c:64-69 via sphere.c:19-32, seeded at main.c:90). That stream
 * cannot be reproduced by a data-parallel renderer, because the number of draws
 * a pixel consumes is data dependent (rejection sampling in
 * random_in_unit_sphere, sphere.c:19-24). SURVEY.md §8.H5 therefore fixes a
 * per-pixel counter-based contract that replaces rand() on the render path:
 *
 *   key(seed, pixel, sample) = mix(seed ^ mix(((u64)sample << 32) | pixel))
 *   draw(key, k)             = mix(key + (k + 1) * 0x9E3779B97F4A7C15) >> 33
 *
 * where mix() is the splitmix64 finaliser, pixel = y*W + x of the full frame,
 * sample = frame/sample index and k counts the rand() calls made while tracing
 * that pixel (0, 1, 2, ...). draw() is a 31-bit value in [0, RAND_MAX], exactly
 * the range of glibc rand(). The product kernel implements the same contract
 * (cs201_sah-bvh_ray_tracer_amd/csrc/rng.h); golden vectors pin both.
 */
#ifndef ORACLE_RNG_CONTRACT_H
#define ORACLE_RNG_CONTRACT_H
#include <stdint.h>

static inline uint64_t oc_mix64(uint64_t z)
{
    z ^= z >> 30;
    z *= 0xBF58476D1CE4E5B9ULL;
    z ^= z >> 27;
    z *= 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return z;
}

static inline uint64_t oc_pixel_key(uint64_t seed, uint32_t pixel, uint32_t sample)
{
    return oc_mix64(seed ^ oc_mix64(((uint64_t)sample << 32) | (uint64_t)pixel));
}

static inline int oc_draw(uint64_t key, uint32_t k)
{
    return (int)(oc_mix64(key + (uint64_t)(k + 1u) * 0x9E3779B97F4A7C15ULL) >> 33);
}

/* Jittered frames (the build's definition; the reference has no jitter):
   pixel (x, y) samples at (x + jx, y + jy), j = (float)draw(key, OC_JITTER_*)
   / 2^31 in [0, 1), draws at indices the bounce sampling never reaches. */
#define OC_JITTER_X 0x7ffffff0u
#define OC_JITTER_Y 0x7ffffff1u

#endif
