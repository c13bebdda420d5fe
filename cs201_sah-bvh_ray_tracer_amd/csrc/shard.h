// Row-block shard geometry of a frame (mirt_frame_desc row_block / shard /
// num_shards / lead_skip), shared by the host code and the kernels.
//
// The image's rows are cut into blocks of row_block rows. With lead_skip d = 0
// block b belongs to shard b % n (interleaved: the dense middle of the image
// is spread over every shard). With d > 0 the blocks are dealt in periods of
// kLeadRounds rounds: a round gives one block to every shard in order
// 0, 1, .., n - 1, except that shard 0 sits out the first d rounds of each
// period, so a period is P = kLeadRounds * n - d blocks and shard 0 gets
// kLeadRounds - d of them, every other shard kLeadRounds. That is the gather's
// balance: rank 0 also receives, de-interleaves and delivers the frame, so it
// renders fewer rows (mirt_multi's MIRT_MULTI_OPT_LEAD_SKIP). d = 0 is exactly
// b % n. A shard's blocks are compacted in image order into its slab.
#pragma once
#include "rng.h"   // MIRT_HD

namespace mirt {

constexpr int kLeadRounds = 8;

// Blocks of shard s in one period, and the period's length in blocks.
MIRT_HD int shard_period_blocks(int s, int d) { return kLeadRounds - (s == 0 ? d : 0); }
MIRT_HD int shard_period(int n, int d) { return kLeadRounds * n - d; }

// Position inside a period of shard s's k-th block of that period.
MIRT_HD int shard_block_pos(int s, int k, int n, int d)
{
    const int j = s == 0 ? k + d : k;   // the round
    return j < d ? j * (n - 1) + (s - 1) : d * (n - 1) + (j - d) * n + s;
}

// Image block of shard s's compact block c.
MIRT_HD int shard_block(int s, int c, int n, int d)
{
    if (d == 0) return c * n + s;
    const int w = shard_period_blocks(s, d);
    return (c / w) * shard_period(n, d) + shard_block_pos(s, c % w, n, d);
}

// Owner shard of image block b and the block's compact index in that shard.
MIRT_HD void block_owner(int b, int n, int d, int& s, int& c)
{
    if (d == 0) {
        s = b % n;
        c = b / n;
        return;
    }
    const int P = shard_period(n, d), per = b / P, p = b - per * P;
    int j;
    if (p < d * (n - 1)) {
        j = p / (n - 1);
        s = 1 + p % (n - 1);
    } else {
        const int q = p - d * (n - 1);
        j = d + q / n;
        s = q % n;
    }
    c = per * shard_period_blocks(s, d) + (s == 0 ? j - d : j);
}

// Blocks of shard s among the first nb blocks of the image.
MIRT_HD int shard_block_count(int s, int nb, int n, int d)
{
    if (d == 0) return s < nb ? (nb - 1 - s) / n + 1 : 0;
    const int P = shard_period(n, d), w = shard_period_blocks(s, d);
    const int full = nb / P, rest = nb - full * P;
    int c = full * w;
    for (int k = 0; k < w && shard_block_pos(s, k, n, d) < rest; k++) c++;
    return c;
}

}  // namespace mirt
