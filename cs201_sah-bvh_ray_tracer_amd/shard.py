"""Row-block sharding of one frame across ranks: the geometry mirt_multi uses
(include/mirt_multi.h, csrc/multi.hip), restated for host-side code and
tests.

A frame's rows are cut into blocks of `row_block` rows; block b belongs to
rank b % world (interleaved, so the expensive dense middle of the image is
spread over all ranks), or with the lead-skip weighting (csrc/shard.h) rank 0
sits out `lead_skip` of every 8 rounds of that dealing. Each rank renders its blocks, compacted in row order,
into a slab of shard_row_count(...) rows (shard 0 has the most rows). The
frame is then assembled either on rank 0 from the gathered slabs
(multi.hip's deinterleave_kernel) or by every rank writing its blocks into
the host frame directly (multi.hip's strided copies). Pixels do not depend on
the sharding (the RNG contract keys on the full-frame pixel index), so any
world size produces the same bytes as one GPU.
"""
import numpy as np

LEAD_ROUNDS = 8   # csrc/shard.h kLeadRounds


def _period(world, lead_skip):
    return LEAD_ROUNDS * world - lead_skip


def _period_blocks(s, lead_skip):
    return LEAD_ROUNDS - (lead_skip if s == 0 else 0)


def _block_pos(s, k, world, d):
    j = k + d if s == 0 else k
    return j * (world - 1) + (s - 1) if j < d else d * (world - 1) + (j - d) * world + s


def shard_block(s, c, world, lead_skip=0):
    """Image block of shard s's compact block c (csrc/shard.h shard_block)."""
    if lead_skip == 0:
        return c * world + s
    w = _period_blocks(s, lead_skip)
    return (c // w) * _period(world, lead_skip) + _block_pos(s, c % w, world, lead_skip)


def block_owner(b, world, lead_skip=0):
    """(shard, compact block) of image block b (csrc/shard.h block_owner)."""
    d = lead_skip
    if d == 0:
        return b % world, b // world
    P = _period(world, d)
    per, p = divmod(b, P)
    if p < d * (world - 1):
        j, s = p // (world - 1), 1 + p % (world - 1)
    else:
        q = p - d * (world - 1)
        j, s = d + q // world, q % world
    return s, per * _period_blocks(s, d) + (j - d if s == 0 else j)


def shard_rows_of(height, row_block, world, shard, lead_skip=0):
    """Image rows of a shard in its slab's (compact) order."""
    blocks = (height + row_block - 1) // row_block
    rows = []
    for b in range(blocks):
        if block_owner(b, world, lead_skip)[0] == shard:
            rows.extend(range(b * row_block, min((b + 1) * row_block, height)))
    return np.array(rows, dtype=np.int64)


def shard_row_count(height, row_block, world, shard, lead_skip=0):
    """Rows of shard `shard` (matches shard_row_count in csrc/host_scene.cpp)."""
    return len(shard_rows_of(height, row_block, world, shard, lead_skip))


def slab_rows(height, row_block, world, lead_skip=0):
    """Padded slab height: the largest shard's rows (shard 0 without weighting)."""
    return max(shard_row_count(height, row_block, world, s, lead_skip) for s in range(world))


def row_sources(height, row_block, world, lead_skip=0):
    """For every image row y: (shard, row inside that shard's slab)."""
    y = np.arange(height)
    src, pos = np.empty(height, np.int64), np.empty(height, np.int64)
    for i in range(height):
        s, c = block_owner(y[i] // row_block, world, lead_skip)
        src[i], pos[i] = s, c * row_block + y[i] % row_block
    return src, pos


def assemble_gather(slabs, height, row_block, lead_skip=0):
    """multi.hip deinterleave_kernel, restated: slabs[s] is shard s's
    (frames, rows_s, W, ...) array (the gathered displays) -> (frames,
    height, W, ...)."""
    world = len(slabs)
    src, pos = row_sources(height, row_block, world, lead_skip)
    frames = slabs[0].shape[0]
    out = np.empty((frames, height) + slabs[0].shape[2:], slabs[0].dtype)
    for y in range(height):
        out[:, y] = slabs[src[y]][:, pos[y]]
    return out


def assemble_direct(slabs, height, row_block, lead_skip=0):
    """multi.hip's host-direct delivery, restated: shard s writes its full
    blocks as strided copies -- one (destination pitch world * row_block
    rows) without weighting, one per position of a period with it -- and
    the image's short last block, if it is s's, after them -> (frames,
    height, W)."""
    world = len(slabs)
    frames = slabs[0].shape[0]
    out = np.zeros((frames, height) + slabs[0].shape[2:], slabs[0].dtype)
    width = int(np.prod(slabs[0].shape[2:]))     # elements per image row (pixels x channels)
    blocks = (height + row_block - 1) // row_block
    last = blocks - 1
    last_full = last - 1 if height % row_block else last
    flat = out.reshape(frames, -1)
    seg = row_block * width
    for s in range(world):
        src = slabs[s].reshape(frames, -1)
        if lead_skip == 0:
            copies = [(s, world, 0, 1)]          # (first block, block pitch, first compact block, compact pitch)
        else:
            w = _period_blocks(s, lead_skip)
            copies = [(_block_pos(s, k, world, lead_skip), _period(world, lead_skip), k, w) for k in range(w)]
        for b0, bp, c0, cp in copies:
            cnt = (last_full - b0) // bp + 1 if last_full >= b0 else 0
            for i in range(cnt):    # the 2D copy: row i of the copy -> dst + i * pitch
                d0, s0 = (b0 + i * bp) * seg, (c0 + i * cp) * seg
                flat[:, d0:d0 + seg] = src[:, s0:s0 + seg]
        owner, c_last = block_owner(last, world, lead_skip)
        if height % row_block and owner == s:
            n = (height - last * row_block) * width
            flat[:, last * seg:last * seg + n] = src[:, c_last * seg:c_last * seg + n]
    return out


def as_rgba(frame_i32):
    """(H, W) int32 packed RGBA8 -> (H, W, 4) uint8 view."""
    a = np.ascontiguousarray(frame_i32)
    return a.view(np.uint8).reshape(a.shape[0], a.shape[1], 4)
