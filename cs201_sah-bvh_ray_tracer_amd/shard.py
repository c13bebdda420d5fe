"""Row-block sharding of one frame across ranks: the geometry mirt_multi uses
(include/mirt_multi.h, csrc/multi.hip), restated for host-side code and
tests.

A frame's rows are cut into blocks of `row_block` rows; block b belongs to
rank b % world (interleaved, so the expensive dense middle of the image is
spread over all ranks). Each rank renders its blocks, compacted in row order,
into a slab of shard_row_count(...) rows (shard 0 has the most rows). The
frame is then assembled either on rank 0 from the gathered slabs
(multi.hip's deinterleave_kernel) or by every rank writing its blocks into
the host frame directly (multi.hip's strided copies). Pixels do not depend on
the sharding (the RNG contract keys on the full-frame pixel index), so any
world size produces the same bytes as one GPU.
"""
import numpy as np


def shard_row_count(height, row_block, world, shard):
    """Rows of shard `shard` (matches shard_row_count in csrc/host_scene.cpp)."""
    blocks = (height + row_block - 1) // row_block
    rows = 0
    for b in range(shard, blocks, world):
        rows += min(row_block, height - b * row_block)
    return rows


def slab_rows(height, row_block, world):
    """Padded slab height: shard 0 always holds the most rows."""
    return shard_row_count(height, row_block, world, 0)


def row_sources(height, row_block, world):
    """For every image row y: (shard, row inside that shard's slab)."""
    y = np.arange(height)
    blk = y // row_block
    return blk % world, (blk // world) * row_block + (y % row_block)


def assemble_gather(slabs, height, row_block):
    """multi.hip deinterleave_kernel, restated: slabs[s] is shard s's
    (frames, rows_s, W, ...) array (the gathered displays) -> (frames,
    height, W, ...)."""
    world = len(slabs)
    src, pos = row_sources(height, row_block, world)
    frames = slabs[0].shape[0]
    out = np.empty((frames, height) + slabs[0].shape[2:], slabs[0].dtype)
    for y in range(height):
        out[:, y] = slabs[src[y]][:, pos[y]]
    return out


def assemble_direct(slabs, height, row_block):
    """multi.hip's host-direct delivery, restated: shard s writes its full
    blocks b = s, s + world, ... as one strided copy (rows of row_block * W
    pixels, destination pitch world * row_block rows) and the image's short
    last block, if it is s's, after them -> (frames, height, W)."""
    world = len(slabs)
    frames = slabs[0].shape[0]
    out = np.zeros((frames, height) + slabs[0].shape[2:], slabs[0].dtype)
    width = int(np.prod(slabs[0].shape[2:]))     # elements per image row (pixels x channels)
    blocks = (height + row_block - 1) // row_block
    last = blocks - 1
    flat = out.reshape(frames, -1)
    for s in range(world):
        nb = (last - s) // world + 1 if s < blocks else 0
        has_short = height % row_block != 0 and nb > 0 and last % world == s
        nfull = nb - (1 if has_short else 0)
        src = slabs[s].reshape(frames, -1)
        seg = row_block * width
        for i in range(nfull):      # the 2D copy: row i of the copy -> dst + i * pitch
            d0 = s * seg + i * world * seg
            flat[:, d0:d0 + seg] = src[:, i * seg:(i + 1) * seg]
        if has_short:
            n = (height - last * row_block) * width
            flat[:, last * seg:last * seg + n] = src[:, nfull * seg:nfull * seg + n]
    return out


def as_rgba(frame_i32):
    """(H, W) int32 packed RGBA8 -> (H, W, 4) uint8 view."""
    a = np.ascontiguousarray(frame_i32)
    return a.view(np.uint8).reshape(a.shape[0], a.shape[1], 4)
