"""Row-block sharding of one frame across ranks (one process per GPU) and the
RCCL gather of the per-rank RGBA8 slabs to rank 0.

A frame's rows are cut into blocks of `row_block` rows; block b belongs to
rank b % world (interleaved, so the expensive dense middle of the image is
spread over all ranks). Each rank renders its blocks, compacted in row order,
into a slab of slab_rows(...) rows (shard 0 has the most rows; the others
are padded to that), then `dist.gather` brings the slabs to rank 0, which
de-interleaves them on the device. The scene is replicated per rank, so the
gather is the only exchange. Pixels do not depend on the sharding (the RNG
contract keys on the full-frame pixel index), so any world size produces the
same bytes as one GPU.

Frames in flight (`samples` > 1): one launch renders this rank's rows of
`samples` successive frames of the accumulating display loop (main.c:379-408,
RNG samples sample .. sample + samples - 1) and folds them into the rank's
accumulation buffer on the device (slab j holds the display after frame j);
only the display after the last frame is gathered. The bounce pass's latency tail (its longest chains) is then paid
once per launch rather than once per frame, which is what lets the frame
rate grow with the number of GPUs: at N GPUs with samples = N every rank
traces one frame's worth of rays per step (weak scaling).
"""
import torch
import torch.distributed as dist


def shard_row_count(height, row_block, world, shard):
    """Rows of shard `shard` (matches mirt_shard_rows in csrc/host_scene.cpp)."""
    blocks = (height + row_block - 1) // row_block
    rows = 0
    for b in range(shard, blocks, world):
        rows += min(row_block, height - b * row_block)
    return rows


def slab_rows(height, row_block, world):
    """Padded slab height: shard 0 always holds the most rows."""
    return shard_row_count(height, row_block, world, 0)


def row_sources(height, row_block, world, device=None):
    """For every image row y: (shard, row inside that shard's slab)."""
    y = torch.arange(height, device=device)
    blk = y // row_block
    shard = blk % world
    pos = (blk // world) * row_block + (y % row_block)
    return shard, pos


def assemble(stacked, height, row_block):
    """stacked: (world, slab_rows, W) int32 slabs -> (height, W) int32 frame."""
    world = stacked.shape[0]
    shard, pos = row_sources(height, row_block, world, stacked.device)
    return stacked[shard, pos]


def gather_frame(slab, height, row_block, group=None, dst=0):
    """Gather every rank's (slab_rows, W) int32 slab to `dst` and assemble the
    frame there. Returns the (height, W) int32 frame on dst, None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if world == 1:
        return assemble(slab.unsqueeze(0), height, row_block)
    bufs = [torch.empty_like(slab) for _ in range(world)] if rank == dst else None
    dist.gather(slab, bufs, dst=dst, group=group)
    if rank != dst:
        return None
    return assemble(torch.stack(bufs), height, row_block)


def as_rgba(frame_i32):
    """(H, W) int32 packed RGBA8 -> (H, W, 4) uint8 view."""
    return frame_i32.contiguous().view(torch.uint8).reshape(frame_i32.shape[0], frame_i32.shape[1], 4)


class ShardedFrame:
    """Renders frames with this rank's mirt Renderer(s) and gathers them.

    renderer: a renderer.Renderer bound to this rank's GPU with the scene
    uploaded. With `renderers` (two or more contexts on the same GPU, the
    same scene uploaded to each) successive frames alternate between them,
    each on its own stream with its own slabs and queue: frame k + 1's
    launches are enqueued while frame k's bounce pass is still draining its
    last chains, so the GPU fills the slots those waves free (double
    buffering; each frame's bytes are unchanged). Otherwise torch's current
    stream carries the kernel and RCCL.
    """

    def __init__(self, renderer, width, height, row_block=8, group=None, samples=1, renderers=None):
        self.rs = list(renderers) if renderers else [renderer]
        self.r = self.rs[0]
        self.width, self.height, self.row_block = width, height, row_block
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.samples = samples
        dev = torch.device("cuda", torch.cuda.current_device())
        self.rows = slab_rows(height, row_block, self.world)
        # per context: one slab per frame in flight (the last one is the
        # display that is gathered) and the accumulation buffer of a
        # multi-frame launch
        self.bufs = []
        for _ in self.rs:
            slabs = torch.zeros((samples, self.rows, width), dtype=torch.int32, device=dev)
            acc = torch.zeros((self.rows, width, 3), dtype=torch.float32, device=dev) if samples > 1 else None
            self.bufs.append((slabs, acc))
        # each context's own stream (created by mirt_create), seen by torch as
        # an external stream
        self.streams = ([torch.cuda.ExternalStream(x.stream_handle) for x in self.rs] if len(self.rs) > 1
                        else [None])
        self.k = 0
        self.slab = self.bufs[0][0][-1]
        self.stream = None

    def desc(self, depth=5, use_bvh=True, seed=1, sample=0, accumulate=False, frames=1, jitter=False):
        from .renderer import frame_desc
        return frame_desc(self.width, self.height, depth, use_bvh, seed, sample, accumulate, frames, self.row_block,
                          self.rank, self.world, self.samples, jitter)

    def render_local(self, cam, fd):
        """Enqueue this rank's rows of the next frame; returns its display slab."""
        i = self.k % len(self.rs)
        self.k += 1
        slabs, acc = self.bufs[i]
        self.stream = self.streams[i] or torch.cuda.current_stream()
        self.rs[i].render_frame_device(cam, fd, slabs.data_ptr(), acc.data_ptr() if acc is not None else None,
                                       self.stream.cuda_stream)
        self.slab = slabs[-1]
        return self.slab

    def gather(self):
        """Gather the last rendered slab (on its stream); the frame on rank 0."""
        with torch.cuda.stream(self.stream):
            if self.world == 1:
                return assemble(self.slab.unsqueeze(0), self.height, self.row_block)
            return gather_frame(self.slab, self.height, self.row_block, self.group)

    def render(self, cam, fd):
        """Render this rank's rows and gather; the (H, W) int32 frame on rank 0."""
        self.render_local(cam, fd)
        return self.gather()
