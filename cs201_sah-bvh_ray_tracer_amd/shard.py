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


_SOURCES = {}


def _sources(height, row_block, world, device):
    """row_sources, built once per geometry and device (the gather runs every
    frame: rebuilding the index tensors cost several launches each time)."""
    key = (height, row_block, world, str(device))
    if key not in _SOURCES:
        _SOURCES[key] = row_sources(height, row_block, world, device)
    return _SOURCES[key]


def assemble(stacked, height, row_block):
    """stacked: (world, slab_rows, W) int32 slabs -> (height, W) int32 frame."""
    world = stacked.shape[0]
    shard, pos = _sources(height, row_block, world, stacked.device)
    return stacked[shard, pos]


def assemble_frames(stacked, height, row_block):
    """stacked: (world, frames, slab_rows, W) -> (frames, height, W): every
    frame of a launch de-interleaved by ONE indexing kernel."""
    world = stacked.shape[0]
    shard, pos = _sources(height, row_block, world, stacked.device)
    return stacked[shard, :, pos].transpose(0, 1)


def gather_frame(slab, height, row_block, group=None, dst=0, recv=None):
    """Gather every rank's (slab_rows, W) int32 slab -- or (frames, slab_rows,
    W) slabs of several frames -- to `dst` and assemble the frame(s) there.
    Returns the (height, W) / (frames, height, W) int32 frame(s) on dst, None
    elsewhere. recv: a preallocated (world, *slab.shape) buffer on dst (the
    per-frame gather then allocates nothing)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if not dist.is_initialized():
        st = slab[None]
    else:
        # gloo gathers host tensors (a rehearsal / CPU run): stage device slabs
        # through host memory; RCCL gathers device memory directly
        staged = slab.is_cuda and dist.get_backend(group) == "gloo"
        src = slab.contiguous().cpu() if staged else slab.contiguous()
        if rank == dst:
            if recv is None or staged or recv.shape[1:] != src.shape or recv.dtype != src.dtype:
                recv = torch.empty((world, *src.shape), dtype=src.dtype, device=src.device)
            bufs = list(recv.unbind(0))
        else:
            bufs = None
        dist.gather(src, bufs, dst=dst, group=group)
        if rank != dst:
            return None
        st = recv.to(slab.device) if staged else recv
    if slab.dim() == 2:
        return assemble(st, height, row_block)
    return assemble_frames(st, height, row_block)


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

    def __init__(self, renderer, width, height, row_block=8, group=None, samples=1, renderers=None,
                 share_accum=False, accum=None):
        self.rs = list(renderers) if renderers else [renderer]
        self.r = self.rs[0]
        self.width, self.height, self.row_block = width, height, row_block
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.samples = samples
        dev = torch.device("cuda", torch.cuda.current_device())
        self.rows = slab_rows(height, row_block, self.world)
        # per context: one slab per frame in flight (slab j: the display
        # after frame j) and the accumulation buffer of a multi-frame launch.
        # share_accum: the contexts render successive frames of ONE
        # accumulating display loop (main.c:379-408) into one buffer, their
        # folds ordered in call order (mirt_ctx_share_accum). accum=False: no
        # accumulation buffer (a multi-frame launch leaves raw frames)
        accum = samples > 1 if accum is None else accum
        self.bufs = []
        shared = torch.zeros((self.rows, width, 3), dtype=torch.float32, device=dev) if share_accum else None
        for x in self.rs:
            slabs = torch.zeros((samples, self.rows, width), dtype=torch.int32, device=dev)
            acc = shared if share_accum else (
                torch.zeros((self.rows, width, 3), dtype=torch.float32, device=dev) if accum else None)
            if share_accum and x is not self.rs[0]:
                x.share_accum(self.rs[0])
            self.bufs.append((slabs, acc))
        self.shared = share_accum
        # each context's own stream (created by mirt_create), seen by torch as
        # an external stream
        self.streams = ([torch.cuda.ExternalStream(x.stream_handle) for x in self.rs] if len(self.rs) > 1
                        else [None])
        self.k = 0
        self.slab = self.bufs[0][0][-1]
        self.stream = None
        self.recv = []

    def desc(self, depth=5, use_bvh=True, seed=1, sample=0, accumulate=False, frames=1, jitter=False, samples=None):
        from .renderer import frame_desc
        return frame_desc(self.width, self.height, depth, use_bvh, seed, sample, accumulate, frames, self.row_block,
                          self.rank, self.world, self.samples if samples is None else samples, jitter)

    def render_local(self, cam, fd):
        """Enqueue this rank's rows of the next launch (fd.samples <= samples
        frames); returns the display slab after its last frame."""
        if max(fd.samples, 1) > self.samples:
            raise ValueError(f"a launch of {fd.samples} frames, slabs for {self.samples}")
        i = self.k % len(self.rs)
        self.k += 1
        slabs, acc = self.bufs[i]
        self.stream = self.streams[i] or torch.cuda.current_stream()
        self.rs[i].render_frame_device(cam, fd, slabs.data_ptr(), acc.data_ptr() if acc is not None else None,
                                       self.stream.cuda_stream)
        self.launched = slabs[:max(fd.samples, 1)]
        self.slab = self.launched[-1]
        return self.slab

    def gather(self, every=None):
        """Gather the last launch's display slab (on its stream); the frame on
        rank 0. every=k: the displays of every k-th frame of the launch (the
        display after each group of k samples: one per displayed frame),
        stacked."""
        with torch.cuda.stream(self.stream):
            slab = self.slab if every is None else self.launched[every - 1::every]
            # one receive buffer per context on rank 0, reused every launch
            # (a launch's gather and assembly run on its context's stream, so
            # the buffer is free again when that context's next launch gathers)
            i = (self.k - 1) % len(self.rs)
            recv = self.recv[i] if i < len(self.recv) else None
            if self.rank == 0 and self.world > 1 and (recv is None or recv.shape[1:] != slab.shape):
                recv = torch.empty((self.world, *slab.shape), dtype=slab.dtype, device=slab.device)
                while len(self.recv) <= i:
                    self.recv.append(None)
                self.recv[i] = recv
            return gather_frame(slab, self.height, self.row_block, self.group, recv=recv)

    def render(self, cam, fd):
        """Render this rank's rows and gather; the (H, W) int32 frame on rank 0."""
        self.render_local(cam, fd)
        return self.gather()
