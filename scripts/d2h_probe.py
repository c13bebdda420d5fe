"""Host-link copy rates of one GPU: D2H of one 1080p RGBA8 frame (8.3 MB)
from HBM into page-locked memory, back to back on one stream and on two, and
the strided copy of one of 8 shards' row blocks (hipMemcpy2DAsync's shape in
mirt_multi's host-direct delivery) -- the ceiling of a frame loop whose frames
all leave through one GPU's link (the gather delivery at N GPUs)."""
import json
import time

import torch

W, H = 1920, 1080


def rate(fn, reps=200):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def main():
    dev = torch.zeros((H, W), dtype=torch.int32, device="cuda")
    host = [torch.zeros((H, W), dtype=torch.int32).pin_memory() for _ in range(2)]
    s = [torch.cuda.Stream() for _ in range(2)]
    nbytes = W * H * 4

    def one():
        with torch.cuda.stream(s[0]):
            host[0].copy_(dev, non_blocking=True)

    def two():
        for k in range(2):
            with torch.cuda.stream(s[k]):
                host[k].copy_(dev, non_blocking=True)

    t1 = rate(one)
    t2 = rate(two) / 2
    # 1/8 of the frame as 8-row blocks at a pitch of 64 rows (host-direct, N = 8)
    view = host[0].view(-1, 8, W)[::8]
    src = dev.view(-1, 8, W)[: view.shape[0]]

    def strided():
        with torch.cuda.stream(s[0]):
            view.copy_(src, non_blocking=True)

    t3 = rate(strided)
    print(json.dumps({"frame_bytes": nbytes, "d2h_one_stream_gbs": round(nbytes / t1 / 1e9, 2),
                      "d2h_two_streams_gbs": round(nbytes / t2 / 1e9, 2),
                      "frame_ms": round(t1 * 1e3, 4),
                      "strided_eighth_gbs": round(nbytes / 8 / t3 / 1e9, 2),
                      "strided_eighth_ms": round(t3 * 1e3, 4),
                      "frames_per_s_ceiling_one_link": round(1 / t2, 1)}), flush=True)


if __name__ == "__main__":
    main()
