"""Row-band sharding of the stackers over the GPUs of one node (one process per GPU).

Stacking shards over pixels, not frames: every output pixel needs all N samples of its
column (median / sigma-clip are not associative), so each rank owns a band of rows
[begin, end) of every frame -- the reference's own block partition
(src/stacking/stacking.c:1397-1476) lifted to GPUs.  The data path has no collective: a
rank reads its band (+ the rows its shifts reach) and writes its band of the output.
Only the 3x2 rejection counters (:1796-1817) are summed, the step time is max-reduced,
and the output bands are gathered when the caller wants the whole image on one rank.

torch.distributed is plumbing here: "nccl" is RCCL over xGMI on the GPU node, "gloo" on
CPU for the tests.  The stacking itself is whatever `stack_band` the caller passes (the
C-ABI `sg_stack_u16_device` on a GPU).
"""
import numpy as np


def row_band(rank, world, height):
    """Balanced contiguous row band [begin, end) of `rank` (memory rows)."""
    q, r = divmod(height, world)
    begin = rank * q + min(rank, r)
    return begin, begin + q + (1 if rank < r else 0)


def _tensor(x, device):
    import torch
    return torch.as_tensor(np.ascontiguousarray(x), device=device)


def sum_counters(rej, dist, device="cpu"):
    """All-reduce (sum) of the per-channel low/high rejection counters."""
    import torch
    t = _tensor(np.asarray(rej, dtype=np.int64).reshape(-1), device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t.cpu().numpy().astype(np.uint64).reshape(3, 2)


def max_time(seconds, dist, device="cpu"):
    import torch
    t = torch.tensor([float(seconds)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_bands(band, begin, end, height, dist, world, device="cpu"):
    """Gather the [C][end-begin][W] output bands of every rank into a [C][H][W] image
    (on every rank; bands are padded to the largest band for all_gather)."""
    import torch
    C, h, W = band.shape
    hmax = -(-height // world)
    buf = np.zeros((C, hmax, W), dtype=np.int32)      # gloo has no 16-bit all_gather
    buf[:, :h] = band
    t = _tensor(buf, device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    img = np.zeros((C, height, W), dtype=np.uint16)
    for r in range(world):
        b, e = row_band(r, world, height)
        img[:, b:e] = outs[r].cpu().numpy()[:, :e - b].astype(np.uint16)
    return img


def stack_sharded(stack_band, height, dist, rank, world, device="cpu"):
    """Run `stack_band(begin, end) -> (band[C][end-begin][W], rej[3][2])` on this rank's
    band, then gather the image and sum the counters (both on every rank)."""
    begin, end = row_band(rank, world, height)
    band, rej = stack_band(begin, end)
    img = gather_bands(band, begin, end, height, dist, world, device)
    return img, sum_counters(rej, dist, device)
