"""Row-band sharding of the stackers over the GPUs of one node (one process per GPU).

Stacking shards over pixels, not frames: every output pixel needs all N samples of its
column (median / sigma-clip are not associative), so each rank owns a band of rows
[begin, end) of every frame -- the reference's own block partition
(src/stacking/stacking.c:1397-1476) lifted to GPUs.  The data path has no collective: a
rank reads its band (+ the rows its shifts reach) and writes its band of the output.
Only the 3x2 rejection counters (:1796-1817) are summed, the step time is max-reduced,
and the output bands are gathered when the caller wants the whole image on one rank.

Registration shards over FRAMES (each frame is registered against the reference
independently, register_shift_dft src/registration/registration.c:182-400): rank r takes a
contiguous block of frame indices, every rank computes the reference spectrum itself, and
only the per-frame (shiftx, shifty, raw quality) are all-gathered; normalizeQualityData
(:163-176, with the min/max loop of :384-392) then runs over all frames in index order on
every rank, so the result equals the single-process one bit for bit.

torch.distributed is plumbing here: "nccl" is RCCL over xGMI on the GPU node, "gloo" on
CPU for the tests.  The stacking itself is whatever `stack_band` the caller passes (the
C-ABI `sg_stack_u16_device` on a GPU); the per-shard registration is `register_part`
(`sg_register_dft_u16_device_raw` on a GPU).
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


def frame_band(rank, world, nframes):
    """Contiguous block [begin, end) of frame indices registered by `rank`."""
    return row_band(rank, world, nframes)


def normalize_quality(qraw, nframes, ref_image, included):
    """The quality bookkeeping of register_shift_dft on all frames: q_min / q_max seeded by
    the reference, the registered frames in index order with the reference's min() macro and
    `>` test, then normalizeQualityData (registration.c:163-176) on the included frames."""
    ref = ref_image if ref_image >= 0 else 0
    quality = np.zeros(nframes, dtype=np.float64)
    q_min = q_max = float(qraw[ref])
    quality[ref] = qraw[ref]
    for f in range(nframes):
        if f == ref or (included is not None and not included[f]):
            continue
        qv = float(qraw[f])
        quality[f] = qv
        if qv > q_max:
            q_max = qv
        q_min = q_min if q_min < qv else qv
    with np.errstate(divide="ignore", invalid="ignore"):     # x / 0.0 as in C: inf / NaN
        for f in range(nframes):
            if included is not None and not included[f]:
                continue
            quality[f] = quality[f] - q_min
            quality[f] = quality[f] / np.float64(q_max - q_min)
    return quality


def register_sharded(register_part, nframes, ref_image, included, dist, rank, world, device="cpu"):
    """Frame-sharded registration.  `register_part(included_local)` registers the frames
    whose mask entry is set (plus the reference) and returns (shiftx, shifty, raw quality)
    arrays of length nframes; this rank's mask is `included` restricted to its frame block.
    Returns (shiftx, shifty, normalised quality) on every rank."""
    import torch
    ref = ref_image if ref_image >= 0 else 0
    inc = np.ones(nframes, dtype=np.int32) if included is None else np.asarray(included, dtype=np.int32)
    b, e = frame_band(rank, world, nframes)
    mine = np.zeros(nframes, dtype=np.int32)
    mine[b:e] = inc[b:e]
    sx, sy, q = register_part(mine)
    rows = np.zeros((3, nframes), dtype=np.float64)
    rows[0], rows[1], rows[2] = sx, sy, q
    t = _tensor(rows, device)
    outs = [torch.empty_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    gx = np.zeros(nframes, dtype=np.int32)
    gy = np.zeros(nframes, dtype=np.int32)
    gq = np.zeros(nframes, dtype=np.float64)
    for r in range(world):
        rb, re = frame_band(r, world, nframes)
        o = outs[r].cpu().numpy()
        gx[rb:re], gy[rb:re], gq[rb:re] = o[0, rb:re], o[1, rb:re], o[2, rb:re]
    gq[ref] = outs[0].cpu().numpy()[2, ref]         # every rank measured the reference
    gx[ref] = gy[ref] = 0
    return gx, gy, normalize_quality(gq, nframes, ref, included)


class BandGatherPipeline:
    """Output bands of successive stack calls gathered to rank 0 without serialising the calls
    behind the gathers (configs[3]'s strong form): two band buffers, so the band
    call of step k + 1 writes one buffer while the gather of step k still reads the other.

    Per step k (slot = k mod 2):
      1. ops.wait_free(slot):  the compute stream waits until the gather of step k - 2 has read
                               buffer `slot` (nothing to wait for the first time);
      2. stack_into(buf):      the caller queues its band call writing buf (async, its redo / replay
                               tail allowed to run on the library's tail stream);
      3. ops.to_comm():        the comm stream waits for this band's result (main kernel and tail:
                               sg_stack_wait_tail), not for anything queued later;
      4. gather_fn on comm:    rank 0 receives every rank's band into gathered[slot];
      5. ops.release(slot):    buffer `slot` may be written again once the gather is done.
    The reference's team likewise reads, stacks and writes block after block with no global
    barrier between them (stacking.c:1513-1591).  `ops` supplies the stream / event plumbing
    (TorchStreamOps on a GPU; the default no-op ops for synchronous CPU collectives, gloo)."""

    class NoOps:
        def __init__(self):
            self.log = []

        def wait_free(self, slot):
            self.log.append(("wait_free", slot))

        def to_comm(self):
            self.log.append(("to_comm",))

        def on_comm(self):
            import contextlib
            return contextlib.nullcontext()

        def release(self, slot):
            self.log.append(("release", slot))

    def __init__(self, make_buf, rank, world, gather_fn, ops=None, nslots=2):
        self.bufs = [make_buf() for _ in range(nslots)]
        self.gathered = [[make_buf() for _ in range(world)] if rank == 0 else None for _ in range(nslots)]
        self.gather_fn = gather_fn
        self.ops = ops if ops is not None else BandGatherPipeline.NoOps()
        self.nslots = nslots
        self.k = 0

    def step(self, stack_into):
        slot = self.k % self.nslots
        self.k += 1
        self.ops.wait_free(slot)
        stack_into(self.bufs[slot])
        self.ops.to_comm()
        with self.ops.on_comm():
            self.gather_fn(self.bufs[slot], self.gathered[slot])
            self.ops.release(slot)
        return slot


class TorchStreamOps:
    """BandGatherPipeline plumbing on one GPU: `stream` is the stream the band calls are queued
    on, `comm` a second stream the gathers run on; `wait_tail(stream_handle)` is the library's
    sg_stack_wait_tail (a device-side wait for the async calls' tail kernels)."""

    def __init__(self, stream, comm, wait_tail, nslots=2):
        import torch
        self.stream, self.comm, self.wait_tail = stream, comm, wait_tail
        self.ev = [torch.cuda.Event() for _ in range(nslots)]
        self.used = [False] * nslots

    def wait_free(self, slot):
        if self.used[slot]:
            self.stream.wait_event(self.ev[slot])

    def to_comm(self):
        self.comm.wait_stream(self.stream)          # the band's main kernel
        self.wait_tail(self.comm.cuda_stream)       # and its tail (redo list, replay, literal)

    def on_comm(self):
        import torch
        return torch.cuda.stream(self.comm)

    def release(self, slot):
        self.ev[slot].record(self.comm)
        self.used[slot] = True
