"""debug: the refill-between-async-calls case of tests/test_gpu_bands.py::test_async_tail_frames_refilled
in four forms (sync, async without refill, async + wait_tail + refill, async + refill without the wait)"""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "siril-0.9_amd", "python"), os.path.join(ROOT, "tests")]
import numpy as np
import torch
import oracle_lib as orc
import sirilgpu as sg

N, C, H, W = 16, 1, 40, 160
for rejection, sig in [(sg.SIGMA, (0.2, 0.2)), (sg.WINSORIZED, (0.3, 0.3)), (sg.SIGMA, (4.0, 3.0))]:
    fa = orc.synth(N, C, H, W, seed=71, maxshift=4)
    fb = orc.synth(N, C, H, W, seed=72, maxshift=4)
    sx, sy = orc.synth_shifts(N, seed=71, maxshift=4)
    rca, refa, rja = orc.stack_rejection(fa, rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=4)
    rcb, refb, rjb = orc.stack_rejection(fb, rejection, sig=sig, shiftx=sx, shifty=sy, max_thread=4)
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int16)).cuda()
    with sg.Context([0]) as ctx:
        for mode in ["sync", "sync_sorted", "async", "async_refill_wait", "async_refill_nowait"]:
            buf, srcb = dev(fa), dev(fb)
            outa = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
            outb = torch.zeros(C * H * W, dtype=torch.int16, device="cuda")
            torch.cuda.synchronize()
            sobj = torch.cuda.Stream()
            stream = sobj.cuda_stream
            torch.cuda.set_stream(sobj)
            desc, keep = sg.make_desc(sg.MEAN, N, W, H, C, rejection=rejection, sig=sig, shiftx=sx, shifty=sy,
                                      max_thread=4, max_number_of_rows=H,
                                      flags=0 if mode.startswith("sync") else sg.RESULT_AT_COLLECT,
                                      kernel_path=sg.PATH_SORTED if mode == "sync_sorted" else 0)
            if mode.startswith("sync"):
                rj, _ = ctx.stack_device(desc, buf.data_ptr(), C * H * W, H * W, outa.data_ptr(), 0, H, stream=stream)
                st = ctx.stats()
                ga = outa.cpu().numpy().view(np.uint16).reshape(C, H, W)
                print(rejection, sig, mode, "A diff", int((ga != refa).sum()), "rej", rj.tolist(), rja.tolist(),
                      "slow", st.slow_pixels, "chain", st.chain_pixels, flush=True)
                continue
            ctx.stack_device_async(desc, buf.data_ptr(), C * H * W, H * W, outa.data_ptr(), 0, H, stream=stream)
            if mode == "async_refill_wait":
                ctx.wait_tail(stream)
            if mode != "async":
                buf.copy_(srcb)
            ctx.stack_device_async(desc, buf.data_ptr(), C * H * W, H * W, outb.data_ptr(), 0, H, stream=stream)
            rc, rej, _ = ctx.collect()
            st = ctx.stats()
            ga = outa.cpu().numpy().view(np.uint16).reshape(C, H, W)
            gb = outb.cpu().numpy().view(np.uint16).reshape(C, H, W)
            wantb = refa if mode == "async" else refb
            print(rejection, sig, mode, "rc", rc, "A diff", int((ga != refa).sum()), "B diff", int((gb != wantb).sum()),
                  "rej", rej.tolist(), "slow", st.slow_pixels, "chain", st.chain_pixels, flush=True)
