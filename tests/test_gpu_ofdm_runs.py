"""The <= 16K OFDM kernel's runs of units per workgroup (launches of >= 8192 (symbol, frame) units: 2 units
per workgroup for 4K and below, up to 4 for 8K / 16K, with the next unit's data slots prefetched during the
current transform and the tables stored once) at the shapes that take them, checked by a size-independent
property: every frame of a large launch equals the same frame encoded alone (one unit per
workgroup, no prefetch), bit for bit -- including the launch's last, partial run and the multi-PLP kernel,
which runs units back to back without the prefetch.  Each single-frame reference is itself checked against
the oracle by test_gpu_chain / test_gpu_mplp."""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, MPLP_CONFIGS, ts_for_frames

pytestmark = pytest.mark.gpu


def _frames_device(ch, cfg, first, n, fmt):
    import torch
    ts, base = ts_for_frames(cfg, first, n)
    d = torch.from_numpy(ts).cuda()
    dt = torch.float32 if fmt == dvbt2ll.IQ_CF32 else torch.int16
    iq = torch.empty((n * ch.iq_per_frame, 2), dtype=dt, device="cuda")
    ch.run_device(d.data_ptr(), base, len(ts), first, n, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return iq


@pytest.mark.parametrize("name,B,fmt", [("cfg4", 601, dvbt2ll.IQ_CF32),      # 36,661 units: runs of 4, a tail of 1
                                         ("cfg4", 270, dvbt2ll.IQ_SC16),      # 16,470 units: runs of 2
                                         ("cfg1", 2400, dvbt2ll.IQ_CF32)])    # 16,800 4K units: runs of 2
def test_large_launch_frames_equal_single(gpu, name, B, fmt):
    import torch
    cfg = CONFIGS[name]
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    if fmt == dvbt2ll.IQ_SC16:
        ch.set_output(0.2, dvbt2ll.IQ_SC16)
    big = _frames_device(ch, cfg, 0, B, fmt)
    per = ch.iq_per_frame
    for f in sorted({0, 1, B // 3, B // 2 + 1, B - 2, B - 1}):
        one = _frames_device(ch, cfg, f, 1, fmt)
        got = big[f * per:(f + 1) * per]
        if fmt == dvbt2ll.IQ_CF32:   # bit for bit (signed zeros included)
            got, one = got.view(torch.int32), one.view(torch.int32)
        assert bool((got == one).all()), (name, B, f)


def test_mplp_large_launch_frames_equal_single(gpu):
    """the multi-PLP <= 16K kernel (runs without the slot prefetch) at 300 8K frames (18,300 units)"""
    import torch
    from test_gpu_mplp import _device_ts
    m = MPLP_CONFIGS["mplp2_8k"]
    B = 300
    ch = dvbt2ll.Chain(m, max_frames=B)
    per = ch.iq_per_frame
    bufs, bases, lens = _device_ts(m, 0, B)
    big = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
    ch.run_plps([b.data_ptr() for b in bufs], bases, lens, 0, B, big.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for f in (0, B // 2, B - 1):
        one = torch.empty((per, 2), dtype=torch.float32, device="cuda")
        ch.run_plps([b.data_ptr() for b in bufs], bases, lens, f, 1, one.data_ptr(),
                    torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert bool((big[f * per:(f + 1) * per].view(torch.int32) == one.view(torch.int32)).all()), f
