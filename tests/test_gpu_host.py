"""The streaming host path (dvbt2ll_chain_host_submit / _host_wait / _run_host_pipelined): host TS in, host IQ
out, copy-in / kernels / copy-out of consecutive submissions overlapped on three streams through a ring of
DVBT2LL_HOST_RING device buffer sets.  The reference's output is host memory feeding a sink
(lib/pilotgenp1insert_cc_impl.cc:2785-2906 -> apps/vv009-4kshort.grc:801-1623).  Every output is compared
byte for byte with the device path (run_device), itself bit-exact against the oracle (test_gpu_chain.py)."""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, ts_for_frames

pytestmark = pytest.mark.gpu


def _device_ref(cfg, first, n, fmt=dvbt2ll.IQ_CF32, gain=1.0):
    ch = dvbt2ll.Chain(cfg, max_frames=n)
    ch.set_output(gain, fmt)
    return ch.run(first, n)


@pytest.mark.parametrize("name,fmt", [("cfg1", dvbt2ll.IQ_CF32), ("cfg1", dvbt2ll.IQ_SC16), ("cfg4", dvbt2ll.IQ_SC16)])
def test_host_submit_ring_wraps(gpu, name, fmt):
    """seven submissions of two frames each (the ring of three entries wraps twice), page-locked host
    buffers, all in flight before the first wait: every frame equals the device path's"""
    import torch
    cfg = CONFIGS[name]
    B, K = 2, 7
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    gain = 0.2 if fmt == dvbt2ll.IQ_SC16 else 1.0
    ch.set_output(gain, fmt)
    per = ch.iq_per_frame
    ts, base = ts_for_frames(cfg, 0, B * K)
    ts_pin = torch.from_numpy(ts).pin_memory()
    dt = torch.int16 if fmt == dvbt2ll.IQ_SC16 else torch.float32
    outs = [torch.zeros((B * per, 2), dtype=dt).pin_memory() for _ in range(K)]
    tickets = [ch.host_submit(ts_pin.data_ptr(), base, len(ts), k * B, B, outs[k].data_ptr()) for k in range(K)]
    assert tickets == list(range(K))
    ch.host_wait(tickets[-1])
    want = _device_ref(cfg, 0, B * K, fmt, gain)
    got = torch.cat(outs).numpy()
    np.testing.assert_array_equal(got.view(np.uint8).reshape(-1), want.view(np.uint8).reshape(-1))
    for t in tickets:                   # waiting on completed / recycled tickets returns at once
        ch.host_wait(t)


@pytest.mark.parametrize("name,chunk", [("cfg3", 1), ("cfg1", 3), ("cfg1", 0)])
def test_run_host_pipelined(gpu, name, chunk):
    """run_host_pipelined over pageable numpy buffers (the runtime stages them) in chunks, cf32 and sc16"""
    cfg = CONFIGS[name]
    n = 4 if name == "cfg3" else 7
    ch = dvbt2ll.Chain(cfg, max_frames=4)
    ts, base = ts_for_frames(cfg, 0, n)
    iq = np.zeros(n * ch.iq_per_frame, np.complex64)
    ch.run_host_pipelined(ts, base, 0, n, iq, chunk)
    want = _device_ref(cfg, 0, n)
    np.testing.assert_array_equal(iq.view(np.uint32), want.view(np.uint32))
    ch.set_output(0.2, dvbt2ll.IQ_SC16)
    iq16 = np.zeros((n * ch.iq_per_frame, 2), np.int16)
    ch.run_host_pipelined(ts, base, 0, n, iq16, chunk)
    np.testing.assert_array_equal(iq16, _device_ref(cfg, 0, n, dvbt2ll.IQ_SC16, 0.2))


def test_host_submit_rejects(gpu):
    import torch
    from dvbt2ll.configs import MPLP_CONFIGS
    cfg = CONFIGS["cfg1"]
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    ts, base = ts_for_frames(cfg, 0, 2)
    iq = torch.zeros((2 * ch.iq_per_frame, 2), dtype=torch.float32).pin_memory()
    tsp = torch.from_numpy(ts).pin_memory()
    with pytest.raises(dvbt2ll.DVBT2Error):           # TS too short for the frames
        ch.host_submit(tsp.data_ptr(), base, len(ts) - 400, 0, 2, iq.data_ptr())
    with pytest.raises(dvbt2ll.DVBT2Error):           # more frames than max_frames
        ch.host_submit(tsp.data_ptr(), base, len(ts), 0, 3, iq.data_ptr())
    with pytest.raises(dvbt2ll.DVBT2Error):           # no submission with that ticket yet
        ch.host_wait(5)
    m = dvbt2ll.Chain(MPLP_CONFIGS["mplp3_4k"], max_frames=1)
    with pytest.raises(dvbt2ll.DVBT2Error):           # single-PLP chains only
        m.host_submit(tsp.data_ptr(), base, len(ts), 0, 1, iq.data_ptr())


def test_host_paths_unit_checks_before_any_copy(gpu):
    """a chain whose launch unit is 2 T2 frames (FRAME_INTERVAL 2, ij2_4k_single): submissions and pipelined
    calls off the unit grid are refused before any copy is queued (a refused call must leave no DMA
    into or out of the caller's buffers); pipelined chunks are rounded down to whole units and the output equals
    the device path's"""
    import torch
    from dvbt2ll.configs import IF_CONFIGS
    from test_gpu_mplp import _run
    m = IF_CONFIGS["ij2_4k_single"]
    assert m.unit_frames == 2
    n = 6
    ch = dvbt2ll.Chain(m, max_frames=4)
    ts, base = ts_for_frames(m.plps[0], 0, n, seed=1)
    tsp = torch.from_numpy(ts).pin_memory()
    iq = torch.zeros((n * ch.iq_per_frame, 2), dtype=torch.float32).pin_memory()
    for first, nf in ((1, 2), (0, 3)):
        with pytest.raises(dvbt2ll.DVBT2Error):
            ch.host_submit(tsp.data_ptr(), base, len(ts), first, nf, iq.data_ptr())
    out = np.zeros(n * ch.iq_per_frame, np.complex64)
    with pytest.raises(dvbt2ll.DVBT2Error):          # 5 frames: the last chunk would not be a whole unit
        ch.run_host_pipelined(ts, base, 0, 5, out, 2)
    with pytest.raises(dvbt2ll.DVBT2Error):          # a chunk smaller than the unit
        ch.run_host_pipelined(ts, base, 0, n, out, 1)
    assert not out.any()                            # nothing was copied out by the refused calls
    ch.run_host_pipelined(ts, base, 0, n, out, 3)   # chunks of 3 -> 2 frames
    want = _run(dvbt2ll.Chain(m, max_frames=n), m, 0, n)
    np.testing.assert_array_equal(out.view(np.uint32), want.view(np.uint32))
    ch.synchronize()
