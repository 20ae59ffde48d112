"""The launch shapes bench.py times, parity-tested:

* cfg3 (BASELINE's metric configuration) at the bench's step: 192 T2 frames in one run_device
  launch on a 2-slot handle (the second slot's buffers are the ones a pipelined step writes), issued
  twice so both slots run; frames 0, 95 and 191 equal single-frame runs bit for bit and frame 191
  equals the oracle chain (bit-exact against the CPU model of the GPU IFFT, SURVEY 8(c) bounds
  against a float64 IFFT).  Large launches are where 32-bit offsets and per-frame strides would fail.
* cfg5 as BASELINE words it: an 8-stream batch through dvbt2ll_chain_run_streams, direct and hipGraph
  launches; every stream equals a single-stream handle on its own TS and stream 7 equals the oracle.
* the largest cfg3 launch a handle admits (1359 frames: the 32-bit index-pair offsets), and the refusal
  of one frame more.
* misaligned TS input: a device TS pointer 188 bytes into the buffer (188 % 16 = 12) and
  a run_streams stride that is odd; the FEC kernel's byte-load staging path must give the aligned
  call's IQ bit for bit."""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, ts_for_frames
import oracle_lib as O
import iq_check

pytestmark = pytest.mark.gpu


def _oracle_frames(cfg, frames, seed=1):
    """oracle chain carriers of the given frames of one stream: the BB block runs over every frame
    up to the last one (its state is sequential), the other blocks only over the frames asked for
    (the frame mapper's FRAME_IDX follows its call count, so it starts at a frame == 0 mod t2frames)"""
    last = max(frames)
    ts, base = ts_for_frames(cfg, 0, last + 1, seed)
    assert base == 0
    F = cfg.fecblocks
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args()); pg = O.PG(*cfg.pg_args())
    first_fm = min(frames) - min(frames) % cfg.t2frames
    off, out = 0, {}
    for k in range(last + 1):
        bits, cons = bb.work(ts[off:], F)
        off += cons
        if k >= first_fm:
            mapped = fm.work(im.work(ld.work(bits, F), F))
            if k in frames:
                out[k] = pg.carriers(mapped)
    return out, pg


def test_cfg3_bench_launch_192_frames_two_slots(gpu):
    import torch
    cfg = CONFIGS["cfg3"]
    B = 192
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    ch.set_slots(2)
    per = ch.iq_per_frame
    ts, base = ts_for_frames(cfg, 0, B)
    ts_d = torch.from_numpy(ts).cuda()
    iq = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(2):                       # slot 0, then slot 1 (the pipelined bench's second buffer set)
        ch.run_device(ts_d.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), st)
        torch.cuda.synchronize()
        got = {k: iq[k * per:(k + 1) * per].cpu().numpy().view(np.complex64).reshape(-1) for k in (0, 95, 191)}
        for k, g in got.items():
            one = ch.run(k, 1)
            np.testing.assert_array_equal(g.view(np.uint32), one.view(np.uint32), err_msg="frame %d" % k)
    del iq, ts_d
    ref, pg = _oracle_frames(cfg, [191])
    iq_check.check_frame_exact(got[191], ref[191], cfg.pg_args(), pg.guard, pg.normalization, "cfg3 frame 191 of 192")
    iq_check.check_frame(got[191], ref[191], pg.vlength, pg.guard, pg.normalization, pg.p1(), "cfg3 frame 191 of 192")


def test_cfg3_max_batch_32bit_offsets(gpu):
    """the largest launch a cfg3 handle accepts: the OFDM kernel addresses the index-pair buffer with
    32-bit byte offsets, so create admits max_frames <= (2^32 - 1) // (2 * pair_stride) (pair_stride =
    the frame's data cells rounded up to 8, t2_capi chain_build) and refuses one more.  One launch of all
    of them (1359 frames, 2.8 G IQ samples, above the bench's 1280) gives the IQ of a one-frame handle for
    the first, a middle and the last frame, bit for bit"""
    import torch
    cfg = CONFIGS["cfg3"]
    one = dvbt2ll.Chain(cfg, max_frames=1)
    stride = (one.info["stream_items"] + 7) // 8 * 8
    B = ((1 << 32) - 1) // (2 * stride)
    assert B >= 1280
    with pytest.raises(dvbt2ll.DVBT2Error):
        dvbt2ll.Chain(cfg, max_frames=B + 1)
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    per = ch.iq_per_frame
    ts, base = ts_for_frames(cfg, 0, B)
    ts_d = torch.from_numpy(ts).cuda()
    del ts
    iq = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
    ch.run_device(ts_d.data_ptr(), base, ts_d.numel(), 0, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    for k in (0, B // 2, B - 1):
        got = iq[k * per:(k + 1) * per].cpu().numpy().view(np.complex64).reshape(-1)
        want = one.run(k, 1)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg="frame %d of %d" % (k, B))


@pytest.mark.parametrize("graph", [False, True], ids=["direct", "graph"])
def test_cfg5_eight_stream_batch(gpu, graph):
    import torch
    cfg = CONFIGS["cfg5"]
    S, first, B = 8, 2, 1
    ch = dvbt2ll.Chain(cfg, max_frames=S * B)
    ref = dvbt2ll.Chain(cfg, max_frames=B)
    if graph:
        ch.set_graph(True)
    per = ch.iq_per_frame
    tss = [ts_for_frames(cfg, first, B, seed=s + 1) for s in range(S)]
    base, n = tss[0][1], len(tss[0][0])
    stride = (n + 255) // 256 * 256
    buf = np.zeros((S, stride), np.uint8)
    for s, (t, b) in enumerate(tss):
        assert b == base and len(t) == n
        buf[s, :n] = t
    ts_d = torch.from_numpy(buf.reshape(-1)).cuda()
    iq = torch.empty((S * B * per, 2), dtype=torch.float32, device="cuda")
    for _ in range(2 if graph else 1):       # graph mode: capture, then a re-armed replay
        iq.zero_()
        torch.cuda.synchronize()
        ch.run_streams(ts_d.data_ptr(), stride, S, base, n, first, B, iq.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
    got = iq.cpu().numpy().view(np.complex64).reshape(S, B * per)
    for s in range(S):
        want = ref.run(first, B, ts=tss[s][0], ts_base=base)
        np.testing.assert_array_equal(got[s].view(np.uint32), want.view(np.uint32), err_msg="stream %d" % s)
    if not graph:
        orc, pg = _oracle_frames(cfg, [first], seed=8)
        iq_check.check_frame_exact(got[7], orc[first], cfg.pg_args(), pg.guard, pg.normalization, "cfg5 stream 7")


def test_misaligned_ts_pointer(gpu):
    import torch
    cfg = CONFIGS["cfg1"]
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    per = ch.iq_per_frame
    ts, base = ts_for_frames(cfg, 1, 2)
    assert base % 188 == 0 and base >= 188
    # the same stream bytes behind one unused packet: the aligned call sees the buffer from byte 0
    # (ts_base - 188), the misaligned one from byte 188 (ts_base), 12 mod 16 past a 16-byte boundary
    d = torch.from_numpy(np.concatenate([np.zeros(188, np.uint8), ts])).cuda()
    assert d.data_ptr() % 16 == 0 and (d.data_ptr() + 188) % 16 == 12
    out = []
    for ptr, b, ln in ((d.data_ptr(), base - 188, len(ts) + 188), (d.data_ptr() + 188, base, len(ts))):
        iq = torch.empty((2 * per, 2), dtype=torch.float32, device="cuda")
        ch.run_device(ptr, b, ln, 1, 2, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        out.append(iq.cpu().numpy().view(np.complex64).reshape(-1))
    np.testing.assert_array_equal(out[0].view(np.uint32), out[1].view(np.uint32))
    np.testing.assert_array_equal(out[1].view(np.uint32), ch.run(1, 2).view(np.uint32))


def test_odd_stream_stride(gpu):
    import torch
    cfg = CONFIGS["cfg1"]
    S, first, B = 3, 1, 1
    ch = dvbt2ll.Chain(cfg, max_frames=S * B)
    ref = dvbt2ll.Chain(cfg, max_frames=B)
    per = ch.iq_per_frame
    tss = [ts_for_frames(cfg, first, B, seed=s + 1) for s in range(S)]
    base, n = tss[0][1], len(tss[0][0])
    stride = n + 37                          # odd: every stream but the first starts misaligned
    buf = np.zeros(S * stride, np.uint8)
    for s, (t, _) in enumerate(tss):
        buf[s * stride:s * stride + n] = t
    d = torch.from_numpy(buf).cuda()
    iq = torch.empty((S * B * per, 2), dtype=torch.float32, device="cuda")
    ch.run_streams(d.data_ptr(), stride, S, base, n, first, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = iq.cpu().numpy().view(np.complex64).reshape(S, B * per)
    for s in range(S):
        want = ref.run(first, B, ts=tss[s][0], ts_base=base)
        np.testing.assert_array_equal(got[s].view(np.uint32), want.view(np.uint32), err_msg="stream %d" % s)


def test_chain_graph_back_to_back_one_slot(gpu):
    """hipGraph mode: consecutive calls on one buffer slot are issued without waiting for each other
    (a ring of DVBT2LL_CHAIN_GRAPH_RING instantiations per slot); each call's frames come out as the
    direct launches give them, with more calls queued than the ring holds"""
    import torch
    cfg = CONFIGS["cfg1"]
    n = 6
    ts, base = ts_for_frames(cfg, 0, n)
    d = torch.from_numpy(ts).cuda()
    ch = dvbt2ll.Chain(cfg, max_frames=1)
    per = ch.iq_per_frame
    want = torch.empty((n, per, 2), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    for k in range(n):
        ch.run_device(d.data_ptr(), base, len(ts), k, 1, want[k].data_ptr(), st)
    torch.cuda.synchronize()
    ch.set_graph(True)
    got = torch.zeros((n, per, 2), dtype=torch.float32, device="cuda")
    for k in range(n):   # no synchronisation between the calls
        ch.run_device(d.data_ptr(), base, len(ts), k, 1, got[k].data_ptr(), st)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(got.cpu().numpy().view(np.uint32), want.cpu().numpy().view(np.uint32))
