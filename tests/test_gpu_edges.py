"""GPU: edge cases of the drop-in boundary -- empty and ragged calls, short input, out-of-range
arguments -- with the reference's runtime contract: a call with fewer output
items than output_multiple produces and consumes nothing; a ragged request produces the largest
multiple that fits; too little input is an error (DVBT2LL_ESHORT), never a partial frame."""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, ts_for_frames

pytestmark = pytest.mark.gpu


def _blocks(cfg):
    return [dvbt2ll.bbheaderbch_bb(*cfg.bb_args()), dvbt2ll.ldpc_bb(cfg.framesize, cfg.rate),
            dvbt2ll.interleavermod_bc(*cfg.im_args()), dvbt2ll.framemapperfint_cc(*cfg.fm_args()),
            dvbt2ll.pilotgenp1insert_cc(*cfg.pg_args())]


@pytest.mark.parametrize("name", ["cfg1", "cfg4"])
def test_blocks_empty_calls(gpu, name):
    """nout < output_multiple (including 0): returns 0, consumes 0, output untouched"""
    for b in _blocks(CONFIGS[name]):
        om = b.output_multiple()
        for nout in (0, om - 1):
            out = np.full(max(nout, 1), 7, b.out_dtype)
            inp = np.zeros(b.forecast(om)[0] + 1000, b.in_dtype)
            assert b.general_work([inp], [out], nout) == 0, type(b).__name__
            assert b.last_consumed == 0
            assert (out == 7).all()


def test_bbheaderbch_ragged_request(gpu):
    """nout = 2.5 output multiples -> exactly 2 FEC blocks, consuming forecast(2 nbch) bytes"""
    cfg = CONFIGS["cfg1"]
    b = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    om = b.output_multiple()
    ts, _ = ts_for_frames(cfg, 0, 1)
    out = np.zeros(om * 3, np.uint8)
    n = b.general_work([ts], [out], om * 2 + om // 2)
    assert n == 2 * om
    assert b.last_consumed <= b.forecast(2 * om)[0] + 188


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_short_input_is_an_error(gpu, name):
    cfg = CONFIGS[name]
    bb = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    om = bb.output_multiple()
    need = bb.forecast(om)[0]
    with pytest.raises(dvbt2ll.DVBT2Error):
        bb.general_work([np.zeros(need // 2, np.uint8)], [np.zeros(om, np.uint8)], om)
    assert bb.nitems_consumed == 0
    fm = dvbt2ll.framemapperfint_cc(*cfg.fm_args())
    M = fm.output_multiple()
    with pytest.raises(dvbt2ll.DVBT2Error):
        fm.general_work([np.zeros(fm.stream_items() - 1, np.complex64)], [np.zeros(M, np.complex64)], M)


def test_chain_argument_checks(gpu):
    cfg = CONFIGS["cfg1"]
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    ts, base = ts_for_frames(cfg, 0, 2)
    iq = np.zeros(3 * ch.iq_per_frame, np.complex64)
    import ctypes
    lib = dvbt2ll.lib()

    def run(ts_arr, ts_base, first, n):
        return lib.dvbt2ll_chain_run_host(ch._h, ts_arr.ctypes.data_as(ctypes.c_void_p), int(ts_base), len(ts_arr),
                                          int(first), int(n), iq.ctypes.data_as(ctypes.c_void_p))

    assert run(ts, base, 0, 2) == 0
    assert run(ts, base, 0, 3) == -1            # more frames than max_frames
    assert run(ts, base, 0, 0) == -1            # empty call
    assert run(ts, base, -1, 1) == -1           # negative frame index
    assert run(ts[:-1000], base, 0, 2) == -1    # TS slice ends before the last consumed byte
    assert run(ts, base, 5, 1) == -1            # TS slice does not reach frame 5
    ts5, base5 = ts_for_frames(cfg, 5, 1)
    assert run(ts5, base5, 5, 1) == 0
    assert run(ts5[188:], base5 + 188, 5, 1) == -1   # missing the packet before the first byte


def test_chain_rejects_oversized_fecblocks(gpu):
    """a frame that cannot carry fecblocks is refused at create time (the reference
    only warns and overruns)"""
    import dataclasses
    cfg = CONFIGS["cfg1"]
    big = dataclasses.replace(cfg, fecblocks=cfg.fecblocks * 4)
    with pytest.raises(dvbt2ll.DVBT2Error):
        dvbt2ll.Chain(big, max_frames=1)


@pytest.mark.parametrize("mode", [dvbt2ll.INPUTMODE_NORMAL, dvbt2ll.INPUTMODE_HIEFF], ids=["nm", "hem"])
def test_sync_errors_counted_output_unchanged(gpu, mode):
    """a TS sync byte != 0x47 is what the reference warns about ("Transport Stream sync error!",
    bbheaderbch_bb_impl.cc:675-677, 703-705) without changing its output (NM: the slot carries the
    CRC-8; HEM: the byte is dropped).  Block and chain count exactly the corrupted sync bytes the
    encoded frames consume, and produce the same output as for the clean stream."""
    import oracle_lib as O
    cfg = CONFIGS["cfg1"].with_(inputmode=mode)
    ts, base = ts_for_frames(cfg, 0, 2)
    assert base == 0
    bad = ts.copy()
    corrupt = [3, 10, 17]               # packets whose sync byte the first frame consumes
    bad[[188 * p for p in corrupt]] = 0x46
    F = cfg.fecblocks
    want, cons = O.BB(*cfg.bb_args()).work(ts, F)
    assert cons > 188 * 18
    blk = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    got = np.zeros_like(want)
    blk.general_work([bad], [got])
    np.testing.assert_array_equal(got, want)
    assert blk.sync_errors() == len(corrupt)
    ch = dvbt2ll.Chain(cfg, max_frames=1)
    clean = ch.run(0, 1)
    assert ch.sync_errors() == 0
    dirty = ch.run(0, 1, ts=bad, ts_base=0)
    np.testing.assert_array_equal(dirty.view(np.uint32), clean.view(np.uint32))
    assert ch.sync_errors() == len(corrupt)


def test_chain_rejects_unaligned_ts_base(gpu):
    cfg = CONFIGS["cfg1"]
    ch = dvbt2ll.Chain(cfg, max_frames=1)
    ts, base = ts_for_frames(cfg, 2, 1)
    with pytest.raises(dvbt2ll.DVBT2Error):
        ch.run(2, 1, ts=ts[1:], ts_base=base + 1)


def test_graph_mode_async_calls_on_two_streams(gpu):
    """hipGraph mode re-armed by back-to-back asynchronous calls on two streams with two slots (no
    host synchronisation between calls): every call's IQ equals the direct launches' bit-exactly"""
    import torch
    cfg = CONFIGS["cfg1"]
    B, ncalls = 1, 8
    ref = dvbt2ll.Chain(cfg, max_frames=B)
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    ch.set_slots(2)
    ch.set_graph(True)
    per = ch.iq_per_frame
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ts_all, base_all = ts_for_frames(cfg, 0, B * ncalls)
    ts_dev = torch.from_numpy(ts_all).cuda()
    outs = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(ncalls)]
    torch.cuda.synchronize()
    for c in range(ncalls):
        ch.run_device(ts_dev.data_ptr(), base_all, len(ts_all), c * B, B, outs[c].data_ptr(),
                      streams[c % 2].cuda_stream)
    torch.cuda.synchronize()
    for c in range(ncalls):
        want = ref.run(c * B, B)
        got = outs[c].cpu().numpy().view(np.complex64).reshape(-1)
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg="call %d" % c)


def test_timing_with_two_streams(gpu):
    """stage timing enabled while calls alternate over two streams and two slots: every call's
    three stages are counted once and the fold succeeds (each run's end event is waited on)"""
    import torch
    cfg = CONFIGS["cfg1"]
    ch = dvbt2ll.Chain(cfg, max_frames=2)
    ch.set_slots(2)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    ts_all, base_all = ts_for_frames(cfg, 0, 2)
    ts_dev = torch.from_numpy(ts_all).cuda()
    outs = [torch.empty((2 * ch.iq_per_frame, 2), dtype=torch.float32, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    ch.set_timing(True)
    for c in range(10):
        ch.run_device(ts_dev.data_ptr(), base_all, len(ts_all), 0, 2, outs[c % 2].data_ptr(),
                      streams[c % 2].cuda_stream)
    ms, n = ch.timing()
    assert n == [10, 10, 10, 0] and all(t > 0 for t in ms[:3])   # stage 3 reserved: L1-post runs inside the map launch
    ch.set_timing(False)
