"""GPU parity of every block against the CPU oracle (bit-exact except after the IFFT).

Run on an MI355X: python -m pytest tests -m gpu.  The HIP library is called through its C
ABI (dvbt2ll python mirror -> ctypes -> libdvbt2ll_hip.so); there is no CPU fallback.
"""
import numpy as np
import pytest

import dvbt2ll
from dvbt2ll import enums as E
from dvbt2ll.configs import CONFIGS, ts_for_frames, ts_packets
import oracle_lib as O
import iq_check

pytestmark = pytest.mark.gpu

def _ts(cfg, nframes=1):
    ts, base = ts_for_frames(cfg, 0, nframes)
    assert base == 0
    return ts


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_bbheaderbch_bit_exact(gpu, name):
    cfg = CONFIGS[name]
    ts = _ts(cfg)
    ref = O.BB(*cfg.bb_args())
    blk = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    F = cfg.fecblocks
    want, cons = ref.work(ts, F)
    got = np.zeros(F * ref.nbch, np.uint8)
    n = blk.general_work([ts], [got])
    assert n == F * ref.nbch
    assert blk.last_consumed == cons
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("name", ["cfg1", "cfg3"])
def test_bbheaderbch_split_calls(gpu, name):
    """state (count, crc, fec_block) carried across general_work calls like the reference"""
    cfg = CONFIGS[name]
    ts = _ts(cfg, 2)
    ref = O.BB(*cfg.bb_args())
    blk = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    nb = ref.nbch
    off = 0
    for calls in (1, 3, 2, 5):
        want, cons = ref.work(ts[off:], calls)
        got = np.zeros(calls * nb, np.uint8)
        blk.general_work([ts[off:]], [got])
        assert blk.last_consumed == cons
        np.testing.assert_array_equal(got, want)
        off += cons


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_ldpc_bit_exact(gpu, name):
    cfg = CONFIGS[name]
    bb = O.BB(*cfg.bb_args())
    bits, _ = bb.work(_ts(cfg), 4)
    want = O.LDPC(cfg.framesize, cfg.rate).work(bits, 4)
    blk = dvbt2ll.ldpc_bb(cfg.framesize, cfg.rate)
    got = np.zeros_like(want)
    assert blk.general_work([bits], [got]) == len(want)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_interleavermod_bit_exact(gpu, name):
    cfg = CONFIGS[name]
    bb = O.BB(*cfg.bb_args())
    bits, _ = bb.work(_ts(cfg), 3)
    cw = O.LDPC(cfg.framesize, cfg.rate).work(bits, 3)
    im = O.IM(*cfg.im_args())
    want = im.work(cw, 3)
    blk = dvbt2ll.interleavermod_bc(*cfg.im_args())
    got = np.zeros_like(want)
    assert blk.general_work([cw], [got]) == len(want)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


def _oracle_cells(cfg):
    F = cfg.fecblocks
    bits, _ = O.BB(*cfg.bb_args()).work(_ts(cfg), F)
    cw = O.LDPC(cfg.framesize, cfg.rate).work(bits, F)
    return O.IM(*cfg.im_args()).work(cw, F)


@pytest.mark.parametrize("name", ["cfg1", "cfg3", "cfg4"])
def test_framemapper_bit_exact(gpu, name):
    cfg = CONFIGS[name]
    cells = _oracle_cells(cfg)
    fm = O.FM(*cfg.fm_args())
    blk = dvbt2ll.framemapperfint_cc(*cfg.fm_args())
    assert blk.output_multiple() == fm.mapped_items
    for frame in range(3):      # t2_frame_num cycles through t2frames (L1-post FRAME_IDX)
        want = fm.work(cells)
        got = np.zeros(fm.mapped_items, np.complex64)
        assert blk.general_work([cells], [got]) == fm.mapped_items
        assert blk.last_consumed == fm.stream_items
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_pilotgen_carriers_bit_exact_and_iq(gpu, name):
    cfg = CONFIGS[name]
    cells = _oracle_cells(cfg)
    mapped = O.FM(*cfg.fm_args()).work(cells)
    pg = O.PG(*cfg.pg_args())
    blk = dvbt2ll.pilotgenp1insert_cc(*cfg.pg_args())
    want_car = pg.carriers(mapped)
    got_car = blk.debug_carriers(mapped, pg.num_symbols, pg.vlength)
    np.testing.assert_array_equal(got_car.view(np.uint32), want_car.view(np.uint32))
    iq = np.zeros(pg.output_items, np.complex64)
    assert blk.general_work([mapped], [iq]) == pg.output_items
    iq_check.check_frame(iq, want_car, pg.vlength, pg.guard, pg.normalization, pg.p1(), "pilotgen " + name)
    iq_check.check_frame_exact(iq, want_car, cfg.pg_args(), pg.guard, pg.normalization, "pilotgen " + name)


ALL_CODES = [(1, r) for r in range(6)] + [(0, r) for r in range(8)]
MODES = [(E.INPUTMODE_NORMAL, E.INBAND_OFF), (E.INPUTMODE_HIEFF, E.INBAND_OFF), (E.INPUTMODE_NORMAL, E.INBAND_ON)]


@pytest.mark.parametrize("framesize,rate", ALL_CODES)
@pytest.mark.parametrize("mode,inband", MODES, ids=["nm", "hem", "nm-inband"])
def test_bbheader_ldpc_all_codes(gpu, framesize, rate, mode, inband):
    """every FECFRAME size x code rate, normal / high-efficiency mode, in-band type B:
    BBHEADER+CRC-8+scrambler+BCH and LDPC bit-exact, state carried across two calls"""
    cfg = CONFIGS["cfg1"].with_(framesize=framesize, rate=rate, inputmode=mode, inband=inband, fecblocks=3)
    ts = ts_packets(0, 600)
    ref = O.BB(*cfg.bb_args())
    blk = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    off = 0
    for calls in (2, 5):
        want, cons = ref.work(ts[off:], calls)
        got = np.zeros_like(want)
        blk.general_work([ts[off:]], [got])
        assert blk.last_consumed == cons
        np.testing.assert_array_equal(got, want)
        off += cons
    cw_want = O.LDPC(framesize, rate).work(want, 5)
    ld = dvbt2ll.ldpc_bb(framesize, rate)
    cw = np.zeros_like(cw_want)
    ld.general_work([want], [cw])
    np.testing.assert_array_equal(cw, cw_want)


@pytest.mark.parametrize("framesize,rate", ALL_CODES)
@pytest.mark.parametrize("const", [E.MOD_QPSK, E.MOD_16QAM, E.MOD_64QAM, E.MOD_256QAM])
def test_interleavermod_all_codes(gpu, framesize, rate, const):
    rng = np.random.default_rng(1000 * framesize + 10 * rate + const)
    nldpc = 64800 if framesize else 16200
    cw = rng.integers(0, 2, 3 * nldpc, dtype=np.uint8)
    for rot in (E.ROTATION_OFF, E.ROTATION_ON):
        args = (framesize, rate, const, rot)
        want = O.IM(*args).work(cw, 3)
        got = np.zeros_like(want)
        dvbt2ll.interleavermod_bc(*args).general_work([cw], [got])
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))
