"""GPU: the HIP blocks, chained like apps/vv009-4kshort.grc, reproduce the committed golden
fixtures (tests/golden/make_golden.py) stage by stage, bit-exact up to the pre-IFFT carriers; the fused
chain reproduces each fixture's IQ digest (the benched 32K frame shapes included)."""
import hashlib
from pathlib import Path

import numpy as np
import pytest

import dvbt2ll
from dvbt2ll.configs import CONFIGS, ts_for_frames

pytestmark = pytest.mark.gpu
GOLD = Path(__file__).resolve().parent / "golden"


def _eq(got, g, key):
    if key in g:
        np.testing.assert_array_equal(got.view(np.uint8), g[key].view(np.uint8), err_msg=key)
    else:
        assert hashlib.sha256(np.ascontiguousarray(got).tobytes()).digest() == g[key + "_sha256"].tobytes(), key


NAMES = ["cfg1", "cfg1q", "cfg4", "cfg2", "cfg3", "cfg5"]


@pytest.mark.parametrize("name", NAMES)
def test_blocks_reproduce_golden(gpu, name):
    cfg = CONFIGS[name]
    g = np.load(GOLD / ("%s.npz" % name))
    nframes = int(g["nframes"])
    F = cfg.fecblocks
    bb = dvbt2ll.bbheaderbch_bb(*cfg.bb_args())
    ld = dvbt2ll.ldpc_bb(cfg.framesize, cfg.rate)
    im = dvbt2ll.interleavermod_bc(*cfg.im_args())
    fm = dvbt2ll.framemapperfint_cc(*cfg.fm_args())
    pg = dvbt2ll.pilotgenp1insert_cc(*cfg.pg_args())
    ts = g["ts"] if "ts" in g else ts_for_frames(cfg, 0, nframes)[0]
    off = 0
    got = {k: [] for k in ("bbbits", "codeword", "cells", "mapped", "carriers")}
    for k in range(nframes):
        bits = np.zeros(F * bb.output_multiple(), np.uint8)
        bb.general_work([ts[off:]], [bits])
        off += bb.last_consumed
        got["bbbits"].append(np.packbits(bits))
        cw = np.zeros(F * ld.output_multiple(), np.uint8)
        ld.general_work([bits], [cw])
        got["codeword"].append(np.packbits(cw))
        cells = np.zeros(F * im.output_multiple(), np.complex64)
        im.general_work([cw], [cells])
        mapped = np.zeros(fm.output_multiple(), np.complex64)
        fm.general_work([cells], [mapped])
        got["cells"].append(cells)
        got["mapped"].append(mapped)
        got["carriers"].append(pg.debug_carriers(mapped, _num_symbols(cfg), cfg.vlength))
    assert off == int(g["ts_consumed"])
    for key in got:
        _eq(np.stack(got[key]), g, key)


@pytest.mark.parametrize("name", NAMES)
def test_chain_reproduces_golden_iq(gpu, name):
    """the fused chain's IQ of the fixture's frames (complex64, gain 1) has the fixture's digest"""
    cfg = CONFIGS[name]
    g = np.load(GOLD / ("%s.npz" % name))
    nframes = int(g["nframes"])
    ch = dvbt2ll.Chain(cfg, max_frames=nframes)
    iq = ch.run(0, nframes)
    assert hashlib.sha256(np.ascontiguousarray(iq).tobytes()).digest() == g["iq_sha256"].tobytes()


def _num_symbols(cfg):
    import plan_probe as PP
    return PP.pilot_plan(cfg.pg_args())["Nsym"]
