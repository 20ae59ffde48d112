"""CPU: known-answer and structural checks pinning the oracle restatement (the reference has
no tests or golden vectors; its lib/*.cc needs GNU Radio and is unbuildable here)."""
import numpy as np
import pytest

from dvbt2ll import enums as E
from dvbt2ll.configs import CONFIGS, ts_for_frames, ts_packets
import oracle_lib as O
import std_tables as T


def test_crc8_dvbs2_check_value():
    # CRC-8/DVB-S2 (poly 0xD5, init 0) check value of "123456789"
    assert O.lib().orc_crc8_dvbs2(b"123456789", 9) == 0xBC


def test_crc32_mpeg2_check_value():
    bits = np.unpackbits(np.frombuffer(b"123456789", np.uint8))
    assert O.lib().orc_crc32_bits(bits.ctypes.data, len(bits)) == 0x0376E6E7


def test_bb_scrambler_prbs_known_start():
    # PRBS 1+x^14+x^15 from 100101010000000 (EN 300 421 energy dispersal / EN 302 755 5.2.2)
    b = np.zeros(64, np.uint8)
    O.lib().orc_bb_prbs(b.ctypes.data, 64)
    assert np.packbits(b).tobytes().hex() == "03f6083430b8a393"


def _poly_mod(bits, g):
    """remainder of the polynomial with coefficient list bits (highest power first) mod g"""
    r = list(bits[: len(g) - 1])
    for b in bits[len(g) - 1:]:
        r.append(int(b))
        if r[0]:
            r = [x ^ y for x, y in zip(r, g)]
        r = r[1:]
    return r


@pytest.mark.parametrize("framesize,rate", [(1, E.C3_5), (1, E.C2_3), (0, E.C4_5)])
def test_bch_codeword_divisible_by_generator(framesize, rate):
    cfg = CONFIGS["cfg3"].with_(framesize=framesize, rate=rate)
    bb = O.BB(*cfg.bb_args())
    ts, _ = ts_for_frames(cfg.with_(fecblocks=1), 0, 1)
    cw, _ = bb.work(ts, 1)
    P = bb.nbch - bb.kbch
    g = T.bch_generator(framesize == 1, P)              # highest power first, degree P
    assert not any(_poly_mod(cw[: bb.nbch], g))


@pytest.mark.parametrize("framesize,rate", [(1, r) for r in range(6)] + [(0, r) for r in range(8)])
def test_ldpc_parity_check_equations(framesize, rate):
    """H c = 0 evaluated check by check from the standard tables (independent of the encoder's
    accumulate formulation): p_j ^ p_{j-1} ^ XOR(info bits on check j) == 0"""
    nbch, q = T.fec(framesize, rate)
    nldpc = 64800 if framesize else 16200
    rng = np.random.default_rng(rate + 10 * framesize)
    info = rng.integers(0, 2, nbch, dtype=np.uint8)
    cw = O.LDPC(framesize, rate).work(info, 1)
    p = cw[nbch:].astype(np.int64)
    pb = nldpc - nbch
    syn = p.copy()
    syn[1:] ^= p[:-1]
    for g, addrs in enumerate(T.ldpc_rows(framesize, rate)):
        d = info[360 * g: 360 * g + 360].astype(np.int64)
        for x in addrs:
            idx = (x + np.arange(360) * q) % pb
            np.bitwise_xor.at(syn, idx, d)
    assert not syn.any()


def test_ts_generator_structure_and_slicing():
    a = ts_packets(0, 40)
    assert (a.reshape(-1, 188)[:, 0] == 0x47).all()
    b = ts_packets(17, 5)
    np.testing.assert_array_equal(a[17 * 188:22 * 188], b)
    cfg = CONFIGS["cfg3"]
    buf, base = ts_for_frames(cfg, 3, 2)
    assert base % 188 == 0
    full = ts_packets(0, (base + len(buf)) // 188)
    np.testing.assert_array_equal(full[base:], buf)


@pytest.mark.parametrize("name", ["cfg1", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_oracle_cell_counts_consistent(name):
    """framemapper mapped_items == pilotgen active_items: C_P2/C_DATA/N_FC tables agree with the
    pilot maps, and the interleaver cell counts match"""
    cfg = CONFIGS[name]
    fm = O.FM(*cfg.fm_args())
    pg = O.PG(*cfg.pg_args())
    assert fm.mapped_items == pg.active_items
    assert fm.stream_items == cfg.fecblocks * O.IM(*cfg.im_args()).cell_size


def test_bbheader_hem_and_inband_run():
    cfg = CONFIGS["cfg1"].with_(inputmode=E.INPUTMODE_HIEFF, inband=E.INBAND_ON)
    bb = O.BB(*cfg.bb_args())
    ts = ts_packets(0, 200)
    out, cons = bb.work(ts, 4)
    assert len(out) == 4 * bb.nbch and cons > 0
