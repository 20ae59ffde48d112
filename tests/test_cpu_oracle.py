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


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
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


# ---------------------------------------------------------------- independent cross-checks of the
# extracted tables (the oracle and the product share tools/extract_tables.py's header, so an
# extraction error would be common-mode; these tie it to data extracted from elsewhere)

def _pilot_combos():
    """every (FFT size, pilot pattern, carrier mode, PAPR, preamble) the framemapper's cell-count
    table accepts, with one guard interval per distinct frame-closing (N_FC) behaviour"""
    import plan_probe as PP
    seen = {}
    for fft in (0, 1, 2, 3, 4, 5, 6, 7, 11):
        for pp in range(8):
            for car in (0, 1):
                for papr in range(4):
                    for gi in range(7):
                        for pre in (0, 1, 3, 4):
                            c = PP.cell_counts(fft, car, pp, papr, gi, pre)
                            if c and c["C_DATA"] > 0:
                                seen.setdefault((fft, pp, car, papr, pre, c["N_FC"] > 0), (gi, c))
    return sorted(seen.items())


@pytest.mark.parametrize("fft", [0, 1, 2, 3, 4, 5, 6, 7, 11])
def test_pilot_maps_match_cell_count_tables(fft):
    """For every accepted combination: the data carriers per symbol of the oracle's pilot maps
    (pilotgen:1285-2782, from the pilot-position tables :2909-3505) and of the product planner's
    maps equal C_P2 for the P2 symbols, C_DATA for data symbols and N_FC for the frame-closing
    symbol -- the framemapper's own tables (framemapper:290-356, 425-915), extracted separately.
    The data cells fill the carriers in input order."""
    import plan_probe as PP
    from dvbt2ll.configs import FFT_POINTS
    nds = 3
    for (f, pp, car, papr, pre, _), (gi, c) in _pilot_combos():
        if f != fft:
            continue
        args = (car, f, pp, gi, nds, papr, 0, pre, 0, 0, 3, FFT_POINTS[f])
        want = [c["C_P2"]] * c["N_P2"] + [c["C_DATA"]] * (nds - (1 if c["N_FC"] else 0)) + \
               ([c["N_FC"]] if c["N_FC"] else [])
        plan = PP.pilot_plan(args)
        got = list((plan["bin_map"] >= 0).sum(axis=1))
        assert got == want, (args, got, want)
        pg = O.PG(*args)
        active = pg.active_items
        assert active == sum(want)
        cells = (np.arange(active, dtype=np.float32) + 1.0) + 1j * np.float32(4321.0)
        car_ = pg.carriers(cells.astype(np.complex64))
        mark = car_.imag == np.float32(4321.0)
        assert list(mark.sum(axis=1)) == want, (args, list(mark.sum(axis=1)), want)
        np.testing.assert_array_equal(car_.real[mark], np.arange(active, dtype=np.float32) + 1.0)


# LDPC edge counts from the DVB-S2/T2 degree distributions (EN 302 307 table 7a, EN 302 755 table
# A.1): normal frames have q * 360 parity bits and info-bit degrees {high, 3}
LDPC_EDGES = {(1, 0): 12960 * 8 + 19440 * 3, (1, 1): 12960 * 12 + 25920 * 3, (1, 2): 4320 * 13 + 38880 * 3,
              (1, 3): 5400 * 12 + 43200 * 3, (1, 4): 6480 * 11 + 45360 * 3, (1, 5): 5400 * 13 + 48600 * 3,
              (0, 4): 12600 * 3}


@pytest.mark.parametrize("framesize,rate", [(1, r) for r in range(6)] + [(0, r) for r in range(8)])
def test_ldpc_table_structure(framesize, rate):
    """the extracted LDPC tables have the standard's shape: k/360 rows (one per info group), every
    row of one of two degrees with the low degree 3, entries < nldpc - k, and the known edge
    counts (e.g. 3/5 normal 233,280; 4/5 short 37,800)"""
    import plan_probe as PP
    f = PP.fec_plan(framesize, rate)
    nldpc = 64800 if framesize else 16200
    k = f["nbch"]
    q = f["q"]
    assert q * 360 == nldpc - k
    ent = f["ent"]
    groups = ent >> 16
    deg = np.bincount(groups, minlength=k // 360)
    assert len(deg) == k // 360
    degs = set(deg.tolist())
    assert 3 in degs and len(degs - {3}) <= 1, degs
    assert (ent & 0xFFFF).max() < 360
    edges = int(deg.sum()) * 360
    if (framesize, rate) in LDPC_EDGES:
        assert edges == LDPC_EDGES[(framesize, rate)]


def test_extracted_tables_match_reference():
    """tools/extract_tables.py re-run on the reference tree reproduces the committed generated
    header byte for byte (build container only: the reference does not travel)"""
    import subprocess
    import sys
    from pathlib import Path
    ref = Path("/root/reference")
    if not (ref / "lib").is_dir():
        pytest.skip("reference tree not present")
    root = Path(__file__).resolve().parents[1]
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        out = Path(d) / "t.h"
        subprocess.run([sys.executable, str(root / "tools" / "extract_tables.py"), str(ref), str(out)], check=True)
        assert out.read_bytes() == (root / "gr-dvbt2ll_amd" / "csrc" / "gen" / "dvbt2_std_tables.h").read_bytes()
