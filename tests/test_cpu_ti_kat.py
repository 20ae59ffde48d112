"""CPU known-answer tests for the standard-only placements (verdict r5 item 7): TIME_IL_TYPE 1 (EN 302 755 6.5),
FRAME_INTERVAL / FIRST_FRAME_IDX (7.2.3.1) and sub-sliced Type-2 PLPs (8.3.6.3), with the L1-post fields that
signal them (7.2.3.1 / 7.2.3.2, Tables 14-15).

The planner (t2_plan.cpp) and the oracle (oracle/dvbt2_oracle.c) restate these clauses from the same reading, so
test_cpu_ti.py, which compares them with each other, cannot catch a misreading they share.  Here the expected
values are written out by hand, for three small configurations on the GRC's 4K short frame (cfg1: 16200 data
cells per T2 frame), as literal index lists, cell counts and bit strings:
  - which data cells of each T2 frame carry which PLP, and which FEC block each cell comes from;
  - the TI output range each T2 frame carries (D = N_FEC x N_cells / P_I cells per frame, in order);
  - the L1-post field values.
The one thing not written out by hand is the cell interleaver's pseudo-random permutation.  That is the
reference's own (framemapper:1973-1998, identical for TIME_IL_TYPE 0).  It is read from an ANCHOR: the same PLP
alone in a one-PLP TIME_IL_TYPE 0 frame, the reference's configuration.  The anchor's data cell d is TI output
cell d of the PLP's interleaving frame.  Every check runs against both the planner and the oracle.

PARITY UNPINNED beyond these hand-derived values: the reference implements one Type-1 TIME_IL_TYPE 0 PLP only
(lib/framemapperfint_cc_impl.cc:159, 198-200)."""
import numpy as np
import pytest

from dvbt2ll import enums as E
from dvbt2ll.configs import CONFIGS, mplp_from, _plp
import oracle_lib as O
import plan_probe as PP

C1 = CONFIGS["cfg1"]   # 4K, 16200 data cells per T2 frame (the GRC's frame)


def _p16(**kw):   # one 16-QAM 3/5 short FEC block = 4050 cells (EN 302 755 Table 13: 16200 / 4)
    d = dict(framesize=E.FECFRAME_SHORT, rate=E.C3_5, constellation=E.MOD_16QAM, rotation=E.ROTATION_OFF,
             fecblocks=1, tiblocks=1, inputmode=E.INPUTMODE_NORMAL, inband=E.INBAND_OFF)
    d.update(kw)
    return _plp(C1, **d)


def _pq(**kw):    # one QPSK 1/2 short FEC block = 8100 cells
    return _p16(rate=E.C1_2, constellation=E.MOD_QPSK, **kw)


# KAT A: TIME_IL_TYPE 1, one TI block of 2 FEC blocks (16-QAM short: N_cells 4050) over P_I = 4 T2 frames
KAT_A = mplp_from(C1, "kat-ti1-PI4", [_p16(fecblocks=2, ti_type=1, ti_frames=4)]).with_(t2frames=4)
# KAT B: FRAME_INTERVAL: X in every T2 frame, Y (I_JUMP 3, FIRST_FRAME_IDX 1) in frames 1, 4, ..
KAT_B = mplp_from(C1, "kat-ijump3", [_p16(), _pq(frame_interval=3, first_frame_idx=1)]).with_(t2frames=6)
# KAT C: a Type-1 QPSK PLP, then two Type-2 16-QAM PLPs in 3 sub-slices (fills the 16200 cells exactly)
KAT_C = mplp_from(C1, "kat-type2x3", [_pq(), _p16(plp_type=2), _p16(plp_type=2)]).with_(num_subslices=3)


def _anchor(p):
    """the PLP alone in a one-PLP TIME_IL_TYPE 0 / FRAME_INTERVAL 1 / Type-1 frame (the reference's frame): data
    cell d -> the PLP's interleaving-frame input index, for d < N_FEC x N_cells (TI output order)"""
    import dataclasses
    a = mplp_from(C1, "anchor", [dataclasses.replace(p, plp_type=1, ti_type=0, ti_frames=1, frame_interval=1,
                                                     first_frame_idx=0)])
    src = _planner_sources(a, 1)[0]
    n = p.fecblocks * (4050 if p.constellation == E.MOD_16QAM else 8100)
    assert np.all(src[:n] >= 0) and np.all(src[n:] < 0)
    np.testing.assert_array_equal(np.sort(src[:n]), np.arange(n))   # a permutation of the interleaving frame
    np.testing.assert_array_equal(_oracle_sources(a, 1)[0][0], src)
    return src[:n]


def _region(fr):
    """output position of the framemapper -> data-region index (data or dummy cell), -1 for L1 / zero cells;
    from frame class 0's gather map (its dummy codes count on from S_0)"""
    gd = fr["gather_d"]
    aux_dummy = fr["aux_len"] - fr["D"]   # AUX_L1PRE + 1840 + Lp: the first dummy code
    S0 = int((gd >= 0).sum())
    c = -gd - 1
    dummy = (gd < 0) & (c >= aux_dummy) & (c < aux_dummy + fr["D"])
    return np.where(gd >= 0, gd, np.where(dummy, S0 + c - aux_dummy, -1))


def _planner_sources(m, nframes):
    """[nframes, data region]: the input index (into the concatenated current interleaving frames of the PLPs,
    PLP k at in_off[k]) each data-region cell carries, -1 for a dummy cell"""
    fr = PP.frame_plan_mplp(m)
    reg = _region(fr)
    n = int(reg.max()) + 1
    out = np.full((nframes, n), -2, np.int64)
    for f in range(nframes):
        g = fr["gather_in"][f % fr["unit"]]
        sel = reg >= 0
        out[f, reg[sel]] = np.where(g[sel] >= 0, g[sel], -1)
    assert (out > -2).all()
    return out


def _oracle_sources(m, nframes):
    """the same read from the oracle framemapper's output: PLP k's consumed cells are coded as in_off[k] + j + 1
    (real) and 1000 + the PLP's interleaving-frame count (imag); returns (sources, interleaving-frame index)"""
    fr = PP.frame_plan_mplp(m)
    reg = _region(fr)
    n = int(reg.max()) + 1
    fm = O.FMM(m)
    ifs = [0] * m.nplp
    src = np.full((nframes, n), -2, np.int64)
    ifm = np.full((nframes, n), -1, np.int64)
    consumed = []
    for f in range(nframes):
        fresh, row = [], []
        for k in range(m.nplp):
            c = fm.consume(k)
            row.append(c)
            if c:
                j = np.arange(c)
                fresh.append((fr["in_off"][k] + j + 1).astype(np.float32) + 1j * np.float32(1000 + ifs[k]))
                ifs[k] += 1
        consumed.append(row)
        out = fm.work(np.concatenate(fresh).astype(np.complex64) if fresh else np.zeros(0, np.complex64))
        sel = reg >= 0
        v = out[sel]
        coded = v.imag >= 1000
        src[f, reg[sel]] = np.where(coded, np.rint(v.real).astype(np.int64) - 1, -1)
        ifm[f, reg[sel]] = np.where(coded, np.rint(v.imag).astype(np.int64) - 1000, -1)
    assert (src > -2).all()
    return src, ifm, consumed


# EN 302 755 Table 14 (L1-post configurable: the per-PLP loop) and Table 15 (L1-post dynamic), in bits
CONF_HEAD = [("SUB_SLICES_PER_FRAME", 15), ("NUM_PLP", 8), ("NUM_AUX", 4), ("AUX_CONFIG_RFU", 8), ("RF_IDX", 3),
             ("FREQUENCY", 32)]
CONF_PLP = [("PLP_ID", 8), ("PLP_TYPE", 3), ("PLP_PAYLOAD_TYPE", 5), ("FF_FLAG", 1), ("FIRST_RF_IDX", 3),
            ("FIRST_FRAME_IDX", 8), ("PLP_GROUP_ID", 8), ("PLP_COD", 3), ("PLP_MOD", 3), ("PLP_ROTATION", 1),
            ("PLP_FEC_TYPE", 2), ("PLP_NUM_BLOCKS_MAX", 10), ("FRAME_INTERVAL", 8), ("TIME_IL_LENGTH", 8),
            ("TIME_IL_TYPE", 1), ("IN_BAND_A_FLAG", 1), ("IN_BAND_B_FLAG", 1), ("RESERVED_1", 11), ("PLP_MODE", 2),
            ("STATIC_FLAG", 1), ("STATIC_PADDING_FLAG", 1)]
CONF_TAIL = [("FEF_LENGTH_MSB", 2), ("RESERVED_2", 30)]
DYN_HEAD = [("FRAME_IDX", 8), ("SUB_SLICE_INTERVAL", 22), ("TYPE_2_START", 22), ("L1_CHANGE_COUNTER", 8),
            ("START_RF_IDX", 3), ("RESERVED_1", 8)]
DYN_PLP = [("PLP_ID", 8), ("PLP_START", 22), ("PLP_NUM_BLOCKS", 10), ("RESERVED_2", 8)]


def _parse(bits, nplp):
    """L1-post bits -> (configurable head, [per PLP], dynamic head, [per PLP]) as bit strings"""
    s = "".join(str(int(b)) for b in bits)
    pos = 0

    def take(fields):
        nonlocal pos
        d = {}
        for name, n in fields:
            d[name] = s[pos:pos + n]
            pos += n
        return d
    ch = take(CONF_HEAD)
    cp = [take(CONF_PLP) for _ in range(nplp)]
    take(CONF_TAIL)
    dh = take(DYN_HEAD)
    dp = [take(DYN_PLP) for _ in range(nplp)]
    take([("RESERVED_3", 8)])
    assert pos == len(s)
    return ch, cp, dh, dp


def _l1_both(m, frame):
    """the L1-post signalling bits of T2 frame `frame` from the planner and from the oracle (equal), parsed"""
    a = PP.l1post_bits_mplp(m, frame % m.t2frames)
    b = O.FMM(m).l1post_bits(frame)
    np.testing.assert_array_equal(a, b)
    return _parse(a, m.nplp)


def _both(m, nframes):
    ps = _planner_sources(m, nframes)
    os_, ifm, consumed = _oracle_sources(m, nframes)
    np.testing.assert_array_equal(ps, os_)
    return ps, ifm, consumed


def test_kat_ti_type1_cells():
    """6.5, TIME_IL_TYPE 1, P_I = 4: the TI block (N_FEC = 2 FEC blocks of N_cells = 4050, written column-wise
    into N_r = 4050 / 5 = 810 rows x N_c = 5 x 2 = 10 columns, read row-wise) is spread in order over the P_I T2
    frames of its interleaving frame: T2 frame i carries TI output cells [i D, (i + 1) D), D = 2 x 4050 / 4 =
    2025, at data cells [0, 2025); the rest of the 16200 are dummy cells.  D / N_c = 202.5 rows, so frames 1 and
    3 start in the middle of a TI row, with block 1's five cells"""
    m = KAT_A
    anchor = _anchor(m.plps[0])
    src, ifm, consumed = _both(m, 8)
    assert consumed == [[8100], [0], [0], [0], [8100], [0], [0], [0]]      # the whole interleaving frame on frame 0 of 4
    D = 2025
    for f in range(8):
        i = f % 4
        assert np.all(src[f, :D] >= 0) and np.all(src[f, D:] == -1), f
        assert np.all(ifm[f, :D] == f // 4)
        np.testing.assert_array_equal(src[f, :D], anchor[i * D:(i + 1) * D], err_msg="frame %d" % f)
    blk = src // 4050                                                        # FEC block of each cell
    assert blk[0, :15].tolist() == [0] * 5 + [1] * 5 + [0] * 5
    assert blk[1, :15].tolist() == [1] * 5 + [0] * 5 + [1] * 5               # row 202, columns 5..9 first
    assert blk[2, :15].tolist() == [0] * 5 + [1] * 5 + [0] * 5
    assert blk[3, :15].tolist() == [1] * 5 + [0] * 5 + [1] * 5
    assert blk[3, D - 5:D].tolist() == [1] * 5                               # TI output 8095..8099: row 809
    for f, want in enumerate([[1015, 1010], [1010, 1015], [1015, 1010], [1010, 1015]]):
        assert np.bincount(blk[f, :D], minlength=2).tolist() == want


def test_kat_ti_type1_l1post():
    """7.2.3.1: TIME_IL_TYPE = 1 and TIME_IL_LENGTH = P_I = 4; PLP_NUM_BLOCKS = PLP_NUM_BLOCKS_MAX = 2 (the FEC
    blocks of the interleaving frame) in all four T2 frames; FRAME_INTERVAL 1, PLP_START 0"""
    for f in range(4):
        ch, cp, dh, dp = _l1_both(KAT_A, f)
        assert ch["SUB_SLICES_PER_FRAME"] == "000000000000001" and ch["NUM_PLP"] == "00000001"
        assert cp[0]["PLP_TYPE"] == "001"
        assert cp[0]["TIME_IL_TYPE"] == "1" and cp[0]["TIME_IL_LENGTH"] == "00000100"
        assert cp[0]["FRAME_INTERVAL"] == "00000001" and cp[0]["FIRST_FRAME_IDX"] == "00000000"
        assert cp[0]["PLP_NUM_BLOCKS_MAX"] == "0000000010"
        assert dh["FRAME_IDX"] == ["00000000", "00000001", "00000010", "00000011"][f]
        assert dp[0]["PLP_START"] == "0" * 22 and dp[0]["PLP_NUM_BLOCKS"] == "0000000010"
        assert dh["SUB_SLICE_INTERVAL"] == "0" * 22 and dh["TYPE_2_START"] == "0" * 22


def test_kat_frame_interval_cells():
    """7.2.3.1 / 8.3.6.3, FRAME_INTERVAL: X (4050 cells) is in every T2 frame at [0, 4050); Y (I_JUMP = 3,
    FIRST_FRAME_IDX = 1, 8100 cells) only in the frames with FRAME_IDX mod 3 = 1, i.e. 1 and 4 of the superframe
    of 6, right after X at [4050, 12150); in frames 0, 2, 3, 5 those cells are dummy cells.  Each present frame
    takes a new interleaving frame of Y"""
    m = KAT_B
    ax, ay = _anchor(m.plps[0]), _anchor(m.plps[1])
    src, ifm, consumed = _both(m, 6)
    assert consumed == [[4050, 0], [4050, 8100], [4050, 0], [4050, 0], [4050, 8100], [4050, 0]]
    off_y = 4050   # in_off of Y: after X's interleaving frame
    for f in range(6):
        np.testing.assert_array_equal(src[f, :4050], ax)
        assert np.all(ifm[f, :4050] == f)
        if f in (1, 4):
            np.testing.assert_array_equal(src[f, 4050:12150], off_y + ay)
            assert np.all(ifm[f, 4050:12150] == (0 if f == 1 else 1))
        else:
            assert np.all(src[f, 4050:] == -1), f
        assert np.all(src[f, 12150:] == -1)


def test_kat_frame_interval_l1post():
    """7.2.3.1: Y signals FIRST_FRAME_IDX 1 and FRAME_INTERVAL 3; PLP_START = 4050 and PLP_NUM_BLOCKS = 1 in the
    frames that carry it, PLP_START = PLP_NUM_BLOCKS = 0 in the others; X: PLP_START 0, PLP_NUM_BLOCKS 1"""
    for f in range(6):
        ch, cp, dh, dp = _l1_both(KAT_B, f)
        assert ch["NUM_PLP"] == "00000010"
        assert cp[0]["FRAME_INTERVAL"] == "00000001" and cp[0]["FIRST_FRAME_IDX"] == "00000000"
        assert cp[1]["FRAME_INTERVAL"] == "00000011" and cp[1]["FIRST_FRAME_IDX"] == "00000001"
        assert cp[1]["TIME_IL_TYPE"] == "0" and cp[1]["TIME_IL_LENGTH"] == "00000001"
        assert cp[1]["PLP_NUM_BLOCKS_MAX"] == "0000000001"
        assert dp[0]["PLP_ID"] == "00000000" and dp[1]["PLP_ID"] == "00000001"
        assert dp[0]["PLP_START"] == "0" * 22 and dp[0]["PLP_NUM_BLOCKS"] == "0000000001"
        if f in (1, 4):
            assert dp[1]["PLP_START"] == "0000000000111111010010"          # 4050
            assert dp[1]["PLP_NUM_BLOCKS"] == "0000000001"
        else:
            assert dp[1]["PLP_START"] == "0" * 22 and dp[1]["PLP_NUM_BLOCKS"] == "0000000000"


# KAT C's data region, by hand (8.3.6.3): TYPE_2_START = 8100 (the Type-1 cells), each Type-2 PLP's 4050 cells
# cut into 3 sub-slices of 1350, SUB_SLICE_INTERVAL = 1350 + 1350 = 2700: (PLP, first cell, end) in cell order
KAT_C_RUNS = [(0, 0, 8100),
              (1, 8100, 9450), (2, 9450, 10800),
              (1, 10800, 12150), (2, 12150, 13500),
              (1, 13500, 14850), (2, 14850, 16200)]


def test_kat_type2_subslices_cells():
    """8.3.6.3: the Type-1 PLP first, then sub-slice 0 of every Type-2 PLP in PLP_ID order, sub-slice 1, ..;
    each Type-2 PLP's TI output is cut in order: sub-slice s carries its cells [1350 s, 1350 (s + 1))"""
    m = KAT_C
    anchors = [_anchor(p) for p in m.plps]
    src, _, consumed = _both(m, 2)
    assert consumed == [[8100, 4050, 4050], [8100, 4050, 4050]]
    in_off = [0, 8100, 12150]
    seen = [0, 0, 0]
    for k, a, b in KAT_C_RUNS:
        n = b - a
        for f in range(2):
            np.testing.assert_array_equal(src[f, a:b], in_off[k] + anchors[k][seen[k]:seen[k] + n],
                                          err_msg="PLP %d cells [%d, %d)" % (k, a, b))
        seen[k] += n
    assert seen == [8100, 4050, 4050] and src.shape[1] == 16200


def test_kat_type2_subslices_l1post():
    """7.2.3.1 / 7.2.3.2: SUB_SLICES_PER_FRAME 3, PLP_TYPE 001 / 010 / 010, SUB_SLICE_INTERVAL 2700, TYPE_2_START
    8100, PLP_START 0 / 8100 / 9450 (a Type-2 PLP's start is its first sub-slice)"""
    for f in range(2):
        ch, cp, dh, dp = _l1_both(KAT_C, f)
        assert ch["SUB_SLICES_PER_FRAME"] == "000000000000011" and ch["NUM_PLP"] == "00000011"
        assert [p["PLP_TYPE"] for p in cp] == ["001", "010", "010"]
        assert dh["SUB_SLICE_INTERVAL"] == "0000000000101010001100"         # 2700
        assert dh["TYPE_2_START"] == "0000000001111110100100"               # 8100
        assert [p["PLP_START"] for p in dp] == ["0" * 22,
                                                "0000000001111110100100",   # 8100
                                                "0000000010010011101010"]   # 9450
        assert [p["PLP_NUM_BLOCKS"] for p in dp] == ["0000000001"] * 3
