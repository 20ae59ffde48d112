"""CPU: TIME_IL_TYPE 1 interleaving frames and sub-sliced Type-2 PLPs (EN 302 755 6.5,
7.2.3.1, 8.3.6.3).  The planner's per-phase gather maps against the oracle's framemapper generalised to
interleaving frames of P_I T2 frames and Type-2 sub-slices, the L1-post fields that signal them, the fused
chain's slot layout, and the consumption / sharding unit.

PARITY UNPINNED: the reference hard-wires plp_type 1, time_il_type 0, frame_interval 1 and
time_il_length = tiblocks (lib/framemapperfint_cc_impl.cc:159, 198-200; serialised at :1581, 1619-1627) and
its time interleaver implements type 0 only (:1999-2028).  Both sides here restate the standard; a one-PLP,
type-0 frame through the same code is the reference's frame (test_cpu_mplp.py)."""
import numpy as np
import pytest

from dvbt2ll.configs import IF_CONFIGS, CONFIGS, mplp_from, _plp, ts_for_frames, ts_packets
from dvbt2ll import distributed as D
import oracle_lib as O
import plan_probe as PP

rng = np.random.default_rng(23)
NAMES = list(IF_CONFIGS)


def _apply(gmap, src, aux):
    return np.where(gmap >= 0, src[np.clip(gmap, 0, None)], aux[np.clip(-gmap - 1, 0, None)]).astype(np.complex64)


def _rand(n):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)


@pytest.mark.parametrize("name", NAMES)
def test_if_frame_matches_oracle(name):
    """two launch units of T2 frames: the planner's gather map of each frame phase, applied to the current
    interleaving frame of every PLP (random cells), equals the oracle framemapper fed the cells each PLP
    consumes (a whole interleaving frame on its first T2 frame, nothing on the others)"""
    m = IF_CONFIGS[name]
    fr = PP.frame_plan_mplp(m)
    fm = O.FMM(m)
    assert fr is not None and fr["unit"] == m.unit_frames
    assert (fr["M"], fr["S"], fr["Lp"]) == (fm.mapped_items, fm.stream_items, fm.l1post_cells)
    cur = [np.zeros(p.fecblocks * c, np.complex64) for p, c in zip(m.plps, fr["cs"])]   # before a PLP's first
    for f in range(2 * fr["unit"]):
        fresh = []
        for k, p in enumerate(m.plps):
            n = fm.consume(k)
            assert n == (p.fecblocks * fr["cs"][k] if p.starts_if(f) else 0)
            if n:
                cur[k] = _rand(n)
                fresh.append(cur[k])
        want = fm.work(np.concatenate(fresh) if fresh else np.zeros(0, np.complex64))
        src = np.concatenate(cur)
        assert len(src) == fr["S_in"]
        got = _apply(fr["gather_in"][f % fr["unit"]], src, fr["aux"][f % m.t2frames])
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg="%s frame %d" % (name, f))


def _field(bits, pos, n):
    return int("".join(str(int(b)) for b in bits[pos:pos + n]), 2)


def _placement(m, frame, per):
    """8.3.6.3 restated independently: the PLPs present in T2 frame `frame` (f mod I_JUMP = FIRST_FRAME_IDX),
    Type-1 runs back to back in PLP_ID order, then the Type-2 sub-slices; returns (present, PLP_START per PLP
    (0 when absent), TYPE_2_START, SUB_SLICE_INTERVAL, cells)"""
    present = [frame % p.frame_interval == p.first_frame_idx for p in m.plps]
    start, cells = [0] * m.nplp, 0
    for k, p in enumerate(m.plps):
        if present[k] and p.plp_type == 1:
            start[k], cells = cells, cells + per[k]
    t2 = [k for k, p in enumerate(m.plps) if present[k] and p.plp_type == 2]
    ssi = 0
    for k in t2:
        start[k] = cells + ssi
        ssi += per[k] // m.num_subslices
    return present, start, (cells if t2 else 0), ssi, cells + ssi * m.num_subslices


@pytest.mark.parametrize("name", NAMES)
def test_if_l1post_fields(name):
    """the L1-post (EN 302 755 7.2.3): SUB_SLICES_PER_FRAME, per PLP PLP_TYPE, PLP_NUM_BLOCKS_MAX,
    FRAME_INTERVAL 1, TIME_IL_LENGTH (P_I for type 1, N_TI for type 0), TIME_IL_TYPE; dynamic
    SUB_SLICE_INTERVAL, TYPE_2_START, PLP_START and PLP_NUM_BLOCKS -- parsed from the planner's signalling
    bits at the standard's field offsets"""
    m = IF_CONFIGS[name]
    fr = PP.frame_plan_mplp(m)
    for fidx in range(m.t2frames):
        bits = PP.l1post_bits_mplp(m, fidx)
        present, start, t2start, ssi, _ = _placement(m, fidx, fr["plp_S"])
        assert _field(bits, 0, 15) == m.num_subslices and _field(bits, 15, 8) == m.nplp
        o = 15 + 8 + 4 + 8 + 3 + 32
        for k, p in enumerate(m.plps):
            assert _field(bits, o, 8) == k                          # PLP_ID
            assert _field(bits, o + 8, 3) == p.plp_type             # PLP_TYPE
            q = o + 8 + 3 + 5 + 1 + 3
            assert _field(bits, q, 8) == p.first_frame_idx          # FIRST_FRAME_IDX
            q += 8 + 8 + 3 + 3 + 1 + 2
            assert _field(bits, q, 10) == p.fecblocks               # PLP_NUM_BLOCKS_MAX
            assert _field(bits, q + 10, 8) == p.frame_interval      # FRAME_INTERVAL
            assert _field(bits, q + 18, 8) == (p.ti_frames if p.ti_type else p.tiblocks)   # TIME_IL_LENGTH
            assert _field(bits, q + 26, 1) == p.ti_type             # TIME_IL_TYPE
            o += 89
        o += 2 + 30
        assert _field(bits, o, 8) == fidx                           # FRAME_IDX
        assert _field(bits, o + 8, 22) == ssi                       # SUB_SLICE_INTERVAL
        assert _field(bits, o + 30, 22) == t2start                  # TYPE_2_START
        o += 8 + 22 + 22 + 8 + 3 + 8
        for k, p in enumerate(m.plps):
            assert _field(bits, o, 8) == k
            assert _field(bits, o + 8, 22) == start[k]             # PLP_START (0 when absent)
            assert _field(bits, o + 30, 10) == (p.fecblocks if present[k] else 0)   # PLP_NUM_BLOCKS
            o += 48


@pytest.mark.parametrize("name", NAMES)
def test_if_geometry(name):
    """8.3.6.3: Type-1 PLPs back to back in PLP_ID order, then the Type-2 PLPs' sub-slices interleaved
    (SUB_SLICE_INTERVAL = the Type-2 cells per frame / N_subslices, TYPE_2_START = the Type-1 cells); a
    TIME_IL_TYPE 1 PLP carries fecblocks x cell size / P_I cells per T2 frame"""
    m = IF_CONFIGS[name]
    fr = PP.frame_plan_mplp(m)
    per = [p.fecblocks * c * p.frame_interval // p.if_frames for p, c in zip(m.plps, fr["cs"])]
    assert fr["plp_S"] == per
    present, start, t2start, ssi, cells = _placement(m, 0, per)   # the frame class of T2 frame 0
    assert fr["start"] == start and fr["t2start"] == t2start and fr["ssi"] == ssi
    assert fr["S"] == max(_placement(m, f, per)[4] for f in range(m.t2frames))


@pytest.mark.parametrize("name", NAMES)
def test_if_chain_layout(name):
    """the fused chain's slot order stays PLP-major in every (symbol, half) group with sub-sliced and
    multi-frame PLPs, and plp_bnd delimits exactly each PLP's slots"""
    m = IF_CONFIGS[name]
    cl = PP.chain_layout_mplp(m)
    fr = cl["frame"]
    P = cl["nplp"]
    present, _, _, _, S = _placement(m, 0, fr["plp_S"])   # class 0's layout
    assert cl["S"] == S
    plp_of_cell = np.full(S, -1, np.int64)
    for k, p in enumerate(m.plps):
        if not present[k]:
            continue
        c = np.arange(fr["plp_S"][k])
        if p.plp_type == 1:
            pos = fr["start"][k] + c
        else:
            ss = fr["plp_S"][k] // m.num_subslices
            pos = fr["start"][k] + (c // ss) * fr["ssi"] + c % ss
        assert np.all(plp_of_cell[pos] == -1)
        plp_of_cell[pos] = k
    assert np.all(plp_of_cell >= 0)
    plp_of_slot = np.zeros(S, np.int64)
    plp_of_slot[cl["part"]] = plp_of_cell
    for j in range(cl["Nsym"]):
        halves = [(cl["d0"][j], cl["d0"][j] + cl["dn0"][j]), (cl["d0"][j] + cl["dn0"][j], cl["d0"][j] + cl["dn"][j])]
        for h, (a, b) in enumerate(halves):
            bnd = cl["bnd"][2 * j + h]
            assert bnd[0] == a and bnd[P] == b
            for k in range(P):
                assert np.all(plp_of_slot[bnd[k]:bnd[k + 1]] == k), (name, j, h, k)


def _bad(m, **plp0):
    import dataclasses
    return m.with_(plps=(dataclasses.replace(m.plps[0], **plp0),) + m.plps[1:])


def test_if_rejects_invalid():
    """create-time validation: TIME_IL_TYPE 1 needs one TI block, P_I dividing the superframe and the
    interleaving frame's cells; TIME_IL_TYPE 0 has P_I = 1; N_subslices needs Type-2 PLPs whose cells per
    frame it divides"""
    m = IF_CONFIGS["ti1_32k_p2"]
    assert PP.frame_plan_mplp(_bad(m, tiblocks=2)) is None                  # type 1 with N_TI = 2
    assert PP.frame_plan_mplp(_bad(m, ti_type=0)) is None                   # type 0 with P_I = 2
    assert PP.frame_plan_mplp(_bad(m, ti_frames=4)) is None                 # t2frames 2 not a multiple of 4
    x = IF_CONFIGS["mix_4k"]
    assert PP.frame_plan_mplp(x) is not None
    assert PP.frame_plan_mplp(_bad(x, fecblocks=3)) is None                 # 3 x 2025 cells odd: P_I = 2 fails
    assert PP.frame_plan_mplp(m.with_(num_subslices=2)) is None             # sub-slices without Type-2 PLPs
    s = IF_CONFIGS["t2sub_32k"]
    assert PP.frame_plan_mplp(s.with_(num_subslices=11)) is None            # 756000 % 11 != 0
    assert PP.frame_plan_mplp(_bad(m, plp_type=3)) is None
    for bad in (_bad(m, tiblocks=2), m.with_(num_subslices=2)):
        plp = np.array([list(p.plp_args()[:8]) + [p.plp_type, p.ti_type, p.ti_frames, p.frame_interval,
                                                   p.first_frame_idx] for p in bad.plps], np.int32).reshape(-1)
        assert not O.lib().orc_fm_create_mplp(bad.nplp, O._p(plp), bad.num_subslices, *bad.common_args())


def test_if_type0_unchanged():
    """a TIME_IL_TYPE 1 PLP with P_I = 1 is the type-0 frame with one TI block except for the TIME_IL_TYPE
    bit: same gather map; and plp_type 2 with one sub-slice and one PLP is the Type-1 frame's geometry"""
    c = CONFIGS["cfg4"]
    a = PP.frame_plan_mplp(mplp_from(c, "a", [_plp(c, tiblocks=1)]))
    b = PP.frame_plan_mplp(mplp_from(c, "b", [_plp(c, tiblocks=1, ti_type=1, ti_frames=1)]))
    np.testing.assert_array_equal(a["gather_in"], b["gather_in"])
    t = PP.frame_plan_mplp(mplp_from(c, "t", [_plp(c, tiblocks=1, plp_type=2)]))
    np.testing.assert_array_equal(a["gather_in"], t["gather_in"])
    assert t["t2start"] == 0 and t["ssi"] == a["S"]


@pytest.mark.parametrize("name", ["ti1_8k_p4", "mix_4k"])
def test_if_ts_slices(name):
    """a run starting at a launch unit needs exactly the global stream's bytes for its interleaving frames
    (ts_for_frames per PLP), and the oracle framemapper seeked to that frame produces the sequential
    run's frames (closed-form state at interleaving-frame starts)"""
    m = IF_CONFIGS[name]
    u = m.unit_frames
    full_cells, _, _ = O.mplp_cells(m, 0, 2 * u)
    tail_cells, _, _ = O.mplp_cells(m, u, u)
    for f in range(u):
        np.testing.assert_array_equal(full_cells[u + f], tail_cells[f])
    for k, p in enumerate(m.plps):
        ts, base = ts_for_frames(p, u, u, seed=k + 1)
        np.testing.assert_array_equal(ts_packets(0, (base + len(ts)) // 188, seed=k + 1)[base:], ts)
    seq, one = O.FMM(m), O.FMM(m)
    want = [seq.work(c) for c in full_cells][u:]
    one.seek(u)
    for f in range(u):
        np.testing.assert_array_equal(one.work(tail_cells[f]).view(np.uint32), want[f].view(np.uint32))


def test_frame_range_units():
    """shards are whole launch units (interleaving frames) and cover every frame once"""
    for total in (0, 4, 8, 12, 20):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                f, c = D.frame_range(total, r, world, first_frame=8, unit=4)
                assert f % 4 == 0 and c % 4 == 0
                seen += list(range(f, f + c))
            assert seen == list(range(8, 8 + total))
    with pytest.raises(ValueError):
        D.frame_range(6, 0, 2, unit=4)
