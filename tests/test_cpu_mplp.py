"""CPU: multi-PLP frames (EN 302 755 8.3.6.3).  The planner's composed gather map
of a frame carrying several Type-1 data PLPs against the oracle's framemapper generalised to several PLPs
(orc_fm_create_mplp), and the fused chain's PLP-major slot layout.

PARITY UNPINNED: the reference carries exactly one PLP (lib/framemapperfint_cc_impl.cc:152-250, serialised
at :1553-1691); both sides restate EN 302 755's PLP loops of the L1-post and its sequential Type-1 PLP
mapping.  With one PLP the same code paths reproduce the committed single-PLP goldens
(test_cpu_golden.py) and every single-PLP planner check (test_cpu_plan.py)."""
import numpy as np
import pytest

from dvbt2ll.configs import MPLP_CONFIGS, CONFIGS, mplp_from, _plp
import oracle_lib as O
import plan_probe as PP

rng = np.random.default_rng(11)
NAMES = list(MPLP_CONFIGS)


def _apply(gmap, src, aux):
    return np.where(gmap >= 0, src[np.clip(gmap, 0, None)], aux[np.clip(-gmap - 1, 0, None)]).astype(np.complex64)


@pytest.mark.parametrize("name", NAMES)
def test_mplp_frame_matches_oracle(name):
    """every mapped cell of the frame (L1-pre, L1-post with the PLP loops, each PLP's cell + time
    interleaved cells at its PLP_START, dummy cells, frequency interleaving) for consecutive
    t2_frame_num values"""
    m = MPLP_CONFIGS[name]
    fr = PP.frame_plan_mplp(m)
    fm = O.FMM(m)
    assert fr is not None
    assert (fr["M"], fr["S"], fr["Lp"]) == (fm.mapped_items, fm.stream_items, fm.l1post_cells)
    # PLPs back to back after the L1 signalling, PLP_ID order
    starts = np.cumsum([0] + [p.fecblocks * c for p, c in zip(m.plps, fr["cs"])])[:-1]
    assert fr["start"] == list(starts)
    for f in range(min(3, m.t2frames + 1)):
        cells = (rng.standard_normal(fr["S"]) + 1j * rng.standard_normal(fr["S"])).astype(np.complex64)
        want = fm.work(cells)
        got = _apply(fr["gather_in"][0], cells, fr["aux"][f % m.t2frames])
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32), err_msg="%s frame %d" % (name, f))


@pytest.mark.parametrize("name", NAMES)
def test_mplp_l1post_size(name):
    """K_sig = 350 + 137 (nplp - 1) L1-post signalling bits (89 configurable + 48 dynamic per PLP,
    framemapper:1577-1639, 1672-1687); N_post from framemapper:978-987 with that K_sig"""
    m = MPLP_CONFIGS[name]
    cells, info = PP.l1post_mplp(m, 1)
    assert info["nsig"] == 350 + 137 * (m.nplp - 1)
    assert info["Lp"] == O.FMM(m).l1post_cells == len(cells)


def test_one_plp_is_the_reference_frame():
    """a one-PLP 'multi-PLP' frame is the reference's single-PLP frame, cell for cell (planner and oracle)"""
    c = CONFIGS["cfg1"]
    m = mplp_from(c, "one", [_plp(c)])
    fr1 = PP.frame_plan(c.fm_args())
    frm = PP.frame_plan_mplp(m)
    np.testing.assert_array_equal(fr1["gather_in"], frm["gather_in"][0])
    np.testing.assert_array_equal(fr1["aux"].view(np.uint32), frm["aux"].view(np.uint32))
    cells = (rng.standard_normal(fr1["S"]) + 1j * rng.standard_normal(fr1["S"])).astype(np.complex64)
    np.testing.assert_array_equal(O.FM(*c.fm_args()).work(cells).view(np.uint32), O.FMM(m).work(cells).view(np.uint32))


@pytest.mark.parametrize("name", NAMES)
def test_mplp_chain_layout(name):
    """the fused chain's slot order: every (symbol, half) group's data slots are PLP-major, and the
    boundaries plp_bnd the OFDM kernel selects each PLP's constellation by delimit exactly the slots whose
    data cells lie in [PLP_START, PLP_START + S) of that PLP"""
    m = MPLP_CONFIGS[name]
    cl = PP.chain_layout_mplp(m)
    fr = cl["frame"]
    P, S = cl["nplp"], cl["S"]
    plp_of_cell = np.zeros(S, np.int64)
    for k in range(P):
        plp_of_cell[fr["start"][k]:fr["start"][k] + fr["cs"][k] * fr["F"][k]] = k
    # part: TI output (data cell) index -> slot; slot -> PLP of its cell
    plp_of_slot = np.zeros(S, np.int64)
    plp_of_slot[cl["part"]] = plp_of_cell
    assert sorted(cl["part"].tolist()) == list(range(S))
    for j in range(cl["Nsym"]):
        halves = [(cl["d0"][j], cl["d0"][j] + cl["dn0"][j]), (cl["d0"][j] + cl["dn0"][j], cl["d0"][j] + cl["dn"][j])]
        for h, (a, b) in enumerate(halves):
            bnd = cl["bnd"][2 * j + h]
            assert bnd[0] == a and bnd[P] == b and np.all(np.diff(bnd) >= 0)
            for k in range(P):
                assert np.all(plp_of_slot[bnd[k]:bnd[k + 1]] == k), (name, j, h, k)


def test_mplp_oracle_bbheader_mis():
    """MIS BBHEADER of a PLP (bbheader:288-298): MATYPE-1 SIS/MIS bit 0, MATYPE-2 = ISI, CRC-8 over it"""
    c = CONFIGS["cfg1"]
    from dvbt2ll.configs import ts_for_frames
    ts, _ = ts_for_frames(c, 0, 1)
    sis, _ = O.BB(*c.bb_args()).work(ts, 1)
    mis, _ = O.BB(*c.bb_args(), isi=5).work(ts, 1)
    prbs = np.zeros(80, np.uint8)
    O.lib().orc_bb_prbs(O._p(prbs), 80)
    hs, hm = sis[:80] ^ prbs, mis[:80] ^ prbs          # descrambled headers
    assert hs[2] == 1 and hm[2] == 0                    # SIS / MIS
    assert hs[8:16].tolist() == [0] * 8 and hm[8:16].tolist() == [0, 0, 0, 0, 0, 1, 0, 1]   # ISI = 5
    np.testing.assert_array_equal(hs[16:72], hm[16:72])
    # CRC-8 (poly 0xAB, LSB-first register) over the 72 header bits, written LSB first
    def crc8(bits):
        crc = 0
        for b in bits:
            x = int(b) ^ (crc & 1)
            crc >>= 1
            if x:
                crc ^= 0xAB
        return [(crc >> n) & 1 for n in range(8)]
    assert hm[72:80].tolist() == crc8(hm[:72]) and hs[72:80].tolist() == crc8(hs[:72])
