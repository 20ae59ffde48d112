"""CPU: the product's host planner (composed gather maps, L1/dummy/pilot tables, LDPC
schedule) against the oracle, across the parameter space.  No GPU needed."""
import itertools

import numpy as np
import pytest

from dvbt2ll import enums as E
from dvbt2ll.configs import CONFIGS, T2Config
import oracle_lib as O
import plan_probe as PP
import std_tables as T

rng = np.random.default_rng(7)


def rand_cells(n):
    return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)


def fitting_fecblocks(cfg):
    """largest fecblocks the frame can carry (the reference warns and overflows beyond it)"""
    lo, hi = 1, 4000
    if PP.frame_plan(cfg.with_(fecblocks=1, tiblocks=min(cfg.tiblocks, 1)).fm_args()) is None:
        return None
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if PP.frame_plan(cfg.with_(fecblocks=mid, tiblocks=min(cfg.tiblocks, mid)).fm_args()) is None:
            hi = mid - 1
        else:
            lo = mid
    return lo


def _apply(gmap, src, aux):
    out = np.where(gmap >= 0, src[np.clip(gmap, 0, None)], aux[np.clip(-gmap - 1, 0, None)])
    return out.astype(np.complex64)


BASE = CONFIGS["cfg1"]
BENCH_CFGS = ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"]
GRID = [
    # (name, overrides)
    ("4k_grc", {}),
    ("4k_l1bpsk", dict(l1constellation=E.L1_MOD_BPSK)),
    ("4k_l1qpsk_ti0", dict(l1constellation=E.L1_MOD_QPSK, tiblocks=0)),
    ("4k_l1_16qam_pp2", dict(l1constellation=E.L1_MOD_16QAM, pilotpattern=E.PILOT_PP2, guardinterval=E.GI_1_8)),
    ("2k_pp3_qpsk_short", dict(fftsize=E.FFTSIZE_2K, pilotpattern=E.PILOT_PP3, constellation=E.MOD_QPSK, rate=E.C1_3,
                               guardinterval=E.GI_1_4, numdatasyms=6)),
    ("1k_pp1_16qam", dict(fftsize=E.FFTSIZE_1K, pilotpattern=E.PILOT_PP1, constellation=E.MOD_16QAM, rate=E.C2_5,
                          guardinterval=E.GI_1_8, numdatasyms=8)),
    ("8k_pp8_ext_64qam", dict(fftsize=E.FFTSIZE_8K, pilotpattern=E.PILOT_PP8, carriermode=E.CARRIERS_EXTENDED,
                              constellation=E.MOD_64QAM, guardinterval=E.GI_1_128, numdatasyms=4)),
    ("8k_pp2_miso_tx2", dict(fftsize=E.FFTSIZE_8K, pilotpattern=E.PILOT_PP2, preamble=E.PREAMBLE_T2_MISO,
                             misogroup=E.MISO_TX2, guardinterval=E.GI_1_8, numdatasyms=5)),
    ("16k_pp5_tr", dict(fftsize=E.FFTSIZE_16K, pilotpattern=E.PILOT_PP5, paprmode=E.PAPR_TR, numdatasyms=3,
                        guardinterval=E.GI_1_8)),
    ("16k_pp6_ext_v131", dict(fftsize=E.FFTSIZE_16K, pilotpattern=E.PILOT_PP6, carriermode=E.CARRIERS_EXTENDED,
                              version=E.VERSION_131, l1scrambled=E.L1_SCRAMBLED_ON, reservedbiasbits=E.RESERVED_ON,
                              numdatasyms=3, guardinterval=E.GI_1_32)),
    ("32k_pp4_ext_cfg3like", dict(fftsize=E.FFTSIZE_32K, pilotpattern=E.PILOT_PP4, carriermode=E.CARRIERS_EXTENDED,
                                  guardinterval=E.GI_1_16, numdatasyms=3, framesize=E.FECFRAME_NORMAL, rate=E.C3_5)),
    ("32k_pp2_miso_tx2_tr", dict(fftsize=E.FFTSIZE_32K, pilotpattern=E.PILOT_PP2, preamble=E.PREAMBLE_T2_MISO,
                                 misogroup=E.MISO_TX2, paprmode=E.PAPR_TR, guardinterval=E.GI_1_8, numdatasyms=3,
                                 framesize=E.FECFRAME_NORMAL, rate=E.C2_3)),
    ("32k_pp7_eq", dict(fftsize=E.FFTSIZE_32K, pilotpattern=E.PILOT_PP7, guardinterval=E.GI_1_128, numdatasyms=2,
                        equalization=E.EQUALIZATION_ON, bandwidth=E.BANDWIDTH_6_0_MHZ, framesize=E.FECFRAME_NORMAL,
                        rate=E.C5_6)),
    ("8k_t2gi_pp4_tr_ext", dict(fftsize=E.FFTSIZE_8K_T2GI, pilotpattern=E.PILOT_PP4, paprmode=E.PAPR_BOTH,
                                carriermode=E.CARRIERS_EXTENDED, guardinterval=E.GI_19_256, numdatasyms=4)),
    # P1 preamble variants the reference accepts (pilotgen:54-56, 295, 898): T2-Lite SISO / MISO
    ("8k_t2lite_siso", dict(fftsize=E.FFTSIZE_8K, preamble=E.PREAMBLE_T2_LITE_SISO, pilotpattern=E.PILOT_PP4,
                            guardinterval=E.GI_1_16, numdatasyms=4)),
    ("4k_t2lite_miso_tx2", dict(preamble=E.PREAMBLE_T2_LITE_MISO, misogroup=E.MISO_TX2, pilotpattern=E.PILOT_PP3,
                                guardinterval=E.GI_1_8)),
    # SURVEY 8(f) rank 2 through the fused chain: high-efficiency mode, in-band type B signalling
    ("4k_hem", dict(inputmode=E.INPUTMODE_HIEFF)),
    ("4k_inband_v131", dict(inband=E.INBAND_ON, version=E.VERSION_131, tsrate=12345678)),
    ("32k_hem_inband", dict(fftsize=E.FFTSIZE_32K, pilotpattern=E.PILOT_PP4, carriermode=E.CARRIERS_EXTENDED,
                            guardinterval=E.GI_1_16, numdatasyms=3, framesize=E.FECFRAME_NORMAL, rate=E.C3_5,
                            inputmode=E.INPUTMODE_HIEFF, inband=E.INBAND_ON, version=E.VERSION_131)),
]


def grid_cfg(over):
    cfg = BASE.with_(**over)
    fb = fitting_fecblocks(cfg)
    assert fb, "config cannot carry a FEC block"
    fb = max(1, (fb * 3) // 4)
    return cfg.with_(fecblocks=fb, tiblocks=min(cfg.tiblocks, fb))


@pytest.mark.parametrize("name,over", GRID, ids=[g[0] for g in GRID])
def test_framemapper_map_matches_oracle(name, over):
    cfg = grid_cfg(over)
    plan = PP.frame_plan(cfg.fm_args())
    fm = O.FM(*cfg.fm_args())
    assert (plan["M"], plan["S"]) == (fm.mapped_items, fm.stream_items)
    for frame in range(min(3, cfg.t2frames + 1)):
        cells = rand_cells(plan["S"])
        want = fm.work(cells)
        got = _apply(plan["gather_in"], cells, plan["aux"][frame % plan["t2frames"]])
        np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("name,over", GRID + [(n, None) for n in BENCH_CFGS],
                         ids=[g[0] for g in GRID] + BENCH_CFGS)
def test_chain_cell_layout_matches_oracle(name, over):
    """the fused chain's indexing, as the kernels apply it: the map kernel stores QAM cell (r, j)
    at ti_dest(r, (perm[j] + shift[r]) mod cs); the OFDM kernel fills aux bins from cmap < 0 and
    scatters its symbol's contiguous data slots into bins through inv.  The carriers equal the
    oracle's framemapper + pilotgen for every parameter combination."""
    cfg = CONFIGS[name] if over is None else grid_cfg(over)
    lay = PP.chain_layout(cfg)
    fplan = PP.frame_plan(cfg.fm_args())
    pplan = PP.pilot_plan(cfg.pg_args())
    fm = O.FM(*cfg.fm_args())
    pg = O.PG(*cfg.pg_args())
    cs, F = fplan["cs"], fplan["F"]
    cells = rand_cells(lay["S"])
    r = np.repeat(np.arange(F), cs)
    jj = np.tile(np.arange(cs), F)
    t = (fplan["ci_perm"][jj] + fplan["ci_shift"][r]) % cs
    data = np.zeros(lay["S"], np.complex64)
    data[lay["part"][PP.ti_dest(fplan, r, t)]] = cells
    want = pg.carriers(fm.work(cells))
    aux = fplan["aux"][0].copy()
    aux[1:13] = pplan["pilot_values"]
    N = lay["N"]
    k = np.arange(N)
    assert lay["n"].sum() == lay["S"]
    for j in range(lay["Nsym"]):
        code = lay["cmap_stored"][j]
        row = np.where(code < 0, aux[np.clip(-code - 1, 0, None)], 0).astype(np.complex64)
        sl = np.arange(lay["d0"][j], lay["d0"][j] + lay["n"][j])
        assert (code[lay["inv"][sl]] >= 0).all()
        if lay["split"]:   # the first n0 slots feed stored half 0 (even k >> 10), the rest half 1
            n0 = lay["n0"][j]
            assert (lay["inv"][sl[:n0]] < N // 2).all() and (lay["inv"][sl[n0:]] >= N // 2).all()
        row[lay["inv"][sl]] = data[sl]
        row = PP.stored_to_natural(row, N, lay["split"])
        bins = np.empty(N, np.complex64)
        bins[(k + N // 2) % N] = row
        if pplan["eq"]:
            bins = (bins.view(np.float32).reshape(-1, 2) * pplan["isinc"][:, None]).view(np.complex64).reshape(-1)
        np.testing.assert_array_equal(bins.view(np.uint32), want[j].view(np.uint32), err_msg="symbol %d" % j)


@pytest.mark.parametrize("name,over", GRID + [(n, None) for n in BENCH_CFGS],
                         ids=[g[0] for g in GRID] + BENCH_CFGS)
def test_chain_aux_lists_match_cmap(name, over):
    """the OFDM kernel's non-data bins (t2_kernels.hip sub_ifft, scatter mode): the zero run
    [z0, z1), the direct (bin, value) quads and the indirect entries through aux variant v.  For
    every t2_frame_num variant, every symbol and half, they rebuild exactly the non-data bins the
    per-bin code row (cmap < 0) gives, every such bin is written exactly once, and no data bin
    (cmap >= 0) is touched."""
    cfg = CONFIGS[name] if over is None else grid_cfg(over)
    lay = PP.chain_layout(cfg)
    al = PP.aux_lists(cfg)
    N, split = lay["N"], lay["split"]
    nsub = N // 2 if split else N
    grp, auxv = al["grp"], al["auxv"]
    assert grp.shape[0] == 2 * lay["Nsym"] and (grp[:, 0] % 4 == 0).all() and (grp[:, 1] % 4 == 0).all()
    for v in range(auxv.shape[0]):
        for j in range(lay["Nsym"]):
            for h in range(2 if split else 1):
                code = lay["cmap_stored"][j][h * nsub:(h + 1) * nsub]
                want = np.where(code < 0, auxv[v][np.clip(-code - 1, 0, None)], 0).astype(np.complex64)
                got = np.full(nsub, np.nan, np.complex64)
                hits = np.zeros(nsub, np.int32)
                z0, z1 = al["zrun"][2 * j + h]
                assert 0 <= z0 <= z1 <= nsub
                got[z0:z1] = 0
                hits[z0:z1] += 1
                d0, dn, i0, ni = grp[2 * j + h]
                b = al["dbin"][d0:d0 + dn]
                real = b != 0xFFFF
                assert (al["dval"][d0:d0 + dn][~real] == 0).all()
                got[b[real]] = al["dval"][d0:d0 + dn][real]
                np.add.at(hits, b[real], 1)
                e = al["ind"][i0:i0 + ni]     # L1-post cell (e >> 15) - 1 of the frame
                got[e & 0x7FFF] = auxv[v][al["l1_lo"] + (e >> 15) - 1]
                np.add.at(hits, e & 0x7FFF, 1)
                assert hits.max(initial=0) <= 1
                assert (code[hits > 0] < 0).all()
                assert (hits[code < 0] == 1).all(), "variant %d symbol %d half %d" % (v, j, h)
                aux = code < 0
                np.testing.assert_array_equal(got[aux].view(np.uint64), want[aux].view(np.uint64),
                                              err_msg="variant %d symbol %d half %d" % (v, j, h))


@pytest.mark.parametrize("name,over", GRID, ids=[g[0] for g in GRID])
def test_pilot_map_matches_oracle(name, over):
    cfg = grid_cfg(over)
    plan = PP.pilot_plan(cfg.pg_args())
    pg = O.PG(*cfg.pg_args())
    assert plan["active"] == pg.active_items
    cells = rand_cells(plan["active"])
    want = pg.carriers(cells)
    aux = np.zeros(16, np.complex64)
    aux[1:13] = plan["pilot_values"]
    N = plan["N"]
    k = np.arange(N)
    for j in range(plan["Nsym"]):
        row = _apply(plan["bin_map"][j], cells, aux)       # IFFT-input order k
        bins = np.empty(N, np.complex64)
        bins[(k + N // 2) % N] = row
        if plan["eq"]:
            bins = (bins.view(np.float32).reshape(-1, 2) * plan["isinc"][:, None]).view(np.complex64).reshape(-1)
        np.testing.assert_array_equal(bins.view(np.uint32), want[j].view(np.uint32), err_msg="symbol %d" % j)
    assert abs(plan["norm"] - pg.normalization) == 0
    # the planner's P1 samples (the GPU copies them) are the oracle's, bit for bit (both evaluate the
    # 1024-point inverse DFT term by term in double in the same order)
    np.testing.assert_array_equal(np.asarray(plan["p1"], np.complex64).view(np.uint32),
                                  np.asarray(pg.p1(), np.complex64).view(np.uint32))


@pytest.mark.parametrize("name", ["cfg1", "cfg1q", "cfg2", "cfg3", "cfg4", "cfg5"])
def test_benchmark_configs_plan(name):
    cfg = CONFIGS[name]
    fplan = PP.frame_plan(cfg.fm_args())
    pplan = PP.pilot_plan(cfg.pg_args())
    assert fplan["M"] == pplan["active"]
    # chain composition: every mapped data cell points into the frame data region once
    t = fplan["gather_d"]
    data = np.sort(t[t >= 0])
    np.testing.assert_array_equal(data, np.arange(fplan["S"]))
    gi = fplan["gather_in"]
    np.testing.assert_array_equal(np.sort(gi[gi >= 0]), np.arange(fplan["S"]))


ALL_CODES = [(1, r) for r in range(6)] + [(0, r) for r in range(8)]


@pytest.mark.parametrize("framesize,rate", ALL_CODES)
def test_ldpc_quasi_cyclic_schedule_matches_oracle(framesize, rate):
    """the GPU formulation: parity row a = XOR of info groups rotated by b, prefix-XOR over rows,
    exclusive bit-prefix of the column parities -> natural parity p[a + q c]"""
    plan = PP.fec_plan(framesize, rate)
    nbch, q = plan["nbch"], plan["q"]
    nldpc = 64800 if framesize else 16200
    info = rng.integers(0, 2, nbch, dtype=np.uint8)
    want = O.LDPC(framesize, rate).work(info, 1)[nbch:]
    groups = info.reshape(-1, 360)
    rows = np.zeros((q, 360), np.uint8)
    for a in range(q):
        for e in plan["ent"][plan["rowptr"][a]:plan["rowptr"][a + 1]]:
            g, b = int(e) >> 16, int(e) & 0xFFFF
            rows[a] ^= np.roll(groups[g], b)          # column c <- d_g[(c - b) mod 360]
    R = np.bitwise_xor.accumulate(rows, axis=0)
    V = R[-1]
    W = np.concatenate([[0], np.bitwise_xor.accumulate(V)[:-1]]).astype(np.uint8)
    P = R ^ W[None, :]
    got = P.T.reshape(-1)                              # natural index a + q c
    assert got.size == nldpc - nbch
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("const,rot", list(itertools.product(range(4), range(2))))
def test_qam_tables(const, rot):
    """constellation LUT: unit mean energy, Gray structure, rotation angle (interleavermod:169-253)"""
    plan = PP.map_plan(1, E.C3_5, const, rot)
    n = 1 << plan["mod"]
    lut = plan["lut"][:n].astype(np.complex128)
    assert abs(np.mean(np.abs(lut) ** 2) - 1) < 1e-6
    deg = {0: 29.0, 1: 16.8, 2: 8.6, 3: 3.576334375}[const]
    unrot = lut * np.exp(-1j * np.deg2rad(deg)) if rot else lut
    # axis-aligned square grid after de-rotation
    assert np.allclose(np.abs(unrot.real), np.abs(unrot.real).round(6), atol=1e-5)
    levels = np.unique(np.round(unrot.real * np.sqrt({0: 2, 1: 10, 2: 42, 3: 170}[const]), 4))
    assert len(levels) == int(np.sqrt(n)) * (2 if const == 0 else 1) // (2 if const == 0 else 1)


@pytest.mark.parametrize("name,over", GRID + [(n, None) for n in BENCH_CFGS],
                         ids=[g[0] for g in GRID] + BENCH_CFGS)
def test_l1post_plan_matches_host_encoder(name, over):
    """the L1-post plan the GPU kernel runs (template + FRAME_IDX, CRC-32 as XOR of per-bit
    contributions, scrambler, shortening, BCH as XOR of per-position remainders, LDPC accumulate,
    puncturing, L1 constellation), applied on the host in the kernel's order, equals the bit-by-bit
    host encoder (itself checked against the oracle through test_framemapper_map_matches_oracle)
    for several FRAME_IDX values"""
    cfg = CONFIGS[name] if over is None else grid_cfg(over)
    for fi in sorted({0, 1, cfg.t2frames - 1, (7 * cfg.t2frames) // 11}):
        a = PP.l1post(cfg.fm_args(), fi, plan=True)
        b = PP.l1post(cfg.fm_args(), fi, plan=False)
        np.testing.assert_array_equal(a.view(np.uint64), b.view(np.uint64), err_msg="FRAME_IDX %d" % fi)


@pytest.mark.parametrize("l1c", [0, 1, 2, 3])
@pytest.mark.parametrize("extra", [dict(), dict(version=2, l1scrambled=1, reservedbiasbits=1)], ids=["v111", "v131"])
def test_l1post_plan_all_frame_idx(l1c, extra):
    """t2frames = 255: every FRAME_IDX value, every L1 constellation, with and without the v1.3.1
    L1 scrambler / bias bits"""
    cfg = grid_cfg(dict(l1constellation=l1c, t2frames=255, **extra))
    for fi in range(255):
        a = PP.l1post(cfg.fm_args(), fi, plan=True)
        b = PP.l1post(cfg.fm_args(), fi, plan=False)
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), "FRAME_IDX %d" % fi


def _gf2_mod(v, g):
    """remainder of the GF(2) polynomial v (int, bit i = x^i) modulo g (int)"""
    dg = g.bit_length() - 1
    while v.bit_length() - 1 >= dg:
        v ^= g << (v.bit_length() - 1 - dg)
    return v


@pytest.mark.parametrize("framesize,rate", [(1, r) for r in range(6)] + [(0, r) for r in range(8)])
def test_bch_lane_shift_tables(framesize, rate):
    """The FEC kernel's BCH (t2_kernels.hip bch_wave_part, FEC_BCH_TAB): 64 lanes divide
    consecutive chunks of the BBFRAME by the byte table, then each lane moves its remainder to
    the end of the message with P/4 nibble-table lookups and the lanes' results are XORed.  That
    must equal the byte-table division of the whole message, and message || parity must be a
    multiple of the generator (bbheaderbch:504-531)."""
    t = PP.bch_tables(framesize, rate)
    P, C, L = t["P"], t["chunk"], t["L"]
    tab = [int(a) | int(b) << 64 | int(c) << 128 for a, b, c in t["tab"]]
    ctab = t["ctab"]
    mask = (1 << P) - 1

    def divide(msg):
        r = 0
        for byte in msg:
            r = ((r << 8) & mask) ^ tab[((r >> (P - 8)) & 0xFF) ^ int(byte)]
        return r

    gl = T.bch_generator(framesize == 1, P)   # highest power first, degree P
    g = int("".join(str(int(b)) for b in gl), 2)
    rng = np.random.default_rng(1000 + 10 * framesize + rate)
    for _ in range(2):
        msg = rng.integers(0, 256, L, dtype=np.uint8)
        total = 0
        for lane in range(64):
            lo, hi = max(L - (64 - lane) * C, 0), max(L - (63 - lane) * C, 0)
            r = divide(msg[lo:hi])
            for j in range(P // 4):
                e = ctab[j, (r >> (4 * j)) & 15, lane]
                total ^= int(e[0]) | int(e[1]) << 64 | int(e[2]) << 128
        assert total == divide(msg)
        m = int.from_bytes(msg.tobytes(), "big")
        assert _gf2_mod((m << P) | total, g) == 0


@pytest.mark.parametrize("framesize,rate", [(1, r) for r in range(6)] + [(0, r) for r in range(8)])
def test_bch_matrix_core_table(framesize, rate):
    """The chain's BCH (t2_kernels.hip bbch_kernel) computes every block's parity as a GF(2)
    matrix product on the matrix cores: fp4 A fragments masked from the message words, fp4 B fragments
    from the planner table (build_bch_mfma), exact sums, parity = sum & 1, K split into slices whose
    partial parities are XORed (BCH_KS = 8).  Replayed here with the kernel's operand pairing (lane half h,
    K-step u, A dword d, nibble e: bit 4 e + d of the little-endian word of message bytes 32 q + 16 h + 4 u
    .. + 3; column = lane & 31 of tile t) on random
    messages whose bytes past the BBFRAME are garbage (the kernel reads them and must ignore them);
    the parities must equal the byte-table division of the message (bbheaderbch:504-531)."""
    t = PP.bch_tables(framesize, rate)
    P, L = t["P"], t["L"]
    tabb = [int(a) | int(b) << 64 | int(c) << 128 for a, b, c in t["tab"]]
    mask = (1 << P) - 1

    def divide(msg):
        r = 0
        for byte in msg:
            r = ((r << 8) & mask) ^ tabb[((r >> (P - 8)) & 0xFF) ^ int(byte)]
        return r

    tab = PP.bch_mfma_table(framesize, rate)
    nq, nt = tab.shape[0], tab.shape[2]
    assert nq == (L + 31) // 32 and nt == (P + 31) // 32
    nib = (tab[..., None] >> (4 * np.arange(8, dtype=np.uint32))) & 0xF    # (nq, 4, nt, 64, 4, 8)
    # B's set entries per A dword d: fp4 2.0, 1.0, 0.5, 0.5 against the kernel's A values 0.5, 1.0, 2.0, 2.0
    # (dword d keeps bit d of each nibble in place, d = 3 moved down one): every product of set bits is 1
    code, fp4 = np.array([4, 2, 1, 1]), {0: 0.0, 1: 0.5, 2: 1.0, 4: 2.0}
    for d in range(4):
        assert set(np.unique(nib[..., d, :])) <= {0, int(code[d])}
        assert fp4[int(code[d])] * [0.5, 1.0, 2.0, 2.0][d] == 1.0
    tb = (nib != 0).astype(np.int64).reshape(nq, 4, nt, 2, 32, 4, 8)       # lane = 32 h + c
    rng = np.random.default_rng(2000 + 10 * framesize + rate)
    for _ in range(2):
        msg = rng.integers(0, 256, 32 * nq, dtype=np.uint8)                # garbage past L
        words = msg.view("<u4").reshape(nq, 2, 4).astype(np.int64)         # [q][h][u] message words
        sh = 4 * np.arange(8)[None, :] + np.arange(4)[:, None]              # [d][e] -> bit 4 e + d
        bits = (words[..., None, None] >> sh) & 1                           # [q][h][u][d][e]
        bits = bits.transpose(0, 2, 1, 3, 4)                                # [q][u][h][d][e]
        acc = np.einsum("quhde,quthcde->qtc", bits, tb)
        bounds = [s * nq // 8 for s in range(9)]
        par = np.zeros((nt, 32), np.int64)
        for s in range(8):                                                  # XOR of slice partials
            par ^= acc[bounds[s]:bounds[s + 1]].sum(axis=0) & 1
        ref = divide(msg[:L])
        got = 0
        for p in range(P):
            got |= int(par[p // 32, p % 32]) << (P - 1 - p)
        assert got == ref
        assert not par.reshape(-1)[P:].any()
