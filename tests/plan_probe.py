"""ctypes binding of the host-only planner probe (gr-dvbt2ll_amd/csrc/t2_plan_probe.cpp).

It exposes the product's configuration-time gather maps so CPU tests can check them against
the oracle for the whole parameter space; the GPU kernels that consume them are checked by
the -m gpu tests."""
import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
CSRC = ROOT / "gr-dvbt2ll_amd" / "csrc"
LIB = CSRC / "_obj" / ("asan/" if os.environ.get("DVBT2LL_SANITIZED") == "1" else "") / "libt2plan_probe.so"
_L = None


def lib():
    global _L
    if _L is None:
        if not LIB.exists():
            subprocess.run(["make", "-s", "-C", str(CSRC), "probe"], check=True)
        L = ctypes.CDLL(str(LIB))
        vp = ctypes.c_void_p
        L.t2probe_frame.argtypes = [vp] * 7
        L.t2probe_pilot.argtypes = [vp, vp, vp, vp, vp, vp, vp]
        L.t2probe_map.argtypes = [ctypes.c_int] * 4 + [vp, vp]
        L.t2probe_fec.argtypes = [ctypes.c_int] * 3 + [vp, vp, vp]
        L.t2probe_bch.argtypes = [ctypes.c_int] * 2 + [vp, vp, vp]
        L.t2probe_bch_mfma.argtypes = [ctypes.c_int] * 2 + [vp, vp]
        L.t2probe_chain.argtypes = [vp] * 9
        L.t2probe_counts.argtypes = [ctypes.c_int] * 6 + [vp]
        L.t2probe_aux_lists.argtypes = [vp] * 9
        L.t2probe_l1post.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp]
        L.t2probe_frame_mplp.argtypes = [vp] * 5
        L.t2probe_chain_mplp.argtypes = [vp] * 10
        L.t2probe_l1post_mplp.argtypes = [vp, ctypes.c_int, vp, vp]
        L.t2probe_l1post_bits_mplp.argtypes = [vp, ctypes.c_int, vp, ctypes.c_int]
        _L = L
    return _L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def frame_plan(fm_args):
    p = np.array(fm_args, np.int32)
    info = np.zeros(17, np.int32)
    if lib().t2probe_frame(_p(p), _p(info), None, None, None, None, None):
        return None
    M, S, aux_len, t2frames = (int(x) for x in info[:4])
    gin = np.zeros(M, np.int32)
    gd = np.zeros(M, np.int32)
    aux = np.zeros(t2frames * aux_len, np.complex64)
    cs, F = int(info[4]), int(info[5])
    perm = np.zeros(cs, np.int16)
    shift = np.zeros(F, np.int32)
    assert lib().t2probe_frame(_p(p), _p(info), _p(gin), _p(gd), _p(aux), _p(perm), _p(shift)) == 0
    keys = ["M", "S", "aux_len", "t2frames", "cs", "F", "N_P2", "C_P2", "C_DATA", "N_FC", "C_FC", "Lp", "D",
            "ti_on", "ti_small", "ti_big", "ti_nsmall"]
    d = dict(zip(keys, (int(x) for x in info)))
    d.update(gather_in=gin, gather_d=gd, aux=aux.reshape(t2frames, aux_len), ci_perm=perm.astype(np.int64),
             ci_shift=shift.astype(np.int64))
    return d


def pilot_plan(pg_args):
    p = np.array(pg_args, np.int32)
    info = np.zeros(6, np.int32)
    if lib().t2probe_pilot(_p(p), _p(info), None, None, None, None, None):
        return None
    Nsym, N = int(info[0]), int(info[1])
    bm = np.zeros(Nsym * N, np.int32)
    pv = np.zeros(12, np.complex64)
    p1 = np.zeros(2048, np.complex64)
    isinc = np.zeros(N, np.float32)
    norm = np.zeros(1, np.float32)
    assert lib().t2probe_pilot(_p(p), _p(info), _p(bm), _p(pv), _p(p1), _p(isinc), _p(norm)) == 0
    return dict(Nsym=Nsym, N=N, active=int(info[2]), G=int(info[3]), C_PS=int(info[4]), eq=int(info[5]),
                bin_map=bm.reshape(Nsym, N), pilot_values=pv, p1=p1, isinc=isinc, norm=float(norm[0]))


def twiddle_tables(pg_args):
    """the OFDM kernels' two-level twiddle table (128 + N/128) and w_1024 table, as uploaded"""
    N = int(pg_args[11])
    p = np.array(pg_args, np.int32)
    tw = np.zeros(128 + N // 128, np.complex64)
    tw1k = np.zeros(1024, np.complex64)
    assert lib().t2probe_twiddle(_p(p), _p(tw), _p(tw1k)) == 0
    return tw, tw1k


def cell_counts(fftsize, carriermode, pp, papr, gi, preamble):
    """framemapper cell-count table entry {N_P2, C_P2, C_DATA, N_FC, C_FC} or None"""
    out = np.zeros(5, np.int32)
    if lib().t2probe_counts(fftsize, carriermode, pp, papr, gi, preamble, _p(out)):
        return None
    return dict(zip(["N_P2", "C_P2", "C_DATA", "N_FC", "C_FC"], (int(x) for x in out)))


def map_plan(framesize, rate, constellation, rotation):
    info = np.zeros(5, np.int32)
    lut = np.zeros(256, np.complex64)
    assert lib().t2probe_map(framesize, rate, constellation, rotation, _p(info), _p(lut)) == 0
    return dict(zip(["mode", "mod", "W", "R", "cs"], (int(x) for x in info)), lut=lut)


def fec_plan(framesize, rate, constellation=3):
    info = np.zeros(7, np.int32)
    assert lib().t2probe_fec(framesize, rate, constellation, _p(info), None, None) == 0
    kbch, nbch, P, q, nent, chunk, pil = (int(x) for x in info)
    ent = np.zeros(nent, np.uint32)
    rp = np.zeros(q + 1, np.uint16)
    assert lib().t2probe_fec(framesize, rate, constellation, _p(info), _p(ent), _p(rp)) == 0
    return dict(kbch=kbch, nbch=nbch, P=P, q=q, ent=ent, rowptr=rp, chunk=chunk, parity_il=pil)


def bch_tables(framesize, rate):
    """the FEC kernel's BCH tables: byte table (256 x 3 words) and the per-lane chunk-shift
    nibble tables ((P/4) x 16 x 64 x 4 words), with P, the chunk length and the BBFRAME bytes"""
    info = np.zeros(3, np.int32)
    assert lib().t2probe_bch(framesize, rate, _p(info), None, None) == 0
    P, chunk, L = (int(x) for x in info)
    tab = np.zeros(256 * 3, np.uint64)
    ctab = np.zeros((P // 4) * 16 * 64 * 4, np.uint64)
    assert lib().t2probe_bch(framesize, rate, _p(info), _p(tab), _p(ctab)) == 0
    return dict(P=P, chunk=chunk, L=L, tab=tab.reshape(256, 3), ctab=ctab.reshape(P // 4, 16, 64, 4))


def bch_mfma_table(framesize, rate):
    """the chain's BCH matrix-core table (t2_plan build_bch_mfma): uint32 [nq][4][nt][64][4]"""
    info = np.zeros(2, np.int32)
    assert lib().t2probe_bch_mfma(framesize, rate, _p(info), None) == 0
    nq, nt = (int(x) for x in info)
    tab = np.zeros(nq * 4 * nt * 64 * 4, np.uint32)
    assert lib().t2probe_bch_mfma(framesize, rate, _p(info), _p(tab)) == 0
    return tab.reshape(nq, 4, nt, 64, 4)


def ti_dest(plan, r, t):
    """frame data-region index of cell t (cell-interleaved position) of FEC block r: the
    time-interleaver write the chain's map kernel performs (t2_kernels.hip map_kernel)"""
    cs = plan["cs"]
    if not plan["ti_on"]:
        return r * cs + t
    small, big, ns = plan["ti_small"], plan["ti_big"], plan["ti_nsmall"]
    r = np.asarray(r)
    in_small = r < ns * small
    r0 = np.where(in_small, (r // max(small, 1)) * small, ns * small + ((r - ns * small) // big) * big)
    nb = np.where(in_small, small, big)
    rows = cs // 5
    return r0 * cs + (t % rows) * (5 * nb) + 5 * (r - r0) + t // rows


def chain_layout(cfg):
    """the fused chain's layout: cmap (Nsym x N, natural FFT-input order; data codes are frame data
    slots), inv (slot -> bin), each symbol's contiguous slot range [d0, d0 + n) with its first n0
    slots feeding the bins < N/2 when split (32K), and part (TI output index -> slot)"""
    p = np.array(cfg.fm_args(), np.int32)
    g = np.array([cfg.misogroup, cfg.equalization, cfg.bandwidth], np.int32)
    info = np.zeros(4, np.int32)
    assert lib().t2probe_chain(_p(p), _p(g), _p(info), None, None, None, None, None, None) == 0
    Nsym, N, S, split = (int(x) for x in info)
    cmap = np.zeros(Nsym * N, np.int32)
    inv = np.zeros(S, np.uint16)
    d0 = np.zeros(Nsym, np.int32)
    dn = np.zeros(Nsym, np.int32)
    dn0 = np.zeros(Nsym, np.int32)
    part = np.zeros(S, np.int32)
    assert lib().t2probe_chain(_p(p), _p(g), _p(info), _p(cmap), _p(inv), _p(d0), _p(dn), _p(dn0), _p(part)) == 0
    return dict(Nsym=Nsym, N=N, S=S, split=split, cmap_stored=cmap.reshape(Nsym, N), inv=inv.astype(np.int64),
                d0=d0, n=dn, n0=dn0, part=part.astype(np.int64))


def aux_lists(cfg):
    """the fused chain's compact non-data bin lists (t2_plan.h AuxLists) and the per-variant aux
    table they index: dbin, dval (direct (bin, value) entries, quads), ind (bin | code << 15),
    grp (groups 2 j + h: direct offset, count, indirect offset, count), auxv [t2frames, aux_len],
    zrun (groups: the [z0, z1) run of zero bins the kernel zeroes as a range)"""
    p = np.array(cfg.fm_args(), np.int32)
    g = np.array([cfg.misogroup, cfg.equalization, cfg.bandwidth], np.int32)
    sz = np.zeros(6, np.int32)
    assert lib().t2probe_aux_lists(_p(p), _p(g), _p(sz), None, None, None, None, None, None) == 0
    nd, ni, ng, aux_len, t2f, l1_lo = (int(x) for x in sz)
    dbin = np.zeros(nd, np.uint16)
    dval = np.zeros(nd, np.complex64)
    ind = np.zeros(max(ni, 1), np.uint32)
    grp = np.zeros(4 * ng, np.int32)
    auxv = np.zeros(aux_len * t2f, np.complex64)
    zrun = np.zeros(2 * ng, np.int32)
    assert lib().t2probe_aux_lists(_p(p), _p(g), _p(sz), _p(dbin), _p(dval), _p(ind), _p(grp), _p(auxv),
                                   _p(zrun)) == 0
    return dict(dbin=dbin.astype(np.int64), dval=dval, ind=ind[:ni].astype(np.int64), grp=grp.reshape(ng, 4),
                auxv=auxv.reshape(t2f, aux_len), zrun=zrun.reshape(ng, 2), l1_lo=l1_lo)


def l1post(fm_args, frame_idx, plan=True):
    """one FRAME_IDX's L1-post cells: the GPU plan applied on the host in the kernel's order
    (plan=True) or the bit-by-bit host encoder (plan=False)"""
    p = np.array(fm_args, np.int32)
    info = np.zeros(4, np.int32)
    assert lib().t2probe_l1post(_p(p), 0, 1, None, _p(info)) == 0
    out = np.zeros(int(info[2]), np.complex64)
    assert lib().t2probe_l1post(_p(p), int(frame_idx), int(bool(plan)), _p(out), None) == 0
    return out


def stored_index(N, split):
    """natural FFT-input index k -> the chain's stored index (t2_plan.h ofdm_stored_index): 32K halves
    are the bins of even / odd k >> 10"""
    k = np.arange(N)
    if not split:
        return k
    return ((k >> 10) & 1) * (N // 2) + ((k & 1023) | ((k >> 11) << 10))


def stored_to_natural(row, N, split):
    """a symbol row in the chain's stored order -> natural FFT-input order"""
    return np.asarray(row)[stored_index(N, split)]


def frame_plan_mplp(mcfg):
    """the planner's multi-PLP frame (build_frame_mplp): gather maps, aux variants, PLP geometry"""
    a = np.array(mcfg.mplp_array(), np.int32)
    info = np.zeros(68, np.int32)
    if lib().t2probe_frame_mplp(_p(a), _p(info), None, None, None):
        return None
    M, S, aux_len, t2frames = (int(x) for x in info[:4])
    unit = int(info[31])
    gin = np.zeros(unit * M, np.int32)
    gd = np.zeros(M, np.int32)
    aux = np.zeros(t2frames * aux_len, np.complex64)
    assert lib().t2probe_frame_mplp(_p(a), _p(info), _p(gin), _p(gd), _p(aux)) == 0
    n = int(info[6])
    lst = lambda o: [int(x) for x in info[o:o + n]]   # noqa: E731
    return dict(M=M, S=S, aux_len=aux_len, t2frames=t2frames, Lp=int(info[4]), D=int(info[5]), nplp=n,
                start=lst(7), cs=lst(15), F=lst(23), unit=unit, nss=int(info[32]), ssi=int(info[33]),
                t2start=int(info[34]), S_in=int(info[35]), plp_S=lst(36), P=lst(44), in_off=lst(52), type2=lst(60),
                gather_in=gin.reshape(unit, M), gather_d=gd, aux=aux.reshape(t2frames, aux_len))


def chain_layout_mplp(mcfg):
    a = np.array(mcfg.mplp_array(), np.int32)
    pg3 = np.array([mcfg.misogroup, mcfg.equalization, mcfg.bandwidth], np.int32)
    info = np.zeros(5, np.int32)
    fr = frame_plan_mplp(mcfg)
    pl = pilot_plan(mcfg.pg_args())
    assert lib().t2probe_chain_mplp(_p(a), _p(pg3), _p(info), *([None] * 7)) == 0
    Nsym, N, S, P = pl["Nsym"], pl["N"], int(info[2]), fr["nplp"]   # frame class 0's data cells
    cmap = np.zeros(Nsym * N, np.int32)
    inv = np.zeros(S, np.uint16)
    d0, dn, dn0 = (np.zeros(Nsym, np.int32) for _ in range(3))
    part = np.zeros(S, np.int32)
    bnd = np.zeros(2 * Nsym * (P + 1), np.int32)
    assert lib().t2probe_chain_mplp(_p(a), _p(pg3), _p(info), _p(cmap), _p(inv), _p(d0), _p(dn), _p(dn0), _p(part),
                                    _p(bnd)) == 0
    return dict(Nsym=Nsym, N=N, S=S, split=int(info[3]), nplp=P, cmap=cmap.reshape(Nsym, N), inv=inv, d0=d0,
                dn=dn, dn0=dn0, part=part, bnd=bnd.reshape(2 * Nsym, P + 1), frame=fr)


def l1post_bits_mplp(mcfg, frame_idx):
    """the planner's L1-post signalling bits before the CRC-32 (one per byte)"""
    a = np.array(mcfg.mplp_array(), np.int32)
    out = np.zeros(4096, np.uint8)
    n = lib().t2probe_l1post_bits_mplp(_p(a), int(frame_idx), _p(out), len(out))
    assert n > 0
    return out[:n]


def l1post_mplp(mcfg, frame_idx):
    a = np.array(mcfg.mplp_array(), np.int32)
    info = np.zeros(3, np.int32)
    assert lib().t2probe_l1post_mplp(_p(a), frame_idx, None, _p(info)) == 0
    out = np.zeros(int(info[2]), np.complex64)
    assert lib().t2probe_l1post_mplp(_p(a), frame_idx, _p(out), _p(info)) == 0
    return out, dict(nsig=int(info[0]), npost=int(info[1]), Lp=int(info[2]))
