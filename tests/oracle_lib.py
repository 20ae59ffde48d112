"""ctypes binding of the CPU oracle (TEST INFRASTRUCTURE ONLY).

The oracle is a plain-C restatement of the reference blocks (oracle/dvbt2_oracle.c);
only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
"""
import ctypes
import os
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
LIB_PATH = ROOT / "oracle" / "_build" / ("asan/" if os.environ.get("DVBT2LL_SANITIZED") == "1" else "") / "libdvbt2_oracle.so"

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            subprocess.run(["make", "-s", "-C", str(ROOT / "oracle")], check=True)
        L = ctypes.CDLL(str(LIB_PATH))
        vp, ci = ctypes.c_void_p, ctypes.c_int
        L.orc_bb_create.restype = vp
        L.orc_bb_create.argtypes = [ci] * 6
        L.orc_bb_work.argtypes = [vp, ci, vp, vp, ctypes.POINTER(ci)]
        L.orc_bb_forecast.argtypes = [vp, ci]
        L.orc_bb_nbch.argtypes = [vp]
        L.orc_bb_kbch.argtypes = [vp]
        L.orc_bb_destroy.argtypes = [vp]
        L.orc_bb_set_isi.argtypes = [vp, ci]
        L.orc_fm_create_mplp.restype = vp
        L.orc_fm_create_mplp.argtypes = [ci, vp] + [ci] * 13
        L.orc_fm_consume.argtypes = [vp, ci]
        L.orc_fm_seek.argtypes = [vp, ctypes.c_long]
        L.orc_fm_l1post_cells.argtypes = [vp]
        L.orc_fm_l1post_bits.argtypes = [vp, ctypes.c_long, vp, ci]
        L.orc_ldpc_create.restype = vp
        L.orc_ldpc_create.argtypes = [ci, ci]
        L.orc_ldpc_work.argtypes = [vp, ci, vp, vp]
        L.orc_ldpc_destroy.argtypes = [vp]
        L.orc_im_create.restype = vp
        L.orc_im_create.argtypes = [ci] * 4
        L.orc_im_work.argtypes = [vp, ci, vp, vp, ctypes.POINTER(ci)]
        L.orc_im_cell_size.argtypes = [vp]
        L.orc_im_destroy.argtypes = [vp]
        L.orc_fm_create.restype = vp
        L.orc_fm_create.argtypes = [ci] * 20
        L.orc_fm_work.argtypes = [vp, vp, vp]
        L.orc_fm_stream_items.argtypes = [vp]
        L.orc_fm_mapped_items.argtypes = [vp]
        L.orc_fm_destroy.argtypes = [vp]
        L.orc_pg_create.restype = vp
        L.orc_pg_create.argtypes = [ci] * 12
        for f in ("orc_pg_active_items", "orc_pg_output_items", "orc_pg_num_symbols", "orc_pg_guard"):
            getattr(L, f).argtypes = [vp]
        L.orc_pg_normalization.argtypes = [vp]
        L.orc_pg_normalization.restype = ctypes.c_float
        L.orc_pg_carriers.argtypes = [vp, vp, vp]
        L.orc_pg_work.argtypes = [vp, vp, vp]
        L.orc_pg_p1.argtypes = [vp, vp]
        L.orc_pg_destroy.argtypes = [vp]
        L.t2m_tables.argtypes = [ci, vp, vp]
        L.t2m_symbols.argtypes = [ci, ci, ci, vp, ctypes.c_float, ctypes.c_float, ci, vp]
        L.orc_crc8_dvbs2.restype = ctypes.c_uint8
        L.orc_crc8_dvbs2.argtypes = [vp, ci]
        L.orc_crc32_bits.restype = ctypes.c_uint32
        L.orc_crc32_bits.argtypes = [vp, ci]
        L.orc_bb_prbs.argtypes = [vp, ci]
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class BB:
    def __init__(self, framesize, rate, mode=0, inband=0, fecblocks=168, tsrate=4000000, isi=None):
        self.h = lib().orc_bb_create(framesize, rate, mode, inband, fecblocks, tsrate)
        assert self.h, "oracle bbheaderbch create failed"
        if isi is not None:            # one PLP of a multi-PLP frame: MIS, MATYPE-2 = PLP_ID
            lib().orc_bb_set_isi(self.h, isi)
        self.nbch = lib().orc_bb_nbch(self.h)
        self.kbch = lib().orc_bb_kbch(self.h)

    def forecast(self, nout):
        return lib().orc_bb_forecast(self.h, nout)

    def work(self, ts, nblocks):
        out = np.zeros(nblocks * self.nbch, np.uint8)
        ts = np.ascontiguousarray(ts, np.uint8)
        c = ctypes.c_int(0)
        lib().orc_bb_work(self.h, nblocks * self.nbch, _p(ts), _p(out), ctypes.byref(c))
        return out, c.value

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_bb_destroy(self.h)


class LDPC:
    def __init__(self, framesize, rate):
        self.h = lib().orc_ldpc_create(framesize, rate)
        self.nldpc = 64800 if framesize == 1 else 16200

    def work(self, bits, nblocks):
        out = np.zeros(nblocks * self.nldpc, np.uint8)
        bits = np.ascontiguousarray(bits, np.uint8)
        lib().orc_ldpc_work(self.h, nblocks, _p(bits), _p(out))
        return out

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ldpc_destroy(self.h)


class IM:
    def __init__(self, framesize, rate, constellation, rotation):
        self.h = lib().orc_im_create(framesize, rate, constellation, rotation)
        self.cell_size = lib().orc_im_cell_size(self.h)
        self.nldpc = 64800 if framesize == 1 else 16200

    def work(self, bits, nblocks):
        out = np.zeros(nblocks * self.cell_size, np.complex64)
        bits = np.ascontiguousarray(bits, np.uint8)
        c = ctypes.c_int(0)
        lib().orc_im_work(self.h, nblocks * self.cell_size, _p(bits), _p(out), ctypes.byref(c))
        return out

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_im_destroy(self.h)


class FM:
    def __init__(self, *params):
        assert len(params) == 20
        self.h = lib().orc_fm_create(*params)
        assert self.h, "oracle framemapper create failed"
        self.stream_items = lib().orc_fm_stream_items(self.h)
        self.mapped_items = lib().orc_fm_mapped_items(self.h)

    def work(self, cells):
        cells = np.ascontiguousarray(cells, np.complex64)
        out = np.zeros(self.mapped_items, np.complex64)
        lib().orc_fm_work(self.h, _p(cells), _p(out))
        return out

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_fm_destroy(self.h)


class FMM(FM):
    """framemapperfint for a multi-PLP frame (orc_fm_create_mplp; parity unpinned beyond the reference's one
    Type-1 PLP): work() takes the cells every PLP consumes this T2 frame (consume(k): a whole interleaving
    frame on its first T2 frame, else none), PLP 0 first"""
    def __init__(self, mcfg):
        plp = np.array([list(p.plp_args()[:8]) + [p.plp_type, p.ti_type, p.ti_frames, p.frame_interval,
                                                   p.first_frame_idx] for p in mcfg.plps], np.int32).reshape(-1)
        self._plp = plp
        self.h = lib().orc_fm_create_mplp(mcfg.nplp, _p(plp), mcfg.num_subslices, *mcfg.common_args())
        assert self.h, "oracle multi-PLP framemapper create failed"
        self.stream_items = lib().orc_fm_stream_items(self.h)
        self.mapped_items = lib().orc_fm_mapped_items(self.h)
        self.l1post_cells = lib().orc_fm_l1post_cells(self.h)

    def consume(self, k):
        return lib().orc_fm_consume(self.h, k)

    def seek(self, frame):
        """start at absolute T2 frame `frame` (a launch unit boundary)"""
        lib().orc_fm_seek(self.h, int(frame))

    def l1post_bits(self, frame):
        """the L1-post signalling bits (before the CRC-32, one per byte) the oracle builds for T2 frame `frame`"""
        out = np.zeros(4096, np.uint8)
        n = lib().orc_fm_l1post_bits(self.h, int(frame), _p(out), len(out))
        assert n > 0
        return out[:n]


def mplp_cells(mcfg, first_frame, nframes):
    """oracle per-PLP chain up to the framemapper input: for each T2 frame, the cells the PLPs consume
    there, concatenated (PLP k: TS seed k + 1, BBHEADER MIS with ISI = k when nplp > 1; a TIME_IL_TYPE 1
    PLP delivers its interleaving frame's F FEC blocks on the first of its P_I T2 frames and nothing on
    the others); returns (list of per-frame cell arrays, per-PLP BB bits and codewords of the
    interleaving frames starting in the frames)"""
    from dvbt2ll.configs import ts_for_frames
    assert first_frame % mcfg.unit_frames == 0
    frames = [[] for _ in range(nframes)]
    bb_bits, codewords = [], []
    for k, p in enumerate(mcfg.plps):
        F, P = p.fecblocks, p.if_frames
        bb = BB(*p.bb_args(), isi=k if mcfg.nplp > 1 else None)
        ld, im = LDPC(p.framesize, p.rate), IM(*p.im_args())
        ts, base = ts_for_frames(p, 0, first_frame + nframes, seed=k + 1)
        off = 0
        bits_k, cw_k = [], []
        for f in range(p.first_frame_idx, first_frame + nframes, P):   # its interleaving frames' first T2 frames
            bits, c = bb.work(ts[off:], F)
            off += c
            if f >= first_frame:
                cw = ld.work(bits, F)
                bits_k.append(bits)
                cw_k.append(cw)
                frames[f - first_frame].append(im.work(cw, F))
        bb_bits.append(bits_k)
        codewords.append(cw_k)
    return [np.concatenate(c) if c else np.zeros(0, np.complex64) for c in frames], bb_bits, codewords


class PG:
    def __init__(self, *params):
        assert len(params) == 12
        self.h = lib().orc_pg_create(*params)
        assert self.h, "oracle pilotgen create failed"
        self.vlength = params[11]
        self.active_items = lib().orc_pg_active_items(self.h)
        self.output_items = lib().orc_pg_output_items(self.h)
        self.num_symbols = lib().orc_pg_num_symbols(self.h)
        self.guard = lib().orc_pg_guard(self.h)
        self.normalization = lib().orc_pg_normalization(self.h)

    def carriers(self, cells):
        cells = np.ascontiguousarray(cells, np.complex64)
        out = np.zeros(self.num_symbols * self.vlength, np.complex64)
        lib().orc_pg_carriers(self.h, _p(cells), _p(out))
        return out.reshape(self.num_symbols, self.vlength)

    def work(self, cells):
        cells = np.ascontiguousarray(cells, np.complex64)
        out = np.zeros(self.output_items, np.complex64)
        lib().orc_pg_work(self.h, _p(cells), _p(out))
        return out

    def p1(self):
        out = np.zeros(2048, np.complex64)
        lib().orc_pg_p1(self.h, _p(out))
        return out

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_pg_destroy(self.h)


# ---------------------------------------------------------------- GPU-order IFFT model (oracle/ifft_model.c)
def model_tables(N):
    tw = np.zeros(128 + N // 128, np.complex64)
    tw1k = np.zeros(1024, np.complex64)
    assert lib().t2m_tables(N, _p(tw), _p(tw1k)) == 0
    return tw, tw1k


def model_symbols(carriers, G, norm, gain=1.0, fmt=0):
    """carriers (nsym x N, pilotgen's pre-IFFT symbols) -> the OFDM symbols with guard intervals
    exactly as the GPU kernels compute them (same operation order); complex64, or
    int16 I/Q pairs for fmt 1"""
    car = np.ascontiguousarray(carriers, np.complex64)
    nsym, N = car.shape
    out = np.zeros(nsym * (G + N), np.complex64) if fmt == 0 else np.zeros((nsym * (G + N), 2), np.int16)
    assert lib().t2m_symbols(N, G, nsym, _p(car), float(norm), float(gain), fmt, _p(out)) == 0
    return out


def model_frame(carriers, G, norm, p1, gain=1.0, fmt=0):
    """a whole T2 frame as the GPU writes it: P1 (the planner's precomputed samples) then the symbols"""
    sy = model_symbols(carriers, G, norm, gain, fmt)
    p1 = np.asarray(p1, np.complex64)
    a = np.stack([p1.real, p1.imag], axis=1).astype(np.float32) * np.float32(gain)   # per component, as the GPU
    if fmt == 0:
        return np.concatenate([a.reshape(-1).view(np.complex64), sy])
    q = np.clip(np.rint(a * np.float32(32767.0)), -32768, 32767).astype(np.int16)
    return np.concatenate([q, sy])
