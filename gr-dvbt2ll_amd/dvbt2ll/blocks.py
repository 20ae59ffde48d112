"""Host-side mirror of the gr-dvbt2ll block API (include/dvbt2ll/*.h), backed by the HIP library.

Each class keeps the reference block's name, make() arguments, output multiple, forecast()
and general_work() contract (one general_work call = the reference's call with the same
noutput_items; the number of consumed input items is what the reference passes to
consume_each()).  Buffers are numpy arrays (GNU Radio's python block convention:
general_work(input_items, output_items) with lists of arrays).
"""
import ctypes

import numpy as np

from ._lib import lib, check, _BbParams, _LdpcParams, _ImParams, _FmParams, _PgParams, _MplpParams


class _Block:
    _name = None
    _params = None
    in_dtype = np.uint8
    out_dtype = np.uint8

    def __init__(self, *args, device=0):
        self._h = None
        p = self._params(*[int(a) for a in args])
        h = ctypes.c_void_p()
        check(getattr(lib(), "dvbt2ll_%s_create" % self._name)(ctypes.byref(p), int(device), ctypes.byref(h)),
              "%s make" % self._name)
        self._h = h
        self.nitems_consumed = 0
        self.last_consumed = 0

    @classmethod
    def make(cls, *args, **kw):
        return cls(*args, **kw)

    def output_multiple(self):
        return getattr(lib(), "dvbt2ll_%s_output_multiple" % self._name)(self._h)

    def forecast(self, noutput_items):
        n = ctypes.c_int(0)
        check(getattr(lib(), "dvbt2ll_%s_forecast" % self._name)(self._h, int(noutput_items), ctypes.byref(n)),
              "forecast")
        return [n.value]

    def general_work(self, input_items, output_items, noutput_items=None):
        inp = np.ascontiguousarray(input_items[0], dtype=self.in_dtype)
        out = output_items[0]
        assert out.dtype == self.out_dtype and out.flags.c_contiguous
        nout = len(out) if noutput_items is None else int(noutput_items)
        consumed = ctypes.c_int(0)
        r = getattr(lib(), "dvbt2ll_%s_general_work" % self._name)(
            self._h, nout, len(inp), inp.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p),
            ctypes.byref(consumed))
        check(r, "%s general_work" % self._name)
        self.last_consumed = consumed.value
        self.nitems_consumed += consumed.value
        return r

    def __del__(self):
        if getattr(self, "_h", None):
            getattr(lib(), "dvbt2ll_%s_destroy" % self._name)(self._h)
            self._h = None


class bbheaderbch_bb(_Block):
    """bbheaderbch_bb::make(framesize, rate, mode, inband, fecblocks, tsrate)
    (include/dvbt2ll/bbheaderbch_bb.h:49): TS bytes -> BBFRAME + BCH, one bit per byte."""
    _name, _params = "bbheaderbch", _BbParams

    def sync_errors(self):
        """TS sync bytes != 0x47 consumed so far (reference: a GR_LOG_WARN each, :675, :703)"""
        return lib().dvbt2ll_bbheaderbch_sync_errors(self._h)

    def set_isi(self, isi):
        """one PLP of a multi-PLP frame: BBHEADER MATYPE multiple input streams, ISI = the PLP_ID
        (the reference add_bbheader's MIS branch, lib/bbheaderbch_bb_impl.cc:288-298)"""
        check(lib().dvbt2ll_bbheaderbch_set_isi(self._h, int(isi)), "set_isi")


class ldpc_bb(_Block):
    """gr-dtv dvb_ldpc_bb(DVBT2, framesize, rate, MOD_OTHER) replacement used between
    bbheaderbch and interleavermod in apps/vv009-4kshort.grc:386-460."""
    _name, _params = "ldpc", _LdpcParams


class interleavermod_bc(_Block):
    """interleavermod_bc::make(framesize, rate, constellation, rotation)
    (include/dvbt2ll/interleavermod_bc.h:49): LDPC bits -> complex64 cells."""
    _name, _params = "interleavermod", _ImParams
    out_dtype = np.complex64


class framemapperfint_cc(_Block):
    """framemapperfint_cc::make(...20 args...) (include/dvbt2ll/framemapperfint_cc.h:49):
    one T2 frame of cells per call -> frame-mapped, frequency-interleaved cells."""
    _name, _params = "framemapperfint", _FmParams
    in_dtype = np.complex64
    out_dtype = np.complex64

    def stream_items(self):
        return lib().dvbt2ll_framemapperfint_stream_items(self._h)


class pilotgenp1insert_cc(_Block):
    """pilotgenp1insert_cc::make(carriermode, fftsize, pilotpattern, guardinterval, numdatasyms,
    paprmode, version, preamble, misogroup, equalization, bandwidth, vlength)
    (include/dvbt2ll/pilotgenp1insert_cc.h:49): one T2 frame per call -> P1 + OFDM symbols."""
    _name, _params = "pilotgenp1insert", _PgParams
    in_dtype = np.complex64
    out_dtype = np.complex64

    def active_items(self):
        return lib().dvbt2ll_pilotgenp1insert_active_items(self._h)

    def debug_carriers(self, cells, num_symbols, vlength):
        cells = np.ascontiguousarray(cells, np.complex64)
        out = np.zeros((num_symbols, vlength), np.complex64)
        check(lib().dvbt2ll_pilotgenp1insert_debug_carriers(self._h, cells.ctypes.data_as(ctypes.c_void_p),
                                                             out.ctypes.data_as(ctypes.c_void_p)), "carriers")
        return out


class framemapper_mplp_cc:
    """framemapperfint_cc with one input port per data PLP (the reference carries one
    PLP, lib/framemapperfint_cc_impl.cc:152-250): make(MplpConfig); one T2 frame per general_work call,
    consuming stream_items(k) cells from every port k -- or, for a TIME_IL_TYPE 1 PLP, its whole
    interleaving frame on the first of its P_I T2 frames and nothing on the others (forecast() and
    last_consumed say which)"""
    in_dtype = np.complex64
    out_dtype = np.complex64

    def __init__(self, mcfg, device=0):
        self._h = None
        self.nplp = mcfg.nplp
        p = _MplpParams.from_config(mcfg)
        h = ctypes.c_void_p()
        check(lib().dvbt2ll_framemapper_mplp_create(ctypes.byref(p), int(device), ctypes.byref(h)),
              "framemapper_mplp make")
        self._h = h
        self.nitems_consumed = [0] * self.nplp

    @classmethod
    def make(cls, *args, **kw):
        return cls(*args, **kw)

    def output_multiple(self):
        return lib().dvbt2ll_framemapper_mplp_output_multiple(self._h)

    def stream_items(self, plp):
        return lib().dvbt2ll_framemapper_mplp_stream_items(self._h, int(plp))

    def forecast(self, noutput_items):
        n = (ctypes.c_int * self.nplp)()
        check(lib().dvbt2ll_framemapper_mplp_forecast(self._h, int(noutput_items), n), "forecast")
        return list(n)

    def general_work(self, input_items, output_items, noutput_items=None):
        assert len(input_items) == self.nplp
        ins = [np.ascontiguousarray(x, np.complex64) for x in input_items]
        out = output_items[0]
        assert out.dtype == self.out_dtype and out.flags.c_contiguous
        nout = len(out) if noutput_items is None else int(noutput_items)
        nin = (ctypes.c_int * self.nplp)(*[len(x) for x in ins])
        ptrs = (ctypes.c_void_p * self.nplp)(*[x.ctypes.data for x in ins])
        cons = (ctypes.c_int * self.nplp)()
        r = lib().dvbt2ll_framemapper_mplp_general_work(self._h, nout, nin, ptrs, out.ctypes.data_as(ctypes.c_void_p),
                                                         cons)
        check(r, "framemapper_mplp general_work")
        for k in range(self.nplp):
            self.nitems_consumed[k] += cons[k]
        self.last_consumed = list(cons)
        return r

    def __del__(self):
        if getattr(self, "_h", None):
            lib().dvbt2ll_framemapper_mplp_destroy(self._h)
            self._h = None
