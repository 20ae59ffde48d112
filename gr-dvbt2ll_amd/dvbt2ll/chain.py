"""Fused TS -> IQ chain (dvbt2ll_chain_* in include/dvbt2ll_hip.h).

Equivalent to bbheaderbch_bb -> ldpc_bb -> interleavermod_bc -> framemapperfint_cc ->
pilotgenp1insert_cc for whole T2 frames, with device-resident buffers.  Frame k of the
stream is encoded with the state the reference blocks would hold at that point, so frames
(and therefore GPUs) can be processed independently.
"""
import ctypes

import numpy as np

from ._lib import lib, check, _ChainParams, _ChainInfo, _FmParams, _MplpParams, _MplpChainParams
from .configs import ts_for_frames, MplpConfig

IQ_CF32 = 0   # DVBT2LL_IQ_CF32
IQ_SC16 = 1   # DVBT2LL_IQ_SC16


class Chain:
    def __init__(self, cfg, max_frames=1, device=0):
        """cfg: a T2Config (the reference's single-PLP frame) or an MplpConfig (several data PLPs, Type 1 / 2,
        TIME_IL_TYPE 0 / 1; dvbt2ll_chain_create_mplp)"""
        self.cfg = cfg
        h = ctypes.c_void_p()
        self._h = None
        if isinstance(cfg, MplpConfig):
            p = _MplpChainParams(_MplpParams.from_config(cfg), int(cfg.misogroup), int(cfg.equalization),
                                 int(cfg.bandwidth), int(max_frames))
            check(lib().dvbt2ll_chain_create_mplp(ctypes.byref(p), int(device), ctypes.byref(h)), "chain create")
        else:
            fm = _FmParams(*[int(v) for v in cfg.fm_args()])
            p = _ChainParams(fm, int(cfg.misogroup), int(cfg.equalization), int(cfg.bandwidth), int(max_frames),
                             int(cfg.tsrate))
            check(lib().dvbt2ll_chain_create(ctypes.byref(p), int(device), ctypes.byref(h)), "chain create")
        self._h = h
        self.max_frames = max_frames
        self.nplp = lib().dvbt2ll_chain_num_plps(self._h)
        # runs cover whole interleaving frames: first_frame and nframes multiples of unit_frames
        self.unit_frames = lib().dvbt2ll_chain_unit_frames(self._h)
        info = _ChainInfo()
        check(lib().dvbt2ll_chain_get_info(self._h, ctypes.byref(info)), "chain info")
        self.info = {f: getattr(info, f) for f, _ in _ChainInfo._fields_}
        self.plp_info = []
        for k in range(self.nplp):
            check(lib().dvbt2ll_chain_get_plp_info(self._h, k, ctypes.byref(info)), "plp info")
            self.plp_info.append({f: getattr(info, f) for f, _ in _ChainInfo._fields_})
        self.iq_format = IQ_CF32
        self.nslots = 1

    def set_output(self, gain=1.0, fmt=IQ_CF32):
        """output gain (the flowgraph's multiply_const after pilotgen) and IQ format: IQ_CF32
        (complex64, pilotgen's own output) or IQ_SC16 (int16 I/Q pairs, full scale 32767)"""
        check(lib().dvbt2ll_chain_set_output(self._h, float(gain), int(fmt)), "chain output")
        self.iq_format = int(fmt)

    def set_slots(self, nslots):
        """intermediate buffer slots taken round-robin by run calls: with nslots > 1, calls
        issued on different streams overlap on the GPU (dvbt2ll_chain_set_slots)"""
        check(lib().dvbt2ll_chain_set_slots(self._h, int(nslots)), "chain slots")
        self.nslots = int(nslots)

    def set_graph(self, enable=True):
        """launch the three kernels as one hipGraph per call (dvbt2ll_chain_set_graph)"""
        check(lib().dvbt2ll_chain_set_graph(self._h, int(bool(enable))), "chain graph")

    @property
    def iq_bytes_per_sample(self):
        return 4 if self.iq_format == IQ_SC16 else 8

    @property
    def iq_per_frame(self):
        return self.info["iq_samples_per_frame"]

    def run_device(self, ts_ptr, ts_base, ts_len, first_frame, nframes, iq_ptr, stream=0):
        check(lib().dvbt2ll_chain_run_device(self._h, ctypes.c_void_p(ts_ptr), int(ts_base), int(ts_len),
                                             int(first_frame), int(nframes), ctypes.c_void_p(iq_ptr),
                                             ctypes.c_void_p(stream or None)), "chain run")

    def run_streams(self, ts_ptr, ts_stride, nstreams, ts_base, ts_len, first_frame, nframes, iq_ptr, stream=0):
        """nstreams independent TS streams (stream s at ts_ptr + s * ts_stride, each laid out as
        run_device's buffer) -> IQ of frames [first_frame, first_frame + nframes) of every stream in one
        launch, stream-major (dvbt2ll_chain_run_streams)"""
        check(lib().dvbt2ll_chain_run_streams(self._h, ctypes.c_void_p(ts_ptr), int(ts_stride), int(nstreams),
                                              int(ts_base), int(ts_len), int(first_frame), int(nframes),
                                              ctypes.c_void_p(iq_ptr), ctypes.c_void_p(stream or None)),
              "chain run streams")

    def run_plps(self, ts_ptrs, ts_bases, ts_lens, first_frame, nframes, iq_ptr, stream=0):
        """multi-PLP frames: PLP k's TS at device pointer ts_ptrs[k] (absolute offset ts_bases[k], ts_lens[k]
        bytes) -> IQ of frames [first_frame, first_frame + nframes) (dvbt2ll_chain_run_plps)"""
        n = self.nplp
        assert len(ts_ptrs) == len(ts_bases) == len(ts_lens) == n
        check(lib().dvbt2ll_chain_run_plps(self._h, (ctypes.c_void_p * n)(*ts_ptrs),
                                           (ctypes.c_int64 * n)(*[int(x) for x in ts_bases]),
                                           (ctypes.c_int64 * n)(*[int(x) for x in ts_lens]), int(first_frame),
                                           int(nframes), ctypes.c_void_p(iq_ptr), ctypes.c_void_p(stream or None)),
              "chain run plps")

    def debug_plp_codewords(self, plp, nblocks):
        stride = self.plp_info[plp]["cw_stride_bytes"]
        out = np.zeros(nblocks * stride, np.uint8)
        check(lib().dvbt2ll_chain_debug_plp_codewords(self._h, int(plp), out.ctypes.data_as(ctypes.c_void_p),
                                                      len(out)), "cw")
        return out.reshape(nblocks, stride)

    def run(self, first_frame, nframes, ts=None, ts_base=None, seed=1):
        """host convenience: synthetic TS (or the given buffer) -> IQ numpy array"""
        if ts is None:
            ts, ts_base = ts_for_frames(self.cfg, first_frame, nframes, seed)
        ts = np.ascontiguousarray(ts, np.uint8)
        if self.iq_format == IQ_SC16:   # interleaved int16 I, Q
            iq = np.zeros((nframes * self.iq_per_frame, 2), np.int16)
        else:
            iq = np.zeros(nframes * self.iq_per_frame, np.complex64)
        check(lib().dvbt2ll_chain_run_host(self._h, ts.ctypes.data_as(ctypes.c_void_p), int(ts_base), len(ts),
                                           int(first_frame), int(nframes), iq.ctypes.data_as(ctypes.c_void_p)),
              "chain run")
        return iq

    def host_submit(self, ts_ptr, ts_base, ts_len, first_frame, nframes, iq_ptr):
        """streaming host path (dvbt2ll_chain_host_submit): host TS -> host IQ for nframes frames on the handle's
        copy-in / compute / copy-out streams; returns a ticket at once (the buffers stay the caller's until
        host_wait(ticket))"""
        t = ctypes.c_int64(0)
        check(lib().dvbt2ll_chain_host_submit(self._h, ctypes.c_void_p(ts_ptr), int(ts_base), int(ts_len),
                                              int(first_frame), int(nframes), ctypes.c_void_p(iq_ptr),
                                              ctypes.byref(t)), "host submit")
        return t.value

    def host_wait(self, ticket):
        check(lib().dvbt2ll_chain_host_wait(self._h, int(ticket)), "host wait")

    def run_host_pipelined(self, ts, ts_base, first_frame, nframes, iq, chunk_frames=0):
        """host numpy TS -> host numpy IQ (complex64, or (n, 2) int16 after set_output(.., IQ_SC16)) through the
        submission ring in chunks of chunk_frames (0: max_frames); synchronous"""
        ts = np.ascontiguousarray(ts, np.uint8)
        assert iq.flags.c_contiguous and iq.nbytes >= nframes * self.iq_per_frame * self.iq_bytes_per_sample
        check(lib().dvbt2ll_chain_run_host_pipelined(self._h, ts.ctypes.data_as(ctypes.c_void_p), int(ts_base),
                                                     len(ts), int(first_frame), int(nframes),
                                                     iq.ctypes.data_as(ctypes.c_void_p), int(chunk_frames)),
              "run host pipelined")
        return iq

    def set_timing(self, enable):
        check(lib().dvbt2ll_chain_set_timing(self._h, int(bool(enable))), "timing")

    def timing(self):
        """accumulated HIP-event milliseconds and launch counts of the stages (fec, map, ofdm, l1post)"""
        ms = (ctypes.c_double * 4)()
        n = (ctypes.c_int64 * 4)()
        check(lib().dvbt2ll_chain_get_timing(self._h, ms, n, 4), "timing")
        return list(ms), list(n)

    def debug_keep_codewords(self, enable=True):
        """test hook: the following runs also store the packed codewords (the LDPC + map kernel keeps
        them on chip otherwise); debug_codewords / debug_plp_codewords need it"""
        check(lib().dvbt2ll_chain_debug_keep_codewords(self._h, int(bool(enable))), "keep codewords")

    def debug_codewords(self, nblocks):
        stride = self.info["cw_stride_bytes"]
        out = np.zeros(nblocks * stride, np.uint8)
        check(lib().dvbt2ll_chain_debug_codewords(self._h, out.ctypes.data_as(ctypes.c_void_p), len(out)), "cw")
        return out.reshape(nblocks, stride)

    def debug_cell_pairs(self, ncells):
        out = np.zeros(ncells, np.uint16)
        check(lib().dvbt2ll_chain_debug_cell_pairs(self._h, out.ctypes.data_as(ctypes.c_void_p), ncells), "pairs")
        return out

    def debug_cells(self, ncells):
        out = np.zeros(ncells, np.complex64)
        check(lib().dvbt2ll_chain_debug_cells(self._h, out.ctypes.data_as(ctypes.c_void_p), ncells), "cells")
        return out

    def sync_errors(self):
        """TS sync bytes != 0x47 consumed so far (the reference's "Transport Stream sync error!"
        warnings, bbheaderbch_bb_impl.cc:675, 703); synchronises the device"""
        n = ctypes.c_int64(0)
        check(lib().dvbt2ll_chain_sync_errors(self._h, ctypes.byref(n)), "sync errors")
        return n.value

    def synchronize(self):
        check(lib().dvbt2ll_chain_synchronize(self._h), "sync")

    def __del__(self):
        if getattr(self, "_h", None):
            lib().dvbt2ll_chain_destroy(self._h)
            self._h = None
