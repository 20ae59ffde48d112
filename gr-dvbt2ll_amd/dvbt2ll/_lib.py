"""ctypes loader for the in-tree HIP library libdvbt2ll_hip.so (built by __graft_entry__.build()).

There is no CPU fallback: if the shared library is missing this module raises, so a GPU
test can never pass on a silent host path.
"""
import ctypes
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "libdvbt2ll_hip.so"

_lib = None


class DVBT2Error(RuntimeError):
    pass


class _FmParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "framesize", "rate", "constellation", "rotation", "fecblocks", "tiblocks", "carriermode",
        "fftsize", "guardinterval", "l1constellation", "pilotpattern", "t2frames", "numdatasyms",
        "paprmode", "version", "preamble", "inputmode", "reservedbiasbits", "l1scrambled", "inband")]


class _BbParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("framesize", "rate", "mode", "inband", "fecblocks", "tsrate")]


class _LdpcParams(ctypes.Structure):
    _fields_ = [("framesize", ctypes.c_int), ("rate", ctypes.c_int)]


class _ImParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("framesize", "rate", "constellation", "rotation")]


class _PgParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "carriermode", "fftsize", "pilotpattern", "guardinterval", "numdatasyms", "paprmode", "version",
        "preamble", "misogroup", "equalization", "bandwidth", "vlength")]


class _ChainParams(ctypes.Structure):
    _fields_ = [("fm", _FmParams), ("misogroup", ctypes.c_int), ("equalization", ctypes.c_int),
                ("bandwidth", ctypes.c_int), ("max_frames", ctypes.c_int), ("tsrate", ctypes.c_int)]


MAX_PLP = 8   # DVBT2LL_MAX_PLP
ABI_VERSION = 2   # DVBT2LL_ABI_VERSION


class _PlpParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "framesize", "rate", "constellation", "rotation", "fecblocks", "tiblocks", "inputmode", "inband", "tsrate",
        "plp_type", "ti_type", "ti_frames", "frame_interval", "first_frame_idx")]


PLP_INTS = len(_PlpParams._fields_)


class _MplpParams(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "carriermode", "fftsize", "guardinterval", "l1constellation", "pilotpattern", "t2frames", "numdatasyms",
        "paprmode", "version", "preamble", "reservedbiasbits", "l1scrambled", "nplp")] + [
        ("plp", _PlpParams * MAX_PLP), ("num_subslices", ctypes.c_int)]

    @classmethod
    def from_config(cls, mcfg):
        """dvbt2ll_mplp_params of a dvbt2ll.configs.MplpConfig"""
        a = mcfg.mplp_array()
        p = cls(*a[:13])
        for k in range(MAX_PLP):
            p.plp[k] = _PlpParams(*a[13 + PLP_INTS * k:13 + PLP_INTS * (k + 1)])
        p.num_subslices = a[13 + PLP_INTS * MAX_PLP]
        return p


class _MplpChainParams(ctypes.Structure):
    _fields_ = [("fm", _MplpParams), ("misogroup", ctypes.c_int), ("equalization", ctypes.c_int),
                ("bandwidth", ctypes.c_int), ("max_frames", ctypes.c_int)]


class _ChainInfo(ctypes.Structure):
    _fields_ = [("fec_blocks_per_frame", ctypes.c_int), ("payload_bytes_per_block", ctypes.c_int),
                ("ts_bytes_per_frame", ctypes.c_int64), ("iq_samples_per_frame", ctypes.c_int64),
                ("cell_size", ctypes.c_int), ("stream_items", ctypes.c_int), ("mapped_items", ctypes.c_int),
                ("num_symbols", ctypes.c_int), ("fft_size", ctypes.c_int), ("guard_interval", ctypes.c_int),
                ("cw_stride_bytes", ctypes.c_int64), ("frames_per_if", ctypes.c_int)]


BLOCKS = ("bbheaderbch", "ldpc", "interleavermod", "framemapperfint", "pilotgenp1insert")
PARAMS = {"bbheaderbch": _BbParams, "ldpc": _LdpcParams, "interleavermod": _ImParams,
          "framemapperfint": _FmParams, "pilotgenp1insert": _PgParams}

# every symbol include/dvbt2ll_hip.h declares (checked by the CPU test suite)
EXPORTS = ["dvbt2ll_strerror", "dvbt2ll_version", "dvbt2ll_device_count", "dvbt2ll_abi_version", "dvbt2ll_abi_check"]
for _b in BLOCKS:
    EXPORTS += ["dvbt2ll_%s_%s" % (_b, f) for f in
                ("create", "output_multiple", "forecast", "general_work", "destroy")]
EXPORTS += ["dvbt2ll_framemapperfint_stream_items", "dvbt2ll_pilotgenp1insert_active_items",
            "dvbt2ll_pilotgenp1insert_debug_carriers", "dvbt2ll_bbheaderbch_sync_errors"]
EXPORTS += ["dvbt2ll_bbheaderbch_set_isi"]
EXPORTS += ["dvbt2ll_framemapper_mplp_" + f for f in ("create", "output_multiple", "stream_items", "forecast",
                                                      "general_work", "destroy")]
EXPORTS += ["dvbt2ll_chain_" + f for f in ("host_submit", "host_wait", "run_host_pipelined", "run_plps_host")]
EXPORTS += ["dvbt2ll_host_alloc", "dvbt2ll_host_free"]
EXPORTS += ["dvbt2ll_chain_" + f for f in ("create_mplp", "num_plps", "unit_frames", "get_plp_info", "run_plps",
                                           "debug_plp_codewords", "debug_keep_codewords")]
EXPORTS += ["dvbt2ll_chain_" + f for f in ("create", "get_info", "run_device", "run_streams", "run_host", "set_output", "set_slots", "set_graph", "set_timing",
                                           "get_timing", "debug_codewords", "debug_cell_pairs", "debug_cells",
                                           "synchronize", "sync_errors",
                                           "destroy")]


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not LIB_PATH.exists():
        raise DVBT2Error("%s is missing: run __graft_entry__.build() (no CPU fallback exists)" % LIB_PATH)
    L = ctypes.CDLL(str(LIB_PATH))
    vp, ci, i64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
    L.dvbt2ll_strerror.restype = ctypes.c_char_p
    L.dvbt2ll_strerror.argtypes = [ci]
    L.dvbt2ll_version.restype = ctypes.c_char_p
    L.dvbt2ll_device_count.restype = ci
    L.dvbt2ll_abi_version.restype = ci
    L.dvbt2ll_abi_check.argtypes = [ci] + [ctypes.c_size_t] * 5
    # this mirror's struct layouts must be the library's (include/dvbt2ll_hip.h DVBT2LL_ABI_VERSION)
    if L.dvbt2ll_abi_check(ABI_VERSION, ctypes.sizeof(_ChainParams), ctypes.sizeof(_ChainInfo),
                           ctypes.sizeof(_PlpParams), ctypes.sizeof(_MplpParams), ctypes.sizeof(_MplpChainParams)):
        raise DVBT2Error("%s: ABI version %d with other struct layouts than this mirror's (ABI %d)"
                         % (LIB_PATH, L.dvbt2ll_abi_version(), ABI_VERSION))
    for b in BLOCKS:
        getattr(L, "dvbt2ll_%s_create" % b).argtypes = [ctypes.POINTER(PARAMS[b]), ci, ctypes.POINTER(vp)]
        getattr(L, "dvbt2ll_%s_output_multiple" % b).argtypes = [vp]
        getattr(L, "dvbt2ll_%s_forecast" % b).argtypes = [vp, ci, ctypes.POINTER(ci)]
        getattr(L, "dvbt2ll_%s_general_work" % b).argtypes = [vp, ci, ci, vp, vp, ctypes.POINTER(ci)]
        getattr(L, "dvbt2ll_%s_destroy" % b).argtypes = [vp]
        getattr(L, "dvbt2ll_%s_destroy" % b).restype = None
    L.dvbt2ll_framemapperfint_stream_items.argtypes = [vp]
    L.dvbt2ll_pilotgenp1insert_active_items.argtypes = [vp]
    L.dvbt2ll_pilotgenp1insert_debug_carriers.argtypes = [vp, vp, vp]
    L.dvbt2ll_chain_create.argtypes = [ctypes.POINTER(_ChainParams), ci, ctypes.POINTER(vp)]
    L.dvbt2ll_chain_get_info.argtypes = [vp, ctypes.POINTER(_ChainInfo)]
    L.dvbt2ll_chain_run_device.argtypes = [vp, vp, i64, i64, i64, ci, vp, vp]
    L.dvbt2ll_chain_run_streams.argtypes = [vp, vp, i64, ci, i64, i64, i64, ci, vp, vp]
    L.dvbt2ll_chain_run_host.argtypes = [vp, vp, i64, i64, i64, ci, vp]
    L.dvbt2ll_chain_set_output.argtypes = [vp, ctypes.c_float, ci]
    L.dvbt2ll_chain_host_submit.argtypes = [vp, vp, i64, i64, i64, ci, vp, ctypes.POINTER(i64)]
    L.dvbt2ll_chain_host_wait.argtypes = [vp, i64]
    L.dvbt2ll_chain_run_plps_host.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(i64), ctypes.POINTER(i64), i64,
                                              ci, vp]
    L.dvbt2ll_chain_run_host_pipelined.argtypes = [vp, vp, i64, i64, i64, ci, vp, ci]
    L.dvbt2ll_host_alloc.restype = vp
    L.dvbt2ll_host_alloc.argtypes = [ctypes.c_size_t]
    L.dvbt2ll_host_free.argtypes = [vp]
    L.dvbt2ll_host_free.restype = None
    L.dvbt2ll_chain_set_slots.argtypes = [vp, ci]
    L.dvbt2ll_chain_set_graph.argtypes = [vp, ci]
    L.dvbt2ll_chain_set_timing.argtypes = [vp, ci]
    L.dvbt2ll_chain_get_timing.argtypes = [vp, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(i64), ci]
    L.dvbt2ll_chain_debug_codewords.argtypes = [vp, vp, i64]
    L.dvbt2ll_chain_debug_keep_codewords.argtypes = [vp, ci]
    L.dvbt2ll_chain_debug_cell_pairs.argtypes = [vp, vp, i64]
    L.dvbt2ll_chain_debug_cells.argtypes = [vp, vp, i64]
    L.dvbt2ll_chain_synchronize.argtypes = [vp]
    L.dvbt2ll_chain_sync_errors.argtypes = [vp, ctypes.POINTER(i64)]
    L.dvbt2ll_bbheaderbch_sync_errors.argtypes = [vp]
    L.dvbt2ll_bbheaderbch_sync_errors.restype = i64
    L.dvbt2ll_bbheaderbch_set_isi.argtypes = [vp, ci]
    L.dvbt2ll_framemapper_mplp_create.argtypes = [ctypes.POINTER(_MplpParams), ci, ctypes.POINTER(vp)]
    L.dvbt2ll_framemapper_mplp_output_multiple.argtypes = [vp]
    L.dvbt2ll_framemapper_mplp_stream_items.argtypes = [vp, ci]
    L.dvbt2ll_framemapper_mplp_forecast.argtypes = [vp, ci, ctypes.POINTER(ci)]
    L.dvbt2ll_framemapper_mplp_general_work.argtypes = [vp, ci, ctypes.POINTER(ci), ctypes.POINTER(vp), vp,
                                                        ctypes.POINTER(ci)]
    L.dvbt2ll_framemapper_mplp_destroy.argtypes = [vp]
    L.dvbt2ll_framemapper_mplp_destroy.restype = None
    L.dvbt2ll_chain_create_mplp.argtypes = [ctypes.POINTER(_MplpChainParams), ci, ctypes.POINTER(vp)]
    L.dvbt2ll_chain_num_plps.argtypes = [vp]
    L.dvbt2ll_chain_unit_frames.argtypes = [vp]
    L.dvbt2ll_chain_get_plp_info.argtypes = [vp, ci, ctypes.POINTER(_ChainInfo)]
    L.dvbt2ll_chain_run_plps.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(i64), ctypes.POINTER(i64), i64, ci,
                                         vp, vp]
    L.dvbt2ll_chain_debug_plp_codewords.argtypes = [vp, ci, vp, i64]
    L.dvbt2ll_chain_destroy.argtypes = [vp]
    L.dvbt2ll_chain_destroy.restype = None
    _lib = L
    return L


def check(status, what):
    if status < 0:
        msg = lib().dvbt2ll_strerror(status).decode()
        if status == -2:
            raise MemoryError("%s: %s" % (what, msg))     # reference: std::bad_alloc
        raise DVBT2Error("%s failed (%d): %s" % (what, status, msg))
    return status
