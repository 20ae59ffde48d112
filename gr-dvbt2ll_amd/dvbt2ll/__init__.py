"""dvbt2ll -- MI355X-native DVB-T2 transmit chain with the gr-dvbt2ll block API.

Python module name and block names follow the reference's SWIG module
(swig/dvbt2ll_swig.i:19-27): dvbt2ll.bbheaderbch_bb, interleavermod_bc, framemapperfint_cc,
pilotgenp1insert_cc (+ ldpc_bb standing in for gr-dtv's dvb_ldpc_bb), all backed by the
HIP/gfx950 library libdvbt2ll_hip.so through its C ABI (include/dvbt2ll_hip.h).
"""
from .enums import *  # noqa: F401,F403
from .blocks import bbheaderbch_bb, ldpc_bb, interleavermod_bc, framemapperfint_cc, pilotgenp1insert_cc  # noqa: F401
from .blocks import framemapper_mplp_cc  # noqa: F401
from .chain import Chain, IQ_CF32, IQ_SC16  # noqa: F401
from .configs import CONFIGS, T2Config, ts_packets, ts_for_frames  # noqa: F401
from .configs import MPLP_CONFIGS, MplpConfig, PlpConfig  # noqa: F401
from ._lib import lib, LIB_PATH, EXPORTS, DVBT2Error  # noqa: F401
