"""Enumerations of include/dvbt2ll/dvbt2ll_config.h:60-202 (same names and values)."""
# dvbt2_code_rate_t
C1_2, C3_5, C2_3, C3_4, C4_5, C5_6, C1_3, C2_5 = range(8)
# dvbt2_constellation_t
MOD_QPSK, MOD_16QAM, MOD_64QAM, MOD_256QAM = range(4)
# dvbt2_rotation_t
ROTATION_OFF, ROTATION_ON = range(2)
# dvbt2_framesize_t
FECFRAME_SHORT, FECFRAME_NORMAL = range(2)
# dvbt2_streamtype_t
STREAMTYPE_TS, STREAMTYPE_GS, STREAMTYPE_BOTH = range(3)
# dvbt2_inputmode_t
INPUTMODE_NORMAL, INPUTMODE_HIEFF = range(2)
# dvbt2_extended_carrier_t
CARRIERS_NORMAL, CARRIERS_EXTENDED = range(2)
# dvbt2_preamble_t
PREAMBLE_T2_SISO, PREAMBLE_T2_MISO, PREAMBLE_NON_T2, PREAMBLE_T2_LITE_SISO, PREAMBLE_T2_LITE_MISO = range(5)
# dvbt2_fftsize_t
FFTSIZE_2K, FFTSIZE_8K, FFTSIZE_4K, FFTSIZE_1K, FFTSIZE_16K, FFTSIZE_32K, FFTSIZE_8K_T2GI, FFTSIZE_32K_T2GI = range(8)
FFTSIZE_16K_T2GI = 11
# dvbt2_guardinterval_t
GI_1_32, GI_1_16, GI_1_8, GI_1_4, GI_1_128, GI_19_128, GI_19_256 = range(7)
# dvbt2_papr_t
PAPR_OFF, PAPR_ACE, PAPR_TR, PAPR_BOTH = range(4)
# dvbt2_l1constellation_t
L1_MOD_BPSK, L1_MOD_QPSK, L1_MOD_16QAM, L1_MOD_64QAM = range(4)
# dvbt2_pilotpattern_t
PILOT_PP1, PILOT_PP2, PILOT_PP3, PILOT_PP4, PILOT_PP5, PILOT_PP6, PILOT_PP7, PILOT_PP8 = range(8)
# dvbt2_version_t
VERSION_111, VERSION_121, VERSION_131 = range(3)
# dvbt2_reservedbiasbits_t
RESERVED_OFF, RESERVED_ON = range(2)
# dvbt2_l1scrambled_t
L1_SCRAMBLED_OFF, L1_SCRAMBLED_ON = range(2)
# dvbt2_misogroup_t
MISO_TX1, MISO_TX2 = range(2)
# dvbt2_showlevels_t
SHOWLEVELS_OFF, SHOWLEVELS_ON = range(2)
# dvbt2_inband_t
INBAND_OFF, INBAND_ON = range(2)
# dvbt2_equalization_t
EQUALIZATION_OFF, EQUALIZATION_ON = range(2)
# dvbt2_bandwidth_t
BANDWIDTH_1_7_MHZ, BANDWIDTH_5_0_MHZ, BANDWIDTH_6_0_MHZ, BANDWIDTH_7_0_MHZ, BANDWIDTH_8_0_MHZ, BANDWIDTH_10_0_MHZ = range(6)
