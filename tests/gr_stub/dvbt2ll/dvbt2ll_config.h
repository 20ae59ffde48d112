// Test-only stand-in for gr-dvbt2ll's public enum header (include/dvbt2ll/dvbt2ll_config.h:60-227):
// the same type names, with the numeric values the C ABI takes (dvbt2ll/enums.py lists them).
#pragma once
namespace gr {
namespace dvbt2ll {
enum dvbt2_code_rate_t : int {};
enum dvbt2_constellation_t : int {};
enum dvbt2_rotation_t : int {};
enum dvbt2_framesize_t : int {};
enum dvbt2_inputmode_t : int {};
enum dvbt2_extended_carrier_t : int {};
enum dvbt2_preamble_t : int {};
enum dvbt2_fftsize_t : int {};
enum dvbt2_guardinterval_t : int {};
enum dvbt2_papr_t : int {};
enum dvbt2_l1constellation_t : int {};
enum dvbt2_pilotpattern_t : int {};
enum dvbt2_version_t : int {};
enum dvbt2_reservedbiasbits_t : int {};
enum dvbt2_l1scrambled_t : int {};
enum dvbt2_misogroup_t : int {};
enum dvbt2_inband_t : int {};
enum dvbt2_equalization_t : int {};
enum dvbt2_bandwidth_t : int {};
}  // namespace dvbt2ll
}  // namespace gr
typedef gr::dvbt2ll::dvbt2_code_rate_t dvbt2_code_rate_t;
typedef gr::dvbt2ll::dvbt2_constellation_t dvbt2_constellation_t;
typedef gr::dvbt2ll::dvbt2_rotation_t dvbt2_rotation_t;
typedef gr::dvbt2ll::dvbt2_framesize_t dvbt2_framesize_t;
typedef gr::dvbt2ll::dvbt2_inputmode_t dvbt2_inputmode_t;
typedef gr::dvbt2ll::dvbt2_extended_carrier_t dvbt2_extended_carrier_t;
typedef gr::dvbt2ll::dvbt2_preamble_t dvbt2_preamble_t;
typedef gr::dvbt2ll::dvbt2_fftsize_t dvbt2_fftsize_t;
typedef gr::dvbt2ll::dvbt2_guardinterval_t dvbt2_guardinterval_t;
typedef gr::dvbt2ll::dvbt2_papr_t dvbt2_papr_t;
typedef gr::dvbt2ll::dvbt2_l1constellation_t dvbt2_l1constellation_t;
typedef gr::dvbt2ll::dvbt2_pilotpattern_t dvbt2_pilotpattern_t;
typedef gr::dvbt2ll::dvbt2_version_t dvbt2_version_t;
typedef gr::dvbt2ll::dvbt2_reservedbiasbits_t dvbt2_reservedbiasbits_t;
typedef gr::dvbt2ll::dvbt2_l1scrambled_t dvbt2_l1scrambled_t;
typedef gr::dvbt2ll::dvbt2_misogroup_t dvbt2_misogroup_t;
typedef gr::dvbt2ll::dvbt2_inband_t dvbt2_inband_t;
typedef gr::dvbt2ll::dvbt2_equalization_t dvbt2_equalization_t;
typedef gr::dvbt2ll::dvbt2_bandwidth_t dvbt2_bandwidth_t;
