// Test-only stand-in for gr-dvbt2ll's public block header include/dvbt2ll/framemapperfint_cc.h:36-49 (the
// abstract block with its make() factory), so the HIP adapter compiles without GNU Radio.
#pragma once
#include <dvbt2ll/dvbt2ll_config.h>
#include <gnuradio/block.h>

namespace gr {
namespace dvbt2ll {
class framemapperfint_cc : virtual public gr::block {
 public:
  typedef std::shared_ptr<framemapperfint_cc> sptr;
  static sptr make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_constellation_t constellation, dvbt2_rotation_t rotation, int fecblocks, int tiblocks, dvbt2_extended_carrier_t carriermode, dvbt2_fftsize_t fftsize, dvbt2_guardinterval_t guardinterval, dvbt2_l1constellation_t l1constellation, dvbt2_pilotpattern_t pilotpattern, int t2frames, int numdatasyms, dvbt2_papr_t paprmode, dvbt2_version_t version, dvbt2_preamble_t preamble, dvbt2_inputmode_t inputmode, dvbt2_reservedbiasbits_t reservedbiasbits, dvbt2_l1scrambled_t l1scrambled, dvbt2_inband_t inband);
};
}  // namespace dvbt2ll
}  // namespace gr
