// Test-only stand-in for gr-dvbt2ll's public block header include/dvbt2ll/bbheaderbch_bb.h:36-49 (the
// abstract block with its make() factory), so the HIP adapter compiles without GNU Radio.
#pragma once
#include <dvbt2ll/dvbt2ll_config.h>
#include <gnuradio/block.h>

namespace gr {
namespace dvbt2ll {
class bbheaderbch_bb : virtual public gr::block {
 public:
  typedef std::shared_ptr<bbheaderbch_bb> sptr;
  static sptr make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_inputmode_t mode, dvbt2_inband_t inband, int fecblocks, int tsrate);
};
}  // namespace dvbt2ll
}  // namespace gr
