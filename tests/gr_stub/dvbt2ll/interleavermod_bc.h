// Test-only stand-in for gr-dvbt2ll's public block header include/dvbt2ll/interleavermod_bc.h:36-49 (the
// abstract block with its make() factory), so the HIP adapter compiles without GNU Radio.
#pragma once
#include <dvbt2ll/dvbt2ll_config.h>
#include <gnuradio/block.h>

namespace gr {
namespace dvbt2ll {
class interleavermod_bc : virtual public gr::block {
 public:
  typedef std::shared_ptr<interleavermod_bc> sptr;
  static sptr make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_constellation_t constellation, dvbt2_rotation_t rotation);
};
}  // namespace dvbt2ll
}  // namespace gr
