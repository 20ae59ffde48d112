// Test-only stand-in for gr-dvbt2ll's public block header include/dvbt2ll/pilotgenp1insert_cc.h:36-49 (the
// abstract block with its make() factory), so the HIP adapter compiles without GNU Radio.
#pragma once
#include <dvbt2ll/dvbt2ll_config.h>
#include <gnuradio/block.h>

namespace gr {
namespace dvbt2ll {
class pilotgenp1insert_cc : virtual public gr::block {
 public:
  typedef std::shared_ptr<pilotgenp1insert_cc> sptr;
  static sptr make(dvbt2_extended_carrier_t carriermode, dvbt2_fftsize_t fftsize, dvbt2_pilotpattern_t pilotpattern, dvbt2_guardinterval_t guardinterval, int numdatasyms, dvbt2_papr_t paprmode, dvbt2_version_t version, dvbt2_preamble_t preamble, dvbt2_misogroup_t misogroup, dvbt2_equalization_t equalization, dvbt2_bandwidth_t bandwidth, int vlength);
};
}  // namespace dvbt2ll
}  // namespace gr
