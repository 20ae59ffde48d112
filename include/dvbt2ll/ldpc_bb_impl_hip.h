// ldpc_bb_impl_hip.h -- gr::dvbt2ll::ldpc_bb, the LDPC encoder block over libdvbt2ll_hip.so.
// Replaces gr-dtv's dtv::dvb_ldpc_bb::make(STANDARD_DVBT2, framesize, rate, MOD_OTHER), which the
// shipped flowgraph wires between bbheaderbch_bb and interleavermod_bc
// (apps/vv009-4kshort.grc:386-460); arithmetic = lib/bbheaderbch_bb_impl.cc:533-646.
// gr-dvbt2ll has no public header for it, so this header declares the block class too.
#ifndef DVBT2LL_LDPC_BB_IMPL_HIP_H
#define DVBT2LL_LDPC_BB_IMPL_HIP_H

#include <dvbt2ll/dvbt2ll_config.h>
#include <gnuradio/block.h>
#include <gnuradio/io_signature.h>

#include "dvbt2ll_hip_adapter.h"

namespace gr {
namespace dvbt2ll {

class ldpc_bb : virtual public gr::block {
 public:
  typedef boost::shared_ptr<ldpc_bb> sptr;   // GNU Radio 3.7 block pointers
  static sptr make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate);
};

class ldpc_bb_impl : public ldpc_bb {
 public:
  ldpc_bb_impl(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate)
      : gr::block("ldpc_bb", gr::io_signature::make(1, 1, sizeof(unsigned char)),
                  gr::io_signature::make(1, 1, sizeof(unsigned char))) {
    const dvbt2ll_ldpc_params p = {(int)framesize, (int)rate};
    hip::check(dvbt2ll_ldpc_create(&p, hip::device(), &d_h), "ldpc_bb");
    set_output_multiple(dvbt2ll_ldpc_output_multiple(d_h));
  }
  ~ldpc_bb_impl() { dvbt2ll_ldpc_destroy(d_h); }

  void forecast(int noutput_items, gr_vector_int &ninput_items_required) {
    hip::check(dvbt2ll_ldpc_forecast(d_h, noutput_items, &ninput_items_required[0]), "forecast");
  }

  int general_work(int noutput_items, gr_vector_int &ninput_items, gr_vector_const_void_star &input_items,
                   gr_vector_void_star &output_items) {
    int consumed = 0;
    const int produced = hip::check(
        dvbt2ll_ldpc_general_work(d_h, noutput_items, ninput_items[0], input_items[0], output_items[0], &consumed),
        "ldpc_bb general_work");
    consume_each(consumed);
    return produced;
  }

 private:
  dvbt2ll_ldpc *d_h = nullptr;
};

#ifdef DVBT2LL_HIP_DEFINE_MAKE
ldpc_bb::sptr ldpc_bb::make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate) {
  return gnuradio::get_initial_sptr(new ldpc_bb_impl(framesize, rate));
}
#endif

}  // namespace dvbt2ll
}  // namespace gr

#endif
