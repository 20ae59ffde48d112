// bbheaderbch_bb_impl_hip.h -- gr::dvbt2ll::bbheaderbch_bb_impl over libdvbt2ll_hip.so.
// Replaces lib/bbheaderbch_bb_impl.{h,cc}: make() include/dvbt2ll/bbheaderbch_bb.h:49, ctor :42-196
// (set_output_multiple(nbch) :195), forecast :207-216, general_work :648-742 (consume_each :738).
#ifndef DVBT2LL_BBHEADERBCH_BB_IMPL_HIP_H
#define DVBT2LL_BBHEADERBCH_BB_IMPL_HIP_H

#include <dvbt2ll/bbheaderbch_bb.h>
#include <gnuradio/io_signature.h>

#include "dvbt2ll_hip_adapter.h"

namespace gr {
namespace dvbt2ll {

class bbheaderbch_bb_impl : public bbheaderbch_bb {
 public:
  bbheaderbch_bb_impl(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_inputmode_t mode,
                      dvbt2_inband_t inband, int fecblocks, int tsrate)
      : gr::block("bbheaderbch_bb", gr::io_signature::make(1, 1, sizeof(unsigned char)),
                  gr::io_signature::make(1, 1, sizeof(unsigned char))) {
    const dvbt2ll_bbheaderbch_params p = {(int)framesize, (int)rate, (int)mode, (int)inband, fecblocks, tsrate};
    hip::check(dvbt2ll_bbheaderbch_create(&p, hip::device(), &d_h), "bbheaderbch_bb");
    set_output_multiple(dvbt2ll_bbheaderbch_output_multiple(d_h));
  }
  ~bbheaderbch_bb_impl() { dvbt2ll_bbheaderbch_destroy(d_h); }

  void forecast(int noutput_items, gr_vector_int &ninput_items_required) {
    hip::check(dvbt2ll_bbheaderbch_forecast(d_h, noutput_items, &ninput_items_required[0]), "forecast");
  }

  int general_work(int noutput_items, gr_vector_int &ninput_items, gr_vector_const_void_star &input_items,
                   gr_vector_void_star &output_items) {
    int consumed = 0;
    const int produced = hip::check(dvbt2ll_bbheaderbch_general_work(d_h, noutput_items, ninput_items[0],
                                                                     input_items[0], output_items[0], &consumed),
                                    "bbheaderbch_bb general_work");
    // one warning per TS sync byte != 0x47, as the reference logs them (:675-677, :703-705)
    for (const int64_t n = dvbt2ll_bbheaderbch_sync_errors(d_h); d_sync_errors < n; d_sync_errors++)
      GR_LOG_WARN(d_logger, "Transport Stream sync error!");
    consume_each(consumed);
    return produced;
  }

 private:
  dvbt2ll_bbheaderbch *d_h = nullptr;
  int64_t d_sync_errors = 0;
};

#ifdef DVBT2LL_HIP_DEFINE_MAKE
bbheaderbch_bb::sptr bbheaderbch_bb::make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate,
                                          dvbt2_inputmode_t mode, dvbt2_inband_t inband, int fecblocks,
                                          int tsrate) {
  return gnuradio::get_initial_sptr(new bbheaderbch_bb_impl(framesize, rate, mode, inband, fecblocks, tsrate));
}
#endif

}  // namespace dvbt2ll
}  // namespace gr

#endif
