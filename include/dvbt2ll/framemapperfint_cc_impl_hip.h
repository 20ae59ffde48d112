// framemapperfint_cc_impl_hip.h -- gr::dvbt2ll::framemapperfint_cc_impl over libdvbt2ll_hip.so.
// Replaces lib/framemapperfint_cc_impl.{h,cc}: make() include/dvbt2ll/framemapperfint_cc.h:49,
// ctor :41-1190 (set_output_multiple(mapped_items) :1135 / :1159), forecast :1942-1946,
// general_work :1948-2151 (consume_each(stream_items) :2147).
//
// Return value: the reference consumes exactly one T2 frame per call (:2147) but returns
// noutput_items, so for noutput_items >= 2 mapped_items everything after the first frame is stale
// buffer content.  The ABI produces the one frame it consumed and returns mapped_items, which GNU
// Radio's general_work contract allows (items produced <= noutput_items); the stream is identical
// to the reference's wherever the reference's is valid.
#ifndef DVBT2LL_FRAMEMAPPERFINT_CC_IMPL_HIP_H
#define DVBT2LL_FRAMEMAPPERFINT_CC_IMPL_HIP_H

#include <dvbt2ll/framemapperfint_cc.h>
#include <gnuradio/io_signature.h>

#include "dvbt2ll_hip_adapter.h"

namespace gr {
namespace dvbt2ll {

class framemapperfint_cc_impl : public framemapperfint_cc {
 public:
  framemapperfint_cc_impl(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_constellation_t constellation,
                          dvbt2_rotation_t rotation, int fecblocks, int tiblocks,
                          dvbt2_extended_carrier_t carriermode, dvbt2_fftsize_t fftsize,
                          dvbt2_guardinterval_t guardinterval, dvbt2_l1constellation_t l1constellation,
                          dvbt2_pilotpattern_t pilotpattern, int t2frames, int numdatasyms, dvbt2_papr_t paprmode,
                          dvbt2_version_t version, dvbt2_preamble_t preamble, dvbt2_inputmode_t inputmode,
                          dvbt2_reservedbiasbits_t reservedbiasbits, dvbt2_l1scrambled_t l1scrambled,
                          dvbt2_inband_t inband)
      : gr::block("framemapperfint_cc", gr::io_signature::make(1, 1, sizeof(gr_complex)),
                  gr::io_signature::make(1, 1, sizeof(gr_complex))) {
    const dvbt2ll_framemapperfint_params p = {
        (int)framesize,       (int)rate,      (int)constellation, (int)rotation,   fecblocks,
        tiblocks,             (int)carriermode, (int)fftsize,     (int)guardinterval, (int)l1constellation,
        (int)pilotpattern,    t2frames,       numdatasyms,        (int)paprmode,   (int)version,
        (int)preamble,        (int)inputmode, (int)reservedbiasbits, (int)l1scrambled, (int)inband};
    hip::check(dvbt2ll_framemapperfint_create(&p, hip::device(), &d_h), "framemapperfint_cc");
    set_output_multiple(dvbt2ll_framemapperfint_output_multiple(d_h));
  }
  ~framemapperfint_cc_impl() { dvbt2ll_framemapperfint_destroy(d_h); }

  void forecast(int noutput_items, gr_vector_int &ninput_items_required) {
    hip::check(dvbt2ll_framemapperfint_forecast(d_h, noutput_items, &ninput_items_required[0]), "forecast");
  }

  int general_work(int noutput_items, gr_vector_int &ninput_items, gr_vector_const_void_star &input_items,
                   gr_vector_void_star &output_items) {
    int consumed = 0;
    const int produced = hip::check(dvbt2ll_framemapperfint_general_work(d_h, noutput_items, ninput_items[0],
                                                                         input_items[0], output_items[0], &consumed),
                                    "framemapperfint_cc general_work");
    consume_each(consumed);
    return produced;
  }

 private:
  dvbt2ll_framemapperfint *d_h = nullptr;
};

#ifdef DVBT2LL_HIP_DEFINE_MAKE
framemapperfint_cc::sptr framemapperfint_cc::make(
    dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_constellation_t constellation,
    dvbt2_rotation_t rotation, int fecblocks, int tiblocks, dvbt2_extended_carrier_t carriermode,
    dvbt2_fftsize_t fftsize, dvbt2_guardinterval_t guardinterval, dvbt2_l1constellation_t l1constellation,
    dvbt2_pilotpattern_t pilotpattern, int t2frames, int numdatasyms, dvbt2_papr_t paprmode, dvbt2_version_t version,
    dvbt2_preamble_t preamble, dvbt2_inputmode_t inputmode, dvbt2_reservedbiasbits_t reservedbiasbits,
    dvbt2_l1scrambled_t l1scrambled, dvbt2_inband_t inband) {
  return gnuradio::get_initial_sptr(new framemapperfint_cc_impl(
      framesize, rate, constellation, rotation, fecblocks, tiblocks, carriermode, fftsize, guardinterval,
      l1constellation, pilotpattern, t2frames, numdatasyms, paprmode, version, preamble, inputmode, reservedbiasbits,
      l1scrambled, inband));
}
#endif

}  // namespace dvbt2ll
}  // namespace gr

#endif
