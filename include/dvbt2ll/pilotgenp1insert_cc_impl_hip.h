// pilotgenp1insert_cc_impl_hip.h -- gr::dvbt2ll::pilotgenp1insert_cc_impl over libdvbt2ll_hip.so.
// Replaces lib/pilotgenp1insert_cc_impl.{h,cc}: make() include/dvbt2ll/pilotgenp1insert_cc.h:49,
// ctor :43-1229 (set_output_multiple(2048 + Nsym (N + GI)) :1228), forecast :1239-1243,
// general_work :2784-2907 (consume_each(active_items) :2903).
// Return value: one T2 frame per call, as framemapperfint_cc_impl_hip.h explains.
#ifndef DVBT2LL_PILOTGENP1INSERT_CC_IMPL_HIP_H
#define DVBT2LL_PILOTGENP1INSERT_CC_IMPL_HIP_H

#include <dvbt2ll/pilotgenp1insert_cc.h>
#include <gnuradio/io_signature.h>

#include "dvbt2ll_hip_adapter.h"

namespace gr {
namespace dvbt2ll {

class pilotgenp1insert_cc_impl : public pilotgenp1insert_cc {
 public:
  pilotgenp1insert_cc_impl(dvbt2_extended_carrier_t carriermode, dvbt2_fftsize_t fftsize,
                           dvbt2_pilotpattern_t pilotpattern, dvbt2_guardinterval_t guardinterval, int numdatasyms,
                           dvbt2_papr_t paprmode, dvbt2_version_t version, dvbt2_preamble_t preamble,
                           dvbt2_misogroup_t misogroup, dvbt2_equalization_t equalization, dvbt2_bandwidth_t bandwidth,
                           int vlength)
      : gr::block("pilotgenp1insert_cc", gr::io_signature::make(1, 1, sizeof(gr_complex)),
                  gr::io_signature::make(1, 1, sizeof(gr_complex))) {
    const dvbt2ll_pilotgenp1insert_params p = {(int)carriermode, (int)fftsize,  (int)pilotpattern, (int)guardinterval,
                                               numdatasyms,      (int)paprmode, (int)version,      (int)preamble,
                                               (int)misogroup,   (int)equalization, (int)bandwidth, vlength};
    hip::check(dvbt2ll_pilotgenp1insert_create(&p, hip::device(), &d_h), "pilotgenp1insert_cc");
    set_output_multiple(dvbt2ll_pilotgenp1insert_output_multiple(d_h));
  }
  ~pilotgenp1insert_cc_impl() { dvbt2ll_pilotgenp1insert_destroy(d_h); }

  void forecast(int noutput_items, gr_vector_int &ninput_items_required) {
    hip::check(dvbt2ll_pilotgenp1insert_forecast(d_h, noutput_items, &ninput_items_required[0]), "forecast");
  }

  int general_work(int noutput_items, gr_vector_int &ninput_items, gr_vector_const_void_star &input_items,
                   gr_vector_void_star &output_items) {
    int consumed = 0;
    const int produced = hip::check(dvbt2ll_pilotgenp1insert_general_work(d_h, noutput_items, ninput_items[0],
                                                                          input_items[0], output_items[0], &consumed),
                                    "pilotgenp1insert_cc general_work");
    consume_each(consumed);
    return produced;
  }

 private:
  dvbt2ll_pilotgenp1insert *d_h = nullptr;
};

#ifdef DVBT2LL_HIP_DEFINE_MAKE
pilotgenp1insert_cc::sptr pilotgenp1insert_cc::make(dvbt2_extended_carrier_t carriermode, dvbt2_fftsize_t fftsize,
                                                    dvbt2_pilotpattern_t pilotpattern,
                                                    dvbt2_guardinterval_t guardinterval, int numdatasyms,
                                                    dvbt2_papr_t paprmode, dvbt2_version_t version,
                                                    dvbt2_preamble_t preamble, dvbt2_misogroup_t misogroup,
                                                    dvbt2_equalization_t equalization, dvbt2_bandwidth_t bandwidth,
                                                    int vlength) {
  return gnuradio::get_initial_sptr(new pilotgenp1insert_cc_impl(carriermode, fftsize, pilotpattern, guardinterval,
                                                                 numdatasyms, paprmode, version, preamble, misogroup,
                                                                 equalization, bandwidth, vlength));
}
#endif

}  // namespace dvbt2ll
}  // namespace gr

#endif
