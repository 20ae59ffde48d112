// interleavermod_bc_impl_hip.h -- gr::dvbt2ll::interleavermod_bc_impl over libdvbt2ll_hip.so.
// Replaces lib/interleavermod_bc_impl.{h,cc}: make() include/dvbt2ll/interleavermod_bc.h:49,
// ctor :42-255 (set_output_multiple(cell_size) :254), forecast :264-268, general_work :270-704.
// The reference is only correct for up to 64800 / cell_size FEC blocks per call (larger
// calls overrun its 64800-cell buffer); here any whole number of blocks per call is encoded.
#ifndef DVBT2LL_INTERLEAVERMOD_BC_IMPL_HIP_H
#define DVBT2LL_INTERLEAVERMOD_BC_IMPL_HIP_H

#include <dvbt2ll/interleavermod_bc.h>
#include <gnuradio/io_signature.h>

#include "dvbt2ll_hip_adapter.h"

namespace gr {
namespace dvbt2ll {

class interleavermod_bc_impl : public interleavermod_bc {
 public:
  interleavermod_bc_impl(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate, dvbt2_constellation_t constellation,
                         dvbt2_rotation_t rotation)
      : gr::block("interleavermod_bc", gr::io_signature::make(1, 1, sizeof(unsigned char)),
                  gr::io_signature::make(1, 1, sizeof(gr_complex))) {
    const dvbt2ll_interleavermod_params p = {(int)framesize, (int)rate, (int)constellation, (int)rotation};
    hip::check(dvbt2ll_interleavermod_create(&p, hip::device(), &d_h), "interleavermod_bc");
    set_output_multiple(dvbt2ll_interleavermod_output_multiple(d_h));
  }
  ~interleavermod_bc_impl() { dvbt2ll_interleavermod_destroy(d_h); }

  void forecast(int noutput_items, gr_vector_int &ninput_items_required) {
    hip::check(dvbt2ll_interleavermod_forecast(d_h, noutput_items, &ninput_items_required[0]), "forecast");
  }

  int general_work(int noutput_items, gr_vector_int &ninput_items, gr_vector_const_void_star &input_items,
                   gr_vector_void_star &output_items) {
    int consumed = 0;
    const int produced = hip::check(dvbt2ll_interleavermod_general_work(d_h, noutput_items, ninput_items[0],
                                                                        input_items[0], output_items[0], &consumed),
                                    "interleavermod_bc general_work");
    consume_each(consumed);
    return produced;
  }

 private:
  dvbt2ll_interleavermod *d_h = nullptr;
};

#ifdef DVBT2LL_HIP_DEFINE_MAKE
interleavermod_bc::sptr interleavermod_bc::make(dvbt2_framesize_t framesize, dvbt2_code_rate_t rate,
                                                dvbt2_constellation_t constellation, dvbt2_rotation_t rotation) {
  return gnuradio::get_initial_sptr(new interleavermod_bc_impl(framesize, rate, constellation, rotation));
}
#endif

}  // namespace dvbt2ll
}  // namespace gr

#endif
