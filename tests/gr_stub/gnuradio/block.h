// Test-only stand-in for GNU Radio 3.7's gr::block (GNU Radio is not installed in this image): the members the dvbt2ll HIP adapters use
// (io signatures, set_output_multiple, forecast, general_work, consume_each, d_logger) plus two
// accessors the test scheduler (tests/adapter/gr_flowgraph.cpp) reads after each call.
#pragma once
#include <complex>
#include <cstdio>
#include <memory>
#include <string>
#include <vector>

#include <boost/shared_ptr.hpp>
#include <gnuradio/io_signature.h>

typedef std::vector<int> gr_vector_int;
typedef std::vector<const void *> gr_vector_const_void_star;
typedef std::vector<void *> gr_vector_void_star;
typedef std::complex<float> gr_complex;

namespace gr {
struct logger {
  std::string name;
  int warnings = 0;
};
typedef boost::shared_ptr<logger> logger_ptr;

class block {
 public:
  block() {}
  block(const std::string &name, io_signature::sptr in, io_signature::sptr out)
      : d_logger(std::make_shared<logger>()), d_name(name), d_in(in), d_out(out) {
    d_logger->name = name;
  }
  virtual ~block() {}
  virtual void forecast(int noutput_items, gr_vector_int &ninput_items_required) {
    for (auto &n : ninput_items_required) n = noutput_items;
  }
  virtual int general_work(int noutput_items, gr_vector_int &ninput_items, gr_vector_const_void_star &input_items,
                           gr_vector_void_star &output_items) = 0;
  void set_output_multiple(int multiple) { d_output_multiple = multiple; }
  int output_multiple() const { return d_output_multiple; }
  void consume_each(int how_many_items) { d_consumed = how_many_items; }
  const std::string &name() const { return d_name; }
  io_signature::sptr input_signature() const { return d_in; }
  io_signature::sptr output_signature() const { return d_out; }
  // test scheduler hooks (not GNU Radio API)
  int stub_take_consumed() {
    int c = d_consumed;
    d_consumed = 0;
    return c;
  }
  int stub_warnings() const { return d_logger ? d_logger->warnings : 0; }

 protected:
  logger_ptr d_logger;

 private:
  std::string d_name;
  io_signature::sptr d_in, d_out;
  int d_output_multiple = 1;
  int d_consumed = 0;
};
}  // namespace gr

#define GR_LOG_WARN(log, msg)                                                          \
  do {                                                                                 \
    (log)->warnings++;                                                                 \
    std::fprintf(stderr, "WARN %s: %s\n", (log)->name.c_str(), std::string(msg).c_str()); \
  } while (0)

namespace gnuradio {
template <class T>
boost::shared_ptr<T> get_initial_sptr(T *p) {
  return boost::shared_ptr<T>(p);
}
}  // namespace gnuradio
