// Test-only stand-in for GNU Radio's gr::io_signature (just enough for the dvbt2ll HIP adapters;
// GNU Radio is not installed in this image).  Not used by the product.
#pragma once
#include <boost/shared_ptr.hpp>

namespace gr {
class io_signature {
 public:
  typedef boost::shared_ptr<io_signature> sptr;
  static sptr make(int min_streams, int max_streams, int sizeof_stream_item) {
    return sptr(new io_signature(min_streams, max_streams, sizeof_stream_item));
  }
  int min_streams() const { return d_min; }
  int max_streams() const { return d_max; }
  int sizeof_stream_item(int) const { return d_size; }

 private:
  io_signature(int mn, int mx, int sz) : d_min(mn), d_max(mx), d_size(sz) {}
  int d_min, d_max, d_size;
};
}  // namespace gr
