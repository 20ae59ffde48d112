// Test-only stand-in for boost/shared_ptr.hpp (Boost is not installed in this image): GNU Radio
// 3.7's block headers name boost::shared_ptr, which std::shared_ptr replaces here.  Not used by the product.
#pragma once
#include <memory>
namespace boost {
using std::shared_ptr;
}  // namespace boost
