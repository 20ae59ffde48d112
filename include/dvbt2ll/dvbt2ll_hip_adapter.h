// dvbt2ll_hip_adapter.h -- shared pieces of the header-only gr::dvbt2ll::*_impl adapters that put
// libdvbt2ll_hip.so (include/dvbt2ll_hip.h) behind gr-dvbt2ll's GNU Radio block API.
//
// Each adapter replaces one reference lib/<block>_impl.{h,cc}: same class name, same make()
// arguments, same set_output_multiple / forecast / general_work / consume_each contract.  A
// maintainer includes the five *_impl_hip.h headers from one .cc of the module with
// DVBT2LL_HIP_DEFINE_MAKE defined (that TU then defines the make() factories) and links the
// module against libdvbt2ll_hip.so; INTEGRATION.md has the CMake lines.
//
// Errors: the reference throws std::bad_alloc from its constructors (e.g. framemapperfint_cc_impl.cc
// :1121-1130) and otherwise only logs; the ABI returns negative status codes, rethrown here as
// std::bad_alloc (DVBT2LL_ENOMEM) or std::runtime_error (everything else).
// Device: the HIP device the blocks run on is DVBT2LL_DEVICE from the environment (default 0).
#ifndef DVBT2LL_HIP_ADAPTER_H
#define DVBT2LL_HIP_ADAPTER_H

#include <cstdlib>
#include <new>
#include <stdexcept>
#include <string>

#include "../dvbt2ll_hip.h"

namespace gr {
namespace dvbt2ll {
namespace hip {

inline int check(int status, const char *what) {
  if (status == DVBT2LL_ENOMEM) throw std::bad_alloc();
  if (status < 0) throw std::runtime_error(std::string(what) + ": " + dvbt2ll_strerror(status));
  return status;
}

// every adapter constructor calls this before its create: the library's struct layouts must be this header's
inline int device() {
  check(DVBT2LL_ABI_CHECK(), "libdvbt2ll_hip.so ABI version / struct layouts differ from dvbt2ll_hip.h");
  const char *e = std::getenv("DVBT2LL_DEVICE");
  return e ? std::atoi(e) : 0;
}

}  // namespace hip
}  // namespace dvbt2ll
}  // namespace gr

#endif
