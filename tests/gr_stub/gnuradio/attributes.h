// Test-only stand-in for GNU Radio's gnuradio/attributes.h: the symbol visibility macros that
// gr-dvbt2ll's include/dvbt2ll/api.h uses.  Not used by the product.
#pragma once
#define __GR_ATTR_EXPORT __attribute__((visibility("default")))
#define __GR_ATTR_IMPORT __attribute__((visibility("default")))
