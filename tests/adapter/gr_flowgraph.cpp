// gr_flowgraph.cpp -- test driver: the shipped flowgraph (apps/vv009-4kshort.grc:1695-1736:
// TS source -> bbheaderbch_bb -> ldpc -> interleavermod_bc -> framemapperfint_cc ->
// pilotgenp1insert_cc -> sink) built from the header-only gr::dvbt2ll::*_impl adapters
// (include/dvbt2ll/*_impl_hip.h) and run by a small scheduler that calls them the way GNU Radio's
// does: per block, pick noutput_items as a (random) multiple of the output multiple, shrink it
// until forecast() is satisfied by the items waiting on the input buffer, call general_work()
// with all of them available, then advance the input by what consume_each() reported and the
// output by the return value.  The TS source delivers the file in random-size chunks.
//
//   gr_flowgraph TS_FILE IQ_OUT NFRAMES SEED  framesize rate constellation rotation fecblocks
//                tiblocks carriermode fftsize guardinterval l1constellation pilotpattern t2frames
//                numdatasyms paprmode version preamble inputmode reservedbiasbits l1scrambled inband
//                misogroup equalization bandwidth tsrate
//
// Writes NFRAMES T2 frames of complex64 IQ; prints the calls and warnings per block.  Test-only
// (built against the stand-in GNU Radio headers in tests/gr_stub), not part of the product.
#define DVBT2LL_HIP_DEFINE_MAKE 1
#include <dvbt2ll/bbheaderbch_bb_impl_hip.h>
#include <dvbt2ll/framemapperfint_cc_impl_hip.h>
#include <dvbt2ll/interleavermod_bc_impl_hip.h>
#include <dvbt2ll/ldpc_bb_impl_hip.h>
#include <dvbt2ll/pilotgenp1insert_cc_impl_hip.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <exception>
#include <random>
#include <vector>

namespace {

// a block's output buffer: items appended at the end, read from rd
struct Buffer {
  size_t itemsize;
  std::vector<uint8_t> data;
  size_t rd = 0;
  explicit Buffer(size_t sz) : itemsize(sz) {}
  size_t items() const { return data.size() / itemsize - rd; }
  const void *read_ptr() const { return data.data() + rd * itemsize; }
  void consume(size_t n) {
    rd += n;
    if (rd * itemsize > (1u << 24)) {   // compact now and then
      data.erase(data.begin(), data.begin() + rd * itemsize);
      rd = 0;
    }
  }
  void append(const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    data.insert(data.end(), b, b + n * itemsize);
  }
};

struct Node {
  std::shared_ptr<gr::block> blk;
  Buffer *in, *out;
  long calls;
  Node(std::shared_ptr<gr::block> b, Buffer *i, Buffer *o) : blk(b), in(i), out(o), calls(0) {}
};

int pilotgen_points(int fftsize) {
  static const int pts[12] = {2048, 8192, 4096, 1024, 16384, 32768, 8192, 32768, 0, 0, 0, 16384};
  return fftsize >= 0 && fftsize < 12 ? pts[fftsize] : 0;
}

}  // namespace

int main(int argc, char **argv) {
  if (argc != 5 + 24) {
    std::fprintf(stderr, "usage: gr_flowgraph TS_FILE IQ_OUT NFRAMES SEED <24 chain parameters>\n");
    return 2;
  }
  int v[24];
  for (int i = 0; i < 24; i++) v[i] = std::atoi(argv[5 + i]);
  const int nframes = std::atoi(argv[3]);
  std::mt19937 rng((unsigned)std::atoi(argv[4]));
  enum { FS, RATE, CONST, ROT, FEC, TI, CAR, FFT, GI, L1C, PP, T2F, NSYM, PAPR, VER, PRE, INM, RBB, L1S, INB, MISO,
         EQ, BW, TSR };
  FILE *f = std::fopen(argv[1], "rb");
  if (!f) { std::perror("ts file"); return 2; }
  std::vector<uint8_t> ts;
  for (int c; (c = std::fgetc(f)) != EOF;) ts.push_back((uint8_t)c);
  std::fclose(f);

  using namespace gr::dvbt2ll;
  try {
    Buffer b_ts(1), b_bb(1), b_ldpc(1), b_cells(sizeof(gr_complex)), b_mapped(sizeof(gr_complex)),
        b_iq(sizeof(gr_complex));
    std::vector<Node> g = {
        {bbheaderbch_bb::make((dvbt2_framesize_t)v[FS], (dvbt2_code_rate_t)v[RATE], (dvbt2_inputmode_t)v[INM],
                              (dvbt2_inband_t)v[INB], v[FEC], v[TSR]),
         &b_ts, &b_bb},
        {ldpc_bb::make((dvbt2_framesize_t)v[FS], (dvbt2_code_rate_t)v[RATE]), &b_bb, &b_ldpc},
        {interleavermod_bc::make((dvbt2_framesize_t)v[FS], (dvbt2_code_rate_t)v[RATE],
                                 (dvbt2_constellation_t)v[CONST], (dvbt2_rotation_t)v[ROT]),
         &b_ldpc, &b_cells},
        {framemapperfint_cc::make((dvbt2_framesize_t)v[FS], (dvbt2_code_rate_t)v[RATE], (dvbt2_constellation_t)v[CONST],
                                  (dvbt2_rotation_t)v[ROT], v[FEC], v[TI], (dvbt2_extended_carrier_t)v[CAR],
                                  (dvbt2_fftsize_t)v[FFT], (dvbt2_guardinterval_t)v[GI],
                                  (dvbt2_l1constellation_t)v[L1C], (dvbt2_pilotpattern_t)v[PP], v[T2F], v[NSYM],
                                  (dvbt2_papr_t)v[PAPR], (dvbt2_version_t)v[VER], (dvbt2_preamble_t)v[PRE],
                                  (dvbt2_inputmode_t)v[INM], (dvbt2_reservedbiasbits_t)v[RBB],
                                  (dvbt2_l1scrambled_t)v[L1S], (dvbt2_inband_t)v[INB]),
         &b_cells, &b_mapped},
        {pilotgenp1insert_cc::make((dvbt2_extended_carrier_t)v[CAR], (dvbt2_fftsize_t)v[FFT], (dvbt2_pilotpattern_t)v[PP],
                                   (dvbt2_guardinterval_t)v[GI], v[NSYM], (dvbt2_papr_t)v[PAPR],
                                   (dvbt2_version_t)v[VER], (dvbt2_preamble_t)v[PRE], (dvbt2_misogroup_t)v[MISO],
                                   (dvbt2_equalization_t)v[EQ], (dvbt2_bandwidth_t)v[BW], pilotgen_points(v[FFT])),
         &b_mapped, &b_iq},
    };
    const size_t frame_iq = (size_t)g.back().blk->output_multiple();
    const size_t want = frame_iq * (size_t)nframes;
    size_t ts_pos = 0;
    std::vector<uint8_t> scratch;
    long idle = 0;
    while (b_iq.items() < want) {
      bool progress = false;
      if (ts_pos < ts.size()) {   // source: a random-size chunk of the TS file
        const size_t n = std::min(ts.size() - ts_pos, (size_t)(1 + rng() % 30000));
        b_ts.append(ts.data() + ts_pos, n);
        ts_pos += n;
        progress = true;
      }
      for (auto &nd : g) {
        const int om = nd.blk->output_multiple();
        for (int k = 1 + (int)(rng() % 3); k >= 1; k--) {   // shrink the request until forecast fits
          const int nout = k * om;
          gr_vector_int req(1, 0);
          nd.blk->forecast(nout, req);
          if ((size_t)req[0] > nd.in->items()) continue;
          gr_vector_int nin(1, (int)nd.in->items());
          gr_vector_const_void_star ins(1, nd.in->read_ptr());
          scratch.assign((size_t)nout * nd.out->itemsize, 0);
          gr_vector_void_star outs(1, scratch.data());
          const int produced = nd.blk->general_work(nout, nin, ins, outs);
          const int consumed = nd.blk->stub_take_consumed();
          if (produced < 0 || produced > nout || consumed < 0 || (size_t)consumed > nd.in->items()) {
            std::fprintf(stderr, "%s: bad general_work result %d / consumed %d\n", nd.blk->name().c_str(), produced,
                         consumed);
            return 1;
          }
          nd.in->consume((size_t)consumed);
          nd.out->append(scratch.data(), (size_t)produced);
          nd.calls++;
          if (produced || consumed) progress = true;
          break;
        }
      }
      if (!progress && ++idle > 2) {
        std::fprintf(stderr, "flowgraph stalled at %zu of %zu IQ samples\n", b_iq.items(), want);
        return 1;
      }
    }
    FILE *o = std::fopen(argv[2], "wb");
    if (!o || std::fwrite(b_iq.read_ptr(), sizeof(gr_complex), want, o) != want) {
      std::perror("iq out");
      return 1;
    }
    std::fclose(o);
    for (auto &nd : g)
      std::printf("%s calls=%ld warnings=%d\n", nd.blk->name().c_str(), nd.calls, nd.blk->stub_warnings());
  } catch (const std::exception &e) {
    std::fprintf(stderr, "gr_flowgraph: %s\n", e.what());
    return 1;
  }
  return 0;
}
