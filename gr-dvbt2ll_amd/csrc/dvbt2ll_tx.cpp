// dvbt2ll_tx -- native command-line DVB-T2 transmitter over the C ABI (include/dvbt2ll_hip.h):
// MPEG-TS file in, baseband IQ file out, whole T2 frames per GPU call.  It is the file-sink
// form of the shipped flowgraph apps/vv009-4kshort.grc (TS source -> the five blocks ->
// multiply_const -> sink): TS bytes -> the chain's streaming host path (dvbt2ll_chain_host_submit /
// _host_wait: a ring of DVBT2LL_HOST_RING batches in flight, page-locked buffers, so reading batch k + 1,
// encoding batch k and writing batch k - 2 overlap) -> complex64 or sc16 samples.
//
//   dvbt2ll_tx --preset cfg3 --in stream.ts --out iq.sc16 --format sc16 --gain 0.2
//
// The TS is consumed as one continuous stream (absolute offsets from the start of the file);
// frame k is encoded with the stream state the reference blocks would hold at that point.
// Trailing bytes that do not complete a T2 frame are left unused.
#include <cerrno>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "dvbt2ll_hip.h"

namespace {

struct Preset {
  const char *name;
  int framesize, rate, constellation, rotation, fecblocks, tiblocks, carriermode, fftsize, guardinterval,
      l1constellation, pilotpattern, t2frames, numdatasyms;
};
// SURVEY.md section 6 configurations (enum values of include/dvbt2ll/dvbt2ll_config.h:60-202);
// cfg1 is the shipped flowgraph (apps/vv009-4kshort.grc:524-709)
const Preset kPresets[] = {
    {"cfg1", 0, 4, 3, 1, 8, 3, 0, 2, 0, 3, 6, 2, 3},
    {"cfg2", 1, 2, 2, 0, 148, 3, 0, 5, 4, 3, 6, 2, 59},
    {"cfg3", 1, 1, 3, 1, 195, 3, 1, 5, 1, 3, 3, 2, 59},
    {"cfg4", 1, 0, 1, 0, 24, 3, 0, 1, 0, 3, 6, 2, 59},
    {"cfg5", 1, 5, 3, 0, 197, 3, 0, 5, 4, 3, 6, 2, 59},
    {"cfg1q", 0, 0, 0, 1, 2, 3, 0, 2, 0, 3, 6, 2, 3},   // BASELINE config 1 as worded: QPSK 1/2
};

void usage(FILE *f) {
  std::fprintf(f,
               "usage: dvbt2ll_tx --in TS_FILE --out IQ_FILE [options]\n"
               "  --preset cfg1..cfg5|cfg1q parameter preset (default cfg1, the shipped flowgraph)\n"
               "  --set NAME=VALUE        override one chain parameter (framemapperfint_cc names:\n"
               "                          framesize rate constellation rotation fecblocks tiblocks\n"
               "                          carriermode fftsize guardinterval l1constellation\n"
               "                          pilotpattern t2frames numdatasyms paprmode version preamble\n"
               "                          inputmode reservedbiasbits l1scrambled inband; pilotgen:\n"
               "                          misogroup equalization bandwidth; bbheaderbch: tsrate)\n"
               "  --format cf32|sc16      IQ sample format (default cf32, pilotgen's complex64)\n"
               "  --gain G                output gain (the flowgraph's multiply_const; default 1)\n"
               "  --frames N              T2 frames to encode (default: as many as the input holds)\n"
               "  --batch B               T2 frames per GPU call (default 16)\n"
               "  --device D              GPU index (default 0)\n"
               "  --print-params          print the resolved parameters and exit (no GPU)\n");
}

struct Field { const char *n; int *v; };
std::vector<Field> fields(dvbt2ll_chain_params &p) {
  dvbt2ll_framemapperfint_params &f = p.fm;
  return {
      {"framesize", &f.framesize}, {"rate", &f.rate}, {"constellation", &f.constellation},
      {"rotation", &f.rotation}, {"fecblocks", &f.fecblocks}, {"tiblocks", &f.tiblocks},
      {"carriermode", &f.carriermode}, {"fftsize", &f.fftsize}, {"guardinterval", &f.guardinterval},
      {"l1constellation", &f.l1constellation}, {"pilotpattern", &f.pilotpattern}, {"t2frames", &f.t2frames},
      {"numdatasyms", &f.numdatasyms}, {"paprmode", &f.paprmode}, {"version", &f.version},
      {"preamble", &f.preamble}, {"inputmode", &f.inputmode}, {"reservedbiasbits", &f.reservedbiasbits},
      {"l1scrambled", &f.l1scrambled}, {"inband", &f.inband}, {"misogroup", &p.misogroup},
      {"equalization", &p.equalization}, {"bandwidth", &p.bandwidth}, {"tsrate", &p.tsrate}};
}
int *field(dvbt2ll_chain_params &p, const std::string &n) {
  for (auto &e : fields(p))
    if (n == e.n) return e.v;
  return nullptr;
}

// stream position of payload byte J (HEM drops each packet's sync byte)
int64_t payload_pos(int64_t J, bool hem) { return hem ? 188 * (J / 187) + 1 + J % 187 : J; }

}  // namespace

int main(int argc, char **argv) {
  std::string in_path, out_path, preset = "cfg1";
  std::vector<std::string> sets;
  int fmt = DVBT2LL_IQ_CF32, batch = 16, device = 0;
  bool print_params = false;
  int64_t frames = -1;
  float gain = 1.f;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> const char * {
      if (i + 1 >= argc) {
        std::fprintf(stderr, "dvbt2ll_tx: %s needs a value\n", a.c_str());
        std::exit(2);
      }
      return argv[++i];
    };
    if (a == "-h" || a == "--help") { usage(stdout); return 0; }
    else if (a == "--in") in_path = next();
    else if (a == "--out") out_path = next();
    else if (a == "--preset") preset = next();
    else if (a == "--set") sets.push_back(next());
    else if (a == "--format") {
      std::string v = next();
      if (v == "cf32") fmt = DVBT2LL_IQ_CF32;
      else if (v == "sc16") fmt = DVBT2LL_IQ_SC16;
      else { std::fprintf(stderr, "dvbt2ll_tx: unknown format %s\n", v.c_str()); return 2; }
    } else if (a == "--gain") gain = std::strtof(next(), nullptr);
    else if (a == "--frames") frames = std::strtoll(next(), nullptr, 10);
    else if (a == "--batch") batch = std::atoi(next());
    else if (a == "--device") device = std::atoi(next());
    else if (a == "--print-params") print_params = true;
    else { std::fprintf(stderr, "dvbt2ll_tx: unknown option %s\n", a.c_str()); usage(stderr); return 2; }
  }

  dvbt2ll_chain_params p;
  std::memset(&p, 0, sizeof(p));
  const Preset *ps = nullptr;
  for (auto &q : kPresets)
    if (preset == q.name) ps = &q;
  if (!ps) { std::fprintf(stderr, "dvbt2ll_tx: unknown preset %s\n", preset.c_str()); return 2; }
  dvbt2ll_framemapperfint_params &f = p.fm;
  f.framesize = ps->framesize; f.rate = ps->rate; f.constellation = ps->constellation; f.rotation = ps->rotation;
  f.fecblocks = ps->fecblocks; f.tiblocks = ps->tiblocks; f.carriermode = ps->carriermode; f.fftsize = ps->fftsize;
  f.guardinterval = ps->guardinterval; f.l1constellation = ps->l1constellation; f.pilotpattern = ps->pilotpattern;
  f.t2frames = ps->t2frames; f.numdatasyms = ps->numdatasyms;
  p.tsrate = 4000000;
  p.bandwidth = 4;   // BANDWIDTH_8_0_MHZ
  for (auto &s : sets) {
    size_t eq = s.find('=');
    int *v = eq == std::string::npos ? nullptr : field(p, s.substr(0, eq));
    if (!v) { std::fprintf(stderr, "dvbt2ll_tx: bad --set %s\n", s.c_str()); return 2; }
    *v = std::atoi(s.c_str() + eq + 1);
  }
  p.max_frames = batch;
  if (print_params) {
    for (auto &e : fields(p)) std::printf("%s=%d\n", e.n, *e.v);
    return 0;
  }
  if (in_path.empty() || out_path.empty() || batch < 1) { usage(stderr); return 2; }

  dvbt2ll_chain *h = nullptr;
  int st = dvbt2ll_chain_create(&p, device, &h);
  if (st) { std::fprintf(stderr, "dvbt2ll_tx: chain create: %s\n", dvbt2ll_strerror(st)); return 1; }
  dvbt2ll_chain_info info;
  if ((st = dvbt2ll_chain_get_info(h, &info)) || (st = dvbt2ll_chain_set_output(h, gain, fmt))) {
    std::fprintf(stderr, "dvbt2ll_tx: %s\n", dvbt2ll_strerror(st));
    dvbt2ll_chain_destroy(h);
    return 1;
  }
  FILE *fin = in_path == "-" ? stdin : std::fopen(in_path.c_str(), "rb");
  FILE *fout = out_path == "-" ? stdout : std::fopen(out_path.c_str(), "wb");
  if (!fin || !fout) {
    std::fprintf(stderr, "dvbt2ll_tx: cannot open %s: %s\n", !fin ? in_path.c_str() : out_path.c_str(),
                 std::strerror(errno));
    dvbt2ll_chain_destroy(h);
    return 1;
  }
  const bool hem = f.inputmode != 0;
  // payload bytes per frame: F BBFRAME payloads less the in-band type B field of the first
  const int64_t pay_frame = (int64_t)info.fec_blocks_per_frame * info.payload_bytes_per_block - (f.inband ? 13 : 0);
  const size_t sample_bytes = fmt == DVBT2LL_IQ_SC16 ? 4 : 8;
  std::vector<uint8_t> ts;                 // stream bytes [ts_base, ts_base + ts.size())
  int64_t ts_base = 0;
  bool eof = false;
  // the ring: batch k's TS span and IQ in page-locked buffers of slot k % R until it is written out
  constexpr int R = DVBT2LL_HOST_RING;
  const size_t iq_slot = (size_t)batch * info.iq_samples_per_frame * sample_bytes;
  const size_t ts_slot = (size_t)(payload_pos((int64_t)batch * pay_frame, hem) + 4 * 188);
  void *ts_pin[R] = {}, *iq_pin[R] = {};
  int64_t ticket[R] = {}, slot_frames[R] = {};
  for (int k = 0; k < R; k++)
    if (!(ts_pin[k] = dvbt2ll_host_alloc(ts_slot)) || !(iq_pin[k] = dvbt2ll_host_alloc(iq_slot))) {
      std::fprintf(stderr, "dvbt2ll_tx: page-locked host buffers: out of memory\n");
      st = DVBT2LL_ENOMEM;
    }
  int64_t done = 0, written = 0, submitted = 0;
  // write out the oldest batch in flight (waits for its copy-out)
  auto drain_one = [&]() -> bool {
    const int sl = (int)(written % R);
    int e = dvbt2ll_chain_host_wait(h, ticket[sl]);
    if (e) { std::fprintf(stderr, "dvbt2ll_tx: run: %s\n", dvbt2ll_strerror(e)); st = e; return false; }
    const size_t bytes = (size_t)slot_frames[sl] * info.iq_samples_per_frame * sample_bytes;
    if (std::fwrite(iq_pin[sl], 1, bytes, fout) != bytes) {
      std::fprintf(stderr, "dvbt2ll_tx: write failed: %s\n", std::strerror(errno));
      st = -1;
      return false;
    }
    written++;
    return true;
  };
  const auto t0 = std::chrono::steady_clock::now();
  while (!st && (frames < 0 || done < frames)) {
    int n = batch;
    if (frames >= 0 && frames - done < n) n = (int)(frames - done);
    // stream bytes the frames [done, done + n) consume, plus the packet before the first
    // (its CRC-8 replaces the next sync byte): [lo, end)
    const int64_t start = payload_pos(done * pay_frame, hem);
    int64_t end = payload_pos((done + n) * pay_frame, hem) + 1;
    const int64_t lo = start >= 188 ? (start / 188) * 188 - 188 : 0;
    if (lo > ts_base) {                    // drop bytes no later frame needs
      ts.erase(ts.begin(), ts.begin() + (lo - ts_base));
      ts_base = lo;
    }
    while (!eof && ts_base + (int64_t)ts.size() < end) {
      size_t old = ts.size();
      ts.resize(old + (1 << 20));
      size_t got = std::fread(ts.data() + old, 1, ts.size() - old, fin);
      ts.resize(old + got);
      if (got == 0) eof = true;
    }
    while (n > 0 && ts_base + (int64_t)ts.size() < end) {   // short input: fewer frames
      n--;
      end = payload_pos((done + n) * pay_frame, hem) + 1;
    }
    if (n == 0) break;
    if (submitted - written == R && !drain_one()) break;   // the slot's previous batch goes out first
    const int sl = (int)(submitted % R);
    const int64_t span = end - lo;
    if ((size_t)span > ts_slot) { st = DVBT2LL_EINVAL; break; }
    std::memcpy(ts_pin[sl], ts.data() + (lo - ts_base), (size_t)span);
    st = dvbt2ll_chain_host_submit(h, ts_pin[sl], lo, span, done, n, iq_pin[sl], &ticket[sl]);
    if (st) { std::fprintf(stderr, "dvbt2ll_tx: run: %s\n", dvbt2ll_strerror(st)); break; }
    slot_frames[sl] = n;
    submitted++;
    done += n;
  }
  while (!st && written < submitted && drain_one()) {
  }
  const double dt = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "dvbt2ll_tx: %lld T2 frames, %lld samples (%s, gain %g) in %.3f s: %.1f Msamples/s\n",
               (long long)done, (long long)(done * info.iq_samples_per_frame), fmt ? "sc16" : "cf32", gain, dt,
               dt > 0 ? done * info.iq_samples_per_frame / dt / 1e6 : 0.0);
  if (fin != stdin) std::fclose(fin);
  if (fout != stdout) std::fclose(fout);
  (void)dvbt2ll_chain_synchronize(h);
  for (int k = 0; k < R; k++) {
    if (submitted > written) (void)dvbt2ll_chain_host_wait(h, ticket[k]);   // nothing in flight on the buffers
    dvbt2ll_host_free(ts_pin[k]);
    dvbt2ll_host_free(iq_pin[k]);
  }
  dvbt2ll_chain_destroy(h);
  return st ? 1 : 0;
}
