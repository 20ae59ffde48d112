// dvbt2ll_tx -- native command-line DVB-T2 transmitter over the C ABI (include/dvbt2ll_hip.h):
// MPEG-TS file in, baseband IQ file out, whole T2 frames per GPU call.  It is the file-sink
// form of the shipped flowgraph apps/vv009-4kshort.grc (TS source -> the five blocks ->
// multiply_const -> sink): TS bytes -> the chain's streaming host path (dvbt2ll_chain_host_submit /
// _host_wait: a ring of DVBT2LL_HOST_RING batches in flight, page-locked buffers, so reading batch k + 1,
// encoding batch k and writing batch k - 2 overlap) -> complex64 or sc16 samples.
//
//   dvbt2ll_tx --preset cfg3 --in stream.ts --out iq.sc16 --format sc16 --gain 0.2
//   dvbt2ll_tx --mplp mix_4k --in plp0.ts --in plp1.ts --in plp2.ts --out iq.cf32
//
// --mplp runs a multi-PLP frame preset (one TS file per PLP, dvbt2ll_chain_create_mplp / _run_plps_host;
// batches are whole launch units, dvbt2ll_chain_unit_frames).
//
// The TS is consumed as one continuous stream (absolute offsets from the start of the file);
// frame k is encoded with the stream state the reference blocks would hold at that point.
// Trailing bytes that do not complete a T2 frame are left unused.
#include <algorithm>
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

// multi-PLP presets (gr-dvbt2ll_amd/dvbt2ll/configs.py MPLP_CONFIGS / IF_CONFIGS of the same names): the
// common fields of dvbt2ll_mplp_params, then per PLP {framesize, rate, constellation, rotation, fecblocks,
// tiblocks, inputmode, inband, tsrate, plp_type, ti_type, ti_frames, frame_interval, first_frame_idx}
struct MplpPreset {
  const char *name;
  int common[12];
  int nplp;
  dvbt2ll_plp_params plp[3];
  int num_subslices;
};
const MplpPreset kMplpPresets[] = {
    // the GRC's 4K short frame as three Type-1 PLPs (256-QAM 4/5 rotated, QPSK 1/2, 16-QAM 3/5 HEM)
    {"mplp3_4k", {0, 2, 0, 3, 6, 2, 3, 0, 0, 0, 0, 0}, 3,
     {{0, 4, 3, 1, 2, 1, 0, 0, 4000000, 1, 0, 1, 1, 0}, {0, 0, 0, 0, 1, 0, 0, 0, 4000000, 1, 0, 1, 1, 0},
      {0, 1, 1, 1, 1, 2, 1, 0, 4000000, 1, 0, 1, 1, 0}}, 1},
    // the same frame with a Type-2 TIME_IL_TYPE 1 PLP (P_I = 2), a Type-1 PLP and a Type-2 HEM PLP, 6 sub-slices
    {"mix_4k", {0, 2, 0, 3, 6, 2, 3, 0, 0, 0, 0, 0}, 3,
     {{0, 4, 3, 1, 4, 1, 0, 0, 4000000, 2, 1, 2, 1, 0}, {0, 0, 0, 0, 1, 1, 0, 0, 4000000, 1, 0, 1, 1, 0},
      {0, 1, 1, 1, 1, 1, 1, 0, 4000000, 2, 0, 1, 1, 0}}, 6},
};

void usage(FILE *f) {
  std::fprintf(f,
               "usage: dvbt2ll_tx --in TS_FILE --out IQ_FILE [options]\n"
               "  --preset cfg1..cfg5|cfg1q parameter preset (default cfg1, the shipped flowgraph)\n"
               "  --mplp mplp3_4k|mix_4k    multi-PLP frame preset: give one --in per PLP\n"
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

// one TS input: the stream window [base, base + buf.size()) of a file read as the frames need it
struct TsIn {
  FILE *f = nullptr;
  std::vector<uint8_t> buf;
  int64_t base = 0;
  bool eof = false;
  // make [lo, end) available (dropping bytes before lo); false if the file ends first
  bool span(int64_t lo, int64_t end) {
    if (lo > base) {
      const size_t drop = (size_t)std::min<int64_t>(lo - base, (int64_t)buf.size());
      buf.erase(buf.begin(), buf.begin() + drop);
      base = lo;
    }
    while (!eof && base + (int64_t)buf.size() < end) {
      size_t old = buf.size();
      buf.resize(old + (1 << 20));
      size_t got = std::fread(buf.data() + old, 1, buf.size() - old, f);
      buf.resize(old + got);
      if (got == 0) eof = true;
    }
    return base + (int64_t)buf.size() >= end;
  }
};

// the multi-PLP transmitter: whole launch units per batch, each PLP's TS span from its own file
int run_mplp(const MplpPreset &ps, const std::vector<std::string> &ins, const std::string &out_path, int fmt,
             float gain, int64_t frames, int batch, int device, bool print_params) {
  dvbt2ll_mplp_chain_params p;
  std::memset(&p, 0, sizeof(p));
  dvbt2ll_mplp_params &m = p.fm;
  int *c[12] = {&m.carriermode, &m.fftsize, &m.guardinterval, &m.l1constellation, &m.pilotpattern, &m.t2frames,
                &m.numdatasyms, &m.paprmode, &m.version, &m.preamble, &m.reservedbiasbits, &m.l1scrambled};
  for (int i = 0; i < 12; i++) *c[i] = ps.common[i];
  m.nplp = ps.nplp;
  for (int k = 0; k < ps.nplp; k++) m.plp[k] = ps.plp[k];
  m.num_subslices = ps.num_subslices;
  p.bandwidth = 4;   // BANDWIDTH_8_0_MHZ
  if (print_params) {   // the dvbt2ll_mplp_params ints (configs.MplpConfig.mplp_array layout)
    for (int i = 0; i < 12; i++) std::printf("%d ", *c[i]);
    std::printf("%d", m.nplp);
    for (int k = 0; k < DVBT2LL_MAX_PLP; k++) {
      const dvbt2ll_plp_params &q = m.plp[k];
      const int v[14] = {q.framesize, q.rate, q.constellation, q.rotation, q.fecblocks, q.tiblocks, q.inputmode,
                         q.inband, q.tsrate, q.plp_type, q.ti_type, q.ti_frames, q.frame_interval,
                         q.first_frame_idx};
      for (int x : v) std::printf(" %d", x);
    }
    std::printf(" %d\n", m.num_subslices);
    return 0;
  }
  if ((int)ins.size() != ps.nplp || out_path.empty()) {
    std::fprintf(stderr, "dvbt2ll_tx: --mplp %s needs %d --in files and --out\n", ps.name, ps.nplp);
    return 2;
  }
  dvbt2ll_chain *h = nullptr;
  p.max_frames = batch;
  int st = dvbt2ll_chain_create_mplp(&p, device, &h);
  const int unit = st ? 1 : dvbt2ll_chain_unit_frames(h);
  if (!st && batch % unit) st = DVBT2LL_EINVAL;   // batches of whole launch units
  if (!st) st = dvbt2ll_chain_set_output(h, gain, fmt);
  if (st) {
    std::fprintf(stderr, "dvbt2ll_tx: chain: %s (batch must be a multiple of the launch unit)\n", dvbt2ll_strerror(st));
    dvbt2ll_chain_destroy(h);
    return 1;
  }
  dvbt2ll_chain_info pi[DVBT2LL_MAX_PLP];
  std::vector<TsIn> ts(ps.nplp);
  for (int k = 0; k < ps.nplp && !st; k++) {
    st = dvbt2ll_chain_get_plp_info(h, k, &pi[k]);
    ts[k].f = std::fopen(ins[k].c_str(), "rb");
    if (!ts[k].f) { std::fprintf(stderr, "dvbt2ll_tx: cannot open %s\n", ins[k].c_str()); st = -1; }
  }
  FILE *fout = st ? nullptr : (out_path == "-" ? stdout : std::fopen(out_path.c_str(), "wb"));
  if (!st && !fout) { std::fprintf(stderr, "dvbt2ll_tx: cannot open %s\n", out_path.c_str()); st = -1; }
  const size_t sb = fmt == DVBT2LL_IQ_SC16 ? 4 : 8;
  std::vector<uint8_t> iq;
  if (!st) iq.resize((size_t)batch * pi[0].iq_samples_per_frame * sb);
  int64_t done = 0;
  while (!st && (frames < 0 || done < frames)) {
    int n = batch;
    if (frames >= 0 && frames - done < n) n = (int)((frames - done) / unit * unit);
    const void *ptr[DVBT2LL_MAX_PLP];
    int64_t base[DVBT2LL_MAX_PLP], len[DVBT2LL_MAX_PLP];
    for (; n > 0; n -= unit) {   // the most whole units every PLP's input still covers
      bool ok = true;
      for (int k = 0; k < ps.nplp && ok; k++) {
        const dvbt2ll_plp_params &q = ps.plp[k];
        const int P = pi[k].frames_per_if;
        const bool hem = q.inputmode != 0;
        const int64_t pay = (int64_t)pi[k].fec_blocks_per_frame * pi[k].payload_bytes_per_block - (q.inband ? 13 : 0);
        const int64_t start = payload_pos(done / P * pay, hem), end = payload_pos((done + n) / P * pay, hem) + 1;
        const int64_t lo = start >= 188 ? (start / 188) * 188 - 188 : 0;
        ok = ts[k].span(lo, end);
        ptr[k] = ts[k].buf.data();
        base[k] = ts[k].base;
        len[k] = (int64_t)ts[k].buf.size();
      }
      if (ok) break;
    }
    if (n <= 0) break;
    st = dvbt2ll_chain_run_plps_host(h, ptr, base, len, done, n, iq.data());
    if (st) { std::fprintf(stderr, "dvbt2ll_tx: run: %s\n", dvbt2ll_strerror(st)); break; }
    const size_t bytes = (size_t)n * pi[0].iq_samples_per_frame * sb;
    if (std::fwrite(iq.data(), 1, bytes, fout) != bytes) { st = -1; break; }
    done += n;
  }
  std::fprintf(stderr, "dvbt2ll_tx: %s: %lld T2 frames\n", ps.name, (long long)done);
  for (auto &t : ts)
    if (t.f) std::fclose(t.f);
  if (fout && fout != stdout) std::fclose(fout);
  dvbt2ll_chain_destroy(h);
  return st ? 1 : 0;
}

}  // namespace

int main(int argc, char **argv) {
  std::string in_path, out_path, preset = "cfg1", mplp;
  std::vector<std::string> sets, ins;
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
    else if (a == "--in") ins.push_back(in_path = next());
    else if (a == "--mplp") mplp = next();
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

  if (!mplp.empty()) {
    for (auto &q : kMplpPresets)
      if (mplp == q.name) return run_mplp(q, ins, out_path, fmt, gain, frames, batch, device, print_params);
    std::fprintf(stderr, "dvbt2ll_tx: unknown multi-PLP preset %s\n", mplp.c_str());
    return 2;
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
