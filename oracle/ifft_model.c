/*
 * ifft_model.c -- TEST INFRASTRUCTURE ONLY: a CPU restatement of the OFDM kernels' IFFT in the
 * GPU's exact operation order ("between the build's CPU restatement and its GPU
 * kernel, require bit-exact IQ: same Stockham op order, same twiddle table").
 *
 * The reference computes the IFFT with FFTW (pilotgenp1insert_cc_impl.cc:2890-2894), which is not
 * in this image, so IQ is pinned two ways: this model against a float64 IFFT of the oracle's
 * carriers within the 8(c) tolerance (CPU tests), and the GPU against this model bit-exactly
 * (GPU tests).  Every arithmetic step below is the one gr-dvbt2ll_amd/csrc/t2_kernels.hip issues:
 *   complex product  cmulf(a, b) = (fma(a.y, -b.y, a.x b.x), fma(a.y, b.x, a.x b.y))
 *                    (v_pk_mul_f32 + v_pk_fma_f32, t2_kernels.hip cmulf)
 *   a + i b, a - i b (a.x - b.y, a.y + b.x), (a.x + b.y, a.y - b.x)
 *   in-register DFT  bit reversal, then radix-2 stages with the kCos32 / kSin32 constants (Dft<R>)
 *   N <= 16K         Stockham passes 16 x 16 x {4, 8, 16, 16 x 2, 16 x 4} (FftPlan), twiddles
 *                    w^(r e) from the table bases w^e, w^(4e), w^(8e) (twiddle_unit)
 *   32K              32 x 32 x 32 with the seven-lookup twiddle bases (o32_fft, o32_twiddle)
 *   store            (y * norm) * gain, then (sc16) saturate(rint(x * 32767))
 * Built with -ffp-contract=off: every product is rounded before the add unless fmaf says so.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <stdlib.h>

typedef struct {
  float x, y;
} c32;

static c32 mk(float x, float y) {
  c32 r = {x, y};
  return r;
}
static c32 cmulf(c32 a, c32 b) {
  const float tx = a.x * b.x, ty = a.x * b.y;
  return mk(fmaf(a.y, -b.y, tx), fmaf(a.y, b.x, ty));
}
static c32 cadd(c32 a, c32 b) { return mk(a.x + b.x, a.y + b.y); }
static c32 csub(c32 a, c32 b) { return mk(a.x - b.x, a.y - b.y); }
static c32 cadd_i(c32 a, c32 b) { return mk(a.x - b.y, a.y + b.x); }
static c32 csub_i(c32 a, c32 b) { return mk(a.x + b.y, a.y - b.x); }

/* exp(+2 pi i k / 32), the kernel's float literals */
static const float kCos32[32] = {
    1.0f, 0.98078528040323043f, 0.92387953251128674f, 0.83146961230254524f, 0.70710678118654757f,
    0.55557023301960218f, 0.38268343236508978f, 0.19509032201612828f, 0.0f, -0.19509032201612828f,
    -0.38268343236508978f, -0.55557023301960218f, -0.70710678118654757f, -0.83146961230254524f,
    -0.92387953251128674f, -0.98078528040323043f, -1.0f, -0.98078528040323043f, -0.92387953251128674f,
    -0.83146961230254524f, -0.70710678118654757f, -0.55557023301960218f, -0.38268343236508978f,
    -0.19509032201612828f, 0.0f, 0.19509032201612828f, 0.38268343236508978f, 0.55557023301960218f,
    0.70710678118654757f, 0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f};
static const float kSin32[32] = {
    0.0f, 0.19509032201612828f, 0.38268343236508978f, 0.55557023301960218f, 0.70710678118654757f,
    0.83146961230254524f, 0.92387953251128674f, 0.98078528040323043f, 1.0f, 0.98078528040323043f,
    0.92387953251128674f, 0.83146961230254524f, 0.70710678118654757f, 0.55557023301960218f,
    0.38268343236508978f, 0.19509032201612828f, 0.0f, -0.19509032201612828f, -0.38268343236508978f,
    -0.55557023301960218f, -0.70710678118654757f, -0.83146961230254524f, -0.92387953251128674f,
    -0.98078528040323043f, -1.0f, -0.98078528040323043f, -0.92387953251128674f, -0.83146961230254524f,
    -0.70710678118654757f, -0.55557023301960218f, -0.38268343236508978f, -0.19509032201612828f};

static int ilog2(int n) {
  int l = 0;
  while ((1 << l) < n) l++;
  return l;
}
static int brev(int i, int bits) {
  int r = 0;
  for (int b = 0; b < bits; b++) r |= ((i >> b) & 1) << (bits - 1 - b);
  return r;
}

/* Dft<R>::run: natural order in and out */
static void dft(c32 *x, int R) {
  const int L = ilog2(R);
  for (int i = 0; i < R; i++) {
    const int j = brev(i, L);
    if (i < j) {
      c32 t = x[i];
      x[i] = x[j];
      x[j] = t;
    }
  }
  for (int len = 2; len <= R; len <<= 1)
    for (int i = 0; i < R; i += len)
      for (int k = 0; k < len / 2; k++) {
        const c32 a = x[i + k], b = x[i + k + len / 2];
        if (4 * k == len && k != 0) {
          x[i + k] = cadd_i(a, b);
          x[i + k + len / 2] = csub_i(a, b);
          continue;
        }
        const c32 t = k == 0 ? b : cmulf(b, mk(kCos32[k * (32 / len)], kSin32[k * (32 / len)]));
        x[i + k] = cadd(a, t);
        x[i + k + len / 2] = csub(a, t);
      }
}

/* two-level table lookup w^i = hi[i >> 7] * lo[i & 127] (tw_at) */
static c32 tw_at(const c32 *tw, uint32_t i) { return cmulf(tw[128 + (i >> 7)], tw[i & 127]); }

/* twiddle_unit<R> (R <= 16): v[r] *= w^(r e); bases w^e, w^(4e) and (R = 16) w^(8e) from the table, the other
 * lo = w^(l e), hi = w^(4 h e) (l, h < 4) as products of those, w^(r e) = hi * lo */
static void twiddle_unit(c32 *v, int R, const c32 *tw, uint32_t e) {
  c32 lo[4], hi[4];
  lo[1] = tw_at(tw, e);
  if (R > 2) {
    lo[2] = cmulf(lo[1], lo[1]);
    lo[3] = cmulf(lo[2], lo[1]);
  }
  if (R > 4) hi[1] = tw_at(tw, 4 * e);
  if (R > 8) {
    hi[2] = tw_at(tw, 8 * e);
    hi[3] = cmulf(hi[2], hi[1]);
  }
  for (int r = 1; r < R; r++) {
    const int h = (r >> 2) & 3, l = r & 3;
    const c32 w = h == 0 ? lo[l] : (l == 0 ? hi[h] : cmulf(hi[h], lo[l]));
    v[r] = cmulf(v[r], w);
  }
}

/* o32_twiddle: the seven table values w^(e k), k = 1, 2, 3, 4, 8, 12, 16 given in t[0..6] */
static void o32_twiddle(c32 *v, const c32 *t) {
  const c32 lo[4] = {{1, 0}, t[0], t[1], t[2]}, hi[4] = {{1, 0}, t[3], t[4], t[5]};
  const c32 top = t[6];
  for (int r = 1; r < 32; r++) {
    const int tt = r >> 4, h = (r >> 2) & 3, l = r & 3;
    c32 w = h == 0 ? lo[l] : (l == 0 ? hi[h] : cmulf(hi[h], lo[l]));
    if (tt) w = (h == 0 && l == 0) ? top : cmulf(top, w);
    v[r] = cmulf(v[r], w);
  }
}

/* the kernels' twiddle tables (t2_plan.cpp build_pilot): [w^l, l < 128][w^(128 h), h < N/128],
 * w = exp(2 pi i / N); and exp(2 pi i m / 1024) */
static void tables(int N, c32 *tw, c32 *tw1k) {
  for (int e = 0; e < 128; e++) {
    const double a = 2.0 * M_PI * (double)e / (double)N;
    tw[e] = mk((float)cos(a), (float)sin(a));
  }
  for (int h = 0; h < N / 128; h++) {
    const double a = 2.0 * M_PI * (double)(128 * h) / (double)N;
    tw[128 + h] = mk((float)cos(a), (float)sin(a));
  }
  for (int m = 0; m < 1024; m++) {
    const double a = 2.0 * M_PI * (double)m / 1024.0;
    tw1k[m] = mk((float)cos(a), (float)sin(a));
  }
}

int t2m_tables(int N, float *tw, float *tw1k) {
  if (N < 1024 || N > 32768 || (N & (N - 1))) return -1;
  tables(N, (c32 *)tw, (c32 *)tw1k);
  return 0;
}

/* N <= 16K: X (natural FFT-input order) -> y, Stockham radix 16 then the plan's tail */
static void stockham(int N, const c32 *X, c32 *y, const c32 *tw, c32 *buf) {
  int tail[4], nt = 0;
  switch (N) {
    case 1024: tail[nt++] = 16; tail[nt++] = 4; break;
    case 2048: tail[nt++] = 16; tail[nt++] = 8; break;
    case 4096: tail[nt++] = 16; tail[nt++] = 16; break;
    case 8192: tail[nt++] = 16; tail[nt++] = 16; tail[nt++] = 2; break;
    default: tail[nt++] = 16; tail[nt++] = 16; tail[nt++] = 4; break;   /* 16384 */
  }
  c32 v[32];
  c32 *A = buf, *B = y;
  /* first pass: radix 16, NS = 1, no twiddles; out B[16 j + r] */
  c32 *dst = nt % 2 ? A : B;   /* ping-pong so that the last pass lands in y */
  for (int j = 0; j < N / 16; j++) {
    for (int r = 0; r < 16; r++) v[r] = X[j + r * (N / 16)];
    dft(v, 16);
    for (int r = 0; r < 16; r++) dst[16 * j + r] = v[r];
  }
  int NS = 16;
  c32 *src = dst;
  for (int p = 0; p < nt; p++) {
    const int R = tail[p];
    dst = src == A ? B : A;
    for (int j = 0; j < N / R; j++) {
      for (int r = 0; r < R; r++) v[r] = src[j + r * (N / R)];
      twiddle_unit(v, R, tw, (uint32_t)((j % NS) * (N / (NS * R))));
      dft(v, R);
      for (int r = 0; r < R; r++) dst[(j / NS) * NS * R + j % NS + r * NS] = v[r];
    }
    src = dst;
    NS *= R;
  }
  if (src != y) memcpy(y, src, sizeof(c32) * (size_t)N);
}

/* 32K: stages A, B, C of o32_fft over the 32 x 32 x 32 decomposition */
static void fft32k(const c32 *X, c32 *y, const c32 *tw, const c32 *tw1k, c32 *T) {
  enum { N = 32768 };
  c32 v[32], t[7];
  static const int K[7] = {1, 2, 3, 4, 8, 12, 16};
  /* stage A: thread (m0, m1): DFT over m2 of X[m0 + 32 m1 + 1024 m2], times w^((m0 + 32 m1) n2);
   * T[m0][m1][n2] */
  for (int m1 = 0; m1 < 32; m1++)
    for (int m0 = 0; m0 < 32; m0++) {
      const uint32_t kin = (uint32_t)(m0 + 32 * m1);
      for (int r = 0; r < 32; r++) v[r] = X[kin + 1024u * (uint32_t)r];
      dft(v, 32);
      for (int k = 0; k < 7; k++) t[k] = tw_at(tw, kin * (uint32_t)K[k]);
      o32_twiddle(v, t);
      for (int r = 0; r < 32; r++) T[(m0 * 32 + m1) * 32 + r] = v[r];
    }
  /* stage B: thread (m0, n2): DFT over m1, times w_1024^(m0 n1); y used as scratch U[m0][n2][n1] */
  for (int m0 = 0; m0 < 32; m0++)
    for (int n2 = 0; n2 < 32; n2++) {
      for (int r = 0; r < 32; r++) v[r] = T[(m0 * 32 + r) * 32 + n2];
      dft(v, 32);
      for (int k = 0; k < 7; k++) t[k] = tw1k[((uint32_t)m0 * (uint32_t)K[k]) & 1023u];
      o32_twiddle(v, t);
      for (int r = 0; r < 32; r++) y[(m0 * 32 + n2) * 32 + r] = v[r];
    }
  memcpy(T, y, sizeof(c32) * N);
  /* stage C: thread (n1, n2): DFT over m0 -> x[n2 + 32 n1 + 1024 n0] */
  for (int n1 = 0; n1 < 32; n1++)
    for (int n2 = 0; n2 < 32; n2++) {
      for (int r = 0; r < 32; r++) v[r] = T[(r * 32 + n2) * 32 + n1];
      dft(v, 32);
      for (int r = 0; r < 32; r++) y[n2 + 32 * n1 + 1024 * r] = v[r];
    }
}

/* One T2 frame's OFDM symbols as the GPU writes them (after P1):
 *   carriers: nsym x N complex64, pilotgen's frequency-domain symbols after EQ, before fftshift
 *             (orc_pg_carriers layout: bin c, DC at N / 2)
 *   out:      nsym x (G + N) complex64 (fmt 0) or int16 I/Q pairs (fmt 1): GI copy, then the symbol,
 *             each sample (y norm) gain
 * Returns 0, or -1 on a bad size / allocation failure. */
int t2m_symbols(int N, int G, int nsym, const float *carriers, float norm, float gain, int fmt, void *out) {
  if (N < 1024 || N > 32768 || (N & (N - 1)) || G < 0 || G > N || nsym < 0 || (fmt != 0 && fmt != 1)) return -1;
  c32 *tw = malloc(sizeof(c32) * (128 + N / 128)), *tw1k = malloc(sizeof(c32) * 1024);
  c32 *X = malloc(sizeof(c32) * N), *y = malloc(sizeof(c32) * N), *T = malloc(sizeof(c32) * N);
  int rc = 0;
  if (!tw || !tw1k || !X || !y || !T) {
    rc = -1;
    goto done;
  }
  tables(N, tw, tw1k);
  const c32 *car = (const c32 *)carriers;
  for (int j = 0; j < nsym; j++) {
    for (int k = 0; k < N; k++) X[k] = car[(size_t)j * N + ((k + N / 2) & (N - 1))];   /* fftshift */
    if (N == 32768)
      fft32k(X, y, tw, tw1k, T);
    else
      stockham(N, X, y, tw, T);
    for (int n = 0; n < N; n++) {
      c32 a = mk(y[n].x * norm, y[n].y * norm);
      a = mk(a.x * gain, a.y * gain);
      const size_t o0 = (size_t)j * (G + N) + G + n, o1 = (size_t)j * (G + N) + n - (N - G);
      if (fmt == 0) {
        ((c32 *)out)[o0] = a;
        if (n >= N - G) ((c32 *)out)[o1] = a;
      } else {
        const float i = fminf(fmaxf(rintf(a.x * 32767.f), -32768.f), 32767.f);
        const float q = fminf(fmaxf(rintf(a.y * 32767.f), -32768.f), 32767.f);
        int16_t *o = (int16_t *)out;
        o[2 * o0] = (int16_t)i;
        o[2 * o0 + 1] = (int16_t)q;
        if (n >= N - G) {
          o[2 * o1] = (int16_t)i;
          o[2 * o1 + 1] = (int16_t)q;
        }
      }
    }
  }
done:
  free(tw);
  free(tw1k);
  free(X);
  free(y);
  free(T);
  return rc;
}
