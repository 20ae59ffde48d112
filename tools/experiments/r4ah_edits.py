# text edits for tools/exp_variant.py (r4ah): QBL = branchless index-pair reads in the TI quad store (kept),
# CBAT = map_cells column windows read eight at a time (spilled; the four-at-a-time form cbat4 measured slower)
QBL = [("""  auto pair_of = [&](uint32_t j) -> uint32_t {
    const uint32_t lo = idx[j], hi = d.rotation ? (uint32_t)idx[j == 0 ? (uint32_t)cs - 1u : j - 1u] : lo;
    return lo | (hi << 8);
  };""", """  // (idx[j], idx[j - 1] under rotation, else idx[j]) without branches, so a quad's eight byte reads
  // go out together (a branch per read had put an LDS wait after each); j = 0xFFFF (another block's
  // slot) reads idx[0], and the caller drops it
  const uint32_t rmask = d.rotation ? 0xFFFFFFFFu : 0u;
  auto pair_of = [&](uint32_t j) -> uint32_t {
    j = j == 0xFFFFu ? 0u : j;
    const uint32_t jm = j == 0 ? (uint32_t)cs - 1u : j - 1u, jh = (jm & rmask) | (j & ~rmask);
    return (uint32_t)idx[j] | ((uint32_t)idx[jh] << 8);
  };"""),
("""      const int c = c0 + u * NW + wv;
      if (c < nch && 64 * c + lane < nqd) {
        const uint32_t j0 = e[u].x & 0xFFFFu, j1 = e[u].x >> 16, j2 = e[u].y & 0xFFFFu, j3 = e[u].y >> 16;
        if (j0 != 0xFFFFu && j1 != 0xFFFFu && j2 != 0xFFFFu && j3 != 0xFFFFu) {
          st_off((uint2 *)dst, qa[u] * 8u, make_uint2(pair_of(j0) | (pair_of(j1) << 16), pair_of(j2) | (pair_of(j3) << 16)));
        } else {
          if (j0 != 0xFFFFu) st_off(dst, (4u * qa[u] + 0u) * 2u, (uint16_t)pair_of(j0));
          if (j1 != 0xFFFFu) st_off(dst, (4u * qa[u] + 1u) * 2u, (uint16_t)pair_of(j1));
          if (j2 != 0xFFFFu) st_off(dst, (4u * qa[u] + 2u) * 2u, (uint16_t)pair_of(j2));
          if (j3 != 0xFFFFu) st_off(dst, (4u * qa[u] + 3u) * 2u, (uint16_t)pair_of(j3));
        }
      }""", """      const int c = c0 + u * NW + wv;
      const uint32_t j0 = e[u].x & 0xFFFFu, j1 = e[u].x >> 16, j2 = e[u].y & 0xFFFFu, j3 = e[u].y >> 16;
      const uint32_t p0 = pair_of(j0), p1 = pair_of(j1), p2 = pair_of(j2), p3 = pair_of(j3);
      if (c < nch && 64 * c + lane < nqd) {
        if (j0 != 0xFFFFu && j1 != 0xFFFFu && j2 != 0xFFFFu && j3 != 0xFFFFu) {
          st_off((uint2 *)dst, qa[u] * 8u, make_uint2(p0 | (p1 << 16), p2 | (p3 << 16)));
        } else {
          if (j0 != 0xFFFFu) st_off(dst, (4u * qa[u] + 0u) * 2u, (uint16_t)p0);
          if (j1 != 0xFFFFu) st_off(dst, (4u * qa[u] + 1u) * 2u, (uint16_t)p1);
          if (j2 != 0xFFFFu) st_off(dst, (4u * qa[u] + 2u) * 2u, (uint16_t)p2);
          if (j3 != 0xFFFFu) st_off(dst, (4u * qa[u] + 3u) * 2u, (uint16_t)p3);
        }
      }""")]
CBAT = [("""      uint64_t xa[2] = {0, 0}, xb[2] = {0, 0};
#pragma unroll
      for (int b = 0; b < 16; b++) {
        const int c0 = d.colstart[b];
        if (c0 < 0) continue;
        int off = j0 - d.coltw[b];
        off += off < 0 ? R : 0;
        uint32_t win = window(c0 + off);
        if (off + 16 > R) {                      // the column wraps inside these 16 rows
          const int n1 = R - off;
          win = (win & ~(0xFFFFFFFFu >> n1)) | (window(c0) >> n1);
        }
        xa[b >> 3] |= (uint64_t)(win >> 24) << (8 * (b & 7));
        xb[b >> 3] |= (uint64_t)((win >> 16) & 0xFFu) << (8 * (b & 7));
      }""", """      uint64_t xa[2] = {0, 0}, xb[2] = {0, 0};
#pragma unroll
      for (int h = 0; h < 2; h++) {
        // the eight columns' window words requested together (one LDS wait instead of one per column)
        uint32_t w0[8], w1[8];
#pragma unroll
        for (int bb = 0; bb < 8; bb++) {
          const int b = 8 * h + bb, c0 = d.colstart[b];
          if (c0 < 0) continue;
          int off = j0 - d.coltw[b];
          off += off < 0 ? R : 0;
          const int s = c0 + off;
          w0[bb] = cww[s >> 5];
          w1[bb] = cww[(s >> 5) + 1];
        }
#pragma unroll
        for (int bb = 0; bb < 8; bb++) {
          const int b = 8 * h + bb, c0 = d.colstart[b];
          if (c0 < 0) continue;
          int off = j0 - d.coltw[b];
          off += off < 0 ? R : 0;
          const int s = c0 + off;
          uint32_t win = (uint32_t)(((((uint64_t)w0[bb] << 32) | w1[bb]) << (s & 31)) >> 32);
          if (off + 16 > R) {                    // the column wraps inside these 16 rows
            const int n1 = R - off;
            win = (win & ~(0xFFFFFFFFu >> n1)) | (window(c0) >> n1);
          }
          xa[h] |= (uint64_t)(win >> 24) << (8 * bb);
          xb[h] |= (uint64_t)((win >> 16) & 0xFFu) << (8 * bb);
        }
      }""")]
