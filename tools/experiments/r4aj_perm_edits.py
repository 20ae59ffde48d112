# text edits for tools/exp_variant.py (r4aj, kept): map_cells assembles the column windows' bytes with v_perm_b32
EDITS = [("""      uint64_t xa[2] = {0, 0}, xb[2] = {0, 0};
#pragma unroll
      for (int b = 0; b < 16; b++) {
        const int2 cw = d.col[b];   // scalar loads at the point of use (kernel-argument arrays stayed live
        const int c0 = cw.x;         // in SGPRs through the whole kernel and spilled)
        if (c0 < 0) continue;
        int off = j0 - cw.y;
        off += off < 0 ? R : 0;
        uint32_t win = window(c0 + off);
        if (off + 16 > R) {                      // the column wraps inside these 16 rows
          const int n1 = R - off;
          win = (win & ~(0xFFFFFFFFu >> n1)) | (window(c0) >> n1);
        }
        xa[b >> 3] |= (uint64_t)(win >> 24) << (8 * (b & 7));
        xb[b >> 3] |= (uint64_t)((win >> 16) & 0xFFu) << (8 * (b & 7));
      }
      emit(2 * g2, tr8(xa[0]), d.W > 8 ? tr8(xa[1]) : 0ull);
      emit(2 * g2 + 1, tr8(xb[0]), d.W > 8 ? tr8(xb[1]) : 0ull);""",
"""      // xa / xb dword q: byte i = bits 31..24 / 23..16 of column 4 q + i's window, assembled with byte
      // permutes (four per four columns) instead of a shift and an OR per byte
      uint32_t xa[4], xb[4];
#pragma unroll
      for (int qd = 0; qd < 4; qd++) {
        uint32_t win[4];
#pragma unroll
        for (int i = 0; i < 4; i++) {
          const int b = 4 * qd + i;
          const int2 cw = d.col[b];   // scalar loads at the point of use
          const int c0 = cw.x;
          win[i] = 0u;
          if (c0 < 0) continue;
          int off = j0 - cw.y;
          off += off < 0 ? R : 0;
          win[i] = window(c0 + off);
          if (off + 16 > R) {                    // the column wraps inside these 16 rows
            const int n1 = R - off;
            win[i] = (win[i] & ~(0xFFFFFFFFu >> n1)) | (window(c0) >> n1);
          }
        }
        const uint32_t t = __builtin_amdgcn_perm(win[1], win[0], 0x06020703u);   // w0.b3 w1.b3 w0.b2 w1.b2
        const uint32_t u = __builtin_amdgcn_perm(win[3], win[2], 0x06020703u);   // w2.b3 w3.b3 w2.b2 w3.b2
        xa[qd] = __builtin_amdgcn_perm(u, t, 0x05040100u);
        xb[qd] = __builtin_amdgcn_perm(u, t, 0x07060302u);
      }
      const uint64_t xa0 = xa[0] | ((uint64_t)xa[1] << 32), xa1 = xa[2] | ((uint64_t)xa[3] << 32);
      const uint64_t xb0 = xb[0] | ((uint64_t)xb[1] << 32), xb1 = xb[2] | ((uint64_t)xb[3] << 32);
      emit(2 * g2, tr8(xa0), d.W > 8 ? tr8(xa1) : 0ull);
      emit(2 * g2 + 1, tr8(xb0), d.W > 8 ? tr8(xb1) : 0ull);""")]
