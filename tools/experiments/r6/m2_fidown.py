# wrong-output probe (verdict r5 item 3, downside of "FI permutation upstream"): the map's index-pair stores
# land in IFFT-input order instead of stored-slot quads: each slot of a quad stored as its own 2-byte store at
# a permuted position within the symbol's 32K window (odd multiplier mod 32768), no 8-byte quad stores
EDITS = [("""        if (!((e.x | e.y) & 0x80008000u)) {
          st_off((uint2 *)dst, R.qa[u] * 8u, v);
        } else {""", """        if (!((e.x | e.y) & 0x80008000u)) {
          const uint32_t s0 = 4u * R.qa[u], w0 = s0 & ~32767u;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const uint32_t sp = (w0 + (((s0 + k) * 4097u + 12345u) & 32767u)) % (uint32_t)frame_stride;   // inside the frame
            st_off(dst, sp * 2u, (uint16_t)((k < 2 ? v.x : v.y) >> (16 * (k & 1))));
          }
        } else {""")]
