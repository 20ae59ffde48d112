# 32K OFDM scatter: the index-pair octets (read once per frame) as nontemporal loads
EDITS = [(
    """        c[u] = ld_off((const uint4 *)src.pairs, (src.cbase + s) * 2u);
      }
      if (pending) {""",
    """        c[u] = [&] { typedef unsigned int u4nt __attribute__((ext_vector_type(4))); const u4nt t = __builtin_nontemporal_load((const u4nt *)((const char *)src.pairs + (src.cbase + s) * 2u)); return make_uint4(t.x, t.y, t.z, t.w); }();
      }
      if (pending) {""")]
