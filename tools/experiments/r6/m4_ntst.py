# experiment: the TI store's 8-byte quad stores nontemporal
EDITS = [("""          st_off((uint2 *)dst, R.qa[u] * 8u, v);""",
          """          __builtin_nontemporal_store(((uint64_t)v.y << 32) | v.x, (uint64_t *)((char *)dst + R.qa[u] * 8u));""")]
