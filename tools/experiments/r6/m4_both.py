# experiment: m4_ntld + m4_ntst
EDITS = [("""      u[k] = tid + FEC_THREADS * k < nqi ? rowq[tid + FEC_THREADS * k] : make_uint4(0u, 0u, 0u, 0u);""",
          """      u[k] = tid + FEC_THREADS * k < nqi ? [&]() { const u32x4 x = __builtin_nontemporal_load((const u32x4 *)(rowq + tid + FEC_THREADS * k)); return make_uint4(x[0], x[1], x[2], x[3]); }() : make_uint4(0u, 0u, 0u, 0u);"""),
("""          st_off((uint2 *)dst, R.qa[u] * 8u, v);""",
          """          __builtin_nontemporal_store(((uint64_t)v.y << 32) | v.x, (uint64_t *)((char *)dst + R.qa[u] * 8u));""")]
