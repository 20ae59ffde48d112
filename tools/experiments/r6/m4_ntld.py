# experiment: ldpc_map_kernel reads the BBFRAME rows with nontemporal loads (read once; keep the TI quad table in L2)
EDITS = [("""      u[k] = tid + FEC_THREADS * k < nqi ? rowq[tid + FEC_THREADS * k] : make_uint4(0u, 0u, 0u, 0u);""",
          """      u[k] = tid + FEC_THREADS * k < nqi ? [&]() { const u32x4 x = __builtin_nontemporal_load((const u32x4 *)(rowq + tid + FEC_THREADS * k)); return make_uint4(x[0], x[1], x[2], x[3]); }() : make_uint4(0u, 0u, 0u, 0u);""")]
