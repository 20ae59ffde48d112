# LDPC + map kernel: the block's BBFRAME 16-byte units (read once) as nontemporal loads
EDITS = [(
    """      u[k] = tid + FEC_THREADS * k < nqi ? rowq[tid + FEC_THREADS * k] : make_uint4(0u, 0u, 0u, 0u);""",
    """      u[k] = tid + FEC_THREADS * k < nqi ? [&] { typedef unsigned int u4nt __attribute__((ext_vector_type(4))); const u4nt t = __builtin_nontemporal_load((const u4nt *)(rowq + tid + FEC_THREADS * k)); return make_uint4(t.x, t.y, t.z, t.w); }() : make_uint4(0u, 0u, 0u, 0u);""")]
