# wrong-output probe: no BCH MFMAs (and no B-fragment reads)
EDITS = [("""          acc[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A, Bv, acc[t], 4, 4, 0, 128, 0, 127);""",
          """          acc[t][0] += (float)(A[0] ^ Bv[0]);""")]
