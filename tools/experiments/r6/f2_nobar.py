# wrong-output probe: no workgroup barrier per chunk (B staging races)
EDITS = [("""      bstore(cur ^ 1, bs);   // the other buffer was last read before the previous barrier
      __syncthreads();""", """      bstore(cur ^ 1, bs);""")]
