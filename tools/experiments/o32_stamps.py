# 32K OFDM phase probe (wrong-output build): thread 0 of every (symbol, frame) workgroup stamps
# s_memrealtime (100 MHz) at the phase boundaries and, once every wave's stores have completed, writes
# the stamps over the first 6 samples of its symbol's output.  Read by tools/experiments/o32_stamps_run.py.
ST = "  if (threadIdx.x == 0) g_o32st[blockIdx.x * 12 + %d] = (uint32_t)__builtin_amdgcn_s_memrealtime();\n"
EDITS = [
    ("""// last LDS access of the symbol on return.
__device__ __forceinline__ void o32_fft(""", """// last LDS access of the symbol on return.
__device__ uint32_t g_o32st[1 << 20];
__device__ __forceinline__ void o32_fft("""),
    ("""  o32_exchange<8>(v, lds, tid, ta, tb);
  // stage B: DFT over m1, twiddle w_1024^(m0 n1) = w_1024^(a r)""", """  o32_exchange<8>(v, lds, tid, ta, tb);
""" + ST % 5 + """  // stage B: DFT over m1, twiddle w_1024^(m0 n1) = w_1024^(a r)"""),
    ("""  o32_exchange<9>(v, lds, tid, ta, tb);
  // stage C: DFT over m0 -> x[b + 32 a + 1024 r]
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
}""", """  o32_exchange<9>(v, lds, tid, ta, tb);
""" + ST % 6 + """  // stage C: DFT over m0 -> x[b + 32 a + 1024 r]
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
""" + ST % 7 + """}"""),
    ("""  const int u = xcd_major(blockIdx.x, gridDim.x);
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase""", ST % 0 + """  const int u = xcd_major(blockIdx.x, gridDim.x);
  const int j = u / io.nframes;                   // symbol
  const int f = u - j * io.nframes;               // frame within launch
  const int64_t frame = io.first_frame + (io.frames_per_stream ? f % io.frames_per_stream : f);   // stream-major batch
  const float2 *data = io.data;
  const uint32_t cbase"""),
    ("""      scatter_group<NT, 4, MULTI>(lds, src, 0, src.d0, src.dn0, dummy, tid);
      __syncthreads();
""", """      scatter_group<NT, 4, MULTI>(lds, src, 0, src.d0, src.dn0, dummy, tid);
      __syncthreads();
""" + ST % 1),
    ("""    __syncthreads();                              // half 0 read back before half 1 overwrites it
""", """    __syncthreads();                              // half 0 read back before half 1 overwrites it
""" + ST % 2),
    ("""      scatter_group<NT, 4, MULTI>(lds, src, 1, src.d0 + src.dn0, src.dn - src.dn0, dummy, tid, dft_even);
      __syncthreads();
""", """      scatter_group<NT, 4, MULTI>(lds, src, 1, src.d0 + src.dn0, src.dn - src.dn0, dummy, tid, dft_even);
      __syncthreads();
""" + ST % 3),
    ("""  o32_fft(v, lds, tw1k, tw2, (uint32_t)tid, ta, tb);   // its first barrier publishes the tables
  const IqOut<FMT> o{(char *)io.out + ((int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + d.G)) * SB, d.gain};
  if ((((uintptr_t)o.base + (uint32_t)d.G * SB) & (2u * SB - 1u)) == 0)
    o32_store_pairs<FMT>(v, o, tb + 32u * ta, d.norm, d.G);
  else
    o32_store<FMT, 0, 32>(v, o, tb + 32u * ta, d.norm, d.G);
}""", ST % 4 + """  o32_fft(v, lds, tw1k, tw2, (uint32_t)tid, ta, tb);   // its first barrier publishes the tables
  const IqOut<FMT> o{(char *)io.out + ((int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + d.G)) * SB, d.gain};
  if ((((uintptr_t)o.base + (uint32_t)d.G * SB) & (2u * SB - 1u)) == 0)
    o32_store_pairs<FMT>(v, o, tb + 32u * ta, d.norm, d.G);
  else
    o32_store<FMT, 0, 32>(v, o, tb + 32u * ta, d.norm, d.G);
""" + ST % 8 + """  __builtin_amdgcn_s_waitcnt(0x0F70);
  __syncthreads();
""" + ST % 9 + """  if (threadIdx.x == 0) {
    uint32_t *w = (uint32_t *)o.base;
    for (int k = 0; k < 12; k++) w[k] = g_o32st[blockIdx.x * 12 + k];
    w[11] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | ((16 - 1) << 11));   // HW_ID (CU / SE / XCC ids)
  }
}"""),
]
