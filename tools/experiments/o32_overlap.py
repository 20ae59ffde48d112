# 32K OFDM: the two closed halves of each exchange in staggered epochs, so one half's DFT / twiddle /
# IQ store work runs while the other half's LDS round trip is in flight (same barriers count as the
# product: each epoch ends with one workgroup barrier)
OLD_FFT = """  o32_exchange<8>(v, lds, tid, ta, tb);
  // stage B: DFT over m1, twiddle w_1024^(m0 n1) = w_1024^(a r)
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
  o32_twiddle(v, [&](int k) { return tw1k[(ta * (uint32_t)k) & 1023u]; });
  o32_exchange<9>(v, lds, tid, ta, tb);
  // stage C: DFT over m0 -> x[b + 32 a + 1024 r]
  __builtin_amdgcn_sched_barrier(0);
  Dft<32>::run(v);
}"""
NEW_FFT = """  const uint32_t a = ta, b = tb;
  const bool g1 = (tid >> 8) & 1u, h1 = (tid >> 9) & 1u;
  auto x1w = [&]() {
#pragma unroll
    for (uint32_t r = 0; r < 32; r++) lds[o32_x((b & 15u) + 16u * (a & 15u) + 256u * (b >> 4) + 512u * r)] = v[r];
  };
  auto x1r = [&]() {
#pragma unroll
    for (uint32_t r = 0; r < 32; r += 2) {
      const float4 q = *(const float4 *)(lds + o32_x((r & 15u) + 16u * (a & 15u) + 256u * (r >> 4) + 512u * b));
      v[r] = make_float2(q.x, q.y);
      v[r + 1] = make_float2(q.z, q.w);
    }
  };
  auto x2w = [&]() {
#pragma unroll
    for (uint32_t r = 0; r < 32; r++) lds[o32_x((b & 15u) + 16u * (r & 15u) + 256u * (r >> 4) + 512u * a)] = v[r];
  };
  auto x2r = [&]() {
#pragma unroll
    for (uint32_t r = 0; r < 32; r++) v[r] = lds[o32_x((b & 15u) + 16u * (a & 15u) + 256u * (a >> 4) + 512u * r)];
  };
  auto stage_b = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    Dft<32>::run(v);
    o32_twiddle(v, [&](int k) { return tw1k[(ta * (uint32_t)k) & 1023u]; });
  };
  __syncthreads();
  if (!g1) x1w();
  __syncthreads();
  if (!g1) x1r();
  __syncthreads();
  if (g1) x1w(); else stage_b();
  __syncthreads();
  if (g1) {
    x1r();
    stage_b();
  }
  __syncthreads();
  if (!h1) x2w();
  __syncthreads();
  if (!h1) {
    x2r();
    __builtin_amdgcn_sched_barrier(0);
    Dft<32>::run(v);
  }
  __syncthreads();
  if (h1) x2w(); else store();
  __syncthreads();   // (every barrier at top level: a wave-uniform branch around s_barrier is not safe)
  if (h1) {
    x2r();
    __builtin_amdgcn_sched_barrier(0);
    Dft<32>::run(v);
    store();
  }
}"""
EDITS = [
    ("""__device__ __forceinline__ void o32_fft(float2 *v, float2 *lds, const float2 *tw1k, const float2 *tw2, uint32_t tid,
                                        uint32_t ta, uint32_t tb) {""",
     """template <class Store>
__device__ __forceinline__ void o32_fft(float2 *v, float2 *lds, const float2 *tw1k, const float2 *tw2, uint32_t tid,
                                        uint32_t ta, uint32_t tb, const Store &store) {"""),
    (OLD_FFT, NEW_FFT),
    ("""  o32_fft(v, lds, tw1k, tw2, (uint32_t)tid, ta, tb);   // its first barrier publishes the tables
  const IqOut<FMT> o{(char *)io.out + ((int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + d.G)) * SB, d.gain};
  if ((((uintptr_t)o.base + (uint32_t)d.G * SB) & (2u * SB - 1u)) == 0)
    o32_store_pairs<FMT>(v, o, tb + 32u * ta, d.norm, d.G);
  else
    o32_store<FMT, 0, 32>(v, o, tb + 32u * ta, d.norm, d.G);""",
     """  const IqOut<FMT> o{(char *)io.out + ((int64_t)f * io.out_stride + 2048 + (int64_t)j * (N + d.G)) * SB, d.gain};
  const bool pairs_ok = (((uintptr_t)o.base + (uint32_t)d.G * SB) & (2u * SB - 1u)) == 0;
  o32_fft(v, lds, tw1k, tw2, (uint32_t)tid, ta, tb, [&]() {   // its first barrier publishes the tables
    if (pairs_ok)
      o32_store_pairs<FMT>(v, o, tb + 32u * ta, d.norm, d.G);
    else
      o32_store<FMT, 0, 32>(v, o, tb + 32u * ta, d.norm, d.G);
  });"""),
]
