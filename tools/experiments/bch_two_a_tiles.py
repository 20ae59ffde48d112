# BCH matrix-core pass with two A tiles per wave (64 FEC blocks per wave, 256 per workgroup tile): every B
# fragment read from LDS feeds two MFMAs instead of one (the pass is as LDS-read-bound as MFMA-bound at
# one A tile); 12 accumulators per wave, one workgroup per CU
BODY_OLD_START = "    const int row0 = tile * BCH_ROWS + wave * 32;"
BODY_NEW = r'''    const int row0 = tile * BCH_ROWS + wave * 64;
    bool live[2];
    const uint4 *msg[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {
      const int blk = row0 + 32 * i + (lane & 31);
      live[i] = blk < io.nblocks;
      msg[i] = (const uint4 *)(io.out + (int64_t)(live[i] ? blk : 0) * io.cw_stride) + (lane >> 5);
    }
    bch_v16f acc[2][NT];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int t = 0; t < NT; t++) acc[i][t] = bch_v16f{};
    __syncthreads();   // the previous segment's epilogue has read its parity words out of buffer 0
    stage(q0, 0);
    uint4 a[2];
#pragma unroll
    for (int i = 0; i < 2; i++) a[i] = live[i] ? msg[i][2 * q0] : make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();   // (its vmcnt(0) retires the DMA)
    for (int q = q0; q < q1; q++) {
      const int cur = (q - q0) & 1;
      uint4 an[2] = {make_uint4(0u, 0u, 0u, 0u), make_uint4(0u, 0u, 0u, 0u)};
      if (q + 1 < q1) {   // the other buffer was last read before the previous barrier
        stage(q + 1, cur ^ 1);
#pragma unroll
        for (int i = 0; i < 2; i++)
          if (live[i]) an[i] = msg[i][2 * (q + 1)];
      }
      const uint4 *bq = bsm + cur * PER;
      uint4 bc[NT], bx[NT];
#pragma unroll
      for (int t = 0; t < NT; t++) bc[t] = bq[t * 64 + lane];
#pragma unroll
      for (int s = 0; s < 4; s++) {
        if (s < 3) {
#pragma unroll
          for (int t = 0; t < NT; t++) bx[t] = bq[((s + 1) * NT + t) * 64 + lane];
        }
        bch_v8i A[2];
#pragma unroll
        for (int i = 0; i < 2; i++) {
          const uint32_t w = s == 0 ? a[i].x : s == 1 ? a[i].y : s == 2 ? a[i].z : a[i].w;
          A[i] = bch_v8i{(int)(w & 0x11111111u), (int)((w >> 1) & 0x11111111u), (int)((w >> 2) & 0x11111111u),
                         (int)((w >> 3) & 0x11111111u), 0, 0, 0, 0};
        }
#pragma unroll
        for (int t = 0; t < NT; t++) {
          const bch_v8i Bv = {(int)bc[t].x, (int)bc[t].y, (int)bc[t].z, (int)bc[t].w, 0, 0, 0, 0};
#pragma unroll
          for (int i = 0; i < 2; i++)
            acc[i][t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(A[i], Bv, acc[i][t], 4, 4, 0, 128, 0, 127);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < NT; t++) bc[t] = bx[t];
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 2; i++) a[i] = an[i];
    }
    uint32_t *pw = (uint32_t *)bsm + wave * 64 * BCH_PART_WORDS;   // after the loop's last barrier
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
      for (int t = 0; t < NT; t++)
#pragma unroll
        for (int r = 0; r < 16; r++) {
          const uint64_t m = __builtin_amdgcn_ballot_w64(((int)acc[i][t][r] & 1) != 0);
          const int row = 32 * i + (r & 3) + 8 * (r >> 2);
          if (lane == 0) pw[row * BCH_PART_WORDS + t] = __builtin_bswap32(__builtin_bitreverse32((uint32_t)m));
          if (lane == 1) pw[(row + 4) * BCH_PART_WORDS + t] = __builtin_bswap32(__builtin_bitreverse32((uint32_t)(m >> 32)));
        }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int i = lane; i < 64 * BCH_PART_WORDS; i += 64) {
      const int row = i / BCH_PART_WORDS, t = i % BCH_PART_WORDS;
      if (t < NT && row0 + row < io.nblocks) atomicXor(&io.bch_part[(int64_t)(row0 + row) * BCH_PART_WORDS + t], pw[i]);
    }
  }
}
'''
import pathlib
_src = (pathlib.Path(__file__).resolve().parents[2] / "gr-dvbt2ll_amd" / "csrc" / "t2_kernels.hip").read_text()
_a = _src.find(BODY_OLD_START)
_b = _src.find("\n}\n", _a) + 3
EDITS = [(_src[_a:_b], BODY_NEW),
         ("constexpr int BCH_WG_PER_CU = 3;", "constexpr int BCH_WG_PER_CU = 1;"),
         ("constexpr int BCH_ROWS = 128;           // bch_gemm_kernel: FEC blocks per workgroup (4 waves x 32)",
          "constexpr int BCH_ROWS = 256;           // bch_gemm_kernel: FEC blocks per workgroup (4 waves x 64)")]
