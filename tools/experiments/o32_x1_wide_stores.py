# 32K exchange 1 written with ds_write_b128 value pairs (lanes b, b ^ 1 swap halves) on a swizzled slot map that the
# bank model (tools/experiments/x1_banks.py) finds conflict-free for the writes and the ds_read_b128 reads; bit-exact,
# measured slower (r4ad: ofdm 1.187 -> 1.252 ms per 192 cfg3 frames)
EDITS = [
("""template <int SPLIT>
__device__ __forceinline__ void o32_exchange(float2 *v, float2 *lds, uint32_t tid, uint32_t a, uint32_t b) {""",
"""// exchange-1 slots: block B = e >> 9 starts at 528 B (16 pad slots per 512) plus an offset 2 sigma(B) < 16
// (sigma: 4-bit entries of two constants), so that the pair stores of rows r, r + 1 (blocks r, r + 1) fall
// on the two halves of the 32 banks and each ds_read_b128 group reads 16 distinct bank quads
// (tools/experiments/x1_banks.py); the largest slot is 16889, inside the data area
__device__ __forceinline__ uint32_t o32_x1(uint32_t e) {
  const uint32_t B = e >> 9;
  const uint64_t c = B < 16u ? 0x3704372615042615ull : 0x5115264004737326ull;
  return e + 16u * B + 2u * (uint32_t)((c >> (4u * (B & 15u))) & 15u);
}
template <int SPLIT>
__device__ __forceinline__ void o32_exchange(float2 *v, float2 *lds, uint32_t tid, uint32_t a, uint32_t b) {"""),
("""    if (mine) {
#pragma unroll
      for (uint32_t r = 0; r < 32; r++) {
        const uint32_t e = SPLIT == 8 ? (b & 15u) + 16u * (a & 15u) + 256u * (b >> 4) + 512u * r
                                      : (b & 15u) + 16u * (r & 15u) + 256u * (r >> 4) + 512u * a;
        lds[o32_x(e)] = v[r];
      }
    }""",
"""    if (mine) {
      if (SPLIT == 8) {
        // values (b, r) and (b ^ 1, r) are adjacent slots: lanes b and b ^ 1 swap half their values
        // (as o32_store_pairs) and each writes one pair with ds_write_b128 (a wide store keeps its rate
        // with the 8 active waves of a half; ds_write_b64 needs about 4 waves per SIMD)
        const bool odd = (b & 1u) != 0;
        const uint32_t be = b & ~1u;
#pragma unroll
        for (uint32_t k = 0; k < 16; k++) {
          const float2 e0 = v[2 * k], d0 = v[2 * k + 1];
          const float2 re = make_float2(swap_adjacent_lane(e0.x), swap_adjacent_lane(e0.y));
          const float2 rd = make_float2(swap_adjacent_lane(d0.x), swap_adjacent_lane(d0.y));
          const float2 lo = odd ? rd : e0, hi = odd ? d0 : re;
          const uint32_t e = (be & 15u) + 16u * (a & 15u) + 256u * (be >> 4) + 512u * (2u * k + (odd ? 1u : 0u));
          *(float4 *)(lds + o32_x1(e)) = make_float4(lo.x, lo.y, hi.x, hi.y);
        }
      } else {
#pragma unroll
        for (uint32_t r = 0; r < 32; r++) {
          const uint32_t e = (b & 15u) + 16u * (r & 15u) + 256u * (r >> 4) + 512u * a;
          lds[o32_x(e)] = v[r];
        }
      }
    }"""),
("""          const uint32_t e = (r & 15u) + 16u * (a & 15u) + 256u * (r >> 4) + 512u * b;
          const float4 q = *(const float4 *)(lds + o32_x(e));""",
"""          const uint32_t e = (r & 15u) + 16u * (a & 15u) + 256u * (r >> 4) + 512u * b;
          const float4 q = *(const float4 *)(lds + o32_x1(e));"""),
]
