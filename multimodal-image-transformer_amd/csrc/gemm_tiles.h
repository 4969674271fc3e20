// LDS operand tiles of the bf16 MFMA GEMM kernels (gemm.hip): the 128 x 64 / 64 x 128 bf16
// tile images filled by LDS-DMA with the swizzle applied on the source address, MFMA fragment reads,
// the XCD-aware block order and the DMA-safe barrier. Included inside gemm.hip's anonymous namespace.
#pragma once

// ------------------------------------------------------------------------------------------------
// operand tiles in LDS
// ------------------------------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;          // 16 KiB per operand per stage
constexpr int CST = BN + 4;                      // fp32 C-tile row stride in LDS (floats)
constexpr int smem_bytes(int nst) {
  return (2 * nst * TILE_BYTES > BM * CST * 4) ? 2 * nst * TILE_BYTES : BM * CST * 4;
}
constexpr uint32_t OOB = 0x80000000u;            // buffer offset past any num_records -> loads 0

// byte offset of 16-B chunk c (0..7) of row r in a K-contig [128][64] bf16 tile
__device__ __forceinline__ int koff(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// swizzle of a k-row in an MN-contig [64][128] bf16 tile (256-B rows): rows kr and kr+8 of a
// 32-lane transposed read land in different 32-B bank groups
__device__ __forceinline__ int mn_swz(int kr) { return ((kr & 3) | ((((kr >> 2) ^ (kr >> 3)) & 1) << 2)) << 5; }
__device__ __forceinline__ int mnoff(int kr, int byte_in_row) { return kr * 256 + (byte_in_row ^ mn_swz(kr)); }

// LDS-DMA fill of one 16 KiB operand tile: 1024 16-B chunks = 16 wave-instructions, wave w issues
// w*NPW .. w*NPW+NPW-1 (NPW = 16 / waves). The DMA writes each instruction's 1 KiB linearly
// (base + lane*16), so the swizzle is applied to the SOURCE address instead: linear position p holds
// logical chunk phys ^ swizzle(row) (the XOR is an involution), which reproduces exactly the
// koff / mnoff images read by frag().
template <int LAY, int NPW = 4>
__device__ __forceinline__ void glds_tile(__amdgpu_buffer_rsrc_t rs, char* tile, long ld, long rows_total, long K,
                                          long row0, long k0, int w, int lane) {
#pragma unroll
  for (int j = 0; j < NPW; ++j) {
    const int inst = w * NPW + j;
    const int id = inst * 64 + lane;
    bool ok;
    long off;
    if (LAY == MIT_K_CONTIG) {
      const int r = id >> 3, c = (id & 7) ^ ((r >> 1) & 7);
      ok = (row0 + r < rows_total) && (k0 + c * 8 < K);
      off = (row0 + r) * ld + k0 + c * 8;
    } else {
      const int kr = id >> 4, c = (id & 15) ^ (mn_swz(kr) >> 4);
      ok = (k0 + kr < K) && (row0 + c * 8 < rows_total);
      off = (k0 + kr) * ld + row0 + c * 8;
    }
    const uint32_t boff = ok ? (uint32_t)(off * 2) : OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(tile + inst * 1024), 16,
                                             boff, 0, 0, 0);
  }
}

// MFMA operand fragment: rows [rbase, rbase+16) of the tile, k-slice kk (32 wide)
template <int LAY>
__device__ __forceinline__ bf16x8 frag(const char* lds, int rbase, int kk, int lane) {
  if (LAY == MIT_K_CONTIG) {
    const int r = rbase + (lane & 15), c = kk * 4 + (lane >> 4);
    u32x4 v = *(const u32x4*)(lds + koff(r, c));
    return __builtin_bit_cast(bf16x8, v);
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int k0 = kk * 32 + g * 8 + q;
    const int colb = (rbase + 4 * p) * 2;
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + mnoff(k0, colb)));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + mnoff(k0 + 4, colb)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  }
}

// XCD-aware block order: hardware block ids round-robin over the 8 XCDs; give each XCD a
// contiguous run of tiles (bijective for any grid size) so neighbours share its L2 (guide §5.5 T1)
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / 8, rr = nwg % 8, x = bid % 8, y = bid / 8;
  return (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + y;
}

typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
// sum of the 8 bf16 of a fragment into r (fused bias-gradient row sums), v_dot2_f32_bf16
__device__ __forceinline__ float frag_rowsum(bf16x8 a, float r) {
  const bf16x2 one2 = {(bf16)1.0f, (bf16)1.0f};
  r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 0, 1), one2, r, false);
  r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 2, 3), one2, r, false);
  r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 4, 5), one2, r, false);
  r = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(a, a, 6, 7), one2, r, false);
  return r;
}

// workgroup barrier that is also a compiler scheduling / memory fence but emits no vmcnt wait
// (an in-flight LDS-DMA must survive it)
__device__ __forceinline__ void bar_raw() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
