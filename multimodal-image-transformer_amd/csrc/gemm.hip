// Dense GEMM for every contraction of the train step (SURVEY.md §2b rows E1,E4,E6,E7,P1,D3,D5-D8
// and their backward): C[M,N] = epi( alpha * sum_k A(m,k) * B(k,n) ).
//
// Operand storage (no transpose copies ever):
//   A: MIT_K_CONTIG  -> A[m*lda + k]      (activations X, dY)
//      MIT_MN_CONTIG -> A[k*lda + m]      (dY^T in weight-grad GEMMs)
//   B: MIT_K_CONTIG  -> B[n*ldb + k]      (nn.Linear weight W[out,in] in Y = X W^T)
//      MIT_MN_CONTIG -> B[k*ldb + n]      (W in dX = dY W, X in dW = dY^T X)
//
// bf16 path: 128x128x64 block tile, 4 waves (2x2), each wave 64x64 = 4x4 tiles of
// v_mfma_f32_16x16x32_bf16, fp32 accumulation.
//   * staging: buffer loads (SRSRC descriptors) into registers -> LDS double buffer, one barrier
//     per K step. Edge tiles need no branches: an out-of-range chunk gets an offset past the
//     descriptor's num_records and the hardware returns zeros.
//   * K-contig tiles are XOR-swizzled for conflict-free ds_read_b128 fragment reads; MN-contig
//     tiles are read with ds_read_b64_tr_b16 (CDNA4 hardware transpose) so one kernel serves
//     NT / NN / TN without materialising a transpose.
//   * epilogue: the fp32 accumulator tile is staged through LDS, then every thread applies
//     bias / activation / relu-dropout mask / dropout / residual to 8 consecutive columns and
//     writes 16 bytes (coalesced rows instead of the MFMA layout's 4-row x 16-column scatter).
//   * tile order: XCD-aware remap + 8-row grouping so tiles sharing A/B panels share an L2.
// fp32 path (parity mode): a plain LDS-tiled FMA kernel with the identical epilogue semantics.
#include <stdlib.h>

#include "common.h"

namespace {

struct Epi {
  const float* bias;
  const void* res;
  long ldr;
  const void* aux;
  long ld_aux;
  float aux_scale;
  float alpha;
  int act;
  int out_f32;
  int accumulate;
  const uint64_t* seed;
  uint32_t site;
  uint32_t thresh;
  float dscale;
  int dropout;
  int vec;  // 16-B vector epilogue legal (alignments / leading dims / N multiple of 8)
};

__device__ __forceinline__ float epi_pre(const Epi& e, float v, float bias) {
  v = v * e.alpha + bias;
  if (e.act == MIT_ACT_RELU) v = fmaxf(v, 0.0f);
  else if (e.act == MIT_ACT_GELU) v = gelu_erf(v);
  else if (e.act == MIT_ACT_QUICK_GELU) v = quick_gelu(v);
  return v;
}

template <typename T>
__device__ __forceinline__ void epi_store(const Epi& e, void* C, long ldc, long N, long r, long c, float v) {
  v = epi_pre(e, v, e.bias ? e.bias[c] : 0.0f);
  if (e.aux) v *= (to_f(((const T*)e.aux)[r * e.ld_aux + c]) > 0.0f) ? e.aux_scale : 0.0f;
  if (e.dropout) v *= drop_mul(site_key(e.seed, e.site), (uint64_t)r * (uint64_t)N + (uint64_t)c, e.thresh, e.dscale);
  if (e.res) v += to_f(((const T*)e.res)[r * e.ldr + c]);
  if (e.out_f32) {
    float* o = (float*)C + r * ldc + c;
    if (e.accumulate) v += *o;
    *o = v;
  } else {
    ((T*)C)[r * ldc + c] = from_f<T>(v);
  }
}

// 8 consecutive columns [c, c+8) of row r; vector loads / stores (bf16 operands)
__device__ __forceinline__ void epi_store8_bf16(const Epi& e, void* C, long ldc, long N, long r, long c, float* v) {
  float b[8];
  if (e.bias) {
    const f32x4 b0 = *(const f32x4*)(e.bias + c), b1 = *(const f32x4*)(e.bias + c + 4);
    b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2]; b[3] = b0[3]; b[4] = b1[0]; b[5] = b1[1]; b[6] = b1[2]; b[7] = b1[3];
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = epi_pre(e, v[k], b[k]);
  if (e.aux) {
    const bf16x8 a = *(const bf16x8*)((const bf16*)e.aux + r * e.ld_aux + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= ((float)a[k] > 0.0f) ? e.aux_scale : 0.0f;
  }
  if (e.dropout) {
    const uint64_t key = site_key(e.seed, e.site);
    const uint64_t base = (uint64_t)r * (uint64_t)N + (uint64_t)c;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= drop_mul(key, base + k, e.thresh, e.dscale);
  }
  if (e.res) {
    const bf16x8 a = *(const bf16x8*)((const bf16*)e.res + r * e.ldr + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += (float)a[k];
  }
  if (e.out_f32) {
    f32x4* o = (f32x4*)((float*)C + r * ldc + c);
    f32x4 lo = {v[0], v[1], v[2], v[3]}, hi = {v[4], v[5], v[6], v[7]};
    if (e.accumulate) {
      lo += o[0];
      hi += o[1];
    }
    o[0] = lo;
    o[1] = hi;
  } else {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
    *(bf16x8*)((bf16*)C + r * ldc + c) = o;
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA kernel
// ------------------------------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;          // 16 KiB per operand per stage
constexpr int CST = BN + 4;                      // fp32 C-tile row stride in LDS (floats)
constexpr int SMEM_BYTES = (4 * TILE_BYTES > BM * CST * 4) ? 4 * TILE_BYTES : BM * CST * 4;
constexpr uint32_t OOB = 0x80000000u;            // buffer offset past any num_records -> loads 0

// byte offset of 16-B chunk c (0..7) of row r in a K-contig [128][64] bf16 tile
__device__ __forceinline__ int koff(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
// swizzle of a k-row in an MN-contig [64][128] bf16 tile (256-B rows): rows kr and kr+8 of a
// 32-lane transposed read land in different 32-B bank groups
__device__ __forceinline__ int mn_swz(int kr) { return ((kr & 3) | ((((kr >> 2) ^ (kr >> 3)) & 1) << 2)) << 5; }
__device__ __forceinline__ int mnoff(int kr, int byte_in_row) { return kr * 256 + (byte_in_row ^ mn_swz(kr)); }

template <int LAY>
struct Stage {
  u32x4 r[4];
  // BM (or BN) x BK tile at (row0 = m/n offset, k0) -> registers; out-of-range chunks read 0
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t rs, long ld, long rows_total, long K, long row0, long k0,
                                       int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i;
      bool ok;
      long off;
      if (LAY == MIT_K_CONTIG) {
        const int rr = id >> 3, c = id & 7;
        ok = (row0 + rr < rows_total) && (k0 + c * 8 < K);
        off = (row0 + rr) * ld + k0 + c * 8;
      } else {
        const int kr = id >> 4, c = id & 15;
        ok = (k0 + kr < K) && (row0 + c * 8 < rows_total);
        off = (k0 + kr) * ld + row0 + c * 8;
      }
      const uint32_t boff = ok ? (uint32_t)(off * 2) : OOB;
      r[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)boff, 0, 0));
    }
  }
  __device__ __forceinline__ void store(char* lds, int tid) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i;
      int off;
      if (LAY == MIT_K_CONTIG) off = koff(id >> 3, id & 7);
      else off = mnoff(id >> 4, (id & 15) * 16);
      *(u32x4*)(lds + off) = r[i];
    }
  }
};

// LDS-DMA fill of one 16 KiB operand tile: 1024 16-B chunks = 16 wave-instructions, wave w issues
// w*4 .. w*4+3. The DMA writes each instruction's 1 KiB linearly (base + lane*16), so the swizzle is
// applied to the SOURCE address instead: linear position p holds logical chunk phys ^ swizzle(row)
// (the XOR is an involution), which reproduces exactly the koff / mnoff images read by frag().
template <int LAY>
__device__ __forceinline__ void glds_tile(__amdgpu_buffer_rsrc_t rs, char* tile, long ld, long rows_total, long K,
                                          long row0, long k0, int w, int lane) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int inst = w * 4 + j;
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

template <int ALAY, int BLAY, bool GLDS>
__global__ __launch_bounds__(256) void gemm_bf16_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                        long M, long N, long K, long lda, long ldb, long ldc,
                                                        int a_bytes, int b_bytes, Epi e, int ksplit, long kchunk,
                                                        float* __restrict__ ws, float* __restrict__ rowsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware tile order: hardware block ids round-robin over the 8 XCDs; give each XCD a
  // contiguous run of tiles (bijective for any grid size) so neighbours share its L2 (guide §5.5 T1).
  const int nbn = (int)((N + BN - 1) / BN), nbm = (int)((M + BM - 1) / BM);
  const int ntiles = nbn * nbm, nwg = ntiles * ksplit;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, rr = nwg % 8, x = bid % 8, y = bid / 8;
    bid = (x < rr ? x * (q + 1) : rr * (q + 1) + (x - rr) * q) + y;
  }
  // split-K: slice `split` covers k in [kb, ke)
  const int split = bid / ntiles;
  bid -= split * ntiles;
  const long kb = (long)split * kchunk, ke = min(K, kb + kchunk);
  // groups of 8 M-blocks walk the N-blocks together (B panel reuse in L2)
  const int GROUP = 8;
  const int group_id = bid / (GROUP * nbn);
  const int first_m = group_id * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  const int bm = first_m + (bid % (GROUP * nbn)) % gsize;
  const int bn = (bid % (GROUP * nbn)) / gsize;
  const long m0 = (long)bm * BM, n0 = (long)bn * BN;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);

#define AS(b) (smem + (b) * 2 * TILE_BYTES)
#define BS(b) (smem + (b) * 2 * TILE_BYTES + TILE_BYTES)

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused row sums of A (bias gradients): one extra MFMA against a ones fragment, only in the
  // blocks of the first column tile and the waves of its first column half (wave-uniform branch)
  // (compiled only into the TN instance — the weight-gradient GEMMs — so the other instances
  // keep their register budget)
  const bool do_rs = ALAY == MIT_MN_CONTIG && BLAY == MIT_MN_CONTIG && rowsum != nullptr && bn == 0 && wn == 0;
  // per lane: partial row sums of its 8 k-values of rows rbase + (lane&15), via v_dot2_f32_bf16
  float rs[4] = {0.f, 0.f, 0.f, 0.f};
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
  const bf16x2 one2 = {(bf16)1.0f, (bf16)1.0f};

  const int nk = (int)((ke - kb + BK - 1) / BK);
  auto compute = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = frag<ALAY>(AS(cur), wm * 64 + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BLAY>(BS(cur), wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (do_rs) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          rs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(af[i], af[i], 0, 1), one2, rs[i], false);
          rs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(af[i], af[i], 2, 3), one2, rs[i], false);
          rs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(af[i], af[i], 4, 5), one2, rs[i], false);
          rs[i] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_shufflevector(af[i], af[i], 6, 7), one2, rs[i], false);
        }
      }
    }
  };

  if constexpr (GLDS) {
    // direct-to-LDS buffer loads (LDS-DMA): no staging registers, no ds_write pass. Two stages:
    // the next tile's DMA is in flight while this tile computes; counted vmcnt + raw barriers
    // (a __syncthreads() would drain the in-flight DMA with vmcnt(0), guide §5).
    glds_tile<ALAY>(ra, AS(0), lda, M, ke, m0, kb, wid, lane);
    glds_tile<BLAY>(rb, BS(0), ldb, N, ke, n0, kb, wid, lane);
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      if (kt + 1 < nk) {
        glds_tile<ALAY>(ra, AS(cur ^ 1), lda, M, ke, m0, kb + (long)(kt + 1) * BK, wid, lane);
        glds_tile<BLAY>(rb, BS(cur ^ 1), ldb, N, ke, n0, kb + (long)(kt + 1) * BK, wid, lane);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this tile's 8 DMAs done, next 8 in flight
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();  // every wave's DMA of tile kt has landed
      compute(cur);
      __builtin_amdgcn_s_barrier();  // every wave is done reading buffer cur before it is refilled
    }
  } else {
    Stage<ALAY> sa;
    Stage<BLAY> sb;
    sa.load(ra, lda, M, ke, m0, kb, tid);
    sb.load(rb, ldb, N, ke, n0, kb, tid);
    sa.store(AS(0), tid);
    sb.store(BS(0), tid);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      const bool more = kt + 1 < nk;
      if (more) {
        sa.load(ra, lda, M, ke, m0, kb + (long)(kt + 1) * BK, tid);
        sb.load(rb, ldb, N, ke, n0, kb + (long)(kt + 1) * BK, tid);
      }
      compute(cur);
      if (more) {
        sa.store(AS(cur ^ 1), tid);
        sb.store(BS(cur ^ 1), tid);
      }
      __syncthreads();
    }
  }
#undef AS
#undef BS

  // ---- epilogue: accumulators -> LDS (fp32 [128][CST]) -> 8-column vector rows ----
  float* cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        cs[(wm * 64 + i * 16 + (lane >> 4) * 4 + t) * CST + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][t];
  if (do_rs) {
    // lanes l, l+16, l+32, l+48 hold the four k-groups of row (l & 15): reduce across them
    float* dst = ksplit > 1 ? ws + (long)ksplit * M * N + (long)split * M : rowsum;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const long r = m0 + wm * 64 + i * 16 + (lane & 15);
      if (lane < 16 && r < M) dst[r] = v;
    }
  }
  __syncthreads();
#pragma unroll 2
  for (int pass = 0; pass < (BM * BN / 8) / 256; ++pass) {
    const int id = pass * 256 + tid;
    const int r = id >> 4, c8 = (id & 15) * 8;
    const long gr = m0 + r, gc = n0 + c8;
    if (gr >= M || gc >= N) continue;
    float v[8];
    const f32x4 lo = *(const f32x4*)(cs + r * CST + c8), hi = *(const f32x4*)(cs + r * CST + c8 + 4);
    if (ksplit > 1) {  // raw fp32 partial slab; gemm_splitk_reduce applies the (plain) epilogue
      f32x4* o = (f32x4*)(ws + ((long)split * M + gr) * N + gc);
      o[0] = lo;
      o[1] = hi;
      continue;
    }
    v[0] = lo[0]; v[1] = lo[1]; v[2] = lo[2]; v[3] = lo[3]; v[4] = hi[0]; v[5] = hi[1]; v[6] = hi[2]; v[7] = hi[3];
    if (e.vec && gc + 8 <= N) {
      epi_store8_bf16(e, C, ldc, N, gr, gc, v);
    } else {
      for (int k = 0; k < 8; ++k)
        if (gc + k < N) epi_store<bf16>(e, C, ldc, N, gr, gc + k, v[k]);
    }
  }
}

// C = alpha * sum_s slab[s] (f32 or bf16 out, optional accumulate); rowsum = sum_s rowslab[s]
__global__ void gemm_splitk_reduce(long M, long N, int ksplit, const float* __restrict__ ws, void* C, long ldc,
                                   float alpha, int out_f32, int accumulate, float* rowsum) {
  const long n4 = N / 4, total = M * n4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long r = i / n4, c = (i % n4) * 4;
    f32x4 s = *(const f32x4*)(ws + r * N + c);
    for (int k = 1; k < ksplit; ++k) s += *(const f32x4*)(ws + ((long)k * M + r) * N + c);
    s *= alpha;
    if (out_f32) {
      f32x4* o = (f32x4*)((float*)C + r * ldc + c);
      if (accumulate) s += *o;
      *o = s;
    } else {
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      *(bf16x4*)((bf16*)C + r * ldc + c) = bf16x4{(bf16)s[0], (bf16)s[1], (bf16)s[2], (bf16)s[3]};
    }
  }
  if (rowsum) {
    const float* rw = ws + (long)ksplit * M * N;
    for (long r = (long)blockIdx.x * blockDim.x + threadIdx.x; r < M; r += (long)gridDim.x * blockDim.x) {
      float s = 0.f;
      for (int k = 0; k < ksplit; ++k) s += rw[(long)k * M + r];
      rowsum[r] = s;
    }
  }
}

// split-K plan for a plain-epilogue bf16 GEMM: only when the output has too few 128x128 tiles to
// fill 256 CUs and K is long (the weight-gradient shapes). Returns 1 (no split) otherwise.
int splitk_plan(long M, long N, long K, long* kchunk) {
  const long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  *kchunk = K;
  if (tiles >= 256 || K < 1024 || N % 8) return 1;
  long s = (512 + tiles - 1) / tiles;
  s = min(s, K / 512);
  s = min(s, 16L);
  if (s < 2) return 1;
  long kc = (K + s - 1) / s;
  kc = (kc + BK - 1) / BK * BK;
  *kchunk = kc;
  return (int)((K + kc - 1) / kc);
}
long splitk_ws_bytes(long M, long N, int s) { return s > 1 ? 4L * s * M * N + 4L * s * M : 0; }

// ------------------------------------------------------------------------------------------------
// fp32 FMA kernel (parity mode): 64x64x16 tile, 256 threads x (4x4) outputs
// ------------------------------------------------------------------------------------------------
template <int ALAY, int BLAY>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, const float* __restrict__ B, void* C,
                                                       long M, long N, long K, long lda, long ldb, long ldc, Epi e,
                                                       float* __restrict__ rowsum) {
  __shared__ float As[16][64 + 4];
  __shared__ float Bs[16][64 + 4];
  const int tid = threadIdx.x;
  const long m0 = (long)blockIdx.y * 64, n0 = (long)blockIdx.x * 64;
  const int tm = (tid >> 4) * 4, tn = (tid & 15) * 4;
  float acc[4][4] = {};
  float rsum[4] = {0.f, 0.f, 0.f, 0.f};
  const bool do_rs = rowsum != nullptr && blockIdx.x == 0 && tn == 0;
  for (long k0 = 0; k0 < K; k0 += 16) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int id = tid + 256 * i;  // 0..1023 over 64 x 16
      int mm, kk;
      if (ALAY == MIT_K_CONTIG) { mm = id >> 4; kk = id & 15; } else { kk = id >> 6; mm = id & 63; }
      const long gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < M && gk < K) v = (ALAY == MIT_K_CONTIG) ? A[gm * lda + gk] : A[gk * lda + gm];
      As[kk][mm] = v;
      int nn;
      if (BLAY == MIT_K_CONTIG) { nn = id >> 4; kk = id & 15; } else { kk = id >> 6; nn = id & 63; }
      const long gn = n0 + nn, gk2 = k0 + kk;
      float w = 0.f;
      if (gn < N && gk2 < K) w = (BLAY == MIT_K_CONTIG) ? B[gn * ldb + gk2] : B[gk2 * ldb + gn];
      Bs[kk][nn] = w;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < 16; ++kk) {
      float a[4], b[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = As[kk][tm + i];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = Bs[kk][tn + j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(a[i], b[j], acc[i][j]);
      if (do_rs) {
#pragma unroll
        for (int i = 0; i < 4; ++i) rsum[i] += a[i];
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const long r = m0 + tm + i, c = n0 + tn + j;
      if (r < M && c < N) epi_store<float>(e, C, ldc, N, r, c, acc[i][j]);
    }
  if (do_rs) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (m0 + tm + i < M) rowsum[m0 + tm + i] = rsum[i];
  }
}

template <int AL, int BL>
void launch_bf16(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, int ksplit, long kchunk,
                 hipStream_t s) {
  const long nbm = (g->M + BM - 1) / BM, nbn = (g->N + BN - 1) / BN;
  static const int glds = getenv("MIT_GEMM_GLDS") ? atoi(getenv("MIT_GEMM_GLDS")) : 1;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<AL, BL, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              SMEM_BYTES);
    (void)hipFuncSetAttribute((const void*)gemm_bf16_kernel<AL, BL, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              SMEM_BYTES);
    attr = true;
  }
  if (glds)
    hipLaunchKernelGGL((gemm_bf16_kernel<AL, BL, true>), dim3((unsigned)(nbm * nbn * ksplit)), dim3(256), SMEM_BYTES, s,
                       (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                       b_bytes, e, ksplit, kchunk, (float*)g->workspace, g->rowsum);
  else
    hipLaunchKernelGGL((gemm_bf16_kernel<AL, BL, false>), dim3((unsigned)(nbm * nbn * ksplit)), dim3(256), SMEM_BYTES,
                       s, (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                       b_bytes, e, ksplit, kchunk, (float*)g->workspace, g->rowsum);
}
template <int AL, int BL>
void launch_f32(const mit_gemm_args* g, const Epi& e, hipStream_t s) {
  dim3 grid((unsigned)((g->N + 63) / 64), (unsigned)((g->M + 63) / 64));
  hipLaunchKernelGGL((gemm_f32_kernel<AL, BL>), grid, dim3(256), 0, s, (const float*)g->A, (const float*)g->B, g->C, g->M,
                     g->N, g->K, g->lda, g->ldb, g->ldc, e, g->rowsum);
}

inline bool al16(const void* p) { return ((uintptr_t)p % 16) == 0; }

}  // namespace



extern "C" long mit_gemm_workspace_bytes(long M, long N, long K) {
  long kc;
  return splitk_ws_bytes(M, N, splitk_plan(M, N, K, &kc));
}

extern "C" int mit_gemm(const mit_gemm_args* g, void* stream) {
  MIT_CHECK_ARG(g != nullptr, "mit_gemm: null args");
  MIT_CHECK_ARG(g->dtype == MIT_F32 || g->dtype == MIT_BF16, "mit_gemm: bad dtype %d", g->dtype);
  MIT_CHECK_ARG(g->M >= 0 && g->N >= 0 && g->K >= 0, "mit_gemm: negative extent");
  MIT_CHECK_ARG(g->A && g->B && g->C, "mit_gemm: null operand");
  MIT_CHECK_ARG(g->a_layout == MIT_K_CONTIG || g->a_layout == MIT_MN_CONTIG, "mit_gemm: bad a_layout");
  MIT_CHECK_ARG(g->b_layout == MIT_K_CONTIG || g->b_layout == MIT_MN_CONTIG, "mit_gemm: bad b_layout");
  if (g->M == 0 || g->N == 0) return MIT_OK;
  MIT_CHECK_ARG(g->lda >= (g->a_layout == MIT_K_CONTIG ? g->K : g->M), "mit_gemm: lda too small");
  MIT_CHECK_ARG(g->ldb >= (g->b_layout == MIT_K_CONTIG ? g->K : g->N), "mit_gemm: ldb too small");
  MIT_CHECK_ARG(g->ldc >= g->N, "mit_gemm: ldc too small");
  MIT_CHECK_ARG(!g->accumulate || g->out_f32, "mit_gemm: accumulate needs an f32 output");
  MIT_CHECK_ARG(!g->rowsum || g->dtype == MIT_F32 || (g->a_layout == MIT_MN_CONTIG && g->b_layout == MIT_MN_CONTIG),
                "mit_gemm(bf16): rowsum is fused into the weight-gradient (MN, MN) layout only");
  long a_bytes = 0, b_bytes = 0;
  if (g->dtype == MIT_BF16) {
    // 16-byte vector staging: contiguous extents and leading dims in multiples of 8 elements
    MIT_CHECK_ARG(g->lda % 8 == 0 && g->ldb % 8 == 0, "mit_gemm(bf16): lda/ldb must be multiples of 8");
    MIT_CHECK_ARG(g->a_layout == MIT_MN_CONTIG ? g->M % 8 == 0 : g->K % 8 == 0,
                  "mit_gemm(bf16): A's contiguous extent must be a multiple of 8");
    MIT_CHECK_ARG(g->b_layout == MIT_MN_CONTIG ? g->N % 8 == 0 : g->K % 8 == 0,
                  "mit_gemm(bf16): B's contiguous extent must be a multiple of 8");
    MIT_CHECK_ARG(al16(g->A) && al16(g->B), "mit_gemm(bf16): A/B must be 16-B aligned");
    a_bytes = 2 * (g->a_layout == MIT_K_CONTIG ? (g->M - 1) * g->lda + g->K : (g->K - 1) * g->lda + g->M);
    b_bytes = 2 * (g->b_layout == MIT_K_CONTIG ? (g->N - 1) * g->ldb + g->K : (g->K - 1) * g->ldb + g->N);
    if (g->K == 0) a_bytes = b_bytes = 0;
    MIT_CHECK_ARG(a_bytes < (1L << 31) && b_bytes < (1L << 31), "mit_gemm(bf16): operand spans >= 2 GiB");
  }
  Epi e;
  e.bias = g->bias;
  e.res = g->residual;
  e.ldr = g->ldr;
  e.aux = g->aux;
  e.ld_aux = g->ld_aux;
  e.aux_scale = g->aux_scale;
  e.alpha = g->alpha;
  e.act = g->act;
  e.out_f32 = g->out_f32;
  e.accumulate = g->accumulate;
  e.seed = g->seed;
  e.site = g->site;
  e.dropout = g->drop_p > 0.0f;
  e.thresh = drop_threshold(g->drop_p);
  e.dscale = g->drop_p < 1.0f ? 1.0f / (1.0f - g->drop_p) : 0.0f;
  e.vec = (g->N % 8 == 0) && (g->ldc % 8 == 0) && al16(g->C) && (!g->bias || al16(g->bias)) &&
          (!g->residual || (g->ldr % 8 == 0 && al16(g->residual))) && (!g->aux || (g->ld_aux % 8 == 0 && al16(g->aux)));
  hipStream_t s = (hipStream_t)stream;
  if (g->dtype == MIT_BF16) {
    const int ab = (int)a_bytes, bb = (int)b_bytes;
    long kchunk = g->K;
    int ks = 1;
    const bool plain = !g->bias && g->act == MIT_ACT_NONE && !g->residual && !g->aux && g->drop_p <= 0.f;
    if (plain && g->workspace) {
      ks = splitk_plan(g->M, g->N, g->K, &kchunk);
      if (ks > 1 && (splitk_ws_bytes(g->M, g->N, ks) > g->workspace_bytes || !al16(g->workspace) ||
                     (g->out_f32 ? false : (g->ldc % 4 != 0)) || g->ldc % 4 != 0 || !al16(g->C))) {
        ks = 1;
        kchunk = g->K;
      }
    }
    if (g->a_layout == 0 && g->b_layout == 0) launch_bf16<0, 0>(g, e, ab, bb, ks, kchunk, s);
    else if (g->a_layout == 0 && g->b_layout == 1) launch_bf16<0, 1>(g, e, ab, bb, ks, kchunk, s);
    else if (g->a_layout == 1 && g->b_layout == 0) launch_bf16<1, 0>(g, e, ab, bb, ks, kchunk, s);
    else launch_bf16<1, 1>(g, e, ab, bb, ks, kchunk, s);
    if (ks > 1) {
      MIT_LAUNCH_CHECK("mit_gemm");
      const long total = g->M * (g->N / 4);
      long blocks = (total + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, g->M, g->N, ks,
                         (const float*)g->workspace, g->C, g->ldc, g->alpha, g->out_f32, g->accumulate, g->rowsum);
    }
  } else {
    if (g->a_layout == 0 && g->b_layout == 0) launch_f32<0, 0>(g, e, s);
    else if (g->a_layout == 0 && g->b_layout == 1) launch_f32<0, 1>(g, e, s);
    else if (g->a_layout == 1 && g->b_layout == 0) launch_f32<1, 0>(g, e, s);
    else launch_f32<1, 1>(g, e, s);
  }
  MIT_LAUNCH_CHECK("mit_gemm");
  return MIT_OK;
}
