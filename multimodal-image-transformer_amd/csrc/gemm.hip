// Dense GEMM for every contraction of the train step (SURVEY.md §2b rows E1,E4,E6,E7,P1,D3,D5-D8
// and their backward): C[M,N] = epi( alpha * sum_k A(m,k) * B(k,n) ).
//
// Operand storage (no transpose copies ever):
//   A: MIT_K_CONTIG  -> A[m*lda + k]      (activations X, dY)
//      MIT_MN_CONTIG -> A[k*lda + m]      (dY^T in weight-grad GEMMs)
//   B: MIT_K_CONTIG  -> B[n*ldb + k]      (nn.Linear weight W[out,in] in Y = X W^T)
//      MIT_MN_CONTIG -> B[k*ldb + n]      (W in dX = dY W, X in dW = dY^T X)
//
// Two bf16 tile kernels, fp32 accumulation on v_mfma_f32_16x16x32_bf16, both staging operands
// HBM -> LDS by LDS-DMA (buffer_load ... lds) with the swizzle applied on the source address:
//   * gemm_bf16_kernel: 128x128x64, 8 waves (4x2, 32x64 each), 2 blocks per CU, 2 LDS stages,
//     optional split-K with fused bias-gradient row sums (weight gradients).
//   * gemm256_kernel: 256x256x64, 8 waves (2x4, 128x64 each), 1 block per CU, 4-phase ping-pong
//     schedule with half-tile DMA granularity and counted vmcnt (large GEMMs: the encoder's
//     M = B*197 rows). mit_gemm picks per shape with an occupancy-quantised cost model.
//   * K-contig tiles are XOR-swizzled for conflict-free ds_read_b128 fragment reads; MN-contig
//     tiles are read with ds_read_b64_tr_b16 (CDNA4 hardware transpose) so one kernel serves
//     NT / NN / TN without materialising a transpose. Out-of-range chunks get a buffer offset
//     past num_records and read as zeros: no edge branches in the main loops.
//   * epilogue: each lane applies the fused epilogue to 8 consecutive columns and writes 16 bytes,
//     with every operand load (bias, residual / aux mask) issued before the tile's first store
//     (vmcnt counts stores on gfx9). The 128 kernel stages accumulators through LDS; the 256
//     kernel (K-contig A) accumulates C^T blocks (swapped MFMA operands) so a lane holds 4
//     consecutive columns, and v_permlane16_swap pairs make 8 -- no LDS stage, no barrier. The
//     activation and dropout are TEMPLATE parameters (an 8-wide GELU / dropout-hash epilogue
//     evaluated behind runtime flags costs ~20 % of a K=768 GEMM); bias / residual / aux-mask /
//     f32-accumulate stay runtime flags.
//   * tile order: XCD-aware remap + row grouping so tiles sharing A/B panels share an L2.
// fp32 path (parity mode): an LDS-tiled kernel on the exact-f32 MFMA (v_mfma_f32_32x32x2_f32) with the
// identical epilogue semantics.
#include <stdlib.h>

#include <cmath>
#include <type_traits>
#include <vector>

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
  // LayerNorm folded into the GEMM (256 kernel, STG 3): A = the raw rows x, the epilogue applies
  // rstd_m (acc - mean_m colsum_n) + bias_n with (mean, rstd) merged from ln_stats [M][ln_parts][2]
  const float* ln_stats;
  const float* ln_colsum;
  int ln_parts;
  float ln_eps;
  // per-64-column (mean, M2) of each output row (256 kernel, STG 4): stats_out [M][N / 64][2]
  float* stats_out;
  // the greedy argmax of each row folded in (128 kernel, gathered epilogue): keys [MIT_ARGMAX_SLOTS][M]
  unsigned long long* argmax_keys;
};

// ord(v) << 32 | (0xFFFFFFFF - column): the order of (value, first column) as one u64, NaN largest
// (mit_decode_gemm's argmax keys, decode.hip)
__device__ __forceinline__ uint64_t argmax_key(float v, long col) {
  const uint32_t u = __float_as_uint(v);
  const uint32_t o = v != v ? 0xFFFFFFFFu : ((u & 0x80000000u) ? ~u : (u | 0x80000000u));
  return ((uint64_t)o << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)col);
}

constexpr int ACT_RT = -1;
  // activation read from Epi::act at run time (generic instance)

// FAST: bf16 vector epilogues use the one-exp GELU (gelu_fast, relative error <= 6.6e-6, far below
// bf16 rounding); the scalar / fp32-parity path keeps ocml's erff
template <int ACT, bool FAST = false>
__device__ __forceinline__ float act_apply(int rt, float v) {
  const int a = ACT == ACT_RT ? rt : ACT;
  if (a == MIT_ACT_RELU) v = fmaxf(v, 0.0f);
  else if (a == MIT_ACT_GELU) v = FAST ? gelu_fast(v) : gelu_erf(v);
  else if (a == MIT_ACT_QUICK_GELU) v = quick_gelu(v);
  return v;
}

// scalar epilogue (ragged column edges and the fp32 kernel): every feature at run time
template <typename T>
__device__ __forceinline__ void epi_store(const Epi& e, void* C, long ldc, long N, long r, long c, float v) {
  v = act_apply<ACT_RT>(e.act, v * e.alpha + (e.bias ? e.bias[c] : 0.0f));
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

// 8 consecutive columns [c, c+8) of row r (bf16 operands), vector loads / stores
template <int ACT, bool DROP>
__device__ __forceinline__ void epi8(const Epi& e, void* C, long ldc, long N, long r, long c, float* v) {
  float b[8];
  if (e.bias) {
    const f32x4 b0 = *(const f32x4*)(e.bias + c), b1 = *(const f32x4*)(e.bias + c + 4);
    b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2]; b[3] = b0[3]; b[4] = b1[0]; b[5] = b1[1]; b[6] = b1[2]; b[7] = b1[3];
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = 0.f;
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = v[k] * e.alpha + b[k];
  if (ACT == MIT_ACT_GELU) {  // packed pairs (v_pk_* FP32): the fc1 + GELU epilogue is VALU-bound
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      const f32x2 r = gelu_fast2(f32x2{v[k], v[k + 1]});
      v[k] = r[0];
      v[k + 1] = r[1];
    }
  } else if (ACT == MIT_ACT_QUICK_GELU) {
    quick_gelu_fast_n<8>(v);
  } else if (ACT != MIT_ACT_NONE) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_apply<ACT, true>(e.act, v[k]);
  }
  if (e.aux) {
    const bf16x8 a = *(const bf16x8*)((const bf16*)e.aux + r * e.ld_aux + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= ((float)a[k] > 0.0f) ? e.aux_scale : 0.0f;
  }
  if (DROP && e.dropout) {
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

// one staged row segment: vector epilogue when legal, else the scalar one per in-range column
template <int ACT, bool DROP>
__device__ __forceinline__ void epi_row8(const Epi& e, void* C, long ldc, long N, long gr, long gc, float* v) {
  if (e.vec && gc + 8 <= N) {
    epi8<ACT, DROP>(e, C, ldc, N, gr, gc, v);
  } else {
    for (int k = 0; k < 8; ++k)
      if (gc + k < N) epi_store<bf16>(e, C, ldc, N, gr, gc + k, v[k]);
  }
}

// ---- gathered epilogue: every operand load of a tile's epilogue issued before its first store ----
// On gfx9 vmcnt counts stores as well as loads, so a load issued after a store is waited for
// together with that store: an epilogue that loads bias / residual per row segment between its
// stores serialises one store round trip per segment (7-35 us per launch of the 256 kernel on the
// encoder shapes). The gathered form loads the bias of the thread's fixed columns once and the
// residual (or aux mask) of all its segments, then only computes and stores. It covers every
// epilogue except residual AND aux together, f32 accumulate and the non-vector (ragged ldc)
// case, which keep the per-segment form (epi_row8).
__host__ __device__ __forceinline__ bool epi_gatherable(const Epi& e) { return e.vec && !(e.res && e.aux) && !e.accumulate; }
__device__ __forceinline__ void epi_bias8(const Epi& e, long c, long N, float* b) {
  if (e.bias && c < N) {
    const f32x4 b0 = *(const f32x4*)(e.bias + c), b1 = *(const f32x4*)(e.bias + c + 4);
    b[0] = b0[0]; b[1] = b0[1]; b[2] = b0[2]; b[3] = b0[3]; b[4] = b1[0]; b[5] = b1[1]; b[6] = b1[2]; b[7] = b1[3];
  } else {
#pragma unroll
    for (int k = 0; k < 8; ++k) b[k] = 0.f;
  }
}
// the residual (or aux) segment of row r, columns [c, c+8); zeros when absent / out of range
__device__ __forceinline__ bf16x8 epi_x8(const Epi& e, long M, long N, long r, long c) {
  bf16x8 x = {};
  const bf16* src = (const bf16*)(e.res ? e.res : e.aux);
  if (src && r < M && c < N) x = *(const bf16x8*)(src + r * (e.res ? e.ldr : e.ld_aux) + c);
  return x;
}
// s_waitcnt vmcnt(0) as a builtin (the compiler's waitcnt pass sees it, unlike inline asm): closes a
// gathered epilogue's load phase (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15)
__device__ __forceinline__ void gather_wait() { __builtin_amdgcn_s_waitcnt(0x0F70); }
template <bool DROP>
__device__ __forceinline__ uint64_t epi_key(const Epi& e) {
  return (DROP && e.dropout) ? site_key(e.seed, e.site) : 0ull;
}
// epi8 with the operands from registers (b: bias of the 8 columns, x: residual or aux segment)
template <int ACT, bool DROP>
__device__ __forceinline__ void epi8x(const Epi& e, void* C, long ldc, long N, long r, long c, float* v, const float* b,
                                      bf16x8 x, uint64_t key) {
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = v[k] * e.alpha + b[k];
  if (ACT == MIT_ACT_GELU) {
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      const f32x2 g = gelu_fast2(f32x2{v[k], v[k + 1]});
      v[k] = g[0];
      v[k + 1] = g[1];
    }
  } else if (ACT == MIT_ACT_QUICK_GELU) {
    quick_gelu_fast_n<8>(v);
  } else if (ACT != MIT_ACT_NONE) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = act_apply<ACT, true>(e.act, v[k]);
  }
  if (e.aux) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= ((float)x[k] > 0.0f) ? e.aux_scale : 0.0f;
  }
  if (DROP && e.dropout) {
    const uint64_t base = (uint64_t)r * (uint64_t)N + (uint64_t)c;
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] *= drop_mul(key, base + k, e.thresh, e.dscale);
  }
  if (e.res) {
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] += (float)x[k];
  }
  if (e.out_f32) {
    f32x4* o = (f32x4*)((float*)C + r * ldc + c);
    o[0] = f32x4{v[0], v[1], v[2], v[3]};
    o[1] = f32x4{v[4], v[5], v[6], v[7]};
  } else {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
    *(bf16x8*)((bf16*)C + r * ldc + c) = o;
  }
}

#include "gemm_tiles.h"  // LDS operand tiles, LDS-DMA fill, MFMA fragments


// ------------------------------------------------------------------------------------------------
// bf16 MFMA kernel, 128x128 block tile
// ------------------------------------------------------------------------------------------------
// this wave's DMAs of all but `younger` tiles landed (PER = DMA pieces per tile per wave)
template <int NST, int PER = 8>
__device__ __forceinline__ void wait_tiles(int younger) {
  if constexpr (PER == 8) {
    if (NST > 3 && younger >= 3) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
    else if (NST > 2 && younger == 2) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else if (younger >= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    static_assert(PER == 4, "wait_tiles: 4 or 8 pieces per tile");
    if (NST > 3 && younger >= 3) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (NST > 2 && younger == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (younger >= 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// NST = LDS stages (K-tiles resident at once). Launched with 2 (64 KiB: two blocks per CU). Four
// stages (three tiles in flight) on the 1-block-per-CU decoder grids measured no faster (within
// 2 %, tools/gemm_bench.py): those blocks are bound by per-iteration latency, not DMA depth.
// The body takes its block index (blk) so a grouped launch (gemm_bf16_grouped) can run several
// problems' blocks in one grid.
template <int ALAY, int BLAY, int ACT, bool DROP, int NST, int NW>
__device__ __forceinline__ void gemm_bf16_body(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                               long M, long N, long K, long lda, long ldb, long ldc, int a_bytes,
                                               int b_bytes, const Epi& e, int ksplit, long kchunk,
                                               float* __restrict__ ws, float* __restrict__ rowsum, int blk,
                                               int GROUP = 8) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // NW = 4: waves 2 (M) x 2 (N), 64x64 each; NW = 8: 4 (M) x 2 (N), 32x64 each (MI 16-row blocks)
  constexpr int NT = 64 * NW, WR = 128 / (NW / 2), MI = WR / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int nbn = (int)((N + BN - 1) / BN), nbm = (int)((M + BM - 1) / BM);
  const int ntiles = nbn * nbm, nwg = ntiles * ksplit;
  // GROUP = 0 (the grouped dW launch): blk is already the tile's index in its problem's XCD-piece
  // order (grouped_tile), no remap
  int bid = GROUP ? xcd_remap(blk, nwg) : blk;
  // split-K: slice `split` covers k in [kb, ke); a tile's slices are neighbours in the remapped
  // order, i.e. on one XCD
  const int split = bid % ksplit;
  bid /= ksplit;
  const long kb = (long)split * kchunk, ke = min(K, kb + kchunk);
  int bm, bn;
  if (GROUP) {
    // groups of GROUP M-blocks walk the N-blocks together (B panel reuse in L2)
    const int group_id = bid / (GROUP * nbn);
    const int first_m = group_id * GROUP;
    const int gsize = min(nbm - first_m, GROUP);
    bm = first_m + (bid % (GROUP * nbn)) % gsize;
    bn = (bid % (GROUP * nbn)) / gsize;
  } else if (nbn <= nbm) {  // the shorter side fastest: a contiguous run of tiles is a compact block
    bm = bid / nbn;
    bn = bid % nbn;
  } else {
    bm = bid % nbm;
    bn = bid / nbm;
  }
  const long m0 = (long)bm * BM, n0 = (long)bn * BN;
  MIT_DASSERT(blk < nwg && split < ksplit && bm < nbm && bn < nbn && m0 < M && n0 < N);
  MIT_DASSERT(lda >= (ALAY == MIT_K_CONTIG ? K : M) && ldb >= (BLAY == MIT_K_CONTIG ? K : N) && ldc >= N);

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);

#define AS(b) (smem + (b) * 2 * TILE_BYTES)
#define BS(b) (smem + (b) * 2 * TILE_BYTES + TILE_BYTES)

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fused row sums of A (bias gradients): only the TN instance (weight-gradient GEMMs), blocks of
  // the first column tile, waves of its first column half (wave-uniform branch)
  const bool do_rs = ALAY == MIT_MN_CONTIG && BLAY == MIT_MN_CONTIG && rowsum != nullptr && bn == 0 && wn == 0;
  float rs[MI] = {};

  const int nk = (int)((ke - kb + BK - 1) / BK);
  auto compute = [&](int cur) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[4];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = frag<ALAY>(AS(cur), wm * WR + i * 16, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[j] = frag<BLAY>(BS(cur), wn * 64 + j * 16, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      if (do_rs) {
#pragma unroll
        for (int i = 0; i < MI; ++i) rs[i] = frag_rowsum(af[i], rs[i]);
      }
    }
  };

  {
  // LDS-DMA, NST stages: NST-1 tiles' DMA in flight while one computes; counted vmcnt (8 DMAs per
  // tile per wave) + raw barriers (a __syncthreads() would drain the in-flight DMA with vmcnt(0), guide §5)
  constexpr int PF = NST - 1;
#pragma unroll
  for (int t = 0; t < PF; ++t)
    if (t < nk) {
      glds_tile<ALAY, 16 / NW>(ra, AS(t), lda, M, ke, m0, kb + (long)t * BK, wid, lane);
      glds_tile<BLAY, 16 / NW>(rb, BS(t), ldb, N, ke, n0, kb + (long)t * BK, wid, lane);
    }
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % NST;
    if (kt + PF < nk) {  // refills the buffer computed in iteration kt-1 (behind its closing barrier)
      const int nb = (kt + PF) % NST;
      glds_tile<ALAY, 16 / NW>(ra, AS(nb), lda, M, ke, m0, kb + (long)(kt + PF) * BK, wid, lane);
      glds_tile<BLAY, 16 / NW>(rb, BS(nb), ldb, N, ke, n0, kb + (long)(kt + PF) * BK, wid, lane);
    }
    wait_tiles<NST, 2 * (16 / NW)>(min(nk - 1 - kt, PF));
    bar_raw();  // every wave's DMA of tile kt has landed
    compute(cur);
    // every wave's fragment reads of buffer cur have RETURNED before any wave refills it: a bare
    // __builtin_amdgcn_s_barrier() is no memory fence, and hipcc issued the second k-slice's ds_reads
    // before it with their lgkmcnt waits after, so a fast wave's next DMA could overwrite the buffer
    // under a slow wave's in-flight reads (seen as run-to-run differences of the decoder GEMMs when
    // the encoder prefetch shared the chip: tools/diag_race.py)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar_raw();
  }
  }
#undef AS
#undef BS

  // ---- epilogue: accumulators -> LDS (fp32 [128][CST]) -> 8-column vector rows ----
  float* cs = (float*)smem;
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t)
        cs[(wm * WR + i * 16 + (lane >> 4) * 4 + t) * CST + wn * 64 + j * 16 + (lane & 15)] = acc[i][j][t];
  if (do_rs) {
    // lanes l, l+16, l+32, l+48 hold the four k-groups of row (l & 15): reduce across them
    float* dst = ksplit > 1 ? ws + (long)ksplit * M * N + (long)split * M : rowsum;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const long r = m0 + wm * WR + i * 16 + (lane & 15);
      if (lane < 16 && r < M) dst[r] = v;
    }
  }
  __syncthreads();
  if (ksplit == 1 && epi_gatherable(e)) {  // gathered epilogue: all loads, then all stores
    constexpr int NP = (BM * BN / 8) / NT;
    const long gc = n0 + (tid & 15) * 8;  // this thread's columns are the same in every pass
    float b[8];
    epi_bias8(e, gc, N, b);
    bf16x8 xs[NP];
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) xs[pass] = epi_x8(e, M, N, m0 + ((pass * NT + tid) >> 4), gc);
    gather_wait();
    const uint64_t key = epi_key<DROP>(e);
    if (ACT == MIT_ACT_NONE && !DROP && e.argmax_keys) {  // the rows' argmax over this tile's 128 columns
#pragma unroll
      for (int pass = 0; pass < NP; ++pass) {
        const int r = (pass * NT + tid) >> 4, c8 = (tid & 15) * 8;
        const long gr = m0 + r;
        uint64_t best = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint64_t kk = argmax_key(cs[r * CST + c8 + k] + b[k], gc + k);
          if (gc + k < N && kk > best) best = kk;
        }
#pragma unroll
        for (int x = 1; x < 16; x <<= 1) {  // the row's 16 lanes (tid & 15)
          const uint64_t o = ((uint64_t)(uint32_t)__shfl_xor((int)(best >> 32), x, 64) << 32) |
                             (uint32_t)__shfl_xor((int)(uint32_t)best, x, 64);
          best = o > best ? o : best;
        }
        if ((tid & 15) == 0 && gr < M) atomicMax(e.argmax_keys + (long)(bn % MIT_ARGMAX_SLOTS) * M + gr, (unsigned long long)best);
      }
      return;
    }
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) {
      const int r = (pass * NT + tid) >> 4, c8 = (tid & 15) * 8;
      const long gr = m0 + r;
      if (gr >= M || gc >= N) continue;
      const f32x4 lo = *(const f32x4*)(cs + r * CST + c8), hi = *(const f32x4*)(cs + r * CST + c8 + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      epi8x<ACT, DROP>(e, C, ldc, N, gr, gc, v, b, xs[pass], key);
    }
    return;
  }
#pragma unroll 2
  for (int pass = 0; pass < (BM * BN / 8) / NT; ++pass) {
    const int id = pass * NT + tid;
    const int r = id >> 4, c8 = (id & 15) * 8;
    const long gr = m0 + r, gc = n0 + c8;
    if (gr >= M || gc >= N) continue;
    const f32x4 lo = *(const f32x4*)(cs + r * CST + c8), hi = *(const f32x4*)(cs + r * CST + c8 + 4);
    if (ksplit > 1) {  // raw fp32 partial slab; gemm_splitk_reduce applies the epilogue (no activation)
      f32x4* o = (f32x4*)(ws + ((long)split * M + gr) * N + gc);
      o[0] = lo;
      o[1] = hi;
      continue;
    }
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    epi_row8<ACT, DROP>(e, C, ldc, N, gr, gc, v);
  }
}

template <int ALAY, int BLAY, int ACT, bool DROP>
__global__ __launch_bounds__(512) void gemm_bf16_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                        long M, long N, long K, long lda, long ldb, long ldc,
                                                        int a_bytes, int b_bytes, Epi e, int ksplit, long kchunk,
                                                        float* __restrict__ ws, float* __restrict__ rowsum) {
  gemm_bf16_body<ALAY, BLAY, ACT, DROP, 2, 8>(A, B, C, M, N, K, lda, ldb, ldc, a_bytes, b_bytes, e, ksplit, kchunk, ws,
                                             rowsum, blockIdx.x);
}

// Grouped weight-gradient GEMMs (dW = dY^T X, both operands MN-contig, f32 out, fused bias-gradient
// row sums, optional split-K into fp32 slabs): one launch runs every problem's blocks (problem i owns
// blocks [start_i, start_{i+1})), so a decoder layer's six small dW GEMMs (16-64 tiles each) fill the
// chip together instead of one after another.
constexpr int MAXG = 8;
struct GroupProb {
  const bf16* A;
  const bf16* B;
  void* C;
  long M, N, K, lda, ldb, ldc;
  int a_bytes, b_bytes, ksplit, start, rblocks, rstart;
  long kchunk;
  float* ws;
  float* rowsum;
  Epi e;
};
// LayerNorm dgamma/dbeta column reductions riding in the same grid (the partials mit_layernorm_bwd
// left in ws: nblk rows of [dgamma | dbeta]); 32 columns per block
constexpr int MAXLN = 4;
struct GroupLn {
  const float* ws;
  float* dgamma;
  float* dbeta;
  long nblk, cols;
  int start;
};
// XCD pieces of a grouped launch: block b runs on XCD b % 8 (round-robin dispatch), as its (b / 8)-th
// block there. The host deals each problem's tiles (in the order of gemm_bf16_body's GROUP = 0 branch)
// to the XCDs in contiguous runs of at most ceil(tiles / 8), so one XCD's L2 holds few problems and
// compact tile blocks of them (their dY / X panels read once per XCD, not once per XCD per problem).
constexpr int MAXP = MAXG + 8;
struct GroupPiece {
  int prob, t0, count;
};
struct GroupArgs {
  GroupProb p[MAXG];
  GroupLn ln[MAXLN];
  GroupPiece pc[MAXP];
  int xfirst[9];  // pieces of XCD x: [xfirst[x], xfirst[x + 1])
  int n, nln, gemm_blocks;
};

__device__ __forceinline__ void ln_grads_block(const GroupLn& j, int blk) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  float(*part)[33] = (float(*)[33])smem;
  const int cl = threadIdx.x & 31, grp = threadIdx.x >> 5;  // 16 row groups x 32 columns
  const long c = (long)blk * 32 + cl, w2 = 2 * j.cols;
  float s = 0.f;
  if (c < w2) {
    long b = grp;
    for (; b + 48 < j.nblk; b += 64)
      s += (j.ws[b * w2 + c] + j.ws[(b + 16) * w2 + c]) + (j.ws[(b + 32) * w2 + c] + j.ws[(b + 48) * w2 + c]);
    for (; b < j.nblk; b += 16) s += j.ws[b * w2 + c];
  }
  part[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < w2) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += part[g][cl];
    if (c < j.cols) j.dgamma[c] = t;
    else j.dbeta[c - j.cols] = t;
  }
}

__global__ __launch_bounds__(512) void gemm_bf16_grouped(GroupArgs ga) {
  if ((int)blockIdx.x >= ga.gemm_blocks) {
    int j = 0;
    while (j + 1 < ga.nln && (int)blockIdx.x >= ga.ln[j + 1].start) ++j;
    ln_grads_block(ga.ln[j], (int)blockIdx.x - ga.ln[j].start);
    return;
  }
  const int x = (int)blockIdx.x & 7;
  int slot = (int)blockIdx.x >> 3, j = ga.xfirst[x];
  while (j < ga.xfirst[x + 1] && slot >= ga.pc[j].count) slot -= ga.pc[j++].count;
  if (j == ga.xfirst[x + 1]) return;  // this XCD's share is shorter than the longest
  const GroupProb& q = ga.p[ga.pc[j].prob];
  // weight gradients dW = dY^T X with K = B*T
  gemm_bf16_body<MIT_MN_CONTIG, MIT_MN_CONTIG, MIT_ACT_NONE, false, 2, 8>(
      q.A, q.B, q.C, q.M, q.N, q.K, q.lda, q.ldb, q.ldc, q.a_bytes, q.b_bytes, q.e, q.ksplit, q.kchunk, q.ws, q.rowsum,
      ga.pc[j].t0 + slot, 0);
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA kernel, 256x256 block tile (large GEMMs: the encoder's M = B*197 rows)
//
// 8 waves as 2 (M) x 4 (N); each wave owns a 128x64 output tile = 8x4 accumulators. LDS: two
// K-tile buffers (BK = 64), each cut into four 16 KiB "half-tiles" (A rows 0-127 / 128-255,
// B rows 0-127 / 128-255) whose images are exactly the 128-row tiles of the kernel above (same
// swizzles, same frag() reads, all four layouts); the epilogue reuses the space.
//
// Each K-tile is consumed in 4 phases (one 64x32 quadrant of the wave's tile x K=64 = 16 MFMAs):
//   q0: read A rows 0-63 + B cols 0-31    q1: read B cols 32-63
//   q2: read A rows 64-127                q3: no reads (A hi x B lo from registers)
// A phase = {fragment ds_reads, one half-tile LDS-DMA issue, [counted vmcnt]} barrier
//           {16 MFMAs} barrier.
// Wave group wr = 1 runs one barrier behind wr = 0 (ping-pong): on every SIMD one wave issues
// MFMAs while its partner reads fragments / issues DMA.
// Buffer hazards (phase numbers within the 2-K-tile iteration, tile t in buf0, t+1 in buf1):
//   DMA schedule   ph0 B1(t+1) ph1 A0(t+1) ph2 A1(t+1) ph3 B0(t+2) ph4 B1(t+2) ph5 A0(t+2) ph6 A1(t+2)
//                  ph7 B0(t+3)
//   WAR: a half is refilled >= 2 phases after its last ds_read (buf0 B read ph0-1 -> refilled ph3-4,
//        A read ph0,ph2 -> ph5-6; buf1 B ph4-5 -> ph7,ph0'; A ph4,ph6 -> ph1',ph2'), which with the
//        one-barrier stagger still orders the partner group's reads before the DMA.
//   RAW: ph3 waits vmcnt(2) (every half of t+1 landed, ph3's own DMA in flight) and ph7 vmcnt(2)
//        (t+2); vmcnt(0) where that younger DMA was not issued. The first read is one phase later,
//        behind both groups' barriers.
// ------------------------------------------------------------------------------------------------
constexpr int B2 = 256;
constexpr int HALF_BYTES = 128 * 64 * 2;  // one 128-row x BK half-tile
constexpr int BUF_BYTES = 4 * HALF_BYTES;
constexpr int EPI_LD = 68;                // per-wave fp32 epilogue stage [64][68]
constexpr int SMEM2_BYTES = (2 * BUF_BYTES > 8 * 64 * EPI_LD * 4) ? 2 * BUF_BYTES : 8 * 64 * EPI_LD * 4;
constexpr int LN_PMAX = 16;                                 // LN fold: statistics partials per row (K <= 1024)
constexpr int SMEM2_EPI_BYTES = SMEM2_BYTES + 4096;  // staged epilogues: + the tile's per-row (rstd, -rstd mean),
                                                     // per-column bias and LN-fold column sums

// Per-lane LDS-DMA source plan for one operand (8 waves x 2 wave-instructions per half-tile):
// byte offsets of this lane's two 16-B chunks in each half at K-tile 0 (OOB when the row / column
// is out of range), the chunk's k inside the tile, and the per-K-tile byte step. Precomputed once
// so the main loop issues each DMA with one compare and one add.
template <int LAY, int HR = 128>
struct DmaPlan {
  uint32_t base[2][2];
  int kc[2];
  uint32_t step;
  __device__ __forceinline__ void init(long ld, long rows_total, long row0, long kb, int w, int lane) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int id = (w * 2 + j) * 64 + lane;
      if (LAY == MIT_K_CONTIG) {
        const int r = id >> 3, c = (id & 7) ^ ((r >> 1) & 7);
        kc[j] = c * 8;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // a half holds HR rows (rows HR..127 of its image load 0)
          const long row = row0 + h * HR + r;
          base[h][j] = (r < HR && row < rows_total) ? (uint32_t)((row * ld + kb + c * 8) * 2) : OOB;
        }
      } else {
        const int kr = id >> 4, c = (id & 15) ^ (mn_swz(kr) >> 4);
        kc[j] = kr;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const long col = row0 + h * 128 + c * 8;
          base[h][j] = col < rows_total ? (uint32_t)(((kb + kr) * ld + col) * 2) : OOB;
        }
      }
    }
    step = LAY == MIT_K_CONTIG ? (uint32_t)(BK * 2) : (uint32_t)(BK * ld * 2);
  }
  // dst = this wave's 2 KiB slice of the half-tile; t = K-tile index
  __device__ __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, char* dst, int h, int t, int klen) const {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t boff = (t * BK + kc[j] < klen) ? base[h][j] + (uint32_t)t * step : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(dst + j * 1024), 16,
                                               boff, 0, 0, 0);
    }
  }
};

// tile order of the 256 kernel: XCD remap + groups of 4 row tiles walking the column tiles (row-group
// heights 2 / 8 / 16 and no remap measured within +-1 %, profiles/r01_gemm256_tile_order_ab.txt)
constexpr int G256_GROUP = 4;

// Gathered register epilogue of one wave's (16 MI) x 64 output block, accumulated as C^T blocks
// (MFMA operands swapped: lane holds row (lane & 15), columns 4 * (lane >> 4) + t of block j); rows
// from mw, columns from nw. v_permlane16_swap of column blocks (2jp, 2jp+1) leaves lane group g
// with 8 consecutive columns of row (lane & 15): block 2jp + (g & 1), columns 8 * (g >> 1) .. +8.
// Stored as they are, each instruction would write 16 rows x 64 B (half cache lines): ~3.5x slower
// per CU than whole lines (tools/store_bench.hip: 8000 vs 2250 cycles per wave for a tile's 16
// stores), the largest fixed cost of a K = 768 tile. So a DPP row_ror:8 exchange swaps the jp = 1
// segments of rows 0-7 with the jp = 0 segments of rows 8-15 (lanes l <-> l ^ 8): every store
// (and residual / aux load) then covers 8 whole rows x 128 B. Same values, same arithmetic.
template <int ACT, bool DROP, int MI>
__device__ __forceinline__ void reg_epilogue(const f32x4 (&acc)[MI][4], const Epi& e, void* C, long ldc, long M, long N,
                                             long mw, long nw, int lane) {
  const int g = lane >> 4;
  const bool hi = (lane & 8) != 0;
  const long rl = mw + (lane & 7);  // row of store A of row block i: rl + 16 i; store B: + 8
  const long cl = nw + (g & 1) * 16 + (g >> 1) * 8 + (hi ? 32 : 0);
  float bb[8];
  epi_bias8(e, cl, N, bb);
  // residual / aux operands exist only with ACT == NONE on these kernels (mit_gemm routes an
  // activation plus a residual / aux to the 128 kernel): the activation instances keep no operand registers
  constexpr bool XOPS = ACT == MIT_ACT_NONE;
  bf16x8 xs[XOPS ? MI : 1][2];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if constexpr (XOPS) xs[i][h] = epi_x8(e, M, N, rl + i * 16 + h * 8, cl);
  // every operand load has landed before the first store: the loads sit in exec-masked branches
  // (bounds, optional operands), after which the compiler cannot count them and waits vmcnt(0) before
  // each later use -- i.e. behind every store issued so far (vmcnt counts stores): one store round
  // trip per row block. An explicit wait here clears its scoreboard.
  gather_wait();
  const uint64_t key = epi_key<DROP>(e);
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const bf16x8 x0 = XOPS ? xs[XOPS ? i : 0][0] : bf16x8{}, x1 = XOPS ? xs[XOPS ? i : 0][1] : bf16x8{};
    float v[2][8];
#pragma unroll
    for (int jp = 0; jp < 2; ++jp)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][t]),
                                                         __float_as_uint(acc[i][2 * jp + 1][t]), false, false);
        v[jp][t] = __uint_as_float(sw[0]);
        v[jp][4 + t] = __uint_as_float(sw[1]);
      }
    float va[8], vb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float snd = hi ? v[0][k] : v[1][k];
      const float rcv = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(snd), 0x128, 0xF, 0xF, false));
      va[k] = hi ? rcv : v[0][k];
      vb[k] = hi ? v[1][k] : rcv;
    }
    const long ra = rl + i * 16;
    if (cl < N) {
      if (ra < M) epi8x<ACT, DROP>(e, C, ldc, N, ra, cl, va, bb, x0, key);
      if (ra + 8 < M) epi8x<ACT, DROP>(e, C, ldc, N, ra + 8, cl, vb, bb, x1, key);
    }
  }
}

// LDS-staged bf16 epilogue of one wave's 128 x 64 block (C^T accumulators as above), through the
// wave's PRIVATE 16 KiB of LDS (no barrier): the fused epilogue (alpha, bias, activation, aux mask,
// dropout, residual) runs in f32 in the accumulator layout -- lane = row 16 i + (lane & 15), columns
// 16 j + 4 g + t, g = lane >> 4 -- rounds once to bf16, writes 4 bf16 per (i, j) with ds_write_b64, and
// reads whole 8-column chunks back for stores of 8 rows x 128 B. A residual / aux block is loaded in
// that same whole-line pattern before any store, written to the image, and read back per (i, j) segment
// just before the output segment overwrites it (the LDS does the transpose). Replaces reg_epilogue's
// permlane16_swap / DPP exchange and its selects (~40 VALU per 16-row block per wave): the epilogue of
// a K = 768 tile is VALU-bound. Measured (tools/g256_stamps.py, 8 tiles): plain 4.1 -> 2.4 us, residual
// 5.9 -> 4.8 us; enc qkv+bias 51.1 -> 48.8 us, fc1 73.8 -> 68.8, kv_all 102 -> 94.7; residual loads as
// 8-B segments in the accumulator layout instead: slower (o+res 28.6 -> 31.9 us). Image: row r at
// r * 128 B, 16-B chunk c at (c ^ (r & 7)) * 16 (the 8-row x 8-chunk read-back is conflict-free).
__device__ __forceinline__ float sum_rows(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// LNX: 0 = plain; 1 = LayerNorm-folded operand (v = rstd (acc - mean colsum) + bias, with the wave's rows'
// (rstd, -rstd mean) from lnrow: merged once per tile row in the kernel's prologue, ln_rows); 2 = also
// write the per-64-column (mean, M2) of the bf16-rounded output rows to e.stats_out (the next LayerNorm's
// statistics: this wave's 64 columns are one partial)
// lcol: the wave's 64 columns' bias (lcol[0, 64)) and, LNX 1, folded-weight column sums (lcol[256, 320)),
// staged in LDS by the kernel's prologue (zero past N)
template <int ACT, bool DROP, bool XOPS, int LNX = 0>
__device__ __forceinline__ void stage_epilogue(const f32x4 (&acc)[8][4], const Epi& e, void* C, long ldc, long M,
                                               long N, long mw, long nw, int lane, char* stg, const float* lcol,
                                               const f32x2* lnrow = nullptr) {
  constexpr int PASSES = 1, IP = 8;  // one pass over the wave's 8 16-row blocks
  const int g = lane >> 4, r16 = lane & 15;
  float bj[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const f32x4 b = *(const f32x4*)(lcol + 16 * j + 4 * g);
    bj[j][0] = b[0]; bj[j][1] = b[1]; bj[j][2] = b[2]; bj[j][3] = b[3];
  }
  float sj[LNX == 1 ? 4 : 1][4];  // LN fold: the column sums of the folded weight rows
  if constexpr (LNX == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 b = *(const f32x4*)(lcol + 256 + 16 * j + 4 * g);
      sj[j][0] = b[0]; sj[j][1] = b[1]; sj[j][2] = b[2]; sj[j][3] = b[3];
    }
  }
  typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
  const long cw = nw + 8 * (lane & 7);
  // the residual / aux block arrives in whole-line loads (8 rows x 128 B per instruction, the store
  // pattern) and is transposed to the accumulator layout through the same LDS image: each (i, j)
  // segment is read back (ds_read_b64) right before the output segment overwrites it
  u32x4 xl[XOPS ? 16 : 1];
  if constexpr (XOPS) {
    const bf16* src = (const bf16*)(e.res ? e.res : e.aux);
    const long ldx = e.res ? e.ldr : e.ld_aux;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const long row = mw + 8 * q + (lane >> 3);
      xl[q] = (row < M && cw < N) ? *(const u32x4*)(src + row * ldx + cw) : u32x4{0u, 0u, 0u, 0u};
    }
  }
  gather_wait();
  const uint64_t key = epi_key<DROP>(e);
  float rs_i[LNX == 1 ? 8 : 1], nr_i[LNX == 1 ? 8 : 1];  // rstd, -rstd * mean of the lane's 8 rows
  if constexpr (LNX == 1) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x2 v = lnrow[16 * i + r16];
      rs_i[i] = v[0];
      nr_i[i] = v[1];
    }
  }
#pragma unroll
  for (int ps = 0; ps < PASSES; ++ps) {
    if constexpr (XOPS) {
#pragma unroll
      for (int q = 0; q < 16 / PASSES; ++q) {
        const int rr = 8 * q + (lane >> 3);
        *(u32x4*)(stg + rr * 128 + (((lane & 7) ^ (rr & 7)) << 4)) = xl[ps * (16 / PASSES) + q];
      }
    }
#pragma unroll
    for (int ii = 0; ii < IP; ++ii) {
      const int i = ps * IP + ii;
      const int rr = 16 * ii + r16;  // row in the image
      const long row = mw + 16 * i + r16;
      float st_s = 0.f;
      float vr[LNX == 2 ? 4 : 1][4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
        if constexpr (LNX == 1) {  // in pairs (v_pk_fma_f32: the same fused ops as two v_fma_f32)
#pragma unroll
          for (int t = 0; t < 4; t += 2) {
            const f32x2 c = __builtin_elementwise_fma(f32x2{nr_i[i], nr_i[i]}, f32x2{sj[j][t], sj[j][t + 1]},
                                                      f32x2{bj[j][t], bj[j][t + 1]});
            const f32x2 r = __builtin_elementwise_fma(f32x2{acc[i][j][t], acc[i][j][t + 1]}, f32x2{rs_i[i], rs_i[i]}, c);
            v[t] = r[0];
            v[t + 1] = r[1];
          }
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = acc[i][j][t] * e.alpha + bj[j][t];
        }
        if (ACT == MIT_ACT_GELU) {
#pragma unroll
          for (int t = 0; t < 4; t += 2) {
            const f32x2 q = gelu_fast2(f32x2{v[t], v[t + 1]});
            v[t] = q[0];
            v[t + 1] = q[1];
          }
        } else if (ACT == MIT_ACT_QUICK_GELU) {
          quick_gelu_fast_n<4>(v);
        } else if (ACT != MIT_ACT_NONE) {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = act_apply<ACT, true>(e.act, v[t]);
        }
        const int ch = 2 * j + (g >> 1);
        char* seg = stg + rr * 128 + ((ch ^ (rr & 7)) << 4) + (g & 1) * 8;
        if constexpr (XOPS) {
          // LNX 2 (mit_gemm checked it): a residual, no aux operand, no dropout -- no run-time selects
          const u32x2 x = *(const u32x2*)seg;
          const float x0 = __uint_as_float(x[0] << 16), x1 = __uint_as_float(x[0] & 0xFFFF0000u);
          const float x2 = __uint_as_float(x[1] << 16), x3 = __uint_as_float(x[1] & 0xFFFF0000u);
          if (LNX != 2 && e.aux) {
            v[0] *= x0 > 0.f ? e.aux_scale : 0.f;
            v[1] *= x1 > 0.f ? e.aux_scale : 0.f;
            v[2] *= x2 > 0.f ? e.aux_scale : 0.f;
            v[3] *= x3 > 0.f ? e.aux_scale : 0.f;
          }
          if (DROP && e.dropout) {
            const uint64_t base = (uint64_t)row * (uint64_t)N + (uint64_t)(nw + 16 * j + 4 * g);
#pragma unroll
            for (int t = 0; t < 4; ++t) v[t] *= drop_mul(key, base + t, e.thresh, e.dscale);
          }
          if (LNX == 2 || e.res) {
            v[0] += x0;
            v[1] += x1;
            v[2] += x2;
            v[3] += x3;
          }
        } else if (DROP && e.dropout) {
          const uint64_t base = (uint64_t)row * (uint64_t)N + (uint64_t)(nw + 16 * j + 4 * g);
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] *= drop_mul(key, base + t, e.thresh, e.dscale);
        }
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        const bf16x4 o = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        *(bf16x4*)seg = o;
        if constexpr (LNX == 2) {  // the rounded values from the packed words (one shift / mask each)
          const u32x2 w = __builtin_bit_cast(u32x2, o);
          vr[j][0] = __uint_as_float(w[0] << 16);
          vr[j][1] = __uint_as_float(w[0] & 0xFFFF0000u);
          vr[j][2] = __uint_as_float(w[1] << 16);
          vr[j][3] = __uint_as_float(w[1] & 0xFFFF0000u);
#pragma unroll
          for (int t = 0; t < 4; ++t) st_s += vr[j][t];
        }
      }
      if constexpr (LNX == 2) {  // (mean, M2) of the row's 64 columns nw .. nw + 63 (two passes)
        const float mean = sum_rows(st_s) * (1.f / 64.f);
        float q = 0.f;
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) q += (vr[j][t] - mean) * (vr[j][t] - mean);
        q = sum_rows(q);
        if (g == 0 && row < M && nw < N) *(f32x2*)(e.stats_out + (row * (N >> 6) + (nw >> 6)) * 2) = f32x2{mean, q};
      }
    }
#pragma unroll
    for (int q = 0; q < 16 / PASSES; ++q) {
      const int rr = 8 * q + (lane >> 3);
      const u32x4 o = *(const u32x4*)(stg + rr * 128 + (((lane & 7) ^ (rr & 7)) << 4));
      const long row = mw + 64 * ps + rr;
      if (row < M && cw < N) *(u32x4*)((bf16*)C + row * ldc + cw) = o;
    }
  }
}

// STG (bf16 out, gathered epilogue, K-contig A): 1 = the LDS-staged epilogue without operands, 2 = with
// the residual / aux block, 3 = LayerNorm-folded A (no operand), 4 = residual + the output rows'
// per-64-column statistics; 0 = the register (f32 out) or LDS-stage (MN-contig A) epilogue. A template
// flag, not a run-time branch: two epilogues in one instance spill in the K loop.
template <int ALAY, int BLAY, int ACT, bool DROP, int STG = 0>
__global__ __launch_bounds__(512) void gemm256_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                      long M, long N, long K, long lda, long ldb, long ldc, int a_bytes,
                                                      int b_bytes, Epi e, float* __restrict__ ws,
                                                      float* __restrict__ rowsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  (void)ws;
  constexpr int MI = 8, HR = 128, BMT = 256, IH0 = 4;  // 16-row blocks per wave, rows per wave group / tile

  const int nbn = (int)((N + B2 - 1) / B2), nbm = (int)((M + BMT - 1) / BMT);
  const int ntiles = nbn * nbm;
  const int bid = xcd_remap(blockIdx.x, ntiles);
  const long kb = 0, ke = K;
  const int GROUP = G256_GROUP;
  const int group_id = bid / (GROUP * nbn);
  const int first_m = group_id * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  const int bm = first_m + (bid % (GROUP * nbn)) % gsize;
  const int bn = (bid % (GROUP * nbn)) / gsize;
  const long m0 = (long)bm * BMT, n0 = (long)bn * B2;
  MIT_DASSERT((int)blockIdx.x < ntiles && bm < nbm && bn < nbn && m0 < M && n0 < N);
  MIT_DASSERT(lda >= (ALAY == MIT_K_CONTIG ? K : M) && ldb >= (BLAY == MIT_K_CONTIG ? K : N) && ldc >= N);

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool TN = ALAY == MIT_MN_CONTIG && BLAY == MIT_MN_CONTIG;
  const bool do_rs = TN && rowsum != nullptr && bn == 0 && wc == 0;
  // REG: accumulate C^T blocks (MFMA operands swapped: a lane holds 4 consecutive columns of one
  // row) so the epilogue can run from registers (no LDS stage, no barrier); used when the epilogue
  // is gatherable, else the C^T blocks are staged through LDS transposed
  constexpr bool REG = ALAY == MIT_K_CONTIG;
  const bool regepi = REG && epi_gatherable(e);
  const bool stage = STG && regepi;  // LDS-staged bf16 epilogue (stage_epilogue)
  float rs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((ke - kb + BK - 1) / BK);
  DmaPlan<ALAY, HR> pa;
  DmaPlan<BLAY> pb;
  pa.init(lda, M, m0, kb, wid, lane);
  pb.init(ldb, N, n0, kb, wid, lane);
  const int klen = (int)(ke - kb);
  // half-tile LDS-DMA: operand X (0 = A, 1 = B), half h, K-tile t -> buffer t & 1; false if t >= nk
  auto issue = [&](int X, int h, int t) -> bool {
    if (t >= nk) return false;
    char* dst = smem + (t & 1) * BUF_BYTES + (X * 2 + h) * HALF_BYTES + wid * 2048;
    if (X == 0) pa.issue(ra, dst, h, t, klen);
    else pb.issue(rb, dst, h, t, klen);
    return true;
  };
  auto wait_dma = [&](bool younger_issued) {
    if (younger_issued) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  bf16x8 af[IH0][2], blo[2][2], bhi[2][2];
  auto read_a = [&](int buf, int ih) {  // A row blocks [ih*IH0, ...) of this wave's MI (64 rows each half at MI = 8)
    const char* base = smem + buf * BUF_BYTES + wr * HALF_BYTES;
    const int ni = ih ? MI - IH0 : IH0;
#pragma unroll
    for (int i = 0; i < IH0; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        if (i < ni) af[i][kk] = frag<ALAY>(base, (ih * IH0 + i) * 16, kk, lane);
    if (TN && do_rs) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) rs[ih * 4 + i] = frag_rowsum(af[i][kk], rs[ih * 4 + i]);
    }
  };
  auto read_b = [&](int buf, int jh, bf16x8 (&bf)[2][2]) {  // B cols jh*32 .. +32 of this wave's 64
    const char* base = smem + buf * BUF_BYTES + (2 + (wc >> 1)) * HALF_BYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = frag<BLAY>(base, (wc & 1) * 64 + jh * 32 + j * 16, kk, lane);
  };
  auto mma = [&](int ih, int jh, bf16x8 (&bf)[2][2]) {
    const int ni = ih ? MI - IH0 : IH0;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < IH0; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          if (i < ni)
            acc[ih * IH0 + i][jh * 2 + j] =
                REG ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af[i][kk], acc[ih * IH0 + i][jh * 2 + j], 0, 0, 0)
                    : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i][kk], bf[j][kk], acc[ih * IH0 + i][jh * 2 + j], 0, 0, 0);
  };

  // LN fold (STG 3): each of the tile's 256 rows' K / 64 statistics partials merged ONCE here (thread r
  // takes row m0 + r, Chan's rule in column order) into (rstd, -rstd mean) in LDS past the K-tile buffers,
  // read by the epilogue's 8 rows per lane. The partial loads go out before the first LDS-DMA, so the
  // K loop's counted vmcnt waits (younger DMAs only) stay exact, and the merge after the prologue's DMA
  // issue waits for them alone; their round trip overlaps the first K-tile's.
  f32x2* ln_rows = (f32x2*)(smem + SMEM2_BYTES);
  // staged epilogues: the tile's 256 bias values (and LN-fold column sums) loaded here too, into LDS
  float* lcol = (float*)(smem + SMEM2_BYTES + 2048);
  float pbias = 0.f, pcols = 0.f;
  if constexpr (STG != 0) {
    const long c = n0 + tid;
    if (tid < B2 && c < N) {
      if (e.bias) pbias = e.bias[c];
      if constexpr (STG == 3) pcols = e.ln_colsum[c];
    }
  }
  f32x2 lnp[STG == 3 ? LN_PMAX : 1];
  if constexpr (STG == 3) {
    const long row = m0 + tid;
    const bool ok = tid < BMT && row < M;
#pragma unroll
    for (int p = 0; p < LN_PMAX; ++p)
      lnp[p] = (ok && p < e.ln_parts) ? *(const f32x2*)(e.ln_stats + (row * e.ln_parts + p) * 2) : f32x2{0.f, 0.f};
  }
  // prologue: K-tile 0 (all four halves) and B0 of K-tile 1
  issue(0, 0, 0);
  issue(0, 1, 0);
  issue(1, 0, 0);
  issue(1, 1, 0);
  const bool b01 = issue(1, 0, 1);
  if constexpr (STG == 3) {
    if (tid < BMT) {  // Chan, partial p (64 columns) onto the first 64 p: weights 1 / (p + 1) are constants
      float mu = 0.f, q = 0.f;
#pragma unroll
      for (int p = 0; p < LN_PMAX; ++p)
        if (p < e.ln_parts) {
          const float d = lnp[p][0] - mu, f = 1.0f / (float)(p + 1);
          mu = fmaf(d, f, mu);
          q += lnp[p][1] + d * d * (64.0f * (float)p * f);
        }
      const float rs = __builtin_amdgcn_rsqf(q / (64.0f * (float)e.ln_parts) + e.ln_eps);
      ln_rows[tid] = f32x2{rs, -rs * mu};
    }
  }
  if constexpr (STG != 0) {
    if (tid < B2) {
      lcol[tid] = pbias;
      if constexpr (STG == 3) lcol[256 + tid] = pcols;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible to every wave past the next barrier
  }
  wait_dma(b01);
  bar_raw();
  if (wr == 1) bar_raw();  // stagger: group 1 runs one barrier behind group 0

  // 4 barriers per K-tile (two quarter-tile MFMA blocks per phase: a 512-cycle MFMA segment per group
  // hides more of the other group's LDS-read latency), every next-tile half-tile DMA issued in the
  // first phase, one full MFMA block before its counted wait (+3-5 % on every 256-tile shape over
  // the 8-phase loop, profiles/r01_gemm256_schedule_ab.txt)
  for (int t = 0; t < nk; t += 2) {
    const bool two = t + 1 < nk;
    read_a(0, 0);
    read_b(0, 0, blo);
    issue(1, 1, t + 1);
    read_b(0, 1, bhi);
    issue(0, 0, t + 1);
    issue(0, 1, t + 1);
    bar_raw();
    mma(0, 0, blo);
    mma(0, 1, bhi);
    bar_raw();

    read_a(0, 1);
    wait_dma(issue(1, 0, t + 2));
    bar_raw();
    mma(1, 1, bhi);
    mma(1, 0, blo);
    bar_raw();

    if (two) {
      read_a(1, 0);
      read_b(1, 0, blo);
    }
    issue(1, 1, t + 2);
    if (two) read_b(1, 1, bhi);
    issue(0, 0, t + 2);
    issue(0, 1, t + 2);
    bar_raw();
    if (two) {
      mma(0, 0, blo);
      mma(0, 1, bhi);
    }
    bar_raw();

    if (two) read_a(1, 1);
    wait_dma(issue(1, 0, t + 3));
    // staged epilogue: the lagging group writes its LDS stage into the last K-tile's buffer right after
    // its last MFMA block, so every wave's reads of that buffer must have RETURNED by this (for group 1:
    // its last) barrier, not only been issued
    if (stage && t + 2 >= nk) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar_raw();
    if (two) {
      mma(1, 1, bhi);
      mma(1, 0, blo);
    }
    // register epilogue: the lagging group skips the loop's last barrier (nothing after it reads
    // LDS), so the leading group's epilogue overlaps its last MFMA block and neither waits
    if (!(regepi && wr == 1 && t + 2 >= nk)) bar_raw();  // (never skipped by the LDS-staged epilogue)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (regepi) {
    if constexpr (STG) {
      if (stage) {
        // group 0 stages into the buffer NOT holding the last K-tile (its last reads were >= 2 phases
        // ago), group 1 into the last K-tile's buffer (every read of it returned by the last barrier)
        const int buf = wr == 0 ? (nk & 1) : ((nk - 1) & 1);
        char* stg = smem + buf * BUF_BYTES + wc * 16384;
        stage_epilogue<ACT, DROP, STG == 2 || STG == 4, STG == 3 ? 1 : (STG == 4 ? 2 : 0)>(
            acc, e, C, ldc, M, N, m0 + wr * HR, n0 + wc * 64, lane, stg, lcol + wc * 64, ln_rows + wr * HR);
        return;
      }
    }
    reg_epilogue<ACT, DROP, MI>(acc, e, C, ldc, M, N, m0 + wr * HR, n0 + wc * 64, lane);
    return;
  }
  if (wr == 0) bar_raw();  // re-align the groups
  bar_raw();

  if (do_rs) {
    float* dst = rowsum;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float v = rs[i];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      const long r = m0 + wr * 128 + i * 16 + (lane & 15);
      if (lane < 16 && r < M) dst[r] = v;
    }
  }

  // ---- epilogue: per wave, two passes of 64 rows x 64 cols through a private fp32 LDS stage ----
  float* cs = (float*)smem + wid * 64 * EPI_LD;
  const bool gather = epi_gatherable(e);
  const long gcw = n0 + wc * 64 + (lane & 7) * 8;  // this lane's columns in every pass / row
  float bw[8];
  uint64_t key = 0;
  if (gather) {
    epi_bias8(e, gcw, N, bw);
    key = epi_key<DROP>(e);
  }
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (REG)  // C^T block: lane holds row (lane & 15), columns 4 * (lane >> 4) + t
            cs[(i * 16 + (lane & 15)) * EPI_LD + j * 16 + (lane >> 4) * 4 + t] = acc[pass * 4 + i][j][t];
          else
            cs[(i * 16 + (lane >> 4) * 4 + t) * EPI_LD + j * 16 + (lane & 15)] = acc[pass * 4 + i][j][t];
    __builtin_amdgcn_wave_barrier();
    if (gather) {  // this pass's residual / aux segments first, then only stores
      bf16x8 xs[8];
#pragma unroll
      for (int it = 0; it < 8; ++it) xs[it] = epi_x8(e, M, N, m0 + wr * 128 + pass * 64 + it * 8 + (lane >> 3), gcw);
      gather_wait();
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        const int r = it * 8 + (lane >> 3), c8 = (lane & 7) * 8;
        const long gr = m0 + wr * 128 + pass * 64 + r;
        if (gr >= M || gcw >= N) continue;
        const f32x4 lo = *(const f32x4*)(cs + r * EPI_LD + c8), hi = *(const f32x4*)(cs + r * EPI_LD + c8 + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        epi8x<ACT, DROP>(e, C, ldc, N, gr, gcw, v, bw, xs[it], key);
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int id = it * 64 + lane;
      const int r = id >> 3, c8 = (id & 7) * 8;
      const long gr = m0 + wr * 128 + pass * 64 + r, gc = n0 + wc * 64 + c8;
      if (gr >= M || gc >= N) continue;
      const f32x4 lo = *(const f32x4*)(cs + r * EPI_LD + c8), hi = *(const f32x4*)(cs + r * EPI_LD + c8 + 4);
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      epi_row8<ACT, DROP>(e, C, ldc, N, gr, gc, v);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// ------------------------------------------------------------------------------------------------
// 256x256 tile with ONE wave per SIMD (opt-in: mit_gemm_set_variant(4); NT, bf16, K % 64 == 0, the STG 1 /
// 3 / 4 epilogues): 4 waves as 2 (M) x 2 (N), each owning a 128x128 output tile = 8 x 8 accumulator blocks
// (256 registers per lane, AGPRs, accumulated in place by inline-asm MFMAs). The K-tile's LDS image and DMA
// plan are gemm256_kernel's (each wave issues the pieces of two of its virtual waves; the K-tile step in
// soffset). Per K-tile two phases of 64 MFMAs, one barrier:
//   X(t): MFMAs of k-slice 0 of tile t  | ds_reads of k-slice 1 of tile t
//   [own DMA of tile t+1 landed, own reads returned] barrier
//   Y(t): DMA of tile t+2 into tile t's buffer, MFMAs of k-slice 1 | ds_reads of k-slice 0 of tile t+1
// Every output element sums the same MFMAs in the same K order as gemm256_kernel: bitwise equal
// (tests/test_gemm256_gpu.py). Measured (profiles/r06_gemm256w_ab.txt): 4096^3 1350-1358 vs 1305-1315 TFLOP/s,
// but 4-12 % slower on the encoder's shapes and the train step 2.3 % slower -- not the default.
// ------------------------------------------------------------------------------------------------
template <int ACT, int STG>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void gemm256w_kernel(
    const bf16* __restrict__ A, const bf16* __restrict__ B, void* C, long M, long N, long K, long lda, long ldb,
    long ldc, int a_bytes, int b_bytes, Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 1, wc = wid & 1;
  constexpr int BMT = 256;
  const int nbn = (int)((N + B2 - 1) / B2), nbm = (int)((M + BMT - 1) / BMT);
  const int ntiles = nbn * nbm;
  const int bid = xcd_remap(blockIdx.x, ntiles);
  const int GROUP = G256_GROUP;
  const int group_id = bid / (GROUP * nbn);
  const int first_m = group_id * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  const int bm = first_m + (bid % (GROUP * nbn)) % gsize;
  const int bn = (bid % (GROUP * nbn)) / gsize;
  const long m0 = (long)bm * BMT, n0 = (long)bn * B2;
  MIT_DASSERT((int)blockIdx.x < ntiles && m0 < M && n0 < N);

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)(K / BK);  // K % 64 == 0 (the dispatcher's condition)
  // LDS-DMA sources: piece p = (operand X, half h, virtual wave vw = wid + 4 v, instruction j) of a K-tile;
  // the voffset (row / k-chunk, OOB past the operand) is fixed, the K-tile's byte step goes in soffset
  // (scalar), the LDS destination is wave-uniform (M0): scalar ops only per piece in the loop
  uint32_t voff[2][2][2][2];  // [X][h][v][j]
#pragma unroll
  for (int X = 0; X < 2; ++X)
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int id = ((wid + 4 * v) * 2 + j) * 64 + lane;
        const int r = id >> 3, c = (id & 7) ^ ((r >> 1) & 7);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const long row = (X ? n0 : m0) + h * 128 + r;
          const long ld = X ? ldb : lda;
          voff[X][h][v][j] = row < (X ? N : M) ? (uint32_t)((row * ld + c * 8) * 2) : OOB;
        }
      }
  // a tile t >= nk loads nothing (soffset past any num_records: the pieces read as zeros into a buffer no
  // one reads again; the epilogue waits vmcnt(0) before reusing it), so every K-tile runs the same code
  auto issue_piece = [&](int t, int p) {  // p = ((X * 2 + h) * 2 + v) * 2 + j
    const int X = p >> 3, h = (p >> 2) & 1, v = (p >> 1) & 1, j = p & 1;
    char* dst = smem + (t & 1) * BUF_BYTES + (X * 2 + h) * HALF_BYTES + (wid + 4 * v) * 2048 + j * 1024;
    const int soff = t < nk ? t * BK * 2 : (int)OOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(X ? rb : ra, (__attribute__((address_space(3))) void*)dst, 16,
                                             voff[X][h][v][j], soff, 0, 0);
  };
  auto issue_tile = [&](int t) {
#pragma unroll
    for (int p = 0; p < 16; ++p) issue_piece(t, p);
  };
  bf16x8 fa[2][8], fb[2][8];
  auto read_frag = [&](int t, int kk, int q) {  // q < 8: A row block q, else B column block q - 8
    const char* buf = smem + (t & 1) * BUF_BYTES;
    if (q < 8) fa[kk][q] = frag<MIT_K_CONTIG>(buf + wr * HALF_BYTES, q * 16, kk, lane);
    else fb[kk][q - 8] = frag<MIT_K_CONTIG>(buf + (2 + wc) * HALF_BYTES, (q - 8) * 16, kk, lane);
  };
  // in-place accumulation (dst = srcC, "+a": the accumulators stay put in the AGPRs; with the builtin the
  // register allocator re-homed some of the 64 blocks every K-tile, ~130 v_accvgpr copies per iteration)
  auto mma4 = [&](int kk, int n) {  // MFMAs 4n .. 4n+3 of the k-slice (row block n / 2, four column blocks)
    const int i = n >> 1;
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) {
      const int j = (n & 1) * 4 + jj;
      asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fb[kk][j]), "v"(fa[kk][i]));
    }
  };
  // One fragment read and one DMA piece per group of four MFMAs. Measured on 4096^3 (tools/gemm_bench.py,
  // profiles/r06_gemm256w_ab.txt): the DMA pieces cost ~14 % (issued among this wave's own MFMAs: no partner
  // wave's MFMAs cover their issue), the fragment reads ~8 %, the barrier ~2.5 %; splitting the pieces over
  // both phases (half a phase to land) measured the same.
  // X(t): k-slice 0's 64 MFMAs | k-slice 1's reads of tile t
  auto phase_x = [&](int t) {
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      read_frag(t, 1, n);
      mma4(0, n);
    }
  };
  // Y(t): k-slice 1's 64 MFMAs | the DMA of tile t+2, k-slice 0's reads of tile t+1 (past the last tile:
  // stale contents into registers no MFMA uses)
  auto phase_y = [&](int t) {
#pragma unroll
    for (int n = 0; n < 16; ++n) {
      issue_piece(t + 2, n);
      read_frag(t + 1, 0, n);
      mma4(1, n);
    }
  };

  // prologue: bias / LN-fold operands staged as gemm256_kernel does, K-tiles 0 and 1 in flight
  f32x2* ln_rows = (f32x2*)(smem + SMEM2_BYTES);
  float* lcol = (float*)(smem + SMEM2_BYTES + 2048);
  float pbias = 0.f, pcols = 0.f;
  {
    const long c = n0 + tid;
    if (c < N) {
      if (e.bias) pbias = e.bias[c];
      if constexpr (STG == 3) pcols = e.ln_colsum[c];
    }
  }
  f32x2 lnp[STG == 3 ? LN_PMAX : 1];
  if constexpr (STG == 3) {
    const long row = m0 + tid;
    const bool ok = row < M;
#pragma unroll
    for (int p = 0; p < LN_PMAX; ++p)
      lnp[p] = (ok && p < e.ln_parts) ? *(const f32x2*)(e.ln_stats + (row * e.ln_parts + p) * 2) : f32x2{0.f, 0.f};
  }
  issue_tile(0);
  issue_tile(1);
  if constexpr (STG == 3) {
    float mu = 0.f, q = 0.f;
#pragma unroll
    for (int p = 0; p < LN_PMAX; ++p)
      if (p < e.ln_parts) {
        const float d = lnp[p][0] - mu, f = 1.0f / (float)(p + 1);
        mu = fmaf(d, f, mu);
        q += lnp[p][1] + d * d * (64.0f * (float)p * f);
      }
    const float rs = __builtin_amdgcn_rsqf(q / (64.0f * (float)e.ln_parts) + e.ln_eps);
    ln_rows[tid] = f32x2{rs, -rs * mu};
  }
  lcol[tid] = pbias;
  if constexpr (STG == 3) lcol[256 + tid] = pcols;
  asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)" ::: "memory");
  bar_raw();
#pragma unroll
  for (int q = 0; q < 16; ++q) read_frag(0, 0, q);

  for (int t = 0; t < nk; ++t) {
    phase_x(t);
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // tile t+1 landed; k-slice 1 returned
    bar_raw();                                                  // ... on every wave: tile t's buffer is free
    phase_y(t);
  }
  // the last MFMAs' results reach the AGPRs before any VALU reads them (the hazard recognizer does not see
  // into the asm): 3 x 8 wait states past the 16x16x32 MFMA's 8 passes
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  bar_raw();  // every wave's last reads returned: the K-tile buffers become the epilogue stages

  char* stg = smem + wid * 16384;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    f32x4 a2[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) a2[i][j] = acc[i][h * 4 + j];
    stage_epilogue<ACT, false, STG == 4, STG == 3 ? 1 : (STG == 4 ? 2 : 0)>(
        a2, e, C, ldc, M, N, m0 + wr * 128, n0 + wc * 128 + h * 64, lane, stg, lcol + wc * 128 + h * 64, ln_rows + wr * 128);
  }
}

// ------------------------------------------------------------------------------------------------
// Register-streaming NT kernel for the decode step's B-row GEMMs (M = B <= 256, short K: the 128
// kernel runs 2 x N/128 blocks through a K loop bound by per-K-step DMA issue / barrier / fragment
// read latency). 64x64 output tile per 4-wave block; no operand staging: each wave loads
// its MFMA fragments straight from global memory into registers (16-B buffer loads, out-of-range
// rows / k read as 0), one K-step ahead of its MFMAs, and the four waves split K (wave w takes
// K-steps w, w+4, ...), so the K loop has no barrier at all. The four partial tiles meet once in
// LDS (fp32, padded rows: conflict-free), then every thread sums 16 outputs and runs the gathered
// epilogue. Both operands K-contig (NT).
// ------------------------------------------------------------------------------------------------
constexpr int RS_LD = 68;                                 // fp32 row stride of a partial tile in LDS
constexpr int RS_SMEM = 4 * 64 * RS_LD * 4;               // 4 partial 64x64 tiles (69632 B)

template <int ACT, bool DROP>
__global__ __launch_bounds__(256) void gemm_rs_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                      long M, long N, long K, long lda, long ldb, long ldc, int a_bytes,
                                                      int b_bytes, Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int nbn = (int)((N + 63) / 64), nbm = (int)((M + 63) / 64);
  const int bid = xcd_remap(blockIdx.x, nbm * nbn);  // an XCD's blocks: consecutive row blocks share A
  const int bm = bid / nbn, bn = bid % nbn;
  const long m0 = (long)bm * 64, n0 = (long)bn * 64;
  MIT_DASSERT((int)blockIdx.x < nbm * nbn && m0 < M && n0 < N && lda >= K && ldb >= K && ldc >= N);
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);

  // this lane's fragment rows (16-row block i: + 16 i) and k offset inside a 32-wide slice
  const long ar = m0 + (lane & 15), brow = n0 + (lane & 15);
  const int kl = 8 * (lane >> 4);
  auto ld8 = [&](__amdgpu_buffer_rsrc_t rs, long row, long rows, long ld, long k) -> bf16x8 {
    const uint32_t off = (row < rows && k < K) ? (uint32_t)((row * ld + k) * 2) : OOB;
    return __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
  };
  auto load = [&](int s, bf16x8 (&a)[4][2], bf16x8 (&b)[4][2]) {
    const long k0 = (long)s * BK + kl;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        a[i][kk] = ld8(ra, ar + i * 16, M, lda, k0 + kk * 32);
        b[i][kk] = ld8(rb, brow + i * 16, N, ldb, k0 + kk * 32);
      }
  };
  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](bf16x8 (&a)[4][2], bf16x8 (&b)[4][2]) {
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i][kk], b[j][kk], acc[i][j], 0, 0, 0);
  };

  const int ns = (int)((K + BK - 1) / BK);
  bf16x8 a0[4][2], b0[4][2], a1[4][2], b1[4][2];
  int s = w;
  if (s < ns) load(s, a0, b0);
  for (; s < ns; s += 8) {
    if (s + 4 < ns) load(s + 4, a1, b1);
    mma(a0, b0);
    if (s + 4 >= ns) break;
    if (s + 8 < ns) load(s + 8, a0, b0);
    mma(a1, b1);
  }

  // the four partial tiles -> LDS, then thread t sums row t/4, columns 16 (t%4) .. +16
  float* red = (float*)smem;
  {
    float* mine = red + w * 64 * RS_LD;
    const int g = lane >> 4;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int t = 0; t < 4; ++t) mine[(i * 16 + g * 4 + t) * RS_LD + j * 16 + (lane & 15)] = acc[i][j][t];
  }
  const int r = tid >> 2, cq = (tid & 3) * 16;
  const long gr = m0 + r;
  const bool gather = epi_gatherable(e);
  float bias0[8], bias1[8];
  bf16x8 x0 = {}, x1 = {};
  uint64_t key = 0;
  if (gather) {  // operand loads before the barrier (and before any store)
    epi_bias8(e, n0 + cq, N, bias0);
    epi_bias8(e, n0 + cq + 8, N, bias1);
    x0 = epi_x8(e, M, N, gr, n0 + cq);
    x1 = epi_x8(e, M, N, gr, n0 + cq + 8);
    key = epi_key<DROP>(e);
  }
  __syncthreads();
  float v[16];
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    f32x4 a = *(const f32x4*)(red + r * RS_LD + cq + c);
#pragma unroll
    for (int q = 1; q < 4; ++q) a += *(const f32x4*)(red + (q * 64 + r) * RS_LD + cq + c);
    v[c] = a[0];
    v[c + 1] = a[1];
    v[c + 2] = a[2];
    v[c + 3] = a[3];
  }
  if (gr >= M) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const long gc = n0 + cq + h * 8;
    if (gc >= N) continue;
    if (gather) epi8x<ACT, DROP>(e, C, ldc, N, gr, gc, v + h * 8, h ? bias1 : bias0, h ? x1 : x0, key);
    else epi_row8<ACT, DROP>(e, C, ldc, N, gr, gc, v + h * 8);
  }
}

// C = alpha * sum_s slab[s] (f32 or bf16 out, optional accumulate); rowsum = sum_s rowslab[s]
__global__ void gemm_splitk_reduce(long M, long N, int ksplit, const float* __restrict__ ws, void* C, long ldc,
                                   float alpha, int out_f32, int accumulate, float* rowsum) {
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
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

// the split-K combine of a grouped launch: problem i's slabs summed by blocks [rstart_i, +rblocks_i)
__global__ __launch_bounds__(256) void gemm_splitk_reduce_grouped(GroupArgs ga) {
  int i = 0;
  while (i + 1 < ga.n && (int)blockIdx.x >= ga.p[i + 1].rstart) ++i;
  const GroupProb& q = ga.p[i];
  const long M = q.M, N = q.N, n4 = N / 4, total = M * n4;
  const long b0 = (long)blockIdx.x - q.rstart, stride = (long)q.rblocks * blockDim.x;
  for (long t = b0 * blockDim.x + threadIdx.x; t < total; t += stride) {
    const long r = t / n4, c = (t % n4) * 4;
    f32x4 s = *(const f32x4*)(q.ws + r * N + c);
    for (int k = 1; k < q.ksplit; ++k) s += *(const f32x4*)(q.ws + ((long)k * M + r) * N + c);
    s *= q.e.alpha;
    f32x4* o = (f32x4*)((float*)q.C + r * q.ldc + c);
    if (q.e.accumulate) s += *o;
    *o = s;
  }
  if (q.rowsum) {
    const float* rw = q.ws + (long)q.ksplit * M * N;
    for (long r = b0 * blockDim.x + threadIdx.x; r < M; r += stride) {
      float s = 0.f;
      for (int k = 0; k < q.ksplit; ++k) s += rw[(long)k * M + r];
      q.rowsum[r] = s;
    }
  }
}

// split-K plan for a plain-epilogue bf16 GEMM: only when the output has too few 128x128 tiles to
// fill 256 CUs and K is long (the weight-gradient shapes). Returns 1 (no split) otherwise.
int splitk_plan(long M, long N, long K, long* kchunk, int a_layout = MIT_MN_CONTIG) {
  const long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  *kchunk = K;
  if (tiles >= 256 || K < 1024 || N % 8) return 1;
  // blocks the split aims for: 256 for the data gradients (dX fc_out, K = 10000 on 128 tiles: +0.4 % step
  // over 128) and the weight gradients (128 / 256 / 384 within +-0.3 % in the step)
  const long target = 256;
  (void)a_layout;
  long s = (target + tiles - 1) / tiles;
  s = min(s, K / 512);
  s = min(s, 16L);
  if (s < 2) return 1;
  long kc = (K + s - 1) / s;
  kc = (kc + BK - 1) / BK * BK;
  *kchunk = kc;
  return (int)((K + kc - 1) / kc);
}
long splitk_ws_bytes(long M, long N, int s) { return s > 1 ? 4096 + 4L * s * M * N + 4L * s * M : 0; }

// ------------------------------------------------------------------------------------------------
// fp32 kernel (parity mode) on the exact-f32 matrix cores: v_mfma_f32_32x32x2_f32 (f32 in, f32
// accumulate; each MFMA is a chain of correctly rounded f32 FMAs, MI355X_MICROARCH.md: 155 TF vs the
// VALU's 52 on a GEMM). 64x64x16 block tile, 4 waves (2 x 2) of 32x32, A / B staged k-major in LDS
// (both operand layouts, any edges: out-of-range elements stage as 0), 8 MFMAs per wave per K-tile.
// Same run-time epilogue (epi_store) and fused row sums as the bf16 kernels.
// MFMA 32x32x2 operand layout: lane l gives A(m = l & 31, k = l >> 5) and B(k = l >> 5, n = l & 31);
// accumulator j of lane l is C(8 (j >> 2) + 4 (l >> 5) + (j & 3), l & 31).
// ------------------------------------------------------------------------------------------------
typedef __attribute__((ext_vector_type(16))) float f32x16;
template <int ALAY, int BLAY>
__global__ __launch_bounds__(256) void gemm_f32_kernel(const float* __restrict__ A, const float* __restrict__ B, void* C,
                                                       long M, long N, long K, long lda, long ldb, long ldc, Epi e,
                                                       float* __restrict__ rowsum) {
  constexpr int FT = 64, FK = 16, FP = FT + 4;
  __shared__ float As[FK][FP];
  __shared__ float Bs[FK][FP];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const long m0 = (long)blockIdx.y * FT, n0 = (long)blockIdx.x * FT;
  MIT_DASSERT(m0 < M && n0 < N && ldc >= N);
  f32x16 acc = {};
  float rsum = 0.f;
  const bool do_rs = rowsum != nullptr && blockIdx.x == 0 && wn == 0;
  const int lm = lane & 31, lk = lane >> 5;
  for (long k0 = 0; k0 < K; k0 += FK) {
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
    for (int kk = 0; kk < FK; kk += 2) {
      const float a = As[kk + lk][wm * 32 + lm], b = Bs[kk + lk][wn * 32 + lm];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
      if (do_rs) rsum += a;
    }
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const long r = m0 + wm * 32 + 8 * (j >> 2) + 4 * lk + (j & 3), c = n0 + wn * 32 + lm;
    if (r < M && c < N) epi_store<float>(e, C, ldc, N, r, c, acc[j]);
  }
  if (do_rs) {  // lanes l and l + 32 hold the even / odd k of row l & 31
    rsum += __shfl_xor(rsum, 32, 64);
    const long r = m0 + wm * 32 + lm;
    if (lane < 32 && r < M) rowsum[r] = rsum;
  }
}

// ------------------------------------------------------------------------------------------------
// host side: kernel / epilogue-instance selection
// ------------------------------------------------------------------------------------------------

template <typename KernelT>
void set_lds(KernelT k, int bytes) {
  (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

// split-K decision for a bf16 GEMM on the 128x128 kernel. The workspace's first WS_HDR bytes hold
// the in-launch combine's per-tile counters; slabs follow.
constexpr long WS_HDR = 4096;
struct Split {
  int ks = 1;
  long kchunk = 0;
};

int g_num_cus = 0;
int num_cus() {
  if (!g_num_cus) {
    int dev = 0;
    hipDeviceProp_t p;
    g_num_cus = (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&p, dev) == hipSuccess) ? p.multiProcessorCount : 256;
  }
  return g_num_cus;
}

// 8 waves per 128x128 block (2 per SIMD, each issuing half the LDS-DMA pieces of a K-tile): with 4
// waves every K-tile's 8 DMA pieces per wave sat serially in front of its 32 MFMAs (+2.7 % step)
template <int AL, int BL, int ACT, bool DROP>
void launch_bf16(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, const Split& sp, hipStream_t s) {
  const int ksplit = sp.ks;
  const long kchunk = sp.ks > 1 ? sp.kchunk : g->K;
  float* ws = g->workspace ? (float*)((char*)g->workspace + WS_HDR) : nullptr;
  const long nbm = (g->M + BM - 1) / BM, nbn = (g->N + BN - 1) / BN;
  const long nblk = nbm * nbn * ksplit;
  static bool attr = false;
  if (!attr) {
    set_lds(gemm_bf16_kernel<AL, BL, ACT, DROP>, smem_bytes(2));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<AL, BL, ACT, DROP>), dim3((unsigned)nblk), dim3(512), smem_bytes(2), s,
                     (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                     b_bytes, e, ksplit, kchunk, ws, g->rowsum);
}

template <int ACT, bool DROP>
void launch_rs(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    set_lds(gemm_rs_kernel<ACT, DROP>, RS_SMEM);
    attr = true;
  }
  const long nb = ((g->M + 63) / 64) * ((g->N + 63) / 64);
  hipLaunchKernelGGL((gemm_rs_kernel<ACT, DROP>), dim3((unsigned)nb), dim3(256), RS_SMEM, s, (const bf16*)g->A,
                     (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e);
}

// 0 = pick per shape, 1 = always the 128x128 kernel, 2 = the 256x256 kernel wherever it has an
// instance for the epilogue, 3 = the register-streaming kernel where it applies (tests / tools)
#ifndef MIT_GEMM_DEFAULT_VARIANT
#define MIT_GEMM_DEFAULT_VARIANT 0  // A/B builds (tools/build_variants.sh) may start in another variant
#endif
int g_variant = MIT_GEMM_DEFAULT_VARIANT;
int gemm_variant() { return g_variant; }

// bf16 outputs with a gatherable epilogue leave through each wave's LDS stage (STG 1: no operand,
// STG 2: with the residual / aux block); f32 outputs and the other epilogues through registers
template <int AL, int BL, int ACT, bool DROP>
void launch_bf16_256(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, hipStream_t s) {
  const long nbm = (g->M + 255) / 256, nbn = (g->N + B2 - 1) / B2;
  static bool attr = false;
  if (!attr) {
    set_lds(gemm256_kernel<AL, BL, ACT, DROP>, SMEM2_BYTES);
    if constexpr (AL == MIT_K_CONTIG) {
      set_lds(gemm256_kernel<AL, BL, ACT, DROP, 1>, SMEM2_EPI_BYTES);
      if constexpr (ACT == MIT_ACT_NONE) set_lds(gemm256_kernel<AL, BL, ACT, DROP, 2>, SMEM2_EPI_BYTES);
    }
    if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {
      if constexpr (ACT == MIT_ACT_NONE) set_lds(gemm256_kernel<AL, BL, ACT, DROP, 4>, SMEM2_EPI_BYTES);
      if constexpr (!DROP) set_lds(gemm256_kernel<AL, BL, ACT, DROP, 3>, SMEM2_EPI_BYTES);
    }
    attr = true;
  }
  const dim3 grid((unsigned)(nbm * nbn));
  if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG && !DROP) {  // one-wave-per-SIMD prototype (variant 4)
    if (gemm_variant() == 4 && g->K % BK == 0 && (!e.res || e.stats_out) && !e.aux && !e.out_f32 && epi_gatherable(e)) {
      static bool wattr = false;
      if (!wattr) {
        set_lds(gemm256w_kernel<ACT, 1>, SMEM2_EPI_BYTES);
        set_lds(gemm256w_kernel<ACT, 3>, SMEM2_EPI_BYTES);
        if constexpr (ACT == MIT_ACT_NONE) set_lds(gemm256w_kernel<ACT, 4>, SMEM2_EPI_BYTES);
        wattr = true;
      }
      if constexpr (ACT == MIT_ACT_NONE) {
        if (e.stats_out) {
          hipLaunchKernelGGL((gemm256w_kernel<ACT, 4>), grid, dim3(256), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                             (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e);
          return;
        }
      }
      if (e.ln_stats)
        hipLaunchKernelGGL((gemm256w_kernel<ACT, 3>), grid, dim3(256), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                           (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e);
      else
        hipLaunchKernelGGL((gemm256w_kernel<ACT, 1>), grid, dim3(256), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                           (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e);
      return;
    }
  }
  if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {  // LayerNorm fold / statistics (mit_gemm checked them)
    if constexpr (!DROP) {
      if (e.ln_stats) {
        hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, 3>), grid, dim3(512), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                           (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e,
                           (float*)g->workspace, g->rowsum);
        return;
      }
    }
    if constexpr (ACT == MIT_ACT_NONE) {
      if (e.stats_out) {
        hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, 4>), grid, dim3(512), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                           (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e,
                           (float*)g->workspace, g->rowsum);
        return;
      }
    }
  }
  if constexpr (AL == MIT_K_CONTIG) {
    const bool ops = e.res || e.aux;
    if (epi_gatherable(e) && !e.out_f32) {
      if constexpr (ACT == MIT_ACT_NONE) {
        if (ops) {
          hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, 2>), grid, dim3(512), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                             (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e,
                             (float*)g->workspace, g->rowsum);
          return;
        }
      }
      if (!ops) {
        hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, 1>), grid, dim3(512), SMEM2_EPI_BYTES, s, (const bf16*)g->A,
                           (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e,
                           (float*)g->workspace, g->rowsum);
        return;
      }
    }
  }
  hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP>), grid, dim3(512), SMEM2_BYTES, s, (const bf16*)g->A,
                     (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e,
                     (float*)g->workspace, g->rowsum);
}

// register-streaming kernel (gemm_rs_kernel): the decode step's B-row GEMMs (M <= 256) with a short
// K and N <= 2048 -- 7.2 vs 9.9 us per launch on 256 x {512, 1536, 2048} x 512. Everywhere else it
// loses: each wave streams its own A and B fragments from L2 (8 FLOP per L2 byte vs 64 for the 128
// kernel's LDS tiles): 2.5-3x slower on the M = 4032 decoder shapes, 2x on the decode fc_out
// (tools/blas_reference.py)
bool use_rs(const mit_gemm_args* g) {
  if (g->a_layout != MIT_K_CONTIG || g->b_layout != MIT_K_CONTIG || g->rowsum || g->ln_stats || g->stats_out) return false;
  const int v = gemm_variant();
  if (v == 3) return true;
  if (v != 0 && v != 4) return false;
  return g->M <= 256 && g->N <= 2048 && g->K <= 1024;
}

// Occupancy-quantised cost model: the 128x128 kernel runs 2 blocks per CU, the 256x256 kernel 1;
// a "round" fills every slot once, and a round of the 256 kernel moves 4 tiles' worth of 128x128
// work per CU-slot at REL256 x the 128 kernel's per-FLOP speed (tools/gemm_bench.py).
bool use_256(long M, long N, long K, int a_layout, int tiles) {
  const int v = gemm_variant();
  if (v == 1) return false;
  if (v == 2) return true;
  // the MN-contig-A instances (weight gradients) exceed 256 VGPRs and spill: 128 kernel (+ split-K)
  if (a_layout != MIT_K_CONTIG) return false;
  if (M < 256 || N < 256 || K < 128 || tiles == 128) return false;
  if (tiles == 256) return true;  // the caller runs other work beside this launch (mit_gemm_args.tiles)
  const double REL256 = 1.3, CUS = 256.0;
  const double t128 = (double)(((M + 127) / 128) * ((N + 127) / 128));
  const double t256 = (double)(((M + 255) / 256) * ((N + 255) / 256));
  const double c128 = std::ceil(t128 / (2 * CUS));             // rounds of 2 concurrent 128-tiles per CU
  const double c256 = std::ceil(t256 / CUS) * 2.0 / REL256;    // one 256-tile = 4 128-tiles on 1 slot of 2
  return c256 < c128;
}

// epilogue instance for a bf16 GEMM: {act, dropout} as template parameters where an instance
// exists (the combinations the train step uses), else the generic run-time instance
enum EpiKind { EK_PLAIN, EK_RELU, EK_RELU_DROP, EK_GELU, EK_QGELU, EK_GENERIC };
EpiKind epi_kind(const mit_gemm_args* g) {
  const bool drop = g->drop_p > 0.f;
  if (g->act == MIT_ACT_NONE && !drop) return EK_PLAIN;
  if (g->a_layout != MIT_K_CONTIG || g->b_layout != MIT_K_CONTIG) return EK_GENERIC;
  if (g->act == MIT_ACT_RELU) return drop ? EK_RELU_DROP : EK_RELU;
  if (drop) return EK_GENERIC;
  return g->act == MIT_ACT_GELU ? EK_GELU : EK_QGELU;
}

template <int AL, int BL>
void launch_layout(const mit_gemm_args* g, const Epi& e, int ab, int bb, const Split& sp, bool big, hipStream_t s) {
  const EpiKind k = epi_kind(g);
  if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {
    if (sp.ks == 1 && use_rs(g)) {
      switch (k) {
        case EK_PLAIN: return launch_rs<MIT_ACT_NONE, false>(g, e, ab, bb, s);
        case EK_RELU: return launch_rs<MIT_ACT_RELU, false>(g, e, ab, bb, s);
        case EK_RELU_DROP: return launch_rs<MIT_ACT_RELU, true>(g, e, ab, bb, s);
        case EK_GELU: return launch_rs<MIT_ACT_GELU, false>(g, e, ab, bb, s);
        case EK_QGELU: return launch_rs<MIT_ACT_QUICK_GELU, false>(g, e, ab, bb, s);
        default: return launch_rs<ACT_RT, true>(g, e, ab, bb, s);
      }
    }
  }
  // the 256 kernel's activation instances take no residual / aux operand (gemm256_kernel, XOPS)
  if (big && k != EK_GENERIC && (g->act == MIT_ACT_NONE || (!g->residual && !g->aux))) {
    if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {
      switch (k) {
        case EK_RELU: return launch_bf16_256<AL, BL, MIT_ACT_RELU, false>(g, e, ab, bb, s);
        case EK_RELU_DROP: return launch_bf16_256<AL, BL, MIT_ACT_RELU, true>(g, e, ab, bb, s);
        case EK_GELU: return launch_bf16_256<AL, BL, MIT_ACT_GELU, false>(g, e, ab, bb, s);
        case EK_QGELU: return launch_bf16_256<AL, BL, MIT_ACT_QUICK_GELU, false>(g, e, ab, bb, s);
        default: break;
      }
    }
    return launch_bf16_256<AL, BL, MIT_ACT_NONE, false>(g, e, ab, bb, s);
  }
  if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {
    switch (k) {
      case EK_PLAIN: return launch_bf16<AL, BL, MIT_ACT_NONE, false>(g, e, ab, bb, sp, s);
      case EK_RELU: return launch_bf16<AL, BL, MIT_ACT_RELU, false>(g, e, ab, bb, sp, s);
      case EK_RELU_DROP: return launch_bf16<AL, BL, MIT_ACT_RELU, true>(g, e, ab, bb, sp, s);
      case EK_GELU: return launch_bf16<AL, BL, MIT_ACT_GELU, false>(g, e, ab, bb, sp, s);
      case EK_QGELU: return launch_bf16<AL, BL, MIT_ACT_QUICK_GELU, false>(g, e, ab, bb, sp, s);
      default: return launch_bf16<AL, BL, ACT_RT, true>(g, e, ab, bb, sp, s);
    }
  }
  if (k == EK_PLAIN) return launch_bf16<AL, BL, MIT_ACT_NONE, false>(g, e, ab, bb, sp, s);
  return launch_bf16<AL, BL, ACT_RT, true>(g, e, ab, bb, sp, s);
}

template <int AL, int BL>
void launch_f32(const mit_gemm_args* g, const Epi& e, hipStream_t s) {
  dim3 grid((unsigned)((g->N + 63) / 64), (unsigned)((g->M + 63) / 64));
  hipLaunchKernelGGL((gemm_f32_kernel<AL, BL>), grid, dim3(256), 0, s, (const float*)g->A, (const float*)g->B, g->C, g->M,
                     g->N, g->K, g->lda, g->ldb, g->ldc, e, g->rowsum);
}

inline bool al16(const void* p) { return ((uintptr_t)p % 16) == 0; }

Split plan_split(const mit_gemm_args* g) {
  Split p;
  p.kchunk = g->K;
  if (!g->workspace || !al16(g->workspace)) return p;
  // plain epilogues only: splitting the decoder's long-K GEMMs that carry a bias / residual (fc2 forward,
  // the fc1 / self_in data gradients; the reduce applying them) cost 1.8 % of the step (12639 / 12702 vs
  // 12885 / 12898 pairs/s): their extra workgroups and reduce launches take CUs from the encoder prefetch
  const bool plain = !g->bias && g->act == MIT_ACT_NONE && !g->residual && !g->aux && g->drop_p <= 0.f;
  long kc;
  if (plain && g->ldc % 4 == 0 && al16(g->C)) {
    const int s = splitk_plan(g->M, g->N, g->K, &kc, g->a_layout);
    if (s > 1 && splitk_ws_bytes(g->M, g->N, s) <= g->workspace_bytes) {
      p.ks = s;
      p.kchunk = kc;
      return p;
    }
  }
  return p;
}

}  // namespace

extern "C" int mit_gemm_set_variant(int v) {
  MIT_CHECK_ARG(v >= 0 && v <= 4, "mit_gemm_set_variant: %d not in {0,1,2,3,4}", v);
  g_variant = v;
  return MIT_OK;
}

extern "C" long mit_gemm_workspace_bytes(long M, long N, long K) {
  long kc;
  return max(splitk_ws_bytes(M, N, splitk_plan(M, N, K, &kc)),
             splitk_ws_bytes(M, N, splitk_plan(M, N, K, &kc, MIT_K_CONTIG)));
}

extern "C" int mit_gemm_plan(const mit_gemm_args* g, int* ksplit) {
  if (ksplit) *ksplit = 1;
  if (!g || g->M <= 0 || g->N <= 0) return 0;
  if (g->dtype != MIT_BF16) return 64;
  if (g->argmax_keys) return 128;
  const Split sp = plan_split(g);
  if (ksplit) *ksplit = sp.ks;
  if (sp.ks == 1 && use_rs(g)) return 65;  // the 64x64 register-streaming kernel
  const bool big = sp.ks == 1 && (use_256(g->M, g->N, g->K, g->a_layout, g->tiles) || g->ln_stats || g->stats_out) &&
                   epi_kind(g) != EK_GENERIC && (g->act == MIT_ACT_NONE || (!g->residual && !g->aux));
  return big ? 256 : 128;
}

extern "C" int mit_gemm(const mit_gemm_args* g, void* stream) {
  MIT_CHECK_ARG(g != nullptr, "mit_gemm: null args");
  MIT_RECORD([c = *g, stream]() { return mit_gemm(&c, stream); });
  MIT_CHECK_ARG(g->dtype == MIT_F32 || g->dtype == MIT_BF16, "mit_gemm: bad dtype %d", g->dtype);
  MIT_CHECK_ARG(g->M >= 0 && g->N >= 0 && g->K >= 0, "mit_gemm: negative extent");
  MIT_CHECK_ARG(g->A && g->B && (g->C || g->argmax_keys), "mit_gemm: null operand");
  MIT_CHECK_ARG(g->a_layout == MIT_K_CONTIG || g->a_layout == MIT_MN_CONTIG, "mit_gemm: bad a_layout");
  MIT_CHECK_ARG(g->b_layout == MIT_K_CONTIG || g->b_layout == MIT_MN_CONTIG, "mit_gemm: bad b_layout");
  MIT_CHECK_ARG(g->act >= MIT_ACT_NONE && g->act <= MIT_ACT_QUICK_GELU, "mit_gemm: bad act %d", g->act);
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
  if (g->argmax_keys) {
    MIT_CHECK_ARG(g->dtype == MIT_BF16 && g->a_layout == MIT_K_CONTIG && g->b_layout == MIT_K_CONTIG && !g->C &&
                      g->act == MIT_ACT_NONE && !g->residual && !g->aux && g->drop_p <= 0.f && g->alpha == 1.0f &&
                      !g->rowsum && !g->accumulate && !g->ln_stats && !g->stats_out && (!g->bias || al16(g->bias)) &&
                      ((uintptr_t)g->argmax_keys % 8) == 0 && g->N < (1L << 32),
                  "mit_gemm: argmax_keys needs bf16 NT operands, a bias only and no C");
  }
  if (g->ln_stats || g->stats_out) {
    // the LayerNorm fold / row statistics exist only in the 256 kernel's LDS-staged bf16 epilogue
    MIT_CHECK_ARG(g->dtype == MIT_BF16 && g->a_layout == MIT_K_CONTIG && g->b_layout == MIT_K_CONTIG && !g->out_f32 &&
                      !g->accumulate && !g->aux && g->drop_p <= 0.f && g->alpha == 1.0f && !g->rowsum && !g->workspace &&
                      g->N % 8 == 0 && g->ldc % 8 == 0 && al16(g->C) && (!g->bias || al16(g->bias)),
                  "mit_gemm: ln_stats / stats_out need bf16 NT operands, a bf16 output with a plain vector epilogue");
    MIT_CHECK_ARG(!(g->ln_stats && g->stats_out), "mit_gemm: ln_stats and stats_out are exclusive");
  }
  if (g->ln_stats) {
    MIT_CHECK_ARG(g->ln_colsum && al16(g->ln_colsum) && g->K % 64 == 0 && g->ln_parts == g->K / 64 && g->ln_parts <= 16 &&
                      !g->residual && g->ln_eps >= 0.f,
                  "mit_gemm: ln_stats needs ln_colsum (16-B aligned), K %% 64 == 0, ln_parts = K / 64 <= 16, no residual");
  }
  if (g->stats_out) {
    MIT_CHECK_ARG(g->N % 64 == 0 && g->act == MIT_ACT_NONE && g->residual && g->ldr % 8 == 0 && al16(g->residual),
                  "mit_gemm: stats_out needs N %% 64 == 0, no activation and a (16-B aligned) residual");
  }
  Epi e;
  e.ln_stats = g->ln_stats;
  e.ln_colsum = g->ln_colsum;
  e.ln_parts = g->ln_parts;
  e.ln_eps = g->ln_eps;
  e.stats_out = g->stats_out;
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
  e.argmax_keys = g->argmax_keys;
  hipStream_t s = (hipStream_t)stream;
  if (g->argmax_keys) {  // the 128 kernel's gathered epilogue (any N: columns >= N never enter a key)
    e.vec = 1;
    launch_bf16<MIT_K_CONTIG, MIT_K_CONTIG, MIT_ACT_NONE, false>(g, e, (int)a_bytes, (int)b_bytes, Split{}, s);
    MIT_LAUNCH_CHECK("mit_gemm");
    return MIT_OK;
  }
  if (g->dtype == MIT_BF16) {
    const int ab = (int)a_bytes, bb = (int)b_bytes;
    const Split sp = plan_split(g);
    const bool big = sp.ks == 1 && (use_256(g->M, g->N, g->K, g->a_layout, g->tiles) || g->ln_stats || g->stats_out);
    if (g->a_layout == 0 && g->b_layout == 0) launch_layout<0, 0>(g, e, ab, bb, sp, big, s);
    else if (g->a_layout == 0 && g->b_layout == 1) launch_layout<0, 1>(g, e, ab, bb, sp, big, s);
    else if (g->a_layout == 1 && g->b_layout == 0) launch_layout<1, 0>(g, e, ab, bb, sp, big, s);
    else launch_layout<1, 1>(g, e, ab, bb, sp, big, s);
    if (sp.ks > 1) {
      MIT_LAUNCH_CHECK("mit_gemm");
      const long total = g->M * (g->N / 4);
      long blocks = (total + 255) / 256;
      if (blocks > 4096) blocks = 4096;
      hipLaunchKernelGGL(gemm_splitk_reduce, dim3((unsigned)blocks), dim3(256), 0, s, g->M, g->N, sp.ks,
                         (const float*)((char*)g->workspace + WS_HDR), g->C, g->ldc, g->alpha, g->out_f32,
                         g->accumulate, g->rowsum);
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

// group split-K factor: about one block per CU over all problems -- at cfg1 (224 tiles per layer, 216
// for the cross-K/V + projection pair) no split: 12482-12503 pairs/s vs 12278-12433 with 2 (two blocks
// per CU), 12232-12263 with 3, 12081-12153 with 4 (interleaved, one box); the fp32 slabs and their
// combine cost more than the shorter K loops save once the group fills the chip.
long grouped_split(long tiles) {
  return tiles > 0 ? max(1L, min(16L, (long)num_cus() / tiles)) : 1;
}

extern "C" long mit_gemm_grouped_ws_bytes(const mit_gemm_args* args, int n) {
  if (!args || n <= 0 || n > MAXG) return 0;
  long tiles = 0;
  for (int i = 0; i < n; ++i) tiles += ((args[i].M + BM - 1) / BM) * ((args[i].N + BN - 1) / BN);
  long s = grouped_split(tiles);
  long bytes = WS_HDR;
  for (int i = 0; i < n; ++i) {
    const long si = max(1L, min(s, args[i].K / 512));
    bytes += si > 1 ? (4L * si * args[i].M * args[i].N + 4L * si * args[i].M + 255) / 256 * 256 : 0;
  }
  return bytes;
}

// Grouped dW launch (see gemm_bf16_grouped): split-K factor chosen for the group (about two blocks
// per CU over all problems), slabs of problem i at consecutive 256-B aligned offsets of workspace.
extern "C" int mit_gemm_grouped(const mit_gemm_args* args, int n, const mit_ln_grads_job* ln, int n_ln,
                                void* workspace, long workspace_bytes, void* stream) {
  MIT_CHECK_ARG(args && n >= 1 && n <= MAXG, "mit_gemm_grouped: 1..%d problems", MAXG);
  MIT_CHECK_ARG(n_ln >= 0 && n_ln <= MAXLN && (n_ln == 0 || ln), "mit_gemm_grouped: 0..%d LayerNorm jobs", MAXLN);
  MIT_RECORD([v = std::vector<mit_gemm_args>(args, args + n),
              lv = std::vector<mit_ln_grads_job>(ln, ln + n_ln), workspace, workspace_bytes, stream]() {
    return mit_gemm_grouped(v.data(), (int)v.size(), lv.data(), (int)lv.size(), workspace, workspace_bytes, stream);
  });
  for (int j = 0; j < n_ln; ++j)
    MIT_CHECK_ARG(ln[j].ws && ln[j].dgamma && ln[j].dbeta && ln[j].rows > 0 && ln[j].cols > 0,
                  "mit_gemm_grouped: LayerNorm job %d: null pointer or empty", j);
  MIT_CHECK_ARG(workspace_bytes >= mit_gemm_grouped_ws_bytes(args, n) && (workspace || workspace_bytes == 0) &&
                    al16(workspace),
                "mit_gemm_grouped: workspace too small (%ld < %ld)", workspace_bytes, mit_gemm_grouped_ws_bytes(args, n));
  long tiles = 0;
  for (int i = 0; i < n; ++i) {
    const mit_gemm_args* g = args + i;
    MIT_CHECK_ARG(g->dtype == MIT_BF16 && g->a_layout == MIT_MN_CONTIG && g->b_layout == MIT_MN_CONTIG,
                  "mit_gemm_grouped: problem %d: bf16 MN-contig operands (weight gradients) only", i);
    MIT_CHECK_ARG(!g->bias && g->act == MIT_ACT_NONE && !g->residual && !g->aux && g->drop_p <= 0.f && g->out_f32,
                  "mit_gemm_grouped: problem %d: plain epilogue with an f32 output only", i);
    MIT_CHECK_ARG(g->A && g->B && g->C && g->M > 0 && g->N > 0 && g->K > 0, "mit_gemm_grouped: problem %d: empty", i);
    MIT_CHECK_ARG(g->lda >= g->M && g->ldb >= g->N && g->ldc >= g->N && g->lda % 8 == 0 && g->ldb % 8 == 0 &&
                      g->M % 8 == 0 && g->N % 8 == 0 && g->ldc % 4 == 0 && al16(g->A) && al16(g->B) && al16(g->C),
                  "mit_gemm_grouped: problem %d: extents / alignment", i);
    MIT_CHECK_ARG(2 * ((g->K - 1) * g->lda + g->M) < (1L << 31) && 2 * ((g->K - 1) * g->ldb + g->N) < (1L << 31),
                  "mit_gemm_grouped: problem %d: operand spans >= 2 GiB", i);
    tiles += ((g->M + BM - 1) / BM) * ((g->N + BN - 1) / BN);
  }
  const long s = grouped_split(tiles);
  GroupArgs ga;
  ga.n = n;
  int start = 0, rstart = 0;
  bool any_split = false;
  char* wsp = (char*)workspace + WS_HDR;
  for (int i = 0; i < n; ++i) {
    const mit_gemm_args* g = args + i;
    GroupProb& q = ga.p[i];
    q.A = (const bf16*)g->A;
    q.B = (const bf16*)g->B;
    q.C = g->C;
    q.M = g->M; q.N = g->N; q.K = g->K; q.lda = g->lda; q.ldb = g->ldb; q.ldc = g->ldc;
    q.a_bytes = (int)(2 * ((g->K - 1) * g->lda + g->M));
    q.b_bytes = (int)(2 * ((g->K - 1) * g->ldb + g->N));
    long si = max(1L, min(s, g->K / 512));
    long kc = (g->K + si - 1) / si;
    kc = (kc + BK - 1) / BK * BK;
    si = (g->K + kc - 1) / kc;
    q.ksplit = (int)si;
    q.kchunk = kc;
    q.rowsum = g->rowsum;
    q.ws = nullptr;
    if (si > 1) {
      q.ws = (float*)wsp;
      wsp += (4L * si * g->M * g->N + 4L * si * g->M + 255) / 256 * 256;
      any_split = true;
    }
    Epi& e = q.e;
    e = Epi{};
    e.alpha = g->alpha;
    e.act = MIT_ACT_NONE;
    e.out_f32 = 1;
    e.accumulate = g->accumulate;
    e.vec = (g->N % 8 == 0) && (g->ldc % 8 == 0) && al16(g->C);
    q.start = start;
    start += (int)(((g->M + BM - 1) / BM) * ((g->N + BN - 1) / BN) * si);
    q.rblocks = si > 1 ? (int)min(1024L, (g->M * (g->N / 4) + 255) / 256) : 0;
    q.rstart = rstart;
    rstart += q.rblocks;
  }
  hipStream_t st = (hipStream_t)stream;
  static bool attr = false;
  if (!attr) {
    set_lds(gemm_bf16_grouped, smem_bytes(2));
    attr = true;
  }
  // deal the tiles to the XCDs: problem after problem, at most cap per XCD
  const int cap = (start + 7) / 8;
  int np = 0, xc = 0, used = 0;
  ga.xfirst[0] = 0;
  for (int i = 0; i < n; ++i) {
    const int ti = (i + 1 < n ? ga.p[i + 1].start : start) - ga.p[i].start;
    for (int t = 0; t < ti;) {
      const int take = min(ti - t, cap - used);
      ga.pc[np++] = GroupPiece{i, t, take};
      t += take;
      used += take;
      if (used == cap) {
        ga.xfirst[++xc] = np;
        used = 0;
      }
    }
  }
  while (xc < 8) ga.xfirst[++xc] = np;
  MIT_CHECK_ARG(np <= MAXP, "mit_gemm_grouped: %d XCD pieces", np);
  start = 8 * cap;
  ga.gemm_blocks = start;
  ga.nln = n_ln;
  for (int j = 0; j < n_ln; ++j) {
    GroupLn& q = ga.ln[j];
    q.ws = ln[j].ws;
    q.dgamma = ln[j].dgamma;
    q.dbeta = ln[j].dbeta;
    q.cols = ln[j].cols;
    q.nblk = mit_layernorm_bwd_ws_floats(ln[j].rows, ln[j].cols) / (2 * ln[j].cols);
    q.start = start;
    start += (int)((2 * ln[j].cols + 31) / 32);
  }
  hipLaunchKernelGGL(gemm_bf16_grouped, dim3((unsigned)start), dim3(512), smem_bytes(2), st, ga);
  MIT_LAUNCH_CHECK("mit_gemm_grouped");
  if (any_split) {
    hipLaunchKernelGGL(gemm_splitk_reduce_grouped, dim3((unsigned)rstart), dim3(256), 0, st, ga);
    MIT_LAUNCH_CHECK("mit_gemm_grouped");
  }
  return MIT_OK;
}

