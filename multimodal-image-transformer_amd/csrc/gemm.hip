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
//   * gemm_bf16_kernel: 128x128x64, 4 waves (2x2, 64x64 each), 2 blocks per CU, 2 LDS stages,
//     optional split-K with fused bias-gradient row sums (weight gradients).
//   * gemm256_kernel: 256x256x64, 8 waves (2x4, 128x64 each), 1 block per CU, 8-phase ping-pong
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
// fp32 path (parity mode): a plain LDS-tiled FMA kernel with the identical epilogue semantics.
#include <stdlib.h>

#include <cmath>
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
};

constexpr int ACT_RT = -1;
  // activation read from Epi::act at run time (generic instance)

// FAST: bf16 vector epilogues use the branch-free GELU (gelu_fast, |err| ~1e-7, far below bf16
// rounding); the scalar / fp32-parity path keeps ocml's erff
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

// ------------------------------------------------------------------------------------------------
// operand tiles in LDS
// ------------------------------------------------------------------------------------------------
constexpr int BM = 128, BN = 128, BK = 64;
constexpr int TILE_BYTES = BM * BK * 2;          // 16 KiB per operand per stage
constexpr int CST = BN + 4;                      // fp32 C-tile row stride in LDS (floats)
// + 16 B past the fp32 C stage: the split-K combine's "last slice" flag
constexpr int smem_bytes(int nst) {
  return (2 * nst * TILE_BYTES > BM * CST * 4 + 16) ? 2 * nst * TILE_BYTES : BM * CST * 4 + 16;
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
                                               float* __restrict__ ws, float* __restrict__ rowsum,
                                               int* __restrict__ tile_cnt, long ws_bytes, int blk, int GROUP = 8) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // NW = 4: waves 2 (M) x 2 (N), 64x64 each; NW = 8: 4 (M) x 2 (N), 32x64 each (MI 16-row blocks)
  constexpr int NT = 64 * NW, WR = 128 / (NW / 2), MI = WR / 16;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int nbn = (int)((N + BN - 1) / BN), nbm = (int)((M + BM - 1) / BM);
  const int ntiles = nbn * nbm, nwg = ntiles * ksplit;
  int bid = xcd_remap(blk, nwg);
  // split-K: slice `split` covers k in [kb, ke); a tile's slices are neighbours in the remapped
  // order, i.e. on one XCD (the in-launch combine below reads same-XCD slabs fastest)
  const int split = bid % ksplit;
  bid /= ksplit;
  const long kb = (long)split * kchunk, ke = min(K, kb + kchunk);
  // groups of GROUP M-blocks walk the N-blocks together (B panel reuse in L2); GROUP = 1: row-major
  // tiles, so an XCD's contiguous run of tiles shares its A row panels (the grouped dW launch)
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
  // In-launch split-K combine (tile_cnt != NULL): every slice stores its fp32 partial tile as a
  // write-through (sc1) slab, drains, and draws a ticket from the tile's counter; the slice that
  // draws ksplit-1 acquires, sums the slabs in slice order (its own from LDS: the same bits) and
  // runs the full epilogue, so the result does not depend on arrival order. It also re-zeroes the
  // counter for the next launch (the caller zero-fills the workspace once).
  if (tile_cnt) {
    const __amdgpu_buffer_rsrc_t rw = __builtin_amdgcn_make_buffer_rsrc((void*)ws, (short)0, (int)ws_bytes, 0x00020000);
    const int slab = (split * ntiles + bid) * (BM * BN);
#pragma unroll 4
    for (int pass = 0; pass < (BM * BN / 4) / NT; ++pass) {
      const int id = pass * NT + tid;
      const int r = id >> 5, c4 = (id & 31) * 4;
      const f32x4 v = *(const f32x4*)(cs + r * CST + c4);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rw, (slab + r * BN + c4) * 4, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* flag = (int*)(smem + BM * CST * 4);
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(tile_cnt + bid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int last = t == ksplit - 1;
      if (last) {
        __hip_atomic_store(tile_cnt + bid, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      *flag = last;
    }
    __syncthreads();
    if (!*flag) return;
  }
  if (!tile_cnt && ksplit == 1 && epi_gatherable(e)) {  // gathered epilogue: all loads, then all stores
    constexpr int NP = (BM * BN / 8) / NT;
    const long gc = n0 + (tid & 15) * 8;  // this thread's columns are the same in every pass
    float b[8];
    epi_bias8(e, gc, N, b);
    bf16x8 xs[NP];
#pragma unroll
    for (int pass = 0; pass < NP; ++pass) xs[pass] = epi_x8(e, M, N, m0 + ((pass * NT + tid) >> 4), gc);
    gather_wait();
    const uint64_t key = epi_key<DROP>(e);
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
    f32x4 lo = *(const f32x4*)(cs + r * CST + c8), hi = *(const f32x4*)(cs + r * CST + c8 + 4);
    if (tile_cnt) {
      f32x4 sl = {0.f, 0.f, 0.f, 0.f}, sh = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < ksplit; ++k) {
        if (k == split) {
          sl += lo;
          sh += hi;
        } else {
          const float* p = ws + (long)(k * ntiles + bid) * (BM * BN) + r * BN + c8;
          sl += *(const f32x4*)p;
          sh += *(const f32x4*)(p + 4);
        }
      }
      lo = sl;
      hi = sh;
    } else if (ksplit > 1) {  // raw fp32 partial slab; gemm_splitk_reduce applies the (plain) epilogue
      f32x4* o = (f32x4*)(ws + ((long)split * M + gr) * N + gc);
      o[0] = lo;
      o[1] = hi;
      continue;
    }
    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    epi_row8<ACT, DROP>(e, C, ldc, N, gr, gc, v);
  }
}

template <int ALAY, int BLAY, int ACT, bool DROP, int NST, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemm_bf16_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                        long M, long N, long K, long lda, long ldb, long ldc,
                                                        int a_bytes, int b_bytes, Epi e, int ksplit, long kchunk,
                                                        float* __restrict__ ws, float* __restrict__ rowsum,
                                                        int* __restrict__ tile_cnt, long ws_bytes) {
  gemm_bf16_body<ALAY, BLAY, ACT, DROP, NST, NW>(A, B, C, M, N, K, lda, ldb, ldc, a_bytes, b_bytes, e, ksplit, kchunk,
                                                ws, rowsum, tile_cnt, ws_bytes, blockIdx.x);
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
struct GroupArgs {
  GroupProb p[MAXG];
  GroupLn ln[MAXLN];
  int n, nln, gemm_blocks, group;
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
  int i = 0;
  while (i + 1 < ga.n && (int)blockIdx.x >= ga.p[i + 1].start) ++i;
  const GroupProb& q = ga.p[i];
  // weight gradients dW = dY^T X with K = B*T: the dY column panel (K x 128, the A operand) of a
  // tile row is read once when that row's tiles sit on one XCD (GROUP 1, MIT_GROUPED_GROUP)
  gemm_bf16_body<MIT_MN_CONTIG, MIT_MN_CONTIG, MIT_ACT_NONE, false, 2, 8>(
      q.A, q.B, q.C, q.M, q.N, q.K, q.lda, q.ldb, q.ldc, q.a_bytes, q.b_bytes, q.e, q.ksplit, q.kchunk, q.ws, q.rowsum,
      nullptr, 0, (int)blockIdx.x - q.start, ga.group);
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

// compile-time A/B switches of the 256 kernel (tools/build_variants.sh): row-group height of the
// tile order and the XCD remap
#ifndef MIT_G256_GROUP
#define MIT_G256_GROUP 4
#endif
#ifndef MIT_G256_NOREMAP
#define MIT_G256_NOREMAP 0
#endif
// 4 barriers per K-tile (merged phases) with the A half-1 DMA issued one phase earlier is the
// default (+3-5 % on the 256-tile shapes, profiles/r01_gemm256_schedule_ab.txt); 0 = the 8-phase loop
#ifndef MIT_G256_PH4
#define MIT_G256_PH4 1
#endif
#ifndef MIT_G256_EARLY_A1
#define MIT_G256_EARLY_A1 1
#endif
#ifndef MIT_G256_REGEPI  // register epilogue in the one-tile 256 kernel (K-contig A)
#define MIT_G256_REGEPI 1
#endif
// Wave priority A/B (round 3, step A/B on one box): raising the priority around each MFMA
// block (=1, round 2's default) and one static priority for the younger wave group
// (MIT_G256_STATIC_PRIO) both measured 0.5 % slower in the step than no s_setprio at all with the
// staged epilogue (12.42 k vs 12.49 k pairs/s, 3 alternations) -> off by default.
#ifndef MIT_G256_PRIO
#define MIT_G256_PRIO 0
#endif
#ifndef MIT_G256_STATIC_PRIO
#define MIT_G256_STATIC_PRIO 0
#endif
// Epilogue staged through LDS (f32, two passes of 128 tile rows) so that every store instruction
// writes MIT_G256_EPR whole rows of the tile (2: two 512-B row runs per wave instruction). The
// register epilogue's stores (16 rows x 64 B per instruction) and the 8-rows x 128-B form both run
// at ~30 GB/s per CU (4.4-5 us per 256x256 bf16 tile, tools/g256_stamps.py), ~4x slower than
// long contiguous runs: the store INSTRUCTION pattern, not bytes, bounds the epilogue.
#ifndef MIT_G256_EPI_LDS
#define MIT_G256_EPI_LDS 0
#endif
#ifndef MIT_G256_EPR
#define MIT_G256_EPR 2
#endif
// bf16 outputs through each wave's private LDS stage (stage_epilogue) instead of the register
// exchange (reg_epilogue)
#ifndef MIT_G256_EPI_STAGE
#define MIT_G256_EPI_STAGE 1
#endif


// Diagnostic build only (-DMIT_G256_STAMP, tools/g256_stamps.py): per workgroup, wave 0 and wave 4 stamp
// the shader clock (s_memtime) at entry, after the prologue's first barrier, after the K loop and after
// the epilogue's stores have drained, plus the 100 MHz global clock at entry / exit and the XCC id. The
// stamps go to their own __device__ buffer (never an output); the shipped library compiles none of it.
#ifdef MIT_G256_STAMP
constexpr int G256_SLOTS = 24;  // wave 0: 0-5, wave 4: 6-11, 12 = exit global clock, 13/14 = stores issued, 15-22 epilogue steps (wave 0)
__device__ unsigned long long g256_stamp[16384 * G256_SLOTS];
#define G256_STAMP(slot, val)                                                                        \
  do {                                                                                               \
    if (lane == 0 && (wid == 0 || wid == 4) && blockIdx.x < 16384)                                   \
      g256_stamp[blockIdx.x * G256_SLOTS + (slot) + (wid == 4 ? 6 : 0)] = (unsigned long long)(val); \
  } while (0)
__device__ __forceinline__ unsigned xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15;
}
#define G256_STEP(slot)                                                                             \
  do {                                                                                              \
    if (lane == 0 && wid == 0 && blockIdx.x < 16384)                                                \
      g256_stamp[blockIdx.x * G256_SLOTS + (slot)] = (unsigned long long)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define G256_STEP(slot) \
  do {                  \
  } while (0)
#define G256_STAMP(slot, val) \
  do {                        \
  } while (0)
#endif

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
// PASSES = 2 (the persistent kernel): the 128 rows go through an 8 KiB image in two halves of 64 rows,
// so half the LDS stays free for the next tile's first K-tile; after_loads() runs once the operand
// loads have returned and before the first store (the persistent kernel issues that K-tile's DMA there).
struct NoHook {
  __device__ void operator()() const {}
};
template <int ACT, bool DROP, bool XOPS, int PASSES = 1, typename Hook = NoHook>
__device__ __forceinline__ void stage_epilogue(const f32x4 (&acc)[8][4], const Epi& e, void* C, long ldc, long M,
                                               long N, long mw, long nw, int lane, char* stg,
                                               const Hook& after_loads = Hook{}) {
  static_assert(PASSES == 1 || PASSES == 2, "stage_epilogue: 1 or 2 passes");
  constexpr int IP = 8 / PASSES;  // 16-row blocks per pass
  const int g = lane >> 4, r16 = lane & 15;
  float bj[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const long c = nw + 16 * j + 4 * g;
    if (e.bias && c < N) {
      const f32x4 b = *(const f32x4*)(e.bias + c);
      bj[j][0] = b[0]; bj[j][1] = b[1]; bj[j][2] = b[2]; bj[j][3] = b[3];
    } else {
      bj[j][0] = bj[j][1] = bj[j][2] = bj[j][3] = 0.f;
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
  after_loads();
  const uint64_t key = epi_key<DROP>(e);
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
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) v[t] = acc[i][j][t] * e.alpha + bj[j][t];
        if (ACT == MIT_ACT_GELU) {
#pragma unroll
          for (int t = 0; t < 4; t += 2) {
            const f32x2 q = gelu_fast2(f32x2{v[t], v[t + 1]});
            v[t] = q[0];
            v[t + 1] = q[1];
          }
        } else if (ACT != MIT_ACT_NONE) {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[t] = act_apply<ACT, true>(e.act, v[t]);
        }
        const int ch = 2 * j + (g >> 1);
        char* seg = stg + rr * 128 + ((ch ^ (rr & 7)) << 4) + (g & 1) * 8;
        if constexpr (XOPS) {
          const u32x2 x = *(const u32x2*)seg;
          const float x0 = __uint_as_float(x[0] << 16), x1 = __uint_as_float(x[0] & 0xFFFF0000u);
          const float x2 = __uint_as_float(x[1] << 16), x3 = __uint_as_float(x[1] & 0xFFFF0000u);
          if (e.aux) {
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
          if (e.res) {
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

// MI = 16-row MFMA blocks per wave in M: 8 (256-row tiles) or 5 / 6 (160 / 192-row tiles, K-contig A
// with the register epilogue only): the N = 768 / 1024 encoder GEMMs (o-proj, fc2) have 150 / 580
// 256-row tiles -- one round on 150 of 256 CUs, or a third round for 68 tiles -- and shorter tiles fill
// the rounds (mit_gemm picks per shape, tile_rounds_cost)
template <int ALAY, int BLAY, int ACT, bool DROP, int MI = 8, int STG = 0>
__global__ __launch_bounds__(512) void gemm256_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                      long M, long N, long K, long lda, long ldb, long ldc, int a_bytes,
                                                      int b_bytes, Epi e, int ksplit, long kchunk,
                                                      float* __restrict__ ws, float* __restrict__ rowsum) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  static_assert(MI == 8 || (MI >= 4 && MI < 8 && ALAY == MIT_K_CONTIG), "gemm256_kernel: short tiles need K-contig A");
#ifdef MIT_G256_STAMP
  G256_STAMP(0, __builtin_amdgcn_s_memrealtime());
  G256_STAMP(1, __builtin_amdgcn_s_memtime());
  G256_STAMP(5, xcc_id());
#endif
  constexpr int HR = 16 * MI;          // rows per wave group = rows per A half-tile
  constexpr int BMT = 2 * HR;          // tile rows
  constexpr int IH0 = (MI + 1) / 2;    // row blocks in the wave's first row half (ih = 0)

  const int nbn = (int)((N + B2 - 1) / B2), nbm = (int)((M + BMT - 1) / BMT);
  const int ntiles = nbn * nbm, nwg = ntiles * ksplit;
#if MIT_G256_NOREMAP
  int bid = blockIdx.x;
#else
  int bid = xcd_remap(blockIdx.x, nwg);
#endif
  const int split = bid / ntiles;
  bid -= split * ntiles;
  const long kb = (long)split * kchunk, ke = min(K, kb + kchunk);
  const int GROUP = MIT_G256_GROUP;
  const int group_id = bid / (GROUP * nbn);
  const int first_m = group_id * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  const int bm = first_m + (bid % (GROUP * nbn)) % gsize;
  const int bn = (bid % (GROUP * nbn)) / gsize;
  const long m0 = (long)bm * BMT, n0 = (long)bn * B2;

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
  constexpr bool REG = ALAY == MIT_K_CONTIG && MIT_G256_REGEPI;
  // LDS-staged row-run epilogue for every gatherable epilogue, else the register one
  constexpr bool LDSEPI = REG && MIT_G256_EPI_LDS && MI == 8;
  const bool ldsepi = LDSEPI && ksplit == 1 && epi_gatherable(e);
  const bool regepi = REG && !ldsepi && ksplit == 1 && epi_gatherable(e);
  // LDS-staged bf16 epilogue (stage_epilogue) for bf16 outputs of the 256-row tile
  // STG (launch_256_mi, bf16 out): the LDS-staged epilogue, 1 = no operand, 2 = with the residual /
  // aux operand. A template flag, not a run-time branch: two epilogues in one instance spill in the K loop
  const bool stage = STG && MI == 8 && regepi;
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
#ifdef MIT_G256_DIAG_NOWAIT  // timing diagnostic only (WRONG results): what the DMA waits cost
    (void)younger_issued;
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
#else
    if (younger_issued) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
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
    if (TN && do_rs && MI == 8) {
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
    if (MIT_G256_PRIO) __builtin_amdgcn_s_setprio(1);
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
    if (MIT_G256_PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // prologue: K-tile 0 (all four halves) and B0 of K-tile 1
  issue(0, 0, 0);
  issue(0, 1, 0);
  issue(1, 0, 0);
  issue(1, 1, 0);
  wait_dma(issue(1, 0, 1));
  bar_raw();
  if (wr == 1) bar_raw();  // stagger: group 1 runs one barrier behind group 0
#if MIT_G256_STATIC_PRIO  // A/B: one static priority for the younger half (guide: Two waves per SIMD, item 4)
  if (wr == 1) __builtin_amdgcn_s_setprio(1);
#endif
  G256_STAMP(2, __builtin_amdgcn_s_memtime());

#if MIT_G256_PH4
  // 4 barriers per K-tile instead of 8: the same reads, DMA issues and waits in the same order,
  // two quarter-tile MFMA blocks per phase (a 512-cycle MFMA segment per group hides more of the
  // other group's LDS-read latency)
  for (int t = 0; t < nk; t += 2) {
    const bool two = t + 1 < nk;
    read_a(0, 0);
    read_b(0, 0, blo);
    issue(1, 1, t + 1);
    read_b(0, 1, bhi);
    issue(0, 0, t + 1);
#if MIT_G256_EARLY_A1
    issue(0, 1, t + 1);
#endif
    bar_raw();
    mma(0, 0, blo);
    mma(0, 1, bhi);
    bar_raw();

    read_a(0, 1);
#if !MIT_G256_EARLY_A1
    issue(0, 1, t + 1);
#endif
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
#if MIT_G256_EARLY_A1
    issue(0, 1, t + 2);
#endif
    bar_raw();
    if (two) {
      mma(0, 0, blo);
      mma(0, 1, bhi);
    }
    bar_raw();

    if (two) read_a(1, 1);
#if !MIT_G256_EARLY_A1
    issue(0, 1, t + 2);
#endif
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
#else
  for (int t = 0; t < nk; t += 2) {
    const bool two = t + 1 < nk;  // second K-tile of this iteration exists
    // ---- K-tile t (buffer 0) ----
    read_a(0, 0);
    read_b(0, 0, blo);
    issue(1, 1, t + 1);
    bar_raw();
    mma(0, 0, blo);
    bar_raw();

    read_b(0, 1, bhi);
    issue(0, 0, t + 1);
    bar_raw();
    mma(0, 1, bhi);
    bar_raw();

    read_a(0, 1);
    issue(0, 1, t + 1);
    bar_raw();
    mma(1, 1, bhi);
    bar_raw();

    wait_dma(issue(1, 0, t + 2));
    bar_raw();
    mma(1, 0, blo);
    bar_raw();

    // ---- K-tile t+1 (buffer 1) ----
    if (two) {
      read_a(1, 0);
      read_b(1, 0, blo);
    }
    issue(1, 1, t + 2);
    bar_raw();
    if (two) mma(0, 0, blo);
    bar_raw();

    if (two) read_b(1, 1, bhi);
    issue(0, 0, t + 2);
    bar_raw();
    if (two) mma(0, 1, bhi);
    bar_raw();

    if (two) read_a(1, 1);
    issue(0, 1, t + 2);
    bar_raw();
    if (two) mma(1, 1, bhi);
    bar_raw();

    wait_dma(issue(1, 0, t + 3));
    bar_raw();
    if (two) mma(1, 0, blo);
    bar_raw();
  }
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  G256_STAMP(3, __builtin_amdgcn_s_memtime());
#ifdef MIT_G256_STAMP
  struct StampEnd {  // stamps the epilogue's end (stores drained) on every return path
    int lane, wid;
    __device__ ~StampEnd() {
      if (lane == 0 && (wid == 0 || wid == 4) && blockIdx.x < 16384)  // stores issued, not yet drained
        g256_stamp[blockIdx.x * G256_SLOTS + 13 + (wid == 4)] = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      G256_STAMP(4, __builtin_amdgcn_s_memtime());
      if (wid == 0 && lane == 0 && blockIdx.x < 16384)
        g256_stamp[blockIdx.x * G256_SLOTS + 12] = __builtin_amdgcn_s_memrealtime();
    }
  } stamp_end{lane, wid};
#endif
  if constexpr (LDSEPI) {
    if (ldsepi) {
      // Two passes over the accumulators: pass p stages row blocks i in [4p, 4p+4) of every wave
      // (tile rows p*64 .. p*64+63 and 128+p*64 .. +63) as f32 in LDS ([128][256], 16-B chunks
      // XOR-swizzled by row so the C^T-block writes are conflict-free), then every wave reads back
      // whole-row runs and runs the same gathered epilogue (epi8x: identical arithmetic, bit-identical
      // outputs) with its operands loaded in the same coalesced layout before any store.
      constexpr int EPR = MIT_G256_EPR, LPR = 64 / EPR, CPI = 256 / (LPR * 8);
      static_assert(EPR == 2 || EPR == 4 || EPR == 8, "MIT_G256_EPR: 2, 4 or 8 rows per store");
      if (wr == 0) bar_raw();  // re-align the staggered groups: every LDS read of the loop is done
      bar_raw();
      G256_STEP(15);
      auto lrow = [&](int q) { return wid * 16 + (q / CPI) * EPR + lane / LPR; };   // local row 0..127
      auto lcol = [&](int q) { return (q % CPI) * (LPR * 8) + (lane % LPR) * 8; };  // tile column
      auto grow = [&](int p, int q) {
        const int lr = lrow(q);
        return m0 + (lr >> 6) * 128 + p * 64 + (lr & 63);
      };
      auto chunk_off = [](int lr, int ch) { return lr * 1024 + ((ch ^ (lr & 7)) << 4); };
      auto stage = [&](int p) {  // pass p's accumulators -> LDS (f32, C^T block: lane = row, 4 columns)
#pragma unroll
        for (int ii = 0; ii < 4; ++ii)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int lr = wr * 64 + ii * 16 + (lane & 15);
            const int ch = wc * 16 + j * 4 + (lane >> 4);
            *(f32x4*)(smem + chunk_off(lr, ch)) = acc[p * 4 + ii][j];
          }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        bar_raw();
      };
      auto fetch = [&](int q, float* v) {
        const int lr = lrow(q), ch = lcol(q) >> 2;
        const f32x4 a = *(const f32x4*)(smem + chunk_off(lr, ch)), b = *(const f32x4*)(smem + chunk_off(lr, ch + 1));
        v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
      };
      float bq[CPI][8];
#pragma unroll
      for (int c = 0; c < CPI; ++c) epi_bias8(e, n0 + lcol(c), N, bq[c]);
      const uint64_t key = epi_key<DROP>(e);
      bf16x8 x0[8], x1[8];  // residual / aux segments of both passes, loaded before any store
#pragma unroll
      for (int q = 0; q < 8; ++q) x0[q] = epi_x8(e, M, N, grow(0, q), n0 + lcol(q));
      stage(0);
      G256_STEP(16);
#pragma unroll
      for (int q = 0; q < 8; ++q) x1[q] = epi_x8(e, M, N, grow(1, q), n0 + lcol(q));
      gather_wait();
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v[8];
        fetch(q, v);
        const long gr = grow(0, q), gc = n0 + lcol(q);
        if (gr < M && gc < N) epi8x<ACT, DROP>(e, C, ldc, N, gr, gc, v, bq[q % CPI], x0[q], key);
      }
      G256_STEP(17);
      bar_raw();  // every wave's pass-0 reads are consumed (used above) before pass 1 overwrites LDS
      G256_STEP(18);
      stage(1);
      G256_STEP(19);
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float v[8];
        fetch(q, v);
        const long gr = grow(1, q), gc = n0 + lcol(q);
        if (gr < M && gc < N) epi8x<ACT, DROP>(e, C, ldc, N, gr, gc, v, bq[q % CPI], x1[q], key);
      }
      return;
    }
  }
  if (regepi) {
    if constexpr (MI == 8 && STG) {
      if (stage) {
        // group 0 stages into the buffer NOT holding the last K-tile (its last reads were >= 2 phases
        // ago), group 1 into the last K-tile's buffer (every read of it returned by the last barrier)
        const int buf = wr == 0 ? (nk & 1) : ((nk - 1) & 1);
        char* stg = smem + buf * BUF_BYTES + wc * 16384;
        stage_epilogue<ACT, DROP, STG == 2>(acc, e, C, ldc, M, N, m0 + wr * HR, n0 + wc * 64, lane, stg);
        return;
      }
    }
    reg_epilogue<ACT, DROP, MI>(acc, e, C, ldc, M, N, m0 + wr * HR, n0 + wc * 64, lane);
    return;
  }
  if constexpr (MI == 8) {  // short tiles launch only with the register epilogue (launch_bf16_256)
  if (wr == 0) bar_raw();  // re-align the groups
  bar_raw();

  if (do_rs) {
    float* dst = ksplit > 1 ? ws + (long)ksplit * M * N + (long)split * M : rowsum;
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
  const bool gather = ksplit == 1 && epi_gatherable(e);
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
      if (ksplit > 1) {
        f32x4* o = (f32x4*)(ws + ((long)split * M + gr) * N + gc);
        o[0] = lo;
        o[1] = hi;
        continue;
      }
      float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      epi_row8<ACT, DROP>(e, C, ldc, N, gr, gc, v);
    }
    __builtin_amdgcn_wave_barrier();
  }
  }
}

// ------------------------------------------------------------------------------------------------
// Persistent form of gemm256_kernel for multi-round NT grids (K-contig A and B, bf16 out, gathered
// epilogue, an even number of 64-deep K-tiles): one workgroup per CU walks its tiles v, v + G, ...
// (the same XCD-grouped order as the one-tile grid). Between two tiles the next tile's first K-tile
// (buffer 0, free since K-tile nk-2) is DMA'd while this tile's epilogue runs -- its operand loads
// return, the DMA goes out, then the stores -- with the epilogue staged through buffer 1 in two
// 64-row passes. What it removes per tile after a workgroup's first: the ~2 us prologue (first
// K-tile from L2 / HBM) and the dispatch gap of a new workgroup. Same K loop, same per-element MFMA
// order and epilogue arithmetic as gemm256_kernel: bit-identical outputs.
// ------------------------------------------------------------------------------------------------
template <int ACT, bool DROP, int STG>
__global__ __launch_bounds__(512) void gemm256p_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, void* C,
                                                       long M, long N, long K, long lda, long ldb, long ldc,
                                                       int a_bytes, int b_bytes, Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int MI = 8, HR = 128, IH0 = 4, L = MIT_K_CONTIG;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 2, wc = wid & 3;
  const int nbn = (int)((N + B2 - 1) / B2), nbm = (int)((M + 255) / 256);
  const int ntiles = nbn * nbm, G = (int)gridDim.x;
  auto tile_of = [&](int v, long& m0, long& n0) {
    const int bid = xcd_remap(v, ntiles);
    const int GROUP = MIT_G256_GROUP;
    const int first_m = (bid / (GROUP * nbn)) * GROUP;
    const int gsize = min(nbm - first_m, GROUP);
    m0 = (long)(first_m + (bid % (GROUP * nbn)) % gsize) * 256;
    n0 = (long)((bid % (GROUP * nbn)) / gsize) * B2;
  };
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);
  const int nk = (int)((K + BK - 1) / BK), klen = (int)K;
  int v = blockIdx.x;
  long m0, n0;
  tile_of(v, m0, n0);
  DmaPlan<L, HR> pa;
  DmaPlan<L> pb;
  pa.init(lda, M, m0, 0, wid, lane);
  pb.init(ldb, N, n0, 0, wid, lane);
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
  f32x4 acc[MI][4];
  bf16x8 af[IH0][2], blo[2][2], bhi[2][2];
  auto read_a = [&](int buf, int ih) {
    const char* base = smem + buf * BUF_BYTES + wr * HALF_BYTES;
#pragma unroll
    for (int i = 0; i < IH0; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) af[i][kk] = frag<L>(base, (ih * IH0 + i) * 16, kk, lane);
  };
  auto read_b = [&](int buf, int jh, bf16x8 (&bf)[2][2]) {
    const char* base = smem + buf * BUF_BYTES + (2 + (wc >> 1)) * HALF_BYTES;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) bf[j][kk] = frag<L>(base, (wc & 1) * 64 + jh * 32 + j * 16, kk, lane);
  };
  auto mma = [&](int ih, int jh, bf16x8 (&bf)[2][2]) {
    if (MIT_G256_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < IH0; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ih * IH0 + i][jh * 2 + j] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j][kk], af[i][kk], acc[ih * IH0 + i][jh * 2 + j], 0, 0, 0);
    if (MIT_G256_PRIO) __builtin_amdgcn_s_setprio(0);
  };

  // first tile's prologue: K-tile 0 (all four halves) and B0 of K-tile 1
  issue(0, 0, 0);
  issue(0, 1, 0);
  issue(1, 0, 0);
  issue(1, 1, 0);
  wait_dma(issue(1, 0, 1));
  bar_raw();
  if (wr == 1) bar_raw();  // stagger: group 1 runs one barrier behind group 0
  for (;;) {
#pragma unroll
    for (int i = 0; i < MI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the K loop of gemm256_kernel (MIT_G256_PH4, early A1 DMA)
    for (int t = 0; t < nk; t += 2) {
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

      read_a(1, 0);
      read_b(1, 0, blo);
      issue(1, 1, t + 2);
      read_b(1, 1, bhi);
      issue(0, 0, t + 2);
      issue(0, 1, t + 2);
      bar_raw();
      mma(0, 0, blo);
      mma(0, 1, bhi);
      bar_raw();

      read_a(1, 1);
      wait_dma(issue(1, 0, t + 3));
      // the epilogue stages into buffer 1 (the last K-tile's): its reads must have returned
      if (t + 2 >= nk) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar_raw();
      mma(1, 1, bhi);
      mma(1, 0, blo);
      if (!(wr == 1 && t + 2 >= nk)) bar_raw();  // the lagging group skips the last barrier
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int vn = v + G;
    const bool more = vn < ntiles;
    long m1 = 0, n1 = 0;
    if (more) {
      tile_of(vn, m1, n1);
      pa.init(lda, M, m1, 0, wid, lane);
      pb.init(ldb, N, n1, 0, wid, lane);
    }
    auto next_k0 = [&]() {  // the next tile's K-tile 0 into buffer 0 (last read at K-tile nk - 2)
      if (more) {
        issue(0, 0, 0);
        issue(0, 1, 0);
        issue(1, 0, 0);
        issue(1, 1, 0);
      }
    };
    // an opaque copy of the lane id: the epilogue's addresses are loop-invariant, and hoisted out of
    // the tile loop they spilled (and their scratch reloads then waited behind the tile's stores)
    int ln = lane;
    asm volatile("" : "+v"(ln));
    stage_epilogue<ACT, DROP, STG == 2, 2>(acc, e, C, ldc, M, N, m0 + wr * HR, n0 + wc * 64, ln,
                                           smem + BUF_BYTES + wid * 8192, next_k0);
    if (!more) break;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar_raw();  // every wave's image reads of buffer 1 returned: B0 of K-tile 1 may land there
    wait_dma(issue(1, 0, 1));
    bar_raw();
    if (wr == 1) bar_raw();
    v = vn;
    m0 = m1;
    n0 = n1;
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA kernel, 256x128 block tile, TWO workgroups per CU (NT: both operands K-contig; the
// encoder's GEMMs and the decoder's kv_all / fc_out).
//
// Why: the 256x256 kernel's epilogue is a per-CU store stream (~11 B per clock per CU: a K = 768
// tile spends 6-10 us of its 25-29 us writing 128 KiB, tools/g256_stamps.py), and with one
// workgroup per CU nothing computes meanwhile. Here each CU holds two 4-wave workgroups (72 KiB LDS,
// <= 256 VGPRs each), so one workgroup's prologue / epilogue runs beside the other's K loop and the
// ping-pong of the 256 kernel's wave groups comes from the two workgroups instead of a schedule.
//
// 4 waves as 2 (M) x 2 (N), 128x64 each (8x4 accumulators, C^T blocks -> register epilogue). K in
// steps of 32: three LDS stages of 24 KiB (A 256 x 32, B 128 x 32, 64-B rows), filled by LDS-DMA
// two steps ahead (6 pieces per wave per stage), one barrier per step:
//   wait vmcnt(6) (this wave's pieces of stage t landed, stage t+1's in flight) -> barrier (every
//   wave's pieces of t landed; every wave's reads of step t-1 done) -> DMA stage t+2 into the slot of
//   t-1 -> fragment reads of t -> 32 MFMAs.
// ------------------------------------------------------------------------------------------------
constexpr int T2_BK = 32;
constexpr int T2_A_BYTES = 256 * T2_BK * 2;          // 16 KiB
constexpr int T2_STAGE = T2_A_BYTES + 128 * T2_BK * 2;  // + B 8 KiB = 24 KiB
constexpr int T2_NST = 3;
constexpr int T2_SMEM = T2_NST * T2_STAGE;            // 72 KiB: two workgroups per CU
#ifndef MIT_GT_GROUP
#define MIT_GT_GROUP 4
#endif
// 16-B chunk c (0..3) of row r in a [rows][32] bf16 image (64-B rows). The chunks of rows 8-15 of
// every 16-row fragment are XOR 3: the four lane groups of a ds_read_b128 ({0-3,12-15,20-27}, ...)
// then each cover all 64 banks once (conflict-free fragment reads).
__device__ __forceinline__ int t2off(int r, int c) { return r * 64 + ((c ^ (((r >> 3) & 1) * 3)) << 4); }

template <int ACT, bool DROP>
__global__ __launch_bounds__(256, 2) void gemm_tall_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                           void* C, long M, long N, long K, long lda, long ldb, long ldc,
                                                           int a_bytes, int b_bytes, Epi e) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wr = wid >> 1, wc = wid & 1;
  const int nbn = (int)((N + 127) / 128), nbm = (int)((M + 255) / 256);
  const int ntiles = nbn * nbm;
  const int bid = xcd_remap(blockIdx.x, ntiles);
  const int GROUP = MIT_GT_GROUP;  // row groups of GROUP M-tiles walk the N-tiles together (L2 reuse)
  const int group_id = bid / (GROUP * nbn);
  const int first_m = group_id * GROUP;
  const int gsize = min(nbm - first_m, GROUP);
  const int bm = first_m + (bid % (GROUP * nbn)) % gsize;
  const int bn = (bid % (GROUP * nbn)) / gsize;
  const long m0 = (long)bm * 256, n0 = (long)bn * 128;

  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc((void*)A, (short)0, a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc((void*)B, (short)0, b_bytes, 0x00020000);

  // LDS-DMA plan: piece p (1 KiB = 16 rows x 64 B) of the A image is issued by wave p / 4, of the B
  // image by wave p / 2; lane l fills row 16p + l / 4, physical chunk l % 4 = logical chunk c ^ swz
  uint32_t abase[4], bbase[2];
  int akc[4], bkc[2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int r = (wid * 4 + j) * 16 + (lane >> 2), c = (lane & 3) ^ (((r >> 3) & 1) * 3);
    akc[j] = c * 8;
    abase[j] = m0 + r < M ? (uint32_t)(((m0 + r) * lda + c * 8) * 2) : OOB;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r = (wid * 2 + j) * 16 + (lane >> 2), c = (lane & 3) ^ (((r >> 3) & 1) * 3);
    bkc[j] = c * 8;
    bbase[j] = n0 + r < N ? (uint32_t)(((n0 + r) * ldb + c * 8) * 2) : OOB;
  }
  const int nk = (int)((K + T2_BK - 1) / T2_BK);
  auto issue = [&](int t) {
    char* st = smem + (t % T2_NST) * T2_STAGE;
    const uint32_t koff = (uint32_t)t * (T2_BK * 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t boff = (t * T2_BK + akc[j] < K) ? abase[j] + koff : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(st + (wid * 4 + j) * 1024),
                                               16, boff, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const uint32_t boff = (t * T2_BK + bkc[j] < K) ? bbase[j] + koff : OOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(st + T2_A_BYTES + (wid * 2 + j) * 1024), 16, boff, 0, 0, 0);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fragment read offsets inside a stage: A row block i of this wave, B column block j
  const int aoff = t2off(wr * 128 + (lane & 15), lane >> 4);
  const int boff0 = T2_A_BYTES + t2off(wc * 64 + (lane & 15), lane >> 4);

  // Software pipeline: the fragments of step t+1 are read while step t's MFMAs run (two register
  // sets, the loop unrolled by two so both are statically named). Step t: wait for this wave's
  // pieces of stage t+1 and its own reads of stage t -> barrier (stage t+1 visible to all; every
  // wave's stage-t fragments are in registers, so slot t is free) -> DMA stage t+3 into slot t ->
  // read stage t+1 -> MFMAs of t. Three slots: t+1 (read now), t+2 (in flight), t+3 (issued now).
  auto wait_next = [&](int t) {  // this wave's pieces of stage t+1 landed (t+2, if any, may fly)
    if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(6) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  };
  auto read = [&](int t, bf16x8 (&af)[8], bf16x8 (&bfr)[4]) {
    const char* st = smem + (t % T2_NST) * T2_STAGE;
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = __builtin_bit_cast(bf16x8, *(const u32x4*)(st + boff0 + j * 1024));
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = __builtin_bit_cast(bf16x8, *(const u32x4*)(st + aoff + i * 1024));
  };
  auto mma = [&](const bf16x8 (&af)[8], const bf16x8 (&bfr)[4]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
  };
  auto step = [&](int t, const bf16x8 (&ac)[8], const bf16x8 (&bc)[4], bf16x8 (&an)[8], bf16x8 (&bn)[4]) {
    if (t + 1 < nk) {
      wait_next(t);
      bar_raw();
      if (t + 3 < nk) issue(t + 3);
      read(t + 1, an, bn);
    }
    mma(ac, bc);
  };

  issue(0);
  if (nk > 1) issue(1);
  if (nk > 2) issue(2);
  if (nk > 2) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (nk > 1) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  bar_raw();
  bf16x8 a0[8], b0[4], a1[8], b1[4];
  read(0, a0, b0);
  for (int t = 0; t < nk; t += 2) {
    step(t, a0, b0, a1, b1);
    if (t + 1 < nk) step(t + 1, a1, b1, a0, b0);
  }
  reg_epilogue<ACT, DROP, 8>(acc, e, C, ldc, M, N, m0 + wr * 128, n0 + wc * 64, lane);
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
int g_split_target = -1;  // blocks the split aims for (env MIT_SPLITK_TARGET; 128 beat 512 / 256 / 64 by 0.8-4 % in the step: fewer fp32 slabs)
int g_split_target_dx = -1;  // the same for K-contig A (data gradients on the main stream; env MIT_SPLITK_TARGET_DX)
int splitk_plan(long M, long N, long K, long* kchunk, int a_layout = MIT_MN_CONTIG) {
  const long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  *kchunk = K;
  if (g_split_target < 0) g_split_target = getenv("MIT_SPLITK_TARGET") ? atoi(getenv("MIT_SPLITK_TARGET")) : 128;
  if (g_split_target_dx < 0)
    g_split_target_dx = getenv("MIT_SPLITK_TARGET_DX") ? atoi(getenv("MIT_SPLITK_TARGET_DX")) : 256;  // 256 beat 128 by 0.4 % in the step (dX fc_out: K = 10000 on 128 tiles)
  if (tiles >= 256 || K < 1024 || N % 8) return 1;
  const long target = a_layout == MIT_K_CONTIG ? g_split_target_dx : 256;  // 256 beat 128 by 0.4 % in the step (dX fc_out: K = 10000 on 128 tiles)
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

// split-K with the in-launch combine (any epilogue): grids of <= 128 output tiles -- the d_model =
// 512 decoder GEMMs (M = B*T rows, N = 512: 128 tiles on 256 CUs) -- cut K so that about one block
// runs per CU. Per-block latency, not throughput, bounds these.
int fused_plan(long M, long N, long K, long* kchunk) {
  const long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  *kchunk = K;
  if (tiles > 128 || N % 8) return 1;
  long s = min(256 / tiles, K / 768);  // the combine costs ~4-5 us: only slices >= 12 K-tiles pay
  s = min(s, 8L);
  if (s < 2) return 1;
  long kc = (K + s - 1) / s;
  kc = (kc + BK - 1) / BK * BK;
  *kchunk = kc;
  return (int)((K + kc - 1) / kc);
}
long fused_ws_bytes(long M, long N, int s) {
  const long tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  return s > 1 ? 4096 + 4L * s * tiles * BM * BN : 0;
}

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
  bool fused = false;
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
int g_w8 = -1;  // 8-wave 128 kernel: 0 = off, 1 = grids of <= one block per CU, 2 = always (env MIT_GEMM_W8)
int waves8() {
  if (g_w8 < 0) g_w8 = getenv("MIT_GEMM_W8") ? atoi(getenv("MIT_GEMM_W8")) : 2;
  return g_w8;
}

template <int AL, int BL, int ACT, bool DROP>
void launch_bf16(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, const Split& sp, hipStream_t s) {
  const int ksplit = sp.ks;
  const long kchunk = sp.ks > 1 ? sp.kchunk : g->K;
  float* ws = g->workspace ? (float*)((char*)g->workspace + WS_HDR) : nullptr;
  int* cnt = sp.fused ? (int*)g->workspace : nullptr;
  const long wsb = g->workspace ? max(0L, min(g->workspace_bytes - WS_HDR, (long)INT32_MAX)) : 0;
  const long nbm = (g->M + BM - 1) / BM, nbn = (g->N + BN - 1) / BN;
  const long nblk = nbm * nbn * ksplit;
  static bool attr = false;
  if (!attr) {
    set_lds(gemm_bf16_kernel<AL, BL, ACT, DROP, 2>, smem_bytes(2));
    set_lds(gemm_bf16_kernel<AL, BL, ACT, DROP, 2, 8>, smem_bytes(2));
    attr = true;
  }
  // grids of at most one block per CU: 8 waves per block (2 per SIMD, each issuing half the LDS-DMA
  // pieces of a K-tile) -- with one 4-wave block per CU every K-tile's 8 DMA pieces per wave sit
  // serially in front of its 32 MFMAs
  if (waves8() && (waves8() == 2 || nblk <= num_cus())) {
    hipLaunchKernelGGL((gemm_bf16_kernel<AL, BL, ACT, DROP, 2, 8>), dim3((unsigned)nblk), dim3(512), smem_bytes(2), s,
                       (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                       b_bytes, e, ksplit, kchunk, ws, g->rowsum, cnt, wsb);
    return;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<AL, BL, ACT, DROP, 2>), dim3((unsigned)nblk), dim3(256), smem_bytes(2), s,
                     (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                     b_bytes, e, ksplit, kchunk, ws, g->rowsum, cnt, wsb);
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

int gemm_variant();
int g_persist = -1;  // mit_gemm_set_persist; -1 = from env on first use
// persistent 256 kernel (gemm256p_kernel): NT, gathered bf16 epilogue, more tiles than CUs, an even
// K-tile count. Opt-in (MIT_G256_PERSIST=1; variant 8 forces the one-tile grid): alone it is 0-5 %
// faster on the multi-round shapes (kv_all 93.1 -> 88.7 us, fc1+GELU 89.0 -> 86.9, CLIP-L o+res
// 100.6 -> 103.9), but in the train step it is 9 % SLOWER (11605-11655 vs 12763-12806 pairs/s,
// interleaved): a grid that holds every CU until its last tile starves the decoder's concurrent
// kernels, which the one-tile grid lets in between tiles.
template <int ACT, bool DROP>
bool launch_256p(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, hipStream_t s) {
  if (g_persist < 0) g_persist = getenv("MIT_G256_PERSIST") ? atoi(getenv("MIT_G256_PERSIST")) != 0 : 0;
  const int on = g_persist;
  const long tiles = ((g->M + 255) / 256) * ((g->N + B2 - 1) / B2), nk = (g->K + BK - 1) / BK;
  const long G = (min((long)num_cus(), tiles) / 8) * 8;
  if (!on || e.out_f32 || !epi_gatherable(e) || nk % 2 || G < 8 || tiles <= G) return false;
  const bool ops = e.res || e.aux;
  if (ops && ACT != MIT_ACT_NONE) return false;
  static bool attr = false;
  if (!attr) {
    set_lds(gemm256p_kernel<ACT, DROP, 1>, SMEM2_BYTES);
    if constexpr (ACT == MIT_ACT_NONE) set_lds(gemm256p_kernel<ACT, DROP, 2>, SMEM2_BYTES);
    attr = true;
  }
  if constexpr (ACT == MIT_ACT_NONE) {
    if (ops) {
      hipLaunchKernelGGL((gemm256p_kernel<ACT, DROP, 2>), dim3((unsigned)G), dim3(512), SMEM2_BYTES, s,
                         (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                         b_bytes, e);
      return true;
    }
  }
  hipLaunchKernelGGL((gemm256p_kernel<ACT, DROP, 1>), dim3((unsigned)G), dim3(512), SMEM2_BYTES, s, (const bf16*)g->A,
                     (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e);
  return true;
}

template <int AL, int BL, int ACT, bool DROP, int MI>
void launch_256_mi(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, hipStream_t s) {
  if constexpr (MI == 8 && AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {
    if (gemm_variant() != 8 && launch_256p<ACT, DROP>(g, e, a_bytes, b_bytes, s)) return;
  }
  const long nbm = (g->M + 32 * MI - 1) / (32 * MI), nbn = (g->N + B2 - 1) / B2;
  static bool attr = false;
  if (!attr) {
    set_lds(gemm256_kernel<AL, BL, ACT, DROP, MI>, SMEM2_BYTES);
    if constexpr (MI == 8 && AL == MIT_K_CONTIG) {
      set_lds(gemm256_kernel<AL, BL, ACT, DROP, MI, 1>, SMEM2_BYTES);
      if constexpr (ACT == MIT_ACT_NONE) set_lds(gemm256_kernel<AL, BL, ACT, DROP, MI, 2>, SMEM2_BYTES);
    }
    attr = true;
  }
  if constexpr (MI == 8 && AL == MIT_K_CONTIG && MIT_G256_EPI_STAGE) {
    // MIT_G256_STAGE: 0 = register epilogue everywhere, 1 = staged without operands only, 2 = staged
    // everywhere it applies (default)
    static const int on = getenv("MIT_G256_STAGE") ? atoi(getenv("MIT_G256_STAGE")) : 2;
    const bool ops = e.res || e.aux;
    if (on && epi_gatherable(e) && !e.out_f32 && (!ops || on == 2)) {
      if constexpr (ACT == MIT_ACT_NONE) {
        if (ops) {
          hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, MI, 2>), dim3((unsigned)(nbm * nbn)), dim3(512),
                             SMEM2_BYTES, s, (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda,
                             g->ldb, g->ldc, a_bytes, b_bytes, e, 1, g->K, (float*)g->workspace, g->rowsum);
          return;
        }
      }
      if (!ops) {
        hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, MI, 1>), dim3((unsigned)(nbm * nbn)), dim3(512),
                           SMEM2_BYTES, s, (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb,
                           g->ldc, a_bytes, b_bytes, e, 1, g->K, (float*)g->workspace, g->rowsum);
        return;
      }
    }
  }
  hipLaunchKernelGGL((gemm256_kernel<AL, BL, ACT, DROP, MI>), dim3((unsigned)(nbm * nbn)), dim3(512), SMEM2_BYTES, s,
                     (const bf16*)g->A, (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes,
                     b_bytes, e, 1, g->K, (float*)g->workspace, g->rowsum);
}

// 0 = pick per shape, 1 = always the 128x128 kernel, 2 = the 256x256 kernel wherever it has an
// instance for the epilogue, 3 = the register-streaming kernel where it applies, 5 / 6 = the
// 256-column kernel with 160 / 192-row tiles where it applies (tuning / tests)
int g_variant = -1;

// rows per wave of the 256-column kernel: 16 x (8, 6 or 5). Short tiles need K-contig A and the
// register epilogue; among those the fewest (rounds of one tile per CU) x (per-tile time) wins, the
// per-tile time modelled as a fixed part + K-steps at a per-row-count rate (tools/gemm_bench.py)
int gemm_variant();
int tile_mi(const mit_gemm_args* g, const Epi& e) {
  static const int forced = getenv("MIT_G256_MI") ? atoi(getenv("MIT_G256_MI")) : 0;
  const bool shortok = g->a_layout == MIT_K_CONTIG && epi_gatherable(e);
  if (!shortok) return 8;
  const int v = gemm_variant();
  if (v == 5 || v == 6) return v;
  if (forced == 5 || forced == 6) return forced;
  // off by default: in the train step the encoder GEMMs run beside the decoder's kernels, and the
  // 150-tile o-proj / fc2 grids leave 106 CUs to them -- 160-row tiles (237 blocks) measured 7 %
  // slower end to end (11353-11414 vs 12205-12212 pairs/s interleaved) though 1-2 % faster alone.
  // MIT_G256_MI=-1 enables the per-shape model below.
  if (forced != -1) return 8;
  const double cus = (double)num_cus(), nk = (double)((g->K + BK - 1) / BK), nbn = (double)((g->N + B2 - 1) / B2);
  // per-tile K-step cost relative to MI = 8, measured on equal-round shapes (enc o / fc2, cfg3 o / fc2:
  // 160-row tiles 0.98-0.99x the time of 256-row ones, 192-row 1.02-1.04x): the chip holds a lower
  // clock when more CUs run MFMA loops, so shorter tiles pay only where they keep the round count
  // (profiles/r02_gemm_short_tiles.txt)
  const double FIX = 6.0, STEP = 1.54;  // us per tile, us per 64-deep K-step (MI = 8)
  const int mis[3] = {8, 6, 5};
  const double rate[3] = {1.0, 1.03, 0.975};
  int best = 8;
  double tbest = 1e30;
  for (int i = 0; i < 3; ++i) {
    const double tiles = (double)((g->M + 32 * mis[i] - 1) / (32 * mis[i])) * nbn;
    const double t = std::ceil(tiles / cus) * (FIX + nk * STEP * rate[i]);
    if (t < tbest * 0.995) {
      tbest = t;
      best = mis[i];
    }
  }
  return best;
}

template <int ACT, bool DROP>
void launch_tall(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    set_lds(gemm_tall_kernel<ACT, DROP>, T2_SMEM);
    attr = true;
  }
  const long nb = ((g->M + 255) / 256) * ((g->N + 127) / 128);
  hipLaunchKernelGGL((gemm_tall_kernel<ACT, DROP>), dim3((unsigned)nb), dim3(256), T2_SMEM, s, (const bf16*)g->A,
                     (const bf16*)g->B, g->C, g->M, g->N, g->K, g->lda, g->ldb, g->ldc, a_bytes, b_bytes, e);
}

// the two-workgroup 256x128 kernel replaces the 256x256 one for NT GEMMs with a register
// (gathered) epilogue: MIT_GEMM_TALL=0 keeps the 256x256 kernel; variant 7 forces it (tests)
bool use_tall(const mit_gemm_args* g, const Epi& e) {
  static int on = -1;
  if (on < 0) on = getenv("MIT_GEMM_TALL") ? atoi(getenv("MIT_GEMM_TALL")) : 0;
  if (g->a_layout != MIT_K_CONTIG || g->b_layout != MIT_K_CONTIG || !epi_gatherable(e)) return false;
  const int v = gemm_variant();
  return v == 7 || (v == 0 && on);
}

template <int AL, int BL, int ACT, bool DROP>
void launch_bf16_256(const mit_gemm_args* g, const Epi& e, int a_bytes, int b_bytes, hipStream_t s) {
  if constexpr (AL == MIT_K_CONTIG && BL == MIT_K_CONTIG) {
    if (use_tall(g, e)) return launch_tall<ACT, DROP>(g, e, a_bytes, b_bytes, s);
  }
  if constexpr (AL == MIT_K_CONTIG) {
    switch (tile_mi(g, e)) {
      case 6: return launch_256_mi<AL, BL, ACT, DROP, 6>(g, e, a_bytes, b_bytes, s);
      case 5: return launch_256_mi<AL, BL, ACT, DROP, 5>(g, e, a_bytes, b_bytes, s);
      default: break;
    }
  }
  launch_256_mi<AL, BL, ACT, DROP, 8>(g, e, a_bytes, b_bytes, s);
}
int gemm_variant() {
  if (g_variant < 0) g_variant = getenv("MIT_GEMM_VARIANT") ? atoi(getenv("MIT_GEMM_VARIANT")) : 0;
  return g_variant;
}

// register-streaming kernel (gemm_rs_kernel): the decode step's B-row GEMMs (M <= 256) with a short
// K and N <= 2048 -- 7.2 vs 9.9 us per launch on 256 x {512, 1536, 2048} x 512. Everywhere else it
// loses: each wave streams its own A and B fragments from L2 (8 FLOP per L2 byte vs 64 for the 128
// kernel's LDS tiles): 2.5-3x slower on the M = 4032 decoder shapes, 2x on the decode fc_out
// (tools/blas_reference.py, MIT_GEMM_RS=0 turns it off)
int g_rs = -1;
bool use_rs(const mit_gemm_args* g) {
  if (g_rs < 0) g_rs = getenv("MIT_GEMM_RS") ? atoi(getenv("MIT_GEMM_RS")) : 1;
  if (g->a_layout != MIT_K_CONTIG || g->b_layout != MIT_K_CONTIG || g->rowsum) return false;
  const int v = gemm_variant();
  if (v == 3) return true;
  if (!g_rs || v != 0) return false;
  return g->M <= 256 && g->N <= 2048 && g->K <= 1024;
}

// Occupancy-quantised cost model: the 128x128 kernel runs 2 blocks per CU, the 256x256 kernel 1;
// a "round" fills every slot once, and a round of the 256 kernel moves 4 tiles' worth of 128x128
// work per CU-slot at REL256 x the 128 kernel's per-FLOP speed (tools/gemm_bench.py).
bool use_256(long M, long N, long K, int a_layout) {
  const int v = gemm_variant();
  if (v == 1) return false;
  if (v == 2 || v == 5 || v == 6 || v == 7 || v == 8) return true;
  // the MN-contig-A instances (weight gradients) exceed 256 VGPRs and spill: 128 kernel (+ split-K)
  if (a_layout != MIT_K_CONTIG) return false;
  if (M < 256 || N < 256 || K < 128) return false;
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

int g_fused = -1;  // in-launch split-K combine: -1 = from env on first use

Split plan_split(const mit_gemm_args* g) {
  Split p;
  p.kchunk = g->K;
  if (!g->workspace || !al16(g->workspace)) return p;
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
  // off by default: in the train step the 128-block decoder GEMMs share the chip with the encoder
  // prefetch and weight-gradient streams, and splitting them measured 0.6 % slower end to end
  // (9645 vs 9700 pairs/s) though 8-18 % faster alone. MIT_GEMM_FUSED_SPLIT=1 or
  // mit_gemm_set_fused_split(1) enables it.
  if (g_fused < 0) g_fused = getenv("MIT_GEMM_FUSED_SPLIT") && atoi(getenv("MIT_GEMM_FUSED_SPLIT")) != 0;
  // long-K data gradients only (K-contig A, K >= MIT_GEMM_FUSED_MINK; 0 = off): the decoder's
  // linear1 / self in_proj dX (K = d_ff / 3 d on 128 tiles) run 24-32 K-steps per block. Measured
  // -1.0 % (1536) / -0.3 % (2048) in the step (interleaved, 3 rounds): off
  static long fused_mink = -1;
  if (fused_mink < 0) fused_mink = getenv("MIT_GEMM_FUSED_MINK") ? atol(getenv("MIT_GEMM_FUSED_MINK")) : 0;
  const bool fused = g_fused || (fused_mink > 0 && g->K >= fused_mink && g->a_layout == MIT_K_CONTIG);
  if (fused && !g->rowsum && !use_256(g->M, g->N, g->K, g->a_layout)) {
    const int s = fused_plan(g->M, g->N, g->K, &kc);
    if (s > 1 && fused_ws_bytes(g->M, g->N, s) <= g->workspace_bytes) {
      p.ks = s;
      p.kchunk = kc;
      p.fused = true;
    }
  }
  return p;
}

}  // namespace

extern "C" int mit_gemm_set_variant(int v) {
  MIT_CHECK_ARG((v >= 0 && v <= 3) || (v >= 5 && v <= 8), "mit_gemm_set_variant: %d not in {0,1,2,3,5,6,7,8}", v);
  g_variant = v;
  return MIT_OK;
}

extern "C" int mit_gemm_set_persist(int on) {
  MIT_CHECK_ARG(on == 0 || on == 1, "mit_gemm_set_persist: %d not in {0,1}", on);
  g_persist = on;
  return MIT_OK;
}

extern "C" int mit_gemm_set_fused_split(int on) {
  MIT_CHECK_ARG(on == 0 || on == 1, "mit_gemm_set_fused_split: %d not in {0,1}", on);
  g_fused = on;
  return MIT_OK;
}

extern "C" long mit_gemm_workspace_bytes(long M, long N, long K) {
  long kc;
  const long a = max(splitk_ws_bytes(M, N, splitk_plan(M, N, K, &kc)),
                     splitk_ws_bytes(M, N, splitk_plan(M, N, K, &kc, MIT_K_CONTIG)));
  const long b = fused_ws_bytes(M, N, fused_plan(M, N, K, &kc));
  return a > b ? a : b;
}

extern "C" int mit_gemm_plan(const mit_gemm_args* g, int* ksplit) {
  if (ksplit) *ksplit = 1;
  if (!g || g->M <= 0 || g->N <= 0) return 0;
  if (g->dtype != MIT_BF16) return 64;
  const Split sp = plan_split(g);
  if (ksplit) *ksplit = sp.ks;
  if (sp.ks == 1 && use_rs(g)) return 65;  // the 64x64 register-streaming kernel
  const bool big = sp.ks == 1 && use_256(g->M, g->N, g->K, g->a_layout) && epi_kind(g) != EK_GENERIC &&
                   (g->act == MIT_ACT_NONE || (!g->residual && !g->aux));
  return big ? 256 : 128;
}

extern "C" int mit_gemm(const mit_gemm_args* g, void* stream) {
  MIT_CHECK_ARG(g != nullptr, "mit_gemm: null args");
  MIT_RECORD([c = *g, stream]() { return mit_gemm(&c, stream); });
  MIT_CHECK_ARG(g->dtype == MIT_F32 || g->dtype == MIT_BF16, "mit_gemm: bad dtype %d", g->dtype);
  MIT_CHECK_ARG(g->M >= 0 && g->N >= 0 && g->K >= 0, "mit_gemm: negative extent");
  MIT_CHECK_ARG(g->A && g->B && g->C, "mit_gemm: null operand");
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
    const Split sp = plan_split(g);
    const bool big = sp.ks == 1 && use_256(g->M, g->N, g->K, g->a_layout);
    if (g->a_layout == 0 && g->b_layout == 0) launch_layout<0, 0>(g, e, ab, bb, sp, big, s);
    else if (g->a_layout == 0 && g->b_layout == 1) launch_layout<0, 1>(g, e, ab, bb, sp, big, s);
    else if (g->a_layout == 1 && g->b_layout == 0) launch_layout<1, 0>(g, e, ab, bb, sp, big, s);
    else launch_layout<1, 1>(g, e, ab, bb, sp, big, s);
    if (sp.ks > 1 && !sp.fused) {
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
// combine cost more than the shorter K loops save once the group fills the chip. Env
// MIT_GROUPED_SPLIT overrides (A/B).
long grouped_split(long tiles) {
  static long forced = -1;
  if (forced < 0) forced = getenv("MIT_GROUPED_SPLIT") ? atol(getenv("MIT_GROUPED_SPLIT")) : 0;
  if (forced > 0) return min(forced, 16L);
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
  static const int grp = getenv("MIT_GROUPED_GROUP") ? atoi(getenv("MIT_GROUPED_GROUP")) : 1;
  ga.group = grp > 0 ? grp : 1;
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

#ifdef MIT_G256_STAMP
// diagnostic build only: copy / clear the gemm256_kernel stamp buffer (tools/g256_stamps.py)
extern "C" int mit_g256_stamps(unsigned long long* host, long n) {
  const long cap = 16384L * G256_SLOTS;
  if (n > cap) n = cap;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g256_stamp), n * 8, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
extern "C" int mit_g256_stamps_clear() {
  static unsigned long long zero[16384 * G256_SLOTS];
  return hipMemcpyToSymbol(HIP_SYMBOL(g256_stamp), zero, sizeof(zero), 0, hipMemcpyHostToDevice) == hipSuccess ? 0 : -1;
}
#endif
