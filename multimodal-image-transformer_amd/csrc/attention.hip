// Scaled-dot-product attention: MFMA kernels for head_dim 64, generic kernels for 16/32/64/128.
//
// Semantics (the reference's SDPA call, torch/nn/functional.py:6615-6633):
//   s_ij = scale * q_i . k_j  (+ -inf where j > i if causal, or key j is PAD)
//   P = softmax_j(s);  O = (P o M) V,  M_ij = dropout multiplier (0 or 1/(1-p)), index
//   ((b*H + h)*Lq + i)*Lk + j;  lse_i = log sum_j exp(s_ij).
// Backward: dV = (P o M)^T dO; dP = (dO V^T) o M; dS = P o (dP - delta), delta_i = dO_i . O_i;
//           dQ = scale * dS K;  dK = scale * dS^T Q.
//
// This file holds two implementations:
//   * *_simple: one query (or key) row per thread, fp32 math, LDS-broadcast K/V tiles. Any dtype.
//     Used for fp32 parity mode and for the decoder backward.
//   * attn_fwd_mfma (bf16): 64-query block per 4-wave workgroup, v_mfma_f32_16x16x32_bf16 for
//     Q K^T and P V with online softmax over 64-key tiles staged in LDS.
#include "common.h"

namespace {

constexpr int D = 64;

struct AttnK {
  const void* q;
  long q_row, q_batch;
  const void* k;
  long k_row, k_batch;
  const void* v;
  long v_row, v_batch;
  void* o;
  long o_row, o_batch;
  float* lse;
  const int64_t* tok;
  long tok_batch;
  int pad;
  int causal;
  float scale;
  const uint64_t* seed;
  uint32_t site;
  uint32_t thresh;
  float dscale;
  int dropout;
};

__device__ __forceinline__ bool key_masked(const AttnK& a, long b, long i, long j) {
  if (a.causal && j > i) return true;
  if (a.tok && a.tok[b * a.tok_batch + j] == a.pad) return true;
  return false;
}

// ------------------------------------------------------------------------------------------------
// simple forward: one query row per thread, fp32 math, K/V tiles of 64 keys broadcast from LDS.
// Any dtype and any head_dim DH in {16, 32, 64, 128} (the decoder of configs[0] is d128 / 8 heads).
// Scores are evaluated in chunks of KC keys (KC = 16 at DH = 128 keeps q, o and the chunk's scores
// in registers).
// ------------------------------------------------------------------------------------------------
template <typename T, int DH>
__global__ __launch_bounds__(64) void attn_fwd_simple(long H, long Lq, long Lk, AttnK a) {
  constexpr int KC = DH <= 64 ? 64 : 16;
  __shared__ float Ks[64][DH + 1];
  __shared__ float Vs[64][DH + 1];
  const int tid = threadIdx.x;
  const long b = blockIdx.z, h = blockIdx.y, i = (long)blockIdx.x * 64 + tid;
  const bool live = i < Lq;
  const T* Q = (const T*)a.q + b * a.q_batch + h * DH;
  const T* K = (const T*)a.k + b * a.k_batch + h * DH;
  const T* V = (const T*)a.v + b * a.v_batch + h * DH;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const uint64_t rowbase = ((uint64_t)(b * H + h) * (uint64_t)Lq + (uint64_t)i) * (uint64_t)Lk;
  float q[DH], o[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    q[d] = live ? to_f(Q[i * a.q_row + d]) * a.scale : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (long j0 = 0; j0 < Lk; j0 += 64) {
    const int nj = (int)min((long)64, Lk - j0);
    __syncthreads();
    for (int idx = tid; idx < 64 * DH; idx += 64) {
      const int r = idx / DH, c = idx % DH;
      float kv = 0.f, vv = 0.f;
      if (r < nj) {
        kv = to_f(K[(j0 + r) * a.k_row + c]);
        vv = to_f(V[(j0 + r) * a.v_row + c]);
      }
      Ks[r][c] = kv;
      Vs[r][c] = vv;
    }
    __syncthreads();
    if (!live) continue;
    for (int c0 = 0; c0 < 64; c0 += KC) {
      float s[KC];
      float tmax = -INFINITY;
#pragma unroll
      for (int jj = 0; jj < KC; ++jj) {
        float acc = 0.f;
#pragma unroll
        for (int d = 0; d < DH; ++d) acc = fmaf(q[d], Ks[c0 + jj][d], acc);
        const bool msk = (c0 + jj >= nj) || key_masked(a, b, i, j0 + c0 + jj);
        s[jj] = msk ? -INFINITY : acc;
        tmax = fmaxf(tmax, s[jj]);
      }
      const float mnew = fmaxf(m, tmax);
      const float corr = (mnew == -INFINITY) ? 1.f : __expf(m - mnew);
      l *= corr;
#pragma unroll
      for (int d = 0; d < DH; ++d) o[d] *= corr;
#pragma unroll
      for (int jj = 0; jj < KC; ++jj) {
        const float p = (s[jj] == -INFINITY) ? 0.f : __expf(s[jj] - mnew);
        l += p;
        float pd = p;
        if (a.dropout) pd *= drop_mul(key, rowbase + (uint64_t)(j0 + c0 + jj), a.thresh, a.dscale);
        if (pd != 0.f) {
#pragma unroll
          for (int d = 0; d < DH; ++d) o[d] = fmaf(pd, Vs[c0 + jj][d], o[d]);
        }
      }
      m = mnew;
    }
  }
  if (!live) return;
  const float inv = 1.0f / l;  // l == 0 (fully masked row) -> inf * 0 = NaN, as the reference
  T* O = (T*)a.o + b * a.o_batch + i * a.o_row + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) O[d] = from_f<T>(o[d] * inv);
  if (a.lse) a.lse[(b * H + h) * Lq + i] = m + __logf(l);
}

// ------------------------------------------------------------------------------------------------
// simple backward: (1) dQ + delta, thread per query; (2) dK/dV, thread per key. Any head_dim DH.
// ------------------------------------------------------------------------------------------------
struct AttnG {
  const void* dout;
  long do_row, do_batch;
  void* dq;
  long dq_row, dq_batch;
  void* dk;
  long dk_row, dk_batch;
  void* dv;
  long dv_row, dv_batch;
  float* delta;
};

template <typename T, int DH>
__global__ __launch_bounds__(64) void attn_bwd_dq_simple(long H, long Lq, long Lk, AttnK a, AttnG g) {
  __shared__ float Ks[64][DH + 1];
  __shared__ float Vs[64][DH + 1];
  const int tid = threadIdx.x;
  const long b = blockIdx.z, h = blockIdx.y, i = (long)blockIdx.x * 64 + tid;
  const bool live = i < Lq;
  const T* Q = (const T*)a.q + b * a.q_batch + h * DH;
  const T* K = (const T*)a.k + b * a.k_batch + h * DH;
  const T* V = (const T*)a.v + b * a.v_batch + h * DH;
  const T* O = (const T*)a.o + b * a.o_batch + h * DH;
  const T* dO = (const T*)g.dout + b * g.do_batch + h * DH;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const uint64_t rowbase = ((uint64_t)(b * H + h) * (uint64_t)Lq + (uint64_t)i) * (uint64_t)Lk;
  float q[DH], dout[DH], dq[DH];
  float delta = 0.f, lse = 0.f;
  if (live) {
#pragma unroll
    for (int d = 0; d < DH; ++d) {
      q[d] = to_f(Q[i * a.q_row + d]);
      dout[d] = to_f(dO[i * g.do_row + d]);
      delta = fmaf(dout[d], to_f(O[i * a.o_row + d]), delta);
      dq[d] = 0.f;
    }
    lse = a.lse[(b * H + h) * Lq + i];
    g.delta[(b * H + h) * Lq + i] = delta;
  }
  for (long j0 = 0; j0 < Lk; j0 += 64) {
    const int nj = (int)min((long)64, Lk - j0);
    __syncthreads();
    for (int idx = tid; idx < 64 * DH; idx += 64) {
      const int r = idx / DH, c = idx % DH;
      float kv = 0.f, vv = 0.f;
      if (r < nj) {
        kv = to_f(K[(j0 + r) * a.k_row + c]);
        vv = to_f(V[(j0 + r) * a.v_row + c]);
      }
      Ks[r][c] = kv;
      Vs[r][c] = vv;
    }
    __syncthreads();
    if (!live) continue;
    for (int jj = 0; jj < nj; ++jj) {
      if (key_masked(a, b, i, j0 + jj)) continue;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        s = fmaf(q[d], Ks[jj][d], s);
        dp = fmaf(dout[d], Vs[jj][d], dp);
      }
      const float p = __expf(s * a.scale - lse);
      if (a.dropout) dp *= drop_mul(key, rowbase + (uint64_t)(j0 + jj), a.thresh, a.dscale);
      const float ds = p * (dp - delta);
#pragma unroll
      for (int d = 0; d < DH; ++d) dq[d] = fmaf(ds, Ks[jj][d], dq[d]);
    }
  }
  if (!live) return;
  T* DQ = (T*)g.dq + b * g.dq_batch + i * g.dq_row + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) DQ[d] = from_f<T>(dq[d] * a.scale);
}

template <typename T, int DH>
__global__ __launch_bounds__(64) void attn_bwd_dkv_simple(long H, long Lq, long Lk, AttnK a, AttnG g) {
  __shared__ float Kp[64][DH + 1];  // this block's keys, one private row per thread
  __shared__ float Vp[64][DH + 1];
  __shared__ float Qs[64][DH + 1];  // query tile (broadcast reads)
  __shared__ float Ds[64][DH + 1];  // dO tile
  __shared__ float Ls[64], Dl[64];
  const int tid = threadIdx.x;
  const long b = blockIdx.z, h = blockIdx.y, j = (long)blockIdx.x * 64 + tid;
  const bool live = j < Lk;
  const T* Q = (const T*)a.q + b * a.q_batch + h * DH;
  const T* K = (const T*)a.k + b * a.k_batch + h * DH;
  const T* V = (const T*)a.v + b * a.v_batch + h * DH;
  const T* dO = (const T*)g.dout + b * g.do_batch + h * DH;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  for (int idx = tid; idx < 64 * DH; idx += 64) {
    const int r = idx / DH, c = idx % DH;
    const long jj = (long)blockIdx.x * 64 + r;
    Kp[r][c] = jj < Lk ? to_f(K[jj * a.k_row + c]) : 0.f;
    Vp[r][c] = jj < Lk ? to_f(V[jj * a.v_row + c]) : 0.f;
  }
  const bool kpad = live && a.tok && a.tok[b * a.tok_batch + j] == a.pad;
  float dk[DH], dv[DH];
#pragma unroll
  for (int d = 0; d < DH; ++d) dk[d] = dv[d] = 0.f;
  for (long i0 = 0; i0 < Lq; i0 += 64) {
    const int ni = (int)min((long)64, Lq - i0);
    __syncthreads();
    for (int idx = tid; idx < 64 * DH; idx += 64) {
      const int r = idx / DH, c = idx % DH;
      Qs[r][c] = r < ni ? to_f(Q[(i0 + r) * a.q_row + c]) : 0.f;
      Ds[r][c] = r < ni ? to_f(dO[(i0 + r) * g.do_row + c]) : 0.f;
    }
    if (tid < ni) {
      Ls[tid] = a.lse[(b * H + h) * Lq + i0 + tid];
      Dl[tid] = g.delta[(b * H + h) * Lq + i0 + tid];
    }
    __syncthreads();
    if (!live || kpad) continue;
    for (int ii = 0; ii < ni; ++ii) {
      const long i = i0 + ii;
      if (a.causal && j > i) continue;
      float s = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        s = fmaf(Qs[ii][d], Kp[tid][d], s);
        dp = fmaf(Ds[ii][d], Vp[tid][d], dp);
      }
      const float p = __expf(s * a.scale - Ls[ii]);
      const float mul = a.dropout ? drop_mul(key, ((uint64_t)(b * H + h) * (uint64_t)Lq + (uint64_t)i) * (uint64_t)Lk + j,
                                             a.thresh, a.dscale)
                                  : 1.f;
      const float pd = p * mul;
      const float ds = p * (dp * mul - Dl[ii]);
#pragma unroll
      for (int d = 0; d < DH; ++d) {
        dv[d] = fmaf(pd, Ds[ii][d], dv[d]);
        dk[d] = fmaf(ds, Qs[ii][d], dk[d]);
      }
    }
  }
  if (!live) return;
  T* DK = (T*)g.dk + b * g.dk_batch + j * g.dk_row + h * DH;
  T* DV = (T*)g.dv + b * g.dv_batch + j * g.dv_row + h * DH;
#pragma unroll
  for (int d = 0; d < DH; ++d) {
    DK[d] = from_f<T>(dk[d] * a.scale);
    DV[d] = from_f<T>(dv[d]);
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA forward. Workgroup = 4 waves x 16 queries of one (b, h); 64-key K/V tiles, LDS double
// buffer filled by buffer loads (rows past Lk read as zero, then masked).
//   S^T = K Q^T  (A = K tile rows from LDS via ds_read_b128, B = Q fragment held in registers):
//     lane l owns query q = l&15 and keys 16nb + 4(l>>4) + t  -> row softmax = 16 in-lane values
//     + two cross-lane shuffles (xor 16, 32); online max/sum in log2 units.
//   O^T = V^T P^T (A = V^T via ds_read_b64_tr_b16 from the row-major V tile, B = P^T straight
//     from the S^T accumulators, k index permuted consistently: element j<4 -> key 32kk+4g+j,
//     j>=4 -> key 32kk+16+4g+j-4), so P never touches LDS.
// ------------------------------------------------------------------------------------------------
constexpr int AQ = 64;  // queries per workgroup
constexpr int AK = 64;  // keys per tile
constexpr uint32_t A_OOB = 0x80000000u;

__device__ __forceinline__ int koff_k(int r, int c) { return r * 128 + ((c ^ ((r >> 1) & 7)) << 4); }
__device__ __forceinline__ int koff_v(int r, int byte) { return r * 128 + (byte ^ (((r >> 1) & 3) << 5)); }

__global__ __launch_bounds__(256) void attn_fwd_mfma(long H, long Lq, long Lk, AttnK a, int kbytes, int vbytes) {
  __shared__ __attribute__((aligned(16))) char lds[2 * 2 * AK * D * 2];  // 2 stages x (K, V) x 8 KiB
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const long b = blockIdx.z, h = blockIdx.y;
  const long qblk = (long)blockIdx.x * AQ;
  MIT_DASSERT(h < H && qblk < Lq && Lk > 0);
  const long qi = qblk + w * 16 + (lane & 15);
  const bool qlive = qi < Lq;
  const bf16* Kb = (const bf16*)a.k + b * a.k_batch + h * D;
  const bf16* Vb = (const bf16*)a.v + b * a.v_batch + h * D;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)Kb, (short)0, kbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)Vb, (short)0, vbytes, 0x00020000);
  // Q fragments (B operand): Q[qi][32kk + 8g .. +8]
  bf16x8 qf[2];
  {
    const bf16* Qr = (const bf16*)a.q + b * a.q_batch + h * D + (qlive ? qi : 0) * a.q_row;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x4 v = *(const u32x4*)(Qr + kk * 32 + g * 8);
      if (!qlive) v = u32x4{0u, 0u, 0u, 0u};
      qf[kk] = __builtin_bit_cast(bf16x8, v);
    }
  }
  const float sl2 = a.scale * 1.4426950408889634f;  // scores in log2 units
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  // dropout index (bh * Lq + qi) * Lk + key < 2^32 (host-checked): 32-bit, drop_mul32
  const uint32_t rowbase = ((uint32_t)(b * H + h) * (uint32_t)Lq + (uint32_t)qi) * (uint32_t)Lk + (uint32_t)(g * 4);
  const uint32_t kf = key_fold(key);
  const int64_t* tok = a.tok ? a.tok + b * a.tok_batch : nullptr;
  const int qi32 = (int)qi;

  long kend = Lk;
  if (a.causal) kend = min(Lk, min(Lq, qblk + AQ));  // keys beyond the block's last query are masked
  const int nt = (int)((kend + AK - 1) / AK);

  u32x4 kr[2], vr[2];
  auto gload = [&](long j0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 256 * i, r = id >> 3, c = id & 7;
      const long kj = j0 + r;
      const bool ok = kj < Lk;
      kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rk, (int)(ok ? (uint32_t)((kj * a.k_row + c * 8) * 2) : A_OOB), 0, 0));
      vr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rv, (int)(ok ? (uint32_t)((kj * a.v_row + c * 8) * 2) : A_OOB), 0, 0));
    }
  };
  auto lstore = [&](int s) {
    char* Ks = lds + s * (2 * AK * D * 2);
    char* Vs = Ks + AK * D * 2;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int id = tid + 256 * i, r = id >> 3, c = id & 7;
      *(u32x4*)(Ks + koff_k(r, c)) = kr[i];
      *(u32x4*)(Vs + koff_v(r, c * 16)) = vr[i];
    }
  };

  f32x4 ot[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) ot[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;

  if (nt > 0) {
    gload(0);
    lstore(0);
  }
  __syncthreads();
  for (int it = 0; it < nt; ++it) {
    const int cur = it & 1;
    const long j0 = (long)it * AK;
    const bool more = it + 1 < nt;
    if (more) gload(j0 + AK);
    const char* Ks = lds + cur * (2 * AK * D * 2);
    const char* Vs = Ks + AK * D * 2;
    // ---- S^T = K Q^T ----
    f32x4 st[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) st[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const u32x4 kv = *(const u32x4*)(Ks + koff_k(nb * 16 + (lane & 15), kk * 4 + g));
        st[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, kv), qf[kk], st[nb], 0, 0, 0);
      }
    // ---- mask + online softmax (per query = per lane&15) ----
    // the tile's live keys (in range, not PAD) as one wave ballot: lane l tests key j0 + l (one token load
    // per lane instead of 16 per-element loads behind branches)
    uint64_t live;
    {
      const long kj = j0 + lane;
      bool ok = kj < Lk;
      if (ok && tok) ok = tok[kj] != a.pad;
      live = __ballot(ok);
    }
    float s[16];
    float tmax = -INFINITY;
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int kb = nb * 16 + g * 4 + t;
        const bool msk = !((live >> kb) & 1ull) | ((a.causal != 0) & ((int)j0 + kb > qi32));
        const float v = msk ? -INFINITY : st[nb][t] * sl2;
        s[nb * 4 + t] = v;
        tmax = fmaxf(tmax, v);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 16, 64));
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = (mnew == -INFINITY) ? 1.f : __builtin_amdgcn_exp2f(m - mnew);
    float psum = 0.f;
    float p[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      p[k] = (s[k] == -INFINITY) ? 0.f : __builtin_amdgcn_exp2f(s[k] - mnew);
      psum += p[k];
    }
    psum += __shfl_xor(psum, 16, 64);
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
    m = mnew;
    if (a.dropout) {
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          p[nb * 4 + t] *= drop_mul32(kf, rowbase + (uint32_t)(j0 + nb * 16 + t), a.thresh, a.dscale);
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) ot[i] *= alpha;
    // ---- O^T += V^T P^T ----
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 pb;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        pb[j] = (bf16)p[(2 * kk) * 4 + j];
        pb[4 + j] = (bf16)p[(2 * kk + 1) * 4 + j];
      }
      const int q = (lane & 15) >> 2, pp = lane & 3;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int colb = (i * 16 + 4 * pp) * 2;
        s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vs + koff_v(kk * 32 + g * 4 + q, colb)));
        s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vs + koff_v(kk * 32 + 16 + g * 4 + q, colb)));
        s16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        ot[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pb, ot[i], 0, 0, 0);
      }
    }
    if (more) lstore(cur ^ 1);
    __syncthreads();
  }
  if (!qlive) return;
  const float inv = 1.0f / l;  // fully masked row: 0 * inf = NaN, as the reference
  bf16* O = (bf16*)a.o + b * a.o_batch + qi * a.o_row + h * D;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
    bf16x4 o4 = {(bf16)(ot[i][0] * inv), (bf16)(ot[i][1] * inv), (bf16)(ot[i][2] * inv), (bf16)(ot[i][3] * inv)};
    *(bf16x4*)(O + i * 16 + g * 4) = o4;
  }
  if (a.lse && g == 0) a.lse[(b * H + h) * Lq + qi] = (m + __log2f(l)) * 0.6931471805599453f;
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA forward, head-resident K/V (no causal / PAD mask: the encoder MHSA and the decoder
// cross-attention). One workgroup per (b, h) stages the WHOLE K and V of the head in LDS once
// (Lk rounded up to 64 rows, <= 640 rows = 160 KiB; rows past Lk read as zero and are masked),
// then NW waves sweep 16-query tiles (ceil(Lq/16) tiles, so L = 197 wastes 5 % instead of the 30 %
// of 64-query blocks) against 32-key chunks with no barrier, no global load and no LDS write inside
// the key loop. Per 64-key chunk and wave: S^T = K Q^T (8 MFMAs) -> online softmax on 16 in-lane
// scores (scale folded into the exp2 FMA) -> O^T += V^T P^T (8 MFMAs, P straight from the
// accumulators, same key permutation as attn_fwd_mfma per 32-key half).
// Dropout (decoder cross-attention in training) is a template flag.
// ------------------------------------------------------------------------------------------------
constexpr int HK_MAX = 640;  // keys per head the LDS can hold (K + V = 256 B per key)
// K/V staging: chunk rows per thread with their loads in flight together (4 vs 1, tools/attn_bench.py:
// decoder cross 8.8 vs 9.4 us, ViT-B/16 and CLIP-L equal). Measured and rejected: a lazy
// softmax rescale (ViT-B/16 -0.3 us, CLIP-L -2.9 us, step neutral, but the cfg3 bf16 logits over the 1e-2
// bound) and two 16-query tiles per wave (ViT-B/16 26.7 -> 30.6 us, decoder cross 8.8 -> 12.3 us).
constexpr int HS = 4;

// cross-lane reductions over the 4 lane groups of a 16-query tile (lanes l, l ^ 16, l ^ 32, l ^ 48
// hold one query's key groups): v_permlane16_swap / v_permlane32_swap of a value with itself leave
// the (l, l ^ 16) / (l, l ^ 32) pair in the two results -- VALU, no LDS round trip
__device__ __forceinline__ float xmax_rows(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __builtin_fmaxf(__uint_as_float(a[0]), __uint_as_float(a[1]));
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __builtin_fmaxf(__uint_as_float(b[0]), __uint_as_float(b[1]));
}
__device__ __forceinline__ float xsum_rows(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}
__device__ __forceinline__ float max16(const float (&s)[16]) {
  const float a = __builtin_fmaxf(__builtin_fmaxf(s[0], s[1]), s[2]), b = __builtin_fmaxf(__builtin_fmaxf(s[3], s[4]), s[5]);
  const float c = __builtin_fmaxf(__builtin_fmaxf(s[6], s[7]), s[8]), d = __builtin_fmaxf(__builtin_fmaxf(s[9], s[10]), s[11]);
  const float e = __builtin_fmaxf(__builtin_fmaxf(s[12], s[13]), s[14]);
  return __builtin_fmaxf(__builtin_fmaxf(__builtin_fmaxf(a, b), c), __builtin_fmaxf(__builtin_fmaxf(d, e), s[15]));
}
constexpr bf16x8 ones8 = {(bf16)1.0f, (bf16)1.0f, (bf16)1.0f, (bf16)1.0f, (bf16)1.0f, (bf16)1.0f, (bf16)1.0f, (bf16)1.0f};

template <bool DROP>
__global__ __attribute__((amdgpu_flat_work_group_size(64, DROP ? 512 : 1024))) void attn_fwd_head(long H, long Lq, long Lk, AttnK a, int kbytes, int vbytes,
                                                      int lkp) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ks = lds;
  char* Vs = lds + (long)lkp * 128;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4, nw = blockDim.x >> 6;
  const long h = blockIdx.x, b = blockIdx.y;
  MIT_DASSERT(h < H && Lk <= lkp && lkp <= HK_MAX && Lq > 0);
  const bf16* Kb = (const bf16*)a.k + b * a.k_batch + h * D;
  const bf16* Vb = (const bf16*)a.v + b * a.v_batch + h * D;
  const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)Kb, (short)0, kbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)Vb, (short)0, vbytes, 0x00020000);
  // stage K and V: 8 16-B chunks per row, HS rows of chunks per thread with all their loads in flight
  // before the first LDS write (one round trip per HS, not per chunk row)
  const int nid = lkp * 8;
  for (int base = tid; base < nid; base += HS * (int)blockDim.x) {
    u32x4 kv[HS], vv[HS];
#pragma unroll
    for (int u = 0; u < HS; ++u) {
      const int id = base + u * (int)blockDim.x, r = id >> 3, c = id & 7;
      const bool ok = r < Lk;  // id >= nid gives r >= lkp >= Lk
      kv[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rk, (int)(ok ? (uint32_t)((r * a.k_row + c * 8) * 2) : A_OOB), 0, 0));
      vv[u] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rv, (int)(ok ? (uint32_t)((r * a.v_row + c * 8) * 2) : A_OOB), 0, 0));
    }
#pragma unroll
    for (int u = 0; u < HS; ++u) {
      const int id = base + u * (int)blockDim.x, r = id >> 3, c = id & 7;
      if (id < nid) {
        *(u32x4*)(Ks + koff_k(r, c)) = kv[u];
        *(u32x4*)(Vs + koff_v(r, c * 16)) = vv[u];
      }
    }
  }
  __syncthreads();

  const float sl2 = a.scale * 1.4426950408889634f;  // scores in log2 units
  const uint64_t key = DROP ? site_key(a.seed, a.site) : 0ull;
  const int nqt = (int)((Lq + 15) / 16);
  const int q = (lane & 15) >> 2, pp = lane & 3;
  // LDS byte offsets at key chunk 0; the swizzles only see row bits below 5, so chunk j0 (a
  // multiple of 32) just adds j0 * 128
  const int kofs = koff_k(lane & 15, g);           // + nb*2048 (16 rows), kk: chunk c ^ 4
  const int kofs1 = koff_k(lane & 15, 4 + g);
  int vofs[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int colb = (i * 16 + 4 * pp) * 2;
    vofs[i][0] = koff_v(g * 4 + q, colb);
    vofs[i][1] = koff_v(16 + g * 4 + q, colb);
  }
  for (int qt = w; qt < nqt; qt += nw) {
    const long qi = (long)qt * 16 + (lane & 15);
    const bool qlive = qi < Lq;
    bf16x8 qf[2];
    {
      const bf16* Qr = (const bf16*)a.q + b * a.q_batch + h * D + (qlive ? qi : 0) * a.q_row;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        u32x4 v = *(const u32x4*)(Qr + kk * 32 + g * 8);
        if (!qlive) v = u32x4{0u, 0u, 0u, 0u};
        qf[kk] = __builtin_bit_cast(bf16x8, v);
      }
    }
    // dropout index (bh * Lq + qi) * Lk + key < 2^32 (host-checked for the DROP instance): 32-bit, drop_mul32
    const uint32_t rowbase = ((uint32_t)(b * H + h) * (uint32_t)Lq + (uint32_t)qi) * (uint32_t)Lk + (uint32_t)(g * 4);
    const uint32_t kf = key_fold(key);
    f32x4 ot[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) ot[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = -INFINITY, l = 0.f;
    f32x4 lacc = {0.f, 0.f, 0.f, 0.f};  // MFMA-accumulated denominator of the full chunks (!DROP)
    const char* Kc = Ks;
    const char* Vc = Vs;
    int j0 = 0;
    const int ilk = (int)Lk;
    for (; j0 + 64 <= lkp; j0 += 64, Kc += 64 * 128, Vc += 64 * 128) {
      // ---- S^T = K Q^T for keys j0 .. j0+63 (4 key tiles of 16) ----
      f32x4 st[4];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        const u32x4 k0 = *(const u32x4*)(Kc + nb * 2048 + kofs);
        const u32x4 k1 = *(const u32x4*)(Kc + nb * 2048 + kofs1);
        st[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, k0), qf[0],
                                                          f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        st[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, k1), qf[1], st[nb], 0, 0, 0);
      }
      // V^T fragments (2 x 32-key halves x 4 d-tiles): issued before the softmax to hide latency
      s16x8 vv[2][4];
#pragma unroll
      for (int hh = 0; hh < 2; ++hh)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vc + hh * 4096 + vofs[i][0]));
          s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vc + hh * 4096 + vofs[i][1]));
          vv[hh][i] = s16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
      // scores stay unscaled: max commutes with the positive scale, which folds into the exp2 FMA
      float s[16];
#pragma unroll
      for (int nb = 0; nb < 4; ++nb)
#pragma unroll
        for (int t = 0; t < 4; ++t) s[nb * 4 + t] = st[nb][t];
      // ragged last chunk (wave-uniform; 32-bit compares, and a real branch: left to the compiler it was
      // if-converted into 48 64-bit compare / select VALU ops in every chunk, ~35 % of the chunk's VALU --
      // measured neutral on this latency-bound loop, CLIP-L/14@336 48.3 -> 47.6 us)
      if (__builtin_expect(j0 + 64 > ilk, 0)) {
        const int live = ilk - j0 - g * 4;
#pragma unroll
        for (int k = 0; k < 16; ++k)
          if ((k >> 2) * 16 + (k & 3) >= live) s[k] = -INFINITY;
      }
      // row max: v_max3 tree over the 16 in-lane scores, then the query's 4 lane groups (l, l ^ 16,
      // l ^ 32, l ^ 48) through v_permlane16/32_swap (VALU) instead of ds_bpermute round trips
      float tmax = max16(s);
      tmax = xmax_rows(tmax);
      {
        const float mnew = __builtin_fmaxf(m, tmax * sl2);  // finite: >= 1 unmasked key per chunk
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        l *= alpha;
        lacc *= alpha;
#pragma unroll
        for (int i = 0; i < 4; ++i) ot[i] *= alpha;
        m = mnew;
      }
      float p[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) p[k] = __builtin_amdgcn_exp2f(fmaf(s[k], sl2, -m));
      if (DROP) {  // the denominator sums the undropped p (VALU); without dropout an MFMA sums them below
        float psum = 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k) psum += p[k];
        l += xsum_rows(psum);
      }
      if (DROP) {
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            p[nb * 4 + t] *= drop_mul32(kf, rowbase + (uint32_t)(j0 + nb * 16 + t), a.thresh, a.dscale);
      }
      // ---- O^T += V^T P^T, two 32-key halves ----
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (bf16)p[hh * 8 + j];
#pragma unroll
        for (int i = 0; i < 4; ++i)
          ot[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv[hh][i]), pb, ot[i], 0, 0, 0);
        // softmax denominator: ones^T P^T = the query's sum of its 32 (bf16) p in every accumulator
        // row -- one MFMA instead of 16 VALU adds and two cross-lane reductions
        if (!DROP) lacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones8, pb, lacc, 0, 0, 0);
      }
    }
    if (!DROP) l += lacc[0];
    // ---- tail: the last 16 / 32 / 48 keys (K/V are staged to a multiple of 16 rows, not 64) ----
    const int ntail = (lkp - j0) >> 4;  // wave-uniform
    if (ntail) {
      f32x4 st[3];
      float s[12];
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) {
        if (nb < ntail) {
          const u32x4 k0 = *(const u32x4*)(Kc + nb * 2048 + kofs);
          const u32x4 k1 = *(const u32x4*)(Kc + nb * 2048 + kofs1);
          st[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, k0), qf[0],
                                                            f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
          st[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, k1), qf[1], st[nb], 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t)
          s[nb * 4 + t] = (nb < ntail && j0 + nb * 16 + g * 4 + t < Lk) ? st[nb][t] : -INFINITY;
      }
      float tmax = s[0];
#pragma unroll
      for (int k = 1; k < 12; ++k) tmax = __builtin_fmaxf(tmax, s[k]);
      tmax = xmax_rows(tmax);
      const float mnew = __builtin_fmaxf(m, tmax * sl2);  // finite: key j0 < Lk
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      float p[12], psum = 0.f;
#pragma unroll
      for (int k = 0; k < 12; ++k) {
        p[k] = __builtin_amdgcn_exp2f(fmaf(s[k], sl2, -mnew));
        psum += p[k];
      }
      l = l * alpha + xsum_rows(psum);
      m = mnew;
      if (DROP) {
#pragma unroll
        for (int nb = 0; nb < 3; ++nb)
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (nb < ntail)
              p[nb * 4 + t] *= drop_mul32(kf, rowbase + (uint32_t)(j0 + nb * 16 + t), a.thresh, a.dscale);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) ot[i] *= alpha;
      if (ntail >= 2) {  // keys 0..31 of the tail: one 16x16x32 block per d-tile, as the main loop
        bf16x8 pb;
#pragma unroll
        for (int j = 0; j < 8; ++j) pb[j] = (bf16)p[j];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vc + vofs[i][0]));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vc + vofs[i][1]));
          const s16x8 vv = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          ot[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, vv), pb, ot[i], 0, 0, 0);
        }
      }
      if (ntail & 1) {  // the odd 16-key tile (tile 0 or 2): 16x16x16, k = g*4 + t on both operands
        const int tb = ntail - 1;
        const int voff = tb == 2 ? 4096 : 0;
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 pq;
#pragma unroll
        for (int t = 0; t < 4; ++t) pq[t] = (bf16)p[(tb == 2 ? 8 : 0) + t];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Vc + voff + vofs[i][0]));
          ot[i] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(lo, __builtin_bit_cast(s16x4, pq), ot[i], 0, 0, 0);
        }
      }
    }
    if (qlive) {
      const float inv = 1.0f / l;
      bf16* O = (bf16*)a.o + b * a.o_batch + qi * a.o_row + h * D;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 o4 = {(bf16)(ot[i][0] * inv), (bf16)(ot[i][1] * inv), (bf16)(ot[i][2] * inv), (bf16)(ot[i][3] * inv)};
        *(bf16x4*)(O + i * 16 + g * 4) = o4;
      }
      if (a.lse && g == 0) a.lse[(b * H + h) * Lq + qi] = (m + __log2f(l)) * 0.6931471805599453f;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA backward, two kernels (launched dQ first: it also produces delta = rowsum(dO o O)).
//   dQ kernel  (grid: query blocks): per 64-key tile  S^T = K Q^T, dP^T = V dO^T (A = K/V rows from
//     LDS, B = Q/dO fragments in registers) -> dS^T -> dQ^T += K^T dS^T (A = K^T by transposed
//     LDS read, B = dS^T from the accumulators, same permuted k index as the forward).
//   dKV kernel (grid: key blocks, wave = 16 keys): per 64-query tile  S = Q K^T, dP = dO V^T
//     (A = Q/dO rows from LDS, B = K/V fragments in registers; key on the lane) -> P, dS ->
//     dV^T += dO^T (P o M), dK^T += Q^T dS (A by transposed LDS reads of the dO / Q tiles).
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bf16x8 lds_row_frag(const char* tile, int row, int chunk) {
  return __builtin_bit_cast(bf16x8, *(const u32x4*)(tile + koff_k(row, chunk)));
}
// A operand (m = column block [c0, c0+16) of the tile, k = rows kbase+{4g..4g+3, 16+4g..16+4g+3})
__device__ __forceinline__ bf16x8 lds_tr_frag(const char* tile, int kbase, int c0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int colb = (c0 + 4 * p) * 2;
  const int r0 = kbase + g * 4 + q;
  // koff_k chunk swizzle applied to the 8-byte half-chunk the lane reads
  auto addr = [&](int r) { return r * 128 + ((((colb >> 4) ^ ((r >> 1) & 7)) << 4) | (colb & 15)); };
  s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, tile + addr(r0)));
  s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, tile + addr(r0 + 16)));
  s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, v);
}
__device__ __forceinline__ void load_tile_rows(char* tile, const bf16* base, long row_stride, long r0, long nrows, int bytes,
                                               int tid) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int id = tid + 256 * i, r = id >> 3, c = id & 7;
    const long row = r0 + r;
    const uint32_t off = row < nrows ? (uint32_t)((row * row_stride + c * 8) * 2) : A_OOB;
    *(u32x4*)(tile + koff_k(r, c)) = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
  }
}

struct AttnBwdBytes {
  int q, k, v, dO;
};

__global__ __launch_bounds__(256) void attn_bwd_dq_mfma(long H, long Lq, long Lk, AttnK a, AttnG gr, AttnBwdBytes nb_) {
  __shared__ __attribute__((aligned(16))) char lds[2 * AK * D * 2];  // K tile, V tile
  char* Ks = lds;
  char* Vs = lds + AK * D * 2;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const long b = blockIdx.z, h = blockIdx.y;
  const long qblk = (long)blockIdx.x * AQ;
  const long qi = qblk + w * 16 + (lane & 15);
  const bool qlive = qi < Lq;
  const long qr = qlive ? qi : 0;
  const bf16* Qr = (const bf16*)a.q + b * a.q_batch + h * D + qr * a.q_row;
  const bf16* Or = (const bf16*)a.o + b * a.o_batch + h * D + qr * a.o_row;
  const bf16* dOr = (const bf16*)gr.dout + b * gr.do_batch + h * D + qr * gr.do_row;
  bf16x8 qf[2], df[2];
  float delta = 0.f;
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    u32x4 qv = *(const u32x4*)(Qr + kk * 32 + g * 8), dv = *(const u32x4*)(dOr + kk * 32 + g * 8);
    const bf16x8 ov = __builtin_bit_cast(bf16x8, *(const u32x4*)(Or + kk * 32 + g * 8));
    if (!qlive) qv = dv = u32x4{0u, 0u, 0u, 0u};
    qf[kk] = __builtin_bit_cast(bf16x8, qv);
    df[kk] = __builtin_bit_cast(bf16x8, dv);
#pragma unroll
    for (int j = 0; j < 8; ++j) delta += (float)df[kk][j] * (float)ov[j];
  }
  delta += __shfl_xor(delta, 16, 64);
  delta += __shfl_xor(delta, 32, 64);
  const long row = (b * H + h) * Lq + qi;
  if (qlive && g == 0) gr.delta[row] = delta;
  const float l2e = 1.4426950408889634f;
  const float lse2 = qlive ? a.lse[row] * l2e : 0.f;
  const float sl2 = a.scale * l2e;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const uint64_t rowbase = (uint64_t)row * (uint64_t)Lk;
  const int64_t* tok = a.tok ? a.tok + b * a.tok_batch : nullptr;
  const bf16* Kb = (const bf16*)a.k + b * a.k_batch + h * D;
  const bf16* Vb = (const bf16*)a.v + b * a.v_batch + h * D;
  long kend = Lk;
  if (a.causal) kend = min(Lk, min(Lq, qblk + AQ));
  f32x4 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (long j0 = 0; j0 < kend; j0 += AK) {
    __syncthreads();
    load_tile_rows(Ks, Kb, a.k_row, j0, Lk, nb_.k, tid);
    load_tile_rows(Vs, Vb, a.v_row, j0, Lk, nb_.v, tid);
    __syncthreads();
    f32x4 st[4], dp[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) st[nb] = dp[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        st[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_row_frag(Ks, nb * 16 + (lane & 15), kk * 4 + g), qf[kk],
                                                         st[nb], 0, 0, 0);
        dp[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_row_frag(Vs, nb * 16 + (lane & 15), kk * 4 + g), df[kk],
                                                         dp[nb], 0, 0, 0);
      }
    float ds[16];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const long kj = j0 + nb * 16 + g * 4 + t;
        bool msk = !qlive || kj >= Lk || (a.causal && kj > qi);
        if (!msk && tok) msk = tok[kj] == a.pad;
        const float p = msk ? 0.f : exp2f(st[nb][t] * sl2 - lse2);
        const float mul = a.dropout ? drop_mul(key, rowbase + (uint64_t)kj, a.thresh, a.dscale) : 1.f;
        ds[nb * 4 + t] = p * (dp[nb][t] * mul - delta);
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bs;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bs[j] = (bf16)ds[(2 * kk) * 4 + j];
        bs[4 + j] = (bf16)ds[(2 * kk + 1) * 4 + j];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) dq[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_tr_frag(Ks, kk * 32, i * 16, lane), bs,
                                                                              dq[i], 0, 0, 0);
    }
  }
  if (!qlive) return;
  bf16* DQ = (bf16*)gr.dq + b * gr.dq_batch + qi * gr.dq_row + h * D;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *(bf16x4*)(DQ + i * 16 + g * 4) = bf16x4{(bf16)(dq[i][0] * a.scale), (bf16)(dq[i][1] * a.scale),
                                             (bf16)(dq[i][2] * a.scale), (bf16)(dq[i][3] * a.scale)};
}

__global__ __launch_bounds__(256) void attn_bwd_dkv_mfma(long H, long Lq, long Lk, AttnK a, AttnG gr, AttnBwdBytes nb_) {
  __shared__ __attribute__((aligned(16))) char lds[2 * AQ * D * 2 + 2 * AQ * 4];  // Q tile, dO tile, lse, delta
  char* Qs = lds;
  char* Ds = lds + AQ * D * 2;
  float* Ls = (float*)(lds + 2 * AQ * D * 2);
  float* Dl = Ls + AQ;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const long b = blockIdx.z, h = blockIdx.y;
  const long kblk = (long)blockIdx.x * AK;
  const long kl = kblk + w * 16 + (lane & 15);
  const bool klive = kl < Lk;
  const long kr = klive ? kl : 0;
  const bf16* Kr = (const bf16*)a.k + b * a.k_batch + h * D + kr * a.k_row;
  const bf16* Vr = (const bf16*)a.v + b * a.v_batch + h * D + kr * a.v_row;
  bf16x8 kf[2], vf[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    u32x4 k4 = *(const u32x4*)(Kr + kk * 32 + g * 8), v4 = *(const u32x4*)(Vr + kk * 32 + g * 8);
    if (!klive) k4 = v4 = u32x4{0u, 0u, 0u, 0u};
    kf[kk] = __builtin_bit_cast(bf16x8, k4);
    vf[kk] = __builtin_bit_cast(bf16x8, v4);
  }
  const bool kpad = klive && a.tok && a.tok[b * a.tok_batch + kl] == a.pad;
  const float l2e = 1.4426950408889634f;
  const float sl2 = a.scale * l2e;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const bf16* Qb = (const bf16*)a.q + b * a.q_batch + h * D;
  const bf16* dOb = (const bf16*)gr.dout + b * gr.do_batch + h * D;
  const long bh = b * H + h;
  f32x4 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long qstart = a.causal ? (kblk / AQ) * AQ : 0;  // queries before the block's first key see none of it
  for (long q0 = qstart; q0 < Lq; q0 += AQ) {
    __syncthreads();
    load_tile_rows(Qs, Qb, a.q_row, q0, Lq, nb_.q, tid);
    load_tile_rows(Ds, dOb, gr.do_row, q0, Lq, nb_.dO, tid);
    if (tid < AQ) {
      const long q = q0 + tid;
      Ls[tid] = q < Lq ? a.lse[bh * Lq + q] * l2e : 0.f;
      Dl[tid] = q < Lq ? gr.delta[bh * Lq + q] : 0.f;
    }
    __syncthreads();
    f32x4 s[4], dp[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) s[nb] = dp[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        s[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_row_frag(Qs, nb * 16 + (lane & 15), kk * 4 + g), kf[kk], s[nb],
                                                        0, 0, 0);
        dp[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_row_frag(Ds, nb * 16 + (lane & 15), kk * 4 + g), vf[kk],
                                                         dp[nb], 0, 0, 0);
      }
    float pd[16], ds[16];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int qq = nb * 16 + g * 4 + t;
        const long q = q0 + qq;
        const bool msk = !klive || kpad || q >= Lq || (a.causal && kl > q);
        const float p = msk ? 0.f : exp2f(s[nb][t] * sl2 - Ls[qq]);
        const float mul = a.dropout ? drop_mul(key, ((uint64_t)bh * (uint64_t)Lq + (uint64_t)q) * (uint64_t)Lk + kl, a.thresh,
                                               a.dscale)
                                    : 1.f;
        pd[nb * 4 + t] = p * mul;
        ds[nb * 4 + t] = p * (dp[nb][t] * mul - Dl[qq]);
      }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bp, bs;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bp[j] = (bf16)pd[(2 * kk) * 4 + j];
        bp[4 + j] = (bf16)pd[(2 * kk + 1) * 4 + j];
        bs[j] = (bf16)ds[(2 * kk) * 4 + j];
        bs[4 + j] = (bf16)ds[(2 * kk + 1) * 4 + j];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dv[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_tr_frag(Ds, kk * 32, i * 16, lane), bp, dv[i], 0, 0, 0);
        dk[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_tr_frag(Qs, kk * 32, i * 16, lane), bs, dk[i], 0, 0, 0);
      }
    }
  }
  if (!klive) return;
  bf16* DK = (bf16*)gr.dk + b * gr.dk_batch + kl * gr.dk_row + h * D;
  bf16* DV = (bf16*)gr.dv + b * gr.dv_batch + kl * gr.dv_row + h * D;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    *(bf16x4*)(DK + i * 16 + g * 4) = bf16x4{(bf16)(dk[i][0] * a.scale), (bf16)(dk[i][1] * a.scale),
                                             (bf16)(dk[i][2] * a.scale), (bf16)(dk[i][3] * a.scale)};
    *(bf16x4*)(DV + i * 16 + g * 4) = bf16x4{(bf16)dv[i][0], (bf16)dv[i][1], (bf16)dv[i][2], (bf16)dv[i][3]};
  }
}

// ------------------------------------------------------------------------------------------------
// bf16 MFMA backward, head-resident and fused (the decoder: Lq <= 64 queries, Lk <= 256 keys).
// One 8-wave workgroup per (b, h). The split dQ / dKV kernels above each walk a dependent chain
// of global round trips per 64-row tile (a 63 x 197 head is 55 us for two launches at under one
// resident wave per SIMD); here every operand of the head -- K, Q, dO into LDS; each wave's V
// strips, O / lse for delta into registers -- is requested in ONE batch of loads, and then:
//   phase A (waves over 16-key strips, key on the lane): S = Q K^T, dP = dO V^T for all 64 queries
//     -> P (mask, dropout), dS = P o (dP o M - delta); dV += (P o M)^T dO, dK += dS^T Q (A by
//     transposed LDS reads), written straight out; dS^T (bf16) kept in LDS as a [key][64 query]
//     tile in the K-tile swizzle (four 8-byte stores per strip and lane).
//   phase B (waves over 16 queries x 32 head dims): dQ^T = K^T dS^T, both operands by transposed
//     LDS reads of the K and dS^T tiles (the same permuted k order on both sides).
// The dropout mask and exp are evaluated once per element (the split kernels evaluate both twice).
// LDS: (2 * Lk + 128) rows x 128 B <= 80 KiB, so two workgroups share a CU (<= 128 VGPRs).
// ------------------------------------------------------------------------------------------------
constexpr int HB_MAXK = 256;  // keys per head
constexpr int HB_NT = 512;    // 8 waves
constexpr int HB_SPW = HB_MAXK / 16 / 8;  // key strips per wave (<= 2)

__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4))) void attn_bwd_head(long H, long Lq, long Lk, AttnK a, AttnG gr, AttnBwdBytes nb_,
                                                        int lkp) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Ks = lds;                // [lkp][64] bf16
  char* St = Ks + lkp * 128;     // dS^T [lkp][64] bf16
  char* Qs = St + lkp * 128;     // [64][64]
  char* Ds = Qs + 64 * 128;      // dO [64][64]
  float* Ls = (float*)(Ds + 64 * 128);
  float* Dl = Ls + 64;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 4;
  const long h = blockIdx.x, b = blockIdx.y, bh = b * H + h;
  MIT_DASSERT(h < H && Lq <= 64 && Lk <= lkp && lkp <= HB_MAXK);
  const bf16* Qb = (const bf16*)a.q + b * a.q_batch + h * D;
  const bf16* Kb = (const bf16*)a.k + b * a.k_batch + h * D;
  const bf16* Vb = (const bf16*)a.v + b * a.v_batch + h * D;
  const bf16* dOb = (const bf16*)gr.dout + b * gr.do_batch + h * D;
  const bf16* Ob = (const bf16*)a.o + b * a.o_batch + h * D;
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc((void*)Vb, (short)0, nb_.v, 0x00020000);
  // ---- one batch of loads ----
  bf16x8 vf[HB_SPW][2];  // B operand of dP = dO V^T for this wave's strips (key on the lane)
#pragma unroll
  for (int si = 0; si < HB_SPW; ++si)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const long kl = (w + 8 * si) * 16 + (lane & 15);
      const bool ok = kl < Lk;
      vf[si][kk] = __builtin_bit_cast(
          bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                      rv, (int)(ok ? (uint32_t)((kl * a.v_row + kk * 32 + g * 8) * 2) : A_OOB), 0, 0));
    }
  {
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc((void*)Kb, (short)0, nb_.k, 0x00020000);
    const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)Qb, (short)0, nb_.q, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc((void*)dOb, (short)0, nb_.dO, 0x00020000);
    u32x4 kr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + HB_NT * i, r = c >> 3, ch = c & 7;
      const bool ok = r < Lk && c < lkp * 8;
      kr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                            rk, (int)(ok ? (uint32_t)((r * a.k_row + ch * 8) * 2) : A_OOB), 0, 0));
    }
    const int r = tid >> 3, ch = tid & 7;  // 64 rows x 8 chunks = 512 threads
    const bool qok = r < Lq;
    const u32x4 qr = __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rq, (int)(qok ? (uint32_t)((r * a.q_row + ch * 8) * 2) : A_OOB), 0, 0));
    const u32x4 dr = __builtin_bit_cast(
        u32x4, __builtin_amdgcn_raw_buffer_load_b128(rd, (int)(qok ? (uint32_t)((r * gr.do_row + ch * 8) * 2) : A_OOB), 0, 0));
    bf16x8 ov = {};
    if (qok) ov = *(const bf16x8*)(Ob + r * a.o_row + ch * 8);
    const float l = (qok && ch == 0) ? a.lse[bh * Lq + r] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + HB_NT * i;
      if (c < lkp * 8) *(u32x4*)(Ks + koff_k(c >> 3, c & 7)) = kr[i];
    }
    *(u32x4*)(Qs + koff_k(r, ch)) = qr;
    *(u32x4*)(Ds + koff_k(r, ch)) = dr;
    // delta = rowsum(dO o O): 8 lanes per query
    const bf16x8 dv8 = __builtin_bit_cast(bf16x8, dr);
    float dl = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += (float)dv8[j] * (float)ov[j];
    dl += __shfl_xor(dl, 1, 64);
    dl += __shfl_xor(dl, 2, 64);
    dl += __shfl_xor(dl, 4, 64);
    if (ch == 0) {
      Ls[r] = l * 1.4426950408889634f;
      Dl[r] = dl;
      if (qok) gr.delta[bh * Lq + r] = dl;
    }
  }
  __syncthreads();
  const float sl2 = a.scale * 1.4426950408889634f;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const int64_t* tok = a.tok ? a.tok + b * a.tok_batch : nullptr;
  typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
  // ---- phase A: key strips ----
#pragma unroll
  for (int si = 0; si < HB_SPW; ++si) {
    const int ks = w + 8 * si;
    if (ks * 16 >= lkp) break;
    const int kloc = ks * 16 + (lane & 15);
    const long kl = kloc;
    const bool klive = kl < Lk;
    const bool kpad = klive && tok && tok[kl] == a.pad;
    f32x4 s[4], dp[4];
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) s[nb] = dp[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 kf = lds_row_frag(Ks, kloc, kk * 4 + g);
#pragma unroll
      for (int nb = 0; nb < 4; ++nb) {
        s[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_row_frag(Qs, nb * 16 + (lane & 15), kk * 4 + g), kf, s[nb],
                                                        0, 0, 0);
        dp[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_row_frag(Ds, nb * 16 + (lane & 15), kk * 4 + g), vf[si][kk],
                                                         dp[nb], 0, 0, 0);
      }
    }
    bf16x4 bp4[4], bs4[4];  // (P o M) and dS, 4 consecutive queries (t) per 16-query block nb
    const bool kdead = !klive || kpad;
    // dropout index (bh * Lq + qq) * Lk + kl < 2^32 (host-checked): the lane's part once, then a wave-uniform
    // step per (nb, t); drop_mul32 hashes it exactly as drop_mul does
    const uint32_t ilane = ((uint32_t)bh * (uint32_t)Lq + (uint32_t)(g * 4)) * (uint32_t)Lk + (uint32_t)kl;
    const uint32_t kf = key_fold(key);
#pragma unroll
    for (int nb = 0; nb < 4; ++nb) {
      // the 4 queries' log-sum-exp and delta in one 16-B LDS read each (were 8 ds_read_b32)
      const f32x4 lq4 = *(const f32x4*)(Ls + nb * 16 + g * 4), dl4 = *(const f32x4*)(Dl + nb * 16 + g * 4);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int qq = nb * 16 + g * 4 + t;
        // bitwise, 32-bit: a short-circuit || over 64-bit compares compiled into exec-masked branches
        const bool msk = kdead | (qq >= (int)Lq) | ((a.causal != 0) & (kloc > qq));
        // branch-free: v_exp_f32 for every element, the mask selects (ocml's exp2f added a denormal-range
        // rescale per element, and the masked form compiled into exec-masked branches)
        const float e = __builtin_amdgcn_exp2f(s[nb][t] * sl2 - lq4[t]);
        const float p = msk ? 0.f : e;
        const float mul =
            a.dropout ? drop_mul32(kf, ilane + (uint32_t)(nb * 16 + t) * (uint32_t)Lk, a.thresh, a.dscale) : 1.f;
        bp4[nb][t] = (bf16)(p * mul);
        bs4[nb][t] = (bf16)(p * (dp[nb][t] * mul - dl4[t]));
      }
      // dS^T row kloc, queries nb*16+4g .. +4: 8 bytes in the K-tile swizzle
      *(bf16x4*)(St + koff_k(kloc, nb * 2 + (g >> 1)) + (g & 1) * 8) = bs4[nb];
    }
    f32x4 dk[4], dv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) dk[i] = dv[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 bp = {bp4[2 * kk][0], bp4[2 * kk][1], bp4[2 * kk][2], bp4[2 * kk][3],
                         bp4[2 * kk + 1][0], bp4[2 * kk + 1][1], bp4[2 * kk + 1][2], bp4[2 * kk + 1][3]};
      const bf16x8 bs = {bs4[2 * kk][0], bs4[2 * kk][1], bs4[2 * kk][2], bs4[2 * kk][3],
                         bs4[2 * kk + 1][0], bs4[2 * kk + 1][1], bs4[2 * kk + 1][2], bs4[2 * kk + 1][3]};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        dv[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_tr_frag(Ds, kk * 32, i * 16, lane), bp, dv[i], 0, 0, 0);
        dk[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_tr_frag(Qs, kk * 32, i * 16, lane), bs, dk[i], 0, 0, 0);
      }
    }
    if (klive) {
      bf16* DK = (bf16*)gr.dk + b * gr.dk_batch + kl * gr.dk_row + h * D;
      bf16* DV = (bf16*)gr.dv + b * gr.dv_batch + kl * gr.dv_row + h * D;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        *(bf16x4*)(DK + i * 16 + g * 4) = bf16x4{(bf16)(dk[i][0] * a.scale), (bf16)(dk[i][1] * a.scale),
                                                 (bf16)(dk[i][2] * a.scale), (bf16)(dk[i][3] * a.scale)};
        *(bf16x4*)(DV + i * 16 + g * 4) = bf16x4{(bf16)dv[i][0], (bf16)dv[i][1], (bf16)dv[i][2], (bf16)dv[i][3]};
      }
    }
  }
  __syncthreads();
  // ---- phase B: dQ^T (16 head dims x 16 queries tiles) = K^T dS^T; wave = (query strip, dim half) ----
  {
    const int qs = w & 3, dh = w >> 2;
    const int qq = qs * 16 + (lane & 15);
    f32x4 dq[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
    for (int k0 = 0; k0 < lkp; k0 += 32) {
      const bf16x8 bsf = lds_tr_frag(St, k0, qs * 16, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i)
        dq[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(lds_tr_frag(Ks, k0, dh * 32 + i * 16, lane), bsf, dq[i], 0, 0, 0);
    }
    if (qq < Lq) {
      bf16* DQ = (bf16*)gr.dq + b * gr.dq_batch + (long)qq * gr.dq_row + h * D + dh * 32;
#pragma unroll
      for (int i = 0; i < 2; ++i)
        *(bf16x4*)(DQ + i * 16 + g * 4) = bf16x4{(bf16)(dq[i][0] * a.scale), (bf16)(dq[i][1] * a.scale),
                                                 (bf16)(dq[i][2] * a.scale), (bf16)(dq[i][3] * a.scale)};
    }
  }
}

// head_dim dispatch for the generic kernels: DH in {16, 32, 64, 128}
#define DISPATCH_DH(dh, ...)                    \
  do {                                          \
    switch (dh) {                               \
      case 16: { constexpr int DH = 16; __VA_ARGS__; } break;   \
      case 32: { constexpr int DH = 32; __VA_ARGS__; } break;   \
      case 64: { constexpr int DH = 64; __VA_ARGS__; } break;   \
      default: { constexpr int DH = 128; __VA_ARGS__; } break;  \
    }                                           \
  } while (0)

inline bool head_dim_ok(long dh) { return dh == 16 || dh == 32 || dh == 64 || dh == 128; }

AttnK make_k(const mit_attn_args* x) {
  AttnK a;
  a.q = x->q; a.q_row = x->q_row; a.q_batch = x->q_batch;
  a.k = x->k; a.k_row = x->k_row; a.k_batch = x->k_batch;
  a.v = x->v; a.v_row = x->v_row; a.v_batch = x->v_batch;
  a.o = x->o; a.o_row = x->o_row; a.o_batch = x->o_batch;
  a.lse = x->lse; a.tok = x->key_tokens; a.tok_batch = x->tok_batch; a.pad = x->pad_idx;
  a.causal = x->causal; a.scale = x->scale; a.seed = x->seed; a.site = x->site;
  a.dropout = x->drop_p > 0.f;
  a.thresh = drop_threshold(x->drop_p);
  a.dscale = x->drop_p < 1.f ? 1.f / (1.f - x->drop_p) : 0.f;
  return a;
}

}  // namespace


// dropout calls with B*H*Lq*Lk at or past this run the 64-bit mask-index kernels (mit_attention_set_index_limit)
static double g_idx32_limit = 4294967296.0;
extern "C" int mit_attention_set_index_limit(double limit) {
  g_idx32_limit = limit > 0 ? limit : 4294967296.0;
  return MIT_OK;
}

extern "C" int mit_attention_fwd(int dtype, long B, long H, long Lq, long Lk, long Dh, const mit_attn_args* x,
                                 void* stream) {
  MIT_CHECK_ARG(x && x->q && x->k && x->v && x->o, "mit_attention_fwd: null pointer");
  MIT_RECORD([=, c = *x]() { return mit_attention_fwd(dtype, B, H, Lq, Lk, Dh, &c, stream); });
  MIT_CHECK_ARG(head_dim_ok(Dh), "mit_attention_fwd: head_dim %ld unsupported (16, 32, 64, 128)", Dh);
  if (B <= 0 || H <= 0 || Lq <= 0) return MIT_OK;
  MIT_CHECK_ARG(Lk > 0, "mit_attention_fwd: Lk must be > 0");
  AttnK a = make_k(x);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((Lq + 63) / 64), (unsigned)H, (unsigned)B);
  // the MFMA kernels are written for head_dim 64 (every ViT / CLIP tower and the 512/768-wide
  // decoders); other head dims run the generic kernels
  const bool mfma_ok = Dh == D && dtype == MIT_BF16 && x->q_row % 8 == 0 && x->q_batch % 8 == 0 && x->k_row % 8 == 0 &&
                       x->k_batch % 8 == 0 && x->v_row % 8 == 0 && x->v_batch % 8 == 0 && x->o_row % 4 == 0 &&
                       x->o_batch % 4 == 0 && ((uintptr_t)x->q | (uintptr_t)x->k | (uintptr_t)x->v) % 16 == 0 &&
                       ((uintptr_t)x->o % 8) == 0;
  if (mfma_ok) {
    const long kb = 2 * ((Lk - 1) * x->k_row + D), vb = 2 * ((Lk - 1) * x->v_row + D);
    MIT_CHECK_ARG(kb < (1L << 31) && vb < (1L << 31), "mit_attention_fwd: K/V span >= 2 GiB");
    if (!a.causal && !a.tok && Lk <= HK_MAX && H <= 65535 && B <= 65535 &&
        (!a.dropout || (double)B * (double)H * (double)Lq * (double)Lk < g_idx32_limit)) {
      // head-resident K/V: one workgroup per (b, h), NW waves balanced over the 16-query tiles.
      // K/V rows are staged to a multiple of 16 (the key tail of < 64 runs 16-key tiles: a ViT-B/16
      // head of 197 keys sweeps 208 instead of 256; 28.5 -> 27.7 us, tools/attn_bench.py). <= 8 waves
      // whenever two heads fit the LDS, so a CU holds two workgroups and one stages its K/V while the
      // other computes. Three 5-wave workgroups per CU (one round of the 768 heads instead of 1.5,
      // 52 KiB each) measured slower (30.8 us): the CU's VALU, not the rounds, bounds this kernel.
      // The dropout instance is built for <= 512 threads.
      constexpr int pad = 16;
      const int lkp = (int)((Lk + pad - 1) / pad * pad);
      const int nqt = (int)((Lq + 15) / 16);
      const int maxw = (a.dropout || 2 * lkp * 256 <= 160 * 1024) ? 8 : 16;
      // every wave the occupancy allows, the query tiles' rounds unbalanced (CLIP-L/14@336: 37 = 16 + 16 + 5
      // in one workgroup per CU; ViT-B/16: 13 = 8 + 5 in two) rather than fewer balanced waves (13 + 13 + 11,
      // 7 + 6): more waves to hide the sweep's latency, 47.2 -> 45.2 / 26.7 -> 26.5 us, configs[2]
      // 2067 -> 2078 pairs/s (profiles/r05_decoder_experiments.txt)
      const int nw = std::min(nqt, maxw);
      const int lds = lkp * 256;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)attn_fwd_head<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  HK_MAX * 256);
        (void)hipFuncSetAttribute((const void*)attn_fwd_head<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  HK_MAX * 256);
        attr = true;
      }
      dim3 hg((unsigned)H, (unsigned)B);
      if (a.dropout)
        hipLaunchKernelGGL(attn_fwd_head<true>, hg, dim3(64 * nw), lds, s, H, Lq, Lk, a, (int)kb, (int)vb, lkp);
      else
        hipLaunchKernelGGL(attn_fwd_head<false>, hg, dim3(64 * nw), lds, s, H, Lq, Lk, a, (int)kb, (int)vb, lkp);
    } else if (!a.dropout || (double)B * (double)H * (double)Lq * (double)Lk < g_idx32_limit) {
      hipLaunchKernelGGL(attn_fwd_mfma, grid, dim3(256), 0, s, H, Lq, Lk, a, (int)kb, (int)vb);
    } else {  // dropout indices past 2^32 (the MFMA kernels form them in 32 bits)
      hipLaunchKernelGGL((attn_fwd_simple<bf16, 64>), grid, dim3(64), 0, s, H, Lq, Lk, a);
    }
  } else if (dtype == MIT_BF16) {
    DISPATCH_DH(Dh, hipLaunchKernelGGL((attn_fwd_simple<bf16, DH>), grid, dim3(64), 0, s, H, Lq, Lk, a));
  } else {
    DISPATCH_DH(Dh, hipLaunchKernelGGL((attn_fwd_simple<float, DH>), grid, dim3(64), 0, s, H, Lq, Lk, a));
  }
  MIT_LAUNCH_CHECK("mit_attention_fwd");
  return MIT_OK;
}

extern "C" int mit_attention_bwd(int dtype, long B, long H, long Lq, long Lk, long Dh, const mit_attn_args* x,
                                 const mit_attn_grads* gg, void* stream) {
  MIT_CHECK_ARG(x && gg && x->q && x->k && x->v && x->o && x->lse, "mit_attention_bwd: null forward pointer");
  MIT_CHECK_ARG(gg->dout && gg->dq && gg->dk && gg->dv && gg->delta_ws, "mit_attention_bwd: null grad pointer");
  MIT_RECORD([=, c = *x, cg = *gg]() { return mit_attention_bwd(dtype, B, H, Lq, Lk, Dh, &c, &cg, stream); });
  MIT_CHECK_ARG(head_dim_ok(Dh), "mit_attention_bwd: head_dim %ld unsupported (16, 32, 64, 128)", Dh);
  if (B <= 0 || H <= 0 || Lq <= 0 || Lk <= 0) return MIT_OK;
  AttnK a = make_k(x);
  AttnG g;
  g.dout = gg->dout; g.do_row = gg->do_row; g.do_batch = gg->do_batch;
  g.dq = gg->dq; g.dq_row = gg->dq_row; g.dq_batch = gg->dq_batch;
  g.dk = gg->dk; g.dk_row = gg->dk_row; g.dk_batch = gg->dk_batch;
  g.dv = gg->dv; g.dv_row = gg->dv_row; g.dv_batch = gg->dv_batch;
  g.delta = gg->delta_ws;
  hipStream_t s = (hipStream_t)stream;
  dim3 gq((unsigned)((Lq + 63) / 64), (unsigned)H, (unsigned)B);
  dim3 gk((unsigned)((Lk + 63) / 64), (unsigned)H, (unsigned)B);
  auto al = [](const void* p, int n) { return ((uintptr_t)p % n) == 0; };
  const bool mfma_ok = Dh == D && dtype == MIT_BF16 && x->q_row % 8 == 0 && x->q_batch % 8 == 0 && x->k_row % 8 == 0 &&
                       x->k_batch % 8 == 0 && x->v_row % 8 == 0 && x->v_batch % 8 == 0 && x->o_row % 8 == 0 &&
                       x->o_batch % 8 == 0 && gg->do_row % 8 == 0 && gg->do_batch % 8 == 0 && gg->dq_row % 4 == 0 &&
                       gg->dq_batch % 4 == 0 && gg->dk_row % 4 == 0 && gg->dk_batch % 4 == 0 && gg->dv_row % 4 == 0 &&
                       gg->dv_batch % 4 == 0 && al(x->q, 16) && al(x->k, 16) && al(x->v, 16) && al(x->o, 16) &&
                       al(gg->dout, 16) && al(gg->dq, 8) && al(gg->dk, 8) && al(gg->dv, 8);
  if (mfma_ok) {
    AttnBwdBytes nb;
    const long qb = 2 * ((Lq - 1) * x->q_row + D), kb = 2 * ((Lk - 1) * x->k_row + D);
    const long vb = 2 * ((Lk - 1) * x->v_row + D), db = 2 * ((Lq - 1) * gg->do_row + D);
    MIT_CHECK_ARG(qb < (1L << 31) && kb < (1L << 31) && vb < (1L << 31) && db < (1L << 31),
                  "mit_attention_bwd: operand span >= 2 GiB");
    nb.q = (int)qb;
    nb.k = (int)kb;
    nb.v = (int)vb;
    nb.dO = (int)db;
    // (the head kernel forms its dropout indices in 32 bits: B * H * Lq * Lk < 2^32)
    if (Lq <= 64 && Lk <= HB_MAXK && H <= 65535 && B <= 65535 && x->o_row % 8 == 0 &&
        (double)B * (double)H * (double)Lq * (double)Lk < g_idx32_limit) {
      const int lkp = (int)((Lk + 31) / 32 * 32);
      const int lds = 2 * lkp * 128 + 2 * 64 * 128 + 2 * 64 * 4;
      static bool attr = false;
      if (!attr) {
        (void)hipFuncSetAttribute((const void*)attn_bwd_head, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  2 * HB_MAXK * 128 + 2 * 64 * 128 + 2 * 64 * 4);
        attr = true;
      }
      hipLaunchKernelGGL(attn_bwd_head, dim3((unsigned)H, (unsigned)B), dim3(HB_NT), lds, s, H, Lq, Lk, a, g, nb, lkp);
    } else {
      hipLaunchKernelGGL(attn_bwd_dq_mfma, gq, dim3(256), 0, s, H, Lq, Lk, a, g, nb);
      hipLaunchKernelGGL(attn_bwd_dkv_mfma, gk, dim3(256), 0, s, H, Lq, Lk, a, g, nb);
    }
  } else if (dtype == MIT_BF16) {
    DISPATCH_DH(Dh, hipLaunchKernelGGL((attn_bwd_dq_simple<bf16, DH>), gq, dim3(64), 0, s, H, Lq, Lk, a, g);
                    hipLaunchKernelGGL((attn_bwd_dkv_simple<bf16, DH>), gk, dim3(64), 0, s, H, Lq, Lk, a, g));
  } else {
    DISPATCH_DH(Dh, hipLaunchKernelGGL((attn_bwd_dq_simple<float, DH>), gq, dim3(64), 0, s, H, Lq, Lk, a, g);
                    hipLaunchKernelGGL((attn_bwd_dkv_simple<float, DH>), gk, dim3(64), 0, s, H, Lq, Lk, a, g));
  }
  MIT_LAUNCH_CHECK("mit_attention_bwd");
  return MIT_OK;
}
