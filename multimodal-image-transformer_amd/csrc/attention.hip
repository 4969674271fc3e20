// Scaled-dot-product attention, head_dim 64.
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
// simple forward
// ------------------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(64) void attn_fwd_simple(long H, long Lq, long Lk, AttnK a) {
  __shared__ float Ks[64][D + 1];
  __shared__ float Vs[64][D + 1];
  const int tid = threadIdx.x;
  const long b = blockIdx.z, h = blockIdx.y, i = (long)blockIdx.x * 64 + tid;
  const bool live = i < Lq;
  const T* Q = (const T*)a.q + b * a.q_batch + h * D;
  const T* K = (const T*)a.k + b * a.k_batch + h * D;
  const T* V = (const T*)a.v + b * a.v_batch + h * D;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const uint64_t rowbase = ((uint64_t)(b * H + h) * (uint64_t)Lq + (uint64_t)i) * (uint64_t)Lk;
  float q[D], o[D];
#pragma unroll
  for (int d = 0; d < D; ++d) {
    q[d] = live ? to_f(Q[i * a.q_row + d]) * a.scale : 0.f;
    o[d] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (long j0 = 0; j0 < Lk; j0 += 64) {
    const int nj = (int)min((long)64, Lk - j0);
    __syncthreads();
    for (int idx = tid; idx < 64 * D; idx += 64) {
      const int r = idx / D, c = idx % D;
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
    float s[64];
    float tmax = -INFINITY;
#pragma unroll
    for (int jj = 0; jj < 64; ++jj) {
      float acc = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) acc = fmaf(q[d], Ks[jj][d], acc);
      const bool msk = (jj >= nj) || key_masked(a, b, i, j0 + jj);
      s[jj] = msk ? -INFINITY : acc;
      tmax = fmaxf(tmax, s[jj]);
    }
    const float mnew = fmaxf(m, tmax);
    const float corr = (mnew == -INFINITY) ? 1.f : __expf(m - mnew);
    l *= corr;
#pragma unroll
    for (int d = 0; d < D; ++d) o[d] *= corr;
#pragma unroll
    for (int jj = 0; jj < 64; ++jj) {
      const float p = (s[jj] == -INFINITY) ? 0.f : __expf(s[jj] - mnew);
      l += p;
      float pd = p;
      if (a.dropout) pd *= drop_mul(key, rowbase + (uint64_t)(j0 + jj), a.thresh, a.dscale);
      if (pd != 0.f) {
#pragma unroll
        for (int d = 0; d < D; ++d) o[d] = fmaf(pd, Vs[jj][d], o[d]);
      }
    }
    m = mnew;
  }
  if (!live) return;
  const float inv = 1.0f / l;  // l == 0 (fully masked row) -> inf * 0 = NaN, as the reference
  T* O = (T*)a.o + b * a.o_batch + i * a.o_row + h * D;
#pragma unroll
  for (int d = 0; d < D; ++d) O[d] = from_f<T>(o[d] * inv);
  if (a.lse) a.lse[(b * H + h) * Lq + i] = m + __logf(l);
}

// ------------------------------------------------------------------------------------------------
// simple backward: (1) dQ + delta, thread per query; (2) dK/dV, thread per key
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

template <typename T>
__global__ __launch_bounds__(64) void attn_bwd_dq_simple(long H, long Lq, long Lk, AttnK a, AttnG g) {
  __shared__ float Ks[64][D + 1];
  __shared__ float Vs[64][D + 1];
  const int tid = threadIdx.x;
  const long b = blockIdx.z, h = blockIdx.y, i = (long)blockIdx.x * 64 + tid;
  const bool live = i < Lq;
  const T* Q = (const T*)a.q + b * a.q_batch + h * D;
  const T* K = (const T*)a.k + b * a.k_batch + h * D;
  const T* V = (const T*)a.v + b * a.v_batch + h * D;
  const T* O = (const T*)a.o + b * a.o_batch + h * D;
  const T* dO = (const T*)g.dout + b * g.do_batch + h * D;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  const uint64_t rowbase = ((uint64_t)(b * H + h) * (uint64_t)Lq + (uint64_t)i) * (uint64_t)Lk;
  float q[D], dout[D], dq[D];
  float delta = 0.f, lse = 0.f;
  if (live) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
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
    for (int idx = tid; idx < 64 * D; idx += 64) {
      const int r = idx / D, c = idx % D;
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
      for (int d = 0; d < D; ++d) {
        s = fmaf(q[d], Ks[jj][d], s);
        dp = fmaf(dout[d], Vs[jj][d], dp);
      }
      const float p = __expf(s * a.scale - lse);
      if (a.dropout) dp *= drop_mul(key, rowbase + (uint64_t)(j0 + jj), a.thresh, a.dscale);
      const float ds = p * (dp - delta);
#pragma unroll
      for (int d = 0; d < D; ++d) dq[d] = fmaf(ds, Ks[jj][d], dq[d]);
    }
  }
  if (!live) return;
  T* DQ = (T*)g.dq + b * g.dq_batch + i * g.dq_row + h * D;
#pragma unroll
  for (int d = 0; d < D; ++d) DQ[d] = from_f<T>(dq[d] * a.scale);
}

template <typename T>
__global__ __launch_bounds__(64) void attn_bwd_dkv_simple(long H, long Lq, long Lk, AttnK a, AttnG g) {
  __shared__ float Kp[64][D + 1];  // this block's keys, one private row per thread
  __shared__ float Vp[64][D + 1];
  __shared__ float Qs[64][D + 1];  // query tile (broadcast reads)
  __shared__ float Ds[64][D + 1];  // dO tile
  __shared__ float Ls[64], Dl[64];
  const int tid = threadIdx.x;
  const long b = blockIdx.z, h = blockIdx.y, j = (long)blockIdx.x * 64 + tid;
  const bool live = j < Lk;
  const T* Q = (const T*)a.q + b * a.q_batch + h * D;
  const T* K = (const T*)a.k + b * a.k_batch + h * D;
  const T* V = (const T*)a.v + b * a.v_batch + h * D;
  const T* dO = (const T*)g.dout + b * g.do_batch + h * D;
  const uint64_t key = a.dropout ? site_key(a.seed, a.site) : 0ull;
  for (int idx = tid; idx < 64 * D; idx += 64) {
    const int r = idx / D, c = idx % D;
    const long jj = (long)blockIdx.x * 64 + r;
    Kp[r][c] = jj < Lk ? to_f(K[jj * a.k_row + c]) : 0.f;
    Vp[r][c] = jj < Lk ? to_f(V[jj * a.v_row + c]) : 0.f;
  }
  const bool kpad = live && a.tok && a.tok[b * a.tok_batch + j] == a.pad;
  float dk[D], dv[D];
#pragma unroll
  for (int d = 0; d < D; ++d) dk[d] = dv[d] = 0.f;
  for (long i0 = 0; i0 < Lq; i0 += 64) {
    const int ni = (int)min((long)64, Lq - i0);
    __syncthreads();
    for (int idx = tid; idx < 64 * D; idx += 64) {
      const int r = idx / D, c = idx % D;
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
      for (int d = 0; d < D; ++d) {
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
      for (int d = 0; d < D; ++d) {
        dv[d] = fmaf(pd, Ds[ii][d], dv[d]);
        dk[d] = fmaf(ds, Qs[ii][d], dk[d]);
      }
    }
  }
  if (!live) return;
  T* DK = (T*)g.dk + b * g.dk_batch + j * g.dk_row + h * D;
  T* DV = (T*)g.dv + b * g.dv_batch + j * g.dv_row + h * D;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    DK[d] = from_f<T>(dk[d] * a.scale);
    DV[d] = from_f<T>(dv[d]);
  }
}

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


extern "C" int mit_attention_fwd(int dtype, long B, long H, long Lq, long Lk, long Dh, const mit_attn_args* x,
                                 void* stream) {
  MIT_CHECK_ARG(x && x->q && x->k && x->v && x->o, "mit_attention_fwd: null pointer");
  MIT_CHECK_ARG(Dh == D, "mit_attention_fwd: head_dim %ld unsupported (64 only)", Dh);
  if (B <= 0 || H <= 0 || Lq <= 0) return MIT_OK;
  MIT_CHECK_ARG(Lk > 0, "mit_attention_fwd: Lk must be > 0");
  AttnK a = make_k(x);
  hipStream_t s = (hipStream_t)stream;
  dim3 grid((unsigned)((Lq + 63) / 64), (unsigned)H, (unsigned)B);
  if (dtype == MIT_BF16)
    hipLaunchKernelGGL(attn_fwd_simple<bf16>, grid, dim3(64), 0, s, H, Lq, Lk, a);
  else
    hipLaunchKernelGGL(attn_fwd_simple<float>, grid, dim3(64), 0, s, H, Lq, Lk, a);
  MIT_LAUNCH_CHECK("mit_attention_fwd");
  return MIT_OK;
}

extern "C" int mit_attention_bwd(int dtype, long B, long H, long Lq, long Lk, long Dh, const mit_attn_args* x,
                                 const mit_attn_grads* gg, void* stream) {
  MIT_CHECK_ARG(x && gg && x->q && x->k && x->v && x->o && x->lse, "mit_attention_bwd: null forward pointer");
  MIT_CHECK_ARG(gg->dout && gg->dq && gg->dk && gg->dv && gg->delta_ws, "mit_attention_bwd: null grad pointer");
  MIT_CHECK_ARG(Dh == D, "mit_attention_bwd: head_dim %ld unsupported (64 only)", Dh);
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
  if (dtype == MIT_BF16) {
    hipLaunchKernelGGL(attn_bwd_dq_simple<bf16>, gq, dim3(64), 0, s, H, Lq, Lk, a, g);
    hipLaunchKernelGGL(attn_bwd_dkv_simple<bf16>, gk, dim3(64), 0, s, H, Lq, Lk, a, g);
  } else {
    hipLaunchKernelGGL(attn_bwd_dq_simple<float>, gq, dim3(64), 0, s, H, Lq, Lk, a, g);
    hipLaunchKernelGGL(attn_bwd_dkv_simple<float>, gk, dim3(64), 0, s, H, Lq, Lk, a, g);
  }
  MIT_LAUNCH_CHECK("mit_attention_bwd");
  return MIT_OK;
}
