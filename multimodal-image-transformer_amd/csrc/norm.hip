// LayerNorm forward/backward, one wave per row, fp32 statistics.
// Forward fuses the post-LN residual block of torch/nn/modules/transformer.py:1144-1153:
// z = x + dropout(r); y = (z - mean) * rstd * gamma + beta.
#include "common.h"

namespace {
constexpr int MAXV_ALL = 32;  // cols <= 64 * 32 = 2048 (per-lane register arrays sized by template)

template <typename T, int MAXV>
__global__ __launch_bounds__(256) void ln_fwd_kernel(long rows, long cols, const T* __restrict__ x, long ldx,
                                                     const T* __restrict__ r, long ldr, const uint64_t* seed,
                                                     uint32_t site, uint32_t thresh, float dscale, int dropout,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, T* z, T* y, long ldy, float* mean, float* rstd) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float v[MAXV];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const long c = lane + 64 * i;
    float a = 0.f;
    if (c < cols) {
      a = to_f(x[row * ldx + c]);
      if (r) {
        float b = to_f(r[row * ldr + c]);
        if (dropout) b *= drop_mul(key, (uint64_t)row * (uint64_t)cols + c, thresh, dscale);
        a += b;
      }
    }
    v[i] = a;
    s += a;
  }
  const float mu = wave_sum(s) / (float)cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const long c = lane + 64 * i;
    if (c < cols) {
      const float dd = v[i] - mu;
      q += dd * dd;
    }
  }
  const float var = wave_sum(q) / (float)cols;
  const float rs = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const long c = lane + 64 * i;
    if (c < cols) {
      if (z) z[row * cols + c] = from_f<T>(v[i]);
      y[row * ldy + c] = from_f<T>((v[i] - mu) * rs * gamma[c] + beta[c]);
    }
  }
  if (lane == 0) {
    if (mean) mean[row] = mu;
    if (rstd) rstd[row] = rs;
  }
}

constexpr int BWD_ROWS = 32;  // rows per block in the backward (4 waves x 8 rows)

template <typename T, int MAXV>
__global__ __launch_bounds__(256) void ln_bwd_kernel(long rows, long cols, const T* __restrict__ dy,
                                                     const T* __restrict__ z, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, const float* __restrict__ gamma,
                                                     T* dx, T* dr, const uint64_t* seed, uint32_t site, uint32_t thresh,
                                                     float dscale, int dropout, float* ws) {
  __shared__ float red[4][2][64 * 4];  // per-wave partials for up to 256 columns per pass
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float pg[MAXV], pb[MAXV];
#pragma unroll
  for (int i = 0; i < MAXV; ++i) pg[i] = pb[i] = 0.f;
  const long r0 = (long)blockIdx.x * BWD_ROWS;
  for (int rr = w; rr < BWD_ROWS; rr += 4) {
    const long row = r0 + rr;
    if (row >= rows) break;
    const float mu = mean[row], rs = rstd[row];
    float g[MAXV], xh[MAXV];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const long c = lane + 64 * i;
      g[i] = xh[i] = 0.f;
      if (c < cols) {
        const float d = to_f(dy[row * cols + c]);
        xh[i] = (to_f(z[row * cols + c]) - mu) * rs;
        g[i] = d * gamma[c];
        pg[i] += d * xh[i];
        pb[i] += d;
        s1 += g[i];
        s2 += g[i] * xh[i];
      }
    }
    s1 = wave_sum(s1) / (float)cols;
    s2 = wave_sum(s2) / (float)cols;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
      const long c = lane + 64 * i;
      if (c < cols) {
        const float d = rs * (g[i] - s1 - xh[i] * s2);
        dx[row * cols + c] = from_f<T>(d);
        if (dr) {
          const float m = dropout ? drop_mul(key, (uint64_t)row * (uint64_t)cols + c, thresh, dscale) : 1.0f;
          dr[row * cols + c] = from_f<T>(d * m);
        }
      }
    }
  }
  // reduce the 4 waves' column partials, 4 column-groups of 64 at a time
#pragma unroll
  for (int base = 0; base < MAXV; base += 4) {
    if (base * 64 >= cols) continue;  // uniform
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      red[w][0][k * 64 + lane] = (base + k < MAXV) ? pg[(base + k) < MAXV ? base + k : 0] : 0.f;
      red[w][1][k * 64 + lane] = (base + k < MAXV) ? pb[(base + k) < MAXV ? base + k : 0] : 0.f;
    }
    __syncthreads();
    // 256 threads: thread t -> column group (t>>6), lane column
    {
      const int k = threadIdx.x >> 6;
      const long c = (long)(base + k) * 64 + lane;
      if (c < cols) {
        float a = red[0][0][k * 64 + lane] + red[1][0][k * 64 + lane] + red[2][0][k * 64 + lane] + red[3][0][k * 64 + lane];
        float b = red[0][1][k * 64 + lane] + red[1][1][k * 64 + lane] + red[2][1][k * 64 + lane] + red[3][1][k * 64 + lane];
        ws[(long)blockIdx.x * 2 * cols + c] = a;
        ws[(long)blockIdx.x * 2 * cols + cols + c] = b;
      }
    }
    __syncthreads();
  }
}

__global__ void ln_param_reduce(long nblk, long cols, const float* __restrict__ ws, float* dgamma, float* dbeta) {
  const long c = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= 2 * cols) return;
  float s = 0.f;
  for (long b = 0; b < nblk; ++b) s += ws[b * 2 * cols + c];
  if (c < cols) dgamma[c] = s;
  else dbeta[c - cols] = s;
}
}  // namespace

extern "C" int mit_layernorm_fwd(int dtype, long rows, long cols, const void* x, long ldx, const void* r, long ldr,
                                 float r_drop_p, const uint64_t* seed, uint32_t site, const float* gamma,
                                 const float* beta, float eps, void* z, void* y, long ldy, float* mean, float* rstd,
                                 void* stream) {
  MIT_CHECK_ARG(cols > 0 && cols <= 64 * MAXV_ALL, "mit_layernorm_fwd: cols %ld out of range", cols);
  MIT_CHECK_ARG(x && y && gamma && beta, "mit_layernorm_fwd: null pointer");
  MIT_CHECK_ARG(ldx >= cols && ldy >= cols && (!r || ldr >= cols), "mit_layernorm_fwd: bad leading dim");
  if (rows <= 0) return MIT_OK;
  const int dropout = (r != nullptr) && r_drop_p > 0.f;
  const uint32_t th = drop_threshold(r_drop_p);
  const float sc = r_drop_p < 1.f ? 1.f / (1.f - r_drop_p) : 0.f;
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
#define LNF(T, NV)                                                                                              \
  hipLaunchKernelGGL((ln_fwd_kernel<T, NV>), grid, dim3(256), 0, s, rows, cols, (const T*)x, ldx, (const T*)r, ldr, \
                     seed, site, th, sc, dropout, gamma, beta, eps, (T*)z, (T*)y, ldy, mean, rstd)
#define LNF_DT(T)                 \
  if (cols <= 128) LNF(T, 2);     \
  else if (cols <= 256) LNF(T, 4); \
  else if (cols <= 512) LNF(T, 8); \
  else if (cols <= 1024) LNF(T, 16); \
  else LNF(T, 32);
  if (dtype == MIT_BF16) { LNF_DT(bf16) } else { LNF_DT(float) }
#undef LNF_DT
#undef LNF
  MIT_LAUNCH_CHECK("mit_layernorm_fwd");
  return MIT_OK;
}

extern "C" long mit_layernorm_bwd_ws_floats(long rows, long cols) {
  return ((rows + BWD_ROWS - 1) / BWD_ROWS) * 2 * cols;
}

extern "C" int mit_layernorm_bwd(int dtype, long rows, long cols, const void* dy, const void* z, const float* mean,
                                 const float* rstd, const float* gamma, void* dx, void* dr, float r_drop_p,
                                 const uint64_t* seed, uint32_t site, float* dgamma, float* dbeta, float* ws,
                                 void* stream) {
  MIT_CHECK_ARG(cols > 0 && cols <= 64 * MAXV_ALL, "mit_layernorm_bwd: cols %ld out of range", cols);
  MIT_CHECK_ARG(dy && z && mean && rstd && gamma && dx && dgamma && dbeta && ws, "mit_layernorm_bwd: null pointer");
  if (rows <= 0) return MIT_OK;
  const int dropout = r_drop_p > 0.f;
  const uint32_t th = drop_threshold(r_drop_p);
  const float sc = r_drop_p < 1.f ? 1.f / (1.f - r_drop_p) : 0.f;
  const long nblk = (rows + BWD_ROWS - 1) / BWD_ROWS;
  hipStream_t s = (hipStream_t)stream;
#define LNB(T, NV)                                                                                          \
  hipLaunchKernelGGL((ln_bwd_kernel<T, NV>), dim3((unsigned)nblk), dim3(256), 0, s, rows, cols, (const T*)dy, \
                     (const T*)z, mean, rstd, gamma, (T*)dx, (T*)dr, seed, site, th, sc, dropout, ws)
#define LNB_DT(T)                 \
  if (cols <= 128) LNB(T, 2);     \
  else if (cols <= 256) LNB(T, 4); \
  else if (cols <= 512) LNB(T, 8); \
  else if (cols <= 1024) LNB(T, 16); \
  else LNB(T, 32);
  if (dtype == MIT_BF16) { LNB_DT(bf16) } else { LNB_DT(float) }
#undef LNB_DT
#undef LNB
  MIT_LAUNCH_CHECK("mit_layernorm_bwd");
  hipLaunchKernelGGL(ln_param_reduce, dim3((unsigned)((2 * cols + 255) / 256)), dim3(256), 0, s, nblk, cols, ws, dgamma,
                     dbeta);
  MIT_LAUNCH_CHECK("mit_layernorm_bwd(reduce)");
  return MIT_OK;
}
