// LayerNorm forward/backward, one wave per row, fp32 statistics.
// Forward fuses the post-LN residual block of torch/nn/modules/transformer.py:1144-1153:
//   z = x + dropout(r); y = (z - mean) * rstd * gamma + beta.
// Rows are read as 4-element vectors (8 B bf16 / 16 B f32 per lane) when cols % 256 == 0
// (512, 768, 1024 — every production width), else element by element.
// Backward: dz = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = dy * gamma; dgamma/dbeta are
// reduced in two stages (16-row block partials in registers + LDS, then a column-parallel pass).
#include "common.h"

namespace {
constexpr int MAXV_ALL = 32;  // cols <= 64 * 32 = 2048

template <typename T>
struct Vec4;
template <>
struct Vec4<bf16> {
  typedef __attribute__((ext_vector_type(4))) __bf16 type;
};
template <>
struct Vec4<float> {
  typedef f32x4 type;
};

template <typename T>
__device__ __forceinline__ void ld4(const T* p, float* v) {
  const typename Vec4<T>::type x = *(const typename Vec4<T>::type*)p;
  v[0] = (float)x[0];
  v[1] = (float)x[1];
  v[2] = (float)x[2];
  v[3] = (float)x[3];
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const float* v) {
  typename Vec4<T>::type x;
  x[0] = (T)v[0];
  x[1] = (T)v[1];
  x[2] = (T)v[2];
  x[3] = (T)v[3];
  *(typename Vec4<T>::type*)p = x;
}

// element (lane, i, k) of a row: column = (i * 64 + lane) * 4 + k   when VEC; lane + 64 * i otherwise
template <bool VEC>
__device__ __forceinline__ long colof(int lane, int i, int k) {
  return VEC ? (long)(i * 64 + lane) * 4 + k : (long)lane + 64 * i;
}

template <typename T, int NV, bool VEC>
__global__ __launch_bounds__(256) void ln_fwd_kernel(long rows, long cols, const T* __restrict__ x, long ldx,
                                                     const T* __restrict__ r, long ldr, const uint64_t* seed,
                                                     uint32_t site, uint32_t thresh, float dscale, int dropout,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, T* z, T* y, long ldy, float* mean, float* rstd) {
  constexpr int E = VEC ? 4 : 1;  // elements per (lane, i)
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float v[NV][E];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long c0 = colof<VEC>(lane, i, 0);
    if (c0 >= cols) {
#pragma unroll
      for (int k = 0; k < E; ++k) v[i][k] = 0.f;
      continue;
    }
    float a[E], b[E];
    if (VEC) {
      ld4(x + row * ldx + c0, a);
      if (r) ld4(r + row * ldr + c0, b);
    } else {
      a[0] = to_f(x[row * ldx + c0]);
      if (r) b[0] = to_f(r[row * ldr + c0]);
    }
#pragma unroll
    for (int k = 0; k < E; ++k) {
      if (r) {
        if (dropout) b[k] *= drop_mul(key, (uint64_t)row * (uint64_t)cols + c0 + k, thresh, dscale);
        a[k] += b[k];
      }
      v[i][k] = a[k];
      s += a[k];
    }
  }
  const float mu = wave_sum(s) / (float)cols;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
    if (colof<VEC>(lane, i, 0) < cols) {
#pragma unroll
      for (int k = 0; k < E; ++k) {
        const float dd = v[i][k] - mu;
        q += dd * dd;
      }
    }
  const float var = wave_sum(q) / (float)cols;
  const float rs = rsqrtf(var + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long c0 = colof<VEC>(lane, i, 0);
    if (c0 >= cols) continue;
    float o[E];
    if (VEC) {
      const f32x4 g4 = *(const f32x4*)(gamma + c0), b4 = *(const f32x4*)(beta + c0);
#pragma unroll
      for (int k = 0; k < E; ++k) o[k] = (v[i][k] - mu) * rs * g4[k] + b4[k];
      if (z) st4(z + row * cols + c0, v[i]);
      st4(y + row * ldy + c0, o);
    } else {
      o[0] = (v[i][0] - mu) * rs * gamma[c0] + beta[c0];
      if (z) z[row * cols + c0] = from_f<T>(v[i][0]);
      y[row * ldy + c0] = from_f<T>(o[0]);
    }
  }
  if (lane == 0) {
    if (mean) mean[row] = mu;
    if (rstd) rstd[row] = rs;
  }
}

constexpr int BWD_ROWS = 8;  // rows per block in the backward (4 waves x 2 rows)
constexpr int BWD_RPW = BWD_ROWS / 4;

template <typename T, int NV, bool VEC>
__global__ __launch_bounds__(256) void ln_bwd_kernel(long rows, long cols, const T* dy, const T* __restrict__ z,
                                                     const float* __restrict__ mean, const float* __restrict__ rstd,
                                                     const float* __restrict__ gamma, T* dx, T* dr, const uint64_t* seed,
                                                     uint32_t site, uint32_t thresh, float dscale, int dropout,
                                                     float* ws) {
  constexpr int E = VEC ? 4 : 1;
  __shared__ float red[4][2][256];  // per-wave column partials, 256 columns per pass
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float pg[NV][E], pb[NV][E];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < E; ++k) pg[i][k] = pb[i][k] = 0.f;
  const long r0 = (long)blockIdx.x * BWD_ROWS;
  // every row of this wave is requested before any is reduced: the row-at-a-time form was bound
  // by one load round trip per row (12.8 us for 4032 x 512 at 16 rows per block)
  float dd[BWD_RPW][NV][E], zv[BWD_RPW][NV][E], mus[BWD_RPW], rss[BWD_RPW];
#pragma unroll
  for (int j = 0; j < BWD_RPW; ++j) {
    const long row = r0 + w + 4 * j;
    const bool live = row < rows;
    mus[j] = live ? mean[row] : 0.f;
    rss[j] = live ? rstd[row] : 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = colof<VEC>(lane, i, 0);
      if (live && c0 < cols) {
        if (VEC) {
          ld4(dy + row * cols + c0, dd[j][i]);
          ld4(z + row * cols + c0, zv[j][i]);
        } else {
          dd[j][i][0] = to_f(dy[row * cols + c0]);
          zv[j][i][0] = to_f(z[row * cols + c0]);
        }
      } else {
#pragma unroll
        for (int k = 0; k < E; ++k) dd[j][i][k] = zv[j][i][k] = 0.f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < BWD_RPW; ++j) {
    const long row = r0 + w + 4 * j;
    if (row >= rows) break;
    const float mu = mus[j], rs = rss[j];
    float g[NV][E], xh[NV][E];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = colof<VEC>(lane, i, 0);
      float ga[E];
      if (c0 < cols) {
        if (VEC) {
          const f32x4 g4 = *(const f32x4*)(gamma + c0);
#pragma unroll
          for (int k = 0; k < E; ++k) ga[k] = g4[k];
        } else {
          ga[0] = gamma[c0];
        }
      } else {
#pragma unroll
        for (int k = 0; k < E; ++k) ga[k] = 0.f;
      }
#pragma unroll
      for (int k = 0; k < E; ++k) {
        const float d = dd[j][i][k];
        xh[i][k] = (c0 < cols) ? (zv[j][i][k] - mu) * rs : 0.f;
        g[i][k] = d * ga[k];
        pg[i][k] += d * xh[i][k];
        pb[i][k] += d;
        s1 += g[i][k];
        s2 += g[i][k] * xh[i][k];
      }
    }
    s1 = wave_sum(s1) / (float)cols;
    s2 = wave_sum(s2) / (float)cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = colof<VEC>(lane, i, 0);
      if (c0 >= cols) continue;
      float o[E], om[E];
#pragma unroll
      for (int k = 0; k < E; ++k) {
        o[k] = rs * (g[i][k] - s1 - xh[i][k] * s2);
        om[k] = dropout ? o[k] * drop_mul(key, (uint64_t)row * (uint64_t)cols + c0 + k, thresh, dscale) : o[k];
      }
      if (VEC) {
        st4(dx + row * cols + c0, o);
        if (dr) st4(dr + row * cols + c0, om);
      } else {
        dx[row * cols + c0] = from_f<T>(o[0]);
        if (dr) dr[row * cols + c0] = from_f<T>(om[0]);
      }
    }
  }
  // reduce the 4 waves' column partials (one (lane, i) slot = E columns); 256 columns per pass
  constexpr int SLOTS_PER_PASS = 256 / (64 * E);  // i-values per pass
#pragma unroll
  for (int base = 0; base < NV; base += SLOTS_PER_PASS) {
#pragma unroll
    for (int s = 0; s < SLOTS_PER_PASS; ++s)
#pragma unroll
      for (int k = 0; k < E; ++k) {
        const int li = (base + s < NV) ? base + s : 0;
        const int slot = (s * 64 + lane) * E + k;
        red[w][0][slot] = (base + s < NV) ? pg[li][k] : 0.f;
        red[w][1][slot] = (base + s < NV) ? pb[li][k] : 0.f;
      }
    __syncthreads();
    {
      const int slot = threadIdx.x;  // 0..255 -> (s, lane, k)
      const int k = slot % E, l2 = (slot / E) % 64, s = slot / (64 * E);
      const long c = colof<VEC>(l2, base + s, k);
      if (base + s < NV && c < cols) {
        const float a = red[0][0][slot] + red[1][0][slot] + red[2][0][slot] + red[3][0][slot];
        const float b = red[0][1][slot] + red[1][1][slot] + red[2][1][slot] + red[3][1][slot];
        ws[(long)blockIdx.x * 2 * cols + c] = a;
        ws[(long)blockIdx.x * 2 * cols + cols + c] = b;
      }
    }
    __syncthreads();
  }
}

// bf16 backward with 16-B loads / stores (8 columns per lane per 512-column pass, cols % 8 == 0,
// cols <= 1024); same row mapping (BWD_ROWS rows per block, BWD_RPW per wave) and the same ws layout
// of per-block column partials as ln_bwd_kernel (512 columns per LDS reduction pass)
template <int NV>
__global__ __launch_bounds__(256) void ln_bwd_wide_kernel(long rows, long cols, const bf16* dy, const bf16* __restrict__ z,
                                                          const float* __restrict__ mean, const float* __restrict__ rstd,
                                                          const float* __restrict__ gamma, bf16* dx, bf16* dr,
                                                          const uint64_t* seed, uint32_t site, uint32_t thresh,
                                                          float dscale, int dropout, float* ws) {
  __shared__ float red[4][2][512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float pg[NV][8], pb[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < 8; ++k) pg[i][k] = pb[i][k] = 0.f;
  const long r0 = (long)blockIdx.x * BWD_ROWS;
  bf16x8 dd[BWD_RPW][NV], zv[BWD_RPW][NV];
  float mus[BWD_RPW], rss[BWD_RPW];
#pragma unroll
  for (int j = 0; j < BWD_RPW; ++j) {
    const long row = r0 + w + 4 * j;
    const bool live = row < rows;
    mus[j] = live ? mean[row] : 0.f;
    rss[j] = live ? rstd[row] : 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = (long)(i * 64 + lane) * 8;
      const bool ok = live && c0 < cols;
      dd[j][i] = ok ? *(const bf16x8*)(dy + row * cols + c0) : bf16x8{};
      zv[j][i] = ok ? *(const bf16x8*)(z + row * cols + c0) : bf16x8{};
    }
  }
#pragma unroll
  for (int j = 0; j < BWD_RPW; ++j) {
    const long row = r0 + w + 4 * j;
    if (row >= rows) break;
    const float mu = mus[j], rs = rss[j];
    float g[NV][8], xh[NV][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = (long)(i * 64 + lane) * 8;
      const bool ok = c0 < cols;
      const f32x4 g0 = ok ? *(const f32x4*)(gamma + c0) : f32x4{}, g1 = ok ? *(const f32x4*)(gamma + c0 + 4) : f32x4{};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float d = (float)dd[j][i][k];
        const float ga = k < 4 ? g0[k] : g1[k - 4];
        xh[i][k] = ok ? ((float)zv[j][i][k] - mu) * rs : 0.f;
        g[i][k] = d * ga;
        pg[i][k] += d * xh[i][k];
        pb[i][k] += d;
        s1 += g[i][k];
        s2 += g[i][k] * xh[i][k];
      }
    }
    s1 = wave_sum(s1) / (float)cols;
    s2 = wave_sum(s2) / (float)cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = (long)(i * 64 + lane) * 8;
      if (c0 >= cols) continue;
      bf16x8 o, om;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float v = rs * (g[i][k] - s1 - xh[i][k] * s2);
        o[k] = (bf16)v;
        om[k] = (bf16)(dropout ? v * drop_mul(key, (uint64_t)row * (uint64_t)cols + c0 + k, thresh, dscale) : v);
      }
      *(bf16x8*)(dx + row * cols + c0) = o;
      if (dr) *(bf16x8*)(dr + row * cols + c0) = om;
    }
  }
  // the 4 waves' column partials: one 512-column pass per i, 2 columns per thread
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[w][0][lane * 8 + k] = pg[i][k];
      red[w][1][lane * 8 + k] = pb[i][k];
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int slot = threadIdx.x + 256 * h;
      const long c = (long)i * 512 + slot;
      if (c < cols) {
        const float a = red[0][0][slot] + red[1][0][slot] + red[2][0][slot] + red[3][0][slot];
        const float b = red[0][1][slot] + red[1][1][slot] + red[2][1][slot] + red[3][1][slot];
        ws[(long)blockIdx.x * 2 * cols + c] = a;
        ws[(long)blockIdx.x * 2 * cols + cols + c] = b;
      }
    }
    __syncthreads();
  }
}

// column-parallel sum of the block partials: 16 columns x 16 strided partial-row groups per block
// (at 4032 rows x 512 columns: 252 partial rows, 64 blocks, 16 loads in flight per thread), then a
// fixed-order LDS reduction over the groups (deterministic)
__global__ __launch_bounds__(256) void ln_param_reduce(long nblk, long cols, const float* __restrict__ ws,
                                                       float* dgamma, float* dbeta) {
  __shared__ float part[16][17];
  const int cl = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const long c = (long)blockIdx.x * 16 + cl;
  float s = 0.f;
  if (c < 2 * cols) {
    long b = grp;
    for (; b + 48 < nblk; b += 64)
      s += (ws[b * 2 * cols + c] + ws[(b + 16) * 2 * cols + c]) +
           (ws[(b + 32) * 2 * cols + c] + ws[(b + 48) * 2 * cols + c]);
    for (; b < nblk; b += 16) s += ws[b * 2 * cols + c];
  }
  part[grp][cl] = s;
  __syncthreads();
  if (grp == 0 && c < 2 * cols) {
    float t = 0.f;
#pragma unroll
    for (int g = 0; g < 16; ++g) t += part[g][cl];
    if (c < cols) dgamma[c] = t;
    else dbeta[c - cols] = t;
  }
}

template <typename T, bool VEC, typename F>
void dispatch_nv(long cols, F&& f) {
  const long per = VEC ? 256 : 64;
  const long nv = (cols + per - 1) / per;
  if (nv <= 1) f(std::integral_constant<int, 1>());
  else if (nv <= 2) f(std::integral_constant<int, 2>());
  else if (nv <= 3) f(std::integral_constant<int, 3>());
  else if (nv <= 4) f(std::integral_constant<int, 4>());
  else if (nv <= 8) f(std::integral_constant<int, 8>());
  else if (nv <= 16) f(std::integral_constant<int, 16>());
  else f(std::integral_constant<int, 32>());
}
// bf16 rows with cols % 8 == 0, cols <= 1024 (every production width: 128 .. 1024): 16-B loads and
// stores (8 columns per lane per 512-column pass) and RW rows per wave, all their loads issued before
// the first reduction -- the 8-B-per-lane form moved 38.8 MB per encoder LayerNorm at ~3.5 TB/s
// 8 consecutive columns of a row as floats: one 16-B bf16x8 load or two 16-B f32x4 loads
__device__ __forceinline__ void ld8(const bf16* p, float* v) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = (float)x[k];
}
__device__ __forceinline__ void ld8(const float* p, float* v) {
  const f32x4 a = *(const f32x4*)p, b = *(const f32x4*)(p + 4);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = a[k];
    v[k + 4] = b[k];
  }
}
__device__ __forceinline__ void st8(bf16* p, const float* v) {
  bf16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
  *(bf16x8*)p = o;
}
__device__ __forceinline__ void st8(float* p, const float* v) {
  *(f32x4*)p = f32x4{v[0], v[1], v[2], v[3]};
  *(f32x4*)(p + 4) = f32x4{v[4], v[5], v[6], v[7]};
}

// wide rows (cols % 8 == 0, cols <= 1024), 8 columns per lane per 512-column pass, RW rows per wave,
// every load of the wave's rows issued before the first reduction (so z may alias x: each lane reads
// its elements before it writes them). TX / TY / TR = input (and z) / output / residual element type:
// bf16 throughout (the 8-B-per-lane form moved 38.8 MB per encoder LayerNorm at ~3.5 TB/s), or the
// encoder's f32 residual stream (TX = float) plus a bf16 sublayer output r (TR = bf16), normalised
// into bf16 or f32 (TY)
template <int NV, int RW, bool HASR, typename TX = bf16, typename TY = bf16, typename TR = TX>
__global__ __launch_bounds__(256) void ln_fwd_wide_kernel(long rows, long cols, const TX* x, long ldx,
                                                          const TR* __restrict__ r, long ldr, const uint64_t* seed,
                                                          uint32_t site, uint32_t thresh, float dscale, int dropout,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, TX* z, TY* y,
                                                          long ldy, float* mean, float* rstd) {
  const int lane = threadIdx.x & 63;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * RW;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float xa[RW][NV][8], ra[HASR ? RW : 1][NV][HASR ? 8 : 1];
#pragma unroll
  for (int q = 0; q < RW; ++q)
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = (long)(i * 64 + lane) * 8, row = row0 + q;
      const bool ok = row < rows && c0 < cols;
      if (ok) {
        ld8(x + row * ldx + c0, xa[q][i]);
        if (HASR) ld8(r + row * ldr + c0, ra[q][i]);
      } else {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xa[q][i][k] = 0.f;
          if (HASR) ra[q][i][k] = 0.f;
        }
      }
    }
#pragma unroll
  for (int q = 0; q < RW; ++q) {
    const long row = row0 + q;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = (long)(i * 64 + lane) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float a = xa[q][i][k];
        if (HASR) {
          float b = ra[q][i][k];
          if (dropout) b *= drop_mul(key, (uint64_t)row * (uint64_t)cols + c0 + k, thresh, dscale);
          a += b;
        }
        v[i][k] = c0 < cols ? a : 0.f;
        s += v[i][k];
      }
    }
    const float mu = wave_sum(s) / (float)cols;
    float qq = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
      if ((long)(i * 64 + lane) * 8 < cols) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dd = v[i][k] - mu;
          qq += dd * dd;
        }
      }
    const float rs = rsqrtf(wave_sum(qq) / (float)cols + eps);
    if (row >= rows) continue;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const long c0 = (long)(i * 64 + lane) * 8;
      if (c0 >= cols) continue;
      const f32x4 g0 = *(const f32x4*)(gamma + c0), g1 = *(const f32x4*)(gamma + c0 + 4);
      const f32x4 b0 = *(const f32x4*)(beta + c0), b1 = *(const f32x4*)(beta + c0 + 4);
      float o[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        o[k] = (v[i][k] - mu) * rs * g0[k] + b0[k];
        o[k + 4] = (v[i][k + 4] - mu) * rs * g1[k] + b1[k];
      }
      if (z) st8(z + row * cols + c0, v[i]);
      st8(y + row * ldy + c0, o);
    }
    if (lane == 0) {
      if (mean) mean[row] = mu;
      if (rstd) rstd[row] = rs;
    }
  }
}

// Two rows per wave packed into whole 16-B chunks: a row of C = cols / 8 chunks, the wave's 2C chunks
// spread over NV = 2C / 64 passes of all 64 lanes (cols 768: 3 passes, every lane busy; the one-row
// form runs its second pass on half the lanes). Chunk j of the pair belongs to row j >= C; the two
// rows' sums are two wave reductions over lane-selected partials. bf16 in / out.
template <int NV, bool HASR>
__global__ __launch_bounds__(256) void ln_fwd_pair_kernel(long rows, long cols, const bf16* x, long ldx,
                                                          const bf16* __restrict__ r, long ldr, const uint64_t* seed,
                                                          uint32_t site, uint32_t thresh, float dscale, int dropout,
                                                          const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, bf16* z, bf16* y,
                                                          long ldy, float* mean, float* rstd) {
  const int lane = threadIdx.x & 63;
  const long C = cols >> 3;
  const long row0 = ((long)blockIdx.x * 4 + (threadIdx.x >> 6)) * 2;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  float v[NV][8];
  bool hi[NV], ok[NV];
  long cc[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const long j = i * 64 + lane;
    hi[i] = j >= C;
    cc[i] = (j - (hi[i] ? C : 0)) * 8;
    const long row = row0 + (hi[i] ? 1 : 0);
    ok[i] = row < rows;
    float ra[HASR ? 8 : 1];
    if (ok[i]) {
      ld8(x + row * ldx + cc[i], v[i]);
      if (HASR) ld8(r + row * ldr + cc[i], ra);
    } else {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[i][k] = 0.f;
    }
    if (HASR && ok[i]) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float b = ra[k];
        if (dropout) b *= drop_mul(key, (uint64_t)row * (uint64_t)cols + cc[i] + k, thresh, dscale);
        v[i][k] += b;
      }
    }
  }
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += v[i][k];
    if (hi[i]) s1 += s;
    else s0 += s;
  }
  const float inv = 1.f / (float)cols;
  const float mu0 = wave_sum(s0) * inv, mu1 = wave_sum(s1) * inv;
  float q0 = 0.f, q1 = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const float mu = hi[i] ? mu1 : mu0;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = v[i][k] - mu;
      q += d * d;
    }
    if (hi[i]) q1 += q;
    else q0 += q;
  }
  const float rs0 = rsqrtf(wave_sum(q0) * inv + eps), rs1 = rsqrtf(wave_sum(q1) * inv + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    if (!ok[i]) continue;
    const long row = row0 + (hi[i] ? 1 : 0), c0 = cc[i];
    const float mu = hi[i] ? mu1 : mu0, rs = hi[i] ? rs1 : rs0;
    const f32x4 g0 = *(const f32x4*)(gamma + c0), g1 = *(const f32x4*)(gamma + c0 + 4);
    const f32x4 b0 = *(const f32x4*)(beta + c0), b1 = *(const f32x4*)(beta + c0 + 4);
    float o[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      o[k] = (v[i][k] - mu) * rs * g0[k] + b0[k];
      o[k + 4] = (v[i][k + 4] - mu) * rs * g1[k] + b1[k];
    }
    if (z) st8(z + row * cols + c0, v[i]);
    st8(y + row * ldy + c0, o);
  }
  if (lane == 0) {
    if (mean) {
      if (row0 < rows) mean[row0] = mu0;
      if (row0 + 1 < rows) mean[row0 + 1] = mu1;
    }
    if (rstd) {
      if (row0 < rows) rstd[row0] = rs0;
      if (row0 + 1 < rows) rstd[row0 + 1] = rs1;
    }
  }
}

}  // namespace

extern "C" int mit_layernorm_fwd(int dtype, long rows, long cols, const void* x, long ldx, const void* r, long ldr,
                                 float r_drop_p, const uint64_t* seed, uint32_t site, const float* gamma,
                                 const float* beta, float eps, void* z, void* y, long ldy, float* mean, float* rstd,
                                 void* stream) {
  MIT_RECORD([=]() { return mit_layernorm_fwd(dtype, rows, cols, x, ldx, r, ldr, r_drop_p, seed, site, gamma, beta, eps, z, y, ldy, mean, rstd, stream); });
  MIT_CHECK_ARG(cols > 0 && cols <= 64 * MAXV_ALL, "mit_layernorm_fwd: cols %ld out of range", cols);
  MIT_CHECK_ARG(x && y && gamma && beta, "mit_layernorm_fwd: null pointer");
  MIT_CHECK_ARG(ldx >= cols && ldy >= cols && (!r || ldr >= cols), "mit_layernorm_fwd: bad leading dim");
  if (rows <= 0) return MIT_OK;
  const int dropout = (r != nullptr) && r_drop_p > 0.f;
  const uint32_t th = drop_threshold(r_drop_p);
  const float sc = r_drop_p < 1.f ? 1.f / (1.f - r_drop_p) : 0.f;
  const size_t esz = dtype == MIT_BF16 ? 2 : 4;
  const bool vec = cols % 256 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && (!r || ldr % 4 == 0) &&
                   ((uintptr_t)x % (4 * esz)) == 0 && ((uintptr_t)y % (4 * esz)) == 0 &&
                   (!r || ((uintptr_t)r % (4 * esz)) == 0) && (!z || ((uintptr_t)z % (4 * esz)) == 0) &&
                   ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0;
  dim3 grid((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == MIT_BF16 && cols % 8 == 0 && cols <= 1024 && ldx % 8 == 0 && ldy % 8 == 0 &&
      (!r || ldr % 8 == 0) && (((uintptr_t)x | (uintptr_t)y | (uintptr_t)r | (uintptr_t)z) % 16) == 0 &&
      ((uintptr_t)gamma % 16) == 0 && ((uintptr_t)beta % 16) == 0) {
    // one row per wave (2 / 4 rows per wave alone, tools/ln_bench.py: encoder 12608 x 768 9.4 vs
    // 10.2 / 11.6 us, CLIP-L 36928 x 1024 24.7 vs 26.9 / 29.7 us, decoder 4032 x 512 + residual +
    // dropout 6.3 vs 6.5 / 8.7 us): the most waves in flight
    // widths whose two rows fill whole 64-lane passes (256: 1 pass, 768: 3): two rows per wave. Alone (tools/ln_bench.py, interleaved): 16384 x 256
    // 6.1 vs 7.6-8.2 us, 12608 x 768 + residual + dropout (configs[3]'s decoder width) 18.3 vs
    // 19.7-20.0 us; the encoder's 768-wide LayerNorm without residual is not faster (10.0 vs 9.9 us:
    // x -> y alone copies in 6.2 us, the rest is per-row latency) and keeps the one-row form
    if ((cols == 256 || (cols == 768 && r))) {
      const dim3 g2((unsigned)((rows + 7) / 8));
      auto go = [&](auto nvc) {
        constexpr int NVc = decltype(nvc)::value;
        if (r)
          hipLaunchKernelGGL((ln_fwd_pair_kernel<NVc, true>), g2, dim3(256), 0, s, rows, cols, (const bf16*)x, ldx,
                             (const bf16*)r, ldr, seed, site, th, sc, dropout, gamma, beta, eps, (bf16*)z, (bf16*)y,
                             ldy, mean, rstd);
        else
          hipLaunchKernelGGL((ln_fwd_pair_kernel<NVc, false>), g2, dim3(256), 0, s, rows, cols, (const bf16*)x, ldx,
                             (const bf16*)r, ldr, seed, site, th, sc, dropout, gamma, beta, eps, (bf16*)z, (bf16*)y,
                             ldy, mean, rstd);
      };
      if (cols == 256) go(std::integral_constant<int, 1>());
      else go(std::integral_constant<int, 3>());
      MIT_LAUNCH_CHECK("mit_layernorm_fwd");
      return MIT_OK;
    }
    auto launch = [&](auto nvc, auto rwc) {
      constexpr int NVc = decltype(nvc)::value, RWc = decltype(rwc)::value;
      const dim3 g2((unsigned)((rows + 4 * RWc - 1) / (4 * RWc)));
      if (r)
        hipLaunchKernelGGL((ln_fwd_wide_kernel<NVc, RWc, true>), g2, dim3(256), 0, s, rows, cols, (const bf16*)x, ldx,
                           (const bf16*)r, ldr, seed, site, th, sc, dropout, gamma, beta, eps, (bf16*)z, (bf16*)y, ldy,
                           mean, rstd);
      else
        hipLaunchKernelGGL((ln_fwd_wide_kernel<NVc, RWc, false>), g2, dim3(256), 0, s, rows, cols, (const bf16*)x, ldx,
                           (const bf16*)r, ldr, seed, site, th, sc, dropout, gamma, beta, eps, (bf16*)z, (bf16*)y, ldy,
                           mean, rstd);
    };
    auto by_rw = [&](auto nvc) { launch(nvc, std::integral_constant<int, 1>()); };
    if (cols <= 512) by_rw(std::integral_constant<int, 1>());
    else by_rw(std::integral_constant<int, 2>());
    MIT_LAUNCH_CHECK("mit_layernorm_fwd");
    return MIT_OK;
  }
  auto go = [&](auto tt, auto vv) {
    typedef decltype(tt) T;
    constexpr bool V = decltype(vv)::value;
    dispatch_nv<T, V>(cols, [&](auto nv) {
      constexpr int NV = decltype(nv)::value;
      hipLaunchKernelGGL((ln_fwd_kernel<T, NV, V>), grid, dim3(256), 0, s, rows, cols, (const T*)x, ldx, (const T*)r,
                         ldr, seed, site, th, sc, dropout, gamma, beta, eps, (T*)z, (T*)y, ldy, mean, rstd);
    });
  };
  if (dtype == MIT_BF16) {
    if (vec) go(bf16(), std::true_type());
    else go(bf16(), std::false_type());
  } else {
    if (vec) go(float(), std::true_type());
    else go(float(), std::false_type());
  }
  MIT_LAUNCH_CHECK("mit_layernorm_fwd");
  return MIT_OK;
}

// LayerNorm forward of an f32 row stream (the encoder's f32 residual stream): z = x + r (r: the bf16
// output of the sublayer, may be NULL; z: f32, may be NULL or alias x), y = LN(z) in y_dtype (bf16: the
// next GEMM's operand; f32: a new residual stream, e.g. CLIP's pre_layrnorm). No saved statistics.
extern "C" int mit_layernorm_fwd_x32(long rows, long cols, const float* x, long ldx, const void* r, long ldr, float* z,
                                     const float* gamma, const float* beta, float eps, void* y, int y_dtype, long ldy,
                                     void* stream) {
  MIT_RECORD([=]() { return mit_layernorm_fwd_x32(rows, cols, x, ldx, r, ldr, z, gamma, beta, eps, y, y_dtype, ldy, stream); });
  MIT_CHECK_ARG(x && y && gamma && beta, "mit_layernorm_fwd_x32: null pointer");
  MIT_CHECK_ARG(y_dtype == MIT_BF16 || y_dtype == MIT_F32, "mit_layernorm_fwd_x32: bad y dtype %d", y_dtype);
  MIT_CHECK_ARG(cols > 0 && cols % 8 == 0 && cols <= 1024, "mit_layernorm_fwd_x32: cols %ld (multiple of 8, <= 1024)",
                cols);
  MIT_CHECK_ARG(ldx >= cols && ldy >= cols && ldx % 8 == 0 && ldy % 8 == 0 && (!r || (ldr >= cols && ldr % 8 == 0)),
                "mit_layernorm_fwd_x32: bad leading dim");
  MIT_CHECK_ARG(!z || ldx == cols, "mit_layernorm_fwd_x32: z (row stride cols) needs ldx == cols");
  MIT_CHECK_ARG((((uintptr_t)x | (uintptr_t)y | (uintptr_t)r | (uintptr_t)z | (uintptr_t)gamma | (uintptr_t)beta) % 16) == 0,
                "mit_layernorm_fwd_x32: pointers must be 16-B aligned");
  MIT_CHECK_ARG((const void*)y != (const void*)x && (const void*)y != r, "mit_layernorm_fwd_x32: y must not alias x or r");
  if (rows <= 0) return MIT_OK;
  const dim3 g((unsigned)((rows + 3) / 4));
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto nvc, auto hasr, auto ty) {
    constexpr int NV = decltype(nvc)::value;
    constexpr bool HR = decltype(hasr)::value;
    typedef decltype(ty) TY;
    hipLaunchKernelGGL((ln_fwd_wide_kernel<NV, 1, HR, float, TY, bf16>), g, dim3(256), 0, s, rows, cols, x, ldx,
                       (const bf16*)r, ldr, (const uint64_t*)nullptr, 0u, 0u, 0.f, 0, gamma, beta, eps, z, (TY*)y, ldy,
                       (float*)nullptr, (float*)nullptr);
  };
  auto by_r = [&](auto nvc, auto ty) {
    if (r) go(nvc, std::true_type(), ty);
    else go(nvc, std::false_type(), ty);
  };
  auto by_y = [&](auto nvc) {
    if (y_dtype == MIT_BF16) by_r(nvc, bf16());
    else by_r(nvc, float());
  };
  if (cols <= 512) by_y(std::integral_constant<int, 1>());
  else by_y(std::integral_constant<int, 2>());
  MIT_LAUNCH_CHECK("mit_layernorm_fwd_x32");
  return MIT_OK;
}

namespace {
// y = bf16(x + r): the f32 residual stream's last update, rounded for the consumers (CLIP's
// last_hidden_state has no final LayerNorm)
__global__ __launch_bounds__(256) void residual_out_kernel(long rows, long cols, const float* __restrict__ x, long ldx,
                                                           const bf16* __restrict__ r, long ldr, bf16* __restrict__ y,
                                                           long ldy) {
  const long per = cols / 8, n = rows * per;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / per, c = (i - row * per) * 8;
    float a[8], b[8];
    ld8(x + row * ldx + c, a);
    if (r) ld8(r + row * ldr + c, b);
#pragma unroll
    for (int k = 0; k < 8; ++k) a[k] += r ? b[k] : 0.f;
    st8(y + row * ldy + c, a);
  }
}
}  // namespace

extern "C" int mit_residual_out(long rows, long cols, const float* x, long ldx, const void* r, long ldr, void* y, long ldy,
                                void* stream) {
  MIT_RECORD([=]() { return mit_residual_out(rows, cols, x, ldx, r, ldr, y, ldy, stream); });
  MIT_CHECK_ARG(x && y, "mit_residual_out: null pointer");
  MIT_CHECK_ARG(cols > 0 && cols % 8 == 0 && ldx >= cols && ldy >= cols && ldx % 8 == 0 && ldy % 8 == 0 &&
                    (!r || (ldr >= cols && ldr % 8 == 0)),
                "mit_residual_out: cols / leading dims must be multiples of 8");
  MIT_CHECK_ARG((((uintptr_t)x | (uintptr_t)y | (uintptr_t)r) % 16) == 0, "mit_residual_out: 16-B aligned pointers");
  if (rows <= 0) return MIT_OK;
  const long n = rows * (cols / 8);
  const long blocks = std::min((n + 255) / 256, 8192L);
  hipLaunchKernelGGL(residual_out_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, rows, cols, x, ldx,
                     (const bf16*)r, ldr, (bf16*)y, ldy);
  MIT_LAUNCH_CHECK("mit_residual_out");
  return MIT_OK;
}

extern "C" long mit_layernorm_bwd_ws_floats(long rows, long cols) {
  return ((rows + BWD_ROWS - 1) / BWD_ROWS) * 2 * cols;
}

extern "C" int mit_layernorm_bwd(int dtype, long rows, long cols, const void* dy, const void* z, const float* mean,
                                 const float* rstd, const float* gamma, void* dx, void* dr, float r_drop_p,
                                 const uint64_t* seed, uint32_t site, float* dgamma, float* dbeta, float* ws,
                                 void* stream) {
  MIT_RECORD([=]() { return mit_layernorm_bwd(dtype, rows, cols, dy, z, mean, rstd, gamma, dx, dr, r_drop_p, seed, site, dgamma, dbeta, ws, stream); });
  MIT_CHECK_ARG(cols > 0 && cols <= 64 * MAXV_ALL, "mit_layernorm_bwd: cols %ld out of range", cols);
  MIT_CHECK_ARG(dy && z && mean && rstd && gamma && dx && ws, "mit_layernorm_bwd: null pointer");
  MIT_CHECK_ARG(!dgamma == !dbeta, "mit_layernorm_bwd: dgamma and dbeta must both be set or both be NULL");
  if (rows <= 0) return MIT_OK;
  const int dropout = r_drop_p > 0.f;
  const uint32_t th = drop_threshold(r_drop_p);
  const float sc = r_drop_p < 1.f ? 1.f / (1.f - r_drop_p) : 0.f;
  const long nblk = (rows + BWD_ROWS - 1) / BWD_ROWS;
  const size_t esz = dtype == MIT_BF16 ? 2 : 4;
  const bool vec = cols % 256 == 0 && ((uintptr_t)dy % (4 * esz)) == 0 && ((uintptr_t)z % (4 * esz)) == 0 &&
                   ((uintptr_t)dx % (4 * esz)) == 0 && (!dr || ((uintptr_t)dr % (4 * esz)) == 0) &&
                   ((uintptr_t)gamma % 16) == 0;
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto tt, auto vv) {
    typedef decltype(tt) T;
    constexpr bool V = decltype(vv)::value;
    dispatch_nv<T, V>(cols, [&](auto nv) {
      constexpr int NV = decltype(nv)::value;
      hipLaunchKernelGGL((ln_bwd_kernel<T, NV, V>), dim3((unsigned)nblk), dim3(256), 0, s, rows, cols, (const T*)dy,
                         (const T*)z, mean, rstd, gamma, (T*)dx, (T*)dr, seed, site, th, sc, dropout, ws);
    });
  };
  if (dtype == MIT_BF16 && cols % 8 == 0 && cols <= 1024 &&
      (((uintptr_t)dy | (uintptr_t)z | (uintptr_t)dx | (uintptr_t)dr | (uintptr_t)gamma) % 16) == 0) {
    if (cols <= 512)
      hipLaunchKernelGGL((ln_bwd_wide_kernel<1>), dim3((unsigned)nblk), dim3(256), 0, s, rows, cols, (const bf16*)dy,
                         (const bf16*)z, mean, rstd, gamma, (bf16*)dx, (bf16*)dr, seed, site, th, sc, dropout, ws);
    else
      hipLaunchKernelGGL((ln_bwd_wide_kernel<2>), dim3((unsigned)nblk), dim3(256), 0, s, rows, cols, (const bf16*)dy,
                         (const bf16*)z, mean, rstd, gamma, (bf16*)dx, (bf16*)dr, seed, site, th, sc, dropout, ws);
  } else if (dtype == MIT_BF16) {
    if (vec) go(bf16(), std::true_type());
    else go(bf16(), std::false_type());
  } else {
    if (vec) go(float(), std::true_type());
    else go(float(), std::false_type());
  }
  MIT_LAUNCH_CHECK("mit_layernorm_bwd");
  if (!dgamma) return MIT_OK;  // partials stay in ws for mit_layernorm_param_grads
  hipLaunchKernelGGL(ln_param_reduce, dim3((unsigned)((2 * cols + 15) / 16)), dim3(256), 0, s, nblk, cols, ws, dgamma,
                     dbeta);
  MIT_LAUNCH_CHECK("mit_layernorm_bwd(reduce)");
  return MIT_OK;
}

extern "C" int mit_layernorm_param_grads(long rows, long cols, const float* ws, float* dgamma, float* dbeta,
                                         void* stream) {
  MIT_RECORD([=]() { return mit_layernorm_param_grads(rows, cols, ws, dgamma, dbeta, stream); });
  MIT_CHECK_ARG(ws && dgamma && dbeta, "mit_layernorm_param_grads: null pointer");
  MIT_CHECK_ARG(cols > 0, "mit_layernorm_param_grads: cols %ld", cols);
  if (rows <= 0) return MIT_OK;
  const long nblk = (rows + BWD_ROWS - 1) / BWD_ROWS;
  hipLaunchKernelGGL(ln_param_reduce, dim3((unsigned)((2 * cols + 15) / 16)), dim3(256), 0, (hipStream_t)stream, nblk,
                     cols, ws, dgamma, dbeta);
  MIT_LAUNCH_CHECK("mit_layernorm_param_grads");
  return MIT_OK;
}

namespace {
// per-64-column (mean, M2) of each bf16 row: 8 lanes per 64-column chunk (8 bf16 each, one 16-B load),
// reductions over the chunk's 8 lanes by shuffles, two passes (mean, then squared deviations); one wave per
// row, 512 columns per wave pass
__global__ __launch_bounds__(256) void row_stats64_kernel(long rows, long cols, const bf16* __restrict__ x, long ldx,
                                                          float* __restrict__ out) {
  const long r = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const long P = cols / 64;
  for (long c = 8L * lane; c - 8L * lane < cols; c += 512) {
    float v[8];
    const bool ok = c < cols;
    if (ok) ld8(x + r * ldx + c, v);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += ok ? v[k] : 0.f;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) s += __shfl_xor(s, o, 64);
    const float mean = s * (1.f / 64.f);
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) q += ok ? (v[k] - mean) * (v[k] - mean) : 0.f;
#pragma unroll
    for (int o = 1; o < 8; o <<= 1) q += __shfl_xor(q, o, 64);
    if (ok && (lane & 7) == 0) {
      float* dst = out + (r * P + c / 64) * 2;
      dst[0] = mean;
      dst[1] = q;
    }
  }
}
}  // namespace

extern "C" int mit_row_stats64(long rows, long cols, const void* x, long ldx, float* out, void* stream) {
  MIT_RECORD([=]() { return mit_row_stats64(rows, cols, x, ldx, out, stream); });
  MIT_CHECK_ARG(x && out, "mit_row_stats64: null pointer");
  MIT_CHECK_ARG(cols > 0 && cols % 64 == 0 && ldx >= cols && ldx % 8 == 0 && ((uintptr_t)x % 16) == 0,
                "mit_row_stats64: cols %% 64 == 0, ldx %% 8 == 0, 16-B aligned rows");
  if (rows <= 0) return MIT_OK;
  hipLaunchKernelGGL(row_stats64_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream, rows, cols,
                     (const bf16*)x, ldx, out);
  MIT_LAUNCH_CHECK("mit_row_stats64");
  return MIT_OK;
}
