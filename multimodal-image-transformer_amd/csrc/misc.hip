// Memory-bound kernels of the train step: encoder input assembly, decoder embedding, cross-entropy,
// bias-gradient column sums, and the fused clip_grad_norm_ + AdamW optimizer step.
#include "common.h"

namespace {

// ---------------------------------------------------------------------------------------------
// im2col for the stride == kernel patch Conv2d; one thread per 8 output columns of a patch row
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void im2col_kernel(long B, long C, long H, long W, long P, const float* __restrict__ img, T* __restrict__ out,
                              long kpad) {
  const long npw = W / P, nph = H / P, np = nph * npw;
  const long total = B * np * kpad;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long col = i % kpad, row = i / kpad;
    const long b = row / np, p = row % np;
    float v = 0.f;
    if (col < C * P * P) {
      const long c = col / (P * P), ky = (col / P) % P, kx = col % P;
      const long y = (p / npw) * P + ky, x = (p % npw) * P + kx;
      v = img[((b * C + c) * H + y) * W + x];
    }
    out[i] = from_f<T>(v);
  }
}

// bf16, P % 8 == 0 (ViT-B/16): one thread per 8 consecutive columns = 8 pixels of one patch row
// (two 16-B f32 loads, one 16-B bf16 store), 32-bit index math (the scalar form's 64-bit
// divisions per element made it 1.2 TB/s)
__global__ __launch_bounds__(256) void im2col8_kernel(int B, int C, int H, int W, int P, const float* __restrict__ img,
                                                      bf16* __restrict__ out, int kpad) {
  const int npw = W / P, np = (H / P) * npw, g8 = kpad / 8, PP = P * P;
  const int total = B * np * g8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int row = i / g8, col = (i - row * g8) * 8;
    const int b = row / np, p = row - b * np;
    bf16x8 o;
    if (col < C * PP) {
      const int c = col / PP, r = col - c * PP, ky = r / P, kx = r - ky * P;
      const int y = (p / npw) * P + ky, x = (p % npw) * P + kx;
      const float* src = img + (((long)b * C + c) * H + y) * W + x;
      const f32x4 a = *(const f32x4*)src, d = *(const f32x4*)(src + 4);
      o = bf16x8{(bf16)a[0], (bf16)a[1], (bf16)a[2], (bf16)a[3], (bf16)d[0], (bf16)d[1], (bf16)d[2], (bf16)d[3]};
    } else {
      o = bf16x8{};
    }
    *(bf16x8*)(out + (long)row * kpad + col) = o;
  }
}

// bf16, E % 8 == 0: 8 columns per thread, 32-bit index math
__global__ __launch_bounds__(256) void assemble8_kernel(int B, int np, int E, const bf16* __restrict__ patch,
                                                        const float* __restrict__ cls, const float* __restrict__ pos,
                                                        bf16* __restrict__ h) {
  const int e8 = E / 8, total = B * (np + 1) * e8;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < total; i += gridDim.x * blockDim.x) {
    const int bt = i / e8, e = (i - bt * e8) * 8, b = bt / (np + 1), t = bt - b * (np + 1);
    float v[8];
    if (t == 0) {
      const f32x4 a = *(const f32x4*)(cls + e), d = *(const f32x4*)(cls + e + 4);
      v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3]; v[4] = d[0]; v[5] = d[1]; v[6] = d[2]; v[7] = d[3];
    } else {
      const bf16x8 pv = *(const bf16x8*)(patch + ((long)b * np + t - 1) * E + e);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = (float)pv[k];
    }
    const f32x4 p0 = *(const f32x4*)(pos + (long)t * E + e), p1 = *(const f32x4*)(pos + (long)t * E + e + 4);
    *(bf16x8*)(h + (long)bt * E + e) = bf16x8{(bf16)(v[0] + p0[0]), (bf16)(v[1] + p0[1]), (bf16)(v[2] + p0[2]),
                                              (bf16)(v[3] + p0[3]), (bf16)(v[4] + p1[0]), (bf16)(v[5] + p1[1]),
                                              (bf16)(v[6] + p1[2]), (bf16)(v[7] + p1[3])};
  }
}

template <typename T>
__global__ void assemble_kernel(long B, long np, long E, const T* __restrict__ patch, const float* __restrict__ cls,
                                const float* __restrict__ pos, T* __restrict__ h) {
  const long total = B * (np + 1) * E;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long e = i % E, t = (i / E) % (np + 1), b = i / (E * (np + 1));
    const float base = (t == 0) ? cls[e] : to_f(patch[(b * np + t - 1) * E + e]);
    h[i] = from_f<T>(base + pos[t * E + e]);
  }
}

// ---------------------------------------------------------------------------------------------
// decoder embedding
// ---------------------------------------------------------------------------------------------
template <typename T>
__global__ void embed_fwd_kernel(long B, long T_, long d, const int64_t* __restrict__ tok, const T* __restrict__ table,
                                 float scale, const float* __restrict__ pe, const uint64_t* seed, uint32_t site,
                                 uint32_t thresh, float dscale, int dropout, T* __restrict__ out) {
  const long total = B * T_ * d;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long c = i % d, bt = i / d, t = bt % T_;
    const int64_t id = tok[bt];
    float v = to_f(table[id * d + c]) * scale + pe[t * d + c];
    if (dropout) v *= drop_mul(key, (uint64_t)i, thresh, dscale);
    out[i] = from_f<T>(v);
  }
}

template <typename T>
__global__ void embed_bwd_kernel(long B, long T_, long d, const int64_t* __restrict__ tok, const T* __restrict__ dx,
                                 float scale, const uint64_t* seed, uint32_t site, uint32_t thresh, float dscale,
                                 int dropout, int pad, float* __restrict__ dtable) {
  const long total = B * T_ * d;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long c = i % d, bt = i / d;
    const int64_t id = tok[bt];
    if (id == pad) continue;
    float g = to_f(dx[i]) * scale;
    if (dropout) g *= drop_mul(key, (uint64_t)i, thresh, dscale);
    atomicAdd(&dtable[id * d + c], g);
  }
}

// Deterministic embedding backward (replaces the float atomics above): the gradient row of token v
// is the sum over the positions holding v, taken in a FIXED order. Plan (depends on the tokens
// only): ONE 1024-thread workgroup bitonic-sorts the (token << 20 | position) keys, then
// plan[k] = position of sorted slot k and plan[n + k] = the length of the token's run starting at k
// (0 if slot k is not the first of its token). Each thread keeps KPT consecutive keys in registers:
// compare-exchange distances j < KPT stay in the thread, KPT <= j < 64 KPT cross lanes of one wave
// (__shfl_xor), and only j >= 64 KPT go through LDS (2 barriers each) -- 10 of the 78 stages at
// n = 4032 (was: all 78 through LDS behind a barrier each, 86 us per step).
constexpr int EMB_PLAN_MAX = 16384;
__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const unsigned lo = (unsigned)__shfl_xor((int)(unsigned)v, m, 64);
  const unsigned hi = (unsigned)__shfl_xor((int)(unsigned)(v >> 32), m, 64);
  return ((uint64_t)hi << 32) | lo;
}
template <int KPT>
__global__ __launch_bounds__(1024) void embed_plan_kernel(const int64_t* __restrict__ tok, int n, int npow2,
                                                          int* __restrict__ plan) {
  extern __shared__ uint64_t keys[];
  const int t = threadIdx.x;
  uint64_t x[KPT];
#pragma unroll
  for (int e = 0; e < KPT; ++e) {
    const int i = t * KPT + e;
    x[e] = i < n ? ((uint64_t)tok[i] << 20) | (uint64_t)i : ~0ull;
  }
  for (int k = 2; k <= npow2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j < KPT) {  // both elements in this thread
#pragma unroll
        for (int e = 0; e < KPT; ++e) {
          const int f = e ^ j;
          if (f > e) {
            const bool asc = ((t * KPT + e) & k) == 0;
            const uint64_t a = x[e], b = x[f];
            if ((a > b) == asc) {
              x[e] = b;
              x[f] = a;
            }
          }
        }
      } else if (j < 64 * KPT) {  // partner element = same slot of lane ^ (j / KPT)
        const int m = j / KPT;
        const bool lower = (t & m) == 0;
#pragma unroll
        for (int e = 0; e < KPT; ++e) {
          const uint64_t o = shfl_xor_u64(x[e], m);
          const bool asc = ((t * KPT + e) & k) == 0;
          x[e] = (lower == asc) ? (x[e] < o ? x[e] : o) : (x[e] > o ? x[e] : o);
        }
      } else {
        const int m = j / KPT;
        const bool lower = (t & m) == 0;
#pragma unroll
        for (int e = 0; e < KPT; ++e) keys[t * KPT + e] = x[e];
        __syncthreads();
#pragma unroll
        for (int e = 0; e < KPT; ++e) {
          const uint64_t o = keys[(t ^ m) * KPT + e];
          const bool asc = ((t * KPT + e) & k) == 0;
          x[e] = (lower == asc) ? (x[e] < o ? x[e] : o) : (x[e] > o ? x[e] : o);
        }
        __syncthreads();
      }
    }
  }
#pragma unroll
  for (int e = 0; e < KPT; ++e) keys[t * KPT + e] = x[e];
  __syncthreads();
  for (int k = t; k < n; k += 1024) {
    const uint64_t tk = keys[k] >> 20;
    plan[k] = (int)(keys[k] & 0xFFFFFu);
    int len = 0;
    if (k == 0 || (keys[k - 1] >> 20) != tk) {
      len = 1;
      while (k + len < n && (keys[k + len] >> 20) == tk) ++len;
    }
    plan[n + k] = len;
  }
}

// one wave per sorted slot; the first slot of each token's run sums the run's dx rows in position
// order (each lane owns 8 consecutive columns per 512) and STORES the row (dtable is zeroed once
// before; PAD's row receives nothing). d % 8 == 0.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_seg_kernel(int n, int d, const int64_t* __restrict__ tok,
                                                            const T* __restrict__ dx, float scale,
                                                            const uint64_t* seed, uint32_t site, uint32_t thresh,
                                                            float dscale, int dropout, int pad,
                                                            const int* __restrict__ plan, float* __restrict__ dtable) {
  const int k = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (k >= n) return;
  const int len = plan[n + k];
  if (len == 0) return;
  const int* perm = plan + k;
  const int64_t id = tok[perm[0]];
  if (id == pad) return;
  const int lane = threadIdx.x & 63;
  const uint64_t key = dropout ? site_key(seed, site) : 0ull;
  // a token's rows are summed in position order, ER rows' loads in flight at a time (the run of a
  // token every caption has -- START at position 0 -- is B rows long and sits on the backward's
  // critical path: one dependent load per row made it the longest wave of the kernel)
  constexpr int ER = 16;
  for (int c0 = lane * 8; c0 < d; c0 += 512) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r0 = 0; r0 < len; r0 += ER) {
      long jj[ER];
#pragma unroll
      for (int u = 0; u < ER; ++u) jj[u] = r0 + u < len ? (long)perm[r0 + u] : -1;
      float v[ER][8];
#pragma unroll
      for (int u = 0; u < ER; ++u) {
        if (jj[u] < 0) continue;
        const long j = jj[u];
        if constexpr (sizeof(T) == 2) {
          const bf16x8 x = *(const bf16x8*)(dx + j * d + c0);
#pragma unroll
          for (int q = 0; q < 8; ++q) v[u][q] = (float)x[q];
        } else {
          const f32x4 x0 = *(const f32x4*)(dx + j * d + c0), x1 = *(const f32x4*)(dx + j * d + c0 + 4);
          v[u][0] = x0[0]; v[u][1] = x0[1]; v[u][2] = x0[2]; v[u][3] = x0[3];
          v[u][4] = x1[0]; v[u][5] = x1[1]; v[u][6] = x1[2]; v[u][7] = x1[3];
        }
      }
#pragma unroll
      for (int u = 0; u < ER; ++u) {
        if (jj[u] < 0) continue;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          float g = v[u][q] * scale;
          if (dropout) g *= drop_mul(key, (uint64_t)(jj[u] * d + c0 + q), thresh, dscale);
          acc[q] += g;
        }
      }
    }
    f32x4* o = (f32x4*)(dtable + id * d + c0);
    o[0] = f32x4{acc[0], acc[1], acc[2], acc[3]};
    o[1] = f32x4{acc[4], acc[5], acc[6], acc[7]};
  }
}

// ---------------------------------------------------------------------------------------------
// cross entropy (one 256-thread block per row), in-place gradient
// ---------------------------------------------------------------------------------------------
__global__ void count_kernel(const int64_t* __restrict__ t, long n, int ignore, float* count) {
  __shared__ float scratch[16];
  float c = 0.f;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    c += (t[i] != ignore) ? 1.f : 0.f;
  c = block_sum(c, scratch);
  if (threadIdx.x == 0) atomicAdd(count, c);
}

template <typename T>
__global__ __launch_bounds__(256) void ce_kernel(long V, T* logits, long ld, const int64_t* __restrict__ targets,
                                                 int ignore, const float* __restrict__ count, float* loss_sum,
                                                 int want_grad, float* row_loss) {
  __shared__ float scratch[16];
  const long row = blockIdx.x;
  T* x = logits + row * ld;
  const int64_t tg = targets[row];
  const bool ign = (tg == ignore);
  float mx = -INFINITY;
  for (long j = threadIdx.x; j < V; j += blockDim.x) mx = fmaxf(mx, to_f(x[j]));
  mx = block_max(mx, scratch);
  float se = 0.f;
  for (long j = threadIdx.x; j < V; j += blockDim.x) se += __expf(to_f(x[j]) - mx);
  se = block_sum(se, scratch);
  const float lse = mx + __logf(se);
  if (threadIdx.x == 0) {
    if (row_loss) row_loss[row] = ign ? 0.f : lse - to_f(x[tg]);
    else if (!ign) atomicAdd(loss_sum, lse - to_f(x[tg]));
  }
  if (want_grad) {
    __syncthreads();  // every thread has read x[tg] above before anyone overwrites it
    const float gs = ign ? 0.f : 1.0f / *count;
    const float inv = 1.0f / se;
    for (long j = threadIdx.x; j < V; j += blockDim.x) {
      float p = __expf(to_f(x[j]) - mx) * inv;
      if (j == tg) p -= 1.0f;
      x[j] = from_f<T>(p * gs);
    }
  }
}

// bf16 rows with V <= CE_NCH * 512 (the decoder head, V = 10000): one wave per row, the row held in
// registers (CE_NCH x 16-B loads per lane), so HBM sees one read and one write of the logits; each
// row's loss goes to row_loss[row] and ce_sum adds them up in row order (deterministic, no
// single-address float atomics: 4032 of those serialised cost ~100 us). V need not be a multiple
// of 8 when ld is (the head padded to Vp = round8(V) columns): the tail of the last 16-B chunk is
// masked out of the softmax and its gradient is written as 0.
constexpr int CE_NCH = 20;
__global__ __launch_bounds__(256) void ce_rows_bf16(long rows, long V, bf16* logits, long ld,
                                                     const int64_t* __restrict__ targets, int ignore,
                                                     const float* __restrict__ count, float* __restrict__ row_loss,
                                                     int want_grad) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  bf16* x = logits + row * ld;
  const int64_t tg = targets[row];
  const bool ign = tg == ignore;
  bf16x8 v[CE_NCH];
#pragma unroll
  for (int c = 0; c < CE_NCH; ++c) {
    const long j = (long)c * 512 + lane * 8;
    if (j < V) v[c] = *(const bf16x8*)(x + j);
  }
  const float xt = (!ign && tg >= 0 && tg < V) ? (float)x[tg] : 0.f;
  // masked tail of a padded head: -inf (exp2 -> 0, max unaffected); whole 16-B chunks are in range
  // (ld % 8 == 0), only the last may hold columns >= V
#pragma unroll
  for (int c = 0; c < CE_NCH; ++c) {
    const long j = (long)c * 512 + lane * 8;
    if (j < V && j + 8 > V) {
#pragma unroll
      for (int k = 0; k < 8; ++k)
        if (j + k >= V) v[c][k] = (bf16)(-INFINITY);
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < CE_NCH; ++c) {
    const long j = (long)c * 512 + lane * 8;
    if (j < V) {
#pragma unroll
      for (int k = 0; k < 8; k += 2) mx = __builtin_fmaxf(mx, __builtin_fmaxf((float)v[c][k], (float)v[c][k + 1]));
    }
  }
  mx = wave_max(mx);
  // exp(x - mx) as exp2(x log2e - mx log2e): one FMA + v_exp per element
  constexpr float L2E = 1.4426950408889634f;
  const float mxl = mx * L2E;
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < CE_NCH; ++c) {
    const long j = (long)c * 512 + lane * 8;
    if (j < V) {
#pragma unroll
      for (int k = 0; k < 8; ++k) se += __builtin_amdgcn_exp2f(fmaf((float)v[c][k], L2E, -mxl));
    }
  }
  se = wave_sum(se);
  const float lse = mx + __logf(se);
  if (lane == 0) row_loss[row] = ign ? 0.f : lse - xt;
  if (!want_grad) return;
  const float gs = ign ? 0.f : 1.0f / *count;
  // dlogit = gs * softmax - gs * [j == tg] = exp2(x log2e - (mx log2e + log2 se - log2 gs)) - gs [j == tg]
  const float off = mxl + __log2f(se) - (gs > 0.f ? __log2f(gs) : 0.f);
#pragma unroll
  for (int c = 0; c < CE_NCH; ++c) {
    const long j = (long)c * 512 + lane * 8;
    if (j < V) {
      float q[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) q[k] = gs > 0.f ? __builtin_amdgcn_exp2f(fmaf((float)v[c][k], L2E, -off)) : 0.f;
      if (tg >= j && tg < j + 8) {  // the target column (one lane of one chunk per row)
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (j + k == tg) q[k] -= gs;
      }
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = (bf16)q[k];
      *(bf16x8*)(x + j) = o;
    }
  }
}

// loss_sum += sum(row_loss[0..rows)) in a fixed order (one block)
__global__ __launch_bounds__(1024) void ce_sum(long rows, const float* __restrict__ row_loss, float* loss_sum) {
  __shared__ float scratch[16];
  float s = 0.f;
  for (long r = threadIdx.x; r < rows; r += blockDim.x) s += row_loss[r];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) *loss_sum += s;
}

// ---------------------------------------------------------------------------------------------
// column sums (bias gradients): partial sums over 128-row chunks, then a reduction over chunks
// ---------------------------------------------------------------------------------------------
constexpr long CS_ROWS = 128;
template <typename T>
__global__ void colsum_partial(long M, long N, const T* __restrict__ dy, long ld, float* __restrict__ ws) {
  const long n = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  const long r0 = (long)blockIdx.y * CS_ROWS, r1 = min(M, r0 + CS_ROWS);
  float s = 0.f;
  for (long r = r0; r < r1; ++r) s += to_f(dy[r * ld + n]);
  ws[blockIdx.y * N + n] = s;
}
__global__ void colsum_final(long nch, long N, const float* __restrict__ ws, float* out, int acc) {
  const long n = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (long c = 0; c < nch; ++c) s += ws[c * N + n];
  out[n] = acc ? out[n] + s : s;
}

// ---------------------------------------------------------------------------------------------
// clip_grad_norm_ + AdamW
// ---------------------------------------------------------------------------------------------
constexpr int GN_BLOCKS = 1024;
__global__ __launch_bounds__(256) void sumsq_kernel(const float* __restrict__ g, long n, float* __restrict__ ws) {
  __shared__ float scratch[16];
  float s = 0.f;
  const long n4 = n / 4;
  const f32x4* g4 = (const f32x4*)g;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    const f32x4 v = g4[i];
    s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
  }
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    s += g[i] * g[i];
  s = block_sum(s, scratch);
  if (threadIdx.x == 0) ws[blockIdx.x] = s;
}
__global__ void norm_final(const float* __restrict__ ws, int nb, float max_norm, float* out) {
  __shared__ double sh[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) s += (double)ws[i];
  sh[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) sh[threadIdx.x] += sh[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float total = (float)sqrt(sh[0]);
    float coef = max_norm / (total + 1e-6f);  // clip_grad.py: clamp(max_norm / (norm + 1e-6), max=1)
    if (!(coef < 1.0f)) coef = 1.0f;
    if (max_norm <= 0.f) coef = 1.0f;
    out[0] = total;
    out[1] = coef;
  }
}
__global__ void step_inc_kernel(int64_t* step) { *step += 1; }
// stream timestamp: the constant-rate device clock (wall_clock64, hipDeviceAttributeWallClockRate)
// when this point of the stream is reached (phase timing of a recorded step, tools/phase_timing.py)
__global__ void stamp_kernel(uint64_t* out, int i) { out[i] = wall_clock64(); }
__global__ void scalar_div_kernel(const float* a, const float* b, float* out) { *out = *a / *b; }

template <bool SHADOW>
__global__ __launch_bounds__(256) void adamw_kernel(long n, float* __restrict__ p, const float* __restrict__ g,
                                                    float* __restrict__ m, float* __restrict__ v, bf16* __restrict__ sh,
                                                    const float* __restrict__ norm_out, const float* __restrict__ lr_p,
                                                    const int64_t* __restrict__ step_p, float b1, float b2, float eps,
                                                    float wd) {
  const float coef = norm_out ? norm_out[1] : 1.0f;
  const float lr = *lr_p;
  const double t = (double)*step_p;
  const float bc1 = (float)(1.0 - pow((double)b1, t));
  const float bc2 = (float)(1.0 - pow((double)b2, t));
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float decay = 1.0f - lr * wd;
  const long n4 = n / 4;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (long)gridDim.x * blockDim.x) {
    f32x4 pp = ((f32x4*)p)[i], gg = ((const f32x4*)g)[i], mm = ((f32x4*)m)[i], vv = ((f32x4*)v)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float gk = gg[k] * coef;
      pp[k] *= decay;
      mm[k] = mm[k] + (1.0f - b1) * (gk - mm[k]);
      vv[k] = vv[k] * b2 + (1.0f - b2) * gk * gk;
      const float denom = sqrtf(vv[k]) / bc2s + eps;
      pp[k] = pp[k] - step_size * (mm[k] / denom);
    }
    ((f32x4*)p)[i] = pp;
    ((f32x4*)m)[i] = mm;
    ((f32x4*)v)[i] = vv;
    if (SHADOW) {
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      ((bf16x4*)sh)[i] = bf16x4{(bf16)pp[0], (bf16)pp[1], (bf16)pp[2], (bf16)pp[3]};
    }
  }
  for (long i = n4 * 4 + (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float gk = g[i] * coef;
    float pp = p[i] * decay;
    const float mm = m[i] + (1.0f - b1) * (gk - m[i]);
    const float vv = v[i] * b2 + (1.0f - b2) * gk * gk;
    pp = pp - step_size * (mm / (sqrtf(vv) / bc2s + eps));
    p[i] = pp;
    m[i] = mm;
    v[i] = vv;
    if (SHADOW) sh[i] = (bf16)pp;
  }
}

template <typename T>
__global__ void cast_kernel(long n, const float* __restrict__ src, T* __restrict__ dst) {
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    dst[i] = from_f<T>(src[i]);
}
__global__ void mask_kernel(long n, const uint64_t* seed, uint32_t site, uint32_t thresh, float dscale, float* out) {
  const uint64_t key = site_key(seed, site);
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    out[i] = drop_mul(key, (uint64_t)i, thresh, dscale);
}

inline unsigned grid_for(long n, int block = 256, long cap = 8192) {
  long g = (n + block - 1) / block;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (unsigned)g;
}
}  // namespace

#define DISPATCH_T(dtype, ...)        \
  do {                                \
    if ((dtype) == MIT_BF16) {        \
      typedef bf16 T;                 \
      __VA_ARGS__;                    \
    } else {                          \
      typedef float T;                \
      __VA_ARGS__;                    \
    }                                 \
  } while (0)

extern "C" int mit_im2col(int dtype, long B, long C, long H, long W, long P, const float* img, void* out, long kpad,
                          void* stream) {
  MIT_RECORD([=]() { return mit_im2col(dtype, B, C, H, W, P, img, out, kpad, stream); });
  MIT_CHECK_ARG(img && out && P > 0 && H % P == 0 && W % P == 0 && kpad >= C * P * P, "mit_im2col: bad arguments");
  const long total = B * (H / P) * (W / P) * kpad;
  if (dtype == MIT_BF16 && P % 8 == 0 && W % 4 == 0 && kpad % 8 == 0 && ((uintptr_t)img % 16) == 0 &&
      ((uintptr_t)out % 16) == 0 && total / 8 < INT32_MAX && B * C * H * W < INT32_MAX) {
    hipLaunchKernelGGL(im2col8_kernel, dim3(grid_for(total / 8)), dim3(256), 0, (hipStream_t)stream, (int)B, (int)C,
                       (int)H, (int)W, (int)P, img, (bf16*)out, (int)kpad);
    MIT_LAUNCH_CHECK("mit_im2col");
    return MIT_OK;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(im2col_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B,
                                       C, H, W, P, img, (T*)out, kpad));
  MIT_LAUNCH_CHECK("mit_im2col");
  return MIT_OK;
}

extern "C" int mit_vit_assemble(int dtype, long B, long np, long E, const void* patch, const float* cls,
                                const float* pos, void* h, void* stream) {
  MIT_RECORD([=]() { return mit_vit_assemble(dtype, B, np, E, patch, cls, pos, h, stream); });
  MIT_CHECK_ARG(patch && cls && pos && h, "mit_vit_assemble: null pointer");
  const long total = B * (np + 1) * E;
  if (dtype == MIT_BF16 && E % 8 == 0 && ((uintptr_t)patch % 16) == 0 && ((uintptr_t)h % 16) == 0 &&
      ((uintptr_t)cls % 16) == 0 && ((uintptr_t)pos % 16) == 0 && total / 8 < INT32_MAX) {
    hipLaunchKernelGGL(assemble8_kernel, dim3(grid_for(total / 8)), dim3(256), 0, (hipStream_t)stream, (int)B, (int)np,
                       (int)E, (const bf16*)patch, cls, pos, (bf16*)h);
    MIT_LAUNCH_CHECK("mit_vit_assemble");
    return MIT_OK;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(assemble_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream, B,
                                       np, E, (const T*)patch, cls, pos, (T*)h));
  MIT_LAUNCH_CHECK("mit_vit_assemble");
  return MIT_OK;
}

extern "C" int mit_embed_fwd(int dtype, long B, long T_, long d, const int64_t* tokens, const void* table, float scale,
                             const float* pe, float drop_p, const uint64_t* seed, uint32_t site, void* out,
                             void* stream) {
  MIT_RECORD([=]() { return mit_embed_fwd(dtype, B, T_, d, tokens, table, scale, pe, drop_p, seed, site, out, stream); });
  MIT_CHECK_ARG(tokens && table && pe && out, "mit_embed_fwd: null pointer");
  const long total = B * T_ * d;
  const int dropout = drop_p > 0.f;
  const uint32_t th = drop_threshold(drop_p);
  const float sc = drop_p < 1.f ? 1.f / (1.f - drop_p) : 0.f;
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_fwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                                       B, T_, d, tokens, (const T*)table, scale, pe, seed, site, th, sc, dropout,
                                       (T*)out));
  MIT_LAUNCH_CHECK("mit_embed_fwd");
  return MIT_OK;
}

extern "C" long mit_embed_plan_ints(long n) { return 2 * n; }

extern "C" int mit_embed_plan(const int64_t* tokens, long n, int* plan, void* stream) {
  MIT_RECORD([=]() { return mit_embed_plan(tokens, n, plan, stream); });
  MIT_CHECK_ARG(tokens && plan && n >= 0 && n <= EMB_PLAN_MAX, "mit_embed_plan: n = %ld positions (max %d)", n,
                EMB_PLAN_MAX);
  if (n == 0) return MIT_OK;
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  if (np2 < 1024) np2 = 1024;  // one key slot per thread at least (pads sort last)
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)embed_plan_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              EMB_PLAN_MAX * 8);
    (void)hipFuncSetAttribute((const void*)embed_plan_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              EMB_PLAN_MAX * 8);
    attr = true;
  }
  hipStream_t s = (hipStream_t)stream;
  switch (np2 / 1024) {
    case 1: hipLaunchKernelGGL(embed_plan_kernel<1>, dim3(1), dim3(1024), np2 * 8, s, tokens, (int)n, np2, plan); break;
    case 2: hipLaunchKernelGGL(embed_plan_kernel<2>, dim3(1), dim3(1024), np2 * 8, s, tokens, (int)n, np2, plan); break;
    case 4: hipLaunchKernelGGL(embed_plan_kernel<4>, dim3(1), dim3(1024), np2 * 8, s, tokens, (int)n, np2, plan); break;
    case 8: hipLaunchKernelGGL(embed_plan_kernel<8>, dim3(1), dim3(1024), np2 * 8, s, tokens, (int)n, np2, plan); break;
    default: hipLaunchKernelGGL(embed_plan_kernel<16>, dim3(1), dim3(1024), np2 * 8, s, tokens, (int)n, np2, plan); break;
  }
  MIT_LAUNCH_CHECK("mit_embed_plan");
  return MIT_OK;
}

extern "C" int mit_embed_bwd(int dtype, long B, long T_, long d, const int64_t* tokens, const void* dx, float scale,
                             float drop_p, const uint64_t* seed, uint32_t site, int pad_idx, const int* plan,
                             float* dtable, void* stream) {
  MIT_RECORD([=]() { return mit_embed_bwd(dtype, B, T_, d, tokens, dx, scale, drop_p, seed, site, pad_idx, plan, dtable, stream); });
  MIT_CHECK_ARG(tokens && dx && dtable, "mit_embed_bwd: null pointer");
  const long total = B * T_ * d;
  const int dropout = drop_p > 0.f;
  const uint32_t th = drop_threshold(drop_p);
  const float sc = drop_p < 1.f ? 1.f / (1.f - drop_p) : 0.f;
  if (plan) {
    MIT_CHECK_ARG(d % 8 == 0 && B * T_ <= EMB_PLAN_MAX && ((uintptr_t)dx % 16) == 0 && ((uintptr_t)dtable % 16) == 0,
                  "mit_embed_bwd: the deterministic path takes d %% 8 == 0, <= %d positions, 16-B aligned rows",
                  EMB_PLAN_MAX);
    if (B * T_ == 0) return MIT_OK;
    DISPATCH_T(dtype, hipLaunchKernelGGL(embed_bwd_seg_kernel<T>, dim3((unsigned)((B * T_ + 3) / 4)), dim3(256), 0,
                                         (hipStream_t)stream, (int)(B * T_), (int)d, tokens, (const T*)dx, scale, seed,
                                         site, th, sc, dropout, pad_idx, plan, dtable));
    MIT_LAUNCH_CHECK("mit_embed_bwd");
    return MIT_OK;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_bwd_kernel<T>, dim3(grid_for(total)), dim3(256), 0, (hipStream_t)stream,
                                       B, T_, d, tokens, (const T*)dx, scale, seed, site, th, sc, dropout, pad_idx,
                                       dtable));
  MIT_LAUNCH_CHECK("mit_embed_bwd");
  return MIT_OK;
}

extern "C" int mit_count_targets(const int64_t* targets, long n, int ignore_index, float* count, void* stream) {
  MIT_RECORD([=]() { return mit_count_targets(targets, n, ignore_index, count, stream); });
  MIT_CHECK_ARG(targets && count, "mit_count_targets: null pointer");
  if (n <= 0) return MIT_OK;
  hipLaunchKernelGGL(count_kernel, dim3(grid_for(n, 256, 64)), dim3(256), 0, (hipStream_t)stream, targets, n,
                     ignore_index, count);
  MIT_LAUNCH_CHECK("mit_count_targets");
  return MIT_OK;
}

extern "C" int mit_cross_entropy(int dtype, long rows, long V, void* logits, long ld, const int64_t* targets,
                                 int ignore_index, const float* count, float* loss_sum, int want_grad,
                                 float* row_loss, void* stream) {
  MIT_RECORD([=]() { return mit_cross_entropy(dtype, rows, V, logits, ld, targets, ignore_index, count, loss_sum, want_grad, row_loss, stream); });
  MIT_CHECK_ARG(logits && targets && loss_sum && (!want_grad || count), "mit_cross_entropy: null pointer");
  MIT_CHECK_ARG(ld >= V, "mit_cross_entropy: ld < V");
  if (rows <= 0) return MIT_OK;
  if (row_loss && dtype == MIT_BF16 && V <= CE_NCH * 512 && ld % 8 == 0 && (V % 8 == 0 || ld >= (V + 7) / 8 * 8) &&
      ((uintptr_t)logits % 16) == 0) {
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(ce_rows_bf16, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, s, rows, V, (bf16*)logits, ld,
                       targets, ignore_index, count, row_loss, want_grad);
    MIT_LAUNCH_CHECK("mit_cross_entropy");
    hipLaunchKernelGGL(ce_sum, dim3(1), dim3(1024), 0, s, rows, (const float*)row_loss, loss_sum);
    MIT_LAUNCH_CHECK("mit_cross_entropy(sum)");
    return MIT_OK;
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(ce_kernel<T>, dim3((unsigned)rows), dim3(256), 0, (hipStream_t)stream, V,
                                       (T*)logits, ld, targets, ignore_index, count, loss_sum, want_grad, row_loss));
  MIT_LAUNCH_CHECK("mit_cross_entropy");
  if (row_loss) {
    hipLaunchKernelGGL(ce_sum, dim3(1), dim3(1024), 0, (hipStream_t)stream, rows, (const float*)row_loss, loss_sum);
    MIT_LAUNCH_CHECK("mit_cross_entropy(sum)");
  }
  return MIT_OK;
}

extern "C" long mit_colsum_ws_floats(long M, long N) { return ((M + CS_ROWS - 1) / CS_ROWS) * N; }

extern "C" int mit_colsum(int dtype, long M, long N, const void* dy, long ld, float* out, int accumulate, float* ws,
                          void* stream) {
  MIT_RECORD([=]() { return mit_colsum(dtype, M, N, dy, ld, out, accumulate, ws, stream); });
  MIT_CHECK_ARG(dy && out && ws && ld >= N, "mit_colsum: bad arguments");
  if (N <= 0) return MIT_OK;
  const long nch = (M + CS_ROWS - 1) / CS_ROWS;
  hipStream_t s = (hipStream_t)stream;
  if (nch > 0) {
    dim3 grid((unsigned)((N + 255) / 256), (unsigned)nch);
    DISPATCH_T(dtype, hipLaunchKernelGGL(colsum_partial<T>, grid, dim3(256), 0, s, M, N, (const T*)dy, ld, ws));
    MIT_LAUNCH_CHECK("mit_colsum");
  }
  hipLaunchKernelGGL(colsum_final, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, s, nch, N, ws, out, accumulate);
  MIT_LAUNCH_CHECK("mit_colsum(final)");
  return MIT_OK;
}

extern "C" long mit_grad_norm_ws_floats(long n) { (void)n; return GN_BLOCKS; }

extern "C" int mit_grad_norm(const float* grads, long n, float max_norm, float* ws, float* norm_out, void* stream) {
  MIT_RECORD([=]() { return mit_grad_norm(grads, n, max_norm, ws, norm_out, stream); });
  MIT_CHECK_ARG(grads && ws && norm_out, "mit_grad_norm: null pointer");
  MIT_CHECK_ARG(((uintptr_t)grads % 16) == 0, "mit_grad_norm: grads must be 16-B aligned");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sumsq_kernel, dim3(GN_BLOCKS), dim3(256), 0, s, grads, n, ws);
  MIT_LAUNCH_CHECK("mit_grad_norm");
  hipLaunchKernelGGL(norm_final, dim3(1), dim3(256), 0, s, ws, GN_BLOCKS, max_norm, norm_out);
  MIT_LAUNCH_CHECK("mit_grad_norm(final)");
  return MIT_OK;
}

extern "C" int mit_stamp(uint64_t* buf, int idx, void* stream) {
  MIT_RECORD([=]() { return mit_stamp(buf, idx, stream); });
  MIT_CHECK_ARG(buf && idx >= 0, "mit_stamp: null buffer or negative index");
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, buf, idx);
  MIT_LAUNCH_CHECK("mit_stamp");
  return MIT_OK;
}

extern "C" int mit_step_inc(int64_t* step, void* stream) {
  MIT_RECORD([=]() { return mit_step_inc(step, stream); });
  MIT_CHECK_ARG(step, "mit_step_inc: null pointer");
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step);
  MIT_LAUNCH_CHECK("mit_step_inc");
  return MIT_OK;
}

extern "C" int mit_adamw(long n, float* param, const float* grad, float* m, float* v, void* shadow_bf16,
                         const float* norm_out, const float* lr, const int64_t* step, float beta1, float beta2,
                         float eps, float weight_decay, void* stream) {
  MIT_RECORD([=]() { return mit_adamw(n, param, grad, m, v, shadow_bf16, norm_out, lr, step, beta1, beta2, eps, weight_decay, stream); });
  MIT_CHECK_ARG(param && grad && m && v && lr && step, "mit_adamw: null pointer");
  MIT_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)m | (uintptr_t)v) % 16 == 0,
                "mit_adamw: buffers must be 16-B aligned");
  MIT_CHECK_ARG(!shadow_bf16 || ((uintptr_t)shadow_bf16 % 8) == 0, "mit_adamw: shadow must be 8-B aligned");
  if (n <= 0) return MIT_OK;
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = grid_for(n / 4 + 1, 256, 4096);
  if (shadow_bf16)
    hipLaunchKernelGGL(adamw_kernel<true>, dim3(g), dim3(256), 0, s, n, param, grad, m, v, (bf16*)shadow_bf16, norm_out,
                       lr, step, beta1, beta2, eps, weight_decay);
  else
    hipLaunchKernelGGL(adamw_kernel<false>, dim3(g), dim3(256), 0, s, n, param, grad, m, v, (bf16*)nullptr, norm_out,
                       lr, step, beta1, beta2, eps, weight_decay);
  MIT_LAUNCH_CHECK("mit_adamw");
  return MIT_OK;
}

extern "C" int mit_cast_f32(int dtype, long n, const float* src, void* dst, void* stream) {
  MIT_RECORD([=]() { return mit_cast_f32(dtype, n, src, dst, stream); });
  MIT_CHECK_ARG(src && dst, "mit_cast_f32: null pointer");
  if (n <= 0) return MIT_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(cast_kernel<T>, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, src,
                                       (T*)dst));
  MIT_LAUNCH_CHECK("mit_cast_f32");
  return MIT_OK;
}

extern "C" int mit_dropout_mask(long n, float p, const uint64_t* seed, uint32_t site, float* out, void* stream) {
  MIT_RECORD([=]() { return mit_dropout_mask(n, p, seed, site, out, stream); });
  MIT_CHECK_ARG(out, "mit_dropout_mask: null pointer");
  if (n <= 0) return MIT_OK;
  const float sc = p < 1.f ? 1.f / (1.f - p) : 0.f;
  hipLaunchKernelGGL(mask_kernel, dim3(grid_for(n)), dim3(256), 0, (hipStream_t)stream, n, seed, site,
                     drop_threshold(p), sc, out);
  MIT_LAUNCH_CHECK("mit_dropout_mask");
  return MIT_OK;
}

extern "C" int mit_scalar_div(const float* a, const float* b, float* out, void* stream) {
  MIT_RECORD([=]() { return mit_scalar_div(a, b, out, stream); });
  MIT_CHECK_ARG(a && b && out, "mit_scalar_div: null pointer");
  hipLaunchKernelGGL(scalar_div_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, a, b, out);
  MIT_LAUNCH_CHECK("mit_scalar_div");
  return MIT_OK;
}

extern "C" int mit_zero(void* p, long bytes, void* stream) {
  MIT_RECORD([=]() { return mit_zero(p, bytes, stream); });
  MIT_CHECK_ARG(p || bytes == 0, "mit_zero: null pointer");
  if (bytes <= 0) return MIT_OK;
  hipError_t e = hipMemsetAsync(p, 0, (size_t)bytes, (hipStream_t)stream);
  if (e != hipSuccess) {
    mit_set_error("mit_zero: %s", hipGetErrorString(e));
    return MIT_ERR_HIP;
  }
  return MIT_OK;
}
