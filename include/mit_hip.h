/* mit_hip.h — C ABI of libmit_hip.so, the MI355X (gfx950) kernels behind the captioning train step
 * of wazzuck/multimodal-image-transformer (frozen ViT/CLIP encoder + Transformer decoder).
 *
 * The reference has no native FFI: its "operator API" is the torch.nn / HF modules it calls
 * (SURVEY.md §8b). Each entry point below names the reference call site (file:line under
 * /root/reference, or the torch/transformers code those lines dispatch to) that it replaces.
 *
 * Conventions (all entry points):
 *   - plain device pointers + element counts/strides; no torch types. `stream` is a hipStream_t
 *     (NULL = default stream). Every launch is asynchronous on that stream; no entry point
 *     allocates, frees or synchronises, so any sequence of calls can be captured into a hipGraph.
 *   - dtype: MIT_BF16 (bf16 storage, fp32 math) or MIT_F32 (fp32 end to end: parity mode).
 *     Master weights, gradients, optimizer state, LayerNorm statistics and losses are always f32.
 *   - return 0 on success; MIT_ERR_INVALID for a rejected argument (nothing launched),
 *     MIT_ERR_HIP for a launch failure; mit_last_error() returns the message (thread-local).
 *   - dropout: p in [0,1); keep(i) = hash(*seed, site, i) >= p*2^32, kept values scaled by
 *     1/(1-p). `seed` is a DEVICE pointer (so graph replays draw fresh masks); NULL means 0.
 */
#ifndef MIT_HIP_H
#define MIT_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MIT_OK 0
#define MIT_ERR_INVALID 1
#define MIT_ERR_HIP 2

enum { MIT_F32 = 0, MIT_BF16 = 1 };
enum { MIT_K_CONTIG = 0, MIT_MN_CONTIG = 1 };
enum { MIT_ACT_NONE = 0, MIT_ACT_RELU = 1, MIT_ACT_GELU = 2, MIT_ACT_QUICK_GELU = 3 };
/* slots per row of the decode head's argmax keys (mit_decode_gemm_args.argmax_keys, mit_greedy_pick_keys) */
#define MIT_ARGMAX_SLOTS 16

const char* mit_last_error(void);
int mit_abi_version(void);

/* ---------------------------------------------------------------------------------------------
 * Launch plans (the host runtime of a train step; no reference counterpart — the reference's
 * per-op Python dispatch, train.py:80-100, is what it removes from the critical path).
 * mit_plan_begin() starts recording on the calling thread: every launching entry point below (and
 * mit_event_record / mit_stream_wait_event) still runs normally and ALSO appends a replay closure
 * with its arguments copied by value. mit_plan_end() stops and returns the plan; mit_plan_run()
 * re-issues the recorded launches, in order, on the recorded streams (device pointers and scalars
 * are fixed; per-step values must live in device memory, as they do in the train step). Host work
 * between launches (a collective) is not recorded: end the plan there and begin another. */
void* mit_plan_begin(void);
void* mit_plan_end(void);
long mit_plan_size(const void* plan);
int mit_plan_run(const void* plan);
void mit_plan_destroy(void* plan);
/* hipEventRecord / hipStreamWaitEvent on hipEvent_t / hipStream_t handles passed as void* (recordable) */
int mit_event_record(void* event, void* stream);
int mit_stream_wait_event(void* stream, void* event);

/* ---------------------------------------------------------------------------------------------
 * GEMM with fused epilogue. Replaces every nn.Linear / F.linear / addmm / mm of the hot path:
 *   encoder  tf/models/vit/modeling_vit.py:213-215,233,249-254 (q/k/v, o_proj, fc1+GELU, fc2+res)
 *            tf/models/clip/modeling_clip.py:338-350 (fc1 + quick_gelu)
 *   model    model.py:99,145 (projection)
 *   decoder  torch/nn/functional.py:6435 (packed in_proj), torch/nn/modules/transformer.py:1197-1199
 *            (linear1 + ReLU + dropout, linear2), decoder.py:124,191 (fc_out)
 *   backward the dX / dW products autograd would issue for the same layers (train.py:93).
 *
 * C[m,n] = out( dropout( auxmask( act( alpha * sum_k A(m,k) B(k,n) + bias[n] ) ) ) + residual[m,n] )
 *   A(m,k) = A[m*lda+k] (a_layout K_CONTIG) or A[k*lda+m] (MN_CONTIG)
 *   B(k,n) = B[n*ldb+k] (b_layout K_CONTIG) or B[k*ldb+n] (MN_CONTIG)
 *   auxmask: if aux != NULL, multiply by (aux[m*ld_aux+n] > 0 ? aux_scale : 0)  (ReLU/dropout bwd)
 *   dropout index = m*N + n ; residual/aux in the operand dtype; bias f32 [N]
 *   out_f32: write f32 (accumulate: C += value), else the operand dtype.
 *   rowsum (optional, f32 [M]): rowsum[m] = sum_k A(m,k) — the bias gradient when A = dY^T in a
 *     weight-gradient GEMM, fused in (no separate column-sum pass over dY).
 *   workspace: split-K scratch, size from mit_gemm_workspace_bytes(M, N, K); NULL / too small -> no
 *     split. One workspace per stream (launches sharing one must be ordered). Plain-epilogue GEMMs with
 *     few output tiles and a long K (weight gradients, the fc_out data gradient) write fp32 partials
 *     and a second launch reduces them in slice order (deterministic).
 * bf16 requirements: lda, ldb and the contiguous extent of each operand multiples of 8; A, B 16-B aligned. */
typedef struct {
  int dtype, a_layout, b_layout;
  long M, N, K;
  const void* A;
  long lda;
  const void* B;
  long ldb;
  void* C;
  long ldc;
  float alpha;
  const float* bias;
  int act;
  const void* residual;
  long ldr;
  const void* aux;
  long ld_aux;
  float aux_scale;
  float drop_p;
  const uint64_t* seed;
  uint32_t site;
  int out_f32;
  int accumulate;
  float* rowsum;
  void* workspace;
  long workspace_bytes;
  /* LayerNorm folded into the GEMM (the frozen encoder's pre-LN sublayers, encoder.py): A holds the raw
   * rows x of LN(x) = (x - mean) rstd gamma + beta, B = W o gamma (the folded weight), bias = b + W beta,
   * ln_colsum[n] = sum_k B(k, n): C = rstd_m (sum_k x_mk B_kn - mean_m ln_colsum_n) + bias_n, then the
   * activation; (mean_m, rstd_m) merged from ln_stats [M][ln_parts][2] = per-64-column (mean, M2) of
   * each row (ln_parts = K / 64), eps ln_eps. NULL: off. */
  const float* ln_stats;
  const float* ln_colsum;
  int ln_parts;
  float ln_eps;
  /* stats_out (f32 [M][N / 64][2], NULL: off): per-64-column (mean, M2) of each bf16-rounded output row
   * (the next LayerNorm's ln_stats). Both need bf16 NT operands and a plain bf16 vector epilogue
   * (stats_out: a residual, no activation); they run on the 256x256 tile kernel. */
  float* stats_out;
  /* tiles: the output tile choice. 0 = per shape (a cost model of this launch's rounds on an otherwise
   * idle chip); 256 = the 256x256 kernel wherever it applies (bf16 NT, M and N >= 256, no split-K): for a
   * caller whose other stream runs beside this launch, so a partial last round is not left idle
   * (encoder.forward_iter_groups); 128 = the 128x128 kernel. mit_gemm_set_variant 1 / 2 / 3 override it. */
  int tiles;
  /* argmax_keys (u64 [MIT_ARGMAX_SLOTS][M], NULL: off): the greedy pick folded into a vocabulary head, as
   * mit_decode_gemm_args.argmax_keys (same packed keys, slot = 128-column block % MIT_ARGMAX_SLOTS; C may be
   * NULL and is not written). bf16 NT operands, bias only (no activation, residual, aux, dropout, alpha 1; the
   * bias is read in 8-float vectors up to round8(N));
   * runs on the 128x128 kernel: the batched decode's head (M = 256, N = V) in one round of 158 blocks, 9-10 us,
   * against 20 us for mit_decode_gemm's 628 split-K 64x64 blocks at one per CU. */
  unsigned long long* argmax_keys;
} mit_gemm_args;
int mit_gemm(const mit_gemm_args* args, void* stream);
long mit_gemm_workspace_bytes(long M, long N, long K);
/* Tile-kernel choice for bf16 GEMMs: 0 = per shape (default), 1 = 128x128 kernel only, 2 = 256x256
 * kernel wherever split-K is not planned, 3 = the 64x64 register-streaming kernel for every NT GEMM
 * without rowsum / split-K, 4 = as 0 with the one-wave-per-SIMD 256x256 kernel for the NT GEMMs it
 * covers (K % 64 == 0; plain / bias / activation, LayerNorm fold, residual + statistics; bitwise equal to
 * the 256x256 kernel). Results are identical up to fp32 summation order; a test knob, not a numerics
 * switch. */
int mit_gemm_set_variant(int variant);
/* The launch mit_gemm would make for these args (no launch): returns the output tile edge of the
 * kernel (256 or 128 for bf16, 65 for the bf16 64x64 register-streaming kernel, 64 for the f32
 * kernel, 0 for an empty problem) and stores the
 * split-K factor in *ksplit (may be NULL). For profiling tools that attribute kernel time. */
int mit_gemm_plan(const mit_gemm_args* args, int* ksplit);
/* Grouped weight-gradient GEMMs: n (<= 8) problems in ONE launch (+ one split-K combine launch),
 * each a bf16 dW = dY^T X with both operands MN-contig, f32 output (alpha / accumulate honoured),
 * optional fused bias-gradient rowsum, no other epilogue. Replaces a decoder layer's six
 * nn.Linear / MHA weight gradients of autograd (torch/nn/functional.py linear backward), which at
 * d_model 512 are 16-64-tile grids that each leave most CUs idle. The split-K factor is chosen for the
 * group; workspace: >= mit_gemm_grouped_ws_bytes(args, n) bytes, 16-B aligned (no zero-fill needed). */
typedef struct {
  long rows, cols;    /* the mit_layernorm_bwd call that left its partials in ws (dgamma == NULL) */
  const float* ws;
  float* dgamma;      /* f32 [cols], overwritten */
  float* dbeta;
} mit_ln_grads_job;
/* ln (may be NULL, n_ln <= 4): LayerNorm parameter gradients reduced by extra blocks of the same grid
 * (what mit_layernorm_param_grads does in its own launch) -- a decoder layer's three norms. */
long mit_gemm_grouped_ws_bytes(const mit_gemm_args* args, int n);
int mit_gemm_grouped(const mit_gemm_args* args, int n, const mit_ln_grads_job* ln, int n_ln, void* workspace,
                     long workspace_bytes, void* stream);

/* ---------------------------------------------------------------------------------------------
 * LayerNorm over the last dim, fp32 statistics.
 * Replaces nn.LayerNorm in tf/models/vit/modeling_vit.py:274,281,385 (pre-LN, eps 1e-12),
 * tf/models/clip/modeling_clip.py:358,360,642 (eps 1e-5) and the post-LN residual blocks of
 * torch/nn/modules/transformer.py:1144-1153: y = LN(x + dropout(r)).
 *   r may be NULL (plain LN). z (may be NULL) receives x + dropout(r) (saved for the backward).
 *   mean/rstd (f32 [rows], may be NULL) saved for the backward. gamma/beta f32 [cols]. */
int mit_layernorm_fwd(int dtype, long rows, long cols, const void* x, long ldx, const void* r, long ldr,
                      float r_drop_p, const uint64_t* seed, uint32_t site, const float* gamma, const float* beta,
                      float eps, void* z, void* y, long ldy, float* mean, float* rstd, void* stream);

/* The encoder's f32 residual stream (encoder.py, as torch.autocast keeps HF ViT/CLIP's residual
 * adds: modeling_vit.py:312-323, modeling_clip.py:379-393): z = x + r, y = LN(z).
 *   x f32 [rows, ldx]; r = the sublayer's bf16 output (NULL: z = x); z f32 [rows, cols] (NULL: not
 *   written; may alias x; needs ldx == cols); y in y_dtype (MIT_BF16: the next GEMM's operand; MIT_F32: a new
 *   f32 stream, CLIP's pre_layrnorm). cols % 8 == 0, cols <= 1024, leading dims % 8 == 0, 16-B
 *   aligned pointers, y aliases neither x nor r. Replaces the same nn.LayerNorm calls as
 *   mit_layernorm_fwd (modeling_vit.py:274,281,385; modeling_clip.py:358,360,642). */
int mit_layernorm_fwd_x32(long rows, long cols, const float* x, long ldx, const void* r, long ldr, float* z,
                          const float* gamma, const float* beta, float eps, void* y, int y_dtype, long ldy, void* stream);
/* y (bf16) = x + r: the last residual add of the f32 stream, rounded for the encoder's consumers
 * (CLIP's last_hidden_state, modeling_clip.py:649, has no final LayerNorm). r may be NULL. */
int mit_residual_out(long rows, long cols, const float* x, long ldx, const void* r, long ldr, void* y, long ldy,
                     void* stream);

/* Backward of y = LN(z), z = x + dropout(r):
 *   dx = dz = dLN(dy) (dx may alias dy), dr = dz * dropout_mask (may be NULL)
 *   dgamma/dbeta: f32 [cols], overwritten. Both NULL: the per-block column partials are left in
 *     ws and mit_layernorm_param_grads reduces them later (e.g. on another stream, off the dX chain).
 *   ws: f32 workspace of >= mit_layernorm_bwd_ws_floats(rows, cols) floats. */
long mit_layernorm_bwd_ws_floats(long rows, long cols);
int mit_layernorm_bwd(int dtype, long rows, long cols, const void* dy, const void* z, const float* mean,
                      const float* rstd, const float* gamma, void* dx, void* dr, float r_drop_p, const uint64_t* seed,
                      uint32_t site, float* dgamma, float* dbeta, float* ws, void* stream);
int mit_layernorm_param_grads(long rows, long cols, const float* ws, float* dgamma, float* dbeta, void* stream);
/* Per-64-column (mean, M2) of each bf16 row: out[r][c / 64] = (mean, sum of squared deviations) over
 * columns c .. c + 63 (cols % 64 == 0): the ln_stats of a LayerNorm-folded GEMM (mit_gemm) whose input
 * rows no producer GEMM annotated (the encoder's embeddings). Replaces the statistics half of
 * nn.LayerNorm at modeling_vit.py:274 for layer 0. */
int mit_row_stats64(long rows, long cols, const void* x, long ldx, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Scaled-dot-product attention, head_dim Dh in {16, 32, 64, 128} (MFMA kernels at 64, generic
 * kernels otherwise), heads interleaved inside a token row (column h*Dh). The reference accepts any
 * nhead dividing d_model (decoder.py:112-118); configs[0] is d128 / 8 heads = head_dim 16.
 * Replaces: encoder MHSA (tf/models/vit/modeling_vit.py:164-189, no mask, scale 1/8);
 * decoder self-attention with the merged causal + key-padding float mask and attention dropout
 * (torch/nn/functional.py:6370-6404, 6553-6566, 6615-6633; masks from utils.py:30-36,66 — the
 * mask is never materialised: key j of batch b is masked iff j > i (causal) or
 * key_tokens[b*tok_batch + j] == pad_idx); decoder cross-attention (no mask).
 * Element strides: X(b, t, h, :) = X + b*X_batch + t*X_row + h*Dh. lse: f32 [B*H*Lq] (log-sum-exp
 * of the scaled, masked scores; required by the backward). A fully masked row yields NaN, as in
 * the reference. */
typedef struct {
  const void* q;
  long q_row, q_batch;
  const void* k;
  long k_row, k_batch;
  const void* v;
  long v_row, v_batch;
  void* o;
  long o_row, o_batch;
  float* lse;
  const int64_t* key_tokens;
  long tok_batch;
  int pad_idx;
  int causal;
  float scale;
  float drop_p;
  const uint64_t* seed;
  uint32_t site;
} mit_attn_args;
int mit_attention_fwd(int dtype, long B, long H, long Lq, long Lk, long Dh, const mit_attn_args* a, void* stream);

/* Backward (autograd of the same SDPA call). dq/dk/dv are overwritten (not accumulated).
 * delta_ws: f32 [B*H*Lq] workspace. */
typedef struct {
  const void* dout;
  long do_row, do_batch;
  void* dq;
  long dq_row, dq_batch;
  void* dk;
  long dk_row, dk_batch;
  void* dv;
  long dv_row, dv_batch;
  float* delta_ws;
} mit_attn_grads;
int mit_attention_bwd(int dtype, long B, long H, long Lq, long Lk, long Dh, const mit_attn_args* a,
                      const mit_attn_grads* g, void* stream);

/* Test knob: with dropout, the head-resident / 64-query MFMA attention kernels form the mask's element
 * index (b*H + h)*Lq*Lk + i*Lk + j in 32 bits, so calls with B*H*Lq*Lk >= limit (default 2^32) run the
 * 64-bit-index kernels (forward attn_fwd_simple, backward attn_bwd_dq/dkv_mfma). A smaller limit sends
 * small calls down that path (tests/test_kernels_gpu.py); limit <= 0 restores 2^32. Process-wide. */
int mit_attention_set_index_limit(double limit);

/* ---------------------------------------------------------------------------------------------
 * Encoder input assembly.
 * im2col of the patch Conv2d (tf/models/vit/modeling_vit.py:60,69; clip 148-154):
 *   out[(b*np + p) * kpad + (c*P*P + ky*P + kx)] = img[b, c, py*P+ky, px*P+kx]; columns >= C*P*P are 0.
 * assemble (modeling_vit.py:146-157, modeling_clip.py:212-219):
 *   h[b, 0, :] = cls + pos[0];  h[b, 1+p, :] = patch[b*np+p] + pos[1+p]. */
int mit_im2col(int dtype, long B, long C, long H, long W, long P, const float* img, void* out, long kpad, void* stream);
int mit_vit_assemble(int dtype, long B, long np, long E, const void* patch, const float* cls, const float* pos, void* h,
                     void* stream);

/* ---------------------------------------------------------------------------------------------
 * Decoder input: x = dropout(Emb[tok] * scale + pe[t]) (decoder.py:168-171, 71-72).
 * table in the operand dtype [V, d]; pe f32 [>=T, d]. */
int mit_embed_fwd(int dtype, long B, long T, long d, const int64_t* tokens, const void* table, float scale,
                  const float* pe, float drop_p, const uint64_t* seed, uint32_t site, void* out, void* stream);
/* dtable[tok] += scale * dropout_mask * dx (f32; caller zeroes dtable); the padding_idx row receives
 * no gradient (nn.Embedding(padding_idx=PAD), decoder.py:105; embedding backward of autograd).
 * plan != NULL: DETERMINISTIC — each token's row is the sum of its positions' rows in position order
 * (d % 8 == 0, B*T <= 16384); plan = int32 [mit_embed_plan_ints(B*T)] filled by mit_embed_plan from
 * the same tokens (one workgroup sorts (token, position); any time after the tokens are final).
 * plan == NULL: float atomics (order-dependent rounding). */
long mit_embed_plan_ints(long n);
int mit_embed_plan(const int64_t* tokens, long n, int* plan, void* stream);
int mit_embed_bwd(int dtype, long B, long T, long d, const int64_t* tokens, const void* dx, float scale, float drop_p,
                  const uint64_t* seed, uint32_t site, int pad_idx, const int* plan, float* dtable, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Cross-entropy with ignore_index (train.py:90,327 -> torch/nn/functional.py cross_entropy).
 * count_targets: *count += #(targets != ignore) as f32 (device scalar, caller zeroes).
 * ce: per row of logits [rows, V] (ld): loss_sum += -log_softmax(row)[t] for t != ignore;
 *     if want_grad, logits are overwritten IN PLACE by d(loss)/d(logits) =
 *     (softmax - onehot) / count[0], and by 0 for ignored rows. count is a device scalar (the
 *     GLOBAL non-PAD count: the reference's mean reduction, exact under data parallelism).
 *     row_loss (f32 [rows], may be NULL): scratch for a deterministic loss sum (per-row losses added
 *     in row order; bf16 rows with V <= 10240 also take the register-resident one-wave-per-row
 *     kernel). NULL: per-row float atomics into loss_sum (order-dependent rounding).
 * scalar_div: out[0] = a[0] / b[0] (mean loss = loss_sum / count, on device, no host sync). */
int mit_count_targets(const int64_t* targets, long n, int ignore_index, float* count, void* stream);
int mit_cross_entropy(int dtype, long rows, long V, void* logits, long ld, const int64_t* targets, int ignore_index,
                      const float* count, float* loss_sum, int want_grad, float* row_loss, void* stream);
int mit_scalar_div(const float* a, const float* b, float* out, void* stream);

/* bias gradient: out[n] (+)= sum_m dy[m*ld + n]  (f32 out; accumulate flag) */
int mit_colsum(int dtype, long M, long N, const void* dy, long ld, float* out, int accumulate, float* ws, void* stream);
long mit_colsum_ws_floats(long M, long N);

/* ---------------------------------------------------------------------------------------------
 * Optimizer: torch.nn.utils.clip_grad_norm_ (train.py:96-97; torch/nn/utils/clip_grad.py:165-186)
 * fused with torch.optim.AdamW (train.py:100,319-325; torch/optim/adam.py:419-547) over ONE flat
 * f32 parameter buffer. Sequence per step: mit_grad_norm (total norm + clip coefficient into
 * `norm_out` = {total_norm, coef}) then mit_adamw (reads coef, lr and the step count from device
 * memory, increments nothing — mit_step_inc bumps the device step counter first). */
long mit_grad_norm_ws_floats(long n);
int mit_grad_norm(const float* grads, long n, float max_norm, float* ws, float* norm_out, void* stream);
int mit_step_inc(int64_t* step, void* stream);
/* Profiling marker: buf[idx] = the device's constant-rate wall clock (hipDeviceAttributeWallClockRate)
 * when the stream reaches this point. Recorded into launch plans like any launch. */
int mit_stamp(uint64_t* buf, int idx, void* stream);
int mit_adamw(long n, float* param, const float* grad, float* m, float* v, void* shadow_bf16, const float* norm_out,
              const float* lr, const int64_t* step, float beta1, float beta2, float eps, float weight_decay,
              void* stream);

/* ---------------------------------------------------------------------------------------------
 * Batched greedy decoding with a KV cache (BASELINE config 5). Replaces the per-token full-prefix
 * recompute of ImageToTextModel.generate (model.py:171-242: decoder forward over ids[0..t], argmax
 * of the last position, stop at END) by one cached step per token for a whole batch. Every position
 * is read from the DEVICE scalar `pos` (int64), so one step captures into a hipGraph and replays.
 *
 * attention_decode: o[b, h*Dh:(h+1)*Dh] = softmax(q_bh . K_bh^T * scale) V_bh for ONE query per
 *   (b, h); keys j < Lk with Lk = *pos + 1 when pos != NULL (causal self-attention over the cache),
 *   else the fixed Lk (cross-attention over the image memory). Key j is masked when
 *   key_tokens[b*tok_batch + j] == pad_idx (the reference's key-padding mask, utils.py:47-70), when
 *   key_tokens != NULL. Head dim Dh in {16, 32, 64, 128}, heads at column h*Dh. All keys masked -> NaN.
 * kv_store: cache[b*c_batch + (*pos)*c_row + e] = src[b*s_batch + e], e < n.
 * embed_decode: out[b, :] = table[ids[b*ld_ids + *pos]] * scale + pe[*pos]   (decoder.py:168-171)
 * greedy_pick: ids[b*ld_ids + *pos + 1] = argmax_v logits[b*ld + v] (first maximal index, like
 *   torch.argmax, model.py:236) for rows not yet finished (finished rows get pad_id); a row whose
 *   pick is end_id sets finished[b] = 1 and increments *n_finished (int32 device scalars). */
int mit_attention_decode(int dtype, long B, long H, long Dh, const void* q, long q_batch, const void* k, long k_row,
                         long k_batch, const void* v, long v_row, long v_batch, void* o, long o_batch, long Lk,
                         const int64_t* pos, const int64_t* key_tokens, long tok_batch, int pad_idx, float scale,
                         void* stream);
int mit_kv_store(int dtype, long B, long n, const void* src, long s_batch, void* cache, long c_row, long c_batch,
                 const int64_t* pos, void* stream);
int mit_embed_decode(int dtype, long B, long d, const int64_t* ids, long ld_ids, const int64_t* pos, const void* table,
                     float scale, const float* pe, void* out, void* stream);
int mit_greedy_pick(long B, long V, const float* logits, long ld, int64_t* ids, long ld_ids, const int64_t* pos,
                    int64_t end_id, int64_t pad_id, int* finished, int* n_finished, void* stream);
/* greedy_pick, then *pos += 1 once every row's pick is stored (the last block to take `ticket`, an
 * int32 device counter that must start at 0 and is left at 0, advances it): the per-token step's
 * separate mit_step_inc launch folded in. */
int mit_greedy_pick_advance(long B, long V, const float* logits, long ld, int64_t* ids, long ld_ids, int64_t* pos,
                            int64_t end_id, int64_t pad_id, int* finished, int* n_finished, int* ticket, void* stream);
/* greedy_pick_advance from the argmax keys a mit_decode_gemm (argmax_keys) left (u64 [MIT_ARGMAX_SLOTS][B]):
 * with k the largest of row b's slot keys, column 0xFFFFFFFF - (u32)k is its pick; the keys are reset to 0
 * and *pos advanced (one block). */
int mit_greedy_pick_keys(long B, unsigned long long* keys, int64_t* ids, long ld_ids, int64_t* pos, int64_t end_id,
                         int64_t pad_id, int* finished, int* n_finished, void* stream);

/* Decode-step GEMM with the decoder's post-LN residual blocks folded in (bf16 only; the B-row GEMMs of
 * one token step, torch/nn/modules/transformer.py:1144-1153 norm_first=False):
 *   C[M, N] = act(A'[M, K] . B[N, K]^T + bias) (+ residual),  B = bf16 weights (nn.Linear layout)
 *   A' = A (bf16 rows, a_stats == NULL) or LN(A) with A = f32 pre-LN sums z and a_stats their row
 *        statistics as written by a producer's stats_out, gamma/beta f32 [K] (K <= 1024);
 *   residual (r_mode): 0 none, 1 bf16 rows r, 2 LN(r) with r = f32 pre-LN sums, r_stats, gamma/beta [N];
 *   outputs: C (bf16, or f32 when c_f32 -- the vocabulary head), z_out f32 (the pre-LN sum of the
 *   NEXT LayerNorm) with stats_out [M][ceil(N/64)][2] = per 64-column tile (mean, M2) of each row,
 *   merged exactly by the consumer (Chan); cache (bf16, may be NULL): for columns n >= kv_col0,
 *   cache[m*c_batch + (*pos)*c_row + n - kv_col0] = C value (the self-attention K|V row of this token).
 * LayerNorm eps = eps for both A and the residual. ReLU only without a residual. */
typedef struct {
  long M, N, K;
  const void* A;
  long lda;
  const float* a_stats;
  const float* a_gamma;
  const float* a_beta;
  const void* B;
  long ldb;
  const float* bias;
  int act;
  int c_f32;
  void* C;
  long ldc;
  int r_mode;
  const void* r;
  long ldr;
  const float* r_stats;
  const float* r_gamma;
  const float* r_beta;
  float eps;
  float* z_out;
  long ldz;
  float* stats_out;
  void* cache;
  long c_row, c_batch, kv_col0;
  const int64_t* pos;
  /* argmax_keys (u64 [MIT_ARGMAX_SLOTS][M], NULL: off): the greedy pick folded into the vocabulary head.
   * Each 64-column block's maximum of row m over act(A . B^T + bias) leaves as one atomic max of
   * ord(value) << 32 | (0xFFFFFFFF - column) (ord: the order-preserving u32 image of an f32, NaN
   * largest) into slot (column block % MIT_ARGMAX_SLOTS) of the row, so the largest key over the row's
   * slots is its first maximal column (torch.argmax). The slots spread the atomics: with one key per
   * row all 157 column blocks of a 10000-word head hit the same 32 cache lines of 256 rows' keys, and the
   * memory-side atomics on them serialised the launch (~29 us per token step). bf16 A rows, no residual
   * or activation; C / z_out may be NULL. The keys must be 0 before the launch (mit_greedy_pick_keys
   * leaves them 0). N need not be a multiple of 8 in this mode (any vocabulary: columns >= N never
   * enter the maximum). */
  unsigned long long* argmax_keys;
} mit_decode_gemm_args;
int mit_decode_gemm(const mit_decode_gemm_args* args, void* stream);
/* out[m, :] = LN(z[m, :]) (bf16) from the statistics a mit_decode_gemm stats_out wrote (W <= 1024):
 * the vocabulary head's operand, which then runs on mit_gemm. */
int mit_decode_layernorm(long M, long W, const float* z, long ldz, const float* stats, const float* gamma,
                         const float* beta, float eps, void* out, long ldo, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Utilities. cast: f32 -> operand dtype copy (weights to the bf16 shadow); fill f32.
 * dropout_mask_debug: writes the keep-multiplier (0 or 1/(1-p)) the kernels use at
 * (seed, site, idx) for idx in [0, n) — tests rebuild reference masks from it. */
int mit_cast_f32(int dtype, long n, const float* src, void* dst, void* stream);
/* zero `bytes` bytes at p (hipMemsetAsync on the stream; graph-capturable) */
int mit_zero(void* p, long bytes, void* stream);
int mit_dropout_mask(long n, float p, const uint64_t* seed, uint32_t site, float* out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Data path: rescale + normalise + HWC->CHW of a batch of uint8 RGB images
 * already resized / centre-cropped on the host (PIL, as the reference's HF processors do:
 * dataset.py:135, model.py:192; ViT mean = std = 0.5, CLIP OPENAI mean/std):
 *   dst[b, c, y, x] = ((float)src[b, y, x, c] / 255 - mean3[c]) / std3[c]   (f32, bit-identical
 *   to the processor's numpy pixel_values). src [B,H,W,3] uint8 (4-B aligned), dst [B,3,H,W] f32
 *   (16-B aligned); H*W % 4 == 0. mean3/std3: HOST arrays of 3 floats. */
int mit_image_normalize(long B, long H, long W, const uint8_t* src, float* dst, const float* mean3, const float* std3,
                        void* stream);

#ifdef __cplusplus
}
#endif
#endif
