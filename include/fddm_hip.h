/* libfddm_hip — C-ABI of the MI355X (gfx950) kernels behind the FDDM-ASR train step.
 *
 * The reference (TeemoCaption/FDDM-asr) has no FFI layer: its hot path is the Python module API
 * consumed by train.py. Each entry point below replaces the implicit torch op site(s)
 * cited next to it; the Python package fddm-asr_amd/ (models/*, losses/*, fddm/sched/*, train.py)
 * keeps the reference's module API and calls these through ctypes (fddm_hip/_lib.py).
 *
 * Conventions
 *  - All pointers are device pointers owned by the caller (torch tensors); the library allocates
 *    nothing and keeps no global state other than the persistent-GEMM workgroup cap below. Every call is
 *    asynchronous on `stream` (a hipStream_t).
 *  - dtype codes: 0 = f32, 1 = bf16. "T" below means the selected compute/storage dtype.
 *  - Return value: hipError_t as int (0 = success); fddm_error_string() describes it.
 *  - Randomness: counter-based (seed, stream, element index) splitmix64 — see oracle/fddm_oracle.py; the
 *    attention-probability dropout draws from per-(b, h) splitmix64 tables with per-row offsets (contract v2,
 *    oracle attn_dropout_keep).
 */
#ifndef FDDM_HIP_H
#define FDDM_HIP_H
#ifdef __cplusplus
extern "C" {
#endif

int fddm_abi_version(void);
const char* fddm_error_string(int code);

/* ---- GEMM (MFMA). C[m][n] = alpha * sum_k A(m,k) B(n,k) + bias[n], fused epilogue `epi`:
 *      0 store (out_dtype), 1 GELU (C = pre-activation, C2 = dropout(gelu)), 2 accumulate into f32 C,
 *      3 GELU only (C = gelu(acc); bf16 output on the 256x256 kernel: the bf16-output GELU fit, |err| <= 2.6e-5 —
 *      the frozen encoder's FF1 / conv layers), 4 dGELU (C = acc * gelu'(C2) * dropout mask).
 *      a_kc/b_kc: operand K-contiguous (1) or
 *      M/N-contiguous (0).  A rows batched: A + (m/Mi)*sAb + (m%Mi)*lda (Mi <= 0: unbatched).
 *      colsum (optional, M/N-contiguous A only): colsum[m] = sum_k A(m,k) — the fused bias gradient of
 *      a weight-gradient GEMM dW = dY^T X (colsum = sum over tokens of dY); like C it is overwritten
 *      for EPI_STORE and accumulated (+=) for EPI_ACC.
 *      Replaces every nn.Linear / F.linear forward and backward on the path:
 *      models/denoise_decoder.py:98-100,129-145,229,238  models/projection.py:14-55
 *      models/acoustic_encoder.py:55  HF modeling_wavlm.py:93-105,125-128,274-295 */
int fddm_gemm(int dtype, int a_dtype, int a_kc, int b_kc, int epi, int out_dtype, const void* A, long lda, long Mi,
              long sAb, const void* B, long ldb, void* C, long ldc, void* C2, const float* bias, float alpha, long M,
              long N, long K, unsigned long long seed, unsigned long long stream, float drop_p, float* colsum,
              void* hip_stream);

/* ---- self-attention input gradient through RoPE: dx[M][N] += rope_bwd(dy[M][K] @ w[K][N]) in one launch (the
 *      RoPE pairing of fddm_rope_bwd: column j with j + N/2, into columns 2j, 2j+1; tables cs / sn [L][N], row m at
 *      position m % L). bf16 dy (row stride ldy) and w (stored [K][N], row stride ldw), f32 dx; N % 128 == 0.
 *      Replaces fddm_gemm (A K-contiguous, B as stored, f32 store) into a temporary followed by fddm_rope_bwd
 *      (reference: models/denoise_decoder.py:150-156, apply_rope's backward). hipErrorInvalidValue when the shape
 *      or the kernel override (fddm_gemm_force_path) rules it out: the caller then takes the two-launch path. */
int fddm_linear_dx_rope(const void* dy, long ldy, const void* w, long ldw, float* dx, long lddx, const float* cs,
                        const float* sn, long M, long N, long K, long L, void* hip_stream);

/* ---- launch shape of the persistent 256x256 GEMM: at most `cap` workgroups (rounded down to a multiple
 *      of 8; 0 = one per CU). Returns the previous cap. train.py lowers it while it enqueues the frozen
 *      encoder of the next batch on a second stream, so the decoder's launches keep CUs of their own
 *      (reference: train.py:359 `encoder(wave)` inside the step loop). */
int fddm_gemm_persistent_cap(int cap);

/* ---- grouped weight-gradient GEMMs (one launch for the n <= 12 dW GEMMs of a decoder block):
 *      dw[p][m][n] += sum_k dy[p][k][m] * x[p][k][n]   (dy: [K][M] bf16, x: [K][N] bf16, row strides ldy/ldx;
 *      dw: f32, row stride lddw), db[p][m] += sum_k dy[p][k][m] (db[p] may be NULL). K is split into
 *      slices of about `kchunk` tokens (kchunk <= 0: no split); slices combine with f32 atomics.
 *      Arrays are host arrays of n entries. Replaces the weight/bias gradients autograd computes for the
 *      block's Linear / MultiheadAttention parameters: models/denoise_decoder.py:129-145 */
int fddm_gemm_dw_grouped(int n, const void* const* dy, const long* ldy, const void* const* x, const long* ldx,
                         float* const* dw, const long* lddw, float* const* db, const long* M, const long* N,
                         const long* K, long kchunk, void* hip_stream);

/* ---- implicit-GEMM Conv1d on channels-last input (epi 0 store / 3 GELU), `groups` along gridDim.z.
 *      HF modeling_wavlm.py:675-693 (conv layers 1..6), 37-90 (positional grouped conv). */
int fddm_conv1d_gemm(int dtype, int epi, const void* x, long lda, long sAb, long Tin, long Cg, long cstride,
                     long cpad, const void* W, void* out, long ldc, const float* bias, long Bn, long Tout, long N,
                     long K, int groups, void* hip_stream);

/* ---- WavLM positional conv embedding + GELU (bf16): pos[b][t][g*Cg+n] = gelu(bias + sum_{tap,c}
 *      x[b][t+tap-kp/2][g*Cg+c] W[g][n][tap*Cg+c]), t < S (the SamePad drops the conv's last frame).
 *      x/out [B][S][E], W [G][Cg][kp*Cg], Cg = E/G a multiple of 16 (<= 64). HF modeling_wavlm.py:37-90. */
int fddm_posconv_gelu(const void* x, const void* W, const float* bias, void* out, long B, long S, long E, int G,
                      int kp, void* hip_stream);

/* ---- conv layer 0 + GroupNorm + GELU. HF modeling_wavlm.py:723-744. ws: f64 scratch (need not be zeroed) of
 *      B*nb*(K + K*(K+1)/2) + B*C doubles, nb = ceil(T0 / 4096) (per-block Gram statistics, then the GroupNorm
 *      affine). */
int fddm_conv0_gn_gelu(int out_dtype, const float* x, const float* w, const float* gamma, const float* beta,
                       double* ws, void* out, long B, long nsamp, long T0, int C, int K, int S, float eps,
                       void* hip_stream);

/* ---- WavLM gated rel-pos gate [B*H][S]. HF modeling_wavlm.py:166-180. */
int fddm_wavlm_gate(int dtype, const void* x, const float* W, const float* bias, const float* cst, float* gate, long B,
                    long S, int H, long E, void* hip_stream);

/* ---- attention (head_dim 64). Element (b,pos,h,d) at base + (b*L+pos)*stride + h*64 + d.
 *      nn.MultiheadAttention (models/denoise_decoder.py:129-130,164,169-174) with key_padding_mask
 *      (key_keep[b][k] != 0 keeps) and attention-prob dropout (drop_bits, optional: a buffer of
 *      fddm_attn_drop_words u64 holding the keep bits — round-4 layout: [B*H][ceil(Lk/64)][Lq] words, bit kk of word
 *      (bh, t, q) = keep(q, key 64t + kk); layout v3: see fddm_attn_drop_words — the backward reads them instead of
 *      rehashing); drop_bits_ready != 0: fddm_attn_drop_bits already wrote this site's words (the forward only reads
 *      them), else the forward produces them itself;
 *      WavLM relative-bias attention
 *      (HF modeling_wavlm.py:152-200) via gate [B*H][Lq] and table [H][2*Lk-1]. lse: [B*H][Lq].
 *      fddm_attn_drop_bits: the keep-bit words of nsites sites of one shape at once (rng streams stream0 +
 *      s*stream_step, site s at out + s*site_words) — the decoder produces every block's words in two launches ahead
 *      of its forward (models/denoise_decoder.py:164,169-176 dropout sites 1 and 3 of each block). */
int fddm_attn_fwd(int dtype, const void* Q, long sq, const void* K, long sk, const void* V, long sv, void* O, long so,
                  float* lse, const unsigned char* key_keep, const float* gate, const float* table, int B, int H,
                  int Lq, int Lk, float scale, float drop_p, unsigned long long seed, unsigned long long stream,
                  unsigned long long* drop_bits, int drop_bits_ready, void* hip_stream);
int fddm_attn_drop_bits(unsigned long long* out, long site_words, int nsites, int B, int H, int Lq, int Lk,
                        float drop_p, unsigned long long seed, unsigned long long stream0,
                        unsigned long long stream_step, void* hip_stream);
/* u64 words per site of a keep-bit buffer (room for either storage layout; site_words must be at least this).
 * fddm_attn_drop_bits writes the layout of the kernels that will read it: for Lk <= 1024 under the default family
 * (the bf16 32x32x16 kernels) layout v3 of csrc/attn7.hip (one
 * 64-bit lane mask per score-MFMA accumulator register: word ((bh*ceil(Lq/32) + qg)*ceil(Lk/64) + t)*32 + 16*kb + r,
 * bit l = keep(query 32*qg + (l&31), key 64*t + 32*kb + 8*(r>>2) + 4*(l>>5) + (r&3))); for Lk > 1024 or under
 * fddm_attn_set_kernels(1) the round-4 words above. Recorded bits are for bf16 attention (the fp32 kernels draw
 * their own). The keep decisions are the same (RNG contract v2). */
long fddm_attn_drop_words(int B, int H, int Lq, int Lk);
/* WavLM variant (bf16): the gate is computed in the kernel from the 8 gru_rel_pos_linear pre-activations per
 * (token, head) stored at graw + (b*Lq+q)*sgr + h*8 (bf16, appended to the Q|K|V projection's output) and
 * gconst [H] (gru_rel_pos_const) — HF modeling_wavlm.py:177-186. */
int fddm_attn_fwd_relgate(const void* Q, long sq, const void* K, long sk, const void* V, long sv, void* O, long so,
                          const void* graw, long sgr, const float* gconst, const float* table, int B, int H, int Lq,
                          int Lk, float scale, void* hip_stream);
/* WavLM variant (bf16) with the gate computed in the kernel from the attention input x (bf16 rows at x + (b*Lq+q)*sx,
 * head h's 64 inputs at + h*64) and the folded gru_rel_pos_linear weights gw = [sum of weight rows 0-3 (64 floats) |
 * rows 4-7 (64) | sum of bias 0-3 | sum of bias 4-7] (the reference sums the 4 + 4 pre-activations, so the sums of
 * the rows give the same gate): no extra Q|K|V columns and no gate pass — HF modeling_wavlm.py:177-186. */
int fddm_attn_fwd_relgate_x(const void* Q, long sq, const void* K, long sk, const void* V, long sv, void* O, long so,
                            const void* x, long sx, const float* gw, const float* gconst, const float* table, int B,
                            int H, int Lq, int Lk, float scale, void* hip_stream);
/* Backward: dQ, dK, dV. bf16 with recorded or no dropout, Lq <= 256 and Lk <= 512: one fused
 * 32x32x16-MFMA launch per (b, h) (csrc/attn7.hip bwdf7: P and dP computed once, dQ of each query tile from the keys
 * in LDS; with Lk > 256 two key passes, the first leaving f32 dQ partials in delta_ws, 64 floats per query row).
 * Other bf16 shapes with Lk <= 1024 (or fddm_attn_set_kernels(2)): the 32x32x16-MFMA pair (a query-owned dQ launch
 * that also writes the per-query row terms delta = rowsum(dO O) and -LSE log2(e) into delta_ws, laid out
 * [2][B*H][LqP] with LqP = Lq rounded up to 64, and Q pre-scaled by scale*log2(e) in bf16 as [B*H][LqP][64] after
 * them, then a key-owned dK/dV launch that reads them). delta_ws must hold fddm_attn_bwd_ws_floats(B, H, Lq, Lk)
 * = 64 * B*H*LqP floats whichever kernels run (ABI 6; ABI 5 needed 34, ABI 4 B*H*Lq). Otherwise (fp32, rehashed dropout,
 * longer keys, or fddm_attn_set_kernels(1)): bf16 self-attention shapes Lq == Lk <= 256 as one fused launch, else a
 * dQ launch writing delta_ws [B*H][Lq] and a dK/dV launch. */
long fddm_attn_bwd_ws_floats(int B, int H, int Lq, int Lk);
int fddm_attn_bwd(int dtype, const void* Q, long sq, const void* K, long sk, const void* V, long sv, const void* O,
                  long so, const void* dO, long sdo, const float* lse, void* dQ, long sdq, void* dK, long sdk,
                  void* dV, long sdv, float* delta_ws, const unsigned char* key_keep, int B, int H, int Lq, int Lk,
                  float scale, float drop_p, unsigned long long seed, unsigned long long stream,
                  const unsigned long long* drop_bits, void* hip_stream);

/* ---- residual + dropout + LayerNorm (+FiLM). models/denoise_decoder.py:87-89,165-191;
 *      HF modeling_wavlm.py:102,313-317,405. rope_out (optional, bf16; the decoder's LN3 only: f32 x, bf16 y and
 *      output, no FiLM): also writes RoPE(out) with the [rope_L][d] cos / sin tables, as fddm_rope_fwd would
 *      (models/denoise_decoder.py:42-53,157-159: the next block's q = k input). */
int fddm_ln_fwd(int x_dtype, int y_dtype, int out_dtype, const void* x, const void* y, const float* gamma,
                const float* beta, const float* film_scale, const float* film_shift, float* out_f32, void* out_t,
                float* save_s, float* mean, float* rstd, long N, long d, long rows_per_batch, float eps, float drop_p,
                unsigned long long seed, unsigned long long stream, const float* rope_cos, const float* rope_sin,
                void* rope_out, long rope_L, void* hip_stream);
int fddm_ln_bwd(int dy_dtype, const float* dout, const float* s, const float* mean, const float* rstd,
                const float* gamma, const float* beta, const float* film_scale, float* dres, void* dy_t,
                float* dgamma, float* dbeta, float* dfilm_scale, float* dfilm_shift, long N, long d,
                long rows_per_batch, float drop_p, unsigned long long seed, unsigned long long stream,
                float* partials, void* hip_stream);
/* partials (optional; the fused pass, dgamma given): instead of adding its dgamma / dbeta (and FiLM) sums with device
 * atomics, row slab k of fddm_ln_bwd_slab_rows() rows stores them to partials[k][q][0..d), q = dgamma, dbeta, dFiLM
 * scale, dFiLM shift (ceil(N / rows) slabs x 4 x d floats); fddm_ln_fold adds them to their destinations later, up
 * to 4 LayerNorms in one launch, in a fixed order (dfilm_* [B][d] per FiLM batch of slabs_per_batch slabs; NULL
 * arrays or entries: no FiLM). Shapes the fused pass does not take (unaligned rows, FiLM batches not a multiple of
 * the slab) add with atomics and zero the partials. */
int fddm_ln_bwd_slab_rows(void);
int fddm_ln_fold(int n, const float* const* partials, const long* nslab, const long* d, float* const* dgamma,
                 float* const* dbeta, float* const* dfilm_scale, float* const* dfilm_shift,
                 const long* slabs_per_batch, void* hip_stream);

/* ---- RoPE on the block input (models/denoise_decoder.py:42-53,157-159). cs/sn: [L][d]. */
int fddm_rope_fwd(int out_dtype, const float* x, const float* cs, const float* sn, void* out, long N, long L, long d,
                  void* hip_stream);
int fddm_rope_bwd(const float* dy, const float* cs, const float* sn, float* dx, long N, long L, long d,
                  void* hip_stream);

/* ---- token embedding + time bias (models/denoise_decoder.py:214,254,272-274). */
int fddm_embed_fwd(int out_dtype, const long* tok, const float* E, const float* tbias, float* out, void* out_t, long N,
                   long L, long d, void* hip_stream);
int fddm_embed_bwd(const long* tok, const float* dx, float* dE, float* dtb, long N, long L, long d, long pad_id,
                   void* hip_stream);

/* ---- helpers: column sums (bias grads), dtype casts */
int fddm_colsum(int dtype, const void* X, float* out, long M, long N, long ldx, void* hip_stream);
int fddm_cast(int src_dtype, int dst_dtype, const void* x, void* y, long n, void* hip_stream);

/* ---- discrete diffusion: q_sample draw (train.py:180-188; diffusion_scheduler.py:31-50) and the
 *      categorical KL + exact gradient (train.py:190-255). thr: [T] uint32 keep thresholds. */
int fddm_sample_q(const long* x0, const long* t, const unsigned* thr, long* xt, long B, long L, long K,
                  unsigned long long seed, unsigned long long stream, void* hip_stream);
int fddm_kl_fwd(const float* logits, const long* xt, const long* x0, const long* t, const float* betas, float* kl_tok,
                long N, long L, long V, void* hip_stream);
int fddm_kl_bwd(const float* logits, const long* xt, const long* x0, const long* t, const float* betas,
                const float* w, const float* gscale, void* dz, int dz_dtype, long N, long L, long V,
                void* hip_stream);
/* the train step's form: kl_tok and dz = w * d kl_tok / d logits in one pass over the logits (w = the masked-mean
 * weights of fddm_kl_reduce, from mask [N] uint8 or NULL = plain mean over L); the upstream scalar is applied by
 * fddm_scale_if afterwards (no memory traffic when it is 1). */
int fddm_kl_fused(const float* logits, const long* xt, const long* x0, const long* t, const float* betas,
                  const unsigned char* mask, float* kl_tok, void* dz, int dz_dtype, long N, long L, long V,
                  void* hip_stream);
int fddm_scale_if(void* x, int dtype, const float* g, long n, void* hip_stream);
/* L_fd steps, bf16: the TextEmbedding softmax backward summed with the KL's gradient straight into the bf16
 * logits gradient the head GEMMs read (out may alias add), and the KL's upstream scalar applied to its share. */
int fddm_softmax_bwd_add_bf16(const void* y, const void* dy, const void* add, void* out, long N, long V,
                              void* hip_stream);
int fddm_axpy_if_bf16(void* x, const void* y, const float* g, long n, void* hip_stream);

/* ---- TextEmbedding softmax (models/projection.py:41-47) */
int fddm_softmax_rows(const float* x, void* y, int out_dtype, long N, long V, void* hip_stream);
int fddm_softmax_bwd_rows(const void* y, const void* dy, float* dz, int dtype, long N, long V, int accumulate,
                          void* hip_stream);

/* ---- L_fd (losses/fddm_losses.py:18-58): batch-dim standardisation and the Barlow-Twins loss */
int fddm_lfd_std_fwd(int out_dtype, const float* z, void* zt, float* inv_std, long B, long C, float eps,
                     void* hip_stream);
int fddm_lfd_std_bwd(int zt_dtype, const float* dzt, const void* zt, const float* inv_std, float* dz, long B, long C,
                     void* hip_stream);
int fddm_lfd_loss(const float* Cm, float* loss, long D, float lam, void* hip_stream);
int fddm_lfd_dloss(int out_dtype, const float* Cm, const float* gscale, void* dC, long D, float lam, void* hip_stream);
/*      data-parallel L_fd with global-batch statistics (fddm_losses.py:23-24 standardises over the
 *      whole batch): per-rank column partial sums, all-reduced by the caller between the passes (inv_n = 1/N_global).
 *      colstat: mean_sum == NULL -> out = sum_b z; else out = sum_b (z - mean_sum*inv_n)^2.
 *      bwd_colstat: out[0:C] = sum_b dz~, out[C:2C] = sum_b dz~ z~.  std_bwd_apply multiplies dz by `scale`. */
int fddm_lfd_colstat(const float* z, float* out, const float* mean_sum, float inv_n, long B, long C, void* hip_stream);
int fddm_lfd_std_apply(int out_dtype, const float* z, void* zt, float* inv_std, const float* s1, const float* s2,
                       float inv_n, float eps, long B, long C, void* hip_stream);
int fddm_lfd_bwd_colstat(int zt_dtype, const float* dzt, const void* zt, float* out, long B, long C, void* hip_stream);
int fddm_lfd_std_bwd_apply(int zt_dtype, const float* dzt, const void* zt, const float* inv_std, const float* sums,
                           float inv_n, float scale, float* dz, long B, long C, void* hip_stream);

/* ---- GEMM kernel-family override for tests and diagnostics (0 = automatic; 1 no 256x256 kernel, 2 register-staged
 *      128x128 only, 3 256x256 wherever its preconditions hold, 4 128x128 LDS-DMA ring wherever they hold). Returns
 *      the previous setting. Process-wide; the train step never sets it. */
int fddm_gemm_force_path(int path);
/* ---- attention kernel-family override for tests and diagnostics: 1 = the 16x16x32-MFMA kernels (fwd6, dq4 / dkv4,
 *      bwd3s) wherever the 32x32x16-MFMA family (csrc/attn7.hip) would run, 2 = the 32x32x16 family without its fused
 *      backward (dq7 + dkv7 at every Lk), 3 = the default with every forward on the one-chain fwd7, 4 = the default
 *      with every forward on the two-chain fwd8 (csrc/attn8.hip), 5 = the default with WavLM's gated relative-position
 *      attention on the round-2 fwd5 instead of fwd7's bias build, 0 = automatic (default: fwd8 unless its 256-query
 *      workgroups load the busiest CU with more queries than fwd7's 128-query ones; WavLM attention with Lk <= 1024 on
 *      fwd7 with the bias). Returns the previous setting.
 *      Process-wide; the train step never sets it. */
int fddm_attn_set_kernels(int v6);


/* ---- dropout-seed offset for HIP-graph replays of the train step: every launch enqueued while `off` (a device u64)
 *      is set reads its effective dropout seed as seed + *off at run time (null: none), so one captured step replays
 *      with the seeds the host's counter has moved on to (identical to an eager step's). Returns 1 if one was set. */
int fddm_set_seed_offset(const unsigned long long* off);

/* ---- clip_grad_norm_ + AdamW (train.py:411-423), multi-tensor over a chunk table.
 *      fddm_adamw: bias corrections from the per-tensor device step counters `step` (advanced by the call);
 *      max_norm > 0 clips by the gradient norm sqrt(*total); a non-finite *total skips the whole step (the
 *      reference's GradScaler skip, train.py:401-413) and increments *skipped (optional). zero_g != 0: every
 *      gradient element is set to 0 in the same pass, applied or skipped (the next step's zero_grad of the grad
 *      arena, folded into the optimizer's read of it). grad_scale multiplies every gradient before the clip and the
 *      update (1 normally; 1/W under data parallelism, where the gradient all-reduce leaves the ranks' SUM and the
 *      average is folded in here instead of a separate pass over the gradients). */
int fddm_grad_sumsq(const long* chunk_tensor, const long* chunk_start, const long* numel, const float* const* g,
                    long nchunks, float* total, void* hip_stream);
int fddm_adamw(const long* chunk_tensor, const long* chunk_start, const long* numel, float* const* p,
               const float* const* g, float* const* m, float* const* v, unsigned short* const* pbf,
               float* const* step, long ntensors, long nchunks, const float* total, float max_norm, float lr,
               float lr_wd, float b1, float b2, float eps, int* skipped, int zero_g, float grad_scale,
               void* hip_stream);

/* ---- small per-batch ops (rows = the batch, fp32): the decoder's conditioning path and the KL reduction.
 *      rows_mean: out[b][j] = mean_s x[b][s][j] — the pooled condition of FiLM (models/denoise_decoder.py:185).
 *      time_embed: SinusoidalTimeEmbedding features (models/denoise_decoder.py:108-116).
 *      small_linear: for each of njobs weight sets, out_j = act(in W_j^T + b_j) (transpose_w: in W_j), act 0 none,
 *        1 out = pre and out2 = silu(pre), 2 out = acc * silu'(aux) — the time MLP and FiLM Linears
 *        (models/denoise_decoder.py:89,98-100,274) and their input gradients; njobs <= 16.
 *      small_dw: dW_j += dy_j^T x_j, db_j += colsum(dy_j) over R rows — their weight gradients.
 *      kl_reduce: SchedulerAdapter.kl_term's masked mean over L and mean over B of kl_tok (train.py:247-253),
 *        plus w = d loss / d kl_tok for the closed-form gradient; mask may be NULL (plain mean). */
int fddm_rows_mean(int dtype, const void* x, float* out, long B, long S, long d, void* hip_stream);
int fddm_time_embed(const long* t, float* emb, long B, long d, float max_steps, void* hip_stream);
int fddm_small_linear(const float* in, long ldi, int njobs, const float* const* W, const float* const* bias,
                      float* const* out, float* const* out2, long ldw, long ldo, const float* aux, long R, long N, long K,
                      int act, int transpose_w, void* hip_stream);
int fddm_small_dw(int njobs, const float* const* dy, const long* lddy, const float* const* x, const long* ldx,
                  float* const* dW, float* const* db, const long* N, const long* K, long R, void* hip_stream);
int fddm_kl_reduce(const float* kl_tok, const unsigned char* mask, float* w, float* loss, long B, long L,
                   void* hip_stream);

/* ---- jumpy sampler denoise step (sampler/jumpy_sampler.py:167-215 + q_posterior_multi_step,
 *      fddm/sched/diffusion_scheduler.py:106-208): x_next = argmax (or a tempered draw) of the
 *      multi-step posterior q(x_{t-Δ} | x_t, softmax(logits)); x0hat = argmax logits.
 *      coef: per batch element {a_cum, b_cum, a_tg, b_tg} (exact) or {abar, 0, 0, 0} (fast).
 *      mode: bit0 fast (ᾱ/uniform mix, jumpy_sampler.py:138-151), bit1 sample (Categorical). */
int fddm_jump(const float* logits, long ldz, const long* xt, const float* coef, long* x_next, long* x0hat, long N,
              long L, long V, int mode, float temperature, unsigned long long seed, unsigned long long stream,
              void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif
