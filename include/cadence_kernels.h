/*
 * cadence_kernels.h -- C ABI of the MI355X (gfx950) CadenceGemma forward path.
 *
 * Plain pointers + sizes only (no torch types).  Every entry point:
 *   - takes device pointers that the caller allocated (no allocation inside),
 *   - enqueues on `stream` (a hipStream_t passed as void*), never syncs, so
 *     it is safe to capture into a hipGraph,
 *   - returns 0 on success or a hipError_t value (hipErrorInvalidValue = 1
 *     for a shape/alignment contract violation, checked on the host).
 *
 * Tensor conventions: bf16 is raw 16-bit storage (uint16_t on the host),
 * row-major, leading dimensions ("ld*") are in elements.  M = rows (tokens),
 * N = output features, K = reduction.  Weights W are [N][K] (nn.Linear
 * layout; weights stored [K][N] by the reference, e.g. Einsum ffw_up, are
 * packed once by the host).
 *
 * Decode weight layout: a weight leading dimension of 0 (ldw / lde == 0)
 * means W is FRAGMENT-PACKED, accepted by the M <= 64 (decode) engines only:
 *   Wp[((n / 16) * (K / 32) + k / 32) * 512 + l * 8 + e]
 *       = W[16 * (n / 16) + l % 16][32 * (k / 32) + 8 * (l / 16) + e]
 * for lane l in [0, 64), e in [0, 8) -- the MFMA 16x16x32 operand fragment
 * order, so every wave load is 1 KiB contiguous and a workgroup's weight
 * stream is one contiguous range.  Requires N % 16 == 0, K % 32 == 0;
 * grouped launches pack each group separately.
 *
 * Decode activation layout ("packed rows"): an ACTIVATION leading dimension
 * of 0 (lda of a GEMM A operand, ldo / ld_norm / ldy / ld_out of the
 * decode-side producers) means the M <= 32 rows are stored in the MFMA
 * A-fragment order, mt = ceil(M / 16):
 *   Xp[((k / 32) * mt + m / 16) * 512 + (m % 16 + 16 * ((k % 32) / 8)) * 8 + k % 8]
 *       = X[m][k]
 * so a decode GEMV loads 1 KiB of contiguous activations per wave
 * instruction (row-major fragment loads halve its weight-stream rate).
 * Requires K % 32 == 0; a packed buffer holds K * 16 * mt elements.
 * Producers: cadence_rmsnorm (ldo = 0), cadence_gemm_linear_rmsnorm
 * (ld_norm = 0), cadence_gemm_linear_residual_rows (out_rows, unnormalised),
 * cadence_gemm_gated_gelu (ldo = 0), cadence_rglru_step
 * (ldy = 0), cadence_local_attention_decode (ld_out = 0).  Consumers: the
 * A operand of cadence_gemm_linear, cadence_gemm_linear_rmsnorm,
 * cadence_gemm_gated_gelu, cadence_gemm_logits, cadence_logits_argmax.
 *
 * Deferred RMSNorm (decode): a residual projection that feeds an RMSNorm
 * (y = RMSNorm(x) = bf16(bf16(x * r) * (1 + s)), r = rsqrt(mean(x^2) + eps),
 * layers.py:70-78) may hand the consuming GEMV the unnormalised rows x
 * (cadence_gemm_linear_residual_rows).  The consumer's W then holds
 * bf16(W[n][k] * bf16(1 + s[k])) (the scale folded into the weight columns,
 * once per weight), and the kernel computes each row's r from x (sum of
 * squares in fp32 on the MFMA pipe; var, var + eps and r rounded to bf16 as
 * the reference) and scales the fp32 dot products by r before its
 * epilogue.  Equal to the reference up to the per-element bf16 roundings of
 * x * r and of the product with 1 + s, which it skips (tolerance-tested,
 * tests/test_decode_norm_gpu.py).
 *
 * The reference (`surakku/cadence-gemma`) has no native layer: each entry
 * point replaces a sequence of eager PyTorch ops (or timm ops) of the
 * reference Python path, cited per function.  The Python host
 * (cadence-gemma_amd/cadence) binds these as torch.ops.cadence.* custom ops.
 */
#ifndef CADENCE_KERNELS_H_
#define CADENCE_KERNELS_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- library info ------------------------------------------------------ */

/* Returns the ABI version (bumped on any signature change). */
int cadence_abi_version(void);

/* Bytes of fp32 split-K workspace the GEMM entry points need for (M, N, K)
 * (0 for the tile engine).  `groups` multiplies N for grouped launches. */
int64_t cadence_gemm_workspace_bytes(int64_t M, int64_t N, int64_t K,
                                     int64_t groups);

/* Output-tile height (rows) the prefill GEMM engine uses for (M, N, K,
 * groups): 256, 224, 192 or 160; 0 when M is small enough for the decode engines.
 * Host-only arithmetic (profiling / kernel-name bookkeeping). */
int cadence_gemm_tile_rows(int64_t M, int64_t N, int64_t K, int64_t groups);

/* K splits the prefill GEMM engine uses for (M, N, K, groups): > 1 when its
 * output tiles would leave most CUs idle (small M: one image / one prompt),
 * then gemm_big_kernel<EpiPartial, ...> writes fp32 split partials to the
 * workspace (cadence_gemm_workspace_bytes) and splitk_reduce_kernel applies
 * the epilogue to the split-order sums.  Host-only arithmetic. */
int cadence_gemm_big_splits(int64_t M, int64_t N, int64_t K, int64_t groups);

/* The prefill engine a launch of this shape takes: 1 = the 4-wave
 * gemm_w4_kernel<Epi, rows / 32>, 0 = gemm_big_kernel (or, M <= 64, the
 * decode engines).  Host-side plan query. */
int cadence_gemm_engine(int64_t M, int64_t N, int64_t K, int64_t groups);

/* Lab A/B switch of the prefill engines, a bit mask (default 15): bit 0 =
 * the 4-wave gemm_w4_kernel for K >= 2048 on 224 / 256-row tile plans (else
 * the 8-wave gemm_big_kernel), bit 1 = prefill RG-LRU gates of 64 / 128 /
 * 256-wide blocks on rglru_gates_stream_kernel, bit 2 = the linear GEMM with
 * a residual loads its residual rows ahead of the staged epilogue (same
 * bits), bit 3 = cadence_vit_attention on the streaming kernel with
 * MFMA-computed softmax sums for every sequence length (else the LDS-resident
 * kernel up to 288 tokens and the round-3 streaming kernel above); 0 = the
 * 8-wave block engine with the plain epilogues for everything.  A negative
 * value only queries.  Returns the previous value.  Host state only. */
int cadence_gemm_set_engine(int engine);

/* ---- GEMMs with fused epilogues ---------------------------------------- */

/* out[map(m), n] = act(A[m,:] . W[n,:] + bias[n]) (+ resid[map(m), n])
 *   act: 0 = none, 1 = GELU(erf), 3 = GELU(tanh).  map(m) = (m / row_div) * row_mul +
 *   (m % row_div) + row_off (row_div = M, row_mul = 0, row_off = 0 -> id).
 * Replaces nn.Linear / F.linear (+ the residual add):
 *   recurrentgemma/torch/modules.py:634,637,652 (RecurrentBlock linears),
 *   :429-431,481 (attention projections), :757 (ffw_down), :908,913
 *   (residual adds); recurrentgemma/projector/mlp.py:13-31 (projector);
 *   timm ViT qkv / fc1 (+GELU) (dino_siglip.py:85-86 call sites). */
int cadence_gemm_linear(const void* A, int64_t lda, const void* W, int64_t ldw,
                        const void* bias, const void* resid, int64_t ld_resid,
                        void* out, int64_t ldo, int64_t M, int64_t N, int64_t K,
                        int act, int64_t row_div, int64_t row_mul,
                        int64_t row_off, void* workspace, int64_t ws_bytes,
                        void* stream);

/* Decode (M <= 32 sequences, one token each) projection of the recurrent
 * block's two branches fused with the Conv1D decode step of the x branch
 * (replaces cadence_gemm_linear + cadence_conv1d with a cache, L == 1;
 * reference modules.py:340-352 linear_y / linear_x, layers.py:478-483):
 *   yx = A . W^T + bias                    (W = [linear_y; linear_x], N = 2E)
 *   out[:, :conv_lo]  = yx[:, :conv_lo]    (the y branch, as is)
 *   out[:, conv_lo:]  = conv1d_step(yx[:, conv_lo:]; conv_w [TW][E], conv_b,
 *                                   conv_state [M][TW-1][E], shifted in place)
 * W may be fragment-packed (ldw == 0) and A packed rows (lda == 0).  K must
 * fit one split of the weight-streaming engine (K <= 2560); TW <= 4.
 * norm != 0: normalise on load (see "Deferred RMSNorm" above): A is the
 * unnormalised packed rows of cadence_gemm_linear_residual_rows and W carries
 * the block's temporal_pre_norm scale. */
int cadence_gemm_linear_conv1d(const void* A, int64_t lda, const void* W,
                               int64_t ldw, const void* bias, void* out,
                               int64_t ldo, int64_t M, int64_t N, int64_t K,
                               int64_t conv_lo, const void* conv_w,
                               const void* conv_b, void* conv_state,
                               int64_t temporal_width, int norm,
                               float norm_eps, void* stream);

/* Decode recurrent-block front in ONE launch: cadence_gemm_linear_conv1d
 * (conv_lo = E, TW = 4, packed W and A) followed, in the same workgroups, by
 * cadence_rglru_step on its output with gate = the y branch and packed-rows
 * y_out (reference modules.py:340-352 linear_y / linear_x, layers.py:478-483
 * the Conv1D step, layers.py:345-365 + :175-182 the RG-LRU gates and T == 1
 * scan step).  yx_out [M][2E] row-major receives (y, conv1d(x)) as
 * cadence_gemm_linear_conv1d writes them; conv_state and h advance in place;
 * y_out (packed rows) = bf16(h) * y.  Wgates: the decode-packed [heads][2 bw][bw]
 * gate weights of cadence_rglru_step.  Bitwise equal to the two launches.
 * Each head's 2 bw / 32 workgroups wait for one another (one agent-scope
 * counter per head, one per 128-B line): counters = >= 64 * heads zeroed
 * int32, left zeroed;
 * err (int32) is set to 1 if a wait gave up (never expected).  Accepted
 * shapes: cadence_recurrent_decode_front_plan. */
int cadence_recurrent_decode_front_plan(int64_t M, int64_t E, int64_t K, int64_t heads,
                                        int64_t bw);
int cadence_recurrent_decode_front(const void* A, const void* Wyx, const void* bias,
                                   void* yx_out, int64_t M, int64_t E, int64_t K,
                                   const void* conv_w, const void* conv_b, void* conv_state,
                                   int norm, float norm_eps, const void* Wgates,
                                   const void* bias_x, const void* bias_a,
                                   const void* softplus_a, const int32_t* segment_pos,
                                   float* h, void* y_out, int64_t heads, int64_t bw,
                                   int32_t* counters, int32_t* err, void* stream);

/* Residual GEMM that feeds an RMSNorm (the temporal-block output projection
 * and ffw_down, each followed by the next norm; modules.py:908-913):
 *   out = A . W^T + bias + resid          (as cadence_gemm_linear, act 0)
 *   norm_out = RMSNorm(out; norm_scale)    (as cadence_rmsnorm)
 * For M <= 32 the GEMM runs split-K (K = 2560: 2 splits) and one row-owned kernel finishes the
 * reduction, the residual and the norm (workspace:
 * cadence_gemm_rmsnorm_workspace_bytes); otherwise GEMM + norm kernels. */
int64_t cadence_gemm_rmsnorm_workspace_bytes(int64_t M, int64_t N, int64_t K);
int cadence_gemm_linear_rmsnorm(const void* A, int64_t lda, const void* W,
                                int64_t ldw, const void* bias,
                                const void* resid, int64_t ld_resid, void* out,
                                int64_t ldo, int64_t M, int64_t N, int64_t K,
                                const void* norm_scale, float eps,
                                void* norm_out, int64_t ld_norm,
                                void* workspace, int64_t ws_bytes,
                                void* stream);

/* Decode form of the residual GEMM above whose RMSNorm is deferred to the
 * GEMM that consumes it (M <= 32 sequences; same K split plan and workspace
 * as cadence_gemm_linear_rmsnorm):
 *   out      = A . W^T + bias + resid      (row-major, ldo)
 *   out_rows = the same values in the packed decode layout, NOT normalised
 * The K splits of each column tile are combined inside the launch by the
 * last split to arrive, in split order (the sums of the two-kernel form).
 * Consumers normalise on load (norm != 0): cadence_gemm_linear_conv1d,
 * cadence_qkv_rope_decode, cadence_gemm_gated_gelu.  counters: >= N / 16 zeroed int32, left zeroed
 * (launches that may overlap need their own).  Replaces the same reference
 * lines as cadence_gemm_linear_rmsnorm (modules.py:908-913 + the next
 * norm). */
int cadence_gemm_linear_residual_rows(const void* A, int64_t lda, const void* W,
                                      int64_t ldw, const void* bias,
                                      const void* resid, int64_t ld_resid,
                                      void* out, int64_t ldo, void* out_rows,
                                      int64_t M, int64_t N, int64_t K,
                                      void* workspace, int64_t ws_bytes,
                                      int32_t* counters, void* stream);

/* MLP up-projection + gating: out[m, f] = gelu_tanh(x.Wg[f] + bg[f]) *
 * (x.Wu[f] + bu[f]).  W is the packed [2F][K] matrix in which every 64-row
 * group g holds 32 gate rows then the 32 up rows of features
 * [32g, 32g + 32).  Replaces modules.py:754-756 (Einsum ffw_up + gelu + mul;
 * layers.py:726-729).  norm != 0 (M <= 32, packed rows, K <= 2560):
 * normalise on load ("Deferred RMSNorm" above; W carries channel_pre_norm's
 * scale). */
int cadence_gemm_gated_gelu(const void* A, int64_t lda, const void* Wpacked,
                            int64_t ldw, const void* bias_gate,
                            const void* bias_up, void* out, int64_t ldo,
                            int64_t M, int64_t F, int64_t K, void* workspace,
                            int64_t ws_bytes, int norm, float norm_eps,
                            void* stream);

/* RG-LRU gates: both BlockDiagonalLinear layers of one RG-LRU as a grouped
 * GEMM (one group per head, K = block width) with the full gate chain fused
 * in the epilogue, producing the scan inputs
 *   a_out  = reset ? 0 : exp(-8 * sigmoid(gate_a) * softplus(a_param))
 *   nx_out = x * sigmoid(gate_x) * (reset ? 1 : sqrt(1 - a^2))
 * with the bf16 rounding chain of the reference.  Wpacked is
 * [heads][2*bw][bw] (per 64-row group: 32 input-gate rows, 32 a-gate rows).
 * ldw is bw (row-major) or 0 (fragment-packed per head).
 * Replaces layers.py:345-365 (+ 132-142 BlockDiagonalLinear, + 173). */
int cadence_rglru_gates(const void* X, int64_t ldx, const void* Wpacked,
                        int64_t ldw, const void* bias_x, const void* bias_a,
                        const void* softplus_a, const int32_t* segment_pos,
                        void* a_out, void* nx_out, int64_t ldo, int64_t M,
                        int64_t heads, int64_t bw, void* workspace,
                        int64_t ws_bytes, void* stream);

/* Plan query (host only, no GPU work): 1 when cadence_rglru_gates with these
 * operands runs the block-bound streaming kernel (rglru_gates_stream_kernel:
 * bw in {64, 128, 256}, row-major weights, M > 32, 16-byte aligned X and W,
 * ldx and ldo multiples of 8), 0 when it runs the block engine's grouped GEMM
 * with the gate-chain epilogue.  Used to name the kernel a timed launch ran. */
int cadence_rglru_gates_stream_plan(const void* X, int64_t ldx, const void* Wpacked,
                                    int64_t ldw, int64_t ldo, int64_t M, int64_t bw);

/* Prefill RG-LRU with the scan fused in: cadence_rglru_gates (row-major
 * packed weights) followed by cadence_rnn_scan (no segment_pos: the resets
 * are already in a) in one launch, bitwise equal to the two:
 *   a, nx = gate chain of X (layers.py:321-365);
 *   h_t = a_t h_{t-1} + nx_t (fp32, from h0 or 0);  out = bf16(h) [* gate]
 * (layers.py:145-199; the `x * y` join of modules.py:652 when gate != NULL).
 * X, gate, out are [B * L] rows (sequence-major); h0 / h_last [B][heads*bw]
 * fp32 (either may be NULL).  Only where cadence_rglru_scan_plan says 1
 * (bw 128 / 256, enough sequences x blocks to fill the chip, aligned rows);
 * otherwise returns hipErrorInvalidValue without launching.
 * Replaces layers.py:345-375 + 145-199 in RecurrentBlock (modules.py:644-652). */
int cadence_rglru_scan(const void* X, int64_t ldx, const void* Wpacked,
                       const void* bias_x, const void* bias_a, const void* softplus_a,
                       const int32_t* segment_pos, const float* h0, const void* gate,
                       int64_t ldg, void* out, int64_t ldo, float* h_last, int64_t B,
                       int64_t L, int64_t heads, int64_t bw, void* stream);

/* Plan query (host only, no GPU work): 1 when cadence_rglru_scan accepts
 * these operands. */
int cadence_rglru_scan_plan(const void* X, int64_t ldx, const void* gate, int64_t ldg,
                            int64_t ldo, int64_t B, int64_t L, int64_t heads,
                            int64_t bw);

/* Single-token RG-LRU step (decode, T = 1): the gate GEMM + chain of
 * cadence_rglru_gates with the scan step of rnn_scan's T == 1 branch fused
 * into the epilogue (layers.py:175-182, modules.py:652):
 *   h[m, e] = a * h[m, e] + nx (fp32, in place);  y = bf16(h) [* gate]
 * h is [M][heads * bw] fp32; gate (may be NULL) is the linear_y branch. */
int cadence_rglru_step(const void* X, int64_t ldx, const void* Wpacked,
                       int64_t ldw, const void* bias_x, const void* bias_a,
                       const void* softplus_a, const int32_t* segment_pos,
                       float* h, const void* gate, int64_t ldg, void* y_out,
                       int64_t ldy, int64_t M, int64_t heads, int64_t bw,
                       void* workspace, int64_t ws_bytes, void* stream);

/* ViT residual branch (fp32 residual stream, in place):
 *   resid[m, n] += gamma[n] * (A[m,:] . W[n,:] + bias[n])   (gamma may be 0)
 * Replaces timm Block `x + ls(attn.proj(.))` / `x + ls(mlp.fc2(.))`. */
int cadence_gemm_vit_residual(const void* A, int64_t lda, const void* W,
                              int64_t ldw, const void* bias, const void* gamma,
                              float* resid, int64_t ld_resid, int64_t M,
                              int64_t N, int64_t K, void* workspace,
                              int64_t ws_bytes, void* stream);

/* Patch embedding as GEMM over im2col patches (K padded to 64):
 *   resid[b, prefix + p, n] = patches[b*P + p, :] . W[n, :] + bias[n] + pos[p, n]
 * Replaces timm PatchEmbed conv + _pos_embed (no_embed_class). */
int cadence_gemm_patch_embed(const void* patches, int64_t ldp, const void* W,
                             int64_t ldw, const void* bias, const void* pos,
                             float* resid, int64_t B, int64_t P, int64_t ntok,
                             int64_t prefix, int64_t N, int64_t K,
                             void* workspace, int64_t ws_bytes, void* stream);

/* Last-position logits with soft-cap and greedy argmax:
 *   l = bf16(x . E[v]); l = bf16(bf16(tanh(bf16(l / cap))) * cap)
 *   next[m] = argmax_v l (lowest index on ties); logits_out optional.
 * Replaces modules.py:1003-1006 + griffin.py:216-221 + the greedy
 * torch.argmax of examples/cadence_sampler.py:101-110.  `scratch` must hold
 * M * ceil(V / 64) * 8 bytes plus the split-K workspace. */
int cadence_logits_argmax(const void* X, int64_t ldx, const void* E,
                          int64_t lde, int64_t M, int64_t V, int64_t D,
                          float soft_cap, void* logits_out, int32_t* next_token,
                          void* scratch, int64_t scratch_bytes, void* stream);
int64_t cadence_logits_scratch_bytes(int64_t M, int64_t V, int64_t D);

/* The greedy decode step's tail in one launch after the logits: what
 * cadence_logits_argmax's argmax, cadence_decode_advance and
 * cadence_embed_packed do in three, for the captured decode step whose next
 * replay starts from the rows this writes.  One workgroup per row m:
 * next_token[m] = the argmax (as cadence_logits_argmax); the bookkeeping of
 * cadence_decode_advance for row m (tokens_out, positions, cur_out, done[m]);
 * then the embedding of the token written (E[t] * scale, an id outside [0,
 * vocab) reads row 0) into x_out (row-major, ldx_out) and packed_out (the
 * decode activation layout).  The last workgroup to arrive on `counter` (one
 * int32, zero before the first launch; left zero) advances *step and sets
 * done[M].  M <= 32, D % 32 == 0. */
typedef struct CadenceDecodeTail {
  int32_t* tokens_out;
  int64_t ld_out;
  int32_t* step;
  int32_t* positions;
  int32_t* cur_out;
  int32_t* done;
  int32_t eos_id, pad_id, eos_from;
  int32_t* counter;
  const void* embed;
  int64_t vocab;
  float scale;
  void* x_out;
  int64_t ldx_out;
  void* packed_out;
} CadenceDecodeTail;
int cadence_logits_argmax_tail(const void* X, int64_t ldx, const void* E, int64_t lde,
                               int64_t M, int64_t V, int64_t D, float soft_cap,
                               int32_t* next_token, void* scratch, int64_t scratch_bytes,
                               const CadenceDecodeTail* tail, void* stream);

/* All-position logits (Griffin.forward with return_logits=True,
 * griffin.py:216-221): out[m, v] = softcap(bf16(x[m] . E[v])) (cap 0 = off).
 * Uses the GEMM workspace rules of cadence_gemm_linear. */
int cadence_gemm_logits(const void* X, int64_t ldx, const void* E, int64_t lde,
                        int64_t M, int64_t V, int64_t D, float soft_cap, void* out,
                        int64_t ldo, void* workspace, int64_t ws_bytes,
                        void* stream);

/* ---- normalisation / embedding ----------------------------------------- */

/* Griffin RMSNorm, bf16 rounding at every op: layers.py:70-78. */
int cadence_rmsnorm(const void* x, int64_t ldx, const void* scale, void* out,
                    int64_t ldo, int64_t rows, int64_t width, float eps,
                    void* stream);

/* LayerNorm over an fp32 residual stream -> bf16 (timm ViT norm1/norm2,
 * eps 1e-6). */
int cadence_layernorm(const float* x, int64_t ldx, const void* weight,
                      const void* bias, void* out, int64_t ldo, int64_t rows,
                      int64_t width, float eps, void* stream);

/* Embedder.encode (modules.py:994-1001): out[map(m)] = E[tok[m]] * scale
 * (scale = bf16(sqrt(width)) or 1), row remap as in cadence_gemm_linear.
 * E is [V, D]; an id outside [0, V) reads row 0 (no fault). */
int cadence_embed(const int32_t* tokens, const void* E, void* out,
                  int64_t ldo, int64_t M, int64_t D, int64_t V, float scale,
                  int64_t row_div, int64_t row_mul, int64_t row_off,
                  void* stream);

/* The decode step's embedding (M <= 32 rows, D % 32 == 0): as cadence_embed
 * with the identity row map, and the same rows again in the decode
 * activation layout (`packed`, D * 16 * ceil(M / 16) bf16): the first
 * block's decode GEMVs apply its temporal_pre_norm on load from them, as
 * every later block does from its predecessor's output (modules.py:994-1001
 * and the block's RMSNorm, layers.py:60-78). */
int cadence_embed_packed(const int32_t* tokens, const void* E, void* out,
                         int64_t ldo, void* packed, int64_t M, int64_t D,
                         int64_t V, float scale, void* stream);

/* ---- recurrent block ----------------------------------------------------- */

/* Conv1D, prefill (cache_in == NULL) or single-token decode (L == 1,
 * cache_in = previous [B,3,E] state).  compat = 1 keeps the reference
 * document mask (layers.py:629, range(1, shift-1); App. A Q3).  Writes the
 * new [B, W-1, E] state to cache_out (may alias cache_in only for decode).
 * Replaces layers.py:457-546 (+ :592-633). */
int cadence_conv1d(const void* x, int64_t ldx, const void* w, const void* b,
                   const int32_t* segment_pos, const void* cache_in,
                   void* out, int64_t ldo, void* cache_out, int64_t B,
                   int64_t L, int64_t E, int64_t temporal_width, int compat,
                   void* stream);

/* Linear recurrence h_t = a_t * h_{t-1} + x_t (fp32 state, separate mul and
 * add as the eager reference), y_t = bf16(h_t), optionally gated:
 * out_t = bf16(y_t * gate_t) (RecurrentBlock `x * y`, modules.py:651).
 * `reset` (int32 segment positions, may be NULL) zeroes a where pos == 0.
 * h0 may be NULL (zeros).  h_last [B,E] fp32.  Replaces layers.py:145-199
 * (`rnn_scan`) and the join of modules.py:651. */
int cadence_rnn_scan(const void* x, int64_t ldx, const void* a, int64_t lda,
                     const int32_t* segment_pos, const float* h0,
                     const void* gate, int64_t ldg, void* out, int64_t ldo,
                     float* h_last, int64_t B, int64_t L, int64_t E,
                     void* workspace, int64_t ws_bytes, void* stream);

/* Workspace bytes the chunked (segmented) form of cadence_rnn_scan needs
 * for (B, L, E); 0 when the one-lane-per-sequence kernel is used.  With a
 * workspace of at least this size, batches whose B * E / 2 lanes cannot
 * fill the chip run time-chunked: per-chunk affine summaries, an in-order
 * carry over them, and an exact rescan of each chunk from its carry-in
 * (chunks 0 and 1 bit-exact; later chunks differ only through the carry's
 * rounding).  workspace may be NULL: the sequential kernel then runs. */
int64_t cadence_rnn_scan_workspace_bytes(int64_t B, int64_t L, int64_t E);

/* ---- local attention ------------------------------------------------------ */

/* Segment bookkeeping for the forward-pass mask (modules.py:130-152):
 * seg_id = cumsum(pos == 0), seg_start = first index of the row's segment. */
int cadence_segment_info(const int32_t* segment_pos, int32_t* seg_id,
                         int32_t* seg_start, int64_t B, int64_t L,
                         void* stream);

/* RoPE on the first half of each head (modules.py:53-87) for q (H heads)
 * and k (1 head) read from the fused qkv projection rows; v copied.
 * q_out [M, H*hd], k_out/v_out [M, hd]. */
int cadence_rope_qkv(const void* qkv, int64_t ldqkv, const int32_t* positions,
                     void* q_out, void* k_out, void* v_out, int64_t M,
                     int64_t H, int64_t hd, const void* table,
                     int64_t table_len, void* stream);

/* Decode (M <= 32 sequences, one token each) q|k|v projection with RoPE in
 * the epilogue (replaces cadence_gemm_linear + cadence_rope_qkv for the
 * cached attention step; reference modules.py:429-440 proj_q/k/v + apply_rope):
 * Wperm is the [(H + 2) * hd][K] matrix [proj_q; proj_k; proj_v] with, in each
 * of the H + 1 q / k heads, row 2i holding dim i and row 2i + 1 dim i + hd/4
 * for i < hd/4 (the rotated half's pairs side by side; rows hd/2.. and the
 * v head in natural order).  Outputs q [M][H*hd], k [M][hd], v [M][hd] as
 * cadence_rope_qkv writes them.  Wperm may be fragment-packed (ldw == 0), A
 * packed rows (lda == 0); K <= 2560 (one split).  norm != 0: normalise on
 * load ("Deferred RMSNorm" above; W carries temporal_pre_norm's scale). */
int cadence_qkv_rope_decode(const void* A, int64_t lda, const void* Wperm,
                            int64_t ldw, const int32_t* positions, void* q_out,
                            void* k_out, void* v_out, int64_t M, int64_t H,
                            int64_t hd, int64_t K, const void* table,
                            int64_t table_len, int norm, float norm_eps,
                            void* stream);

/* Prefill (M > 64 rows) q|k|v projection with RoPE in the GEMM epilogue
 * (replaces cadence_gemm_linear + cadence_rope_qkv of the prompt pass;
 * reference modules.py:429-440 proj_q/k/v + apply_rope, :53-87): the block
 * engine with Wperm in cadence_qkv_rope_decode's row order, each 8 staged
 * output columns (4 rotation pairs) rotated and written to q [M][H*hd],
 * k [M][hd], v [M][hd] in natural dim order, with cadence_rope_qkv's
 * products and roundings.  Row-major A and Wperm (lda, ldw >= K); hd % 64
 * == 0, K % 64 == 0.  Returns hipErrorInvalidValue for a shape whose plan is
 * not one unsplit block-engine launch (small M: split K, or the 4-wave
 * engine); the caller then runs the two-launch form. */
int cadence_qkv_rope_prefill(const void* A, int64_t lda, const void* Wperm,
                             int64_t ldw, const int32_t* positions, void* q_out,
                             void* k_out, void* v_out, int64_t M, int64_t H, int64_t hd,
                             int64_t K, const void* table, int64_t table_len,
                             void* stream);

/* sin / cos table for cadence_rope_qkv: table[p][0][i] = bf16(sin(p * f_i)),
 * table[p][1][i] = bf16(cos(p * f_i)), i < hd / 4, f_i as modules.py:73-77
 * computes it (fp32 inverse frequencies, fp32 angle).  Positions >= the
 * table length are computed in-kernel instead. */
int cadence_rope_table(void* table, int64_t positions, int64_t hd,
                       void* stream);

/* Prefill local MQA attention, flash-style (modules.py:466-480):
 * logits = bf16(q.k) * hd^-0.5, mask = same segment & causal & window,
 * fp32 online softmax, out [B*L, H*hd] bf16. */
int cadence_local_attention(const void* q, const void* k, const void* v,
                            const int32_t* seg_id, const int32_t* seg_start,
                            void* out, int64_t B, int64_t L, int64_t H,
                            int64_t hd, int64_t window, void* stream);

/* KV cache from the prompt (modules.py:260-290): roll by num_tokens and
 * right-pad to the window; num_tokens = pos[:, -1] + 1. */
int cadence_kv_cache_fill(const void* k, const void* v,
                          const int32_t* segment_pos, void* cache_k,
                          void* cache_v, int32_t* num_tokens, int64_t B,
                          int64_t L, int64_t hd, int64_t window, void* stream);

/* Single-token decode attention over the ring buffer + the new key, with the
 * slot positions of _compute_cache_mask (modules.py:155-185), then the
 * in-place cache update of _update_attention_cache (modules.py:210-218).
 * With `workspace` (>= cadence_local_attention_decode_workspace_bytes) and
 * `sems` (B zeroed int32 counters, left at zero) the window is split over 8
 * workgroups per sequence and combined in-kernel in a fixed order; with
 * either NULL one workgroup walks the whole window. */
int64_t cadence_local_attention_decode_workspace_bytes(int64_t B, int64_t hd);
int cadence_local_attention_decode(const void* q, const void* k_new,
                                   const void* v_new, void* cache_k,
                                   void* cache_v, int32_t* num_tokens,
                                   void* out, int64_t ld_out, int64_t B, int64_t H,
                                   int64_t hd, int64_t window, void* workspace,
                                   int64_t ws_bytes, int32_t* sems,
                                   void* stream);

/* ---- vision tower ---------------------------------------------------------- */

/* im2col with the per-encoder Normalize folded in: pixels [B,3,S,S] fp32 in
 * [0,1] -> patches [B*g*g, Kpad] bf16 (c, kh, kw order, zero padded). */
int cadence_im2col_normalize(const float* pixels, void* patches, int64_t ldp,
                             int64_t B, int64_t S, int64_t patch,
                             const float* mean3, const float* std3,
                             void* stream);

/* Writes the prefix tokens (cls / register) into rows [0, prefix) of every
 * image of the fp32 residual stream. */
int cadence_vit_prefix(const void* tokens, float* resid, int64_t B,
                       int64_t ntok, int64_t prefix, int64_t D, void* stream);

/* Plan query (host only): the kernel cadence_vit_attention runs for N
 * tokens of head dim hd -- 0 the LDS-resident vit_attn_kernel, 1 the
 * round-3 streaming vit_stream_attn_kernel, 2 vit_flash_attn_kernel (the
 * streaming kernel with MFMA-computed softmax sums), -1 unsupported. */
int cadence_vit_attention_kernel(int64_t N, int64_t hd);

/* Bidirectional multi-head attention (timm Attention, fused SDPA):
 * qkv [B*N, 3*H*hd] bf16 -> out [B*N, H*hd] bf16; hd in {64, 72}; qkv and
 * out 16-B aligned (returns hipErrorInvalidValue otherwise). */
int cadence_vit_attention(const void* qkv, void* out, int64_t B, int64_t N,
                          int64_t H, int64_t hd, void* stream);

/* Drops the prefix tokens and converts the fp32 stream to the bf16
 * projector input at a column offset: out[b*P + p, col_off + d] =
 * bf16(resid[b, prefix + p, d])  (dino_siglip.py:153-154 cat + mlp.py:30
 * `.to(bfloat16)`). */
int cadence_vit_features(const float* resid, void* out, int64_t ldo,
                         int64_t col_off, int64_t B, int64_t ntok,
                         int64_t prefix, int64_t D, void* stream);

/* Image preprocessing of the img_path API: torchvision Resize((S, S),
 * BICUBIC) on a PIL RGB image + ToTensor (dino_siglip.py:12-16, 88-124,
 * 148-151; both encoders' transforms share it), i.e. Pillow's
 * ImagingResample (libImaging/Resample.c) bit for bit, for a ragged batch:
 *   images  packed uint8 HWC RGB, images_bytes long; meta[b] = {byte offset,
 *           H, W, tmp offset}; max_h / max_w bound every H / W;
 *           images, coef and tmp 16-byte aligned
 *   KS      taps per coefficient row, a multiple of 4 >= 2 * ceil(2 *
 *           max(in / S, 1)) + 1 over every image side (host computes it)
 *   coef    workspace, B * 2 * S * (2 + KS) int32
 *   tmp     workspace, tmp_bytes >= sum_b H_b * S * 3 (row-pass images)
 *   out     [B, 3, S, S] fp32 in [0, 1]
 * Replaces the host PIL resize per image in VisionEncoder.forward. */
int cadence_resize_bicubic(const void* images, int64_t images_bytes,
                           const int64_t* meta, int64_t B, int64_t S,
                           int64_t KS, int64_t max_h, int64_t max_w, void* coef,
                           void* tmp, int64_t tmp_bytes, float* out,
                           void* stream);

/* ---- misc ------------------------------------------------------------------ */

/* Image splice positions (griffin.py:186-191, n_vis generalised):
 * out[b] = [0, 1, ..., n_vis-1, text_pos[b, :]]. */
int cadence_splice_positions(const int32_t* text_pos, int32_t* out,
                             int64_t B, int64_t T, int64_t n_vis,
                             void* stream);

/* Local attention of T query rows against [cache ring | T new keys] with
 * the cache-mask semantics of modules.py:155-185 (positions from
 * num_tokens, no segment ids): the multi-token cached step of
 * modules.py:206-225 (n_fill == window) and the single-token step for head
 * dims the tuned decode kernel does not cover.  Any hd % 4 == 0, hd <= 1024,
 * window + T <= 6144.  Reads the caches only (update them with
 * cadence_kv_cache_fill / cadence_kv_ring_update).  q [B*T, H*hd], k_new /
 * v_new [B*T, hd], cache_k / cache_v [B, window, hd], out [B*T, H*hd]. */
int cadence_local_attention_cached(const void* q, const void* k_new,
                                   const void* v_new, const void* cache_k,
                                   const void* cache_v,
                                   const int32_t* num_tokens, void* out,
                                   int64_t B, int64_t T, int64_t H, int64_t hd,
                                   int64_t window, void* stream);

/* Batched device-to-device copies in one launch per 32 descriptors: region
 * i is desc[i].rows rows of desc[i].row_bytes bytes, consecutive rows
 * src_stride / dst_stride bytes apart.  Sizes, strides and pointers are
 * multiples of 4 bytes (16 for the wide path).  Regions must not overlap.
 * Replaces the per-tensor copies of the decode graph's cache hand-over
 * (the host side of recurrentgemma/torch/sampler.py:209-225 keeps the
 * prefill cache and the step cache as separate tensors). */
typedef struct CadenceCopyDesc {
  const void* src;
  void* dst;
  int64_t rows, row_bytes, src_stride, dst_stride;
} CadenceCopyDesc;
int cadence_copy_batched(const CadenceCopyDesc* desc, int64_t n, void* stream);

/* Single-token ring update (modules.py:206-215): slot num_tokens[b] % window
 * <- k_new[b] / v_new[b]; num_tokens[b] += 1. */
int cadence_kv_ring_update(const void* k_new, const void* v_new, void* cache_k,
                           void* cache_v, int32_t* num_tokens, int64_t B,
                           int64_t hd, int64_t window, void* stream);

/* Greedy decode bookkeeping (the host loop of examples/cadence_sampler.py:
 * 131-151 and the done test of recurrentgemma/torch/sampler.py:217-223
 * moved on device): tokens_out[b, *step] = next_token[b], or pad_id once
 * row b has emitted eos_id; positions[b] += 1; *step += 1; cur_out[b] = the
 * token written (the next step's input; cur_out may be null).  done (may be
 * null: no EOS handling) is int32[B + 1]: done[b] latches when row b emits
 * eos_id into a column >= eos_from (1: the reference loop, which never tests
 * the token sampled from the prompt; 0: every column), done[B] = 1 when
 * every row is done.  B <= 1024. */
int cadence_decode_advance(const int32_t* next_token, int32_t* tokens_out,
                           int64_t ld_out, int32_t* step, int32_t* positions,
                           int32_t* cur_out, int32_t* done, int32_t eos_id,
                           int32_t pad_id, int32_t eos_from, int64_t B,
                           void* stream);

#ifdef __cplusplus
}  // extern "C"
#endif

#endif  // CADENCE_KERNELS_H_
