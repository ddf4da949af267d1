/* lc_clip.h — C ABI of liblcclip.so, the MI355X (gfx950) kernels for the CLIP dual-encoder
 * PEFT training step of qcNPU/LifeLong-CLIP (methods/adapter_clip.py:86-96).
 *
 * The reference has no FFI: its boundary is a torch.nn.Module (models/adapter_clip.py,
 * models/clip/model.py) whose arithmetic is ATen. Each entry point below replaces the ATen call
 * sites cited next to it; lifelong-clip_amd/lcclip binds them with ctypes behind the same
 * nn.Module surface.
 *
 * Conventions (all entry points):
 *  - plain device pointers + sizes; no allocation inside; re-entrant across streams/devices;
 *  - `stream` is a hipStream_t (the caller's current stream);
 *  - bf16 tensors are raw 16-bit bfloat16 bits; f32 tensors are IEEE float; ld* = row strides
 *    in elements; all matrices are row-major;
 *  - return 0 on success, LC_EINVAL (-1) on an argument/shape violation detected on the host
 *    (nothing is launched), LC_ELAUNCH (-2) if the launch failed. The Python shim raises
 *    RuntimeError on any nonzero return (the reference's own error behaviour is an exception
 *    propagating to main(), nohup.out:30-43).
 */
#ifndef LC_CLIP_H
#define LC_CLIP_H
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LC_OK 0
#define LC_EINVAL (-1)
#define LC_ELAUNCH (-2)

/* GEMM epilogues for lc_gemm_nt */
#define LC_EPI_BF16 0     /* out0 bf16 = alpha*acc + bias                                    */
#define LC_EPI_F32 1      /* out0 f32  = alpha*acc + bias                                    */
#define LC_EPI_RESID 2    /* out0 f32  = aux_f32 + alpha*acc + bias     (x + sublayer(x))    */
#define LC_EPI_GELU 3     /* out0 bf16 = acc + bias; out1 bf16 = QuickGELU(acc + bias)        */
#define LC_EPI_GELU_BWD 4 /* out0 bf16 = alpha*acc * QuickGELU'(aux_bf16)                    */
#define LC_EPI_BF16_F32 5 /* out0 bf16 and out1 f32 of alpha*acc + bias                     */
#define LC_EPI_GELU_D 6   /* out0 bf16 = QuickGELU'(pre); out1 bf16 = QuickGELU(pre), pre =    */
                          /* acc + bias: saves the derivative for the backward, not pre        */
#define LC_EPI_MUL 7      /* out0 bf16 = alpha*acc * aux_bf16   (dX of c_fc with saved GELU')  */
/* fp8-output epilogues (lc_gemm_nt_fp8 only): out1 = e4m3 codes + E8M0 scales (q_scale, q_rows)
 * of the bf16-rounded result, bit-identical to the bf16 epilogue followed by lc_quant_fp8 */
#define LC_EPI_GELU_D_Q8 12 /* out0 bf16 = QuickGELU'(pre); out1 fp8 = QuickGELU(pre)          */
#define LC_EPI_MUL_Q8 13    /* out1 fp8 = alpha*acc * aux_bf16 (out0 unused)                   */
/* the image tower's half residual stream (see the _x16 entry points below) */
#define LC_EPI_RESID16 14   /* out0 half = aux_half + alpha*acc + bias  (x + sublayer(x))      */

/* C[M,N] = A[M,K] . B[N,K]^T with a fused epilogue; A, B bf16, K % 64 == 0, N % 64 == 0,
 * lda / ldb (elements) multiples of 8 and below 2^22, ldo0 / ldo1 below 2^21 (the kernels address
 * a tile's rows through buffer descriptors with 32-bit byte offsets; LC_EINVAL otherwise).
 * Replaces: F.linear for QKV / out-proj (models/clip/lora.py:837, 1072; torch MHA for
 * model.py:217,230), nn.Linear c_fc/c_proj + QuickGELU + residual adds (model.py:219-222,
 * 234-235, 203-206), conv1 as a patch GEMM (model.py:709-713, 756), `@ proj` / `@
 * text_projection` (model.py:785, 954), and the dX GEMMs of their autograd backward. */
int lc_gemm_nt(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
               const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
               void* out1, long ldo1, const void* aux, long ldaux);

/* lc_gemm_nt with a caller-owned workspace for the split-K tail: when the 256x256 tiles of a
 * launch leave the last round over the CUs at most half full (e.g. N = 768 at M = 50 432: 591
 * tiles on 256 CUs), those tiles are cut along K into 2-4 slices whose f32 partial tiles meet in
 * ws and are summed (in slice order, deterministic) by the last slice before the epilogue.
 * ws: device memory, 256-B aligned, ws_bytes >= LC_SPLITK_TICKET_BYTES; its first
 * LC_SPLITK_TICKET_BYTES must be zero before the first use (the kernel leaves them zero), the
 * rest is scratch (up to 64 MiB is used). ws = NULL is plain lc_gemm_nt. Launches that share a
 * workspace must be stream-ordered. Same call sites as lc_gemm_nt. */
#define LC_SPLITK_TICKET_BYTES 16384
int lc_gemm_nt_ws(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                  const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
                  void* out1, long ldo1, const void* aux, long ldaux, void* ws, long ws_bytes);

/* Block-scaled fp8 GEMM (MX-style e4m3 operands, E8M0 scale per 32 k; fp8 MFMA
 * v_mfma_scale_f32_16x16x128_f8f6f4 at twice the bf16 rate): out = epilogue(alpha * A @ B^T + bias)
 * with A [M,K] / B [N,K] e4m3 (row strides lda / ldb in BYTES, multiples of 16) and their scales
 * sa [K/128][sa_rows][4] / sb [K/128][sb_rows][4] (sa_rows = M rounded up to 256, sb_rows >= N;
 * lc_quant_fp8 produces both). K % 128 == 0, N % 256 == 0. Epilogues LC_EPI_BF16 / F32 / RESID /
 * GELU / GELU_D / MUL as lc_gemm_nt; ws as lc_gemm_nt_ws. LC_EPI_GELU_D_Q8 / MUL_Q8 write out1 as
 * the NEXT fp8 GEMM's A operand: codes [M, ldo1 bytes] (ldo1 % 16 == 0, 16-B aligned) and scales
 * q_scale [N/128][q_rows][4] (q_rows = M rounded up to 256); q_scale is ignored otherwise.
 * Replaces: the fp16 frozen-backbone GEMMs of MaPLe (models/maple_clip/model.py:749-772, 826:
 * convert_weights to half; the QKV / c_fc / c_proj products of :316-401), run in fp8 as BASELINE
 * config 5 names. */
int lc_gemm_nt_fp8(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                   const void* sa, long sa_rows, const void* B, long ldb, const void* sb,
                   long sb_rows, const float* bias, float alpha, void* out0, long ldo0,
                   void* out1, long ldo1, const void* aux, long ldaux, void* ws, long ws_bytes,
                   void* q_scale, long q_rows);

/* Quantise src [rows, K] (bf16, or f32 when src_f32; element (r, k) at src[r*sr + k*sk], so a
 * transposed view quantises along its other axis) to e4m3 dst [rows, ldd] + E8M0 scales
 * [K/128][rows_pad][4]: per block of 32 k, scale = 2^(floor(log2 amax) - 8) clamped to
 * [2^-126, 2^126] (amax = 0 -> scale byte 0, values 0), value = RNE_e4m3(clamp(x / scale, +-448)).
 * K % 128 == 0, rows_pad % 256 == 0. */
int lc_quant_fp8(hipStream_t stream, long rows, int K, const void* src, int src_f32, long sr,
                 long sk, void* dst, long ldd, void* scales, long rows_pad);

/* Tile-shape override for lc_gemm_nt (tuning): 0 = automatic, 1 = 128x128 (4 waves),
 * 2 = 256x128 (8 waves, 3-stage LDS ring), 3 = 256x256 (8 waves, 2 stages), 4 = 128x64,
 * 5 = 256x256 ping-pong (8 waves in two staggered groups, 4-slot k-half LDS ring), 6 = same,
 * 7 = 256x256 4-wave AGPR kernel, 8 = 256x256 phase-interleaved kernel (the fp8 GEMM's, bf16),
 * 11 = 128x64 one-stage.
 * (A diagnostic build, make DIAG=1, also takes the initial value from LC_GEMM_TILE; the
 * production library reads no environment variables.) */
int lc_gemm_set_tile(int tile);

/* Stream-K schedule of the 256x256 bf16 GEMM (plain / f32 / residual epilogues) for launches
 * whose last round of tiles is ragged: one workgroup per CU, each owning an equal range of the
 * launch's (tile, k-tile) units, a tile cut between two ranges summed through the split-K
 * workspace. mode 0 = off, 1 = N = 768 with K >= 2048, 2 = every N = 768 launch, 3 = every
 * ragged launch, 4 = N = 768 as one workgroup per 256-row panel walking its 3 column tiles.
 * Process-wide; needs the launch's workspace (lc_gemm_nt_ws). */
int lc_gemm_set_streamk(int mode);

/* Diagnostic (builds with -DLC_GEMM_TRACE only): when p != NULL, the ping-pong GEMM stores
 * s_memtime stamps of its segments
 * (workgroup 0, waves 0 and 4) to p[512] (tools/gemm_trace.py). NULL disables (default). */
int lc_gemm_set_debug(unsigned long long* p);

/* C[N1,N2] += alpha * A[M,N1]^T . B[M,N2] (f32 C, atomically accumulated; split over M);
 * if colsum != NULL also colsum[N1] += colsum_scale * sum_m A[m][:] (the bias gradient).
 * A and B rows are read in 64-column blocks: lda >= N1 and ldb >= N2 rounded up to 64 (the
 * padding columns are read, their products masked) — this is how the rank-4 LoRA gradients
 * run on it with zero-padded [M,64] operands.
 * Replaces: the autograd weight- and bias-gradient reductions of adapter down_proj / up_proj
 * (models/clip/adapter.py:38-40, 59-62). */
int lc_gemm_tn(hipStream_t stream, int M, int N1, int N2, const void* A, long lda, const void* B,
               long ldb, float alpha, float* C, long ldc, float* colsum, float colsum_scale);
/* The same with a workspace (ws after its first LC_SPLITK_TICKET_BYTES, which stay untouched:
 * the launch stream's split-K workspace can be passed): in the wide x skinny case with the wide
 * side a multiple of 256 columns, 256-column panels and a two-stage reduction (partials to ws, a
 * summing launch) replace the f32 atomics. Falls back to lc_gemm_tn's path otherwise. */
int lc_gemm_tn_ws(hipStream_t stream, int M, int N1, int N2, const void* A, long lda,
                  const void* B, long ldb, float alpha, float* C, long ldc, float* colsum,
                  float colsum_scale, void* ws, long ws_bytes);

/* LayerNorm over rows of width D (64 <= D <= 1024, D % 64 == 0), fp32 statistics, eps 1e-5.
 * y is bf16 (y_f32 = 0) or f32 (y_f32 = 1); row_idx (optional) gathers input rows.
 * mean/rstd (optional, f32[rows]) are saved for the backward.
 * Replaces: LayerNorm.forward (model.py:194-200) for ln_1/ln_2/ln_pre/ln_post/ln_final. */
int lc_layernorm_fwd(hipStream_t stream, int rows, int D, const float* x, long ldx,
                     const int* row_idx, const float* gamma, const float* beta, void* y,
                     int y_f32, long ldy, float* mean, float* rstd);

/* The same writing the normalised rows as the A operand of an fp8 GEMM (lc_gemm_nt_fp8): e4m3
 * codes q [rows, ldq bytes] (ldq % 16 == 0, 16-B aligned) + E8M0 scales q_scale
 * [D/128][q_rows][4] (q_rows = rows rounded up to 256), bit-identical to the bf16 output followed
 * by lc_quant_fp8; y (bf16, optional: NULL skips it) as lc_layernorm_fwd. D % 256 == 0.
 * Replaces: the ln_1 / ln_2 -> fp16 GEMM input cast of MaPLe's frozen tower (BASELINE config 5
 * fp8; models/maple_clip/model.py:316-401). */
int lc_layernorm_fwd_fp8(hipStream_t stream, int rows, int D, const float* x, long ldx,
                         const int* row_idx, const float* gamma, const float* beta, void* y,
                         long ldy, float* mean, float* rstd, void* q, long ldq, void* q_scale,
                         long q_rows);

/* dx[row_idx[r]] = dres[row_idx[r]] + LayerNorm_backward(dy[r]) (gamma/beta frozen), written
 * as f32 (dx) and optionally bf16 (dx_bf16). dy is bf16 or f32 (dy_f32). dres may be NULL.
 * Replaces: autograd of F.layer_norm (model.py:199). */
int lc_layernorm_bwd(hipStream_t stream, int rows, int D, const void* dy, int dy_f32, long ldy,
                     const float* x, long ldx, const float* mean, const float* rstd,
                     const float* gamma, const float* dres, float* dx, void* dx_bf16, long ldo,
                     const int* row_idx);

/* lc_layernorm_bwd (no row gather) whose result is also written as the next fp8 GEMM's A
 * operand: e4m3 codes q [rows, ldq bytes] + E8M0 scales (q_scale, q_rows as in
 * lc_layernorm_fwd_fp8), bit-identical to dx_bf16 followed by lc_quant_fp8. Used by the fp8
 * towers for the block output gradient the next (lower) block's c_proj input-gradient GEMM
 * quantises. Replaces: autograd of F.layer_norm (model.py:199) under MaPLe's fp8 mode. */
int lc_layernorm_bwd_fp8(hipStream_t stream, int rows, int D, const void* dy, int dy_f32,
                         long ldy, const float* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, float* dx, void* dx_bf16,
                         long ldo, const int* row_idx, void* q, long ldq, void* q_scale,
                         long q_rows);

/* The image tower's residual stream in IEEE half (x16). The reference's residual stream is
 * fp16 under autocast: its LayerNorm returns the input's dtype (model.py:194-200), conv1's
 * output is fp16 (model.py:756-766) and every `x = x + ...` stays fp16 (model.py:439-442).
 * The _x16 entry points take and return x as half [rows, ldx] (ldx % 4 == 0, 8-B aligned;
 * 16-B for lc_adapter_ln_fwd_x16 with ldx % 8 == 0); the LayerNorm statistics are f32 and a
 * LayerNorm of a stored x reads the rounded value. Everything else as the f32 forms. */
int lc_layernorm_fwd_x16(hipStream_t stream, int rows, int D, const void* x, long ldx,
                         const int* row_idx, const float* gamma, const float* beta, void* y,
                         int y_f32, long ldy, float* mean, float* rstd);
int lc_layernorm_bwd_x16(hipStream_t stream, int rows, int D, const void* dy, int dy_f32,
                         long ldy, const void* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, float* dx, void* dx_bf16,
                         long ldo, const int* row_idx);
int lc_vit_embed_ln_x16(hipStream_t stream, int n_img, int n_patch, int D, const float* patch,
                        const float* cls, const float* pos, const float* ln_pre_w,
                        const float* ln_pre_b, void* x0, const float* ln1_w, const float* ln1_b,
                        void* y, float* mean1, float* rstd1);
/* lc_layernorm_bwd_x16 with the residual gradient in IEEE half as well: dres and dx half
 * [rows, ldo] (ldo % 4 == 0, 8-B aligned), the gradient carrying a power-of-two scale set
 * upstream (lc_grad_pow2_normalize: the reference's GradScaler, methods/adapter_clip.py:93);
 * dx_bf16 is the bf16 copy of the stored half value, or NULL (the adapter tower: its
 * consumers read the half gradient directly, lc_adapter_bwd_g16 / _wgrad_ws_unscaled_g16). */
int lc_layernorm_bwd_g16(hipStream_t stream, int rows, int D, const void* dy, int dy_f32,
                         long ldy, const void* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const void* dres, void* dx, void* dx_bf16,
                         long ldo, const int* row_idx);
/* lc_adapter_wgrad_ws whose results are divided by *gscale (device f32: the power-of-two scale
 * gout / dpre carry; exact), so the scaled backward's weight gradients land unscaled. */
int lc_adapter_wgrad_ws_unscaled(hipStream_t stream, int M, int D, const void* gout, long ldg,
                                 const void* h, const void* z, long ldz, const void* dpre,
                                 float scale, float* dWu, float* dbu, float* dWd, float* dbd,
                                 void* ws, long ws_bytes, const float* gscale);
/* The two adapter backward launches reading the half residual gradient itself: gout IEEE half
 * [M, ldg] (16-B aligned), every other 16-bit operand bf16, so lc_layernorm_bwd_g16 writes no
 * bf16 copy (77 MB per LayerNorm backward at ViT-B/16 B = 256).
 * lc_adapter_bwd_g16: dpre = mask(scale * gout Wu) / keep on the f16 MFMA (Wu cast to half, the
 * reference's fp16 autocast product), dz = gout + dpre Wd with the exact half gout; D = 512 or
 * 768, any M, dz may be NULL (dpre only).
 * lc_adapter_wgrad_ws_unscaled_g16: each gout value enters as its bf16 rounding (the value the
 * copy held): the results equal lc_adapter_wgrad_ws_unscaled on the copy bit for bit.
 * Replaces: adapter.py:59-72 autograd, as lc_adapter_bwd and lc_adapter_wgrad. */
int lc_adapter_bwd_g16(hipStream_t stream, int M, int D, const void* gout, long ldg, const void* h,
                       const void* WuT, const void* WdT, float scale, float keep, void* dpre,
                       void* dz, long ldz);
int lc_adapter_wgrad_ws_unscaled_g16(hipStream_t stream, int M, int D, const void* gout, long ldg,
                                     const void* h, const void* z, long ldz, const void* dpre,
                                     float scale, float* dWu, float* dbu, float* dWd, float* dbd,
                                     void* ws, long ws_bytes, const float* gscale);
int lc_adapter_ln_fwd_x16(hipStream_t stream, int M, int D, const void* z, long ldz,
                          const void* Wd, const float* bd, const void* Wu, const float* bu,
                          float scale, float keep, unsigned long long seed,
                          const unsigned long long* seed_dev, const void* resid, void* xout,
                          long ldx, void* hout, const float* gamma, const float* beta, void* y,
                          long ldy, float* mean, float* rstd);
/* lc_layernorm_fwd_fp8 / lc_layernorm_bwd_fp8 over a half x: the prompt towers (MVP, MaPLe),
 * whose prompt rows the reference casts to the stream's dtype (mvp_clip.py:256-257,
 * maple.py:243), with their QKV / c_fc / c_proj GEMMs on the fp8 MFMA. */
int lc_layernorm_fwd_fp8_x16(hipStream_t stream, int rows, int D, const void* x, long ldx,
                             const int* row_idx, const float* gamma, const float* beta, void* y,
                             long ldy, float* mean, float* rstd, void* q, long ldq, void* q_scale,
                             long q_rows);
int lc_layernorm_bwd_fp8_x16(hipStream_t stream, int rows, int D, const void* dy, int dy_f32,
                             long ldy, const void* x, long ldx, const float* mean,
                             const float* rstd, const float* gamma, const float* dres, float* dx,
                             void* dx_bf16, long ldo, const int* row_idx, void* q, long ldq,
                             void* q_scale, long q_rows);

/* im2col of NCHW f32 images into bf16 patches [n*g*g, 3*P*P] in conv1's (c, kh, kw) order.
 * Replaces: the input side of conv1 (model.py:756-758). */
int lc_patchify(hipStream_t stream, int n_img, int res, int patch, const float* img, void* out);

/* x[n][0] = cls + pos[0]; x[n][1+p] = patch[n*np+p] + pos[1+p]   (model.py:759-764). */
int lc_vit_assemble(hipStream_t stream, int n_img, int n_patch, int D, const float* patch,
                    const float* cls, const float* pos, float* x);

/* lc_vit_assemble, then x0 = ln_pre(x) (f32 [n*(np+1), D], the residual stream) and the first
 * block's y = bf16(ln_1(x0)) with its mean1 / rstd1 [rows], in one pass over the rows (one
 * launch instead of three; the assembled rows and x0 are not re-read). D in {512, 768, 1024};
 * x0 and y row-major with stride D. Replaces: model.py:759-766 (+ the first block's ln_1,
 * model.py:194-200, 233). */
int lc_vit_embed_ln(hipStream_t stream, int n_img, int n_patch, int D, const float* patch,
                    const float* cls, const float* pos, const float* ln_pre_w,
                    const float* ln_pre_b, float* x0, const float* ln1_w, const float* ln1_b,
                    void* y, float* mean1, float* rstd1);

/* x[c][t] = emb[tokens[c][t]] + pos[t]   (model.py:943-946). */
int lc_text_embed(hipStream_t stream, int C, int L, int D, const int64_t* tokens,
                  const float* emb, const float* pos, float* x);

/* row_idx[c] = c*L + argmax_t tokens[c][t]   (EOT pooling, model.py:953-954). */
int lc_eot_rows(hipStream_t stream, int C, int L, const int64_t* tokens, int* row_idx);

/* Multi-head attention core, d_head = 64, L <= 256. qkv [n_seq*L, ldq] holds
 * q|k|v at columns 0, H*64, 2*H*64; O [n_seq*L, ldo]; lse f32 [n_seq*H, L] (log2 domain).
 * ldq, ldo, lddq % 8 == 0; O and dqkv 16-B aligned (each row's 64 head columns are written as
 * 16-B pieces).
 * causal = 1 applies the text tower's upper-triangular -inf mask.
 * Replaces: lora.py:950-1071 (q scaling, bmm, mask, softmax, dropout p=0, bmm) and the SDPA
 * path of torch nn.MultiheadAttention (model.py:217,230), forward and backward. */
int lc_attn_fwd(hipStream_t stream, int n_seq, int L, int H, const void* qkv, long ldq, void* O,
                long ldo, float* lse, int causal);
int lc_attn_bwd(hipStream_t stream, int n_seq, int L, int H, const void* qkv, long ldq,
                const void* O, const void* dO, long ldo, const float* lse, void* dqkv, long lddq,
                int causal);
/* Testing / A-B: the kernel form lc_attn_bwd uses (process-wide): 0 automatic (default),
 * 1 fused single pass (dS^T parked in LDS), 2 key-major + query-major kernel pair, 3 two-phase
 * (dQ, then dK / dV, in one workgroup with 59 KB of LDS: two workgroups per CU; L <= 224).
 * All forms compute the same dq|dk|dv up to f32 summation order. -1 for other values. */
int lc_attn_bwd_set_form(int form);
/* The backward with dq|dk|dv written as the A operand of the fp8 QKV input-gradient GEMM
 * (lc_gemm_nt_fp8): e4m3 codes dqkv [n_seq*L, lddq BYTES] (lddq % 16 == 0, 16-B aligned) + E8M0
 * scales q_scale [3*H*64/128][q_rows][4] (q_rows = n_seq*L rounded up to 256), bit-identical to
 * lc_attn_bwd followed by lc_quant_fp8. L <= 224 (the fused single-pass kernel).
 * Replaces: the same backward feeding MaPLe's fp16 in-proj input gradient
 * (models/maple_clip/model.py:316-401, BASELINE config 5 in fp8). */
int lc_attn_bwd_fp8(hipStream_t stream, int n_seq, int L, int H, const void* qkv, long ldq,
                    const void* O, const void* dO, long ldo, const float* lse, void* dqkv, long lddq,
                    void* q_scale, long q_rows, int causal);

/* GPU train transform of the online step: the torchvision Compose of methods/_trainer.py:212-242
 * as applied to the batch at methods/adapter_clip.py:81 — optional uint8 round trip of the
 * autoaug branch (quantize: (x*255).type(uint8).float()/255, _trainer.py:216/229; the
 * AutoAugment op itself is not applied), Resize((R,R)) bilinear align_corners=False,
 * RandomCrop(R, padding=pad) at offset (crop_i, crop_j) of the zero-padded image,
 * RandomHorizontalFlip when flip != 0 (torchvision draws one decision per batch call),
 * Normalize(mean, std). x: f32 NCHW [n, C, Hin, Win] (ToTensor values in [0,1]); C <= 4;
 * mean_host / std_host: HOST arrays of C floats. layout 0: out f32 NCHW [n, C, R, R];
 * layout 1: out bf16 patch rows [n*(R/patch)^2, C*patch*patch] in conv1's (c, ky, kx) order
 * (the lc_patchify layout, i.e. the transform fused into conv1's im2col). */
int lc_train_transform(hipStream_t stream, int n, int C, int Hin, int Win, const float* x, int R,
                       int pad, int crop_i, int crop_j, int flip, const float* mean_host,
                       const float* std_host, int quantize, int layout, int patch, void* out);

/* AutoAugment (torchvision 0.16 AutoAugment, the 'autoaug' branch of methods/_trainer.py:215-229)
 * on the uint8-quantised batch: x f32 [n, C, H, W] in [0, 1] -> out f32 = augmented uint8 / 255.
 * n_ops (0..2) ops of one drawn sub-policy, shared by the batch (torchvision draws once per call):
 * codes[i] in 0..9 (invert, brightness, color, contrast, sharpness blends, posterize, solarize,
 * autocontrast, equalize, nearest affine) with 6 f32 parameters each in params (the host computes
 * blend ratios, masks, thresholds and the rescaled inverse affine grid matrix, lcclip/transforms.py).
 * C*H*W <= 12288 (CIFAR 32x32, TinyImageNet 64x64; larger: lc_autoaugment_ws). Replaces: transforms.AutoAugment(policy)
 * (methods/_trainer.py:217-228). */
int lc_autoaugment(hipStream_t stream, int n, int C, int H, int W, const float* x, float* out,
                   int n_ops, const int* codes, const float* params);

/* lc_autoaugment for any image size: images with C*H*W > 12288 (ImageNet / ImageNet-R at
 * 224x224, the policy methods/_trainer.py:222-224 selects) keep their working image in `out`
 * and a scratch image in the caller's workspace ws (ws_bytes >= n*C*H*W*4); smaller ones ignore
 * ws and run the LDS form. Bit-identical results to lc_autoaugment where both apply. */
int lc_autoaugment_ws(hipStream_t stream, int n, int C, int H, int W, const float* x, float* out,
                      int n_ops, const int* codes, const float* params, void* ws, long ws_bytes);

/* f32 -> bf16 cast of n elements (weight staging). */
int lc_cast_bf16(hipStream_t stream, long n, const float* src, void* dst);

/* out = bf16(W + scaling * B @ A) [N,K] and optionally outT = its transpose [K,N]; r = 0 casts W.
 * Replaces: the LoRA residual of lora.py:838-839 (in-proj, A [r,D] shared by q/k/v, B [3D,r])
 * and lora.py:1073-1074 / lora.Linear.forward :162-171 (out-proj), merged once per step. */
int lc_merge_weight(hipStream_t stream, int N, int K, int r, const float* W, const float* A,
                    const float* B, float scaling, void* out, void* outT);

/* Batched plain casts: out[i] = bf16(W[i]) ([N[i], K[i]]) and, when outT[i] != NULL, the
 * transposed copy [K[i], N[i]], for n <= LC_CAST_MAX matrices in one launch (host arrays of
 * device pointers). Used for the adapter weights after every optimizer step.
 * Replaces: the per-call fp32 -> half weight casts autocast performs inside F.linear for the
 * adapter's down/up projections (adapter.py:11-72 under the autocast at
 * methods/adapter_clip.py:87). */
#define LC_CAST_MAX 64
int lc_cast_weights_bf16(hipStream_t stream, int n, const float* const* W, const int* N,
                         const int* K, void* const* out, void* const* outT);

/* Batched merges: lc_merge_weight for n <= LC_CAST_MAX items in one launch (host arrays; A[i] /
 * B[i] NULL with r[i] == 0 for a plain cast). The LoRA towers re-merge every block's in-proj and
 * out-proj weights and re-stage the bf16 A / B^T gradient operands after each optimizer step:
 * 6 items per block, 72 launches of 3-9 us on the critical path before.
 * Replaces: the per-step LoRA residual merges of lora.py:838-839, 1073-1074 (as lc_merge_weight). */
int lc_merge_weights_bf16(hipStream_t stream, int n, const float* const* W, const float* const* A,
                          const float* const* B, const int* r, const float* scaling, const int* N,
                          const int* K, void* const* out, void* const* outT);

/* dB[N,r] += scaling * dY^T (X A^T);  dA[r,K] += scaling * (dY B)^T X   (r == 4).
 * Replaces: autograd of the two F.linear LoRA products (lora.py:838-839, 1073-1074). */
int lc_lora_grad(hipStream_t stream, int M, int N, int K, int r, const void* dY, long ldy,
                 const void* X, long ldx, const float* A, const float* B, float scaling,
                 float* dA, float* dB);

/* The same gradients in ONE pass over X [M,K] and dY [M,N] (bf16), MFMA form: apad = A as bf16
 * [>= 16 rows, K] and btpad = B^T as bf16 [>= 16 rows, N], rows >= r zero (the engine stages
 * both per step); dA [r,K] / dB [N,r] f32 accumulated (+=). 32-row blocks, one persistent
 * workgroup per CU, partial sums in ws after its first LC_SPLITK_TICKET_BYTES (needs
 * walkers x (16 N + 16 K) x 4 B, walkers = min(CUs, ceil(M/32))) summed by a second launch in
 * walker order (deterministic). Shapes: (K, N) in {(768, 2304), (768, 768), (512, 1536),
 * (512, 512)} (ViT-B/16 image / text QKV and out-proj sites); r <= 4 (the reference's lora_r).
 * Replaces: autograd of the two F.linear LoRA products (lora.py:838-839, 1073-1074). */
int lc_lora_grad_ws(hipStream_t stream, int M, int N, int K, int r, const void* dY, long ldy,
                    const void* X, long ldx, const void* apad, long lda, const void* btpad,
                    long ldbt, float scaling, float* dA, float* dB, void* ws, long ws_bytes);
/* lc_lora_grad_ws whose sums are divided by *gscale (device f32: the power-of-two scale the
 * image tower's half residual gradient carries, lc_layernorm_bwd_g16; exact) before the
 * scaling and the accumulation. bf16 storage build only. */
int lc_lora_grad_ws_unscaled(hipStream_t stream, int M, int N, int K, int r, const void* dY,
                             long ldy, const void* X, long ldx, const void* apad, long lda,
                             const void* btpad, long ldbt, float scaling, float* dA, float* dB,
                             void* ws, long ws_bytes, const float* gscale);

/* xout = resid + z + scale*(drop(relu(z Wd^T + bd)) Wu^T + bu); h (bf16 [M,64]) is saved.
 * keep = 1 - dropout p; the counter-based dropout mask is selected by
 * seed + (*seed_dev) * const when seed_dev != NULL (a device-side RNG epoch, so a captured HIP
 * graph draws fresh masks on every replay), else by seed alone.
 * Replaces: Adapter.forward (adapter.py:53-72) + the block residual (model.py:440-441). */
int lc_adapter_fwd(hipStream_t stream, int M, int D, const void* z, long ldz, const void* Wd,
                   const float* bd, const void* Wu, const float* bu, float scale, float keep,
                   unsigned long long seed, const unsigned long long* seed_dev,
                   const float* resid, float* xout, long ldx, void* h);

/* lc_adapter_fwd followed by the LayerNorm of its output, in one launch: xout and h as
 * lc_adapter_fwd, then y = bf16(LayerNorm(xout) * gamma + beta) (fp32 statistics, eps 1e-5)
 * with mean / rstd [M] saved — the ln_2 of the same block or the ln_1 of the next
 * (model.py:194-200). z, resid and xout cross HBM once (separately: two GEMM launches and a
 * LayerNorm launch re-reading xout). D in {512, 768}; xout and y 16-B aligned, ldy % 8 == 0
 * (both are written as whole-row 16-B pieces). Replaces: Adapter.forward
 * (adapter.py:53-72) + the residual (model.py:440-441) + the next ln_x (model.py:194-200). */
int lc_adapter_ln_fwd(hipStream_t stream, int M, int D, const void* z, long ldz, const void* Wd,
                      const float* bd, const void* Wu, const float* bu, float scale, float keep,
                      unsigned long long seed, const unsigned long long* seed_dev,
                      const float* resid, float* xout, long ldx, void* hout,
                      const float* gamma, const float* beta, void* y, long ldy, float* mean,
                      float* rstd);

/* Row-local adapter backward: dpre (bf16 [M,64]) and dz = gout + dpre Wd (bf16; dz = NULL
 * computes dpre only).
 * WuT = Wu^T [64,D], WdT = Wd^T [D,64] (bf16). Weight/bias gradients: lc_gemm_tn.
 * Replaces: autograd of adapter.py:59-72. */
int lc_adapter_bwd(hipStream_t stream, int M, int D, const void* gout, long ldg, const void* h,
                   const void* WuT, const void* WdT, float scale, float keep, void* dpre,
                   void* dz, long ldz);

/* Testing: the form lc_adapter_bwd uses at D = 512 / 768 — 1 (default) the one-pass row-block
 * kernel, 0 the two skinny GEMMs (EPI_AD_MASK + EPI_AD_ADD) it must equal bit for bit. */
int lc_adapter_bwd_set_form(int fused);

/* Adapter weight and bias gradients of one application, accumulated (f32, one launch):
 *   dWu [D,64] += scale * gout^T h      dbu [D]  += scale * sum_m gout[m]   (up_proj)
 *   dWd [64,D] += dpre^T z              dbd [64] += sum_m dpre[m]           (down_proj)
 * gout, z bf16 [M,D] (row strides ldg, ldz); h, dpre bf16 [M,64] contiguous. dbu / dbd may be
 * NULL. Replaces: the autograd weight/bias reductions of adapter.py:38-40 applied at :59-62. */
int lc_adapter_wgrad(hipStream_t stream, int M, int D, const void* gout, long ldg, const void* h,
                     const void* z, long ldz, const void* dpre, float scale, float* dWu,
                     float* dbu, float* dWd, float* dbd);
/* The same with a two-stage reduction: every walker's partial goes to ws (after its first
 * LC_SPLITK_TICKET_BYTES, left untouched: the split-K workspace of the launch stream can be
 * passed) and a second launch sums them into the outputs, instead of f32 atomics. Falls back to
 * the atomics when ws is NULL or smaller than LC_SPLITK_TICKET_BYTES + 2 x 256 x 8384 x 4 B. */
int lc_adapter_wgrad_ws(hipStream_t stream, int M, int D, const void* gout, long ldg,
                        const void* h, const void* z, long ldz, const void* dpre, float scale,
                        float* dWu, float* dbu, float* dWd, float* dbd, void* ws, long ws_bytes);

/* *flag |= any(!isfinite(g))  (GradScaler's inf check, _trainer.py:163, adapter_clip.py:94). */
int lc_check_finite(hipStream_t stream, long n, const float* g, int* flag);

/* torch.optim.AdamW step over a flat fp32 buffer; skipped when *skip != 0. The bias-correction
 * step is `step`, or *step_dev when step_dev != NULL (device-side counter, graph replay).
 * Replaces: optimizer.step() (utils/train_utils.py:27-28, methods/adapter_clip.py:94). */
int lc_adamw(hipStream_t stream, long n, float* p, const float* g, float* m, float* v, float lr,
             float b1, float b2, float eps, float wd, int step, const int* skip,
             const long long* step_dev);

/* ctr[i] += delta for i < n (n <= 64): the per-step device counters (RNG epoch, AdamW step) a
 * captured step graph advances on every replay. */
int lc_counter_add(hipStream_t stream, int n, long long* ctr, long long delta);

/* *ctr += 1 unless *skip != 0 (skip may be NULL): the AdamW step counter, which advances only
 * for applied updates — GradScaler.step skips optimizer.step() on inf/NaN gradients, so torch's
 * state['step'] stays (methods/adapter_clip.py:94-95). Feeds lc_adamw's step_dev. */
int lc_adam_step_advance(hipStream_t stream, long long* ctr, const int* skip);

/* out[r] = f[r] / ||f[r]||, norms[r] = ||f[r]||   (model.py:966-969, adapter_clip.py:78). */
int lc_l2norm_rows(hipStream_t stream, int R, int E, const float* f, long ldf, float* out,
                   float* norms);

/* Head forward+backward: logits = exp(*logit_scale) img_n txt_n^T, probs = softmax(logits),
 * *loss += mean_b CE(probs_b, labels_b), dlogits = d loss / d logits. *loss must be zeroed.
 * A label outside [0, C) makes *loss and that row of dlogits NaN (so lc_check_finite skips
 * the update) — torch's CrossEntropyLoss raises on it.
 * Replaces: model.py:972-973, models/adapter_clip.py:99, methods/adapter_clip.py:88-89. */
int lc_clip_head(hipStream_t stream, int B, int C, int E, const float* img_n, const float* txt_n,
                 const float* logit_scale, const int64_t* labels, float* probs, float* dlogits,
                 float* loss);

/* dF[r] = (dn - n (n.dn)) / norm[r], dn = exp(*logit_scale) sum_c dlog(r,c) other_n[c] + dn_ext[r];
 * dlog(r,c) = dlogits[r*sr + c*sc]; dn_ext (grad arriving at the normalised features) may be
 * NULL. Backward of the normalisation + logit GEMM (model.py:966-973). */
int lc_head_feat_grad(hipStream_t stream, int R, int Co, int E, const float* dlogits, long sr,
                      long sc, const float* other_n, const float* self_n, const float* norms,
                      const float* logit_scale, const float* dn_ext, float* dF);

/* logits = exp(*logit_scale) img_n txt_n^T [B,C]; probs = softmax(logits) when probs != NULL.
 * Replaces: model.py:972-973 and models/adapter_clip.py:99 (module path). */
int lc_head_logits(hipStream_t stream, int B, int C, int E, const float* img_n, const float* txt_n,
                   const float* logit_scale, float* logits, float* probs);

/* dlogits = probs * (dprobs - rowsum(probs * dprobs))   (softmax backward). */
int lc_softmax_bwd_rows(hipStream_t stream, int B, int C, const float* probs, const float* dprobs,
                        float* dlogits);

/* x [n] f32 *= s, s = 2^(target_exp - floor(log2 max|x|)) computed on the device and written to
 * scale[0] (1 when max|x| is 0 or not finite): the loss scaling of the IEEE-half text tower's
 * backward, per call (torch.cuda.amp.GradScaler's role, methods/adapter_clip.py:93). */
int lc_grad_pow2_normalize(hipStream_t stream, long n, float* x, float* scale, int target_exp);

/* y[i] += x[i] / scale[0] (n elements, f32): the scaled gradients back to their true size. */
int lc_add_unscaled(hipStream_t stream, long n, float* y, const float* x, const float* scale);

/* ---- streams -------------------------------------------------------------------------------
 * The step's side streams (text tower, PEFT weight gradients) run beside the image chain's
 * GEMMs. The reference has no counterpart: nn.DataParallel runs one replica per GPU on torch's
 * default stream (methods/_trainer.py:167-168). A side stream confined to a subset of the CUs
 * keeps its workgroups off the CUs the main stream's GEMM tiles refill. */
/* n_cu[0] = the device's compute-unit count. */
int lc_device_cu_count(int device, int* n_cu);
/* A HIP stream on `device` whose kernels run only on CUs first, first + stride, ...,
 * first + (count - 1) * stride (hipExtStreamCreateWithCUMask); the caller owns it
 * (lc_stream_destroy). */
int lc_stream_create_cumask(int device, int first, int count, int stride, void** stream);
int lc_stream_destroy(void* stream);

/* ---- IEEE-half storage: the text tower ------------------------------------------------------
 * Each _f16 entry point is its namesake above with every 16-bit operand, output and weight
 * image in IEEE half (binary16, round-to-nearest-even) instead of bf16: same arguments, same
 * shape rules and error codes, f32 operands unchanged; the MFMA is v_mfma_f32_16x16x32_f16.
 * The reference computes both towers under fp16 autocast (methods/adapter_clip.py:87); the
 * text tower keeps that precision here (its bf16 rounding carries half of the logits' distance
 * from fp32 and most of the C = 100 gradients'), the image tower keeps bf16
 * (BASELINE config 2) unless AdapterCLIP(image_precision="fp16") asks for the reference's
 * arithmetic there too. Built from the same kernel sources with -DLC_F16. */
int lc_gemm_nt_f16(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                   const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
                   void* out1, long ldo1, const void* aux, long ldaux);
int lc_gemm_nt_ws_f16(hipStream_t stream, int epi, int M, int N, int K, const void* A, long lda,
                      const void* B, long ldb, const float* bias, float alpha, void* out0, long ldo0,
                      void* out1, long ldo1, const void* aux, long ldaux, void* ws, long ws_bytes);
int lc_gemm_tn_f16(hipStream_t stream, int M, int N1, int N2, const void* A, long lda, const void* B,
                   long ldb, float alpha, float* C, long ldc, float* colsum, float colsum_scale);
int lc_gemm_tn_ws_f16(hipStream_t stream, int M, int N1, int N2, const void* A, long lda,
                      const void* B, long ldb, float alpha, float* C, long ldc, float* colsum,
                      float colsum_scale, void* ws, long ws_bytes);
int lc_layernorm_fwd_f16(hipStream_t stream, int rows, int D, const float* x, long ldx,
                         const int* row_idx, const float* gamma, const float* beta, void* y,
                         int y_f32, long ldy, float* mean, float* rstd);
int lc_layernorm_bwd_f16(hipStream_t stream, int rows, int D, const void* dy, int dy_f32, long ldy,
                         const float* x, long ldx, const float* mean, const float* rstd,
                         const float* gamma, const float* dres, float* dx, void* dx_bf16, long ldo,
                         const int* row_idx);
int lc_attn_fwd_f16(hipStream_t stream, int n_seq, int L, int H, const void* qkv, long ldq, void* O,
                    long ldo, float* lse, int causal);
int lc_attn_bwd_f16(hipStream_t stream, int n_seq, int L, int H, const void* qkv, long ldq,
                    const void* O, const void* dO, long ldo, const float* lse, void* dqkv, long lddq,
                    int causal);
int lc_attn_bwd_set_form_f16(int form);
int lc_cast_bf16_f16(hipStream_t stream, long n, const float* src, void* dst);
int lc_merge_weight_f16(hipStream_t stream, int N, int K, int r, const float* W, const float* A,
                        const float* B, float scaling, void* out, void* outT);
int lc_cast_weights_bf16_f16(hipStream_t stream, int n, const float* const* W, const int* N,
                             const int* K, void* const* out, void* const* outT);
int lc_merge_weights_bf16_f16(hipStream_t stream, int n, const float* const* W, const float* const* A,
                              const float* const* B, const int* r, const float* scaling, const int* N,
                              const int* K, void* const* out, void* const* outT);
int lc_lora_grad_f16(hipStream_t stream, int M, int N, int K, int r, const void* dY, long ldy,
                     const void* X, long ldx, const float* A, const float* B, float scaling,
                     float* dA, float* dB);
int lc_lora_grad_ws_f16(hipStream_t stream, int M, int N, int K, int r, const void* dY, long ldy,
                        const void* X, long ldx, const void* apad, long lda, const void* btpad,
                        long ldbt, float scaling, float* dA, float* dB, void* ws, long ws_bytes);
int lc_adapter_fwd_f16(hipStream_t stream, int M, int D, const void* z, long ldz, const void* Wd,
                       const float* bd, const void* Wu, const float* bu, float scale, float keep,
                       unsigned long long seed, const unsigned long long* seed_dev,
                       const float* resid, float* xout, long ldx, void* h);
int lc_adapter_ln_fwd_f16(hipStream_t stream, int M, int D, const void* z, long ldz, const void* Wd,
                          const float* bd, const void* Wu, const float* bu, float scale, float keep,
                          unsigned long long seed, const unsigned long long* seed_dev,
                          const float* resid, float* xout, long ldx, void* hout,
                          const float* gamma, const float* beta, void* y, long ldy, float* mean,
                          float* rstd);
int lc_adapter_bwd_f16(hipStream_t stream, int M, int D, const void* gout, long ldg, const void* h,
                       const void* WuT, const void* WdT, float scale, float keep, void* dpre,
                       void* dz, long ldz);
int lc_adapter_wgrad_f16(hipStream_t stream, int M, int D, const void* gout, long ldg, const void* h,
                         const void* z, long ldz, const void* dpre, float scale, float* dWu,
                         float* dbu, float* dWd, float* dbd);
int lc_adapter_wgrad_ws_f16(hipStream_t stream, int M, int D, const void* gout, long ldg,
                            const void* h, const void* z, long ldz, const void* dpre, float scale,
                            float* dWu, float* dbu, float* dWd, float* dbd, void* ws, long ws_bytes);
/* The image tower at the reference's own arithmetic (AdapterCLIP(image_precision="fp16"):
 * conv1's im2col rows and the first ln_1 output in IEEE half, the residual stream f32). */
int lc_patchify_f16(hipStream_t stream, int n_img, int res, int patch, const float* img, void* out);
int lc_vit_embed_ln_f16(hipStream_t stream, int n_img, int n_patch, int D, const float* patch,
                        const float* cls, const float* pos, const float* ln_pre_w,
                        const float* ln_pre_b, float* x0, const float* ln1_w, const float* ln1_b,
                        void* y, float* mean1, float* rstd1);

#ifdef __cplusplus
}
#endif
#endif /* LC_CLIP_H */
