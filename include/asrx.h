/*
 * asrx — C-ABI of the MI355X (gfx950) Speech-Transformer attention path.
 *
 * The reference (shockless/asr-transformer) has no FFI: every hot-path op is an ATen call made from the
 * Python modules in modules/Transformer/{layers,model}.py.  Each entry point below replaces the ATen
 * call sequence cited next to it; the drop-in nn.Modules in asr-transformer_amd/asrx bind these symbols
 * through ctypes (INTEGRATION.md shows the binding).
 *
 * Conventions (all entry points):
 *   - plain device pointers, element counts/strides in ELEMENTS (not bytes), int64 sizes;
 *   - `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream); every call is asynchronous
 *     on that stream; the library never allocates, frees or synchronises (graph-capturable);
 *   - return 0 on success, a negative ASRX_ERR_* code on bad arguments or launch failure;
 *   - dtype codes: ASRX_BF16 (bfloat16 storage) or ASRX_F32.
 */
#ifndef ASRX_H
#define ASRX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ASRX_OK 0
#define ASRX_ERR_ARG (-1)
#define ASRX_ERR_LAUNCH (-2)
#define ASRX_ERR_UNSUPPORTED (-3)

#define ASRX_BF16 0
#define ASRX_F32 1
#define ASRX_BITS 2   /* gate operand only: 1 bit per element, uint32 words (ld in words; see mask_out) */

/* Library version / build identification (3: dq_acc holds one slab per key block, asrx_attn_dq_acc_elems;
 * asrx_adam_spans takes bounds that are not multiples of 4). */
int asrx_version(void);

/* sizeof of the descriptor structs as this library was compiled (binding check: a ctypes / cgo mirror of a
 * struct must have the same size): out[0] = asrx_gemm_desc, out[1] = asrx_attn_desc, out[2] =
 * asrx_gemm_group_dev, out[3] = asrx_rowsum_group, out[4] = asrx_adam_desc.  Returns the number of entries written
 * (<= n). */
int asrx_struct_sizes(int64_t* out, int32_t n);

/* ---------------------------------------------------------------------------------------------------
 * GEMM with fused epilogue:   C[z][m][n] = epi( alpha * sum_k A(z,m,k) * B(z,n,k) )
 *   A(m,k) = a_trans ? A[k*lda + m] : A[m*lda + k]
 *   B(n,k) = b_trans ? B[k*ldb + n] : B[n*ldb + k]          (b_trans=0 is the nn.Linear weight layout)
 *   batch index z in [0, batch): element offsets (z / batch_inner)*s?_outer + (z % batch_inner)*s?_inner
 *   epi order: +bias[n] -> +rowadd[(m % rowadd_mod)*ld_rowadd + n] -> relu -> dropout(p, seed, idx =
 *              (z*M + m)*N + n) -> *gate (keep where gate[m][n] > 0) -> +resid[m][n] -> +beta*C_old -> store
 * Replaces: nn.Linear (layers.py:10-12,36,48,51; model.py:32,102) = aten::addmm/linear, the per-head
 * q@k^T and attn@v aten::bmm (layers.py:20,27), and the conv2 implicit GEMM (model.py:168-171).
 * Split-K (splitk > 1, batch == 1) needs workspace of splitk*M*N floats (reduced in fixed split order).
 * ------------------------------------------------------------------------------------------------- */
typedef struct asrx_gemm_desc {
  int32_t m, n, k;
  int32_t in_dtype;             /* dtype of A and B */
  const void* a; int64_t lda; int32_t a_trans;
  const void* b; int64_t ldb; int32_t b_trans;
  void* c; int64_t ldc; int32_t c_dtype;
  int32_t batch, batch_inner;
  int64_t sa_outer, sa_inner, sb_outer, sb_inner, sc_outer, sc_inner;
  float alpha, beta;
  const float* bias;
  const float* rowadd; int64_t ld_rowadd; int32_t rowadd_mod;
  int32_t relu;
  float dropout_p; uint64_t seed;
  const void* gate; int64_t ld_gate; int32_t gate_dtype;
  const void* resid; int64_t ld_resid; int32_t resid_dtype;
  int32_t splitk; float* workspace; int64_t workspace_elems;
  int32_t tile;                 /* 0 = auto, 64 or 128 = forced square tile (bf16 path) */
  /* rowsum_a[m] += sum_k A(m,k)  (a_trans = 1 only): the bias gradient of a weight-gradient GEMM
   * dW = dY^T X is the row sum of its A operand dY^T — fused into the staging loads, no extra HBM pass.
   * With splitk > 1 the per-split partials use rowsum_ws[splitk*M]. */
  float* rowsum_a; float* rowsum_ws;
  /* mask_out (optional; bf16 C with relu only): the bits C[m][n] > 0 as stored — the ReLU/dropout mask of an
   * FFN hidden layer, read back by its data gradient as a gate_dtype = ASRX_BITS gate (1 bit instead of 2 bytes
   * per element).  Layout (also that of ASRX_BITS gates): uint32 word [m][n / 32] (row stride ld_mask words),
   * column c = n % 32 at bit 8*((c & 15) >> 2) + 4*(c >> 4) + (c & 3), i.e. byte q holds columns 4q..4q+3 and
   * 16+4q..16+4q+3.  Requires N % 32 == 0, ldc % 8 == 0, 16-B aligned C and the fast fused epilogue; else
   * ASRX_ERR_UNSUPPORTED. */
  uint32_t* mask_out; int64_t ld_mask;
  /* kernel family (tests / A-B; 0 = auto): 1 = 256x128 LDS-DMA ring (p3), 3 = register-staged tiles, 4 = 64x64
   * LDS-DMA ring, 5 = 128x64 LDS-DMA ring, 6 = 256x256 LDS-DMA ring (p4), 8 = warp-specialised 256x128 tiles
   * (ws: 4 MFMA waves + 4 LDS-DMA loader waves; A k-contiguous, N % 128 == 0), 10 = ws on 64x128 tiles (the
   * 4096-row decoder GEMMs) — honoured where the family's preconditions hold, else auto (codes 9 and 11, round 4's
   * persistent ws variants, were removed in version 3 and plan as auto).  Every family is a hand-written kernel of
   * this library. */
  int32_t kernel;
} asrx_gemm_desc;

int asrx_gemm(const asrx_gemm_desc* d, void* stream);

/* Grouped GEMM: `count` independent problems C_i = epi(alpha * op(A_i) op(B_i)^T) in ONE launch (no split-K),
 * the group table in DEVICE memory: entries of 64 B; group i's output tiles are numbered consecutively from
 * tile_start; tile_group[t] (device) = the group of tile t.  Layout flags, dtypes, alpha/beta come from
 * `common` (its pointers/shapes are ignored).  Supported: bf16 in, a_trans = b_trans = 1 (weight gradients
 * dW = dY^T X), 16-byte aligned operand rows (the table is not inspected on the host).
 * Replaces: the per-layer weight-gradient aten::mm + bias-gradient sum of autograd's nn.Linear backward
 * (layers.py:10-12,36,48,51; model.py:32) — issued together once the backward has produced every dY. */
typedef struct asrx_gemm_group_dev {
  const void* a; const void* b; void* c; float* rowsum_a;
  int32_t lda, ldb, ldc, m, n, k, tile_start, reserved;
} asrx_gemm_group_dev;

/* Launch with an explicit workgroup -> tile map: block_tile[b] (device, `blocks` entries, 0xFFFF = idle) names
 * the tile workgroup b computes.  Workgroup b runs on XCD b % 8, so a host that lays the tiles of one group on
 * one XCD at the same time lets them share that XCD's L2 (the operand panels of dW = dY^T X are re-read by
 * every tile of the group).  common->tile selects the tile: 3 = the p3 LDS-DMA ring, 256x128 tiles (m x n;
 * fp32 C with 16-byte aligned rows, every group's n % 4 == 0, alpha 1, beta 0 or 1), 4 = the p4 ring, 256x256
 * tiles (same conditions), 5 = the warp-specialised ws kernel, 256x128 tiles (4 MFMA waves + 4 LDS-DMA loader
 * waves, 3-stage ring; same conditions; with common->workspace set and common->workspace_elems >= 16 it is read
 * as int32 counters, ZERO on entry — [0, 8) per-XCD queues, [16, 16 + P) one per 256-row panel of the groups that
 * carry a rowsum_a (group entry `reserved` = its first panel's index, panels numbered over those groups) — and
 * common->rowsum_ws as [tiles][256] fp32 scratch: the launch runs min(blocks, 256) persistent workgroups that take
 * the slots x, x + 8, x + 16, ... of block_tile from per-XCD queues (x = b % 8; blocks % 8 == 0; an empty queue
 * takes the others' last slots), and each panel's column tiles share its row sums (the last to finish adds them in
 * column order); the counters are left non-zero: zero them before the next launch), 128 = register-staged
 * 128x128 tiles (any alignment-checked table; common->relu carries its "every C row 16-byte aligned" flag).
 * Replaces the weight/bias-gradient mm + sum of autograd for every nn.Linear (layers.py:10-12,36,48,51). */
int asrx_gemm_grouped_xcd(const asrx_gemm_desc* common, const asrx_gemm_group_dev* groups,
                          const uint16_t* tile_group, const uint16_t* block_tile, int32_t count, int32_t tiles,
                          int32_t blocks, void* stream);

/* AdamW state for asrx_gemm_grouped_xcd_adam: flat fp32 parameter / moment buffers (and the optional bf16 shadow)
 * laid out like the gradient buffer whose base is g_base — the update of gradient element g_base[i] goes to
 * p[i], m[i], v[i], p_bf16[i].  Hyper-parameters as asrx_adam (hyp: device {lr, bias_corr1, bias_corr2} or null). */
typedef struct asrx_adam_desc {
  float* p; float* m; float* v; void* p_bf16; const float* g_base; const float* hyp;
  float lr, beta1, beta2, eps, weight_decay, bias_corr1, bias_corr2, grad_scale;
  int32_t decoupled, reserved;
} asrx_adam_desc;

/* asrx_gemm_grouped_xcd (tile 5, the persistent queue launch: fp32 C, beta 0, workspace counters and rowsum_ws
 * slabs) with the optimizer step fused into the epilogue: each dW element and each group's bias gradient (rowsum_a)
 * is stored and the AdamW update of its parameter applied at once, the parameter / moment / shadow bytes moving
 * while the other tiles compute (single-GPU training: the gradients need no exchange first).  Replaces the
 * optimizer.step() (train.py:35) of every nn.Linear parameter together with its gradient mm + sum. */
int asrx_gemm_grouped_xcd_adam(const asrx_gemm_desc* common, const asrx_gemm_group_dev* groups,
                               const uint16_t* tile_group, const uint16_t* block_tile, int32_t count, int32_t tiles,
                               int32_t blocks, const asrx_adam_desc* adam, void* stream);

/* Name of the kernel instantiation asrx_gemm would launch for d (as rocprofv3 lists it, without the
 * namespace/argument list), e.g. "gemm_bf16_p3_kernel<false, false, 1>".  Host-only: no launch, no GPU
 * needed.  Used by bench.py to time exactly the kernel the roofline names. */
int asrx_gemm_kernel_name(const asrx_gemm_desc* d, char* buf, int32_t len);

/* Diagnostics only (tools/, never the product path): process-wide GEMM debug flags, overriding the ASRX_GEMM_DBG
 * environment variable — 1 = skip the epilogue stores, 4 = issue each LDS-DMA stage in one block, 8 = skip the
 * operand loads (compute on stale LDS); 0 = normal.  Results are garbage while any flag is set. */
int asrx_gemm_set_debug(int32_t flags);

/* Process-wide kernel-variant switches (value 0 = back to the default; there is no environment fallback since
 * round 5).  key ASRX_TUNE_SOFTMAX_U: rows per lane group of the short-row softmax kernels (1, 2, 4; default 1);
 * key ASRX_TUNE_LN_RW: rows per wave of the LayerNorm forward (1, 2, 4; default 2).  Every variant computes the same
 * values; the switch exists so tests and tools can run each one in one process. */
#define ASRX_TUNE_SOFTMAX_U 1
#define ASRX_TUNE_LN_RW 2
#define ASRX_TUNE_LN_PF 3    /* rows in flight per wave of the d = 512 LayerNorm kernels (1, 2, 4; 8 = the general kernels) */
#define ASRX_TUNE_LN_BPC 4   /* blocks per CU of the d = 512 LayerNorm forward (1..16; 0 = default 4) */
int asrx_set_tuning(int32_t key, int32_t value);

/* ---------------------------------------------------------------------------------------------------
 * Fused multi-head attention (bf16 in/out, fp32 softmax): per (batch b, head h)
 *   S = scale * Q K^T ; masked -> -inf ; P = nan_to_num(softmax(S)) ; O = dropout(P) V
 * Tensors are token-major: row r of batch b of X starts at X + b*x_bstride + r*x_rstride; head h's dh
 * columns start at +h*dh.  lse[(b*heads+h)*lq + q] receives the log2-domain log-sum-exp (+inf for a
 * fully-masked row, whose output is 0 exactly as layers.py:25 nan_to_num gives).
 * mask_mode: 0 none (encoder self / cross, model.py:21,71);
 *            1 structured: causal (if causal) OR key invalid (kvalid[b*valid_bstride+key]==0) OR query
 *              invalid (qvalid[...]==0) — the decoder mask of model.py:108-115 without materialising it;
 *            2 dense bytes: masked where mask[b*mask_sb + q*mask_sq + key*mask_sk] != 0 (layers.py:22-23).
 * Replaces MHAHead.forward's bmm/mul/masked_fill/softmax/nan_to_num/dropout/bmm (layers.py:20-27).
 * Supported dh: 32, 64.
 * ------------------------------------------------------------------------------------------------- */
typedef struct asrx_attn_desc {
  int32_t batch, heads, lq, lk, dh;
  const void* q; int64_t q_rstride, q_bstride;
  const void* k; int64_t k_rstride, k_bstride;
  const void* v; int64_t v_rstride, v_bstride;
  void* o; int64_t o_rstride, o_bstride;
  float* lse;
  float scale;
  int32_t mask_mode, causal;
  const uint8_t* kvalid; const uint8_t* qvalid; int64_t valid_bstride;
  const uint8_t* mask; int64_t mask_sb, mask_sq, mask_sk;
  float dropout_p; uint64_t seed;
  /* backward only */
  const void* dout; int64_t do_rstride, do_bstride;
  void* dq; int64_t dq_rstride, dq_bstride;
  void* dk; int64_t dk_rstride, dk_bstride;
  void* dv; int64_t dv_rstride, dv_bstride;
  float* delta;                 /* [batch*heads*lq] workspace */
  float* dq_acc;                /* optional fp32 workspace of asrx_attn_dq_acc_elems() floats (version >= 3:
                                 * ceil(lk/128)*batch*lq*heads*dh): dQ partials, one [batch*lq*heads*dh] slab per key
                                 * block of the kernel (required for lk > 256; version 2 and earlier took ONE slab, a
                                 * caller sized by that rule overflows it; the tiled fallback accumulates into the
                                 * first slab) */
  /* optional dropout keep-bit workspace (dh = 64, dropout_p > 0, any lk): key-major words
   * [batch*heads][ceil(lq/32)][lk] (bit i = query 32c+i) followed by query-major words
   * [batch*heads][lq][qmaj_stride(lk)] (bit j = key 32c+j), where qmaj_stride(lk) = ceil(lk/32) for lk <= 256 and
   * ceil(lk/32) rounded up to a multiple of 4 for lk > 256 (the streamed kernels move 4 words per query and
   * 128-key chunk).  Total size: batch*heads*(ceil(lq/32)*lk + lq*qmaj_stride(lk)) 32-bit words — the value
   * asrx_attn_dropmask_words() returns; size the buffer from it.  Generated by the forward (or
   * asrx_attn_dropgen) and read by the backward instead of re-hashing.  The bits equal the counter-based RNG's
   * decisions, so results do not depend on it; without it the forward uses the tiled kernel. */
  uint32_t* dropmask;
  int32_t dropmask_ready;       /* nonzero: the forward finds the bits already generated (asrx_attn_dropgen) */
  /* optional (training): bf16 buffer with o's strides; the forward writes the rounding residual O - bf16(O)
   * there and the backward forms delta = rowsum(dO * (O + residual)), i.e. sum_key P dP to fp32 accuracy.
   * (With the d_model^-1/2 scale the softmax rows are flat and dS = P (dP - delta) is a small difference: the
   * bf16 rounding of O alone perturbs dQ by delta's error times the mean key.) */
  void* o_lo;
} asrx_attn_desc;

int asrx_attention_fwd(const asrx_attn_desc* d, void* stream);
/* Number of 32-bit words of the dropmask workspace for these shapes (see asrx_attn_desc.dropmask); -1 on bad
 * arguments.  Host-only arithmetic, no device access. */
int64_t asrx_attn_dropmask_words(int32_t batch, int32_t heads, int32_t lq, int32_t lk);
/* Number of fp32 elements of the dq_acc workspace asrx_attention_bwd needs for these shapes (0: none needed, lk <=
 * 128; -1 on bad arguments).  Host-only arithmetic.  Size dq_acc from it (the rule changed in version 3). */
int64_t asrx_attn_dq_acc_elems(int32_t batch, int32_t heads, int32_t lq, int32_t lk, int32_t dh);
/* Fill d->dropmask with the dropout keep bits of (seed, dropout_p, shapes) — both layouts (see dropmask).  Only
 * the shape/dropout fields of d are read; independent of the Q/K/V data, so it can run ahead on another stream. */
int asrx_attn_dropgen(const asrx_attn_desc* d, void* stream);
/* asrx_layernorm_fwd (x fp32 [rows][512], y bf16) and asrx_attn_dropgen(d) in ONE launch (their block types share
 * the CUs: the VALU-bound hashing runs in the HBM-bound LayerNorm's memory waits).  Replaces the pre-attention
 * nn.LayerNorm (model.py:20,66) and the keep-bit draw of the attention dropout (layers.py:26). */
int asrx_layernorm_fwd_attn_dropgen(const float* x, void* y, const float* gamma, const float* beta, float* mean,
                                    float* rstd, int64_t rows, int32_t d_model, float eps, const asrx_attn_desc* d,
                                    void* stream);
int asrx_attention_bwd(const asrx_attn_desc* d, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Row softmax over materialised scores (the unfused path; HBM-roofline kernel of BASELINE.md §3):
 *   rows = nbh*lq rows of length lk (row stride ld); row r -> (bh = r / lq, q = r % lq, b = bh / heads)
 *   p = nan_to_num(softmax(scale * s  masked -> -inf)); if pd != NULL also pd = dropout(p)
 * Replaces layers.py:20 (scale), :22-23 masked_fill, :25 softmax+nan_to_num, :26 dropout.
 * bwd: ds = p * (dpd*keep/(1-p_drop) - sum_k p*dpd*keep/(1-p_drop)) * scale
 * Outputs (p, pd, ds) get zeros in the padding columns [lk, ld) of every row but the last: whole 16-B stores, no
 * partially written HBM sectors.  Inputs' padding is ignored.
 * ------------------------------------------------------------------------------------------------- */
int asrx_softmax_fwd(int32_t dtype, const void* s, void* p, void* pd, int64_t nbh, int32_t heads, int32_t lq,
                     int32_t lk, int64_t ld, float scale, int32_t mask_mode, int32_t causal,
                     const uint8_t* kvalid, const uint8_t* qvalid, int64_t valid_bstride, const uint8_t* mask,
                     int64_t mask_sb, int64_t mask_sq, int64_t mask_sk, float dropout_p, uint64_t seed,
                     void* stream);
int asrx_softmax_bwd(int32_t dtype, const void* p, const void* dpd, void* ds, int64_t nbh, int32_t lq, int32_t lk,
                     int64_t ld, float scale, float dropout_p, uint64_t seed, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * LayerNorm over the last dim d (nn.LayerNorm, eps, affine: model.py:14,16,33,59,61,63,101).
 * fwd: y = (x - mean) * rstd * gamma + beta; saves mean/rstd (fp32, one per row).
 * bwd: dx = rstd*(g - mean(g) - xhat*mean(g*xhat)), g = dy*gamma;  dx_out = dx + dres (dres nullable)
 *      if dx_drop != NULL also dx_drop = (drop_dtype)(dx_out * keep/(1-p))  (upstream sublayer's dropout bwd)
 *      per-block partial dgamma/dbeta go to part[nblocks][2][d]; finish with asrx_reduce_rows.
 * ------------------------------------------------------------------------------------------------- */
int asrx_layernorm_fwd(int32_t x_dtype, const void* x, int32_t y_dtype, void* y, const float* gamma,
                       const float* beta, float* mean, float* rstd, int64_t rows, int32_t d, float eps,
                       void* stream);
int asrx_layernorm_bwd(int32_t x_dtype, const void* x, int32_t dy_dtype, const void* dy, const float* gamma,
                       const float* mean, const float* rstd, const float* dres, float* dx_out, void* dx_drop,
                       int32_t drop_dtype, float dropout_p, uint64_t seed, float* part, int32_t nblocks,
                       int64_t rows, int32_t d, void* stream);

/* out[c] (+)= sum_r in[r*ld + c] for r < rows (fp32 or bf16 in, fp32 out). Deterministic two-level sum.
 * Used for bias gradients (column sums of dY) and to finish LayerNorm/conv partials. */
int asrx_reduce_rows(int32_t dtype, const void* in, int64_t rows, int32_t cols, int64_t ld, float* out,
                     int32_t accumulate, float* part, int32_t nblocks, void* stream);

/* Grouped version for many fp32 [rows][cols] matrices in ONE launch (count <= 64): out_g[c] (+)= sum_r in_g[r][c],
 * rows summed in a fixed order (deterministic).  Used for the LayerNorm dgamma|dbeta partials of a whole backward
 * pass, deferred like the weight gradients. */
typedef struct asrx_rowsum_group {
  const float* in; int64_t rows; int32_t cols; float* out; int32_t accumulate;
} asrx_rowsum_group;

int asrx_reduce_rows_grouped(const asrx_rowsum_group* groups, int32_t count, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Conv2d front-end (model.py:168-171): conv(1->64,3x3,s2)+ReLU -> conv(64->64,3x3,s2)+ReLU, no padding.
 * conv1_fwd: x (B,1,F,T) fp32 -> y1 channels-last (B,F1,T1,64) in y_dtype (bf16 or fp32); y1_mask (optional,
 *            (B,F1,T1,8) bytes): bit c of byte q = y1[..][8q + c] > 0 as stored (the ReLU gate of the backward)
 * im2col_conv2: y1 -> cols [(b,t2,f2)][(kh,kw,c)] (B*T2*F2, 576), same dtype: conv2 = GEMM(cols, W2p^T)
 * col2im_conv2: dcols -> dy1 (B,F1,T1,64) fp32, gated by y1 > 0 (ReLU backward)
 * conv1_bwd_w: dW1[c][kh*3+kw] += sum dy1*x, db1[c] += sum dy1 (partials in part[nblocks][64*10])
 * ------------------------------------------------------------------------------------------------- */
int asrx_conv1_fwd(const float* x, int32_t B, int32_t F, int32_t T, const float* w, const float* b, void* y1,
                   int32_t y_dtype, uint8_t* y1_mask, void* stream);
/* conv2 (Conv2d(64,64,3,s2) + bias + ReLU, model.py:170-171) as an implicit GEMM over the channels-last conv1
 * output y1 (B, F1, T1, 64) bf16, no im2col image: out[(b*T2 + t2)*F2 + f2][64] bf16 — the encoder input rows.
 * w2: [64][576] bf16, columns (kh, kw, c); bias fp32 [64].  y1 must be < 2 GiB (32-bit DMA offsets). */
int asrx_conv2_fwd(const void* y1, const void* w2, const float* bias, void* out, int32_t B, int32_t F1, int32_t T1,
                   void* stream);
/* conv2 weight/bias gradient (+=, fp32) without an im2col image: dw[64][576] += dy2^T im2col(y1), db[64] +=
 * colsum(dy2); dy2 [B*T2*F2][64] bf16, y1 (B, F1, T1, 64) bf16.  ws: >= splitk*64*576 floats, rws: splitk*64
 * floats (when db).  model.py:170 Conv2d backward. */
int asrx_conv2_wgrad(const void* dy2, const void* y1, int32_t B, int32_t F1, int32_t T1, float* dw, float* db,
                     float* ws, int64_t ws_elems, float* rws, int32_t splitk, void* stream);
/* conv1 weight/bias gradient (+=) straight from the conv2 output gradient: dy1 = relu'(y1) * conv2^T(dy2) is
 * formed on the fly, neither the column gradient nor dy1 is stored (model.py:168-171 backward).  dy2
 * [B*T2*F2][64] bf16 (ReLU-gated), w2 [64][576] bf16, y1_mask = conv1_fwd's sign bits, x (B,1,F,T) fp32; part:
 * [nblocks + 128][640] workspace, nblocks >= 2 persistent workgroups (about 2/3 take the even-f1 rows).
 * T1 <= 1024 and 48 KiB + T1*8 B + 12*T B of LDS <= 80 KiB. */
int asrx_conv_bwd_implicit(const void* dy2, const void* w2, const uint8_t* y1_mask, const float* x, int32_t B, int32_t F,
                           int32_t T, float* part, int32_t nblocks, float* dw, float* db, void* stream);
int asrx_im2col_conv2(int32_t dtype, const void* y1, int32_t B, int32_t F1, int32_t T1, void* cols, void* stream);
int asrx_col2im_conv2(int32_t dcols_dtype, const void* dcols, int32_t y1_dtype, const void* y1, int32_t B,
                      int32_t F1, int32_t T1, float* dy1, void* stream);
int asrx_conv1_bwd_w(const float* x, const float* dy1, int32_t B, int32_t F, int32_t T, float* part,
                     int32_t nblocks, float* dw, float* db, void* stream);

/* Fused conv1 backward (dW1 += sum dy1 * x-taps, db1 += sum dy1) straight from the conv2 column gradient:
 * dy1 = relu'(y1) * col2im(dcols) is formed on the fly and never stored (replaces col2im + conv1_bwd_w on the
 * training path; model.py:168-169).  nblocks = ceil(B * F1 * 8 / 4) (8 waves per conv1 output row), part:
 * [nblocks + 128][640] workspace (per-block partials, then the finish's first-pass rows). */
int asrx_conv1_bwd_fused(int32_t dcols_dtype, const void* dcols, int32_t y1_dtype, const void* y1, const float* x,
                         int32_t B, int32_t F, int32_t T, float* part, int32_t nblocks, float* dw, float* db,
                         void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Decoder embedding (model.py:94-96,117): out[t] = dropout(E[tok[t]] + pe[t % L]) (fp32 residual stream);
 * bwd: dE[v] += sum over tokens == v (v != pad_id) of dropout_bwd(dout)   (padding_idx row gets none).
 * ------------------------------------------------------------------------------------------------- */
int asrx_embed_fwd(const int64_t* tok, int64_t ntok, int32_t L, const float* table, int32_t d, const float* pe,
                   float dropout_p, uint64_t seed, float* out, void* stream);
int asrx_embed_bwd(const int64_t* tok, int64_t ntok, int32_t L, const float* dout, int32_t d, int32_t vocab,
                   int32_t pad_id, float dropout_p, uint64_t seed, float* dtable, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Cross-entropy over V classes (train.py:32, caller-supplied CE): logits fp32 rows (stride ld);
 * loss = mean over rows with target != ignore_index of (lse - logit[target]);
 * dlogits (bf16, stride ld, padded columns zeroed) = grad_scale*(softmax - onehot)/count; argmax (nullable).
 * ws: >= rows + 2 floats.
 * ------------------------------------------------------------------------------------------------- */
int asrx_cross_entropy(const float* logits, int64_t rows, int32_t V, int64_t ld, const int64_t* target,
                       int64_t ignore_index, float grad_scale, float* loss, void* dlogits, int64_t* argmax,
                       float* ws, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * Elementwise utilities.
 * ------------------------------------------------------------------------------------------------- */
int asrx_cast(int32_t src_dtype, const void* src, int32_t dst_dtype, void* dst, int64_t n, void* stream);
/* out[i] (dtype_out) = op(a[i], b[i]) over n contiguous elements (any of a, b, out may alias; ASRX_F32 / ASRX_BF16):
 *   ASRX_EW_RELU_GRAD  b[i] > 0 ? a[i] : 0        ReLU backward gated by its output b (the standalone FrontEnd's
 *                                                   conv2 ReLU, model.py:170, torch.where in round 2)
 *   ASRX_EW_DROPOUT    keep(seed, i) ? a[i] / (1 - p) : 0   dropout backward with the element mask of the GEMM
 *                                                   dropout epilogues (layers.py:40, the standalone MHA's output)
 *   ASRX_EW_ADD        a[i] + b[i]                  gradient accumulation (the standalone MHA's K/V input, split
 *                                                   LayerNorm gradients) */
#define ASRX_EW_RELU_GRAD 0
#define ASRX_EW_DROPOUT 1
#define ASRX_EW_ADD 2
int asrx_ewise(int32_t op, int32_t dtype_a, const void* a, int32_t dtype_b, const void* b, int32_t dtype_out,
               void* out, int64_t n, float p, uint64_t seed, void* stream);

/* Power spectrogram of a batch of waveforms (the featuriser of modules/dataset.py:34-55:
 * torchaudio.transforms.Spectrogram(n_fft, center=False) -> |STFT|^power):
 *   audio  fp32 [batch][samples] (row stride batch_stride), frames = (samples - n_fft) / hop + 1
 *   basis  fp32 [2 nbins][n_fft]: rows 2n / 2n+1 = window[k] * cos / -sin(2 pi n k / n_fft) (the caller's window,
 *          zero-padded to n_fft as torch.stft does; see asrx.features)
 *   out    fp32 [batch][nbins][frames] = scale * (re^2 + im^2)^(power/2), power 1 or 2
 *   ws     fp32 workspace of >= batch * frames * 2 nbins elements (the DFT GEMM's output)
 * One fp32 MFMA GEMM (frames as overlapping rows of the waveform, lda = hop) plus a square/transpose pass. */
int asrx_spectrogram(const float* audio, int64_t batch, int64_t samples, int64_t batch_stride, const float* basis,
                     int32_t n_fft, int32_t hop, int32_t nbins, int32_t power, float scale, float* ws,
                     int64_t ws_elems, float* out, void* stream);

/* Greedy decode step (Decoder.evaluate, model.py:144 `prob.argmax(dim=-1)[:, -1]`): for each of `rows` logit rows
 * (fp32, row stride ld, V used columns) the first index of the maximum, stored as int64 at tok[r * tok_stride] and,
 * if cur != NULL, at cur[r] (the next step's embedding input). */
int asrx_greedy_argmax(const float* logits, int64_t rows, int32_t V, int64_t ld, int64_t* tok, int64_t tok_stride,
                       int64_t* cur, void* stream);

/* Data-parallel gradient exchange on a bf16 wire (asrx.dist.GradAllReduce, wire="bf16"; the reference trains on one
 * device, train.py:16-35, so this is the build's own DDP step): in = the W peers' bf16 copies of one chunk of c
 * elements, [world][chunk]; out[i] = bf16(sum over w of in[w][i]) with the sum in fp32 and one final rounding. */
int asrx_sum_chunks_bf16(const void* in, int32_t world, int64_t chunk, void* out, void* stream);
/* Fused Adam/AdamW over flat fp32 buffers; optionally refreshes the bf16 shadow copy of the params.
 * Replaces optimizer.step() (train.py:35).  hyp (optional, device): {lr, bias_corr1, bias_corr2} read at run
 * time instead of the scalar arguments, so a captured step (HIP graph) takes the current step's values. */
int asrx_adam(float* p, const float* g, float* m, float* v, void* p_bf16, int64_t n, float lr, float beta1,
              float beta2, float eps, float weight_decay, float bias_corr1, float bias_corr2, float grad_scale,
              int32_t decoupled, const float* hyp, void* stream);
/* AdamW (as asrx_adam) over the element ranges [spans[2i], spans[2i+1]) of the flat buffers, one workgroup per
 * range (device int64 table, nspans pairs): the parameters a fused weight-gradient launch
 * (asrx_gemm_grouped_xcd_adam) did not update.  Bounds that are multiples of 4 take the 16-B path only; since
 * version 3 any other bound is handled too (head / tail elements one at a time; version 2 skipped them). */
int asrx_adam_spans(float* p, const float* g, float* m, float* v, void* p_bf16, const int64_t* spans, int32_t nspans,
                    float lr, float beta1, float beta2, float eps, float weight_decay, float bias_corr1,
                    float bias_corr2, float grad_scale, int32_t decoupled, const float* hyp, void* stream);
/* Zero the spans [spans[2i], spans[2i+1]) (element offsets, device int64 table of nspans pairs) of an fp32 buffer
 * (16-B aligned base), one workgroup per span.  The training step zeroes the accumulating gradient regions with it
 * (optimizer.zero_grad, train.py:27, for everything a weight-gradient GEMM does not overwrite). */
int asrx_zero_spans(float* base, const int64_t* spans, int32_t nspans, void* stream);

/* torch.nn.utils.clip_grad_norm_(parameters, max_norm) (new/train.py:31, round 5): spans = device int64 table
 * [count][2] of {address of an fp32 gradient tensor, numel}; the total 2-norm over all of them, then every element
 * times min(max_norm / (norm + 1e-6), 1) (always applied, as torch does).  Deterministic: part = device workspace of
 * nparts floats (1..4096; one workgroup each, a fixed share of every tensor), out = device float[2] {norm, coef}.
 * Two launches, no host synchronisation. */
int asrx_clip_grad_norm(const int64_t* spans, int32_t count, float max_norm, float* part, int32_t nparts, float* out,
                        void* stream);
/* new/train.py:122-128 remove_after_eos on the device: for each sample i, pred[i][t] = eos_token for t >= eoses[i]
 * (pred int64 [batch][pred_len]) and logits[i][t][:] = the one-hot row of index eoses[i] for t >= eoses[i] (fp32
 * [batch][logit_len][vocab]; the reference writes the EOS *position* as the hot index, kept here). */
int asrx_remove_after_eos(int64_t* pred, int32_t batch, int32_t pred_len, float* logits, int32_t logit_len,
                          int32_t vocab, const int64_t* eoses, int64_t eos_token, void* stream);
/* Teacher-forced step inputs (train.py:22-24,32 without the index_put quirk; model.py:108-115): from the (B, L+1)
 * token rows `text` (targets) and `inp` (decoder input; = text unless shifted), row strides in elements, and the
 * float pad mask (B, L+1): dec_in[b*L+t] = inp[b][t], tgt[b*L+t] = text[b][t+1], valid[b*L+t] = mask[b][t] >= 1. */
int asrx_step_tokens(const int64_t* text, int64_t ld_text, const int64_t* inp, int64_t ld_inp, const float* mask,
                     int64_t ld_mask, int32_t B, int32_t L, int64_t* dec_in, int64_t* tgt, uint8_t* valid,
                     void* stream);
/* Row-wise fp32 ops of the post-LN model family (modules/Transformer/new/model.py, asrx.new): op 0 (ROWSCALE)
 * out[r][c] = a[r][c] * b[r] (the non_pad_mask products, new/model.py:25,28,83-89); op 1 (ROWADD) out[r][c] =
 * a[r][c] + b[r % period][c] (the positional table, new/model.py:60).  out may alias a. */
int asrx_rowwise(int32_t op, const float* a, const float* b, float* out, int64_t rows, int32_t d, int64_t period,
                 void* stream);
/* out[b][c][r] = x[b][r][c] (fp32, batch <= 65535): the encoder input's view/transpose (new/model.py:53-55). */
int asrx_transpose_last2(const float* x, int64_t batch, int32_t R, int32_t C, float* out, void* stream);
/* delta[(b*heads+h)*lq+q] = sum_d dO*O (attention backward prologue). */
int asrx_attn_delta(const asrx_attn_desc* d, void* stream);
/* y = dropout(x) with the library RNG (idx = element index); used for tests of the RNG stream. */
int asrx_dropout_mask(uint8_t* keep, int64_t n, float p, uint64_t seed, void* stream);

/* ---------------------------------------------------------------------------------------------------
 * HIP-graph support.  A captured training step replays every launch with the arguments recorded at capture.
 * ------------------------------------------------------------------------------------------------- */
/* Copy nbytes (multiple of 4) of HOST memory to dst (device, 4-byte aligned) through kernel arguments, ordered
 * on `stream`; the host buffer may be reused as soon as the call returns, and the copy is capturable (a replay
 * writes the same bytes again).  Used for grouped-launch tables and per-step scalars. */
int asrx_upload(void* dst, const void* src, int64_t nbytes, void* stream);
/* Device-resident dropout seed offset folded into the seed of every dropout-drawing kernel at its start
 * (offset 0 = seeds used as given).  Set once per training step, BEFORE the step's forward: a replayed graph
 * then draws fresh masks each step while forward and backward of one step still agree. */
int asrx_set_seed_offset(uint64_t offset, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ASRX_H */
