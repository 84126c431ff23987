/*
 * naz_hip.h — C ABI of libnazhip.so, the MI355X (gfx950) implementation of naz's
 * normalizing-flow log_prob / sample hot path.
 *
 * Conventions:
 *   - every pointer is a DEVICE pointer owned by the caller, row-major fp32; no
 *     allocation happens inside a call;
 *   - `stream` is a hipStream_t passed as void* (NULL = the default stream);
 *   - return 0 on success, nonzero on error; naz_last_error() returns a
 *     thread-local message describing the last failure;
 *   - calls are stateless and thread-safe across streams.
 *
 * Each entry point names the reference interface it replaces.  In the reference
 * those interfaces are Python calls into pyro-ppl (not vendored; semantics restated
 * in SURVEY.md §8a); the call sites are in /root/reference/src/naz.
 */
#ifndef NAZ_HIP_H
#define NAZ_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- constants ---------------------------------------------------------- */
#define NAZ_LAYOUT_DENSE 0 /* DenseNN hypernet output: [w(Dt*K) | h(Dt*K) | d(Dt*(K-1))]  */
#define NAZ_LAYOUT_ARN 1   /* AutoRegressiveNN output: column p*Dt + i, p in [0, 3K-1)    */
#define NAZ_RQS_FAST 16    /* OR into naz_rqs_fwd/inv's layout: hardware-transcendental
                              select-first evaluation (fp32-grade, ~2x faster); default is the
                              libm-grade evaluator that naz_rqs_bwd's VJP matches            */

#define NAZ_LD_PERDIM 0      /* ld is [B, Dt], per dimension                                */
#define NAZ_LD_ROWSUM 1      /* ld is [B], ld[r]  = sum_i ld[r, i]                          */
#define NAZ_LD_ROWSUM_ADD 2  /* ld is [B], ld[r] += sum_i ld[r, i]                          */
#define NAZ_LD_ROWSUM_SUB 3  /* ld is [B], ld[r] -= sum_i ld[r, i]                          */

#define NAZ_ACT_IDENTITY 0
#define NAZ_ACT_TANH 1 /* naz default activation: flows/transforms.py:133,165,201 */
#define NAZ_ACT_RELU 2
#define NAZ_ACT_SOFTPLUS 3
#define NAZ_ACT_SIGMOID 4

#define NAZ_MFMA_BF16X6 0 /* default: FP32 GEMMs as 6 exact-split bf16 MFMA products (fp32-grade error) */
#define NAZ_MFMA_F32 1    /* exact FP32 MFMA (v_mfma_f32_32x32x2_f32)                                  */
#define NAZ_MFMA_F16X3 2  /* GEMM1 bf16x6, GEMM2/3 as 3 exact-split fp16 products (fp32-grade error;
                             requires every packed |W1|, |W2| < 2^15 — the caller checks at pack time;
                             GEMM1 also fp16x3 for workgroups whose data is inside fp16 range)         */
#define NAZ_MFMA_F16X3_R16 3 /* the f16x3 arithmetic on 16-row waves (16x16x32 MFMA, 4 waves/SIMD);
                                GEMM1 falls back to exact fp32 MFMA per workgroup; S, D-S multiples of 4 */

/* ---- library ------------------------------------------------------------ */
const char* naz_last_error(void);
int naz_abi_version(void); /* bumps on any signature or contract change (2: naz_ar_desc.flags, affine clip modes,
                             * naz_ar_flow_supported = 2 for forward-only shapes; 3: packed-image headers and
                             * registry, caller-owned workspace for the autoregressive log_prob entries) */

/* ---- Packed images (ABI 3) -----------------------------------------------
 * Every packed weight image (naz_coupling_pack, naz_coupling_pack_bwd, naz_ar_flow_pack[_host],
 * naz_ar_flow_pack_fwd[_host], naz_ar_flow_pack_bwd, naz_cnf_pack) starts with a 256-byte header:
 * magic "NAZI", layout version, image kind, a layout tag hashed from the descriptor fields the layout
 * depends on, layers, flags (pass-0 constants), body bytes.  The *_packed_bytes functions include
 * it.  The device packers register each image they write (base address, header, draw stride,
 * draws) with the library; a host-packed image, once copied to the device, is registered by
 * naz_image_attach (reads its header back once, synchronising `stream`; `bytes` = the device
 * buffer's size).  Every launch entry resolves its image argument through the registry before it
 * launches and refuses, with an error, an address that holds no registered image (or is not a draw
 * of one), an image of another kind, descriptor or layout version, a different layer count or body
 * size, or a draw range outside the packed set.  The registry trusts the last packer or attach at an
 * address: memory overwritten by other means is not detected.  naz_image_release forgets one.
 * Python-assembled images of the per-layer MADE kernels (naz_made_*) carry no header.          */
int naz_image_attach(const void* image, int64_t bytes, void* stream);
/* Library-wide launch choices.  "rowgemm_split": the batch-row GEMM (naz_linear_act, naz_gemm_dact,
 * naz_gemm_jvp_bwd, naz_gemm's dX shape) runs outputs wider than 128 columns as balanced panels of at
 * most 128 (1, default; NAZ_RG_SPLIT in the environment sets the initial value) or as one (0).  "rowgemm_fill":
 * for short batches it narrows the column panels until the grid holds this many workgroups per CU
 * (0 = off, at most 16; default 2, NAZ_RG_FILL).  Neither changes a result.  "rowgemm_x6": its
 * arithmetic, exact FP32 MFMA (0, default; NAZ_RG_X6) or the bf16x6 split (1: fp32-grade, other
 * rounding).  value >= 0 sets one; returns the value before the call (-1 and an error for an unknown
 * key). */
int naz_tuning(const char* key, int value);
int naz_image_release(const void* image);
/* Diagnostics (no reference counterpart): the first non-finite row state a fused log_prob
 * kernel met, as {1, workgroup, layer, stage counter, row} ({0, ...} = none), optionally
 * cleared.  Fails unless the library was built with -DNAZ_DEBUG_NONFINITE.               */
int naz_debug_nonfinite(int64_t* out5, int clear);

/* ---- a1+a2: conditional spline -------------------------------------------
 * Replaces [pyro] ConditionedSpline._call / ._inverse over a conditioner output,
 * i.e. ConditionalSpline._params (softmax, softmax, softplus) followed by
 * _monotonic_rational_spline(order="quadratic"), reached from
 * naz/flows/transforms.py:190 (ConditionalSplineAutoregressive) and :228
 * (SplineCoupling's upper spline).
 *   x   [B, Dt] (row stride ldx)       raw [B, Dt*(3K-1)] (row stride ldr, `layout`)
 *   y   [B, Dt] (row stride ldy)       ld  per `ld_mode`; the log|det| of the map applied
 *                                           (naz_rqs_inv: of the inverse map)            */
int naz_rqs_fwd(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy, float* ld,
                int ld_mode, int64_t B, int Dt, int K, int layout, float bound, void* stream);
int naz_rqs_inv(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy, float* ld,
                int ld_mode, int64_t B, int Dt, int K, int layout, float bound, void* stream);

/* ---- a1: unconditional elementwise spline ([pyro] Spline, the coupling's lower
 * spline, naz/flows/transforms.py:128 intent).  uw/uh [Dt,K], ud [Dt,K-1] are the
 * UNNORMALISED parameters; ld is per-dim [B, Dt].                                   */
int naz_spline_elementwise(int inverse, const float* x, int64_t ldx, const float* uw, const float* uh,
                           const float* ud, float* y, int64_t ldy, float* ld, int64_t B, int Dt, int K, float bound,
                           void* stream);

/* ---- a6/a7: one conditioner layer ----------------------------------------
 * Replaces torch F.linear(cat([ctx, x]), W ⊙ mask, b) + nonlinearity inside
 * [pyro] ConditionalDenseNN / ConditionalAutoRegressiveNN._forward
 * (naz/flows/transforms.py:142,180,223).  The concatenation is fused: input column
 * k < C reads ctx[m*ldc + k] (ldc = 0 broadcasts one context row), k >= C reads
 * x[m*ldx + k - C].  W is [N, C+Kx] row-major; mask (same shape) may be NULL.
 *   y[m, n] = act( sum_k in[m,k] * (W[n,k]*mask[n,k]) + b[n] )                       */
int naz_linear_act(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
                   const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act, void* stream);

/* ---- §8f rank 1: conditioner layer batched over parameter draws -----------
 * Replaces jax.vmap over the weights of bflow_jax_maf.py:113-116 (masked_linear), i.e. the
 * per-draw evaluation loops of the Bayesian front end (plot.py:192-204, calibrate.py:145-151,
 * hmc_maf_exact.py:128-133): nbatch independent problems
 *   y_z = act(cat([ctx_z, x_z]) @ (W_z * mask)^T + b_z),  z = 0 .. nbatch-1,
 * with problem z's operands at ctx + z*sctx, x + z*sx, W + z*sw, b + z*sb, y + z*sy (strides in
 * floats; sctx = 0 / ldc = 0 broadcast a context). The mask [N, C+Kx] is shared. M rows each. */
int naz_linear_act_batched(const float* ctx, int64_t ldc, int64_t sctx, int C, const float* x, int64_t ldx,
                           int64_t sx, int Kx, const float* W, int64_t sw, const float* mask, const float* b,
                           int64_t sb, float* y, int64_t ldy, int64_t sy, int64_t M, int N, int nbatch, int act,
                           void* stream);

/* ---- a10: chained input gradient of a Linear/act conditioner -------------------
 * C[m, n] = (Σ_k A[m, k] · W[k, n] · mask[k, n]) · act'(dy[m, n]), act' taken from the
 * post-activation value dy (tanh 1 - y², relu y > 0, softplus 1 - e^-y, sigmoid y(1 - y)):
 * dPre_{l-1} = (dPre_l · (W_l ⊙ M_l)) ⊙ act'(h_{l-1}) in one batch-row GEMM (replaces the
 * naz_gemm dX + naz_act_bwd pair of the autograd walk). mask nullable; W, mask rows at ldw, ldm. */
int naz_gemm_dact(const float* A, int64_t lda, int K, const float* W, int64_t ldw, const float* mask, int64_t ldm,
                  float* C, int64_t ldc, const float* dy, int64_t lddy, int dact, int64_t M, int N, void* stream);

/* ---- a5/a6 forward + §8f rank 2: fused MADE conditioner + affine step ------
 * One MAF layer in the sampling direction for P weight draws in one launch: replaces
 * ConditionalAutoRegressiveNN.forward + AffineAutoregressive._call (naz/flows/transforms.py:
 * 133-160) and the JAX front end's forward_fn (bflow_jax_maf.py:172-178):
 *   raw = W_out·act(…act(W_0·[ctx|x] + b_0)…) + b_out;  y = raw[:D] + x·exp(clamp(raw[D:],-5,3));
 *   ld  = / += / -= Σ clamp(raw[D:], -5, 3)   (ld_mode ROWSUM / ROWSUM_ADD / ROWSUM_SUB)
 * packed: per-draw nets at packed + z*wstride in the layout documented in made.hip (masked
 * weights, MFMA fragment order), naz_made_packed_floats() floats each; nh = hidden width in
 * 32-blocks (1..5), nhid hidden layers, 2D <= 32, act tanh or relu. x/y/ld: S rows per draw,
 * draw strides sx/sy/sld; ctx [C] (ldc = sctx = 0), rows at ldc, draw stride sctx. */
int64_t naz_made_packed_floats(int nhid, int nh, int C, int D);
int naz_made_affine_fwd(const float* packed, int64_t wstride, int nhid, int nh, int C, int D, const float* ctx,
                        int64_t ldc, int64_t sctx, const float* x, int64_t ldx, int64_t sx, float* y, int64_t ldy,
                        int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, void* stream);

/* Inverse single-dim variant (the last pass of a 2-dim MAF inverse, §8f rank 1): a context-free
 * MADE chain on x (C = 0) whose output rows 0, 1 are (mean, log_scale) of dim `dim`; then
 * y = x except y[dim] = (v[dim] - mean)·exp(-clamp(ls, -5, 3)), ld op= clamp(ls). v (the data
 * being inverted) rows at ldv, draw stride sv; packed as naz_made_packed_floats(nhid, nh, 0, D). */
int naz_made_affine_inv1(const float* packed, int64_t wstride, int nhid, int nh, int D, const float* x, int64_t ldx,
                         int64_t sx, const float* v, int64_t ldv, int64_t sv, int dim, float* y, int64_t ldy,
                         int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, void* stream);

/* ---- a5: affine autoregressive elementwise step --------------------------
 * Replaces the elementwise part of [pyro] AffineAutoregressive._call / ._inverse
 * (naz/flows/transforms.py:159; JAX restatement bflow_jax_maf.py:169-194):
 *   fwd: y = exp(clamp(ls,-5,3)) * x + mean       inv: y = (x - mean) * exp(-clamp(ls,-5,3))
 * raw is the ARN output [B, 2*D] (mean = columns 0..D-1, log_scale = D..2D-1);
 * ld (per ld_mode) is the FORWARD log|det| = clamp(ls) for both directions.         */
int naz_affine_ar(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
                  float* ld, int ld_mode, int64_t B, int D, void* stream);

/* ---- a8: base density and bounding ----------------------------------------
 * out[r] (+)= sum_i (-z^2/2 - log sqrt(2 pi))   (Independent(Normal(0,1)), naz/flows/flow.py:37)
 * accumulate = 1 adds into out, 0 overwrites.                                        */
int naz_base_log_prob(const float* z, int64_t ldz, float* out, int64_t B, int D, int accumulate, void* stream);
/* naz/flows/transforms.py:20-23: y = logit((x-low)/(high-low)); out_logjac[r] = -sum log u + log1p(-u) - sum log(high-low) */
int naz_bounding_fwd(const float* x, int64_t ldx, const float* low, const float* high, float* y, int64_t ldy,
                     float* out_logjac, int64_t B, int D, void* stream);
/* naz/flows/transforms.py:25-27: x = sigmoid(y)*(high-low) + low */
int naz_bounding_inv(const float* y, int64_t ldy, const float* low, const float* high, float* x, int64_t ldx,
                     int64_t B, int D, void* stream);

/* ---- a10: backward of the NLL training step --------------------------------
 * naz's `train` (naz/trainers/train_flows.py:194-213) calls loss.backward() through pyro's
 * transforms; these are the VJPs of the kernels above.
 *
 * naz_rqs_bwd: x = the INPUT the forward/inverse map was applied to; g_out [B, Dt] (may be
 * NULL) = dL/d(map output); g_ld = dL/d(the ld that naz_rqs_{fwd,inv} returned), per
 * g_ld_mode 0 none / 1 [B] row-sum / 2 [B, Dt]; writes g_in [B, Dt] (may be NULL) and
 * g_raw (same layout as raw).  ldr = 0 (one shared parameter row, e.g. a lower spline):
 * g_raw is [Dt*(3K-1)] and is ACCUMULATED (+=) over the batch.                        */
int naz_rqs_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* g_out,
                int64_t ldgo, const float* g_ld, int g_ld_mode, float* g_in, int64_t ldgi, float* g_raw, int64_t ldgr,
                int64_t B, int Dt, int K, int layout, float bound, void* stream);
/* C[m,n] (+)= sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn]; exact fp32 MFMA.  With a mask:
 * mask_b = 0 multiplies the OUTPUT by mask[m*smm + n*smn] (dW of a MADE layer), mask_b = 1
 * multiplies the B OPERAND by mask[k*smm + n*smn] (dX through W*mask).
 * split_k > 1 accumulates atomically (zero C first for an overwrite).
 * rowsum (may be NULL): also (+)= sum_k A(m,k) into rowsum[m] — with A = dPre^T this is the
 * bias gradient, computed as an extra all-ones column of B in the same MFMA reduction.      */
int naz_gemm(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
             int64_t sbn, float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn,
             int mask_b, int accumulate, int split_k, float* rowsum, void* stream);
/* nbatch weight-gradient reductions in one launch (bf16x6 MFMA, exact to fp32 products):
 * C[b][n1][n2] += sum_m G[b][m][n1] X[b][m][n2] and (rowsum != NULL) rowsum[b][n1] += sum_m G[b][m][n1],
 * with G[b] = g + b*bg (row stride sgm = N1), X[b] = x + b*bx (row stride sxm = N2), C[b] = c + b*bc
 * (row stride scm, unit column stride), rowsum[b] = rowsum + b*br; 16-byte aligned rows,
 * N1 <= 256, N2 <= 160, both multiples of 4.  Accumulates (zero C / rowsum first).  The fused maf
 * backward's dW of all layers (flows/maf_grad.py), replacing per-layer jax.grad reductions. */
int naz_wgrad_batched(int64_t M, int N1, int N2, int nbatch, const float* g, int64_t sgm, int64_t bg, const float* x,
                      int64_t sxm, int64_t bx, float* c, int64_t scm, int64_t bc, float* rowsum, int64_t br,
                      void* stream);
/* VJP of naz_affine_ar (the kernel reports the FORWARD log-det sum(clamp(ls)) in both
 * directions).  x = the map's input, y = its output, g_ld [B] = dL/d(row ld) (may be NULL).
 * pyro clamps log_scale with clamp_preserve_gradients: the clamp passes gradients through.
 * `mode`: bit 0 = inverse direction; bit 1 (NAZ_AFFINE_CLIP_ZERO_GRAD) = differentiate the clamp
 * as jnp.clip instead (zero gradient outside [-5, 3]; the JAX Bayesian MAF, bflow_jax_maf.py:177-192).
 * Writes g_x [B, D] (may be NULL) and g_raw [B, 2D].                                       */
#define NAZ_AFFINE_CLIP_ZERO_GRAD 2
int naz_affine_ar_bwd(int mode, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* y,
                      int64_t ldy, const float* g_y, int64_t ldgy, const float* g_ld, float* g_x, int64_t ldgx,
                      float* g_raw, int64_t ldgr, int64_t B, int D, void* stream);
/* One dim of the maf inverse's VJP, for a maf backward composed of GEMMs (the shapes without the
 * fused naz_ar_flow_bwd_layer; flows/maf_grad_wide.py).  Replaces, for one dim, the autograd of
 * pyro AffineAutoregressive._inverse (naz transforms.py:159) + its log-det under naz train's loss
 * (train_flows.py:195,208).  Layer output s_d = (y_d - m_d) e^{-c(a_d)}, raw = the MADE output
 * [B, 2D] (mean cols 0..D-1, log_scale cols D..2D-1), g = dL/ds [B, D] (complete for `dim`),
 * g_lp [B] (NULL: 1).  Writes g_next[:, dim] = dL/dy_dim, tot[:, dim] / tot[:, D + dim] =
 * dL/d(mean, log_scale), and chain (may be NULL) = a [B, 2D] row zero but for those two columns.
 * mode: NAZ_AFFINE_CLIP_ZERO_GRAD = jnp.clip's gradient, else pyro's clamp_preserve_gradients. */
int naz_maf_dim_vjp(int mode, const float* raw, int64_t ldr, const float* s_out, int64_t lds, const float* g,
                    int64_t ldg, const float* g_lp, float* g_next, int64_t ldgn, float* tot, int64_t ldt, float* chain,
                    int64_t ldch, int64_t B, int D, int dim, void* stream);
/* out[n] += sum_m A[m*lda + n]  (atomic; zero `out` first for a plain column sum)         */
int naz_colsum(const float* A, int64_t lda, int64_t M, int N, float* out, void* stream);
/* gpre = gy * act'(pre) computed from the post-activation y (tanh, relu, softplus, sigmoid) */
int naz_act_bwd(const float* gy, int64_t ldg, const float* y, int64_t ldy, float* gpre, int64_t ldp, int64_t M, int N,
                int act, void* stream);
/* MC dropout on a conditioner activation [M, N] (naz transforms.py:29-95, the Dropout
 * conditioners behind dropout_p; mcdpflow.py:39-56 samples with them active):
 *   y[m, n] = keep(seed, m, n) ? x[m, n] / (1 - p) : 0,   P(keep) = 1 - p,  0 <= p < 1.
 * keep is a hash of (seed, m, n): the backward applies the same call (same seed) to the
 * gradient. y may alias x.                                                                */
int naz_dropout(const float* x, int64_t ldx, float* y, int64_t ldy, int64_t M, int N, float p, uint64_t seed,
                void* stream);
/* g_z[r, i] = -z[r, i] * g_lp[r]   (VJP of naz_base_log_prob)                             */
int naz_base_log_prob_bwd(const float* z, int64_t ldz, const float* g_lp, float* g_z, int64_t ldgz, int64_t B, int D,
                          void* stream);

/* ---- a3+a8+a9: fused conditional spline-coupling flow ---------------------
 * Replaces the whole of NormalizingFlow.log_prob / .sample (naz/flows/flow.py:45-79,
 * 94-129) for flow_type "nsc" (naz/flows/transforms.py:201-236 intent = pyro
 * SplineCoupling with a (Conditional)DenseNN hypernet), L layers in one launch.
 *
 * Parameters live in ONE flat fp32 buffer, per layer in this order:
 *   nn.layers.0.weight [H, C+S]  nn.layers.0.bias [H]
 *   nn.layers.1.weight [H, H]    nn.layers.1.bias [H]
 *   nn.layers.2.weight [(D-S)(3K-1), H]  nn.layers.2.bias [(D-S)(3K-1)]
 *   lower_spline.unnormalized_{widths [S,K], heights [S,K], derivatives [S,K-1]}   (if has_lower)
 * naz_coupling_pack re-lays them (on the device) into the kernel's MFMA operand
 * order; re-pack after every weight update.                                          */
typedef struct naz_coupling_desc {
  int D, C, S, K, L, H;   /* data dim, context dim, split dim, bins, layers, hidden width (2 hidden layers) */
  int act;                /* NAZ_ACT_* */
  int has_lower;          /* 1: lower (unconditional) spline on x1; 0: pyro identity=True */
  float bound;            /* spline box half-width (pyro default 3.0) */
  int mfma_mode;          /* NAZ_MFMA_BF16X6 (0), NAZ_MFMA_F32, NAZ_MFMA_F16X3 or NAZ_MFMA_F16X3_R16; the packed
                             layout depends on it (naz_amd's "auto" picks F16X3_R16 when supported)          */
  int reserved[6];
} naz_coupling_desc;

int naz_coupling_supported(const naz_coupling_desc* d); /* 1 if a fused instantiation exists */
int64_t naz_coupling_param_count(const naz_coupling_desc* d);
int64_t naz_coupling_packed_bytes(const naz_coupling_desc* d);
int naz_coupling_pack(const naz_coupling_desc* d, const float* flat_params, void* packed, void* stream);
/* out_lp[r] = log p(x_r | ctx_r); ctx may be NULL when C == 0; ldc = 0 broadcasts one
 * context row.  low/high (length D) enable naz's logit bounding prologue (flow.py:70-73);
 * pass NULL for bounds=None.                                                          */
int naz_coupling_log_prob(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                          const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                          int64_t B, void* stream);
/* y = T_L ∘ … ∘ T_1 (z) (TransformedDistribution.sample's transform chain);
 * out_ld (may be NULL) receives sum_l log|det J_l| per row.  low/high as above apply
 * inverse_bounding_transform to the output (flow.py:129).                             */
int naz_coupling_sample(const naz_coupling_desc* d, const void* packed, const float* z, int64_t ldz,
                        const float* ctx, int64_t ldc, const float* low, const float* high, float* y, int64_t ldy,
                        float* out_ld, int64_t B, void* stream);
/* ONE layer of the same image (SURVEY §8b naz_coupling_layer_{fwd,inv}; replaces pyro
 * SplineCoupling._call / ._inverse of one naz transform, transforms.py:113-129,201-236, as the
 * per-Transform protocol calls it: t(x), t.inv(y)): layer `layer` of the packed flow (mode
 * NAZ_MFMA_F16X3_R16), fwd: y = T_l(x), inv: y = T_l^{-1}(x); ld [B] receives the layer's FORWARD
 * log|det J| at the pre-image (pyro's log_abs_det_jacobian) by ld_mode NAZ_LD_ROWSUM (=),
 * NAZ_LD_ROWSUM_ADD (+=) or NAZ_LD_ROWSUM_SUB (-=).  One launch; no bounding, no base density. */
int naz_coupling_layer_fwd(const naz_coupling_desc* d, const void* packed, int layer, const float* x, int64_t ldx,
                           const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                           void* stream);
int naz_coupling_layer_inv(const naz_coupling_desc* d, const void* packed, int layer, const float* x, int64_t ldx,
                           const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                           void* stream);

/* ---- a10 over a3: the fused NLL training step of the coupling flow ----------------
 * Replaces the autograd walk of train's loss.backward() (naz/trainers/train_flows.py:195,208)
 * through NormalizingFlow.log_prob (flow.py:45-79) for the spline-coupling flow.  Requires a
 * packed image of mode NAZ_MFMA_F16X3_R16 (naz_coupling_pack) plus the backward image:
 *   naz_coupling_pack_bwd: per-layer fp32 transposed-weight images (size
 *     naz_coupling_bwd_packed_bytes) from the same flat parameters; re-pack after updates.
 *   naz_coupling_log_prob_train: out_lp as naz_coupling_log_prob, computed with libm-grade
 *     activations / splines (the reference walk's precision), and states [L+1][B][D] with
 *     states[l+1] = layer l's input in the log_prob direction, states[0] = z.
 *   naz_coupling_bwd_layer: for layer l (call l = 0 .. L-1), given g_in = dLoss/dstates[l]
 *     and g_lp[r] = dLoss/dlog p_r, writes g_out = dLoss/dstates[l+1], adds the lower
 *     spline's parameter gradients into g_low [S(3K-1)] (zero it first), and writes the
 *     weight-gradient operands: h1, h2 [B,H] (tanh activations), dp1, dp2 [B,H] (dLoss/d
 *     pre-activation), dp3 [B, naz_coupling_dp3_columns] (dLoss/d GEMM3 output, column c
 *     holding DenseNN output row rows[c], -1 = zero padding), x0 [B, C+S] = [ctx | x1].
 *     Then dW2 = dp3ᵀ·h2, dW1 = dp2ᵀ·h1, dW0 = dp1ᵀ·x0, db = column sums (naz_gemm).       */
int64_t naz_coupling_bwd_packed_bytes(const naz_coupling_desc* d);
int naz_coupling_pack_bwd(const naz_coupling_desc* d, const float* flat_params, void* packed_bwd, void* stream);
int naz_coupling_log_prob_train(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                                const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                                float* states, int64_t B, void* stream);
int naz_coupling_bwd_layer(const naz_coupling_desc* d, const void* packed, const void* packed_bwd, const float* flat,
                           int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                           const float* g_lp, float* h1, float* h2, float* dp1, float* dp2, float* dp3, float* x0,
                           float* g_out, float* g_low, int64_t B, void* stream);
/* writes the DenseNN output row of every dp3 column into rows (may be NULL); returns the count */
int naz_coupling_dp3_columns(const naz_coupling_desc* d, int* rows);

/* ---- a11: continuous normalizing flow (FFJORD block, Hutchinson trace) --------
 * naz FFJORDTransform (naz/flows/continuous_transforms.py:70-106) over ConditionalFCNN
 * (:38-60, input cat([x, ctx]), Softplus default).  One call integrates ONE block
 *     d[a, x]/dt = [-eps^T (df/dx) eps, f(x, ctx)],  a(t0) = 0
 * from t0 to t1 with `steps` fixed classical RK4 steps (naz odeint.py:12-19,46-52; SURVEY.md
 * §8d pins config 5 to 8 steps).  log_prob direction = t 0 -> 1 (`_inverse`), sampling
 * = 1 -> 0 (`_call`).  eps [B, D] is the solve's Hutchinson probe.  ld receives a(t1) per
 * ld_mode (ROWSUM write / ROWSUM_ADD / ROWSUM_SUB).  ctx may be NULL (C = 0) or one
 * broadcast row (ldc = 0).  Flat params: W0 [H0, D+C], b0, ..., W_out [D, H_last], b_out.  */
typedef struct naz_cnf_desc {
  int D, C;
  int n_hidden;
  int H[4];
  int act;       /* NAZ_ACT_* (softplus = naz default) */
  int mfma_mode; /* NAZ_CNF_F32 (0): exact FP32 MFMA; NAZ_CNF_F16X3 (1): layer 0 exact FP32, the
                    hidden and output layers as 3 exact-split fp16 products (hidden widths multiples
                    of 32; caller checks |W| < 2^15 at pack time); the packed layout depends on it */
  int reserved[7];
} naz_cnf_desc;
#define NAZ_CNF_F32 0
#define NAZ_CNF_F16X3 1
int naz_cnf_supported(const naz_cnf_desc* d);
int64_t naz_cnf_param_count(const naz_cnf_desc* d);
int64_t naz_cnf_packed_bytes(const naz_cnf_desc* d);
int naz_cnf_pack(const naz_cnf_desc* d, const float* flat, void* packed, void* stream);
int naz_cnf_integrate(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* eps, int64_t lde, float t0, float t1, int steps, float* y,
                      int64_t ldy, float* ld, int ld_mode, int64_t B, void* stream);
/* §8f rank 3: the same block solve with adaptive Dormand-Prince 5(4) (naz FFJORDTransform
 * solver='dopri5', atol = rtol = 1e-4: continuous_transforms.py:73-81; tableau as naz's
 * odeint.py:136-160).  Step control per 16-row group (RMS error norm over the group's [x, a],
 * accept at <= 1, h *= clamp(0.9 e^-1/5, 0.2 | 1 on accept, 10), Hairer initial step, FSAL, last
 * step clipped to t1).  nfe (nullable, device int[ceil(B/16)]): RHS evaluations per group,
 * negated when max_steps ran out before t1. */
int naz_cnf_integrate_dopri5(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                             const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                             float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld, int ld_mode,
                             int* nfe, int64_t B, void* stream);
/* The same solve with torchdyn's BATCH-GLOBAL step control, the reference's semantics (naz
 * FFJORDTransform -> torchdyn odeint, continuous_transforms.py:73-82): one step size for the
 * whole batch, the error norm = RMS over every element of the augmented state [B, D + 1].  Each
 * attempted step is one launch over all rows plus a one-workgroup controller launch; the call
 * polls the controller every 4 attempts, so it SYNCHRONISES `stream` (not graph-capturable).
 * workspace: device buffer of naz_cnf_dopri5_global_workspace_bytes(d, B) bytes.  nfe
 * (nullable, device int[1]): the batch's RHS evaluations, negated when max_steps ran out. */
int64_t naz_cnf_dopri5_global_workspace_bytes(const naz_cnf_desc* d, int64_t B);
int naz_cnf_integrate_dopri5_global(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                                    const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                                    float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld,
                                    int ld_mode, int* nfe, void* workspace, int64_t B, void* stream);
/* CNF training (§8f rank 3; replaces the autograd graph torchdyn's adjoint builds through naz's
 * hutch_trace, continuous_transforms.py:75-89): the input-adjoint GEMM of one vector-field layer
 * under the Hutchinson JVP, with the VJP of the layer's activation fused into its epilogue.  The
 * forward maps (h_in, dh_in) to (h, dh) = (act(W h_in + b), act'(W h_in + b) (W dh_in))
 * (naz_linear_act with its activation epilogue + naz_gemm_dact), kept as row PAIRS: S [M = 2B, N]
 * (lds) with row 2i = h and 2i + 1 = dh of batch row i.  A [M, K] (lda) = the adjoints of the next
 * layer's pre-activations in the same pairing, W [K, N] (ldw), G = A · W, and
 *   C[2i] = G[2i] act' + G[2i+1] (act''/act') dh_i,   C[2i+1] = G[2i+1] act'
 * with act', act''/act' recovered from h_i (softplus: 1 - e^-h, e^-h; tanh: 1 - h², -2h) — the
 * adjoints of this layer's pre-activations.  M even; C rows 16-byte aligned (ldc % 4 == 0). */
int naz_gemm_jvp_bwd(const float* A, int64_t lda, int K, const float* W, int64_t ldw, float* C, int64_t ldc,
                     const float* S, int64_t lds, int act, int64_t M, int N, void* stream);

/* ---- §8b naz_spline_ar_inv / naz_affine_ar_inv: fused log_prob of a whole naz "nsa" or "maf" flow
 * Replaces the D-pass loop of pyro ConditionedSplineAutoregressive._inverse (naz
 * flows/transforms.py:165-198) and ConditionedAffineAutoregressive._inverse (transforms.py:133-160),
 * driven by NormalizingFlow.log_prob (flow.py:45-79), over L layers of
 * ConditionalAutoRegressiveNN(C + D -> H x n_hidden -> D P, tanh) conditioners: ONE launch, every MADE
 * hidden unit computed once (in the pass of its mask degree), f16x3 MFMA, the select-first inverse
 * spline (P = 3K - 1) or the clamped affine inverse (P = 2: mean, log_scale in [-5, 3]) per pass.
 * The hidden-unit degrees the kernel assumes are pyro's (naz_ar_flow_degrees); the caller checks
 * its masks against them. */
#define NAZ_AR_SPLINE 0 /* ConditionalSplineAutoregressive, quadratic RQ spline (naz nsa) */
#define NAZ_AR_AFFINE 1 /* ConditionalAffineAutoregressive, stable=False (naz maf) */
typedef struct naz_ar_desc {
  int D, C, H, K, L; /* data dim, context dim, hidden width, bins (spline only), layers */
  int act;           /* NAZ_ACT_TANH */
  float bound;       /* spline box half-width (spline only) */
  int n_hidden;      /* hidden layers, all of width H */
  int kind;          /* NAZ_AR_SPLINE | NAZ_AR_AFFINE */
  int flags;         /* NAZ_AR_CLIP_ZERO_GRAD (affine backward only); 0 = pyro semantics */
  int reserved[5];
} naz_ar_desc;
/* flags: the affine backward (naz_ar_flow_bwd_layer) differentiates the log_scale clip to [-5, 3]
 * as jnp.clip (zero gradient outside the range: the reference's JAX Bayesian MAF,
 * bflow_jax_maf.py:177,188,192, whose potential NUTS differentiates) instead of pyro's
 * clamp_preserve_gradients (identity gradient: naz's torch maf, transforms.py:133-160). */
#define NAZ_AR_CLIP_ZERO_GRAD 1
/* 1: both directions fused (log_prob + sample); 2: the forward (sample) direction only (the
 * inverse-direction entry points report the shape as unsupported; no instance today); 0: not
 * instantiated.  The wide production MAFs (D=4 | C=2, H=[512]x5) are 1 since ABI 2's round 4:
 * their log_prob is the persistent-grid wide inverse (one launch; its hidden layers 2.. persist in
 * caller-owned WORKSPACE, 128 KB per resident wave: naz_ar_flow_workspace_bytes), without the
 * pass-0-constants form (naz_ar_flow_pass0_floats < 0) and without a fused backward. */
int naz_ar_flow_supported(const naz_ar_desc* d);
int64_t naz_ar_flow_packed_bytes(const naz_ar_desc* d);
/* Device workspace (bytes, 16-byte aligned) that naz_ar_flow_log_prob[_batched|_train] need for B rows
 * x P draws on the current device: 0 for every shape but the wide MAFs (one 4-wave workgroup per CU,
 * 128 KB per wave); -1 for an unsupported descriptor.  Pass it as (workspace, workspace_bytes): a call
 * given less returns an error; no entry allocates.  One workspace per stream. */
int64_t naz_ar_flow_workspace_bytes(const naz_ar_desc* d, int64_t B, int64_t P);
/* deg[u] (u < H) = mask index of hidden unit u in every hidden layer (pyro create_mask) */
int naz_ar_flow_degrees(const naz_ar_desc* d, int* deg);
/* HOST memory in and out.  flat: per layer W0 (x) mask0 [H][C + D] | b0 [H] | {Wi (x) maski [H][H] | bi [H]}
 * for hidden layers 2 .. n_hidden | Wout (x) maskout [D P][H] (ARN rows p D + i) | bout [D P]; perm [L][D]:
 * dim of order p (the ARN's permutation).  packed: naz_ar_flow_packed_bytes bytes, to be copied to the
 * device. */
int naz_ar_flow_pack_host(const naz_ar_desc* d, const float* flat, const int* perm, void* packed);
/* out_lp[r] = log p(x_r | ctx_r) (+ naz bounding map when low/high are set); ldc = 0 broadcasts one
 * context row.  |x|, |ctx| must stay below 2^15 (the f16x3 input split); the caller checks. */
int naz_ar_flow_log_prob(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                         int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* workspace,
                         int64_t workspace_bytes, void* stream);

/* The sampling direction of the same flows (pyro *Autoregressive._call, flow.py:94-129): one launch
 * for all L layers in forward order, each layer ONE MADE pass over its input followed by every dim's
 * map; y = T_L ∘ … ∘ T_1(z), out_ld (nullable) = Σ forward log-dets, low/high: inverse bounding of
 * y.  Its own packed image (naz_ar_flow_fwd_packed_bytes; host pack from the same flat layout as
 * naz_ar_flow_pack_host, no permutation: the masks carry the order).  |ctx| < 2^15. */
int64_t naz_ar_flow_fwd_packed_bytes(const naz_ar_desc* d);
int naz_ar_flow_pack_fwd_host(const naz_ar_desc* d, const float* flat, void* packed);
int naz_ar_flow_sample(const naz_ar_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                       int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld,
                       int64_t B, void* stream);

/* §8f ranks 1-2: the sampler batched over P weight draws of one flow (naz's Bayesian MAF,
 * bflow_jax_maf.py:196-236 sampler per draw: calibrate.py:145-151).  naz_ar_flow_pack_fwd packs the
 * forward images of P draws ON THE DEVICE: flat rows at flat + p sflat (the naz_ar_flow_pack_host
 * flat layout, masks applied), images at packed + p spk (spk >= naz_ar_flow_fwd_packed_bytes / 4).
 * naz_ar_flow_sample_batched: draw p maps z + p sz -> y + p sy (B rows each, row strides ldz /
 * ldy), out_ld + p sld (nullable) = Σ forward log-dets; ctx shared by every draw (ldc = 0: one
 * context vector).  P <= 65535 per call.  mask (nullable, both device packers): the L x per masks
 * in the flat layout (biases 1), shared by every draw; then flat rows are the UNMASKED weights
 * (e.g. the front end's posterior draws as stored) and the packer applies the masks. */
int naz_ar_flow_pack_fwd(const naz_ar_desc* d, const float* flat, int64_t sflat, void* packed, int64_t spk, int64_t P,
                         const float* mask, void* stream);
int naz_ar_flow_sample_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* z, int64_t ldz,
                               int64_t sz, const float* ctx, int64_t ldc, float* y, int64_t ldy, int64_t sy,
                               float* out_ld, int64_t sld, int64_t B, int64_t P, void* stream);

/* §8f rank 1: the log-density batched over P weight draws (naz's Bayesian MAF lp over the training
 * set per posterior draw, bflow_jax_maf.py:196-225 log_prob vmapped over draws: the NUTS potential
 * of calibrate.py).  naz_ar_flow_pack packs the inverse images of P draws ON THE DEVICE: flat rows
 * at flat + p sflat (the naz_ar_flow_pack_host flat layout, masks applied), perm [L][D] in device
 * memory shared by every draw (a permutation of 0..D-1 per layer: the caller checks), images at
 * packed + p spk (spk >= naz_ar_flow_packed_bytes / 4).  naz_ar_flow_log_prob_batched: out_lp + p slp
 * [B] = log p(x + p sx | ctx) under draw p (sx = 0: the same rows for every draw; ldc = 0: one
 * context vector); no bounding.  P <= 65535 per call. */
/* pass0 (nullable, conditional flows with ONE context vector): per draw (stride sp0 >=
 * naz_ar_flow_pass0_floats) and layer, the per-draw constants of the first degree pass — the
 * degree-0 hidden units see only the context — as n_hidden x ceil(E0 / 16) blocks of 16 values
 * (2.8853900817779268 · pre-activation of units 0 .. E0 - 1, E0 = units of mask index 0 per
 * naz_ar_flow_degrees, the block's remaining slots 0) then ceil(P / 16) blocks of 16 (the ARN outputs
 * of the first dim in order, rows p D + perm[0], p < P); the packer writes them in place of that
 * pass's weights, and the image must then be evaluated with pass0_const = 1 and ldc = 0: the
 * kernel skips the first pass's MFMA work. */
int64_t naz_ar_flow_pass0_floats(const naz_ar_desc* d);
int naz_ar_flow_pack(const naz_ar_desc* d, const float* flat, int64_t sflat, const int* perm, void* packed, int64_t spk,
                     int64_t P, const float* pass0, int64_t sp0, const float* mask, void* stream);
int naz_ar_flow_log_prob_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* x, int64_t ldx,
                                 int64_t sx, const float* ctx, int64_t ldc, float* out_lp, int64_t slp, int64_t B,
                                 int64_t P, int pass0_const, void* workspace, int64_t workspace_bytes, void* stream);

/* ---- fused maf backward: the NUTS potential's gradient ------------------
 * Replaces jax.grad of bayesian_normalizing_flow's potential Σ_rows flow_lp(unravel(p))
 * (naz/flows/bflow_jax_maf.py:231-235; examples/papers/2506.05657/hmc_maf_exact.py:118-133) and
 * loss.backward() of a maf NLL (naz/trainers/train_flows.py:194-213).  Affine autoregressive flows
 * at the compiled shapes (naz_ar_flow_bwd_packed_bytes < 0 otherwise; the paper shape
 * D=2 | C=2, H=[150]x3 and the 4-parameter Bayesian D=4 | C=2, H=[150]x3).
 *   naz_ar_flow_log_prob_train: naz_ar_flow_log_prob (one draw, no bounding) that also writes
 *     states [L][B][D]: states[l] = s_l, layer l's output (layer l maps s_{l+1} -> s_l; s_0 = z).
 *     Every affine flow whose inverse is fused (naz_ar_flow_supported == 1): at the shapes without
 *     backward images (the wide MLE MAFs) the backward is composed of naz_linear_act /
 *     naz_gemm_dact / naz_gemm / naz_maf_dim_vjp (flows/maf_grad_wide.py).
 *   naz_ar_flow_pack_bwd: per-layer backward images (naz_ar_flow_bwd_packed_bytes) from the
 *     naz_ar_flow_pack_host flat layout on the device; mask (nullable, same layout) multiplies.
 *   naz_ar_flow_bwd_dims: dims[6] = {n_hidden, HP, XA, XB, X0W, rows per tile}.
 *   naz_ar_flow_bwd_layer: layer `layer`'s backward (call l = 0 .. L-1): g_in [B][D] = dL/ds_l,
 *     g_lp [B] = dL/dlog p (nullable: 1), state = states[layer], packed_fwd = the
 *     naz_ar_flow_pack_fwd image, perm = [L][D] dim of order p; writes g_out [B][D] = dL/ds_{l+1}
 *     and the weight-gradient operands bufs[2 + 3 n_hidden]: x0 [B][X0W] = [ctx | s_l | 0], per
 *     hidden layer i (h_i [B][XA] units < XA, [B][XB] units >= XA; natural tanh), then per hidden
 *     layer i dp_i [B][HP] = dL/d pre-activation, then gout [B][X0W] = dL/d ARN output row
 *     (pi D + d), zero padded.  dW_0 = dp_1ᵀ x0, dW_i = dp_{i+1}ᵀ h_i, dW_out = goutᵀ h_n,
 *     biases = column sums of dp_i / gout (naz_gemm), then times the masks. */
int naz_ar_flow_log_prob_train(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                               int64_t ldc, float* out_lp, float* states, int64_t B, void* workspace,
                               int64_t workspace_bytes, void* stream);
int64_t naz_ar_flow_bwd_packed_bytes(const naz_ar_desc* d);
int naz_ar_flow_bwd_dims(const naz_ar_desc* d, int* dims);
int naz_ar_flow_pack_bwd(const naz_ar_desc* d, const float* flat, const float* mask, void* packed, void* stream);
int naz_ar_flow_bwd_layer(const naz_ar_desc* d, const void* packed_fwd, const void* packed_bwd, const int* perm,
                          int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                          const float* g_lp, float* const* bufs, float* g_out, int64_t B, void* stream);

/* ---- §8b: whole-flow entries over the fused kinds -------------------------------------
 * One descriptor for the flows whose whole log_prob is one launch: the spline coupling flow (naz
 * "nsc": naz_coupling_*) and the autoregressive flows (naz "nsa" / "maf": naz_ar_flow_*).  The
 * packed image is the kind's own (naz_coupling_pack on the device, naz_ar_flow_pack_host on the
 * host); these entries only dispatch.  Replaces NormalizingFlow.log_prob / .sample
 * (naz/flows/flow.py:45-79, 94-129).  naz_workspace_bytes(d, B) = the workspace naz_flow_log_prob
 * needs for B rows: 0 for the coupling kernels and the narrow AR kernels (every intermediate stays
 * on chip), naz_ar_flow_workspace_bytes for the wide MAFs.  naz_flow_sample of an AR flow takes its forward image (naz_ar_flow_pack_fwd_host). */
#define NAZ_FLOW_COUPLING 1
#define NAZ_FLOW_AR 2
typedef struct naz_flow_desc {
  int kind;                   /* NAZ_FLOW_COUPLING | NAZ_FLOW_AR */
  naz_coupling_desc coupling; /* kind == NAZ_FLOW_COUPLING */
  naz_ar_desc ar;             /* kind == NAZ_FLOW_AR */
  int reserved[8];
} naz_flow_desc;
int64_t naz_flow_packed_bytes(const naz_flow_desc* d);
int64_t naz_workspace_bytes(const naz_flow_desc* d, int64_t B);
int naz_flow_log_prob(const naz_flow_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* workspace,
                      int64_t workspace_bytes, void* stream);
int naz_flow_sample(const naz_flow_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                    int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B,
                    void* stream);

#ifdef __cplusplus
}
#endif
#endif /* NAZ_HIP_H */
