// extern "C" entry points of libnazhip.so (declared in include/naz_hip.h).
// Thin argument validation + dispatch into the HIP translation units.
#include <stdarg.h>
#include <stdio.h>

#include "naz_internal.h"

namespace naz {

static thread_local char g_err[1024] = "";

int set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return -1;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error("%s launch failed: %s", what, hipGetErrorString(e));
  return 0;
}

static hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static int check_spline_args(const char* fn, const float* x, const float* y, int64_t B, int Dt, int K, float bound) {
  if (B < 0 || Dt <= 0) return set_error("%s: bad shape B=%lld Dt=%d", fn, (long long)B, Dt);
  if (B > 0 && (x == nullptr || y == nullptr)) return set_error("%s: null x/y", fn);
  if (K < 2) return set_error("%s: count_bins must be >= 2 (got %d)", fn, K);
  if (1e-3 * K > 1.0) return set_error("%s: Minimal bin width too large for the number of bins", fn);
  if (!(bound > 0.f)) return set_error("%s: bound must be positive", fn);
  return 0;
}

}  // namespace naz

using namespace naz;

extern "C" {

const char* naz_last_error(void) { return g_err; }
int naz_abi_version(void) { return 2; }

int naz_rqs_fwd(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy, float* ld,
                int ld_mode, int64_t B, int Dt, int K, int layout, float bound, void* stream) {
  if (int rc = check_spline_args("naz_rqs_fwd", x, y, B, Dt, K, bound)) return rc;
  return rqs_cond(0, x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, Dt, K, layout, bound, as_stream(stream));
}

int naz_rqs_inv(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy, float* ld,
                int ld_mode, int64_t B, int Dt, int K, int layout, float bound, void* stream) {
  if (int rc = check_spline_args("naz_rqs_inv", x, y, B, Dt, K, bound)) return rc;
  return rqs_cond(1, x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, Dt, K, layout, bound, as_stream(stream));
}

int naz_spline_elementwise(int inverse, const float* x, int64_t ldx, const float* uw, const float* uh,
                           const float* ud, float* y, int64_t ldy, float* ld, int64_t B, int Dt, int K, float bound,
                           void* stream) {
  if (int rc = check_spline_args("naz_spline_elementwise", x, y, B, Dt, K, bound)) return rc;
  return rqs_uncond(inverse, x, ldx, uw, uh, ud, y, ldy, ld, B, Dt, K, bound, as_stream(stream));
}

int naz_linear_act(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
                   const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act, void* stream) {
  if (M < 0 || N < 0 || C < 0 || Kx < 0) return set_error("naz_linear_act: negative shape");
  return linear_act(ctx, ldc, C, x, ldx, Kx, W, mask, b, y, ldy, M, N, act, as_stream(stream));
}

int naz_linear_act_batched(const float* ctx, int64_t ldc, int64_t sctx, int C, const float* x, int64_t ldx,
                           int64_t sx, int Kx, const float* W, int64_t sw, const float* mask, const float* b,
                           int64_t sb, float* y, int64_t ldy, int64_t sy, int64_t M, int N, int nbatch, int act,
                           void* stream) {
  if (M < 0 || N < 0 || C < 0 || Kx < 0 || nbatch < 0) return set_error("naz_linear_act_batched: negative shape");
  if (nbatch > 65535) return set_error("naz_linear_act_batched: nbatch %d > 65535 (grid z)", nbatch);
  if (C > 0 && ctx == nullptr) return set_error("naz_linear_act_batched: C=%d but ctx is NULL", C);
  if (Kx > 0 && x == nullptr) return set_error("naz_linear_act_batched: Kx=%d but x is NULL", Kx);
  if (W == nullptr || y == nullptr) return set_error("naz_linear_act_batched: NULL W or y");
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_linear_act_batched: unknown activation %d", act);
  if ((int64_t)N * (C + Kx) * 4 >= (1ll << 31)) return set_error("naz_linear_act_batched: weight block too large");
  return rowgemm_linear_batched(ctx, ldc, sctx, C, x, ldx, sx, Kx, W, sw, mask, b, sb, y, ldy, sy, M, N, nbatch, act,
                                as_stream(stream));
}

int64_t naz_made_packed_floats(int nhid, int nh, int C, int D) {
  if (nhid < 1 || nh < 1 || C < 0 || D < 1) return -1;
  return made_packed_floats(nhid, nh, C, D);
}

int naz_made_affine_fwd(const float* packed, int64_t wstride, int nhid, int nh, int C, int D, const float* ctx,
                        int64_t ldc, int64_t sctx, const float* x, int64_t ldx, int64_t sx, float* y, int64_t ldy,
                        int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, void* stream) {
  if (S < 0 || P < 0 || x == nullptr || y == nullptr || packed == nullptr)
    return set_error("naz_made_affine_fwd: bad arguments");
  return made_affine_fwd(packed, wstride, nhid, nh, C, D, ctx, ldc, sctx, x, ldx, sx, y, ldy, sy, ld, sld, ld_mode, S,
                         P, act, as_stream(stream));
}

int naz_gemm_dact(const float* A, int64_t lda, int K, const float* W, int64_t ldw, const float* mask, int64_t ldm,
                  float* C, int64_t ldc, const float* dy, int64_t lddy, int dact, int64_t M, int N, void* stream) {
  if (M < 0 || N < 0 || K < 0) return set_error("naz_gemm_dact: negative shape");
  if (M == 0 || N == 0) return 0;
  if (A == nullptr || W == nullptr || C == nullptr || dy == nullptr) return set_error("naz_gemm_dact: null pointer");
  if (dact < 0 || dact > NAZ_ACT_SIGMOID) return set_error("naz_gemm_dact: unknown activation %d", dact);
  const int rc = rowgemm_dact(A, lda, K, W, ldw, mask, ldm, C, ldc, dy, lddy, dact, M, N, as_stream(stream));
  if (rc == 1) return set_error("naz_gemm_dact: weights too large for the batch-row kernel");
  return rc;
}

int naz_made_affine_inv1(const float* packed, int64_t wstride, int nhid, int nh, int D, const float* x, int64_t ldx,
                         int64_t sx, const float* v, int64_t ldv, int64_t sv, int dim, float* y, int64_t ldy,
                         int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, void* stream) {
  if (S < 0 || P < 0 || x == nullptr || y == nullptr || packed == nullptr)
    return set_error("naz_made_affine_inv1: bad arguments");
  return made_affine_inv1(packed, wstride, nhid, nh, D, x, ldx, sx, v, ldv, sv, dim, y, ldy, sy, ld, sld, ld_mode, S,
                          P, act, as_stream(stream));
}

int naz_affine_ar(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
                  float* ld, int ld_mode, int64_t B, int D, void* stream) {
  if (B < 0 || D <= 0) return set_error("naz_affine_ar: bad shape");
  return affine_ar(inverse, x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, D, as_stream(stream));
}

int naz_base_log_prob(const float* z, int64_t ldz, float* out, int64_t B, int D, int accumulate, void* stream) {
  return base_log_prob(z, ldz, out, B, D, accumulate, as_stream(stream));
}

int naz_bounding_fwd(const float* x, int64_t ldx, const float* low, const float* high, float* y, int64_t ldy,
                     float* out_logjac, int64_t B, int D, void* stream) {
  return bounding_fwd(x, ldx, low, high, y, ldy, out_logjac, B, D, as_stream(stream));
}

int naz_bounding_inv(const float* y, int64_t ldy, const float* low, const float* high, float* x, int64_t ldx,
                     int64_t B, int D, void* stream) {
  return bounding_inv(y, ldy, low, high, x, ldx, B, D, as_stream(stream));
}

int naz_rqs_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* g_out,
                int64_t ldgo, const float* g_ld, int g_ld_mode, float* g_in, int64_t ldgi, float* g_raw, int64_t ldgr,
                int64_t B, int Dt, int K, int layout, float bound, void* stream) {
  if (int rc = check_spline_args("naz_rqs_bwd", x, x, B, Dt, K, bound)) return rc;
  if (B > 0 && g_raw == nullptr) return set_error("naz_rqs_bwd: g_raw is required");
  if (g_ld_mode < 0 || g_ld_mode > 2 || (g_ld_mode != 0 && g_ld == nullptr))
    return set_error("naz_rqs_bwd: bad g_ld / g_ld_mode");
  return rqs_bwd(inverse, x, ldx, raw, ldr, g_out, ldgo, g_ld, g_ld_mode, g_in, ldgi, g_raw, ldgr, B, Dt, K, layout,
                 bound, as_stream(stream));
}

int naz_gemm(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
             int64_t sbn, float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn,
             int mask_b, int accumulate, int split_k, float* rowsum, void* stream) {
  if (M < 0 || N < 0 || K < 0) return set_error("naz_gemm: negative shape");
  return gemm(M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, mask, smm, smn, mask_b, accumulate, split_k, rowsum,
              as_stream(stream));
}

int naz_wgrad_batched(int64_t M, int N1, int N2, int nbatch, const float* g, int64_t sgm, int64_t bg, const float* x,
                      int64_t sxm, int64_t bx, float* c, int64_t scm, int64_t bc, float* rowsum, int64_t br,
                      void* stream) {
  if (M > 0 && nbatch > 0 && (g == nullptr || x == nullptr || c == nullptr))
    return set_error("naz_wgrad_batched: null pointer");
  return wgrad_batched(M, N1, N2, nbatch, g, sgm, bg, x, sxm, bx, c, scm, bc, rowsum, br, as_stream(stream));
}

int naz_affine_ar_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* y,
                      int64_t ldy, const float* g_y, int64_t ldgy, const float* g_ld, float* g_x, int64_t ldgx,
                      float* g_raw, int64_t ldgr, int64_t B, int D, void* stream) {
  if (B > 0 && (g_raw == nullptr || g_y == nullptr)) return set_error("naz_affine_ar_bwd: g_y and g_raw are required");
  return affine_ar_bwd(inverse, x, ldx, raw, ldr, y, ldy, g_y, ldgy, g_ld, g_x, ldgx, g_raw, ldgr, B, D,
                       as_stream(stream));
}

int naz_maf_dim_vjp(int mode, const float* raw, int64_t ldr, const float* s_out, int64_t lds, const float* g,
                    int64_t ldg, const float* g_lp, float* g_next, int64_t ldgn, float* tot, int64_t ldt, float* chain,
                    int64_t ldch, int64_t B, int D, int dim, void* stream) {
  if (D <= 0 || dim < 0 || dim >= D) return set_error("naz_maf_dim_vjp: dim %d outside [0, %d)", dim, D);
  if (B > 0 && (raw == nullptr || s_out == nullptr || g == nullptr || g_next == nullptr || tot == nullptr))
    return set_error("naz_maf_dim_vjp: null pointer");
  return maf_dim_vjp(mode, raw, ldr, s_out, lds, g, ldg, g_lp, g_next, ldgn, tot, ldt, chain, ldch, B, D, dim,
                     as_stream(stream));
}

int naz_colsum(const float* A, int64_t lda, int64_t M, int N, float* out, void* stream) {
  return colsum(A, lda, M, N, out, as_stream(stream));
}

int naz_act_bwd(const float* gy, int64_t ldg, const float* y, int64_t ldy, float* gpre, int64_t ldp, int64_t M, int N,
                int act, void* stream) {
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_act_bwd: unknown activation %d", act);
  return act_bwd(gy, ldg, y, ldy, gpre, ldp, M, N, act, as_stream(stream));
}

int naz_dropout(const float* x, int64_t ldx, float* y, int64_t ldy, int64_t M, int N, float p, uint64_t seed,
                void* stream) {
  if (M < 0 || N < 0) return set_error("naz_dropout: negative shape");
  if (!(p >= 0.f && p < 1.f)) return set_error("naz_dropout: p must be in [0, 1)");
  return dropout(x, ldx, y, ldy, M, N, p, seed, as_stream(stream));
}

int naz_base_log_prob_bwd(const float* z, int64_t ldz, const float* g_lp, float* g_z, int64_t ldgz, int64_t B, int D,
                          void* stream) {
  return base_log_prob_bwd(z, ldz, g_lp, g_z, ldgz, B, D, as_stream(stream));
}

int naz_cnf_supported(const naz_cnf_desc* d) { return cnf_supported(d); }
int64_t naz_cnf_param_count(const naz_cnf_desc* d) { return cnf_param_count(d); }
int64_t naz_cnf_packed_bytes(const naz_cnf_desc* d) { return cnf_packed_bytes(d); }
int naz_cnf_pack(const naz_cnf_desc* d, const float* flat, void* packed, void* stream) {
  if (flat == nullptr || packed == nullptr) return set_error("naz_cnf_pack: null pointer");
  return cnf_pack(d, flat, packed, as_stream(stream));
}
int naz_cnf_integrate(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* eps, int64_t lde, float t0, float t1, int steps, float* y,
                      int64_t ldy, float* ld, int ld_mode, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_cnf_integrate: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || eps == nullptr || y == nullptr))
    return set_error("naz_cnf_integrate: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr) return set_error("naz_cnf_integrate: context required");
  return cnf_integrate(d, packed, x, ldx, ctx, ldc, eps, lde, t0, t1, steps, y, ldy, ld, ld_mode, B,
                       as_stream(stream));
}

int naz_cnf_integrate_dopri5(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                             const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                             float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld, int ld_mode,
                             int* nfe, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_cnf_integrate_dopri5: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || eps == nullptr || y == nullptr))
    return set_error("naz_cnf_integrate_dopri5: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_cnf_integrate_dopri5: context required");
  return cnf_integrate_dopri5(d, packed, x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps, y, ldy, ld,
                              ld_mode, nfe, B, as_stream(stream));
}

int64_t naz_cnf_dopri5_global_workspace_bytes(const naz_cnf_desc* d, int64_t B) {
  if (B < 0) return -1;
  return cnf_dopri5_global_workspace_bytes(d, B);
}

int naz_cnf_integrate_dopri5_global(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                                    const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                                    float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld,
                                    int ld_mode, int* nfe, void* workspace, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_cnf_integrate_dopri5_global: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || eps == nullptr || y == nullptr))
    return set_error("naz_cnf_integrate_dopri5_global: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_cnf_integrate_dopri5_global: context required");
  return cnf_integrate_dopri5_global(d, packed, x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps, y, ldy,
                                     ld, ld_mode, nfe, workspace, B, as_stream(stream));
}

int naz_gemm_jvp_bwd(const float* A, int64_t lda, int K, const float* W, int64_t ldw, float* C, int64_t ldc,
                     const float* S, int64_t lds, int act, int64_t M, int N, void* stream) {
  if (M < 0 || N < 0 || K < 0) return set_error("naz_gemm_jvp_bwd: negative shape");
  if (M == 0 || N == 0) return 0;
  if (A == nullptr || W == nullptr || C == nullptr || S == nullptr) return set_error("naz_gemm_jvp_bwd: null pointer");
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_gemm_jvp_bwd: unknown activation %d", act);
  const int rc = rowgemm_jvp_bwd(A, lda, K, W, ldw, C, ldc, S, lds, act, M, N, as_stream(stream));
  if (rc == 1) return set_error("naz_gemm_jvp_bwd: weights too large for the batch-row kernel");
  return rc;
}

int naz_coupling_supported(const naz_coupling_desc* d) { return coupling_supported(d); }
int64_t naz_coupling_param_count(const naz_coupling_desc* d) { return coupling_param_count(d); }
int64_t naz_coupling_packed_bytes(const naz_coupling_desc* d) { return coupling_packed_bytes(d); }

int naz_coupling_pack(const naz_coupling_desc* d, const float* flat_params, void* packed, void* stream) {
  return coupling_pack(d, flat_params, packed, as_stream(stream));
}

int naz_coupling_log_prob(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                          const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                          int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_log_prob: conditional flow needs ctx");
  return coupling_log_prob(d, packed, x, ldx, ctx, ldc, low, high, out_lp, B, as_stream(stream));
}

int naz_coupling_sample(const naz_coupling_desc* d, const void* packed, const float* z, int64_t ldz,
                        const float* ctx, int64_t ldc, const float* low, const float* high, float* y, int64_t ldy,
                        float* out_ld, int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_sample: conditional flow needs ctx");
  return coupling_sample(d, packed, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, as_stream(stream));
}

int64_t naz_coupling_bwd_packed_bytes(const naz_coupling_desc* d) { return coupling_bwd_packed_bytes(d); }

int naz_coupling_pack_bwd(const naz_coupling_desc* d, const float* flat_params, void* packed_bwd, void* stream) {
  return coupling_pack_bwd(d, flat_params, packed_bwd, as_stream(stream));
}

int naz_coupling_log_prob_train(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                                const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                                float* states, int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_log_prob_train: conditional flow needs ctx");
  return coupling_log_prob_train(d, packed, x, ldx, ctx, ldc, low, high, out_lp, states, B, as_stream(stream));
}

int naz_coupling_bwd_layer(const naz_coupling_desc* d, const void* packed, const void* packed_bwd, const float* flat,
                           int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                           const float* g_lp, float* h1, float* h2, float* dp1, float* dp2, float* dp3, float* x0,
                           float* g_out, float* g_low, int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_bwd_layer: conditional flow needs ctx");
  return coupling_bwd_layer(d, packed, packed_bwd, flat, layer, state, ctx, ldc, g_in, g_lp, h1, h2, dp1, dp2, dp3,
                            x0, g_out, g_low, B, as_stream(stream));
}

int naz_coupling_dp3_columns(const naz_coupling_desc* d, int* rows) { return coupling_dp3_columns(d, rows); }

static int coupling_layer_api(const char* what, const naz_coupling_desc* d, int inv, const void* packed, int layer,
                              const float* x, int64_t ldx, const float* ctx, int64_t ldc, float* y, int64_t ldy,
                              float* ld, int ld_mode, int64_t B, void* stream) {
  if (B < 0) return set_error("%s: negative batch", what);
  if (B > 0 && (packed == nullptr || x == nullptr || y == nullptr || ld == nullptr))
    return set_error("%s: null pointer", what);
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr) return set_error("%s: conditional flow needs ctx", what);
  return coupling_layer(d, inv, packed, layer, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B, as_stream(stream));
}
int naz_coupling_layer_fwd(const naz_coupling_desc* d, const void* packed, int layer, const float* x, int64_t ldx,
                           const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                           void* stream) {
  return coupling_layer_api("naz_coupling_layer_fwd", d, 0, packed, layer, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B,
                            stream);
}
int naz_coupling_layer_inv(const naz_coupling_desc* d, const void* packed, int layer, const float* x, int64_t ldx,
                           const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                           void* stream) {
  return coupling_layer_api("naz_coupling_layer_inv", d, 1, packed, layer, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B,
                            stream);
}

int naz_ar_flow_supported(const naz_ar_desc* d) { return ar_flow_supported(d); }
int64_t naz_ar_flow_packed_bytes(const naz_ar_desc* d) { return ar_flow_packed_bytes(d); }
int naz_ar_flow_degrees(const naz_ar_desc* d, int* deg) { return ar_flow_degrees(d, deg); }
int naz_ar_flow_pack_host(const naz_ar_desc* d, const float* flat, const int* perm, void* packed) {
  return ar_flow_pack_host(d, flat, perm, packed);
}
int naz_ar_flow_log_prob(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                           int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_log_prob: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || out_lp == nullptr))
    return set_error("naz_ar_flow_log_prob: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_log_prob: conditional flow needs ctx");
  return ar_flow_log_prob(d, packed, x, ldx, ctx, ldc, low, high, out_lp, B, as_stream(stream));
}

int64_t naz_ar_flow_fwd_packed_bytes(const naz_ar_desc* d) { return ar_flow_fwd_packed_bytes(d); }
int naz_ar_flow_pack_fwd_host(const naz_ar_desc* d, const float* flat, void* packed) {
  return ar_flow_pack_fwd_host(d, flat, packed);
}
int naz_ar_flow_sample(const naz_ar_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                       int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld,
                       int64_t B, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_sample: negative batch");
  if (B > 0 && (packed == nullptr || z == nullptr || y == nullptr)) return set_error("naz_ar_flow_sample: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_sample: conditional flow needs ctx");
  return ar_flow_sample(d, packed, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, as_stream(stream));
}

int naz_ar_flow_pack_fwd(const naz_ar_desc* d, const float* flat, int64_t sflat, void* packed, int64_t spk, int64_t P,
                         const float* mask, void* stream) {
  if (P < 0) return set_error("naz_ar_flow_pack_fwd: negative draw count");
  return ar_flow_pack_fwd(d, flat, sflat, packed, spk, P, mask, as_stream(stream));
}
int naz_ar_flow_sample_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* z, int64_t ldz,
                               int64_t sz, const float* ctx, int64_t ldc, float* y, int64_t ldy, int64_t sy,
                               float* out_ld, int64_t sld, int64_t B, int64_t P, void* stream) {
  if (B < 0 || P < 0) return set_error("naz_ar_flow_sample_batched: negative size");
  if (B > 0 && P > 0 && (packed == nullptr || z == nullptr || y == nullptr))
    return set_error("naz_ar_flow_sample_batched: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && P > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_sample_batched: conditional flow needs ctx");
  return ar_flow_sample_batched(d, packed, spk, z, ldz, sz, ctx, ldc, y, ldy, sy, out_ld, sld, B, P, as_stream(stream));
}

int64_t naz_ar_flow_pass0_floats(const naz_ar_desc* d) { return ar_flow_pass0_floats(d); }
int naz_ar_flow_pack(const naz_ar_desc* d, const float* flat, int64_t sflat, const int* perm, void* packed, int64_t spk,
                     int64_t P, const float* pass0, int64_t sp0, const float* mask, void* stream) {
  if (P < 0) return set_error("naz_ar_flow_pack: negative draw count");
  return ar_flow_pack(d, flat, sflat, perm, packed, spk, P, pass0, sp0, mask, as_stream(stream));
}
int naz_ar_flow_log_prob_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* x, int64_t ldx,
                                 int64_t sx, const float* ctx, int64_t ldc, float* out_lp, int64_t slp, int64_t B,
                                 int64_t P, int pass0_const, void* stream) {
  if (B < 0 || P < 0) return set_error("naz_ar_flow_log_prob_batched: negative size");
  if (B > 0 && P > 0 && (packed == nullptr || x == nullptr || out_lp == nullptr))
    return set_error("naz_ar_flow_log_prob_batched: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && P > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_log_prob_batched: conditional flow needs ctx");
  return ar_flow_log_prob_batched(d, packed, spk, x, ldx, sx, ctx, ldc, out_lp, slp, B, P, pass0_const,
                                  as_stream(stream));
}

// ---- fused maf backward (made_ar_bwd.h): NUTS potential gradient / maf NLL step ----------
int naz_ar_flow_log_prob_train(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                               int64_t ldc, float* out_lp, float* states, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_log_prob_train: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || out_lp == nullptr))
    return set_error("naz_ar_flow_log_prob_train: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_log_prob_train: conditional flow needs ctx");
  if (d == nullptr || d->kind != NAZ_AR_AFFINE || naz_ar_flow_supported(d) != 1)
    return set_error("naz_ar_flow_log_prob_train: no fused affine inverse for this flow");
  return ar_flow_log_prob_train(d, packed, x, ldx, ctx, ldc, out_lp, states, B, as_stream(stream));
}
int64_t naz_ar_flow_bwd_packed_bytes(const naz_ar_desc* d) { return ar_flow_bwd_packed_bytes(d); }
int naz_ar_flow_bwd_dims(const naz_ar_desc* d, int* dims) { return ar_flow_bwd_dims(d, dims); }
int naz_ar_flow_pack_bwd(const naz_ar_desc* d, const float* flat, const float* mask, void* packed, void* stream) {
  return ar_flow_pack_bwd(d, flat, mask, packed, as_stream(stream));
}
int naz_ar_flow_bwd_layer(const naz_ar_desc* d, const void* packed_fwd, const void* packed_bwd, const int* perm,
                          int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                          const float* g_lp, float* const* bufs, float* g_out, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_bwd_layer: negative batch");
  if (B > 0 && (packed_fwd == nullptr || packed_bwd == nullptr || perm == nullptr || state == nullptr ||
                g_in == nullptr || bufs == nullptr || g_out == nullptr))
    return set_error("naz_ar_flow_bwd_layer: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_bwd_layer: conditional flow needs ctx");
  return ar_flow_bwd_layer(d, packed_fwd, packed_bwd, perm, layer, state, ctx, ldc, g_in, g_lp, bufs, g_out, B,
                           as_stream(stream));
}

// ---- §8b whole-flow entries over the fused kinds ----------------------------------------
int64_t naz_flow_packed_bytes(const naz_flow_desc* d) {
  if (d == nullptr) return -1;
  if (d->kind == NAZ_FLOW_COUPLING) return coupling_packed_bytes(&d->coupling);
  if (d->kind == NAZ_FLOW_AR) return ar_flow_packed_bytes(&d->ar);
  return -1;
}

int64_t naz_workspace_bytes(const naz_flow_desc* d, int64_t B) {
  (void)B;  // the fused kernels keep every intermediate on chip
  return naz_flow_packed_bytes(d) < 0 ? -1 : 0;
}

int naz_flow_log_prob(const naz_flow_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* stream) {
  if (d == nullptr) return set_error("naz_flow_log_prob: null descriptor");
  if (d->kind == NAZ_FLOW_COUPLING)
    return naz_coupling_log_prob(&d->coupling, packed, x, ldx, ctx, ldc, low, high, out_lp, B, stream);
  if (d->kind == NAZ_FLOW_AR) return naz_ar_flow_log_prob(&d->ar, packed, x, ldx, ctx, ldc, low, high, out_lp, B, stream);
  return set_error("naz_flow_log_prob: unknown flow kind %d", d->kind);
}

int naz_flow_sample(const naz_flow_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                    int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B,
                    void* stream) {
  if (d == nullptr) return set_error("naz_flow_sample: null descriptor");
  if (d->kind == NAZ_FLOW_COUPLING)
    return naz_coupling_sample(&d->coupling, packed, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, stream);
  if (d->kind == NAZ_FLOW_AR)  // packed = the forward image (naz_ar_flow_pack_fwd_host)
    return naz_ar_flow_sample(&d->ar, packed, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, stream);
  return set_error("naz_flow_sample: unknown flow kind %d", d->kind);
}

}  // extern "C"
