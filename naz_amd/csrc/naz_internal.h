// Host-side internals shared by the naz_amd HIP translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/naz_hip.h"

namespace naz {

// Thread-local last-error message (naz_last_error); returns -1 for `return set_error(...)`.
int set_error(const char* fmt, ...);
// Checks hipGetLastError after a launch; sets the message and returns nonzero on failure.
int check_launch(const char* what);

int rqs_cond(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
             float* ld, int ld_mode, int64_t B, int Dt, int K, int layout, float bound, hipStream_t s);
int rqs_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* g_out, int64_t ldgo,
            const float* g_ld, int g_ld_mode, float* g_in, int64_t ldgi, float* g_raw, int64_t ldgr, int64_t B, int Dt,
            int K, int layout, float bound, hipStream_t s);
int rqs_uncond(int inverse, const float* x, int64_t ldx, const float* uw, const float* uh, const float* ud, float* y,
               int64_t ldy, float* ld, int64_t B, int Dt, int K, float bound, hipStream_t s);
int linear_act(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
               const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act, hipStream_t s);
int affine_ar(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
              float* ld, int ld_mode, int64_t B, int D, hipStream_t s);
int base_log_prob(const float* z, int64_t ldz, float* out, int64_t B, int D, int accumulate, hipStream_t s);
int bounding_fwd(const float* x, int64_t ldx, const float* low, const float* high, float* y, int64_t ldy,
                 float* out_logjac, int64_t B, int D, hipStream_t s);
int bounding_inv(const float* y, int64_t ldy, const float* low, const float* high, float* x, int64_t ldx, int64_t B,
                 int D, hipStream_t s);

int gemm(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
         float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn, int mask_b, int accumulate,
         int split_k, float* rowsum, hipStream_t s);
// gemm_rows.hip: batch-row GEMMs (forward linear layers, dX, dW)
int rowgemm_linear(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
                   const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act, hipStream_t s);
int rowgemm_linear_batched(const float* ctx, int64_t ldc, int64_t zc, int C, const float* x, int64_t ldx, int64_t zx,
                           int Kx, const float* W, int64_t zw, const float* mask, const float* b, int64_t zb,
                           float* y, int64_t ldy, int64_t zy, int64_t M, int N, int nz, int act, hipStream_t s);
// made.hip: fused MADE conditioner + affine step (forward), batched over weight draws
int64_t made_packed_floats(int nhid, int nh, int C, int D);
int made_affine_fwd(const float* packed, int64_t wstride, int nhid, int nh, int C, int D, const float* ctx,
                    int64_t ldc, int64_t sctx, const float* x, int64_t ldx, int64_t sx, float* y, int64_t ldy,
                    int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, hipStream_t s);
int rowgemm_dact(const float* A, int64_t lda, int K, const float* W, int64_t ldw, const float* mask, int64_t ldm,
                 float* C, int64_t ldc, const float* dy, int64_t lddy, int dact, int64_t M, int N, hipStream_t s);
int made_affine_inv1(const float* packed, int64_t wstride, int nhid, int nh, int D, const float* x, int64_t ldx,
                     int64_t sx, const float* v, int64_t ldv, int64_t sv, int dim, float* y, int64_t ldy, int64_t sy,
                     float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, hipStream_t s);
int gemm_rows_try(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                  int64_t sbn, float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn,
                  int mask_b, int accumulate, float* rowsum, hipStream_t s, int* rc);
int affine_ar_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* y, int64_t ldy,
                  const float* g_y, int64_t ldgy, const float* g_ld, float* g_x, int64_t ldgx, float* g_raw,
                  int64_t ldgr, int64_t B, int D, hipStream_t s);
int maf_dim_vjp(int mode, const float* raw, int64_t ldr, const float* sv, int64_t lds, const float* g, int64_t ldg,
                const float* g_lp, float* g_next, int64_t ldgn, float* tot, int64_t ldt, float* chain, int64_t ldch,
                int64_t B, int D, int d, hipStream_t s);
int colsum(const float* A, int64_t lda, int64_t M, int N, float* out, hipStream_t s);
int act_bwd(const float* gy, int64_t ldg, const float* y, int64_t ldy, float* gp, int64_t ldp, int64_t M, int N, int act,
            hipStream_t s);
int dropout(const float* x, int64_t ldx, float* y, int64_t ldy, int64_t M, int N, float p, uint64_t seed,
            hipStream_t s);
int base_log_prob_bwd(const float* z, int64_t ldz, const float* g_lp, float* g_z, int64_t ldgz, int64_t B, int D,
                      hipStream_t s);

int coupling_supported(const naz_coupling_desc* d);
int64_t coupling_param_count(const naz_coupling_desc* d);
int64_t coupling_packed_bytes(const naz_coupling_desc* d);
int coupling_pack(const naz_coupling_desc* d, const float* flat, void* packed, hipStream_t s);
int coupling_log_prob(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, hipStream_t s);
int coupling_sample(const naz_coupling_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                    int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B,
                    hipStream_t s);
int64_t coupling_bwd_packed_bytes(const naz_coupling_desc* d);
int coupling_pack_bwd(const naz_coupling_desc* d, const float* flat, void* packed, hipStream_t s);
int coupling_log_prob_train(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                            const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                            float* states, int64_t B, hipStream_t s);
int coupling_bwd_layer(const naz_coupling_desc* d, const void* packed, const void* packed_bwd, const float* flat,
                       int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                       const float* g_lp, float* h1, float* h2, float* dp1, float* dp2, float* dp3, float* x0,
                       float* g_out, float* g_low, int64_t B, hipStream_t s);
int coupling_dp3_columns(const naz_coupling_desc* d, int* rows);
int coupling_layer(const naz_coupling_desc* d, int inv, const void* packed, int layer, const float* x, int64_t ldx,
                   const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                   hipStream_t s);

int ar_flow_supported(const naz_ar_desc* d);
int64_t ar_flow_packed_bytes(const naz_ar_desc* d);
int ar_flow_degrees(const naz_ar_desc* d, int* deg);
int ar_flow_pack_host(const naz_ar_desc* d, const float* flat, const int* perm, void* packed);
int64_t ar_flow_fwd_packed_bytes(const naz_ar_desc* d);
int ar_flow_pack_fwd_host(const naz_ar_desc* d, const float* flat, void* packed);
int ar_flow_sample(const naz_ar_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx, int64_t ldc,
                   const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B, hipStream_t s);
int ar_flow_pack_fwd(const naz_ar_desc* d, const float* flat, int64_t sflat, void* packed, int64_t spk, int64_t P,
                     const float* mask, hipStream_t s);
int ar_flow_sample_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* z, int64_t ldz,
                           int64_t sz, const float* ctx, int64_t ldc, float* y, int64_t ldy, int64_t sy, float* out_ld,
                           int64_t sld, int64_t B, int64_t P, hipStream_t s);
int64_t ar_flow_pass0_floats(const naz_ar_desc* d);
int ar_flow_pack(const naz_ar_desc* d, const float* flat, int64_t sflat, const int* perm, void* packed, int64_t spk,
                 int64_t P, const float* pass0, int64_t sp0, const float* mask, hipStream_t s);
int64_t ar_flow_workspace_bytes(const naz_ar_desc* d, int64_t B, int64_t P);
int ar_flow_log_prob_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* x, int64_t ldx,
                             int64_t sx, const float* ctx, int64_t ldc, float* out_lp, int64_t slp, int64_t B, int64_t P,
                             int pass0_const, void* ws, int64_t ws_bytes, hipStream_t s);
int ar_flow_log_prob(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                     int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* ws,
                     int64_t ws_bytes, hipStream_t s);
int ar_flow_log_prob_train(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                           int64_t ldc, float* out_lp, float* states, int64_t B, void* ws, int64_t ws_bytes,
                           hipStream_t s);
int64_t ar_flow_bwd_packed_bytes(const naz_ar_desc* d);
int ar_flow_bwd_dims(const naz_ar_desc* d, int* dims);
int ar_flow_pack_bwd(const naz_ar_desc* d, const float* flat, const float* mask, void* packed, hipStream_t s);
int ar_flow_bwd_layer(const naz_ar_desc* d, const void* packed_fwd, const void* packed_bwd, const int* perm, int layer,
                      const float* state, const float* ctx, int64_t ldc, const float* g_in, const float* g_lp,
                      float* const* bufs, float* g_out, int64_t B, hipStream_t s);

int cnf_supported(const naz_cnf_desc* d);
int64_t cnf_param_count(const naz_cnf_desc* d);
int64_t cnf_packed_bytes(const naz_cnf_desc* d);
int cnf_pack(const naz_cnf_desc* d, const float* flat, void* packed, hipStream_t s);
int cnf_integrate(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                  int64_t ldc, const float* eps, int64_t lde, float t0, float t1, int steps, float* y, int64_t ldy,
                  float* ld, int ld_mode, int64_t B, hipStream_t s);
int cnf_integrate_dopri5(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                         int64_t ldc, const float* eps, int64_t lde, float t0, float t1, float atol, float rtol,
                         int max_steps, float* y, int64_t ldy, float* ld, int ld_mode, int* nfe, int64_t B,
                         hipStream_t s);
int64_t cnf_dopri5_global_workspace_bytes(const naz_cnf_desc* d, int64_t B);
int cnf_integrate_dopri5_global(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                                const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                                float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld, int ld_mode,
                                int* nfe, void* work, int64_t B, hipStream_t s);
int wgrad_batched(int64_t M, int N1, int N2, int nbatch, const float* g, int64_t sgm, int64_t bg, const float* x,
                  int64_t sxm, int64_t bx, float* c, int64_t scm, int64_t bc, float* rowsum, int64_t br,
                  hipStream_t s);
// elementwise.hip: the 256-byte header in front of each of P packed images (image p at base + p * stride)
int write_image_headers(void* base, int64_t stride_bytes, int64_t P, const uint32_t* words, int nwords, hipStream_t s);
// gemm_rows.hip: the batch-row GEMM's panel-split setting (v >= 0 sets; returns the previous value)
int rowgemm_split_setting(int v);
// ... and its arithmetic: exact FP32 MFMA (0) or the bf16x6 split (1, rowgemm_x6_kernel)
int rowgemm_x6_setting(int v);
// ... and its small-batch grid fill: column panels narrowed to reach v workgroups per CU (0 = off)
int rowgemm_fill_setting(int v);
// ... and its f16x3 form (rowgemm_h3_kernel: the caller keeps |B| < 2^9)
int rowgemm_h3_setting(int v);
int rowgemm_bres_setting(int v);
// elementwise.hip: compute units of the current device (cached per device)
int device_cus();
int rowgemm_jvp_bwd(const float* A, int64_t lda, int K, const float* W, int64_t ldw, float* C, int64_t ldc,
                    const float* S, int64_t lds, int act, int64_t M, int N, hipStream_t s);

}  // namespace naz
