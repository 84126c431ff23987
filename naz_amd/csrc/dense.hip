// Generic conditioner layer: y = act(cat([ctx, x]) @ (W ⊙ mask)^T + b)  (SURVEY.md §8a a6/a7).
//
// Replaces F.linear + nonlinearity inside pyro's ConditionalDenseNN._forward and
// ConditionalAutoRegressiveNN._forward (MaskedLinear = F.linear(x, mask*W, b)),
// reached from naz/flows/transforms.py:142,180,223.  Used by the per-layer Transform
// path for any shape the fused kernels do not instantiate (MADE/nsa/maf layers).
//
// Tiling: 64 batch rows × 64 output features per 256-thread workgroup, 4 waves as
// 2×2 tiles of 32×32, exact-fp32 MFMA v_mfma_f32_32x32x2_f32, BK = 16 staged through
// LDS.  The concat with the context, the MADE mask and the bias+activation
// epilogue are fused, so no [B, C+D] or masked-weight tensor is ever materialised.
#include "naz_device.h"
#include "naz_internal.h"

namespace naz {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int BM = 64, BN = 64, BK = 16, PAD = 4;

__global__ void __launch_bounds__(256) linear_act_kernel(
    const float* __restrict__ ctx, int64_t ldc, int C, const float* __restrict__ x, int64_t ldx, int Kx,
    const float* __restrict__ W, const float* __restrict__ mask, const float* __restrict__ bias,
    float* __restrict__ y, int64_t ldy, int64_t M, int N, int act) {
  __shared__ float As[BK][BM + PAD];
  __shared__ float Bs[BK][BN + PAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t m0 = (int64_t)blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  const int Ktot = C + Kx;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  for (int k0 = 0; k0 < Ktot; k0 += BK) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      const int mm = e >> 4, kk = e & 15;
      const int64_t m = m0 + mm;
      const int k = k0 + kk;
      float av = 0.f;
      if (m < M && k < Ktot) av = (k < C) ? ctx[m * ldc + k] : x[m * ldx + (k - C)];
      As[kk][mm] = av;
      const int n = n0 + mm;
      float bv = 0.f;
      if (n < N && k < Ktot) {
        bv = W[(int64_t)n * Ktot + k];
        if (mask != nullptr) bv *= mask[(int64_t)n * Ktot + k];
      }
      Bs[kk][mm] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const float a = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= N) return;
  const float bn = bias != nullptr ? bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m < M) y[m * ldy + n] = activate_rt(act, acc[r] + bn);
  }
}

int linear_act(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
               const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act, hipStream_t s) {
  if (M == 0 || N == 0) return 0;
  if (C > 0 && ctx == nullptr) return set_error("naz_linear_act: C=%d but ctx is NULL", C);
  if (Kx > 0 && x == nullptr) return set_error("naz_linear_act: Kx=%d but x is NULL", Kx);
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_linear_act: unknown activation %d", act);
  if (M >= 1024) {  // batch-row kernel (gemm_rows.hip); 1 = shape not taken
    const int rc = rowgemm_linear(ctx, ldc, C, x, ldx, Kx, W, mask, b, y, ldy, M, N, act, s);
    if (rc != 1) return rc;
  }
  dim3 grid((unsigned)((M + BM - 1) / BM), (unsigned)((N + BN - 1) / BN));
  hipLaunchKernelGGL(linear_act_kernel, grid, dim3(256), 0, s, ctx, ldc, C, x, ldx, Kx, W, mask, b, y, ldy, M, N,
                     act);
  return check_launch("linear_act_kernel");
}

}  // namespace naz
