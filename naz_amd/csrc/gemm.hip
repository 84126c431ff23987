// Backward building blocks for the NLL training step: the conditioner
// GEMMs' VJPs  dX = dPre·(W⊙mask),  dW = mask ⊙ (dPreᵀ·X),  db = Σ_rows dPre,  and the
// activation derivative dPre = dY ⊙ act'(Y).
//
// gemm_kernel is a generic strided exact-fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32):
//   C[m, n] (+)= Σ_k A(m, k) · B(k, n) [· mask(m, n)]        (mask_b = 0: the dW case)
//   C[m, n] (+)= Σ_k A(m, k) · B(k, n) · mask(k, n)           (mask_b = 1: the dX case)
// with A(m,k) = A[m·sam + k·sak], B(k,n) = B[k·sbk + n·sbn], mask(i,j) = mask[i·smm + j·smn].  64×64 tiles per 256-thread
// workgroup (4 waves × 32×32), BK = 16 through LDS; the global loads run along whichever
// index has unit stride.  split_k > 1 partitions K over grid.z and accumulates with fp32
// atomics — the dW GEMMs reduce over the batch (K = 2^20 rows) into a tiny output.
#include "naz_device.h"
#include "naz_internal.h"

namespace naz {

typedef float floatx16 __attribute__((ext_vector_type(16)));

constexpr int GBM = 64, GBN = 64, GBK = 16, GPAD = 4;

__global__ void __launch_bounds__(256) gemm_kernel(int M, int N, int64_t K, const float* __restrict__ A, int64_t sam,
                                                   int64_t sak, const float* __restrict__ Bm, int64_t sbk, int64_t sbn,
                                                   float* __restrict__ Cm, int64_t scm, int64_t scn,
                                                   const float* __restrict__ mask, int64_t smm, int64_t smn,
                                                   int mask_b, int accumulate, int atomic, int64_t k_per_split,
                                                   float* __restrict__ rowsum) {
  __shared__ float As[GBK][GBM + GPAD];
  __shared__ float Bs[GBK][GBN + GPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * GBM, n0 = blockIdx.y * GBN;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = (kbeg + k_per_split) < K ? (kbeg + k_per_split) : K;
  const bool a_kfast = sak == 1, b_nfast = sbn == 1;
  // rowsum != null: logical column N is an all-ones B column, its C column goes to rowsum[m]
  const int NE = rowsum != nullptr ? N + 1 : N;
  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
  for (int64_t k0 = kbeg; k0 < kend; k0 += GBK) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = tid + 256 * u;
      int mm, kk;
      if (a_kfast) { mm = e >> 4; kk = e & 15; } else { kk = e >> 6; mm = e & 63; }
      const int m = m0 + mm;
      const int64_t k = k0 + kk;
      As[kk][mm] = (m < M && k < kend) ? A[(int64_t)m * sam + k * sak] : 0.f;
      int nn, kb;
      if (b_nfast) { kb = e >> 6; nn = e & 63; } else { nn = e >> 4; kb = e & 15; }
      const int n = n0 + nn;
      const int64_t kq = k0 + kb;
      float bv = (n < N && kq < kend) ? Bm[kq * sbk + (int64_t)n * sbn] : ((n == N && n < NE && kq < kend) ? 1.f : 0.f);
      if (mask_b && n < N && kq < kend) bv *= mask[kq * smm + (int64_t)n * smn];
      Bs[kb][nn] = bv;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const float a = As[kk + (lane >> 5)][wm * 32 + (lane & 31)];
      const float b = Bs[kk + (lane >> 5)][wn * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    __syncthreads();
  }
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= NE) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m >= M) continue;
    float v = acc[r];
    if (mask != nullptr && !mask_b && n < N) v *= mask[(int64_t)m * smm + (int64_t)n * smn];
    float* dst = n < N ? Cm + (int64_t)m * scm + (int64_t)n * scn : rowsum + m;
    if (atomic) atomicAdd(dst, v);
    else *dst = accumulate ? *dst + v : v;
  }
}

// out[n] (+)= Σ_m A[m, n]   (A row-major with row stride lda).  A block is `cw` adjacent columns
// (a power of two <= 64, >= N when N is narrow) x 256 / cw row lanes, so a wave reads whole
// 256-byte row pieces (the [B, 16] bias gradients of the CNF walk: 16 x 16), walking
// `rows_per_block` rows; the row lanes reduce through LDS, one atomic per column per block.
__global__ void colsum_kernel(const float* __restrict__ A, int64_t lda, int64_t M, int N, float* __restrict__ out,
                              int64_t rows_per_block, int cw) {
  __shared__ float red[256];
  const int tx = threadIdx.x & (cw - 1), ty = threadIdx.x / cw, lanes = 256 / cw;
  const int n = blockIdx.y * cw + tx;
  const int64_t m0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t m1 = (m0 + rows_per_block) < M ? (m0 + rows_per_block) : M;
  float s = 0.f;
  if (n < N) {
#pragma unroll 8
    for (int64_t m = m0 + ty; m < m1; m += lanes) s += A[m * lda + n];  // (unrolled: 8 loads in flight)
  }
  red[threadIdx.x] = s;
  __syncthreads();
  if (ty == 0 && n < N) {
    for (int r = 1; r < lanes; ++r) s += red[r * cw + tx];
    atomicAdd(out + n, s);
  }
}

// dPre = dY ⊙ act'(Y), both [M, N] with row strides
__global__ void act_bwd_kernel(const float* __restrict__ gy, int64_t ldg, const float* __restrict__ y, int64_t ldy,
                               float* __restrict__ gp, int64_t ldp, int64_t M, int N, int act) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= M * N) return;
  const int64_t m = e / N;
  const int n = (int)(e - m * N);
  gp[m * ldp + n] = gy[m * ldg + n] * activate_grad_from_out(act, y[m * ldy + n]);
}

int gemm(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
         float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn, int mask_b, int accumulate,
         int split_k, float* rowsum, hipStream_t s) {
  if (M <= 0 || (N <= 0 && rowsum == nullptr)) return 0;
  if (K <= 0) {
    if (!accumulate && split_k <= 1) return set_error("naz_gemm: K = 0 with overwrite is not supported");
    return 0;
  }
  {  // batch-row fast paths (gemm_rows.hip)
    int rc = 0;
    if (gemm_rows_try(M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, mask, smm, smn, mask_b, accumulate, rowsum, s,
                      &rc) == 0)
      return rc;
  }
  if (split_k < 1) split_k = 1;
  int64_t kps = (K + split_k - 1) / split_k;
  kps = (kps + GBK - 1) / GBK * GBK;
  const int64_t splits = (K + kps - 1) / kps;
  const int NE = rowsum != nullptr ? N + 1 : N;
  dim3 grid((unsigned)((M + GBM - 1) / GBM), (unsigned)((NE + GBN - 1) / GBN), (unsigned)splits);
  // split-K always accumulates atomically into C (the caller zeroes C for an overwrite)
  const int atomic = splits > 1 ? 1 : 0;
  hipLaunchKernelGGL(gemm_kernel, grid, dim3(256), 0, s, M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, mask, smm,
                     smn, mask_b && mask != nullptr, accumulate, atomic, kps, rowsum);
  return check_launch("gemm_kernel");
}

int colsum(const float* A, int64_t lda, int64_t M, int N, float* out, hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  int cw = 1;
  while (cw < N && cw < 64) cw *= 2;
  // rows per block: about 1024 blocks over the rows (enough to fill the chip; more would pile
  // atomics onto the same N addresses), at least 64
  int64_t rpb = (M + 1023) / 1024;
  rpb = rpb < 64 ? 64 : (rpb + 63) / 64 * 64;
  dim3 grid((unsigned)((M + rpb - 1) / rpb), (unsigned)((N + cw - 1) / cw));
  hipLaunchKernelGGL(colsum_kernel, grid, dim3(256), 0, s, A, lda, M, N, out, rpb, cw);
  return check_launch("colsum_kernel");
}

int act_bwd(const float* gy, int64_t ldg, const float* y, int64_t ldy, float* gp, int64_t ldp, int64_t M, int N, int act,
            hipStream_t s) {
  if (M <= 0 || N <= 0) return 0;
  const int64_t n = M * N;
  hipLaunchKernelGGL(act_bwd_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, gy, ldg, y, ldy, gp, ldp, M,
                     N, act);
  return check_launch("act_bwd_kernel");
}

}  // namespace naz
