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

// gemm_tn128_kernel: the same contract for the batch-reduction shape with wide outputs —
//   C[m, n] (+)= Σ_k A[k·sak + m] · B[k·sbk + n] [· mask(m, n)]   (A = Gᵀ, B = X, unit m / n strides)
// dW = mask ⊙ (δᵀ·h) of a 512-wide MADE's degree blocks (flows/maf_grad_wide.py), whose outputs
// exceed the batch-reduction kernel's 256 x 256 (gemm_rows.hip wgrad).  128 x 128 tiles per 256-thread
// workgroup (4 waves x 64 x 64 = 2 x 2 v_mfma_f32_32x32x2_f32 blocks), BK = 16 through a
// double-buffered LDS pair with the next chunk's global loads (coalesced along m / n) in flight
// during this chunk's MFMAs: twice the generic tile's FLOPs per loaded byte.
constexpr int TB = 128, TPAD = 4;
__global__ void __launch_bounds__(256) gemm_tn128_kernel(int M, int N, int64_t K, const float* __restrict__ A,
                                                         int64_t sak, const float* __restrict__ Bm, int64_t sbk,
                                                         float* __restrict__ Cm, int64_t scm, int64_t scn,
                                                         const float* __restrict__ mask, int64_t smm, int64_t smn,
                                                         int accumulate, int atomic, int64_t k_per_split,
                                                         float* __restrict__ rowsum, int vec) {
  __shared__ __attribute__((aligned(16))) float As[2][GBK][TB + TPAD];
  __shared__ __attribute__((aligned(16))) float Bs[2][GBK][TB + TPAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.x * TB, n0 = blockIdx.y * TB;
  const int64_t kbeg = (int64_t)blockIdx.z * k_per_split;
  const int64_t kend = (kbeg + k_per_split) < K ? (kbeg + k_per_split) : K;
  const int NE = rowsum != nullptr ? N + 1 : N;  // column N: an all-ones B column -> rowsum
  const int mm = tid & (TB - 1), kq = tid >> 7;  // loader: column mm, k rows kq + 2u
  const int am = m0 + mm, bn = n0 + mm;
  // vec (16-byte aligned rows of A and B, m / n strides 1): 16-byte loads, thread -> (4 columns
  // 4 m4 .. 4 m4 + 3, k rows kr and kr + 8): a quarter of the load instructions and address math of
  // the scalar form (PMC r05: 4.7 VALU per MFMA, two thirds of the wave-cycles issue-stalled)
  const int m4 = tid & 31, kr = tid >> 5;
  float ra[8], rb[8];
  auto ld4 = [&](const float* __restrict__ base, int64_t sk, int64_t k, int c0, int lim, bool ones) {
    float4 v = {0.f, 0.f, 0.f, 0.f};
    if (k < kend) {
      if (c0 + 3 < lim) {
        v = *reinterpret_cast<const float4*>(base + k * sk + c0);
      } else {  // the ragged last group (and the rowsum's all-ones column N)
        float t[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) t[e] = c0 + e < lim ? base[k * sk + c0 + e] : ((ones && c0 + e == N) ? 1.f : 0.f);
        v = {t[0], t[1], t[2], t[3]};
      }
    }
    return v;
  };
  auto load = [&](int64_t k0) {
    if (vec) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t k = k0 + kr + 8 * u;
        const float4 a = ld4(A, sak, k, m0 + 4 * m4, M, false);
        const float4 b = ld4(Bm, sbk, k, n0 + 4 * m4, N, NE > N);
        ra[4 * u] = a.x; ra[4 * u + 1] = a.y; ra[4 * u + 2] = a.z; ra[4 * u + 3] = a.w;
        rb[4 * u] = b.x; rb[4 * u + 1] = b.y; rb[4 * u + 2] = b.z; rb[4 * u + 3] = b.w;
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int64_t k = k0 + kq + 2 * u;
      const bool kin = k < kend;
      ra[u] = (kin && am < M) ? A[k * sak + am] : 0.f;
      rb[u] = (kin && bn < N) ? Bm[k * sbk + bn] : ((kin && bn == N && bn < NE) ? 1.f : 0.f);
    }
  };
  auto store = [&](int buf) {
    if (vec) {
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        *reinterpret_cast<float4*>(&As[buf][kr + 8 * u][4 * m4]) = {ra[4 * u], ra[4 * u + 1], ra[4 * u + 2], ra[4 * u + 3]};
        *reinterpret_cast<float4*>(&Bs[buf][kr + 8 * u][4 * m4]) = {rb[4 * u], rb[4 * u + 1], rb[4 * u + 2], rb[4 * u + 3]};
      }
      return;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      As[buf][kq + 2 * u][mm] = ra[u];
      Bs[buf][kq + 2 * u][mm] = rb[u];
    }
  };
  floatx16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  const int64_t nk = (kend - kbeg + GBK - 1) / GBK;
  if (nk > 0) {
    load(kbeg);
    store(0);
  }
  __syncthreads();
  for (int64_t c = 0; c < nk; ++c) {
    const int buf = (int)(c & 1);
    if (c + 1 < nk) load(kbeg + (c + 1) * GBK);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const int kr = kk + (lane >> 5), cl = lane & 31;
      const float a0 = As[buf][kr][wm * 64 + cl], a1 = As[buf][kr][wm * 64 + 32 + cl];
      const float b0 = Bs[buf][kr][wn * 64 + cl], b1 = Bs[buf][kr][wn * 64 + 32 + cl];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (c + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + 32 * j + (lane & 31);
    if (n >= NE) continue;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= M) continue;
        float v = acc[i][j][r];
        if (mask != nullptr && n < N) v *= mask[(int64_t)m * smm + (int64_t)n * smn];
        float* dst = n < N ? Cm + (int64_t)m * scm + (int64_t)n * scn : rowsum + m;
        if (atomic) atomicAdd(dst, v);
        else *dst = accumulate ? *dst + v : v;
      }
    }
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

static bool gemm_tn128_enabled() {  // NAZ_GEMM_TN128=0: the generic 64 x 64 tile kernel (A/B)
  static const bool on = [] {
    const char* e = getenv("NAZ_GEMM_TN128");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
}

int gemm(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
         float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn, int mask_b, int accumulate,
         int split_k, float* rowsum, hipStream_t s) {
  if (M <= 0 || (N <= 0 && rowsum == nullptr)) return 0;
  if (K <= 0) {
    if (!accumulate && split_k <= 1) return set_error("naz_gemm: K = 0 with overwrite is not supported");
    return 0;
  }
  // the batch reduction over strided column views with outputs >= 64 x 64 (a wide MADE's degree
  // blocks): the 128 x 128 tiles below; gemm_rows.hip's reductions are built for contiguous rows
  const bool tn = sam == 1 && sbn == 1 && !(mask_b && mask != nullptr) && M >= 64 &&
                  N + (rowsum != nullptr ? 1 : 0) >= 64 && K >= 2048 && gemm_tn128_enabled();
  if (!(tn && (sak != M || sbk != N))) {  // batch-row fast paths (gemm_rows.hip)
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
  // split-K always accumulates atomically into C (the caller zeroes C for an overwrite)
  const int atomic = splits > 1 ? 1 : 0;
  if (tn) {  // the batch reduction with wide outputs: 128 x 128 tiles
    dim3 g128((unsigned)((M + TB - 1) / TB), (unsigned)((NE + TB - 1) / TB), (unsigned)splits);
    const auto a16 = [](const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; };
    const int vec = a16(A) && a16(B) && sak % 4 == 0 && sbk % 4 == 0;
    hipLaunchKernelGGL(gemm_tn128_kernel, g128, dim3(256), 0, s, M, N, K, A, sak, B, sbk, C, scm, scn, mask, smm, smn,
                       accumulate, atomic, kps, rowsum, vec);
    return check_launch("gemm_tn128_kernel");
  }
  dim3 grid((unsigned)((M + GBM - 1) / GBM), (unsigned)((NE + GBN - 1) / GBN), (unsigned)splits);
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
