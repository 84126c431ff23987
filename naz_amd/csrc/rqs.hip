// Standalone rational-quadratic spline kernels (SURVEY.md §8a rows a1+a2).
//
// Replaces, for one ConditionedSpline call, pyro's ~40 eager kernels
// (softmax/softplus in ConditionalSpline._params, pad, cumsum, searchsorted,
// seven gathers, the rational evaluation and the logs) reached from
// naz/flows/transforms.py:190 (nsa) and :228 (nsc intent).
//
// Layout: one workgroup owns R = 256 / Dt consecutive rows.  The rows' raw
// conditioner outputs (R × Dt·(3K−1) floats, contiguous when the caller's row
// stride equals the row length) are copied HBM→LDS with 16-byte loads, then each
// thread evaluates one (row, dim) with its knots in registers.  The per-row
// log-det sum is a fixed-order LDS reduction (dims 0..Dt−1, like torch's .sum(-1)).
// Two evaluators: the libm-grade one (knot cumsum in double, expf/logf, IEEE divides; what the
// autograd walk and its VJP use) is VALU-bound at ~2.1 TB/s; `layout | NAZ_RQS_FAST` selects the
// select-first evaluator of the fused kernels (rqs_select: hardware transcendentals, only the
// selected bin formed), HBM-bound at ~4.4-4.7 TB/s algorithmic (2^20 rows, Dt=8, K=8), used by
// the inference paths.  Per (row, dim) 4·(3K−1) + 4 bytes in, 4 (+4) bytes out.
#include "naz_device.h"
#include "naz_internal.h"
#include "spline_bwd.h"

// backward of the training walk on the hardware transcendentals (spline_bwd.h FAST)
#ifndef NAZ_RQS_BWD_FAST
#define NAZ_RQS_BWD_FAST true
#endif

namespace naz {

// Copy `n` floats starting at src[0] into lds[0..n) with 16-B loads where aligned.
NAZ_DEV void block_copy_to_lds(float* lds, const float* __restrict__ src, int n, int tid, int nthreads) {
  uintptr_t addr = reinterpret_cast<uintptr_t>(src);
  int head = (int)(((16 - (addr & 15)) & 15) >> 2);
  if ((addr & 3) != 0) head = n;  // not even 4-B aligned: scalar path
  if (head > n) head = n;
  for (int i = tid; i < head; i += nthreads) lds[i] = src[i];
  int nvec = (n - head) >> 2;
  const float4* s4 = reinterpret_cast<const float4*>(src + head);
  for (int i = tid; i < nvec; i += nthreads) {
    float4 v = s4[i];
    int o = head + 4 * i;
    lds[o + 0] = v.x; lds[o + 1] = v.y; lds[o + 2] = v.z; lds[o + 3] = v.w;
  }
  for (int i = head + 4 * nvec + tid; i < n; i += nthreads) lds[i] = src[i];
}

template <int K, bool INV, bool FAST>
__global__ void __launch_bounds__(256) rqs_cond_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ raw, int64_t ldr,
    float* __restrict__ y, int64_t ldy, float* __restrict__ ld_out, int ld_mode, int64_t B, int Dt,
    int layout, float bound) {
  extern __shared__ float lds[];
  constexpr int PD = 3 * K - 1;
  const int P = Dt * PD;
  const int R = (Dt >= 256) ? 1 : 256 / Dt;
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int rows = (int)((B - r0) < R ? (B - r0) : R);
  float* raw_s = lds;              // [R][P]
  float* ld_s = lds + (size_t)R * P;  // [R][Dt]

  if (ldr == P) {
    block_copy_to_lds(raw_s, raw + r0 * ldr, rows * P, tid, blockDim.x);
  } else {
    for (int i = tid; i < rows * P; i += blockDim.x) {
      int r = i / P, c = i - r * P;
      raw_s[i] = raw[(r0 + r) * ldr + c];
    }
  }
  __syncthreads();

  const RqsConsts<K, INV> rc(bound);
  for (int e = tid; e < rows * Dt; e += blockDim.x) {
    const int r = e / Dt, i = e - r * Dt;
    const float* pr = raw_s + (size_t)r * P;
    float uw[K], uh[K], ud[K - 1];
    if (layout == NAZ_LAYOUT_DENSE) {
#pragma unroll
      for (int k = 0; k < K; ++k) { uw[k] = pr[i * K + k]; uh[k] = pr[Dt * K + i * K + k]; }
#pragma unroll
      for (int k = 0; k < K - 1; ++k) ud[k] = pr[2 * Dt * K + i * (K - 1) + k];
    } else {  // ARN: raw column p*Dt + i
#pragma unroll
      for (int k = 0; k < K; ++k) { uw[k] = pr[k * Dt + i]; uh[k] = pr[(K + k) * Dt + i]; }
#pragma unroll
      for (int k = 0; k < K - 1; ++k) ud[k] = pr[(2 * K + k) * Dt + i];
    }
    const float xv = x[(r0 + r) * ldx + i];
    float ld;
    float yv;
    if constexpr (FAST) {
      yv = rqs_select<K, INV>(uw, uh, ud, xv, bound, rc, ld);
    } else {
      SplineTables<K> t;
      build_tables<K>(uw, uh, ud, bound, t);
      yv = rqs_apply<K, INV>(t, xv, bound, ld);
    }
    y[(r0 + r) * ldy + i] = yv;
    if (ld_mode == NAZ_LD_PERDIM) ld_out[(r0 + r) * Dt + i] = ld;
    else ld_s[r * Dt + i] = ld;
  }
  if (ld_mode == NAZ_LD_PERDIM) return;
  __syncthreads();
  for (int r = tid; r < rows; r += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < Dt; ++i) s += ld_s[r * Dt + i];
    if (ld_mode == NAZ_LD_ROWSUM) ld_out[r0 + r] = s;
    else if (ld_mode == NAZ_LD_ROWSUM_ADD) ld_out[r0 + r] += s;
    else ld_out[r0 + r] -= s;
  }
}

// Unconditional elementwise spline ([pyro] Spline, the coupling's lower spline):
// params uw [Dt,K], uh [Dt,K], ud [Dt,K-1] shared by all rows.
template <int K, bool INV>
__global__ void __launch_bounds__(256) rqs_uncond_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ uwp, const float* __restrict__ uhp,
    const float* __restrict__ udp, float* __restrict__ y, int64_t ldy, float* __restrict__ ld_out, int ld_mode,
    int64_t B, int Dt, float bound) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * Dt) return;
  const int64_t r = e / Dt;
  const int i = (int)(e - r * Dt);
  float uw[K], uh[K], ud[K - 1];
#pragma unroll
  for (int k = 0; k < K; ++k) { uw[k] = uwp[i * K + k]; uh[k] = uhp[i * K + k]; }
#pragma unroll
  for (int k = 0; k < K - 1; ++k) ud[k] = udp[i * (K - 1) + k];
  SplineTables<K> t;
  build_tables<K>(uw, uh, ud, bound, t);
  float ld;
  y[r * ldy + i] = rqs_apply<K, INV>(t, x[r * ldx + i], bound, ld);
  ld_out[r * Dt + i] = ld;  // per-dim only (row sums are formed by the caller's layer)
  (void)ld_mode;
}

template <int K, bool INV>
static int launch_rqs_cond(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
                           float* ld, int ld_mode, int64_t B, int Dt, int layout, float bound, hipStream_t s) {
  const bool fast = (layout & NAZ_RQS_FAST) != 0;
  layout &= ~NAZ_RQS_FAST;
  const int R = (Dt >= 256) ? 1 : 256 / Dt;
  const size_t lds = ((size_t)R * Dt * (3 * K - 1) + (size_t)R * Dt) * sizeof(float);
  if (lds > 160 * 1024) return set_error("naz_rqs: Dt*K too large for one LDS block (%zu bytes)", lds);
  const int64_t grid = (B + R - 1) / R;
  if (fast)
    hipLaunchKernelGGL((rqs_cond_kernel<K, INV, true>), dim3((unsigned)grid), dim3(256), lds, s, x, ldx, raw, ldr, y,
                       ldy, ld, ld_mode, B, Dt, layout, bound);
  else
    hipLaunchKernelGGL((rqs_cond_kernel<K, INV, false>), dim3((unsigned)grid), dim3(256), lds, s, x, ldx, raw, ldr,
                       y, ldy, ld, ld_mode, B, Dt, layout, bound);
  return check_launch("rqs_cond_kernel");
}

template <int K, bool INV>
static int launch_rqs_uncond(const float* x, int64_t ldx, const float* uw, const float* uh, const float* ud, float* y,
                             int64_t ldy, float* ld, int64_t B, int Dt, float bound, hipStream_t s) {
  const int64_t n = B * Dt;
  const int64_t grid = (n + 255) / 256;
  hipLaunchKernelGGL((rqs_uncond_kernel<K, INV>), dim3((unsigned)grid), dim3(256), 0, s, x, ldx, uw, uh, ud, y, ldy,
                     ld, NAZ_LD_PERDIM, B, Dt, bound);
  return check_launch("rqs_uncond_kernel");
}

// ---------------------------------------------------------------------------
// Backward (a10): d(input) and d(raw) from upstream d(output) and d(ld).
//   g_ld_mode: 0 none, 1 one value per row (the row-sum ld), 2 per (row, dim)
//   BCAST:     raw is ONE row shared by all rows (ldr = 0, e.g. the coupling's lower spline):
//              the block reduces d(raw) over its rows in LDS and adds it atomically to g_raw[P].
// ---------------------------------------------------------------------------
template <int K, bool INV, bool BCAST>
__global__ void __launch_bounds__(256) rqs_bwd_kernel(
    const float* __restrict__ x, int64_t ldx, const float* __restrict__ raw, int64_t ldr,
    const float* __restrict__ g_out, int64_t ldgo, const float* __restrict__ g_ld, int g_ld_mode,
    float* __restrict__ g_in, int64_t ldgi, float* __restrict__ g_raw, int64_t ldgr, int64_t B, int Dt, int layout,
    float bound) {
  extern __shared__ float lds[];
  constexpr int PD = 3 * K - 1;
  const int P = Dt * PD;
  const int R = (Dt >= 256) ? 1 : 256 / Dt;
  const int tid = threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int rows = (int)((B - r0) < R ? (B - r0) : R);
  float* raw_s = lds;  // [R][P] (BCAST: [1][P]) then, for BCAST, grads [R][P]
  float* gr_s = lds + (BCAST ? P : (size_t)R * P);
  if (BCAST) {
    for (int i = tid; i < P; i += blockDim.x) raw_s[i] = raw[i];
    for (int i = tid; i < R * P; i += blockDim.x) gr_s[i] = 0.f;
  } else if (ldr == P) {
    block_copy_to_lds(raw_s, raw + r0 * ldr, rows * P, tid, blockDim.x);
  } else {
    for (int i = tid; i < rows * P; i += blockDim.x) {
      const int r = i / P, c = i - r * P;
      raw_s[i] = raw[(r0 + r) * ldr + c];
    }
  }
  __syncthreads();
  for (int e = tid; e < rows * Dt; e += blockDim.x) {
    const int r = e / Dt, i = e - r * Dt;
    const float* pr = raw_s + (BCAST ? 0 : (size_t)r * P);
    float uw[K], uh[K], ud[K - 1];
    auto col_w = [&](int k) { return layout == NAZ_LAYOUT_DENSE ? i * K + k : k * Dt + i; };
    auto col_h = [&](int k) { return layout == NAZ_LAYOUT_DENSE ? Dt * K + i * K + k : (K + k) * Dt + i; };
    auto col_d = [&](int k) { return layout == NAZ_LAYOUT_DENSE ? 2 * Dt * K + i * (K - 1) + k : (2 * K + k) * Dt + i; };
#pragma unroll
    for (int k = 0; k < K; ++k) { uw[k] = pr[col_w(k)]; uh[k] = pr[col_h(k)]; }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) ud[k] = pr[col_d(k)];
    const int64_t row = r0 + r;
    const float go = g_out != nullptr ? g_out[row * ldgo + i] : 0.f;
    const float gl = g_ld_mode == 1 ? g_ld[row] : (g_ld_mode == 2 ? g_ld[row * Dt + i] : 0.f);
    float gw[K], gh[K], gd[K - 1];
    const float gi = rqs_vjp<K, INV, NAZ_RQS_BWD_FAST>(uw, uh, ud, bound, x[row * ldx + i], go, gl, gw, gh, gd);
    if (g_in != nullptr) g_in[row * ldgi + i] = gi;
    float* dst = BCAST ? gr_s + (size_t)r * P : g_raw + row * ldgr;
#pragma unroll
    for (int k = 0; k < K; ++k) { dst[col_w(k)] = gw[k]; dst[col_h(k)] = gh[k]; }
#pragma unroll
    for (int k = 0; k < K - 1; ++k) dst[col_d(k)] = gd[k];
  }
  if (BCAST) {
    __syncthreads();
    for (int c = tid; c < P; c += blockDim.x) {
      float s = 0.f;
      for (int r = 0; r < rows; ++r) s += gr_s[(size_t)r * P + c];
      atomicAdd(g_raw + c, s);
    }
  }
}

template <int K, bool INV>
static int launch_rqs_bwd(const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* g_out,
                          int64_t ldgo, const float* g_ld, int g_ld_mode, float* g_in, int64_t ldgi, float* g_raw,
                          int64_t ldgr, int64_t B, int Dt, int layout, float bound, bool bcast, hipStream_t s) {
  const int R = (Dt >= 256) ? 1 : 256 / Dt;
  const size_t P = (size_t)Dt * (3 * K - 1);
  const size_t lds = (bcast ? (P + (size_t)R * P) : (size_t)R * P) * sizeof(float);
  if (lds > 160 * 1024) return set_error("naz_rqs_bwd: Dt*K too large for one LDS block (%zu bytes)", lds);
  const int64_t grid = (B + R - 1) / R;
  if (bcast)
    hipLaunchKernelGGL((rqs_bwd_kernel<K, INV, true>), dim3((unsigned)grid), dim3(256), lds, s, x, ldx, raw, ldr, g_out,
                       ldgo, g_ld, g_ld_mode, g_in, ldgi, g_raw, ldgr, B, Dt, layout, bound);
  else
    hipLaunchKernelGGL((rqs_bwd_kernel<K, INV, false>), dim3((unsigned)grid), dim3(256), lds, s, x, ldx, raw, ldr,
                       g_out, ldgo, g_ld, g_ld_mode, g_in, ldgi, g_raw, ldgr, B, Dt, layout, bound);
  return check_launch("rqs_bwd_kernel");
}

#define NAZ_K_DISPATCH(K_, CALL) \
  switch (K_) {                  \
    case 2: CALL(2); break;      \
    case 3: CALL(3); break;      \
    case 4: CALL(4); break;      \
    case 5: CALL(5); break;      \
    case 6: CALL(6); break;      \
    case 8: CALL(8); break;      \
    case 10: CALL(10); break;    \
    case 12: CALL(12); break;    \
    case 16: CALL(16); break;    \
    default: return set_error("naz_rqs: count_bins=%d not instantiated (2,3,4,5,6,8,10,12,16)", K_); \
  }

int rqs_cond(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
             float* ld, int ld_mode, int64_t B, int Dt, int K, int layout, float bound, hipStream_t s) {
  if (B == 0) return 0;
  int rc = 0;
#define CALLC(KK)                                                                                              \
  rc = inverse ? launch_rqs_cond<KK, true>(x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, Dt, layout, bound, s) \
               : launch_rqs_cond<KK, false>(x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, Dt, layout, bound, s)
  NAZ_K_DISPATCH(K, CALLC)
#undef CALLC
  return rc;
}

int rqs_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* g_out, int64_t ldgo,
            const float* g_ld, int g_ld_mode, float* g_in, int64_t ldgi, float* g_raw, int64_t ldgr, int64_t B, int Dt,
            int K, int layout, float bound, hipStream_t s) {
  if (B == 0) return 0;
  const bool bcast = ldr == 0;
  int rc = 0;
#define CALLB(KK)                                                                                                 \
  rc = inverse ? launch_rqs_bwd<KK, true>(x, ldx, raw, ldr, g_out, ldgo, g_ld, g_ld_mode, g_in, ldgi, g_raw, ldgr, \
                                          B, Dt, layout, bound, bcast, s)                                       \
               : launch_rqs_bwd<KK, false>(x, ldx, raw, ldr, g_out, ldgo, g_ld, g_ld_mode, g_in, ldgi, g_raw,    \
                                           ldgr, B, Dt, layout, bound, bcast, s)
  NAZ_K_DISPATCH(K, CALLB)
#undef CALLB
  return rc;
}

int rqs_uncond(int inverse, const float* x, int64_t ldx, const float* uw, const float* uh, const float* ud, float* y,
               int64_t ldy, float* ld, int64_t B, int Dt, int K, float bound, hipStream_t s) {
  if (B == 0) return 0;
  int rc = 0;
#define CALLU(KK)                                                                                   \
  rc = inverse ? launch_rqs_uncond<KK, true>(x, ldx, uw, uh, ud, y, ldy, ld, B, Dt, bound, s) \
               : launch_rqs_uncond<KK, false>(x, ldx, uw, uh, ud, y, ldy, ld, B, Dt, bound, s)
  NAZ_K_DISPATCH(K, CALLU)
#undef CALLU
  return rc;
}

}  // namespace naz
