// Small row-wise kernels on the flow path.
#include <atomic>

#include "naz_device.h"
#include "naz_internal.h"

namespace naz {

constexpr float kLogSqrt2Pi = 0.91893853320467274178f;

// [pyro] AffineAutoregressive elementwise step (naz/flows/transforms.py:159):
//   fwd  y = exp(clamp(ls, -5, 3)) * x + mean
//   inv  y = (x - mean) * exp(-clamp(ls, -5, 3))
// raw = ARN output [B, 2D]: mean = cols 0..D-1, log_scale = cols D..2D-1.
// One thread per row (D is small for MAFs; the MADE GEMMs dominate).
__global__ void affine_ar_kernel(int inverse, const float* __restrict__ x, int64_t ldx, const float* __restrict__ raw,
                                 int64_t ldr, float* __restrict__ y, int64_t ldy, float* __restrict__ ld, int ld_mode,
                                 int64_t B, int D) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  float s = 0.f;
  for (int i = 0; i < D; ++i) {
    const float mean = raw[r * ldr + i];
    const float raw_ls = raw[r * ldr + D + i];
  const float ls = fminf(fmaxf(raw_ls, -5.f), 3.f);
    const float xv = x[r * ldx + i];
    y[r * ldy + i] = inverse ? (xv - mean) * expf(-ls) : expf(ls) * xv + mean;
    if (ld_mode == NAZ_LD_PERDIM) ld[r * D + i] = ls;
    else s += ls;
  }
  if (ld_mode == NAZ_LD_ROWSUM) ld[r] = s;
  else if (ld_mode == NAZ_LD_ROWSUM_ADD) ld[r] += s;
  else if (ld_mode == NAZ_LD_ROWSUM_SUB) ld[r] -= s;
}

// Independent(Normal(0, 1), 1).log_prob (naz/flows/flow.py:37)
__global__ void base_log_prob_kernel(const float* __restrict__ z, int64_t ldz, float* __restrict__ out, int64_t B,
                                     int D, int accumulate) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  float s = 0.f;
  for (int i = 0; i < D; ++i) {
    const float v = z[r * ldz + i];
    s += -(v * v) / 2.f - kLogSqrt2Pi;
  }
  out[r] = accumulate ? out[r] + s : s;
}

// naz bounding_transform (naz/flows/transforms.py:20-23)
__global__ void bounding_fwd_kernel(const float* __restrict__ x, int64_t ldx, const float* __restrict__ low,
                                    const float* __restrict__ high, float* __restrict__ y, int64_t ldy,
                                    float* __restrict__ logjac, int64_t B, int D) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  float s = 0.f, c = 0.f;
  for (int i = 0; i < D; ++i) {
    const float u = (x[r * ldx + i] - low[i]) / (high[i] - low[i]);
    s += logf(u) + log1pf(-u);
    c += logf(high[i] - low[i]);
    y[r * ldy + i] = logf(u / (1.f - u));
  }
  logjac[r] = -s - c;
}

// naz inverse_bounding_transform (naz/flows/transforms.py:25-27)
__global__ void bounding_inv_kernel(const float* __restrict__ yv, int64_t ldy, const float* __restrict__ low,
                                    const float* __restrict__ high, float* __restrict__ x, int64_t ldx, int64_t B,
                                    int D) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * D) return;
  const int64_t r = e / D;
  const int i = (int)(e - r * D);
  const float sg = 1.f / (1.f + expf(-yv[r * ldy + i]));
  x[r * ldx + i] = sg * (high[i] - low[i]) + low[i];
}

__global__ void base_log_prob_bwd_kernel(const float* __restrict__ z, int64_t ldz, const float* __restrict__ g_lp,
                                         float* __restrict__ g_z, int64_t ldgz, int64_t B, int D) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * D) return;
  const int64_t r = e / D;
  const int i = (int)(e - r * D);
  g_z[r * ldgz + i] = -z[r * ldz + i] * g_lp[r];
}

// VJP of affine_ar_kernel (clamp_preserve_gradients: the clamp is the identity for gradients)
//   fwd  y = e^ls x + mean :  g_x = g_y e^ls,   g_mean = g_y,          g_ls = g_y (y - mean) + g_ld
//   inv  y = (x - mean)e^-ls: g_x = g_y e^-ls,  g_mean = -g_y e^-ls,   g_ls = -g_y y + g_ld
__global__ void affine_ar_bwd_kernel(int inverse, const float* __restrict__ x, int64_t ldx,
                                     const float* __restrict__ raw, int64_t ldr, const float* __restrict__ y,
                                     int64_t ldy, const float* __restrict__ g_y, int64_t ldgy,
                                     const float* __restrict__ g_ld, float* __restrict__ g_x, int64_t ldgx,
                                     float* __restrict__ g_raw, int64_t ldgr, int64_t B, int D) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= B * D) return;
  const int64_t r = e / D;
  const int i = (int)(e - r * D);
  const float mean = raw[r * ldr + i];
  const float raw_ls = raw[r * ldr + D + i];
  const float ls = fminf(fmaxf(raw_ls, -5.f), 3.f);
  const float gy = g_y[r * ldgy + i], yv = y[r * ldy + i];
  const float gl = g_ld != nullptr ? g_ld[r] : 0.f;
  float gx, gm, gs;
  if (inverse & 1) {
    const float sc = expf(-ls);
    gx = gy * sc;
    gm = -gx;
    gs = -gy * yv + gl;
  } else {
    const float sc = expf(ls);
    gx = gy * sc;
    gm = gy;
    gs = gy * (yv - mean) + gl;
  }
  if ((inverse & 2) && !(raw_ls >= -5.f && raw_ls <= 3.f)) gs = 0.f;  // jnp.clip's gradient
  (void)x;
  (void)ldx;
  if (g_x != nullptr) g_x[r * ldgx + i] = gx;
  g_raw[r * ldgr + i] = gm;
  g_raw[r * ldgr + D + i] = gs;
}

// One dim of the maf inverse's VJP (the wide maf backward, flows/maf_grad_wide.py).  Layer output
// s_d = (y_d - m_d) e^{-c(a_d)}, log p += -c(a_d); with g = dL/ds (complete for dim d: every later
// dim's chain has already added its share) and L = sum_rows g_lp log p:
//   dL/dy_d = g_d e^{-c},  dL/dm_d = -g_d e^{-c},  dL/da_d = -g_lp - g_d s_d  (x 1[-5 <= a <= 3]: jnp.clip)
// Writes g_next[:, d]; tot[:, d], tot[:, D + d] (the layer's output gradient, for the dW chain);
// chain (may be NULL) = the whole row, zero but for those two columns (the dim's own input chain).
__global__ void maf_dim_vjp_kernel(int mode, const float* __restrict__ raw, int64_t ldr, const float* __restrict__ sv,
                                   int64_t lds, const float* __restrict__ g, int64_t ldg,
                                   const float* __restrict__ g_lp, float* __restrict__ g_next, int64_t ldgn,
                                   float* __restrict__ tot, int64_t ldt, float* __restrict__ chain, int64_t ldch,
                                   int64_t B, int D, int d) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= B) return;
  const float raw_ls = raw[r * ldr + D + d];
  const float ls = fminf(fmaxf(raw_ls, -5.f), 3.f);
  const float gd = g[r * ldg + d];
  const float gy = gd * expf(-ls);
  float ga = -(g_lp != nullptr ? g_lp[r] : 1.f) - gd * sv[r * lds + d];
  if ((mode & NAZ_AFFINE_CLIP_ZERO_GRAD) && !(raw_ls >= -5.f && raw_ls <= 3.f)) ga = 0.f;
  g_next[r * ldgn + d] = gy;
  tot[r * ldt + d] = -gy;
  tot[r * ldt + D + d] = ga;
  if (chain != nullptr)
    for (int j = 0; j < 2 * D; ++j) chain[r * ldch + j] = j == d ? -gy : j == D + d ? ga : 0.f;
}

static unsigned blocks_for(int64_t n) { return (unsigned)((n + 255) / 256); }

int maf_dim_vjp(int mode, const float* raw, int64_t ldr, const float* sv, int64_t lds, const float* g, int64_t ldg,
                const float* g_lp, float* g_next, int64_t ldgn, float* tot, int64_t ldt, float* chain, int64_t ldch,
                int64_t B, int D, int d, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(maf_dim_vjp_kernel, dim3(blocks_for(B)), dim3(256), 0, s, mode, raw, ldr, sv, lds, g, ldg, g_lp,
                     g_next, ldgn, tot, ldt, chain, ldch, B, D, d);
  return check_launch("maf_dim_vjp_kernel");
}

int affine_ar_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* y, int64_t ldy,
                  const float* g_y, int64_t ldgy, const float* g_ld, float* g_x, int64_t ldgx, float* g_raw,
                  int64_t ldgr, int64_t B, int D, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(affine_ar_bwd_kernel, dim3(blocks_for(B * D)), dim3(256), 0, s, inverse, x, ldx, raw, ldr, y,
                     ldy, g_y, ldgy, g_ld, g_x, ldgx, g_raw, ldgr, B, D);
  return check_launch("affine_ar_bwd_kernel");
}

int base_log_prob_bwd(const float* z, int64_t ldz, const float* g_lp, float* g_z, int64_t ldgz, int64_t B, int D,
                      hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(base_log_prob_bwd_kernel, dim3(blocks_for(B * D)), dim3(256), 0, s, z, ldz, g_lp, g_z, ldgz, B,
                     D);
  return check_launch("base_log_prob_bwd_kernel");
}

// MC dropout on a conditioner activation (naz ConditionalAutoRegressiveNNDropout /
// ConditionalDenseNNDropout, transforms.py:29-95: nn.Dropout(p) after every hidden activation):
//   y[m, n] = keep(seed, m, n) ? x[m, n] / (1 - p) : 0,   P(keep) = 1 - p.
// keep is a counter-based hash of (seed, m, n) — no mask tensor in HBM, and the backward
// (the same call on the gradient) regenerates exactly the forward's mask.  In place allowed.
NAZ_DEV uint32_t drop_hash(uint64_t seed, int64_t m, int n) {
  uint64_t h = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(m + 1)) ^ (0xC2B2AE3D27D4EB4Full * (uint64_t)(n + 1));
  h ^= h >> 33;  // murmur3 fmix64
  h *= 0xFF51AFD7ED558CCDull;
  h ^= h >> 33;
  h *= 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 33;
  return (uint32_t)h;
}

__global__ void dropout_kernel(const float* __restrict__ x, int64_t ldx, float* y, int64_t ldy, int64_t M, int N,
                               uint32_t thresh, float scale, uint64_t seed) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M * N) return;
  const int64_t m = i / N;
  const int n = (int)(i - m * N);
  const float v = x[m * ldx + n];
  y[m * ldy + n] = drop_hash(seed, m, n) >= thresh ? v * scale : 0.f;
}

int dropout(const float* x, int64_t ldx, float* y, int64_t ldy, int64_t M, int N, float p, uint64_t seed,
            hipStream_t s) {
  if (M == 0 || N == 0) return 0;
  const double t = (double)p * 4294967296.0;
  const uint32_t thresh = t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
  const float scale = p >= 1.f ? 0.f : 1.f / (1.f - p);
  hipLaunchKernelGGL(dropout_kernel, dim3(blocks_for(M * N)), dim3(256), 0, s, x, ldx, y, ldy, M, N, thresh, scale,
                     seed);
  return check_launch("dropout_kernel");
}

int affine_ar(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
              float* ld, int ld_mode, int64_t B, int D, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(affine_ar_kernel, dim3(blocks_for(B)), dim3(256), 0, s, inverse, x, ldx, raw, ldr, y, ldy, ld,
                     ld_mode, B, D);
  return check_launch("affine_ar_kernel");
}

int base_log_prob(const float* z, int64_t ldz, float* out, int64_t B, int D, int accumulate, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(base_log_prob_kernel, dim3(blocks_for(B)), dim3(256), 0, s, z, ldz, out, B, D, accumulate);
  return check_launch("base_log_prob_kernel");
}

int bounding_fwd(const float* x, int64_t ldx, const float* low, const float* high, float* y, int64_t ldy,
                 float* out_logjac, int64_t B, int D, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(bounding_fwd_kernel, dim3(blocks_for(B)), dim3(256), 0, s, x, ldx, low, high, y, ldy,
                     out_logjac, B, D);
  return check_launch("bounding_fwd_kernel");
}

int bounding_inv(const float* y, int64_t ldy, const float* low, const float* high, float* x, int64_t ldx, int64_t B,
                 int D, hipStream_t s) {
  if (B == 0) return 0;
  hipLaunchKernelGGL(bounding_inv_kernel, dim3(blocks_for(B * D)), dim3(256), 0, s, y, ldy, low, high, x, ldx, B, D);
  return check_launch("bounding_inv_kernel");
}

// The 256-byte header in front of every packed weight image (capi.cpp: magic, image kind, layout tag,
// layers, body bytes; include/naz_hip.h "Packed images").  Written by a kernel, not a host copy, so
// that a packer call captured in a HIP graph replays it without a host pointer.
struct ImageHeaderWords {
  uint32_t w[16];
};

__global__ void image_header_kernel(uint32_t* __restrict__ base, int64_t stride_words, ImageHeaderWords h, int nwords) {
  const int i = threadIdx.x;  // 64 threads: one 32-bit header word each (the words past nwords are 0)
  base[(int64_t)blockIdx.x * stride_words + i] = i < nwords ? h.w[i] : 0u;
}

int write_image_headers(void* base, int64_t stride_bytes, int64_t P, const uint32_t* words, int nwords, hipStream_t s) {
  if (P <= 0) return 0;
  if (P > 65535) return set_error("packed image headers: at most 65535 images per call");
  if (nwords < 0 || nwords > 16 || (stride_bytes & 3) != 0) return set_error("packed image headers: bad layout");
  ImageHeaderWords h{};
  for (int i = 0; i < nwords; ++i) h.w[i] = words[i];
  hipLaunchKernelGGL(image_header_kernel, dim3((unsigned)P), dim3(64), 0, s, static_cast<uint32_t*>(base),
                     stride_bytes / 4, h, nwords);
  return check_launch("image_header_kernel");
}

int device_cus() {
  static std::atomic<int> cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  int n = cached[dev].load();
  if (n == 0) {
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev].store(n);
  }
  return n;
}

}  // namespace naz
