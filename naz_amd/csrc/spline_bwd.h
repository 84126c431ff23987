// Vector-Jacobian product of the rational-quadratic spline (SURVEY.md §8a a1+a2, backward for
// the NLL training step a10).
//
// Both directions share the per-bin parameterisation  x = cw0 + W·θ,  y = F(θ) with
//   F(θ)  = ch0 + H·N/Dn,   N = δθ² + d0·θ(1-θ),   Dn = δ + (d0 + d1 − 2δ)·θ(1-θ),   δ = H/W
//   ldf(θ) = log δ² + log G − 2 log Dn,   G = d1θ² + 2δθ(1-θ) + d0(1-θ)²      (= log dy/dx)
// forward:  θ = (x − cw0)/W, outputs (y, ldf);   inverse: θ solves F(θ) = y (pyro's root formula),
// outputs (x, −ldf).  The inverse's parameter gradient uses the implicit-function rule
// dθ/dp = −F_p / F_θ (equal to differentiating pyro's closed-form root in exact arithmetic).
// Then: bin quantities -> knots (pinned ends carry no gradient, like pyro's in-place
// knots[...,0] = lower) -> cumsum -> min-width blend -> softmax, and slopes -> softplus.
#pragma once
#include "naz_device.h"

namespace naz {

// Returns dL/d(input); accumulates nothing else — writes dL/d(unnormalised params) into
// gw[K], gh[K], gd[K-1].  g_out: upstream gradient on the map's output; g_ld: upstream gradient on
// the log-det the kernel returns for this direction (forward ld, or the inverse map's ld).
// FAST: hardware transcendentals / reciprocals (Math<true>) and fp32 knot prefix sums (the
// training walk's backward, where gradients are compared statistically, not bitwise).
template <int K, bool INV, bool FAST = false>
NAZ_DEV float rqs_vjp(const float* uw, const float* uh, const float* ud, float bound, float v, float g_out,
                      float g_ld, float* gw, float* gh, float* gd) {
  using M = Math<FAST>;
  auto rcp = [](float b) { return FAST ? Math<true>::rcp(b) : 1.f / b; };
#pragma unroll
  for (int k = 0; k < K; ++k) { gw[k] = 0.f; gh[k] = 0.f; }
#pragma unroll
  for (int k = 0; k < K - 1; ++k) gd[k] = 0.f;
  if (!(v >= -bound && v <= bound)) return g_out;  // identity tails

  float fw[K], fh[K];
  softmax_k<K, FAST>(uw, fw);
  softmax_k<K, FAST>(uh, fh);
  SplineTables<K> t;
  if constexpr (FAST) {
    auto knots32 = [&](const float* frac, float minw, float* knots) {
      const float scale = 1.f - minw * (float)K, two_b = 2.f * bound;
      float acc = 0.f;
      knots[0] = -bound;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        acc += minw + scale * frac[k];
        knots[k + 1] = two_b * acc - bound;
      }
      knots[K] = bound;
    };
    knots32(fw, kMinBinWidth, t.cw);
    knots32(fh, kMinBinHeight, t.ch);
  } else {
    knots_from_fractions<K>(fw, kMinBinWidth, bound, t.cw);
    knots_from_fractions<K>(fh, kMinBinHeight, bound, t.ch);
  }
  t.dv[0] = 1.f - kMinDerivative;
  t.dv[K] = 1.f - kMinDerivative;
#pragma unroll
  for (int k = 0; k < K - 1; ++k) t.dv[k + 1] = kMinDerivative + softplus<FAST>(ud[k]);

  int cnt = 0;
#pragma unroll
  for (int k = 0; k <= K; ++k) cnt += (v >= (INV ? t.ch[k] : t.cw[k]) + kSearchEps) ? 1 : 0;
  int idx = cnt - 1;
  idx = idx < 0 ? 0 : (idx > K - 1 ? K - 1 : idx);
  float cw0 = t.cw[0], cw1 = t.cw[1], ch0 = t.ch[0], ch1 = t.ch[1], d0 = t.dv[0], d1 = t.dv[1];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    const bool s = idx == k;
    cw0 = s ? t.cw[k] : cw0;
    cw1 = s ? t.cw[k + 1] : cw1;
    ch0 = s ? t.ch[k] : ch0;
    ch1 = s ? t.ch[k + 1] : ch1;
    d0 = s ? t.dv[k] : d0;
    d1 = s ? t.dv[k + 1] : d1;
  }
  const float W = cw1 - cw0, H = ch1 - ch0, iW = rcp(W), delta = H * iW;
  const float T1 = (d0 + d1) - 2.f * delta;
  float th;
  if constexpr (INV) {
    const float dy = v - ch0;
    const float a = dy * T1 + H * (delta - d0);
    const float b = H * d0 - dy * T1;
    const float c = -delta * dy;
    th = (2.f * c) * rcp(-b - M::sqrt(b * b - 4.f * a * c));
  } else {
    th = (v - cw0) * iW;
  }
  const float om = 1.f - th, tt = th * om;
  const float N = delta * th * th + d0 * tt;
  const float Dn = delta + T1 * tt;
  const float G = d1 * th * th + 2.f * delta * tt + d0 * om * om;
  const float iDn = rcp(Dn), iG = rcp(G);
  // dF/dθ and the other partials of F and ldf
  const float Np = 2.f * delta * th + d0 * (1.f - 2.f * th);
  const float Dp = T1 * (1.f - 2.f * th);
  const float F_th = H * (Np * Dn - N * Dp) * iDn * iDn;
  const float F_H = N * iDn;
  const float F_dl = H * (th * th * Dn - N * (1.f - 2.f * tt)) * iDn * iDn;
  const float F_d0 = H * tt * (Dn - N) * iDn * iDn;
  const float F_d1 = -H * N * tt * iDn * iDn;
  const float Gp = 2.f * d1 * th + 2.f * delta * (1.f - 2.f * th) - 2.f * d0 * om;
  const float L_th = Gp * iG - 2.f * Dp * iDn;
  const float L_dl = 2.f * rcp(delta) + 2.f * tt * iG - 2.f * (1.f - 2.f * tt) * iDn;
  const float L_d0 = om * om * iG - 2.f * tt * iDn;
  const float L_d1 = th * th * iG - 2.f * tt * iDn;

  float g_in, gch0, gH, gdl, gd0, gd1, gcw0, gW;
  if constexpr (!INV) {
    const float gth = g_out * F_th + g_ld * L_th;
    gch0 = g_out;
    gH = g_out * F_H;
    gdl = g_out * F_dl + g_ld * L_dl;
    gd0 = g_out * F_d0 + g_ld * L_d0;
    gd1 = g_out * F_d1 + g_ld * L_d1;
    g_in = gth * iW;
    gcw0 = -gth * iW;
    gW = -gth * th * iW;
  } else {
    // outputs x = cw0 + W·θ and ld_inv = −ldf(θ)
    const float gth = g_out * W - g_ld * L_th;
    gcw0 = g_out;
    gW = g_out * th;
    gdl = -g_ld * L_dl;
    gd0 = -g_ld * L_d0;
    gd1 = -g_ld * L_d1;
    // implicit θ(y, p): dθ/dy = 1/F_θ, dθ/dp = −F_p/F_θ
    const float r = gth * rcp(F_th);
    g_in = r;
    gch0 = -r;
    gH = -r * F_H;
    gdl += -r * F_dl;
    gd0 += -r * F_d0;
    gd1 += -r * F_d1;
  }
  // δ = H / W
  gH += gdl * iW;
  gW += -gdl * delta * iW;
  // bin quantities -> knot / slope arrays
  float gcw[K + 1], gch[K + 1], gdv[K + 1];
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    const float a0 = (k == idx) ? 1.f : 0.f, a1 = (k == idx + 1) ? 1.f : 0.f;
    gcw[k] = a0 * (gcw0 - gW) + a1 * gW;
    gch[k] = a0 * (gch0 - gH) + a1 * gH;
    gdv[k] = a0 * gd0 + a1 * gd1;
  }
  // knots j = 1..K-1 (ends pinned): cw_j = 2B·Σ_{i<j} w_i − B  ->  g_w_i = 2B Σ_{j=i+1}^{K-1} g_cw_j
  const float s_w = 1.f - kMinBinWidth * (float)K, s_h = 1.f - kMinBinHeight * (float)K;
  float gfw[K], gfh[K];
  float accw = 0.f, acch = 0.f;
#pragma unroll
  for (int i = K - 1; i >= 0; --i) {
    gfw[i] = 2.f * bound * accw * s_w;
    gfh[i] = 2.f * bound * acch * s_h;
    if (i >= 1) {
      accw += gcw[i];
      acch += gch[i];
    }
  }
  float dotw = 0.f, doth = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    dotw += fw[i] * gfw[i];
    doth += fh[i] * gfh[i];
  }
#pragma unroll
  for (int i = 0; i < K; ++i) {
    gw[i] = fw[i] * (gfw[i] - dotw);
    gh[i] = fh[i] * (gfh[i] - doth);
  }
#pragma unroll
  for (int k = 0; k < K - 1; ++k) gd[k] = gdv[k + 1] * rcp(1.f + M::exp(-ud[k]));  // softplus' = sigmoid
  return g_in;
}

}  // namespace naz

namespace naz {

// Lean VJP of the INVERSE map in the select-first parameterisation (rqs_select<K, true>, the
// fused kernels' evaluator): knot k of either table is −B + 2B(k·m + s·E_k/E_K) from the prefix
// sums E of the softmax numerators.  Only the selected bin's two knots per table and two slopes
// carry gradient, so the knot -> fraction -> softmax chain collapses to closed forms:
//   g_u_i = f_i · 2Bs · (A·[i < idx] + Bv·[i ≤ idx] − A·F_idx − Bv·F_{idx+1}),
// A / Bv = the gradients on the bin's left / right knot (0 for the pinned end knots), F_k = E_k/E_K,
// and only ud[idx−1], ud[idx] (the bin's interior slopes) get gradient.  Hardware
// transcendentals throughout.  Returns dL/dy; writes the unnormalised-parameter gradients.
//
// Tails (|y| > B, NaN): the map is the identity there and the parameters get no gradient.  The
// bin arithmetic runs on y clamped into [−B, B] and the results are SELECTED, never multiplied
// by an inside flag: evaluated at an out-of-box y the extrapolated rational map's θ leaves [0, 1]
// and its F_θ can be exactly 0 (r06: y = 3.00408 at B = 3 gave θ = 1.046, F_θ = 0, r = ∞, and
// 0 · ∞ = NaN in the lower spline's shared gradient — the configs[3] NLL step's non-finite
// parameters after ~27 Adam steps, VERDICT r05 Weak #2).  Clamped, every quantity is the bin
// edge's, finite, and an inside row's arithmetic is unchanged bit for bit.
template <int K>
NAZ_DEV float rqs_vjp_select_inv(const float* uw, const float* uh, const float* ud, float y_in, float g_x, float g_ld,
                                 float bound, const RqsConsts<K, true>& rc, float* gw, float* gh, float* gd) {
  using M = Math<true>;
  constexpr float kL2E = 1.44269504088896341f;
  const bool inside = y_in >= -bound && y_in <= bound;  // false for NaN
  const float y = fminf(fmaxf(y_in, -bound), bound);  // fmaxf(NaN, −B) = −B: finite either way
  float ew[K], eh[K], Ew[K + 1], Eh[K + 1];
  {
    float mw = uw[0], mh = uh[0];
#pragma unroll
    for (int k = 1; k < K; ++k) {
      mw = fmaxf(mw, uw[k]);
      mh = fmaxf(mh, uh[k]);
    }
    const float mwl = mw * kL2E, mhl = mh * kL2E;
    Ew[0] = 0.f;
    Eh[0] = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      ew[k] = __builtin_amdgcn_exp2f(__builtin_fmaf(uw[k], kL2E, -mwl));
      eh[k] = __builtin_amdgcn_exp2f(__builtin_fmaf(uh[k], kL2E, -mhl));
      Ew[k + 1] = Ew[k] + ew[k];
      Eh[k + 1] = Eh[k] + eh[k];
    }
  }
  const float rw = M::rcp(Ew[K]), rh = M::rcp(Eh[K]);
  const float Aw = rc.cA * rw, Ah = rc.cA * rh;
  // search on the height knots (inverse map), select the bin's prefix sums and slopes
  float s0 = 0.f, s1 = Eh[1], o0 = 0.f, o1 = Ew[1], udl = ud[0], udh = ud[0];
  int idx = 0;
#pragma unroll
  for (int k = 1; k < K; ++k) {
    const bool s = y >= __builtin_fmaf(Ah, Eh[k], rc.key[k]);
    s0 = s ? Eh[k] : s0;
    s1 = s ? Eh[k + 1] : s1;
    o0 = s ? Ew[k] : o0;
    o1 = s ? Ew[k + 1] : o1;
    udl = s ? ud[k - 1] : udl;
    if (k < K - 1) udh = s ? ud[k] : udh;
    idx += s ? 1 : 0;
  }
  const bool first = idx == 0, last = idx == K - 1;
  const float fi = (float)idx;
  const float ch0 = __builtin_fmaf(Ah, s0, __builtin_fmaf(rc.ms, fi, rc.nb));
  const float ch1 = last ? bound : __builtin_fmaf(Ah, s1, __builtin_fmaf(rc.ms, fi + 1.f, rc.nb));
  const float cw0 = __builtin_fmaf(Aw, o0, __builtin_fmaf(rc.mo, fi, rc.nb));
  const float cw1 = last ? bound : __builtin_fmaf(Aw, o1, __builtin_fmaf(rc.mo, fi + 1.f, rc.nb));
  // slopes: softplus and its derivative (sigmoid) from one exp
  auto sp = [](float u, float& sig) {
    const float e = M::exp(-fabsf(u));
    const float r = M::rcp(1.f + e);
    sig = u >= 0.f ? r : e * r;
    return u > 20.f ? u : fmaxf(u, 0.f) + M::log1p(e);
  };
  float sgl, sgh;
  const float spl = sp(udl, sgl), sph = sp(udh, sgh);
  const float d0 = first ? 1.f - kMinDerivative : kMinDerivative + spl;
  const float d1 = last ? 1.f - kMinDerivative : kMinDerivative + sph;
  const float W = cw1 - cw0, H = ch1 - ch0, iW = M::rcp(W), delta = H * iW;
  const float T1 = (d0 + d1) - 2.f * delta;
  const float dy = y - ch0;
  const float a = dy * T1 + H * (delta - d0);
  const float b = H * d0 - dy * T1;
  const float c = -delta * dy;
  const float th = (2.f * c) * M::rcp(-b - M::sqrt(fmaxf(b * b - 4.f * a * c, 0.f)));
  const float om = 1.f - th, tt = th * om;
  const float N = delta * th * th + d0 * tt;
  const float Dn = delta + T1 * tt;
  const float G = d1 * th * th + 2.f * delta * tt + d0 * om * om;
  const float iDn = M::rcp(Dn), iG = M::rcp(G), iDn2 = iDn * iDn;
  const float Np = 2.f * delta * th + d0 * (1.f - 2.f * th);
  const float Dp = T1 * (1.f - 2.f * th);
  const float F_th = H * (Np * Dn - N * Dp) * iDn2;
  const float F_H = N * iDn;
  const float F_dl = H * (th * th * Dn - N * (1.f - 2.f * tt)) * iDn2;
  const float F_d0 = H * tt * (Dn - N) * iDn2;
  const float F_d1 = -H * N * tt * iDn2;
  const float Gp = 2.f * d1 * th + 2.f * delta * (1.f - 2.f * th) - 2.f * d0 * om;
  const float L_th = Gp * iG - 2.f * Dp * iDn;
  const float L_dl = 2.f * M::rcp(delta) + 2.f * tt * iG - 2.f * (1.f - 2.f * tt) * iDn;
  const float L_d0 = om * om * iG - 2.f * tt * iDn;
  const float L_d1 = th * th * iG - 2.f * tt * iDn;
  const float gth = g_x * W - g_ld * L_th;
  const float r = gth * M::rcp(F_th);
  float gW = g_x * th, gH = -r * F_H;
  const float gdl = -g_ld * L_dl - r * F_dl;
  const float gd0 = -g_ld * L_d0 - r * F_d0;
  const float gd1 = -g_ld * L_d1 - r * F_d1;
  const float gcw0 = g_x, gch0 = -r;
  gH += gdl * iW;
  gW += -gdl * delta * iW;
  // left / right knot gradients (pinned end knots carry none)
  const float Aw_ = first ? 0.f : gcw0 - gW, Bw_ = last ? 0.f : gW;
  const float Ah_ = first ? 0.f : gch0 - gH, Bh_ = last ? 0.f : gH;
  const float Tw = (Aw_ * o0 + Bw_ * o1) * rw, Th = (Ah_ * s0 + Bh_ * s1) * rh;
  const float cwk = rc.cA * rw, chk = rc.cA * rh;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const float sw_ = (i < idx ? Aw_ : 0.f) + (i <= idx ? Bw_ : 0.f) - Tw;
    const float sh_ = (i < idx ? Ah_ : 0.f) + (i <= idx ? Bh_ : 0.f) - Th;
    gw[i] = inside ? ew[i] * cwk * sw_ : 0.f;  // identity tails: no parameter gradient
    gh[i] = inside ? eh[i] * chk * sh_ : 0.f;
  }
#pragma unroll
  for (int k = 0; k < K - 1; ++k)
    gd[k] = inside ? (k == idx - 1 ? gd0 * sgl : 0.f) + (k == idx ? gd1 * sgh : 0.f) : 0.f;
  return inside ? r : g_x;
}

}  // namespace naz
