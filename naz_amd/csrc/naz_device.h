// Device-side building blocks shared by the naz_amd HIP kernels (gfx950 / CDNA4).
//
// The rational-quadratic spline below restates pyro-ppl 1.9's
// distributions/transforms/spline.py::_monotonic_rational_spline (order="quadratic",
// the naz default: naz/flows/transforms.py:165,201) one (row, dim) at a time, with the
// K+1 knots held in registers instead of ~40 separate [B,Dt,K] tensors.
//   * knot cumsum is accumulated in double and rounded per prefix, which is exactly what
//     torch's CPU cumsum does for float32 (acc_type<float> == double on CPU), so knot
//     positions match the CPU reference bit for bit given equal bin fractions;
//   * knot affine map (2B·c − B) uses separately rounded mul/add like torch's eager ops;
//   * bin search = count(x >= knot + eps) − 1, clamped — pyro's _searchsorted/_select_bins.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define NAZ_DEV __device__ __forceinline__

namespace naz {

constexpr float kMinBinWidth = 1e-3f;
constexpr float kMinBinHeight = 1e-3f;
constexpr float kMinDerivative = 1e-3f;
constexpr float kSearchEps = 1e-6f;

// Publish an LDS-DMA ring slot.  A global_load_lds write is pending on the issuing wave's
// vmcnt until it lands in LDS; __syncthreads() alone does NOT reliably drain it: on a loop
// back edge hipcc (ROCm 7.2) emitted only lgkmcnt(0) before the barrier, so a wave could read
// a 1 KB chunk another wave's DMA had not written yet (the intermittent non-finite rows of
// the coupling kernel at 2^20 rows, round 2).  Each wave waits for its OWN DMAs, then the
// barrier makes every wave's chunks visible to all.  tests/test_isa_ring.py checks the built
// code object: every s_barrier reachable with a global_load_lds in flight must be preceded
// by an s_waitcnt vmcnt(0) on every path, loop back edges included.
// The wait is the s_waitcnt builtin (gfx9 encoding 0x0F70 = vmcnt(0), expcnt/lgkmcnt unchanged),
// not inline asm: the compiler's waitcnt pass sees it and drops the loads it covers from its
// scoreboard (after an opaque asm wait it re-waits vmcnt(0) at the first use of a register loaded
// before the barrier — which then also waits for the DMAs issued after it).
NAZ_DEV void ring_barrier() {
#ifndef NAZ_ABL_RING_NOWAIT  // A/B only: the round-2 (racy) form
  __builtin_amdgcn_s_waitcnt(0x0F70);
#endif
  __syncthreads();
}

enum Act : int { ACT_IDENTITY = 0, ACT_TANH = 1, ACT_RELU = 2, ACT_SOFTPLUS = 3, ACT_SIGMOID = 4 };

// Math policy.  ACCURATE = the ocml (libm-grade, ~1 ulp, many instructions) functions,
// used by the HBM-bound kernels.  FAST = the hardware transcendentals (v_exp_f32, v_log_f32,
// v_rcp_f32, v_sqrt_f32; ~1-2 ulp, one instruction each) used by the MFMA-bound fused
// kernel, where the VALU instruction count competes with the matrix pipe for issue.
template <bool FAST>
struct Math;

template <>
struct Math<false> {
  static NAZ_DEV float exp(float x) { return expf(x); }
  static NAZ_DEV float log(float x) { return logf(x); }
  static NAZ_DEV float log1p(float x) { return log1pf(x); }
  static NAZ_DEV float div(float a, float b) { return a / b; }
  static NAZ_DEV float sqrt(float x) { return sqrtf(x); }
};

template <>
struct Math<true> {
  static NAZ_DEV float exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
  static NAZ_DEV float log(float x) { return __builtin_amdgcn_logf(x) * 0.693147180559945309f; }
  static NAZ_DEV float rcp(float x) { return __builtin_amdgcn_rcpf(x); }
  static NAZ_DEV float div(float a, float b) { return a * __builtin_amdgcn_rcpf(b); }
  static NAZ_DEV float sqrt(float x) { return __builtin_amdgcn_sqrtf(x); }
  // log1p with full relative precision for small x (Kahan: log(u) * x / (u - 1), u = 1 + x)
  static NAZ_DEV float log1p(float x) {
    const float u = 1.f + x;
    const float d = u - 1.f;
    return d == 0.f ? x : log(u) * div(x, d);
  }
  // expm1 with full relative precision for small x (Kahan: (u - 1) x / log(u), u = e^x)
  static NAZ_DEV float expm1(float x) {
    const float u = exp(x);
    if (u == 1.f) return x;
    const float um1 = u - 1.f;
    return um1 == -1.f ? -1.f : um1 * div(x, log(u));
  }
};

// torch.nn.functional.softplus(beta=1, threshold=20)
template <bool FAST = false>
NAZ_DEV float softplus(float x) {
  if constexpr (FAST) {
    if (x > 20.f) return x;
    return fmaxf(x, 0.f) + Math<true>::log1p(Math<true>::exp(-fabsf(x)));
  } else {
    return x > 20.f ? x : log1pf(expf(x));
  }
}

template <bool FAST = false>
NAZ_DEV float tanh_f(float x) {
  if constexpr (FAST) {
    // 1 - 2 / (1 + e^{2x}): mul, exp, add, rcp, fma.  Saturates correctly (e^{2x} = inf -> 1,
    // e^{2x} = 0 -> -1); |err| <= ~1e-7 absolute, which is what the next GEMM consumes.
    const float e = __builtin_amdgcn_exp2f(x * 2.88539008177792681f);
    return __builtin_fmaf(-2.f, __builtin_amdgcn_rcpf(1.f + e), 1.f);
  } else {
    const float ax = fabsf(x);
    const float t = expf(-2.f * ax);
    return copysignf((1.f - t) / (1.f + t), x);
  }
}

template <int ACT>
NAZ_DEV float activate(float x) {
  if constexpr (ACT == ACT_TANH) return tanh_f(x);
  else if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
  else if constexpr (ACT == ACT_SOFTPLUS) return softplus(x);
  else if constexpr (ACT == ACT_SIGMOID) return 1.f / (1.f + expf(-x));
  else return x;
}

NAZ_DEV float activate_rt(int act, float x) {
  switch (act) {
    case ACT_TANH: return tanh_f(x);
    case ACT_RELU: return fmaxf(x, 0.f);
    // hardware exp/log with a Kahan log1p (~10 VALU, fp32-grade; the libm form cost the CNF walk's
    // 128-wide layer GEMMs ~55 VALU per element in the epilogue).  Softplus only appears in the
    // CNF vector field, whose fused kernel uses the same forms (cnf.hip act_jvp).
    case ACT_SOFTPLUS: return softplus<true>(x);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-x));
    default: return x;
  }
}

// d act / d pre expressed through the post-activation value y (all supported acts allow it)
NAZ_DEV float activate_grad_from_out(int act, float y) {
  switch (act) {
    case ACT_TANH: return 1.f - y * y;
    case ACT_RELU: return y > 0.f ? 1.f : 0.f;
    case ACT_SOFTPLUS: return -Math<true>::expm1(-y);  // sigmoid(pre) = 1 - exp(-softplus(pre))
    case ACT_SIGMOID: return y * (1.f - y);
    default: return 1.f;
  }
}

// act'(pre) and act''(pre) / act'(pre) from h = act(pre) (torch's forms: softplus with beta = 1,
// threshold 20 — above it the identity, act' = 1 - e^-h -> 1 and act''/act' = e^-h -> 0 in fp32)
NAZ_DEV void act_d1_ratio(int act, float h, float& d1, float& r) {
  switch (act) {
    case ACT_SOFTPLUS: d1 = -Math<true>::expm1(-h), r = 1.f - d1; break;  // sigmoid(pre), 1 - sigmoid(pre)
    case ACT_TANH: d1 = 1.f - h * h, r = -2.f * h; break;
    case ACT_RELU: d1 = h > 0.f ? 1.f : 0.f, r = 0.f; break;
    case ACT_SIGMOID: d1 = h * (1.f - h), r = 1.f - 2.f * h; break;
    default: d1 = 1.f, r = 0.f;
  }
}

// Normalised spline tables for one dimension: K+1 knots in x and y, K+1 knot slopes.
template <int K>
struct SplineTables {
  float cw[K + 1];  // x knots
  float ch[K + 1];  // y knots
  float dv[K + 1];  // slopes (edge slopes pinned to 1 - min_derivative)
};

// softmax over K register values, torch order: exp(x - max) then divide by the sum
template <int K, bool FAST = false>
NAZ_DEV void softmax_k(const float* u, float* out) {
  float m = u[0];
#pragma unroll
  for (int k = 1; k < K; ++k) m = fmaxf(m, u[k]);
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    out[k] = Math<FAST>::exp(u[k] - m);
    s += out[k];
  }
  if constexpr (FAST) {
    const float r = Math<true>::rcp(s);
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] = out[k] * r;
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) out[k] = out[k] / s;
  }
}

// [pyro] _calculate_knots applied to softmaxed fractions (min-width blend included)
template <int K>
NAZ_DEV void knots_from_fractions(const float* frac, float minw, float bound, float* knots) {
  const float scale = 1.f - minw * (float)K;
  double acc = 0.0;
  knots[0] = 0.f;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    float wk = __fadd_rn(minw, __fmul_rn(scale, frac[k]));
    acc += (double)wk;
    knots[k + 1] = (float)acc;
  }
  const float two_b = 2.f * bound;
#pragma unroll
  for (int k = 0; k <= K; ++k) knots[k] = __fadd_rn(__fmul_rn(two_b, knots[k]), -bound);
  knots[0] = -bound;
  knots[K] = bound;
}

// Build tables from UNNORMALISED params (uw[K], uh[K], ud[K-1]).
template <int K, bool FAST = false>
NAZ_DEV void build_tables(const float* uw, const float* uh, const float* ud, float bound,
                          SplineTables<K>& t) {
  float f[K];
  softmax_k<K, FAST>(uw, f);
  knots_from_fractions<K>(f, kMinBinWidth, bound, t.cw);
  softmax_k<K, FAST>(uh, f);
  knots_from_fractions<K>(f, kMinBinHeight, bound, t.ch);
  t.dv[0] = 1.f - kMinDerivative;
  t.dv[K] = 1.f - kMinDerivative;
#pragma unroll
  for (int k = 0; k < K - 1; ++k) t.dv[k + 1] = kMinDerivative + softplus<FAST>(ud[k]);
}

// Evaluate the spline (forward or inverse) with the bin quantities selected in registers.
// Returns ld of the map actually applied (inverse map's ld for INV), 0 outside [-B, B].
template <int K, bool INV, bool FAST = false>
NAZ_DEV float rqs_apply(const SplineTables<K>& t, float x, float bound, float& ld) {
  using M = Math<FAST>;
  if (!(x >= -bound && x <= bound)) {  // identity tails (NaN also falls through unchanged)
    ld = 0.f;
    return x;
  }
  // bin search on (knots + eps)
  int cnt = 0;
#pragma unroll
  for (int k = 0; k <= K; ++k) {
    float knot = INV ? t.ch[k] : t.cw[k];
    cnt += (x >= knot + kSearchEps) ? 1 : 0;
  }
  int idx = cnt - 1;
  idx = idx < 0 ? 0 : (idx > K - 1 ? K - 1 : idx);
  float cw0 = t.cw[0], cw1 = t.cw[1], ch0 = t.ch[0], ch1 = t.ch[1], d0 = t.dv[0], d1 = t.dv[1];
#pragma unroll
  for (int k = 1; k < K; ++k) {
    bool s = (idx == k);
    cw0 = s ? t.cw[k] : cw0;
    cw1 = s ? t.cw[k + 1] : cw1;
    ch0 = s ? t.ch[k] : ch0;
    ch1 = s ? t.ch[k + 1] : ch1;
    d0 = s ? t.dv[k] : d0;
    d1 = s ? t.dv[k + 1] : d1;
  }
  const float w = cw1 - cw0;
  const float h = ch1 - ch0;
  const float delta = M::div(h, w);
  const float t1 = (d0 + d1) - 2.f * delta;
  float out, dnum, den;
  if constexpr (INV) {
    const float dy = x - ch0;
    const float a = dy * t1 + h * (delta - d0);
    const float b = h * d0 - dy * t1;
    const float c = -delta * dy;
    const float disc = b * b - 4.f * a * c;
    const float root = M::div(2.f * c, -b - M::sqrt(disc));
    out = root * w + cw0;
    const float tomt = root * (1.f - root);
    den = delta + t1 * tomt;
    const float omr = 1.f - root;
    dnum = delta * delta * (d1 * root * root + 2.f * delta * tomt + d0 * omr * omr);
    ld = -(M::log(dnum) - 2.f * M::log(den));
  } else {
    const float th = M::div(x - cw0, w);
    const float tomt = th * (1.f - th);
    const float num = h * (delta * th * th + d0 * tomt);
    den = delta + t1 * tomt;
    out = ch0 + M::div(num, den);
    const float omt = 1.f - th;
    dnum = delta * delta * (d1 * th * th + 2.f * delta * tomt + d0 * omt * omt);
    ld = M::log(dnum) - 2.f * M::log(den);
  }
  return out;
}

// Rational-quadratic map on one selected bin (cw0, w, ch0, h, d0, d1): forward or inverse,
// with the ld of the map applied.  Shared by the select-first evaluators below.
template <bool INV>
NAZ_DEV float rqs_bin(float x, float cw0, float w, float ch0, float h, float d0, float d1, float& ld) {
  using M = Math<true>;
  const float delta = h * M::rcp(w);
  const float t1 = (d0 + d1) - 2.f * delta;
  if constexpr (INV) {
    const float dy = x - ch0;
    const float a = dy * t1 + h * (delta - d0);
    const float b = h * d0 - dy * t1;
    const float c = -delta * dy;
    const float disc = fmaxf(b * b - 4.f * a * c, 0.f);
    const float root = M::div(2.f * c, -b - M::sqrt(disc));
    const float tomt = root * (1.f - root);
    const float den = delta + t1 * tomt;
    const float omr = 1.f - root;
    const float dnum = delta * delta * (d1 * root * root + 2.f * delta * tomt + d0 * omr * omr);
    ld = -(M::log(dnum) - 2.f * M::log(den));
    return root * w + cw0;
  } else {
    const float th = M::div(x - cw0, w);
    const float tomt = th * (1.f - th);
    const float num = h * (delta * th * th + d0 * tomt);
    const float den = delta + t1 * tomt;
    const float omt = 1.f - th;
    const float dnum = delta * delta * (d1 * th * th + 2.f * delta * tomt + d0 * omt * omt);
    ld = M::log(dnum) - 2.f * M::log(den);
    return ch0 + M::div(num, den);
  }
}

// A wave-uniform float held in an SGPR: gfx950 has no scalar float ALU, so uniform float
// constants otherwise occupy one VGPR each for the whole kernel (and were spilled).
// The empty asm hides how the value was formed, so the combiner cannot push that arithmetic
// back past the readfirstlane (into a VGPR) nor drop the readfirstlane as a no-op.
NAZ_DEV float uniform_f(float v) {
  asm volatile("" : "+v"(v));
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}

// rqs_select's bound-only constants, formed ONCE per kernel (before the layer loop) and held in
// SGPRs.  Formed inside the loop, the compiler hoists their VALU part and holds ~K VGPRs.
template <int K, bool INV>
struct RqsConsts {
  float key[K];  // key[k] = 2B·k·m_s − B + eps: interior search knot k without its softmax term
  float cA;      // 2B·(1 − K·m)
  float ms, mo;  // 2B·m of the searched / other table
  float nb;      // −B
  NAZ_DEV explicit RqsConsts(float bound) {
    const float two_b = 2.f * bound;
    ms = uniform_f(two_b * (INV ? kMinBinHeight : kMinBinWidth));
    mo = uniform_f(two_b * (INV ? kMinBinWidth : kMinBinHeight));
    cA = uniform_f(two_b * (1.f - kMinBinWidth * (float)K));
    nb = uniform_f(-bound);
    key[0] = 0.f;
#pragma unroll
    for (int k = 1; k < K; ++k) key[k] = uniform_f(__builtin_fmaf(ms, (float)k, -bound) + kSearchEps);
  }
};
static_assert(kMinBinWidth == kMinBinHeight, "RqsConsts::cA serves both tables");

// Select-first spline for the fused MFMA kernels: the same map as build_tables<K, true> +
// rqs_apply<K, INV, true> (pyro _monotonic_rational_spline, quadratic), restated so that only
// the selected bin's quantities are formed:
//   * knot k of either table is  2B·(k·m + (1 − K·m)·E_k / E_K) − B  with E_k the prefix sum of
//     the softmax numerators exp(u − max u): ONE fma per knot, no normalised fractions;
//   * only the searched table (y knots for INV, x knots for the forward map) is formed at all
//     K−1 interior knots; bin k = #{interior knots with x ≥ knot + eps} (pyro's
//     clamp(searchsorted − 1, 0, K−1) over the padded knots);
//   * the other table's two knots and the two knot slopes (softplus) are formed only for that bin.
// Knot positions agree with the cumsum form to a few ulp (fp32 prefix sums, fused multiply-add);
// the map is C¹ across knots, so a bin flip at a knot changes y and ld only at rounding level.
// Out-of-box inputs (|x| > B, NaN) pass through with ld = 0, branch-free.  `rc` holds the
// bound-only constants (RqsConsts, built once per kernel).
template <int K, bool INV>
NAZ_DEV float rqs_select(const float* uw, const float* uh, const float* ud, float x, float bound,
                         const RqsConsts<K, INV>& rc, float& ld) {
  constexpr float kL2E = 1.44269504088896341f;
  float Ew[K + 1], Eh[K + 1];
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
      Ew[k + 1] = Ew[k] + __builtin_amdgcn_exp2f(__builtin_fmaf(uw[k], kL2E, -mwl));
      Eh[k + 1] = Eh[k] + __builtin_amdgcn_exp2f(__builtin_fmaf(uh[k], kL2E, -mhl));
    }
  }
  const float Aw = rc.cA * Math<true>::rcp(Ew[K]);
  const float Ah = rc.cA * Math<true>::rcp(Eh[K]);
  const float* Es = INV ? Eh : Ew;  // searched table
  const float* Eo = INV ? Ew : Eh;
  const float As = INV ? Ah : Aw, Ao = INV ? Aw : Ah;
  const float ms = rc.ms, mo = rc.mo;
  float s0 = 0.f, s1 = Es[1], o0 = 0.f, o1 = Eo[1], udl = ud[0], udh = ud[0];
  int idx = 0;
#pragma unroll
  for (int k = 1; k < K; ++k) {
    const float key = __builtin_fmaf(As, Es[k], rc.key[k]);
    const bool s = x >= key;
    s0 = s ? Es[k] : s0;
    s1 = s ? Es[k + 1] : s1;
    o0 = s ? Eo[k] : o0;
    o1 = s ? Eo[k + 1] : o1;
    udl = s ? ud[k - 1] : udl;
    if (k < K - 1) udh = s ? ud[k] : udh;
    idx += s ? 1 : 0;
  }
  const bool first = idx == 0, last = idx == K - 1;
  const float fi = (float)idx;
  const float cs0 = __builtin_fmaf(As, s0, __builtin_fmaf(ms, fi, rc.nb));
  const float cs1 = last ? bound : __builtin_fmaf(As, s1, __builtin_fmaf(ms, fi + 1.f, rc.nb));
  const float co0 = __builtin_fmaf(Ao, o0, __builtin_fmaf(mo, fi, rc.nb));
  const float co1 = last ? bound : __builtin_fmaf(Ao, o1, __builtin_fmaf(mo, fi + 1.f, rc.nb));
  const float d0 = first ? 1.f - kMinDerivative : kMinDerivative + softplus<true>(udl);
  const float d1 = last ? 1.f - kMinDerivative : kMinDerivative + softplus<true>(udh);
  float lb;
  const float y = INV ? rqs_bin<true>(x, co0, co1 - co0, cs0, cs1 - cs0, d0, d1, lb)
                      : rqs_bin<false>(x, cs0, cs1 - cs0, co0, co1 - co0, d0, d1, lb);
  const bool inside = x >= -bound && x <= bound;
  ld = inside ? lb : 0.f;
  return inside ? y : x;
}

// Select-first evaluation from a precomputed table [cw(K+1) | ch(K+1) | dv(K+1)] in LDS (the
// fused kernels' lower spline): K−1 compares against the searched knots, then the bin's six
// values are fetched by a per-lane LDS index instead of being selected in registers.
template <int K, bool INV>
NAZ_DEV float rqs_table(const float* tb, float x, float bound, float& ld) {
  const float* srch = tb + (INV ? (K + 1) : 0);
  int idx = 0;
#pragma unroll
  for (int k = 1; k < K; ++k) idx += (x >= srch[k] + kSearchEps) ? 1 : 0;
  const float cw0 = tb[idx], cw1 = tb[idx + 1];
  const float ch0 = tb[K + 1 + idx], ch1 = tb[K + 2 + idx];
  const float d0 = tb[2 * (K + 1) + idx], d1 = tb[2 * (K + 1) + idx + 1];
  float lb;
  const float y = rqs_bin<INV>(x, cw0, cw1 - cw0, ch0, ch1 - ch0, d0, d1, lb);
  const bool inside = x >= -bound && x <= bound;
  ld = inside ? lb : 0.f;
  return inside ? y : x;
}

}  // namespace naz
