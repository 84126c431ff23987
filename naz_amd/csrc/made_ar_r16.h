// Fused autoregressive-inverse flow: log_prob of a whole naz "nsa" flow (L layers of pyro
// ConditionalSplineAutoregressive over a ConditionalAutoRegressiveNN with two tanh hidden layers)
// in ONE launch.  SURVEY.md §8a rows a4/a6/a8 (naz/flows/transforms.py:165-198, pyro
// SplineAutoregressive._inverse); the §8b `naz_spline_ar_inv` entry.  Included by coupling.hip
// after coupling_r16.h (Frag2, split8_f16, sig_fold, kSigScale, stage_issue, r16_feat, ...).
//
// The reference inverts a layer with D sequential passes of the WHOLE MADE network (pass k makes
// the dim of order k final).  A hidden unit with mask index m ("degree": it reads the context and
// the dims of order < m) has its final value from pass m on, and pyro's hidden degrees
// round(linspace(1, D, H)) - 1 (C > 0; round(linspace(1, D - 1, H)) without context) do not
// depend on the permutation and are non-decreasing in the unit index.  So here, for a 16-row
// wave (lane = batch row l & 15, quarter q = l >> 4, the r16 layout):
//   pass p (order p, dim d_p = perm[p]):
//     * recompute the 16-unit blocks of hidden layer 1 that hold units of degree p (f16x3 MFMA
//       over [ctx | x]; dims of order >= p are still 0 or garbage-free zeros, and units of
//       higher degree in the same block are recomputed in their own pass), activate, and keep
//       them as f16 hi/lo B fragments in registers (the whole layer: H/32 fragments);
//     * the same for hidden layer 2 from layer 1's fragments (k-steps up to unit E[p]);
//     * the 3K-1 spline parameters of dim d_p from layer 2's fragments (2 output blocks);
//     * gather the parameters of the row into every lane of the row (ds_bpermute) and run the
//       select-first inverse spline on x[d_p] (every quarter redundantly: no broadcast after).
//   Masked-out products are exact zeros of the packed image (W ⊙ mask), so the values equal
//   pyro's D full passes; the conditioner work is one triangular network per layer instead of D.
// Weights stream per pass through the coupling kernels' two-slot LDS-DMA ring (one <= 40 KB
// stage per pass, packed on the host by made_ar_pack); x stays in registers in natural dim order
// (the uniform dim index d_p addresses it through M0-relative moves).
#pragma once

namespace naz {

// pyro create_mask hidden index of unit u (numpy/torch round half to even)
constexpr int ar_round_half_even(double v) {
  const double f = static_cast<double>(static_cast<long long>(v));  // v > 0
  const double r = v - f;
  long long i = static_cast<long long>(f);
  if (r > 0.5 || (r == 0.5 && (i & 1))) ++i;
  return static_cast<int>(i);
}

template <int D_, int C_, int H_, int K_>
struct CfgAR {
  static constexpr int D = D_, C = C_, H = H_, K = K_, P = 3 * K - 1;
  static constexpr int HB = H / 16, KSH = H / 32;      // hidden 16-unit blocks, 32-k steps over them
  static constexpr int KC = (C + 31) / 32;             // context k-steps of hidden layer 1
  static constexpr int KI = KC + 1;                    // + one k-step over x (D <= 32)
  static constexpr int NOB = (P + 15) / 16;            // output blocks (params of one dim)
  static constexpr int OT = 2 * kChunk;                // floats per (block, k-step): hi + lo
  static constexpr int deg(int u) {
    if (C > 0) return ar_round_half_even(1.0 + (double)u * (double)(D - 1) / (double)(H - 1)) - 1;
    return ar_round_half_even(1.0 + (double)u * (double)(D - 2) / (double)(H - 1));
  }
  // E(p) = number of hidden units of degree <= p (a prefix: degrees are non-decreasing)
  static constexpr int E(int p) {
    int n = 0;
    for (int u = 0; u < H; ++u) n += deg(u) <= p ? 1 : 0;
    return n;
  }
  static constexpr int Ep(int p) { return p < 0 ? 0 : E(p); }
  // blocks (re)computed in pass p: those holding units of degree p; blo > bhi = none
  static constexpr int blo(int p) { return Ep(p - 1) >> 4; }
  static constexpr int bhi(int p) { return Ep(p) > Ep(p - 1) ? (Ep(p) - 1) >> 4 : blo(p) - 1; }
  static constexpr int nb(int p) { return bhi(p) - blo(p) + 1; }
  static constexpr int kt(int p) { return (Ep(p) + 31) / 32; }  // k-steps over units of degree <= p
  static constexpr int pad(int n) { return (n + 255) / 256 * 256; }
  // stage of pass p: [L1 blocks nb x KI x OT] [L2 blocks nb x kt x OT] [out NOB x kt x OT]
  //                  [bias: L1 blocks nb x 16 | L2 blocks nb x 16 | out NOB x 16]
  static constexpr int off_l2(int p) { return nb(p) * KI * OT; }
  static constexpr int off_out(int p) { return off_l2(p) + nb(p) * kt(p) * OT; }
  static constexpr int off_bias(int p) { return off_out(p) + NOB * kt(p) * OT; }
  static constexpr int stage_floats(int p) { return pad(off_bias(p) + 32 * nb(p) + 16 * NOB); }
  static constexpr int max_stage() {
    int m = 0;
    for (int p = 0; p < D; ++p) m = stage_floats(p) > m ? stage_floats(p) : m;
    return m;
  }
  static constexpr int STG = max_stage();              // stage stride = LDS ring slot (floats)
  // per layer: D stages | perm (D ints)
  static constexpr int PERM_OFF = D * STG;
  static constexpr int LAYER = pad(PERM_OFF + D);
  static_assert(H % 32 == 0 && H <= 256 && D <= 32 && D >= 2, "unsupported fused autoregressive shape");
  static_assert(P <= 16 * NOB && NOB <= 2, "output blocks");
};

// ---------------------------------------------------------------- host packer (made_ar_pack)
// flat per layer (natural layouts, masks already applied): W0m [H][C + D], b0 [H], W1m [H][H],
// b1 [H], W2m [D P][H] (ARN rows p D + i), b2 [D P]; perm[l][p] = dim of order p.
static unsigned short ar_f16_bits(float v) {
  const _Float16 h = (_Float16)v;
  return __builtin_bit_cast(unsigned short, h);
}
static unsigned ar_piece(float v, int piece) {
  const _Float16 hi = (_Float16)v;
  if (piece == 0) return ar_f16_bits(v);
  return ar_f16_bits(v - (float)hi);
}

template <class CF>
static void made_ar_pack_layer(const float* W0, const float* b0, const float* W1, const float* b1, const float* W2,
                               const float* b2, const int* perm, float* out) {
  constexpr int D = CF::D, C = CF::C, H = CF::H, P = CF::P;
  unsigned* ou = reinterpret_cast<unsigned*>(out);
  for (int i = 0; i < CF::LAYER; ++i) out[i] = 0.f;
  // one (block, k-step) fragment image: word (piece, lane, pair) holds slots j = 2 pair, 2 pair + 1
  auto frag = [&](unsigned* dst, auto&& wf) {
    for (int piece = 0; piece < 2; ++piece)
      for (int lane = 0; lane < 64; ++lane)
        for (int pair = 0; pair < 4; ++pair) {
          unsigned w = 0;
          for (int e = 0; e < 2; ++e) w |= ar_piece(wf(lane & 15, lane >> 4, 2 * pair + e), piece) << (16 * e);
          dst[(piece * 64 + lane) * 4 + pair] = w;
        }
  };
  for (int p = 0; p < D; ++p) {
    unsigned* st = ou + p * CF::STG;
    const int dp = perm[p];
    for (int bi = 0; bi < CF::nb(p); ++bi) {
      const int b = CF::blo(p) + bi;
      for (int t = 0; t < CF::KI; ++t)  // hidden layer 1 over [ctx | x]
        frag(st + (bi * CF::KI + t) * CF::OT, [&](int m, int kg, int j) -> float {
          const int u = 16 * b + m;
          if (u >= H) return 0.f;
          const int col = t < CF::KC ? 32 * t + 8 * kg + j : -1;
          if (t < CF::KC) return col < C ? kSigScale * W0[u * (C + D) + col] : 0.f;
          const int d = 8 * kg + j;
          return d < D ? kSigScale * W0[u * (C + D) + C + d] : 0.f;
        });
      for (int t = 0; t < CF::kt(p); ++t)  // hidden layer 2 over layer 1's fragments
        frag(st + CF::off_l2(p) + (bi * CF::kt(p) + t) * CF::OT, [&](int m, int kg, int j) -> float {
          const int u = 16 * b + m, v = r16_feat(t, kg, j);
          return (u < H && v < H) ? -2.f * kSigScale * W1[u * H + v] : 0.f;
        });
    }
    for (int o = 0; o < CF::NOB; ++o)
      for (int t = 0; t < CF::kt(p); ++t)  // the 3K-1 parameters of dim d_p
        frag(st + CF::off_out(p) + (o * CF::kt(p) + t) * CF::OT, [&](int m, int kg, int j) -> float {
          const int pi = 16 * o + m, v = r16_feat(t, kg, j);
          return (pi < P && v < H) ? -2.f * W2[(pi * D + dp) * H + v] : 0.f;
        });
    float* bias = out + p * CF::STG + CF::off_bias(p);
    for (int bi = 0; bi < CF::nb(p); ++bi)
      for (int r = 0; r < 16; ++r) {
        const int u = 16 * (CF::blo(p) + bi) + r;
        bias[16 * bi + r] = u < H ? kSigScale * b0[u] : 0.f;
        bias[16 * (CF::nb(p) + bi) + r] = u < H ? kSigScale * b1[u] : 0.f;
      }
    for (int r = 0; r < 16 * CF::NOB; ++r) bias[32 * CF::nb(p) + r] = r < P ? b2[r * D + dp] : 0.f;
  }
  for (int p = 0; p < D; ++p) reinterpret_cast<int*>(out)[CF::PERM_OFF + p] = perm[p];
}

// ---------------------------------------------------------------- device
// split 4 activated values into the hi / lo halves (words 2 HALF, 2 HALF + 1) of a B fragment
template <int HALF>
NAZ_DEV void ar_split4(Frag2& f, const floatx4& a) {
  u32x4 H = __builtin_bit_cast(u32x4, f.h), Lo = __builtin_bit_cast(u32x4, f.l);
#pragma unroll
  for (int w = 0; w < 2; ++w) {
    const float v0 = sig_fold(a[2 * w]), v1 = sig_fold(a[2 * w + 1]);
    const unsigned hp = pack_f16x2(v0, v1);
    H[2 * HALF + w] = hp;
    Lo[2 * HALF + w] = pack_f16x2(sub_f16_piece<false>(v0, hp), sub_f16_piece<true>(v1, hp));
  }
  f.h = __builtin_bit_cast(half8, H);
  f.l = __builtin_bit_cast(half8, Lo);
}

#ifndef NAZ_AR_WAVES
#define NAZ_AR_WAVES 12
#endif
// waves (16 rows each) per workgroup; one workgroup per CU (the two pass stages take ~84 KB of
// LDS), NAZ_AR_WAVES / 4 waves per SIMD
constexpr int kARWaves = NAZ_AR_WAVES;
#ifndef NAZ_AR_STAGGER
constexpr bool kARStagger = false;
#else
constexpr bool kARStagger = true;
#endif

template <class CF>
__global__ void __launch_bounds__(64 * kARWaves, kARWaves / 4) made_ar_r16_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ out_lp, int64_t B, float bound) {
  constexpr int D = CF::D, K = CF::K, P = CF::P;
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + CF::STG;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  const int64_t row = (int64_t)blockIdx.x * (16 * kARWaves) + wave * 16 + (lane & 15);
  const bool valid = row < B;
  const int64_t crow = valid ? row : 0;

  float v[D];  // the row's values in natural dim order (every quarter holds all of them)
  float logjac = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) v[d] = valid ? x[crow * ldx + d] : 0.f;
  if (low != nullptr) {  // naz bounding_transform (transforms.py:20-23), as the coupling kernel
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float lo = low[d], hi = high[d];
      const float u = (v[d] - lo) / (hi - lo);
      logjac -= logf(u) + log1pf(-u) + logf(hi - lo);
      v[d] = logf(u / (1.f - u));
    }
  }
  // context B fragments: the same for every pass and layer
  Frag2 cf[CF::KC > 0 ? CF::KC : 1];
#pragma unroll
  for (int t = 0; t < CF::KC; ++t) {
    float c8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = 32 * t + 8 * q + j;
      c8[j] = col < CF::C ? ctx[crow * ldc + col] : 0.f;
    }
    cf[t] = split8_f16(c8);
  }

  const RqsConsts<K, true> rc(bound);
  float ldsum = 0.f;
  // Stagger (NAZ_AR_STAGGER, off: measured 8.60 vs 8.24 ms per 2^20 rows): the late half of the
  // workgroup (waves >= NW/2, which share SIMDs with the early half) runs each pass's spline at
  // the head of the NEXT pass interval, before that pass's MFMAs, so that inside an interval one
  // half would be on the matrix pipe while the other is on the vector pipe.  The pending
  // parameters (o3) and dim stay in registers across the barrier.
  const bool late = kARStagger && __builtin_amdgcn_readfirstlane(wave) >= kARWaves / 2;
  floatx4 o3[CF::NOB];
  int pend = -1;  // dim whose parameters o3 holds, not yet applied (late waves)
  auto spline = [&](int dp) {
    // parameter pi sits in block pi >> 4, register pi & 3 of quarter (pi & 15) >> 2
    float uw[K], uh[K], ud[K - 1];
#pragma unroll
    for (int pi = 0; pi < P; ++pi) {
      const float val = __shfl(o3[pi >> 4][pi & 3], (lane & 15) + 16 * ((pi & 15) >> 2));
      if (pi < K) uw[pi] = val;
      else if (pi < 2 * K) uh[pi - K] = val;
      else ud[pi - 2 * K] = val;
    }
    float ld;
    const float y = v[dp];
    v[dp] = rqs_select<K, true>(uw, uh, ud, y, bound, rc, ld);
    ldsum -= ld;
  };
  stage_issue<CF::stage_floats(0), kARWaves>(slot0, packed + (int64_t)(L - 1) * CF::LAYER);
  int g = 0;
  for (int li = 0; li < L; ++li) {
    const int l = L - 1 - li;
    const float* lp = packed + (int64_t)l * CF::LAYER;
    const float* lnext = packed + (int64_t)(l - 1) * CF::LAYER;
    const int* perm = reinterpret_cast<const int*>(lp + CF::PERM_OFF);
    int dps[D];  // dim of order p, wave-uniform (SGPRs)
#pragma unroll
    for (int p = 0; p < D; ++p) dps[p] = __builtin_amdgcn_readfirstlane(perm[p]);
    Frag2 h1[CF::KSH], h2[CF::KSH];  // hidden layers as B fragments; zero = nothing computed yet
#pragma unroll
    for (int t = 0; t < CF::KSH; ++t) {
      h1[t] = Frag2{half8{}, half8{}};
      h2[t] = Frag2{half8{}, half8{}};
    }
    static_for<0, D>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      // pass constants bound to constexpr locals (a constexpr function in a loop bound or argument
      // is not folded reliably: the loops then stay rolled and the fragments go to scratch)
      constexpr int NBP = CF::nb(p), BLO = CF::blo(p), KT = CF::kt(p);
      constexpr int OFF_L2 = CF::off_l2(p), OFF_OUT = CF::off_out(p), OFF_BIAS = CF::off_bias(p);
      constexpr int SF_NEXT = p + 1 < D ? CF::stage_floats(p + 1) : CF::stage_floats(0);
      __syncthreads();  // stage p has landed in slot (g & 1); every wave is done with the other slot
      const float* cur = (g & 1) ? slot1 : slot0;
      float* nxt = (g & 1) ? slot0 : slot1;
      if constexpr (p + 1 < D) {
        stage_issue<SF_NEXT, kARWaves>(nxt, lp + (p + 1) * CF::STG);
      } else {
        if (li + 1 < L) stage_issue<SF_NEXT, kARWaves>(nxt, lnext);
      }
      ++g;
      const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
      auto afrag = [&](int off_floats, int idx) {  // A fragment idx of the region at off_floats
        const int base = (off_floats >> 2) + idx * 128 + lane;
        return Frag2{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      };
      const int dp = dps[p];
      if (late && pend >= 0) spline(pend);  // the previous pass's spline (previous layer's at p = 0)
      const float4* bias4 = reinterpret_cast<const float4*>(cur + OFF_BIAS);
      // ---- hidden layer 1: blocks holding degree-p units, over [ctx | x]
      if constexpr (NBP > 0) {
        Frag2 xf;
        {
          float x8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float s = 0.f;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
              if (8 * qq + j < D) s = q == qq ? v[8 * qq + j] : s;
            x8[j] = s;
          }
          xf = split8_f16(x8);
        }
        static_for<0, NBP>([&](auto bc) {
          constexpr int bi = decltype(bc)::value, b = BLO + bi;
          const float4 bv = bias4[4 * bi + q];
          floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
#pragma unroll
          for (int t = 0; t < CF::KC; ++t) acc = mfma3_16(afrag(0, bi * CF::KI + t), cf[t], acc);
          acc = mfma3_16(afrag(0, bi * CF::KI + CF::KC), xf, acc);
          ar_split4<b & 1>(h1[b >> 1], acc);
        });
        // ---- hidden layer 2: the same blocks, over layer 1's units of degree <= p
        static_for<0, NBP>([&](auto bc) {
          constexpr int bi = decltype(bc)::value, b = BLO + bi;
          const float4 bv = bias4[4 * (NBP + bi) + q];
          floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
#pragma unroll
          for (int t = 0; t < KT; ++t) acc = mfma3_16(afrag(OFF_L2, bi * KT + t), h1[t], acc);
          ar_split4<b & 1>(h2[b >> 1], acc);
        });
      }
      // ---- the 3K-1 raw spline parameters of dim d_p
#pragma unroll
      for (int o = 0; o < CF::NOB; ++o) {
        const float4 bv = bias4[4 * (2 * NBP + o) + q];
        o3[o] = floatx4{bv.x, bv.y, bv.z, bv.w};
      }
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int o = 0; o < CF::NOB; ++o) o3[o] = mfma3_16(afrag(OFF_OUT, o * KT + t), h2[t], o3[o]);
      if (late) pend = dp;
      else spline(dp);
    });
  }
  if (late && pend >= 0) spline(pend);
  constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
  float base = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) base += -(v[d] * v[d]) / 2.f - kLogSqrt2Pi;
  if (q == 0 && valid) out_lp[row] = base - ldsum + logjac;
}

}  // namespace naz
