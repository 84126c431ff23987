// Fused autoregressive-inverse flow: log_prob of a whole naz "nsa" or "maf" flow (L layers of
// pyro ConditionalSplineAutoregressive / ConditionalAffineAutoregressive over a
// ConditionalAutoRegressiveNN with NHID tanh hidden layers) in ONE launch.  SURVEY.md §8a rows
// a4/a5/a6/a8 (naz/flows/transforms.py:133-198, pyro SplineAutoregressive._inverse /
// AffineAutoregressive._inverse); the §8b `naz_spline_ar_inv` / `naz_affine_ar_inv` entries.
// Included by coupling.hip after coupling_r16.h (Frag2, split8_f16, sig_fold, kSigScale,
// stage_issue, r16_feat, ...).
//
// The reference inverts a layer with D sequential passes of the WHOLE MADE network (pass k makes
// the dim of order k final).  A hidden unit with mask index m ("degree": it reads the context and
// the dims of order < m) has its final value from pass m on, and pyro's hidden degrees
// round(linspace(1, D, H)) - 1 (C > 0; round(linspace(1, D - 1, H)) without context) do not
// depend on the permutation and are non-decreasing in the unit index.  So here, for a 16-row
// wave (lane = batch row l & 15, quarter q = l >> 4, the r16 layout):
//   pass p (order p, dim d_p = perm[p]):
//     * recompute the 16-unit blocks of hidden layer 1 that hold units of degree p (f16x3 MFMA
//       over [ctx | x]; dims of order >= p only reach units of higher degree, which are
//       recomputed in their own pass), activate, and keep them as f16 hi/lo B fragments in
//       registers (the whole layer: ceil(H/32) fragments);
//     * the same for every further hidden layer from the previous one's fragments (k-steps up to
//       unit E[p]);
//     * the output rows of dim d_p (3K-1 spline parameters, or (mean, log_scale));
//     * spline: gather the row's parameters into every lane of the row (ds_bpermute) and run the
//       select-first inverse spline on x[d_p]; affine: x[d_p] = (y - mean) exp(-clamp(ls, -5, 3))
//       (every quarter redundantly: no broadcast after).
//   Masked-out products are exact zeros of the packed image (W ⊙ mask), so the values equal
//   pyro's D full passes; the conditioner work is one triangular network per layer instead of D.
// Weights stream through the coupling kernels' two-slot LDS-DMA ring: the per-pass sub-layers
// (hidden layer 1, 2, ..., output) are grouped greedily into stages of at most kARCap floats
// (nsa at H = 128: one stage per pass).  x stays in registers in natural dim order (the uniform
// dim index d_p addresses it through M0-relative moves).
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

constexpr int kARCap = 20480;  // floats per ring slot at most (2 slots = 160 KB, one workgroup per CU)
#ifndef NAZ_AR_INV_NW
#define NAZ_AR_INV_NW 12
#endif
#ifndef NAZ_AR_INV_CAP
#define NAZ_AR_INV_CAP kARCap  // the inverse's per-stage cap (CfgAR::make_layout)
#endif

// The inverse select-first spline of ONE dim per row, spread over the row's four lanes (quarters q
// = lane >> 4 of the 16-row MFMA layout) instead of evaluated four times.  The output blocks of
// the dim's 3K - 1 = 23 parameters leave parameter 16 o + 4 q + i in register i of block o on
// quarter q: widths 0-3 | 4-7 on quarters 0 | 1, heights 0-3 | 4-7 on quarters 2 | 3 (block 0),
// slope parameters 0-3 | 4-6 on quarters 0 | 1 (block 1).  Each quarter forms the softmax
// numerators, prefix sums and knots of ITS half-table (4 exps instead of 16), the bin index is
// counted on the height quarters (the inverse searches the y knots) and shared, and every quarter
// assembles the selected bin's knots and slopes through xor-16 (partner half-table) and xor-32
// (other table) exchanges, then evaluates the bin — the same arithmetic as rqs_select<K, true>
// (same knot formula, prefix sums in the same order), so the map and log-det agree with it to
// the rounding of the split prefix sums.  All four lanes of a row return the same value.
template <int K>
NAZ_DEV float rqs_select_inv_quad(const floatx4& b0, const floatx4& b1, int q, float y, float bound,
                                  const RqsConsts<K, true>& rc, float& ld) {
  static_assert(K == 8, "the quarter layout holds 8 bins: two half-tables of 4 per table");
  constexpr float kL2E = 1.44269504088896341f;
  const int qh = q & 1;          // half-table: knots 1-4 (0) or 5-8 (1)
  const bool hq = q >= 2;        // this quarter holds heights (the searched table)
  // softmax numerators of this half-table, max over the whole table
  float m = fmaxf(fmaxf(b0[0], b0[1]), fmaxf(b0[2], b0[3]));
  m = fmaxf(m, __shfl_xor(m, 16));
  const float ml = m * kL2E;
  // E[i] = cumulative numerator through knot 4 qh + i + 1, summed in rqs_select's order (the
  // upper half-table continues from the lower one's total), so the knots are bit-identical to it
  float e[4], E[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) e[i] = __builtin_amdgcn_exp2f(__builtin_fmaf(b0[i], kL2E, -ml));
  const float lower_total = __shfl_xor(((e[0] + e[1]) + e[2]) + e[3], 16);  // used by the upper half
  {
    float p = qh ? lower_total : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      p = (qh || i > 0) ? p + e[i] : e[i];
      E[i] = p;
    }
  }
  // (every cross-lane read below runs on all lanes, outside any select: a shuffle in a divergent
  // branch reads the inactive source lanes' stale values)
  const float upper_end = __shfl_xor(E[3], 16);
  const float S = qh ? E[3] : upper_end;  // the table's total E_K (the upper half's end)
  const float A = rc.cA * Math<true>::rcp(S);
  // bin index: interior height knots 1..7 with y >= A E_k + key_k (the upper half-table's knot 8 is
  // the box edge, not searched)
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int k = 4 * qh + i + 1;
    const float key = __builtin_fmaf(A, E[i], __builtin_fmaf(rc.ms, (float)k, rc.nb) + kSearchEps);
    cnt += (k < K && y >= key) ? 1 : 0;
  }
  cnt += __shfl_xor(cnt, 16);
  const int cnt_h = __shfl_xor(cnt, 32);
  const int idx = hq ? cnt : cnt_h;  // the height quarters' count, on every quarter
  const bool first = idx == 0, last = idx == K - 1;
  // this table's knots of bin idx: E[idx] and E[idx + 1] (E_0 = 0) from their owner half-table
  auto pick = [&](int n) {  // the table's cumulative numerator through knot n (1 <= n <= 8)
    const int j = (n - 1) & 3;
    const float mine = j == 0 ? E[0] : (j == 1 ? E[1] : (j == 2 ? E[2] : E[3]));
    const float theirs = __shfl_xor(mine, 16);
    return ((n - 1) >> 2) == qh ? mine : theirs;
  };
  const float p0 = pick(first ? 1 : idx), e1 = pick(idx + 1);
  const float e0 = first ? 0.f : p0;
  const float fi = (float)idx;
  const float c0 = __builtin_fmaf(A, e0, __builtin_fmaf(rc.ms, fi, rc.nb));
  const float c1 = last ? bound : __builtin_fmaf(A, e1, __builtin_fmaf(rc.ms, fi + 1.f, rc.nb));
  const float c0o = __shfl_xor(c0, 32), c1o = __shfl_xor(c1, 32);
  const float cs0 = hq ? c0 : c0o, cs1 = hq ? c1 : c1o;  // y (height) knots
  const float co0 = hq ? c0o : c0, co1 = hq ? c1o : c1;  // x (width) knots
  // slope parameters ud[idx - 1], ud[idx] from quarters 0 | 1 (block 1)
  auto pick_ud = [&](int n) {  // 0 <= n <= 6
    const int j = n & 3;
    const float mine = j == 0 ? b1[0] : (j == 1 ? b1[1] : (j == 2 ? b1[2] : b1[3]));
    const float theirs = __shfl_xor(mine, 16);
    const float pair = ((n >> 2) == qh) ? mine : theirs;
    const float v = __shfl_xor(pair, 32);
    return hq ? v : pair;
  };
  const float udl = pick_ud(first ? 0 : idx - 1), udh = pick_ud(last ? 0 : idx);
  const float d0 = first ? 1.f - kMinDerivative : kMinDerivative + softplus<true>(udl);
  const float d1 = last ? 1.f - kMinDerivative : kMinDerivative + softplus<true>(udh);
  float lb;
  const float x = rqs_bin<true>(y, co0, co1 - co0, cs0, cs1 - cs0, d0, d1, lb);
  const bool inside = y >= -bound && y <= bound;
  ld = inside ? lb : 0.f;
  return inside ? x : y;
}

template <int D_, int C_, int H_, int K_, int NHID_ = 2, bool AFFINE_ = false>
struct CfgAR {
  static constexpr int D = D_, C = C_, H = H_, K = K_, NHID = NHID_;
  static constexpr bool AFFINE = AFFINE_;
  static constexpr int P = AFFINE ? 2 : 3 * K - 1;      // ARN outputs per dim
  static constexpr int HP = (H + 31) / 32 * 32;         // padded hidden width
  static constexpr int HB = HP / 16, KSH = HP / 32;     // hidden 16-unit blocks, 32-k steps over them
  static constexpr int KC = (C + 31) / 32;              // context k-steps of hidden layer 1
  static constexpr int KI = KC + 1;                     // + one k-step over x (D <= 32)
  static constexpr int NOB = (P + 15) / 16;             // output blocks (params of one dim)
  static constexpr int OT = 2 * kChunk;                 // floats per (block, k-step): hi + lo
  static constexpr int deg(int u) {
    if (C > 0) return ar_round_half_even(1.0 + (double)u * (double)(D - 1) / (double)(H - 1)) - 1;
    return ar_round_half_even(1.0 + (double)u * (double)(D - 2) / (double)(H - 1));
  }
  static constexpr int pad(int n) { return (n + 255) / 256 * 256; }
  // the per-layer plan, computed once per instantiation (a table: the nested constexpr calls of a
  // direct formulation exceed the compiler's constant-evaluation step limit)
  struct Layout {
    int E[32];         // E[p] = number of hidden units of degree <= p (a prefix: degrees are non-decreasing)
    int sid[32][4];    // stage holding sub-layer i of pass p
    int off[32][4];    // its offset in the stage (floats)
    int sfl[128];      // floats of stage s (padded)
    int nstg, stg;
  };
  static constexpr int E_of(const Layout& y, int p) { return p < 0 ? 0 : y.E[p]; }
  static constexpr int blo_of(const Layout& y, int p) { return E_of(y, p - 1) >> 4; }
  static constexpr int bhi_of(const Layout& y, int p) {
    return E_of(y, p) > E_of(y, p - 1) ? (E_of(y, p) - 1) >> 4 : blo_of(y, p) - 1;
  }
  static constexpr int nb_of(const Layout& y, int p) { return bhi_of(y, p) - blo_of(y, p) + 1; }
  static constexpr int kt_of(const Layout& y, int p) { return (E_of(y, p) + 31) / 32; }
  // sub-layer i of pass p: 0 = hidden layer 1 over [ctx | x], 1 .. NHID-1 = hidden layer i + 1,
  // NHID = output rows; image: [fragments (block, k-step)] [bias: 16 per block]
  static constexpr int frags_of(const Layout& y, int p, int i) {
    return i == 0 ? nb_of(y, p) * KI : (i < NHID ? nb_of(y, p) * kt_of(y, p) : NOB * kt_of(y, p));
  }
  static constexpr int sub_floats_of(const Layout& y, int p, int i) {
    return frags_of(y, p, i) * OT + 16 * (i < NHID ? nb_of(y, p) : NOB);
  }
  static constexpr Layout make_layout() {
    Layout y{};
    int cnt[32] = {};
    for (int u = 0; u < H; ++u) ++cnt[deg(u) < 0 ? 0 : deg(u)];
    for (int p = 0, run = 0; p < D; ++p) y.E[p] = run += cnt[p];
    // greedy grouping of each pass's sub-layers into stages of <= kARCap floats
    int s = -1;
    for (int p = 0; p < D; ++p) {
      int run = 0;
      for (int i = 0; i <= NHID; ++i) {
        const int sz = sub_floats_of(y, p, i);
        if (i == 0 || run + sz > NAZ_AR_INV_CAP) {
          ++s;
          run = 0;
        }
        y.sid[p][i] = s;
        y.off[p][i] = run;
        run += sz;
        y.sfl[s] = pad(run);
      }
    }
    y.nstg = s + 1;
    for (int t = 0; t < y.nstg; ++t) y.stg = y.sfl[t] > y.stg ? y.sfl[t] : y.stg;
    return y;
  }
  static constexpr Layout LY = make_layout();
  static constexpr int E(int p) { return E_of(LY, p); }
  static constexpr int blo(int p) { return blo_of(LY, p); }  // blocks (re)computed in pass p: those
  static constexpr int bhi(int p) { return bhi_of(LY, p); }  // holding units of degree p; none if blo > bhi
  static constexpr int nb(int p) { return nb_of(LY, p); }
  static constexpr int kt(int p) { return kt_of(LY, p); }    // k-steps over units of degree <= p
  static constexpr int frags(int p, int i) { return frags_of(LY, p, i); }
  static constexpr int stage_id(int p, int i) { return LY.sid[p][i]; }
  static constexpr int sub_off(int p, int i) { return LY.off[p][i]; }
  static constexpr int stage_floats(int s) { return LY.sfl[s]; }
  static constexpr int NSTG = LY.nstg;
  static constexpr int STG = LY.stg;                  // stage stride = LDS ring slot (floats)
  // per layer: NSTG stages | perm (D ints)
  static constexpr int PERM_OFF = NSTG * STG;
  // pass-0 constants per layer (one context vector): NHID x nb(0) blocks of 16 kSigScale-scaled
  // pre-activations, then NOB blocks of 16 output values of the first dim in order
  static constexpr int C0 = 16 * (NHID * nb_of(LY, 0) + NOB);
  // in a pass-0-constant image the constants of pass 0's sub-layer i sit compactly at c0_off(i) of
  // its stage (pass 0's stages hold nothing else), so those stages stream only c0_chunks(s) KB
  static constexpr int c0_cnt(int i) { return 16 * (i < NHID ? nb_of(LY, 0) : NOB); }
  static constexpr int c0_off(int i) {
    int o = 0;
    for (int j = 0; j < i; ++j)
      if (LY.sid[0][j] == LY.sid[0][i]) o += c0_cnt(j);
    return o;
  }
  static constexpr int c0_chunks(int s) {
    if (s > LY.sid[0][NHID]) return LY.sfl[s] / 256;
    int e = 0;
    for (int i = 0; i <= NHID; ++i)
      if (LY.sid[0][i] == s && c0_off(i) + c0_cnt(i) > e) e = c0_off(i) + c0_cnt(i);
    return (e + 255) / 256;
  }
  static constexpr int LAYER = pad(PERM_OFF + D);
  // waves per SIMD the inverse kernel is compiled for: 3 when the live set fits 168 VGPRs; the
  // forward kernel's workgroup (CfgARF) keeps one workgroup per CU of 4 x WPE waves
  static constexpr int WPE = NHID * KSH <= 8 ? 3 : 2;
  static constexpr int NW_FWD = 4 * WPE;
  // inverse workgroup: NAZ_AR_INV_NW waves (12: one workgroup per CU; 6 with NAZ_AR_INV_CAP =
  // 10240: two per CU, each on its own 2 x <= 40 KB ring, so the two do not share barriers)
  static constexpr int NW = WPE == 3 ? NAZ_AR_INV_NW : NW_FWD;
  // the inverse kernel's waves per SIMD (NAZ_AR_INV_WPE overrides: e.g. 2 with NAZ_AR_INV_NW = 8)
  // and its prefetched MFMA chains (NAZ_AR_INV_PF: mfma3_16_chain_lds)
#ifdef NAZ_AR_INV_WPE
  static constexpr int WPE_INV = WPE == 3 ? NAZ_AR_INV_WPE : WPE;
#else
  static constexpr int WPE_INV = WPE;
#endif
#ifdef NAZ_AR_INV_PF
  static constexpr bool PF = true;
#else
  static constexpr bool PF = false;
#endif
  static_assert(H <= 256 && D <= 32 && D >= 2 && NHID >= 1 && NHID <= 3, "unsupported fused autoregressive shape");
  static_assert(NOB <= 2 && NSTG <= 128, "output blocks / stages");
};

// acc += sum over t < N of (A fragment t at LDS byte address ub + 2048 t, hi | lo 1 KB apart) x
// bset[t] on the f16x3 16-row MFMA.  Fragment t + 1 is read while fragment t's MFMAs run (untracked
// reads with a counted wait, coupling.hip's lds_read_b128_untracked): for the one-wave-per-SIMD
// wide MADE kernels, which have no other wave to hide an LDS read behind.
template <int N, class BS>
NAZ_DEV floatx4 mfma3_16_chain_lds(unsigned ub, const BS& bset, floatx4 acc) {
  auto rd = [&](auto tc) {
    constexpr int o = 2048 * decltype(tc)::value;
    return Frag2{__builtin_bit_cast(half8, lds_read_b128_untracked<o>(ub)),
                 __builtin_bit_cast(half8, lds_read_b128_untracked<o + 1024>(ub))};
  };
  Frag2 an = rd(std::integral_constant<int, 0>{});
  static_for<0, N>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    const Frag2 a = an;
    if constexpr (t + 1 < N) {
      an = rd(std::integral_constant<int, t + 1>{});
      __builtin_amdgcn_sched_barrier(0);
      lds_wait<2>();
    } else {
      __builtin_amdgcn_sched_barrier(0);
      lds_wait<0>();
    }
    __builtin_amdgcn_sched_barrier(0);
    acc = mfma3_16(a, bset[t], acc);
  });
  return acc;
}

// ---------------------------------------------------------------- host packer (ar_flow_pack)
// flat per layer (natural layouts, masks already applied): W0m [H][C + D], b0 [H],
// {Wim [H][H], bi [H]} for hidden layers 2 .. NHID, Woutm [D P][H] (ARN rows p D + i), bout [D P];
// perm[l][p] = dim of order p.
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
static void made_ar_pack_layer(const float* flat, const int* perm, float* out) {
  constexpr int D = CF::D, C = CF::C, H = CF::H, P = CF::P;
  const float* Wl[CF::NHID + 1];
  const float* bl[CF::NHID + 1];
  {
    const float* f = flat;
    for (int i = 0; i <= CF::NHID; ++i) {
      const int rows = i < CF::NHID ? H : D * P, cols = i == 0 ? C + D : H;
      Wl[i] = f;
      bl[i] = f + rows * cols;
      f += rows * cols + rows;
    }
  }
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
    const int dp = perm[p];
    for (int i = 0; i <= CF::NHID; ++i) {
      const int base = CF::stage_id(p, i) * CF::STG + CF::sub_off(p, i);
      unsigned* st = ou + base;
      float* bias = out + base + CF::frags(p, i) * CF::OT;
      if (i < CF::NHID) {
        const int kts = i == 0 ? CF::KI : CF::kt(p);
        for (int bi = 0; bi < CF::nb(p); ++bi) {
          const int b = CF::blo(p) + bi;
          for (int t = 0; t < kts; ++t)
            frag(st + (bi * kts + t) * CF::OT, [&](int m, int kg, int j) -> float {
              const int u = 16 * b + m;
              if (u >= H) return 0.f;
              if (i > 0) {  // over the previous hidden layer's fragments
                const int v = r16_feat(t, kg, j);
                return v < H ? -2.f * kSigScale * Wl[i][u * H + v] : 0.f;
              }
              if (t < CF::KC) {
                const int col = 32 * t + 8 * kg + j;
                return col < C ? kSigScale * Wl[0][u * (C + D) + col] : 0.f;
              }
              const int d = 8 * kg + j;
              return d < D ? kSigScale * Wl[0][u * (C + D) + C + d] : 0.f;
            });
          for (int r = 0; r < 16; ++r) {
            const int u = 16 * b + r;
            bias[16 * bi + r] = u < H ? kSigScale * bl[i][u] : 0.f;
          }
        }
      } else {
        for (int o = 0; o < CF::NOB; ++o)
          for (int t = 0; t < CF::kt(p); ++t)  // the output rows of dim d_p
            frag(st + (o * CF::kt(p) + t) * CF::OT, [&](int m, int kg, int j) -> float {
              const int pi = 16 * o + m, v = r16_feat(t, kg, j);
              return (pi < P && v < H) ? -2.f * Wl[CF::NHID][(pi * D + dp) * H + v] : 0.f;
            });
        for (int r = 0; r < 16 * CF::NOB; ++r) bias[r] = r < P ? bl[CF::NHID][r * D + dp] : 0.f;
      }
    }
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

template <class CF>
__global__ void __launch_bounds__(64 * CF::NW, CF::WPE_INV) made_ar_r16_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ out_lp, int64_t B, float bound, int64_t spk = 0, int64_t sx = 0, int64_t slp = 0,
    int c0mode = 0, float* __restrict__ states = nullptr) {
  constexpr int D = CF::D, K = CF::K, P = CF::P, NW = CF::NW, NHID = CF::NHID;
  {  // blockIdx.y = draw (naz_ar_flow_log_prob_batched): image packed + draw spk, rows x + draw sx
    const int64_t dz = blockIdx.y;
    packed += dz * spk;
    x += dz * sx;
    out_lp += dz * slp;
  }
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + CF::STG;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  const int64_t row = (int64_t)blockIdx.x * (16 * NW) + wave * 16 + (lane & 15);
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
  float ldsum = 0.f;  // the layers' forward log-dets (log p = base - ldsum + logjac)
  const int ch0 = c0mode ? CF::c0_chunks(0) : CF::stage_floats(0) / 256;  // stage 0's KB to stream
  stage_issue_lim<CF::stage_floats(0), NW>(slot0, packed + (int64_t)(L - 1) * CF::LAYER, ch0);
  int g = 0;
  for (int li = 0; li < L; ++li) {
    const int l = L - 1 - li;
    const float* lp = packed + (int64_t)l * CF::LAYER;
    const float* lnext = packed + (int64_t)(l - 1) * CF::LAYER;
    const int* perm = reinterpret_cast<const int*>(lp + CF::PERM_OFF);
    int dps[D];  // dim of order p, wave-uniform (SGPRs)
#pragma unroll
    for (int p = 0; p < D; ++p) dps[p] = __builtin_amdgcn_readfirstlane(perm[p]);
    Frag2 hf[NHID][CF::KSH];  // hidden layers as B fragments; zero = nothing computed yet
#pragma unroll
    for (int i = 0; i < NHID; ++i)
#pragma unroll
      for (int t = 0; t < CF::KSH; ++t) hf[i][t] = Frag2{half8{}, half8{}};
    float xmax = 0.f;
    if constexpr (CF::AFFINE) {
#pragma unroll
      for (int d = 0; d < D; ++d) xmax = fmaxf(xmax, fabsf(v[d]));
    }
    const float* cur = slot0;
    static_for<0, D>([&](auto pc) {
      constexpr int p = decltype(pc)::value;
      // pass constants bound to constexpr locals (a constexpr function in a loop bound or argument
      // is not folded reliably: the loops then stay rolled and the fragments go to scratch)
      constexpr int NBP = CF::nb(p), BLO = CF::blo(p), KT = CF::kt(p);
      const int dp = dps[p];
      floatx4 o3[CF::NOB];
      static_for<0, NHID + 1>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        constexpr int SID = CF::stage_id(p, i), OFF = CF::sub_off(p, i);
        constexpr int OFF_BIAS = OFF + CF::frags(p, i) * CF::OT;
        // a stage starts at sub-layer 0 of every pass and wherever the grouping opened a new one
        // (not at OFF == 0: empty sub-layers — no units of degree p, e.g. pass 0 without a
        // context — also sit at offset 0 of their pass's stage)
        constexpr bool NEW_STAGE = i == 0 || SID != CF::stage_id(p, i > 0 ? i - 1 : 0);
        if constexpr (NEW_STAGE) {  // it has landed in slot (g & 1)
          constexpr int SF_NEXT = SID + 1 < CF::NSTG ? CF::stage_floats(SID + 1) : CF::stage_floats(0);
          ring_barrier();  // ... and every wave is done with the other slot
          cur = (g & 1) ? slot1 : slot0;
          float* nxt = (g & 1) ? slot0 : slot1;
          if constexpr (SID + 1 < CF::NSTG) {
            stage_issue_lim<SF_NEXT, NW>(nxt, lp + (SID + 1) * CF::STG,
                                         c0mode ? CF::c0_chunks(SID + 1) : SF_NEXT / 256);
          } else {
            if (li + 1 < L) stage_issue_lim<SF_NEXT, NW>(nxt, lnext, ch0);
          }
          ++g;
        }
        const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
        auto afrag = [&](int idx) {  // A fragment idx of this sub-layer
          const int base = (OFF >> 2) + idx * 128 + lane;
          return Frag2{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
        };
        [[maybe_unused]] const unsigned ub = (unsigned)(uintptr_t)to_lds(cur) + 16u * lane + 4u * OFF;
        const float4* bias4 = reinterpret_cast<const float4*>(cur + OFF_BIAS);
        bool done0 = false;
        if constexpr (p == 0) {
          if (c0mode) {
            // one context vector (naz_ar_flow_pack with pass0): the degree-0 units and the first
            // dim's parameters are per-draw constants, written by the packer in place of this
            // pass's fragments (kSigScale-scaled pre-activations / output values, 16 per block)
            const float4* cv = reinterpret_cast<const float4*>(cur + CF::c0_off(i));
            if constexpr (i < NHID) {
              static_for<0, NBP>([&](auto bc) {
                constexpr int bi = decltype(bc)::value, b = BLO + bi;
                const float4 c = cv[4 * bi + q];
                ar_split4<b & 1>(hf[i][b >> 1], floatx4{c.x, c.y, c.z, c.w});
              });
            } else {
#pragma unroll
              for (int o = 0; o < CF::NOB; ++o) {
                const float4 c = cv[4 * o + q];
                o3[o] = floatx4{c.x, c.y, c.z, c.w};
              }
            }
            done0 = true;
          }
        }
        if constexpr (i == 0 && NBP > 0) {
         if (!done0) {
          // ---- hidden layer 1: blocks holding degree-p units, over [ctx | x]
          // the row's values (inverted dims and still-pending ones alike: a masked weight times an
          // f16 overflow would be NaN) split at a per-row power-of-two scale, |x| sc < 2^14: the
          // inverse maps can grow values (maf: e^5 per layer) past the launch-time input check
          // (xmax: a running bound, max |v| at the layer's start and every value written since).
          // Affine flows only: a spline maps [-B, B] into itself and is the identity outside, so an
          // nsa row never exceeds max(|input|, B) and the launch-time input check covers it.
          int e = 0;
          if constexpr (CF::AFFINE) e = xmax >= 16384.f ? __builtin_amdgcn_frexp_expf(xmax) - 14 : 0;
          const float sc = __builtin_amdgcn_ldexpf(1.f, -e), us = __builtin_amdgcn_ldexpf(1.f, e);
          float x8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float s = 0.f;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
              if (8 * qq + j < D) s = q == qq ? v[8 * qq + j] : s;
            x8[j] = s * sc;
          }
          const Frag2 xf = split8_f16(x8);
          static_for<0, NBP>([&](auto bc) {
            constexpr int bi = decltype(bc)::value, b = BLO + bi;
            const float4 bv = bias4[4 * bi + q];
            floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
#pragma unroll
            for (int t = 0; t < CF::KC; ++t) acc = mfma3_16(afrag(bi * CF::KI + t), cf[t], acc);
            if constexpr (CF::AFFINE) {
              const floatx4 ax = mfma3_16(afrag(bi * CF::KI + CF::KC), xf, floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
              for (int r = 0; r < 4; ++r) acc[r] = __builtin_fmaf(ax[r], us, acc[r]);
            } else {
              acc = mfma3_16(afrag(bi * CF::KI + CF::KC), xf, acc);
            }
            ar_split4<b & 1>(hf[0][b >> 1], acc);
          });
         }
        } else if constexpr (i > 0 && i < NHID && NBP > 0) {
          // ---- hidden layer i + 1: the same blocks, over layer i's units of degree <= p
          if (!done0) static_for<0, NBP>([&](auto bc) {
            constexpr int bi = decltype(bc)::value, b = BLO + bi;
            const float4 bv = bias4[4 * bi + q];
            floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
            if constexpr (CF::PF) {
              acc = mfma3_16_chain_lds<KT>(ub + 2048u * (bi * KT), hf[i - 1], acc);
            } else {
#pragma unroll
              for (int t = 0; t < KT; ++t) acc = mfma3_16(afrag(bi * KT + t), hf[i - 1][t], acc);
            }
            ar_split4<b & 1>(hf[i][b >> 1], acc);
          });
        } else if constexpr (i == NHID) {
          // ---- the output rows of dim d_p, then the elementwise inverse on x[d_p]
          if (!done0) {
#pragma unroll
            for (int o = 0; o < CF::NOB; ++o) {
              const float4 bv = bias4[4 * o + q];
              o3[o] = floatx4{bv.x, bv.y, bv.z, bv.w};
            }
            if constexpr (CF::PF) {
#pragma unroll
              for (int o = 0; o < CF::NOB; ++o) o3[o] = mfma3_16_chain_lds<KT>(ub + 2048u * (o * KT), hf[NHID - 1], o3[o]);
            } else {
#pragma unroll
              for (int t = 0; t < KT; ++t)
#pragma unroll
                for (int o = 0; o < CF::NOB; ++o) o3[o] = mfma3_16(afrag(o * KT + t), hf[NHID - 1][t], o3[o]);
            }
          }
          const float y = v[dp];
          if constexpr (CF::AFFINE) {
            // pyro AffineAutoregressive._inverse: rows 0, 1 = (mean, log_scale) of dim d_p, held by
            // quarter 0 registers 0, 1; log_scale clamped to [-5, 3]; log|det| = the clamped ls
            const float mean = __shfl(o3[0][0], lane & 15);
            const float ls = fminf(fmaxf(__shfl(o3[0][1], lane & 15), -5.f), 3.f);
            v[dp] = (y - mean) * __expf(-ls);
            xmax = fmaxf(xmax, fabsf(v[dp]));
            ldsum += ls;
          } else {
#ifndef NAZ_AR_SPLINE_GATHER
            // one spline per row spread over its four quarters (rqs_select_inv_quad)
            float ld;
            v[dp] = rqs_select_inv_quad<K>(o3[0], o3[CF::NOB > 1 ? 1 : 0], q, y, bound, rc, ld);
            ldsum -= ld;
#else
            // (A/B) every quarter gathers the row's parameters and evaluates the whole spline:
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
            v[dp] = rqs_select<K, true>(uw, uh, ud, y, bound, rc, ld);
            ldsum -= ld;
#endif
          }
        }
      });
    });
    // the training forward (naz_ar_flow_log_prob_train, one draw): layer l's output s_l for the
    // backward (made_ar_bwd.h)
    if (states != nullptr && q == 0 && valid) {
      // (row re-formed at the store from an opaque thread index: a 64-bit per-lane address held across
      // the layer loop is what the nsa16 instance spilled)
      unsigned tid = threadIdx.x;
      asm volatile("" : "+v"(tid));
      const int64_t r2 = (int64_t)blockIdx.x * (16 * NW) + (tid >> 6) * 16 + (tid & 15);
      float* const sp = states + ((int64_t)l * B + r2) * D;
#pragma unroll
      for (int d = 0; d < D; ++d) sp[d] = v[d];
    }
  }
  constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
  float base = 0.f;
#pragma unroll
  for (int d = 0; d < D; ++d) base += -(v[d] * v[d]) / 2.f - kLogSqrt2Pi;
  if (q == 0 && valid) {
    unsigned tid = threadIdx.x;
    asm volatile("" : "+v"(tid));
    out_lp[(int64_t)blockIdx.x * (16 * NW) + (tid >> 6) * 16 + (tid & 15)] = base - ldsum + logjac;
  }
}

// ================================================================ forward (sample) direction
// pyro ConditionedSplineAutoregressive._call / AffineAutoregressive._call (naz transforms.py:
// 133-198), the sampling direction of TransformedDistribution.sample (flow.py:94-129): ONE MADE pass
// per layer over the layer input, then every dim's map — y_d = spline(x_d) or x_d exp(ls_d) + m_d —
// all of a layer's dims from the same hidden activations (no sequential dependence: the masks
// already encode the order).  The whole flow is one launch: per layer, all hidden blocks (f16x3
// MFMA, register-resident B fragments, the inverse kernel's machinery), then per group of four
// dims their output rows and the elementwise maps (one dim per row quarter).  Weights: per layer
// "units" — (hidden layer i, 16-unit block b) with its k-steps and bias, then (dim group g) with
// its output blocks — grouped greedily into LDS-ring stages of <= kARCap floats.  Forward values can grow through the layers (affine scales up to
// e^3 per layer), so the layer input is split into f16 pieces at a per-row power-of-two scale and
// the x part of hidden layer 1 rescaled in fp32 (the context keeps the caller's |ctx| < 2^15).
// Wide affine MADE (naz's production MAFs: the 4-parameter MLE flow D=4 | C=2, H=[512]x5, L=18,
// examples/papers/2506.05657/train_mle_all_data_4param.py:87-92; POSYDON D=4, 512x5, L=16,
// eposydon/train_maf_mle.py:84-90), forward (sample) direction only: CfgARF over this gives
// made_ar_fwd_kernel's per-layer image and schedule.  Two hidden layers of B fragments are 256
// VGPRs at H = 512, so one 4-wave workgroup per CU (one wave per SIMD, AGPRs in use) with 64
// rows per weight stream; each ring stage carries two 16-unit blocks (2 x 32 KB of f16 pieces).
template <int D_, int C_, int H_, int NHID_>
struct CfgARW {
  static constexpr int D = D_, C = C_, H = H_, K = 8, NHID = NHID_;
  static constexpr bool AFFINE = true;
  static constexpr int P = 2, HP = (H + 31) / 32 * 32, HB = HP / 16, KSH = HP / 32;
  static constexpr int KC = (C + 31) / 32, KI = KC + 1, NOB = 1, OT = 2 * kChunk;
  static constexpr int deg(int u) {
    if (C > 0) return ar_round_half_even(1.0 + (double)u * (double)(D - 1) / (double)(H - 1)) - 1;
    return ar_round_half_even(1.0 + (double)u * (double)(D - 2) / (double)(H - 1));
  }
  static constexpr int pad(int n) { return (n + 255) / 256 * 256; }
  static constexpr int NW = 4, NW_FWD = 4;
  static_assert(H > 256 && H % 32 == 0 && D >= 2 && D <= 8 && NHID >= 1, "wide MADE instances only");
};

template <class G>
struct CfgARF {
  static constexpr int D = G::D, C = G::C, H = G::H, K = G::K, NHID = G::NHID, P = G::P;
  static constexpr int HB = G::HB, KSH = G::KSH, KC = G::KC, KI = G::KI, OT = G::OT;
  // output units: dims in groups of four, one per row quarter — output row 4 q + i of block o is
  // parameter 4 o + i of dim 4 g + q, so every lane receives ITS dim's parameters in its own
  // accumulator registers and runs one dim's map (no gather, no 4x redundant spline)
  static constexpr int NG = (D + 3) / 4, NOG = (P + 3) / 4;
  // the forward spline's live set at D = 16 exceeds the 168 VGPRs of 12-wave workgroups (spilled
  // 352-468 B/lane): 8 waves (2 per SIMD) there
  static constexpr int NW = (G::AFFINE || D <= 8) ? G::NW_FWD : 8;
  static constexpr bool AFFINE = G::AFFINE;
  static constexpr int NU = NHID * HB + NG;  // units: hidden (i, b) row-major, then one per dim group
  static constexpr int unit_blocks(int u) { return u < NHID * HB ? 1 : NOG; }
  // k-steps a hidden block b of layers 2.. reads: the units of degree <= the block's largest. The
  // MADE mask of a hidden layer is deg(u) >= deg(v) and degrees do not decrease along the unit
  // index, so every later k-step of the block is masked to exact zeros (about a third of each
  // hidden matrix at D = 4, H = 512): neither streamed nor multiplied — the same values, bit for
  // bit (adding +0 products changes no fp32 sum)
  struct KtTab {
    int kt[64];
  };
  static constexpr KtTab make_kt() {
    KtTab y{};
    for (int b = 0; b < HB; ++b) {
      const int last = 16 * b + 15 < H ? 16 * b + 15 : H - 1;
      const int dmax = G::deg(last);
      int e = 0;
      for (int v = 0; v < H; ++v) e += G::deg(v) <= dmax ? 1 : 0;
      y.kt[b] = (e + 31) / 32;
    }
    return y;
  }
  static constexpr KtTab KTT = make_kt();
#ifdef NAZ_AR_FWD_DENSE_K  // (A/B: every hidden block reads all KSH k-steps)
  static constexpr int hid_kts(int) { return KSH; }
#else
  static constexpr int hid_kts(int b) { return KTT.kt[b]; }
#endif
  static constexpr int unit_kts(int u) { return u < HB ? KI : (u < NHID * HB ? hid_kts(u % HB) : KSH); }
  static constexpr int unit_floats(int u) { return unit_blocks(u) * (unit_kts(u) * OT + 16); }
  struct Layout {
    int sid[NU], off[NU], sfl[NU];
    int nstg, stg;
  };
  static constexpr Layout make_layout() {
    Layout y{};
    int s = -1, run = 0;
    for (int u = 0; u < NU; ++u) {
      const int sz = unit_floats(u);
      if (u == 0 || run + sz > kARCap) {
        ++s;
        run = 0;
      }
      y.sid[u] = s;
      y.off[u] = run;
      run += sz;
      y.sfl[s] = G::pad(run);
    }
    y.nstg = s + 1;
    for (int t = 0; t < y.nstg; ++t) y.stg = y.sfl[t] > y.stg ? y.sfl[t] : y.stg;
    return y;
  }
  static constexpr Layout LY = make_layout();
  static constexpr int stage_id(int u) { return LY.sid[u]; }
  static constexpr int unit_off(int u) { return LY.off[u]; }
  static constexpr int stage_floats(int s) { return LY.sfl[s]; }
  static constexpr int NSTG = LY.nstg, STG = LY.stg;
  static constexpr int LAYER = G::pad(NSTG * STG);
  static_assert(2 * STG * 4 <= 160 * 1024, "two forward weight stages exceed the LDS");
};

// host packer of one layer's forward image (flat as made_ar_pack_layer's, masks applied)
template <class CF>
static void made_ar_pack_fwd_layer(const float* flat, float* out) {
  constexpr int D = CF::D, C = CF::C, H = CF::H, P = CF::P, HB = CF::HB, KSH = CF::KSH;
  const float* Wl[CF::NHID + 1];
  const float* bl[CF::NHID + 1];
  {
    const float* f = flat;
    for (int i = 0; i <= CF::NHID; ++i) {
      const int rows = i < CF::NHID ? H : D * P, cols = i == 0 ? C + D : H;
      Wl[i] = f;
      bl[i] = f + rows * cols;
      f += rows * cols + rows;
    }
  }
  unsigned* ou = reinterpret_cast<unsigned*>(out);
  for (int i = 0; i < CF::LAYER; ++i) out[i] = 0.f;
  auto frag = [&](unsigned* dst, auto&& wf) {  // as made_ar_pack_layer's
    for (int piece = 0; piece < 2; ++piece)
      for (int lane = 0; lane < 64; ++lane)
        for (int pair = 0; pair < 4; ++pair) {
          unsigned w = 0;
          for (int e = 0; e < 2; ++e) w |= ar_piece(wf(lane & 15, lane >> 4, 2 * pair + e), piece) << (16 * e);
          dst[(piece * 64 + lane) * 4 + pair] = w;
        }
  };
  for (int u = 0; u < CF::NU; ++u) {
    const int base = CF::stage_id(u) * CF::STG + CF::unit_off(u);
    unsigned* st = ou + base;
    if (u < CF::NHID * HB) {
      const int i = u / HB, b = u % HB, kts = CF::unit_kts(u);
      for (int t = 0; t < kts; ++t)
        frag(st + t * CF::OT, [&](int m, int kg, int j) -> float {
          const int un = 16 * b + m;
          if (un >= H) return 0.f;
          if (i > 0) {
            const int v = r16_feat(t, kg, j);
            return v < H ? -2.f * kSigScale * Wl[i][un * H + v] : 0.f;
          }
          if (t < CF::KC) {
            const int col = 32 * t + 8 * kg + j;
            return col < C ? kSigScale * Wl[0][un * (C + D) + col] : 0.f;
          }
          const int d = 8 * kg + j;
          return d < D ? kSigScale * Wl[0][un * (C + D) + C + d] : 0.f;
        });
      float* bias = out + base + kts * CF::OT;
      for (int r = 0; r < 16; ++r) bias[r] = 16 * b + r < H ? kSigScale * bl[i][16 * b + r] : 0.f;
    } else {
      const int g = u - CF::NHID * HB;  // dims 4 g + q, quarter q: row 4 q + i = parameter 4 o + i
      for (int o = 0; o < CF::NOG; ++o)
        for (int t = 0; t < KSH; ++t)
          frag(st + (o * KSH + t) * CF::OT, [&](int m, int kg, int j) -> float {
            const int d = 4 * g + (m >> 2), pi = 4 * o + (m & 3), v = r16_feat(t, kg, j);
            return (d < D && pi < P && v < H) ? -2.f * Wl[CF::NHID][(pi * D + d) * H + v] : 0.f;
          });
      float* bias = out + base + CF::NOG * KSH * CF::OT;
      for (int o = 0; o < CF::NOG; ++o)
        for (int m = 0; m < 16; ++m) {
          const int d = 4 * g + (m >> 2), pi = 4 * o + (m & 3);
          bias[16 * o + m] = (d < D && pi < P) ? bl[CF::NHID][pi * D + d] : 0.f;
        }
    }
  }
}

// Device form of made_ar_pack_fwd_layer (the Bayesian sampler packs every weight draw on the GPU):
// thread = one 32-bit word of one layer image; blockIdx.y = layer, blockIdx.z = draw.  flat rows at
// flat + draw * sflat (L layers of the made_ar_pack_fwd_layer flat layout, masks applied), images
// at packed + draw * spk.
// f16 code of v, round-to-nearest-even also below 2^-14, where v_cvt_f16_f32 was measured to round
// the lo pieces of f16-split weights 1 code off the host packer's conversion: there the code is
// rint(|v| 2^24) (exact scaling, v_rndne_f32; 1024 carries into the smallest normal)
NAZ_DEV unsigned ar_f16_rne_dev(float v) {
  const float a = fabsf(v);
  if (a < 6.103515625e-05f)
    return (unsigned)__builtin_rintf(a * 16777216.f) | ((__builtin_bit_cast(unsigned, v) >> 16) & 0x8000u);
  return (unsigned)__builtin_bit_cast(unsigned short, (_Float16)v);
}
NAZ_DEV unsigned ar_piece_dev(float v, int piece) {
  const unsigned hi = ar_f16_rne_dev(v);
  if (piece == 0) return hi;
  return ar_f16_rne_dev(v - (float)__builtin_bit_cast(_Float16, (unsigned short)hi));
}

template <class CF>
__global__ void made_ar_pack_fwd_kernel(const float* __restrict__ flat, int64_t sflat, float* __restrict__ packed,
                                        int64_t spk, const float* __restrict__ mask) {
  constexpr int D = CF::D, C = CF::C, H = CF::H, P = CF::P, HB = CF::HB, KSH = CF::KSH, NHID = CF::NHID;
  constexpr int64_t per = (int64_t)H * (C + D) + H + (int64_t)(NHID - 1) * (H * H + H) + (int64_t)D * P * H + D * P;
  const int pos = blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= CF::LAYER) return;
  const int l = blockIdx.y;
  const float* f = flat + blockIdx.z * sflat + (int64_t)l * per;
  float* out = packed + blockIdx.z * spk + (int64_t)l * CF::LAYER;
  // per-sub-layer base pointers of the flat layout
  auto Wl = [&](int i) {
    int64_t o = 0;
    for (int j = 0; j < i; ++j) o += (int64_t)H * (j == 0 ? C + D : H) + H;
    return f + o;
  };
  auto bl = [&](int i) { return Wl(i) + (int64_t)(i < NHID ? H : D * P) * (i == 0 ? C + D : H); };
  // weight idx of sub-layer i, times its mask entry when the caller passes the masks (per layer,
  // the flat layout, shared by every draw) instead of pre-masked rows
  const float* mk = mask == nullptr ? nullptr : mask + (int64_t)l * per;
  auto wv = [&](int i, int64_t idx) {
    const int64_t o = (Wl(i) - f) + idx;
    return mk == nullptr ? f[o] : f[o] * mk[o];
  };
  unsigned word = 0;
  bool done = false;
  static_for<0, CF::NU>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    constexpr int base = CF::stage_id(u) * CF::STG + CF::unit_off(u);
    constexpr int nfr = CF::unit_blocks(u) * CF::unit_kts(u);
    if (done || pos < base || pos >= base + CF::unit_floats(u)) return;
    done = true;
    const int rel = pos - base;
    if (rel >= nfr * CF::OT) {  // bias
      const int r = rel - nfr * CF::OT;
      float v = 0.f;
      if constexpr (u < NHID * HB) {
        constexpr int i = u / HB, b = u % HB;
        if (16 * b + r < H) v = kSigScale * bl(i)[16 * b + r];
      } else {
        constexpr int g = u - NHID * HB;
        const int d = 4 * g + ((r & 15) >> 2), pi = 4 * (r >> 4) + (r & 3);
        if (d < D && pi < P) v = bl(NHID)[pi * D + d];
      }
      word = __builtin_bit_cast(unsigned, v);
      return;
    }
    const int fr = rel / CF::OT, w = rel % CF::OT;
    const int piece = w / 256, lane = (w % 256) / 4, pair = w % 4;
    const int m = lane & 15, kg = lane >> 4;
    for (int e = 0; e < 2; ++e) {
      const int j = 2 * pair + e;
      float v = 0.f;
      if constexpr (u < NHID * HB) {
        constexpr int i = u / HB, b = u % HB;
        const int t = fr, un = 16 * b + m;
        if (un < H) {
          if constexpr (i > 0) {
            const int vv = r16_feat(t, kg, j);
            if (vv < H) v = -2.f * kSigScale * wv(i, (int64_t)un * H + vv);
          } else {
            if (t < CF::KC) {
              const int col = 32 * t + 8 * kg + j;
              if (col < C) v = kSigScale * wv(0, (int64_t)un * (C + D) + col);
            } else {
              const int dd = 8 * kg + j;
              if (dd < D) v = kSigScale * wv(0, (int64_t)un * (C + D) + C + dd);
            }
          }
        }
      } else {
        constexpr int g = u - NHID * HB;
        const int o = fr / KSH, t = fr % KSH;
        const int d = 4 * g + (m >> 2), pi = 4 * o + (m & 3), vv = r16_feat(t, kg, j);
        if (d < D && pi < P && vv < H) v = -2.f * wv(NHID, ((int64_t)pi * D + d) * H + vv);
      }
      word |= ar_piece_dev(v, piece) << (16 * e);
    }
  });
  reinterpret_cast<unsigned*>(out)[pos] = word;  // padding words (no unit) stay 0
}

// Device form of made_ar_pack_layer (the Bayesian log-density packs every weight draw on the GPU,
// naz_ar_flow_pack): thread = one 32-bit word of one layer image, blockIdx.y = layer, blockIdx.z =
// draw; flat as made_ar_pack_fwd_kernel's, perm [L][D] shared by every draw (checked on the host).
template <class CF>
__global__ void made_ar_pack_kernel(const float* __restrict__ flat, int64_t sflat, const int* __restrict__ perm,
                                    float* __restrict__ packed, int64_t spk, const float* __restrict__ c0,
                                    int64_t sc0, const float* __restrict__ mask) {
  constexpr int D = CF::D, C = CF::C, H = CF::H, P = CF::P, NHID = CF::NHID;
  constexpr int64_t per = (int64_t)H * (C + D) + H + (int64_t)(NHID - 1) * (H * H + H) + (int64_t)D * P * H + D * P;
  const int pos = blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= CF::LAYER) return;
  const int l = blockIdx.y;
  const float* f = flat + blockIdx.z * sflat + (int64_t)l * per;
  const int* pm = perm + l * D;
  unsigned* out = reinterpret_cast<unsigned*>(packed + blockIdx.z * spk + (int64_t)l * CF::LAYER);
  if (pos >= CF::PERM_OFF) {
    out[pos] = pos - CF::PERM_OFF < D ? (unsigned)pm[pos - CF::PERM_OFF] : 0u;
    return;
  }
  auto Wl = [&](int i) {
    int64_t o = 0;
    for (int j = 0; j < i; ++j) o += (int64_t)H * (j == 0 ? C + D : H) + H;
    return f + o;
  };
  auto bl = [&](int i) { return Wl(i) + (int64_t)(i < NHID ? H : D * P) * (i == 0 ? C + D : H); };
  // weight idx of sub-layer i, times its mask entry when the caller passes the masks (per layer,
  // the flat layout, shared by every draw) instead of pre-masked rows
  const float* mk = mask == nullptr ? nullptr : mask + (int64_t)l * per;
  auto wv = [&](int i, int64_t idx) {
    const int64_t o = (Wl(i) - f) + idx;
    return mk == nullptr ? f[o] : f[o] * mk[o];
  };
  unsigned word = 0;
  bool done = false;
  if (c0 != nullptr) {  // pass-0 stages: only the constants, compact per stage (CfgAR::c0_off)
    static_for<0, NHID + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int sb = CF::stage_id(0, i) * CF::STG, co = sb + CF::c0_off(i), cnt = CF::c0_cnt(i);
      constexpr int cb = 16 * CF::nb(0) * (i < NHID ? i : NHID);
      if (pos >= sb && pos < sb + CF::STG) done = true;
      if (pos >= co && pos < co + cnt) word = __builtin_bit_cast(unsigned, c0[blockIdx.z * sc0 + (int64_t)l * CF::C0 + cb + pos - co]);
    });
  }
  static_for<0, D>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    static_for<0, NHID + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int base = CF::stage_id(p, i) * CF::STG + CF::sub_off(p, i);
      constexpr int nfr = CF::frags(p, i);
      constexpr int size = nfr * CF::OT + 16 * (i < NHID ? CF::nb(p) : CF::NOB);
      if (done || pos < base || pos >= base + size) return;
      done = true;
      const int rel = pos - base;
      const int dp = pm[p];
      if (rel >= nfr * CF::OT) {  // bias
        const int r = rel - nfr * CF::OT;
        float v = 0.f;
        if constexpr (i < NHID) {
          const int u = 16 * (CF::blo(p) + r / 16) + r % 16;
          if (u < H) v = kSigScale * bl(i)[u];
        } else {
          if (r < P) v = bl(NHID)[r * D + dp];
        }
        word = __builtin_bit_cast(unsigned, v);
        return;
      }
      if constexpr (nfr > 0) {
        const int fr = rel / CF::OT, w = rel % CF::OT;
        const int piece = w / 256, lane = (w % 256) / 4, pair = w % 4;
        const int m = lane & 15, kg = lane >> 4;
        for (int e = 0; e < 2; ++e) {
          const int j = 2 * pair + e;
          float v = 0.f;
          if constexpr (i < NHID) {
            constexpr int kts = i == 0 ? CF::KI : CF::kt(p);
            const int t = fr % kts, u = 16 * (CF::blo(p) + fr / kts) + m;
            if (u < H) {
              if constexpr (i > 0) {
                const int vv = r16_feat(t, kg, j);
                if (vv < H) v = -2.f * kSigScale * wv(i, (int64_t)u * H + vv);
              } else if (t < CF::KC) {
                const int col = 32 * t + 8 * kg + j;
                if (col < C) v = kSigScale * wv(0, (int64_t)u * (C + D) + col);
              } else {
                const int dd = 8 * kg + j;
                if (dd < D) v = kSigScale * wv(0, (int64_t)u * (C + D) + C + dd);
              }
            }
          } else {
            constexpr int kts = CF::kt(p);
            const int o = fr / kts, t = fr % kts;
            const int pi = 16 * o + m, vv = r16_feat(t, kg, j);
            if (pi < P && vv < H) v = -2.f * wv(NHID, ((int64_t)pi * D + dp) * H + vv);
          }
          word |= ar_piece_dev(v, piece) << (16 * e);
        }
      }
    });
  });
  out[pos] = word;  // padding words (no sub-layer) stay 0
}

// blockIdx.y = draw (the Bayesian front end's weight draws, naz_ar_flow_sample_batched): its image at
// packed + draw * spk, its rows at z + draw * sz, y + draw * sy, out_ld + draw * sld
template <class CF>
__global__ void __launch_bounds__(64 * CF::NW, CF::NW / 4) made_ar_fwd_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ z, int64_t ldz,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ y, int64_t ldy, float* __restrict__ out_ld, int64_t B, float bound, int64_t spk = 0,
    int64_t sz = 0, int64_t sy = 0, int64_t sld = 0) {
  constexpr int D = CF::D, K = CF::K, P = CF::P, NW = CF::NW, NHID = CF::NHID, HB = CF::HB, KSH = CF::KSH;
  {
    const int64_t dz = blockIdx.y;
    packed += dz * spk;
    z += dz * sz;
    y += dz * sy;
    if (out_ld != nullptr) out_ld += dz * sld;
  }
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + CF::STG;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  const int64_t row = (int64_t)blockIdx.x * (16 * NW) + wave * 16 + (lane & 15);
  const bool valid = row < B;
  const int64_t crow = valid ? row : 0;

  float v[D];
#pragma unroll
  for (int d = 0; d < D; ++d) v[d] = valid ? z[crow * ldz + d] : 0.f;
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
  const RqsConsts<K, false> rc(bound);
  float ldsum = 0.f;
  stage_issue<CF::stage_floats(0), NW>(slot0, packed);
  int g = 0;
  for (int l = 0; l < L; ++l) {
    const float* lp = packed + (int64_t)l * CF::LAYER;
    const float* lnext = packed + (int64_t)(l + 1) * CF::LAYER;
    // hidden layer i's B fragments in hf[i & 1]: only two layers are ever live (the wide H = 512
    // instances hold 2 x 128 VGPRs of them)
    Frag2 hf[2][KSH];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int t = 0; t < KSH; ++t) hf[i][t] = Frag2{half8{}, half8{}};
    // the layer input's f16 split at a per-row power-of-two scale (|x| sc < 2^14)
    float xmax = 0.f;  // (affine only: splines keep a row within max(|z|, B), see the inverse kernel)
    if constexpr (CF::AFFINE) {
#pragma unroll
      for (int d = 0; d < D; ++d) xmax = fmaxf(xmax, fabsf(v[d]));
    }
    const int e = xmax >= 16384.f ? __builtin_amdgcn_frexp_expf(xmax) - 14 : 0;
    const float sc = __builtin_amdgcn_ldexpf(1.f, -e), us = __builtin_amdgcn_ldexpf(1.f, e);
    float x8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = 0.f;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        if (8 * qq + j < D) s = q == qq ? v[8 * qq + j] : s;
      x8[j] = s * sc;
    }
    const Frag2 xf = split8_f16(x8);
    const float* cur = slot0;
    static_for<0, CF::NU>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      constexpr int SID = CF::stage_id(u), OFF = CF::unit_off(u);
      constexpr bool NEW_STAGE = u == 0 || SID != CF::stage_id(u > 0 ? u - 1 : 0);
      if constexpr (NEW_STAGE) {  // stage SID has landed in slot (g & 1)
        ring_barrier();  // ... and every wave is done with the other slot
        cur = (g & 1) ? slot1 : slot0;
        float* nxt = (g & 1) ? slot0 : slot1;
        if constexpr (SID + 1 < CF::NSTG) {
          stage_issue<CF::stage_floats(SID + 1), NW>(nxt, lp + (SID + 1) * CF::STG);
        } else {
          if (l + 1 < L) stage_issue<CF::stage_floats(0), NW>(nxt, lnext);
        }
        ++g;
      }
      const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
      auto afrag = [&](int idx) {
        const int base = (OFF >> 2) + idx * 128 + lane;
        return Frag2{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      };
      if constexpr (u < NHID * HB) {
        constexpr int i = u / HB, b = u % HB, KT = CF::unit_kts(u);
        const float4 bv = reinterpret_cast<const float4*>(cur + OFF + KT * CF::OT)[q];
        floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
        if constexpr (i == 0) {
#pragma unroll
          for (int t = 0; t < CF::KC; ++t) acc = mfma3_16(afrag(t), cf[t], acc);
          const floatx4 ax = mfma3_16(afrag(CF::KC), xf, floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
          for (int r = 0; r < 4; ++r) acc[r] = __builtin_fmaf(ax[r], us, acc[r]);
        } else if constexpr (NW == 4) {  // the wide instances (one wave per SIMD): prefetched chain
          acc = mfma3_16_chain_lds<KT>((unsigned)(uintptr_t)to_lds(cur) + 16u * lane + 4u * OFF,
                                       hf[(i - 1) & 1], acc);
        } else {
#pragma unroll
          for (int t = 0; t < KT; ++t) acc = mfma3_16(afrag(t), hf[(i - 1) & 1][t], acc);
        }
        ar_split4<b & 1>(hf[i & 1][b >> 1], acc);
      } else {
        // dims 4 g .. 4 g + 3: quarter q's lanes map dim 4 g + q with its parameters in their own
        // accumulator registers (register i of block o = parameter 4 o + i), then every lane
        // takes the group's new values from the owning quarters (four shuffles)
        constexpr int g = u - NHID * HB, NOG = CF::NOG;
        floatx4 o3[NOG];
        const float4* bias4 = reinterpret_cast<const float4*>(cur + OFF + NOG * KSH * CF::OT);
#pragma unroll
        for (int o = 0; o < NOG; ++o) {
          const float4 bv = bias4[4 * o + q];
          o3[o] = floatx4{bv.x, bv.y, bv.z, bv.w};
        }
        if constexpr (NW == 4 && NOG == 1) {
          o3[0] = mfma3_16_chain_lds<KSH>((unsigned)(uintptr_t)to_lds(cur) + 16u * lane + 4u * OFF,
                                          hf[(NHID - 1) & 1], o3[0]);
        } else {
#pragma unroll
          for (int t = 0; t < KSH; ++t)
#pragma unroll
            for (int o = 0; o < NOG; ++o) o3[o] = mfma3_16(afrag(o * KSH + t), hf[(NHID - 1) & 1][t], o3[o]);
        }
        float xv = 0.f;  // this quarter's dim
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          if (4 * g + qq < D) xv = q == qq ? v[4 * g + qq < D ? 4 * g + qq : 0] : xv;
        const bool own = 4 * g + q < D;
        float yv, ld;
        if constexpr (CF::AFFINE) {
          // pyro AffineAutoregressive._call: y = exp(clamp(ls)) x + mean, log|det| = clamp(ls)
          const float ls = fminf(fmaxf(o3[0][1], -5.f), 3.f);
          yv = __builtin_fmaf(xv, __expf(ls), o3[0][0]);
          ld = ls;
        } else {
          float uw[K], uh[K], ud[K - 1];
#pragma unroll
          for (int pi = 0; pi < P; ++pi) {
            const float val = o3[pi >> 2][pi & 3];
            if (pi < K) uw[pi] = val;
            else if (pi < 2 * K) uh[pi - K] = val;
            else ud[pi - 2 * K] = val;
          }
          yv = rqs_select<K, false>(uw, uh, ud, xv, bound, rc, ld);
        }
        ldsum += own ? ld : 0.f;  // summed over the quarters at the end
#pragma unroll
        for (int qq = 0; qq < 4; ++qq)
          if (4 * g + qq < D) v[4 * g + qq < D ? 4 * g + qq : 0] = __shfl(yv, (lane & 15) + 16 * qq);
        // the groups are independent: unpinned, the scheduler hoists later groups' output MFMAs
        // over this group's map and their accumulators spill
        __builtin_amdgcn_sched_barrier(0);
      }
    });
  }
  if (low != nullptr) {  // naz inverse_bounding_transform (transforms.py:24-27, flow.py:129)
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = (1.f / (1.f + expf(-v[d]))) * (high[d] - low[d]) + low[d];
  }
  ldsum += __shfl_xor(ldsum, 16);  // each quarter summed its own dims' log-dets
  ldsum += __shfl_xor(ldsum, 32);
  if (q == 0 && valid) {
#pragma unroll
    for (int d = 0; d < D; ++d) y[row * ldy + d] = v[d];
    if (out_ld != nullptr) out_ld[row] = ldsum;
  }
}

}  // namespace naz
