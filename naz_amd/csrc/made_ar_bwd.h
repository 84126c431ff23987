// Backward of the fused affine-autoregressive (naz "maf") flow: dL/dθ and dL/dx of
// L = Σ_rows g_lp · log p(x | ctx) for the NUTS / HMC potential of naz's Bayesian MAF
// (bflow_jax_maf.py:231-235: jax.grad of flow_lp(unravel(p)).sum(); hmc_maf_exact.py:118-133) and
// the maf NLL step (train_flows.py:194-213).  SURVEY.md §8f rank 1 over §8a a5/a6.
// Included by coupling.hip (part 3) after made_ar_r16.h (CfgAR, CfgARF, split8_f16, sig_fold,
// stage_issue, ring_barrier, bwd_row_scale, ...).
//
// The forward is the fused inverse kernel (made_ar_r16_kernel) with its per-layer outputs saved:
// states[l] = s_l, the output of layer l's inverse (layer l maps s_{l+1} -> s_l; s_0 = z).
// One launch of made_ar_bwd_kernel per layer l = 0 .. L-1 takes g(s_l) and produces g(s_{l+1}) and
// the weight-gradient operands of layer l:
//   1. one DENSE MADE pass on (ctx, s_l) with the forward (sample-direction) image: every hidden
//      unit and every dim's (mean, log_scale) at its final value (the masks make a unit of degree m
//      depend only on dims of order < m, so the D-pass inverse's values are these); the hidden
//      activations h_i go to HBM (weight-gradient operands, re-read for tanh');
//   2. the affine step's VJP per dim: s_d = (y_d - m_d) e^{-c(a_d)}, c = clamp(., -5, 3) with
//      pyro's clamp_preserve_gradients (identity gradient), and log p gaining -c(a_d):
//        dL/dm_d = -g_d e^{-c},  dL/da_d = -g_lp - g_d s_d,  dL/dy_d = g_d e^{-c};
//      with clip_zero (NAZ_AR_CLIP_ZERO_GRAD: jnp.clip, bflow_jax_maf.py:177,188,192) dL/da_d = 0
//      wherever a_d lies outside [-5, 3];
//   3. the D sequential dependencies of the inverse, in reverse: for order p = D-1 .. 1, the output
//      gradient of dim d_p alone is backpropagated through the MADE (δ_NHID = W_outᵀ g ⊙ tanh',
//      δ_i = W_iᵀ δ_{i+1} ⊙ tanh', dx = W_0[:, C:]ᵀ δ_1) and dx added to g of the dims of order < p
//      (masked weights are exact zeros, so nothing else receives any); then ONE final chain with
//      every dim's output gradient gives the total δ_i (linearity), written as operands;
//   4. dW_i = δ_{i+1}ᵀ h_i and the biases' column sums run as batch-reduction GEMMs (naz_gemm).
// Precision: the MADE pass on the forward kernels' f16x3 split; the transposed GEMMs on f16x3 with
// the gradient operand scaled per row by a power of two (bwd_row_scale: row maximum in
// [2^13, 2^14)) and 2^6 W images, as the coupling backward; W_outᵀ g in exact fp32 (VALU).
// Layout: the r16 16-row waves (lane = row l & 15, quarter q = l >> 4; accumulator register r of
// 16-block b on quarter q = unit 16 b + 4 q + r); a backward GEMM's k-step t feeds each quarter's
// OWN accumulator registers of blocks 2t, 2t + 1 (k-slot (t, q, j) = unit r16_feat(t, q, j)), and
// the backward images order Wᵀ's columns to match, so every chain step lands in the forward's
// activation layout with no shuffles.
#pragma once

namespace naz {

template <class CF>
struct CfgARB {
  using FW = CfgARF<CF>;
  static constexpr int D = CF::D, C = CF::C, H = CF::H, NHID = CF::NHID, P = CF::P;
  static constexpr int HP = CF::HP, HB = CF::HB, KSH = CF::KSH, KC = CF::KC, OT = CF::OT;
  static constexpr int NW = 8;           // 2 waves per SIMD, one workgroup per CU (two 80 KB ring slots)
  static constexpr int NO = 2 * D;       // ARN outputs (mean, log_scale) x D, row pi D + d
  static constexpr int X0W = 8;          // [ctx | s | 0] operand width (wgrad's whole-chunk rule)
  static constexpr int XA = HP, XB = 0;  // h operand column groups (one: naz_wgrad_batched takes N2 <= 160)
  // backward image units: 0 = W_out (natural fp32 [NO][HP]); 1 .. (NHID-1) HB = (W_iᵀ, output
  // block b) for i = NHID-1 down to 1; last = the input unit W_0[:, C:]ᵀ (one block, rows = dims)
  static constexpr int NUB = 2 + (NHID - 1) * HB;
  static constexpr int TBLF = NO * HP;
  static constexpr int hid_i(int j) { return NHID - 1 - (j - 1) / HB; }
  static constexpr int hid_b(int j) { return (j - 1) % HB; }
  // the transposed products skip their leading k-steps: W_i[v][u] (u: unit of output block b, v:
  // unit of the layer above, the k index) is masked unless deg(v) >= deg(u), and degrees do not
  // decrease along the unit index, so k-steps of units all below the block's smallest degree are
  // exact zeros (bit-identical results, as CfgARF::hid_kts in the forward image)
  struct T0Tab {
    int t0[64];
  };
  static constexpr T0Tab make_t0() {
    T0Tab y{};
    for (int b = 0; b < HB; ++b) {
      const int first = 16 * b < H ? 16 * b : H - 1;
      const int dmin = CF::deg(first);
      int e = 0;
      for (int v = 0; v < H; ++v) e += CF::deg(v) < dmin ? 1 : 0;
      y.t0[b] = e >> 5;
    }
    return y;
  }
  static constexpr T0Tab T0T = make_t0();
#ifdef NAZ_AR_BWD_DENSE_K  // (A/B: every k-step)
  static constexpr int kt0(int) { return 0; }
#else
  static constexpr int kt0(int j) { return j >= 1 && j < NUB - 1 ? T0T.t0[hid_b(j)] : 0; }
#endif
  static constexpr int unit_floats(int j) { return j == 0 ? (TBLF + 255) / 256 * 256 : (KSH - kt0(j)) * OT; }
  struct Layout {
    int sid[NUB], off[NUB], sfl[NUB];
    int nstg, stg;
  };
  static constexpr Layout make_layout() {
    Layout y{};
    int s = -1, run = 0;
    for (int j = 0; j < NUB; ++j) {
      const int sz = unit_floats(j);
      if (j == 0 || run + sz > kARCap) {
        ++s;
        run = 0;
      }
      y.sid[j] = s;
      y.off[j] = run;
      run += sz;
      y.sfl[s] = CF::pad(run);
    }
    y.nstg = s + 1;
    for (int t = 0; t < y.nstg; ++t) y.stg = y.sfl[t] > y.stg ? y.sfl[t] : y.stg;
    return y;
  }
  static constexpr Layout LY = make_layout();
  static constexpr int stage_id(int j) { return LY.sid[j]; }
  static constexpr int unit_off(int j) { return LY.off[j]; }
  static constexpr int stage_floats(int s) { return LY.sfl[s]; }
  static constexpr int NSTG = LY.nstg, STG = LY.stg;
  static constexpr int LAYER = CF::pad(NSTG * STG);
  static constexpr int SLOT = FW::STG > STG ? FW::STG : STG;  // LDS ring slot: either image's stage
  static constexpr int64_t per() {
    return (int64_t)H * (C + D) + H + (int64_t)(NHID - 1) * (H * H + H) + (int64_t)D * P * H + D * P;
  }
  static_assert(CF::AFFINE && P == 2, "the fused backward covers affine autoregressive flows");
  static_assert(D <= 4 && C + D <= X0W && NHID >= 2 && NHID <= 3, "unsupported fused maf backward shape");
  static_assert(2 * SLOT * 4 <= 160 * 1024, "two ring slots exceed the LDS");
};

// Device packer of the backward images: thread = one 32-bit word of layer blockIdx.y's image.
// flat: L layers of the naz_ar_flow_pack_host flat layout; mask (same layout, optional) multiplies.
template <class CB>
__global__ void made_ar_pack_bwd_kernel(const float* __restrict__ flat, const float* __restrict__ mask,
                                        float* __restrict__ packed) {
  constexpr int D = CB::D, C = CB::C, H = CB::H, HP = CB::HP, NHID = CB::NHID, NO = CB::NO;
  const int pos = blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= CB::LAYER) return;
  const int l = blockIdx.y;
  const float* f = flat + (int64_t)l * CB::per();
  const float* mk = mask == nullptr ? nullptr : mask + (int64_t)l * CB::per();
  auto woff = [&](int i) {  // sub-layer i's weight offset in the flat row
    int64_t o = 0;
    for (int j = 0; j < i; ++j) o += (int64_t)H * (j == 0 ? C + D : H) + H;
    return o;
  };
  auto wv = [&](int i, int64_t idx) {
    const int64_t o = woff(i) + idx;
    return mk == nullptr ? f[o] : f[o] * mk[o];
  };
  unsigned word = 0;
  bool done = false;
  static_for<0, CB::NUB>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int base = CB::stage_id(j) * CB::STG + CB::unit_off(j);
    if (done || pos < base || pos >= base + CB::unit_floats(j)) return;
    done = true;
    const int rel = pos - base;
    if constexpr (j == 0) {  // W_out rows, natural fp32
      const int o = rel / HP, u = rel - o * HP;
      const float v = (o < NO && u < H) ? wv(NHID, (int64_t)o * H + u) : 0.f;
      word = __builtin_bit_cast(unsigned, v);
      return;
    } else {
      const int t = rel / CB::OT + CB::kt0(j), w = rel % CB::OT;  // (leading masked k-steps not stored)
      const int piece = w / 256, lane = (w % 256) / 4, pair = w % 4;
      const int m = lane & 15, kg = lane >> 4;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const int vv = r16_feat(t, kg, 2 * pair + e);  // k: unit of the layer above
        float v = 0.f;
        if constexpr (j < CB::NUB - 1) {
          constexpr int i = CB::hid_i(j), b = CB::hid_b(j);
          const int u = 16 * b + m;  // output: unit of hidden layer i (1-based: W_i maps it upward)
          if (vv < H && u < H) v = kBwdWScale * wv(i, (int64_t)vv * H + u);
        } else {
          if (m < D && vv < H) v = kBwdWScale * wv(0, (int64_t)vv * (C + D) + C + m);
        }
        word |= ar_piece_dev(v, piece) << (16 * e);
      }
    }
  });
  reinterpret_cast<unsigned*>(packed + (int64_t)l * CB::LAYER)[pos] = word;
}

struct ArBwdOut {
  float* x0;       // [B, X0W]  [ctx | s_l | 0]
  float* ha[3];    // [B, XA]   hidden layer i + 1 units [0, XA) (natural tanh)
  float* hb[3];    // [B, XB]   units [XA, HP)
  float* dp[3];    // [B, HP]   dL/d pre-activation of hidden layer i + 1
  float* gout;     // [B, X0W]  dL/d ARN outputs (row pi D + d), zero padded
  float* g_next;   // [B, D]    dL/d s_{l+1}
};

template <class CB, int LAYER_I, int B0>
NAZ_DEV float4* ar_h_ptr(const ArBwdOut& o, int64_t row, int q) {
  if constexpr (16 * B0 < CB::XA) return reinterpret_cast<float4*>(o.ha[LAYER_I] + row * CB::XA + 16 * B0 + 4 * q);
  else return reinterpret_cast<float4*>(o.hb[LAYER_I] + row * CB::XB + 16 * B0 - CB::XA + 4 * q);
}

// 8 waves x 16 rows per workgroup.  g_lp == nullptr: g_lp = 1.
template <class CB>
__global__ void __launch_bounds__(64 * CB::NW, CB::NW / 4) made_ar_bwd_kernel(
    const float* __restrict__ fimg, const float* __restrict__ bimg, const int* __restrict__ perm,
    const float* __restrict__ s_in, const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ g_in,
    const float* __restrict__ g_lp, ArBwdOut o, int64_t B, int clip_zero) {
  using FW = typename CB::FW;
  constexpr int D = CB::D, C = CB::C, NW = CB::NW, NHID = CB::NHID, HB = CB::HB, KSH = CB::KSH, HP = CB::HP;
  constexpr int NO = CB::NO, ROWS = 16 * NW, SLOT = CB::SLOT, NUF = FW::NU;
  constexpr int NSF = FW::NSTG, NSB = CB::NSTG;
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + SLOT;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;

  // one 128-row tile per workgroup (a persistent tile loop lets the compiler hoist ~60 per-unit LDS
  // addresses out of it, which then spill)
  stage_issue<FW::stage_floats(0), NW>(slot0, fimg);
  int g = 0;  // stage counter: stage g lives in slot (g & 1)
  {
    const int64_t row = (int64_t)blockIdx.x * ROWS + wave * 16 + (lane & 15);
    const bool valid = row < B;
    const int64_t crow = valid ? row : 0;
    float s[D], gs[D];
#pragma unroll
    for (int d = 0; d < D; ++d) {
      s[d] = valid ? s_in[crow * D + d] : 0.f;
      gs[d] = valid ? g_in[crow * D + d] : 0.f;
    }
    const float gl = g_lp == nullptr ? 1.f : (valid ? g_lp[crow] : 0.f);
    Frag2 cf[CB::KC > 0 ? CB::KC : 1];
    float cv[C > 0 ? C : 1];
#pragma unroll
    for (int t = 0; t < CB::KC; ++t) {
      float c8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = 32 * t + 8 * q + j;
        c8[j] = col < C ? ctx[crow * ldc + col] : 0.f;
      }
      cf[t] = split8_f16(c8);
    }
#pragma unroll
    for (int c = 0; c < C; ++c) cv[c] = ctx[crow * ldc + c];
    if (valid && q == 0) {
      float x0[CB::X0W];
#pragma unroll
      for (int k = 0; k < CB::X0W; ++k) x0[k] = k < C ? cv[k < C ? k : 0] : (k < C + D ? s[k - C < D ? k - C : 0] : 0.f);
#pragma unroll
      for (int k = 0; k < CB::X0W; k += 4)
        *reinterpret_cast<float4*>(o.x0 + row * CB::X0W + k) = float4{x0[k], x0[k + 1], x0[k + 2], x0[k + 3]};
    }
    // the layer input's f16 split at a per-row power-of-two scale (|s| sc < 2^14), as the forward kernel
    float xmax = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) xmax = fmaxf(xmax, fabsf(s[d]));
    const int ex2 = xmax >= 16384.f ? __builtin_amdgcn_frexp_expf(xmax) - 14 : 0;
    const float sc = __builtin_amdgcn_ldexpf(1.f, -ex2), us = __builtin_amdgcn_ldexpf(1.f, ex2);
    Frag2 xf;
    {
      float x8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) x8[j] = (q == 0 && j < D) ? s[j < D ? j : 0] * sc : 0.f;
      xf = split8_f16(x8);
    }
    float ex[D];  // e^{-c(a_d)}
    const float* cur = slot0;
    // stage ring: the whole stream of a tile is NSF forward stages, then D passes over the NSB
    // backward stages; each advance publishes the current stage and issues the next one
    auto advance = [&](auto kc) {
      constexpr int k = decltype(kc)::value;  // position in the tile's stream
      ring_barrier();  // stage k has landed in slot (g & 1); every wave is done with the other slot
      cur = (g & 1) ? slot1 : slot0;
      float* nxt = (g & 1) ? slot0 : slot1;
      constexpr int kn = k + 1;
      if constexpr (kn < NSF) {
        stage_issue<FW::stage_floats(kn), NW>(nxt, fimg + kn * FW::STG);
      } else {  // the first backward stage (the chains' own advances issue the rest)
        stage_issue<CB::stage_floats(0), NW>(nxt, bimg);
      }
      ++g;
    };

    // ---- 1. dense MADE pass on (ctx, s): hidden activations to HBM, (mean, log_scale) per dim
    float mu[D], la[D];
    {
      Frag2 hf[2][KSH];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int t = 0; t < KSH; ++t) hf[i][t] = Frag2{half8{}, half8{}};
      static_for<0, NUF>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int SID = FW::stage_id(u), OFF = FW::unit_off(u);
        if constexpr (u == 0 || SID != FW::stage_id(u > 0 ? u - 1 : 0)) advance(std::integral_constant<int, SID>{});
        __builtin_amdgcn_sched_barrier(0);  // one unit's operands live at a time
        const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
        auto afrag = [&](int idx) {
          const int base = (OFF >> 2) + idx * 128 + lane;
          return Frag2{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
        };
        if constexpr (u < NHID * HB) {
          constexpr int i = u / HB, b = u % HB, KT = FW::unit_kts(u);
          const float4 bv = reinterpret_cast<const float4*>(cur + OFF + KT * CB::OT)[q];
          floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
          if constexpr (i == 0) {
#pragma unroll
            for (int t = 0; t < CB::KC; ++t) acc = mfma3_16(afrag(t), cf[t], acc);
            const floatx4 ax = mfma3_16(afrag(CB::KC), xf, floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = __builtin_fmaf(ax[r], us, acc[r]);
          } else {
#pragma unroll
            for (int t = 0; t < KT; ++t) acc = mfma3_16(afrag(t), hf[(i - 1) & 1][t], acc);  // FW::hid_kts
          }
          floatx4 v;
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = sig_fold(acc[r]);  // -tanh/2 (the packed fold)
          if (valid) *ar_h_ptr<CB, i, b>(o, row, q) = float4{-2.f * v[0], -2.f * v[1], -2.f * v[2], -2.f * v[3]};
          // split into the B fragment (k-step b >> 1, half b & 1) of the next layer
          Frag2& f = hf[i & 1][b >> 1];
          u32x4 Hh = __builtin_bit_cast(u32x4, f.h), Lo = __builtin_bit_cast(u32x4, f.l);
#pragma unroll
          for (int w = 0; w < 2; ++w) {
            const unsigned hp = pack_f16x2(v[2 * w], v[2 * w + 1]);
            Hh[2 * (b & 1) + w] = hp;
            Lo[2 * (b & 1) + w] = pack_f16x2(sub_f16_piece<false>(v[2 * w], hp), sub_f16_piece<true>(v[2 * w + 1], hp));
          }
          f.h = __builtin_bit_cast(half8, Hh);
          f.l = __builtin_bit_cast(half8, Lo);
        } else {
          // dims 4 g + qq: quarter qq's registers 0, 1 hold that dim's (mean, log_scale) (the
          // forward image's dim groups); every lane takes all of the group's
          constexpr int g = u - NHID * HB;
          static_assert(FW::NOG == 1, "affine: one output block per dim group");
          const float4 bv = reinterpret_cast<const float4*>(cur + OFF + KSH * CB::OT)[q];
          floatx4 o3 = floatx4{bv.x, bv.y, bv.z, bv.w};
#pragma unroll
          for (int t = 0; t < KSH; ++t) o3 = mfma3_16(afrag(t), hf[(NHID - 1) & 1][t], o3);
#pragma unroll
          for (int qq = 0; qq < 4; ++qq)
            if (4 * g + qq < D) {
              mu[4 * g + qq < D ? 4 * g + qq : 0] = __shfl(o3[0], (lane & 15) + 16 * qq);
              la[4 * g + qq < D ? 4 * g + qq : 0] = __shfl(o3[1], (lane & 15) + 16 * qq);
            }
        }
      });
    }
    // ex[d] = e^{-c(a_d)} > 0; with clip_zero its SIGN carries whether a_d lies inside [-5, 3] (the
    // jnp.clip gradient's support), so no per-dim flag stays live through the chains
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const float e = __expf(-fminf(fmaxf(la[d], -5.f), 3.f));
      ex[d] = (clip_zero && !(la[d] >= -5.f && la[d] <= 3.f)) ? -e : e;
    }

    // ---- 2./3. the chains: orders p = D-1 .. 1 for the input gradients, then the final one with
    // every dim's output gradient.  The input chains run as a RUNTIME loop (one chain's code and
    // operands live at a time: unrolled over D = 4 the compiler interleaved the chains' LDS reads and
    // needed ~470 registers); a chain streams the NSB backward stages, its last one issuing stage 0
    // of the next chain.
    auto advance_b = [&](auto sc, auto morec) {
      constexpr int sb = decltype(sc)::value;
      ring_barrier();  // backward stage sb has landed in slot (g & 1); every wave is done with the other
      cur = (g & 1) ? slot1 : slot0;
      float* nxt = (g & 1) ? slot0 : slot1;
      if constexpr (sb + 1 < NSB) {
        stage_issue<CB::stage_floats(sb + 1), NW>(nxt, bimg + (sb + 1) * CB::STG);
      } else if constexpr (decltype(morec)::value) {
        stage_issue<CB::stage_floats(0), NW>(nxt, bimg);
      }
      ++g;
    };
    auto chain = [&](auto finalc, const int dsel) {  // dsel: dim of this chain's order (input chains)
      constexpr bool FINAL = decltype(finalc)::value;
      // dL/d (mean_d, log_scale_d); with clip_zero the clip's gradient is jnp.clip's (0 outside
      // [-5, 3]).  Input chain: go[0], go[1] = dim dsel's pair (the others are zero).
      float go[NO];
      if constexpr (FINAL) {
#pragma unroll
        for (int d = 0; d < D; ++d) {
          go[d] = -gs[d] * fabsf(ex[d]);
          go[D + d] = ex[d] > 0.f ? -gl - gs[d] * s[d] : 0.f;
        }
      } else {
        float gsd = gs[0], sd = s[0], exd = ex[0];
#pragma unroll
        for (int d = 1; d < D; ++d) {
          gsd = dsel == d ? gs[d] : gsd;
          sd = dsel == d ? s[d] : sd;
          exd = dsel == d ? ex[d] : exd;
        }
        go[0] = -gsd * fabsf(exd);
        go[1] = exd > 0.f ? -gl - gsd * sd : 0.f;
#pragma unroll
        for (int k = 2; k < NO; ++k) go[k] = 0.f;
      }
      if constexpr (FINAL) {
        if (valid && q == 0) {
          float gp[CB::X0W];
#pragma unroll
          for (int k = 0; k < CB::X0W; ++k) gp[k] = k < NO ? go[k < NO ? k : 0] : 0.f;
#pragma unroll
          for (int k = 0; k < CB::X0W; k += 4)
            *reinterpret_cast<float4*>(o.gout + row * CB::X0W + k) = float4{gp[k], gp[k + 1], gp[k + 2], gp[k + 3]};
        }
      }
      floatx4 dcur[HB];  // δ of the layer above until its B fragments are formed, then this layer's
      Frag2 bfr[KSH];
      float gscale = 1.f;
      static_for<0, CB::NUB>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        constexpr int SID = CB::stage_id(j), OFF = CB::unit_off(j);
        if constexpr (j == 0 || SID != CB::stage_id(j > 0 ? j - 1 : 0))
          advance_b(std::integral_constant<int, SID>{}, std::integral_constant<bool, !FINAL>{});
        if constexpr (FINAL && j == CB::NUB - 1) return;  // no input gradient after the last chain
        __builtin_amdgcn_sched_barrier(0);
        const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
        auto afrag = [&](int idx) {
          const int base = (OFF >> 2) + idx * 128 + lane;
          return Frag2{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
        };
        if constexpr (j == 0) {
          // δ_NHID = (W_outᵀ go) ⊙ (1 - h²), exact fp32 from the natural W_out rows
          const float4* tb = reinterpret_cast<const float4*>(cur + OFF);
          // an input chain has only dim dsel's two outputs (mean, log_scale) nonzero
          const float gm = FINAL ? 0.f : go[0], gsl = FINAL ? 0.f : go[1];
          floatx4 tie1 = floatx4{0.f, 0.f, 0.f, 0.f}, tie2 = tie1;  // the final chain's last two blocks' products
          static_for<0, HB>([&](auto bc) {
            constexpr int b = decltype(bc)::value;
            __builtin_amdgcn_sched_barrier(0);
            float a[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (FINAL) {
              // block b's NO float4 reads of W_out take their address through a register tied to
              // block b - 2's products: at most two blocks' reads in flight.  Untied, the scheduler
              // issued all HB x NO reads ahead of the products (320 VGPRs at D = 4: spills), across
              // sched_barrier and asm memory fences alike.
              int woff = 0;
              asm volatile("" : "+v"(woff) : "v"(tie2[0]), "v"(tie2[1]), "v"(tie2[2]), "v"(tie2[3]));
              const float4* tbb = tb + woff;
#pragma unroll
              for (int oo = 0; oo < NO; ++oo) {
                const float4 w = tbb[(oo * HP + 16 * b) / 4 + q];
                a[0] = __builtin_fmaf(w.x, go[oo], a[0]);
                a[1] = __builtin_fmaf(w.y, go[oo], a[1]);
                a[2] = __builtin_fmaf(w.z, go[oo], a[2]);
                a[3] = __builtin_fmaf(w.w, go[oo], a[3]);
              }
              tie2 = tie1;
              tie1 = floatx4{a[0], a[1], a[2], a[3]};
            } else {
              const float4 w0 = tb[(dsel * HP + 16 * b) / 4 + q], w1 = tb[((D + dsel) * HP + 16 * b) / 4 + q];
              a[0] = __builtin_fmaf(w1.x, gsl, w0.x * gm);
              a[1] = __builtin_fmaf(w1.y, gsl, w0.y * gm);
              a[2] = __builtin_fmaf(w1.z, gsl, w0.z * gm);
              a[3] = __builtin_fmaf(w1.w, gsl, w0.w * gm);
            }
            const float4 hv = valid ? *ar_h_ptr<CB, NHID - 1, b>(o, row, q) : float4{0.f, 0.f, 0.f, 0.f};
            dcur[b] = floatx4{a[0] * (1.f - hv.x * hv.x), a[1] * (1.f - hv.y * hv.y), a[2] * (1.f - hv.z * hv.z),
                              a[3] * (1.f - hv.w * hv.w)};
          });
        } else {
          constexpr bool INPUT = j == CB::NUB - 1;
          constexpr int i = INPUT ? 0 : CB::hid_i(j), b = INPUT ? 0 : CB::hid_b(j);
          if constexpr (INPUT || b == 0) {
            // the layer-above gradient (δ_{i+1}, hidden layer i + 1) complete: operand store
            // (final chain), then its per-row scale and the B fragments of every k-step
            if constexpr (FINAL) {
              if (valid)
#pragma unroll
                for (int bb = 0; bb < HB; ++bb)
                  *reinterpret_cast<float4*>(o.dp[i] + row * HP + 16 * bb + 4 * q) =
                      float4{dcur[bb][0], dcur[bb][1], dcur[bb][2], dcur[bb][3]};
            }
            gscale = bwd_row_scale(dcur);
#pragma unroll
            for (int t = 0; t < KSH; ++t) {
              float v8[8];
#pragma unroll
              for (int jj = 0; jj < 8; ++jj) {
                const int blk = 2 * t + (jj >> 2);
                v8[jj] = blk < HB ? dcur[blk < HB ? blk : 0][jj & 3] : 0.f;
              }
              bfr[t] = split8_f16(v8);
            }
          }
          floatx4 acc = floatx4{0.f, 0.f, 0.f, 0.f};
          constexpr int T0 = CB::kt0(j);  // leading k-steps masked to zero: not stored, not multiplied
#pragma unroll
          for (int t = T0; t < KSH; ++t) acc = mfma3_16(afrag(t - T0), bfr[t], acc);
          if constexpr (INPUT) {
            // dx of dims m = 4 q + r sits on quarter 0 (D <= 4): every quarter takes the row's values
#pragma unroll
            for (int d = 0; d < D; ++d) gs[d] += __shfl(acc[d], lane & 15) * gscale;
          } else {
            const float4 hv = valid ? *ar_h_ptr<CB, i - 1, b>(o, row, q) : float4{0.f, 0.f, 0.f, 0.f};
            dcur[b] = floatx4{acc[0] * gscale * (1.f - hv.x * hv.x), acc[1] * gscale * (1.f - hv.y * hv.y),
                              acc[2] * gscale * (1.f - hv.z * hv.z), acc[3] * gscale * (1.f - hv.w * hv.w)};
            if constexpr (b == HB - 1) {
              if constexpr (FINAL && i == 1) {  // δ_1: the last operand
                if (valid)
#pragma unroll
                  for (int bb = 0; bb < HB; ++bb)
                    *reinterpret_cast<float4*>(o.dp[0] + row * HP + 16 * bb + 4 * q) =
                        float4{dcur[bb][0], dcur[bb][1], dcur[bb][2], dcur[bb][3]};
              }
            }
          }
        }
      });
    };
#pragma unroll 1
    for (int c = 0; c < D - 1; ++c) chain(std::false_type{}, __builtin_amdgcn_readfirstlane(perm[D - 1 - c]));
    chain(std::true_type{}, -1);
    if (valid && q == 0) {
#pragma unroll
      for (int d = 0; d < D; ++d) o.g_next[row * D + d] = gs[d] * fabsf(ex[d]);
    }
  }
}

}  // namespace naz
