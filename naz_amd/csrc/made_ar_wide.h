// Fused log_prob of naz's WIDE production MAFs (the 4-parameter MLE flow D=4 | C=2, H=[512]x5, L=18,
// examples/papers/2506.05657/train_mle_all_data_4param.py:87-92; POSYDON D=4, 512x5, L=16,
// eposydon/train_maf_mle.py:84-90): pyro ConditionedAffineAutoregressive._inverse (naz
// flows/transforms.py:133-160) over every layer, driven by NormalizingFlow.log_prob (flow.py:45-79),
// in ONE launch.  Included by coupling.hip after made_ar_r16.h (CfgARW, Frag2, ar_split4, mfma3_16,
// r16_feat, stage_issue, ring_barrier, ar_piece / ar_piece_dev).
//
// made_ar_r16_kernel computes every MADE hidden unit once, in the pass of its mask degree, and keeps
// all hidden layers as register-resident B fragments.  At H = 512 one hidden layer is 16 fragments =
// 128 VGPRs, five of them do not fit, so here:
//   * two register sets hold the layer being read and the layer being written (as the wide
//     sampler, made_ar_fwd_kernel);
//   * hidden layer 1 (from [ctx | x]: two k-steps per block) is recomputed in full every pass
//     (blocks 0 .. of degree <= p), which costs ~6 % more MFMAs than its degree-p blocks alone and
//     keeps it out of memory;
//   * hidden layers 2 .. n_hidden persist between passes in a per-wave global scratch area (4
//     layers x 16 fragments x 2 KB = 128 KB per wave, 128 MB per launch at 256 resident
//     workgroups): pass p loads the fragments of units computed in earlier passes into the set it
//     writes, computes the blocks holding degree-p units, and stores their halves for later passes
//     (the last pass stores nothing).  A store is issued one ring stage after its block when the
//     fragment's registers survive that long (known at compile time), so the ring barrier's
//     vmcnt(0) does not wait for store acknowledgements issued just before it;
//   * a persistent grid (one 4-wave workgroup per CU, 64 rows per weight stream) walks the
//     (draw, row-tile) space, so the scratch is sized by the grid, not by the batch.
// Per pass p, layer i >= 2: blocks blo(p) .. bhi(p) over the previous layer's kt(p) k-steps; the
// output unit: the (mean, log_scale) rows of dim perm[p]; then x[perm[p]] = (y - mean) exp(-clamp(ls))
// on every quarter (pyro AffineAutoregressive._inverse), as made_ar_r16_kernel's affine epilogue.
#pragma once

#ifndef NAZ_HD
#define NAZ_HD __host__ __device__ inline
#endif

namespace naz {

template <class G>
struct CfgARIW {
  static constexpr int D = G::D, C = G::C, H = G::H, K = G::K, NHID = G::NHID, P = G::P;
  static constexpr bool AFFINE = G::AFFINE;
  static constexpr int HP = G::HP, HB = G::HB, KSH = G::KSH, KC = G::KC, KI = G::KI, OT = G::OT;
  static constexpr int NOB = 1, NW = 4;
  static_assert(AFFINE && P <= 16 && NHID >= 2, "wide inverse: affine MADE with >= 2 hidden layers");
  static constexpr int deg(int u) { return G::deg(u); }
  static constexpr int pad(int n) { return G::pad(n); }
  static constexpr int MAXU = D * (NHID * HB + 1);
  struct Layout {
    int E[32];
    int up[MAXU], ui[MAXU], ub[MAXU];  // unit: pass, sub-layer (NHID = output rows), 16-unit block
    int sid[MAXU], off[MAXU], sz[MAXU];
    int sfl[MAXU], sfu[MAXU], scnt[MAXU];  // per stage: floats (padded), first unit, unit count
    int nu, nstg, stg, maxcnt;
  };
  static constexpr int kt_of(const Layout& y, int p) { return (y.E[p] + 31) / 32; }
  static constexpr Layout make_layout() {
    Layout y{};
    int cnt[32] = {};
    for (int u = 0; u < H; ++u) ++cnt[deg(u) < 0 ? 0 : deg(u)];
    for (int p = 0, run = 0; p < D; ++p) y.E[p] = run += cnt[p];
    int n = 0;
    for (int p = 0; p < D; ++p) {
      const int ep = y.E[p], em = p > 0 ? y.E[p - 1] : 0;
      const int bhi = ep > 0 ? (ep - 1) >> 4 : -1;
      for (int i = 0; i < NHID; ++i) {
        // layer 1: every block of degree <= p (recomputed); deeper layers: the blocks holding
        // degree-p units (none when the pass has no units)
        const int blo = i == 0 ? 0 : (ep > em ? em >> 4 : bhi + 1);
        for (int b = blo; b <= bhi; ++b) {
          y.up[n] = p, y.ui[n] = i, y.ub[n] = b;
          y.sz[n] = (i == 0 ? KI : kt_of(y, p)) * OT + 16;
          ++n;
        }
      }
      y.up[n] = p, y.ui[n] = NHID, y.ub[n] = 0;
      y.sz[n] = NOB * kt_of(y, p) * OT + 16 * NOB;
      ++n;
    }
    y.nu = n;
    int s = -1, run = 0;
    for (int u = 0; u < n; ++u) {
      if (u == 0 || run + y.sz[u] > kARCap) {
        ++s;
        run = 0;
        y.sfu[s] = u;
      }
      y.sid[u] = s;
      y.off[u] = run;
      run += y.sz[u];
      y.sfl[s] = pad(run);
      ++y.scnt[s];
    }
    y.nstg = s + 1;
    for (int t = 0; t < y.nstg; ++t) {
      y.stg = y.sfl[t] > y.stg ? y.sfl[t] : y.stg;
      y.maxcnt = y.scnt[t] > y.maxcnt ? y.scnt[t] : y.maxcnt;
    }
    return y;
  }
  static constexpr Layout LY = make_layout();
  static constexpr int NU = LY.nu, NSTG = LY.nstg, STG = LY.stg, MAXCNT = LY.maxcnt;
  static constexpr int E(int p) { return p < 0 ? 0 : LY.E[p]; }
  static constexpr int kt(int p) { return kt_of(LY, p); }
  // first block of layer >= 2 recomputed in pass p (its fragment's other half may be older)
  static constexpr int blo(int p) { return E(p - 1) >> 4; }
  // fragments of a layer >= 2 loaded from scratch at the start of pass p: those holding any unit of
  // an earlier pass's blocks, i.e. blocks < blo(p) (the boundary fragment's other half is recomputed)
  static constexpr int oldt(int p) { return p == 0 ? 0 : (blo(p) + 1) >> 1; }
  static constexpr int unit_kts(int u) { return LY.ui[u] == 0 ? KI : (LY.ui[u] == NHID ? NOB * kt(LY.up[u]) : kt(LY.up[u])); }
  // a block of layer i >= 2 is stored for later passes (never in the last pass); deferred to the
  // start of the next stage when no later unit of its stage overwrites its register set (only
  // the same sub-layer, the next one and the output rows of the same pass may follow)
  static constexpr bool stores(int u) { return LY.ui[u] >= 1 && LY.ui[u] < NHID && LY.up[u] < D - 1; }
  static constexpr bool deferred(int u) {
    if (!stores(u)) return false;
    for (int w = u + 1; w < NU && LY.sid[w] == LY.sid[u]; ++w)
      if (LY.up[w] != LY.up[u] || !(LY.ui[w] == LY.ui[u] || LY.ui[w] == LY.ui[u] + 1 || LY.ui[w] == NHID))
        return false;
    return LY.sid[u] + 1 < NSTG;  // a next stage of the same layer exists
  }
  static constexpr int PERM_OFF = NSTG * STG;
  static constexpr int LAYER = pad(PERM_OFF + D);
  // per-wave scratch: layers 2 .. NHID, KSH fragments each, 64 lanes x (hi, lo) u32x4
  static constexpr int64_t SCRATCH_U4 = (int64_t)(NHID - 1) * KSH * 128;
  static_assert(2 * STG * 4 <= 160 * 1024, "two weight stages exceed the LDS");
  static_assert(NU <= MAXU && D <= 32, "layout");
};

// value of word-slot (m, kg, j) of fragment t of unit u (dim dp for the output rows); wv(i, idx) =
// the masked weight idx of sub-layer i in the flat layout (made_ar_pack_layer's)
template <class CF, class WV>
NAZ_HD float ariw_weight(int u, int t, int m, int kg, int j, int dp, const WV& wv) {
  constexpr int D = CF::D, C = CF::C, H = CF::H, P = CF::P;
  const int i = CF::LY.ui[u], b = CF::LY.ub[u];
  if (i == CF::NHID) {
    const int pi = m, v = r16_feat(t, kg, j);
    return (pi < P && v < H) ? -2.f * wv(i, ((int64_t)pi * D + dp) * H + v) : 0.f;
  }
  const int un = 16 * b + m;
  if (un >= H) return 0.f;
  if (i > 0) {
    const int v = r16_feat(t, kg, j);
    return v < H ? -2.f * kSigScale * wv(i, (int64_t)un * H + v) : 0.f;
  }
  if (t < CF::KC) {
    const int col = 32 * t + 8 * kg + j;
    return col < C ? kSigScale * wv(0, (int64_t)un * (C + D) + col) : 0.f;
  }
  const int d = 8 * kg + j;
  return d < D ? kSigScale * wv(0, (int64_t)un * (C + D) + C + d) : 0.f;
}

// bias slot r (0..15) of unit u: bv(i, idx) = bias idx of sub-layer i
template <class CF, class BV>
NAZ_HD float ariw_bias(int u, int r, int dp, const BV& bv) {
  const int i = CF::LY.ui[u], b = CF::LY.ub[u];
  if (i == CF::NHID) return r < CF::P ? bv(i, r * CF::D + dp) : 0.f;
  const int un = 16 * b + r;
  return un < CF::H ? kSigScale * bv(i, un) : 0.f;
}

template <class CF>
struct ARIWFlat {  // sub-layer offsets of one layer's flat rows (made_ar_pack_layer's layout)
  static constexpr int64_t w_off(int i) {
    int64_t o = 0;
    for (int j = 0; j < i; ++j) o += (int64_t)CF::H * (j == 0 ? CF::C + CF::D : CF::H) + CF::H;
    return o;
  }
  static constexpr int64_t b_off(int i) {
    return w_off(i) + (int64_t)(i < CF::NHID ? CF::H : CF::D * CF::P) * (i == 0 ? CF::C + CF::D : CF::H);
  }
  static constexpr int64_t per() { return w_off(CF::NHID) + (int64_t)CF::D * CF::P * (CF::H + 1); }
};

template <class CF>
static void made_ar_pack_wide_layer(const float* flat, const int* perm, float* out) {
  using F = ARIWFlat<CF>;
  unsigned* ou = reinterpret_cast<unsigned*>(out);
  for (int i = 0; i < CF::LAYER; ++i) out[i] = 0.f;
  auto wv = [&](int i, int64_t idx) { return flat[F::w_off(i) + idx]; };
  auto bv = [&](int i, int64_t idx) { return flat[F::b_off(i) + idx]; };
  for (int u = 0; u < CF::NU; ++u) {
    const int dp = perm[CF::LY.up[u]];
    const int base = CF::LY.sid[u] * CF::STG + CF::LY.off[u], kts = CF::unit_kts(u);
    for (int t = 0; t < kts; ++t)
      for (int piece = 0; piece < 2; ++piece)
        for (int lane = 0; lane < 64; ++lane)
          for (int pair = 0; pair < 4; ++pair) {
            unsigned w = 0;
            for (int e = 0; e < 2; ++e)
              w |= ar_piece(ariw_weight<CF>(u, t, lane & 15, lane >> 4, 2 * pair + e, dp, wv), piece) << (16 * e);
            ou[base + t * CF::OT + (piece * 64 + lane) * 4 + pair] = w;
          }
    for (int r = 0; r < 16 * CF::NOB; ++r) out[base + kts * CF::OT + r] = ariw_bias<CF>(u, r, dp, bv);
  }
  for (int p = 0; p < CF::D; ++p) reinterpret_cast<int*>(out)[CF::PERM_OFF + p] = perm[p];
}

// device packer: thread = one 32-bit word of one layer image (blockIdx.y = layer, blockIdx.z = draw),
// flat / perm / mask as made_ar_pack_kernel's (no pass-0 constants: the wide inverse has none)
template <class CF>
__global__ void made_ar_pack_wide_kernel(const float* __restrict__ flat, int64_t sflat, const int* __restrict__ perm,
                                         float* __restrict__ packed, int64_t spk, const float* __restrict__ mask) {
  using F = ARIWFlat<CF>;
  const int pos = blockIdx.x * blockDim.x + threadIdx.x;
  if (pos >= CF::LAYER) return;
  const int l = blockIdx.y;
  const float* f = flat + blockIdx.z * sflat + (int64_t)l * F::per();
  const float* mk = mask == nullptr ? nullptr : mask + (int64_t)l * F::per();
  const int* pm = perm + l * CF::D;
  unsigned* out = reinterpret_cast<unsigned*>(packed + blockIdx.z * spk + (int64_t)l * CF::LAYER);
  if (pos >= CF::PERM_OFF) {
    out[pos] = pos - CF::PERM_OFF < CF::D ? (unsigned)pm[pos - CF::PERM_OFF] : 0u;
    return;
  }
  auto wv = [&](int i, int64_t idx) {
    const int64_t o = F::w_off(i) + idx;
    return mk == nullptr ? f[o] : f[o] * mk[o];
  };
  auto bv = [&](int i, int64_t idx) { return f[F::b_off(i) + idx]; };
  const int s = pos / CF::STG, o = pos % CF::STG;
  unsigned word = 0;
  for (int k = 0; k < CF::LY.scnt[s]; ++k) {
    const int u = CF::LY.sfu[s] + k, rel = o - CF::LY.off[u];
    if (rel < 0 || rel >= CF::LY.sz[u]) continue;
    const int dp = pm[CF::LY.up[u]], kts = CF::unit_kts(u);
    if (rel >= kts * CF::OT) {
      word = __builtin_bit_cast(unsigned, ariw_bias<CF>(u, rel - kts * CF::OT, dp, bv));
    } else {
      const int t = rel / CF::OT, w = rel % CF::OT;
      const int piece = w / 256, lane = (w % 256) / 4, pair = w % 4;
      for (int e = 0; e < 2; ++e)
        word |= ar_piece_dev(ariw_weight<CF>(u, t, lane & 15, lane >> 4, 2 * pair + e, dp, wv), piece) << (16 * e);
    }
    break;
  }
  out[pos] = word;  // stage padding stays 0
}

template <class CF>
__global__ void __launch_bounds__(64 * CF::NW, 1) made_ar_inv_wide_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ out_lp, int64_t B, int64_t ndraw, int64_t spk, int64_t sx, int64_t slp,
    u32x4* __restrict__ scratch, float* __restrict__ states) {
  constexpr int D = CF::D, NW = CF::NW, NHID = CF::NHID, KSH = CF::KSH;
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + CF::STG;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  // this wave's scratch as a buffer resource: one VGPR offset (lane * 16) for every access and the
  // fragment offset in soffset — per-fragment 64-bit addresses were hoisted out of the loops by
  // the compiler and held (2 VGPRs per fragment of every layer: spills at n_hidden = 5)
  const int wave_u = __builtin_amdgcn_readfirstlane(wave);
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      scratch + ((int64_t)blockIdx.x * NW + wave_u) * CF::SCRATCH_U4, 0, (int)(CF::SCRATCH_U4 * 16), 0x00020000);
  const int voff = lane * 16;
  const int64_t ntile = (B + 16 * NW - 1) / (16 * NW), total = ntile * ndraw;

  // hidden layer i's B fragments in hf[i & 1] (zeroed per layer: finite, as every value that
  // ever lands there)
  Frag2 hf[2][KSH];

  int64_t gt = blockIdx.x;
  if (gt < total) stage_issue<CF::LY.sfl[0], NW>(slot0, packed + (gt / ntile) * spk + (int64_t)(L - 1) * CF::LAYER);
  int g = 0;
  for (; gt < total; gt += gridDim.x) {
    const int64_t dz = gt / ntile, tile = gt % ntile;
    const float* const pk = packed + dz * spk;
    const int64_t ngt = gt + gridDim.x;
    const float* const pk_next = ngt < total ? packed + (ngt / ntile) * spk + (int64_t)(L - 1) * CF::LAYER : nullptr;
    const int64_t row = tile * (16 * NW) + wave * 16 + (lane & 15);
    const bool valid = row < B;
    const int64_t crow = valid ? row : 0;
    const float* xr = x + dz * sx;

    float v[D];
    float logjac = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) v[d] = valid ? xr[crow * ldx + d] : 0.f;
    if (low != nullptr) {  // naz bounding_transform (transforms.py:20-23)
#pragma unroll
      for (int d = 0; d < D; ++d) {
        const float lo = low[d], hi = high[d];
        const float u = (v[d] - lo) / (hi - lo);
        logjac -= logf(u) + log1pf(-u) + logf(hi - lo);
        v[d] = logf(u / (1.f - u));
      }
    }
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
    float ldsum = 0.f;
    for (int li = 0; li < L; ++li) {
      const int l = L - 1 - li;
      const float* lp = pk + (int64_t)l * CF::LAYER;
      const float* lnext = li + 1 < L ? pk + (int64_t)(l - 1) * CF::LAYER : pk_next;
      const int* perm = reinterpret_cast<const int*>(lp + CF::PERM_OFF);
      int dps[D];
#pragma unroll
      for (int p = 0; p < D; ++p) dps[p] = __builtin_amdgcn_readfirstlane(perm[p]);
      float xmax = 0.f;
#pragma unroll
      for (int d = 0; d < D; ++d) xmax = fmaxf(xmax, fabsf(v[d]));
      // fresh sets per layer: nothing in them is carried across the layer loop's back edge
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
        for (int t = 0; t < KSH; ++t) hf[s2][t] = Frag2{half8{}, half8{}};
      const float* cur = slot0;
      Frag2 xf;
      float us = 1.f;
      // the half of fragment (i, b >> 1) written by block b of layer i >= 2, to scratch
      auto store_half = [&](auto uc) {
        constexpr int u = decltype(uc)::value, i = CF::LY.ui[u], b = CF::LY.ub[u];
        const Frag2& f = hf[i & 1][b >> 1];
        const u32x4 H4 = __builtin_bit_cast(u32x4, f.h), L4 = __builtin_bit_cast(u32x4, f.l);
        constexpr int w0 = 2 * (b & 1), fo = ((i - 1) * KSH + (b >> 1)) * 2048 + 8 * (b & 1);
        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{H4[w0], H4[w0 + 1]}, srs, voff, fo, 0);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{L4[w0], L4[w0 + 1]}, srs, voff, fo + 1024, 0);
      };
      static_for<0, CF::NU>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        constexpr int p = CF::LY.up[u], i = CF::LY.ui[u], b = CF::LY.ub[u];
        constexpr int SID = CF::LY.sid[u], OFF = CF::LY.off[u], KT = CF::kt(p);
        constexpr bool NEW_STAGE = u == 0 || SID != CF::LY.sid[u > 0 ? u - 1 : 0];
        constexpr bool FIRST_OF_SUB = u == 0 || CF::LY.up[u > 0 ? u - 1 : 0] != p || CF::LY.ui[u > 0 ? u - 1 : 0] != i;
        if constexpr (NEW_STAGE) {  // stage SID has landed in slot (g & 1)
          ring_barrier();           // ... and every wave is done with the other slot
          cur = (g & 1) ? slot1 : slot0;
          float* nxt = (g & 1) ? slot0 : slot1;
          if constexpr (SID + 1 < CF::NSTG) {
            stage_issue<CF::LY.sfl[SID + 1], NW>(nxt, lp + (SID + 1) * CF::STG);
          } else {
            if (lnext != nullptr) stage_issue<CF::LY.sfl[0], NW>(nxt, lnext);
          }
          ++g;
          // the previous stage's deferred stores, a whole stage ahead of the next barrier
          if constexpr (SID > 0) {
            static_for<0, CF::MAXCNT>([&](auto kc) {
              constexpr int k = decltype(kc)::value;
              constexpr int w = CF::LY.sfu[SID - 1] + k;
              if constexpr (k < CF::LY.scnt[SID - 1]) {
                if constexpr (CF::deferred(w)) store_half(std::integral_constant<int, w>{});
              }
            });
          }
        }
        const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
        auto afrag = [&](int idx) {
          const int base = (OFF >> 2) + idx * 128 + lane;
          return Frag2{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
        };
        const float4* bias4 = reinterpret_cast<const float4*>(cur + OFF + CF::unit_kts(u) * CF::OT);
        // this unit's A fragments (byte address of fragment 0 for this lane), for the prefetched
        // MFMA chains (mfma3_16_chain_lds: one wave per SIMD has nothing else to hide LDS reads)
        const unsigned ub = (unsigned)(uintptr_t)to_lds(cur) + 16u * lane + 4u * OFF;
        if constexpr (i == 0 && FIRST_OF_SUB) {
          // the row's values split at a per-row power-of-two scale, |x| sc < 2^14 (the inverse maps
          // grow values by up to e^5 per layer; xmax: max |v| at the layer's start and since)
          const int e = xmax >= 16384.f ? __builtin_amdgcn_frexp_expf(xmax) - 14 : 0;
          const float sc = __builtin_amdgcn_ldexpf(1.f, -e);
          us = __builtin_amdgcn_ldexpf(1.f, e);
          float x8[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float s = 0.f;
#pragma unroll
            for (int qq = 0; qq < 4; ++qq)
              if (8 * qq + j < D) s = q == qq ? v[8 * qq + j] : s;
            x8[j] = s * sc;
          }
          xf = split8_f16(x8);
        }
        if constexpr (i >= 1 && i < NHID && FIRST_OF_SUB && CF::oldt(p) > 0) {
          // this layer's fragments from earlier passes into the set it is written to (the boundary
          // fragment first: the first new block completes its other half).  Pinned here: hoisted
          // above the previous sub-layer's MFMAs they would be live beside the set those still
          // read (+128 VGPRs: spills)
          __builtin_amdgcn_sched_barrier(0);
          static_for<0, CF::oldt(p)>([&](auto tc) {
            constexpr int t = CF::oldt(p) - 1 - decltype(tc)::value;
            constexpr int fo = ((i - 1) * KSH + t) * 2048;
            hf[i & 1][t] = Frag2{__builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(srs, voff, fo, 0)),
                                 __builtin_bit_cast(half8, __builtin_amdgcn_raw_buffer_load_b128(srs, voff, fo + 1024, 0))};
          });
        }
        if constexpr (i < NHID) {
          const float4 bv = bias4[q];
          floatx4 acc = floatx4{bv.x, bv.y, bv.z, bv.w};
          if constexpr (i == 0) {
#pragma unroll
            for (int t = 0; t < CF::KC; ++t) acc = mfma3_16(afrag(t), cf[t], acc);
            const floatx4 ax = mfma3_16(afrag(CF::KC), xf, floatx4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[r] = __builtin_fmaf(ax[r], us, acc[r]);
          } else {
            acc = mfma3_16_chain_lds<KT>(ub, hf[(i - 1) & 1], acc);
          }
          ar_split4<b & 1>(hf[i & 1][b >> 1], acc);
          if constexpr (CF::stores(u) && !CF::deferred(u)) store_half(uc);
        } else {
          // the output rows of dim d_p: (mean, log_scale) in registers 0, 1 of quarter 0
          const float4 bv = bias4[q];
          floatx4 o3 = floatx4{bv.x, bv.y, bv.z, bv.w};
          o3 = mfma3_16_chain_lds<KT>(ub, hf[(NHID - 1) & 1], o3);
          const int dp = dps[p];
          const float y = v[dp];
          const float mean = __shfl(o3[0], lane & 15);
          const float ls = fminf(fmaxf(__shfl(o3[1], lane & 15), -5.f), 3.f);
          v[dp] = (y - mean) * __expf(-ls);
          xmax = fmaxf(xmax, fabsf(v[dp]));
          ldsum += ls;
        }
      });
      // the training forward: layer l's output s_l [L, B, D] (one draw) for the wide maf backward
      if (states != nullptr && q == 0 && valid) {
#pragma unroll
        for (int d = 0; d < D; ++d) states[((int64_t)l * B + row) * D + d] = v[d];
      }
    }
    constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
    float base = 0.f;
#pragma unroll
    for (int d = 0; d < D; ++d) base += -(v[d] * v[d]) / 2.f - kLogSqrt2Pi;
    if (q == 0 && valid) out_lp[dz * slp + row] = base - ldsum + logjac;
  }
}

}  // namespace naz
