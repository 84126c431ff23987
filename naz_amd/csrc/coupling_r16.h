// 16-row-wave variant of the fused coupling flow (NAZ_MFMA_F16X3_R16; included by coupling.hip,
// which supplies split8_f16, f16_piece_bits, sig_fold, kSigScale, stage_issue, kChunk, ...).
//
// Why: the 32-row x6 kernel keeps each activation block in a 32x32 accumulator (16 VGPRs per
// feature block) and needs ~250 VGPRs, i.e. two waves per SIMD; PMC shows ~28 % of its cycles
// with neither the matrix nor the vector pipe busy.  Here every wave owns 16 batch rows and
// every GEMM runs on v_mfma_f32_16x16x32_f16 (same FLOP per cycle as 32x32x16): a 16-feature
// block costs 4 VGPRs per lane, the whole live set fits 128 VGPRs and FOUR waves share each
// SIMD (512-thread workgroups of 128 rows, two per CU, the same 2 x 40 KB LDS ring per
// workgroup).
//
// Lane l owns batch row (l & 15) and quarter q = l >> 4 of that row's dims: lower dims
// [q*SQ, q*SQ + SQ) and upper dims [q*DQ, q*DQ + DQ) (S, D - S multiples of 4).
//   * accumulator register i of block b on quarter q = feature 16b + 4q + i (16x16 C layout);
//   * B operand of a 32-k step t on quarter q, element j = k-slot 8q + j; the packer maps that
//     slot to feature 32t + 16(j >> 2) + 4q + (j & 3), i.e. the lane's OWN accumulator
//     registers of blocks 2t, 2t + 1 — layers chain with no LDS and no shuffles;
//   * GEMM3's rows are permuted so quarter q receives, in (block, register) order, the 3K-1
//     parameters of its own DQ upper dims;
//   * GEMM1's k-slots put quarter q's x1 dims (which only that lane computes) in its own
//     slots of the last k-step; the context fills the other slots (loaded from HBM/L2).
// Precision: fp16 hi/lo pieces, 3 products (Wh·Xh + Wh·Xl + Wl·Xh) as in the x6 kernel's
// f16x3 GEMM2/3.  GEMM1 takes that path when every context/data value of the workgroup's rows
// is below 2^15; otherwise the workgroup runs GEMM1 in EXACT fp32 (v_mfma_f32_16x16x4_f32,
// a second stage-A image of the same size).  Activation fold, select-first spline and LDS-DMA
// ring as in coupling_x6_kernel.
#pragma once

namespace naz {

typedef float floatx4 __attribute__((ext_vector_type(4)));

NAZ_DEV floatx4 mfma16_f16(half8 a, half8 b, floatx4 c) { return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0); }
NAZ_DEV floatx4 mfma16_f32(float a, float b, floatx4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

NAZ_DEV floatx4 mfma3_16(const Frag2& a, const Frag2& b, floatx4 acc) {
  acc = mfma16_f16(a.l, b.h, acc);  // small terms first
  acc = mfma16_f16(a.h, b.l, acc);
  acc = mfma16_f16(a.h, b.h, acc);
  return acc;
}

// GEMM stages run at wave priority 1, the splines at 0: a SIMD's matrix pipe is fed first
// and the spline VALU of the other waves fills the MFMA issue gaps (+0.5 %, same-box A/B).
// NAZ_R16_STATIC_PRIO (experiment): no per-stage flips; the second-dispatched half of the workgroup
// (waves 4-7, the arbitration losers) runs at priority 1 for the whole kernel (MI355X_MICROARCH.md,
// "two waves per SIMD" item 4).
#if defined(NAZ_R16_NO_PRIO) || defined(NAZ_R16_STATIC_PRIO)
#define R16_PRIO(p) ((void)0)
#else
#define R16_PRIO(p) __builtin_amdgcn_s_setprio(p)
#endif

#ifndef NAZ_R16_WAVES
#define NAZ_R16_WAVES 8
#endif
constexpr int kR16Waves = NAZ_R16_WAVES;     // 8 waves x 16 rows = 128 rows per workgroup
constexpr int kR16Rows = 16 * kR16Waves;

// feature carried by k-slot 8q + j of 32-k step t (GEMM2/3 inputs)
__host__ __device__ constexpr int r16_feat(int t, int q, int j) { return 32 * t + 16 * (j >> 2) + 4 * q + (j & 3); }

template <int D_, int C_, int S_, int K_, int H_, bool LOWER_>
struct CfgR16 {
  static constexpr int D = D_, C = C_, S = S_, K = K_, H = H_;
  static constexpr bool LOWER = LOWER_;
  static constexpr int Dt = D - S, P = 3 * K - 1, DQ = Dt / 4, SQ = S / 4;
  static constexpr int HB = H / 16;                    // 16-feature blocks
  static constexpr int KS1 = (C + S + 31) / 32;        // GEMM1 32-k steps
  static constexpr int KS2 = H / 32;                   // GEMM2/3 32-k steps
  static constexpr int NO = (DQ * P + 3) / 4;          // GEMM3 output blocks
  static constexpr int TBL = 3 * (K + 1);
  static constexpr int OT = 2 * kChunk;                // floats per (block, k-step): hi + lo pieces
  static constexpr int pad(int n) { return (n + 255) / 256 * 256; }
  static constexpr int pick_kb(int nb, int bias) {
    int best = 1;
    for (int kb = 1; kb <= KS2; ++kb)
      if (KS2 % kb == 0 && pad(nb * kb * OT + bias) <= kX6Slot) best = kb;
    return best;
  }
  static constexpr int KB2 = pick_kb(HB, H), NB2 = KS2 / KB2;
  // GEMM3 in two halves of NO/2 output blocks (SPLIT3, two upper dims per quarter): half 0 holds
  // every parameter of dim 0, so dim 0's spline can run beside half 1's MFMAs, and half 1 reuses
  // half 0's B fragments instead of the GEMM2 accumulators
#ifdef NAZ_R16_NOSPLIT3
  static constexpr bool SPLIT3 = false;
#else
  static constexpr bool SPLIT3 = DQ == 2 && NO % 2 == 0 && (P + 3) / 4 <= NO / 2;
#endif
  static constexpr int NOC = SPLIT3 ? NO / 2 : NO;     // output blocks per GEMM3 stage
  static constexpr int KB3 = pick_kb(NOC, 16 * NO), NB3H = KS2 / KB3, NB3 = (SPLIT3 ? 2 : 1) * NB3H;
  // stage A (fp16 image; the fp32 image A32 has the same size and bias/table offsets):
  //   [HB][KS1][2][256] | bias [H] | tables [S][TBL]
  static constexpr int A_BIAS = HB * KS1 * OT;
  static constexpr int A_TBL = A_BIAS + H;
  static constexpr int A_SIZE = pad(A_TBL + S * TBL);
  static constexpr int B_OFF = A_SIZE;
  static constexpr int B_BIAS = HB * KB2 * OT;
  static constexpr int B_SIZE = pad(B_BIAS + H);
  static constexpr int C_OFF = B_OFF + NB2 * B_SIZE;
  static constexpr int C_BIAS = NOC * KB3 * OT;
  static constexpr int C_SIZE = pad(C_BIAS + 16 * NO);
  static constexpr int A32_OFF = C_OFF + NB3 * C_SIZE;
  static constexpr int LAYER = A32_OFF + A_SIZE;
  static constexpr int NSTG = 1 + NB2 + NB3;
  static constexpr int MAXSTAGE = 2 * kX6Slot;
  static constexpr __host__ __device__ int stage_off(int j) {
    return j == 0 ? 0 : (j <= NB2 ? B_OFF + (j - 1) * B_SIZE : C_OFF + (j - 1 - NB2) * C_SIZE);
  }
  static constexpr __host__ __device__ int stage_size(int j) { return j == 0 ? A_SIZE : (j <= NB2 ? B_SIZE : C_SIZE); }
  // natural flat layout (same as every other coupling variant)
  static constexpr int N_W0 = H * (C + S), N_B0 = H, N_W1 = H * H, N_B1 = H, N_W2 = Dt * P * H, N_B2 = Dt * P;
  static constexpr int N_LOW = LOWER ? S * (3 * K - 1) : 0;
  static constexpr int FLAT = N_W0 + N_B0 + N_W1 + N_B1 + N_W2 + N_B2 + N_LOW;
  static_assert(S % 4 == 0 && Dt % 4 == 0 && H % 32 == 0 && S > 0 && SQ <= 8, "unsupported r16 coupling shape");
  static_assert(A_SIZE <= kX6Slot && B_SIZE <= kX6Slot && C_SIZE <= kX6Slot, "stage exceeds one LDS ring slot");
  static_assert(HB <= 8 && NO <= 16, "register budget");
};

// GEMM1 input column for k-slot j of 32-k step t on quarter q (cat([ctx, x1]) order), -1 = pad.
// Quarter q's own x1 dims sit in slots j < SQ of the last step; the context fills the rest.
template <class CF>
__host__ __device__ constexpr int r16_in_col(int t, int q, int j) {
  constexpr int TX = CF::KS1 - 1;
  if (t == TX && j < CF::SQ) return CF::C + q * CF::SQ + j;
  int idx = 0;
  if (t < TX) idx = 32 * t + 8 * q + j;
  else idx = 32 * TX + q * (8 - CF::SQ) + (j - CF::SQ);
  return idx < CF::C ? idx : -1;
}

// DenseNN output column of GEMM3 output row r (0..15) of block o; -1 = pad
template <class CF>
__host__ __device__ constexpr int r16_out_row(int o, int r) {
  const int q = r >> 2, slot = 4 * o + (r & 3), dq = slot / CF::P, p = slot - dq * CF::P;
  if (dq >= CF::DQ) return -1;
  const int dim = q * CF::DQ + dq;
  if (p < CF::K) return dim * CF::K + p;
  if (p < 2 * CF::K) return CF::Dt * CF::K + dim * CF::K + (p - CF::K);
  return 2 * CF::Dt * CF::K + dim * (CF::K - 1) + (p - 2 * CF::K);
}

template <class CF>
__global__ void coupling_pack_r16_kernel(const float* __restrict__ flat, float* __restrict__ packed, int L,
                                         float bound) {
  const int64_t n = (int64_t)L * CF::LAYER;
  unsigned* pu = reinterpret_cast<unsigned*>(packed);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(e / CF::LAYER);
    const int off = (int)(e - (int64_t)l * CF::LAYER);
    const float* W0 = flat + (int64_t)l * CF::FLAT;
    const float* b0 = W0 + CF::N_W0;
    const float* W1 = b0 + CF::N_B0;
    const float* b1 = W1 + CF::N_W1;
    const float* W2 = b1 + CF::N_B1;
    const float* b2 = W2 + CF::N_W2;
    const float* low = b2 + CF::N_B2;
    // f16 chunk word: (o, t, piece, lane, pair) -> two fp16 pieces of the scaled weight
    auto chunk_word = [&](int q, int nt, int t0, int which, int obase = 0) -> unsigned {
      const int o = q / (nt * CF::OT), r1 = q - o * nt * CF::OT;
      const int tl = r1 / CF::OT, r2 = r1 - tl * CF::OT;
      const int piece = r2 / kChunk, u = r2 - piece * kChunk;
      const int lane = u >> 2, pair = u & 3, i = lane & 15, qq = lane >> 4;
      const int t = t0 + tl;
      unsigned out = 0;
      for (int e2 = 0; e2 < 2; ++e2) {
        const int j = 2 * pair + e2;
        float v = 0.f;
        if (which == 0) {
          const int col = r16_in_col<CF>(t, qq, j);
          v = col >= 0 ? kSigScale * W0[(16 * o + i) * (CF::C + CF::S) + col] : 0.f;
        } else if (which == 1) {
          v = -2.f * kSigScale * W1[(16 * o + i) * CF::H + r16_feat(t, qq, j)];
        } else {
          const int orow = r16_out_row<CF>(obase + o, i);
          v = orow >= 0 ? -2.f * W2[orow * CF::H + r16_feat(t, qq, j)] : 0.f;
        }
        out |= f16_piece_bits(v, piece) << (16 * e2);
      }
      return out;
    };
    unsigned word = 0;
    float fv = 0.f;
    bool is_word = false;
    const bool a32 = off >= CF::A32_OFF;
    if (off < CF::A_SIZE || a32) {
      const int oa = a32 ? off - CF::A32_OFF : off;
      if (oa < CF::A_BIAS) {
        if (!a32) {
          word = chunk_word(oa, CF::KS1, 0, 0);
          is_word = true;
        } else {
          // fp32 image [o][s4][lane][4]: k-step s = 4 s4 + i of v_mfma_f32_16x16x4_f32 on quarter
          // lane >> 4 carries the fp16 path's slot (t = s / 8, j = s % 8)
          const int i4 = oa & 3, lane = (oa >> 2) & 63, rest = oa >> 8;
          const int s4 = rest % (2 * CF::KS1), o = rest / (2 * CF::KS1);
          const int s = 4 * s4 + i4;
          const int col = r16_in_col<CF>(s / 8, lane >> 4, s % 8);
          fv = col >= 0 ? kSigScale * W0[(16 * o + (lane & 15)) * (CF::C + CF::S) + col] : 0.f;
        }
      } else if (oa < CF::A_TBL) {
        fv = kSigScale * b0[oa - CF::A_BIAS];
      } else if (CF::LOWER && oa < CF::A_TBL + CF::S * CF::TBL) {
        const int q = oa - CF::A_TBL, g = q / CF::TBL, w = q - g * CF::TBL;
        float uw[CF::K], uh[CF::K], ud[CF::K - 1];
        for (int k = 0; k < CF::K; ++k) {
          uw[k] = low[g * CF::K + k];
          uh[k] = low[CF::S * CF::K + g * CF::K + k];
        }
        for (int k = 0; k < CF::K - 1; ++k) ud[k] = low[2 * CF::S * CF::K + g * (CF::K - 1) + k];
        SplineTables<CF::K> tb;
        build_tables<CF::K>(uw, uh, ud, bound, tb);
        const int which = w / (CF::K + 1), k = w - which * (CF::K + 1);
        fv = which == 0 ? tb.cw[k] : (which == 1 ? tb.ch[k] : tb.dv[k]);
      }
    } else if (off < CF::C_OFF) {
      const int sq = (off - CF::B_OFF) / CF::B_SIZE, q = off - CF::B_OFF - sq * CF::B_SIZE;
      if (q < CF::B_BIAS) {
        word = chunk_word(q, CF::KB2, sq * CF::KB2, 1);
        is_word = true;
      } else if (q < CF::B_BIAS + CF::H) {
        fv = kSigScale * b1[q - CF::B_BIAS];
      }
    } else {
      const int sq = (off - CF::C_OFF) / CF::C_SIZE, q = off - CF::C_OFF - sq * CF::C_SIZE;
      if (q < CF::C_BIAS) {
        const int hh = sq / CF::NB3H, s2 = sq - hh * CF::NB3H;
        word = chunk_word(q, CF::KB3, s2 * CF::KB3, 2, hh * CF::NOC);
        is_word = true;
      } else if (q < CF::C_BIAS + 16 * CF::NO) {
        const int r = q - CF::C_BIAS, orow = r16_out_row<CF>(r >> 4, r & 15);
        fv = orow >= 0 ? b2[orow] : 0.f;
      }
    }
    if (is_word) pu[e] = word;
    else packed[e] = fv;
  }
}

// acc[o] += A(o, t) · B(t) over k-steps [0, KB), t outer, o inner, with each A fragment read one
// MFMA triple ahead (untracked LDS reads with counted waits, coupling.hip lds_read_b128_untracked):
// for kernels with too few waves per SIMD to hide an LDS read behind other waves' work (the
// training backward: two).  bfn(t) returns k-step t's B fragment (formed inside the loop, so the
// lazy forms' activation VALU still lands between MFMAs).
template <int NB, int KB, class BFn>
NAZ_DEV void gemm_r16_pf(floatx4 (&acc)[NB], const float* __restrict__ stage, int lane, BFn&& bfn) {
  static_assert(2 * NB * KB * 1024 <= 65536, "A fragment offsets must fit the 16-bit LDS offset");
  const unsigned ub = (unsigned)(uintptr_t)to_lds(stage) + 16u * lane;
  auto rd = [&](auto oc, auto tc) {
    constexpr int off = ((decltype(oc)::value * KB + decltype(tc)::value) * 2) * 1024;
    return Frag2{__builtin_bit_cast(half8, lds_read_b128_untracked<off>(ub)),
                 __builtin_bit_cast(half8, lds_read_b128_untracked<off + 1024>(ub))};
  };
  Frag2 an = rd(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  static_for<0, KB>([&](auto tc) {
    constexpr int t = decltype(tc)::value;
    const Frag2 b = bfn(tc);
    static_for<0, NB>([&](auto oc) {
      constexpr int o = decltype(oc)::value;
      const Frag2 a = an;
      if constexpr (o + 1 < NB || t + 1 < KB) {
        an = rd(std::integral_constant<int, (o + 1 < NB ? o + 1 : 0)>{},
                std::integral_constant<int, (o + 1 < NB ? t : t + 1)>{});
        __builtin_amdgcn_sched_barrier(0);
        lds_wait<2>();
      } else {
        __builtin_amdgcn_sched_barrier(0);
        lds_wait<0>();
      }
      __builtin_amdgcn_sched_barrier(0);
      acc[o] = mfma3_16(a, b, acc[o]);
    });
  });
}

// acc[o] += A(o, t) · B(t) over k-steps [0, KB) with B fragments given (PF: gemm_r16_pf)
template <int NB, int KB, bool PF = false>
NAZ_DEV void gemm_r16_stage(floatx4 (&acc)[NB], const float* __restrict__ stage, int lane, const Frag2 (&bf)[KB]) {
#ifdef NAZ_ABL_NOGEMM
  for (int o = 0; o < NB; ++o) acc[o][0] += (float)bf[0].h[0] * 1e-30f;
  return;
#endif
  if constexpr (PF) {
    gemm_r16_pf<NB, KB>(acc, stage, lane, [&](auto tc) -> Frag2 { return bf[decltype(tc)::value]; });
    return;
  }
  const u32x4* c4 = reinterpret_cast<const u32x4*>(stage);
#pragma unroll
  for (int t = 0; t < KB; ++t)
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int base = ((o * KB + t) * 2) * 64 + lane;
      const Frag2 a{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      acc[o] = mfma3_16(a, bf[t], acc[o]);
    }
}

// k-steps [T0, T0 + KB) with each B fragment split from the activated accumulators just
// before its MFMAs (blocks 2t, 2t + 1 hold the step's 8 values).  ACT: the step's 8 values are
// activated here too (sig_fold), so that work can fill the previous step's MFMA shadow.
template <int NB, int KB, int T0, bool ACT, int NX, bool PF = false>
NAZ_DEV void gemm_r16_lazy(floatx4 (&acc)[NB], const float* __restrict__ stage, int lane, floatx4 (&x)[NX]) {
  if constexpr (PF) {
    gemm_r16_pf<NB, KB>(acc, stage, lane, [&](auto tc) -> Frag2 {
      constexpr int t = decltype(tc)::value;
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int blk = 2 * (T0 + t) + (j >> 2);
        v[j] = blk < NX ? x[blk < NX ? blk : 0][j & 3] : 0.f;
        if constexpr (ACT) v[j] = sig_fold(v[j]);
      }
      return split8_f16(v);
    });
    return;
  }
  const u32x4* c4 = reinterpret_cast<const u32x4*>(stage);
#pragma unroll
  for (int t = 0; t < KB; ++t) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int blk = 2 * (T0 + t) + (j >> 2);  // past the last block (odd NX): zero k-slots
      v[j] = blk < NX ? x[blk < NX ? blk : 0][j & 3] : 0.f;
      if constexpr (ACT) v[j] = sig_fold(v[j]);
    }
    const Frag2 b = split8_f16(v);
#ifdef NAZ_ABL_NOGEMM
    for (int o = 0; o < NB; ++o) acc[o][0] += (float)b.h[0] * 1e-30f;
    continue;
#endif
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int base = ((o * KB + t) * 2) * 64 + lane;
      const Frag2 a{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      acc[o] = mfma3_16(a, b, acc[o]);
    }
  }
}

// GEMM3 stage s: k-steps [T0, T0 + KB3) of output blocks [OB, OB + NOC) (OB = half · NOC).
// Half 0 forms each k-step's B fragment from the GEMM2 accumulators (ACT: activated here) and
// keeps it in f3; half 1 reads f3.  Bias from the stage's bias block at the half's first stage.
template <class CF, int s, bool ACT, int NX>
NAZ_DEV void gemm3_stage(floatx4 (&acc)[CF::NO], const float* __restrict__ cur, int lane, int q, floatx4 (&x)[NX],
                         Frag2 (&f3)[CF::KS2]) {
  constexpr int h = s / CF::NB3H, s2 = s % CF::NB3H, T0 = s2 * CF::KB3, OB = h * CF::NOC;
  if constexpr (s2 == 0) {
    const float4* b4 = reinterpret_cast<const float4*>(cur + CF::C_BIAS);
#pragma unroll
    for (int o = 0; o < CF::NOC; ++o) {
      const float4 bv = b4[4 * (OB + o) + q];
      acc[OB + o] = floatx4{bv.x, bv.y, bv.z, bv.w};
    }
  }
  const u32x4* c4 = reinterpret_cast<const u32x4*>(cur);
#pragma unroll
  for (int t = 0; t < CF::KB3; ++t) {
    if constexpr (h == 0) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int blk = 2 * (T0 + t) + (j >> 2);
        v[j] = blk < NX ? x[blk < NX ? blk : 0][j & 3] : 0.f;
        if constexpr (ACT) v[j] = sig_fold(v[j]);
      }
      f3[T0 + t] = split8_f16(v);
    }
#ifdef NAZ_ABL_NOGEMM
    for (int o = 0; o < CF::NOC; ++o) acc[OB + o][0] += (float)f3[T0 + t].h[0] * 1e-30f;
    continue;
#endif
#pragma unroll
    for (int o = 0; o < CF::NOC; ++o) {
      const int base = ((o * CF::KB3 + t) * 2) * 64 + lane;
      const Frag2 a{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      acc[OB + o] = mfma3_16(a, f3[T0 + t], acc[OB + o]);
    }
  }
}

// Training forward (VAR = 1, coupling_train.h): the log_prob walk of the NLL step with the
// reference walk's libm-grade activation and spline (tanh_f / build_tables + rqs_apply, not
// the hardware-transcendental fold and select-first spline) and every layer's input state
// written to states[l + 1][row][:] (states[0] = z), for the backward kernel to recompute from.
// The GEMMs keep the f16x3 split.  Activated values are -tanh/2 (the fold's convention), so the
// packed image is the same.
constexpr float kInvSigScale = 0.34657359027997264f;  // 1 / kSigScale = ln 2 / 2
// Training kernels' math: by default the fused inference kernel's own (sigmoid-fold activation,
// select-first spline on hardware transcendentals, table lower spline), so the NLL step's loss is
// the log_prob the metric kernel computes.  NAZ_TRAIN_ACCURATE: libm-grade tanh and spline.
#ifdef NAZ_TRAIN_ACCURATE
constexpr bool kTrainFast = false;
#else
constexpr bool kTrainFast = true;
#endif
NAZ_DEV float acc_fold(float v) { return -0.5f * tanh_f<kTrainFast>(v * kInvSigScale); }

// waves per SIMD: the training forward (VAR = 1) as inference, 4 (128 VGPRs, 12 B of scratch at
// config 3); NAZ_R16_TRAIN_W2: 2, the round-2 form (A/B)
#ifdef NAZ_R16_TRAIN_W2
#define NAZ_R16_TRAIN_WAVES_PER_SIMD_SEL(VAR) ((VAR) == 0 ? 4 : 2)
#else
#define NAZ_R16_TRAIN_WAVES_PER_SIMD_SEL(VAR) 4
#endif
template <class CF, bool DIR_INV, int VAR = 0>
__global__ void __launch_bounds__(kR16Rows * 4, NAZ_R16_TRAIN_WAVES_PER_SIMD_SEL(VAR)) coupling_r16_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ out_lp, float* __restrict__ yout, int64_t ldy, int64_t B, float bound,
    float* __restrict__ states = nullptr, int layer_ld_mode = NAZ_LD_ROWSUM) {
  // VAR 2 (naz_coupling_layer_{fwd,inv}): ONE layer (`packed` at its image, L = 1), y to yout and
  // the layer's FORWARD log|det J| per row to out_lp by layer_ld_mode (=, +=, -=); no base density
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + kX6Slot;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  const int64_t row = (int64_t)blockIdx.x * kR16Rows + wave * 16 + (lane & 15);
  const bool valid = row < B;
  const int64_t crow = valid ? row : 0;
#ifdef NAZ_R16_STATIC_PRIO
  if (wave >= kR16Waves / 2) __builtin_amdgcn_s_setprio(1);
#endif

  float zl[CF::SQ], zu[CF::DQ];
  float ldsum = 0.f, logjac = 0.f;
#pragma unroll
  for (int u = 0; u < CF::SQ; ++u) zl[u] = valid ? x[crow * ldx + q * CF::SQ + u] : 0.f;
#pragma unroll
  for (int u = 0; u < CF::DQ; ++u) zu[u] = valid ? x[crow * ldx + CF::S + q * CF::DQ + u] : 0.f;
  if (DIR_INV && low != nullptr) {  // naz bounding_transform (transforms.py:20-23)
    auto bnd = [&](float& v, int dim) {
      const float lo = low[dim], hi = high[dim];
      const float u = (v - lo) / (hi - lo);
      logjac -= logf(u) + log1pf(-u);
      v = logf(u / (1.f - u));
    };
#pragma unroll
    for (int u = 0; u < CF::SQ; ++u) bnd(zl[u], q * CF::SQ + u);
#pragma unroll
    for (int u = 0; u < CF::DQ; ++u) bnd(zu[u], CF::S + q * CF::DQ + u);
    if (q == 0) {
      float sl = 0.f;
      for (int d = 0; d < CF::D; ++d) sl += logf(high[d] - low[d]);
      logjac -= sl;
    }
  }

  // GEMM1 precision path of this workgroup (see the file comment); reduced through ring slot 1
  bool ok = bound < kG1F16Limit;
#pragma unroll
  for (int u = 0; u < CF::SQ; ++u) ok = ok && fabsf(zl[u]) < kG1F16Limit;
#pragma unroll
  for (int u = 0; u < CF::DQ; ++u) ok = ok && fabsf(zu[u]) < kG1F16Limit;
#pragma unroll
  for (int t = 0; t < CF::KS1; ++t)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = r16_in_col<CF>(t, q, j);
      if (col >= 0 && col < CF::C) ok = ok && fabsf(ctx[crow * ldc + col]) < kG1F16Limit;
    }
  {
    int* flags = reinterpret_cast<int*>(slot1);
    if (lane == 0) flags[wave] = __all(ok) ? 1 : 0;
    __syncthreads();
    bool all_ok = true;
#pragma unroll
    for (int w = 0; w < kR16Waves; ++w) all_ok = all_ok && flags[w] != 0;
    ok = all_ok;
  }
  const bool g1f16 = ok;
  const int a_off = g1f16 ? 0 : CF::A32_OFF;

  const RingSrc ring(packed, (int64_t)L * CF::LAYER);
  stage_issue<CF::A_SIZE, kR16Waves>(slot0, ring, (DIR_INV ? (L - 1) : 0) * CF::LAYER + a_off);

  const RqsConsts<CF::K, DIR_INV> rc(bound);
  // GEMM1's context k-slots of this lane, loaded for layer li + 1 before layer li's upper spline
  // (and for layer 0 here).  vmcnt retires in order: a context load issued AFTER a stage's
  // LDS-DMA (as when it sits in stage A) can only be waited for together with that DMA, so
  // stage A would stall on stage B's weights (3 % of the kernel, same-box A/B).  Issued before
  // the stage-A barrier, the barrier's vmcnt(0) covers them with the stage-A weights.
  float cpre[CF::KS1 * 8];
  auto load_ctx = [&]() {
#pragma unroll
    for (int t = 0; t < CF::KS1; ++t)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int col = r16_in_col<CF>(t, q, jj);
        cpre[8 * t + jj] = (col >= 0 && col < CF::C) ? ctx[crow * ldc + col] : 0.f;
      }
  };
  load_ctx();
  int g = 0;  // global stage counter: stage g lives in slot (g & 1)
  for (int li = 0; li < L; ++li) {
    const int l = DIR_INV ? (L - 1 - li) : li;
    if constexpr (VAR == 1) {  // layer l's input state P[l + 1]
      if (valid) {
        float* st = states + ((int64_t)(l + 1) * B + row) * CF::D;
#pragma unroll
        for (int u = 0; u < CF::SQ; ++u) st[q * CF::SQ + u] = zl[u];
#pragma unroll
        for (int u = 0; u < CF::DQ; ++u) st[CF::S + q * CF::DQ + u] = zu[u];
      }
    }
    floatx4 acc1[CF::HB], acc2[CF::HB], acc3[CF::NO];
    Frag2 f3[CF::KS2];  // GEMM3's B fragments (half 0 forms them, half 1 reuses them)
    // upper spline on this quarter's dim u (parameters in acc3 slots u P .. u P + P - 1)
    auto upper = [&](auto uc) {
      constexpr int u = decltype(uc)::value;
      float uw[CF::K], uh[CF::K], ud[CF::K - 1];
#pragma unroll
      for (int k = 0; k < CF::K; ++k) {
        constexpr int b0 = u * CF::P;
        uw[k] = acc3[(b0 + k) >> 2][(b0 + k) & 3];
        uh[k] = acc3[(b0 + CF::K + k) >> 2][(b0 + CF::K + k) & 3];
      }
#pragma unroll
      for (int k = 0; k < CF::K - 1; ++k) {
        constexpr int b0 = u * CF::P + 2 * CF::K;
        ud[k] = acc3[(b0 + k) >> 2][(b0 + k) & 3];
      }
      float ld;
#ifdef NAZ_ABL_NOSPLINE
      if constexpr (VAR == 0) {
        float sacc = 0.f;
#pragma unroll
        for (int k = 0; k < CF::K; ++k) sacc += uw[k] + uh[k];
        zu[u] += 1e-30f * sacc;
        return;
      }
#endif
      if constexpr (VAR == 1 && !kTrainFast) {
        SplineTables<CF::K> tb;
        build_tables<CF::K, kTrainFast>(uw, uh, ud, bound, tb);
        zu[u] = rqs_apply<CF::K, DIR_INV, kTrainFast>(tb, zu[u], bound, ld);
        ldsum += DIR_INV ? -ld : ld;
      } else {
        zu[u] = rqs_select<CF::K, DIR_INV>(uw, uh, ud, zu[u], bound, rc, ld);
        ldsum += DIR_INV ? -ld : ld;
      }
    };

    static_for<0, CF::NSTG>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
#ifndef NAZ_ABL_NOBARRIER
      ring_barrier();  // stage j has landed in slot (g&1); every wave is done with the other slot
#endif
      const float* cur = (g & 1) ? slot1 : slot0;
      float* nxt = (g & 1) ? slot0 : slot1;
      if constexpr (j + 1 < CF::NSTG) {
        stage_issue<CF::stage_size(j + 1), kR16Waves>(nxt, ring, l * CF::LAYER + CF::stage_off(j + 1));
      } else {
        if (li + 1 < L) stage_issue<CF::A_SIZE, kR16Waves>(nxt, ring, (DIR_INV ? (l - 1) : (l + 1)) * CF::LAYER + a_off);
      }
      ++g;

      if constexpr (j == 0) {
        // ---------------- stage A: lower spline (inverse), GEMM1 over [ctx | x1]
#pragma unroll
        for (int u = 0; u < CF::SQ; ++u) {
#ifdef NAZ_ABL_NOLOWER
          if constexpr (false) {
#else
          if constexpr (DIR_INV && CF::LOWER) {
#endif
            float ld;
            if constexpr (VAR == 1 && !kTrainFast) {
              SplineTables<CF::K> tb;
              const float* tp = cur + CF::A_TBL + (q * CF::SQ + u) * CF::TBL;
#pragma unroll
              for (int k = 0; k <= CF::K; ++k) {
                tb.cw[k] = tp[k];
                tb.ch[k] = tp[CF::K + 1 + k];
                tb.dv[k] = tp[2 * (CF::K + 1) + k];
              }
              zl[u] = rqs_apply<CF::K, true, kTrainFast>(tb, zl[u], bound, ld);
              ldsum -= ld;  // ldsum carries the forward maps' log-dets (rqs_apply: the inverse's)
            } else {
              zl[u] = rqs_table<CF::K, true>(cur + CF::A_TBL + (q * CF::SQ + u) * CF::TBL, zl[u], bound, ld);
              ldsum -= ld;
            }
          }
        }
        float in[CF::KS1 * 8];
#pragma unroll
        for (int t = 0; t < CF::KS1; ++t)
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const int col = r16_in_col<CF>(t, q, jj);
            float v = 0.f;
            if (col >= CF::C) v = zl[(col - CF::C - q * CF::SQ) < CF::SQ ? (col - CF::C - q * CF::SQ) : 0];
            else if (col >= 0) v = cpre[8 * t + jj];
            in[8 * t + jj] = v;
          }
        {
          const float4* b4 = reinterpret_cast<const float4*>(cur + CF::A_BIAS);
#pragma unroll
          for (int o = 0; o < CF::HB; ++o) {
            const float4 bv = b4[4 * o + q];
            acc1[o] = floatx4{bv.x, bv.y, bv.z, bv.w};
          }
        }
#ifdef NAZ_R16_NO_F32_G1
        if (true) {
#else
        if (g1f16) {
#endif
          Frag2 bf[CF::KS1];
#pragma unroll
          for (int t = 0; t < CF::KS1; ++t) {
            float v[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] = in[8 * t + jj];
            bf[t] = split8_f16(v);
          }
          R16_PRIO(1);
          gemm_r16_stage<CF::HB, CF::KS1>(acc1, cur, lane, bf);
          R16_PRIO(0);
        } else {
          // exact fp32: 8 KS1 k-steps of 4; k-step s on this lane = slot (s / 8, s % 8)
          const float4* p4 = reinterpret_cast<const float4*>(cur);
#pragma unroll
          for (int s4 = 0; s4 < 2 * CF::KS1; ++s4)
#pragma unroll
            for (int o = 0; o < CF::HB; ++o) {
              const float4 a = p4[(o * 2 * CF::KS1 + s4) * 64 + lane];
              acc1[o] = mfma16_f32(a.x, in[4 * s4 + 0], acc1[o]);
              acc1[o] = mfma16_f32(a.y, in[4 * s4 + 1], acc1[o]);
              acc1[o] = mfma16_f32(a.z, in[4 * s4 + 2], acc1[o]);
              acc1[o] = mfma16_f32(a.w, in[4 * s4 + 3], acc1[o]);
            }
        }
        if constexpr (!DIR_INV && CF::LOWER) {
#pragma unroll
          for (int u = 0; u < CF::SQ; ++u) {
            float ld;
            zl[u] = rqs_table<CF::K, false>(cur + CF::A_TBL + (q * CF::SQ + u) * CF::TBL, zl[u], bound, ld);
            ldsum += ld;
          }
        }
      } else if constexpr (j <= CF::NB2) {
        // ---------------- stage B_s: GEMM2 k-steps [T0, T0 + KB2)
        constexpr int s = j - 1, T0 = s * CF::KB2;
#ifdef NAZ_R16_EAGER_ACT
#pragma unroll
        for (int b = 2 * T0; b < 2 * (T0 + CF::KB2); ++b)  // activate the blocks these k-steps read
#pragma unroll
          for (int r = 0; r < 4; ++r) acc1[b][r] = sig_fold(acc1[b][r]);
        constexpr bool kLazyAct = false;
#else
#ifdef NAZ_ABL_NOTANH
        constexpr bool kLazyAct = false, kNoAct = true;
#else
        constexpr bool kLazyAct = VAR == 0 || kTrainFast, kNoAct = false;  // activated per k-step inside gemm_r16_lazy
#endif
        if constexpr (!kLazyAct && !kNoAct) {
#pragma unroll
          for (int b = 2 * T0; b < 2 * (T0 + CF::KB2); ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc1[b][r] = acc_fold(acc1[b][r]);
        }
#endif
        if constexpr (s == 0) {
          const float4* b4 = reinterpret_cast<const float4*>(cur + CF::B_BIAS);
#pragma unroll
          for (int o = 0; o < CF::HB; ++o) {
            const float4 bv = b4[4 * o + q];
            acc2[o] = floatx4{bv.x, bv.y, bv.z, bv.w};
          }
        }
        R16_PRIO(1);
        gemm_r16_lazy<CF::HB, CF::KB2, T0, kLazyAct>(acc2, cur, lane, acc1);
        R16_PRIO(0);
      } else {
        // ---------------- stage C_s: GEMM3 (two halves of output blocks when SPLIT3)
        constexpr int s = j - 1 - CF::NB2, T0s = (s % CF::NB3H) * CF::KB3;
#ifdef NAZ_ABL_NOTANH
        constexpr bool kLazyAct = false, kNoAct = true;
#else
        constexpr bool kLazyAct = VAR == 0 || kTrainFast, kNoAct = false;
#endif
        if constexpr (!kLazyAct && !kNoAct && s < CF::NB3H) {  // accurate training forward: eager
#pragma unroll
          for (int b = 2 * T0s; b < 2 * (T0s + CF::KB3); ++b)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc2[b][r] = acc_fold(acc2[b][r]);
        }
        constexpr bool kHost = CF::SPLIT3 && s == CF::NB3H;  // first stage of half 1: dim 0's spline
        if constexpr (!kHost) R16_PRIO(1);
        gemm3_stage<CF, s, kLazyAct>(acc3, cur, lane, q, acc2, f3);
        if constexpr (!kHost) R16_PRIO(0);
        // dim 0's spline in the stage that issues half 1's MFMAs (the compiler still issues the
        // MFMAs first: measured the same as NAZ_R16_NOSPLIT3, also with sched_group_barrier pins)
        if constexpr (kHost) upper(std::integral_constant<int, 0>{});
      }
    });

    // ---------------- upper spline on this quarter's remaining dims (next layer's stage A in flight)
    if (li + 1 < L) load_ctx();
    static_for<CF::SPLIT3 ? 1 : 0, CF::DQ>([&](auto uc) { upper(uc); });
#ifdef NAZ_DEBUG_NONFINITE
    {
      bool fin = isfinite(ldsum);
#pragma unroll
      for (int u = 0; u < CF::SQ; ++u) fin = fin && isfinite(zl[u]);
#pragma unroll
      for (int u = 0; u < CF::DQ; ++u) fin = fin && isfinite(zu[u]);
      debug_nonfinite_probe(valid && !fin, row, li, g);
    }
#endif
  }
  if constexpr (VAR == 1) {  // P[0] = z
    if (valid) {
      float* st = states + row * CF::D;
#pragma unroll
      for (int u = 0; u < CF::SQ; ++u) st[q * CF::SQ + u] = zl[u];
#pragma unroll
      for (int u = 0; u < CF::DQ; ++u) st[CF::S + q * CF::DQ + u] = zu[u];
    }
  }

  if constexpr (VAR == 2) {
    if (valid) {
#pragma unroll
      for (int u = 0; u < CF::SQ; ++u) yout[row * ldy + q * CF::SQ + u] = zl[u];
#pragma unroll
      for (int u = 0; u < CF::DQ; ++u) yout[row * ldy + CF::S + q * CF::DQ + u] = zu[u];
    }
    float v = ldsum;
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (q == 0 && valid) {
      if (layer_ld_mode == NAZ_LD_ROWSUM_ADD) out_lp[row] += v;
      else if (layer_ld_mode == NAZ_LD_ROWSUM_SUB) out_lp[row] -= v;
      else out_lp[row] = v;
    }
  } else if constexpr (DIR_INV) {
    constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
    float base = 0.f;
#pragma unroll
    for (int u = 0; u < CF::SQ; ++u) base += -(zl[u] * zl[u]) / 2.f - kLogSqrt2Pi;
#pragma unroll
    for (int u = 0; u < CF::DQ; ++u) base += -(zu[u] * zu[u]) / 2.f - kLogSqrt2Pi;
    float v = base - ldsum + logjac;
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    if (q == 0 && valid) out_lp[row] = v;
  } else {
    if (low != nullptr) {
#pragma unroll
      for (int u = 0; u < CF::SQ; ++u) {
        const int d = q * CF::SQ + u;
        zl[u] = (1.f / (1.f + expf(-zl[u]))) * (high[d] - low[d]) + low[d];
      }
#pragma unroll
      for (int u = 0; u < CF::DQ; ++u) {
        const int d = CF::S + q * CF::DQ + u;
        zu[u] = (1.f / (1.f + expf(-zu[u]))) * (high[d] - low[d]) + low[d];
      }
    }
    if (valid) {
#pragma unroll
      for (int u = 0; u < CF::SQ; ++u) yout[row * ldy + q * CF::SQ + u] = zl[u];
#pragma unroll
      for (int u = 0; u < CF::DQ; ++u) yout[row * ldy + CF::S + q * CF::DQ + u] = zu[u];
    }
    if (out_lp != nullptr) {
      float v = ldsum;
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      if (q == 0 && valid) out_lp[row] = v;
    }
  }
}

}  // namespace naz
