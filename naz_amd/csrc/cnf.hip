// Fused FFJORD solve: one launch integrates a whole continuous-flow block (SURVEY.md §8a row
// a11, config 5).
//
// Reference semantics: naz FFJORDTransform (naz/flows/continuous_transforms.py:70-106) =
// torchdyn CNF(net, trace_estimator=hutch_trace) on the augmented state [a, x]:
//     dx/dt = f(x, ctx),   da/dt = -eps^T (df/dx) eps      (eps ~ N(0, I) fixed per solve)
// f = ConditionalFCNN (continuous_transforms.py:38-60): Linear/act chain, input cat([x, ctx]).
// Solver pinned by SURVEY.md §8d: fixed-step classical RK4 in the form of naz's in-tree
// odeint.py:12-19,46-52 (k_i = dt f(.), x += (k1 + 2k2 + 2k3 + k4) / 6).
//
// MI355X mapping:
//   * the reference takes eps^T J with a reverse-mode VJP per RHS evaluation (autograd graph,
//     ~3x the MLP forward); here it is a FORWARD-mode JVP carried alongside the values:
//     every layer computes pre = W h + b and dpre = W dh with the SAME weight operand, so
//     J eps costs one extra MFMA per weight read and eps^T (J eps) is a per-row dot product;
//   * one workgroup per CU (8 waves) keeps the whole vector-field MLP in LDS (config 5:
//     37k fp32 = 146 KB of 160 KB) for the kernel's lifetime and walks row tiles
//     persistently — weights are read from HBM once per CU, not once per RHS evaluation;
//   * a wave owns 16 rows; activations live TRANSPOSED in v_mfma_f32_16x16x4_f32
//     accumulators (lane l: feature 4(l>>4)+i of a 16-block, row l&15).  Accumulator
//     register i of block b IS the B operand of k-step (b, i) of the next layer (B[k=l>>4]
//     [j=l&15]), so the layers chain with no LDS or shuffles; the packer permutes W
//     columns to match, and the last layer's rows so its output lands in the lane layout of
//     the ODE state (lane l: state feature (l>>4) + 4s in register s);
//   * all RK4 stages, the state, eps and the trace accumulator stay in registers: HBM sees
//     x, ctx, eps in and y, ld out once per solve.
// Exact fp32 MFMA (bitwise an fmaf chain); activations on the hardware transcendentals.
#include "naz_device.h"
#include "naz_internal.h"

namespace naz {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef _Float16 cnf_half8 __attribute__((ext_vector_type(8)));
typedef unsigned int cnf_u32x4 __attribute__((ext_vector_type(4)));

NAZ_DEV floatx4 mfma16(float a, float b, floatx4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// ---- fp16x3 (NAZ_CNF_F16X3): W = Wh + Wl (round-to-nearest pieces, packed), v = vh + vl
// (round-to-nearest pieces, exact residual, on the fly), W·v ≈ Wl·vh + Wh·vl + Wh·vh on
// v_mfma_f32_16x16x32_f16 — fp32-grade products at 3 × 16 cycles per 16x16x32 block instead of
// 8 × 32 cycles of v_mfma_f32_16x16x4_f32.  Activations/tangents whose wave maximum reaches
// kCnfF16Limit are scaled by an exact power of two around the GEMM (rare path).
struct CnfFrag2 {
  cnf_half8 h, l;
};

NAZ_DEV floatx4 mfma16h(cnf_half8 a, cnf_half8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

NAZ_DEV floatx4 mfma16x3(const CnfFrag2& a, const CnfFrag2& b, floatx4 acc) {
  acc = mfma16h(a.l, b.h, acc);
  acc = mfma16h(a.h, b.l, acc);
  acc = mfma16h(a.h, b.h, acc);
  return acc;
}

template <bool HI>
NAZ_DEV float cnf_sub_piece(float v, unsigned hp) {
  float r;
  if constexpr (HI)
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(v));
  else
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(v));
  return r;
}

typedef _Float16 cnf_half2 __attribute__((ext_vector_type(2)));

// two floats -> packed fp16 pair, round-to-nearest-even (one v_cvt_pk_f16_f32 on gfx950).  The
// activation/tangent split rounds to nearest on both pieces: the trace estimate accumulates
// products over the whole solve, and round-toward-zero pieces bias it (measured: ld error
// median 3.8e-6 with RTZ pieces on a [32, 32] field).
NAZ_DEV unsigned cnf_pack2(float a, float b) {
  const cnf_half2 h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, h);
}

NAZ_DEV CnfFrag2 cnf_split8(const float (&v)[8]) {
  cnf_u32x4 H, Lo;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned hp = cnf_pack2(v[2 * q], v[2 * q + 1]);
    const float r0 = cnf_sub_piece<false>(v[2 * q], hp), r1 = cnf_sub_piece<true>(v[2 * q + 1], hp);
    H[q] = hp;
    Lo[q] = cnf_pack2(r0, r1);
  }
  return CnfFrag2{__builtin_bit_cast(cnf_half8, H), __builtin_bit_cast(cnf_half8, Lo)};
}

// fp16 piece of a weight (0 = round-to-nearest hi, 1 = lo = fp16(W - hi))
NAZ_DEV unsigned cnf_f16_piece(float v, int piece) {
  const _Float16 hi = (_Float16)v;
  if (piece == 0) return (unsigned)__builtin_bit_cast(unsigned short, hi);
  const _Float16 lo = (_Float16)(v - (float)hi);
  return (unsigned)__builtin_bit_cast(unsigned short, lo);
}

// input feature carried by k-slot 8q + j of 32-k step t: the lane's own accumulator registers
// of blocks 2t, 2t + 1 (16x16 C layout: register i of block b on quarter q = feature 16b+4q+i)
__host__ __device__ constexpr int cnf_feat32(int t, int q, int j) { return 32 * t + 16 * (j >> 2) + 4 * q + (j & 3); }

constexpr float kCnfF16Limit = 16384.f;

constexpr int cnf_up(int v, int m) { return (v + m - 1) / m * m; }
constexpr int cnf_max(int a, int b) { return a > b ? a : b; }

// LDS image layout (floats): [W0][b0][W1][b1]...[W_last][b_last]; layer-0 weights are
// [NB0][KS0/4][64][4], later layers [NBout][NBin][64][4] (one ds_read_b128 = 4 k-steps).
constexpr int cnf_hid(int j, int h0, int h1, int h2, int h3) { return j == 0 ? h0 : j == 1 ? h1 : j == 2 ? h2 : h3; }
constexpr int cnf_wsize(int j, int ks0, int h0, int h1, int h2, int h3) {
  return j == 0 ? cnf_hid(0, h0, h1, h2, h3) / 16 * ks0 * 64
                : cnf_hid(j, h0, h1, h2, h3) / 16 * (cnf_hid(j - 1, h0, h1, h2, h3) / 16) * 256;
}
// non-recursive on purpose: every use must fold to a constant (a recursive constexpr helper
// called outside a constant expression becomes a real device call with an unbounded stack)
constexpr int cnf_offw(int j, int ks0, int h0, int h1, int h2, int h3) {
  int off = 0;
  for (int i = 0; i < j; ++i) off += cnf_wsize(i, ks0, h0, h1, h2, h3) + cnf_hid(i, h0, h1, h2, h3);
  return off;
}

template <int D_, int C_, int H0_, int H1_, int H2_, int H3_, int ACT_>
struct CnfCfg {
  static constexpr int D = D_, C = C_, ACT = ACT_;
  static constexpr int NH = (H0_ > 0) + (H1_ > 0) + (H2_ > 0) + (H3_ > 0);
  static constexpr int XS = cnf_up(D, 4) / 4;     // state / eps registers per lane
  static constexpr int CS = cnf_up(C, 4) / 4;     // context registers per lane
  static constexpr int KS0 = cnf_up(XS + CS, 4);  // layer-0 k-steps (padded to a multiple of 4)
  static constexpr int NBL = cnf_up(D, 16) / 16;  // 16-blocks of the output layer
  static constexpr int NBMAX = cnf_max(cnf_max(H0_, H1_), cnf_max(H2_, H3_)) / 16;
  static constexpr int HL = cnf_hid(NH - 1, H0_, H1_, H2_, H3_);
  static constexpr int OFF_WL = cnf_offw(NH, KS0, H0_, H1_, H2_, H3_);
  static constexpr int WL_SIZE = NBL * (HL / 16) * 256;
  static constexpr int OFF_BL = OFF_WL + WL_SIZE;
  static constexpr int TOTAL = OFF_BL + NBL * 16;
  static constexpr int in0 = D + C;
  static_assert(NH >= 1 && H0_ % 16 == 0 && H1_ % 16 == 0 && H2_ % 16 == 0 && H3_ % 16 == 0, "hidden widths");
  static_assert(NBMAX <= 8, "hidden width <= 128 (register budget)");
  static_assert(TOTAL * 4 <= 160 * 1024, "vector-field MLP must fit one CU's LDS");
  static constexpr int hid(int j) { return cnf_hid(j, H0_, H1_, H2_, H3_); }
  static constexpr int NB(int j) { return hid(j) / 16; }
  static constexpr int off_w(int j) { return cnf_offw(j, KS0, H0_, H1_, H2_, H3_); }
  static constexpr int off_b(int j) { return off_w(j) + cnf_wsize(j, KS0, H0_, H1_, H2_, H3_); }
  // offset of W_j in the natural flat parameter vector (W_j [out, in] then b_j, layer by layer;
  // j == NH is the output layer)
  static constexpr int64_t flat_off_w(int j) {
    int64_t n = 0;
    int in = in0;
    for (int i = 0; i < j; ++i) {
      n += (int64_t)hid(i) * in + hid(i);
      in = hid(i);
    }
    return n;
  }
};

constexpr int kCnfWaves = 8, kCnfRows = 16 * kCnfWaves;

template <int I, int N, class F>
NAZ_DEV void cnf_static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    cnf_static_for<I + 1, N>(f);
  }
}

// ---------------------------------------------------------------------------
// Packing: natural flat parameters -> the LDS image (one thread per image float)
// ---------------------------------------------------------------------------
template <class CF, bool X3>
__global__ void cnf_pack_kernel(const float* __restrict__ flat, float* __restrict__ img) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= CF::TOTAL) return;
  float v = 0.f;
  // f16x3 word of a weight chunk [ob][t][piece][lane][pair]: rows via row_of(ob, lane & 15),
  // columns cnf_feat32(t, lane >> 4, j) of the layer's [rows, hin] weight at flat offset fo
  auto x3_word = [&](int r, int nbi, int64_t fo, int hin, auto row_of) -> unsigned {
    const int u = r & 255, chunk = r >> 8;
    const int piece = chunk & 1, rest = chunk >> 1, t = rest % (nbi / 2), ob = rest / (nbi / 2);
    const int lane = u >> 2, pair = u & 3;
    const int orow = row_of(ob, lane & 15);
    unsigned out = 0;
    for (int e2 = 0; e2 < 2; ++e2) {
      const int jj = 2 * pair + e2;
      const float w = orow >= 0 ? flat[fo + (int64_t)orow * hin + cnf_feat32(t, lane >> 4, jj)] : 0.f;
      out |= cnf_f16_piece(w, piece) << (16 * e2);
    }
    return out;
  };
  // layer 0 weights: [ob][s4][lane][i], k-step s = 4 s4 + i carries x feature q + 4s (s < XS)
  // or context feature q + 4(s - XS) (XS <= s < XS + CS), q = lane >> 4
  constexpr int OB0 = CF::off_b(0);
  if (e < OB0) {
    const int i = e & 3, lane = (e >> 2) & 63, rest = e >> 8;
    const int s4 = rest % (CF::KS0 / 4), ob = rest / (CF::KS0 / 4);
    const int s = 4 * s4 + i, o = 16 * ob + (lane & 15), q = lane >> 4;
    int col = -1;
    if (s < CF::XS) {
      const int f = q + 4 * s;
      col = f < CF::D ? f : -1;
    } else if (s < CF::XS + CF::CS) {
      const int f = q + 4 * (s - CF::XS);
      col = f < CF::C ? CF::D + f : -1;
    }
    if (col >= 0) v = flat[(int64_t)o * CF::in0 + col];
    img[e] = v;
    return;
  }
  bool done = false, word = false;
  cnf_static_for<0, CF::NH>([&](auto J) {
    constexpr int j = decltype(J)::value;
    if (done) return;
    constexpr int ob_ = CF::off_b(j), ow_ = CF::off_w(j);
    constexpr int nbi = CF::NB(j > 0 ? j - 1 : 0), hin = j == 0 ? CF::in0 : CF::hid(j > 0 ? j - 1 : 0);
    constexpr int hj = CF::hid(j);
    constexpr int64_t fo = CF::flat_off_w(j);
    if (j > 0 && e >= ow_ && e < ob_) {
      const int r = e - ow_;
      if constexpr (X3) {
        reinterpret_cast<unsigned*>(img)[e] = x3_word(r, nbi, fo, hin, [](int ob, int rl) { return 16 * ob + rl; });
        done = word = true;
        return;
      }
      const int i = r & 3, lane = (r >> 2) & 63, rest = r >> 8;
      const int b = rest % nbi, ob = rest / nbi;
      const int o = 16 * ob + (lane & 15), k = 16 * b + 4 * (lane >> 4) + i;
      v = flat[fo + (int64_t)o * hin + k];
      done = true;
    } else if (e >= ob_ && e < ob_ + hj) {
      v = flat[fo + (int64_t)hj * hin + (e - ob_)];
      done = true;
    }
  });
  if (word) return;
  if (!done) {
    constexpr int HL = CF::HL;
    constexpr int64_t fw = CF::flat_off_w(CF::NH);
    if (X3 && e >= CF::OFF_WL && e < CF::OFF_BL) {
      reinterpret_cast<unsigned*>(img)[e] = x3_word(e - CF::OFF_WL, HL / 16, fw, HL, [](int ob, int rl) {
        const int nf = (rl >> 2) + 4 * (4 * ob + (rl & 3));
        return nf < CF::D ? nf : -1;
      });
      return;
    }
    if (e < CF::OFF_BL) {  // output layer: packed row r_local = lane & 15 <-> state feature q_r + 4(4 ob + i_r)
      const int r = e - CF::OFF_WL;
      const int i = r & 3, lane = (r >> 2) & 63, rest = r >> 8;
      constexpr int nbl_in = CF::HL / 16;
      const int b = rest % nbl_in, ob = rest / nbl_in;
      const int rl = lane & 15, nf = (rl >> 2) + 4 * (4 * ob + (rl & 3));
      const int k = 16 * b + 4 * (lane >> 4) + i;
      if (nf < CF::D) v = flat[fw + (int64_t)nf * HL + k];
    } else {
      const int p = e - CF::OFF_BL, ob = p >> 4, rl = p & 15;
      const int nf = (rl >> 2) + 4 * (4 * ob + (rl & 3));
      if (nf < CF::D) v = flat[fw + (int64_t)CF::D * HL + nf];
    }
  }
  img[e] = v;
}

// value and tangent through the activation: v = act(pre), t <- t * act'(pre)
// (torch softplus: pre > 20 -> identity; backward grad * z / (z + 1), z = exp(pre))
// Hardware transcendentals (v_exp / v_log / v_rcp, ~1-2 ulp) with a Kahan log1p: ~10 VALU per
// element instead of ~40 for the libm forms; the MLP's MFMA rate makes this VALU the budget.
#ifndef NAZ_CNF_ACCURATE_ACT
template <int ACT>
NAZ_DEV void act_jvp(float& v, float& t) {
  const float pre = v;
  if constexpr (ACT == ACT_SOFTPLUS) {
    const float z = __builtin_amdgcn_exp2f(pre * 1.44269504088896341f);
    const float u = 1.f + z, d = u - 1.f;
    const float lp = d == 0.f ? z : __builtin_amdgcn_logf(u) * 0.693147180559945309f * (z * __builtin_amdgcn_rcpf(d));
    const bool big = pre > 20.f;  // torch softplus threshold: identity, gradient 1
    v = big ? pre : lp;
    t = big ? t : t * (z * __builtin_amdgcn_rcpf(u));
  } else if constexpr (ACT == ACT_TANH) {
    v = tanh_f<true>(pre);
    t = t * (1.f - v * v);
  } else if constexpr (ACT == ACT_RELU) {
    v = fmaxf(pre, 0.f);
    t = pre > 0.f ? t : 0.f;
  } else if constexpr (ACT == ACT_SIGMOID) {
    v = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-pre * 1.44269504088896341f));
    t = t * (v * (1.f - v));
  }
}
#else
template <int ACT>
NAZ_DEV void act_jvp(float& v, float& t) {
  const float pre = v;
  if constexpr (ACT == ACT_SOFTPLUS) {
    if (pre > 20.f) return;
    const float z = expf(pre);
    v = log1pf(z);
    t = (t * z) / (z + 1.f);
  } else if constexpr (ACT == ACT_TANH) {
    v = tanh_f(pre);
    t = t * (1.f - v * v);
  } else if constexpr (ACT == ACT_RELU) {
    v = fmaxf(pre, 0.f);
    t = pre > 0.f ? t : 0.f;
  } else if constexpr (ACT == ACT_SIGMOID) {
    v = 1.f / (1.f + expf(-pre));
    t = t * (v * (1.f - v));
  }
}
#endif

template <int NB>
NAZ_DEV void init_bias4(floatx4 (&ov)[8], floatx4 (&ot)[8], const float* bias, int q) {
#pragma unroll
  for (int ob = 0; ob < NB; ++ob) {
    ov[ob] = *reinterpret_cast<const floatx4*>(bias + 16 * ob + 4 * q);
    ot[ob] = floatx4{0.f, 0.f, 0.f, 0.f};
  }
}

template <int ACT, int NB>
NAZ_DEV void act_all(floatx4 (&ov)[8], floatx4 (&ot)[8]) {
#pragma unroll
  for (int ob = 0; ob < NB; ++ob)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v = ov[ob][i], t = ot[ob][i];
      act_jvp<ACT>(v, t);
      ov[ob][i] = v;
      ot[ob][i] = t;
    }
}

// one Linear between 16-blocked activations: (ov, ot) = W (iv, it) (+ b for the value)
template <int NBI, int NBO>
NAZ_DEV void cnf_linear(const float* __restrict__ W, const floatx4 (&iv)[8], const floatx4 (&it)[8],
                        floatx4 (&ov)[8], floatx4 (&ot)[8], int lane) {
#pragma unroll
  for (int b = 0; b < NBI; ++b) {
    // one input block at a time: its NBO weight reads, then 8·NBO MFMAs.  The barrier keeps
    // the scheduler from hoisting every block's ds_reads (64 x 4 VGPRs at H = 128) up front.
    floatx4 a4[NBO];
#pragma unroll
    for (int ob = 0; ob < NBO; ++ob) a4[ob] = *reinterpret_cast<const floatx4*>(W + ((ob * NBI + b) * 64 + lane) * 4);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int ob = 0; ob < NBO; ++ob) {
        ov[ob] = mfma16(a4[ob][i], iv[b][i], ov[ob]);
        ot[ob] = mfma16(a4[ob][i], it[b][i], ot[ob]);
      }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// the same Linear on the fp16x3 path: W chunks [NBO][NBI/2][piece][64 lanes][16 B]
template <int NBI, int NBO>
NAZ_DEV void cnf_linear_x3(const float* __restrict__ W, floatx4 (&iv)[8], floatx4 (&it)[8], floatx4 (&ov)[8],
                           floatx4 (&ot)[8], int lane) {
  // Exponent management for the fp16 pieces (exact powers of two, undone on the outputs):
  //   * tangents, per batch row (= MFMA column, the 4 lanes l & 15 of that row): scaled so the
  //     row's largest tangent lands in [2^14, 2^15).  Tangents span many decades and fp16's lo
  //     piece goes subnormal below 2^-14 (absolute step 2^-24), which would cap their relative
  //     precision; with the scaling every tangent within 2^-11 of its row maximum keeps ~22 bits;
  //   * activations, per batch row, only in waves where one reaches kCnfF16Limit (rare; bias
  //     pre-scaled).
  float mv = 0.f, mt = 0.f;
#pragma unroll
  for (int b = 0; b < NBI; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      mv = fmaxf(mv, fabsf(iv[b][i]));
      mt = fmaxf(mt, fabsf(it[b][i]));
    }
  mt = fmaxf(mt, __shfl_xor(mt, 16));
  mt = fmaxf(mt, __shfl_xor(mt, 32));
  int et = mt > 0.f ? 14 - ilogbf(mt) : 0;  // scaled row maximum in [2^14, 2^15)
  et = et > 100 ? 100 : (et < -100 ? -100 : et);
  const float st = ldexpf(1.f, et);
#pragma unroll
  for (int b = 0; b < NBI; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i) it[b][i] *= st;
  float sv = 1.f;
  const bool scaled = __builtin_amdgcn_ballot_w64(mv >= kCnfF16Limit) != 0;
  if (scaled) {  // per batch row, like the tangents (bias in the row's own accumulators)
    mv = fmaxf(mv, __shfl_xor(mv, 16));
    mv = fmaxf(mv, __shfl_xor(mv, 32));
    const int ev = mv >= kCnfF16Limit ? (mv > 1e30f ? 100 : ilogbf(mv) - 13) : 0;
    sv = ldexpf(1.f, -ev);
#pragma unroll
    for (int b = 0; b < NBI; ++b)
#pragma unroll
      for (int i = 0; i < 4; ++i) iv[b][i] *= sv;
#pragma unroll
    for (int ob = 0; ob < NBO; ++ob) ov[ob] *= sv;
  }
  const cnf_u32x4* c4 = reinterpret_cast<const cnf_u32x4*>(W);
#pragma unroll
  for (int t = 0; t < NBI / 2; ++t) {
    float v[8], tv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = iv[2 * t + (j >> 2)][j & 3];
      tv[j] = it[2 * t + (j >> 2)][j & 3];
    }
    const CnfFrag2 bv = cnf_split8(v), bt = cnf_split8(tv);
#pragma unroll
    for (int ob = 0; ob < NBO; ++ob) {
      const int base = ((ob * (NBI / 2) + t) * 2) * 64 + lane;
      const CnfFrag2 a{__builtin_bit_cast(cnf_half8, c4[base]), __builtin_bit_cast(cnf_half8, c4[base + 64])};
      ov[ob] = mfma16x3(a, bv, ov[ob]);
      ot[ob] = mfma16x3(a, bt, ot[ob]);
    }
    __builtin_amdgcn_sched_barrier(0);  // one k-step's fragment reads at a time (register budget)
  }
  const float it_ = ldexpf(1.f, -et);  // exact inverse scalings
#pragma unroll
  for (int ob = 0; ob < NBO; ++ob) ot[ob] *= it_;
  if (scaled) {
    const float iv_ = 1.f / sv;
#pragma unroll
    for (int ob = 0; ob < NBO; ++ob) ov[ob] *= iv_;
  }
}

template <bool X3, int NBI, int NBO>
NAZ_DEV void cnf_lin(const float* __restrict__ W, floatx4 (&iv)[8], floatx4 (&it)[8], floatx4 (&ov)[8],
                     floatx4 (&ot)[8], int lane) {
  if constexpr (X3) cnf_linear_x3<NBI, NBO>(W, iv, it, ov, ot, lane);
  else cnf_linear<NBI, NBO>(W, iv, it, ov, ot, lane);
}

// f(x) in the state layout and g = -eps^T (df/dx) eps (row total on every lane of the row)
template <class CF, bool X3>
NAZ_DEV void cnf_rhs(const float* __restrict__ lds, const float (&xin)[CF::XS], const float (&e)[CF::XS],
                     const float (&c)[CF::CS > 0 ? CF::CS : 1], float (&f)[CF::XS], float& g, int lane) {
  const int q = lane >> 4;
  floatx4 av[8], at[8], bv[8], bt[8];
  // layer 0: k-steps over [x | ctx | pad]
  {
    constexpr int NB0 = CF::NB(0), OW0 = CF::off_w(0), OB0 = CF::off_b(0);
    const float* W = lds + OW0;
    init_bias4<NB0>(av, at, lds + OB0, q);
#pragma unroll
    for (int s4 = 0; s4 < CF::KS0 / 4; ++s4)
#pragma unroll
      for (int ob = 0; ob < NB0; ++ob) {
        const floatx4 a4 = *reinterpret_cast<const floatx4*>(W + ((ob * (CF::KS0 / 4) + s4) * 64 + lane) * 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int s = 4 * s4 + i;
          if (s < CF::XS) {
            av[ob] = mfma16(a4[i], xin[s], av[ob]);
            at[ob] = mfma16(a4[i], e[s], at[ob]);
          } else if (s < CF::XS + CF::CS) {
            av[ob] = mfma16(a4[i], c[s - CF::XS], av[ob]);
          }
        }
      }
    act_all<CF::ACT, NB0>(av, at);
  }
  // hidden layers 1..NH-1, ping-pong between (av, at) and (bv, bt)
  cnf_static_for<1, CF::NH>([&](auto J) {
    constexpr int j = decltype(J)::value;
    constexpr int NBI = CF::NB(j - 1), NBO = CF::NB(j), OW = CF::off_w(j), OB = CF::off_b(j);
    if constexpr (j % 2 == 1) {
      init_bias4<NBO>(bv, bt, lds + OB, q);
      cnf_lin<X3, NBI, NBO>(lds + OW, av, at, bv, bt, lane);
      act_all<CF::ACT, NBO>(bv, bt);
    } else {
      init_bias4<NBO>(av, at, lds + OB, q);
      cnf_lin<X3, NBI, NBO>(lds + OW, bv, bt, av, at, lane);
      act_all<CF::ACT, NBO>(av, at);
    }
  });
  // output layer (no activation); rows permuted so register i of block ob = state slot 4 ob + i
  constexpr int NBI = CF::HL / 16;
  floatx4 ov[8], ot[8];
  init_bias4<CF::NBL>(ov, ot, lds + CF::OFF_BL, q);
  if constexpr ((CF::NH - 1) % 2 == 0)
    cnf_lin<X3, NBI, CF::NBL>(lds + CF::OFF_WL, av, at, ov, ot, lane);
  else
    cnf_lin<X3, NBI, CF::NBL>(lds + CF::OFF_WL, bv, bt, ov, ot, lane);
  float tr = 0.f;
#pragma unroll
  for (int s = 0; s < CF::XS; ++s) {
    f[s] = ov[s >> 2][s & 3];
    tr += e[s] * ot[s >> 2][s & 3];
  }
  tr += __shfl_xor(tr, 16);
  tr += __shfl_xor(tr, 32);
  g = -tr;
}

template <class CF, bool X3>
__global__ void __launch_bounds__(kCnfRows * 4, 1) cnf_kernel(
    const float* __restrict__ packed, const float* __restrict__ x, int64_t ldx, const float* __restrict__ ctx,
    int64_t ldc, const float* __restrict__ eps, int64_t lde, float dt, int steps, float* __restrict__ y,
    int64_t ldy, float* __restrict__ ld, int ld_mode, int64_t B) {
  __shared__ __attribute__((aligned(16))) float lds[CF::TOTAL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4;
  for (int i = tid * 4; i < CF::TOTAL; i += blockDim.x * 4)
    *reinterpret_cast<floatx4*>(lds + i) = *reinterpret_cast<const floatx4*>(packed + i);
  __syncthreads();
  constexpr int CSR = CF::CS > 0 ? CF::CS : 1;
  for (int64_t tile = blockIdx.x; tile * kCnfRows < B; tile += gridDim.x) {
    const int64_t row = tile * kCnfRows + wave * 16 + (lane & 15);
    const bool valid = row < B;
    float xs[CF::XS], es[CF::XS], cs[CSR];
#pragma unroll
    for (int s = 0; s < CF::XS; ++s) {
      const int fi = q + 4 * s;
      const bool ok = valid && fi < CF::D;
      xs[s] = ok ? x[row * ldx + fi] : 0.f;
      es[s] = ok ? eps[row * lde + fi] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < CSR; ++s) {
      const int fi = q + 4 * s;
      cs[s] = (CF::CS > 0 && valid && fi < CF::C) ? ctx[(ldc ? row * ldc : 0) + fi] : 0.f;
    }
    float a = 0.f;
    // classical RK4 (odeint.py:46-52), one RHS body for the four stages:
    //   k_i = dt f(x_i);  x_2 = x + k1/2, x_3 = x + k2/2, x_4 = x + k3;  x += (k1 + 2k2 + 2k3 + k4)/6
    float xst[CF::XS], sx[CF::XS], f[CF::XS];
    float sa = 0.f;
#pragma unroll
    for (int s = 0; s < CF::XS; ++s) xst[s] = xs[s];
    for (int it = 0; it < 4 * steps; ++it) {
      const int stage = it & 3;
      float g;
      cnf_rhs<CF, X3>(lds, xst, es, cs, f, g, lane);
      const float kg = dt * g;
      if (stage == 3) {
#pragma unroll
        for (int s = 0; s < CF::XS; ++s) {
          xs[s] = xs[s] + (sx[s] + dt * f[s]) / 6.f;
          xst[s] = xs[s];
        }
        a = a + (sa + kg) / 6.f;
      } else {
        const float w = stage == 0 ? 1.f : 2.f;     // weight of k_i in the final sum
        const float h = stage == 2 ? 1.f : 0.5f;    // x_{i+1} = x + h k_i
#pragma unroll
        for (int s = 0; s < CF::XS; ++s) {
          const float k = dt * f[s];
          sx[s] = stage == 0 ? k : sx[s] + w * k;
          xst[s] = xs[s] + h * k;
        }
        sa = stage == 0 ? kg : sa + w * kg;
      }
    }
    if (valid) {
#pragma unroll
      for (int s = 0; s < CF::XS; ++s) {
        const int fi = q + 4 * s;
        if (fi < CF::D) y[row * ldy + fi] = xs[s];
      }
      if (q == 0 && ld != nullptr) {
        if (ld_mode == NAZ_LD_ROWSUM_ADD) ld[row] += a;
        else if (ld_mode == NAZ_LD_ROWSUM_SUB) ld[row] -= a;
        else ld[row] = a;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Adaptive Dormand-Prince 5(4) solve (naz FFJORDTransform's
// solver='dopri5', atol = rtol = 1e-4, continuous_transforms.py:73-81).  Same residency and
// RHS as cnf_kernel; each WAVE (16 rows) integrates with its own step size: the controller
// (RMS error norm over the wave's [x, a] elements, accept at <= 1, h *= clamp(0.9 e^-1/5,
// 0.2 | 1 on accept, 10), Hairer's initial step, FSAL, last step clipped to t1) is restated in
// oracle/naz_oracle.py::dopri5_augmented with the same 16-row groups.  The waves of a
// workgroup never synchronise inside a tile (the weights are read-only LDS), so a wave that
// needs more steps does not hold the others.  One RHS call site: the stage machine keeps
// every k_i in named registers (no dynamically indexed arrays).
// ---------------------------------------------------------------------------
__constant__ float kDpA[15] = {1.f / 5,          3.f / 40,          9.f / 40,         44.f / 45,     -56.f / 15,
                               32.f / 9,         19372.f / 6561,    -25360.f / 2187,  64448.f / 6561, -212.f / 729,
                               9017.f / 3168,    -355.f / 33,       46732.f / 5247,   49.f / 176,    -5103.f / 18656};

NAZ_DEV float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

template <class CF, bool X3>
__global__ void __launch_bounds__(kCnfRows * 4, 1) cnf_dopri5_kernel(
    const float* __restrict__ packed, const float* __restrict__ x, int64_t ldx, const float* __restrict__ ctx,
    int64_t ldc, const float* __restrict__ eps, int64_t lde, float t0, float t1, float atol, float rtol,
    int max_steps, float* __restrict__ y, int64_t ldy, float* __restrict__ ld, int ld_mode, int* __restrict__ nfe_out,
    int64_t B) {
  __shared__ __attribute__((aligned(16))) float lds[CF::TOTAL];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4;
  for (int i = tid * 4; i < CF::TOTAL; i += blockDim.x * 4)
    *reinterpret_cast<floatx4*>(lds + i) = *reinterpret_cast<const floatx4*>(packed + i);
  __syncthreads();
  constexpr int CSR = CF::CS > 0 ? CF::CS : 1;
  constexpr int XS = CF::XS;
  constexpr float b0 = 35.f / 384, b2 = 500.f / 1113, b3 = 125.f / 192, b4 = -2187.f / 6784, b5 = 11.f / 84;
  constexpr float e0 = 35.f / 384 - 5179.f / 57600, e2 = 500.f / 1113 - 7571.f / 16695,
                  e3 = 125.f / 192 - 393.f / 640, e4 = -2187.f / 6784 + 92097.f / 339200,
                  e5 = 11.f / 84 - 187.f / 2100, e6 = -1.f / 40;
  const float dir = t1 > t0 ? 1.f : -1.f;
  for (int64_t tile = blockIdx.x; tile * kCnfRows < B; tile += gridDim.x) {
    const int64_t row0 = tile * kCnfRows + wave * 16;
    const int64_t row = row0 + (lane & 15);
    const bool valid = row < B;
    if (row0 >= B) continue;  // whole wave past the end (wave-uniform)
    float xs[XS], es[XS], cs[CSR];
    bool live[XS];
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      const int fi = q + 4 * s;
      live[s] = valid && fi < CF::D;
      xs[s] = live[s] ? x[row * ldx + fi] : 0.f;
      es[s] = live[s] ? eps[row * lde + fi] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < CSR; ++s) {
      const int fi = q + 4 * s;
      cs[s] = (CF::CS > 0 && valid && fi < CF::C) ? ctx[(ldc ? row * ldc : 0) + fi] : 0.f;
    }
    const bool alive = valid && q == 0;  // the lane that owns a row's log-det element
    const int64_t nrows = B - row0 < 16 ? B - row0 : 16;
    const float inv_n = 1.f / (float)(nrows * (CF::D + 1));
    // RMS over the wave's [x, a] elements of u / (atol + rtol * w)
    auto rms2 = [&](const float (&u)[XS], float ua, const float (&w)[XS], float wa) {
      float acc = 0.f;
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        const float r = u[s] / (atol + rtol * fabsf(w[s]));
        acc += live[s] ? r * r : 0.f;
      }
      const float ra = ua / (atol + rtol * wa);
      acc += alive ? ra * ra : 0.f;
      return sqrtf(wave_sum(acc) * inv_n);
    };

    float a = 0.f;
    float k0[XS], k1[XS], k2[XS], k3[XS], k4[XS], k5[XS], xin[XS], x5[XS], f[XS];
    float k0a = 0.f, k1a = 0.f, k2a = 0.f, k3a = 0.f, k4a = 0.f, k5a = 0.f, a5 = 0.f, g;
#pragma unroll
    for (int s = 0; s < XS; ++s) xin[s] = xs[s];
    int phase = -2, steps = 0, nfe = 0;
    float t = t0, h = 0.f, hh = 0.f, h0 = 0.f, d1 = 0.f;
    bool last = false;
    for (;;) {
      cnf_rhs<CF, X3>(lds, xin, es, cs, f, g, lane);
      ++nfe;
      bool start_step = false;
      if (phase == -2) {  // f(y0); initial-step heuristic part 1
#pragma unroll
        for (int s = 0; s < XS; ++s) k0[s] = f[s];
        k0a = g;
        const float d0 = rms2(xs, a, xs, 0.f);  // scale atol + rtol |y0|
        d1 = rms2(k0, k0a, xs, 0.f);
        h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : 0.01f * d0 / d1;
#pragma unroll
        for (int s = 0; s < XS; ++s) xin[s] = xs[s] + dir * h0 * k0[s];
        phase = -1;
      } else if (phase == -1) {  // part 2: h = min(100 h0, (0.01 / max(d1, d2))^(1/6))
        float df[XS];
#pragma unroll
        for (int s = 0; s < XS; ++s) df[s] = f[s] - k0[s];
        const float d2 = rms2(df, g - k0a, xs, 0.f) / h0;
        const float dm = fmaxf(d1, d2);
        const float h1 = dm <= 1e-15f ? fmaxf(1e-6f, h0 * 1e-3f) : powf(0.01f / dm, 1.f / 6.f);
        h = fminf(100.f * h0, h1);
        start_step = true;
      } else if (phase == 1) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k1[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[1] * k0[s] + kDpA[2] * k1[s]);
        }
        k1a = g;
        phase = 2;
      } else if (phase == 2) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k2[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[3] * k0[s] + kDpA[4] * k1[s] + kDpA[5] * k2[s]);
        }
        k2a = g;
        phase = 3;
      } else if (phase == 3) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k3[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[6] * k0[s] + kDpA[7] * k1[s] + kDpA[8] * k2[s] + kDpA[9] * k3[s]);
        }
        k3a = g;
        phase = 4;
      } else if (phase == 4) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k4[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[10] * k0[s] + kDpA[11] * k1[s] + kDpA[12] * k2[s] + kDpA[13] * k3[s] +
                                 kDpA[14] * k4[s]);
        }
        k4a = g;
        phase = 5;
      } else if (phase == 5) {  // 5th-order solution; its f is the FSAL stage k6
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k5[s] = f[s];
          x5[s] = xs[s] + hh * (b0 * k0[s] + b2 * k2[s] + b3 * k3[s] + b4 * k4[s] + b5 * k5[s]);
          xin[s] = x5[s];
        }
        k5a = g;
        a5 = a + hh * (b0 * k0a + b2 * k2a + b3 * k3a + b4 * k4a + b5 * k5a);
        phase = 6;
      } else {  // phase 6: error estimate, accept / reject, next step size
        float err[XS], w[XS];
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          err[s] = hh * (e0 * k0[s] + e2 * k2[s] + e3 * k3[s] + e4 * k4[s] + e5 * k5[s] + e6 * f[s]);
          w[s] = fmaxf(fabsf(xs[s]), fabsf(x5[s]));
        }
        const float erra = hh * (e0 * k0a + e2 * k2a + e3 * k3a + e4 * k4a + e5 * k5a + e6 * g);
        const float en = rms2(err, erra, w, fmaxf(fabsf(a), fabsf(a5)));
        const bool accept = en <= 1.f;
        if (accept) {
#pragma unroll
          for (int s = 0; s < XS; ++s) {
            xs[s] = x5[s];
            k0[s] = f[s];
          }
          a = a5;
          k0a = g;
          t = last ? t1 : t + hh;
        }
        const float fac = en == 0.f ? 10.f : fminf(10.f, fmaxf(0.9f * powf(en, -0.2f), accept ? 1.f : 0.2f));
        h = fabsf(hh) * fac;
        ++steps;
        if (t == t1 || steps >= max_steps) break;
        start_step = true;
      }
      if (start_step) {  // stage 1 input of the next step (clipped to end at t1)
        const float rem = fabsf(t1 - t);
        last = h >= rem;
        hh = dir * (last ? rem : h);
#pragma unroll
        for (int s = 0; s < XS; ++s) xin[s] = xs[s] + hh * kDpA[0] * k0[s];
        phase = 1;
      }
    }
    if (valid) {
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        const int fi = q + 4 * s;
        if (fi < CF::D) y[row * ldy + fi] = xs[s];
      }
      if (q == 0 && ld != nullptr) {
        if (ld_mode == NAZ_LD_ROWSUM_ADD) ld[row] += a;
        else if (ld_mode == NAZ_LD_ROWSUM_SUB) ld[row] -= a;
        else ld[row] = a;
      }
    }
    if (nfe_out != nullptr && lane == 0) nfe_out[row0 / 16] = steps >= max_steps && t != t1 ? -nfe : nfe;
  }
}

// ---------------------------------------------------------------------------
// Batch-global dopri5: torchdyn's controller as naz configures it (ONE step size for the whole
// batch; hairer_norm = the RMS over every element of the augmented state [B, D + 1]).  The grid
// cannot agree on a step inside one launch without a grid barrier, so each attempted step is
// one launch of cnf_dp5g_step_kernel (the six stages k1..k5, f(y5) for all rows, the rows' sum
// of squared scaled errors as one partial per workgroup) followed by the one-workgroup
// controller cnf_dp5g_ctrl_kernel (fixed-order reduction of the partials: deterministic;
// accept / reject, next step size).  State and the FSAL stage live in HBM between launches in
// two parities; the controller flips the parity on accept.  Launches after the solve has
// finished return at once (ctrl->done); the host polls `done` every few attempts
// (cnf_integrate_dopri5_global).  oracle/naz_oracle.py::dopri5_global restates it in fp64.
// ---------------------------------------------------------------------------
struct Dp5Ctrl {
  float t, h, hh, h0, d1;
  int cur, last, steps, nfe, done, exhausted, pad[5];
};
constexpr int kDp5MaxParts = 2048;

template <class CF>
NAZ_DEV void dp5g_load(const float* __restrict__ st, int64_t row, bool valid, int q, float (&xs)[CF::XS], float& a) {
  constexpr int W = CF::D + 1;
#pragma unroll
  for (int s = 0; s < CF::XS; ++s) {
    const int fi = q + 4 * s;
    xs[s] = (valid && fi < CF::D) ? st[row * W + fi] : 0.f;
  }
  a = valid ? st[row * W + CF::D] : 0.f;
}

template <class CF>
NAZ_DEV void dp5g_store(float* __restrict__ st, int64_t row, bool valid, int q, const float (&xs)[CF::XS], float a) {
  constexpr int W = CF::D + 1;
  if (!valid) return;
#pragma unroll
  for (int s = 0; s < CF::XS; ++s) {
    const int fi = q + 4 * s;
    if (fi < CF::D) st[row * W + fi] = xs[s];
  }
  if (q == 0) st[row * W + CF::D] = a;
}

// per-workgroup fixed-order sum of one value per wave (lane 0 holds the wave's total)
NAZ_DEV float dp5g_block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

// PHASE 0: k0 = f(x0), partials of |x0 / sc|^2 and |k0 / sc|^2 (sc = atol + rtol |x0|; a0 = 0)
// PHASE 1: f1 = f(x0 + dir h0 k0), partial of |(f1 - k0) / sc|^2
template <class CF, bool X3, int PHASE>
__global__ void __launch_bounds__(kCnfRows * 4, 1) cnf_dp5g_init_kernel(
    const float* __restrict__ packed, const float* __restrict__ x, int64_t ldx, const float* __restrict__ ctx,
    int64_t ldc, const float* __restrict__ eps, int64_t lde, float t0, float t1, float atol, float rtol,
    float* __restrict__ st, float* __restrict__ kb, float* __restrict__ parts, const Dp5Ctrl* __restrict__ ctrl,
    int64_t B) {
  __shared__ __attribute__((aligned(16))) float lds[CF::TOTAL];
  __shared__ float red[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4;
  for (int i = tid * 4; i < CF::TOTAL; i += blockDim.x * 4)
    *reinterpret_cast<floatx4*>(lds + i) = *reinterpret_cast<const floatx4*>(packed + i);
  __syncthreads();
  constexpr int CSR = CF::CS > 0 ? CF::CS : 1, XS = CF::XS;
  const float dir = t1 > t0 ? 1.f : -1.f;
  const float h0 = PHASE == 1 ? ctrl->h0 : 0.f;
  float acc0 = 0.f, acc1 = 0.f;
  for (int64_t tile = blockIdx.x; tile * kCnfRows < B; tile += gridDim.x) {
    const int64_t row = tile * kCnfRows + wave * 16 + (lane & 15);
    const bool valid = row < B;
    float xs[XS], es[XS], cs[CSR], f[XS], g;
    bool live[XS];
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      const int fi = q + 4 * s;
      live[s] = valid && fi < CF::D;
      xs[s] = live[s] ? x[row * ldx + fi] : 0.f;
      es[s] = live[s] ? eps[row * lde + fi] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < CSR; ++s) {
      const int fi = q + 4 * s;
      cs[s] = (CF::CS > 0 && valid && fi < CF::C) ? ctx[(ldc ? row * ldc : 0) + fi] : 0.f;
    }
    const bool alive = valid && q == 0;
    if constexpr (PHASE == 0) {
      cnf_rhs<CF, X3>(lds, xs, es, cs, f, g, lane);
      dp5g_store<CF>(st, row, valid, q, xs, 0.f);
      dp5g_store<CF>(kb, row, valid, q, f, g);
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        const float sc = atol + rtol * fabsf(xs[s]);
        acc0 += live[s] ? (xs[s] / sc) * (xs[s] / sc) : 0.f;
        acc1 += live[s] ? (f[s] / sc) * (f[s] / sc) : 0.f;
      }
      acc1 += alive ? (g / atol) * (g / atol) : 0.f;  // a0 = 0: |a0 / sca|^2 = 0
    } else {
      float k0[XS], k0a, xin[XS];
      dp5g_load<CF>(kb, row, valid, q, k0, k0a);
#pragma unroll
      for (int s = 0; s < XS; ++s) xin[s] = xs[s] + dir * h0 * k0[s];
      cnf_rhs<CF, X3>(lds, xin, es, cs, f, g, lane);
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        const float sc = atol + rtol * fabsf(xs[s]), r = (f[s] - k0[s]) / sc;
        acc0 += live[s] ? r * r : 0.f;
      }
      acc0 += alive ? ((g - k0a) / atol) * ((g - k0a) / atol) : 0.f;
    }
  }
  const float s0 = dp5g_block_sum(wave_sum(acc0), red);
  const float s1 = PHASE == 0 ? dp5g_block_sum(wave_sum(acc1), red) : 0.f;
  if (tid == 0) {
    parts[blockIdx.x] = s0;
    if (PHASE == 0) parts[kDp5MaxParts + blockIdx.x] = s1;
  }
}

template <class CF, bool X3>
__global__ void __launch_bounds__(kCnfRows * 4, 1) cnf_dp5g_step_kernel(
    const float* __restrict__ packed, const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ eps,
    int64_t lde, float atol, float rtol, float* __restrict__ st0, float* __restrict__ st1, float* __restrict__ kb0,
    float* __restrict__ kb1, float* __restrict__ parts, const Dp5Ctrl* __restrict__ ctrl, int64_t B) {
  if (ctrl->done) return;
  __shared__ __attribute__((aligned(16))) float lds[CF::TOTAL];
  __shared__ float red[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = lane >> 4;
  for (int i = tid * 4; i < CF::TOTAL; i += blockDim.x * 4)
    *reinterpret_cast<floatx4*>(lds + i) = *reinterpret_cast<const floatx4*>(packed + i);
  __syncthreads();
  constexpr int CSR = CF::CS > 0 ? CF::CS : 1, XS = CF::XS;
  constexpr float b0 = 35.f / 384, b2 = 500.f / 1113, b3 = 125.f / 192, b4 = -2187.f / 6784, b5 = 11.f / 84;
  constexpr float e0 = 35.f / 384 - 5179.f / 57600, e2 = 500.f / 1113 - 7571.f / 16695,
                  e3 = 125.f / 192 - 393.f / 640, e4 = -2187.f / 6784 + 92097.f / 339200,
                  e5 = 11.f / 84 - 187.f / 2100, e6 = -1.f / 40;
  const int cur = ctrl->cur;
  const float hh = ctrl->hh;
  const float* sc_ = cur ? st1 : st0;  // current state / FSAL stage
  const float* kc_ = cur ? kb1 : kb0;
  float* sn_ = cur ? st0 : st1;        // candidate
  float* kn_ = cur ? kb0 : kb1;
  float acc = 0.f;
  for (int64_t tile = blockIdx.x; tile * kCnfRows < B; tile += gridDim.x) {
    const int64_t row = tile * kCnfRows + wave * 16 + (lane & 15);
    const bool valid = row < B;
    float xs[XS], es[XS], cs[CSR], a;
    bool live[XS];
    dp5g_load<CF>(sc_, row, valid, q, xs, a);
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      const int fi = q + 4 * s;
      live[s] = valid && fi < CF::D;
      es[s] = live[s] ? eps[row * lde + fi] : 0.f;
    }
#pragma unroll
    for (int s = 0; s < CSR; ++s) {
      const int fi = q + 4 * s;
      cs[s] = (CF::CS > 0 && valid && fi < CF::C) ? ctx[(ldc ? row * ldc : 0) + fi] : 0.f;
    }
    const bool alive = valid && q == 0;
    float k0[XS], k1[XS], k2[XS], k3[XS], k4[XS], k5[XS], xin[XS], x5[XS], f[XS];
    float k0a, k1a = 0.f, k2a = 0.f, k3a = 0.f, k4a = 0.f, k5a = 0.f, a5 = 0.f, g;
    dp5g_load<CF>(kc_, row, valid, q, k0, k0a);
#pragma unroll
    for (int s = 0; s < XS; ++s) xin[s] = xs[s] + hh * kDpA[0] * k0[s];
    // one RHS call site; the stage machine of cnf_dopri5_kernel (phases 1..6)
    for (int phase = 1; phase <= 6; ++phase) {
      cnf_rhs<CF, X3>(lds, xin, es, cs, f, g, lane);
      if (phase == 1) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k1[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[1] * k0[s] + kDpA[2] * k1[s]);
        }
        k1a = g;
      } else if (phase == 2) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k2[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[3] * k0[s] + kDpA[4] * k1[s] + kDpA[5] * k2[s]);
        }
        k2a = g;
      } else if (phase == 3) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k3[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[6] * k0[s] + kDpA[7] * k1[s] + kDpA[8] * k2[s] + kDpA[9] * k3[s]);
        }
        k3a = g;
      } else if (phase == 4) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k4[s] = f[s];
          xin[s] = xs[s] + hh * (kDpA[10] * k0[s] + kDpA[11] * k1[s] + kDpA[12] * k2[s] + kDpA[13] * k3[s] +
                                 kDpA[14] * k4[s]);
        }
        k4a = g;
      } else if (phase == 5) {
#pragma unroll
        for (int s = 0; s < XS; ++s) {
          k5[s] = f[s];
          x5[s] = xs[s] + hh * (b0 * k0[s] + b2 * k2[s] + b3 * k3[s] + b4 * k4[s] + b5 * k5[s]);
          xin[s] = x5[s];
        }
        k5a = g;
        a5 = a + hh * (b0 * k0a + b2 * k2a + b3 * k3a + b4 * k4a + b5 * k5a);
      }
    }
    // f is now f(y5) (FSAL); the error of this row's elements
#pragma unroll
    for (int s = 0; s < XS; ++s) {
      const float err = hh * (e0 * k0[s] + e2 * k2[s] + e3 * k3[s] + e4 * k4[s] + e5 * k5[s] + e6 * f[s]);
      const float r = err / (atol + rtol * fmaxf(fabsf(xs[s]), fabsf(x5[s])));
      acc += live[s] ? r * r : 0.f;
    }
    {
      const float erra = hh * (e0 * k0a + e2 * k2a + e3 * k3a + e4 * k4a + e5 * k5a + e6 * g);
      const float r = erra / (atol + rtol * fmaxf(fabsf(a), fabsf(a5)));
      acc += alive ? r * r : 0.f;
    }
    dp5g_store<CF>(sn_, row, valid, q, x5, a5);
    dp5g_store<CF>(kn_, row, valid, q, f, g);
  }
  const float sum = dp5g_block_sum(wave_sum(acc), red);
  if (tid == 0) parts[blockIdx.x] = sum;
}

// one 256-thread workgroup: fixed-order sum of `nparts` partials (twice for PHASE 0)
NAZ_DEV float dp5g_sum_parts(const float* __restrict__ p, int n, float* red) {
  float v = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) v += p[i];
  return dp5g_block_sum(wave_sum(v), red);
}

// MODE 0: after init PHASE 0 (h0); 1: after PHASE 1 (h, first attempt); 2: after a step attempt
template <int MODE>
__global__ void __launch_bounds__(256, 1) cnf_dp5g_ctrl_kernel(Dp5Ctrl* __restrict__ ctrl,
                                                                 const float* __restrict__ parts, int nparts,
                                                                 double n_elem, float t0, float t1, int max_steps) {
  __shared__ float red[16];
  if (MODE == 2 && ctrl->done) return;
  const float s0 = dp5g_sum_parts(parts, nparts, red);
  const float s1 = MODE == 0 ? dp5g_sum_parts(parts + kDp5MaxParts, nparts, red) : 0.f;
  if (threadIdx.x != 0) return;
  const float dir = t1 > t0 ? 1.f : -1.f;
  const float inv_n = (float)(1.0 / n_elem);
  bool start = false;
  if constexpr (MODE == 0) {
    const float d0 = sqrtf(s0 * inv_n), d1 = sqrtf(s1 * inv_n);
    ctrl->t = t0;
    ctrl->d1 = d1;
    ctrl->h0 = (d0 < 1e-5f || d1 < 1e-5f) ? 1e-6f : 0.01f * d0 / d1;
    ctrl->cur = 0;
    ctrl->steps = 0;
    ctrl->nfe = 1;
    ctrl->done = 0;
    ctrl->exhausted = 0;
  } else if constexpr (MODE == 1) {
    const float h0 = ctrl->h0, d1 = ctrl->d1;
    const float d2 = sqrtf(s0 * inv_n) / h0, dm = fmaxf(d1, d2);
    const float h1 = dm <= 1e-15f ? fmaxf(1e-6f, h0 * 1e-3f) : powf(0.01f / dm, 1.f / 6.f);
    ctrl->h = fminf(100.f * h0, h1);
    ctrl->nfe = 2;
    start = true;
  } else {
    const float en = sqrtf(s0 * inv_n);
    const bool accept = en <= 1.f;
    const float hh = ctrl->hh;
    if (accept) {
      ctrl->cur ^= 1;
      ctrl->t = ctrl->last ? t1 : ctrl->t + hh;
    }
    const float fac = en == 0.f ? 10.f : fminf(10.f, fmaxf(0.9f * powf(en, -0.2f), accept ? 1.f : 0.2f));
    ctrl->h = fabsf(hh) * fac;
    ctrl->steps += 1;
    ctrl->nfe += 6;
    if (ctrl->t == t1) {
      ctrl->done = 1;
    } else if (ctrl->steps >= max_steps) {
      ctrl->done = 1;
      ctrl->exhausted = 1;
    } else {
      start = true;
    }
  }
  if (start) {  // the next attempt's step, clipped to end at t1
    const float rem = fabsf(t1 - ctrl->t);
    ctrl->last = ctrl->h >= rem ? 1 : 0;
    ctrl->hh = dir * (ctrl->last ? rem : ctrl->h);
  }
}

template <class CF>
__global__ void cnf_dp5g_finish_kernel(const float* __restrict__ st0, const float* __restrict__ st1,
                                       const Dp5Ctrl* __restrict__ ctrl, float* __restrict__ y, int64_t ldy,
                                       float* __restrict__ ld, int ld_mode, int* __restrict__ nfe_out, int64_t B) {
  const float* st = ctrl->cur ? st1 : st0;
  constexpr int W = CF::D + 1;
  for (int64_t row = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; row < B; row += (int64_t)gridDim.x * blockDim.x) {
    for (int d = 0; d < CF::D; ++d) y[row * ldy + d] = st[row * W + d];
    if (ld != nullptr) {
      const float a = st[row * W + CF::D];
      if (ld_mode == NAZ_LD_ROWSUM_ADD) ld[row] += a;
      else if (ld_mode == NAZ_LD_ROWSUM_SUB) ld[row] -= a;
      else ld[row] = a;
    }
  }
  if (nfe_out != nullptr && blockIdx.x == 0 && threadIdx.x == 0) nfe_out[0] = ctrl->exhausted ? -ctrl->nfe : ctrl->nfe;
}

// ---------------------------------------------------------------------------
// Instantiations and dispatch
// ---------------------------------------------------------------------------
template <class CF>
struct CnfOps {
  // fp16x3 needs every hidden width (the GEMM k of the hidden and output layers) in 32-k steps
  static constexpr bool kX3 = CF::NB(0) % 2 == 0 && CF::NB(CF::NH - 1) % 2 == 0 &&
                              (CF::NH < 2 || CF::NB(1) % 2 == 0) && (CF::NH < 3 || CF::NB(2) % 2 == 0);
  static bool supports(int mode) { return mode == NAZ_CNF_F32 || (mode == NAZ_CNF_F16X3 && kX3); }
  static int64_t packed_bytes() { return (int64_t)CF::TOTAL * 4; }
  static int pack(const float* flat, void* packed, int mode, hipStream_t s) {
    if (mode == NAZ_CNF_F16X3) {
      if constexpr (kX3)
        hipLaunchKernelGGL((cnf_pack_kernel<CF, true>), dim3((CF::TOTAL + 255) / 256), dim3(256), 0, s, flat,
                           static_cast<float*>(packed));
    } else {
      hipLaunchKernelGGL((cnf_pack_kernel<CF, false>), dim3((CF::TOTAL + 255) / 256), dim3(256), 0, s, flat,
                         static_cast<float*>(packed));
    }
    return check_launch("cnf_pack_kernel");
  }
  static int run(const void* packed, const float* x, int64_t ldx, const float* ctx, int64_t ldc, const float* eps,
                 int64_t lde, float dt, int steps, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B, int mode,
                 hipStream_t s) {
    const int64_t tiles = (B + kCnfRows - 1) / kCnfRows;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      cus = 256;
    const int per_cu = (160 * 1024) / (CF::TOTAL * 4) >= 2 ? 2 : 1;
    const int64_t grid = tiles < (int64_t)cus * per_cu ? tiles : (int64_t)cus * per_cu;
    if (mode == NAZ_CNF_F16X3) {
      if constexpr (kX3)
        hipLaunchKernelGGL((cnf_kernel<CF, true>), dim3((unsigned)grid), dim3(kCnfRows * 4), 0, s,
                           static_cast<const float*>(packed), x, ldx, ctx, ldc, eps, lde, dt, steps, y, ldy, ld,
                           ld_mode, B);
    } else {
      hipLaunchKernelGGL((cnf_kernel<CF, false>), dim3((unsigned)grid), dim3(kCnfRows * 4), 0, s,
                         static_cast<const float*>(packed), x, ldx, ctx, ldc, eps, lde, dt, steps, y, ldy, ld,
                         ld_mode, B);
    }
    return check_launch("cnf_kernel");
  }
  static int run_dopri5(const void* packed, const float* x, int64_t ldx, const float* ctx, int64_t ldc,
                        const float* eps, int64_t lde, float t0, float t1, float atol, float rtol, int max_steps,
                        float* y, int64_t ldy, float* ld, int ld_mode, int* nfe, int64_t B, int mode, hipStream_t s) {
    const int64_t tiles = (B + kCnfRows - 1) / kCnfRows;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      cus = 256;
    const int per_cu = (160 * 1024) / (CF::TOTAL * 4) >= 2 ? 2 : 1;
    const int64_t grid = tiles < (int64_t)cus * per_cu ? tiles : (int64_t)cus * per_cu;
    if (mode == NAZ_CNF_F16X3) {
      if constexpr (kX3)
        hipLaunchKernelGGL((cnf_dopri5_kernel<CF, true>), dim3((unsigned)grid), dim3(kCnfRows * 4), 0, s,
                           static_cast<const float*>(packed), x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol,
                           max_steps, y, ldy, ld, ld_mode, nfe, B);
    } else {
      hipLaunchKernelGGL((cnf_dopri5_kernel<CF, false>), dim3((unsigned)grid), dim3(kCnfRows * 4), 0, s,
                         static_cast<const float*>(packed), x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps,
                         y, ldy, ld, ld_mode, nfe, B);
    }
    return check_launch("cnf_dopri5_kernel");
  }
  // workspace floats: two state parities and two FSAL parities [B][D + 1], the partials, the control block
  static int64_t dp5g_workspace_floats(int64_t B) { return 4 * B * (CF::D + 1) + 2 * kDp5MaxParts + 64; }
  static int run_dopri5_global(const void* packed, const float* x, int64_t ldx, const float* ctx, int64_t ldc,
                               const float* eps, int64_t lde, float t0, float t1, float atol, float rtol, int max_steps,
                               float* y, int64_t ldy, float* ld, int ld_mode, int* nfe, void* work, int64_t B,
                               int mode, hipStream_t s) {
    if constexpr (!kX3) {
      if (mode == NAZ_CNF_F16X3) return set_error("naz_cnf: f16x3 not available for this shape");
    }
    // the host polls the controller (hipMemcpyAsync + hipStreamSynchronize every few attempts), which
    // a stream capture cannot record
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &cap) == hipSuccess && cap != hipStreamCaptureStatusNone)
      return set_error("naz_cnf_integrate_dopri5_global: the batch-global controller polls the host and cannot be "
                       "captured into a HIP graph; use step_control='group' (one launch per solve) under capture");
    const int64_t tiles = (B + kCnfRows - 1) / kCnfRows;
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                hipSuccess)
      cus = 256;
    const int per_cu = (160 * 1024) / (CF::TOTAL * 4) >= 2 ? 2 : 1;
    int64_t grid = tiles < (int64_t)cus * per_cu ? tiles : (int64_t)cus * per_cu;
    if (grid > kDp5MaxParts) grid = kDp5MaxParts;
    const int64_t n = B * (CF::D + 1);
    float* w = static_cast<float*>(work);
    float *st0 = w, *st1 = w + n, *kb0 = w + 2 * n, *kb1 = w + 3 * n, *parts = w + 4 * n;
    Dp5Ctrl* ctrl = reinterpret_cast<Dp5Ctrl*>(parts + 2 * kDp5MaxParts);
    const float* pk = static_cast<const float*>(packed);
    const dim3 g((unsigned)grid), b(kCnfRows * 4);
    const double n_elem = (double)n;
    auto launch = [&](auto x3) {
      constexpr bool X3 = decltype(x3)::value;
      hipLaunchKernelGGL((cnf_dp5g_init_kernel<CF, X3, 0>), g, b, 0, s, pk, x, ldx, ctx, ldc, eps, lde, t0, t1, atol,
                         rtol, st0, kb0, parts, ctrl, B);
      hipLaunchKernelGGL((cnf_dp5g_ctrl_kernel<0>), dim3(1), dim3(256), 0, s, ctrl, parts, (int)grid, n_elem, t0, t1,
                         max_steps);
      hipLaunchKernelGGL((cnf_dp5g_init_kernel<CF, X3, 1>), g, b, 0, s, pk, x, ldx, ctx, ldc, eps, lde, t0, t1, atol,
                         rtol, st0, kb0, parts, ctrl, B);
      hipLaunchKernelGGL((cnf_dp5g_ctrl_kernel<1>), dim3(1), dim3(256), 0, s, ctrl, parts, (int)grid, n_elem, t0, t1,
                         max_steps);
      if (check_launch("cnf_dp5g_init") != 0) return -1;
      // attempts in rounds of 4, then one poll of `done` (torchdyn's controller is host-driven too)
      int done = 0;
      for (int issued = 0; issued < max_steps && !done;) {
        const int k = max_steps - issued < 4 ? max_steps - issued : 4;
        for (int i = 0; i < k; ++i) {
          hipLaunchKernelGGL((cnf_dp5g_step_kernel<CF, X3>), g, b, 0, s, pk, ctx, ldc, eps, lde, atol, rtol, st0, st1,
                             kb0, kb1, parts, ctrl, B);
          hipLaunchKernelGGL((cnf_dp5g_ctrl_kernel<2>), dim3(1), dim3(256), 0, s, ctrl, parts, (int)grid, n_elem, t0,
                             t1, max_steps);
        }
        issued += k;
        if (check_launch("cnf_dp5g_step") != 0) return -1;
        if (hipMemcpyAsync(&done, &ctrl->done, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
          return set_error("naz_cnf_integrate_dopri5_global: polling the controller failed");
      }
      const int64_t fg = (B + 255) / 256 < 4096 ? (B + 255) / 256 : 4096;
      hipLaunchKernelGGL((cnf_dp5g_finish_kernel<CF>), dim3((unsigned)fg), dim3(256), 0, s, st0, st1, ctrl, y, ldy, ld,
                         ld_mode, nfe, B);
      return check_launch("cnf_dp5g_finish_kernel");
    };
    if (mode == NAZ_CNF_F16X3) {
      if constexpr (kX3) return launch(std::integral_constant<bool, true>{});
      return -1;
    }
    return launch(std::integral_constant<bool, false>{});
  }
};

// (D, C, H0, H1, H2, H3, act): config 5 (D=16, H=[128]x3, softplus), the
// reference's conditional CNF examples (train_mle_all_data_cnf.py:96 D=2, C=2, H=[128,64,64]),
// and small test shapes.
#ifndef NAZ_CNF_CONFIGS
#define NAZ_CNF_CONFIGS(X)                          \
  X(16, 0, 128, 128, 128, 0, ACT_SOFTPLUS)          \
  X(2, 2, 128, 64, 64, 0, ACT_SOFTPLUS)             \
  X(4, 2, 32, 32, 0, 0, ACT_SOFTPLUS)               \
  X(4, 2, 32, 32, 0, 0, ACT_TANH)                   \
  X(5, 3, 48, 32, 16, 16, ACT_SOFTPLUS)
#endif

template <class F>
static int cnf_dispatch(const naz_cnf_desc* d, F&& f) {
  if (d == nullptr) return set_error("naz_cnf: null descriptor");
  int H[4] = {0, 0, 0, 0};
  if (d->n_hidden < 1 || d->n_hidden > 4) return set_error("naz_cnf: n_hidden must be 1..4");
  for (int j = 0; j < d->n_hidden; ++j) H[j] = d->H[j];
#define NAZ_CNF_CASE(D_, C_, H0, H1, H2, H3, A_)                                                              \
  if (d->D == D_ && d->C == C_ && H[0] == H0 && H[1] == H1 && H[2] == H2 && H[3] == H3 && d->act == A_) {  \
    using Ops = CnfOps<CnfCfg<D_, C_, H0, H1, H2, H3, A_>>;                                               \
    if (!Ops::supports(d->mfma_mode))                                                                     \
      return set_error("naz_cnf: mfma_mode %d is not available for this shape", d->mfma_mode);           \
    return f(Ops{});                                                                                      \
  }
  NAZ_CNF_CONFIGS(NAZ_CNF_CASE)
#undef NAZ_CNF_CASE
  return set_error("naz_cnf: shape D=%d C=%d H=[%d,%d,%d,%d] act=%d is not instantiated (NAZ_CNF_CONFIGS)", d->D,
                   d->C, H[0], H[1], H[2], H[3], d->act);
}

int cnf_supported(const naz_cnf_desc* d) {
  return cnf_dispatch(d, [](auto) { return 1; }) == 1 ? 1 : 0;
}

int64_t cnf_param_count(const naz_cnf_desc* d) {
  if (d == nullptr || d->n_hidden < 1 || d->n_hidden > 4) return -1;
  int in = d->D + d->C;
  int64_t n = 0;
  for (int j = 0; j < d->n_hidden; ++j) {
    n += (int64_t)d->H[j] * in + d->H[j];
    in = d->H[j];
  }
  return n + (int64_t)d->D * in + d->D;
}

int64_t cnf_packed_bytes(const naz_cnf_desc* d) {
  int64_t n = -1;
  if (cnf_dispatch(d, [&](auto ops) {
        n = decltype(ops)::packed_bytes();
        return 0;
      }) != 0)
    return -1;
  return n;
}

int cnf_pack(const naz_cnf_desc* d, const float* flat, void* packed, hipStream_t s) {
  return cnf_dispatch(d, [&](auto ops) { return decltype(ops)::pack(flat, packed, d->mfma_mode, s); });
}

int cnf_integrate(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                  int64_t ldc, const float* eps, int64_t lde, float t0, float t1, int steps, float* y, int64_t ldy,
                  float* ld, int ld_mode, int64_t B, hipStream_t s) {
  if (B == 0) return 0;
  if (steps < 1) return set_error("naz_cnf_integrate: steps must be >= 1");
  // odeint.py:15-16: dt = t1 - t0 of consecutive grid points (a single value for a uniform grid)
  const float dt = (float)(((double)t1 - (double)t0) / (double)steps);
  return cnf_dispatch(d, [&](auto ops) {
    return decltype(ops)::run(packed, x, ldx, ctx, ldc, eps, lde, dt, steps, y, ldy, ld, ld_mode, B, d->mfma_mode,
                              s);
  });
}

int cnf_integrate_dopri5(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                         int64_t ldc, const float* eps, int64_t lde, float t0, float t1, float atol, float rtol,
                         int max_steps, float* y, int64_t ldy, float* ld, int ld_mode, int* nfe, int64_t B,
                         hipStream_t s) {
  if (B == 0) return 0;
  if (!(atol > 0.f) || !(rtol >= 0.f)) return set_error("naz_cnf_integrate_dopri5: atol must be > 0, rtol >= 0");
  if (max_steps < 1) return set_error("naz_cnf_integrate_dopri5: max_steps must be >= 1");
  if (t0 == t1) return set_error("naz_cnf_integrate_dopri5: empty interval");
  return cnf_dispatch(d, [&](auto ops) {
    return decltype(ops)::run_dopri5(packed, x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps, y, ldy, ld,
                                     ld_mode, nfe, B, d->mfma_mode, s);
  });
}

int64_t cnf_dopri5_global_workspace_bytes(const naz_cnf_desc* d, int64_t B) {
  int64_t n = -1;
  if (cnf_dispatch(d, [&](auto ops) {
        n = decltype(ops)::dp5g_workspace_floats(B) * 4;
        return 0;
      }) != 0)
    return -1;
  return n;
}

int cnf_integrate_dopri5_global(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                                const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                                float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld, int ld_mode,
                                int* nfe, void* work, int64_t B, hipStream_t s) {
  if (B == 0) return 0;
  if (!(atol > 0.f) || !(rtol >= 0.f)) return set_error("naz_cnf_integrate_dopri5_global: atol must be > 0, rtol >= 0");
  if (max_steps < 1) return set_error("naz_cnf_integrate_dopri5_global: max_steps must be >= 1");
  if (t0 == t1) return set_error("naz_cnf_integrate_dopri5_global: empty interval");
  if (work == nullptr) return set_error("naz_cnf_integrate_dopri5_global: workspace required");
  return cnf_dispatch(d, [&](auto ops) {
    return decltype(ops)::run_dopri5_global(packed, x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps, y, ldy,
                                            ld, ld_mode, nfe, work, B, d->mfma_mode, s);
  });
}

}  // namespace naz
