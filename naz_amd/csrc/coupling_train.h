// Backward of one spline-coupling layer for the NLL training step (SURVEY.md §8a a10 over a3;
// naz train_flows.py:194-213 differentiating NormalizingFlow.log_prob).  Included by
// coupling.hip after coupling_r16.h (CfgR16, the packed forward image, split8_f16, ...).
//
// The training forward (coupling_r16_kernel<.., VAR = 1>) stores every layer's input state
// P[l + 1] (P[L] = data, P[0] = z; layer l maps P[l + 1] -> P[l] in the log_prob direction).
// One launch of coupling_bwd_r16_kernel per layer l, in the order l = 0 .. L-1, takes
// g(P[l]) = dLoss/dP[l] and the per-row weight of the log-det terms g_lp = dLoss/dlog p, and
//   1. recomputes the layer's conditioner forward from P[l + 1] exactly as the training forward
//      did (same packed f16x3 image, same libm-grade tanh and spline), keeping H1, H2
//      (natural tanh values) and the raw spline parameters in registers;
//   2. runs the upper spline's VJP per (row, dim) in registers (rqs_vjp: implicit-function rule
//      for the inverse) -> dRaw (= dPre3, GEMM3 has no activation) and g(y2);
//   3. backpropagates through the MLP with EXACT fp32 MFMA (v_mfma_f32_16x16x4_f32; gradients
//      have no fixed range, so no fp16 split): dH2 = dPre3·W2, dPre2 = dH2 ⊙ (1 − H2²),
//      dH1 = dPre2·W1, dPre1 = dH1 ⊙ (1 − H1²), dx1 = dPre1·W0[:, C:];
//   4. runs the lower spline's VJP (shared parameters: per-workgroup sums in LDS, one atomic
//      per parameter per workgroup) and writes g(P[l + 1]);
//   5. writes the weight-gradient operands dPre3, H2, dPre2, H1, dPre1 and X0 = [ctx | x1] (the
//      batch reductions dW = dPreᵀ·X run as separate GEMMs).
// Layout: the forward kernel's 16-row waves — lane l owns row l & 15 and quarter q = l >> 4,
// accumulator register i of block b on quarter q = feature 16b + 4q + i.  The transposed GEMMs
// keep that layout: in step 3 a k-step feeds each quarter's OWN values (its 48 GEMM3 slots, or
// its 32 hidden features) as the B operand, and the backward images order the weight columns to
// match, so the results land in the forward's activation layout with no shuffles.
#pragma once
#include "spline_bwd.h"

namespace naz {

// Backward GEMM precision.  Default: f16x3 (v_mfma_f32_16x16x32_f16, three products as the
// forward) with a per-row power-of-2 scale of the gradient operand (its row maximum maps into
// [2^13, 2^14), so the lo pieces stay clear of the f16 subnormals) and weight images held at 2^6 W;
// 5.3x the matrix rate of the exact-fp32 form.  NAZ_BWD_EXACT_F32: v_mfma_f32_16x16x4_f32.
#ifdef NAZ_BWD_EXACT_F32
constexpr bool kBwdF16 = false;
#else
constexpr bool kBwdF16 = true;
#endif
constexpr float kBwdWScale = 64.f;

template <class CF>
struct BwdR16 {
  static constexpr int NS3 = 4 * CF::NO;  // GEMM3 slots per quarter = dH2 k-steps
  static constexpr int HB = CF::HB;
  // exact fp32 — units of 4 MFMA k-steps (one 16x16x4 k-step takes one value from each
  // quarter): dH2 has NS3 k-steps, dH1 and dx1 H/4 (each quarter feeds its H/4 own features)
  static constexpr int U3ALL = NS3 / 4, UH = CF::H / 16;
  static constexpr int pick_u(int nb, int units) {
    int best = 1;
    for (int u = 1; u <= units; ++u)
      if (units % u == 0 && nb * u * 256 <= kX6Slot) best = u;
    return best;
  }
  static constexpr int U3 = pick_u(HB, U3ALL), U2 = pick_u(HB, UH);
  // f16x3 — 32-k steps of 8 own values per quarter (slot s = 8 t + j), images laid out as the
  // forward's [block][k-step][hi | lo][lane][8 x f16]
  static constexpr int KS3 = (NS3 + 7) / 8, KSH = CF::H / 32;
  static constexpr int pick_kb(int nb, int ks) {
    int best = 1;
    for (int kb = 1; kb <= ks; ++kb)
      if (ks % kb == 0 && nb * kb * CF::OT <= kX6Slot) best = kb;
    return best;
  }
  static constexpr int KB3 = pick_kb(HB, KS3), KB2 = pick_kb(HB, KSH);
  static constexpr int NB3 = kBwdF16 ? KS3 / KB3 : U3ALL / U3;  // dH2 stages
  static constexpr int NB2 = kBwdF16 ? KSH / KB2 : UH / U2;     // dH1 stages
  static constexpr int S3 = kBwdF16 ? HB * KB3 * CF::OT : HB * U3 * 256;
  static constexpr int S2 = kBwdF16 ? HB * KB2 * CF::OT : HB * U2 * 256;
  static constexpr int SA = kBwdF16 ? KSH * CF::OT : UH * 256;
  static constexpr int OFF2 = NB3 * S3, OFFA = OFF2 + NB2 * S2;
  static constexpr int LAYER = OFFA + SA;
  static constexpr int NSTG = NB3 + NB2 + 1;
  static_assert(CF::SQ <= 4, "dx1 block holds at most 4 lower dims per quarter");
  static_assert(NS3 % 4 == 0 && CF::H % 16 == 0, "k-step units");
  static constexpr __host__ __device__ int stage_off(int j) { return j < NB3 ? j * S3 : (j < NB3 + NB2 ? OFF2 + (j - NB3) * S2 : OFFA); }
  static constexpr __host__ __device__ int stage_size(int j) { return j < NB3 ? S3 : (j < NB3 + NB2 ? S2 : SA); }
  // DenseNN output row of quarter q's GEMM3 slot s (-1 = pad)
  static constexpr __host__ __device__ int slot_row(int q, int s) { return r16_out_row<CF>(s >> 2, 4 * q + (s & 3)); }
  // hidden feature fed by quarter q at k-step s of a hidden-layer backward GEMM
  static constexpr __host__ __device__ int hid_feat(int q, int s) { return 16 * (s >> 2) + 4 * q + (s & 3); }
};

// Backward images (fp32) of every layer from the natural flat weights: [L][BwdR16::LAYER].
template <class CF>
__global__ void coupling_pack_bwd_r16_kernel(const float* __restrict__ flat, float* __restrict__ packed, int L) {
  using BW = BwdR16<CF>;
  const int64_t n = (int64_t)L * BW::LAYER;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(e / BW::LAYER);
    const int off = (int)(e - (int64_t)l * BW::LAYER);
    const float* W0 = flat + (int64_t)l * CF::FLAT;
    const float* W1 = W0 + CF::N_W0 + CF::N_B0;
    const float* W2 = W1 + CF::N_W1 + CF::N_B1;
    if constexpr (kBwdF16) {
      // word (b, tl, piece, lane, pair) of a stage: two f16 pieces of 2^6 W at k-slots
      // j = 2 pair + e of 32-k step t = stage k-step base + tl, fed by quarter kg = lane >> 4
      const int gsel = off < BW::OFF2 ? 0 : (off < BW::OFFA ? 1 : 2);
      const int kb = gsel == 0 ? BW::KB3 : (gsel == 1 ? BW::KB2 : BW::KSH);
      const int so = gsel == 0 ? off : (gsel == 1 ? off - BW::OFF2 : off - BW::OFFA);
      const int ssz = gsel == 0 ? BW::S3 : (gsel == 1 ? BW::S2 : BW::SA);
      const int js = so / ssz, r = so - js * ssz;
      const int b = r / (kb * CF::OT), r1 = r - b * kb * CF::OT;
      const int tl = r1 / CF::OT, r2 = r1 - tl * CF::OT;
      const int piece = r2 / kChunk, u = r2 - piece * kChunk;
      const int lane = u >> 2, pair = u & 3, m = lane & 15, kg = lane >> 4;
      const int t = js * kb + tl;
      unsigned word = 0;
      for (int e2 = 0; e2 < 2; ++e2) {
        const int jj = 2 * pair + e2;
        float v = 0.f;
        if (gsel == 0) {
          const int s = 8 * t + jj;
          const int orow = s < BW::NS3 ? BW::slot_row(kg, s) : -1;
          if (orow >= 0) v = W2[orow * CF::H + 16 * b + m];
        } else if (gsel == 1) {
          v = W1[r16_feat(t, kg, jj) * CF::H + 16 * b + m];
        } else {
          const int qq = m >> 2, i = m & 3;
          if (i < CF::SQ) v = W0[r16_feat(t, kg, jj) * (CF::C + CF::S) + CF::C + qq * CF::SQ + i];
        }
        word |= f16_piece_bits(kBwdWScale * v, piece) << (16 * e2);
      }
      reinterpret_cast<unsigned*>(packed)[e] = word;
      continue;
    }
    float v = 0.f;
    if (off < BW::OFF2) {  // dH2 stages: [b][u][lane][e], k-step s = 4(j U3 + u) + e
      const int j = off / BW::S3, r = off - j * BW::S3;
      const int b = r / (BW::U3 * 256), r2 = r - b * BW::U3 * 256;
      const int u = r2 >> 8, lane = (r2 >> 2) & 63, ee = r2 & 3;
      const int s = 4 * (j * BW::U3 + u) + ee, q = lane >> 4, m = lane & 15;
      const int orow = BW::slot_row(q, s);
      if (orow >= 0) v = W2[orow * CF::H + 16 * b + m];
    } else if (off < BW::OFFA) {  // dH1 stages
      const int o2 = off - BW::OFF2;
      const int j = o2 / BW::S2, r = o2 - j * BW::S2;
      const int b = r / (BW::U2 * 256), r2 = r - b * BW::U2 * 256;
      const int u = r2 >> 8, lane = (r2 >> 2) & 63, ee = r2 & 3;
      const int s = 4 * (j * BW::U2 + u) + ee, q = lane >> 4, m = lane & 15;
      v = W1[BW::hid_feat(q, s) * CF::H + 16 * b + m];
    } else {  // dx1: [u][lane][e]; output row m = 4q' + i -> lower dim q' SQ + i (i < SQ)
      const int r = off - BW::OFFA;
      const int u = r >> 8, lane = (r >> 2) & 63, ee = r & 3;
      const int s = 4 * u + ee, q = lane >> 4, m = lane & 15;
      const int qq = m >> 2, i = m & 3;
      if (i < CF::SQ) v = W0[BW::hid_feat(q, s) * (CF::C + CF::S) + CF::C + qq * CF::SQ + i];
    }
    packed[e] = v;
  }
}

// acc[b] += Σ_k A_b(k) B(k) over the stage's units [U0, U0 + NU) of 4 k-steps; A from the
// stage image [b][u][lane][4], B = the lane's own values bv[s].
template <int NBLK, int NU, int U0, int NV>
NAZ_DEV void bwd_gemm_stage(floatx4 (&acc)[NBLK], const float* __restrict__ stage, int lane, const floatx4 (&bv)[NV]) {
  // block-interleaved: consecutive MFMAs hit different accumulators (the f32 16x16x4 form's
  // dependent-accumulator latency, 40 cycles, exceeds its 32-cycle issue)
  const float4* p4 = reinterpret_cast<const float4*>(stage);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    float4 a[NBLK];
#pragma unroll
    for (int b = 0; b < NBLK; ++b) a[b] = p4[(b * NU + u) * 64 + lane];
#pragma unroll
    for (int b = 0; b < NBLK; ++b) acc[b] = mfma16_f32(a[b].x, bv[U0 + u][0], acc[b]);
#pragma unroll
    for (int b = 0; b < NBLK; ++b) acc[b] = mfma16_f32(a[b].y, bv[U0 + u][1], acc[b]);
#pragma unroll
    for (int b = 0; b < NBLK; ++b) acc[b] = mfma16_f32(a[b].z, bv[U0 + u][2], acc[b]);
#pragma unroll
    for (int b = 0; b < NBLK; ++b) acc[b] = mfma16_f32(a[b].w, bv[U0 + u][3], acc[b]);
  }
}

// f16x3 backward operand scale: multiplies the row's values (this lane's NB blocks; the row
// spans the four quarters, lanes n, n + 16, n + 32, n + 48) by 2^k so the row maximum lies in
// [2^13, 2^14); returns 2^-k / kBwdWScale, which turns the GEMM result back into natural units.
template <int NB>
NAZ_DEV float bwd_row_scale(floatx4 (&x)[NB]) {
  float mx = 0.f;
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) mx = fmaxf(mx, fabsf(x[b][r]));
  mx = fmaxf(mx, __shfl_xor(mx, 16));
  mx = fmaxf(mx, __shfl_xor(mx, 32));
  int k = 140 - (int)((__float_as_uint(mx) >> 23) & 255u);  // 13 - unbiased exponent
  k = k < -100 ? -100 : (k > 110 ? 110 : k);
  const float s = __uint_as_float((unsigned)(k + 127) << 23);
#pragma unroll
  for (int b = 0; b < NB; ++b)
#pragma unroll
    for (int r = 0; r < 4; ++r) x[b][r] *= s;
  return __uint_as_float((unsigned)(127 - k - 6) << 23);  // 2^-k / 2^6
}
static_assert(kBwdWScale == 64.f, "bwd_row_scale folds 2^-6");

// the training forward's activation of a packed (sigmoid-folded) accumulator: -tanh(a)/2
NAZ_DEV float train_fold(float v) {
  if constexpr (kTrainFast) return sig_fold(v);
  else return acc_fold(v);
}

template <int K>
NAZ_DEV float train_vjp_inv(const float* uw, const float* uh, const float* ud, float bound, float y, float g_x,
                            float g_ld, const RqsConsts<K, true>& rc, float* gw, float* gh, float* gd) {
  if constexpr (kTrainFast) return rqs_vjp_select_inv<K>(uw, uh, ud, y, g_x, g_ld, bound, rc, gw, gh, gd);
  else return rqs_vjp<K, true, false>(uw, uh, ud, bound, y, g_x, g_ld, gw, gh, gd);
}

struct BwdOut {
  float* h1;   // [B, H]   H1 (natural tanh)
  float* h2;   // [B, H]   H2
  float* dp1;  // [B, H]   dL/dpre1
  float* dp2;  // [B, H]   dL/dpre2
  float* dp3;  // [B, 4 NS3] dL/draw in lane-slot order (column q NS3 + s)
  float* x0;   // [B, C + S] [ctx | x1]
  float* g_out;       // [B, D]  dL/dP[l + 1]
  float* g_low;       // [S (3K - 1)] lower-spline parameter gradients (atomically accumulated)
};

// Workgroups of NW waves (16 rows each).  NW = 4: two independent workgroups per CU, so one's
// VALU phases (activations, spline VJPs) overlap the other's MFMA phases; the waves of ONE
// workgroup run the same phase between stage barriers.
#ifndef NAZ_BWD_WAVES
#define NAZ_BWD_WAVES 4
#endif
constexpr int kBwdWaves = NAZ_BWD_WAVES;
// the backward's GEMMs read their A fragments one MFMA triple ahead (gemm_r16_pf): two waves per
// SIMD do not hide the LDS latency hipcc's lgkmcnt(0) waits expose (NAZ_BWD_NO_PF: the plain form)
#ifdef NAZ_BWD_NO_PF
constexpr bool kBwdPF = false;
#else
constexpr bool kBwdPF = true;
#endif

// NAZ_ABL_BWD_NOSTORE (timing ablation only, wrong gradients): the six dW operand stores skipped, so a
// run measures what the operand writes (their bandwidth and the ring barriers' vmcnt(0) on their
// acknowledgements) cost the kernel
#ifdef NAZ_ABL_BWD_NOSTORE
constexpr bool kBwdStore = false;
#else
constexpr bool kBwdStore = true;
#endif

// NAZ_BWD_NT_STORES (A/B): the operands nothing in this kernel re-reads (dPre3, dPre2, dPre1, X0) stored
// non-temporally, so 9 GB of them per 2^22 rows and layer do not push the weight images and the H1 / H2
// rows this kernel re-reads out of L2
template <class T>
NAZ_DEV void bwd_store_stream(T* p, T v) {
#ifdef NAZ_BWD_NT_STORES
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

template <class CF>
struct BwdSlot {  // LDS ring slot: the largest forward or backward stage
  static constexpr int v = std::max({CF::A_SIZE, CF::B_SIZE, CF::C_SIZE, BwdR16<CF>::S3, BwdR16<CF>::S2,
                                     BwdR16<CF>::SA});
};

template <class CF>
__global__ void __launch_bounds__(kBwdWaves * 64, 2) coupling_bwd_r16_kernel(
    const float* __restrict__ packed, const float* __restrict__ bwd, const float* __restrict__ flat, int l,
    const float* __restrict__ state, const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ g_in,
    const float* __restrict__ g_lp, BwdOut o, int64_t B, float bound) {
  using BW = BwdR16<CF>;
  constexpr int K = CF::K, P = CF::P, H = CF::H, D = CF::D, C = CF::C, S = CF::S;
  constexpr int NLOW = S * (3 * K - 1);
  constexpr int SLOT = BwdSlot<CF>::v, ROWS = 16 * kBwdWaves;
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + SLOT;
  float* const glow = slot1 + SLOT;  // [NLOW] per-workgroup lower-spline gradient sums
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int q = lane >> 4;
  // the layer's raw lower-spline parameters, staged once per workgroup into LDS (read by the lower
  // spline VJP at the end of every tile: as global loads there they queued behind the next
  // tile's stage-0 LDS-DMA, vmcnt retiring in order)
  float* const lowp = glow + NLOW;
  for (int i = threadIdx.x; i < NLOW; i += blockDim.x) glow[i] = 0.f;

  const float* lp = packed + (int64_t)l * CF::LAYER;
  const float* lb = bwd + (int64_t)l * BW::LAYER;
  const float* low = flat + (int64_t)l * CF::FLAT + CF::N_W0 + CF::N_B0 + CF::N_W1 + CF::N_B1 + CF::N_W2 + CF::N_B2;
  if constexpr (CF::LOWER)
    for (int i = threadIdx.x; i < NLOW; i += blockDim.x) lowp[i] = low[i];  // published by the first ring barrier
  const int64_t ntiles = (B + ROWS - 1) / ROWS;
  const RqsConsts<K, true> rc(bound);
  constexpr int NSTG_F = CF::NSTG, NSTG = NSTG_F + BW::NSTG;
  auto stage_src = [&](int j) -> const float* { return j < NSTG_F ? lp + CF::stage_off(j) : lb + BW::stage_off(j - NSTG_F); };

  int g = 0;  // global stage counter: stage g lives in slot (g & 1)
  int64_t tile = blockIdx.x;
  if (tile < ntiles) stage_issue<CF::A_SIZE, kBwdWaves>(slot0, lp);  // A32 image never used: f16x3 path only
  for (; tile < ntiles; tile += gridDim.x) {
    const int64_t row = tile * ROWS + wave * 16 + (lane & 15);
    const bool valid = row < B;
    const int64_t crow = valid ? row : 0;
    float y1[CF::SQ], y2[CF::DQ], x1[CF::SQ];
#pragma unroll
    for (int u = 0; u < CF::SQ; ++u) y1[u] = valid ? state[crow * D + q * CF::SQ + u] : 0.f;
#pragma unroll
    for (int u = 0; u < CF::DQ; ++u) y2[u] = valid ? state[crow * D + S + q * CF::DQ + u] : 0.f;
    const float gl = valid ? g_lp[crow] : 0.f;
    // GEMM1's context k-slots and the upper dims' incoming gradients, loaded here, before the
    // stage-0 barrier: vmcnt retires in order, so a load issued after a stage's LDS-DMA (as when
    // these sat in stages 0 and C) is waited for together with that DMA
    float cpre[CF::KS1 * 8], gin[CF::DQ], ginl[CF::SQ];
#pragma unroll
    for (int t = 0; t < CF::KS1; ++t)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int col = r16_in_col<CF>(t, q, jj);
        cpre[8 * t + jj] = (col >= 0 && col < C) ? ctx[crow * ldc + col] : 0.f;
      }
#pragma unroll
    for (int u = 0; u < CF::DQ; ++u) gin[u] = valid ? g_in[crow * D + S + q * CF::DQ + u] : 0.f;
#pragma unroll
    for (int u = 0; u < CF::SQ; ++u) ginl[u] = valid ? g_in[crow * D + q * CF::SQ + u] : 0.f;

    floatx4 h1[CF::HB], h2[CF::HB], a3[CF::NO];
    float in[CF::KS1 * 8];
    floatx4 dp2[CF::HB];  // dPre2, then dPre1
    floatx4 dacc[CF::HB];
    Frag2 f3[CF::KS2];  // GEMM3's B fragments (gemm3_stage)
    floatx4 dx1;
    float gscale = 1.f;  // f16x3: natural units of the current backward GEMM's accumulator
    float gy2[CF::DQ];
    const bool has_next = tile + gridDim.x < ntiles;

    // tanh' epilogues of the dH2 / dH1 GEMMs: H re-read from this lane's own stores.  vmcnt
    // retires in order, so a load issued after a stage's LDS-DMA is waited for together with that
    // DMA: the epilogue of the last dH2 (dH1) stage therefore runs at the head of the NEXT stage,
    // after its barrier and before its DMA is issued (NAZ_BWD_EPI_LATE: at the stage's end, r02).
    auto epi_dh2 = [&]() {
#pragma unroll
      for (int b = 0; b < CF::HB; ++b) {
        // H2 re-read from this lane's own store (frees 32 VGPRs across the dH2 GEMM)
        const float4 hv = valid ? *reinterpret_cast<const float4*>(o.h2 + row * H + 16 * b + 4 * q)
                                : float4{0.f, 0.f, 0.f, 0.f};
        const float hh[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) dp2[b][r] = (dacc[b][r] * gscale) * (1.f - hh[r] * hh[r]);
        dacc[b] = floatx4{0.f, 0.f, 0.f, 0.f};
      }
    };
    auto epi_dh1 = [&]() {
#pragma unroll
      for (int b = 0; b < CF::HB; ++b) {
        const float4 hv = valid ? *reinterpret_cast<const float4*>(o.h1 + row * H + 16 * b + 4 * q)
                                : float4{0.f, 0.f, 0.f, 0.f};
        const float hh[4] = {hv.x, hv.y, hv.z, hv.w};
#pragma unroll
        for (int r = 0; r < 4; ++r) dp2[b][r] = (dacc[b][r] * gscale) * (1.f - hh[r] * hh[r]);  // now dPre1
      }
    };
#ifdef NAZ_BWD_EPI_LATE
    constexpr bool kEpiEarly = false;
#else
    constexpr bool kEpiEarly = true;
#endif

    static_for<0, NSTG>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      ring_barrier();  // stage j has landed in slot (g&1); every wave is done with the other slot
      if constexpr (kEpiEarly && j == NSTG_F + BW::NB3) epi_dh2();
      if constexpr (kEpiEarly && j == NSTG_F + BW::NB3 + BW::NB2) epi_dh1();
      const float* cur = (g & 1) ? slot1 : slot0;
      float* nxt = (g & 1) ? slot0 : slot1;
      if constexpr (j + 1 < NSTG_F) {
        stage_issue<CF::stage_size(j + 1), kBwdWaves>(nxt, stage_src(j + 1));
      } else if constexpr (j + 1 < NSTG) {
        stage_issue<BW::stage_size(j + 1 - NSTG_F), kBwdWaves>(nxt, stage_src(j + 1));
      } else {
        if (has_next) stage_issue<CF::A_SIZE, kBwdWaves>(nxt, lp);
      }
      ++g;

      if constexpr (j == 0) {
        // lower spline inverse (libm-grade, as the training forward), GEMM1 over [ctx | x1]
#pragma unroll
        for (int u = 0; u < CF::SQ; ++u) {
          x1[u] = y1[u];
          if constexpr (CF::LOWER) {
            const float* tp = cur + CF::A_TBL + (q * CF::SQ + u) * CF::TBL;
            float ld;
            if constexpr (kTrainFast) {
              x1[u] = rqs_table<K, true>(tp, y1[u], bound, ld);
            } else {
              SplineTables<K> tb;
#pragma unroll
              for (int k = 0; k <= K; ++k) {
                tb.cw[k] = tp[k];
                tb.ch[k] = tp[K + 1 + k];
                tb.dv[k] = tp[2 * (K + 1) + k];
              }
              x1[u] = rqs_apply<K, true, false>(tb, y1[u], bound, ld);
            }
          }
        }
#pragma unroll
        for (int t = 0; t < CF::KS1; ++t)
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            const int col = r16_in_col<CF>(t, q, jj);
            float v = 0.f;
            if (col >= C) {
              const int di = col - C - q * CF::SQ;  // this quarter's own x1 dims (static select)
#pragma unroll
              for (int u = 0; u < CF::SQ; ++u) v = di == u ? x1[u] : v;
            } else if (col >= 0) {
#ifdef NAZ_BWD_LATE_LOADS  // A/B only: the round-2 placement
              v = ctx[crow * ldc + col];
#else
              v = cpre[8 * t + jj];
#endif
            }
            in[8 * t + jj] = v;
            if (kBwdStore && valid && col >= 0) bwd_store_stream(o.x0 + row * (C + S) + col, v);
          }
        const float4* b4 = reinterpret_cast<const float4*>(cur + CF::A_BIAS);
#pragma unroll
        for (int b = 0; b < CF::HB; ++b) {
          const float4 bv = b4[4 * b + q];
          h1[b] = floatx4{bv.x, bv.y, bv.z, bv.w};
        }
        {  // f16x3 GEMM1: the caller guarantees |x|, |ctx| < 2^15 (so the training forward took
           // the same path; states stay within max(|x|, bound))
          Frag2 bf[CF::KS1];
#pragma unroll
          for (int t = 0; t < CF::KS1; ++t) {
            float v[8];
#pragma unroll
            for (int jj = 0; jj < 8; ++jj) v[jj] = in[8 * t + jj];
            bf[t] = split8_f16(v);
          }
          gemm_r16_stage<CF::HB, CF::KS1, kBwdPF>(h1, cur, lane, bf);
        }
        // activation -> natural tanh (stored) ; the next GEMM consumes -tanh/2 (the fold)
#pragma unroll
        for (int b = 0; b < CF::HB; ++b) {
#pragma unroll
          for (int r = 0; r < 4; ++r) h1[b][r] = train_fold(h1[b][r]);  // -tanh/2: GEMM2's operand
        }
      } else if constexpr (j <= CF::NB2) {
        constexpr int s = j - 1, T0 = s * CF::KB2;
        if constexpr (s == 0) {
          // weight-gradient operand stores go out at the HEAD of the stage after the one that
          // produced them: the next barrier's vmcnt(0) then waits on stores that drained under a
          // whole stage of compute, not on stores issued just before it
          if (kBwdStore && valid)
#pragma unroll
            for (int b = 0; b < CF::HB; ++b)
              *reinterpret_cast<float4*>(o.h1 + row * H + 16 * b + 4 * q) =
                  float4{-2.f * h1[b][0], -2.f * h1[b][1], -2.f * h1[b][2], -2.f * h1[b][3]};
          const float4* b4 = reinterpret_cast<const float4*>(cur + CF::B_BIAS);
#pragma unroll
          for (int b = 0; b < CF::HB; ++b) {
            const float4 bv = b4[4 * b + q];
            h2[b] = floatx4{bv.x, bv.y, bv.z, bv.w};
          }
        }
        gemm_r16_lazy<CF::HB, CF::KB2, T0, false, CF::HB, kBwdPF>(h2, cur, lane, h1);
        if constexpr (s == CF::NB2 - 1) {
#pragma unroll
          for (int b = 0; b < CF::HB; ++b) {
#pragma unroll
            for (int r = 0; r < 4; ++r) h2[b][r] = train_fold(h2[b][r]);
          }
        }
      } else if constexpr (j < NSTG_F) {
        constexpr int s = j - 1 - CF::NB2;
        if constexpr (s == 0) {
          if (kBwdStore && valid)
#pragma unroll
            for (int b = 0; b < CF::HB; ++b)
              *reinterpret_cast<float4*>(o.h2 + row * H + 16 * b + 4 * q) =
                  float4{-2.f * h2[b][0], -2.f * h2[b][1], -2.f * h2[b][2], -2.f * h2[b][3]};
        }
        gemm3_stage<CF, s, false>(a3, cur, lane, q, h2, f3);
        if constexpr (s == CF::NB3 - 1) {
          // ---- upper spline VJP (inverse map, libm-grade) -> dPre3 slots (in place of the raw
          // parameters: dim u's slots are read, then overwritten), g(y2)
#pragma unroll
          for (int u = 0; u < CF::DQ; ++u) {
            __builtin_amdgcn_sched_barrier(0);
            float uw[K], uh[K], ud[K - 1], gw[K], gh[K], gd[K - 1];
#pragma unroll
            for (int k = 0; k < K; ++k) {
              uw[k] = a3[(u * P + k) >> 2][(u * P + k) & 3];
              uh[k] = a3[(u * P + K + k) >> 2][(u * P + K + k) & 3];
            }
#pragma unroll
            for (int k = 0; k < K - 1; ++k) ud[k] = a3[(u * P + 2 * K + k) >> 2][(u * P + 2 * K + k) & 3];
#ifdef NAZ_BWD_LATE_LOADS
            const float go = valid ? g_in[crow * D + S + q * CF::DQ + u] : 0.f;
#else
            const float go = gin[u];
#endif
            gy2[u] = train_vjp_inv<K>(uw, uh, ud, bound, y2[u], go, gl, rc, gw, gh, gd);
#pragma unroll
            for (int k = 0; k < K; ++k) {
              a3[(u * P + k) >> 2][(u * P + k) & 3] = gw[k];
              a3[(u * P + K + k) >> 2][(u * P + K + k) & 3] = gh[k];
            }
#pragma unroll
            for (int k = 0; k < K - 1; ++k) a3[(u * P + 2 * K + k) >> 2][(u * P + 2 * K + k) & 3] = gd[k];
          }
#pragma unroll
          for (int sl = CF::DQ * P; sl < BW::NS3; ++sl) a3[sl >> 2][sl & 3] = 0.f;  // pad slots
#pragma unroll
          for (int b = 0; b < CF::HB; ++b) dacc[b] = floatx4{0.f, 0.f, 0.f, 0.f};
        }
      } else if constexpr (j < NSTG_F + BW::NB3) {
        // ---- dH2 = dPre3 · W2, k-steps of stage sb
        constexpr int sb = j - NSTG_F;
        if constexpr (sb == 0) {
          if (kBwdStore && valid) {
            float* dst = o.dp3 + row * (4 * BW::NS3) + q * BW::NS3;
#pragma unroll
            for (int b = 0; b < CF::NO; ++b)
              bwd_store_stream(reinterpret_cast<floatx4*>(dst + 4 * b), floatx4{a3[b][0], a3[b][1], a3[b][2], a3[b][3]});
          }
        }
        if constexpr (kBwdF16) {
          if constexpr (sb == 0) gscale = bwd_row_scale(a3);  // dPre3 already stored unscaled
          gemm_r16_lazy<CF::HB, BW::KB3, sb * BW::KB3, false, CF::NO, kBwdPF>(dacc, cur, lane, a3);
        } else {
          bwd_gemm_stage<CF::HB, BW::U3, sb * BW::U3>(dacc, cur, lane, a3);
        }
        if constexpr (!kEpiEarly && sb == BW::NB3 - 1) epi_dh2();
      } else if constexpr (j < NSTG_F + BW::NB3 + BW::NB2) {
        // ---- dH1 = dPre2 · W1
        constexpr int sb = j - NSTG_F - BW::NB3;
        if constexpr (sb == 0) {
          if (kBwdStore && valid)
#pragma unroll
            for (int b = 0; b < CF::HB; ++b)
              bwd_store_stream(reinterpret_cast<floatx4*>(o.dp2 + row * H + 16 * b + 4 * q), dp2[b]);
          if constexpr (kBwdF16) gscale = bwd_row_scale(dp2);
        }
        if constexpr (kBwdF16) gemm_r16_lazy<CF::HB, BW::KB2, sb * BW::KB2, false, CF::HB, kBwdPF>(dacc, cur, lane, dp2);
        else bwd_gemm_stage<CF::HB, BW::U2, sb * BW::U2>(dacc, cur, lane, dp2);
        if constexpr (!kEpiEarly && sb == BW::NB2 - 1) epi_dh1();
      } else {
        // ---- dx1 = dPre1 · W0[:, C:], lower spline VJP, g(P[l + 1])
        if (kBwdStore && valid)
#pragma unroll
          for (int b = 0; b < CF::HB; ++b)
            bwd_store_stream(reinterpret_cast<floatx4*>(o.dp1 + row * H + 16 * b + 4 * q), dp2[b]);
        if constexpr (kBwdF16) gscale = bwd_row_scale(dp2);
        floatx4 a1[1] = {floatx4{0.f, 0.f, 0.f, 0.f}};
        if constexpr (kBwdF16) {
          gemm_r16_lazy<1, BW::KSH, 0, false, CF::HB, kBwdPF>(a1, cur, lane, dp2);
#pragma unroll
          for (int r = 0; r < 4; ++r) a1[0][r] *= gscale;
        } else {
          bwd_gemm_stage<1, BW::UH, 0>(a1, cur, lane, dp2);
        }
        dx1 = a1[0];
        float gy1[CF::SQ];
#pragma unroll
        for (int u = 0; u < CF::SQ; ++u) {
          __builtin_amdgcn_sched_barrier(0);  // one dim's VJP at a time (its temporaries are large)
          const int dim = q * CF::SQ + u;
#ifdef NAZ_BWD_LATE_LOADS
          const float go = (valid ? g_in[crow * D + dim] : 0.f) + dx1[u];
#else
          const float go = ginl[u] + dx1[u];
#endif
          gy1[u] = go;
          if constexpr (CF::LOWER) {
            float uw[K], uh[K], ud[K - 1], gw[K], gh[K], gd[K - 1];
#pragma unroll
            for (int k = 0; k < K; ++k) {
              uw[k] = lowp[dim * K + k];
              uh[k] = lowp[S * K + dim * K + k];
            }
#pragma unroll
            for (int k = 0; k < K - 1; ++k) ud[k] = lowp[2 * S * K + dim * (K - 1) + k];
            gy1[u] = train_vjp_inv<K>(uw, uh, ud, bound, y1[u], go, gl, rc, gw, gh, gd);
            // sum over the wave's 16 rows (lanes of this quarter), then one LDS add per value
            auto red = [&](float v) {
              v += __shfl_xor(v, 1);
              v += __shfl_xor(v, 2);
              v += __shfl_xor(v, 4);
              v += __shfl_xor(v, 8);
              return v;
            };
#pragma unroll
            for (int k = 0; k < K; ++k) {
              const float a = red(gw[k]), b = red(gh[k]);
              if ((lane & 15) == 0) {
                atomicAdd(&glow[dim * K + k], a);
                atomicAdd(&glow[S * K + dim * K + k], b);
              }
            }
#pragma unroll
            for (int k = 0; k < K - 1; ++k) {
              const float a = red(gd[k]);
              if ((lane & 15) == 0) atomicAdd(&glow[2 * S * K + dim * (K - 1) + k], a);
            }
          }
        }
        if (valid) {
#pragma unroll
          for (int u = 0; u < CF::SQ; ++u) o.g_out[row * D + q * CF::SQ + u] = gy1[u];
#pragma unroll
          for (int u = 0; u < CF::DQ; ++u) o.g_out[row * D + S + q * CF::DQ + u] = gy2[u];
        }
      }
    });
  }
  __syncthreads();
  if constexpr (CF::LOWER)
    for (int i = threadIdx.x; i < NLOW; i += blockDim.x) atomicAdd(&o.g_low[i], glow[i]);
}

}  // namespace naz
