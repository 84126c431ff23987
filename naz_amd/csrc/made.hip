// Fused MADE conditioner + affine step: one launch per MAF layer in the forward (sampling)
// direction, batched over weight draws (SURVEY.md §8a a5/a6 forward, §8f rank 2).
//
// Replaces, per layer, pyro's ConditionalAutoRegressiveNN forward + AffineAutoregressive._call
// (naz/flows/transforms.py:133-160) and the JAX front end's forward_fn (bflow_jax_maf.py:172-178):
//   raw = W_out · act(… act(W_0 · [ctx | x] + b_0) …) + b_out     (masked weights)
//   y   = raw[:D] + x · exp(clamp(raw[D:], -5, 3)),   ld (+)= Σ clamp(raw[D:], -5, 3)
// Per row the kernel reads x (D floats) and writes y (D) and ld (1); the hidden activations
// never leave the registers.
//
// Mapping: a wave owns 32 rows; every GEMM runs TRANSPOSED on v_mfma_f32_32x32x2_f32 (exact
// fp32): A = weights (32 output features × 2 k), B = activations (2 k × 32 rows), so a layer's
// accumulator block o holds, in lane l, row l & 31 and features 32o + (r & 3) + 8(r >> 2) +
// 4(l >> 5) for register r — exactly the B operand of the next layer's k-steps 16o + r
// (lane-half l >> 5 supplies k = feature + 4(l >> 5)).  The packer permutes the weight columns to
// that order, so no shuffles or LDS round trips happen between layers.  Hidden/output weights
// stream from L2 through a double-buffered LDS ring in chunks of one input 32-block (NH KB × 4),
// shared by the workgroup's 4 waves (128 rows), with the next chunk's loads in flight during the
// current chunk's MFMAs; each lane reads 4 k-steps of A per ds_read_b128.  Layer 0 (K = C + D,
// small) reads A from global directly; the output block goes through LDS once for the affine step.
//
// Packed layout per draw (floats; NH = 32-wide blocks per hidden layer, S0 = k-steps of layer 0
// = ceil((C + D) / 2) rounded up to 4; all weights already multiplied by the MADE masks):
//   A0   [NH][S0/4][64 lanes][4]       lane l, step s: W0[32o + (l & 31)][2s + (l >> 5)]
//   b0   [NH][16][64]                  bias in accumulator order (feature of (o, r, lane))
//   hidden j = 1 .. nhid-1:  Aj [NH*4 t][NH o][64][4] (step s = 4t + q ↔ input feature of
//                            (s >> 4, s & 15)), bj [NH][16][64]
//   Aout [NH*4][64][4] (one 32-row output block: raw rows 0 .. 2D-1), bout [16][64]
#include "naz_device.h"
#include "naz_internal.h"

namespace naz {

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

struct MadeArgs {
  const float* w;  // packed nets, draw z at w + z * wstride
  int64_t wstride;
  int nhid, C, D, s0;
  const float* ctx;  // [C] (ldc = sctx = 0) or rows at ldc, draw stride sctx
  int64_t ldc, sctx;
  const float* x;
  int64_t ldx, sx;
  float* y;
  int64_t ldy, sy;
  float* ld;  // [rows] per draw at ld + z * sld
  int64_t sld;
  int ld_mode;
  int64_t S;  // rows per draw
  // inverse single-dim mode (naz_made_affine_inv1, inv_dim >= 0): raw rows 0, 1 = (mean, ls)
  // of dim inv_dim; y = x except y[inv_dim] = (v[inv_dim] - mean) exp(-clamp(ls))
  int inv_dim;
  const float* v;
  int64_t ldv, sv;
};

NAZ_DEV floatx16 mfma32(float a, float b, floatx16 c) { return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0); }

NAZ_DEV float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }

template <int NH, int ACT, int NW>
__global__ void __launch_bounds__(64 * NW, 8 / NW) made_affine_fwd_kernel(MadeArgs p) {
  // weight chunks of the hidden and output layers, double-buffered: one chunk = one input
  // 32-block of a hidden layer for all NH output blocks, or the whole output layer
  constexpr int CH4 = NH * 256;  // float4 per chunk
  __shared__ float4 Wl[2][CH4];
  constexpr int T = 64 * NW, PF = (CH4 + T - 1) / T;  // threads; prefetched float4 per thread
  constexpr bool RAGGED = CH4 % T != 0;
  __shared__ float E[NW][32][33];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, h = lane >> 5;
  const int64_t z = blockIdx.z;
  const float* W = p.w + z * p.wstride;
  const int64_t row = (int64_t)blockIdx.x * (32 * NW) + wave * 32 + (lane & 31);
  const bool live = row < p.S;
  const float* xr = p.x + z * p.sx + row * p.ldx;
  const float* cr = p.ctx + z * p.sctx + row * p.ldc;
  const int K0 = p.C + p.D;

  // chunk g -> float offset: hidden layer j = 1 + g / NH, input block c = g % NH; g = nchunk-1: output
  const int64_t hid0 = (int64_t)NH * p.s0 * 64 + NH * 1024;  // first hidden layer's A
  const int nchunk = (p.nhid - 1) * NH + 1;
  auto chunk_at = [&](int g) -> const float4* {
    const int j = g / NH, c = g % NH;  // j = hidden layers done before (0-based)
    return reinterpret_cast<const float4*>(W + hid0 + (int64_t)j * (NH * NH * 1024 + NH * 1024) +
                                           (int64_t)c * NH * 1024);
  };
  // the next chunk, in flight: named registers (an indexed array was kept in memory)
  float4 pf0, pf1, pf2, pf3, pf4;
#define NAZ_MADE_PF(K, OP) \
  if constexpr (PF > K) {  \
    if (!RAGGED || K * T + tid < CH4) OP; \
  }
#define NAZ_MADE_FETCH(G)                             \
  {                                                   \
    const float4* src_ = chunk_at(G);                 \
    NAZ_MADE_PF(0, pf0 = src_[tid])                   \
    NAZ_MADE_PF(1, pf1 = src_[T + tid])               \
    NAZ_MADE_PF(2, pf2 = src_[2 * T + tid])           \
    NAZ_MADE_PF(3, pf3 = src_[3 * T + tid])           \
    NAZ_MADE_PF(4, pf4 = src_[4 * T + tid])           \
  }
#define NAZ_MADE_STASH(BUF)                           \
  {                                                   \
    float4* dst_ = Wl[BUF];                           \
    NAZ_MADE_PF(0, dst_[tid] = pf0)                   \
    NAZ_MADE_PF(1, dst_[T + tid] = pf1)               \
    NAZ_MADE_PF(2, dst_[2 * T + tid] = pf2)           \
    NAZ_MADE_PF(3, dst_[3 * T + tid] = pf3)           \
    NAZ_MADE_PF(4, dst_[4 * T + tid] = pf4)           \
  }
  NAZ_MADE_FETCH(0)

  floatx16 acc[NH];
  float hv[NH][16];
#pragma unroll
  for (int o = 0; o < NH; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = 0.f;

  // layer 0: A from global (small), B operand straight from the row's [ctx | x]
  for (int t = 0; t < p.s0 / 4; ++t) {
    float bv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = 2 * (4 * t + q) + h;
      bv[q] = (live && k < K0) ? (k < p.C ? cr[k] : xr[k - p.C]) : 0.f;
    }
#pragma unroll
    for (int o = 0; o < NH; ++o) {
      const float4 a = ld4(W + ((int64_t)(o * (p.s0 / 4) + t) * 64 + lane) * 4);
      acc[o] = mfma32(a.x, bv[0], acc[o]);
      acc[o] = mfma32(a.y, bv[1], acc[o]);
      acc[o] = mfma32(a.z, bv[2], acc[o]);
      acc[o] = mfma32(a.w, bv[3], acc[o]);
    }
  }
  {
    const float* bias = W + (int64_t)NH * p.s0 * 64;
#pragma unroll
    for (int o = 0; o < NH; ++o)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        hv[o][r] = activate<ACT>(acc[o][r] + bias[(o * 16 + r) * 64 + lane]);
        acc[o][r] = 0.f;
      }
  }
  NAZ_MADE_STASH(0)
  __syncthreads();

  int g = 0;  // chunk being computed
  for (int j = 1; j < p.nhid; ++j) {
#pragma unroll
    for (int c = 0; c < NH; ++c) {  // input 32-block c of hidden layer j
      const float4* Wb = Wl[g & 1];
      if (g + 1 < nchunk) NAZ_MADE_FETCH(g + 1)  // in flight during this chunk's MFMAs
#ifndef NAZ_MADE_NO_PRIO  // MFMA chunk at wave priority 1 (same-box A/B: lp -1 %, sample -0.3 %)
      __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
      for (int t = 0; t < 4; ++t) {
#pragma unroll
        for (int o = 0; o < NH; ++o) {
          const float4 a = Wb[(t * NH + o) * 64 + lane];
          acc[o] = mfma32(a.x, hv[c][t * 4 + 0], acc[o]);
          acc[o] = mfma32(a.y, hv[c][t * 4 + 1], acc[o]);
          acc[o] = mfma32(a.z, hv[c][t * 4 + 2], acc[o]);
          acc[o] = mfma32(a.w, hv[c][t * 4 + 3], acc[o]);
        }
      }
#ifndef NAZ_MADE_NO_PRIO  // MFMA chunk at wave priority 1 (same-box A/B: lp -1 %, sample -0.3 %)
      __builtin_amdgcn_s_setprio(0);
#endif
      if (g + 1 < nchunk) {  // hand the prefetched chunk to the other buffer
        NAZ_MADE_STASH((g & 1) ^ 1)
      }
      __syncthreads();
      ++g;
    }
    // hidden layer complete: bias + activation -> next B operand
    const float* bj = W + hid0 + (int64_t)(j - 1) * (NH * NH * 1024 + NH * 1024) + NH * NH * 1024;
#pragma unroll
    for (int o = 0; o < NH; ++o)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        hv[o][r] = activate<ACT>(acc[o][r] + bj[(o * 16 + r) * 64 + lane]);
        acc[o][r] = 0.f;
      }
  }
  // output layer (chunk nchunk - 1): one 32-row block, raw rows 0 .. 2D-1
  floatx16 out;
#pragma unroll
  for (int r = 0; r < 16; ++r) out[r] = 0.f;
  {
    const float4* Wb = Wl[g & 1];
#pragma unroll
    for (int t = 0; t < NH * 4; ++t) {
      const float4 a = Wb[t * 64 + lane];
      out = mfma32(a.x, hv[t >> 2][(t & 3) * 4 + 0], out);
      out = mfma32(a.y, hv[t >> 2][(t & 3) * 4 + 1], out);
      out = mfma32(a.z, hv[t >> 2][(t & 3) * 4 + 2], out);
      out = mfma32(a.w, hv[t >> 2][(t & 3) * 4 + 3], out);
    }
  }

  const float* bo = W + hid0 + (int64_t)(p.nhid - 1) * (NH * NH * 1024 + NH * 1024) + NH * 1024;
#pragma unroll
  for (int r = 0; r < 16; ++r) E[wave][lane & 31][(r & 3) + 8 * (r >> 2) + 4 * h] = out[r] + bo[r * 64 + lane];
  __syncthreads();

  // affine step, one lane per row
  if (h == 0 && live && p.inv_dim >= 0) {
    float* yr = p.y + z * p.sy + row * p.ldy;
    const float ls = fminf(fmaxf(E[wave][lane][1], -5.f), 3.f);
    for (int i = 0; i < p.D; ++i)
      yr[i] = i == p.inv_dim ? (p.v[z * p.sv + row * p.ldv + i] - E[wave][lane][0]) * expf(-ls) : xr[i];
    float* l = p.ld + z * p.sld + row;
    if (p.ld_mode == NAZ_LD_ROWSUM) *l = ls;
    else if (p.ld_mode == NAZ_LD_ROWSUM_ADD) *l += ls;
    else if (p.ld_mode == NAZ_LD_ROWSUM_SUB) *l -= ls;
  } else if (h == 0 && live) {
    float s = 0.f;
    float* yr = p.y + z * p.sy + row * p.ldy;
    for (int i = 0; i < p.D; ++i) {
      const float mean = E[wave][lane][i];
      const float ls = fminf(fmaxf(E[wave][lane][p.D + i], -5.f), 3.f);
      yr[i] = expf(ls) * xr[i] + mean;
      s += ls;
    }
    float* l = p.ld + z * p.sld + row;
    if (p.ld_mode == NAZ_LD_ROWSUM) *l = s;
    else if (p.ld_mode == NAZ_LD_ROWSUM_ADD) *l += s;
    else if (p.ld_mode == NAZ_LD_ROWSUM_SUB) *l -= s;
  }
}

#undef NAZ_MADE_PF
#undef NAZ_MADE_FETCH
#undef NAZ_MADE_STASH

template <int NH, int NW>
void launch_nw(const MadeArgs& a, int act, int P, hipStream_t s) {
  dim3 grid((unsigned)((a.S + 32 * NW - 1) / (32 * NW)), 1, (unsigned)P);
  if (act == ACT_TANH) hipLaunchKernelGGL((made_affine_fwd_kernel<NH, ACT_TANH, NW>), grid, dim3(64 * NW), 0, s, a);
  else hipLaunchKernelGGL((made_affine_fwd_kernel<NH, ACT_RELU, NW>), grid, dim3(64 * NW), 0, s, a);
}

// waves per workgroup: rows sharing one staged weight chunk (NAZ_MADE_WAVES=4|8 overrides)
template <int NH>
void launch_nh(const MadeArgs& a, int act, int P, hipStream_t s) {
  static const int nw = [] {
    const char* e = getenv("NAZ_MADE_WAVES");
    return e ? atoi(e) : 4;
  }();
  if (nw == 8) launch_nw<NH, 8>(a, act, P, s);
  else launch_nw<NH, 4>(a, act, P, s);
}

}  // namespace

static int made_launch(const MadeArgs& a, int nh, int act, int P, hipStream_t s);

int64_t made_packed_floats(int nhid, int nh, int C, int D) {
  const int s0 = ((C + D + 1) / 2 + 3) / 4 * 4;
  return (int64_t)nh * s0 * 64 + (int64_t)nh * 1024 + (int64_t)(nhid - 1) * (nh * nh * 1024 + nh * 1024) +
         (int64_t)nh * 1024 + 1024;
}

int made_affine_fwd(const float* packed, int64_t wstride, int nhid, int nh, int C, int D, const float* ctx,
                    int64_t ldc, int64_t sctx, const float* x, int64_t ldx, int64_t sx, float* y, int64_t ldy,
                    int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, hipStream_t s) {
  if (S == 0 || P == 0) return 0;
  if (nh < 1 || nh > 5) return set_error("naz_made_affine_fwd: hidden blocks %d not in 1..5 (width <= 160)", nh);
  if (nhid < 1) return set_error("naz_made_affine_fwd: needs >= 1 hidden layer");
  if (D < 1 || 2 * D > 32) return set_error("naz_made_affine_fwd: D=%d (2D must fit one 32-row block)", D);
  if (C < 0 || (C > 0 && ctx == nullptr)) return set_error("naz_made_affine_fwd: bad context");
  if (act != ACT_TANH && act != ACT_RELU) return set_error("naz_made_affine_fwd: activation %d not built", act);
  if (P > 65535) return set_error("naz_made_affine_fwd: P=%d > 65535", P);
  if (ld == nullptr || ld_mode < NAZ_LD_ROWSUM || ld_mode > NAZ_LD_ROWSUM_SUB)
    return set_error("naz_made_affine_fwd: ld must be a row-sum buffer (mode %d)", ld_mode);
  if ((reinterpret_cast<uintptr_t>(packed) & 15) || (wstride & 3))
    return set_error("naz_made_affine_fwd: packed nets must be 16-byte aligned");
  if (wstride < made_packed_floats(nhid, nh, C, D)) return set_error("naz_made_affine_fwd: wstride too small");
  MadeArgs a{};
  a.w = packed;
  a.wstride = wstride;
  a.nhid = nhid;
  a.C = C;
  a.D = D;
  a.s0 = ((C + D + 1) / 2 + 3) / 4 * 4;
  a.ctx = C > 0 ? ctx : x;
  a.ldc = ldc;
  a.sctx = sctx;
  a.x = x;
  a.ldx = ldx;
  a.sx = sx;
  a.y = y;
  a.ldy = ldy;
  a.sy = sy;
  a.ld = ld;
  a.sld = sld;
  a.ld_mode = ld_mode;
  a.S = S;
  a.inv_dim = -1;
  a.v = nullptr;
  return made_launch(a, nh, act, P, s);
}

int made_affine_inv1(const float* packed, int64_t wstride, int nhid, int nh, int D, const float* x, int64_t ldx,
                     int64_t sx, const float* v, int64_t ldv, int64_t sv, int dim, float* y, int64_t ldy, int64_t sy,
                     float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, hipStream_t s) {
  if (S == 0 || P == 0) return 0;
  if (nh < 1 || nh > 5) return set_error("naz_made_affine_inv1: hidden blocks %d not in 1..5 (width <= 160)", nh);
  if (nhid < 1) return set_error("naz_made_affine_inv1: needs >= 1 hidden layer");
  if (D < 1 || dim < 0 || dim >= D) return set_error("naz_made_affine_inv1: dim %d not in [0, D=%d)", dim, D);
  if (act != ACT_TANH && act != ACT_RELU) return set_error("naz_made_affine_inv1: activation %d not built", act);
  if (P > 65535) return set_error("naz_made_affine_inv1: P=%d > 65535", P);
  if (ld == nullptr || v == nullptr || ld_mode < NAZ_LD_ROWSUM || ld_mode > NAZ_LD_ROWSUM_SUB)
    return set_error("naz_made_affine_inv1: v and a row-sum ld buffer are required");
  if ((reinterpret_cast<uintptr_t>(packed) & 15) || (wstride & 3))
    return set_error("naz_made_affine_inv1: packed nets must be 16-byte aligned");
  if (wstride < made_packed_floats(nhid, nh, 0, D)) return set_error("naz_made_affine_inv1: wstride too small");
  MadeArgs a{};
  a.w = packed;
  a.wstride = wstride;
  a.nhid = nhid;
  a.C = 0;
  a.D = D;
  a.s0 = ((D + 1) / 2 + 3) / 4 * 4;
  a.ctx = x;
  a.x = x;
  a.ldx = ldx;
  a.sx = sx;
  a.y = y;
  a.ldy = ldy;
  a.sy = sy;
  a.ld = ld;
  a.sld = sld;
  a.ld_mode = ld_mode;
  a.S = S;
  a.inv_dim = dim;
  a.v = v;
  a.ldv = ldv;
  a.sv = sv;
  return made_launch(a, nh, act, P, s);
}

static int made_launch(const MadeArgs& a, int nh, int act, int P, hipStream_t s) {
  switch (nh) {
    case 1: launch_nh<1>(a, act, P, s); break;
    case 2: launch_nh<2>(a, act, P, s); break;
    case 3: launch_nh<3>(a, act, P, s); break;
    case 4: launch_nh<4>(a, act, P, s); break;
    default: launch_nh<5>(a, act, P, s); break;
  }
  return check_launch("made_affine_fwd_kernel");
}

}  // namespace naz
