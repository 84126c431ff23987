// Fused conditional spline-coupling flow: log_prob and sample for all L layers in
// ONE launch (§7 steps 4-5).
//
// Reference semantics: naz NormalizingFlow.log_prob (naz/flows/flow.py:45-79) over
// flow_type "nsc" (naz/flows/transforms.py:201-236 intent = pyro SplineCoupling
// with a ConditionalDenseNN hypernet, DenseNN input cat([ctx, x1]), tanh):
//   for l = L-1 .. 0:  x1 = lower.inv(y1);  raw = MLP([ctx, x1]);  x2 = RQS^-1(y2; raw)
//                      lp -= sum(ld_upper) + sum(ld_lower)
//   lp += sum(-z^2/2 - log sqrt(2 pi))
//
// MI355X mapping (see DESIGN.md §Fused coupling kernel):
//   * workgroup = 4 waves = 128 batch rows; wave = 32 rows; lane l owns batch row
//     (l & 31) and lane-half h = l >> 5 owns half of that row's dims;
//   * activations live TRANSPOSED in MFMA accumulators (feature = accumulator row,
//     batch row = accumulator column = lane & 31).  v_mfma_f32_32x32x2_f32's B operand
//     is B[k = l>>5][j = l&31], so accumulator register r of layer n IS the B operand
//     of k-step r of layer n+1 — the three GEMMs chain with no LDS and no shuffles;
//     the weight packer permutes W's columns to match (hid_feature below);
//   * the last GEMM's output rows are permuted so that lane-half h receives all
//     3K-1 spline parameters of its own Dt/2 upper dims in registers: the spline,
//     log-det and base density run per lane with no cross-lane traffic until the
//     final one-shuffle row reduction;
//   * weights (the A operands, exact fp32 MFMA) are staged per GEMM into LDS as
//     [block][k/4][lane][4] panels read by ds_read_b128; one stage <= 64 KB so two
//     workgroups share a CU and overlap each other's VALU (spline/tanh) with MFMA.
// Compiled three times by naz_amd/build.py (objects built in parallel): NAZ_PART=1 the coupling
// flows' dispatch and kernels, NAZ_PART=2 the autoregressive (made_ar_r16.h) ones, NAZ_PART=3 the
// autoregressive backward (made_ar_bwd.h); the parts share the device helpers above the dispatch
// sections.  Without NAZ_PART all are built.
#ifndef NAZ_PART
#define NAZ_PART 0
#endif
#include "naz_device.h"
#include "naz_internal.h"

#include <algorithm>
#include <type_traits>

namespace naz {

typedef float floatx16 __attribute__((ext_vector_type(16)));

NAZ_DEV floatx16 mfma32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// accumulator register r on lane-half h holds feature row (within a 32-block)
__host__ __device__ constexpr int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }
// Feature (input column of the next GEMM) carried by k-step t on lane-half h.
__host__ __device__ constexpr int hid_feature(int t, int h) { return 32 * (t >> 4) + acc_row(t & 15, h); }

constexpr int kStageFloats = 16384;  // 64 KB per LDS stage
constexpr int kRowsPerWG = 128;

template <int D_, int C_, int S_, int K_, int H_, bool LOWER_>
struct CouplingCfg {
  static constexpr int D = D_, C = C_, S = S_, K = K_, H = H_;
  static constexpr bool LOWER = LOWER_;
  static constexpr int Dt = D - S;
  static constexpr int P = 3 * K - 1;       // raw params per upper dim
  static constexpr int DH = Dt / 2;         // upper dims per lane-half
  static constexpr int SH = S / 2;          // lower dims per lane-half
  static constexpr int CH = (C + 1) / 2;    // context features per lane-half
  static constexpr int CHA = CH > 0 ? CH : 1;
  static constexpr int KS0 = CH + SH;       // GEMM1 k-steps (2 features each)
  static constexpr int KS0P = (KS0 + 3) / 4 * 4;
  static constexpr int HB = H / 32;         // hidden 32-row blocks
  static constexpr int KS1 = H / 2;         // GEMM2/3 k-steps
  static constexpr int NO = (DH * P + 15) / 16;  // GEMM3 output blocks
  static constexpr int TBL = 3 * (K + 1);   // lower-spline table floats per dim
  static constexpr int PANEL0 = KS0P * 64;
  static constexpr int PANEL1 = KS1 * 64;
  static constexpr int PPS = kStageFloats / PANEL1;  // GEMM2/3 panels per stage
  static constexpr int NSTG3 = (NO + PPS - 1) / PPS;
  // stage A: [HB panels0][HB*32 bias][S*TBL tables]  (padded to 4 floats)
  static constexpr int A_BIAS = HB * PANEL0;
  static constexpr int A_TBL = A_BIAS + HB * 32;
  static constexpr int A_SIZE = (A_TBL + S * TBL + 255) / 256 * 256;
  // stage B: [HB panels1][HB*32 bias]
  static constexpr int B_OFF = A_SIZE;
  static constexpr int B_BIAS = HB * PANEL1;
  static constexpr int B_SIZE = (B_BIAS + HB * 32 + 255) / 256 * 256;
  // stages C_j: [n_j panels1][n_j*32 bias]
  static constexpr int C_OFF = B_OFF + B_SIZE;
  static constexpr int C_STRIDE = (PPS * PANEL1 + PPS * 32 + 255) / 256 * 256;
  static constexpr __host__ __device__ int c_count(int j) { return (NO - j * PPS) < PPS ? (NO - j * PPS) : PPS; }
  static constexpr __host__ __device__ int c_off(int j) { return C_OFF + j * C_STRIDE; }
  static constexpr __host__ __device__ int c_size(int j) { return (c_count(j) * (PANEL1 + 32) + 255) / 256 * 256; }
  static constexpr int LAYER = C_OFF + (NSTG3 - 1) * C_STRIDE + c_size(NSTG3 - 1);
  static constexpr int MAX_AB = A_SIZE > B_SIZE ? A_SIZE : B_SIZE;
  static constexpr int MAXSTAGE = MAX_AB > C_STRIDE ? MAX_AB : C_STRIDE;
  // flat (natural) parameter layout per layer
  static constexpr int N_W0 = H * (C + S), N_B0 = H, N_W1 = H * H, N_B1 = H, N_W2 = Dt * P * H, N_B2 = Dt * P;
  static constexpr int N_LOW = LOWER ? S * (3 * K - 1) : 0;
  static constexpr int FLAT = N_W0 + N_B0 + N_W1 + N_B1 + N_W2 + N_B2 + N_LOW;
  static_assert(Dt % 2 == 0 && S % 2 == 0 && H % 32 == 0 && S > 0 && Dt > 0, "unsupported coupling shape");
  static_assert(PPS >= 1, "hidden width too large for one LDS stage");
  static_assert(MAXSTAGE * 4 <= 80 * 1024, "stage exceeds the per-workgroup LDS budget");
  static_assert(A_SIZE % 256 == 0 && B_SIZE % 256 == 0 && C_STRIDE % 256 == 0 && LAYER % 256 == 0, "stage alignment");
};

// ---------------------------------------------------------------------------
// Packing kernel: flat natural params -> MFMA panel order (+ lower-spline tables)
// ---------------------------------------------------------------------------
template <class CF>
__global__ void coupling_pack_kernel(const float* __restrict__ flat, float* __restrict__ packed, int L, float bound) {
  const int64_t n = (int64_t)L * CF::LAYER;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int l = (int)(e / CF::LAYER);
    const int off = (int)(e - (int64_t)l * CF::LAYER);
    const float* W0 = flat + (int64_t)l * CF::FLAT;
    const float* b0 = W0 + CF::N_W0;
    const float* W1 = b0 + CF::N_B0;
    const float* b1 = W1 + CF::N_W1;
    const float* W2 = b1 + CF::N_B1;
    const float* b2 = W2 + CF::N_W2;
    const float* low = b2 + CF::N_B2;  // unnormalized widths [S,K] | heights [S,K] | derivatives [S,K-1]
    float v = 0.f;
    if (off < CF::A_SIZE) {
      if (off < CF::A_BIAS) {  // W0 panels: [o][t/4][lane][t%4]
        const int o = off / CF::PANEL0, rem = off - o * CF::PANEL0;
        const int t = (rem / 256) * 4 + (rem & 3), lane = (rem >> 2) & 63;
        const int i = lane & 31, kh = lane >> 5;
        int col = -1;
        if (t < CF::CH) {
          const int c = kh * CF::CH + t;
          if (c < CF::C) col = c;
        } else if (t < CF::KS0) {
          col = CF::C + kh * CF::SH + (t - CF::CH);
        }
        if (col >= 0) v = W0[(32 * o + i) * (CF::C + CF::S) + col];
      } else if (off < CF::A_TBL) {
        const int q = off - CF::A_BIAS, o = q / 32, h = (q >> 4) & 1, r = q & 15;
        v = b0[32 * o + acc_row(r, h)];
      } else if (CF::LOWER && off < CF::A_TBL + CF::S * CF::TBL) {
        const int q = off - CF::A_TBL, g = q / CF::TBL, w = q - g * CF::TBL;
        float uw[CF::K], uh[CF::K], ud[CF::K - 1];
        for (int k = 0; k < CF::K; ++k) {
          uw[k] = low[g * CF::K + k];
          uh[k] = low[CF::S * CF::K + g * CF::K + k];
        }
        for (int k = 0; k < CF::K - 1; ++k) ud[k] = low[2 * CF::S * CF::K + g * (CF::K - 1) + k];
        SplineTables<CF::K> tb;
        build_tables<CF::K>(uw, uh, ud, bound, tb);
        const int which = w / (CF::K + 1), k = w - which * (CF::K + 1);
        v = which == 0 ? tb.cw[k] : (which == 1 ? tb.ch[k] : tb.dv[k]);
      }
    } else if (off < CF::C_OFF) {
      const int q = off - CF::B_OFF;
      if (q < CF::B_BIAS) {
        const int o = q / CF::PANEL1, rem = q - o * CF::PANEL1;
        const int t = (rem / 256) * 4 + (rem & 3), lane = (rem >> 2) & 63;
        v = W1[(32 * o + (lane & 31)) * CF::H + hid_feature(t, lane >> 5)];
      } else {
        const int qq = q - CF::B_BIAS, o = qq / 32, h = (qq >> 4) & 1, r = qq & 15;
        v = b1[32 * o + acc_row(r, h)];
      }
    } else {
      int j = (off - CF::C_OFF) / CF::C_STRIDE;
      const int q = off - CF::c_off(j), cnt = CF::c_count(j);
      const bool is_w = q < cnt * CF::PANEL1;
      int o, h, r, col = 0;
      if (is_w) {
        const int ob = q / CF::PANEL1, rem = q - ob * CF::PANEL1;
        const int t = (rem / 256) * 4 + (rem & 3), lane = (rem >> 2) & 63;
        const int i = lane & 31;               // A row = output row within block
        o = j * CF::PPS + ob;
        h = (i >> 2) & 1;                      // which lane-half's accumulator holds row i
        r = (i & 3) + 4 * (i >> 3);            // ... in which register
        col = hid_feature(t, lane >> 5);       // A column = k-step feature
      } else {
        const int qq = q - cnt * CF::PANEL1, ob = qq / 32;
        o = j * CF::PPS + ob;
        h = (qq >> 4) & 1;
        r = qq & 15;
      }
      // slot (o, r) on half h -> (upper dim, param) -> DenseNN output column
      const int slot = 16 * o + r, qd = slot / CF::P, p = slot - qd * CF::P;
      if (qd < CF::DH) {
        const int dim = h * CF::DH + qd;
        int orig;
        if (p < CF::K) orig = dim * CF::K + p;
        else if (p < 2 * CF::K) orig = CF::Dt * CF::K + dim * CF::K + (p - CF::K);
        else orig = 2 * CF::Dt * CF::K + dim * (CF::K - 1) + (p - 2 * CF::K);
        v = is_w ? W2[orig * CF::H + col] : b2[orig];
      }
    }
    packed[e] = v;
  }
}

// ---------------------------------------------------------------------------
// Stage copy HBM/L2 -> LDS (16-byte loads, all 256 threads)
// ---------------------------------------------------------------------------
// LDS (address space 3) pointer of a generic pointer into __shared__ memory: the low 32 bits
// of a flat LDS address are the LDS offset.  An addrspacecast would instead emit a null check
// against src_shared_base, which hipcc (ROCm 7.2) mis-encodes (v_cmp_ne_u32_e32 with
// src_shared_base as src1: "Operand has incorrect register class") once the address space
// cannot be inferred (the wide H = 512 forward kernel).
NAZ_DEV __attribute__((address_space(3))) void* to_lds(const void* p) {
  return (__attribute__((address_space(3))) void*)(uint32_t)(uintptr_t)p;
}

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
// One 16-byte LDS read whose destination hipcc does not track (inline asm): the compiler's waitcnt
// model treats LDS returns as out of order while an LDS-DMA (global_load_lds) is in flight — i.e.
// always inside the ring kernels — and so waits lgkmcnt(0) before every use, including on the
// reads just issued for the NEXT use.  Here the wait is explicit and counted (lds_wait<N>): LDS
// reads return in order (LGKM also counts SMEM, which returns out of order: the kernels using this
// issue none across a counted wait — tests/test_isa_ring.py's counted-wait rule — and the DMA
// counts on vmcnt).  Users: coupling_w32.h (A fragments), made_ar_wide.h.
template <int OFF>
NAZ_DEV u32x4_t lds_read_b128_untracked(unsigned addr) {
  u32x4_t v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF));
  return v;
}
template <int N>
NAZ_DEV void lds_wait() {
  // s_waitcnt lgkmcnt(N), vmcnt / expcnt left at their maxima (gfx9 encoding)
  __builtin_amdgcn_s_waitcnt(0xC07F | (N << 8));
}


// Asynchronous stage copy HBM/L2 -> LDS with LDS-DMA (global_load_lds_dwordx4): wave w
// moves 1 KB chunks w, w+4, ...; no VGPRs hold the data.  Completion is published by the
// next ring_barrier() (naz_device.h: explicit vmcnt(0), then the barrier) — never by a bare
// __syncthreads(), which hipcc does not always precede with vmcnt(0).
template <int NFLOATS, int NW = 4>
NAZ_DEV void stage_issue(float* lds, const float* __restrict__ src) {
#ifdef NAZ_ABL_NOCOPY
  return;
#endif
  static_assert(NFLOATS % 256 == 0, "stage must be whole 1 KB chunks");
  constexpr int CHUNKS = NFLOATS / 256;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int c0 = 0; c0 < CHUNKS; c0 += NW) {
    const int c = c0 + wave;
    if (c0 + NW - 1 < CHUNKS || c < CHUNKS) {
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(src + c * 256 + lane * 4),
          to_lds(lds + c * 256), 16, 0, 0);
    }
  }
}

// NAZ_DEBUG_NONFINITE builds (python -m naz_amd.build debug -DNAZ_DEBUG_NONFINITE): the fused
// log_prob kernels record the FIRST non-finite row state as {1, workgroup, layer, stage counter,
// row} (naz_debug_nonfinite reads and clears it).  The record exists in every build; only the
// debug build writes it.
#if NAZ_PART == 0 || NAZ_PART == 1
__device__ int64_t g_nonfinite[5];
#else
extern __device__ int64_t g_nonfinite[5];
#endif
NAZ_DEV void debug_nonfinite_probe(bool bad, int64_t row, int layer, int stage) {
  if (bad && atomicCAS(reinterpret_cast<unsigned long long*>(&g_nonfinite[0]), 0ull, 1ull) == 0ull) {
    g_nonfinite[1] = blockIdx.x;
    g_nonfinite[2] = layer;
    g_nonfinite[3] = stage;
    g_nonfinite[4] = row;
  }
}

// The same copy through a buffer resource (buffer_load_dwordx4 ... lds): the per-lane offset is
// one VGPR set once (lane * 16) and each chunk's offset is scalar (soffset), so a chunk costs no
// 64-bit VALU address add (global_load_lds needs one per chunk and lane).  `off` = the stage's
// float offset from the resource base (wave-uniform).  Out-of-range chunks read zeros, never fault.
struct RingSrc {
  const float* base;
  __amdgpu_buffer_rsrc_t r;
  NAZ_DEV RingSrc(const float* base_, int64_t nfloats)
      : base(base_), r(__builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base_), 0,
                                            (int)(nfloats * 4 < 0x7fffffff ? nfloats * 4 : 0x7fffffff), 0x00020000)) {}
};

// Default OFF (NAZ_RING_BUF enables it): same-box A/B on the headline kernel, 2^20 rows, two
// repetitions: global_load_lds 2.242 / 2.243 ms, buffer_load ... lds 2.284 / 2.290 ms
// (profiles/r03_s3_ab_ring.txt) — the saved 64-bit address adds do not pay for the slower form.
template <int NFLOATS, int NW>
NAZ_DEV void stage_issue(float* lds, const RingSrc& src, int off) {
#ifndef NAZ_RING_BUF
  return stage_issue<NFLOATS, NW>(lds, src.base + off);
#endif
  static_assert(NFLOATS % 256 == 0, "stage must be whole 1 KB chunks");
  constexpr int CHUNKS = NFLOATS / 256;
  const int vo = (threadIdx.x & 63) * 16;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#pragma unroll
  for (int c0 = 0; c0 < CHUNKS; c0 += NW) {
    const int c = c0 + wave;
    if (c0 + NW - 1 < CHUNKS || c < CHUNKS) {
      __builtin_amdgcn_raw_ptr_buffer_load_lds(src.r, to_lds(lds + c * 256), 16, vo,
                                               (off + c * 256) * 4, 0, 0);
    }
  }
}

// stage_issue of the first nch (wave-uniform, <= NFLOATS / 256) 1 KB chunks only
template <int NFLOATS, int NW>
NAZ_DEV void stage_issue_lim(float* lds, const float* __restrict__ src, int nch) {
  static_assert(NFLOATS % 256 == 0, "stage must be whole 1 KB chunks");
  constexpr int CHUNKS = NFLOATS / 256;
  // (the lane offset is formed here, per issue: hoisted out of the layer loop as a 64-bit per-lane
  // source base it was one of the three pointers the nsa16 inverse spilled, and its scratch reload
  // sat right before a stage's DMA issue)
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  nch = nch < CHUNKS ? nch : CHUNKS;
#pragma unroll
  for (int c0 = 0; c0 < CHUNKS; c0 += NW) {
    const int c = c0 + wave;
    if (c < nch) {
      __builtin_amdgcn_global_load_lds(
          (const void __attribute__((address_space(1)))*)(src + c * 256 + lane * 4),
          to_lds(lds + c * 256), 16, 0, 0);
    }
  }
}

// Accumulators init from the packed bias block [o][h][16]
template <int NB>
NAZ_DEV void init_bias(floatx16 (&acc)[NB], const float* __restrict__ bias, int h) {
#pragma unroll
  for (int o = 0; o < NB; ++o) {
    const float4* b4 = reinterpret_cast<const float4*>(bias + (o * 2 + h) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 v = b4[q];
      acc[o][4 * q + 0] = v.x;
      acc[o][4 * q + 1] = v.y;
      acc[o][4 * q + 2] = v.z;
      acc[o][4 * q + 3] = v.w;
    }
  }
}

// acc[o] += W-panel(o) x B for all NT k-steps; B operand for k-step t is bop(t).
// panels: [NB][NT/4][64][4] in LDS.
template <int NB, int NT, class BOp>
NAZ_DEV void gemm_panels(floatx16 (&acc)[NB], const float* __restrict__ panels, int lane, BOp bop) {
  const float4* p4 = reinterpret_cast<const float4*>(panels);
#pragma unroll
  for (int t4 = 0; t4 < NT / 4; ++t4) {
    float4 a[NB];
#pragma unroll
    for (int o = 0; o < NB; ++o) a[o] = p4[(o * (NT / 4) + t4) * 64 + lane];
#pragma unroll
    for (int o = 0; o < NB; ++o) acc[o] = mfma32(a[o].x, bop(4 * t4 + 0), acc[o]);
#pragma unroll
    for (int o = 0; o < NB; ++o) acc[o] = mfma32(a[o].y, bop(4 * t4 + 1), acc[o]);
#pragma unroll
    for (int o = 0; o < NB; ++o) acc[o] = mfma32(a[o].z, bop(4 * t4 + 2), acc[o]);
#pragma unroll
    for (int o = 0; o < NB; ++o) acc[o] = mfma32(a[o].w, bop(4 * t4 + 3), acc[o]);
  }
}

template <int NB>
NAZ_DEV void tanh_all(floatx16 (&acc)[NB]) {
#pragma unroll
  for (int o = 0; o < NB; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = tanh_f<true>(acc[o][r]);
}

template <int I, int N, class F>
NAZ_DEV void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// ---------------------------------------------------------------------------
// Main fused kernel.  DIR_INV = true: log_prob (layers reversed, inverse maps).
//
// Per layer the LDS buffer holds, in turn, stage A (W0 + b0 + lower tables), B (W1 + b1)
// and C_j (W2 panel groups + b2).  Each stage's LDS-DMA copy is issued right after the
// barrier that frees the buffer and lands while the waves run the VALU epilogue of the
// GEMM just finished (tanh, or the spline), so copies hide behind VALU work and the
// second co-resident workgroup keeps the matrix pipe busy meanwhile.
// ---------------------------------------------------------------------------
template <class CF>
NAZ_DEV void load_tables(const float* tb, SplineTables<CF::K>& t) {
#pragma unroll
  for (int k = 0; k <= CF::K; ++k) {
    t.cw[k] = tb[k];
    t.ch[k] = tb[CF::K + 1 + k];
    t.dv[k] = tb[2 * (CF::K + 1) + k];
  }
}

template <class CF, bool DIR_INV>
__global__ void __launch_bounds__(256, 2) coupling_flow_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ out_lp, float* __restrict__ yout, int64_t ldy, int64_t B, float bound) {
  extern __shared__ float4 lds4[];
  float* lds = reinterpret_cast<float*>(lds4);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int64_t row = (int64_t)blockIdx.x * kRowsPerWG + wave * 32 + (lane & 31);
  const bool valid = row < B;
  const int64_t crow = valid ? row : 0;  // clamp so every lane can load unconditionally

  // first layer's stage A goes out before anything else
  stage_issue<CF::A_SIZE>(lds, packed + (int64_t)(DIR_INV ? (L - 1) : 0) * CF::LAYER);

  // ---- per-lane state: lower dims {h*SH..}, upper dims {S + h*DH..}
  float zl[CF::SH], zu[CF::DH];
  float ldsum = 0.f;   // sum of per-dim FORWARD log-dets over this lane's dims
  float logjac = 0.f;  // bounding prologue contribution (log_prob only)
#pragma unroll
  for (int q = 0; q < CF::SH; ++q) zl[q] = valid ? x[crow * ldx + h * CF::SH + q] : 0.f;
#pragma unroll
  for (int q = 0; q < CF::DH; ++q) zu[q] = valid ? x[crow * ldx + CF::S + h * CF::DH + q] : 0.f;

  if (DIR_INV && low != nullptr) {  // naz bounding_transform (transforms.py:20-23)
    auto bnd = [&](float& v, int dim) {
      const float lo = low[dim], hi = high[dim];
      const float u = (v - lo) / (hi - lo);
      logjac -= logf(u) + log1pf(-u);
      v = logf(u / (1.f - u));
    };
#pragma unroll
    for (int q = 0; q < CF::SH; ++q) bnd(zl[q], h * CF::SH + q);
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) bnd(zu[q], CF::S + h * CF::DH + q);
    if (h == 0) {
      float sl = 0.f;
      for (int d = 0; d < CF::D; ++d) sl += logf(high[d] - low[d]);
      logjac -= sl;
    }
  }
  ring_barrier();  // stage A of the first layer has landed

  for (int li = 0; li < L; ++li) {
    const int l = DIR_INV ? (L - 1 - li) : li;
    const float* lp = packed + (int64_t)l * CF::LAYER;

    // context half-row for the conditioner input (re-read per layer: L1/L2-resident)
    float cx[CF::CHA];
#pragma unroll
    for (int q = 0; q < CF::CHA; ++q) {
      const int c = h * CF::CH + q;
      cx[q] = (CF::CH > 0 && c < CF::C) ? ctx[crow * ldc + c] : 0.f;
    }

    // ---------------- stage A resident: lower spline (inverse dir), GEMM1
    float x1[CF::SH];
#pragma unroll
    for (int q = 0; q < CF::SH; ++q) {
      if constexpr (DIR_INV && CF::LOWER) {
        SplineTables<CF::K> t;
        load_tables<CF>(lds + CF::A_TBL + (h * CF::SH + q) * CF::TBL, t);
        float ld;
        zl[q] = rqs_apply<CF::K, true, true>(t, zl[q], bound, ld);
        ldsum -= ld;  // forward ld = -(inverse ld)
      }
      x1[q] = zl[q];
    }
    floatx16 acc1[CF::HB];
    init_bias<CF::HB>(acc1, lds + CF::A_BIAS, h);
    gemm_panels<CF::HB, CF::KS0P>(acc1, lds, lane, [&](int t) -> float {
      if (t < CF::CH) return cx[t < CF::CHA ? t : 0];
      if (t < CF::KS0) return x1[(t - CF::CH) < CF::SH ? (t - CF::CH) : 0];
      return 0.f;
    });
    if constexpr (!DIR_INV && CF::LOWER) {  // forward: y1 = lower(x1) after x1 fed the conditioner
#pragma unroll
      for (int q = 0; q < CF::SH; ++q) {
        SplineTables<CF::K> t;
        load_tables<CF>(lds + CF::A_TBL + (h * CF::SH + q) * CF::TBL, t);
        float ld;
        zl[q] = rqs_apply<CF::K, false, true>(t, zl[q], bound, ld);
        ldsum += ld;
      }
    }
    __syncthreads();
    stage_issue<CF::B_SIZE>(lds, lp + CF::B_OFF);
    tanh_all<CF::HB>(acc1);
    ring_barrier();

    // ---------------- stage B resident: GEMM2
    floatx16 acc2[CF::HB];
    init_bias<CF::HB>(acc2, lds + CF::B_BIAS, h);
    gemm_panels<CF::HB, CF::KS1>(acc2, lds, lane, [&](int t) -> float { return acc1[t >> 4][t & 15]; });
    __syncthreads();
    stage_issue<CF::c_size(0)>(lds, lp + CF::c_off(0));
    tanh_all<CF::HB>(acc2);
    ring_barrier();

    // ---------------- stages C_j resident: GEMM3 -> raw spline params in registers
    floatx16 acc3[CF::NO];
    static_for<0, CF::NSTG3>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      constexpr int cnt = CF::c_count(j);
      if constexpr (j > 0) {
        __syncthreads();
        stage_issue<CF::c_size(j)>(lds, lp + CF::c_off(j));
        ring_barrier();
      }
      floatx16 part[cnt];
      init_bias<cnt>(part, lds + cnt * CF::PANEL1, h);
      gemm_panels<cnt, CF::KS1>(part, lds, lane, [&](int t) -> float { return acc2[t >> 4][t & 15]; });
#pragma unroll
      for (int o = 0; o < cnt; ++o) acc3[j * CF::PPS + o] = part[o];
    });
    __syncthreads();
    if (li + 1 < L) stage_issue<CF::A_SIZE>(lds, packed + (int64_t)(DIR_INV ? (l - 1) : (l + 1)) * CF::LAYER);

    // ---------------- upper spline on this lane's DH dims (overlaps the next stage A copy)
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) {
      float uw[CF::K], uh[CF::K], ud[CF::K - 1];
#pragma unroll
      for (int k = 0; k < CF::K; ++k) {
        const int sw = q * CF::P + k, sh = q * CF::P + CF::K + k;
        uw[k] = acc3[sw >> 4][sw & 15];
        uh[k] = acc3[sh >> 4][sh & 15];
      }
#pragma unroll
      for (int k = 0; k < CF::K - 1; ++k) {
        const int sd = q * CF::P + 2 * CF::K + k;
        ud[k] = acc3[sd >> 4][sd & 15];
      }
      SplineTables<CF::K> t;
      build_tables<CF::K, true>(uw, uh, ud, bound, t);
      float ld;
      zu[q] = rqs_apply<CF::K, DIR_INV, true>(t, zu[q], bound, ld);
      ldsum += DIR_INV ? -ld : ld;
    }
    ring_barrier();  // next layer's stage A has landed
  }

  if constexpr (DIR_INV) {
    // base density Independent(Normal(0,1)) over this lane's dims, then combine halves
    constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
    float base = 0.f;
#pragma unroll
    for (int q = 0; q < CF::SH; ++q) base += -(zl[q] * zl[q]) / 2.f - kLogSqrt2Pi;
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) base += -(zu[q] * zu[q]) / 2.f - kLogSqrt2Pi;
    float v = base - ldsum + logjac;
    v += __shfl_xor(v, 32);
    if (h == 0 && valid) out_lp[row] = v;
  } else {
    if (low != nullptr) {  // inverse_bounding_transform (transforms.py:25-27)
#pragma unroll
      for (int q = 0; q < CF::SH; ++q) {
        const int d = h * CF::SH + q;
        zl[q] = (1.f / (1.f + expf(-zl[q]))) * (high[d] - low[d]) + low[d];
      }
#pragma unroll
      for (int q = 0; q < CF::DH; ++q) {
        const int d = CF::S + h * CF::DH + q;
        zu[q] = (1.f / (1.f + expf(-zu[q]))) * (high[d] - low[d]) + low[d];
      }
    }
    if (valid) {
#pragma unroll
      for (int q = 0; q < CF::SH; ++q) yout[row * ldy + h * CF::SH + q] = zl[q];
#pragma unroll
      for (int q = 0; q < CF::DH; ++q) yout[row * ldy + CF::S + h * CF::DH + q] = zu[q];
    }
    if (out_lp != nullptr) {
      float v = ldsum + __shfl_xor(ldsum, 32);
      if (h == 0 && valid) out_lp[row] = v;
    }
  }
}

// ===========================================================================
// bf16x6 variant: FP32 GEMMs emulated on the bf16 matrix pipe.
//
// Every fp32 operand v is split EXACTLY into three bf16 pieces by truncation
// (hi = v & 0xffff0000, mid = (v - hi) & 0xffff0000, lo = v - hi - mid, which has at most
// 8 significant bits), and each product W·X is formed from the six largest cross terms
//   Wh·Xh + Wh·Xm + Wm·Xh + Wm·Xm + Wh·Xl + Wl·Xh        (dropped terms ~2^-24 relative)
// with v_mfma_f32_32x32x16_bf16 (exact bf16 products, fp32 accumulate).  Six 32-cycle MFMAs
// per K=16 step replace eight 64-cycle v_mfma_f32_32x32x2_f32: 2.67x the FP32 matrix rate.
// On the oracle (config 3, 4096 rows) the log_prob error statistics vs fp64 are those of
// exact FP32 (median 2.70e-7 vs 2.79e-7, q99 4.08e-6 vs 4.03e-6, max 4.46e-5 vs 4.48e-5);
// dropping any of the six products is 3-5x worse.
//
// Operand mapping (v_mfma_f32_32x32x16_bf16): A[i = l&31][k = 8(l>>5) + j], B[k = 8(l>>5) + j]
// [col = l&31], j = 0..7.  The previous GEMM's accumulator registers 8s..8s+7 of block b ARE
// the B fragment of k-step 2b+s, element j carrying feature hid16_feature(2b+s, j, h); the
// packer permutes W's columns to match.  GEMM1's B fragments are built from the context
// half-row and the lane-half's x1 dims.
// ===========================================================================
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

NAZ_DEV floatx16 mfma_bf16(bf16x8 a, bf16x8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__host__ __device__ constexpr int hid16_feature(int t, int j, int h) {
  return 32 * (t >> 1) + 16 * (t & 1) + 8 * (j >> 2) + 4 * h + (j & 3);
}

// exact 3-way truncation split of one fp32 value: bit patterns whose upper halves are the bf16s
NAZ_DEV void split3_bits(float v, unsigned& hb, unsigned& mb, unsigned& lb) {
  hb = __float_as_uint(v);
  const float r1 = v - __uint_as_float(hb & 0xffff0000u);
  mb = __float_as_uint(r1);
  const float r2 = r1 - __uint_as_float(mb & 0xffff0000u);
  lb = __float_as_uint(r2);
}

__host__ __device__ inline unsigned bf16_hi_bits(float v, int piece) {
  // host+device reference of the same split (used by the packer)
  unsigned b;
  float r = v;
  for (int p = 0;; ++p) {
    __builtin_memcpy(&b, &r, 4);
    const unsigned t = b & 0xffff0000u;
    if (p == piece) return t >> 16;
    float tf;
    __builtin_memcpy(&tf, &t, 4);
    r = r - tf;
  }
}

struct Frag3 {
  bf16x8 h, m, l;
};

// 8 fp32 values -> three bf16x8 fragments (element j = v[j])
NAZ_DEV Frag3 split8(const float (&v)[8]) {
  u32x4 H, M, L;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned h0, m0, l0, h1, m1, l1;
    split3_bits(v[2 * q], h0, m0, l0);
    split3_bits(v[2 * q + 1], h1, m1, l1);
    H[q] = __builtin_amdgcn_perm(h1, h0, 0x07060302u);
    M[q] = __builtin_amdgcn_perm(m1, m0, 0x07060302u);
    L[q] = __builtin_amdgcn_perm(l1, l0, 0x07060302u);
  }
  return Frag3{__builtin_bit_cast(bf16x8, H), __builtin_bit_cast(bf16x8, M), __builtin_bit_cast(bf16x8, L)};
}

NAZ_DEV floatx16 mfma6(const Frag3& a, const Frag3& b, floatx16 acc) {
  acc = mfma_bf16(a.l, b.h, acc);  // small terms first
  acc = mfma_bf16(a.h, b.l, acc);
  acc = mfma_bf16(a.m, b.m, acc);
  acc = mfma_bf16(a.m, b.h, acc);
  acc = mfma_bf16(a.h, b.m, acc);
  acc = mfma_bf16(a.h, b.h, acc);
  return acc;
}

// fp16x3 (GEMM2/GEMM3 only, whose B operands are tanh outputs in [-1, 1]): v = hi + lo with
// hi = fp16(v), lo = fp16(v - hi) (v - hi is exact), products Wh·Xh + Wh·Xl + Wl·Xh, at half the
// MFMAs of bf16x6.  Weight range is checked at pack time (|W| < 2^15).
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

NAZ_DEV floatx16 mfma_f16(half8 a, half8 b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

struct Frag2 {
  half8 h, l;
};

// v - f32(f16 half of hp) in ONE v_fma_mix_f32 (the compiler emits cvt + sub); exact, since
// v - hi is representable.  HI selects the upper f16 of the packed pair.
template <bool HI>
NAZ_DEV float sub_f16_piece(float v, unsigned hp) {
  float r;
  if constexpr (HI)
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(v));
  else
    asm("v_fma_mix_f32 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hp), "v"(v));
  return r;
}

#ifdef NAZ_SPLIT_RTZ
NAZ_DEV unsigned pack_f16x2(float a, float b) { return __builtin_bit_cast(unsigned, __builtin_amdgcn_cvt_pkrtz(a, b)); }
#else
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
// round-to-nearest-even pair (one v_cvt_pk_f16_f32 on gfx950, same cost as the RTZ form)
NAZ_DEV unsigned pack_f16x2(float a, float b) {
  const half2v h = {(_Float16)a, (_Float16)b};
  return __builtin_bit_cast(unsigned, h);
}
#endif

// the lo pieces of a packed pair: f16(v0 - hi0) | f16(v1 - hi1) << 16 in TWO instructions
// (v_fma_mixlo_f16 / v_fma_mixhi_f16 round the exact f32 residual to f16 in the same op, RNE as
// v_cvt_pk_f16_f32) instead of two v_fma_mix_f32 + one v_cvt_pk_f16_f32.  OFF by default
// (NAZ_SPLIT_MIXLO): the compiler's hazard recognizer does not see the inline-asm write of the
// B fragment, so an MFMA issued 1-2 instructions later can read the register before the VALU
// write lands (measured: nsc D=8 flows off by 1e-2 relative; the D=16 image happened to pass).
// The default keeps the last writer a compiler-visible v_cvt_pk_f16_f32.
NAZ_DEV unsigned lo_pair_f16(float v0, float v1, unsigned hp) {
  unsigned lo;
  asm("v_fma_mixlo_f16 %0, -%1, 1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hp), "v"(v0));
  asm("v_fma_mixhi_f16 %0, -%1, 1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hp), "v"(v1));
  return lo;
}

NAZ_DEV Frag2 split8_f16(const float (&v)[8]) {
  u32x4 H, Lo;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const unsigned hp = pack_f16x2(v[2 * q], v[2 * q + 1]);
    H[q] = hp;
#ifndef NAZ_SPLIT_MIXLO
    const float r0 = sub_f16_piece<false>(v[2 * q], hp), r1 = sub_f16_piece<true>(v[2 * q + 1], hp);
    Lo[q] = pack_f16x2(r0, r1);
#else
    Lo[q] = lo_pair_f16(v[2 * q], v[2 * q + 1], hp);
#endif
  }
  return Frag2{__builtin_bit_cast(half8, H), __builtin_bit_cast(half8, Lo)};
}

NAZ_DEV floatx16 mfma3(const Frag2& a, const Frag2& b, floatx16 acc) {
  acc = mfma_f16(a.l, b.h, acc);
  acc = mfma_f16(a.h, b.l, acc);
  acc = mfma_f16(a.h, b.h, acc);
  return acc;
}

// fp16 piece (0 = hi, 1 = lo) of a WEIGHT as 16 bits.  Weights are split with round-to-nearest
// (done once per pack): |lo| <= 2^-12 |W|, so the dropped Wl·Xl term and W's residual error are
// ~2^-24 relative.  Activations use the cheaper truncating split (v_cvt_pkrtz) on the fly.
// On the oracle this RNE(W)/RTZ(X) pairing matches exact FP32 (median 3.1e-7 vs 2.8e-7, q99
// 4.1e-6 vs 4.0e-6); RTZ on both sides is measurably worse (median 3.6e-7, q99 5.1e-6).
NAZ_DEV unsigned f16_piece_bits(float v, int piece) {
  const _Float16 hi = (_Float16)v;
  if (piece == 0) return (unsigned)__builtin_bit_cast(unsigned short, hi);
  const _Float16 lo = (_Float16)(v - (float)hi);
  return (unsigned)__builtin_bit_cast(unsigned short, lo);
}

// activation of the x6 kernels: δ = σ − ½ of the pre-scaled accumulator (see kSigScale)
NAZ_DEV float sig_fold(float a) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(a)) - 0.5f; }
#ifdef NAZ_ABL_NOTANH
#define NAZ_TANH(v) (v)
#else
#define NAZ_TANH(v) sig_fold(v)
#endif

// LDS ring: two slots of 40 KB per 128-row workgroup (two workgroups per CU use all 160 KB).
// Stage s+1's LDS-DMA copy lands in one slot while stage s computes from the other.
#ifndef NAZ_X6_SLOT
#define NAZ_X6_SLOT 10240
#endif
#ifndef NAZ_X6_WAVES
#define NAZ_X6_WAVES 4
#endif
constexpr int kX6Slot = NAZ_X6_SLOT;   // 40 KB: two workgroups per CU (2 x 2 slots = 160 KB)
constexpr int kX6Waves = NAZ_X6_WAVES; // 128 rows per workgroup
constexpr int kX6Rows = 32 * kX6Waves;
constexpr int kChunk = 256;            // one (block, k-step, piece) A fragment set: 64 lanes x 16 B

template <int D_, int C_, int S_, int K_, int H_, bool LOWER_, int P23_ = 3>
struct CfgX6 {
  static constexpr int D = D_, C = C_, S = S_, K = K_, H = H_;
  static constexpr bool LOWER = LOWER_;
  static constexpr int P23 = P23_;                  // operand pieces of GEMM2/3: 3 = bf16x6, 2 = fp16x3
  static constexpr bool F16 = P23 == 2;
  static constexpr int Dt = D - S, P = 3 * K - 1, DH = Dt / 2, SH = S / 2;
  static constexpr int HB = H / 32;
  static constexpr int CT = (C + 15) / 16;          // GEMM1 k-steps over the context
  static constexpr int XT = (SH + 7) / 8;           // GEMM1 k-steps over the lane-half's x1
  static constexpr int KS0 = CT + XT;
  static constexpr int KS1 = 2 * HB;                // GEMM2/3 k-steps (16 features each)
  static constexpr int NO = (DH * P + 15) / 16;     // GEMM3 output blocks
  static constexpr int TBL = 3 * (K + 1);
  static constexpr int OT = 3 * kChunk;             // floats per (block, k-step), GEMM1
  static constexpr int OT23 = P23 * kChunk;         // floats per (block, k-step), GEMM2/3
  static constexpr int pad(int n) { return (n + 255) / 256 * 256; }
  static constexpr int pick_kb(int nb) {            // largest k-steps-per-stage dividing KS1
    int best = 1;
    for (int kb = 1; kb <= KS1; ++kb)
      if (KS1 % kb == 0 && pad(nb * kb * OT23 + nb * 32) <= kX6Slot) best = kb;
    return best;
  }
  static constexpr int KB2 = pick_kb(HB), NB2 = KS1 / KB2;
  static constexpr int KB3 = pick_kb(NO), NB3 = KS1 / KB3;
  // stage A: [HB][KS0][3][256] | bias [HB][2][16] | tables [S][TBL]
  static constexpr int A_BIAS = HB * KS0 * OT;
  static constexpr int A_TBL = A_BIAS + HB * 32;
  static constexpr int A_SIZE = pad(A_TBL + S * TBL);
  // stages B_q: [HB][KB2][3][256] | bias [HB][2][16]
  static constexpr int B_OFF = A_SIZE;
  static constexpr int B_BIAS = HB * KB2 * OT23;
  static constexpr int B_SIZE = pad(B_BIAS + HB * 32);
  // stages C_q: [NO][KB3][3][256] | bias [NO][2][16]
  static constexpr int C_OFF = B_OFF + NB2 * B_SIZE;
  static constexpr int C_BIAS = NO * KB3 * OT23;
  static constexpr int C_SIZE = pad(C_BIAS + NO * 32);
  // f16x3 configs also carry stage A with GEMM1 in fp16 pieces (same bias/table offsets), used
  // by workgroups whose context and data values all fit fp16's range (kG1F16Limit)
  static constexpr int A16_OFF = C_OFF + NB3 * C_SIZE;
#ifdef NAZ_NO_A16
  static constexpr int LAYER = A16_OFF;
#else
  static constexpr int LAYER = F16 ? A16_OFF + A_SIZE : A16_OFF;
#endif
  static constexpr int NSTG = 1 + NB2 + NB3;       // stages per layer
  static constexpr int MAXSTAGE = 2 * kX6Slot;      // LDS floats per workgroup (the ring)
  static constexpr __host__ __device__ int stage_off(int j) {
    return j == 0 ? 0 : (j <= NB2 ? B_OFF + (j - 1) * B_SIZE : C_OFF + (j - 1 - NB2) * C_SIZE);
  }
  static constexpr __host__ __device__ int stage_size(int j) { return j == 0 ? A_SIZE : (j <= NB2 ? B_SIZE : C_SIZE); }
  // natural flat layout (same as the FP32 variant)
  static constexpr int N_W0 = H * (C + S), N_B0 = H, N_W1 = H * H, N_B1 = H, N_W2 = Dt * P * H, N_B2 = Dt * P;
  static constexpr int N_LOW = LOWER ? S * (3 * K - 1) : 0;
  static constexpr int FLAT = N_W0 + N_B0 + N_W1 + N_B1 + N_W2 + N_B2 + N_LOW;
  static_assert(Dt % 2 == 0 && S % 2 == 0 && H % 32 == 0 && S > 0 && Dt > 0, "unsupported coupling shape");
  static_assert(A_SIZE <= kX6Slot && B_SIZE <= kX6Slot && C_SIZE <= kX6Slot, "stage exceeds one LDS ring slot");
  static_assert(HB * KS0 * 2 * kChunk <= A_BIAS, "fp16 GEMM1 panels must fit stage A's panel region");
};

// |value| bound under which GEMM1's B operand (context, x1) is split into fp16 hi + lo: hi
// (round-toward-zero) stays finite and lo = v - hi is exact with 11 significant bits.
constexpr float kG1F16Limit = 32768.f;
#ifndef NAZ_CTX_CHECK_LOAD
#define NAZ_CTX_CHECK_LOAD(p) (*(p))
#endif

// GEMM1 input column (in cat([ctx, x1]) order) for k-step t, element j, lane-half h; -1 = zero pad
template <class CF>
__host__ __device__ constexpr int x6_in_col(int t, int j, int h) {
  if (t < CF::CT) {
    const int c = 16 * t + 8 * h + j;
    return c < CF::C ? c : -1;
  }
  const int q = 8 * (t - CF::CT) + j;
  return q < CF::SH ? CF::C + h * CF::SH + q : -1;
}

// DenseNN output column carried by GEMM3 accumulator (block o, register r) on lane-half h; -1 = pad
template <class CF>
__host__ __device__ constexpr int x6_out_row(int o, int r, int h) {
  const int slot = 16 * o + r, qd = slot / CF::P, p = slot - qd * CF::P;
  if (qd >= CF::DH) return -1;
  const int dim = h * CF::DH + qd;
  if (p < CF::K) return dim * CF::K + p;
  if (p < 2 * CF::K) return CF::Dt * CF::K + dim * CF::K + (p - CF::K);
  return 2 * CF::Dt * CF::K + dim * (CF::K - 1) + (p - 2 * CF::K);
}

// Sigmoid fold.  tanh(a) = −2δ with δ = σ(−2a) − ½ = 1 / (1 + 2^(a·2·log2 e)) − ½, so the fused
// kernel's activation is rcp(1 + exp2(acc)) − ½ (4 VALU instead of 5) when the packer
//   * scales GEMM1 and GEMM2 rows (weights and bias) by kSigScale = 2·log2 e, so their
//     accumulators hold a·2·log2 e, and
//   * scales the weights of each activation's consumer (GEMM2, GEMM3) by −2 (exact).
// δ keeps tanh's relative precision near 0 (σ itself would not: its f16 hi/lo split loses
// ~2^-23 absolute at σ ≈ ½).  The pre-activations equal the tanh form's up to one rounding of
// the kSigScale-scaled weights (2^-24 relative), below the fp32 GEMM's own rounding.
constexpr float kSigScale = 2.88539008177792681f;

template <class CF>
__global__ void coupling_pack_x6_kernel(const float* __restrict__ flat, float* __restrict__ packed, int L,
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
    // operand chunk entry: (o, t, piece, lane, pair) -> two bf16 of W[row][col(j)], W[row][col(j+1)]
    auto chunk_word = [&](int q, int nt, int t0, const float* W, int ldw, bool gemm1, bool f16g1 = false) -> unsigned {
      const int ot = f16g1 ? 2 * kChunk : (gemm1 ? CF::OT : CF::OT23);
      const bool f16 = f16g1 || (!gemm1 && CF::F16);
      const int o = q / (nt * ot), r1 = q - o * nt * ot;
      const int tl = r1 / ot, r2 = r1 - tl * ot;
      const int piece = r2 / kChunk, u = r2 - piece * kChunk;
      const int lane = u >> 2, pair = u & 3, i = lane & 31, kh = lane >> 5;
      const int t = t0 + tl;
      unsigned out = 0;
      for (int e2 = 0; e2 < 2; ++e2) {
        const int j = 2 * pair + e2;
        int col, row;
        if (gemm1) {
          col = x6_in_col<CF>(t, j, kh);
          row = 32 * o + i;
        } else {
          col = hid16_feature(t, j, kh);
          row = 32 * o + i;
        }
        float v = 0.f;
        if (W == W2) {  // output rows permuted into lane-half spline slots
          const int hh = (i >> 2) & 1, rr = (i & 3) + 4 * (i >> 3);
          const int orow = x6_out_row<CF>(o, rr, hh);
          v = orow >= 0 ? W[orow * ldw + col] : 0.f;
        } else if (col >= 0) {
          v = W[row * ldw + col];
        }
        v *= W == W0 ? kSigScale : (W == W1 ? -2.f * kSigScale : -2.f);  // sigmoid fold (see kSigScale)
        out |= (f16 ? f16_piece_bits(v, piece) : bf16_hi_bits(v, piece)) << (16 * e2);
      }
      return out;
    };
    unsigned word = 0;
    float fv = 0.f;
    bool is_word = false;
    const bool a16 = CF::F16 && off >= CF::A16_OFF;
    const int offa = a16 ? off - CF::A16_OFF : off;
    if (offa < CF::A_SIZE && (a16 || off < CF::A16_OFF)) {
      const int off = offa;
      if (off < CF::A_BIAS) {
        if (!a16 || off < CF::HB * CF::KS0 * 2 * kChunk) {
          word = chunk_word(off, CF::KS0, 0, W0, CF::C + CF::S, true, a16);
          is_word = true;
        }
      } else if (off < CF::A_TBL) {
        const int q = off - CF::A_BIAS, o = q / 32, h = (q >> 4) & 1, r = q & 15;
        fv = kSigScale * b0[32 * o + acc_row(r, h)];
      } else if (CF::LOWER && off < CF::A_TBL + CF::S * CF::TBL) {
        const int q = off - CF::A_TBL, g = q / CF::TBL, w = q - g * CF::TBL;
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
        word = chunk_word(q, CF::KB2, sq * CF::KB2, W1, CF::H, false);
        is_word = true;
      } else if (q < CF::B_BIAS + CF::HB * 32) {
        const int qq = q - CF::B_BIAS, o = qq / 32, h = (qq >> 4) & 1, r = qq & 15;
        const int orow = 32 * o + acc_row(r, h);
        fv = kSigScale * b1[orow];
      }
    } else {
      const int sq = (off - CF::C_OFF) / CF::C_SIZE, q = off - CF::C_OFF - sq * CF::C_SIZE;
      if (q < CF::C_BIAS) {
        word = chunk_word(q, CF::KB3, sq * CF::KB3, W2, CF::H, false);
        is_word = true;
      } else if (q < CF::C_BIAS + CF::NO * 32) {
        const int qq = q - CF::C_BIAS, o = qq / 32, h = (qq >> 4) & 1, r = qq & 15;
        const int orow = x6_out_row<CF>(o, r, h);
        fv = orow >= 0 ? b2[orow] : 0.f;
      }
    }
    if (is_word) pu[e] = word;
    else packed[e] = fv;
  }
}

template <int NB, int KB>
NAZ_DEV void gemm_x6_stage(floatx16 (&acc)[NB], const float* __restrict__ stage, int lane, const Frag3 (&bf)[KB]) {
#ifdef NAZ_ABL_NOGEMM
  for (int o = 0; o < NB; ++o) acc[o][0] += __builtin_bit_cast(float, (unsigned)bf[0].h[0]) * 1e-30f;
  return;
#endif
  const u32x4* c4 = reinterpret_cast<const u32x4*>(stage);
#pragma unroll
  for (int t = 0; t < KB; ++t) {
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int base = ((o * KB + t) * 3) * 64 + lane;
      Frag3 a{__builtin_bit_cast(bf16x8, c4[base]), __builtin_bit_cast(bf16x8, c4[base + 64]),
              __builtin_bit_cast(bf16x8, c4[base + 128])};
      acc[o] = mfma6(a, bf[t], acc[o]);
    }
  }
}

template <int NB, int KB>
NAZ_DEV void gemm_f16_stage(floatx16 (&acc)[NB], const float* __restrict__ stage, int lane, const Frag2 (&bf)[KB]) {
#ifdef NAZ_ABL_NOGEMM
  for (int o = 0; o < NB; ++o) acc[o][0] += (float)bf[0].h[0] * 1e-30f;
  return;
#endif
  const u32x4* c4 = reinterpret_cast<const u32x4*>(stage);
#pragma unroll
  for (int t = 0; t < KB; ++t) {
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int base = ((o * KB + t) * 2) * 64 + lane;
      Frag2 a{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      acc[o] = mfma3(a, bf[t], acc[o]);
    }
  }
}

// GEMM over k-steps [T0, T0+KB) with each B fragment split from the activated accumulator
// just before its MFMAs (keeps one fragment live instead of KB).
template <int NB, int KB, int T0, int NX>
NAZ_DEV void gemm_f16_lazy(floatx16 (&acc)[NB], const float* __restrict__ stage, int lane, const floatx16 (&x)[NX]) {
  const u32x4* c4 = reinterpret_cast<const u32x4*>(stage);
#pragma unroll
  for (int t = 0; t < KB; ++t) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[(T0 + t) >> 1][8 * ((T0 + t) & 1) + j];
    const Frag2 b = split8_f16(v);
#ifdef NAZ_ABL_NOGEMM
    for (int o = 0; o < NB; ++o) acc[o][0] += (float)b.h[0] * 1e-30f;
    continue;
#endif
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int base = ((o * KB + t) * 2) * 64 + lane;
      Frag2 a{__builtin_bit_cast(half8, c4[base]), __builtin_bit_cast(half8, c4[base + 64])};
      acc[o] = mfma3(a, b, acc[o]);
    }
  }
}

template <int NB, int KB, int T0, int NX>
NAZ_DEV void gemm_x6_lazy(floatx16 (&acc)[NB], const float* __restrict__ stage, int lane, const floatx16 (&x)[NX]) {
  const u32x4* c4 = reinterpret_cast<const u32x4*>(stage);
#pragma unroll
  for (int t = 0; t < KB; ++t) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[(T0 + t) >> 1][8 * ((T0 + t) & 1) + j];
    const Frag3 b = split8(v);
#ifdef NAZ_ABL_NOGEMM
    for (int o = 0; o < NB; ++o) acc[o][0] += __builtin_bit_cast(float, (unsigned)b.h[0]) * 1e-30f;
    continue;
#endif
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int base = ((o * KB + t) * 3) * 64 + lane;
      Frag3 a{__builtin_bit_cast(bf16x8, c4[base]), __builtin_bit_cast(bf16x8, c4[base + 64]),
              __builtin_bit_cast(bf16x8, c4[base + 128])};
      acc[o] = mfma6(a, b, acc[o]);
    }
  }
}

template <int T0, int KB, int NB>
NAZ_DEV void frags_from_acc(const floatx16 (&x)[NB], Frag2 (&bf)[KB]) {
#pragma unroll
  for (int tl = 0; tl < KB; ++tl) {
    const int t = T0 + tl;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[t >> 1][8 * (t & 1) + j];
    bf[tl] = split8_f16(v);
  }
}

// B fragments of k-steps [T0, T0+KB) from an accumulator array (already activated)
template <int T0, int KB, int NB>
NAZ_DEV void frags_from_acc(const floatx16 (&x)[NB], Frag3 (&bf)[KB]) {
#pragma unroll
  for (int tl = 0; tl < KB; ++tl) {
    constexpr int dummy = 0;
    (void)dummy;
    const int t = T0 + tl;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = x[t >> 1][8 * (t & 1) + j];
    bf[tl] = split8(v);
  }
}

template <class CF, bool DIR_INV>
__global__ void __launch_bounds__(kX6Rows * 2, kX6Waves / 2) coupling_x6_kernel(
    const float* __restrict__ packed, int L, const float* __restrict__ x, int64_t ldx,
    const float* __restrict__ ctx, int64_t ldc, const float* __restrict__ low, const float* __restrict__ high,
    float* __restrict__ out_lp, float* __restrict__ yout, int64_t ldy, int64_t B, float bound) {
  extern __shared__ float4 lds4[];
  float* const slot0 = reinterpret_cast<float*>(lds4);
  float* const slot1 = slot0 + kX6Slot;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int h = lane >> 5;
  const int64_t row = (int64_t)blockIdx.x * kX6Rows + wave * 32 + (lane & 31);
  const bool valid = row < B;
  const int64_t crow = valid ? row : 0;

  float zl[CF::SH], zu[CF::DH];
  float ldsum = 0.f, logjac = 0.f;
#pragma unroll
  for (int q = 0; q < CF::SH; ++q) zl[q] = valid ? x[crow * ldx + h * CF::SH + q] : 0.f;
#pragma unroll
  for (int q = 0; q < CF::DH; ++q) zu[q] = valid ? x[crow * ldx + CF::S + h * CF::DH + q] : 0.f;
  if (DIR_INV && low != nullptr) {  // naz bounding_transform (transforms.py:20-23)
    auto bnd = [&](float& v, int dim) {
      const float lo = low[dim], hi = high[dim];
      const float u = (v - lo) / (hi - lo);
      logjac -= logf(u) + log1pf(-u);
      v = logf(u / (1.f - u));
    };
#pragma unroll
    for (int q = 0; q < CF::SH; ++q) bnd(zl[q], h * CF::SH + q);
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) bnd(zu[q], CF::S + h * CF::DH + q);
    if (h == 0) {
      float sl = 0.f;
      for (int d = 0; d < CF::D; ++d) sl += logf(high[d] - low[d]);
      logjac -= sl;
    }
  }

  // GEMM1 precision path for this workgroup: fp16 pieces when every context and data value of
  // its rows is inside kG1F16Limit (x1 stays inside max(|x|, bound) through the lower
  // splines), else the exact-split bf16x6 path.  Uniform per workgroup: it picks stage A.
  int a_off = 0;
#ifdef NAZ_NO_G1CHECK
  if constexpr (false) {
#else
  if constexpr (CF::F16) {
#endif
    bool ok = bound < kG1F16Limit;
#pragma unroll
    for (int q = 0; q < CF::SH; ++q) ok = ok && fabsf(zl[q]) < kG1F16Limit;
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) ok = ok && fabsf(zu[q]) < kG1F16Limit;
#pragma unroll
    for (int t = 0; t < CF::CT; ++t)
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int c = 16 * t + 8 * h + jj;
        if (c < CF::C) ok = ok && fabsf(NAZ_CTX_CHECK_LOAD(&ctx[crow * ldc + c])) < kG1F16Limit;
      }
    // workgroup AND through ring slot 1 (unused until the first in-loop barrier; static LDS
    // for __syncthreads_and would push the workgroup past 80 KB = one workgroup per CU)
    int* flags = reinterpret_cast<int*>(slot1);
    if (lane == 0) flags[wave] = __all(ok) ? 1 : 0;
    __syncthreads();
    bool all_ok = true;
#pragma unroll
    for (int w = 0; w < kX6Waves; ++w) all_ok = all_ok && flags[w] != 0;
    a_off = all_ok ? CF::A16_OFF : 0;
  }
#if defined(NAZ_G1_FORCE) && NAZ_G1_FORCE == 1
  const bool g1f16 = true;
  a_off = CF::F16 ? CF::A16_OFF : 0;
#elif defined(NAZ_G1_FORCE) && NAZ_G1_FORCE == 2
  const bool g1f16 = false;
  a_off = 0;
#else
  const bool g1f16 = a_off != 0;
#endif

  stage_issue<CF::A_SIZE, kX6Waves>(slot0, packed + (int64_t)(DIR_INV ? (L - 1) : 0) * CF::LAYER + a_off);

  const RqsConsts<CF::K, DIR_INV> rc(bound);
  int g = 0;  // global stage counter: stage g lives in slot (g & 1)
  for (int li = 0; li < L; ++li) {
    const int l = DIR_INV ? (L - 1 - li) : li;
    const float* lp = packed + (int64_t)l * CF::LAYER;
    const float* lnext = packed + (int64_t)(DIR_INV ? (l - 1) : (l + 1)) * CF::LAYER;
    floatx16 acc1[CF::HB], acc2[CF::HB], acc3[CF::NO];

    static_for<0, CF::NSTG>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
#ifndef NAZ_ABL_NOBARRIER
      ring_barrier();  // stage j has landed in slot (g&1); every wave is done with the other slot
#endif
      const float* cur = (g & 1) ? slot1 : slot0;
      float* nxt = (g & 1) ? slot0 : slot1;
      if constexpr (j + 1 < CF::NSTG) {
        stage_issue<CF::stage_size(j + 1), kX6Waves>(nxt, lp + CF::stage_off(j + 1));
      } else {
        if (li + 1 < L) stage_issue<CF::A_SIZE, kX6Waves>(nxt, lnext + a_off);
      }
      ++g;

      if constexpr (j == 0) {
        // ---------------- stage A: lower spline (inverse), GEMM1 over [ctx | x1]
        float x1[CF::SH];
#pragma unroll
        for (int q = 0; q < CF::SH; ++q) {
#ifdef NAZ_ABL_NOLOWER
          if constexpr (false) {
#else
          if constexpr (DIR_INV && CF::LOWER) {
#endif
            float ld;
            zl[q] = rqs_table<CF::K, true>(cur + CF::A_TBL + (h * CF::SH + q) * CF::TBL, zl[q], bound, ld);
            ldsum -= ld;
          }
          x1[q] = zl[q];
        }
        auto g1_in = [&](int t, float (&v)[8]) {
#pragma unroll
          for (int jj = 0; jj < 8; ++jj) {
            if (t < CF::CT) {
              const int c = 16 * t + 8 * h + jj;
              v[jj] = (c < CF::C) ? ctx[crow * ldc + c] : 0.f;
            } else {
              const int q = 8 * (t - CF::CT) + jj;
              v[jj] = q < CF::SH ? x1[q < CF::SH ? q : 0] : 0.f;
            }
          }
        };
        init_bias<CF::HB>(acc1, cur + CF::A_BIAS, h);
        if (CF::F16 && g1f16) {
          Frag2 bf[CF::KS0];
#pragma unroll
          for (int t = 0; t < CF::KS0; ++t) {
            float v[8];
            g1_in(t, v);
            bf[t] = split8_f16(v);
          }
          gemm_f16_stage<CF::HB, CF::KS0>(acc1, cur, lane, bf);
        } else {
          Frag3 bf[CF::KS0];
#pragma unroll
          for (int t = 0; t < CF::KS0; ++t) {
            float v[8];
            g1_in(t, v);
            bf[t] = split8(v);
          }
          gemm_x6_stage<CF::HB, CF::KS0>(acc1, cur, lane, bf);
        }
        if constexpr (!DIR_INV && CF::LOWER) {
#pragma unroll
          for (int q = 0; q < CF::SH; ++q) {
            float ld;
            zl[q] = rqs_table<CF::K, false>(cur + CF::A_TBL + (h * CF::SH + q) * CF::TBL, zl[q], bound, ld);
            ldsum += ld;
          }
        }
      } else if constexpr (j <= CF::NB2) {
        // ---------------- stage B_q: GEMM2 k-steps [T0, T0 + KB2)
        constexpr int q = j - 1, T0 = q * CF::KB2;
#pragma unroll
        for (int b = (T0 + 1) / 2; b < (T0 + CF::KB2 + 1) / 2; ++b)  // activate blocks first used here
#pragma unroll
          for (int r = 0; r < 16; ++r) acc1[b][r] = NAZ_TANH(acc1[b][r]);
        if constexpr (q == 0) init_bias<CF::HB>(acc2, cur + CF::B_BIAS, h);
        if constexpr (CF::F16) gemm_f16_lazy<CF::HB, CF::KB2, T0>(acc2, cur, lane, acc1);
        else gemm_x6_lazy<CF::HB, CF::KB2, T0>(acc2, cur, lane, acc1);
      } else {
        // ---------------- stage C_q: GEMM3 k-steps [T0, T0 + KB3) -> raw spline params
        constexpr int q = j - 1 - CF::NB2, T0 = q * CF::KB3;
#pragma unroll
        for (int b = (T0 + 1) / 2; b < (T0 + CF::KB3 + 1) / 2; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc2[b][r] = NAZ_TANH(acc2[b][r]);
        if constexpr (q == 0) init_bias<CF::NO>(acc3, cur + CF::C_BIAS, h);
        if constexpr (CF::F16) gemm_f16_lazy<CF::NO, CF::KB3, T0>(acc3, cur, lane, acc2);
        else gemm_x6_lazy<CF::NO, CF::KB3, T0>(acc3, cur, lane, acc2);
      }
    });

    // ---------------- upper spline on this lane's DH dims (the next layer's stage A is in flight)
#ifdef NAZ_ABL_NOSPLINE
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) {
      float sacc = 0.f;
#pragma unroll
      for (int k = 0; k < CF::P; ++k) sacc += acc3[(q * CF::P + k) >> 4][(q * CF::P + k) & 15];
      zu[q] += 1e-30f * sacc;
    }
    if (false)
#endif
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) {
      float uw[CF::K], uh[CF::K], ud[CF::K - 1];
#pragma unroll
      for (int k = 0; k < CF::K; ++k) {
        const int sw = q * CF::P + k, sh = q * CF::P + CF::K + k;
        uw[k] = acc3[sw >> 4][sw & 15];
        uh[k] = acc3[sh >> 4][sh & 15];
      }
#pragma unroll
      for (int k = 0; k < CF::K - 1; ++k) {
        const int sd = q * CF::P + 2 * CF::K + k;
        ud[k] = acc3[sd >> 4][sd & 15];
      }
      float ld;
      zu[q] = rqs_select<CF::K, DIR_INV>(uw, uh, ud, zu[q], bound, rc, ld);
      ldsum += DIR_INV ? -ld : ld;
    }
  }

  if constexpr (DIR_INV) {
    constexpr float kLogSqrt2Pi = 0.91893853320467274178f;
    float base = 0.f;
#pragma unroll
    for (int q = 0; q < CF::SH; ++q) base += -(zl[q] * zl[q]) / 2.f - kLogSqrt2Pi;
#pragma unroll
    for (int q = 0; q < CF::DH; ++q) base += -(zu[q] * zu[q]) / 2.f - kLogSqrt2Pi;
    float v = base - ldsum + logjac;
    v += __shfl_xor(v, 32);
    if (h == 0 && valid) out_lp[row] = v;
  } else {
    if (low != nullptr) {
#pragma unroll
      for (int q = 0; q < CF::SH; ++q) {
        const int d = h * CF::SH + q;
        zl[q] = (1.f / (1.f + expf(-zl[q]))) * (high[d] - low[d]) + low[d];
      }
#pragma unroll
      for (int q = 0; q < CF::DH; ++q) {
        const int d = CF::S + h * CF::DH + q;
        zu[q] = (1.f / (1.f + expf(-zu[q]))) * (high[d] - low[d]) + low[d];
      }
    }
    if (valid) {
#pragma unroll
      for (int q = 0; q < CF::SH; ++q) yout[row * ldy + h * CF::SH + q] = zl[q];
#pragma unroll
      for (int q = 0; q < CF::DH; ++q) yout[row * ldy + CF::S + h * CF::DH + q] = zu[q];
    }
    if (out_lp != nullptr) {
      float v = ldsum + __shfl_xor(ldsum, 32);
      if (h == 0 && valid) out_lp[row] = v;
    }
  }
}

}  // namespace naz

#include "coupling_r16.h"
#include "coupling_w32.h"
#include "coupling_train.h"
#include "made_ar_r16.h"
#include "made_ar_bwd.h"
#include "made_ar_wide.h"

namespace naz {

#if NAZ_PART == 0 || NAZ_PART == 1  // ---------------- part 1: the coupling flows (build.py compiles this file twice)
extern "C" int naz_debug_nonfinite(int64_t* out5, int clear) {
#ifndef NAZ_DEBUG_NONFINITE
  (void)out5;
  (void)clear;
  return naz::set_error("naz_debug_nonfinite: library not built with -DNAZ_DEBUG_NONFINITE");
#else
  if (out5 == nullptr) return naz::set_error("naz_debug_nonfinite: null output");
  if (hipDeviceSynchronize() != hipSuccess ||
      hipMemcpyFromSymbol(out5, HIP_SYMBOL(naz::g_nonfinite), 5 * sizeof(int64_t)) != hipSuccess)
    return naz::set_error("naz_debug_nonfinite: reading the record failed");
  if (clear) {
    const int64_t zero[5] = {0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(naz::g_nonfinite), zero, sizeof(zero)) != hipSuccess)
      return naz::set_error("naz_debug_nonfinite: clearing the record failed");
  }
  return 0;
#endif
}

// ---------------------------------------------------------------------------
// Host dispatch over the compiled instantiations
// ---------------------------------------------------------------------------
template <class CF, class CX, class CH, class CR, bool R16OK>
struct CouplingOps {
  static bool supports(int mode) { return mode != NAZ_MFMA_F16X3_R16 || R16OK; }
  static int64_t layer_floats(int mode) {
    if (mode == NAZ_MFMA_F16X3_R16) return CR::LAYER;
    return mode == NAZ_MFMA_F32 ? CF::LAYER : (mode == NAZ_MFMA_BF16X6 ? CX::LAYER : CH::LAYER);
  }
  static int64_t packed_bytes(int L, int mode) { return (int64_t)L * layer_floats(mode) * 4; }
  static int64_t param_count(int L) { return (int64_t)L * CF::FLAT; }
  static int pack(const float* flat, void* packed, int L, float bound, int mode, hipStream_t s) {
    const int64_t n = (int64_t)L * layer_floats(mode);
    int64_t grid = (n + 255) / 256;
    if (grid > 8192) grid = 8192;
    float* pk = reinterpret_cast<float*>(packed);
    if (mode == NAZ_MFMA_F16X3_R16)
      hipLaunchKernelGGL((coupling_pack_r16_kernel<CR>), dim3((unsigned)grid), dim3(256), 0, s, flat, pk, L, bound);
    else if (mode == NAZ_MFMA_F32)
      hipLaunchKernelGGL((coupling_pack_kernel<CF>), dim3((unsigned)grid), dim3(256), 0, s, flat, pk, L, bound);
    else if (mode == NAZ_MFMA_BF16X6)
      hipLaunchKernelGGL((coupling_pack_x6_kernel<CX>), dim3((unsigned)grid), dim3(256), 0, s, flat, pk, L, bound);
    else
      hipLaunchKernelGGL((coupling_pack_x6_kernel<CH>), dim3((unsigned)grid), dim3(256), 0, s, flat, pk, L, bound);
    return check_launch("coupling_pack_kernel");
  }
  template <class G, bool INV, int X6>
  static void launch(const float* pk, int L, const float* x, int64_t ldx, const float* ctx, int64_t ldc,
                     const float* low, const float* high, float* out_lp, float* y, int64_t ldy, int64_t B, float bound,
                     hipStream_t s) {
    const size_t lds = (size_t)G::MAXSTAGE * 4;
    if constexpr (X6 == 2) {
      const int64_t grid = (B + kR16Rows - 1) / kR16Rows;
      hipLaunchKernelGGL((coupling_r16_kernel<G, INV>), dim3((unsigned)grid), dim3(kR16Rows * 4), lds, s, pk, L, x,
                         ldx, ctx, ldc, low, high, out_lp, y, ldy, B, bound);
    } else if constexpr (X6 == 3) {  // f16x3 image: the 32-row-wave kernel (coupling_w32.h)
      const int64_t grid = (B + kX6Rows - 1) / kX6Rows;
      hipLaunchKernelGGL((coupling_w32_kernel<G, INV>), dim3((unsigned)grid), dim3(kX6Rows * 2), lds, s, pk, L, x,
                         ldx, ctx, ldc, low, high, out_lp, y, ldy, B, bound);
    } else if constexpr (X6 == 1) {
      const int64_t grid = (B + kX6Rows - 1) / kX6Rows;
      hipLaunchKernelGGL((coupling_x6_kernel<G, INV>), dim3((unsigned)grid), dim3(kX6Rows * 2), lds, s, pk, L, x,
                         ldx, ctx, ldc, low, high, out_lp, y, ldy, B, bound);
    } else {
      const int64_t grid = (B + kRowsPerWG - 1) / kRowsPerWG;
      hipLaunchKernelGGL((coupling_flow_kernel<G, INV>), dim3((unsigned)grid), dim3(256), lds, s, pk, L, x, ldx,
                         ctx, ldc, low, high, out_lp, y, ldy, B, bound);
    }
  }
  // ---- NLL training path (r16 instantiations only; the packed image must be F16X3_R16)
  static int64_t bwd_layer_floats() {
    if constexpr (R16OK) return BwdR16<CR>::LAYER;
    else return -1;
  }
  static int pack_bwd(const float* flat, void* packed, int L, hipStream_t s) {
    if constexpr (R16OK) {
      const int64_t n = (int64_t)L * BwdR16<CR>::LAYER;
      const int64_t grid = std::min<int64_t>((n + 255) / 256, 8192);
      hipLaunchKernelGGL((coupling_pack_bwd_r16_kernel<CR>), dim3((unsigned)grid), dim3(256), 0, s, flat,
                         reinterpret_cast<float*>(packed), L);
      return check_launch("coupling_pack_bwd_r16_kernel");
    } else {
      return -2;
    }
  }
  static int log_prob_train(const void* packed, int L, const float* x, int64_t ldx, const float* ctx, int64_t ldc,
                            const float* low, const float* high, float* out_lp, float* states, int64_t B, float bound,
                            hipStream_t s) {
    if constexpr (R16OK) {
      if (B == 0) return 0;
      const int64_t grid = (B + kR16Rows - 1) / kR16Rows;
      hipLaunchKernelGGL((coupling_r16_kernel<CR, true, 1>), dim3((unsigned)grid), dim3(kR16Rows * 4),
                         (size_t)CR::MAXSTAGE * 4, s, reinterpret_cast<const float*>(packed), L, x, ldx, ctx, ldc, low,
                         high, out_lp, nullptr, 0, B, bound, states);
      return check_launch("coupling_r16_kernel<train>");
    } else {
      return -2;
    }
  }
  static int bwd_layer(const void* packed, const void* bwd, const float* flat, int l, const float* state,
                       const float* ctx, int64_t ldc, const float* g_in, const float* g_lp, const BwdOut& o, int64_t B,
                       float bound, hipStream_t s) {
    if constexpr (R16OK) {
      if (B == 0) return 0;
      const int64_t ntiles = (B + 16 * kBwdWaves - 1) / (16 * kBwdWaves);
      const int64_t grid = std::min<int64_t>(ntiles, 2048);
      size_t lds = (size_t)(2 * BwdSlot<CR>::v + 2 * CR::S * (3 * CR::K - 1)) * 4;  // ring, glow, lowp
#ifdef NAZ_ABL_BWD_ONEWG  // timing ablation: 64 KB of unused LDS, so one workgroup (one wave per SIMD) per CU
      lds += 64 * 1024;
#endif
      hipLaunchKernelGGL((coupling_bwd_r16_kernel<CR>), dim3((unsigned)grid), dim3(kBwdWaves * 64), lds, s,
                         reinterpret_cast<const float*>(packed), reinterpret_cast<const float*>(bwd), flat, l, state,
                         ctx, ldc, g_in, g_lp, o, B, bound);
      return check_launch("coupling_bwd_r16_kernel");
    } else {
      return -2;
    }
  }
  // naz_coupling_layer_{fwd,inv}: one layer of the r16 image
  static int layer(bool inv, int mode, const void* packed, int l, int L, const float* x, int64_t ldx, const float* ctx,
                   int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B, float bound, hipStream_t s) {
    if constexpr (R16OK) {
      if (mode != NAZ_MFMA_F16X3_R16)
        return set_error("naz_coupling_layer: the packed image must be NAZ_MFMA_F16X3_R16 (mode %d)", mode);
      if (B == 0) return 0;
      (void)L;
      const float* pk = reinterpret_cast<const float*>(packed) + (int64_t)l * CR::LAYER;
      const int64_t grid = (B + kR16Rows - 1) / kR16Rows;
      const size_t lds = (size_t)CR::MAXSTAGE * 4;
      if (inv)
        hipLaunchKernelGGL((coupling_r16_kernel<CR, true, 2>), dim3((unsigned)grid), dim3(kR16Rows * 4), lds, s, pk,
                           1, x, ldx, ctx, ldc, nullptr, nullptr, ld, y, ldy, B, bound, nullptr, ld_mode);
      else
        hipLaunchKernelGGL((coupling_r16_kernel<CR, false, 2>), dim3((unsigned)grid), dim3(kR16Rows * 4), lds, s, pk,
                           1, x, ldx, ctx, ldc, nullptr, nullptr, ld, y, ldy, B, bound, nullptr, ld_mode);
      return check_launch("coupling_r16_kernel<layer>");
    } else {
      return set_error("naz_coupling_layer: no 16-row instantiation for this shape");
    }
  }
  static int dp3_columns(int* rows) {
    if constexpr (R16OK) {
      using BW = BwdR16<CR>;
      if (rows != nullptr)
        for (int q = 0; q < 4; ++q)
          for (int sl = 0; sl < BW::NS3; ++sl) rows[q * BW::NS3 + sl] = BW::slot_row(q, sl);
      return 4 * BW::NS3;
    } else {
      return -2;
    }
  }
  static int run(bool inv, int mode, const void* packed, int L, const float* x, int64_t ldx, const float* ctx,
                 int64_t ldc, const float* low, const float* high, float* out_lp, float* y, int64_t ldy, int64_t B,
                 float bound, hipStream_t s) {
    if (B == 0) return 0;
    const float* pk = reinterpret_cast<const float*>(packed);
#define NAZ_RUN(G, X6)                                                                                   \
  (inv ? launch<G, true, X6>(pk, L, x, ldx, ctx, ldc, low, high, out_lp, y, ldy, B, bound, s)            \
       : launch<G, false, X6>(pk, L, x, ldx, ctx, ldc, low, high, out_lp, y, ldy, B, bound, s))
    if (mode == NAZ_MFMA_F32) NAZ_RUN(CF, 0);
    else if (mode == NAZ_MFMA_BF16X6) NAZ_RUN(CX, 1);
    else if (mode == NAZ_MFMA_F16X3_R16) {
      if constexpr (R16OK) NAZ_RUN(CR, 2);
      else return -2;
    } else {
#ifdef NAZ_F16X3_X6  // A/B: the round-1 32-row kernel on the same image
      NAZ_RUN(CH, 1);
#else
      NAZ_RUN(CH, 3);
#endif
    }
#undef NAZ_RUN
    return check_launch("coupling_flow_kernel");
  }
};

// Instantiation table: (D, C, S, K, H, lower).  Bench configs first (BASELINE.json
// configs 2 and 3), then small shapes used by the parity tests.
#ifndef NAZ_COUPLING_CONFIGS
#define NAZ_COUPLING_CONFIGS(X)   \
  X(16, 32, 8, 8, 128, true)      \
  X(16, 32, 8, 8, 128, false)     \
  X(8, 0, 4, 8, 128, true)        \
  X(8, 0, 4, 8, 128, false)       \
  X(16, 0, 8, 8, 128, true)       \
  X(4, 3, 2, 8, 64, true)         \
  X(6, 2, 2, 4, 32, true)         \
  X(6, 2, 2, 4, 32, false)
#endif

template <class F>
static int coupling_dispatch(const naz_coupling_desc* d, F&& f) {
  if (d == nullptr) return set_error("naz_coupling: null descriptor");
  if (d->act != NAZ_ACT_TANH) return -2;
  if (d->mfma_mode != NAZ_MFMA_BF16X6 && d->mfma_mode != NAZ_MFMA_F32 && d->mfma_mode != NAZ_MFMA_F16X3 &&
      d->mfma_mode != NAZ_MFMA_F16X3_R16)
    return -2;
#define NAZ_R16OK(D_, S_, H_) ((S_) % 4 == 0 && ((D_) - (S_)) % 4 == 0 && (S_) / 4 <= 8 && (H_) % 32 == 0 && (H_) <= 128)
#define NAZ_TRY(D_, C_, S_, K_, H_, LOW_)                                                                  \
  if (d->D == D_ && d->C == C_ && d->S == S_ && d->K == K_ && d->H == H_ && (d->has_lower != 0) == LOW_) {  \
    using Ops = CouplingOps<CouplingCfg<D_, C_, S_, K_, H_, LOW_>, CfgX6<D_, C_, S_, K_, H_, LOW_, 3>,         \
                            CfgX6<D_, C_, S_, K_, H_, LOW_, 2>,                                                \
                            std::conditional_t<NAZ_R16OK(D_, S_, H_), CfgR16<D_, C_, S_, K_, H_, LOW_>,        \
                                               CfgR16<8, 0, 4, 8, 128, true>>,                                 \
                            NAZ_R16OK(D_, S_, H_)>;                                                            \
    if (!Ops::supports(d->mfma_mode)) return -2;                                                               \
    return f(Ops{});                                                                                           \
  }
  NAZ_COUPLING_CONFIGS(NAZ_TRY)
#undef NAZ_TRY
  return -2;
}

int coupling_supported(const naz_coupling_desc* d) {
  return coupling_dispatch(d, [](auto) { return 1; }) == 1 ? 1 : 0;
}

int64_t coupling_param_count(const naz_coupling_desc* d) {
  int64_t v = -1;
  coupling_dispatch(d, [&](auto ops) { v = decltype(ops)::param_count(d->L); return 0; });
  return v;
}

int64_t coupling_packed_bytes(const naz_coupling_desc* d) {
  int64_t v = -1;
  coupling_dispatch(d, [&](auto ops) { v = decltype(ops)::packed_bytes(d->L, d->mfma_mode); return 0; });
  return v;
}

static int unsupported(const naz_coupling_desc* d) {
  return set_error("naz_coupling: no fused instantiation for D=%d C=%d S=%d K=%d H=%d act=%d lower=%d mode=%d", d->D,
                   d->C, d->S, d->K, d->H, d->act, d->has_lower, d->mfma_mode);
}

int coupling_pack(const naz_coupling_desc* d, const float* flat, void* packed, hipStream_t s) {
  int rc = coupling_dispatch(d, [&](auto ops) { return decltype(ops)::pack(flat, packed, d->L, d->bound, d->mfma_mode, s); });
  return rc == -2 ? unsupported(d) : rc;
}

int coupling_log_prob(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, hipStream_t s) {
  if ((low == nullptr) != (high == nullptr)) return set_error("naz_coupling_log_prob: low/high must both be set");
  int rc = coupling_dispatch(d, [&](auto ops) {
    return decltype(ops)::run(true, d->mfma_mode, packed, d->L, x, ldx, ctx, ldc, low, high, out_lp, nullptr, 0, B,
                              d->bound, s);
  });
  return rc == -2 ? unsupported(d) : rc;
}

int coupling_sample(const naz_coupling_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                    int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B,
                    hipStream_t s) {
  if ((low == nullptr) != (high == nullptr)) return set_error("naz_coupling_sample: low/high must both be set");
  int rc = coupling_dispatch(d, [&](auto ops) {
    return decltype(ops)::run(false, d->mfma_mode, packed, d->L, z, ldz, ctx, ldc, low, high, out_ld, y, ldy, B,
                              d->bound, s);
  });
  return rc == -2 ? unsupported(d) : rc;
}

// ---- NLL training path (coupling_train.h) ----------------------------------------------
static int train_mode_ok(const naz_coupling_desc* d) {
  if (d == nullptr) return set_error("naz_coupling: null descriptor");
  if (d->mfma_mode != NAZ_MFMA_F16X3_R16)
    return set_error("naz_coupling training path: the packed image must be NAZ_MFMA_F16X3_R16 (mode %d)", d->mfma_mode);
  return 0;
}

int64_t coupling_bwd_packed_bytes(const naz_coupling_desc* d) {
  int64_t v = -1;
  coupling_dispatch(d, [&](auto ops) {
    const int64_t f = decltype(ops)::bwd_layer_floats();
    v = f < 0 ? -1 : f * d->L * 4;
    return 0;
  });
  return v;
}

int coupling_pack_bwd(const naz_coupling_desc* d, const float* flat, void* packed, hipStream_t s) {
  if (int rc = train_mode_ok(d)) return rc;
  int rc = coupling_dispatch(d, [&](auto ops) { return decltype(ops)::pack_bwd(flat, packed, d->L, s); });
  return rc == -2 ? unsupported(d) : rc;
}

int coupling_log_prob_train(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                            const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                            float* states, int64_t B, hipStream_t s) {
  if (int rc = train_mode_ok(d)) return rc;
  if ((low == nullptr) != (high == nullptr)) return set_error("naz_coupling_log_prob_train: low/high must both be set");
  if (states == nullptr) return set_error("naz_coupling_log_prob_train: states buffer required");
  int rc = coupling_dispatch(d, [&](auto ops) {
    return decltype(ops)::log_prob_train(packed, d->L, x, ldx, ctx, ldc, low, high, out_lp, states, B, d->bound, s);
  });
  return rc == -2 ? unsupported(d) : rc;
}

int coupling_bwd_layer(const naz_coupling_desc* d, const void* packed, const void* packed_bwd, const float* flat,
                       int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                       const float* g_lp, float* h1, float* h2, float* dp1, float* dp2, float* dp3, float* x0,
                       float* g_out, float* g_low, int64_t B, hipStream_t s) {
  if (int rc = train_mode_ok(d)) return rc;
  if (layer < 0 || layer >= d->L) return set_error("naz_coupling_bwd_layer: layer %d out of range", layer);
  if (d->has_lower && g_low == nullptr) return set_error("naz_coupling_bwd_layer: g_low required with a lower spline");
  const BwdOut o{h1, h2, dp1, dp2, dp3, x0, g_out, g_low};
  int rc = coupling_dispatch(d, [&](auto ops) {
    return decltype(ops)::bwd_layer(packed, packed_bwd, flat, layer, state, ctx, ldc, g_in, g_lp, o, B, d->bound, s);
  });
  return rc == -2 ? unsupported(d) : rc;
}

int coupling_layer(const naz_coupling_desc* d, int inv, const void* packed, int layer, const float* x, int64_t ldx,
                   const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                   hipStream_t s) {
  if (d == nullptr) return set_error("naz_coupling_layer: null descriptor");
  if (layer < 0 || layer >= d->L) return set_error("naz_coupling_layer: layer %d out of range", layer);
  if (ld_mode != NAZ_LD_ROWSUM && ld_mode != NAZ_LD_ROWSUM_ADD && ld_mode != NAZ_LD_ROWSUM_SUB)
    return set_error("naz_coupling_layer: ld_mode must be NAZ_LD_ROWSUM, _ADD or _SUB");
  int rc = coupling_dispatch(d, [&](auto ops) {
    return decltype(ops)::layer(inv != 0, d->mfma_mode, packed, layer, d->L, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B,
                                d->bound, s);
  });
  return rc == -2 ? unsupported(d) : rc;
}

int coupling_dp3_columns(const naz_coupling_desc* d, int* rows) {
  int rc = coupling_dispatch(d, [&](auto ops) { return decltype(ops)::dp3_columns(rows); });
  return rc == -2 ? unsupported(d) : rc;
}

#endif  // part 1

#if NAZ_PART == 0 || NAZ_PART == 2  // ---------------- part 2: the autoregressive flows
// ---- fused autoregressive inverse (made_ar_r16.h): naz nsa / maf log_prob -------------
template <class CF>
struct AROps {
  static int64_t layer_floats() { return CF::LAYER; }
  static int degrees(int* deg) {
    for (int u = 0; u < CF::H; ++u) deg[u] = CF::deg(u);
    return 0;
  }
  // flat per layer: W0m [H][C + D] | b0 [H] | {Wim [H][H] | bi [H]} x (NHID - 1) | Woutm [D P][H] | bout [D P]
  static int pack_host(const float* flat, const int* perm, int L, float* out) {
    constexpr int H = CF::H, D = CF::D, C = CF::C, P = CF::P;
    constexpr int64_t per = (int64_t)H * (C + D) + H + (int64_t)(CF::NHID - 1) * (H * H + H) + (int64_t)D * P * H + D * P;
    for (int l = 0; l < L; ++l) {
      bool seen[32] = {};
      for (int p = 0; p < D; ++p) {
        const int v = perm[l * D + p];
        if (v < 0 || v >= D || seen[v]) return set_error("naz_ar_flow_pack: layer %d: bad permutation", l);
        seen[v] = true;
      }
      made_ar_pack_layer<CF>(flat + l * per, perm + l * D, out + (int64_t)l * CF::LAYER);
    }
    return 0;
  }
  static int log_prob(const float* packed, int L, const float* x, int64_t ldx, const float* ctx, int64_t ldc,
                      const float* low, const float* high, float* out_lp, int64_t B, float bound, hipStream_t s,
                      int64_t P = 1, int64_t spk = 0, int64_t sx = 0, int64_t slp = 0, int c0mode = 0,
                      float* states = nullptr, void* = nullptr, int64_t = 0) {
    static_assert(2 * CF::STG * 4 <= 160 * 1024, "two weight stages exceed the LDS");
    if (B == 0 || L == 0 || P == 0) return 0;
    if (P > 65535) return set_error("naz_ar_flow_log_prob_batched: at most 65535 draws per call");
    const int64_t rows = 16 * CF::NW, grid = (B + rows - 1) / rows;
    const size_t lds = (size_t)2 * CF::STG * 4;
    hipLaunchKernelGGL((made_ar_r16_kernel<CF>), dim3((unsigned)grid, (unsigned)P), dim3(64 * CF::NW), lds, s, packed,
                       L, x, ldx, ctx, ldc, low, high, out_lp, B, bound, spk, sx, slp, c0mode, states);
    return check_launch("made_ar_r16_kernel");
  }
  static int64_t workspace_bytes(int64_t, int64_t) { return 0; }  // every intermediate stays on chip
  static int64_t pass0_floats() { return CF::C0; }
  static int pack_device(const float* flat, int64_t sflat, const int* perm, float* packed, int64_t spk, int L,
                         int64_t P, hipStream_t s, const float* c0 = nullptr, int64_t sc0 = 0,
                         const float* mask = nullptr) {
    if (L == 0 || P == 0) return 0;
    if (P > 65535 || L > 65535) return set_error("naz_ar_flow_pack: at most 65535 draws / layers per call");
    const dim3 grid((unsigned)((CF::LAYER + 255) / 256), (unsigned)L, (unsigned)P);
    hipLaunchKernelGGL((made_ar_pack_kernel<CF>), grid, dim3(256), 0, s, flat, sflat, perm, packed, spk, c0, sc0,
                       mask);
    return check_launch("made_ar_pack_kernel");
  }
  // forward (sample) direction: made_ar_fwd_kernel over CfgARF's per-layer image
  using FW = CfgARF<CF>;
  static int64_t fwd_layer_floats() { return FW::LAYER; }
  static int pack_fwd_host(const float* flat, int L, float* out) {
    constexpr int H = CF::H, D = CF::D, C = CF::C, P = CF::P;
    constexpr int64_t per = (int64_t)H * (C + D) + H + (int64_t)(CF::NHID - 1) * (H * H + H) + (int64_t)D * P * H + D * P;
    for (int l = 0; l < L; ++l) made_ar_pack_fwd_layer<FW>(flat + l * per, out + (int64_t)l * FW::LAYER);
    return 0;
  }
  static int sample(const float* packed, int L, const float* z, int64_t ldz, const float* ctx, int64_t ldc,
                    const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B, float bound,
                    hipStream_t s, int64_t P = 1, int64_t spk = 0, int64_t sz = 0, int64_t sy = 0, int64_t sld = 0) {
    if (B == 0 || P == 0) return 0;
    if (P > 65535) return set_error("naz_ar_flow_sample_batched: at most 65535 draws per call");
    const int64_t rows = 16 * FW::NW, grid = (B + rows - 1) / rows;
    const size_t lds = (size_t)2 * FW::STG * 4;
    hipLaunchKernelGGL((made_ar_fwd_kernel<FW>), dim3((unsigned)grid, (unsigned)P), dim3(64 * FW::NW), lds, s, packed,
                       L, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, bound, spk, sz, sy, sld);
    return check_launch("made_ar_fwd_kernel");
  }
  static int64_t flat_floats() {
    constexpr int H = CF::H, D = CF::D, C = CF::C, P = CF::P;
    return (int64_t)H * (C + D) + H + (int64_t)(CF::NHID - 1) * (H * H + H) + (int64_t)D * P * H + D * P;
  }
  static int pack_fwd_device(const float* flat, int64_t sflat, float* packed, int64_t spk, int L, int64_t P,
                             hipStream_t s, const float* mask = nullptr) {
    if (L == 0 || P == 0) return 0;
    if (P > 65535 || L > 65535) return set_error("naz_ar_flow_pack_fwd: at most 65535 draws / layers per call");
    const dim3 grid((unsigned)((FW::LAYER + 255) / 256), (unsigned)L, (unsigned)P);
    hipLaunchKernelGGL((made_ar_pack_fwd_kernel<FW>), grid, dim3(256), 0, s, flat, sflat, packed, spk, mask);
    return check_launch("made_ar_pack_fwd_kernel");
  }
};

// wide affine MADE (CfgARW): the sampler over CfgARF's image, log_prob over CfgARIW's
// (made_ar_wide.h: the persistent-grid inverse with hidden layers 2.. in per-wave scratch)
static int device_cu_count() { return device_cus(); }

template <class CW>
struct AROpsW {
  using FW = CfgARF<CW>;
  using IW = CfgARIW<CW>;
  static int64_t layer_floats() { return IW::LAYER; }
  static int degrees(int* deg) {
    for (int u = 0; u < CW::H; ++u) deg[u] = CW::deg(u);
    return 0;
  }
  static constexpr int64_t per() { return ARIWFlat<IW>::per(); }
  static int pack_host(const float* flat, const int* perm, int L, float* out) {
    for (int l = 0; l < L; ++l) {
      bool seen[32] = {};
      for (int p = 0; p < CW::D; ++p) {
        const int v = perm[l * CW::D + p];
        if (v < 0 || v >= CW::D || seen[v]) return set_error("naz_ar_flow_pack: layer %d: bad permutation", l);
        seen[v] = true;
      }
      made_ar_pack_wide_layer<IW>(flat + l * per(), perm + l * CW::D, out + (int64_t)l * IW::LAYER);
    }
    return 0;
  }
  static int log_prob(const float* packed, int L, const float* x, int64_t ldx, const float* ctx, int64_t ldc,
                      const float* low, const float* high, float* out_lp, int64_t B, float, hipStream_t s,
                      int64_t P = 1, int64_t spk = 0, int64_t sx = 0, int64_t slp = 0, int c0mode = 0,
                      float* states = nullptr, void* ws = nullptr, int64_t ws_bytes = 0) {
    if (c0mode) return set_error("naz_ar_flow: D=%d H=%d x %d: no pass-0 constants form", CW::D, CW::H, CW::NHID);
    if (states != nullptr && (P != 1 || low != nullptr))
      return set_error("naz_ar_flow_log_prob_train: one draw, no bounds");
    if (B == 0 || L == 0 || P == 0) return 0;
    const int64_t grid = grid_size(B, P);
    // the hidden layers 2.. of every resident wave persist in caller-owned workspace (no allocation
    // inside a call: a captured HIP graph replays one fixed address)
    const int64_t need = workspace_bytes(B, P);
    if (ws == nullptr || ws_bytes < need || (reinterpret_cast<uintptr_t>(ws) & 15) != 0)
      return set_error("naz_ar_flow_log_prob: D=%d H=%d x %d needs %lld B of 16-byte aligned workspace "
                       "(naz_ar_flow_workspace_bytes), got %lld B at %p", CW::D, CW::H, CW::NHID, (long long)need,
                       (long long)ws_bytes, ws);
    const size_t lds = (size_t)2 * IW::STG * 4;
    hipLaunchKernelGGL((made_ar_inv_wide_kernel<IW>), dim3((unsigned)grid), dim3(64 * IW::NW), lds, s, packed, L, x,
                       ldx, ctx, ldc, low, high, out_lp, B, P, spk, sx, slp, static_cast<u32x4*>(ws), states);
    return check_launch("made_ar_inv_wide_kernel");
  }
  // the persistent grid: one 4-wave workgroup per CU (at most one per (draw, row tile))
  static int64_t grid_size(int64_t B, int64_t P) {
    const int64_t tiles = (B + 16 * IW::NW - 1) / (16 * IW::NW) * P;
    return std::min<int64_t>(tiles, device_cu_count());
  }
  static int64_t workspace_bytes(int64_t B, int64_t P) {
    if (B <= 0 || P <= 0) return 0;
    return grid_size(B, P) * IW::NW * IW::SCRATCH_U4 * (int64_t)sizeof(u32x4);
  }
  static int64_t pass0_floats() { return -1; }
  static int pack_device(const float* flat, int64_t sflat, const int* perm, float* packed, int64_t spk, int L,
                         int64_t P, hipStream_t s, const float* c0 = nullptr, int64_t = 0,
                         const float* mask = nullptr) {
    if (c0 != nullptr) return set_error("naz_ar_flow_pack: D=%d H=%d x %d: no pass-0 constants form", CW::D, CW::H,
                                        CW::NHID);
    if (L == 0 || P == 0) return 0;
    if (P > 65535 || L > 65535) return set_error("naz_ar_flow_pack: at most 65535 draws / layers per call");
    const dim3 grid((unsigned)((IW::LAYER + 255) / 256), (unsigned)L, (unsigned)P);
    hipLaunchKernelGGL((made_ar_pack_wide_kernel<IW>), grid, dim3(256), 0, s, flat, sflat, perm, packed, spk, mask);
    return check_launch("made_ar_pack_wide_kernel");
  }
  static int64_t fwd_layer_floats() { return FW::LAYER; }
  static int64_t flat_floats() { return per(); }
  static int pack_fwd_host(const float* flat, int L, float* out) {
    for (int l = 0; l < L; ++l) made_ar_pack_fwd_layer<FW>(flat + l * per(), out + (int64_t)l * FW::LAYER);
    return 0;
  }
  static int sample(const float* packed, int L, const float* z, int64_t ldz, const float* ctx, int64_t ldc,
                    const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B, float bound,
                    hipStream_t s, int64_t P = 1, int64_t spk = 0, int64_t sz = 0, int64_t sy = 0, int64_t sld = 0) {
    if (B == 0 || P == 0) return 0;
    if (P > 65535) return set_error("naz_ar_flow_sample_batched: at most 65535 draws per call");
    const int64_t rows = 16 * FW::NW, grid = (B + rows - 1) / rows;
    const size_t lds = (size_t)2 * FW::STG * 4;
    hipLaunchKernelGGL((made_ar_fwd_kernel<FW>), dim3((unsigned)grid, (unsigned)P), dim3(64 * FW::NW), lds, s, packed,
                       L, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, bound, spk, sz, sy, sld);
    return check_launch("made_ar_fwd_kernel");
  }
  static int pack_fwd_device(const float* flat, int64_t sflat, float* packed, int64_t spk, int L, int64_t P,
                             hipStream_t s, const float* mask = nullptr) {
    if (L == 0 || P == 0) return 0;
    if (P > 65535 || L > 65535) return set_error("naz_ar_flow_pack_fwd: at most 65535 draws / layers per call");
    const dim3 grid((unsigned)((FW::LAYER + 255) / 256), (unsigned)L, (unsigned)P);
    hipLaunchKernelGGL((made_ar_pack_fwd_kernel<FW>), grid, dim3(256), 0, s, flat, sflat, packed, spk, mask);
    return check_launch("made_ar_pack_fwd_kernel");
  }
};

template <class F>
static int ar_dispatch(const naz_ar_desc* d, F&& f) {
  if (d == nullptr || d->act != NAZ_ACT_TANH || d->L < 0) return -2;
#ifdef NAZ_AR_ONLY_WIDE  // resource experiments on the wide instance alone (minutes instead of ten)
  if (d->kind == NAZ_AR_AFFINE && d->D == 4 && d->C == 2 && d->H == 512 && d->n_hidden == 5)
    return f(AROpsW<CfgARW<4, 2, 512, 5>>{});
  return -2;
#endif
  if (d->kind == NAZ_AR_SPLINE) {
    if (d->K != 8 || d->H != 128 || d->n_hidden != 2 || !(d->bound > 0.f)) return -2;
    if (d->D == 16 && d->C == 32) return f(AROps<CfgAR<16, 32, 128, 8>>{});
    if (d->D == 16 && d->C == 0) return f(AROps<CfgAR<16, 0, 128, 8>>{});
    if (d->D == 8 && d->C == 0) return f(AROps<CfgAR<8, 0, 128, 8>>{});
    if (d->D == 4 && d->C == 2) return f(AROps<CfgAR<4, 2, 128, 8>>{});  // naz nsa bench shape
    return -2;
  }
  if (d->kind == NAZ_AR_AFFINE) {
    // K is unused (the instances carry 8); the maf paper shape (train_mle_all_data.py:62-70) and
    // SURVEY §8d's config-3 AR variant
    if (d->D == 2 && d->C == 2 && d->H == 150 && d->n_hidden == 3) return f(AROps<CfgAR<2, 2, 150, 8, 3, true>>{});
    // the 4-parameter Bayesian MAF (calibrate_4p.py:75,90-96; hmc_maf_exact.py:101-133)
    if (d->D == 4 && d->C == 2 && d->H == 150 && d->n_hidden == 3) return f(AROps<CfgAR<4, 2, 150, 8, 3, true>>{});
    if (d->D == 16 && d->C == 32 && d->H == 128 && d->n_hidden == 2) return f(AROps<CfgAR<16, 32, 128, 8, 2, true>>{});
    // naz's production MAFs (4-parameter MLE, POSYDON; AROpsW: the wide sampler and inverse)
    if (d->D == 4 && d->C == 2 && d->H == 512 && d->n_hidden == 5) return f(AROpsW<CfgARW<4, 2, 512, 5>>{});
    return -2;
  }
  return -2;
}

// 1: both directions fused; 2: the forward (sample) direction only (AROpsW); 0: neither
int ar_flow_supported(const naz_ar_desc* d) {
  const int r = ar_dispatch(d, [](auto ops) { return decltype(ops)::layer_floats() < 0 ? 2 : 1; });
  return r > 0 ? r : 0;
}

int64_t ar_flow_packed_bytes(const naz_ar_desc* d) {
  int64_t v = -1;
  ar_dispatch(d, [&](auto ops) {
    v = decltype(ops)::layer_floats() * d->L * 4;
    return 0;
  });
  return v;
}

static int ar_unsupported(const naz_ar_desc* d) {
  if (d == nullptr) return set_error("naz_ar_flow: null descriptor");
  return set_error("naz_ar_flow: no fused instantiation for kind=%d D=%d C=%d H=%d x %d K=%d act=%d", d->kind, d->D,
                   d->C, d->H, d->n_hidden, d->K, d->act);
}

int ar_flow_degrees(const naz_ar_desc* d, int* deg) {
  if (deg == nullptr) return set_error("naz_ar_flow_degrees: null output");
  const int rc = ar_dispatch(d, [&](auto ops) { return decltype(ops)::degrees(deg); });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int ar_flow_pack_host(const naz_ar_desc* d, const float* flat, const int* perm, void* packed) {
  if (flat == nullptr || perm == nullptr || packed == nullptr) return set_error("naz_ar_flow_pack_host: null pointer");
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::pack_host(flat, perm, d->L, static_cast<float*>(packed));
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int64_t ar_flow_fwd_packed_bytes(const naz_ar_desc* d) {
  int64_t v = -1;
  ar_dispatch(d, [&](auto ops) {
    v = decltype(ops)::fwd_layer_floats() * d->L * 4;
    return 0;
  });
  return v;
}

int ar_flow_pack_fwd_host(const naz_ar_desc* d, const float* flat, void* packed) {
  if (flat == nullptr || packed == nullptr) return set_error("naz_ar_flow_pack_fwd_host: null pointer");
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::pack_fwd_host(flat, d->L, static_cast<float*>(packed));
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int ar_flow_sample(const naz_ar_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx, int64_t ldc,
                   const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B, hipStream_t s) {
  if ((low == nullptr) != (high == nullptr)) return set_error("naz_ar_flow_sample: low/high must both be set");
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::sample(static_cast<const float*>(packed), d->L, z, ldz, ctx, ldc, low, high, y, ldy, out_ld,
                                 B, d->bound, s);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int ar_flow_pack_fwd(const naz_ar_desc* d, const float* flat, int64_t sflat, void* packed, int64_t spk, int64_t P,
                     const float* mask, hipStream_t s) {
  if (flat == nullptr || packed == nullptr) return set_error("naz_ar_flow_pack_fwd: null pointer");
  const int rc = ar_dispatch(d, [&](auto ops) {
    using O = decltype(ops);
    if (sflat < O::flat_floats() * d->L || spk < O::fwd_layer_floats() * d->L)
      return set_error("naz_ar_flow_pack_fwd: draw strides shorter than one flow");
    return O::pack_fwd_device(flat, sflat, static_cast<float*>(packed), spk, d->L, P, s, mask);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int ar_flow_sample_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* z, int64_t ldz,
                           int64_t sz, const float* ctx, int64_t ldc, float* y, int64_t ldy, int64_t sy, float* out_ld,
                           int64_t sld, int64_t B, int64_t P, hipStream_t s) {
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::sample(static_cast<const float*>(packed), d->L, z, ldz, ctx, ldc, nullptr, nullptr, y, ldy,
                                 out_ld, B, d->bound, s, P, spk, sz, sy, sld);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int64_t ar_flow_pass0_floats(const naz_ar_desc* d) {
  int64_t v = -1;
  ar_dispatch(d, [&](auto ops) {
    v = decltype(ops)::pass0_floats() * d->L;
    return 0;
  });
  return v;
}

int ar_flow_pack(const naz_ar_desc* d, const float* flat, int64_t sflat, const int* perm, void* packed, int64_t spk,
                 int64_t P, const float* pass0, int64_t sp0, const float* mask, hipStream_t s) {
  if (flat == nullptr || perm == nullptr || packed == nullptr) return set_error("naz_ar_flow_pack: null pointer");
  if (pass0 != nullptr && (d == nullptr || d->C <= 0))
    return set_error("naz_ar_flow_pack: pass-0 constants need a conditional flow");
  const int rc = ar_dispatch(d, [&](auto ops) {
    using O = decltype(ops);
    if (sflat < O::flat_floats() * d->L || spk < O::layer_floats() * d->L)
      return set_error("naz_ar_flow_pack: draw strides shorter than one flow");
    if (pass0 != nullptr && sp0 < O::pass0_floats() * d->L)
      return set_error("naz_ar_flow_pack: pass-0 stride shorter than one flow");
    return O::pack_device(flat, sflat, perm, static_cast<float*>(packed), spk, d->L, P, s, pass0, sp0, mask);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int64_t ar_flow_workspace_bytes(const naz_ar_desc* d, int64_t B, int64_t P) {
  int64_t v = -1;
  ar_dispatch(d, [&](auto ops) {
    v = decltype(ops)::workspace_bytes(B, P);
    return 0;
  });
  return v;
}

int ar_flow_log_prob_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* x, int64_t ldx,
                             int64_t sx, const float* ctx, int64_t ldc, float* out_lp, int64_t slp, int64_t B, int64_t P,
                             int pass0_const, void* ws, int64_t ws_bytes, hipStream_t s) {
  if (pass0_const && (d == nullptr || d->C <= 0 || ldc != 0))
    return set_error("naz_ar_flow_log_prob_batched: pass-0 constants need one context vector (ldc = 0)");
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::log_prob(static_cast<const float*>(packed), d->L, x, ldx, ctx, ldc, nullptr, nullptr, out_lp,
                                   B, d->bound, s, P, spk, sx, slp, pass0_const ? 1 : 0, nullptr, ws, ws_bytes);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int ar_flow_log_prob(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                     int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* ws,
                     int64_t ws_bytes, hipStream_t s) {
  if ((low == nullptr) != (high == nullptr)) return set_error("naz_ar_flow_log_prob: low/high must both be set");
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::log_prob(static_cast<const float*>(packed), d->L, x, ldx, ctx, ldc, low, high, out_lp, B,
                                   d->bound, s, 1, 0, 0, 0, 0, nullptr, ws, ws_bytes);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

int ar_flow_log_prob_train(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                           int64_t ldc, float* out_lp, float* states, int64_t B, void* ws, int64_t ws_bytes,
                           hipStream_t s) {
  if (states == nullptr) return set_error("naz_ar_flow_log_prob_train: null states");
  const int rc = ar_dispatch(d, [&](auto ops) {
    return decltype(ops)::log_prob(static_cast<const float*>(packed), d->L, x, ldx, ctx, ldc, nullptr, nullptr, out_lp,
                                   B, d->bound, s, 1, 0, 0, 0, 0, states, ws, ws_bytes);
  });
  return rc == -2 ? ar_unsupported(d) : rc;
}

#endif  // part 2

#if NAZ_PART == 0 || NAZ_PART == 3  // ---------------- part 3: the autoregressive backward
// ---- fused maf backward (made_ar_bwd.h): the NUTS potential's gradient / the maf NLL step --------
template <class CF>
struct ARBwdOps {
  using CB = CfgARB<CF>;
  static int64_t layer_floats() { return CB::LAYER; }
  static int dims(int* w) {  // operand widths: n_hidden, HP, XA, XB, X0W, rows per tile
    w[0] = CB::NHID;
    w[1] = CB::HP;
    w[2] = CB::XA;
    w[3] = CB::XB;
    w[4] = CB::X0W;
    w[5] = 16 * CB::NW;
    return 0;
  }
  static int pack(const float* flat, const float* mask, float* packed, int L, hipStream_t s) {
    if (L == 0) return 0;
    if (L > 65535) return set_error("naz_ar_flow_pack_bwd: at most 65535 layers");
    const dim3 grid((unsigned)((CB::LAYER + 255) / 256), (unsigned)L);
    hipLaunchKernelGGL((made_ar_pack_bwd_kernel<CB>), grid, dim3(256), 0, s, flat, mask, packed);
    return check_launch("made_ar_pack_bwd_kernel");
  }
  static int layer(const float* fimg, const float* bimg, const int* perm, const float* s_in, const float* ctx,
                   int64_t ldc, const float* g_in, const float* g_lp, const ArBwdOut& o, int64_t B, int clip_zero,
                   hipStream_t s) {
    if (B == 0) return 0;
    const int64_t grid = (B + 16 * CB::NW - 1) / (16 * CB::NW);  // one workgroup per CU at a time (160 KB ring)
    if (grid > 0x7fffffff) return set_error("naz_ar_flow_bwd_layer: batch too large for one launch");
    const size_t lds = (size_t)2 * CB::SLOT * 4;
    hipLaunchKernelGGL((made_ar_bwd_kernel<CB>), dim3((unsigned)grid), dim3(64 * CB::NW), lds, s, fimg, bimg, perm,
                       s_in, ctx, ldc, g_in, g_lp, o, B, clip_zero);
    return check_launch("made_ar_bwd_kernel");
  }
};

template <class F>
static int ar_bwd_dispatch(const naz_ar_desc* d, F&& f) {
  if (d == nullptr || d->act != NAZ_ACT_TANH || d->L < 0 || d->kind != NAZ_AR_AFFINE) return -2;
  // the maf paper shape (train_mle_all_data.py:62-70; the NUTS potential of hmc_maf_exact.py)
  if (d->D == 2 && d->C == 2 && d->H == 150 && d->n_hidden == 3) return f(ARBwdOps<CfgAR<2, 2, 150, 8, 3, true>>{});
  // the 4-parameter Bayesian MAF's NUTS potential (calibrate_4p.py:75,90-96; hmc_maf_exact.py:101-133)
  if (d->D == 4 && d->C == 2 && d->H == 150 && d->n_hidden == 3) return f(ARBwdOps<CfgAR<4, 2, 150, 8, 3, true>>{});
  return -2;
}

static int ar_bwd_unsupported(const naz_ar_desc* d) {
  if (d == nullptr) return set_error("naz_ar_flow_bwd: null descriptor");
  return set_error("naz_ar_flow_bwd: no fused backward for kind=%d D=%d C=%d H=%d x %d act=%d", d->kind, d->D, d->C,
                   d->H, d->n_hidden, d->act);
}

int64_t ar_flow_bwd_packed_bytes(const naz_ar_desc* d) {
  int64_t v = -1;
  ar_bwd_dispatch(d, [&](auto ops) {
    v = decltype(ops)::layer_floats() * d->L * 4;
    return 0;
  });
  return v;
}

int ar_flow_bwd_dims(const naz_ar_desc* d, int* dims) {
  if (dims == nullptr) return set_error("naz_ar_flow_bwd_dims: null output");
  const int rc = ar_bwd_dispatch(d, [&](auto ops) { return decltype(ops)::dims(dims); });
  return rc == -2 ? ar_bwd_unsupported(d) : rc;
}

int ar_flow_pack_bwd(const naz_ar_desc* d, const float* flat, const float* mask, void* packed, hipStream_t s) {
  if (flat == nullptr || packed == nullptr) return set_error("naz_ar_flow_pack_bwd: null pointer");
  const int rc = ar_bwd_dispatch(d, [&](auto ops) {
    return decltype(ops)::pack(flat, mask, static_cast<float*>(packed), d->L, s);
  });
  return rc == -2 ? ar_bwd_unsupported(d) : rc;
}

int ar_flow_bwd_layer(const naz_ar_desc* d, const void* packed_fwd, const void* packed_bwd, const int* perm, int layer,
                      const float* state, const float* ctx, int64_t ldc, const float* g_in, const float* g_lp,
                      float* const* bufs, float* g_out, int64_t B, hipStream_t s) {
  if (d == nullptr || layer < 0 || layer >= d->L) return set_error("naz_ar_flow_bwd_layer: layer out of range");
  const int rc = ar_bwd_dispatch(d, [&](auto ops) {
    using O = decltype(ops);
    using CB = typename O::CB;
    // bufs: x0, then per hidden layer i (ha_i, hb_i), then dp_i, then gout
    ArBwdOut o{};
    o.x0 = bufs[0];
    for (int i = 0; i < CB::NHID; ++i) {
      o.ha[i] = bufs[1 + 2 * i];
      o.hb[i] = bufs[2 + 2 * i];
      o.dp[i] = bufs[1 + 2 * CB::NHID + i];
    }
    o.gout = bufs[1 + 3 * CB::NHID];
    o.g_next = g_out;
    for (int k = 0; k < 2 + 3 * CB::NHID; ++k)
      if (bufs[k] == nullptr && !(k >= 1 && k <= 2 * CB::NHID && (k & 1) == 0 && CB::XB == 0))
        return set_error("naz_ar_flow_bwd_layer: null operand buffer %d", k);
    const float* fimg = static_cast<const float*>(packed_fwd) + (int64_t)layer * CB::FW::LAYER;
    const float* bimg = static_cast<const float*>(packed_bwd) + (int64_t)layer * CB::LAYER;
    return O::layer(fimg, bimg, perm + (int64_t)layer * CB::D, state, ctx, ldc, g_in, g_lp, o, B,
                    (d->flags & NAZ_AR_CLIP_ZERO_GRAD) ? 1 : 0, s);
  });
  return rc == -2 ? ar_bwd_unsupported(d) : rc;
}

#endif  // part 3

}  // namespace naz

#if NAZ_PART == 9  // register-allocation experiments on one wide-inverse instance (not built by build.py)
#ifndef NAZ_EXP_NHID
#define NAZ_EXP_NHID 5
#endif
template __global__ void naz::made_ar_inv_wide_kernel<naz::CfgARIW<naz::CfgARW<4, 2, 512, NAZ_EXP_NHID>>>(
    const float*, int, const float*, int64_t, const float*, int64_t, const float*, const float*, float*, int64_t,
    int64_t, int64_t, int64_t, int64_t, naz::u32x4*, float*);
#endif

#if NAZ_PART == 8  // schedule experiments on the w32 log_prob kernel alone (not built by build.py)
template __global__ void naz::coupling_w32_kernel<naz::CfgX6<16, 32, 8, 8, 128, true, 2>, true>(
    const float*, int, const float*, int64_t, const float*, int64_t, const float*, const float*, float*, float*,
    int64_t, int64_t, float);
#endif

#if NAZ_PART == 7  // the wide sampler alone (not built by build.py)
template __global__ void naz::made_ar_fwd_kernel<naz::CfgARF<naz::CfgARW<4, 2, 512, 5>>>(
    const float*, int, const float*, int64_t, const float*, int64_t, const float*, const float*, float*, int64_t,
    float*, int64_t, float, int64_t, int64_t, int64_t, int64_t);
#endif

#if NAZ_PART == 6  // the config-3 training backward alone (not built by build.py)
template __global__ void naz::coupling_bwd_r16_kernel<naz::CfgR16<16, 32, 8, 8, 128, true>>(
    const float*, const float*, const float*, int, const float*, const float*, int64_t, const float*, const float*,
    naz::BwdOut, int64_t, float);
#endif

#if NAZ_PART == 5  // the nsa16 log_prob kernel alone (not built by build.py)
template __global__ void naz::made_ar_r16_kernel<naz::CfgAR<16, 32, 128, 8>>(
    const float*, int, const float*, int64_t, const float*, int64_t, const float*, const float*, float*, int64_t,
    float, int64_t, int64_t, int64_t, int, float*);
#endif

#if NAZ_PART == 4  // the 4-parameter Bayesian MAF backward alone (not built by build.py)
template struct naz::CfgARB<naz::CfgAR<4, 2, 150, 8, 3, true>>;
#endif
