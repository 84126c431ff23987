// Batch-row GEMMs for the NLL training step: every conditioner GEMM
// of a flow has one huge dimension — the batch (2^20 rows per GPU at config 4) — and small
// feature dimensions (<= a few hundred).  Two shapes cover all of them:
//
//   rowgemm  C[m, n] = act(Σ_k A(m, k) · B(k, n) + bias[n])   m over the batch, n, k small
//            forward F.linear / MaskedLinear (A = cat[ctx, x], B = (W ⊙ mask)ᵀ) and the input
//            gradients dX = dPre · (W ⊙ mask) of the backward pass;
//   wgrad    C[n1, n2] (+)= Σ_m G(m, n1) · X(m, n2) [· mask(n1, n2)]   reduction over the batch
//            the weight gradients dW = mask ⊙ (dPreᵀ · X), with db = Σ_m dPre riding along as an
//            all-ones X column.
//
// Both are exact fp32 (v_mfma_f32_32x32x2_f32, the gfx950 FP32 matrix rate) and tile the batch
// into 128-row workgroup panels so that every HBM byte of the big operand is read once:
//   * rowgemm: a workgroup owns 128 rows × up to 256 output columns (NB 32-column blocks per
//     wave, the wave's 32 rows); k runs in 16-deep chunks through a double-buffered LDS pair
//     [k][m] / [k][n] with the next chunk's global loads in flight during the current chunk's
//     MFMAs; the epilogue fuses bias + activation (+ accumulate);
//   * wgrad: a workgroup reduces a contiguous slice of rows into the full (small) output in
//     registers — each wave owns a set of 32×32 output blocks — and adds it to C with one fp32
//     atomic per element at the end (split-K over workgroups, no partial buffers).
#include <algorithm>
#include <atomic>

#include "naz_device.h"
#include "naz_internal.h"

namespace naz {

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

#ifndef NAZ_RG_BM
#define NAZ_RG_BM 128
#endif
constexpr int RG_BM = NAZ_RG_BM;  // batch rows per workgroup (4 waves x 32)
constexpr int RG_T = 2 * RG_BM;   // threads: one (row, k-half) A loader each
#ifndef NAZ_RG_BK
#define NAZ_RG_BK 16
#endif
constexpr int RG_BK = NAZ_RG_BK;  // k per LDS chunk
constexpr int RG_PAD = 4;
constexpr int RG_APAD = 1;  // As rows 129 floats: the two k-halves a thread pair stores differ by 8 banks

NAZ_DEV floatx16 mfma_f32(float a, float b, floatx16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

struct RowGemmArgs {
  const float* a0;  // first A segment: [M, ka0] rows at stride lda0 (lda0 = 0: one broadcast row)
  int64_t lda0;
  int ka0;
  const float* a1;  // second A segment: [M, ka1] rows at stride lda1
  int64_t lda1;
  int ka1;
  const float* b;  // B(k, n) = b[k * sbk + n * sbn] (* mask[k * smk + n * smn])
  int64_t sbk, sbn;
  const float* mask;
  int64_t smk, smn;
  const float* bias;  // [N] or null
  float* c;           // C[m * ldc + n]
  int64_t ldc;
  int64_t M;
  int N;
  int act;
  int accumulate;
  int vec;  // A segments allow 16-byte loads of 8-k groups (set by rowgemm())
  int vst;  // C rows allow 16-byte stores (row stride % 4 == 0, aligned; set by rowgemm())
  // batch of independent problems along blockIdx.z (per-draw weights, naz_linear_act_batched):
  // problem z reads a0 + z*za0, a1 + z*za1, b + z*zb, bias + z*zbias and writes c + z*zc
  // (the mask is shared); all zero for a single problem
  int64_t za0, za1, zb, zbias, zc;
  // optional epilogue factor act'(dy[m, n]) from a post-activation value (the chained dX of a
  // Linear/act conditioner: dPre_{l-1} = (dPre_l · W_l) ⊙ act'(h_{l-1})); null = none
  const float* dy;
  int64_t lddy;
  int dact;
  int dyvec;  // dy rows allow 16-byte loads (set by rowgemm())
  int bn1;    // B's n index has unit stride: the B chunk is loaded along n (set by rowgemm())
  int bbytes, mbytes;  // byte spans of B / the mask (buffer range: out-of-range loads return 0)
  // optional VJP epilogue of a CNF vector-field layer under the Hutchinson JVP (naz_gemm_jvp_bwd):
  // rows come in (value, tangent) pairs 2i, 2i + 1 and jvp = the layer's stacked output S with the
  // same pairing; C[2i] = G[2i] act' + G[2i+1] (act''/act') S[2i+1], C[2i+1] = G[2i+1] act',
  // act', act''/act' from h = S[2i] (act_d1_ratio).  null = none
  const float* jvp;
  int64_t ldjvp;
  int jact;
  // host-side launch choice (rowgemm()): outputs of more than 4 column blocks in half-width panels
  // (1), in one panel (0), or the library's setting (-1: naz_tuning "rowgemm_split")
  int split = -1;
  // arithmetic (rowgemm()): exact FP32 MFMA (0), bf16x6 (1: rowgemm_x6_kernel), or the library's
  // setting (-1: naz_tuning "rowgemm_x6")
  int x6 = -1;
  // ... or the f16x3 split (1: rowgemm_h3_kernel, |B| < 2^9), or the library's setting (-1:
  // naz_tuning "rowgemm_h3"); x6 wins when both are on
  int h3 = -1;
  // small batches: narrow the column panels until the grid holds this many workgroups per CU
  // (0: off, -1: the library's setting, naz_tuning "rowgemm_fill")
  int fill = -1;
  // ... or the B-resident f16x3 kernel (1: rowgemm_bres_kernel), or the library's setting (-1:
  // naz_tuning "rowgemm_bres"); tried before x6 / h3
  int bres = -1;
};

// A(m, k) of the concatenated row [a0 | a1]
NAZ_DEV float rg_a(const RowGemmArgs& p, int64_t m, int k) {
  if (k < p.ka0) return p.a0[m * p.lda0 + k];
  return p.a1[m * p.lda1 + (k - p.ka0)];
}

// The batch-row GEMM's epilogue (shared by rowgemm_kernel and rowgemm_x6_kernel): accumulator
// (block o, reg r) = C[row, col] with row = (r & 3) + 8 (r >> 2) + 4 (lane >> 5) of the wave's 32 rows
// and col = 32 o + (lane & 31) of the panel; bias + activation, the chained act' (dy), the CNF pair
// VJP (jvp) or accumulation, staged through SHARE floats of LDS per wave into 16-byte row pieces
template <int NB, int SHARE>
NAZ_DEV void rowgemm_epilogue(const RowGemmArgs& p, floatx16 (&acc)[NB], float* smem, int64_t m0, int n0, int wave,
                              int lane) {
  if (p.vst) {
    // staged through this wave's share of the (now free) LDS: EG blocks at a time are written
    // [32 rows][32 EG cols] and stored back as whole 16-byte row pieces
    constexpr int EG = SHARE >= 32 * (64 + 4) ? 2 : 1;
    constexpr int EP = 32 * EG + 4;  // pitch
    float* E = smem + wave * SHARE;
#pragma unroll
    for (int o0 = 0; o0 < NB; o0 += EG) {
#pragma unroll
      for (int oo = 0; oo < EG; ++oo) {
        if (o0 + oo >= NB) continue;
        const int n = n0 + 32 * (o0 + oo) + (lane & 31);
        const float bn = (p.bias != nullptr && n < p.N) ? p.bias[n] : 0.f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          E[row * EP + 32 * oo + (lane & 31)] = activate_rt(p.act, acc[o0 + oo][r] + bn);
        }
      }
      // 8 EG float4 per row; 64 / (8 EG) rows per wave-instruction
      constexpr int F4R = 8 * EG, RPI = 64 / F4R;
      const int rr = lane / F4R, c4 = lane % F4R;
      const int col = n0 + 32 * o0 + 4 * c4;
      const bool inpanel = 32 * o0 + 4 * c4 < 32 * NB;  // odd NB, EG = 2: the pair's second block is absent
      if (p.jvp != nullptr) {  // naz_gemm_jvp_bwd: RPI (value, tangent) row pairs per wave-instruction
#pragma unroll
        for (int it = 0; it < 16 / RPI; ++it) {
          const int pr = it * RPI + rr;
          const int64_t m = m0 + wave * 32 + 2 * pr;  // value row; m + 1 = its tangent row (M is even)
          if (m >= p.M || col >= p.N || !inpanel) continue;
          const float* ev = E + (2 * pr) * EP + 4 * c4;
          const float* sv = p.jvp + m * p.ldjvp + col;
          float* cv = p.c + m * p.ldc + col;
          const int nt = p.N - col < 4 ? p.N - col : 4;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            if (j >= nt) continue;
            float d1, rat;
            act_d1_ratio(p.jact, sv[j], d1, rat);
            const float gv = ev[j], gt = ev[EP + j];
            cv[j] = gv * d1 + gt * sv[p.ldjvp + j] * rat;
            cv[p.ldc + j] = gt * d1;
          }
        }
        continue;
      }
#pragma unroll
      for (int it = 0; it < 32 / RPI; ++it) {
        const int row = it * RPI + rr;
        const int64_t m = m0 + wave * 32 + row;
        if (m >= p.M || col >= p.N || !inpanel) continue;
        float4 v = *reinterpret_cast<const float4*>(E + row * EP + 4 * c4);
        if (p.dy != nullptr) {  // chained act' (naz_gemm_dact), applied on the 16-byte row piece
          const float* dyr = p.dy + m * p.lddy + col;
          if (p.dyvec && col + 4 <= p.N) {  // one 16-byte load of the row piece
            const float4 d4 = *reinterpret_cast<const float4*>(dyr);
            v.x *= activate_grad_from_out(p.dact, d4.x);
            v.y *= activate_grad_from_out(p.dact, d4.y);
            v.z *= activate_grad_from_out(p.dact, d4.z);
            v.w *= activate_grad_from_out(p.dact, d4.w);
          } else {
            v.x *= activate_grad_from_out(p.dact, dyr[0]);
            if (col + 1 < p.N) v.y *= activate_grad_from_out(p.dact, dyr[1]);
            if (col + 2 < p.N) v.z *= activate_grad_from_out(p.dact, dyr[2]);
            if (col + 3 < p.N) v.w *= activate_grad_from_out(p.dact, dyr[3]);
          }
        }
        if (col + 4 <= p.N) {
          float4* dst = reinterpret_cast<float4*>(p.c + m * p.ldc + col);
          if (p.accumulate) {
            const float4 o = *dst;
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *dst = v;
        } else {  // row tail (N % 4 != 0): only the real columns (static indices: no scratch)
          float* d1 = p.c + m * p.ldc + col;
          const int nt = p.N - col;
          d1[0] = p.accumulate ? d1[0] + v.x : v.x;
          if (nt > 1) d1[1] = p.accumulate ? d1[1] + v.y : v.y;
          if (nt > 2) d1[2] = p.accumulate ? d1[2] + v.z : v.z;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int o = 0; o < NB; ++o) {
    const int n = n0 + 32 * o + (lane & 31);
    if (n >= p.N) continue;
    const float bn = p.bias != nullptr ? p.bias[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (m >= p.M) continue;
      float* dst = p.c + m * p.ldc + n;
      const float v = activate_rt(p.act, acc[o][r] + bn);  // (dy: vst path only, see rowgemm_dact)
      *dst = p.accumulate ? *dst + v : v;
    }
  }
}

#ifndef NAZ_RG_OCC
#define NAZ_RG_OCC 4
#endif
// waves per SIMD: up to 4 blocks of accumulators fit 128 VGPRs (4 waves/SIMD); wider tiles 2
template <int NB>
__global__ void __launch_bounds__(RG_T, NB <= 4 ? NAZ_RG_OCC : 2) rowgemm_kernel(RowGemmArgs p) {
  {  // problem of this z slice (uniform: stays in SGPRs)
    const int64_t z = blockIdx.z;
    p.a0 += z * p.za0;
    p.a1 += z * p.za1;
    p.b += z * p.zb;
    if (p.bias != nullptr) p.bias += z * p.zbias;
    p.c += z * p.zc;
  }
  constexpr int BN = 32 * NB;
  constexpr int AS_F = 2 * RG_BK * (RG_BM + RG_APAD), BS_F = 2 * RG_BK * (BN + RG_PAD);
  __shared__ float smem[AS_F + BS_F];
  auto As = reinterpret_cast<float(*)[RG_BK][RG_BM + RG_APAD]>(smem);
  auto Bs = reinterpret_cast<float(*)[RG_BK][BN + RG_PAD]>(smem + AS_F);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = (int64_t)blockIdx.x * RG_BM;
  const int n0 = blockIdx.y * BN;
  const int K = p.ka0 + p.ka1;
  const int nk = (K + RG_BK - 1) / RG_BK;

  // A chunk: 128 rows x RG_BK k, APT per thread in 8-k groups: thread -> (row = tid >> 1, k-half)
  constexpr int APT = RG_BK / 2;
  const int ar = tid >> 1, ak = (tid & 1) * APT;
  const int64_t am = m0 + ar;
  const bool arow = am < p.M;
  // B chunk: RG_BK k x BN n, BPT values per thread.  k-major (B = Wᵀ, unit k stride): thread ->
  // (k = tid % RG_BK, n = tid / RG_BK + (256 / RG_BK) j); n-major (p.bn1: B = W, unit n stride, the
  // dX products): 32 lanes along n, value j = (block j % NB, row half j / NB) -> (k = tid / 32 +
  // 8 (j / NB), n = tid % 32 + 32 (j % NB)).  A k-major load of a row-major W put each lane on another
  // row: 64 cache lines per wave instruction (gemm_dact at half linear_act's rate, r05_g8 probe).
  constexpr int BKS = RG_T / RG_BK;
  static_assert(RG_BK == 16 && RG_T == 256, "the n-major B mapping assumes 16-deep chunks of 256 threads");
  const bool bn1 = p.bn1 != 0;
  const int bk = bn1 ? (tid >> 5) : tid % RG_BK, bn0 = bn1 ? (tid & 31) : tid / RG_BK;
  constexpr int BPT = BN / BKS;
  auto bkj = [&](int j) { return bn1 ? bk + 8 * (j / NB) : bk; };
  auto bnj = [&](int j) { return bn1 ? bn0 + 32 * (j % NB) : bn0 + BKS * j; };

  // B and mask reads are buffer loads over their exact byte spans: an element outside the k x n box
  // reads at offset `span` and returns 0, so the loads are branch-free, and the mask factors are
  // applied at the LDS store (after this chunk's MFMAs), not right behind their loads
  const auto bsrd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.b), (short)0, p.bbytes, 0x00020000);
  const auto msrd =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.mask ? p.mask : p.b), (short)0, p.mbytes, 0x00020000);
  const int sbk = (int)p.sbk, sbn = (int)p.sbn, smk = (int)p.smk, smn = (int)p.smn;
  const bool masked = p.mask != nullptr;
  float ra[APT], rb[BPT], rm[BPT];
  auto load = [&](int kc) {
    const int kc0 = kc * RG_BK;
#pragma unroll
    for (int g8 = 0; g8 < APT; g8 += 8) {
      const int kb = kc0 + ak + g8;
      if (p.vec && arow && kb + 8 <= K && (kb >= p.ka0 || kb + 8 <= p.ka0)) {
        // 8 consecutive k inside one segment, 16-byte aligned rows (checked on the host)
        const float* src = kb < p.ka0 ? p.a0 + am * p.lda0 + kb : p.a1 + am * p.lda1 + (kb - p.ka0);
        const float4 v0 = *reinterpret_cast<const float4*>(src);
        const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
        ra[g8 + 0] = v0.x; ra[g8 + 1] = v0.y; ra[g8 + 2] = v0.z; ra[g8 + 3] = v0.w;
        ra[g8 + 4] = v1.x; ra[g8 + 5] = v1.y; ra[g8 + 6] = v1.z; ra[g8 + 7] = v1.w;
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = kb + i;
          ra[g8 + i] = (arow && k < K) ? rg_a(p, am, k) : 0.f;
        }
      }
    }
#pragma unroll
    for (int j = 0; j < BPT; ++j) {
      // weights / masks are small: 32-bit buffer offsets (no 64-bit address registers)
      const int k = kc0 + bkj(j), n = n0 + bnj(j);
      const bool in = k < K && n < p.N;
      rb[j] = __builtin_bit_cast(
          float, __builtin_amdgcn_raw_buffer_load_b32(bsrd, in ? 4 * (k * sbk + n * sbn) : p.bbytes, 0, 0));
      if (masked)
        rm[j] = __builtin_bit_cast(
            float, __builtin_amdgcn_raw_buffer_load_b32(msrd, in ? 4 * (k * smk + n * smn) : p.mbytes, 0, 0));
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < APT; ++i) As[buf][ak + i][ar] = ra[i];
#pragma unroll
    for (int j = 0; j < BPT; ++j) Bs[buf][bkj(j)][bnj(j)] = masked ? rb[j] * rm[j] : rb[j];
  };

  floatx16 acc[NB];
#pragma unroll
  for (int o = 0; o < NB; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = 0.f;

  load(0);
  store(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    if (kc + 1 < nk) load(kc + 1);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int kk = 0; kk < RG_BK; kk += 2) {
      const float a = As[buf][kk + (lane >> 5)][wave * 32 + (lane & 31)];
#pragma unroll
      for (int o = 0; o < NB; ++o) acc[o] = mfma_f32(a, Bs[buf][kk + (lane >> 5)][32 * o + (lane & 31)], acc[o]);
    }
    if (kc + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  rowgemm_epilogue<NB, (AS_F + BS_F) / (RG_T / 64)>(p, acc, smem, m0, n0, wave, lane);
}

template <int NB>
void rowgemm_launch(const RowGemmArgs& p, int nz, hipStream_t s) {
  dim3 grid((unsigned)((p.M + RG_BM - 1) / RG_BM), (unsigned)((p.N + 32 * NB - 1) / (32 * NB)), (unsigned)nz);
  hipLaunchKernelGGL(rowgemm_kernel<NB>, grid, dim3(RG_T), 0, s, p);
}

static bool al16(const void* q) { return (reinterpret_cast<uintptr_t>(q) & 15) == 0; }

}  // namespace

// the library-wide panel-split setting (naz_tuning "rowgemm_split"): NAZ_RG_SPLIT at first use, else
// on (round 5 same-box A/B of the wide maf NLL step); v >= 0 sets it; returns the
// setting before the call
int rowgemm_x6_setting(int v) {
  // NAZ_RG_X6 at first use, else off until a same-box A/B sets the default
  static std::atomic<int> cur{[] {
    const char* e = getenv("NAZ_RG_X6");
    return e ? (atoi(e) != 0 ? 1 : 0) : 0;
  }()};
  return v >= 0 ? cur.exchange(v != 0 ? 1 : 0) : cur.load();
}

int rowgemm_h3_setting(int v) {
  // NAZ_RG_H3 at first use, else off until a same-box A/B sets the default
  static std::atomic<int> cur{[] {
    const char* e = getenv("NAZ_RG_H3");
    return e ? (atoi(e) != 0 ? 1 : 0) : 0;
  }()};
  return v >= 0 ? cur.exchange(v != 0 ? 1 : 0) : cur.load();
}

int rowgemm_bres_setting(int v) {
  // NAZ_RG_BRES at first use, else off until a same-box A/B sets the default
  static std::atomic<int> cur{[] {
    const char* e = getenv("NAZ_RG_BRES");
    return e ? (atoi(e) != 0 ? 1 : 0) : 0;
  }()};
  return v >= 0 ? cur.exchange(v != 0 ? 1 : 0) : cur.load();
}

int rowgemm_fill_setting(int v) {
  // NAZ_RG_FILL at first use, else 2 workgroups (= waves per SIMD) per CU (with the wide-maf step's
  // side streams: 163.5 ms at 2^16 rows vs 168.5 at 4 and 179.5 at 8; 10,752 rows 49.3 vs 48.7 / 48.9;
  // profiles/r05_g25_*)
  static std::atomic<int> cur{[] {
    const char* e = getenv("NAZ_RG_FILL");
    const int f = e ? atoi(e) : 2;
    return f < 0 ? 0 : (f > 16 ? 16 : f);
  }()};
  return v >= 0 ? cur.exchange(v > 16 ? 16 : v) : cur.load();
}

int rowgemm_split_setting(int v) {
  static std::atomic<int> cur{[] {
    const char* e = getenv("NAZ_RG_SPLIT");
    return e ? (atoi(e) != 0 ? 1 : 0) : 1;
  }()};
  return v >= 0 ? cur.exchange(v != 0 ? 1 : 0) : cur.load();
}

namespace {

int rowgemm_x6_dispatch(const RowGemmArgs& p, int nz, int nb, hipStream_t s);  // below
int rowgemm_h3_dispatch(const RowGemmArgs& p, int nz, int nb, hipStream_t s);
int rowgemm_bres_nb(const RowGemmArgs& p, int nz);
int rowgemm_bres_dispatch(const RowGemmArgs& p, int nb, hipStream_t s);

int rowgemm(RowGemmArgs p, hipStream_t s, int nz = 1) {
  if (p.M <= 0 || p.N <= 0 || nz <= 0) return 0;
  const int64_t K = p.ka0 + p.ka1;
  const int64_t bspan = (K - 1) * (p.sbk < 0 ? -p.sbk : p.sbk) + (int64_t)(p.N - 1) * (p.sbn < 0 ? -p.sbn : p.sbn);
  const int64_t mspan = (K - 1) * (p.smk < 0 ? -p.smk : p.smk) + (int64_t)(p.N - 1) * (p.smn < 0 ? -p.smn : p.smn);
  if (p.sbk < 0 || p.sbn < 0 || p.smk < 0 || p.smn < 0 || 4 * bspan >= (1ll << 31) || 4 * mspan >= (1ll << 31))
    return 1;  // weights too large for the 32-bit buffer offsets: caller falls back
  p.vec = (p.ka0 % 8 == 0) && (p.ka0 == 0 || (al16(p.a0) && p.lda0 % 4 == 0)) &&
          (p.ka1 == 0 || (al16(p.a1) && p.lda1 % 4 == 0));
  p.vst = p.ldc % 4 == 0 && al16(p.c);  // 16-byte row pieces; a ragged row tail is stored per column
  p.dyvec = p.dy != nullptr && p.lddy % 4 == 0 && al16(p.dy);
  p.bn1 = p.sbn == 1 && p.sbk != 1;  // the dX products' B = W (row-major [k][n]): lanes along n
  p.bbytes = (int)(4 * (bspan + 1));
  p.mbytes = (int)(4 * (mspan + 1));
  if (nz > 1) {  // every problem's base keeps the alignment
    p.vec = p.vec && p.za0 % 4 == 0 && p.za1 % 4 == 0;
    p.vst = p.vst && p.zc % 4 == 0;
  }
  // the B-resident f16x3 form (naz_tuning "rowgemm_bres") where a panel of B fits the LDS
  const int bres = p.bres >= 0 ? p.bres : rowgemm_bres_setting(-1);
  if (bres && K >= 16) {
    const int bnb = rowgemm_bres_nb(p, nz);
    if (bnb > 0) return rowgemm_bres_dispatch(p, bnb, s);
  }
  int nb = (p.N + 31) / 32;
  // panel split: outputs of more than 4 column blocks in balanced panels of at most 4 blocks (4 waves
  // per SIMD instead of 2: the wide maf's 168-172-unit degree blocks as 2 x 3, its 512-unit layers as
  // 4 x 4 instead of 2 x 8 — 42 -> 100 TF at 2^16 rows, profiles/r05_g8_rg_probe.txt).  An odd NB's
  // paired epilogue (EG = 2) stores only inside its panel (`inpanel` above);
  // tests/test_gpu_grad.py::test_rowgemm_panel_split runs every epilogue at N = 168 / 172 / 300 with
  // the split on and off against fp64.
  const int split = p.split >= 0 ? p.split : rowgemm_split_setting(-1);
  if (split && nb > 4) {
    const int panels = (nb + 3) / 4;
    nb = (nb + panels - 1) / panels;
  }
  // grid fill: at naz's 10,752-row minibatch a 128-row panel grid is 84 workgroups tall, so the wide
  // maf's 512-unit layers ran 168 workgroups (one wave on two of three SIMDs).  Narrower column
  // panels (nb halved, down to one 32-column block) until the grid holds `fill` workgroups per CU:
  // A panels are re-read once per column panel, from L2.
  const int fill = p.fill >= 0 ? p.fill : rowgemm_fill_setting(-1);
  if (fill > 0) {
    const int64_t target = (int64_t)fill * device_cus();
    const int64_t gx = (p.M + RG_BM - 1) / RG_BM * nz;
    while (nb > 1 && gx * ((p.N + 32 * (nb > 8 ? 8 : nb) - 1) / (32 * (nb > 8 ? 8 : nb))) < target) nb = (nb + 1) / 2;
  }
  // the bf16x6 form where the batch is long enough to fill the chip and k deep enough to pay the split
  const int x6 = p.x6 >= 0 ? p.x6 : rowgemm_x6_setting(-1);
  if (x6 && K >= 32 && p.M >= 2048) return rowgemm_x6_dispatch(p, nz, nb, s);
  // the f16x3 form (the caller's |B| < 2^9: naz_tuning "rowgemm_h3")
  const int h3 = p.h3 >= 0 ? p.h3 : rowgemm_h3_setting(-1);
  if (h3 && K >= 32 && p.M >= 2048) return rowgemm_h3_dispatch(p, nz, nb, s);
  switch (nb > 8 ? 8 : nb) {
    case 1: rowgemm_launch<1>(p, nz, s); break;
    case 2: rowgemm_launch<2>(p, nz, s); break;
    case 3: rowgemm_launch<3>(p, nz, s); break;
    case 4: rowgemm_launch<4>(p, nz, s); break;
    case 5: rowgemm_launch<5>(p, nz, s); break;
    case 6: rowgemm_launch<6>(p, nz, s); break;
    case 7: rowgemm_launch<7>(p, nz, s); break;
    default: rowgemm_launch<8>(p, nz, s); break;
  }
  return check_launch("rowgemm_kernel");
}

// ------------------------------------------------------------------------------------------
// wgrad: C[n1, n2] += Σ_{m in slice} G[m * sgm + n1] · X[m * sxm + n2]
// ------------------------------------------------------------------------------------------
constexpr int WG_BK = 16;     // rows per LDS chunk
constexpr int WG_MAXB = 8;    // 32x32 output blocks per wave (<= 128 accumulator regs)

struct WGradArgs {
  const float* g;  // [M, N1] at row stride sgm, unit column stride
  int64_t sgm;
  const float* x;  // [M, N2] at row stride sxm (0: one broadcast row), unit column stride
  int64_t sxm;
  int64_t M;
  int N1, N2;
  int ones;        // 1: logical X column N2 is all ones, its C column goes to rowsum[n1]
  float* c;        // C[n1 * scm + n2 * scn]
  int64_t scm, scn;
  const float* mask;  // mask[n1 * smm + n2 * smn] or null
  int64_t smm, smn;
  float* rowsum;
  int64_t rows_per_wg;
  int blk0;        // first output block (of NB1 x NB2, n2-fastest) this launch owns
  // batched reductions (wgrad_x6 only, blockIdx.y = batch b): g, x, c, rowsum advance by b times these
  int64_t bg, bx, bc, br;
  // wgrad_x6 only: > 0 = workgroup w takes the R-row chunks starting at w R, w R + chunk_stride, ...
  // (interleaved over the grid) instead of the contiguous rows_per_wg block
  int64_t chunk_stride;
};

// one workgroup: rows [mb, me) of G and X -> its share of every output block, added atomically
__global__ void __launch_bounds__(256, 2) wgrad_kernel(WGradArgs p) {
  constexpr int BN = 256;  // max n1 / n2 (8 blocks of 32)
  __shared__ float Gs[2][WG_BK][BN + RG_PAD];
  __shared__ float Xs[2][WG_BK][BN + RG_PAD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N2e = p.N2 + p.ones;
  const int NB1 = (p.N1 + 31) / 32, NB2 = (N2e + 31) / 32;
  const int64_t mb = (int64_t)blockIdx.x * p.rows_per_wg;
  const int64_t me = (mb + p.rows_per_wg) < p.M ? (mb + p.rows_per_wg) : p.M;
  int bi[WG_MAXB], bj[WG_MAXB];
  bool bv[WG_MAXB];
#pragma unroll
  for (int j = 0; j < WG_MAXB; ++j) {
    const int q = p.blk0 + wave + 4 * j;
    bv[j] = q < NB1 * NB2;
    bi[j] = bv[j] ? q / NB2 : 0;
    bj[j] = bv[j] ? q - (q / NB2) * NB2 : 0;
  }
  floatx16 acc[WG_MAXB];
#pragma unroll
  for (int j = 0; j < WG_MAXB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;

  const int ncol1 = NB1 * 32, ncol2 = NB2 * 32;
  const int rr = tid >> 4, cc = tid & 15;  // chunk load: row rr, columns cc + 16 i
  float rg[16], rx[16];
  auto load = [&](int64_t m0) {
    const int64_t m = m0 + rr;
    const bool mrow = m < me;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = cc + 16 * i;
      rg[i] = (mrow && n < p.N1) ? p.g[m * p.sgm + n] : 0.f;
      rx[i] = mrow ? (n < p.N2 ? p.x[m * p.sxm + n] : (n == p.N2 && p.ones ? 1.f : 0.f)) : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int n = cc + 16 * i;
      if (n < ncol1) Gs[buf][rr][n] = rg[i];
      if (n < ncol2) Xs[buf][rr][n] = rx[i];
    }
  };
  if (mb < me) {
    load(mb);
    store(0);
  }
  __syncthreads();
  int buf = 0;
  for (int64_t m0 = mb; m0 < me; m0 += WG_BK, buf ^= 1) {
    const bool more = m0 + WG_BK < me;
    if (more) load(m0 + WG_BK);
#pragma unroll
    for (int kk = 0; kk < WG_BK; kk += 2) {
      const int k = kk + (lane >> 5);
#pragma unroll
      for (int j = 0; j < WG_MAXB; ++j) {
        if (!bv[j]) continue;
        const float a = Gs[buf][k][32 * bi[j] + (lane & 31)];
        const float b = Xs[buf][k][32 * bj[j] + (lane & 31)];
        acc[j] = mfma_f32(a, b, acc[j]);
      }
    }
    if (more) store(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int j = 0; j < WG_MAXB; ++j) {
    if (!bv[j]) continue;
    const int n2 = 32 * bj[j] + (lane & 31);
    if (n2 >= N2e) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n1 = 32 * bi[j] + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (n1 >= p.N1) continue;
      float v = acc[j][r];
      if (n2 < p.N2) {
        if (p.mask != nullptr) v *= p.mask[(int64_t)n1 * p.smm + (int64_t)n2 * p.smn];
        atomicAdd(p.c + (int64_t)n1 * p.scm + (int64_t)n2 * p.scn, v);
      } else {
        atomicAdd(p.rowsum + n1, v);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------
// wgrad_flat: the same reduction for dense operands (G and X contiguous [M, N] rows, 16-byte
// aligned, N % 4 == 0), which is what the training walk passes.  A chunk of R rows of either
// operand is then ONE contiguous span: it is fetched with flat 16-byte loads spread over all
// 256 threads, R sized so every chunk moves ~32 KB (narrow X -> more rows), and copied to LDS
// unpadded ([row][N]; MFMA operand reads past column N only feed discarded outputs).  db is a
// VALU column sum of the G chunk, so it costs no MFMA block.  Loads of chunk i+1 are in flight
// (registers) while chunk i's MFMAs run.
// ------------------------------------------------------------------------------------------
#ifndef NAZ_WF_Q
#define NAZ_WF_Q 8
#endif
constexpr int WF_Q = NAZ_WF_Q;   // float4 prefetch slots per thread (16 B x 256 x WF_Q per chunk)

template <int MAXB>
__global__ void __launch_bounds__(256, MAXB <= 1 ? 4 : (MAXB <= 2 ? 3 : 2)) wgrad_flat_kernel(WGradArgs p, int R) {
  extern __shared__ float wlds[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int N1 = p.N1, N2 = p.N2;
  float* const Gs = wlds;             // [R][N1]
  float* const Xs = wlds + R * N1;    // [R][N2] (+ slack for reads past the last row)
  const int NB1 = (N1 + 31) / 32, NB2 = (N2 + 31) / 32;
  const int64_t mb = (int64_t)blockIdx.x * p.rows_per_wg;
  const int64_t me = (mb + p.rows_per_wg) < p.M ? (mb + p.rows_per_wg) : p.M;
  // this wave's output blocks q = blk0 + wave + 4j; past-the-end slots duplicate block 0 (their
  // MFMAs run unconditionally so the k loop has no per-block branches; results are dropped)
  int bi[MAXB], bj[MAXB], ga[MAXB], xb[MAXB];
  bool bv[MAXB];
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    const int q = p.blk0 + wave + 4 * j;
    bv[j] = q < NB1 * NB2;
    bi[j] = bv[j] ? q / NB2 : 0;
    bj[j] = bv[j] ? q - (q / NB2) * NB2 : 0;
    ga[j] = 32 * bi[j] + (lane & 31);
    xb[j] = 32 * bj[j] + (lane & 31);
  }
  floatx16 acc[MAXB];
#pragma unroll
  for (int j = 0; j < MAXB; ++j)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
  float dbs = 0.f;  // column sum of G for column tid (db)

  const int fg = R * N1 / 4, fx = R * N2 / 4;  // float4 per chunk
  float4 rq[WF_Q];
  auto load = [&](int64_t m0) {
    const int64_t rows = (me - m0) < R ? (me - m0) : R;
    const int lg = (int)(rows * N1 / 4), lx = (int)(rows * N2 / 4);  // valid float4 (zero past them)
    const float4* g4 = reinterpret_cast<const float4*>(p.g + m0 * N1);
    const float4* x4 = reinterpret_cast<const float4*>(p.x + m0 * N2);
#pragma unroll
    for (int i = 0; i < WF_Q; ++i) {
      const int q = tid + 256 * i;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < fg) {
        if (q < lg) v = g4[q];
      } else if (q - fg < fx) {
        if (q - fg < lx) v = x4[q - fg];
      }
      rq[i] = v;
    }
  };
  auto store = [&]() {
    float4* l4 = reinterpret_cast<float4*>(wlds);
#pragma unroll
    for (int i = 0; i < WF_Q; ++i) {
      const int q = tid + 256 * i;
      if (q < fg + fx) l4[q] = rq[i];
    }
  };
  if (mb < me) load(mb);
  for (int64_t m0 = mb; m0 < me; m0 += R) {
    __syncthreads();  // the previous chunk's readers are done
    store();
    __syncthreads();
    if (m0 + R < me) load(m0 + R);  // in flight during this chunk's MFMAs
    // R is a multiple of 16; rows past the chunk's end were loaded as zeros
    constexpr int U = MAXB >= 8 ? 2 : 4;  // k rows per unrolled group (8 blocks: no room to pipeline)
    for (int kk = 0; kk < R; kk += U) {
#pragma unroll
      for (int u = 0; u < U; u += 2) {
        const int k = kk + u + (lane >> 5);
        float a[MAXB], b[MAXB];
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          a[j] = Gs[k * N1 + ga[j]];
          b[j] = Xs[k * N2 + xb[j]];
        }
#pragma unroll
        for (int j = 0; j < MAXB; ++j) acc[j] = mfma_f32(a[j], b[j], acc[j]);
      }
    }
    if (p.ones && tid < N1)
      for (int r = 0; r < R; ++r) dbs += Gs[r * N1 + tid];
  }
#pragma unroll
  for (int j = 0; j < MAXB; ++j) {
    if (!bv[j]) continue;
    const int n2 = 32 * bj[j] + (lane & 31);
    if (n2 >= N2) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int n1 = 32 * bi[j] + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      if (n1 >= N1) continue;
      float v = acc[j][r];
      if (p.mask != nullptr) v *= p.mask[(int64_t)n1 * p.smm + (int64_t)n2 * p.smn];
      atomicAdd(p.c + (int64_t)n1 * p.scm + (int64_t)n2 * p.scn, v);
    }
  }
  if (p.ones && tid < N1) atomicAdd(p.rowsum + tid, dbs);
}

// wgrad_t16: the same reduction C += Gᵀ X (+ rowsum += Σ_r G[r]) on v_mfma_f32_16x16x4_f32.
// A chunk of R rows of G and X is copied to LDS as it lies in memory (row-major, 16-byte
// pieces, all of a thread's loads issued before its stores).  Wave w owns output row-blocks
// w, w + 4, ... (NOW of them) x all NB2 column blocks; a 16x16x4 step takes A = G[r][o] and
// B = X[r][j] from lane (m, kq) for ONE batch row r = base + 4 kq + t (t = step within the
// group of four), so each operand block costs one ds_read_b32 per step and feeds NB2 (or NOW)
// MFMAs — against one ds_read_b32 per operand per 32x32x2 MFMA in wgrad_flat.  The k order
// inside the sum is free; it only has to be the same for A and B.
typedef float floatx4w __attribute__((ext_vector_type(4)));
// rows per chunk: a multiple of 16 with both operand pieces whole 1 KB DMA pieces and the
// two-slot ring within `cap` bytes; 0 = no such R
static int wgrad_t16_rows(int n1, int n2, int cap) {
  int best = 0;
  for (int R = 16; R <= 128; R += 16)
    if ((R * n1) % 256 == 0 && (R * n2) % 256 == 0 && 2 * R * (n1 + n2) * 4 <= cap) best = R;
  return best;
}

// JS = 2: eight waves, the column blocks split in halves between waves w and w + 4 (keeps a
// wave's accumulators <= 12 blocks)
template <int NOW, int NB2, int JS>
__global__ void __launch_bounds__(256 * JS, 2 / JS) wgrad_t16_kernel(WGradArgs p, int R) {
  extern __shared__ float tl[];
  constexpr int NT = 256 * JS, NBW = NB2 / JS;
  const int tid = threadIdx.x, lane = tid & 63, wave = (tid >> 6) & 3, jh = tid >> 8, m = lane & 15,
            kq = lane >> 4;
  const int N1 = p.N1, N2 = p.N2;
  {
    const int64_t bz = blockIdx.y;
    p.g += bz * p.bg;
    p.x += bz * p.bx;
    p.c += bz * p.bc;
    if (p.rowsum != nullptr) p.rowsum += bz * p.br;
  }
  const int64_t mb = (int64_t)blockIdx.x * p.rows_per_wg;
  const int64_t me = (mb + p.rows_per_wg) < p.M ? (mb + p.rows_per_wg) : p.M;
  floatx4w acc[NOW][NBW];
#pragma unroll
  for (int i = 0; i < NOW; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = floatx4w{0.f, 0.f, 0.f, 0.f};
  float dsum[NOW];
#pragma unroll
  for (int i = 0; i < NOW; ++i) dsum[i] = 0.f;
  // operand columns are NOT masked: a lane of a past-the-end block (o >= N1 or j >= N2) reads
  // whatever lies there in LDS (the next row / the ring slack) and only feeds accumulator rows
  // or columns the write-back drops, because an MFMA never mixes C rows or C columns.
  // chunks stream through a two-slot LDS ring by LDS-DMA (global_load_lds_dwordx4, 1 KB per
  // wave-instruction): chunk c + 1 lands while chunk c computes.  A partial last chunk is copied
  // with bounds-checked loads instead (the DMA would read past the arrays).
  const int CH = R * (N1 + N2);  // floats per chunk = per ring slot
  const int nw = NT / 64, wv = tid >> 6;
  auto issue = [&](int64_t m0, float* dst) {
    const float* src[2] = {p.g + m0 * N1, p.x + m0 * N2};
    const int cnt[2] = {R * N1 / 256, R * N2 / 256};
    float* d = dst;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      for (int c = wv; c < cnt[h]; c += nw)
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src[h] + c * 256 + lane * 4),
                                         (void __attribute__((address_space(3)))*)(d + c * 256), 16, 0, 0);
      d += R * (h == 0 ? N1 : N2);
    }
  };
  auto copy_tail = [&](int64_t m0, float* dst) {
    const int64_t rows = me - m0;
    const int lg = (int)(rows * N1 / 4), lx = (int)(rows * N2 / 4), fg = R * N1 / 4;
    const float4* gp = reinterpret_cast<const float4*>(p.g + m0 * N1);
    const float4* xp = reinterpret_cast<const float4*>(p.x + m0 * N2);
    float4* l4 = reinterpret_cast<float4*>(dst);
    for (int q = tid; q < CH / 4; q += NT) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < fg) {
        if (q < lg) v = gp[q];
      } else if (q - fg < lx) {
        v = xp[q - fg];
      }
      l4[q] = v;
    }
  };
  auto fill = [&](int64_t m0, float* dst) {
    if (m0 + R <= me) issue(m0, dst);
    else copy_tail(m0, dst);
  };
  int slot = 0;
  if (mb < me) fill(mb, tl);
  for (int64_t m0 = mb; m0 < me; m0 += R, slot ^= 1) {
    ring_barrier();  // chunk m0 has landed (vmcnt drained); every wave is done with the other slot
    float* const Gs = tl + slot * CH;
    float* const Xs = Gs + R * N1;
    if (m0 + R < me) fill(m0 + R, tl + (slot ^ 1) * CH);
    // step s reads batch row 4 s + kq; lane bases advance 4 rows per step and the block offsets
    // (64 i for A, 16 j for B) are immediate ds_read offsets.  Operands of step s + 1 are read
    // before the MFMAs of step s (ping-pong registers, two steps per trip), so LDS latency hides
    // under 12 MFMAs.  The read one step past the chunk lands in the next operand / the slack.
    const float* pa = Gs + kq * N1 + wave * 16 + m;
    const float* pb = Xs + kq * N2 + jh * NBW * 16 + m;
    const int sa = 4 * N1, sb = 4 * N2;
    float a0[NOW], b0[NBW], a1[NOW], b1[NBW];
    auto rd = [&](float (&a)[NOW], float (&b)[NBW]) {
#pragma unroll
      for (int i = 0; i < NOW; ++i) a[i] = pa[64 * i];
#pragma unroll
      for (int j = 0; j < NBW; ++j) b[j] = pb[16 * j];
      pa += sa;
      pb += sb;
    };
    auto step = [&](const float (&a)[NOW], const float (&b)[NBW]) {
#pragma unroll
      for (int i = 0; i < NOW; ++i) dsum[i] += a[i];
#pragma unroll
      for (int i = 0; i < NOW; ++i)
#pragma unroll
        for (int j = 0; j < NBW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    };
    rd(a0, b0);
    for (int s = 0; s < R / 4; s += 2) {  // sched_barrier: keep the reads ahead of the MFMAs
      rd(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      step(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      rd(a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      step(a1, b1);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // C[o][j]: lane holds rows o = ob 16 + 4 kq + r, column j = jb 16 + m
#pragma unroll
  for (int i = 0; i < NOW; ++i) {
    const int ob = wave + 4 * i;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int n2 = 16 * (jh * NBW + j) + m;
      if (n2 >= N2) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n1 = 16 * ob + 4 * kq + r;
        if (n1 >= N1) continue;
        float v = acc[i][j][r];
        if (p.mask != nullptr) v *= p.mask[(int64_t)n1 * p.smm + (int64_t)n2 * p.smn];
        atomicAdd(p.c + (int64_t)n1 * p.scm + (int64_t)n2 * p.scn, v);
      }
    }
    if (p.ones && jh == 0) {  // db: column sums of G, partial per quarter -> reduce over kq
      float v = dsum[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int o = 16 * ob + m;
      if (kq == 0 && o < N1) atomicAdd(p.rowsum + o, v);
    }
  }
}

template <int NOW, int NB2>
static void wgrad_t16_go(const WGradArgs& q, int R, size_t lds, unsigned gx, hipStream_t s) {
  constexpr int JS = (NOW * NB2 > 12 && NB2 % 2 == 0) ? 2 : 1;
  hipLaunchKernelGGL((wgrad_t16_kernel<NOW, NB2, JS>), dim3(gx), dim3(256 * JS), lds, s, q, R);
}

template <int NOW>
static bool wgrad_t16_launch(int nb2, const WGradArgs& q, int R, size_t lds, unsigned gx, hipStream_t s) {
  switch (nb2) {
    case 1: wgrad_t16_go<NOW, 1>(q, R, lds, gx, s); return true;
    case 2: wgrad_t16_go<NOW, 2>(q, R, lds, gx, s); return true;
    case 3: wgrad_t16_go<NOW, 3>(q, R, lds, gx, s); return true;
    case 4: wgrad_t16_go<NOW, 4>(q, R, lds, gx, s); return true;
    case 6: wgrad_t16_go<NOW, 6>(q, R, lds, gx, s); return true;
    case 8: wgrad_t16_go<NOW, 8>(q, R, lds, gx, s); return true;
    default: return false;
  }
}

// wgrad on the 16x16x4 transposed-tile kernel when the shape has an instantiation (N1 <= 256,
// N2 <= 128, both multiples of 4); false = not taken
static bool wgrad_t16(WGradArgs p, hipStream_t s) {
  const int nb1 = (p.N1 + 15) / 16, now = (nb1 + 3) / 4;
  int nb2 = (p.N2 + 15) / 16;
  nb2 = nb2 <= 4 ? nb2 : (nb2 <= 6 ? 6 : (nb2 <= 8 ? 8 : 0));
  if (now < 1 || now > 4 || nb2 == 0) return false;
  // 8-wave workgroups (JS = 2) run one per CU: give them most of the LDS; 4-wave ones three
  const bool js2 = now * nb2 > 12 && nb2 % 2 == 0;
  const int R = wgrad_t16_rows(p.N1, p.N2, js2 ? 147456 : 49152);
  if (R == 0) return false;
  // + slack for the unmasked past-the-end reads (the prefetch one step past slot 1's chunk and
  // the padding columns of its last rows)
  const size_t lds = ((size_t)2 * R * (p.N1 + p.N2) + 4 * p.N2 + 16 * nb2 + 64) * 4;
  int64_t rpw = (p.M + (js2 ? 511 : 767)) / (js2 ? 512 : 768);
  rpw = (rpw + R - 1) / R * R;
  if (rpw < 4 * R) rpw = 4 * R;
  p.rows_per_wg = rpw;
  const unsigned gx = (unsigned)((p.M + rpw - 1) / rpw);
  switch (now) {
    case 1: return wgrad_t16_launch<1>(nb2, p, R, lds, gx, s);
    case 2: return wgrad_t16_launch<2>(nb2, p, R, lds, gx, s);
    case 3: return wgrad_t16_launch<3>(nb2, p, R, lds, gx, s);
    default: return wgrad_t16_launch<4>(nb2, p, R, lds, gx, s);
  }
}

// wgrad_x6: the same reduction on the bf16 matrix pipe, exact to fp32 products.  Every operand
// value is split EXACTLY into three bf16 pieces by truncation (hi = the top 16 bits, mid = those of
// v - hi, lo = v - hi - mid, which fits 8 bits) and C += sum of the six largest piece products
// (hh, hm, mh, hl, mm, lh; the dropped ml, lm, ll are <= 2^-24 relative) on
// v_mfma_f32_16x16x32_bf16 with fp32 accumulation: 6 x 16 = 96 cycles per 32 rows against 8 x 32 =
// 256 for the fp32 16x16x4 form (2.67x the matrix rate), so the reduction becomes bound by the
// HBM stream of G and X.  No range limit (bf16 keeps fp32's exponent).  Same chunking, ring and
// write-back as wgrad_t16; a 32-row step takes rows 8 kq .. 8 kq + 7 of lane (m, kq) from LDS.
typedef short wg_bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned wg_u32x4 __attribute__((ext_vector_type(4)));
struct WgFrag3 {
  wg_bf16x8 h, m, l;
};
NAZ_DEV WgFrag3 wg_split8(const float (&v)[8]) {
  wg_u32x4 H, M, L;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned hb[2], mb[2], lb[2];
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const float x = v[2 * q + e];
      hb[e] = __float_as_uint(x);
      const float r1 = x - __uint_as_float(hb[e] & 0xffff0000u);
      mb[e] = __float_as_uint(r1);
      lb[e] = __float_as_uint(r1 - __uint_as_float(mb[e] & 0xffff0000u));
    }
    H[q] = __builtin_amdgcn_perm(hb[1], hb[0], 0x07060302u);
    M[q] = __builtin_amdgcn_perm(mb[1], mb[0], 0x07060302u);
    L[q] = __builtin_amdgcn_perm(lb[1], lb[0], 0x07060302u);
  }
  return WgFrag3{__builtin_bit_cast(wg_bf16x8, H), __builtin_bit_cast(wg_bf16x8, M), __builtin_bit_cast(wg_bf16x8, L)};
}
NAZ_DEV floatx4w wg_mfma6(const WgFrag3& a, const WgFrag3& b, floatx4w c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.l, b.h, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.l, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.m, b.h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.m, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.h, b.h, c, 0, 0, 0);
}

// ---------------------------------------------------------------------------------------------
// rowgemm_x6_kernel: the batch-row GEMM on the bf16 matrix pipe (naz_tuning "rowgemm_x6").  The same
// C = epi(A · B) as rowgemm_kernel, with every A and B value split EXACTLY into three bf16 pieces by
// truncation (wg_split8) and C += the six largest piece products on v_mfma_f32_32x32x16_bf16 (fp32
// accumulate; the dropped ml, lm, ll terms are <= 2^-24 relative, no range limit: fp32-grade at
// 2.67x the FP32 MFMA rate).  16-k chunks.  Wave w of the 128-row panel owns rows 32 w .. 32 w + 31
// and reads its A values straight into registers, one chunk ahead (lane (i, kh): row i, k 8 kh ..
// 8 kh + 7 of the chunk — the MFMA's A layout).  The workgroup splits each B chunk once into LDS in
// the MFMA's B layout ([32-column block][piece][lane][8 bf16], one 16-byte read per piece), double
// buffered, one barrier per chunk; the epilogue is rowgemm_kernel's.
NAZ_DEV floatx16 rg_mfma6(const WgFrag3& a, const WgFrag3& b, floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.l, b.h, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.l, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.m, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.m, b.h, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.m, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a.h, b.h, c, 0, 0, 0);
}

constexpr int RX_SHARE = 32 * (64 + 4);  // epilogue staging per wave (two 32-column blocks at a time)

template <int NB>
__global__ void __launch_bounds__(RG_T, NB <= 2 ? 4 : (NB <= 4 ? 3 : 2)) rowgemm_x6_kernel(RowGemmArgs p) {
  {  // problem of this z slice (uniform: stays in SGPRs)
    const int64_t z = blockIdx.z;
    p.a0 += z * p.za0;
    p.a1 += z * p.za1;
    p.b += z * p.zb;
    if (p.bias != nullptr) p.bias += z * p.zbias;
    p.c += z * p.zc;
  }
  constexpr int BN = 32 * NB;
  constexpr int BSLOT = NB * 3 * 64 * 4;  // u32 words of one B chunk: [NB][piece][64 lanes][4]
  constexpr int SMEM = 2 * BSLOT > 4 * RX_SHARE ? 2 * BSLOT : 4 * RX_SHARE;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  unsigned* const bsm = reinterpret_cast<unsigned*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kh = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * RG_BM;
  const int n0 = blockIdx.y * BN;
  const int K = p.ka0 + p.ka1;
  const int nk = (K + 15) / 16;
  const int64_t am = m0 + wave * 32 + (lane & 31);
  const bool arow = am < p.M;

  // A: this lane's 8 k values of the chunk (one segment: ka0 % 8 == 0 or the group inside one)
  auto load_a = [&](int kc, float (&v)[8]) {
    const int kb = 16 * kc + 8 * kh;
    if (p.vec && arow && kb + 8 <= K && (kb >= p.ka0 || kb + 8 <= p.ka0)) {
      const float* src = kb < p.ka0 ? p.a0 + am * p.lda0 + kb : p.a1 + am * p.lda1 + (kb - p.ka0);
      const float4 v0 = *reinterpret_cast<const float4*>(src);
      const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
      v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
      v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (arow && kb + e < K) ? rg_a(p, am, kb + e) : 0.f;
    }
  };
  // B: thread -> fragment fr = (column block fr >> 6, lane fr & 63: column lane & 31, k-half lane >> 5)
  const auto bsrd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.b), (short)0, 0x7fffffff, 0x00020000);
  const auto msrd =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.mask ? p.mask : p.b), (short)0, 0x7fffffff, 0x00020000);
  const int sbk = (int)p.sbk, sbn = (int)p.sbn, smk = (int)p.smk, smn = (int)p.smn;
  constexpr int FR = 64 * NB;  // B fragments per chunk
  constexpr int FPT = (FR + RG_T - 1) / RG_T;
  float rb[FPT][8];
  auto load_b = [&](int kc) {
#pragma unroll
    for (int f = 0; f < FPT; ++f) {
      const int fr = tid + RG_T * f, fl = fr & 63, n = n0 + 32 * (fr >> 6) + (fl & 31);
      const int kb = 16 * kc + 8 * (fl >> 5);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = 0.f;
        if (fr < FR && kb + e < K && n < p.N) {
          v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bsrd, 4 * ((kb + e) * sbk + n * sbn), 0, 0));
          if (p.mask != nullptr)
            v *= __builtin_bit_cast(float,
                                    __builtin_amdgcn_raw_buffer_load_b32(msrd, 4 * ((kb + e) * smk + n * smn), 0, 0));
        }
        rb[f][e] = v;
      }
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int f = 0; f < FPT; ++f) {
      const int fr = tid + RG_T * f;
      if (fr < FR) {
        const WgFrag3 q = wg_split8(rb[f]);
        wg_u32x4* d = reinterpret_cast<wg_u32x4*>(bsm + buf * BSLOT) + (fr >> 6) * 3 * 64 + (fr & 63);
        d[0] = __builtin_bit_cast(wg_u32x4, q.h);
        d[64] = __builtin_bit_cast(wg_u32x4, q.m);
        d[128] = __builtin_bit_cast(wg_u32x4, q.l);
      }
    }
  };

  floatx16 acc[NB];
#pragma unroll
  for (int o = 0; o < NB; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = 0.f;

  float va[8];
  load_a(0, va);
  load_b(0);
  store_b(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    float vn[8];
    if (kc + 1 < nk) {  // in flight during this chunk's MFMAs
      load_a(kc + 1, vn);
      load_b(kc + 1);
    }
    const WgFrag3 a = wg_split8(va);
    const wg_u32x4* bp = reinterpret_cast<const wg_u32x4*>(bsm + buf * BSLOT) + lane;
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const WgFrag3 b{__builtin_bit_cast(wg_bf16x8, bp[(o * 3 + 0) * 64]),
                      __builtin_bit_cast(wg_bf16x8, bp[(o * 3 + 1) * 64]),
                      __builtin_bit_cast(wg_bf16x8, bp[(o * 3 + 2) * 64])};
      acc[o] = rg_mfma6(a, b, acc[o]);
    }
    if (kc + 1 < nk) {
      store_b(buf ^ 1);
#pragma unroll
      for (int e = 0; e < 8; ++e) va[e] = vn[e];
    }
    __syncthreads();
  }
  rowgemm_epilogue<NB, RX_SHARE>(p, acc, smem, m0, n0, wave, lane);
}

template <int NB>
void rowgemm_x6_launch(const RowGemmArgs& p, int nz, hipStream_t s) {
  dim3 grid((unsigned)((p.M + RG_BM - 1) / RG_BM), (unsigned)((p.N + 32 * NB - 1) / (32 * NB)), (unsigned)nz);
  hipLaunchKernelGGL(rowgemm_x6_kernel<NB>, grid, dim3(RG_T), 0, s, p);
}

int rowgemm_x6_dispatch(const RowGemmArgs& p, int nz, int nb, hipStream_t s) {
  switch (nb > 8 ? 8 : nb) {
    case 1: rowgemm_x6_launch<1>(p, nz, s); break;
    case 2: rowgemm_x6_launch<2>(p, nz, s); break;
    case 3: rowgemm_x6_launch<3>(p, nz, s); break;
    case 4: rowgemm_x6_launch<4>(p, nz, s); break;
    case 5: rowgemm_x6_launch<5>(p, nz, s); break;
    case 6: rowgemm_x6_launch<6>(p, nz, s); break;
    case 7: rowgemm_x6_launch<7>(p, nz, s); break;
    default: rowgemm_x6_launch<8>(p, nz, s); break;
  }
  return check_launch("rowgemm_x6_kernel");
}

// ---------------------------------------------------------------------------------------------
// rowgemm_h3_kernel: the batch-row GEMM on the f16 matrix pipe (naz_tuning "rowgemm_h3").  The same
// C = epi(A · B) as rowgemm_kernel with A and B split into f16 hi / lo pieces (hi = f16(v), lo =
// f16(v - hi); v - hi is exact) and C += Ah·Bh + Ah·Bl + Al·Bh on v_mfma_f32_32x32x16_f16 — the
// fused kernels' f16x3 form (§4.1): 5.3x the FP32 MFMA rate per product set, the dropped Al·Bl term
// <= 2^-22 relative.  f16 has 5 exponent bits, so every A row is split at a power-of-two scale that
// puts its largest |value| in [2^13, 2^14) (a pre-pass over the wave's 32 rows; the lo pieces stay
// clear of f16's subnormals, the gradients' range is unbounded), and B at 2^6 (weights: the caller
// guarantees |B| < 2^9); the accumulators are unscaled exactly before the shared epilogue.  16-k
// chunks; a wave reads its A values straight into registers two chunks ahead; the workgroup splits
// each B chunk once into LDS in the MFMA's B layout ([block][piece][lane][8 f16]), double buffered.
typedef _Float16 rg_half8 __attribute__((ext_vector_type(8)));
typedef unsigned rg_u32x4 __attribute__((ext_vector_type(4)));
struct RgH2 {
  rg_half8 h, l;
};
constexpr float kRgH3BScale = 64.f;

NAZ_DEV RgH2 rg_split8_f16(const float (&v)[8], float sc) {
  RgH2 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float x = v[e] * sc;  // (a power of two: exact)
    const _Float16 hh = (_Float16)x;
    r.h[e] = hh;
    r.l[e] = (_Float16)(x - (float)hh);
  }
  return r;
}
NAZ_DEV floatx16 rg_mfma3(const RgH2& a, const RgH2& b, floatx16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.l, b.h, c, 0, 0, 0);  // small terms first
  c = __builtin_amdgcn_mfma_f32_32x32x16_f16(a.h, b.l, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a.h, b.h, c, 0, 0, 0);
}

template <int NB>
__global__ void __launch_bounds__(RG_T, NB <= 2 ? 4 : (NB <= 4 ? 3 : 2)) rowgemm_h3_kernel(RowGemmArgs p) {
  {  // problem of this z slice (uniform: stays in SGPRs)
    const int64_t z = blockIdx.z;
    p.a0 += z * p.za0;
    p.a1 += z * p.za1;
    p.b += z * p.zb;
    if (p.bias != nullptr) p.bias += z * p.zbias;
    p.c += z * p.zc;
  }
  constexpr int BSLOT = NB * 2 * 64 * 4;  // u32 words of one B chunk: [NB][piece][64 lanes][4]
  constexpr int SMEM = 2 * BSLOT > 4 * RX_SHARE ? 2 * BSLOT : 4 * RX_SHARE;
  __shared__ __attribute__((aligned(16))) float smem[SMEM];
  __shared__ float rinv[4][32];  // per row: 1 / (row scale x B scale)
  unsigned* const bsm = reinterpret_cast<unsigned*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kh = lane >> 5;
  const int64_t m0 = (int64_t)blockIdx.x * RG_BM;
  const int n0 = blockIdx.y * 32 * NB;
  const int K = p.ka0 + p.ka1;
  const int nk = (K + 15) / 16;
  const int64_t am = m0 + wave * 32 + (lane & 31);
  const bool arow = am < p.M;

  // A: this lane's 8 k values of the chunk (lane (row i, k-half kh): the MFMA's A layout)
  auto load_a = [&](int kc, float (&v)[8]) {
    const int kb = 16 * kc + 8 * kh;
    if (p.vec && arow && kb + 8 <= K && (kb >= p.ka0 || kb + 8 <= p.ka0)) {
      const float* src = kb < p.ka0 ? p.a0 + am * p.lda0 + kb : p.a1 + am * p.lda1 + (kb - p.ka0);
      const float4 v0 = *reinterpret_cast<const float4*>(src);
      const float4 v1 = *reinterpret_cast<const float4*>(src + 4);
      v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
      v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (arow && kb + e < K) ? rg_a(p, am, kb + e) : 0.f;
    }
  };
  // the row's scale: its largest |A| into [2^13, 2^14) (both lanes of a row agree); all-zero rows 1
  float sc;
  {
    float mx = 0.f;
    for (int kc = 0; kc < nk; ++kc) {
      float v[8];
      load_a(kc, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(v[e]));
    }
    mx = fmaxf(mx, __shfl_xor(mx, 32));
    int ex = mx > 0.f ? __builtin_amdgcn_frexp_expf(mx) : 14;  // mx < 2^ex (a non-finite row: 0)
    ex = ex < -100 ? -100 : ex;
    sc = __builtin_amdgcn_ldexpf(1.f, 14 - ex);
    if (kh == 0) rinv[wave][lane & 31] = __builtin_amdgcn_ldexpf(1.f, ex - 14) * (1.f / kRgH3BScale);
  }
  // B: thread -> fragment fr = (column block fr >> 6, lane fr & 63: column lane & 31, k-half lane >> 5)
  const auto bsrd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.b), (short)0, 0x7fffffff, 0x00020000);
  const auto msrd =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.mask ? p.mask : p.b), (short)0, 0x7fffffff, 0x00020000);
  const int sbk = (int)p.sbk, sbn = (int)p.sbn, smk = (int)p.smk, smn = (int)p.smn;
  constexpr int FR = 64 * NB;  // B fragments per chunk
  constexpr int FPT = (FR + RG_T - 1) / RG_T;
  float rb[FPT][8];
  auto load_b = [&](int kc) {
#pragma unroll
    for (int f = 0; f < FPT; ++f) {
      const int fr = tid + RG_T * f, fl = fr & 63, n = n0 + 32 * (fr >> 6) + (fl & 31);
      const int kb = 16 * kc + 8 * (fl >> 5);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = 0.f;
        if (fr < FR && kb + e < K && n < p.N) {
          v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bsrd, 4 * ((kb + e) * sbk + n * sbn), 0, 0));
          if (p.mask != nullptr)
            v *= __builtin_bit_cast(float,
                                    __builtin_amdgcn_raw_buffer_load_b32(msrd, 4 * ((kb + e) * smk + n * smn), 0, 0));
        }
        rb[f][e] = v;
      }
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int f = 0; f < FPT; ++f) {
      const int fr = tid + RG_T * f;
      if (fr < FR) {
        const RgH2 q = rg_split8_f16(rb[f], kRgH3BScale);
        rg_u32x4* d = reinterpret_cast<rg_u32x4*>(bsm + buf * BSLOT) + (fr >> 6) * 2 * 64 + (fr & 63);
        d[0] = __builtin_bit_cast(rg_u32x4, q.h);
        d[64] = __builtin_bit_cast(rg_u32x4, q.l);
      }
    }
  };

  floatx16 acc[NB];
#pragma unroll
  for (int o = 0; o < NB; ++o)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[o][r] = 0.f;

  float va[8], vb[8];
  load_a(0, va);
  if (nk > 1) load_a(1, vb);
  load_b(0);
  store_b(0);
  __syncthreads();
  for (int kc = 0; kc < nk; ++kc) {
    const int buf = kc & 1;
    float vc[8];
    if (kc + 2 < nk) load_a(kc + 2, vc);  // two chunks ahead: in flight during two chunks' MFMAs
    if (kc + 1 < nk) load_b(kc + 1);
    const RgH2 a = rg_split8_f16(va, sc);
    const rg_u32x4* bp = reinterpret_cast<const rg_u32x4*>(bsm + buf * BSLOT) + lane;
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const RgH2 b{__builtin_bit_cast(rg_half8, bp[(o * 2 + 0) * 64]), __builtin_bit_cast(rg_half8, bp[(o * 2 + 1) * 64])};
      acc[o] = rg_mfma3(a, b, acc[o]);
    }
    if (kc + 1 < nk) store_b(buf ^ 1);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      va[e] = vb[e];
      vb[e] = vc[e];
    }
    __syncthreads();
  }
  // unscale: accumulator register r of a block holds row (r & 3) + 8 (r >> 2) + 4 kh of the wave's 32
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float u = rinv[wave][(r & 3) + 8 * (r >> 2) + 4 * kh];
#pragma unroll
    for (int o = 0; o < NB; ++o) acc[o][r] *= u;
  }
  __syncthreads();  // (the epilogue stages through the B ring's LDS)
  rowgemm_epilogue<NB, RX_SHARE>(p, acc, smem, m0, n0, wave, lane);
}

template <int NB>
void rowgemm_h3_launch(const RowGemmArgs& p, int nz, hipStream_t s) {
  dim3 grid((unsigned)((p.M + RG_BM - 1) / RG_BM), (unsigned)((p.N + 32 * NB - 1) / (32 * NB)), (unsigned)nz);
  hipLaunchKernelGGL(rowgemm_h3_kernel<NB>, grid, dim3(RG_T), 0, s, p);
}

int rowgemm_h3_dispatch(const RowGemmArgs& p, int nz, int nb, hipStream_t s) {
  switch (nb > 8 ? 8 : nb) {
    case 1: rowgemm_h3_launch<1>(p, nz, s); break;
    case 2: rowgemm_h3_launch<2>(p, nz, s); break;
    case 3: rowgemm_h3_launch<3>(p, nz, s); break;
    case 4: rowgemm_h3_launch<4>(p, nz, s); break;
    case 5: rowgemm_h3_launch<5>(p, nz, s); break;
    case 6: rowgemm_h3_launch<6>(p, nz, s); break;
    case 7: rowgemm_h3_launch<7>(p, nz, s); break;
    default: rowgemm_h3_launch<8>(p, nz, s); break;
  }
  return check_launch("rowgemm_h3_kernel");
}

// rowgemm_bres_kernel: the batch-row GEMM on the f16 matrix pipe with the B panel RESIDENT in LDS
// (naz_tuning "rowgemm_bres").  rowgemm_h3 streamed and split every 16-k B chunk per 128-row
// workgroup behind a barrier: the B split cost as much VALU as the A split and the barrier held the
// waves in step (CNF training 94 vs 83 ms, r05).  Here a persistent workgroup owns one column panel
// of 32 NB columns for the whole call: it splits B (times its mask) ONCE into f16 hi / lo fragments
// in the MFMA's B layout ([k-step][block][piece][lane][8 f16], K x 32 NB x 4 bytes of LDS) at a
// power-of-two panel scale (its largest |B| into [2^13, 2^14)), then every wave walks 32-row tiles
// on its own — no barrier after the panel load.  Per tile: a pre-pass over the wave's A rows finds
// each row's power-of-two scale (the gradients' range is unbounded; f16's lo pieces must stay clear
// of subnormals), then C += Ah·Bh + Ah·Bl + Al·Bh on v_mfma_f32_32x32x16_f16 (the dropped Al·Bl
// term <= 2^-22 relative) with A read straight into registers two k-steps ahead, and the
// accumulators unscaled exactly in a register epilogue (bias, activation, chained act', accumulate;
// the CNF pair VJP stays on the other kernels).  Panels of one row range are mapped to one XCD
// (workgroup w runs on XCD w mod 8), so their A rows are fetched into one L2.
// KSR > 0: K <= 16 KSR, and a wave's whole 32-row A tile is loaded into registers at once (all loads in
// flight together; the row maxima from those registers: A is read once), for the CNF's 128-wide layers
template <int NB, int KSR>
__global__ void __launch_bounds__(256, (NB <= 3 && KSR == 0) ? 4 : 2) rowgemm_bres_kernel(RowGemmArgs p, int npanels,
                                                                                         int per_panel) {
  extern __shared__ __attribute__((aligned(16))) float bres_lds[];
  __shared__ unsigned bmax_bits;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, kh = lane >> 5;
  const int K = p.ka0 + p.ka1, KSP = (K + 15) / 16;
  // workgroup -> (panel, slot): the npanels workgroups sharing a slot sit on one XCD (w mod 8 = XCD)
  const int w = blockIdx.x;
  const int xcd = w & 7, wq = w >> 3;
  const int panel = wq % npanels, slot = (wq / npanels) * 8 + xcd;
  const int nslots = per_panel;
  if (slot >= nslots) return;  // (the grid is rounded to whole XCD groups)
  const int n0 = panel * 32 * NB;
  unsigned* const bsm = reinterpret_cast<unsigned*>(bres_lds);

  // ---- the panel's B: max |B|, then the split fragments
  const auto bsrd = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.b), (short)0, p.bbytes, 0x00020000);
  const auto msrd =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p.mask ? p.mask : p.b), (short)0, p.mbytes, 0x00020000);
  const int sbk = (int)p.sbk, sbn = (int)p.sbn, smk = (int)p.smk, smn = (int)p.smn;
  auto bval = [&](int k, int n) -> float {
    const bool in = k < K && n < p.N;
    float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(bsrd, in ? 4 * (k * sbk + n * sbn) : p.bbytes, 0, 0));
    if (p.mask != nullptr)
      v *= __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(msrd, in ? 4 * (k * smk + n * smn) : p.mbytes, 0, 0));
    return v;
  };
  if (tid == 0) bmax_bits = 0u;
  __syncthreads();
  const int nfl = KSP * NB * 64;  // fragment lanes: (k-step t, block o, lane l)
  {
    float mx = 0.f;
    for (int fl = tid; fl < nfl; fl += 256) {
      const int l = fl & 63, o = (fl >> 6) % NB, t = (fl >> 6) / NB;
      const int kb = 16 * t + 8 * (l >> 5), n = n0 + 32 * o + (l & 31);
#pragma unroll
      for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(bval(kb + e, n)));
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) mx = fmaxf(mx, __shfl_xor(mx, d));
    if (lane == 0) atomicMax(&bmax_bits, __float_as_uint(mx));  // |B| >= 0: the bits order as the values
  }
  __syncthreads();
  const float bmx = __uint_as_float(bmax_bits);
  int bex = bmx > 0.f ? __builtin_amdgcn_frexp_expf(bmx) : 14;
  bex = bex < -100 ? -100 : (bex > 100 ? 100 : bex);
  const float bsc = __builtin_amdgcn_ldexpf(1.f, 14 - bex);
  for (int fl = tid; fl < nfl; fl += 256) {
    const int l = fl & 63, fo = fl >> 6;  // fo = t NB + o
    const int o = fo % NB, t = fo / NB;
    const int kb = 16 * t + 8 * (l >> 5), n = n0 + 32 * o + (l & 31);
    float v[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = bval(kb + e, n);
    const RgH2 q = rg_split8_f16(v, bsc);
    rg_u32x4* d = reinterpret_cast<rg_u32x4*>(bsm) + (fo * 2) * 64 + l;
    d[0] = __builtin_bit_cast(rg_u32x4, q.h);
    d[64] = __builtin_bit_cast(rg_u32x4, q.l);
  }
  __syncthreads();
  const float binv = __builtin_amdgcn_ldexpf(1.f, bex - 14);

  // ---- 32-row tiles: wave (slot, wave) takes tiles slot 4 + wave, + 4 nslots, ...
  const int64_t ntiles = (p.M + 31) / 32;
  const rg_u32x4* bfr = reinterpret_cast<const rg_u32x4*>(bsm) + lane;
  for (int64_t tile = (int64_t)slot * 4 + wave; tile < ntiles; tile += (int64_t)nslots * 4) {
    const int64_t am = tile * 32 + (lane & 31);
    const bool arow = am < p.M;
    // (p.vec: 16-byte aligned rows, ka0 % 8 == 0, so an 8-k group never straddles the two segments)
    const float* const row0 = p.a0 + (arow ? am : 0) * p.lda0;
    const float* const row1 = p.a1 + (arow ? am : 0) * p.lda1;
    auto load_a = [&](int t, float (&v)[8]) {
      const int kb = 16 * t + 8 * kh;
      const bool s0 = kb < p.ka0;
      const float* seg = s0 ? row0 + kb : row1 + (kb - p.ka0);
      const int lim = arow ? (s0 ? p.ka0 - kb : K - kb) : 0;  // valid k of this group
      if (lim >= 8) {
        const float4 v0 = *reinterpret_cast<const float4*>(seg);
        const float4 v1 = *reinterpret_cast<const float4*>(seg + 4);
        v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w;
        v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = e < lim ? seg[e] : 0.f;
      }
    };
    // the row's scale (both lanes of a row agree): its largest |A| into [2^13, 2^14); zero rows 1
    float sc, rinv;
    auto row_scale = [&](float mx) {
      mx = fmaxf(mx, __shfl_xor(mx, 32));
      int ex = mx > 0.f ? __builtin_amdgcn_frexp_expf(mx) : 14;  // mx < 2^ex (a non-finite row: 0)
      ex = ex < -100 ? -100 : ex;
      sc = __builtin_amdgcn_ldexpf(1.f, 14 - ex);
      rinv = __builtin_amdgcn_ldexpf(1.f, ex - 14) * binv;
    };
    floatx16 acc[NB];
#pragma unroll
    for (int o = 0; o < NB; ++o)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[o][r] = 0.f;
    if constexpr (KSR > 0) {
      float areg[KSR][8];
      if (p.ka1 == 0 && K == 16 * KSR && arow) {  // one segment of exactly KSR k-steps: plain 16-byte loads
#pragma unroll
        for (int t = 0; t < KSR; ++t) {
          const float4 v0 = *reinterpret_cast<const float4*>(row0 + 16 * t + 8 * kh);
          const float4 v1 = *reinterpret_cast<const float4*>(row0 + 16 * t + 8 * kh + 4);
          areg[t][0] = v0.x; areg[t][1] = v0.y; areg[t][2] = v0.z; areg[t][3] = v0.w;
          areg[t][4] = v1.x; areg[t][5] = v1.y; areg[t][6] = v1.z; areg[t][7] = v1.w;
        }
      } else {
#pragma unroll
        for (int t = 0; t < KSR; ++t) load_a(t, areg[t]);
      }
      float mx = 0.f;
#pragma unroll
      for (int t = 0; t < KSR; ++t)
#pragma unroll
        for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(areg[t][e]));
      row_scale(mx);
#pragma unroll
      for (int t = 0; t < KSR; ++t) {
        const RgH2 a = rg_split8_f16(areg[t], sc);
#pragma unroll
        for (int o = 0; o < NB; ++o) {
          const int f = (t * NB + o) * 2 * 64;
          const RgH2 b{__builtin_bit_cast(rg_half8, bfr[f]), __builtin_bit_cast(rg_half8, bfr[f + 64])};
          acc[o] = rg_mfma3(a, b, acc[o]);
        }
      }
    } else {
      {
        float mx = 0.f;
        for (int t = 0; t < KSP; ++t) {
          float v[8];
          load_a(t, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) mx = fmaxf(mx, fabsf(v[e]));
        }
        row_scale(mx);
      }
      float va[8], vb[8];
      load_a(0, va);
      if (KSP > 1) load_a(1, vb);
      for (int t = 0; t < KSP; ++t) {
        float vc[8];
        if (t + 2 < KSP) load_a(t + 2, vc);  // two k-steps ahead
        const RgH2 a = rg_split8_f16(va, sc);
#pragma unroll
        for (int o = 0; o < NB; ++o) {
          const int f = (t * NB + o) * 2 * 64;
          const RgH2 b{__builtin_bit_cast(rg_half8, bfr[f]), __builtin_bit_cast(rg_half8, bfr[f + 64])};
          acc[o] = rg_mfma3(a, b, acc[o]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          va[e] = vb[e];
          vb[e] = vc[e];
        }
      }
    }
    // register epilogue: accumulator register r of a block = row (r & 3) + 8 (r >> 2) + 4 kh of the tile
    // (its scale from the lane that loaded that row), column 32 o + (lane & 31) of the panel.  Rows are
    // addressed by 32-bit offsets from the tile's first row (a wave-uniform base: SGPRs), so the
    // unrolled stores do not each hold a 64-bit address
    const int64_t tb = (int64_t)__builtin_amdgcn_readfirstlane((int)(tile >> 5)) * 1024 +
                       __builtin_amdgcn_readfirstlane((int)(tile & 31)) * 32;
    float* const cb = p.c + tb * p.ldc;
    const float* const dyb = p.dy != nullptr ? p.dy + tb * p.lddy : nullptr;
    // (the row offsets below are the same for every tile: made opaque per tile, or the compiler hoists
    // all 16 of them out of the tile loop as 64-bit values and spills)
    int ldc = (int)p.ldc, lddy = (int)p.lddy, lc = lane & 31, kh4 = 4 * kh;
    asm volatile("" : "+v"(lc), "+v"(kh4), "+s"(ldc), "+s"(lddy));
    float bn[NB];
#pragma unroll
    for (int o = 0; o < NB; ++o) {
      const int n = n0 + 32 * o + (lane & 31);
      bn[o] = (p.bias != nullptr && n < p.N) ? p.bias[n] : 0.f;
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rr = (r & 3) + 8 * (r >> 2) + kh4;
      const float u = __shfl(rinv, rr);
      if (tb + rr >= p.M) continue;
#pragma unroll
      for (int o = 0; o < NB; ++o) {
        const int n = n0 + 32 * o + lc;
        if (n >= p.N) continue;
        float v = activate_rt(p.act, acc[o][r] * u + bn[o]);
        if (dyb != nullptr) v *= activate_grad_from_out(p.dact, dyb[(uint32_t)(rr * lddy + n)]);
        float* dst = cb + (uint32_t)(rr * ldc + n);
        *dst = p.accumulate ? *dst + v : v;
      }
    }
  }
}

// LDS bytes of a B-resident panel of NB blocks over K
static int64_t bres_lds_bytes(int K, int nb) { return (int64_t)((K + 15) / 16) * nb * 2048; }

template <int NB, int KSR>
int rowgemm_bres_launch(const RowGemmArgs& p, hipStream_t s) {
  const int npanels = (p.N + 32 * NB - 1) / (32 * NB);
  const int64_t lds = bres_lds_bytes(p.ka0 + p.ka1, NB);
  const int per_cu = (int)std::min<int64_t>(4, (160 * 1024) / (lds + 64));
  const int64_t ntiles = (p.M + 31) / 32;
  // slots per panel: enough workgroups to hold per_cu per CU, no more than the tiles need, whole XCD groups
  int64_t slots = std::max<int64_t>(1, (int64_t)per_cu * device_cus() / npanels);
  slots = std::min<int64_t>(slots, (ntiles + 3) / 4);
  slots = (slots + 7) / 8 * 8;
  const int64_t grid = slots / 8 * npanels * 8;
  hipLaunchKernelGGL((rowgemm_bres_kernel<NB, KSR>), dim3((unsigned)grid), dim3(256), (size_t)lds, s, p, npanels,
                     (int)slots);
  return check_launch("rowgemm_bres_kernel");
}

// the B-resident form applies: one problem, no CNF pair VJP, a panel of >= 2 blocks (or the whole
// output) fits the LDS.  Returns the blocks per panel, or 0.
int rowgemm_bres_nb(const RowGemmArgs& p, int nz) {
  if (nz != 1 || p.jvp != nullptr || p.M < 1024 || !p.vec) return 0;
  if (p.ldc * 32 + p.N >= (1ll << 31) || (p.dy != nullptr && p.lddy * 32 + p.N >= (1ll << 31))) return 0;
  const int K = p.ka0 + p.ka1, nball = (p.N + 31) / 32;
  for (int nb = 4; nb >= 1; --nb) {
    if (bres_lds_bytes(K, nb) > 144 * 1024) continue;
    if (nb >= 2 || nball == 1) {
      const int panels = (nball + nb - 1) / nb;
      return (nball + panels - 1) / panels;  // balanced panels
    }
  }
  return 0;
}

int rowgemm_bres_dispatch(const RowGemmArgs& p, int nb, hipStream_t s) {
  if (p.ka0 + p.ka1 <= 128) {  // the whole A tile in registers
    switch (nb) {
      case 1: return rowgemm_bres_launch<1, 8>(p, s);
      case 2: return rowgemm_bres_launch<2, 8>(p, s);
      case 3: return rowgemm_bres_launch<3, 8>(p, s);
      default: return rowgemm_bres_launch<4, 8>(p, s);
    }
  }
  switch (nb) {
    case 1: return rowgemm_bres_launch<1, 0>(p, s);
    case 2: return rowgemm_bres_launch<2, 0>(p, s);
    case 3: return rowgemm_bres_launch<3, 0>(p, s);
    default: return rowgemm_bres_launch<4, 0>(p, s);
  }
}

template <int NOW, int NB2, int JS>
__global__ void __launch_bounds__(256 * JS, 2 / JS) wgrad_x6_kernel(WGradArgs p, int R) {
  extern __shared__ float tl[];
  constexpr int NT = 256 * JS, NBW = NB2 / JS;
  const int tid = threadIdx.x, lane = tid & 63, wave = (tid >> 6) & 3, jh = tid >> 8, m = lane & 15,
            kq = lane >> 4;
  const int N1 = p.N1, N2 = p.N2;
  {
    const int64_t bz = blockIdx.y;
    p.g += bz * p.bg;
    p.x += bz * p.bx;
    p.c += bz * p.bc;
    if (p.rowsum != nullptr) p.rowsum += bz * p.br;
  }
  // rows: the contiguous block [mb, me) in steps of R, or (chunk_stride > 0) the chunks mb, mb +
  // chunk_stride, ... of all M rows: the grid's concurrently streamed chunks then lie side by side
  // in HBM instead of rows_per_wg apart
  const bool il = p.chunk_stride > 0;
  const int64_t mb = (int64_t)blockIdx.x * (il ? R : p.rows_per_wg);
  const int64_t me = il ? p.M : ((mb + p.rows_per_wg) < p.M ? (mb + p.rows_per_wg) : p.M);
  const int64_t step = il ? p.chunk_stride : R;
  floatx4w acc[NOW][NBW];
#pragma unroll
  for (int i = 0; i < NOW; ++i)
#pragma unroll
    for (int j = 0; j < NBW; ++j) acc[i][j] = floatx4w{0.f, 0.f, 0.f, 0.f};
  float dsum[NOW];
#pragma unroll
  for (int i = 0; i < NOW; ++i) dsum[i] = 0.f;
  const int CH = R * (N1 + N2);
  const int nw = NT / 64, wv = tid >> 6;
  auto issue = [&](int64_t m0, float* dst) {
    const float* src[2] = {p.g + m0 * N1, p.x + m0 * N2};
    const int cnt[2] = {R * N1 / 256, R * N2 / 256};
    float* d = dst;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      for (int c = wv; c < cnt[h]; c += nw)
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src[h] + c * 256 + lane * 4),
                                         (void __attribute__((address_space(3)))*)(uint32_t)(uintptr_t)(d + c * 256), 16, 0, 0);
      d += R * (h == 0 ? N1 : N2);
    }
  };
  auto copy_tail = [&](int64_t m0, float* dst) {  // zero-filled past me: padding rows add nothing
    const int64_t rows = me - m0;
    const int lg = (int)(rows * N1 / 4), lx = (int)(rows * N2 / 4), fg = R * N1 / 4;
    const float4* gp = reinterpret_cast<const float4*>(p.g + m0 * N1);
    const float4* xp = reinterpret_cast<const float4*>(p.x + m0 * N2);
    float4* l4 = reinterpret_cast<float4*>(dst);
    for (int q = tid; q < CH / 4; q += NT) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < fg) {
        if (q < lg) v = gp[q];
      } else if (q - fg < lx) {
        v = xp[q - fg];
      }
      l4[q] = v;
    }
  };
  auto fill = [&](int64_t m0, float* dst) {
    if (m0 + R <= me) issue(m0, dst);
    else copy_tail(m0, dst);
  };
  int slot = 0;
  if (mb < me) fill(mb, tl);
  for (int64_t m0 = mb; m0 < me; m0 += step, slot ^= 1) {
    ring_barrier();  // chunk m0 has landed; every wave is done with the other slot
    const float* const Gs = tl + slot * CH;
    const float* const Xs = Gs + R * N1;
    if (m0 + step < me) fill(m0 + step, tl + (slot ^ 1) * CH);
    // lane (m, kq) of a 32-row step reads rows 8 kq .. 8 kq + 7; past-the-end blocks read LDS
    // slack / neighbours and only feed dropped accumulator rows or columns (as wgrad_t16)
    const float* pa = Gs + (8 * kq) * N1 + wave * 16 + m;
    const float* pb = Xs + (8 * kq) * N2 + jh * NBW * 16 + m;
    for (int st = 0; st < R / 32; ++st) {
      WgFrag3 fa[NOW], fb[NBW];
#pragma unroll
      for (int i = 0; i < NOW; ++i) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = pa[j * N1 + 64 * i];
#pragma unroll
        for (int j = 0; j < 8; ++j) dsum[i] += v[j];
        fa[i] = wg_split8(v);
      }
#pragma unroll
      for (int jb = 0; jb < NBW; ++jb) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = pb[j * N2 + 16 * jb];
        fb[jb] = wg_split8(v);
      }
      pa += 32 * N1;
      pb += 32 * N2;
#pragma unroll
      for (int i = 0; i < NOW; ++i)
#pragma unroll
        for (int jb = 0; jb < NBW; ++jb) acc[i][jb] = wg_mfma6(fa[i], fb[jb], acc[i][jb]);
    }
  }
#pragma unroll
  for (int i = 0; i < NOW; ++i) {
    const int ob = wave + 4 * i;
#pragma unroll
    for (int j = 0; j < NBW; ++j) {
      const int n2 = 16 * (jh * NBW + j) + m;
      if (n2 >= N2) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n1 = 16 * ob + 4 * kq + r;
        if (n1 >= N1) continue;
        float v = acc[i][j][r];
        if (p.mask != nullptr) v *= p.mask[(int64_t)n1 * p.smm + (int64_t)n2 * p.smn];
        atomicAdd(p.c + (int64_t)n1 * p.scm + (int64_t)n2 * p.scn, v);
      }
    }
    if (p.ones && jh == 0) {  // db: lane (m, kq) summed rows 8 kq .. of column 16 ob + m
      float v = dsum[i];
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      const int o = 16 * ob + m;
      if (kq == 0 && o < N1) atomicAdd(p.rowsum + o, v);
    }
  }
}

template <int NOW, int NB2>
static void wgrad_x6_go(const WGradArgs& q, int R, size_t lds, dim3 grid, hipStream_t s, bool js2) {
  if constexpr (NOW * NB2 > 12 && NB2 % 2 == 0) {
    if (js2) {
      hipLaunchKernelGGL((wgrad_x6_kernel<NOW, NB2, 2>), grid, dim3(512), lds, s, q, R);
      return;
    }
  }
  hipLaunchKernelGGL((wgrad_x6_kernel<NOW, NB2, 1>), grid, dim3(256), lds, s, q, R);
}

template <int NOW>
static bool wgrad_x6_launch(int nb2, const WGradArgs& q, int R, size_t lds, dim3 grid, hipStream_t s, bool js2) {
  switch (nb2) {
    case 1: wgrad_x6_go<NOW, 1>(q, R, lds, grid, s, js2); return true;
    case 2: wgrad_x6_go<NOW, 2>(q, R, lds, grid, s, js2); return true;
    case 3: wgrad_x6_go<NOW, 3>(q, R, lds, grid, s, js2); return true;
    case 4: wgrad_x6_go<NOW, 4>(q, R, lds, grid, s, js2); return true;
    case 6: wgrad_x6_go<NOW, 6>(q, R, lds, grid, s, js2); return true;
    case 8: wgrad_x6_go<NOW, 8>(q, R, lds, grid, s, js2); return true;
    case 10: wgrad_x6_go<NOW, 10>(q, R, lds, grid, s, js2); return true;
    default: return false;
  }
}

static bool wgrad_x6_interleave() {
  static const bool on = [] {
    const char* e = getenv("NAZ_WGRAD_INTERLEAVE");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

// wgrad on the bf16x6 kernel for the shapes wgrad_t16 takes (R a multiple of 32 here), plus
// N2 <= 160 (the maf's 150-wide layers); nbatch independent reductions (blockIdx.y)
static bool wgrad_x6(WGradArgs p, hipStream_t s, int nbatch = 1) {
  const int nb1 = (p.N1 + 15) / 16, now = (nb1 + 3) / 4;
  int nb2 = (p.N2 + 15) / 16;
  nb2 = nb2 <= 4 ? nb2 : (nb2 <= 6 ? 6 : (nb2 <= 8 ? 8 : (nb2 <= 10 ? 10 : 0)));
  if (now < 1 || now > 4 || nb2 == 0) return false;
  // 4-wave workgroups, two per CU (two DMA rings in flight per CU: one 8-wave workgroup with a
  // single ring streamed G + X at ~3.7 TB/s) when two rings of 32-row chunks fit the LDS; else one
  // 8-wave workgroup per CU (the wide 192 x 128 reduction)
  auto lds_of = [&](int r) {  // + slack for the unmasked past-the-end reads
    return ((size_t)2 * r * (p.N1 + p.N2) + 16 * p.N2 + 16 * nb2 + 64 * nb1 + 64) * 4;
  };
  const bool whole = (32 * p.N1) % 256 == 0 && (32 * p.N2) % 256 == 0;
  if (!whole) return false;
  bool js2 = 2 * lds_of(32) > 160 * 1024;
  if (js2 && !(now * nb2 > 12 && nb2 % 2 == 0)) return false;
  int R = 32;
  for (int r = 64; r <= 128; r += 32)
    if ((r * p.N1) % 256 == 0 && (r * p.N2) % 256 == 0 && lds_of(r) * (js2 ? 1 : 2) <= 160 * 1024) R = r;
  if (lds_of(R) * (js2 ? 1 : 2) > 160 * 1024) return false;
  const size_t lds = lds_of(R);
  // two rounds of resident workgroups (one per CU for 8-wave ones, two per CU for 4-wave ones)
  // over all nbatch reductions
  const int64_t slots = js2 ? 512 : 1024;
  int64_t rpw = (p.M * nbatch + slots - 1) / slots;
  rpw = (rpw + R - 1) / R * R;
  if (rpw < 4 * R) rpw = 4 * R;
  p.rows_per_wg = rpw;
  const dim3 grid((unsigned)((p.M + rpw - 1) / rpw), (unsigned)nbatch);
  p.chunk_stride = wgrad_x6_interleave() ? (int64_t)grid.x * R : 0;
  switch (now) {
    case 1: return wgrad_x6_launch<1>(nb2, p, R, lds, grid, s, js2);
    case 2: return wgrad_x6_launch<2>(nb2, p, R, lds, grid, s, js2);
    case 3: return wgrad_x6_launch<3>(nb2, p, R, lds, grid, s, js2);
    default: return wgrad_x6_launch<4>(nb2, p, R, lds, grid, s, js2);
  }
}

static bool wgrad_x6_enabled() {
  static const bool on = [] {
    const char* e = getenv("NAZ_WGRAD_X6");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

__global__ void zero2d_kernel(float* c, int64_t scm, int64_t scn, int M, int N) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)M * N) return;
  const int m = (int)(e / N), n = (int)(e - (int64_t)m * N);
  c[m * scm + n * scn] = 0.f;
}

static bool wgrad_t16_enabled() {
  static const bool on = [] {
    const char* e = getenv("NAZ_WGRAD_T16");
    return e == nullptr || e[0] != '0';
  }();
  return on;
}

int wgrad(WGradArgs p, int accumulate, hipStream_t s) {
  if (p.N1 <= 0 || (p.N2 <= 0 && !p.ones)) return 0;
  if (!accumulate) {
    if (p.N2 > 0) {
      const int64_t n = (int64_t)p.N1 * p.N2;
      hipLaunchKernelGGL(zero2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p.c, p.scm, p.scn, p.N1,
                         p.N2);
    }
    // the db vector zeroed by a kernel too: a hipMemsetAsync captured into a HIP graph was measured
    // to leave stale sums on replay (tests/test_bayes_maf.py, fused maf gradient)
    if (p.ones) hipLaunchKernelGGL(zero2d_kernel, dim3((unsigned)((p.N1 + 255) / 256)), dim3(256), 0, s, p.rowsum,
                                   (int64_t)1, (int64_t)0, p.N1, 1);
  }
  if (p.M <= 0) return check_launch("zero2d_kernel");
  const bool flat = p.sgm == p.N1 && p.sxm == p.N2 && p.N1 % 4 == 0 && p.N2 % 4 == 0 && p.N2 > 0 &&
                    (reinterpret_cast<uintptr_t>(p.g) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.x) & 15) == 0 &&
                    p.N1 <= 256 && p.N2 <= 256;
  if (flat && p.N2 <= 160 && wgrad_x6_enabled() && wgrad_x6(p, s)) return check_launch("wgrad_x6_kernel");
  if (flat && p.N2 <= 128 && wgrad_t16_enabled() && wgrad_t16(p, s)) return check_launch("wgrad_t16_kernel");
  if (flat) {
    // rows per chunk: ~8192 floats of G + X (a multiple of 16, <= 128); ~1024 workgroups
    int R = 1024 * WF_Q / (p.N1 + p.N2);
    R = R > 128 ? 128 : (R / 16) * 16;
    if (R < 16) R = 16;
    while (R * (p.N1 + p.N2) / 4 > 256 * WF_Q) R -= 16;
    int64_t rpw = (p.M + 1023) / 1024;
    rpw = (rpw + R - 1) / R * R;
    if (rpw < 4 * R) rpw = 4 * R;
    p.rows_per_wg = rpw;
    const int nblk = ((p.N1 + 31) / 32) * ((p.N2 + 31) / 32);
    const int per_wave = (nblk + 3) / 4;  // blocks per wave (4 waves): no idle MFMA slots for nblk % 4 == 0
    const int maxb = per_wave <= 1 ? 1 : per_wave <= 2 ? 2 : per_wave <= 3 ? 3 : per_wave <= 4 ? 4
                   : per_wave <= 6 ? 6 : 8;
    const size_t lds = sizeof(float) * (R * (p.N1 + p.N2) + 64);
    const unsigned gx = (unsigned)((p.M + rpw - 1) / rpw);
    for (int b0 = 0; b0 < nblk; b0 += 4 * maxb) {
      p.blk0 = b0;
      WGradArgs q = p;
      if (b0 > 0) q.ones = 0;  // db once
      switch (maxb) {
        case 1: hipLaunchKernelGGL(wgrad_flat_kernel<1>, dim3(gx), dim3(256), lds, s, q, R); break;
        case 2: hipLaunchKernelGGL(wgrad_flat_kernel<2>, dim3(gx), dim3(256), lds, s, q, R); break;
        case 3: hipLaunchKernelGGL(wgrad_flat_kernel<3>, dim3(gx), dim3(256), lds, s, q, R); break;
        case 4: hipLaunchKernelGGL(wgrad_flat_kernel<4>, dim3(gx), dim3(256), lds, s, q, R); break;
        case 6: hipLaunchKernelGGL(wgrad_flat_kernel<6>, dim3(gx), dim3(256), lds, s, q, R); break;
        default: hipLaunchKernelGGL(wgrad_flat_kernel<8>, dim3(gx), dim3(256), lds, s, q, R); break;
      }
    }
    return check_launch("wgrad_flat_kernel");
  }
  // enough workgroups to fill the chip twice over, each reducing a multiple of 16 rows
  int64_t rpw = (p.M + 1023) / 1024;
  rpw = (rpw + WG_BK - 1) / WG_BK * WG_BK;
  if (rpw < 256) rpw = 256;
  p.rows_per_wg = rpw;
  const int NB1 = (p.N1 + 31) / 32, NB2 = (p.N2 + p.ones + 31) / 32;
  const int nblk = NB1 * NB2, per = 4 * WG_MAXB;
  const unsigned gx = (unsigned)((p.M + rpw - 1) / rpw);
  for (int b0 = 0; b0 < nblk; b0 += per) {  // output-block slices of 16 (one grid each)
    p.blk0 = b0;
    hipLaunchKernelGGL(wgrad_kernel, dim3(gx), dim3(256), 0, s, p);
  }
  return check_launch("wgrad_kernel");
}

// nbatch independent dW-type reductions C[b] += G[b]ᵀ X[b] (+ rowsum[b] += column sums of G[b]) in
// ONE bf16x6 launch (blockIdx.y = b): the maf backward's per-layer dW over all layers at once.
// Row-major G [M, N1] / X [M, N2] with unit column stride, 16-byte aligned, C unit column stride.
int wgrad_batched_impl(int64_t M, int N1, int N2, int nbatch, const float* g, int64_t sgm, int64_t bg,
                       const float* x, int64_t sxm, int64_t bx, float* c, int64_t scm, int64_t bc, float* rowsum,
                       int64_t br, hipStream_t s) {
  if (M < 0 || N1 <= 0 || N2 <= 0 || nbatch < 0) return set_error("naz_wgrad_batched: bad shape");
  if (M == 0 || nbatch == 0) return 0;
  if (nbatch > 65535) return set_error("naz_wgrad_batched: at most 65535 reductions per call");
  WGradArgs p{};
  p.g = g;
  p.sgm = sgm;
  p.x = x;
  p.sxm = sxm;
  p.M = M;
  p.N1 = N1;
  p.N2 = N2;
  p.ones = rowsum != nullptr;
  p.c = c;
  p.scm = scm;
  p.scn = 1;
  p.rowsum = rowsum;
  p.bg = bg;
  p.bx = bx;
  p.bc = bc;
  p.br = br;
  const bool aligned = (reinterpret_cast<uintptr_t>(g) & 15) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                       bg % 4 == 0 && bx % 4 == 0;
  if (!(sgm == N1 && sxm == N2 && N1 % 4 == 0 && N2 % 4 == 0 && N1 <= 256 && N2 <= 160 && aligned))
    return set_error("naz_wgrad_batched: operands must be contiguous, 16-byte aligned rows of N1, N2 <= 160 (N %% 4 == 0)");
  if (!wgrad_x6(p, s, nbatch)) return set_error("naz_wgrad_batched: no bf16x6 instance for N1=%d N2=%d", N1, N2);
  return check_launch("wgrad_x6_kernel (batched)");
}

}  // namespace

int wgrad_batched(int64_t M, int N1, int N2, int nbatch, const float* g, int64_t sgm, int64_t bg, const float* x,
                  int64_t sxm, int64_t bx, float* c, int64_t scm, int64_t bc, float* rowsum, int64_t br,
                  hipStream_t s) {
  return wgrad_batched_impl(M, N1, N2, nbatch, g, sgm, bg, x, sxm, bx, c, scm, bc, rowsum, br, s);
}

// ------------------------------------------------------------------------------------------
// Entry points used by dense.hip / gemm.hip
// ------------------------------------------------------------------------------------------
int rowgemm_linear(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
                   const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act,
                   hipStream_t s) {
  RowGemmArgs p{};
  p.a0 = ctx;
  p.lda0 = ldc;
  p.ka0 = C;
  p.a1 = x;
  p.lda1 = ldx;
  p.ka1 = Kx;
  p.b = W;  // B(k, n) = W[n, k]
  p.sbk = 1;
  p.sbn = C + Kx;
  p.mask = mask;
  p.smk = 1;
  p.smn = C + Kx;
  p.bias = b;
  p.c = y;
  p.ldc = ldy;
  p.M = M;
  p.N = N;
  p.act = act;
  p.accumulate = 0;
  return rowgemm(p, s);
}

// naz_linear_act_batched: nz problems with their own weights / bias over their own row blocks
int rowgemm_linear_batched(const float* ctx, int64_t ldc, int64_t zc, int C, const float* x, int64_t ldx, int64_t zx,
                           int Kx, const float* W, int64_t zw, const float* mask, const float* b, int64_t zb,
                           float* y, int64_t ldy, int64_t zy, int64_t M, int N, int nz, int act, hipStream_t s) {
  RowGemmArgs p{};
  p.a0 = ctx;
  p.lda0 = ldc;
  p.ka0 = C;
  p.za0 = zc;
  p.a1 = x;
  p.lda1 = ldx;
  p.ka1 = Kx;
  p.za1 = zx;
  p.b = W;
  p.sbk = 1;
  p.sbn = C + Kx;
  p.zb = zw;
  p.mask = mask;
  p.smk = 1;
  p.smn = C + Kx;
  p.bias = b;
  p.zbias = zb;
  p.c = y;
  p.ldc = ldy;
  p.zc = zy;
  p.M = M;
  p.N = N;
  p.act = act;
  p.accumulate = 0;
  return rowgemm(p, s, nz);
}

// naz_gemm_dact: C[m, n] = (Σ_k A[m, k] W[k, n] mask[k, n]) · act'(dy[m, n])   (A rows at lda)
int rowgemm_dact(const float* A, int64_t lda, int K, const float* W, int64_t ldw, const float* mask, int64_t ldm,
                 float* C, int64_t ldc, const float* dy, int64_t lddy, int dact, int64_t M, int N, hipStream_t s) {
  // the act' factor is applied in the 16-byte row-piece epilogue only (in the per-element one it
  // pushed the accumulators to scratch): C rows must allow it
  if (ldc % 4 != 0 || (reinterpret_cast<uintptr_t>(C) & 15) != 0)
    return set_error("naz_gemm_dact: C needs 16-byte aligned rows (ldc %% 4 == 0)");
  RowGemmArgs p{};
  p.a1 = A;
  p.lda1 = lda;
  p.ka1 = K;
  p.b = W;  // B(k, n) = W[k, n]
  p.sbk = ldw;
  p.sbn = 1;
  p.mask = mask;
  p.smk = ldm;
  p.smn = 1;
  p.c = C;
  p.ldc = ldc;
  p.M = M;
  p.N = N;
  p.act = NAZ_ACT_IDENTITY;
  p.dy = dy;
  p.lddy = lddy;
  p.dact = dact;
  return rowgemm(p, s);
}

// naz_gemm_jvp_bwd: C = (A · W) through the VJP epilogue of the CNF layer activation (see jvp above)
int rowgemm_jvp_bwd(const float* A, int64_t lda, int K, const float* W, int64_t ldw, float* C, int64_t ldc,
                    const float* S, int64_t lds, int act, int64_t M, int N, hipStream_t s) {
  if (M % 2 != 0) return set_error("naz_gemm_jvp_bwd: M must pair value and tangent rows (even)");
  if (ldc % 4 != 0 || (reinterpret_cast<uintptr_t>(C) & 15) != 0)
    return set_error("naz_gemm_jvp_bwd: C needs 16-byte aligned rows (ldc %% 4 == 0)");
  RowGemmArgs p{};
  p.a1 = A;
  p.lda1 = lda;
  p.ka1 = K;
  p.b = W;  // B(k, n) = W[k, n]
  p.sbk = ldw;
  p.sbn = 1;
  p.c = C;
  p.ldc = ldc;
  p.M = M;
  p.N = N;
  p.act = NAZ_ACT_IDENTITY;
  p.jvp = S;
  p.ldjvp = lds;
  p.jact = act;
  return rowgemm(p, s);
}

// gemm() fast paths; return 1 when the shape was not taken (caller falls back)
int gemm_rows_try(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
                  int64_t sbn, float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn,
                  int mask_b, int accumulate, float* rowsum, hipStream_t s, int* rc) {
  // dX-type: A row-major over a long M, small K and N, plain output rows
  if (sak == 1 && scn == 1 && rowsum == nullptr && (mask == nullptr || mask_b) && M >= 1024 && K <= 4096 &&
      N <= 4096) {
    RowGemmArgs p{};
    p.a0 = nullptr;
    p.lda0 = 0;
    p.ka0 = 0;
    p.a1 = A;
    p.lda1 = sam;
    p.ka1 = (int)K;
    p.b = B;
    p.sbk = sbk;
    p.sbn = sbn;
    p.mask = mask;
    p.smk = smm;
    p.smn = smn;
    p.c = C;
    p.ldc = scm;
    p.M = M;
    p.N = N;
    p.act = NAZ_ACT_IDENTITY;
    p.accumulate = accumulate;
    const int r = rowgemm(p, s);
    if (r == 1) return 1;  // not taken
    *rc = r;
    return 0;
  }
  // dW-type: C[M, N] = Σ_k A(m, k) B(k, n) with A = Gᵀ (unit m stride) and B = X (unit n stride)
  // over a long K: the reduction runs over the batch
  if (sam == 1 && sbn == 1 && (mask == nullptr || !mask_b) && M <= 256 && N + (rowsum != nullptr) <= 256 &&
      K >= 1024) {
    WGradArgs p{};
    p.g = A;
    p.sgm = sak;
    p.x = B;
    p.sxm = sbk;
    p.M = K;
    p.N1 = M;
    p.N2 = N;
    p.ones = rowsum != nullptr;
    p.c = C;
    p.scm = scm;
    p.scn = scn;
    p.mask = mask;
    p.smm = smm;
    p.smn = smn;
    p.rowsum = rowsum;
    *rc = wgrad(p, accumulate, s);
    return 0;
  }
  return 1;
}

}  // namespace naz
