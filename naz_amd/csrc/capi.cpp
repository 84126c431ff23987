// extern "C" entry points of libnazhip.so (declared in include/naz_hip.h).
// Thin argument validation + dispatch into the HIP translation units.
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <initializer_list>
#include <map>
#include <mutex>

#include "naz_internal.h"

namespace naz {

static thread_local char g_err[1024] = "";

int set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return -1;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_error("%s launch failed: %s", what, hipGetErrorString(e));
  return 0;
}

static hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static int check_spline_args(const char* fn, const float* x, const float* y, int64_t B, int Dt, int K, float bound) {
  if (B < 0 || Dt <= 0) return set_error("%s: bad shape B=%lld Dt=%d", fn, (long long)B, Dt);
  if (B > 0 && (x == nullptr || y == nullptr)) return set_error("%s: null x/y", fn);
  if (K < 2) return set_error("%s: count_bins must be >= 2 (got %d)", fn, K);
  if (1e-3 * K > 1.0) return set_error("%s: Minimal bin width too large for the number of bins", fn);
  if (!(bound > 0.f)) return set_error("%s: bound must be positive", fn);
  return 0;
}

// ---- packed weight images: header + registry (include/naz_hip.h "Packed images") -------------
// Every image a packer writes starts with a 256-byte header (the body stays 256-byte aligned for the
// kernels' LDS-DMA rings): magic, layout version, image kind, a layout tag hashed from the
// descriptor fields the layout depends on, layers, flags, body bytes.  The device packers record
// (base, header, draw stride, draws) in a host-side registry; host-packed images enter it through
// naz_image_attach, which reads the header back once.  Every launch entry resolves its image
// pointer through the registry BEFORE launching, so an image that is foreign, truncated, packed for
// another descriptor, kind or layer count, or by another layout version is refused with an error
// instead of being streamed into LDS out of bounds.
constexpr int64_t kImgHdr = 256;
constexpr uint32_t kImgMagic = 0x495a414eu;  // "NAZI"
constexpr uint32_t kImgVersion = 3;          // bump whenever any packed layout changes
enum : uint32_t { IMG_COUPLING = 1, IMG_COUPLING_BWD = 2, IMG_AR_INV = 3, IMG_AR_FWD = 4, IMG_AR_BWD = 5, IMG_CNF = 6 };
enum : uint32_t { IMG_FLAG_PASS0 = 1 };
static const char* const kImgKindName[] = {"?", "coupling", "coupling backward", "autoregressive inverse",
                                           "autoregressive forward", "autoregressive backward", "cnf"};

struct ImgSpec {  // what a descriptor expects of an image
  uint32_t kind, tag;
  int L;
  int64_t body;  // bytes after the header (-1: unsupported descriptor)
};
struct ImgRec {
  uint32_t kind, tag, L, flags;
  int64_t body, stride, draws;
};
static std::mutex g_img_mu;
static std::map<uintptr_t, ImgRec> g_img;  // image base -> record

static uint32_t fnv(uint32_t h, uint32_t v) {
  for (int i = 0; i < 4; ++i) {
    h ^= (v >> (8 * i)) & 0xffu;
    h *= 16777619u;
  }
  return h;
}
static uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
static uint32_t layout_tag(uint32_t kind, std::initializer_list<uint32_t> fields) {
  uint32_t h = fnv(fnv(2166136261u, kImgVersion), kind);
  for (uint32_t v : fields) h = fnv(h, v);
  return h;
}
static ImgSpec spec_coupling(const naz_coupling_desc* d, uint32_t kind) {
  if (d == nullptr) return {kind, 0, 0, -1};
  const int64_t b = kind == IMG_COUPLING ? coupling_packed_bytes(d) : coupling_bwd_packed_bytes(d);
  return {kind,
          layout_tag(kind, {(uint32_t)d->D, (uint32_t)d->C, (uint32_t)d->S, (uint32_t)d->K, (uint32_t)d->H,
                            (uint32_t)d->act, (uint32_t)d->has_lower, fbits(d->bound), (uint32_t)d->mfma_mode}),
          d->L, b};
}
static ImgSpec spec_ar(const naz_ar_desc* d, uint32_t kind) {
  if (d == nullptr) return {kind, 0, 0, -1};
  const int64_t b = kind == IMG_AR_INV ? ar_flow_packed_bytes(d)
                    : kind == IMG_AR_FWD ? ar_flow_fwd_packed_bytes(d)
                                         : ar_flow_bwd_packed_bytes(d);
  return {kind,
          layout_tag(kind, {(uint32_t)d->D, (uint32_t)d->C, (uint32_t)d->H, (uint32_t)d->K, (uint32_t)d->act,
                            d->kind == NAZ_AR_SPLINE ? fbits(d->bound) : 0u, (uint32_t)d->n_hidden,
                            (uint32_t)d->kind}),
          d->L, b};
}
static ImgSpec spec_cnf(const naz_cnf_desc* d) {
  if (d == nullptr) return {IMG_CNF, 0, 0, -1};
  uint32_t hs[4] = {};
  for (int i = 0; i < 4 && i < d->n_hidden; ++i) hs[i] = (uint32_t)d->H[i];
  return {IMG_CNF,
          layout_tag(IMG_CNF, {(uint32_t)d->D, (uint32_t)d->C, (uint32_t)d->n_hidden, hs[0], hs[1], hs[2], hs[3],
                               (uint32_t)d->act, (uint32_t)d->mfma_mode}),
          1, cnf_packed_bytes(d)};
}
static int64_t img_bytes(int64_t body) { return body < 0 ? body : body + kImgHdr; }
static void img_words(const ImgSpec& sp, uint32_t flags, uint32_t* w) {
  w[0] = kImgMagic;
  w[1] = kImgVersion;
  w[2] = sp.kind;
  w[3] = sp.tag;
  w[4] = (uint32_t)sp.L;
  w[5] = flags;
  w[6] = (uint32_t)((uint64_t)sp.body & 0xffffffffu);
  w[7] = (uint32_t)((uint64_t)sp.body >> 32);
}
static void img_record(const void* base, const ImgRec& r) {
  std::lock_guard<std::mutex> lk(g_img_mu);
  const uintptr_t b = reinterpret_cast<uintptr_t>(base);
  // a new image over the span of older ones replaces them
  auto it = g_img.lower_bound(b);
  while (it != g_img.end() && it->first < b + (uintptr_t)(r.stride * r.draws)) it = g_img.erase(it);
  it = g_img.lower_bound(b);
  if (it != g_img.begin()) {
    auto pv = std::prev(it);
    if (pv->first + (uintptr_t)(pv->second.stride * pv->second.draws) > b) g_img.erase(pv);
  }
  g_img[b] = r;
}
// the device packers: headers for P images at `stride` bytes, then the registry record
static int img_publish(const char* fn, const ImgSpec& sp, void* base, int64_t stride, int64_t P, uint32_t flags,
                       hipStream_t s) {
  if (P <= 0) return 0;
  uint32_t w[8];
  img_words(sp, flags, w);
  if (int rc = write_image_headers(base, stride, P, w, 8, s)) return rc;
  (void)fn;
  img_record(base, ImgRec{sp.kind, sp.tag, (uint32_t)sp.L, flags, sp.body, stride, P});
  return 0;
}
// resolve an image pointer (a registered base, or draw p of a registered multi-draw buffer) for a
// launch over P draws at spk floats per draw (P = 1: spk unused); returns the body pointer
static int img_resolve(const char* fn, const ImgSpec& sp, const void* image, int64_t P, int64_t spk, uint32_t flags,
                       const void** body) {
  if (sp.body < 0) {  // no instance: the dispatch behind the entry reports the descriptor (nothing launches)
    *body = image;
    return 0;
  }
  if (image == nullptr) return set_error("%s: null packed image", fn);
  const uintptr_t p = reinterpret_cast<uintptr_t>(image);
  ImgRec r{};
  int64_t draw = 0;
  {
    std::lock_guard<std::mutex> lk(g_img_mu);
    auto it = g_img.upper_bound(p);
    if (it == g_img.begin())
      return set_error("%s: %p is not a packed image (pack it with a naz_*_pack entry, or naz_image_attach a "
                       "host-packed copy)", fn, image);
    --it;
    r = it->second;
    const uintptr_t off = p - it->first;
    if (off % (uintptr_t)r.stride != 0 || off / (uintptr_t)r.stride >= (uintptr_t)r.draws)
      return set_error("%s: %p is not a packed image (inside one at %p)", fn, image, (const void*)it->first);
    draw = (int64_t)(off / (uintptr_t)r.stride);
  }
  if (r.kind != sp.kind)
    return set_error("%s: image %p is a %s image, expected a %s image", fn, image,
                     kImgKindName[r.kind < 7 ? r.kind : 0], kImgKindName[sp.kind]);
  if (r.tag != sp.tag)
    return set_error("%s: image %p was packed for another descriptor or layout (tag %08x, expected %08x)", fn, image,
                     r.tag, sp.tag);
  if ((int)r.L != sp.L || r.body != sp.body)
    return set_error("%s: image %p holds %u layers / %lld B, the descriptor needs %d layers / %lld B", fn, image, r.L,
                     (long long)r.body, sp.L, (long long)sp.body);
  if ((r.flags & IMG_FLAG_PASS0) != (flags & IMG_FLAG_PASS0))
    return set_error("%s: image %p %s pass-0 constants, the call %s them", fn, image,
                     (r.flags & IMG_FLAG_PASS0) ? "carries" : "has no", (flags & IMG_FLAG_PASS0) ? "expects" : "does not expect");
  if (P > 1 && (spk * 4 != r.stride || draw + P > r.draws))
    return set_error("%s: %lld draws at %lld floats per draw from draw %lld of an image set of %lld draws at %lld B",
                     fn, (long long)P, (long long)spk, (long long)draw, (long long)r.draws, (long long)r.stride);
  *body = static_cast<const char*>(image) + kImgHdr;
  return 0;
}
#define NAZ_IMG(fn, spec, image, P, spk, flags, body) \
  const void* body = nullptr;                           \
  if (int rc_ = img_resolve(fn, spec, image, P, spk, flags, &body)) return rc_

}  // namespace naz

using namespace naz;

extern "C" {

const char* naz_last_error(void) { return g_err; }
int naz_abi_version(void) { return 3; }

int naz_image_attach(const void* image, int64_t bytes, void* stream) {
  if (image == nullptr || bytes < kImgHdr) return set_error("naz_image_attach: null image or fewer than 256 bytes");
  uint32_t w[8];
  hipStream_t s = as_stream(stream);
  if (hipMemcpyAsync(w, image, sizeof(w), hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
    return set_error("naz_image_attach: cannot read the header of %p", image);
  if (w[0] != kImgMagic) return set_error("naz_image_attach: %p holds no packed-image header", image);
  if (w[1] != kImgVersion)
    return set_error("naz_image_attach: %p was packed by layout version %u, this library reads %u", image, w[1],
                     kImgVersion);
  if (w[2] < IMG_COUPLING || w[2] > IMG_CNF) return set_error("naz_image_attach: %p: unknown image kind %u", image, w[2]);
  const int64_t body = (int64_t)((uint64_t)w[6] | ((uint64_t)w[7] << 32));
  if (body <= 0 || body > bytes - kImgHdr)
    return set_error("naz_image_attach: %p: the header announces %lld B of weights, the buffer holds %lld B", image,
                     (long long)body, (long long)(bytes - kImgHdr));
  img_record(image, ImgRec{w[2], w[3], w[4], w[5], body, body + kImgHdr, 1});
  return 0;
}

int naz_tuning(const char* key, int value) {
  if (key != nullptr && strcmp(key, "rowgemm_split") == 0) return rowgemm_split_setting(value);
  if (key != nullptr && strcmp(key, "rowgemm_x6") == 0) return rowgemm_x6_setting(value);
  if (key != nullptr && strcmp(key, "rowgemm_fill") == 0) return rowgemm_fill_setting(value);
  if (key != nullptr && strcmp(key, "rowgemm_h3") == 0) return rowgemm_h3_setting(value);
  if (key != nullptr && strcmp(key, "rowgemm_bres") == 0) return rowgemm_bres_setting(value);
  return set_error("naz_tuning: unknown key '%s'", key ? key : "(null)");
}

int naz_image_release(const void* image) {
  std::lock_guard<std::mutex> lk(g_img_mu);
  return g_img.erase(reinterpret_cast<uintptr_t>(image)) ? 0 : set_error("naz_image_release: %p is not registered", image);
}

int naz_rqs_fwd(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy, float* ld,
                int ld_mode, int64_t B, int Dt, int K, int layout, float bound, void* stream) {
  if (int rc = check_spline_args("naz_rqs_fwd", x, y, B, Dt, K, bound)) return rc;
  return rqs_cond(0, x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, Dt, K, layout, bound, as_stream(stream));
}

int naz_rqs_inv(const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy, float* ld,
                int ld_mode, int64_t B, int Dt, int K, int layout, float bound, void* stream) {
  if (int rc = check_spline_args("naz_rqs_inv", x, y, B, Dt, K, bound)) return rc;
  return rqs_cond(1, x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, Dt, K, layout, bound, as_stream(stream));
}

int naz_spline_elementwise(int inverse, const float* x, int64_t ldx, const float* uw, const float* uh,
                           const float* ud, float* y, int64_t ldy, float* ld, int64_t B, int Dt, int K, float bound,
                           void* stream) {
  if (int rc = check_spline_args("naz_spline_elementwise", x, y, B, Dt, K, bound)) return rc;
  return rqs_uncond(inverse, x, ldx, uw, uh, ud, y, ldy, ld, B, Dt, K, bound, as_stream(stream));
}

int naz_linear_act(const float* ctx, int64_t ldc, int C, const float* x, int64_t ldx, int Kx, const float* W,
                   const float* mask, const float* b, float* y, int64_t ldy, int64_t M, int N, int act, void* stream) {
  if (M < 0 || N < 0 || C < 0 || Kx < 0) return set_error("naz_linear_act: negative shape");
  return linear_act(ctx, ldc, C, x, ldx, Kx, W, mask, b, y, ldy, M, N, act, as_stream(stream));
}

int naz_linear_act_batched(const float* ctx, int64_t ldc, int64_t sctx, int C, const float* x, int64_t ldx,
                           int64_t sx, int Kx, const float* W, int64_t sw, const float* mask, const float* b,
                           int64_t sb, float* y, int64_t ldy, int64_t sy, int64_t M, int N, int nbatch, int act,
                           void* stream) {
  if (M < 0 || N < 0 || C < 0 || Kx < 0 || nbatch < 0) return set_error("naz_linear_act_batched: negative shape");
  if (nbatch > 65535) return set_error("naz_linear_act_batched: nbatch %d > 65535 (grid z)", nbatch);
  if (C > 0 && ctx == nullptr) return set_error("naz_linear_act_batched: C=%d but ctx is NULL", C);
  if (Kx > 0 && x == nullptr) return set_error("naz_linear_act_batched: Kx=%d but x is NULL", Kx);
  if (W == nullptr || y == nullptr) return set_error("naz_linear_act_batched: NULL W or y");
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_linear_act_batched: unknown activation %d", act);
  if ((int64_t)N * (C + Kx) * 4 >= (1ll << 31)) return set_error("naz_linear_act_batched: weight block too large");
  return rowgemm_linear_batched(ctx, ldc, sctx, C, x, ldx, sx, Kx, W, sw, mask, b, sb, y, ldy, sy, M, N, nbatch, act,
                                as_stream(stream));
}

int64_t naz_made_packed_floats(int nhid, int nh, int C, int D) {
  if (nhid < 1 || nh < 1 || C < 0 || D < 1) return -1;
  return made_packed_floats(nhid, nh, C, D);
}

int naz_made_affine_fwd(const float* packed, int64_t wstride, int nhid, int nh, int C, int D, const float* ctx,
                        int64_t ldc, int64_t sctx, const float* x, int64_t ldx, int64_t sx, float* y, int64_t ldy,
                        int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, void* stream) {
  if (S < 0 || P < 0 || x == nullptr || y == nullptr || packed == nullptr)
    return set_error("naz_made_affine_fwd: bad arguments");
  return made_affine_fwd(packed, wstride, nhid, nh, C, D, ctx, ldc, sctx, x, ldx, sx, y, ldy, sy, ld, sld, ld_mode, S,
                         P, act, as_stream(stream));
}

int naz_gemm_dact(const float* A, int64_t lda, int K, const float* W, int64_t ldw, const float* mask, int64_t ldm,
                  float* C, int64_t ldc, const float* dy, int64_t lddy, int dact, int64_t M, int N, void* stream) {
  if (M < 0 || N < 0 || K < 0) return set_error("naz_gemm_dact: negative shape");
  if (M == 0 || N == 0) return 0;
  if (A == nullptr || W == nullptr || C == nullptr || dy == nullptr) return set_error("naz_gemm_dact: null pointer");
  if (dact < 0 || dact > NAZ_ACT_SIGMOID) return set_error("naz_gemm_dact: unknown activation %d", dact);
  const int rc = rowgemm_dact(A, lda, K, W, ldw, mask, ldm, C, ldc, dy, lddy, dact, M, N, as_stream(stream));
  if (rc == 1) return set_error("naz_gemm_dact: weights too large for the batch-row kernel");
  return rc;
}

int naz_made_affine_inv1(const float* packed, int64_t wstride, int nhid, int nh, int D, const float* x, int64_t ldx,
                         int64_t sx, const float* v, int64_t ldv, int64_t sv, int dim, float* y, int64_t ldy,
                         int64_t sy, float* ld, int64_t sld, int ld_mode, int64_t S, int P, int act, void* stream) {
  if (S < 0 || P < 0 || x == nullptr || y == nullptr || packed == nullptr)
    return set_error("naz_made_affine_inv1: bad arguments");
  return made_affine_inv1(packed, wstride, nhid, nh, D, x, ldx, sx, v, ldv, sv, dim, y, ldy, sy, ld, sld, ld_mode, S,
                          P, act, as_stream(stream));
}

int naz_affine_ar(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, float* y, int64_t ldy,
                  float* ld, int ld_mode, int64_t B, int D, void* stream) {
  if (B < 0 || D <= 0) return set_error("naz_affine_ar: bad shape");
  return affine_ar(inverse, x, ldx, raw, ldr, y, ldy, ld, ld_mode, B, D, as_stream(stream));
}

int naz_base_log_prob(const float* z, int64_t ldz, float* out, int64_t B, int D, int accumulate, void* stream) {
  return base_log_prob(z, ldz, out, B, D, accumulate, as_stream(stream));
}

int naz_bounding_fwd(const float* x, int64_t ldx, const float* low, const float* high, float* y, int64_t ldy,
                     float* out_logjac, int64_t B, int D, void* stream) {
  return bounding_fwd(x, ldx, low, high, y, ldy, out_logjac, B, D, as_stream(stream));
}

int naz_bounding_inv(const float* y, int64_t ldy, const float* low, const float* high, float* x, int64_t ldx,
                     int64_t B, int D, void* stream) {
  return bounding_inv(y, ldy, low, high, x, ldx, B, D, as_stream(stream));
}

int naz_rqs_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* g_out,
                int64_t ldgo, const float* g_ld, int g_ld_mode, float* g_in, int64_t ldgi, float* g_raw, int64_t ldgr,
                int64_t B, int Dt, int K, int layout, float bound, void* stream) {
  if (int rc = check_spline_args("naz_rqs_bwd", x, x, B, Dt, K, bound)) return rc;
  if (B > 0 && g_raw == nullptr) return set_error("naz_rqs_bwd: g_raw is required");
  if (g_ld_mode < 0 || g_ld_mode > 2 || (g_ld_mode != 0 && g_ld == nullptr))
    return set_error("naz_rqs_bwd: bad g_ld / g_ld_mode");
  return rqs_bwd(inverse, x, ldx, raw, ldr, g_out, ldgo, g_ld, g_ld_mode, g_in, ldgi, g_raw, ldgr, B, Dt, K, layout,
                 bound, as_stream(stream));
}

int naz_gemm(int M, int N, int64_t K, const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk,
             int64_t sbn, float* C, int64_t scm, int64_t scn, const float* mask, int64_t smm, int64_t smn,
             int mask_b, int accumulate, int split_k, float* rowsum, void* stream) {
  if (M < 0 || N < 0 || K < 0) return set_error("naz_gemm: negative shape");
  return gemm(M, N, K, A, sam, sak, B, sbk, sbn, C, scm, scn, mask, smm, smn, mask_b, accumulate, split_k, rowsum,
              as_stream(stream));
}

int naz_wgrad_batched(int64_t M, int N1, int N2, int nbatch, const float* g, int64_t sgm, int64_t bg, const float* x,
                      int64_t sxm, int64_t bx, float* c, int64_t scm, int64_t bc, float* rowsum, int64_t br,
                      void* stream) {
  if (M > 0 && nbatch > 0 && (g == nullptr || x == nullptr || c == nullptr))
    return set_error("naz_wgrad_batched: null pointer");
  return wgrad_batched(M, N1, N2, nbatch, g, sgm, bg, x, sxm, bx, c, scm, bc, rowsum, br, as_stream(stream));
}

int naz_affine_ar_bwd(int inverse, const float* x, int64_t ldx, const float* raw, int64_t ldr, const float* y,
                      int64_t ldy, const float* g_y, int64_t ldgy, const float* g_ld, float* g_x, int64_t ldgx,
                      float* g_raw, int64_t ldgr, int64_t B, int D, void* stream) {
  if (B > 0 && (g_raw == nullptr || g_y == nullptr)) return set_error("naz_affine_ar_bwd: g_y and g_raw are required");
  return affine_ar_bwd(inverse, x, ldx, raw, ldr, y, ldy, g_y, ldgy, g_ld, g_x, ldgx, g_raw, ldgr, B, D,
                       as_stream(stream));
}

int naz_maf_dim_vjp(int mode, const float* raw, int64_t ldr, const float* s_out, int64_t lds, const float* g,
                    int64_t ldg, const float* g_lp, float* g_next, int64_t ldgn, float* tot, int64_t ldt, float* chain,
                    int64_t ldch, int64_t B, int D, int dim, void* stream) {
  if (D <= 0 || dim < 0 || dim >= D) return set_error("naz_maf_dim_vjp: dim %d outside [0, %d)", dim, D);
  if (B > 0 && (raw == nullptr || s_out == nullptr || g == nullptr || g_next == nullptr || tot == nullptr))
    return set_error("naz_maf_dim_vjp: null pointer");
  return maf_dim_vjp(mode, raw, ldr, s_out, lds, g, ldg, g_lp, g_next, ldgn, tot, ldt, chain, ldch, B, D, dim,
                     as_stream(stream));
}

int naz_colsum(const float* A, int64_t lda, int64_t M, int N, float* out, void* stream) {
  return colsum(A, lda, M, N, out, as_stream(stream));
}

int naz_act_bwd(const float* gy, int64_t ldg, const float* y, int64_t ldy, float* gpre, int64_t ldp, int64_t M, int N,
                int act, void* stream) {
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_act_bwd: unknown activation %d", act);
  return act_bwd(gy, ldg, y, ldy, gpre, ldp, M, N, act, as_stream(stream));
}

int naz_dropout(const float* x, int64_t ldx, float* y, int64_t ldy, int64_t M, int N, float p, uint64_t seed,
                void* stream) {
  if (M < 0 || N < 0) return set_error("naz_dropout: negative shape");
  if (!(p >= 0.f && p < 1.f)) return set_error("naz_dropout: p must be in [0, 1)");
  return dropout(x, ldx, y, ldy, M, N, p, seed, as_stream(stream));
}

int naz_base_log_prob_bwd(const float* z, int64_t ldz, const float* g_lp, float* g_z, int64_t ldgz, int64_t B, int D,
                          void* stream) {
  return base_log_prob_bwd(z, ldz, g_lp, g_z, ldgz, B, D, as_stream(stream));
}

int naz_cnf_supported(const naz_cnf_desc* d) { return cnf_supported(d); }
int64_t naz_cnf_param_count(const naz_cnf_desc* d) { return cnf_param_count(d); }
int64_t naz_cnf_packed_bytes(const naz_cnf_desc* d) { return img_bytes(cnf_packed_bytes(d)); }
int naz_cnf_pack(const naz_cnf_desc* d, const float* flat, void* packed, void* stream) {
  if (flat == nullptr || packed == nullptr) return set_error("naz_cnf_pack: null pointer");
  const ImgSpec sp = spec_cnf(d);
  if (int rc = cnf_pack(d, flat, static_cast<char*>(packed) + kImgHdr, as_stream(stream))) return rc;
  return img_publish("naz_cnf_pack", sp, packed, img_bytes(sp.body), 1, 0, as_stream(stream));
}
int naz_cnf_integrate(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* eps, int64_t lde, float t0, float t1, int steps, float* y,
                      int64_t ldy, float* ld, int ld_mode, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_cnf_integrate: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || eps == nullptr || y == nullptr))
    return set_error("naz_cnf_integrate: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr) return set_error("naz_cnf_integrate: context required");
  if (B == 0) return 0;
  NAZ_IMG("naz_cnf_integrate", spec_cnf(d), packed, 1, 0, 0, body);
  return cnf_integrate(d, body, x, ldx, ctx, ldc, eps, lde, t0, t1, steps, y, ldy, ld, ld_mode, B,
                       as_stream(stream));
}

int naz_cnf_integrate_dopri5(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                             const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                             float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld, int ld_mode,
                             int* nfe, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_cnf_integrate_dopri5: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || eps == nullptr || y == nullptr))
    return set_error("naz_cnf_integrate_dopri5: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_cnf_integrate_dopri5: context required");
  if (B == 0) return 0;
  NAZ_IMG("naz_cnf_integrate_dopri5", spec_cnf(d), packed, 1, 0, 0, body);
  return cnf_integrate_dopri5(d, body, x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps, y, ldy, ld,
                              ld_mode, nfe, B, as_stream(stream));
}

int64_t naz_cnf_dopri5_global_workspace_bytes(const naz_cnf_desc* d, int64_t B) {
  if (B < 0) return -1;
  return cnf_dopri5_global_workspace_bytes(d, B);
}

int naz_cnf_integrate_dopri5_global(const naz_cnf_desc* d, const void* packed, const float* x, int64_t ldx,
                                    const float* ctx, int64_t ldc, const float* eps, int64_t lde, float t0, float t1,
                                    float atol, float rtol, int max_steps, float* y, int64_t ldy, float* ld,
                                    int ld_mode, int* nfe, void* workspace, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_cnf_integrate_dopri5_global: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || eps == nullptr || y == nullptr))
    return set_error("naz_cnf_integrate_dopri5_global: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_cnf_integrate_dopri5_global: context required");
  if (B == 0) return 0;
  NAZ_IMG("naz_cnf_integrate_dopri5_global", spec_cnf(d), packed, 1, 0, 0, body);
  return cnf_integrate_dopri5_global(d, body, x, ldx, ctx, ldc, eps, lde, t0, t1, atol, rtol, max_steps, y, ldy,
                                     ld, ld_mode, nfe, workspace, B, as_stream(stream));
}

int naz_gemm_jvp_bwd(const float* A, int64_t lda, int K, const float* W, int64_t ldw, float* C, int64_t ldc,
                     const float* S, int64_t lds, int act, int64_t M, int N, void* stream) {
  if (M < 0 || N < 0 || K < 0) return set_error("naz_gemm_jvp_bwd: negative shape");
  if (M == 0 || N == 0) return 0;
  if (A == nullptr || W == nullptr || C == nullptr || S == nullptr) return set_error("naz_gemm_jvp_bwd: null pointer");
  if (act < 0 || act > NAZ_ACT_SIGMOID) return set_error("naz_gemm_jvp_bwd: unknown activation %d", act);
  const int rc = rowgemm_jvp_bwd(A, lda, K, W, ldw, C, ldc, S, lds, act, M, N, as_stream(stream));
  if (rc == 1) return set_error("naz_gemm_jvp_bwd: weights too large for the batch-row kernel");
  return rc;
}

int naz_coupling_supported(const naz_coupling_desc* d) { return coupling_supported(d); }
int64_t naz_coupling_param_count(const naz_coupling_desc* d) { return coupling_param_count(d); }
int64_t naz_coupling_packed_bytes(const naz_coupling_desc* d) { return img_bytes(coupling_packed_bytes(d)); }

int naz_coupling_pack(const naz_coupling_desc* d, const float* flat_params, void* packed, void* stream) {
  const ImgSpec sp = spec_coupling(d, IMG_COUPLING);
  if (sp.body < 0) return set_error("naz_coupling_pack: no fused instantiation for this descriptor");
  if (packed == nullptr) return set_error("naz_coupling_pack: null image");
  if (int rc = coupling_pack(d, flat_params, static_cast<char*>(packed) + kImgHdr, as_stream(stream))) return rc;
  return img_publish("naz_coupling_pack", sp, packed, img_bytes(sp.body), 1, 0, as_stream(stream));
}

int naz_coupling_log_prob(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                          const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                          int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_log_prob: conditional flow needs ctx");
  if (B == 0) return 0;
  NAZ_IMG("naz_coupling_log_prob", spec_coupling(d, IMG_COUPLING), packed, 1, 0, 0, body);
  return coupling_log_prob(d, body, x, ldx, ctx, ldc, low, high, out_lp, B, as_stream(stream));
}

int naz_coupling_sample(const naz_coupling_desc* d, const void* packed, const float* z, int64_t ldz,
                        const float* ctx, int64_t ldc, const float* low, const float* high, float* y, int64_t ldy,
                        float* out_ld, int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_sample: conditional flow needs ctx");
  if (B == 0) return 0;
  NAZ_IMG("naz_coupling_sample", spec_coupling(d, IMG_COUPLING), packed, 1, 0, 0, body);
  return coupling_sample(d, body, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, as_stream(stream));
}

int64_t naz_coupling_bwd_packed_bytes(const naz_coupling_desc* d) { return img_bytes(coupling_bwd_packed_bytes(d)); }

int naz_coupling_pack_bwd(const naz_coupling_desc* d, const float* flat_params, void* packed_bwd, void* stream) {
  const ImgSpec sp = spec_coupling(d, IMG_COUPLING_BWD);
  if (sp.body < 0) return set_error("naz_coupling_pack_bwd: no fused instantiation for this descriptor");
  if (packed_bwd == nullptr) return set_error("naz_coupling_pack_bwd: null image");
  if (int rc = coupling_pack_bwd(d, flat_params, static_cast<char*>(packed_bwd) + kImgHdr, as_stream(stream))) return rc;
  return img_publish("naz_coupling_pack_bwd", sp, packed_bwd, img_bytes(sp.body), 1, 0, as_stream(stream));
}

int naz_coupling_log_prob_train(const naz_coupling_desc* d, const void* packed, const float* x, int64_t ldx,
                                const float* ctx, int64_t ldc, const float* low, const float* high, float* out_lp,
                                float* states, int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_log_prob_train: conditional flow needs ctx");
  if (B == 0) return 0;
  NAZ_IMG("naz_coupling_log_prob_train", spec_coupling(d, IMG_COUPLING), packed, 1, 0, 0, body);
  return coupling_log_prob_train(d, body, x, ldx, ctx, ldc, low, high, out_lp, states, B, as_stream(stream));
}

int naz_coupling_bwd_layer(const naz_coupling_desc* d, const void* packed, const void* packed_bwd, const float* flat,
                           int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                           const float* g_lp, float* h1, float* h2, float* dp1, float* dp2, float* dp3, float* x0,
                           float* g_out, float* g_low, int64_t B, void* stream) {
  if (d != nullptr && d->C > 0 && ctx == nullptr) return set_error("naz_coupling_bwd_layer: conditional flow needs ctx");
  if (B < 0) return set_error("naz_coupling_bwd_layer: negative batch");
  if (B == 0) return 0;  // an empty batch is a no-op, as in every other entry (no image is read)
  NAZ_IMG("naz_coupling_bwd_layer", spec_coupling(d, IMG_COUPLING), packed, 1, 0, 0, body);
  NAZ_IMG("naz_coupling_bwd_layer", spec_coupling(d, IMG_COUPLING_BWD), packed_bwd, 1, 0, 0, body_bwd);
  return coupling_bwd_layer(d, body, body_bwd, flat, layer, state, ctx, ldc, g_in, g_lp, h1, h2, dp1, dp2, dp3,
                            x0, g_out, g_low, B, as_stream(stream));
}

int naz_coupling_dp3_columns(const naz_coupling_desc* d, int* rows) { return coupling_dp3_columns(d, rows); }

static int coupling_layer_api(const char* what, const naz_coupling_desc* d, int inv, const void* packed, int layer,
                              const float* x, int64_t ldx, const float* ctx, int64_t ldc, float* y, int64_t ldy,
                              float* ld, int ld_mode, int64_t B, void* stream) {
  if (B < 0) return set_error("%s: negative batch", what);
  if (B > 0 && (packed == nullptr || x == nullptr || y == nullptr || ld == nullptr))
    return set_error("%s: null pointer", what);
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr) return set_error("%s: conditional flow needs ctx", what);
  if (B == 0) return 0;  // an empty batch is a no-op, as in every other entry (no image is read)
  NAZ_IMG(what, spec_coupling(d, IMG_COUPLING), packed, 1, 0, 0, body);
  return coupling_layer(d, inv, body, layer, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B, as_stream(stream));
}
int naz_coupling_layer_fwd(const naz_coupling_desc* d, const void* packed, int layer, const float* x, int64_t ldx,
                           const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                           void* stream) {
  return coupling_layer_api("naz_coupling_layer_fwd", d, 0, packed, layer, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B,
                            stream);
}
int naz_coupling_layer_inv(const naz_coupling_desc* d, const void* packed, int layer, const float* x, int64_t ldx,
                           const float* ctx, int64_t ldc, float* y, int64_t ldy, float* ld, int ld_mode, int64_t B,
                           void* stream) {
  return coupling_layer_api("naz_coupling_layer_inv", d, 1, packed, layer, x, ldx, ctx, ldc, y, ldy, ld, ld_mode, B,
                            stream);
}

int naz_ar_flow_supported(const naz_ar_desc* d) { return ar_flow_supported(d); }
int64_t naz_ar_flow_packed_bytes(const naz_ar_desc* d) { return img_bytes(ar_flow_packed_bytes(d)); }
int64_t naz_ar_flow_workspace_bytes(const naz_ar_desc* d, int64_t B, int64_t P) {
  if (B < 0 || P < 0) return -1;
  return ar_flow_workspace_bytes(d, B, P);
}
int naz_ar_flow_degrees(const naz_ar_desc* d, int* deg) { return ar_flow_degrees(d, deg); }
// host packers: the header goes into the host buffer; the caller uploads it and naz_image_attach-es it
static int host_image(const ImgSpec& sp, void* packed) {
  uint32_t w[8];
  img_words(sp, 0, w);
  memset(packed, 0, kImgHdr);
  memcpy(packed, w, sizeof(w));
  return 0;
}
int naz_ar_flow_pack_host(const naz_ar_desc* d, const float* flat, const int* perm, void* packed) {
  if (packed == nullptr) return set_error("naz_ar_flow_pack_host: null image");
  if (int rc = ar_flow_pack_host(d, flat, perm, static_cast<char*>(packed) + kImgHdr)) return rc;
  return host_image(spec_ar(d, IMG_AR_INV), packed);
}
int naz_ar_flow_log_prob(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                         int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* workspace,
                         int64_t workspace_bytes, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_log_prob: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || out_lp == nullptr))
    return set_error("naz_ar_flow_log_prob: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_log_prob: conditional flow needs ctx");
  if (B == 0) return 0;
  NAZ_IMG("naz_ar_flow_log_prob", spec_ar(d, IMG_AR_INV), packed, 1, 0, 0, body);
  return ar_flow_log_prob(d, body, x, ldx, ctx, ldc, low, high, out_lp, B, workspace, workspace_bytes,
                          as_stream(stream));
}

int64_t naz_ar_flow_fwd_packed_bytes(const naz_ar_desc* d) { return img_bytes(ar_flow_fwd_packed_bytes(d)); }
int naz_ar_flow_pack_fwd_host(const naz_ar_desc* d, const float* flat, void* packed) {
  if (packed == nullptr) return set_error("naz_ar_flow_pack_fwd_host: null image");
  if (int rc = ar_flow_pack_fwd_host(d, flat, static_cast<char*>(packed) + kImgHdr)) return rc;
  return host_image(spec_ar(d, IMG_AR_FWD), packed);
}
int naz_ar_flow_sample(const naz_ar_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                       int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld,
                       int64_t B, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_sample: negative batch");
  if (B > 0 && (packed == nullptr || z == nullptr || y == nullptr)) return set_error("naz_ar_flow_sample: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_sample: conditional flow needs ctx");
  if (B == 0) return 0;
  NAZ_IMG("naz_ar_flow_sample", spec_ar(d, IMG_AR_FWD), packed, 1, 0, 0, body);
  return ar_flow_sample(d, body, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, as_stream(stream));
}

int naz_ar_flow_pack_fwd(const naz_ar_desc* d, const float* flat, int64_t sflat, void* packed, int64_t spk, int64_t P,
                         const float* mask, void* stream) {
  if (P < 0) return set_error("naz_ar_flow_pack_fwd: negative draw count");
  const ImgSpec sp = spec_ar(d, IMG_AR_FWD);
  if (sp.body < 0) return set_error("naz_ar_flow_pack_fwd: no fused instantiation for this descriptor");
  if (packed == nullptr) return set_error("naz_ar_flow_pack_fwd: null image");
  if (sp.body >= 0 && P > 1 && spk * 4 < img_bytes(sp.body))
    return set_error("naz_ar_flow_pack_fwd: draw stride %lld floats shorter than one image", (long long)spk);
  if (int rc = ar_flow_pack_fwd(d, flat, sflat, static_cast<char*>(packed) + kImgHdr, P > 1 ? spk : sp.body / 4 + 64, P,
                                mask, as_stream(stream)))
    return rc;
  return img_publish("naz_ar_flow_pack_fwd", sp, packed, P > 1 ? spk * 4 : img_bytes(sp.body), P, 0, as_stream(stream));
}
int naz_ar_flow_sample_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* z, int64_t ldz,
                               int64_t sz, const float* ctx, int64_t ldc, float* y, int64_t ldy, int64_t sy,
                               float* out_ld, int64_t sld, int64_t B, int64_t P, void* stream) {
  if (B < 0 || P < 0) return set_error("naz_ar_flow_sample_batched: negative size");
  if (B > 0 && P > 0 && (packed == nullptr || z == nullptr || y == nullptr))
    return set_error("naz_ar_flow_sample_batched: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && P > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_sample_batched: conditional flow needs ctx");
  if (B == 0 || P == 0) return 0;
  NAZ_IMG("naz_ar_flow_sample_batched", spec_ar(d, IMG_AR_FWD), packed, P, spk, 0, body);
  return ar_flow_sample_batched(d, body, spk, z, ldz, sz, ctx, ldc, y, ldy, sy, out_ld, sld, B, P, as_stream(stream));
}

int64_t naz_ar_flow_pass0_floats(const naz_ar_desc* d) { return ar_flow_pass0_floats(d); }
int naz_ar_flow_pack(const naz_ar_desc* d, const float* flat, int64_t sflat, const int* perm, void* packed, int64_t spk,
                     int64_t P, const float* pass0, int64_t sp0, const float* mask, void* stream) {
  if (P < 0) return set_error("naz_ar_flow_pack: negative draw count");
  const ImgSpec sp = spec_ar(d, IMG_AR_INV);
  if (sp.body < 0) return set_error("naz_ar_flow_pack: no fused instantiation for this descriptor");
  if (packed == nullptr) return set_error("naz_ar_flow_pack: null image");
  if (sp.body >= 0 && P > 1 && spk * 4 < img_bytes(sp.body))
    return set_error("naz_ar_flow_pack: draw stride %lld floats shorter than one image", (long long)spk);
  if (int rc = ar_flow_pack(d, flat, sflat, perm, static_cast<char*>(packed) + kImgHdr, P > 1 ? spk : sp.body / 4 + 64,
                            P, pass0, sp0, mask, as_stream(stream)))
    return rc;
  return img_publish("naz_ar_flow_pack", sp, packed, P > 1 ? spk * 4 : img_bytes(sp.body), P,
                     pass0 != nullptr ? IMG_FLAG_PASS0 : 0u, as_stream(stream));
}
int naz_ar_flow_log_prob_batched(const naz_ar_desc* d, const void* packed, int64_t spk, const float* x, int64_t ldx,
                                 int64_t sx, const float* ctx, int64_t ldc, float* out_lp, int64_t slp, int64_t B,
                                 int64_t P, int pass0_const, void* workspace, int64_t workspace_bytes, void* stream) {
  if (B < 0 || P < 0) return set_error("naz_ar_flow_log_prob_batched: negative size");
  if (B > 0 && P > 0 && (packed == nullptr || x == nullptr || out_lp == nullptr))
    return set_error("naz_ar_flow_log_prob_batched: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && P > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_log_prob_batched: conditional flow needs ctx");
  if (B == 0 || P == 0) return 0;
  NAZ_IMG("naz_ar_flow_log_prob_batched", spec_ar(d, IMG_AR_INV), packed, P, spk, pass0_const ? IMG_FLAG_PASS0 : 0u, body);
  return ar_flow_log_prob_batched(d, body, spk, x, ldx, sx, ctx, ldc, out_lp, slp, B, P, pass0_const, workspace,
                                  workspace_bytes, as_stream(stream));
}

// ---- fused maf backward (made_ar_bwd.h): NUTS potential gradient / maf NLL step ----------
int naz_ar_flow_log_prob_train(const naz_ar_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                               int64_t ldc, float* out_lp, float* states, int64_t B, void* workspace,
                               int64_t workspace_bytes, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_log_prob_train: negative batch");
  if (B > 0 && (packed == nullptr || x == nullptr || out_lp == nullptr))
    return set_error("naz_ar_flow_log_prob_train: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_log_prob_train: conditional flow needs ctx");
  if (d == nullptr || d->kind != NAZ_AR_AFFINE || naz_ar_flow_supported(d) != 1)
    return set_error("naz_ar_flow_log_prob_train: no fused affine inverse for this flow");
  if (B == 0) return 0;
  NAZ_IMG("naz_ar_flow_log_prob_train", spec_ar(d, IMG_AR_INV), packed, 1, 0, 0, body);
  return ar_flow_log_prob_train(d, body, x, ldx, ctx, ldc, out_lp, states, B, workspace, workspace_bytes,
                                as_stream(stream));
}
int64_t naz_ar_flow_bwd_packed_bytes(const naz_ar_desc* d) { return img_bytes(ar_flow_bwd_packed_bytes(d)); }
int naz_ar_flow_bwd_dims(const naz_ar_desc* d, int* dims) { return ar_flow_bwd_dims(d, dims); }
int naz_ar_flow_pack_bwd(const naz_ar_desc* d, const float* flat, const float* mask, void* packed, void* stream) {
  const ImgSpec sp = spec_ar(d, IMG_AR_BWD);
  if (sp.body < 0) return set_error("naz_ar_flow_pack_bwd: no fused instantiation for this descriptor");
  if (packed == nullptr) return set_error("naz_ar_flow_pack_bwd: null image");
  if (int rc = ar_flow_pack_bwd(d, flat, mask, static_cast<char*>(packed) + kImgHdr, as_stream(stream))) return rc;
  return img_publish("naz_ar_flow_pack_bwd", sp, packed, img_bytes(sp.body), 1, 0, as_stream(stream));
}
int naz_ar_flow_bwd_layer(const naz_ar_desc* d, const void* packed_fwd, const void* packed_bwd, const int* perm,
                          int layer, const float* state, const float* ctx, int64_t ldc, const float* g_in,
                          const float* g_lp, float* const* bufs, float* g_out, int64_t B, void* stream) {
  if (B < 0) return set_error("naz_ar_flow_bwd_layer: negative batch");
  if (B > 0 && (packed_fwd == nullptr || packed_bwd == nullptr || perm == nullptr || state == nullptr ||
                g_in == nullptr || bufs == nullptr || g_out == nullptr))
    return set_error("naz_ar_flow_bwd_layer: null pointer");
  if (d != nullptr && d->C > 0 && B > 0 && ctx == nullptr)
    return set_error("naz_ar_flow_bwd_layer: conditional flow needs ctx");
  if (d == nullptr || layer < 0 || layer >= d->L) return set_error("naz_ar_flow_bwd_layer: layer out of range");
  if (ar_flow_bwd_packed_bytes(d) < 0) {  // no backward instance: report the descriptor
    int dims[6];
    return ar_flow_bwd_dims(d, dims);
  }
  if (B == 0) return 0;
  NAZ_IMG("naz_ar_flow_bwd_layer", spec_ar(d, IMG_AR_FWD), packed_fwd, 1, 0, 0, body_fwd);
  NAZ_IMG("naz_ar_flow_bwd_layer", spec_ar(d, IMG_AR_BWD), packed_bwd, 1, 0, 0, body_bwd);
  return ar_flow_bwd_layer(d, body_fwd, body_bwd, perm, layer, state, ctx, ldc, g_in, g_lp, bufs, g_out, B,
                           as_stream(stream));
}

// ---- §8b whole-flow entries over the fused kinds ----------------------------------------
int64_t naz_flow_packed_bytes(const naz_flow_desc* d) {
  if (d == nullptr) return -1;
  if (d->kind == NAZ_FLOW_COUPLING) return naz_coupling_packed_bytes(&d->coupling);
  if (d->kind == NAZ_FLOW_AR) return naz_ar_flow_packed_bytes(&d->ar);
  return -1;
}

int64_t naz_workspace_bytes(const naz_flow_desc* d, int64_t B) {
  if (naz_flow_packed_bytes(d) < 0 || B < 0) return -1;
  // the coupling kernels keep every intermediate on chip; the wide autoregressive inverse keeps its
  // hidden layers 2.. in per-wave workspace
  return d->kind == NAZ_FLOW_AR ? ar_flow_workspace_bytes(&d->ar, B, 1) : 0;
}

int naz_flow_log_prob(const naz_flow_desc* d, const void* packed, const float* x, int64_t ldx, const float* ctx,
                      int64_t ldc, const float* low, const float* high, float* out_lp, int64_t B, void* workspace,
                      int64_t workspace_bytes, void* stream) {
  if (d == nullptr) return set_error("naz_flow_log_prob: null descriptor");
  if (d->kind == NAZ_FLOW_COUPLING)
    return naz_coupling_log_prob(&d->coupling, packed, x, ldx, ctx, ldc, low, high, out_lp, B, stream);
  if (d->kind == NAZ_FLOW_AR)
    return naz_ar_flow_log_prob(&d->ar, packed, x, ldx, ctx, ldc, low, high, out_lp, B, workspace, workspace_bytes,
                                stream);
  return set_error("naz_flow_log_prob: unknown flow kind %d", d->kind);
}

int naz_flow_sample(const naz_flow_desc* d, const void* packed, const float* z, int64_t ldz, const float* ctx,
                    int64_t ldc, const float* low, const float* high, float* y, int64_t ldy, float* out_ld, int64_t B,
                    void* stream) {
  if (d == nullptr) return set_error("naz_flow_sample: null descriptor");
  if (d->kind == NAZ_FLOW_COUPLING)
    return naz_coupling_sample(&d->coupling, packed, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, stream);
  if (d->kind == NAZ_FLOW_AR)  // packed = the forward image (naz_ar_flow_pack_fwd_host)
    return naz_ar_flow_sample(&d->ar, packed, z, ldz, ctx, ldc, low, high, y, ldy, out_ld, B, stream);
  return set_error("naz_flow_sample: unknown flow kind %d", d->kind);
}

}  // extern "C"
