// torch.ops.tpamd.* registrations for the fused conv / GEMM engine kernels (conv_mfma.hip).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include "tp_launchers.h"

extern "C" {
hipError_t tp_conv_igemm(const float* x, const uint8_t* x_argmax, const float* w, int B, int H, int W, int Cin,
                         int Cout, int ks, int pooled_m, int unpool, int epi, int cfg, int splits, const float* scale,
                         const float* shift, int relu, float* out, uint8_t* out_argmax, const float* act,
                         float* taylor, int HWo, int tay_group, float* ws, int tay_mode, float* apoz,
                         float slope, hipStream_t st);
int tp_conv_gen_k(int ks, int Cin);
int tp_bn_groups(int P, int C);
hipError_t tp_bn_fwd_train(const float* x, float* y, int P, int C, const float* gamma, const float* beta, float eps,
                           float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* a,
                           float* b, double* ws, hipStream_t st);
hipError_t tp_bn_bwd_train(const float* g, const float* x, float* dx, int P, int C, const float* gamma,
                           const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a, float* k1,
                           float* k2, double* ws, hipStream_t st);
hipError_t tp_bn_fwd_train3(const float* x, float* y, int P, int C, const float* gamma, const float* beta, float eps,
                            float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* a,
                            float* b, double* ws, const float* res, int relu, uint8_t* mko, hipStream_t st);
hipError_t tp_bn_bwd_train3(const float* g, const float* x, float* dx, int P, int C, const float* gamma,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a, float* k1,
                            float* k2, double* ws, const float* ym, float* dres, const uint8_t* mk, hipStream_t st);
hipError_t tp_bn_fwd_train2(const float* x, float* y, int P, int C, const float* gamma, const float* beta, float eps,
                            float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* a,
                            float* b, double* ws, const float* res, int relu, hipStream_t st);
hipError_t tp_bn_bwd_train2(const float* g, const float* x, float* dx, int P, int C, const float* gamma,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a, float* k1,
                            float* k2, double* ws, const float* ym, float* dres, hipStream_t st);
hipError_t tp_conv_wgrad(const float* g, const float* x, float* dw, float* ws, int B, int H, int W, int Cin, int Cout,
                         int ks, int stride, int pad, int Kpad, int cfg, int splits, hipStream_t st);
hipError_t tp_conv_gen2(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks, int stride,
                        int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits, const float* scale,
                        const float* shift, int relu, const float* res, int res_stride, const float* mask,
                        float* apoz, float* out, float* ws, hipStream_t st);
hipError_t tp_conv_gen(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks, int stride,
                       int pad, int cfg, int splits, const float* scale, const float* shift, int relu,
                       const float* res, float* apoz, float* out, float* ws, hipStream_t st);
hipError_t tp_maxpool_nhwc(const float* x, float* y, int B, int H, int W, int C, int k, int s, int pad,
                           hipStream_t st);
hipError_t tp_avgpool_nhwc(const float* x, float* y, int B, int HW, int C, hipStream_t st);
hipError_t tp_maxpool2_nhwc(const float* x, float* y, uint8_t* am, int B, int H, int W, int C, hipStream_t st);
hipError_t tp_unpool2_nhwc(const float* g, const uint8_t* am, float* out, int B, int H, int W, int C, hipStream_t st);
hipError_t tp_conv_first_wave(const float* x, const float* wt, const float* scale, const float* shift, float* out,
                              int B, int Cin, int H, int W, int Cout, int relu, hipStream_t st);
hipError_t tp_conv_first_direct(const float* x, const float* w, const float* scale, const float* shift, float* out,
                                int B, int Cin, int H, int W, int Cout, int relu, hipStream_t st);
int tp_wino_taylor_slots(int H, int W);
int tp_wino_lds_bytes();
int tp_wino_staged_ok(int H, int W, int unpool);
hipError_t tp_nchw_to_nhwc_pad(const float* x, float* y, int B, int C, int H, int W, int Cp, hipStream_t st);
hipError_t tp_conv_wino(const float* x, const uint8_t* x_argmax, const float* u, int B, int H, int W, int C, int K,
                        int unpool, int epi, int splits, int staged, const float* scale, const float* shift, int relu,
                        float* out, uint8_t* out_argmax, const float* act, float* taylor, float* apoz, float* ws,
                        int tay_mode, hipStream_t st);
hipError_t tp_wino_weights(const float* w, float* u, int K, int C, int flip_t, hipStream_t st);
hipError_t tp_wino_weights2(const float* w, float* u, int K, int C, int flip_t, int S0, int S1, hipStream_t st);
hipError_t tp_wino_weights_bf16(const float* w, void* u, int K, int C, int flip_t, int S0, int S1, hipStream_t st);
hipError_t tp_pack_conv_weights_multi(const long long* desc, int n, long long total, hipStream_t st);
hipError_t tp_pack_conv_weight(const float* w, float* out, int O, int I, int KS, int rows, int cols, int cpad, int mode,
                               hipStream_t st);
long long tp_wino_wgrad_ws_elems(int B, int H, int W, int Cin, int Cout, int splits);
hipError_t tp_wino_wgrad(const float* g, const float* x, float* ws, int B, int H, int W, int Cin, int Cout, int cfg,
                         int splits, float* fin, int fin_co, int fin_ci, const long long* fs, hipStream_t st);
hipError_t tp_conv_gen3(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks, int stride,
                        int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits, const float* scale,
                        const float* shift, int relu, const float* res, int res_stride, const float* mask,
                        float* apoz, float* out, float* ws, double* bnpart, hipStream_t st);
int tp_conv_tile_m(int cfg);
long long tp_conv_sk_ws_floats(int cfg, int ks, int transposed, int tay, int M, int N);
hipError_t tp_conv_gen4(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks, int stride,
                        int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits, const float* scale,
                        const float* shift, int relu, const float* res, int res_stride, const float* mask,
                        float* apoz, float* out, float* ws, double* bnpart, float* tay_part, int tay_mode,
                        hipStream_t st);
int tp_conv_gen_tay_slots(int cfg, int HWo);
hipError_t tp_conv_gen5(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks, int stride,
                        int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits, const float* scale,
                        const float* shift, int relu, const float* res, int res_stride, const float* mask,
                        float* apoz, float* out, float* ws, double* bnpart, float* tay_part, int tay_mode,
                        const uint8_t* res_bits, const float* bnb_y, const float* bnb_mean, const float* bnb_invstd,
                        const uint8_t* bnb_bits, hipStream_t st);
hipError_t tp_bn_bwd_train_pre(const float* g, const float* x, float* dx, int P, int C, int Cr, const float* gamma,
                               const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a,
                               float* k1, float* k2, double* ws, const double* pre, int G, const float* ym,
                               float* dres, const uint8_t* mk, hipStream_t st);
hipError_t tp_bn_fwd_train_pre2(const float* x, float* y, int P, int C, int Cr, const float* gamma,
                                const float* beta, float eps, float momentum, float* run_mean, float* run_var,
                                float* mean, float* invstd, float* a, float* b, double* ws, const double* pre, int G,
                                const float* res, int relu, uint8_t* mko, long long* nbt, hipStream_t st);
hipError_t tp_bn_fwd_train5(const float* x, float* y, int P, int C, int Cr, const float* gamma, const float* beta,
                            float eps, float momentum, float* run_mean, float* run_var, float* mean, float* invstd,
                            float* a, float* b, double* ws, const float* res, int relu, uint8_t* mko, long long* nbt,
                            hipStream_t st);
hipError_t tp_bn_bwd_train4(const float* g, const float* x, float* dx, int P, int C, int Cr, const float* gamma,
                            const float* mean, const float* invstd, float* dgamma, float* dbeta, float* a, float* k1,
                            float* k2, double* ws, const float* ym, float* dres, const uint8_t* mk, hipStream_t st);
hipError_t tp_conv_wgrad2(const float* g, const float* x, float* dw, float* ws, int B, int H, int W, int Cin, int Cout,
                          int ks, int stride, int pad, int Kpad, int cfg, int splits, float* fin, int fin_co,
                          int fin_ci, const long long* fs, hipStream_t st);
hipError_t tp_prefix_delta_gemm(const float* T, const float* Wsub, const float* neg_one, const float* Y0, int M, int Kc,
                                int N, int B0, int relu, float slope, int cfg, float* out, hipStream_t st);
hipError_t tp_prefix_tri_operands(const float* z, const float* W, const int* perm, int B, int C, int N, int p0,
                                  int cnt, int Kc, float* T, float* Wsub, hipStream_t st);
hipError_t tp_wino4_weights(const float* w, float* u, int K, int C, int flip_t, int S0, int S1, hipStream_t st);
hipError_t tp_wino4_weights_multi(const long long* desc, int n, long long total, hipStream_t st);
hipError_t tp_wino4_weights_strided(const float* w, float* u, int K, int C, int flip_t, int S0, int S1, long long st0,
                                    long long st1, int st2, int st3, hipStream_t st);
int tp_wino4_u_img();
int tp_wino4_ok(int H, int W, int C, int K);
int tp_wino4_taylor_slots(int S);
int tp_wino4_lds_bytes(int S, int variant);
hipError_t tp_conv_wino4_ko(const float* x, const float* u, int B, int S, int C, int K, int epi, const float* scale,
                           const float* shift, int relu, float* out, uint8_t* out_argmax, const float* act,
                           float* taylor, float* apoz, int tay_mode, int splits, float* ws, int variant,
                           hipStream_t st, const uint8_t* unpool_am, int ko);
hipError_t tp_conv_wino4(const float* x, const float* u, int B, int S, int C, int K, int epi, const float* scale,
                         const float* shift, int relu, float* out, uint8_t* out_argmax, const float* act, float* taylor,
                         float* apoz, int tay_mode, int splits, float* ws, int variant, hipStream_t st,
                         const uint8_t* unpool_am);
}

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define TP_CHECK_HIP(expr)                                                                  \
  do {                                                                                      \
    hipError_t _e = (expr);                                                                 \
    TORCH_CHECK(_e == hipSuccess, "tpamd conv launch failed: ", hipGetErrorString(_e));     \
  } while (0)

void need(const at::Tensor& t, const char* name, int64_t dim) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat, name, " must be a float32 GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(dim < 0 || t.dim() == dim, name, " must have ", dim, " dims, got ", t.dim());
}

const float* opt_ptr(const c10::optional<at::Tensor>& t, int64_t n, const char* name) {
  if (!t.has_value() || !t->defined()) return nullptr;
  need(*t, name, 1);
  TORCH_CHECK(t->numel() == n, name, " must have ", n, " elements");
  // the epilogues read per-channel vectors as float4
  TORCH_CHECK(reinterpret_cast<uintptr_t>(t->data_ptr<float>()) % 16 == 0, name, " must be 16-byte aligned");
  return t->data_ptr<float>();
}

enum { EPI_FWD = 0, EPI_FWD_POOL = 1, EPI_BWD = 2 };

int64_t splits_ws(int64_t splits, int64_t K) {
  const int64_t kt = K / 32;
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, kt));
  const int64_t per = (kt + splits - 1) / splits;
  return (kt + per - 1) / per;
}

// Forward conv / linear: x (B,H,W,Cin) NHWC, w (Cout, K) with K = ks*ks*Cin.
// Returns out (B,H,W,Cout) or pooled (B,H/2,W/2,Cout) + argmax bytes.
std::tuple<at::Tensor, at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w,
                                            const c10::optional<at::Tensor>& scale,
                                            const c10::optional<at::Tensor>& shift, bool relu, bool pool, int64_t ks,
                                            int64_t cfg, int64_t splits, const c10::optional<at::Tensor>& apoz,
                                            double slope) {
  need(x, "x", 4);
  need(w, "w", 2);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = w.size(0);
  TORCH_CHECK(ks == 1 || ks == 3, "ks must be 1 or 3");
  TORCH_CHECK(w.size(1) == ks * ks * Cin, "weight K mismatch: ", w.size(1), " vs ", ks * ks * Cin);
  TORCH_CHECK(Cin % 32 == 0, "Cin must be a multiple of 32");
  TORCH_CHECK(!pool || (H % 2 == 0 && W % 2 == 0), "pooling needs even H, W");
  TORCH_CHECK((cfg >= 0 && cfg <= 6) || (ks == 3 && (cfg == 256 || cfg == 258 || cfg == 259)),
              "bad tile config (bf16 operands: 256 + {0, 2, 3}, 3x3 only)");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* sc = opt_ptr(scale, Cout, "scale");
  const float* sh = opt_ptr(shift, Cout, "shift");
  at::Tensor out, am;
  if (pool) {
    out = at::empty({B, H / 2, W / 2, Cout}, x.options());
    am = at::empty({B, H / 2, W / 2, Cout}, x.options().dtype(at::kByte));
  } else {
    out = at::empty({B, H, W, Cout}, x.options());
  }
  const int64_t sp = splits_ws(splits, ks * ks * Cin);
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * H * W * Cout}, x.options());
  float* ap = nullptr;  // (B, Cout) counts of positive (pre-pool) outputs, accumulated
  if (apoz.has_value() && apoz->defined()) {
    TORCH_CHECK(apoz->is_cuda() && apoz->scalar_type() == at::kFloat && apoz->is_contiguous() &&
                    apoz->numel() == B * Cout, "apoz must be a contiguous float32 (B, Cout) tensor");
    ap = apoz->data_ptr<float>();
  }
  TP_CHECK_HIP(tp_conv_igemm(x.data_ptr<float>(), nullptr, w.data_ptr<float>(), (int)B, (int)H, (int)W, (int)Cin,
                             (int)Cout, (int)ks, pool ? 1 : 0, 0, pool ? EPI_FWD_POOL : EPI_FWD, (int)cfg, (int)sp, sc,
                             sh, relu ? 1 : 0, out.data_ptr<float>(), pool ? am.data_ptr<uint8_t>() : nullptr, nullptr,
                             nullptr, (int)(H * W), 0, sp > 1 ? ws.data_ptr<float>() : nullptr, 0, ap, (float)slope,
                             cur_stream()));
  return {out, am};
}

// dgrad + fused consumer epilogue.
// g: grad w.r.t. the conv output, (B,H,W,Cout); or, with g_argmax, the masked grad at pooled
//    resolution (B,H/2,W/2,Cout) whose full-resolution form is implied by the argmax bytes.
// wt: flipped/transposed weight (Cin, ks*ks*Cout). act: activation at the conv input (B,H,W,Cin).
// taylor (B,Cin) fp32 accumulated atomically with sum_hw -(dL/dact * act) (nullable).
// Returns dL/d(pre-activation) * bn_scale masked by act>0 (B,H,W,Cin), or an empty tensor.
at::Tensor conv_dgrad(const at::Tensor& g, const c10::optional<at::Tensor>& g_argmax, const at::Tensor& wt,
                      const at::Tensor& act, const c10::optional<at::Tensor>& bn_scale,
                      const c10::optional<at::Tensor>& taylor, bool want_out, int64_t ks, int64_t cfg,
                      int64_t splits, int64_t tay_group, int64_t tay_mode, double slope) {
  need(g, "g", 4);
  need(wt, "wt", 2);
  need(act, "act", 4);
  const bool unpool = g_argmax.has_value() && g_argmax->defined();
  const int64_t B = act.size(0), H = act.size(1), W = act.size(2), Cin = act.size(3);
  const int64_t Cout = g.size(3);
  if (unpool) {
    TORCH_CHECK(g.size(1) * 2 == H && g.size(2) * 2 == W, "pooled grad shape mismatch");
    TORCH_CHECK(g_argmax->scalar_type() == at::kByte && g_argmax->sizes() == g.sizes() && g_argmax->is_contiguous(),
                "g_argmax must be uint8 with g's shape");
  } else {
    TORCH_CHECK(g.size(1) == H && g.size(2) == W, "grad shape mismatch");
  }
  TORCH_CHECK(g.size(0) == B, "batch mismatch");
  TORCH_CHECK(wt.size(0) == Cin && wt.size(1) == ks * ks * Cout, "wt must be (Cin, ks*ks*Cout)");
  TORCH_CHECK(Cout % 32 == 0, "Cout must be a multiple of 32 for dgrad");
  TORCH_CHECK(tay_group >= 0 && (tay_group == 0 || Cin % tay_group == 0), "tay_group must divide Cin");
  TORCH_CHECK((cfg >= 0 && cfg <= 6) || (ks == 3 && (cfg == 256 || cfg == 258 || cfg == 259)),
              "bad tile config (bf16 operands: 256 + {0, 2, 3}, 3x3 only)");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  const float* sc = opt_ptr(bn_scale, Cin, "bn_scale");
  float* tay = nullptr;
  if (taylor.has_value() && taylor->defined()) {
    TORCH_CHECK(taylor->is_cuda() && taylor->scalar_type() == at::kFloat && taylor->is_contiguous() &&
                    taylor->numel() > 0 && taylor->numel() % (B * Cin) == 0,
                "taylor must be a contiguous float32 (B, Cin) or (R, B, Cin) GPU tensor (slot 0 is written)");
    tay = taylor->data_ptr<float>();
  }
  at::Tensor out;
  if (want_out) out = at::empty({B, H, W, Cin}, g.options());
  const int64_t sp = splits_ws(splits, ks * ks * Cout);
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * H * W * Cin}, g.options());
  TP_CHECK_HIP(tp_conv_igemm(g.data_ptr<float>(), unpool ? g_argmax->data_ptr<uint8_t>() : nullptr,
                             wt.data_ptr<float>(), (int)B, (int)H, (int)W, (int)Cout, (int)Cin, (int)ks, 0,
                             unpool ? 1 : 0, EPI_BWD, (int)cfg, (int)sp, sc, nullptr, 0,
                             want_out ? out.data_ptr<float>() : nullptr, nullptr, act.data_ptr<float>(), tay,
                             (int)(H * W), (int)tay_group, sp > 1 ? ws.data_ptr<float>() : nullptr, (int)tay_mode,
                             nullptr, (float)slope, cur_stream()));
  return out;
}

// First conv layer (tiny Cin) on the VALU: NCHW input -> NHWC output, BN affine + ReLU fused.
// ``wt``: optional tap-major copy of w, [Cin][3][3][Cout], packed once by the caller (the
// wave-uniform kernel's operand layout); built here per call when absent.
at::Tensor conv_first(const at::Tensor& x, const at::Tensor& w, const at::Tensor& scale, const at::Tensor& shift,
                      bool relu, const c10::optional<at::Tensor>& wt_packed) {
  need(x, "x", 4);
  need(w, "w", 4);
  const int64_t B = x.size(0), Cin = x.size(1), H = x.size(2), W = x.size(3), Cout = w.size(0);
  TORCH_CHECK(w.size(1) == Cin && w.size(2) == 3 && w.size(3) == 3, "w must be (Cout, Cin, 3, 3)");
  need(scale, "scale", 1);
  need(shift, "shift", 1);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto out = at::empty({B, H, W, Cout}, x.options());
  if ((Cout == 16 || Cout == 32 || Cout == 64) && Cin <= 16) {  // wave-uniform weights (scalar loads)
    at::Tensor wt;
    if (wt_packed.has_value() && wt_packed->defined()) {
      wt = *wt_packed;
      need(wt, "wt", 4);
      TORCH_CHECK(wt.size(0) == Cin && wt.size(1) == 3 && wt.size(2) == 3 && wt.size(3) == Cout,
                  "wt must be (Cin, 3, 3, Cout)");
    } else {
      wt = w.permute({1, 2, 3, 0}).contiguous();  // [Cin][3][3][Cout]
    }
    TP_CHECK_HIP(tp_conv_first_wave(x.data_ptr<float>(), wt.data_ptr<float>(), scale.data_ptr<float>(),
                                    shift.data_ptr<float>(), out.data_ptr<float>(), (int)B, (int)Cin, (int)H, (int)W,
                                    (int)Cout, relu ? 1 : 0, cur_stream()));
    return out;
  }
  TP_CHECK_HIP(tp_conv_first_direct(x.data_ptr<float>(), w.data_ptr<float>(), scale.data_ptr<float>(),
                                    shift.data_ptr<float>(), out.data_ptr<float>(), (int)B, (int)Cin, (int)H, (int)W,
                                    (int)Cout, relu ? 1 : 0, cur_stream()));
  return out;
}

// Winograd U images of a 3x3 weight: w (K, C, 3, 3) -> (C/8, K/32, 4096); flip_t: the data-gradient
// operand of the forward weight w (Cout = K', Cin = C', 3, 3) -> images of (C', K') with rotated taps.
// bf16: the bf16 images of the BF kernels (same shape, dtype bfloat16; opt-in compute_dtype).
at::Tensor wino_weights(const at::Tensor& w, bool flip_t, int64_t K, int64_t C, bool bf16) {
  need(w, "w", 4);
  TORCH_CHECK(w.size(2) == 3 && w.size(3) == 3, "w must be (.., .., 3, 3)");
  // K, C: the padded GEMM sizes (0 = the weight's own); the source may be narrower (zero padding)
  if (K <= 0) K = flip_t ? w.size(1) : w.size(0);
  if (C <= 0) C = flip_t ? w.size(0) : w.size(1);
  TORCH_CHECK(K % 32 == 0 && C % 8 == 0, "Winograd images need K % 32 == 0 and C % 8 == 0");
  TORCH_CHECK(flip_t ? (w.size(0) <= C && w.size(1) <= K) : (w.size(0) <= K && w.size(1) <= C),
              "weight wider than the padded GEMM");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(w.device());
  auto u = at::empty({C / 8, K / 32, 4096}, w.options().dtype(bf16 ? at::kBFloat16 : at::kFloat));
  if (bf16)
    TP_CHECK_HIP(tp_wino_weights_bf16(w.data_ptr<float>(), u.data_ptr(), (int)K, (int)C, flip_t ? 1 : 0,
                                      (int)w.size(0), (int)w.size(1), cur_stream()));
  else
    TP_CHECK_HIP(tp_wino_weights2(w.data_ptr<float>(), u.data_ptr<float>(), (int)K, (int)C, flip_t ? 1 : 0,
                                  (int)w.size(0), (int)w.size(1), cur_stream()));
  return u;
}

// Conv weight (O, I, KS, KS) -> a zero-padded GEMM operand (rows, cols): mode 0 forward
// [n][(kh, kw, ci)], 1 stride-1 dgrad [ci][(kh, kw, co)] with flipped taps, 2 strided dgrad
// (natural taps); cpad = channel granule of the column index.
at::Tensor pack_conv_weight(const at::Tensor& w, int64_t rows, int64_t cols, int64_t cpad, int64_t mode) {
  need(w, "w", 4);
  TORCH_CHECK(w.size(2) == w.size(3), "square kernels only");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(w.device());
  auto out = at::empty({rows, cols}, w.options());
  TP_CHECK_HIP(tp_pack_conv_weight(w.data_ptr<float>(), out.data_ptr<float>(), (int)w.size(0), (int)w.size(1),
                                   (int)w.size(2), (int)rows, (int)cols, (int)cpad, (int)mode, cur_stream()));
  return out;
}

// Every operand of ``pack_conv_weight`` for a list of weights in one launch: outs[i] (rows, cols)
// <- ws[i] per cfg[4i:4i+4] = (rows, cols, cpad, mode). ws may be strided (channels_last
// parameters are read in place). The descriptors travel through pinned memory (async copy).
void pack_conv_weights_multi(const std::vector<at::Tensor>& ws, const std::vector<at::Tensor>& outs,
                             const std::vector<int64_t>& cfg) {
  constexpr int D = 14;
  const int64_t n = (int64_t)ws.size();
  TORCH_CHECK(n > 0 && (int64_t)outs.size() == n && (int64_t)cfg.size() == 4 * n,
              "pack_conv_weights_multi: ws, outs and 4 ints per operand");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ws[0].device());
  auto hd = at::empty({n * D}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
  int64_t* h = hd.data_ptr<int64_t>();
  int64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    const at::Tensor& w = ws[i];
    const at::Tensor& o = outs[i];
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(2) == w.size(3) &&
                    w.device() == ws[0].device(), "pack_conv_weights_multi: fp32 (O, I, KS, KS) GPU weights");
    const int64_t rows = cfg[4 * i], cols = cfg[4 * i + 1], cpad = cfg[4 * i + 2], mode = cfg[4 * i + 3];
    const int64_t O = w.size(0), I = w.size(1);
    TORCH_CHECK(mode >= 0 && mode <= 2 && rows > 0 && cols > 0 && cpad > 0 &&
                    (mode == 0 ? (rows >= O && cpad >= I) : (rows >= I && cpad >= O)),
                "pack_conv_weights_multi: bad operand shape");
    TORCH_CHECK(o.is_cuda() && o.scalar_type() == at::kFloat && o.is_contiguous() && o.numel() == rows * cols &&
                    o.device() == w.device(), "pack_conv_weights_multi: out must be a contiguous fp32 (rows, cols)");
    int64_t* d = h + i * D;
    d[0] = reinterpret_cast<int64_t>(w.data_ptr<float>());
    d[1] = reinterpret_cast<int64_t>(o.data_ptr<float>());
    d[2] = total;
    d[3] = O;
    d[4] = I;
    d[5] = w.size(2);
    d[6] = rows;
    d[7] = cols;
    d[8] = cpad;
    d[9] = mode;
    d[10] = w.stride(0);
    d[11] = w.stride(1);
    d[12] = w.stride(2);
    d[13] = w.stride(3);
    if (mode == 0) {
      total += (rows * cols + 4095) / 4096 * 4096;  // next operand on a chunk boundary (PACK_CHUNK)
    } else {  // one 4096-element chunk per 64 x 64 (ci, co) tile of a tap
      TORCH_CHECK(cols == w.size(2) * w.size(2) * cpad, "pack_conv_weights_multi: dgrad operands need cols = KS*KS*cpad");
      total += ((rows + 63) / 64) * w.size(2) * w.size(2) * ((cpad + 63) / 64) * 4096;
    }
  }
  auto dd = hd.to(ws[0].device(), /*non_blocking=*/true);
  TP_CHECK_HIP(tp_pack_conv_weights_multi(reinterpret_cast<const long long*>(dd.data_ptr<int64_t>()), (int)n,
                                          (long long)total, cur_stream()));
}

// Shapley prefix-delta operands: z (B, C) block output, W (N, C) next Linear, perm (n) int32
// permutation; returns T (cnt*B, Kc) lower-triangular gathered activations and Wsub (N, Kc).
std::tuple<at::Tensor, at::Tensor> prefix_tri_operands(const at::Tensor& z, const at::Tensor& w, const at::Tensor& perm,
                                                       int64_t p0, int64_t cnt, int64_t Kc) {
  need(z, "z", 2);
  need(w, "w", 2);
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == at::kInt && perm.is_contiguous() && perm.dim() == 1,
              "perm must be a contiguous int32 GPU vector");
  const int64_t B = z.size(0), C = z.size(1), N = w.size(0);
  TORCH_CHECK(w.size(1) == C, "w must be (N, C) with z's C");
  TORCH_CHECK(cnt >= 1 && Kc >= cnt && Kc % 32 == 0, "need 1 <= cnt <= Kc, Kc % 32 == 0");
  // prefixes p0 .. p0+cnt-1 read perm[p0 .. p0+cnt-2] (the last copy's extra units)
  TORCH_CHECK(p0 >= 0 && p0 + cnt - 1 <= perm.numel() && perm.numel() <= C, "prefix range out of the permutation");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(z.device());
  auto T = at::empty({cnt * B, Kc}, z.options());
  auto Ws = at::empty({N, Kc}, z.options());
  TP_CHECK_HIP(tp_prefix_tri_operands(z.data_ptr<float>(), w.data_ptr<float>(), perm.data_ptr<int>(), (int)B, (int)C,
                                      (int)N, (int)p0, (int)cnt, (int)Kc, T.data_ptr<float>(), Ws.data_ptr<float>(),
                                      cur_stream()));
  return {T, Ws};
}

// out (M, N) = act(Y0[r % B0] - T @ Wsub^T) on the MFMA GEMM (prefix-delta Shapley evaluation).
at::Tensor prefix_delta(const at::Tensor& T, const at::Tensor& wsub, const at::Tensor& neg_one, const at::Tensor& y0,
                        bool relu, double slope, int64_t cfg) {
  need(T, "T", 2);
  need(wsub, "wsub", 2);
  need(y0, "y0", 2);
  const int64_t M = T.size(0), Kc = T.size(1), N = wsub.size(0), B0 = y0.size(0);
  TORCH_CHECK(wsub.size(1) == Kc && y0.size(1) == N, "shape mismatch: T (M, Kc), wsub (N, Kc), y0 (B0, N)");
  TORCH_CHECK(Kc % 32 == 0 && N % 4 == 0 && M % B0 == 0, "need Kc % 32 == 0, N % 4 == 0, M % B0 == 0");
  TORCH_CHECK(cfg >= 0 && cfg <= 6, "bad tile config");
  const float* no = opt_ptr(neg_one, N, "neg_one");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(T.device());
  auto out = at::empty({M, N}, T.options());
  TP_CHECK_HIP(tp_prefix_delta_gemm(T.data_ptr<float>(), wsub.data_ptr<float>(), no, y0.data_ptr<float>(), (int)M,
                                    (int)Kc, (int)N, (int)B0, relu ? 1 : 0, (float)slope, (int)cfg,
                                    out.data_ptr<float>(), cur_stream()));
  return out;
}

int64_t wino_splits(int64_t splits, int64_t C) {
  const int64_t chunks = C / 8;
  splits = std::max<int64_t>(1, std::min<int64_t>(splits, chunks));
  const int64_t per = (chunks + splits - 1) / splits;
  return (chunks + per - 1) / per;
}

// fp32 images, or bf16 ones (the BF kernels; staged input modes only): returns the staged-flag bit
int need_u(const at::Tensor& u, int64_t C, int64_t K) {
  TORCH_CHECK(u.is_cuda() && u.is_contiguous() && u.dim() == 3 &&
                  (u.scalar_type() == at::kFloat || u.scalar_type() == at::kBFloat16),
              "u must be a contiguous float32 or bfloat16 GPU tensor (C/8, K/32, 4096)");
  TORCH_CHECK(C % 8 == 0 && K % 32 == 0 && u.size(0) == C / 8 && u.size(1) == K / 32 && u.size(2) == 4096,
              "u must be the Winograd U images (C/8, K/32, 4096) = (", C / 8, ", ", K / 32, ", 4096), got ",
              u.sizes());
  return u.scalar_type() == at::kBFloat16 ? 2 : 0;
}

// Winograd F(2x2,3x3) forward: x (B,H,W,C) NHWC, u (16, C, K) from winograd_weights().
std::tuple<at::Tensor, at::Tensor> conv_wino_fwd(const at::Tensor& x, const at::Tensor& u,
                                                 const c10::optional<at::Tensor>& scale,
                                                 const c10::optional<at::Tensor>& shift, bool relu, bool pool,
                                                 int64_t splits, bool staged, const c10::optional<at::Tensor>& apoz) {
  need(x, "x", 4);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), K = u.size(1) * 32;
  const int ubf = need_u(u, C, K);
  TORCH_CHECK(!ubf || staged, "bf16 U images need the staged kernels");
  TORCH_CHECK(!pool || (H % 2 == 0 && W % 2 == 0), "Winograd with pooling needs even H, W");
  TORCH_CHECK(C % 8 == 0 && K % 32 == 0, "Winograd needs C % 8 == 0 and K % 32 == 0");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* sc = opt_ptr(scale, K, "scale");
  const float* sh = opt_ptr(shift, K, "shift");
  at::Tensor out, am;
  if (pool) {
    out = at::empty({B, H / 2, W / 2, K}, x.options());
    am = at::empty({B, H / 2, W / 2, K}, x.options().dtype(at::kByte));
  } else {
    out = at::empty({B, H, W, K}, x.options());
  }
  const int64_t sp = wino_splits(splits, C);
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * H * W * K}, x.options());
  float* ap = nullptr;
  if (apoz.has_value() && apoz->defined()) {
    TORCH_CHECK(apoz->is_cuda() && apoz->scalar_type() == at::kFloat && apoz->is_contiguous() &&
                    apoz->numel() == B * K, "apoz must be a contiguous float32 (B, K) tensor");
    ap = apoz->data_ptr<float>();
  }
  TP_CHECK_HIP(tp_conv_wino(x.data_ptr<float>(), nullptr, static_cast<const float*>(u.data_ptr()), (int)B, (int)H,
                            (int)W, (int)C, (int)K, 0, pool ? EPI_FWD_POOL : EPI_FWD, (int)sp, (staged ? 1 : 0) | ubf,
                            sc, sh, relu ? 1 : 0,
                            out.data_ptr<float>(),
                            pool ? am.data_ptr<uint8_t>() : nullptr, nullptr, nullptr, ap,
                            sp > 1 ? ws.data_ptr<float>() : nullptr, 0, cur_stream()));
  return {out, am};
}

// Winograd dgrad with the conv_dgrad epilogue contract; ut = winograd_weights of the
// flipped/transposed kernel, (16, Cout, Cin).
at::Tensor conv_wino_dgrad(const at::Tensor& g, const c10::optional<at::Tensor>& g_argmax, const at::Tensor& ut,
                           const at::Tensor& act, const c10::optional<at::Tensor>& bn_scale,
                           const c10::optional<at::Tensor>& taylor, bool want_out, int64_t splits, bool staged,
                           int64_t tay_mode) {
  need(g, "g", 4);
  need(act, "act", 4);
  const bool unpool = g_argmax.has_value() && g_argmax->defined();
  const int64_t B = act.size(0), H = act.size(1), W = act.size(2), Cin = act.size(3), Cout = g.size(3);
  const int ubf = need_u(ut, Cout, Cin);
  TORCH_CHECK(!ubf || staged, "bf16 U images need the staged kernels");
  if (unpool) {
    TORCH_CHECK(g.size(1) * 2 == H && g.size(2) * 2 == W, "pooled grad shape mismatch");
    TORCH_CHECK(g_argmax->scalar_type() == at::kByte && g_argmax->sizes() == g.sizes() && g_argmax->is_contiguous(),
                "g_argmax must be uint8 with g's shape");
  } else {
    TORCH_CHECK(g.size(1) == H && g.size(2) == W, "grad shape mismatch");
  }
  TORCH_CHECK(g.size(0) == B, "batch mismatch");
  TORCH_CHECK(!unpool || (H % 2 == 0 && W % 2 == 0), "Winograd with unpooling needs even H, W");
  TORCH_CHECK(Cout % 8 == 0 && Cin % 32 == 0, "Winograd dgrad needs Cout % 8 == 0 and Cin % 32 == 0");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  const float* sc = opt_ptr(bn_scale, Cin, "bn_scale");
  float* tay = nullptr;
  if (taylor.has_value() && taylor->defined()) {
    const int64_t R = tp_wino_taylor_slots((int)H, (int)W);
    TORCH_CHECK(taylor->is_cuda() && taylor->scalar_type() == at::kFloat && taylor->is_contiguous() &&
                    taylor->numel() % (B * Cin) == 0 && taylor->numel() >= R * B * Cin,
                "taylor must be a contiguous float32 (R', B, Cin) GPU tensor with R' >= ", R,
                " partial slots (winograd_taylor_slots)");
    tay = taylor->data_ptr<float>();
  }
  at::Tensor out;
  if (want_out) out = at::empty({B, H, W, Cin}, g.options());
  const int64_t sp = wino_splits(splits, Cout);
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * H * W * Cin}, g.options());
  TP_CHECK_HIP(tp_conv_wino(g.data_ptr<float>(), unpool ? g_argmax->data_ptr<uint8_t>() : nullptr,
                            static_cast<const float*>(ut.data_ptr()), (int)B, (int)H, (int)W, (int)Cout, (int)Cin,
                            unpool ? 1 : 0, EPI_BWD, (int)sp, (staged ? 1 : 0) | ubf, sc, nullptr, 0, want_out ? out.data_ptr<float>() : nullptr, nullptr,
                            act.data_ptr<float>(), tay, nullptr, sp > 1 ? ws.data_ptr<float>() : nullptr,
                            (int)tay_mode, cur_stream()));
  return out;
}

// ---- Winograd F(4x4,3x3) (wino4.hip): square 4/8/16/32-pixel maps --------------------------------
at::Tensor wino4_weights(const at::Tensor& w, bool flip_t, int64_t K, int64_t C) {
  // strided weights welcome (channels_last parameters are read in place)
  TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4, "w must be a 4-d float32 GPU tensor");
  TORCH_CHECK(w.stride(0) > 0 && w.stride(1) > 0 && w.stride(2) > 0 && w.stride(3) > 0, "w: positive strides only");
  TORCH_CHECK(w.size(2) == 3 && w.size(3) == 3, "w must be (.., .., 3, 3)");
  if (K <= 0) K = flip_t ? w.size(1) : w.size(0);
  if (C <= 0) C = flip_t ? w.size(0) : w.size(1);
  TORCH_CHECK(K % 32 == 0 && C % 8 == 0, "F(4x4) U images need K % 32 == 0 and C % 8 == 0");
  TORCH_CHECK(flip_t ? (w.size(0) <= C && w.size(1) <= K) : (w.size(0) <= K && w.size(1) <= C),
              "weight wider than the padded GEMM");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(w.device());
  auto u = at::empty({C / 8, K / 32, (int64_t)tp_wino4_u_img()}, w.options());
  TP_CHECK_HIP(tp_wino4_weights_strided(w.data_ptr<float>(), u.data_ptr<float>(), (int)K, (int)C, flip_t ? 1 : 0,
                                        (int)w.size(0), (int)w.size(1), w.stride(0), w.stride(1), (int)w.stride(2),
                                        (int)w.stride(3), cur_stream()));
  return u;
}

void need_u4(const at::Tensor& u, int64_t C, int64_t K);

// F(4x4) U images of many 3x3 weights in one launch: us[i] <- ws[i] per cfg[3i:3i+3] = (K, C,
// flip_t) (the padded GEMM widths, as wino4_weights). ws may be strided (channels_last).
void wino4_weights_multi(const std::vector<at::Tensor>& ws, const std::vector<at::Tensor>& us,
                         const std::vector<int64_t>& cfg) {
  constexpr int D = 12;
  const int64_t n = (int64_t)ws.size();
  TORCH_CHECK(n > 0 && (int64_t)us.size() == n && (int64_t)cfg.size() == 3 * n,
              "wino4_weights_multi: ws, us and 3 ints per operand");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ws[0].device());
  auto hd = at::empty({n * D}, at::TensorOptions().dtype(at::kLong).pinned_memory(true));
  int64_t* h = hd.data_ptr<int64_t>();
  int64_t total = 0;
  for (int64_t i = 0; i < n; ++i) {
    const at::Tensor& w = ws[i];
    const int64_t K = cfg[3 * i], C = cfg[3 * i + 1], flip = cfg[3 * i + 2];
    TORCH_CHECK(w.is_cuda() && w.scalar_type() == at::kFloat && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 &&
                    w.device() == ws[0].device() && w.stride(0) > 0 && w.stride(1) > 0 && w.stride(2) > 0 &&
                    w.stride(3) > 0, "wino4_weights_multi: fp32 (O, I, 3, 3) GPU weights");
    TORCH_CHECK(K > 0 && C > 0 && K % 32 == 0 && C % 8 == 0 &&
                    (flip ? (w.size(0) <= C && w.size(1) <= K) : (w.size(0) <= K && w.size(1) <= C)),
                "wino4_weights_multi: bad padded widths");
    need_u4(us[i], C, K);
    TORCH_CHECK(us[i].device() == w.device(), "wino4_weights_multi: u on w's device");
    int64_t* d = h + i * D;
    d[0] = reinterpret_cast<int64_t>(w.data_ptr<float>());
    d[1] = reinterpret_cast<int64_t>(us[i].data_ptr<float>());
    d[2] = total;
    d[3] = K;
    d[4] = C;
    d[5] = flip ? 1 : 0;
    d[6] = w.size(0);
    d[7] = w.size(1);
    d[8] = w.stride(0);
    d[9] = w.stride(1);
    d[10] = w.stride(2);
    d[11] = w.stride(3);
    total += C * K;  // a multiple of 256: every block stays inside one operand
  }
  auto dd = hd.to(ws[0].device(), /*non_blocking=*/true);
  TP_CHECK_HIP(tp_wino4_weights_multi(reinterpret_cast<const long long*>(dd.data_ptr<int64_t>()), (int)n,
                                      (long long)total, cur_stream()));
}

void need_u4(const at::Tensor& u, int64_t C, int64_t K) {
  need(u, "u", 3);
  TORCH_CHECK(C % 8 == 0 && K % 32 == 0 && u.size(0) == C / 8 && u.size(1) == K / 32 && u.size(2) == tp_wino4_u_img(),
              "u must be the F(4x4) U images (C/8, K/32, ", tp_wino4_u_img(), "), got ", u.sizes());
}

std::tuple<at::Tensor, at::Tensor> conv_wino4_fwd(const at::Tensor& x, const at::Tensor& u,
                                                  const c10::optional<at::Tensor>& scale,
                                                  const c10::optional<at::Tensor>& shift, bool relu, bool pool,
                                                  const c10::optional<at::Tensor>& apoz, int64_t splits,
                                                  int64_t variant, int64_t ko) {
  need(x, "x", 4);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3), Kc = u.size(1) * 32;
  need_u4(u, C, Kc);
  TORCH_CHECK(tp_wino4_ok((int)H, (int)W, (int)C, (int)Kc), "F(4x4) Winograd needs square 4/8/16/32 (or, split-points "
              "variant 3 without pooling, 56/28/14/7) maps, C % 8 == 0, "
              "K % 32 == 0; got ", x.sizes(), " K=", Kc);
  // ko: stored output channels (pruned widths: the U images / MFMAs are 32-padded, HBM rows are not)
  const int64_t K = ko > 0 ? ko : Kc;
  TORCH_CHECK(K % 4 == 0 && K <= Kc && K > Kc - 32, "ko must be a multiple of 4 in (K - 32, K]; got ko=", ko, " K=", Kc);
  TORCH_CHECK(K == Kc || splits <= 1, "ko < K needs one K pass (splits=1)");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* sc = opt_ptr(scale, K, "scale");
  const float* sh = opt_ptr(shift, K, "shift");
  at::Tensor out, am;
  if (pool) {
    out = at::empty({B, H / 2, W / 2, K}, x.options());
    am = at::empty({B, H / 2, W / 2, K}, x.options().dtype(at::kByte));
  } else {
    out = at::empty({B, H, W, K}, x.options());
  }
  float* ap = nullptr;
  if (apoz.has_value() && apoz->defined()) {
    TORCH_CHECK(apoz->is_cuda() && apoz->scalar_type() == at::kFloat && apoz->is_contiguous() &&
                    apoz->numel() == B * K, "apoz must be a contiguous float32 (B, K) tensor");
    ap = apoz->data_ptr<float>();
  }
  const int64_t sp = std::max<int64_t>(1, std::min<int64_t>(splits, C / 8));
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * H * W * K}, x.options());
  TP_CHECK_HIP(tp_conv_wino4_ko(x.data_ptr<float>(), u.data_ptr<float>(), (int)B, (int)H, (int)C, (int)Kc,
                                pool ? EPI_FWD_POOL : EPI_FWD, sc, sh, relu ? 1 : 0, out.data_ptr<float>(),
                                pool ? am.data_ptr<uint8_t>() : nullptr, nullptr, nullptr, ap, 0, (int)sp,
                                sp > 1 ? ws.data_ptr<float>() : nullptr, (int)variant, cur_stream(), nullptr, (int)K));
  return {out, am};
}

// F(4x4) dgrad with the conv_wino_dgrad epilogue contract (input: the unpooled grad). unpool_am
// (B, H, W, Cin) uint8, with want_out and one K pass: the output is written unpooled through those
// 2x2-pool argmax bytes at (B, 2H, 2W, Cin) — the operand of the previous layer's data gradient
at::Tensor conv_wino4_dgrad(const at::Tensor& g, const at::Tensor& ut, const at::Tensor& act,
                            const c10::optional<at::Tensor>& bn_scale, const c10::optional<at::Tensor>& taylor,
                            bool want_out, int64_t tay_mode, int64_t splits, int64_t variant,
                            const c10::optional<at::Tensor>& unpool_am) {
  need(g, "g", 4);
  need(act, "act", 4);
  // Cin: the stored input-gradient channels (act's width); the U images cover Cin rounded up to 32
  const int64_t B = act.size(0), H = act.size(1), W = act.size(2), Cin = act.size(3), Cout = g.size(3);
  const int64_t Kc = ut.dim() == 3 ? ut.size(1) * 32 : 0;
  need_u4(ut, Cout, Kc);
  TORCH_CHECK(Cin % 4 == 0 && Cin <= Kc && Cin > Kc - 32, "act width must be the U images' output width up to its "
              "32-granule; got ", Cin, " vs ", Kc);
  TORCH_CHECK(g.size(0) == B && g.size(1) == H && g.size(2) == W, "grad shape mismatch");
  TORCH_CHECK(tp_wino4_ok((int)H, (int)W, (int)Cout, (int)Kc), "F(4x4) dgrad needs square 4/8/16/32/56/28/14/7 maps, "
              "Cout % 8 == 0, Cin % 32 == 0");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  const float* sc = opt_ptr(bn_scale, Cin, "bn_scale");
  float* tay = nullptr;
  if (taylor.has_value() && taylor->defined()) {
    const int64_t R = tp_wino4_taylor_slots((int)H);
    TORCH_CHECK(taylor->is_cuda() && taylor->scalar_type() == at::kFloat && taylor->is_contiguous() &&
                    taylor->numel() % (B * Cin) == 0 && taylor->numel() >= R * B * Cin,
                "taylor must be a contiguous float32 (R', B, Cin) GPU tensor with R' >= ", R, " partial slots");
    tay = taylor->data_ptr<float>();
  }
  const int64_t sp = std::max<int64_t>(1, std::min<int64_t>(splits, Cout / 8));
  TORCH_CHECK(Cin == Kc || sp == 1, "an unpadded output width needs one K pass (splits=1)");
  const uint8_t* unp = nullptr;
  if (unpool_am.has_value() && unpool_am->defined()) {
    const auto& m = *unpool_am;
    TORCH_CHECK(want_out && sp == 1, "fused unpooling needs want_out and one K pass (splits=1)");
    TORCH_CHECK(m.is_cuda() && m.scalar_type() == at::kByte && m.is_contiguous() && m.dim() == 4 && m.size(0) == B &&
                    m.size(1) == H && m.size(2) == W && m.size(3) == Cin,
                "unpool_am must be contiguous uint8 (B, H, W, Cin) argmax bytes on the GPU");
    unp = m.data_ptr<uint8_t>();
  }
  at::Tensor out;
  if (want_out) out = unp ? at::empty({B, 2 * H, 2 * W, Cin}, g.options()) : at::empty({B, H, W, Cin}, g.options());
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * H * W * Cin}, g.options());
  TP_CHECK_HIP(tp_conv_wino4_ko(g.data_ptr<float>(), ut.data_ptr<float>(), (int)B, (int)H, (int)Cout, (int)Kc,
                                EPI_BWD, sc, nullptr, 0, want_out ? out.data_ptr<float>() : nullptr, nullptr,
                                act.data_ptr<float>(), tay, nullptr, (int)tay_mode, (int)sp,
                                sp > 1 ? ws.data_ptr<float>() : nullptr, (int)variant, cur_stream(), unp, (int)Cin));
  return out;
}

}  // namespace

int64_t wino_taylor_slots(int64_t H, int64_t W) { return tp_wino_taylor_slots((int)H, (int)W); }

// Stream-K fixup workspace of a GEN conv launch whose cfg carries the stream-K flag (32): undefined
// when the flag is absent or stream-K does not apply at this shape (the launcher then runs the
// data-parallel grid).
static constexpr int64_t kCfgSK = 32;
static at::Tensor sk_workspace(int64_t cfg, int64_t ks, bool transposed, bool tay, int64_t M, int64_t N,
                        const at::TensorOptions& o) {
  if (cfg < 0 || !(cfg & kCfgSK)) return at::Tensor();
  const long long n = tp_conv_sk_ws_floats((int)(cfg & ~kCfgSK), (int)ks, transposed ? 1 : 0, tay ? 1 : 0, (int)M,
                                           (int)N);
  return n > 0 ? at::empty({(int64_t)n}, o) : at::Tensor();
}

// General strided conv forward (ResNet): x NHWC (B,H,W,Cin) with Cin % 32 == 0 (ks 1 or 3) or
// Cin == 4 (ks 7, padded stem input); w (Cout, K) with K = conv_gen_k(ks, Cin), k = (kh,kw,ci).
// Epilogue: out = relu?(acc*scale + shift + res); apoz (B, Cout) += count(out > 0).
at::Tensor conv_gen(const at::Tensor& x, const at::Tensor& w, const c10::optional<at::Tensor>& scale,
                    const c10::optional<at::Tensor>& shift, bool relu, const c10::optional<at::Tensor>& res,
                    const c10::optional<at::Tensor>& apoz, int64_t ks, int64_t stride, int64_t pad, int64_t cfg,
                    int64_t splits) {
  need(x, "x", 4);
  need(w, "w", 2);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = w.size(0);
  TORCH_CHECK((Cin % 4 == 0 && Cin >= 8 && (ks == 1 || ks == 3 || ks == 5)) ||
                  (Cin == 4 && (ks == 3 || ks == 5 || ks == 7)),
              "conv_gen supports ks 1/3/5 with Cin % 4 == 0 (>= 8), or ks 3/5/7 with a 4-channel input");
  TORCH_CHECK(w.size(1) == tp_conv_gen_k((int)ks, (int)Cin), "weight K mismatch");
  TORCH_CHECK(stride >= 1 && pad >= 0, "bad stride/pad");
  TORCH_CHECK(Cout % 4 == 0, "conv_gen needs Cout % 4 == 0");
  const int64_t Ho = (H + 2 * pad - ks) / stride + 1, Wo = (W + 2 * pad - ks) / stride + 1;
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* sc = opt_ptr(scale, Cout, "scale");
  const float* sh = opt_ptr(shift, Cout, "shift");
  const float* rp = nullptr;
  if (res.has_value() && res->defined()) {
    need(*res, "res", 4);
    TORCH_CHECK(res->size(0) == B && res->size(1) == Ho && res->size(2) == Wo && res->size(3) == Cout,
                "res must be (B, Ho, Wo, Cout)");
    rp = res->data_ptr<float>();
  }
  float* ap = nullptr;
  if (apoz.has_value() && apoz->defined()) {
    TORCH_CHECK(apoz->is_cuda() && apoz->scalar_type() == at::kFloat && apoz->is_contiguous() &&
                    apoz->numel() == B * Cout, "apoz must be a contiguous float32 (B, Cout) tensor");
    ap = apoz->data_ptr<float>();
  }
  auto out = at::empty({B, Ho, Wo, Cout}, x.options());
  const int64_t K = w.size(1), kt = K / 32;
  int64_t sp = std::max<int64_t>(1, std::min<int64_t>(splits, kt));
  const int64_t per = (kt + sp - 1) / sp;
  sp = (kt + per - 1) / per;
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * Ho * Wo * Cout}, x.options());
  int64_t cf = cfg;
  if (sp == 1 && Cin != 4) {
    ws = sk_workspace(cfg, ks, false, false, B * Ho * Wo, Cout, x.options());
    if (!ws.defined()) cf = cfg & ~kCfgSK;
  } else if (cfg >= 0) {
    cf = cfg & ~kCfgSK;
  }
  TP_CHECK_HIP(tp_conv_gen(x.data_ptr<float>(), w.data_ptr<float>(), (int)B, (int)H, (int)W, (int)Cin, (int)Cout,
                           (int)ks, (int)stride, (int)pad, (int)cf, (int)sp, sc, sh, relu ? 1 : 0, rp, ap,
                           out.data_ptr<float>(), ws.defined() ? ws.data_ptr<float>() : nullptr, cur_stream()));
  return out;
}

int64_t conv_gen_k(int64_t ks, int64_t Cin) { return tp_conv_gen_k((int)ks, (int)Cin); }

// NHWC k x k / stride s / padding p max-pool (NaN-propagating, padded taps skipped)
at::Tensor maxpool_nhwc(const at::Tensor& x, int64_t k, int64_t s, int64_t pad) {
  need(x, "x", 4);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(C % 4 == 0, "maxpool_nhwc needs C % 4 == 0");
  const int64_t Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({B, Ho, Wo, C}, x.options());
  TP_CHECK_HIP(tp_maxpool_nhwc(x.data_ptr<float>(), y.data_ptr<float>(), (int)B, (int)H, (int)W, (int)C, (int)k,
                               (int)s, (int)pad, cur_stream()));
  return y;
}

// NHWC global average pool -> (B, C)
at::Tensor avgpool_nhwc(const at::Tensor& x) {
  need(x, "x", 4);
  const int64_t B = x.size(0), HW = x.size(1) * x.size(2), C = x.size(3);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({B, C}, x.options());
  TP_CHECK_HIP(tp_avgpool_nhwc(x.data_ptr<float>(), y.data_ptr<float>(), (int)B, (int)HW, (int)C, cur_stream()));
  return y;
}

// NHWC 2x2/stride-2 max-pool (NaN-propagating) -> (pooled, argmax bytes)
std::tuple<at::Tensor, at::Tensor> maxpool2_nhwc(const at::Tensor& x) {
  need(x, "x", 4);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0, "maxpool2 needs even H, W");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({B, H / 2, W / 2, C}, x.options());
  auto am = at::empty({B, H / 2, W / 2, C}, x.options().dtype(at::kByte));
  TP_CHECK_HIP(tp_maxpool2_nhwc(x.data_ptr<float>(), y.data_ptr<float>(), am.data_ptr<uint8_t>(), (int)B, (int)H,
                                (int)W, (int)C, cur_stream()));
  return {y, am};
}

// inverse of maxpool2_nhwc: scatter the pooled gradient to the argmax positions
at::Tensor unpool2_nhwc(const at::Tensor& g, const at::Tensor& am) {
  need(g, "g", 4);
  TORCH_CHECK(am.scalar_type() == at::kByte && am.sizes() == g.sizes() && am.is_contiguous(), "am must match g");
  const int64_t B = g.size(0), H = g.size(1) * 2, W = g.size(2) * 2, C = g.size(3);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  auto out = at::empty({B, H, W, C}, g.options());
  TP_CHECK_HIP(tp_unpool2_nhwc(g.data_ptr<float>(), am.data_ptr<uint8_t>(), out.data_ptr<float>(), (int)B, (int)H,
                               (int)W, (int)C, cur_stream()));
  return out;
}

// NCHW -> NHWC with the channel dim zero-padded to Cp (first-layer input of the MFMA kernels).
at::Tensor nchw_to_nhwc_pad(const at::Tensor& x, int64_t Cp) {
  need(x, "x", 4);
  const int64_t B = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  TORCH_CHECK(Cp >= C && Cp % 4 == 0, "Cp must be >= C and a multiple of 4");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({B, H, W, Cp}, x.options());
  TP_CHECK_HIP(tp_nchw_to_nhwc_pad(x.data_ptr<float>(), y.data_ptr<float>(), (int)B, (int)C, (int)H, (int)W, (int)Cp,
                                   cur_stream()));
  return y;
}

// Data gradient of a ResNet conv for the backward engine: g (B, H, W, C = forward Cout) NHWC,
// wt (N = forward Cin, ks*ks*C) with k = (kh, kw, co) and the BN scale folded into co.
// transposed: output (B, Ho, Wo, N) gathers y pixel ((oh + pad - kh)/stride, ...) (strided
// conv dgrad); otherwise a plain stride-1 conv of g (1x1, or 3x3 with flipped taps).
// Epilogue: v (+ res, res_stride-scattered) then out = mask > 0 ? v : 0 when mask is given.
at::Tensor conv_gen_bwd(const at::Tensor& g, const at::Tensor& wt, const c10::optional<at::Tensor>& res,
                        int64_t res_stride, const c10::optional<at::Tensor>& mask, int64_t ks, int64_t stride,
                        int64_t pad, int64_t Ho, int64_t Wo, bool transposed, int64_t cfg, int64_t splits,
                        const c10::optional<at::Tensor>& taylor, int64_t tay_mode) {
  need(g, "g", 4);
  need(wt, "wt", 2);
  const int64_t B = g.size(0), H = g.size(1), W = g.size(2), C = g.size(3), N = wt.size(0);
  TORCH_CHECK(C % 4 == 0 && C >= 8 && (ks == 1 || ks == 3 || (ks == 5 && !transposed)),
              "conv_gen_bwd needs C % 4 == 0 (>= 8) and ks 1/3 (5 for stride-1 convs)");
  TORCH_CHECK(wt.size(1) == tp_conv_gen_k((int)ks, (int)C), "wt must be (N, ks*ks*ceil32(C))");
  TORCH_CHECK(N % 4 == 0 && res_stride >= 1 && stride >= 1 && pad >= 0, "bad N/stride/pad");
  if (!transposed) {
    TORCH_CHECK(stride == 1, "non-transposed conv_gen_bwd is stride 1");
    Ho = (H + 2 * pad - ks) + 1;
    Wo = (W + 2 * pad - ks) + 1;
  } else {
    TORCH_CHECK((Ho + 2 * pad - ks) / stride + 1 == H && (Wo + 2 * pad - ks) / stride + 1 == W,
                "Ho/Wo inconsistent with the forward conv geometry");
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  const float* rp = nullptr;
  if (res.has_value() && res->defined()) {
    need(*res, "res", 4);
    const int64_t Hr = (Ho + res_stride - 1) / res_stride, Wr = (Wo + res_stride - 1) / res_stride;
    TORCH_CHECK(res->size(0) == B && res->size(1) == Hr && res->size(2) == Wr && res->size(3) == N,
                "res must be (B, ceil(Ho/s), ceil(Wo/s), N)");
    rp = res->data_ptr<float>();
  }
  const float* mp = nullptr;
  if (mask.has_value() && mask->defined()) {
    need(*mask, "mask", 4);
    TORCH_CHECK(mask->size(0) == B && mask->size(1) == Ho && mask->size(2) == Wo && mask->size(3) == N,
                "mask must be (B, Ho, Wo, N)");
    mp = mask->data_ptr<float>();
  }
  auto out = at::empty({B, Ho, Wo, N}, g.options());
  const int64_t kt = wt.size(1) / 32;
  int64_t sp = transposed ? 1 : std::max<int64_t>(1, std::min<int64_t>(splits, kt));
  const int64_t per = (kt + sp - 1) / sp;
  sp = (kt + per - 1) / per;
  float* tp_ = nullptr;
  if (taylor.has_value() && taylor->defined()) {
    // fused Taylor / Sensitivity partials (R, B, N) of the masked output: a 1x1 stride-1 dgrad
    // (one K pass), or a transposed 3x3 stride-2 one at even Ho / Wo (the parity row order: one
    // slot range per stride phase, R = 4 x the slots of an Ho/2 x Wo/2 group)
    const bool t3 = transposed && ks == 3 && stride == 2 && Ho % 2 == 0 && Wo % 2 == 0;
    const int R = t3 ? 4 * tp_conv_gen_tay_slots((int)cfg, (int)(Ho * Wo / 4))
                     : tp_conv_gen_tay_slots((int)cfg, (int)(Ho * Wo));
    TORCH_CHECK(((!transposed && ks == 1) || t3) && mp != nullptr && sp == 1 && R > 0,
                "conv_gen_bwd taylor partials need a mask and a 1x1 stride-1 dgrad (one K pass) or a transposed "
                "3x3 stride-2 dgrad at even output size, and a tile config spanning <= 4 row groups");
    TORCH_CHECK(taylor->is_cuda() && taylor->scalar_type() == at::kFloat && taylor->is_contiguous() &&
                    taylor->numel() == (int64_t)R * B * N,
                "taylor must be a contiguous float32 (R, B, N) GPU tensor with R = ", R);
    tp_ = taylor->data_ptr<float>();
  }
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * B * Ho * Wo * N}, g.options());
  int64_t cf = cfg;
  if (sp == 1 && !transposed) {
    ws = sk_workspace(cfg, ks, false, tp_ != nullptr, B * Ho * Wo, N, g.options());
    if (!ws.defined()) cf = cfg & ~kCfgSK;
  } else if (cfg >= 0) {
    cf = cfg & ~kCfgSK;
  }
  TP_CHECK_HIP(tp_conv_gen4(g.data_ptr<float>(), wt.data_ptr<float>(), (int)B, (int)H, (int)W, (int)C, (int)N,
                            (int)ks, (int)stride, (int)pad, transposed ? 1 : 0, (int)Ho, (int)Wo, (int)cf, (int)sp,
                            nullptr, nullptr, 0, rp, (int)res_stride, mp, nullptr, out.data_ptr<float>(),
                            ws.defined() ? ws.data_ptr<float>() : nullptr, nullptr, tp_, (int)tay_mode,
                            cur_stream()));
  return out;
}

int64_t conv_gen_tay_slots(int64_t cfg, int64_t HWo) { return tp_conv_gen_tay_slots((int)cfg, (int)HWo); }

static const uint8_t* bit_mask_ptr(const c10::optional<at::Tensor>& t, int64_t elems, const at::Tensor& like,
                                   const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kByte && t->is_contiguous() && t->numel() == (elems + 3) / 4 &&
                  t->device() == like.device(),
              what, " must be a ReLU bit mask of ceil(elements / 4) uint8 on the device");
  return t->data_ptr<uint8_t>();
}

// Data gradient of a 1x1 stride-1 conv (the training path's residual-block conv1) with the two
// fusions of a bottleneck's backward (tp_conv_gen5):
//   res_bits: ``res`` is the raw gradient of the block output's ReLU, masked here by its bit mask;
//   bn_y / bn_mean / bn_invstd (/ bn_bits): the output gradient reaches a BatchNorm (+ ReLU) whose
//     backward statistics (sum gm, sum gm * xhat) come back per M tile, [tiles][2][N] fp64.
// Returns (dx (B, H, W, N), tile statistics or an empty tensor).
std::tuple<at::Tensor, at::Tensor> conv_gen_bwd_bn(const at::Tensor& g, const at::Tensor& wt,
                                                   const c10::optional<at::Tensor>& res, int64_t res_stride,
                                                   const c10::optional<at::Tensor>& res_bits,
                                                   const c10::optional<at::Tensor>& bn_y,
                                                   const c10::optional<at::Tensor>& bn_mean,
                                                   const c10::optional<at::Tensor>& bn_invstd,
                                                   const c10::optional<at::Tensor>& bn_bits, int64_t cfg) {
  need(g, "g", 4);
  need(wt, "wt", 2);
  const int64_t B = g.size(0), H = g.size(1), W = g.size(2), C = g.size(3), N = wt.size(0), M = B * H * W;
  TORCH_CHECK(C % 4 == 0 && C >= 8 && N % 4 == 0, "conv_gen_bwd_bn needs C % 4 == 0 (>= 8) and N % 4 == 0");
  TORCH_CHECK(wt.size(1) == tp_conv_gen_k(1, (int)C), "wt must be (N, ceil32(C))");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  TORCH_CHECK(res_stride >= 1, "res_stride must be >= 1");
  const float* rp = nullptr;
  if (res.has_value() && res->defined()) {
    need(*res, "res", 4);
    const int64_t Hr = (H + res_stride - 1) / res_stride, Wr = (W + res_stride - 1) / res_stride;
    TORCH_CHECK(res->size(0) == B && res->size(1) == Hr && res->size(2) == Wr && res->size(3) == N,
                "res must be (B, ceil(H/s), ceil(W/s), N)");
    rp = res->data_ptr<float>();
  }
  const uint8_t* rb = bit_mask_ptr(res_bits, M * N, g, "res_bits");
  TORCH_CHECK(!rb || (rp && res_stride == 1), "res_bits needs a stride-1 res");
  const float* yp = nullptr;
  at::Tensor part;
  if (bn_y.has_value() && bn_y->defined()) {
    need(*bn_y, "bn_y", 4);
    TORCH_CHECK(bn_y->size(0) == B && bn_y->size(1) == H && bn_y->size(2) == W && bn_y->size(3) == N,
                "bn_y must be (B, H, W, N)");
    yp = bn_y->data_ptr<float>();
    part = at::empty({(M + tp_conv_tile_m((int)cfg) - 1) / tp_conv_tile_m((int)cfg), 2, N},
                     g.options().dtype(at::kDouble));
  }
  const float* mp = yp ? opt_ptr(bn_mean, N, "bn_mean") : nullptr;
  const float* ip = yp ? opt_ptr(bn_invstd, N, "bn_invstd") : nullptr;
  TORCH_CHECK(!yp || (mp && ip), "bn_y needs bn_mean and bn_invstd");
  const uint8_t* bb = yp ? bit_mask_ptr(bn_bits, M * N, g, "bn_bits") : nullptr;
  auto out = at::empty({B, H, W, N}, g.options());
  at::Tensor ws = sk_workspace(cfg, 1, false, false, M, N, g.options());
  const int64_t cf = ws.defined() || cfg < 0 ? cfg : cfg & ~kCfgSK;
  TP_CHECK_HIP(tp_conv_gen5(g.data_ptr<float>(), wt.data_ptr<float>(), (int)B, (int)H, (int)W, (int)C, (int)N, 1, 1,
                            0, 0, 0, 0, (int)cf, 1, nullptr, nullptr, 0, rp, (int)res_stride, nullptr, nullptr,
                            out.data_ptr<float>(), ws.defined() ? ws.data_ptr<float>() : nullptr,
                            yp ? part.data_ptr<double>() : nullptr, nullptr, 0, rb, yp, mp, ip, bb, cur_stream()));
  return {out, part};
}

// Fixup-workspace floats of a stream-K GEN launch of tile config cfg at an M x N GEMM (0 = stream-K
// does not apply; the launcher then runs the data-parallel grid).
int64_t conv_sk_ws(int64_t cfg, int64_t ks, bool tay, int64_t M, int64_t N) {
  return tp_conv_sk_ws_floats((int)(cfg & ~kCfgSK), (int)ks, 0, tay ? 1 : 0, (int)M, (int)N);
}

// Weight gradient: g (B, Ho, Wo, Cout) and x (B, H, W, Cin) NHWC -> dW (Cout, Kpad) with column
// k = (kh, kw, ci) (Kpad = ks*ks*Cin rounded up to 32; padded columns are zero).
// ``out`` (optional): the parameter-shaped gradient (Cout_r, Cin_r, ks, ks), any strides, written
// directly (real channels only); the (Cout, Kpad) GEMM result is then not materialised and an
// empty tensor is returned.
at::Tensor conv_wgrad(const at::Tensor& g, const at::Tensor& x, int64_t ks, int64_t stride, int64_t pad, int64_t cfg,
                      int64_t splits, const c10::optional<at::Tensor>& out) {
  need(g, "g", 4);
  need(x, "x", 4);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = g.size(3);
  TORCH_CHECK(Cin % 4 == 0 && Cout % 4 == 0, "conv_wgrad needs Cin % 4 == 0 and Cout % 4 == 0");
  TORCH_CHECK(ks >= 1 && stride >= 1 && pad >= 0, "bad conv geometry");
  const int64_t Ho = (H + 2 * pad - ks) / stride + 1, Wo = (W + 2 * pad - ks) / stride + 1;
  TORCH_CHECK(g.size(0) == B && g.size(1) == Ho && g.size(2) == Wo, "g must be (B, Ho, Wo, Cout) of this conv");
  const int64_t Kpad = (ks * ks * Cin + 31) / 32 * 32;
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  float* fin = nullptr;
  long long fs[4] = {0, 0, 0, 0};
  int fco = 0, fci = 0;
  if (out.has_value()) {
    const at::Tensor& o = *out;
    TORCH_CHECK(o.is_cuda() && o.scalar_type() == at::kFloat && o.dim() == 4 && o.device() == g.device(),
                "out must be a float32 (Cout, Cin, ks, ks) tensor on the device");
    TORCH_CHECK(o.size(0) <= Cout && o.size(1) <= Cin && o.size(2) == ks && o.size(3) == ks && o.size(0) > 0 &&
                    o.size(1) > 0, "out must be (Cout_r <= Cout, Cin_r <= Cin, ks, ks)");
    fin = o.data_ptr<float>();
    fco = (int)o.size(0);
    fci = (int)o.size(1);
    for (int i = 0; i < 4; ++i) fs[i] = o.stride(i);
  }
  at::Tensor dw = fin ? at::Tensor() : at::empty({Cout, Kpad}, g.options());
  const int64_t slices = (B * Ho * Wo + 31) / 32;
  int64_t sp = std::max<int64_t>(1, std::min<int64_t>(splits, slices));
  const int64_t per = (slices + sp - 1) / sp;
  sp = (slices + per - 1) / per;
  at::Tensor ws;
  if (sp > 1) ws = at::empty({sp * Cout * Kpad}, g.options());
  TP_CHECK_HIP(tp_conv_wgrad2(g.data_ptr<float>(), x.data_ptr<float>(), fin ? nullptr : dw.data_ptr<float>(),
                              sp > 1 ? ws.data_ptr<float>() : nullptr, (int)B, (int)H, (int)W, (int)Cin, (int)Cout,
                              (int)ks, (int)stride, (int)pad, (int)Kpad, (int)cfg, (int)sp, fin, fco, fci,
                              fin ? fs : nullptr, cur_stream()));
  return fin ? at::empty({0}, g.options()) : dw;  // with ``out`` the result is in ``out``
}

// Training conv forward that also returns the BatchNorm statistics of its output: y (B, Ho, Wo,
// Cout) and per M tile the column sums / sums of squares, (ceil(M / tile_m(cfg)), 2, Cout) fp64
// (fold with bn_train_fwd(..., pre=)). No split-K, no epilogue besides the bias.
std::tuple<at::Tensor, at::Tensor> conv_gen_stats(const at::Tensor& x, const at::Tensor& w,
                                                  const c10::optional<at::Tensor>& shift, int64_t ks, int64_t stride,
                                                  int64_t pad, int64_t cfg) {
  need(x, "x", 4);
  need(w, "w", 2);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = w.size(0);
  TORCH_CHECK((Cin % 4 == 0 && Cin >= 8 && (ks == 1 || ks == 3 || ks == 5)) ||
                  (Cin == 4 && (ks == 3 || ks == 5 || ks == 7)),
              "conv_gen_stats supports ks 1/3/5 with Cin % 4 == 0 (>= 8), or ks 3/5/7 with a 4-channel input");
  TORCH_CHECK(w.size(1) == tp_conv_gen_k((int)ks, (int)Cin), "weight K mismatch");
  TORCH_CHECK(stride >= 1 && pad >= 0 && Cout % 4 == 0, "bad geometry / Cout % 4");
  const int64_t Ho = (H + 2 * pad - ks) / stride + 1, Wo = (W + 2 * pad - ks) / stride + 1;
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* sh = opt_ptr(shift, Cout, "shift");
  auto out = at::empty({B, Ho, Wo, Cout}, x.options());
  const int64_t M = B * Ho * Wo, tm = tp_conv_tile_m((int)cfg);
  auto part = at::empty({(M + tm - 1) / tm, 2, Cout}, x.options().dtype(at::kDouble));
  at::Tensor ws = Cin != 4 ? sk_workspace(cfg, ks, false, false, M, Cout, x.options()) : at::Tensor();
  const int64_t cf = ws.defined() || cfg < 0 ? cfg : cfg & ~kCfgSK;
  TP_CHECK_HIP(tp_conv_gen3(x.data_ptr<float>(), w.data_ptr<float>(), (int)B, (int)H, (int)W, (int)Cin, (int)Cout,
                            (int)ks, (int)stride, (int)pad, 0, 0, 0, (int)cf, 1, nullptr, sh, 0, nullptr, 1, nullptr,
                            nullptr, out.data_ptr<float>(), ws.defined() ? ws.data_ptr<float>() : nullptr,
                            part.data_ptr<double>(), cur_stream()));
  return {out, part};
}

// Winograd F(2x2,3x3) weight gradient of a stride-1 pad-1 3x3 conv: g (B, H, W, Cout), x (B, H, W,
// Cin) NHWC (H, W even, Cin % 32 == 0) -> ``out`` (Cout_r, Cin_r, 3, 3), any strides (real channels).
void wino_wgrad(const at::Tensor& g, const at::Tensor& x, int64_t cfg, int64_t splits, at::Tensor& out) {
  need(g, "g", 4);
  need(x, "x", 4);
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), Cin = x.size(3), Cout = g.size(3);
  TORCH_CHECK(g.size(0) == B && g.size(1) == H && g.size(2) == W, "g must be (B, H, W, Cout) of a same-size conv");
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0 && Cin % 4 == 0 && Cin >= 8 && Cout % 4 == 0,
              "wino_wgrad needs even H/W, Cin % 4 (>= 8), Cout % 4");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.dim() == 4 && out.size(2) == 3 &&
                  out.size(3) == 3 && out.size(0) <= Cout && out.size(1) <= Cin && out.device() == g.device(),
              "out must be a float32 (Cout_r, Cin_r, 3, 3) tensor on the device");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  const int64_t T = B * (H / 2) * (W / 2);
  const int64_t slices = (T + 31) / 32;
  int64_t sp = std::max<int64_t>(1, std::min<int64_t>(splits, slices));
  const int64_t per = (slices + sp - 1) / sp;
  sp = (slices + per - 1) / per;
  auto ws = at::empty({tp_wino_wgrad_ws_elems((int)B, (int)H, (int)W, (int)Cin, (int)Cout, (int)sp)}, g.options());
  long long fs[4];
  for (int i = 0; i < 4; ++i) fs[i] = out.stride(i);
  TP_CHECK_HIP(tp_wino_wgrad(g.data_ptr<float>(), x.data_ptr<float>(), ws.data_ptr<float>(), (int)B, (int)H, (int)W,
                             (int)Cin, (int)Cout, (int)cfg, (int)sp, out.data_ptr<float>(), (int)out.size(0),
                             (int)out.size(1), fs, cur_stream()));
}

// Training-mode BatchNorm over the last dim of an NHWC activation x (..., C), C % 4 == 0.
// Updates running_mean / running_var in place (momentum, unbiased variance) when given.
// Training BN on (.., C) channels-last data; optional fused residual add and ReLU:
// y = relu?(BN(x) + res?). Returns (y, mean, invstd).
// With ``relu`` also returns the ReLU bit mask (ceil(P*C/4) bytes; else an empty tensor) for bn_train_bwd.
// Any C (C % 4 == 0: float4 rows; else per-element). ``cr`` (0 = C): the channels with parameters /
// running statistics; x's channels c >= cr are the zero padding of a pruned width (outputs 0).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_train_fwd(const at::Tensor& x, const c10::optional<at::Tensor>& gamma,
                                                             const c10::optional<at::Tensor>& beta,
                                                             const c10::optional<at::Tensor>& running_mean,
                                                             const c10::optional<at::Tensor>& running_var, double eps,
                                                             double momentum, const c10::optional<at::Tensor>& res,
                                                             bool relu, const c10::optional<at::Tensor>& pre,
                                                             const c10::optional<at::Tensor>& num_batches,
                                                             int64_t cr) {
  need(x, "x", -1);
  const int64_t C = x.size(-1), P = x.numel() / std::max<int64_t>(C, 1);
  TORCH_CHECK(C > 0 && P > 0, "bn_train_fwd needs a non-empty batch");
  const int64_t Cr = cr > 0 ? cr : C;
  TORCH_CHECK(Cr <= C, "cr must be <= the channel count");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* ga = opt_ptr(gamma, Cr, "gamma");
  const float* be = opt_ptr(beta, Cr, "beta");
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    need(*running_mean, "running_mean", 1);
    need(*running_var, "running_var", 1);
    TORCH_CHECK(running_mean->numel() == Cr && running_var->numel() == Cr, "running stats must have cr elements");
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  const float* rp = nullptr;
  if (res.has_value() && res->defined()) {
    need(*res, "res", -1);
    TORCH_CHECK(res->sizes() == x.sizes(), "res must have x's shape");
    rp = res->data_ptr<float>();
  }
  long long* nbt = nullptr;  // the module's num_batches_tracked, incremented by the finalize kernel
  if (num_batches.has_value() && num_batches->defined()) {
    TORCH_CHECK(num_batches->is_cuda() && num_batches->scalar_type() == at::kLong && num_batches->numel() == 1 &&
                    num_batches->device() == x.device(), "num_batches must be a one-element int64 GPU tensor");
    nbt = reinterpret_cast<long long*>(num_batches->data_ptr<int64_t>());
  }
  auto y = at::empty_like(x);
  auto mk = at::empty({relu ? (P * C + 3) / 4 : 0}, x.options().dtype(at::kByte));
  const int64_t Cs = (C + 3) / 4 * 4;  // row stride: every row 16-byte aligned (float4 reads) for any C
  auto stats = at::empty({4, Cs}, x.options()).narrow(1, 0, C);  // mean, invstd, a, b
  float* sp = stats.data_ptr<float>();
  if (pre.has_value() && pre->defined()) {  // statistics reduced per tile by the producing conv
    TORCH_CHECK(pre->is_cuda() && pre->scalar_type() == at::kDouble && pre->is_contiguous() && pre->dim() == 3 &&
                    pre->size(1) == 2 && pre->size(2) == C && pre->device() == x.device(),
                "pre must be conv_gen_stats' (G, 2, C) fp64 tile statistics");
    const int64_t G = pre->size(0);
    auto ws = at::empty({2 * std::min<int64_t>(G, 256) * C}, x.options().dtype(at::kDouble));
    TP_CHECK_HIP(tp_bn_fwd_train_pre2(x.data_ptr<float>(), y.data_ptr<float>(), (int)P, (int)C, (int)Cr, ga, be, (float)eps,
                                     (float)momentum, rm, rv, sp, sp + Cs, sp + 2 * Cs, sp + 3 * Cs, ws.data_ptr<double>(),
                                     pre->data_ptr<double>(), (int)G, rp, relu ? 1 : 0,
                                     relu ? mk.data_ptr<uint8_t>() : nullptr, nbt, cur_stream()));
    return {y, stats[0], stats[1], mk};
  }
  auto ws = at::empty({2 * (int64_t)tp_bn_groups((int)P, (int)C) * C}, x.options().dtype(at::kDouble));
  TP_CHECK_HIP(tp_bn_fwd_train5(x.data_ptr<float>(), y.data_ptr<float>(), (int)P, (int)C, (int)Cr, ga, be, (float)eps,
                                (float)momentum, rm, rv, sp, sp + Cs, sp + 2 * Cs, sp + 3 * Cs, ws.data_ptr<double>(), rp,
                                relu ? 1 : 0, relu ? mk.data_ptr<uint8_t>() : nullptr, nbt, cur_stream()));
  return {y, stats[0], stats[1], mk};
}

// Backward of bn_train_fwd: (dx or undefined, dgamma, dbeta, dres or undefined). ``ym``: the
// forward output y when it was ReLU'd (the gradient is masked by y > 0 first); ``want_dres``:
// also return that masked gradient (the residual branch's gradient).
std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> bn_train_bwd(
    const at::Tensor& g, const at::Tensor& x, const c10::optional<at::Tensor>& gamma, const at::Tensor& mean,
    const at::Tensor& invstd, bool want_dx, const c10::optional<at::Tensor>& ym, bool want_dres,
    const c10::optional<at::Tensor>& mask, int64_t cr, const c10::optional<at::Tensor>& pre) {
  need(g, "g", -1);
  need(x, "x", -1);
  TORCH_CHECK(g.sizes() == x.sizes(), "g and x must have the same shape");
  const int64_t C = x.size(-1), P = x.numel() / std::max<int64_t>(C, 1);
  TORCH_CHECK(C > 0 && P > 0, "bn_train_bwd needs a non-empty batch");
  const int64_t Cr = cr > 0 ? cr : C;
  TORCH_CHECK(Cr <= C, "cr must be <= the channel count");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  const float* ga = opt_ptr(gamma, Cr, "gamma");
  const float* mp = opt_ptr(mean, C, "mean");
  const float* ip = opt_ptr(invstd, C, "invstd");
  const float* yp = nullptr;
  if (ym.has_value() && ym->defined()) {
    need(*ym, "ym", -1);
    TORCH_CHECK(ym->sizes() == x.sizes(), "ym must have x's shape");
    yp = ym->data_ptr<float>();
  }
  const uint8_t* mkp = nullptr;
  if (mask.has_value() && mask->defined() && mask->numel() > 0) {
    TORCH_CHECK(mask->is_cuda() && mask->scalar_type() == at::kByte && mask->is_contiguous() &&
                    mask->numel() == (P * C + 3) / 4 && mask->device() == x.device(),
                "mask must be bn_train_fwd's ReLU bit mask (ceil(P*C/4) uint8)");
    mkp = mask->data_ptr<uint8_t>();
  }
  const int64_t Cs = (C + 3) / 4 * 4;
  auto coef = at::empty({5, Cs}, x.options());  // dgamma, dbeta, a, k1, k2 (16-byte aligned rows)
  at::Tensor dx, dres;
  if (want_dx) dx = at::empty_like(x);
  if (want_dres) dres = at::empty_like(x);
  float* cp = coef.data_ptr<float>();
  if (pre.has_value() && pre->defined()) {  // statistics from the producing GEMM's epilogue (conv_gen_bwd_bn)
    TORCH_CHECK(pre->is_cuda() && pre->scalar_type() == at::kDouble && pre->is_contiguous() && pre->dim() == 3 &&
                    pre->size(1) == 2 && pre->size(2) == C && pre->size(0) > 0 && pre->device() == x.device(),
                "pre must be (G, 2, C) float64 tile statistics");
    const int64_t G = pre->size(0);
    auto wsp = at::empty({2 * std::min<int64_t>(G, 256) * C}, x.options().dtype(at::kDouble));
    TP_CHECK_HIP(tp_bn_bwd_train_pre(g.data_ptr<float>(), x.data_ptr<float>(),
                                     want_dx ? dx.data_ptr<float>() : nullptr, (int)P, (int)C, (int)Cr, ga, mp, ip, cp,
                                     cp + Cs, cp + 2 * Cs, cp + 3 * Cs, cp + 4 * Cs, wsp.data_ptr<double>(),
                                     pre->data_ptr<double>(), (int)G, mkp ? nullptr : yp,
                                     want_dres ? dres.data_ptr<float>() : nullptr, mkp, cur_stream()));
    return {dx, coef[0].narrow(0, 0, Cr), coef[1].narrow(0, 0, Cr), dres};
  }
  auto ws = at::empty({2 * (int64_t)tp_bn_groups((int)P, (int)C) * C}, x.options().dtype(at::kDouble));
  TP_CHECK_HIP(tp_bn_bwd_train4(g.data_ptr<float>(), x.data_ptr<float>(), want_dx ? dx.data_ptr<float>() : nullptr,
                                (int)P, (int)C, (int)Cr, ga, mp, ip, cp, cp + Cs, cp + 2 * Cs, cp + 3 * Cs, cp + 4 * Cs,
                                ws.data_ptr<double>(), mkp ? nullptr : yp, want_dres ? dres.data_ptr<float>() : nullptr,
                                mkp, cur_stream()));
  return {dx, coef[0].narrow(0, 0, Cr), coef[1].narrow(0, 0, Cr), dres};
}

void register_engine_ops_def(torch::Library& m) {
  m.def("wino_taylor_slots(int H, int W) -> int", &wino_taylor_slots);
  m.def("wino_lds_bytes() -> int", []() -> int64_t { return tp_wino_lds_bytes(); });
  m.def("wino_staged_ok(int H, int W, bool unpool) -> bool",
        [](int64_t H, int64_t W, bool unpool) -> bool { return tp_wino_staged_ok((int)H, (int)W, unpool ? 1 : 0) != 0; });
  m.def("wino4_taylor_slots(int S) -> int", [](int64_t S) -> int64_t { return tp_wino4_taylor_slots((int)S); });
  m.def("wino4_u_img() -> int", []() -> int64_t { return tp_wino4_u_img(); });
  m.def("wino4_lds_bytes(int S, int variant=0) -> int",
        [](int64_t S, int64_t variant) -> int64_t { return tp_wino4_lds_bytes((int)S, (int)variant); });
  m.def("nchw_to_nhwc_pad(Tensor x, int Cp) -> Tensor");
  m.def("maxpool2_nhwc(Tensor x) -> (Tensor, Tensor)");
  m.def("maxpool_nhwc(Tensor x, int k, int s, int pad) -> Tensor");
  m.def("avgpool_nhwc(Tensor x) -> Tensor");
  m.def("conv_gen(Tensor x, Tensor w, Tensor? scale, Tensor? shift, bool relu, Tensor? res, Tensor(a!)? apoz, "
        "int ks, int stride, int pad, int cfg, int splits) -> Tensor");
  m.def("conv_gen_k(int ks, int Cin) -> int", &conv_gen_k);
  m.def("bn_train_fwd(Tensor x, Tensor? gamma, Tensor? beta, Tensor(a!)? running_mean, Tensor(b!)? running_var, "
        "float eps, float momentum, Tensor? res=None, bool relu=False, Tensor? pre=None, "
        "Tensor(c!)? num_batches=None, int cr=0) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("bn_train_bwd(Tensor g, Tensor x, Tensor? gamma, Tensor mean, Tensor invstd, bool want_dx, Tensor? ym=None, "
        "bool want_dres=False, Tensor? mask=None, int cr=0, Tensor? pre=None) -> (Tensor, Tensor, Tensor, Tensor)");
  m.def("conv_wgrad(Tensor g, Tensor x, int ks, int stride, int pad, int cfg, int splits, Tensor(a!)? out=None) "
        "-> Tensor");
  m.def("pack_conv_weight(Tensor w, int rows, int cols, int cpad, int mode) -> Tensor");
  m.def("pack_conv_weights_multi(Tensor[] ws, Tensor(a!)[] outs, int[] cfg) -> ()");
  m.def("wino4_weights_multi(Tensor[] ws, Tensor(a!)[] us, int[] cfg) -> ()");
  m.def("conv_gen_stats(Tensor x, Tensor w, Tensor? shift, int ks, int stride, int pad, int cfg) -> (Tensor, Tensor)");
  m.def("wino_wgrad(Tensor g, Tensor x, int cfg, int splits, Tensor(a!) out) -> ()");
  m.def("conv_gen_bwd(Tensor g, Tensor wt, Tensor? res, int res_stride, Tensor? mask, int ks, int stride, int pad, "
        "int Ho, int Wo, bool transposed, int cfg, int splits, Tensor(a!)? taylor=None, int tay_mode=0) -> Tensor");
  m.def("conv_gen_tay_slots(int cfg, int HWo) -> int", &conv_gen_tay_slots);
  m.def("conv_gen_bwd_bn(Tensor g, Tensor wt, Tensor? res, int res_stride, Tensor? res_bits, Tensor? bn_y, Tensor? bn_mean, "
        "Tensor? bn_invstd, Tensor? bn_bits, int cfg) -> (Tensor, Tensor)");
  m.def("conv_sk_ws(int cfg, int ks, bool tay, int M, int N) -> int", &conv_sk_ws);
  m.def("unpool2_nhwc(Tensor g, Tensor am) -> Tensor");
  m.def("conv_fwd(Tensor x, Tensor w, Tensor? scale, Tensor? shift, bool relu, bool pool, int ks, int cfg, "
        "int splits, Tensor(a!)? apoz=None, float slope=0.0) -> (Tensor, Tensor)");
  m.def("conv_dgrad(Tensor g, Tensor? g_argmax, Tensor wt, Tensor act, Tensor? bn_scale, Tensor(a!)? taylor, "
        "bool want_out, int ks, int cfg, int splits, int tay_group=0, int tay_mode=0, float slope=0.0) -> Tensor");
  m.def("conv_first(Tensor x, Tensor w, Tensor scale, Tensor shift, bool relu, Tensor? wt=None) -> Tensor");
  m.def("wino_weights(Tensor w, bool flip_t, int K=0, int C=0, bool bf16=False) -> Tensor");
  m.def("prefix_tri_operands(Tensor z, Tensor w, Tensor perm, int p0, int cnt, int Kc) -> (Tensor, Tensor)");
  m.def("prefix_delta(Tensor T, Tensor wsub, Tensor neg_one, Tensor y0, bool relu, float slope, int cfg) -> Tensor");
  m.def("conv_wino_fwd(Tensor x, Tensor u, Tensor? scale, Tensor? shift, bool relu, bool pool, int splits, "
        "bool staged=True, Tensor(a!)? apoz=None) -> (Tensor, Tensor)");
  m.def("conv_wino_dgrad(Tensor g, Tensor? g_argmax, Tensor ut, Tensor act, Tensor? bn_scale, "
        "Tensor(a!)? taylor, bool want_out, int splits, bool staged=True, int tay_mode=0) -> Tensor");
  m.def("wino4_weights(Tensor w, bool flip_t, int K=0, int C=0) -> Tensor");
  m.def("conv_wino4_fwd(Tensor x, Tensor u, Tensor? scale, Tensor? shift, bool relu, bool pool, "
        "Tensor(a!)? apoz=None, int splits=1, int variant=0, int ko=0) -> (Tensor, Tensor)");
  m.def("conv_wino4_dgrad(Tensor g, Tensor ut, Tensor act, Tensor? bn_scale, Tensor(a!)? taylor, bool want_out, "
        "int tay_mode=0, int splits=1, int variant=0, Tensor? unpool_am=None) -> Tensor");
}

void register_engine_ops_impl(torch::Library& m) {
  m.impl("conv_fwd", &conv_fwd);
  m.impl("conv_dgrad", &conv_dgrad);
  m.impl("conv_first", &conv_first);
  m.impl("prefix_tri_operands", &prefix_tri_operands);
  m.impl("wino_weights", &wino_weights);
  m.impl("prefix_delta", &prefix_delta);
  m.impl("conv_wino_fwd", &conv_wino_fwd);
  m.impl("nchw_to_nhwc_pad", &nchw_to_nhwc_pad);
  m.impl("maxpool2_nhwc", &maxpool2_nhwc);
  m.impl("maxpool_nhwc", &maxpool_nhwc);
  m.impl("avgpool_nhwc", &avgpool_nhwc);
  m.impl("conv_gen", &conv_gen);
  m.impl("conv_gen_bwd", &conv_gen_bwd);
  m.impl("conv_gen_bwd_bn", &conv_gen_bwd_bn);
  m.impl("conv_wgrad", &conv_wgrad);
  m.impl("pack_conv_weight", &pack_conv_weight);
  m.impl("pack_conv_weights_multi", &pack_conv_weights_multi);
  m.impl("wino4_weights_multi", &wino4_weights_multi);
  m.impl("conv_gen_stats", &conv_gen_stats);
  m.impl("wino_wgrad", &wino_wgrad);
  m.impl("bn_train_fwd", &bn_train_fwd);
  m.impl("bn_train_bwd", &bn_train_bwd);
  m.impl("unpool2_nhwc", &unpool2_nhwc);
  m.impl("conv_wino_dgrad", &conv_wino_dgrad);
  m.impl("wino4_weights", &wino4_weights);
  m.impl("conv_wino4_fwd", &conv_wino4_fwd);
  m.impl("conv_wino4_dgrad", &conv_wino4_dgrad);
}
