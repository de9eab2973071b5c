// Host-side validation of the kernel launchers, built with AddressSanitizer + UBSan on the host
// code (SURVEY.md §5 "race detection / sanitizers"; GPU sanitizers are not available on this
// pool). Every launcher must reject shapes its kernels do not support BEFORE touching the GPU,
// and the host-side geometry helpers (tile/slot/group counts, the Winograd LDS-region search)
// must be memory-clean. Runs on a CPU-only machine: no kernel is launched.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

extern "C" {
int tp_conv_gen_k(int ks, int Cin);
int tp_wino_taylor_slots(int H, int W);
int tp_wino_staged_ok(int H, int W, int unpool);
void tp_wino_geometry(int H, int W, int unpool, int* out9);
int tp_bn_groups(int P, int C);
long long tp_conv_sk_ws_floats(int cfg, int ks, int transposed, int tay, int M, int N);
int tp_wino4_ok(int H, int W, int C, int K);
int tp_wino4_taylor_slots(int S);
hipError_t tp_conv_wino4(const float* x, const float* u, int B, int S, int C, int K, int epi, const float* scale,
                         const float* shift, int relu, float* out, uint8_t* out_argmax, const float* act, float* taylor,
                         float* apoz, int tay_mode, int splits, float* ws, int variant, hipStream_t st,
                         const uint8_t* unpool_am);
hipError_t tp_conv_gen2(const float* x, const float* w, int B, int H, int W, int Cin, int Cout, int ks, int stride,
                        int pad, int transposed, int Ho_t, int Wo_t, int cfg, int splits, const float* scale,
                        const float* shift, int relu, const float* res, int res_stride, const float* mask,
                        float* apoz, float* out, float* ws, hipStream_t st);
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
hipError_t tp_conv_wgrad(const float* g, const float* x, float* dw, float* ws, int B, int H, int W, int Cin, int Cout,
                         int ks, int stride, int pad, int Kpad, int cfg, int splits, hipStream_t st);
hipError_t tp_conv_wino(const float* x, const uint8_t* x_argmax, const float* u, int B, int H, int W, int C, int K,
                        int unpool, int epi, int splits, int staged, const float* scale, const float* shift, int relu,
                        float* out, uint8_t* out_argmax, const float* act, float* taylor, float* apoz, float* ws,
                        int tay_mode, hipStream_t st);
hipError_t tp_conv_wino4_ko(const float* x, const float* u, int B, int S, int C, int K, int epi, const float* scale,
                            const float* shift, int relu, float* out, uint8_t* out_argmax, const float* act,
                            float* taylor, float* apoz, int tay_mode, int splits, float* ws, int variant,
                            hipStream_t st, const uint8_t* unpool_am, int ko);
hipError_t tp_pack_conv_weights_multi(const long long* desc, int n, long long total, hipStream_t st);
hipError_t tp_wino4_weights_multi(const long long* desc, int n, long long total, hipStream_t st);
hipError_t tp_wino4_weights_strided(const float* w, float* u, int K, int C, int flip_t, int S0, int S1, long long st0,
                                    long long st1, int st2, int st3, hipStream_t st);
hipError_t tp_bn_fwd_train(const float* x, float* y, int P, int C, const float* gamma, const float* beta, float eps,
                           float momentum, float* run_mean, float* run_var, float* mean, float* invstd, float* a,
                           float* b, double* ws, hipStream_t st);
}

static int failures = 0;
#define EXPECT(cond)                                                   \
  do {                                                                 \
    if (!(cond)) {                                                     \
      std::fprintf(stderr, "%s:%d: EXPECT(%s) failed\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

int main() {
  // geometry helpers
  EXPECT(tp_conv_gen_k(3, 64) == 576);
  EXPECT(tp_conv_gen_k(3, 104) == 9 * 128 && tp_conv_gen_k(1, 52) == 64);  // pruned widths: 32-padded taps
  EXPECT(tp_conv_gen_k(7, 4) == 224);
  EXPECT(tp_wino_taylor_slots(2, 2) == 1);
  EXPECT(tp_wino_taylor_slots(32, 32) == 4);
  for (int h = 2; h <= 64; h += 2)
    for (int w = 2; w <= 64; w += 2)
      for (int up = 0; up < 2; ++up) {
        int g[9];
        tp_wino_geometry(h, w, up, g);
        EXPECT(g[0] == tp_wino_staged_ok(h, w, up));
        if (g[0]) EXPECT(g[1] >= 1 && g[3] > 0 && g[4] > 0);
      }
  for (int p = 1; p < 5000; p = p * 3 + 1)
    for (int c = 4; c <= 2048; c *= 2) EXPECT(tp_bn_groups(p, c) >= 1);

  // launchers reject unsupported shapes before any GPU work (null pointers are never touched)
  float* n = nullptr;
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 50, 64, 3, 1, 1, 0, 0, 0, 0, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // Cin % 4 (pruned widths: any multiple of 4 from 8 up)
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 62, 3, 1, 1, 0, 0, 0, 0, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // Cout % 4
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 5, 2, 2, 1, 16, 16, 0, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // transposed 5x5
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 3, 1, 1, 0, 0, 0, 64 | 2, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // single-buffered LDS stage: 1x1 only
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 64 | 2, 2, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // single-buffered LDS stage: one K pass
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 64 | 32 | 2, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // single-buffered LDS stage: not with stream-K
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 3, 1, 1, 0, 0, 0, 0, 1, n, n, 0, n, 0, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // res_stride 0
  EXPECT(tp_conv_gen2(n, n, 4096, 256, 256, 64, 64, 3, 1, 1, 0, 0, 0, 0, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // exceeds the 32-bit buffer-descriptor range
  // Taylor partials of the GEN data gradients: 1x1 stride 1, or transposed 3x3 stride 2 at even Ho / Wo
  float* tp_ = reinterpret_cast<float*>(16);
  const float* mk = reinterpret_cast<const float*>(16);
  EXPECT(tp_conv_gen_tay_slots(2, 3136) == 50 && tp_conv_gen_tay_slots(0, 49) == 2);
  EXPECT(tp_conv_gen_tay_slots(1, 49) == 0 && tp_conv_gen_tay_slots(4, 3136) == 0);  // > 4 images / spilling cfg
  EXPECT(tp_conv_gen4(n, n, 2, 8, 8, 64, 64, 3, 1, 1, 0, 0, 0, 2, 1, n, n, 0, n, 1, mk, n, n, n, nullptr, tp_, 0, 0) ==
         hipErrorInvalidValue);  // GEN 1 3x3: no partials
  EXPECT(tp_conv_gen4(n, n, 2, 4, 4, 64, 64, 1, 2, 0, 1, 8, 8, 2, 1, n, n, 0, n, 1, mk, n, n, n, nullptr, tp_, 0, 0) ==
         hipErrorInvalidValue);  // transposed 1x1: no partials
  EXPECT(tp_conv_gen4(n, n, 2, 4, 4, 64, 64, 3, 2, 1, 1, 7, 7, 2, 1, n, n, 0, n, 1, mk, n, n, n, nullptr, tp_, 0, 0) ==
         hipErrorInvalidValue);  // odd output: no parity row order
  EXPECT(tp_conv_gen4(n, n, 2, 4, 4, 64, 64, 3, 2, 1, 1, 8, 8, 4, 1, n, n, 0, n, 1, mk, n, n, n, nullptr, tp_, 0, 0) ==
         hipErrorInvalidValue);  // cfg 4: no partials
  EXPECT(tp_conv_gen4(n, n, 2, 4, 4, 64, 64, 3, 2, 1, 1, 8, 8, 2, 1, n, n, 0, n, 1, nullptr, n, n, n, nullptr, tp_, 0,
                      0) == hipErrorInvalidValue);  // no mask
  // bottleneck backward fusions (tp_conv_gen5): residual bit mask needs a stride-1 res, no mask, GEN 1;
  // BN-backward statistics need bnpart + mean / invstd, no ReLU / mask / partials
  const uint8_t* bits = reinterpret_cast<const uint8_t*>(16);
  double* bp = reinterpret_cast<double*>(16);
  EXPECT(tp_conv_gen5(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 2, 1, n, n, 0, n, 1, n, n, n, n, nullptr, nullptr, 0,
                      bits, n, n, n, nullptr, 0) == hipErrorInvalidValue);  // res_bits without res
  EXPECT(tp_conv_gen5(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 2, 1, n, n, 0, mk, 2, n, n, n, n, nullptr, nullptr, 0,
                      bits, n, n, n, nullptr, 0) == hipErrorInvalidValue);  // res_bits with a strided res
  EXPECT(tp_conv_gen5(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 2, 1, n, n, 0, n, 1, n, n, n, n, nullptr, nullptr, 0,
                      nullptr, mk, mk, mk, nullptr, 0) == hipErrorInvalidValue);  // bnb without bnpart
  EXPECT(tp_conv_gen5(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 2, 1, n, n, 0, n, 1, n, n, n, n, bp, nullptr, 0,
                      nullptr, mk, nullptr, mk, nullptr, 0) == hipErrorInvalidValue);  // bnb without mean
  EXPECT(tp_conv_gen5(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 2, 1, n, n, 1, n, 1, n, n, n, n, bp, nullptr, 0,
                      nullptr, mk, mk, mk, nullptr, 0) == hipErrorInvalidValue);  // bnb with a ReLU epilogue
  EXPECT(tp_conv_gen5(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 2, 1, n, n, 0, n, 1, n, n, n, n, bp, nullptr, 0,
                      nullptr, nullptr, nullptr, nullptr, bits, 0) == hipErrorInvalidValue);  // bnb_bits alone
  EXPECT(tp_bn_bwd_train_pre(n, n, n, 64, 8, 8, n, n, n, n, n, n, n, n, nullptr, nullptr, 0, n, n, nullptr, 0) ==
         hipErrorInvalidValue);  // no tiles
  EXPECT(tp_conv_wgrad(n, n, n, n, 2, 8, 8, 6, 64, 3, 1, 1, 64, 0, 1, 0) == hipErrorInvalidValue);   // Cin % 4
  EXPECT(tp_conv_wgrad(n, n, n, n, 2, 8, 8, 64, 64, 3, 1, 1, 96, 0, 1, 0) == hipErrorInvalidValue);  // Kpad small
  EXPECT(tp_conv_wgrad(n, n, n, n, 2, 8, 8, 64, 64, 3, 1, 1, 576, 7, 1, 0) == hipErrorInvalidValue); // bad cfg
  EXPECT(tp_conv_wino(n, nullptr, n, 2, 7, 8, 64, 64, 0, 1, 1, 1, n, n, 0, n, nullptr, n, n, n, n, 0, 0) ==
         hipErrorInvalidValue);  // odd H with 2x2 pooling
  EXPECT(tp_conv_wino(n, nullptr, n, 2, 7, 8, 64, 64, 1, 2, 1, 1, n, n, 0, n, nullptr, n, n, n, n, 0, 0) ==
         hipErrorInvalidValue);  // odd H with unpooling
  EXPECT(tp_conv_wino(n, nullptr, n, 2, 8, 8, 12, 64, 0, 0, 1, 1, n, n, 0, n, nullptr, n, n, n, n, 0, 0) ==
         hipErrorInvalidValue);  // C % 8
  EXPECT(tp_conv_wino(n, nullptr, n, 2, 8, 8, 64, 64, 0, 0, 1, 2, n, n, 0, n, nullptr, n, n, n, n, 0, 0) ==
         hipErrorInvalidValue);  // bf16 U images (staged bit 1) without a staged input mode
  EXPECT(tp_conv_wino(n, nullptr, n, 2, 7, 7, 64, 64, 0, 0, 1, 3, n, n, 0, n, nullptr, n, n, n, n, 0, 0) ==
         hipErrorInvalidValue);  // bf16 on an odd map (direct loads only)
  EXPECT(tp_bn_fwd_train(n, n, 0, 6, n, n, 1e-5f, 0.1f, n, n, n, n, n, n, nullptr, 0) == hipErrorInvalidValue);  // P = 0
  EXPECT(tp_bn_fwd_train(n, n, 1 << 20, 1 << 12, n, n, 1e-5f, 0.1f, n, n, n, n, n, n, nullptr, 0) ==
         hipErrorInvalidValue);  // P * C >= 2^32 elements
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 3, 1, 1, 0, 0, 0, 16, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // unknown tile config
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 17, 1, n, n, 0, n, 2, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // unknown tile config
  // stream-K (cfg | 32): GEN 1 only, one K pass, a fixup workspace, ks 1 / 3; no workspace is
  // asked for where it cannot apply (transposed, 5x5, warp-specialised cfgs)
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 3, 2, 1, 1, 16, 16, 32, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // transposed
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 32, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // no workspace
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 1, 1, 0, 0, 0, 0, 32 + 2, 2, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // split-K and stream-K together
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 64, 64, 5, 1, 2, 0, 0, 0, 32, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // 5x5
  EXPECT(tp_conv_gen2(n, n, 2, 8, 8, 4, 64, 7, 2, 3, 0, 0, 0, 32, 1, n, n, 0, n, 1, n, n, n, n, 0) ==
         hipErrorInvalidValue);  // 4-channel stem (GEN 2)
  EXPECT(tp_conv_sk_ws_floats(0, 1, 1, 0, 1 << 20, 512) == 0);  // transposed
  EXPECT(tp_conv_sk_ws_floats(0, 5, 0, 0, 1 << 20, 512) == 0);  // 5x5
  EXPECT(tp_conv_sk_ws_floats(16, 1, 0, 0, 1 << 20, 512) == 0); // unknown cfg
  EXPECT(tp_conv_sk_ws_floats(0, 3, 0, 1, 1 << 20, 512) == 0);  // Taylor partials are 1x1 only
  // F(4x4): VGG sizes and the band geometry's ResNet sizes; bands never pool / unpool and only the
  // split-points kernel (variant 3) has them; Taylor slots per image = the most bands overlapping it
  EXPECT(tp_wino4_ok(32, 32, 64, 64) && tp_wino4_ok(56, 56, 64, 64) && tp_wino4_ok(7, 7, 512, 512));
  EXPECT(!tp_wino4_ok(12, 12, 64, 64) && !tp_wino4_ok(56, 28, 64, 64) && !tp_wino4_ok(56, 56, 64, 48));
  EXPECT(tp_wino4_taylor_slots(56) == 8 && tp_wino4_taylor_slots(28) == 3 && tp_wino4_taylor_slots(14) == 2);
  EXPECT(tp_wino4_taylor_slots(7) == 2 && tp_wino4_taylor_slots(32) == 2 && tp_wino4_taylor_slots(8) == 1);
  EXPECT(tp_conv_wino4(n, n, 2, 56, 64, 64, 1, n, n, 1, n, nullptr, n, n, n, 0, 1, n, 3, 0, nullptr) ==
         hipErrorInvalidValue);  // band + 2x2 pool
  EXPECT(tp_conv_wino4(n, n, 2, 28, 64, 64, 0, n, n, 1, n, nullptr, n, n, n, 0, 1, n, 0, 0, nullptr) ==
         hipErrorInvalidValue);  // band on the MODE 3 kernel
  EXPECT(tp_conv_wino4(n, n, 2, 14, 64, 64, 2, n, n, 0, n, nullptr, n, n, n, 0, 1, n, 3, 0,
                       reinterpret_cast<const uint8_t*>(n)) == hipErrorInvalidValue);  // dgrad without act
  // unpadded output widths (ko): a multiple of 4 inside the last 32-channel block, one K pass
  EXPECT(tp_conv_wino4_ko(n, n, 2, 56, 64, 64, 0, n, n, 1, n, nullptr, n, n, n, 0, 1, n, 3, 0, nullptr, 30) ==
         hipErrorInvalidValue);  // ko % 4
  EXPECT(tp_conv_wino4_ko(n, n, 2, 56, 64, 64, 0, n, n, 1, n, nullptr, n, n, n, 0, 1, n, 3, 0, nullptr, 28) ==
         hipErrorInvalidValue);  // ko <= K - 32: a whole empty channel block
  EXPECT(tp_conv_wino4_ko(n, n, 2, 56, 64, 64, 0, n, n, 1, n, nullptr, n, n, n, 0, 1, n, 3, 0, nullptr, 68) ==
         hipErrorInvalidValue);  // ko > K
  EXPECT(tp_conv_wino4_ko(n, n, 2, 56, 64, 64, 0, n, n, 1, n, nullptr, n, n, n, 0, 2, n, 3, 0, nullptr, 60) ==
         hipErrorInvalidValue);  // split-K slabs are K wide
  EXPECT(tp_conv_wino4_ko(n, n, 2, 32, 64, 64, 0, n, n, 1, n, nullptr, n, n, n, 0, 1, n, 1, 0, nullptr, 0) ==
         hipErrorInvalidValue);  // the removed WIDE variant
  EXPECT(tp_pack_conv_weights_multi(nullptr, 0, 16, nullptr) == hipErrorInvalidValue);  // no operands
  EXPECT(tp_pack_conv_weights_multi(nullptr, 2, 0, nullptr) == hipErrorInvalidValue);   // nothing to write
  EXPECT(tp_wino4_weights_multi(nullptr, 1, 100, nullptr) == hipErrorInvalidValue);     // not whole blocks
  EXPECT(tp_wino4_weights_strided(n, n, 64, 64, 0, 64, 64, 0, 9, 3, 1, nullptr) == hipErrorInvalidValue);  // stride 0
  EXPECT(tp_wino4_weights_strided(n, n, 64, 64, 0, 96, 64, 576, 9, 3, 1, nullptr) == hipErrorInvalidValue);  // S0 > K

  if (failures) {
    std::fprintf(stderr, "%d failure(s)\n", failures);
    return 1;
  }
  std::printf("launcher validation ok\n");
  return 0;
}
