// torch.ops.tpamd.* registrations for the gfx950 kernels. This is the only translation
// unit that sees torch headers; kernels live in csrc/kernels/*.hip behind C launchers.
// Every op validates device/dtype/layout and throws (TORCH_CHECK) instead of silently
// falling back: on a GPU box the HIP path is the one that runs, or the call fails.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <hip/hip_runtime.h>

#include "tp_launchers.h"

namespace {

inline hipStream_t cur_stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

#define TP_CHECK_HIP(expr)                                                     \
  do {                                                                         \
    hipError_t _e = (expr);                                                    \
    TORCH_CHECK(_e == hipSuccess, "tpamd kernel launch failed: ", hipGetErrorString(_e)); \
  } while (0)

void check_cuda_f32(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == at::kFloat, name, " must be float32, got ", t.scalar_type());
}

// Returns (B, C, S) and whether the tensor is channels_last. Accepts (B,C), (B,C,*) contiguous,
// or 4D channels_last.
struct BCS {
  int64_t B, C, S;
  bool cl;
};
BCS bcs_of(const at::Tensor& t) {
  TORCH_CHECK(t.dim() >= 2, "expected a (B, C, ...) tensor, got dim ", t.dim());
  BCS r{t.size(0), t.size(1), 1, false};
  for (int64_t d = 2; d < t.dim(); ++d) r.S *= t.size(d);
  if (t.is_contiguous()) return r;
  if (t.dim() == 4 && t.is_contiguous(at::MemoryFormat::ChannelsLast)) {
    r.cl = true;
    return r;
  }
  TORCH_CHECK(false, "tensor must be contiguous (NCHW) or channels_last");
  return r;
}

at::Tensor channel_reduce(const c10::optional<at::Tensor>& act, const c10::optional<at::Tensor>& grad,
                          int64_t mode) {
  const at::Tensor& ref = act.has_value() ? *act : *grad;
  TORCH_CHECK(act.has_value() || grad.has_value(), "channel_reduce needs act or grad");
  check_cuda_f32(ref, "input");
  BCS s = bcs_of(ref);
  if (act.has_value() && grad.has_value()) {
    TORCH_CHECK(act->sizes() == grad->sizes(), "act/grad shape mismatch");
    BCS s2 = bcs_of(*grad);
    TORCH_CHECK(s2.cl == s.cl, "act/grad layout mismatch");
    check_cuda_f32(*grad, "grad");
  }
  const bool need_a = (mode == 0 || mode == 1 || mode == 3);
  const bool need_g = (mode != 3);
  TORCH_CHECK(!need_a || act.has_value(), "mode ", mode, " needs the activation");
  TORCH_CHECK(!need_g || grad.has_value(), "mode ", mode, " needs the gradient");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(ref.device());
  auto out = at::empty({s.B, s.C}, ref.options());
  const int wse = tp_channel_reduce_ws_elems((int)s.B, (int)s.C, (int)s.S, s.cl ? 1 : 0);
  at::Tensor ws;
  if (wse > 0) ws = at::empty({wse}, ref.options());
  TP_CHECK_HIP(tp_channel_reduce(need_a ? act->data_ptr<float>() : nullptr,
                                 need_g ? grad->data_ptr<float>() : nullptr, out.data_ptr<float>(),
                                 wse > 0 ? ws.data_ptr<float>() : nullptr, (int)s.B, (int)s.C, (int)s.S, (int)mode,
                                 s.cl ? 1 : 0, cur_stream()));
  return out;
}

void column_accumulate(const at::Tensor& v, at::Tensor& acc_sum, const c10::optional<at::Tensor>& acc_sq) {
  check_cuda_f32(v, "v");
  TORCH_CHECK(v.dim() == 2 && v.is_contiguous(), "v must be contiguous (B, C)");
  TORCH_CHECK(acc_sum.scalar_type() == at::kDouble && acc_sum.numel() == v.size(1) && acc_sum.is_contiguous(),
              "acc_sum must be a contiguous float64 (C,) tensor");
  double* sq = nullptr;
  if (acc_sq.has_value()) {
    TORCH_CHECK(acc_sq->scalar_type() == at::kDouble && acc_sq->numel() == v.size(1) && acc_sq->is_contiguous(),
                "acc_sq must be a contiguous float64 (C,) tensor");
    sq = acc_sq->data_ptr<double>();
  }
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(v.device());
  TP_CHECK_HIP(tp_column_accumulate(v.data_ptr<float>(), acc_sum.data_ptr<double>(), sq, (int)v.size(0),
                                    (int)v.size(1), cur_stream()));
}

// For every i: T[i] is (B, C) or (R, B, C) partial slots summed in slot order;
// v = |sum| (or sum); acc[i] += v.sum(0) (acc[i] may be empty = skip);
// after: 0 leave T, 1 write v back (slot 0; other slots zeroed), 2 zero T. One launch per 16 tensors.
void score_fold_(at::TensorList T, at::TensorList acc, bool take_abs, int64_t after) {
  TORCH_CHECK(T.size() == acc.size(), "one accumulator per score tensor");
  if (T.empty()) return;
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(T[0].device());
  std::vector<float*> tp;
  std::vector<double*> ap;
  std::vector<int> bs, cs, rs;
  auto flush = [&]() {
    if (tp.empty()) return;
    const int n_ws = tp_score_fold_ws_elems(bs.data(), cs.data(), (int)tp.size());
    at::Tensor ws = at::empty({std::max(n_ws, 1)}, T[0].options().dtype(at::kDouble));
    TP_CHECK_HIP(tp_score_fold_multi(tp.data(), ap.data(), bs.data(), cs.data(), rs.data(), (int)tp.size(),
                                     take_abs ? 1 : 0, (int)after, ws.data_ptr<double>(), cur_stream()));
    tp.clear(); ap.clear(); bs.clear(); cs.clear(); rs.clear();
  };
  for (size_t i = 0; i < T.size(); ++i) {
    check_cuda_f32(T[i], "T");
    TORCH_CHECK((T[i].dim() == 2 || T[i].dim() == 3) && T[i].is_contiguous(),
                "T must be contiguous (B, C) or (R, B, C) partial slots");
    const int64_t nb = T[i].size(-2), nc = T[i].size(-1), nr = T[i].dim() == 3 ? T[i].size(0) : 1;
    double* a = nullptr;
    if (acc[i].defined() && acc[i].numel() > 0) {
      TORCH_CHECK(acc[i].scalar_type() == at::kDouble && acc[i].is_contiguous() && acc[i].numel() == nc,
                  "acc must be a contiguous float64 (C,) tensor");
      a = acc[i].data_ptr<double>();
    }
    tp.push_back(T[i].data_ptr<float>());
    ap.push_back(a);
    bs.push_back((int)nb);
    cs.push_back((int)nc);
    rs.push_back((int)nr);
    if (tp.size() == 16) flush();
  }
  flush();
}

void channel_fill_(at::Tensor& x, const at::Tensor& idx, double value) {
  check_cuda_f32(x, "x");
  TORCH_CHECK(x.is_contiguous(), "channel_fill_ needs a contiguous NC* tensor");
  TORCH_CHECK(idx.scalar_type() == at::kLong && idx.is_cuda() && idx.dim() == 1, "idx must be int64 (n,) on GPU");
  BCS s = bcs_of(x);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto ic = idx.contiguous();
  TP_CHECK_HIP(tp_channel_fill(x.data_ptr<float>(), s.B, (int)s.C, s.S, ic.data_ptr<int64_t>(), (int)ic.numel(),
                               (float)value, cur_stream()));
}

at::Tensor nan_channels(const at::Tensor& x_) {
  check_cuda_f32(x_, "x");
  auto x = x_.contiguous();
  BCS s = bcs_of(x);
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto flags = at::empty({s.C}, x.options().dtype(at::kByte));
  TP_CHECK_HIP(tp_nan_channels(x.data_ptr<float>(), s.B, (int)s.C, s.S, flags.data_ptr<uint8_t>(), cur_stream()));
  return flags;
}

std::vector<at::Tensor> gather_multi(at::TensorList srcs, at::IntArrayRef axes, const at::Tensor& keep_) {
  TORCH_CHECK(srcs.size() == axes.size(), "one axis per tensor");
  TORCH_CHECK(keep_.scalar_type() == at::kLong && keep_.dim() == 1, "keep must be int64 (k,)");
  std::vector<at::Tensor> outs;
  outs.reserve(srcs.size());
  if (srcs.empty()) return outs;
  auto keep = keep_.to(srcs[0].device()).contiguous();
  const int64_t nkeep = keep.numel();
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(srcs[0].device());
  // Group tensors with equal element size into launches of up to 8 descriptors.
  std::vector<at::Tensor> csrc;
  for (size_t i = 0; i < srcs.size(); ++i) {
    TORCH_CHECK(srcs[i].is_cuda(), "gather_multi inputs must be GPU tensors");
    auto c = srcs[i].contiguous();
    int64_t ax = axes[i] < 0 ? axes[i] + c.dim() : axes[i];
    TORCH_CHECK(ax >= 0 && ax < c.dim(), "bad axis");
    auto sz = c.sizes().vec();
    sz[ax] = nkeep;
    outs.push_back(at::empty(sz, c.options()));
    csrc.push_back(c);
  }
  for (int es : {1, 2, 4, 8}) {
    std::vector<const void*> s;
    std::vector<void*> d;
    std::vector<long long> outer, n, inner;
    auto flush = [&]() {
      if (s.empty()) return;
      TP_CHECK_HIP(tp_gather_multi(s.data(), d.data(), outer.data(), n.data(), inner.data(), (int)s.size(), es,
                                   keep.data_ptr<int64_t>(), nkeep, cur_stream()));
      s.clear(); d.clear(); outer.clear(); n.clear(); inner.clear();
    };
    for (size_t i = 0; i < csrc.size(); ++i) {
      if ((int)csrc[i].element_size() != es) continue;
      const auto& c = csrc[i];
      int64_t ax = axes[i] < 0 ? axes[i] + c.dim() : axes[i];
      long long o = 1, in = 1;
      for (int64_t k = 0; k < ax; ++k) o *= c.size(k);
      for (int64_t k = ax + 1; k < c.dim(); ++k) in *= c.size(k);
      s.push_back(c.data_ptr());
      d.push_back(outs[i].data_ptr());
      outer.push_back(o);
      n.push_back(c.size(ax));
      inner.push_back(in);
      if (s.size() == 8) flush();
    }
    flush();
  }
  return outs;
}

at::Tensor prefix_mask(const at::Tensor& z, const at::Tensor& rank, int64_t p0, int64_t K) {
  check_cuda_f32(z, "z");
  TORCH_CHECK(rank.scalar_type() == at::kInt && rank.is_cuda() && rank.dim() == 1 && rank.is_contiguous(),
              "rank must be a contiguous int32 (C,) GPU tensor");
  BCS s = bcs_of(z);
  TORCH_CHECK(rank.numel() == s.C, "rank length must equal channel count");
  auto sz = z.sizes().vec();
  sz[0] = sz[0] * K;
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(z.device());
  auto out = at::empty(sz, z.options().memory_format(s.cl ? at::MemoryFormat::ChannelsLast
                                                            : at::MemoryFormat::Contiguous));
  TP_CHECK_HIP(tp_prefix_mask(z.data_ptr<float>(), out.data_ptr<float>(), rank.data_ptr<int>(), z.numel(), (int)s.C,
                              (int)s.S, s.cl ? 1 : 0, (int)p0, (int)K, cur_stream()));
  return out;
}

void shapley_scatter(const at::Tensor& L, const at::Tensor& perm, at::Tensor& sv, int64_t row0, int64_t k0,
                     double scale) {
  check_cuda_f32(L, "losses");
  TORCH_CHECK(L.dim() == 2 && L.is_contiguous(), "losses must be contiguous (K+1, B)");
  TORCH_CHECK(perm.scalar_type() == at::kInt && perm.is_contiguous(), "perm must be int32");
  TORCH_CHECK(sv.scalar_type() == at::kDouble && sv.dim() == 2 && sv.is_contiguous(), "sv must be float64 (d, n)");
  const int64_t K = L.size(0) - 1, B = L.size(1);
  TORCH_CHECK(row0 + B <= sv.size(0) && k0 + K <= perm.numel() && perm.numel() == sv.size(1), "shape mismatch");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(L.device());
  TP_CHECK_HIP(tp_shapley_scatter(L.data_ptr<float>(), perm.data_ptr<int>(), sv.data_ptr<double>(), (int)row0,
                                  (int)B, (int)sv.size(1), (int)k0, (int)K, scale, cur_stream()));
}

void shapley_column(const at::Tensor& L, const at::Tensor& perm, at::Tensor& sv_col, int64_t k0, double scale) {
  check_cuda_f32(L, "losses");
  TORCH_CHECK(L.dim() == 2 && L.is_contiguous(), "losses must be contiguous (K+1, B)");
  TORCH_CHECK(perm.scalar_type() == at::kInt && perm.is_contiguous(), "perm must be int32");
  TORCH_CHECK(sv_col.scalar_type() == at::kDouble && sv_col.is_contiguous(), "sv_col must be float64 (n,)");
  const int64_t K = L.size(0) - 1;
  TORCH_CHECK(k0 + K <= perm.numel() && perm.numel() == sv_col.numel(), "shape mismatch");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(L.device());
  TP_CHECK_HIP(tp_shapley_column(L.data_ptr<float>(), perm.data_ptr<int>(), sv_col.data_ptr<double>(),
                                 (int)L.size(1), (int)k0, (int)K, scale, cur_stream()));
}

std::tuple<at::Tensor, at::Tensor> cross_entropy(const at::Tensor& logits_, const at::Tensor& target_,
                                                 double gscale, bool want_grad) {
  check_cuda_f32(logits_, "logits");
  TORCH_CHECK(logits_.dim() == 2, "logits must be (B, classes)");
  auto logits = logits_.contiguous();
  auto target = target_.to(at::kLong).contiguous();
  TORCH_CHECK(target.numel() == logits.size(0), "target length mismatch");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(logits.device());
  auto loss = at::empty({logits.size(0)}, logits.options());
  at::Tensor grad = want_grad ? at::empty_like(logits) : at::Tensor();
  TP_CHECK_HIP(tp_cross_entropy(logits.data_ptr<float>(), target.data_ptr<int64_t>(), loss.data_ptr<float>(),
                                want_grad ? grad.data_ptr<float>() : nullptr, (int)logits.size(0),
                                (int)logits.size(1), (float)gscale, cur_stream()));
  return {loss, grad};
}

// Batch of a device-resident uint8 dataset: gather rows ``idx`` of src (N, C, H, W), optional
// per-image (dy, dx, flip) augmentation ``aug`` (B, 3) int32 with zero padding ``pad``, then
// ToTensor + Normalize -> fp32 (B, C, H, W).
at::Tensor augment_u8(const at::Tensor& src, const at::Tensor& idx, const c10::optional<at::Tensor>& aug, int64_t pad,
                      const at::Tensor& mean, const at::Tensor& inv_std) {
  TORCH_CHECK(src.is_cuda() && src.scalar_type() == at::kByte && src.dim() == 4 && src.is_contiguous(),
              "src must be a contiguous uint8 (N, C, H, W) GPU tensor");
  TORCH_CHECK(idx.is_cuda() && idx.scalar_type() == at::kLong && idx.dim() == 1 && idx.is_contiguous(),
              "idx must be a contiguous int64 GPU vector");
  const int64_t B = idx.size(0), C = src.size(1), H = src.size(2), W = src.size(3);
  const int* ap = nullptr;
  if (aug.has_value() && aug->defined()) {
    TORCH_CHECK(aug->is_cuda() && aug->scalar_type() == at::kInt && aug->is_contiguous() && aug->numel() == 3 * B,
                "aug must be a contiguous int32 (B, 3) GPU tensor");
    ap = aug->data_ptr<int>();
  }
  check_cuda_f32(mean, "mean");
  check_cuda_f32(inv_std, "inv_std");
  TORCH_CHECK(mean.numel() == C && inv_std.numel() == C && mean.is_contiguous() && inv_std.is_contiguous(),
              "mean / inv_std must have C elements");
  TORCH_CHECK(pad >= 0, "pad must be >= 0");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(src.device());
  auto out = at::empty({B, C, H, W}, src.options().dtype(at::kFloat));
  TP_CHECK_HIP(tp_augment_u8(src.data_ptr<uint8_t>(), idx.data_ptr<int64_t>(), ap, (int)B, (int)C, (int)H, (int)W,
                             (int)pad, mean.data_ptr<float>(), inv_std.data_ptr<float>(), out.data_ptr<float>(),
                             cur_stream()));
  return out;
}

// Inverted dropout with a counter-based Philox mask (forward and, with the same seed, backward).
at::Tensor dropout(const at::Tensor& x_, int64_t seed, double p) {
  check_cuda_f32(x_, "x");
  auto x = x_.contiguous();
  TORCH_CHECK(p >= 0.0 && p < 1.0, "dropout p must be in [0, 1)");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty_like(x);
  TP_CHECK_HIP(tp_dropout(x.data_ptr<float>(), y.data_ptr<float>(), x.numel(), (unsigned long long)seed, p,
                          cur_stream()));
  return y;
}

// Training max-pool on NHWC (B, H, W, C), C % 4 == 0: (y, window-local argmax bytes); the
// backward gathers (deterministic). avgpool_bwd: global average pool gradient (B, C) -> (B, H, W, C).
std::tuple<at::Tensor, at::Tensor> maxpool_train_fwd(const at::Tensor& x, int64_t k, int64_t s, int64_t pad) {
  check_cuda_f32(x, "x");
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.size(3) % 4 == 0, "x must be contiguous NHWC with C % 4 == 0");
  const int64_t B = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  const int64_t Ho = (H + 2 * pad - k) / s + 1, Wo = (W + 2 * pad - k) / s + 1;
  TORCH_CHECK(k >= 1 && k * k <= 255 && s >= 1 && pad >= 0 && 2 * pad <= k && Ho > 0 && Wo > 0, "bad pool geometry");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(x.device());
  auto y = at::empty({B, Ho, Wo, C}, x.options());
  auto am = at::empty({B, Ho, Wo, C}, x.options().dtype(at::kByte));
  TP_CHECK_HIP(tp_maxpool_fwd_arg(x.data_ptr<float>(), y.data_ptr<float>(), am.data_ptr<uint8_t>(), (int)B, (int)H,
                                  (int)W, (int)C, (int)k, (int)s, (int)pad, cur_stream()));
  return {y, am};
}

at::Tensor maxpool_train_bwd(const at::Tensor& g_, const at::Tensor& am, int64_t H, int64_t W, int64_t k, int64_t s,
                             int64_t pad) {
  check_cuda_f32(g_, "g");
  auto g = g_.contiguous();
  TORCH_CHECK(g.dim() == 4 && am.sizes() == g.sizes() && am.scalar_type() == at::kByte && am.is_contiguous() &&
                  am.device() == g.device(), "am must be the forward's (B, Ho, Wo, C) uint8 argmax");
  const int64_t B = g.size(0), C = g.size(3);
  TORCH_CHECK(g.size(1) == (H + 2 * pad - k) / s + 1 && g.size(2) == (W + 2 * pad - k) / s + 1, "g shape mismatch");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  auto dx = at::empty({B, H, W, C}, g.options());
  TP_CHECK_HIP(tp_maxpool_bwd(g.data_ptr<float>(), am.data_ptr<uint8_t>(), dx.data_ptr<float>(), (int)B, (int)H,
                              (int)W, (int)C, (int)k, (int)s, (int)pad, cur_stream()));
  return dx;
}

at::Tensor avgpool_bwd(const at::Tensor& g_, int64_t H, int64_t W) {
  check_cuda_f32(g_, "g");
  auto g = g_.contiguous();
  TORCH_CHECK(g.dim() == 2 && g.size(1) % 4 == 0 && H > 0 && W > 0, "g must be (B, C) with C % 4 == 0");
  at::hip::OptionalHIPGuardMasqueradingAsCUDA guard(g.device());
  auto dx = at::empty({g.size(0), H, W, g.size(1)}, g.options());
  TP_CHECK_HIP(tp_avgpool_bwd(g.data_ptr<float>(), dx.data_ptr<float>(), (int)g.size(0), (int)(H * W),
                              (int)g.size(1), cur_stream()));
  return dx;
}

}  // namespace

TORCH_LIBRARY(tpamd, m) {
  m.def("channel_reduce(Tensor? act, Tensor? grad, int mode) -> Tensor");
  m.def("column_accumulate(Tensor v, Tensor(a!) acc_sum, Tensor(b!)? acc_sq) -> ()");
  m.def("channel_fill_(Tensor(a!) x, Tensor idx, float value) -> ()");
  m.def("score_fold_(Tensor(a!)[] T, Tensor(b!)[] acc, bool take_abs, int after) -> ()");
  m.def("nan_channels(Tensor x) -> Tensor");
  m.def("gather_multi(Tensor[] srcs, int[] axes, Tensor keep) -> Tensor[]");
  m.def("prefix_mask(Tensor z, Tensor rank, int p0, int K) -> Tensor");
  m.def("shapley_scatter(Tensor L, Tensor perm, Tensor(a!) sv, int row0, int k0, float scale) -> ()");
  m.def("shapley_column(Tensor L, Tensor perm, Tensor(a!) sv_col, int k0, float scale) -> ()");
  m.def("cross_entropy(Tensor logits, Tensor target, float gscale, bool want_grad) -> (Tensor, Tensor)");
  m.def("augment_u8(Tensor src, Tensor idx, Tensor? aug, int pad, Tensor mean, Tensor inv_std) -> Tensor");
  m.def("dropout(Tensor x, int seed, float p) -> Tensor");
  m.def("maxpool_train_fwd(Tensor x, int k, int s, int pad) -> (Tensor, Tensor)");
  m.def("maxpool_train_bwd(Tensor g, Tensor am, int H, int W, int k, int s, int pad) -> Tensor");
  m.def("avgpool_bwd(Tensor g, int H, int W) -> Tensor");
  register_engine_ops_def(m);
}

TORCH_LIBRARY_IMPL(tpamd, CUDA, m) {
  m.impl("channel_reduce", &channel_reduce);
  m.impl("column_accumulate", &column_accumulate);
  m.impl("channel_fill_", &channel_fill_);
  m.impl("score_fold_", &score_fold_);
  m.impl("nan_channels", &nan_channels);
  m.impl("gather_multi", &gather_multi);
  m.impl("prefix_mask", &prefix_mask);
  m.impl("shapley_scatter", &shapley_scatter);
  m.impl("shapley_column", &shapley_column);
  m.impl("cross_entropy", &cross_entropy);
  m.impl("augment_u8", &augment_u8);
  m.impl("dropout", &dropout);
  m.impl("maxpool_train_fwd", &maxpool_train_fwd);
  m.impl("maxpool_train_bwd", &maxpool_train_bwd);
  m.impl("avgpool_bwd", &avgpool_bwd);
  register_engine_ops_impl(m);
}
