// C launchers exported by csrc/kernels/*.hip (no torch types cross this boundary).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {
// channel_reduce.hip
hipError_t tp_channel_reduce(const float* act, const float* grad, float* out, float* ws, int B, int C, int S,
                             int mode, int channels_last, hipStream_t st);
int tp_channel_reduce_ws_elems(int B, int C, int S, int channels_last);
hipError_t tp_column_accumulate(const float* v, double* acc_sum, double* acc_sq, int B, int C, hipStream_t st);
// prune_ops.hip
hipError_t tp_channel_fill(float* x, long long B, int C, long long S, const int64_t* idx, int nidx, float value,
                           hipStream_t st);
hipError_t tp_nan_channels(const float* x, long long B, int C, long long S, uint8_t* flags, hipStream_t st);
hipError_t tp_gather_multi(const void* const* srcs, void* const* dsts, const long long* outer, const long long* n,
                           const long long* inner, int count, int elsize, const int64_t* keep, long long nkeep,
                           hipStream_t st);
// shapley.hip
hipError_t tp_prefix_mask(const float* z, float* out, const int* rank, long long N, int C, int S, int channels_last,
                          int p0, int K, hipStream_t st);
hipError_t tp_shapley_scatter(const float* L, const int* perm, double* sv, int row0, int B, int n, int k0, int K,
                              double scale, hipStream_t st);
hipError_t tp_shapley_column(const float* L, const int* perm, double* sv_col, int B, int k0, int K, double scale,
                             hipStream_t st);
hipError_t tp_cross_entropy(const float* logits, const int64_t* target, float* loss, float* grad, int B, int NC,
                            float gscale, hipStream_t st);
// train_ops.hip
hipError_t tp_dropout(const float* x, float* y, long long n, unsigned long long seed, double p, hipStream_t st);
hipError_t tp_maxpool_fwd_arg(const float* x, float* y, uint8_t* am, int B, int H, int W, int C, int k, int s, int pad,
                              hipStream_t st);
hipError_t tp_maxpool_bwd(const float* g, const uint8_t* am, float* dx, int B, int H, int W, int C, int k, int s,
                          int pad, hipStream_t st);
hipError_t tp_avgpool_bwd(const float* g, float* dx, int B, int HW, int C, hipStream_t st);
// data_ops.hip
hipError_t tp_augment_u8(const uint8_t* src, const int64_t* idx, const int* aug, int B, int C, int H, int W, int pad,
                         const float* mean, const float* inv_std, float* out, hipStream_t st);
}

#ifdef __cplusplus
namespace torch { class Library; }
void register_engine_ops_def(torch::Library& m);
void register_engine_ops_impl(torch::Library& m);
#endif

extern "C" int tp_score_fold_ws_elems(const int* B, const int* C, int count);
extern "C" hipError_t tp_score_fold_multi(float* const* T, double* const* acc, const int* B, const int* C,
                                          const int* R, int count, int take_abs, int after, double* ws,
                                          hipStream_t st);
