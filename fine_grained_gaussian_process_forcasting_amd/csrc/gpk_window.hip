// GPU-resident window sampler: gather of (enc, dec, y) training windows from a
// device-resident, (id, time)-sorted feature table.
//
// Reference: Utils/base_train.py:29-97 (sample_train_val_test) slices each chosen
// window sliced = group.iloc[start - T : start] into enc = rows [0, n_enc),
// dec = rows [n_enc, T - pred_len), outputs = target column of rows [T - pred_len, T),
// as float64 numpy, then torch.FloatTensor and a per-step host->device copy
// (train.py:160-161). Here the table lives in HBM as float32 (the same rounding as
// FloatTensor) and a window is one contiguous run of T * F floats: the gather is a
// batched copy, HBM-bound byte work (no arithmetic), coalesced 16-B loads/stores when
// the run is 16-B aligned. A window row of -1 yields zeros (the reference's
// zero-filled windows when max_samples exceeds the valid locations).
#include "gpk_common.h"
#include "gpk_internal.h"

namespace {

__global__ void __launch_bounds__(256)
gpk_window_gather_kernel(const float* __restrict__ table, int F, const long long* __restrict__ rows,
                         int n_enc, int n_dec, int pred_len, int tcol, float* __restrict__ enc,
                         float* __restrict__ dec, float* __restrict__ y) {
  const int b = blockIdx.x, tid = threadIdx.x;
  const long long r0 = rows[b];
  const bool zero = r0 < 0;
  const size_t ne = (size_t)n_enc * F, nd = (size_t)n_dec * F;
  const float* src = table + (zero ? 0 : (size_t)r0 * F);
  float* de = enc + (size_t)b * ne;
  float* dd = dec + (size_t)b * nd;
  // enc and dec are contiguous in the table: [src, src + ne) and [src + ne, src + ne + nd)
  const bool vec = ((((uintptr_t)src) | ((uintptr_t)de) | ((uintptr_t)dd) | (ne * 4)) & 15) == 0;
  if (vec) {
    for (size_t e = (size_t)tid * 4; e < ne; e += 256 * 4)
      *(float4*)&de[e] = zero ? float4{0.f, 0.f, 0.f, 0.f} : *(const float4*)&src[e];
    const size_t nd4 = nd & ~(size_t)3;
    for (size_t e = (size_t)tid * 4; e < nd4; e += 256 * 4)
      *(float4*)&dd[e] = zero ? float4{0.f, 0.f, 0.f, 0.f} : *(const float4*)&src[ne + e];
    for (size_t e = nd4 + tid; e < nd; e += 256) dd[e] = zero ? 0.f : src[ne + e];
  } else {
    for (size_t e = tid; e < ne; e += 256) de[e] = zero ? 0.f : src[e];
    for (size_t e = tid; e < nd; e += 256) dd[e] = zero ? 0.f : src[ne + e];
  }
  for (int k = tid; k < pred_len; k += 256)
    y[(size_t)b * pred_len + k] = zero ? 0.f : src[(size_t)(n_enc + n_dec + k) * F + tcol];
}

}  // namespace

int gpk_launch_window_gather(const float* table, int F, const long long* rows, int B, int n_enc,
                             int n_dec, int pred_len, int tcol, float* enc, float* dec, float* y,
                             hipStream_t stream) {
  hipLaunchKernelGGL(gpk_window_gather_kernel, dim3(B), dim3(256), 0, stream, table, F, rows, n_enc,
                     n_dec, pred_len, tcol, enc, dec, y);
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : (int)e;
}
