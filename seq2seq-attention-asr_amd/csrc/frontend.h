// Encoder front-end operators (frontend.hip) -- SURVEY.md 8f.4.
#pragma once
#include "s2s_common.h"

namespace s2s {

size_t tconv_scratch_bytes(int B, int L, int Din, int Dout, int kW);
int tconv_fwd(hipStream_t st, int B, int L, int Din, int Dout, int kW, int relu, const float* x, const float* W,
              const float* b, float* y);
int tconv_bwd(hipStream_t st, int B, int L, int Din, int Dout, int kW, int relu, const float* x, const float* W,
              const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db, float scale,
              void* scratch, size_t scratch_bytes, hipStream_t wst = nullptr, hipEvent_t wev = nullptr);
int tmaxpool_fwd(hipStream_t st, int B, int L, int D, int kW, int dW, const float* x, float* y, int* idx);
int tmaxpool_bwd(hipStream_t st, int B, int L, int D, int kW, int dW, const int* idx, const float* dy, float* dx);
size_t sconv_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW);
int sconv_fwd(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x,
              const float* Wt, const float* bias, float* y, void* scratch, size_t scratch_bytes);
int sconv_bwd(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x,
              const float* Wt, const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db,
              float scale, void* scratch, size_t scratch_bytes, int col_from_fwd);
int smaxpool_fwd(hipStream_t st, int B, int C, int H, int W, int kW, int kH, int dW, int dH, const float* x, float* y,
                 int* idx);
int smaxpool_bwd(hipStream_t st, int B, int C, int H, int W, int kW, int kH, int dW, int dH, const int* idx,
                 const float* dy, float* dx);
int swap12(hipStream_t st, int B, int D1, int D2, int D3, const float* x, float* y);
int relu_fwd(hipStream_t st, long n, const float* x, float* y);
int relu_bwd(hipStream_t st, long n, const float* x, const float* dy, float* dx);
int logsoftmax_fwd(hipStream_t st, long rows, int n, const float* x, float* y);
int logsoftmax_bwd(hipStream_t st, long rows, int n, const float* y, const float* dy, float* dx);

}  // namespace s2s
