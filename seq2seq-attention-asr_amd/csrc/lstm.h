// LSTM layer sequence (nn.RNN(nn.LSTM(D, H, peepholes), reverse), LSTM.lua:6-136 under
// RNN.lua:120-201) -- SURVEY.md §8 row A7.
#pragma once
#include "s2s_common.h"

namespace s2s {

// Parameter pointers per direction, in this order (W = (out, in), all fp32):
//   for q in (i, f, g, o):  Wqx (H, D), bqx (H), Wqh (H, H), bqh (H)        -> 16 pointers
//   peepholes adds:         Wic (H, H), bic (H), Wfc (H, H), bfc (H), Woc (H, H), boc (H)
constexpr int kLstmParams = 16, kLstmPeepParams = 22;
inline int lstm_nparams(int peep) { return peep ? kLstmPeepParams : kLstmParams; }

struct LstmLayerIO {
  int ndir, B, L, D, H, peep;
  const float* x;  // x[(b*L + t)*ldx + c], c < D
  long ldx;
  const float* const* W;  // W[d * lstm_nparams(peep) + p]
  int reverse[2];
  float* y[2];  // y[d][(b*L + t)*ldy + j]
  long ldy;
  float* saved[2];  // per direction (B, L, 8H): i | f | g | o | c | c_{t-1} | h_{t-1} | tanh(c)
};
struct LstmLayerGrad {
  const float* dy[2];
  long lddy;
  float* dx;  // may be null; sum over directions
  long lddx;
  int dx_accumulate;
  float* const* dW;  // same layout as W; accumulated dW += scale * ...
  float scale;
};

size_t lstm_saved_bytes(int B, int L, int H);
size_t lstm_scratch_bytes(int ndir, int B, int L, int D, int H, int peep);
int lstm_layer_fwd(hipStream_t st, const LstmLayerIO& io, void* scratch, size_t scratch_bytes);
int lstm_layer_bwd(hipStream_t st, const LstmLayerIO& io, const LstmLayerGrad& gr, void* scratch,
                   size_t scratch_bytes);

}  // namespace s2s
