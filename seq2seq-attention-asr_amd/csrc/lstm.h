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
// saved activations per (utterance, step): 8 rows of H
enum LstmSv { SV_I = 0, SV_F, SV_G, SV_O, SV_C, SV_CP, SV_HP, SV_TC, SV_N };

struct LstmLayerIO {
  int ndir, B, L, D, H, peep;
  const float* x;  // x[(b*L + t)*ldx + c], c < D
  long ldx;
  const float* const* W;  // W[d * lstm_nparams(peep) + p]
  int reverse[2];
  float* y[2];  // y[d][(b*L + t)*ldy + j]
  long ldy;
  float* saved[2];  // per direction (B, L, 8H): i | f | g | o | c | c_{t-1} | h_{t-1} | tanh(c)
  // (B) frames per utterance (device), null = all L: h_t = c_t = 0 for t >= len_b; the backward zeroes dh, dc there
  const int* len = nullptr;
  // the calling context's status words: the persistent launches are followed by a harvest of their sync region
  // into them (s2s_ctx_status); null = no harvest
  unsigned* status = nullptr;
};
struct LstmLayerGrad {
  const float* dy[2];
  long lddy;
  float* dx;  // may be null; sum over directions
  long lddx;
  int dx_accumulate;
  float* const* dW;  // same layout as W; accumulated dW += scale * ...
  float scale;
  // optional: the weight / bias gradients go to stream wst, forked from st by event wev once dA is final (the
  // caller joins wst later; dx then runs its GEMM without the split-K workspace the gradients use)
  hipStream_t wst = nullptr;
  hipEvent_t wev = nullptr;
};

// Persistent recurrences (lstm_persist.hip): the whole sweep of a layer's directions in one launch (no peepholes)
struct LstmPersistArgs {
  int ndir, B, L, H;
  int reverse[2];
  const float* xp[2];  // fwd: x-projections (+ biases) of direction d at column 0 of its 4H block
  long ldxp;
  const float* Wh[2][4];
  float* y[2];
  long ldy;
  float* sv[2];
  const float* Wb[2];  // bwd: packed (2H, 4H)
  const float* dy[2];
  long lddy;
  float* dA[2];
  long ldA;
  const int* len;  // (B) frames per utterance or null (LstmLayerIO::len)
};
bool lstm_persist_supported(int ndir, int B, int H, int peep);
size_t lstm_persist_sync_bytes(int ndir, int B, int L, int H);
int lstm_persist_fwd(hipStream_t st, const LstmPersistArgs& f, void* sync, unsigned* status);
int lstm_persist_bwd(hipStream_t st, const LstmPersistArgs& b, void* sync, unsigned* status);

size_t lstm_saved_bytes(int B, int L, int H);
size_t lstm_scratch_bytes(int ndir, int B, int L, int D, int H, int peep);
int lstm_layer_fwd(hipStream_t st, const LstmLayerIO& io, void* scratch, size_t scratch_bytes);
int lstm_layer_bwd(hipStream_t st, const LstmLayerIO& io, const LstmLayerGrad& gr, void* scratch,
                   size_t scratch_bytes);

}  // namespace s2s
