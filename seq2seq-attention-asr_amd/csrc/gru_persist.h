#pragma once
#include "s2s_common.h"

namespace s2s {

struct GruPersistFwd {
  int ndir, B, L, H;
  // fused x-projection (gru_persist_fused_xproj): x (B*L, ldx) with Kx readable columns and the
  // packed x-weights Wx (ndir*3H, Kx); xp[0] is then the (B*L, ldxp) output base.  x = nullptr: xp
  // precomputed by the caller
  const float* x = nullptr;
  long ldx = 0;
  int Kx = 0;
  const float* Wx = nullptr;
  const float* xp[2];
  long ldxp;
  const float* Uzr[2];
  const float* Uh[2];
  float* y[2];
  long ldy;
  float* sv[2];
  int reverse[2];
  const int* len = nullptr;  // (B) frames per utterance (null: all L)
  // sync-region hand-over between consecutive persistent launches: prepared = the region was prepared by
  // the launch before (no sync_prep in front of this one); next_sync / next_prep: this launch's spare slots
  // prepare that region for the next launch (gru_persist_can_prep_next)
  int prepared = 0;
  void* next_sync = nullptr;
  size_t next_prep = 0;
};
struct GruPersistBwd {
  int ndir, B, L, H;
  const float* UhT[2];
  const float* UzrT[2];
  float* sv[2];
  const float* dy[2];
  long lddy;
  float* dA[2];
  long ldA;
  int reverse[2];
  hipEvent_t prep_event;  // optional: recorded after the sync prep, right before the launch
  const int* len = nullptr;  // (B) frames per utterance (null: all L)
  // optional fused dy: dy[0] .. (the dy buffer, both directions at column d H) = ydA (B*L, yK; row stride
  // yldA) . yWx (yK, ndir H; row stride yldw) -- the dX of the layer above, computed by the spare slots
  const float* ydA = nullptr;
  long yldA = 0;
  int yK = 0;
  const float* yWx = nullptr;
  long yldw = 0;
  // optional: dy += sum_t yalpha[b, t, l] ydc[b, t, :] (the decoder's context term of dh; row stride lddy)
  const float* yalpha = nullptr;
  const float* ydc = nullptr;
  int yT = 0;
  int prepared = 0;  // as GruPersistFwd
  void* next_sync = nullptr;
  size_t next_prep = 0;
};

bool gru_persist_supported(int ndir, int B, int H);
// the backward's spare slots can produce its dy (the dX GEMM of the layer above) in-launch
bool gru_persist_fused_dy(int ndir, int B, int H, int K, long ldw, long lddy);
bool gru_persist_fused_xproj(int ndir, int B, int H, int Kx);
// 1 = persistent GRU launches reserve their CU (see kExclLds); set around a step whose weight-gradient
// GEMMs run on a side stream
void gru_persist_set_exclusive(int on);
size_t gru_persist_sync_bytes(int B, int L, int H);
size_t gru_persist_prep_bytes(int B, int L, int H);  // the part sync_prep (or a preparing launch) zeroes
bool gru_persist_can_prep_next(int ndir, int B, int H, bool fwd);
int gru_persist_fwd(hipStream_t st, const GruPersistFwd& f, void* sync);
int gru_persist_bwd(hipStream_t st, const GruPersistBwd& b, void* sync);

}  // namespace s2s
