#pragma once
#include "s2s_common.h"

namespace s2s {

// Packing one layer-direction's W{z,r,h} (H, H+D) into the kernel layouts (gru_layers_pack): Uzr (2H,H),
// Uh (H,H), UhT (H,H), UzrT (H,2H), Wx rows [z;r;h] (3H, Kx; columns [D, Kx) zero); a null target is skipped
struct GruPackJob {
  const float* W[3];
  float *Uzr, *Uh, *UhT, *UzrT, *Wx;
  int H, D, Kx;
};
constexpr int kMaxPackJobs = 8;
struct GruPackJobs {
  GruPackJob j[kMaxPackJobs];
  int n;
};
// element range [i0, ...) with stride of one job (the gru_pack kernels and the persistent forward's spare slots)
__device__ __forceinline__ void gru_pack_elems(const GruPackJob& p, long i0, long stride) {
  const int H = p.H, D = p.D, HD = H + D, Kx = p.Kx;
  const long nU = 3L * H * H, nX = p.Wx ? 3L * H * Kx : 0;
  for (long i = i0; i < nU + nX; i += stride) {
    if (i < nU) {
      const int g = (int)(i / ((long)H * H));
      const int rem = (int)(i - (long)g * H * H);
      const int n = rem / H, k = rem - n * H;
      const float w = p.W[g][(long)n * HD + k];
      if (g < 2) {
        if (p.Uzr) p.Uzr[(long)(g * H + n) * H + k] = w;
        if (p.UzrT) p.UzrT[(long)k * 2 * H + g * H + n] = w;
      } else {
        if (p.Uh) p.Uh[(long)n * H + k] = w;
        if (p.UhT) p.UhT[(long)k * H + n] = w;
      }
    } else {
      const long j = i - nU;
      const int g = (int)(j / ((long)H * Kx));
      const long rem = j - (long)g * H * Kx;
      const int n = (int)(rem / Kx), c = (int)(rem - (long)n * Kx);
      p.Wx[(long)(g * H + n) * Kx + c] = c < D ? p.W[g][(long)n * HD + H + c] : 0.f;
    }
  }
}

// the model step's head in one launch (gru_step_head, gru.hip): pad the layer-1 input, pack jobs, prepare the
// first persistent launch's sync region (sync_prep's work: sync null = none)
struct GruStepHead {
  const float* src;
  long lds;
  float* dst;
  int rows, cols, dcols;  // rows = 0: no padding
  GruPackJobs pack;
  char* sync;
  size_t prep_bytes;
  char* clear;
  // optional: the loss seed dlogp = -labelmask ((B, T, O), steps t >= tlen[b] zero; nll_seed's dlogp) and a zero
  // fill of n4 16-byte words at zero (the step's gradient zeroing)
  float* dlogp = nullptr;
  const int* labels = nullptr;
  const int* tlen = nullptr;
  int B = 0, T = 0, O = 0;
  void* zero = nullptr;
  size_t zero_n4 = 0;
  int zero_tail = 0;  // floats after the n4 words (< 4)
};
int gru_persist_step_head(hipStream_t st, const GruStepHead& h);

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
  // weight packing deferred to this launch's spare slots (the layouts later launches read), or null
  const GruPackJobs* pack = nullptr;
  int excl = 0;                // reserve the CU (kExclLds) beside side-stream GEMMs
  unsigned* status = nullptr;  // harvest this launch's failure words into these status words (null: the caller does)
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
  int excl = 0;
  unsigned* status = nullptr;
  // optional in-launch weight gradients (gru_persist_wgrad_fits): wdW[d][g] += wscale dA^T [h_{t-1} or q | x]
  // (gru_layer_wgrad's products) by workers beside the chains; wx (B*L, wldx) the layer input, wD columns;
  // wpart: ndir * ceil(B/16) * 3H * (H + round_up(wD, 16)) floats of the utterance tiles' partials
  int wgrad = 0;
  float* wdW[2][3] = {};
  float wscale = 1.f;
  const float* wx = nullptr;
  long wldx = 0;
  int wD = 0;
  float* wpart = nullptr;
};

bool gru_persist_supported(int ndir, int B, int H);
// the BPTT launch can carry its layer's weight gradients (GruPersistBwd::wgrad) at this shape (input width D)
bool gru_persist_wgrad_fits(int ndir, int B, int H, int D);
// the backward's spare slots can produce its dy (the dX GEMM of the layer above) in-launch
bool gru_persist_fused_dy(int ndir, int B, int H, int K, long ldw, long lddy);
bool gru_persist_fused_xproj(int ndir, int B, int H, int Kx);
size_t gru_persist_sync_bytes(int B, int L, int H);
size_t gru_persist_prep_bytes(int B, int L, int H);  // the part sync_prep (or a preparing launch) zeroes
bool gru_persist_can_prep_next(int ndir, int B, int H, bool fwd);
int gru_persist_fwd(hipStream_t st, const GruPersistFwd& f, void* sync);
int gru_persist_bwd(hipStream_t st, const GruPersistBwd& b, void* sync);
// test probe of the hand-off timeout path (sync: >= 768 bytes of device memory)
int handoff_timeout_probe_launch(hipStream_t st, void* sync, unsigned* status);

}  // namespace s2s
