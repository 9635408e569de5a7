#pragma once
#include "s2s_common.h"

namespace s2s {

// GRU gate nonlinearities of the encoder kernels (per-step gru.hip and persistent gru_persist.hip, bitwise the
// same in both): v_exp_f32 + v_rcp_f32 forms instead of expf / an IEEE divide / libm tanhf (~40 dependent
// instructions per gate on the recurrences' critical path).  sigmoid: relative error ~1e-7 (x*log2e rounding,
// 1-ulp exp and rcp), saturating to 0 / 1; tanh = 1 - 2 / (exp(2x) + 1): ~1e-7 absolute, saturating to +-1.
__device__ __forceinline__ float gru_sigmoid(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
__device__ __forceinline__ float gru_tanh(float x) { return 1.0f - 2.0f * __builtin_amdgcn_rcpf(__expf(2.0f * x) + 1.0f); }

struct GruPackJobs;  // gru_persist.h

// One GRU layer, 1 or 2 directions sharing the same input x (the bidirectional
// encoder layer of timit/model_chorowski_baseline.lua:22-32 runs both in each launch).
struct GruLayerIO {
  int ndir, B, L, D, H;
  const float* x;  // x[(b*L + t)*ldx + c], c < D
  long ldx;
  const float* W[2][3];  // per direction Wz, Wr, Wh, each (H, H+D) row-major
  int reverse[2];
  float* y[2];  // y[d][(b*L + t)*ldy + j]
  long ldy;
  float* saved[2];  // per direction (B, L, 5H)
  int Dx = 0;       // x columns [D, Dx) are readable zeros (0 = D; Dx <= round_up(D, 32)):
                    // the input GEMMs then run over K = Dx on aligned, unguarded tiles
  const float* packed = nullptr;  // gru_layer_pack output for these weights (null: pack per call)
  // variable-length batch: (B) device int32 frames per utterance, 1 <= len_b <= L (null: all L).  The
  // recurrence is h_t = m_t GRU(h_{t-1}, x_t), m_t = 1[t < len_b]: outputs are 0 on the padding frames and
  // the reverse direction starts at each utterance's own last frame (RNN.lua:142-145 on the utterance alone)
  const int* len = nullptr;
  // optional sync-region hand-over of the persistent launches (model step): use `sync` (>=
  // gru_persist_sync_bytes) instead of the scratch's; sync_prepared = the launch before prepared it;
  // sync_next / sync_next_prep: this launch prepares that region for the next one (when it can:
  // gru_layer_preps_next)
  void* sync = nullptr;
  int sync_prepared = 0;
  void* sync_next = nullptr;
  size_t sync_next_prep = 0;
  // forward only: weight packing (gru_layers_pack's deferred jobs) done by this launch's spare slots
  const GruPackJobs* pack_jobs = nullptr;
  // the persistent launches reserve their CU (unused dynamic LDS) so side-stream GEMMs only take idle CUs
  int excl = 0;
  // the calling context's status words (handoff.h): the layer's persistent launch is followed by a harvest of
  // its sync region into them (s2s_ctx_status); null = no harvest (the model step harvests once at its end)
  unsigned* status = nullptr;
};
struct GruLayerGrad {
  const float* dy[2];  // dy[d][(b*L+t)*lddy + j]
  long lddy;
  float* dx;  // may be null; dx[(b*L+t)*lddx + c]
  long lddx;
  int dx_accumulate;
  float* dW[2][3];  // accumulated: dW += scale * ...
  float scale;
  hipEvent_t prep_event;  // optional: recorded between the persistent BPTT's sync prep and its launch
  // optional: dy[0] (both directions, dy[1] = dy[0] + H) is the layer above's dX, ydA (B*L, yK; stride
  // yldA) . yWx (yK, yN; stride yldw), not yet computed -- the persistent BPTT's spare slots produce it
  // in-launch (gru_persist_fused_dy), otherwise one GEMM in front of the BPTT
  const float* ydA;
  long yldA;
  int yK, yN;
  const float* yWx;
  long yldw;
  // optional with ydA (the top layer, whose dy is the decoder's dh; fused launch only): dy also gets
  // sum_t yalpha[b, t, l] ydc[b, t, :] (yalpha (B, yT, L), ydc (B, yT, lddy)) -- then ydA . yWx is dVh V
  const float* yalpha = nullptr;
  const float* ydc = nullptr;
  int yT = 0;
  // optional (persistent BPTT, gru_layer_wgrad_fused): the launch computes this layer's weight gradients itself
  // (dW += scale ..., gru_layer_wgrad's products) -- no gru_layer_wgrad after it; wpart: gru_layer_wgrad_part_floats
  int wgrad = 0;
  float* wpart = nullptr;
};

size_t gru_layer_scratch_bytes(int ndir, int B, int L, int D, int H);
// the layer's persistent BPTT launch can carry its weight gradients (GruLayerGrad::wgrad), and the partials'
// workspace that needs (floats)
bool gru_layer_wgrad_fused(const GruLayerIO& io);
size_t gru_layer_wgrad_part_floats(const GruLayerIO& io);
// the layer's recurrences run as persistent launches (sync regions, hand-offs) rather than per-step kernels
bool gru_layer_persistent(const GruLayerIO& io);
// Every kernel layout of one layer's weights (recurrent Uzr/Uh and their transposes, the padded
// x-projection rows), packed once per step so the forward and backward launches skip it.
size_t gru_layer_pack_bytes(int ndir, int D, int H);
int gru_layer_pack(hipStream_t st, const GruLayerIO& io, float* packed);
// one launch; defer (optional): pack only layer 1's forward layouts now and append the rest (layer 1's
// backward transposes, every later layer) to *defer for layer 1's persistent forward (GruLayerIO::pack_jobs)
int gru_layers_pack(hipStream_t st, const GruLayerIO* ios, float* const* packed, int nlayers,
                    GruPackJobs* defer = nullptr);
// The model step's head as ONE launch (step_head_kernel): the layer-1 input padded to Dp columns (x (rows, ldx)
// -> xpad (rows, dcols), zeros past cols), gru_layers_pack's jobs for `ios` (deferred jobs returned in *defer as
// there) and, when sync != null, the sync_prep of the step's first persistent launch (its region, prep bytes and
// the other region's header `clear`) -- three back-to-back launches on the critical path before (pad_cols_kernel,
// gru_pack_multi, sync_prep: 24 us in the r05 trace)
struct GruStepHead;
int gru_step_head(hipStream_t st, const GruLayerIO* ios, float* const* packed, int nlayers, GruPackJobs* defer,
                  const float* x, long ldx, float* xpad, int rows, int cols, int dcols, void* sync, size_t prep_bytes,
                  void* clear, const GruStepHead* extra = nullptr);
int gru_layer_fwd(hipStream_t st, const GruLayerIO& io, void* scratch, size_t scratch_bytes);
int gru_layer_bwd(hipStream_t st, const GruLayerIO& io, const GruLayerGrad& gr, void* scratch, size_t scratch_bytes);
// split form used by the model step: core = weight packing + BPTT + dx (critical path), writing the
// gate gradients into dA (B, L, 3*ndir*H) (dA == nullptr: inside scratch); wgrad = the dW GEMMs.
int gru_layer_bwd_core(hipStream_t st, const GruLayerIO& io, const GruLayerGrad& gr, float* dA, void* scratch,
                       size_t scratch_bytes);
int gru_layer_wgrad(hipStream_t st, const GruLayerIO& io, const GruLayerGrad& gr, const float* dA, GemmWs ws);
float* gru_layer_dA(const GruLayerIO& io, void* scratch);
// the layer's persistent launch (forward or backward) would prepare io.sync_next for the next launch
bool gru_layer_preps_next(const GruLayerIO& io, bool fwd);
size_t gru_layer_sync_prep_bytes(const GruLayerIO& io);
// gru_layer_bwd_core will produce gr's dy (ydA . yWx) inside its persistent BPTT launch
bool gru_layer_dy_fused(const GruLayerIO& io, const GruLayerGrad& gr);
// the x-weights (3 ndir H, Kx) rows of a packed layer (gru_layers_pack) and their row stride Kx
const float* gru_layer_packed_wx(const GruLayerIO& io, long* ldw);

}  // namespace s2s
