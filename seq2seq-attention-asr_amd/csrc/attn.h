#pragma once
#include "s2s_common.h"

namespace s2s {

// Attention decoder dims: nn.Attention(decoder_recurrent, decoder_mlp, scoreDepth, ...,
// stateDepth, annotationDepth, outputDepth, monoAlignPenalty, penaltyLambda)
// (Attention.lua:15-24) with the Chorowski decoder_recurrent = GRU(S,S) and
// decoder_mlp = Maxout(S+A, M, K) -> Linear(M, O) -> LogSoftMax
// (timit/model_chorowski_baseline.lua:48-59).
struct AttnDims {
  int B, L, T;
  int A;   // annotationDepth
  int Sc;  // scoreDepth
  int S;   // stateDepth
  int O;   // outputDepth
  int M;   // mlpDepth
  int K;   // maxout window
  float penalty;
  float dropout = 0.f;                    // nn.Dropout(p) before the Maxout (0 = none)
  unsigned long long dropout_seed = 0;
  const float* dropout_mask = nullptr;    // injected (B, T, S+A) multipliers, or null
  // hybrid location-aware attention (Attention.lua:75-98): hybridAttendFilterSize kW and
  // hybridAttendFeatureMaps nF; nF = 0: content-only (the Chorowski baseline)
  int hk = 0, hf = 0;
  // external decoder_mlp: the forward stops at the MLP input [s_t; c_t] (saved VV rows) and the
  // backward takes its gradient in place of dlogp; Wm / bm / Wo / bo are not used
  int ext = 0;
  // decoder_recurrent = nn.LSTM(S, S) (no peepholes) instead of nn.GRU(S, S): the conv + BiLSTM
  // model of timit/timit.lua:137 (per-step decoder kernels)
  int lstm = 0;
  // when set, the in-kernel dropout seed is read from this device word (a replayed graph: the host
  // writes each step's seed there before the replay) instead of dropout_seed
  const unsigned long long* dropout_seed_dev = nullptr;
  // variable-length batch (device int32, B each, or null = all full length): frames L_b of each
  // utterance's annotations (1 <= L_b <= L; alpha = 0 on frames >= L_b, MonotonicAlignment over its L_b
  // frames) and labels T_b (1 <= T_b <= T; decoder steps >= T_b carry no penalty gradient -- the caller's
  // dlogp is 0 there, the reference never runs them)
  const int* flen = nullptr;
  const int* tlen = nullptr;
  // the XCD-local decoder's sync regions were prepared by attn_fwd_prologue (the model step runs it, and
  // joins it, before the decoder): attn_fwd / attn_bwd_core then launch no sync_prep of their own
  int syncs_in_prologue = 0;
  // the loss seed dlogp (B*T, O) is final when attn_fwd runs (the model step's head writes it): the XCD-local
  // forward's merged head launch then also runs the MLP head's backward (do, dm, the Maxout scatter into dU) and
  // attn_bwd_core launches no dec_mlp_head_bwd (attn_head_bwd_fused); attn_bwd_core's dlogp must be this pointer
  const float* dlogp_early = nullptr;
};
int set_device_u64(hipStream_t st, unsigned long long* p, unsigned long long v);
constexpr int kMaxHybK = 8;  // largest hybrid filter served (the reference's fallback model uses 5)
struct AttnParams {
  const float *V, *Ws, *bs, *we, *Wy, *by, *Wc, *bc, *Wd, *bd, *Wz, *Wr, *Wh, *Wm, *bm, *Wo, *bo;
  const float *hybW = nullptr, *hybb = nullptr, *hybU = nullptr;  // (nF, kW), (nF), (Sc, nF) when hf > 0
  // decoder LSTM (lstm = 1): for q in (i, f, g, o): Wqx (S, S), bqx (S), Wqh (S, S), bqh (S) (LSTM.lua:25-29)
  const float* lstm[16] = {};
};
struct AttnGrads {
  float *V, *Ws, *bs, *we, *Wy, *by, *Wc, *bc, *Wd, *bd, *Wz, *Wr, *Wh, *Wm, *bm, *Wo, *bo;
  float *hybW = nullptr, *hybb = nullptr, *hybU = nullptr;
  float* lstm[16] = {};
};

int attn_check_dims(const AttnDims& d);
size_t attn_saved_bytes(const AttnDims& d);
size_t attn_scratch_bytes(const AttnDims& d);
// h (B, L, A) contiguous; labels (B, T) int32 0-based; logp (B, T, O) out.
// side / ev (optional, both or neither): a second stream and 5 events for work off the critical
// path (the model step's split mode); attn_fwd and attn_bwd_core must then use the same ones.
int attn_fwd(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P, float* logp,
             void* saved, void* scratch, size_t scratch_bytes, bool prologue_done = false, hipStream_t side = nullptr,
             hipEvent_t* ev = nullptr);
// The decoder's parameter folds / teacher-forced constants (needs only P and labels): the model
// step issues it beside the encoder and then calls attn_fwd(..., prologue_done = true).
int attn_fwd_prologue(hipStream_t st, const AttnDims& d, const int* labels, const AttnParams& P, void* saved,
                      void* scratch);
// dlogp (B, T, O); dh (B, L, A) written (accumulate_dh=0) or accumulated; grads accumulated with scale.
int attn_bwd(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P,
             const void* saved, const float* dlogp, float* dh, int accumulate_dh, const AttnGrads& G, float scale,
             void* scratch, size_t scratch_bytes);
// The two terms of the XCD-local path's dh (after its loop): dh[b, l, :] = sum_t alpha[b, t, l] dc[b, t, :]
// (alpha (B, T, L), dc (B, T, A)) + dVh[b, l, :] V (dVh (B, L, Sc), V (Sc, A)).
struct AttnDhTerms {
  const float* alpha = nullptr;
  const float* dc = nullptr;
  const float* dvh = nullptr;
  const float* V = nullptr;
  int B = 0, L = 0, T = 0, A = 0, Sc = 0;
  GemmWs gws;  // split-K workspace for attn_dh_gemms
};
// dh = the two terms, as GEMMs (alpha^T dc per utterance, then -- after dvh_ready when given -- dh += dVh V)
int attn_dh_gemms(hipStream_t st, const AttnDhTerms& t, float* dh, int accumulate_dh, hipEvent_t dvh_ready = nullptr);
// split form used by the model step (wgrad may run on a side stream after core).  defer_dh (optional):
// when the XCD-local path runs and dh is not accumulated, dh is NOT computed; its terms are returned there
// (defer_dh->dvh != nullptr) for the caller to fuse into the encoder's BPTT launch.
int attn_bwd_core(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P,
                  const void* saved, const float* dlogp, float* dh, int accumulate_dh, void* scratch,
                  size_t scratch_bytes, hipStream_t side = nullptr, hipEvent_t* ev = nullptr,
                  AttnDhTerms* defer_dh = nullptr);
int attn_bwd_wgrad(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P,
                   const void* saved, const AttnGrads& G, float scale, void* scratch);
// alpha (B, T, L) view into the saved buffer (Attention:alpha(), Attention.lua:241-243)
const float* attn_saved_alpha(const AttnDims& d, const void* saved);
const int* attn_saved_maxout_argmax(const AttnDims& d, const void* saved);
// the sync-region headers the decoder launches of d's path use (both null for the per-step path); returns
// how many (0 or 2) -- the caller harvests their failure words after the call (handoff.h)
int attn_sync_regions(const AttnDims& d, void* saved, void* scratch, void** fwd, void** bwd);
const float* attn_saved_mlp_input(const AttnDims& d, const void* saved);
const float* attn_saved_mono_ind(const AttnDims& d, const void* saved);
const float* attn_saved_ws(const AttnDims& d, const void* saved);  // ws_t rows (B, T, Sc)
const float* attn_saved_vh(const AttnDims& d, const void* saved);  // Vh (B, L, Sc)
const float* attn_saved_dropout_mask(const AttnDims& d, const void* saved);

// Attention:BeamSearch (Attention.lua:332-438) for B utterances: h (B, L, A); labels 0-based; out
// (B, ldo >= maxlen + 1) best hypothesis per utterance (tokens, -1 padded), out_len, out_score (its
// summed log-probability).  Synchronises the stream (stops when every utterance has K finished).
size_t attn_beam_workspace_bytes(const AttnDims& d, int K, int maxlen);
int attn_beam_search(hipStream_t st, const AttnDims& d, const float* h, const AttnParams& P, int eos, int K,
                     int maxlen, int* out, int ldo, int* out_len, float* out_score, void* ws, size_t ws_bytes);
// the same search in stages (an external decoder_mlp runs between step and advance on beam_mlp_input's
// (B*K, S+A) rows and hands back (B*K, O) log-probabilities)
int attn_beam_init(hipStream_t st, const AttnDims& d, const float* h, const AttnParams& P, int eos, int K, int maxlen,
                   void* ws, size_t ws_bytes);
int attn_beam_step(hipStream_t st, const AttnDims& d, const AttnParams& P, int K, int maxlen, int count, void* ws,
                   size_t ws_bytes);
const float* attn_beam_mlp_input(const AttnDims& d, int K, int maxlen, void* ws);
int attn_beam_advance(hipStream_t st, const AttnDims& d, int eos, int K, int maxlen, int count, const float* logp_ext,
                      void* ws, size_t ws_bytes);
int attn_beam_done(hipStream_t st, const AttnDims& d, int K, int maxlen, void* ws, int* all_done);
int attn_beam_finish(hipStream_t st, const AttnDims& d, int K, int maxlen, void* ws, int* out, int ldo, int* out_len,
                     float* out_score);
// WagnerFischer (utils.lua:3-27) over n sequence pairs (row-major, lengths alen / blen)
int edit_distance(hipStream_t st, int n, const int* a, const int* alen, int lda, const int* b, const int* blen,
                  int ldb, int* out);

// -log p of the labels and the reference's seed dlogp = -labelmask (timit/timit.lua:262-282).
// tlen (B, or null): labels per utterance -- steps t >= T_b get dlogp = 0 and no nll term (normalize: / T_b)
int nll_seed(hipStream_t st, int B, int T, int O, const float* logp, const int* labels, int normalize, float* nll,
             float* dlogp, const int* tlen = nullptr);

}  // namespace s2s
