/* libs2s_hip.so -- MI355X (gfx950) drop-in for the hot path of
 * Ajay-Wong/seq2seq-attention-asr: the attention-seq2seq training step, forward + backward.
 *
 * C ABI only: plain pointers, sizes and an opaque HIP stream; no torch types.  It is what
 * a LuaJIT `ffi.cdef` shim binds in place of the Torch7 nn.Module methods it replaces
 * (see INTEGRATION.md), and what the Python ctypes host layer (seq2seq-attention-asr_amd/s2s_amd)
 * binds in this repo's tests and bench.
 *
 * Conventions:
 *   - every buffer is a caller-owned DEVICE pointer, fp32 unless stated, row-major;
 *   - the batch axis is leading: x (B, L, F), h (B, L, A), labels (B, T) int32, 0-based class ids;
 *     utterances share the padded length L (and T); variable-length batches pass per-utterance
 *     lengths (device int32 arrays of B, 1 <= L_b <= L, 1 <= T_b <= T; NULL = all full length) and
 *     get exactly the reference's per-utterance results (timit/timit.lua:239-295 forwards each
 *     utterance alone): padding frames / labels contribute nothing;
 *   - weight layouts are the reference's: W (out, in) row-major (LinearZeroBias.lua:8,
 *     nn.Linear, TemporalConvolution (out, in*kW));
 *   - gradients ACCUMULATE (dW += scale * ...), as Torch's accGradParameters; zero them
 *     yourself (zeroGradParameters) or pass S2S_ZERO_GRADS to the model step;
 *   - calls return 0 on success, nonzero on error, never abort; s2s_last_error() has the text;
 *   - the persistent (whole-sequence) launches hand data between workgroups with bounded waits: a wait
 *     that times out makes the launch give up and sets the context's failure status (host-visible, no
 *     device sync needed); every later compute call of that context then returns nonzero until
 *     s2s_ctx_status(..., clear = 1) has reported it (RNN.lua:8-9 / Attention.lua:316 error() semantics);
 *   - `stream` is a hipStream_t (NULL = legacy default stream); calls are asynchronous on it
 *     and allocate nothing (scratch/saved buffers come from the caller, sized by the *_bytes
 *     queries);
 *   - one context per process/GPU; a context is not thread-safe.
 */
#ifndef S2S_HIP_H_
#define S2S_HIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct s2s_ctx s2s_ctx;
typedef void* s2s_stream_t; /* hipStream_t */

/* ---------------------------------------------------------------- context */
int s2s_version(void);
const char* s2s_last_error(void);
int s2s_ctx_create(int device, s2s_ctx** out);
void s2s_ctx_destroy(s2s_ctx* ctx);
/* flags: S2S_CTX_GRAPH = capture the model step into a hipGraph and replay it when the
 * dims / pointers repeat (the step is ~2000 dependent launches). */
#define S2S_CTX_GRAPH 1
/* S2S_CTX_OVERLAP = run the weight-gradient GEMMs on a side stream beside the next layer's BPTT;
 * the persistent GRU workgroups then reserve their CU (unused dynamic LDS) so GEMM workgroups
 * only fill the idle CUs (config-2 step 7.39 vs 7.61 ms on MI355X; bitwise-equal results). */
#define S2S_CTX_OVERLAP 2
int s2s_ctx_set_flags(s2s_ctx* ctx, int flags);
/* S2S_CTX_GRAPH keeps one captured step per (dims, buffer pointers, scale, flags, stream) key, up to
 * `capacity` (default 8, least recently used evicted; an evicted graph's streams are drained before
 * it is destroyed).  The in-kernel dropout seed is not part of the key (it is read from a device word
 * the host writes before each replay).  Stats: graphs captured, replays launched, graphs cached. */
int s2s_ctx_set_graph_cache(s2s_ctx* ctx, int capacity);
/* Operand precision of the hoisted GEMMs of the context's calls (the recurrences stay fp32):
 *   S2S_PREC_FP32 (default): exact f32 MFMA (v_mfma_f32_32x32x2_f32) everywhere;
 *   S2S_PREC_BF16_GEMM: the forward and data-gradient GEMMs (front-end convolutions, x-projections, Vh,
 *     decoder MLP, dX / dh) round their operands to bf16 when staged (v_mfma_f32_16x16x32_bf16, fp32
 *     accumulation and output, fp32 master weights / activations in HBM); weight gradients and the
 *     decoder's weight folds stay fp32 (cancelling sums: BASELINE configs 3 and 5);
 *   S2S_PREC_BF16_ALL: the weight-gradient GEMMs in bf16 too. */
#define S2S_PREC_FP32 0
#define S2S_PREC_BF16_GEMM 1
#define S2S_PREC_BF16_ALL 2
int s2s_ctx_set_precision(s2s_ctx* ctx, int precision);
/* Parameter gradients beside the input gradients (Torch's backward = updateGradInput + accGradParameters, the
 * second made asynchronous).  With on = 1, s2s_attn_bwd, s2s_lstm_bwd and s2s_tconv_bwd issue their weight / bias
 * gradient work on a stream of the context's own (s2s_ctx_side_stream; not the model step's side stream), forked
 * from the call's stream once its inputs are final, and order only the input gradient on the call's stream, so the
 * next module's backward overlaps them.  Until s2s_ctx_join_wgrad(ctx, stream) the parameter gradients are not final
 * on `stream`, and the buffers those calls read (x, y, dy, saved, scratch) must stay untouched (a caller's allocator
 * records their uses on s2s_ctx_side_stream).  Captured inside a hipGraph the fork / join become graph edges. */
int s2s_ctx_set_wgrad_overlap(s2s_ctx* ctx, int on);
int s2s_ctx_join_wgrad(s2s_ctx* ctx, s2s_stream_t stream);
s2s_stream_t s2s_ctx_side_stream(s2s_ctx* ctx);
int s2s_ctx_graph_stats(s2s_ctx* ctx, long* captures, long* replays, int* cached);
/* Failure status of the context's persistent launches, after synchronising `stream` (and the context's
 * side stream): 0, or a bitwise OR of
 *   S2S_STATUS_HANDOFF_TIMEOUT: a hand-off wait of a persistent launch exceeded its spin limit -- that
 *     launch's outputs / gradients (and everything computed from them) are invalid;
 *   S2S_STATUS_ABORTED_REGION: a persistent launch found its sync region already aborted and returned at
 *     once (a preparing launch failed, or the s2s_debug_inject_abort test knob).
 * clear = 1 resets it (compute calls fail while it is nonzero). */
#define S2S_STATUS_HANDOFF_TIMEOUT 1
#define S2S_STATUS_ABORTED_REGION 2
int s2s_ctx_status(s2s_ctx* ctx, s2s_stream_t stream, int* status, int clear);

/* ---------------------------------------------------------------- GRU layer
 * nn.RNN(nn.GRU(D, H), reverse)  (RNN.lua:120-201, GRU.lua:16-51, Recurrent.lua:104-151).
 * ndir = 1: one nn.RNN.  ndir = 2: the two directions of a bidirectional encoder layer that read
 * the same x (timit/model_chorowski_baseline.lua:22-32) in the same launches; W[d*3 + g] is
 * direction d's gate g in (z, r, h) order, each (H, H+D) with columns [h | x] (GRU.lua:22).
 * y[d] rows: y[d][(b*L + t)*ldy + j]; ldy = 2H with y[1] = y[0] + H reproduces JoinTable(2,2).
 * saved[d]: s2s_gru_saved_bytes(B, L, H) each, written by fwd and read by bwd.
 * lengths: (B) frames per utterance or NULL.  With lengths the recurrence is h_t = m_t GRU(h_{t-1}, x_t),
 * m_t = 1[t < L_b]: y = 0 on padding frames, the reverse direction starts at the utterance's own last
 * frame, and the backward treats dL/dh_t = 0 there (pass the same lengths to fwd and bwd). */
size_t s2s_gru_saved_bytes(int B, int L, int H);
size_t s2s_gru_scratch_bytes(int ndir, int B, int L, int D, int H);
int s2s_gru_fwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, const int* reverse,
                const float* x, long ldx, const float* const* W, float* const* y, long ldy, void* const* saved,
                const int* lengths, void* scratch, size_t scratch_bytes);
/* dy[d] rows with stride lddy; dx (may be NULL) = sum over directions, overwritten unless
 * dx_accumulate; dW[d*3+g] += scale * ...  (LinearZeroBias.lua:50-74)                      */
int s2s_gru_bwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, const int* reverse,
                const float* x, long ldx, const float* const* W, void* const* saved, const float* const* dy,
                long lddy, float* dx, long lddx, int dx_accumulate, float* const* dW, float scale,
                const int* lengths, void* scratch, size_t scratch_bytes);

/* ---------------------------------------------------------------- LSTM layer
 * nn.RNN(nn.LSTM(D, H, peepholes), reverse) for ndir directions -- LSTM.lua:6-136 (gates i, f, g, o,
 * each Linear(D,H)(x) + Linear(H,H)(h) with biases; peepholes add full Linear(H,H)(c) terms, the o
 * gate peeking the new cell) under RNN.lua:120-201.  Replaces the per-step clone graph the
 * reference runs for the conv+BiLSTM encoder (timit/timit.lua:108-125).
 * W[d*NP + p], NP = 16 (22 with peepholes), W = (out, in):
 *   for q in (i, f, g, o): Wqx (H, D), bqx (H), Wqh (H, H), bqh (H)
 *   peepholes:             Wic (H, H), bic (H), Wfc (H, H), bfc (H), Woc (H, H), boc (H)
 * y / saved / dy / dx / dW conventions as the GRU calls; dW and the bias grads accumulate.
 * lengths: (B) frames per utterance or NULL, as for the GRU calls: h_t = c_t = 0 on padding frames t >= L_b
 * (y = 0 there, the reverse direction starts from zero state at the utterance's own last frame), and the
 * backward treats dL/dh_t = dL/dc_t = 0 there (pass the same lengths to fwd and bwd). */
size_t s2s_lstm_saved_bytes(int B, int L, int H);
size_t s2s_lstm_scratch_bytes(int ndir, int B, int L, int D, int H, int peepholes);
int s2s_lstm_fwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, int peepholes,
                 const int* reverse, const float* x, long ldx, const float* const* W, float* const* y, long ldy,
                 void* const* saved, const int* lengths, void* scratch, size_t scratch_bytes);
int s2s_lstm_bwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, int peepholes,
                 const int* reverse, const float* x, long ldx, const float* const* W, void* const* saved,
                 const float* const* dy, long lddy, float* dx, long lddx, int dx_accumulate, float* const* dW,
                 float scale, const int* lengths, void* scratch, size_t scratch_bytes);

/* ---------------------------------------------------------------- attention decoder
 * nn.Attention(decoder_recurrent = GRU(S,S), decoder_mlp = Maxout(S+A, M, K) -> Linear(M, O)
 * -> LogSoftMax, scoreDepth Sc, hybrid features (optional), stateDepth S, annotationDepth A, outputDepth O,
 * monoAlignPenalty true, penaltyLambda) -- Attention.lua:15-211, RNNAttention.lua:144-253,
 * MonotonicAlignment.lua, Maxout.lua, timit/model_chorowski_baseline.lua:37-70.
 * Parameter pointers, in this order (W = (out, in)):
 *   0 V (Sc, A)  [Vh TCZB]     1 Ws (Sc, S)  2 bs (Sc)   [TemporalConvolution(1, Sc, S)]
 *   3 we (1, Sc) [e TCZB]      4 Wy (S, O)   5 by (S)    6 Wc (S, A)   7 bc (S)
 *   8 Wd (S, 2S) 9 bd (S)     10 Wz (S, 2S) 11 Wr (S, 2S) 12 Wh (S, 2S)   [decoder GRU]
 *  13 Wm (M*K, S+A) 14 bm (M*K)   15 Wo (O, M) 16 bo (O)
 * and with hybrid attention (hybridAttendFeatureMaps nF > 0, Attention.lua:75-98):
 *  17 hybW (nF, kW) 18 hybb (nF)  [TemporalConvolution(1, nF, kW) on the padded alpha_{t-1}]
 *  19 hybU (Sc, nF)               [UF = TCZB(nF, Sc, 1)]                                        */
#define S2S_ATTN_NPARAMS 17
#define S2S_ATTN_NPARAMS_HYBRID 20
/* dropout: nn.Dropout(p) in front of the Maxout of the decoder MLP (timit/model_chorowski_baseline_
 * dropout.lua:56), Torch7 semantics in training mode: [s_t; c_t] * mask, mask = Bernoulli(1-p)/(1-p).
 * p = 0: no dropout.  dropout_mask: optional (B, T, S+A) multipliers (scaling included) used as given
 * (parity with an external RNG); NULL: drawn in-kernel from dropout_seed (counter-based, so a seed
 * reproduces the masks for any launch geometry).  The masks stay in `saved` for the backward. */
typedef struct {
  int B, L, T;
  int annotationDepth, scoreDepth, stateDepth, outputDepth, mlpDepth, maxoutWindow;
  float penalty;
  float dropout;
  unsigned long long dropout_seed;
  const float* dropout_mask;
  /* hybrid location-aware attention: Attention(..., hybridAttendFilterSize kW, hybridAttendFeatureMaps
   * nF, ...); nF = 0 is the content-only baseline (model_chorowski_baseline.lua:39-40); nF > 0 needs
   * 1 <= kW <= 8 and runs the per-step decoder kernels */
  int hybridAttendFilterSize, hybridAttendFeatureMaps;
  /* external_mlp = 1: a decoder_mlp other than Maxout -> Linear -> LogSoftMax (e.g. the two-Maxout MLP of
   * librispeech/model_vgg.lua:71-77) runs on the caller's side: s2s_attn_fwd stops at the MLP input
   * [s_t; c_t] (s2s_attn_mlp_input; logp may be NULL), s2s_attn_bwd takes d[s_t; c_t] (B, T, S+A) in place of
   * dlogp, and params / grads 13-16 (Wm, bm, Wo, bo) are unused (may be NULL).  Needs dropout == 0. */
  int external_mlp;
  /* decoder_lstm = 1: decoder_recurrent = nn.LSTM(S, S) without peepholes (the conv + BiLSTM model,
   * timit/timit.lua:137: s_t = h_t, the carried mem = the cell) instead of nn.GRU(S, S); per-step decoder
   * kernels.  Params 10-12 are then unused (may be NULL) and params 20-35 are the LSTM's, for q in (i, f, g, o):
   * Wqx (S, S), bqx (S), Wqh (S, S), bqh (S) (LSTM.lua:25-29); 17-19 stay the hybrid ones (NULL when nF = 0). */
  int decoder_lstm;
  /* variable-length batch (device int32 (B) arrays, or NULL): frames per utterance of h (softmax and
   * MonotonicAlignment over its own L_b frames; alpha = 0 past them) and labels per utterance (no
   * MonotonicAlignment gradient at steps >= T_b; the caller's dlogp must be 0 there, s2s_nll_seed does it) */
  const int* frame_lengths;
  const int* label_lengths;
} s2s_attn_dims;
#define S2S_ATTN_NPARAMS_LSTM 36
size_t s2s_attn_saved_bytes(const s2s_attn_dims* d);
size_t s2s_attn_scratch_bytes(const s2s_attn_dims* d);
/* Attention:updateOutput (Attention.lua:305-322): h (B, L, A), labels (B, T) -> logp (B, T, O) */
int s2s_attn_fwd(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const int* labels,
                 const float* const* params, float* logp, void* saved, void* scratch, size_t scratch_bytes);
/* Attention:updateGradInput (Attention.lua:324-327) + accGradParameters: dlogp (B, T, O) -> dh (B, L, A) */
int s2s_attn_bwd(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const int* labels,
                 const float* const* params, const void* saved, const float* dlogp, float* dh, int dh_accumulate,
                 float* const* grads, float scale, void* scratch, size_t scratch_bytes);
/* the decoder_mlp input rows [s_t; c_t] (B, T, S+A) of the last forward inside `saved` (RNNAttention.lua:165) */
const float* s2s_attn_mlp_input(const s2s_attn_dims* d, const void* saved);
/* decoder:alpha() (Attention.lua:241-243): device pointer to alpha (B, T, L) inside `saved` */
const float* s2s_attn_alpha(const s2s_attn_dims* d, const void* saved);
/* decoder:Ws() (Attention.lua:247-249, timit/timit.lua:520): the 'Ws' node is ExpandAs(ws_t, Vh), i.e. the
 * rows ws_t = W_s s_{t-1} + b_s broadcast over the L frames.  Device pointer to the (B, T, Sc) rows ws_t
 * inside `saved`; the (B, T, L, Sc) tensor the reference returns is their expansion over L (a view). */
const float* s2s_attn_ws(const s2s_attn_dims* d, const void* saved);
/* decoder.Vh.output (Attention.lua:43-47, timit/timit.lua:521): Vh = h V^T, (B, L, Sc) inside `saved`.
 * decoder:penalty() (Attention.lua:244-246) returns the output of the node named 'penalty', which is
 * MonotonicAlignment's output = alpha (MonotonicAlignment.lua:40): s2s_attn_alpha serves both. */
const float* s2s_attn_vh(const s2s_attn_dims* d, const void* saved);
/* (B, T) MonotonicAlignment indicators 1[penalty_t > 0] of the last forward (MonotonicAlignment.lua:
 * 27-39): the discrete decision behind the penalty gradient (MonotonicAlignment.lua:44-77). */
const float* s2s_attn_mono_ind(const s2s_attn_dims* d, const void* saved);
/* (B, T, S+A) dropout multipliers of the last forward inside `saved` (NULL when dropout == 0) */
const float* s2s_attn_dropout_mask(const s2s_attn_dims* d, const void* saved);
/* (B, T, mlpDepth) int32 Maxout decisions of the last forward inside `saved`: which unit i < maxoutWindow of
 * group j won (first maximum, TemporalMaxPooling; Maxout.lua:14-18) -- the discrete decision the backward
 * routes each gradient row by (the fused Chorowski decoder_mlp only) */
const int* s2s_attn_maxout_argmax(const s2s_attn_dims* d, const void* saved);

/* decoder:BeamSearch(annotations, eos, K, maxseqlength) (Attention.lua:332-438; timit/timit.lua:401) for
 * B utterances at once, in evaluate() mode: h (B, L, A); eos and the output tokens 0-based; out (B, ldo),
 * ldo >= maxseqlength + 1, the best finished hypothesis of each utterance padded with -1; out_len (B);
 * out_score (B, may be NULL) its summed log-probability.  Hypotheses finish on eos or at maxseqlength;
 * K in [1, 16].  Blocks until done (it polls for the end of the search).  Content or hybrid attention
 * (alpha_{t-1} carried per hypothesis), GRU or LSTM decoder_recurrent (the cell carried: the reference's
 * hidden {alpha, s, mem}, Attention.lua:360-403), fused decoder_mlp; frame_lengths must be NULL. */
size_t s2s_attn_beam_workspace_bytes(const s2s_attn_dims* d, int K, int maxseqlength);
int s2s_attn_beam_search(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h,
                         const float* const* params, int eos, int K, int maxseqlength, int* out, int ldo, int* out_len,
                         float* out_score, void* workspace, size_t workspace_bytes);
/* The same search in stages, for an external decoder_mlp (external_mlp = 1; also usable with the fused one):
 *   s2s_attn_beam_init;  for count = 0 .. maxseqlength: s2s_attn_beam_step(count) -> [run the decoder_mlp on
 *   the (B*K, S+A) rows at s2s_attn_beam_mlp_input -> (B*K, O) log-probabilities] -> s2s_attn_beam_advance(count,
 *   logp; NULL with the fused decoder_mlp) -> stop once s2s_attn_beam_done reports 1;  s2s_attn_beam_finish.
 * Rows are hypothesis r = b*K + j (inactive ones are computed and ignored).  The workspace holds all state. */
int s2s_attn_beam_init(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h,
                       const float* const* params, int eos, int K, int maxseqlength, void* workspace,
                       size_t workspace_bytes);
int s2s_attn_beam_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* const* params, int K,
                       int maxseqlength, int count, void* workspace, size_t workspace_bytes);
const float* s2s_attn_beam_mlp_input(const s2s_attn_dims* d, int K, int maxseqlength, void* workspace);
int s2s_attn_beam_advance(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int eos, int K,
                          int maxseqlength, int count, const float* logp, void* workspace, size_t workspace_bytes);
int s2s_attn_beam_done(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int K, int maxseqlength,
                       void* workspace, int* all_done);
int s2s_attn_beam_finish(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int K, int maxseqlength,
                         int* out, int ldo, int* out_len, float* out_score, void* workspace);
/* WagnerFischer(a, b) (utils.lua:3-27) for n pairs on the device: a (n, lda) with lengths alen, b (n, ldb)
 * with blen, out (n) the edit distances (PER/CER numerators, timit/timit.lua:396-410). */
int s2s_edit_distance(s2s_ctx* ctx, s2s_stream_t stream, int n, const int* a, const int* alen, int lda, const int* b,
                      const int* blen, int ldb, int* out);

/* ---------------------------------------------------------------- encoder front-ends
 * The operators of the reference's two other encoders: the conv + BiLSTM encoder of timit/timit.lua:108-125
 * (3 x [TemporalConvolution(D, 256, 3) -> ReLU -> TemporalMaxPooling(2, 2)] -> BiLSTM, s2s_lstm_*) and the VGG
 * stack of librispeech/model_vgg.lua:23-51.  Torch7 semantics and layouts; `relu` = 1 fuses the nn.ReLU that
 * follows the convolution in both encoders (its backward then needs the conv's output y).  Batches of
 * equal-length utterances, batch axis leading.  Gradients accumulate (dW += scale * ...); dx is overwritten
 * unless dx_accumulate; any gradient pointer may be NULL (not computed).
 *
 * nn.TemporalConvolution(Din, Dout, kW) (dW = 1): x (B, L, Din) -> y (B, L - kW + 1, Dout); weight (Dout, kW*Din),
 * bias (Dout) or NULL (TemporalConvolutionZeroBias, TemporalConvolutionZeroBias.lua:37-54). */
size_t s2s_tconv_scratch_bytes(int B, int L, int Din, int Dout, int kW);
int s2s_tconv_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x,
                  const float* W, const float* b, float* y);
int s2s_tconv_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x,
                  const float* W, const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db,
                  float scale, void* scratch, size_t scratch_bytes);
/* nn.TemporalMaxPooling(kW, dW): x (B, L, D) -> y (B, (L - kW)/dW + 1, D); idx (same shape as y, int32) = argmax
 * offset within the window, first maximum wins; the backward overwrites dx (B, L, D). */
int s2s_tmaxpool_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int D, int kW, int dW, const float* x, float* y,
                     int* idx);
int s2s_tmaxpool_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int D, int kW, int dW, const int* idx,
                     const float* dy, float* dx);
/* nn.SpatialConvolutionMM(Cin, Cout, kW, kH) (stride 1, no padding): x (B, Cin, H, W) -> y (B, Cout, H-kH+1, W-kW+1);
 * weight (Cout, Cin*kH*kW) in (c, i, j) order, bias (Cout) or NULL.  Scratch holds the im2col panel of x:
 * col_from_fwd = 1 lets the backward reuse the panel the forward left in the SAME scratch (same x, scratch
 * untouched in between) instead of rebuilding it. */
size_t s2s_sconv_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW);
int s2s_sconv_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu,
                  const float* x, const float* weight, const float* bias, float* y, void* scratch,
                  size_t scratch_bytes);
int s2s_sconv_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu,
                  const float* x, const float* weight, const float* y, const float* dy, float* dx, int dx_accumulate,
                  float* dweight, float* dbias, float scale, void* scratch, size_t scratch_bytes,
                  int col_from_fwd);
/* nn.SpatialMaxPooling(kW, kH, dW, dH) (floor mode): x (B, C, H, W) -> y (B, C, (H-kH)/dH+1, (W-kW)/dW+1);
 * idx = i*kW + j of the window's first maximum. */
int s2s_smaxpool_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH,
                     const float* x, float* y, int* idx);
int s2s_smaxpool_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH,
                     const int* idx, const float* dy, float* dx);
/* nn.Transpose2({1,2},3) on a batch (Transpose2.lua:23-37): (B, D1, D2, D3) -> (B, D2, D1, D3); the
 * backward is the same call with D1 and D2 exchanged.  nn.ReLU: y = max(x, 0), dx = dy * 1[x > 0]. */
int s2s_swap12(s2s_ctx* ctx, s2s_stream_t stream, int B, int D1, int D2, int D3, const float* x, float* y);
int s2s_relu_fwd(s2s_ctx* ctx, s2s_stream_t stream, long n, const float* x, float* y);
int s2s_relu_bwd(s2s_ctx* ctx, s2s_stream_t stream, long n, const float* x, const float* dy, float* dx);
/* nn.LogSoftMax over `rows` rows of n (the output layer of an external decoder_mlp): forward and
 * dx = dy - exp(y) * sum(dy). */
int s2s_logsoftmax_fwd(s2s_ctx* ctx, s2s_stream_t stream, long rows, int n, const float* x, float* y);
int s2s_logsoftmax_bwd(s2s_ctx* ctx, s2s_stream_t stream, long rows, int n, const float* y, const float* dy,
                       float* dx);
/* ---------------------------------------------------------------- loss seed
 * timit/timit.lua:262-282: nll[b] = -sum(labelmask * logp) (/T if normalize);
 * dlogp = -labelmask (never normalised: opt.normalizeGrad is false in every config).
 * label_lengths (B) or NULL: only steps t < T_b count (normalize: / T_b); dlogp = 0 past them. */
int s2s_nll_seed(s2s_ctx* ctx, s2s_stream_t stream, int B, int T, int O, const float* logp, const int* labels,
                 const int* label_lengths, int normalize, float* nll, float* dlogp);

/* ---------------------------------------------------------------- whole training step
 * autoencoder:forward({X, labelmask}); nll; autoencoder:backward({X, labelmask}, -labelmask)
 * for a batch of B equal-length utterances (timit/timit.lua:240-295), flat parameter and
 * gradient buffers (timit.lua:172 getParameters).  Flat layout: see s2s_model_param_offset
 * and DESIGN.md.                                                                             */
typedef struct {
  int B, L, T;
  int inputFrameSize, hiddenFrameSize, outputFrameSize, numLayers;
  int scoreDepth, stateDepth, outputDepth, mlpDepth, maxoutWindow;
  float penalty;
  float dropout;                   /* as in s2s_attn_dims (model_chorowski_baseline_dropout.lua) */
  unsigned long long dropout_seed;
  const float* dropout_mask;
  /* variable-length minibatch (device int32 (B) arrays, or NULL = all L / T): the step then equals the
   * reference's per-utterance loop over utterances of L_b frames and T_b labels (timit/timit.lua:239-295):
   * masked encoder recurrences (s2s_gru_*), masked attention (s2s_attn_dims), masked loss seed.  The
   * arrays are read on the device at run time: a captured step replays with new lengths in place. */
  const int* frame_lengths;
  const int* label_lengths;
} s2s_model_dims;
#define S2S_ZERO_GRADS 1
#define S2S_NORMALIZE_NLL 2
/* S2S_BUCKET_EVENTS: the step records one ctx-owned event per gradient bucket at the point where
 * that bucket's gradients are final (also inside a captured hipGraph, as external event nodes), so
 * a data-parallel caller can start each bucket's all-reduce while the encoder BPTT of the layers
 * below is still running: s2s_stream_wait_bucket(ctx, comm_stream, i) then the
 * collective on comm_stream.  Buckets in completion order: 0 = the decoder's parameters, then
 * encoder layers numLayers .. 1 (s2s_model_bucket gives each one's slice of the flat buffer). */
#define S2S_BUCKET_EVENTS 4
int s2s_model_bucket_count(const s2s_model_dims* d);
int s2s_model_bucket(const s2s_model_dims* d, int i, size_t* offset, size_t* count);
int s2s_stream_wait_bucket(s2s_ctx* ctx, s2s_stream_t stream, int i);
size_t s2s_model_param_count(const s2s_model_dims* d);
/* offset (in floats) of parameter #i of the flat layout and its element count; -1 past the end */
long s2s_model_param_offset(const s2s_model_dims* d, int i, long* numel);
size_t s2s_model_workspace_bytes(const s2s_model_dims* d);
/* grads (+)= scale * dL/dparams; logp (B, T, O) and nll (B) are outputs (may be NULL). */
int s2s_model_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_model_dims* d, const float* params, float* grads,
                   const float* x, const int* labels, float scale, int flags, float* logp, float* nll,
                   void* workspace, size_t workspace_bytes);
/* encoder output (the annotations h, B x L x 2*outputFrameSize) of the last step, inside workspace
 * (encoder.output, timit/timit.lua:397). */
const float* s2s_model_encoder_output(const s2s_model_dims* d, const void* workspace);
/* the model step's decoder: its s2s_attn_dims and its `saved` buffer inside workspace, for the
 * decoder accessors above after a step (decoder:alpha(), Ws(), Vh.output, penalty(): timit/timit.lua:
 * 519-521, 534-536) and s2s_attn_dropout_mask. */
int s2s_model_attn_dims(const s2s_model_dims* d, s2s_attn_dims* out);
const void* s2s_model_attn_saved(const s2s_model_dims* d, const void* workspace);

/* ---------------------------------------------------------------- optimizer step
 * After the (all-reduced) backward, timit/timit.lua:292-347 on the flat buffers, fused on the device:
 * clip the global gradient norm to maxnorm (:297-302), g += weightDecay * x (:305-308), optim.adadelta
 * (rho, eps; timit.lua:179, exp_logmel7_chorowski_normNLL_colnorm.lua:32-33), then -- colnorm_max > 0 --
 * TrainUtils.columnNormConstraint(colnorm_max) on every weight matrix (TrainUtils.lua:52-104, applied
 * to the graph at timit.lua:344-346): rows with ||W_r|| + 1e-8 >= max are divided by that / max.
 * `gradients` is left clipped / decayed in place as the reference leaves it.  state: the optimizer's
 * paramVariance / accDelta (s2s_optim_state_bytes, zero it with s2s_optim_reset).  mats: n_mats
 * (offset, rows, cols) weight matrices of the flat buffer (s2s_model_weight_matrices for the model).
 * gradnorm (device float, may be NULL) receives ||g|| before clipping (timit.lua:297 gradnorms).
 * gradnoise_eta != 0 adds the trainer's gradient noise after the L2 term (timit.lua:310-315, gradnoise =
 * {eta, gamma, t}, :185-189): t += 1 (the counter lives in `state`, 0 after s2s_optim_reset), sigma =
 * sqrt(eta / (1 + t)^gamma), g += sigma * N(0, 1); the normals are a counter-based function of
 * (gradnoise_seed, t, element), identical on every data-parallel rank for the same seed. */
typedef struct {
  float rho, eps, maxnorm, weightDecay, colnorm_max;
  float gradnoise_eta, gradnoise_gamma;
  unsigned long long gradnoise_seed;
} s2s_optim_config;
size_t s2s_optim_state_bytes(size_t n);
int s2s_optim_reset(s2s_ctx* ctx, s2s_stream_t stream, void* state, size_t n);
/* set the state's gradient-noise counter to gradnoise.t (a resumed trainer's checkpointed table,
 * timit/timit.lua:92,312): the next step draws with t + 1 */
int s2s_optim_set_noise_step(s2s_ctx* ctx, s2s_stream_t stream, void* state, size_t n, unsigned t);
/* If the context's failure status (s2s_ctx_status) is set when the update RUNS -- a persistent launch of an
 * earlier step on this stream timed out, its gradients are invalid -- the update is skipped on the device
 * (params, state and the noise counter untouched; *gradnorm is still written).  This covers calls already
 * queued in program order behind the failed step; calls made after the host has seen it fail outright. */
int s2s_optim_adadelta_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params,
                            float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm);
/* Data parallel: a rank whose persistent launch failed still sends its (invalid) gradients into the all-reduce,
 * so every replica must skip that update, not only the failing one.  s2s_ctx_status_flag writes flag[0] = 1.0f
 * if the context's failure status is set when it runs on `stream` (stream-ordered, no host sync), else 0.0f;
 * all-reduce it (sum or max) across the ranks and pass it as skip_flag: the update is then skipped on every rank
 * when *skip_flag != 0 (or the local status is set).  skip_flag NULL = s2s_optim_adadelta_step. */
int s2s_ctx_status_flag(s2s_ctx* ctx, s2s_stream_t stream, float* flag);
int s2s_optim_adadelta_step_flag(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params,
                                 float* grads, size_t n, void* state, const long* mats, int n_mats,
                                 float* gradnorm, const float* skip_flag);
/* the model's weight matrices (every module weight: encoder W_z/W_r/W_h, V, Ws, we, Wy, Wc, Wd, decoder
 * W_z/W_r/W_h, Wm, Wo) as (offset, rows, cols) triples; returns their count (mats may be NULL) */
int s2s_model_weight_matrices(const s2s_model_dims* d, long* mats);

/* ---------------------------------------------------------------- live kernel timing
 * s2s_prof_enable(1): every subsequent eager (non-captured) launch is bracketed by two
 * hipEvents on its stream and tagged with its kernel family's algorithmic flops/bytes.
 * s2s_prof_collect: synchronises, writes "name\tlaunches\ttotal_us\tflops\tbytes\n" per family. */
int s2s_prof_enable(int on);
int s2s_prof_collect(char* buf, size_t cap);

/* ---------------------------------------------------------------- data parallel (RCCL)
 * One process per GPU.  Rank 0 calls s2s_comm_unique_id, the bytes are shared out of band,
 * every rank calls s2s_comm_init; s2s_allreduce_sum sums a float buffer in place over xGMI. */
#define S2S_UNIQUE_ID_BYTES 128
int s2s_comm_unique_id(void* out_bytes);
int s2s_comm_init(s2s_ctx* ctx, const void* id_bytes, int nranks, int rank);
int s2s_allreduce_sum(s2s_ctx* ctx, s2s_stream_t stream, float* buf, size_t count);

#ifdef __cplusplus
}
#endif
#endif /* S2S_HIP_H_ */
