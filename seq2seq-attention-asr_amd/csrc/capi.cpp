// C-ABI surface of libs2s_hip.so (include/s2s_hip.h): argument checking, the model-level
// training step (encoder -> attention decoder -> NLL seed -> backward), hipGraph capture
// of that step, and RCCL data-parallel gradient sums.
#include "../../include/s2s_hip.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "attn.h"
#include "frontend.h"
#include "gru_persist.h"
#include "handoff.h"
#include "gru.h"
#include "lstm.h"
#include "s2s_common.h"

namespace s2s {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }

// ------------------------------------------------------------ live kernel timing
struct ProfRec {
  const char* name;
  double flops, bytes;
  hipEvent_t a, b;
};
static bool g_prof = false;
static std::vector<ProfRec> g_recs;
static std::vector<hipEvent_t> g_pool;
static std::mutex g_prof_mu;

static hipEvent_t prof_event() {
  if (!g_pool.empty()) {
    hipEvent_t e = g_pool.back();
    g_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}
static bool capturing(hipStream_t st) {
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(st, &cs) != hipSuccess) return true;
  return cs != hipStreamCaptureStatusNone;
}
bool prof_on() { return g_prof; }
void prof_begin(hipStream_t st, const char* name, double flops, double bytes) {
  if (capturing(st)) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  ProfRec r{name, flops, bytes, prof_event(), nullptr};
  if (!r.a) return;
  (void)hipEventRecord(r.a, st);
  g_recs.push_back(r);
}
void prof_end(hipStream_t st) {
  if (capturing(st)) return;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  for (auto it = g_recs.rbegin(); it != g_recs.rend(); ++it)
    if (it->b == nullptr) {
      it->b = prof_event();
      if (it->b) (void)hipEventRecord(it->b, st);
      return;
    }
}

}  // namespace s2s

using namespace s2s;

struct GraphKey {
  s2s_model_dims d;
  const void* ptrs[7];
  float scale;
  int flags;
  int precision;
  void* stream;
  bool operator==(const GraphKey& o) const { return std::memcmp(this, &o, sizeof(GraphKey)) == 0; }
};

constexpr int kMaxBuckets = 17;  // decoder + up to 16 encoder layers

struct CachedGraph {
  GraphKey key;
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
  hipStream_t launched_on = nullptr;  // the stream of its last replay (drained before destroy)
  unsigned long long used = 0;        // LRU clock
};
constexpr int kGraphCacheDefault = 8;

struct s2s_ctx {
  int device = 0;
  int flags = 0;
  int precision = S2S_PREC_FP32;  // S2S_PREC_*: operand precision of the hoisted GEMMs
  hipStream_t side = nullptr;     // weight-gradient GEMMs run here beside the critical path
  hipEvent_t ev[32] = {};  // model step: 0 / 1+l wgrad forks, 13-15 prologue + join, 16-20 decoder (attn_*)
  unsigned long long* seed_dev = nullptr;  // dropout seed word read by this context's replayed graphs
  hipEvent_t bev[kMaxBuckets] = {};  // S2S_BUCKET_EVENTS: gradient bucket i is final
  // s2s_ctx_set_wgrad_overlap: the module-level backward calls fork their parameter gradients onto a stream of their
  // own (wside, event wev) -- not `side`, which the captured model steps' graphs hold
  int wgrad_overlap = 0;
  hipStream_t wside = nullptr;
  hipEvent_t wev = nullptr;
  // captured model steps, one per GraphKey (least recently used evicted past graph_cap): a caller
  // alternating shapes / buffers (a data loader's double buffers, length buckets) replays instead of
  // re-capturing every step
  std::vector<CachedGraph> graphs;
  int graph_cap = kGraphCacheDefault;
  unsigned long long graph_clock = 0;
  long captures = 0, replays = 0;
  ncclComm_t comm = nullptr;
  // failure status of the context's persistent launches (handoff.h: [0] a hand-off wait timed out, [1] a
  // launch started on an aborted region): host-coherent memory the kernels write, so every call can check
  // it without a device sync; s2s_ctx_status reads it after a stream sync and clears it
  unsigned* status_host = nullptr;
  unsigned* status_dev = nullptr;
  s2s::GemmStage lt;  // bf16 operand copies of the big bf16 GEMMs (gemm_bf16.hip), one buffer per stream
};

namespace {

// the stream a module-level backward issues its parameter gradients on: `st`, or the context's side stream forked
// from `st` here when the caller set s2s_ctx_set_wgrad_overlap (joined by s2s_ctx_join_wgrad)
int wgrad_stream(s2s_ctx* ctx, hipStream_t st, hipStream_t* out) {
  *out = st;
  if (!ctx->wgrad_overlap || !ctx->wside || !ctx->wev || ctx->wside == st) return 0;
  S2S_CHECK_HIP(hipEventRecord(ctx->wev, st));
  S2S_CHECK_HIP(hipStreamWaitEvent(ctx->wside, ctx->wev, 0));
  *out = ctx->wside;
  return 0;
}

// every compute entry point starts here: the device, the context's GEMM precision for this call, and the
// context's failure status -- a persistent launch of an earlier call that timed out left wrong results, so
// every later call fails until the caller has seen it (s2s_ctx_status with clear = 1); Torch's error()
int set_device(s2s_ctx* ctx) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  if (ctx->status_host) {
    const unsigned t = __atomic_load_n(ctx->status_host, __ATOMIC_ACQUIRE);
    const unsigned a = __atomic_load_n(ctx->status_host + 1, __ATOMIC_ACQUIRE);
    S2S_REQUIRE(t == 0u && a == 0u,
                std::string("a persistent launch of an earlier call failed (") +
                    (t ? "hand-off wait timed out" : "launch started on an aborted sync region") +
                    "): its outputs and gradients are invalid; s2s_ctx_status(ctx, stream, &st, 1) clears it");
  }
  S2S_CHECK_HIP(hipSetDevice(ctx->device));
  set_gemm_precision(ctx->precision == S2S_PREC_FP32 ? kGemmF32 : kGemmBf16);
  set_wgrad_bf16(ctx->precision == S2S_PREC_BF16_ALL);
  set_gemm_stage(&ctx->lt);
  return 0;
}

AttnDims to_attn(const s2s_attn_dims* d) {
  AttnDims a{d->B, d->L, d->T, d->annotationDepth, d->scoreDepth, d->stateDepth, d->outputDepth, d->mlpDepth,
             d->maxoutWindow, d->penalty, d->dropout, d->dropout_seed, d->dropout_mask};
  a.hk = d->hybridAttendFilterSize;
  a.hf = d->hybridAttendFeatureMaps;
  a.ext = d->external_mlp ? 1 : 0;
  a.lstm = d->decoder_lstm ? 1 : 0;
  a.flen = d->frame_lengths;
  a.tlen = d->label_lengths;
  return a;
}
int attn_nparams(const s2s_attn_dims* d) {
  if (d->decoder_lstm) return S2S_ATTN_NPARAMS_LSTM;
  return d->hybridAttendFeatureMaps > 0 ? S2S_ATTN_NPARAMS_HYBRID : S2S_ATTN_NPARAMS;
}
// parameter slots a call may leave NULL: the fused MLP's with an external decoder_mlp, the GRU's with a
// decoder LSTM, the hybrid ones without hybrid features
bool attn_param_optional(const s2s_attn_dims* d, int i) {
  if (d->external_mlp && i >= 13 && i <= 16) return true;
  if (d->decoder_lstm && i >= 10 && i <= 12) return true;
  if (d->hybridAttendFeatureMaps <= 0 && i >= 17 && i <= 19) return true;
  return false;
}

// ------------------------------------------------------------ model layout
struct LayerDims {
  int D, H;
};
std::vector<LayerDims> enc_layers(const s2s_model_dims* d) {
  std::vector<LayerDims> v;
  int D = d->inputFrameSize;
  for (int l = 1; l <= d->numLayers; ++l) {
    const int H = l == d->numLayers ? d->outputFrameSize : d->hiddenFrameSize;
    v.push_back({D, H});
    D = 2 * H;
  }
  return v;
}
AttnDims model_attn(const s2s_model_dims* d) {
  AttnDims a{d->B, d->L, d->T, 2 * d->outputFrameSize, d->scoreDepth, d->stateDepth, d->outputDepth,
             d->mlpDepth, d->maxoutWindow, d->penalty, d->dropout, d->dropout_seed, d->dropout_mask};
  a.flen = d->frame_lengths;
  a.tlen = d->label_lengths;
  return a;
}
std::vector<long> param_sizes(const s2s_model_dims* d) {
  std::vector<long> s;
  for (auto& ld : enc_layers(d))
    for (int i = 0; i < 6; ++i) s.push_back((long)ld.H * (ld.H + ld.D));
  const long A = 2L * d->outputFrameSize, Sc = d->scoreDepth, S = d->stateDepth, O = d->outputDepth,
             M = d->mlpDepth, Mk = (long)d->mlpDepth * d->maxoutWindow;
  const long dec[S2S_ATTN_NPARAMS] = {Sc * A, Sc * S, Sc, Sc, S * O, S, S * A, S, S * 2 * S, S,
                                      S * 2 * S, S * 2 * S, S * 2 * S, Mk * (S + A), Mk, O * M, O};
  for (long v : dec) s.push_back(v);
  return s;
}

struct ModelWs {
  std::vector<float*> saved;  // 2 per layer
  std::vector<float*> Y;      // per layer output (B, L, 2H)
  std::vector<float*> dA;     // per layer gate gradients (B, L, 6H), read by the side-stream dW GEMMs
  std::vector<float*> pack;   // per layer packed weight layouts (gru_layer_pack)
  void* attn_saved;
  void* attn_scratch;
  size_t attn_scratch_bytes;
  void* scratch;
  size_t scratch_bytes;
  float *dlogp, *nll, *logp, *dY0, *dY1;
  GemmWs gws_side;  // split-K slabs of the encoder weight-gradient GEMMs (may run on the side stream)
  float* wpart;     // the first layer's in-launch weight gradients: utterance tiles' partials (S2S_BPTT_WGRAD)
  char* gsync[2];   // the persistent GRU launches' sync regions, alternating (gru_layer_preps_next)
  float* xpad;      // (B*L, Dp) zero-padded copy of the input when inputFrameSize % 32 != 0, else null
  int Dp;
  size_t total;
};
ModelWs model_ws(const s2s_model_dims* d, void* base) {
  ModelWs w{};
  Bump bp{static_cast<char*>(base), 0, 0};
  const long B = d->B, L = d->L, T = d->T, O = d->outputDepth;
  size_t scr = 0;
  long hmax = 0;
  for (auto& ld : enc_layers(d)) {
    w.saved.push_back(bp.take<float>(B * L * 5 * ld.H));
    w.saved.push_back(bp.take<float>(B * L * 5 * ld.H));
    w.Y.push_back(bp.take<float>(B * L * 2 * ld.H));
    w.dA.push_back(bp.take<float>(B * L * 6 * ld.H));
    w.pack.push_back(bp.take<float>(gru_layer_pack_bytes(2, ld.D, ld.H) / sizeof(float)));
    size_t s = gru_layer_scratch_bytes(2, d->B, d->L, ld.D, ld.H);
    scr = s > scr ? s : scr;
    hmax = ld.H > hmax ? ld.H : hmax;
  }
  const AttnDims ad = model_attn(d);
  w.attn_saved = bp.take<char>(attn_saved_bytes(ad));
  w.attn_scratch_bytes = attn_scratch_bytes(ad);
  w.attn_scratch = bp.take<char>(w.attn_scratch_bytes);
  w.scratch = bp.take<char>(scr);
  w.scratch_bytes = scr;
  w.dlogp = bp.take<float>(B * T * O);
  w.nll = bp.take<float>(B);
  w.logp = bp.take<float>(B * T * O);
  w.dY0 = bp.take<float>(B * L * 2 * hmax);
  w.dY1 = bp.take<float>(B * L * 2 * hmax);
  w.gws_side = GemmWs{bp.take<float>(kGemmWsFloats), kGemmWsFloats};
  {
    const LayerDims l0 = enc_layers(d)[0];
    GruLayerIO io{};
    io.ndir = 2; io.B = d->B; io.L = d->L; io.D = l0.D; io.H = l0.H;
    const size_t n = gru_layer_wgrad_part_floats(io);
    w.wpart = n ? bp.take<float>(n) : nullptr;
  }
  {
    size_t sb = 0;
    for (auto& ld : enc_layers(d)) sb = std::max(sb, gru_persist_sync_bytes(d->B, d->L, ld.H));
    w.gsync[0] = bp.take<char>(sb);
    w.gsync[1] = bp.take<char>(sb);
  }
  w.Dp = (d->inputFrameSize + 31) / 32 * 32;
  w.xpad = d->inputFrameSize % 32 != 0 ? bp.take<float>(B * L * w.Dp) : nullptr;
  w.total = bp.off + 256;
  return w;
}

int check_model_dims(const s2s_model_dims* d) {
  S2S_REQUIRE(d != nullptr, "null dims");
  S2S_REQUIRE(d->B > 0 && d->L > 0 && d->T > 0, "model: empty B/L/T");
  S2S_REQUIRE(d->numLayers >= 1 && d->inputFrameSize > 0, "model: bad encoder dims");
  S2S_REQUIRE(d->hiddenFrameSize % 16 == 0 && d->outputFrameSize % 16 == 0, "model: hidden sizes must be multiples of 16");
  S2S_TRY(attn_check_dims(model_attn(d)));
  return 0;
}

// fork: `side` waits for everything issued so far on `st`
int fork_to(hipStream_t st, hipStream_t side, hipEvent_t ev) {
  S2S_CHECK_HIP(hipEventRecord(ev, st));
  S2S_CHECK_HIP(hipStreamWaitEvent(side, ev, 0));
  return 0;
}

// bucket i's gradients are final on stream s (S2S_BUCKET_EVENTS); an external event node when captured
int mark_bucket(hipEvent_t* bev, int i, hipStream_t s) {
  if (!bev) return 0;
  if (!capturing(s)) {
    S2S_CHECK_HIP(hipEventRecord(bev[i], s));
    return 0;
  }
  // an event-record node appended to the capture (hipEventRecordWithFlags(..., hipEventRecordExternal)
  // is refused by this runtime): it fires on every replay, after everything captured on s so far
  hipStreamCaptureStatus cs;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t nd = 0;
  S2S_CHECK_HIP(hipStreamGetCaptureInfo_v2(s, &cs, &id, &g, &deps, &nd));
  hipGraphNode_t node;
  S2S_CHECK_HIP(hipGraphAddEventRecordNode(&node, g, deps, nd, bev[i]));
  S2S_CHECK_HIP(hipStreamUpdateCaptureDependencies(s, &node, 1, hipStreamSetCaptureDependencies));
  return 0;
}

// s2s_debug_bptt_wgrad(1) (A/B, tests): the first encoder layer's weight gradients inside its BPTT launch
// (gru_persist.hip bptt_wgrad) instead of a GEMM behind it on the side stream (measured slower)
std::atomic<int> g_bptt_wgrad{0};
// process-wide diagnostic knobs (s2s_debug_*, not in the C ABI header; A/B tools and tests only), read when a
// call issues its launches; no per-step state lives in globals (exclusive-CU mode, precision and the failure
// status are per call / per context)
std::atomic<int> g_defer_pack{1};  // s2s_debug_defer_pack(0): every layer packed in front of layer 1
std::atomic<int> g_dec_sync_prologue{1};  // s2s_debug_dec_sync_prologue(0): decoder sync preps in place
std::atomic<int> g_sync_handover{1};  // s2s_debug_sync_handover(0): a sync_prep in front of every GRU launch
std::atomic<int> g_fuse_dh{1};  // s2s_debug_fuse_dh(0): the decoder's dh by GEMMs in front of the top BPTT
// seed_dev: the context's dropout seed word when a captured step reads its seed from the device (the
// host writes it before each replay), else null (the seed is d->dropout_seed)
int model_step_impl(hipStream_t st, hipStream_t side, hipEvent_t* ev, hipEvent_t* bev, const s2s_model_dims* d,
                    const float* params, float* grads, const float* x, const int* labels, float scale, int flags,
                    float* logp, float* nll, void* workspace, const unsigned long long* seed_dev, unsigned* status) {
  const bool split = side != nullptr;
  ModelWs w = model_ws(d, workspace);
  const std::vector<LayerDims> layers = enc_layers(d);
  const std::vector<long> sizes = param_sizes(d);
  std::vector<const float*> P;
  std::vector<float*> G;
  long off = 0;
  for (long s : sizes) {
    P.push_back(params + off);
    G.push_back(grads + off);
    off += s;
  }
  // gradients are first written by the side stream's weight-gradient work when split: zero them
  // there (the fork precedes every gradient writer), off the critical path
  // the step head (when fused) also writes the loss seed dlogp = -labelmask and zeroes the gradients: no side-stream
  // kernel then runs in front of it (a replayed graph ran the side branch's first two kernels -- the zeroing and the
  // seed, 15 us -- before the head)
  GruLayerIO io0{};
  io0.ndir = 2;
  io0.B = d->B;
  io0.H = layers[0].H;
  const bool head_fused = g_sync_handover && gru_layer_persistent(io0);
  const bool head_seed = head_fused && split;                               // dlogp in the head
  const bool head_zero = head_seed && (flags & S2S_ZERO_GRADS);            // zeroing in the head
  // the side stream forks at the step's top (ev[13]).  Measured and rejected: forking after the head, or
  // creating the side branch's nodes after layer 1's launch (the decoder prologue then starts after layer 1 holds
  // every CU and is stretched over whole GRU layers); zeroing the gradients late on the side stream
  if (split) {
    S2S_CHECK_HIP(hipEventRecord(ev[13], st));
    S2S_CHECK_HIP(hipStreamWaitEvent(side, ev[13], 0));
  }
  if ((flags & S2S_ZERO_GRADS) && !head_zero) S2S_TRY(zero_async(split ? side : st, grads, sizeof(float) * (size_t)off));
  const int B = d->B, L = d->L, T = d->T, O = d->outputDepth;
  const int nl = (int)layers.size();
  AttnDims ad = model_attn(d);
  ad.dropout_seed_dev = seed_dev;
  ad.syncs_in_prologue = g_dec_sync_prologue;  // attn_fwd_prologue runs (and is joined) before the decoder
  // the step head wrote the loss seed: the decoder forward's head launch runs the MLP head's backward too
  if (head_seed) ad.dlogp_early = w.dlogp;
  AttnParams ap;
  AttnGrads ag;
  const float** pp = reinterpret_cast<const float**>(&ap);
  float** gp = reinterpret_cast<float**>(&ag);
  for (int i = 0; i < S2S_ATTN_NPARAMS; ++i) {
    pp[i] = P[6 * nl + i];
    gp[i] = G[6 * nl + i];
  }
  // layer-1 input padded to a multiple of 32 columns: its GEMMs then run on aligned full tiles
  const float* x0 = x;
  long ldx0 = d->inputFrameSize;
  if (w.xpad) {
    x0 = w.xpad;
    ldx0 = w.Dp;
  }
  // encoder layer l's operands (fwd: io.x is the layer input; bwd adds the grads)
  auto layer_io = [&](int l) {
    const int H = layers[l].H;
    GruLayerIO io{};
    io.ndir = 2; io.B = B; io.L = L; io.D = layers[l].D; io.H = H;
    io.x = l == 0 ? x0 : w.Y[l - 1];
    io.ldx = l == 0 ? ldx0 : 2L * layers[l - 1].H;
    io.Dx = (l == 0 && w.xpad) ? w.Dp : 0;
    for (int dd = 0; dd < 2; ++dd) {
      for (int g = 0; g < 3; ++g) io.W[dd][g] = P[6 * l + 3 * dd + g];
      io.reverse[dd] = dd;
      io.y[dd] = w.Y[l] + dd * H;
      io.saved[dd] = w.saved[2 * l + dd];
    }
    io.ldy = 2L * H;
    io.packed = w.pack[l];
    io.len = d->frame_lengths;
    // the persistent launches reserve their CU while the weight-gradient GEMMs run on the side stream
    io.excl = split ? 1 : 0;
    return io;  // io.status stays null: the step harvests every sync region once, at its end
  };
  // the step's head (pad, pack, the first persistent launch's sync prep) as one launch when layer 1 is persistent
  if (w.xpad && !head_fused) S2S_TRY(pad_cols_f32(st, x, d->inputFrameSize, w.xpad, B * L, d->inputFrameSize, w.Dp));
  // weight packing for every layer (both passes) and the decoder's parameter folds need only params
  // and labels: layer 1 on the critical path, the rest beside layer 1's recurrence when split
  // weight packing for every layer and both passes: one launch on the critical path (~10 us); the
  // decoder's parameter folds (params and labels only) beside the encoder when split
  // (when layer 1's persistent forward has spare slots, only what it reads is packed here; its spare slots
  // pack the rest -- the backward transposes and the later layers -- while it runs)
  GruPackJobs deferred{};
  bool defer_pack = false;
  {
    std::vector<GruLayerIO> ios;
    for (int l = 0; l < nl; ++l) ios.push_back(layer_io(l));
    defer_pack = g_defer_pack && 2 * nl <= kMaxPackJobs && gru_layer_preps_next(ios[0], true);
    if (head_fused) {
      GruStepHead extra{};
      if (head_seed) {
        extra.dlogp = w.dlogp; extra.labels = labels; extra.tlen = d->label_lengths;
        extra.B = B; extra.T = T; extra.O = O;
      }
      if (head_zero) {
        extra.zero = grads; extra.zero_n4 = (size_t)off / 4; extra.zero_tail = (int)(off % 4);
      }
      S2S_TRY(gru_step_head(st, ios.data(), w.pack.data(), nl, defer_pack ? &deferred : nullptr, x,
                            d->inputFrameSize, w.xpad, B * L, d->inputFrameSize, w.Dp, w.gsync[0],
                            gru_layer_sync_prep_bytes(ios[0]), w.gsync[1], &extra));
    }
    else
      S2S_TRY(gru_layers_pack(st, ios.data(), w.pack.data(), nl, defer_pack ? &deferred : nullptr));
  }
  // decoder parameter folds + dlogp = -labelmask (params and labels only): on the side stream, joined before the
  // decoder (the persistent GRU launches hold every CU, so it runs in their gaps); inline without a side stream
  if (split) {
    if (!head_seed)  // dlogp = -labelmask
      S2S_TRY(nll_seed(side, B, T, O, nullptr, labels, 0, nullptr, w.dlogp, d->label_lengths));
    S2S_TRY(attn_fwd_prologue(side, ad, labels, ap, w.attn_saved, w.attn_scratch));
    S2S_CHECK_HIP(hipEventRecord(ev[14], side));
  } else {
    S2S_TRY(attn_fwd_prologue(st, ad, labels, ap, w.attn_saved, w.attn_scratch));
  }
  // the persistent GRU launches of the step (forward layers 1..nl, then backward nl..1) alternate between
  // two sync regions; a launch with spare slots prepares the next launch's region itself, so only the
  // first launch has a sync_prep in front of it
  int glaunch = 0;
  bool gprepared = head_fused;  // the step head prepared the first launch's region
  bool gused[2] = {false, false};  // a persistent launch of this step used the region (harvested at the end)
  auto hand_over = [&](GruLayerIO& io, bool fwd, const GruLayerIO* next) {
    if (!g_sync_handover) return;
    if (gru_layer_persistent(io)) gused[glaunch & 1] = true;
    io.sync = w.gsync[glaunch & 1];
    io.sync_prepared = gprepared ? 1 : 0;
    io.sync_next = next ? w.gsync[(glaunch + 1) & 1] : nullptr;
    io.sync_next_prep = next ? gru_layer_sync_prep_bytes(*next) : 0;
    gprepared = next != nullptr && gru_layer_preps_next(io, fwd);
    ++glaunch;
  };
  // the region headers hold failure words: the first persistent launch's sync_prep clears the other region's
  // header too (sync_prep `clear`); when layer 1 runs per-step kernels, clear both here instead
  if (g_sync_handover && !gru_layer_persistent(layer_io(0))) {
    bool later = false;
    for (int l = 1; l < nl; ++l) later = later || gru_layer_persistent(layer_io(l));
    if (later)
      for (int r = 0; r < 2; ++r) S2S_TRY(zero_async(st, w.gsync[r], 256));
  }
  // ---- encoder forward (3 x BiGRU, JoinTable(2,2) by strided writes)
  for (int l = 0; l < nl; ++l) {
    GruLayerIO io = layer_io(l);
    const GruLayerIO next = layer_io(l + 1 < nl ? l + 1 : nl - 1);
    hand_over(io, true, &next);
    if (l == 0 && defer_pack) io.pack_jobs = &deferred;
    S2S_TRY(gru_layer_fwd(st, io, w.scratch, w.scratch_bytes));
  }
  // ---- attention decoder forward
  if (split) S2S_CHECK_HIP(hipStreamWaitEvent(st, ev[14], 0));
  float* lp = logp ? logp : w.logp;
  S2S_TRY(attn_fwd(st, ad, w.Y[nl - 1], labels, ap, lp, w.attn_saved, w.attn_scratch, w.attn_scratch_bytes, true,
                   nullptr, nullptr));
  // ---- loss seed: dlogp = -labelmask needs only the labels (computed beside the encoder when split);
  // the reported nll (timit.lua:268-272) is computed on the side stream at the end of the step
  if (!split)
    S2S_TRY(nll_seed(st, B, T, O, lp, labels, (flags & S2S_NORMALIZE_NLL) ? 1 : 0, nll ? nll : w.nll, w.dlogp,
                     d->label_lengths));
  // ---- decoder backward -> dh
  float* dYcur = w.dY0;
  float* dYnext = w.dY1;
  // the decoder's dh (context term + dVh V) is produced by the top layer's BPTT launch itself when it can
  // (gru_layer_dy_fused), otherwise by GEMMs in front of it
  AttnDhTerms dht{};
  S2S_TRY(attn_bwd_core(st, ad, w.Y[nl - 1], labels, ap, w.attn_saved, w.dlogp, dYcur, 0, w.attn_scratch,
                        w.attn_scratch_bytes, nullptr, nullptr, g_fuse_dh ? &dht : nullptr));
  // the decoder's weight gradients beside the top BPTT (side stream).  (Creating their nodes after the top BPTT's
  // launch measured 3.167 -> 3.680 ms: the replayed graph then ran the whole side branch after the last BPTT.)
  if (split) {
    S2S_CHECK_HIP(hipEventRecord(ev[0], st));
    S2S_CHECK_HIP(hipStreamWaitEvent(side, ev[0], 0));
  }
  S2S_TRY(attn_bwd_wgrad(split ? side : st, ad, w.Y[nl - 1], labels, ap, w.attn_saved, ag, scale, w.attn_scratch));
  S2S_TRY(mark_bucket(bev, 0, split ? side : st));
  // the reported nll (timit.lua:268-272) beside the encoder BPTT
  if (split)
    S2S_TRY(nll_seed(side, B, T, O, lp, labels, (flags & S2S_NORMALIZE_NLL) ? 1 : 0, nll ? nll : w.nll, nullptr,
                     d->label_lengths));
  // ---- encoder backward.  Layer l's weight-gradient GEMMs (side stream) wait for an event recorded between layer
  // l-1's BPTT sync prep and its launch, so the persistent BPTT is dispatched before the GEMM's workgroups take the
  // CUs (forked right after layer l's own BPTT, the replayed graph started the GEMM first and layers 2 and 1's BPTT
  // ran 590-618 us instead of 533-540 us, profiles/r01)
  const bool defer = split;
  int pending = -1;  // layer whose weight gradients wait for the next BPTT's sync prep
  auto issue_wgrad = [&](int l) -> int {
    const GruLayerIO io = layer_io(l);
    GruLayerGrad gr{};
    for (int dd = 0; dd < 2; ++dd)
      for (int g = 0; g < 3; ++g) gr.dW[dd][g] = G[6 * l + 3 * dd + g];
    gr.scale = scale;
    S2S_TRY(gru_layer_wgrad(split ? side : st, io, gr, w.dA[l], w.gws_side));
    S2S_TRY(mark_bucket(bev, nl - l, split ? side : st));
    return 0;
  };
  for (int l = nl - 1; l >= 0; --l) {
    const int H = layers[l].H;
    GruLayerIO io = layer_io(l);
    const GruLayerIO next = layer_io(l > 0 ? l - 1 : 0);
    hand_over(io, false, l > 0 ? &next : nullptr);
    GruLayerGrad gr{};
    for (int dd = 0; dd < 2; ++dd) {
      for (int g = 0; g < 3; ++g) gr.dW[dd][g] = G[6 * l + 3 * dd + g];
      gr.dy[dd] = dYcur + dd * H;
    }
    gr.lddy = 2L * H;
    // this layer's dX is the dy of the layer below: produced inside that layer's BPTT launch (or by one
    // GEMM in front of it), so the critical path has no GEMM between two BPTT launches
    gr.dx = nullptr;
    if (l == nl - 1 && dht.dvh) {  // dy = dh = sum_t alpha dc + dVh V, in-launch
      gr.ydA = dht.dvh;
      gr.yldA = dht.Sc;
      gr.yK = dht.Sc;
      gr.yN = dht.A;
      gr.yWx = dht.V;
      gr.yldw = dht.A;
      gr.yalpha = dht.alpha;
      gr.ydc = dht.dc;
      gr.yT = dht.T;
      if (dht.A != 2 * H || !gru_layer_dy_fused(io, gr)) {
        gr = GruLayerGrad{};
        for (int dd = 0; dd < 2; ++dd) {
          for (int g = 0; g < 3; ++g) gr.dW[dd][g] = G[6 * l + 3 * dd + g];
          gr.dy[dd] = dYcur + dd * H;
        }
        gr.lddy = 2L * H;
        S2S_TRY(attn_dh_gemms(st, dht, dYcur, 0));
      }
    }
    if (l + 1 < nl) {
      const GruLayerIO up = layer_io(l + 1);
      gr.ydA = w.dA[l + 1];
      gr.yldA = 3L * up.ndir * up.H;
      gr.yK = 3 * up.ndir * up.H;
      gr.yN = up.D;
      gr.yWx = gru_layer_packed_wx(up, &gr.yldw);
      S2S_REQUIRE(gr.yWx != nullptr && up.ldx == 2L * H, "model step: dX of layer above needs packed weights");
    }
    gr.scale = scale;
    // the first layer's weight gradients inside its BPTT launch: nothing behind the step's last recurrence
    const bool wg_in = l == 0 && g_bptt_wgrad && gru_layer_wgrad_fused(io);
    if (wg_in) {
      gr.wgrad = 1;
      gr.wpart = w.wpart;
    }
    if (defer && pending >= 0) gr.prep_event = ev[1 + pending];
    S2S_TRY(gru_layer_bwd_core(st, io, gr, w.dA[l], w.scratch, w.scratch_bytes));
    if (defer) {
      if (pending >= 0) {  // the layer above: after this BPTT's dispatch point
        S2S_CHECK_HIP(hipStreamWaitEvent(side, ev[1 + pending], 0));
        S2S_TRY(issue_wgrad(pending));
      }
      pending = l;
      if (l == 0 && wg_in) {
        S2S_TRY(mark_bucket(bev, nl, st));
      } else if (l == 0) {  // the last BPTT: nothing left to dispatch ahead of layer 1's GEMMs
        S2S_TRY(fork_to(st, side, ev[1 + l]));
        S2S_TRY(issue_wgrad(l));
      }
    } else if (wg_in) {
      S2S_TRY(mark_bucket(bev, nl - l, st));
    } else {
      if (split) S2S_TRY(fork_to(st, side, ev[1 + l]));
      S2S_TRY(gru_layer_wgrad(split ? side : st, io, gr, w.dA[l], w.gws_side));
      S2S_TRY(mark_bucket(bev, nl - l, split ? side : st));
    }
    float* tmp = dYcur;
    dYcur = dYnext;
    dYnext = tmp;
  }
  // failure words of every sync region the step's persistent launches used -> the context's status (handoff.h),
  // on the main stream after the last BPTT (beside the side stream's weight-gradient tail)
  if (status) {
    void* regions[4];
    int nr = 0;
    for (int r = 0; r < 2; ++r)
      if (gused[r]) regions[nr++] = w.gsync[r];
    nr += attn_sync_regions(ad, w.attn_saved, w.attn_scratch, &regions[nr], &regions[nr + 1]);
    S2S_TRY(launch_sync_harvest(st, regions, nr, status));
  }
  if (split) {  // join: the step ends when the side stream's gradient GEMMs are done
    S2S_CHECK_HIP(hipEventRecord(ev[15], side));
    S2S_CHECK_HIP(hipStreamWaitEvent(st, ev[15], 0));
  }
  return 0;
}

// Destroy a cached executable graph.  A replay of it may still be running (the host runs ahead of the
// device): HIP's hipGraphExecDestroy frees the executable's kernel-argument and node storage at once
// instead of deferring the free to the end of an in-flight launch (CUDA's documented behaviour), so
// destroying it under a running replay is a use-after-free in the runtime -- the round-1 segfaults
// inside s2s_model_step, which re-captured (and destroyed the previous exec) on every dropout step.
// Drain the streams the replay used first.
int drop_graph(s2s_ctx* ctx, CachedGraph& g) {
  if (g.exec) {
    if (g.launched_on) S2S_CHECK_HIP(hipStreamSynchronize(g.launched_on));
    if (ctx->side) S2S_CHECK_HIP(hipStreamSynchronize(ctx->side));
    (void)hipGraphExecDestroy(g.exec);
  }
  if (g.graph) (void)hipGraphDestroy(g.graph);
  g.exec = nullptr;
  g.graph = nullptr;
  return 0;
}

}  // namespace

// ================================================================== C ABI
extern "C" {

int s2s_version(void) { return 1; }

int s2s_prof_enable(int on) {
  s2s::g_prof = on != 0;
  return 0;
}

// Aggregates every recorded launch per kernel family (after synchronising on its events):
// one line per family "name<TAB>launches<TAB>total_us<TAB>flops<TAB>bytes\n", then clears.
int s2s_prof_collect(char* buf, size_t cap) {
  using namespace s2s;
  std::lock_guard<std::mutex> lk(g_prof_mu);
  struct Agg {
    std::string name;
    long n;
    double us, flops, bytes;
  };
  std::vector<Agg> aggs;
  for (auto& r : g_recs) {
    float ms = 0.f;
    if (r.b) {
      S2S_CHECK_HIP(hipEventSynchronize(r.b));
      S2S_CHECK_HIP(hipEventElapsedTime(&ms, r.a, r.b));
    }
    Agg* a = nullptr;
    for (auto& x : aggs)
      if (x.name == r.name) a = &x;
    if (!a) {
      aggs.push_back({r.name, 0, 0.0, 0.0, 0.0});
      a = &aggs.back();
    }
    a->n += 1;
    a->us += 1000.0 * ms;
    a->flops += r.flops;
    a->bytes += r.bytes;
    g_pool.push_back(r.a);
    if (r.b) g_pool.push_back(r.b);
  }
  g_recs.clear();
  std::string out;
  for (auto& a : aggs) {
    char line[256];
    snprintf(line, sizeof(line), "%s\t%ld\t%.3f\t%.6e\t%.6e\n", a.name.c_str(), a.n, a.us, a.flops, a.bytes);
    out += line;
  }
  S2S_REQUIRE(buf != nullptr && cap > out.size(), "prof: buffer too small");
  std::memcpy(buf, out.c_str(), out.size() + 1);
  return 0;
}
const char* s2s_last_error(void) { return s2s::get_error(); }

int s2s_ctx_create(int device, s2s_ctx** out) {
  S2S_REQUIRE(out != nullptr, "null out");
  int n = 0;
  S2S_CHECK_HIP(hipGetDeviceCount(&n));
  S2S_REQUIRE(device >= 0 && device < n, "device index out of range");
  S2S_CHECK_HIP(hipSetDevice(device));
  auto* c = new s2s_ctx();
  c->device = device;
  if (hipHostMalloc(reinterpret_cast<void**>(&c->status_host), 64, hipHostMallocMapped | hipHostMallocCoherent) !=
          hipSuccess ||
      hipHostGetDevicePointer(reinterpret_cast<void**>(&c->status_dev), c->status_host, 0) != hipSuccess) {
    if (c->status_host) (void)hipHostFree(c->status_host);
    delete c;
    S2S_REQUIRE(false, "ctx: host-coherent status word allocation failed");
  }
  if (c->status_host) std::memset(c->status_host, 0, 64);
  // (the side stream at the lowest queue priority measured no change)
  if (hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) {
    c->side = nullptr;
  }
  for (auto& e : c->ev)
    if (c->side && hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
      (void)hipStreamDestroy(c->side);
      c->side = nullptr;
    }
  if (hipStreamCreateWithFlags(&c->wside, hipStreamNonBlocking) != hipSuccess) c->wside = nullptr;
  if (c->wside && hipEventCreateWithFlags(&c->wev, hipEventDisableTiming) != hipSuccess) c->wev = nullptr;
  *out = c;
  return 0;
}

void s2s_ctx_destroy(s2s_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  for (auto& g : ctx->graphs) (void)drop_graph(ctx, g);
  ctx->graphs.clear();
  if (ctx->seed_dev) (void)hipFree(ctx->seed_dev);
  s2s::gemm_stage_free(&ctx->lt);
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  for (auto& e : ctx->ev)
    if (e) (void)hipEventDestroy(e);
  for (auto& e : ctx->bev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->wev) (void)hipEventDestroy(ctx->wev);
  if (ctx->wside) (void)hipStreamDestroy(ctx->wside);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->status_host) (void)hipHostFree(ctx->status_host);
  delete ctx;
}

int s2s_ctx_set_flags(s2s_ctx* ctx, int flags) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  ctx->flags = flags;
  return 0;
}

int s2s_ctx_set_wgrad_overlap(s2s_ctx* ctx, int on) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  S2S_REQUIRE(!on || (ctx->wside && ctx->wev), "ctx: no stream for the parameter gradients");
  ctx->wgrad_overlap = on ? 1 : 0;
  return 0;
}

int s2s_ctx_join_wgrad(s2s_ctx* ctx, s2s_stream_t stream) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  if (!ctx->wside || !ctx->wev || static_cast<hipStream_t>(stream) == ctx->wside) return 0;
  S2S_CHECK_HIP(hipSetDevice(ctx->device));
  S2S_CHECK_HIP(hipEventRecord(ctx->wev, ctx->wside));
  S2S_CHECK_HIP(hipStreamWaitEvent(static_cast<hipStream_t>(stream), ctx->wev, 0));
  return 0;
}

s2s_stream_t s2s_ctx_side_stream(s2s_ctx* ctx) { return ctx ? static_cast<s2s_stream_t>(ctx->wside) : nullptr; }

int s2s_ctx_status(s2s_ctx* ctx, s2s_stream_t stream, int* status, int clear) {
  S2S_REQUIRE(ctx != nullptr && status != nullptr, "null argument");
  S2S_CHECK_HIP(hipSetDevice(ctx->device));
  S2S_CHECK_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  if (ctx->side) S2S_CHECK_HIP(hipStreamSynchronize(ctx->side));
  if (ctx->wside) S2S_CHECK_HIP(hipStreamSynchronize(ctx->wside));
  *status = 0;
  if (!ctx->status_host) return 0;
  *status = (__atomic_load_n(ctx->status_host, __ATOMIC_ACQUIRE) ? S2S_STATUS_HANDOFF_TIMEOUT : 0) |
            (__atomic_load_n(ctx->status_host + 1, __ATOMIC_ACQUIRE) ? S2S_STATUS_ABORTED_REGION : 0);
  if (clear)
    for (int i = 0; i < 16; ++i) __atomic_store_n(ctx->status_host + i, 0u, __ATOMIC_RELEASE);
  return 0;
}

int s2s_ctx_set_precision(s2s_ctx* ctx, int precision) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  S2S_REQUIRE(precision == S2S_PREC_FP32 || precision == S2S_PREC_BF16_GEMM || precision == S2S_PREC_BF16_ALL,
              "unknown precision");
  ctx->precision = precision;
  return 0;
}

size_t s2s_gru_saved_bytes(int B, int L, int H) { return sizeof(float) * (size_t)B * L * 5 * H; }
size_t s2s_gru_scratch_bytes(int ndir, int B, int L, int D, int H) {
  return gru_layer_scratch_bytes(ndir, B, L, D, H);
}

static int fill_gru_io(GruLayerIO& io, int ndir, int B, int L, int D, int H, const int* reverse, const float* x,
                       long ldx, const float* const* W, float* const* y, long ldy, void* const* saved,
                       const int* lengths) {
  S2S_REQUIRE(ndir == 1 || ndir == 2, "gru: ndir must be 1 or 2");
  S2S_REQUIRE(reverse && x && W && saved, "gru: null argument");
  S2S_REQUIRE(ldx >= D, "gru: ldx < D");
  io.ndir = ndir; io.B = B; io.L = L; io.D = D; io.H = H; io.x = x; io.ldx = ldx; io.ldy = ldy;
  io.len = lengths;
  for (int d = 0; d < ndir; ++d) {
    for (int g = 0; g < 3; ++g) {
      io.W[d][g] = W[3 * d + g];
      S2S_REQUIRE(io.W[d][g] != nullptr, "gru: null weight");
    }
    io.reverse[d] = reverse[d] ? 1 : 0;
    io.y[d] = y ? y[d] : nullptr;
    io.saved[d] = static_cast<float*>(saved[d]);
    S2S_REQUIRE(io.saved[d] != nullptr, "gru: null saved buffer");
  }
  return 0;
}

int s2s_gru_fwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, const int* reverse,
                const float* x, long ldx, const float* const* W, float* const* y, long ldy, void* const* saved,
                const int* lengths, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  GruLayerIO io{};
  S2S_TRY(fill_gru_io(io, ndir, B, L, D, H, reverse, x, ldx, W, y, ldy, saved, lengths));
  S2S_REQUIRE(y != nullptr, "gru: null y");
  for (int d = 0; d < ndir; ++d) S2S_REQUIRE(y[d] != nullptr, "gru: null y");
  S2S_REQUIRE(ldy >= H, "gru: ldy < H");
  io.status = ctx->status_dev;
  return gru_layer_fwd(static_cast<hipStream_t>(stream), io, scratch, scratch_bytes);
}

int s2s_gru_bwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, const int* reverse,
                const float* x, long ldx, const float* const* W, void* const* saved, const float* const* dy,
                long lddy, float* dx, long lddx, int dx_accumulate, float* const* dW, float scale,
                const int* lengths, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  GruLayerIO io{};
  S2S_TRY(fill_gru_io(io, ndir, B, L, D, H, reverse, x, ldx, W, nullptr, H, saved, lengths));
  S2S_REQUIRE(dy && dW, "gru: null dy/dW");
  GruLayerGrad gr{};
  for (int d = 0; d < ndir; ++d) {
    gr.dy[d] = dy[d];
    S2S_REQUIRE(gr.dy[d] != nullptr, "gru: null dy");
    for (int g = 0; g < 3; ++g) {
      gr.dW[d][g] = dW[3 * d + g];
      S2S_REQUIRE(gr.dW[d][g] != nullptr, "gru: null dW");
    }
  }
  gr.lddy = lddy;
  gr.dx = dx;
  gr.lddx = lddx;
  gr.dx_accumulate = dx_accumulate;
  gr.scale = scale;
  io.status = ctx->status_dev;
  return gru_layer_bwd(static_cast<hipStream_t>(stream), io, gr, scratch, scratch_bytes);
}

size_t s2s_lstm_saved_bytes(int B, int L, int H) { return lstm_saved_bytes(B, L, H); }
size_t s2s_lstm_scratch_bytes(int ndir, int B, int L, int D, int H, int peepholes) {
  return lstm_scratch_bytes(ndir, B, L, D, H, peepholes);
}

static int fill_lstm_io(LstmLayerIO& io, int ndir, int B, int L, int D, int H, int peep, const int* reverse,
                        const float* x, long ldx, const float* const* W, float* const* y, long ldy,
                        void* const* saved) {
  S2S_REQUIRE(ndir == 1 || ndir == 2, "lstm: ndir must be 1 or 2");
  S2S_REQUIRE(reverse && x && W && saved, "lstm: null argument");
  S2S_REQUIRE(ldx >= D, "lstm: ldx < D");
  io.ndir = ndir; io.B = B; io.L = L; io.D = D; io.H = H; io.peep = peep ? 1 : 0;
  io.x = x; io.ldx = ldx; io.W = W; io.ldy = ldy;
  for (int d = 0; d < ndir; ++d) {
    for (int p = 0; p < lstm_nparams(io.peep); ++p) S2S_REQUIRE(W[d * lstm_nparams(io.peep) + p], "lstm: null weight");
    io.reverse[d] = reverse[d] ? 1 : 0;
    io.y[d] = y ? y[d] : nullptr;
    io.saved[d] = static_cast<float*>(saved[d]);
    S2S_REQUIRE(io.saved[d] != nullptr, "lstm: null saved buffer");
  }
  return 0;
}

int s2s_lstm_fwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, int peepholes,
                 const int* reverse, const float* x, long ldx, const float* const* W, float* const* y, long ldy,
                 void* const* saved, const int* lengths, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  LstmLayerIO io{};
  S2S_TRY(fill_lstm_io(io, ndir, B, L, D, H, peepholes, reverse, x, ldx, W, y, ldy, saved));
  io.len = lengths;
  S2S_REQUIRE(y != nullptr, "lstm: null y");
  for (int d = 0; d < ndir; ++d) S2S_REQUIRE(y[d] != nullptr, "lstm: null y");
  io.status = ctx->status_dev;
  return lstm_layer_fwd(static_cast<hipStream_t>(stream), io, scratch, scratch_bytes);
}

int s2s_lstm_bwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, int peepholes,
                 const int* reverse, const float* x, long ldx, const float* const* W, void* const* saved,
                 const float* const* dy, long lddy, float* dx, long lddx, int dx_accumulate, float* const* dW,
                 float scale, const int* lengths, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  LstmLayerIO io{};
  S2S_TRY(fill_lstm_io(io, ndir, B, L, D, H, peepholes, reverse, x, ldx, W, nullptr, H, saved));
  io.len = lengths;
  S2S_REQUIRE(dy && dW, "lstm: null dy/dW");
  LstmLayerGrad gr{};
  for (int d = 0; d < ndir; ++d) {
    gr.dy[d] = dy[d];
    S2S_REQUIRE(gr.dy[d] != nullptr, "lstm: null dy");
    for (int p = 0; p < lstm_nparams(io.peep); ++p)
      S2S_REQUIRE(dW[d * lstm_nparams(io.peep) + p], "lstm: null dW");
  }
  gr.lddy = lddy; gr.dx = dx; gr.lddx = lddx; gr.dx_accumulate = dx_accumulate; gr.dW = dW; gr.scale = scale;
  if (ctx->wgrad_overlap) {  // the parameter gradients beside the caller's next launches, forked once dA is final
    gr.wst = ctx->wside;
    gr.wev = ctx->wev;
  }
  io.status = ctx->status_dev;
  return lstm_layer_bwd(static_cast<hipStream_t>(stream), io, gr, scratch, scratch_bytes);
}

size_t s2s_attn_saved_bytes(const s2s_attn_dims* d) { return d ? attn_saved_bytes(to_attn(d)) : 0; }
size_t s2s_attn_scratch_bytes(const s2s_attn_dims* d) { return d ? attn_scratch_bytes(to_attn(d)) : 0; }
const float* s2s_attn_mlp_input(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_mlp_input(to_attn(d), saved) : nullptr;
}
const float* s2s_attn_alpha(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_alpha(to_attn(d), saved) : nullptr;
}
const float* s2s_attn_ws(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_ws(to_attn(d), saved) : nullptr;
}
const float* s2s_attn_vh(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_vh(to_attn(d), saved) : nullptr;
}
const float* s2s_attn_mono_ind(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_mono_ind(to_attn(d), saved) : nullptr;
}
const int* s2s_attn_maxout_argmax(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_maxout_argmax(to_attn(d), saved) : nullptr;
}
const float* s2s_attn_dropout_mask(const s2s_attn_dims* d, const void* saved) {
  return d && saved ? attn_saved_dropout_mask(to_attn(d), saved) : nullptr;
}

// the decoder's persistent launch of this call (which = 0 forward, 1 backward) -> the context's status
static int harvest_attn(s2s_ctx* ctx, s2s_stream_t stream, const AttnDims& ad, void* saved, void* scratch, int which) {
  void* r[2];
  if (attn_sync_regions(ad, saved, scratch, &r[0], &r[1]) == 0) return 0;
  return launch_sync_harvest(static_cast<hipStream_t>(stream), &r[which], 1, ctx->status_dev);
}

int s2s_attn_fwd(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const int* labels,
                 const float* const* params, float* logp, void* saved, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && h && labels && params && (logp || d->external_mlp) && saved, "attn: null argument");
  AttnParams ap;
  const float** pp = reinterpret_cast<const float**>(&ap);
  for (int i = 0; i < attn_nparams(d); ++i) {
    pp[i] = params[i];
    S2S_REQUIRE(pp[i] != nullptr || attn_param_optional(d, i), "attn: null parameter");
  }
  const AttnDims ad = to_attn(d);
  S2S_TRY(attn_fwd(static_cast<hipStream_t>(stream), ad, h, labels, ap, logp, saved, scratch, scratch_bytes));
  return harvest_attn(ctx, stream, ad, saved, scratch, 0);
}

int s2s_attn_bwd(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const int* labels,
                 const float* const* params, const void* saved, const float* dlogp, float* dh, int dh_accumulate,
                 float* const* grads, float scale, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && h && labels && params && saved && dlogp && dh && grads, "attn: null argument");
  AttnParams ap;
  AttnGrads ag;
  const float** pp = reinterpret_cast<const float**>(&ap);
  float** gp = reinterpret_cast<float**>(&ag);
  for (int i = 0; i < attn_nparams(d); ++i) {
    pp[i] = params[i];
    gp[i] = grads[i];
    S2S_REQUIRE((pp[i] != nullptr && gp[i] != nullptr) || attn_param_optional(d, i), "attn: null parameter/grad");
  }
  const AttnDims ad = to_attn(d);
  const hipStream_t st = static_cast<hipStream_t>(stream);
  S2S_TRY(attn_bwd_core(st, ad, h, labels, ap, saved, dlogp, dh, dh_accumulate, scratch, scratch_bytes));
  // accGradParameters beside the caller's next launches (s2s_ctx_set_wgrad_overlap): it reads only saved and scratch
  hipStream_t wst;
  S2S_TRY(wgrad_stream(ctx, st, &wst));
  S2S_TRY(attn_bwd_wgrad(wst, ad, h, labels, ap, saved, ag, scale, scratch));
  return harvest_attn(ctx, stream, ad, const_cast<void*>(saved), scratch, 1);
}

size_t s2s_attn_beam_workspace_bytes(const s2s_attn_dims* d, int K, int maxseqlength) {
  if (!d || K < 1 || maxseqlength < 1) return 0;
  return attn_beam_workspace_bytes(to_attn(d), K, maxseqlength);
}

static int beam_params(const s2s_attn_dims* d, const float* const* params, AttnParams& ap) {
  S2S_REQUIRE(params, "beam search: null parameters");
  const float** pp = reinterpret_cast<const float**>(&ap);
  for (int i = 0; i < attn_nparams(d); ++i) {
    pp[i] = params[i];
    S2S_REQUIRE(pp[i] != nullptr || attn_param_optional(d, i), "beam search: null parameter");
  }
  return 0;
}

int s2s_attn_beam_search(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h,
                         const float* const* params, int eos, int K, int maxseqlength, int* out, int ldo, int* out_len,
                         float* out_score, void* workspace, size_t workspace_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && h && out && out_len && workspace, "beam search: null argument");
  AttnParams ap{};
  S2S_TRY(beam_params(d, params, ap));
  return attn_beam_search(static_cast<hipStream_t>(stream), to_attn(d), h, ap, eos, K, maxseqlength, out, ldo,
                          out_len, out_score, workspace, workspace_bytes);
}

int s2s_attn_beam_init(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h,
                       const float* const* params, int eos, int K, int maxseqlength, void* workspace,
                       size_t workspace_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && h && workspace, "beam search: null argument");
  AttnParams ap{};
  S2S_TRY(beam_params(d, params, ap));
  return attn_beam_init(static_cast<hipStream_t>(stream), to_attn(d), h, ap, eos, K, maxseqlength, workspace,
                        workspace_bytes);
}

int s2s_attn_beam_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* const* params, int K,
                       int maxseqlength, int count, void* workspace, size_t workspace_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && workspace && count >= 0 && count <= maxseqlength, "beam search: bad step");
  AttnParams ap{};
  S2S_TRY(beam_params(d, params, ap));
  return attn_beam_step(static_cast<hipStream_t>(stream), to_attn(d), ap, K, maxseqlength, count, workspace,
                        workspace_bytes);
}

const float* s2s_attn_beam_mlp_input(const s2s_attn_dims* d, int K, int maxseqlength, void* workspace) {
  return d && workspace ? attn_beam_mlp_input(to_attn(d), K, maxseqlength, workspace) : nullptr;
}

int s2s_attn_beam_advance(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int eos, int K,
                          int maxseqlength, int count, const float* logp, void* workspace, size_t workspace_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && workspace && count >= 0 && count <= maxseqlength, "beam search: bad step");
  return attn_beam_advance(static_cast<hipStream_t>(stream), to_attn(d), eos, K, maxseqlength, count, logp, workspace,
                           workspace_bytes);
}

int s2s_attn_beam_done(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int K, int maxseqlength,
                       void* workspace, int* all_done) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && workspace && all_done, "beam search: null argument");
  return attn_beam_done(static_cast<hipStream_t>(stream), to_attn(d), K, maxseqlength, workspace, all_done);
}

int s2s_attn_beam_finish(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int K, int maxseqlength,
                         int* out, int ldo, int* out_len, float* out_score, void* workspace) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(d && out && out_len && workspace, "beam search: null argument");
  return attn_beam_finish(static_cast<hipStream_t>(stream), to_attn(d), K, maxseqlength, workspace, out, ldo, out_len,
                          out_score);
}

int s2s_edit_distance(s2s_ctx* ctx, s2s_stream_t stream, int n, const int* a, const int* alen, int lda, const int* b,
                      const int* blen, int ldb, int* out) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(n == 0 || (a && alen && b && blen && out), "edit distance: null argument");
  return edit_distance(static_cast<hipStream_t>(stream), n, a, alen, lda, b, blen, ldb, out);
}

// ---------------------------------------------------------------- encoder front-ends (frontend.hip)
size_t s2s_tconv_scratch_bytes(int B, int L, int Din, int Dout, int kW) {
  return tconv_scratch_bytes(B, L, Din, Dout, kW);
}
int s2s_tconv_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x,
                  const float* W, const float* b, float* y) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && W && y, "TemporalConvolution: null argument");
  return tconv_fwd(static_cast<hipStream_t>(stream), B, L, Din, Dout, kW, relu, x, W, b, y);
}
int s2s_tconv_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x,
                  const float* W, const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db,
                  float scale, void* scratch, size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && W && dy && scratch, "TemporalConvolution: null argument");
  return tconv_bwd(static_cast<hipStream_t>(stream), B, L, Din, Dout, kW, relu, x, W, y, dy, dx, dx_accumulate, dW, db,
                   scale, scratch, scratch_bytes, ctx->wgrad_overlap ? ctx->wside : nullptr, ctx->wev);
}
int s2s_tmaxpool_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int D, int kW, int dW, const float* x, float* y,
                     int* idx) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && y && idx, "TemporalMaxPooling: null argument");
  return tmaxpool_fwd(static_cast<hipStream_t>(stream), B, L, D, kW, dW, x, y, idx);
}
int s2s_tmaxpool_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int D, int kW, int dW, const int* idx,
                     const float* dy, float* dx) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(idx && dy && dx, "TemporalMaxPooling: null argument");
  return tmaxpool_bwd(static_cast<hipStream_t>(stream), B, L, D, kW, dW, idx, dy, dx);
}
size_t s2s_sconv_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW) {
  return sconv_scratch_bytes(B, Cin, H, W, Cout, kH, kW);
}
int s2s_sconv_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu,
                  const float* x, const float* weight, const float* bias, float* y, void* scratch,
                  size_t scratch_bytes) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && weight && y && scratch, "SpatialConvolutionMM: null argument");
  return sconv_fwd(static_cast<hipStream_t>(stream), B, Cin, H, W, Cout, kH, kW, relu, x, weight, bias, y, scratch,
                   scratch_bytes);
}
int s2s_sconv_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu,
                  const float* x, const float* weight, const float* y, const float* dy, float* dx, int dx_accumulate,
                  float* dweight, float* dbias, float scale, void* scratch, size_t scratch_bytes, int col_from_fwd) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && weight && dy && scratch, "SpatialConvolutionMM: null argument");
  return sconv_bwd(static_cast<hipStream_t>(stream), B, Cin, H, W, Cout, kH, kW, relu, x, weight, y, dy, dx,
                   dx_accumulate, dweight, dbias, scale, scratch, scratch_bytes, col_from_fwd);
}
int s2s_smaxpool_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH,
                     const float* x, float* y, int* idx) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && y && idx, "SpatialMaxPooling: null argument");
  return smaxpool_fwd(static_cast<hipStream_t>(stream), B, C, H, W, kW, kH, dW, dH, x, y, idx);
}
int s2s_smaxpool_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH,
                     const int* idx, const float* dy, float* dx) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(idx && dy && dx, "SpatialMaxPooling: null argument");
  return smaxpool_bwd(static_cast<hipStream_t>(stream), B, C, H, W, kW, kH, dW, dH, idx, dy, dx);
}
int s2s_swap12(s2s_ctx* ctx, s2s_stream_t stream, int B, int D1, int D2, int D3, const float* x, float* y) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && y && x != y, "Transpose2: null or in-place argument");
  return swap12(static_cast<hipStream_t>(stream), B, D1, D2, D3, x, y);
}
int s2s_relu_fwd(s2s_ctx* ctx, s2s_stream_t stream, long n, const float* x, float* y) {
  S2S_TRY(set_device(ctx));
  return relu_fwd(static_cast<hipStream_t>(stream), n, x, y);
}
int s2s_relu_bwd(s2s_ctx* ctx, s2s_stream_t stream, long n, const float* x, const float* dy, float* dx) {
  S2S_TRY(set_device(ctx));
  return relu_bwd(static_cast<hipStream_t>(stream), n, x, dy, dx);
}
int s2s_logsoftmax_fwd(s2s_ctx* ctx, s2s_stream_t stream, long rows, int n, const float* x, float* y) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(x && y, "LogSoftMax: null argument");
  return logsoftmax_fwd(static_cast<hipStream_t>(stream), rows, n, x, y);
}
int s2s_logsoftmax_bwd(s2s_ctx* ctx, s2s_stream_t stream, long rows, int n, const float* y, const float* dy,
                       float* dx) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(y && dy && dx, "LogSoftMax: null argument");
  return logsoftmax_bwd(static_cast<hipStream_t>(stream), rows, n, y, dy, dx);
}

int s2s_nll_seed(s2s_ctx* ctx, s2s_stream_t stream, int B, int T, int O, const float* logp, const int* labels,
                 const int* label_lengths, int normalize, float* nll, float* dlogp) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(logp && labels && nll, "nll: null argument");
  S2S_REQUIRE(B > 0 && T > 0 && O > 0, "nll: empty dims");
  return nll_seed(static_cast<hipStream_t>(stream), B, T, O, logp, labels, normalize, nll, dlogp, label_lengths);
}

size_t s2s_model_param_count(const s2s_model_dims* d) {
  if (!d) return 0;
  size_t n = 0;
  for (long s : param_sizes(d)) n += (size_t)s;
  return n;
}

long s2s_model_param_offset(const s2s_model_dims* d, int i, long* numel) {
  if (!d) return -1;
  const std::vector<long> s = param_sizes(d);
  if (i < 0 || i >= (int)s.size()) return -1;
  long off = 0;
  for (int j = 0; j < i; ++j) off += s[j];
  if (numel) *numel = s[i];
  return off;
}

size_t s2s_model_workspace_bytes(const s2s_model_dims* d) {
  if (check_model_dims(d) != 0) return 0;
  return model_ws(d, nullptr).total;
}

int s2s_model_attn_dims(const s2s_model_dims* d, s2s_attn_dims* out) {
  S2S_REQUIRE(d != nullptr && out != nullptr, "null argument");
  std::memset(out, 0, sizeof(*out));
  out->B = d->B; out->L = d->L; out->T = d->T;
  out->annotationDepth = 2 * d->outputFrameSize; out->scoreDepth = d->scoreDepth; out->stateDepth = d->stateDepth;
  out->outputDepth = d->outputDepth; out->mlpDepth = d->mlpDepth; out->maxoutWindow = d->maxoutWindow;
  out->penalty = d->penalty; out->dropout = d->dropout; out->dropout_seed = d->dropout_seed;
  out->dropout_mask = d->dropout_mask;
  return 0;
}

const void* s2s_model_attn_saved(const s2s_model_dims* d, const void* workspace) {
  if (!d || !workspace || check_model_dims(d) != 0) return nullptr;
  ModelWs w = model_ws(d, const_cast<void*>(workspace));
  return w.attn_saved;
}

const float* s2s_model_encoder_output(const s2s_model_dims* d, const void* workspace) {
  if (!d || !workspace) return nullptr;
  ModelWs w = model_ws(d, const_cast<void*>(workspace));
  return w.Y.back();
}

int s2s_model_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_model_dims* d, const float* params, float* grads,
                   const float* x, const int* labels, float scale, int flags, float* logp, float* nll,
                   void* workspace, size_t workspace_bytes) {
  S2S_TRY(set_device(ctx));
  // the model step keeps its GEMMs on gemm_f32's tiles: it is captured into a HIP graph at its first call (graph
  // mode), where the big GEMM's staging buffer could not be grown
  set_gemm_stage(nullptr);
  S2S_TRY(check_model_dims(d));
  S2S_REQUIRE(params && grads && x && labels && workspace, "model: null argument");
  S2S_REQUIRE(workspace_bytes >= model_ws(d, nullptr).total, "model: workspace too small");
  hipStream_t st = static_cast<hipStream_t>(stream);
  hipEvent_t* bev = nullptr;
  if (flags & S2S_BUCKET_EVENTS) {
    S2S_REQUIRE(d->numLayers + 1 <= kMaxBuckets, "model: too many layers for S2S_BUCKET_EVENTS");
    for (auto& e : ctx->bev)
      if (!e) S2S_CHECK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    bev = ctx->bev;
  }
  if (!(ctx->flags & S2S_CTX_GRAPH) || st == nullptr)
    return model_step_impl(st, (st && (ctx->flags & S2S_CTX_OVERLAP)) ? ctx->side : nullptr, ctx->ev, bev, d,
                           params, grads, x, labels, scale, flags, logp, nll, workspace, nullptr, ctx->status_dev);
  // In-kernel dropout draws from a new seed every step: the replayed graph reads it from the context's
  // device word, written before each replay, so the seed is not part of the graph key.  Injected masks
  // (or no dropout) leave the seed unread: it is not part of the key either.
  const bool dev_seed = d->dropout > 0.f && d->dropout_mask == nullptr;
  if (dev_seed && !ctx->seed_dev) S2S_CHECK_HIP(hipMalloc(reinterpret_cast<void**>(&ctx->seed_dev), 64));
  GraphKey key;
  std::memset(&key, 0, sizeof(key));
  key.d = *d;
  key.d.dropout_seed = 0;
  const void* ptrs[7] = {params, grads, x, labels, logp, nll, workspace};
  std::memcpy(key.ptrs, ptrs, sizeof(ptrs));
  key.scale = scale;
  key.flags = flags;
  key.precision = ctx->precision;
  key.stream = stream;
  CachedGraph* hit = nullptr;
  for (auto& g : ctx->graphs)
    if (g.key == key) hit = &g;
  if (!hit) {
    if ((int)ctx->graphs.size() >= ctx->graph_cap) {  // evict the least recently used
      size_t lru = 0;
      for (size_t i = 1; i < ctx->graphs.size(); ++i)
        if (ctx->graphs[i].used < ctx->graphs[lru].used) lru = i;
      S2S_TRY(drop_graph(ctx, ctx->graphs[lru]));
      ctx->graphs.erase(ctx->graphs.begin() + (long)lru);
    }
    S2S_CHECK_HIP(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    const int rc = model_step_impl(st, (ctx->flags & S2S_CTX_OVERLAP) ? ctx->side : nullptr, ctx->ev, bev, d,
                                   params, grads, x, labels, scale, flags, logp, nll, workspace,
                                   dev_seed ? ctx->seed_dev : nullptr, ctx->status_dev);
    hipGraph_t g = nullptr;
    const hipError_t ec = hipStreamEndCapture(st, &g);
    if (rc != 0) {
      if (g) (void)hipGraphDestroy(g);
      return rc;
    }
    S2S_CHECK_HIP(ec);
    CachedGraph cg;
    cg.key = key;
    cg.graph = g;
    const hipError_t ei = hipGraphInstantiate(&cg.exec, g, nullptr, nullptr, 0);
    if (ei != hipSuccess) {
      (void)hipGraphDestroy(g);
      S2S_CHECK_HIP(ei);
    }
    ctx->graphs.push_back(cg);
    hit = &ctx->graphs.back();
    ctx->captures += 1;
  }
  hit->used = ++ctx->graph_clock;
  hit->launched_on = st;
  if (dev_seed) S2S_TRY(set_device_u64(st, ctx->seed_dev, d->dropout_seed));
  S2S_CHECK_HIP(hipGraphLaunch(hit->exec, st));
  ctx->replays += 1;
  return 0;
}

int s2s_ctx_graph_stats(s2s_ctx* ctx, long* captures, long* replays, int* cached) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  if (captures) *captures = ctx->captures;
  if (replays) *replays = ctx->replays;
  if (cached) *cached = (int)ctx->graphs.size();
  return 0;
}

int s2s_ctx_set_graph_cache(s2s_ctx* ctx, int capacity) {
  S2S_REQUIRE(ctx != nullptr, "null context");
  S2S_REQUIRE(capacity >= 1 && capacity <= 64, "graph cache capacity must be in [1, 64]");
  S2S_TRY(set_device(ctx));
  ctx->graph_cap = capacity;
  while ((int)ctx->graphs.size() > capacity) {
    size_t lru = 0;
    for (size_t i = 1; i < ctx->graphs.size(); ++i)
      if (ctx->graphs[i].used < ctx->graphs[lru].used) lru = i;
    S2S_TRY(drop_graph(ctx, ctx->graphs[lru]));
    ctx->graphs.erase(ctx->graphs.begin() + (long)lru);
  }
  return 0;
}

int s2s_model_weight_matrices(const s2s_model_dims* d, long* mats) {
  if (check_model_dims(d) != 0) return -1;
  const std::vector<long> sizes = param_sizes(d);
  std::vector<long> t;
  long off = 0;
  int p = 0;
  for (auto& ld : enc_layers(d))
    for (int i = 0; i < 6; ++i, ++p) {
      t.insert(t.end(), {off, (long)ld.H, (long)ld.H + ld.D});
      off += sizes[p];
    }
  const long A = 2L * d->outputFrameSize, Sc = d->scoreDepth, S = d->stateDepth, O = d->outputDepth,
             M = d->mlpDepth, Mk = (long)d->mlpDepth * d->maxoutWindow;
  // decoder parameters in s2s_attn order; rows x cols of the weights, 0 for the biases
  const long shp[S2S_ATTN_NPARAMS][2] = {{Sc, A}, {Sc, S}, {0, 0}, {1, Sc}, {S, O}, {0, 0}, {S, A}, {0, 0},
                                         {S, 2 * S}, {0, 0}, {S, 2 * S}, {S, 2 * S}, {S, 2 * S}, {Mk, S + A},
                                         {0, 0}, {O, M}, {0, 0}};
  for (int i = 0; i < S2S_ATTN_NPARAMS; ++i, ++p) {
    if (shp[i][0] > 0) t.insert(t.end(), {off, shp[i][0], shp[i][1]});
    off += sizes[p];
  }
  if (mats) std::copy(t.begin(), t.end(), mats);
  return (int)(t.size() / 3);
}

size_t s2s_optim_state_bytes(size_t n) { return optim_state_bytes(n); }

int s2s_optim_reset(s2s_ctx* ctx, s2s_stream_t stream, void* state, size_t n) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(state && n > 0, "optim: null state");
  return optim_state_reset(static_cast<hipStream_t>(stream), state, n);
}

int s2s_optim_set_noise_step(s2s_ctx* ctx, s2s_stream_t stream, void* state, size_t n, unsigned t) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(state && n > 0, "optim: null state");
  return optim_set_noise_step(static_cast<hipStream_t>(stream), state, n, t);
}

static int adadelta_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params,
                         float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm,
                         const float* skip_flag) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(cfg != nullptr, "optim: null config");
  S2S_REQUIRE(cfg->rho >= 0.f && cfg->rho < 1.f && cfg->eps > 0.f && cfg->maxnorm > 0.f, "optim: bad config");
  const OptimConfig c{cfg->rho,           cfg->eps,           cfg->maxnorm,       cfg->weightDecay,
                      cfg->colnorm_max,   cfg->gradnoise_eta, cfg->gradnoise_gamma, cfg->gradnoise_seed};
  // device-side guard: the update is skipped if the context's failure status (or *skip_flag) is set when it runs
  return optim_adadelta_step(static_cast<hipStream_t>(stream), c, params, grads, n, state, mats, n_mats, gradnorm,
                             ctx->status_dev, skip_flag);
}

int s2s_optim_adadelta_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params,
                            float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm) {
  return adadelta_step(ctx, stream, cfg, params, grads, n, state, mats, n_mats, gradnorm, nullptr);
}

int s2s_optim_adadelta_step_flag(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params,
                                 float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm,
                                 const float* skip_flag) {
  return adadelta_step(ctx, stream, cfg, params, grads, n, state, mats, n_mats, gradnorm, skip_flag);
}

int s2s_ctx_status_flag(s2s_ctx* ctx, s2s_stream_t stream, float* flag) {
  S2S_REQUIRE(ctx != nullptr && flag != nullptr, "null argument");
  S2S_CHECK_HIP(hipSetDevice(ctx->device));
  S2S_REQUIRE(ctx->status_dev != nullptr, "context has no status words");
  return status_flag(static_cast<hipStream_t>(stream), ctx->status_dev, flag);
}

int s2s_model_bucket_count(const s2s_model_dims* d) {
  if (check_model_dims(d) != 0) return -1;
  return d->numLayers + 1;
}

int s2s_model_bucket(const s2s_model_dims* d, int i, size_t* offset, size_t* count) {
  S2S_TRY(check_model_dims(d));
  const int nl = d->numLayers;
  S2S_REQUIRE(offset && count && i >= 0 && i <= nl, "bucket: bad index");
  const std::vector<long> sizes = param_sizes(d);
  // bucket 0: the decoder (params 6 nl ..); bucket j >= 1: encoder layer nl - j (params 6 l .. 6 l + 5)
  const int p0 = i == 0 ? 6 * nl : 6 * (nl - i), p1 = i == 0 ? (int)sizes.size() : p0 + 6;
  size_t off = 0, n = 0;
  for (int p = 0; p < (int)sizes.size(); ++p) {
    if (p < p0) off += sizes[p];
    else if (p < p1) n += sizes[p];
  }
  *offset = off;
  *count = n;
  return 0;
}

int s2s_stream_wait_bucket(s2s_ctx* ctx, s2s_stream_t stream, int i) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(i >= 0 && i < kMaxBuckets && ctx->bev[i], "bucket: no event (step without S2S_BUCKET_EVENTS?)");
  S2S_CHECK_HIP(hipStreamWaitEvent(static_cast<hipStream_t>(stream), ctx->bev[i], 0));
  return 0;
}

int s2s_comm_unique_id(void* out_bytes) {
  S2S_REQUIRE(out_bytes != nullptr, "null out");
  ncclUniqueId id;
  const ncclResult_t r = ncclGetUniqueId(&id);
  S2S_REQUIRE(r == ncclSuccess, std::string("ncclGetUniqueId: ") + ncclGetErrorString(r));
  std::memcpy(out_bytes, &id, sizeof(id));
  return 0;
}

int s2s_comm_init(s2s_ctx* ctx, const void* id_bytes, int nranks, int rank) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(id_bytes && nranks > 0 && rank >= 0 && rank < nranks, "comm: bad arguments");
  ncclUniqueId id;
  std::memcpy(&id, id_bytes, sizeof(id));
  if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
  ctx->comm = nullptr;
  const ncclResult_t r = ncclCommInitRank(&ctx->comm, nranks, id, rank);
  S2S_REQUIRE(r == ncclSuccess, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
  return 0;
}

int s2s_allreduce_sum(s2s_ctx* ctx, s2s_stream_t stream, float* buf, size_t count) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(ctx->comm != nullptr, "allreduce: s2s_comm_init first");
  const ncclResult_t r =
      ncclAllReduce(buf, buf, count, ncclFloat32, ncclSum, ctx->comm, static_cast<hipStream_t>(stream));
  S2S_REQUIRE(r == ncclSuccess, std::string("ncclAllReduce: ") + ncclGetErrorString(r));
  return 0;
}

}  // extern "C"

// diagnostic: 1 runs the decoder's off-path kernels (vbar, alpha/indicators, dVh) on the side stream

// diagnostic (not part of the C ABI header): one GEMM C = alpha op(A) op(B) + beta C through the library's
// MFMA GEMM (bf16 = 1: the bf16-operand kernels), on the legacy default stream; for the layout tests
extern "C" int s2s_debug_gemm(int transA, int transB, int M, int N, int K, float alpha, const float* A, long lda,
                              const float* B, long ldb, float beta, float* C, long ldc, int bf16, float* ws,
                              size_t ws_floats) {
  s2s::set_gemm_precision(bf16 ? s2s::kGemmBf16 : s2s::kGemmF32);
  const int rc = s2s::gemm1(nullptr, transA != 0, transB != 0, M, N, K, alpha, A, lda, B, ldb, beta, C, ldc, nullptr,
                            s2s::GemmWs{ws, ws ? ws_floats : 0});
  s2s::set_gemm_precision(s2s::kGemmF32);
  return rc;
}
// test / bench entry: one problem straight on the big-tile bf16 GEMM (gemm_bf16.hip) with the context's staging
// buffer; *done = 0 when the kernel declined it (nothing launched)
extern "C" int s2s_debug_gemm_big_run(s2s_ctx* ctx, s2s_stream_t stream, int transA, int transB, int M, int N, int K,
                                      float alpha, const float* A, long lda, const float* B, long ldb, float beta,
                                      float* C, long ldc, const float* bias, int relu, int* done) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(done != nullptr, "null argument");
  s2s::GemmProblem q{A, B, C, bias, lda, ldb, ldc, M, N, K, alpha, beta};
  q.relu = relu;
  bool d = false;
  const int rc = s2s::gemm_big_bf16(static_cast<hipStream_t>(stream), q, transA != 0, transB != 0, &d);
  *done = d ? 1 : 0;
  return rc;
}
extern "C" void s2s_debug_fuse_dh(int on) { g_fuse_dh = on; }
// test knob: the next n sync_preps (any context) start their region aborted, so the persistent launch behind
// each reports S2S_STATUS_ABORTED_REGION and returns at once (tests/test_gpu_status.py)
static std::atomic<int> g_inject_abort{0};
// diagnostic: the context's 16 status words ([0] timeout, [1] aborted region, [4 + i] raw failure bits of the
// last harvest's region i) -- tools/status_diag.py
extern "C" int s2s_debug_status_words(s2s_ctx* ctx, unsigned* out16) {
  S2S_REQUIRE(ctx && out16, "null argument");
  for (int i = 0; i < 16; ++i) out16[i] = ctx->status_host ? __atomic_load_n(ctx->status_host + i, __ATOMIC_ACQUIRE) : 0u;
  return 0;
}
// test probe: one wave of a persistent-style launch that waits for a value nobody writes (region: >= 768 bytes
// of device memory); the context's status must then read S2S_STATUS_HANDOFF_TIMEOUT
extern "C" int s2s_debug_handoff_timeout(s2s_ctx* ctx, s2s_stream_t stream, void* region) {
  S2S_TRY(set_device(ctx));
  S2S_REQUIRE(region != nullptr, "null region");
  return handoff_timeout_probe_launch(static_cast<hipStream_t>(stream), region, ctx->status_dev);
}
extern "C" void s2s_debug_inject_abort(int n) { g_inject_abort = n; }
int s2s::inject_abort_take() {
  int v = g_inject_abort.load(std::memory_order_relaxed);
  while (v > 0 && !g_inject_abort.compare_exchange_weak(v, v - 1)) {
  }
  return v > 0 ? 1 : 0;
}
extern "C" void s2s_debug_sync_handover(int on) { g_sync_handover = on; }
extern "C" void s2s_debug_dec_sync_prologue(int on) { g_dec_sync_prologue = on; }
extern "C" void s2s_debug_defer_pack(int on) { g_defer_pack = on; }
// diagnostic: the first encoder layer's weight gradients inside its BPTT launch (1) or by the GEMM behind it (0)
extern "C" void s2s_debug_bptt_wgrad(int on) { g_bptt_wgrad = on; }
