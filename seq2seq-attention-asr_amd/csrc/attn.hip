// Attention decoder forward/backward: the drop-in for nn.Attention's decoder graph
// (Attention.lua:43-211, 305-327) unrolled by nn.RNNAttention (RNNAttention.lua:144-253)
// with the Chorowski decoder_recurrent / decoder_mlp (timit/model_chorowski_baseline.lua:48-59).
//
// Per decoder step t (teacher forcing, RNNAttention.lua:172-176), one launch each:
//   F1 ws = Ws s_{t-1} + bs                           skinny MFMA  (Attention.lua:65-66)
//   F2 e_l = we . tanh(ws + Vh_l); local softmax stats
//      and partial context over a 16-frame chunk       wave-dot + wave reductions (Attention.lua:98-117, 132-134)
//   F3 combine chunks -> alpha, c, lse, MonoAlign ind  (MonotonicAlignment.lua:19-42)
//   F4 c_in = Wc c + bc, y_in = Wy[:,y_{t-1}] + by      skinny MFMA  (Attention.lua:149-150)
//   F5 d = Wd [c_in; y_in] + bd                        skinny MFMA  (Attention.lua:151)
//   F6/F7 decoder GRU (GRU.lua:22-30) on [s_{t-1}; d]   skinny MFMA x2
// The decoder MLP (Maxout -> Linear -> LogSoftMax) is not on the recurrence, so it runs
// once for all B*T rows after the loop (one GEMM + one per-row head kernel).
// Backward mirrors RNNAttention:updateGradInput's reverse loop (RNNAttention.lua:233-250):
// MLP backward for all rows first, then per step GRU p1/p2, Wd^T, Wc^T, the fused
// attention backward (softmax, tanh, dVh, dh += alpha dc), the dws combine and Ws^T;
// every weight gradient is one GEMM over all B*T rows afterwards.
#include "attn.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

#include "handoff.h"
#include "skinny.h"

namespace s2s {

namespace {

constexpr int LC = 16;  // frames per attention workgroup (4 waves x 4 frames)

struct AttnK {
  // dims
  int B, L, T, A, Sc, S, O, M, K, NCH, t;
  float penalty;
  int hk, hf;  // hybrid attention filter size / feature maps (hf = 0: off)
  const int *flen, *tlen;  // variable-length batch: frames / labels per utterance (null: L / T)
  // params
  AttnParams P;
  const float* h;
  const int* labels;
  // saved
  float *Vh, *WS, *E, *ALPHA, *LSE, *IND, *C, *HX, *RHX, *CY, *GSV, *VV, *MM, *LOGP, *MASK;
  int* AM;
  // fwd scratch
  float *PM, *PL, *PC, *U;
  // the MLP GEMM's unreduced split-K slabs (UPS > 1: U = sum of UP[s * UPMN + e] in slice order + bm, summed by the
  // MLP head instead of a reduce launch in front of it), or null
  const float* UP;
  int UPS;
  long UPMN;
  // bwd scratch
  float *DO, *DU, *DV, *DGA, *DS, *DSP, *DSPF, *DD, *DCY, *DC, *DVH, *PDWS, *DWS, *DWEACC, *YP;
  // hybrid attention: HGT (kW, Sc) = (U W)^T and HCU (Sc) = U b (saved); QA [2][B][L][kW] the
  // d alpha_{t-1} partials q_{l,i} of the step after; PDG [B*NCH][kW][Sc] dG partials; DGT, DCU (bwd)
  float *HGT, *HCU, *QA, *PDG, *DGT, *DCU;
  float *WhT, *GT, *WdT, *WcT, *WsT;
  // decoder LSTM: LW (4S, 2S) rows [Wqh | Wqx] per gate q in (i, f, g, o), LB (4S) = bqx + bqh (saved),
  // LC (B*T, S) cell states (saved), LDW (4S, 2S) weight-gradient staging (bwd scratch); GT holds LW^T
  float *LW, *LB, *LC, *LDW;
  int lstm;
  // persistent-kernel granule buffers ([2 slots][...]) and abort word; one zeroed region each
  granule_t *gS, *gWS, *gPM, *gPL, *gPC, *gC, *gCY, *gD, *gQ;           // forward
  granule_t *gZ, *gR, *gH, *gDD, *gDCY, *gDC, *gPDWS, *gDWS;           // backward
  char *fsync, *bsync;
  size_t fsync_bytes, bsync_bytes;
  // the regions' 256-byte headers (abort word, epoch, sticky failure bits), kept apart from the overlapping
  // forward / backward working sets: the forward region's header must survive the backward for the harvest
  char *fhdr, *bhdr;
  unsigned long long* stamps;  // diagnostic phase stamps (nullptr = off)
  float* dh;
  long lddh;
  const float* dlogp;
  float* logp;
};

struct Layout {
  size_t saved, fwd, bwd;
};

// operands of the XCD-local decoder kernels (dec_xcd.inc)
struct XArgs {
  int U, nchains, allow_local, XLC, NCH;
  float* WX;    // (3S, A)  Wx' = [Wz_d; Wr_d; Wh_d] Wd_c Wc          (saved)
  float* WXT;   // (A, 3S)  Wx'^T                                    (saved)
  float* WXD;   // (3S, S)  [Wz_d; Wr_d; Wh_d] packed                (saved)
  float* WDC;   // (S, A)   Wd_c Wc                                  (fwd scratch)
  float* KX;    // (B*T, 3S) d-part constants of the gates            (fwd scratch)
  float* KD;    // (B*T, S)  Wd_c bc + Wd_y y_in + bd                 (fwd scratch)
  float* BKD;   // (S)       Wd_c bc + bd                             (fwd scratch)
  float* DE;    // (B*T, L)  de_{t,l}                                 (bwd scratch)
  float* DCS;   // (B*T, A)  dc_t (= AttnK::DC)                       (bwd scratch)
  float* VBAR;  // (B, Sc)   mean Vh row per utterance                 (bwd scratch)
  float* XWHT;  // (S, S)    Wh[:, :S]^T                               (saved)
  float* XZRT;  // (S, 2S)   [Wz[:, :S]; Wr[:, :S]]^T                   (saved)
  float* XWST;  // (S, Sc)   Ws^T                                      (saved)
  // prologue operand re-layouts (dec_xcd_pack_ops) so its GEMMs batch as NN problems (fwd scratch)
  float* PWDYT;  // (S, S)   Wd[:, S:]^T
  float* PWDCT;  // (S, S)   Wd[:, :S]^T
  float* PWCT;   // (A, S)   Wc^T
  float* PWXDT;  // (S, 3S)  WXD^T
  float* WDCT;   // (A, S)   (Wd_c Wc)^T
  // granule buffers, [2 slots][...]
  granule_t *gS, *gWS, *gPM, *gPL, *gPC, *gC, *gQ;     // forward (inside fsync)
  granule_t *gDGZ, *gDGR, *gDGH, *gDC, *gPDWS, *gDWS;  // backward (inside bsync)
  unsigned *fcensus, *bcensus;
  // sentinel rows of XCD-local chains (handoff.h), [T slots][B][...] floats, outside the zeroed regions
  float *sS, *sQ, *sC, *sWS;  // forward: s_t, q_t (S), c_t (A), ws_t (Sc)
  float *sDGZ, *sDGR, *sDGH, *sDC, *sDWS;  // backward: da_z, da_r, da_h (S), dc (A), dws (Sc)
};
// extra operands of the LSTM / hybrid kernels (carve, dec_xcd_lstm_prologue)
struct XLArgs {
  int S;          // real state width (the kernels carry SP)
  int hk, pl;     // hybrid taps kW and the left pad
  float* WG;      // (4SP, SP)  Wq_h, gate-major rows q SP + u, zero-padded             (saved)
  float* WXG;     // (4SP, A)   Wq_x Wd_c Wc, rows as WG                                 (saved)
  float* WSP;     // (Sc, SP)   Ws with zero columns past S                              (saved)
  float* WUT;     // (SP, 4SP)  WUT[n][q SP + u] = Wq_h[u][n]                            (saved)
  float* WXGT;    // (A, 4SP)   WXG^T                                                    (saved)
  float* WSTP;    // (SP, SCP)  Ws^T, zero-padded                                        (saved)
  float* WXD4;    // (4S, S)    [Wi_x; Wf_x; Wg_x; Wo_x] (the weight gradients' dd)      (saved)
  float* BQ;      // (4S)       bq_x + bq_h                                              (fwd scratch)
  float* KXG;     // (B T, 4SP) Wq_x KD_t + bq, zero-padded                              (fwd scratch)
  float* sS;      // [T][B][SP] s_t (chain-interleaved sentinel rows)                    (fwd)
  float* sDG[4];  // [T][B][SP] da_q (chain-interleaved)                                 (bwd)
  float* sDC[2];  // [T][B][A] the two K halves of dc                                    (bwd)
  float* sDWS;    // [T][B][SCP] dws (chain-interleaved; columns past Sc published as 0)  (bwd)
  granule_t *gS, *gE, *gA;  // [2][B][SP], [2][B][L] scores and alpha (hybrid location features)   (inside fsync)
  granule_t *gDG[4], *gDC[2], *gDWS, *gQA;  // [2][B][SP] x 4, [2][B][A] x 2, [2][B][SCP], [2][B][L][kW] (bsync)
  float* PDG;     // [B NX][kW][Sc] dG partials per (utterance, chunk)                   (bwd scratch)
};
constexpr int kXLC = 32;     // largest attention chunk (frames) of the XCD-local decoder, LDS-resident
constexpr int kXLCStream = 64;  // largest chunk when h / Vh rows are read from global memory each step
constexpr int kXMaxCh = 16;  // chunks per utterance
constexpr int kXChains = 8;  // chains per launch (one per XCD)
constexpr int kXWG = 32;     // workgroups per chain

// ---- XCD-local decoder (dec_xcd.inc) plan: chains of U utterances, one per XCD (U as small as
// 8 chains allow, so the attention work spreads over as many XCDs as possible), each utterance cut
// into NCH chunks of XLC frames (U * NCH <= 32 workgroups).  var = 0: the shape is served by the
// older kernels (S2S_DEC_MODE=persist / step force those).
struct XPlan {
  int var = 0, U = 0, nchains = 0, XLC = 0, NCH = 0, res = 1;
};
// S2S_DEC_MODE=step / persist (tests, A/B): force the per-step launches / the 7-seam persistent kernels; read once.
// s2s_debug_dec_mode(m) overrides it in-process (m = 0 auto, 1 step, 2 persist; -1 back to the environment's)
std::atomic<int> g_dec_mode_force{-1};
int dec_mode() {
  static const int m = [] {
    const char* e = std::getenv("S2S_DEC_MODE");
    return e && std::strcmp(e, "step") == 0 ? 1 : e && std::strcmp(e, "persist") == 0 ? 2 : 0;
  }();
  const int f = g_dec_mode_force.load();
  return f >= 0 ? f : m;
}
XPlan dec_xcd_plan(const AttnDims& d) {
  XPlan p;
  if (dec_mode() != 0) return p;
  int var = 0;
  if (d.lstm) {
    // the LSTM decoder with hybrid attention (dec_xcd_lstm.inc): the conv + BiLSTM model's shape (timit/timit.lua:
    // 127-155: S = 400, A = 256, scoreDepth 150 padded to 160, kW = 5), chains of <= 4 utterances, resident chunks
    if (d.hf > 0 && d.hk == 5 && d.S == 400 && d.A == 256 && d.Sc == 160) var = 3;
  } else if (d.hf == 0) {  // (hybrid attention with the GRU decoder: the per-step kernels)
    if (d.S == 256 && d.A == 512 && d.Sc == 512) var = 1;
    else if (d.S == 64 && d.A == 128 && d.Sc == 128) var = 2;
  }
  if (!var) return p;
  const int U = (d.B + kXChains - 1) / kXChains;
  if (U > 16 || (var == 3 && U > 4)) return p;
  const int nmax = std::min(kXMaxCh, kXWG / U);
  const int xlc = ((d.L + nmax - 1) / nmax + 3) / 4 * 4;
  if (xlc > kXLCStream || d.T > 256) return p;  // (dec_xcd_dvh stages up to 256 steps)
  // resident chunks while they fit LDS (U utterances x L frames x (A + Sc) floats per XCD); longer
  // utterances stream their h / Vh rows from global memory (L2 / MALL) every step
  // (S2S_DEC_STREAM = 1 / 0: force Vh-only / no residency -- diagnostics and the bitwise tests)
  const char* fs = std::getenv("S2S_DEC_STREAM");
  p.res = xlc <= kXLC ? 2 : 1;
  if (fs && std::strcmp(fs, "1") == 0) p.res = 1;
  if (fs && std::strcmp(fs, "0") == 0) p.res = 0;
  if (var == 3 && p.res != 2) return p;  // (the LSTM kernels keep their chunks resident)
  p.var = var;
  p.U = U;
  p.nchains = (d.B + U - 1) / U;
  p.XLC = xlc;
  p.NCH = (d.L + xlc - 1) / xlc;
  return p;
}

constexpr int kXlSP = 448, kXlSCP = 192;  // the LSTM kernels' padded S and Sc (var 3: S = 400, Sc = 160)
Layout carve(const AttnDims& d, AttnK* k, char* saved, char* scratch, XArgs* x = nullptr, XLArgs* y = nullptr) {
  const long B = d.B, L = d.L, T = d.T, A = d.A, Sc = d.Sc, S = d.S, O = d.O, M = d.M, Mk = (long)d.M * d.K;
  const long NCH = (d.L + LC - 1) / LC, BT = B * T;
  Bump sv{saved, 0, 0};
  float* Vh = sv.take<float>(B * L * Sc);
  float* WS = sv.take<float>(BT * Sc);
  float* E = sv.take<float>(BT * L);
  float* ALPHA = sv.take<float>(BT * L);
  float* LSE = sv.take<float>(BT);
  float* IND = sv.take<float>(BT);
  float* C = sv.take<float>(BT * A);
  float* HX = sv.take<float>(BT * 2 * S);
  float* RHX = sv.take<float>(BT * 2 * S);
  float* CY = sv.take<float>(BT * 2 * S);
  const long NG = d.lstm ? 4 : 3;  // gate rows per step: GRU z, r, hh / LSTM i, f, g, o
  float* GSV = sv.take<float>(BT * NG * S);
  float* VV = sv.take<float>(BT * (S + A));
  float* MM = sv.take<float>(BT * M);
  int* AM = sv.take<int>(BT * M);
  float* LOGP = sv.take<float>(BT * O);
  float* MASK = d.dropout > 0.f ? sv.take<float>(BT * (S + A)) : nullptr;
  float* WX = sv.take<float>(3 * S * A);
  float* WXT = sv.take<float>(3 * S * A);
  float* WXD = sv.take<float>(3 * S * S);
  float* XWHT = sv.take<float>(S * S);
  float* XZRT = sv.take<float>(2 * S * S);
  float* XWST = sv.take<float>(S * Sc);
  float* VBAR = sv.take<float>(B * Sc);  // mean Vh row per utterance (computed by the forward)
  float* LW = d.lstm ? sv.take<float>(4 * S * 2 * S) : nullptr;
  float* LB = d.lstm ? sv.take<float>(4 * S) : nullptr;
  float* LCS = d.lstm ? sv.take<float>(BT * S) : nullptr;
  const long HK = d.hf > 0 ? d.hk : 0;
  float* HGT = HK ? sv.take<float>(HK * Sc) : nullptr;
  float* HCU = HK ? sv.take<float>(Sc) : nullptr;
  const XPlan xpl = dec_xcd_plan(d);
  const long NX = std::max(1, xpl.NCH);
  // the LSTM / hybrid XCD-local kernels' operands (var 3; empty otherwise)
  const bool v3 = xpl.var == 3;
  const long SP = v3 ? kXlSP : 0, SCP = v3 ? kXlSCP : 0, S4 = v3 ? 4 * S : 0;
  float* lWG = sv.take<float>(4 * SP * SP);
  float* lWXG = sv.take<float>(4 * SP * A);
  float* lWSP = sv.take<float>(v3 ? Sc * SP : 0);
  float* lWUT = sv.take<float>(SP * 4 * SP);
  float* lWXGT = sv.take<float>(v3 ? A * 4 * SP : 0);
  float* lWSTP = sv.take<float>(SP * SCP);
  float* lWXD4 = sv.take<float>(S4 * (v3 ? S : 0));
  Bump f{scratch, 0, 0};
  float* PM = f.take<float>(B * NCH);
  float* PL = f.take<float>(B * NCH);
  float* PC = f.take<float>(B * NCH * A);
  float* U = f.take<float>(BT * Mk);
  float* WDC = f.take<float>(S * A);
  float* PWDYT = f.take<float>(S * S);
  float* PWDCT = f.take<float>(S * S);
  float* PWCT = f.take<float>(A * S);
  float* PWXDT = f.take<float>(S * 3 * S);
  float* WDCT = f.take<float>(A * S);
  float* KX = f.take<float>(BT * 3 * S);
  float* KD = f.take<float>(BT * S);
  float* BKD = f.take<float>(S);
  float* lBQ = f.take<float>(S4);
  float* lKXG = f.take<float>(v3 ? BT * 4 * SP : 0);
  Bump g{scratch, 0, 0};
  float* DO = g.take<float>(BT * O);
  float* DU = g.take<float>(BT * Mk);
  float* DV = g.take<float>(BT * (S + A));
  float* DGA = g.take<float>(BT * NG * S);
  float* DS = g.take<float>(B * S);
  float* DSP = g.take<float>(B * S);
  float* DSPF = g.take<float>(B * S);
  float* DD = g.take<float>(BT * S);
  float* DCY = g.take<float>(BT * 2 * S);
  float* DC = g.take<float>(BT * A);
  float* DVH = g.take<float>(B * L * Sc);
  float* PDWS = g.take<float>(B * NCH * Sc);
  float* DWS = g.take<float>(BT * Sc);
  float* DWEACC = g.take<float>(B * NCH * Sc);
  float* YP = g.take<float>(BT * O);
  float* WhT = g.take<float>(S * S);
  float* GT = g.take<float>(2 * S * NG * S);
  float* LDW = d.lstm ? g.take<float>(4 * S * 2 * S) : nullptr;
  float* WdT = g.take<float>(2 * S * S);
  float* WcT = g.take<float>(A * S);
  float* WsT = g.take<float>(S * Sc);
  float* DE = g.take<float>(BT * L);

  float* QA = HK ? g.take<float>(2 * B * L * HK) : nullptr;
  float* PDG = HK ? g.take<float>(B * NCH * HK * Sc) : nullptr;
  float* DGT = HK ? g.take<float>(HK * Sc) : nullptr;
  float* DCU = HK ? g.take<float>(Sc) : nullptr;
  // granule regions (256-byte header = abort word), zeroed by one memset before each persistent launch
  char* fsync = f.take<char>(256);
  granule_t* gS = f.take<granule_t>(2 * B * S);
  granule_t* gWS = f.take<granule_t>(2 * B * Sc);
  granule_t* gPM = f.take<granule_t>(2 * B * NCH);
  granule_t* gPL = f.take<granule_t>(2 * B * NCH);
  granule_t* gPC = f.take<granule_t>(2 * B * NCH * A);
  granule_t* gC = f.take<granule_t>(2 * B * A);
  granule_t* gCY = f.take<granule_t>(2 * B * 2 * S);
  granule_t* gD = f.take<granule_t>(2 * B * S);
  granule_t* gQ = f.take<granule_t>(2 * B * S);
  granule_t* xgS = f.take<granule_t>(2 * B * S);
  granule_t* xgWS = f.take<granule_t>(2 * B * Sc);
  granule_t* xgPM = f.take<granule_t>(2 * B * NX);
  granule_t* xgPL = f.take<granule_t>(2 * B * NX);
  granule_t* xgPC = f.take<granule_t>(2 * B * NX * A);
  granule_t* xgC = f.take<granule_t>(2 * B * A);
  granule_t* xgQ = f.take<granule_t>(2 * B * S);
  granule_t* lgS = f.take<granule_t>(2 * B * SP);
  granule_t* lgE = f.take<granule_t>(v3 ? 2 * B * L : 0);
  granule_t* lgA = f.take<granule_t>(v3 ? 2 * B * L : 0);
  unsigned* fcensus = f.take<unsigned>(kXChains * kXWG);
  const size_t fsync_bytes = f.off - (size_t)(fsync - scratch);
  float* lsS = f.take<float>(BT * SP);
  float* xsS = f.take<float>(BT * S);
  float* xsQ = f.take<float>(BT * S);
  float* xsC = f.take<float>(BT * A);
  float* xsWS = f.take<float>(BT * Sc);
  char* bsync = g.take<char>(256);
  granule_t* gZ = g.take<granule_t>(2 * B * S);
  granule_t* gR = g.take<granule_t>(2 * B * S);
  granule_t* gH = g.take<granule_t>(2 * B * S);
  granule_t* gDD = g.take<granule_t>(2 * B * S);
  granule_t* gDCY = g.take<granule_t>(2 * B * S);
  granule_t* gDC = g.take<granule_t>(2 * B * A);
  granule_t* gPDWS = g.take<granule_t>(2 * B * NCH * Sc);
  granule_t* gDWS = g.take<granule_t>(2 * B * Sc);
  granule_t* xgDGZ = g.take<granule_t>(2 * B * S);
  granule_t* xgDGR = g.take<granule_t>(2 * B * S);
  granule_t* xgDGH = g.take<granule_t>(2 * B * S);
  granule_t* xgDC = g.take<granule_t>(2 * B * A);
  granule_t* xgPDWS = g.take<granule_t>(2 * B * NX * Sc);
  granule_t* xgDWS = g.take<granule_t>(2 * B * Sc);
  granule_t* lgDG[4];
  for (auto& q : lgDG) q = g.take<granule_t>(2 * B * SP);
  granule_t* lgDC[2];
  for (auto& q : lgDC) q = g.take<granule_t>(v3 ? 2 * B * A : 0);
  granule_t* lgDWS = g.take<granule_t>(2 * B * SCP);
  granule_t* lgQA = g.take<granule_t>(v3 ? 2 * B * L * HK : 0);
  unsigned* bcensus = g.take<unsigned>(kXChains * kXWG);
  const size_t bsync_bytes = g.off - (size_t)(bsync - scratch);
  float* lsDG[4];
  for (auto& q : lsDG) q = g.take<float>(BT * SP);
  float* lsDC[2];
  for (auto& q : lsDC) q = g.take<float>(v3 ? BT * A : 0);
  float* lsDWS = g.take<float>(BT * SCP);
  float* lPDG = g.take<float>(v3 ? B * NX * HK * Sc : 0);
  float* xsDGZ = g.take<float>(BT * S);
  float* xsDGR = g.take<float>(BT * S);
  float* xsDGH = g.take<float>(BT * S);
  float* xsDC = g.take<float>(BT * A);
  float* xsDWS = g.take<float>(BT * Sc);
  if (k) {
    k->gS = gS; k->gWS = gWS; k->gPM = gPM; k->gPL = gPL; k->gPC = gPC; k->gC = gC; k->gCY = gCY; k->gD = gD;
    k->gQ = gQ; k->gZ = gZ; k->gR = gR; k->gH = gH; k->gDD = gDD; k->gDCY = gDCY; k->gDC = gDC; k->gPDWS = gPDWS;
    k->gDWS = gDWS; k->fsync = fsync; k->bsync = bsync; k->fsync_bytes = fsync_bytes; k->bsync_bytes = bsync_bytes;
  }
  if (k) {
    k->B = d.B; k->L = d.L; k->T = d.T; k->A = d.A; k->Sc = d.Sc; k->S = d.S; k->O = d.O; k->M = d.M; k->K = d.K;
    k->NCH = (int)NCH; k->penalty = d.penalty; k->t = 0;
    k->flen = d.flen; k->tlen = d.tlen;
    k->hk = (int)HK; k->hf = d.hf;
    k->lstm = d.lstm; k->LW = LW; k->LB = LB; k->LC = LCS; k->LDW = LDW;
    k->HGT = HGT; k->HCU = HCU; k->QA = QA; k->PDG = PDG; k->DGT = DGT; k->DCU = DCU;
    k->MASK = MASK;
    k->Vh = Vh; k->WS = WS; k->E = E; k->ALPHA = ALPHA; k->LSE = LSE; k->IND = IND; k->C = C; k->HX = HX;
    k->RHX = RHX; k->CY = CY; k->GSV = GSV; k->VV = VV; k->MM = MM; k->AM = AM; k->LOGP = LOGP;
    k->PM = PM; k->PL = PL; k->PC = PC; k->U = U;
    k->DO = DO; k->DU = DU; k->DV = DV; k->DGA = DGA; k->DS = DS; k->DSP = DSP; k->DSPF = DSPF; k->DD = DD;
    k->DCY = DCY; k->DC = DC; k->DVH = DVH; k->PDWS = PDWS; k->DWS = DWS; k->DWEACC = DWEACC; k->YP = YP;
    k->WhT = WhT; k->GT = GT; k->WdT = WdT; k->WcT = WcT; k->WsT = WsT;
  }
  if (x) {
    x->WX = WX; x->WXT = WXT; x->WXD = WXD; x->WDC = WDC; x->KX = KX; x->KD = KD; x->BKD = BKD; x->DE = DE;
    x->DCS = DC; x->VBAR = VBAR; x->XWHT = XWHT; x->XZRT = XZRT; x->XWST = XWST;
    x->PWDYT = PWDYT; x->PWDCT = PWDCT; x->PWCT = PWCT; x->PWXDT = PWXDT; x->WDCT = WDCT;
    x->gS = xgS; x->gWS = xgWS; x->gPM = xgPM; x->gPL = xgPL; x->gPC = xgPC; x->gC = xgC; x->gQ = xgQ;
    x->gDGZ = xgDGZ; x->gDGR = xgDGR; x->gDGH = xgDGH; x->gDC = xgDC; x->gPDWS = xgPDWS; x->gDWS = xgDWS;
    x->fcensus = fcensus; x->bcensus = bcensus;
    x->sS = xsS; x->sQ = xsQ; x->sC = xsC; x->sWS = xsWS;
    x->sDGZ = xsDGZ; x->sDGR = xsDGR; x->sDGH = xsDGH; x->sDC = xsDC; x->sDWS = xsDWS;
  }
  if (y) {
    y->S = d.S; y->hk = (int)HK; y->pl = HK ? (HK % 2 ? (int)(HK - 1) / 2 : (int)HK / 2) : 0;
    y->WG = lWG; y->WXG = lWXG; y->WSP = lWSP; y->WUT = lWUT; y->WXGT = lWXGT; y->WSTP = lWSTP; y->WXD4 = lWXD4;
    y->BQ = lBQ; y->KXG = lKXG; y->sS = lsS; y->gS = lgS; y->gE = lgE; y->gA = lgA;
    for (int q = 0; q < 4; ++q) { y->sDG[q] = lsDG[q]; y->gDG[q] = lgDG[q]; }
    for (int q = 0; q < 2; ++q) { y->sDC[q] = lsDC[q]; y->gDC[q] = lgDC[q]; }
    y->sDWS = lsDWS; y->gDWS = lgDWS; y->gQA = lgQA; y->PDG = lPDG;
  }
  if (k && scratch) {  // headers behind the GEMM slabs (attn_scratch_bytes)
    const size_t hoff = ((std::max(f.off + 256, g.off + 256) + 255) & ~size_t(255)) + sizeof(float) * kGemmWsFloats;
    k->fhdr = scratch + hoff;
    k->bhdr = scratch + hoff + 256;
  }
  return Layout{sv.off + 256, f.off + 256, g.off + 256};
}

__device__ __forceinline__ int brow(int b0, int lane, int B) { return min(b0 + (lane & 15), B - 1); }
// frames / labels of utterance b in a variable-length batch
__device__ __forceinline__ int frames_of(const AttnK& k, int b) { return k.flen ? k.flen[b] : k.L; }
__device__ __forceinline__ int labels_of(const AttnK& k, int b) { return k.tlen ? k.tlen[b] : k.T; }

// ------------------------------------------------------------------ forward step kernels

// ---- hybrid location-aware attention (Attention.lua:75-98), per-step path only
// F = TemporalConvolution(1, nF, kW)(pad(alpha_{t-1})) with bias, UF = TCZB(nF, Sc, 1)(F): both are
// linear in alpha_{t-1}, so UF_{l,j} = HCU_j + sum_i HG_{j,i} alpha_{t-1}[l + i - pad_left] with
// HG = U W (Sc x kW) and HCU = U b, folded once per call (dec_hyb_fold).
__device__ __forceinline__ int hyb_pad_left(int kw) { return kw % 2 ? (kw - 1) / 2 : kw / 2; }

__global__ void dec_hyb_fold(AttnK k) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= k.Sc) return;
  const int nf = k.hf, kw = k.hk;
  const float* u = k.P.hybU + (long)j * nf;
  for (int i = 0; i < kw; ++i) {
    float s = 0.f;
    for (int f = 0; f < nf; ++f) s += u[f] * k.P.hybW[f * kw + i];
    k.HGT[(long)i * k.Sc + j] = s;
  }
  float c = 0.f;
  for (int f = 0; f < nf; ++f) c += u[f] * k.P.hybb[f];
  k.HCU[j] = c;
}

// alpha_{t-1} of frames ch*LC - pad_left .. ch*LC + LC - 1 + (kW - 1 - pad_left) into apl (0 outside [0, L) and
// at t = 0): apl[lloc + i] is the tap-i input of chunk frame lloc.  All threads call it; ends on a barrier.
__device__ __forceinline__ void hyb_stage_alpha(const AttnK& k, const float* ap, int ch, float* apl) {
  const int pl = hyb_pad_left(k.hk), n = LC + k.hk - 1;
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    const int m = ch * LC + i - pl;
    apl[i] = (ap && m >= 0 && m < k.L) ? ap[m] : 0.f;
  }
  __syncthreads();
}
// UF of chunk frame lloc for the 4 score columns of float4 c4 (UF_{l,j} = HCU_j + sum_i HG_{j,i} apl[lloc + i]);
// apl = the staged alpha_{t-1} halo, hg = the taps HGT ([kW][Sc], global or staged in LDS)
__device__ __forceinline__ float4 hyb_uf4_lds(const AttnK& k, int c4, const float* apl, const float* hg, int lloc) {
  float4 u = reinterpret_cast<const float4*>(k.HCU)[c4];
  for (int i = 0; i < k.hk; ++i) {
    const float a = apl[lloc + i];
    const float4 g = reinterpret_cast<const float4*>(hg + (long)i * k.Sc)[c4];
    u.x += g.x * a; u.y += g.y * a; u.z += g.z * a; u.w += g.w * a;
  }
  return u;
}

// d alpha_t[l] from the hybrid features of step t + 1: sum_i q_{t+1}[l - i + pad_left][i]
__device__ __forceinline__ float hyb_carry(const AttnK& k, int b, int l) {
  if (k.t + 1 >= k.T) return 0.f;
  const int kw = k.hk, pl = hyb_pad_left(kw);
  const float* q = k.QA + ((long)((k.t + 1) & 1) * k.B + b) * k.L * kw;
  float s = 0.f;
  for (int i = 0; i < kw; ++i) {
    const int lp = l - i + pl;
    if (lp >= 0 && lp < k.L) s += q[(long)lp * kw + i];
  }
  return s;
}

// weight gradients of the hybrid features from DGT = sum dG^T (kW x Sc) and DCU = sum dws (Sc):
// G = U W, cu = U b  ->  dU = dG W^T + dcu b^T, dW = U^T dG, db = U^T dcu
// one wave per output element: the dW / db sums run over Sc across the lanes (a thread-serial loop over Sc put ~160
// dependent L2 loads behind each of those outputs: 33 us at the conv + BiLSTM model's Sc = 160)
__global__ __launch_bounds__(256) void dec_hyb_wgrad(AttnK k, AttnGrads G, float scale) {
  const int nf = k.hf, kw = k.hk, Sc = k.Sc, lane = threadIdx.x & 63;
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (idx < Sc * nf) {
    const int j = idx / nf, f = idx % nf;
    if (lane == 0) {
      float v = 0.f;
      for (int i = 0; i < kw; ++i) v += k.DGT[(long)i * Sc + j] * k.P.hybW[f * kw + i];
      v += k.DCU[j] * k.P.hybb[f];
      G.hybU[idx] += scale * v;
    }
  } else if (idx < Sc * nf + nf * kw) {
    const int r = idx - Sc * nf, f = r / kw, i = r % kw;
    float v = 0.f;
    for (int j = lane; j < Sc; j += 64) v += k.P.hybU[(long)j * nf + f] * k.DGT[(long)i * Sc + j];
    v = wave_sum(v);
    if (lane == 0) G.hybW[r] += scale * v;
  } else if (idx < Sc * nf + nf * kw + nf) {
    const int f = idx - Sc * nf - nf * kw;
    float v = 0.f;
    for (int j = lane; j < Sc; j += 64) v += k.P.hybU[(long)j * nf + f] * k.DCU[j];
    v = wave_sum(v);
    if (lane == 0) G.hybb[f] += scale * v;
  }
}

// F1: ws[b] = Ws s_{t-1}[b] + bs  (N = Sc, K = S)
__global__ __launch_bounds__(256) void dec_f1_ws(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (t > 0)
    acc = skinny_wave(k.HX + ((long)brow(b0, lane, k.B) * k.T + t) * 2 * S, k.P.Ws + (long)(n0 + (lane & 15)) * S,
                      S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b < k.B) k.WS[((long)b * k.T + t) * k.Sc + n] = s + k.P.bs[n];
}

// F2: scores + chunk-local softmax stats + partial context.  grid (NCH, B)
// WV waves per workgroup (LC / WV frames each): every frame's score is one wave's, so the wave count does not
// change a bit of the results; the training loop runs 8 (half the serial frame chain of 4 x 4)
template <int WV>
__global__ __launch_bounds__(64 * WV) void dec_f2_attn(AttnK k) {
  constexpr int FPW = LC / WV, NT = 64 * WV;
  __shared__ float sc[LC];
  __shared__ float pw[LC];
  __shared__ float apl[LC + kMaxHybK];  // hybrid: alpha_{t-1} halo of the chunk (hyb_stage_alpha)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = blockIdx.x, b = blockIdx.y, t = k.t;
  const int L = k.L, Sc = k.Sc, A = k.A;
  const float* ws = k.WS + ((long)b * k.T + t) * Sc;
  const float* we = k.P.we;
  const float* ap = (k.hf > 0 && t > 0) ? k.ALPHA + ((long)b * k.T + t - 1) * L : nullptr;  // alpha_{t-1}
  if (k.hf > 0) hyb_stage_alpha(k, ap, ch, apl);
  const int Lb = frames_of(k, b);
  for (int i = 0; i < FPW; ++i) {
    const int li = wave * FPW + i, l = ch * LC + li;
    float part = 0.f;
    if (l < Lb) {
      const float* vh = k.Vh + ((long)b * L + l) * Sc;
      for (int c4 = lane; c4 < Sc / 4; c4 += 64) {
        float4 v = reinterpret_cast<const float4*>(vh)[c4];
        const float4 w = reinterpret_cast<const float4*>(ws)[c4];
        const float4 e = reinterpret_cast<const float4*>(we)[c4];
        float4 z = make_float4(w.x + v.x, w.y + v.y, w.z + v.z, w.w + v.w);
        if (k.hf > 0) {  // Z = Ws + Vh + UF (Attention.lua:95)
          const float4 u = hyb_uf4_lds(k, c4, apl, k.HGT, li);
          z.x += u.x; z.y += u.y; z.z += u.z; z.w += u.w;
        }
        part += e.x * tanhf(z.x) + e.y * tanhf(z.y) + e.z * tanhf(z.z) + e.w * tanhf(z.w);
      }
    }
    part = wave_sum(part);
    if (lane == 0) sc[li] = l < Lb ? part : -INFINITY;
  }
  __syncthreads();
  float m = -INFINITY;
  for (int i = 0; i < LC; ++i) m = fmaxf(m, sc[i]);
  if (tid < LC) {
    const int l = ch * LC + tid;
    const float p = l < Lb ? expf(sc[tid] - m) : 0.f;
    pw[tid] = p;
    if (l < L) k.E[((long)b * k.T + t) * L + l] = sc[tid];
  }
  __syncthreads();
  if (tid == 0) {
    float s = 0.f;
    for (int i = 0; i < LC; ++i) s += pw[i];
    k.PM[b * k.NCH + ch] = m;
    k.PL[b * k.NCH + ch] = s;
  }
  float* pc = k.PC + ((long)b * k.NCH + ch) * A;
  const int lend = min(LC, L - ch * LC);
  for (int a4 = tid; a4 < A / 4; a4 += NT) {
    // every frame's row load in flight before the first add; the sum runs in frame order (as before)
    float4 hv[LC];
#pragma unroll
    for (int i = 0; i < LC; ++i)
      hv[i] = i < lend ? reinterpret_cast<const float4*>(k.h + ((long)b * L + ch * LC + i) * A)[a4]
                       : make_float4(0.f, 0.f, 0.f, 0.f);
    float4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < LC; ++i) {
      if (i < lend) {
        const float p = pw[i];
        acc.x += p * hv[i].x; acc.y += p * hv[i].y; acc.z += p * hv[i].z; acc.w += p * hv[i].w;
      }
    }
    reinterpret_cast<float4*>(pc)[a4] = acc;
  }
}

// F3: combine chunks (grid B): lse, alpha, c, MonoAlign indicator
__global__ __launch_bounds__(256) void dec_f3_combine(AttnK k) {
  __shared__ float wj[64];
  __shared__ float red[4];
  __shared__ float stat[2];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, b = blockIdx.x, t = k.t;
  const int L = k.L, A = k.A, S = k.S, NCH = k.NCH;
  const long row = (long)b * k.T + t;
  if (tid == 0) {
    float m = -INFINITY;
    for (int j = 0; j < NCH; ++j) m = fmaxf(m, k.PM[b * NCH + j]);
    float den = 0.f;
    for (int j = 0; j < NCH; ++j) {
      const float w = expf(k.PM[b * NCH + j] - m);
      if (j < 64) wj[j] = w;
      den += w * k.PL[b * NCH + j];
    }
    stat[0] = m;
    stat[1] = den;
    k.LSE[row] = m + logf(den);
  }
  __syncthreads();
  const float m = stat[0], inv = 1.0f / stat[1];
  // context c = sum_j w_j pc_j / den  -> C and the MLP input VV[:, S:]
  for (int a = tid; a < A; a += 256) {
    float acc = 0.f;
    for (int j = 0; j < NCH; ++j) {
      const float w = j < 64 ? wj[j] : expf(k.PM[b * NCH + j] - m);
      acc += w * k.PC[((long)b * NCH + j) * A + a];
    }
    const float c = acc * inv;
    k.C[row * A + a] = c;
    k.VV[row * (S + A) + S + a] = c;
  }
  // alpha_l = exp(e_l - lse) and sum_l (L - l)(alpha_l - alpha_prev_l)   (MonotonicAlignment.lua:27-35)
  const float lse = m + logf(stat[1]);
  const int Lb = frames_of(k, b);
  float diff = 0.f;
  for (int l = tid; l < L; l += 256) {
    const float a = expf(k.E[row * L + l] - lse);  // 0 on padding frames (E = -inf)
    k.ALPHA[row * L + l] = a;
    const float ap = t > 0 ? k.ALPHA[(row - 1) * L + l] : 0.f;  // alpha_{t-1} (written by step t-1)
    diff += (float)(Lb - l) * (a - ap);
  }
  diff = wave_sum(diff);
  if (lane == 0) red[wave] = diff;
  __syncthreads();
  if (tid == 0) {
    const float d = ((red[0] + red[1]) + red[2]) + red[3];
    const float pen = k.penalty * fmaxf(d, 0.f);
    k.IND[row] = (pen > 0.f && t < labels_of(k, b)) ? 1.f : 0.f;
  }
}

// F4: c_in = Wc c + bc (N = S, K = A); y_in = Wy[:, y_{t-1}] + by   -> CY = [c_in | y_in]
__global__ __launch_bounds__(256) void dec_f4_cin(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S, A = k.A;
  floatx4 acc = skinny_wave(k.C + ((long)brow(b0, lane, k.B) * k.T + t) * A, k.P.Wc + (long)(n0 + (lane & 15)) * A,
                            A, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  k.CY[row * 2 * S + n] = s + k.P.bc[n];
  float yin = k.P.by[n];
  // y_{t-1} one-hot (teacher forcing, RNNAttention.lua:172-176); a negative label = zeros_y (beam search's
  // first step, Attention.lua:359)
  if (t > 0 && k.labels[(long)b * k.T + t - 1] >= 0) yin += k.P.Wy[(long)n * k.O + k.labels[(long)b * k.T + t - 1]];
  k.CY[row * 2 * S + S + n] = yin;
}

// F5: d = Wd [c_in; y_in] + bd (N = S, K = 2S) -> HX[:, S:] and RHX[:, S:]
__global__ __launch_bounds__(256) void dec_f5_d(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave(k.CY + ((long)brow(b0, lane, k.B) * k.T + t) * 2 * S,
                            k.P.Wd + (long)(n0 + (lane & 15)) * 2 * S, 2 * S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  const float d = s + k.P.bd[n];
  k.HX[row * 2 * S + S + n] = d;
  k.RHX[row * 2 * S + S + n] = d;
}

// ---- folded F4 + F5 of the per-step path (LSTM decoder / hybrid attention: the shapes the XCD-local kernels do
// not serve).  d = Wd [Wc c + bc; y_in] + bd = WDC c + KD with WDC = Wd_c Wc (S x A) and KD = Wd_y y_in + Wd_c bc
// + bd per row (teacher-forced y_in), both formed before the loop -- one launch per step instead of two.
// y_in rows of every step: CY[:, S:] = by + Wy[:, y_{t-1}] (zeros_y at t = 0 or a negative label)
__global__ void dec_fold_yin(AttnK k) {
  const int S = k.S;
  const long n = (long)k.B * k.T * S;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / S;
    const int j = (int)(i - row * S), t = (int)(row % k.T);
    float v = k.P.by[j];
    if (t > 0 && k.labels[row - 1] >= 0) v += k.P.Wy[(long)j * k.O + k.labels[row - 1]];
    k.CY[row * 2 * S + S + j] = v;
  }
}
// F45: d = WDC c_t + KD_t (N = S, K = A) -> HX[:, S:] and RHX[:, S:]
__global__ __launch_bounds__(512) void dec_f45_fold(AttnK k, const float* __restrict__ wdc, const float* __restrict__ kd) {
  __shared__ SkinnyRed8 red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S, A = k.A;
  floatx4 acc = skinny_wave8(k.C + ((long)brow(b0, lane, k.B) * k.T + t) * A, wdc + (long)(n0 + (lane & 15)) * A, A,
                            wave, lane);
  const float s = skinny_reduce8(red, acc, wave, lane, tid);
  if (tid >= 256) return;
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  const float d = s + kd[row * S + n];
  k.HX[row * 2 * S + S + n] = d;
  k.RHX[row * 2 * S + S + n] = d;
}

// F6: [z|r] = sig(W{z,r} [s_{t-1}; d])  (N = 2S, K = 2S)
__global__ __launch_bounds__(256) void dec_f6_gru1(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  const float* W = n0 < S ? k.P.Wz + (long)n0 * 2 * S : k.P.Wr + (long)(n0 - S) * 2 * S;
  floatx4 acc = skinny_wave(k.HX + ((long)brow(b0, lane, k.B) * k.T + t) * 2 * S, W + (long)(lane & 15) * 2 * S,
                            2 * S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  const float g = sigmoidf_(s);
  if (n < S) {
    k.GSV[row * 3 * S + n] = g;
  } else {
    const int j = n - S;
    k.GSV[row * 3 * S + S + j] = g;
    k.RHX[row * 2 * S + j] = g * k.HX[row * 2 * S + j];
  }
}

// F7: hh = tanh(Wh [r*s; d]); s_t = (1-z) s_{t-1} + z hh  (N = S, K = 2S)
__global__ __launch_bounds__(256) void dec_f7_gru2(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave(k.RHX + ((long)brow(b0, lane, k.B) * k.T + t) * 2 * S,
                            k.P.Wh + (long)(n0 + (lane & 15)) * 2 * S, 2 * S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  const float hh = tanhf(s);
  const float z = k.GSV[row * 3 * S + n], sp = k.HX[row * 2 * S + n];
  k.GSV[row * 3 * S + 2 * S + n] = hh;
  const float snew = (-z + 1.0f) * sp + z * hh;
  k.VV[row * (S + k.A) + n] = snew;
  if (t + 1 < k.T) k.HX[(row + 1) * 2 * S + n] = snew;
}

// ---- decoder LSTM (LSTM.lua:16-58 as decoder_recurrent, timit/timit.lua:137): s = h, mem = c
// LW rows interleave the four gates of each unit: row 4 u + q = [Wqh[u] | Wqx[u]] (q = i, f, g, o) against HX rows
// [s_{t-1} | d]; LB[4 u + q] = bqx + bqh.  (GT, the backward's LW^T, keeps the gate-major column order q S + u of
// the gate gradients: dec_lstm_gt.)
__global__ void dec_lstm_pack(AttnK k) {
  const int S = k.S;
  const long n = 4L * S * 2 * S;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int r = (int)(i / (2 * S)), c = (int)(i - (long)r * 2 * S), u = r >> 2, q = r & 3;
    k.LW[i] = c < S ? k.P.lstm[4 * q + 2][(long)u * S + c] : k.P.lstm[4 * q][(long)u * S + c - S];
    if (c == 0) k.LB[r] = k.P.lstm[4 * q + 1][u] + k.P.lstm[4 * q + 3][u];
  }
}
// GT (2S, 4S) = LW^T with the gate-major column order of the gate gradients: GT[n][q S + u] = LW[4 u + q][n]
__global__ void dec_lstm_gt(AttnK k) {
  const int S = k.S;
  const long n = 2L * S * 4 * S;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int c = (int)(i / (4 * S)), j = (int)(i - (long)c * 4 * S), q = j / S, u = j - q * S;
    k.GT[i] = k.LW[(long)(4 * u + q) * 2 * S + c];
  }
}

// F6 + F7 (LSTM), one launch per step: the block's 16 output rows are the four gates of four units (LW's
// interleaved rows), gate = act(LW[4u+q] . [s_{t-1}; d] + LB) (N = 4S, K = 2S; act = sigmoid, g: tanh), then
// the unit's four gates meet in four adjacent lanes and the lane of gate i updates the cell: c = f c_{t-1} + i g,
// s = o tanh(c).  (The cell update used to be its own launch per decoder step.)
__global__ __launch_bounds__(512) void dec_f6_lstm(AttnK k) {
  __shared__ SkinnyRed8 red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave8(k.HX + ((long)brow(b0, lane, k.B) * k.T + t) * 2 * S,
                            k.LW + (long)(n0 + (lane & 15)) * 2 * S, 2 * S, wave, lane);
  const float s = skinny_reduce8(red, acc, wave, lane, tid);
  if (tid >= 256) return;
  const int b = b0 + (tid >> 4), r = n0 + (tid & 15), u = r >> 2, q = r & 3;
  if (b >= k.B) return;  // (uniform over each group of four lanes: one row)
  const long row = (long)b * k.T + t;
  const float x = s + k.LB[r];
  const float gv = q == 2 ? tanhf(x) : sigmoidf_(x);
  k.GSV[row * 4 * S + q * S + u] = gv;
  const int l0 = lane & ~3;
  const float gi = __shfl(gv, l0, 64), gf = __shfl(gv, l0 + 1, 64), gg = __shfl(gv, l0 + 2, 64),
              go = __shfl(gv, l0 + 3, 64);
  if (q != 0) return;
  const float cp = t > 0 ? k.LC[(row - 1) * S + u] : 0.f;
  const float c = gf * cp + gi * gg;
  const float snew = go * tanhf(c);
  k.LC[row * S + u] = c;
  k.VV[row * (S + k.A) + u] = snew;
  if (t + 1 < k.T) k.HX[(row + 1) * 2 * S + u] = snew;
}

__global__ void dec_init_fwd(AttnK k) {
  // s_0 = 0 (Recurrent.lua:112 zeros_hidden)
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < k.B * k.S) {
    const int b = i / k.S, n = i - b * k.S;
    k.HX[((long)b * k.T) * 2 * k.S + n] = 0.f;
  }
}

// MLP head (per row b*T+t, one wave each): maxout (first max wins), Linear(M,O), LogSoftMax; with k.dlogp set (the
// seed is final before the forward, AttnDims::dlogp_early) also its backward, dec_mlp_head_bwd's per-row work with
// the same sums: do = dlogp - exp(logp) sum(dlogp), dm = Wo^T do, dU = scatter(dm, argmax).  LDS: 4 M (+ 4 O) floats
__device__ __forceinline__ void mlp_head_body(const AttnK& k, int rows, int blk) {
  extern __shared__ float sm[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = blk * 4 + wave;
  const int M = k.M, Kw = k.K, O = k.O;
  float* mv = sm + wave * M;
  const bool live = r < rows;
  if (live) {
    const float* u = k.U + (long)r * M * Kw;
    // U[r][c] from the MLP GEMM's slabs when it left them unreduced: splitk_reduce's expression (alpha = 1)
    auto uv = [&](int c) -> float {
      if (!k.UP) return u[c];
      const long e = (long)r * M * Kw + c;
      float sum = 0.f;
      for (int s = 0; s < k.UPS; ++s) sum += k.UP[s * k.UPMN + e];
      return 1.f * sum + k.P.bm[c];
    };
    for (int j = lane; j < M; j += 64) {
      float best = uv(j * Kw);
      int bi = 0;
      for (int i = 1; i < Kw; ++i) {
        const float v = uv(j * Kw + i);
        if (v > best) { best = v; bi = i; }
      }
      mv[j] = best;
      k.MM[(long)r * M + j] = best;
      k.AM[(long)r * M + j] = bi;
    }
  }
  __syncthreads();
  if (live) {
    float mx = -INFINITY;
    for (int n = lane; n < O; n += 64) {
      float o = k.P.bo[n];
      const float* w = k.P.Wo + (long)n * M;
      for (int j = 0; j < M; ++j) o += w[j] * mv[j];
      k.LOGP[(long)r * O + n] = o;
      mx = fmaxf(mx, o);
    }
    mx = wave_max(mx);
    float se = 0.f;
    for (int n = lane; n < O; n += 64) se += expf(k.LOGP[(long)r * O + n] - mx);
    se = wave_sum(se);
    const float lz = mx + logf(se);
    for (int n = lane; n < O; n += 64) {
      const float v = k.LOGP[(long)r * O + n] - lz;
      k.LOGP[(long)r * O + n] = v;
      if (k.logp) k.logp[(long)r * O + n] = v;
    }
  }
  if (!k.dlogp) return;
  float* dov = sm + 4 * M + wave * O;
  float sd = 0.f;
  if (live)
    for (int n = lane; n < O; n += 64) sd += k.dlogp[(long)r * O + n];
  sd = wave_sum(sd);
  if (live)
    for (int n = lane; n < O; n += 64) {
      const float v = k.dlogp[(long)r * O + n] - expf(k.LOGP[(long)r * O + n]) * sd;
      dov[n] = v;
      k.DO[(long)r * O + n] = v;
    }
  __syncthreads();
  if (!live) return;
  float* du = k.DU + (long)r * M * Kw;
  for (int j = lane; j < M; j += 64) {
    float dm = 0.f;
    for (int n = 0; n < O; ++n) dm += k.P.Wo[(long)n * M + j] * dov[n];
    const int am = k.AM[(long)r * M + j];
    for (int i = 0; i < Kw; ++i) du[j * Kw + i] = i == am ? dm : 0.f;
  }
}
__global__ __launch_bounds__(256) void dec_mlp_head(AttnK k, int rows) { mlp_head_body(k, rows, blockIdx.x); }

// ------------------------------------------------------------------ backward kernels

// per row: do = dlogp - exp(logp) sum(dlogp) (LogSoftMax bwd); dm = Wo^T do; du = scatter(dm, argmax)
__global__ __launch_bounds__(256) void dec_mlp_head_bwd(AttnK k, int rows) {
  extern __shared__ float sm[];  // 4 * O
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = blockIdx.x * 4 + wave;
  const int M = k.M, Kw = k.K, O = k.O;
  float* dov = sm + wave * O;
  float sd = 0.f;
  if (r < rows)
    for (int n = lane; n < O; n += 64) sd += k.dlogp[(long)r * O + n];
  sd = wave_sum(sd);
  if (r < rows)
    for (int n = lane; n < O; n += 64) {
      const float v = k.dlogp[(long)r * O + n] - expf(k.LOGP[(long)r * O + n]) * sd;
      dov[n] = v;
      k.DO[(long)r * O + n] = v;
    }
  __syncthreads();
  if (r >= rows) return;
  float* du = k.DU + (long)r * M * Kw;
  for (int j = lane; j < M; j += 64) {
    float dm = 0.f;
    for (int n = 0; n < O; ++n) dm += k.P.Wo[(long)n * M + j] * dov[n];
    const int am = k.AM[(long)r * M + j];
    for (int i = 0; i < Kw; ++i) du[j * Kw + i] = i == am ? dm : 0.f;
  }
}

__device__ __forceinline__ void dec_gate_grads(const AttnK& k, int b, int t, int n, float ds) {
  const int S = k.S;
  const long row = (long)b * k.T + t;
  const float z = k.GSV[row * 3 * S + n], hh = k.GSV[row * 3 * S + 2 * S + n], sp = k.HX[row * 2 * S + n];
  k.DS[b * S + n] = ds;
  k.DGA[row * 3 * S + n] = ds * (hh - sp) * (z * (1.0f - z));
  k.DGA[row * 3 * S + 2 * S + n] = (ds * z) * (1.0f - hh * hh);
}

// LSTM gate grads of step t from ds = dL/ds_t and the cell carry dcar = dL/dc_t from step t+1
// (LSTM.lua:118-136 under RNNAttention's BPTT); leaves dL/dc_{t-1} in DSP
__device__ __forceinline__ void dec_lstm_gate_grads(const AttnK& k, int b, int t, int n, float ds, float dcar) {
  const int S = k.S;
  const long row = (long)b * k.T + t;
  const float* g = k.GSV + row * 4 * S;
  const float gi = g[n], gf = g[S + n], gg = g[2 * S + n], go = g[3 * S + n];
  const float c = k.LC[row * S + n], cp = t > 0 ? k.LC[(row - 1) * S + n] : 0.f;
  const float tc = tanhf(c);
  const float dc = dcar + ds * go * (1.0f - tc * tc);
  float* dga = k.DGA + row * 4 * S;
  dga[n] = dc * gg * (gi * (1.0f - gi));
  dga[S + n] = dc * cp * (gf * (1.0f - gf));
  dga[2 * S + n] = dc * gi * (1.0f - gg * gg);
  dga[3 * S + n] = ds * tc * (go * (1.0f - go));
  k.DSP[b * S + n] = dc * gf;
}

__global__ void dec_bwd_init(AttnK k) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= k.B * k.S) return;
  const int b = i / k.S, n = i - b * k.S, t = k.T - 1;
  if (k.lstm) dec_lstm_gate_grads(k, b, t, n, k.DV[((long)b * k.T + t) * (k.S + k.A) + n], 0.f);
  else dec_gate_grads(k, b, t, n, k.DV[((long)b * k.T + t) * (k.S + k.A) + n]);
}

// K3 (LSTM): [ds_prev | dd] = LW^T dGA  (N = 2S, K = 4S; GT = LW^T)
__global__ __launch_bounds__(512) void dec_b3_lstm(AttnK k) {
  __shared__ SkinnyRed8 red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave8(k.DGA + ((long)brow(b0, lane, k.B) * k.T + t) * 4 * S,
                            k.GT + (long)(n0 + (lane & 15)) * 4 * S, 4 * S, wave, lane);
  const float s = skinny_reduce8(red, acc, wave, lane, tid);
  if (tid >= 256) return;
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  if (n < S) k.DSPF[b * S + n] = s;
  else k.DD[((long)b * k.T + t) * S + n - S] = s;
}

// K2: dq = Wh[:, :S]^T da_h (N = S, K = S) -> da_r, DSP = ds(1-z) + dq r
__global__ __launch_bounds__(256) void dec_b2_gru1(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave(k.DGA + ((long)brow(b0, lane, k.B) * k.T + t) * 3 * S + 2 * S,
                            k.WhT + (long)(n0 + (lane & 15)) * S, S, wave, lane);
  const float dq = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  const float z = k.GSV[row * 3 * S + n], r = k.GSV[row * 3 * S + S + n], sp = k.HX[row * 2 * S + n];
  k.DGA[row * 3 * S + S + n] = (dq * sp) * (r * (1.0f - r));
  k.DSP[b * S + n] = k.DS[b * S + n] * (-z + 1.0f) + dq * r;
}

// K3: [ds_prev | dd] = GT [da_z; da_r; da_h]  (N = 2S, K = 3S)
__global__ __launch_bounds__(256) void dec_b3_gru2(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave(k.DGA + ((long)brow(b0, lane, k.B) * k.T + t) * 3 * S,
                            k.GT + (long)(n0 + (lane & 15)) * 3 * S, 3 * S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  if (n < S) k.DSPF[b * S + n] = k.DSP[b * S + n] + s;
  else k.DD[((long)b * k.T + t) * S + n - S] = s;
}

// K4: [dc_in | dy_in] = Wd^T dd  (N = 2S, K = S)
__global__ __launch_bounds__(256) void dec_b4_wd(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave(k.DD + ((long)brow(b0, lane, k.B) * k.T + t) * S, k.WdT + (long)(n0 + (lane & 15)) * S,
                            S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b < k.B) k.DCY[((long)b * k.T + t) * 2 * S + n] = s;
}

// K5: dc = dv_c + Wc^T dc_in  (N = A, K = S)
__global__ __launch_bounds__(256) void dec_b5_wc(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave(k.DCY + ((long)brow(b0, lane, k.B) * k.T + t) * 2 * S,
                            k.WcT + (long)(n0 + (lane & 15)) * S, S, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  k.DC[row * k.A + n] = k.DV[row * (S + k.A) + S + n] + s;
}

// K45 (folded, the per-step path's LSTM / hybrid shapes): dc = dv_c + WDC^T dd (N = A, K = S; wdct = WDC^T);
// DCY = dd Wd for the weight gradients is one GEMM after the loop
__global__ __launch_bounds__(512) void dec_b45_fold(AttnK k, const float* __restrict__ wdct) {
  __shared__ SkinnyRed8 red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  floatx4 acc = skinny_wave8(k.DD + ((long)brow(b0, lane, k.B) * k.T + t) * S, wdct + (long)(n0 + (lane & 15)) * S, S,
                            wave, lane);
  const float s = skinny_reduce8(red, acc, wave, lane, tid);
  if (tid >= 256) return;
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B) return;
  const long row = (long)b * k.T + t;
  k.DC[row * k.A + n] = k.DV[row * (S + k.A) + S + n] + s;
}

// K6: fused attention backward for one 16-frame chunk.  grid (NCH, B)
//   d alpha_l = dc . h_l + carry_l + gdiff_l      (MM bwd + MonotonicAlignment.lua:44-77)
//   de_l = alpha_l (d alpha_l - sum_j alpha_j d alpha_j)   with sum = dc . c + sum alpha (carry + gdiff)
//   dZ = de_l we (1 - tanh^2);  dVh_l += dZ;  partial dws, dwe  (dh_l = sum_t alpha_{t,l} dc_t is one GEMM per
//   utterance after the loop, attn_dh_gemms: a read-modify-write of dh per frame and step cost 5.3 us of 28)
//   HYB (hybrid attention): Z includes UF; d alpha_l also gets the carry from step t+1's location
//   features (hyb_carry); q_{l,i} = sum_j dZ_lj HG_ji -> QA for step t-1; dG partials -> PDG
//   HYB keeps this chunk's dZ rows in LDS (dynamic, LC x Sc floats) and forms q and the dG partials from them
//   after the frame loop: per-lane register partials over every tap (kMaxHybK x 16 floats) spilled to scratch
//   at one wave per SIMD (37.7 us per step at the conv + BiLSTM model's B = 32, Sc = 160; tools/ab_convlstm.py)
template <bool HYB>
__global__ __launch_bounds__(HYB ? 512 : 256) void dec_b6_attn(AttnK k) {
  // HYB: 8 waves x 2 frames (the content-attention form keeps 4 x 4: it is bitwise equal to the persistent
  // kernels of attn_persist.inc, and the wave count sets the order of the cross-wave sums)
  constexpr int WV = HYB ? 8 : 4, FPW = LC / WV, NT = 64 * WV;
  __shared__ float redv[WV];
  __shared__ float pws[WV][1024];
  extern __shared__ float zl[];  // HYB: [LC][Sc] dZ rows of this chunk, then HGT [kW][Sc], then the alpha halo
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = blockIdx.x, b = blockIdx.y, t = k.t;
  const int L = k.L, A = k.A, Sc = k.Sc, T = k.T;
  const long row = (long)b * T + t;
  const float* dc = k.DC + row * A;
  const float* c = k.C + row * A;
  const float* alpha = k.ALPHA + row * L;
  const float lam = k.penalty;
  const float ind = k.IND[row], indn = t + 1 < T ? k.IND[row + 1] : 0.f;
  const int Lb = frames_of(k, b);  // MonotonicAlignment's L (alpha = 0 past it)
  // sum_j alpha_j d alpha_j
  float part = 0.f;
  for (int a = tid; a < A; a += NT) part += dc[a] * c[a];
  for (int l = tid; l < L; l += NT)
    part += alpha[l] * (HYB ? lam * (float)(Lb - l) * (ind - indn) + hyb_carry(k, b, l)
                            : lam * (float)(Lb - l) * (ind - indn));
  part = wave_sum(part);
  if (lane == 0) redv[wave] = part;
  __syncthreads();
  float ssum = redv[0];
#pragma unroll
  for (int w = 1; w < WV; ++w) ssum += redv[w];
  const float* ws = k.WS + row * Sc;
  const float* we = k.P.we;
  // Sc <= 1024 asserted on the host: each lane owns k = 4*(lane + 64 i)
  float dwsp[16], dwep[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) { dwsp[i] = 0.f; dwep[i] = 0.f; }
  const float* ap = (HYB && t > 0) ? k.ALPHA + (row - 1) * L : nullptr;  // alpha_{t-1}
  const int lend = min(LC, L - ch * LC);  // frames of this chunk
  float* hg = zl + (long)LC * Sc;         // HYB: the taps HGT, staged
  float* apl = hg + (long)k.hk * Sc;      // HYB: alpha_{t-1} halo of the chunk
  if (HYB) {
    for (int i = tid; i < k.hk * Sc; i += NT) hg[i] = k.HGT[i];
    hyb_stage_alpha(k, ap, ch, apl);
  }
  for (int i4 = 0; i4 < FPW; ++i4) {
    const int lloc = wave * FPW + i4, l = ch * LC + lloc;
    if (l >= L) break;
    const float* hl = k.h + ((long)b * L + l) * A;
    float dd = 0.f;
    for (int a4 = lane; a4 < A / 4; a4 += 64) {
      const float4 hv = reinterpret_cast<const float4*>(hl)[a4];
      const float4 dv = reinterpret_cast<const float4*>(dc)[a4];
      dd += hv.x * dv.x + hv.y * dv.y + hv.z * dv.z + hv.w * dv.w;
    }
    dd = wave_sum(dd);
    const float al = alpha[l];
    const float dal = HYB ? dd + (lam * (float)(Lb - l) * (ind - indn) + hyb_carry(k, b, l))
                          : dd + lam * (float)(Lb - l) * (ind - indn);
    const float de = al * (dal - ssum);
    const float* vh = k.Vh + ((long)b * L + l) * Sc;
    float* dvh = k.DVH + ((long)b * L + l) * Sc;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < Sc / 4) {
        const float4 v = reinterpret_cast<const float4*>(vh)[c4];
        const float4 w = reinterpret_cast<const float4*>(ws)[c4];
        const float4 e = reinterpret_cast<const float4*>(we)[c4];
        float4 o = reinterpret_cast<float4*>(dvh)[c4];
        float4 zz = make_float4(w.x + v.x, w.y + v.y, w.z + v.z, w.w + v.w);
        if (HYB) {
          const float4 u = hyb_uf4_lds(k, c4, apl, hg, lloc);
          zz.x += u.x; zz.y += u.y; zz.z += u.z; zz.w += u.w;
        }
        const float th0 = tanhf(zz.x), th1 = tanhf(zz.y), th2 = tanhf(zz.z), th3 = tanhf(zz.w);
        const float z0 = de * e.x * (1.f - th0 * th0), z1 = de * e.y * (1.f - th1 * th1);
        const float z2 = de * e.z * (1.f - th2 * th2), z3 = de * e.w * (1.f - th3 * th3);
        if (HYB) reinterpret_cast<float4*>(zl + (long)lloc * Sc)[c4] = make_float4(z0, z1, z2, z3);
        o.x += z0; o.y += z1; o.z += z2; o.w += z3;
        reinterpret_cast<float4*>(dvh)[c4] = o;
        dwsp[4 * i] += z0; dwsp[4 * i + 1] += z1; dwsp[4 * i + 2] += z2; dwsp[4 * i + 3] += z3;
        dwep[4 * i] += de * th0; dwep[4 * i + 1] += de * th1; dwep[4 * i + 2] += de * th2; dwep[4 * i + 3] += de * th3;
      }
    }
  }
  // cross-wave sums of the per-wave partials (fixed order), dws then dwe
  float* pd = k.PDWS + ((long)b * k.NCH + ch) * Sc;
  float* pe = k.DWEACC + ((long)b * k.NCH + ch) * Sc;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < Sc / 4) {
        float* dst = &pws[wave][4 * c4];
        const float* src = pass == 0 ? &dwsp[4 * i] : &dwep[4 * i];
        dst[0] = src[0]; dst[1] = src[1]; dst[2] = src[2]; dst[3] = src[3];
      }
    }
    __syncthreads();
    for (int kk = tid; kk < Sc; kk += NT) {
      float v = pws[0][kk];
#pragma unroll
      for (int w = 1; w < WV; ++w) v += pws[w][kk];
      if (pass == 0) pd[kk] = v; else pe[kk] += v;
    }
  }
  if (HYB) {  // (the passes above ended on a barrier after every zl store)
    const int hk = k.hk;
    // q_{l,i} = sum_j dZ_lj HG_ji for d alpha_{t-1} (read by step t-1's kernel through hyb_carry): four threads
    // per (frame, tap) pair, float4 columns c4 = r, r + 4, ... then a 4-lane butterfly (a wave reduction per
    // pair cost 6.5 us of the kernel's 28 at Sc = 160, kW = 5)
    float* qa = k.QA + ((long)(t & 1) * k.B + b) * L * hk + (long)ch * LC * hk;
    for (int p0 = 0; p0 < lend * hk; p0 += NT / 4) {
      const int p = p0 + (tid >> 2), r = tid & 3;
      float q = 0.f;
      if (p < lend * hk) {
        const int lloc = p / hk, ii = p - lloc * hk;
        const float4* z4 = reinterpret_cast<const float4*>(zl + (long)lloc * Sc);
        const float4* g4 = reinterpret_cast<const float4*>(hg + (long)ii * Sc);
        for (int c4 = r; c4 < Sc / 4; c4 += 4) {
          const float4 z = z4[c4], g = g4[c4];
          q += ((z.x * g.x + z.y * g.y) + z.z * g.z) + z.w * g.w;
        }
      }
      q += __shfl_xor(q, 1, 64);
      q += __shfl_xor(q, 2, 64);
      if (p < lend * hk && r == 0) qa[p] = q;
    }
    // dG partials of this chunk, accumulated over the steps (PDG zeroed before the loop): sum_l dZ_lj
    // alpha_{t-1}[l + i - pad_left] (no term at t = 0)
    if (ap) {
      float* pg = k.PDG + ((long)b * k.NCH + ch) * hk * Sc;
      for (int e = tid; e < hk * Sc; e += NT) {
        const int ii = e / Sc, kk = e - ii * Sc;
        float g = 0.f;
        for (int lloc = 0; lloc < lend; ++lloc) g += zl[(long)lloc * Sc + kk] * apl[lloc + ii];
        pg[e] += g;
      }
    }
  }
}

// skinny_wave over the chunk-summed dws row: operand chunk = sum_j PDWS[b][j][k..k+3] in chunk order from 0 (the
// sum dec_b7_dws formed, bitwise); `store` (the workgroups of blockIdx.x == 0) also writes the summed row to DWS
__device__ __forceinline__ float4 dws_chunk(const float* __restrict__ p, int nch, long stride, int off) {
  float4 x = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int j = 0; j < nch; ++j) {
    const float4 v = *reinterpret_cast<const float4*>(p + j * stride + off);
    x.x += v.x; x.y += v.y; x.z += v.z; x.w += v.w;
  }
  return x;
}
__device__ __forceinline__ floatx4 skinny_wave_dws(const float* __restrict__ prow, int nch, float* __restrict__ dws_row,
                                                   bool store, const float* __restrict__ wrow, int K, int wave,
                                                   int lane) {
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int kq = 4 * (lane >> 4);
  int kc = wave * 16;
  for (; kc + 64 < K; kc += 128) {
    const float4 a0 = dws_chunk(prow, nch, K, kc + kq);
    const float4 b0 = *reinterpret_cast<const float4*>(wrow + kc + kq);
    const float4 a1 = dws_chunk(prow, nch, K, kc + 64 + kq);
    const float4 b1 = *reinterpret_cast<const float4*>(wrow + kc + 64 + kq);
    if (store) {
      *reinterpret_cast<float4*>(dws_row + kc + kq) = a0;
      *reinterpret_cast<float4*>(dws_row + kc + 64 + kq) = a1;
    }
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc1, 0, 0, 0);
  }
  for (; kc < K; kc += 64) {
    const float4 a0 = dws_chunk(prow, nch, K, kc + kq);
    const float4 b0 = *reinterpret_cast<const float4*>(wrow + kc + kq);
    if (store) *reinterpret_cast<float4*>(dws_row + kc + kq) = a0;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc0, 0, 0, 0);
  }
  return acc0 + acc1;
}

// K7 + K8: dws_t = sum over the attention chunks' partials (-> DWS, the weight gradients' rows), ds_{t-1} = DSPF +
// Ws^T dws (N = S, K = Sc); then the gate grads of step t-1.  (The chunk sum was its own launch, dec_b7_dws: one
// launch per decoder step fewer.)
__global__ __launch_bounds__(256) void dec_b8_ws(AttnK k) {
  __shared__ SkinnyRed red;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16, t = k.t, S = k.S;
  const int bl = b0 + (lane & 15), br = min(bl, k.B - 1);
  floatx4 acc = skinny_wave_dws(k.PDWS + (long)br * k.NCH * k.Sc, k.NCH, k.DWS + ((long)br * k.T + t) * k.Sc,
                                blockIdx.x == 0 && bl < k.B, k.WsT + (long)(n0 + (lane & 15)) * k.Sc, k.Sc, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= k.B || t == 0) return;
  const float carry = k.DSPF[b * S + n] + s;
  if (k.lstm) dec_lstm_gate_grads(k, b, t - 1, n, k.DV[((long)b * k.T + t - 1) * (S + k.A) + n] + carry,
                                  k.DSP[b * S + n]);
  else dec_gate_grads(k, b, t - 1, n, k.DV[((long)b * k.T + t - 1) * (S + k.A) + n] + carry);
}

// G.lstm[4 q] (Wqx) += LDW[q S + r][S + c], G.lstm[4 q + 2] (Wqh) += LDW[q S + r][c]  (LDW: (4S, 2S) gate-major)
__global__ void lstm_dw_scatter(const float* __restrict__ ldw, int S, AttnGrads G) {
  const long n = 8L * S * S;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const int h = (int)(i / (4L * S * S));  // 0: x half, 1: h half
    const long e = i - h * 4L * S * S;
    const int q = (int)(e / ((long)S * S));
    const long rc = e - (long)q * S * S;
    const int r = (int)(rc / S), c = (int)(rc - (long)r * S);
    const float v = ldw[((long)q * S + r) * 2 * S + (h == 0 ? S + c : c)];
    float* dst = G.lstm[4 * q + (h == 0 ? 0 : 2)] + rc;
    *dst = *dst + v;
  }
}

__global__ void dec_onehot_prev(AttnK k) {
  // YP[b][t] = onehot(y_{t-1}), zeros at t = 0 (RNNAttention.lua:172-176)
  const long n = (long)k.B * k.T * k.O;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long row = i / k.O;
    const int o = (int)(i - row * k.O);
    const int t = (int)(row % k.T);
    k.YP[i] = (t > 0 && k.labels[row - 1] == o) ? 1.f : 0.f;
  }
}

__global__ void fill2d_kernel(float* dst, long ldd, int rows, int cols, float v) {
  const long n = (long)rows * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, c = i - r * cols;
    dst[r * ldd + c] = v;
  }
}

__global__ void nll_seed_kernel(int B, int T, int O, const float* logp, const int* labels, int normalize, float* nll,
                                float* dlogp, const int* tlen) {
  const int b = blockIdx.x;
  __shared__ float red[4];
  const int Tb = tlen ? tlen[b] : T;  // labels of this utterance; later steps are padding
  float s = 0.f;
  for (int i = threadIdx.x; i < T * O; i += blockDim.x) {
    const int t = i / O, o = i - t * O;
    const bool hit = t < Tb && labels[b * T + t] == o;
    if (hit && logp) s += logp[((long)b * T + t) * O + o];
    if (dlogp) dlogp[((long)b * T + t) * O + o] = hit ? -1.f : 0.f;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0 && nll) {
    float v = -(((red[0] + red[1]) + red[2]) + red[3]);
    nll[b] = normalize ? v / (float)Tb : v;
  }
}

// nn.Dropout(p) (Torch7, training mode) on the decoder MLP input [s_t; c_t]
// (timit/model_chorowski_baseline_dropout.lua:56): MASK = injected multipliers, or Bernoulli(1-p)/(1-p)
// from a counter-based hash of (seed, element) -- any launch geometry draws the same mask -- and
// VV *= MASK.  The backward multiplies dVV by the same MASK (dec_dropout_bwd).
__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// one word written on the stream (graph replays read each step's dropout seed from it)
__global__ void set_u64_kernel(unsigned long long* p, unsigned long long v) { *p = v; }
__global__ void dec_dropout_fwd(AttnK k, float p, unsigned long long seed, const unsigned long long* seedp,
                                const float* inj) {
  if (seedp) seed = *seedp;
  const long n = (long)k.B * k.T * (k.S + k.A);
  const float keep = 1.0f / (1.0f - p);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    float m;
    if (inj) {
      m = inj[i];
    } else {
      const unsigned long long h = mix64(seed * 0x9e3779b97f4a7c15ull + (unsigned long long)i);
      const float u = (float)(h >> 40) * (1.0f / 16777216.0f);  // [0, 1)
      m = u >= p ? keep : 0.f;
    }
    k.MASK[i] = m;
    k.VV[i] = k.VV[i] * m;
  }
}
__global__ void dec_dropout_bwd(AttnK k) {
  const long n = (long)k.B * k.T * (k.S + k.A);
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    k.DV[i] = k.DV[i] * k.MASK[i];
}

#include "attn_persist.inc"
#include "dec_xcd.inc"
#include "dec_xcd_lstm.inc"

}  // namespace

int attn_check_dims(const AttnDims& d) {
  S2S_REQUIRE(d.B > 0 && d.L > 0 && d.T > 0, "attn: empty B/L/T");
  S2S_REQUIRE(d.S % 16 == 0 && d.A % 16 == 0 && d.Sc % 16 == 0, "attn: S, A, scoreDepth must be multiples of 16");
  S2S_REQUIRE(d.Sc <= 1024, "attn: scoreDepth > 1024 not supported");
  S2S_REQUIRE(d.O > 0 && d.M > 0 && d.K > 0, "attn: bad output/mlp dims");
  S2S_REQUIRE(!d.ext || d.dropout == 0.f, "attn: dropout belongs to the external decoder_mlp");
  S2S_REQUIRE(d.dropout >= 0.f && d.dropout < 1.f, "attn: dropout must be in [0, 1)");
  S2S_REQUIRE(d.hf >= 0 && (d.hf == 0 || (d.hk >= 1 && d.hk <= kMaxHybK)),
              "attn: hybridAttendFilterSize must be in [1, 8] when hybridAttendFeatureMaps > 0");
  return 0;
}

size_t attn_saved_bytes(const AttnDims& d) { return carve(d, nullptr, nullptr, nullptr).saved; }
// scratch = [forward | backward working sets (overlapping)] + split-K slabs of the GEMMs
static size_t attn_ws_offset(const AttnDims& d) {
  Layout l = carve(d, nullptr, nullptr, nullptr);
  return ((l.fwd > l.bwd ? l.fwd : l.bwd) + 255) & ~size_t(255);
}
// + the two sync-region headers (carve: fhdr, bhdr)
size_t attn_scratch_bytes(const AttnDims& d) { return attn_ws_offset(d) + sizeof(float) * kGemmWsFloats + 512; }
static GemmWs attn_gemm_ws(const AttnDims& d, void* scratch) {
  return GemmWs{reinterpret_cast<float*>(static_cast<char*>(scratch) + attn_ws_offset(d)), kGemmWsFloats};
}
const float* attn_saved_mlp_input(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.VV;
}
const float* attn_saved_alpha(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.ALPHA;
}
const float* attn_saved_ws(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.WS;
}
const float* attn_saved_vh(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.Vh;
}
const float* attn_saved_mono_ind(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.IND;
}
const int* attn_saved_maxout_argmax(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.AM;
}
const float* attn_saved_dropout_mask(const AttnDims& d, const void* saved) {
  AttnK k{};
  carve(d, &k, (char*)saved, nullptr);
  return k.MASK;
}

// S2S_DEC_MODE=step forces the per-step launch path (A/B and fallback); default: the persistent
// decoder kernels whenever the shape has an instantiation.
static std::atomic<unsigned long long*> g_dec_stamps[2] = {{nullptr}, {nullptr}};

static int dec_persist_variant(const AttnDims& d) {
  if (dec_mode() == 1) return 0;
  if (d.hf > 0 || d.lstm) return 0;
  if (d.flen || d.tlen) return 0;  // variable-length batches: the XCD-local or the per-step kernels
  if ((d.L + LC - 1) / LC > 256) return 0;
  if (d.S == 256 && d.A == 512 && d.Sc == 512) return 1;
  if (d.S == 64 && d.A == 128 && d.Sc == 128) return 2;
  return 0;
}

// The per-step path folds F4 + F5 (and K4 + K5) for the shapes only it serves: the LSTM decoder and hybrid attention
// (the GRU content-attention per-step path stays bitwise equal to the persistent kernels of attn_persist.inc)
static bool dec_fold_f45(const AttnDims& d) { return d.lstm || d.hf > 0; }

// algorithmic flops of one decoder recurrence launch (T P_step + T L (2 Sc + A) per utterance,
// times 2; the backward does twice the forward's products)
static double dec_flops(const AttnDims& d, bool bwd) {
  const double S = d.S, Sc = d.Sc, A = d.A, O = d.O, Mk = (double)d.M * d.K;
  const double p_step = S * Sc + O * S + A * S + 2 * S * S + 3 * S * 2 * S + (S + A) * Mk + d.M * O;
  const double f = 2.0 * d.B * ((double)d.T * p_step + (double)d.T * d.L * (2 * Sc + A));
  return bwd ? 2.0 * f : f;
}

// A persistent launch must be fully co-resident (its workgroups wait on each other).
static bool co_resident(const void* fn, int grid, size_t dyn_lds) {
  int dev = 0, cus = 0, per_cu = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return false;
  if (dyn_lds > 0 && hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dyn_lds) != hipSuccess)
    return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, 256, dyn_lds) != hipSuccess) return false;
  return (long)per_cu * cus >= grid;
}

// resident-chunk variant (attn_persist.inc) when the chunks fit
static bool dec_res_enabled(const AttnDims& d) {
  return 16 * ((d.L + LC - 1) / LC) <= kDecWG;
}

struct PersistLaunch {
  const void* fn = nullptr;
  size_t lds = 0;
};

static PersistLaunch pick_dec_fwd(int var, const AttnDims& d, int grid) {
  PersistLaunch c[2];
  if (var == 1) {
    c[0] = {(const void*)dec_fwd_persist<4, 8, 2, true>, dec_fwd_res_lds(d.A, d.Sc)};
    c[1] = {(const void*)dec_fwd_persist<4, 8, 2, false>, 0};
  } else {
    c[0] = {(const void*)dec_fwd_persist<1, 2, 1, true>, dec_fwd_res_lds(d.A, d.Sc)};
    c[1] = {(const void*)dec_fwd_persist<1, 2, 1, false>, 0};
  }
  for (int i = dec_res_enabled(d) ? 0 : 1; i < 2; ++i)
    if (co_resident(c[i].fn, grid, c[i].lds)) return c[i];
  return {};
}

static PersistLaunch pick_dec_bwd(int var, const AttnDims& d, int grid) {
  PersistLaunch c[2];
  if (var == 1) {
    c[0] = {(const void*)dec_bwd_persist<4, 8, true>, dec_bwd_res_lds(d.A, d.Sc)};
    c[1] = {(const void*)dec_bwd_persist<4, 8, false>, 0};
  } else {
    c[0] = {(const void*)dec_bwd_persist<1, 2, true>, dec_bwd_res_lds(d.A, d.Sc)};
    c[1] = {(const void*)dec_bwd_persist<1, 2, false>, 0};
  }
  for (int i = dec_res_enabled(d) ? 0 : 1; i < 2; ++i)
    if (co_resident(c[i].fn, grid, c[i].lds)) return c[i];
  return {};
}

static int launch_persist(const PersistLaunch& p, int grid, hipStream_t st, AttnK& k) {
  void* args[] = {&k};
  S2S_TRY(check_resident(p.fn, grid, 256, p.lds, "decoder persistent launch"));
  S2S_CHECK_HIP(hipLaunchKernel(p.fn, dim3(grid), dim3(256), args, p.lds, st));
  return 0;
}

static std::atomic<int> g_dec_allow_local{1};
// s2s_debug_head_sums_slabs(0) (A/B): the decoder MLP GEMM's split-K reduce as its own launch in front of the MLP head
static std::atomic<int> g_head_sums_slabs{1};
static std::atomic<int> g_merge_alpha_head{1};  // s2s_debug_merge_alpha_head(0) (diagnostic): alpha / VBAR launched alone
// attn_fwd's merged launch after the MLP GEMM: alpha / indicators, VBAR and the MLP head (the XCD-local path, no split
// side stream, the in-library MLP)
static bool merged_head(const AttnDims& d, const XPlan& xp, hipStream_t side) {
  return xp.var && !side && !d.ext && g_merge_alpha_head;
}
// ... which also runs the head's backward when the seed is final before the forward (AttnDims::dlogp_early); the same
// predicate in attn_bwd_core decides that dec_mlp_head_bwd is not launched there
static bool attn_head_bwd_fused(const AttnDims& d) {
  return d.dlogp_early && merged_head(d, dec_xcd_plan(d), nullptr);
}

// s2s_debug_dec_r4(0) (A/B): chains of <= 4 utterances keep the 16 x 16 x 4 skinny products
static std::atomic<int> g_dec_r4{1};
template <int S, int A, int SC, bool R4>
static const void* xcd_kernel(bool fwd, int res) {
  return res == 2 ? (fwd ? (const void*)dec_xcd_fwd<S, A, SC, 2, R4> : (const void*)dec_xcd_bwd<S, A, SC, 2, R4>)
       : res == 1 ? (fwd ? (const void*)dec_xcd_fwd<S, A, SC, 1, R4> : (const void*)dec_xcd_bwd<S, A, SC, 1, R4>)
                  : (fwd ? (const void*)dec_xcd_fwd<S, A, SC, 0, R4> : (const void*)dec_xcd_bwd<S, A, SC, 0, R4>);
}
template <int S, int A, int SC>
static int launch_xcd_t(bool fwd, int res, hipStream_t st, AttnK& k, XArgs& x) {
  const size_t lds = xdec_lds<S, A, SC>(x.XLC, res);
  // a chain of at most 4 utterances (B <= 32): its skinny products on the 4 x 4 x 1 MFMA (handoff.h mfma4_aw_acc)
  const void* fn = x.U <= 4 && g_dec_r4.load() ? xcd_kernel<S, A, SC, true>(fwd, res) : xcd_kernel<S, A, SC, false>(fwd, res);
  if (lds) S2S_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* args[] = {&k, &x};
  S2S_TRY(check_resident(fn, chain_grid(x.nchains, kXWG), 256, lds, fwd ? "dec_xcd_fwd" : "dec_xcd_bwd"));
  S2S_CHECK_HIP(hipLaunchKernel(fn, dim3(chain_grid(x.nchains, kXWG)), dim3(256), args, lds, st));
  return 0;
}
static int launch_xcd(const XPlan& xp, bool fwd, hipStream_t st, AttnK& k, XArgs& x) {
  if (xp.var == 1) return launch_xcd_t<256, 512, 512>(fwd, xp.res, st, k, x);
  return launch_xcd_t<64, 128, 128>(fwd, xp.res, st, k, x);
}
// the LSTM / hybrid kernels (var 3: S = 400 carried as 448, A = 256, Sc = 160, resident chunks, 4 x 4 x 1 products)
static int launch_xcd_lstm(bool fwd, hipStream_t st, AttnK& k, XArgs& x, XLArgs& y) {
  const size_t lds = xdec_lds<kXlSP, 256, 160>(x.XLC, 2);
  const void* fn = fwd ? (const void*)dec_xcd_lstm_fwd<kXlSP, 256, 160, 5, true>
                       : (const void*)dec_xcd_lstm_bwd<kXlSP, 256, 160, kXlSCP, 5, true>;
  if (lds) S2S_CHECK_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  void* args[] = {&k, &x, &y};
  S2S_TRY(check_resident(fn, chain_grid(x.nchains, kXWG), 256, lds, fwd ? "dec_xcd_lstm_fwd" : "dec_xcd_lstm_bwd"));
  S2S_CHECK_HIP(hipLaunchKernel(fn, dim3(chain_grid(x.nchains, kXWG)), dim3(256), args, lds, st));
  return 0;
}

// Folds and teacher-forced constants of the LSTM / hybrid kernels (params and labels only): the re-layouts, y_in,
// BKD, the hybrid fold (HGT, HCU), WDC = Wd_c Wc, KD = y_in Wd_y^T + BKD, then per gate q: WXG_q = Wq_x WDC and
// KXG_q = KD Wq_x^T + bq (the padded rows / columns stay zero), WXGT = WXG^T.
static int dec_xcd_lstm_prologue(hipStream_t st, const AttnDims& d, AttnK& k, const XArgs& x, const XLArgs& y,
                                 const GemmWs& gws) {
  WgradPrecision wp;  // the folds are reused by every step: fp32
  const int S = d.S, A = d.A, rows = d.B * d.T;
  const long SP = kXlSP;
  hipLaunchKernelGGL(dec_xcd_lstm_pack, dim3(1024), dim3(256), 0, st, k, y, kXlSP, kXlSCP);
  hipLaunchKernelGGL(dec_xcd_bkd, dim3((S + 3) / 4), dim3(256), 0, st, k, x.BKD);
  hipLaunchKernelGGL(dec_hyb_fold, dim3((d.Sc + 255) / 256), dim3(256), 0, st, k);
  S2S_CHECK_HIP(hipGetLastError());
  S2S_TRY(zero_async(st, y.WXG, sizeof(float) * 4 * SP * A));
  S2S_TRY(zero_async(st, y.KXG, sizeof(float) * (size_t)rows * 4 * SP));
  S2S_TRY(gemm1(st, false, false, S, A, S, 1.f, k.P.Wd, 2L * S, k.P.Wc, A, 0.f, x.WDC, A, nullptr, gws));
  S2S_TRY(gemm1(st, false, true, rows, S, S, 1.f, k.CY + S, 2L * S, k.P.Wd + S, 2L * S, 0.f, x.KD, S, x.BKD, gws));
  GemmProblem pw[4], pk[4];
  for (int q = 0; q < 4; ++q) {
    pw[q] = GemmProblem{y.WXD4 + (long)q * S * S, x.WDC, y.WXG + q * SP * A, nullptr, S, A, A, S, A, S, 1.f, 0.f};
    pk[q] = GemmProblem{x.KD, y.WXD4 + (long)q * S * S, y.KXG + q * SP, y.BQ + (long)q * S, S, S, 4 * SP, rows, S, S,
                        1.f, 0.f};
  }
  S2S_TRY(gemm_f32(st, pw, 4, false, false, gws));
  S2S_TRY(gemm_f32(st, pk, 4, false, true, gws));
  return transpose_f32(st, y.WXG, A, (int)(4 * SP), A, y.WXGT, 4 * SP);
}

// Weight folds and teacher-forced constants of the XCD-local decoder (params and labels only, so
// the model step runs it on the side stream beside the encoder).
static int dec_xcd_prologue(hipStream_t st, const AttnDims& d, AttnK& k, const XArgs& x, const GemmWs& gws) {
  WgradPrecision wp;  // the weight folds Wx' = W_d Wd_c Wc are reused by every step: fp32
  const int S = d.S, A = d.A, rows = d.B * d.T;
  // On the side stream beside the encoder its kernels run only where the persistent GRU launches leave
  // room -- and a kernel with a workgroup dealt to an XCD the layer's chains fill waits for the layer to
  // end -- so the chain is kept to 4 launches: the re-layouts (incl. the transposed operands below) and
  // y_in, BKD, then two batched NN GEMM launches (done by the end of encoder layer 2; the transposes and
  // the separate NT launches of the earlier chain left its last GEMM after layer 3, in front of the decoder)
  hipLaunchKernelGGL(dec_xcd_pack_ops, dim3(1024), dim3(256), 0, st, k, x);
  hipLaunchKernelGGL(dec_xcd_bkd, dim3((S + 3) / 4), dim3(256), 0, st, k, x.BKD);  // BKD = Wd_c bc + bd
  S2S_CHECK_HIP(hipGetLastError());
  // WDC = Wd_c Wc (S x A), WDCT = WDC^T = Wc^T Wd_c^T (A x S), KD = y_in Wd_y^T + BKD (B*T x S)
  const GemmProblem pa[3] = {
      GemmProblem{k.P.Wd, k.P.Wc, x.WDC, nullptr, 2L * S, A, A, S, A, S, 1.f, 0.f},
      GemmProblem{x.PWCT, x.PWDCT, x.WDCT, nullptr, S, S, S, A, S, S, 1.f, 0.f},
      GemmProblem{k.CY + S, x.PWDYT, x.KD, x.BKD, 2L * S, S, S, rows, S, S, 1.f, 0.f}};
  S2S_TRY(gemm_f32(st, pa, 3, false, false, gws));
  // WX = WXD WDC (3S x A), WXT = WX^T = WDC^T WXD^T (A x 3S), KX = KD WXD^T (B*T x 3S)
  const GemmProblem pb[3] = {
      GemmProblem{x.WXD, x.WDC, x.WX, nullptr, S, A, A, 3 * S, A, S, 1.f, 0.f},
      GemmProblem{x.WDCT, x.PWXDT, x.WXT, nullptr, S, 3L * S, 3L * S, A, 3 * S, S, 1.f, 0.f},
      GemmProblem{x.KD, x.PWXDT, x.KX, nullptr, S, 3L * S, 3L * S, rows, 3 * S, S, 1.f, 0.f}};
  S2S_TRY(gemm_f32(st, pb, 3, false, false, gws));
  return 0;
}

// the decoder launches of d's path hand off through the fsync / bsync regions of `scratch` (the XCD-local or
// the persistent kernels; the per-step path has none): their headers, for the caller's harvest
int attn_sync_regions(const AttnDims& d, void* saved, void* scratch, void** fwd, void** bwd) {
  *fwd = *bwd = nullptr;
  if (!dec_xcd_plan(d).var && !dec_persist_variant(d)) return 0;
  AttnK k{};
  carve(d, &k, static_cast<char*>(saved), static_cast<char*>(scratch));
  *fwd = k.fhdr;
  *bwd = k.bhdr;
  return 2;
}

int attn_fwd_prologue(hipStream_t st, const AttnDims& d, const int* labels, const AttnParams& P, void* saved,
                      void* scratch) {
  const XPlan xp = dec_xcd_plan(d);
  if (!xp.var) return 0;
  AttnK k{};
  XArgs x{};
  XLArgs y{};
  carve(d, &k, (char*)saved, (char*)scratch, &x, &y);
  k.P = P;
  k.labels = labels;
  if (xp.var == 3) S2S_TRY(dec_xcd_lstm_prologue(st, d, k, x, y, attn_gemm_ws(d, scratch)));
  else S2S_TRY(dec_xcd_prologue(st, d, k, x, attn_gemm_ws(d, scratch)));
  if (d.syncs_in_prologue) {  // both decoder launches' sync regions, off the decoder's critical path
    S2S_TRY(launch_sync_prep(st, k.fsync, k.fsync_bytes, nullptr, k.fhdr));
    S2S_TRY(launch_sync_prep(st, k.bsync, k.bsync_bytes, nullptr, k.bhdr));
  }
  return 0;
}

int attn_fwd(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P, float* logp,
             void* saved, void* scratch, size_t scratch_bytes, bool prologue_done, hipStream_t side, hipEvent_t* ev) {
  S2S_TRY(attn_check_dims(d));
  S2S_REQUIRE(scratch_bytes >= attn_scratch_bytes(d), "attn: scratch too small");
  AttnK k{};
  XArgs x{};
  XLArgs y{};
  carve(d, &k, (char*)saved, (char*)scratch, &x, &y);
  k.P = P;
  k.h = h;
  k.labels = labels;
  k.logp = logp;
  k.stamps = g_dec_stamps[0];
  const int B = d.B, L = d.L, T = d.T, S = d.S;
  const int bt = (B + 15) / 16;
  // Vh = h V^T  (TemporalConvolutionZeroBias(A, Sc, 1), Attention.lua:44)
  const GemmWs gws = attn_gemm_ws(d, scratch);
  S2S_TRY(gemm1(st, false, true, B * L, d.Sc, d.A, 1.f, h, d.A, P.V, d.A, 0.f, k.Vh, d.Sc, nullptr, gws));
  const XPlan xp = dec_xcd_plan(d);
  const bool merge_head = merged_head(d, xp, side);  // dec_xcd_alpha_vbar_head
  // s_0 = 0: the XCD-local path's prologue (dec_xcd_pack_ops) writes it
  if (!xp.var) hipLaunchKernelGGL(dec_init_fwd, dim3((B * S + 255) / 256), dim3(256), 0, st, k);
  const int pgrid = kDecWG * ((B + 15) / 16);
  const int pvar = xp.var ? 0 : dec_persist_variant(d);
  const PersistLaunch pf = pvar ? pick_dec_fwd(pvar, d, pgrid) : PersistLaunch{};
  if (xp.var) {
    if (!prologue_done)
      S2S_TRY(xp.var == 3 ? dec_xcd_lstm_prologue(st, d, k, x, y, gws) : dec_xcd_prologue(st, d, k, x, gws));
    x.U = xp.U;
    x.nchains = xp.nchains;
    x.XLC = xp.XLC;
    x.NCH = xp.NCH;
    x.allow_local = g_dec_allow_local;
    if (!(d.syncs_in_prologue && prologue_done)) S2S_TRY(launch_sync_prep(st, k.fsync, k.fsync_bytes, nullptr, k.fhdr));
    {
      // algorithmic units: the attention re-streams Vh and h every step, T B L (Sc + A) 4 bytes
      // per forward; flops = the step products + the attention contractions
      ProfScope ps(st, xp.var == 3 ? "dec_fwd_xcd_lstm" : "dec_fwd_xcd", dec_flops(d, false),
                   4.0 * d.T * d.B * d.L * (double)(d.Sc + d.A));
      S2S_TRY(xp.var == 3 ? launch_xcd_lstm(true, st, k, x, y) : launch_xcd(xp, true, st, k, x));
    }
    // alpha / MonotonicAlignment indicators from the saved scores and VBAR (the backward's dws reference
    // point) from Vh, in one launch: only the backward (and alpha()) read them, so beside the MLP head
    // when split (joined by attn_bwd_core through ev[2])
    if (side) {
      S2S_CHECK_HIP(hipEventRecord(ev[1], st));
      S2S_CHECK_HIP(hipStreamWaitEvent(side, ev[1], 0));
    }
    // (on the main stream, the MLP head's launch below runs them: one launch fewer between the decoder and
    // its backward)
    if (!merge_head) {
      hipLaunchKernelGGL(dec_xcd_alpha_vbar, dim3(T * B + ((d.Sc + 63) / 64) * B), dim3(256), 0, side ? side : st, k,
                         x);
      if (side) S2S_CHECK_HIP(hipEventRecord(ev[2], side));
      S2S_CHECK_HIP(hipGetLastError());
    }
  } else if (pf.fn) {
    S2S_TRY(launch_sync_prep(st, k.fsync, k.fsync_bytes, nullptr, k.fhdr));
    {
      ProfScope ps(st, "dec_fwd_persist", 0.0, 0.0);
      S2S_TRY(launch_persist(pf, pgrid, st, k));
    }
    hipLaunchKernelGGL(dec_alpha_ind, dim3(T, B), dim3(256), 0, st, k);
    S2S_CHECK_HIP(hipGetLastError());
  } else {
  ProfScope ps(st, "dec_fwd_steps", 0.0, 0.0);
  if (d.hf > 0) hipLaunchKernelGGL(dec_hyb_fold, dim3((d.Sc + 255) / 256), dim3(256), 0, st, k);
  if (d.lstm) hipLaunchKernelGGL(dec_lstm_pack, dim3(256), dim3(256), 0, st, k);
  const bool fold = dec_fold_f45(d);
  const int A = d.A, rows = B * T;
  if (fold) {  // y_in rows, BKD = Wd_c bc + bd, WDC = Wd_c Wc, KD = y_in Wd_y^T + BKD
    WgradPrecision wp;  // the folds are reused by every step: fp32
    hipLaunchKernelGGL(dec_fold_yin, dim3(512), dim3(256), 0, st, k);
    hipLaunchKernelGGL(dec_xcd_bkd, dim3((S + 3) / 4), dim3(256), 0, st, k, x.BKD);
    S2S_CHECK_HIP(hipGetLastError());
    S2S_TRY(gemm1(st, false, false, S, A, S, 1.f, P.Wd, 2L * S, P.Wc, A, 0.f, x.WDC, A, nullptr, gws));
    S2S_TRY(gemm1(st, false, true, rows, S, S, 1.f, k.CY + S, 2L * S, P.Wd + S, 2L * S, 0.f, x.KD, S, x.BKD, gws));
  }
  for (int t = 0; t < T; ++t) {
    k.t = t;
    hipLaunchKernelGGL(dec_f1_ws, dim3(d.Sc / 16, bt), dim3(256), 0, st, k);
    hipLaunchKernelGGL(dec_f2_attn<8>, dim3(k.NCH, B), dim3(512), 0, st, k);
    hipLaunchKernelGGL(dec_f3_combine, dim3(B), dim3(256), 0, st, k);
    if (fold) {
      hipLaunchKernelGGL(dec_f45_fold, dim3(S / 16, bt), dim3(512), 0, st, k, x.WDC, x.KD);
    } else {
      hipLaunchKernelGGL(dec_f4_cin, dim3(S / 16, bt), dim3(256), 0, st, k);
      hipLaunchKernelGGL(dec_f5_d, dim3(S / 16, bt), dim3(256), 0, st, k);
    }
    if (d.lstm) {
      hipLaunchKernelGGL(dec_f6_lstm, dim3(4 * S / 16, bt), dim3(512), 0, st, k);
    } else {
      hipLaunchKernelGGL(dec_f6_gru1, dim3(2 * S / 16, bt), dim3(256), 0, st, k);
      hipLaunchKernelGGL(dec_f7_gru2, dim3(S / 16, bt), dim3(256), 0, st, k);
    }
  }
  S2S_CHECK_HIP(hipGetLastError());
  // c_in rows for the weight gradients (the folded steps never formed them): CY[:, :S] = C Wc^T + bc
  if (fold) S2S_TRY(gemm1(st, false, true, rows, S, A, 1.f, k.C, A, P.Wc, A, 0.f, k.CY, 2L * S, P.bc, gws));
  }
  // decoder MLP over all B*T rows: U = [s; c] Wm^T + bm, then maxout / Linear / LogSoftMax
  if (d.ext) return 0;  // external decoder_mlp: the caller runs it on the saved VV rows
  const int rows = B * T;
  if (d.dropout > 0.f) {
    hipLaunchKernelGGL(dec_dropout_fwd, dim3(512), dim3(256), 0, st, k, d.dropout, d.dropout_seed, d.dropout_seed_dev,
                       d.dropout_mask);
    S2S_CHECK_HIP(hipGetLastError());
  }
  {
    // the merged head sums the MLP GEMM's split-K slabs itself (no reduce launch between them)
    GemmDeferred dr{};
    GemmDeferReduce scope(merge_head && g_head_sums_slabs ? &dr : nullptr);
    S2S_TRY(gemm1(st, false, true, rows, d.M * d.K, S + d.A, 1.f, k.VV, S + d.A, P.Wm, S + d.A, 0.f, k.U,
                  (long)d.M * d.K, P.bm, gws));
    if (dr.splits > 1) {
      k.UP = dr.part;
      k.UPS = dr.splits;
      k.UPMN = dr.mn;
    }
  }
  if (merge_head) {
    const bool hb = attn_head_bwd_fused(d);
    k.dlogp = hb ? d.dlogp_early : nullptr;
    hipLaunchKernelGGL(dec_xcd_alpha_vbar_head, dim3(T * B + ((d.Sc + 63) / 64) * B + (rows + 3) / 4), dim3(256),
                       4 * (d.M + (hb ? d.O : 0)) * sizeof(float), st, k, x, rows);
  }
  else
    hipLaunchKernelGGL(dec_mlp_head, dim3((rows + 3) / 4), dim3(256), 4 * d.M * sizeof(float), st, k, rows);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int attn_dh_gemms(hipStream_t st, const AttnDhTerms& t, float* dh, int accumulate_dh, hipEvent_t dvh_ready) {
  const int B = t.B, L = t.L, T = t.T, A = t.A;
  const GemmWs gws = t.gws;
  // dh_l (+)= sum_t alpha_{t,l} dc_t  (one GEMM per utterance: alpha_b^T (L x T) . dc_b (T x A))
  for (int b0 = 0; b0 < B; b0 += kMaxGemmBatch) {
    GemmProblem pr[kMaxGemmBatch];
    const int nb = std::min(kMaxGemmBatch, B - b0);
    for (int i = 0; i < nb; ++i) {
      const long b = b0 + i;
      pr[i] = GemmProblem{t.alpha + b * T * L, t.dc + b * T * A, dh + b * L * A, nullptr, L, A, A, L, A, T,
                          1.f, accumulate_dh ? 1.f : 0.f};
    }
    S2S_TRY(gemm_f32(st, pr, nb, true, false, gws));
  }
  if (dvh_ready) S2S_CHECK_HIP(hipStreamWaitEvent(st, dvh_ready, 0));
  // dh += dVh V   (Vh = h V^T)
  return gemm1(st, false, false, B * L, A, t.Sc, 1.f, t.dvh, t.Sc, t.V, A, 1.f, dh, A, nullptr, gws);
}

int attn_bwd_core(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P,
                  const void* saved, const float* dlogp, float* dh, int accumulate_dh, void* scratch,
                  size_t scratch_bytes, hipStream_t side, hipEvent_t* ev, AttnDhTerms* defer_dh) {
  if (defer_dh) *defer_dh = AttnDhTerms{};
  S2S_TRY(attn_check_dims(d));
  S2S_REQUIRE(scratch_bytes >= attn_scratch_bytes(d), "attn: scratch too small");
  AttnK k{};
  XArgs x{};
  XLArgs y{};
  carve(d, &k, (char*)saved, (char*)scratch, &x, &y);
  k.P = P;
  k.h = h;
  k.labels = labels;
  k.dlogp = dlogp;
  k.stamps = g_dec_stamps[1];
  k.dh = dh;
  k.lddh = d.A;
  const int B = d.B, L = d.L, T = d.T, S = d.S, A = d.A, Sc = d.Sc, O = d.O, Mk = d.M * d.K;
  const int rows = B * T, bt = (B + 15) / 16;
  const XPlan xp = dec_xcd_plan(d);
  // the XCD-local path's first dh writer is the alpha^T dc GEMM (beta 0 when not accumulating)
  const int pvar = xp.var ? 0 : dec_persist_variant(d);
  // the persistent kernels accumulate dh in place (the XCD-local and the per-step paths write it by GEMMs after
  // their loop, beta 0 when not accumulating)
  if (!accumulate_dh && pvar) S2S_TRY(zero_async(st, dh, sizeof(float) * (size_t)B * L * A));
  if (!xp.var) {  // the XCD-local path writes DVH / DWEACC whole after its loop
    S2S_TRY(zero_async(st, k.DVH, sizeof(float) * (size_t)B * L * Sc));
    S2S_TRY(zero_async(st, k.DWEACC, sizeof(float) * (size_t)B * k.NCH * Sc));
  }
  // packed transposes for the backward products
  if (d.lstm && !xp.var) {  // GT = LW^T in the gate gradients' gate-major order
    hipLaunchKernelGGL(dec_lstm_gt, dim3(512), dim3(256), 0, st, k);
    S2S_CHECK_HIP(hipGetLastError());
  }
  if (!xp.var) {  // (the XCD-local path's operand layouts come from its prologue)
  if (!d.lstm) {
  S2S_TRY(transpose_f32(st, P.Wh, 2L * S, S, S, k.WhT, S));          // WhT[k][n] = Wh[n][k], k < S
  S2S_TRY(transpose_f32(st, P.Wz, 2L * S, S, 2 * S, k.GT, 3L * S));   // GT[c][n]      = Wz[n][c]
  S2S_TRY(transpose_f32(st, P.Wr, 2L * S, S, 2 * S, k.GT + S, 3L * S));
  S2S_TRY(transpose_f32(st, P.Wh, 2L * S, S, 2 * S, k.GT + 2 * S, 3L * S));
  // the h-half of Wh reaches ds_{t-1} through dq = Wh[:, :S]^T da_h (K2), not through GT
  hipLaunchKernelGGL(fill2d_kernel, dim3(64), dim3(256), 0, st, k.GT + 2 * S, 3L * S, S, S, 0.f);
  }
  if (!dec_fold_f45(d)) {
    S2S_TRY(transpose_f32(st, P.Wd, 2L * S, S, 2 * S, k.WdT, S));
    S2S_TRY(transpose_f32(st, P.Wc, A, S, A, k.WcT, S));
  }
  S2S_TRY(transpose_f32(st, P.Ws, S, Sc, S, k.WsT, Sc));
  }
  const GemmWs gws = attn_gemm_ws(d, scratch);
  // folded K4 + K5 (per-step path, LSTM / hybrid shapes): WDC^T = Wc^T Wd_c^T (A x S) in WcT's place
  const bool fold = !xp.var && !dec_persist_variant(d) && dec_fold_f45(d);
  if (fold) {
    WgradPrecision wp;
    S2S_TRY(gemm1(st, true, true, A, S, S, 1.f, P.Wc, A, P.Wd, 2L * S, 0.f, k.WcT, S, nullptr, gws));
  }
  if (d.ext) {  // external decoder_mlp: dlogp holds d[s_t; c_t] (B*T, S+A)
    S2S_TRY(copy2d_f32(st, dlogp, S + A, k.DV, S + A, rows, S + A, false));
  } else {
  // MLP backward for all rows (not on the recurrence), unless the forward's head launch ran it
  if (attn_head_bwd_fused(d)) {
    S2S_REQUIRE(dlogp == d.dlogp_early, "attn: dlogp_early differs from the backward's dlogp");
  } else {
    hipLaunchKernelGGL(dec_mlp_head_bwd, dim3((rows + 3) / 4), dim3(256), 4 * O * sizeof(float), st, k, rows);
    S2S_CHECK_HIP(hipGetLastError());
  }
  // dV = dU Wm  ->  [ds_mlp | dc_mlp]
  S2S_TRY(gemm1(st, false, false, rows, S + A, Mk, 1.f, k.DU, Mk, P.Wm, S + A, 0.f, k.DV, S + A, nullptr, gws));
  }
  if (d.dropout > 0.f) {
    hipLaunchKernelGGL(dec_dropout_bwd, dim3(512), dim3(256), 0, st, k);
    S2S_CHECK_HIP(hipGetLastError());
  }
  const int pgrid = kDecWG * ((B + 15) / 16);
  const PersistLaunch pb = pvar ? pick_dec_bwd(pvar, d, pgrid) : PersistLaunch{};
  if (xp.var) {
    x.U = xp.U;
    x.nchains = xp.nchains;
    x.XLC = xp.XLC;
    x.NCH = xp.NCH;
    x.allow_local = g_dec_allow_local;
    if (!d.syncs_in_prologue) S2S_TRY(launch_sync_prep(st, k.bsync, k.bsync_bytes, nullptr, k.bhdr));
    if (side) S2S_CHECK_HIP(hipStreamWaitEvent(st, ev[2], 0));  // VBAR, ALPHA, IND from the forward's side stream
    {
      ProfScope ps(st, xp.var == 3 ? "dec_bwd_xcd_lstm" : "dec_bwd_xcd", dec_flops(d, true),
                   8.0 * d.T * d.B * d.L * (double)(d.Sc + d.A));
      S2S_TRY(xp.var == 3 ? launch_xcd_lstm(false, st, k, x, y) : launch_xcd(xp, false, st, k, x));
    }
    // dVh / dwe (dec_xcd_dvh) beside the alpha^T dc GEMMs when split; both feed dh
    if (side) {
      S2S_CHECK_HIP(hipEventRecord(ev[3], st));
      S2S_CHECK_HIP(hipStreamWaitEvent(side, ev[3], 0));
    }
    if (d.hf > 0) {  // the location features inside the tanh terms (dec_xcd_lstm.inc)
      const size_t lds = dec_xcd_dvh_hyb_lds(T);
      if (lds > 64 * 1024)
        S2S_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dec_xcd_dvh_hyb),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(dec_xcd_dvh_hyb, dim3((Sc + 63) / 64, k.NCH, B), dim3(256), lds, side ? side : st, k, x);
      S2S_CHECK_HIP(hipGetLastError());
    } else {
      const size_t lds = dec_xcd_dvh_lds(T);
      if (lds > 64 * 1024)
        S2S_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dec_xcd_dvh),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
      hipLaunchKernelGGL(dec_xcd_dvh, dim3((Sc + 63) / 64, (L + kDvhF - 1) / kDvhF, B), dim3(256), lds, side ? side : st, k,
                         x);
      S2S_CHECK_HIP(hipGetLastError());
    }
    if (side) S2S_CHECK_HIP(hipEventRecord(ev[4], side));
    const AttnDhTerms terms{k.ALPHA, x.DCS, k.DVH, P.V, B, L, T, A, Sc, gws};
    if (defer_dh && !accumulate_dh) {  // the caller fuses both terms into the encoder BPTT launch
      if (side) S2S_CHECK_HIP(hipStreamWaitEvent(st, ev[4], 0));
      *defer_dh = terms;
      return 0;
    }
    return attn_dh_gemms(st, terms, dh, accumulate_dh, side ? ev[4] : nullptr);
  } else if (pb.fn) {
    S2S_TRY(launch_sync_prep(st, k.bsync, k.bsync_bytes, nullptr, k.bhdr));
    ProfScope ps(st, "dec_bwd_persist", 0.0, 0.0);
    S2S_TRY(launch_persist(pb, pgrid, st, k));
    S2S_CHECK_HIP(hipGetLastError());
  } else {
  hipLaunchKernelGGL(dec_bwd_init, dim3((B * S + 255) / 256), dim3(256), 0, st, k);
  // dec_b6_attn<true>'s dZ rows, staged taps and alpha halo
  const size_t b6_lds = d.hf > 0 ? sizeof(float) * ((LC + (size_t)d.hk) * Sc + LC + kMaxHybK) : 0;
  if (b6_lds > 32 * 1024)
    S2S_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(dec_b6_attn<true>),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)b6_lds));
  if (d.hf > 0) {
    S2S_TRY(zero_async(st, k.QA, sizeof(float) * 2 * (size_t)B * L * d.hk));
    S2S_TRY(zero_async(st, k.PDG, sizeof(float) * (size_t)B * k.NCH * d.hk * Sc));
  }
  ProfScope ps(st, "dec_bwd_steps", 0.0, 0.0);
  for (int t = T - 1; t >= 0; --t) {
    k.t = t;
    if (d.lstm) {
      hipLaunchKernelGGL(dec_b3_lstm, dim3(2 * S / 16, bt), dim3(512), 0, st, k);
    } else {
      hipLaunchKernelGGL(dec_b2_gru1, dim3(S / 16, bt), dim3(256), 0, st, k);
      hipLaunchKernelGGL(dec_b3_gru2, dim3(2 * S / 16, bt), dim3(256), 0, st, k);
    }
    if (fold) {
      hipLaunchKernelGGL(dec_b45_fold, dim3(A / 16, bt), dim3(512), 0, st, k, k.WcT);
    } else {
      hipLaunchKernelGGL(dec_b4_wd, dim3(2 * S / 16, bt), dim3(256), 0, st, k);
      hipLaunchKernelGGL(dec_b5_wc, dim3(A / 16, bt), dim3(256), 0, st, k);
    }
    if (d.hf > 0) hipLaunchKernelGGL(dec_b6_attn<true>, dim3(k.NCH, B), dim3(512), b6_lds, st, k);
    else hipLaunchKernelGGL(dec_b6_attn<false>, dim3(k.NCH, B), dim3(256), 0, st, k);
    hipLaunchKernelGGL(dec_b8_ws, dim3(S / 16, bt), dim3(256), 0, st, k);
  }
  S2S_CHECK_HIP(hipGetLastError());
  // [dc_in | dy_in] rows for the weight gradients (the folded steps never formed them): DCY = DD Wd
  if (fold) S2S_TRY(gemm1(st, false, false, rows, 2 * S, S, 1.f, k.DD, S, P.Wd, 2L * S, 0.f, k.DCY, 2L * S, nullptr, gws));
  // dh (+)= sum_t alpha_t^T dc_t (per utterance) + dVh V
  return attn_dh_gemms(st, AttnDhTerms{k.ALPHA, k.DC, k.DVH, P.V, B, L, T, A, Sc, gws}, dh, accumulate_dh, nullptr);
  }
  // dh += dVh V   (Vh = h V^T)
  S2S_TRY(gemm1(st, false, false, B * L, A, Sc, 1.f, k.DVH, Sc, P.V, A, 1.f, dh, A, nullptr, gws));
  return 0;
}

// Weight gradients: one GEMM per parameter over all B*T rows (accumulate, alpha = scale), then
// the bias column sums.  Reads only the saved buffer and attn_bwd_core's scratch, so the model
// step runs it on a side stream beside the encoder BPTT.
int attn_bwd_wgrad(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P,
                   const void* saved, const AttnGrads& G, float scale, void* scratch) {
  WgradPrecision wp;
  AttnK k{};
  XArgs x{};
  XLArgs y{};
  carve(d, &k, (char*)saved, (char*)scratch, &x, &y);
  k.labels = labels;
  const int B = d.B, L = d.L, T = d.T, S = d.S, A = d.A, Sc = d.Sc, O = d.O, Mk = d.M * d.K;
  const int rows = B * T;
  hipLaunchKernelGGL(dec_onehot_prev, dim3(256), dim3(256), 0, st, k);
  S2S_CHECK_HIP(hipGetLastError());
  const XPlan xpw = dec_xcd_plan(d);
  if (xpw.var == 3) {
    // the LSTM kernels folded c -> c_in -> d away as well: c_in, d = HX[:, S:] (the LSTM input), dd = dGA WXD4 (the
    // four gates' x-weights) and [dc_in | dy_in] = dd Wd for the weight gradients, all B*T rows at once
    const GemmWs gws = attn_gemm_ws(d, scratch);
    S2S_TRY(gemm1(st, false, true, rows, S, A, 1.f, k.C, A, P.Wc, A, 0.f, k.CY, 2L * S, P.bc, gws));
    S2S_TRY(gemm1(st, false, true, rows, S, 2 * S, 1.f, k.CY, 2L * S, P.Wd, 2L * S, 0.f, k.HX + S, 2L * S, P.bd, gws));
    S2S_TRY(gemm1(st, false, false, rows, S, 4 * S, 1.f, k.DGA, 4L * S, y.WXD4, S, 0.f, k.DD, S, nullptr, gws));
    S2S_TRY(gemm1(st, false, false, rows, 2 * S, S, 1.f, k.DD, S, P.Wd, 2L * S, 0.f, k.DCY, 2L * S, nullptr, gws));
  } else if (xpw.var) {
    // the XCD-local loop folded c -> c_in -> d away: recompute them (and dd, [dc_in | dy_in]) for
    // the weight gradients, all B*T rows at once
    const GemmWs gws = attn_gemm_ws(d, scratch);
    S2S_TRY(gemm1(st, false, true, rows, S, A, 1.f, k.C, A, P.Wc, A, 0.f, k.CY, 2L * S, P.bc, gws));
    S2S_TRY(gemm1(st, false, true, rows, S, 2 * S, 1.f, k.CY, 2L * S, P.Wd, 2L * S, 0.f, k.HX + S, 2L * S, P.bd, gws));
    S2S_TRY(copy2d_f32(st, k.HX + S, 2L * S, k.RHX + S, 2L * S, rows, S, false));
    S2S_TRY(gemm1(st, false, false, rows, S, 3 * S, 1.f, k.DGA, 3L * S, x.WXD, S, 0.f, k.DD, S, nullptr, gws));
    S2S_TRY(gemm1(st, false, false, rows, 2 * S, S, 1.f, k.DD, S, P.Wd, 2L * S, 0.f, k.DCY, 2L * S, nullptr, gws));
  }
  {
    GemmProblem pr[16];
    int n = 0;
    if (!d.ext) {
      pr[n++] = GemmProblem{k.DO, k.MM, G.Wo, nullptr, O, d.M, d.M, O, d.M, rows, scale, 1.f};
      pr[n++] = GemmProblem{k.DU, k.VV, G.Wm, nullptr, Mk, S + A, S + A, Mk, S + A, rows, scale, 1.f};
    }
    if (d.lstm) {  // all four gates' [Wqh | Wqx] grads at once, staged in LDW (scattered below)
      pr[n++] = GemmProblem{k.DGA, k.HX, k.LDW, nullptr, 4L * S, 2L * S, 2L * S, 4 * S, 2 * S, rows, scale, 0.f};
    } else {
      pr[n++] = GemmProblem{k.DGA, k.HX, G.Wz, nullptr, 3L * S, 2L * S, 2L * S, S, 2 * S, rows, scale, 1.f};
      pr[n++] = GemmProblem{k.DGA + S, k.HX, G.Wr, nullptr, 3L * S, 2L * S, 2L * S, S, 2 * S, rows, scale, 1.f};
      pr[n++] = GemmProblem{k.DGA + 2 * S, k.RHX, G.Wh, nullptr, 3L * S, 2L * S, 2L * S, S, 2 * S, rows, scale,
                            1.f};
    }
    pr[n++] = GemmProblem{k.DD, k.CY, G.Wd, nullptr, S, 2L * S, 2L * S, S, 2 * S, rows, scale, 1.f};
    pr[n++] = GemmProblem{k.DCY, k.C, G.Wc, nullptr, 2L * S, A, A, S, A, rows, scale, 1.f};
    pr[n++] = GemmProblem{k.DCY + S, k.YP, G.Wy, nullptr, 2L * S, O, O, S, O, rows, scale, 1.f};
    pr[n++] = GemmProblem{k.DWS, k.HX, G.Ws, nullptr, Sc, 2L * S, S, Sc, S, rows, scale, 1.f};
    pr[n++] = GemmProblem{k.DVH, h, G.V, nullptr, Sc, A, A, Sc, A, B * L, scale, 1.f};
    S2S_TRY(gemm_f32(st, pr, n, true, false, attn_gemm_ws(d, scratch)));
  }
  const GemmWs cws = attn_gemm_ws(d, scratch);  // free again once the GEMMs above are done (stream order)
  if (!d.ext) {
    S2S_TRY(colsum_f32(st, k.DO, O, rows, O, scale, 1.f, G.bo, cws));
    S2S_TRY(colsum_f32(st, k.DU, Mk, rows, Mk, scale, 1.f, G.bm, cws));
  }
  S2S_TRY(colsum_f32(st, k.DD, S, rows, S, scale, 1.f, G.bd, cws));
  if (d.lstm) {
    ColsumOut outs[4];
    // LSTM.lua:25-29: Linear(S,S)(x) + Linear(S,S)(h), both with bias: the four gates' Wqx / Wqh blocks of LDW added
    // into their tensors in one launch (eight copy launches before)
    hipLaunchKernelGGL(lstm_dw_scatter, dim3(1024), dim3(256), 0, st, k.LDW, S, G);
    S2S_CHECK_HIP(hipGetLastError());
    for (int q = 0; q < 4; ++q) outs[q] = ColsumOut{q * S, S, {G.lstm[4 * q + 1], G.lstm[4 * q + 3], nullptr}, 2};  // bqx, bqh
    S2S_TRY(colsum_scatter_f32(st, k.DGA, 4L * S, rows, 4 * S, scale, outs, 4, cws));
  }
  {
    const ColsumOut outs[2] = {{0, S, {G.bc, nullptr, nullptr}, 1}, {S, S, {G.by, nullptr, nullptr}, 1}};
    S2S_TRY(colsum_scatter_f32(st, k.DCY, 2L * S, rows, 2 * S, scale, outs, 2, cws));
  }
  S2S_TRY(colsum_f32(st, k.DWS, Sc, rows, Sc, scale, 1.f, G.bs, cws));
  S2S_TRY(colsum_f32(st, k.DWEACC, Sc, B * k.NCH, Sc, scale, 1.f, G.we, cws));
  if (d.hf > 0) {  // hybrid features: dG (sum over utterances, chunks; steps summed in the loop), dcu = sum dws
    k.P = P;
    if (xpw.var == 3)  // the XCD-local chunks' partials (dec_xcd_lstm_bwd)
      S2S_TRY(colsum_f32(st, y.PDG, (long)d.hk * Sc, B * xpw.NCH, d.hk * Sc, 1.f, 0.f, k.DGT, cws));
    else
      S2S_TRY(colsum_f32(st, k.PDG, (long)d.hk * Sc, B * k.NCH, d.hk * Sc, 1.f, 0.f, k.DGT, cws));
    S2S_TRY(colsum_f32(st, k.DWS, Sc, rows, Sc, 1.f, 0.f, k.DCU, cws));
    const int n = Sc * d.hf + d.hf * d.hk + d.hf;
    hipLaunchKernelGGL(dec_hyb_wgrad, dim3((n + 3) / 4), dim3(256), 0, st, k, G, scale);
    S2S_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

int attn_bwd(hipStream_t st, const AttnDims& d, const float* h, const int* labels, const AttnParams& P,
             const void* saved, const float* dlogp, float* dh, int accumulate_dh, const AttnGrads& G, float scale,
             void* scratch, size_t scratch_bytes) {
  S2S_TRY(attn_bwd_core(st, d, h, labels, P, saved, dlogp, dh, accumulate_dh, scratch, scratch_bytes));
  return attn_bwd_wgrad(st, d, h, labels, P, saved, G, scale, scratch);
}

// ================================================================== beam search
// Attention:BeamSearch (Attention.lua:332-438) for B utterances at once, all on the device.  The
// K hypotheses of every utterance are R = B*K rows of the per-step decoder kernels run as a T = 2
// problem: row t = 1 of each is the decode step, its s_{t-1} and y_{t-1} written by beam_prep into
// the t = 1 slots (HX[:, :S], labels[:, 0]; label -1 = zeros_y at the first step).  beam_update then
// does the reference's bookkeeping per utterance: p_next = logp + p_beam over the active hypotheses,
// torch.topk(K) of the flattened candidates (sorted; ties -> lower index), the first K - finished of
// them extend their parent (finished on eos or at maxseqlength), states gathered from the parents.
namespace {

struct BeamK {
  int B, K, maxlen, eos, S, O, L, hyb, lstm;
  int *nact, *nfin, *done;
  int *yprev, *hist, *hlen, *fseq, *flen, *lab2;
  // per hypothesis, double-buffered by step parity: decoder state s, attention alpha (hybrid attention's
  // location features read alpha_{t-1}) and the LSTM cell (mem) -- the reference's hidden {alpha, s, mem}
  // (Attention.lua:360-403)
  float *pbeam, *s, *fscore, *alpha, *mem;
  float* mlp_in;  // (R, S + A) decoder_mlp input rows of the current step (external decoder_mlp)
};

// hypothesis row r = b*K + k gets utterance b's annotations (grid.y = utterance)
__global__ void beam_rep_h(const float* h, float* hr, int K, long per) {
  const int b = blockIdx.y;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (long)K * per; i += (long)gridDim.x * blockDim.x)
    hr[(long)b * K * per + i] = h[(long)b * per + i % per];
}

__global__ void beam_init(BeamK q) {
  const int R = q.B * q.K;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R * q.S; i += gridDim.x * blockDim.x) {
    q.s[i] = 0.f;
    if (q.lstm) q.mem[i] = 0.f;
  }
  if (q.hyb)
    for (long i = blockIdx.x * blockDim.x + threadIdx.x; i < (long)R * q.L; i += gridDim.x * blockDim.x) q.alpha[i] = 0.f;
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
    q.pbeam[r] = 0.f;
    q.yprev[r] = -1;
    q.hlen[r] = 0;
    q.flen[r] = 0;
    if (r < q.B) {
      q.nact[r] = 1;
      q.nfin[r] = 0;
      q.done[r] = 0;
    }
  }
}

// s_{t-1} and y_{t-1} of every hypothesis row into the t = 1 slots of the T = 2 problem; alpha_{t-1} (hybrid)
// and the LSTM cell c_{t-1} into its t = 0 slots (what the step kernels read as the previous step's)
__global__ void beam_prep(AttnK k, BeamK q, int par) {
  const int R = q.B * q.K, S = q.S, L = q.L;
  const float* s = q.s + (long)par * R * S;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < R * S; i += gridDim.x * blockDim.x) {
    const int r = i / S, n = i - r * S;
    k.HX[((long)r * 2 + 1) * 2 * S + n] = s[i];
    if (q.lstm) k.LC[((long)r * 2) * S + n] = q.mem[(long)par * R * S + i];
  }
  if (q.hyb)
    for (long i = blockIdx.x * blockDim.x + threadIdx.x; i < (long)R * L; i += gridDim.x * blockDim.x) {
      const long r = i / L, l = i - r * L;
      k.ALPHA[(r * 2) * L + l] = q.alpha[(long)par * R * L + i];
    }
  for (int r = blockIdx.x * blockDim.x + threadIdx.x; r < R; r += gridDim.x * blockDim.x) {
    q.lab2[2 * r] = q.yprev[r];
    q.lab2[2 * r + 1] = 0;
  }
}

constexpr int kBeamMaxK = 16;

__global__ __launch_bounds__(256) void beam_update(AttnK k, BeamK q, int count) {
  __shared__ float bv[256];
  __shared__ int bi[256];
  __shared__ int sel[kBeamMaxK];
  __shared__ float selv[kBeamMaxK];
  __shared__ int fpar[kBeamMaxK], ftok[kBeamMaxK], fdst[kBeamMaxK], npar[kBeamMaxK], ntok[kBeamMaxK];
  __shared__ float fsc[kBeamMaxK], np_[kBeamMaxK];
  __shared__ int nf_new, nn_new;
  const int b = blockIdx.x, tid = threadIdx.x, K = q.K, O = q.O, S = q.S, R = q.B * K;
  if (q.done[b]) return;
  const int nact = q.nact[b], ncand = nact * O;
  const int par = count & 1, nxt = par ^ 1;
  auto cval = [&](int c) {
    const int i = c / O, j = c - i * O;
    return k.LOGP[((long)(b * K + i) * 2 + 1) * O + j] + q.pbeam[b * K + i];
  };
  // torch.topk(p_next, K, 1, true): K rounds of a block arg-max over the unselected candidates
  const int nsel = min(K, ncand);
  for (int m = 0; m < nsel; ++m) {
    float best = -INFINITY;
    int bidx = 0x7fffffff;
    for (int c = tid; c < ncand; c += 256) {
      bool taken = false;
      for (int p = 0; p < m; ++p) taken = taken || sel[p] == c;
      if (taken) continue;
      const float v = cval(c);
      if (v > best || (v == best && c < bidx)) { best = v; bidx = c; }
    }
    bv[tid] = best;
    bi[tid] = bidx;
    __syncthreads();
    if (tid == 0) {
      float bb = bv[0];
      int ii = bi[0];
      for (int x = 1; x < 256; ++x)
        if (bv[x] > bb || (bv[x] == bb && bi[x] < ii)) { bb = bv[x]; ii = bi[x]; }
      sel[m] = ii;
      selv[m] = bb;
    }
    __syncthreads();
  }
  // the first K - finished of the sorted candidates extend their parents (Attention.lua:413-430); at
  // count 0 the one zero-state row offers all K (:369-387), later the K - finished survivors
  if (tid == 0) {
    int nf = 0, nn = 0;
    const int fin = q.nfin[b];
    for (int m = 0; m < K - fin && m < nsel; ++m) {
      const int i = sel[m] / O, j = sel[m] - i * O;
      if (j == q.eos || (count > 0 && count == q.maxlen)) {
        fpar[nf] = i; ftok[nf] = j; fsc[nf] = selv[m]; fdst[nf] = fin + nf; ++nf;
      } else {
        npar[nn] = i; ntok[nn] = j; np_[nn] = selv[m]; ++nn;
      }
    }
    nf_new = nf;
    nn_new = nn;
  }
  __syncthreads();
  const int nf = nf_new, nn = nn_new, L1 = q.maxlen + 1;
  const int* hcur = q.hist + (long)par * R * L1;
  int* hnew = q.hist + (long)nxt * R * L1;
  const int* lcur = q.hlen + par * R;
  int* lnew = q.hlen + nxt * R;
  for (int f = 0; f < nf; ++f) {  // finished hypotheses: parent's tokens + the final token
    const int src = b * K + fpar[f], dst = b * K + fdst[f], len = lcur[src];
    for (int x = tid; x < len; x += 256) q.fseq[(long)dst * L1 + x] = hcur[(long)src * L1 + x];
    if (tid == 0) {
      q.fseq[(long)dst * L1 + len] = ftok[f];
      q.flen[dst] = len + 1;
      q.fscore[dst] = fsc[f];
    }
  }
  float* snew = q.s + (long)nxt * R * S;
  for (int e = 0; e < nn; ++e) {  // surviving hypotheses: gather tokens and the decoder state of the parent
    const int src = b * K + npar[e], dst = b * K + e, len = lcur[src];
    for (int x = tid; x < len; x += 256) hnew[(long)dst * L1 + x] = hcur[(long)src * L1 + x];
    const float* sv = k.VV + ((long)src * 2 + 1) * (S + k.A);
    for (int n = tid; n < S; n += 256) snew[(long)dst * S + n] = sv[n];
    if (q.lstm)
      for (int n = tid; n < S; n += 256)
        q.mem[(long)nxt * R * S + (long)dst * S + n] = k.LC[((long)src * 2 + 1) * S + n];
    if (q.hyb)
      for (int l = tid; l < q.L; l += 256)
        q.alpha[(long)nxt * R * q.L + (long)dst * q.L + l] = k.ALPHA[((long)src * 2 + 1) * q.L + l];
    if (tid == 0) {
      hnew[(long)dst * L1 + len] = ntok[e];
      lnew[dst] = len + 1;
      q.pbeam[dst] = np_[e];
      q.yprev[dst] = ntok[e];
    }
  }
  if (tid == 0) {
    q.nfin[b] += nf;
    q.nact[b] = nn;
    q.done[b] = (q.nfin[b] >= K || count >= q.maxlen) ? 1 : 0;
  }
}

// external decoder_mlp: the step's [s_t; c_t] rows (t = 1 slots) out, the caller's log-probabilities in
__global__ void beam_mlp_rows(AttnK k, BeamK q) {
  const int R = q.B * q.K, W = q.S + k.A;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (long)R * W; i += (long)gridDim.x * blockDim.x) {
    const long r = i / W, c = i - r * W;
    q.mlp_in[i] = k.VV[(r * 2 + 1) * W + c];
  }
}
__global__ void beam_put_logp(AttnK k, BeamK q, const float* logp) {
  const int R = q.B * q.K, O = q.O;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (long)R * O; i += (long)gridDim.x * blockDim.x) {
    const long r = i / O, o = i - r * O;
    k.LOGP[(r * 2 + 1) * O + o] = logp[i];
  }
}

// prediction = y_finished[argmax p_finished] (first maximum)
__global__ void beam_final(BeamK q, int* out, int ldo, int* out_len, float* out_score) {
  const int b = blockIdx.x, K = q.K, L1 = q.maxlen + 1;
  __shared__ int best;
  if (threadIdx.x == 0) {
    int bi = 0;
    float bs = -INFINITY;
    for (int f = 0; f < q.nfin[b]; ++f)
      if (q.fscore[b * K + f] > bs) { bs = q.fscore[b * K + f]; bi = f; }
    best = bi;
    out_len[b] = q.nfin[b] > 0 ? q.flen[b * K + bi] : 0;
    if (out_score) out_score[b] = bs;
  }
  __syncthreads();
  const int len = q.nfin[b] > 0 ? q.flen[b * K + best] : 0;
  for (int x = threadIdx.x; x < ldo; x += blockDim.x)
    out[(long)b * ldo + x] = x < len ? q.fseq[((long)b * K + best) * L1 + x] : -1;
}

// WagnerFischer (utils.lua:3-27): Levenshtein distance of one sequence pair per block
__global__ void edit_distance_kernel(int n, const int* a, const int* alen, int lda, const int* b, const int* blen,
                                     int ldb, int* out) {
  extern __shared__ int row[];
  const int p = blockIdx.x;
  if (p >= n || threadIdx.x != 0) return;
  const int m = alen[p], nb = blen[p];
  const int* x = a + (long)p * lda;
  const int* y = b + (long)p * ldb;
  for (int i = 0; i <= m; ++i) row[i] = i;  // column j = 0: d[i][0] = i
  for (int j = 1; j <= nb; ++j) {
    int diag = row[0];
    row[0] = j;
    for (int i = 1; i <= m; ++i) {
      const int up = row[i];
      row[i] = x[i - 1] == y[j - 1] ? diag : min(min(up + 1, row[i - 1] + 1), diag + 1);
      diag = up;
    }
  }
  out[p] = row[m];
}

AttnDims beam_dims(const AttnDims& d, int K) {
  AttnDims d2 = d;
  d2.B = d.B * K;
  d2.T = 2;
  d2.dropout = 0.f;  // evaluate() mode
  d2.dropout_mask = nullptr;
  d2.flen = nullptr;  // rows are hypotheses; every utterance's annotations are searched whole
  d2.tlen = nullptr;
  return d2;
}

struct BeamLayout {
  size_t hrep, saved, scratch, state, fstate, total;
};
BeamLayout beam_layout(const AttnDims& d, int K, int maxlen) {
  const AttnDims d2 = beam_dims(d, K);
  const size_t R = (size_t)d.B * K, L1 = (size_t)maxlen + 1;
  auto up = [](size_t x) { return (x + 255) / 256 * 256; };
  BeamLayout l;
  l.hrep = 0;
  l.saved = up(sizeof(float) * R * d.L * d.A);
  l.scratch = l.saved + up(attn_saved_bytes(d2));
  l.state = l.scratch + up(attn_scratch_bytes(d2));
  const size_t ints = 3 * (size_t)d.B + R /*yprev*/ + 2 * R * L1 /*hist*/ + 2 * R /*hlen*/ + R * L1 /*fseq*/ +
                      R /*flen*/ + 2 * R /*lab2*/;
  const size_t floats = R /*pbeam*/ + 2 * R * d.S /*s*/ + R /*fscore*/ + 2 * R * d.L /*alpha*/ + 2 * R * d.S /*mem*/ +
                        R * (size_t)(d.S + d.A) /*mlp_in*/;
  l.fstate = l.state + up(4 * ints);
  l.total = l.fstate + up(4 * floats);
  return l;
}

}  // namespace

size_t attn_beam_workspace_bytes(const AttnDims& d, int K, int maxlen) { return beam_layout(d, K, maxlen).total; }

// The beam's device state inside the workspace (beam_layout): the T = 2 decoder problem of R = B*K rows and
// the per-hypothesis bookkeeping.  Every stage re-derives the same views from (d, K, maxlen, ws).
struct BeamView {
  AttnDims d2;
  AttnK k;
  BeamK q;
  float* hrep;
  GemmWs gws;
};
static int beam_view(const AttnDims& d, const AttnParams& P, int eos, int K, int maxlen, void* ws, size_t ws_bytes,
                     BeamView& v) {
  S2S_TRY(attn_check_dims(d));
  S2S_REQUIRE(K >= 1 && K <= kBeamMaxK && K <= d.O, "beam search: K must be in [1, 16] and <= outputDepth");
  S2S_REQUIRE(maxlen >= 1 && eos >= 0 && eos < d.O, "beam search: bad eos / maxlen");
  S2S_REQUIRE(!d.flen, "beam search: frame lengths unsupported (search an utterance's own frames)");
  const BeamLayout bl = beam_layout(d, K, maxlen);
  S2S_REQUIRE(ws && ws_bytes >= bl.total, "beam search: workspace too small");
  v.d2 = beam_dims(d, K);
  char* base = static_cast<char*>(ws);
  v.hrep = reinterpret_cast<float*>(base + bl.hrep);
  v.k = AttnK{};
  carve(v.d2, &v.k, base + bl.saved, base + bl.scratch);
  const int B = d.B, R = B * K, S = d.S, L1 = maxlen + 1;
  BeamK& q = v.q;
  q = BeamK{};
  q.B = B; q.K = K; q.maxlen = maxlen; q.eos = eos; q.S = S; q.O = d.O; q.L = d.L;
  q.hyb = d.hf > 0 ? 1 : 0;
  q.lstm = d.lstm ? 1 : 0;
  int* ip = reinterpret_cast<int*>(base + bl.state);
  q.nact = ip; ip += B;
  q.nfin = ip; ip += B;
  q.done = ip; ip += B;
  q.yprev = ip; ip += R;
  q.hist = ip; ip += 2L * R * L1;
  q.hlen = ip; ip += 2 * R;
  q.fseq = ip; ip += (long)R * L1;
  q.flen = ip; ip += R;
  q.lab2 = ip;
  float* fp = reinterpret_cast<float*>(base + bl.fstate);
  q.pbeam = fp; fp += R;
  q.s = fp; fp += 2L * R * S;
  q.fscore = fp; fp += R;
  q.alpha = fp; fp += 2L * R * d.L;
  q.mem = fp; fp += 2L * R * S;
  q.mlp_in = fp;
  v.k.P = P;
  v.k.h = v.hrep;
  v.k.labels = q.lab2;
  v.k.logp = nullptr;
  v.k.t = 1;
  v.gws = attn_gemm_ws(v.d2, base + bl.scratch);
  return 0;
}

int attn_beam_init(hipStream_t st, const AttnDims& d, const float* h, const AttnParams& P, int eos, int K, int maxlen,
                   void* ws, size_t ws_bytes) {
  BeamView v;
  S2S_TRY(beam_view(d, P, eos, K, maxlen, ws, ws_bytes, v));
  const int B = d.B, R = B * K, L = d.L;
  // annotations and Vh once per hypothesis row (Attention.lua:356-357: vh = Vh:forward(annotations))
  hipLaunchKernelGGL(beam_rep_h, dim3(64, B), dim3(256), 0, st, h, v.hrep, K, (long)L * d.A);
  S2S_TRY(gemm1(st, false, true, R * L, d.Sc, d.A, 1.f, v.hrep, d.A, P.V, d.A, 0.f, v.k.Vh, d.Sc, nullptr, v.gws));
  hipLaunchKernelGGL(beam_init, dim3(64), dim3(256), 0, st, v.q);
  if (d.hf > 0) hipLaunchKernelGGL(dec_hyb_fold, dim3((d.Sc + 255) / 256), dim3(256), 0, st, v.k);
  if (d.lstm) hipLaunchKernelGGL(dec_lstm_pack, dim3(256), dim3(256), 0, st, v.k);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// one decoder_base forward of every active hypothesis (Attention.lua:386-399); with the fused decoder_mlp
// through the log-probabilities, with an external one up to its input rows (beam mlp_in)
int attn_beam_step(hipStream_t st, const AttnDims& d, const AttnParams& P, int K, int maxlen, int count, void* ws,
                   size_t ws_bytes) {
  BeamView v;
  S2S_TRY(beam_view(d, P, 0, K, maxlen, ws, ws_bytes, v));
  AttnK& k = v.k;
  const int R = d.B * K, S = d.S, bt = (R + 15) / 16, rows = 2 * R;
  hipLaunchKernelGGL(beam_prep, dim3(64), dim3(256), 0, st, k, v.q, count & 1);
  hipLaunchKernelGGL(dec_f1_ws, dim3(d.Sc / 16, bt), dim3(256), 0, st, k);
  hipLaunchKernelGGL(dec_f2_attn<8>, dim3(k.NCH, R), dim3(512), 0, st, k);
  hipLaunchKernelGGL(dec_f3_combine, dim3(R), dim3(256), 0, st, k);
  hipLaunchKernelGGL(dec_f4_cin, dim3(S / 16, bt), dim3(256), 0, st, k);
  hipLaunchKernelGGL(dec_f5_d, dim3(S / 16, bt), dim3(256), 0, st, k);
  if (d.lstm) {
    hipLaunchKernelGGL(dec_f6_lstm, dim3(4 * S / 16, bt), dim3(512), 0, st, k);
  } else {
    hipLaunchKernelGGL(dec_f6_gru1, dim3(2 * S / 16, bt), dim3(256), 0, st, k);
    hipLaunchKernelGGL(dec_f7_gru2, dim3(S / 16, bt), dim3(256), 0, st, k);
  }
  if (d.ext) {
    hipLaunchKernelGGL(beam_mlp_rows, dim3(256), dim3(256), 0, st, k, v.q);
  } else {
    S2S_TRY(gemm1(st, false, true, rows, d.M * d.K, S + d.A, 1.f, k.VV, S + d.A, P.Wm, S + d.A, 0.f, k.U,
                  (long)d.M * d.K, P.bm, v.gws));
    hipLaunchKernelGGL(dec_mlp_head, dim3((rows + 3) / 4), dim3(256), 4 * d.M * sizeof(float), st, k, rows);
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

const float* attn_beam_mlp_input(const AttnDims& d, int K, int maxlen, void* ws) {
  BeamView v;
  AttnParams P{};
  if (beam_view(d, P, 0, K, maxlen, ws, beam_layout(d, K, maxlen).total, v) != 0) return nullptr;
  return v.q.mlp_in;
}

// topk + bookkeeping of the step (Attention.lua:400-430); logp_ext: (R, O) log-probabilities of an external
// decoder_mlp (null with the fused one)
int attn_beam_advance(hipStream_t st, const AttnDims& d, int eos, int K, int maxlen, int count, const float* logp_ext,
                      void* ws, size_t ws_bytes) {
  BeamView v;
  AttnParams P{};
  S2S_TRY(beam_view(d, P, eos, K, maxlen, ws, ws_bytes, v));
  S2S_REQUIRE(!d.ext || logp_ext, "beam search: an external decoder_mlp needs the step's log-probabilities");
  if (logp_ext) hipLaunchKernelGGL(beam_put_logp, dim3(256), dim3(256), 0, st, v.k, v.q, logp_ext);
  hipLaunchKernelGGL(beam_update, dim3(d.B), dim3(256), 0, st, v.k, v.q, count);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int attn_beam_done(hipStream_t st, const AttnDims& d, int K, int maxlen, void* ws, int* all_done) {
  BeamView v;
  AttnParams P{};
  S2S_TRY(beam_view(d, P, 0, K, maxlen, ws, beam_layout(d, K, maxlen).total, v));
  std::vector<int> done(d.B);
  S2S_CHECK_HIP(hipMemcpyAsync(done.data(), v.q.done, sizeof(int) * d.B, hipMemcpyDeviceToHost, st));
  S2S_CHECK_HIP(hipStreamSynchronize(st));
  bool all = true;
  for (int x : done) all = all && x;
  *all_done = all ? 1 : 0;
  return 0;
}

int attn_beam_finish(hipStream_t st, const AttnDims& d, int K, int maxlen, void* ws, int* out, int ldo, int* out_len,
                     float* out_score) {
  BeamView v;
  AttnParams P{};
  S2S_TRY(beam_view(d, P, 0, K, maxlen, ws, beam_layout(d, K, maxlen).total, v));
  S2S_REQUIRE(ldo >= maxlen + 1, "beam search: ldo < maxseqlength + 1");
  hipLaunchKernelGGL(beam_final, dim3(d.B), dim3(256), 0, st, v.q, out, ldo, out_len, out_score);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int attn_beam_search(hipStream_t st, const AttnDims& d, const float* h, const AttnParams& P, int eos, int K,
                     int maxlen, int* out, int ldo, int* out_len, float* out_score, void* ws, size_t ws_bytes) {
  S2S_REQUIRE(!d.ext, "beam search: an external decoder_mlp runs through the stepwise calls");
  S2S_REQUIRE(ldo >= maxlen + 1, "beam search: ldo < maxseqlength + 1");
  S2S_TRY(attn_beam_init(st, d, h, P, eos, K, maxlen, ws, ws_bytes));
  for (int count = 0; count <= maxlen; ++count) {
    S2S_TRY(attn_beam_step(st, d, P, K, maxlen, count, ws, ws_bytes));
    S2S_TRY(attn_beam_advance(st, d, eos, K, maxlen, count, nullptr, ws, ws_bytes));
    if ((count & 3) == 3 || count == maxlen) {  // stop once every utterance has K finished hypotheses
      int all = 0;
      S2S_TRY(attn_beam_done(st, d, K, maxlen, ws, &all));
      if (all) break;
    }
  }
  return attn_beam_finish(st, d, K, maxlen, ws, out, ldo, out_len, out_score);
}

int edit_distance(hipStream_t st, int n, const int* a, const int* alen, int lda, const int* b, const int* blen,
                  int ldb, int* out) {
  S2S_REQUIRE(n >= 0 && lda >= 0 && ldb >= 0 && lda < 16384, "edit distance: bad sizes");
  if (n == 0) return 0;
  hipLaunchKernelGGL(edit_distance_kernel, dim3(n), dim3(64), sizeof(int) * (lda + 1), st, n, a, alen, lda, b, blen,
                     ldb, out);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int nll_seed(hipStream_t st, int B, int T, int O, const float* logp, const int* labels, int normalize, float* nll,
             float* dlogp, const int* tlen) {
  hipLaunchKernelGGL(nll_seed_kernel, dim3(B), dim3(256), 0, st, B, T, O, logp, labels, normalize, nll, dlogp, tlen);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace s2s

// Diagnostic (not part of the C ABI header): device buffers of uint64 s_memrealtime stamps the persistent
// decoder kernels fill at phase ends -- (grid, T, 8) for attn_persist.inc, (chains * 32, T, 16) for
// dec_xcd.inc (tools/xdec_stamps.py, tools/xdec_substamps.py); nullptr turns it off.
// diagnostic: 0 forces write-through (sc1) hand-offs in every XCD-local decoder chain
extern "C" void s2s_debug_dec_local(int allow) { s2s::g_dec_allow_local = allow; }
extern "C" void s2s_debug_merge_alpha_head(int on) { s2s::g_merge_alpha_head = on; }
// diagnostic: the merged MLP head sums the MLP GEMM's split-K slabs (1) or a reduce launch runs in front of it (0)
extern "C" void s2s_debug_head_sums_slabs(int on) { s2s::g_head_sums_slabs = on; }
extern "C" void s2s_debug_dec_r4(int on) { s2s::g_dec_r4 = on; }
extern "C" void s2s_debug_dvh_wide(int on) {
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(s2s::g_dvh_force_wide), &v, sizeof(int));
}
extern "C" void s2s_debug_dec_mode(int m) { s2s::g_dec_mode_force = m; }
extern "C" void s2s_debug_dec_pf(int on) {  // 0: the XCD decoder's per-term attention form everywhere (A/B, tests)
  const int v = on ? 1 : 0;
  (void)hipMemcpyToSymbol(HIP_SYMBOL(s2s::g_dec_pf), &v, sizeof(int));
}
extern "C" int s2s_debug_dec_stamps(void* fwd, void* bwd) {
  s2s::g_dec_stamps[0] = static_cast<unsigned long long*>(fwd);
  s2s::g_dec_stamps[1] = static_cast<unsigned long long*>(bwd);
  return 0;
}

namespace s2s {
int set_device_u64(hipStream_t st, unsigned long long* p, unsigned long long v) {
  hipLaunchKernelGGL(set_u64_kernel, dim3(1), dim3(64), 0, st, p, v);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}
}  // namespace s2s
