// LSTM layer sequence forward/backward: the drop-in for nn.RNN(nn.LSTM(D, H, peepholes), reverse)
// (LSTM.lua:6-136 under RNN.lua:120-201) -- SURVEY.md §8 row A7.
//
// Reference cell (LSTM.lua:16-58), every gate Linear(D,H)(x) + Linear(H,H)(h) with biases:
//   i = sig(Wix x + Wih h [+ Wic c])   f = sig(Wfx x + Wfh h [+ Wfc c])   g = tanh(Wgx x + Wgh h)
//   c' = f*c + i*g                      o = sig(Wox x + Woh h [+ Woc c'])  h' = o * tanh(c')
// (peepholes are full H x H matrices with biases; the o gate peeks the NEW cell, LSTM.lua:47-50).
// MI355X decomposition (same building blocks as gru.hip):
//   * the x-half of all four gates, with every constant bias folded in, is ONE hoisted MFMA GEMM
//     over all B*L rows, both directions in the same launch;
//   * per step: k1 skinny MFMA [i|f|g|o] from [h_{t-1} (; c_{t-1})], k2 the cell update, and with
//     peepholes k3 the o gate from c_t (skinny over the new cell);
//   * BPTT per step: b1 elementwise (do, dc, gate pre-activation grads), b2 (peepholes) dc += Woc^T
//     da_o first, b3 one skinny launch for [dh_{t-1} | dc_{t-1}];
//   * dx and every dW / db are GEMMs / column sums over all B*L rows after the sweep.
// Saved per direction: sv (B, L, 8H) = i | f | g | o | c | c_{t-1} | h_{t-1} | tanh(c).
#include "lstm.h"

#include "skinny.h"

namespace s2s {

namespace {

struct LstmFwdDir {
  const float* xp;   // (B, L, ldxp): [i | f | g | o] x-projections + all biases
  long ldxp;
  const float* Wh[4];  // Wqh (H, H)
  const float* Wc[3];  // Wic, Wfc, Woc (H, H) or null
  float* y;
  long ldy;
  float* sv;
  int reverse;
};
struct LstmFwdArgs {
  LstmFwdDir d[2];
  int B, L, H, peep, step;
  const int* len;  // (B) frames per utterance or null: h_t = c_t = 0 for t >= len_b
};

// k1: gate pre-activations.  Workgroup tile = 16 columns of one gate q = n0 / H.
__global__ __launch_bounds__(256) void lstm_fwd_gates(LstmFwdArgs a) {
  __shared__ SkinnyRed red;
  const LstmFwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tp = g.reverse ? t + 1 : t - 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int q = n0 / H, j0 = n0 - q * H;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (step > 0) {
    const int br = min(b0 + (lane & 15), B - 1);
    acc = skinny_wave(g.y + ((long)br * L + tp) * g.ldy, g.Wh[q] + (long)(j0 + (lane & 15)) * H, H, wave, lane);
    if (a.peep && q < 2) {
      const floatx4 pc = skinny_wave(g.sv + ((long)br * L + tp) * SV_N * H + SV_C * H,
                                     g.Wc[q] + (long)(j0 + (lane & 15)) * H, H, wave, lane);
      acc += pc;
    }
  }
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), j = j0 + (tid & 15);
  if (b >= B) return;
  const long row = (long)b * L + t;
  const float pre = s + g.xp[row * g.ldxp + q * H + j];
  float* sv = g.sv + row * SV_N * H;
  float v;
  if (q == 2) v = tanhf(pre);
  else if (q == 3 && a.peep) v = pre;  // o gate completed by k3 (peeks the new cell)
  else v = sigmoidf_(pre);
  sv[q * H + j] = v;
  if (q == 0) {
    sv[SV_HP * H + j] = step > 0 ? g.y[((long)b * L + tp) * g.ldy + j] : 0.f;
    sv[SV_CP * H + j] = step > 0 ? g.sv[((long)b * L + tp) * SV_N * H + SV_C * H + j] : 0.f;
  }
}

// k2: c' = f*c + i*g (LSTM.lua:45-46); without peepholes also h' = o * tanh(c')
__global__ void lstm_fwd_cell(LstmFwdArgs a) {
  const LstmFwdDir& g = a.d[blockIdx.y];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H) return;
  const int b = idx / H, j = idx - b * H;
  const int t = g.reverse ? L - 1 - step : step;
  const long row = (long)b * L + t;
  float* sv = g.sv + row * SV_N * H;
  const float cp = step > 0 ? g.sv[((long)b * L + (g.reverse ? t + 1 : t - 1)) * SV_N * H + SV_C * H + j] : 0.f;
  float c = sv[SV_F * H + j] * cp + sv[SV_I * H + j] * sv[SV_G * H + j];
  if (a.len && t >= a.len[b]) c = 0.f;  // padding frame: zero state (the o gate's k3 then gives h = 0)
  sv[SV_C * H + j] = c;
  if (!a.peep) {
    const float tc = tanhf(c);
    sv[SV_TC * H + j] = tc;
    g.y[row * g.ldy + j] = sv[SV_O * H + j] * tc;
  }
}

// k1 + k2 in one launch (no peepholes): the 1024-thread workgroup computes all four gates of its 16 units -- four
// skinny products in the same order as lstm_fwd_gates, one per four waves (skinny4_1024) -- then the cell update of
// those units (bitwise equal to the two-launch form, one launch per step fewer)
__global__ __launch_bounds__(1024) void lstm_fwd_step(LstmFwdArgs a) {
  __shared__ SkinnyRed red[4];
  const LstmFwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tp = g.reverse ? t + 1 : t - 1;
  const int tid = threadIdx.x, lane = tid & 63;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int br = min(b0 + (lane & 15), B - 1);
  float s[4];
  skinny4_1024(red, g.y + ((long)br * L + (step > 0 ? tp : t)) * g.ldy,
               [&](int q) { return g.Wh[q] + (long)(j0 + (lane & 15)) * H; }, H, step == 0, s);
  const int b = b0 + (tid >> 4), j = j0 + (tid & 15);
  if (tid >= 256 || b >= B) return;
  const long row = (long)b * L + t;
  const float* xp = g.xp + row * g.ldxp;
  float* sv = g.sv + row * SV_N * H;
  const float gi = sigmoidf_(s[0] + xp[j]), gf = sigmoidf_(s[1] + xp[H + j]);
  const float gg = tanhf(s[2] + xp[2 * H + j]), go = sigmoidf_(s[3] + xp[3 * H + j]);
  sv[SV_I * H + j] = gi;
  sv[SV_F * H + j] = gf;
  sv[SV_G * H + j] = gg;
  sv[SV_O * H + j] = go;
  const float cp = step > 0 ? g.sv[((long)b * L + tp) * SV_N * H + SV_C * H + j] : 0.f;
  sv[SV_HP * H + j] = step > 0 ? g.y[((long)b * L + tp) * g.ldy + j] : 0.f;
  sv[SV_CP * H + j] = cp;
  float c = gf * cp + gi * gg, tc = tanhf(c), h = go * tc;
  if (a.len && t >= a.len[b]) c = tc = h = 0.f;  // padding frame: zero state and output
  sv[SV_C * H + j] = c;
  sv[SV_TC * H + j] = tc;
  g.y[row * g.ldy + j] = h;
}

// k3 (peepholes): o = sig(pre_o + Woc c'), h' = o * tanh(c')
__global__ __launch_bounds__(256) void lstm_fwd_ogate(LstmFwdArgs a) {
  __shared__ SkinnyRed red;
  const LstmFwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int br = min(b0 + (lane & 15), B - 1);
  const floatx4 acc = skinny_wave(g.sv + ((long)br * L + t) * SV_N * H + SV_C * H,
                                  g.Wc[2] + (long)(n0 + (lane & 15)) * H, H, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), j = n0 + (tid & 15);
  if (b >= B) return;
  const long row = (long)b * L + t;
  float* sv = g.sv + row * SV_N * H;
  const float o = sigmoidf_(sv[SV_O * H + j] + s);
  const float tc = tanhf(sv[SV_C * H + j]);
  sv[SV_O * H + j] = o;
  sv[SV_TC * H + j] = tc;
  g.y[row * g.ldy + j] = o * tc;
}

struct LstmBwdDir {
  const float* dy;
  long lddy;
  const float* sv;
  const float* WocT;  // (H, H) WocT[m][j] = Woc[j][m]   (peepholes)
  const float* Wb;    // (2H, 4H): rows m < H: [Wih; Wfh; Wgh; Woh][:, m];  rows H + m: [Wic; Wfc; 0; 0][:, m]
  float* dA;          // dA[(b*L+t)*ldA + q*H + j]: gate pre-activation gradients
  long ldA;
  float* dhc;  // (B, H) carried dL/dh_t
  float* dcc;  // (B, H) carried dL/dc_t
  float* dcp;  // (B, H) partial dL/dc_{t-1} = dc_t * f
  float* dcn;  // (B, H) dL/dc_t before the o-gate peephole term (peepholes)
  int reverse;
};
struct LstmBwdArgs {
  LstmBwdDir d[2];
  int B, L, H, peep, step;
  const int* len;  // (B) frames per utterance or null: dL/dh_t = dL/dc_t = 0 for t >= len_b
};

// cell-side gate gradients from the complete dL/dc_t (LSTM.lua:118-136 via the graph)
__device__ __forceinline__ void lstm_cell_grads(const LstmBwdDir& g, int H, long row, int b, int j, float dc) {
  const float* sv = g.sv + row * SV_N * H;
  const float i = sv[SV_I * H + j], f = sv[SV_F * H + j], gg = sv[SV_G * H + j], cp = sv[SV_CP * H + j];
  float* dA = g.dA + row * g.ldA;
  dA[0 * H + j] = (dc * gg) * (i * (1.0f - i));
  dA[1 * H + j] = (dc * cp) * (f * (1.0f - f));
  dA[2 * H + j] = (dc * i) * (1.0f - gg * gg);
  g.dcp[b * H + j] = dc * f;
}

// b1: dh = dy + carry; do, dc (+ the h' = o*tanh(c') path); da_o; without peepholes the rest
__global__ void lstm_bwd_elem(LstmBwdArgs a) {
  const LstmBwdDir& g = a.d[blockIdx.y];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * H) return;
  const int b = idx / H, j = idx - b * H;
  const int t = g.reverse ? L - 1 - step : step;
  const long row = (long)b * L + t;
  const float* sv = g.sv + row * SV_N * H;
  const float o = sv[SV_O * H + j], tc = sv[SV_TC * H + j];
  const bool pad = a.len && t >= a.len[b];
  const float dh = pad ? 0.f : g.dy[row * g.lddy + j] + g.dhc[idx];
  const float dc = pad ? 0.f : g.dcc[idx] + dh * o * (1.0f - tc * tc);
  g.dA[row * g.ldA + 3 * H + j] = (dh * tc) * (o * (1.0f - o));
  if (a.peep) g.dcn[idx] = dc;
  else lstm_cell_grads(g, H, row, b, j, dc);
}

// b2 (peepholes): dc_t += Woc^T da_o (the o gate peeks c_t), then the cell-side gate grads
__global__ __launch_bounds__(256) void lstm_bwd_peep(LstmBwdArgs a) {
  __shared__ SkinnyRed red;
  const LstmBwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int br = min(b0 + (lane & 15), B - 1);
  const floatx4 acc = skinny_wave(g.dA + ((long)br * L + t) * g.ldA + 3 * H, g.WocT + (long)(n0 + (lane & 15)) * H,
                                  H, wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), j = n0 + (tid & 15);
  if (b >= B) return;
  lstm_cell_grads(g, H, (long)b * L + t, b, j, g.dcn[b * H + j] + s);
}

// b3: [dh_{t-1} | dc_{t-1}] = Wb [da_i; da_f; da_g; da_o] (+ dc*f for the cell); columns < H are
// dh, columns >= H dc (peepholes add [Wic; Wfc]^T [da_i; da_f])
__global__ __launch_bounds__(256) void lstm_bwd_carry(LstmBwdArgs a) {
  __shared__ SkinnyRed red;
  const LstmBwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const bool cpart = n0 >= H;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (!cpart || a.peep) {
    const int br = min(b0 + (lane & 15), B - 1);
    acc = skinny_wave(g.dA + ((long)br * L + t) * g.ldA, g.Wb + (long)(n0 + (lane & 15)) * 4 * H,
                      cpart ? 2 * H : 4 * H, wave, lane);
  }
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= B) return;
  if (cpart) g.dcc[b * H + n - H] = g.dcp[b * H + n - H] + s;
  else g.dhc[b * H + n] = s;
}

// b3 of step s + 1 and b1 of step s in one launch (no peepholes): the workgroup's 16 units get dL/dh_t from the
// skinny product over the row the previous launch wrote (dc_t = dc_{t+1} * f, the dc half of b3 being zero
// without peepholes), then their gate pre-activation gradients -- the same sums as lstm_bwd_carry +
// lstm_bwd_elem, one launch per step (the product in 512-thread workgroups, skinny_wave8).  At the first step of
// the sweep (first = 1) the carries are zero.
__global__ __launch_bounds__(512) void lstm_bwd_step(LstmBwdArgs a, int first) {
  __shared__ SkinnyRed8 red;
  const LstmBwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tn = g.reverse ? t - 1 : t + 1;  // the row of step + 1 (processed by the previous launch)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (!first) {
    const int br = min(b0 + (lane & 15), B - 1);
    acc = skinny_wave8(g.dA + ((long)br * L + tn) * g.ldA, g.Wb + (long)(j0 + (lane & 15)) * 4 * H, 4 * H, wave, lane);
  }
  const float sh = skinny_reduce8(red, acc, wave, lane, tid);
  if (tid >= 256) return;
  const int b = b0 + (tid >> 4), j = j0 + (tid & 15);
  if (b >= B) return;
  const int idx = b * H + j;
  const float dhc = first ? 0.f : sh;
  const float dcc = first ? 0.f : g.dcp[idx] + 0.f;  // lstm_bwd_carry's dc column: dcp + (a zero product)
  const long row = (long)b * L + t;
  const float* sv = g.sv + row * SV_N * H;
  const float o = sv[SV_O * H + j], tc = sv[SV_TC * H + j];
  const bool pad = a.len && t >= a.len[b];
  const float dh = pad ? 0.f : g.dy[row * g.lddy + j] + dhc;
  const float dc = pad ? 0.f : dcc + dh * o * (1.0f - tc * tc);
  g.dA[row * g.ldA + 3 * H + j] = (dh * tc) * (o * (1.0f - o));
  lstm_cell_grads(g, H, row, b, j, dc);
}

// packs: Wx4 (4H, D) rows [Wix; Wfx; Wgx; Wox]; bias4 (4H) = bqx + bqh (+ bqc for i, f, o);
// Wb (2H, 4H) as lstm_bwd_carry reads it; WocT (H, H)
struct LstmPackArgs {
  const float* W[kLstmPeepParams];
  float *Wx4, *bias4, *Wb, *WocT;
  int H, D, peep;
};
__global__ void lstm_pack(LstmPackArgs p) {
  const int H = p.H, D = p.D;
  const long nX = 4L * H * D, nB = 4L * H, nW = p.Wb ? 2L * H * 4 * H : 0, nT = (p.WocT && p.peep) ? (long)H * H : 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < nX + nB + nW + nT; i += (long)gridDim.x * blockDim.x) {
    if (i < nX) {
      if (!p.Wx4) continue;
      const int q = (int)(i / ((long)H * D));
      const long r = i - (long)q * H * D;
      p.Wx4[i] = p.W[4 * q][r];
    } else if (i < nX + nB) {
      if (!p.bias4) continue;
      const int n = (int)(i - nX), q = n / H, j = n - q * H;
      float b = p.W[4 * q + 1][j] + p.W[4 * q + 3][j];
      if (p.peep && q != 2) b += p.W[kLstmParams + 2 * (q == 3 ? 2 : q) + 1][j];
      p.bias4[n] = b;
    } else if (i < nX + nB + nW) {
      const long e = i - nX - nB;
      const int m = (int)(e / (4L * H)), k = (int)(e - (long)m * 4 * H);
      const int q = k / H, jj = k - q * H;
      float v = 0.f;
      if (m < H) v = p.W[4 * q + 2][(long)jj * H + m];
      else if (p.peep && q < 2) v = p.W[kLstmParams + 2 * q][(long)jj * H + (m - H)];
      p.Wb[e] = v;
    } else {
      const long e = i - nX - nB - nW;
      const int m = (int)(e / H), j = (int)(e - (long)m * H);
      p.WocT[e] = p.W[kLstmParams + 4][(long)j * H + m];
    }
  }
}

int launch_lstm_pack(hipStream_t st, const float* const* W, int H, int D, int peep, float* Wx4, float* bias4,
                     float* Wb, float* WocT) {
  LstmPackArgs p{};
  for (int i = 0; i < lstm_nparams(peep); ++i) p.W[i] = W[i];
  p.Wx4 = Wx4; p.bias4 = bias4; p.Wb = Wb; p.WocT = WocT; p.H = H; p.D = D; p.peep = peep;
  const long n = 4L * H * D + 4L * H + (Wb ? 8L * H * H : 0) + ((WocT && peep) ? (long)H * H : 0);
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(lstm_pack, dim3(blocks), dim3(256), 0, st, p);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

__global__ void bias_rows_kernel(float* C, long ldc, int rows, int cols, const float* bias) {
  const long n = (long)rows * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, c = i - r * cols;
    C[r * ldc + c] = bias[c];
  }
}

struct Carve {
  float *Wx4, *bias4, *xp, *dA, *Wb[2], *WocT[2], *dhc[2], *dcc[2], *dcp[2], *dcn[2];
  GemmWs ws;
  void* sync;  // the persistent launches' hand-off region (lstm_persist_sync_bytes)
  size_t bytes;
};
Carve carve(void* scratch, int nd, int B, int L, int D, int H, int peep) {
  Carve c{};
  Bump bp{static_cast<char*>(scratch), 0, 0};
  c.Wx4 = bp.take<float>(4L * nd * H * D);
  c.bias4 = bp.take<float>(4L * nd * H);
  c.xp = bp.take<float>((long)B * L * 4 * nd * H);  // forward: x-projections; backward: gate gradients
  c.dA = c.xp;
  for (int d = 0; d < 2; ++d) {
    c.Wb[d] = bp.take<float>(8L * H * H);
    c.WocT[d] = bp.take<float>((long)H * H);
    c.dhc[d] = bp.take<float>((long)B * H);
    c.dcc[d] = bp.take<float>((long)B * H);
    c.dcp[d] = bp.take<float>((long)B * H);
    c.dcn[d] = bp.take<float>((long)B * H);
  }
  c.ws = GemmWs{bp.take<float>(kGemmWsFloats), kGemmWsFloats};
  // the persistent launches' hand-off region, only where they run (lstm_persist_supported)
  c.sync = lstm_persist_supported(nd, B, H, peep) ? bp.take<char>(lstm_persist_sync_bytes(nd, B, L, H)) : nullptr;
  c.bytes = bp.off + 256;
  return c;
}

int check(const LstmLayerIO& io) {
  S2S_REQUIRE(io.ndir == 1 || io.ndir == 2, "lstm: ndir must be 1 or 2");
  S2S_REQUIRE(io.B > 0 && io.L > 0 && io.D > 0 && io.H > 0, "lstm: empty dims");
  S2S_REQUIRE(io.H % 16 == 0, "lstm: H must be a multiple of 16");
  S2S_REQUIRE(io.ldy % 4 == 0 && io.ldy >= io.H, "lstm: ldy must be a multiple of 4 and >= H");
  S2S_REQUIRE(io.x && io.W, "lstm: null x / W");
  return 0;
}

}  // namespace

size_t lstm_saved_bytes(int B, int L, int H) { return sizeof(float) * (size_t)B * L * SV_N * H; }
size_t lstm_scratch_bytes(int ndir, int B, int L, int D, int H, int peep) {
  return carve(nullptr, ndir, B, L, D, H, peep).bytes;
}

int lstm_layer_fwd(hipStream_t st, const LstmLayerIO& io, void* scratch, size_t scratch_bytes) {
  S2S_TRY(check(io));
  const int nd = io.ndir, B = io.B, L = io.L, D = io.D, H = io.H, np = lstm_nparams(io.peep);
  S2S_REQUIRE(scratch_bytes >= lstm_scratch_bytes(nd, B, L, D, H, io.peep), "lstm: scratch too small");
  Carve c = carve(scratch, nd, B, L, D, H, io.peep);
  for (int d = 0; d < nd; ++d)
    S2S_TRY(launch_lstm_pack(st, io.W + d * np, H, D, io.peep, c.Wx4 + 4L * d * H * D, c.bias4 + 4L * d * H, nullptr,
                             nullptr));
  // xp (B*L, 4*nd*H) = bias4 + x Wx4^T  (GEMM bias epilogue)
  S2S_TRY(gemm1(st, false, true, B * L, 4 * nd * H, D, 1.f, io.x, io.ldx, c.Wx4, D, 0.f, c.xp, 4L * nd * H, c.bias4,
                c.ws));
  if (lstm_persist_supported(nd, B, H, io.peep)) {  // the whole sweep in one launch (lstm_persist.hip)
    LstmPersistArgs f{};
    f.ndir = nd; f.B = B; f.L = L; f.H = H; f.ldxp = 4L * nd * H; f.ldy = io.ldy; f.len = io.len;
    for (int d = 0; d < nd; ++d) {
      const float* const* W = io.W + d * np;
      f.reverse[d] = io.reverse[d];
      f.xp[d] = c.xp + 4L * d * H;
      for (int q = 0; q < 4; ++q) f.Wh[d][q] = W[4 * q + 2];
      f.y[d] = io.y[d];
      f.sv[d] = io.saved[d];
    }
    return lstm_persist_fwd(st, f, c.sync, io.status);
  }
  LstmFwdArgs a{};
  for (int d = 0; d < nd; ++d) {
    const float* const* W = io.W + d * np;
    a.d[d] = LstmFwdDir{c.xp + 4L * d * H, 4L * nd * H, {W[2], W[6], W[10], W[14]},
                        {io.peep ? W[16] : nullptr, io.peep ? W[18] : nullptr, io.peep ? W[20] : nullptr},
                        io.y[d], io.ldy, io.saved[d], io.reverse[d]};
  }
  a.B = B; a.L = L; a.H = H; a.peep = io.peep; a.len = io.len;
  const dim3 gg(4 * H / 16, (B + 15) / 16, nd), gc((B * H + 255) / 256, nd), go(H / 16, (B + 15) / 16, nd);
  ProfScope ps(st, "lstm_fwd_steps", 2.0 * nd * B * L * 4.0 * H * H * (io.peep ? 1.75 : 1.0), 0.0);
  const dim3 gs(H / 16, (B + 15) / 16, nd);
  for (int s = 0; s < L; ++s) {
    a.step = s;
    if (io.peep) {
      hipLaunchKernelGGL(lstm_fwd_gates, gg, dim3(256), 0, st, a);
      hipLaunchKernelGGL(lstm_fwd_cell, gc, dim3(256), 0, st, a);
      hipLaunchKernelGGL(lstm_fwd_ogate, go, dim3(256), 0, st, a);
    } else {
      hipLaunchKernelGGL(lstm_fwd_step, gs, dim3(1024), 0, st, a);
    }
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int lstm_layer_bwd(hipStream_t st, const LstmLayerIO& io, const LstmLayerGrad& gr, void* scratch,
                   size_t scratch_bytes) {
  S2S_TRY(check(io));
  const int nd = io.ndir, B = io.B, L = io.L, D = io.D, H = io.H, np = lstm_nparams(io.peep);
  S2S_REQUIRE(scratch_bytes >= lstm_scratch_bytes(nd, B, L, D, H, io.peep), "lstm: scratch too small");
  S2S_REQUIRE(gr.dW != nullptr, "lstm: null dW");
  Carve c = carve(scratch, nd, B, L, D, H, io.peep);
  const long ldA = 4L * nd * H;
  LstmBwdArgs a{};
  for (int d = 0; d < nd; ++d) {
    S2S_TRY(launch_lstm_pack(st, io.W + d * np, H, D, io.peep, c.Wx4 + 4L * d * H * D, nullptr, c.Wb[d],
                             io.peep ? c.WocT[d] : nullptr));
    if (io.peep) {  // (the fused step of the peephole-free form starts from zero carries itself)
      S2S_TRY(zero_async(st, c.dhc[d], sizeof(float) * (size_t)B * H));
      S2S_TRY(zero_async(st, c.dcc[d], sizeof(float) * (size_t)B * H));
    }
    a.d[d] = LstmBwdDir{gr.dy[d], gr.lddy, io.saved[d], c.WocT[d], c.Wb[d], c.dA + 4L * d * H, ldA,
                        c.dhc[d], c.dcc[d], c.dcp[d], c.dcn[d], io.reverse[d]};
  }
  a.B = B; a.L = L; a.H = H; a.peep = io.peep; a.len = io.len;
  const dim3 ge((B * H + 255) / 256, nd), gp(H / 16, (B + 15) / 16, nd), gb(2 * H / 16, (B + 15) / 16, nd);
  if (lstm_persist_supported(nd, B, H, io.peep)) {  // the whole BPTT sweep in one launch (lstm_persist.hip)
    LstmPersistArgs b{};
    b.ndir = nd; b.B = B; b.L = L; b.H = H; b.lddy = gr.lddy; b.ldA = ldA; b.len = io.len;
    for (int d = 0; d < nd; ++d) {
      b.reverse[d] = io.reverse[d];
      b.Wb[d] = c.Wb[d];
      b.sv[d] = io.saved[d];
      b.dy[d] = gr.dy[d];
      b.dA[d] = c.dA + 4L * d * H;
    }
    S2S_TRY(lstm_persist_bwd(st, b, c.sync, io.status));
  } else {
    ProfScope ps(st, "lstm_bwd_steps", 2.0 * nd * B * L * 4.0 * H * H * (io.peep ? 1.75 : 1.0), 0.0);
    const dim3 gs(H / 16, (B + 15) / 16, nd);
    for (int s = L - 1; s >= 0; --s) {
      a.step = s;
      if (io.peep) {
        hipLaunchKernelGGL(lstm_bwd_elem, ge, dim3(256), 0, st, a);
        hipLaunchKernelGGL(lstm_bwd_peep, gp, dim3(256), 0, st, a);
        if (s > 0) hipLaunchKernelGGL(lstm_bwd_carry, gb, dim3(256), 0, st, a);
      } else {
        hipLaunchKernelGGL(lstm_bwd_step, gs, dim3(512), 0, st, a, s == L - 1 ? 1 : 0);
      }
    }
    S2S_CHECK_HIP(hipGetLastError());
  }
  // weight gradients beside the caller's next launches when it forks them (LstmLayerGrad::wst); dx and the
  // parameter gradients split the split-K workspace in halves either way (the same plans, bitwise the same sums)
  const GemmWs wsx{c.ws.p, c.ws.n / 2}, wsw{c.ws.p + c.ws.n / 2, c.ws.n - c.ws.n / 2};
  hipStream_t pst = st;
  if (gr.wst && gr.wst != st && gr.wev) {
    S2S_CHECK_HIP(hipEventRecord(gr.wev, st));
    S2S_CHECK_HIP(hipStreamWaitEvent(gr.wst, gr.wev, 0));
    pst = gr.wst;
  }
  // dx (+)= dA (B*L, 4*nd*H) . Wx4 (4*nd*H, D): both directions summed (RNN.lua:196)
  if (gr.dx)
    S2S_TRY(gemm1(st, false, false, B * L, D, 4 * nd * H, 1.f, c.dA, ldA, c.Wx4, D, gr.dx_accumulate ? 1.f : 0.f,
                  gr.dx, gr.lddx, nullptr, wsx));
  st = pst;
  // weight gradients over all B*L rows (Linear:accGradParameters per step, summed)
  for (int d = 0; d < nd; ++d) {
    float* const* G = gr.dW + d * np;
    const float* dAd = c.dA + 4L * d * H;
    const float* sv = io.saved[d];
    const long lsv = (long)SV_N * H;
    GemmProblem pr[11];
    int n = 0;
    for (int q = 0; q < 4; ++q) {
      pr[n++] = GemmProblem{dAd + q * H, io.x, G[4 * q], nullptr, ldA, io.ldx, D, H, D, B * L, gr.scale, 1.f};
      pr[n++] = GemmProblem{dAd + q * H, sv + SV_HP * H, G[4 * q + 2], nullptr, ldA, lsv, H, H, H, B * L, gr.scale,
                            1.f};
    }
    if (io.peep) {
      pr[n++] = GemmProblem{dAd, sv + SV_CP * H, G[16], nullptr, ldA, lsv, H, H, H, B * L, gr.scale, 1.f};
      pr[n++] = GemmProblem{dAd + H, sv + SV_CP * H, G[18], nullptr, ldA, lsv, H, H, H, B * L, gr.scale, 1.f};
      pr[n++] = GemmProblem{dAd + 3 * H, sv + SV_C * H, G[20], nullptr, ldA, lsv, H, H, H, B * L, gr.scale, 1.f};
    }
    {
    WgradPrecision wp;  // weight gradients: fp32 under S2S_PREC_BF16_GEMM
    S2S_TRY(gemm_f32(st, pr, n, true, false, wsw));
  }
  }
  // every bias gradient (bqx = bqh = sum_rows da_q, + bqc with peepholes) of both directions: the column sums of
  // dA in one pass
  ColsumOut outs[8];
  int no = 0;
  for (int d = 0; d < nd; ++d) {
    float* const* G = gr.dW + d * np;
    for (int q = 0; q < 4; ++q) {
      ColsumOut& o = outs[no++];
      o = ColsumOut{(int)(4L * d * H + q * H), H, {G[4 * q + 1], G[4 * q + 3], nullptr}, 2};
      if (io.peep && q != 2) o.dst[o.ndst++] = G[kLstmParams + 2 * (q == 3 ? 2 : q) + 1];
    }
  }
  S2S_TRY(colsum_scatter_f32(st, c.dA, ldA, B * L, (int)ldA, gr.scale, outs, no, wsw));
  return 0;
}

}  // namespace s2s
