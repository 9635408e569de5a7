// GRU layer sequence forward/backward: the drop-in for nn.RNN(nn.GRU(D,H), reverse)
// (RNN.lua:120-201 over GRU.lua:16-51 / Recurrent.lua:104-151).
//
// Reference cell (GRU.lua:22-30), no biases, hx = [h; x] (h first):
//   z = sig(Wz hx), r = sig(Wr hx), hh = tanh(Wh [r*h; x]), h' = (1-z)*h + z*hh
// MI355X decomposition:
//   * the x-half of all three gates for every (b, t) is ONE hoisted MFMA GEMM
//     (B*L x D) x (D x 3H) -- both directions of a layer in the same launch;
//   * per time step two dependent skinny MFMA launches (r gates the candidate):
//       p1: [z|r] = sig(Uzr h_{t-1} + xp)  ->  z, r, q = r*h_{t-1}
//       p2: hh = tanh(Uh q + xp_h), h_t = (1-z) h_{t-1} + z hh
//   * BPTT: two skinny launches per step (dq = Uh^T da_h; dh_{t-1} = Uzr^T [da_z; da_r] + ...),
//     with the next step's gate gradients computed in p2's epilogue;
//   * dW (the reference's per-step rank-1 GER, LinearZeroBias.lua:70) and dx are
//     GEMMs over all B*L rows after the sweep.
// Saved activations per direction: sv (B, L, 5H) = z | r | hh | h_{t-1} | q.
#include "gru.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "gru_persist.h"
#include "skinny.h"

namespace s2s {

namespace {

struct GruFwdDir {
  const float* xp;  // (B, L, ldxp): [z | r | h] x-projections at offset 0
  long ldxp;
  const float* Uzr;  // (2H, H)
  const float* Uh;   // (H, H)
  float* y;          // y[(b*L + t)*ldy + j]
  long ldy;
  float* sv;  // (B, L, 5H)
  int reverse;
};
struct GruFwdArgs {
  GruFwdDir d[2];
  int B, L, H, step;
  const int* len;  // (B) frames per utterance or null
};

__global__ __launch_bounds__(256) void gru_fwd_p1(GruFwdArgs a) {
  __shared__ SkinnyRed red;
  const GruFwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tp = g.reverse ? t + 1 : t - 1;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (step > 0) {
    const int br = min(b0 + (lane & 15), B - 1);
    acc = skinny_wave(g.y + ((long)br * L + tp) * g.ldy, g.Uzr + (long)(n0 + (lane & 15)) * H, H, wave, lane);
  }
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= B) return;
  const long row = (long)b * L + t;
  const float gate = gru_sigmoid(s + g.xp[row * g.ldxp + n]);
  float* sv = g.sv + row * 5 * H;
  if (n < H) {
    sv[n] = gate;  // z
  } else {
    const int j = n - H;
    const float hp = step > 0 ? g.y[((long)b * L + tp) * g.ldy + j] : 0.f;
    sv[H + j] = gate;          // r
    sv[3 * H + j] = hp;        // h_{t-1}
    sv[4 * H + j] = gate * hp; // q = r*h  (CMulTable, GRU.lua:25)
  }
}

__global__ __launch_bounds__(256) void gru_fwd_p2(GruFwdArgs a) {
  __shared__ SkinnyRed red;
  const GruFwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (step > 0) {
    const int br = min(b0 + (lane & 15), B - 1);
    acc = skinny_wave(g.sv + ((long)br * L + t) * 5 * H + 4 * H, g.Uh + (long)(n0 + (lane & 15)) * H, H, wave,
                      lane);
  }
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), n = n0 + (tid & 15);
  if (b >= B) return;
  const long row = (long)b * L + t;
  const float hh = gru_tanh(s + g.xp[row * g.ldxp + 2 * H + n]);
  float* sv = g.sv + row * 5 * H;
  const float z = sv[n], hp = sv[3 * H + n];
  sv[2 * H + n] = hh;
  // GRU.lua:27-30: v1 = (-z)+1; v2 = v1*h; h' = v2 + z*hh  (0 on a padding frame)
  const bool valid = !a.len || t < a.len[b];
  g.y[row * g.ldy + n] = valid ? (-z + 1.0f) * hp + z * hh : 0.f;
}

struct GruBwdDir {
  const float* dy;  // dy[(b*L+t)*lddy + j]
  long lddy;
  const float* sv;    // (B, L, 5H)
  const float* UhT;   // (H, H)   UhT[k][n]  = Uh[n][k]
  const float* UzrT;  // (H, 2H)  UzrT[k][n] = Uzr[n][k]
  float* dA;          // dA[(b*L+t)*ldA + {0,H,2H}] = da_z | da_r | da_h
  long ldA;
  float* dhc;  // (B, H) carried dL/dh_t from step t+1
  float* dhp;  // (B, H) partial dL/dh_{t-1} from p1
  int reverse;
};
struct GruBwdArgs {
  GruBwdDir d[2];
  int B, L, H, step;  // step = forward step index being back-propagated (L-1 .. 0)
  const int* len;     // (B) frames per utterance or null: dL/dh_t = 0 on padding frames
};
__device__ __forceinline__ bool frame_valid(const int* len, int b, int t) { return !len || t < len[b]; }

__device__ __forceinline__ void gru_gate_grads(const GruBwdDir& g, int B, int L, int H, int b, int t, int k,
                                               float dhcarry, const int* len) {
  const long row = (long)b * L + t;
  const float* sv = g.sv + row * 5 * H;
  const float dh = frame_valid(len, b, t) ? g.dy[row * g.lddy + k] + dhcarry : 0.f;
  const float z = sv[k], hh = sv[2 * H + k], hp = sv[3 * H + k];
  float* dA = g.dA + row * g.ldA;
  dA[k] = dh * (hh - hp) * (z * (1.0f - z));          // da_z
  dA[2 * H + k] = (dh * z) * (1.0f - hh * hh);        // da_h
}

// gate gradients for the last forward step (carry = 0)
__global__ void gru_bwd_init(GruBwdArgs a) {
  const GruBwdDir& g = a.d[blockIdx.y];
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.B * a.H) return;
  const int b = idx / a.H, k = idx - b * a.H;
  const int t = g.reverse ? 0 : a.L - 1;
  g.dhc[idx] = 0.f;
  gru_gate_grads(g, a.B, a.L, a.H, b, t, k, 0.f, a.len);
}

__global__ __launch_bounds__(256) void gru_bwd_p1(GruBwdArgs a) {
  __shared__ SkinnyRed red;
  const GruBwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int br = min(b0 + (lane & 15), B - 1);
  floatx4 acc = skinny_wave(g.dA + ((long)br * L + t) * g.ldA + 2 * H, g.UhT + (long)(n0 + (lane & 15)) * H, H,
                            wave, lane);
  const float dq = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), k = n0 + (tid & 15);
  if (b >= B) return;
  const long row = (long)b * L + t;
  const float* sv = g.sv + row * 5 * H;
  const float z = sv[k], r = sv[H + k], hp = sv[3 * H + k];
  g.dA[row * g.ldA + H + k] = (dq * hp) * (r * (1.0f - r));  // da_r
  const float dh = frame_valid(a.len, b, t) ? g.dy[row * g.lddy + k] + g.dhc[b * H + k] : 0.f;
  g.dhp[b * H + k] = dh * (-z + 1.0f) + dq * r;
}

__global__ __launch_bounds__(256) void gru_bwd_p2(GruBwdArgs a) {
  __shared__ SkinnyRed red;
  const GruBwdDir& g = a.d[blockIdx.z];
  const int B = a.B, L = a.L, H = a.H, step = a.step;
  const int t = g.reverse ? L - 1 - step : step;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n0 = blockIdx.x * 16, b0 = blockIdx.y * 16;
  const int br = min(b0 + (lane & 15), B - 1);
  floatx4 acc = skinny_wave(g.dA + ((long)br * L + t) * g.ldA, g.UzrT + (long)(n0 + (lane & 15)) * 2 * H, 2 * H,
                            wave, lane);
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  const int b = b0 + (tid >> 4), k = n0 + (tid & 15);
  if (b >= B || step == 0) return;
  const int tn = g.reverse ? t + 1 : t - 1;
  const float dhprev = frame_valid(a.len, b, tn) ? g.dhp[b * H + k] + s : 0.f;
  g.dhc[b * H + k] = dhprev;
  gru_gate_grads(g, B, L, H, b, tn, k, dhprev, a.len);
}

// Pack W{z,r,h} (H, H+D) into kernel layouts (gru_pack_elems).
using PackArgs = GruPackJob;
__device__ __forceinline__ void pack_body(const PackArgs& p) {
  gru_pack_elems(p, blockIdx.x * (long)blockDim.x + threadIdx.x, (long)gridDim.x * blockDim.x);
}
__global__ void gru_pack(PackArgs p) { pack_body(p); }
// several layer-directions in one launch (blockIdx.y = which)
constexpr int kMaxPack = 8;
struct PackBatch {
  PackArgs p[kMaxPack];
};
__global__ void gru_pack_multi(PackBatch b) { pack_body(b.p[blockIdx.y]); }

int launch_pack(hipStream_t st, const float* Wz, const float* Wr, const float* Wh, int H, int D, int Kx, float* Uzr,
                float* Uh, float* UhT, float* UzrT, float* Wx) {
  PackArgs p{{Wz, Wr, Wh}, Uzr, Uh, UhT, UzrT, Wx, H, D, Kx};
  long n = 3L * H * (H + Kx);
  int blocks = (int)((n + 255) / 256);
  if (blocks > 1024) blocks = 1024;
  hipLaunchKernelGGL(gru_pack, dim3(blocks), dim3(256), 0, st, p);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace

// S2S_GRU_MODE=step forces the per-step launch path (A/B and fallback); default: persistent
// whenever the shape is supported.
static bool use_persistent(int nd, int B, int H) {
  const char* m = std::getenv("S2S_GRU_MODE");
  if (m && std::strcmp(m, "step") == 0) return false;
  return gru_persist_supported(nd, B, H);
}

bool gru_layer_persistent(const GruLayerIO& io) { return use_persistent(io.ndir, io.B, io.H); }

size_t gru_layer_scratch_bytes(int ndir, int B, int L, int D, int H) {
  Bump bp{nullptr, 0, 0};
  for (int d = 0; d < ndir; ++d) {
    bp.take<float>(2L * H * H);
    bp.take<float>((long)H * H);
    bp.take<float>((long)H * H);
    bp.take<float>(2L * H * H);
    bp.take<float>((long)B * H);
    bp.take<float>((long)B * H);
  }
  bp.take<float>(3L * ndir * H * ((D + 31) / 32 * 32));  // Wx (both dirs, rows padded)
  bp.take<float>((long)B * L * 3 * ndir * H);    // xp or dA (both dirs)
  bp.take<char>(gru_persist_sync_bytes(B, L, H));   // persistent-kernel granule buffers
  bp.take<float>(kGemmWsFloats);                 // split-K slabs of this layer's GEMMs
  return bp.off + 256;
}

// packed layout: per direction Uzr (2H,H) | Uh (H,H) | UhT (H,H) | UzrT (H,2H), then Wx (3*ndir*H, Kp)
size_t gru_layer_pack_bytes(int ndir, int D, int H) {
  return sizeof(float) * ((size_t)ndir * 6 * H * H + 3ull * ndir * H * ((D + 31) / 32 * 32));
}
struct PackView {
  const float *Uzr[2], *Uh[2], *UhT[2], *UzrT[2], *Wx;
};
static PackView pack_view(const float* pk, int nd, int H) {
  PackView v{};
  for (int d = 0; d < nd; ++d) {
    v.Uzr[d] = pk;
    v.Uh[d] = pk + 2L * H * H;
    v.UhT[d] = pk + 3L * H * H;
    v.UzrT[d] = pk + 4L * H * H;
    pk += 6L * H * H;
  }
  v.Wx = pk;
  return v;
}
// the pack jobs of `ios` (now) and, with defer, the jobs left to layer 1's spare slots
static int pack_jobs(const GruLayerIO* ios, float* const* packed, int nlayers, GruPackJobs* defer,
                     std::vector<PackArgs>& now) {
  for (int l = 0; l < nlayers; ++l) {
    const GruLayerIO& io = ios[l];
    const int nd = io.ndir, D = io.D, H = io.H;
    const int Kx = io.Dx > D ? io.Dx : D;
    S2S_REQUIRE(Kx <= (D + 31) / 32 * 32, "gru: Dx must be <= round_up(D, 32)");
    const PackView v = pack_view(packed[l], nd, H);
    for (int d = 0; d < nd; ++d) {
      PackArgs job{{io.W[d][0], io.W[d][1], io.W[d][2]}, const_cast<float*>(v.Uzr[d]),
                   const_cast<float*>(v.Uh[d]), const_cast<float*>(v.UhT[d]), const_cast<float*>(v.UzrT[d]),
                   const_cast<float*>(v.Wx) + 3L * d * H * Kx, H, D, Kx};
      if (defer) {  // now: only what layer 1's forward reads; the rest goes to that launch's spare slots
        PackArgs later = job;
        later.Uzr = later.Uh = later.Wx = nullptr;
        if (l > 0) later = job;
        else job.UhT = job.UzrT = nullptr;
        S2S_REQUIRE(defer->n < kMaxPackJobs, "gru: too many deferred pack jobs");
        defer->j[defer->n++] = later;
        if (l > 0) continue;
      }
      now.push_back(job);
    }
  }
  return 0;
}

int gru_layers_pack(hipStream_t st, const GruLayerIO* ios, float* const* packed, int nlayers, GruPackJobs* defer) {
  std::vector<PackArgs> now;
  S2S_TRY(pack_jobs(ios, packed, nlayers, defer, now));
  PackBatch b{};
  int n = 0;
  long most = 0;
  auto flush = [&]() -> int {
    if (n == 0) return 0;
    int blocks = (int)((most + 255) / 256);
    if (blocks > 512) blocks = 512;
    hipLaunchKernelGGL(gru_pack_multi, dim3(blocks, n), dim3(256), 0, st, b);
    S2S_CHECK_HIP(hipGetLastError());
    n = 0;
    most = 0;
    return 0;
  };
  for (const PackArgs& job : now) {
    if (n == kMaxPack) S2S_TRY(flush());
    b.p[n++] = job;
    most = std::max(most, 3L * job.H * (job.H + job.Kx));
  }
  return flush();
}

int gru_step_head(hipStream_t st, const GruLayerIO* ios, float* const* packed, int nlayers, GruPackJobs* defer,
                  const float* x, long ldx, float* xpad, int rows, int cols, int dcols, void* sync, size_t prep_bytes,
                  void* clear, const GruStepHead* extra) {
  std::vector<PackArgs> now;
  S2S_TRY(pack_jobs(ios, packed, nlayers, defer, now));
  GruStepHead h = extra ? *extra : GruStepHead{};
  h.pack.n = 0;
  S2S_REQUIRE((int)now.size() <= kMaxPackJobs, "gru: too many pack jobs for the step head");
  for (const PackArgs& job : now) h.pack.j[h.pack.n++] = job;
  h.src = x; h.lds = ldx; h.dst = xpad; h.rows = xpad ? rows : 0; h.cols = cols; h.dcols = dcols;
  h.sync = static_cast<char*>(sync); h.prep_bytes = prep_bytes; h.clear = static_cast<char*>(clear);
  return gru_persist_step_head(st, h);
}

int gru_layer_pack(hipStream_t st, const GruLayerIO& io, float* packed) {
  const int nd = io.ndir, D = io.D, H = io.H;
  const int Kx = io.Dx > D ? io.Dx : D;
  S2S_REQUIRE(Kx <= (D + 31) / 32 * 32, "gru: Dx must be <= round_up(D, 32)");
  const PackView v = pack_view(packed, nd, H);
  for (int d = 0; d < nd; ++d)
    S2S_TRY(launch_pack(st, io.W[d][0], io.W[d][1], io.W[d][2], H, D, Kx, const_cast<float*>(v.Uzr[d]),
                        const_cast<float*>(v.Uh[d]), const_cast<float*>(v.UhT[d]), const_cast<float*>(v.UzrT[d]),
                        const_cast<float*>(v.Wx) + 3L * d * H * Kx));
  return 0;
}

// the split-K region at the tail of a layer scratch (gru_layer_scratch_bytes)
static GemmWs layer_gemm_ws(void* scratch, int ndir, int B, int L, int D, int H) {
  const size_t tail = gru_layer_scratch_bytes(ndir, B, L, D, H) - 256 - sizeof(float) * kGemmWsFloats;
  return GemmWs{reinterpret_cast<float*>(static_cast<char*>(scratch) + tail), kGemmWsFloats};
}

int gru_layer_fwd(hipStream_t st, const GruLayerIO& io, void* scratch, size_t scratch_bytes) {
  const int nd = io.ndir, B = io.B, L = io.L, D = io.D, H = io.H;
  S2S_REQUIRE(nd == 1 || nd == 2, "gru: ndir must be 1 or 2");
  S2S_REQUIRE(B > 0 && L > 0 && D > 0 && H > 0, "gru: empty dims");
  S2S_REQUIRE(H % 16 == 0, "gru: H must be a multiple of 16");
  S2S_REQUIRE(io.ldy % 4 == 0, "gru: ldy must be a multiple of 4");
  S2S_REQUIRE(scratch_bytes >= gru_layer_scratch_bytes(nd, B, L, D, H), "gru: scratch too small");
  Bump bp{static_cast<char*>(scratch), 0, scratch_bytes};
  float *Uzr[2], *Uh[2];
  for (int d = 0; d < nd; ++d) {
    Uzr[d] = bp.take<float>(2L * H * H);
    Uh[d] = bp.take<float>((long)H * H);
    bp.take<float>((long)H * H);
    bp.take<float>(2L * H * H);
    bp.take<float>((long)B * H);
    bp.take<float>((long)B * H);
  }
  const int Kx = io.Dx > D ? io.Dx : D;
  S2S_REQUIRE(Kx <= (D + 31) / 32 * 32 && io.ldx >= Kx, "gru: Dx must be <= round_up(D, 32) and <= ldx");
  float* Wx = bp.take<float>(3L * nd * H * ((D + 31) / 32 * 32));
  float* xp = bp.take<float>((long)B * L * 3 * nd * H);
  char* sync = bp.take<char>(gru_persist_sync_bytes(B, L, H));
  if (io.sync) sync = static_cast<char*>(io.sync);
  if (io.packed) {
    const PackView v = pack_view(io.packed, nd, H);
    for (int d = 0; d < nd; ++d) {
      Uzr[d] = const_cast<float*>(v.Uzr[d]);
      Uh[d] = const_cast<float*>(v.Uh[d]);
    }
    Wx = const_cast<float*>(v.Wx);
  } else {
    for (int d = 0; d < nd; ++d)
      S2S_TRY(launch_pack(st, io.W[d][0], io.W[d][1], io.W[d][2], H, D, Kx, Uzr[d], Uh[d], nullptr, nullptr,
                          Wx + 3L * d * H * Kx));
  }
  // hoisted x-projections for both directions: xp (B*L, 3*nd*H) = x (B*L, Kx) . Wx^T -- one GEMM, or
  // computed inside the persistent launch by its spare workgroups (gru_persist_fused_xproj)
  const bool fuse = use_persistent(nd, B, H) && gru_persist_fused_xproj(nd, B, H, Kx) && io.ldx % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(io.x) & 15) == 0;
  if (!fuse)
    S2S_TRY(gemm1(st, false, true, B * L, 3 * nd * H, Kx, 1.f, io.x, io.ldx, Wx, Kx, 0.f, xp, 3L * nd * H, nullptr,
                  layer_gemm_ws(scratch, nd, B, L, D, H)));
  GruFwdArgs a{};
  for (int d = 0; d < nd; ++d)
    a.d[d] = GruFwdDir{xp + 3L * d * H, 3L * nd * H, Uzr[d], Uh[d], io.y[d], io.ldy, io.saved[d], io.reverse[d]};
  a.B = B;
  a.L = L;
  a.H = H;
  a.len = io.len;
  S2S_REQUIRE(!io.pack_jobs || gru_layer_preps_next(io, true),
              "gru: deferred weight packing needs a persistent forward with spare slots");
  if (use_persistent(nd, B, H)) {
    GruPersistFwd f{};
    f.len = io.len;
    f.ndir = nd; f.B = B; f.L = L; f.H = H; f.ldxp = 3L * nd * H; f.ldy = io.ldy;
    if (fuse) {
      f.x = io.x; f.ldx = io.ldx; f.Kx = Kx; f.Wx = Wx;
    }
    for (int d = 0; d < nd; ++d) {
      f.xp[d] = xp + 3L * d * H; f.Uzr[d] = Uzr[d]; f.Uh[d] = Uh[d]; f.y[d] = io.y[d]; f.sv[d] = io.saved[d];
      f.reverse[d] = io.reverse[d];
    }
    f.prepared = io.sync ? io.sync_prepared : 0;
    if (io.sync_next && gru_layer_preps_next(io, true)) {
      f.next_sync = io.sync_next;
      f.next_prep = io.sync_next_prep;
    }
    f.pack = io.pack_jobs;
    f.excl = io.excl;
    f.status = io.status;
    return gru_persist_fwd(st, f, sync);
  }
  const dim3 g1(2 * H / 16, (B + 15) / 16, nd), g2(H / 16, (B + 15) / 16, nd);
  ProfScope ps(st, "gru_fwd_steps", 2.0 * nd * B * L * 3.0 * H * H, 0.0);
  for (int s = 0; s < L; ++s) {
    a.step = s;
    hipLaunchKernelGGL(gru_fwd_p1, g1, dim3(256), 0, st, a);
    hipLaunchKernelGGL(gru_fwd_p2, g2, dim3(256), 0, st, a);
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int gru_layer_bwd_core(hipStream_t st, const GruLayerIO& io, const GruLayerGrad& gr, float* dA_ext, void* scratch,
                       size_t scratch_bytes) {
  const int nd = io.ndir, B = io.B, L = io.L, D = io.D, H = io.H;
  S2S_REQUIRE(nd == 1 || nd == 2, "gru: ndir must be 1 or 2");
  S2S_REQUIRE(H % 16 == 0, "gru: H must be a multiple of 16");
  S2S_REQUIRE(scratch_bytes >= gru_layer_scratch_bytes(nd, B, L, D, H), "gru: scratch too small");
  Bump bp{static_cast<char*>(scratch), 0, scratch_bytes};
  float *UhT[2], *UzrT[2], *dhc[2], *dhp[2];
  for (int d = 0; d < nd; ++d) {
    bp.take<float>(2L * H * H);
    bp.take<float>((long)H * H);
    UhT[d] = bp.take<float>((long)H * H);
    UzrT[d] = bp.take<float>(2L * H * H);
    dhc[d] = bp.take<float>((long)B * H);
    dhp[d] = bp.take<float>((long)B * H);
  }
  const int Kx = io.Dx > D ? io.Dx : D;
  S2S_REQUIRE(Kx <= (D + 31) / 32 * 32 && io.ldx >= Kx, "gru: Dx must be <= round_up(D, 32) and <= ldx");
  float* Wx = bp.take<float>(3L * nd * H * ((D + 31) / 32 * 32));
  float* dA_int = bp.take<float>((long)B * L * 3 * nd * H);
  float* dA = dA_ext ? dA_ext : dA_int;
  char* sync = bp.take<char>(gru_persist_sync_bytes(B, L, H));
  if (io.sync) sync = static_cast<char*>(io.sync);
  const long ldA = 3L * nd * H;
  if (io.packed) {
    const PackView v = pack_view(io.packed, nd, H);
    for (int d = 0; d < nd; ++d) {
      UhT[d] = const_cast<float*>(v.UhT[d]);
      UzrT[d] = const_cast<float*>(v.UzrT[d]);
    }
    Wx = const_cast<float*>(v.Wx);
  } else {
    for (int d = 0; d < nd; ++d)
      S2S_TRY(launch_pack(st, io.W[d][0], io.W[d][1], io.W[d][2], H, D, Kx, nullptr, nullptr, UhT[d], UzrT[d],
                          Wx + 3L * d * H * Kx));
  }
  GruBwdArgs a{};
  for (int d = 0; d < nd; ++d)
    a.d[d] = GruBwdDir{gr.dy[d], gr.lddy, io.saved[d], UhT[d], UzrT[d], dA + 3L * d * H, ldA, dhc[d], dhp[d],
                       io.reverse[d]};
  a.B = B;
  a.L = L;
  a.H = H;
  a.len = io.len;
  const bool persist = use_persistent(nd, B, H);
  const bool yfuse = gru_layer_dy_fused(io, gr);
  S2S_REQUIRE(!gr.yalpha || yfuse, "gru: the dh context term is only produced inside the fused BPTT launch");
  S2S_REQUIRE(!gr.wgrad || persist, "gru: in-launch weight gradients need the persistent BPTT");
  if (gr.ydA && !yfuse) {  // the layer above's dX as one GEMM in front of the BPTT (same order as in-launch)
    GemmProblem p{gr.ydA, gr.yWx, const_cast<float*>(gr.dy[0]), nullptr, gr.yldA, gr.yldw, gr.lddy, B * L, gr.yN,
                  gr.yK, 1.f, 0.f};
    p.Nread = (int)gr.yldw;
    S2S_TRY(gemm_f32(st, &p, 1, false, false, layer_gemm_ws(scratch, nd, B, L, D, H)));
  }
  if (persist) {
    GruPersistBwd f{};
    f.len = io.len;
    if (yfuse) {
      f.ydA = gr.ydA; f.yldA = gr.yldA; f.yK = gr.yK; f.yWx = gr.yWx; f.yldw = gr.yldw;
      f.yalpha = gr.yalpha; f.ydc = gr.ydc; f.yT = gr.yT;
    }
    f.ndir = nd; f.B = B; f.L = L; f.H = H; f.lddy = gr.lddy; f.ldA = ldA;
    for (int d = 0; d < nd; ++d) {
      f.UhT[d] = UhT[d]; f.UzrT[d] = UzrT[d]; f.sv[d] = io.saved[d]; f.dy[d] = gr.dy[d]; f.dA[d] = dA + 3L * d * H;
      f.reverse[d] = io.reverse[d];
    }
    f.prep_event = gr.prep_event;
    f.prepared = io.sync ? io.sync_prepared : 0;
    if (io.sync_next && gru_layer_preps_next(io, false)) {
      f.next_sync = io.sync_next;
      f.next_prep = io.sync_next_prep;
    }
    f.excl = io.excl;
    f.status = io.status;
    if (gr.wgrad) {
      S2S_REQUIRE(gru_layer_wgrad_fused(io), "gru: in-launch weight gradients need a persistent BPTT that fits them");
      f.wgrad = 1;
      for (int d = 0; d < 2; ++d)
        for (int g = 0; g < 3; ++g) f.wdW[d][g] = gr.dW[d][g];
      f.wscale = gr.scale;
      f.wx = io.x; f.wldx = io.ldx; f.wD = D;
      f.wpart = gr.wpart;
    }
    S2S_TRY(gru_persist_bwd(st, f, sync));
  } else {
    ProfScope ps(st, "gru_bwd_steps", 2.0 * nd * B * L * 3.0 * H * H, 0.0);
    hipLaunchKernelGGL(gru_bwd_init, dim3((B * H + 255) / 256, nd), dim3(256), 0, st, a);
    const dim3 g1(H / 16, (B + 15) / 16, nd);
    for (int s = L - 1; s >= 0; --s) {
      a.step = s;
      hipLaunchKernelGGL(gru_bwd_p1, g1, dim3(256), 0, st, a);
      hipLaunchKernelGGL(gru_bwd_p2, g1, dim3(256), 0, st, a);
    }
    S2S_CHECK_HIP(hipGetLastError());
    if (gr.prep_event) S2S_CHECK_HIP(hipEventRecord(gr.prep_event, st));
  }
  // dx (+)= dA (B*L, 3*nd*H) . Wx (3*nd*H, D)   (RNN.lua:196 gradInput; both directions summed,
  // which is what the encoder graph's fan-out of the layer input accumulates)
  if (gr.dx) {
    GemmProblem p{dA, Wx, gr.dx, nullptr, ldA, Kx, gr.lddx, B * L, D, 3 * nd * H, 1.f, gr.dx_accumulate ? 1.f : 0.f};
    p.Nread = Kx;  // Wx's zero columns
    S2S_TRY(gemm_f32(st, &p, 1, false, false, layer_gemm_ws(scratch, nd, B, L, D, H)));
  }
  return 0;
}

bool gru_layer_wgrad_fused(const GruLayerIO& io) {
  return use_persistent(io.ndir, io.B, io.H) && gru_persist_wgrad_fits(io.ndir, io.B, io.H, io.D);
}
size_t gru_layer_wgrad_part_floats(const GruLayerIO& io) {
  const int MT = (io.B + 15) / 16;
  return (size_t)io.ndir * MT * 3 * io.H * (io.H + (io.D + 15) / 16 * 16);
}

bool gru_layer_preps_next(const GruLayerIO& io, bool fwd) {
  return use_persistent(io.ndir, io.B, io.H) && gru_persist_can_prep_next(io.ndir, io.B, io.H, fwd);
}
size_t gru_layer_sync_prep_bytes(const GruLayerIO& io) { return gru_persist_prep_bytes(io.B, io.L, io.H); }

bool gru_layer_dy_fused(const GruLayerIO& io, const GruLayerGrad& gr) {
  const int nd = io.ndir, B = io.B, H = io.H;
  return gr.ydA && use_persistent(nd, B, H) && (nd == 1 || gr.dy[1] == gr.dy[0] + H) &&
         gru_persist_fused_dy(nd, B, H, gr.yK, gr.yldw, gr.lddy);
}

const float* gru_layer_packed_wx(const GruLayerIO& io, long* ldw) {
  const int Kx = io.Dx > io.D ? io.Dx : io.D;
  *ldw = Kx;
  return io.packed ? pack_view(io.packed, io.ndir, io.H).Wx : nullptr;
}

float* gru_layer_dA(const GruLayerIO& io, void* scratch) {
  Bump bp{static_cast<char*>(scratch), 0, 0};
  for (int d = 0; d < io.ndir; ++d) {
    bp.take<float>(2L * io.H * io.H);
    bp.take<float>((long)io.H * io.H);
    bp.take<float>((long)io.H * io.H);
    bp.take<float>(2L * io.H * io.H);
    bp.take<float>((long)io.B * io.H);
    bp.take<float>((long)io.B * io.H);
  }
  bp.take<float>(3L * io.ndir * io.H * ((io.D + 31) / 32 * 32));  // Wx (padded rows), as in the layer calls
  return bp.take<float>((long)io.B * io.L * 3 * io.ndir * io.H);
}

// dW += scale * dA_g^T . [h_{t-1} | q ; x]   (LinearZeroBias.lua:67-74 summed over all steps).
// Off the recurrence: the model step runs it on a side stream beside the next layer's BPTT.
int gru_layer_wgrad(hipStream_t st, const GruLayerIO& io, const GruLayerGrad& gr, const float* dA, GemmWs ws) {
  WgradPrecision wp;
  const int nd = io.ndir, B = io.B, L = io.L, D = io.D, H = io.H;
  const long ldA = 3L * nd * H;
  GemmProblem probs[12];
  int np = 0;
  for (int d = 0; d < nd; ++d) {
    for (int g = 0; g < 3; ++g) {
      const float* dAg = dA + 3L * d * H + (long)g * H;
      float* dW = gr.dW[d][g];
      // h-part columns [0, H): z,r use h_{t-1} (sv + 3H), h-gate uses q = r*h (sv + 4H)
      probs[np++] = GemmProblem{dAg, io.saved[d] + (g == 2 ? 4 : 3) * H, dW, nullptr, ldA, 5L * H, (long)H + D,
                                H, H, B * L, gr.scale, 1.f};
      // x-part columns [H, H+D)
      probs[np] = GemmProblem{dAg, io.x, dW + H, nullptr, ldA, io.ldx, (long)H + D, H, D, B * L, gr.scale, 1.f};
      probs[np++].Nread = io.Dx > D ? io.Dx : D;  // x's zero columns
    }
  }
  return gemm_f32(st, probs, np, true, false, ws);
}

int gru_layer_bwd(hipStream_t st, const GruLayerIO& io, const GruLayerGrad& gr, void* scratch, size_t scratch_bytes) {
  S2S_TRY(gru_layer_bwd_core(st, io, gr, nullptr, scratch, scratch_bytes));
  if (gr.wgrad) return 0;  // computed inside the BPTT launch
  return gru_layer_wgrad(st, io, gr, gru_layer_dA(io, scratch),
                         layer_gemm_ws(scratch, io.ndir, io.B, io.L, io.D, io.H));
}

}  // namespace s2s
