// Persistent LSTM layer recurrence (no peepholes): the whole L-step sweep of one (bidirectional) nn.RNN(nn.LSTM)
// layer in ONE launch instead of one launch per step (LSTM.lua:16-58 forward, :96-136 backward, under
// RNN.lua:120-201) -- the conv + BiLSTM encoder of timit/timit.lua:108-125.
//
// The GRU's persistent design (gru_persist.hip) with the LSTM's single seam per step:
//   * chain = (direction, 16-utterance row tile), members = 16-unit column tiles, placed on one XCD
//     (chain_slot / chain_is_local); a member keeps its weight fragments in VGPRs for the whole sweep;
//   * forward step: sweep h_{t-1} (16 rows x H) -> the four gate products of the member's 16 units (K = H split
//     over 4 waves, the chunk order and 4-partial LDS sum of lstm_fwd_step's skinny4_1024, so the results are
//     bitwise the per-step launches') -> cell update in registers (c_{t-1} and h_{t-1} of the thread's own
//     (utterance, unit) never leave it) -> publish h_t;
//   * backward step: sweep the gate gradients of the step after (16 rows x 4H) -> dh = dy + Wb row . dgates
//     (K = 4H split over 8 waves as lstm_bwd_step's skinny_wave8, bitwise the same) -> dc = dc_carry + dh o
//     (1 - tanh^2 c), the four gate gradients -> publish them; dc_carry = dc f stays in the thread;
//   * hand-offs: XCD-local chains publish plain fp32 values into per-step sentinel slots (tile-major,
//     re-armed to kSent by each producer at launch start), other chains tagged 8-byte granules (handoff.h);
//     every wait is bounded, failures reach the context's status through the harvest behind the launch.
// The x-projections, dx and the weight gradients stay GEMMs over all B L rows (lstm.hip).
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>

#include "handoff.h"
#include "lstm.h"
#include "skinny.h"

namespace s2s {

namespace {

struct LDir {
  const float* xp;     // fwd: (B L, ldxp) [i | f | g | o] x-projections with every bias folded in
  long ldxp;
  const float* Wh[4];  // fwd: Wqh (H, H)
  const float* Wb;     // bwd: (2H, 4H) packed (lstm.hip launch_lstm_pack): row u = [Wih; Wfh; Wgh; Woh][:, u]
  float* y;            // fwd output y[(b L + t) ldy + j]
  long ldy;
  float* sv;           // (B, L, 8H) saved activations (lstm.h LstmSv)
  const float* dy;     // bwd
  long lddy;
  float* dA;           // bwd gate pre-activation gradients dA[(b L + t) ldA + q H + j]
  long ldA;
  int reverse;
  float* sent;         // sentinel slots [L][MT 16][W], tile-major
  granule_t* gran;     // granules [2 parities][B][W]
};
struct LArgs {
  LDir d[2];
  const int* len;  // (B) frames per utterance or null (lstm.h LstmLayerIO::len)
  int B, L, H, MT, nmem, nchains, allow_local;
  unsigned* abort_word;
  unsigned* census;
};

// chunk i of a wave over a tile-major sentinel slot of width W: column tile (wave + NW i) (NW = waves that split
// K); rowt = this lane's row within the row tile; tbase = byte offset of the slot's row tile
template <int NC, int NW>
__device__ __forceinline__ bool sweep_tile_w(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long tbase, int rowt,
                                             int wave, int lane, unsigned* abort_word) {
  const long lo = tbase + 4 * tile_lane(rowt, lane);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const uint4 p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                                    rs, (int)(lo + 4L * 256 * (wave + NW * i)), 0, 16));
      ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
      a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}
// the same over a granule row (row_off in bytes): k = 16 wave + 16 NW i + the lane's quad
template <int NC, int NW>
__device__ __forceinline__ bool sweep_gran_w(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long row_off, unsigned tag,
                                             int wave, int lane, unsigned* abort_word) {
  const long kq = 4 * (lane >> 4);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = row_off + 8 * (16 * (wave + NW * i) + kq);
      const uint4 p0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      const uint4 p1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off + 16, 0, 16));
      ok = ok && p0.y == tag && p0.w == tag && p1.y == tag && p1.w == tag;
      a[i] = make_float4(__uint_as_float(p0.x), __uint_as_float(p0.z), __uint_as_float(p1.x), __uint_as_float(p1.z));
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}
// weight fragment of an NW-wave K split: chunk i = k 16 (wave + NW i) + the lane's quad
template <int NC, int NW>
__device__ __forceinline__ void load_wfrag_w(float4 (&w)[NC], const float* row, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NC; ++i) w[i] = *reinterpret_cast<const float4*>(row + 16 * (wave + NW * i) + 4 * (lane >> 4));
}

// ------------------------------------------------------------------------------ forward
template <int NC>  // NC = H / 64
__global__ __launch_bounds__(256) void lstm_fwd_persist(LArgs a) {
  __shared__ SkinnyRed red[4];
  __shared__ int abort_lds, local_lds;
  __shared__ unsigned tb_lds;
  const ChainSlot cs = chain_slot(a.nmem);
  if (cs.chain >= a.nchains) return;
  const int H = a.H, B = a.B, L = a.L;
  const int dir = cs.chain / a.MT, mt = cs.chain % a.MT, m = cs.member;
  const LDir& g = a.d[dir];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = mt * 16, ob = b0 + (tid >> 4), j = m * 16 + (tid & 15);
  const bool live = ob < B;
  const int lenb = (a.len && live) ? a.len[ob] : L;  // padding frames t >= lenb: zero state and output
  if (tid == 0) abort_lds = 0;
  const unsigned tb = launch_tagbase(a.abort_word, &tb_lds);
  const long slotS = (long)a.MT * 16 * H, tileS = (long)mt * 16 * H, mytile = tileS + (long)m * 256;
  rearm_rect(g.sent + mytile, slotS, L, 16, 0, 16, 0, 16);
  rearm_done();
  const bool loc = chain_is_local(a.census, cs.chain, a.nmem, m, a.allow_local != 0, a.abort_word, &local_lds, tb);
  float4 w[4][NC];
#pragma unroll
  for (int q = 0; q < 4; ++q) load_wfrag(w[q], g.Wh[q] + (long)(m * 16 + (lane & 15)) * H, wave, lane);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(g.sent), rg = rsrc_of(g.gran);
  const int br = min(b0 + (lane & 15), B - 1), rowt = br - b0;
  const long slotG = (long)B * H;
  // this step's x-projections, loaded one step ahead (independent of the hand-off)
  auto xload = [&](int s, float (&x)[4]) {
    const int t = g.reverse ? L - 1 - s : s;
    const float* xp = g.xp + ((long)(live ? ob : 0) * L + t) * g.ldxp + j;
#pragma unroll
    for (int q = 0; q < 4; ++q) x[q] = xp[q * H];
  };
  float xn[4];
  xload(0, xn);
  float creg = 0.f, hreg = 0.f;
  for (int s = 0; s < L; ++s) {
    const int t = g.reverse ? L - 1 - s : s;
    const long row = (long)ob * L + t;
    float xc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) xc[q] = xn[q];
    if (s + 1 < L) xload(s + 1, xn);
    floatx4 acc[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = floatx4{0.f, 0.f, 0.f, 0.f};
    bool ok = true;
    if (s > 0) {
      float4 av[NC];
      if (loc) ok = sweep_tile_w<NC, 4>(av, rs, 4 * ((s - 1) * slotS + tileS), rowt, wave, lane, a.abort_word);
      else ok = sweep_gran_w<NC, 4>(av, rg, 8 * (((s - 1) & 1) * slotG + (long)br * H), tb + s, wave, lane, a.abort_word);
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = mfma_chunks<NC>(av, w[q]);
    }
    // the four partial tiles of every gate, one barrier (skinny4_1024's sum order per gate)
    if (!ok) abort_lds = 1;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[q].v[wave][4 * (lane >> 4) + r][lane & 15] = acc[q][r];
    __syncthreads();
    float sg[4];
    {
      const int i = tid >> 4, jj = tid & 15;
#pragma unroll
      for (int q = 0; q < 4; ++q) sg[q] = ((red[q].v[0][i][jj] + red[q].v[1][i][jj]) + red[q].v[2][i][jj]) + red[q].v[3][i][jj];
    }
    const bool aborted = abort_lds != 0;
    // LSTM.lua:38-50: i, f, o sigmoid, g tanh; c = f c' + i g; h = o tanh(c)  (lstm_fwd_step's expressions)
    const float gi = sigmoidf_(sg[0] + xc[0]), gf = sigmoidf_(sg[1] + xc[1]);
    const float gg = tanhf(sg[2] + xc[2]), go = sigmoidf_(sg[3] + xc[3]);
    float c = gf * creg + gi * gg, tc = tanhf(c), h = go * tc;
    if (t >= lenb) c = tc = h = 0.f;  // lstm_fwd_step's masking
    if (loc) {  // critical first
      if (live) put_sent(g.sent + s * slotS + tile_off(ob, j, H), h);
    } else {
      put_granule_pair(g.gran, (s & 1) * slotG + (long)ob * H + j, h, tb + s + 1, live);
    }
    if (live) {
      float* sv = g.sv + row * SV_N * H;
      sv[SV_I * H + j] = gi;
      sv[SV_F * H + j] = gf;
      sv[SV_G * H + j] = gg;
      sv[SV_O * H + j] = go;
      sv[SV_HP * H + j] = hreg;
      sv[SV_CP * H + j] = creg;
      sv[SV_C * H + j] = c;
      sv[SV_TC * H + j] = tc;
      g.y[row * g.ldy + j] = h;
    }
    creg = c;
    hreg = h;
    if (aborted) return;
  }
}

// ------------------------------------------------------------------------------ backward
constexpr int kBwdWaves = 8;
template <int NCB>  // NCB = 4H / 128 chunks per wave (K = 4H over 8 waves)
__global__ __launch_bounds__(512) void lstm_bwd_persist(LArgs a) {
  __shared__ SkinnyRed8 red;
  __shared__ int abort_lds, local_lds;
  __shared__ unsigned tb_lds;
  const ChainSlot cs = chain_slot(a.nmem);
  if (cs.chain >= a.nchains) return;
  const int H = a.H, B = a.B, L = a.L, W = 4 * H;
  const int dir = cs.chain / a.MT, mt = cs.chain % a.MT, m = cs.member;
  const LDir& g = a.d[dir];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool out = tid < 256;  // threads 0..255 own (utterance, unit) outputs
  const int b0 = mt * 16, ob = b0 + ((tid & 255) >> 4), j = m * 16 + (tid & 15);
  const bool live = out && ob < B;
  const int lenb = (a.len && live) ? a.len[ob] : L;  // padding frames t >= lenb: dL/dh = dL/dc = 0
  if (tid == 0) abort_lds = 0;
  const unsigned tb = launch_tagbase(a.abort_word, &tb_lds);
  const long slotS = (long)a.MT * 16 * W, tileS = (long)mt * 16 * W;
  // this member publishes four 16 x 16 tiles per step (gate q: column tile q H / 16 + m); waves 0..3 re-arm one
  // gate's tile each
  if (wave < 4) {
    const long tq = tileS + (long)(wave * (H / 16) + m) * 256;
    for (int i = lane; i < L * 64; i += 64) {
      const int s = i >> 6, c4 = i & 63;
      const float4 sv = make_float4(__uint_as_float(kSent), __uint_as_float(kSent), __uint_as_float(kSent),
                                    __uint_as_float(kSent));
      *reinterpret_cast<float4*>(g.sent + (long)s * slotS + tq + 4 * c4) = sv;
    }
  }
  rearm_done();
  // chain_is_local: all threads of the workgroup take part (it polls with threadIdx.x < nmem)
  const bool loc = chain_is_local(a.census, cs.chain, a.nmem, m, a.allow_local != 0, a.abort_word, &local_lds, tb);
  float4 wb[NCB];
  load_wfrag_w<NCB, kBwdWaves>(wb, g.Wb + (long)(m * 16 + (lane & 15)) * W, wave, lane);
  const __amdgpu_buffer_rsrc_t rs = rsrc_of(g.sent), rg = rsrc_of(g.gran);
  const int br = min(b0 + (lane & 15), B - 1), rowt = br - b0;
  const long slotG = (long)B * W;
  struct Row {
    float i, f, gg, o, cp, tc, dy;
  };
  auto rload = [&](int p) {
    Row r{0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (!live) return r;
    const int s = L - 1 - p, t = g.reverse ? L - 1 - s : s;
    const long row = (long)ob * L + t;
    const float* sv = g.sv + row * SV_N * H + j;
    r.i = sv[SV_I * H]; r.f = sv[SV_F * H]; r.gg = sv[SV_G * H]; r.o = sv[SV_O * H];
    r.cp = sv[SV_CP * H]; r.tc = sv[SV_TC * H];
    r.dy = g.dy[row * g.lddy + j];
    return r;
  };
  Row nx = rload(0);
  float dcp = 0.f;  // dL/dc_{t+1} * f_{t+1}: the cell carry (lstm_cell_grads' dcp)
  for (int p = 0; p < L; ++p) {
    const int s = L - 1 - p, t = g.reverse ? L - 1 - s : s;
    const long row = (long)ob * L + t;
    const Row cur = nx;
    if (p + 1 < L) nx = rload(p + 1);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    bool ok = true;
    if (p > 0) {
      float4 av[NCB];
      if (loc) ok = sweep_tile_w<NCB, kBwdWaves>(av, rs, 4 * ((p - 1) * slotS + tileS), rowt, wave, lane, a.abort_word);
      else ok = sweep_gran_w<NCB, kBwdWaves>(av, rg, 8 * (((p - 1) & 1) * slotG + (long)br * W), tb + p, wave, lane,
                                             a.abort_word);
      acc = mfma_chunks<NCB>(av, wb);
    }
    if (!ok) abort_lds = 1;
    const float sh = skinny_reduce8(red, acc, wave, lane, tid);
    const bool aborted = abort_lds != 0;
    if (out) {
      // lstm_bwd_step's expressions: dh = dy + carry; dc = dcc + dh o (1 - tanh^2 c); gate gradients
      const bool pad = t >= lenb;
      const float dh = pad ? 0.f : cur.dy + (p > 0 ? sh : 0.f);
      const float dc = pad ? 0.f : (p > 0 ? dcp + 0.f : 0.f) + dh * cur.o * (1.0f - cur.tc * cur.tc);
      const float dao = (dh * cur.tc) * (cur.o * (1.0f - cur.o));
      const float dai = (dc * cur.gg) * (cur.i * (1.0f - cur.i));
      const float daf = (dc * cur.cp) * (cur.f * (1.0f - cur.f));
      const float dag = (dc * cur.i) * (1.0f - cur.gg * cur.gg);
      dcp = dc * cur.f;
      if (loc) {
        if (live) {
          float* sl = g.sent + p * slotS;
          put_sent(sl + tile_off(ob, j, W), dai);
          put_sent(sl + tile_off(ob, H + j, W), daf);
          put_sent(sl + tile_off(ob, 2 * H + j, W), dag);
          put_sent(sl + tile_off(ob, 3 * H + j, W), dao);
        }
      } else {
        const long o = (p & 1) * slotG + (long)ob * W + j;
        put_granule_pair(g.gran, o, dai, tb + p + 1, live);
        put_granule_pair(g.gran, o + H, daf, tb + p + 1, live);
        put_granule_pair(g.gran, o + 2 * H, dag, tb + p + 1, live);
        put_granule_pair(g.gran, o + 3 * H, dao, tb + p + 1, live);
      }
      if (live) {
        float* dA = g.dA + row * g.ldA;
        dA[j] = dai;
        dA[H + j] = daf;
        dA[2 * H + j] = dag;
        dA[3 * H + j] = dao;
      }
    }
    if (aborted) return;
  }
}

std::atomic<int> g_lstm_local{1};  // s2s_debug_lstm_local(0): tagged granules even on XCD-local chains

template <int NC>
int launch_fwd_nc(hipStream_t st, const LArgs& a) {
  S2S_TRY(check_resident(reinterpret_cast<const void*>(lstm_fwd_persist<NC>), chain_grid(a.nchains, a.nmem), 256, 0,
                         "lstm_fwd_persist"));
  hipLaunchKernelGGL(lstm_fwd_persist<NC>, dim3(chain_grid(a.nchains, a.nmem)), dim3(256), 0, st, a);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}
template <int NCB>
int launch_bwd_nc(hipStream_t st, const LArgs& a) {
  S2S_TRY(check_resident(reinterpret_cast<const void*>(lstm_bwd_persist<NCB>), chain_grid(a.nchains, a.nmem), 512, 0,
                         "lstm_bwd_persist"));
  hipLaunchKernelGGL(lstm_bwd_persist<NCB>, dim3(chain_grid(a.nchains, a.nmem)), dim3(512), 0, st, a);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

size_t census_bytes_l(int nchains, int nmem) { return ((size_t)4 * nchains * nmem + 255) / 256 * 256; }
// [ndir][2][B][4H] tagged granules: ndir = nchains / row tiles
size_t gran_bytes_l(int nd, int B, int H) { return (size_t)nd * sizeof(granule_t) * 2 * (size_t)B * 4 * H; }
size_t prep_bytes_l(int B, int H, int nchains, int nmem) {
  return 256 + census_bytes_l(nchains, nmem) + gran_bytes_l(nchains / ((B + 15) / 16), B, H);
}

void carve_sync(char* sync, int B, int L, int H, int nchains, int nmem, LArgs& a) {
  a.abort_word = reinterpret_cast<unsigned*>(sync);
  a.census = reinterpret_cast<unsigned*>(sync + 256);
  granule_t* gp = reinterpret_cast<granule_t*>(sync + 256 + census_bytes_l(nchains, nmem));
  float* sp = reinterpret_cast<float*>(sync + prep_bytes_l(B, H, nchains, nmem));
  const int MT = (B + 15) / 16, nd = nchains / MT;
  for (int d = 0; d < 2; ++d) {
    a.d[d].gran = d < nd ? gp + (long)d * 2 * B * 4 * H : nullptr;
    a.d[d].sent = d < nd ? sp + (long)d * L * MT * 16 * 4 * H : nullptr;
  }
}

}  // namespace

bool lstm_persist_supported(int ndir, int B, int H, int peep) {
  const char* m = std::getenv("S2S_LSTM_MODE");
  if (m && std::strcmp(m, "step") == 0) return false;
  if (peep || H % 64 != 0 || H > 256) return false;  // (H = 512: the backward's 16 weight chunks spill)
  const int MT = (B + 15) / 16, nchains = ndir * MT, nmem = H / 16;
  // every member of the chains dealt to one XCD co-resident there, one per CU (32 CUs per XCD)
  return nmem * ((nchains + 7) / 8) <= 32;
}

// the hand-off region of ndir directions (sentinel slots: one per step, [ndir][L][row tiles][16][4H])
size_t lstm_persist_sync_bytes(int ndir, int B, int L, int H) {
  const int MT = (B + 15) / 16, nchains = ndir * MT, nmem = H / 16;
  return prep_bytes_l(B, H, nchains, nmem) + sizeof(float) * (size_t)ndir * L * MT * 16 * 4 * H;
}

int lstm_persist_fwd(hipStream_t st, const LstmPersistArgs& f, void* sync, unsigned* status) {
  LArgs a{};
  const int MT = (f.B + 15) / 16;
  a.B = f.B; a.L = f.L; a.H = f.H; a.MT = MT; a.nmem = f.H / 16; a.nchains = f.ndir * MT; a.len = f.len;
  a.allow_local = g_lstm_local;
  carve_sync(static_cast<char*>(sync), f.B, f.L, f.H, a.nchains, a.nmem, a);
  for (int d = 0; d < f.ndir; ++d) {
    LDir& g = a.d[d];
    g.xp = f.xp[d]; g.ldxp = f.ldxp;
    for (int q = 0; q < 4; ++q) g.Wh[q] = f.Wh[d][q];
    g.y = f.y[d]; g.ldy = f.ldy; g.sv = f.sv[d]; g.reverse = f.reverse[d];
  }
  S2S_TRY(launch_sync_prep(st, sync, prep_bytes_l(f.B, f.H, a.nchains, a.nmem)));
  {
    ProfScope ps(st, "lstm_fwd_persist", 2.0 * f.ndir * f.B * f.L * 4.0 * f.H * f.H,
                 4.0 * f.ndir * (4.0 * f.H * f.H + (double)f.B * f.L * (4 * f.H + 8 * f.H + f.H)));
    switch (f.H / 64) {
      case 1: S2S_TRY(launch_fwd_nc<1>(st, a)); break;
      case 2: S2S_TRY(launch_fwd_nc<2>(st, a)); break;
      case 4: S2S_TRY(launch_fwd_nc<4>(st, a)); break;
      case 8: S2S_TRY(launch_fwd_nc<8>(st, a)); break;
      default: set_error("lstm persistent: unsupported H"); return 2;
    }
  }
  void* r[1] = {sync};
  return launch_sync_harvest(st, r, 1, status);
}

int lstm_persist_bwd(hipStream_t st, const LstmPersistArgs& b, void* sync, unsigned* status) {
  LArgs a{};
  const int MT = (b.B + 15) / 16;
  a.B = b.B; a.L = b.L; a.H = b.H; a.MT = MT; a.nmem = b.H / 16; a.nchains = b.ndir * MT; a.len = b.len;
  a.allow_local = g_lstm_local;
  carve_sync(static_cast<char*>(sync), b.B, b.L, b.H, a.nchains, a.nmem, a);
  for (int d = 0; d < b.ndir; ++d) {
    LDir& g = a.d[d];
    g.Wb = b.Wb[d]; g.sv = b.sv[d]; g.dy = b.dy[d]; g.lddy = b.lddy; g.dA = b.dA[d]; g.ldA = b.ldA;
    g.reverse = b.reverse[d];
  }
  S2S_TRY(launch_sync_prep(st, sync, prep_bytes_l(b.B, b.H, a.nchains, a.nmem)));
  {
    ProfScope ps(st, "lstm_bwd_persist", 2.0 * b.ndir * b.B * b.L * 4.0 * b.H * b.H,
                 4.0 * b.ndir * (4.0 * b.H * b.H + (double)b.B * b.L * (6 * b.H + b.H + 4 * b.H)));
    switch (4 * b.H / 128) {
      case 2: S2S_TRY(launch_bwd_nc<2>(st, a)); break;
      case 4: S2S_TRY(launch_bwd_nc<4>(st, a)); break;
      case 8: S2S_TRY(launch_bwd_nc<8>(st, a)); break;
      case 16: S2S_TRY(launch_bwd_nc<16>(st, a)); break;
      default: set_error("lstm persistent: unsupported H"); return 2;
    }
  }
  void* r[1] = {sync};
  return launch_sync_harvest(st, r, 1, status);
}

}  // namespace s2s

// diagnostic: 0 forces tagged-granule hand-offs in every persistent LSTM chain (tests cover both forms)
extern "C" void s2s_debug_lstm_local(int allow) { s2s::g_lstm_local = allow; }
