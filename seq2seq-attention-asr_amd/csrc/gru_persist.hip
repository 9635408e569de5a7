// Persistent GRU layer recurrence: the whole L-step sweep of one bidirectional layer
// (both directions) in ONE launch instead of 2*L launches.
//
// Same arithmetic and summation order as the per-step kernels in gru.hip (bitwise-equal
// results, tested), reorganised for MI355X:
//   * workgroup = one fixed (16-unit column tile, 16-utterance row tile) task for the whole
//     sweep; its weight slices live in VGPRs (per wave: its K-quarter of 16 rows, H/64 float4
//     per matrix), so no weight byte is re-read per step;
//   * the two all-to-all seams of a GRU step (h_{t-1} -> [z|r], q = r*h -> hh) are in-launch
//     hand-offs in the "data is the flag" form (MI355X guide §6 Guideline 16, R2): every
//     handed-off fp32 value travels as ONE 8-byte {value, tag} granule stored write-through
//     (sc1); a consumer wave re-reads exactly the granules its MFMA operands need (16-byte sc1
//     loads) until every tag equals the step's epoch -- no flags, fences or counters;
//   * 16-utterance row tiles are independent chains (a tile only waits on its own rows);
//     granule buffers are double-buffered by step parity (a slot is rewritten two steps later,
//     which the dependency chain orders after every read of it) and zeroed by a memset node
//     before each launch; epochs are 1 + step index within the launch;
//   * operands that come from earlier kernels (x-projections, saved activations, dy) are
//     loaded before the wait so their latency hides under it;
//   * every wait is bounded: on timeout a wave raises the launch's abort word, every waiting
//     wave sees it within 64 polls, all workgroups leave at their next barrier.
#include <algorithm>
#include <cstdlib>

#include "gru.h"
#include "gru_persist.h"
#include "handoff.h"
#include "skinny.h"

namespace s2s {

namespace {

struct PDir {
  const float* xp;
  long ldxp;
  const float* Wa;  // fwd: Uzr (2H,H)   bwd: UhT (H,H)
  const float* Wb;  // fwd: Uh  (H,H)    bwd: UzrT (H,2H)
  float* y;
  long ldy;
  float* sv;  // (B, L, 5H)
  const float* dy;
  long lddy;
  float* dA;
  long ldA;
  int reverse;
  // granule buffers, each [2 slots][B][H] x 8 bytes
  granule_t* g0;  // fwd: h      bwd: da_z
  granule_t* g1;  // fwd: q      bwd: da_r
  granule_t* g2;  //             bwd: da_h
  // sentinel rows (XCD-local chains), each [L slots][B][H] floats, same roles as g0..g2
  float* s0;
  float* s1;
  float* s2;
};
// Fused x-projection (forward): the placement grid's spare XCDs (slots past the chains) compute
// xp = x Wx^T themselves, time slice by time slice in the order the recurrence consumes them, instead
// of a GEMM launch in front of the layer.  Work item = (slice, direction, 64-column tile) of a
// 64-row tile whose rows are (utterance b, step j of the slice); the MFMA schedule and k order are
// gemm_f32's 64x64 NT kernel (bitwise-equal xp; work items dealt round-robin to the producers, so
// every loop bound is uniform).  Hand-off (cross-XCD): write-through stores, every
// wave drains, one agent-scope add per tile to the slice's counter; a consumer polls the counter
// (sc1) and then reads xp with sc1 loads (MI355X guide, visibility table row 1).
// The backward uses the same producers for its dy (fused dX of the layer above, gemm_f32's 64x64 NN
// kernel order): x = that layer's gate gradients dA (K = 3 nd H' columns), W = its x-weights (K, D')
// read row-contiguous (nn = 1), xp = this layer's dy; slices follow the BPTT's processing order
// (flip = 1: processing index s is time L-1-s for the forward direction).
struct XProj {
  const float* x;
  long ldx;
  int K;            // padded input width (% 32 == 0): x and W hold K readable columns
  const float* W;   // NT (forward): (nd*ncd, ldw) x-weights, direction d's rows [ncd d, ncd (d+1)); NN: (K, ldw)
  long ldw;
  int ncd, flip;  // (the W layout is the producer's NN template argument: forward NT, backward NN)
  float* xp;
  long ldxp;
  int tpt;          // steps per slice (64 / B)
  int nslices, ntn, nwork, nd;
  unsigned* done;   // [nd][nslices] finished column tiles
  // optional (the top layer's dy = the decoder's dh): xp += sum_t alpha[b, t, l] dc[b, t, col], alpha
  // (B, T, L), dc (B, T, ldxp) -- the context term, beside the MFMA's dVh V
  const float* alpha;
  const float* dc;
  int T;
  // split-K start (backward): slices [0, sA) are cut into PA K-parts, [sA, sB) into PB, the rest whole, so
  // the first slices the recurrence needs are ready after a fraction of a tile's K loop; a split item's parts
  // write partial tiles to `slab` ([item][PA][16][256]) and the last part to finish (icnt[item]) sums them in
  // part order and publishes the tile.  nwork counts units (parts).
  int sA, sB, PA, PB;
  float* slab;
  unsigned* icnt;
  // XCD-grouped dealing of the whole (unsplit) units (G > 0): the producers come in G groups of gsz, one
  // group per XCD (consecutive spare-slot indices share a chain slot); group g takes direction g % nd and every
  // (G / nd)-th slice from sB + g / nd, its members round-robin over that class's (slice, column tile) units.
  // An XCD then streams one direction's x-weights (K x 4 column tiles: 1.6 MB at config 2) instead of all of
  // them (3.1 MB) next to its slices' x tiles, which with plain round-robin dealing (two slices x all units
  // per XCD) overflowed its 4 MB L2 and re-read the weights from memory for every pair of slices.
  int G, gsz, nsplit;
};
constexpr int kXpMaxSplitItems = 64;

// work unit u of the producers' round-robin: slice, direction, column tile, K-part of P, split item (-1: whole)
struct XUnit {
  int sl, d, ct, part, P, item;
};
__device__ __forceinline__ XUnit xunit(const XProj& q, int nd, int u) {
  const int per = nd * q.ntn, nA = q.sA * per * q.PA, nB = (q.sB - q.sA) * per * q.PB;
  XUnit x;
  int rem;
  if (u < nA) {
    const int i = u / q.PA;
    x.P = q.PA; x.part = u - i * q.PA; x.item = i; x.sl = i / per; rem = i - x.sl * per;
  } else if (u < nA + nB) {
    const int v = u - nA, i = v / q.PB;
    x.P = q.PB; x.part = v - i * q.PB; x.item = q.sA * per + i; x.sl = q.sA + i / per; rem = i % per;
  } else {
    const int v = u - nA - nB;
    x.P = 1; x.part = 0; x.item = -1; x.sl = q.sB + v / per; rem = v % per;
  }
  x.d = rem / q.ntn;
  x.ct = rem - x.d * q.ntn;
  return x;
}
// the it-th unit of producer p (false: none left).  Split units (w < nsplit) and, without grouping, all units:
// the round-robin w = p + it nprod; with grouping (XProj::G), the whole units of p's group in class order
__device__ __forceinline__ bool xunit_of(const XProj& q, int nd, int p, int nprod, int it, XUnit& x) {
  const int w = p + it * nprod;
  if (q.G == 0 || w < q.nsplit) {
    if (w >= q.nwork) return false;
    x = xunit(q, nd, w);
    return true;
  }
  const int nsp = q.nsplit > p ? (q.nsplit - p + nprod - 1) / nprod : 0;  // p's split units
  const int g = p / q.gsz, v = p - g * q.gsz + (it - nsp) * q.gsz;
  const int ncls = q.G / nd, i = v / q.ntn;
  x.sl = q.sB + i * ncls + g / nd;
  if (x.sl >= q.nslices) return false;
  x.d = g % nd;
  x.ct = v - i * q.ntn;
  x.part = 0;
  x.P = 1;
  x.item = -1;
  return true;
}
constexpr int kXpLds = 4 * 64 * 36 * 4;  // producer LDS: A and B tiles, double-buffered

// In-launch weight gradients of a BPTT (bptt_wgrad; gru_persist_bwd's wgrad): nw = 3H/64 workers per chain, or 0
struct WArgs {
  int nw;
  float* dW[2][3];  // dW[d][gate] (3 gates x H rows, H + D columns): dW += scale dA^T [h_{t-1} or q | x]
  float scale;
  const float* x;  // the layer input (B*L, ldx), D columns read (zero past D)
  long ldx;
  int D, NP;        // x columns; partial row length H + round_up(D, 16)
  float* part;      // [ndir][MT][3H][NP] the 16-utterance tiles' partial sums (MT > 1)
  unsigned* ticket;  // [ndir][nw] arrival counters (zeroed with the sync region)
  // diagnostic (s2s_debug_gru_wg_stamps): [nchains][nw][L + 4] s_memrealtime at entry, census checked, each
  // step's products issued, loop end, exit
  unsigned long long* stamps;
};

struct PArgs {
  XProj xq;
  int fused;
  PDir d[2];
  int B, L, H, MT, nwg;  // nwg = workgroups per direction
  int nmem, nchains;     // chains = (direction, 16-row tile); members = column tiles
  int allow_local;       // 0 forces write-through (sc1) hand-offs even on an XCD-local chain
  unsigned* abort_word;
  unsigned* census;      // [nchains][nmem] XCC ids (chain_is_local)
  const int* len;        // (B) frames per utterance (null: all L): h_t = 0 for t >= len_b
  // the next persistent GRU launch's sync region (other than this one's), prepared by this launch's spare
  // slots -- what sync_prep would do in front of that launch (zero [256, next_prep), fresh epoch, abort 0)
  char* next_sync;
  size_t next_prep;
  GruPackJobs pack;  // weight packing for later launches, done by the forward's spare slots (pack.n = 0: none)
  // sentinel slots in use per role: kSentRing (a ring, re-armed by the loader wave two steps after every
  // consumer has read a slot) or 0 (one slot per step, all re-armed at launch start; s2s_debug_gru_ring(0))
  int ring;
  // the BPTT's first sweep (da_h) multiplied chunk by chunk as the chunks arrive (sweep_sent_mfma); 0: sweep, then
  // multiply.  (The forward's sweeps stay whole: streamed, the forward measured 1030 -> 1349 us per config-2 step.)
  int stream_sweep;
  unsigned long long* stamps;  // diagnostic: [grid][L][8] s_memrealtime, or nullptr
  unsigned long long* pstamps;  // diagnostic: producers [producer][kProdStampItems][2] item start / end
  // BPTT row prefetchers (bwd only): prefetch = lookahead in steps (0: off), progress = [nchains][nmem] words each
  // member's loader sets to its step (zeroed with the region)
  int prefetch, prefetch_wg;  // lookahead, prefetcher workgroups per chain
  unsigned* progress;
  WArgs wg;  // bwd: in-launch weight gradients (wg.nw = 0: off); needs progress
};

// diagnostic stamps (s2s_debug_gru_stamps): per (workgroup, step) at p1 sweep start / done /
// end and p2 sweep start / done / end; forward p1 sub-phases: 6 = MFMA issued, 7 = reduced
// S2S_GRU_DIAG=1 (a diagnostic build, tools/ab_variant.sh): 16 slots per (workgroup, step), slots 8.. hold the
// poll passes of each sweep and the da_z sweep's end (tools/gru_stamps.py --diag); production builds keep 8
#ifndef S2S_GRU_DIAG
#define S2S_GRU_DIAG 0
#endif
constexpr int kStampSlots = S2S_GRU_DIAG ? 16 : 8;
#define GRU_STAMP(ph)                                                                      \
  do {                                                                                     \
    if (a.stamps && threadIdx.x == 0)                                                      \
      a.stamps[((long)lw * a.L + s) * kStampSlots + (ph)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#define GRU_STAMP_V(ph, v)                                                                 \
  do {                                                                                     \
    if (a.stamps && threadIdx.x == 0) a.stamps[((long)lw * a.L + s) * kStampSlots + (ph)] = (v); \
  } while (0)
#if S2S_GRU_DIAG
// sweep_sent_tile counting its poll passes (diagnostic builds only)
template <int NC>
__device__ __forceinline__ bool sweep_sent_n(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long tbase, int rowt,
                                             int wave, int lane, unsigned* abort_word, unsigned& n) {
  const long lo = tbase + 4 * tile_lane(rowt, lane);
  unsigned spins = 0;
  while (true) {
    ++n;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = lo + 4L * 256 * (wave + 4 * i);
      const uint4 p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
      a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}
#define SWEEP_SENT(slot_, ...) sweep_sent_n<NC>(__VA_ARGS__, npoll[slot_])
#else
#define SWEEP_SENT(slot_, ...) sweep_sent_tile<NC>(__VA_ARGS__)
#endif
std::atomic<unsigned long long*> g_gru_stamps[2] = {{nullptr}, {nullptr}};
std::atomic<unsigned long long*> g_gru_pstamps[2] = {{nullptr}, {nullptr}};
std::atomic<unsigned long long*> g_gru_wstamps{nullptr};
constexpr int kProdStampItems = 32;

// cross-wave sum + abort agreement at the same barrier
__device__ __forceinline__ float reduce_or_abort(SkinnyRed& red, int* abort_lds, bool ok, floatx4 acc, int wave,
                                                 int lane, int tid, bool* aborted) {
  if (!ok) *abort_lds = 1;
  const float s = skinny_reduce(red, acc, wave, lane, tid);
  *aborted = *abort_lds != 0;
  return s;
}

// ------------------------------------------------------------------------------ fused x-projection
// producer p of nprod takes work items p, p + nprod, ... (a static round-robin in consumption order:
// uniform loop bounds, no shared work counter).  NN: W is (K, ldw) read row-contiguous (the backward's
// dy); D: K-tiles in flight, a divisor of K / 32 (xproj_depth).
// K-tiles are loaded D ahead into a register ring: a producer owns its CU with one wave per SIMD, so one
// tile of MFMA work (~0.4 us) cannot cover an HBM load.  The main loop is branch-free (a steady part that
// loads, stores and multiplies every iteration, then a D-iteration drain), so the compiler's vmcnt waits
// count exactly the loads of the tile being stored.  Out-of-range tile rows load row 0 of x (valid, finite
// data) as they are: a GEMM's output row depends on its own A row only, and those rows are never stored
// (zeroing them with a select made the compiler hoist every ring slot's select, i.e. wait for every load).
template <bool NN, int D>
__device__ __forceinline__ void xproj_produce(const PArgs& a, float* lds, int p, int nprod) {
  const XProj& q = a.xq;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nk = q.K / 32;
  __shared__ int last_part;  // split item: this block's part was the last to finish
  const int nd = q.nd;
  if (tid >= 256) {  // a 320-thread block's 5th (row loader) wave: only the producer's barriers
    XUnit x;
    for (int it = 0; xunit_of(q, nd, p, nprod, it, x); ++it) {
      const int nb = 1 + nk / x.P + (q.alpha ? 1 : 0);
      for (int i = 0; i < nb; ++i) __syncthreads();
      if (x.P == 1) {
        __syncthreads();
      } else {
        __syncthreads();
        __syncthreads();
        if (last_part) __syncthreads();
      }
    }
    return;
  }
  const int wy = wave >> 1, wx = wave & 1, li = lane & 31, lk = lane >> 5;
  const int B = a.B, L = a.L, H3 = q.ncd;
  constexpr int LDK = 36;
  float* As[2] = {lds, lds + 64 * LDK};
  float* Bs[2] = {lds + 128 * LDK, lds + 192 * LDK};
  int item = 0;
  XUnit xu;
  for (; xunit_of(q, nd, p, nprod, item, xu); ++item) {
    if (a.pstamps && tid == 0 && item < kProdStampItems)
      a.pstamps[((long)p * kProdStampItems + item) * 2] = __builtin_amdgcn_s_memrealtime();
    const int sl = xu.sl, d = xu.d, ct = xu.ct;
    const int nkp = nk / xu.P, kb = xu.part * nkp;  // this unit's K-tiles [kb, kb + nkp)
    const int rev = a.d[d].reverse ^ q.flip;
    // this thread's two A rows (tile rows tid/8 and 32 + tid/8) and B rows (NN: B columns 4 (f / 32) ..
    // + 3 of k row f % 32, gemm_f32's row-contiguous loader)
    const float* arow[2];
    const float* brow[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = (tid >> 3) + 32 * j, jt = r / B, b = r - jt * B, s = sl * q.tpt + jt;
      const bool aval = jt < q.tpt && s < L;
      const int t = rev ? L - 1 - s : s;
      arow[j] = q.x + (aval ? ((long)b * L + t) * q.ldx : 0);
      const int f = tid + 256 * j;
      brow[j] = NN ? q.W + (long)(f & 31) * q.ldw + d * H3 + ct * 64 + 4 * (f >> 5)
                   : q.W + (long)(d * H3 + ct * 64 + r) * q.ldw;
    }
    const int kq = 4 * (tid & 7);
    const long bstep = NN ? 32 * q.ldw : 32;  // B advance per K-tile
    floatx4 ra[D][2], rb[D][2];
    auto gload = [&](floatx4 (&xa)[2], floatx4 (&xb)[2], int kt) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        xa[j] = *reinterpret_cast<const floatx4*>(arow[j] + 32 * kt + kq);
        xb[j] = *reinterpret_cast<const floatx4*>(brow[j] + kt * bstep + (NN ? 0 : kq));
      }
    };
    auto lstore = [&](const floatx4 (&xa)[2], const floatx4 (&xb)[2], int buf) {
      float* as = As[0] + buf * (64 * LDK);
      float* bs = Bs[0] + buf * (64 * LDK);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int f = tid + 256 * j;
        *reinterpret_cast<floatx4*>(as + (f >> 3) * LDK + 4 * (f & 7)) = xa[j];
        if (NN) {
          float* pb = bs + (4 * (f >> 5)) * LDK + (f & 31);
          pb[0] = xb[j][0];
          pb[LDK] = xb[j][1];
          pb[2 * LDK] = xb[j][2];
          pb[3 * LDK] = xb[j][3];
        } else {
          *reinterpret_cast<floatx4*>(bs + (f >> 3) * LDK + 4 * (f & 7)) = xb[j];
        }
      }
    };
    floatx16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    // gemm_f32's double-buffered 64x64 main loop, same MFMA order
    // the MFMAs of one K-tile with `mid` (the next tile's LDS store) issued between its two halves, so the
    // LDS writes and their wait overlap the second half's MFMAs (sched_barrier pins the placement)
    auto mma = [&](int buf, auto&& mid) {
      floatx4 av[4], bv[4];
      const float* pa = As[0] + buf * (64 * LDK) + (wy * 32 + li) * LDK + 16 * lk;
      const float* pb = Bs[0] + buf * (64 * LDK) + (wx * 32 + li) * LDK + 16 * lk;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        av[c] = *reinterpret_cast<const floatx4*>(pa + 4 * c);
        bv[c] = *reinterpret_cast<const floatx4*>(pb + 4 * c);
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[c][e], bv[c][e], acc, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      mid();
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int c = 2; c < 4; ++c)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[c][e], bv[c][e], acc, 0, 0, 0);
    };
#pragma unroll
    for (int i = 0; i < D; ++i) gload(ra[i], rb[i], kb + i);
    lstore(ra[0], rb[0], 0);
    __syncthreads();
    // steady part: iteration kt (slot kt % D holds tile kt, already in LDS) reloads that slot with tile
    // kt + D, multiplies LDS buffer kt & 1 and stores slot (kt + 1) % D into the other buffer
    for (int kt0 = 0; kt0 < nkp - D; kt0 += D) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const int kt = kt0 + j;
        gload(ra[j], rb[j], kb + kt + D);
        mma(kt & 1, [&] { lstore(ra[(j + 1) % D], rb[(j + 1) % D], (kt + 1) & 1); });
        __syncthreads();
      }
    }
    // drain: the last D tiles are all loaded
#pragma unroll
    for (int j = 0; j < D; ++j) {
      const int kt = nkp - D + j;
      mma(kt & 1, [&] {
        if (j + 1 < D) lstore(ra[(j + 1) % D], rb[(j + 1) % D], (kt + 1) & 1);
      });
      __syncthreads();
    }
    const int col = d * H3 + ct * 64 + wx * 32 + li;
    if (q.alpha) {
      // the decoder's context term of dh: ctx[row][c] = sum_t alpha[b, t, l] dc[b, t, c] in a fixed t order,
      // computed with its own mapping (4 rows x 4 consecutive columns per thread: float4 dc loads, 4 steps
      // of loads in flight) into the (now free) LDS tile area, then added to the MFMA outputs.  Rows outside
      // the tile read utterance 0, frame 0 and are not stored.
      float* ctxl = lds;  // [64][68]
      const int c4 = 4 * (tid & 15), r0 = 4 * (tid >> 4);
      long arow_[4], drow_[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int tr = r0 + i, jt = tr / B, s = sl * q.tpt + jt;
        const bool v = jt < q.tpt && s < L;
        const int b = v ? tr - jt * B : 0, l = v ? (rev ? L - 1 - s : s) : 0;
        arow_[i] = (long)b * q.T * L + l;
        drow_[i] = (long)b * q.T * q.ldxp + d * H3 + ct * 64 + c4;
      }
      floatx4 cx[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) cx[i] = floatx4{0.f, 0.f, 0.f, 0.f};
      // a split item's parts take consecutive ranges of t
      const int te = ((xu.part + 1) * q.T) / xu.P;
      int tt = (xu.part * q.T) / xu.P;
      for (; tt + 4 <= te; tt += 4) {
        float av[4][4];
        floatx4 dv[4][4];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            av[u][i] = q.alpha[arow_[i] + (long)(tt + u) * L];
            dv[u][i] = *reinterpret_cast<const floatx4*>(q.dc + drow_[i] + (long)(tt + u) * q.ldxp);
          }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int e = 0; e < 4; ++e) cx[i][e] += av[u][i] * dv[u][i][e];
      }
      for (; tt < te; ++tt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float av = q.alpha[arow_[i] + (long)tt * L];
          const floatx4 dv = *reinterpret_cast<const floatx4*>(q.dc + drow_[i] + (long)tt * q.ldxp);
#pragma unroll
          for (int e = 0; e < 4; ++e) cx[i][e] += av * dv[e];
        }
#pragma unroll
      for (int i = 0; i < 4; ++i) *reinterpret_cast<floatx4*>(ctxl + (r0 + i) * 68 + c4) = cx[i];
      __syncthreads();  // (a 320-thread block's 5th wave matches it in its barrier loop)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += ctxl[(wy * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk) * 68 + wx * 32 + li];
    }
    if (xu.P > 1) {
      // split item: publish this part's partial tile (write-through 16-byte stores, each thread's 16 values
      // contiguous); the last part to finish sums all parts in part order
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const __amdgpu_buffer_rsrc_t srs = rsrc_of(q.slab);
      const int ibase = (xu.item * q.PA) * 16384 + tid * 64;  // byte offset of part 0, this thread
#pragma unroll
      for (int i = 0; i < 4; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, floatx4{acc[4 * i], acc[4 * i + 1], acc[4 * i + 2], acc[4 * i + 3]}), srs,
            ibase + xu.part * 16384 + 16 * i, 0, 16);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0)
        last_part = __hip_atomic_fetch_add(q.icnt + xu.item, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                    (unsigned)(xu.P - 1);
      __syncthreads();
      if (!last_part) {
        if (a.pstamps && tid == 0 && item < kProdStampItems)
          a.pstamps[((long)p * kProdStampItems + item) * 2 + 1] = __builtin_amdgcn_s_memrealtime();
        continue;
      }
      floatx4 pv[4][4];  // [part][quad], all loads in flight together (sc1: written by other XCDs)
#pragma unroll
      for (int pp = 0; pp < 4; ++pp)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          pv[pp][i] = pp < xu.P ? __builtin_bit_cast(floatx4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                  srs, ibase + pp * 16384 + 16 * i, 0, 16))
                                : floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float v = pv[0][i][e] + pv[1][i][e];
          if (xu.P > 2) v = (v + pv[2][i][e]) + pv[3][i][e];
          acc[4 * i + e] = v;
        }
    }
    // epilogue: write-through stores of the valid rows, drain, one counter add per tile
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int tr = wy * 32 + (r & 3) + 8 * (r >> 2) + 4 * lk, jt = tr / B, b = tr - jt * B, s = sl * q.tpt + jt;
      if (jt < q.tpt && s < L) {
        const int t = rev ? L - 1 - s : s;
        __hip_atomic_store(q.xp + ((long)b * L + t) * q.ldxp + col, 1.f * acc[r], __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(q.done + d * q.nslices + sl, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (a.pstamps && tid == 0 && item < kProdStampItems)
      a.pstamps[((long)p * kProdStampItems + item) * 2 + 1] = __builtin_amdgcn_s_memrealtime();
  }
}

// the producer with the deepest ring that divides K / 32
template <bool NN>
__device__ __forceinline__ void xproj_produce_any(const PArgs& a, float* lds, int p, int nprod) {
  const int nk = a.xq.K / 32;  // (a split start needs nk / PA % 4 == 0: xproj_split)
  if (nk % 4 == 0) xproj_produce<NN, 4>(a, lds, p, nprod);
  else if (nk % 3 == 0) xproj_produce<NN, 3>(a, lds, p, nprod);
  else if (nk % 2 == 0) xproj_produce<NN, 2>(a, lds, p, nprod);
  else xproj_produce<NN, 1>(a, lds, p, nprod);
}

// consumer side: is slice `sl` of direction d complete?  (one sc1 load)
__device__ __forceinline__ bool xproj_ready(const XProj& q, int d, int sl) {
  return __hip_atomic_load(q.done + d * q.nslices + sl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >=
         (unsigned)q.ntn;
}

// loader wave: wait until slice `need` of direction d is complete.  `ready` = slices known complete; a
// refresh reads the 64 counters ahead at once (lane i: slice ready + i) and advances to the first one not
// yet complete.  MUST run with all 64 lanes active (wave-uniform call site): an inactive lane's ballot bit
// reads as "complete", which would advance `ready` past a slice still being produced.
__device__ __forceinline__ void xproj_wait(const XProj& q, int d, int need, int& ready, int lane, unsigned* abort_word) {
  unsigned spins = 0;
  while (need >= ready) {
    const int sl = ready + lane;
    const unsigned long long nr = __ballot(!(sl >= q.nslices || xproj_ready(q, d, sl)));
    const int upto = nr ? ready + (int)__builtin_ctzll(nr) : ready + 64;
    if (upto <= need && spin_give_up(spins, abort_word)) break;
    ready = upto;
  }
}

// spare slot sp of nsp: its share of preparing the next launch's sync region (sync_prep's work; the region
// is not in use -- the launch before this one used it -- and the writes are visible when this launch ends)
__device__ __forceinline__ void prep_next_sync(const PArgs& a, int sp, int nsp) {
  if (!a.next_sync) return;
  if (sp == 0 && threadIdx.x == 0) {
    unsigned* hdr = reinterpret_cast<unsigned*>(a.next_sync);
    const unsigned e = __hip_atomic_fetch_add(&g_s2s_epoch_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_exchange(hdr + kEpochWord, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    rearm_abort_word(hdr);  // the previous launch's failure stays in the sticky bits until the harvest
  }
  const size_t n16 = (a.next_prep - 256) / 16;
  uint4* p = reinterpret_cast<uint4*>(a.next_sync + 256);
  for (size_t i = (size_t)sp * blockDim.x + threadIdx.x; i < n16; i += (size_t)nsp * blockDim.x)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
  if (threadIdx.x == 0 && sp == 0 && (a.next_prep - 256) % 16) {  // a last partial 16-byte piece
    unsigned* t = reinterpret_cast<unsigned*>(a.next_sync + 256 + n16 * 16);
    for (size_t i = 0; i < ((a.next_prep - 256) % 16) / 4; ++i) t[i] = 0u;
  }
}

// ------------------------------------------------------------------------------ forward
// chain (dir, mt) has nmem = 2H/16 members c1 (chain_slot placement, handoff.h); z-column
// workgroups (c1 < H/16) also own the candidate tile of the same units.
// Like the backward, forward blocks carry a 5th wave that loads the x-projections of coming steps into
// an LDS ring (and, with the fused x-projection, waits for their slices), so no global load or counter
// poll sits in front of a recurrence wave's sweep.  It joins the barriers [P], [A] (p1 reduce) and, in
// z-column blocks, [B] (p2 reduce); step q + 2's values are written between [A] of step q and [A] of
// step q + 1, after which the recurrence waves read them.
constexpr int kRowRing = 4;  // steps of loaded operands in flight (LDS ring)
// Sentinel slot ring (XCD-local chains).  A slot of step s is consumed by every chain member within the
// step after it was produced, and a member's sweep proves that every other member has finished with it:
//   forward  h_s  (z tiles; read by all members in p1 of step s+1): once a member's p1 sweep of step s+2 is
//            complete, every z member has published h_{s+1} (after reading h_s and, in p2 of s+1, every r
//            member's q_{s+1}, itself published after that r member read h_s) -- re-arm at [A] of step s+2;
//            q_s  (r tiles; read by z members in p2 of step s): the p1 sweep of step s+1 saw every z member's
//            h_s, published after its p2 read of q_s -- re-arm at [A] of step s+1;
//   backward da_h_p, da_z_p, da_r_p (read by all in p1 / p2 of step p): the p1 sweep of step p+1 saw every
//            member's da_h_{p+1}, published after its p2 of step p -- re-arm at [A] of step p+1.
// The re-arm of a member's own 1-KB tile is done by its loader wave between barriers and drained (vmcnt(0))
// before the barrier after which the member publishes again, so every value a consumer sees from that member
// later than the re-arm is ordered after it in the XCD's L2: with kSentRing = 4 the consumer of slot s + 4
// has already taken a value the member published after re-arming slot s, and cannot mistake slot s's stale
// value for step s + 4's.  Only kSentRing slots are live (a few KB per member instead of L KB), so the slots
// stay in L2: the per-step slots were re-armed at launch start and written again per step, most of both
// recurrences' HBM write traffic (profiles/r03/pmc_hbm.csv), and re-arming L slots delayed each launch's start.
constexpr int kSentRing = 4;
__device__ __forceinline__ int sent_slot(const PArgs& a, int s) { return a.ring ? (s & (a.ring - 1)) : s; }
// re-arm this member's 1-KB tile of slot s of one tile-major sentinel role (the loader wave's 64 lanes)
__device__ __forceinline__ void rearm_tile(float* role, const PArgs& a, int s, long tile, int lane) {
  const float4 sv = make_float4(__uint_as_float(kSent), __uint_as_float(kSent), __uint_as_float(kSent),
                                __uint_as_float(kSent));
  *reinterpret_cast<float4*>(role + (long)sent_slot(a, s) * a.MT * 16 * a.H + tile + 4 * lane) = sv;
}
constexpr int kFwdThreads = 320;
template <int NC>  // NC = H / 64
__global__ __launch_bounds__(kFwdThreads) void gru_fwd_persist(PArgs a) {
  __shared__ SkinnyRed red;
  __shared__ int abort_lds, local_lds;
  __shared__ unsigned tb_lds;
  __shared__ __attribute__((aligned(16))) float hprev[16][16];  // r tiles: h_{t-1} of the tile's units
  __shared__ __attribute__((aligned(16))) float xring[kRowRing][2][256];  // [step % ring][gate | candidate][thread]
  // this step's saved activations and output, staged for the loader wave's global stores: z tiles [z | hh | h],
  // r tiles [r | h_{t-1} | q] (a recurrence wave's own global stores sat in its vmcnt queue in front of its next
  // sweep: forward step 2.52 -> 2.40 us with them switched off)
  __shared__ __attribute__((aligned(16))) float stg[2][3][256];
  extern __shared__ __attribute__((aligned(16))) float xlds[];  // producer tiles (fused x-projection)
  const int H = a.H, B = a.B, L = a.L;
  const ChainSlot cs = chain_slot(a.nmem);
  if (cs.chain >= a.nchains) {  // spare slot of the placement grid: x-projection producer (or idle)
    const int gch = 8 * ((a.nchains + 7) / 8);
    const int sp = (cs.chain - a.nchains) * a.nmem + cs.member, nsp = (gch - a.nchains) * a.nmem;
    prep_next_sync(a, sp, nsp);
    if (a.fused) xproj_produce_any<false>(a, xlds, sp, nsp);
    for (int j = 0; j < a.pack.n; ++j)  // after the x-projections: the chains wait for those, not for this
      gru_pack_elems(a.pack.j[j], (long)sp * blockDim.x + threadIdx.x, (long)nsp * blockDim.x);
    return;
  }
  const int dir = cs.chain / a.MT, mt = cs.chain % a.MT;
  const PDir& g = a.d[dir];
  const int ncol = 2 * H / 16;
  const int c1 = cs.member;
  const int lw = dir * a.nwg + mt * ncol + c1;  // logical workgroup id (stamps)
  const bool isz = c1 < H / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = mt * 16;
  if (tid == 0) abort_lds = 0;
  const unsigned tb = launch_tagbase(a.abort_word, &tb_lds);
  // z tiles publish h, r tiles q
  const bool loader = wave == 4;
  const long mytile = (long)mt * 16 * H + (long)(isz ? c1 : c1 - H / 16) * 256;  // this member's tile in a slot
  if (!loader)  // this member's 1-KB tile of every (tile-major) slot in use
    rearm_rect((isz ? g.s0 : g.s1) + mytile, (long)a.MT * 16 * H, a.ring ? a.ring : L, 16, 0, 16, 0, 16);
  rearm_done();
  const bool loc = chain_is_local(a.census, cs.chain, a.nmem, c1, a.allow_local != 0, a.abort_word, &local_lds, tb);

  if (loader) {
    // lane l: utterance b0 + (l >> 2) of the tile, columns c1 * 16 + 4 (l & 3) .. + 3
    const int bl = b0 + (lane >> 2), col = c1 * 16 + 4 * (lane & 3);
    const bool lv = bl < B;
    const __amdgpu_buffer_rsrc_t xr = rsrc_of(g.xp);
    int xready = 0;  // fused: slices known complete (one refresh of 64 counters at a time)
    auto issue = [&](int q, float4 (&r)[2]) {
      r[0] = r[1] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q >= L) return;
      if (a.fused) xproj_wait(a.xq, dir, q / a.xq.tpt, xready, lane, a.abort_word);  // all lanes
      if (!lv) return;
      const int t = g.reverse ? L - 1 - q : q;
      const long off = ((long)bl * L + t) * g.ldxp + col;
      if (a.fused) {
        r[0] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(4 * off), 0, 16));
        if (isz)
          r[1] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(xr, (int)(4 * (off + 2 * H)), 0, 16));
      } else {
        r[0] = *reinterpret_cast<const float4*>(g.xp + off);
        if (isz) r[1] = *reinterpret_cast<const float4*>(g.xp + off + 2 * H);
      }
    };
    auto put = [&](int q, const float4 (&r)[2]) {
      *reinterpret_cast<float4*>(&xring[q % kRowRing][0][4 * lane]) = r[0];
      *reinterpret_cast<float4*>(&xring[q % kRowRing][1][4 * lane]) = r[1];
    };
    // step q's staged values -> saved activations / output (float4 of this lane's 4 columns)
    auto store = [&](int q) {
      if (!lv) return;
      const int t = g.reverse ? L - 1 - q : q;
      const long row = (long)bl * L + t;
      const float4 v0 = *reinterpret_cast<const float4*>(&stg[q & 1][0][4 * lane]);
      const float4 v1 = *reinterpret_cast<const float4*>(&stg[q & 1][1][4 * lane]);
      const float4 v2 = *reinterpret_cast<const float4*>(&stg[q & 1][2][4 * lane]);
      float* sv = g.sv + row * 5 * H;
      if (isz) {
        *reinterpret_cast<float4*>(sv + col) = v0;
        *reinterpret_cast<float4*>(sv + 2 * H + col) = v1;
        *reinterpret_cast<float4*>(g.y + row * g.ldy + col) = v2;
      } else {
        const int j = col - H;
        *reinterpret_cast<float4*>(sv + H + j) = v0;
        *reinterpret_cast<float4*>(sv + 3 * H + j) = v1;
        *reinterpret_cast<float4*>(sv + 4 * H + j) = v2;
      }
    };
    float4 ra[2], rb[2];
    issue(0, ra);
    issue(1, rb);
    put(0, ra);
    put(1, rb);
    issue(2, ra);
    __syncthreads();  // [P]
    const bool ring = a.ring && loc;
    for (int s = 0; s < L; ++s) {
      if (ring) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the last step's re-arms have landed
      __syncthreads();  // [A]
      if (abort_lds) return;
      if (s > 0) store(s - 1);  // written by the recurrence waves before this barrier
      put(s + 2, ra);   // loaded during the previous step
      issue(s + 3, ra);
      if (ring) {  // slots every member has finished with (h_{s-2} of z tiles, q_{s-1} of r tiles)
        if (isz && s >= 2) rearm_tile(g.s0, a, s - 2, mytile, lane);
        if (!isz && s >= 1) rearm_tile(g.s1, a, s - 1, mytile, lane);
      }
      if (!isz) continue;
      __syncthreads();  // [B]
      if (abort_lds) return;
    }
    __syncthreads();  // [C]: the last step's values are staged
    store(L - 1);
    return;
  }

  float4 w1[NC], w2[NC];
  load_wfrag(w1, g.Wa + (long)(c1 * 16 + (lane & 15)) * H, wave, lane);
  if (isz) load_wfrag(w2, g.Wb + (long)(c1 * 16 + (lane & 15)) * H, wave, lane);

  const __amdgpu_buffer_rsrc_t hg = rsrc_of(g.g0), qg = rsrc_of(g.g1), hs = rsrc_of(g.s0), qs = rsrc_of(g.s1);
  const long slot = (long)B * H;  // granules per slot
  const long slotS = (long)a.MT * 16 * H, tileS = (long)mt * 16 * H;  // tile-major sentinel slot, this row tile
  const int rowt = min(b0 + (lane & 15), B - 1) - b0;
  const int br = min(b0 + (lane & 15), B - 1);
  const int ob = b0 + (tid >> 4), on = c1 * 16 + (tid & 15);  // this thread's output
  const bool live = ob < B;
  // variable-length batch: h_t = m_t GRU(h_{t-1}, x_t), m_t = 1[t < len_b] -- the reverse direction then
  // starts from h = 0 at the utterance's own last frame, as the reference's per-utterance nn.RNN does
  const int lenb = (a.len && live) ? a.len[ob] : L;
  // r tiles: units [jt, jt + 16) of h_{t-1} are chunk it of wave wt in the sweep layout
  const int jt = c1 * 16 - H, wt = (jt % 64) / 16, it = jt / 64;
  float zreg = 0.f, hreg = 0.f;
  bool aborted = false;

  __syncthreads();  // [P]
  for (int s = 0; s < L; ++s) {
    const int t = g.reverse ? L - 1 - s : s;
    // ---- p1: [z | r] = sig(Uzr h_{t-1} + xp)
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    bool ok = true;
    GRU_STAMP(0);
    if (s > 0) {
      float4 av[NC];
#if S2S_GRU_DIAG
      unsigned npoll[1] = {0};
#endif
      {
      if (loc) ok = SWEEP_SENT(0, av, hs, 4 * (sent_slot(a, s - 1) * slotS + tileS), rowt, wave, lane, a.abort_word);
      else ok = sweep_skinny<NC>(av, hg, 8 * (((s - 1) & 1) * slot + (long)br * H), tb + s, wave, lane, a.abort_word);
      GRU_STAMP(1);
#if S2S_GRU_DIAG
      GRU_STAMP_V(8, npoll[0]);
#endif
      acc = mfma_chunks<NC>(av, w1);
      }
      // r tiles: the swept operand already holds h_{t-1} of this tile's 16 units (chunk it of
      // wave wt); park it in LDS for the q = r * h epilogue (read after the reduce barrier)
      if (!isz && wave == wt) {
#pragma unroll
        for (int i = 0; i < NC; ++i)
          if (i == it) *reinterpret_cast<float4*>(&hprev[lane & 15][4 * (lane >> 4)]) = av[i];
      }
    }
    GRU_STAMP(6);
    float sum = reduce_or_abort(red, &abort_lds, ok, acc, wave, lane, tid, &aborted);
    GRU_STAMP(7);
    // this step's x-projections from the loader's ring (written before [A] of the previous step)
    const float xpv = xring[s % kRowRing][0][tid], xph = xring[s % kRowRing][1][tid];
    // r tiles' h_{t-1} (parked before the reduce barrier), read by every thread so the load is issued with the
    // reduce's reads instead of one more LDS round trip inside the r-tile epilogue
    const float hpark = hprev[tid >> 4][tid & 15];
    {
      const float gate = gru_sigmoid(sum + xpv);
      float* st3 = &stg[s & 1][0][tid];  // [0] / [256] / [512]: the three staged values of this step
      if (isz) {
        st3[0] = gate;
        zreg = gate;
      } else {
        const int j = on - H;
        const float hp = s > 0 ? hpark : 0.f;
        const float q = gate * hp;
        if (loc) {  // critical first
          if (live) put_sent(g.s1 + sent_slot(a, s) * slotS + tile_off(ob, j, H), q);
        } else {
          put_granule_pair(g.g1, (s & 1) * slot + (long)ob * H + j, q, tb + s + 1, live);
        }
        st3[0] = gate;
        st3[256] = hp;
        st3[512] = q;
      }
    }
    GRU_STAMP(2);
    if (aborted) return;  // checked after the epilogue: its LDS read is issued with the reduce's reads
    if (!isz) continue;
    // ---- p2: hh = tanh(Uh q + xp_h); h = (1-z) h_{t-1} + z hh
    acc = floatx4{0.f, 0.f, 0.f, 0.f};
    ok = true;
    GRU_STAMP(3);
    if (s > 0) {
      float4 av[NC];
#if S2S_GRU_DIAG
      unsigned npoll[1] = {0};
#endif
      {
      if (loc) ok = SWEEP_SENT(0, av, qs, 4 * (sent_slot(a, s) * slotS + tileS), rowt, wave, lane, a.abort_word);
      else ok = sweep_skinny<NC>(av, qg, 8 * ((s & 1) * slot + (long)br * H), tb + s + 1, wave, lane, a.abort_word);
      GRU_STAMP(4);
#if S2S_GRU_DIAG
      GRU_STAMP_V(9, npoll[0]);
#endif
      acc = mfma_chunks<NC>(av, w2);
      }
    }
    sum = reduce_or_abort(red, &abort_lds, ok, acc, wave, lane, tid, &aborted);
    {
      const float hh = gru_tanh(sum + xph);
      const float hp = hreg;
      hreg = (-zreg + 1.0f) * hp + zreg * hh;
      if (t >= lenb) hreg = 0.f;
      if (loc) {  // first
        if (live) put_sent(g.s0 + sent_slot(a, s) * slotS + tile_off(ob, on, H), hreg);
      } else {
        put_granule_pair(g.g0, (s & 1) * slot + (long)ob * H + on, hreg, tb + s + 1, live);
      }
      stg[s & 1][1][tid] = hh;
      stg[s & 1][2][tid] = hreg;
    }
    GRU_STAMP(5);
    if (aborted) return;  // checked after the epilogue: its LDS read is issued with the reduce's reads
  }
  __syncthreads();  // [C]: the loader stores the last step's staged values
}

// ------------------------------------------------------------------------------ backward
// chain (dir, mt) has nmem = H/16 members c, each the same column tile in both seams.
// Backward blocks have a 5th wave that only moves the saved activations and dy of the coming steps
// from HBM into an LDS ring (kRowRing steps): vmcnt is per wave and retires in order, so a row load
// issued by a recurrence wave would hold that wave's next sweep check for the HBM latency (measured:
// most of the p2 hand-off), while the loader wave's waits delay nothing but itself.  The loader joins
// every block barrier of the recurrence waves: [P] before the loop, [A] and [B] (the p1 / p2 reduces)
// per step; it writes row q + 2 between [A] and [B] of step q, which the recurrence waves read after
// [B] of step q + 1.
constexpr int kBwdThreads = 320;

// BPTT row prefetcher (one workgroup on an idle CU of each chain's XCD): the saved activations of a layer's BPTT
// were written by its forward pass a whole layer-stack earlier and, for the lower layers, have left the Infinity
// Cache: a member's loader wave then waits on HBM misses, either in front of the p2 barrier (its loads drained
// there) or beside the next sweep (in flight across it) -- the lower layers' BPTT step measured ~0.3 us longer
// than the top layer's even with the dy GEMM outside the launch.  The prefetcher reads the rows every member's
// loader will load `a.prefetch` steps before it does (following member 0's progress), so their loads hit this
// XCD's L2.  dy rows are touched only once their slice is complete (an earlier copy left in L2 would be served
// to the loader's sc1 loads: stale).  One workgroup per chain, not one per member: the other idle CUs stay free
// for the side stream's weight-gradient GEMMs (with a prefetcher per member the step measured 3.22 -> 3.59 ms
// before the skip-ahead below, 3.46 after it).  A prefetcher that starts late (its CU still held by a side-stream
// GEMM) skips the rows the loader has already taken, so it never holds the launch open past the chains.
// prefetcher w of nwg for chain `chain` takes members [w nmem / nwg, (w + 1) nmem / nwg): 64 nmem / nwg loader lanes
template <int NC>  // NC = H / 64 (nmem = 4 NC members, 256 NC (member, lane) tasks per chain and step)
__device__ __forceinline__ void bptt_prefetch(const PArgs& a, int chain, int w, int nwg) {
  if (threadIdx.x >= 256) return;
  const int tid = threadIdx.x, L = a.L, H = a.H, B = a.B, nmem = a.nmem;
  const int tasks = 64 * nmem / nwg, task0 = w * tasks;
  const int dir = chain / a.MT, mt = chain % a.MT;
  const PDir& g = a.d[dir];
  const unsigned* prog = a.progress + (long)chain * nmem;  // member 0's step
  int yready = 0, have = 0;
  float sink = 0.f;
  // member 0's progress is read by thread 0 alone and handed to the workgroup through LDS behind a barrier, so every
  // wave takes the same rows q: waves that polled on their own could skip ahead to different rows, and the fused-dy
  // barrier below would then line one wave's row q + 1 up with wave 0's readiness check for row q (a dy row of an
  // unfinished slice loaded into L2 early would later be served stale to the loader's sc1 loads).  Double-buffered by
  // iteration, so one barrier per row suffices (thread 0 rewrites a slot only after every thread passed the barrier
  // behind which it was last read).
  __shared__ int have_lds[2];
  int it = 0;
  // the (member, lane) tasks of one step, 256 at a time (member = task / 64, the loader's lane = task % 64), every
  // load of a step in flight together
  constexpr int kMaxTasks = NC;  // 64 nmem / 256 with nmem = H / 16
  for (int q = 3; q < L; ++q, ++it) {
    if (tid == 0) {
      unsigned spins = 0;
      bool gave_up = false;
      while (have + 3 + a.prefetch < q) {  // member 0's loader loads row q at its step q - 3
        have = (int)__hip_atomic_load(prog, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (have + 3 + a.prefetch >= q) break;
        if (spin_give_up(spins, a.abort_word)) {
          gave_up = true;
          break;
        }
      }
      have_lds[it & 1] = gave_up ? -1 : have;
    }
    __syncthreads();
    const int hv = have_lds[it & 1];
    if (hv < 0) return;  // (uniform) aborted launch
    have = hv;
    if (q < have + 4) q = have + 4;  // rows the loader has loaded (or is loading) already: skip ahead (uniform)
    if (q >= L) break;
    if (a.fused && tid < 64) xproj_wait(a.xq, dir, q / a.xq.tpt, yready, tid, a.abort_word);  // one wave, all lanes
    if (a.fused) __syncthreads();
    const int t = g.reverse ? q : L - 1 - q;
    float4 v[kMaxTasks][5];
#pragma unroll
    for (int k = 0; k < kMaxTasks; ++k) {
      if (256 * k >= tasks) break;  // (uniform)
      // (unconditional loads from valid rows -- the values are discarded: padding utterances read the last one)
      const int kt = tid + 256 * k, task = task0 + (kt < tasks ? kt : 0), m = task >> 6, lane = task & 63;
      const int bl = min(mt * 16 + (lane >> 2), B - 1), u = m * 16 + 4 * (lane & 3);
      const long row = (long)bl * L + t;
      const float* sv = g.sv + row * 5 * H + u;
#pragma unroll
      for (int f = 0; f < 4; ++f) v[k][f] = *reinterpret_cast<const float4*>(sv + f * H);
      v[k][4] = *reinterpret_cast<const float4*>(g.dy + row * g.lddy + u);
    }
    // the in-launch weight-gradient workers' own operand rows (bptt_wgrad): q = r h (sv + 4H, which the members do
    // not read) and the layer input x of the chain's 16 utterances at this step, one float4 per thread and 64 B
    float4 wv[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    if (a.wg.nw) {
      const int bl = min(mt * 16 + (tid >> 4), B - 1), cq = 4 * (tid & 15);  // 16 threads per utterance
      const long row = (long)bl * L + t;
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (cq + 64 * i < H) wv[0].x += g.sv[row * 5 * H + 4 * H + cq + 64 * i];
      if (cq < a.wg.D) wv[1].x = a.wg.x[row * a.wg.ldx + cq] + a.wg.x[row * a.wg.ldx + min(cq + 64, a.wg.D - 1)];
    }
#pragma unroll
    for (int k = 0; k < kMaxTasks; ++k) {
      if (256 * k >= tasks) break;
#pragma unroll
      for (int f = 0; f < 5; ++f) sink += v[k][f].x;
    }
    sink += wv[0].x + wv[1].x;
  }
  asm volatile("" ::"v"(sink));  // the loads stay
}

// In-launch weight gradients (gru_persist_bwd's wgrad: the model step's first encoder layer, whose BPTT is the
// step's last recurrence -- its weight-gradient GEMM used to follow the launch, ~90 us on the critical path):
//   dW_d[gate] += scale sum_{b, t} dA_d[b, t, gate]^T [h_{t-1} (q = r h for the candidate) | x]_{b, t}
// the GemmProblems of gru_layer_wgrad (LinearZeroBias.lua:67-74 accGradParameters, RNN.lua:194), computed by nw =
// 3H/64 workgroups on each chain's XCD (blockIdx = 8 w + chain past the prefetchers) step by step behind the chain:
// worker w of chain (dir, mt) owns the 64 gate rows [64 w, 64 w + 64) of direction dir (one gate) and every column,
// summed over the chain's 16 utterances; four waves of 16 x 16 x 4 fp32 MFMAs, wave v taking column blocks
// [kWgCB v, kWgCB (v + 1)).  Step p's gate gradients are final once every member's loader has passed [A] of step
// p + 3 (the member's p2 sweep of step p + 1 waited for loads issued after all its dA stores of step p: vmcnt retires
// in order), or at the members' final mark (L + 3, behind a vmcnt(0) + barrier after their last step).  The chain's
// dA rows stay in its XCD's L2 (plain stores), so a worker must share that XCD: one that does not (never seen; the
// round-robin placement every chain relies on) fails the launch rather than read stale rows.  The utterance tiles'
// partials are written through (sc1) and the last arriving tile (ticket) adds them in tile order into dW (guide's
// valid form: sc1 stores drained, one agent-scope add, sc1 loads) with one flat, coalesced loop.
constexpr int kWgCB = 6;  // column blocks of 16 per wave (H + D <= 384)
template <int NC>
__device__ __forceinline__ void bptt_wgrad(const PArgs& a, int chain, int w, unsigned* tb_lds, int* flag_lds) {
  if (threadIdx.x >= 256) return;
  const WArgs& q = a.wg;
  // (wave through readfirstlane: the column-block branches below are then scalar, not divergent -- as divergent
  // branches each B load was followed by its own vmcnt(0), ~3.5 us per step instead of ~1.3)
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int H = a.H, L = a.L, B = a.B, nmem = a.nmem, NP = q.NP, nblk = NP / 16;
  const int dir = chain / a.MT, mt = chain % a.MT;
  const PDir& g = a.d[dir];
  const int row0 = 64 * w, gate = row0 / H;
  unsigned long long* ws = q.stamps ? q.stamps + ((long)chain * q.nw + w) * (L + 4) : nullptr;
  auto stamp = [&](int k) {
    if (ws && tid == 0) ws[k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const unsigned tb = launch_tagbase(a.abort_word, tb_lds);
  if (tid < 64) {  // co-location with every member of the chain (their census words)
    const unsigned me = tb | 0x100u | (__builtin_amdgcn_s_getreg(kXccIdHwreg) & 15u);
    bool same = true;
    if (lane < nmem) {
      unsigned spins = 0, v;
      while (((v = __hip_atomic_load(a.census + (long)chain * nmem + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) &
              0xffff0100u) != (tb | 0x100u))
        if (spin_give_up(spins, a.abort_word)) break;
      same = v == me;
    }
    const bool all = __ballot(!same) == 0ull;
    if (lane == 0) *flag_lds = all ? 1 : 0;
  }
  __syncthreads();
  if (!*flag_lds) {
    if (tid == 0) __hip_atomic_store(a.abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  stamp(1);
  const unsigned* prog = a.progress + (long)chain * nmem;
  const long svo = (gate == 2 ? 4L : 3L) * H;
  const int jl = lane & 15, kq = lane >> 4, cb0 = wave * kWgCB;
  // every member's loader at [A] of step p + 3 or later (lanes past nmem read as done)
  // nrdy = steps known final: p < nrdy once every member's loader is past [A] of step p + 3 (the slowest member's
  // progress word v gives v - 2 steps; the final mark L + 3 gives all).  Re-read only when the next step is not
  // among them: a worker behind the chain issues no poll (whose wait would also drain its operand loads)
#ifdef S2S_EXP_WG_NOWAIT  // diagnostic (timing only, wrong results): the workers do not wait for the chain
  int nrdy = L;
#else
  int nrdy = 0;
#endif
  auto refresh = [&]() {
    unsigned v = lane < nmem ? __hip_atomic_load(prog + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : ~0u;
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) v = min(v, (unsigned)__shfl_xor((int)v, o, 64));
    v = (unsigned)__builtin_amdgcn_readfirstlane((int)v);
    const int n = v >= (unsigned)L + 3u ? L : (int)v - 2;
    nrdy = max(nrdy, min(n, L));
  };
  auto ready = [&](int p) -> bool {
    if (p >= nrdy) refresh();
    return p < nrdy;
  };
  auto wait = [&](int p) -> bool {
    unsigned spins = 0;
    while (!ready(p)) {
      if (spin_give_up(spins, a.abort_word)) return false;
      __builtin_amdgcn_s_sleep(4);
    }
    return true;
  };
  // Iteration i = 4 p + kk: processing step p, utterances mt*16 + 4 kk + (0..3) as one K = 4 slice (lane: k = lane >> 4,
  // row / column lane & 15): 4 A values (dA, 64 gate rows) and kWgCB B values (this wave's columns) per lane, then
  // 4 kWgCB MFMAs (~0.3 us).  A ring of kWgRing operand sets keeps kWgRing - 1 iterations of loads in flight behind
  // the products (the loop is unrolled by the ring size, so the code stays a few KB: the instruction cache is shared
  // with a chain member's CU).  Buffer loads with 32-bit offsets; dA sc1 (the chain's rows, L2-resident).
  constexpr int kWgRing = 8;
  const __amdgpu_buffer_rsrc_t ar = rsrc_of(g.dA), sr = rsrc_of(g.sv), xr = rsrc_of(q.x);
  const int ldA = (int)g.ldA, ldx = (int)q.ldx, s5 = 5 * H, svoi = (int)svo;
  float ra[kWgRing][4], rb[kWgRing][kWgCB];
  auto issue = [&](int i, float (&av)[4], float (&bv)[kWgCB]) {
    const int p = i >> 2, kk = i & 3;
    const int t = g.reverse ? p : L - 1 - p;
    const int row = min(mt * 16 + 4 * kk + kq, B - 1) * L + t;
#ifdef S2S_EXP_WG_NOLOAD  // diagnostic (timing only, wrong results): operands from registers
#pragma unroll
    for (int r = 0; r < 4; ++r) av[r] = (float)(row + r);
#pragma unroll
    for (int c = 0; c < kWgCB; ++c) bv[c] = (float)(kk + c);
    return;
#endif
    // no select behind a load (the compiler would wait for the load right there): padding utterances' dA is zeroed
    // where the products use it (mma), x columns past D load column D - 1 into output columns that are not stored
    const int oa = 4 * (row * ldA + row0 + jl);
#pragma unroll
    for (int r = 0; r < 4; ++r) av[r] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(ar, oa + 64 * r, 0, 16));
    const int os = 4 * (row * s5 + svoi + cb0 * 16 + jl), ox = 4 * (row * ldx + cb0 * 16 + jl - H),
              oxl = 4 * (row * ldx + q.D - 1);
#pragma unroll
    for (int c = 0; c < kWgCB; ++c) {  // one unconditional load per column block (branch-free: exact vmcnt waits)
      const int cb = cb0 + c, xc = cb * 16 + jl - H;
      const bool hp = cb * 16 < H;  // (uniform: a block is all h or all x, H % 16 == 0; blocks past nblk load x)
      const __amdgpu_buffer_rsrc_t rs = hp ? sr : xr;
      bv[c] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, hp ? os + 64 * c : (xc < q.D ? ox + 64 * c : oxl), 0, 0));
    }
  };
  floatx4 acc[4][kWgCB];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int c = 0; c < kWgCB; ++c) acc[r][c] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const float (&av)[4], const float (&bv)[kWgCB], int kk) {
    const bool live = mt * 16 + 4 * kk + kq < B;
#ifdef S2S_EXP_WG_NOMMA  // diagnostic (timing only, wrong results): one add per operand instead of the products
#pragma unroll
    for (int c = 0; c < kWgCB; ++c)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r][c][0] += av[r] + bv[c];
    return;
#endif
#pragma unroll
    for (int c = 0; c < kWgCB; ++c)  // (blocks past nblk too, unbranched: their columns are never stored)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(live ? av[r] : 0.f, bv[c], acc[r][c], 0, 0, 0);
  };
  // the steps a group of kWgRing iterations will load are checked final once, in front of the group (the poll's
  // wait would drain the loads in flight anyway), so the unrolled body has no wait and no branch in it (a branch
  // there made the compiler's vmcnt waits assume fewer loads in flight); the last group is peeled
  const int niter = 4 * L;  // a multiple of kWgRing / 2
  auto need = [&](int last_iter) -> bool { return wait(min(last_iter, niter - 1) >> 2); };
  if (!need(kWgRing - 2)) return;
#pragma unroll
  for (int u = 0; u < kWgRing - 1; ++u)
    if (u < niter) issue(u, ra[u], rb[u]);
  int i = 0;
  for (; i + 2 * kWgRing - 2 < niter; i += kWgRing) {
    if (!need(i + 2 * kWgRing - 2)) return;
#pragma unroll
    for (int u = 0; u < kWgRing; ++u) {
      issue(i + u + kWgRing - 1, ra[(u + kWgRing - 1) % kWgRing], rb[(u + kWgRing - 1) % kWgRing]);
      __builtin_amdgcn_sched_barrier(0);  // each iteration's loads stay ahead of the products behind them
      mma(ra[u], rb[u], u & 3);  // (i is a multiple of 4: iteration i + u has kk = u & 3)
      __builtin_amdgcn_sched_barrier(0);
    }
    stamp(2 + (i >> 2));
  }
  for (; i < niter; i += kWgRing) {
    if (!need(niter - 1)) return;
#pragma unroll
    for (int u = 0; u < kWgRing; ++u) {
      const int nx = i + u + kWgRing - 1;
      if (nx < niter) issue(nx, ra[(u + kWgRing - 1) % kWgRing], rb[(u + kWgRing - 1) % kWgRing]);
      if (i + u < niter) mma(ra[u], rb[u], u & 3);
    }
    stamp(2 + (i >> 2));
  }
  stamp(L + 2);
  // D[i][j] of block (r, c) at lane (j = lane & 15, i = 4 (lane >> 4) + e): gate row row0 + 16 r + 4 kq + e
  const int D = q.D;
  const __amdgpu_buffer_rsrc_t pr = rsrc_of(q.part);
  const int tile = 3 * H * NP;  // one utterance tile's partial (per direction: MT tiles)
  const int mine = (dir * a.MT + mt) * tile + row0 * NP + (4 * kq) * NP + cb0 * 16 + jl;
#pragma unroll
  for (int c = 0; c < kWgCB; ++c) {
    if (cb0 + c >= nblk) continue;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc[r][c][e]), pr, 4 * (mine + (16 * r + e) * NP + 16 * c),
                                              0, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0)
    *flag_lds = (int)__hip_atomic_fetch_add(q.ticket + dir * q.nw + w, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*flag_lds != a.MT - 1) return;
  // the last tile to arrive: dW rows [u0, u0 + 64) of (dir, gate) += scale * (sum of the MT partials in tile order)
  const long ldw = (long)H + D;
  float* dW = q.dW[dir][gate];
  const int u0 = row0 - gate * H, first = dir * a.MT * tile + row0 * NP;
  for (int idx = tid; idx < 64 * NP; idx += 256) {
    const int rr = idx / NP, j = idx - rr * NP;
    if (j >= H + D) continue;
    float sum = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, 4 * (first + idx), 0, 16));
    for (int m = 1; m < a.MT; ++m)
      sum += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(pr, 4 * (first + m * tile + idx), 0, 16));
    float* o = dW + (long)(u0 + rr) * ldw + j;
    *o = q.scale * sum + *o;
  }
}

template <int NC>
__global__ __launch_bounds__(kBwdThreads) void gru_bwd_persist(PArgs a) {
  __shared__ SkinnyRed red;
  __shared__ int abort_lds, local_lds;
  __shared__ unsigned tb_lds;
  __shared__ __attribute__((aligned(16))) float rowq[kRowRing][5][256];  // [step % ring][z r hh hp dy][thread]
  extern __shared__ __attribute__((aligned(16))) float ylds[];  // producer tiles (fused dy)
  const int H = a.H, B = a.B, L = a.L;
  const ChainSlot cs = chain_slot(a.nmem);
  const int gch = 8 * ((a.nchains + 7) / 8);
  if ((int)blockIdx.x >= chain_grid(a.nchains, a.nmem)) {
    const int pre = chain_grid(a.nchains, a.nmem) + (a.prefetch ? 8 * a.prefetch_wg : 0);
    if ((int)blockIdx.x < pre) {  // (a.prefetch) chain c's row prefetchers, on its XCD
      const int e = (int)blockIdx.x - chain_grid(a.nchains, a.nmem), c = e & 7, w = e >> 3;
      if (c < a.nchains) bptt_prefetch<NC>(a, c, w, a.prefetch_wg);
      return;
    }
    const int e = (int)blockIdx.x - pre, c = e & 7, w = e >> 3;  // (a.wg.nw) chain c's weight-gradient workers
    if (c < a.nchains) bptt_wgrad<NC>(a, c, w, &tb_lds, &abort_lds);
    return;
  }
  if (cs.chain >= a.nchains) {  // spare slot of the placement grid: dy producer (or idle)
    const int sp = (cs.chain - a.nchains) * a.nmem + cs.member, nsp = (gch - a.nchains) * a.nmem;
    prep_next_sync(a, sp, nsp);
    if (a.fused) xproj_produce_any<true>(a, ylds, sp, nsp);
    return;
  }
  const int dir = cs.chain / a.MT, mt = cs.chain % a.MT;
  const PDir& g = a.d[dir];
  const int ncol = H / 16;
  const int c = cs.member;
  const int lw = dir * a.nwg + mt * ncol + c;  // logical workgroup id (stamps)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b0 = mt * 16;
  if (a.stamps && tid == 0) a.stamps[((long)lw * L + L - 1) * 8 + 6] = __builtin_amdgcn_s_memrealtime();  // entry
  if (tid == 0) abort_lds = 0;
  const unsigned tb = launch_tagbase(a.abort_word, &tb_lds);
  const bool loader = wave == 4;
  const long mytile = (long)mt * 16 * H + (long)c * 256;  // this member's tile in a slot
  if (!loader) {  // this member's 1-KB tile of every (tile-major) slot in use
    const long st = (long)a.MT * 16 * H;
    const int ns = a.ring ? a.ring : L;
    rearm_rect(g.s0 + mytile, st, ns, 16, 0, 16, 0, 16);
    rearm_rect(g.s1 + mytile, st, ns, 16, 0, 16, 0, 16);
    rearm_rect(g.s2 + mytile, st, ns, 16, 0, 16, 0, 16);
  }
  rearm_done();
  const bool loc = chain_is_local(a.census, cs.chain, a.nmem, c, a.allow_local != 0, a.abort_word, &local_lds, tb);
  if (a.stamps && tid == 0) a.stamps[((long)lw * L + L - 1) * 8 + 7] = __builtin_amdgcn_s_memrealtime();  // census done

  if (loader) {
    // lane l: utterance b0 + (l >> 2) of the tile, units c * 16 + 4 (l & 3) .. + 3
    const int bl = b0 + (lane >> 2), u = c * 16 + 4 * (lane & 3);
    const bool lv = bl < B;
    const int lenl = (a.len && lv) ? a.len[bl] : L;
    const __amdgpu_buffer_rsrc_t dyr = rsrc_of(g.dy);
    // fused dy: `yready` slices are known complete; a step past them refreshes all 64 slice counters
    // ahead at once (one round trip), so the poll is rare once the producers are ahead
    int yready = 0;
    auto issue = [&](int q, float4 (&r)[5]) {  // loads of processing step q
#pragma unroll
      for (int v = 0; v < 5; ++v) r[v] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q >= L) return;
      // this step's dy slice must be complete (written through by the producers); polled by all lanes,
      // also those of padding rows or frames, which load no dy
      if (a.fused) xproj_wait(a.xq, dir, q / a.xq.tpt, yready, lane, a.abort_word);
      if (!lv) return;
#ifdef S2S_EXP_NOLOAD  // diagnostic (timing only, wrong results): no HBM row loads in the BPTT loader wave
      return;
#endif
      const int t = g.reverse ? q : L - 1 - q;
      const long row = (long)bl * L + t;
      const float* sv = g.sv + row * 5 * H + u;
#pragma unroll
      for (int v = 0; v < 4; ++v) r[v] = *reinterpret_cast<const float4*>(sv + v * H);
      if (t >= lenl) return;
      if (a.fused) {
        r[4] = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(
                                              dyr, (int)(4 * (row * g.lddy + u)), 0, 16));
      } else {
        r[4] = *reinterpret_cast<const float4*>(g.dy + row * g.lddy + u);
      }
    };
    auto put = [&](int q, const float4 (&r)[5]) {
#pragma unroll
      for (int v = 0; v < 5; ++v) *reinterpret_cast<float4*>(&rowq[q % kRowRing][v][4 * lane]) = r[v];
    };
    float4 ra[5], rb[5];
    issue(0, ra);
    issue(1, rb);
    put(0, ra);
    put(1, rb);
    issue(2, ra);
    __syncthreads();  // [P]
    const bool ring = a.ring && loc;
    unsigned* prog = a.progress ? a.progress + (long)cs.chain * a.nmem + c : nullptr;
    for (int p = 0; p < L; ++p) {
      __syncthreads();  // [A]
      if (abort_lds) return;
      put(p + 2, ra);   // loaded during the previous step
      // (progress for the row prefetchers, which only warm caches, and for the in-launch weight-gradient workers
      // (s2s_debug_bptt_wgrad, off): those treat step p - 2 as final on the recurrence waves' dA stores having been
      // acknowledged by the sweeps' vmcnt waits since -- not a release at agent scope; it would need one (vmcnt(0) in
      // every storing wave before [A], an agent-scope release here) before that path could be turned on)
      if (prog && lane == 0) __hip_atomic_store(prog, (unsigned)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      // The next rows' loads are issued behind [A] and drained before [B] (the vmcnt(0) below): they are then in
      // this CU's memory queue only during the da_r hand-off -- whose consumers run the da_z half of their product
      // meanwhile -- and never beside the da_h sweep behind [B], which gates the step (an HBM load in the queue slows
      // the sweeps behind it: loader loads switched off entirely, backward step 2.78 -> 2.66 us).  Same box, config-2
      // step: 3.268 ms issued behind [B] (round 4), 3.295 issued behind [A] but left in flight across [B], 3.244
      // issued behind [A] and drained.
#ifndef S2S_EXP_LOADB
      issue(p + 3, ra);
#endif
      if (ring && p >= 1) {  // step p-1's slots: every member has finished with them (header comment)
        rearm_tile(g.s0, a, p - 1, mytile, lane);
        rearm_tile(g.s1, a, p - 1, mytile, lane);
        rearm_tile(g.s2, a, p - 1, mytile, lane);
      }
      // the re-arms land before the member publishes step p+1 (and the row loads before [B])
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // [B]
      if (abort_lds) return;
#ifdef S2S_EXP_LOADB  // A/B: the round-4 placement behind [B]
      issue(p + 3, ra);
#endif
    }
    if (a.wg.nw) {  // the weight-gradient workers' final mark: every dA store of this member has landed ([C])
      __syncthreads();  // [C]
      if (lane == 0) __hip_atomic_store(prog, (unsigned)L + 3u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }

  float4 wh[NC], wzr[2 * NC];
  load_wfrag(wh, g.Wa + (long)(c * 16 + (lane & 15)) * H, wave, lane);
  load_wfrag(wzr, g.Wb + (long)(c * 16 + (lane & 15)) * 2 * H, wave, lane);
  const __amdgpu_buffer_rsrc_t zg = rsrc_of(g.g0), rg = rsrc_of(g.g1), hg = rsrc_of(g.g2);
  const __amdgpu_buffer_rsrc_t zs = rsrc_of(g.s0), rs_ = rsrc_of(g.s1), hs = rsrc_of(g.s2);
  const long slot = (long)B * H;
  const int br = min(b0 + (lane & 15), B - 1);
  const long slotS = (long)a.MT * 16 * H, tileS = (long)mt * 16 * H;  // tile-major sentinel slot, this row tile
  const int rowt = br - b0;
  const int ob = b0 + (tid >> 4), ok_ = c * 16 + (tid & 15);
  const bool live = ob < B;
  const int lenb = (a.len && live) ? a.len[ob] : L;  // masked frames: dL/dh_t = 0 (forward h_t = 0)
  float dhc = 0.f, dhp = 0.f;
  bool aborted = false;

  // saved activations and dy of one step for this thread's (utterance, unit), from the loader's ring
  struct Row {
    float z, r, hh, hp, dy;
  };
  auto load_row = [&](int q) {
    const float(*r)[256] = rowq[q % kRowRing];
    return Row{r[0][tid], r[1][tid], r[2][tid], r[3][tid], r[4][tid]};
  };
  // gate gradients of dh = dy_t + carry at time t (rows that are live), published as hand-off
  // step pn (tag tb + pn + 1, slot pn & 1; sentinel slot pn) when `pub`; every lane calls it
  auto gate = [&](int t, const Row& v, float dh, int pn, bool pub) {
    const long row = (long)ob * L + t;
    const float daz = dh * (v.hh - v.hp) * (v.z * (1.0f - v.z));
    const float dah = (dh * v.z) * (1.0f - v.hh * v.hh);
    if (loc) {
      const long off = sent_slot(a, pn) * slotS + tile_off(ob, ok_, H);
      if (pub) {
        put_sent(g.s2 + off, dah);  // da_h gates the next p1: first
        put_sent(g.s0 + off, daz);
      }
    } else {
      const long off = (pn & 1) * slot + (long)ob * H + ok_;
      put_granule_pair(g.g2, off, dah, tb + pn + 1, pub);
      put_granule_pair(g.g0, off, daz, tb + pn + 1, pub);
    }
#ifndef S2S_EXP_NODA  // diagnostic (timing only): no dA stores
    if (pub) {
      g.dA[row * g.ldA + ok_] = daz;
      g.dA[row * g.ldA + 2 * H + ok_] = dah;
    }
#endif
  };

  const int tl = g.reverse ? 0 : L - 1;
  __syncthreads();  // [P]
  Row cur = load_row(0);
  gate(tl, cur, cur.dy, 0, live);

  for (int p = 0; p < L; ++p) {
    const int s = L - 1 - p;
    const int t = g.reverse ? L - 1 - s : s;
    const long row = (long)ob * L + t;
    const unsigned tag = tb + p + 1;
    const int sl = p & 1;
    // ---- p1: dq = Uh^T da_h -> da_r, partial dh_{t-1}
    float4 av[NC];
    GRU_STAMP(0);
#if S2S_GRU_DIAG
    unsigned npoll[3] = {0, 0, 0};
#endif
    bool ok;
    floatx4 acc;
    // da_z of this step (published with da_h, at the end of the previous step's p2) is loaded here, behind the da_h
    // sweep, so p2 starts with it in registers instead of with a sweep of its own (checked there; polled further
    // only if some value was not yet published)
    uint4 zraw[NC];
    bool zpre = false;
#if !S2S_GRU_DIAG
    if (loc && a.stream_sweep) {
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      ok = sweep_sent_mfma<NC>(av, hs, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane, wh, acc0, acc1,
                               a.abort_word);
      GRU_STAMP(1);  // (the last chunk arrived and its MFMAs are issued)
      if constexpr (NC % 2 == 0) {
        sent_tile_issue<NC>(zraw, zs, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane);
        zpre = true;
      }
      acc = acc0 + acc1;
    } else
#endif
    {
    ok = loc ? SWEEP_SENT(0, av, hs, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane, a.abort_word)
             : sweep_skinny<NC>(av, hg, 8 * (sl * slot + (long)br * H), tag, wave, lane, a.abort_word);
    GRU_STAMP(1);
#if S2S_GRU_DIAG
    GRU_STAMP_V(8, npoll[0]);
#endif
    acc = mfma_chunks<NC>(av, wh);
    }
    const float dq = reduce_or_abort(red, &abort_lds, ok, acc, wave, lane, tid, &aborted);
    if (loc) {
      if (live) put_sent(g.s1 + sent_slot(a, p) * slotS + tile_off(ob, ok_, H), (dq * cur.hp) * (cur.r * (1.0f - cur.r)));
    } else {
      put_granule_pair(g.g1, sl * slot + (long)ob * H + ok_, (dq * cur.hp) * (cur.r * (1.0f - cur.r)), tag, live);
    }
    if (live) {
      const float dar = (dq * cur.hp) * (cur.r * (1.0f - cur.r));
#ifndef S2S_EXP_NODA
      g.dA[row * g.ldA + H + ok_] = dar;
#endif
      const float dh = cur.dy + dhc;
      dhp = dh * (-cur.z + 1.0f) + dq * cur.r;
    }
    GRU_STAMP(2);
    if (aborted) return;  // checked after the epilogue: its LDS read is issued with the reduce's reads
    // ---- p2: dh_{t-1} = dhp + Uzr^T [da_z; da_r]; gate gradients of step t-1
    const int tn = g.reverse ? t + 1 : t - 1;
    float4 azr[2 * NC];
    GRU_STAMP(3);
    bool split = false;
    if constexpr (NC % 2 == 0 && !S2S_GRU_DIAG) split = loc;
    if constexpr (NC % 2 == 0 && !S2S_GRU_DIAG) if (split) {
      // da_z (ready since the previous step) first; da_r (this step's p1) is loaded once before the da_z half of
      // the K = 2H product runs, checked behind it (polled further only if some tile was not yet published): the
      // da_z MFMAs overlap the da_r hand-off.  Same instruction sequence as mfma_chunks<2 NC> (bitwise equal).
      float4 az[NC], ar[NC];
      uint4 rraw[NC];
      ok = true;
      if (!zpre || !sent_tile_check<NC>(zraw, az))
        ok = sweep_sent_tile<NC>(az, zs, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane, a.abort_word);
      sent_tile_issue<NC>(rraw, rs_, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane);
      floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
      __builtin_amdgcn_sched_barrier(0);  // the da_r loads stay ahead of the da_z MFMAs
      mfma_pairs<NC>(az, wzr, acc0, acc1);
      __builtin_amdgcn_sched_barrier(0);
      // (checked whole: multiplying the da_r chunks as they arrive, sent_tile_mfma, measured 1305 -> 1355 us per
      // config-2 step)
      if (!sent_tile_check<NC>(rraw, ar))
        ok = ok && sweep_sent_tile<NC>(ar, rs_, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane, a.abort_word);
      GRU_STAMP(4);
      mfma_pairs<NC>(ar, wzr + NC, acc0, acc1);
      acc = acc0 + acc1;
    }
    if (!split) {
      // da_z (ready since the previous step) first, then poll da_r (this step's p1) alone: a
      // merged poll of both rows re-reads da_z while waiting for da_r (measured slower)
      float4 az[NC], ar[NC];
      if (loc) {
        ok = SWEEP_SENT(1, az, zs, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane, a.abort_word);
#if S2S_GRU_DIAG
        GRU_STAMP(10);  // the da_z sweep (published a whole phase earlier) is done
#endif
        ok = ok && SWEEP_SENT(2, ar, rs_, 4 * (sent_slot(a, p) * slotS + tileS), rowt, wave, lane, a.abort_word);
#if S2S_GRU_DIAG
        GRU_STAMP_V(9, npoll[1]);
        GRU_STAMP_V(11, npoll[2]);
#endif
      } else {
        ok = sweep_skinny<NC>(az, zg, 8 * (sl * slot + (long)br * H), tag, wave, lane, a.abort_word);
        ok = ok && sweep_skinny<NC>(ar, rg, 8 * (sl * slot + (long)br * H), tag, wave, lane, a.abort_word);
      }
      GRU_STAMP(4);
      // chunk i of the K = 2H product: i < NC reads da_z, i >= NC reads da_r (H % 64 == 0)
#pragma unroll
      for (int i = 0; i < NC; ++i) { azr[i] = az[i]; azr[NC + i] = ar[i]; }
      acc = mfma_chunks<2 * NC>(azr, wzr);
    }
    const float sm = reduce_or_abort(red, &abort_lds, ok, acc, wave, lane, tid, &aborted);
    const Row nxt = s > 0 ? load_row(p + 1) : Row{0.f, 0.f, 0.f, 0.f, 0.f};
    if (live && s > 0) dhc = tn < lenb ? dhp + sm : 0.f;
    if (s > 0) gate(tn, nxt, nxt.dy + dhc, p + 1, live);
    cur = nxt;
    GRU_STAMP(5);
    if (aborted) return;  // checked after the epilogue: its LDS read is issued with the reduce's reads
  }
  if (a.wg.nw) {  // [C]: the loader's final mark for the weight-gradient workers follows this wave's last dA stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
}

// Exclusive-CU mode (set while weight-gradient GEMMs run on a side stream beside the recurrence):
// each persistent workgroup reserves kExclLds bytes of dynamic LDS it never touches, so no GEMM
// workgroup (37 KB of LDS) can share its CU; the GEMMs fill the CUs the recurrence leaves idle.
constexpr int kExclLds = 124 * 1024;

// Prefetcher workgroups per chain (s2s_debug_bptt_prefetch(wg, lookahead) for A/Bs).  Same box, config-2 step (three alternating runs each,
// profiles/r05/ab_bptt_prefetch.txt): none 3.248 ms, 1 per chain 3.250 (one workgroup cannot keep 8 steps of rows
// in flight), 2 per chain 3.182, 4 per chain 3.184, 16 (one per member) 3.463 (the side stream's weight-gradient
// GEMMs lose the chain XCDs' idle CUs); the lower layers' BPTT step 3.05 -> 2.68 us (tools/gru_stamps.py, 2 layers)
std::atomic<int> g_bptt_prefetch_wg{2};
// lookahead (steps) of the BPTT row prefetchers (bptt_prefetch), 0 = off (4 / 8 / 12 measured alike; 8)
std::atomic<int> g_bptt_prefetch{8};
// prefetcher workgroups per chain of a BPTT launch of this shape (0: none)
int bptt_prefetch_wg(int ndir, int B, int H) {
  const int nch = ndir * ((B + 15) / 16), nm = H / 16;
  const int nwg = std::max(1, std::min((int)g_bptt_prefetch_wg, nm));
  return g_bptt_prefetch > 0 && nch <= 8 && nm + nwg <= 32 && nm % nwg == 0 ? nwg : 0;
}
std::atomic<int> g_allow_local{1};
std::atomic<int> g_sent_ring{kSentRing};  // s2s_debug_gru_ring(0): one sentinel slot per step (A/B)
std::atomic<int> g_stream_sweep{1};  // s2s_debug_gru_stream_sweep(0): sweep the whole tile, then multiply (A/B)

template <int NC>
int launch_nc(hipStream_t st, const PArgs& a, bool excl_req, bool fwd) {
  // (the BPTT's row prefetchers: 8 prefetch_wg more workgroups, chain c's at chain_grid + 8 w + c, on its XCD)
  // and the in-launch weight-gradient workers: 8 nw more, chain c's worker w at the prefetchers' end + 8 w + c)
  const dim3 grid(chain_grid(a.nchains, a.nmem) + (!fwd && a.prefetch ? 8 * a.prefetch_wg : 0) +
                  (!fwd ? 8 * a.wg.nw : 0));
  // exclusive only while one chain per XCD fits one workgroup per CU (32 CUs per XCD)
  const bool excl = excl_req && a.nchains <= 8 && a.nmem <= 32;
  const unsigned shm = excl ? kExclLds : (a.fused ? kXpLds : 0);
  if (fwd) {
    if (excl) S2S_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gru_fwd_persist<NC>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, kExclLds));
    S2S_TRY(check_resident(reinterpret_cast<const void*>(gru_fwd_persist<NC>), grid.x, kFwdThreads, shm,
                           "gru_fwd_persist"));
    hipLaunchKernelGGL(gru_fwd_persist<NC>, grid, dim3(kFwdThreads), shm, st, a);
  } else {
    if (excl) S2S_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(gru_bwd_persist<NC>),
                                                hipFuncAttributeMaxDynamicSharedMemorySize, kExclLds));
    S2S_TRY(check_resident(reinterpret_cast<const void*>(gru_bwd_persist<NC>), grid.x, kBwdThreads, shm,
                           "gru_bwd_persist"));
    hipLaunchKernelGGL(gru_bwd_persist<NC>, grid, dim3(kBwdThreads), shm, st, a);
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int launch(hipStream_t st, const PArgs& a, bool excl, bool fwd) {
  switch (a.H / 64) {
    case 1: return launch_nc<1>(st, a, excl, fwd);
    case 2: return launch_nc<2>(st, a, excl, fwd);
    case 4: return launch_nc<4>(st, a, excl, fwd);
    case 8: return launch_nc<8>(st, a, excl, fwd);
  }
  set_error("gru persistent: unsupported H");
  return 2;
}

}  // namespace

std::atomic<int> g_fuse_xproj{1};  // S2S_GRU_FUSED_XPROJ=0 (diagnostic) keeps the separate x-projection GEMM

bool gru_persist_fused_xproj(int ndir, int B, int H, int Kx) {
  if (!g_fuse_xproj || B > 64 || Kx % 32 != 0 || H % 64 != 0) return false;
  const int MT = (B + 15) / 16, nchains = ndir * MT, nmem = 2 * H / 16;
  return chain_grid(nchains, nmem) - nchains * nmem >= 32;  // spare slots to produce on
}

std::atomic<int> g_xp_split{1};  // s2s_debug_gru_xp_split(0) (diagnostic): no split-K start of the fused dy producers
std::atomic<int> g_fuse_dy{1};  // s2s_debug_gru_fused_dy(0) (diagnostic): the dX GEMM in front of the BPTT instead

bool gru_persist_fused_dy(int ndir, int B, int H, int K, long ldw, long lddy) {
  if (!g_fuse_xproj || !g_fuse_dy || B > 64 || K % 32 != 0 || H % 64 != 0 || ldw % 4 != 0 || lddy < (long)ndir * H) return false;
  const int MT = (B + 15) / 16, nchains = ndir * MT, nmem = H / 16;
  return chain_grid(nchains, nmem) - nchains * nmem >= 32;  // spare slots to produce on
}

bool gru_persist_wgrad_fits(int ndir, int B, int H, int D) {
  const int nch = ndir * ((B + 15) / 16), nm = H / 16, nw = 3 * H / 64;
  // one chain per XCD, its members, prefetchers and workers one per CU; a worker wave's columns fit kWgCB blocks
  return H % 64 == 0 && D > 0 && nch <= 8 && nm + bptt_prefetch_wg(ndir, B, H) + nw <= 32 &&
         H + (D + 15) / 16 * 16 <= 4 * kWgCB * 16;
}

bool gru_persist_supported(int ndir, int B, int H) {
  if (!(H == 64 || H == 128 || H == 256 || H == 512)) return false;
  const int MT = (B + 15) / 16;
  // the chains placed on one XCD must be co-resident there (32 CUs, >= 2 workgroups per CU at
  // this footprint): forward members 2H/16 per chain, chains (dir, tile) dealt 8 per round
  return (2 * H / 16) * ((ndir * MT + 7) / 8) <= 64;
}

static size_t census_bytes(int B, int H) { return 4 * (size_t)(2 * ((B + 15) / 16)) * (2 * H / 16); }

// header | tagged granules | census | x-projection counters (zeroed by sync_prep every launch) |
// sentinel rows (re-armed in-kernel)
// slice counters [2][L] and split-item counters [kXpMaxSplitItems]
static size_t xcount_words(int L) { return 2 * (size_t)L + kXpMaxSplitItems; }
// header | granules | census | slice / item counters | prefetch progress words (as many as census words)
static size_t prep_bytes(int B, int L, int H) {
  return 256 + 2 * 3 * 2 * sizeof(unsigned long long) * (size_t)B * H + census_bytes(B, H) + 4 * xcount_words(L) +
         census_bytes(B, H);
}
static size_t sent_offset(int B, int L, int H) { return (prep_bytes(B, L, H) + 255) / 256 * 256; }
// sentinel rows are tile-major: 16 rows per row tile (handoff.h tile_off)
static size_t sent_rows(int B) { return (size_t)(B + 15) / 16 * 16; }
static size_t slab_offset(int B, int L, int H) {
  return sent_offset(B, L, H) + 2 * 3 * sizeof(float) * (size_t)L * sent_rows(B) * H;
}
constexpr size_t kXpSlabBytes = (size_t)kXpMaxSplitItems * 4 * 4096 * sizeof(float);  // PA <= 4

size_t gru_persist_sync_bytes(int B, int L, int H) { return slab_offset(B, L, H) + kXpSlabBytes; }
size_t gru_persist_prep_bytes(int B, int L, int H) { return prep_bytes(B, L, H); }
bool gru_persist_can_prep_next(int ndir, int B, int H, bool fwd) {
  const int MT = (B + 15) / 16, nchains = ndir * MT, nmem = fwd ? 2 * H / 16 : H / 16;
  return chain_grid(nchains, nmem) > nchains * nmem;  // spare slots exist
}

// split-K start of a fused producer grid (XProj::sA ..): the first round of units is the first slices cut
// into 4 K-parts, the second the next slices into 2, so the recurrence's first slices come after a quarter
// / half of a tile's K loop; only when every part keeps the 4-deep ring (nk / 4 % 4 == 0)
static void xproj_split(XProj& q, int nd, int nprod) {
  q.sA = q.sB = 0;
  q.PA = q.PB = 1;
  q.nsplit = 0;
  const int nk = q.K / 32, per = nd * q.ntn;
  if (!g_xp_split || nk % 16 != 0 || per <= 0) return;
  const int sA = std::max(1, nprod / (per * 4));
  const int sB = std::min(q.nslices, sA + std::max(1, nprod / (per * 2)));
  if (sB > q.nslices || sB * per > kXpMaxSplitItems || sA >= sB) return;
  q.sA = sA; q.sB = sB; q.PA = 4; q.PB = 2;
  q.nwork = (sA * 4 + (sB - sA) * 2 + (q.nslices - sB)) * per;
  q.nsplit = (sA * 4 + (sB - sA) * 2) * per;
}

// XCD-grouped dealing of the dy units (s2s_debug_gru_xp_group; on by default since round 5): at
// config 2 the BPTT launch moves 214 -> 144 MB (the producers' x-weights stay in their XCD's L2), at config 4
// 1,089 -> 806 MB.  Round 4 measured the step ~20 us slower with it; round 5 (sleepless polls, the loader's
// rows drained before [B]) measures no difference: 3.2295 vs 3.2305 ms over three alternating runs each, same box
// (profiles/r05/ab_xp_group.txt)
std::atomic<int> g_xp_group{1};

// XCD-grouped dealing (XProj::G) when the spare slots form whole per-XCD groups of gsz producers and every
// direction gets at least one group
static void xproj_group(XProj& q, int nd, int nprod, int gsz) {
  q.G = 0;
  q.gsz = gsz;
  if (!g_xp_group || gsz <= 0 || nprod % gsz != 0) return;
  const int G = nprod / gsz;
  if (G < nd || G % nd != 0) return;
  q.G = G;
}

static void carve_granules(char* sync, int B, int L, int H, unsigned** abort_word, granule_t* (&g)[2][3],
                           float* (&sv)[2][3], unsigned** census, unsigned** xcount = nullptr) {
  *abort_word = reinterpret_cast<unsigned*>(sync);
  granule_t* p = reinterpret_cast<granule_t*>(sync + 256);
  for (int d = 0; d < 2; ++d)
    for (int k = 0; k < 3; ++k) {
      g[d][k] = p;
      p += 2L * B * H;
    }
  *census = reinterpret_cast<unsigned*>(p);
  if (xcount) *xcount = *census + census_bytes(B, H) / 4;
  float* q = reinterpret_cast<float*>(sync + sent_offset(B, L, H));
  for (int d = 0; d < 2; ++d)
    for (int k = 0; k < 3; ++k) {
      sv[d][k] = q;
      q += (long)L * sent_rows(B) * H;
    }
}

int gru_persist_fwd(hipStream_t st, const GruPersistFwd& f, void* sync) {
  PArgs a{};
  const int MT = (f.B + 15) / 16;
  granule_t* gr[2][3];
  float* sr[2][3];
  unsigned* xcount = nullptr;
  carve_granules(static_cast<char*>(sync), f.B, f.L, f.H, &a.abort_word, gr, sr, &a.census, &xcount);
  for (int d = 0; d < f.ndir; ++d)
    a.d[d] = PDir{f.xp[d], f.ldxp, f.Uzr[d], f.Uh[d], f.y[d], f.ldy, f.sv[d], nullptr, 0, nullptr, 0, f.reverse[d],
                  gr[d][0], gr[d][1], gr[d][2], sr[d][0], sr[d][1], sr[d][2]};
  a.len = f.len;
  a.B = f.B; a.L = f.L; a.H = f.H; a.MT = MT; a.nwg = (2 * f.H / 16) * MT;
  a.nmem = 2 * f.H / 16; a.nchains = f.ndir * MT; a.allow_local = g_allow_local;
  a.ring = f.L > kSentRing ? (int)g_sent_ring : 0;
  a.stream_sweep = g_stream_sweep;
  a.stamps = g_gru_stamps[0];
  a.pstamps = g_gru_pstamps[0];
  if (f.x) {  // fused x-projection by the grid's spare slots
    XProj& q = a.xq;
    q.x = f.x; q.ldx = f.ldx; q.K = f.Kx; q.W = f.Wx; q.ldw = f.Kx; q.ncd = 3 * f.H; q.flip = 0;
    q.xp = const_cast<float*>(f.xp[0]); q.ldxp = f.ldxp;
    q.tpt = 64 / f.B;
    q.nslices = (f.L + q.tpt - 1) / q.tpt;
    q.ntn = 3 * f.H / 64;
    q.nd = f.ndir;
    q.nwork = q.nslices * f.ndir * q.ntn;
    q.done = xcount;
    q.sA = q.sB = 0; q.PA = q.PB = 1;
    a.fused = 1;
  }
  if (f.next_sync) {
    a.next_sync = static_cast<char*>(f.next_sync);
    a.next_prep = f.next_prep;
  }
  if (f.pack) a.pack = *f.pack;
  if (!f.prepared) S2S_TRY(launch_sync_prep(st, sync, prep_bytes(f.B, f.L, f.H), a.next_sync));
  // algorithmic work of the launch: the recurrence, plus the x-projection GEMM when its spare slots compute it
  // bytes: the recurrence's weights, x-projection reads, saved activations and outputs, plus the in-launch GEMM's
  // operands and its x-projection writes (x once for both directions, Wx, xp)
  const double xflops = f.x ? 2.0 * f.B * f.L * 3.0 * f.ndir * f.H * f.Kx : 0.0;
  const double xbytes = f.x ? 4.0 * ((double)f.B * f.L * f.Kx + 3.0 * f.ndir * f.H * f.Kx + 3.0 * f.ndir * f.B * f.L * f.H)
                            : 0.0;
  ProfScope ps(st, "gru_fwd_persist", 2.0 * f.ndir * f.B * f.L * 3.0 * f.H * f.H + xflops,
               4.0 * f.ndir * (3.0 * f.H * f.H + (double)f.B * f.L * (3 * f.H + 5 * f.H + f.H)) + xbytes);
  S2S_TRY(launch(st, a, f.excl != 0, true));
  void* r[1] = {sync};
  return launch_sync_harvest(st, r, 1, f.status);
}

int gru_persist_bwd(hipStream_t st, const GruPersistBwd& b, void* sync) {
  PArgs a{};
  const int MT = (b.B + 15) / 16;
  granule_t* gr[2][3];
  float* sr[2][3];
  unsigned* xcount = nullptr;
  carve_granules(static_cast<char*>(sync), b.B, b.L, b.H, &a.abort_word, gr, sr, &a.census, &xcount);
  // row prefetchers: one workgroup per chain on an idle CU of its XCD (the chain's members leave at least one)
  {
    const int nwg = bptt_prefetch_wg(b.ndir, b.B, b.H);
    if (nwg) {
      a.prefetch = g_bptt_prefetch;
      a.prefetch_wg = nwg;
      a.progress = xcount + xcount_words(b.L);
    }
  }
  if (b.wgrad) {  // in-launch weight gradients (bptt_wgrad)
    S2S_REQUIRE(gru_persist_wgrad_fits(b.ndir, b.B, b.H, b.wD) && b.wx && b.wpart,
                "gru persistent bwd: in-launch weight gradients do not fit this shape");
    WArgs& q = a.wg;
    q.nw = 3 * b.H / 64;
    for (int d = 0; d < 2; ++d)
      for (int g = 0; g < 3; ++g) q.dW[d][g] = b.wdW[d][g];
    q.scale = b.wscale;
    q.x = b.wx; q.ldx = b.wldx; q.D = b.wD; q.NP = b.H + (b.wD + 15) / 16 * 16;
    q.part = b.wpart;
    q.stamps = g_gru_wstamps;
    a.progress = xcount + xcount_words(b.L);
    q.ticket = a.progress + (long)b.ndir * MT * (b.H / 16);  // past the progress words (census-sized region)
  }
  for (int d = 0; d < b.ndir; ++d)
    a.d[d] = PDir{nullptr, 0, b.UhT[d], b.UzrT[d], nullptr, 0, b.sv[d], b.dy[d], b.lddy, b.dA[d], b.ldA,
                  b.reverse[d], gr[d][0], gr[d][1], gr[d][2], sr[d][0], sr[d][1], sr[d][2]};
  a.len = b.len;
  a.B = b.B; a.L = b.L; a.H = b.H; a.MT = MT; a.nwg = (b.H / 16) * MT;
  a.nmem = b.H / 16; a.nchains = b.ndir * MT; a.allow_local = g_allow_local;
  a.ring = b.L > kSentRing ? (int)g_sent_ring : 0;
  a.stream_sweep = g_stream_sweep;
  a.stamps = g_gru_stamps[1];
  a.pstamps = g_gru_pstamps[1];
  if (b.ydA) {  // fused dy (the layer above's dX) by the grid's spare slots
    XProj& q = a.xq;
    q.x = b.ydA; q.ldx = b.yldA; q.K = b.yK; q.W = b.yWx; q.ldw = b.yldw; q.ncd = b.H; q.flip = 1;
    q.xp = const_cast<float*>(b.dy[0]); q.ldxp = b.lddy;
    q.tpt = 64 / b.B;
    q.nslices = (b.L + q.tpt - 1) / q.tpt;
    q.ntn = b.H / 64;
    q.nd = b.ndir;
    q.nwork = q.nslices * b.ndir * q.ntn;
    q.done = xcount;
    q.alpha = b.yalpha; q.dc = b.ydc; q.T = b.yT;
    q.icnt = xcount + 2 * b.L;
    q.slab = reinterpret_cast<float*>(static_cast<char*>(sync) + slab_offset(b.B, b.L, b.H));
    const int gch = 8 * ((a.nchains + 7) / 8);
    xproj_split(q, b.ndir, (gch - a.nchains) * a.nmem);
    xproj_group(q, b.ndir, (gch - a.nchains) * a.nmem, a.nmem);
    a.fused = 1;
  }
  if (b.next_sync) {
    a.next_sync = static_cast<char*>(b.next_sync);
    a.next_prep = b.next_prep;
  }
  if (!b.prepared) S2S_TRY(launch_sync_prep(st, sync, prep_bytes(b.B, b.L, b.H), a.next_sync));
  if (b.prep_event) S2S_CHECK_HIP(hipEventRecord(b.prep_event, st));
  // algorithmic work of the launch: the recurrence, plus the dy its spare slots compute (the layer above's
  // dX GEMM, or the decoder's dh: dVh V and the context term sum_t alpha dc)
  // bytes: the recurrence's weights, saved activations, dy reads and gate-gradient writes, plus the in-launch GEMM's
  // operands (dA of the layer above or the decoder's dVh, the weights, the context term's alpha and dc) and its dy
  // writes
  const double yflops = b.ydA ? 2.0 * b.B * b.L * (double)b.ndir * b.H * (b.yK + b.yT) : 0.0;
  const double ybytes = b.ydA ? 4.0 * ((double)b.B * b.L * b.yK + (double)b.yK * b.ndir * b.H +
                                       (double)b.B * b.yT * (b.L + b.ndir * b.H) + (double)b.B * b.L * b.ndir * b.H)
                              : 0.0;
  // (+ the in-launch weight gradients: dA, the h / q rows and x read once more, dW read and written)
  const double wflops = b.wgrad ? 2.0 * b.ndir * b.B * b.L * 3.0 * b.H * (b.H + b.wD) : 0.0;
  const double wbytes = b.wgrad ? 4.0 * ((double)b.B * b.L * (b.ndir * 3.0 * b.H + b.ndir * 2.0 * b.H + b.wD) +
                                         2.0 * b.ndir * 3.0 * b.H * (b.H + b.wD))
                                : 0.0;
  ProfScope ps(st, "gru_bwd_persist", 2.0 * b.ndir * b.B * b.L * 3.0 * b.H * b.H + yflops + wflops,
               4.0 * b.ndir * (3.0 * b.H * b.H + (double)b.B * b.L * (5 * b.H + b.H + 3 * b.H)) + ybytes + wbytes);
  S2S_TRY(launch(st, a, b.excl != 0, false));
  void* r[1] = {sync};
  return launch_sync_harvest(st, r, 1, b.status);
}

// Test probe of the timeout path (s2s_debug_handoff_timeout): one wave waits for a granule nobody writes,
// in a region prepared by sync_prep, with a short spin limit -- it must give up and raise the abort word,
// which the harvest behind it reports as S2S_STATUS_HANDOFF_TIMEOUT, exactly as for a stalled launch.
__global__ __launch_bounds__(64) void handoff_timeout_probe(char* sync) {
  unsigned* hdr = reinterpret_cast<unsigned*>(sync);
  const granule_t* g = reinterpret_cast<const granule_t*>(sync + 256);
  unsigned spins = 0;
  while (true) {
    const granule_t x = __hip_atomic_load(g + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__all((unsigned)(x >> 32) == 0xfffffffeu)) break;  // never: the region is zeroed
    if (spin_give_up(spins, hdr, 4096u)) break;
  }
}
int handoff_timeout_probe_launch(hipStream_t st, void* sync, unsigned* status) {
  S2S_TRY(launch_sync_prep(st, sync, 256 + 64 * sizeof(granule_t)));
  hipLaunchKernelGGL(handoff_timeout_probe, dim3(1), dim3(64), 0, st, static_cast<char*>(sync));
  S2S_CHECK_HIP(hipGetLastError());
  void* r[1] = {sync};
  return launch_sync_harvest(st, r, 1, status);
}

// The model step's head (gru_step_head): one grid-stride pass over the layer-1 input padding, the pack jobs and
// the first persistent launch's sync-region preparation (sync_prep's work, in this translation unit so the epoch
// comes from the same counter as every other GRU region's)
__global__ __launch_bounds__(256) void step_head_kernel(GruStepHead h, unsigned abort0) {
  const long gid = blockIdx.x * 256L + threadIdx.x, gsz = (long)gridDim.x * 256;
  if (h.sync && gid == 0) {
    if (h.clear) {
      unsigned* c = reinterpret_cast<unsigned*>(h.clear);
      __hip_atomic_exchange(c + kStickyWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned* hdr = reinterpret_cast<unsigned*>(h.sync);
    const unsigned e = __hip_atomic_fetch_add(&g_s2s_epoch_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_exchange(hdr + kEpochWord, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(hdr + kStickyWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(hdr, abort0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (h.sync) {
    const size_t body = h.prep_bytes - 256, n16 = body / 16;
    uint4* p = reinterpret_cast<uint4*>(h.sync + 256);
    for (long i = gid; i < (long)n16; i += gsz) p[i] = make_uint4(0u, 0u, 0u, 0u);
    unsigned* t = reinterpret_cast<unsigned*>(h.sync + 256 + n16 * 16);
    for (long i = gid; i < (long)((body % 16) / 4); i += gsz) t[i] = 0u;
  }
  const long n = (long)h.rows * h.dcols;
  for (long i = gid; i < n; i += gsz) {
    const long r = i / h.dcols, c = i - r * h.dcols;
    h.dst[i] = c < h.cols ? h.src[r * h.lds + c] : 0.f;
  }
  for (int j = 0; j < h.pack.n; ++j) gru_pack_elems(h.pack.j[j], gid, gsz);
  if (h.dlogp) {
    const long nd = (long)h.B * h.T * h.O;
    for (long i = gid; i < nd; i += gsz) {
      const long bt = i / h.O;
      const int o = (int)(i - bt * h.O), b = (int)(bt / h.T), t = (int)(bt - (long)b * h.T);
      const bool hit = t < (h.tlen ? h.tlen[b] : h.T) && h.labels[bt] == o;
      h.dlogp[i] = hit ? -1.f : 0.f;
    }
  }
  uint4* z = static_cast<uint4*>(h.zero);
  for (long i = gid; i < (long)h.zero_n4; i += gsz) z[i] = make_uint4(0u, 0u, 0u, 0u);
  if (gid < h.zero_tail) reinterpret_cast<float*>(z + h.zero_n4)[gid] = 0.f;
}
int gru_persist_step_head(hipStream_t st, const GruStepHead& h) {
  long most = (long)h.rows * h.dcols;
  for (int j = 0; j < h.pack.n; ++j) most = std::max(most, 3L * h.pack.j[j].H * (h.pack.j[j].H + h.pack.j[j].Kx));
  if (h.sync) most = std::max<long>(most, (long)((h.prep_bytes - 256) / 16));
  most = std::max<long>(most, std::max<long>((long)h.B * h.T * h.O, (long)h.zero_n4));
  const int blocks = (int)std::max<long>(1, std::min<long>(1024, (most + 255) / 256));
  hipLaunchKernelGGL(step_head_kernel, dim3(blocks), dim3(256), 0, st, h, inject_abort_take() ? 2u : 0u);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// Test stand-in for a collective beside the persistent launches (RCCL's all-reduce kernels run on a
// communication stream while the encoder BPTT runs): nwg workgroups that each hold lds_bytes of dynamic LDS and stay
// resident for `ticks` of the 100 MHz real-time clock, touching their LDS and sleeping -- a bounded kernel, so
// whatever the dispatcher does with the persistent launch behind it, every workgroup eventually runs.
__global__ __launch_bounds__(256) void lds_hog_kernel(float* out, int n, unsigned long long ticks) {
  extern __shared__ float hog[];
  for (int i = threadIdx.x; i < n; i += 256) hog[i] = (float)i;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  float acc = 0.f;
  int k = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) {
    k = (k * 7 + 13) % n;
    acc += hog[k];
    __builtin_amdgcn_s_sleep(8);
  }
  if (acc == -1.f) out[blockIdx.x] = acc;  // never: keeps the loop
}
int lds_hog_launch(hipStream_t st, int nwg, int lds_bytes, double usec, float* out) {
  S2S_REQUIRE(nwg > 0 && nwg <= 4096 && lds_bytes >= 1024 && lds_bytes <= 160 * 1024 && usec > 0 && usec < 1e6,
              "lds hog: bad arguments");
  S2S_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(lds_hog_kernel),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  hipLaunchKernelGGL(lds_hog_kernel, dim3(nwg), dim3(256), lds_bytes, st, out, lds_bytes / 4,
                     (unsigned long long)(usec * 100.0));
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// Diagnostic clock probe (tools/clock_probe.py): nwg single-lane workgroups (workgroup w on XCD w % 8) that record
// (real-time 100 MHz, shader-clock) counter pairs every `period` real-time ticks, n pairs each: the shader clock's rate
// over the window is the XCD's core frequency while the step runs beside it.
__global__ __launch_bounds__(64) void clock_probe_kernel(unsigned long long* out, int n, unsigned long long period) {
  if (threadIdx.x != 0) return;
  unsigned long long* o = out + 2ull * n * blockIdx.x;
  for (int i = 0; i < n; ++i) {
    const unsigned long long r = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    o[2 * i] = r;
    o[2 * i + 1] = c;
    while (__builtin_amdgcn_s_memrealtime() - r < period) __builtin_amdgcn_s_sleep(2);
  }
}
int clock_probe_launch(hipStream_t st, int nwg, int n, int period, unsigned long long* out) {
  S2S_REQUIRE(nwg > 0 && nwg <= 64 && n > 0 && n <= (1 << 20) && period > 0 && (double)n * period < 2e8,
              "clock probe: bad arguments");
  hipLaunchKernelGGL(clock_probe_kernel, dim3(nwg), dim3(64), 0, st, out, n, (unsigned long long)period);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace s2s

extern "C" int s2s_debug_clock_probe(void* stream, int nwg, int n, int period, unsigned long long* out) {
  return s2s::clock_probe_launch(static_cast<hipStream_t>(stream), nwg, n, period, out);
}

// test stand-in for a collective on another stream (tests/test_gpu_coresident.py): nwg resident workgroups holding
// lds_bytes of LDS each for usec microseconds
extern "C" int s2s_debug_lds_hog(void* stream, int nwg, int lds_bytes, double usec, float* out) {
  return s2s::lds_hog_launch(static_cast<hipStream_t>(stream), nwg, lds_bytes, usec, out);
}

// diagnostic: the next persistent GRU launches fill these with stamps (tools/gru_stamps.py);
// nullptr turns it off.  Not part of the C ABI header.
// diagnostic: 0 forces write-through (sc1) hand-offs in every chain (tests cover both forms)
extern "C" void s2s_debug_gru_local(int allow) { s2s::g_allow_local = allow; }
extern "C" void s2s_debug_gru_fused_xproj(int on) { s2s::g_fuse_xproj = on; }
extern "C" void s2s_debug_gru_fused_dy(int on) { s2s::g_fuse_dy = on; }
extern "C" void s2s_debug_gru_xp_split(int on) { s2s::g_xp_split = on; }
extern "C" void s2s_debug_gru_xp_group(int on) { s2s::g_xp_group = on; }
extern "C" void s2s_debug_bptt_prefetch(int wg, int lookahead) {
  s2s::g_bptt_prefetch_wg = wg;
  s2s::g_bptt_prefetch = lookahead;
}
extern "C" void s2s_debug_gru_stream_sweep(int on) { s2s::g_stream_sweep = on; }
// diagnostic: 0 = one sentinel slot per step re-armed at launch start (the round-2 form), else the 4-slot ring
extern "C" void s2s_debug_gru_ring(int on) { s2s::g_sent_ring = on ? s2s::kSentRing : 0; }
extern "C" void s2s_debug_gru_stamps(void* fwd, void* bwd) {
  s2s::g_gru_stamps[0] = static_cast<unsigned long long*>(fwd);
  s2s::g_gru_stamps[1] = static_cast<unsigned long long*>(bwd);
}
// diagnostic: in-launch weight-gradient worker stamps [nchains][nw][L + 4] of the next BPTT launches (nullptr: off)
extern "C" void s2s_debug_gru_wg_stamps(void* p) { s2s::g_gru_wstamps = static_cast<unsigned long long*>(p); }
// diagnostic: producer item stamps [producer][32][2] of the next fused persistent launches (nullptr: off)
extern "C" void s2s_debug_gru_prod_stamps(void* fwd, void* bwd) {
  s2s::g_gru_pstamps[0] = static_cast<unsigned long long*>(fwd);
  s2s::g_gru_pstamps[1] = static_cast<unsigned long long*>(bwd);
}
