// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32 products,
// fp32 accumulation in a fixed k order -> deterministic, run to run and graph replay).
//
// Used for every "plain" contraction of the training step that is hoisted out of
// the recurrences: encoder input projections (the x-half of every GRU gate
// LinearZeroBias, LinearZeroBias.lua:31-48), the Vh precompute
// (TemporalConvolutionZeroBias(A,Sc,1), Attention.lua:43-47), the decoder MLP
// (Maxout.lua:15, model_chorowski_baseline.lua:56-57), and all weight-gradient
// GEMMs that the reference accumulates one rank-1 GER per time step
// (LinearZeroBias.lua:67-74) -- here one GEMM over all B*L rows.
//
// Tiles BM x BN x 32 (BM, BN in {128, 64}), 256 threads = 4 waves in 2 x 2, each wave
// (BM/64) x (BN/64) 32x32 accumulators.  Both operands are staged row-major in LDS with k
// contiguous ([r][32 + 4]); MFMA step ks of a K-tile pairs k = ks (lanes 0-31) with
// k = 16 + ks (lanes 32-63), so each lane's operands for the whole tile are 16 contiguous
// floats = 4 ds_read_b128 per fragment (row stride 36 floats: conflict-free per 16-lane group).
// Global reads are float4 (any row length): k-contiguous operands go to LDS with
// ds_write_b128, row-contiguous ones (A of TN, B of NN) are transposed by ds_write_b32 with
// lanes running along k (conflict-free).
// Batched problems are flattened into one 1-D grid; logical blocks are dealt XCD-contiguously
// (hardware deals blockIdx round-robin over the 8 XCDs), so neighbouring output tiles that
// share an A panel share an L2.  When the output has too few tiles to fill 256 CUs, K is cut
// into equal slices (split-K): each slice writes a partial slab and one reduce kernel sums the
// slabs in slice order (deterministic) and applies alpha / bias / beta.
#include "s2s_common.h"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

namespace s2s {

namespace {

constexpr int BK = 32, LDK = BK + 4;
// the operand loaders' float4: rows of any length (a TemporalConvolution window over 123-float frames, the GRU weight
// gradients' [h | x] rows) load as global_load_dwordx4 from 4-byte-aligned addresses (unaligned access mode)
typedef float floatx4u __attribute__((ext_vector_type(4), aligned(4)));

// Out-of-range lanes of the guarded operand loaders read this zero instead of branching around the
// load: a conditional value (cond ? x : 0) let the compiler sink each load into an exec-masked block
// followed by its own vmcnt(0) wait, serialising a tile's loads; a select between two addresses
// keeps every load of the tile in flight together.
__device__ float g_zero_f32 = 0.f;

struct GemmTile {
  GemmProblem p;
  float* part;  // split-K partial slabs (splits x M x N) or nullptr
  int tiles_n, tiles_m, splits, kslice;
  int base;  // first logical block of this problem
};
struct GemmLaunch {
  GemmTile q[kMaxGemmBatch];
  int nprob, nblocks;
};

// k-contiguous operand (element (r, k) at X[r * ld + k]): f -> row f / 8, k quad f % 8.
// FAST: interior tile -> unguarded float4.  Otherwise branch-free scalar loads
// from clamped addresses, zeroed outside the problem (no divergent waits between loads).
template <int R, bool FAST>
__device__ __forceinline__ void load_kc(floatx4 (&v)[R / 32], const float* X, long ld, int r0, int rmax, int k0,
                                        int kend) {
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int f = threadIdx.x + 256 * j;
    const int gr = r0 + (f >> 3), k = k0 + 4 * (f & 7);
    if (FAST) {
      v[j] = *reinterpret_cast<const floatx4u*>(X + (long)gr * ld + k);
    } else {
      const float* row = X + (long)min(gr, rmax - 1) * ld;
      float e[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        e[c] = *((gr < rmax && k + c < kend) ? row + k + c : &g_zero_f32);
      }
      v[j] = floatx4{e[0], e[1], e[2], e[3]};
    }
  }
}
template <int R>
__device__ __forceinline__ void store_kc(float* Xs, const floatx4 (&v)[R / 32]) {
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int f = threadIdx.x + 256 * j;
    *reinterpret_cast<floatx4*>(Xs + (f >> 3) * LDK + 4 * (f & 7)) = v[j];
  }
}
// row-contiguous operand (element (r, k) at X[k * ld + r]): f -> k = f % 32, row quad f / 32
template <int R, bool FAST>
__device__ __forceinline__ void load_rc(floatx4 (&v)[R / 32], const float* X, long ld, int r0, int rmax, int k0,
                                        int kend) {
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int f = threadIdx.x + 256 * j;
    const int k = k0 + (f & 31), r = r0 + 4 * (f >> 5);
    if (FAST) {
      v[j] = *reinterpret_cast<const floatx4u*>(X + (long)k * ld + r);
    } else {
      const float* row = X + (long)min(k, kend - 1) * ld;
      float e[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        e[c] = *((k < kend && r + c < rmax) ? row + r + c : &g_zero_f32);
      }
      v[j] = floatx4{e[0], e[1], e[2], e[3]};
    }
  }
}
template <int R>
__device__ __forceinline__ void store_rc(float* Xs, const floatx4 (&v)[R / 32]) {
#pragma unroll
  for (int j = 0; j < R / 32; ++j) {
    const int f = threadIdx.x + 256 * j;
    float* p = Xs + (4 * (f >> 5)) * LDK + (f & 31);
    p[0] = v[j][0];
    p[LDK] = v[j][1];
    p[2 * LDK] = v[j][2];
    p[3 * LDK] = v[j][3];
  }
}

// One K-tile's operand loads.  FAST (an interior tile): unguarded float4 loads while the K-tile is whole, the
// guarded form for a K tail (K = 3 x 123 for the first convolution: every tile used to take the guarded form).
template <bool TA, bool TB, int BM, int BN, bool FAST>
__device__ __forceinline__ void load_tile(floatx4 (&ra)[BM / 32], floatx4 (&rb)[BN / 32], const float* A,
                                          const float* Bm, long lda, long ldb, int m0, int n0, int M, int N, int k0,
                                          int kend) {
  if (FAST && k0 + BK <= kend) {
    if (TA) load_rc<BM, true>(ra, A, lda, m0, M, k0, kend); else load_kc<BM, true>(ra, A, lda, m0, M, k0, kend);
    if (TB) load_kc<BN, true>(rb, Bm, ldb, n0, N, k0, kend); else load_rc<BN, true>(rb, Bm, ldb, n0, N, k0, kend);
  } else {
    if (TA) load_rc<BM, false>(ra, A, lda, m0, M, k0, kend); else load_kc<BM, false>(ra, A, lda, m0, M, k0, kend);
    if (TB) load_kc<BN, false>(rb, Bm, ldb, n0, N, k0, kend); else load_rc<BN, false>(rb, Bm, ldb, n0, N, k0, kend);
  }
}

// Double-buffered K loop: the next K-tile's global loads are in flight (registers) while the
// current tile's 16 x FM x FN MFMAs run; one barrier per K-tile.  No lambdas here: captured
// prefetch arrays were left in scratch memory by the compiler.
template <bool TA, bool TB, int BM, int BN, bool FAST>
__device__ __forceinline__ void gemm_mainloop(floatx16 (&acc)[BM / 64][BN / 64], float (&As)[2][BM * LDK],
                                              float (&Bs)[2][BN * LDK], const float* __restrict__ A,
                                              const float* __restrict__ Bm, long lda, long ldb, int m0, int n0, int M,
                                              int N, int kbeg, int kend, int nk, int wy, int wx, int li, int lk) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 32, FN = WN / 32;
  floatx4 ra[BM / 32], rb[BN / 32];
  load_tile<TA, TB, BM, BN, FAST>(ra, rb, A, Bm, lda, ldb, m0, n0, M, N, kbeg, kend);
  if (TA) store_rc<BM>(As[0], ra); else store_kc<BM>(As[0], ra);
  if (TB) store_kc<BN>(Bs[0], rb); else store_rc<BN>(Bs[0], rb);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      load_tile<TA, TB, BM, BN, FAST>(ra, rb, A, Bm, lda, ldb, m0, n0, M, N, kbeg + (kt + 1) * BK, kend);
    }
    floatx4 a[FM][4], b[FN][4];
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const float* p = As[buf] + (wy * WM + 32 * f + li) * LDK + 16 * lk;
#pragma unroll
      for (int c = 0; c < 4; ++c) a[f][c] = *reinterpret_cast<const floatx4*>(p + 4 * c);
    }
#pragma unroll
    for (int g = 0; g < FN; ++g) {
      const float* p = Bs[buf] + (wx * WN + 32 * g + li) * LDK + 16 * lk;
#pragma unroll
      for (int c = 0; c < 4; ++c) b[g][c] = *reinterpret_cast<const floatx4*>(p + 4 * c);
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int g = 0; g < FN; ++g)
            acc[f][g] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[f][c][e], b[g][c][e], acc[f][g], 0, 0, 0);
      }
    }
    if (more) {
      if (TA) store_rc<BM>(As[buf ^ 1], ra); else store_kc<BM>(As[buf ^ 1], ra);
      if (TB) store_kc<BN>(Bs[buf ^ 1], rb); else store_rc<BN>(Bs[buf ^ 1], rb);
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ bf16 MFMA variant
// Same problem batching, XCD dealing and split-K as gemm_f32_kernel; the fp32 operands are rounded to bf16
// (RNE, v_cvt_pk_bf16_f32) while staged into LDS and multiplied with v_mfma_f32_16x16x32_bf16 (fp32
// accumulate; 16x the f32-MFMA rate), fp32 master operands in HBM, fp32 output.
//  * K-tile HBK = 64 (one barrier per 64-deep step); LDS rows of 64 bf16 + 8 pad (144-byte rows:
//    conflict-free ds_read_b128 per 16-lane group);
//  * each wave owns a (BM/2) x (BN/2) sub-tile = FM x FN accumulators of 16 x 16 (4 x 4 at 128 x 128);
//    lane l reads k = 8 (l >> 4) .. +7 of row l & 15 per 32-deep k-step (the bf16 A/B maps);
//  * k-contiguous operands: float4 global loads -> 4 bf16 -> ds_write_b64; row-contiguous ones
//    (A of TN, B of NN): a 4 (k) x 4 (rows) block per thread, transposed in registers, 4 ds_write_b64.
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int HBK = 64, HLD = HBK + 8;

// k-contiguous operand, R rows x HBK k: thread f (of R * 16 float4) -> row f / 16, k quad f % 16
template <int R, bool FAST>
__device__ __forceinline__ void hload_kc(floatx4 (&v)[R / 16], const float* X, long ld, int r0, int rmax, int k0,
                                         int kend) {
#pragma unroll
  for (int j = 0; j < R / 16; ++j) {
    const int f = threadIdx.x + 256 * j;
    const int gr = r0 + (f >> 4), k = k0 + 4 * (f & 15);
    if (FAST) {
      v[j] = *reinterpret_cast<const floatx4u*>(X + (long)gr * ld + k);
    } else {
      const float* row = X + (long)min(gr, rmax - 1) * ld;
      float e[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        e[c] = *((gr < rmax && k + c < kend) ? row + k + c : &g_zero_f32);
      }
      v[j] = floatx4{e[0], e[1], e[2], e[3]};
    }
  }
}
template <int R>
__device__ __forceinline__ void hstore_kc(__bf16* Xs, const floatx4 (&v)[R / 16]) {
#pragma unroll
  for (int j = 0; j < R / 16; ++j) {
    const int f = threadIdx.x + 256 * j;
    *reinterpret_cast<bf16x4*>(Xs + (f >> 4) * HLD + 4 * (f & 15)) = __builtin_convertvector(v[j], bf16x4);
  }
}
// row-contiguous operand (element (r, k) at X[k * ld + r]): thread block b (of R * HBK / 16) -> rows
// 4 (b % (R/4)) .. +3, k 4 (b / (R/4)) .. +3; v[4 j + c] = the float4 of rows at k + c
template <int R, bool FAST>
__device__ __forceinline__ void hload_rc(floatx4 (&v)[R / 16], const float* X, long ld, int r0, int rmax, int k0,
                                         int kend) {
#pragma unroll
  for (int j = 0; j < R / 64; ++j) {
    const int b = threadIdx.x + 256 * j;
    const int r = r0 + 4 * (b % (R / 4)), kb = k0 + 4 * (b / (R / 4));
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = kb + c;
      if (FAST) {
        v[4 * j + c] = *reinterpret_cast<const floatx4u*>(X + (long)k * ld + r);
      } else {
        const float* row = X + (long)min(k, kend - 1) * ld;
        float e[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          e[q] = *((k < kend && r + q < rmax) ? row + r + q : &g_zero_f32);
        }
        v[4 * j + c] = floatx4{e[0], e[1], e[2], e[3]};
      }
    }
  }
}
template <int R>
__device__ __forceinline__ void hstore_rc(__bf16* Xs, const floatx4 (&v)[R / 16]) {
#pragma unroll
  for (int j = 0; j < R / 64; ++j) {
    const int b = threadIdx.x + 256 * j;
    const int r = 4 * (b % (R / 4)), kb = 4 * (b / (R / 4));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 col = {v[4 * j][q], v[4 * j + 1][q], v[4 * j + 2][q], v[4 * j + 3][q]};
      *reinterpret_cast<bf16x4*>(Xs + (r + q) * HLD + kb) = __builtin_convertvector(col, bf16x4);
    }
  }
}

template <bool TA, bool TB, int BM, int BN, bool FAST>
__device__ __forceinline__ void gemm_mainloop_bf16(floatx4 (&acc)[BM / 32][BN / 32], __bf16 (&As)[2][BM * HLD],
                                                   __bf16 (&Bs)[2][BN * HLD], const float* __restrict__ A,
                                                   const float* __restrict__ Bm, long lda, long ldb, int m0, int n0,
                                                   int M, int N, int kbeg, int kend, int nk, int wy, int wx,
                                                   int lane) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  floatx4 ra[BM / 16], rb[BN / 16];
  if (TA) hload_rc<BM, FAST>(ra, A, lda, m0, M, kbeg, kend); else hload_kc<BM, FAST>(ra, A, lda, m0, M, kbeg, kend);
  if (TB) hload_kc<BN, FAST>(rb, Bm, ldb, n0, N, kbeg, kend); else hload_rc<BN, FAST>(rb, Bm, ldb, n0, N, kbeg, kend);
  if (TA) hstore_rc<BM>(As[0], ra); else hstore_kc<BM>(As[0], ra);
  if (TB) hstore_kc<BN>(Bs[0], rb); else hstore_rc<BN>(Bs[0], rb);
  __syncthreads();
  const int lr = lane & 15, lq = 8 * (lane >> 4);
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      const int k0 = kbeg + (kt + 1) * HBK;
      if (TA) hload_rc<BM, FAST>(ra, A, lda, m0, M, k0, kend); else hload_kc<BM, FAST>(ra, A, lda, m0, M, k0, kend);
      if (TB) hload_kc<BN, FAST>(rb, Bm, ldb, n0, N, k0, kend); else hload_rc<BN, FAST>(rb, Bm, ldb, n0, N, k0, kend);
    }
#pragma unroll
    for (int s = 0; s < HBK / 32; ++s) {
      bf16x8 a[FM], b[FN];
#pragma unroll
      for (int f = 0; f < FM; ++f)
        a[f] = *reinterpret_cast<const bf16x8*>(As[buf] + (wy * WM + 16 * f + lr) * HLD + 32 * s + lq);
#pragma unroll
      for (int g = 0; g < FN; ++g)
        b[g] = *reinterpret_cast<const bf16x8*>(Bs[buf] + (wx * WN + 16 * g + lr) * HLD + 32 * s + lq);
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int g = 0; g < FN; ++g)
          acc[f][g] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[f], b[g], acc[f][g], 0, 0, 0);
    }
    if (more) {
      if (TA) hstore_rc<BM>(As[buf ^ 1], ra); else hstore_kc<BM>(As[buf ^ 1], ra);
      if (TB) hstore_kc<BN>(Bs[buf ^ 1], rb); else hstore_rc<BN>(Bs[buf ^ 1], rb);
    }
    __syncthreads();
  }
}

template <bool TA, bool TB, int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_bf16_kernel(GemmLaunch Lc) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
  __shared__ __attribute__((aligned(16))) __bf16 As[2][BM * HLD];
  __shared__ __attribute__((aligned(16))) __bf16 Bs[2][BN * HLD];
  const int lin = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (lin >= Lc.nblocks) return;
  int pi = 0;
  while (pi + 1 < Lc.nprob && lin >= Lc.q[pi + 1].base) ++pi;
  const GemmTile& q = Lc.q[pi];
  int loc = lin - q.base;
  const int tn = loc % q.tiles_n;
  loc /= q.tiles_n;
  const int tm = loc % q.tiles_m, s = loc / q.tiles_m;
  const int M = q.p.M, N = q.p.N, K = q.p.K;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = s * q.kslice, kend = min(K, kbeg + q.kslice);
  floatx4 acc[FM][FN];
#pragma unroll
  for (int f = 0; f < FM; ++f)
#pragma unroll
    for (int g = 0; g < FN; ++g) acc[f][g] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wy = wave >> 1, wx = wave & 1;
  const int nk = (kend - kbeg + HBK - 1) / HBK;
  if (nk > 0) {
    const int Mr = max(M, q.p.Mread), Nr = max(N, q.p.Nread);
    const bool fast = m0 + BM <= Mr && n0 + BN <= Nr && (kend - kbeg) % HBK == 0;
    if (fast)
      gemm_mainloop_bf16<TA, TB, BM, BN, true>(acc, As, Bs, q.p.A, q.p.B, q.p.lda, q.p.ldb, m0, n0, M, N, kbeg, kend,
                                               nk, wy, wx, lane);
    else
      gemm_mainloop_bf16<TA, TB, BM, BN, false>(acc, As, Bs, q.p.A, q.p.B, q.p.lda, q.p.ldb, m0, n0, M, N, kbeg,
                                                kend, nk, wy, wx, lane);
  }
  // epilogue (16 x 16 accumulator map: column lane & 15, rows 4 (lane >> 4) + r)
  const float alpha = q.p.alpha, beta = q.p.beta;
  const float* __restrict__ bias = q.p.bias;
  float* __restrict__ C = q.p.C;
  float* __restrict__ part = q.part;
#pragma unroll
  for (int f = 0; f < FM; ++f)
#pragma unroll
    for (int g = 0; g < FN; ++g) {
      const int col = n0 + wx * WN + 16 * g + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wy * WM + 16 * f + 4 * (lane >> 4) + r;
        if (row < M && col < N) {
          if (part) {
            part[((long)s * M + row) * N + col] = acc[f][g][r];
          } else {
            float v = alpha * acc[f][g][r];
            if (bias) v += bias[col];
            if (q.p.rbias) v += q.p.rbias[row];
            float* c = C + (long)row * q.p.ldc + col;
            if (beta != 0.f) v += beta * *c;
            if (q.p.relu) v = fmaxf(v, 0.f);
            *c = v;
          }
        }
      }
    }
}

template <bool TA, bool TB, int BM, int BN>
__global__ __launch_bounds__(256, 2) void gemm_f32_kernel(GemmLaunch Lc) {
  constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 32, FN = WN / 32;
  __shared__ __attribute__((aligned(16))) float As[2][BM * LDK];
  __shared__ __attribute__((aligned(16))) float Bs[2][BN * LDK];

  const int lin = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
  if (lin >= Lc.nblocks) return;
  int pi = 0;
  while (pi + 1 < Lc.nprob && lin >= Lc.q[pi + 1].base) ++pi;
  const GemmTile& q = Lc.q[pi];
  int loc = lin - q.base;
  const int tn = loc % q.tiles_n;
  loc /= q.tiles_n;
  const int tm = loc % q.tiles_m, s = loc / q.tiles_m;
  const int M = q.p.M, N = q.p.N, K = q.p.K;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kbeg = s * q.kslice, kend = min(K, kbeg + q.kslice);
  const float* __restrict__ A = q.p.A;
  const float* __restrict__ Bm = q.p.B;
  const long lda = q.p.lda, ldb = q.p.ldb;

  floatx16 acc[FM][FN];
#pragma unroll
  for (int f = 0; f < FM; ++f)
#pragma unroll
    for (int g = 0; g < FN; ++g)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[f][g][r] = 0.f;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wy = wave >> 1, wx = wave & 1, li = lane & 31, lk = lane >> 5;
  const int nk = (kend - kbeg + BK - 1) / BK;

  if (nk > 0) {
    const int Mr = max(M, q.p.Mread), Nr = max(N, q.p.Nread);
    const bool fast = m0 + BM <= Mr && n0 + BN <= Nr;
    if (fast)
      gemm_mainloop<TA, TB, BM, BN, true>(acc, As, Bs, A, Bm, lda, ldb, m0, n0, M, N, kbeg, kend, nk, wy, wx, li, lk);
    else
      gemm_mainloop<TA, TB, BM, BN, false>(acc, As, Bs, A, Bm, lda, ldb, m0, n0, M, N, kbeg, kend, nk, wy, wx, li, lk);
  }

  const float alpha = q.p.alpha, beta = q.p.beta;
  const float* __restrict__ bias = q.p.bias;
  float* __restrict__ C = q.p.C;
  float* __restrict__ part = q.part;
#pragma unroll
  for (int f = 0; f < FM; ++f)
#pragma unroll
    for (int g = 0; g < FN; ++g) {
      const int col = n0 + wx * WN + 32 * g + li;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wy * WM + 32 * f + (r & 3) + 8 * (r >> 2) + 4 * lk;
        if (row < M && col < N) {
          if (part) {
            part[((long)s * M + row) * N + col] = acc[f][g][r];
          } else {
            float v = alpha * acc[f][g][r];
            if (bias) v += bias[col];
            if (q.p.rbias) v += q.p.rbias[row];
            float* c = C + (long)row * q.p.ldc + col;
            if (beta != 0.f) v += beta * *c;
            if (q.p.relu) v = fmaxf(v, 0.f);
            *c = v;
          }
        }
      }
    }
}

// C = alpha * (sum of the split slabs in slice order) (+ bias) + beta * C; blockIdx.y = problem.
// Every slab's load of a group of up to 8 in flight before its adds (a runtime-bounded loop issued them one by one
// behind each add: the 40-slice weight gradient of the 123-feature convolution took 42 us); the sum is the running
// sum in slice order either way.
template <typename V>
__device__ __forceinline__ V slab_ld(const float* p) { return *reinterpret_cast<const V*>(p); }
template <int S, typename V>
__device__ __forceinline__ void slab_add(V& sum, const float* part, long mn, long e) {
  V v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) v[s] = slab_ld<V>(part + s * mn + e);
#pragma unroll
  for (int s = 0; s < S; ++s) sum += v[s];
}
template <typename V>
__device__ __forceinline__ V slab_sum(const float* part, long mn, long e, int splits) {
  V sum = V(0.f);
  int s = 0;
  for (; s + 8 <= splits; s += 8) slab_add<8>(sum, part + s * mn, mn, e);
  switch (splits - s) {  // (the planner's fill rule picks any count, e.g. 7 for the encoder weight gradients)
    case 1: slab_add<1>(sum, part + s * mn, mn, e); break;
    case 2: slab_add<2>(sum, part + s * mn, mn, e); break;
    case 3: slab_add<3>(sum, part + s * mn, mn, e); break;
    case 4: slab_add<4>(sum, part + s * mn, mn, e); break;
    case 5: slab_add<5>(sum, part + s * mn, mn, e); break;
    case 6: slab_add<6>(sum, part + s * mn, mn, e); break;
    case 7: slab_add<7>(sum, part + s * mn, mn, e); break;
    default: break;
  }
  return sum;
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(GemmLaunch Lc) {
  const GemmTile& q = Lc.q[blockIdx.y];
  if (q.part == nullptr) return;
  const int M = q.p.M, N = q.p.N;
  const long mn = (long)M * N;
  const float alpha = q.p.alpha, beta = q.p.beta;
  const float* __restrict__ bias = q.p.bias;
  // float4 slab reads whenever the slabs allow them (mn % 4 = 0); float4 C writes only when C's rows do too -- else
  // the four outputs one by one (the GRU weight gradients' [H | D] rows of 379 floats, the convolution's 369)
  const bool vec = (mn % 4 == 0) && ((reinterpret_cast<uintptr_t>(q.part) & 15) == 0);
  const bool vc = (N % 4 == 0) && (q.p.ldc % 4 == 0) && ((reinterpret_cast<uintptr_t>(q.p.C) & 15) == 0);
  if (vec) {
    for (long e = 4 * (blockIdx.x * 256L + threadIdx.x); e < mn; e += 4L * gridDim.x * 256) {
      const floatx4 sum = slab_sum<floatx4>(q.part, mn, e, q.splits);
      if (vc) {
        const int row = (int)(e / N), col = (int)(e % N);
        floatx4 v = alpha * sum;
        if (bias) v += floatx4{bias[col], bias[col + 1], bias[col + 2], bias[col + 3]};
        if (q.p.rbias) v += q.p.rbias[row];
        floatx4* c = reinterpret_cast<floatx4*>(q.p.C + (long)row * q.p.ldc + col);
        if (beta != 0.f) v += beta * *c;
        if (q.p.relu)
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) v[e2] = fmaxf(v[e2], 0.f);
        *c = v;
      } else {
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const int row = (int)((e + e2) / N), col = (int)((e + e2) % N);
          float w = alpha * sum[e2];
          if (bias) w += bias[col];
          if (q.p.rbias) w += q.p.rbias[row];
          float* c = q.p.C + (long)row * q.p.ldc + col;
          if (beta != 0.f) w += beta * *c;
          if (q.p.relu) w = fmaxf(w, 0.f);
          *c = w;
        }
      }
    }
    return;
  }
  for (long e = blockIdx.x * 256L + threadIdx.x; e < mn; e += (long)gridDim.x * 256) {
    const float sum = slab_sum<float>(q.part, mn, e, q.splits);
    const int row = (int)(e / N), col = (int)(e % N);
    float v = alpha * sum;
    if (bias) v += bias[col];
    if (q.p.rbias) v += q.p.rbias[row];
    float* c = q.p.C + (long)row * q.p.ldc + col;
    if (beta != 0.f) v += beta * *c;
    if (q.p.relu) v = fmaxf(v, 0.f);
    *c = v;
  }
}

__global__ void colsum_kernel(const float* __restrict__ X, long ldx, int M, int N, float alpha, float beta,
                              float* __restrict__ out) {
  // 1024 threads = 64 columns x 16 row groups; fixed summation order (deterministic).
  __shared__ float red[16][65];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  float s = 0.f;
  if (col < N)
    for (int i = g; i < M; i += 16) s += X[(long)i * ldx + col];
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) {
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 16; ++j) t += red[j][c];
    out[col] = (beta == 0.f ? 0.f : beta * out[col]) + alpha * t;
  }
}

// two-stage column sums: part[p][col] = sum of row slice p (grid (N/64, parts), 64 columns x 4 row
// groups per workgroup), then out[col] = beta*out + alpha * sum_p part[p][col] in slice order.  Slices of >= 64
// rows (colsum_parts); a row group's rows go round-robin into four running sums (rows i, i + 4, i + 8, i + 12 into
// sums 0..3), so four loads are in flight per thread instead of one add chain behind each load (a 1280 x 256 bias
// gradient: 17 -> ~4 us), summed (s0 + s1) + (s2 + s3) -- one fixed order for a given M
constexpr int kColParts = 64;
__host__ __device__ inline int colsum_parts(int M) { return M < 128 ? 1 : (M + 63) / 64 < kColParts ? (M + 63) / 64 : kColParts; }
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ X, long ldx, int M, int N,
                                                          float* __restrict__ part) {
  __shared__ float red[4][65];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  const int chunk = (M + gridDim.y - 1) / gridDim.y;
  const int r0 = blockIdx.y * chunk, r1 = min(M, r0 + chunk);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (col < N) {
    const float* xc = X + col;
    int i = r0 + g;
    for (; i + 12 < r1; i += 16) {
      const float a0 = xc[(long)i * ldx], a1 = xc[(long)(i + 4) * ldx], a2 = xc[(long)(i + 8) * ldx],
                  a3 = xc[(long)(i + 12) * ldx];
      s0 += a0; s1 += a1; s2 += a2; s3 += a3;
    }
    if (i < r1) s0 += xc[(long)i * ldx];
    if (i + 4 < r1) s1 += xc[(long)(i + 4) * ldx];
    if (i + 8 < r1) s2 += xc[(long)(i + 8) * ldx];
  }
  const float s = (s0 + s1) + (s2 + s3);
  red[g][c] = s;
  __syncthreads();
  if (g == 0 && col < N) part[(long)blockIdx.y * N + col] = (red[0][c] + red[1][c]) + (red[2][c] + red[3][c]);
}
__global__ void colsum_final_kernel(const float* __restrict__ part, int parts, int N, float alpha, float beta,
                                    float* __restrict__ out) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= N) return;
  float t = 0.f;
  for (int p = 0; p < parts; ++p) t += part[(long)p * N + col];
  out[col] = (beta == 0.f ? 0.f : beta * out[col]) + alpha * t;
}

// colsum_scatter's second stage: output range e = blockIdx.y, columns col0 .. col0 + ncols of the parts, added
// (alpha-scaled, the same expression as colsum_final_kernel with beta = 1) into each of its destinations
__global__ void colsum_scatter_kernel(const float* __restrict__ part, int parts, int N, float alpha, ColsumOuts o) {
  const ColsumOut& e = o.e[blockIdx.y];
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= e.ncols) return;
  float t = 0.f;
  for (int p = 0; p < parts; ++p) t += part[(long)p * N + e.col0 + j];
  for (int q = 0; q < e.ndst; ++q) e.dst[q][j] = 1.f * e.dst[q][j] + alpha * t;
}

__global__ void copy2d_kernel(const float* __restrict__ src, long lds, float* __restrict__ dst, long ldd, int rows,
                              int cols, int accumulate) {
  const long n = (long)rows * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, c = i - r * cols;
    const float v = src[r * lds + c];
    if (accumulate) dst[r * ldd + c] += v; else dst[r * ldd + c] = v;
  }
}

__global__ void transpose_kernel(const float* __restrict__ src, long lds, int rows, int cols, float* __restrict__ dst,
                                 long ldd) {
  // dst[c*ldd + r] = src[r*lds + c]
  __shared__ float tile[32][33];
  const int r0 = blockIdx.y * 32, c0 = blockIdx.x * 32;
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int r = r0 + i, c = c0 + threadIdx.x;
    if (r < rows && c < cols) tile[i][threadIdx.x] = src[(long)r * lds + c];
  }
  __syncthreads();
  for (int i = threadIdx.y; i < 32; i += 8) {
    const int c = c0 + i, r = r0 + threadIdx.x;
    if (r < rows && c < cols) dst[(long)c * ldd + r] = tile[threadIdx.x][i];
  }
}

__global__ void pad_cols_kernel(const float* __restrict__ src, long lds, float* __restrict__ dst, int rows, int cols,
                                int dcols) {
  const long n = (long)rows * dcols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / dcols, c = i - r * dcols;
    dst[i] = c < cols ? src[r * lds + c] : 0.f;
  }
}

__global__ void fill_words_kernel(unsigned* __restrict__ dst, size_t n, unsigned v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) dst[i] = v;
}

__global__ void axpby_kernel(const float* __restrict__ src, float* __restrict__ dst, size_t n, float alpha,
                             float beta) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = alpha * src[i] + (beta == 0.f ? 0.f : beta * dst[i]);
}

#include "conv_bf16.inc"

}  // namespace

int check_resident(const void* fn, long grid, int block, size_t lds, const char* what) {
  struct Key {
    const void* fn;
    int block, dev;
    size_t lds;
  };
  static std::mutex mu;
  static std::vector<std::pair<Key, long>> cache;  // key -> resident workgroups on the device
  int dev = 0;
  S2S_CHECK_HIP(hipGetDevice(&dev));
  long cap = -1;
  {
    std::lock_guard<std::mutex> g(mu);
    for (const auto& e : cache)
      if (e.first.fn == fn && e.first.block == block && e.first.dev == dev && e.first.lds == lds) cap = e.second;
  }
  if (cap < 0) {
    int per_cu = 0, cus = 0;
    S2S_CHECK_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, block, lds));
    S2S_CHECK_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    cap = (long)per_cu * cus;
    std::lock_guard<std::mutex> g(mu);
    cache.push_back({Key{fn, block, dev, lds}, cap});
  }
  S2S_REQUIRE(grid <= cap, std::string(what) + ": persistent grid of " + std::to_string(grid) +
                               " workgroups exceeds the " + std::to_string(cap) + " the device holds at once");
  return 0;
}

static thread_local int g_gemm_prec = kGemmF32;
static thread_local GemmDeferred* g_gemm_defer = nullptr;
void set_gemm_defer_reduce(GemmDeferred* d) { g_gemm_defer = d; }
GemmDeferred* gemm_defer_reduce() { return g_gemm_defer; }
static thread_local bool g_wgrad_bf16 = false;
void set_gemm_precision(int p) { g_gemm_prec = p; }
int gemm_precision() { return g_gemm_prec; }
void set_wgrad_bf16(bool on) { g_wgrad_bf16 = on; }
bool wgrad_bf16() { return g_wgrad_bf16; }

struct GemmPlan {
  int bm = 64, bn = 64, kslice = 0, nblocks = 0;
};

// Pick the tile shape and a uniform K slice for the batch from a simple time model: every CU
// (256) works through ceil(blocks / 256) blocks of bm*bn*kslice MACs at a per-shape efficiency,
// plus the split slabs' HBM round trip and the reduce launch.
static GemmPlan plan_gemm(const GemmProblem* p, int n, size_t ws_floats, bool bf16) {
  int kmax = 0;
  for (int i = 0; i < n; ++i) kmax = p[i].K > kmax ? p[i].K : kmax;
  const int kq = bf16 ? HBK : BK;  // K-slices are whole K-tiles of the kernel
  const int kfull = (kmax + kq - 1) / kq * kq;
  auto count = [&](GemmPlan& pl) {  // blocks and slab floats of a plan; false if the slabs do not fit
    long blocks = 0;
    double slab = 0;
    for (int i = 0; i < n; ++i) {
      const long t = (long)((p[i].M + pl.bm - 1) / pl.bm) * ((p[i].N + pl.bn - 1) / pl.bn);
      const int sp = p[i].K > 0 && pl.kslice > 0 ? (p[i].K + pl.kslice - 1) / pl.kslice : 1;
      blocks += t * sp;
      if (sp > 1) slab += (double)sp * p[i].M * p[i].N;
    }
    pl.nblocks = (int)blocks;
    return slab <= (double)ws_floats;
  };
  GemmPlan pl;
  // Measured on MI355X (tools/gemm_bench.cpp, every GEMM shape of the training step): 64 x 64
  // tiles are the fastest or within a few % everywhere at these sizes (more blocks per CU hide
  // the global->LDS latency); split-K pays only while the output has fewer than 512 tiles
  // (2 per CU), and only down to 512-long K slices, until there are >= 1024 blocks.
  // (128x128 tiles for the VGG front-end's large outputs measured slower too: 15.8 -> 18.0 ms per
  // encoder fwd+bwd.)
  pl.bm = 64; pl.bn = 64; pl.kslice = kfull;
  count(pl);
  if (bf16) {  // bf16: the largest tile that still fills the chip (more MFMA work per staged byte); 64-row
    // tiles when every problem has <= 64 rows (the convolutions' Cout = 64 outputs)
    int mmax = 0;
    for (int i = 0; i < n; ++i) mmax = std::max(mmax, p[i].M);
    GemmPlan big = pl;
    big.bm = mmax <= 64 ? 64 : 128;
    big.bn = 128;
    count(big);
    if (big.nblocks >= 256) pl = big;
  }
  // (128 x 128 fp32 tiles for the encoder weight gradients: half the staged bytes per flop, no step gain)
  const int tiles = pl.nblocks;
  // (an output of fewer tiles than CUs may split down to 256-long slices: the decoder MLP's 1280 x 448 x 768 product
  // and the last layer's weight gradient, both on the critical path)
  const int kmin = tiles < 256 ? 256 : 512;
  if (tiles < 512 && !bf16) {  // (bf16: no step gain measured, config 3 4.063 vs 4.079 ms)
    // The split whose blocks all fit the chip in one round, with the shortest slice: time ~ rounds x slice,
    // rounds = ceil(blocks / resident slots), slots = 256 CUs x the blocks one CU holds by LDS.  A split that
    // leaves a short second round costs a whole slice more (layer 1's weight gradient, 144 tiles x K = 4096:
    // 8 slices of 512 = 1152 blocks, 2 rounds; 7 slices of 608 = 1008 blocks, one round: 96.3 -> 88.7 us in
    // tools/gemm_bench; the decoder MLP 22.8 -> 20.1 us; config-2 step 3.309 -> 3.304 ms, same-box A/B).
    const size_t lds = 2 * (size_t)(pl.bm + pl.bn) * LDK * sizeof(float);
    const long slots = 256L * std::max<long>(1, std::min<long>(8, (long)(160 * 1024 / lds)));
    auto cost = [&](const GemmPlan& q) { return (double)((q.nblocks + slots - 1) / slots) * q.kslice; };
    GemmPlan best = pl;
    double bc = cost(pl);
    int prev = pl.kslice;
    for (int s = 2;; ++s) {
      GemmPlan nx = pl;
      nx.kslice = ((kfull + s - 1) / s + kq - 1) / kq * kq;
      if (nx.kslice < kmin) break;
      if (nx.kslice == prev) continue;
      prev = nx.kslice;
      if (!count(nx)) break;
      const double c = cost(nx);
      if (c < bc) {
        bc = c;
        best = nx;
      }
    }
    return best;
  }
  while (tiles < 512 && pl.nblocks < 1024 && pl.kslice / 2 >= kmin) {
    GemmPlan nx = pl;
    nx.kslice = (pl.kslice / 2 + kq - 1) / kq * kq;
    if (!count(nx)) break;
    pl = nx;
  }
  return pl;
}

template <bool TA, bool TB>
static void launch_tiles(hipStream_t st, const GemmPlan& pl, dim3 grid, const GemmLaunch& L, bool bf16) {
  if (bf16) {
    if (pl.bm == 128 && pl.bn == 128) hipLaunchKernelGGL((gemm_bf16_kernel<TA, TB, 128, 128>), grid, dim3(256), 0, st, L);
    else if (pl.bn == 128) hipLaunchKernelGGL((gemm_bf16_kernel<TA, TB, 64, 128>), grid, dim3(256), 0, st, L);
    else if (pl.bm == 128) hipLaunchKernelGGL((gemm_bf16_kernel<TA, TB, 128, 64>), grid, dim3(256), 0, st, L);
    else hipLaunchKernelGGL((gemm_bf16_kernel<TA, TB, 64, 64>), grid, dim3(256), 0, st, L);
    return;
  }
  if (pl.bm == 128 && pl.bn == 128) hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, 128, 128>), grid, dim3(256), 0, st, L);
  else if (pl.bm == 128) hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, 128, 64>), grid, dim3(256), 0, st, L);
  else hipLaunchKernelGGL((gemm_f32_kernel<TA, TB, 64, 64>), grid, dim3(256), 0, st, L);
}

int gemm_f32(hipStream_t st, const GemmProblem* probs, int nprob, bool transA, bool transB, GemmWs ws) {
  S2S_REQUIRE(nprob >= 1 && nprob <= kMaxGemmBatch, "gemm_f32: bad batch count");
  GemmProblem use[kMaxGemmBatch];
  int used = 0;
  for (int i = 0; i < nprob; ++i) {
    const GemmProblem& q = probs[i];
    if (q.M <= 0 || q.N <= 0) continue;
    S2S_REQUIRE(q.K >= 0 && q.C != nullptr, "gemm_f32: bad problem");
    use[used++] = q;
  }
  if (used == 0) return 0;
  const bool bf16 = gemm_precision() == kGemmBf16;
  // large bf16 problems of the module-level entry points (front-end, attention decoder) on the big-tile kernel
  // (gemm_big_bf16: it needs the calling context's staging buffer, which the model step does not provide) -- one
  // call each, stream-ordered; the rest stay in one launch of this file's kernels
  if (bf16) {
    int keep = 0;
    for (int i = 0; i < used; ++i) {
      const GemmProblem& q = use[i];
      bool done = false;
      if (2.0 * q.M * (double)q.N * q.K >= 1e9) S2S_TRY(gemm_big_bf16(st, q, transA, transB, &done));
      if (!done) use[keep++] = q;
    }
    used = keep;
    if (used == 0) return 0;
  }
  const GemmPlan pl = plan_gemm(use, used, ws.p ? ws.n : 0, bf16);
  GemmLaunch L{};
  L.nprob = used;
  int base = 0;
  size_t woff = 0;
  bool split = false;
  double flops = 0, bytes = 0;
  for (int i = 0; i < used; ++i) {
    GemmTile& t = L.q[i];
    t.p = use[i];
    t.tiles_m = (t.p.M + pl.bm - 1) / pl.bm;
    t.tiles_n = (t.p.N + pl.bn - 1) / pl.bn;
    t.kslice = t.p.K > 0 ? pl.kslice : BK;
    t.splits = t.p.K > 0 ? (t.p.K + pl.kslice - 1) / pl.kslice : 1;
    if (t.p.K == 0) t.kslice = 0;
    t.part = nullptr;
    if (t.splits > 1) {
      t.part = ws.p + woff;
      woff += (size_t)t.splits * t.p.M * t.p.N;
      split = true;
    }
    t.base = base;
    base += t.tiles_m * t.tiles_n * t.splits;
    flops += 2.0 * t.p.M * t.p.N * t.p.K;
    bytes += 4.0 * ((double)t.p.M * t.p.K + (double)t.p.K * t.p.N + (double)t.p.M * t.p.N * (t.p.beta != 0.f ? 2 : 1));
  }
  L.nblocks = base;
  ProfScope ps(st, bf16 ? "gemm_bf16" : "gemm_f32", flops, bytes);
  const dim3 grid((unsigned)((base + 7) / 8 * 8));
  if (!transA && !transB) launch_tiles<false, false>(st, pl, grid, L, bf16);
  else if (!transA && transB) launch_tiles<false, true>(st, pl, grid, L, bf16);
  else if (transA && !transB) launch_tiles<true, false>(st, pl, grid, L, bf16);
  else launch_tiles<true, true>(st, pl, grid, L, bf16);
  GemmDeferred* dr = g_gemm_defer;
  if (dr) dr->splits = 0;
  if (split && dr && used == 1 && L.q[0].p.alpha == 1.f && L.q[0].p.beta == 0.f && !L.q[0].p.rbias && !L.q[0].p.relu) {
    dr->part = L.q[0].part;  // (GemmDeferReduce) the consumer sums the slabs
    dr->splits = L.q[0].splits;
    dr->mn = (long)L.q[0].p.M * L.q[0].p.N;
  } else if (split) {
    long mn_max = 0;
    for (int i = 0; i < used; ++i)
      if (L.q[i].part) mn_max = std::max(mn_max, (long)L.q[i].p.M * L.q[i].p.N);
    const unsigned gx = (unsigned)std::min<long>(1024, (mn_max + 1023) / 1024);
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3(gx, used), dim3(256), 0, st, L);
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int colsum_f32(hipStream_t st, const float* X, long ldx, int M, int N, float alpha, float beta, float* out,
               GemmWs ws) {
  if (N <= 0) return 0;
  // row slices of >= 64 rows, at most kColParts; the fixed slice grid keeps the sum order
  // independent of the workspace size once the two-stage form is taken
  const int parts = colsum_parts(M);
  if (ws.p && parts > 1 && ws.n >= (size_t)kColParts * N) {
    hipLaunchKernelGGL(colsum_part_kernel, dim3((N + 63) / 64, parts), dim3(256), 0, st, X, ldx, M, N, ws.p);
    hipLaunchKernelGGL(colsum_final_kernel, dim3((N + 255) / 256), dim3(256), 0, st, ws.p, parts, N, alpha, beta,
                       out);
  } else {
    hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64), dim3(1024), 0, st, X, ldx, M, N, alpha, beta, out);
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int colsum_scatter_f32(hipStream_t st, const float* X, long ldx, int M, int N, float alpha, const ColsumOut* outs,
                       int nouts, GemmWs ws) {
  S2S_REQUIRE(nouts >= 0 && nouts <= kMaxColsumOuts, "colsum_scatter: too many output ranges");
  if (N <= 0 || nouts == 0) return 0;
  const int parts = colsum_parts(M);
  if (!(ws.p && parts > 1 && ws.n >= (size_t)kColParts * N)) {  // colsum_f32's one-stage form per destination
    for (int e = 0; e < nouts; ++e)
      for (int q = 0; q < outs[e].ndst; ++q)
        S2S_TRY(colsum_f32(st, X + outs[e].col0, ldx, M, outs[e].ncols, alpha, 1.f, outs[e].dst[q], ws));
    return 0;
  }
  ColsumOuts o{};
  int maxc = 0;
  for (int e = 0; e < nouts; ++e) {
    S2S_REQUIRE(outs[e].col0 >= 0 && outs[e].col0 + outs[e].ncols <= N && outs[e].ndst <= 3, "colsum_scatter: bad range");
    o.e[e] = outs[e];
    maxc = std::max(maxc, outs[e].ncols);
  }
  hipLaunchKernelGGL(colsum_part_kernel, dim3((N + 63) / 64, parts), dim3(256), 0, st, X, ldx, M, N, ws.p);
  hipLaunchKernelGGL(colsum_scatter_kernel, dim3((maxc + 255) / 256, nouts), dim3(256), 0, st, ws.p, parts, N, alpha,
                     o);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int copy2d_f32(hipStream_t st, const float* src, long lds, float* dst, long ldd, int rows, int cols, bool acc) {
  if (rows <= 0 || cols <= 0) return 0;
  long n = (long)rows * cols;
  int blocks = (int)((n + 255) / 256);
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(copy2d_kernel, dim3(blocks), dim3(256), 0, st, src, lds, dst, ldd, rows, cols, acc ? 1 : 0);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int transpose_f32(hipStream_t st, const float* src, long lds, int rows, int cols, float* dst, long ldd) {
  hipLaunchKernelGGL(transpose_kernel, dim3((cols + 31) / 32, (rows + 31) / 32), dim3(32, 8), 0, st, src, lds, rows,
                     cols, dst, ldd);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int pad_cols_f32(hipStream_t st, const float* src, long lds, float* dst, int rows, int cols, int dcols) {
  if (rows <= 0 || dcols <= 0) return 0;
  const long n = (long)rows * dcols;
  const int blocks = (int)std::min<long>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(pad_cols_kernel, dim3(blocks), dim3(256), 0, st, src, lds, dst, rows, cols, dcols);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int axpby_f32(hipStream_t st, const float* src, float* dst, size_t n, float alpha, float beta) {
  if (n == 0) return 0;
  size_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, n, alpha, beta);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// Kernel fills instead of hipMemsetAsync / hipMemsetD32Async: measured on MI355X (ROCm 7.2), a memset
// captured into a HIP graph together with the kernels around it did not clear its range on the second and
// later replays (a captured LSTM fwd + bwd read the previous replay's carries: tools/diag_graph.py);
// a fill kernel is an ordinary kernel node.
int fill_u32_async(hipStream_t st, void* dst, unsigned value, size_t count) {
  S2S_REQUIRE((reinterpret_cast<uintptr_t>(dst) & 3) == 0, "fill_u32_async: dst must be 4-byte aligned");
  if (count == 0) return 0;
  size_t blocks = (count + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(fill_words_kernel, dim3((unsigned)blocks), dim3(256), 0, st, static_cast<unsigned*>(dst), count,
                     value);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int zero_async(hipStream_t st, void* dst, size_t bytes) {
  S2S_REQUIRE(bytes % 4 == 0, "zero_async: whole 4-byte words only");
  return fill_u32_async(st, dst, 0u, bytes / 4);
}

// ------------------------------------------------------------------ implicit-GEMM convolutions (conv_bf16.inc)
static int conv_launch(hipStream_t st, bool dx, ConvArgs& c, const float* W, void* scratch, const char* name) {
  S2S_REQUIRE(c.M > 0 && c.K > 0 && c.N > 0, "conv: bad sizes");
  S2S_REQUIRE(c.g.kH == c.g.kW && (c.g.kW == 3 || c.g.kW == 1), "conv: implicit bf16 path for 3x3 / 1x1 kernels");
  const int kk = c.g.kH * c.g.kW;
  float* wr = static_cast<float*>(scratch);
  __bf16* xh = reinterpret_cast<__bf16*>(static_cast<char*>(scratch) +
                                         (sconv_implicit_wscratch_bytes(c.g.Cin, c.g.Cout, c.g.kH, c.g.kW) + 255) / 256 * 256);
  // tap-major K over a channels-last bf16 copy when the gathered tensor's channels fill whole K-tiles
  // (every VGG layer but the first)
  const int C = dx ? c.g.Cout : c.g.Cin;
  const bool tapk = C % HBK == 0;
  if (tapk) {
    const long P = dx ? (long)c.g.B * c.g.Ho * c.g.Wo : (long)c.g.H * c.g.W;  // dx: dyt (Cout, B Ho Wo) as one image
    const int nb = dx ? 1 : c.g.B;
    S2S_REQUIRE(P < (1L << 31) / 64, "conv: image too large");
    hipLaunchKernelGGL(nchw_to_nhwc_bf16, dim3((unsigned)((P + 63) / 64), C / 64, nb), dim3(256), 0, st, c.X, nullptr, C,
                       (int)P, xh);
    c.Xh = xh;
    c.xhlen = (long)nb * P * C;
  }
  if (dx || tapk) {  // weights in the GEMM's K order (the first layer's forward reads W as it is)
    hipLaunchKernelGGL(conv_w_relayout, dim3(std::min(1024, (c.g.Cout * c.g.Cin * kk + 255) / 256)), dim3(256), 0,
                       st, W, c.g.Cout, c.g.Cin, kk, dx ? 1 : 0, tapk ? 1 : 0, wr);
    S2S_CHECK_HIP(hipGetLastError());
    c.A = wr;
  } else {
    c.A = W;
  }
  const long tiles_n = (c.N + kConvBN - 1) / kConvBN;
  c.tiles_m = (c.M + kConvBM - 1) / kConvBM;
  S2S_REQUIRE(tiles_n * c.tiles_m < 2147483647L / 8, "conv: too many tiles");
  c.nblocks = (int)(tiles_n * c.tiles_m);
  const double flops = 2.0 * c.M * (double)c.N * c.K;
  const double bytes = 4.0 * ((double)c.M * c.K + (double)c.N * c.K / kk + (double)c.M * c.N);
  ProfScope ps(st, name, flops, bytes);
  const dim3 grid((unsigned)((c.nblocks + 7) / 8 * 8));
#define S2S_CONV_LAUNCH(DXV, KWV, TK) hipLaunchKernelGGL((conv_bf16_kernel<DXV, KWV, TK>), grid, dim3(256), 0, st, c)
  if (c.g.kW == 3) {
    if (dx) { if (tapk) S2S_CONV_LAUNCH(true, 3, true); else S2S_CONV_LAUNCH(true, 3, false); }
    else { if (tapk) S2S_CONV_LAUNCH(false, 3, true); else S2S_CONV_LAUNCH(false, 3, false); }
  } else {
    if (dx) { if (tapk) S2S_CONV_LAUNCH(true, 1, true); else S2S_CONV_LAUNCH(true, 1, false); }
    else { if (tapk) S2S_CONV_LAUNCH(false, 1, true); else S2S_CONV_LAUNCH(false, 1, false); }
  }
#undef S2S_CONV_LAUNCH
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

size_t sconv_implicit_wscratch_bytes(int Cin, int Cout, int kH, int kW) {
  return sizeof(float) * (size_t)Cin * Cout * kH * kW;
}
size_t sconv_implicit_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW) {
  const size_t act = std::max((size_t)B * Cin * H * W, (size_t)B * Cout * (H - kH + 1) * (W - kW + 1));
  return (sconv_implicit_wscratch_bytes(Cin, Cout, kH, kW) + 255) / 256 * 256 + 2 * act;
}

int sconv_fwd_implicit(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x,
                       const float* Wt, const float* bias, float* y, void* scratch) {
  ConvArgs c{};
  c.g = ConvGeom{B, Cin, H, W, Cout, kH, kW, H - kH + 1, W - kW + 1};
  S2S_REQUIRE((long)B * Cin * H * W < (1L << 29) && (long)B * Cout * c.g.Ho * c.g.Wo < (1L << 29),
              "conv: implicit bf16 path needs tensors below 2^29 elements (32-bit byte offsets)");
  c.X = x;
  c.xlen = (long)B * Cin * H * W;
  c.bias = bias;
  c.Y = y;
  c.M = Cout;
  c.K = Cin * kH * kW;
  c.N = (long)B * c.g.Ho * c.g.Wo;
  c.relu = relu;
  return conv_launch(st, false, c, Wt, scratch, "conv_fwd_bf16");
}

int sconv_dx_implicit(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, const float* Wt,
                      const float* dyt, float* dx, int accumulate, void* scratch) {
  ConvArgs c{};
  c.g = ConvGeom{B, Cin, H, W, Cout, kH, kW, H - kH + 1, W - kW + 1};
  S2S_REQUIRE((long)B * Cin * H * W < (1L << 29) && (long)B * Cout * c.g.Ho * c.g.Wo < (1L << 29),
              "conv: implicit bf16 path needs tensors below 2^29 elements (32-bit byte offsets)");
  c.X = dyt;
  c.xlen = (long)Cout * B * c.g.Ho * c.g.Wo;
  c.Y = dx;
  c.M = Cin;
  c.K = Cout * kH * kW;
  c.N = (long)B * H * W;
  c.accumulate = accumulate;
  return conv_launch(st, true, c, Wt, scratch, "conv_dx_bf16");
}

// weight gradient on the channels-last bf16 copy of x (conv_wgrad_bf16_kernel): xh in xh_scratch, the split-K
// partial tiles in slab (both scratch regions the im2col path would have used for its panels)
size_t sconv_wgrad_slab_floats(int B, int Cin, int H, int W, int Cout, int kH, int kW, int* S_out, long* chunk_out) {
  const long BN = (long)B * (H - kH + 1) * (W - kW + 1);
  const int kk = kH * kW, tiles = ((Cout + kConvBM - 1) / kConvBM) * (kk * Cin / kConvBN);
  const long ktiles = (BN + HBK - 1) / HBK;
  // ~2048 workgroups, at least 8 K-tiles per chunk
  long S = std::max(1L, std::min(ktiles / 8, (2048L + tiles - 1) / tiles));
  const long chunk = (ktiles + S - 1) / S * HBK;
  S = (BN + chunk - 1) / chunk;
  if (S_out) *S_out = (int)S;
  if (chunk_out) *chunk_out = chunk;
  return (size_t)S * Cout * kk * Cin;
}
int sconv_wgrad_implicit(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, const float* x,
                         const float* dyt, float* dW, float scale, void* xh_scratch, size_t xh_bytes, float* slab,
                         size_t slab_bytes) {
  WgradArgs c{};
  c.g = ConvGeom{B, Cin, H, W, Cout, kH, kW, H - kH + 1, W - kW + 1};
  const int kk = kH * kW;
  S2S_REQUIRE(Cin % kConvBN == 0 && Cout > 0 && B > 0, "conv wgrad: implicit bf16 path needs Cin % 64 == 0");
  const long P = (long)H * W;
  c.xhlen = (long)B * P * Cin;
  S2S_REQUIRE(2 * c.xhlen < (1L << 31) - 4096, "conv wgrad: input too large for 32-bit byte offsets");
  S2S_REQUIRE(xh_bytes >= 2 * (size_t)c.xhlen, "conv wgrad: scratch too small");
  int S;
  long chunk;
  const size_t nslab = sconv_wgrad_slab_floats(B, Cin, H, W, Cout, kH, kW, &S, &chunk);
  S2S_REQUIRE(sizeof(float) * nslab <= slab_bytes, "conv wgrad: slab scratch too small");
  __bf16* xh = static_cast<__bf16*>(xh_scratch);
  hipLaunchKernelGGL(nchw_to_nhwc_bf16, dim3((unsigned)((P + 63) / 64), Cin / 64, B), dim3(256), 0, st, x, nullptr, Cin,
                     (int)P, xh);
  c.dyt = dyt;
  c.BN = (long)B * c.g.Ho * c.g.Wo;
  c.xh = xh;
  c.slab = slab;
  c.tiles_m = (Cout + kConvBM - 1) / kConvBM;
  c.tiles_n = kk * Cin / kConvBN;
  c.S = S;
  c.chunk = chunk;
  c.nblocks = c.tiles_m * c.tiles_n * S;
  {
    ProfScope ps(st, "conv_wgrad_bf16", 2.0 * Cout * (double)kk * Cin * c.BN,
                 4.0 * (double)Cout * c.BN + 2.0 * c.xhlen + 4.0 * nslab);
    hipLaunchKernelGGL(conv_wgrad_bf16_kernel, dim3((unsigned)((c.nblocks + 7) / 8 * 8)), dim3(256), 0, st, c);
    S2S_CHECK_HIP(hipGetLastError());
  }
  const long n = (long)Cout * Cin * kk;
  hipLaunchKernelGGL(conv_wgrad_reduce, dim3((unsigned)std::min<long>(1024, (n + 255) / 256)), dim3(256), 0, st, slab,
                     S, Cout, Cin, kk, scale, dW);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace s2s
