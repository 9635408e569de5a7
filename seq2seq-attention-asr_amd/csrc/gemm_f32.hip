// fp32 GEMM on the gfx950 f32-input MFMA (v_mfma_f32_32x32x2_f32: exact f32,
// one rounding per product, bit-identical to a k-ordered fmaf chain).
//
// Used for every "plain" contraction of the training step that is hoisted out of
// the recurrences: encoder input projections (the x-half of every GRU gate
// LinearZeroBias, LinearZeroBias.lua:31-48), the Vh precompute
// (TemporalConvolutionZeroBias(A,Sc,1), Attention.lua:43-47), the decoder MLP
// (Maxout.lua:15, model_chorowski_baseline.lua:56-57), and all weight-gradient
// GEMMs that the reference accumulates one rank-1 GER per time step
// (LinearZeroBias.lua:67-74) -- here one GEMM over all B*L rows.
//
// Tile 64x64x32, 256 threads = 4 waves in 2x2, each wave one 32x32 accumulator.
// LDS k-major [32][64+1] for both operands (column reads conflict-free), two LDS
// buffers, next tile prefetched into registers while the current one computes.
#include "s2s_common.h"

namespace s2s {

namespace {

constexpr int BM = 64, BN = 64, BK = 32, LDSP = BM + 1;

struct GemmBatchArgs {
  GemmProblem p[kMaxGemmBatch];
};

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmBatchArgs args) {
  const GemmProblem& p = args.p[blockIdx.z];
  const int M = p.M, N = p.N, K = p.K;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN;
  if (m0 >= M || n0 >= N) return;

  __shared__ float As[2][BK][LDSP];
  __shared__ float Bs[2][BK][LDSP];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = (wave >> 1) * 32, wn = (wave & 1) * 32;
  const float* __restrict__ A = p.A;
  const float* __restrict__ Bm = p.B;
  const long lda = p.lda, ldb = p.ldb;

  float ra[8], rb[8];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i;
      int kk, mm;
      if (TA) { kk = e >> 6; mm = e & 63; } else { kk = e & 31; mm = e >> 5; }
      const int gm = m0 + mm, gk = k0 + kk;
      float v = 0.f;
      if (gm < M && gk < K) v = TA ? A[(long)gk * lda + gm] : A[(long)gm * lda + gk];
      ra[i] = v;
      int kb, nn;
      if (TB) { kb = e & 31; nn = e >> 5; } else { kb = e >> 6; nn = e & 63; }
      const int gn = n0 + nn, gkb = k0 + kb;
      float w = 0.f;
      if (gn < N && gkb < K) w = TB ? Bm[(long)gn * ldb + gkb] : Bm[(long)gkb * ldb + gn];
      rb[i] = w;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int e = tid + 256 * i;
      int kk, mm;
      if (TA) { kk = e >> 6; mm = e & 63; } else { kk = e & 31; mm = e >> 5; }
      As[buf][kk][mm] = ra[i];
      int kb, nn;
      if (TB) { kb = e & 31; nn = e >> 5; } else { kb = e >> 6; nn = e & 63; }
      Bs[buf][kb][nn] = rb[i];
    }
  };

  floatx16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  const int nk = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  const int li = lane & 31, lk = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < nk) load((kt + 1) * BK);
#pragma unroll
    for (int kp = 0; kp < BK / 2; ++kp) {
      const float a = As[buf][2 * kp + lk][wm + li];
      const float b = Bs[buf][2 * kp + lk][wn + li];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
    }
    if (kt + 1 < nk) store(buf ^ 1);
    __syncthreads();
  }

  const float alpha = p.alpha, beta = p.beta;
  const float* __restrict__ bias = p.bias;
  float* __restrict__ C = p.C;
  const int col = n0 + wn + li;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = m0 + wm + (r & 3) + 8 * (r >> 2) + 4 * lk;
    if (row < M && col < N) {
      float v = alpha * acc[r];
      if (bias) v += bias[col];
      float* c = C + (long)row * p.ldc + col;
      if (beta != 0.f) v += beta * *c;
      *c = v;
    }
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

__global__ void copy2d_kernel(const float* __restrict__ src, long lds, float* __restrict__ dst, long ldd, int rows,
                              int cols, int accumulate) {
  const long n = (long)rows * cols;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const long r = i / cols, c = i - r * cols;
    const float v = src[r * lds + c];
    if (accumulate) dst[r * ldd + c] += v; else dst[r * ldd + c] = v;
  }
}

__global__ void axpby_kernel(const float* __restrict__ src, float* __restrict__ dst, size_t n, float alpha,
                             float beta) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    dst[i] = alpha * src[i] + (beta == 0.f ? 0.f : beta * dst[i]);
}

}  // namespace

int gemm_f32(hipStream_t st, const GemmProblem* probs, int nprob, bool transA, bool transB) {
  S2S_REQUIRE(nprob >= 1 && nprob <= kMaxGemmBatch, "gemm_f32: bad batch count");
  GemmBatchArgs args;
  int gm = 0, gn = 0, used = 0;
  for (int i = 0; i < nprob; ++i) {
    const GemmProblem& q = probs[i];
    if (q.M <= 0 || q.N <= 0) continue;
    S2S_REQUIRE(q.K >= 0 && q.C != nullptr, "gemm_f32: bad problem");
    args.p[used++] = q;
    gm = gm > (q.M + BM - 1) / BM ? gm : (q.M + BM - 1) / BM;
    gn = gn > (q.N + BN - 1) / BN ? gn : (q.N + BN - 1) / BN;
  }
  if (used == 0) return 0;
  double flops = 0, bytes = 0;
  for (int i = 0; i < used; ++i) {
    const GemmProblem& q = args.p[i];
    flops += 2.0 * q.M * q.N * q.K;
    bytes += 4.0 * ((double)q.M * q.K + (double)q.K * q.N + (double)q.M * q.N * (q.beta != 0.f ? 2 : 1));
  }
  ProfScope ps(st, "gemm_f32", flops, bytes);
  dim3 grid(gn, gm, used);
  if (!transA && !transB) hipLaunchKernelGGL((gemm_f32_kernel<false, false>), grid, dim3(256), 0, st, args);
  else if (!transA && transB) hipLaunchKernelGGL((gemm_f32_kernel<false, true>), grid, dim3(256), 0, st, args);
  else if (transA && !transB) hipLaunchKernelGGL((gemm_f32_kernel<true, false>), grid, dim3(256), 0, st, args);
  else hipLaunchKernelGGL((gemm_f32_kernel<true, true>), grid, dim3(256), 0, st, args);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int colsum_f32(hipStream_t st, const float* X, long ldx, int M, int N, float alpha, float beta, float* out) {
  if (N <= 0) return 0;
  hipLaunchKernelGGL(colsum_kernel, dim3((N + 63) / 64), dim3(1024), 0, st, X, ldx, M, N, alpha, beta, out);
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

int axpby_f32(hipStream_t st, const float* src, float* dst, size_t n, float alpha, float beta) {
  if (n == 0) return 0;
  size_t blocks = (n + 255) / 256;
  if (blocks > 2048) blocks = 2048;
  hipLaunchKernelGGL(axpby_kernel, dim3((unsigned)blocks), dim3(256), 0, st, src, dst, n, alpha, beta);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace s2s
