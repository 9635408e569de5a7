// Encoder front-ends: the operators of the two non-GRU encoders the reference
// builds --
//   * the conv + BiLSTM encoder of timit/timit.lua:108-125: 3 x [TemporalConvolution(D, 256, 3) ->
//     ReLU -> TemporalMaxPooling(2, 2)], then a BiLSTM (csrc/lstm.hip);
//   * the VGG stack of librispeech/model_vgg.lua:23-51: SpatialConvolutionMM(3x3) + ReLU pairs,
//     SpatialMaxPooling(2,1,2,1) / (2,2,2,2), Transpose2({1,2},3) + View, four
//     TemporalConvolution(., ., 1) + ReLU layers.
// Torch7 layouts at the boundary: TemporalConvolution x (B, L, Din), W (Dout, kW*Din) with the
// window's frames consecutive (row = [x_t | x_{t+1} | ...]); SpatialConvolutionMM x (B, C, H, W)
// with H = time, W = frequency (model_vgg.lua:37-41), weight (Cout, Cin*kH*kW) in (c, i, j) order.
//
// MI355X mapping: every contraction is the fp32 MFMA GEMM of gemm_f32.hip.
//   * TemporalConvolution needs no unfold: window t of utterance b is the CONTIGUOUS row segment
//     x[b, t:t+kW, :], so the forward is one GEMM per utterance on A = x_b with lda = Din and
//     K = kW*Din (overlapping rows), bias and ReLU in the epilogue.  The weight gradient runs as ONE
//     GEMM over all B*L - kW + 1 window rows of the batch against dY zero-padded to L rows per
//     utterance (the windows that straddle two utterances meet zero rows), and dx is dU = dY W
//     followed by a gather dx[t] = sum_i dU[t - i, i*Din:(i+1)*Din].
//   * SpatialConvolutionMM: im2col into a (K, B*N) panel (K = Cin*kH*kW, N = H'*W'), forward GEMMs
//     write NCHW directly (one problem per utterance, channel bias per output row, ReLU in the
//     epilogue); the backward permutes dY (masked by the ReLU) into (Cout, B*N) once, so dW is one
//     NT GEMM over all B*N columns and the input gradient one TN GEMM (dcol) + a col2im gather.
//   * Pooling, masks, permutes: one thread per output element, coalesced along the innermost dim.
// Every reduction has a fixed order (deterministic, graph-replay safe).
#include "s2s_common.h"

#include <algorithm>

namespace s2s {

namespace {

inline unsigned grid1d(long n, int per = 256) { return (unsigned)std::min<long>(4096, (n + per - 1) / per); }

// dyp[b, t, :] = dy[b, t, :] * (relu ? 1[y > 0] : 1) for t < Lo; 0 for Lo <= t < L.
__global__ void tconv_pad_dy(const float* __restrict__ dy, const float* __restrict__ y, int relu, int B, int L,
                             int Lo, int D, float* __restrict__ dyp) {
  const long n = (long)B * L * D;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % D);
    const long bt = e / D;
    const int t = (int)(bt % L), b = (int)(bt / L);
    float v = 0.f;
    if (t < Lo) {
      const long src = ((long)b * Lo + t) * D + c;
      v = dy[src];
      if (relu && !(y[src] > 0.f)) v = 0.f;
    }
    dyp[e] = v;
  }
}

// dx[b, t, c] (+)= sum_{i <= t, i < kW} dU[b*L + t - i, i*Din + c]  (window rows past Lo are zero in dU)
__global__ void tconv_gather_dx(const float* __restrict__ dU, int B, int L, int Din, int kW, int acc,
                                float* __restrict__ dx) {
  const long n = (long)B * L * Din;
  const long ldu = (long)kW * Din;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % Din);
    const long bt = e / Din;
    const int t = (int)(bt % L);
    float s = 0.f;
    for (int i = 0; i < kW && i <= t; ++i) s += dU[(bt - i) * ldu + (long)i * Din + c];
    dx[e] = acc ? dx[e] + s : s;
  }
}

// TemporalMaxPooling(kW, dW): y[b, o, c] = max_{i < kW} x[b, o*dW + i, c], first maximum wins (strict >)
__global__ void tmaxpool_fwd_kernel(const float* __restrict__ x, int B, int L, int D, int kW, int dW, int Lo,
                                    float* __restrict__ y, int* __restrict__ idx) {
  const long n = (long)B * Lo * D;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % D);
    const long bo = e / D;
    const int o = (int)(bo % Lo), b = (int)(bo / Lo);
    const float* xp = x + ((long)b * L + (long)o * dW) * D + c;
    float m = xp[0];
    int k = 0;
    for (int i = 1; i < kW; ++i) {
      const float v = xp[(long)i * D];
      if (v > m) {
        m = v;
        k = i;
      }
    }
    y[e] = m;
    idx[e] = k;
  }
}

// dx[b, t, c] = sum over windows o containing t whose argmax is t of dy[b, o, c]  (gather: no atomics)
__global__ void tmaxpool_bwd_kernel(const int* __restrict__ idx, const float* __restrict__ dy, int B, int L, int D,
                                    int kW, int dW, int Lo, float* __restrict__ dx) {
  const long n = (long)B * L * D;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int c = (int)(e % D);
    const long bt = e / D;
    const int t = (int)(bt % L), b = (int)(bt / L);
    float s = 0.f;
    const int ohi = min(t / dW, Lo - 1);
    for (int o = ohi; o >= 0 && o * dW + kW > t; --o) {
      const long oe = ((long)b * Lo + o) * D + c;
      if (o * dW + idx[oe] == t) s += dy[oe];
    }
    dx[e] = s;
  }
}

// col[(c*kH + i)*kW + j][b*N + oh*Wo + ow] = x[b, c, oh + i, ow + j]   (col row stride B*N)
// grid (ceil(N/256), K, B): one panel row r and utterance b per (y, z); 32-bit index math only
__global__ __launch_bounds__(256) void im2col_kernel(const float* __restrict__ x, int B, int C, int H, int W, int kH,
                                                     int kW, int Ho, int Wo, float* __restrict__ col) {
  const int N = Ho * Wo;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= N) return;
  const int r = blockIdx.y, b = blockIdx.z;
  const int j = r % kW, i = (r / kW) % kH, c = r / (kW * kH);
  const int oh = p / Wo, ow = p - oh * Wo;
  col[(long)r * B * N + (long)b * N + p] = x[(((long)b * C + c) * H + oh + i) * W + ow + j];
}

// the same with four consecutive panel columns per thread (N % 4 == 0: 16-byte aligned float4 stores);
// grid (ceil(N/1024), K, B)
__global__ __launch_bounds__(256) void im2col4_kernel(const float* __restrict__ x, int B, int C, int H, int W,
                                                      int kH, int kW, int Ho, int Wo, float* __restrict__ col) {
  const int N = Ho * Wo;
  const int p = 4 * (blockIdx.x * 256 + threadIdx.x);
  if (p >= N) return;
  const int r = blockIdx.y, b = blockIdx.z;
  const int j = r % kW, i = (r / kW) % kH, c = r / (kW * kH);
  int oh = p / Wo, ow = p - oh * Wo;
  const float* xp = x + ((long)b * C + c) * H * W + (long)i * W + j;
  floatx4 v;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = xp[(long)oh * W + ow];
    if (++ow == Wo) {
      ow = 0;
      ++oh;
    }
  }
  *reinterpret_cast<floatx4*>(col + (long)r * B * N + (long)b * N + p) = v;
}

// dx[b, c, h, w] (+)= sum_{i, j valid} dcol[(c*kH + i)*kW + j][b*N + (h - i)*Wo + (w - j)]
// grid (ceil(H*W/256), C, B)
__global__ __launch_bounds__(256) void col2im_kernel(const float* __restrict__ dcol, int B, int C, int H, int W,
                                                     int kH, int kW, int Ho, int Wo, int acc, float* __restrict__ dx) {
  const int hw = blockIdx.x * 256 + threadIdx.x;
  if (hw >= H * W) return;
  const int c = blockIdx.y, b = blockIdx.z;
  const int h = hw / W, w = hw - h * W;
  const long N = (long)Ho * Wo, BN = B * N;
  const float* base = dcol + (long)c * kH * kW * BN + (long)b * N;
  float s = 0.f;
  for (int i = 0; i < kH; ++i) {
    const int oh = h - i;
    if (oh < 0 || oh >= Ho) continue;
    for (int j2 = 0; j2 < kW; ++j2) {
      const int ow = w - j2;
      if (ow < 0 || ow >= Wo) continue;
      s += base[(long)(i * kW + j2) * BN + oh * Wo + ow];
    }
  }
  const long e = ((long)b * C + c) * H * W + hw;
  dx[e] = acc ? dx[e] + s : s;
}

// dyt[c][b*N + p] = dy[b, c, p] * (relu ? 1[y > 0] : 1); grid (ceil(N/256), C, B)
__global__ __launch_bounds__(256) void nchw_to_cbn_kernel(const float* __restrict__ dy, const float* __restrict__ y,
                                                          int relu, int B, int C, int N, float* __restrict__ dyt) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= N) return;
  const int c = blockIdx.y, b = blockIdx.z;
  const long e = ((long)b * C + c) * N + p;
  float v = dy[e];
  if (relu && !(y[e] > 0.f)) v = 0.f;
  dyt[(long)c * B * N + (long)b * N + p] = v;
}

// Row sums in two fixed-order stages: part[r][q] = sum of chunk q of row r (grid (kRowParts, rows)),
// then out[r] = beta*out[r] + alpha * sum_q part[r][q].
constexpr int kRowParts = 64;
__global__ __launch_bounds__(256) void rowsum_part_kernel(const float* __restrict__ X, long ld, long ncols,
                                                          float* __restrict__ part) {
  __shared__ float red[4];
  const long chunk = (ncols + kRowParts - 1) / kRowParts;
  const long j0 = blockIdx.x * chunk, j1 = min(ncols, j0 + chunk);
  const float* row = X + blockIdx.y * ld;
  float s = 0.f;
  for (long j = j0 + threadIdx.x; j < j1; j += 256) s += row[j];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.y * kRowParts + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
__global__ void rowsum_final_kernel(const float* __restrict__ part, int rows, float alpha, float beta,
                                    float* __restrict__ out) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= rows) return;
  float t = 0.f;
  for (int q = 0; q < kRowParts; ++q) t += part[r * kRowParts + q];
  out[r] = (beta == 0.f ? 0.f : beta * out[r]) + alpha * t;
}

// SpatialMaxPooling(kW, kH, dW, dH) on (B*C) planes, floor mode; first maximum in (i, j) scan order
__global__ void smaxpool_fwd_kernel(const float* __restrict__ x, long planes, int H, int W, int kW, int kH, int dW,
                                    int dH, int Ho, int Wo, float* __restrict__ y, int* __restrict__ idx) {
  const long n = planes * Ho * Wo;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int ow = (int)(e % Wo);
    const int oh = (int)((e / Wo) % Ho);
    const long pl = e / ((long)Wo * Ho);
    const float* xp = x + (pl * H + (long)oh * dH) * W + (long)ow * dW;
    float m = xp[0];
    int k = 0;
    for (int i = 0; i < kH; ++i)
      for (int j = 0; j < kW; ++j) {
        const float v = xp[(long)i * W + j];
        if (v > m) {
          m = v;
          k = i * kW + j;
        }
      }
    y[e] = m;
    idx[e] = k;
  }
}

// grid (ceil(H*W/256), B*C): 32-bit index math within a plane
__global__ __launch_bounds__(256) void smaxpool_bwd_kernel(const int* __restrict__ idx, const float* __restrict__ dy,
                                                           int H, int W, int kW, int kH, int dW, int dH, int Ho, int Wo,
                                                           float* __restrict__ dx) {
  const int hw = blockIdx.x * 256 + threadIdx.x;
  if (hw >= H * W) return;
  const long pl = blockIdx.y;
  const int h = hw / W, w = hw - h * W;
  const int* ip = idx + pl * Ho * Wo;
  const float* dp = dy + pl * Ho * Wo;
  float s = 0.f;
  for (int oh = min(h / dH, Ho - 1); oh >= 0 && oh * dH + kH > h; --oh)
    for (int ow = min(w / dW, Wo - 1); ow >= 0 && ow * dW + kW > w; --ow) {
      const int oe = oh * Wo + ow;
      const int k = ip[oe];
      if (oh * dH + k / kW == h && ow * dW + k % kW == w) s += dp[oe];
    }
  dx[pl * H * W + hw] = s;
}

// (B, D1, D2, D3) -> (B, D2, D1, D3)   (Transpose2({1,2},3) with the batch leading; its own inverse
// with D1, D2 exchanged).  e enumerates the output, so the stores are coalesced.
__global__ void swap12_kernel(const float* __restrict__ x, int B, int D1, int D2, int D3, float* __restrict__ y) {
  const long n = (long)B * D1 * D2 * D3;
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) {
    const int k = (int)(e % D3);
    const int j = (int)((e / D3) % D1);          // output dim 2 = input dim 1
    const int i = (int)((e / ((long)D3 * D1)) % D2);  // output dim 1 = input dim 2
    const int b = (int)(e / ((long)D3 * D1 * D2));
    y[e] = x[(((long)b * D1 + j) * D2 + i) * D3 + k];
  }
}

// y = relu(x) ; dx = dy * 1[x > 0]
__global__ void relu_fwd_kernel(const float* __restrict__ x, long n, float* __restrict__ y) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) y[e] = fmaxf(x[e], 0.f);
}
__global__ void relu_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, long n,
                                float* __restrict__ dx) {
  for (long e = blockIdx.x * 256L + threadIdx.x; e < n; e += (long)gridDim.x * 256) dx[e] = x[e] > 0.f ? dy[e] : 0.f;
}

// nn.LogSoftMax (3p) over rows of n: y = x - max - log(sum exp(x - max)); one wave per row
__global__ __launch_bounds__(256) void logsoftmax_fwd_kernel(const float* __restrict__ x, long rows, int n,
                                                             float* __restrict__ y) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  const float* xr = x + r * n;
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) m = fmaxf(m, xr[j]);
  m = wave_max(m);
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += expf(xr[j] - m);
  const float lse = m + logf(wave_sum(s));
  for (int j = lane; j < n; j += 64) y[r * n + j] = xr[j] - lse;
}
// dx = dy - exp(y) * sum(dy)
__global__ __launch_bounds__(256) void logsoftmax_bwd_kernel(const float* __restrict__ y,
                                                             const float* __restrict__ dy, long rows, int n,
                                                             float* __restrict__ dx) {
  const long r = blockIdx.x * 4L + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= rows) return;
  float s = 0.f;
  for (int j = lane; j < n; j += 64) s += dy[r * n + j];
  s = wave_sum(s);
  for (int j = lane; j < n; j += 64) dx[r * n + j] = dy[r * n + j] - expf(y[r * n + j]) * s;
}

inline size_t align256(size_t b) { return (b + 255) / 256 * 256; }

void launch_im2col(hipStream_t st, const float* x, int B, int C, int H, int W, int kH, int kW, int Ho, int Wo,
                   float* col) {
  const long N = (long)Ho * Wo;
  const int K = C * kH * kW;
  if (N % 4 == 0 && (reinterpret_cast<uintptr_t>(col) & 15) == 0)
    hipLaunchKernelGGL(im2col4_kernel, dim3((unsigned)((N / 4 + 255) / 256), K, B), dim3(256), 0, st, x, B, C, H, W,
                       kH, kW, Ho, Wo, col);
  else
    hipLaunchKernelGGL(im2col_kernel, dim3((unsigned)((N + 255) / 256), K, B), dim3(256), 0, st, x, B, C, H, W, kH,
                       kW, Ho, Wo, col);
}

}  // namespace

// ------------------------------------------------------------------ TemporalConvolution
// scratch layout: [split-K slabs | ...]: the weight-gradient GEMMs have few output tiles and a very
// long K (every window / pixel of the batch), so they run split-K
constexpr size_t kWsBytes = sizeof(float) * kGemmWsFloats;
inline GemmWs ws_of(void* scratch) { return GemmWs{static_cast<float*>(scratch), kGemmWsFloats}; }

size_t tconv_scratch_bytes(int B, int L, int Din, int Dout, int kW) {
  return kWsBytes + align256(sizeof(float) * (size_t)B * L * Dout) + align256(sizeof(float) * (size_t)B * L * kW * Din);
}

// A large plain GEMM of the front-end: on the big-tile bf16 kernel under the bf16 modes (gemm_bf16.hip), else
// gemm_f32.
// Problems below ~1 GFLOP stay in-house (launch overhead, and they are not the front-end's time).
static int big_gemm(hipStream_t st, bool tA, bool tB, int M, int N, int K, float alpha, const float* A, long lda,
                    const float* Bm, long ldb, float beta, float* C, long ldc, const float* bias, int relu,
                    GemmWs ws = GemmWs{}) {
  GemmProblem q{A, Bm, C, bias, lda, ldb, ldc, M, N, K, alpha, beta};
  q.relu = relu;
  if (gemm_precision() == kGemmBf16 && 2.0 * M * (double)N * K >= 1e9) {
    bool done = false;
    S2S_TRY(gemm_big_bf16(st, q, tA, tB, &done));
    if (done) return 0;
  }
  return gemm_f32(st, &q, 1, tA, tB, ws);
}

int tconv_fwd(hipStream_t st, int B, int L, int Din, int Dout, int kW, int relu, const float* x, const float* W,
              const float* b, float* y) {
  S2S_REQUIRE(B > 0 && Din > 0 && Dout > 0 && kW > 0, "TemporalConvolution: bad sizes");
  S2S_REQUIRE(L >= kW, "TemporalConvolution: input sequence smaller than kernel size");
  const int Lo = L - kW + 1;
  // kW = 1 (nn.Linear, the VGG model's 1x1 layers): the utterances' rows are one (B L x Din) matrix -- one GEMM
  if (kW == 1 && gemm_precision() == kGemmBf16)
    return big_gemm(st, false, true, B * L, Dout, Din, 1.f, x, Din, W, Din, 0.f, y, Dout, b, relu);
  for (int b0 = 0; b0 < B; b0 += kMaxGemmBatch) {
    GemmProblem pr[kMaxGemmBatch];
    const int nb = std::min(kMaxGemmBatch, B - b0);
    for (int i = 0; i < nb; ++i) {
      const long u = b0 + i;
      pr[i] = GemmProblem{x + u * L * Din, W, y + u * Lo * Dout, b, Din, (long)kW * Din, Dout, Lo, Dout, kW * Din,
                          1.f, 0.f};
      pr[i].relu = relu;
    }
    S2S_TRY(gemm_f32(st, pr, nb, false, true));
  }
  return 0;
}

int tconv_bwd(hipStream_t st, int B, int L, int Din, int Dout, int kW, int relu, const float* x, const float* W,
              const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db, float scale,
              void* scratch, size_t scratch_bytes, hipStream_t wst, hipEvent_t wev) {
  S2S_REQUIRE(L >= kW && B > 0, "TemporalConvolution: bad sizes");
  S2S_REQUIRE(!relu || y, "TemporalConvolution: relu backward needs the forward output");
  S2S_REQUIRE(scratch_bytes >= tconv_scratch_bytes(B, L, Din, Dout, kW), "TemporalConvolution: scratch too small");
  const int Lo = L - kW + 1;
  float* dyp = reinterpret_cast<float*>(static_cast<char*>(scratch) + kWsBytes);
  float* dU = reinterpret_cast<float*>(static_cast<char*>(scratch) + kWsBytes +
                                       align256(sizeof(float) * (size_t)B * L * Dout));
  hipLaunchKernelGGL(tconv_pad_dy, dim3(grid1d((long)B * L * Dout)), dim3(256), 0, st, dy, y, relu, B, L, Lo, Dout,
                     dyp);
  S2S_CHECK_HIP(hipGetLastError());
  const long rows = (long)B * L - kW + 1;  // every window start of the flattened batch
  // the parameter gradients on wst when the caller forks them (they read dyp and x; dx's GEMM below needs no
  // split-K workspace)
  hipStream_t pst = st;
  if ((db || dW) && wst && wst != st && wev) {
    S2S_CHECK_HIP(hipEventRecord(wev, st));
    S2S_CHECK_HIP(hipStreamWaitEvent(wst, wev, 0));
    pst = wst;
  }
  // gradBias += scale * sum_t dY_t ; gradWeight += scale * dY^T [x_t | ... | x_{t+kW-1}]
  if (db) S2S_TRY(colsum_f32(pst, dyp, Dout, B * L, Dout, scale, 1.f, db, ws_of(scratch)));
  if (dW) {
    WgradPrecision wp;  // weight gradient: fp32 under S2S_PREC_BF16_GEMM
    S2S_TRY(big_gemm(pst, true, false, Dout, kW * Din, (int)rows, scale, dyp, Dout, x, Din, 1.f, dW, (long)kW * Din,
                     nullptr, 0, ws_of(scratch)));
  }
  if (dx) {
    S2S_TRY(big_gemm(st, false, false, B * L, kW * Din, Dout, 1.f, dyp, Dout, W, (long)kW * Din, 0.f, dU,
                     (long)kW * Din, nullptr, 0));
    hipLaunchKernelGGL(tconv_gather_dx, dim3(grid1d((long)B * L * Din)), dim3(256), 0, st, dU, B, L, Din, kW,
                       dx_accumulate, dx);
    S2S_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

// ------------------------------------------------------------------ TemporalMaxPooling
int tmaxpool_fwd(hipStream_t st, int B, int L, int D, int kW, int dW, const float* x, float* y, int* idx) {
  S2S_REQUIRE(kW > 0 && dW > 0 && L >= kW, "TemporalMaxPooling: input sequence smaller than kernel size");
  const int Lo = (L - kW) / dW + 1;
  hipLaunchKernelGGL(tmaxpool_fwd_kernel, dim3(grid1d((long)B * Lo * D)), dim3(256), 0, st, x, B, L, D, kW, dW, Lo,
                     y, idx);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int tmaxpool_bwd(hipStream_t st, int B, int L, int D, int kW, int dW, const int* idx, const float* dy, float* dx) {
  S2S_REQUIRE(kW > 0 && dW > 0 && L >= kW, "TemporalMaxPooling: bad sizes");
  const int Lo = (L - kW) / dW + 1;
  hipLaunchKernelGGL(tmaxpool_bwd_kernel, dim3(grid1d((long)B * L * D)), dim3(256), 0, st, idx, dy, B, L, D, kW, dW,
                     Lo, dx);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------ SpatialConvolutionMM
// s2s_debug_sconv_wgrad_implicit(0): the bf16 weight gradient through the im2col panel and the bf16 GEMM (A/B, tests)
std::atomic<int> g_sconv_wgrad_implicit{1};
// scratch: split-K slabs | im2col panel (K, B N) | dcol (K, B N) | dyt (Cout, B N); under bf16 the implicit
// forward / input gradient keep their re-laid-out weights (Cin Cout kH kW) in the panel / dcol region
static size_t sconv_dcol_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW) {
  const size_t K = (size_t)Cin * kH * kW, BN = (size_t)B * (H - kH + 1) * (W - kW + 1);
  return align256(std::max(sizeof(float) * K * BN, sconv_implicit_scratch_bytes(B, Cin, H, W, Cout, kH, kW)));
}
size_t sconv_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW) {
  const size_t N = (size_t)(H - kH + 1) * (W - kW + 1);
  return kWsBytes + 2 * sconv_dcol_bytes(B, Cin, H, W, Cout, kH, kW) +
         align256(sizeof(float) * (size_t)Cout * B * N);
}

int sconv_fwd(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x,
              const float* Wt, const float* bias, float* y, void* scratch, size_t scratch_bytes) {
  S2S_REQUIRE(B > 0 && Cin > 0 && Cout > 0 && kH > 0 && kW > 0, "SpatialConvolutionMM: bad sizes");
  S2S_REQUIRE(H >= kH && W >= kW, "SpatialConvolutionMM: input image smaller than kernel");
  S2S_REQUIRE(scratch_bytes >= sconv_scratch_bytes(B, Cin, H, W, Cout, kH, kW), "SpatialConvolutionMM: scratch too small");
  const int Ho = H - kH + 1, Wo = W - kW + 1;
  const long N = (long)Ho * Wo;
  const int K = Cin * kH * kW;
  S2S_REQUIRE(K <= 65535 && B <= 65535 && (long)B * N < 2147483647L, "SpatialConvolutionMM: sizes exceed the grid");
  // bf16 operands: implicit GEMM straight from x (no im2col panel in HBM)
  float* col = reinterpret_cast<float*>(static_cast<char*>(scratch) + kWsBytes);
  if (gemm_precision() == kGemmBf16 && kH == kW && (kW == 3 || kW == 1))  // re-laid-out weights in the panel region
    return sconv_fwd_implicit(st, B, Cin, H, W, Cout, kH, kW, relu, x, Wt, bias, y, col);
  launch_im2col(st, x, B, Cin, H, W, kH, kW, Ho, Wo, col);
  S2S_CHECK_HIP(hipGetLastError());
  // y_b (Cout, N) = W (Cout, K) col[:, b*N : (b+1)*N] + bias (per row), ReLU in the epilogue
  for (int b0 = 0; b0 < B; b0 += kMaxGemmBatch) {
    GemmProblem pr[kMaxGemmBatch];
    const int nb = std::min(kMaxGemmBatch, B - b0);
    for (int i = 0; i < nb; ++i) {
      const long u = b0 + i;
      pr[i] = GemmProblem{Wt, col + u * N, y + u * Cout * N, nullptr, K, (long)B * N, N, Cout, (int)N, K, 1.f, 0.f};
      pr[i].rbias = bias;
      pr[i].relu = relu;
    }
    S2S_TRY(gemm_f32(st, pr, nb, false, false));
  }
  return 0;
}

int sconv_bwd(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x,
              const float* Wt, const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db,
              float scale, void* scratch, size_t scratch_bytes, int col_from_fwd) {
  S2S_REQUIRE(H >= kH && W >= kW && B > 0, "SpatialConvolutionMM: bad sizes");
  S2S_REQUIRE(!relu || y, "SpatialConvolutionMM: relu backward needs the forward output");
  S2S_REQUIRE(scratch_bytes >= sconv_scratch_bytes(B, Cin, H, W, Cout, kH, kW), "SpatialConvolutionMM: scratch too small");
  const int Ho = H - kH + 1, Wo = W - kW + 1;
  const long N = (long)Ho * Wo, BN = B * N;
  const int K = Cin * kH * kW;
  S2S_REQUIRE(K <= 65535 && B <= 65535 && Cin <= 65535 && Cout <= 65535 && BN < 2147483647L,
              "SpatialConvolutionMM: sizes exceed the grid");
  char* base = static_cast<char*>(scratch) + kWsBytes;
  float* col = reinterpret_cast<float*>(base);
  float* dcol = reinterpret_cast<float*>(base + sconv_dcol_bytes(B, Cin, H, W, Cout, kH, kW));
  float* dyt = reinterpret_cast<float*>(base + 2 * sconv_dcol_bytes(B, Cin, H, W, Cout, kH, kW));
  hipLaunchKernelGGL(nchw_to_cbn_kernel, dim3((unsigned)((N + 255) / 256), Cout, B), dim3(256), 0, st, dy, y, relu, B,
                     Cout, (int)N, dyt);
  S2S_CHECK_HIP(hipGetLastError());
  if (db) {
    // the split-K slab region is free until the dW GEMM below (stream order)
    float* part = static_cast<float*>(scratch);
    hipLaunchKernelGGL(rowsum_part_kernel, dim3(kRowParts, Cout), dim3(256), 0, st, dyt, BN, BN, part);
    hipLaunchKernelGGL(rowsum_final_kernel, dim3((Cout + 255) / 256), dim3(256), 0, st, part, Cout, scale, 1.f, db);
    S2S_CHECK_HIP(hipGetLastError());
  }
  // bf16 forward / input gradient are implicit GEMMs (no panels)
  const bool implicit = gemm_precision() == kGemmBf16 && kH == kW && (kW == 3 || kW == 1);
  if (dW) {
    WgradPrecision wp;  // weight gradient: fp32 under S2S_PREC_BF16_GEMM, bf16 under S2S_PREC_BF16_ALL
    const size_t region = sconv_dcol_bytes(B, Cin, H, W, Cout, kH, kW);
    if (gemm_precision() == kGemmBf16 && implicit && Cin % 64 == 0 && g_sconv_wgrad_implicit) {
      // implicit bf16 weight gradient: the channels-last copy of x in the panel region, split partials in dcol's
      S2S_TRY(sconv_wgrad_implicit(st, B, Cin, H, W, Cout, kH, kW, x, dyt, dW, scale, col, region, dcol, region));
    } else {
      if (!col_from_fwd || implicit)  // else: the forward's im2col panel is still in scratch (same x, same scratch)
        launch_im2col(st, x, B, Cin, H, W, kH, kW, Ho, Wo, col);
      S2S_CHECK_HIP(hipGetLastError());
      // gradWeight (Cout, K) += scale * dyt (Cout, B*N) col^T
      S2S_TRY(gemm1(st, false, true, Cout, K, (int)BN, scale, dyt, BN, col, BN, 1.f, dW, K, nullptr, ws_of(scratch)));
    }
  }
  if (dx && implicit)  // dx = transposed convolution of dyt, the re-laid-out weights in the dcol region
    return sconv_dx_implicit(st, B, Cin, H, W, Cout, kH, kW, Wt, dyt, dx, dx_accumulate, dcol);
  if (dx) {
    // dcol (K, B*N) = W^T dyt ; dx = col2im(dcol)
    S2S_TRY(gemm1(st, true, false, K, (int)BN, Cout, 1.f, Wt, K, dyt, BN, 0.f, dcol, BN));
    hipLaunchKernelGGL(col2im_kernel, dim3((unsigned)((H * W + 255) / 256), Cin, B), dim3(256), 0, st, dcol, B, Cin, H,
                       W, kH, kW, Ho, Wo, dx_accumulate, dx);
    S2S_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

// ------------------------------------------------------------------ SpatialMaxPooling, Transpose2, ReLU
int smaxpool_fwd(hipStream_t st, int B, int C, int H, int W, int kW, int kH, int dW, int dH, const float* x, float* y,
                 int* idx) {
  S2S_REQUIRE(kW > 0 && kH > 0 && dW > 0 && dH > 0 && H >= kH && W >= kW, "SpatialMaxPooling: bad sizes");
  const int Ho = (H - kH) / dH + 1, Wo = (W - kW) / dW + 1;
  const long planes = (long)B * C;
  hipLaunchKernelGGL(smaxpool_fwd_kernel, dim3(grid1d(planes * Ho * Wo)), dim3(256), 0, st, x, planes, H, W, kW, kH,
                     dW, dH, Ho, Wo, y, idx);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int smaxpool_bwd(hipStream_t st, int B, int C, int H, int W, int kW, int kH, int dW, int dH, const int* idx,
                 const float* dy, float* dx) {
  S2S_REQUIRE(kW > 0 && kH > 0 && dW > 0 && dH > 0 && H >= kH && W >= kW, "SpatialMaxPooling: bad sizes");
  const int Ho = (H - kH) / dH + 1, Wo = (W - kW) / dW + 1;
  const long planes = (long)B * C;
  S2S_REQUIRE(planes <= 65535, "SpatialMaxPooling: B*C above the grid's 65535 planes");
  hipLaunchKernelGGL(smaxpool_bwd_kernel, dim3((unsigned)((H * W + 255) / 256), (unsigned)planes), dim3(256), 0, st, idx,
                     dy, H, W, kW, kH, dW, dH, Ho, Wo, dx);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int swap12(hipStream_t st, int B, int D1, int D2, int D3, const float* x, float* y) {
  const long n = (long)B * D1 * D2 * D3;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(swap12_kernel, dim3(grid1d(n)), dim3(256), 0, st, x, B, D1, D2, D3, y);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int relu_fwd(hipStream_t st, long n, const float* x, float* y) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(relu_fwd_kernel, dim3(grid1d(n)), dim3(256), 0, st, x, n, y);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int relu_bwd(hipStream_t st, long n, const float* x, const float* dy, float* dx) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(grid1d(n)), dim3(256), 0, st, x, dy, n, dx);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int logsoftmax_fwd(hipStream_t st, long rows, int n, const float* x, float* y) {
  S2S_REQUIRE(rows >= 0 && n > 0, "LogSoftMax: bad sizes");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(logsoftmax_fwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, x, rows, n, y);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

int logsoftmax_bwd(hipStream_t st, long rows, int n, const float* y, const float* dy, float* dx) {
  S2S_REQUIRE(rows >= 0 && n > 0, "LogSoftMax: bad sizes");
  if (rows == 0) return 0;
  hipLaunchKernelGGL(logsoftmax_bwd_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, st, y, dy, rows, n, dx);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace s2s

extern "C" void s2s_debug_sconv_wgrad_implicit(int on) { s2s::g_sconv_wgrad_implicit = on; }
