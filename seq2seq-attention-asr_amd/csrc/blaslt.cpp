// Library GEMMs on hipBLASLt for the bf16 operand modes: the encoder front-end's plain dense products (the 1x1
// TemporalConvolution layers of librispeech/model_vgg.lua:45-52 and nn.Linear, M ~ B L' = 8128 rows x 2048 x
// 2048 at config 5).  The operands are rounded to bf16 (RNE, the in-house kernels' rounding) into a staging
// buffer the calling context owns (two elementwise passes), multiplied by hipBLASLt with fp32 accumulation and an
// fp32 result (HIPBLAS_COMPUTE_32F, bias / ReLU in its epilogue).  (The hipBLASLt a process actually runs is the
// one torch loaded -- same soname -- and that build offers no fp32-input HIPBLAS_COMPUTE_32F_FAST_16BF kernels
// for gfx950; /opt/rocm's does: tools/lt_probe.cpp.)  Measured on MI355X at the config-5 shapes: 760-1100
// TFLOP/s for the bf16-input products against ~150 for gemm_bf16_kernel's 64 x 64 tiles.
//
// Row-major C (M x N) = alpha op(A) op(B) + beta C + bias[n], ReLU optional (the GemmProblem contract), is the
// column-major product C^T (N x M) = op(B)^T op(A)^T with the per-column bias as hipBLASLt's per-row bias.
// Plans (descriptor, layouts, the heuristic's first algorithm) are cached per shape and device; every call
// holds one mutex (the bias pointer is a descriptor attribute).  The staging buffer grows outside stream capture
// only (a capture that finds it too small runs the in-house kernel); callers run an eager step before any HIP
// graph capture of these calls (VGGAttentionModel.graph_step does), so plan creation, the staging allocation and
// the library's first kernel loads happen outside capture.
#include <hip/hip_bf16.h>
#include <hipblaslt/hipblaslt.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

#include "s2s_common.h"

namespace s2s {

std::atomic<int> g_gemm_lt{1};  // s2s_debug_gemm_lt(0): the in-house bf16 GEMM instead (A/B, tests)
std::atomic<long> g_lt_calls{0};  // hipBLASLt matmuls launched (s2s_debug_gemm_lt_calls)
std::atomic<int> g_lt_last{0};
std::atomic<int> g_lt_nres{-1};    // diagnostic: last plan failure (1 desc, 2 pref, 3 heuristic status, 4 none, 5 ws)

namespace {

struct LtPlan {
  hipblasLtMatmulDesc_t desc = nullptr;
  hipblasLtMatrixLayout_t a = nullptr, b = nullptr, c = nullptr;
  hipblasLtMatmulAlgo_t algo{};
  bool ok = false;
};
typedef std::tuple<int, int, int, int, int, int, long, long, long, int, size_t> LtKey;

std::mutex g_lt_mu;
hipblasLtHandle_t g_lt_handle[64] = {};
std::map<LtKey, LtPlan> g_lt_plans;

// dst (rows x cols, dense) = RNE bf16 of src (rows x cols, leading dimension ld)
__global__ __launch_bounds__(256) void to_bf16_kernel(const float* __restrict__ src, long ld, long rows, long cols,
                                                      __hip_bfloat16* __restrict__ dst) {
  const long n = rows * cols;
  if (cols % 4 == 0 && ld % 4 == 0) {
    for (long i = 4 * (blockIdx.x * 256L + threadIdx.x); i < n; i += 4L * gridDim.x * 256) {
      const long r = i / cols, c = i - r * cols;
      const float4 v = *reinterpret_cast<const float4*>(src + r * ld + c);
      dst[i] = __float2bfloat16(v.x);
      dst[i + 1] = __float2bfloat16(v.y);
      dst[i + 2] = __float2bfloat16(v.z);
      dst[i + 3] = __float2bfloat16(v.w);
    }
  } else {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
      const long r = i / cols, c = i - r * cols;
      dst[i] = __float2bfloat16(src[r * ld + c]);
    }
  }
}
void to_bf16(hipStream_t st, const float* src, long ld, long rows, long cols, __hip_bfloat16* dst) {
  const long work = (rows * cols + 3) / 4;
  const unsigned blocks = (unsigned)std::min<long>(4096, std::max<long>(1, (work + 255) / 256));
  hipLaunchKernelGGL(to_bf16_kernel, dim3(blocks), dim3(256), 0, st, src, ld, rows, cols, dst);
}

// one handle per device, created once under its own lock (callers may or may not hold g_lt_mu)
std::mutex g_lt_handle_mu;
hipblasLtHandle_t handle_of(int dev) {
  if (dev < 0 || dev >= 64) return nullptr;
  std::lock_guard<std::mutex> lk(g_lt_handle_mu);
  if (!g_lt_handle[dev] && hipblasLtCreate(&g_lt_handle[dev]) != HIPBLAS_STATUS_SUCCESS) g_lt_handle[dev] = nullptr;
  return g_lt_handle[dev];
}

// column-major problem: D (m x n) = op(A') op(B') (+ beta C) (+ bias[row]) [ReLU]
LtPlan* plan_of(int dev, bool ta, bool tb, int m, int n, int k, long lda, long ldb, long ldc, int epi, size_t wsb) {
  const LtKey key{dev, ta, tb, m, n, k, lda, ldb, ldc, epi, wsb};
  auto it = g_lt_plans.find(key);
  if (it != g_lt_plans.end()) return it->second.ok ? &it->second : nullptr;
  LtPlan& p = g_lt_plans[key];
  hipblasLtHandle_t h = handle_of(dev);
  if (!h) return nullptr;
  if (hipblasLtMatmulDescCreate(&p.desc, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) {
    g_lt_last = 1;
    return nullptr;
  }
  const hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  const hipblasLtEpilogue_t e = epi == 3 ? HIPBLASLT_EPILOGUE_RELU_BIAS
                                : epi == 2 ? HIPBLASLT_EPILOGUE_BIAS
                                : epi == 1 ? HIPBLASLT_EPILOGUE_RELU
                                           : HIPBLASLT_EPILOGUE_DEFAULT;
  hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  if (epi >= 2) {
    const hipDataType bt = HIP_R_32F;
    hipblasLtMatmulDescSetAttribute(p.desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt));
  }
  hipblasLtMatrixLayoutCreate(&p.a, HIP_R_16BF, ta ? k : m, ta ? m : k, lda);
  hipblasLtMatrixLayoutCreate(&p.b, HIP_R_16BF, tb ? n : k, tb ? k : n, ldb);
  hipblasLtMatrixLayoutCreate(&p.c, HIP_R_32F, m, n, ldc);
  hipblasLtMatmulPreference_t pref;
  if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) {
    g_lt_last = 2;
    return nullptr;
  }
  const uint64_t wl = wsb;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl));
  hipblasLtMatmulHeuristicResult_t r[8];
  int nr = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, p.desc, p.a, p.b, p.c, p.c, pref, 8, r, &nr);
  g_lt_nres = nr;
  hipblasLtMatmulPreferenceDestroy(pref);
  if (st != HIPBLAS_STATUS_SUCCESS || nr < 1 || r[0].workspaceSize > wsb) {
    g_lt_last = st != HIPBLAS_STATUS_SUCCESS ? 100 + (int)st : nr < 1 ? 4 : 5;
    if (getenv("S2S_LT_VERBOSE"))
      fprintf(stderr, "[s2s lt] no plan: ta %d tb %d m %d n %d k %d lda %ld ldb %ld ldc %ld epi %d ws %zu: status %d nres %d\n",
              (int)ta, (int)tb, m, n, k, lda, ldb, ldc, epi, wsb, (int)st, nr);
    return nullptr;
  }
  p.algo = r[0].algo;
  p.ok = true;
  return &p;
}

}  // namespace

bool gemm_lt_enabled() { return g_gemm_lt != 0; }

int gemm_lt(hipStream_t st, const GemmProblem& q, bool transA, bool transB, GemmWs ws, bool* done) {
  *done = false;
  if (!g_gemm_lt || q.M <= 0 || q.N <= 0 || q.K <= 0 || q.rbias || q.Mread || q.Nread) return 0;
  int dev = 0;
  S2S_CHECK_HIP(hipGetDevice(&dev));
  // C^T (N x M) = op(B)^T op(A)^T: A' = B's buffer, B' = A's buffer (see the header comment)
  const bool ta = transB, tb = transA;
  const int epi = (q.bias ? 2 : 0) + (q.relu ? 1 : 0);
  const size_t wsb = ws.p ? ws.n * sizeof(float) : 0;
  // stored (row-major) shapes of A and B; their bf16 copies are dense (leading dimension = stored columns)
  const long ar = transA ? q.K : q.M, ac = transA ? q.M : q.K, br = transB ? q.N : q.K, bc = transB ? q.K : q.N;
  const size_t abytes = ((size_t)ar * ac * 2 + 255) / 256 * 256, bbytes = (size_t)br * bc * 2;
  std::lock_guard<std::mutex> lk(g_lt_mu);
  LtPlan* p = plan_of(dev, ta, tb, q.N, q.M, q.K, bc, ac, q.ldc, epi, wsb);
  if (!p) return 0;
  char* stage = static_cast<char*>(stage_acquire(st, abytes + bbytes));
  if (!stage) return 0;
  __hip_bfloat16* Ah = reinterpret_cast<__hip_bfloat16*>(stage);
  __hip_bfloat16* Bh = reinterpret_cast<__hip_bfloat16*>(stage + abytes);
  to_bf16(st, q.A, q.lda, ar, ac, Ah);
  to_bf16(st, q.B, q.ldb, br, bc, Bh);
  S2S_CHECK_HIP(hipGetLastError());
  if (q.bias) {
    const void* bp = q.bias;
    hipblasLtMatmulDescSetAttribute(p->desc, HIPBLASLT_MATMUL_DESC_BIAS_POINTER, &bp, sizeof(bp));
  }
  const float alpha = q.alpha, beta = q.beta;
  ProfScope ps(st, "gemm_lt_bf16", 2.0 * q.M * (double)q.N * q.K,
               4.0 * ((double)q.M * q.K + (double)q.K * q.N + (double)q.M * q.N * (beta != 0.f ? 2 : 1)));
  const hipblasStatus_t s = hipblasLtMatmul(handle_of(dev), p->desc, &alpha, Bh, p->a, Ah, p->b, &beta, q.C, p->c,
                                            q.C, p->c, &p->algo, ws.p, wsb, st);
  S2S_REQUIRE(s == HIPBLAS_STATUS_SUCCESS, "hipblasLtMatmul failed");
  *done = true;
  ++g_lt_calls;
  return 0;
}

}  // namespace s2s

extern "C" void s2s_debug_gemm_lt(int on) { s2s::g_gemm_lt = on; }
// diagnostic: hipBLASLt matmuls launched so far, and the last plan failure code (0 = none)
extern "C" long s2s_debug_gemm_lt_calls() { return s2s::g_lt_calls; }
extern "C" int s2s_debug_gemm_lt_last() { return s2s::g_lt_last * 1000 + s2s::g_lt_nres; }
// diagnostic: how many algorithms the in-process hipBLASLt offers for a column-major problem (bf16in: bf16 A / B
// with HIPBLAS_COMPUTE_32F, else fp32 A / B with HIPBLAS_COMPUTE_32F_FAST_16BF; fp32 C / D); -1 on an API error
extern "C" int s2s_debug_lt_avail(int bf16in, int ta, int tb, int m, int n, int k, int epi, unsigned long wsb) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return -1;
  hipblasLtHandle_t h = s2s::handle_of(dev);
  if (!h) return -2;
  hipblasLtMatmulDesc_t desc;
  if (hipblasLtMatmulDescCreate(&desc, bf16in ? HIPBLAS_COMPUTE_32F : HIPBLAS_COMPUTE_32F_FAST_16BF, HIP_R_32F) !=
      HIPBLAS_STATUS_SUCCESS)
    return -3;
  const hipblasOperation_t oa = ta ? HIPBLAS_OP_T : HIPBLAS_OP_N, ob = tb ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &oa, sizeof(oa));
  hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &ob, sizeof(ob));
  const hipblasLtEpilogue_t e = epi == 3 ? HIPBLASLT_EPILOGUE_RELU_BIAS : epi == 2 ? HIPBLASLT_EPILOGUE_BIAS
                                : epi == 1 ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT;
  hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e));
  const hipDataType ti = bf16in ? HIP_R_16BF : HIP_R_32F;
  hipblasLtMatrixLayout_t la, lb, lc;
  hipblasLtMatrixLayoutCreate(&la, ti, ta ? k : m, ta ? m : k, ta ? k : m);
  hipblasLtMatrixLayoutCreate(&lb, ti, tb ? n : k, tb ? k : n, tb ? n : k);
  hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, m, n, m);
  hipblasLtMatmulPreference_t pref;
  hipblasLtMatmulPreferenceCreate(&pref);
  const uint64_t wl = wsb;
  hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl));
  hipblasLtMatmulHeuristicResult_t r[8];
  int nr = 0;
  const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 8, r, &nr);
  hipblasLtMatmulPreferenceDestroy(pref);
  hipblasLtMatrixLayoutDestroy(la);
  hipblasLtMatrixLayoutDestroy(lb);
  hipblasLtMatrixLayoutDestroy(lc);
  hipblasLtMatmulDescDestroy(desc);
  return st == HIPBLAS_STATUS_SUCCESS ? nr : -100 - (int)st;
}

