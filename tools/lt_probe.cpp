// Probe: hipBLASLt bf16 GEMMs at the config-5 1x1-layer shape (D = op(A) op(B), column-major m x n x k).
//   (a) fp32 A/B/C/D with HIPBLAS_COMPUTE_32F_FAST_16BF (conversion inside the library)
//   (b) bf16 A/B, fp32 C/D, HIPBLAS_COMPUTE_32F
// Reports whether a heuristic exists, the time per call, and the error against a float64 product of
// RNE-bf16-rounded operands on a sampled set of outputs.
// hipcc --offload-arch=gfx950 -O2 tools/lt_probe.cpp -lhipblaslt -o tools/lt_probe && tools/lt_probe
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hipblaslt/hipblaslt.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    auto e_ = (x);                                                             \
    if ((int)e_ != 0) { std::printf("error %d at %s:%d\n", (int)e_, __FILE__, __LINE__); std::exit(1); } \
  } while (0)

static float bf16r(float f) {
  unsigned u;
  std::memcpy(&u, &f, 4);
  u = (u + 0x7fffu + ((u >> 16) & 1u)) & 0xffff0000u;
  std::memcpy(&f, &u, 4);
  return f;
}

static int run(hipblasLtHandle_t h, bool bf16in, int opA, int opB, int m, int n, int k, const char* tag,
               bool f32compute = false) {
  std::mt19937 g(7);
  std::normal_distribution<float> nd;
  const int ra = opA ? k : m, ca = opA ? m : k, rb = opB ? n : k, cb = opB ? k : n;
  std::vector<float> A((size_t)ra * ca), B((size_t)rb * cb);
  for (auto& v : A) v = nd(g);
  for (auto& v : B) v = nd(g);
  void *dA, *dB, *dD, *ws;
  const size_t esz = bf16in ? 2 : 4, wsb = 64 << 20;
  CK(hipMalloc(&dA, A.size() * esz));
  CK(hipMalloc(&dB, B.size() * esz));
  CK(hipMalloc(&dD, (size_t)m * n * 4));
  CK(hipMalloc(&ws, wsb));
  if (bf16in) {
    std::vector<__hip_bfloat16> a(A.size()), b(B.size());
    for (size_t i = 0; i < A.size(); ++i) a[i] = __float2bfloat16(A[i]);
    for (size_t i = 0; i < B.size(); ++i) b[i] = __float2bfloat16(B[i]);
    CK(hipMemcpy(dA, a.data(), a.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, b.data(), b.size() * 2, hipMemcpyHostToDevice));
  } else {
    CK(hipMemcpy(dA, A.data(), A.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dB, B.data(), B.size() * 4, hipMemcpyHostToDevice));
  }
  const hipDataType ti = bf16in ? HIP_R_16BF : HIP_R_32F;
  hipblasLtMatmulDesc_t desc;
  CK(hipblasLtMatmulDescCreate(&desc, (bf16in || f32compute) ? HIPBLAS_COMPUTE_32F : HIPBLAS_COMPUTE_32F_FAST_16BF,
                                HIP_R_32F));
  hipblasOperation_t ta = opA ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = opB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  hipblasLtMatrixLayout_t la, lb, lc;
  CK(hipblasLtMatrixLayoutCreate(&la, ti, ra, ca, ra));
  CK(hipblasLtMatrixLayoutCreate(&lb, ti, rb, cb, rb));
  CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, m, n, m));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wl = wsb;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int nres = 0;
  auto st = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 8, res, &nres);
  if (st != HIPBLAS_STATUS_SUCCESS || nres == 0) {
    std::printf("%s: no algorithm (status %d, %d results)\n", tag, (int)st, nres);
    return 1;
  }
  float alpha = 1.f, beta = 0.f;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e30f;
  int bi = 0;
  for (int r = 0; r < nres; ++r) {
    for (int w = 0; w < 3; ++w)
      CK(hipblasLtMatmul(h, desc, &alpha, dA, la, dB, lb, &beta, dD, lc, dD, lc, &res[r].algo, ws, wsb, 0));
    CK(hipEventRecord(e0, 0));
    for (int w = 0; w < 20; ++w)
      CK(hipblasLtMatmul(h, desc, &alpha, dA, la, dB, lb, &beta, dD, lc, dD, lc, &res[r].algo, ws, wsb, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= 20;
    if (ms < best) { best = ms; bi = r; }
  }
  CK(hipblasLtMatmul(h, desc, &alpha, dA, la, dB, lb, &beta, dD, lc, dD, lc, &res[bi].algo, ws, wsb, 0));
  std::vector<float> D((size_t)m * n);
  CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
  double emax = 0, rmax = 0, eexact = 0;
  for (int s = 0; s < 2000; ++s) {
    const int i = (int)(g() % m), j = (int)(g() % n);
    double ref = 0, ex = 0;
    for (int q = 0; q < k; ++q) {
      const float a = opA ? A[(size_t)i * ra + q] : A[(size_t)q * ra + i];
      const float b = opB ? B[(size_t)q * rb + j] : B[(size_t)j * rb + q];
      ref += (double)bf16r(a) * bf16r(b);
      ex += (double)a * b;
    }
    emax = std::fmax(emax, std::fabs(D[(size_t)j * m + i] - ref));
    eexact = std::fmax(eexact, std::fabs(D[(size_t)j * m + i] - ex));
    rmax = std::fmax(rmax, std::fabs(ref));
  }
  const double tf = 2.0 * m * n * k / (best * 1e-3) / 1e12;
  std::printf("%s: %d algos, best %.3f ms = %.0f TF/s; err vs rounded-operand f64 %.2e, vs exact f64 %.2e (of max %.1f)\n",
              tag, nres, best, tf, emax / rmax, eexact / rmax, rmax);
  hipFree(dA); hipFree(dB); hipFree(dD); hipFree(ws);
  return 0;
}

// heuristic availability of fp32-in FAST_16BF for an epilogue / workspace / transpose combination
static void avail(hipblasLtHandle_t h, int opA, int opB, int m, int n, int k, int epi, size_t wsb) {
  hipblasLtMatmulDesc_t desc;
  CK(hipblasLtMatmulDescCreate(&desc, HIPBLAS_COMPUTE_32F_FAST_16BF, HIP_R_32F));
  hipblasOperation_t ta = opA ? HIPBLAS_OP_T : HIPBLAS_OP_N, tb = opB ? HIPBLAS_OP_T : HIPBLAS_OP_N;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSA, &ta, sizeof(ta)));
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_TRANSB, &tb, sizeof(tb)));
  const hipblasLtEpilogue_t e = epi == 3 ? HIPBLASLT_EPILOGUE_RELU_BIAS : epi == 2 ? HIPBLASLT_EPILOGUE_BIAS
                                : epi == 1 ? HIPBLASLT_EPILOGUE_RELU : HIPBLASLT_EPILOGUE_DEFAULT;
  CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_EPILOGUE, &e, sizeof(e)));
  if (epi >= 2) {
    const hipDataType bt = HIP_R_32F;
    CK(hipblasLtMatmulDescSetAttribute(desc, HIPBLASLT_MATMUL_DESC_BIAS_DATA_TYPE, &bt, sizeof(bt)));
  }
  hipblasLtMatrixLayout_t la, lb, lc;
  CK(hipblasLtMatrixLayoutCreate(&la, HIP_R_32F, opA ? k : m, opA ? m : k, opA ? k : m));
  CK(hipblasLtMatrixLayoutCreate(&lb, HIP_R_32F, opB ? n : k, opB ? k : n, opB ? n : k));
  CK(hipblasLtMatrixLayoutCreate(&lc, HIP_R_32F, m, n, m));
  hipblasLtMatmulPreference_t pref;
  CK(hipblasLtMatmulPreferenceCreate(&pref));
  uint64_t wl = wsb;
  CK(hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wl, sizeof(wl)));
  hipblasLtMatmulHeuristicResult_t res[8];
  int nres = 0;
  auto st = hipblasLtMatmulAlgoGetHeuristic(h, desc, la, lb, lc, lc, pref, 8, res, &nres);
  std::printf("avail op%c%c m %d n %d k %d epi %d ws %zu MB: status %d, %d algos\n", opA ? 'T' : 'N', opB ? 'T' : 'N',
              m, n, k, epi, wsb >> 20, (int)st, nres);
}

int main() {
  hipblasLtHandle_t h;
  CK(hipblasLtCreate(&h));
  if (getenv("LT_F32")) {  // exact fp32 (HIPBLAS_COMPUTE_32F) at the config-2 step's critical-path shapes
    run(h, false, 1, 0, 448, 1280, 768, "f32 MLP u = v Wm^T      (T,N)", true);
    run(h, false, 1, 0, 512, 4096, 512, "f32 Vh = h V^T          (T,N)", true);
    run(h, false, 0, 1, 384, 256, 4096, "f32 wgrad dW_g (N,T)        ", true);
    run(h, false, 0, 0, 768, 1280, 448, "f32 dv = du Wm          (N,N)", true);
    return 0;
  }
  if (getenv("LT_AVAIL")) {
    for (int epi = 0; epi < 4; ++epi)
      for (size_t ws : {(size_t)0, (size_t)32 << 20}) {
        avail(h, 1, 0, 2048, 2032, 896, epi, ws);
        avail(h, 1, 0, 2048, 8128, 2048, epi, ws);
      }
    avail(h, 0, 0, 2048, 2032, 2048, 0, 0);
    avail(h, 0, 1, 896, 2048, 2032, 0, 32 << 20);
    avail(h, 0, 1, 896, 2048, 2032, 0, 0);
    return 0;
  }
  // forward 1x1 layer: y^T (Dout x R) = W^T_cm^T x^T : m = 2048, n = 8128, k = 2048, opA = T, opB = N
  run(h, false, 1, 0, 2048, 8128, 2048, "fp32 in, FAST_16BF, fwd  (T,N)");
  run(h, true, 1, 0, 2048, 8128, 2048, "bf16 in, 32F,       fwd  (T,N)");
  // dx: m = Din, n = R, k = Dout, (N,N)
  run(h, false, 0, 0, 2048, 8128, 2048, "fp32 in, FAST_16BF, dx   (N,N)");
  run(h, true, 0, 0, 2048, 8128, 2048, "bf16 in, 32F,       dx   (N,N)");
  // dW: m = Din, n = Dout, k = R, (N,T)
  run(h, false, 0, 1, 2048, 2048, 8128, "fp32 in, FAST_16BF, dW   (N,T)");
  run(h, true, 0, 1, 2048, 2048, 8128, "bf16 in, 32F,       dW   (N,T)");
  return 0;
}
