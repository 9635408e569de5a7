// Diagnostic: time every GEMM shape of one Chorowski training step (config timit_chorowski_b32)
// through s2s::gemm_f32 and through rocBLAS sgemm, and compare their results.
// Build: make -C tools gemm_bench   Run (GPU box): tools/gemm_bench
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

namespace s2s {
struct GemmProblem {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  long lda, ldb, ldc;
  int M, N, K;
  float alpha, beta;
  int Mread = 0, Nread = 0;  // (mirror of s2s_common.h)
  const float* rbias = nullptr;
  int relu = 0;
};
struct GemmWs {
  float* p = nullptr;
  size_t n = 0;
};
int gemm_f32(hipStream_t st, const GemmProblem* probs, int nprob, bool transA, bool transB, GemmWs ws);
}  // namespace s2s

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

struct Shape {
  int M, N, K;
  float beta;
};
struct Case {
  std::string name;
  bool tA, tB;
  std::vector<Shape> p;
};

static float* dev_rand(size_t n, std::mt19937& g) {
  std::vector<float> h(n);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  for (auto& v : h) v = u(g);
  float* d;
  CK(hipMalloc(&d, n * sizeof(float)));
  CK(hipMemcpy(d, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  return d;
}

int main() {
  const int BL = 32 * 128, R = 32 * 40;
  std::vector<Case> cases = {
      {"xp_l1 NT", false, true, {{BL, 1536, 123, 0.f}}},
      {"xp_l23 NT", false, true, {{BL, 1536, 512, 0.f}}},
      {"Vh NT", false, true, {{BL, 512, 512, 0.f}}},
      {"mlp NT", false, true, {{R, 448, 768, 0.f}}},
      {"dV NN", false, false, {{R, 768, 448, 0.f}}},
      {"dh NN", false, false, {{BL, 512, 512, 1.f}}},
      {"dX NN", false, false, {{BL, 512, 1536, 0.f}}},
      {"attn_wgrad TN", true, false,
       {{62, 64, R, 1.f}, {448, 768, R, 1.f}, {256, 512, R, 1.f}, {256, 512, R, 1.f}, {256, 512, R, 1.f},
        {256, 512, R, 1.f}, {256, 512, R, 1.f}, {256, 62, R, 1.f}, {512, 256, R, 1.f}, {512, 512, BL, 1.f}}},
      {"gru_wgrad_l23 TN", true, false,
       {{256, 256, BL, 1.f}, {256, 512, BL, 1.f}, {256, 256, BL, 1.f}, {256, 512, BL, 1.f}, {256, 256, BL, 1.f},
        {256, 512, BL, 1.f}, {256, 256, BL, 1.f}, {256, 512, BL, 1.f}, {256, 256, BL, 1.f}, {256, 512, BL, 1.f},
        {256, 256, BL, 1.f}, {256, 512, BL, 1.f}}},
      {"gru_wgrad_l1 TN", true, false,
       {{256, 256, BL, 1.f}, {256, 123, BL, 1.f}, {256, 256, BL, 1.f}, {256, 123, BL, 1.f}, {256, 256, BL, 1.f},
        {256, 123, BL, 1.f}, {256, 256, BL, 1.f}, {256, 123, BL, 1.f}, {256, 256, BL, 1.f}, {256, 123, BL, 1.f},
        {256, 256, BL, 1.f}, {256, 123, BL, 1.f}}},
  };
  std::mt19937 g(7);
  hipStream_t st;
  CK(hipStreamCreate(&st));
  rocblas_handle hb;
  rocblas_create_handle(&hb);
  rocblas_set_stream(hb, st);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 20;
  s2s::GemmWs ws;
  ws.n = size_t(8) << 20;
  CK(hipMalloc(&ws.p, ws.n * sizeof(float)));
  double tot_ours = 0, tot_rb = 0;
  std::printf("%-18s %8s %9s %9s %9s %9s %10s\n", "case", "GFLOP", "ours_us", "ours_TF", "rocblas_us", "rb_TF",
              "max_rel");
  for (const Case& c : cases) {
    std::vector<s2s::GemmProblem> pr;
    std::vector<float*> C2;
    std::vector<size_t> csz;
    double fl = 0;
    for (const Shape& s : c.p) {
      const long lda = c.tA ? s.M : s.K, ldb = c.tB ? s.K : s.N, ldc = s.N;
      float* A = dev_rand((size_t)s.M * s.K, g);
      float* B = dev_rand((size_t)s.K * s.N, g);
      float* C = dev_rand((size_t)s.M * s.N, g);
      float* Cr;
      CK(hipMalloc(&Cr, (size_t)s.M * s.N * 4));
      CK(hipMemcpy(Cr, C, (size_t)s.M * s.N * 4, hipMemcpyDeviceToDevice));
      pr.push_back(s2s::GemmProblem{A, B, C, nullptr, lda, ldb, ldc, s.M, s.N, s.K, 1.f, s.beta});
      C2.push_back(Cr);
      csz.push_back((size_t)s.M * s.N);
      fl += 2.0 * s.M * s.N * s.K;
    }
    auto run_ours = [&]() { s2s::gemm_f32(st, pr.data(), (int)pr.size(), c.tA, c.tB, ws); };
    auto run_rb = [&]() {
      for (size_t i = 0; i < pr.size(); ++i) {
        const auto& q = pr[i];
        const float al = q.alpha, be = q.beta;
        // row-major C = op(A) op(B)  <=>  column-major C^T = op(B)^T op(A)^T on the same memory
        rocblas_sgemm(hb, c.tB ? rocblas_operation_transpose : rocblas_operation_none,
                      c.tA ? rocblas_operation_transpose : rocblas_operation_none, q.N, q.M, q.K, &al, q.B, q.ldb,
                      q.A, q.lda, &be, C2[i], q.ldc);
      }
    };
    // correctness on beta = 0 copies (one call each, from equal C)
    run_ours();
    run_rb();
    CK(hipStreamSynchronize(st));
    double mx = 0;
    for (size_t i = 0; i < pr.size(); ++i) {
      std::vector<float> a(csz[i]), b(csz[i]);
      CK(hipMemcpy(a.data(), pr[i].C, csz[i] * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), C2[i], csz[i] * 4, hipMemcpyDeviceToHost));
      double num = 0, den = 0;
      for (size_t j = 0; j < csz[i]; ++j) {
        num = std::fmax(num, std::fabs((double)a[j] - b[j]));
        den = std::fmax(den, std::fabs((double)b[j]));
      }
      mx = std::fmax(mx, num / (den + 1e-30));
    }
    float ms_o = 0, ms_r = 0;
    for (int w = 0; w < 3; ++w) run_ours();
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) run_ours();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms_o, e0, e1));
    for (int w = 0; w < 3; ++w) run_rb();
    CK(hipEventRecord(e0, st));
    for (int r = 0; r < reps; ++r) run_rb();
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms_r, e0, e1));
    const double uo = 1e3 * ms_o / reps, ur = 1e3 * ms_r / reps;
    const int mult = (c.name.rfind("xp_l23", 0) == 0 || c.name.rfind("gru_wgrad_l23", 0) == 0 || c.name.rfind("dX", 0) == 0) ? 2 : 1;
    tot_ours += mult * uo;
    tot_rb += mult * ur;
    std::printf("%-18s %8.2f %9.1f %9.1f %9.1f %9.1f %10.2e  x%d\n", c.name.c_str(), fl / 1e9, uo, fl / uo / 1e6, ur,
                fl / ur / 1e6, mx, mult);
    const char* only = std::getenv("SWEEP_CASE");  // sweep one case by name prefix (default: all)
    if (std::getenv("SWEEP") && (!only || c.name.rfind(only, 0) == 0)) {  // forced plans: tile shape x K slice
      const char* tiles[3] = {"128:128", "128:64", "64:64"};
      int kmax = 0;
      for (const Shape& sh : c.p) kmax = sh.K > kmax ? sh.K : kmax;
      std::vector<int> kss;
      if (const char* l = std::getenv("SWEEP_KS")) {  // "352,416,512": explicit K slices
        for (const char* q = l; *q;) {
          kss.push_back(std::atoi(q));
          while (*q && *q != ',') ++q;
          if (*q == ',') ++q;
        }
      } else {
        for (int ks = 0; ks <= kmax; ks = ks == 0 ? 128 : ks * 2) kss.push_back(ks);
      }
      for (const char* t : tiles) {
        std::printf("    %-8s", t);
        for (int ks : kss) {
          char buf[64];
          std::snprintf(buf, sizeof buf, "%s:%d", t, ks);
          setenv("S2S_GEMM_PLAN", buf, 1);
          for (int w = 0; w < 2; ++w) run_ours();
          CK(hipEventRecord(e0, st));
          for (int r = 0; r < reps; ++r) run_ours();
          CK(hipEventRecord(e1, st));
          CK(hipEventSynchronize(e1));
          float ms = 0;
          CK(hipEventElapsedTime(&ms, e0, e1));
          // one isolated call (the step's tail: nothing queued behind it), averaged over reps
          float iso = 0;
          for (int r = 0; r < reps; ++r) {
            float m1 = 0;
            CK(hipStreamSynchronize(st));
            CK(hipEventRecord(e0, st));
            run_ours();
            CK(hipEventRecord(e1, st));
            CK(hipEventSynchronize(e1));
            CK(hipEventElapsedTime(&m1, e0, e1));
            iso += m1;
          }
          std::printf(" ks%d=%.1f/%.1f", ks, 1e3 * ms / reps, 1e3 * iso / reps);
        }
        std::printf("\n");
      }
      unsetenv("S2S_GEMM_PLAN");
    }
  }
  std::printf("per-step total: ours %.1f us, rocblas %.1f us\n", tot_ours, tot_rb);
  return 0;
}
