// Shared internals of libs2s_hip.so (MI355X / gfx950 only).
#pragma once
#include <vector>
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>

namespace s2s {

// test knob (s2s_debug_inject_abort, capi.cpp): 1 when this sync_prep starts its region aborted
int inject_abort_take();

// ---------------------------------------------------------------- errors
// C-ABI calls never abort: they record a message and return nonzero
// (SURVEY.md §8b "Errors": Lua error() on nonzero status).
void set_error(const std::string& msg);
const char* get_error();

#define S2S_CHECK_HIP(expr)                                                                  \
  do {                                                                                       \
    hipError_t _e = (expr);                                                                  \
    if (_e != hipSuccess) {                                                                  \
      ::s2s::set_error(std::string(#expr) + ": " + hipGetErrorString(_e) + " @" __FILE__ ":" \
                       + std::to_string(__LINE__));                                          \
      return 1;                                                                              \
    }                                                                                        \
  } while (0)

#define S2S_REQUIRE(cond, msg)                          \
  do {                                                  \
    if (!(cond)) {                                      \
      ::s2s::set_error(std::string("s2s: ") + (msg));   \
      return 2;                                         \
    }                                                   \
  } while (0)

#define S2S_TRY(expr)          \
  do {                         \
    int _rc = (expr);          \
    if (_rc != 0) return _rc;  \
  } while (0)

// ---------------------------------------------------------------- device helpers
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// The same reductions on DPP lane moves (VALU latency instead of six LDS-crossbar round trips):
// quad, half-row and row mirrors give every lane its 16-lane row's result, then the four rows are
// combined from lanes 0, 16, 32, 48 (v_readlane).  Different association from wave_sum.  Every lane
// of the wave must be active.
template <int CTRL>
__device__ __forceinline__ float dpp_f32(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// packed fp32 pair (v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32: two lanes' worth of fp32 per VALU instruction)
typedef float floatx2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ floatx2 pk_fma(floatx2 a, floatx2 b, floatx2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ floatx2 rcp2(floatx2 a) {
  return floatx2{__builtin_amdgcn_rcpf(a.x), __builtin_amdgcn_rcpf(a.y)};
}
__device__ __forceinline__ float lane_f32(float v, int l) { return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l)); }
__device__ __forceinline__ float wave_sum_dpp(float v) {
  v += dpp_f32<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_f32<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_f32<0x141>(v);  // row_half_mirror
  v += dpp_f32<0x140>(v);  // row_mirror
  return (lane_f32(v, 0) + lane_f32(v, 16)) + (lane_f32(v, 32) + lane_f32(v, 48));
}
// Four wave sums at once, transposed: lane l ends with the wave's sum of value f(l) = 2 (l & 1) + ((l >> 1) & 1) of
// {v0, v1, v2, v3} (lanes 0, 2, 1, 3 hold sums 0, 1, 2, 3).  Halving exchanges with the partners l ^ 1 and l ^ 2
// (quad_perm: each lane keeps one value of the pair it shares with its partner), row rotations by 4 and 8 (the row's
// four lanes of one value), then the rows by v_permlane32_swap / v_permlane16_swap: 7 lane moves and no v_readlane for
// the four sums, instead of 4 x (4 DPP moves + 4 v_readlane + their wait states).  A fixed association (deterministic),
// not wave_sum_dpp's.  Every lane of the wave must be active.
__device__ __forceinline__ float wave_sum4_t(float v0, float v1, float v2, float v3, int lane) {
  const bool b0 = (lane & 1) != 0, b1 = (lane & 2) != 0;
  const float qa = (b0 ? v2 : v0) + dpp_f32<0xB1>(b0 ? v0 : v2);  // quad_perm [1,0,3,2]: partner l ^ 1
  const float qb = (b0 ? v3 : v1) + dpp_f32<0xB1>(b0 ? v1 : v3);
  float r = (b1 ? qb : qa) + dpp_f32<0x4E>(b1 ? qa : qb);  // quad_perm [2,3,0,1]: partner l ^ 2
  r += dpp_f32<0x124>(r);  // row_ror:4
  r += dpp_f32<0x128>(r);  // row_ror:8
  const unsigned u = __float_as_uint(r);
  const auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);  // lanes l and l ^ 32
  const unsigned y = __float_as_uint(__uint_as_float(p[0]) + __uint_as_float(p[1]));
  const auto q = __builtin_amdgcn_permlane16_swap(y, y, false, false);  // rows 2k and 2k + 1
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
// the value index wave_sum4_t leaves in lane l (l < 4: 0 -> 0, 1 -> 2, 2 -> 1, 3 -> 3)
__device__ __forceinline__ int wave_sum4_slot(int lane) { return 2 * (lane & 1) + ((lane >> 1) & 1); }
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f32<0xB1>(v));
  v = fmaxf(v, dpp_f32<0x4E>(v));
  v = fmaxf(v, dpp_f32<0x141>(v));
  v = fmaxf(v, dpp_f32<0x140>(v));
  return fmaxf(fmaxf(lane_f32(v, 0), lane_f32(v, 16)), fmaxf(lane_f32(v, 32), lane_f32(v, 48)));
}

// ---------------------------------------------------------------- big GEMM (gemm_f32.hip)
// Row-major C[M x N] = alpha * op(A) * op(B) + beta * C (+ bias[n] if bias).
//   op(A)(i,k) = transA ? A[k*lda + i] : A[i*lda + k]
//   op(B)(k,j) = transB ? B[j*ldb + k] : B[k*ldb + j]
// beta == 0 overwrites C without reading it.
// Mread / Nread (0 = M / N): rows of op(A) / columns of op(B) that may be READ (zero padding
// the caller guarantees), so tiles straddling M / N can still take the unguarded load path.
struct GemmProblem {
  const float* A;
  const float* B;
  float* C;
  const float* bias;
  long lda, ldb, ldc;
  int M, N, K;
  float alpha, beta;
  int Mread = 0, Nread = 0;
  const float* rbias = nullptr;  // + rbias[row] (per output row, e.g. conv channels in NCHW)
  int relu = 0;                  // epilogue max(v, 0) after bias and beta (fused nn.ReLU)
};
constexpr int kMaxGemmBatch = 16;
// Operand precision of the hoisted GEMMs of the calling thread's current C-ABI call (the context's
// S2S_PREC_*, set at every entry): fp32 (exact f32 MFMA) or bf16 operands with fp32 accumulation.
enum GemmPrecision { kGemmF32 = 0, kGemmBf16 = 1 };
void set_gemm_precision(int p);
int gemm_precision();
// S2S_PREC_BF16_GEMM keeps the weight-gradient GEMMs (and the decoder's weight folds) in fp32: a weight
// gradient is a sum over B*L rows whose terms cancel, and bf16 operand rounding there costs ~5e-2
// normwise at config 3 (measured) against ~1e-3 elsewhere.  The wgrad sites open this scope; under
// S2S_PREC_BF16_ALL (g_wgrad_bf16) it keeps bf16.
void set_wgrad_bf16(bool on);
bool wgrad_bf16();
struct WgradPrecision {
  int prev;
  WgradPrecision() : prev(gemm_precision()) {
    if (!wgrad_bf16()) set_gemm_precision(kGemmF32);
  }
  ~WgradPrecision() { set_gemm_precision(prev); }
};
// A persistent launch's workgroups hand data to each other, so all of them must be resident at once: checked before
// the launch against the occupancy the runtime reports for the kernel, block size and LDS (cached per key) times the
// device's CUs -- a shape or build past that fails loudly here instead of spinning until the hand-off timeout.  (The
// runtime's answer can be one block per CU high at some SGPR counts, MI355X_MICROARCH.md; the grids here stay well
// inside it: one or two workgroups per CU.)
int check_resident(const void* fn, long grid, int block, size_t lds, const char* what);
// A single-problem split-K GEMM issued while a GemmDeferReduce scope is live on this thread leaves its slabs
// unreduced and describes them here (splits = 0: the GEMM wrote C itself); the consumer sums them in slice order
// as splitk_reduce would (C = alpha * sum + bias; alpha = 1, beta = 0, no row bias, no ReLU only) -- the decoder
// MLP's output, read once by the MLP head
struct GemmDeferred {
  const float* part = nullptr;
  int splits = 0;
  long mn = 0;
};
void set_gemm_defer_reduce(GemmDeferred* d);
GemmDeferred* gemm_defer_reduce();
struct GemmDeferReduce {
  GemmDeferred* prev;
  explicit GemmDeferReduce(GemmDeferred* d) : prev(gemm_defer_reduce()) { set_gemm_defer_reduce(d); }
  ~GemmDeferReduce() { set_gemm_defer_reduce(prev); }
};
// Split-K partial-slab workspace (floats).  A call may cut K into slices only when the slabs
// fit; without a workspace every problem runs unsplit.  Concurrent calls need disjoint ones.
struct GemmWs {
  float* p = nullptr;
  size_t n = 0;
};
constexpr size_t kGemmWsFloats = size_t(8) << 20;  // 32 MiB
// All problems of one call share transA/transB.
int gemm_f32(hipStream_t st, const GemmProblem* probs, int nprob, bool transA, bool transB, GemmWs ws = GemmWs{});
// staging buffers for the big bf16 GEMMs' operand copies, owned by a context (grown outside stream capture
// only): one per stream, so calls the caller issues on different streams never share bytes (a buffer is
// reused only in its own stream's order)
struct GemmStage {
  static constexpr int kStreams = 8;
  void* s[kStreams] = {};   // stream of each buffer
  void* p[kStreams] = {};
  size_t n[kStreams] = {};
  std::vector<void*> old;   // outgrown buffers (queued work may still read them): freed with the context
};
void set_gemm_stage(GemmStage* s);  // the calling thread's current context's buffer (set at every C-ABI entry)
void gemm_stage_free(GemmStage* s);
void* stage_acquire(hipStream_t st, size_t bytes);  // that buffer with >= bytes (nullptr: none, or capturing)
// One large problem on the in-house bf16 GEMM (gemm_bf16.hip: operands staged to bf16 in the context's staging
// buffer, 256 x 256 / 128 x 128 MFMA tiles, LDS-DMA staging, split-K slabs).  *done = false (nothing launched)
// when it does not apply (rbias / Mread / Nread, no staging buffer, disabled by s2s_debug_gemm_big(0)).
bool gemm_big_enabled();
int gemm_big_bf16(hipStream_t st, const GemmProblem& q, bool transA, bool transB, bool* done);
// Implicit-GEMM SpatialConvolutionMM on bf16 MFMA (conv_bf16.inc): no im2col panel.  Forward y (B, Cout, Ho,
// Wo) = conv(x) + bias (per channel), ReLU when relu; input gradient dx (B, Cin, H, W) (+)= transposed
// convolution of dyt (Cout, B Ho Wo) -- the ReLU-masked output gradient -- with W.  scratch:
// sconv_implicit_scratch_bytes (the weights in the GEMM's K order and a channels-last bf16 copy of the input).
size_t sconv_implicit_wscratch_bytes(int Cin, int Cout, int kH, int kW);
size_t sconv_implicit_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW);
int sconv_fwd_implicit(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x,
                       const float* Wt, const float* bias, float* y, void* scratch);
int sconv_dx_implicit(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, const float* Wt,
                      const float* dyt, float* dx, int accumulate, void* scratch);
// weight gradient dW (Cout, Cin kH kW) += scale * dyt (Cout, B Ho Wo) x col^T without the im2col panel (bf16
// operands, fp32 accumulation; Cin % 64 == 0): xh_scratch takes the channels-last bf16 copy of x (2 B Cin H W
// bytes), slab the split partial tiles (sconv_wgrad_slab_floats floats)
size_t sconv_wgrad_slab_floats(int B, int Cin, int H, int W, int Cout, int kH, int kW, int* S_out = nullptr,
                               long* chunk_out = nullptr);
int sconv_wgrad_implicit(hipStream_t st, int B, int Cin, int H, int W, int Cout, int kH, int kW, const float* x,
                         const float* dyt, float* dW, float scale, void* xh_scratch, size_t xh_bytes, float* slab,
                         size_t slab_bytes);
inline int gemm1(hipStream_t st, bool tA, bool tB, int M, int N, int K, float alpha, const float* A, long lda,
                 const float* B, long ldb, float beta, float* C, long ldc, const float* bias = nullptr,
                 GemmWs ws = GemmWs{}) {
  GemmProblem p{A, B, C, bias, lda, ldb, ldc, M, N, K, alpha, beta};
  return gemm_f32(st, &p, 1, tA, tB, ws);
}

// Column sums: out[j] = beta*out[j] + alpha * sum_i X[i*ldx + j], i < M, j < N.
// With a workspace (>= 64*N floats) tall sums run in two fixed-order stages over up to 64 row slices
// (many workgroups instead of N/64), same result for any workspace.
int colsum_f32(hipStream_t st, const float* X, long ldx, int M, int N, float alpha, float beta, float* out,
               GemmWs ws = GemmWs{});
// Strided 2-D copy (rows x cols) dst[r*ldd + c] = src[r*lds + c]  (+ optional accumulate).
// Column sums of several column ranges of one matrix in two launches: out_e,q[j] += alpha * sum_rows X[:, col0_e + j]
// for every destination q of range e (bitwise equal to colsum_f32(..., alpha, 1, dst) per range and destination)
struct ColsumOut {
  int col0, ncols;
  float* dst[3];
  int ndst;
};
constexpr int kMaxColsumOuts = 24;
struct ColsumOuts {
  ColsumOut e[kMaxColsumOuts];
};
int colsum_scatter_f32(hipStream_t st, const float* X, long ldx, int M, int N, float alpha, const ColsumOut* outs,
                       int nouts, GemmWs ws);
int copy2d_f32(hipStream_t st, const float* src, long lds, float* dst, long ldd, int rows, int cols, bool accumulate);
// dst[c*ldd + r] = src[r*lds + c] for the rows x cols block
int transpose_f32(hipStream_t st, const float* src, long lds, int rows, int cols, float* dst, long ldd);
// dst (rows x dcols, ld dcols) = src (rows x cols, ld lds) with columns [cols, dcols) zeroed
int pad_cols_f32(hipStream_t st, const float* src, long lds, float* dst, int rows, int cols, int dcols);
// dst[0, bytes) = 0 / count words = value, by a kernel launch: every clear of the library goes through these
// (no hipMemsetAsync: its graph nodes did not replay reliably, gemm_f32.hip)
int zero_async(hipStream_t st, void* dst, size_t bytes);
int fill_u32_async(hipStream_t st, void* dst, unsigned value, size_t count);
// dst[i] = alpha * src[i] + beta * dst[i]
int axpby_f32(hipStream_t st, const float* src, float* dst, size_t n, float alpha, float beta);

// ---------------------------------------------------------------- live kernel timing
// When enabled (s2s_prof_enable) and the stream is not being captured, every launch site
// brackets its kernel with two hipEvents and records the kernel family's ALGORITHMIC flops
// and bytes for that launch; s2s_prof_collect aggregates per family.  Off by default.
bool prof_on();
void prof_begin(hipStream_t st, const char* name, double flops, double bytes);
void prof_end(hipStream_t st);
struct ProfScope {
  hipStream_t st;
  bool on;
  ProfScope(hipStream_t s, const char* name, double flops, double bytes) : st(s), on(prof_on()) {
    if (on) prof_begin(st, name, flops, bytes);
  }
  ~ProfScope() {
    if (on) prof_end(st);
  }
};

// ---------------------------------------------------------------- workspace bump allocator
struct Bump {
  char* base;
  size_t off;
  size_t cap;
  template <class T>
  T* take(size_t n) {
    size_t a = (off + 255) & ~size_t(255);
    T* p = reinterpret_cast<T*>(base ? base + a : nullptr);
    off = a + n * sizeof(T);
    return p;
  }
};

// ---------------------------------------------------------------- optimizer (optim.hip)
size_t optim_state_bytes(size_t n);
int optim_set_noise_step(hipStream_t st, void* state, size_t n, unsigned t);
int optim_state_reset(hipStream_t st, void* state, size_t n);
struct OptimConfig {
  float rho, eps, maxnorm, weightDecay, colnorm_max, gradnoise_eta, gradnoise_gamma;
  unsigned long long gradnoise_seed;
};
int optim_adadelta_step(hipStream_t st, const OptimConfig& c, float* x, float* g, size_t n, void* state,
                        const long* mats, int n_mats, float* gradnorm,
                        const unsigned* status = nullptr, const float* skip_flag = nullptr);
int status_flag(hipStream_t st, const unsigned* status, float* flag);

}  // namespace s2s
