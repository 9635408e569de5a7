// Optimizer step on the flat parameter / gradient buffers, fused on the device:
// what timit/timit.lua:292-347 does after the backward, minus the host round trips --
//   gradient clipping on the global norm       (timit.lua:297-302: if ||g|| > maxnorm: g *= maxnorm/||g||)
//   L2 regularisation                          (timit.lua:305-308: g += weightDecay * x)
//   gradient noise                             (timit.lua:310-315: t += 1; g += N(0, 1) * sqrt(eta / (1+t)^gamma))
//   optim.adadelta (3p, rho / eps config)      (timit.lua:179, exp_logmel7_chorowski_normNLL_colnorm.lua:32-33)
//   TrainUtils.columnNormConstraint(maxval)    (timit.lua:344-346, TrainUtils.lua:52-104) on every weight matrix
// The 1/B normalisation (timit.lua:292-295) is the model step's `scale`.
//
// HBM-bound elementwise work: the norm is a two-pass deterministic reduction (fixed per-block
// order, then one block over the partials), the update one pass reading x, g, v, u and writing
// x, g, v, u (32 B per parameter), the constraint one wave per weight row.  No host sync: the clip
// factor, the noise counter t and sigma stay on the device, so a captured graph replays them.
// The reference draws the noise with torch.randn; here it is a counter-based normal of (seed, t, i)
// (splitmix64 -> Box-Muller), so any launch geometry -- and every data-parallel rank, which all hold
// the same all-reduced gradients -- draws the same noise.
#include "s2s_common.h"

#include <algorithm>

namespace s2s {

namespace {

constexpr int kNormBlocks = 512;
constexpr int kMaxMats = 64;

struct OptState {
  float* v;        // optim.adadelta paramVariance
  float* u;        // optim.adadelta accDelta
  float* partial;  // [kNormBlocks] sums of squares
  float* scal;     // [0] ||g||, [1] clip factor, [2] noise sigma, [3] noise counter t (uint32 bits),
                   // [4] nonzero: skip this update (the context's failure status was set, see opt_finalize)
};

OptState carve_state(void* state, size_t n) {
  char* p = static_cast<char*>(state);
  const size_t nn = (n + 63) / 64 * 64;
  OptState s;
  s.v = reinterpret_cast<float*>(p);
  s.u = s.v + nn;
  s.partial = s.u + nn;
  s.scal = s.partial + kNormBlocks;
  return s;
}

__global__ __launch_bounds__(256) void opt_sumsq(const float* __restrict__ g, size_t n, float* partial) {
  __shared__ float red[4];
  float s = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) s += g[i] * g[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) partial[blockIdx.x] = ((red[0] + red[1]) + red[2]) + red[3];
}

constexpr unsigned long long kGolden = 0x9e3779b97f4a7c15ull;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// N(0, 1) for element i of the step keyed by mix64(seed * kGolden + t): u1 in (0, 1], u2 in [0, 1)
// from 24-bit fields of mix64(key + i * kGolden), z = sqrt(-2 ln u1) cos(2 pi u2)
// (oracle/s2s_oracle.py: gradient_noise restates it)
__device__ __forceinline__ float noise_normal(unsigned long long key, size_t i) {
  const unsigned long long h = mix64(key + (unsigned long long)i * kGolden);
  const float u1 = (float)((h >> 40) + 1) * (1.0f / 16777216.0f);
  const float u2 = (float)((h >> 16) & 0xffffffull) * (1.0f / 16777216.0f);
  return sqrtf(-2.f * logf(u1)) * cosf(6.28318530717958647692f * u2);
}

// status: the context's failure words (handoff.h; host-coherent, written by the step's harvest kernel earlier
// on this stream).  A set word means a persistent launch of an earlier step timed out and its gradients are
// invalid: the whole update is skipped on the device (parameters, state and noise counter untouched), so calls
// already queued in program order behind the failed step cannot apply them before the host gate sees it.
// skip_flag (optional): a device float, nonzero = skip as well -- data parallel: every rank's failure flag
// (s2s_ctx_status_flag) summed over the ranks, so a failure on ANY rank (whose invalid gradients went into the
// all-reduce) makes every replica skip the same update and the replicas stay identical.
__global__ __launch_bounds__(256) void opt_finalize(const float* partial, int nb, float maxnorm, float eta,
                                                    float gamma, float* scal, float* gradnorm_out,
                                                    const unsigned* status, const float* skip_flag) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < nb; i += 256) s += partial[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    const bool skip = (status && ((__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) |
                                   __hip_atomic_load(status + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != 0u)) ||
                      (skip_flag && *skip_flag != 0.f);
    scal[4] = skip ? 1.f : 0.f;
    const float gn = sqrtf(((red[0] + red[1]) + red[2]) + red[3]);
    if (gradnorm_out) *gradnorm_out = gn;
    if (skip) return;
    scal[0] = gn;
    scal[1] = gn > maxnorm ? maxnorm / gn : 1.f;
    if (eta != 0.f) {  // gradnoise.t = (gradnoise.t or 0) + 1; sigma = (eta / (1 + t)^gamma)^0.5
      const unsigned t = __float_as_uint(scal[3]) + 1u;
      scal[3] = __uint_as_float(t);
      scal[2] = (float)sqrt((double)eta / pow(1.0 + (double)t, (double)gamma));
    }
  }
}

// optim.adadelta (3p):  v = rho v + (1-rho) g^2;  std = sqrt(v + eps);
//   delta = sqrt(u + eps) / std * g;  x -= delta;  u = rho u + (1-rho) delta^2
__global__ __launch_bounds__(256) void opt_adadelta(float* __restrict__ x, float* __restrict__ g,
                                                    float* __restrict__ v, float* __restrict__ u, size_t n,
                                                    const float* scal, float rho, float eps, float wd,
                                                    int noise, unsigned long long seed) {
  if (scal[4] != 0.f) return;
  const float clip = scal[1];
  const float sigma = noise ? scal[2] : 0.f;
  const unsigned long long key = noise ? mix64(seed * kGolden + __float_as_uint(scal[3])) : 0ull;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += 256ull * gridDim.x) {
    float gi = g[i];
    if (clip != 1.f) gi = gi * clip;
    const float xi = x[i];
    if (wd != 0.f) gi = gi + wd * xi;
    if (noise) gi = gi + noise_normal(key, i) * sigma;
    const float vi = v[i] * rho + (1.f - rho) * (gi * gi);
    const float sd = sqrtf(vi + eps);
    const float ui = u[i];
    const float delta = sqrtf(ui + eps) / sd * gi;
    x[i] = xi - delta;
    v[i] = vi;
    u[i] = ui * rho + (1.f - rho) * (delta * delta);
    g[i] = gi;  // the reference clips / decays `gradients` in place
  }
}

struct MatTable {
  long off[kMaxMats];
  int rows[kMaxMats], cols[kMaxMats], first[kMaxMats + 1];  // first[m] = global index of matrix m's row 0
  int n;
};

// TrainUtils.columnNormConstraint: norm_r = ||W_r||_2 + 1e-8 over each output row (W:norm(2,2));
// rows with norm >= maxval are divided by norm / maxval, the others kept.  One wave per row.
__global__ __launch_bounds__(256) void opt_colnorm(float* __restrict__ x, MatTable t, float maxval,
                                                   const float* scal) {
  if (scal[4] != 0.f) return;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= t.first[t.n]) return;
  int m = 0;
  while (row >= t.first[m + 1]) ++m;
  const int r = row - t.first[m], cols = t.cols[m];
  float* w = x + t.off[m] + (long)r * cols;
  float s = 0.f;
  for (int c = lane; c < cols; c += 64) s += w[c] * w[c];
  s = wave_sum(s);
  const float norm = sqrtf(s) + 1e-8f;
  if (norm < maxval) return;
  const float div = norm / maxval;
  for (int c = lane; c < cols; c += 64) w[c] = w[c] / div;
}

}  // namespace

size_t optim_state_bytes(size_t n) {
  const size_t nn = (n + 63) / 64 * 64;
  return sizeof(float) * (2 * nn + kNormBlocks + 64);
}

int optim_adadelta_step(hipStream_t st, const OptimConfig& c, float* x, float* g, size_t n, void* state,
                        const long* mats, int n_mats, float* gradnorm, const unsigned* status,
                        const float* skip_flag) {
  const float rho = c.rho, eps = c.eps, wd = c.weightDecay, colnorm_max = c.colnorm_max;
  const int noise = c.gradnoise_eta != 0.f;
  S2S_REQUIRE(x && g && state && n > 0, "optim: null argument");
  S2S_REQUIRE(colnorm_max <= 0.f || (mats && n_mats > 0 && n_mats <= kMaxMats), "optim: bad weight-matrix table");
  const OptState s = carve_state(state, n);
  const int nb = (int)std::min<size_t>(kNormBlocks, (n + 255) / 256);
  hipLaunchKernelGGL(opt_sumsq, dim3(nb), dim3(256), 0, st, g, n, s.partial);
  hipLaunchKernelGGL(opt_finalize, dim3(1), dim3(256), 0, st, s.partial, nb, c.maxnorm, c.gradnoise_eta,
                     c.gradnoise_gamma, s.scal, gradnorm, status, skip_flag);
  const int ne = (int)std::min<size_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(opt_adadelta, dim3(ne), dim3(256), 0, st, x, g, s.v, s.u, n, s.scal, rho, eps, wd, noise,
                     c.gradnoise_seed);
  if (colnorm_max > 0.f) {
    MatTable t{};
    t.n = n_mats;
    t.first[0] = 0;
    for (int m = 0; m < n_mats; ++m) {
      t.off[m] = mats[3 * m];
      t.rows[m] = (int)mats[3 * m + 1];
      t.cols[m] = (int)mats[3 * m + 2];
      S2S_REQUIRE(t.off[m] >= 0 && t.rows[m] > 0 && t.cols[m] > 0 &&
                      (size_t)t.off[m] + (size_t)t.rows[m] * t.cols[m] <= n,
                  "optim: weight matrix outside the flat buffer");
      t.first[m + 1] = t.first[m] + t.rows[m];
    }
    hipLaunchKernelGGL(opt_colnorm, dim3((t.first[n_mats] + 3) / 4), dim3(256), 0, st, x, t, colnorm_max, s.scal);
  }
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// flag[0] = 1 if the context's failure words are set when this runs on the stream, else 0 (stream-ordered)
__global__ __launch_bounds__(64) void status_flag_kernel(const unsigned* status, float* flag) {
  if (threadIdx.x == 0)
    flag[0] = ((__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) |
                __hip_atomic_load(status + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) != 0u) ? 1.f : 0.f;
}
int status_flag(hipStream_t st, const unsigned* status, float* flag) {
  hipLaunchKernelGGL(status_flag_kernel, dim3(1), dim3(64), 0, st, status, flag);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}

// the gradient-noise counter t (gradnoise.t, timit.lua:312) of a state: a resumed trainer sets it from its
// checkpointed table; stream-ordered, no sync (the next step increments it before drawing)
int optim_set_noise_step(hipStream_t st, void* state, size_t n, unsigned t) {
  const OptState s = carve_state(state, n);
  S2S_TRY(fill_u32_async(st, s.scal + 3, t, 1));
  return 0;
}

// zero paramVariance / accDelta (optim.adadelta's lazily created state) and the noise counter t
int optim_state_reset(hipStream_t st, void* state, size_t n) {
  S2S_TRY(zero_async(st, state, optim_state_bytes(n)));
  return 0;
}

}  // namespace s2s
