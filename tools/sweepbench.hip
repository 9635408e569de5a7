// Micro-benchmark of one GRU seam in an XCD-local chain (diagnostic only, not part of the library).
// NMEM member workgroups of one chain sit on one XCD (blockIdx = 8 * member + xcd-slot); every step each
// member publishes its 16 x 16 tile of fp32 values into a sentinel slot (plain stores, kSent = all-ones
// pre-filled) and then sweeps the 16 rows x H values of that slot the way gru_persist does (4 waves, each its
// K-quarter, 16-byte loads, poll until no word is kSent).  One seam per step: step time = publication ->
// visibility + the sweep.  Variants isolate what a sweep costs:
//   extra  : each thread issues X extra global stores (the saved activations / dA of the real kernel) between
//            its publication and its sweep (vmcnt counts stores and loads together, in order)
//   policy : load cache policy bits of the sweep (0 plain, 1 sc0, 16 sc1)
//   chains : chains on other XCDs running the same loop at the same time
//   hbm    : workgroups on the remaining XCDs streaming HBM reads (the fused GEMM producers)
//   tile   : tile-major slot layout [member][16 rows][16 cols]: every 128-B line has ONE writer and a wave's
//            load instruction reads 1 KB contiguous (8 whole lines) instead of 64 B from each of 16 rows
//   ready  : additionally sweep slot s - 2 (complete for long) before slot s: the cost of a pass alone
//   hipcc --offload-arch=gfx950 -O3 tools/sweepbench.hip -o tools/sweepbench && tools/sweepbench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr unsigned kSent = 0xffffffffu;

template <int NC>
__device__ __forceinline__ bool sweep(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long row_off, int wave, int lane,
                                      int policy, unsigned& polls) {
  const long kq = 4 * (lane >> 4);
  while (true) {
    ++polls;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = row_off + 4 * (wave * 16 + 64 * i + kq);
      uint4 p;
      if (policy == 16) p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      else if (policy == 1) p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 1));
      else p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
      ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
      a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
    }
    if (__all(ok)) return true;
    if (polls > (1u << 22)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

// tile-major sweep that re-polls only the chunks (= producers) not yet complete; sleep = s_sleep between passes
template <int NC>
__device__ __forceinline__ bool sweep_tile_sel(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long s, int H, int wave,
                                               int lane, int sleep, unsigned& polls) {
  unsigned pending = (1u << NC) - 1;  // wave-uniform
  while (true) {
    ++polls;
    uint4 p[NC];
#pragma unroll
    for (int i = 0; i < NC; ++i)
      if (pending & (1u << i)) {
        const long off = 4 * (s * 16 * H + (long)(wave + 4 * i) * 256 + (lane & 15) * 16 + 4 * (lane >> 4));
        p[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      }
#pragma unroll
    for (int i = 0; i < NC; ++i)
      if (pending & (1u << i)) {
        const bool ok = p[i].x != kSent && p[i].y != kSent && p[i].z != kSent && p[i].w != kSent;
        if (__all(ok)) {
          pending &= ~(1u << i);
          a[i] = make_float4(__uint_as_float(p[i].x), __uint_as_float(p[i].y), __uint_as_float(p[i].z),
                             __uint_as_float(p[i].w));
        }
      }
    if (!pending) return true;
    if (polls > (1u << 22)) return false;
    if (sleep) __builtin_amdgcn_s_sleep(1);
  }
}

// the same sweep over the tile-major layout: chunk i of wave w is member (w + 4 i)'s tile; lane l reads its row
// l & 15, columns 4 (l >> 4) .. + 3 of that tile = 16 contiguous bytes at (row * 16 + 4 (l >> 4)) of the 1-KB tile
template <int NC>
__device__ __forceinline__ bool sweep_tile(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long s, int H, int wave,
                                           int lane, int policy, unsigned& polls) {
  while (true) {
    ++polls;
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = 4 * (s * 16 * H + (long)(wave + 4 * i) * 256 + (lane & 15) * 16 + 4 * (lane >> 4));
      uint4 p;
      if (policy == 16) p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      else p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 0));
      ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
      a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
    }
    if (__all(ok)) return true;
    if (polls > (1u << 22)) return false;
    __builtin_amdgcn_s_sleep(1);
  }
}

struct Args {
  float* slots;   // [nchains][L][16][H]
  float* sink;    // extra stores land here ([grid][L][256][X])
  const float* hbm;  // streamed by the hbm workgroups
  long hbm_n;
  int L, H, nmem, nchains, extra, policy, hbm_wgs, tile, ready;
  unsigned long long* out;  // [nchains][nmem] ticks; [.. + 1] polls
  unsigned* fail;
};

template <int NC>
__global__ __launch_bounds__(256) void seam_kernel(Args a) {
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  const int chain = x, member = j;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (chain >= a.nchains || member >= a.nmem) {
    // HBM streamers: the chain-free slots read a large buffer until the chains finish (bounded loop)
    if (a.hbm_wgs && (chain >= a.nchains) && member < a.hbm_wgs) {
      float s = 0.f;
      const long stride = (long)gridDim.x * 256;
      for (int rep = 0; rep < 64; ++rep)
        for (long i = (long)blockIdx.x * 256 + tid; i < a.hbm_n; i += stride) s += a.hbm[i];
      if (s == 12345.f) a.fail[1] = 1;
    }
    return;
  }
  const int H = a.H, L = a.L;
  float* base = a.slots + (long)chain * L * 16 * H;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, 0x7fffffff, 0x00020000);
  const int r = tid >> 4, c = member * 16 + (tid & 15);
  // element (row, col) of slot s: row-major [16][H], or tile-major [H / 16][16][16]
  auto at = [&](long s, int row, int col) -> long {
    return a.tile >= 1 ? s * 16 * H + (long)(col >> 4) * 256 + row * 16 + (col & 15) : (s * 16 + row) * H + col;
  };
  float v = 1.f + tid;
  unsigned polls = 0;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  for (int s = 0; s < L; ++s) {
    // publish this member's tile of slot s (plain store: stays in this XCD's L2)
    __hip_atomic_store(reinterpret_cast<unsigned*>(base + at(s, r, c)), __float_as_uint(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_WORKGROUP);
    for (int e = 0; e < a.extra; ++e)
      a.sink[(((long)blockIdx.x * L + s) * a.extra + e) * 256 + tid] = v;
    float4 av[NC];
    if (a.ready && s >= 2) {
      float4 bv[NC];
      unsigned dummy = 0;
      if (a.tile) sweep_tile<NC>(bv, rs, s - 2, H, wave, lane, a.policy, dummy);
      else sweep<NC>(bv, rs, 4L * ((long)(s - 2) * 16 + (lane & 15)) * H, wave, lane, a.policy, dummy);
      v += bv[0].x * 1e-12f;
    }
    const bool got = a.tile >= 2 ? sweep_tile_sel<NC>(av, rs, s, H, wave, lane, a.tile == 2, polls)
                     : a.tile ? sweep_tile<NC>(av, rs, s, H, wave, lane, a.policy, polls)
                              : sweep<NC>(av, rs, 4L * ((long)s * 16 + (lane & 15)) * H, wave, lane, a.policy, polls);
    if (!got) {
      a.fail[0] = 1;
      return;
    }
    float acc = 0.f;
#pragma unroll
    for (int i = 0; i < NC; ++i) acc += av[i].x + av[i].y + av[i].z + av[i].w;
    v = acc * 1e-9f + 1.f;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (tid == 0) {
    a.out[2 * (chain * a.nmem + member)] = t1 - t0;
    a.out[2 * (chain * a.nmem + member) + 1] = polls;
  }
}

int main() {
  const int L = 512;
  float *slots, *sink, *hbm;
  unsigned long long* out;
  unsigned* fail;
  const long hbm_n = 64L << 20;
  hipMalloc(&slots, sizeof(float) * 8L * L * 16 * 512);
  hipMalloc(&sink, sizeof(float) * 8L * 64 * L * 4 * 256);
  hipMalloc(&hbm, sizeof(float) * hbm_n);
  hipMemset(hbm, 0, sizeof(float) * hbm_n);
  hipMalloc(&out, 8 * 1024);
  hipMalloc(&fail, 8);
  struct Case {
    const char* name;
    int H, extra, policy, nchains, hbm, tile, ready;
  };
  std::vector<Case> cases = {
      {"H256 row-major (the GRU seam)", 256, 0, 16, 1, 0, 0, 0},
      {"H256 row-major + ready sweep", 256, 0, 16, 1, 0, 0, 1},
      {"H256 tile-major", 256, 0, 16, 1, 0, 1, 0},
      {"H256 tile-major + ready sweep", 256, 0, 16, 1, 0, 1, 1},
      {"H256 tile, re-poll failed chunks", 256, 0, 16, 1, 0, 2, 0},
      {"H256 tile, re-poll failed, no sleep", 256, 0, 16, 1, 0, 3, 0},
      {"H256 tile, re-poll, 4 ch + HBM", 256, 0, 16, 4, 1, 2, 0},
      {"H256 tile-major + 3 stores", 256, 3, 16, 1, 0, 1, 0},
      {"H256 tile-major, 4 ch + HBM", 256, 0, 16, 4, 1, 1, 0},
      {"H128 row-major", 128, 0, 16, 1, 0, 0, 0},
      {"H128 tile-major", 128, 0, 16, 1, 0, 1, 0},
      {"H64 row-major", 64, 0, 16, 1, 0, 0, 0},
      {"H64 tile-major", 64, 0, 16, 1, 0, 1, 0},
  };
  for (const Case& k : cases) {
    const int nmem = k.H / 16;
    hipMemset(slots, 0xff, sizeof(float) * 8L * L * 16 * 512);
    hipMemset(out, 0, 8 * 1024);
    hipMemset(fail, 0, 8);
    Args a{slots, sink, hbm, hbm_n, L, k.H, nmem, k.nchains, k.extra, k.policy, k.hbm ? 16 : 0, k.tile, k.ready,
           out, fail};
    const int grid = 8 * 32;
    if (k.H == 256) hipLaunchKernelGGL(seam_kernel<4>, dim3(grid), dim3(256), 0, 0, a);
    else if (k.H == 128) hipLaunchKernelGGL(seam_kernel<2>, dim3(grid), dim3(256), 0, 0, a);
    else hipLaunchKernelGGL(seam_kernel<1>, dim3(grid), dim3(256), 0, 0, a);
    if (hipDeviceSynchronize() != hipSuccess) {
      printf("%s: launch failed\n", k.name);
      return 1;
    }
    std::vector<unsigned long long> h(2 * 8 * 32);
    unsigned f[2];
    hipMemcpy(h.data(), out, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost);
    hipMemcpy(f, fail, 8, hipMemcpyDeviceToHost);
    double tmax = 0, pol = 0;
    int n = 0;
    for (int c = 0; c < k.nchains; ++c)
      for (int m = 0; m < nmem; ++m) {
        tmax = std::max(tmax, (double)h[2 * (c * nmem + m)]);
        pol += (double)h[2 * (c * nmem + m) + 1];
        ++n;
      }
    printf("%-32s step %.3f us  (%.2f poll passes per sweep)%s\n", k.name, tmax * 0.01 / L, pol / n / L,
           f[0] ? "  TIMEOUT" : "");
  }
  return 0;
}
