// Micro-benchmark: one-hop latency of an 8-byte {value, tag} granule hand-off between two
// workgroups, by placement (same XCD / different XCD, read from HW_REG_XCC_ID) and by store /
// load flavour.  Diagnostic only (tools/), not part of the library.
//   hipcc --offload-arch=gfx950 -O3 tools/pingpong.hip -o tools/pingpong && tools/pingpong
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;

template <int ST, int LD>
__device__ __forceinline__ void put(u64* p, u64 v) {
  if (ST == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);      // sc1
  else if (ST == 1) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // plain
  else __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int ST, int LD>
__device__ __forceinline__ u64 get(u64* p) {
  if (LD == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // sc1
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);               // sc0 sc1
}

// blocks a and b ping-pong N times; others exit.  out[0..1] = xcc of a, b; out[2] = ticks (100 MHz)
template <int ST, int LD>
__global__ void pingpong(u64* buf, int a, int b, int n, u64* out, unsigned* fail) {
  const int me = blockIdx.x;
  if ((me != a && me != b) || threadIdx.x != 0) return;
  const unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (3 << 11)) & 15;
  const bool first = me == a;
  out[first ? 0 : 1] = xcc;
  u64* mine = buf + (first ? 0 : 16);   // separate 128-B lines
  u64* theirs = buf + (first ? 16 : 0);
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (int i = 1; i <= n; ++i) {
    if (first) {
      put<ST, LD>(mine, (u64)i << 32);
      unsigned spins = 0;
      while ((unsigned)(get<ST, LD>(theirs) >> 32) != (unsigned)i)
        if (++spins > (1u << 20)) { *fail = 1; return; }
    } else {
      unsigned spins = 0;
      while ((unsigned)(get<ST, LD>(theirs) >> 32) != (unsigned)i)
        if (++spins > (1u << 20)) { *fail = 1; return; }
      put<ST, LD>(mine, (u64)i << 32);
    }
  }
  if (first) out[2] = __builtin_amdgcn_s_memrealtime() - t0;
}

template <int ST, int LD>
void run(const char* name, u64* buf, u64* out, unsigned* fail, int a, int b) {
  const int n = 20000;
  hipMemset(buf, 0, 4096);
  hipMemset(out, 0, 64);
  hipMemset(fail, 0, 4);
  hipLaunchKernelGGL((pingpong<ST, LD>), dim3(64), dim3(64), 0, 0, buf, a, b, n, out, fail);
  hipDeviceSynchronize();
  u64 h[3];
  unsigned f;
  hipMemcpy(h, out, 24, hipMemcpyDeviceToHost);
  hipMemcpy(&f, fail, 4, hipMemcpyDeviceToHost);
  printf("%-22s blocks %2d,%2d xcc %llu,%llu  %s one-hop %.3f us\n", name, a, b, h[0], h[1],
         f ? "FAIL(timeout)" : "ok", h[2] * 10.0 / 1000.0 / (2.0 * n));
}

int main() {
  u64 *buf, *out;
  unsigned* fail;
  hipMalloc(&buf, 4096);
  hipMalloc(&out, 64);
  hipMalloc(&fail, 4);
  for (int rep = 0; rep < 2; ++rep) {
    for (int pair = 0; pair < 2; ++pair) {
      const int a = 0, b = pair == 0 ? 8 : 1;  // 0/8 share an XCD under round-robin, 0/1 do not
      run<0, 0>("sc1 st / sc1 ld", buf, out, fail, a, b);
      run<1, 0>("plain st / sc1 ld", buf, out, fail, a, b);
      run<2, 1>("sys st / sys ld", buf, out, fail, a, b);
      run<1, 1>("plain st / sys ld", buf, out, fail, a, b);
    }
  }
  return 0;
}
