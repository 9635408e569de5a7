// Diagnostic: per-node cost of a chain of dependent kernels in a replayed hipGraph as a function of the
// kernel-argument size (the batched GEMM passes a ~2.3 KB GemmLaunch by value) and of the grid size.
// hipcc --offload-arch=gfx950 -O2 tools/kernarg_bench.hip -o tools/kernarg_bench && tools/kernarg_bench
#include <hip/hip_runtime.h>

#include <cstdio>

template <int N>
struct Args {
  float* out;
  int pad[N];
};

template <int N>
__global__ void tiny(Args<N> a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) a.out[0] += 1.f + a.pad[N - 1];
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      std::printf("%s failed: %s\n", #x, hipGetErrorString(e));          \
      return 1;                                                          \
    }                                                                    \
  } while (0)

template <int N>
int run(float* out, int blocks, int nodes) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Args<N> a{};
  a.out = out;
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < nodes; ++i) hipLaunchKernelGGL(tiny<N>, dim3(blocks), dim3(256), 0, s, a);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e0, s));
  const int reps = 20;
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  // same chain launched eagerly on the stream
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r)
    for (int i = 0; i < nodes; ++i) hipLaunchKernelGGL(tiny<N>, dim3(blocks), dim3(256), 0, s, a);
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms2 = 0.f;
  CK(hipEventElapsedTime(&ms2, e0, e1));
  std::printf("kernarg %5zu B  grid %5d: graph %6.2f us/node   stream %6.2f us/kernel\n", sizeof(Args<N>), blocks,
              1e3 * ms / (reps * nodes), 1e3 * ms2 / (reps * nodes));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return 0;
}

int main() {
  float* out;
  CK(hipMalloc(&out, 64));
  CK(hipMemset(out, 0, 64));
  for (int blocks : {1, 512, 4096}) {
    if (run<2>(out, blocks, 64)) return 1;
    if (run<128>(out, blocks, 64)) return 1;
    if (run<560>(out, blocks, 64)) return 1;
    if (run<1000>(out, blocks, 64)) return 1;
  }
  CK(hipDeviceSynchronize());
  CK(hipFree(out));
  return 0;
}
