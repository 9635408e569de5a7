// Probe for v_mfma_f32_4x4x1_16b_f32 on gfx950: operand / result lane layout and issue cycles against
// v_mfma_f32_16x16x4_f32 (the decoder's skinny products at U = 4 live rows).  Build and run:
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma4_probe tools/mfma4_probe.hip && tools/mfma4_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>

typedef float floatx4 __attribute__((ext_vector_type(4)));

__global__ void layout_kernel(const float* A, const float* B, float* D) {
  const int l = threadIdx.x;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  acc = __builtin_amdgcn_mfma_f32_4x4x1f32(A[l], B[l], acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) D[r * 64 + l] = acc[r];
}

template <int FORM>
__global__ void timing_kernel(const float* X, float* out, long long* cyc) {
  const int l = threadIdx.x;
  float a = X[l], b = X[64 + l];
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < 256; ++i) {
    if (FORM == 0) {
      acc0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, acc1, 0, 0, 0);
    } else {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, acc1, 0, 0, 0);
    }
  }
  const floatx4 s = acc0 + acc1;
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s[0] + s[1] + s[2] + s[3];
  if (l == 0) cyc[0] = t1 - t0;
}


// the production forms: inline asm, W operand from AGPRs, s_nop 1 before each MFMA, two alternating accumulators
template <int FORM>
__global__ void asm_kernel(const float* X, float* out, long long* cyc) {
  const int l = threadIdx.x;
  float a[8], w[8];
  for (int i = 0; i < 8; ++i) { a[i] = X[l] + i; w[i] = X[64 + l] - i; }
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int rep = 0; rep < 32; ++rep) {
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
      if (FORM == 0) {
        asm volatile("s_nop 1\n\tv_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc0) : "v"(a[i]), "a"(w[i]));
        asm volatile("s_nop 1\n\tv_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc1) : "v"(a[i + 1]), "a"(w[i + 1]));
      } else if (FORM == 1) {
        asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc0) : "v"(a[i]), "a"(w[i]));
        asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc1) : "v"(a[i + 1]), "a"(w[i + 1]));
      } else {
        asm volatile("s_nop 1\n\tv_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc0) : "v"(a[i]), "v"(w[i]));
        asm volatile("s_nop 1\n\tv_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc1) : "v"(a[i + 1]), "v"(w[i + 1]));
      }
    }
  }
  asm volatile("s_nop 11" : "+v"(acc0), "+v"(acc1));
  const floatx4 s = acc0 + acc1;
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[l] = s[0] + s[1] + s[2] + s[3];
  if (l == 0) cyc[0] = t1 - t0;
}

int main() {
  float hA[64], hB[64], hD[256];
  for (int l = 0; l < 64; ++l) {
    hA[l] = (float)(l + 1);
    hB[l] = (float)(1000 * (l + 1));
  }
  float *dA, *dB, *dD, *dX, *dO;
  long long* dC;
  hipMalloc(&dA, 256);
  hipMalloc(&dB, 256);
  hipMalloc(&dD, 1024);
  hipMalloc(&dX, 512);
  hipMalloc(&dO, 256);
  hipMalloc(&dC, 8);
  hipMemcpy(dA, hA, 256, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 256, hipMemcpyHostToDevice);
  layout_kernel<<<1, 64>>>(dA, dB, dD);
  hipMemcpy(hD, dD, 1024, hipMemcpyDeviceToHost);
  // assumed: A_b[i][0] at lane 4b + i, B_b[0][j] at lane 4b + j, D_b[i][j] in register i of lane 4b + j
  int bad = 0;
  for (int b = 0; b < 16; ++b)
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        const float want = hA[4 * b + i] * hB[4 * b + j];
        if (hD[i * 64 + 4 * b + j] != want) ++bad;
      }
  printf("4x4x1_16b layout (A lane 4b+i, B lane 4b+j, D reg i lane 4b+j): %s (%d mismatches)\n", bad ? "WRONG" : "ok", bad);
  if (bad)
    for (int l = 0; l < 8; ++l) printf("  lane %d: %g %g %g %g\n", l, hD[l], hD[64 + l], hD[128 + l], hD[192 + l]);
  float hx[128];
  for (int i = 0; i < 128; ++i) hx[i] = 1e-3f * (i % 7);
  hipMemcpy(dX, hx, 512, hipMemcpyHostToDevice);
  for (int form = 0; form < 2; ++form) {
    long long best = 1LL << 60;
    for (int rep = 0; rep < 5; ++rep) {
      if (form == 0) timing_kernel<0><<<1, 64>>>(dX, dO, dC);
      else timing_kernel<1><<<1, 64>>>(dX, dO, dC);
      long long c;
      hipMemcpy(&c, dC, 8, hipMemcpyDeviceToHost);
      if (c < best) best = c;
    }
    printf("%s: %.1f cycles per MFMA (512 in two chains)\n", form == 0 ? "v_mfma_f32_4x4x1_16b_f32" : "v_mfma_f32_16x16x4_f32",
           best / 512.0);
  }
  for (int form = 0; form < 3; ++form) {
    long long best = 1LL << 60;
    for (int rep = 0; rep < 5; ++rep) {
      if (form == 0) asm_kernel<0><<<1, 64>>>(dX, dO, dC);
      else if (form == 1) asm_kernel<1><<<1, 64>>>(dX, dO, dC);
      else asm_kernel<2><<<1, 64>>>(dX, dO, dC);
      long long c;
      hipMemcpy(&c, dC, 8, hipMemcpyDeviceToHost);
      if (c < best) best = c;
    }
    const char* nm[3] = {"asm 4x4x1_16b, W in AGPRs", "asm 16x16x4, W in AGPRs", "asm 4x4x1_16b, W in VGPRs"};
    printf("%s: %.1f cycles per MFMA (256 in two chains, s_nop 1 each)\n", nm[form], best / 256.0);
  }
  return 0;
}
