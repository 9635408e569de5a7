// Per-time-step "skinny" products of the recurrences: out[b][n] = sum_k X[b][k] * W[n][k]
// with b the utterance (batch) row -- B is 32..64, so the step GEMM is (B x K) x (K x N).
//
// One workgroup = 4 waves computes a 16 (batch rows) x 16 (units) tile; K is split
// across the 4 waves (16-wide chunks round-robin), each wave runs
// v_mfma_f32_16x16x4_f32 (exact f32) on float4 operand loads (lane l holds rows
// l&15 and k-quad l>>4; element e of the float4 feeds MFMA e, the same
// permutation of k on both operands), and the 4 partial tiles are summed through
// LDS in a fixed order.  Thread tid of the workgroup then owns output
// (row tid>>4, unit tid&15) for the fused epilogue.
#pragma once
#include "s2s_common.h"

namespace s2s {

struct SkinnyRed {
  float v[4][16][17];
};

// xrow / wrow: this lane's operand rows (already offset to the lane's batch row /
// output unit); both 16-byte aligned; K % 16 == 0.
__device__ __forceinline__ floatx4 skinny_wave(const float* __restrict__ xrow, const float* __restrict__ wrow,
                                               int K, int wave, int lane) {
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int kq = 4 * (lane >> 4);
  int kc = wave * 16;
  for (; kc + 64 < K; kc += 128) {
    const float4 a0 = *reinterpret_cast<const float4*>(xrow + kc + kq);
    const float4 b0 = *reinterpret_cast<const float4*>(wrow + kc + kq);
    const float4 a1 = *reinterpret_cast<const float4*>(xrow + kc + 64 + kq);
    const float4 b1 = *reinterpret_cast<const float4*>(wrow + kc + 64 + kq);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc1, 0, 0, 0);
  }
  for (; kc < K; kc += 64) {
    const float4 a0 = *reinterpret_cast<const float4*>(xrow + kc + kq);
    const float4 b0 = *reinterpret_cast<const float4*>(wrow + kc + kq);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc0, 0, 0, 0);
  }
  return acc0 + acc1;
}

// Writes this wave's partial tile and returns (after the barrier) the summed value
// of output (tid>>4, tid&15).  Must be called by all 256 threads.
__device__ __forceinline__ float skinny_reduce(SkinnyRed& red, floatx4 acc, int wave, int lane, int tid) {
#pragma unroll
  for (int r = 0; r < 4; ++r) red.v[wave][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  const int i = tid >> 4, j = tid & 15;
  return ((red.v[0][i][j] + red.v[1][i][j]) + red.v[2][i][j]) + red.v[3][i][j];
}

// 8-wave form (512-thread workgroup) for the per-step kernels whose K is long (the LSTM decoder's gate and carry
// products, K = 2S / 4S): 16-wide chunks round-robin over 8 waves (stride 128), twice the loads in flight per
// workgroup; the 8 partial tiles are summed in wave order (a different order from skinny_wave's 4).
struct SkinnyRed8 {
  float v[8][16][17];
};
__device__ __forceinline__ floatx4 skinny_wave8(const float* __restrict__ xrow, const float* __restrict__ wrow, int K,
                                                int wave, int lane) {
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const int kq = 4 * (lane >> 4);
  int kc = wave * 16;
  for (; kc + 128 < K; kc += 256) {
    const float4 a0 = *reinterpret_cast<const float4*>(xrow + kc + kq);
    const float4 b0 = *reinterpret_cast<const float4*>(wrow + kc + kq);
    const float4 a1 = *reinterpret_cast<const float4*>(xrow + kc + 128 + kq);
    const float4 b1 = *reinterpret_cast<const float4*>(wrow + kc + 128 + kq);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.x, b1.x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.y, b1.y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.z, b1.z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1.w, b1.w, acc1, 0, 0, 0);
  }
  for (; kc < K; kc += 128) {
    const float4 a0 = *reinterpret_cast<const float4*>(xrow + kc + kq);
    const float4 b0 = *reinterpret_cast<const float4*>(wrow + kc + kq);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.x, b0.x, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.y, b0.y, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.z, b0.z, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0.w, b0.w, acc0, 0, 0, 0);
  }
  return acc0 + acc1;
}
// all 512 threads call it; threads 0..255 get output (tid>>4, tid&15), the others 0
__device__ __forceinline__ float skinny_reduce8(SkinnyRed8& red, floatx4 acc, int wave, int lane, int tid) {
#pragma unroll
  for (int r = 0; r < 4; ++r) red.v[wave][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  if (tid >= 256) return 0.f;
  const int i = tid >> 4, j = tid & 15;
  float s = red.v[0][i][j];
#pragma unroll
  for (int w = 1; w < 8; ++w) s += red.v[w][i][j];
  return s;
}

// Four skinny products (gates q = 0..3 of the same 16 units) in one 1024-thread workgroup: waves 4q .. 4q + 3
// split gate q's K exactly as skinny_wave's four waves do, so s[q] (returned to threads 0..255 for output
// (tid>>4, tid&15)) is bitwise the skinny_reduce of that product -- four times the loads in flight per
// workgroup of a four-launch (or four-product serial) form.  wrow(q) = this lane's weight row of gate q.
template <typename WRow>
__device__ __forceinline__ void skinny4_1024(SkinnyRed (&red)[4], const float* __restrict__ xrow, WRow wrow, int K,
                                             bool zero, float (&s)[4]) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, q = wave >> 2, w4 = wave & 3;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
  if (!zero) acc = skinny_wave(xrow, wrow(q), K, w4, lane);
#pragma unroll
  for (int r = 0; r < 4; ++r) red[q].v[w4][4 * (lane >> 4) + r][lane & 15] = acc[r];
  __syncthreads();
  if (tid < 256) {
    const int i = tid >> 4, j = tid & 15;
#pragma unroll
    for (int g = 0; g < 4; ++g) s[g] = ((red[g].v[0][i][j] + red[g].v[1][i][j]) + red[g].v[2][i][j]) + red[g].v[3][i][j];
  }
}

}  // namespace s2s
