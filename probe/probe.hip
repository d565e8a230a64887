#include <hip/hip_runtime.h>
typedef float f4 __attribute__((ext_vector_type(4)));
// C[16x16] = A[16x4] * B[4x16] with one v_mfma_f32_16x16x4_f32
__global__ void mfma_probe(const float* A, const float* B, float* C) {
  int l = threadIdx.x;
  float a = A[(l & 15) * 4 + (l >> 4)];
  float b = B[(l >> 4) * 16 + (l & 15)];
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[((l >> 4) * 4 + r) * 16 + (l & 15)] = acc[r];
}
extern "C" int probe_mfma(const float* A, const float* B, float* C, void* stream) {
  hipLaunchKernelGGL(mfma_probe, dim3(1), dim3(64), 0, (hipStream_t)stream, A, B, C);
  return (int)hipGetLastError();
}
