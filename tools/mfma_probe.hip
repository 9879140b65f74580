// Probe: verifies the gfx950 bf16 MFMA operand/accumulator lane maps the conv kernels rely on.
// For 16x16x32: lane l holds A[l&15][8*(l>>4)+j], B[8*(l>>4)+j][l&15]; C: col=l&15, row=4*(l>>4)+r.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline short f2bf(float f){ __hip_bfloat16 h = __float2bfloat16(f); return *reinterpret_cast<short*>(&h); }

// A: 16x32 row-major float, B: 32x16 row-major float, C: 16x16 row-major float
__global__ void probe(const float* A, const float* B, float* C){
  int l = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    a[j] = f2bf(A[(l & 15) * 32 + 8 * (l >> 4) + j]);
    b[j] = f2bf(B[(8 * (l >> 4) + j) * 16 + (l & 15)]);
  }
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  for (int r = 0; r < 4; ++r) C[(4 * (l >> 4) + r) * 16 + (l & 15)] = acc[r];
}
extern "C" int run_probe(void* A, void* B, void* C, void* stream){
  hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, (hipStream_t)stream, (const float*)A, (const float*)B, (float*)C);
  return (int)hipGetLastError();
}
