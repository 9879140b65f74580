// Latency calibration for MI355X: kernel floor inside a graph, dependent global-load latency (L2 hit
// vs. HBM), and the cost of 1024-thread blocks.  Built by tools/latency_probe.py with hipcc.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void k_empty() {}

__global__ void k_copy(const float* __restrict__ x, float* __restrict__ y, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = x[i] * 2.f;
}

// one thread follows `hops` dependent pointers; stride chooses L2-resident (small ring) or HBM (big)
__global__ void k_chase(const int* __restrict__ nxt, int hops, int* out) {
  int p = 0;
  for (int h = 0; h < hops; ++h) p = __builtin_nontemporal_load(nxt + p);
  out[0] = p;
}

__global__ void k_chase_cached(const int* __restrict__ nxt, int hops, int* out) {
  int p = 0;
  for (int h = 0; h < hops; ++h) p = nxt[p];
  out[0] = p;
}

extern "C" {
int launch_empty(int blocks, int threads, hipStream_t st) {
  hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(threads), 0, st);
  return (int)hipGetLastError();
}
int launch_copy(const float* x, float* y, int n, int threads, hipStream_t st) {
  hipLaunchKernelGGL(k_copy, dim3((n + threads - 1) / threads), dim3(threads), 0, st, x, y, n);
  return (int)hipGetLastError();
}
int launch_chase(const int* nxt, int hops, int* out, int cached, hipStream_t st) {
  if (cached) hipLaunchKernelGGL(k_chase_cached, dim3(1), dim3(1), 0, st, nxt, hops, out);
  else hipLaunchKernelGGL(k_chase, dim3(1), dim3(1), 0, st, nxt, hops, out);
  return (int)hipGetLastError();
}
}
