// Fused Adam (torch.optim.Adam semantics, coupled L2 weight decay) over the flat fp32 master buffer,
// emitting the bf16 MFMA weight images in the same pass.
//
// Replaces optim.Adam(lr=1e-3, weight_decay=1e-5) of reference utils.py:133-134, which in eager
// PyTorch costs ~1,400 tiny kernels per step for Model A.  Math (per element, step t):
//     g  = grad * grad_scale + wd * p
//     m  = b1 * m + (1 - b1) * g
//     v  = b2 * v + (1 - b2) * g^2
//     p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
// `lr` and the step counter live in device memory, so the reference's LR schedule (lr /= 1.5 every
// validation, utils.py:230-233) and the step count change without re-capturing the HIP graph.
//
// For convolution weights (reference NCHW layout [Co][Ci][KH][KW]) the same thread writes the two
// packed bf16 images consumed by conv.hip: forward [Co][(kh,kw,ci)] and data-gradient
// [Ci][(kh,kw,co)], padded rows/columns stay zero.
#include "kernels.h"

namespace mda {



// Elementwise Adam over the whole flat buffer (padding slots hold p = g = 0 and stay 0).
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a, int64_t n) {
  const float t = a.step[0] + 1.f;
  const float lr = a.lr[0];
  const float c1 = lr / (1.f - powf(a.b1, t));
  const float c2 = 1.f / sqrtf(1.f - powf(a.b2, t));
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 p = reinterpret_cast<float4*>(a.p)[i];
    const float4 g = reinterpret_cast<const float4*>(a.g)[i];
    float4 m = reinterpret_cast<float4*>(a.m)[i];
    float4 v = reinterpret_cast<float4*>(a.v)[i];
    float* pp = &p.x; const float* gg = &g.x; float* mm = &m.x; float* vv = &v.x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float gj = gg[j] * a.grad_scale + a.wd * pp[j];
      mm[j] = a.b1 * mm[j] + (1.f - a.b1) * gj;
      vv[j] = a.b2 * vv[j] + (1.f - a.b2) * gj * gj;
      pp[j] -= c1 * mm[j] / (sqrtf(vv[j]) * c2 + a.eps);
    }
    reinterpret_cast<float4*>(a.p)[i] = p;
    reinterpret_cast<float4*>(a.m)[i] = m;
    reinterpret_cast<float4*>(a.v)[i] = v;
  }
}

// Data-gradient image [Ci][(kh,kw,co)] of one (64 co) x (cit ci) tile of a [Co][Ci][taps] weight, through
// LDS: the reads walk each co's contiguous (ci, tap) run, the writes 16-byte chunks of 8 co -- both
// coalesced.  (The per-element mapping read the masters with a stride of Ci*taps floats: every 4-byte
// value pulled its own cache line, on each of the 8 XCD L2s.)  Padding rows / columns are never written:
// the images are zero-initialised and nothing else writes them.
DEV void pack_dgrad_tile(const float* __restrict__ W, const OptSeg& S, int tile, float (*s_t)[65]) {
  const int taps = S.KH * S.KW;
  const int cit = pack_dgrad_cit(taps);
  const int nci = (S.Ci + cit - 1) / cit;
  const int co0 = (tile / nci) * 64, ci0 = (tile % nci) * cit;
  const int run = min(cit, S.Ci - ci0) * taps;  // contiguous floats per co
  const int nco = min(64, S.Co - co0);
  for (int e = threadIdx.x; e < nco * run; e += 256) {
    const int col = e / run, r = e - col * run;
    s_t[r][col] = W[((int64_t)(co0 + col) * S.Ci + ci0) * taps + r];
  }
  __syncthreads();
  for (int item = threadIdx.x; item < run * 8; item += 256) {
    const int r = item >> 3, ch = item & 7;
    if (ch * 8 >= nco) continue;
    const int ci = ci0 + r / taps, tap = r % taps;
    uint32_t w4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
      w4[j] = (uint32_t)f2bf(s_t[r][ch * 8 + 2 * j]) | ((uint32_t)f2bf(s_t[r][ch * 8 + 2 * j + 1]) << 16);
    *reinterpret_cast<uint4*>(S.wd + (int64_t)ci * S.Kpad_d + tap * (S.tap_ld ? S.tap_ld : S.Co) + co0 + ch * 8) =
        make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

// Forward image [Co][(kh,kw,ci)] of rb consecutive co rows (one contiguous span of the [Co][Ci][taps]
// masters) through LDS: the span is read coalesced, each 16-byte store packs 8 channels of one tap (Cs and
// Kpad_f are multiples of 8) read from LDS with a stride of taps floats (odd for every conv of the models:
// conflict-free).  The direct per-chunk mapping read the masters with a stride of taps floats per lane and
// was address-unit bound.  Padding rows (co >= Co) are never written (zero-initialised images).
DEV void pack_fwd_rows_block(const float* __restrict__ W, const OptSeg& S, int blk, float* s_w) {
  const int taps = S.KH * S.KW, row = S.Ci * taps;
  const int rb = pack_fwd_rows(S.Ci, taps, S.Co);
  const int co0 = blk * rb, nr = min(rb, S.Co - co0);
  const float* src = W + (int64_t)co0 * row;
  for (int e = threadIdx.x; e < nr * row; e += 256) s_w[e] = src[e];
  __syncthreads();
  const int K8 = (S.kext_f ? S.kext_f : S.Kpad_f) >> 3;
  for (int item = threadIdx.x; item < nr * K8; item += 256) {
    const int r = item / K8, k0 = (item - r * K8) * 8;
    const int tap = k0 / S.Cs, ci0 = k0 - tap * S.Cs;
    const float* w = s_w + r * row + ci0 * taps + tap;
    uint32_t w4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x0 = (tap < taps && ci0 + 2 * j < S.Ci) ? w[(2 * j) * taps] : 0.f;
      const float x1 = (tap < taps && ci0 + 2 * j + 1 < S.Ci) ? w[(2 * j + 1) * taps] : 0.f;
      w4[j] = (uint32_t)f2bf(x0) | ((uint32_t)f2bf(x1) << 16);
    }
    *reinterpret_cast<uint4*>(S.wf + (int64_t)(co0 + r) * S.Kpad_f + k0) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
  }
}

// Writes the packed bf16 MFMA images of every conv weight.  Segment `kind` selects the image:
// 1 = forward [Co][(kh,kw,ci)] (rows Npad, cols Kpad_f): one block per pack_fwd_rows co rows
// (pack_fwd_rows_block); 2 = data-gradient [Ci][(kh,kw,co)]: one block per LDS-transposed tile
// (pack_dgrad_tile).
// `step` (non-null after an Adam update): the step counter is advanced here -- the pack runs after the
// Adam kernel that read it, so the separate one-thread launch is not needed.
__global__ __launch_bounds__(256) void pack_kernel(const float* __restrict__ P, const OptSeg* __restrict__ segs, int ns,
                                                   float* step) {
  __shared__ float s_t[PACK_ROWS][65];
  const int bx = (int)blockIdx.x;
  static_assert(PACK_ROWS * 65 >= PACK_FWD_FLOATS, "pack_fwd_rows_block stages its rows in s_t");
  if (step && blockIdx.x == 0 && threadIdx.x == 0) step[0] += 1.f;
  int lo = 0, hi = ns - 1;
  while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (segs[mid].block0 <= (int64_t)bx) lo = mid; else hi = mid - 1; }
  const OptSeg& S = segs[lo];
  const int blk = (int)((int64_t)bx - S.block0);
  if (S.kind == 2) pack_dgrad_tile(P + S.off, S, blk, s_t);
  else pack_fwd_rows_block(P + S.off, S, blk, &s_t[0][0]);
}

__global__ void step_inc_kernel(float* step) { step[0] += 1.f; }

int launch_adam_pack(const AdamArgs& a, const OptSeg* d_segs, int ns, int64_t nblocks, hipStream_t st) {
  if (a.update) {
    const int64_t n4 = a.n >> 2;
    const int blocks = (int)std::min<int64_t>((n4 + 255) / 256, 2048);
    hipLaunchKernelGGL(adam_kernel, dim3(blocks), dim3(256), 0, st, a, a.n);
    int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  float* step = a.update ? const_cast<float*>(a.step) : nullptr;
  if (nblocks > 0)
    hipLaunchKernelGGL(pack_kernel, dim3((unsigned)nblocks), dim3(256), 0, st, (const float*)a.p, d_segs, ns, step);
  int rc = (int)hipGetLastError();
  if (rc || !a.update || nblocks > 0) return rc;
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step);
  return (int)hipGetLastError();
}

}  // namespace mda
