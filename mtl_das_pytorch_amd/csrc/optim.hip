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
// For convolution weights (reference NCHW layout [Co][Ci][KH][KW]) the same block writes the two
// packed bf16 images consumed by conv.hip: forward [Co][(kh,kw,ci)] and data-gradient
// [Ci][(kh,kw,co)]; padded rows / columns are zero-initialised and never written.
#include "kernels.h"

namespace mda {



constexpr int PACK_U = 8;

DEV float adam_update(const AdamArgs& a, float p, float g, float& m, float& v, float c1, float c2) {
  const float gj = g * a.grad_scale + a.wd * p;
  m = a.b1 * m + (1.f - a.b1) * gj;
  v = a.b2 * v + (1.f - a.b2) * gj * gj;
  return p - c1 * m / (sqrtf(v) * c2 + a.eps);
}

// One launch for the whole optimizer step.  Block -> segment by binary search over the segments' first
// blocks:
//   kind 0: a plain range of the flat buffer (BN affine parameters, the fully connected layers, padding),
//           1024 elements per block, Adam only;
//   kind 3: a (8 co) x (tci ci) x (all taps) tile of a conv weight [Co][Ci][taps]: its masters, gradients and
//           moments are read once (each co's (ci, tap) run is contiguous), updated, written back, and the
//           updated values staged in LDS feed BOTH packed bf16 images -- forward [Co][(tap, ci)] (16-byte
//           stores of 8 ci of one tap) and data-gradient [Ci][(tap, co)] (8 co of one tap).  A tile is ~2K elements: one round of PACK_U loads per thread.
// The separate Adam and pack kernels read the masters twice and cost two dependent launches (Model A:
// ~28 us on the step's tail for 1.1 M parameters; Model C 97 + 64 us).  Every flat element belongs to
// exactly one segment (engine/core.py build_optseg_table checks the cover).  update == 0: pack only.
// Every block reads the step counter; a one-thread kernel advances it afterwards (a last-block-done counter
// instead -- one atomic per block on a single address -- serialised ~0.2 us per block: Model C's ~8.7 K
// blocks took 1.7 ms).
__global__ __launch_bounds__(256) void adam_pack_kernel(AdamArgs a, const OptSeg* __restrict__ segs, int ns) {
  __shared__ float s_w[PACK_TCO * (PACK_TILE_FLOATS + 1)];
  const int bx = (int)blockIdx.x;
  int lo = 0, hi = ns - 1;
  while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (segs[mid].block0 <= (int64_t)bx) lo = mid; else hi = mid - 1; }
  const OptSeg& S = segs[lo];
  const int blk = (int)((int64_t)bx - S.block0);
  float c1 = 0.f, c2 = 0.f;
  if (a.update) {
    const float t = a.step[0] + (a.t_pre ? 0.f : 1.f);
    c1 = a.lr[0] / (1.f - powf(a.b1, t));
    c2 = 1.f / sqrtf(1.f - powf(a.b2, t));
  }
  if (S.kind == 0) {
    if (a.update) {
      const int64_t e0 = S.off + (int64_t)blk * 1024 + threadIdx.x, end = S.off + S.n;
      float p[4], g[4], m[4], v[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {  // all loads in flight before the first use
        const int64_t e = e0 + 256 * k;
        if (e < end) { p[k] = a.p[e]; g[k] = a.g[e]; m[k] = a.m[e]; v[k] = a.v[e]; }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t e = e0 + 256 * k;
        if (e < end) {
          a.p[e] = adam_update(a, p[k], g[k], m[k], v[k], c1, c2);
          a.m[e] = m[k];
          a.v[e] = v[k];
        }
      }
    }
  } else {
    const int taps = S.KH * S.KW;
    const int tci = pack_tile_ci(taps);
    const int nci_t = (S.Ci + tci - 1) / tci;
    const int co0 = (blk / nci_t) * PACK_TCO, ci0 = (blk % nci_t) * tci;
    const int nci = min(tci, S.Ci - ci0), nco = min(PACK_TCO, S.Co - co0);
    const int run = nci * taps, ld = tci * taps + 1;  // contiguous floats per co; LDS row pitch
    // PACK_U elements per thread per round, all loads issued before the first use: a round is one memory
    // round trip (a dependent load -> update -> store loop per element was latency-bound, 4x slower)
    for (int e0 = threadIdx.x; e0 < nco * run; e0 += 256 * PACK_U) {
      float p[PACK_U], g[PACK_U], m[PACK_U], v[PACK_U];
      int64_t idx[PACK_U];
      int lds[PACK_U];
#pragma unroll
      for (int u = 0; u < PACK_U; ++u) {
        const int e = e0 + 256 * u;
        const int col = e / run, r = e - col * run;
        idx[u] = S.off + ((int64_t)(co0 + col) * S.Ci + ci0) * taps + r;
        lds[u] = col * ld + r;
        if (e < nco * run) {
          p[u] = a.p[idx[u]];
          if (a.update) { g[u] = a.g[idx[u]]; m[u] = a.m[idx[u]]; v[u] = a.v[idx[u]]; }
        }
      }
#pragma unroll
      for (int u = 0; u < PACK_U; ++u) {
        if (e0 + 256 * u >= nco * run) break;
        if (a.update) {
          p[u] = adam_update(a, p[u], g[u], m[u], v[u], c1, c2);
          a.p[idx[u]] = p[u];
          a.m[idx[u]] = m[u];
          a.v[idx[u]] = v[u];
        }
        s_w[lds[u]] = p[u];
      }
    }
    __syncthreads();
    const int ng = (nci + 7) >> 3;  // 8-ci groups (ci past Ci write the zero padding of the Cs columns)
    const int fcol = S.kext_f ? S.kext_f : taps * S.Cs;  // forward-image columns this weight owns
    for (int item = threadIdx.x; item < nco * taps * ng; item += 256) {
      const int co = item / (taps * ng), rem = item - co * (taps * ng);
      const int tap = rem / ng, gi = rem - tap * ng;
      const int k0 = tap * S.Cs + ci0 + gi * 8;
      if (k0 >= fcol) continue;
      uint32_t w4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c0 = gi * 8 + 2 * j;
        const float x0 = c0 < nci ? s_w[co * ld + c0 * taps + tap] : 0.f;
        const float x1 = c0 + 1 < nci ? s_w[co * ld + (c0 + 1) * taps + tap] : 0.f;
        w4[j] = (uint32_t)f2bf(x0) | ((uint32_t)f2bf(x1) << 16);
      }
      *reinterpret_cast<uint4*>(S.wf + (int64_t)(co0 + co) * S.Kpad_f + k0) = make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
    const int nh = (nco + 7) >> 3;  // 8-co groups (co past Co: zeros into the padding columns)
    const int tld = S.tap_ld ? S.tap_ld : S.Co;
    for (int item = threadIdx.x; item < nci * taps * nh; item += 256) {
      const int ci = item / (taps * nh), rem = item - ci * (taps * nh);
      const int tap = rem / nh, h = rem - tap * nh;
      uint32_t w4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c0 = h * 8 + 2 * j;
        const float x0 = c0 < nco ? s_w[c0 * ld + ci * taps + tap] : 0.f;
        const float x1 = c0 + 1 < nco ? s_w[(c0 + 1) * ld + ci * taps + tap] : 0.f;
        w4[j] = (uint32_t)f2bf(x0) | ((uint32_t)f2bf(x1) << 16);
      }
      *reinterpret_cast<uint4*>(S.wd + (int64_t)(ci0 + ci) * S.Kpad_d + tap * tld + co0 + h * 8) =
          make_uint4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
}

__global__ void step_inc_kernel(float* step, int64_t* cursor) {
  step[0] += 1.f;
  if (cursor) cursor[0] += 1;  // the next step gathers the next row of the batch-index schedule
}

int launch_step_inc(float* step, int64_t* cursor, hipStream_t st) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, st, step, cursor);
  return (int)hipGetLastError();
}

int launch_adam_pack(const AdamArgs& a, const OptSeg* d_segs, int ns, int64_t nblocks, hipStream_t st) {
  if (nblocks <= 0 || nblocks >= (1ll << 31)) return -2;
  hipLaunchKernelGGL(adam_pack_kernel, dim3((unsigned)nblocks), dim3(256), 0, st, a, d_segs, ns);
  int rc = (int)hipGetLastError();
  if (rc || !a.update || !a.inc_step) return rc;
  return launch_step_inc(const_cast<float*>(a.step), a.cursor, st);
}

}  // namespace mda
