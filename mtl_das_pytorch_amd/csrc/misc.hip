// Data movement and pooling kernels.
//
// gather_batch: the on-device replacement of the reference's host data path (DataLoader collate of
//   loadmat'd arrays + pageable .cuda() copies, utils.py:264-266,351-353): picks the batch rows of an
//   HBM-resident fp32 NCHW dataset by index, converts to bf16 NHWC with the channel dim zero-padded to
//   8 (so the 1-channel stem runs on the generic MFMA implicit-GEMM path) and gathers the labels.
// Inception pools (model C, torchvision semantics used by modelC_multiClassifier.py):
//   maxpool 3x3/s2 (valid) and avgpool 3x3/s1/p1 (count_include_pad=True), forward and backward; the
//   backward passes are written in gather form (each input pixel sums the windows that cover it and,
//   for max, recomputes the first-max argmax), so they are deterministic and need no index tensors.
#include "kernels.h"

namespace mda {

// taps > 0 (single-channel input): vertical tap packing for the stem conv -- channel j of pixel (h, w)
// holds x[h - off + j][w] (zero outside the image, j < taps), so a KHxKW stem over 1 channel runs as a
// 1xKW conv over KH real channels (engine/core.py stem_pack_geom) instead of wasting 7/8 of its K on
// zero padding channels.
// zero: the arena's zeroed regions (BN statistic replicas, backward workspaces) cleared by the same launch
// at the start of a training step -- one dependent launch instead of a gather plus a fill per dtype.
__global__ __launch_bounds__(256) void gather_batch_kernel(const float* __restrict__ X, const int64_t* __restrict__ idx,
                                                           const int64_t* __restrict__ lab, int lab_w,
                                                           bf16_t* __restrict__ out, int64_t* __restrict__ lab_out,
                                                           int B, int Cin, int H, int W, int taps, int off,
                                                           ZeroRanges zero, const int64_t* __restrict__ cursor,
                                                           int nrows) {
  // batch-index schedule (cursor set): this step's indices are row (*cursor mod nrows) of a [nrows][B] table;
  // the optimizer's step-counter kernel advances the cursor at the end of the step, so no host copy of the
  // indices precedes each replay
  if (cursor) idx += (*cursor % nrows) * (int64_t)B;
  {
    const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, nt = (int64_t)gridDim.x * 256;
    for (int r = 0; r < zero.n; ++r)
      for (int64_t i = t; i < zero.n16[r]; i += nt) zero.p[r][i] = make_uint4(0, 0, 0, 0);
  }
  const int64_t M = (int64_t)B * H * W;
  const int HW = H * W;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < M; p += (int64_t)gridDim.x * 256) {
    const int b = (int)p / HW;  // M < 2^31 (checked by the launcher)
    const int r = (int)p - b * HW;
    const int64_t src = idx[b];
    float v[8];
    if (taps > 0) {
      const int h = r / W;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int hh = h - off + j;
        v[j] = (j < taps && hh >= 0 && hh < H) ? X[src * (int64_t)H * W + r + (hh - h) * W] : 0.f;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = c < Cin ? X[(src * Cin + c) * (int64_t)H * W + r] : 0.f;
    }
    store8(out + p * 8, v);
  }
  if (blockIdx.x == 0)
    for (int i = threadIdx.x; i < B * lab_w; i += 256) {
      const int b = i / lab_w, k = i - b * lab_w;
      lab_out[i] = lab[idx[b] * lab_w + k];
    }
}

int launch_gather_batch(const float* X, const int64_t* idx, const int64_t* lab, int lab_w, bf16_t* out,
                        int64_t* lab_out, int B, int Cin, int H, int W, int taps, int off, const ZeroRanges& zero,
                        const int64_t* cursor, int nrows, hipStream_t st) {
  if (Cin > 8 || taps > 8 || (taps > 0 && Cin != 1) || (int64_t)B * H * W >= (1ll << 31)) return -2;
  const int64_t M = (int64_t)B * H * W;
  // one pixel per thread (no grid-stride second round: the idx -> X -> store chain is latency-bound)
  int blocks = (int)std::min<int64_t>((M + 255) / 256, 65535);
  hipLaunchKernelGGL(gather_batch_kernel, dim3(blocks), dim3(256), 0, st, X, idx, lab, lab_w, out, lab_out, B, Cin, H, W,
                     taps, off, zero, cursor, nrows);
  return (int)hipGetLastError();
}


// 3x3 pools of the Inception model: MAX = 1 max pool stride 2 (no padding), MAX = 0 average pool stride 1
// padding 1 (count_include_pad: always /9).  One thread per (output pixel, 8-channel group).  All nine
// window loads are issued before any is consumed (with the load and its use in the same bounds-checked
// region, each tap waited for its own memory round trip), and the index math is 32-bit (n < 2^31,
// checked by the launcher).
template <int MAX>
__global__ __launch_bounds__(256) void pool3_fwd_kernel(PoolArgs a) {
  const int CG = a.C >> 3;
  const int HWo = a.Ho * a.Wo;
  const int n = a.B * HWo * CG;
  constexpr int s = MAX ? 2 : 1, pd = MAX ? 0 : 1;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int p = i / CG, cg = i - p * CG;
    const int b = p / HWo, r = p - b * HWo;
    const int oh = r / a.Wo, ow = r - oh * a.Wo;
    uint4 raw[9];
    bool ok[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ih = oh * s - pd + t / 3, iw = ow * s - pd + t % 3;
      ok[t] = ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      raw[t] = ok[t] ? *reinterpret_cast<const uint4*>(a.x + ((int64_t)(b * a.H + ih) * a.W + iw) * a.ldx + cg * 8)
                     : make_uint4(0, 0, 0, 0);
    }
    float acc[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { acc[j] = MAX ? -INFINITY : 0.f; am[j] = 0; }
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (MAX && !ok[t]) continue;  // (the models' max-pool windows are always inside the map)
      float v[8];
      unpack8(raw[t], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        // torch semantics: first max in row-major order, and a NaN wins (propagates; last NaN's index)
        if (MAX) {
          if (v[j] > acc[j] || isnan(v[j])) { acc[j] = v[j]; am[j] = t; }
        } else {
          acc[j] += v[j];
        }
      }
    }
    if (MAX && a.am) {
      uint32_t lo = 0, hi = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) { lo |= (uint32_t)am[j] << (8 * j); hi |= (uint32_t)am[j + 4] << (8 * j); }
      *reinterpret_cast<uint2*>(a.am + (int64_t)p * a.C + cg * 8) = make_uint2(lo, hi);
    }
    if (!MAX) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= (1.f / 9.f);
    }
    store8(a.y + (int64_t)p * a.ldy + cg * 8, acc);
  }
}

// Gradient of the input: sum over the output windows covering an input pixel (<= 4 for the stride-2 max
// pool, <= 9 for the average pool) and over the bf16 gradient sources; per source, every window's loads are
// issued before any is consumed.  MAX = 1: max pool, the argmax stored by the training forward routes the
// gradient (a.am); MAX = 2: max pool without it (eval-mode programs, the functional API without `am`), each window is re-read to find its
// maximum (a separate instantiation: sharing one kernel spilled the argmax path to scratch); MAX = 0: average.
template <int MAX>
__global__ __launch_bounds__(256) void pool3_bwd_kernel(PoolArgs a) {
  const int CG = a.C >> 3;
  const int HW = a.H * a.W;
  const int n = a.B * HW * CG;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const int p = i / CG, cg = i - p * CG;
    const int b = p / HW, r = p - b * HW;
    const int ih = r / a.W, iw = r - ih * a.W;
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    if (MAX == 1) {
      // windows (stride 2, no pad) covering ih: oh in [ceil((ih-2)/2), ih/2] -- at most 2 x 2
      const int oh0 = max(0, (ih - 1) >> 1), oh1 = min(a.Ho - 1, ih >> 1);
      const int ow0 = max(0, (iw - 1) >> 1), ow1 = min(a.Wo - 1, iw >> 1);
      uint2 w[4];
      int q[4], me[4];
      bool ok[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int oh = oh0 + (t >> 1), ow = ow0 + (t & 1);
        ok[t] = oh <= oh1 && ow <= ow1 && ih <= 2 * oh + 2 && iw <= 2 * ow + 2;
        q[t] = (b * a.Ho + oh) * a.Wo + ow;
        me[t] = (ih - 2 * oh) * 3 + (iw - 2 * ow);
        w[t] = ok[t] ? *reinterpret_cast<const uint2*>(a.am + (int64_t)q[t] * a.C + cg * 8) : make_uint2(0, 0);
      }
      for (int sidx = 0; sidx < a.g.n; ++sidx) {
        const bf16_t* gp = a.g.p[sidx];
        const int ld = a.g.ld[sidx];
        uint4 gu[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16_t* src = gp + (int64_t)q[t] * ld + cg * 8;
          gu[t] = ok[t] ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {  // (a window outside the range has w = 0 and g = 0: adds nothing)
          const uint32_t m = (uint32_t)me[t];
          float gv[8];
          unpack8(gu[t], gv);
          const uint32_t wb[2] = {w[t].x, w[t].y};
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += (((wb[j >> 2] >> (8 * (j & 3))) & 255u) == m) ? gv[j] : 0.f;
        }
      }
    } else if (MAX == 2) {
      const int oh0 = max(0, (ih - 1) >> 1), oh1 = min(a.Ho - 1, ih >> 1);
      const int ow0 = max(0, (iw - 1) >> 1), ow1 = min(a.Wo - 1, iw >> 1);
      for (int oh = oh0; oh <= oh1; ++oh)
        for (int ow = ow0; ow <= ow1; ++ow) {
          if (ih < 2 * oh || ih > 2 * oh + 2 || iw < 2 * ow || iw > 2 * ow + 2) continue;
          const int me = (ih - 2 * oh) * 3 + (iw - 2 * ow);
          float mx[8];
          int am[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) { mx[j] = -INFINITY; am[j] = -1; }
          for (int kh = 0; kh < 3; ++kh)
            for (int kw = 0; kw < 3; ++kw) {
              float v[8];
              load8(a.x + ((int64_t)(b * a.H + 2 * oh + kh) * a.W + 2 * ow + kw) * a.ldx + cg * 8, v);
#pragma unroll
              for (int j = 0; j < 8; ++j)
                if (v[j] > mx[j] || isnan(v[j])) { mx[j] = v[j]; am[j] = kh * 3 + kw; }
            }
          float g[8];
          gsum8(a.g, 0, (int64_t)(b * a.Ho + oh) * a.Wo + ow, cg * 8, g);
#pragma unroll
          for (int j = 0; j < 8; ++j) if (am[j] == me) acc[j] += g[j];
        }
    } else {
      // average pool, stride 1, padding 1: the output windows oh in [ih-1, ih+1], ow in [iw-1, iw+1]
      for (int sidx = 0; sidx < a.g.n; ++sidx) {
        const bf16_t* gp = a.g.p[sidx];
        const int ld = a.g.ld[sidx];
        uint4 gu[9];
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int oh = ih - 1 + t / 3, ow = iw - 1 + t % 3;
          const bool ok = oh >= 0 && oh < a.Ho && ow >= 0 && ow < a.Wo;
          const bf16_t* src = gp + (int64_t)((b * a.Ho + oh) * a.Wo + ow) * ld + cg * 8;
          gu[t] = ok ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          float gv[8];
          unpack8(gu[t], gv);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += gv[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= (1.f / 9.f);
    }
    store8(a.dx + (int64_t)p * a.lddx + cg * 8, acc);
  }
}

int launch_pool3(int is_max, int backward, const PoolArgs& a, hipStream_t st) {
  const int64_t n = (int64_t)a.B * (backward ? a.H * a.W : a.Ho * a.Wo) * (a.C / 8);
  if (n >= (1ll << 31) || a.C % 8) return -2;  // 32-bit index math in the kernels, 8-channel groups
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  if (!backward) {
    if (is_max) hipLaunchKernelGGL(pool3_fwd_kernel<1>, dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(pool3_fwd_kernel<0>, dim3(blocks), dim3(256), 0, st, a);
  } else {
    if (is_max && a.am) hipLaunchKernelGGL(pool3_bwd_kernel<1>, dim3(blocks), dim3(256), 0, st, a);
    else if (is_max) hipLaunchKernelGGL(pool3_bwd_kernel<2>, dim3(blocks), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(pool3_bwd_kernel<0>, dim3(blocks), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

// In-graph timeline stamp (tools/timeline.py): one thread stores the 100 MHz wall clock at buf[i] after the
// work enqueued before it on its stream -- a profiler-free view of multi-stream graph replays -- and, when q is
// given, the HSA queue the packet was dispatched from at q[i] (how the HIP graph executor mapped the captured
// streams onto queues).  The caller sizes both buffers for every index it passes (the binding checks i < n).
__global__ void tick_kernel(uint64_t* buf, uint64_t* q, int i) {
  buf[i] = wall_clock64();
  if (q) q[i] = reinterpret_cast<uint64_t>(__builtin_amdgcn_queue_ptr());
}

int launch_tick(uint64_t* buf, uint64_t* q, int i, hipStream_t st) {
  hipLaunchKernelGGL(tick_kernel, dim3(1), dim3(1), 0, st, buf, q, i);
  return (int)hipGetLastError();
}

// sum of up to 6 bf16 gradient sources into one buffer (used where a consumer is not a fused tail)
__global__ __launch_bounds__(256) void grad_sum_kernel(GradSrcs g, bf16_t* out, int ldo, int64_t M, int C) {
  const int CG = C >> 3;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < M * CG; i += (int64_t)gridDim.x * 256) {
    const int64_t p = i / CG;
    const int c = (int)(i - p * CG) * 8;
    float v[8];
    gsum8(g, 0, p, c, v);
    store8(out + p * ldo + c, v);
  }
}

int launch_grad_sum(const GradSrcs& g, bf16_t* out, int ldo, int64_t M, int C, hipStream_t st) {
  const int64_t n = M * (C / 8);
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(grad_sum_kernel, dim3(blocks), dim3(256), 0, st, g, out, ldo, M, C);
  return (int)hipGetLastError();
}

}  // namespace mda
