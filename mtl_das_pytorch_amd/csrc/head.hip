// Fused task heads + losses + on-device metrics.
//
// mtl_head: one launch for all tasks of Models A/B (reference modelA_MTL.py:165-172 and the loss /
//   metric code of utils.py:272-292,359-380):  GAP over HxW -> AvgPool1d over groups of C/ncls channels
//   -> log_softmax -> NLL (mean over batch) weighted per task; writes log-probabilities, the gradient
//   w.r.t. the task features (broadcast back through the pools) and accumulates loss sums, correct
//   counts, |pred - label| (distance MAE in metres) and the confusion matrix with atomics, so the hot
//   loop never synchronises with the host (the reference does 4 .item() syncs per batch).
//
// cls_head (+ cls_wgrad): Model C's GAP -> Dropout(0.5) -> Linear(2048, 32) -> CrossEntropy
//   (modelC_multiClassifier.py:146-152, utils.py:746-771) with the joint label decoded on device into
//   (distance, event) = (j % 16, j / 16) for the metrics (replaces the per-sample Python loop).
#include "kernels.h"

namespace mda {


// One block per (sample, task): the tasks' dependent chains (GAP -> group mean -> softmax -> gradient)
// run side by side instead of one after the other, and the label is fetched before the GAP.
__global__ __launch_bounds__(256) void mtl_head_kernel(HeadArgs a) {
  __shared__ float s_gap[256];
  __shared__ float s_part8[2048];  // [256 / (C/8) lanes][C]
  __shared__ float s_logit[16], s_prob[16];
  __shared__ int s_lab;
  const int b = blockIdx.x, t = blockIdx.y;
  if (threadIdx.x == 0) s_lab = (int)a.labels[(int64_t)b * a.lab_stride + a.lab_off + t];
  const bool valid = a.nvalid == nullptr || b < *a.nvalid;
  {
    const bf16_t* f = a.feat + a.fgs * t + (int64_t)b * a.HW * a.ldf;
    // GAP: thread -> (8-channel group, pixel lane), 16-byte loads, 4 independent pixels in flight
    const int ng = a.C >> 3, lanes = 256 / ng;
    const int cg = threadIdx.x % ng, pl = threadIdx.x / ng;
    float s8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (pl < lanes) {
      int p = pl;
      for (; p + 3 * lanes < a.HW; p += 4 * lanes) {
        float v[4][8];
#pragma unroll
        for (int u = 0; u < 4; ++u) load8(f + (int64_t)(p + u * lanes) * a.ldf + cg * 8, v[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) s8[j] += (v[0][j] + v[1][j]) + (v[2][j] + v[3][j]);
      }
      for (; p < a.HW; p += lanes) {
        float v[8];
        load8(f + (int64_t)p * a.ldf + cg * 8, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s8[j] += v[j];
      }
    }
    float* sp = s_part8 + pl * a.C + cg * 8;  // [lanes][C]
    if (pl < lanes) {
#pragma unroll
      for (int j = 0; j < 8; ++j) sp[j] = s8[j];
    }
    __syncthreads();
    if (threadIdx.x < a.C) {
      float acc = 0.f;
      for (int q = 0; q < lanes; ++q) acc += s_part8[q * a.C + threadIdx.x];
      s_gap[threadIdx.x] = acc / (float)a.HW;
    }
    __syncthreads();
    const int K = a.ncls[t], gsz = a.C / K;
    if (threadIdx.x < K) {
      float acc = 0.f;
      for (int q = 0; q < gsz; ++q) acc += s_gap[threadIdx.x * gsz + q];
      s_logit[threadIdx.x] = acc / (float)gsz;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float mx = -INFINITY;
      int am = 0;
      for (int k = 0; k < K; ++k) if (s_logit[k] > mx) { mx = s_logit[k]; am = k; }
      float se = 0.f;
      for (int k = 0; k < K; ++k) se += __expf(s_logit[k] - mx);
      const float lse = mx + __logf(se);
      const int lab = s_lab;
      for (int k = 0; k < K; ++k) {
        float lp = s_logit[k] - lse;
        a.logp[((int64_t)t * a.B + b) * 16 + k] = lp;
        s_prob[k] = __expf(lp);
      }
      const float loss = lse - s_logit[lab];
      float* mt = a.metrics + t * 4;
      if (valid) {
        atomicAdd(mt + 0, loss);
        atomicAdd(mt + 1, am == lab ? 1.f : 0.f);
        atomicAdd(mt + 2, 1.f);
        atomicAdd(mt + 3, fabsf((float)(am - lab)));
        atomicAdd(a.confusion + (t * 16 + lab) * 16 + am, 1);
      }
      s_prob[lab] -= 1.f;  // softmax - onehot
    }
    __syncthreads();
    if (a.dfeat) {
      // d loss_t / d feat[p][c] = w_t * (p_j - y_j) / B / gsz / HW for channel c in group j
      bf16_t* d = a.dfeat + a.dgs * t + (int64_t)b * a.HW * a.C;
      const float scale = a.w[t] / ((float)a.B * gsz * a.HW);
      const int n4 = a.HW * a.C / 4;  // 8-byte bf16 stores; a group of 4 channels shares its class (gsz % 4 == 0)
      for (int i = threadIdx.x; i < n4; i += 256) {
        const int ch = (i * 4) % a.C;
        const uint32_t h = (uint32_t)f2bf(s_prob[ch / gsz] * scale);
        reinterpret_cast<uint2*>(d)[i] = make_uint2(h | (h << 16), h | (h << 16));
      }
    }
  }
}

int launch_mtl_head(const HeadArgs& a, hipStream_t st) {
  if (a.C > 256 || 256 % a.C || a.C % 8 || a.ldf % 8) return -2;
  for (int t = 0; t < a.T; ++t)
    if (a.ncls[t] <= 0 || a.C % a.ncls[t] || (a.C / a.ncls[t]) % 4) return -2;
  hipLaunchKernelGGL(mtl_head_kernel, dim3(a.B, a.T), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// Model C classifier head
// ------------------------------------------------------------------------------------------------
DEV uint32_t hash3(uint32_t a, uint32_t b, uint32_t c) {
  // a few rounds of a counter-based mixer (splitmix/murmur finaliser style)
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u) * 0x85EBCA77u ^ (c + 0x165667B1u) * 0xC2B2AE3Du;
  h ^= h >> 16; h *= 0x7FEB352Du; h ^= h >> 15; h *= 0x846CA68Bu; h ^= h >> 16;
  return h;
}


// One block of 1024 threads per sample; thread t owns channels t and t + 1024.  It loads its GAP inputs,
// draws its dropout mask and loads its fc weight column W[:, c] ONCE: the column feeds the per-class
// partial dot products (wave DPP sums, then 16 wave partials in LDS) and, after the softmax, the input
// gradient -- no second pass over W, no global round trip for d(logits).  (The previous 256-thread form
// walked W twice with long serial per-thread loops: 134 us per step on Model C.)
constexpr int CLS_T = 1024, CLS_CPT = 2, CLS_NC = 32;  // threads, channels per thread, cached classes
__global__ __launch_bounds__(CLS_T) void cls_head_kernel(ClsArgs a) {
  __shared__ float s_red[CLS_T / 64][64];
  __shared__ float s_logit[64], s_dl[64];
  __shared__ int s_lab;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  if (tid == 0) s_lab = (int)a.labels[b];
  // 64-bit counter: low word = training step, high word = the RNG stream (run seed and DP rank, set by
  // InceptionProgram.set_rng_stream) -- every rank and every --seed draws its own masks
  const uint64_t s64 = a.seed ? (uint64_t)(*a.seed) : 0ull;
  const uint32_t seed = (uint32_t)s64 ^ hash3((uint32_t)(s64 >> 32), 0x632BE5ABu, 0x1B873593u);
  const float keep_scale = a.p_drop > 0.f ? 1.f / (1.f - a.p_drop) : 1.f;
  float f[CLS_CPT], msk[CLS_CPT], w[CLS_NC][CLS_CPT];
#pragma unroll
  for (int i = 0; i < CLS_CPT; ++i) {
    const int c = tid + i * CLS_T;
    f[i] = 0.f; msk[i] = 0.f;
    if (c < a.C) {
      float s = 0.f;
      for (int p = 0; p < a.HW; ++p) s += bf2f(a.x[((int64_t)b * a.HW + p) * a.ldx + c]);
      s /= (float)a.HW;
      float m = 1.f;
      if (a.p_drop > 0.f) {
        float u = (hash3(seed, (uint32_t)b, (uint32_t)c) >> 8) * (1.f / 16777216.f);
        m = u >= a.p_drop ? keep_scale : 0.f;
      }
      msk[i] = m;
      f[i] = s * m;
      a.feat[(int64_t)b * a.C + c] = s * m;
    }
  }
  const bool cached = a.N <= CLS_NC;
  if (cached) {  // fully unrolled: w[][] stays in registers (compile-time indices)
#pragma unroll
    for (int n = 0; n < CLS_NC; ++n) {
      if (n < a.N) {
        float p = 0.f;
#pragma unroll
        for (int i = 0; i < CLS_CPT; ++i) {
          const int c = tid + i * CLS_T;
          w[n][i] = c < a.C ? a.W[(int64_t)n * a.C + c] : 0.f;
          p += w[n][i] * f[i];
        }
        p = wave_sum(p);
        if (lane == 0) s_red[wid][n] = p;
      }
    }
  } else {
    for (int n = 0; n < a.N; ++n) {
      float p = 0.f;
#pragma unroll
      for (int i = 0; i < CLS_CPT; ++i) {
        const int c = tid + i * CLS_T;
        p += (c < a.C ? a.W[(int64_t)n * a.C + c] : 0.f) * f[i];
      }
      p = wave_sum(p);
      if (lane == 0) s_red[wid][n] = p;
    }
  }
  __syncthreads();
  if (tid < a.N) {
    float acc = 0.f;
#pragma unroll
    for (int q = 0; q < CLS_T / 64; ++q) acc += s_red[q][tid];
    s_logit[tid] = acc + a.bias[tid];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float mx = -INFINITY;
    int am = 0;
    for (int n = 0; n < a.N; ++n) if (s_logit[n] > mx) { mx = s_logit[n]; am = n; }
    float se = 0.f;
    for (int n = 0; n < a.N; ++n) se += __expf(s_logit[n] - mx);
    const float lse = mx + __logf(se);
    const int lab = s_lab;
    for (int n = 0; n < a.N; ++n) a.logits[(int64_t)b * a.N + n] = s_logit[n];
    const float loss = lse - s_logit[lab];
    const int pd = am % 16, pe = am / 16, ld_ = lab % 16, le = lab / 16;
    const bool valid = a.nvalid == nullptr || b < *a.nvalid;
    if (valid) {
    atomicAdd(a.metrics + 0, loss);
    atomicAdd(a.metrics + 1, am == lab ? 1.f : 0.f);
    atomicAdd(a.metrics + 2, 1.f);
    atomicAdd(a.metrics + 4 + 1, pd == ld_ ? 1.f : 0.f);
    atomicAdd(a.metrics + 4 + 2, 1.f);
    atomicAdd(a.metrics + 4 + 3, fabsf((float)(pd - ld_)));
    atomicAdd(a.metrics + 8 + 1, pe == le ? 1.f : 0.f);
    atomicAdd(a.metrics + 8 + 2, 1.f);
    atomicAdd(a.confusion + ld_ * 16 + pd, 1);
    atomicAdd(a.confusion + 256 + le * 16 + pe, 1);
    }
    if (a.dlogits) {
      for (int n = 0; n < a.N; ++n) {
        const float dl = (__expf(s_logit[n] - lse) - (n == lab ? 1.f : 0.f)) / (float)a.B;
        s_dl[n] = dl;
        a.dlogits[(int64_t)b * a.N + n] = dl;
      }
    }
  }
  if (!a.dx) return;
  __syncthreads();
  // dx[b][p][c] = (sum_n dlogits[n] W[n][c]) * mask[c] / HW
#pragma unroll
  for (int i = 0; i < CLS_CPT; ++i) {
    const int c = tid + i * CLS_T;
    if (c >= a.C) continue;
    float acc = 0.f;
    if (cached) {
#pragma unroll
      for (int n = 0; n < CLS_NC; ++n)
        if (n < a.N) acc += s_dl[n] * w[n][i];
    } else {
      for (int n = 0; n < a.N; ++n) acc += s_dl[n] * a.W[(int64_t)n * a.C + c];
    }
    const bf16_t h = f2bf(acc * (msk[i] / (float)a.HW));
    for (int p = 0; p < a.HW; ++p) a.dx[((int64_t)b * a.HW + p) * a.C + c] = h;
  }
}

// dW[n][c] = sum_b dlogits[b][n] * feat[b][c];  db[n] = sum_b dlogits[b][n]; advances the dropout seed.
__global__ __launch_bounds__(256) void cls_wgrad_kernel(ClsArgs a, int64_t* seed) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < (int64_t)a.N * a.C) {
    const int n = (int)(i / a.C), c = (int)(i - (int64_t)n * a.C);
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b) acc += a.dlogits[(int64_t)b * a.N + n] * a.feat[(int64_t)b * a.C + c];
    a.dW[i] = acc;
  }
  if (blockIdx.x == 0 && threadIdx.x < a.N) {
    float acc = 0.f;
    for (int b = 0; b < a.B; ++b) acc += a.dlogits[(int64_t)b * a.N + threadIdx.x];
    a.db[threadIdx.x] = acc;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && seed) *seed += 1;
}

int launch_cls_head(const ClsArgs& a, int64_t* seed_mut, hipStream_t st) {
  if (a.N > 64 || a.C > CLS_T * CLS_CPT) return -2;
  hipLaunchKernelGGL(cls_head_kernel, dim3(a.B), dim3(CLS_T), 0, st, a);
  int rc = (int)hipGetLastError();
  if (rc || !a.dx) return rc;
  const int64_t n = (int64_t)a.N * a.C;
  hipLaunchKernelGGL(cls_wgrad_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, a, seed_mut);
  return (int)hipGetLastError();
}

}  // namespace mda
