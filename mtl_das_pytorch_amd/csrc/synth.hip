// On-device synthetic DAS generator: the physical toy model of data/synthetic.py evaluated
// per element on the GPU, with counter-based Philox-4x32-10 Gaussian noise, so a dataset of any size is
// produced in HBM in one launch (no host tensors, no torch elementwise chain of ~30 [n, H, W] temporaries).
//
// One block per sample:
//   pass 1  clean signal at every (h, w) of the sample and its mean power (LDS block reduction);
//   pass 2  out[s, c, h, w] = 100 * (clean(h, (w - c) mod W) + sigma_s * N(0, 1)), channel c > 0 being the
//           time-shifted copy of the clean signal (torch.roll in the torch path).
// The per-sample scalars (distance, event, onset, position, jitter, SNR) come from the same CPU generator
// draws as the torch path, so the clean signals agree to fp32 rounding; the noise is Philox keyed by the
// sample's noise seed with counter (element quad, channel, global sample index): it depends on neither the
// launch geometry nor the device count.
//
// The reference reads field recordings from .mat files (dataset_preparation.py:300-344) and has no
// generator; this replaces its data source for benchmarks and tests (no network for the real dataset).
#include "kernels.h"

namespace mda {

namespace {

constexpr uint32_t PHILOX_M0 = 0xD2511F53u, PHILOX_M1 = 0xCD9E8D57u;
constexpr uint32_t PHILOX_W0 = 0x9E3779B9u, PHILOX_W1 = 0xBB67AE85u;

DEV uint4 philox4x32_10(uint4 ctr, uint2 key) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t hi0 = __umulhi(PHILOX_M0, ctr.x), lo0 = PHILOX_M0 * ctr.x;
    const uint32_t hi1 = __umulhi(PHILOX_M1, ctr.z), lo1 = PHILOX_M1 * ctr.z;
    ctr = make_uint4(hi1 ^ ctr.y ^ key.x, lo1, hi0 ^ ctr.w ^ key.y, lo0);
    key.x += PHILOX_W0;
    key.y += PHILOX_W1;
  }
  return ctr;
}

// uniform in (0, 1]: never 0, so log() is finite
DEV float u01(uint32_t x) { return ((float)(x >> 8) + 1.f) * (1.f / 16777216.f); }

DEV float linspace01(int i, int n) {  // torch.linspace(0, 1, n)[i] (symmetric evaluation from both ends)
  if (n == 1) return 0.f;
  const float step = 1.f / (float)(n - 1);
  return i < n / 2 ? (float)i * step : 1.f - (float)(n - 1 - i) * step;
}

struct SampleConsts {
  float dist_m, x0, t0, amp, f_strike, period, f_dig, dig_phase, ev;
};

DEV float clean_at(const SampleConsts& k, float xs, float ts) {
  const float dx = (xs - k.x0) * 20.f;
  const float arrival = k.t0 + sqrtf(k.dist_m * k.dist_m + dx * dx) / 110.f;
  const float tau = ts - arrival;
  const float fw = 1.5f + 0.6f * k.dist_m;
  const float footprint = expf(-(dx * dx) / (2.f * fw * fw));
  const float phase = tau - floorf(tau / k.period) * k.period;  // torch.remainder (sign of the divisor)
  const float strike = tau > 0.f ? expf(-phase / 0.012f) * cosf(6.283185307179586f * k.f_strike * phase) : 0.f;
  const float db = tau - 0.18f;
  const float burst = expf(-(db * db) / (2.f * 0.09f * 0.09f));
  const float dig = burst * sinf(6.283185307179586f * k.f_dig * tau + k.dig_phase);
  return k.amp * footprint * ((1.f - k.ev) * strike + k.ev * dig);
}

__global__ __launch_bounds__(256) void synth_das_kernel(SynthArgs a) {
  const int s = blockIdx.x;
  const float* q = a.params + (int64_t)s * SYNTH_NPARAM;  // distance, event, x0, t0, jitter[4], snr_db
  SampleConsts k;
  k.dist_m = q[0] + 0.5f;
  k.ev = q[1];
  k.x0 = q[2];
  k.t0 = q[3];
  k.amp = 1.f / (1.f + k.dist_m / 4.f);
  k.f_strike = 38.f + 6.f * q[4];
  k.period = 0.16f + 0.04f * q[5];
  k.f_dig = 9.f + 3.f * q[6];
  k.dig_phase = 6.28f * q[7];
  const float snr_db = q[8];
  const int HW = a.H * a.W;

  // pass 1: mean power of the clean signal
  float acc = 0.f;
  for (int e = threadIdx.x; e < HW; e += 256) {
    const int h = e / a.W, w = e - h * a.W;
    const float v = clean_at(k, linspace01(h, a.H), linspace01(w, a.W));
    acc += v * v;
  }
  __shared__ float s_red[256];
  s_red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) s_red[threadIdx.x] += s_red[threadIdx.x + o];
    __syncthreads();
  }
  const float p_sig = fmaxf(s_red[0] / (float)HW, 1e-12f);
  const float sigma = a.noise ? sqrtf(p_sig / powf(10.f, snr_db / 10.f)) : 0.f;

  // pass 2: signal + noise, four consecutive elements per Philox draw
  const uint2 key = make_uint2((uint32_t)a.key, (uint32_t)(a.key >> 32));
  const uint32_t gs = (uint32_t)(a.sample0 + s);
  float* out = a.out + (int64_t)s * a.C * HW;
  const int nq = (HW + 3) / 4;
  for (int c = 0; c < a.C; ++c) {
    for (int qd = threadIdx.x; qd < nq; qd += 256) {
      float n4[4] = {0.f, 0.f, 0.f, 0.f};
      if (a.noise) {
        const uint4 r = philox4x32_10(make_uint4((uint32_t)qd, (uint32_t)c, gs, 0u), key);
        // Box-Muller on (r.x, r.y) and (r.z, r.w)
        const float m0 = sqrtf(-2.f * logf(u01(r.x))), m1 = sqrtf(-2.f * logf(u01(r.z)));
        float s0, c0, s1, c1;
        sincosf(6.283185307179586f * u01(r.y), &s0, &c0);
        sincosf(6.283185307179586f * u01(r.w), &s1, &c1);
        n4[0] = m0 * c0; n4[1] = m0 * s0; n4[2] = m1 * c1; n4[3] = m1 * s1;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int e = qd * 4 + j;
        if (e >= HW) break;
        const int h = e / a.W, w = e - h * a.W;
        int ws = w - c % a.W;
        if (ws < 0) ws += a.W;
        const float v = clean_at(k, linspace01(h, a.H), linspace01(ws, a.W));
        out[(int64_t)c * HW + e] = 100.f * (v + sigma * n4[j]);
      }
    }
  }
}

}  // namespace

int launch_synth_das(const SynthArgs& a, int n, hipStream_t st) {
  if (n <= 0 || a.H <= 0 || a.W <= 0 || a.C <= 0 || !a.params || !a.out) return -2;
  hipLaunchKernelGGL(synth_das_kernel, dim3(n), dim3(256), 0, st, a);
  return (int)hipGetLastError();
}

// Philox known-answer hook for tests: out[i] = philox(ctr_i, key) words (4 per counter)
__global__ void philox_kat_kernel(const uint32_t* ctr, uint64_t key, uint32_t* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4 r = philox4x32_10(make_uint4(ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3]),
                                make_uint2((uint32_t)key, (uint32_t)(key >> 32)));
  out[4 * i] = r.x; out[4 * i + 1] = r.y; out[4 * i + 2] = r.z; out[4 * i + 3] = r.w;
}

int launch_philox_kat(const uint32_t* ctr, uint64_t key, uint32_t* out, int n, hipStream_t st) {
  hipLaunchKernelGGL(philox_kat_kernel, dim3((n + 63) / 64), dim3(64), 0, st, ctr, key, out, n);
  return (int)hipGetLastError();
}

}  // namespace mda
