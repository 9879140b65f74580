// Common device helpers for the gfx950 (MI355X / CDNA4) kernels of mtl_das_pytorch_amd.
//
// Conventions used by every kernel in this directory:
//   * activations are NHWC, addressed as rows of pixels with a row pitch `ld` (elements), so a
//     channel slice of a concatenation buffer is just (base + channel_offset, ld = total_channels);
//   * MFMA operands are bf16, accumulation and every reduction is fp32;
//   * gradient buffers of activations are bf16 (as under autocast) and written exactly once (no
//     read-modify-write): every producer accumulates in fp32 and rounds once at its store, a consumer that
//     needs the sum of several gradient sources takes a GradSrcs list and sums them in fp32;
//   * per-channel BN statistics are accumulated into NREP replicas (blockIdx % NREP) to spread
//     atomic contention over the 8 XCD L2s; consumers sum the replicas;
//   * wave size is 64; blocks are 256 threads (4 waves).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <cstdlib>
#include <algorithm>

#define DEV __device__ __forceinline__

namespace mda {

constexpr int NREP = 32;  // BN-statistic replicas (atomic contention spread)

typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint16_t bf16_t;  // raw bf16 storage

// Block coordinates of a conv launch, optionally in XCD-contiguous order (ConvArgs::xcd).  The hardware deals
// blocks round-robin over the 8 XCDs (linear ids b and b + 8 share one L2; speed only, never correctness:
// MI355X_MICROARCH.md, workgroup dispatch), so consecutive pixel tiles -- which share the im2col halo rows --
// land on 8 different L2s, and every XCD fetches most of the input.  Remapped, the 8 hardware blocks that
// share an XCD walk one contiguous range of logical tiles, y (channel tiles / K splits) fastest, then x
// (pixel tiles), then z (groups): a tile's channel tiles and its pixel neighbours are read through one L2.
struct Blk { int x, y, z; };
DEV Blk block_coords(int remap) {
  if (!remap) return Blk{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z};
  const unsigned gx = gridDim.x, gy = gridDim.y, n = gx * gy * gridDim.z;
  const unsigned b = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
  const unsigned q = n >> 3, r = n & 7, xc = b & 7;
  unsigned t = xc * q + (xc < r ? xc : r) + (b >> 3);
  Blk k;
  k.y = (int)(t % gy);
  t /= gy;
  k.x = (int)(t % gx);
  k.z = (int)(t / gx);
  return k;
}

// Per-block phase timers (profiling only, tools/kernel_phases.py; the pointer is null in production): thread
// 0 of hardware block b stores the 100 MHz wall clock of phase i (0 entry, 1 prologue done, 2 main loop done,
// 3 exit) at t[4 * b + i], for the first PT_MAX_BLOCKS blocks of the grid.
constexpr unsigned PT_MAX_BLOCKS = 16384;
DEV void ptick(uint64_t* t, int i) {
  if (t != nullptr && threadIdx.x == 0) {
    const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
    if (b < PT_MAX_BLOCKS) t[4 * b + i] = wall_clock64();
  }
}

// n / d for 0 <= n < 2^24 and d >= 1 from inv = 1.f / d: n is exact in fp32 and the rounded quotient is
// within one of floor(n / d), corrected with one multiply-subtract -- ~8 VALU instructions instead of the
// ~30 of a 32-bit integer division (the im2col pixel decomposition of the weight-gradient staging runs it per
// 16-byte unit and chunk)
DEV int fdiv24(int n, int d, float inv) {
  int q = (int)((float)n * inv);
  const int r = n - q * d;
  q += (r >= d) - (r < 0);
  return q;
}

// Transposed LDS read for the 16x16x32 MFMA operands (ds_read_b64_tr_b16): rows r..r+3 and r+HI..r+HI+3 (two
// 4-row transposed reads), 16 columns col0..col0+15.  Lane 4q+p of each 16-lane group supplies &row[q][col0 + 4p];
// lane i receives column col0+i.
typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;
template <int HI = 4>
DEV bf16x8 tr_read8(const bf16_t* lds_row0, int ld_elems, int col0, int lane) {
  const int i = lane & 15, q = i >> 2, p = i & 3;
  const bf16_t* a0 = lds_row0 + q * ld_elems + col0 + 4 * p;
  const bf16_t* a1 = a0 + HI * ld_elems;
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a1));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// lane l receives column col0 + (l & 31) of rows 8 (l >> 5) .. 8 (l >> 5) + 7 of a pixel-major LDS image: the A
// (row = l & 31) or B (column = l & 31) operand of a 32x32x16 MFMA whose k index is the row
DEV bf16x8 tr_read32(const bf16_t* lds_row0, int ld, int col0, int lane) {
  const int i = lane & 15, g = lane >> 4;
  const bf16_t* a0 = lds_row0 + (8 * (g >> 1) + (i >> 2)) * ld + col0 + 16 * (g & 1) + 4 * (i & 3);
  v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0));
  v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(a0 + 4 * ld));
  return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

typedef float f32x16 __attribute__((ext_vector_type(16)));

DEV float bf2f(bf16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
// round-to-nearest-even; NaN-preserving via the hardware conversion
DEV bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);
  return *reinterpret_cast<bf16_t*>(&h);
}

DEV void unpack8(uint4 u, float* v) {  // 8 bf16 -> fp32
  const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
DEV void load8(const bf16_t* p, float* v) {
  uint4 u = *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(w[i] << 16);
    v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
DEV void store8(bf16_t* p, const float* v) {
  uint32_t w[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
  *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
}
DEV void load8f(const float* p, float* v) {
  float4 a = *reinterpret_cast<const float4*>(p);
  float4 b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
DEV void store8f(float* p, const float* v) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

DEV float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

// Cross-lane sums with DPP (data-parallel primitives): one VALU op per step instead of a ds_bpermute
// round trip through the LDS unit per __shfl_xor (measured: 24 six-step shuffle reductions took
// 4-7 us in the BN backward; DPP makes them negligible).  gfx9-family row operations: a row is 16
// lanes; bound_ctrl zero-fills lanes shifted in from outside the row.
template <int CTRL, int ROW_MASK = 0xF, int BANK_MASK = 0xF>
DEV float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROW_MASK,
                                                               BANK_MASK, true));
}
// Sum over each row of 16 lanes; the result is valid in lane 15 of the row.
DEV float row16_sum(float v) {
  v += dpp_f<0x111>(v);  // row_shr:1
  v += dpp_f<0x112>(v);  // row_shr:2
  v += dpp_f<0x114>(v);  // row_shr:4
  v += dpp_f<0x118>(v);  // row_shr:8
  return v;
}
// Sum over the wave, returned in every lane.
DEV float wave_sum(float v) {
  v = row16_sum(v);
  v += dpp_f<0x142, 0xA>(v);  // row_bcast:15 -> rows 1, 3
  v += dpp_f<0x143, 0xC>(v);  // row_bcast:31 -> rows 2, 3
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// ---------------------------------------------------------------------------------------------
// Parameter structs (passed by value as kernel arguments)
// ---------------------------------------------------------------------------------------------

// A bf16 NHWC source made of up to two channel segments (e.g. cat[F_shared, B_task]).
// Segment s covers channels [s ? C0 : 0, s ? C0 + C1 : C0). `gs` = element stride per group
// (grid.z); 0 means the segment is shared by every group.
struct Src2 {
  const bf16_t* p[2];
  int64_t gs[2];
  int ld[2];
  int C0, C1;
};

// Up to 6 bf16 gradient sources summed on load in fp32 (deterministic gradient accumulation).
struct GradSrcs {
  const bf16_t* p[6];
  int64_t gs[6];
  int ld[6];
  int n;
};

DEV void gsum8(const GradSrcs& g, int z, int64_t pix, int c, float* v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  for (int s = 0; s < g.n; ++s) {
    float t[8];
    load8(g.p[s] + g.gs[s] * z + pix * g.ld[s] + c, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += t[j];
  }
}

// fp32 -> bf16 -> fp32 (the value a bf16 gradient store keeps): statistics that a later pass recomputes from
// the stored gradient are accumulated from this rounded value, so both passes see the same numbers
DEV float rbf(float f) { return bf2f(f2bf(f)); }

// 4 consecutive bf16 values (8 bytes) <-> fp32
DEV void store4(bf16_t* p, const float* v) {
  uint2 w;
  w.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
  w.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
  *reinterpret_cast<uint2*>(p) = w;
}
DEV void load4(const bf16_t* p, float* v) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16); v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16); v[3] = __uint_as_float(u.y & 0xffff0000u);
}

// Per-BN-layer state. Everything is indexed by group z with the given strides (0 = shared).
struct BNArgs {
  const double* stats;   // [G][NREP][2][C] sums of y and y^2 (training) -- zeroed every step.  fp64: the
                         // atomic summation order then perturbs results by ~1e-16 instead of ~1e-7,
                         // which the (chaotic at init) networks amplified into run-to-run gradient
                         // differences of up to 10% (tools/dbg_race.py)
  const float* gamma;    // [C] (+ z * pstride)
  const float* beta;
  float* run_mean;       // running stats (+ z * pstride)
  float* run_var;
  int64_t* nbt;          // num_batches_tracked (+ z)
  int64_t pstride;       // element stride of gamma/beta/running stats between groups
  int C;
  int count;             // number of elements per channel reduced into stats (B*H*W)
  float eps, momentum;
  int training;          // 1: batch statistics (and update running), 0: running statistics
  float* consts;         // optional [G][4][C] (+ z * 4C): scale, shift, mean, invstd of the current batch,
                         // written by the forward tail's block 0 (training) and read by every backward
                         // kernel of this BN -- 4 floats per channel instead of 2 x NREP fp64 replicas
  int pnrep;             // backward: replicas in use of the [G][NREP][3][C] partial sums (bnb, dgrad epilogue)
  int nrep;              // replicas in use (power of two <= NREP; the producer wrote blockIdx.x % nrep):
                         // small-M layers have few producer blocks, and every consumer block reads all of
                         // them (Model C's 1x6 layers: 32 replicas x 448 channels = 229 KB per block)
  int sld;               // channel pitch of `stats` ([G][NREP][2][sld]): C, or the width of the combined
                         // replica rows of a horizontally fused conv whose output channels feed several BNs
                         // (this BN's rows then start at its channel offset)
};

template <int R>
DEV void bn_rep_sum(const double* st, int C, int c, double& s, double& ss) {
#pragma unroll
  for (int r = 0; r < R; ++r) { s += st[r * 2 * C + c]; ss += st[r * 2 * C + C + c]; }
}

// BN constants of channel c of group z: out = y * scale + shift == gamma * (y - mean) * invstd + beta.
// Training: batch statistics from the NREP replicas of the conv-epilogue sums (and, when requested,
// the running-statistics update -- done by exactly one block per launch); eval: running statistics.
DEV void bn_channel(const BNArgs& a, int z, int c, bool update_running, float& scale, float& shift, float& mean,
                    float& inv) {
  float var;
  if (a.training) {
    const double* st = a.stats + (int64_t)z * NREP * 2 * a.sld;
    double s = 0.0, ss = 0.0;
    switch (a.nrep) {  // a compile-time trip count keeps all loads of the reduction in flight
      case 1: bn_rep_sum<1>(st, a.sld, c, s, ss); break;
      case 2: bn_rep_sum<2>(st, a.sld, c, s, ss); break;
      case 4: bn_rep_sum<4>(st, a.sld, c, s, ss); break;
      case 8: bn_rep_sum<8>(st, a.sld, c, s, ss); break;
      case 16: bn_rep_sum<16>(st, a.sld, c, s, ss); break;
      default: bn_rep_sum<NREP>(st, a.sld, c, s, ss); break;
    }
    const double inv_n = 1.0 / (double)a.count;
    const double md = s * inv_n;
    mean = (float)md;
    var = (float)fmax(ss * inv_n - md * md, 0.0);
    if (update_running) {
      const float unb = a.count > 1 ? var * (float)a.count / (float)(a.count - 1) : var;
      float* rm = a.run_mean + a.pstride * z;
      float* rv = a.run_var + a.pstride * z;
      rm[c] = (1.f - a.momentum) * rm[c] + a.momentum * mean;
      rv[c] = (1.f - a.momentum) * rv[c] + a.momentum * unb;
    }
  } else {
    mean = a.run_mean[a.pstride * z + c];
    var = a.run_var[a.pstride * z + c];
  }
  inv = rsqrtf(var + a.eps);
  const float g = a.gamma[a.pstride * z + c], b = a.beta[a.pstride * z + c];
  scale = g * inv;
  shift = b - mean * g * inv;
}

// Backward kernels: the constants the forward tail stored (consts), else recomputed from the replicas.
DEV void bn_channel_bwd(const BNArgs& a, int z, int c, float& scale, float& shift, float& mean, float& inv) {
  if (a.consts) {
    const float* k = a.consts + (int64_t)z * 4 * a.C;
    scale = k[c]; shift = k[a.C + c]; mean = k[2 * a.C + c]; inv = k[3 * a.C + c];
  } else {
    bn_channel(a, z, c, false, scale, shift, mean, inv);
  }
}

// All C channels into LDS (mean / invstd arrays optional -- needed by backward kernels).  The block that
// updates the running statistics also publishes the batch constants (BNArgs::consts) for the backward.
DEV void bn_prepare(const BNArgs& a, int z, float* s_scale, float* s_shift, float* s_mean, float* s_invstd,
                    bool update_running) {
  float* kz = (update_running && a.training && a.consts) ? a.consts + (int64_t)z * 4 * a.C : nullptr;
  for (int c = threadIdx.x; c < a.C; c += blockDim.x) {
    float sc, sh, mu, inv;
    bn_channel(a, z, c, update_running, sc, sh, mu, inv);
    s_scale[c] = sc;
    s_shift[c] = sh;
    if (s_mean) s_mean[c] = mu;
    if (s_invstd) s_invstd[c] = inv;
    if (kz) { kz[c] = sc; kz[a.C + c] = sh; kz[2 * a.C + c] = mu; kz[3 * a.C + c] = inv; }
  }
  if (update_running && a.training && threadIdx.x == 0 && a.nbt) a.nbt[z] += 1;
}

}  // namespace mda
