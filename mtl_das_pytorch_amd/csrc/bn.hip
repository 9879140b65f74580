// Fused training-mode BatchNorm tails (forward) and BatchNorm backward for NHWC bf16 activations.
//
// Forward "tails" consume the pre-BN conv output y (whose per-channel sums were accumulated by the
// conv epilogue) and fuse everything that follows a BN in the reference models:
//   ACT_NONE / ACT_RELU / ACT_SIGMOID  BN -> act                  (modelA conv1, resblock left.1-2,
//                                                                 att gen .1-.2, Inception BasicConv2d)
//   SIGMUL     sigmoid(BN(y)) * F      attention mask applied to the shared feature
//                                       (modelA_MTL.py:42-50 + :144,151,157,163)
//   ADD_RELU   relu(BN(y) + BN2(y2))  or relu(BN(y) + x): ResBlock tail (modelA_MTL.py:27-32)
//   POOL_RELU  maxpool2x2_ceil(relu(BN(y))) written straight into the upper half of the next level's
//              concat input (modelA_MTL.py:101-116, 145-159) -- no torch.cat, no pool indices stored.
// Block 0 of each group also updates running_mean / running_var (momentum, unbiased variance) and
// num_batches_tracked, matching nn.BatchNorm2d in train mode.
//
// Backward is two launches per fused op: `reduce` recomputes dz (the gradient w.r.t. the BN output)
// from the saved bf16 y and the upstream bf16 gradients (summed in fp32), and accumulates sum(dz), sum(dz * xhat);
// `apply` recomputes dz and writes dy = gamma*invstd*(dz - mean(dz) - xhat*mean(dz*xhat)) as the bf16
// operand of the conv dgrad/wgrad, and block 0 stores d(gamma), d(beta) into the flat gradient buffer.
// Side outputs (written once, bf16): SIGMUL -> g*sigmoid (gradient of the shared feature F),
// ADD_RELU with identity shortcut -> dz (gradient of the block input through the shortcut).
#include "kernels.h"

namespace mda {

// Kernel-internal kind: ADD_RELU with a BN'ed (projection) residual.  Splitting it from the identity-shortcut
// ADD_RELU at compile time keeps the BN2 constants, xhat2 and its accumulators out of the identity kernels'
// registers (occupancy).  The host API keeps ADD_RELU + TailArgs::r_bn.
constexpr int ADD_RELU2 = 6;
template <int K>
DEV constexpr bool is_add() { return K == ADD_RELU || K == ADD_RELU2; }



// sum of replicas q, q + Q, ... < R of a [R][stride] fp64 array (fixed trip count, predicated)
template <int R, int Q>
DEV double rep_sum_q(const double* b, int64_t stride, int q) {
  double v = 0.0;
#pragma unroll
  for (int i = 0; i < (R + Q - 1) / Q; ++i) {
    const int r = q + i * Q;
    if (r < R) v += b[(int64_t)r * stride];
  }
  return v;
}

// thread -> (channel group, pixel lane) mapping shared by every kernel here
struct Lanes {
  int CG, PL, cg, pl;
  bool active;
  DEV Lanes(int C) {
    CG = C >> 3;
    PL = 256 / CG;
    cg = threadIdx.x % CG;
    pl = threadIdx.x / CG;
    active = pl < PL;
  }
};

// bx / nbx: this block's index among the tail's blocks and their count (the grid's x, or a job's share of a
// batched launch)
template <int KIND>
DEV void tail_fwd_impl(const TailArgs& a, const int bx, const int nbx, const int z) {
  extern __shared__ float sm[];
  float* s_sc = sm;
  float* s_sh = sm + a.C;
  float* s_sc2 = sm + 2 * a.C;
  float* s_sh2 = sm + 3 * a.C;
  const bool upd = bx == 0;
  ptick(a.ptm, 0);
  bn_prepare(a.bn, z, s_sc, s_sh, nullptr, nullptr, upd);
  if (KIND == ADD_RELU2) bn_prepare(a.bn2, z, s_sc2, s_sh2, nullptr, nullptr, upd);
  __syncthreads();
  ptick(a.ptm, 1);
  Lanes L(a.C);
  if (!L.active) return;
  const int c = L.cg * 8;
  const bf16_t* yz = a.y + a.ygs * z;
  bf16_t* oz = a.out + a.ogs * z;
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = s_sc[c + j]; sh[j] = s_sh[c + j]; }

  if (KIND == POOL_RELU) {
    const int Hp = (a.H + 1) >> 1, Wp = (a.W + 1) >> 1;
    const int Mp = a.B * Hp * Wp;
    for (int p = bx * L.PL + L.pl; p < Mp; p += nbx * L.PL) {
      int b = p / (Hp * Wp), r = p - b * Hp * Wp;
      int hp = r / Wp, wp = r - hp * Wp;
      float mx[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) mx[j] = 0.f;  // relu output >= 0, window never empty
      for (int dh = 0; dh < 2; ++dh) {
        int h = 2 * hp + dh;
        if (h >= a.H) break;
        for (int dw = 0; dw < 2; ++dw) {
          int w = 2 * wp + dw;
          if (w >= a.W) break;
          float v[8];
          load8(yz + ((int64_t)(b * a.H + h) * a.W + w) * a.ldy + c, v);
#pragma unroll
          for (int j = 0; j < 8; ++j) mx[j] = fmaxf(mx[j], v[j] * sc[j] + sh[j]);
        }
      }
      store8(oz + (int64_t)p * a.ldo + c, mx);
    }
    return;
  }

  float sc2[8], sh2[8];
  if (KIND == ADD_RELU2) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc2[j] = s_sc2[c + j]; sh2[j] = s_sh2[c + j]; }
  }
  const bf16_t* rz = a.r ? a.r + a.rgs * z : nullptr;
  const int M = a.B * a.H * a.W;
  // two pixels per iteration, every load of both issued before the first store: the stores may alias the
  // inputs as far as the compiler knows, so a one-pixel loop keeps one pixel's loads in flight per thread
  // (the large maps -- Model C's 47x122 stem -- then ran at ~2 TB/s)
  constexpr bool RES = KIND == SIGMUL || is_add<KIND>();
  const int step = nbx * L.PL;
  for (int p = bx * L.PL + L.pl; p < M; p += 2 * step) {
    const int p2 = p + step;
    const bool has2 = p2 < M;
    const int q2 = has2 ? p2 : p;
    const uint4 uy[2] = {*reinterpret_cast<const uint4*>(yz + (int64_t)p * a.ldy + c),
                         *reinterpret_cast<const uint4*>(yz + (int64_t)q2 * a.ldy + c)};
    uint4 ur[2] = {make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (RES) {
      ur[0] = *reinterpret_cast<const uint4*>(rz + (int64_t)p * a.ldr + c);
      ur[1] = *reinterpret_cast<const uint4*>(rz + (int64_t)q2 * a.ldr + c);
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !has2) break;
      float v[8];
      unpack8(uy[h], v);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = v[j] * sc[j] + sh[j];
      if (KIND == ACT_RELU) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j], 0.f);
      } else if (KIND == ACT_SIGMOID) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = sigmoidf_(v[j]);
      } else if (KIND == SIGMUL) {
        float f[8];
        unpack8(ur[h], f);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = sigmoidf_(v[j]) * f[j];
      } else if (is_add<KIND>()) {
        float f[8];
        unpack8(ur[h], f);
        if (KIND == ADD_RELU2) {
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = f[j] * sc2[j] + sh2[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaxf(v[j] + f[j], 0.f);
      }
      store8(oz + (int64_t)(h ? p2 : p) * a.ldo + c, v);
    }
  }
  ptick(a.ptm, 3);
}

// Default register allocation: ~100 VGPRs (4 waves per SIMD) for most kinds, which keeps bn_prepare's fp64
// replica loads in flight.  Budgets measured slower: 6 waves per SIMD (<= 85 VGPRs) A 33.5k -> 30.3k samples/s
// (round 3), 8 waves +170 us on Model A's forward (round 2; docs/PERF.md).
template <int KIND>
__global__ __launch_bounds__(256) void tail_fwd_kernel(TailArgs a) {
  tail_fwd_impl<KIND>(a, blockIdx.x, gridDim.x, blockIdx.z);
}

// Several tails of one kind in one launch (engine/inception.py: the BN+ReLU tails of an Inception block's
// branch outputs, which all land in the block's concat buffer and are only read by the next block): block ->
// job by binary search over the jobs' first blocks.  The branch streams each ended in their own small tail
// (Model C: 44 launches of 4-8 us on 4x13 / 1x6 maps); one launch after the block's join does them all.
template <int KIND>
__global__ __launch_bounds__(256) void tail_fwd_batched_kernel(const TailJob* __restrict__ jobs, int nj) {
  int lo = 0, hi = nj - 1;
  while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (jobs[mid].block0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1; }
  const TailJob& J = jobs[lo];
  tail_fwd_impl<KIND>(J.a, (int)blockIdx.x - J.block0, J.blocks, 0);
}

// ------------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------------
// Per-thread views of the block's BN constants in LDS (8 channels per array).  Reading them where they are
// used instead of caching 64 floats in registers keeps the BN-backward kernels' VGPR count -- and so their
// occupancy, which these latency-bound passes depend on -- down.
struct BwdCtx {
  const float *sc, *sh, *mean, *inv;
  const float *sc2, *sh2, *mean2, *inv2;
};

// dz for the 8 channels [c, c+8) at pre-pool pixel p; also returns xhat (and xhat2 for ADD_RELU+BN2)
// and the side output value.
template <int KIND>
DEV void compute_dz(const TailArgs& a, const BwdCtx& X, int z, int p, int c, float* dz, float* xh, float* xh2,
                    float* side) {
  const bf16_t* yz = a.y + a.ygs * z;
  float y[8];
  load8(yz + (int64_t)p * a.ldy + c, y);
#pragma unroll
  for (int j = 0; j < 8; ++j) xh[j] = (y[j] - X.mean[j]) * X.inv[j];
  if (KIND == POOL_RELU) {
    const int HW = a.H * a.W;
    int b = p / HW, r = p - b * HW;
    int h = r / a.W, w = r - h * a.W;
    const int Hp = (a.H + 1) >> 1, Wp = (a.W + 1) >> 1;
    const int hp = h >> 1, wp = w >> 1;
    float g[8];
    gsum8(a.g, z, (int64_t)(b * Hp + hp) * Wp + wp, c, g);
    // window argmax (first max in row-major scan, as torch max_pool2d) of relu(BN(y))
    float mx[8];
    int am[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { mx[j] = -1.f; am[j] = -1; }
    for (int dh = 0; dh < 2; ++dh) {
      int hh = 2 * hp + dh;
      if (hh >= a.H) break;
      for (int dw = 0; dw < 2; ++dw) {
        int ww = 2 * wp + dw;
        if (ww >= a.W) break;
        float v[8];
        load8(yz + ((int64_t)(b * a.H + hh) * a.W + ww) * a.ldy + c, v);
        int id = dh * 2 + dw;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float t = fmaxf(v[j] * X.sc[j] + X.sh[j], 0.f);
          if (t > mx[j]) { mx[j] = t; am[j] = id; }
        }
      }
    }
    const int me = (h - 2 * hp) * 2 + (w - 2 * wp);
#pragma unroll
    for (int j = 0; j < 8; ++j) dz[j] = (am[j] == me && mx[j] > 0.f) ? g[j] : 0.f;
    return;
  }
  float g[8];
  gsum8(a.g, z, p, c, g);
  if (KIND == ACT_NONE) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dz[j] = g[j];
  } else if (KIND == ACT_RELU) {
#pragma unroll
    for (int j = 0; j < 8; ++j) dz[j] = (y[j] * X.sc[j] + X.sh[j]) > 0.f ? g[j] : 0.f;
  } else if (KIND == ACT_SIGMOID) {
#pragma unroll
    for (int j = 0; j < 8; ++j) { float s = sigmoidf_(y[j] * X.sc[j] + X.sh[j]); dz[j] = g[j] * s * (1.f - s); }
  } else if (KIND == SIGMUL) {
    float f[8];
    load8(a.r + a.rgs * z + (int64_t)p * a.ldr + c, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float s = sigmoidf_(y[j] * X.sc[j] + X.sh[j]);
      dz[j] = g[j] * f[j] * s * (1.f - s);
      side[j] = g[j] * s;
    }
  } else if (is_add<KIND>()) {
    float f[8];
    load8(a.r + a.rgs * z + (int64_t)p * a.ldr + c, f);
    if (KIND == ADD_RELU2) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        xh2[j] = (f[j] - X.mean2[j]) * X.inv2[j];
        f[j] = f[j] * X.sc2[j] + X.sh2[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      dz[j] = (y[j] * X.sc[j] + X.sh[j] + f[j]) > 0.f ? g[j] : 0.f;
      side[j] = dz[j];
    }
  }
}

// ------------------------------------------------------------------------------------------------
// Two-launch BN backward, 2-D tiled: block (chunk, cb, z) owns 8*CGB channels [8*CGB*cb, ...) of group z
// over the pixel chunk [chunk*P, (chunk+1)*P); thread = (channel group cgl = tid % CGB, pixel lane
// tid / CGB), so a wave reads whole NHWC pixel rows (coalesced) for C <= 64 and 64-channel slices above.
// Block partials go into NREP fp64 replicas (atomics on rows chunk % NREP; fp64 makes the summation
// order immaterial after rounding, as for the forward statistics) and the apply sums the NREP replicas of
// its channels.  Per-block cross-lane reductions are strided DPP
// row shifts (lanes of the same channel group are CGB apart), finished in LDS over the block's 16 rows.
// Optionally the reduce stores dz (bf16) so the apply does not re-read multi-source gradients or re-evaluate
// 2x2 pool windows.  The statistics are accumulated from the unrounded fp32 dz, as autocast's fp32 BN
// backward computes them (sum(dz * xhat) is a cancelling sum: rounding dz first costs ~1e-3 in d(gamma));
// only the apply's dz operand carries the bf16 rounding, on a bf16 output.
constexpr int BNB_T = 256;

// channel groups of 8 per block: whole rows for C <= 64 (C/8 must be divisible), 64-channel slices above
int bnb_cgb(int C) {
  const int cg = C / 8;
  for (int g = 8; g > 1; g >>= 1)
    if (cg % g == 0) return g;
  return 1;
}

// Row-strided sum: lanes i, i-S, i-2S ... of each 16-lane row; the row totals of the S lane classes end
// up in lanes 16-S .. 15 of the row.
template <int S>
DEV float row_stride_sum(float v) {
  if (S <= 1) v += dpp_f<0x111>(v);
  if (S <= 2) v += dpp_f<0x112>(v);
  if (S <= 4) v += dpp_f<0x114>(v);
  if (S <= 8) v += dpp_f<0x118>(v);
  return v;
}

// BN constants of the thread's 8 channels (BN1 and, for the residual projection, BN2)
template <int KIND, int CGB>
DEV void bnb_ctx(const TailArgs& a, int z, int cblk, int cgl, BwdCtx& X, float (*s_x)[5][8 * CGB]) {
  constexpr bool two = KIND == ADD_RELU2;
  for (int t = threadIdx.x; t < (two ? 2 : 1) * 8 * CGB; t += BNB_T) {
    const int k = t / (8 * CGB), j = t - k * 8 * CGB;
    const BNArgs& bk = k ? a.bn2 : a.bn;
    float sc, sh, mu, inv;
    bn_channel_bwd(bk, z, cblk + j, sc, sh, mu, inv);
    s_x[k][0][j] = sc; s_x[k][1][j] = sh; s_x[k][2][j] = mu; s_x[k][3][j] = inv;
    s_x[k][4][j] = bk.gamma[bk.pstride * z + cblk + j];
  }
  __syncthreads();
  const int q = cgl * 8;
  X.sc = &s_x[0][0][q]; X.sh = &s_x[0][1][q]; X.mean = &s_x[0][2][q]; X.inv = &s_x[0][3][q];
  X.sc2 = &s_x[1][0][q]; X.sh2 = &s_x[1][1][q]; X.mean2 = &s_x[1][2][q]; X.inv2 = &s_x[1][3][q];
}

// chunk / cy / z: the block's pixel chunk, channel block and group (the grid's x / y / z, or a job's share
// of a batched launch)
template <int KIND, int CGB>
DEV void bnb_reduce_impl(const TailArgs& a, const int chunk, const int cy, const int z) {
  constexpr int PL = BNB_T / CGB, CB = 8 * CGB;
  __shared__ float s_x[2][5][CB];
  __shared__ float s_part[16][3][CB];  // 16 rows of 16 lanes per block
  const int cgl = threadIdx.x % CGB, pl = threadIdx.x / CGB;
  const int cblk = cy * CB, c = cblk + cgl * 8;
  constexpr bool two = KIND == ADD_RELU2;
  BwdCtx X;
  bnb_ctx<KIND, CGB>(a, z, cblk, cgl, X, s_x);
  const int M = a.B * a.H * a.W;
  const int p0 = chunk * a.chunk_px, p1 = min(M, p0 + a.chunk_px);
  float sdz[8], sdx[8], sdx2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sdz[j] = 0.f; sdx[j] = 0.f; sdx2[j] = 0.f; }
  bf16_t* dzz = a.dzbuf ? a.dzbuf + a.dzgs * z : nullptr;
  for (int p = p0 + pl; p < p1; p += PL) {
    float dz[8], xh[8], xh2[8], side[8];
    compute_dz<KIND>(a, X, z, p, c, dz, xh, xh2, side);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sdz[j] += dz[j];
      sdx[j] += dz[j] * xh[j];
      if (two) sdx2[j] += dz[j] * xh2[j];
    }
    if ((KIND == SIGMUL || KIND == ADD_RELU) && a.side)
      store8(a.side + a.sgs * z + (int64_t)p * a.lds + c, side);
    if (dzz) store8(dzz + (int64_t)p * a.lddz + c, dz);
  }
  const int lane = threadIdx.x & 63, row = threadIdx.x >> 4;
  const bool top = (lane & 15) >= 16 - CGB;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float t0 = row_stride_sum<CGB>(sdz[j]), t1 = row_stride_sum<CGB>(sdx[j]);
    const float t2 = two ? row_stride_sum<CGB>(sdx2[j]) : 0.f;
    if (top) { s_part[row][0][cgl * 8 + j] = t0; s_part[row][1][cgl * 8 + j] = t1; s_part[row][2][cgl * 8 + j] = t2; }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 3 * CB; t += BNB_T) {
    const int k = t / CB, q = t - k * CB;
    float v = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) v += s_part[r][k][q];
    atomicAdd(a.part + (((int64_t)z * NREP + chunk % a.bn.pnrep) * 3 + k) * a.C + cblk + q, (double)v);
  }
}

template <int KIND, int CGB>
DEV void bnb_apply_impl(const TailArgs& a, const int chunk, const int cy, const int z) {
  constexpr int PL = BNB_T / CGB, CB = 8 * CGB;
  __shared__ float s_x[2][5][CB];
  __shared__ float s_red[BNB_T];
  __shared__ float s_coef[2][3][CB];
  const int cgl = threadIdx.x % CGB, pl = threadIdx.x / CGB;
  const int cblk = cy * CB, c = cblk + cgl * 8;
  constexpr bool two = KIND == ADD_RELU2;
  ptick(a.ptm, 0);
  BwdCtx X;
  bnb_ctx<KIND, CGB>(a, z, cblk, cgl, X, s_x);
  // the NREP replicas of this block's channels: item = (stat, channel), Q threads per item
  constexpr int NI = 3 * CB;
  constexpr int Q = BNB_T / NI > 0 ? BNB_T / NI : 1;
  {
    const double* base = a.part + (int64_t)z * NREP * 3 * a.C + cblk;
    for (int t = threadIdx.x; t < NI * Q; t += BNB_T) {
      const int item = t % NI, q = t / NI;
      const int k = item / CB, j = item - k * CB;
      const double* b = base + (int64_t)k * a.C + j;
      double v;
      switch (a.bn.pnrep) {  // compile-time trip counts: every replica load in flight at once
        case 1: v = rep_sum_q<1, Q>(b, 3 * a.C, q); break;
        case 2: v = rep_sum_q<2, Q>(b, 3 * a.C, q); break;
        case 4: v = rep_sum_q<4, Q>(b, 3 * a.C, q); break;
        case 8: v = rep_sum_q<8, Q>(b, 3 * a.C, q); break;
        case 16: v = rep_sum_q<16, Q>(b, 3 * a.C, q); break;
        default: v = rep_sum_q<NREP, Q>(b, 3 * a.C, q); break;
      }
      s_red[q * NI + item] = (float)v;
    }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < (two ? 2 : 1) * CB; t += BNB_T) {
    const int k = t / CB, j = t - k * CB;  // k: BN1 / BN2
    float sd = 0.f, sx = 0.f;
    for (int q = 0; q < Q; ++q) { sd += s_red[q * NI + j]; sx += s_red[q * NI + (k ? 2 : 1) * CB + j]; }
    const BNArgs& bk = k ? a.bn2 : a.bn;
    const float inv_n = 1.f / (float)bk.count;
    const float g = s_x[k][4][j], inv = s_x[k][3][j], mu = s_x[k][2][j];
    const float mdz = sd * inv_n, mdx = sx * inv_n;
    s_coef[k][0][j] = g * inv;                            // dy = A*dz + B*y + C
    s_coef[k][1][j] = -g * inv * inv * mdx;
    s_coef[k][2][j] = g * inv * (mu * inv * mdx - mdz);
    if (chunk == 0) {
      float* dg = k ? a.dgamma2 : a.dgamma;
      float* db = k ? a.dbeta2 : a.dbeta;
      if (dg) dg[a.pgs * z + cblk + j] = sx * a.gscale;
      if (db) db[a.pgs * z + cblk + j] = sd * a.gscale;
    }
  }
  __syncthreads();
  ptick(a.ptm, 1);
  const float *A1 = &s_coef[0][0][cgl * 8], *B1 = &s_coef[0][1][cgl * 8], *C1 = &s_coef[0][2][cgl * 8];
  const float *A2 = &s_coef[1][0][cgl * 8], *B2 = &s_coef[1][1][cgl * 8], *C2 = &s_coef[1][2][cgl * 8];
  const int M = a.B * a.H * a.W;
  const int p0 = chunk * a.chunk_px, p1 = min(M, p0 + a.chunk_px);
  const bf16_t* yz = a.y + a.ygs * z;
  const bf16_t* dzz = a.dzbuf ? a.dzbuf + a.dzgs * z : nullptr;
  for (int p = p0 + pl; p < p1; p += PL) {
    float dz[8], y[8], o[8];
    if (dzz) {
      load8(dzz + (int64_t)p * a.lddz + c, dz);
    } else {
      float xh[8], xh2[8], side[8];
      compute_dz<KIND>(a, X, z, p, c, dz, xh, xh2, side);
      if ((KIND == SIGMUL || KIND == ADD_RELU) && a.side && a.apply_side)
        store8(a.side + a.sgs * z + (int64_t)p * a.lds + c, side);
    }
    load8(yz + (int64_t)p * a.ldy + c, y);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = A1[j] * dz[j] + B1[j] * y[j] + C1[j];
    store8(a.dy + a.dgs * z + (int64_t)p * a.ldd + c, o);
    if (two) {
      float y2[8];
      load8(a.r + a.rgs * z + (int64_t)p * a.ldr + c, y2);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = A2[j] * dz[j] + B2[j] * y2[j] + C2[j];
      store8(a.dy2 + a.d2gs * z + (int64_t)p * a.ldd2 + c, o);
    }
  }
  ptick(a.ptm, 3);
}

// Kernels: plain, and with the register budget of 5 waves per SIMD (<= 96 VGPRs) for the kinds that fit it
// without spilling (every kind but the two-BN residual tail and the pooling tail).
// These passes are latency-bound, and occupancy is what hides the latency (measured: forward tails at 4
// instead of 6 waves per SIMD cost Model A 150 us per step).
template <int KIND, int CGB>
__global__ __launch_bounds__(BNB_T) void bnb_reduce_kernel(TailArgs a) {
  bnb_reduce_impl<KIND, CGB>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}
template <int KIND, int CGB, int W>
__global__ __launch_bounds__(BNB_T) __attribute__((amdgpu_waves_per_eu(W))) void bnb_reduce_kernel_w(TailArgs a) {
  bnb_reduce_impl<KIND, CGB>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}
template <int KIND, int CGB>
__global__ __launch_bounds__(BNB_T) void bnb_apply_kernel(TailArgs a) {
  bnb_apply_impl<KIND, CGB>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}
template <int KIND, int CGB, int W>
__global__ __launch_bounds__(BNB_T) __attribute__((amdgpu_waves_per_eu(W))) void bnb_apply_kernel_w(TailArgs a) {
  bnb_apply_impl<KIND, CGB>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Several BN-tail backward passes of one kind in one launch (engine/inception.py: the branch-output tails of
// an Inception block, whose gradient sources all complete at the block's backward fork): block -> job by
// binary search; a job's blocks are its (chunk, channel block) grid, chunk fastest.  REDUCE: the reduce
// pass, else the apply pass.
template <int KIND, int CGB, int W, bool REDUCE>
__global__ __launch_bounds__(BNB_T) __attribute__((amdgpu_waves_per_eu(W))) void bnb_batched_kernel(
    const TailJob* __restrict__ jobs, int nj) {
  int lo = 0, hi = nj - 1;
  while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (jobs[mid].block0 <= (int)blockIdx.x) lo = mid; else hi = mid - 1; }
  const TailJob& J = jobs[lo];
  const int local = (int)blockIdx.x - J.block0;
  const int nchunk = J.blocks / (J.a.C / (8 * CGB));
  const int cy = local / nchunk, chunk = local - cy * nchunk;
  if (REDUCE) bnb_reduce_impl<KIND, CGB>(J.a, chunk, cy, 0);
  else bnb_apply_impl<KIND, CGB>(J.a, chunk, cy, 0);
}
// waves per SIMD each kind's passes fit without spilling (hipcc -Rpass-analysis=kernel-resource-usage, gfx950);
// 0 = the compiler's default allocation
template <int KIND>
constexpr int bnb_waves() {
  return KIND == ACT_NONE ? 8 : (KIND == ACT_RELU || KIND == ACT_SIGMOID) ? 6 : (KIND == SIGMUL || KIND == ADD_RELU) ? 5 : 0;
}
// Single-launch BN backward for small maps: block (cg, -, z) owns channels [8cg, 8cg+8) for ALL M
// pixels, so the batch reduction is a block reduction (no global atomics, no second launch, exact and
// deterministic).  Each of the 1024 threads keeps the dz / xhat of its R <= 4 pixels in registers, so
// the kernel is just: statistics + gamma (one round trip) -> pixel loads -> block reduction -> stores.
// The autotuner picks it per layer against reduce+apply; it wins where launch and memory latency
// dominate (deep Model A levels, most of Inception-v3 at 100x250).
constexpr int FUSED_T = 1024;
template <int KIND, int R>
__global__ __launch_bounds__(FUSED_T) void tail_bwd_fused_kernel(TailArgs a) {
  __shared__ float s_x[2][5][8];                // BN1/BN2 x (scale, shift, mean, invstd, gamma) x 8 ch
  __shared__ float s_part[FUSED_T / 64][3][8];  // per-wave partial sums
  __shared__ float s_coef[2][3][8];             // dy = A*dz + Bx*xhat + Cc (BN1, BN2)
  const int z = blockIdx.z;
  const int c = blockIdx.x * 8;
  constexpr bool two = KIND == ADD_RELU2;
  const bool tick = a.tsc && blockIdx.x == 0 && blockIdx.z == 0 && threadIdx.x == 0;
#define TICK(i) if (tick) a.tsc[i] = wall_clock64()
  TICK(0);
  if (threadIdx.x < (two ? 16 : 8)) {
    const int k = threadIdx.x >> 3, j = threadIdx.x & 7;
    const BNArgs& bk = k ? a.bn2 : a.bn;
    float sc, sh, mu, inv;
    bn_channel_bwd(bk, z, c + j, sc, sh, mu, inv);
    s_x[k][0][j] = sc; s_x[k][1][j] = sh; s_x[k][2][j] = mu; s_x[k][3][j] = inv;
    s_x[k][4][j] = bk.gamma[bk.pstride * z + c + j];
  }
  __syncthreads();
  TICK(1);
  BwdCtx X;
  X.sc = s_x[0][0]; X.sh = s_x[0][1]; X.mean = s_x[0][2]; X.inv = s_x[0][3];
  X.sc2 = s_x[1][0]; X.sh2 = s_x[1][1]; X.mean2 = s_x[1][2]; X.inv2 = s_x[1][3];
  const int M = a.B * a.H * a.W;
  float sdz[8], sdx[8], sdx2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sdz[j] = 0.f; sdx[j] = 0.f; sdx2[j] = 0.f; }
  float dzc[R][8], xhc[R][8], xh2c[R][8];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p = threadIdx.x + r * FUSED_T;
    float side[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { dzc[r][j] = 0.f; xhc[r][j] = 0.f; xh2c[r][j] = 0.f; }
    if (p < M) {
      compute_dz<KIND>(a, X, z, p, c, dzc[r], xhc[r], xh2c[r], side);
      if ((KIND == SIGMUL || KIND == ADD_RELU) && a.side)
        store8(a.side + a.sgs * z + (int64_t)p * a.lds + c, side);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      sdz[j] += dzc[r][j];
      sdx[j] += dzc[r][j] * xhc[r][j];
      if (two) sdx2[j] += dzc[r][j] * xh2c[r][j];
    }
  }
  TICK(2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t0 = wave_sum(sdz[j]), t1 = wave_sum(sdx[j]);
    float t2 = two ? wave_sum(sdx2[j]) : 0.f;
    if (lane == 0) { s_part[wid][0][j] = t0; s_part[wid][1][j] = t1; s_part[wid][2][j] = t2; }
  }
  __syncthreads();
  TICK(3);
  if (threadIdx.x < (two ? 16 : 8)) {
    const int k = threadIdx.x >> 3, j = threadIdx.x & 7;
    float sd = 0.f, sx = 0.f;
#pragma unroll
    for (int w = 0; w < FUSED_T / 64; ++w) { sd += s_part[w][0][j]; sx += s_part[w][k ? 2 : 1][j]; }
    const BNArgs& bk = k ? a.bn2 : a.bn;
    const float inv_n = 1.f / (float)bk.count;
    const float ginv = s_x[k][4][j] * s_x[k][3][j];
    s_coef[k][0][j] = ginv;                  // dy = g*inv*(dz - mean(dz) - xhat*mean(dz*xhat))
    s_coef[k][1][j] = -ginv * sx * inv_n;
    s_coef[k][2][j] = -ginv * sd * inv_n;
    float* dg = k ? a.dgamma2 : a.dgamma;
    float* db = k ? a.dbeta2 : a.dbeta;
    if (dg) dg[a.pgs * z + c + j] = sx;
    if (db) db[a.pgs * z + c + j] = sd;
  }
  __syncthreads();
  TICK(4);
  const float *A1 = s_coef[0][0], *B1 = s_coef[0][1], *C1 = s_coef[0][2];
  const float *A2 = s_coef[1][0], *B2 = s_coef[1][1], *C2 = s_coef[1][2];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int p = threadIdx.x + r * FUSED_T;
    if (p >= M) break;
    float o[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = A1[j] * dzc[r][j] + B1[j] * xhc[r][j] + C1[j];
    store8(a.dy + a.dgs * z + (int64_t)p * a.ldd + c, o);
    if (two) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = A2[j] * dzc[r][j] + B2[j] * xh2c[r][j] + C2[j];
      store8(a.dy2 + a.d2gs * z + (int64_t)p * a.ldd2 + c, o);
    }
  }
  TICK(5);
#undef TICK
}

// ------------------------------------------------------------------------------------------------
int launch_tail_fwd(int kind, const TailArgs& a, int G, int blocks, hipStream_t st) {
  size_t lds = (size_t)4 * a.C * sizeof(float);
  dim3 grid(blocks, 1, G);
  const int kk = (kind == ADD_RELU && a.r_bn) ? ADD_RELU2 : kind;
#define K(X) case X: hipLaunchKernelGGL(tail_fwd_kernel<X>, grid, dim3(256), lds, st, a); break;
  switch (kk) {
    K(ACT_NONE) K(ACT_RELU) K(ACT_SIGMOID) K(SIGMUL) K(POOL_RELU) K(ADD_RELU) K(ADD_RELU2)
#undef K
    default: return -1;
  }
  return (int)hipGetLastError();
}

// Batched BN-tail backward of ACT_RELU tails (kind 1, no residual / side outputs): the reduce pass of the jobs
// that need one (``reduce``), then the apply pass of all.  cgb: channel groups per block, dividing every job's
// C / 8; each job's ``blocks`` = nchunk * C / (8 * cgb).
int launch_tail_bwd_batched(int kind, int cgb, int reduce, const TailJob* d_jobs, int nj, int nblocks, hipStream_t st) {
  if (nblocks <= 0) return 0;
  if (kind != ACT_RELU) return -1;
#define KB(CG)                                                                                                    \
  if (reduce)                                                                                                     \
    hipLaunchKernelGGL((bnb_batched_kernel<ACT_RELU, CG, bnb_waves<ACT_RELU>(), true>), dim3(nblocks), dim3(BNB_T), \
                       0, st, d_jobs, nj);                                                                        \
  else                                                                                                            \
    hipLaunchKernelGGL((bnb_batched_kernel<ACT_RELU, CG, bnb_waves<ACT_RELU>(), false>), dim3(nblocks),            \
                       dim3(BNB_T), 0, st, d_jobs, nj);
  switch (cgb) {
    case 1: KB(1) break;
    case 2: KB(2) break;
    case 4: KB(4) break;
    case 8: KB(8) break;
    default: return -1;
  }
#undef KB
  return (int)hipGetLastError();
}

int launch_tail_fwd_batched(int kind, const TailJob* d_jobs, int nj, int nblocks, int maxC, hipStream_t st) {
  if (nblocks <= 0) return 0;
  const size_t lds = (size_t)4 * maxC * sizeof(float);
#define K(X) case X: hipLaunchKernelGGL(tail_fwd_batched_kernel<X>, dim3(nblocks), dim3(256), lds, st, d_jobs, nj); break;
  switch (kind) {
    K(ACT_NONE) K(ACT_RELU) K(ACT_SIGMOID)
#undef K
    default: return -1;  // kinds with a second operand or a pooled grid are not batched
  }
  return (int)hipGetLastError();
}

// fused: 0 = reduce + apply, 1 = single-launch kernel (small maps), 2 = apply only -- the statistics were
// accumulated into `part` by the epilogue of the dgrad that produced the (single) gradient source.
// 3 = reduce only: partial statistics over a SUBSET of the gradient sources (the rest are added by their
// producers), no side / dz / dy outputs -- the tail's own launch is then fused == 2.
int launch_tail_bwd(int kind, const TailArgs& a, int G, int nchunk, int fused, hipStream_t st) {
  if (fused == 2 && a.dzbuf) return -5;  // apply-only recomputes dz from the sources (every kind)
  if (fused == 3 && (a.dzbuf || a.dy || a.side || a.dgamma || a.dbeta)) return -5;
  TailArgs b = a;
  b.apply_side = fused == 2;
  const int kk = (kind == ADD_RELU && a.r_bn) ? ADD_RELU2 : kind;  // kernel kind
  if (fused == 1) {
    if (a.gscale != 1.f) return -5;
    const int M = a.B * a.H * a.W;
    const int R = (M + FUSED_T - 1) / FUSED_T;
    // register-cached pixels per thread: up to 4 (2 for the two-BN residual tail) without spilling
    if (R > (kind == ADD_RELU ? 2 : 4)) return -3;  // too large: use reduce + apply
    dim3 grid(a.C / 8, 1, G);
#define KR(X, RR) hipLaunchKernelGGL((tail_bwd_fused_kernel<X, RR>), grid, dim3(FUSED_T), 0, st, a)
#define K(X)                                \
  case X:                                   \
    if (R <= 1) KR(X, 1);                   \
    else if (R <= 2) KR(X, 2);              \
    else KR(X, 4);                          \
    break;
    switch (kk) {
      K(ACT_NONE) K(ACT_RELU) K(ACT_SIGMOID) K(SIGMUL) K(ADD_RELU) K(ADD_RELU2) K(POOL_RELU)
      default: return -1;
    }
#undef K
#undef KR
    return (int)hipGetLastError();
  }
  if (!a.part || a.chunk_px <= 0 || nchunk <= 0) return -4;
  const int cgb = bnb_cgb(a.C);
  dim3 grid(nchunk, a.C / (8 * cgb), G);
#define KC(X, CG)                                                                                    \
  if (fused != 2) {                                                                                  \
    if constexpr (bnb_waves<X>() > 0)                                                                \
      hipLaunchKernelGGL((bnb_reduce_kernel_w<X, CG, bnb_waves<X>()>), grid, dim3(BNB_T), 0, st, b); \
    else                                                                                             \
      hipLaunchKernelGGL((bnb_reduce_kernel<X, CG>), grid, dim3(BNB_T), 0, st, b);                   \
  }                                                                                                  \
  if (fused == 3) break;                                                                             \
  if constexpr (bnb_waves<X>() > 0)                                                                  \
    hipLaunchKernelGGL((bnb_apply_kernel_w<X, CG, bnb_waves<X>()>), grid, dim3(BNB_T), 0, st, b);    \
  else                                                                                               \
    hipLaunchKernelGGL((bnb_apply_kernel<X, CG>), grid, dim3(BNB_T), 0, st, b);
#define K(X)                                                   \
  case X:                                                      \
    if (cgb == 1) { KC(X, 1) } else if (cgb == 2) { KC(X, 2) } \
    else if (cgb == 4) { KC(X, 4) } else { KC(X, 8) }          \
    break;
  switch (kk) {
    K(ACT_NONE) K(ACT_RELU) K(ACT_SIGMOID) K(SIGMUL) K(ADD_RELU) K(ADD_RELU2) K(POOL_RELU)
    default: return -1;
  }
#undef K
#undef KC
  return (int)hipGetLastError();
}

}  // namespace mda
