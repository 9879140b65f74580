// Lean im2col weight gradient (configs WGRAD_LEAN_CFG0 .. + WGRAD_LEAN_NCFG - 1).
//
// dW[n][k] = sum over output pixels m of dy[m][n] * X[m][k], X the im2col of the forward input (k = (kh*KW +
// kw)*Cs + ci, the slab layout of every weight-gradient kernel: [G][splits][Npad][Kpad], summed by
// wgrad_finalize).  A block owns a TN x TK output tile and a contiguous pixel range (one M split); it stages 64
// pixels per chunk through LDS (pixel-major images, read back transposed by ds_read_b64_tr_b16 into
// v_mfma_f32_16x16x32_bf16 operands, as wgrad_block does).
//
// What differs from wgrad_block / wgrad_big_block is the staging.  Those kernels were VALU-bound: every 16-byte
// unit of every chunk decomposed its pixel index m into (image, row, column) with two divisions, built a 64-bit
// address, and branched on its bounds (Model A's largest batch ran 7.4 k VALU instructions per wave at ~1 us per
// 64-pixel chunk, MFMA busy 4 %, profiles/r5_pmc_modelA_end.txt; a deeper load pipeline left it unchanged).  Here:
//   * the chunk's 64 pixels are decomposed ONCE, by 64 threads, into a pixel table in LDS (input-pixel base
//     index and the first tap's row / column), double-buffered one chunk ahead so it costs no extra barrier;
//   * everything a thread's 16-byte units need besides the pixel -- the tap (kh, kw), the channel offset, the
//     source segment, the LDS destination -- is fixed for the block and computed once, before the loop;
//   * loads are branch-free: an out-of-image tap or a pixel past the split loads a valid dummy address and is
//     zeroed by a select, so no exec-mask divergence splits the staging;
//   * 32-bit offsets (every operand here is < 2^31 elements; checked on the host).
// Normalise-on-load inputs (the forward conv read act(BN(y))) are rebuilt on the way into LDS, as in wgrad_block.
//
// Configs 44-47 (BIG) are the same staging under wgrad_big_block's compute: 64 x 64 .. 128 x 128 tiles on the
// 32x32x16 MFMA, each wave a (TN/2) x (TK/2) quarter of 32x32 accumulators, 64-pixel chunks -- the throughput
// form for batched launches of many jobs (Model C's Inception weight gradients: lean 16x16 tiles were 2x faster
// per job alone but 45 % slower as batches, profiles/r6_wgrad_lean.md).  They split M like the large tiles
// (engine/core.py wgrad_plan), not like the lean 16x16 configs.
#include "kernels.h"

namespace mda {

// (TN, TK, MCH pixels per chunk, 32x32x16 MFMA); keep in sync with ops/functional.py WGRAD_TILES (entries
// WGRAD_LEAN_CFG0..)
#define WGRAD_LEAN_CASES(X)                                                                                   \
  case 36: X(16, 64, 256, false) case 37: X(16, 144, 128, false) case 38: X(32, 64, 256, false)               \
  case 39: X(32, 144, 128, false) case 40: X(64, 64, 128, false) case 41: X(64, 128, 128, false)              \
  case 42: X(128, 64, 128, false) case 43: X(128, 128, 64, false)                                             \
  case 44: X(64, 64, 64, true) case 45: X(64, 128, 64, true) case 46: X(128, 64, 64, true)                    \
  case 47: X(128, 128, 64, true)

int wgrad_lean_shape(int cfg, int& TN, int& TK) {
  static const int tn[] = {16, 16, 32, 32, 64, 64, 128, 128, 64, 64, 128, 128};
  static const int tk[] = {64, 144, 64, 144, 64, 128, 64, 128, 64, 128, 64, 128};
  if (cfg < WGRAD_LEAN_CFG0 || cfg >= WGRAD_LEAN_CFG0 + WGRAD_LEAN_NCFG) return -1;
  TN = tn[cfg - WGRAD_LEAN_CFG0];
  TK = tk[cfg - WGRAD_LEAN_CFG0];
  return 0;
}

// im2col column group i (8 channels of one tap): channel offset within its source segment | kw << 14 | kh << 21
// | segment << 28 | valid << 29 (0: the group lies past the reduction -- stages zeros)
DEV int lean_encode(int i, int Ktot, int Cs8, int KW, int C0) {
  if (i * 8 >= Ktot) return 0;
  const int tap = i / Cs8, c = (i - tap * Cs8) * 8;
  const int kh = tap / KW, kw = tap - kh * KW;
  const int seg = c >= C0;
  return (seg ? c - C0 : c) | (kw << 14) | (kh << 21) | (seg << 28) | (1 << 29);
}

constexpr int LEAN_BAD_ROW = -16384;  // first-tap row of a pixel past the split: every tap lands outside the image

template <int TN, int TK, int MCH, bool BIG>
DEV void wgrad_lean_block(const WgradArgs& a, const int tile, const int split, const int z) {
  static_assert(MCH % 64 == 0 && MCH <= 256, "chunk of 64..256 pixels (pixel table: one entry per thread)");
  static_assert(!BIG || (TN % 64 == 0 && TK % 64 == 0), "32x32 quarters per wave");
  // row pitches: 16 x odd elements, so the 8 rows a transposed read touches tile the 64 banks (wgrad_block);
  // BIG: width + 32, the 4 rows of a 32-column transposed read on disjoint bank quarters (wgrad_big_block)
  constexpr int LDY = BIG ? TN + 32 : ((TN / 16) % 2 ? TN : TN + 16);
  constexpr int LDX = BIG ? TK + 32 : ((TK / 16) % 2 ? TK : TK + 16);
  constexpr int YG = TN / 8, KG = TK / 8;
  constexpr int VY = MCH * YG, VX = MCH * KG;
  constexpr int NY = (VY + 255) / 256, NX = (VX + 255) / 256;
  constexpr int FN = TN / 16, FK = TK / 16, NFR = FN * FK, FPW = BIG ? 1 : (NFR + 3) / 4;
  constexpr int FA = BIG ? TN / 64 : 1, FB = BIG ? TK / 64 : 1;  // BIG: 32x32 accumulators of a wave
  __shared__ __attribute__((aligned(16))) bf16_t s_dy[MCH * LDY];
  __shared__ __attribute__((aligned(16))) bf16_t s_x[MCH * LDX];
  __shared__ int s_pix[2][MCH];  // (b * Hi + ih0) * Wi + iw0 of the chunk's pixels
  __shared__ int s_ihw[2][MCH];  // ih0 << 16 | (iw0 & 0xffff)
  __shared__ int s_tab[KG];
  __shared__ __attribute__((aligned(16))) float s_nsc[TK], s_nsh[TK];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntk = (a.Kpad + TK - 1) / TK;
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * TN, k0 = tk * TK;
  const int Ktot = a.KH * a.KW * a.Cs;
  const int HWo = a.Ho * a.Wo;
  const float ihwo = 1.f / (float)HWo, iwo = 1.f / (float)a.Wo;
  const int mbeg = split * a.m_per_split, mend = min(a.B * HWo, mbeg + a.m_per_split);
  const bf16_t* base0 = a.src.p[0] + a.src.gs[0] * z;
  const bf16_t* base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : base0;
  const bf16_t* dyz = a.dy + a.dgs * z;

  auto pix_table = [&](int buf, int mc) {
    if (tid < MCH) {
      const int m = mc + tid;
      int pix = 0, ihw = (int)((unsigned)LEAN_BAD_ROW << 16);
      if (m < mend) {
        const int b = fdiv24(m, HWo, ihwo), r = m - b * HWo;
        const int oh = fdiv24(r, a.Wo, iwo), ow = r - oh * a.Wo;
        const int ih0 = oh * a.sh - a.ph, iw0 = ow * a.sw - a.pw;
        pix = (b * a.Hi + ih0) * a.Wi + iw0;
        ihw = (int)(((unsigned)ih0 << 16) | ((unsigned)iw0 & 0xffffu));
      }
      s_pix[buf][tid] = pix;
      s_ihw[buf][tid] = ihw;
    }
  };

  if (tid < KG) s_tab[tid] = lean_encode(k0 / 8 + tid, Ktot, a.Cs >> 3, a.KW, a.src.C0);
  if (a.nol) {
    const float* kz = a.nol_consts + (int64_t)z * 4 * a.Cs;
    for (int t = tid; t < TK; t += 256) {
      const int e = lean_encode(k0 / 8 + t / 8, Ktot, a.Cs >> 3, a.KW, a.src.C0);
      const int c = (e & 16383) + ((e >> 28) & 1) * a.src.C0 + (t & 7);
      const bool ok = (e >> 29) & 1;
      s_nsc[t] = ok ? kz[c] : 0.f;
      s_nsh[t] = ok ? kz[a.Cs + c] : 0.f;
    }
  }
  pix_table(0, mbeg);
  __syncthreads();

  // per-thread constants of its 16-byte staging units, fixed for the block, two words per unit:
  //   xk: pixel-in-chunk | kh << 8 | kw << 15 | segment << 22 | column valid << 23
  //   xo: channel offset within the segment | LDS destination (element offset) << 14
  int xk[NX], xo[NX];
#pragma unroll
  for (int i = 0; i < NX; ++i) {
    const int v = tid + 256 * i;
    const int p = v / KG, g = v - p * KG;
    const int e = v < VX ? s_tab[g] : 0;
    xk[i] = (v < VX ? p : 0) | (((e >> 21) & 127) << 8) | (((e >> 14) & 127) << 15) | (((e >> 28) & 1) << 22) |
            (((e >> 29) & 1) << 23);
    xo[i] = (e & 16383) | ((p * LDX + g * 8) << 14);
  }
  //   yk: pixel-in-chunk | channel valid << 8; yo: channel | LDS destination << 14
  int yk[NY], yo[NY];
#pragma unroll
  for (int j = 0; j < NY; ++j) {
    const int v = tid + 256 * j;
    const int p = v / YG, cg = v - p * YG;
    yk[j] = (v < VY ? p : 0) | ((v < VY && n0 + cg * 8 < a.Co) ? 256 : 0);
    yo[j] = (n0 + cg * 8) | ((p * LDY + cg * 8) << 14);
  }
  const int ld0 = a.src.ld[0], ld1 = a.src.ld[1];

  uint4 rx[NX], ry[NY];
  uint32_t rok = 0;
#define LEAN_LOAD(BUF, MC)                                                                                     \
  do {                                                                                                         \
    rok = 0;                                                                                                   \
    _Pragma("unroll") for (int i = 0; i < NX; ++i) {                                                           \
      const int k = xk[i], p = k & 255, kh = (k >> 8) & 127, kw = (k >> 15) & 127, seg = (k >> 22) & 1;        \
      const int pix = s_pix[BUF][p], ihw = s_ihw[BUF][p];                                                      \
      const int ih = (ihw >> 16) + kh, iw = (int)(short)(ihw & 0xffff) + kw;                                   \
      const bool ok = ((k >> 23) & 1) && (unsigned)ih < (unsigned)a.Hi && (unsigned)iw < (unsigned)a.Wi;       \
      const int off = ok ? (pix + kh * a.Wi + kw) * (seg ? ld1 : ld0) + (xo[i] & 16383) : 0;                  \
      const uint4 u = *reinterpret_cast<const uint4*>((seg ? base1 : base0) + off);                            \
      const uint32_t mk = ok ? 0xffffffffu : 0u; /* (a select of the uint4 went through scratch) */            \
      rx[i] = make_uint4(u.x & mk, u.y & mk, u.z & mk, u.w & mk);                                              \
      rok |= (ok ? 1u : 0u) << i;                                                                              \
    }                                                                                                          \
    _Pragma("unroll") for (int j = 0; j < NY; ++j) {                                                           \
      const int m = (MC) + (yk[j] & 255);                                                                      \
      const bool ok = (yk[j] & 256) && m < mend;                                                               \
      const uint4 u = *reinterpret_cast<const uint4*>(dyz + (ok ? m * a.ldd + (yo[j] & 16383) : 0));           \
      const uint32_t mk = ok ? 0xffffffffu : 0u;                                                               \
      ry[j] = make_uint4(u.x & mk, u.y & mk, u.z & mk, u.w & mk);                                              \
    }                                                                                                          \
  } while (0)

  f32x4 acc[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x16 bacc[FA][FB];
  const int wn = (wid & 1) * (TN / 2), wk = (wid >> 1) * (TK / 2);
  if (BIG) {
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j)
#pragma unroll
        for (int r = 0; r < 16; ++r) bacc[i][j][r] = 0.f;
  }

  if (mbeg < mend) LEAN_LOAD(0, mbeg);
  int buf = 0;
  for (int mc = mbeg; mc < mend; mc += MCH) {
    // stage the loaded chunk into the LDS images (normalise-on-load columns rebuilt on the way)
#pragma unroll
    for (int j = 0; j < NY; ++j)
      if (tid + 256 * j < VY) *reinterpret_cast<uint4*>(&s_dy[yo[j] >> 14]) = ry[j];
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      if (tid + 256 * i < VX) {
        uint4 u = rx[i];
        const int dst = xo[i] >> 14;
        if (a.nol && ((rok >> i) & 1)) {
          const int g8 = dst % LDX;  // 8 * column group
          uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            float lo = __uint_as_float(w4[h] << 16) * s_nsc[g8 + 2 * h] + s_nsh[g8 + 2 * h];
            float hi = __uint_as_float(w4[h] & 0xffff0000u) * s_nsc[g8 + 2 * h + 1] + s_nsh[g8 + 2 * h + 1];
            if (a.nol_kind == ACT_RELU) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
            w4[h] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
          }
          u = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        *reinterpret_cast<uint4*>(&s_x[dst]) = u;
      }
    }
    const bool more = mc + MCH < mend;
    if (more) pix_table(buf ^ 1, mc + MCH);  // (last read by the load of chunk mc, before the previous barrier)
    __syncthreads();
    if (more) LEAN_LOAD(buf ^ 1, mc + MCH);  // in flight during this chunk's MFMAs
    if (BIG) {
#pragma unroll
      for (int ks = 0; ks < MCH / 16; ++ks) {
        bf16x8 av[FA], bv[FB];
#pragma unroll
        for (int i = 0; i < FA; ++i) av[i] = tr_read32(&s_dy[ks * 16 * LDY], LDY, wn + 32 * i, lane);
#pragma unroll
        for (int j = 0; j < FB; ++j) bv[j] = tr_read32(&s_x[ks * 16 * LDX], LDX, wk + 32 * j, lane);
#pragma unroll
        for (int i = 0; i < FA; ++i)
#pragma unroll
          for (int j = 0; j < FB; ++j)
            bacc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], bacc[i][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int kk = 0; kk < (BIG ? 0 : MCH / 32); ++kk) {
      const int prow = kk * 32 + 16 * (lane >> 5) + 4 * ((lane >> 4) & 1);
#pragma unroll
      for (int j = 0; j < FPW; ++j) {
        const int fr = wid + 4 * j;
        if (fr < NFR) {
          const int fi = fr / FK, fk = fr - fi * FK;
          const bf16x8 av = tr_read8<8>(&s_dy[prow * LDY], LDY, fi * 16, lane);
          const bf16x8 bv = tr_read8<8>(&s_x[prow * LDX], LDX, fk * 16, lane);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[j], 0, 0, 0);
        }
      }
    }
    buf ^= 1;
    __syncthreads();
  }
#undef LEAN_LOAD
  float* slab = a.slab + (((int64_t)z * a.splits + split) * a.Npad) * a.Kpad;
  if (BIG) {
#pragma unroll
    for (int i = 0; i < FA; ++i)
#pragma unroll
      for (int j = 0; j < FB; ++j) {
        const int col = k0 + wk + 32 * j + (lane & 31);
        const int row0 = n0 + wn + 32 * i + 4 * (lane >> 5);
        if (col < a.Kpad) {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int row = row0 + (r & 3) + 8 * (r >> 2);
            if (row < a.Npad) slab[(int64_t)row * a.Kpad + col] = bacc[i][j][r];
          }
        }
      }
    return;
  }
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int fr = wid + 4 * j;
    if (fr < NFR) {
      const int fi = fr / FK, fk = fr - fi * FK;
      const int row = n0 + fi * 16 + 4 * (lane >> 4);
      const int col = k0 + fk * 16 + (lane & 15);
      if (col < a.Kpad) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (row + r < a.Npad) slab[(int64_t)(row + r) * a.Kpad + col] = acc[j][r];
      }
    }
  }
}

template <int TN, int TK, int MCH, bool BIG>
__global__ __launch_bounds__(256) void conv_wgrad_lean_kernel(WgradArgs a) {
  wgrad_lean_block<TN, TK, MCH, BIG>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

template <int TN, int TK, int MCH, bool BIG>
__global__ __launch_bounds__(256) void conv_wgrad_lean_batched_kernel(const WgradJob* __restrict__ jobs, int nj,
                                                                       int64_t nvb) {
  for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {
    int lo = 0, hi = nj - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].block0 <= vb) lo = mid; else hi = mid - 1;
    }
    const WgradJob& J = jobs[lo];
    const int local = (int)(vb - J.block0);
    const int per_z = J.ntiles * J.a.splits;
    const int z = local / per_z, r = local - z * per_z;
    wgrad_lean_block<TN, TK, MCH, BIG>(J.a, r % J.ntiles, r / J.ntiles, z);
    __syncthreads();  // the next virtual block re-stages the LDS tables
  }
}

// the host-side checks every lean launch needs: 32-bit staging offsets, fdiv24's exact range
static bool lean_args_ok(const WgradArgs& a) {
  const int64_t M = (int64_t)a.B * a.Ho * a.Wo;
  const int64_t xin = (int64_t)a.B * a.Hi * a.Wi;
  const int64_t ld = std::max(a.src.ld[0], a.src.C1 > 0 ? a.src.ld[1] : 0);
  return M < (1 << 24) && xin * ld < ((int64_t)1 << 31) && M * a.ldd < ((int64_t)1 << 31) && a.Wi < 32768 &&
         a.Hi < 16384 && a.KH < 128 && a.KW < 128;
}

int wgrad_lean_ntiles(int cfg, const WgradArgs& a) {
  int TN, TK;
  if (wgrad_lean_shape(cfg, TN, TK)) return -1;
  if (!lean_args_ok(a)) return -2;
  return ((a.Npad + TN - 1) / TN) * ((a.Kpad + TK - 1) / TK);
}

int launch_wgrad_lean(const WgradArgs& a, int G, int cfg, hipStream_t st) {
  const int nt = wgrad_lean_ntiles(cfg, a);
  if (nt < 0) return nt;
#define LAUNCH_WGL(TN, TK, MCH, BIG)                                                                          \
  hipLaunchKernelGGL((conv_wgrad_lean_kernel<TN, TK, MCH, BIG>), dim3(nt, a.splits, G), dim3(256), 0, st, a); \
  break;
  switch (cfg) {
    WGRAD_LEAN_CASES(LAUNCH_WGL)
    default: return -1;
  }
#undef LAUNCH_WGL
  return (int)hipGetLastError();
}

int launch_wgrad_lean_batched(int cfg, const WgradJob* d_jobs, int nj, int64_t nblocks, dim3 grid, hipStream_t st) {
#define LAUNCH_WGLB(TN, TK, MCH, BIG)                                                                               \
  hipLaunchKernelGGL((conv_wgrad_lean_batched_kernel<TN, TK, MCH, BIG>), grid, dim3(256), 0, st, d_jobs, nj, nblocks); \
  break;
  switch (cfg) {
    WGRAD_LEAN_CASES(LAUNCH_WGLB)
    default: return -1;
  }
#undef LAUNCH_WGLB
  return (int)hipGetLastError();
}

}  // namespace mda
