// LDS-staged implicit-GEMM convolution on gfx950 MFMA (v_mfma_f32_16x16x32_bf16): forward and data
// gradient, NHWC bf16 operands, fp32 accumulation.  Replaces the same reference ops as conv.hip
// (every nn.Conv2d of model/modelA_MTL.py, model/modelB_singleTask.py and the Inception blocks of
// model/modelC_multiClassifier.py, and their autograd grad_input).
//
// Why a second conv kernel: conv.hip's conv_igemm loads every wave's MFMA fragments straight from
// global memory, 32 k at a time, two stages deep.  On Model C's deep layers (M = B*H*W of 192..8960
// pixels, K = 576..4032) a launch is a chain of ~10-40 dependent load round trips per wave and ran at
// 25..150 TF/s (profiles/r2_conv_layer_times_before.txt).  Here
//
//   * a block's whole K chunk (KC = 64 or 128) of BOTH operands is staged in LDS: 256 threads issue
//     16-byte loads cooperatively (8 pixels x 128 contiguous bytes per wave instruction: full lines),
//     the im2col gather / zero padding / normalise-on-load BN+ReLU happens once per element while
//     storing, and every wave reads its fragments with conflict-free ds_read_b128 -- the tile is read
//     from global memory once per block instead of once per wave;
//   * the next chunk's loads are in flight while the MFMAs of the current one run (double-buffered
//     LDS, one barrier per chunk);
//   * K is split ACROSS blocks (splits = 1..8): short dependency chains and enough blocks to fill the
//     256 CUs on small-M layers.  Partial fp32 tiles go to a workspace; the last block to arrive at a
//     tile (agent-scope release/acquire ticket) sums them in split order -- deterministic -- and runs
//     the epilogue;
//   * a stride-2 data gradient is decomposed into its sub-pixel phases (output parities): each phase
//     reduces over the taps that actually hit a dy element, instead of the gather form's masking of
//     3/4 of the MFMA work (conv.hip conv_load_stage).
//
// LDS image of an operand chunk: [k-group g (8 channels)][row][8 bf16] (16-byte units).  The MFMA
// fragment read of lane (r = lane & 15, q = lane >> 4) at k-step s is row r, group 4s + q: within a
// ds_read_b128 lane group the 16 rows are distinct, so each group touches 16 distinct 16-byte slots of
// a 256-byte bank row (conflict-free).  Staging writes go 8 consecutive lanes -> 8 consecutive rows
// (one 128-byte ds_write_b128 group, conflict-free); the matching global loads read 8 pixels x 8
// k-groups = 8 full 128-byte lines per wave instruction.
//
// Modes: MODE_FWD, MODE_FWD_NOL (normalise-on-load of the input), MODE_DGRAD, MODE_DGRAD_BNS (fused
// BN-backward statistics in the epilogue); the epilogues match conv.hip's (bias, bf16 store, fp64
// replica BN sums / bf16 gradient store, dz statistics).
#include "kernels.h"

namespace mda {

namespace {

template <int MODE>
constexpr bool lds_fwd() { return MODE == MODE_FWD || MODE == MODE_FWD_NOL; }

// (BM pixels, BN channels, waves along M, waves along N) of each tile config
constexpr int LDS_BM[8] = {64, 128, 64, 128, 32, 64, 32, 128};
constexpr int LDS_BN[8] = {64, 64, 128, 128, 64, 32, 32, 16};
constexpr int LDS_WAM[8] = {2, 2, 2, 2, 2, 2, 2, 4};

// Field of phase p (wave-uniform) without indexing the by-value kernel argument at run time (a dynamic
// index would copy the argument struct to scratch memory).
#define PSEL(f) (p == 0 ? pl.ph[0].f : p == 1 ? pl.ph[1].f : p == 2 ? pl.ph[2].f : pl.ph[3].f)

// Cross-block split-K reduction and epilogue of one output tile, shared by the register-staged kernel
// (conv_lds_kernel) and the LDS-DMA kernel (conv_glds_kernel).  Lane: pixel l16 of each fragment,
// channels 4*kgl .. +3 of each 16-channel fragment.
struct TileCtx {
  int tid, lane, wid, wn, wm, l16, kgl, S, split, nt, ntn, z, mbase, nbase, Mq, HWq, Wq, oy0, ox0, bN;
  int bx, gx;  // logical block x (block_coords) and the grid's x extent: split-K tile id, BN replica
};

// Epilogue stores of one output tile (lane: pixel l16 of each fragment, channels 4*kgl .. +3): bias + bf16
// store (forward) / extra gradient sources + bf16 store (data gradient), and this lane's share of the BN
// statistics accumulated into st[i][stat][r] (summed over the tiles of a persistent block before the flush).
template <bool FWD, bool BNS, int BN, int WM, int WN, int FN, int FM>
DEV void tile_store(const ConvArgs& a, const LdsPlan& pl, const TileCtx& t, f32x4 (&acc)[FN][FM], const float* s_k,
                    float (&st)[FN][3][4]) {
  int orow[FM];
  bool pv[FM];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    const int m = t.mbase + t.wm * WM + f * 16 + t.l16;
    pv[f] = m < t.Mq;
    const int mm = pv[f] ? m : 0;
    const int b = mm / t.HWq, r = mm - b * t.HWq;
    const int i = r / t.Wq, jj = r - i * t.Wq;
    orow[f] = (b * a.Ho + t.oy0 + i * pl.qy) * a.Wo + t.ox0 + jj * pl.qx;
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n0 = t.nbase + t.wn * WN + i * 16 + 4 * t.kgl;
    const int cl = t.wn * WN + i * 16 + 4 * t.kgl;
    const bool nok = n0 < a.N;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (FWD && a.bias && nok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[r] = a.bias[a.bgs * t.z + n0 + r];
    }
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      if (!(nok && pv[f])) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][f][r] + bias[r];
      if (FWD) {
        bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + a.ogs * t.z + (int64_t)orow[f] * a.ldo + n0;
        uint2 w;
        w.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
        w.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
        *reinterpret_cast<uint2*>(o) = w;
#pragma unroll
        for (int r = 0; r < 4; ++r) { st[i][0][r] += v[r]; st[i][1][r] += v[r] * v[r]; }
      } else {
        bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + a.ogs * t.z + (int64_t)orow[f] * a.ldo + n0;
        add_sources(a, t.z, (int64_t)orow[f], n0, v);
        store4(o, v);
        if (BNS && n0 < t.bN) {  // dz of the BN tail this gradient feeds, and its statistics
          const uint2 u = *reinterpret_cast<const uint2*>(a.by + a.bygs * t.z + (int64_t)orow[f] * a.ldby + n0);
          const float yv[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                               __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
          uint2 q = make_uint2(0, 0);
          if (a.bkind == ADD_RELU) q = *reinterpret_cast<const uint2*>(a.br + a.brgs * t.z + (int64_t)orow[f] * a.ldbr + n0);
          const float rv[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                               __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u)};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float tv = yv[r] * s_k[cl + r] + s_k[BN + cl + r];
            float dz = rbf(v[r]), xh2 = 0.f;  // the stored gradient: the apply pass recomputes dz from it
            if (a.bkind == ACT_RELU) {
              dz = tv > 0.f ? dz : 0.f;
            } else if (a.bkind == ACT_SIGMOID) {
              const float sg = sigmoidf_(tv);
              dz *= sg * (1.f - sg);
            } else if (a.bkind == ADD_RELU) {
              float rr = rv[r];
              if (a.br_bn) {
                xh2 = (rr - s_k[6 * BN + cl + r]) * s_k[7 * BN + cl + r];
                rr = rr * s_k[4 * BN + cl + r] + s_k[5 * BN + cl + r];
              }
              dz = (tv + rr) > 0.f ? dz : 0.f;
            }
            const float xh = (yv[r] - s_k[2 * BN + cl + r]) * s_k[3 * BN + cl + r];
            st[i][0][r] += dz;
            st[i][1][r] += dz * xh;
            st[i][2][r] += dz * xh2;
          }
        }
      }
    }
  }
}

// Block reduction of the accumulated statistics and one fp64 atomic per (channel, statistic) into replica
// blockIdx.x % nrep: forward (sum y, sum y^2) rows of [G][NREP][2][N], or the fused BN-backward rows 0/1 (2
// with a BN2 residual) of the tail's [G][NREP][3][bN].
template <bool FWD, bool BNS, int BN, int WAM, int WN, int FN>
DEV void tile_flush(const ConvArgs& a, const TileCtx& t, float (&st)[FN][3][4], float* s_st) {
  const bool want_red = (FWD && a.stats != nullptr) || BNS;
  if (!want_red) return;
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int cl = t.wn * WN + i * 16 + 4 * t.kgl;
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // the 16 pixels of a lane row -> lane 15 (DPP, common.h)
      st[i][0][r] = row16_sum(st[i][0][r]);
      st[i][1][r] = row16_sum(st[i][1][r]);
      if (BNS) st[i][2][r] = row16_sum(st[i][2][r]);
    }
    if (t.l16 == 15) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        s_st[(t.wm * BN + cl + r) * 3 + 0] = st[i][0][r];
        s_st[(t.wm * BN + cl + r) * 3 + 1] = st[i][1][r];
        s_st[(t.wm * BN + cl + r) * 3 + 2] = BNS ? st[i][2][r] : 0.f;
      }
    }
  }
  __syncthreads();
  const int rep = t.bx % (BNS ? a.bbn.pnrep : a.stats_nrep);
  double* dst = BNS ? a.bpart : a.stats;
  const int rows = BNS ? 3 : 2, nrow = BNS && a.br_bn ? 3 : 2, nlim = BNS ? t.bN : a.N;
  const int64_t gb = BNS ? (a.bpgs < 0 ? (int64_t)t.z * NREP * 3 * t.bN : (int64_t)t.z * a.bpgs)
                         : (int64_t)t.z * NREP * 2 * a.N;
  for (int q = t.tid; q < BN * 3; q += 256) {
    const int c = q / 3, which = q - c * 3;
    const int n = t.nbase + c;
    if (n < nlim && which < nrow) {
      float v = 0.f;
#pragma unroll
      for (int w2 = 0; w2 < WAM; ++w2) v += s_st[(w2 * BN + c) * 3 + which];
      atomicAdd(dst + gb + ((int64_t)rep * rows + which) * nlim + n, (double)v);
    }
  }
}

template <bool FWD, bool BNS, int BM, int BN, int WAM, int WM, int WN, int FN, int FM>
DEV void tile_epilogue(const ConvArgs& a, const LdsPlan& pl, const TileCtx& t, f32x4 (&acc)[FN][FM], float* s_st,
                       const float* s_k, int* s_flag) {
  // ---- cross-block split of K: deterministic last-arriver reduction.  The fp32 partial tiles are stored
  // WRITE-THROUGH (sc1 buffer stores: they leave the XCD's L2 at once, so no agent-scope release fence --
  // an L2 write-back of ~6.5 us with 16 KB dirtied per block), every wave drains them, one lane draws the
  // tile's arrival ticket (agent-scope atomic), and the last arriver reads all partials with sc1 loads
  // (L1 bypassed: no acquire fence either) in split order.
  if (t.S > 1) {
    const int64_t tile = ((int64_t)t.z * t.gx + t.bx) * t.ntn + t.nt;
    const uint64_t base = reinterpret_cast<uint64_t>(a.ws + tile * t.S * (BM * BN));
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)base);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(base >> 32));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, t.S * BM * BN * 4, 0x00020000);
    typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const u32x4 v = {__float_as_uint(acc[i][f][0]), __float_as_uint(acc[i][f][1]), __float_as_uint(acc[i][f][2]),
                         __float_as_uint(acc[i][f][3])};
        const int off = ((t.split * (BM * BN / 4) + ((t.wid * FN + i) * FM + f) * 64 + t.lane)) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0, 16);  // aux 16 = sc1
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its partial tile
    __syncthreads();
    if (t.tid == 0) {
      const unsigned tk = __hip_atomic_fetch_add(a.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      s_flag[0] = tk == (unsigned)(t.S - 1);
    }
    __syncthreads();
    if (!s_flag[0]) return;
    if (t.tid == 0) __hip_atomic_store(a.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // reusable
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
        for (int sp = 0; sp < t.S; ++sp) {
          const int off = ((sp * (BM * BN / 4) + ((t.wid * FN + i) * FM + f) * 64 + t.lane)) * 16;
          const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 16);
          v[0] += __uint_as_float(u[0]); v[1] += __uint_as_float(u[1]);
          v[2] += __uint_as_float(u[2]); v[3] += __uint_as_float(u[3]);
        }
        acc[i][f] = v;
      }
  }

  float st[FN][3][4] = {};
  tile_store<FWD, BNS, BN, WM, WN, FN, FM>(a, pl, t, acc, s_k, st);
  tile_flush<FWD, BNS, BN, WAM, WN, FN>(a, t, st, s_st);
}

template <int MODE, int BM, int BN, int WAM, int KC>
__global__ __launch_bounds__(256) void conv_lds_kernel(ConvArgs a, LdsPlan pl) {
  const Blk blk = block_coords(a.xcd);
  constexpr int WAN = 4 / WAM;
  constexpr int WM = BM / WAM, WN = BN / WAN, FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile");
  constexpr int NG = KC / 8, NKS = KC / 32;
  constexpr int UA = BN * NG, UB = BM * NG;  // 16-byte staging units of a chunk
  constexpr int NA = (UA + 255) / 256, NB = (UB + 255) / 256;
  constexpr int BUF = (BN + BM) * KC;       // bf16 elements of one stage buffer
  constexpr bool NOL = MODE == MODE_FWD_NOL;
  constexpr bool BNS = MODE == MODE_DGRAD_BNS;
  constexpr bool FWD = lds_fwd<MODE>();

  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16_t* s_buf = reinterpret_cast<bf16_t*>(smem);
  int* s_tx = reinterpret_cast<int*>(smem + 2 * BUF * 2);  // input coordinates / channel per k-group
  int* s_tw = s_tx + pl.ntab;                              // weight column per k-group
  float* s_st = reinterpret_cast<float*>(s_tw + pl.ntab);  // [WAM][BN][3] epilogue sums
  float* s_k = s_st + WAM * BN * 3;                         // NOL: [2][Cs] / BNS: [8][BN] constants
  int* s_flag = reinterpret_cast<int*>(s_k + (NOL ? 2 * a.Cs : (BNS ? 8 * BN : 0)));

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int l16 = lane & 15, kgl = lane >> 4;
  const int wn = wid % WAN, wm = wid / WAN;
  int p = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (q < pl.nph && blk.x >= pl.ph[q].m0) p = q;
  const int oy0 = PSEL(oy0), ox0 = PSEL(ox0), Hq = PSEL(Hq), Wq = PSEL(Wq);
  const int rh = PSEL(rh), nh = PSEL(nh), rw = PSEL(rw), nw = PSEL(nw), ay = PSEL(ay), ax = PSEL(ax);
  const int Kp = PSEL(Kp), m0t = PSEL(m0);
  const int S = pl.splits;
  const int ntn = (a.N + BN - 1) / BN;
  const int nt = blk.y / S, split = blk.y - nt * S;
  const int z = blk.z;
  const int HWq = Hq * Wq;
  const int Mq = a.B * HWq;
  const int mbase = (blk.x - m0t) * BM, nbase = nt * BN;
  const int nch = Kp / KC;
  const int cps = (nch + S - 1) / S;
  const int cb = min(nch, split * cps), ce = min(nch, cb + cps);

  // ---- per-block k-group tables for this split's chunks
  {
    const int cs8 = a.Cs >> 3, ntap = nh * nw;
    const int ng = (ce - cb) * NG;
    for (int i = tid; i < ng; i += 256) {
      const int gabs = cb * NG + i;
      const int t = gabs / cs8;
      const int c = (gabs - t * cs8) * 8;
      int ex = 0, ew = -1;
      if (t < ntap) {
        const int u = t / nw, v = t - u * nw;
        const int kh = rh + pl.th * u, kw = rw + pl.tw * v;
        const int dyo = ay + pl.by * u, dxo = ax + pl.bx * v;
        const int seg = (a.src.C1 > 0 && c >= a.src.C0) ? 1 : 0;
        ex = (c - seg * a.src.C0) | ((dyo + 64) << 14) | ((dxo + 64) << 21) | (seg << 28) | (1 << 29);
        ew = (kh * a.KW + kw) * a.Cs + c;
      }
      s_tx[i] = ex;
      s_tw[i] = ew;
    }
  }
  if (NOL) bn_prepare(a.nbn, z, s_k, s_k + a.Cs, nullptr, nullptr, blk.x == 0 && blk.y == 0);
  const int bN = a.bN > 0 ? a.bN : a.N;  // fused BN statistics: the tail's channels, its group
  const int zb = a.bpgs == 0 ? 0 : z;
  if (BNS) {
    for (int i = tid; i < BN; i += 256) {
      const int n = nbase + i;
      float k[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (n < bN) {
        bn_channel_bwd(a.bbn, zb, n, k[0], k[1], k[2], k[3]);
        if (a.br_bn) bn_channel_bwd(a.bbn2, zb, n, k[4], k[5], k[6], k[7]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s_k[q * BN + i] = k[q];
    }
  }

  // ---- staging units: unit u -> (row = 8 * (u / (8 NG)) + (u & 7), k-group g = (u >> 3) % NG)
  const bf16_t* wz = a.w + a.wgs * z;
  const bf16_t* base0 = a.src.p[0] + a.src.gs[0] * z;
  const bf16_t* base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : base0;
  const int ld0 = a.src.ld[0], ld1 = a.src.ld[1];
  int an[NA], aoff[NA];  // weight row (-1: none), LDS offset (16-byte units)
  int ag[NA];
#pragma unroll
  for (int j = 0; j < NA; ++j) {
    const int u = tid + 256 * j;
    const int rest = u >> 3, g = rest % NG, row = (rest / NG) * 8 + (u & 7);
    const int n = nbase + row;
    an[j] = (u < UA && n < a.Npad) ? n : -1;
    ag[j] = g;
    aoff[j] = g * BN + row;
  }
  int pb[NB], pih[NB], piw[NB], bg[NB], boff[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int u = tid + 256 * j;
    const int rest = u >> 3, g = rest % NG, row = (rest / NG) * 8 + (u & 7);
    const int m = mbase + row;
    const bool ok = u < UB && m < Mq;
    const int mm = ok ? m : 0;
    const int b = mm / HWq, r = mm - b * HWq;
    const int i = r / Wq, jj = r - i * Wq;
    pb[j] = ok ? b : -1;
    pih[j] = i * pl.mh;
    piw[j] = jj * pl.mw;
    bg[j] = g;
    boff[j] = g * BM + row;
  }

  uint4 ra[NA], rb[NB];
  uint32_t bok = 0;
  auto load_chunk = [&](int ch) {
    const int t0 = (ch - cb) * NG;
#pragma unroll
    for (int j = 0; j < NA; ++j) {
      const int e = s_tw[t0 + ag[j]];
      ra[j] = (an[j] >= 0 && e >= 0) ? *reinterpret_cast<const uint4*>(wz + (int64_t)an[j] * a.Kpad + e)
                                      : make_uint4(0, 0, 0, 0);
    }
    bok = 0;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int e = s_tx[t0 + bg[j]];
      const int ih = pih[j] + ((e >> 14) & 127) - 64, iw = piw[j] + ((e >> 21) & 127) - 64;
      const bool ok = ((e >> 29) & 1) && pb[j] >= 0 && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws;
      rb[j] = make_uint4(0, 0, 0, 0);
      if (ok) {
        const int seg = (e >> 28) & 1;
        const bf16_t* sb = seg ? base1 : base0;
        rb[j] = *reinterpret_cast<const uint4*>(sb + ((int64_t)(pb[j] * a.Hs + ih) * a.Ws + iw) * (seg ? ld1 : ld0) +
                                                (e & 16383));
      }
      bok |= (uint32_t)ok << j;
    }
  };
  const bool nol_relu = a.nol_kind == ACT_RELU;
  auto store_chunk = [&](int buf, int ch) {
    bf16_t* A = s_buf + buf * BUF;
    bf16_t* B = A + BN * KC;
#pragma unroll
    for (int j = 0; j < NA; ++j)
      if (tid + 256 * j < UA) *reinterpret_cast<uint4*>(A + aoff[j] * 8) = ra[j];
    const int t0 = (ch - cb) * NG;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      if (tid + 256 * j >= UB) continue;
      uint4 v = rb[j];
      if (NOL && ((bok >> j) & 1)) {  // act(BN(y)) of the producing conv, rounded as its tail would
        const int c = s_tx[t0 + bg[j]] & 16383;
        uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          float lo = __uint_as_float(w4[h] << 16) * s_k[c + 2 * h] + s_k[a.Cs + c + 2 * h];
          float hi = __uint_as_float(w4[h] & 0xffff0000u) * s_k[c + 2 * h + 1] + s_k[a.Cs + c + 2 * h + 1];
          if (nol_relu) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
          w4[h] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
        }
        v = make_uint4(w4[0], w4[1], w4[2], w4[3]);
      }
      *reinterpret_cast<uint4*>(B + boff[j] * 8) = v;
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // tables and constants
  if (cb < ce) {
    load_chunk(cb);
    store_chunk(0, cb);
  }
  __syncthreads();
  for (int ch = cb; ch < ce; ++ch) {
    const int cur = (ch - cb) & 1;
    if (ch + 1 < ce) load_chunk(ch + 1);  // in flight during this chunk's MFMAs
    const bf16_t* A = s_buf + cur * BUF;
    const bf16_t* B = A + BN * KC;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      bf16x8 afr[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        afr[i] = *reinterpret_cast<const bf16x8*>(A + ((s * 4 + kgl) * BN + wn * WN + i * 16 + l16) * 8);
#pragma unroll
      for (int f = 0; f < FM; ++f)
        bfr[f] = *reinterpret_cast<const bf16x8*>(B + ((s * 4 + kgl) * BM + wm * WM + f * 16 + l16) * 8);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < FM; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], bfr[f], acc[i][f], 0, 0, 0);
    }
    if (ch + 1 < ce) store_chunk(cur ^ 1, ch + 1);  // that buffer's last reader finished before the barrier
    __syncthreads();
  }

  const TileCtx tc{tid, lane, wid, wn, wm, l16, kgl, S, split, nt, ntn, z, mbase, nbase, Mq, HWq, Wq, oy0, ox0, bN, blk.x, (int)gridDim.x};
  tile_epilogue<FWD, BNS, BM, BN, WAM, WM, WN, FN, FM>(a, pl, tc, acc, s_st, s_k, s_flag);
}

// ================================================================================================
// LDS-DMA variant (cfg >= CONV_GLDS_CFG0): the operand tiles go global -> LDS with
// global_load_lds_dwordx4 (no register hop, no ds_write pass), through a 3-stage ring of LDS buffers with
// one raw s_barrier per K chunk and a counted vmcnt that keeps the next chunk's DMAs in flight ACROSS the
// barrier (a __syncthreads() would emit vmcnt(0) and drain them).
//
// LDS image of an operand chunk (KC = 64): [row][8 k-groups] with 128-byte rows; k-group g of row r sits
// in 16-byte slot g ^ ((r >> 1) & 7).  An LDS-DMA instruction writes 64 lanes x 16 B contiguously (8 rows),
// so the swizzle is applied on the per-lane SOURCE address (lane l of the instruction fetches k-group
// (l & 7) ^ ((row >> 1) & 7) of row 8i + (l >> 3)) and again on the fragment read; with it the four 16-lane
// groups of every ds_read_b128 of a 16x16x32 MFMA fragment (16 rows, one k-group each) hit 16 distinct
// 16-byte slots of the 256-byte bank row -- conflict-free.  Padding (zero rows / taps outside the image /
// k beyond K) is a DMA from a 16-byte zero page, so every lane always issues its instruction.
constexpr int GL_NT = 8;  // tile configs: BM pixels x BN channels, WAM waves along M
constexpr int GL_BM[GL_NT] = {64, 128, 64, 128, 256, 128, 256, 64};
constexpr int GL_BN[GL_NT] = {64, 64, 128, 128, 64, 32, 128, 32};
constexpr int GL_WAM[GL_NT] = {2, 2, 2, 2, 4, 4, 2, 4};
constexpr int GL_KC = 64, GL_STAGES = 3;
// ring stages of the deep configs: as many 128-byte-row stages as fit ~150 KB of LDS, at most 8, and at
// most 2 + 63 / NPER (the counted vmcnt of NST - 2 chunks in flight must fit the 6-bit counter); 3 = none
constexpr int GL_NST_DEEP[GL_NT] = {8, 6, 6, 4, 3, 7, 3, 8};

__device__ uint4 g_zero16[4];  // never written: the source of every padding lane

typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;

DEV int gl_swz(int r, int g) { return g ^ ((r >> 1) & 7); }

// wait until at most `ahead` chunks (NPER DMA instructions each) of this wave are still in flight
template <int NPER, int NST>
DEV void gl_wait_ahead(int ahead) {
  static_assert((NST - 2) * NPER <= 63, "vmcnt is a 6-bit counter");
  switch (ahead) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NPER) : "memory"); break;
    case 2: if constexpr (NST > 3) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * NPER) : "memory"); break; }
            [[fallthrough]];
    case 3: if constexpr (NST > 4) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * NPER) : "memory"); break; }
            [[fallthrough]];
    case 4: if constexpr (NST > 5) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * NPER) : "memory"); break; }
            [[fallthrough]];
    case 5: if constexpr (NST > 6) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * NPER) : "memory"); break; }
            [[fallthrough]];
    default: if constexpr (NST > 7) { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(6 * NPER) : "memory"); break; }
             asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// NST = stages of the LDS ring: 3 (GL_STAGES, the streaming configs) or up to 8 for the "deep" configs,
// whose blocks issue the DMAs of up to NST - 1 K chunks before waiting for the first -- a block of a
// small-M, long-K layer (Model C's 4x13 / 1x6 Inception convs) pays ONE load latency instead of a chain
// of them.
template <int MODE, int BM, int BN, int WAM, int NST>
__global__ __launch_bounds__(256) void conv_glds_kernel(ConvArgs a, LdsPlan pl) {
  const Blk blk = block_coords(a.xcd);
  constexpr int WAN = 4 / WAM;
  constexpr int WM = BM / WAM, WN = BN / WAN, FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile");
  constexpr int KC = GL_KC, NG = KC / 8, NKS = KC / 32, ROWB = KC * 2;  // 128-byte rows
  constexpr int IA = BN / 32, IB = BM / 32;  // DMA instructions per wave per chunk (8 rows each)
  static_assert(IA >= 1 && IB >= 1, "tile too small for 4 waves x 8 rows");
  constexpr int NPER = IA + IB;
  constexpr int BUF = (BN + BM) * ROWB;  // bytes of one stage
  constexpr bool BNS = MODE == MODE_DGRAD_BNS;
  constexpr bool FWD = MODE == MODE_FWD;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  int* s_tx = reinterpret_cast<int*>(smem + NST * BUF);        // input coordinates / channel per k-group
  int* s_tw = s_tx + pl.ntab;                                  // weight column per k-group
  float* s_st = reinterpret_cast<float*>(s_tw + pl.ntab);      // [WAM][BN][3] epilogue sums
  float* s_k = s_st + WAM * BN * 3;                             // BNS: [8][BN] constants
  int* s_flag = reinterpret_cast<int*>(s_k + (BNS ? 8 * BN : 0));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kgl = lane >> 4;
  const int wn = wid % WAN, wm = wid / WAN;
  int p = 0;
#pragma unroll
  for (int q = 1; q < 4; ++q)
    if (q < pl.nph && blk.x >= pl.ph[q].m0) p = q;
  const int oy0 = PSEL(oy0), ox0 = PSEL(ox0), Hq = PSEL(Hq), Wq = PSEL(Wq);
  const int rh = PSEL(rh), nh = PSEL(nh), rw = PSEL(rw), nw = PSEL(nw), ay = PSEL(ay), ax = PSEL(ax);
  const int Kp = PSEL(Kp), m0t = PSEL(m0);
  const int S = pl.splits;
  const int ntn = (a.N + BN - 1) / BN;
  const int nt = blk.y / S, split = blk.y - nt * S;
  const int z = blk.z;
  const int HWq = Hq * Wq;
  const int Mq = a.B * HWq;
  const int mbase = (blk.x - m0t) * BM, nbase = nt * BN;
  const int nch = Kp / KC;
  const int cps = (nch + S - 1) / S;
  const int cb = min(nch, split * cps), ce = min(nch, cb + cps);

  // ---- per-block k-group tables for this split's chunks (as conv_lds_kernel)
  {
    const int cs8 = a.Cs >> 3, ntap = nh * nw;
    const int ng = (ce - cb) * NG;
    for (int i = tid; i < ng; i += 256) {
      const int gabs = cb * NG + i;
      const int t = gabs / cs8;
      const int c = (gabs - t * cs8) * 8;
      int ex = 0, ew = -1;
      if (t < ntap) {
        const int u = t / nw, v = t - u * nw;
        const int kh = rh + pl.th * u, kw = rw + pl.tw * v;
        const int dyo = ay + pl.by * u, dxo = ax + pl.bx * v;
        const int seg = (a.src.C1 > 0 && c >= a.src.C0) ? 1 : 0;
        ex = (c - seg * a.src.C0) | ((dyo + 64) << 14) | ((dxo + 64) << 21) | (seg << 28) | (1 << 29);
        ew = (kh * a.KW + kw) * a.Cs + c;
      }
      s_tx[i] = ex;
      s_tw[i] = ew;
    }
  }
  const int bN = a.bN > 0 ? a.bN : a.N;
  const int zb = a.bpgs == 0 ? 0 : z;
  if (BNS) {
    for (int i = tid; i < BN; i += 256) {
      const int n = nbase + i;
      float k[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (n < bN) {
        bn_channel_bwd(a.bbn, zb, n, k[0], k[1], k[2], k[3]);
        if (a.br_bn) bn_channel_bwd(a.bbn2, zb, n, k[4], k[5], k[6], k[7]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s_k[q * BN + i] = k[q];
    }
  }

  // ---- per-lane DMA sources: instruction j of wave w covers rows 8 (4j + w) .. +7; this lane fetches
  // k-group ga / gb (swizzled) of row 8 (4j + w) + (lane >> 3)
  const bf16_t* wz = a.w + a.wgs * z;
  const bf16_t* base0 = a.src.p[0] + a.src.gs[0] * z;
  const bf16_t* base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : base0;
  const int ld0 = a.src.ld[0], ld1 = a.src.ld[1];
  const void* zero = &g_zero16[0];
  int an[IA], ga[IA];
#pragma unroll
  for (int j = 0; j < IA; ++j) {
    const int row = 8 * (4 * j + wid) + (lane >> 3);
    const int n = nbase + row;
    an[j] = n < a.Npad ? n : -1;
    ga[j] = gl_swz(row, lane & 7);
  }
  int pb[IB], pih[IB], piw[IB], gb[IB];
#pragma unroll
  for (int j = 0; j < IB; ++j) {
    const int row = 8 * (4 * j + wid) + (lane >> 3);
    const int m = mbase + row;
    const bool ok = m < Mq;
    const int mm = ok ? m : 0;
    const int b = mm / HWq, r = mm - b * HWq;
    const int i = r / Wq, jj = r - i * Wq;
    pb[j] = ok ? b : -1;
    pih[j] = i * pl.mh;
    piw[j] = jj * pl.mw;
    gb[j] = gl_swz(row, lane & 7);
  }
  auto issue = [&](int ch, int buf) {
    char* A = smem + buf * BUF;
    char* Bq = A + BN * ROWB;
    const int t0 = (ch - cb) * NG;
#pragma unroll
    for (int j = 0; j < IA; ++j) {
      const int e = s_tw[t0 + ga[j]];
      const void* src = (an[j] >= 0 && e >= 0) ? (const void*)(wz + (int64_t)an[j] * a.Kpad + e) : zero;
      __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(A + (4 * j + wid) * 8 * ROWB), 16, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < IB; ++j) {
      const int e = s_tx[t0 + gb[j]];
      const int ih = pih[j] + ((e >> 14) & 127) - 64, iw = piw[j] + ((e >> 21) & 127) - 64;
      const bool ok = ((e >> 29) & 1) && pb[j] >= 0 && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws;
      const void* src = zero;
      if (ok) {
        const int seg = (e >> 28) & 1;
        src = (seg ? base1 : base0) + ((int64_t)(pb[j] * a.Hs + ih) * a.Ws + iw) * (seg ? ld1 : ld0) + (e & 16383);
      }
      __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(Bq + (4 * j + wid) * 8 * ROWB), 16, 0, 0);
    }
  };

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // tables and constants (no DMA in flight yet)
#pragma unroll
  for (int j = 0; j < NST - 1; ++j)
    if (cb + j < ce) issue(cb + j, j);
  for (int ch = cb; ch < ce; ++ch) {
    const int k = ch - cb;
    // this wave's DMAs of chunk ch have landed (the up to NST - 2 later chunks may still fly), then every
    // wave's have, and every wave is done reading chunk ch - 1 (whose buffer chunk ch + NST - 1 overwrites)
    gl_wait_ahead<NPER, NST>(min(ce - 1, ch + NST - 2) - ch);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (ch + NST - 1 < ce) issue(ch + NST - 1, (k + NST - 1) % NST);
    const char* A = smem + (k % NST) * BUF;
    const char* Bq = A + BN * ROWB;
#pragma unroll
    for (int s = 0; s < NKS; ++s) {
      const int g = 4 * s + kgl;
      bf16x8 afr[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i) {
        const int row = wn * WN + i * 16 + l16;
        afr[i] = *reinterpret_cast<const bf16x8*>(A + row * ROWB + gl_swz(row, g) * 16);
      }
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int row = wm * WM + f * 16 + l16;
        bfr[f] = *reinterpret_cast<const bf16x8*>(Bq + row * ROWB + gl_swz(row, g) * 16);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < FM; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], bfr[f], acc[i][f], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the stage buffers are dead; s_st / s_flag live past them
  const TileCtx tc{tid, lane, wid, wn, wm, l16, kgl, S, split, nt, ntn, z, mbase, nbase, Mq, HWq, Wq, oy0, ox0, bN, blk.x, (int)gridDim.x};
  tile_epilogue<FWD, BNS, BM, BN, WAM, WM, WN, FN, FM>(a, pl, tc, acc, s_st, s_k, s_flag);
}

#undef PSEL

// ================================================================================================
// Patch convolution (cfg in [CONV_PATCH_CFG0, +CONV_PATCH_NCFG)): 3x3 / stride-1 forward and data gradient
// of the wide maps (Model C's 49x124 / 47x122 / 23x60 stem, Model A's 33x83 / 17x42 stages).  The im2col
// forms above fetch every input element once per tap (9x); here a block owns a STRIP of R whole output
// rows of one image (M tile = R * Wout pixels, row-major, so the shared tile_epilogue applies unchanged)
// and stages the strip's input rows with halo -- (R + 2) rows x (Wout + 2) columns x CB channels -- in LDS
// ONCE per channel slice, together with the slice's weights [BN][9 * CB].  Every tap's MFMA operand is
// then a shifted read of the same strip: lane (pixel p, k-group q) of tap (dh, dw) reads the 16 bytes at
// strip row r(p) + dh, column c(p) + dw, channels 8q'.. -- no im2col gather, no per-tap bounds checks
// (padding is zero in the strip), and a normalise-on-load input is transformed once per element instead of
// 9 times.  The data gradient is the same kernel over dy with the taps flipped (dh = 2 - kh) and the halo
// offsets of the transposed conv.
//
// LDS rows are padded to CBP = CB + 8 channels and the weight rows to WKP = 9 CB (rounded up to 32) + 8, so
// the row pitches are odd multiples of 16 bytes: the 16 lanes of each ds_read_b128 group hit 16 distinct
// 16-byte slots of a 256-byte bank row (conflict-free).
constexpr int PT_NT = 5;  // tile configs: BM pixels (strip capacity) x BN channels, WAM waves along M
constexpr int PT_BM[PT_NT] = {256, 256, 256, 128, 128};
constexpr int PT_BN[PT_NT] = {16, 32, 64, 32, 64};
constexpr int PT_WAM[PT_NT] = {4, 4, 4, 4, 2};
constexpr int PT_CB[3] = {16, 32, 64};

template <int CB>
constexpr int pt_ksteps() { return (9 * CB + 31) / 32; }
template <int CB>
constexpr int pt_wkp() { return pt_ksteps<CB>() * 32 + 8; }

template <int MODE, int BM, int BN, int WAM, int CB>
__global__ __launch_bounds__(256) void conv_patch_kernel(ConvArgs a, PatchPlan pp) {
  const Blk blk = block_coords(a.xcd);
  constexpr int WAN = 4 / WAM;
  constexpr int WM = BM / WAM, WN = BN / WAN, FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile");
  constexpr int CBP = CB + 8, KS = pt_ksteps<CB>(), WKP = pt_wkp<CB>();
  constexpr int CG = CB / 8;  // 16-byte channel groups of a strip pixel
  static_assert(256 % CG == 0, "a thread's strip units keep one channel group");
  constexpr int NU = 8;       // staging units per thread per round
  constexpr bool FWD = lds_fwd<MODE>();
  constexpr bool NOL = MODE == MODE_FWD_NOL;
  constexpr bool BNS = MODE == MODE_DGRAD_BNS;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int WP = pp.Wout + 2;  // strip columns
  const int SR = pp.R + 2;     // strip rows
  bf16_t* s_x = reinterpret_cast<bf16_t*>(smem);
  bf16_t* s_w = s_x + SR * WP * CBP;
  float* s_st = reinterpret_cast<float*>(s_w + BN * WKP);  // [WAM][BN][3] epilogue sums
  float* s_k = s_st + WAM * BN * 3;                         // NOL: [2][Cs] / BNS: [8][BN] constants
  int* s_flag = reinterpret_cast<int*>(s_k + (NOL ? 2 * a.Cs : (BNS ? 8 * BN : 0)));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kgl = lane >> 4;
  const int wn = wid % WAN, wm = wid / WAN;
  const int z = blk.z, nt = blk.y, ntn = gridDim.y;
  const int b = blk.x / pp.nstrip, oh0 = (blk.x - b * pp.nstrip) * pp.R;
  const int rows = min(pp.R, pp.Hout - oh0);
  const int HWo = pp.Hout * pp.Wout;
  const int mbase = b * HWo + oh0 * pp.Wout, nbase = nt * BN;
  const int Mtile = mbase + rows * pp.Wout;  // pixels of this strip end here (the next strip / image starts)

  if (NOL) bn_prepare(a.nbn, z, s_k, s_k + a.Cs, nullptr, nullptr, blk.x == 0 && blk.y == 0);
  const int bN = a.bN > 0 ? a.bN : a.N;
  const int zb = a.bpgs == 0 ? 0 : z;
  if (BNS) {
    for (int i = tid; i < BN; i += 256) {
      const int n = nbase + i;
      float k[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (n < bN) {
        bn_channel_bwd(a.bbn, zb, n, k[0], k[1], k[2], k[3]);
        if (a.br_bn) bn_channel_bwd(a.bbn2, zb, n, k[4], k[5], k[6], k[7]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s_k[q * BN + i] = k[q];
    }
  }

  const bf16_t* wz = a.w + a.wgs * z;
  const bf16_t* base0 = a.src.p[0] + a.src.gs[0] * z;
  const bf16_t* base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : base0;
  const int ld0 = a.src.ld[0], ld1 = a.src.ld[1];
  const int row0 = oh0 + pp.dy0, col0 = pp.dx0;  // source pixel of strip (0, 0)
  const int nux = SR * WP * CG, nuw = BN * (WKP - 8) / 8, nut = nux + nuw;

  // fragment bases: this lane's pixel of each M fragment -> strip element offset of tap (0, 0), channel 0
  int pbase[FM];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    int p = wm * WM + f * 16 + l16;
    p = mbase + p < Mtile ? p : 0;  // rows past the strip: any in-LDS address (the epilogue drops them)
    const int r = p / pp.Wout, c = p - r * pp.Wout;
    pbase[f] = (r * WP + c) * CBP;
  }

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // NOL / BNS constants
  for (int sl = 0; sl < pp.nslice; ++sl) {
    const int cs0 = sl * CB;
    // NOL: a thread's strip units all carry channel group tid % CG (CG divides 256), so its 8 scale and
    // 8 shift constants live in registers for the whole slice (an LDS read per element cost ~17 us on
    // the 47x122 stem conv)
    float nsc[8], nsh[8];
    if (NOL) {
      const int c = cs0 + (tid % CG) * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) { nsc[j] = s_k[c + j]; nsh[j] = s_k[a.Cs + c + j]; }
    }
    // ---- stage the strip slice and the weight slice: unit u < nux -> strip (row j, column q, group g),
    // else weight (row n, k-group g: tap g / CG, channel 8 (g % CG))
    for (int u0 = 0; u0 < nut; u0 += 256 * NU) {
      uint4 v[NU];
      uint32_t okm = 0;
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const int u = u0 + tid + 256 * i;
        v[i] = make_uint4(0, 0, 0, 0);
        if (u < nux) {
          const int g = u % CG, q = (u / CG) % WP, j = u / (CG * WP);
          const int ih = row0 + j, iw = col0 + q;
          if (ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws) {
            const int c = cs0 + g * 8;
            const int seg = (a.src.C1 > 0 && c >= a.src.C0) ? 1 : 0;
            v[i] = *reinterpret_cast<const uint4*>((seg ? base1 : base0) +
                                                   ((int64_t)(b * a.Hs + ih) * a.Ws + iw) * (seg ? ld1 : ld0) +
                                                   (c - seg * a.src.C0));
            okm |= 1u << i;
          }
        } else if (u < nut) {
          const int w = u - nux, g = w % (WKP / 8 - 1), n = nbase + w / (WKP / 8 - 1);
          const int tap = g / CG;
          if (tap < 9 && n < a.Npad)
            v[i] = *reinterpret_cast<const uint4*>(wz + (int64_t)n * a.Kpad + tap * a.Cs + cs0 + (g - tap * CG) * 8);
        }
      }
#pragma unroll
      for (int i = 0; i < NU; ++i) {
        const int u = u0 + tid + 256 * i;
        if (u < nux) {
          const int g = u % CG, pix = u / CG;
          uint4 x = v[i];
          if (NOL && ((okm >> i) & 1)) {  // act(BN(y)) of the producing conv, once per element
            uint32_t w4[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int h = 0; h < 4; ++h) {
              float lo = __uint_as_float(w4[h] << 16) * nsc[2 * h] + nsh[2 * h];
              float hi = __uint_as_float(w4[h] & 0xffff0000u) * nsc[2 * h + 1] + nsh[2 * h + 1];
              if (a.nol_kind == ACT_RELU) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
              w4[h] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
            }
            x = make_uint4(w4[0], w4[1], w4[2], w4[3]);
          }
          *reinterpret_cast<uint4*>(s_x + pix * CBP + g * 8) = x;
        } else if (u < nut) {
          const int w = u - nux, g = w % (WKP / 8 - 1), n = w / (WKP / 8 - 1);
          *reinterpret_cast<uint4*>(s_w + n * WKP + g * 8) = v[i];
        }
      }
    }
    __syncthreads();
    // ---- 9 taps x CB channels: k-group g = 4 ks + kgl is tap g / CG, channels 8 (g % CG)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int g = 4 * ks + kgl;
      const int tap = g / CG < 9 ? g / CG : 0;  // k past 9 CB: zero weights, any strip element
      const int kh = tap / 3, kw = tap - kh * 3;
      const int dh = FWD ? kh : 2 - kh, dw = FWD ? kw : 2 - kw;
      const int off = (dh * WP + dw) * CBP + (g - (g / CG) * CG) * 8;
      bf16x8 afr[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        afr[i] = *reinterpret_cast<const bf16x8*>(s_w + (wn * WN + i * 16 + l16) * WKP + g * 8);
#pragma unroll
      for (int f = 0; f < FM; ++f) bfr[f] = *reinterpret_cast<const bf16x8*>(s_x + pbase[f] + off);
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < FM; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], bfr[f], acc[i][f], 0, 0, 0);
    }
    __syncthreads();  // the next slice overwrites the strip and the weights
  }

  LdsPlan pl{};
  pl.qy = 1; pl.qx = 1;
  const TileCtx tc{tid, lane, wid, wn, wm, l16, kgl, 1, 0, nt, ntn, z, mbase, nbase, Mtile, HWo, pp.Wout, 0, 0, bN, blk.x, (int)gridDim.x};
  tile_epilogue<FWD, BNS, BM, BN, WAM, WM, WN, FN, FM>(a, pl, tc, acc, s_st, s_k, s_flag);
}

// Persistent, software-pipelined patch conv (cfg CONV_PATCHP_CFG0 + 3 * tile + cb; one channel slice,
// Cs == CB).  The one-strip-per-block form above stages, then computes: its blocks expose the load latency
// and only the 2-3 co-resident blocks hide it.  Here a block stages its BN x 9 CB weights once, then loops
// over strips u = blockIdx.x, + gridDim.x, ...: the next strip goes global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, no registers) into the other of two strip buffers while the MFMAs of the
// current one run; the BN statistics are summed in registers over all of the block's strips and flushed
// once.  Strip image: dense [pixel q][CG 16-byte groups], group g of pixel q in slot g ^ ((q / (16 / CG)) %
// CG): the 16 pixels of an MFMA fragment read (16 consecutive q, one g) hit 16 distinct slots of the
// 256-byte bank rows.  Padding / halo bytes are DMA'd from a zero page.
template <int MODE, int BM, int BN, int WAM, int CB>
__global__ __launch_bounds__(256) void conv_patchp_kernel(ConvArgs a, PatchPlan pp) {
  constexpr int WAN = 4 / WAM;
  constexpr int WM = BM / WAM, WN = BN / WAN, FM = WM / 16, FN = WN / 16;
  static_assert(FM >= 1 && FN >= 1 && WM % 16 == 0 && WN % 16 == 0, "wave tile");
  constexpr int KS = pt_ksteps<CB>(), WKP = pt_wkp<CB>();
  constexpr int CG = CB / 8, PPR = 16 / CG;  // 16-byte groups per pixel, pixels per 256-byte bank row
  constexpr bool FWD = MODE == MODE_FWD;
  constexpr bool BNS = MODE == MODE_DGRAD_BNS;
  static_assert(MODE != MODE_FWD_NOL, "the DMA bypasses registers: no on-load transform");

  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int WP = pp.Wout + 2, SR = pp.R + 2;
  const int nq = SR * WP;                       // strip pixels
  const int nins = (nq * CG + 63) / 64;         // 1-KB DMA instructions per strip
  const int SBP = nins * 1024;                  // bytes of one strip buffer
  bf16_t* s_w = reinterpret_cast<bf16_t*>(smem + 2 * SBP);
  float* s_st = reinterpret_cast<float*>(s_w + BN * WKP);  // [WAM][BN][3] epilogue sums
  float* s_k = s_st + WAM * BN * 3;                         // BNS: [8][BN] constants
  int* s_flag = reinterpret_cast<int*>(s_k + (BNS ? 8 * BN : 0));

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int l16 = lane & 15, kgl = lane >> 4;
  const int wn = wid % WAN, wm = wid / WAN;
  const int z = blockIdx.z, nt = blockIdx.y, ntn = gridDim.y;
  const int nbase = nt * BN;
  const int HWo = pp.Hout * pp.Wout;
  const int U = a.B * pp.nstrip;
  const int bN = a.bN > 0 ? a.bN : a.N;
  const int zb = a.bpgs == 0 ? 0 : z;
  if (BNS) {
    for (int i = tid; i < BN; i += 256) {
      const int n = nbase + i;
      float k[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (n < bN) {
        bn_channel_bwd(a.bbn, zb, n, k[0], k[1], k[2], k[3]);
        if (a.br_bn) bn_channel_bwd(a.bbn2, zb, n, k[4], k[5], k[6], k[7]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s_k[q * BN + i] = k[q];
    }
  }
  const bf16_t* wz = a.w + a.wgs * z;
  const bf16_t* base0 = a.src.p[0] + a.src.gs[0] * z;
  const bf16_t* base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : base0;
  const int ld0 = a.src.ld[0], ld1 = a.src.ld[1];
  const void* zero = &g_zero16[0];

  // ---- strip DMA: instruction j of wave w writes strip bytes [(4j + w) KB, +1 KB); lane l fetches 16-byte
  // unit v = 64 (4j + w) + l = (pixel q, slot): the pixel's channel group slot ^ swz(q)
  auto issue = [&](int u, char* buf) {
    const int b = u / pp.nstrip, oh0 = (u - b * pp.nstrip) * pp.R;
    const int row0 = oh0 + pp.dy0;
    for (int j = 0; 4 * j + wid < nins; ++j) {
      const int v = 64 * (4 * j + wid) + lane;
      const int q = v / CG, slot = v - q * CG;
      const void* src = zero;
      if (q < nq) {
        const int jr = q / WP, qc = q - jr * WP;
        const int ih = row0 + jr, iw = pp.dx0 + qc;
        if (ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws) {
          const int c = (slot ^ ((q / PPR) % CG)) * 8;
          const int seg = (a.src.C1 > 0 && c >= a.src.C0) ? 1 : 0;
          src = (seg ? base1 : base0) + ((int64_t)(b * a.Hs + ih) * a.Ws + iw) * (seg ? ld1 : ld0) + (c - seg * a.src.C0);
        }
      }
      __builtin_amdgcn_global_load_lds((glb_vptr)src, (lds_vptr)(buf + (4 * j + wid) * 1024), 16, 0, 0);
    }
  };

  // ---- weights once: [BN][WKP], k-group g = tap g / CG, channels 8 (g % CG) (zero past 9 CB / Npad)
  for (int w = tid; w < BN * (WKP / 8 - 1); w += 256) {
    const int g = w % (WKP / 8 - 1), n = nbase + w / (WKP / 8 - 1);
    const int tap = g / CG;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (tap < 9 && n < a.Npad) v = *reinterpret_cast<const uint4*>(wz + (int64_t)n * a.Kpad + tap * a.Cs + (g - tap * CG) * 8);
    *reinterpret_cast<uint4*>(s_w + (w / (WKP / 8 - 1)) * WKP + g * 8) = v;
  }

  // fragment bases: strip pixel of tap (0, 0) for this lane's pixel of each M fragment
  int q0[FM];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    int p = wm * WM + f * 16 + l16;
    p = p < pp.R * pp.Wout ? p : 0;  // past the strip: any in-LDS pixel (the epilogue drops them)
    const int r = p / pp.Wout, c = p - r * pp.Wout;
    q0[f] = r * WP + c;
  }

  float st[FN][3][4] = {};
  LdsPlan pl{};
  pl.qy = 1; pl.qx = 1;
  int cur = 0;
  if ((int)blockIdx.x < U) issue(blockIdx.x, smem);
  __syncthreads();  // weights and constants
  for (int u = blockIdx.x; u < U; u += gridDim.x) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMAs of strip u (and its last stores)
    __builtin_amdgcn_s_barrier();                      // ... and every wave's; strip u - grid fully read
    asm volatile("" ::: "memory");
    if (u + (int)gridDim.x < U) issue(u + gridDim.x, smem + (cur ^ 1) * SBP);
    const char* X = smem + cur * SBP;
    f32x4 acc[FN][FM];
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int f = 0; f < FM; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int g = 4 * ks + kgl;
      const int tap = g / CG < 9 ? g / CG : 0;  // k past 9 CB: zero weights, any strip element
      const int kh = tap / 3, kw = tap - kh * 3;
      const int dq = (FWD ? kh : 2 - kh) * WP + (FWD ? kw : 2 - kw);
      const int cg = g - (g / CG) * CG;
      bf16x8 afr[FN], bfr[FM];
#pragma unroll
      for (int i = 0; i < FN; ++i)
        afr[i] = *reinterpret_cast<const bf16x8*>(s_w + (wn * WN + i * 16 + l16) * WKP + g * 8);
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int q = q0[f] + dq;
        bfr[f] = *reinterpret_cast<const bf16x8*>(X + (q * CG + (cg ^ ((q / PPR) % CG))) * 16);
      }
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < FM; ++f) acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[i], bfr[f], acc[i][f], 0, 0, 0);
    }
    const int b = u / pp.nstrip, oh0 = (u - b * pp.nstrip) * pp.R;
    const int rows = min(pp.R, pp.Hout - oh0);
    const int mbase = b * HWo + oh0 * pp.Wout;
    const TileCtx tc{tid, lane, wid, wn, wm, l16, kgl, 1, 0, nt, ntn, z, mbase, nbase, mbase + rows * pp.Wout, HWo,
                     pp.Wout, 0, 0, bN, (int)blockIdx.x, (int)gridDim.x};
    tile_store<FWD, BNS, BN, WM, WN, FN, FM>(a, pl, tc, acc, s_k, st);
    cur ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // the strip buffers are dead; s_st lives past the weights
  const TileCtx tf{tid, lane, wid, wn, wm, l16, kgl, 1, 0, nt, ntn, z, 0, nbase, 0, HWo, pp.Wout, 0, 0, bN,
                   (int)blockIdx.x, (int)gridDim.x};
  tile_flush<FWD, BNS, BN, WAM, WN, FN>(a, tf, st, s_st);
}

// Strip plan of a patch launch (host); returns 0 or -2 when the conv is not a 3x3 / stride-1 conv this
// tile can take.  FWD: output Ho x Wo from the input (Hs, Ws); DGRAD: dx (Ho, Wo) from dy (Hs, Ws).
int patch_plan(int mode, const ConvArgs& a, int tile, int cbi, PatchPlan& pp, size_t& lds) {
  const bool fwd = mode == MODE_FWD || mode == MODE_FWD_NOL;
  const int CB = PT_CB[cbi], BM = PT_BM[tile], BN = PT_BN[tile], WAM = PT_WAM[tile];
  if (a.KH != 3 || a.KW != 3 || a.sh != 1 || a.sw != 1) return -2;
  if (a.Cs % CB || a.Cs > 16383) return -2;
  if (a.src.C1 > 0 && a.src.C0 % CB) return -2;  // a channel slice may not straddle the two segments
  pp.Wout = a.Wo;
  pp.Hout = a.Ho;
  if (pp.Wout > BM || pp.Wout < 1) return -2;
  pp.R = std::min(BM / pp.Wout, pp.Hout);
  pp.nstrip = (pp.Hout + pp.R - 1) / pp.R;
  pp.nslice = a.Cs / CB;
  if (fwd) { pp.dy0 = -a.ph; pp.dx0 = -a.pw; }
  else { pp.dy0 = a.ph - 2; pp.dx0 = a.pw - 2; }
  if (fwd ? (a.Hs + 2 * a.ph - 2 != a.Ho || a.Ws + 2 * a.pw - 2 != a.Wo)
          : (a.Ho + 2 * a.ph - 2 != a.Hs || a.Wo + 2 * a.pw - 2 != a.Ws)) return -2;
  const bool nol = mode == MODE_FWD_NOL, bns = mode == MODE_DGRAD_BNS;
  const int wkp = ((9 * CB + 31) / 32) * 32 + 8;
  lds = (size_t)(pp.R + 2) * (pp.Wout + 2) * (CB + 8) * 2 + (size_t)BN * wkp * 2 +
        ((size_t)WAM * BN * 3 + (nol ? 2 * a.Cs : (bns ? 8 * BN : 0))) * 4 + 16;
  if (lds > 160 * 1024) return -2;
  return 0;
}

// LDS bytes of the persistent form: two dense strip buffers (whole 1-KB DMA instructions) + the weights
size_t patchp_lds(const PatchPlan& pp, int tile, int cbi, bool bns) {
  const int CB = PT_CB[cbi], BN = PT_BN[tile], WAM = PT_WAM[tile], CG = CB / 8;
  const int wkp = ((9 * CB + 31) / 32) * 32 + 8;
  const size_t sbp = (size_t)((pp.R + 2) * (pp.Wout + 2) * CG + 63) / 64 * 1024;
  return 2 * sbp + (size_t)BN * wkp * 2 + ((size_t)WAM * BN * 3 + (bns ? 8 * BN : 0)) * 4 + 16;
}

int patchp_check(int mode, const ConvArgs& a, int tile, int cbi, PatchPlan& pp, size_t& lds) {
  size_t l1;
  int rc = patch_plan(mode, a, tile, cbi, pp, l1);
  if (rc) return rc;
  if (mode == MODE_FWD_NOL || pp.nslice != 1) return -2;
  lds = patchp_lds(pp, tile, cbi, mode == MODE_DGRAD_BNS);
  return lds > 160 * 1024 ? -2 : 0;
}

template <int MODE>
int launch_patchp(const ConvArgs& a, int G, int tile, int cbi, hipStream_t st) {
  if constexpr (MODE == MODE_FWD_NOL) {
    return -2;
  } else {
    PatchPlan pp;
    size_t lds;
    int rc = patchp_check(MODE, a, tile, cbi, pp, lds);
    if (rc) return rc;
    const int ntn = (a.N + PT_BN[tile] - 1) / PT_BN[tile];
    const int per_cu = std::max<int>(1, (int)(160 * 1024 / lds));
    const int U = a.B * pp.nstrip;
    const int nblk = std::max(1, std::min(U, (256 * per_cu + ntn * G - 1) / (ntn * G)));
    dim3 grid(nblk, ntn, G);
#define PP_LAUNCH(T, C)                                                                                     \
  if (tile == T && cbi == C) {                                                                              \
    hipLaunchKernelGGL((conv_patchp_kernel<MODE, PT_BM[T], PT_BN[T], PT_WAM[T], PT_CB[C]>), grid, dim3(256), lds, \
                       st, a, pp);                                                                          \
    return (int)hipGetLastError();                                                                          \
  }
#define PP_TILE(T) PP_LAUNCH(T, 0) PP_LAUNCH(T, 1) PP_LAUNCH(T, 2)
    PP_TILE(0) PP_TILE(1) PP_TILE(2) PP_TILE(3) PP_TILE(4)
#undef PP_TILE
#undef PP_LAUNCH
    return -1;
  }
}

template <int MODE>
int launch_patch(const ConvArgs& a, int G, int tile, int cbi, hipStream_t st) {
  PatchPlan pp;
  size_t lds;
  int rc = patch_plan(MODE, a, tile, cbi, pp, lds);
  if (rc) return rc;
  dim3 grid(a.B * pp.nstrip, (a.N + PT_BN[tile] - 1) / PT_BN[tile], G);
#define PT_LAUNCH(T, C)                                                                                     \
  if (tile == T && cbi == C) {                                                                              \
    hipLaunchKernelGGL((conv_patch_kernel<MODE, PT_BM[T], PT_BN[T], PT_WAM[T], PT_CB[C]>), grid, dim3(256), lds, \
                       st, a, pp);                                                                          \
    return (int)hipGetLastError();                                                                          \
  }
#define PT_TILE(T) PT_LAUNCH(T, 0) PT_LAUNCH(T, 1) PT_LAUNCH(T, 2)
  PT_TILE(0) PT_TILE(1) PT_TILE(2) PT_TILE(3) PT_TILE(4)
#undef PT_TILE
#undef PT_LAUNCH
  return -1;
}

// patch conv config -> (tile, channel slice, persistent form)
bool patch_cfg(int cfg, int& tile, int& cbi, bool& pers) {
  pers = cfg >= CONV_PATCHP_CFG0;
  const int k = cfg - (pers ? CONV_PATCHP_CFG0 : CONV_PATCH_CFG0);
  if (k < 0 || k >= PT_NT * 3) return false;
  tile = k / 3;
  cbi = k % 3;
  return true;
}

// ---- host-side plan
struct LdsCfg {
  int tile, BM, BN, WAM, KC, splits;
  bool glds;  // LDS-DMA kernel (conv_glds_kernel)
  int nst;    // its ring stages
};

int decode_cfg(int cfg, LdsCfg& c) {
  const bool deep = cfg >= CONV_GDEEP_CFG0 && cfg < CONV_GDEEP_CFG0 + CONV_GDEEP_NCFG;
  c.glds = deep || (cfg >= CONV_GLDS_CFG0 && cfg < CONV_GLDS_CFG0 + CONV_GLDS_NCFG);
  if (c.glds) {  // cfg = CONV_GLDS_CFG0 (or CONV_GDEEP_CFG0) + 4 * tile + log2(splits)
    const int k = cfg - (deep ? CONV_GDEEP_CFG0 : CONV_GLDS_CFG0);
    c.tile = k / 4;
    c.KC = GL_KC;
    c.splits = 1 << (k % 4);
    c.BM = GL_BM[c.tile]; c.BN = GL_BN[c.tile]; c.WAM = GL_WAM[c.tile];
    c.nst = deep ? GL_NST_DEEP[c.tile] : GL_STAGES;
    if (deep && c.nst <= GL_STAGES) return -2;  // no deeper ring fits this tile
    return 0;
  }
  const int k = cfg - CONV_LDS_CFG0;
  if (k < 0 || k >= CONV_LDS_NCFG) return -1;
  c.tile = k / 8;
  c.KC = (k / 4) % 2 ? 128 : 64;
  c.splits = 1 << (k % 4);
  c.BM = LDS_BM[c.tile]; c.BN = LDS_BN[c.tile]; c.WAM = LDS_WAM[c.tile];
  if (c.KC == 128 && c.BM + c.BN > 192) return -2;  // LDS: two 128-deep stages of a 256-row tile
  return 0;
}

// Phases, grid and table size of a launch.  dgrad: ConvArgs Hs/Ws = dy, Ho/Wo = dx (the conv's input).
int make_plan(int mode, const ConvArgs& a, const LdsCfg& c, LdsPlan& pl, int& gx) {
  pl = LdsPlan{};
  pl.splits = c.splits;
  int maxch = 0;
  if (mode == MODE_FWD || mode == MODE_FWD_NOL) {
    pl.nph = 1;
    pl.mh = a.sh; pl.mw = a.sw; pl.by = 1; pl.bx = 1; pl.th = 1; pl.tw = 1; pl.qy = 1; pl.qx = 1;
    LdsPhase& P = pl.ph[0];
    P.oy0 = 0; P.ox0 = 0; P.Hq = a.Ho; P.Wq = a.Wo;
    P.rh = 0; P.nh = a.KH; P.rw = 0; P.nw = a.KW;
    P.ay = -a.ph; P.ax = -a.pw;
  } else {
    pl.mh = 1; pl.mw = 1; pl.by = -1; pl.bx = -1; pl.th = a.sh; pl.tw = a.sw; pl.qy = a.sh; pl.qx = a.sw;
    int n = 0;
    for (int py = 0; py < std::min(a.sh, a.Ho); ++py)
      for (int px = 0; px < std::min(a.sw, a.Wo); ++px) {
        LdsPhase& P = pl.ph[n++];
        P.oy0 = py; P.ox0 = px;
        P.Hq = (a.Ho - py + a.sh - 1) / a.sh;
        P.Wq = (a.Wo - px + a.sw - 1) / a.sw;
        P.rh = (py + a.ph) % a.sh;
        P.rw = (px + a.pw) % a.sw;
        P.nh = P.rh < a.KH ? (a.KH - P.rh + a.sh - 1) / a.sh : 0;
        P.nw = P.rw < a.KW ? (a.KW - P.rw + a.sw - 1) / a.sw : 0;
        P.ay = (py + a.ph - P.rh) / a.sh;
        P.ax = (px + a.pw - P.rw) / a.sw;
      }
    pl.nph = n;
    if (n < 1 || n > 4) return -2;
  }
  gx = 0;
  for (int p = 0; p < pl.nph; ++p) {
    LdsPhase& P = pl.ph[p];
    const int k = P.nh * P.nw * a.Cs;
    P.Kp = (k + c.KC - 1) / c.KC * c.KC;
    P.m0 = gx;
    gx += (a.B * P.Hq * P.Wq + c.BM - 1) / c.BM;
    maxch = std::max(maxch, (P.Kp / c.KC + c.splits - 1) / c.splits);
    if (std::abs(P.ay) > 56 || std::abs(P.ax) > 56 || a.KH > 56 || a.KW > 56) return -2;
  }
  pl.ntab = std::max(4, maxch * (c.KC / 8));
  return 0;
}

size_t glds_lds_bytes(const LdsCfg& c, const LdsPlan& pl, bool bns) {
  return (size_t)c.nst * (c.BM + c.BN) * GL_KC * 2 + (size_t)2 * pl.ntab * 4 +
         ((size_t)c.WAM * c.BN * 3 + (bns ? 8 * c.BN : 0)) * 4 + 16;
}

template <int MODE>
int launch_glds(const ConvArgs& a, int G, const LdsCfg& c, const LdsPlan& pl, int gx, hipStream_t st) {
  if constexpr (MODE == MODE_FWD_NOL) {
    return -2;  // the DMA bypasses registers: no on-load transform (conv_lds_kernel / conv_igemm do it)
  } else {
    const int ntn = (a.N + c.BN - 1) / c.BN;
    const size_t lds = glds_lds_bytes(c, pl, MODE == MODE_DGRAD_BNS);
    if (lds > 160 * 1024) return -2;
    dim3 grid(gx, ntn * c.splits, G);
#define GL_LAUNCH_N(T, NS)                                                                                \
  if (c.tile == T && c.nst == NS) {                                                                       \
    hipLaunchKernelGGL((conv_glds_kernel<MODE, GL_BM[T], GL_BN[T], GL_WAM[T], NS>), grid, dim3(256), lds, st, a, pl); \
    return (int)hipGetLastError();                                                                        \
  }
#define GL_LAUNCH(T) GL_LAUNCH_N(T, GL_STAGES) if constexpr (GL_NST_DEEP[T] > GL_STAGES) { GL_LAUNCH_N(T, GL_NST_DEEP[T]) }
    GL_LAUNCH(0) GL_LAUNCH(1) GL_LAUNCH(2) GL_LAUNCH(3) GL_LAUNCH(4) GL_LAUNCH(5) GL_LAUNCH(6) GL_LAUNCH(7)
#undef GL_LAUNCH
#undef GL_LAUNCH_N
    return -1;
  }
}

template <int MODE>
int launch_mode(const ConvArgs& a, int G, const LdsCfg& c, hipStream_t st) {
  LdsPlan pl;
  int gx;
  int rc = make_plan(MODE, a, c, pl, gx);
  if (rc) return rc;
  const int ntn = (a.N + c.BN - 1) / c.BN;
  if (c.splits > 1 && (!a.ws || !a.cnt)) return -3;
  if (c.glds) return launch_glds<MODE>(a, G, c, pl, gx, st);
  const bool nol = MODE == MODE_FWD_NOL, bns = MODE == MODE_DGRAD_BNS;
  const size_t lds = (size_t)2 * (c.BM + c.BN) * c.KC * 2 + (size_t)2 * pl.ntab * 4 +
                     ((size_t)c.WAM * c.BN * 3 + (nol ? 2 * a.Cs : (bns ? 8 * c.BN : 0))) * 4 + 16;
  if (lds > 160 * 1024) return -2;
  dim3 grid(gx, ntn * c.splits, G);
#define LDS_LAUNCH(T, KC_)                                                                               \
  if (c.tile == T && c.KC == KC_) {                                                                      \
    hipLaunchKernelGGL((conv_lds_kernel<MODE, LDS_BM[T], LDS_BN[T], LDS_WAM[T], KC_>), grid, dim3(256), lds, st, a, pl); \
    return (int)hipGetLastError();                                                                       \
  }
  LDS_LAUNCH(0, 64) LDS_LAUNCH(0, 128) LDS_LAUNCH(1, 64) LDS_LAUNCH(1, 128) LDS_LAUNCH(2, 64) LDS_LAUNCH(2, 128)
  LDS_LAUNCH(3, 64) LDS_LAUNCH(4, 64) LDS_LAUNCH(4, 128) LDS_LAUNCH(5, 64) LDS_LAUNCH(5, 128) LDS_LAUNCH(6, 64)
  LDS_LAUNCH(6, 128) LDS_LAUNCH(7, 64) LDS_LAUNCH(7, 128)
#undef LDS_LAUNCH
  return -1;
}

}  // namespace

int conv_lds_workspace(int mode, const ConvArgs& a, int G, int cfg, int64_t& ws_floats, int64_t& ntickets) {
  cfg &= ~CONV_XCD;
  if (mode == MODE_FWD && a.nol) mode = MODE_FWD_NOL;  // the launch mode launch_conv will pick
  if (mode == MODE_DGRAD && a.bpart) mode = MODE_DGRAD_BNS;
  int tile, cbi;
  bool pers;
  if (patch_cfg(cfg, tile, cbi, pers)) {
    PatchPlan pp;
    size_t lds;
    ws_floats = 0;
    ntickets = 0;
    return pers ? patchp_check(mode, a, tile, cbi, pp, lds) : patch_plan(mode, a, tile, cbi, pp, lds);
  }
  LdsCfg c;
  int rc = decode_cfg(cfg, c);
  if (rc) return rc;
  LdsPlan pl;
  int gx;
  rc = make_plan(mode, a, c, pl, gx);
  if (rc) return rc;
  if (c.glds && (mode == MODE_FWD_NOL || glds_lds_bytes(c, pl, mode == MODE_DGRAD_BNS) > 160 * 1024)) return -2;
  const int64_t tiles = (int64_t)G * gx * ((a.N + c.BN - 1) / c.BN);
  ws_floats = c.splits > 1 ? tiles * c.splits * c.BM * c.BN : 0;
  ntickets = c.splits > 1 ? tiles : 0;
  return 0;
}

int launch_conv_lds(int mode, const ConvArgs& a, int G, int cfg, hipStream_t st) {
  int tile, cbi;
  bool pers;
  if (patch_cfg(cfg, tile, cbi, pers)) {
    switch (mode) {
      case MODE_FWD: return pers ? launch_patchp<MODE_FWD>(a, G, tile, cbi, st) : launch_patch<MODE_FWD>(a, G, tile, cbi, st);
      case MODE_FWD_NOL: return pers ? -2 : launch_patch<MODE_FWD_NOL>(a, G, tile, cbi, st);
      case MODE_DGRAD: return pers ? launch_patchp<MODE_DGRAD>(a, G, tile, cbi, st) : launch_patch<MODE_DGRAD>(a, G, tile, cbi, st);
      case MODE_DGRAD_BNS:
        return pers ? launch_patchp<MODE_DGRAD_BNS>(a, G, tile, cbi, st) : launch_patch<MODE_DGRAD_BNS>(a, G, tile, cbi, st);
      default: return -1;
    }
  }
  LdsCfg c;
  int rc = decode_cfg(cfg, c);
  if (rc) return rc;
  switch (mode) {
    case MODE_FWD: return launch_mode<MODE_FWD>(a, G, c, st);
    case MODE_FWD_NOL: return launch_mode<MODE_FWD_NOL>(a, G, c, st);
    case MODE_DGRAD: return launch_mode<MODE_DGRAD>(a, G, c, st);
    case MODE_DGRAD_BNS: return launch_mode<MODE_DGRAD_BNS>(a, G, c, st);
    default: return -1;
  }
}

}  // namespace mda
