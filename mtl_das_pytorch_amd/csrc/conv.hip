// Implicit-GEMM convolutions on gfx950 MFMA (v_mfma_f32_16x16x32_bf16), NHWC bf16, fp32 accumulate.
//
// Replaces the reference's implicit cuDNN convolutions (every nn.Conv2d of model/modelA_MTL.py,
// model/modelB_singleTask.py and the Inception blocks of model/modelC_multiClassifier.py) and their
// autograd backward (convolution_backward: grad_input + grad_weight).
//
//  conv_igemm<FWD>   out[m, n] = sum_k W[n, k] * im2col(x)[k, m]      m = (b, oh, ow), n = cout,
//                    k = (kh, kw, cin).  Epilogue: + bias, bf16 store, per-channel BN partial sums
//                    (sum y, sum y^2) into NREP replicas -- the training-mode BN reduction is fused
//                    into the producing conv.
//  conv_igemm<DGRAD> dx[m, n] = sum_k Wt[n, k] * gather(dy)[k, m]      m = (b, ih, iw), n = cin,
//                    k = (kh, kw, cout); strided convs gather only the taps with (ih+p-kh) % s == 0.
//                    bf16 output, rounded once from the fp32 accumulator (plus any extra gradient sources).
//  conv_wgrad        dW[n, k] = sum_m dy[m, n] * im2col(x)[m, k]; both operands are staged in LDS
//                    pixel-major (natural NHWC rows, 16-B writes) and read as MFMA operands with the
//                    gfx950 transpose read ds_read_b64_tr_b16.  Split over m; fp32 partial slabs are
//                    summed (deterministically) by wgrad_finalize into the flat fp32 gradient buffer in
//                    the reference's NCHW weight layout.
//
// MFMA orientation: the weight tile is the A operand (rows = output channels) and the im2col tile
// the B operand (cols = pixels), so each lane's accumulator holds 4 consecutive channels of one
// pixel -> 8-byte (bf16) / 16-byte (fp32) NHWC stores, 16 lanes covering 16 consecutive pixels.
//
// The K dimension is walked in steps of 32 = four 8-channel groups; a per-block LDS table maps each
// k-group to (segment, kh, kw, channel) so two-segment inputs (cat[F_shared, B_task]) need no concat.
#include "kernels.h"

namespace mda {



DEV int encode_kg(int i, int Ktot, int Cs8, int KW, int C0) {
  if (i * 8 >= Ktot) return 0;
  int tap = i / Cs8, c = (i - tap * Cs8) * 8;
  int kh = tap / KW, kw = tap - kh * KW;
  int seg = c >= C0;
  if (seg) c -= C0;
  return c | (kw << 14) | (kh << 21) | (seg << 28) | (1 << 29);
}

template <int MODE>
constexpr bool is_fwd() { return MODE == MODE_FWD || MODE == MODE_FWD_NOL; }
template <int MODE>
constexpr bool has_bns() { return MODE == MODE_DGRAD_BNS; }

// Normalise-on-load: the 8 channels [c, c+8) of an im2col fragment are pre-BN conv outputs y; the operand
// is act(y * scale + shift) (act = ReLU or identity), rounded to bf16 exactly as the BN tail that used to
// materialise it.  Fragments of zero padding (bit f of okm clear) stay zero.
// The stage's 8 scale and 8 shift constants (k[0..7], k[8..15]) are read from LDS when the stage's loads are
// issued (nol_fetch), not here: a read at consumption time put an LDS round trip into every K step's chain.
DEV void nol_fetch(float* k, int c, const float* s_nol, int Cs) {
  const float4* p0 = reinterpret_cast<const float4*>(s_nol + c);
  const float4* p1 = reinterpret_cast<const float4*>(s_nol + Cs + c);
  const float4 a0 = p0[0], a1 = p0[1], b0 = p1[0], b1 = p1[1];
  k[0] = a0.x; k[1] = a0.y; k[2] = a0.z; k[3] = a0.w; k[4] = a1.x; k[5] = a1.y; k[6] = a1.z; k[7] = a1.w;
  k[8] = b0.x; k[9] = b0.y; k[10] = b0.z; k[11] = b0.w; k[12] = b1.x; k[13] = b1.y; k[14] = b1.z; k[15] = b1.w;
}

template <int FM>
DEV void nol_apply(bf16x8* bfr, uint32_t okm, const float* k, bool relu) {
  float sc[8], sh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) { sc[j] = k[j]; sh[j] = k[8 + j]; }
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    if (!((okm >> f) & 1)) continue;
    bf16x8 v = bfr[f];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float x = __uint_as_float(((uint32_t)(uint16_t)v[j]) << 16) * sc[j] + sh[j];
      if (relu) x = fmaxf(x, 0.f);
      v[j] = (short)f2bf(x);
    }
    bfr[f] = v;
  }
}

// One wave's fragment loads for k-step `ks`: FM im2col fragments (B operand) + FN weight fragments (A).
// okm / cch: which im2col fragments hold real (not padding) data and their first channel (for NOL).
template <int MODE, int FN, int FM>
DEV void conv_load_stage(const ConvArgs& a, const int* s_tab, int ks, int kgl, int l16, int n_base,
                         const int* pb, const int* py, const int* px, const bool* pv, const bf16_t* base0,
                         const bf16_t* base1, int ld0, int ld1, const bf16_t* wz, bf16x8* afr, bf16x8* bfr,
                         uint32_t& okm, int& cch) {
  const bf16x8 zero8 = {0, 0, 0, 0, 0, 0, 0, 0};
  const int e = s_tab[ks * 4 + kgl];
  const bool valid = (e >> 29) & 1;
  const int seg = (e >> 28) & 1;
  const int kh = (e >> 21) & 127, kw = (e >> 14) & 127, c = e & 16383;
  const bf16_t* sb = seg ? base1 : base0;
  const int sld = seg ? ld1 : ld0;
  okm = 0;
  cch = c;
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    int ih, iw;
    bool ok;
    if (is_fwd<MODE>()) {
      ih = py[f] + kh; iw = px[f] + kw;
      ok = valid && pv[f] && ih >= 0 && ih < a.Hs && iw >= 0 && iw < a.Ws;
    } else {
      int nh = py[f] - kh, nw = px[f] - kw;
      ok = valid && pv[f] && nh >= 0 && nw >= 0;
      if (a.sh == 2) { ok = ok && !(nh & 1); ih = nh >> 1; } else if (a.sh == 1) { ih = nh; } else { ok = ok && (nh % a.sh == 0); ih = nh / a.sh; }
      if (a.sw == 2) { ok = ok && !(nw & 1); iw = nw >> 1; } else if (a.sw == 1) { iw = nw; } else { ok = ok && (nw % a.sw == 0); iw = nw / a.sw; }
      ok = ok && ih < a.Hs && iw < a.Ws;
    }
    // unconditional load from a valid address, zeroed after: no exec-masked branch around the load, so the
    // waitcnt pass can count the loads of every pipeline stage exactly instead of draining with vmcnt(0)
    const bf16_t* q = ok ? sb + ((int64_t)(pb[f] * a.Hs + ih) * a.Ws + iw) * sld + c : sb;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(q);
    bfr[f] = ok ? v : zero8;
    okm |= (uint32_t)ok << f;
  }
#pragma unroll
  for (int i = 0; i < FN; ++i) {
    const int n = n_base + i * 16 + l16;
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(wz + (int64_t)(n < a.Npad ? n : 0) * a.Kpad + ks * 32 + kgl * 8);
    afr[i] = n < a.Npad ? v : zero8;
  }
}

// Block = 4 waves laid out WAVES_N (channels) x WAVES_M (pixels) x KSPLIT (reduction).  Each wave walks
// its share of K with a two-stage register pipeline (loads of step k+1 in flight during the MFMAs of
// step k); KSPLIT > 1 partial accumulators are summed through LDS, so small-M / long-K layers (the 5x11
// and 9x21 stages, K up to 1152) get up to 4x shorter dependency chains.
// PD = register pipeline depth: fragment loads of PD - 1 K-steps are in flight while one step's MFMAs run.
// The small-M layers (grids below one wave per SIMD) are bound by this load latency, not by occupancy.
template <int MODE, int WN, int WM, int WAVES_N, int WAVES_M, int KSPLIT, int PD>
__global__ __launch_bounds__(256) void conv_igemm_kernel(ConvArgs a) {
  static_assert(WAVES_N * WAVES_M * KSPLIT == 4, "4 waves per block");
  constexpr int FN = WN / 16, FM = WM / 16;
  constexpr int BN_T = WN * WAVES_N, BM_T = WM * WAVES_M;
  constexpr int TILE = FN * FM * 4 * 64;  // floats per wave accumulator tile
  constexpr int RED = (KSPLIT - 1) * WAVES_N * WAVES_M * TILE, ST2 = WAVES_M * BN_T * 3;
  extern __shared__ __attribute__((aligned(16))) int s_dyn[];
  int* s_tab = s_dyn;  // [Kpad/8]
  const int nkg = a.Kpad >> 3;
  float* s_red = reinterpret_cast<float*>(s_dyn + ((nkg + 3) & ~3));  // KSPLIT partials, then stats
  float* s_bn = s_red + (RED > ST2 ? RED : ST2);  // [8][BN_T] fused BN-backward: scale, shift, mean, invstd
                                                  // of the tail's BN, then of its residual's BN2
  float* s_nol = s_bn;                             // [2][Cs] normalise-on-load scale, shift (forward only)
  ptick(a.ptm, 0);
  const Blk blk = block_coords(a.xcd);
  const int z = blk.z;
  const int Ktot = a.KH * a.KW * a.Cs;
  for (int i = threadIdx.x; i < nkg; i += 256) s_tab[i] = encode_kg(i, Ktot, a.Cs >> 3, a.KW, a.src.C0);
  // MODE_DGRAD_BNS: dgrad + fused BN-backward statistics -- its own instantiation, so the extra registers
  // never lower the occupancy of the plain dgrads (104 -> 142 VGPRs measured when they shared one)
  constexpr bool want_bnb = has_bns<MODE>();
  const int bN = a.bN > 0 ? a.bN : a.N;  // the tail's channels (a concat gradient has more)
  const int zb = a.bpgs == 0 ? 0 : z;    // one tail shared by every group: its constants are group 0's
  if (want_bnb) {
    for (int i = threadIdx.x; i < BN_T; i += 256) {
      const int n = blk.y * BN_T + i;
      float k[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (n < bN) {
        bn_channel_bwd(a.bbn, zb, n, k[0], k[1], k[2], k[3]);
        if (a.br_bn) bn_channel_bwd(a.bbn2, zb, n, k[4], k[5], k[6], k[7]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s_bn[q * BN_T + i] = k[q];
    }
  }
  // MODE_FWD_NOL: the input is the previous conv's pre-BN y; its BN constants for all Cs channels go to
  // LDS, and block (0, 0) of each group performs that BN's running-statistics update and publishes its
  // batch constants for the backward (the work of the forward tail this mode replaces)
  constexpr bool NOL = MODE == MODE_FWD_NOL;
  if (NOL) bn_prepare(a.nbn, z, s_nol, s_nol + a.Cs, nullptr, nullptr, blk.x == 0 && blk.y == 0);
  const bool nol_relu = a.nol_kind == ACT_RELU;
  __syncthreads();
  ptick(a.ptm, 1);

  // wave index through readfirstlane: the compiler then knows every K-loop bound and guard below is
  // wave-uniform and branches on it.  An MFMA ignores EXEC, so a guard lowered to an exec mask would still
  // accumulate the stale fragments of a step past kend (seen with the depth-4 pipeline's remainder steps).
  const int lane = threadIdx.x & 63, wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wn = wid % WAVES_N, wm = (wid / WAVES_N) % WAVES_M, wk = wid / (WAVES_N * WAVES_M);
  const int n_base = blk.y * BN_T + wn * WN;
  const int m_base = blk.x * BM_T + wm * WM;
  const int HWo = a.Ho * a.Wo;
  const int M = a.B * HWo;
  const int l16 = lane & 15, kgl = lane >> 4;

  int pb[FM], py[FM], px[FM];
  bool pv[FM];
#pragma unroll
  for (int f = 0; f < FM; ++f) {
    int m = m_base + f * 16 + l16;
    pv[f] = m < M;
    int mm = pv[f] ? m : 0;
    int b = mm / HWo, r = mm - b * HWo;
    int oh = r / a.Wo, ow = r - oh * a.Wo;
    pb[f] = b;
    if (is_fwd<MODE>()) { py[f] = oh * a.sh - a.ph; px[f] = ow * a.sw - a.pw; }
    else { py[f] = oh + a.ph; px[f] = ow + a.pw; }
  }
  const bf16_t* base0 = a.src.p[0] + a.src.gs[0] * z;
  const bf16_t* base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : base0;
  const int ld0 = a.src.ld[0], ld1 = a.src.ld[1];
  const bf16_t* wz = a.w + a.wgs * z;

  f32x4 acc[FN][FM];
#pragma unroll
  for (int i = 0; i < FN; ++i)
#pragma unroll
    for (int f = 0; f < FM; ++f) acc[i][f] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nks = a.Kpad >> 5;
  const int kchunk = (nks + KSPLIT - 1) / KSPLIT;
  const int kbeg = wk * kchunk, kend = min(nks, kbeg + kchunk);
  // fused BN backward: the tail's pre-BN y at this lane's output elements -- in flight during the K loop
  // for small tiles; for large ones loaded at the epilogue (when the K-loop buffers are dead), so the
  // prefetch does not cost occupancy
  constexpr bool PREFETCH_Y = want_bnb && FN * FM <= 4;
  const bool bres = want_bnb && a.bkind == ADD_RELU;  // residual tail: its r' enters the dz mask
  uint2 ypre[FN][FM], rpre[FN][FM];
  auto load_y = [&]() {
#pragma unroll
    for (int i = 0; i < FN; ++i)
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        ypre[i][f] = make_uint2(0, 0);
        rpre[i][f] = make_uint2(0, 0);
        const int n0 = n_base + i * 16 + 4 * kgl;
        const int64_t m = m_base + f * 16 + l16;
        if (wk == 0 && n0 < bN && pv[f]) {
          ypre[i][f] = *reinterpret_cast<const uint2*>(a.by + a.bygs * z + m * a.ldby + n0);
          if (bres) rpre[i][f] = *reinterpret_cast<const uint2*>(a.br + a.brgs * z + m * a.ldbr + n0);
        }
      }
  };
  if (PREFETCH_Y) load_y();
  bf16x8 af[PD][FN], bq[PD][FM];
  uint32_t okq[PD];
  int ccq[PD];
  float nk[NOL ? PD : 1][16];       // NOL: the stage's BN scale / shift
#define LOAD_STAGE(KS, J) do { \
  conv_load_stage<MODE, FN, FM>(a, s_tab, KS, kgl, l16, n_base, pb, py, px, pv, base0, base1, ld0, ld1, wz, af[J], bq[J], \
                                okq[J], ccq[J]); \
  if (NOL) nol_fetch(nk[NOL ? (J) : 0], ccq[J], s_nol, a.Cs); } while (0)
  // NOL: the operand transform runs when the stage is consumed, so the loads stay in flight meanwhile
#define MMA_STAGE(J)                                                                                      \
  if (NOL) nol_apply<FM>(bq[J], okq[J], nk[NOL ? (J) : 0], nol_relu);                                     \
  _Pragma("unroll") for (int i = 0; i < FN; ++i)                                                          \
  _Pragma("unroll") for (int f = 0; f < FM; ++f)                                                          \
    acc[i][f] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[J][i], bq[J][f], acc[i][f], 0, 0, 0);
#pragma unroll
  for (int j = 0; j < PD - 1; ++j)
    if (kbeg + j < kend) LOAD_STAGE(kbeg + j, j);
  int ks = kbeg;
  // steady state: every load of the PD steps is in range, so the body has no branches and the waitcnt pass
  // keeps PD - 1 stages of loads in flight (a guarded body makes it drain with vmcnt(0) at each join)
  for (; ks + 2 * PD - 2 < kend; ks += PD) {
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      LOAD_STAGE(ks + j + PD - 1, (j + PD - 1) % PD);
      MMA_STAGE(j)
    }
  }
  for (; ks < kend; ks += PD) {  // the last 1..2 PD-blocks of steps
#pragma unroll
    for (int j = 0; j < PD; ++j) {
      if (ks + j + PD - 1 < kend) LOAD_STAGE(ks + j + PD - 1, (j + PD - 1) % PD);
      if (ks + j < kend) { MMA_STAGE(j) }
    }
  }
#undef LOAD_STAGE
#undef MMA_STAGE

  if (KSPLIT > 1) {
    const int slot = wn + WAVES_N * wm;
    if (wk > 0) {
      float* dst = s_red + ((wk - 1) * WAVES_N * WAVES_M + slot) * TILE;
#pragma unroll
      for (int i = 0; i < FN; ++i)
#pragma unroll
        for (int f = 0; f < FM; ++f)
#pragma unroll
          for (int r = 0; r < 4; ++r) dst[((i * FM + f) * 4 + r) * 64 + lane] = acc[i][f][r];
    }
    __syncthreads();
    if (wk == 0) {
#pragma unroll
      for (int q = 1; q < KSPLIT; ++q) {
        const float* src = s_red + ((q - 1) * WAVES_N * WAVES_M + slot) * TILE;
#pragma unroll
        for (int i = 0; i < FN; ++i)
#pragma unroll
          for (int f = 0; f < FM; ++f)
#pragma unroll
            for (int r = 0; r < 4; ++r) acc[i][f][r] += src[((i * FM + f) * 4 + r) * 64 + lane];
      }
    }
    __syncthreads();  // partial tiles consumed: s_red may be reused for the statistics below
  }

  ptick(a.ptm, 2);
  // ---------------------------------------------------------------- epilogue
  // BN partial sums are reduced across the block's pixel-waves in LDS and published with ONE atomic per
  // (channel, statistic) per block into replica blk.x % NREP.
  float* s_st = s_red;  // [WAVES_M][BN_T][3]
  const bool want_stats = is_fwd<MODE>() && a.stats != nullptr;
  const bool want_red = want_stats || want_bnb;
  if (want_bnb && !PREFETCH_Y) load_y();
  if (wk == 0) {
#pragma unroll
    for (int i = 0; i < FN; ++i) {
      const int n0 = n_base + i * 16 + 4 * kgl;
      const bool nok = n0 < a.N;
      float bias[4] = {0.f, 0.f, 0.f, 0.f};
      if (is_fwd<MODE>() && a.bias && nok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bias[r] = a.bias[a.bgs * z + n0 + r];
      }
      float s[4] = {0.f, 0.f, 0.f, 0.f}, ss[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int m = m_base + f * 16 + l16;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][f][r] + bias[r];
        if (nok && pv[f]) {
          if (is_fwd<MODE>()) {
            bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + a.ogs * z + (int64_t)m * a.ldo + n0;
            uint2 w;
            w.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
            w.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
            *reinterpret_cast<uint2*>(o) = w;
#pragma unroll
            for (int r = 0; r < 4; ++r) { s[r] += v[r]; ss[r] += v[r] * v[r]; }
          } else {
            bf16_t* o = reinterpret_cast<bf16_t*>(a.out) + a.ogs * z + (int64_t)m * a.ldo + n0;
            add_sources(a, z, (int64_t)m, n0, v);
            store4(o, v);
            if (want_bnb && n0 < bN) {  // dz of the BN tail this gradient feeds, and its statistics
              const uint2 u = ypre[i][f], q = rpre[i][f];
              const float yv[4] = {__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                                   __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
              const float rv[4] = {__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                                   __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u)};
              const int cl = wn * WN + i * 16 + 4 * kgl;
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const float t = yv[r] * s_bn[cl + r] + s_bn[BN_T + cl + r];
                float dz = rbf(v[r]), xh2 = 0.f;  // the stored gradient: the apply pass recomputes dz from it
                if (a.bkind == ACT_RELU) {
                  dz = t > 0.f ? dz : 0.f;
                } else if (a.bkind == ACT_SIGMOID) {
                  const float sg = sigmoidf_(t);
                  dz *= sg * (1.f - sg);
                } else if (a.bkind == ADD_RELU) {
                  float rr = rv[r];
                  if (a.br_bn) {
                    xh2 = (rr - s_bn[6 * BN_T + cl + r]) * s_bn[7 * BN_T + cl + r];
                    rr = rr * s_bn[4 * BN_T + cl + r] + s_bn[5 * BN_T + cl + r];
                  }
                  dz = (t + rr) > 0.f ? dz : 0.f;
                }
                const float xh = (yv[r] - s_bn[2 * BN_T + cl + r]) * s_bn[3 * BN_T + cl + r];
                s[r] += dz;
                ss[r] += dz * xh;
                s2[r] += dz * xh2;
              }
            }
          }
        }
      }
      if (want_red) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // pixels of a 16-lane row -> lane 15 (DPP, common.h)
          s[r] = row16_sum(s[r]);
          ss[r] = row16_sum(ss[r]);
          if (bres) s2[r] = row16_sum(s2[r]);
        }
        if (l16 == 15) {
          const int cl = wn * WN + i * 16 + 4 * kgl;  // channel within the block tile
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            s_st[(wm * BN_T + cl + r) * 3 + 0] = s[r];
            s_st[(wm * BN_T + cl + r) * 3 + 1] = ss[r];
            s_st[(wm * BN_T + cl + r) * 3 + 2] = s2[r];
          }
        }
      }
    }
  }
  if (want_red) {
    __syncthreads();
    const int rep = blk.x % (want_bnb ? a.bbn.pnrep : a.stats_nrep);
    // forward: [G][NREP][2][N] (sum y, sum y^2); fused BN backward: rows 0/1 (2 with a BN2 residual) of
    // the tail's [G][NREP][3][bN]
    const int nrow = want_bnb ? (a.br_bn ? 3 : 2) : 2;
    const int nlim = want_bnb ? bN : a.N;
    const int64_t gb = want_bnb ? (a.bpgs < 0 ? (int64_t)z * NREP * 3 * bN : (int64_t)z * a.bpgs)
                                : (int64_t)z * NREP * 2 * a.N;
    double* dst = want_bnb ? a.bpart : a.stats;
    for (int q = threadIdx.x; q < BN_T * 3; q += 256) {
      const int cl = q / 3, which = q - cl * 3;
      const int n = blk.y * BN_T + cl;
      if (n < nlim && which < nrow) {
        float v = 0.f;
#pragma unroll
        for (int w2 = 0; w2 < WAVES_M; ++w2) v += s_st[(w2 * BN_T + cl) * 3 + which];
        atomicAdd(dst + gb + ((int64_t)rep * (want_bnb ? 3 : 2) + which) * nlim + n, (double)v);
      }
    }
  }
  ptick(a.ptm, 3);
}

// ------------------------------------------------------------------------------------------------
// Staging of one im2col weight-gradient chunk (MCH pixels): dy [MCH][TN] and the im2col rows [MCH][TK] of
// the forward input, loaded by 16-byte units into registers (so that the next chunk's loads are in flight
// while this chunk's MFMAs run) and stored into pixel-major LDS images, with the normalise-on-load
// transform applied on the way (the forward conv read act(BN(y)) on load: rebuild the operand the same way).
struct WgCtx {
  int n0, mend, HWo;
  float ihwo, iwo;  // 1 / HWo, 1 / Wo (fdiv24); ihwo = 0: M >= 2^24, integer division
  const bf16_t *base0, *base1, *dyz;
};

template <int TN, int TK, int MCH>
struct WgStage {
  static constexpr int VY = MCH * (TN / 8), VX = MCH * (TK / 8);
  static constexpr int NY = (VY + 255) / 256, NX = (VX + 255) / 256;
  uint4 ry[NY], rx[NX];
  uint32_t rok;  // which rx hold real input (not zero padding)

  DEV void load(const WgradArgs& a, const WgCtx& c, int mc, const int* s_tab) {
    rok = 0;
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const int v = threadIdx.x + 256 * i;
      ry[i] = make_uint4(0, 0, 0, 0);
      if (v < VY) {
        const int p = v / (TN / 8), cg = v - p * (TN / 8);
        const int m = mc + p, n = c.n0 + cg * 8;
        if (m < c.mend && n < a.Co) ry[i] = *reinterpret_cast<const uint4*>(c.dyz + (int64_t)m * a.ldd + n);
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int v = threadIdx.x + 256 * i;
      rx[i] = make_uint4(0, 0, 0, 0);
      if (v < VX) {
        const int p = v / (TK / 8), g = v - p * (TK / 8);
        const int m = mc + p;
        const int e = s_tab[g];
        if (m < c.mend && ((e >> 29) & 1)) {
          const int b = c.ihwo != 0.f ? fdiv24(m, c.HWo, c.ihwo) : m / c.HWo, r = m - b * c.HWo;
          const int oh = c.ihwo != 0.f ? fdiv24(r, a.Wo, c.iwo) : r / a.Wo, ow = r - oh * a.Wo;
          const int ih = oh * a.sh - a.ph + ((e >> 21) & 127);
          const int iw = ow * a.sw - a.pw + ((e >> 14) & 127);
          if (ih >= 0 && ih < a.Hi && iw >= 0 && iw < a.Wi) {
            const int seg = (e >> 28) & 1;
            const bf16_t* sb = seg ? c.base1 : c.base0;
            rx[i] = *reinterpret_cast<const uint4*>(sb + ((int64_t)(b * a.Hi + ih) * a.Wi + iw) * a.src.ld[seg] + (e & 16383));
            rok |= 1u << i;
          }
        }
      }
    }
  }

  DEV void store(const WgradArgs& a, bf16_t* s_dy, int ldy, bf16_t* s_x, int ldx, const float* s_nsc,
                 const float* s_nsh) const {
#pragma unroll
    for (int i = 0; i < NY; ++i) {
      const int v = threadIdx.x + 256 * i;
      if (v < VY) {
        const int p = v / (TN / 8), cg = v - p * (TN / 8);
        *reinterpret_cast<uint4*>(&s_dy[p * ldy + cg * 8]) = ry[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NX; ++i) {
      const int v = threadIdx.x + 256 * i;
      if (v < VX) {
        const int p = v / (TK / 8), g = v - p * (TK / 8);
        uint4 u = rx[i];
        if (a.nol && ((rok >> i) & 1)) {
          uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            float lo = __uint_as_float(w4[h] << 16) * s_nsc[g * 8 + 2 * h] + s_nsh[g * 8 + 2 * h];
            float hi = __uint_as_float(w4[h] & 0xffff0000u) * s_nsc[g * 8 + 2 * h + 1] + s_nsh[g * 8 + 2 * h + 1];
            if (a.nol_kind == ACT_RELU) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
            w4[h] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
          }
          u = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        *reinterpret_cast<uint4*>(&s_x[p * ldx + g * 8]) = u;
      }
    }
  }
};

// Per-tile setup shared by the im2col weight-gradient kernels: the tap / channel table of the TK columns
// starting at k0 (columns past the reduction encode as invalid and stage zeros), the normalise-on-load
// constants of those columns, and the chunk context.
template <int TK>
DEV WgCtx wgrad_tile_setup(const WgradArgs& a, int n0, int k0, int split, int z, int* s_tab, float* s_nsc,
                           float* s_nsh) {
  const int Ktot = a.KH * a.KW * a.Cs;
  if (threadIdx.x < TK / 8) s_tab[threadIdx.x] = encode_kg(k0 / 8 + threadIdx.x, Ktot, a.Cs >> 3, a.KW, a.src.C0);
  if (a.nol) {
    for (int t = threadIdx.x; t < TK; t += 256) {
      const int e = encode_kg(k0 / 8 + t / 8, Ktot, a.Cs >> 3, a.KW, a.src.C0);
      const int c = (e & 16383) + (t & 7);
      const float* kz = a.nol_consts + (int64_t)z * 4 * a.Cs;
      s_nsc[t] = ((e >> 29) & 1) ? kz[c] : 0.f;
      s_nsh[t] = ((e >> 29) & 1) ? kz[a.Cs + c] : 0.f;
    }
  }
  WgCtx c;
  c.n0 = n0;
  c.HWo = a.Ho * a.Wo;
  c.ihwo = (int64_t)a.B * c.HWo < (1 << 24) ? 1.f / (float)c.HWo : 0.f;
  c.iwo = 1.f / (float)a.Wo;
  c.mend = min(a.B * c.HWo, (split + 1) * a.m_per_split);
  c.base0 = a.src.p[0] + a.src.gs[0] * z;
  c.base1 = a.src.p[1] ? a.src.p[1] + a.src.gs[1] * z : c.base0;
  c.dyz = a.dy + a.dgs * z;
  return c;
}

// Block: 256 threads, output tile TN (rows = cout) x TK (cols = k), MCH pixels staged per iteration.
// Global loads of chunk c+1 are issued into registers before the MFMAs of chunk c (which read LDS), so
// the load latency overlaps compute; one LDS image per operand, two barriers per chunk.
template <int TN, int TK, int MCH>
DEV void wgrad_block(const WgradArgs& a, const int tile, const int split, const int z) {
  // Row pitch 16 x odd elements (TN + 16 for even multiples of 16): with the row permutation below the 32
  // lanes of one ds_read_b64_tr_b16 read rows 0-7 of a 16-row block, whose 8-bank windows then tile the 64
  // banks exactly (the previous pitch TN + 8 with rows 0-3 and 8-11 per instruction left 2-way conflicts:
  // SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE = 0.38)
  constexpr int LDY = (TN / 16) % 2 ? TN : TN + 16, LDX = (TK / 16) % 2 ? TK : TK + 16;
  __shared__ __attribute__((aligned(16))) bf16_t s_dy[MCH * LDY];
  __shared__ __attribute__((aligned(16))) bf16_t s_x[MCH * LDX];
  __shared__ int s_tab[TK / 8];
  __shared__ float s_nsc[TK], s_nsh[TK];  // normalise-on-load constants of this tile's input channels
  constexpr int FN = TN / 16, FK = TK / 16, NFR = FN * FK;
  constexpr int FPW = (NFR + 3) / 4;  // fragments per wave

  const int ntk = a.Kpad / TK;
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * TN, k0 = tk * TK;
  const WgCtx c = wgrad_tile_setup<TK>(a, n0, k0, split, z, s_tab, s_nsc, s_nsh);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int mbeg = split * a.m_per_split, mend = c.mend;

  f32x4 acc[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();

  WgStage<TN, TK, MCH> st;
  if (mbeg < mend) st.load(a, c, mbeg, s_tab);
  for (int mc = mbeg; mc < mend; mc += MCH) {
    st.store(a, s_dy, LDY, s_x, LDX, s_nsc, s_nsh);
    __syncthreads();
    if (mc + MCH < mend) st.load(a, c, mc + MCH, s_tab);  // in flight during this chunk's MFMAs
#pragma unroll
    for (int kk = 0; kk < MCH / 32; ++kk) {
      // the MFMA's k index (pixel) of lane group g = lane >> 4 is any fixed permutation of the chunk's
      // pixels, the same for both operands: group g takes rows 16(g/2) + 4(g%2) + {0..3, 8..11}
      const int prow = kk * 32 + 16 * (lane >> 5) + 4 * ((lane >> 4) & 1);
#pragma unroll
      for (int j = 0; j < FPW; ++j) {
        const int fr = wid + 4 * j;
        if (fr < NFR) {
          const int fi = fr / FK, fk = fr - fi * FK;
          bf16x8 av = tr_read8<8>(&s_dy[prow * LDY], LDY, fi * 16, lane);
          bf16x8 bv = tr_read8<8>(&s_x[prow * LDX], LDX, fk * 16, lane);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  float* slab = a.slab + (((int64_t)z * a.splits + split) * a.Npad) * a.Kpad;
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int fr = wid + 4 * j;
    if (fr < NFR) {
      const int fi = fr / FK, fk = fr - fi * FK;
      const int row = n0 + fi * 16 + 4 * (lane >> 4);
      const int col = k0 + fk * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (row + r < a.Npad) slab[(int64_t)(row + r) * a.Kpad + col] = acc[j][r];
    }
  }
}

template <int TN, int TK, int MCH>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(WgradArgs a) {
  wgrad_block<TN, TK, MCH>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

// Horizontally batched weight gradients: every conv of a backward pass that uses this tile config, in
// ONE launch.  The weight gradient of a layer only needs its dy and forward input, both resident until
// the step ends, so all of them are deferred to the end of the backward pass; the ~40 (Model A) / ~90
// (Model C) small launches become <= 8 large ones that fill the 256 CUs (the deep, small-M layers run
// side by side instead of one after another).  Block -> job by binary search over the jobs' first blocks.
// The batched launches walk nvb virtual blocks with a grid of at most nvb hardware blocks: a side stream's
// batch may run on a capped, persistent grid (launch_wgrad_batched ``cap``), so that it never fills every CU
// slot while the critical data-gradient chain needs blocks (tools/kernel_phases.py: chain kernels waited up
// to 16 us for their blocks to start beside an uncapped batch).
#define WGRAD_FOR_VBLOCKS(BODY)                                                                            \
  for (int64_t vb = blockIdx.x; vb < nvb; vb += gridDim.x) {                                            \
    int lo = 0, hi = nj - 1;                                                                               \
    while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (jobs[mid].block0 <= vb) lo = mid; else hi = mid - 1; } \
    const WgradJob& J = jobs[lo];                                                                          \
    const int local = (int)(vb - J.block0);                                                                \
    const int per_z = J.ntiles * J.a.splits;                                                               \
    const int z = local / per_z, r = local - z * per_z;                                                    \
    BODY;                                                                                                  \
    __syncthreads(); /* the next virtual block re-stages the LDS tiles */                                  \
  }

template <int TN, int TK, int MCH>
__global__ __launch_bounds__(256) void conv_wgrad_batched_kernel(const WgradJob* __restrict__ jobs, int nj, int64_t nvb) {
  WGRAD_FOR_VBLOCKS((wgrad_block<TN, TK, MCH>(J.a, r % J.ntiles, r / J.ntiles, z)))
}

// ------------------------------------------------------------------------------------------------
// Large-tile weight gradient on the 32x32x16 MFMA (configs WGRAD_BIG_CFG0 + i).  The 16-32-wide tiles of
// wgrad_block re-stage dy and the im2col operand once per tile: Model C's wide 1x7 / 7x1 layers staged
// ~1.2 GB per step through LDS for ~50 GFLOP, at one 16x16x32 MFMA per two transposed reads.  Here a
// block owns a TN x TK tile of 64 or 128 rows / columns, its 4 waves a (TN/2) x (TK/2) quarter each, a
// grid of 32x32 accumulators: every k-step of 16 pixels costs (TN + TK)/64 read pairs for TN*TK/4096
// MFMAs of 16K MACs, and the operands are staged 2-4x less often.  Chunks of 64 pixels; the pitch of the
// pixel-major LDS images (width + 32 elements) puts the 4 rows of a transposed read (32 columns each) on
// disjoint bank quarters.  K tiles may run past Kpad (their columns stage zeros and are not stored).

template <int TN, int TK>
DEV void wgrad_big_block(const WgradArgs& a, const int tile, const int split, const int z) {
  constexpr int MCH = 64;
  constexpr int LDY = TN + 32, LDX = TK + 32;
  constexpr int FA = TN / 64, FB = TK / 64;  // 32x32 accumulators of a wave along n / k
  __shared__ __attribute__((aligned(16))) bf16_t s_dy[MCH * LDY];
  __shared__ __attribute__((aligned(16))) bf16_t s_x[MCH * LDX];
  __shared__ int s_tab[TK / 8];
  __shared__ float s_nsc[TK], s_nsh[TK];

  const int ntk = (a.Kpad + TK - 1) / TK;
  const int tn = tile / ntk, tk = tile - tn * ntk;
  const int n0 = tn * TN, k0 = tk * TK;
  const WgCtx c = wgrad_tile_setup<TK>(a, n0, k0, split, z, s_tab, s_nsc, s_nsh);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wn = (wid & 1) * (TN / 2), wk = (wid >> 1) * (TK / 2);
  const int mbeg = split * a.m_per_split, mend = c.mend;

  f32x16 acc[FA][FB];
#pragma unroll
  for (int i = 0; i < FA; ++i)
#pragma unroll
    for (int j = 0; j < FB; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  __syncthreads();

  WgStage<TN, TK, MCH> st;
  if (mbeg < mend) st.load(a, c, mbeg, s_tab);
  for (int mc = mbeg; mc < mend; mc += MCH) {
    st.store(a, s_dy, LDY, s_x, LDX, s_nsc, s_nsh);
    __syncthreads();
    if (mc + MCH < mend) st.load(a, c, mc + MCH, s_tab);
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
        for (int j = 0; j < FB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[i], bv[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  float* slab = a.slab + (((int64_t)z * a.splits + split) * a.Npad) * a.Kpad;
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
          if (row < a.Npad) slab[(int64_t)row * a.Kpad + col] = acc[i][j][r];
        }
      }
    }
}

template <int TN, int TK>
__global__ __launch_bounds__(256) void conv_wgrad_big_kernel(WgradArgs a) {
  wgrad_big_block<TN, TK>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

template <int TN, int TK>
__global__ __launch_bounds__(256) void conv_wgrad_big_batched_kernel(const WgradJob* __restrict__ jobs, int nj, int64_t nvb) {
  WGRAD_FOR_VBLOCKS((wgrad_big_block<TN, TK>(J.a, r % J.ntiles, r / J.ntiles, z)))
}

// ------------------------------------------------------------------------------------------------
// Patch weight gradient for 3x3 / stride 1 convolutions, padding 1 ("same") or 0 ("valid") (tile configs
// 12-19).  The im2col operand of a 3x3 conv re-reads every input pixel 9 times; here a block stages a strip
// of R output rows' INPUT rows (R + 2 rows with halo, CB channels) once in LDS and forms all 9 taps' MFMA operands from it with
// shifted transposed reads -- the input is read once per (strip, channel slice) instead of once per
// (tap, K tile).  Output rows are padded to a multiple of 8 pixels (Wo8) so that each 8-pixel MFMA row
// group stays inside one image row; the pad pixels carry dy = 0.  Work unit = (image, strip); split s of
// a job covers units [s * m_per_split, ...).  Tile = (TN output channels) x (all 9 taps x CB input
// channels), written to the same [split][Npad][Kpad] slab layout as the im2col kernel (k = tap*Cs + ci).
// R = 2 strips for the wide (W8 = 128) stem maps keep the staging registers and LDS within 2 blocks per CU.
template <int TN, int CB, int W8, int R>
DEV void wgrad_patch_block(const WgradArgs& a, const int tile, const int split, const int z) {
  constexpr int TAPS = 9;
  constexpr int CBP = CB + 8, LDY = TN + 8, WP = W8 + 2;
  constexpr int FN = TN / 16, FC = CB / 16, NFR = FN * TAPS * FC, FPW = (NFR + 3) / 4;
  constexpr int NPI = (R + 2) * WP * (CB / 8), NDI = R * W8 * (TN / 8);
  constexpr int NPL = (NPI + 255) / 256, NDL = (NDI + 255) / 256;
  __shared__ __attribute__((aligned(16))) bf16_t s_p[(R + 2) * WP * CBP];
  __shared__ __attribute__((aligned(16))) bf16_t s_y[R * W8 * LDY];
  __shared__ float s_nsc[CB], s_nsh[CB];

  const int ncs = a.Cs / CB;
  const int tn = tile / ncs, tcs = tile - tn * ncs;
  const int n0 = tn * TN, c0 = tcs * CB;
  const int Wo8 = (a.Wo + 7) & ~7;
  const int wpr = Wo8 + 2;  // staged input columns: iw = -pw .. Wo8 + 1 - pw
  const int nstrip = (a.Ho + R - 1) / R;
  const int U = a.B * nstrip;
  const int ubeg = split * a.m_per_split, uend = min(U, ubeg + a.m_per_split);
  const int seg = (a.src.C1 > 0 && c0 >= a.src.C0) ? 1 : 0;
  const bf16_t* xz = a.src.p[seg] + a.src.gs[seg] * z + (c0 - seg * a.src.C0);
  const int ldx = a.src.ld[seg];
  const bf16_t* dyz = a.dy + a.dgs * z;
  if (a.nol) {
    const float* kz = a.nol_consts + (int64_t)z * 4 * a.Cs;
    for (int t = threadIdx.x; t < CB; t += 256) { s_nsc[t] = kz[c0 + t]; s_nsh[t] = kz[a.Cs + c0 + t]; }
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  f32x4 acc[FPW];
#pragma unroll
  for (int j = 0; j < FPW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 rp[NPL], ry[NDL];
  uint32_t pok = 0;
  const int npi = (R + 2) * wpr * (CB / 8), ndi = R * Wo8 * (TN / 8);
  auto load_unit = [&](int u) {
    const int b = u / nstrip, oh0 = (u - b * nstrip) * R;
    pok = 0;
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int v = threadIdx.x + 256 * i;
      rp[i] = make_uint4(0, 0, 0, 0);
      if (v < npi) {
        const int cg = v % (CB / 8), q = v / (CB / 8);
        const int j = q / wpr, c = q - j * wpr;
        const int ih = oh0 - a.ph + j, iw = c - a.pw;
        if (ih >= 0 && ih < a.Hi && iw >= 0 && iw < a.Wi) {
          rp[i] = *reinterpret_cast<const uint4*>(xz + ((int64_t)(b * a.Hi + ih) * a.Wi + iw) * ldx + cg * 8);
          pok |= 1u << i;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NDL; ++i) {
      const int v = threadIdx.x + 256 * i;
      ry[i] = make_uint4(0, 0, 0, 0);
      if (v < ndi) {
        const int cg = v % (TN / 8), p = v / (TN / 8);
        const int r = p / Wo8, ow = p - r * Wo8;
        const int oh = oh0 + r, n = n0 + cg * 8;
        if (oh < a.Ho && ow < a.Wo && n < a.Co)
          ry[i] = *reinterpret_cast<const uint4*>(dyz + ((int64_t)(b * a.Ho + oh) * a.Wo + ow) * a.ldd + n);
      }
    }
  };
  auto store_unit = [&]() {
#pragma unroll
    for (int i = 0; i < NPL; ++i) {
      const int v = threadIdx.x + 256 * i;
      if (v < npi) {
        const int cg = v % (CB / 8), q = v / (CB / 8);
        const int j = q / wpr, c = q - j * wpr;
        uint4 u = rp[i];
        if (a.nol && ((pok >> i) & 1)) {
          uint32_t w4[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            const int cc = cg * 8 + 2 * h;
            float lo = __uint_as_float(w4[h] << 16) * s_nsc[cc] + s_nsh[cc];
            float hi = __uint_as_float(w4[h] & 0xffff0000u) * s_nsc[cc + 1] + s_nsh[cc + 1];
            if (a.nol_kind == ACT_RELU) { lo = fmaxf(lo, 0.f); hi = fmaxf(hi, 0.f); }
            w4[h] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
          }
          u = make_uint4(w4[0], w4[1], w4[2], w4[3]);
        }
        *reinterpret_cast<uint4*>(&s_p[(j * WP + c) * CBP + cg * 8]) = u;
      }
    }
#pragma unroll
    for (int i = 0; i < NDL; ++i) {
      const int v = threadIdx.x + 256 * i;
      if (v < ndi) {
        const int cg = v % (TN / 8), p = v / (TN / 8);
        *reinterpret_cast<uint4*>(&s_y[p * LDY + cg * 8]) = ry[i];
      }
    }
  };

  __syncthreads();  // NOL constants
  const int ksteps = R * Wo8 / 32;
  if (ubeg < uend) load_unit(ubeg);
  for (int u = ubeg; u < uend; ++u) {
    store_unit();
    __syncthreads();
    if (u + 1 < uend) load_unit(u + 1);  // in flight during this strip's MFMAs
    for (int ks = 0; ks < ksteps; ++ks) {
      const int prow = ks * 32 + 8 * (lane >> 4);  // this lane group's 8 pixels: one image row
      const int r = prow / Wo8, ow = prow - r * Wo8;
#pragma unroll
      for (int j = 0; j < FPW; ++j) {
        const int fr = wid + 4 * j;
        if (fr < NFR) {
          const int cs = fr % FC, t2 = fr / FC;
          const int tap = t2 % TAPS, fi = t2 / TAPS;
          const int kh = tap / 3, kw = tap - kh * 3;
          bf16x8 av = tr_read8(&s_y[prow * LDY], LDY, fi * 16, lane);
          bf16x8 bv = tr_read8(&s_p[((r + kh) * WP + ow + kw) * CBP], CBP, cs * 16, lane);
          acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[j], 0, 0, 0);
        }
      }
    }
    __syncthreads();
  }
  float* slab = a.slab + (((int64_t)z * a.splits + split) * a.Npad) * a.Kpad;
#pragma unroll
  for (int j = 0; j < FPW; ++j) {
    const int fr = wid + 4 * j;
    if (fr < NFR) {
      const int cs = fr % FC, t2 = fr / FC;
      const int tap = t2 % TAPS, fi = t2 / TAPS;
      const int row = n0 + fi * 16 + 4 * (lane >> 4);
      const int col = tap * a.Cs + c0 + cs * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (row + q < a.Npad) slab[(int64_t)(row + q) * a.Kpad + col] = acc[j][q];
    }
  }
}

template <int TN, int CB, int W8, int R>
__global__ __launch_bounds__(256) void conv_wgrad_patch_kernel(WgradArgs a) {
  wgrad_patch_block<TN, CB, W8, R>(a, blockIdx.x, blockIdx.y, blockIdx.z);
}

template <int TN, int CB, int W8, int R>
__global__ __launch_bounds__(256) void conv_wgrad_patch_batched_kernel(const WgradJob* __restrict__ jobs, int nj, int64_t nvb) {
  WGRAD_FOR_VBLOCKS((wgrad_patch_block<TN, CB, W8, R>(J.a, r % J.ntiles, r / J.ntiles, z)))
}

// Sums the split-M partial slabs of many convolutions into the flat fp32 gradient buffer (deterministic,
// one launch per backward), reference weight layout [Cout][Cin][KH][KW].  Two thread mappings, chosen per
// descriptor by its split count (D.order, set by the host; D.lanes = threads per weight, a power of two <= 16):
// * order 1 (few splits, one lane; most of the bytes: Model C's wide layers): threads walk the OUTPUT in its
//   own order, a block owning FIN_EPT x 256 consecutive NCHW weights, so every store is a full-line
//   contiguous write.  (Walking the slab's k-fastest order scattered the stores with a KH*KW*4-byte
//   stride: each gradient line was assembled from partial writes of up to KH*KW blocks on different
//   XCDs, and the launch ran at ~1.5 TB/s.)  The slab reads are tap-strided runs of consecutive input
//   channels; a block covers ~FIN_EPT*256/taps channels of every tap, so the lines it reads are its own.
// * order 0 (many splits of a small weight: reads dominate): threads walk the slab's k-fastest order so
//   the split reads are coalesced; lane q sums splits q, q + lanes, ... with 8 loads in flight and the
//   lane partials are added in lane order through LDS -- deterministic.
// Descriptors own whole blocks, so the mapping is uniform within a block.
__global__ __launch_bounds__(256) void wgrad_finalize_kernel(const WgFinDesc* __restrict__ descs, int nd, float scale) {
  __shared__ float s_part[256];
  const int bx = (int)blockIdx.x;
  int lo = 0, hi = nd - 1;  // last descriptor with block0 <= bx
  while (lo < hi) { int mid = (lo + hi + 1) >> 1; if (descs[mid].block0 <= (int64_t)bx) lo = mid; else hi = mid - 1; }
  const WgFinDesc& D = descs[lo];
  const int L = D.lanes, EPB = 256 / L;
  const int taps = D.KH * D.KW;
  const int elems = (int)D.elems, splits = D.splits;
  const int64_t sstride = (int64_t)D.Npad * D.Kpad;
  if (D.order == 0) {  // slab order: elems = G * Co * taps * Cs
    const int Kt = taps * D.Cs, perS = D.Co * Kt;
    const int q = threadIdx.x / EPB, ie = threadIdx.x - q * EPB;
    const int e = (int)((int64_t)bx - D.block0) * EPB + ie;
    const int g = e / perS, r = e - g * perS, co = r / Kt, k = r - co * Kt;
    const int tap = k / D.Cs, ci = k - tap * D.Cs;
    const bool ok = e < elems && ci < D.Ci;
    const float* s = D.slab + ((int64_t)g * splits * D.Npad + co) * D.Kpad + k;
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (ok) {
      int sp = q;
      for (; sp + 7 * L < splits; sp += 8 * L) {
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += s[(int64_t)(sp + j * L) * sstride];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (sp + j * L < splits) acc[j] += s[(int64_t)(sp + j * L) * sstride];
    }
    s_part[threadIdx.x] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
    __syncthreads();
    if (ok && q == 0) {
      float sum = 0.f;
      for (int l = 0; l < L; ++l) sum += s_part[l * EPB + ie];
      D.grad[g * D.ggs + (co * D.Ci + ci) * taps + tap] = sum * scale;
    }
    return;
  }
  // output order: elems = G * Co * Ci * taps, one lane per weight, FIN_EPT weights per thread
  const int row = D.Ci * taps, per = D.Co * row;
  const int base = (int)((int64_t)bx - D.block0) * (256 * FIN_EPT) + threadIdx.x;
  const float* src[FIN_EPT];
  float* dst[FIN_EPT];
  bool ok[FIN_EPT];
  // (g, co, ci, tap) of the first weight by division, then advanced by 256 in mixed radix (one division
  // at most per step: the index math would otherwise rival the memory time of this streaming kernel)
  int g = base / per, r = base - g * per;
  int co = r / row, ci = (r - co * row) / taps, tap = r - co * row - ci * taps;
  const int s_ci = 256 / taps, s_tap = 256 - s_ci * taps;
#pragma unroll
  for (int j = 0; j < FIN_EPT; ++j) {
    const int e = base + j * 256;
    ok[j] = e < elems;
    src[j] = D.slab + ((int64_t)g * splits * D.Npad + co) * D.Kpad + tap * D.Cs + ci;
    dst[j] = D.grad + g * D.ggs + ((co * D.Ci + ci) * taps + tap);  // NCHW offset within group g
    tap += s_tap;
    ci += s_ci;
    if (tap >= taps) { tap -= taps; ++ci; }
    if (ci >= D.Ci) {
      if (s_ci < D.Ci) { ci -= D.Ci; ++co; }
      else { const int c = ci / D.Ci; co += c; ci -= c * D.Ci; }
    }
    while (co >= D.Co) { co -= D.Co; ++g; }
  }
  // (<= 8 splits) two independent chains per weight: up to 8 loads in flight per thread
  float a0[FIN_EPT], a1[FIN_EPT];
#pragma unroll
  for (int j = 0; j < FIN_EPT; ++j) { a0[j] = 0.f; a1[j] = 0.f; }
  int sp = 0;
  for (; sp + 1 < splits; sp += 2) {
#pragma unroll
    for (int j = 0; j < FIN_EPT; ++j) {
      if (ok[j]) {
        a0[j] += src[j][(int64_t)sp * sstride];
        a1[j] += src[j][(int64_t)(sp + 1) * sstride];
      }
    }
  }
  if (sp < splits) {
#pragma unroll
    for (int j = 0; j < FIN_EPT; ++j)
      if (ok[j]) a0[j] += src[j][(int64_t)sp * sstride];
  }
#pragma unroll
  for (int j = 0; j < FIN_EPT; ++j)
    if (ok[j]) *dst[j] = (a0[j] + a1[j]) * scale;
}

// ------------------------------------------------------------------------------------------------
// host launchers
// ------------------------------------------------------------------------------------------------
template <int MODE>
static int launch_conv_cfg(const ConvArgs& a, int G, int cfg, hipStream_t st) {
  const int M = a.B * a.Ho * a.Wo;
  const bool deep = cfg >= CONV_DEEP_CFG0;  // pipeline depth 4 (the same tile as cfg - CONV_DEEP_CFG0)
  if (deep) cfg -= CONV_DEEP_CFG0;
  const int nkg4 = ((a.Kpad / 8) + 3) & ~3;
#define LAUNCH_CFG(WN, WM, WAN, WAM, KS)                                                                \
  if (!deep) LAUNCH_PD(WN, WM, WAN, WAM, KS, 2)                                                         \
  else LAUNCH_PD(WN, WM, WAN, WAM, KS, 4)
#define LAUNCH_PD(WN, WM, WAN, WAM, KS, PD)                                                             \
  {                                                                                                     \
    constexpr int TILE = (WN / 16) * (WM / 16) * 4 * 64;                                                \
    size_t red = (size_t)(KS - 1) * WAN * WAM * TILE;                                                   \
    size_t st2 = (size_t)WAM * WN * WAN * 3;                                                            \
    size_t lds = (size_t)nkg4 * 4 + (red > st2 ? red : st2) * 4 +                                        \
                 (a.nol ? 2 * a.Cs * 4 : (a.bpart ? 8 * WN * WAN * 4 : 0)); \
    dim3 grid((M + WM * WAM - 1) / (WM * WAM), (a.N + WN * WAN - 1) / (WN * WAN), G);                    \
    hipLaunchKernelGGL((conv_igemm_kernel<MODE, WN, WM, WAN, WAM, KS, PD>), grid, dim3(256), lds, st, a); \
  }
  switch (cfg) {
    case 0: LAUNCH_CFG(16, 64, 1, 4, 1) break;
    case 1: LAUNCH_CFG(32, 32, 1, 4, 1) break;
    case 2: LAUNCH_CFG(32, 32, 2, 2, 1) break;
    case 3: LAUNCH_CFG(64, 32, 2, 2, 1) break;
    case 4: LAUNCH_CFG(32, 16, 2, 2, 1) break;
    case 5: LAUNCH_CFG(16, 32, 1, 2, 2) break;
    case 6: LAUNCH_CFG(32, 16, 1, 2, 2) break;
    case 7: LAUNCH_CFG(32, 16, 2, 1, 2) break;
    case 8: LAUNCH_CFG(32, 16, 1, 1, 4) break;
    case 9: LAUNCH_CFG(64, 16, 1, 1, 4) break;
    case 10: LAUNCH_CFG(16, 16, 1, 1, 4) break;
    case 11: LAUNCH_CFG(64, 32, 1, 1, 4) break;
    case 12: LAUNCH_CFG(16, 32, 1, 4, 1) break;
    case 13: LAUNCH_CFG(16, 16, 1, 4, 1) break;
    default: return -1;
  }
#undef LAUNCH_CFG
#undef LAUNCH_PD
  return (int)hipGetLastError();
}

int launch_conv(int mode, const ConvArgs& a0, int G, int cfg, hipStream_t st) {
  ConvArgs a = a0;
  a.xcd = (cfg & CONV_XCD) ? 1 : 0;
  cfg &= ~CONV_XCD;
  if ((cfg >= CONV_LDS_CFG0 && cfg < CONV_DEEP_CFG0) || cfg >= CONV_GLDS_CFG0) {  // LDS-staged kernels (conv_lds.hip)
    const int m = mode == MODE_FWD ? (a.nol ? MODE_FWD_NOL : MODE_FWD) : (a.bpart ? MODE_DGRAD_BNS : MODE_DGRAD);
    return launch_conv_lds(m, a, G, cfg, st);
  }
  if (mode == MODE_FWD)
    return a.nol ? launch_conv_cfg<MODE_FWD_NOL>(a, G, cfg, st) : launch_conv_cfg<MODE_FWD>(a, G, cfg, st);
  return a.bpart ? launch_conv_cfg<MODE_DGRAD_BNS>(a, G, cfg, st) : launch_conv_cfg<MODE_DGRAD>(a, G, cfg, st);
}

// Weight-gradient tile configurations (TN = output channels, TK = reduction columns, MCH = pixels per
// LDS chunk); keep in sync with wgrad_tile_shape and ops/functional.py WGRAD_TILES.  Configs 8-11 cover
// the whole reduction of a small-Cout layer in one tile: dy is read once per pixel and the im2col taps
// of neighbouring pixels re-hit L1, instead of every 32-wide K tile re-reading dy and its im2col slice
// from L2 (Model A's 16-channel 33x83 layers moved ~50 MB of L2 traffic each with TK = 32).
#define WGRAD_CFG_CASES(X)                                                                          \
  case 0: X(16, 32, 128) case 1: X(32, 32, 128) case 2: X(32, 64, 64) case 3: X(64, 64, 64)         \
  case 4: X(16, 64, 128) case 5: X(16, 32, 256) case 6: X(32, 32, 256) case 7: X(64, 32, 64)        \
  case 8: X(16, 192, 64) case 9: X(16, 128, 64) case 10: X(32, 192, 64) case 11: X(32, 320, 32)

// Patch configs 12-19 (TN, CB, max padded output width, strip rows); keep in sync with ops/functional.py
// WGRAD_PATCH.
#define WGRAD_PATCH_CASES(X)                                                                       \
  case 12: X(16, 16, 88, 4) case 13: X(32, 16, 88, 4) case 14: X(32, 32, 48, 4) case 15: X(64, 32, 24, 4) \
  case 16: X(32, 32, 128, 2) case 17: X(64, 32, 128, 2) case 18: X(64, 16, 128, 2) case 19: X(32, 16, 128, 2)

// Large-tile configs 32-35 (TN, TK; 64-pixel chunks); keep in sync with ops/functional.py WGRAD_BIG.
#define WGRAD_BIG_CASES(X) case 32: X(64, 64) case 33: X(64, 128) case 34: X(128, 64) case 35: X(128, 128)

int wgrad_big_shape(int cfg, int& TN, int& TK) {
  if (cfg < WGRAD_BIG_CFG0 || cfg >= WGRAD_BIG_CFG0 + WGRAD_BIG_NCFG) return -1;
  const int k = cfg - WGRAD_BIG_CFG0;
  TN = (k & 2) ? 128 : 64;
  TK = (k & 1) ? 128 : 64;
  return 0;
}

int wgrad_patch_shape(int cfg, int& TN, int& CB, int& W8, int& R) {
  static const int tn[] = {16, 32, 32, 64, 32, 64, 64, 32}, cb[] = {16, 16, 32, 32, 32, 32, 16, 16};
  static const int w8[] = {88, 88, 48, 24, 128, 128, 128, 128}, rr[] = {4, 4, 4, 4, 2, 2, 2, 2};
  if (cfg < WGRAD_PATCH_CFG0 || cfg >= WGRAD_PATCH_CFG0 + WGRAD_PATCH_NCFG) return -1;
  const int k = cfg - WGRAD_PATCH_CFG0;
  TN = tn[k]; CB = cb[k]; W8 = w8[k]; R = rr[k];
  return 0;
}

int wgrad_ntiles(int cfg, const WgradArgs& a) {
  if (cfg >= WGRAD_LEAN_CFG0 && cfg < WGRAD_LEAN_CFG0 + WGRAD_LEAN_NCFG) return wgrad_lean_ntiles(cfg, a);
  int TN, TK, CB, W8, R;
  if (!wgrad_patch_shape(cfg, TN, CB, W8, R)) {
    const int Wo8 = (a.Wo + 7) & ~7;
    const bool seg_ok = a.src.C1 == 0 || a.src.C0 % CB == 0;
    if (a.KH != 3 || a.KW != 3 || a.sh != 1 || a.sw != 1 || a.ph > 1 || a.pw > 1 || a.ph < 0 || a.pw < 0 ||
        a.Ho != a.Hi + 2 * a.ph - 2 || a.Wo != a.Wi + 2 * a.pw - 2 || a.Cs % CB || Wo8 > W8 || (R * Wo8) % 32 ||
        !seg_ok || a.Kpad < 9 * a.Cs)
      return -2;
    return ((a.Npad + TN - 1) / TN) * (a.Cs / CB);
  }
  if (!wgrad_big_shape(cfg, TN, TK)) return ((a.Npad + TN - 1) / TN) * ((a.Kpad + TK - 1) / TK);
  if (wgrad_tile_shape(cfg, TN, TK) || a.Kpad % TK) return -2;  // the K tiles must cover Kpad exactly
  return ((a.Npad + TN - 1) / TN) * (a.Kpad / TK);
}

int launch_wgrad(const WgradArgs& a, int G, int cfg, hipStream_t st) {
  if (cfg >= WGRAD_LEAN_CFG0 && cfg < WGRAD_LEAN_CFG0 + WGRAD_LEAN_NCFG) return launch_wgrad_lean(a, G, cfg, st);
  if (cfg >= WGRAD_BIG_CFG0) {
    const int nt = wgrad_ntiles(cfg, a);
    if (nt < 0) return nt;
#define LAUNCH_WGBIG(TN, TK)                                                                            \
  hipLaunchKernelGGL((conv_wgrad_big_kernel<TN, TK>), dim3(nt, a.splits, G), dim3(256), 0, st, a); \
  break;
    switch (cfg) {
      WGRAD_BIG_CASES(LAUNCH_WGBIG)
      default: return -1;
    }
#undef LAUNCH_WGBIG
    return (int)hipGetLastError();
  }
  if (cfg >= WGRAD_PATCH_CFG0) {
    const int nt = wgrad_ntiles(cfg, a);
    if (nt < 0) return nt;
#define LAUNCH_WGP(TN, CB, W8, R)                                                                      \
  hipLaunchKernelGGL((conv_wgrad_patch_kernel<TN, CB, W8, R>), dim3(nt, a.splits, G), dim3(256), 0, st, a); \
  break;
    switch (cfg) {
      WGRAD_PATCH_CASES(LAUNCH_WGP)
      default: return -1;
    }
#undef LAUNCH_WGP
    return (int)hipGetLastError();
  }
#define LAUNCH_WG(TN, TK, MCH)                                                                      \
  {                                                                                                 \
    dim3 grid(((a.Npad + TN - 1) / TN) * (a.Kpad / TK), a.splits, G);                               \
    hipLaunchKernelGGL((conv_wgrad_kernel<TN, TK, MCH>), grid, dim3(256), 0, st, a);                \
    break;                                                                                          \
  }
  int TN_, TK_;
  if (wgrad_tile_shape(cfg, TN_, TK_) || a.Kpad % TK_) return -2;  // the K tiles must cover Kpad exactly
  switch (cfg) {
    WGRAD_CFG_CASES(LAUNCH_WG)
    default: return -1;
  }
#undef LAUNCH_WG
  return (int)hipGetLastError();
}

int wgrad_tile_shape(int cfg, int& TN, int& TK) {
  static const int tn[] = {16, 32, 32, 64, 16, 16, 32, 64, 16, 16, 32, 32};
  static const int tk[] = {32, 32, 64, 64, 64, 32, 32, 32, 192, 128, 192, 320};
  if (cfg < 0 || cfg >= (int)(sizeof(tn) / sizeof(tn[0]))) return -1;
  TN = tn[cfg]; TK = tk[cfg];
  return 0;
}

int launch_wgrad_batched(int cfg, const WgradJob* d_jobs, int nj, int64_t nblocks, hipStream_t st, int64_t cap) {
  if (nblocks <= 0) return 0;
  dim3 grid((unsigned)(cap > 0 && cap < nblocks ? cap : nblocks));
  if (cfg >= WGRAD_LEAN_CFG0 && cfg < WGRAD_LEAN_CFG0 + WGRAD_LEAN_NCFG)
    return launch_wgrad_lean_batched(cfg, d_jobs, nj, nblocks, grid, st);
  if (cfg >= WGRAD_BIG_CFG0) {
#define LAUNCH_WGBIGB(TN, TK)                                                                                 \
  hipLaunchKernelGGL((conv_wgrad_big_batched_kernel<TN, TK>), grid, dim3(256), 0, st, d_jobs, nj, nblocks); \
  break;
    switch (cfg) {
      WGRAD_BIG_CASES(LAUNCH_WGBIGB)
      default: return -1;
    }
#undef LAUNCH_WGBIGB
    return (int)hipGetLastError();
  }
  if (cfg >= WGRAD_PATCH_CFG0) {
#define LAUNCH_WGPB(TN, CB, W8, R)                                                                              \
  hipLaunchKernelGGL((conv_wgrad_patch_batched_kernel<TN, CB, W8, R>), grid, dim3(256), 0, st, d_jobs, nj, nblocks); \
  break;
    switch (cfg) {
      WGRAD_PATCH_CASES(LAUNCH_WGPB)
      default: return -1;
    }
#undef LAUNCH_WGPB
    return (int)hipGetLastError();
  }
#define LAUNCH_WGB(TN, TK, MCH)                                                                              \
  hipLaunchKernelGGL((conv_wgrad_batched_kernel<TN, TK, MCH>), grid, dim3(256), 0, st, d_jobs, nj, nblocks); \
  break;
  switch (cfg) {
    WGRAD_CFG_CASES(LAUNCH_WGB)
    default: return -1;
  }
#undef LAUNCH_WGB
  return (int)hipGetLastError();
}

int launch_wgrad_finalize(const WgFinDesc* d_descs, int nd, int64_t nblocks, float scale, hipStream_t st) {
  if (nblocks <= 0) return 0;
  hipLaunchKernelGGL(wgrad_finalize_kernel, dim3((unsigned)nblocks), dim3(256), 0, st, d_descs, nd, scale);
  return (int)hipGetLastError();
}

}  // namespace mda
