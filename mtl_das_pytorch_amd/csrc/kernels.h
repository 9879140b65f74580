// Kernel argument structs and host launch entry points of the mtl_das_pytorch_amd HIP library.
// Every launcher enqueues on the given stream (PyTorch's current stream, so HIP-graph capture works)
// and returns hipGetLastError() (negative = rejected arguments).
#pragma once
#include "common.h"

namespace mda {

// 2: dgrad + fused BN-backward statistics; 3: forward with normalise-on-load of its input
enum { MODE_FWD = 0, MODE_DGRAD = 1, MODE_DGRAD_BNS = 2, MODE_FWD_NOL = 3 };

struct ConvArgs {
  Src2 src;
  const bf16_t* w;  // packed [Npad][Kpad] (+ z * wgs)
  int64_t wgs;
  const float* bias;  // FWD only, may be null
  int64_t bgs;
  void* out;  // bf16 [M][ldo] (+ z * ogs): FWD the pre-BN y, DGRAD the data gradient
  int64_t ogs;
  int ldo;
  double* stats;  // FWD: [G][NREP][2][N] fp64 (may be null); replica blockIdx.x % stats_nrep
  int stats_nrep;
  int B, Hs, Ws, Ho, Wo;
  int N, Npad, Cs;
  int KH, KW, sh, sw, ph, pw;
  int Kpad;
  // DGRAD only, optional (bpart null = off): fused BN-backward statistics.  When this dgrad's output is
  // the ONLY gradient source of a BN tail with an elementwise activation (ACT_NONE / ACT_RELU /
  // ACT_SIGMOID), the epilogue recomputes that tail's dz from the stored pre-BN y and accumulates
  // sum(dz), sum(dz * xhat) per channel into the tail's fp64 replica rows ([G][NREP][3][N], rows 0/1) --
  // the tail backward then runs its apply pass only (bn.hip launch_tail_bwd, fused == 2).
  const bf16_t* by; int64_t bygs; int ldby;
  BNArgs bbn;
  double* bpart;
  int bkind;
  // ... generalised to ONE OF SEVERAL gradient sources (statistics are linear in the gradient, so every
  // producer adds its share): bkind ACT_RELU or ADD_RELU, whose dz mask is relu'(BN(y) + r') with the
  // residual r' = r (identity shortcut) or BN2(r) (projection, br_bn = 1: third row sum(dz * xhat2)).
  // bN = the tail's channels (a concatenation gradient may have more: channels >= bN are not the tail's),
  // bpgs = group stride of bpart (-1: z * NREP * 3 * bN; 0: every group adds into the ONE tail of a
  // shared feature, whose BN constants are then group 0's).
  const bf16_t* br; int64_t brgs; int ldbr;
  BNArgs bbn2;
  int br_bn, bN;
  int64_t bpgs;
  // FWD only, optional (nol = 0 off): normalise-on-load.  The (single-segment) input is the previous
  // conv's pre-BN output y and the im2col operand is act(BN(y)) computed on load (act = nol_kind: ACT_NONE
  // or ACT_RELU), so the forward BN tail that materialised act(BN(y)) is not launched.  Block (0, 0) of each
  // group updates that BN's running statistics and publishes its constants (BNArgs::consts).
  BNArgs nbn;
  int nol, nol_kind;
  // DGRAD only, optional (nadd = 0 off): up to 3 more bf16 gradient sources of the same [M][N] tensor
  // ([M][ldadd] + z * addgs) added (in fp32, before the one rounding) in the epilogue, so the output is the
  // WHOLE gradient of the BN tail it feeds (one source: its statistics can then be fused above, and the
  // tail runs apply-only)
  const bf16_t* add[3];
  int64_t addgs[3];
  int ldadd[3];
  int nadd;
  // LDS-staged kernels (cfg >= CONV_LDS_CFG0, conv_lds.hip) with a cross-block split of K: fp32 partial
  // tiles [G][tiles][splits][BM*BN] and one arrival ticket per output tile (zero-initialised; the reducing
  // block resets it), sized by conv_lds_workspace
  float* ws;
  unsigned* cnt;
  int xcd;  // block_coords remap (common.h): XCD-contiguous tile order (set from the CONV_XCD cfg flag)
  uint64_t* ptm;  // optional per-block phase timers (common.h ptick; profiling only)
};

// ConvArgs::add: the extra gradient sources of output element (row m, channels n0 .. n0+3), added in order
DEV void add_sources(const ConvArgs& a, int z, int64_t m, int n0, float* v) {
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (s < a.nadd) {
      float q[4];
      load4(a.add[s] + a.addgs[s] * z + m * a.ldadd[s] + n0, q);
      v[0] += q[0]; v[1] += q[1]; v[2] += q[2]; v[3] += q[3];
    }
  }
}

// One output-pixel phase of an LDS-staged conv launch (conv_lds.hip): output pixels (b, oy0 + i*qy,
// ox0 + j*qx) for i < Hq, j < Wq, reduced over taps (kh, kw) = (rh + th*u, rw + tw*v), u < nh, v < nw,
// whose input pixel is (i*mh + ay + by*u, j*mw + ax + bx*v).  The forward is one phase; a strided data
// gradient has one phase per output parity (sub-pixel decomposition: only the taps that hit a real dy).
struct LdsPhase {
  int oy0, ox0, Hq, Wq;
  int rh, nh, rw, nw;
  int ay, ax;
  int m0;   // first blockIdx.x of the phase
  int Kp;   // nh * nw * Cs padded to the K chunk
};
// Strip plan of a patch conv launch (conv_lds.hip conv_patch_kernel): R output rows per block, nstrip strips
// per image, nslice channel slices; source pixel of strip element (j, q) = (oh0 + dy0 + j, dx0 + q).
struct PatchPlan {
  int R, nstrip, nslice, Hout, Wout, dy0, dx0;
};
struct LdsPlan {
  LdsPhase ph[4];
  int nph;
  int mh, mw, by, bx, th, tw, qy, qx;
  int splits;  // cross-block split of the K chunks
  int ntab;    // per-block k-group table entries (LDS)
};

// ------------------------------------------------------------------------------------------------
// Weight gradient
// ------------------------------------------------------------------------------------------------
struct WgradArgs {
  Src2 src;          // forward input (bf16)
  const bf16_t* dy;  // [M][ldd] (+ z * dgs)
  int64_t dgs;
  int ldd;
  float* slab;       // [G][splits][Npad][Kpad]
  int splits, m_per_split;
  int B, Hi, Wi, Ho, Wo;
  int Co, Npad, Cs;
  int KH, KW, sh, sw, ph, pw;
  int Kpad;
  // optional (nol = 0 off): the forward conv normalised its input on load (ConvArgs::nol); the x operand is
  // rebuilt the same way from the BN constants the forward published ([G][4][Cs]: scale, shift, ...)
  const float* nol_consts;
  int nol, nol_kind;
};

// One conv of a horizontally batched weight-gradient launch (device table, built by wgrad_table).
struct WgradJob {
  WgradArgs a;
  int ntiles;      // (Npad / TN) * (Kpad / TK)
  int G;
  int64_t block0;  // first block of this job in the batched grid
};

// Sums the split-M partial slabs of many convolutions and scatters them into the flat fp32 gradient
// buffer in the reference weight layout [Cout][Cin][KH][KW] (deterministic, one launch per backward).
struct WgFinDesc {
  const float* slab;  // [G][splits][Npad][Kpad]
  float* grad;        // NCHW weight grad of group 0
  int64_t ggs;        // element stride between groups in the flat grad buffer
  int G, splits, Npad, Kpad, Co, Ci, Cs, KH, KW;
  int lanes;          // threads per weight (power of two <= 16): the splits are summed in lanes x parallel
  int order;          // 1: output (NCHW) order, lanes == 1, FIN_EPT weights per thread; 0: slab order
  int _pad;
  int64_t elems;      // G * Co * Ci * KH * KW (order 1); G * Co * KH * KW * Cs (order 0)
  int64_t block0;     // first block index of this descriptor
};
// weights per thread of wgrad_finalize's output-order mapping (order 1): a block owns FIN_EPT * 256
// consecutive NCHW weights
constexpr int FIN_EPT = 2;  // measured 1 / 2 / 4 / 8: C 130 / 101 / 105 / 160 us, A 18.4 / 18.2 / 21.1 / - us

enum TailKind { ACT_NONE = 0, ACT_RELU = 1, ACT_SIGMOID = 2, SIGMUL = 3, ADD_RELU = 4, POOL_RELU = 5 };

struct TailArgs {
  const bf16_t* y; int64_t ygs; int ldy;
  BNArgs bn;
  const bf16_t* r; int64_t rgs; int ldr;  // SIGMUL: multiplier; ADD_RELU: residual (raw x or y2)
  BNArgs bn2; int r_bn;
  bf16_t* out; int64_t ogs; int ldo;
  int B, H, W, C;
  // backward only
  GradSrcs g;                       // upstream bf16 gradient(s) on the tail's output grid
  double* part; int chunk_px;       // [G][NREP][3][C] fp64 replica sums (zeroed per step); pixels per chunk
  bf16_t* dzbuf; int64_t dzgs; int lddz;  // optional dz store (reduce) / load (apply), bf16
  bf16_t* side; int64_t sgs; int lds;     // side gradient output (bf16)
  bf16_t* dy; int64_t dgs; int ldd;
  bf16_t* dy2; int64_t d2gs; int ldd2;
  float* dgamma; float* dbeta; float* dgamma2; float* dbeta2; int64_t pgs;
  uint64_t* tsc;                    // optional phase timestamps (profiling; null in production)
  uint64_t* ptm;                    // optional per-block phase timers (common.h ptick; profiling only)
  // apply-only backward (fused = 2) of a multi-source tail: no reduce pass ran, so the apply pass stores
  // the side output itself (apply_side)
  int apply_side;
  float gscale;                     // factor on the d(gamma), d(beta) the apply writes (SyncBN: 1 / world)
};

struct TailJob {  // one tail of a batched forward-tail launch (bn.hip tail_fwd_batched_kernel)
  TailArgs a;
  int blocks;      // blocks of this tail (its grid x), one group (z = 0)
  int block0;      // first block of this tail in the batched grid
};

struct HeadArgs {
  const bf16_t* feat; int64_t fgs; int ldf;  // per task [B*HW][C] (+ t * fgs)
  const int64_t* labels; int lab_stride, lab_off;  // label of (b, t) = labels[b*lab_stride + lab_off + t]
  int T, B, HW, C;
  int ncls[4];
  float w[4];
  float* logp;      // [T][B][16]
  bf16_t* dfeat;    // [T][B*HW][C] bf16 (+ t * dgs), may be null (eval)
  int64_t dgs;
  float* metrics;   // [T][4]: loss_sum, correct, count, abs_err_sum
  int* confusion;   // [T][16][16]
  const int64_t* nvalid;  // samples b >= *nvalid are padding: no metrics, no gradient (may be null)
};

struct ClsArgs {
  const bf16_t* x; int ldx;      // [B*HW][C] last feature map
  const float* W; const float* bias;  // fc [N][C], [N]
  const int64_t* labels;         // joint labels [B]
  int B, HW, C, N;
  float p_drop;                  // dropout probability (0 in eval)
  const int64_t* seed;           // device counter (advanced by cls_wgrad each training step)
  float* feat;                   // [B][C] post-dropout features (fp32)
  float* logits;                 // [B][N]
  float* dlogits;                // [B][N] (training)
  bf16_t* dx;                    // [B*HW][C] bf16 grad (training), may be null
  float* metrics;                // [3][4]: joint, distance, event -> loss, correct, count, abs_err
  int* confusion;                // [2][16][16]: distance, event
  float* dW; float* db;          // flat-grad slots (cls_wgrad)
  const int64_t* nvalid;         // padding mask for metrics (may be null)
};

// ------------------------------------------------------------------------------------------------
struct PoolArgs {
  const bf16_t* x; int ldx;     // input [B*H*W][C] (bf16)
  bf16_t* y; int ldy;           // output [B*Ho*Wo][C]
  GradSrcs g;                   // backward: grad of output = sum of bf16 sources (concat consumers)
  bf16_t* dx; int lddx;         // backward: grad of input (bf16)
  int B, H, W, C, Ho, Wo;
  uint8_t* am;                  // optional max-pool argmax (window position 0..8) [B*Ho*Wo][C]: written by
                                // the training forward, read by the backward instead of re-reading the windows
};

struct OptSeg {
  int64_t off, n;
  int kind;  // 0 = plain flat range, 3 = conv weight with both images (optim.hip adam_pack_kernel)
  bf16_t* wf;
  bf16_t* wd;
  int Co, Ci, KH, KW, Cs, Kpad_f, Kpad_d;
  // members of a horizontally fused conv (engine/core.py ConvLayer concat): the member's image is a window of
  // the group's -- kext_f = forward-image columns this member writes per row (its own taps, embedded at the
  // group's tap offset by the wf pointer; 0 = Kpad_f), tap_ld = data-gradient-image column stride between taps
  // (the group's Cout; 0 = Co)
  int kext_f, tap_ld;
  int64_t block0;
};

// Conv-weight tiles of the fused Adam + pack (optim.hip adam_pack_kernel): PACK_TCO co x pack_tile_ci(taps) ci x
// all taps (~2K elements: 256 ci of a 1x1, 24 of a 3x3, 8 of a 7x7), staged in LDS rows of at most
// PACK_TILE_FLOATS floats; keep in sync with engine/core.py build_optseg_table.
constexpr int PACK_TCO = 8, PACK_TILE_FLOATS = 512;
__host__ __device__ inline int pack_tile_ci(int taps) { return std::max(8, (256 / taps) & ~7); }

struct AdamArgs {
  float* p; const float* g; float* m; float* v;
  int64_t n;  // flat buffer length (multiple of 4)
  const float* lr; const float* step;  // device scalars (step = number of completed steps)
  float b1, b2, eps, wd, grad_scale;
  int update;  // 0: pack only
  int inc_step;  // advance the step counter after the update (0: a partial update -- another launch of the step does)
  int t_pre;     // 1: this step already advanced the counter (launch_step_inc at the step's start): t = step, else
                 // t = step + 1
  int64_t* cursor;  // optional: the batch-index schedule's cursor (gather_batch), advanced with the step counter
};
// the step counter (+ the schedule cursor) advanced by one thread: after the update (launch_adam_pack, inc_step)
// or early in the step on a side stream (AdamArgs::t_pre)
int launch_step_inc(float* step, int64_t* cursor, hipStream_t st);

int launch_conv(int mode, const ConvArgs& a, int G, int cfg, hipStream_t st);
// LDS-staged implicit GEMM (conv_lds.hip): cfg = CONV_LDS_CFG0 + 8 * tile + 4 * (KC == 128) + log2(splits)
constexpr int CONV_LDS_CFG0 = 16, CONV_LDS_NCFG = 64;
// register-pipelined conv_igemm tiles 0-13 at pipeline depth 4 (conv.hip): cfg = CONV_DEEP_CFG0 + tile
constexpr int CONV_DEEP_CFG0 = 128, CONV_DEEP_NCFG = 14;
// LDS-DMA implicit GEMM (conv_lds.hip conv_glds_kernel): cfg = CONV_GLDS_CFG0 + 4 * tile + log2(splits)
constexpr int CONV_GLDS_CFG0 = 160, CONV_GLDS_NCFG = 32;
// patch conv for 3x3 / stride-1 layers (conv_lds.hip conv_patch_kernel): cfg = CONV_PATCH_CFG0 + 3 * tile + cb
// (tile: BM x BN of PT_BM / PT_BN, cb: channel slice 16 / 32 / 64)
constexpr int CONV_PATCH_CFG0 = 192, CONV_PATCH_NCFG = 15;
// deep-ring LDS-DMA configs (conv_glds_kernel with up to 8 stages): cfg = CONV_GDEEP_CFG0 + 4 * tile + log2(splits)
constexpr int CONV_GDEEP_CFG0 = 208, CONV_GDEEP_NCFG = 32;
// persistent, DMA-pipelined patch conv (one channel slice): cfg = CONV_PATCHP_CFG0 + 3 * tile + cb
constexpr int CONV_PATCHP_CFG0 = 240, CONV_PATCHP_NCFG = 15;
// cfg flag of any conv config: launch it in XCD-contiguous tile order (ConvArgs::xcd, common.h block_coords)
constexpr int CONV_XCD = 4096;
int launch_conv_lds(int mode, const ConvArgs& a, int G, int cfg, hipStream_t st);
// fp32 workspace floats and ticket count a cfg needs (0 when it does not split K); < 0: cfg invalid for a
int conv_lds_workspace(int mode, const ConvArgs& a, int G, int cfg, int64_t& ws_floats, int64_t& ntickets);
int launch_wgrad(const WgradArgs& a, int G, int cfg, hipStream_t st);
int wgrad_tile_shape(int cfg, int& TN, int& TK);
constexpr int WGRAD_PATCH_CFG0 = 12, WGRAD_PATCH_NCFG = 8;  // wgrad cfgs 12-19: 3x3/s1 patch kernels (conv.hip)
constexpr int WGRAD_BIG_CFG0 = 32, WGRAD_BIG_NCFG = 4;  // wgrad cfgs 32-35: 32x32x16 large-tile kernels
constexpr int WGRAD_LEAN_CFG0 = 36, WGRAD_LEAN_NCFG = 12;  // wgrad cfgs 36-47: lean-staging im2col (wgrad_lean.hip;
                                                             // 44-47 on the 32x32x16 MFMA)
int wgrad_lean_shape(int cfg, int& TN, int& TK);
int wgrad_lean_ntiles(int cfg, const WgradArgs& a);
int launch_wgrad_lean(const WgradArgs& a, int G, int cfg, hipStream_t st);
int launch_wgrad_lean_batched(int cfg, const WgradJob* d_jobs, int nj, int64_t nblocks, dim3 grid, hipStream_t st);
int wgrad_patch_shape(int cfg, int& TN, int& CB, int& W8, int& R);
int wgrad_ntiles(int cfg, const WgradArgs& a);  // tiles per group of a wgrad launch, < 0: cfg invalid for a
// cap > 0: at most cap hardware blocks walk the nblocks virtual blocks (persistent grid)
int launch_wgrad_batched(int cfg, const WgradJob* d_jobs, int nj, int64_t nblocks, hipStream_t st, int64_t cap = 0);
int launch_wgrad_finalize(const WgFinDesc* d_descs, int nd, int64_t nblocks, float scale, hipStream_t st);
int launch_tail_fwd(int kind, const TailArgs& a, int G, int blocks, hipStream_t st);
int launch_tail_fwd_batched(int kind, const TailJob* d_jobs, int nj, int nblocks, int maxC, hipStream_t st);
int launch_tail_bwd_batched(int kind, int cgb, int reduce, const TailJob* d_jobs, int nj, int nblocks, hipStream_t st);
int launch_tail_bwd(int kind, const TailArgs& a, int G, int blocks, int fused, hipStream_t st);
int launch_mtl_head(const HeadArgs& a, hipStream_t st);
int launch_cls_head(const ClsArgs& a, int64_t* seed_mut, hipStream_t st);
struct ZeroRanges {  // up to 4 16-byte-aligned regions a launch zeroes (gather_batch: the arena's zeroed buffers)
  uint4* p[4];
  int64_t n16[4];     // 16-byte units
  int n;
};
int launch_gather_batch(const float* X, const int64_t* idx, const int64_t* lab, int lab_w, bf16_t* out,
                        int64_t* lab_out, int B, int Cin, int H, int W, int taps, int off, const ZeroRanges& zero,
                        const int64_t* cursor, int nrows,
                        hipStream_t st);
int launch_pool3(int is_max, int backward, const PoolArgs& a, hipStream_t st);
// synth.hip: on-device synthetic DAS samples (data/synthetic.py physical model, Philox noise)
constexpr int SYNTH_NPARAM = 9;  // per sample: distance, event, x0, t0, jitter[4], snr_db
struct SynthArgs {
  const float* params;  // [n][SYNTH_NPARAM]
  float* out;           // [n][C][H][W] fp32
  int C, H, W;
  int noise;            // 0: clean signal only
  uint64_t key;         // Philox key (the draw's noise seed)
  int64_t sample0;      // global index of sample 0 (Philox counter)
};
int launch_synth_das(const SynthArgs& a, int n, hipStream_t st);
int launch_philox_kat(const uint32_t* ctr, uint64_t key, uint32_t* out, int n, hipStream_t st);
int launch_tick(uint64_t* buf, uint64_t* q, int i, hipStream_t st);
int launch_grad_sum(const GradSrcs& g, bf16_t* out, int ldo, int64_t M, int C, hipStream_t st);
int launch_adam_pack(const AdamArgs& a, const OptSeg* d_segs, int ns, int64_t nblocks, hipStream_t st);

}  // namespace mda
