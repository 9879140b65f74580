// pybind11 bindings of the HIP kernel library (module `_mda_hip`).
//
// The Python side (mtl_das_pytorch_amd/ops/hip.py) passes raw device pointers (tensor.data_ptr()),
// the current HIP stream handle (torch.cuda.current_stream().cuda_stream) and plain dicts of kernel
// arguments; no PyTorch C++ headers are needed, so the library builds in seconds with hipcc and shares
// the HIP runtime (libamdhip64.so.7) that torch has already loaded into the process.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "kernels.h"

namespace py = pybind11;
using namespace mda;

namespace {

int64_t I(const py::dict& d, const char* k, int64_t dflt = 0) {
  if (!d.contains(k)) return dflt;
  py::object o = d[k];
  if (o.is_none()) return dflt;
  return o.cast<int64_t>();
}
double F(const py::dict& d, const char* k, double dflt = 0.0) {
  if (!d.contains(k)) return dflt;
  py::object o = d[k];
  if (o.is_none()) return dflt;
  return o.cast<double>();
}
template <typename T>
T* P(const py::dict& d, const char* k) {
  return reinterpret_cast<T*>(static_cast<intptr_t>(I(d, k, 0)));
}
hipStream_t S(int64_t s) { return reinterpret_cast<hipStream_t>(static_cast<intptr_t>(s)); }

void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("mtl_das_pytorch_amd HIP launch failed: ") + what + " rc=" + std::to_string(rc));
}

Src2 parse_src(const py::dict& d) {
  Src2 s{};
  s.p[0] = P<const bf16_t>(d, "p0");
  s.p[1] = P<const bf16_t>(d, "p1");
  s.gs[0] = I(d, "gs0");
  s.gs[1] = I(d, "gs1");
  s.ld[0] = (int)I(d, "ld0");
  s.ld[1] = (int)I(d, "ld1", s.ld[0]);
  s.C0 = (int)I(d, "C0");
  s.C1 = (int)I(d, "C1");
  return s;
}

GradSrcs parse_grads(const py::list& l) {
  GradSrcs g{};
  if (l.size() > 6) throw std::runtime_error("at most 6 gradient sources");
  g.n = (int)l.size();
  for (int i = 0; i < g.n; ++i) {
    py::tuple t = l[i].cast<py::tuple>();
    g.p[i] = reinterpret_cast<const bf16_t*>(static_cast<intptr_t>(t[0].cast<int64_t>()));
    g.gs[i] = t[1].cast<int64_t>();
    g.ld[i] = t[2].cast<int>();
    // consumers read 8 channels (16 bytes) per load
    if ((reinterpret_cast<uintptr_t>(g.p[i]) & 15) || g.ld[i] % 8 || g.gs[i] % 8)
      throw std::runtime_error("gradient source: 16-byte aligned base, pitch and group stride (multiples of 8) required");
  }
  return g;
}

BNArgs parse_bn(const py::dict& d) {
  BNArgs b{};
  b.stats = P<const double>(d, "stats");
  b.gamma = P<const float>(d, "gamma");
  b.beta = P<const float>(d, "beta");
  b.run_mean = P<float>(d, "run_mean");
  b.run_var = P<float>(d, "run_var");
  b.nbt = P<int64_t>(d, "nbt");
  b.pstride = I(d, "pstride");
  b.C = (int)I(d, "C");
  b.count = (int)I(d, "count");
  b.eps = (float)F(d, "eps", 1e-5);
  b.momentum = (float)F(d, "momentum", 0.1);
  b.training = (int)I(d, "training", 1);
  b.consts = P<float>(d, "consts");
  b.nrep = (int)I(d, "nrep", NREP);
  b.pnrep = (int)I(d, "pnrep", NREP);
  b.sld = (int)I(d, "sld", b.C);
  if (b.sld < b.C) throw std::runtime_error("bn: stats pitch below the channel count");
  if (b.pnrep < 1 || b.pnrep > NREP || (b.pnrep & (b.pnrep - 1))) throw std::runtime_error("bn: pnrep must be a power of two <= NREP");
  if (b.nrep < 1 || b.nrep > NREP || (b.nrep & (b.nrep - 1))) throw std::runtime_error("bn: nrep must be a power of two <= NREP");
  return b;
}

ConvArgs parse_conv(int mode, py::dict d);

void conv(int mode, int cfg, int G, int64_t stream, py::dict d) {
  ConvArgs a = parse_conv(mode, d);
  check(launch_conv(mode, a, G, cfg, S(stream)), "conv");
}

// (workspace floats, tickets) an LDS-staged conv config needs for these arguments; raises if invalid
py::tuple conv_workspace(int mode, int cfg, int G, py::dict d) {
  ConvArgs a = parse_conv(mode, d);
  int64_t ws = 0, nt = 0;
  int rc = 0;
  cfg &= ~CONV_XCD;
  if (cfg >= CONV_DEEP_CFG0 && cfg < CONV_DEEP_CFG0 + CONV_DEEP_NCFG) rc = 0;
  else if (cfg >= CONV_LDS_CFG0) rc = conv_lds_workspace(mode, a, G, cfg, ws, nt);
  return py::make_tuple(rc, ws, nt);
}

ConvArgs parse_conv(int mode, py::dict d) {
  ConvArgs a{};
  a.src = parse_src(d["src"].cast<py::dict>());
  a.w = P<const bf16_t>(d, "w");
  a.wgs = I(d, "wgs");
  a.bias = P<const float>(d, "bias");
  a.bgs = I(d, "bgs");
  a.out = P<void>(d, "out");
  a.ogs = I(d, "ogs");
  a.ldo = (int)I(d, "ldo");
  a.stats = P<double>(d, "stats");
  a.stats_nrep = (int)I(d, "stats_nrep", NREP);
  if (a.stats_nrep < 1 || a.stats_nrep > NREP) throw std::runtime_error("conv: bad stats_nrep");
  a.B = (int)I(d, "B"); a.Hs = (int)I(d, "Hs"); a.Ws = (int)I(d, "Ws"); a.Ho = (int)I(d, "Ho"); a.Wo = (int)I(d, "Wo");
  a.N = (int)I(d, "N"); a.Npad = (int)I(d, "Npad"); a.Cs = (int)I(d, "Cs");
  a.KH = (int)I(d, "KH"); a.KW = (int)I(d, "KW"); a.sh = (int)I(d, "sh"); a.sw = (int)I(d, "sw");
  a.ph = (int)I(d, "ph"); a.pw = (int)I(d, "pw"); a.Kpad = (int)I(d, "Kpad");
  if (a.Cs % 8 || a.N % 4 || a.Kpad % 32 || a.src.C0 + a.src.C1 != a.Cs) throw std::runtime_error("conv: bad geometry");
  if (d.contains("bnb") && !d["bnb"].is_none()) {  // fused BN-backward statistics (dgrad epilogue)
    py::dict b = d["bnb"].cast<py::dict>();
    a.by = P<const bf16_t>(b, "y"); a.bygs = I(b, "ygs"); a.ldby = (int)I(b, "ldy");
    a.bbn = parse_bn(b["bn"].cast<py::dict>());
    a.bpart = P<double>(b, "part");
    a.bkind = (int)I(b, "kind");
    a.bN = (int)I(b, "C", a.N);
    a.bpgs = I(b, "pgs", -1);
    if (a.bkind == ADD_RELU) {
      a.br = P<const bf16_t>(b, "r"); a.brgs = I(b, "rgs"); a.ldbr = (int)I(b, "ldr");
      if (b.contains("bn2") && !b["bn2"].is_none()) { a.bbn2 = parse_bn(b["bn2"].cast<py::dict>()); a.br_bn = 1; }
    }
    if (mode != MODE_DGRAD || !a.bpart || !a.by || !a.bbn.stats || !a.bbn.training || a.bbn.C != a.bN ||
        a.bN > a.N || a.bN % 8 || a.ldby % 4 || (a.bkind > ACT_SIGMOID && a.bkind != ADD_RELU) || a.bkind < ACT_NONE ||
        (a.bkind == ADD_RELU && (!a.br || a.ldbr % 4 || (a.br_bn && (a.bbn2.C != a.bN || !a.bbn2.training)))) ||
        (a.bpgs == 0 && (a.bygs != 0 || a.brgs != 0)))
      throw std::runtime_error("conv: bad fused BN-backward statistics arguments");
  }
  if (d.contains("add") && !d["add"].is_none()) {  // extra gradient sources summed by the dgrad epilogue
    py::list l = d["add"].cast<py::list>();
    if (mode != MODE_DGRAD || l.size() > 3) throw std::runtime_error("conv: bad extra gradient sources");
    for (size_t i = 0; i < l.size(); ++i) {
      py::dict e = l[i].cast<py::dict>();
      a.add[i] = P<const bf16_t>(e, "p");
      a.addgs[i] = I(e, "gs");
      a.ldadd[i] = (int)I(e, "ld");
      // the epilogue reads 4 channels (8 bytes) per load
      if (!a.add[i] || a.ldadd[i] % 4 || a.ldadd[i] < a.N || (reinterpret_cast<uintptr_t>(a.add[i]) & 7) || a.addgs[i] % 4)
        throw std::runtime_error("conv: bad extra gradient source");
    }
    a.nadd = (int)l.size();
  }
  if (d.contains("nol") && !d["nol"].is_none()) {  // normalise-on-load of the input (forward)
    py::dict n = d["nol"].cast<py::dict>();
    a.nbn = parse_bn(n["bn"].cast<py::dict>());
    a.nol = 1;
    a.nol_kind = (int)I(n, "kind");
    if (mode != MODE_FWD || a.src.C1 != 0 || a.nbn.C != a.Cs ||
        (a.nol_kind != ACT_NONE && a.nol_kind != ACT_RELU) || (a.nbn.training && !a.nbn.stats))
      throw std::runtime_error("conv: bad normalise-on-load arguments");
  }
  a.ws = P<float>(d, "ws");
  a.cnt = P<unsigned>(d, "cnt");
  a.ptm = P<uint64_t>(d, "ptm");
  return a;
}

WgradArgs parse_wgrad(const py::dict& d);

void wgrad(int cfg, int G, int64_t stream, py::dict d) {
  check(launch_wgrad(parse_wgrad(d), G, cfg, S(stream)), "wgrad");
}

// Packs the WgradJob table of a batched weight-gradient launch; returns (bytes, total blocks).
py::tuple wgrad_table(int cfg, py::list dicts, py::list groups) {
  std::vector<WgradJob> jobs(dicts.size());
  int64_t b0 = 0;
  for (size_t i = 0; i < jobs.size(); ++i) {
    WgradJob& j = jobs[i];
    j = WgradJob{};
    j.a = parse_wgrad(dicts[i].cast<py::dict>());
    j.G = groups[i].cast<int>();
    j.ntiles = wgrad_ntiles(cfg, j.a);
    if (j.ntiles < 0) throw std::runtime_error("wgrad_table: cfg " + std::to_string(cfg) + " invalid for job " + std::to_string(i));
    j.block0 = b0;
    b0 += (int64_t)j.ntiles * j.a.splits * j.G;
  }
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(jobs.data()), jobs.size() * sizeof(WgradJob)), b0);
}

void wgrad_batched(int cfg, int64_t table, int nj, int64_t nblocks, int64_t stream, int64_t cap) {
  check(launch_wgrad_batched(cfg, reinterpret_cast<const WgradJob*>(static_cast<intptr_t>(table)), nj, nblocks,
                             S(stream), cap), "wgrad_batched");
}

WgradArgs parse_wgrad(const py::dict& d) {
  WgradArgs a{};
  a.src = parse_src(d["src"].cast<py::dict>());
  a.dy = P<const bf16_t>(d, "dy");
  a.dgs = I(d, "dgs");
  a.ldd = (int)I(d, "ldd");
  a.slab = P<float>(d, "slab");
  a.splits = (int)I(d, "splits"); a.m_per_split = (int)I(d, "m_per_split");
  a.B = (int)I(d, "B"); a.Hi = (int)I(d, "Hi"); a.Wi = (int)I(d, "Wi"); a.Ho = (int)I(d, "Ho"); a.Wo = (int)I(d, "Wo");
  a.Co = (int)I(d, "Co"); a.Npad = (int)I(d, "Npad"); a.Cs = (int)I(d, "Cs");
  a.KH = (int)I(d, "KH"); a.KW = (int)I(d, "KW"); a.sh = (int)I(d, "sh"); a.sw = (int)I(d, "sw");
  a.ph = (int)I(d, "ph"); a.pw = (int)I(d, "pw"); a.Kpad = (int)I(d, "Kpad");
  if (a.Cs % 8 || a.Co % 8 || a.Kpad % 64) throw std::runtime_error("wgrad: bad geometry");
  if (d.contains("nol") && !d["nol"].is_none()) {
    py::dict n = d["nol"].cast<py::dict>();
    a.nol_consts = P<const float>(n, "consts");
    a.nol = 1;
    a.nol_kind = (int)I(n, "kind");
    if (!a.nol_consts || a.src.C1 != 0 || (a.nol_kind != ACT_NONE && a.nol_kind != ACT_RELU))
      throw std::runtime_error("wgrad: bad normalise-on-load arguments");
  }
  return a;
}

void wgrad_finalize(int64_t descs, int nd, int64_t nblocks, double scale, int64_t stream) {
  check(launch_wgrad_finalize(reinterpret_cast<const WgFinDesc*>(static_cast<intptr_t>(descs)), nd, nblocks,
                              (float)scale, S(stream)), "wgrad_finalize");
}

TailArgs parse_tail(const py::dict& d) {
  TailArgs a{};
  a.y = P<const bf16_t>(d, "y"); a.ygs = I(d, "ygs"); a.ldy = (int)I(d, "ldy");
  a.bn = parse_bn(d["bn"].cast<py::dict>());
  a.r = P<const bf16_t>(d, "r"); a.rgs = I(d, "rgs"); a.ldr = (int)I(d, "ldr");
  if (d.contains("bn2") && !d["bn2"].is_none()) { a.bn2 = parse_bn(d["bn2"].cast<py::dict>()); a.r_bn = 1; }
  a.out = P<bf16_t>(d, "out"); a.ogs = I(d, "ogs"); a.ldo = (int)I(d, "ldo");
  a.B = (int)I(d, "B"); a.H = (int)I(d, "H"); a.W = (int)I(d, "W"); a.C = (int)I(d, "C");
  if (d.contains("g")) a.g = parse_grads(d["g"].cast<py::list>());
  a.part = P<double>(d, "part"); a.chunk_px = (int)I(d, "chunk_px");
  a.dzbuf = P<bf16_t>(d, "dzbuf"); a.dzgs = I(d, "dzgs"); a.lddz = (int)I(d, "lddz");
  a.side = P<bf16_t>(d, "side"); a.sgs = I(d, "sgs"); a.lds = (int)I(d, "lds");
  a.dy = P<bf16_t>(d, "dy"); a.dgs = I(d, "dgs"); a.ldd = (int)I(d, "ldd");
  a.dy2 = P<bf16_t>(d, "dy2"); a.d2gs = I(d, "d2gs"); a.ldd2 = (int)I(d, "ldd2");
  a.dgamma = P<float>(d, "dgamma"); a.dbeta = P<float>(d, "dbeta");
  a.dgamma2 = P<float>(d, "dgamma2"); a.dbeta2 = P<float>(d, "dbeta2");
  a.pgs = I(d, "pgs");
  a.gscale = (float)F(d, "gscale", 1.0);
  a.tsc = P<uint64_t>(d, "tsc");
  a.ptm = P<uint64_t>(d, "ptm");
  if (a.C % 8 || a.C > 2048) throw std::runtime_error("tail: C must be a multiple of 8 and <= 2048");
  return a;
}

void tail_fwd(int kind, int G, int blocks, int64_t stream, py::dict d) {
  check(launch_tail_fwd(kind, parse_tail(d), G, blocks, S(stream)), "tail_fwd");
}

// Packs the TailJob table of a batched tail launch; returns (bytes, total blocks, largest C).  ``bwd``: backward
// tails (residual-free ACT_RELU tails; the gradient sources, replica sums and outputs of parse_tail).
py::tuple tail_table(py::list dicts, py::list blocks, bool bwd) {
  std::vector<TailJob> jobs(dicts.size());
  int64_t b0 = 0;
  int maxC = 0;
  for (size_t i = 0; i < jobs.size(); ++i) {
    TailJob& j = jobs[i];
    j = TailJob{};
    j.a = parse_tail(dicts[i].cast<py::dict>());
    j.blocks = blocks[i].cast<int>();
    if (j.blocks <= 0 || j.a.C % 8 || j.a.r || j.a.r_bn) throw std::runtime_error("tail_table: unsupported tail");
    // (gscale != 1: SyncBN's batched apply writes d(gamma), d(beta) / world -- bnb_apply_impl reads it)
    if (bwd && (!j.a.part || j.a.chunk_px <= 0 || j.a.side || !(j.a.gscale > 0.f)))
      throw std::runtime_error("tail_table: unsupported backward tail");
    j.block0 = (int)b0;
    b0 += j.blocks;
    maxC = std::max(maxC, j.a.C);
  }
  if (b0 >= (1ll << 31)) throw std::runtime_error("tail_table: too many blocks");
  return py::make_tuple(py::bytes(reinterpret_cast<const char*>(jobs.data()), jobs.size() * sizeof(TailJob)), b0, maxC);
}

void tail_bwd_batched(int kind, int cgb, int reduce, int64_t table, int nj, int64_t nblocks, int64_t stream) {
  check(launch_tail_bwd_batched(kind, cgb, reduce, reinterpret_cast<const TailJob*>(static_cast<intptr_t>(table)), nj,
                                (int)nblocks, S(stream)), "tail_bwd_batched");
}

void tail_fwd_batched(int kind, int64_t table, int nj, int64_t nblocks, int maxC, int64_t stream) {
  check(launch_tail_fwd_batched(kind, reinterpret_cast<const TailJob*>(static_cast<intptr_t>(table)), nj, (int)nblocks,
                                maxC, S(stream)), "tail_fwd_batched");
}
void tail_bwd(int kind, int G, int blocks, int64_t stream, py::dict d) {
  check(launch_tail_bwd(kind, parse_tail(d), G, blocks, (int)I(d, "fused", 0), S(stream)), "tail_bwd");
}

void mtl_head(int64_t stream, py::dict d) {
  HeadArgs a{};
  a.feat = P<const bf16_t>(d, "feat"); a.fgs = I(d, "fgs"); a.ldf = (int)I(d, "ldf");
  a.labels = P<const int64_t>(d, "labels"); a.lab_stride = (int)I(d, "lab_stride"); a.lab_off = (int)I(d, "lab_off");
  a.T = (int)I(d, "T"); a.B = (int)I(d, "B"); a.HW = (int)I(d, "HW"); a.C = (int)I(d, "C");
  py::list ncls = d["ncls"].cast<py::list>(), w = d["w"].cast<py::list>();
  if (a.T > 4 || (int)ncls.size() != a.T || (int)w.size() != a.T) throw std::runtime_error("mtl_head: bad task list");
  for (int t = 0; t < a.T; ++t) { a.ncls[t] = ncls[t].cast<int>(); a.w[t] = w[t].cast<float>(); if (a.ncls[t] > 16) throw std::runtime_error("ncls > 16"); }
  a.logp = P<float>(d, "logp"); a.dfeat = P<bf16_t>(d, "dfeat"); a.dgs = I(d, "dgs");
  a.metrics = P<float>(d, "metrics"); a.confusion = P<int>(d, "confusion");
  a.nvalid = P<const int64_t>(d, "nvalid");
  check(launch_mtl_head(a, S(stream)), "mtl_head");
}

void cls_head(int64_t stream, py::dict d) {
  ClsArgs a{};
  a.x = P<const bf16_t>(d, "x"); a.ldx = (int)I(d, "ldx");
  a.W = P<const float>(d, "W"); a.bias = P<const float>(d, "bias");
  a.labels = P<const int64_t>(d, "labels");
  a.B = (int)I(d, "B"); a.HW = (int)I(d, "HW"); a.C = (int)I(d, "C"); a.N = (int)I(d, "N");
  a.p_drop = (float)F(d, "p_drop");
  a.seed = P<const int64_t>(d, "seed");
  a.feat = P<float>(d, "feat"); a.logits = P<float>(d, "logits"); a.dlogits = P<float>(d, "dlogits");
  a.dx = P<bf16_t>(d, "dx"); a.metrics = P<float>(d, "metrics"); a.confusion = P<int>(d, "confusion");
  a.dW = P<float>(d, "dW"); a.db = P<float>(d, "db");
  a.nvalid = P<const int64_t>(d, "nvalid");
  check(launch_cls_head(a, P<int64_t>(d, "seed"), S(stream)), "cls_head");
}

void gather_batch(int64_t X, int64_t idx, int64_t lab, int lab_w, int64_t out, int64_t lab_out, int B, int Cin, int H,
                  int W, int64_t stream, int taps, int off, py::list zero, int64_t cursor, int nrows) {
  if (cursor && nrows <= 0) throw std::runtime_error("gather_batch: a schedule cursor needs its row count");
  ZeroRanges z{};
  if (zero.size() > 4) throw std::runtime_error("gather_batch: at most 4 zero ranges");
  for (size_t i = 0; i < zero.size(); ++i) {
    auto t = zero[i].cast<py::tuple>();
    const int64_t ptr = t[0].cast<int64_t>(), bytes = t[1].cast<int64_t>();
    if (ptr % 16 || bytes % 16 || bytes < 0) throw std::runtime_error("gather_batch: zero range not 16-byte aligned");
    z.p[i] = reinterpret_cast<uint4*>(static_cast<intptr_t>(ptr));
    z.n16[i] = bytes / 16;
  }
  z.n = (int)zero.size();
  check(launch_gather_batch(reinterpret_cast<const float*>(X), reinterpret_cast<const int64_t*>(idx),
                            reinterpret_cast<const int64_t*>(lab), lab_w, reinterpret_cast<bf16_t*>(out),
                            reinterpret_cast<int64_t*>(lab_out), B, Cin, H, W, taps, off, z,
                            reinterpret_cast<const int64_t*>(static_cast<intptr_t>(cursor)), nrows, S(stream)),
        "gather_batch");
}

void pool3(int is_max, int backward, int64_t stream, py::dict d) {
  PoolArgs a{};
  a.x = P<const bf16_t>(d, "x"); a.ldx = (int)I(d, "ldx");
  a.y = P<bf16_t>(d, "y"); a.ldy = (int)I(d, "ldy");
  if (d.contains("g")) {
    // a list of (ptr, group stride, pitch) sources, or one pointer with pitch "ldg"
    if (py::isinstance<py::list>(d["g"])) a.g = parse_grads(d["g"].cast<py::list>());
    else { a.g.n = 1; a.g.p[0] = P<const bf16_t>(d, "g"); a.g.ld[0] = (int)I(d, "ldg"); }
  }
  a.dx = P<bf16_t>(d, "dx"); a.lddx = (int)I(d, "lddx");
  a.B = (int)I(d, "B"); a.H = (int)I(d, "H"); a.W = (int)I(d, "W"); a.C = (int)I(d, "C");
  a.Ho = (int)I(d, "Ho"); a.Wo = (int)I(d, "Wo");
  a.am = P<uint8_t>(d, "am");
  if (a.C % 8) throw std::runtime_error("pool3: C % 8");
  if (a.am && !is_max) throw std::runtime_error("pool3: argmax only for max pooling");
  check(launch_pool3(is_max, backward, a, S(stream)), "pool3");
}

void synth_das(int64_t stream, py::dict d) {
  SynthArgs a{};
  a.params = P<const float>(d, "params"); a.out = P<float>(d, "out");
  a.C = (int)I(d, "C"); a.H = (int)I(d, "H"); a.W = (int)I(d, "W");
  a.noise = (int)I(d, "noise", 1);
  a.key = (uint64_t)I(d, "key"); a.sample0 = I(d, "sample0", 0);
  check(launch_synth_das(a, (int)I(d, "n"), S(stream)), "synth_das");
}

void grad_sum(py::list g, int64_t out, int ldo, int64_t M, int C, int64_t stream) {
  check(launch_grad_sum(parse_grads(g), reinterpret_cast<bf16_t*>(out), ldo, M, C, S(stream)), "grad_sum");
}

void adam_pack(int64_t stream, py::dict d) {
  AdamArgs a{};
  a.p = P<float>(d, "p"); a.g = P<const float>(d, "g"); a.m = P<float>(d, "m"); a.v = P<float>(d, "v");
  a.n = I(d, "n");
  if (a.n % 4) throw std::runtime_error("adam: flat length must be a multiple of 4");
  a.lr = P<const float>(d, "lr"); a.step = P<const float>(d, "step");
  a.b1 = (float)F(d, "b1", 0.9); a.b2 = (float)F(d, "b2", 0.999); a.eps = (float)F(d, "eps", 1e-8);
  a.wd = (float)F(d, "wd", 0.0); a.grad_scale = (float)F(d, "grad_scale", 1.0);
  a.update = (int)I(d, "update", 1);
  a.inc_step = (int)I(d, "inc_step", 1);
  a.t_pre = (int)I(d, "t_pre", 0);
  if (a.t_pre && a.inc_step && a.update) throw std::runtime_error("adam: t_pre with inc_step would advance the step twice");
  a.cursor = P<int64_t>(d, "cursor");
  check(launch_adam_pack(a, P<const OptSeg>(d, "segs"), (int)I(d, "nsegs"), I(d, "nblocks"), S(stream)), "adam_pack");
}

void step_inc(int64_t step, int64_t cursor, int64_t stream) {
  if (!step) throw std::runtime_error("step_inc: null step counter");
  check(launch_step_inc(reinterpret_cast<float*>(step), reinterpret_cast<int64_t*>(cursor), S(stream)), "step_inc");
}

}  // namespace

namespace mda {
void register_matio(py::module& m);  // matio.cpp: native MAT-file batch loader
}

PYBIND11_MODULE(_mda_hip, m) {
  m.doc() = "gfx950 HIP kernels of mtl_das_pytorch_amd";
  m.attr("NREP") = NREP;
  m.attr("SIZEOF_WGFIN") = (int)sizeof(WgFinDesc);
  m.attr("FIN_EPT") = FIN_EPT;
  m.attr("SIZEOF_OPTSEG") = (int)sizeof(OptSeg);
  m.def("conv", &conv);
  m.def("conv_workspace", &conv_workspace);
  m.attr("CONV_LDS_CFG0") = CONV_LDS_CFG0;
  m.attr("CONV_XCD") = CONV_XCD;
  m.attr("CONV_LDS_NCFG") = CONV_LDS_NCFG;
  m.attr("CONV_DEEP_CFG0") = CONV_DEEP_CFG0;
  m.attr("CONV_DEEP_NCFG") = CONV_DEEP_NCFG;
  m.attr("CONV_GLDS_CFG0") = CONV_GLDS_CFG0;
  m.attr("CONV_GLDS_NCFG") = CONV_GLDS_NCFG;
  m.attr("CONV_PATCH_CFG0") = CONV_PATCH_CFG0;
  m.attr("CONV_PATCH_NCFG") = CONV_PATCH_NCFG;
  m.attr("CONV_GDEEP_CFG0") = CONV_GDEEP_CFG0;
  m.attr("CONV_GDEEP_NCFG") = CONV_GDEEP_NCFG;
  m.attr("CONV_PATCHP_CFG0") = CONV_PATCHP_CFG0;
  m.attr("CONV_PATCHP_NCFG") = CONV_PATCHP_NCFG;
  m.def("wgrad", &wgrad);
  m.def("wgrad_finalize", &wgrad_finalize);
  m.def("tail_fwd", &tail_fwd);
  m.def("tail_table", &tail_table, py::arg("dicts"), py::arg("blocks"), py::arg("bwd") = false);
  m.def("tail_bwd_batched", &tail_bwd_batched);
  m.def("tail_fwd_batched", &tail_fwd_batched);
  m.def("tail_bwd", &tail_bwd);
  m.def("mtl_head", &mtl_head);
  m.def("cls_head", &cls_head);
  m.def("gather_batch", &gather_batch, py::arg("X"), py::arg("idx"), py::arg("lab"), py::arg("lab_w"), py::arg("out"),
        py::arg("lab_out"), py::arg("B"), py::arg("Cin"), py::arg("H"), py::arg("W"), py::arg("stream"),
        py::arg("taps") = 0, py::arg("off") = 0, py::arg("zero") = py::list(), py::arg("cursor") = 0,
        py::arg("nrows") = 0);
  m.def("pool3", &pool3);
  m.def("wgrad_table", &wgrad_table);
  m.def("wgrad_batched", &wgrad_batched, py::arg("cfg"), py::arg("table"), py::arg("nj"), py::arg("nblocks"),
        py::arg("stream"), py::arg("cap") = 0);
  m.def("grad_sum", &grad_sum);
  m.def("synth_das", &synth_das);
  m.def("philox_kat", [](int64_t ctr, uint64_t key, int64_t out, int n, int64_t stream) {
    check(launch_philox_kat(reinterpret_cast<const uint32_t*>(static_cast<intptr_t>(ctr)), key,
                            reinterpret_cast<uint32_t*>(static_cast<intptr_t>(out)), n, S(stream)), "philox_kat");
  });
  m.def("tick", [](int64_t buf, int i, int64_t stream, int64_t n, int64_t q) {
    if (i < 0 || i >= n) throw std::runtime_error("tick: index outside the stamp buffer");
    check(launch_tick(reinterpret_cast<uint64_t*>(static_cast<intptr_t>(buf)),
                      reinterpret_cast<uint64_t*>(static_cast<intptr_t>(q)), i, S(stream)), "tick");
  }, py::arg("buf"), py::arg("i"), py::arg("stream"), py::arg("n"), py::arg("q") = 0);
  m.def("adam_pack", &adam_pack);
  m.def("step_inc", &step_inc);
  m.def("hip_device_sync", []() { return (int)hipDeviceSynchronize(); });
  // engine-owned streams (engine/program.py EngineStreams): created once per device, never drawn from
  // torch's round-robin stream pool, so they cannot alias a capture stream or each other
  m.def("stream_create", [](int priority) {
    hipStream_t s = nullptr;
    check((int)hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority), "hipStreamCreateWithPriority");
    return static_cast<int64_t>(reinterpret_cast<intptr_t>(s));
  });
  m.def("stream_destroy", [](int64_t s) { check((int)hipStreamDestroy(S(s)), "hipStreamDestroy"); });
  // events recorded as EXTERNAL event-record nodes when the stream is capturing (hipEventRecordExternal):
  // the host orders work issued after a graph launch behind a point inside the graph (engine/step.py, the
  // world > 1 data-parallel step; torch.cuda.Event(external=True) is refused on ROCm builds of PyTorch)
  m.def("event_create", []() {
    hipEvent_t e = nullptr;
    check((int)hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreateWithFlags");
    return static_cast<int64_t>(reinterpret_cast<intptr_t>(e));
  });
  m.def("event_destroy", [](int64_t e) {
    check((int)hipEventDestroy(reinterpret_cast<hipEvent_t>(static_cast<intptr_t>(e))), "hipEventDestroy");
  });
  m.def("event_record_external", [](int64_t e, int64_t stream) {
    hipEvent_t ev = reinterpret_cast<hipEvent_t>(static_cast<intptr_t>(e));
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    hipGraph_t g = nullptr;
    const hipGraphNode_t* deps = nullptr;
    size_t nd = 0;
    check((int)hipStreamGetCaptureInfo_v2(S(stream), &st, nullptr, &g, &deps, &nd), "hipStreamGetCaptureInfo_v2");
    if (st != hipStreamCaptureStatusActive) {
      check((int)hipEventRecord(ev, S(stream)), "hipEventRecord");
      return;
    }
    // capturing: an explicit event-record node after the stream's current tail, which becomes the new tail
    hipGraphNode_t node = nullptr;
    check((int)hipGraphAddEventRecordNode(&node, g, deps, nd, ev), "hipGraphAddEventRecordNode");
    check((int)hipStreamUpdateCaptureDependencies(S(stream), &node, 1, hipStreamSetCaptureDependencies),
          "hipStreamUpdateCaptureDependencies");
  });
  m.def("stream_wait_event", [](int64_t stream, int64_t e) {
    check((int)hipStreamWaitEvent(S(stream), reinterpret_cast<hipEvent_t>(static_cast<intptr_t>(e)), 0),
          "hipStreamWaitEvent");
  });
  m.def("stream_priority_range", []() {
    int least = 0, greatest = 0;
    check((int)hipDeviceGetStreamPriorityRange(&least, &greatest), "hipDeviceGetStreamPriorityRange");
    return py::make_tuple(least, greatest);
  });
  register_matio(m);
}
