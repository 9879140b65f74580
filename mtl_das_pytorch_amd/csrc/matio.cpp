// Native MAT-file (Level 5) reader and multi-threaded batch loader for the disk-streaming dataset.
//
// The reference streams its .mat files through torch's DataLoader: scipy.io.loadmat per sample, a
// Python-side float32 cast and collate (dataset_preparation.py:300-344, utils.py:148-156).  Here one call
// loads a whole batch: worker threads of a persistent pool parse the files (uncompressed or zlib
// miCOMPRESSED elements), convert MATLAB's column-major real part of any numeric class to row-major
// float32 and write it straight into the caller's (pinned) staging buffer -- no Python objects per sample,
// and the GIL is released for the whole batch, so the next batch loads while the GPU trains on this one.
//
// Supported: Level-5 MAT files (MATLAB v5/v6/v7, what scipy.io.savemat writes), little- or big-endian,
// real numeric arrays.  Not supported (status != 0, the Python side falls back to scipy for that file):
// v7.3 (HDF5) files, complex / sparse / cell / struct variables.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <sys/stat.h>
#include <zlib.h>

#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace py = pybind11;

namespace mda {
namespace {

enum : uint32_t {
  miINT8 = 1, miUINT8 = 2, miINT16 = 3, miUINT16 = 4, miINT32 = 5, miUINT32 = 6, miSINGLE = 7,
  miDOUBLE = 9, miINT64 = 12, miUINT64 = 13, miMATRIX = 14, miCOMPRESSED = 15
};
constexpr uint32_t mxFLAG_COMPLEX = 0x800;

enum Status : int {
  kOk = 0, kIoError = 1, kNotMat5 = 2, kNoVariable = 3, kUnsupported = 4, kShapeMismatch = 5, kCorrupt = 6
};

struct Cursor {
  const uint8_t* p;
  const uint8_t* end;
  bool swap;
  size_t left() const { return (size_t)(end - p); }
};

inline uint32_t bswap32(uint32_t v) { return __builtin_bswap32(v); }

inline uint32_t rd32(const uint8_t* p, bool swap) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return swap ? bswap32(v) : v;
}

// Element tag: full (8 bytes: type, nbytes) or small (4 bytes: nbytes<<16 | type, data in the next 4).
struct Elem {
  uint32_t type;
  uint32_t nbytes;
  const uint8_t* data;
};

bool next_elem(Cursor& c, Elem& e) {
  if (c.left() < 8) return false;
  const uint32_t w0 = rd32(c.p, c.swap);
  if (w0 >> 16) {  // small data element
    e.type = w0 & 0xFFFF;
    e.nbytes = w0 >> 16;
    e.data = c.p + 4;
    if (e.nbytes > 4) return false;
    c.p += 8;
    return true;
  }
  e.type = w0;
  e.nbytes = rd32(c.p + 4, c.swap);
  e.data = c.p + 8;
  if ((size_t)e.nbytes > c.left() - 8) return false;
  // every non-compressed element's data is padded to a multiple of 8 bytes
  size_t adv = 8 + (size_t)e.nbytes;
  if (e.type != miCOMPRESSED) adv = (adv + 7) & ~(size_t)7;
  c.p += adv > c.left() ? c.left() : adv;
  return true;
}

size_t type_size(uint32_t t) {
  switch (t) {
    case miINT8: case miUINT8: return 1;
    case miINT16: case miUINT16: return 2;
    case miINT32: case miUINT32: case miSINGLE: return 4;
    case miDOUBLE: case miINT64: case miUINT64: return 8;
    default: return 0;
  }
}

template <typename T>
inline T load_swapped(const uint8_t* p, bool swap) {
  T v;
  if (!swap) {
    std::memcpy(&v, p, sizeof(T));
    return v;
  }
  uint8_t b[sizeof(T)];
  for (size_t i = 0; i < sizeof(T); ++i) b[i] = p[sizeof(T) - 1 - i];
  std::memcpy(&v, b, sizeof(T));
  return v;
}

float elem_value(const uint8_t* p, uint32_t type, bool swap) {
  switch (type) {
    case miINT8: return (float)*(const int8_t*)p;
    case miUINT8: return (float)*p;
    case miINT16: return (float)load_swapped<int16_t>(p, swap);
    case miUINT16: return (float)load_swapped<uint16_t>(p, swap);
    case miINT32: return (float)load_swapped<int32_t>(p, swap);
    case miUINT32: return (float)load_swapped<uint32_t>(p, swap);
    case miSINGLE: return load_swapped<float>(p, swap);
    case miDOUBLE: return (float)load_swapped<double>(p, swap);
    case miINT64: return (float)load_swapped<int64_t>(p, swap);
    case miUINT64: return (float)load_swapped<uint64_t>(p, swap);
    default: return 0.f;
  }
}

// Parse one miMATRIX element; if its name is `want`, write its real part row-major into `out`
// (numel must equal `expect` when expect > 0, and the MATLAB dims must equal `want_dims` when given: a
// 250 x 100 variable has the numel of a 100 x 250 slot but would land in it transposed).  Returns kOk,
// kNoVariable (other name) or an error.
int parse_matrix(const uint8_t* data, size_t nbytes, bool swap, const std::string& want, float* out,
                 int64_t expect, std::vector<int64_t>* shape, const std::vector<int64_t>* want_dims) {
  Cursor c{data, data + nbytes, swap};
  Elem flags, dims, name, real;
  if (!next_elem(c, flags) || flags.type != miUINT32 || flags.nbytes < 8) return kCorrupt;
  if (!next_elem(c, dims) || dims.type != miINT32) return kCorrupt;
  if (!next_elem(c, name) || name.type != miINT8) return kCorrupt;
  const std::string nm(reinterpret_cast<const char*>(name.data), name.nbytes);
  if (nm != want) return kNoVariable;
  const uint32_t f0 = rd32(flags.data, swap);
  const uint32_t cls = f0 & 0xFF;
  if ((f0 & mxFLAG_COMPLEX) || cls < 6 || cls > 15) return kUnsupported;  // numeric classes are 6..15
  const int nd = (int)(dims.nbytes / 4);
  std::vector<int64_t> d(nd);
  int64_t numel = 1;
  for (int i = 0; i < nd; ++i) {
    d[i] = (int32_t)rd32(dims.data + 4 * i, swap);
    if (d[i] < 0) return kCorrupt;
    numel *= d[i];
  }
  if (shape) *shape = d;
  if (expect > 0 && numel != expect) return kShapeMismatch;
  if (want_dims && !want_dims->empty() && d != *want_dims) return kShapeMismatch;
  if (!out) return kOk;
  if (!next_elem(c, real)) return kCorrupt;
  const size_t es = type_size(real.type);
  if (!es || (int64_t)(real.nbytes / es) != numel) return kCorrupt;
  // column-major (dims d0..dk-1, d0 fastest) -> row-major (last dim fastest): out index over reversed
  // iteration.  2-D fast path: out[r][c] = in[c * rows + r].
  if (nd == 2) {
    const int64_t R = d[0], Cc = d[1];
    for (int64_t r = 0; r < R; ++r)
      for (int64_t col = 0; col < Cc; ++col)
        out[r * Cc + col] = elem_value(real.data + (size_t)(col * R + r) * es, real.type, swap);
    return kOk;
  }
  std::vector<int64_t> idx(nd, 0), cstride(nd, 1);
  for (int i = 1; i < nd; ++i) cstride[i] = cstride[i - 1] * d[i - 1];
  for (int64_t o = 0; o < numel; ++o) {  // o walks row-major; idx holds its multi-index
    int64_t src = 0;
    for (int i = 0; i < nd; ++i) src += idx[i] * cstride[i];
    out[o] = elem_value(real.data + (size_t)src * es, real.type, swap);
    for (int i = nd - 1; i >= 0; --i) {
      if (++idx[i] < d[i]) break;
      idx[i] = 0;
    }
  }
  return kOk;
}

// `cap`: the largest inflated size accepted (a corrupt or hostile stream cannot make the worker allocate
// without bound).
int inflate_all(const uint8_t* src, size_t n, std::vector<uint8_t>& dst, size_t cap) {
  z_stream zs{};
  if (inflateInit(&zs) != Z_OK) return kCorrupt;
  dst.resize(std::min(cap, n * 4 + 4096));
  zs.next_in = const_cast<Bytef*>(src);
  zs.avail_in = (uInt)n;
  size_t have = 0;
  int rc;
  do {
    if (have == dst.size()) {
      if (dst.size() >= cap) { inflateEnd(&zs); return kCorrupt; }
      dst.resize(std::min(cap, dst.size() * 2));
    }
    zs.next_out = dst.data() + have;
    zs.avail_out = (uInt)(dst.size() - have);
    rc = inflate(&zs, Z_NO_FLUSH);
    have = dst.size() - zs.avail_out;
  } while (rc == Z_OK);
  inflateEnd(&zs);
  if (rc != Z_STREAM_END) return kCorrupt;
  dst.resize(have);
  return kOk;
}

int read_file(const std::string& path, std::vector<uint8_t>& buf) {
  struct stat sb;
  if (::stat(path.c_str(), &sb) != 0 || !S_ISREG(sb.st_mode)) return kIoError;  // directories, devices, fifos
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return kIoError;
  std::fseek(f, 0, SEEK_END);
  const long n = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  if (n < 0) { std::fclose(f); return kIoError; }
  buf.resize((size_t)n);
  const size_t got = n ? std::fread(buf.data(), 1, (size_t)n, f) : 0;
  std::fclose(f);
  return got == (size_t)n ? kOk : kIoError;
}

// Load variable `var` of a Level-5 MAT file as row-major float32.
int load_mat5(const std::string& path, const std::string& var, float* out, int64_t expect,
              std::vector<int64_t>* shape, const std::vector<int64_t>* want_dims = nullptr) {
  std::vector<uint8_t> buf;
  int rc = read_file(path, buf);
  if (rc) return rc;
  if (buf.size() < 128) return kNotMat5;
  const uint16_t ver = (uint16_t)(buf[124] | (buf[125] << 8));
  bool swap;
  if (buf[126] == 'I' && buf[127] == 'M') swap = false;
  else if (buf[126] == 'M' && buf[127] == 'I') swap = true;
  else return kNotMat5;
  if ((swap ? (uint16_t)((ver >> 8) | (ver << 8)) : ver) != 0x0100) return kNotMat5;  // 0x0200 = v7.3/HDF5
  Cursor c{buf.data() + 128, buf.data() + buf.size(), swap};
  Elem e;
  std::vector<uint8_t> inflated;
  while (next_elem(c, e)) {
    const uint8_t* md = e.data;
    size_t mn = e.nbytes;
    if (e.type == miCOMPRESSED) {
      // the variable is at most expect 8-byte values plus its headers; unknown size: 1 GiB
      const size_t cap = expect > 0 ? (size_t)expect * 8 + (1u << 20) : ((size_t)1 << 30);
      if ((rc = inflate_all(e.data, e.nbytes, inflated, cap))) return rc;
      Cursor ic{inflated.data(), inflated.data() + inflated.size(), swap};
      Elem inner;
      if (!next_elem(ic, inner)) return kCorrupt;
      if (inner.type != miMATRIX) continue;
      md = inner.data;
      mn = inner.nbytes;
    } else if (e.type != miMATRIX) {
      continue;
    }
    rc = parse_matrix(md, mn, swap, var, out, expect, shape, want_dims);
    if (rc != kNoVariable) return rc;
  }
  return kNoVariable;
}

// A fixed pool of worker threads; run(n, fn) executes fn(0..n-1) across them and blocks until done.
class Pool {
 public:
  explicit Pool(int n) {
    for (int i = 0; i < n; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  void run(int64_t n, const std::function<void(int64_t)>& fn) {
    std::lock_guard<std::mutex> one_at_a_time(run_mu_);
    std::unique_lock<std::mutex> g(mu_);
    fn_ = &fn;
    next_.store(0);
    n_ = n;
    done_ = 0;
    ++gen_;
    cv_.notify_all();
    done_cv_.wait(g, [&] { return done_ == (int)th_.size(); });
    fn_ = nullptr;
  }
  int size() const { return (int)th_.size(); }

 private:
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      const std::function<void(int64_t)>* fn;
      int64_t n;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        fn = fn_;
        n = n_;
      }
      for (int64_t i; (i = next_.fetch_add(1)) < n;) (*fn)(i);
      {
        std::lock_guard<std::mutex> g(mu_);
        if (++done_ == (int)th_.size()) done_cv_.notify_all();
      }
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int64_t)>* fn_ = nullptr;
  std::atomic<int64_t> next_{0};
  int64_t n_ = 0;
  int done_ = 0;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

// Never lets an exception escape a worker thread (it would std::terminate the training process): a file
// the native reader cannot handle gets a status and falls back to scipy on the Python side.
int load_mat5_safe(const std::string& path, const std::string& var, float* out, int64_t expect,
                   const std::vector<int64_t>* want_dims) {
  try {
    return load_mat5(path, var, out, expect, nullptr, want_dims);
  } catch (const std::bad_alloc&) {
    return kCorrupt;
  } catch (...) {
    return kIoError;
  }
}

class MatBatchLoader {
 public:
  // dims: the MATLAB dimensions every file's variable must have (empty: numel only)
  MatBatchLoader(std::vector<std::string> paths, std::string var, std::vector<int64_t> dims, int threads)
      : paths_(std::move(paths)), var_(std::move(var)), dims_(std::move(dims)), pool_(threads > 0 ? threads : 1) {
    numel_ = 1;
    for (int64_t d : dims_) numel_ *= d;
  }

  // Load files idx[0..n) into out[i * numel ...] (float32, row-major).  Returns one status per file.
  std::vector<int> load(const std::vector<int64_t>& idx, int64_t out_ptr) {
    float* out = reinterpret_cast<float*>(static_cast<intptr_t>(out_ptr));
    std::vector<int> st(idx.size(), kOk);
    {
      py::gil_scoped_release nogil;
      pool_.run((int64_t)idx.size(), [&](int64_t i) {
        const int64_t f = idx[i];
        st[i] = (f < 0 || f >= (int64_t)paths_.size())
                    ? kIoError
                    : load_mat5_safe(paths_[f], var_, out + i * numel_, numel_, &dims_);
      });
    }
    return st;
  }
  int64_t size() const { return (int64_t)paths_.size(); }
  int threads() const { return pool_.size(); }

 private:
  std::vector<std::string> paths_;
  std::string var_;
  std::vector<int64_t> dims_;
  int64_t numel_ = 1;
  Pool pool_;
};

}  // namespace

void register_matio(py::module& m) {
  m.attr("MAT_OK") = (int)kOk;
  m.def("mat_shape", [](const std::string& path, const std::string& var) {
    std::vector<int64_t> shape;
    int rc;
    try {
      rc = load_mat5(path, var, nullptr, 0, &shape);
    } catch (...) {
      rc = kIoError;
    }
    return py::make_tuple(rc, shape);
  });
  m.def("mat_read", [](const std::string& path, const std::string& var, int64_t out_ptr, int64_t numel) {
    py::gil_scoped_release nogil;
    return load_mat5_safe(path, var, reinterpret_cast<float*>(static_cast<intptr_t>(out_ptr)), numel, nullptr);
  });
  py::class_<MatBatchLoader>(m, "MatBatchLoader")
      .def(py::init<std::vector<std::string>, std::string, std::vector<int64_t>, int>(), py::arg("paths"),
           py::arg("var"), py::arg("dims"), py::arg("threads"))
      .def("load", &MatBatchLoader::load)
      .def("__len__", &MatBatchLoader::size)
      .def_property_readonly("threads", &MatBatchLoader::threads);
}

}  // namespace mda
