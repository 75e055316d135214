// lhpc_io.cpp — on-disk CSR container and Matrix Market reader (SURVEY §8f
// rank 4: "fixture exchange and real matrices"; the reference has no file
// formats).  Host-only C++; the Matrix Market path ends in COO triples that
// lhpc_coo_to_csr (GPU) assembles.
//
// .lcsr layout (little-endian), every section 64-byte aligned:
//   [0,64)   header: char magic[8] = "LHPCCSR1", u32 version = 1, u32 dtype
//            (LHPC_F32/F64), i64 n_rows, i64 n_cols, i64 nnz, u32 row_ptr_bits
//            (32|64), u32 index_bits (32), u64 reserved[2] = 0
//   row_ptr  (n_rows+1) × row_ptr_bits/8
//   col_idx  nnz × 4
//   val      nnz × sizeof(dtype)
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "../../include/lhpc.h"
#include "lhpc_abi.hpp"

namespace {

constexpr char kMagic[8] = {'L', 'H', 'P', 'C', 'C', 'S', 'R', '1'};

struct LcsrHeader {
  char magic[8];
  uint32_t version;
  uint32_t dtype;
  int64_t n_rows, n_cols, nnz;
  uint32_t row_ptr_bits, index_bits;
  uint64_t reserved[2];
};
static_assert(sizeof(LcsrHeader) == 64, "header is 64 bytes");

int64_t align64(int64_t v) { return (v + 63) & ~int64_t{63}; }

struct File {
  FILE *f = nullptr;
  ~File() {
    if (f) std::fclose(f);
  }
};

bool write_all(FILE *f, const void *p, size_t n) { return n == 0 || std::fwrite(p, 1, n, f) == n; }
bool pad_to(FILE *f, int64_t off) {
  static const char zeros[64] = {};
  const long cur = std::ftell(f);
  return cur >= 0 && write_all(f, zeros, static_cast<size_t>(off - cur));
}

struct Map {
  const char *p = nullptr;
  size_t n = 0;
  int fd = -1;
  ~Map() {
    if (p && n) munmap(const_cast<char *>(p), n);
    if (fd >= 0) close(fd);
  }
  bool open(const char *path) {
    fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st;
    if (fstat(fd, &st) != 0) return false;
    n = static_cast<size_t>(st.st_size);
    if (n == 0) return true;
    void *m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      p = nullptr;
      n = 0;
      return false;
    }
    p = static_cast<const char *>(m);
    return true;
  }
};

// ------------------------------------------------------------ Matrix Market
enum MmField { MM_REAL, MM_INTEGER, MM_PATTERN };
enum MmSym { MM_GENERAL, MM_SYMMETRIC, MM_SKEW };

struct MmInfo {
  MmField field;
  MmSym sym;
  int64_t n_rows, n_cols, entries;  // entries as listed in the file
  size_t data_off;                  // offset of the first entry line
};

std::string lower(std::string s) {
  for (auto &c : s) c = static_cast<char>(std::tolower(static_cast<unsigned char>(c)));
  return s;
}

int mm_parse_header(const Map &m, MmInfo &info) {
  const char *p = m.p, *e = m.p + m.n;
  auto line_end = [&](const char *q) {
    while (q < e && *q != '\n') ++q;
    return q;
  };
  const char *le = line_end(p);
  std::string banner(p, le);
  char obj[64] = {}, fmt[64] = {}, field[64] = {}, sym[64] = {};
  if (std::sscanf(banner.c_str(), "%%%%MatrixMarket %63s %63s %63s %63s", obj, fmt, field, sym) != 4)
    return LHPC_ERR_INVALID_ARG;
  if (lower(obj) != "matrix" || lower(fmt) != "coordinate") return LHPC_ERR_UNSUPPORTED;  // dense "array" not supported
  const std::string f = lower(field), s = lower(sym);
  if (f == "real" || f == "double") info.field = MM_REAL;
  else if (f == "integer") info.field = MM_INTEGER;
  else if (f == "pattern") info.field = MM_PATTERN;
  else return LHPC_ERR_UNSUPPORTED;  // complex
  if (s == "general") info.sym = MM_GENERAL;
  else if (s == "symmetric") info.sym = MM_SYMMETRIC;
  else if (s == "skew-symmetric") info.sym = MM_SKEW;
  else return LHPC_ERR_UNSUPPORTED;  // hermitian
  p = le < e ? le + 1 : e;
  while (p < e) {  // comments / blank lines, then the size line
    le = line_end(p);
    const char *q = p;
    while (q < le && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
    if (q == le || *q == '%') {
      p = le < e ? le + 1 : e;
      continue;
    }
    long long r = 0, c = 0, z = 0;
    if (std::sscanf(std::string(q, le).c_str(), "%lld %lld %lld", &r, &c, &z) != 3 || r < 0 || c < 0 || z < 0)
      return LHPC_ERR_INVALID_ARG;
    if (info.sym != MM_GENERAL && r != c) return LHPC_ERR_INVALID_ARG;  // symmetric storage needs a square matrix
    info.n_rows = r;
    info.n_cols = c;
    info.entries = z;
    info.data_off = static_cast<size_t>((le < e ? le + 1 : e) - m.p);
    return LHPC_OK;
  }
  return LHPC_ERR_INVALID_ARG;
}

inline const char *skip_ws(const char *p, const char *e) {
  while (p < e && (*p == ' ' || *p == '\t' || *p == '\r' || *p == '\n')) ++p;
  return p;
}

inline bool parse_i64(const char *&p, const char *e, int64_t &v) {
  p = skip_ws(p, e);
  bool neg = false;
  if (p < e && (*p == '-' || *p == '+')) neg = *p++ == '-';
  if (p >= e || !std::isdigit(static_cast<unsigned char>(*p))) return false;
  int64_t x = 0;
  while (p < e && std::isdigit(static_cast<unsigned char>(*p))) x = x * 10 + (*p++ - '0');
  v = neg ? -x : x;
  return true;
}

inline bool parse_f64(const char *&p, const char *e, double &v) {
  p = skip_ws(p, e);
  char buf[128];
  size_t k = 0;
  while (p < e && k < sizeof(buf) - 1 && !std::isspace(static_cast<unsigned char>(*p))) buf[k++] = *p++;
  buf[k] = 0;
  if (!k) return false;
  char *end = nullptr;
  v = std::strtod(buf, &end);
  return end == buf + k;
}

}  // namespace

extern "C" int lhpc_csr_save(const char *path, int dtype, int64_t n_rows, int64_t n_cols, int64_t nnz,
                             const void *row_ptr, int row_ptr_bits, const int32_t *col_idx, const void *val) {
  try {
    if (!path || n_rows < 0 || n_cols < 0 || nnz < 0 || !row_ptr || (row_ptr_bits != 32 && row_ptr_bits != 64) ||
        (nnz > 0 && (!col_idx || !val)) || (dtype != LHPC_F32 && dtype != LHPC_F64))
      return LHPC_ERR_INVALID_ARG;
    LcsrHeader h{};
    std::memcpy(h.magic, kMagic, 8);
    h.version = 1;
    h.dtype = static_cast<uint32_t>(dtype);
    h.n_rows = n_rows;
    h.n_cols = n_cols;
    h.nnz = nnz;
    h.row_ptr_bits = static_cast<uint32_t>(row_ptr_bits);
    h.index_bits = 32;
    File f;
    f.f = std::fopen(path, "wb");
    if (!f.f) return LHPC_ERR_INVALID_ARG;
    const int64_t rpb = (n_rows + 1) * (row_ptr_bits / 8), vb = dtype == LHPC_F32 ? 4 : 8;
    const int64_t o_rp = 64, o_col = align64(o_rp + rpb), o_val = align64(o_col + nnz * 4);
    if (!write_all(f.f, &h, 64) || !write_all(f.f, row_ptr, static_cast<size_t>(rpb)) || !pad_to(f.f, o_col) ||
        !write_all(f.f, col_idx, static_cast<size_t>(nnz * 4)) || !pad_to(f.f, o_val) ||
        !write_all(f.f, val, static_cast<size_t>(nnz * vb)))
      return LHPC_ERR_INTERNAL;
    if (std::fflush(f.f) != 0) return LHPC_ERR_INTERNAL;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_csr_load_header(const char *path, int *dtype, int64_t *n_rows, int64_t *n_cols, int64_t *nnz,
                                    int *row_ptr_bits) {
  try {
    if (!path) return LHPC_ERR_INVALID_ARG;
    File f;
    f.f = std::fopen(path, "rb");
    if (!f.f) return LHPC_ERR_INVALID_ARG;
    LcsrHeader h{};
    if (std::fread(&h, 1, 64, f.f) != 64 || std::memcmp(h.magic, kMagic, 8) != 0 || h.version != 1 ||
        (h.dtype != LHPC_F32 && h.dtype != LHPC_F64) || (h.row_ptr_bits != 32 && h.row_ptr_bits != 64) ||
        h.index_bits != 32 || h.n_rows < 0 || h.n_cols < 0 || h.nnz < 0)
      return LHPC_ERR_BAD_CSR;
    if (dtype) *dtype = static_cast<int>(h.dtype);
    if (n_rows) *n_rows = h.n_rows;
    if (n_cols) *n_cols = h.n_cols;
    if (nnz) *nnz = h.nnz;
    if (row_ptr_bits) *row_ptr_bits = static_cast<int>(h.row_ptr_bits);
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_csr_load(const char *path, void *row_ptr, int32_t *col_idx, void *val) {
  try {
    int dtype = 0, rpbits = 0;
    int64_t n_rows = 0, n_cols = 0, nnz = 0;
    if (int st = lhpc_csr_load_header(path, &dtype, &n_rows, &n_cols, &nnz, &rpbits)) return st;
    if (!row_ptr || (nnz > 0 && (!col_idx || !val))) return LHPC_ERR_INVALID_ARG;
    Map m;
    if (!m.open(path)) return LHPC_ERR_INVALID_ARG;
    const int64_t rpb = (n_rows + 1) * (rpbits / 8), vb = dtype == LHPC_F32 ? 4 : 8;
    const int64_t o_rp = 64, o_col = align64(o_rp + rpb), o_val = align64(o_col + nnz * 4);
    if (static_cast<int64_t>(m.n) < o_val + nnz * vb) return LHPC_ERR_BAD_CSR;  // truncated
    std::memcpy(row_ptr, m.p + o_rp, static_cast<size_t>(rpb));
    if (nnz > 0) {
      std::memcpy(col_idx, m.p + o_col, static_cast<size_t>(nnz * 4));
      std::memcpy(val, m.p + o_val, static_cast<size_t>(nnz * vb));
    }
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_mm_read_header(const char *path, int64_t *n_rows, int64_t *n_cols, int64_t *nnz_max,
                                   int *symmetry, int *field) {
  try {
    if (!path) return LHPC_ERR_INVALID_ARG;
    Map m;
    if (!m.open(path) || !m.p) return LHPC_ERR_INVALID_ARG;
    MmInfo info{};
    if (int st = mm_parse_header(m, info)) return st;
    if (n_rows) *n_rows = info.n_rows;
    if (n_cols) *n_cols = info.n_cols;
    // symmetric / skew files store one triangle: off-diagonal entries expand to two
    if (nnz_max) *nnz_max = info.sym == MM_GENERAL ? info.entries : 2 * info.entries;
    if (symmetry) *symmetry = static_cast<int>(info.sym);
    if (field) *field = static_cast<int>(info.field);
    return LHPC_OK;
  } LHPC_ABI_CATCH
}

extern "C" int lhpc_mm_read_coo(const char *path, int32_t *rows, int32_t *cols, double *vals, int64_t *count) {
  try {
    if (!path || !count) return LHPC_ERR_INVALID_ARG;
    Map m;
    if (!m.open(path) || !m.p) return LHPC_ERR_INVALID_ARG;
    MmInfo info{};
    if (int st = mm_parse_header(m, info)) return st;
    if (info.n_rows > INT32_MAX || info.n_cols > INT32_MAX) return LHPC_ERR_UNSUPPORTED;
    const char *p = m.p + info.data_off, *e = m.p + m.n;
    int64_t k = 0;
    for (int64_t i = 0; i < info.entries; ++i) {
      p = skip_ws(p, e);
      while (p < e && *p == '%') {  // stray comment lines
        while (p < e && *p != '\n') ++p;
        p = skip_ws(p, e);
      }
      int64_t r, c;
      double v = 1.0;
      if (!parse_i64(p, e, r) || !parse_i64(p, e, c)) return LHPC_ERR_INVALID_ARG;
      if (info.field == MM_INTEGER) {
        int64_t iv;
        if (!parse_i64(p, e, iv)) return LHPC_ERR_INVALID_ARG;
        v = static_cast<double>(iv);
      } else if (info.field == MM_REAL) {
        if (!parse_f64(p, e, v)) return LHPC_ERR_INVALID_ARG;
      }
      if (r < 1 || r > info.n_rows || c < 1 || c > info.n_cols) return LHPC_ERR_INVALID_ARG;
      if (rows) {
        rows[k] = static_cast<int32_t>(r - 1);
        cols[k] = static_cast<int32_t>(c - 1);
        vals[k] = v;
      }
      ++k;
      if (info.sym != MM_GENERAL && r != c) {
        if (rows) {
          rows[k] = static_cast<int32_t>(c - 1);
          cols[k] = static_cast<int32_t>(r - 1);
          vals[k] = info.sym == MM_SKEW ? -v : v;
        }
        ++k;
      }
    }
    *count = k;
    return LHPC_OK;
  } LHPC_ABI_CATCH
}
