// Native song-vector CSV reader (include/rqsid_io.h).  Host code: the file is memory-mapped, cut into
// per-thread byte ranges at record boundaries, and every worker parses its range into private
// buffers (kept rows' floats, id bytes, id offsets); rqsid_csv_copy concatenates them in file order.
// Files that contain a quote character are parsed by one worker, since a quoted field may hold a
// line break and a byte range cannot be cut safely without scanning from the start.
//
// Field and value rules follow the reference's reader (csv.reader + np.array(row[1:], float32),
// simplified_semantic_id_generator.py:51-69, train_semantic_ids.py:86-117); see the header.
#include "../../include/rqsid_io.h"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

namespace {

thread_local std::string g_err;

int fail(int rc, const std::string& msg) {
  g_err = msg;
  return rc;
}

struct Part {
  std::vector<float> vec;       // kept rows x dim
  std::vector<char> ids;        // kept ids, concatenated
  std::vector<int64_t> id_end;  // end offset (within ids) of each kept id
  int64_t nonnumeric = 0;
  int64_t records = 0;
};

inline bool is_eol(char c) { return c == '\n' || c == '\r'; }
inline bool is_space(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\f' || c == '\v'; }

// Correctly rounded decimal -> double for the common case, without strtod: s..e is a trimmed literal
// [sign] digits [. digits] [(e|E) [sign] digits] with at least one mantissa digit (anything else, '_'
// included, returns false and is left to the validating slow path).  With at most 19 significant digits the literal is
// w 10^q exactly (w < 2^64).  |q| <= 22 and w <= 2^53: one IEEE operation on exact operands (Clinger).
// |q| <= 27: x87 extended arithmetic (10^27 = 5^27 2^27 is exact in a 64-bit significand) gives w 10^q
// within one unit of the 64-bit significand; rounding that to double is correct unless its 11 extra
// bits sit within one unit of the halfway pattern 0x400.  Anything else returns false (caller: strtod).
bool fast_decimal(const char* s, const char* e, double* out) {
  static const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                                 1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  bool neg = false;
  if (s < e && (*s == '-' || *s == '+')) neg = *s++ == '-';
  uint64_t w = 0;
  int nd = 0, q = 0;
  bool md = false;  // a mantissa digit seen
  for (; s < e && *s >= '0' && *s <= '9'; ++s) {
    md = true;
    if (nd || *s != '0') {
      if (nd == 19) return false;
      w = w * 10 + (uint64_t)(*s - '0');
      ++nd;
    }
  }
  if (s < e && *s == '.') {
    for (++s; s < e && *s >= '0' && *s <= '9'; ++s) {
      md = true;
      if (nd || *s != '0') {
        if (nd == 19) return false;
        w = w * 10 + (uint64_t)(*s - '0');
        ++nd;
      }
      --q;
    }
  }
  if (!md) return false;
  if (s < e && (*s == 'e' || *s == 'E')) {
    ++s;
    bool eneg = false;
    if (s < e && (*s == '-' || *s == '+')) eneg = *s++ == '-';
    if (s == e) return false;
    int x = 0;
    for (; s < e && *s >= '0' && *s <= '9'; ++s) {
      if (x > 10000) return false;
      x = x * 10 + (*s - '0');
    }
    q += eneg ? -x : x;
  }
  if (s != e) return false;
  if (w == 0) {
    *out = neg ? -0.0 : 0.0;
    return true;
  }
  if (q < -27 || q > 27) return false;
  double d;
  if (w <= (1ull << 53) && q >= -22 && q <= 22) {
    d = (double)w;
    d = q < 0 ? d / p10[-q] : d * p10[q];
  } else {
    static const struct P10L {  // 10^0 .. 10^27, exact in the x87 64-bit significand
      long double v[28];
      P10L() {
        v[0] = 1.0L;
        for (int i = 1; i < 28; ++i) v[i] = v[i - 1] * 10.0L;
      }
    } lp;
    const long double r = q < 0 ? (long double)w / lp.v[-q] : (long double)w * lp.v[q];
    // x87 extended layout: explicit 64-bit significand, then sign and 15-bit exponent (bias 16383)
    uint64_t bits;
    uint16_t se;
    memcpy(&bits, &r, 8);
    memcpy(&se, reinterpret_cast<const char*>(&r) + 8, 2);
    const int ex = (int)(se & 0x7fff) - 16383;
    if (ex < -1020 || ex > 1022) return false;  // keep clear of double subnormals and overflow
    const uint32_t low = (uint32_t)(bits & 0x7ffu);
    if (low >= 0x3ffu && low <= 0x401u) return false;
    d = (double)r;
  }
  *out = neg ? -d : d;
  return true;
}

// Python float(str) for ASCII text: optional surrounding whitespace, optional sign, then either a
// decimal literal (digits with single underscores between digits, optional fraction and exponent) or
// nan / inf / infinity in any case.  Returns false for anything Python would reject (hex, "nan(…)",
// suffixes, empty).  The value is strtod's correctly rounded double, as CPython's.
bool parse_py_float(const char* b, const char* e, double* out) {
  while (b < e && is_space(*b)) ++b;
  while (e > b && is_space(e[-1])) --e;
  if (b == e) return false;
  char buf[128];
  size_t n = 0;
  const char* p = b;
  bool neg = false;
  if (*p == '+' || *p == '-') neg = (*p++ == '-');
  const size_t rest = (size_t)(e - p);
  auto ieq = [&](const char* w) {
    const size_t m = strlen(w);
    if (rest != m) return false;
    for (size_t i = 0; i < m; ++i)
      if ((p[i] | 0x20) != w[i]) return false;
    return true;
  };
  if (((*p >= '0' && *p <= '9') || *p == '.') && fast_decimal(b, e, out)) return true;  // no copy
  if (ieq("nan")) { *out = neg ? -NAN : NAN; return true; }
  if (ieq("inf") || ieq("infinity")) { *out = neg ? -INFINITY : INFINITY; return true; }
  // decimal literal: [digits][.digits][(e|E)[sign]digits], at least one mantissa digit,
  // '_' only between two digits
  bool mant_digit = false, exp_digit = false, in_exp = false, dot = false;
  size_t kept = 0;
  for (const char* q = p; q < e; ++q) {
    const char c = *q;
    if (c >= '0' && c <= '9') {
      (in_exp ? exp_digit : mant_digit) = true;
    } else if (c == '_') {
      if (q == p || q + 1 >= e || !(q[-1] >= '0' && q[-1] <= '9') || !(q[1] >= '0' && q[1] <= '9')) return false;
      continue;
    } else if (c == '.') {
      if (dot || in_exp) return false;
      dot = true;
    } else if (c == 'e' || c == 'E') {
      if (in_exp || !mant_digit) return false;
      in_exp = true;
    } else if (c == '+' || c == '-') {
      if (!(in_exp && (q[-1] == 'e' || q[-1] == 'E'))) return false;
    } else {
      return false;
    }
    ++kept;
  }
  if (!mant_digit || (in_exp && !exp_digit)) return false;
  std::string big;
  char* dst = buf;
  if (kept + 2 > sizeof(buf)) {  // very long literal
    big.resize(kept + 2);
    dst = &big[0];
  }
  if (neg) dst[n++] = '-';
  for (const char* q = p; q < e; ++q)
    if (*q != '_') dst[n++] = *q;
  dst[n] = 0;
  if (fast_decimal(dst, dst + n, out)) return true;  // literals with '_'
  char* end = nullptr;
  *out = strtod(dst, &end);  // correctly rounded; overflow -> ±inf, underflow -> 0/subnormal, as CPython
  return end == dst + n;
}

// One csv record starting at p (p < e); returns the position after its line break.  Fields are
// cut per the excel dialect: a field that starts with '"' runs to the closing quote ('""' = one
// quote, line breaks kept), then unquoted text up to the next ',' or line break joins it.
struct Field {
  const char* b;
  const char* e;
  bool quoted;  // b..e holds raw quoted text (needs unescaping)
};

const char* cut_record(const char* p, const char* e, std::vector<Field>& f) {
  f.clear();
  for (;;) {
    Field fd{p, p, false};
    if (p < e && *p == '"') {
      fd.quoted = true;
      const char* q = p + 1;
      for (;;) {
        q = static_cast<const char*>(memchr(q, '"', (size_t)(e - q)));
        if (!q) { q = e; break; }
        if (q + 1 < e && q[1] == '"') { q += 2; continue; }
        ++q;  // past the closing quote
        break;
      }
      while (q < e && *q != ',' && !is_eol(*q)) ++q;
      fd.e = q;
      p = q;
    } else {
      while (p < e && *p != ',' && !is_eol(*p)) ++p;
      fd.e = p;
    }
    f.push_back(fd);
    if (p < e && *p == ',') { ++p; continue; }
    break;
  }
  if (p < e && *p == '\r') ++p;
  if (p < e && *p == '\n') ++p;
  return p;
}

// Text of a quoted field: "a""b"c -> a"bc; \r\n and \r inside quotes read as \n (universal newlines)
void unquote(const Field& fd, std::string& s) {
  s.clear();
  const char* p = fd.b + 1;
  bool open = true;
  for (; p < fd.e; ++p) {
    const char c = *p;
    if (open && c == '"') {
      if (p + 1 < fd.e && p[1] == '"') { s.push_back('"'); ++p; }
      else open = false;
      continue;
    }
    if (c == '\r') { s.push_back('\n'); if (p + 1 < fd.e && p[1] == '\n') ++p; continue; }
    s.push_back(c);
  }
}

void parse_range(const char* p, const char* e, int dim, Part& out) {
  std::vector<Field> f;
  std::vector<float> row((size_t)dim);
  std::string tmp;
  while (p < e) {
    p = cut_record(p, e, f);
    ++out.records;
    if (f.size() == 1 && f[0].b == f[0].e && !f[0].quoted) continue;  // blank line: csv yields []
    if (f.size() < 2) continue;
    bool ok = true;
    const bool right_dim = (int64_t)f.size() - 1 == dim;
    for (size_t j = 1; j < f.size(); ++j) {
      double v;
      if (f[j].quoted) {
        unquote(f[j], tmp);
        ok = parse_py_float(tmp.data(), tmp.data() + tmp.size(), &v);
      } else {
        ok = parse_py_float(f[j].b, f[j].e, &v);
      }
      if (!ok) break;
      if (right_dim) row[j - 1] = (float)v;
    }
    if (!ok) { ++out.nonnumeric; continue; }
    if (!right_dim) continue;
    out.vec.insert(out.vec.end(), row.begin(), row.end());
    if (f[0].quoted) {
      unquote(f[0], tmp);
      out.ids.insert(out.ids.end(), tmp.begin(), tmp.end());
    } else {
      out.ids.insert(out.ids.end(), f[0].b, f[0].e);
    }
    out.id_end.push_back((int64_t)out.ids.size());
  }
}

// end of the first `limit` records (universal newlines; quotes respected only when `quotes`)
const char* limit_end(const char* p, const char* e, int64_t limit, bool quotes) {
  std::vector<Field> f;
  for (int64_t i = 0; i < limit && p < e; ++i) {
    if (quotes) { p = cut_record(p, e, f); continue; }
    while (p < e && !is_eol(*p)) {
      const void* q = memchr(p, '\n', (size_t)(e - p));
      const char* nl = q ? static_cast<const char*>(q) : e;
      const void* r = memchr(p, '\r', (size_t)(nl - p));
      p = r ? static_cast<const char*>(r) : nl;
    }
    if (p < e && *p == '\r') ++p;
    if (p < e && *p == '\n') ++p;
  }
  return p;
}

// h.e (the file's end in ranges): the record boundary at or after x (x itself when it starts a record)
const char* next_record(const char* b, const char* x, const char* e) {
  if (x <= b) return b;
  if (x >= e) return e;
  if (is_eol(x[-1]) && !(x[-1] == '\r' && *x == '\n')) return x;
  while (x < e && !is_eol(*x)) ++x;
  if (x < e && *x == '\r') ++x;
  if (x < e && *x == '\n') ++x;
  return x;
}

uint16_t f32_to_f16(float f) {  // IEEE binary16, round to nearest even (torch .half(), numpy astype)
  uint32_t x;
  memcpy(&x, &f, 4);
  const uint32_t sign = (x >> 16) & 0x8000u;
  uint32_t a = x & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(sign | (a > 0x7f800000u ? 0x7e00u : 0x7c00u));
  if (a >= 0x477ff000u) return (uint16_t)(sign | 0x7c00u);  // rounds to >= 65520: inf
  if (a < 0x38800000u) {                                     // below 2^-14: subnormal half (or 0)
    if (a < 0x33000000u) return (uint16_t)sign;              // < 2^-25: rounds to 0
    const uint32_t m = (a & 0x7fffffu) | 0x800000u;
    const int shift = 126 - (int)(a >> 23);  // 14 + (113 - exp) ... value = m * 2^(exp-150)
    // half subnormal unit 2^-24: result = m * 2^(exp-150+24) = m >> (126 - exp)
    const uint32_t q = m >> shift, rem = m & ((1u << shift) - 1), half = 1u << (shift - 1);
    const uint32_t r = q + (rem > half || (rem == half && (q & 1u)));
    return (uint16_t)(sign | r);
  }
  const uint32_t r = a - 0x38000000u;  // rebias exponent 127 -> 15 (in the f32 field layout)
  const uint32_t q = r >> 13, rem = r & 0x1fffu;
  return (uint16_t)(sign | (q + (rem > 0x1000u || (rem == 0x1000u && (q & 1u)))));
}

}  // namespace

struct rqsid_csv {
  int dim = 0;
  std::vector<Part> parts;
  int64_t rows = 0, id_bytes = 0, nonnumeric = 0, records = 0;
};

extern "C" {

const char* rqsid_io_last_error(void) { return g_err.c_str(); }

int rqsid_csv_open(const char* path, int32_t dim, int64_t limit, int32_t n_threads, rqsid_csv** out) {
  if (!path || !out || dim <= 0) return fail(RQSID_IO_BAD_ARG, "rqsid_csv_open: bad arguments");
  *out = nullptr;
  struct stat st;
  if (stat(path, &st) != 0 || !S_ISREG(st.st_mode))
    return fail(RQSID_IO_NOT_FOUND, std::string("The specified data file was not found: ") + path);
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(RQSID_IO_FAILED, std::string("cannot open ") + path + ": " + strerror(errno));
  const size_t size = (size_t)st.st_size;
  const char* base = nullptr;
  void* map = nullptr;
  if (size) {
    map = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
    if (map == MAP_FAILED) {
      close(fd);
      return fail(RQSID_IO_FAILED, std::string("mmap failed: ") + strerror(errno));
    }
    madvise(map, size, MADV_SEQUENTIAL);
    base = static_cast<const char*>(map);
  }
  close(fd);
  rqsid_csv* h = new (std::nothrow) rqsid_csv;
  if (!h) {
    if (map) munmap(map, size);
    return fail(RQSID_IO_FAILED, "allocation failed");
  }
  h->dim = dim;
  int rc = RQSID_IO_OK;
  try {
    const char* b = base;
    const char* e = base + size;
    const bool quotes = size && memchr(b, '"', size) != nullptr;
    if (limit > 0) e = limit_end(b, e, limit, quotes);
    int t = n_threads > 0 ? n_threads : (int)std::max(1u, std::thread::hardware_concurrency());
    const size_t per = 2u << 20;  // at least 2 MiB per worker
    t = (int)std::min<size_t>((size_t)t, std::max<size_t>(1, (size_t)(e - b) / per));
    if (quotes) t = 1;
    std::vector<const char*> cut((size_t)t + 1);
    cut[0] = b;
    cut[(size_t)t] = e;
    for (int i = 1; i < t; ++i)
      cut[(size_t)i] = std::max(cut[(size_t)i - 1], next_record(b, b + (e - b) * i / t, e));
    h->parts.resize((size_t)t);
    if (t == 1) {
      parse_range(b, e, dim, h->parts[0]);
    } else {
      std::vector<std::thread> th;
      for (int i = 0; i < t; ++i)
        th.emplace_back(parse_range, cut[(size_t)i], cut[(size_t)i + 1], dim, std::ref(h->parts[(size_t)i]));
      for (auto& x : th) x.join();
    }
    for (auto& pt : h->parts) {
      h->rows += (int64_t)pt.id_end.size();
      h->id_bytes += (int64_t)pt.ids.size();
      h->nonnumeric += pt.nonnumeric;
      h->records += pt.records;
    }
    if (h->rows == 0)
      rc = fail(RQSID_IO_NO_ROWS, "No valid data with the correct embedding dimension found in the CSV file.");
  } catch (const std::exception& ex) {
    rc = fail(RQSID_IO_FAILED, std::string("rqsid_csv_open: ") + ex.what());
  }
  if (map) munmap(map, size);
  if (rc == RQSID_IO_FAILED) {
    delete h;
    return rc;
  }
  *out = h;
  return rc;
}

int64_t rqsid_csv_rows(const rqsid_csv* h) { return h ? h->rows : -1; }
int64_t rqsid_csv_id_bytes(const rqsid_csv* h) { return h ? h->id_bytes : -1; }
int64_t rqsid_csv_nonnumeric(const rqsid_csv* h) { return h ? h->nonnumeric : -1; }
int64_t rqsid_csv_records(const rqsid_csv* h) { return h ? h->records : -1; }

int rqsid_csv_copy(const rqsid_csv* h, float* vectors, char* ids, int64_t* id_off) {
  if (!h) return fail(RQSID_IO_BAD_ARG, "rqsid_csv_copy: null handle");
  int64_t row = 0, off = 0;
  if (id_off) id_off[0] = 0;
  for (const auto& pt : h->parts) {
    const int64_t n = (int64_t)pt.id_end.size();
    if (vectors && n) memcpy(vectors + row * h->dim, pt.vec.data(), pt.vec.size() * sizeof(float));
    if (ids && !pt.ids.empty()) memcpy(ids + off, pt.ids.data(), pt.ids.size());
    if (id_off)
      for (int64_t i = 0; i < n; ++i) id_off[row + i + 1] = off + pt.id_end[(size_t)i];
    row += n;
    off += (int64_t)pt.ids.size();
  }
  return RQSID_IO_OK;
}

int rqsid_csv_copy_f16(const rqsid_csv* h, uint16_t* vectors) {
  if (!h || !vectors) return fail(RQSID_IO_BAD_ARG, "rqsid_csv_copy_f16: bad arguments");
  int64_t o = 0;
  for (const auto& pt : h->parts)
    for (float v : pt.vec) vectors[o++] = f32_to_f16(v);
  return RQSID_IO_OK;
}

void rqsid_csv_close(rqsid_csv* h) { delete h; }

}  // extern "C"
