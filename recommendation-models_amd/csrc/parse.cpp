// parse.cpp -- native LIBSVM / LIBFFM sample parser (host C++, multi-threaded).
//
// Restates yr/data/SampleParser.scala:23-85 (/root/reference/src/main/scala/, yr/ =
// io/yaochi/recommendation/) for text already in memory:
//   LIBSVM  "label id:value id:value ..."          parseLIBSVM  :23-51
//   LIBFFM  "label field:id:value ..."             parseLIBFFM  :53-85
// row = line index, col = id - 1 (1-based ids), targets[line] = label.  Token rules follow
// java.lang.String.split(" ") / split(":") + Float.parseFloat / Long.parseLong as used there:
//   - tokens are separated by single spaces; trailing empty tokens are dropped (split drops them),
//     an empty token elsewhere (leading or doubled space) fails like the reference (the label
//     "" is a NumberFormatException, an empty "k:v" an ArrayIndexOutOfBounds);
//   - a pair needs at least 2 (LIBFFM: 3) ':'-fields; extra fields are ignored (kv(0), kv(1) only);
//   - integers: optional sign + decimal digits (Long.parseLong); floats: strtof over the whole token
//     (correctly rounded as Float.parseFloat; Java's 'f'/'d' suffixes are not accepted);
//   - lines end at '\n'; a '\r' before it is dropped (Hadoop LineRecordReader), and a final line
//     without '\n' counts.  Every error names the line (1-based) and the token.
// Lines are split into nthreads contiguous ranges parsed in parallel; outputs are concatenated in
// line order, so the result does not depend on nthreads.
#include <cerrno>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "rmx.h"
#include "rmx_internal.hpp"

struct rmx_samples {
  int format = 0;
  std::vector<int64_t> rows, cols, fields;
  std::vector<float> values, targets;
};

namespace {

struct Chunk {
  const char* b = nullptr;
  const char* e = nullptr;
  int64_t first_line = 0;  // global index of the chunk's first line
  std::vector<int64_t> rows, cols, fields;
  std::vector<float> values, targets;
  std::string err;
};

bool parse_i64(const char* b, const char* e, int64_t* out) {
  if (b == e) return false;
  const char* p = b;
  bool neg = false;
  if (*p == '+' || *p == '-') {
    neg = *p == '-';
    ++p;
  }
  if (p == e) return false;
  unsigned long long v = 0;
  for (; p < e; ++p) {
    const unsigned d = (unsigned)(*p - '0');
    if (d > 9) return false;
    if (__builtin_mul_overflow(v, 10ull, &v) || __builtin_add_overflow(v, (unsigned long long)d, &v)) return false;
  }
  if (v > (neg ? 9223372036854775808ull : 9223372036854775807ull)) return false;  // Long range
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return true;
}

// Clinger's fast path: a decimal with <= 7 significant digits and |exponent| <= 10 is m * 10^e with
// m < 2^24 and 10^|e| exact in fp32, so ONE fp32 multiply / divide rounds it correctly (as
// strtof / Float.parseFloat do).  Everything else goes to strtof.
bool parse_f32_fast(const char* b, const char* e, float* out) {
  static const float p10[] = {1e0f, 1e1f, 1e2f, 1e3f, 1e4f, 1e5f, 1e6f, 1e7f, 1e8f, 1e9f, 1e10f};
  const char* p = b;
  bool neg = false;
  if (p < e && (*p == '+' || *p == '-')) {
    neg = *p == '-';
    ++p;
  }
  uint32_t m = 0;
  int nd = 0, scale = 0, ndig = 0;
  for (; p < e && *p >= '0' && *p <= '9'; ++p, ++ndig) {
    if (m == 0 && *p == '0') continue;  // leading zeros
    if (++nd > 7) return false;
    m = m * 10 + (uint32_t)(*p - '0');
  }
  if (p < e && *p == '.') {
    ++p;
    for (; p < e && *p >= '0' && *p <= '9'; ++p, ++ndig) {
      if (m == 0 && *p == '0') {
        --scale;
        continue;
      }
      if (++nd > 7) return false;
      m = m * 10 + (uint32_t)(*p - '0');
      --scale;
    }
  }
  if (ndig == 0) return false;
  if (p < e && (*p == 'e' || *p == 'E')) {
    ++p;
    bool eneg = false;
    if (p < e && (*p == '+' || *p == '-')) {
      eneg = *p == '-';
      ++p;
    }
    if (p == e) return false;
    int ex = 0;
    for (; p < e && *p >= '0' && *p <= '9'; ++p) {
      ex = ex * 10 + (*p - '0');
      if (ex > 100) return false;
    }
    scale += eneg ? -ex : ex;
  }
  if (p != e) return false;
  if (m == 0) {
    *out = neg ? -0.f : 0.f;
    return true;
  }
  if (scale < -10 || scale > 10) return false;
  float v = (float)m;  // exact: m < 2^24
  v = scale < 0 ? v / p10[-scale] : v * p10[scale];
  *out = neg ? -v : v;
  return true;
}

bool parse_f32(const char* b, const char* e, float* out) {
  if (b == e) return false;
  if (parse_f32_fast(b, e, out)) return true;
  char buf[64];
  const size_t n = (size_t)(e - b);
  if (n >= sizeof(buf)) return false;
  std::memcpy(buf, b, n);
  buf[n] = 0;
  if (buf[0] == ' ' || buf[0] == '\t') return false;
  char* end = nullptr;
  errno = 0;
  const float v = std::strtof(buf, &end);
  if (end != buf + n) return false;
  *out = v;
  return true;
}

std::string tok(const char* b, const char* e) { return std::string(b, (size_t)(e - b)); }

// integer field ending at ':' (returns the char after it) -- nullptr with *why = 'A' when the token
// ends first (too few ':'-fields: ArrayIndexOutOfBounds), 'N' on a non-digit (NumberFormatException)
inline const char* scan_int(const char* p, const char* te, int64_t* out, char* why) {
  const char* b = p;
  while (p < te && *p != ':') ++p;
  if (p == te) {
    *why = 'A';
    return nullptr;
  }
  if (!parse_i64(b, p, out)) {
    *why = 'N';
    return nullptr;
  }
  return p + 1;
}

void parse_chunk(Chunk& c, int format) {
  const char* p = c.b;
  const size_t est = (size_t)(c.e - c.b) / 8;  // ~8 bytes per "id:v " pair on Criteo-like text
  c.rows.reserve(est);
  c.cols.reserve(est);
  c.values.reserve(est);
  if (format == 1) c.fields.reserve(est);
  int64_t line = c.first_line;
  while (p < c.e) {
    const char* nl = (const char*)std::memchr(p, '\n', (size_t)(c.e - p));
    const char* le = nl ? nl : c.e;
    const char* next = nl ? nl + 1 : c.e;
    if (le > p && le[-1] == '\r') --le;
    // split(" ") with trailing empty tokens removed
    const char* end = le;
    while (end > p && end[-1] == ' ') --end;
    const int64_t row = line - c.first_line;
    // label
    const char* t = p;
    while (t < end && *t != ' ') ++t;
    float label;
    if (!parse_f32(p, t, &label)) {
      c.err = "line " + std::to_string(line + 1) + ": bad label \"" + tok(p, t) + "\" (NumberFormatException)";
      return;
    }
    c.targets.push_back(label);
    while (t < end) {  // t at a separating space
      const char* tb = ++t;
      const char* te = tb;
      while (te < end && *te != ' ') ++te;
      int64_t key = 0, field = 0;
      char why = 0;
      const char* q = tb;
      if (format == 1) q = scan_int(q, te, &field, &why);
      if (q) q = scan_int(q, te, &key, &why);
      float value = 0.f;
      if (q) {
        const char* ve = q;
        while (ve < te && *ve != ':') ++ve;  // extra ':'-fields are ignored
        if (ve == q) why = 'A';              // "k:" -> split drops the empty field
        else if (!parse_f32(q, ve, &value)) why = 'N';
      }
      if (why) {
        c.err = "line " + std::to_string(line + 1) + ": token \"" + tok(tb, te) + "\" " +
                (why == 'A' ? std::string("has fewer than ") + (format == 1 ? "3" : "2") +
                                  " ':'-fields (ArrayIndexOutOfBoundsException)"
                            : std::string("(NumberFormatException)"));
        return;
      }
      c.rows.push_back(row);
      c.cols.push_back(key - 1);
      c.values.push_back(value);
      if (format == 1) c.fields.push_back(field);
      t = te;
    }
    ++line;
    p = next;
  }
}

}  // namespace

extern "C" int rmx_samples_parse(const char* text, size_t len, int format, int nthreads, rmx_samples** out) {
  if (!out || (!text && len > 0) || (format != RMX_FORMAT_LIBSVM && format != RMX_FORMAT_LIBFFM)) {
    rmx::set_error("rmx_samples_parse: bad args (format RMX_FORMAT_LIBSVM or RMX_FORMAT_LIBFFM)");
    return RMX_E_INVALID;
  }
  *out = nullptr;
  int T = nthreads > 0 ? nthreads : (int)std::max(1u, std::thread::hardware_concurrency());
  T = (int)std::min<size_t>((size_t)T, std::max<size_t>(1, len / 65536 + 1));
  std::vector<Chunk> ch(T);
  // contiguous byte ranges cut at line starts
  const char* end = text + len;
  const char* s = text;
  for (int i = 0; i < T; ++i) {
    const char* e = i + 1 == T ? end : text + len * (size_t)(i + 1) / (size_t)T;
    if (e < s) e = s;
    if (e < end) {
      const char* nl = (const char*)std::memchr(e, '\n', (size_t)(end - e));
      e = nl ? nl + 1 : end;
    }
    ch[i].b = s;
    ch[i].e = e;
    s = e;
  }
  // line numbers of chunk starts (for messages and row ids)
  int64_t lines = 0;
  for (int i = 0; i < T; ++i) {
    ch[i].first_line = lines;
    for (const char* p = ch[i].b; p < ch[i].e;) {
      const char* nl = (const char*)std::memchr(p, '\n', (size_t)(ch[i].e - p));
      ++lines;
      p = nl ? nl + 1 : ch[i].e;
    }
  }
  if (T == 1) {
    parse_chunk(ch[0], format);
  } else {
    std::vector<std::thread> th;
    for (int i = 0; i < T; ++i) th.emplace_back(parse_chunk, std::ref(ch[i]), format);
    for (auto& t : th) t.join();
  }
  for (auto& c : ch)
    if (!c.err.empty()) {
      rmx::set_error("rmx_samples_parse: " + c.err);
      return RMX_E_INVALID;
    }
  rmx_samples* r = new rmx_samples();
  r->format = format;
  if (T == 1) {  // one chunk: rows are already global (first_line == 0)
    r->rows.swap(ch[0].rows);
    r->cols.swap(ch[0].cols);
    r->values.swap(ch[0].values);
    r->targets.swap(ch[0].targets);
    r->fields.swap(ch[0].fields);
  } else {
    std::vector<size_t> off(T + 1, 0), loff(T + 1, 0);
    for (int i = 0; i < T; ++i) {
      off[i + 1] = off[i] + ch[i].cols.size();
      loff[i + 1] = loff[i] + ch[i].targets.size();
    }
    r->rows.resize(off[T]);
    r->cols.resize(off[T]);
    r->values.resize(off[T]);
    r->targets.resize(loff[T]);
    if (format == RMX_FORMAT_LIBFFM) r->fields.resize(off[T]);
    auto copy = [&](int i) {
      const Chunk& c = ch[i];
      for (size_t n = 0; n < c.rows.size(); ++n) r->rows[off[i] + n] = c.rows[n] + c.first_line;
      std::memcpy(r->cols.data() + off[i], c.cols.data(), sizeof(int64_t) * c.cols.size());
      std::memcpy(r->values.data() + off[i], c.values.data(), sizeof(float) * c.values.size());
      std::memcpy(r->targets.data() + loff[i], c.targets.data(), sizeof(float) * c.targets.size());
      if (format == RMX_FORMAT_LIBFFM)
        std::memcpy(r->fields.data() + off[i], c.fields.data(), sizeof(int64_t) * c.fields.size());
    };
    std::vector<std::thread> th;
    for (int i = 0; i < T; ++i) th.emplace_back(copy, i);
    for (auto& t : th) t.join();
  }
  *out = r;
  return RMX_OK;
}

extern "C" int rmx_samples_free(rmx_samples* s) {
  delete s;
  return RMX_OK;
}

extern "C" int64_t rmx_samples_lines(const rmx_samples* s) { return s ? (int64_t)s->targets.size() : -1; }
extern "C" int64_t rmx_samples_nnz(const rmx_samples* s) { return s ? (int64_t)s->cols.size() : -1; }
extern "C" const int64_t* rmx_samples_rows(const rmx_samples* s) { return s ? s->rows.data() : nullptr; }
extern "C" const int64_t* rmx_samples_cols(const rmx_samples* s) { return s ? s->cols.data() : nullptr; }
extern "C" const float* rmx_samples_values(const rmx_samples* s) { return s ? s->values.data() : nullptr; }
extern "C" const float* rmx_samples_targets(const rmx_samples* s) { return s ? s->targets.data() : nullptr; }
extern "C" const int64_t* rmx_samples_fields(const rmx_samples* s) {
  return (s && s->format == RMX_FORMAT_LIBFFM) ? s->fields.data() : nullptr;
}

// Regular batches (every line exactly n_fields pairs, the Reshape(B, F, k) contract of the models):
// int32 ids [lines][n_fields] for rmx_forward_ids / rmx_backward_ids (ParRecModel.scala:342 .toInt).
extern "C" int rmx_samples_ids(const rmx_samples* s, int32_t n_fields, int32_t* ids, int64_t cap) {
  if (!s || n_fields <= 0 || (!ids && cap > 0)) {
    rmx::set_error("rmx_samples_ids: bad args");
    return RMX_E_INVALID;
  }
  const int64_t L = (int64_t)s->targets.size();
  if ((int64_t)s->cols.size() != L * n_fields) {
    rmx::set_error("rmx_samples_ids: " + std::to_string(s->cols.size()) + " nonzeros is not lines * n_fields = " +
                   std::to_string(L * n_fields) + " (Reshape)");
    return RMX_E_SHAPE;
  }
  if (cap < L * n_fields) {
    rmx::set_error("rmx_samples_ids: capacity " + std::to_string(cap) + " < " + std::to_string(L * n_fields));
    return RMX_E_INVALID;
  }
  for (int64_t n = 0; n < L * n_fields; ++n) {
    if (s->rows[n] != n / n_fields) {
      rmx::set_error("rmx_samples_ids: line " + std::to_string(s->rows[n] + 1) + " does not have " +
                     std::to_string(n_fields) + " pairs");
      return RMX_E_SHAPE;
    }
    const int64_t c = s->cols[n];
    if (c < 0 || c > 2147483647) {
      rmx::set_error("rmx_samples_ids: id " + std::to_string(c + 1) + " outside [1, 2^31]");
      return RMX_E_INDEX;
    }
    ids[n] = (int32_t)c;
  }
  return RMX_OK;
}
