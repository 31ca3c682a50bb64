// Score-file I/O of similarity.main (similarity.py:11-18, util.py:12-21), host side.
//
// The reference reads examples.json with json.loads, walks the nested dict in Python and writes
// every score file with json.dumps. At config 2 (7.5M pairs) that host work is ~90 % of the
// drop-in's end-to-end time (profiles/r02_e2e_c2_v1.json: 12.6 s of 18.9 s). Here:
//   blp_examples_parse  reads examples.json of the shape the reference's dataset_maker writes
//                       ({"user": {"business": label, ...}, ...}, json.dumps text) into flat
//                       arrays: per-pair user / business ids and the byte spans of every key;
//   blp_scores_write    writes one score file in the examples' order with exactly the text
//                       json.dumps({u: {b: value}}) produces: ", " / ": " separators, the keys'
//                       own bytes, ints for counts and the reference's int 0s, floats in Python's
//                       repr (shortest round-trip digits; fixed notation for decimal exponents in
//                       (-4, 16], else d.ddde+XX) -- formatted on 16 threads.
// Anything outside that shape (escaped or non-integer keys, duplicate keys, nested values) is
// BLP_E_UNSUP and the caller falls back to json.loads / json.dumps, so behaviour never differs.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <charconv>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "blp_internal.h"

namespace {
template <class T>
using Vec = blp::HostVec<T>;  // uninitialised on resize(); huge pages from 4 MiB (blp_internal.h)

struct HostFree {
  size_t n = 0;
  void operator()(char* p) const { blp::host_free(p, n); }
};
using HostBytes = std::unique_ptr<char[], HostFree>;
HostBytes host_bytes(size_t n) { return HostBytes(static_cast<char*>(blp::host_alloc(n)), HostFree{n}); }

struct Text {  // the file's bytes, read once (not zero-filled first)
  HostBytes p;
  size_t n = 0;
  const char* data() const { return p.get(); }
  size_t size() const { return n; }
};
}  // namespace

struct blp_examples {
  Text text;               // the file
  Vec<int64_t> u_off;      // [n_users + 1] first pair of each user
  Vec<int64_t> u_key;      // [n_users] byte offset of the user key (inside its quotes)
  Vec<int32_t> u_len;      // [n_users] its length
  Vec<int64_t> u_id;       // [n_users] int(user key)
  Vec<int64_t> v_key;      // [n_pairs] byte offset of the business key
  Vec<int32_t> v_len;      // [n_pairs]
  Vec<int64_t> v_id;       // [n_pairs] int(business key)
};

namespace {

using blp::fail;

struct Cursor {
  const char* p;
  const char* e;
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool eat(char c) {
    ws();
    if (p < e && *p == c) {
      ++p;
      return true;
    }
    return false;
  }
};

// A JSON string key that int() parses the way the reference's int(u) does, written without
// escapes: [+-]?[0-9]+ (json.dumps re-emits such a key byte for byte). Returns false otherwise.
bool int_key(Cursor& c, int64_t* off, int32_t* len, int64_t* id, const char* base) {
  c.ws();
  if (c.p >= c.e || *c.p != '"') return false;
  const char* s = ++c.p;
  while (c.p < c.e && *c.p != '"') {
    if (*c.p == '\\' || (unsigned char)*c.p < 0x20 || (unsigned char)*c.p >= 0x80) return false;
    ++c.p;
  }
  if (c.p >= c.e) return false;
  const char* t = s;
  const char* q = c.p++;
  bool neg = false;
  if (t < q && (*t == '-' || *t == '+')) neg = *t++ == '-';
  if (t == q || q - t > 18) return false;
  int64_t v = 0;
  for (; t < q; ++t) {
    if (*t < '0' || *t > '9') return false;
    v = v * 10 + (*t - '0');
  }
  *off = s - base;
  *len = (int32_t)(q - s);
  *id = neg ? -v : v;
  return true;
}

// a scalar value (the label) exactly as json.loads accepts it: a JSON number
// -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?, true, false, null, or Python's extra
// literals NaN, Infinity, -Infinity. Anything else is refused (BLP_E_UNSUP), so the json.loads
// path raises on it as the reference does.
bool skip_scalar(Cursor& c) {
  c.ws();
  auto lit = [&](const char* w) {
    const size_t n = strlen(w);
    if ((size_t)(c.e - c.p) >= n && memcmp(c.p, w, n) == 0) {
      c.p += n;
      return true;
    }
    return false;
  };
  if (lit("true") || lit("false") || lit("null") || lit("NaN") || lit("Infinity") || lit("-Infinity")) return true;
  auto digit = [&]() { return c.p < c.e && *c.p >= '0' && *c.p <= '9'; };
  if (c.p < c.e && *c.p == '-') ++c.p;
  if (!digit()) return false;
  if (*c.p == '0') {
    ++c.p;
  } else {
    while (digit()) ++c.p;
  }
  if (c.p < c.e && *c.p == '.') {
    ++c.p;
    if (!digit()) return false;
    while (digit()) ++c.p;
  }
  if (c.p < c.e && (*c.p == 'e' || *c.p == 'E')) {
    ++c.p;
    if (c.p < c.e && (*c.p == '+' || *c.p == '-')) ++c.p;
    if (!digit()) return false;
    while (digit()) ++c.p;
  }
  return true;
}

// The users of one byte range of the outer object: [p, e) starts at a user key and ends right
// after the ',' that follows its last user -- or, for the last range, at the end of the text
// (the outer '}' and trailing whitespace).
struct Part {
  std::vector<int64_t> u_key, u_id, v_key, v_id, u_cnt;
  std::vector<int32_t> u_len, v_len;
  int rc = BLP_OK;
  const char* err = nullptr;
};

void parse_part(const char* base, const char* p, const char* e, bool last, Part* o) {
  Cursor c{p, e};
  const size_t est = (size_t)(e - p) / 8 + 16;  // a pair takes >= 8 bytes ("1": 0, ): no regrowth
  o->v_key.reserve(est), o->v_len.reserve(est), o->v_id.reserve(est);
  auto bad = [&](const char* m) {
    o->rc = BLP_E_UNSUP;
    o->err = m;
  };
  for (;;) {
    int64_t off, id;
    int32_t len;
    if (!int_key(c, &off, &len, &id, base) || !c.eat(':') || !c.eat('{'))
      return bad("blp_examples_parse: outer key / inner object not of the simple shape");
    o->u_key.push_back(off);
    o->u_len.push_back(len);
    o->u_id.push_back(id);
    const size_t v0 = o->v_key.size();
    if (!c.eat('}')) {
      for (;;) {
        if (!int_key(c, &off, &len, &id, base) || !c.eat(':') || !skip_scalar(c))
          return bad("blp_examples_parse: inner key / value not of the simple shape");
        o->v_key.push_back(off);
        o->v_len.push_back(len);
        o->v_id.push_back(id);
        if (c.eat(',')) continue;
        if (c.eat('}')) break;
        return bad("blp_examples_parse: malformed inner object");
      }
    }
    o->u_cnt.push_back((int64_t)(o->v_key.size() - v0));
    if (c.eat(',')) {
      c.ws();
      if (!last && c.p == e) return;  // this range ends after the separator
      continue;
    }
    if (last && c.eat('}')) {
      c.ws();
      if (c.p != c.e) return bad("blp_examples_parse: trailing data");
      return;
    }
    return bad("blp_examples_parse: malformed outer object");
  }
}

// Duplicate business keys of users [u0, u1) (json.loads would keep the first position and the
// last value: not handled here, so refused). Equal keys have equal ids: the ids are sorted
// first, and key bytes compared only where two ids are equal ("5" and "05" differ).
bool unique_business_keys(const blp_examples* x, size_t u0, size_t u1) {
  const char* base = x->text.data();
  auto view = [&](int64_t k) { return std::string_view(base + x->v_key[k], (size_t)x->v_len[k]); };
  std::vector<int64_t> ids, ord;
  for (size_t u = u0; u < u1; ++u) {
    const int64_t b = x->u_off[u], e = x->u_off[u + 1];
    ids.assign(x->v_id.begin() + b, x->v_id.begin() + e);
    std::sort(ids.begin(), ids.end());
    if (std::adjacent_find(ids.begin(), ids.end()) == ids.end()) continue;
    ord.resize(e - b);
    for (int64_t k = b; k < e; ++k) ord[k - b] = k;
    std::sort(ord.begin(), ord.end(), [&](int64_t i, int64_t j) {
      if (x->v_id[i] != x->v_id[j]) return x->v_id[i] < x->v_id[j];
      return view(i) < view(j);
    });
    for (size_t k = 1; k < ord.size(); ++k)
      if (x->v_id[ord[k]] == x->v_id[ord[k - 1]] && view(ord[k]) == view(ord[k - 1])) return false;
  }
  return true;
}

// examples.json of the reference's shape, {"user": {"business": label, ...}, ...}, parsed on up
// to 16 threads: the text is cut at user boundaries (in this shape every '}' outside the outer
// braces closes a user's object: keys are digit strings and values scalars -- a '}' anywhere
// else fails the range that holds it, and the whole parse with it), each range parsed on its
// own, the parts concatenated in file order.
int parse(blp_examples* x) {
  const char* base = x->text.data();
  const char* const end = base + x->text.size();
  Cursor c{base, end};
  if (!c.eat('{')) return fail(BLP_E_UNSUP, "blp_examples_parse: not a JSON object");
  x->u_off.assign(1, 0);
  if (c.eat('}')) {
    c.ws();
    return c.p == c.e ? BLP_OK : fail(BLP_E_UNSUP, "blp_examples_parse: trailing data");
  }
  const char* body = c.p;
  const size_t n = (size_t)(end - body);
  const unsigned nt = (unsigned)std::max<size_t>(1, std::min<size_t>({16, std::thread::hardware_concurrency(), n >> 20}));
  std::vector<const char*> cut{body};
  for (unsigned t = 1; t < nt; ++t) {
    const char* q = std::max(body + n * t / nt, cut.back());
    q = static_cast<const char*>(memchr(q, '}', (size_t)(end - q)));
    if (!q) break;
    Cursor k{q + 1, end};
    if (!k.eat(',')) continue;  // the outer object's own '}' (or not this shape: the range fails)
    k.ws();
    if (k.p > cut.back() && k.p < end) cut.push_back(k.p);
  }
  cut.push_back(end);
  const size_t np = cut.size() - 1;
  std::vector<Part> part(np);
  std::vector<std::thread> th;
  for (size_t i = 1; i < np; ++i) th.emplace_back(parse_part, base, cut[i], cut[i + 1], i + 1 == np, &part[i]);
  parse_part(base, cut[0], cut[1], np == 1, &part[0]);
  for (auto& h : th) h.join();
  // the parts back to back, each copied by its own thread into its place
  std::vector<size_t> ub(np + 1, 0), vb(np + 1, 0);
  for (size_t i = 0; i < np; ++i) {
    if (part[i].rc) return fail(part[i].rc, part[i].err);
    ub[i + 1] = ub[i] + part[i].u_key.size();
    vb[i + 1] = vb[i] + part[i].v_key.size();
  }
  const size_t nu = ub[np], nv = vb[np];
  x->u_key.resize(nu), x->u_len.resize(nu), x->u_id.resize(nu), x->u_off.resize(nu + 1);
  x->v_key.resize(nv), x->v_len.resize(nv), x->v_id.resize(nv);
  x->u_off[0] = 0;
  auto place = [&](size_t i) {
    Part& pt = part[i];
    std::copy(pt.u_key.begin(), pt.u_key.end(), x->u_key.begin() + ub[i]);
    std::copy(pt.u_len.begin(), pt.u_len.end(), x->u_len.begin() + ub[i]);
    std::copy(pt.u_id.begin(), pt.u_id.end(), x->u_id.begin() + ub[i]);
    int64_t o = (int64_t)vb[i];
    for (size_t j = 0; j < pt.u_cnt.size(); ++j) x->u_off[ub[i] + j + 1] = (o += pt.u_cnt[j]);
    std::copy(pt.v_key.begin(), pt.v_key.end(), x->v_key.begin() + vb[i]);
    std::copy(pt.v_len.begin(), pt.v_len.end(), x->v_len.begin() + vb[i]);
    std::copy(pt.v_id.begin(), pt.v_id.end(), x->v_id.begin() + vb[i]);
    pt = Part();
  };
  th.clear();
  for (size_t i = 1; i < np; ++i) th.emplace_back(place, i);
  place(0);
  for (auto& h : th) h.join();
  {
    std::unordered_set<std::string_view> seen;
    seen.reserve(x->u_key.size() * 2);
    for (size_t i = 0; i < x->u_key.size(); ++i)
      if (!seen.insert(std::string_view(base + x->u_key[i], (size_t)x->u_len[i])).second)
        return fail(BLP_E_UNSUP, "blp_examples_parse: duplicate user key");
  }
  const size_t nusers = x->u_key.size();
  const unsigned nd = (unsigned)std::max<size_t>(1, std::min<size_t>(nt, nusers / 64));
  std::vector<uint8_t> ok(nd, 1);
  th.clear();
  for (unsigned t = 1; t < nd; ++t)
    th.emplace_back([&, t]() { ok[t] = unique_business_keys(x, nusers * t / nd, nusers * (t + 1) / nd); });
  ok[0] = unique_business_keys(x, 0, nusers / nd);
  for (auto& h : th) h.join();
  for (unsigned t = 0; t < nd; ++t)
    if (!ok[t]) return fail(BLP_E_UNSUP, "blp_examples_parse: duplicate business key");
  return BLP_OK;
}

// Python's repr(float) for a finite double (float_repr_style 'short': Py_DTSF_ADD_DOT_0),
// written at o (at most 24 bytes); returns the end.
char* put_repr(char* o, double v) {
  char buf[64];
  const auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
  // buf = [-]d[.ddd]e(+|-)XX : the shortest round-trip digits
  const char* p = buf;
  if (*p == '-') {
    *o++ = '-';
    ++p;
  }
  char dig[32];
  int nd = 0;
  while (*p != 'e') {
    if (*p != '.') dig[nd++] = *p;
    ++p;
  }
  int ex = 0;
  std::from_chars(p + 1 + (p[1] == '+' ? 1 : 0), r.ptr, ex);
  const int decpt = ex + 1;
  if (decpt <= -4 || decpt > 16) {  // exponent notation
    *o++ = dig[0];
    if (nd > 1) {
      *o++ = '.';
      std::memcpy(o, dig + 1, nd - 1);
      o += nd - 1;
    }
    const int e = decpt - 1;
    *o++ = 'e';
    *o++ = e < 0 ? '-' : '+';
    const int ae = e < 0 ? -e : e;
    if (ae < 10) *o++ = '0';
    o = std::to_chars(o, o + 8, ae).ptr;
  } else if (decpt <= 0) {  // 0.000ddd
    *o++ = '0';
    *o++ = '.';
    std::memset(o, '0', -decpt);
    o += -decpt;
    std::memcpy(o, dig, nd);
    o += nd;
  } else if (decpt >= nd) {  // ddd000.0
    std::memcpy(o, dig, nd);
    o += nd;
    std::memset(o, '0', decpt - nd);
    o += decpt - nd;
    *o++ = '.';
    *o++ = '0';
  } else {
    std::memcpy(o, dig, decpt);
    o += decpt;
    *o++ = '.';
    std::memcpy(o, dig + decpt, nd - decpt);
    o += nd - decpt;
  }
  return o;
}

inline char* put_bytes(char* o, const char* s, size_t n) {
  std::memcpy(o, s, n);
  return o + n;
}

}  // namespace

using namespace blp;

extern "C" {

int blp_examples_parse(const char* path, blp_examples** out) {
  BLP_CHECK(path && out, BLP_E_ARG, "blp_examples_parse: bad arguments");
  int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(BLP_E_ARG, std::string("blp_examples_parse: cannot open ") + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return fail(BLP_E_ARG, "blp_examples_parse: stat failed");
  }
  auto* x = new blp_examples();
  const size_t n = (size_t)st.st_size;
  x->text.p = host_bytes(std::max<size_t>(n, 1));
  x->text.n = n;
  if (!x->text.p) {
    close(fd);
    delete x;
    return fail(BLP_E_ARG, "blp_examples_parse: out of host memory");
  }
  // read in slices of >= 8 MiB on up to 16 threads (a 100 MB examples.json: ~4x one read())
  const size_t nt = std::max<size_t>(1, std::min<size_t>({16, std::thread::hardware_concurrency(), n >> 23}));
  std::vector<uint8_t> rok(nt, 0);
  auto slice = [&](size_t t) {
    size_t at = n * t / nt;
    const size_t to = n * (t + 1) / nt;
    while (at < to) {
      const ssize_t r = pread(fd, x->text.p.get() + at, to - at, (off_t)at);
      if (r <= 0) return;
      at += (size_t)r;
    }
    rok[t] = 1;
  };
  {
    std::vector<std::thread> th;
    for (size_t t = 1; t < nt; ++t) th.emplace_back(slice, t);
    slice(0);
    for (auto& h : th) h.join();
  }
  close(fd);
  if (std::count(rok.begin(), rok.end(), 1) != (long)nt) {
    delete x;
    return fail(BLP_E_ARG, "blp_examples_parse: short read");
  }
  const int rc = parse(x);
  if (rc) {
    delete x;
    return rc;
  }
  *out = x;
  return BLP_OK;
}

int blp_examples_info(const blp_examples* x, int64_t* n_users, int64_t* n_pairs) {
  BLP_CHECK(x, BLP_E_ARG, "blp_examples_info: null handle");
  if (n_users) *n_users = (int64_t)x->u_key.size();
  if (n_pairs) *n_pairs = (int64_t)x->v_key.size();
  return BLP_OK;
}

int blp_examples_ids(const blp_examples* x, int64_t* pair_u, int64_t* pair_v, int64_t* user_off) {
  BLP_CHECK(x, BLP_E_ARG, "blp_examples_ids: null handle");
  const int64_t nu = (int64_t)x->u_key.size(), np = (int64_t)x->v_key.size();
  // users in slices of about equal pair counts, on up to 16 threads (7.5M pairs at config 2)
  const unsigned nt = (unsigned)std::max<int64_t>(1, std::min<int64_t>({16, (int64_t)std::thread::hardware_concurrency(), np >> 18}));
  auto work = [&](unsigned t) {
    const int64_t u0 = std::lower_bound(x->u_off.begin(), x->u_off.end() - 1, np * (int64_t)t / nt) - x->u_off.begin();
    const int64_t u1 = t + 1 == nt ? nu : std::lower_bound(x->u_off.begin(), x->u_off.end() - 1, np * (int64_t)(t + 1) / nt) - x->u_off.begin();
    if (pair_u)
      for (int64_t u = u0; u < u1; ++u) std::fill(pair_u + x->u_off[u], pair_u + x->u_off[u + 1], x->u_id[u]);
    if (pair_v && u1 > u0) std::copy(x->v_id.begin() + x->u_off[u0], x->v_id.begin() + x->u_off[u1], pair_v + x->u_off[u0]);
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& h : th) h.join();
  if (user_off) std::copy(x->u_off.begin(), x->u_off.end(), user_off);
  return BLP_OK;
}

int blp_examples_destroy(blp_examples* x) {
  delete x;
  return BLP_OK;
}

int blp_scores_write(const blp_examples* x, const char* path, int kind, const uint8_t* present, const void* values,
                     int64_t n_values) {
  BLP_CHECK(x && path && kind >= BLP_SCORE_U32 && kind <= BLP_SCORE_REPR24, BLP_E_ARG, "blp_scores_write: bad arguments");
  const int64_t nu = (int64_t)x->u_key.size(), np = (int64_t)x->v_key.size();
  // k-th present pair -> values[k]: the prefix count of present pairs
  std::vector<int64_t> vidx;
  int64_t n_present = np;
  if (present) {
    vidx.resize((size_t)np);
    n_present = 0;
    for (int64_t i = 0; i < np; ++i) {
      vidx[i] = n_present;
      n_present += present[i] ? 1 : 0;
    }
  }
  BLP_CHECK(kind == BLP_SCORE_NONE || (values && n_values == n_present), BLP_E_ARG,
            "blp_scores_write: values must hold one entry per present pair");
  const char* base = x->text.data();
  const unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  // users cut into nt slices of about equal pair counts, formatted concurrently
  std::vector<int64_t> cut(nt + 1, nu);
  cut[0] = 0;
  for (unsigned t = 1; t < nt; ++t)
    cut[t] = std::lower_bound(x->u_off.begin(), x->u_off.end(), np * (int64_t)t / nt) - x->u_off.begin();
  for (unsigned t = 1; t <= nt; ++t) cut[t] = std::max(cut[t], cut[t - 1]);
  // Two passes per slice: the exact byte length of its text (so every slice knows its file offset
  // up front), then the text itself, formatted through a small reusable buffer and written at its
  // offset as the buffer fills (no slice-sized buffers: their first-touch faults and zeroing were
  // most of this call's cost at config 2's ~1.2 GB of text per six files).
  // value text of present pair k (vi = its values index); returns its length, writing at o
  auto value = [&](char* o, int64_t vi) -> char* {
    if (kind == BLP_SCORE_U32) return std::to_chars(o, o + 12, ((const uint32_t*)values)[vi]).ptr;
    if (kind == BLP_SCORE_REPR24) {  // formatted on the device: copy the slot
      const char* sl = (const char*)values + 24 * vi;
      std::memcpy(o, sl, 24);  // within the pair's bound (key + 30)
      return o + strnlen(sl, 24);
    }
    const double v = ((const double*)values)[vi];
    if (kind == BLP_SCORE_F64_INT0 && v == 0.0) {
      *o++ = '0';  // similarity.py:118: nothing added -> the int 0
      return o;
    }
    return put_repr(o, v);
  };
  auto value_len = [&](int64_t vi) -> int64_t {
    if (kind == BLP_SCORE_U32) {
      uint32_t v = ((const uint32_t*)values)[vi];
      int64_t d = 1;
      while (v >= 10) v /= 10, ++d;
      return d;
    }
    if (kind == BLP_SCORE_REPR24) return (int64_t)strnlen((const char*)values + 24 * vi, 24);
    char tmp[40];
    return value(tmp, vi) - tmp;
  };
  std::vector<int64_t> part_len(nt, 0);
  std::vector<uint8_t> nonempty(nt, 0);
  // the walk shared by both passes: emit(bytes) for the structure, val(k, vi) for a value
  auto walk = [&](unsigned t, auto&& put, auto&& put_value, auto&& put_zero) {
    bool first_user = true;
    for (int64_t u = cut[t]; u < cut[t + 1]; ++u) {
      bool opened = false;
      for (int64_t k = x->u_off[u]; k < x->u_off[u + 1]; ++k) {
        const bool pres = !present || present[k];
        // what the reference assigns: 0 for a missing node, the score otherwise, nothing
        // for a present pair under an unmatched method (defaultdict: no empty user dicts)
        if (kind == BLP_SCORE_NONE && pres) continue;
        if (!opened) {
          if (!first_user) put(", ", 2);
          first_user = false;
          put("\"", 1);
          put(base + x->u_key[u], x->u_len[u]);
          put("\": {", 4);
          opened = true;
        } else {
          put(", ", 2);
        }
        put("\"", 1);
        put(base + x->v_key[k], x->v_len[k]);
        put("\": ", 3);
        if (!pres)
          put_zero();
        else
          put_value(present ? vidx[k] : k);
      }
      if (opened) put("}", 1);
    }
    return !first_user;
  };
  std::vector<int64_t> piece_max(nt, 0);  // the longest single piece of a slice's text
  auto count_slice = [&](unsigned t) {
    int64_t len = 0, mx = 0;
    nonempty[t] = walk(
        t,
        [&](const char*, size_t n) {
          len += (int64_t)n;
          mx = std::max<int64_t>(mx, (int64_t)n);
        },
        [&](int64_t vi) { len += value_len(vi); }, [&]() { len += 1; });
    part_len[t] = len;
    piece_max[t] = mx;
  };
  {
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; ++t) th.emplace_back(count_slice, t);
    count_slice(0);
    for (auto& h : th) h.join();
  }
  // "{" part ", " part ... "}": every slice at its own offset
  std::vector<int64_t> at(nt, 0);
  int64_t pos = 1;
  bool any = false;
  for (unsigned t = 0; t < nt; ++t) {
    if (!nonempty[t]) continue;
    if (any) pos += 2;
    at[t] = pos;
    pos += part_len[t];
    any = true;
  }
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) return fail(BLP_E_ARG, std::string("blp_scores_write: cannot open ") + path);
  auto put_at = [fd](const char* p, int64_t len, int64_t off) {
    while (len > 0) {
      const ssize_t w = pwrite(fd, p, (size_t)std::min<int64_t>(len, int64_t(1) << 30), (off_t)off);
      if (w <= 0) return false;
      p += w, len -= w, off += w;
    }
    return true;
  };
  std::vector<uint8_t> wok(nt, 1);
  auto write_slice = [&](unsigned t) {
    if (!nonempty[t]) return;
    // 1 MiB, or room for the slice's longest key (a piece) with the value after it
    const int64_t buf_bytes = std::max<int64_t>(int64_t(1) << 20, 2 * (piece_max[t] + 48));
    std::unique_ptr<char[]> buf(new (std::nothrow) char[(size_t)buf_bytes]);
    if (!buf) {
      wok[t] = 0;
      return;
    }
    char* const b0 = buf.get();
    char* o = b0;
    int64_t off = at[t];
    bool ok = true;
    if (any && at[t] > 1) {  // the ", " before this slice (not before the first non-empty one)
      ok = put_at(", ", 2, off - 2);
    }
    auto flush_if = [&](int64_t need) {
      if ((o - b0) + need <= buf_bytes) return;
      ok = ok && put_at(b0, o - b0, off);
      off += o - b0;
      o = b0;
    };
    walk(
        t,
        [&](const char* p, size_t n) {
          flush_if((int64_t)n);
          o = put_bytes(o, p, n);
        },
        [&](int64_t vi) {
          flush_if(40);
          o = value(o, vi);
        },
        [&]() {
          flush_if(1);
          *o++ = '0';
        });
    ok = ok && put_at(b0, o - b0, off);
    off += o - b0;
    wok[t] = ok && off == at[t] + part_len[t];
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(write_slice, t);
  write_slice(0);
  bool ok = put_at("{", 1, 0) && put_at("}", 1, pos);
  for (auto& h : th) h.join();
  for (unsigned t = 0; t < nt; ++t) ok = ok && wok[t];
  ok = (close(fd) == 0) && ok;
  return ok ? BLP_OK : fail(BLP_E_ARG, std::string("blp_scores_write: write failed: ") + path);
}

}  // extern "C"
