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

struct blp_examples {
  std::string text;               // the file
  std::vector<int64_t> u_off;     // [n_users + 1] first pair of each user
  std::vector<int64_t> u_key;     // [n_users] byte offset of the user key (inside its quotes)
  std::vector<int32_t> u_len;     // [n_users] its length
  std::vector<int64_t> u_id;      // [n_users] int(user key)
  std::vector<int64_t> v_key;     // [n_pairs] byte offset of the business key
  std::vector<int32_t> v_len;     // [n_pairs]
  std::vector<int64_t> v_id;      // [n_pairs] int(business key)
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

int parse(blp_examples* x) {
  const char* base = x->text.data();
  Cursor c{base, base + x->text.size()};
  if (!c.eat('{')) return fail(BLP_E_UNSUP, "blp_examples_parse: not a JSON object");
  x->u_off.push_back(0);
  if (!c.eat('}')) {
    for (;;) {
      int64_t off, id;
      int32_t len;
      if (!int_key(c, &off, &len, &id, base) || !c.eat(':') || !c.eat('{'))
        return fail(BLP_E_UNSUP, "blp_examples_parse: outer key / inner object not of the simple shape");
      x->u_key.push_back(off);
      x->u_len.push_back(len);
      x->u_id.push_back(id);
      if (!c.eat('}')) {
        for (;;) {
          if (!int_key(c, &off, &len, &id, base) || !c.eat(':') || !skip_scalar(c))
            return fail(BLP_E_UNSUP, "blp_examples_parse: inner key / value not of the simple shape");
          x->v_key.push_back(off);
          x->v_len.push_back(len);
          x->v_id.push_back(id);
          if (c.eat(',')) continue;
          if (c.eat('}')) break;
          return fail(BLP_E_UNSUP, "blp_examples_parse: malformed inner object");
        }
      }
      x->u_off.push_back((int64_t)x->v_key.size());
      if (c.eat(',')) continue;
      if (c.eat('}')) break;
      return fail(BLP_E_UNSUP, "blp_examples_parse: malformed outer object");
    }
  }
  c.ws();
  if (c.p != c.e) return fail(BLP_E_UNSUP, "blp_examples_parse: trailing data");
  // duplicate keys (json.loads keeps the first position and the last value): not handled here
  auto view = [&](int64_t off, int32_t len) { return std::string_view(base + off, (size_t)len); };
  {
    std::unordered_set<std::string_view> seen;
    seen.reserve(x->u_key.size() * 2);
    for (size_t i = 0; i < x->u_key.size(); ++i)
      if (!seen.insert(view(x->u_key[i], x->u_len[i])).second)
        return fail(BLP_E_UNSUP, "blp_examples_parse: duplicate user key");
  }
  std::vector<int64_t> ord;
  for (size_t u = 0; u + 1 < x->u_off.size(); ++u) {
    const int64_t b = x->u_off[u], e = x->u_off[u + 1];
    ord.resize(e - b);
    for (int64_t k = b; k < e; ++k) ord[k - b] = k;
    // by (id, key bytes): equal keys are then adjacent even where keys of one id differ ("5", "05")
    std::sort(ord.begin(), ord.end(), [&](int64_t i, int64_t j) {
      if (x->v_id[i] != x->v_id[j]) return x->v_id[i] < x->v_id[j];
      return view(x->v_key[i], x->v_len[i]) < view(x->v_key[j], x->v_len[j]);
    });
    for (size_t k = 1; k < ord.size(); ++k)
      if (x->v_id[ord[k]] == x->v_id[ord[k - 1]] &&
          view(x->v_key[ord[k]], x->v_len[ord[k]]) == view(x->v_key[ord[k - 1]], x->v_len[ord[k - 1]]))
        return fail(BLP_E_UNSUP, "blp_examples_parse: duplicate business key");
  }
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
  x->text.resize((size_t)st.st_size);
  size_t got = 0;
  while (got < x->text.size()) {
    const ssize_t r = read(fd, &x->text[got], x->text.size() - got);
    if (r <= 0) break;
    got += (size_t)r;
  }
  close(fd);
  if (got != x->text.size()) {
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
  const int64_t nu = (int64_t)x->u_key.size();
  for (int64_t u = 0; u < nu; ++u)
    if (pair_u)
      for (int64_t k = x->u_off[u]; k < x->u_off[u + 1]; ++k) pair_u[k] = x->u_id[u];
  if (pair_v) std::copy(x->v_id.begin(), x->v_id.end(), pair_v);
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
  // each slice formats into its own buffer, sized by a bound: per user its key + 8 bytes,
  // per pair its key + 6 + a value of at most 24 bytes (repr of a double; 10 digits of a u32)
  std::vector<std::unique_ptr<char[]>> part(nt);
  std::vector<int64_t> part_len(nt, 0);
  std::vector<uint8_t> nonempty(nt, 0);
  auto work = [&](unsigned t) {
    int64_t bound = 16;
    for (int64_t u = cut[t]; u < cut[t + 1]; ++u) bound += x->u_len[u] + 8;
    for (int64_t k = x->u_off[cut[t]]; k < x->u_off[cut[t + 1]]; ++k) bound += x->v_len[k] + 30;
    part[t].reset(new char[(size_t)bound]);
    char* const o0 = part[t].get();
    char* o = o0;
    bool first_user = true;
    for (int64_t u = cut[t]; u < cut[t + 1]; ++u) {
      bool opened = false;
      for (int64_t k = x->u_off[u]; k < x->u_off[u + 1]; ++k) {
        const bool pres = !present || present[k];
        // what the reference assigns: 0 for a missing node, the score otherwise, nothing
        // for a present pair under an unmatched method (defaultdict: no empty user dicts)
        if (kind == BLP_SCORE_NONE && pres) continue;
        if (!opened) {
          if (!first_user) o = put_bytes(o, ", ", 2);
          first_user = false;
          *o++ = '"';
          o = put_bytes(o, base + x->u_key[u], x->u_len[u]);
          o = put_bytes(o, "\": {", 4);
          opened = true;
        } else {
          o = put_bytes(o, ", ", 2);
        }
        *o++ = '"';
        o = put_bytes(o, base + x->v_key[k], x->v_len[k]);
        o = put_bytes(o, "\": ", 3);
        if (!pres) {
          *o++ = '0';
          continue;
        }
        const int64_t vi = present ? vidx[k] : k;
        if (kind == BLP_SCORE_U32) {
          o = std::to_chars(o, o + 12, ((const uint32_t*)values)[vi]).ptr;
        } else if (kind == BLP_SCORE_REPR24) {  // formatted on the device: copy the slot
          const char* sl = (const char*)values + 24 * vi;
          std::memcpy(o, sl, 24);  // within the pair's bound (key + 30)
          o += strnlen(sl, 24);
        } else {
          const double v = ((const double*)values)[vi];
          if (kind == BLP_SCORE_F64_INT0 && v == 0.0)
            *o++ = '0';  // similarity.py:118: nothing added -> the int 0
          else
            o = put_repr(o, v);
        }
      }
      if (opened) *o++ = '}';
    }
    part_len[t] = o - o0;
    nonempty[t] = !first_user;
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& h : th) h.join();
  // "{" part ", " part ... "}": every slice written at its own offset, concurrently (one
  // sequential fwrite of ~200 MB per file at config 2 dominated the file phase)
  const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC, 0666);
  if (fd < 0) return fail(BLP_E_ARG, std::string("blp_scores_write: cannot open ") + path);
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
  auto put = [fd](const char* p, int64_t len, int64_t off) {
    while (len > 0) {
      const ssize_t w = pwrite(fd, p, (size_t)std::min<int64_t>(len, int64_t(1) << 30), (off_t)off);
      if (w <= 0) return false;
      p += w, len -= w, off += w;
    }
    return true;
  };
  std::vector<uint8_t> wok(nt, 1);
  th.clear();
  bool sep = false;
  for (unsigned t = 0; t < nt; ++t) {
    if (!nonempty[t]) continue;
    const bool with_sep = sep;
    sep = true;
    th.emplace_back([&, t, with_sep]() {
      wok[t] = (!with_sep || put(", ", 2, at[t] - 2)) && put(part[t].get(), part_len[t], at[t]);
    });
  }
  bool ok = put("{", 1, 0) && put("}", 1, pos);
  for (auto& h : th) h.join();
  for (unsigned t = 0; t < nt; ++t) ok = ok && wok[t];
  ok = (close(fd) == 0) && ok;
  return ok ? BLP_OK : fail(BLP_E_ARG, std::string("blp_scores_write: write failed: ") + path);
}

}  // extern "C"
