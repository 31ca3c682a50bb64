// graph.txt ingest (SNAP LoadEdgeList text format, similarity.py:16; written by
// dataset_maker.py:197 as "user business\n"). Host-side, multi-threaded: the file is
// split at line boundaries and each thread parses its slice into a private buffer.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#include "blp_internal.h"

namespace {

struct Slice {
  std::vector<int64_t> a, b;
  int64_t mn = INT64_MAX, mx = INT64_MIN;  // over both columns
};

// "digits ws digits [ws] \n" (the reference's graph.txt line, c0 = 0, c1 = 1) in one pass;
// false (p untouched) for anything else, which then goes through parse_line.
inline bool fast_line(const char*& p, const char* end, int64_t* va, int64_t* vb) {
  const char* q = p;
  if (q >= end || *q < '0' || *q > '9') return false;
  int64_t x = 0;
  int nd = 0;
  while (q < end && *q >= '0' && *q <= '9' && nd < 18) x = x * 10 + (*q++ - '0'), ++nd;
  if (q >= end || (*q != ' ' && *q != '\t')) return false;
  while (q < end && (*q == ' ' || *q == '\t')) ++q;
  if (q >= end || *q < '0' || *q > '9') return false;
  int64_t y = 0;
  nd = 0;
  while (q < end && *q >= '0' && *q <= '9' && nd < 18) y = y * 10 + (*q++ - '0'), ++nd;
  while (q < end && (*q == ' ' || *q == '\t' || *q == '\r')) ++q;
  if (q < end && *q != '\n') return false;
  *va = x;
  *vb = y;
  p = q + 1;
  return true;
}

// fast_line without bounds checks, for text the caller knows holds a '\n' at or after p: every
// scan below stops at the first byte outside its class, and '\n' is outside all of them.
inline bool fast_line_nl(const char*& p, int64_t* va, int64_t* vb) {
  const char* q = p;
  unsigned d = (unsigned char)*q - '0';
  if (d > 9) return false;
  uint64_t x = 0;
  const char* s = q;
  do x = x * 10 + d, d = (unsigned char)*++q - '0';
  while (d <= 9);
  if (q - s > 18 || (*q != ' ' && *q != '\t')) return false;
  do ++q;
  while (*q == ' ' || *q == '\t');
  d = (unsigned char)*q - '0';
  if (d > 9) return false;
  uint64_t y = 0;
  s = q;
  do y = y * 10 + d, d = (unsigned char)*++q - '0';
  while (d <= 9);
  if (q - s > 18) return false;
  while (*q == ' ' || *q == '\t' || *q == '\r') ++q;
  if (*q != '\n') return false;
  *va = (int64_t)x;
  *vb = (int64_t)y;
  p = q + 1;
  return true;
}

inline bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\r' || c == '\v' || c == '\f'; }

// parse one line [p, e) -> columns c0/c1 as int64; false when the line has too few columns
inline bool parse_line(const char* p, const char* e, int c0, int c1, int64_t* va, int64_t* vb) {
  int col = 0;
  bool ga = false, gb = false;
  while (p < e) {
    while (p < e && is_ws(*p)) ++p;
    if (p >= e) break;
    const char* q = p;
    while (q < e && !is_ws(*q)) ++q;
    if (col == c0 || col == c1) {
      const char* t = p;
      bool neg = false;
      if (*t == '-' || *t == '+') neg = (*t++ == '-');
      int64_t v = 0;
      bool ok = t < q;
      for (; t < q; ++t) {
        if (*t < '0' || *t > '9') {
          ok = false;
          break;
        }
        v = v * 10 + (*t - '0');
      }
      if (!ok) return false;
      if (neg) v = -v;
      if (col == c0) {
        *va = v;
        ga = true;
      }
      if (col == c1) {
        *vb = v;
        gb = true;
      }
    }
    ++col;
    p = q;
  }
  return ga && gb;
}


// Parse the file once into per-thread slices (file order within and across slices).
int parse_slices(const char* path, int c0, int c1, std::vector<Slice>& sl) {
  using namespace blp;
  BLP_CHECK(path && c0 >= 0 && c1 >= 0, BLP_E_ARG, "blp_edges_parse: bad arguments");
  int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(BLP_E_ARG, std::string("blp_edges_parse: cannot open ") + path);
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return fail(BLP_E_ARG, "blp_edges_parse: stat failed");
  }
  const size_t size = (size_t)st.st_size;
  const char* data = nullptr;
  if (size) {
    // populated up front: 16 threads faulting the same mapping page by page serialise on the
    // process's mmap lock
    data = (const char*)mmap(nullptr, size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
    if (data == MAP_FAILED) {
      close(fd);
      return fail(BLP_E_ARG, "blp_edges_parse: mmap failed");
    }
  }
  unsigned nt = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  if (size < (1u << 20)) nt = 1;
  std::vector<size_t> cut(nt + 1, size);
  cut[0] = 0;
  for (unsigned t = 1; t < nt; ++t) {
    size_t c = size * t / nt;
    while (c < size && data[c - 1] != '\n') ++c;
    cut[t] = c;
  }
  sl.assign(nt, Slice{});
  auto work = [&](unsigned t) {
    const char* p = data + cut[t];
    const char* end = data + cut[t + 1];
    Slice& S = sl[t];
    S.a.reserve((cut[t + 1] - cut[t]) / 12 + 16);
    S.b.reserve((cut[t + 1] - cut[t]) / 12 + 16);
    int64_t mn = INT64_MAX, mx = INT64_MIN;
    const bool fast = c0 == 0 && c1 == 1;
    // [p, nl_end): whole lines, each ending in '\n', parsed without bounds checks
    const char* nl_end = end;
    while (nl_end > p && nl_end[-1] != '\n') --nl_end;
    while (p < end) {
      int64_t va, vb;
      if (fast && (p < nl_end ? fast_line_nl(p, &va, &vb) : fast_line(p, end, &va, &vb))) {
        S.a.push_back(va);
        S.b.push_back(vb);
        mn = std::min(mn, std::min(va, vb));
        mx = std::max(mx, std::max(va, vb));
        continue;
      }
      const char* e = p;
      while (e < end && *e != '\n') ++e;
      if (e > p && *p != '#' && parse_line(p, e, c0, c1, &va, &vb)) {
        S.a.push_back(va);
        S.b.push_back(vb);
        mn = std::min(mn, std::min(va, vb));
        mx = std::max(mx, std::max(va, vb));
      }
      p = e + 1;
    }
    S.mn = mn;
    S.mx = mx;
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  if (data) munmap((void*)data, size);
  close(fd);
  return BLP_OK;
}

// f(t, lo, hi) over [0, n) cut into `nt` ranges, on nt threads
template <class F>
void par_for(int64_t n, unsigned nt, F f) {
  if (n < (1 << 16)) nt = 1;
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(f, t, n * t / nt, n * (t + 1) / nt);
  f(0u, (int64_t)0, n / nt);
  for (auto& x : th) x.join();
}

unsigned n_threads() { return std::max(1u, std::min(16u, std::thread::hardware_concurrency())); }

}  // namespace

// A parsed edge list and, when the id space is compact, its dense id map: ids seen in column
// 0 ascending, then the ids seen only in column 1 ascending (blp/graph.py HostGraph._ids; a
// reference bipartite graph.txt puts users in one dense range and businesses in another).
struct blp_edges {
  std::vector<Slice> sl;
  int64_t m = 0;
  int64_t n = 0, n_col0 = 0, lo = 0, span = 0;  // span == 0: no dense map (sparse id space)
  std::vector<int32_t> map;                       // [span] dense id of id lo + i, or -1
  std::vector<int64_t> node_ids;                  // [n] dense id -> original id
};

using namespace blp;

extern "C" int blp_edges_parse(const char* path, int c0, int c1, int64_t* a, int64_t* b, int64_t* m_out) {
  BLP_CHECK(m_out, BLP_E_ARG, "blp_edges_parse: bad arguments");
  std::vector<Slice> sl;
  if (int rc = parse_slices(path, c0, c1, sl)) return rc;
  int64_t m = 0;
  for (auto& x : sl) m += (int64_t)x.a.size();
  if (a && b) {
    BLP_CHECK(*m_out >= m, BLP_E_ARG, "blp_edges_parse: output arrays too small");
    int64_t k = 0;
    for (auto& x : sl) {
      std::copy(x.a.begin(), x.a.end(), a + k);
      std::copy(x.b.begin(), x.b.end(), b + k);
      k += (int64_t)x.a.size();
    }
  }
  *m_out = m;
  return BLP_OK;
}

extern "C" int blp_edges_load(const char* path, int c0, int c1, blp_edges** out) {
  BLP_CHECK(out, BLP_E_ARG, "blp_edges_load: null out");
  auto* e = new blp_edges();
  const bool prof = getenv("BLP_INGEST_PROF") != nullptr;
  auto now = []() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double tp = now();
  auto stamp = [&](const char* what) {
    if (prof) {
      const double t = now();
      fprintf(stderr, "blp_edges_load %s %.4f s\n", what, t - tp);
      tp = t;
    }
  };
  if (int rc = parse_slices(path, c0, c1, e->sl)) {
    delete e;
    return rc;
  }
  const unsigned nt = (unsigned)e->sl.size();
  std::vector<int64_t> base(nt + 1, 0);
  for (unsigned t = 0; t < nt; ++t) base[t + 1] = base[t] + (int64_t)e->sl[t].a.size();
  e->m = base[nt];
  if (e->m) {
    std::vector<std::thread> th;
    stamp("parse");
    int64_t lo = INT64_MAX, hi = INT64_MIN;  // tracked by the parse
    for (const Slice& x : e->sl) {
      lo = std::min(lo, x.mn);
      hi = std::max(hi, x.mx);
    }
    const int64_t span = hi - lo + 1;
    if (span > 0 && span <= std::max<int64_t>(4 * e->m, 1 << 20) && span < (int64_t(1) << 31)) {
      // presence per column. Each parse slice marks a private bitmap (random stores from 16
      // threads into one shared array ping-pong its cache lines between cores: 0.14 s at config 2),
      // then the bitmaps are OR-ed word range by word range into byte flags.
      std::vector<uint8_t> in0(span, 0), in1(span, 0);
      th.clear();
      const size_t words = (size_t)(span + 63) / 64;
      if ((size_t)nt * 2 * words * 8 <= (size_t(1) << 30)) {
        std::vector<std::vector<uint64_t>> p0(nt), p1(nt);
        auto mark = [&](unsigned t) {
          p0[t].assign(words, 0);
          p1[t].assign(words, 0);
          uint64_t* m0 = p0[t].data();
          uint64_t* m1 = p1[t].data();
          for (size_t i = 0; i < e->sl[t].a.size(); ++i) {
            const uint64_t u = (uint64_t)(e->sl[t].a[i] - lo), v = (uint64_t)(e->sl[t].b[i] - lo);
            m0[u >> 6] |= 1ull << (u & 63);
            m1[v >> 6] |= 1ull << (v & 63);
          }
        };
        for (unsigned t = 1; t < nt; ++t) th.emplace_back(mark, t);
        mark(0);
        for (auto& x : th) x.join();
        par_for((int64_t)words, n_threads(), [&](unsigned, int64_t w0, int64_t w1) {
          for (int64_t w = w0; w < w1; ++w) {
            uint64_t x0 = 0, x1 = 0;
            for (unsigned t = 0; t < nt; ++t) {
              x0 |= p0[t][w];
              x1 |= p1[t][w];
            }
            const int64_t i0 = 64 * w, i1 = std::min<int64_t>(span, i0 + 64);
            for (int64_t i = i0; i < i1; ++i) {
              in0[i] = (uint8_t)((x0 >> (i - i0)) & 1u);
              in1[i] = (uint8_t)((x1 >> (i - i0)) & 1u);
            }
          }
        });
      } else {  // very wide id spans: byte flags, concurrent stores of the same value only
        auto mark = [&](unsigned t) {
          for (size_t i = 0; i < e->sl[t].a.size(); ++i) {
            in0[e->sl[t].a[i] - lo] = 1;
            in1[e->sl[t].b[i] - lo] = 1;
          }
        };
        for (unsigned t = 1; t < nt; ++t) th.emplace_back(mark, t);
        mark(0);
        for (auto& x : th) x.join();
      }
      stamp("mark");
      // ranks: column-0 ids first, then column-1-only ids, each ascending (block counts + prefix)
      const unsigned nb = n_threads();
      std::vector<int64_t> c0n(nb + 1, 0), c1n(nb + 1, 0);
      par_for(span, nb, [&](unsigned t, int64_t b0, int64_t b1) {
        int64_t x = 0, y = 0;
        for (int64_t i = b0; i < b1; ++i) {
          x += in0[i];
          y += (int)(in0[i] == 0) & (int)(in1[i] != 0);
        }
        c0n[t + 1] = x;
        c1n[t + 1] = y;
      });
      const unsigned used = span < (1 << 16) ? 1u : nb;
      for (unsigned t = 0; t < used; ++t) {
        c0n[t + 1] += c0n[t];
        c1n[t + 1] += c1n[t];
      }
      e->lo = lo;
      e->span = span;
      e->n_col0 = c0n[used];
      e->n = e->n_col0 + c1n[used];
      e->map.assign(span, -1);
      e->node_ids.resize(e->n);
      par_for(span, nb, [&](unsigned t, int64_t b0, int64_t b1) {
        int64_t r0 = c0n[t], r1 = e->n_col0 + c1n[t];
        for (int64_t i = b0; i < b1; ++i) {
          if (in0[i]) {
            e->map[i] = (int32_t)r0;
            e->node_ids[r0++] = lo + i;
          } else if (in1[i]) {
            e->map[i] = (int32_t)r1;
            e->node_ids[r1++] = lo + i;
          }
        }
      });
      stamp("map");
    }
  }
  *out = e;
  return BLP_OK;
}

extern "C" int blp_edges_info(const blp_edges* e, int64_t* m, int64_t* n_nodes, int64_t* n_col0, int64_t* id_lo,
                              int64_t* id_span) {
  BLP_CHECK(e, BLP_E_ARG, "blp_edges_info: null handle");
  if (m) *m = e->m;
  if (n_nodes) *n_nodes = e->n;
  if (n_col0) *n_col0 = e->n_col0;
  if (id_lo) *id_lo = e->lo;
  if (id_span) *id_span = e->span;
  return BLP_OK;
}

extern "C" int blp_edges_fetch(const blp_edges* e, int64_t* a, int64_t* b, int32_t* da, int32_t* db, int64_t* node_ids,
                               int32_t* id_map) {
  BLP_CHECK(e, BLP_E_ARG, "blp_edges_fetch: null handle");
  BLP_CHECK(e->span > 0 || !(da || db || node_ids || id_map), BLP_E_STATE,
            "blp_edges_fetch: no dense id map (sparse id space): fetch a / b only");
  const unsigned nt = (unsigned)e->sl.size();
  std::vector<int64_t> base(nt + 1, 0);
  for (unsigned t = 0; t < nt; ++t) base[t + 1] = base[t] + (int64_t)e->sl[t].a.size();
  std::vector<std::thread> th;
  auto work = [&](unsigned t) {
    const Slice& x = e->sl[t];
    const int64_t k = base[t];
    for (size_t i = 0; i < x.a.size(); ++i) {
      if (a) a[k + i] = x.a[i];
      if (b) b[k + i] = x.b[i];
      if (da) da[k + i] = e->map[x.a[i] - e->lo];
      if (db) db[k + i] = e->map[x.b[i] - e->lo];
    }
  };
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  if (node_ids) std::copy(e->node_ids.begin(), e->node_ids.end(), node_ids);
  if (id_map) std::copy(e->map.begin(), e->map.end(), id_map);
  return BLP_OK;
}

extern "C" int blp_edges_destroy(blp_edges* e) {
  delete e;
  return BLP_OK;
}

// ids -> dense ids through a dense map (blp_edges_fetch's id_map): -1 for ids outside the graph
extern "C" int blp_ids_lookup(const int32_t* id_map, int64_t id_lo, int64_t id_span, const int64_t* ids, int64_t n,
                              int32_t* dense) {
  BLP_CHECK(id_map && n >= 0 && (n == 0 || (ids && dense)), BLP_E_ARG, "blp_ids_lookup: bad arguments");
  par_for(n, n_threads(), [&](unsigned, int64_t b0, int64_t b1) {
    for (int64_t i = b0; i < b1; ++i) {
      const int64_t o = ids[i] - id_lo;
      dense[i] = (o >= 0 && o < id_span) ? id_map[o] : -1;
    }
  });
  return BLP_OK;
}
