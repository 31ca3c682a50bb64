// graph.txt ingest (SNAP LoadEdgeList text format, similarity.py:16; written by
// dataset_maker.py:197 as "user business\n"). Host-side, multi-threaded: the file is
// split at line boundaries and each thread parses its slice into a private buffer.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <thread>
#include <vector>

#include "blp_internal.h"

namespace {

struct Slice {
  std::vector<int64_t> a, b;
};

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

}  // namespace

extern "C" int blp_edges_parse(const char* path, int c0, int c1, int64_t* a, int64_t* b, int64_t* m_out) {
  using namespace blp;
  BLP_CHECK(path && m_out && c0 >= 0 && c1 >= 0, BLP_E_ARG, "blp_edges_parse: bad arguments");
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
    data = (const char*)mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
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
  std::vector<Slice> sl(nt);
  auto work = [&](unsigned t) {
    const char* p = data + cut[t];
    const char* end = data + cut[t + 1];
    while (p < end) {
      const char* e = p;
      while (e < end && *e != '\n') ++e;
      if (e > p && *p != '#') {
        int64_t va, vb;
        if (parse_line(p, e, c0, c1, &va, &vb)) {
          sl[t].a.push_back(va);
          sl[t].b.push_back(vb);
        }
      }
      p = e + 1;
    }
  };
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; ++t) th.emplace_back(work, t);
  work(0);
  for (auto& x : th) x.join();
  if (data) munmap((void*)data, size);
  close(fd);
  int64_t m = 0;
  for (auto& s : sl) m += (int64_t)s.a.size();
  if (a && b) {
    BLP_CHECK(*m_out >= m, BLP_E_ARG, "blp_edges_parse: output arrays too small");
    int64_t k = 0;
    for (auto& s : sl) {
      std::copy(s.a.begin(), s.a.end(), a + k);
      std::copy(s.b.begin(), s.b.end(), b + k);
      k += (int64_t)s.a.size();
    }
  }
  *m_out = m;
  return BLP_OK;
}
