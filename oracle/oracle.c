/*
 * CPU ORACLE (C restatement) — TEST INFRASTRUCTURE ONLY.
 *
 * Checker for the HIP engine on cases too large for the pure-Python oracle, and the
 * `cpu_baseline` leg of bench.py. Never linked or loaded by the product.
 *
 * It restates the reference algorithm with the same structure:
 *   - og_create:       snap.LoadEdgeList(PUNGraph, ...) adjacency (similarity.py:16):
 *                      undirected, deduplicated, a self-loop stored once (GetDeg counts it once).
 *   - og_score_pairs:  similarity.users/business (similarity.py:20-106): per distinct source x
 *                      the exact-distance-2 set H2(x) (GetNodesAtHop(x,2), :29/:74) as a BFS
 *                      marker set; per pair |H2(x) ∩ N(y)| (:113-114), the Jaccard quotient
 *                      float(|∩|)/float(|∪|) (:108-111) and the Adamic-Adar sum of
 *                      (log deg)^-1 over deg > 1 (:116-126), N(y) = GetNodesAtHop(y,1) (:41/:85).
 *                      The Adamic-Adar terms are added exactly (128-bit integer in units of
 *                      2^-58: every term (log d)^-1 in [2^-5, 2) is such an integer) and the
 *                      sum is rounded once: the correctly rounded sum, math.fsum of the same
 *                      terms. The reference adds them in Python set order, rounding at every
 *                      add, and so differs from it by a few ulps at most.
 *   - og_hop3:         dataset_maker.py:139 GetNodesAtHop(G,u,3) candidate sets.
 * Pinned against tests/golden (reference outputs) by tests/test_oracle.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int64_t n;
    int64_t* rp;   /* n+1 */
    int32_t* ci;   /* rp[n]; sorted, unique; includes a self-loop once if present */
    int32_t* deg;  /* SNAP GetDeg = row length */
    uint8_t* self; /* 1 if the node has a self-loop */
} og_graph;

static int cmp_i32(const void* a, const void* b) {
    int32_t x = *(const int32_t*)a, y = *(const int32_t*)b;
    return x < y ? -1 : (x > y);
}

/* snap.LoadEdgeList adjacency (similarity.py:16) by counting sort: every directed entry
 * (a->b, and b->a unless a loop) scattered into its row, then each row sorted and
 * deduplicated. O(m) + the row sorts, so the 1B-edge config-5 graph builds in seconds
 * (bench.py --mode sharded parity); the result is the same CSR as a global sort + unique. */
/* Rows [lo, hi) of the directed entries: count (cnt != NULL) or scatter into raw at cur. */
static void og_rows_pass(int64_t m, const int32_t* a, const int32_t* b, int32_t lo, int32_t hi, int64_t* cnt,
                         int64_t* cur, int32_t* raw) {
    for (int64_t i = 0; i < m; ++i) {
        const int32_t x = a[i], y = b[i];
        if (x >= lo && x < hi) {
            if (cnt) cnt[x + 1]++;
            else raw[cur[x]++] = y;
        }
        if (x != y && y >= lo && y < hi) {
            if (cnt) cnt[y + 1]++;
            else raw[cur[y]++] = x;
        }
    }
}

/* The directed entries grouped by row for many threads: each thread counts its own chunk of the
 * edge list per row RANGE, the entries are scattered once into range order (row << 32 | col),
 * then every range is counting-sorted into its rows on its own (a range's rows belong to it
 * alone). The edge list is read twice in all, instead of twice per thread (the 1B-edge config-5
 * graph: 42.6 s -> seconds). pos[] gets the row offsets (exclusive prefix, pos[n] = total). */
static int32_t* og_raw_partitioned(int64_t n, int64_t m, const int32_t* a, const int32_t* b, int nt,
                                   int64_t* pos) {
    const int64_t R = 64 * (int64_t)nt, rb = (n + R - 1) / R;
    /* per-thread cursors, thread-major ([thread][range]): no two threads share a cache line */
    int64_t* cnt = (int64_t*)calloc((size_t)(R * nt), sizeof(int64_t));
    int64_t* rstart = (int64_t*)calloc((size_t)(R + 1), sizeof(int64_t));
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(static, 1)
#endif
    for (int t = 0; t < nt; ++t) {
        int64_t* c = cnt + (int64_t)t * R;
        const int64_t e0 = m * t / nt, e1 = m * (t + 1) / nt;
        for (int64_t i = e0; i < e1; ++i) {
            c[a[i] / rb]++;
            if (a[i] != b[i]) c[b[i] / rb]++;
        }
    }
    int64_t tot = 0;
    for (int64_t r = 0; r < R; ++r) {
        rstart[r] = tot;
        for (int t = 0; t < nt; ++t) {
            const int64_t c = cnt[(int64_t)t * R + r];
            cnt[(int64_t)t * R + r] = tot;
            tot += c;
        }
    }
    rstart[R] = tot;
    uint64_t* buf = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)(tot + 1));
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(static, 1)
#endif
    for (int t = 0; t < nt; ++t) {
        int64_t* c = cnt + (int64_t)t * R;
        const int64_t e0 = m * t / nt, e1 = m * (t + 1) / nt;
        for (int64_t i = e0; i < e1; ++i) {
            const uint32_t x = (uint32_t)a[i], y = (uint32_t)b[i];
            buf[c[x / rb]++] = (uint64_t)x << 32 | y;
            if (x != y) buf[c[y / rb]++] = (uint64_t)y << 32 | x;
        }
    }
    int32_t* raw = (int32_t*)malloc(sizeof(int32_t) * (size_t)(tot + 1));
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
#endif
    for (int64_t r = 0; r < R; ++r) { /* row counts of the range (its rows are its own) */
        for (int64_t i = rstart[r]; i < rstart[r + 1]; ++i) pos[(buf[i] >> 32) + 1]++;
    }
    for (int64_t i = 0; i < n; ++i) pos[i + 1] += pos[i];
#ifdef _OPENMP
#pragma omp parallel for num_threads(nt) schedule(dynamic, 1)
#endif
    for (int64_t r = 0; r < R; ++r) { /* rows of the range: a cursor per row, from pos */
        const int64_t v0 = r * rb, v1 = v0 + rb < n ? v0 + rb : n;
        if (v0 >= v1) continue;
        int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(v1 - v0));
        for (int64_t v = v0; v < v1; ++v) cur[v - v0] = pos[v];
        for (int64_t i = rstart[r]; i < rstart[r + 1]; ++i) raw[cur[(int64_t)(buf[i] >> 32) - v0]++] = (int32_t)(uint32_t)buf[i];
        free(cur);
    }
    free(buf);
    free(cnt);
    free(rstart);
    return raw;
}

og_graph* og_create(int64_t n, int64_t m, const int32_t* a, const int32_t* b) {
    og_graph* g = (og_graph*)calloc(1, sizeof(og_graph));
    int64_t* pos = (int64_t*)calloc((size_t)n + 2, sizeof(int64_t));
    int nt = 1;
#ifdef _OPENMP
    nt = m > (1 << 22) ? omp_get_max_threads() : 1;
    const char* force = getenv("OG_THREADS"); /* tests: the partitioned path on small graphs */
    if (force && atoi(force) > 0) nt = atoi(force);
#endif
    int32_t* raw;
    if (nt > 1) {
        raw = og_raw_partitioned(n, m, a, b, nt, pos);
    } else {
        og_rows_pass(m, a, b, 0, (int32_t)n, pos, NULL, NULL);
        for (int64_t i = 0; i < n; ++i) pos[i + 1] += pos[i];
        raw = (int32_t*)malloc(sizeof(int32_t) * (size_t)(pos[n] + 1));
        int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * ((size_t)n + 1));
        memcpy(cur, pos, sizeof(int64_t) * (size_t)n);
        og_rows_pass(m, a, b, 0, (int32_t)n, NULL, cur, raw);
        free(cur);
    }
    g->n = n;
    g->rp = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    g->deg = (int32_t*)calloc((size_t)n + 1, sizeof(int32_t));
    g->self = (uint8_t*)calloc((size_t)n + 1, 1);
    const int64_t nwords = (n + 63) / 64;
#ifdef _OPENMP
#pragma omp parallel
#endif
    {
        uint64_t* seen = NULL; /* long rows: sort + unique through a presence bitmap over [0, n) */
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 4096)
#endif
        for (int64_t r = 0; r < n; ++r) { /* sort + unique in place; the row's new length in deg */
            int32_t* row = raw + pos[r];
            int64_t len = pos[r + 1] - pos[r], u = 0;
            if (len > 64 && len * 4 > nwords) {
                if (!seen) seen = (uint64_t*)calloc((size_t)nwords, sizeof(uint64_t));
                for (int64_t i = 0; i < len; ++i) seen[row[i] >> 6] |= 1ull << (row[i] & 63);
                for (int64_t w = 0; w < nwords; ++w)
                    for (uint64_t v = seen[w]; v; v &= v - 1) row[u++] = (int32_t)(w * 64 + __builtin_ctzll(v));
                for (int64_t i = 0; i < u; ++i) seen[row[i] >> 6] = 0;
            } else {
                if (len > 1) qsort(row, (size_t)len, sizeof(int32_t), cmp_i32);
                for (int64_t i = 0; i < len; ++i)
                    if (i == 0 || row[i] != row[i - 1]) row[u++] = row[i];
            }
            g->deg[r] = (int32_t)u;
            for (int64_t i = 0; i < u; ++i)
                if (row[i] == r) g->self[r] = 1;
        }
        free(seen);
    }
    for (int64_t r = 0; r < n; ++r) g->rp[r + 1] = g->rp[r] + g->deg[r];
    g->ci = (int32_t*)malloc(sizeof(int32_t) * (size_t)(g->rp[n] + 1));
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 4096)
#endif
    for (int64_t r = 0; r < n; ++r) memcpy(g->ci + g->rp[r], raw + pos[r], sizeof(int32_t) * (size_t)g->deg[r]);
    free(raw);
    free(pos);
    return g;
}

void og_destroy(og_graph* g) {
    if (!g) return;
    free(g->rp);
    free(g->ci);
    free(g->deg);
    free(g->self);
    free(g);
}

int64_t og_n(const og_graph* g) { return g->n; }
int64_t og_nnz(const og_graph* g) { return g->rp[g->n]; }
/* The oracle's CSR (row_ptr[n + 1], col_idx[nnz]), owned by the graph: for comparisons of whole
 * adjacency structures (the config-5 exchange test). */
void og_csr(const og_graph* g, const int64_t** rp, const int32_t** ci) {
    *rp = g->rp;
    *ci = g->ci;
}
int32_t og_degree(const og_graph* g, int32_t v) { return g->deg[v]; }

/* Exact BFS distances from x up to `depth` into dist[] (-1 = farther). Returns the
 * number of nodes at exactly `depth`. visited[] lists touched nodes for cleanup. */
static int64_t bfs_exact(const og_graph* g, int32_t x, int depth, int8_t* dist, int32_t* visited,
                         int64_t* nvisited) {
    int64_t nv = 0, lo = 0, at = 0;
    dist[x] = 0;
    visited[nv++] = x;
    for (int d = 0; d < depth; ++d) {
        int64_t hi = nv;
        for (int64_t i = lo; i < hi; ++i) {
            int32_t z = visited[i];
            for (int64_t e = g->rp[z]; e < g->rp[z + 1]; ++e) {
                int32_t w = g->ci[e];
                if (dist[w] < 0) {
                    dist[w] = (int8_t)(d + 1);
                    visited[nv++] = w;
                }
            }
        }
        lo = hi;
    }
    at = nv - lo;
    *nvisited = nv;
    return at;
}

/* One pair batch; pairs need not be grouped (we group by x internally, in x order). */
int og_score_pairs(const og_graph* g, int64_t np, const int32_t* xs, const int32_t* ys, uint32_t mask,
                   uint32_t* cn, double* jac, double* aa, uint32_t* h2out, int nthreads) {
    int64_t n = g->n;
    int64_t* cnt = (int64_t*)calloc((size_t)n + 1, sizeof(int64_t));
    int64_t* perm = (int64_t*)malloc(sizeof(int64_t) * (size_t)(np + 1));
    for (int64_t i = 0; i < np; ++i) cnt[xs[i] + 1]++;
    for (int64_t i = 0; i < n; ++i) cnt[i + 1] += cnt[i];
    int64_t* cur = (int64_t*)malloc(sizeof(int64_t) * (size_t)(n + 1));
    memcpy(cur, cnt, sizeof(int64_t) * (size_t)(n + 1));
    for (int64_t i = 0; i < np; ++i) perm[cur[xs[i]]++] = i;
    free(cur);
    int bad = 0;
#ifdef _OPENMP
    if (nthreads <= 0) nthreads = omp_get_max_threads();
#pragma omp parallel num_threads(nthreads) reduction(| : bad)
#endif
    {
        int8_t* dist = (int8_t*)malloc((size_t)n + 1);
        int32_t* visited = (int32_t*)malloc(sizeof(int32_t) * ((size_t)n + 1));
        memset(dist, -1, (size_t)n + 1);
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 1)
#endif
        for (int64_t x = 0; x < n; ++x) {
            if (cnt[x + 1] == cnt[x]) continue;
            int64_t nv = 0;
            int64_t h2 = bfs_exact(g, (int32_t)x, 2, dist, visited, &nv);
            for (int64_t k = cnt[x]; k < cnt[x + 1]; ++k) {
                int64_t p = perm[k];
                int32_t y = ys[p];
                uint32_t c = 0;
                unsigned __int128 s = 0; /* exact, units of 2^-58 */
                int64_t hop1 = g->deg[y] - g->self[y];
                for (int64_t e = g->rp[y]; e < g->rp[y + 1]; ++e) {
                    int32_t w = g->ci[e];
                    if (w == y) continue;
                    if (dist[w] == 2) {
                        ++c;
                        if (g->deg[w] > 1) s += (uint64_t)ldexp(pow(log((double)g->deg[w]), -1.0), 58);
                    }
                }
                if (mask & 1u) cn[p] = c;
                if (mask & 2u) {
                    int64_t uni = h2 + hop1 - (int64_t)c;
                    if (uni == 0) {
                        jac[p] = NAN;
                        bad = 1;
                    } else
                        jac[p] = (double)c / (double)uni;
                }
                if (mask & 4u) aa[p] = ldexp((double)s, -58); /* one rounding: nearest even */
                if (h2out) h2out[p] = (uint32_t)h2;
            }
            for (int64_t i = 0; i < nv; ++i) dist[visited[i]] = -1;
        }
        free(dist);
        free(visited);
    }
    free(cnt);
    free(perm);
    return bad ? 1 : 0;
}

/* Exact distance-3 sets for `nu` sources: counts[i] = |H3(users[i])|; when out != NULL
 * the members are written (ascending) at out[sum(counts[:i])] up to cap entries. */
int64_t og_hop3(const og_graph* g, int64_t nu, const int32_t* users, int64_t* counts, int32_t* out,
                int64_t cap) {
    int64_t n = g->n, total = 0;
    int8_t* dist = (int8_t*)malloc((size_t)n + 1);
    int32_t* visited = (int32_t*)malloc(sizeof(int32_t) * ((size_t)n + 1));
    int32_t* tmp = (int32_t*)malloc(sizeof(int32_t) * ((size_t)n + 1));
    memset(dist, -1, (size_t)n + 1);
    for (int64_t i = 0; i < nu; ++i) {
        int64_t nv = 0;
        int64_t c = bfs_exact(g, users[i], 3, dist, visited, &nv);
        counts[i] = c;
        if (out) {
            int64_t t = 0;
            for (int64_t j = nv - c; j < nv; ++j) tmp[t++] = visited[j];
            qsort(tmp, (size_t)t, sizeof(int32_t), cmp_i32); /* canonical ascending listing */
            for (int64_t j = 0; j < t && total + j < cap; ++j) out[total + j] = tmp[j];
        }
        total += c;
        for (int64_t j = 0; j < nv; ++j) dist[visited[j]] = -1;
    }
    free(dist);
    free(visited);
    free(tmp);
    return total;
}
