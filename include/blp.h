/*
 * blp.h — C-ABI of libblp.so, the MI355X-native bipartite link-scoring engine.
 *
 * Drop-in boundary for the reference's hot path. The reference has no
 * FFI of its own: its boundary is the Python module surface of similarity.py / svd.py /
 * random_walks.py plus the JSON score-file contract. The Python host modules in
 * bipartite-link-prediction_amd/ keep that surface and bind these entry points with ctypes
 * (see INTEGRATION.md). Every function below names the reference computation it replaces.
 *
 * Conventions
 *   - Plain pointers and sizes only; no torch / HIP types cross the ABI.
 *   - Return 0 on success, a negative code on failure (BLP_E_*; HIP errors are
 *     -1000 - hipError_t). blp_last_error() returns a thread-local message.
 *   - Host buffers passed in are read during the call only; the caller keeps ownership.
 *   - A graph handle owns its device memory and one HIP stream; calls on one handle are
 *     serialised by the caller (not re-entrant). One host thread per GPU may drive
 *     several handles concurrently.
 *   - Node ids are dense int32 in [0, n_nodes). The Python host maps the reference's
 *     integer node ids (SNAP TInt) to dense ids.
 *   - Methods are a bit mask: BLP_CN=1 (common_neighbors), BLP_JACCARD=2, BLP_ADAMIC=4.
 */
#ifndef BLP_H_
#define BLP_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BLP_OK 0
#define BLP_E_ARG (-1)      /* bad argument (null pointer, id out of range, size overflow) */
#define BLP_E_STATE (-2)    /* handle used in the wrong state */
#define BLP_E_NOMEM (-3)    /* host allocation failed */
#define BLP_E_UNSUP (-4)    /* configuration not supported by this build */
#define BLP_E_ZERODIV (-5)  /* Jaccard union of size 0 (reference raises ZeroDivisionError) */
#define BLP_E_COMM (-6)     /* a collective failed (RCCL error; blp_multi_*) */
#define BLP_E_HIP_BASE (-1000)

#define BLP_CN 1u
#define BLP_JACCARD 2u
#define BLP_ADAMIC 4u

typedef struct blp_graph blp_graph;
typedef struct blp_batch blp_batch;
typedef struct blp_svd blp_svd;
typedef struct blp_walk blp_walk;
typedef struct blp_topk blp_topk;

/* ---------------------------------------------------------------- runtime */
const char* blp_last_error(void);
const char* blp_version(void);
int blp_device_count(int* n);
int blp_device_sync(int device); /* hipDeviceSynchronize on `device` */
/* blp_stream_prewarm: create n (<= 16) non-blocking streams of `device` into the library's
 * stream pool, which the CSR build, the graph.txt parse, graph handles and pair batches draw
 * from instead of creating their own (a stream costs milliseconds to create): call it on a
 * spare thread while the inputs load (similarity.main does).                                  */
int blp_stream_prewarm(int device, int n);
/* blp_host_alloc / blp_host_free: host memory for large result arrays (fetched scores): from
 * 4 MiB on, an anonymous mapping advised as transparent huge pages (first touch and release
 * cost a fault / an unmap per 2 MiB, not per 4 KiB); malloc below that, or with BLP_NO_THP=1.
 * blp_host_free takes the size given to blp_host_alloc. Not pinned: any host pointer works with
 * the fetch entry points.                                                                   */
int blp_host_alloc(size_t bytes, void** out);
int blp_host_free(void* p, size_t bytes);

/* ---------------------------------------------------------------- graph
 * Replaces snap.LoadEdgeList(snap.PUNGraph, graph_file, 0, 1) (similarity.py:16) and the
 * per-node degree lookups G.GetNI(i).GetDeg() (similarity.py:121).
 *
 * blp_csr_from_edges: host helper. Builds the undirected simple-graph CSR of an edge list
 * over dense ids: both directions, duplicates removed, rows sorted ascending, self-loops
 * NOT stored in the CSR (they never change a BFS hop set) but flagged in self_loop[] because
 * SNAP's GetDeg counts a self-loop once. row_ptr has n_nodes+1 entries; col_idx must hold
 * 2*n_edges entries; *nnz_out receives the stored entry count.                           */
int blp_csr_from_edges(int64_t n_nodes, int64_t n_edges, const int32_t* a, const int32_t* b,
                       int64_t* row_ptr, int32_t* col_idx, uint8_t* self_loop, int64_t* nnz_out);

/* blp_csr_from_edges_device: the same CSR as blp_csr_from_edges (same outputs, host
 * buffers), built on device `device` from device-resident endpoints d_a/d_b (m edges, dense
 * ids) -- e.g. the edge list a rank holds after the RCCL all-gather of the row-block
 * partials (multi-GPU ingest). Radix sort of 64-bit (row, col) keys.      */
int blp_csr_from_edges_device(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n_nodes,
                              int64_t* row_ptr, int32_t* col_idx, uint8_t* self_loop, int64_t* nnz_out);

/* Device-resident CSR (multi-GPU ingest without a host round trip).
 * blp_csr_build_device: the same CSR as blp_csr_from_edges_device, kept in HBM in the layout
 *   blp_graph uses (row offsets int64, column ids int32, self-loop flags). It first waits for
 *   all work queued on `device` (the endpoints may come from the RCCL all-gather's stream).
 * blp_csr_info / blp_csr_fetch: sizes, and device-to-host copies (any pointer may be NULL).
 * blp_graph_create_from_csr: a graph handle over that device CSR (no upload). row_ptr /
 *   col_idx are the host mirror of the same CSR (from blp_csr_fetch); unlike
 *   blp_graph_create, the handle BORROWS them: the caller keeps them alive and unchanged
 *   until blp_graph_destroy. col_idx may be NULL: pair scoring plans on the device and never
 *   reads it, and the calls that do (hop-3 sampling, top-k create, host-planned batches) fetch
 *   their own copy from HBM on first use. On success the csr is consumed (do not destroy it); on failure
 *   it is left intact. aaw as for blp_graph_create.                                       */
typedef struct blp_csr blp_csr;
int blp_csr_build_device(int device, const int32_t* d_a, const int32_t* d_b, int64_t m, int64_t n_nodes,
                         blp_csr** out);
/* blp_csr_build_host: blp_csr_build_device from host-resident endpoints (uploaded first), e.g.
 * the dense ids of a parsed graph.txt: the single-GPU load path of DeviceGraph.            */
int blp_csr_build_host(int device, const int32_t* a, const int32_t* b, int64_t m, int64_t n_nodes, blp_csr** out);
int blp_csr_info(const blp_csr* c, int64_t* n_nodes, int64_t* nnz);
int blp_csr_fetch(const blp_csr* c, int64_t* row_ptr, int32_t* col_idx, uint8_t* self_loop);
int blp_csr_destroy(blp_csr* c);
int blp_graph_create_from_csr(blp_csr* c, const int64_t* row_ptr, const int32_t* col_idx, const double* aaw,
                              blp_graph** out);

/* ---------------------------------------------------------------- multi-GPU exchange (config 5)
 * The reference is single-process (snap.LoadEdgeList, similarity.py:16); its 1B-edge config is
 * this engine's row-block sharded ingest. These entry points are the exchange
 * step of blp/dist.py (allgather_edges + DeviceGraph.from_device_edges) with the engine's own
 * RCCL communicator, for hosts that do not run torch.distributed. One process per GPU.
 * blp_multi_unique_id: rank 0 creates the communicator id; the host ships its
 *   BLP_MULTI_ID_BYTES bytes to every rank over any channel (a file, a socket, MPI).
 * blp_multi_init: every rank joins with the same id (RCCL is loaded at run time: BLP_E_UNSUP
 *   when librccl.so.1 cannot be loaded; a failing collective returns BLP_E_COMM).
 * blp_multi_gather_csr: THE exchange. Each rank passes its edge partial (m_r endpoint pairs,
 *   dense ids in [0, n_nodes), host or device memory); the counts, then the partials padded to
 *   the largest count, are all-gathered over RCCL, the padding is dropped on the device and the
 *   union's CSR is built in HBM as blp_csr_build_device does. Every rank gets the same csr; feed
 *   it to blp_csr_fetch / blp_graph_create_from_csr. *bytes_in (may be NULL): bytes received
 *   from the other ranks. Collective: every rank must call it.
 * blp_multi_allreduce: *v = the sum (BLP_MULTI_SUM) or max (BLP_MULTI_MAX) of every rank's *v,
 *   e.g. the max-over-ranks step time. Collective.
 * blp_multi_compact_csr: the post-gather half of blp_multi_gather_csr on its own (not collective):
 *   recv (host or device) is an all-gather receive buffer of `world` slots, slot r = rank r's a
 *   ids then its b ids, each half padded to m_max = max(counts); counts[world] (host) are the
 *   valid prefixes. They are copied back to back on `device` (padding never read) and the
 *   union's CSR is built in HBM; *bytes_in (may be NULL) = 8 * m_max * (world - 1), what each
 *   rank received. For hosts that run the collective themselves, and for tests.              */
#define BLP_MULTI_ID_BYTES 128
#define BLP_MULTI_SUM 0
#define BLP_MULTI_MAX 1
typedef struct blp_multi blp_multi;
int blp_multi_unique_id(uint8_t* id);
int blp_multi_init(const uint8_t* id, int world, int rank, int device, blp_multi** out);
int blp_multi_info(const blp_multi* m, int* world, int* rank, int* device);
int blp_multi_gather_csr(blp_multi* m, const int32_t* a, const int32_t* b, int64_t m_r, int64_t n_nodes,
                         blp_csr** out, int64_t* bytes_in);
int blp_multi_allreduce(blp_multi* m, double* v, int op);
int blp_multi_compact_csr(int device, const int32_t* recv, const int64_t* counts, int world, int64_t n_nodes,
                          blp_csr** out, int64_t* bytes_in);
int blp_multi_destroy(blp_multi* m);

/* blp_edges_parse: SNAP LoadEdgeList's text format (similarity.py:16): one edge per line,
 * whitespace-separated integer columns c0 and c1, lines starting with '#' skipped, lines
 * with too few columns skipped. Two calls: with a == b == NULL it only counts (*m_out);
 * then call again with arrays of *m_out entries. Multi-threaded, reads the file once per
 * call (the OS page cache serves the second read).                                       */
int blp_edges_parse(const char* path, int c0, int c1, int64_t* a, int64_t* b, int64_t* m_out);

/* blp_edges_load: the same parse, once, into a handle, plus -- when the id space is compact
 * (max - min < 4 * edges or 2^20) -- the dense id map of the engine's graph (similarity.py:16
 * node ids; blp/graph.py HostGraph._ids): ids seen in column c0 ascending, then ids seen only
 * in column c1 ascending. blp_edges_info reports id_span == 0 when there is no map.
 * blp_edges_fetch copies any of: raw endpoints a / b (int64, file order), dense endpoints
 * da / db (int32), node_ids[n_nodes] (dense -> original id) and id_map[id_span] (original id
 * id_lo + i -> dense id or -1). blp_ids_lookup maps ids through id_map (-1: not in the graph),
 * the membership test of similarity.py:22-26 / :66-70. Host-only, multi-threaded.          */
typedef struct blp_edges blp_edges;
int blp_edges_load(const char* path, int c0, int c1, blp_edges** out);
int blp_edges_info(const blp_edges* e, int64_t* m, int64_t* n_nodes, int64_t* n_col0, int64_t* id_lo, int64_t* id_span);
int blp_edges_fetch(const blp_edges* e, int64_t* a, int64_t* b, int32_t* da, int32_t* db, int64_t* node_ids,
                    int32_t* id_map);
int blp_edges_destroy(blp_edges* e);
/* blp_edges_load_device: blp_edges_load with the parse and the id map on `device` when the file
 * is the reference's own graph.txt shape (dataset_maker.py:197: every line "digits ws digits",
 * optional trailing blanks / '\r', c0 = 0, c1 = 1, >= 1 MiB, compact id space): the text is
 * copied to HBM once and the dense endpoints stay there. Anything else is parsed on the host
 * exactly as blp_edges_load does. Same info / fetch / ids results either way.
 * blp_edges_device: *device = the device holding the dense endpoints, or -1 (host slices).
 * blp_edges_csr: the device CSR of the dense endpoints (as blp_csr_build_device; no upload when
 *   they are device-resident, which must then be on `device`).                              */
int blp_edges_load_device(const char* path, int c0, int c1, int device, blp_edges** out);
int blp_edges_device(const blp_edges* e, int* device);
int blp_edges_csr(const blp_edges* e, int device, blp_csr** out);
int blp_ids_lookup(const int32_t* id_map, int64_t id_lo, int64_t id_span, const int64_t* ids, int64_t n, int32_t* dense);

/* Upload a CSR (from blp_csr_from_edges or equivalent) to device `device`.
 * aa_weight[n_nodes]: per-node Adamic-Adar term, (log deg)^-1 for SNAP degree > 1 else 0,
 * computed by the caller with the reference's own arithmetic (similarity.py:121-125);
 * may be NULL when BLP_ADAMIC is never requested.                                        */
/* ---- score-file I/O of similarity.main (similarity.py:11-18; util.py:12-21) ----------------
 * blp_examples_parse: examples.json of the reference's shape -- {"user": {"business": label}},
 *   integer-valued keys without escapes, scalar labels, no duplicate keys -- into flat arrays
 *   (json.loads + the per-pair walk of similarity.py:22-32). Anything else is BLP_E_UNSUP: the
 *   caller then uses json.loads, so results never depend on which path ran.
 * blp_examples_ids: per-pair int(user key) / int(business key) (file order) and the pair
 *   offsets of each user ([n_users + 1]); any pointer may be NULL.
 * blp_scores_write: one score file with exactly the text json.dumps({u: {b: v}}) writes
 *   (util.py:18-21): keys as they appear in examples.json, values in file order. present[i]
 *   (NULL: all) marks pairs whose nodes are both in the graph; absent pairs get the int 0
 *   (similarity.py:59-60, 104-105). values holds one entry per PRESENT pair:
 *     BLP_SCORE_U32       uint32 counts, JSON ints (common_neighbors)
 *     BLP_SCORE_F64       doubles in Python repr (jaccard)
 *     BLP_SCORE_F64_INT0  doubles, 0.0 written as the int 0 (adamic_adar, similarity.py:118)
 *     BLP_SCORE_NONE      values unused: only absent pairs are written (a method string the
 *                         reference does not match, e.g. the b_adamic bug, similarity.py:102)
 *     BLP_SCORE_REPR24    values are 24-byte slots of already formatted text, NUL-padded
 *                         (blp_batch_fetch_repr / blp_repr_format: the doubles formatted on
 *                         the device) */
typedef struct blp_examples blp_examples;
#define BLP_SCORE_U32 0
#define BLP_SCORE_F64 1
#define BLP_SCORE_F64_INT0 2
#define BLP_SCORE_NONE 3
#define BLP_SCORE_REPR24 4
int blp_examples_parse(const char* path, blp_examples** out);
int blp_examples_info(const blp_examples* e, int64_t* n_users, int64_t* n_pairs);
int blp_examples_ids(const blp_examples* e, int64_t* pair_user, int64_t* pair_business, int64_t* user_off);
int blp_examples_destroy(blp_examples* e);
int blp_scores_write(const blp_examples* e, const char* path, int kind, const uint8_t* present, const void* values,
                     int64_t n_values);

int blp_graph_create(const int64_t* row_ptr, const int32_t* col_idx, int64_t n_nodes,
                     const double* aa_weight, int device, blp_graph** out);
int blp_graph_destroy(blp_graph* g);
/* blp_graph_wedge: the graph's wedge-row index (the short-row scorer's second layout: for
 * each node x whose neighbours' rows are all short, the rows N(z), z in N(x), back to back,
 * padded to whole 16-byte vectors with a repeat of the last id). *n_vecs = its size in vectors
 * (-1: not built); wp [n + 1] (vector offsets) and wedge [4 * n_vecs] may be NULL.         */
int blp_graph_wedge(const blp_graph* g, int64_t* n_vecs, int64_t* wp, int32_t* wedge);
int blp_graph_info(const blp_graph* g, int64_t* n_nodes, int64_t* nnz, int* device);
/* blp_graph_col_idx: the graph's column ids (nnz int32, the device CSR's) copied to `out`: the
 * host copy of a graph created from a device CSR without one (blp_graph_create_from_csr).   */
int blp_graph_col_idx(const blp_graph* g, int32_t* out);
int blp_graph_sync(blp_graph* g); /* wait for all work queued on the handle's stream */
/* Fixed-point scale of the Adamic-Adar terms: W = w * 2^shift with shift = 58, exact for every
 * weight the reference produces ((log d)^-1 in [2^-5, 2)); a pair's sum is carried exactly in
 * two 64-bit words and rounded once to the nearest double, i.e. the correctly rounded sum of
 * the reference's terms (math.fsum). aa_weight entries must lie in [0, 2) (else BLP_E_ARG).   */
int blp_graph_aa_shift(const blp_graph* g, int* shift);

/* ---------------------------------------------------------------- pair scoring
 * Replaces the hot loops of similarity.users (similarity.py:20-61) and similarity.business
 * (similarity.py:63-106): for each pair (x, y), with H2(x) = GetNodesAtHop(x, 2) (nodes at
 * exact BFS distance 2) and N(y) = GetNodesAtHop(y, 1):
 *   cn  = |H2(x) ∩ N(y)|                                    common_neighbors  (:113-114)
 *   jac = cn / |H2(x) ∪ N(y)|  (fp64, correctly rounded)    jaccard           (:108-111)
 *   aa  = Σ_{w ∈ H2(x) ∩ N(y)} aa_weight[w]                  adamic_adar       (:116-126)
 * User side (users()):  x = user, y = business.  Business side (business()): x = business,
 * y = user. Pairs whose node is absent from the graph never reach the engine (the host
 * writes the reference's 0, similarity.py:59-60,104-105).
 *
 * blp_score_pairs: one-shot (host in, host out; synchronous).
 *   side 0: x = pair_user, y = pair_business;  side 1: x = pair_business, y = pair_user.
 *   Output arrays may be NULL for methods not in `mask`.                                   */
int blp_score_pairs(blp_graph* g, int side, uint32_t mask, const int32_t* pair_user,
                    const int32_t* pair_business, int64_t n_pairs, uint32_t* cn, double* jac,
                    double* aa);

/* Device-resident batch (bench / repeated scoring). blp_batch_create copies the pairs to
 * HBM and plans the launch (bitmap universe, variant). blp_batch_score enqueues one full
 * pass on the batch's own stream (returns at once): group pairs by source on the device,
 * score, write results in the caller's pair order into device buffers. Batches of one graph
 * run concurrently (similarity.main's user and business passes overlap on the device).
 * blp_batch_fetch waits for the batch and copies results to the host; blp_device_sync waits
 * for every batch of the device. */
int blp_batch_create(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n_pairs,
                     blp_batch** out);
/* blp_batch_create_pair: both passes of similarity.main over one pair list -- *out_xy the
 * batch (x, y) (the user side), *out_yx the batch (y, x) (the business side) -- with ONE
 * host-to-device upload: the second batch copies the first's device arrays, swapped. Each
 * batch is then destroyed on its own (blp_batch_destroy).                                    */
int blp_batch_create_pair(blp_graph* g, const int32_t* x, const int32_t* y, int64_t n_pairs,
                          blp_batch** out_xy, blp_batch** out_yx);
int blp_batch_score(blp_graph* g, blp_batch* b, uint32_t mask);
int blp_batch_fetch(blp_graph* g, blp_batch* b, uint32_t* cn, double* jac, double* aa);
/* blp_batch_fetch_repr: the batch's Jaccard (which = BLP_JACCARD) or Adamic-Adar (BLP_ADAMIC)
 * scores as the text json.dumps writes for them (Python's repr: shortest round-trip digits),
 * formatted on the device into out[n_pairs][24] (NUL-padded slots, caller order); zero_int
 * writes 0.0 as the int 0 (adamic_adar, similarity.py:118). Replaces the host formatting of
 * util.write_json (util.py:18-21) for similarity.main's score files; BLP_E_ZERODIV as
 * blp_batch_fetch for an empty Jaccard union. */
int blp_batch_fetch_repr(blp_graph* g, blp_batch* b, int which, int zero_int, char* out);
/* The same formatting of n doubles: on the host (blp_repr_format; tests pin it against CPython's
 * repr) and of device-resident values on device `device` (blp_repr_format_device). */
int blp_repr_format(const double* values, int64_t n, int zero_int, char* out);
int blp_repr_format_device(int device, const double* d_values, int64_t n, int zero_int, char* d_out);
int blp_batch_destroy(blp_batch* b);
/* Enqueue blp_batch_score for n batches of one graph at once (one similarity.main step: the
 * user and the business pass). They run concurrently; a large-universe (user-side) batch is
 * held to a share of the CUs so the other passes run beside it rather than after it. */
int blp_batches_score(blp_graph* g, int n, blp_batch* const* batches, const uint32_t* masks);
/* Launch plan actually used: universe lo/hi (bitmap range), bitmap chunks, threads per
 * block, number of heavy sources pre-built across workgroups. For tests and DESIGN.md.     */
int blp_batch_plan(const blp_batch* b, int64_t* lo, int64_t* hi, int* chunks, int* block,
                   int* heavy);
/* Source routing of the plan: distinct sources, those on the hash-set scorer (chunk-parallel
 * batches; else 0), 1 if the pairs arrive grouped by source (run-head grouping), and 1 if long
 * sources copy the graph's wedge-row bitmaps as pre-built H2 sets (short-row batches).      */
int blp_batch_routes(const blp_batch* b, int64_t* n_sources, int64_t* n_hash, int* runs, int* wedge_bitmaps);
/* The scorer kernel blp_batch_score launches for this batch under `mask`, as its template
 * instance reads in a rocprofv3 trace (e.g. "k_score<1024, 31744, 896, 8, false, true, true>"),
 * NUL-terminated into name[cap]: what bench.py prices and looks up in the committed profiles. */
int blp_batch_kernel(const blp_batch* b, uint32_t mask, char* name, int cap);

/* Per-batch device time of the last/accumulated blp_batch_score calls (HIP events on the
 * batch stream): which 0 = scorer kernel, 1 = grouping kernels. Reset with blp_batch_stats_reset. */
int blp_batch_stats(blp_batch* b, int which, double* total_ms, int64_t* launches);
int blp_batch_stats_reset(blp_batch* b);

/* ---------------------------------------------------------------- candidate generation
 * Replaces dataset_maker.make_examples' candidate loop (dataset_maker.py:137-144): for each
 * source u in src[], every node at EXACT distance 3 (GetNodesAtHop(G,u,3), :139) is a
 * candidate; candidates listed in u's positives (pos_y[pos_off[i]:pos_off[i+1]], the held-out
 * new edges, :141-142) are emitted with label 1, the others are kept with probability `rate`
 * (:143-144) by a counter-based hash of (seed, u, b) and emitted with label 0.
 * Up to `cap` (x, y, label) triples are written; *n_out receives the total produced (call
 * again with a larger cap if *n_out > cap). Output order across sources is unspecified;
 * within a source: positives first, then negatives by ascending dense id.                   */
int blp_hop3_sample(blp_graph* g, const int32_t* src, int64_t n_src, const int32_t* pos_off,
                    const int32_t* pos_y, double rate, uint64_t seed, int32_t* out_x,
                    int32_t* out_y, uint8_t* out_label, int64_t cap, int64_t* n_out);

/* ---------------------------------------------------------------- full-candidate top-k
 * BASELINE.json configs[2] ("Jaccard + Adamic-Adar full-candidate top-k"; SURVEY.md §8(b)
 * blp_topk). The reference scores only the sampled pairs of examples.json; this scores, for
 * each source x, EVERY target b at exact distance 3 (the complete candidate set
 * GetNodesAtHop(G,x,3) that dataset_maker.py:139 samples from) with similarity.py's
 * common_neighbors / jaccard / adamic_adar of (H2(x), N(b)) (similarity.py:108-126, the
 * user-side orientation of :20-61) and keeps the k best per method: score descending, then
 * dense target id ascending. Scores are bit-identical to blp_score_pairs on the same pair.
 * The graph must be bipartite between [src_lo, src_hi) and [tgt_lo, tgt_hi) (BLP_E_UNSUP
 * otherwise); both ranges are dense ids (users / businesses of a reference graph.txt).
 *   blp_topk_create:      builds the degree-ordered target numbering, the permuted source rows
 *                         and (memory permitting) the expanded wedge rows; blp_topk_info
 *                         reports the counter chunks, tier sizes and wedge entries (-1: none).
 *   blp_topk_set_sources: uploads the sources (kept in HBM across runs) and plans the order the
 *     workgroups claim them in: largest two-hop walk first (BLP_TK_ORDER=0: list order). Results
 *     are indexed by the sources' list positions either way.
 *   blp_topk_run:         k in [1, 256], mask of BLP_CN | BLP_JACCARD | BLP_ADAMIC; async.
 *   blp_topk_fetch:       one method's [n_src][k] lists (col -1 / score 0 past the end) and
 *                         n_cand[i] = |H3(src[i])|, the number of candidates scored.
 *   blp_topk_stats:       which 0: kernel ms/launches; 1 / 2: sources whose Adamic-Adar took
 *                         the candidate-hash / direct-accumulation path (in *launches);
 *                         3: sum of |H2(x)|; 4: sum over x and w in H2(x) of |N(w)| (work);
 *                         5: sources whose AA lists came from the fused sums; 6: row entries the
 *                         count pass pushed (walk + dense corrections); 7: dense hot-target adds;
 *                         8: bytes one dense add reads (counts + fused AA words).                 */
int blp_topk_create(blp_graph* g, int64_t src_lo, int64_t src_hi, int64_t tgt_lo, int64_t tgt_hi,
                    blp_topk** out);
int blp_topk_destroy(blp_topk* t);
int blp_topk_info(const blp_topk* t, int64_t* n_chunks, int64_t* tier32, int64_t* tier16,
                  int64_t* wedge_entries);
int blp_topk_set_sources(blp_topk* t, const int32_t* src, int64_t n_src);
int blp_topk_run(blp_topk* t, int k, uint32_t mask);
int blp_topk_fetch(blp_topk* t, uint32_t method, int32_t* cols, double* scores, int64_t* n_cand);
int blp_topk_stats(blp_topk* t, int which, double* total_ms, int64_t* launches);
int blp_topk_stats_reset(blp_topk* t);

/* ---------------------------------------------------------------- truncated-SVD scorer
 * Replaces the reconstruction of svd.svd_user_business (svd.py:25-30): the host keeps the
 * reference's factorisation (svd.py:24, scipy ARPACK svds) and hands over us = u * s
 * (n_rows x k, row-major) and v = vt^T (n_cols x k, row-major), both fp64.
 *   blp_svd_score_pairs: out[i] = us[rows[i]] . v[cols[i]]       == np.dot(us[row], vt[:, col])
 *   blp_svd_topk:        for each selected user, the `topk` best columns over ALL businesses
 *                        (fp64 MFMA tiles, fused top-k; score descending then column ascending),
 *                        optionally skipping a per-user sorted exclusion list (ex_off/ex_col,
 *                        CSR over the selected users; NULL for none). Missing slots: col -1. */
int blp_svd_create(const double* us, int64_t n_rows, const double* v, int64_t n_cols, int k,
                   int device, blp_svd** out);
int blp_svd_destroy(blp_svd* h);
int blp_svd_score_pairs(blp_svd* h, const int32_t* rows, const int32_t* cols, int64_t n, double* out);
int blp_svd_score_pairs_device(blp_svd* h, const int32_t* d_rows, const int32_t* d_cols, int64_t n,
                               double* d_out);
int blp_svd_topk(blp_svd* h, const int32_t* users, int64_t n_users, const int64_t* ex_off,
                 const int32_t* ex_col, int topk, int32_t* out_cols, double* out_scores);
/* blp_svd_topk on device pointers (users, exclusion CSR or NULLs, outputs), enqueued on the
 * handle's stream without a sync (blp_svd_sync waits). Rows are not range-checked on the host;
 * the kernel treats a row outside [0, n_rows) as an all-zero row (no out-of-bounds read).
 * Ordering contract: the handle's stream is its own (non-blocking). A caller whose inputs
 * are produced on another stream, or who reads / frees the outputs on another stream, joins
 * the streams with blp_svd_stream_join: handle_waits = 1 makes the handle's stream wait for
 * the work queued so far on `stream` (call before blp_svd_topk_device); 0 makes `stream`
 * wait for the handle's work queued so far (call after). `stream` is a hipStream_t passed
 * as void* (NULL = the device's null stream). */
int blp_svd_topk_device(blp_svd* h, const int32_t* d_users, int64_t n_users, const int64_t* d_ex_off,
                        const int32_t* d_ex_col, int topk, int32_t* d_out_cols, double* d_out_scores);
int blp_svd_stream_join(blp_svd* h, void* stream, int handle_waits);
/* blp_svd_set_prune: top-k by norm pruning (on = 1, the default) or the dense pass (0). Both
 * give the same lists: a score is us[u] . v[b], so |score| <= ||us[u]|| ||v[b]||; with the
 * businesses in ||v|| descending order a block of 16 users stops once that bound falls strictly
 * below all its users' k-th scores. The dense pass reconstructs every (user, business) score.
 * blp_svd_tiles: MFMA tiles (16 users x 16 businesses) scored by the top-k calls since the last
 * call, and the tiles the dense pass would have scored over the same calls (then both reset). */
int blp_svd_set_prune(blp_svd* h, int on);
int blp_svd_tiles(blp_svd* h, int64_t* scored, int64_t* dense);
int blp_svd_stats(blp_svd* h, int which, double* total_ms, int64_t* launches); /* 0 pairs, 1 top-k */
int blp_svd_sync(blp_svd* h);

/* ---------------------------------------------------------------- truncated-SVD factorisation
 * Replaces scipy.sparse.linalg.svds(M, k) (svd.py:24) on a binary n_rows x n_cols CSR matrix:
 * block subspace iteration with Rayleigh-Ritz on a P-column fp64 block (P =
 * blp_fact_block_width(), 128). The device runs the SpMMs, Gram products and block updates;
 * the caller (blp.factor.svds) does the P x P Cholesky / eigen solves and the iteration
 * control. Blocks are row-major [rows][P] host arrays at the boundary.
 *   blp_fact_step:    Z = M Q, W = M^T Z, S = Q^T W (S returned, P x P)
 *   blp_fact_gram_w:  G = W^T W
 *   blp_fact_apply_w: W R -> Q (to_q) or back into W
 *   blp_fact_extract: us = Z V[:, :k] (= U S), v = Q V[:, :k]                             */
typedef struct blp_fact blp_fact;
int blp_fact_create(const int64_t* row_ptr, const int32_t* col_idx, int64_t n_rows, int64_t n_cols, int device,
                    blp_fact** out);
int blp_fact_destroy(blp_fact* f);
int blp_fact_block_width(void);
int blp_fact_set_q(blp_fact* f, const double* q);
int blp_fact_step(blp_fact* f, double* S);
int blp_fact_gram_w(blp_fact* f, double* G);
int blp_fact_apply_w(blp_fact* f, const double* R, int to_q);
int blp_fact_extract(blp_fact* f, const double* V, int k, double* us, double* v);
int blp_fact_stats(blp_fact* f, int which, double* total_ms, int64_t* launches); /* 0 SpMM, 1 dense */

/* ---------------------------------------------------------------- damped random walks
 * Replaces random_walks.run_random_walk(s) (random_walks.py:9-53): p <- scale * (p . T) for
 * `iterations` steps from e_start (the reference: scale = 1 - jump_p = 0.8, 10 steps).
 * The matrix is handed over as W = T^T in CSR (row j: entries T[i, j] for every i), so a step
 * is p'[j] = scale * sum_e W[j, e] p[col e]. blp_walk_run walks many starts (32 at a time)
 * and returns q_out[k] = p_{q_start[k]}[q_node[k]]; queries grouped by start.            */
int blp_walk_create(const int64_t* row_ptr, const int32_t* col, const double* val, int64_t n,
                    int device, blp_walk** out);
int blp_walk_destroy(blp_walk* w);
int blp_walk_run(blp_walk* w, const int32_t* starts, int64_t n_starts, int iterations, double scale,
                 const int32_t* q_start, const int32_t* q_node, int64_t n_q, double* q_out);
int blp_walk_run_dense(blp_walk* w, int32_t start, int iterations, double scale, double* p_out);
int blp_walk_stats(blp_walk* w, double* total_ms, int64_t* launches);

/* ---------------------------------------------------------------- stats
 * Per-kernel device time (ms, HIP events on the handle's stream) accumulated since the
 * last reset, for bench.py's roofline figure. kernel: 0 = pair scorer, 1 = grouping
 * (count+scan+scatter), 2 = svd pairs, 3 = svd dense top-k, 4 = random walk, 5 = hop-3. */
int blp_stats_reset(blp_graph* g);
int blp_stats_get(blp_graph* g, int kernel, double* total_ms, int64_t* launches);

#ifdef __cplusplus
}
#endif
#endif /* BLP_H_ */
