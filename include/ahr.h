/*
 * ahr.h — C ABI of libahr_hip.so, the MI355X (gfx950) dense-retrieval + graph-expansion core
 * behind AH-RAG's Python call surface.
 *
 * The reference (Yaron9/AH-RAG, pure Python) has no native code of its own; its hot path calls
 * into third-party objects. Each entry point below names the reference call site it replaces:
 *
 *   ChromaDB collection  (un-vendored HNSW index, cosine space)
 *     coll.upsert(ids, embeddings, ...)      src/ah_rag/graph/hierarchical_graph.py:660
 *     coll.query(query_embeddings, n_results) src/ah_rag/graph/hierarchical_graph.py:714
 *     client.delete_collection / reset        src/ah_rag/graph/hierarchical_graph.py:606-610
 *   networkx neighbour scans
 *     HierarchicalGraph._neighbors_by_edge_type     hierarchical_graph.py:441-453
 *     search(): 1-hop expansion + rerank            hierarchical_graph.py:726-782
 *     GraphEnvironment.expand_{children,parents,related}  src/ah_rag/agent/environment.py:393-480
 *
 * Conventions
 *   - Every function returns an int status: AHR_OK (0) or a negative AHR_E* code;
 *     ahr_last_error() returns a thread-local message for the last failure.
 *   - Pointers documented as "device" are HIP device pointers on the handle's device.
 *     Host pointers are only read during the call.
 *   - `stream` is a hipStream_t passed as void* (NULL = the legacy default stream).
 *     All work is enqueued on it; nothing synchronises unless stated.
 *   - Handles own their device memory. A handle is thread-compatible, not thread-safe.
 *   - Launch functions allocate nothing once ahr_index_reserve() covered the batch,
 *     so they may be captured into a hipGraph.
 */
#ifndef AHR_H_
#define AHR_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AHR_ABI_VERSION 1

enum ahr_status {
  AHR_OK = 0,
  AHR_EINVAL = -1,   /* bad argument / shape */
  AHR_ENOMEM = -2,   /* device allocation failed */
  AHR_EHIP = -3,     /* HIP runtime error */
  AHR_EUNSUP = -4,   /* unsupported parameter (e.g. k above the kernel's cap) */
  AHR_ERANGE = -5    /* slot / node index out of range */
};

enum ahr_dtype {
  AHR_F32 = 0,   /* exact mode: scores are a k-ordered fp32 fma chain (bit-exact vs oracle) */
  AHR_F16 = 1,
  AHR_BF16 = 2
};

/* Largest k the fused kernels serve (Chroma n_results); ahr_index_query / _query_keys accept k up
 * to AHR_MAX_K_LARGE through a two-step path (every score of a chunk of queries, then an exact
 * radix select + bitonic sort per query, same tie rule); ahr_topk_merge likewise (k or k_in
 * above AHR_MAX_K: a radix select over the packed keys). */
#define AHR_MAX_K 32
#define AHR_MAX_K_LARGE 4096

int ahr_abi_version(void);
const char* ahr_last_error(void);
int ahr_device_count(int* n);

/* ------------------------------------------------------------------------------------------
 * Dense index: row-major [capacity][dim] embedding matrix resident in HBM.
 * Rows [0, count) are live. Scores are inner products of the stored rows with the queries;
 * with L2-normalised rows and queries (normalize=1, the reference's normalize_embeddings=True)
 * the score is the cosine similarity, i.e. 1 - Chroma's cosine distance.
 * ---------------------------------------------------------------------------------------- */
typedef struct ahr_index ahr_index;

/* Replaces chromadb.PersistentClient(...).get_or_create_collection("nodes", {"hnsw:space":"cosine"})
 * (hierarchical_graph.py:605-611). */
int ahr_index_create(int dim, int dtype, int64_t capacity, int device, ahr_index** out);
int ahr_index_destroy(ahr_index* ix);

/* Replaces coll.upsert(ids, embeddings=...) (hierarchical_graph.py:660).
 * vecs: device fp32 [n][dim]. slots: device int64 [n] target rows, or NULL for the contiguous
 * rows [start_slot, start_slot+n). Rows past the current count extend it; the live range must
 * stay dense (every slot < count is written). normalize=1 L2-normalises each row first. */
int ahr_index_upsert(ahr_index* ix, const float* vecs, int64_t n, const int64_t* slots,
                     int64_t start_slot, int normalize, void* stream);

/* Replaces client.delete_collection (hierarchical_graph.py:606-610): count := new_count. */
int ahr_index_truncate(ahr_index* ix, int64_t new_count);
int ahr_index_count(const ahr_index* ix, int64_t* count);
int ahr_index_info(const ahr_index* ix, int* dim, int* dtype, int64_t* capacity,
                   int* padded_dim, int64_t* row_bytes);
/* Device pointer to the stored (padded, possibly permuted) rows, for tests / persistence. */
int ahr_index_rows(const ahr_index* ix, const void** dev_rows);

/* Decode stored rows [start, start+n) back to fp32 [n][dim] (device), undoing padding and the
 * fp32 lane permutation. Used to persist the index next to the graph (SURVEY §8b on-disk). */
int ahr_index_read(const ahr_index* ix, int64_t start, int64_t n, float* out, void* stream);

/* Stage timing with HIP events recorded on each query call's stream. Stages:
 * 0 query conversion, 1 threshold pre-pass, 2 fused tile kernel, 3 cross-split merge.
 * begin: arm for up to max_calls calls; end: wait, return per-stage sums (ms) and the call count. */
int ahr_index_profile_begin(ahr_index* ix, int max_calls);
int ahr_index_profile_end(ahr_index* ix, float* stage_ms_sum /* [4] */, int* n_calls);

/* Rows scored by the threshold pre-pass: -1 = automatic (default: 8192; 16384 from 512k, 32768 from 2M rows),
 * 0 disables it, else a power of two in [256, 65536]. */
int ahr_index_set_sample_rows(ahr_index* ix, int rows);
/* Caller-supplied admission thresholds (device pointer to >= B floats, one per query of the next
 * queries; NULL restores the built-in pre-pass). Each value must be a valid lower bound of that
 * query's final k-th best score as this index computes it (e.g. the k-th best over any k rows,
 * less a rounding margin): the fused kernels then skip the threshold pre-pass. B > 16 plans only
 * (the small-batch kernels use no threshold). Replaces nothing in the reference (Chroma has no
 * such knob); it is how a coarse-cluster probe seeds the exact search. */
int ahr_index_set_seed(ahr_index* ix, const float* thr);

/* Cluster-probe seeds for ahr_index_set_seed (bf16 / f16 indexes, dim <= 1024, P <= 64, k <= 256,
 * at most 256 rows per query): per query b, the
 * rows of clusters key_row(cluster_keys[b][0..P)) (the packed keys of a top-P search over the
 * cluster centroids; 0 = none), taken from the CSR list_rows[list_off[c] .. list_off[c+1]) in
 * order until min_rows rows, scored exactly in fp32 against the fp32 query (normalised if
 * normalize_q); thr[b] = the k-th largest of score - err (err bounds the difference from the
 * fused kernels' score of that row), or -inf when fewer than k rows exist. Slots >= the row
 * count are skipped, so lists built before later upserts or truncation stay valid (a stale list
 * only weakens the seed). All pointers are device pointers; stream-ordered. */
int ahr_index_probe_seed(ahr_index* ix, const float* q, int B, int k, int normalize_q, const uint64_t* cluster_keys,
                         int P, const int64_t* list_off, const int32_t* list_rows, int min_rows, float* thr,
                         void* stream);

/* Kernel-selection switches (A/B measurements; results stay correct), a 32-bit unsigned flag word:
 * 4 = qres256's split 0 seeds under a tag no launch has, so every bounded seeding wait on it runs
 * to its time limit (a test of that path), 8 = always the 128x128 tile kernel with cooperative
 * screening, 32 = the 128x128 lane-local tile kernel at any batch (k <= 16), 2048 = no
 * query-resident kernel (qkv or qres256), 16384 = tilelane without the cross-tile prefetch, 32768 =
 * the 256x256 16x16x32 kernel, 131072 = the k-blocked 256x256 kernel wherever it applies, 262144 =
 * never the k-blocked kernel, 1 << 19 = qres256 splits never XCD-balanced, 8192 = small batches
 * (B <= 4) merge in the kernel's last workgroup (the fold) instead of the merge launch (the default
 * since round 5), 1 << 22 = the merge launch even with 8192 set, 1 << 23 = the 256-query
 * register-resident kernel (qres256) wherever it applies (bf16/f16, d_pad 384 or 768, k <= 12),
 * 1 << 26 = qres256 seeded by the sampled pre-pass launch instead of seeding itself, 1 << 27 =
 * qres256's self-seeding with its first event only (no later rounds), 1 << 28 = qres256 splits
 * XCD-balanced at any corpus size (default: from 256 row blocks per split).
 * Accepted only by the ablation build (-DAHR_ABLATION, __graft_entry__.build_ablation; the shipped
 * library returns AHR_EUNSUP): 4096 = the 128-query-resident kernel (qkv) wherever it applies, and
 * the cost-split switches that give WRONG results (2 = skip the top-k epilogue, 256 = group maxima
 * only, 512 = operands of the first tile only, 1024 = loads never waited for, 1048576 / 2097152 =
 * k-blocked tiles read from tile 0 / the split's first tile, 1 << 24 / 1 << 25 = qres256 without
 * stage barriers / LDS fragment reads, 1 << 29 = qres256 per-workgroup timestamps, 1 << 30 /
 * 1 << 31 = qres256 seeding events without the selection / without the landing reads).
 * Unknown bits return AHR_EINVAL. */
int ahr_index_set_debug_flags(ahr_index* ix, uint32_t flags);

/* Launch geometry the next query of batch B, top-k would use (diagnostics / bench reporting).
 * *kernel: 0 = 128x128 tile kernel (cooperative screening; k > 16), 1 = 256x256 lane kernel
 * (k <= 16, B >= 6144), 3 = 128x128 lane-local tile kernel (k <= 16, B < 6144), 5 = query-resident
 * kernel (ablation build only), 6 = 256x256 16x16x32 kernel (opt-in), 7 = small-batch streaming kernel
 * (bf16/f16, B <= 16, k <= 16), 8 = k-blocked 256x256 kernel (bf16/f16, k <= 16, from 512k corpus
 * rows, below the register-resident kernel's batches), 10 = 256-query register-resident kernel
 * (bf16/f16, d_pad 384 or 768, k <= 12, B >= 512, from 32k rows; from 512k rows only where it seeds
 * itself: >= 32 splits, i.e. B <= 2048). Ids 2, 4 and 9 are retired. */
int ahr_index_plan(const ahr_index* ix, int B, int k, int* kernel, int* n_splits, int* tiles_per_split,
                   int* qblocks);

/* Pre-size the per-query workspace so ahr_index_query() allocates nothing (graph-capturable). */
int ahr_index_reserve(ahr_index* ix, int max_batch, int max_k);

/* Select the query workspace (0..3; default 0) that the following ahr_index_query /
 * ahr_index_query_keys / ahr_index_reserve calls use: the converted queries, per-split partial
 * lists and pre-pass buffers. Calls on different workspaces may run concurrently on different
 * streams (a serving loop keeping several batches in flight); calls on one workspace must be
 * ordered on one stream. Exception: batches of the register-resident plan (kernel id 10) fill every
 * CU and their first seeding event waits (bounded) for every split, so the library serializes them
 * across streams itself (each waits for the previous such batch's merge on another stream); under
 * hipGraph capture that cross-stream ordering is not recorded (the captured graph orders its own
 * batches). No reference counterpart (the reference is one synchronous call). */
int ahr_index_set_workspace(ahr_index* ix, int slot);

/* Replaces coll.query(query_embeddings=[q], n_results=k) (hierarchical_graph.py:714), batched.
 * q: device fp32 [B][dim]; scores: device fp32 [B][k] (descending); rows: device int32 [B][k].
 * Ties order by row ascending. If fewer than k live rows exist the tail is (-inf, -1).
 * normalize_q=1 L2-normalises the queries first. */
int ahr_index_query(ahr_index* ix, const float* q, int B, int k, int normalize_q,
                    float* scores, int32_t* rows, void* stream);

/* Same search, but emits packed 64-bit sort keys (ordered score << 32 | ~row) for rows offset
 * by row_base, so shards can all-gather and merge: keys device uint64 [B][k]. */
int ahr_index_query_keys(ahr_index* ix, const float* q, int B, int k, int normalize_q,
                         int64_t row_base, uint64_t* keys, void* stream);

/* Every score: out[b][r] = <q_b, row r> for the live rows r < count (device fp32, row pitch ld >=
 * count), the fused tile kernel's GEMM core in scores mode (fp32 index: each score the k-ordered
 * fma chain). Replaces the all-pairs np.dot loop of the L1 relation builder
 * (src/ah_rag/aggregate/semantic_aggregator.py:620-661) with one device pass. */
int ahr_index_scores(ahr_index* ix, const float* q, int B, int normalize_q, float* out, int64_t ld,
                     void* stream);

/* Merge n_lists descending key lists per query: keys_in device [B][n_lists][k_in] ->
 * top k as scores/rows (and optionally keys_out [B][k]). Used for the cross-shard merge
 * after the RCCL all-gather. */
int ahr_topk_merge(const uint64_t* keys_in, int B, int n_lists, int k_in, int k,
                   float* scores, int32_t* rows, uint64_t* keys_out, void* stream);

/* Decode keys -> (score, row); host-side helper mirrors the device format. */
int ahr_key_decode(const uint64_t* keys, int64_t n, float* scores, int64_t* rows);

/* ------------------------------------------------------------------------------------------
 * Graph: per-edge-type CSR adjacency + node attribute table resident in HBM.
 * ---------------------------------------------------------------------------------------- */
typedef struct ahr_graph ahr_graph;

enum ahr_node_type { AHR_NODE_OTHER = 0, AHR_NODE_ENTITY = 1, AHR_NODE_SUMMARY = 2,
                     AHR_NODE_HYPEREDGE = 3 };

/* Adjacency lists, each a CSR (offsets [n_nodes+1], targets [nnz]) in the order networkx
 * iterates neighbours of the live graph (G._succ / G._pred; for a graph that went through
 * save/load that is the order of hierarchical_graph.py:191-202):
 *   0 belongs_to out   (entity -> summaries, get_belongs_to)
 *   1 belongs_to in    (summary <- members, get_summary_members)
 *   2 related_to out   3 related_to in
 *   4 participates_in out (entity -> hyperedges)   5 participates_in in (hyperedge <- entities)
 * All arrays are host pointers and are copied to the device.
 * judge / confidence: NaN encodes Python None. judge_term / conf_term are the rerank terms
 * 1/(1+exp(-(judge/10))) and conf/10 (hierarchical_graph.py:766-767), computed by the caller with
 * the reference's own float64 arithmetic so the device score matches bit for bit. */
#define AHR_ADJ_COUNT 6
int ahr_graph_create(int64_t n_nodes, const int8_t* node_type, const double* judge,
                     const double* confidence, const double* judge_term, const double* conf_term,
                     const int64_t* const* offsets, const int32_t* const* targets, int device,
                     ahr_graph** out);
int ahr_graph_destroy(ahr_graph* g);

/* Search parameters, hierarchical_graph.py:682-699. */
typedef struct ahr_rerank_params {
  double alpha, beta, gamma, delta;
  double judge_min;       /* NaN = no filter */
  double confidence_min;  /* NaN = no filter */
  double layer_boost[4];  /* indexed by ahr_node_type */
  int type_mask;          /* bit t set = node type t allowed; 0 = no filter */
  int member_top_m;
  int top_k;
} ahr_rerank_params;

/* Batched search() tail: seeds -> 1-hop expansion -> rerank (hierarchical_graph.py:726-782).
 * seed_nodes: device int32 [B][k_seed] (-1 = absent; >= n_nodes = id unknown to the graph);
 * seed_sem: device fp32 [B][k_seed], the dense scores; the kernel forms the reference's
 *   semantic = 1.0 - double(dist) from Chroma's float32 cosine distance dist = 1.0f - score.
 * Outputs (device, per query q):
 *   exp_nodes/exp_sem/exp_src [B][max_exp], exp_count [B]: the `expanded` dict in insertion
 *     order; exp_src = seed index (entry owned by a seed) or -1 - assumed_node_type (added by
 *     expansion with meta {"expanded": True});
 *   out_nodes/out_sem/out_score [B][top_k], out_count [B]: `reranked`, with out_sem and
 *     out_score rounded to 4 decimals exactly like Python round(x, 4), stable-sorted on the
 *     rounded score.
 * max_exp must be >= k_seed * (1 + max(2, member_top_m)). */
int ahr_graph_expand_rerank(ahr_graph* g, const int32_t* seed_nodes, const float* seed_sem,
                            int B, int k_seed, const ahr_rerank_params* params, int max_exp,
                            int32_t* exp_nodes, double* exp_sem, int32_t* exp_src,
                            int32_t* exp_count, int32_t* out_nodes, double* out_sem,
                            double* out_score, int32_t* out_count, void* stream);

/* The same, fed straight from ahr_index_query's rows: seed b,s is node row_to_node[rows[b][s]]
 * (rows[b][s] < 0 or >= n_rows: absent), the search path's row -> node gather folded into the
 * kernel (hierarchical_graph.py:714-726: Chroma ids -> graph nodes). row_to_node: device int32
 * [n_rows] (>= n_nodes = id unknown to the graph). */
int ahr_graph_expand_rerank_rows(ahr_graph* g, const int32_t* rows, const int32_t* row_to_node,
                                 int64_t n_rows, const float* seed_sem, int B, int k_seed,
                                 const ahr_rerank_params* params, int max_exp, int32_t* exp_nodes,
                                 double* exp_sem, int32_t* exp_src, int32_t* exp_count,
                                 int32_t* out_nodes, double* out_sem, double* out_score,
                                 int32_t* out_count, void* stream);

/* The whole drop-in search() of a small host query batch in ONE call (hierarchical_graph.py:
 * 709-789 after the encode: Chroma query :714, distance -> similarity :719-724, expansion and
 * rerank :726-782): copy the fp32 queries in, ahr_index_query (top k_dense), expansion + rerank
 * fed by its rows (ahr_graph_expand_rerank_rows), copy every result back into one host buffer,
 * wait for the stream. One foreign-function call instead of one per stage.
 * Layout (ahr_search_layout, host-only arithmetic): the device workspace ws holds the queries
 * [B][dim] f32 at offset 0 (its part rounded up to 256 B), then the result arena; host_out
 * receives the arena: scores f32 [B][k_dense], rows i32 [B][k_dense], exp_nodes i32 [B][max_exp],
 * exp_sem f64 [B][max_exp], exp_src i32 [B][max_exp], exp_count i32 [B], out_nodes i32 [B][kk],
 * out_sem f64 [B][kk], out_score f64 [B][kk], out_count i32 [B] (kk = max(params->top_k, 1)),
 * each part starting at an 8-B aligned offset (offsets[0..9], relative to the arena).
 * host_q / host_out should be pinned (asynchronous copies); pageable memory works, slower.
 * max_exp must be >= k_dense * (1 + max(2, member_top_m)). */
int ahr_search_layout(int B, int dim, int k_dense, int max_exp, int kk, int64_t offsets[10],
                      int64_t* ws_bytes, int64_t* arena_bytes);
int ahr_search_host(ahr_index* ix, ahr_graph* g, const float* host_q, int B, int k_dense,
                    const int32_t* row_to_node, int64_t n_rows, const ahr_rerank_params* params,
                    int max_exp, void* ws, int64_t ws_bytes, void* host_out, void* stream);

/* Batched environment expansions (environment.py:393-480).
 * action: 0 expand_parents, 1 expand_children, 2 expand_related.
 * inputs: device int32 [B][n_in] (-1 = absent / not in graph); out: device int32 [B][limit],
 * out_count [B]. Reproduces the reference's per-input early break (>= limit after an input
 * node's neighbours were appended), first-occurrence dedupe and truncation to limit. */
int ahr_graph_expand(ahr_graph* g, int action, const int32_t* inputs, int B, int n_in,
                     int limit, int32_t* out, int32_t* out_count, void* stream);

/* ahr_graph_expand from host memory to host memory in one call (the single environment's step,
 * environment.py:393-480 one query at a time): copies host_inputs [B][n_in] into the device
 * workspace, expands, copies out [B][max(limit, 1)] and out_count [B] back into host_out /
 * host_count and waits for the stream. ws: device memory of at least the *bytes that
 * ahr_graph_expand_ws_bytes(B, n_in, limit, &bytes) returns (host-only arithmetic). Host buffers should be pinned (hipHostMalloc / torch pin_memory) for
 * asynchronous copies; pageable ones work, slower. Small batches (B * n_in <= 16, limit <= 32)
 * with pinned outputs take one launch and no copies: the inputs travel as kernel arguments and the
 * kernel stores the results into the pinned buffers (the single environment's expansion). */
int ahr_graph_expand_ws_bytes(int B, int n_in, int limit, int64_t* bytes);
int ahr_graph_expand_host(ahr_graph* g, int action, const int32_t* host_inputs, int B, int n_in,
                          int limit, int32_t* host_out, int32_t* host_count, void* ws, int64_t ws_bytes,
                          void* stream);

/* One step of E vectorised RL environments with their state in device memory (VecAHRAGGymEnv;
 * gym_env.py:77-125 over environment.py:301-355 commit / details and :393-480 expansions): per
 * environment, action 0-2 expands the current selection's top 2 / 2 / 1 graph nodes (limit
 * `limit`; the observation shows the expansion and the frontier before its ids join it), 3 commits
 * the top 3 (graph nodes not yet selected join the selection and leave the frontier), 4 shows the
 * top node's details, anything else (end, invalid, details of an empty selection) keeps the
 * previous observation. The workspace ws (int32, ahr_graph_env_layout's 16 parts, each 256-B
 * aligned; host-only arithmetic) holds, in order: actions [E] (in), the selection sel [E][K] and
 * sel_n [E] (in: the current observation's, out: the new one's), frontier F [E][fcap] (-1 =
 * removed), F_end [E] (slots used), F_n [E], selection set S [E][scap], S_n [E], then the
 * observation outputs kind [E] (1 expansion, 2 commit, 3 details, -1 the previous observation),
 * seed_n [E], f_shown [E] (the frontier slots the observation shows), f_size [E], s_size [E], the
 * environments' step counters step [E], the observations' featurizer vectors vec [E][4 + 8 K] (fp32
 * bits, featurizer.py:21-56; written for a new observation when node_feats is given: fp32 [n_feat][6]
 * = is_entity, is_summary, is_other, layer, judge_overall, confidence per extended node index),
 * and err [1] (set to 1 when a frontier or selection would overflow its capacity: grow and retry
 * from saved state). Needs 3 <= K, limit <= K and limit <= 32. Enqueued on `stream`. */
int ahr_graph_env_layout(int E, int K, int fcap, int scap, int64_t offsets[16], int64_t* bytes);
int ahr_graph_env_step(ahr_graph* g, int E, int K, int fcap, int scap, int limit, const float* node_feats,
                       int64_t n_feat, void* ws, int64_t ws_bytes, void* stream);
/* The same from the host in one call: host_actions [E] int32 are copied into the workspace, the step
 * runs, the whole workspace (state and observation outputs) is copied back into host_out (int32,
 * the layout's bytes) and the stream is waited for. Host buffers should be pinned. */
int ahr_graph_env_step_host(ahr_graph* g, int E, int K, int fcap, int scap, int limit, const float* node_feats,
                            int64_t n_feat, const int32_t* host_actions, void* ws, int64_t ws_bytes, int32_t* host_out,
                            void* stream);

/* Batched GraphEnvironment.expand_to_lca (environment.py:243-299): per query the nodes of the
 * intersection of the inputs' "ancestors or self" sets on the belongs_to DAG (nx.ancestors: nodes
 * with a belongs_to path to the input) that have no belongs_to out-edge to another member.
 * inputs: device int32 [B][n_in] node indices, -1 = padding (queries of fewer inputs; a query
 *   with no input has an empty result);
 * out: device int32 [B][max_out] (unordered), out_count [B] (-1: the query exceeded the kernel's
 * per-query capacity of 4096 visited nodes / 1024 per BFS level, or max_out). The caller sorts
 * by (level, id) and truncates (:289), and checks acyclicity once per graph version. */
int ahr_graph_lca(ahr_graph* g, const int32_t* inputs, int B, int n_in, int max_out, int32_t* out,
                  int32_t* out_count, void* stream);

/* The same computation without per-query capacity limits, for the queries ahr_graph_lca reported
 * as over capacity (count -1 with max_out large enough): the visited set and frontiers live in a
 * caller-owned device workspace of ahr_graph_lca_workspace(B) bytes (5 * n_nodes int32 per query,
 * cleared by the kernel itself). out_count is -1 only when max_out is too small (max_out =
 * n_nodes never is). Same reference semantics (environment.py:243-289). */
int ahr_graph_lca_workspace(const ahr_graph* g, int B, int64_t* bytes);
int ahr_graph_lca_large(ahr_graph* g, const int32_t* inputs, int B, int n_in, int max_out, int32_t* out,
                        int32_t* out_count, void* workspace, int64_t workspace_bytes, void* stream);

int ahr_graph_info(const ahr_graph* g, int64_t* n_nodes, int64_t* n_edges);

#ifdef __cplusplus
}
#endif
#endif  /* AHR_H_ */
