// Library-internal entry points shared between translation units (not part of the C ABI).
#pragma once

#include "ahr.h"

#include <stdint.h>

namespace ahr {

// ahr_index_query, except that when the plan is the small-batch stream and a query's per-split
// lists hold at most kRerankFuseKeys keys, no merge is launched: *lists = the [B][n_lists][k]
// sorted key lists (the index's workspace, valid until its next query), *n_lists set; scores /
// rows are then left for the caller's merge. Otherwise *lists = nullptr and scores / rows hold
// the merged top-k as ahr_index_query writes them. (ahr_dense.hip)
int dense_query_lists(ahr_index* ix, const float* q, int B, int k, int normalize_q, float* scores, int32_t* rows,
                      void* stream, const uint64_t** lists, int* n_lists);

// Whether a rerank of k_seed seeds under params runs on the wave kernel (the only one that can
// merge lists); the caller asks before dense_query_lists, since a large member_top_m or top_k (or
// AHR_RERANK_SERIAL=1) takes the serial kernel, which needs the merged top-k (ahr_graph.hip).
bool graph_rerank_fusable(int k_seed, const ahr_rerank_params* params);

// ahr_graph_expand_rerank_rows over those lists: the rerank wave kernel merges each query's lists
// first and writes the merged rows / scores to rows / scores (ahr_graph.hip).
int graph_rerank_lists(ahr_graph* g, const uint64_t* lists, int n_lists, int32_t* rows, const int32_t* row_to_node,
                       int64_t n_rows, float* scores, int B, int k_seed, const ahr_rerank_params* params,
                       int max_exp, int32_t* exp_nodes, double* exp_sem, int32_t* exp_src, int32_t* exp_count,
                       int32_t* out_nodes, double* out_sem, double* out_score, int32_t* out_count, void* stream);

}  // namespace ahr
