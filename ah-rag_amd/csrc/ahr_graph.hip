// ahr_graph.hip — device graph (per-edge-type CSR + node attribute table) and the two graph
// passes of the hot path, batched over queries / environments:
//
//   expand_rerank_kernel  HierarchicalGraph.search after the dense step
//                         (reference src/ah_rag/graph/hierarchical_graph.py:719-782):
//                         seeds -> 1-hop expansion (belongs_to parents / members) -> rerank ->
//                         stable sort on the 4-decimal rounded score -> top_k.
//   lca_kernel            GraphEnvironment.expand_to_lca (environment.py:243-299): ancestor sets
//                         on the belongs_to DAG by level-synchronous reverse BFS, intersected.
//   expand_kernel         GraphEnvironment.expand_{parents,children,related}
//                         (reference src/ah_rag/agent/environment.py:393-480), incl. the 2-hop
//                         entity -> hyperedge -> co-participant walk of expand_related.
//
// Both are pointer-chasing integer work bounded by a handful of neighbours per query, so one
// thread owns one query/environment and walks its CSR rows; B queries fill the device.
// Layout in HBM: node_type int8 [n], judge/conf/judge_term/conf_term f64 [n] (NaN = None),
// 6 CSR lists (int64 offsets [n+1], int32 targets [nnz]) in networkx iteration order.
#include "ahr_common.h"
#include "ahr_dense_common.h"
#include "ahr_internal.h"
#include "ahr.h"

#include <math.h>
#include <cstdlib>
#include <cstring>
#include <vector>

// The rerank reproduces CPython's float64 arithmetic bit for bit: every multiply and add rounds on
// its own, as in `alpha*sem + beta*jt + ...` evaluated by the interpreter. hipcc contracts a*b + c
// into one fma by default for device code, which rounds once and can move round(x, 4) across a
// half-way point; switch contraction off for this whole translation unit (explicit fma() calls,
// like py_round4's TwoProduct, are unaffected).
#pragma clang fp contract(off)

namespace ahr {
namespace graph {

enum { ADJ_BT_OUT = 0, ADJ_BT_IN = 1, ADJ_REL_OUT = 2, ADJ_REL_IN = 3, ADJ_PI_OUT = 4, ADJ_PI_IN = 5 };

struct DevGraph {
  int64_t n_nodes;
  const int8_t* type;
  const double* judge;       // NaN = None
  const double* conf;        // NaN = None
  const double* judge_term;  // 1/(1+exp(-judge/10)) computed host-side exactly as the reference
  const double* conf_term;   // conf/10
  const int64_t* off[AHR_ADJ_COUNT];
  const int32_t* tgt[AHR_ADJ_COUNT];
};

// Python's round(x, 4) for a double, exactly: the decimal rounding (half to even) of the exact
// binary value of x, then the nearest double to that decimal (CPython float.__round__ via
// dtoa). t = x * 10^4 is held exactly as hi + lo (TwoProduct), so the half-way test is exact.
__device__ double py_round4(double x) {
  if (!isfinite(x)) return x;
  const double hi = x * 10000.0;
  const double lo = fma(x, 10000.0, -hi);  // hi + lo == x * 10^4 exactly
  double f = floor(hi);
  if (hi == f && lo < 0.0) f -= 1.0;       // floor of the exact value
  const double frac_hi = hi - f;           // exact, in [0, 1]
  const double c = frac_hi - 0.5;          // exact when it matters (frac_hi >= 0.25)
  double r;
  if (frac_hi < 0.25) {
    r = f;
  } else if (c > -lo) {
    r = f + 1.0;
  } else if (c < -lo) {
    r = f;
  } else {
    r = (fmod(f, 2.0) == 0.0) ? f : f + 1.0;  // exact tie: half to even
  }
  return r / 10000.0;
}

__device__ __forceinline__ bool has_entry(const int32_t* list, int n, int32_t v) {
  for (int i = 0; i < n; ++i)
    if (list[i] == v) return true;
  return false;
}

__global__ __launch_bounds__(64) void expand_rerank_kernel(
    DevGraph g, const int32_t* __restrict__ seed_nodes, const int32_t* __restrict__ row_map, int64_t n_map,
    const float* __restrict__ seed_sem, int B,
    int k_seed, ahr_rerank_params p, int max_exp, int32_t* __restrict__ exp_nodes,
    double* __restrict__ exp_sem, int32_t* __restrict__ exp_src, int32_t* __restrict__ exp_count,
    int32_t* __restrict__ out_nodes, double* __restrict__ out_sem, double* __restrict__ out_score,
    int32_t* __restrict__ out_count) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  int32_t* en = exp_nodes + (int64_t)q * max_exp;
  double* es = exp_sem + (int64_t)q * max_exp;
  int32_t* ex = exp_src + (int64_t)q * max_exp;
  int n = 0;

  // ---- expansion: hierarchical_graph.py:727-740 (dict insertion order; seeds overwrite in
  // place, expansions only add absent ids)
  for (int s = 0; s < k_seed; ++s) {
    int32_t nid = seed_nodes[(int64_t)q * k_seed + s];
    if (row_map)  // seed_nodes are dense-index rows: their node indices (-1: no hit)
      nid = nid >= 0 && nid < n_map ? row_map[nid] : -1;
    if (nid < 0) continue;  // no hit (Chroma returned fewer ids)
    // semantic = 1.0 - float(dist) (:719-724), dist = Chroma's float32 cosine distance 1 - score
    const float dist = 1.0f - seed_sem[(int64_t)q * k_seed + s];
    const double sem = 1.0 - (double)dist;
    int pos = -1;
    for (int i = 0; i < n; ++i)
      if (en[i] == nid) { pos = i; break; }
    if (pos >= 0) {
      es[pos] = sem;
      ex[pos] = s;
    } else if (n < max_exp) {
      en[n] = nid; es[n] = sem; ex[n] = s; ++n;
    }
    if (nid >= g.n_nodes) continue;  // seed id unknown to the graph: no expansion
    const int8_t t = g.type[nid];
    int adj, lim, code;
    double factor;
    if (t == AHR_NODE_ENTITY) {
      adj = ADJ_BT_OUT; lim = 2; factor = 0.9; code = -1 - AHR_NODE_SUMMARY;
    } else if (t == AHR_NODE_SUMMARY) {
      adj = ADJ_BT_IN; lim = p.member_top_m; factor = 0.85; code = -1 - AHR_NODE_ENTITY;
    } else {
      continue;
    }
    const int64_t b = g.off[adj][nid], e = g.off[adj][nid + 1];
    for (int64_t j = b; j < e && j - b < lim; ++j) {
      const int32_t v = g.tgt[adj][j];
      if (!has_entry(en, n, v) && n < max_exp) {
        en[n] = v; es[n] = sem * factor; ex[n] = code; ++n;
      }
    }
  }
  exp_count[q] = n;

  // ---- rerank: hierarchical_graph.py:743-782, stable sort on the rounded score, [:top_k]
  int32_t* on = out_nodes + (int64_t)q * p.top_k;
  double* os = out_sem + (int64_t)q * p.top_k;
  double* oc = out_score + (int64_t)q * p.top_k;
  int m = 0;
  for (int i = 0; i < n && p.top_k > 0; ++i) {
    const int32_t v = en[i];
    const bool known = v < g.n_nodes;
    const int t = known ? g.type[v] : AHR_NODE_OTHER;
    const double judge = known ? g.judge[v] : NAN;
    const double conf = known ? g.conf[v] : NAN;
    if (p.type_mask && !((p.type_mask >> t) & 1)) continue;
    if (!isnan(p.judge_min) && (isnan(judge) || judge < p.judge_min)) continue;
    if (!isnan(p.confidence_min) && (isnan(conf) || conf < p.confidence_min)) continue;
    const double jt = (known && !isnan(judge)) ? g.judge_term[v] : 0.0;
    const double ct = (known && !isnan(conf)) ? g.conf_term[v] : 0.0;
    const double sem = es[i];
    // left-to-right evaluation order of the reference expression (:768)
    double score = p.alpha * sem;
    score = score + p.beta * jt;
    score = score + p.gamma * ct;
    score = score + p.delta * p.layer_boost[t];
    const double rs = py_round4(score);
    // stable descending insertion: after every kept entry with score >= rs
    int j = m < p.top_k ? m : p.top_k;
    while (j > 0 && oc[j - 1] < rs) --j;
    if (j >= p.top_k) continue;
    const int last = (m < p.top_k ? m : p.top_k - 1);
    for (int u = last; u > j; --u) {
      on[u] = on[u - 1]; os[u] = os[u - 1]; oc[u] = oc[u - 1];
    }
    on[j] = v; os[j] = py_round4(sem); oc[j] = rs;
    if (m < p.top_k) ++m;
  }
  out_count[q] = m;
}

// The same pass with one wave per query and every step parallel over the wave (the default when a
// query's candidates fit kWaveCand): the serial kernel above chains ~30 dependent global loads per
// query and re-reads its own growing dict from memory for every membership test (45 us of the
// drop-in B = 1 search). Here the dict is rebuilt from its definition instead of by insertion:
//   * candidates, in the reference's order (:727-740): per seed s (lane s) the seed itself, then its
//     first `lim` belongs_to parents (entity) / members (summary), laid out by a wave prefix sum of
//     the per-seed counts, all loads of a level issued together;
//   * the dict: a node's position is its first candidate, its value the LAST seed candidate of that
//     node if it has one (a seed assignment overwrites in place), else its first candidate (an
//     expansion only adds an absent id) — exactly the insertion semantics;
//   * rerank (:743-782): each entry's score with the same left-to-right double arithmetic; the
//     stable descending sort on the rounded score is a rank: #{kept j: rs_j > rs_i} + #{kept j < i:
//     rs_j == rs_i}; ranks below top_k are written.
// Bitwise equal to expand_rerank_kernel (tests/test_dropin_gpu.py, test_rerank_rounding.py).
constexpr int kWaveCand = 1024;  // candidates (and dict entries) per query held in LDS
constexpr int kWaveSeeds = 64;   // one seed per lane

// LISTS (the drop-in search's one-call path, ahr_search_host): the dense stage's per-(query, split)
// sorted key lists come in instead of its merged top k_seed — the wave merges them first (the walk
// of merge_block_kernel over the lists in LDS, dense::walk_lists_lds), writes the merged rows and
// scores where the merge kernel would have (seed_nodes / seed_sem, read back by the host) and
// takes its seeds from the winners it holds: one launch and one launch gap fewer per search.
template <bool LISTS>
__global__ __launch_bounds__(64) void expand_rerank_wave_kernel(
    DevGraph g, const int32_t* __restrict__ seed_nodes, const int32_t* __restrict__ row_map, int64_t n_map,
    const float* __restrict__ seed_sem, int B, int k_seed, ahr_rerank_params p, int max_exp,
    int32_t* __restrict__ exp_nodes, double* __restrict__ exp_sem, int32_t* __restrict__ exp_src,
    int32_t* __restrict__ exp_count, int32_t* __restrict__ out_nodes, double* __restrict__ out_sem,
    double* __restrict__ out_score, int32_t* __restrict__ out_count, const uint64_t* __restrict__ lists,
    int n_lists) {
  __shared__ int32_t c_node[kWaveCand];
  __shared__ int32_t c_src[kWaveCand];  // seed index (>= 0) or -1 - assumed node type (expansion)
  __shared__ double c_sem[kWaveCand];
  __shared__ int32_t e_node[kWaveCand];
  __shared__ double e_sem[kWaveCand];
  __shared__ double e_rs[kWaveCand];  // rounded score
  __shared__ uint8_t e_keep[kWaveCand];  // passed the filters
  const int q = blockIdx.x;
  const int lane = threadIdx.x;
  if (q >= B) return;
  uint64_t won = 0;  // LISTS: this lane's merged key (dense result lane)
  if constexpr (LISTS) {
    __shared__ uint64_t kb[kRerankFuseKeys];
    const int n = n_lists * k_seed;  // <= kRerankFuseKeys (the caller's check)
    const uint64_t* src = lists + (int64_t)q * n;
    // every load in flight at once (a load -> LDS store loop waits one memory latency per key)
    constexpr int kPer = kRerankFuseKeys / 64;
    uint64_t v[kPer];
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = lane + 64 * u;
      if (64 * u < n) v[u] = src[i < n ? i : n - 1];  // (64 u < n: wave-uniform)
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int i = lane + 64 * u;
      if (i < n) kb[i] = v[u];
    }
    __syncthreads();
    won = dense::walk_lists_lds(kb, n_lists, k_seed, k_seed, (int64_t)q * k_seed, const_cast<float*>(seed_sem),
                                const_cast<int32_t*>(seed_nodes), nullptr);
  }

  // ---- candidates: lane s owns seed s
  int32_t nid = -1;
  double sem = 0.0;
  int adj = 0, cnt_exp = 0, code = 0;
  double factor = 0.0;
  int64_t b0 = 0;
  if (lane < k_seed) {
    float ss;
    if constexpr (LISTS) {
      nid = won ? (int32_t)key_row(won) : -1;
      ss = won ? key_score(won) : -INFINITY;
    } else {
      nid = seed_nodes[(int64_t)q * k_seed + lane];
      ss = seed_sem[(int64_t)q * k_seed + lane];
    }
    if (row_map) nid = nid >= 0 && nid < n_map ? row_map[nid] : -1;
    const float dist = 1.0f - ss;  // Chroma's float32 distance
    sem = 1.0 - (double)dist;
    if (nid >= 0 && nid < g.n_nodes) {
      const int8_t t = g.type[nid];
      int lim = 0;
      if (t == AHR_NODE_ENTITY) {
        adj = ADJ_BT_OUT; lim = 2; factor = 0.9; code = -1 - AHR_NODE_SUMMARY;
      } else if (t == AHR_NODE_SUMMARY) {
        adj = ADJ_BT_IN; lim = p.member_top_m; factor = 0.85; code = -1 - AHR_NODE_ENTITY;
      }
      if (lim > 0) {
        b0 = g.off[adj][nid];
        const int64_t deg = g.off[adj][nid + 1] - b0;
        cnt_exp = (int)(deg < lim ? deg : lim);
      }
    }
  }
  const int cnt = nid >= 0 ? 1 + cnt_exp : 0;
  // exclusive prefix sum of cnt over the wave
  int incl = cnt;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d, 64);
    if (lane >= d) incl += o;
  }
  const int total = __shfl(incl, 63, 64);
  const int pre = incl - cnt;
  if (cnt) {
    c_node[pre] = nid;
    c_sem[pre] = sem;
    c_src[pre] = lane;
    const double es = sem * factor;
    for (int j = 0; j < cnt_exp; ++j) {
      c_node[pre + 1 + j] = g.tgt[adj][b0 + j];
      c_sem[pre + 1 + j] = es;
      c_src[pre + 1 + j] = code;
    }
  }
  __syncthreads();

  // ---- the dict: first occurrences in candidate order, values from the last seed occurrence
  int n = 0;
  for (int base = 0; base < total; base += 64) {
    const int i = base + lane;
    bool first = false;
    int val = i;
    if (i < total) {
      const int32_t v = c_node[i];
      first = true;
      int last_seed = -1;
      for (int j = 0; j < total; ++j) {
        if (c_node[j] == v) {
          if (j < i) first = false;
          if (c_src[j] >= 0) last_seed = j;
        }
      }
      if (last_seed >= 0) val = last_seed;
    }
    const uint64_t m = __ballot(first);
    const int idx = n + __popcll(m & ((1ull << lane) - 1));
    if (first) {
      const int32_t v = c_node[i];
      e_node[idx] = v;
      e_sem[idx] = c_sem[val];
      exp_nodes[(int64_t)q * max_exp + idx] = v;
      exp_sem[(int64_t)q * max_exp + idx] = c_sem[val];
      exp_src[(int64_t)q * max_exp + idx] = c_src[val];
    }
    n += __popcll(m);
  }
  if (lane == 0) exp_count[q] = n;
  if (p.top_k <= 0) {
    if (lane == 0) out_count[q] = 0;
    return;
  }
  __syncthreads();

  // ---- rerank: scores and filters per entry (hierarchical_graph.py:743-779)
  for (int i = lane; i < n; i += 64) {
    const int32_t v = e_node[i];
    const bool known = v < g.n_nodes;
    const int t = known ? g.type[v] : AHR_NODE_OTHER;
    const double judge = known ? g.judge[v] : NAN;
    const double conf = known ? g.conf[v] : NAN;
    bool keep = true;
    if (p.type_mask && !((p.type_mask >> t) & 1)) keep = false;
    if (!isnan(p.judge_min) && (isnan(judge) || judge < p.judge_min)) keep = false;
    if (!isnan(p.confidence_min) && (isnan(conf) || conf < p.confidence_min)) keep = false;
    const double jt = (known && !isnan(judge)) ? g.judge_term[v] : 0.0;
    const double ct = (known && !isnan(conf)) ? g.conf_term[v] : 0.0;
    const double s = e_sem[i];
    double score = p.alpha * s;  // left-to-right, every operation rounded (:768)
    score = score + p.beta * jt;
    score = score + p.gamma * ct;
    score = score + p.delta * p.layer_boost[t];
    e_rs[i] = py_round4(score);
    e_keep[i] = keep;
  }
  __syncthreads();
  // ---- stable sort descending on the rounded score, [:top_k] (:781-782), as ranks
  int kept = 0;
  for (int i = lane; i < n; i += 64) {
    if (!e_keep[i]) continue;
    const double rs = e_rs[i];
    ++kept;
    int rank = 0;
    for (int j = 0; j < n; ++j) {
      const double o = e_rs[j];
      rank += (e_keep[j] && (o > rs || (j < i && o == rs))) ? 1 : 0;
    }
    if (rank < p.top_k) {
      out_nodes[(int64_t)q * p.top_k + rank] = e_node[i];
      out_sem[(int64_t)q * p.top_k + rank] = py_round4(e_sem[i]);
      out_score[(int64_t)q * p.top_k + rank] = rs;
    }
  }
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) kept += __shfl_xor(kept, d, 64);
  if (lane == 0) out_count[q] = kept < p.top_k ? kept : p.top_k;
}

// GraphEnvironment expansions. Streams the reference's raw neighbour sequence but keeps only
// the first `limit` distinct ids: that prefix is all that survives dict.fromkeys()[:limit],
// and the per-input break (raw length >= limit after an input node) is tracked on the raw count.
struct Emit {
  int32_t* out;   // the kept ids: out[i * stride]
  int stride;
  int limit;
  int n;       // distinct ids kept
  int64_t raw; // raw appends (the reference's len(expanded) before dedupe)
  __device__ bool full() const { return n >= limit; }
  __device__ void push(int32_t v) {
    ++raw;
    if (n >= limit) return;
    for (int i = 0; i < n; ++i)
      if (out[i * stride] == v) return;
    out[n++ * stride] = v;
  }
};

// The kept ids live in LDS while the walk dedupes against them (interleaved per thread: entry i of
// thread t at i * 64 + t, conflict-free) for limits up to kExpLds, else in the output row itself
// (every membership test then an L2 round trip).
constexpr int kExpLds = 32;

// One environment's expansion (environment.py:393-480) of the node indices inputs[0 .. n_in) into em.
__device__ __forceinline__ void expand_one(const DevGraph& g, int action, const int32_t* inputs, int n_in, int limit,
                                           Emit& em) {
  for (int i = 0; i < n_in && !em.full(); ++i) {
    const int32_t nid = inputs[i];
    if (nid < 0 || nid >= g.n_nodes) continue;  // `if nid not in self.hg.G: continue`
    if (action == 0 || action == 1) {
      // 0: successors with belongs_to (expand_parents :424-426)
      // 1: predecessors with belongs_to (expand_children :401-403)
      const int adj = action == 0 ? ADJ_BT_OUT : ADJ_BT_IN;
      for (int64_t j = g.off[adj][nid]; j < g.off[adj][nid + 1] && !em.full(); ++j) em.push(g.tgt[adj][j]);
    } else {
      // expand_related :448-467
      for (int64_t j = g.off[ADJ_REL_OUT][nid]; j < g.off[ADJ_REL_OUT][nid + 1] && !em.full(); ++j)
        em.push(g.tgt[ADJ_REL_OUT][j]);
      for (int64_t j = g.off[ADJ_REL_IN][nid]; j < g.off[ADJ_REL_IN][nid + 1] && !em.full(); ++j)
        em.push(g.tgt[ADJ_REL_IN][j]);
      if (g.type[nid] == AHR_NODE_ENTITY) {
        for (int64_t j = g.off[ADJ_PI_OUT][nid]; j < g.off[ADJ_PI_OUT][nid + 1] && !em.full(); ++j) {
          const int32_t h = g.tgt[ADJ_PI_OUT][j];
          em.push(h);
          for (int64_t u = g.off[ADJ_PI_IN][h]; u < g.off[ADJ_PI_IN][h + 1] && !em.full(); ++u) {
            const int32_t w = g.tgt[ADJ_PI_IN][u];
            if (w != nid) em.push(w);
          }
        }
      }
    }
    if (em.raw >= limit) break;  // `if len(expanded) >= limit: break`
  }
}

template <bool kLds>
__global__ __launch_bounds__(64) void expand_kernel(DevGraph g, int action,
                                                    const int32_t* __restrict__ inputs, int B,
                                                    int n_in, int limit, int32_t* __restrict__ out,
                                                    int32_t* __restrict__ out_count) {
  __shared__ int32_t sbuf[kLds ? kExpLds * 64 : 1];
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= B) return;
  Emit em{kLds ? sbuf + threadIdx.x : out + (int64_t)q * limit, kLds ? 64 : 1, limit, 0, 0};
  expand_one(g, action, inputs + (int64_t)q * n_in, n_in, limit, em);
  if constexpr (kLds)
    for (int i = 0; i < em.n; ++i) out[(int64_t)q * limit + i] = sbuf[i * 64 + threadIdx.x];
  out_count[q] = em.n;
}

// One step of E environments of VecAHRAGGymEnv (gym_env.py:77-125 over environment.py:301-355,
// :393-480), their state resident in device memory (one thread per environment):
//   actions 0-2  expansion of the current selection's top 2 / 2 / 1 graph nodes (limit K): the
//                observation shows the selection = the expansion and the frontier BEFORE its ids
//                join it (f_shown = the frontier slots it shows); then frontier |= expansion;
//   action 3     commit of the top 3: graph nodes not yet selected join the selection (appended)
//                and leave the frontier (their slot set to -1); the observation shows the added ids;
//   action 4     details of the top node (a selection of it alone if it is a graph node; none if
//                the selection is empty: then, like any other action, the previous observation);
//   else         end / invalid: the observation is the previous one (kind -1), no state change.
// State: sel [E][K] / sel_n (the current observation's selection, rewritten in place), frontier F
// [E][fcap] (append-only slots, -1 = removed) / F_end (slots used) / F_n (members), selection S
// [E][scap] / S_n. A full frontier or selection sets *err (the host grows the buffers first).
// With a node table (feats [n_feat][6]: is_entity, is_summary, is_other, layer, judge, confidence
// per extended node index) each new observation's featurizer vector is written too (vec [E][4 + 8 K],
// step [E] the environments' step counters).
constexpr int kEnvTop[5] = {2, 2, 1, 3, 1};

__global__ __launch_bounds__(64) void env_step_kernel(DevGraph g, int E, int K, int fcap, int scap, int limit,
                                                      const int32_t* __restrict__ actions, int32_t* __restrict__ sel,
                                                      int32_t* __restrict__ sel_n, int32_t* __restrict__ F,
                                                      int32_t* __restrict__ F_end, int32_t* __restrict__ F_n,
                                                      int32_t* __restrict__ S, int32_t* __restrict__ S_n,
                                                      int32_t* __restrict__ kind, int32_t* __restrict__ seed_n,
                                                      int32_t* __restrict__ f_shown, int32_t* __restrict__ f_size,
                                                      int32_t* __restrict__ s_size, int32_t* __restrict__ step,
                                                      float* __restrict__ vec, int32_t* __restrict__ err,
                                                      const float* __restrict__ feats, int64_t n_feat) {
  __shared__ int32_t sbuf[kExpLds * 64];
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= E) return;
  const int a = actions[e];
  const int n = sel_n[e];
  int32_t* my_sel = sel + (int64_t)e * K;
  int32_t top[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int32_t x = j < n && j < K ? my_sel[j] : -1;
    top[j] = x >= 0 && x < g.n_nodes ? x : -1;  // graph nodes only (`if nid in self.hg.G`)
  }
  int32_t* myF = F + (int64_t)e * fcap;
  int32_t* myS = S + (int64_t)e * scap;
  int fe = F_end[e], fn = F_n[e], sn = S_n[e];
  int k_out = -1;
  int f_obs = 0;  // the frontier size the new observation shows (before an expansion's union)
  if (a >= 0 && a <= 2) {
    Emit em{sbuf + threadIdx.x, 64, limit, 0, 0};
    expand_one(g, a, top, kEnvTop[a], limit, em);
    f_shown[e] = fe;
    f_size[e] = fn;
    f_obs = fn;
    s_size[e] = sn;
    for (int i = 0; i < K; ++i) my_sel[i] = i < em.n ? sbuf[i * 64 + threadIdx.x] : -1;
    sel_n[e] = em.n;
    seed_n[e] = em.n;
    for (int i = 0; i < em.n; ++i) {  // frontier |= expansion
      const int32_t v = sbuf[i * 64 + threadIdx.x];
      bool found = false;
      for (int j = 0; j < fe && !found; ++j) found = myF[j] == v;
      if (found) continue;
      if (fe >= fcap) {
        *err = 1;
        break;
      }
      myF[fe++] = v;
      ++fn;
    }
    k_out = 1;
  } else if (a == 3) {
    int32_t added[3];
    int na = 0;
    for (int j = 0; j < 3 && j < n; ++j) {
      const int32_t x = top[j];
      if (x < 0) continue;
      bool in_s = false;
      for (int i = 0; i < sn && !in_s; ++i) in_s = myS[i] == x;
      if (in_s) continue;
      if (sn >= scap) {
        *err = 1;
        break;
      }
      myS[sn++] = x;
      added[na++] = x;
      for (int i = 0; i < fe; ++i)
        if (myF[i] == x) {  // `self.frontier_set.discard(nid)`
          myF[i] = -1;
          --fn;
          break;
        }
    }
    for (int i = 0; i < K; ++i) my_sel[i] = i < na ? added[i] : -1;
    sel_n[e] = na;
    seed_n[e] = 0;
    f_shown[e] = fe;
    f_size[e] = fn;
    s_size[e] = sn;
    f_obs = fn;
    k_out = 2;
  } else if (a == 4 && n > 0) {
    const int32_t node = n > 0 && K > 0 ? my_sel[0] : -1;
    const bool in_g = node >= 0 && node < g.n_nodes;
    for (int i = 0; i < K; ++i) my_sel[i] = i == 0 && in_g ? node : -1;
    sel_n[e] = in_g ? 1 : 0;
    seed_n[e] = 0;
    k_out = 3;
  }
  F_end[e] = fe;
  F_n[e] = fn;
  S_n[e] = sn;
  kind[e] = k_out;
  if (k_out < 0 || !feats) return;  // the previous observation: its vector stays
  // the observation's 4 + 8 K featurizer vector (featurizer.py:21-56): [step, |selection|,
  // min(|frontier|, 50), |seeds|] + per shown node [is_entity, is_summary, is_other, layer, score,
  // semantic, judge_overall, confidence] from the node table (score and semantic are 0 after a
  // step); a details observation has no state (zeros)
  const int stp = step[e] + 1;
  step[e] = stp;
  float* v = vec + (int64_t)e * (4 + 8 * K);
  const bool full = k_out != 3;
  v[0] = (float)stp;
  v[1] = full ? (float)sn : 0.f;
  v[2] = full ? (float)(f_obs < 50 ? f_obs : 50) : 0.f;
  v[3] = (float)seed_n[e];
  const int ns = sel_n[e];
  for (int i = 0; i < K; ++i) {
    float* b = v + 4 + 8 * i;
    const int32_t x = i < ns ? my_sel[i] : -1;
    const float* f = x >= 0 && x < n_feat ? feats + (int64_t)x * 6 : nullptr;
    b[0] = f ? f[0] : 0.f;
    b[1] = f ? f[1] : 0.f;
    b[2] = f ? f[2] : 0.f;
    b[3] = f ? f[3] : 0.f;
    b[4] = 0.f;
    b[5] = 0.f;
    b[6] = f ? f[4] : 0.f;
    b[7] = f ? f[5] : 0.f;
  }
}

// The single environment's expansion straight from and to the host: the inputs travel in the
// kernel arguments and the results are stored into pinned host memory, so the call is one launch
// and one stream wait (no copy operations, each a few microseconds of latency at this size).
constexpr int kSmallIn = 16;
struct SmallInputs {
  int32_t v[kSmallIn];
};

__global__ __launch_bounds__(64) void expand_small_kernel(DevGraph g, int action, SmallInputs in, int B, int n_in,
                                                          int limit, int32_t* __restrict__ out,
                                                          int32_t* __restrict__ out_count) {
  __shared__ int32_t sbuf[kExpLds * 64];
  const int q = threadIdx.x;
  if (q >= B) return;
  int32_t x[kSmallIn];
#pragma unroll
  for (int i = 0; i < kSmallIn; ++i) x[i] = in.v[i];
  int32_t mine[kSmallIn];
  int m = 0;
#pragma unroll
  for (int i = 0; i < kSmallIn; ++i)
    if (i >= q * n_in && i < (q + 1) * n_in) mine[m++] = x[i];
  Emit em{sbuf + threadIdx.x, 64, limit, 0, 0};
  expand_one(g, action, mine, n_in, limit, em);
  for (int i = 0; i < em.n; ++i) out[(int64_t)q * (limit > 0 ? limit : 1) + i] = sbuf[i * 64 + threadIdx.x];
  out_count[q] = em.n;
}

// launch on B queries (one thread each)
inline void launch_expand(hipStream_t s, const DevGraph& dg, int action, const int32_t* inputs, int B, int n_in,
                          int limit, int32_t* out, int32_t* out_count) {
  if (limit <= kExpLds)
    hipLaunchKernelGGL(expand_kernel<true>, dim3((B + 63) / 64), dim3(64), 0, s, dg, action, inputs, B, n_in, limit,
                       out, out_count);
  else
    hipLaunchKernelGGL(expand_kernel<false>, dim3((B + 63) / 64), dim3(64), 0, s, dg, action, inputs, B, n_in, limit,
                       out, out_count);
}

// expand_to_lca (environment.py:243-299): per query, the intersection over its input nodes of
// "ancestors or self" on the belongs_to DAG (nx.ancestors: nodes with a belongs_to path TO the
// node, i.e. the reverse walk over belongs_to IN-edges), then its lowest members (no belongs_to
// out-edge to another member). One 256-thread workgroup per query runs a level-synchronous
// reverse BFS per input over the device CSR. Visited nodes live in an LDS hash table (open
// addressing) whose slot holds (node, last input that reached it, number of inputs that reached
// it): a discovery claims (node, input) with one atomic exchange on `last`, so each node enters
// an input's frontier once and is counted once per input; a node is in the intersection iff its
// count is the number of (non-padding) inputs. Capacities: kLcaHash distinct nodes per query, kLcaFront nodes per BFS level; a
// query beyond them reports count -1 (the caller raises) instead of a wrong answer.
constexpr int kLcaHash = 4096;  // power of two
constexpr int kLcaFront = 1024;

__device__ __forceinline__ uint32_t lca_hash(int32_t v) { return ((uint32_t)v * 2654435761u) & (kLcaHash - 1); }

__global__ __launch_bounds__(256) void lca_kernel(DevGraph g, const int32_t* __restrict__ inputs, int n_in,
                                                  int max_out, int32_t* __restrict__ out,
                                                  int32_t* __restrict__ out_count) {
  __shared__ int32_t hkey[kLcaHash];   // node id, -1 = empty
  __shared__ int32_t hlast[kLcaHash];  // last input index that reached the node
  __shared__ int32_t hcnt[kLcaHash];   // inputs that reached it
  __shared__ int32_t front[2][kLcaFront];
  __shared__ int32_t nfront[2];
  __shared__ int32_t nout;
  __shared__ int32_t overflow;
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  for (int i = tid; i < kLcaHash; i += 256) {
    hkey[i] = -1;
    hlast[i] = -1;
    hcnt[i] = 0;
  }
  if (tid == 0) {
    nout = 0;
    overflow = 0;
  }
  // claim (v, input i): true the first time input i reaches v (v's slot is created if absent)
  auto claim = [&](int32_t v, int i) -> bool {
    uint32_t h = lca_hash(v);
    for (int probe = 0; probe < kLcaHash; ++probe, h = (h + 1) & (kLcaHash - 1)) {
      const int32_t prev = atomicCAS(&hkey[h], -1, v);
      if (prev == -1 || prev == v) {
        const int32_t last = atomicExch(&hlast[h], i);
        if (last == i) return false;
        atomicAdd(&hcnt[h], 1);
        return true;
      }
    }
    atomicOr(&overflow, 1);
    return false;
  };
  auto lookup_count = [&](int32_t v) -> int32_t {
    uint32_t h = lca_hash(v);
    for (int probe = 0; probe < kLcaHash; ++probe, h = (h + 1) & (kLcaHash - 1)) {
      if (hkey[h] == -1) return 0;
      if (hkey[h] == v) return hcnt[h];
    }
    return 0;
  };
  __syncthreads();
  int n_valid = 0;  // -1 entries pad a query's input list
  for (int i = 0; i < n_in; ++i) {
    const int32_t src = inputs[(int64_t)q * n_in + i];
    if (src < 0 || src >= g.n_nodes) continue;  // uniform: every thread reads the same input
    ++n_valid;
    if (tid == 0) {
      nfront[0] = 0;
      nfront[1] = 0;
      if (claim(src, i)) {
        front[0][0] = src;
        nfront[0] = 1;
      }
    }
    __syncthreads();
    int cur = 0;
    while (nfront[cur] > 0) {
      const int n = min(nfront[cur], kLcaFront);
      for (int j = tid; j < n; j += 256) {
        const int32_t v = front[cur][j];
        for (int64_t e = g.off[ADJ_BT_IN][v]; e < g.off[ADJ_BT_IN][v + 1]; ++e) {
          const int32_t u = g.tgt[ADJ_BT_IN][e];
          if (!claim(u, i)) continue;
          const int slot = atomicAdd(&nfront[cur ^ 1], 1);
          if (slot < kLcaFront)
            front[cur ^ 1][slot] = u;
          else
            atomicOr(&overflow, 1);
        }
      }
      __syncthreads();
      if (tid == 0) nfront[cur] = 0;
      __syncthreads();
      cur ^= 1;
    }
    __syncthreads();
  }
  // lowest members of the intersection: no belongs_to out-edge to another member
  for (int h = tid; h < kLcaHash; h += 256) {
    const int32_t v = hkey[h];
    if (v < 0 || n_valid == 0 || hcnt[h] != n_valid) continue;
    bool lowest = true;
    for (int64_t e = g.off[ADJ_BT_OUT][v]; e < g.off[ADJ_BT_OUT][v + 1] && lowest; ++e)
      if (lookup_count(g.tgt[ADJ_BT_OUT][e]) == n_valid) lowest = false;
    if (lowest) {
      const int slot = atomicAdd(&nout, 1);
      if (slot < max_out)
        out[(int64_t)q * max_out + slot] = v;
      else
        atomicOr(&overflow, 1);
    }
  }
  __syncthreads();
  if (tid == 0) out_count[q] = overflow ? -1 : min(nout, max_out);
}

// The same walk without capacity limits, for the queries lca_kernel reports as over capacity (a
// topic with more than 1024 members, an L2 summary above 4096 descendants). Per query a direct-
// indexed workspace in global memory of 5 * n_nodes int32: last input per node, inputs per node,
// the visited list (each node once, so the lowest-member scan only looks at reached nodes) and two
// BFS frontiers, each bounded by n_nodes because a node enters an input's frontier once. The
// kernel clears its own workspace, so nothing has to be initialised between calls. The per-node
// words are written with device-scope atomics and read back with agent-scope atomic loads (L2),
// never through the vector L1.
__global__ __launch_bounds__(256) void lca_global_kernel(DevGraph g, const int32_t* __restrict__ inputs, int n_in,
                                                         int max_out, int32_t* __restrict__ out,
                                                         int32_t* __restrict__ out_count, int32_t* __restrict__ ws) {
  __shared__ int32_t nvis;
  __shared__ int32_t nfront[2];
  __shared__ int32_t nout;
  __shared__ int32_t overflow;
  const int q = blockIdx.x;
  const int tid = threadIdx.x;
  const int64_t n = g.n_nodes;
  int32_t* last = ws + (int64_t)q * 5 * n;
  int32_t* cnt = last + n;
  int32_t* vis = cnt + n;
  int32_t* front[2] = {vis + n, vis + 2 * n};
  for (int64_t i = tid; i < n; i += 256) {
    __hip_atomic_store(&last[i], -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(&cnt[i], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (tid == 0) {
    nvis = 0;
    nout = 0;
    overflow = 0;
  }
  __syncthreads();
  auto claim = [&](int32_t v, int i) -> bool {
    const int32_t prev = atomicExch(&last[v], i);
    if (prev == i) return false;
    if (prev == -1) vis[atomicAdd(&nvis, 1)] = v;
    atomicAdd(&cnt[v], 1);
    return true;
  };
  auto count_of = [&](int32_t v) -> int32_t {
    return __hip_atomic_load(&cnt[v], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  };
  int n_valid = 0;
  for (int i = 0; i < n_in; ++i) {
    const int32_t src = inputs[(int64_t)q * n_in + i];
    if (src < 0 || src >= n) continue;  // uniform
    ++n_valid;
    if (tid == 0) {
      nfront[0] = 0;
      nfront[1] = 0;
      if (claim(src, i)) {
        front[0][0] = src;
        nfront[0] = 1;
      }
    }
    __syncthreads();
    int cur = 0;
    while (nfront[cur] > 0) {
      const int nf = nfront[cur];
      for (int j = tid; j < nf; j += 256) {
        const int32_t v = front[cur][j];
        for (int64_t e = g.off[ADJ_BT_IN][v]; e < g.off[ADJ_BT_IN][v + 1]; ++e) {
          const int32_t u = g.tgt[ADJ_BT_IN][e];
          if (claim(u, i)) front[cur ^ 1][atomicAdd(&nfront[cur ^ 1], 1)] = u;
        }
      }
      __syncthreads();
      if (tid == 0) nfront[cur] = 0;
      __syncthreads();
      cur ^= 1;
    }
    __syncthreads();
  }
  const int nv = nvis;
  for (int s = tid; s < nv; s += 256) {
    const int32_t v = vis[s];
    if (n_valid == 0 || count_of(v) != n_valid) continue;
    bool lowest = true;
    for (int64_t e = g.off[ADJ_BT_OUT][v]; e < g.off[ADJ_BT_OUT][v + 1] && lowest; ++e)
      if (count_of(g.tgt[ADJ_BT_OUT][e]) == n_valid) lowest = false;
    if (lowest) {
      const int slot = atomicAdd(&nout, 1);
      if (slot < max_out)
        out[(int64_t)q * max_out + slot] = v;
      else
        atomicOr(&overflow, 1);
    }
  }
  __syncthreads();
  if (tid == 0) out_count[q] = overflow ? -1 : min(nout, max_out);
}

}  // namespace graph
}  // namespace ahr

using namespace ahr;
using namespace ahr::graph;

struct ahr_graph {
  int device = 0;
  int64_t n_nodes = 0;
  int64_t n_edges = 0;
  void* block = nullptr;  // one allocation holds every array
  DevGraph dg{};
};

namespace {

struct DeviceGuardG {
  int prev = -1;
  explicit DeviceGuardG(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceGuardG() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

inline size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

extern "C" {

int ahr_graph_create(int64_t n_nodes, const int8_t* node_type, const double* judge,
                     const double* confidence, const double* judge_term, const double* conf_term,
                     const int64_t* const* offsets, const int32_t* const* targets, int device,
                     ahr_graph** out) {
  if (!out) return fail(AHR_EINVAL, "null out pointer");
  *out = nullptr;
  if (n_nodes < 0 || n_nodes > 0x7FFFFFFF) return fail(AHR_EINVAL, "n_nodes out of range");
  if (n_nodes > 0 && (!node_type || !judge || !confidence || !judge_term || !conf_term))
    return fail(AHR_EINVAL, "null node attribute array");
  if (!offsets || !targets) return fail(AHR_EINVAL, "null adjacency arrays");
  int64_t nnz[AHR_ADJ_COUNT];
  int64_t total_edges = 0;
  for (int a = 0; a < AHR_ADJ_COUNT; ++a) {
    if (!offsets[a]) return fail(AHR_EINVAL, "null CSR offsets");
    nnz[a] = offsets[a][n_nodes];
    if (nnz[a] < 0 || offsets[a][0] != 0) return fail(AHR_EINVAL, "bad CSR offsets");
    if (nnz[a] > 0 && !targets[a]) return fail(AHR_EINVAL, "null CSR targets");
    for (int64_t i = 0; i < nnz[a]; ++i)
      if (targets[a][i] < 0 || targets[a][i] >= n_nodes) return fail(AHR_ERANGE, "CSR target out of range");
    if (a % 2 == 0) total_edges += nnz[a];  // each edge appears once in an *_out list
  }
  // layout of the single device block
  size_t sz = 0;
  const size_t o_type = sz; sz = align16(sz + (size_t)n_nodes);
  const size_t o_j = sz; sz = align16(sz + 8 * (size_t)n_nodes);
  const size_t o_c = sz; sz = align16(sz + 8 * (size_t)n_nodes);
  const size_t o_jt = sz; sz = align16(sz + 8 * (size_t)n_nodes);
  const size_t o_ct = sz; sz = align16(sz + 8 * (size_t)n_nodes);
  size_t o_off[AHR_ADJ_COUNT], o_tgt[AHR_ADJ_COUNT];
  for (int a = 0; a < AHR_ADJ_COUNT; ++a) {
    o_off[a] = sz; sz = align16(sz + 8 * (size_t)(n_nodes + 1));
    o_tgt[a] = sz; sz = align16(sz + 4 * (size_t)nnz[a]);
  }
  std::vector<uint8_t> host(sz, 0);
  if (n_nodes > 0) {
    std::memcpy(host.data() + o_type, node_type, (size_t)n_nodes);
    std::memcpy(host.data() + o_j, judge, 8 * (size_t)n_nodes);
    std::memcpy(host.data() + o_c, confidence, 8 * (size_t)n_nodes);
    std::memcpy(host.data() + o_jt, judge_term, 8 * (size_t)n_nodes);
    std::memcpy(host.data() + o_ct, conf_term, 8 * (size_t)n_nodes);
  }
  for (int a = 0; a < AHR_ADJ_COUNT; ++a) {
    std::memcpy(host.data() + o_off[a], offsets[a], 8 * (size_t)(n_nodes + 1));
    if (nnz[a]) std::memcpy(host.data() + o_tgt[a], targets[a], 4 * (size_t)nnz[a]);
  }
  DeviceGuardG dg(device);
  ahr_graph* g = new ahr_graph();
  g->device = device;
  g->n_nodes = n_nodes;
  g->n_edges = total_edges;
  if (hipMalloc(&g->block, sz ? sz : 16) != hipSuccess) {
    delete g;
    return fail(AHR_ENOMEM, "graph allocation failed");
  }
  if (hipMemcpy(g->block, host.data(), sz, hipMemcpyHostToDevice) != hipSuccess) {
    (void)hipFree(g->block);
    delete g;
    return fail(AHR_EHIP, "graph upload failed");
  }
  uint8_t* base = static_cast<uint8_t*>(g->block);
  g->dg.n_nodes = n_nodes;
  g->dg.type = reinterpret_cast<const int8_t*>(base + o_type);
  g->dg.judge = reinterpret_cast<const double*>(base + o_j);
  g->dg.conf = reinterpret_cast<const double*>(base + o_c);
  g->dg.judge_term = reinterpret_cast<const double*>(base + o_jt);
  g->dg.conf_term = reinterpret_cast<const double*>(base + o_ct);
  for (int a = 0; a < AHR_ADJ_COUNT; ++a) {
    g->dg.off[a] = reinterpret_cast<const int64_t*>(base + o_off[a]);
    g->dg.tgt[a] = reinterpret_cast<const int32_t*>(base + o_tgt[a]);
  }
  *out = g;
  return AHR_OK;
}

int ahr_graph_destroy(ahr_graph* g) {
  if (!g) return AHR_OK;
  DeviceGuardG dg(g->device);
  if (g->block) (void)hipFree(g->block);
  delete g;
  return AHR_OK;
}

int ahr_graph_lca(ahr_graph* g, const int32_t* inputs, int B, int n_in, int max_out, int32_t* out,
                  int32_t* out_count, void* stream) {
  if (!g) return fail(AHR_EINVAL, "null graph");
  if (B < 0 || n_in < 0 || max_out < 0) return fail(AHR_EINVAL, "negative size");
  if (B == 0) return AHR_OK;
  if ((n_in > 0 && !inputs) || !out_count || (max_out > 0 && !out)) return fail(AHR_EINVAL, "null buffer");
  DeviceGuardG dg(g->device);
  hipLaunchKernelGGL(lca_kernel, dim3((unsigned)B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), g->dg,
                     inputs, n_in, max_out, out, out_count);
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_graph_lca_workspace(const ahr_graph* g, int B, int64_t* bytes) {
  if (!g || !bytes) return fail(AHR_EINVAL, "null graph or output");
  if (B < 0) return fail(AHR_EINVAL, "negative size");
  *bytes = (int64_t)B * 5 * g->n_nodes * (int64_t)sizeof(int32_t);
  return AHR_OK;
}

int ahr_graph_lca_large(ahr_graph* g, const int32_t* inputs, int B, int n_in, int max_out, int32_t* out,
                        int32_t* out_count, void* workspace, int64_t workspace_bytes, void* stream) {
  if (!g) return fail(AHR_EINVAL, "null graph");
  if (B < 0 || n_in < 0 || max_out < 0) return fail(AHR_EINVAL, "negative size");
  if (B == 0) return AHR_OK;
  if ((n_in > 0 && !inputs) || !out_count || (max_out > 0 && !out)) return fail(AHR_EINVAL, "null buffer");
  int64_t need = 0;
  (void)ahr_graph_lca_workspace(g, B, &need);
  if (need > 0 && (!workspace || workspace_bytes < need))
    return fail(AHR_EINVAL, "workspace smaller than ahr_graph_lca_workspace(B)");
  if (reinterpret_cast<uintptr_t>(workspace) % 4 != 0) return fail(AHR_EINVAL, "workspace not 4-byte aligned");
  DeviceGuardG dg(g->device);
  hipLaunchKernelGGL(lca_global_kernel, dim3((unsigned)B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     g->dg, inputs, n_in, max_out, out, out_count, static_cast<int32_t*>(workspace));
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_graph_info(const ahr_graph* g, int64_t* n_nodes, int64_t* n_edges) {
  if (!g) return fail(AHR_EINVAL, "null graph");
  if (n_nodes) *n_nodes = g->n_nodes;
  if (n_edges) *n_edges = g->n_edges;
  return AHR_OK;
}

// one wave per query while its candidates fit the wave kernel's LDS (every search() / env reset
// shape: k_seed <= 64); the serial kernel otherwise (large top_k or member_top_m).
// AHR_RERANK_SERIAL=1: always the serial kernel (A/B; both are bitwise equal).
static bool rerank_on_wave(int k_seed, int member_top_m) {
  static const bool serial_only = [] {
    const char* e = getenv("AHR_RERANK_SERIAL");
    return e && atoi(e) != 0;
  }();
  const int lim_max = member_top_m > 2 ? member_top_m : 2;
  return !serial_only && k_seed <= kWaveSeeds && (int64_t)k_seed * (1 + lim_max) <= kWaveCand;
}

static int expand_rerank_impl(ahr_graph* g, const int32_t* seed_nodes, const int32_t* row_map, int64_t n_map,
                              const float* seed_sem, int B, int k_seed, const ahr_rerank_params* params,
                              int max_exp, int32_t* exp_nodes, double* exp_sem, int32_t* exp_src,
                              int32_t* exp_count, int32_t* out_nodes, double* out_sem, double* out_score,
                              int32_t* out_count, void* stream, const uint64_t* lists = nullptr, int n_lists = 0) {
  if (!g || !params) return fail(AHR_EINVAL, "null graph or params");
  if (B < 0 || k_seed < 0 || params->top_k < 0 || params->member_top_m < 0)
    return fail(AHR_EINVAL, "negative size");
  const int fan = params->member_top_m > 2 ? params->member_top_m : 2;
  if (max_exp < k_seed * (1 + fan)) return fail(AHR_EINVAL, "max_exp < k_seed * (1 + max(2, member_top_m))");
  if (B == 0) return AHR_OK;
  if (!seed_nodes || !seed_sem || !exp_nodes || !exp_sem || !exp_src || !exp_count || !out_nodes ||
      !out_sem || !out_score || !out_count)
    return fail(AHR_EINVAL, "null buffer");
  const ahr_rerank_params p = *params;
  DeviceGuardG dg(g->device);
  const bool wave = rerank_on_wave(k_seed, p.member_top_m);
  if (lists) {  // the dense stage's unmerged lists: the wave kernel merges them (ahr_search_host)
    if (!wave || (int64_t)n_lists * k_seed > kRerankFuseKeys || n_lists > 512)
      return fail(AHR_EINVAL, "fused list merge: lists do not fit the wave kernel");
    hipLaunchKernelGGL(expand_rerank_wave_kernel<true>, dim3((unsigned)B), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), g->dg, seed_nodes, row_map, n_map, seed_sem, B,
                       k_seed, p, max_exp, exp_nodes, exp_sem, exp_src, exp_count, out_nodes, out_sem,
                       out_score, out_count, lists, n_lists);
  } else if (wave)
    hipLaunchKernelGGL(expand_rerank_wave_kernel<false>, dim3((unsigned)B), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), g->dg, seed_nodes, row_map, n_map, seed_sem, B,
                       k_seed, p, max_exp, exp_nodes, exp_sem, exp_src, exp_count, out_nodes, out_sem,
                       out_score, out_count, (const uint64_t*)nullptr, 0);
  else
    hipLaunchKernelGGL(expand_rerank_kernel, dim3((B + 63) / 64), dim3(64), 0,
                       reinterpret_cast<hipStream_t>(stream), g->dg, seed_nodes, row_map, n_map, seed_sem, B,
                       k_seed, p, max_exp, exp_nodes, exp_sem, exp_src, exp_count, out_nodes, out_sem,
                       out_score, out_count);
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_graph_expand_rerank(ahr_graph* g, const int32_t* seed_nodes, const float* seed_sem, int B,
                            int k_seed, const ahr_rerank_params* params, int max_exp,
                            int32_t* exp_nodes, double* exp_sem, int32_t* exp_src,
                            int32_t* exp_count, int32_t* out_nodes, double* out_sem,
                            double* out_score, int32_t* out_count, void* stream) {
  return expand_rerank_impl(g, seed_nodes, nullptr, 0, seed_sem, B, k_seed, params, max_exp, exp_nodes, exp_sem,
                            exp_src, exp_count, out_nodes, out_sem, out_score, out_count, stream);
}

int ahr_graph_expand_rerank_rows(ahr_graph* g, const int32_t* rows, const int32_t* row_to_node, int64_t n_rows,
                                 const float* seed_sem, int B, int k_seed, const ahr_rerank_params* params,
                                 int max_exp, int32_t* exp_nodes, double* exp_sem, int32_t* exp_src,
                                 int32_t* exp_count, int32_t* out_nodes, double* out_sem, double* out_score,
                                 int32_t* out_count, void* stream) {
  if (!row_to_node || n_rows < 0) return fail(AHR_EINVAL, "null row map or negative row count");
  return expand_rerank_impl(g, rows, row_to_node, n_rows, seed_sem, B, k_seed, params, max_exp, exp_nodes,
                            exp_sem, exp_src, exp_count, out_nodes, out_sem, out_score, out_count, stream);
}

int ahr_graph_expand(ahr_graph* g, int action, const int32_t* inputs, int B, int n_in, int limit,
                     int32_t* out, int32_t* out_count, void* stream) {
  if (!g) return fail(AHR_EINVAL, "null graph");
  if (action < 0 || action > 2) return fail(AHR_EINVAL, "action must be 0, 1 or 2");
  if (B < 0 || n_in < 0 || limit < 0) return fail(AHR_EINVAL, "negative size");
  if (B == 0) return AHR_OK;
  if ((n_in > 0 && !inputs) || !out_count || (limit > 0 && !out)) return fail(AHR_EINVAL, "null buffer");
  DeviceGuardG dg(g->device);
  launch_expand(reinterpret_cast<hipStream_t>(stream), g->dg, action, inputs, B, n_in, limit, out, out_count);
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

// workspace layout: inputs [B][n_in], out [B][max(limit, 1)], count [B] (int32, 256-B aligned parts)
static int64_t expand_ws_bytes(int B, int n_in, int limit) {
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  return al((int64_t)B * n_in * 4) + al((int64_t)B * (limit > 0 ? limit : 1) * 4) + al((int64_t)B * 4);
}

int ahr_graph_env_layout(int E, int K, int fcap, int scap, int64_t offsets[16], int64_t* bytes) {
  if (!offsets || !bytes) return fail(AHR_EINVAL, "null output");
  if (E < 1 || K < 1 || fcap < 1 || scap < 1) return fail(AHR_EINVAL, "sizes must be >= 1");
  const int64_t e = E;
  const int64_t part[16] = {e, e * K, e, e * fcap, e, e, e * scap, e, e, e, e, e, e, e, e * (4 + 8 * K), 1};
  int64_t o = 0;
  for (int i = 0; i < 16; ++i) {
    offsets[i] = o;
    o += (part[i] + 63) / 64 * 64;  // int32 elements, 256-B aligned parts
  }
  *bytes = o * 4;
  return AHR_OK;
}

int ahr_graph_env_step(ahr_graph* g, int E, int K, int fcap, int scap, int limit, const float* node_feats,
                       int64_t n_feat, void* ws, int64_t ws_bytes, void* stream) {
  if (!g || !ws) return fail(AHR_EINVAL, "null graph or workspace");
  if (limit < 0 || limit > kExpLds || K < 3 || K < limit) return fail(AHR_EINVAL, "need 3 <= K, limit <= K, limit <= 32");
  if (n_feat < 0) return fail(AHR_EINVAL, "negative node table size");
  int64_t off[16], need = 0;
  const int st = ahr_graph_env_layout(E, K, fcap, scap, off, &need);
  if (st != AHR_OK) return st;
  if (ws_bytes < need) return fail(AHR_EINVAL, "workspace smaller than ahr_graph_env_layout's bytes");
  int32_t* w = static_cast<int32_t*>(ws);
  DeviceGuardG dg(g->device);
  hipLaunchKernelGGL(env_step_kernel, dim3((E + 63) / 64), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), g->dg, E,
                     K, fcap, scap, limit, w + off[0], w + off[1], w + off[2], w + off[3], w + off[4], w + off[5],
                     w + off[6], w + off[7], w + off[8], w + off[9], w + off[10], w + off[11], w + off[12], w + off[13],
                     reinterpret_cast<float*>(w + off[14]), w + off[15], node_feats, n_feat);
  AHR_HIP(hipGetLastError());
  return AHR_OK;
}

int ahr_graph_env_step_host(ahr_graph* g, int E, int K, int fcap, int scap, int limit, const float* node_feats,
                            int64_t n_feat, const int32_t* host_actions, void* ws, int64_t ws_bytes, int32_t* host_out,
                            void* stream) {
  if (!host_actions || !host_out) return fail(AHR_EINVAL, "null host buffer");
  int64_t off[16], need = 0;
  int st = ahr_graph_env_layout(E, K, fcap, scap, off, &need);
  if (st != AHR_OK) return st;
  if (!ws || ws_bytes < need) return fail(AHR_EINVAL, "workspace smaller than ahr_graph_env_layout's bytes");
  DeviceGuardG dg(g ? g->device : 0);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  AHR_HIP(hipMemcpyAsync(ws, host_actions, (size_t)E * 4, hipMemcpyHostToDevice, s));
  st = ahr_graph_env_step(g, E, K, fcap, scap, limit, node_feats, n_feat, ws, ws_bytes, stream);
  if (st != AHR_OK) return st;
  AHR_HIP(hipMemcpyAsync(host_out, ws, (size_t)need, hipMemcpyDeviceToHost, s));
  AHR_HIP(hipStreamSynchronize(s));
  return AHR_OK;
}

int ahr_graph_expand_ws_bytes(int B, int n_in, int limit, int64_t* bytes) {
  if (!bytes) return fail(AHR_EINVAL, "null output");
  if (B < 0 || n_in < 0 || limit < 0) return fail(AHR_EINVAL, "negative size");
  *bytes = expand_ws_bytes(B, n_in, limit);
  return AHR_OK;
}

int ahr_graph_expand_host(ahr_graph* g, int action, const int32_t* host_inputs, int B, int n_in, int limit,
                          int32_t* host_out, int32_t* host_count, void* ws, int64_t ws_bytes, void* stream) {
  if (!g) return fail(AHR_EINVAL, "null graph");
  if (action < 0 || action > 2) return fail(AHR_EINVAL, "action must be 0, 1 or 2");
  if (B < 0 || n_in < 0 || limit < 0) return fail(AHR_EINVAL, "negative size");
  if (B == 0) return AHR_OK;
  if ((n_in > 0 && !host_inputs) || !host_count || !host_out || !ws) return fail(AHR_EINVAL, "null buffer");
  if (ws_bytes < expand_ws_bytes(B, n_in, limit)) return fail(AHR_EINVAL, "workspace too small");
  DeviceGuardG dg(g->device);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int lim = limit > 0 ? limit : 1;
  // small batches into pinned host buffers: one launch, no copies (the outputs' device addresses:
  // pinned host memory is mapped; pageable memory takes the copy path below)
  // AHR_EXPAND_SMALL=0 (A/B): every batch takes the copy path
  static const bool small_on = [] {
    const char* e = getenv("AHR_EXPAND_SMALL");
    return !e || atoi(e) != 0;
  }();
  if (small_on && (int64_t)B * n_in <= kSmallIn && B <= 64 && limit <= kExpLds) {
    void *d_out = nullptr, *d_cnt = nullptr;
    if (hipHostGetDevicePointer(&d_out, host_out, 0) == hipSuccess &&
        hipHostGetDevicePointer(&d_cnt, host_count, 0) == hipSuccess) {
      SmallInputs in{};
      for (int i = 0; i < B * n_in; ++i) in.v[i] = host_inputs[i];
      hipLaunchKernelGGL(expand_small_kernel, dim3(1), dim3(64), 0, s, g->dg, action, in, B, n_in, limit,
                         static_cast<int32_t*>(d_out), static_cast<int32_t*>(d_cnt));
      AHR_HIP(hipGetLastError());
      AHR_HIP(hipStreamSynchronize(s));
      return AHR_OK;
    }
    (void)hipGetLastError();  // (pageable memory: clear the lookup's error, copy path)
  }
  auto al = [](int64_t b) { return (b + 255) / 256 * 256; };
  int32_t* d_in = static_cast<int32_t*>(ws);
  int32_t* d_out = reinterpret_cast<int32_t*>(static_cast<char*>(ws) + al((int64_t)B * n_in * 4));
  int32_t* d_cnt = reinterpret_cast<int32_t*>(reinterpret_cast<char*>(d_out) + al((int64_t)B * lim * 4));
  if (n_in > 0) AHR_HIP(hipMemcpyAsync(d_in, host_inputs, (size_t)B * n_in * 4, hipMemcpyHostToDevice, s));
  launch_expand(s, g->dg, action, d_in, B, n_in, limit, d_out, d_cnt);
  AHR_HIP(hipGetLastError());
  // out and count are adjacent (count after out's padded part): one copy when out needs no padding
  if ((int64_t)B * lim * 4 == al((int64_t)B * lim * 4) && host_count == host_out + (int64_t)B * lim) {
    AHR_HIP(hipMemcpyAsync(host_out, d_out, (size_t)B * lim * 4 + (size_t)B * 4, hipMemcpyDeviceToHost, s));
  } else {
    AHR_HIP(hipMemcpyAsync(host_out, d_out, (size_t)B * lim * 4, hipMemcpyDeviceToHost, s));
    AHR_HIP(hipMemcpyAsync(host_count, d_cnt, (size_t)B * 4, hipMemcpyDeviceToHost, s));
  }
  AHR_HIP(hipStreamSynchronize(s));
  return AHR_OK;
}

}  // extern "C"

namespace ahr {

bool graph_rerank_fusable(int k_seed, const ahr_rerank_params* params) {
  return params && k_seed >= 0 && params->member_top_m >= 0 && rerank_on_wave(k_seed, params->member_top_m);
}

int graph_rerank_lists(ahr_graph* g, const uint64_t* lists, int n_lists, int32_t* rows, const int32_t* row_to_node,
                       int64_t n_rows, float* scores, int B, int k_seed, const ahr_rerank_params* params,
                       int max_exp, int32_t* exp_nodes, double* exp_sem, int32_t* exp_src, int32_t* exp_count,
                       int32_t* out_nodes, double* out_sem, double* out_score, int32_t* out_count, void* stream) {
  if (!lists || n_lists < 1) return fail(AHR_EINVAL, "null or empty lists");
  if (!row_to_node || n_rows < 0) return fail(AHR_EINVAL, "null row map or negative row count");
  return expand_rerank_impl(g, rows, row_to_node, n_rows, scores, B, k_seed, params, max_exp, exp_nodes, exp_sem,
                            exp_src, exp_count, out_nodes, out_sem, out_score, out_count, stream, lists, n_lists);
}

}  // namespace ahr
