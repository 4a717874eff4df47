/*
 * ahr_oracle.c — CPU restatement of the dense top-k step of AH-RAG's search, used ONLY as the
 * checker for libahr_hip.so (tests/, __graft_entry__.smoke(), bench.py cpu_baseline). It is
 * never linked into, loaded by, or called from the product path.
 *
 * What it restates
 *   HierarchicalGraph.search queries a Chroma collection created with {"hnsw:space": "cosine"}
 *   (reference src/ah_rag/graph/hierarchical_graph.py:611, :714) over vectors encoded with
 *   normalize_embeddings=True (:656, :712). Chroma is un-vendored (unpinned, requirements.txt:1
 *   pins only python-dotenv); its HNSW walk is approximate. The oracle computes what an
 *   exhaustive walk returns: for unit vectors, cosine distance 1 - q.x, i.e. the n_results rows
 *   of largest inner product, ties by insertion order (row ascending).
 *
 * Arithmetic contracts (match the device kernels, ah-rag_amd/csrc/ahr_dense.hip)
 *   mode 0 (fp32 exact): score = fmaf chain over k = 0..d-1 starting at +0.0f — bit-for-bit what
 *                        v_mfma_f32_32x32x2_f32 produces when one accumulator walks k in order.
 *   mode 1 (double):     score = sum in double of products of the (already rounded) inputs;
 *                        the reference for bf16 / f16 storage, compared with a tolerance.
 *   Ranking key: (score desc, row asc); scores that are NaN are never returned.
 *
 * Build: gcc -O2 -mfma -ffp-contract=off -fopenmp -shared -fPIC (see oracle/build.py).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

static float dot_fma_chain(const float* a, const float* b, int d) {
  float acc = 0.0f;
  for (int k = 0; k < d; ++k) acc = fmaf(a[k], b[k], acc);
  return acc;
}

static double dot_f64(const float* a, const float* b, int d) {
  double acc = 0.0;
  for (int k = 0; k < d; ++k) acc += (double)a[k] * (double)b[k];
  return acc;
}

/* (s1, r1) ranks before (s2, r2)? */
static int better(double s1, int64_t r1, double s2, int64_t r2) {
  return s1 > s2 || (s1 == s2 && r1 < r2);
}

/* Top-k of one query by insertion into a sorted list (k small). */
static void topk_one(const float* corpus, int64_t n, const float* q, int d, int k, int mode,
                     double* ls, int64_t* lr) {
  int fill = 0;
  for (int64_t r = 0; r < n; ++r) {
    const double s = mode == 0 ? (double)dot_fma_chain(corpus + r * d, q, d)
                               : dot_f64(corpus + r * d, q, d);
    if (s != s) continue; /* NaN */
    if (fill == k && !better(s, r, ls[k - 1], lr[k - 1])) continue;
    int j = fill < k ? fill++ : k - 1;
    while (j > 0 && better(s, r, ls[j - 1], lr[j - 1])) {
      ls[j] = ls[j - 1];
      lr[j] = lr[j - 1];
      --j;
    }
    ls[j] = s;
    lr[j] = r;
  }
  for (int j = fill; j < k; ++j) {
    ls[j] = -INFINITY;
    lr[j] = -1;
  }
}

/* corpus [n][d], queries [B][d] (fp32, already rounded to the storage dtype);
 * out_scores [B][k] (as double), out_rows [B][k]. Returns 0. */
int ahr_oracle_dense_topk(const float* corpus, int64_t n, const float* queries, int64_t B, int d,
                          int k, int mode, double* out_scores, int64_t* out_rows) {
  if (k <= 0 || d <= 0 || n < 0 || B < 0) return -1;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t b = 0; b < B; ++b)
    topk_one(corpus, n, queries + b * d, d, k, mode, out_scores + b * k, out_rows + b * k);
  return 0;
}

/* Full score matrix [B][n] (mode 0: fp32 fma chain; mode 1: double rounded to float). */
int ahr_oracle_scores(const float* corpus, int64_t n, const float* queries, int64_t B, int d,
                      int mode, float* out) {
  if (d <= 0 || n < 0 || B < 0) return -1;
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b)
    for (int64_t r = 0; r < n; ++r)
      out[b * n + r] = mode == 0 ? dot_fma_chain(corpus + r * d, queries + b * d, d)
                                 : (float)dot_f64(corpus + r * d, queries + b * d, d);
  return 0;
}

/* Round fp32 -> bf16 (round-to-nearest-even on the bit pattern; the device formula). */
void ahr_oracle_round_bf16(const float* in, float* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t u;
    memcpy(&u, &in[i], 4);
    u += 0x7FFFu + ((u >> 16) & 1u);
    u &= 0xFFFF0000u;
    memcpy(&out[i], &u, 4);
  }
}

int ahr_oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
