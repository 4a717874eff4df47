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
 * Build: gcc -O3 -mavx2 -mfma -ffp-contract=off -fopenmp -shared -fPIC (see oracle/build.py).
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

/* Query blocks: QB queries share every corpus row load; their k-ordered chains run side by side
 * (one SIMD lane per query, each lane still one fmaf chain in k order = mode 0's contract). */
#define QB 32

static void topk_block(const float* corpus, int64_t n, const float* queries, int64_t nq, int d,
                       int k, int mode, double* out_scores, int64_t* out_rows) {
  float* qt = (float*)malloc(sizeof(float) * (size_t)d * QB);      /* [d][QB] transposed */
  double* qd = (double*)malloc(sizeof(double) * (size_t)d * QB);
  double* ls = (double*)malloc(sizeof(double) * (size_t)k * QB);
  int64_t* lr = (int64_t*)malloc(sizeof(int64_t) * (size_t)k * QB);
  int fill[QB];
  for (int j = 0; j < QB; ++j) fill[j] = 0;
  for (int kk = 0; kk < d; ++kk)
    for (int j = 0; j < QB; ++j) {
      const float v = j < nq ? queries[(int64_t)j * d + kk] : 0.0f;
      qt[(size_t)kk * QB + j] = v;
      qd[(size_t)kk * QB + j] = (double)v;
    }
  for (int64_t r = 0; r < n; ++r) {
    const float* row = corpus + r * d;
    double s[QB];
    if (mode == 0) {
      float acc[QB];
      for (int j = 0; j < QB; ++j) acc[j] = 0.0f;
      for (int kk = 0; kk < d; ++kk) {
        const float c = row[kk];
        const float* qk = qt + (size_t)kk * QB;
        for (int j = 0; j < QB; ++j) acc[j] = fmaf(c, qk[j], acc[j]);
      }
      for (int j = 0; j < QB; ++j) s[j] = (double)acc[j];
    } else {
      double acc[QB];
      for (int j = 0; j < QB; ++j) acc[j] = 0.0;
      for (int kk = 0; kk < d; ++kk) {
        const double c = (double)row[kk];
        const double* qk = qd + (size_t)kk * QB;
        for (int j = 0; j < QB; ++j) acc[j] = acc[j] + c * qk[j];
      }
      for (int j = 0; j < QB; ++j) s[j] = acc[j];
    }
    for (int j = 0; j < nq; ++j) {
      double* L = ls + (size_t)j * k;
      int64_t* R = lr + (size_t)j * k;
      const double sc = s[j];
      if (sc != sc) continue; /* NaN */
      if (fill[j] == k && !better(sc, r, L[k - 1], R[k - 1])) continue;
      int p = fill[j] < k ? fill[j]++ : k - 1;
      while (p > 0 && better(sc, r, L[p - 1], R[p - 1])) {
        L[p] = L[p - 1];
        R[p] = R[p - 1];
        --p;
      }
      L[p] = sc;
      R[p] = r;
    }
  }
  for (int j = 0; j < nq; ++j) {
    for (int p = 0; p < k; ++p) {
      out_scores[(int64_t)j * k + p] = p < fill[j] ? ls[(size_t)j * k + p] : -INFINITY;
      out_rows[(int64_t)j * k + p] = p < fill[j] ? lr[(size_t)j * k + p] : -1;
    }
  }
  free(qt);
  free(qd);
  free(ls);
  free(lr);
}

/* corpus [n][d], queries [B][d] (fp32, already rounded to the storage dtype);
 * out_scores [B][k] (as double), out_rows [B][k]. Returns 0.
 * Few query blocks (small B over a large corpus): the rows are cut into chunks, each chunk's
 * top-k is found per block in parallel, and the chunk lists are merged with the same ranking
 * key, which gives the same answer as one pass (top-k of a union = top-k of the parts' top-k). */
int ahr_oracle_dense_topk(const float* corpus, int64_t n, const float* queries, int64_t B, int d,
                          int k, int mode, double* out_scores, int64_t* out_rows) {
  if (k <= 0 || d <= 0 || n < 0 || B < 0) return -1;
  const int64_t nblk = (B + QB - 1) / QB;
  int nth = 1;
#ifdef _OPENMP
  nth = omp_get_max_threads();
#endif
  int64_t nchunk = 1;
  if (nblk < nth && n >= 8192) {
    nchunk = (4 * nth + nblk - 1) / nblk;
    if (nchunk > n / 2048) nchunk = n / 2048;
    if (nchunk < 1) nchunk = 1;
  }
  if (nchunk == 1) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t bb = 0; bb < nblk; ++bb) {
      const int64_t b0 = bb * QB;
      const int64_t nq = B - b0 < QB ? B - b0 : QB;
      topk_block(corpus, n, queries + b0 * d, nq, d, k, mode, out_scores + b0 * k, out_rows + b0 * k);
    }
    return 0;
  }
  const int64_t per = (n + nchunk - 1) / nchunk;
  double* ps = (double*)malloc(sizeof(double) * (size_t)(nchunk * B * k));
  int64_t* pr = (int64_t*)malloc(sizeof(int64_t) * (size_t)(nchunk * B * k));
  if (!ps || !pr) {
    free(ps);
    free(pr);
    return -2;
  }
#pragma omp parallel for schedule(dynamic, 1) collapse(2)
  for (int64_t c = 0; c < nchunk; ++c)
    for (int64_t bb = 0; bb < nblk; ++bb) {
      const int64_t r0 = c * per;
      const int64_t r1 = r0 + per < n ? r0 + per : n;
      const int64_t b0 = bb * QB;
      const int64_t nq = B - b0 < QB ? B - b0 : QB;
      double* os = ps + (c * B + b0) * k;
      int64_t* orow = pr + (c * B + b0) * k;
      topk_block(corpus + r0 * d, r1 > r0 ? r1 - r0 : 0, queries + b0 * d, nq, d, k, mode, os, orow);
      for (int64_t i = 0; i < nq * k; ++i)
        if (orow[i] >= 0) orow[i] += r0;
    }
  /* merge: chunk c's list for query b is ps[(c*B + b)*k ...] */
#pragma omp parallel for schedule(static)
  for (int64_t b = 0; b < B; ++b) {
    double* L = out_scores + b * k;
    int64_t* R = out_rows + b * k;
    int fill = 0;
    for (int64_t c = 0; c < nchunk; ++c)
      for (int j = 0; j < k; ++j) {
        const double sc = ps[(c * B + b) * k + j];
        const int64_t r = pr[(c * B + b) * k + j];
        if (r < 0) break;
        if (fill == k && !better(sc, r, L[k - 1], R[k - 1])) break; /* lists are sorted */
        int p = fill < k ? fill++ : k - 1;
        while (p > 0 && better(sc, r, L[p - 1], R[p - 1])) {
          L[p] = L[p - 1];
          R[p] = R[p - 1];
          --p;
        }
        L[p] = sc;
        R[p] = r;
      }
    for (int j = fill; j < k; ++j) {
      L[j] = -INFINITY;
      R[j] = -1;
    }
  }
  free(ps);
  free(pr);
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
