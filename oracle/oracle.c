/*
 * oracle.c -- CPU restatement of the Distributed Ranges shp/mhp hot path.
 * TEST INFRASTRUCTURE ONLY (see oracle.h): used by tests/, smoke() and the
 * cpu_baseline leg of bench.py; never by the product path.
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ------------------------------------------------------------------ */
/* partitioning                                                        */
/* ------------------------------------------------------------------ */

/* distributed_vector.hpp:142 + segments_tools.hpp:19-64 (take_segments). */
int orc_dv_segments(size_t n, int nprocs, size_t *lens) {
  size_t seg = (n + (size_t)nprocs - 1) / (size_t)nprocs;
  /* n_segs_remainder: walk until a segment holds the remainder. */
  size_t remainder = n;
  int last = 0;
  for (int i = 0; i < nprocs; i++) {
    if (seg >= remainder) break;
    remainder -= seg;
    last++;
  }
  for (int i = 0; i < last; i++) lens[i] = seg;
  lens[last] = remainder;
  return last + 1;
}

/* rng::subrange(first + b, first + e) over segments (drop_segments +
 * take_segments, segments_tools.hpp:37-94). Empty pieces are dropped,
 * as the algorithms skip/assert them anyway. */
int orc_subrange_segments(const size_t *lens, int nseg, size_t b, size_t e,
                          size_t *out, int *rank_out) {
  int cnt = 0;
  size_t base = 0;
  for (int s = 0; s < nseg; s++) {
    size_t lo = base, hi = base + lens[s];
    size_t a = lo > b ? lo : b;
    size_t z = hi < e ? hi : e;
    if (z > a) {
      out[cnt] = z - a;
      if (rank_out) rank_out[cnt] = s;
      cnt++;
    }
    base = hi;
  }
  return cnt;
}

/* zip_view.hpp:172-206 (get_next_segment_size / increment_local_idx). */
int orc_zip_pieces(const size_t *lens_r, int nr, const size_t *lens_o, int no,
                   size_t *piece_lens, int *piece_rank_r, int *piece_rank_o,
                   int cap) {
  size_t tot_r = 0, tot_o = 0;
  for (int i = 0; i < nr; i++) tot_r += lens_r[i];
  for (int i = 0; i < no; i++) tot_o += lens_o[i];
  size_t total = tot_r < tot_o ? tot_r : tot_o;
  int ir = 0, io = 0, cnt = 0;
  size_t lr = 0, lo = 0, done = 0;
  while (done < total && cnt < cap) {
    while (ir < nr && lr == lens_r[ir]) { ir++; lr = 0; }
    while (io < no && lo == lens_o[io]) { io++; lo = 0; }
    size_t a = lens_r[ir] - lr, b = lens_o[io] - lo;
    size_t sz = a < b ? a : b;
    if (sz > total - done) sz = total - done;
    piece_lens[cnt] = sz;
    if (piece_rank_r) piece_rank_r[cnt] = ir;
    if (piece_rank_o) piece_rank_o[cnt] = io;
    cnt++;
    lr += sz; lo += sz; done += sz;
  }
  return cnt;
}

/* ------------------------------------------------------------------ */
/* binary ops                                                          */
/* ------------------------------------------------------------------ */

#define OP_INT(U, a, b, op)                                                  \
  ((op) == ORC_PLUS ? (U)((a) + (b))                                         \
   : (op) == ORC_MUL ? (U)((a) * (b))                                        \
   : (op) == ORC_MIN ? ((b) < (a) ? (b) : (a))                               \
                     : ((a) < (b) ? (b) : (a)))

static inline int32_t op_i32(int32_t a, int32_t b, int op) {
  if (op == ORC_PLUS) return (int32_t)((uint32_t)a + (uint32_t)b);
  if (op == ORC_MUL) return (int32_t)((uint32_t)a * (uint32_t)b);
  if (op == ORC_MIN) return b < a ? b : a;
  return a < b ? b : a;
}
static inline int64_t op_i64(int64_t a, int64_t b, int op) {
  if (op == ORC_PLUS) return (int64_t)((uint64_t)a + (uint64_t)b);
  if (op == ORC_MUL) return (int64_t)((uint64_t)a * (uint64_t)b);
  if (op == ORC_MIN) return b < a ? b : a;
  return a < b ? b : a;
}
static inline uint32_t op_u32(uint32_t a, uint32_t b, int op) { return OP_INT(uint32_t, a, b, op); }
static inline uint64_t op_u64(uint64_t a, uint64_t b, int op) { return OP_INT(uint64_t, a, b, op); }
static inline float op_f32(float a, float b, int op) {
  if (op == ORC_PLUS) return a + b;
  if (op == ORC_MUL) return a * b;
  if (op == ORC_MIN) return b < a ? b : a;
  return a < b ? b : a;
}
static inline double op_f64(double a, double b, int op) {
  if (op == ORC_PLUS) return a + b;
  if (op == ORC_MUL) return a * b;
  if (op == ORC_MIN) return b < a ? b : a;
  return a < b ? b : a;
}

/* ------------------------------------------------------------------ */
/* shp::reduce -- reduce.hpp:40-88                                     */
/* ------------------------------------------------------------------ */

#define DEFINE_SHP_REDUCE(SUF, T)                                            \
  T orc_shp_reduce_##SUF(const T *x, const size_t *lens, int nseg, T init,   \
                         int op) {                                           \
    T *partials = (T *)malloc(sizeof(T) * (size_t)(nseg > 0 ? nseg : 1));    \
    int np = 0;                                                              \
    size_t base = 0;                                                         \
    for (int s = 0; s < nseg; s++) {                                         \
      const T *seg = x + base;                                               \
      size_t len = lens[s];                                                  \
      base += len;                                                           \
      if (len == 0) continue;             /* reduce.hpp:67-68 */             \
      if (len == 1) {                     /* reduce.hpp:69-71 */             \
        init = op_##SUF(init, seg[0], op);                                   \
        continue;                                                            \
      }                                                                      \
      T acc = seg[len - 1];               /* reduce.hpp:26-33 */             \
      for (size_t i = 0; i + 1 < len; i++) acc = op_##SUF(acc, seg[i], op);  \
      partials[np++] = acc;                                                  \
    }                                                                        \
    for (int k = 0; k < np; k++)          /* reduce.hpp:81-83 */             \
      init = op_##SUF(init, partials[k], op);                                \
    free(partials);                                                          \
    return init;                                                             \
  }

DEFINE_SHP_REDUCE(i32, int32_t)
DEFINE_SHP_REDUCE(u32, uint32_t)
DEFINE_SHP_REDUCE(i64, int64_t)
DEFINE_SHP_REDUCE(u64, uint64_t)
DEFINE_SHP_REDUCE(f32, float)
DEFINE_SHP_REDUCE(f64, double)

static double exact_fold(const void *px, int is_f32, size_t n, double init, int op) {
  const float *xf = (const float *)px;
  const double *xd = (const double *)px;
#define XV(i) (is_f32 ? (double)xf[i] : xd[i])
  if (op == ORC_PLUS) {
    /* Neumaier compensated summation in fp64. */
    double s = init, c = 0.0;
    for (size_t i = 0; i < n; i++) {
      double v = XV(i);
      double t = s + v;
      if (fabs(s) >= fabs(v)) c += (s - t) + v;
      else c += (v - t) + s;
      s = t;
    }
    return s + c;
  }
  double acc = init;
  for (size_t i = 0; i < n; i++) acc = op_f64(acc, XV(i), op);
  return acc;
#undef XV
}

double orc_reduce_exact_f32(const float *x, size_t n, double init, int op) {
  return exact_fold(x, 1, n, init, op);
}
double orc_reduce_exact_f64(const double *x, size_t n, double init, int op) {
  return exact_fold(x, 0, n, init, op);
}

/* dot_product.cpp:11-18: reduce(zip(x,y) | transform(a*b), 0, plus). */
double orc_dot_f32(const float *x, const float *y, size_t n, double init) {
  double s = init;
  for (size_t i = 0; i < n; i++) s += (double)x[i] * (double)y[i];
  return s;
}
double orc_dot_f64(const double *x, const double *y, size_t n, double init) {
  double s = init, c = 0.0;
  for (size_t i = 0; i < n; i++) {
    double v = x[i] * y[i];
    double t = s + v;
    if (fabs(s) >= fabs(v)) c += (s - t) + v;
    else c += (v - t) + s;
    s = t;
  }
  return s + c;
}
int32_t orc_dot_i32(const int32_t *x, const int32_t *y, size_t n, int32_t init) {
  uint32_t s = (uint32_t)init;
  for (size_t i = 0; i < n; i++) s += (uint32_t)x[i] * (uint32_t)y[i];
  return (int32_t)s;
}

/* ------------------------------------------------------------------ */
/* shp::inclusive_scan -- inclusive_scan.hpp:22-148                    */
/* ------------------------------------------------------------------ */

#define DEFINE_SHP_SCAN(SUF, T)                                              \
  void orc_shp_scan_##SUF(const T *in, T *out, const size_t *pieces, int np, \
                          int op, int has_init, T init) {                    \
    T *partial = (T *)malloc(sizeof(T) * (size_t)(np > 0 ? np : 1));         \
    size_t base = 0;                                                         \
    /* phase 1: local scans (:77-96) */                                      \
    for (int k = 0; k < np; k++) {                                           \
      size_t len = pieces[k];                                                \
      const T *a = in + base;                                                \
      T *o = out + base;                                                     \
      T acc;                                                                 \
      if (k == 0 && has_init) acc = op_##SUF(init, a[0], op);                \
      else acc = a[0];                                                       \
      o[0] = acc;                                                            \
      for (size_t i = 1; i < len; i++) {                                     \
        acc = op_##SUF(acc, a[i], op);                                       \
        o[i] = acc;                                                          \
      }                                                                      \
      partial[k] = o[len - 1];                                               \
      base += len;                                                           \
    }                                                                        \
    /* phase 2: scan of the partials on the root (:108-116) */               \
    for (int k = 1; k < np; k++)                                             \
      partial[k] = op_##SUF(partial[k - 1], partial[k], op);                 \
    /* phase 3: carry, right operand (:118-143) */                           \
    base = 0;                                                                \
    for (int k = 0; k < np; k++) {                                           \
      size_t len = pieces[k];                                                \
      if (k > 0) {                                                           \
        T c = partial[k - 1];                                                \
        for (size_t i = 0; i < len; i++)                                     \
          out[base + i] = op_##SUF(out[base + i], c, op);                    \
      }                                                                      \
      base += len;                                                           \
    }                                                                        \
    free(partial);                                                           \
  }

DEFINE_SHP_SCAN(i32, int32_t)
DEFINE_SHP_SCAN(u32, uint32_t)
DEFINE_SHP_SCAN(i64, int64_t)
DEFINE_SHP_SCAN(u64, uint64_t)
DEFINE_SHP_SCAN(f32, float)
DEFINE_SHP_SCAN(f64, double)

void orc_scan_exact_f32(const float *in, double *out, size_t n, int op, int has_init,
                        double init) {
  if (n == 0) return;
  double acc = has_init ? op_f64(init, (double)in[0], op) : (double)in[0];
  out[0] = acc;
  for (size_t i = 1; i < n; i++) {
    acc = op_f64(acc, (double)in[i], op);
    out[i] = acc;
  }
}

/* ------------------------------------------------------------------ */
/* mhp CPU path (cpu_algorithms.hpp:102-140) -- the CPU baseline        */
/* ------------------------------------------------------------------ */

static inline int clamp_threads(int t) { return t < 1 ? 1 : t; }

double orc_mhp_reduce_f32(const float *x, size_t n, int nranks, double init, int nthreads) {
  size_t seg = (n + (size_t)nranks - 1) / (size_t)nranks;
  double *locals = (double *)calloc((size_t)nranks, sizeof(double));
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (int r = 0; r < nranks; r++) {
    size_t lo = (size_t)r * seg, hi = lo + seg < n ? lo + seg : n;
    /* std::reduce(par_unseq, seg, T(0), plus): 4 independent fp32
     * accumulators per rank then fp64 combine (vectorisable, like PSTL). */
    double acc = 0.0;
    size_t i = lo;
    float a0 = 0, a1 = 0, a2 = 0, a3 = 0, a4 = 0, a5 = 0, a6 = 0, a7 = 0;
    for (; lo < hi && i + 8 <= hi; i += 8) {
      a0 += x[i]; a1 += x[i + 1]; a2 += x[i + 2]; a3 += x[i + 3];
      a4 += x[i + 4]; a5 += x[i + 5]; a6 += x[i + 6]; a7 += x[i + 7];
      if (((i - lo) & 0xFFFF) == 0xFFF8) { /* flush every 64K to bound fp32 error */
        acc += (double)a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
        a0 = a1 = a2 = a3 = a4 = a5 = a6 = a7 = 0;
      }
    }
    acc += (double)a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    for (; i < hi; i++) acc += x[i];
    locals[r] = acc;
  }
  /* gather to root + root fold with init (:121-129) */
  double result = init;
  for (int r = 0; r < nranks; r++) result += locals[r];
  free(locals);
  return result;
}

int32_t orc_mhp_reduce_i32(const int32_t *x, size_t n, int nranks, int32_t init, int nthreads) {
  size_t seg = (n + (size_t)nranks - 1) / (size_t)nranks;
  uint32_t *locals = (uint32_t *)calloc((size_t)nranks, sizeof(uint32_t));
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (int r = 0; r < nranks; r++) {
    size_t lo = (size_t)r * seg, hi = lo + seg < n ? lo + seg : n;
    uint32_t acc = 0;
    for (size_t i = lo; i < hi; i++) acc += (uint32_t)x[i];
    locals[r] = acc;
  }
  uint32_t result = (uint32_t)init;
  for (int r = 0; r < nranks; r++) result += locals[r];
  free(locals);
  return (int32_t)result;
}

void orc_mhp_scan_f32(const float *in, float *out, size_t n, int nranks, int nthreads) {
  size_t seg = (n + (size_t)nranks - 1) / (size_t)nranks;
  double *tot = (double *)calloc((size_t)nranks + 1, sizeof(double));
  /* phase 1: local scans with fp64 running sums (fp32 sequential is not
   * accurate at these sizes: SURVEY.md 8d) */
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (int r = 0; r < nranks; r++) {
    size_t lo = (size_t)r * seg, hi = lo + seg < n ? lo + seg : n;
    double acc = 0.0;
    for (size_t i = lo; i < hi; i++) { acc += in[i]; out[i] = (float)acc; }
    tot[r + 1] = acc;
  }
  /* phase 2: exclusive prefix of rank totals */
  for (int r = 1; r <= nranks; r++) tot[r] += tot[r - 1];
  /* phase 3: carry pass, recomputed from the input in fp64 so the result is
   * the fp64 prefix rounded once */
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (int r = 1; r < nranks; r++) {
    size_t lo = (size_t)r * seg, hi = lo + seg < n ? lo + seg : n;
    double acc = tot[r];
    for (size_t i = lo; i < hi; i++) { acc += in[i]; out[i] = (float)acc; }
  }
  free(tot);
}

void orc_mhp_scan_i32(const int32_t *in, int32_t *out, size_t n, int nranks, int nthreads) {
  size_t seg = (n + (size_t)nranks - 1) / (size_t)nranks;
  uint32_t *tot = (uint32_t *)calloc((size_t)nranks + 1, sizeof(uint32_t));
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (int r = 0; r < nranks; r++) {
    size_t lo = (size_t)r * seg, hi = lo + seg < n ? lo + seg : n;
    uint32_t acc = 0;
    for (size_t i = lo; i < hi; i++) { acc += (uint32_t)in[i]; out[i] = (int32_t)acc; }
    tot[r + 1] = acc;
  }
  for (int r = 1; r <= nranks; r++) tot[r] += tot[r - 1];
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (int r = 1; r < nranks; r++) {
    size_t lo = (size_t)r * seg, hi = lo + seg < n ? lo + seg : n;
    uint32_t c = tot[r];
    for (size_t i = lo; i < hi; i++) out[i] = (int32_t)((uint32_t)out[i] + c);
  }
  free(tot);
}

/* ------------------------------------------------------------------ */
/* CSR SpMV -- intended semantics of gemv.hpp:13-71                     */
/* ------------------------------------------------------------------ */

void orc_csr_spmv_f32_i32(size_t m, const int32_t *rowptr, const int32_t *colind,
                          const float *vals, const float *x, const float *y_in,
                          double *y_out) {
  for (size_t i = 0; i < m; i++) {
    double acc = y_in ? (double)y_in[i] : 0.0;
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; k++)
      acc += (double)vals[k] * (double)x[colind[k]];
    y_out[i] = acc;
  }
}
void orc_csr_spmv_f64_i32(size_t m, const int32_t *rowptr, const int32_t *colind,
                          const double *vals, const double *x, const double *y_in,
                          double *y_out) {
  for (size_t i = 0; i < m; i++) {
    double acc = y_in ? y_in[i] : 0.0;
    for (int32_t k = rowptr[i]; k < rowptr[i + 1]; k++) acc += vals[k] * x[colind[k]];
    y_out[i] = acc;
  }
}

/* splitmix64-style mixer; identical definition in csrc/spmv.hip. */
uint64_t orc_hash3(uint64_t seed, uint64_t i, uint64_t j) {
  uint64_t z = seed * 0x9E3779B97F4A7C15ull + i * 0xBF58476D1CE4E5B9ull +
               j * 0x94D049BB133111EBull + 0x2545F4914F6CDD1Dull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
float orc_u01(uint64_t seed, uint64_t i, uint64_t j) {
  return (float)(orc_hash3(seed, i, j) >> 40) * (1.0f / 16777216.0f);
}

#define BAND_LO 4
#define BAND_HI 5
static inline size_t band_begin(size_t i) { return i >= BAND_LO ? i - BAND_LO : 0; }
static inline size_t band_end(size_t i, size_t ncols) {
  size_t e = i + BAND_HI + 1;
  return e < ncols ? e : ncols;
}
static size_t band_len(size_t i, size_t ncols) {
  size_t b = band_begin(i), e = band_end(i, ncols);
  return e > b ? e - b : 0;
}

size_t orc_csr_banded_nnz(size_t m, size_t ncols) {
  size_t s = 0;
  for (size_t i = 0; i < m; i++) s += band_len(i, ncols);
  return s;
}

void orc_csr_gen_banded_f32(size_t row0, size_t nrows, size_t ncols, uint64_t seed,
                            int32_t *rowptr, int32_t *colind, float *vals) {
  int32_t nnz = 0;
  for (size_t r = 0; r < nrows; r++) {
    size_t i = row0 + r;
    rowptr[r] = nnz;
    for (size_t c = band_begin(i); c < band_end(i, ncols); c++) {
      colind[nnz] = (int32_t)c;
      vals[nnz] = orc_u01(seed, i, c);
      nnz++;
    }
  }
  rowptr[nrows] = nnz;
}

void orc_csr_gen_random_f32(size_t row0, size_t nrows, size_t ncols, int k, uint64_t seed,
                            int32_t *rowptr, int32_t *colind, float *vals) {
  int kk = (size_t)k < ncols ? k : (int)ncols;
  for (size_t r = 0; r < nrows; r++) {
    size_t i = row0 + r;
    int32_t *c = colind + r * (size_t)kk;
    int cnt = 0;
    for (uint64_t j = 0; cnt < kk; j++) {
      int32_t cand = (int32_t)(orc_hash3(seed ^ 0x5bd1e995ull, i, j) % ncols);
      int dup = 0;
      for (int q = 0; q < cnt; q++) dup |= (c[q] == cand);
      if (!dup) c[cnt++] = cand;
    }
    /* insertion sort ascending */
    for (int a = 1; a < kk; a++) {
      int32_t v = c[a];
      int b = a - 1;
      while (b >= 0 && c[b] > v) { c[b + 1] = c[b]; b--; }
      c[b + 1] = v;
    }
    for (int a = 0; a < kk; a++) vals[r * (size_t)kk + a] = orc_u01(seed, i, (uint64_t)c[a]);
    rowptr[r] = (int32_t)(r * (size_t)kk);
  }
  rowptr[nrows] = (int32_t)(nrows * (size_t)kk);
}

/* Density generator: sparse_matrix(shape, density) (containers/
 * sparse_matrix.hpp:157-166) with generate_random_csr's entry count
 * floor(density*m*n) (util/generate_random.hpp:37), spread evenly over rows,
 * one column per equal-width stratum of each row; values as doubles (U[0,1)
 * floats, or {0,1} hash bits when int_values).  Same definition as the
 * device gen_density (csrc/spmv.hip). */
static size_t dens_prefix(size_t i, size_t m, size_t nnz) {
  return m ? (size_t)(((unsigned __int128)i * nnz) / m) : 0;
}
size_t orc_csr_density_nnz(size_t row0, size_t nrows, size_t m, size_t ncols, double density) {
  size_t tot = (size_t)(density * (double)m * (double)ncols);
  return dens_prefix(row0 + nrows, m, tot) - dens_prefix(row0, m, tot);
}
void orc_csr_gen_density(size_t row0, size_t nrows, size_t m, size_t ncols, double density, uint64_t seed,
                         int int_values, int64_t *rowptr, int64_t *colind, double *vals) {
  size_t tot = (size_t)(density * (double)m * (double)ncols);
  size_t base = dens_prefix(row0, m, tot);
  for (size_t r = 0; r <= nrows; r++) {
    size_t i = row0 + r;
    size_t off = dens_prefix(i, m, tot) - base;
    rowptr[r] = (int64_t)off;
    if (r == nrows) break;
    size_t k = dens_prefix(i + 1, m, tot) - dens_prefix(i, m, tot);
    for (size_t q = 0; q < k; q++) {
      size_t lo = (size_t)(((unsigned __int128)q * ncols) / k);
      size_t hi = (size_t)(((unsigned __int128)(q + 1) * ncols) / k);
      size_t c = lo + orc_hash3(seed ^ 0x2545F491ull, i, q) % (hi - lo);
      colind[off + q] = (int64_t)c;
      vals[off + q] = int_values ? (double)(orc_hash3(seed, i, c) >> 63) : (double)orc_u01(seed, i, c);
    }
  }
}

/* ------------------------------------------------------------------ */
/* sort -- std::sort semantics (no reference implementation exists)     */
/* ------------------------------------------------------------------ */

static int cmp_u32(const void *a, const void *b) {
  uint32_t x = *(const uint32_t *)a, y = *(const uint32_t *)b;
  return (x > y) - (x < y);
}
static int cmp_i32(const void *a, const void *b) {
  int32_t x = *(const int32_t *)a, y = *(const int32_t *)b;
  return (x > y) - (x < y);
}
static int cmp_f32(const void *a, const void *b) {
  float x = *(const float *)a, y = *(const float *)b;
  return (x > y) - (x < y);
}
void orc_sort_u32(uint32_t *x, size_t n) { qsort(x, n, sizeof(uint32_t), cmp_u32); }
void orc_sort_i32(int32_t *x, size_t n) { qsort(x, n, sizeof(int32_t), cmp_i32); }
void orc_sort_f32(float *x, size_t n) { qsort(x, n, sizeof(float), cmp_f32); }
static int cmp_u64(const void *a, const void *b) {
  uint64_t x = *(const uint64_t *)a, y = *(const uint64_t *)b;
  return (x > y) - (x < y);
}
static int cmp_i64(const void *a, const void *b) {
  int64_t x = *(const int64_t *)a, y = *(const int64_t *)b;
  return (x > y) - (x < y);
}
static int cmp_f64(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return (x > y) - (x < y);
}
/* Counting-sort form of the same ordering for BASELINE-sized uint32 inputs
 * (C3: 2^28 keys per GPU, where qsort takes ~70 s): four stable 8-bit LSD
 * passes through a scratch array.  Any correct sort of keys gives the same
 * bytes as std::sort; tests/test_oracle.py pins it to orc_sort_u32. */
int orc_radix_sort_u32(uint32_t *x, size_t n) {
  uint32_t *tmp = (uint32_t *)malloc(n ? n * sizeof(uint32_t) : 4);
  if (!tmp) return -1;
  uint32_t *src = x, *dst = tmp;
  for (int shift = 0; shift < 32; shift += 8) {
    size_t cnt[257] = {0};
    for (size_t i = 0; i < n; i++) cnt[((src[i] >> shift) & 255u) + 1]++;
    for (int d = 0; d < 256; d++) cnt[d + 1] += cnt[d];
    for (size_t i = 0; i < n; i++) dst[cnt[(src[i] >> shift) & 255u]++] = src[i];
    uint32_t *t = src;
    src = dst;
    dst = t;
  }
  /* four passes: the result is back in x */
  free(tmp);
  return 0;
}

/* The same stable LSD order with every pass split over nthreads static
 * chunks (per-thread digit counts, offsets in (digit, thread) order, each
 * thread scatters its chunk in input order): identical output to
 * orc_radix_sort_u32, for the 2^31-key C3 check (tests/cpp/config_tests). */
int orc_radix_sort_u32_par(uint32_t *x, size_t n, int nthreads) {
  const int T = clamp_threads(nthreads);
  uint32_t *tmp = (uint32_t *)malloc(n ? n * sizeof(uint32_t) : 4);
  size_t *cnt = (size_t *)calloc((size_t)T * 256, sizeof(size_t));
  if (!tmp || !cnt) {
    free(tmp);
    free(cnt);
    return -1;
  }
  uint32_t *src = x, *dst = tmp;
  for (int shift = 0; shift < 32; shift += 8) {
    memset(cnt, 0, (size_t)T * 256 * sizeof(size_t));
#pragma omp parallel num_threads(T)
    {
      const int t = omp_get_thread_num();
      const size_t a = n * (size_t)t / (size_t)T, b = n * (size_t)(t + 1) / (size_t)T;
      size_t *c = cnt + (size_t)t * 256;
      for (size_t i = a; i < b; i++) c[(src[i] >> shift) & 255u]++;
#pragma omp barrier
#pragma omp single
      {
        size_t run = 0;
        for (int d = 0; d < 256; d++)
          for (int u = 0; u < T; u++) {
            const size_t v = cnt[(size_t)u * 256 + d];
            cnt[(size_t)u * 256 + d] = run;
            run += v;
          }
      }
      for (size_t i = a; i < b; i++) dst[c[(src[i] >> shift) & 255u]++] = src[i];
    }
    uint32_t *t = src;
    src = dst;
    dst = t;
  }
  free(tmp);
  free(cnt);
  return 0;
}

/* x[i] = high 32 bits of splitmix64(seed + start + i): the synthetic C3
 * keys of tests/cpp/config_tests.cpp (its device generator is the same
 * function). */
static inline uint64_t splitmix64_at(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
void orc_fill_hash_u32(uint32_t *x, size_t n, uint64_t seed, uint64_t start, int nthreads) {
#pragma omp parallel for num_threads(clamp_threads(nthreads)) schedule(static)
  for (size_t i = 0; i < n; i++) x[i] = (uint32_t)(splitmix64_at(seed + start + i) >> 32);
}

void orc_sort_u64(uint64_t *x, size_t n) { qsort(x, n, sizeof(uint64_t), cmp_u64); }
void orc_sort_i64(int64_t *x, size_t n) { qsort(x, n, sizeof(int64_t), cmp_i64); }
void orc_sort_f64(double *x, size_t n) { qsort(x, n, sizeof(double), cmp_f64); }

/* ------------------------------------------------------------------ */
/* stencils -- halo.hpp:336-387, stencil-1d.cpp:16-66, stencil.cpp       */
/* ------------------------------------------------------------------ */

void orc_stencil1d_i32(const int32_t *in, int32_t *out, size_t n, int radius) {
  size_t r = (size_t)radius;
  for (size_t i = r; i + r < n; i++) {
    uint32_t s = 0;
    for (size_t d = i - r; d <= i + r; d++) s += (uint32_t)in[d];
    out[i] = (int32_t)s;
  }
}
void orc_stencil1d_f32(const float *in, float *out, size_t n, int radius) {
  size_t r = (size_t)radius;
  for (size_t i = r; i + r < n; i++) {
    /* p[-r] + ... + p[+r] left to right (stencil-1d.cpp:16-19): the sum
       starts from the first term, so signed zeros come out as the
       reference's do */
    float s = in[i - r];
    for (size_t d = i - r + 1; d <= i + r; d++) s += in[d];
    out[i] = s;
  }
}

void orc_stencil_mhp_test_op_i32(const int32_t *in, int32_t *out, size_t n, int radius) {
  size_t r = (size_t)radius;
  for (size_t i = r; i + r < n; i++) {
    uint32_t s = (uint32_t)in[i];
    for (size_t k = 0; k <= r; k++) s += (uint32_t)in[i - k] + (uint32_t)in[i + k];
    out[i] = (int32_t)s;
  }
}

/* Distributed 1-D 3-point stencil, `steps` steps of
 * stencil-1d.cpp:47-59 (in = a[1..n-1), out = b[1..n-1), swap) on `nranks`
 * mhp ranks with halo radius 1.  Each rank keeps a buffer
 * [1 halo | seg owned | 1 halo] (mhp/containers/distributed_vector.hpp:
 * 190-200); exchange() copies the first owned cell to rank-1's next halo
 * and the last owned cell (buffer tail, halo.hpp:364-368) to rank+1's prev
 * halo.  Results land back in a (even steps) or b (odd steps), exactly as
 * the serial swap; returns 0 if a is current, 1 if b is. */
int orc_stencil1d_mhp_steps_i32(int32_t *a, int32_t *b, size_t n, int nranks, int steps) {
  size_t seg = (n + (size_t)nranks - 1) / (size_t)nranks;
  if (seg < 1) seg = 1;
  size_t bsz = seg + 2;
  int32_t *buf[2];
  buf[0] = (int32_t *)calloc(bsz * (size_t)nranks, sizeof(int32_t));
  buf[1] = (int32_t *)calloc(bsz * (size_t)nranks, sizeof(int32_t));
  for (int r = 0; r < nranks; r++)
    for (size_t l = 0; l < seg && r * seg + l < n; l++) {
      buf[0][r * bsz + 1 + l] = a[r * seg + l];
      buf[1][r * bsz + 1 + l] = b[r * seg + l];
    }
  int cur = 0;
  for (int s = 0; s < steps; s++) {
    int32_t *in = buf[cur], *out = buf[cur ^ 1];
    /* halo exchange (non-periodic): owned groups -> neighbours' halo groups */
    for (int r = 0; r < nranks; r++) {
      int32_t *me = in + r * bsz;
      if (r > 0) in[(r - 1) * bsz + bsz - 1] = me[1];      /* halo_reverse */
      if (r + 1 < nranks) in[(r + 1) * bsz + 0] = me[bsz - 2]; /* halo_forward */
    }
    /* transform over the global interior [1, n-1) restricted per rank */
    for (int r = 0; r < nranks; r++) {
      for (size_t l = 0; l < seg; l++) {
        size_t g = r * seg + l;
        if (g < 1 || g + 1 >= n) continue;
        const int32_t *p = in + r * bsz + 1 + l;
        out[r * bsz + 1 + l] = (int32_t)((uint32_t)p[-1] + (uint32_t)p[0] + (uint32_t)p[1]);
      }
    }
    cur ^= 1;
  }
  /* write back both buffers */
  for (int r = 0; r < nranks; r++)
    for (size_t l = 0; l < seg && r * seg + l < n; l++) {
      a[r * seg + l] = buf[0][r * bsz + 1 + l];
      b[r * seg + l] = buf[1][r * bsz + 1 + l];
    }
  free(buf[0]);
  free(buf[1]);
  return cur;
}

void orc_stencil2d_f32(const float *in, float *out, size_t nx, size_t ny) {
  for (size_t y = 1; y + 1 < ny; y++)
    for (size_t x = 1; x + 1 < nx; x++) {
      size_t i = y * nx + x;
      out[i] = in[i] + in[i - 1] + in[i + 1] + in[i - nx] + in[i + nx];
    }
}

/* ------------------------------------------------------------------ */
/* lrand48 stream (test/gtest/shp/algorithms.cpp:69-70)                 */
/* ------------------------------------------------------------------ */

void orc_lrand48_mod(int32_t *out, size_t n, int32_t mod, int reseed) {
  if (reseed) {
    /* glibc's unseeded drand48 state is zero-initialised (X0 = 0), which is
     * what the reference test sees: it never calls srand48. */
    unsigned short s[3] = {0, 0, 0};
    seed48(s);
  }
  for (size_t i = 0; i < n; i++) out[i] = (int32_t)(lrand48() % mod);
}
