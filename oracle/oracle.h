/*
 * oracle.h -- CPU restatement of the Distributed Ranges shp/mhp hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path (libdrhip.so, the
 * C++ shp header layer, bench.py's measured legs) links, loads or calls
 * this code.  Only tests/, __graft_entry__.smoke() and bench.py's
 * `cpu_baseline` leg use it, and only as the checker / CPU baseline.
 *
 * Reference: sudhirverma/distributed-ranges @ 2025-03-03 (read-only at
 * /root/reference; never shipped).  Every function cites the reference
 * file:line whose semantics it restates.  The reference itself cannot be
 * compiled here (range-v3, oneDPL and SYCL are FetchContent downloads and
 * absent offline -- SURVEY.md 8c), so parity is pinned by the known answers
 * in the reference's own tests (tests/golden/, tests/test_oracle.py).
 *
 * Integer arithmetic is done in unsigned types so that wrapping int32/int64
 * `+`/`*` (e.g. the product scan of test/gtest/shp/algorithms.cpp:100-102)
 * is well defined and bit-exact.
 */
#ifndef DR_ORACLE_H
#define DR_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Operation codes shared with include/drhip.h (same numeric values). */
enum { ORC_PLUS = 0, ORC_MUL = 1, ORC_MIN = 2, ORC_MAX = 3 };
/* Element type codes shared with include/drhip.h. */
enum { ORC_I32 = 0, ORC_U32 = 1, ORC_I64 = 2, ORC_U64 = 3, ORC_F32 = 4, ORC_F64 = 5 };

/* ---- partitioning -------------------------------------------------------
 * shp::distributed_vector(count): segment_size = ceil(count / nprocs)
 * (include/dr/shp/distributed_vector.hpp:142); segments() is
 * take_segments(segments_, size()) (distributed_vector.hpp:178-182 ->
 * details/segments_tools.hpp:37-64): segments up to the one holding the
 * last element, the last one trimmed; an empty vector has one empty segment.
 * Writes the segment lengths to `lens` (capacity nprocs) and returns the
 * number of segments. */
int orc_dv_segments(size_t n, int nprocs, size_t *lens);

/* Segments of a sub-range [b, e) of a distributed vector whose segments
 * have lengths `lens[0..nseg)`  (rng::subrange over a distributed iterator:
 * details/segments_tools.hpp:67-94,149-223 -- drop then take).  Writes the
 * lengths of the non-empty pieces to `out`, their owning segment index to
 * `rank_out` (nullable); returns the count. */
int orc_subrange_segments(const size_t *lens, int nseg, size_t b, size_t e,
                          size_t *out, int *rank_out);

/* zip(r, o).zipped_segments() (include/dr/shp/zip_view.hpp:172-206): the
 * intersection of the two segmentations, truncated to min(total_r, total_o).
 * rank of each piece = rank of the input (r) segment, as used by
 * inclusive_scan.hpp:50-53.  Returns the number of pieces. */
int orc_zip_pieces(const size_t *lens_r, int nr, const size_t *lens_o, int no,
                   size_t *piece_lens, int *piece_rank_r, int *piece_rank_o,
                   int cap);

/* ---- shp::reduce  (include/dr/shp/algorithms/reduce.hpp:40-88) ----------
 * For every segment in order: length 0 -> skipped (:67-68); length 1 ->
 * init = op(init, seg[0]) folded on the host immediately (:69-71);
 * otherwise partial = reduce(seg[0..len-2]) seeded with seg[len-1]
 * (reduce_no_init_async, :22-34).  After the loop the partials are folded
 * into init in segment order (:81-83).  The per-segment order inside oneDPL
 * is unspecified; the oracle folds left-to-right.  Integer results are
 * order independent (two's complement), float results are compared with a
 * tolerance against orc_reduce_exact_f64. */
int32_t  orc_shp_reduce_i32(const int32_t *x, const size_t *lens, int nseg, int32_t init, int op);
uint32_t orc_shp_reduce_u32(const uint32_t *x, const size_t *lens, int nseg, uint32_t init, int op);
int64_t  orc_shp_reduce_i64(const int64_t *x, const size_t *lens, int nseg, int64_t init, int op);
uint64_t orc_shp_reduce_u64(const uint64_t *x, const size_t *lens, int nseg, uint64_t init, int op);
float    orc_shp_reduce_f32(const float *x, const size_t *lens, int nseg, float init, int op);
double   orc_shp_reduce_f64(const double *x, const size_t *lens, int nseg, double init, int op);

/* Exact-as-possible fp reference: fp64 (plus: Neumaier-compensated) fold. */
double orc_reduce_exact_f32(const float *x, size_t n, double init, int op);
double orc_reduce_exact_f64(const double *x, size_t n, double init, int op);

/* transform_reduce / dot: reduce(zip(x, y) | transform(a*b), init, plus)
 * (examples/shp/dot_product.cpp:11-18).  Exact fp64 accumulation. */
double  orc_dot_f32(const float *x, const float *y, size_t n, double init);
double  orc_dot_f64(const double *x, const double *y, size_t n, double init);
int32_t orc_dot_i32(const int32_t *x, const int32_t *y, size_t n, int32_t init);

/* ---- shp::inclusive_scan (include/dr/shp/algorithms/inclusive_scan.hpp:22-148)
 * Phase 1 (:77-83): each zipped piece k is scanned locally with op; init
 *   is applied on piece 0 only (:77-80); its last output becomes
 *   partial[k] (:85-96).
 * Phase 2 (:108-116): partial[] is inclusive-scanned with op.
 * Phase 3 (:118-143, op at :132-134): for k > 0: out[i] = op(out[i], partial[k-1]) -- the
 *   carry is the RIGHT operand.
 * `pieces` are the zipped piece lengths (orc_zip_pieces); their sum is the
 * number of elements scanned.  in and out may alias (in-place). */
void orc_shp_scan_i32(const int32_t *in, int32_t *out, const size_t *pieces, int np, int op, int has_init, int32_t init);
void orc_shp_scan_u32(const uint32_t *in, uint32_t *out, const size_t *pieces, int np, int op, int has_init, uint32_t init);
void orc_shp_scan_i64(const int64_t *in, int64_t *out, const size_t *pieces, int np, int op, int has_init, int64_t init);
void orc_shp_scan_u64(const uint64_t *in, uint64_t *out, const size_t *pieces, int np, int op, int has_init, uint64_t init);
void orc_shp_scan_f32(const float *in, float *out, const size_t *pieces, int np, int op, int has_init, float init);
void orc_shp_scan_f64(const double *in, double *out, const size_t *pieces, int np, int op, int has_init, double init);

/* fp64 reference prefix for float tolerance checks (sequential, in double;
 * an fp32 sequential scan is not a usable oracle at 2^26+). */
void orc_scan_exact_f32(const float *in, double *out, size_t n, int op, int has_init, double init);

/* ---- mhp::reduce (include/dr/mhp/algorithms/cpu_algorithms.hpp:102-140)
 * Rank r owns block r of ceil(n/P) elements (mhp/containers/
 * distributed_vector.hpp:190-200); each rank std::reduce()s its block from
 * T(0) (:111-118), the locals are gathered to the root (:121-125,
 * details/communicator.hpp:51-56) and the root folds them into init
 * (:126-129).  Non-root ranks return 0 (:105).  This is the CPU-baseline
 * path: `nthreads` OpenMP threads play the P ranks (one block each). */
double  orc_mhp_reduce_f32(const float *x, size_t n, int nranks, double init, int nthreads);
int32_t orc_mhp_reduce_i32(const int32_t *x, size_t n, int nranks, int32_t init, int nthreads);
/* mhp-style scan for the CPU baseline: local scans in parallel per rank,
 * exclusive prefix of rank totals, carry pass (the 3 phases of
 * inclusive_scan.hpp restated on host threads).  fp64 carries for f32. */
void orc_mhp_scan_f32(const float *in, float *out, size_t n, int nranks, int nthreads);
void orc_mhp_scan_i32(const int32_t *in, int32_t *out, size_t n, int nranks, int nthreads);

/* ---- gemv (include/dr/shp/algorithms/gemv.hpp:13-71), intended c += A*b.
 * The reference kernel has a racy `c_v += a_v*b_v` (:62) and a colind bug
 * (containers/sparse_matrix.hpp:187); parity is defined against the
 * intended CSR product, accumulated per row in nnz order, in fp64. */
void orc_csr_spmv_f32_i32(size_t m, const int32_t *rowptr, const int32_t *colind,
                          const float *vals, const float *x, const float *y_in, double *y_out);
void orc_csr_spmv_f64_i32(size_t m, const int32_t *rowptr, const int32_t *colind,
                          const double *vals, const double *x, const double *y_in, double *y_out);
/* Synthetic matrices.  Shared, hash-based definition so
 * the device generator (drhip_csr_gen_*) produces the same matrix:
 *   banded: row i has columns i-4 .. i+5 clipped to [0, ncols)
 *   random: row i has `k` distinct columns chosen by a hash of (seed,i,j),
 *           sorted ascending.
 *   value(i, j) = u01(hash(seed, i, j)) as f32. */
size_t orc_csr_banded_nnz(size_t m, size_t ncols);
void   orc_csr_gen_banded_f32(size_t row0, size_t nrows, size_t ncols, uint64_t seed,
                              int32_t *rowptr, int32_t *colind, float *vals);
void   orc_csr_gen_random_f32(size_t row0, size_t nrows, size_t ncols, int k, uint64_t seed,
                              int32_t *rowptr, int32_t *colind, float *vals);
size_t orc_csr_density_nnz(size_t row0, size_t nrows, size_t m, size_t ncols, double density);
void   orc_csr_gen_density(size_t row0, size_t nrows, size_t m, size_t ncols, double density, uint64_t seed,
                           int int_values, int64_t *rowptr, int64_t *colind, double *vals);
float    orc_u01(uint64_t seed, uint64_t i, uint64_t j);
uint64_t orc_hash3(uint64_t seed, uint64_t i, uint64_t j);

/* ---- sort (absent from the reference: std::sort semantics) */
void orc_sort_u32(uint32_t *x, size_t n);
int orc_radix_sort_u32(uint32_t *x, size_t n); /* same order, O(n): full-size C3 checks */
int orc_radix_sort_u32_par(uint32_t *x, size_t n, int nthreads); /* same output, OpenMP passes */
void orc_fill_hash_u32(uint32_t *x, size_t n, uint64_t seed, uint64_t start, int nthreads);
void orc_sort_i32(int32_t *x, size_t n);
void orc_sort_f32(float *x, size_t n);
void orc_sort_u64(uint64_t *x, size_t n);
void orc_sort_i64(int64_t *x, size_t n);
void orc_sort_f64(double *x, size_t n);

/* ---- 1-D stencil with span_halo exchange (details/halo.hpp:336-387,
 * examples/mhp/stencil-1d.cpp:16-66).  One step over the global interior
 * [radius, n-radius): out[i] = sum_{d=-r..r} in[i+d] (3-point at r=1).
 * `orc_stencil1d_mhp_*` runs the distributed form: per-rank buffers
 * [prev halo | owned | next halo], halo exchange, local transform -- and
 * must equal the serial form. */
void orc_stencil1d_i32(const int32_t *in, int32_t *out, size_t n, int radius);
void orc_stencil1d_f32(const float *in, float *out, size_t n, int radius);
int  orc_stencil1d_mhp_steps_i32(int32_t *a, int32_t *b, size_t n, int nranks, int steps);
/* test/gtest/mhp/stencil.cpp:34-42 operator: s = v + sum_{i=0..r}(p[-i]+p[i]) */
void orc_stencil_mhp_test_op_i32(const int32_t *in, int32_t *out, size_t n, int radius);

/* 2-D 5-point stencil over the interior of an nx x ny grid (row-major). */
void orc_stencil2d_f32(const float *in, float *out, size_t nx, size_t ny);

/* glibc lrand48 stream used (unseeded) by test/gtest/shp/algorithms.cpp:69-70. */
void orc_lrand48_mod(int32_t *out, size_t n, int32_t mod, int reseed);

#ifdef __cplusplus
}
#endif
#endif
