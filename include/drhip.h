/*
 * drhip.h -- C-ABI of libdrhip.so, the MI355X (gfx950) device layer and
 * algorithm kernels behind the Distributed Ranges `shp` API.
 *
 * The reference (sudhirverma/distributed-ranges, header-only C++20/SYCL) has
 * no FFI of its own: its device layer is SYCL queues + USM
 * (include/dr/shp/{init,allocators,copy,device_ref}.hpp) and its per-segment
 * arithmetic is oneDPL (reduce_async / inclusive_scan_async / for_each_async)
 * plus SYCL parallel_for kernels.  Each entry point below replaces one of
 * those call sites; the replaced reference interface is cited per function.
 * The C++ drop-in layer (distributed-ranges_amd/include/dr/shp/...) and the
 * Python binding (distributed-ranges_amd/drhip.py) both call only this ABI.
 *
 * Conventions
 *   - Every function returns int: 0 = success, otherwise a drhip_status code
 *     (hip errors are mapped to DRHIP_ERR_HIP and the hipError_t text is
 *     kept for drhip_last_error()).
 *   - A "segment" (seg) is one entry of the ordered device list given to
 *     drhip_init -- the reference's segment rank (shp/init.hpp:40-50).  Each
 *     segment owns one HIP stream; duplicated device ids are allowed
 *     (the reference test harness's --devicesCount duplication,
 *     test/gtest/shp/shp-tests.cpp:34-39).
 *   - Kernel entry points are ASYNCHRONOUS on the segment's stream; buffers
 *     are owned by the caller and must be device-visible (device memory,
 *     peer memory with P2P enabled, or pinned host memory).  `*_host`
 *     arguments are plain host pointers read during the call.
 *   - "ACC" is the accumulation type of an element type: double for F32/F64,
 *     the element type itself for integers (wrapping two's-complement
 *     arithmetic).  Reduce results, scan carries and totals are ACC.
 */
#ifndef DRHIP_H
#define DRHIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  DRHIP_I32 = 0, DRHIP_U32 = 1, DRHIP_I64 = 2, DRHIP_U64 = 3, DRHIP_F32 = 4, DRHIP_F64 = 5
} drhip_dtype;

typedef enum { DRHIP_PLUS = 0, DRHIP_MUL = 1, DRHIP_MIN = 2, DRHIP_MAX = 3 } drhip_op;

typedef enum {
  DRHIP_OK = 0,
  DRHIP_ERR_HIP = 1,          /* a HIP runtime call failed */
  DRHIP_ERR_NOT_INIT = 2,     /* drhip_init not called */
  DRHIP_ERR_BAD_SEG = 3,      /* segment index out of range */
  DRHIP_ERR_BAD_ARG = 4,      /* null pointer, unsupported dtype/op, bad size */
  DRHIP_ERR_NO_DEVICE = 5,    /* no HIP device visible */
  DRHIP_ERR_TIMEOUT = 6,      /* a bounded in-kernel spin gave up */
  DRHIP_ERR_UNSUPPORTED = 7,
  DRHIP_ERR_COMM = 8,         /* an RCCL call failed (text has the ncclResult_t) */
  DRHIP_ERR_ALLOC = 9         /* the allocator returned memory overlapping a live block,
                                 or a guard red zone was overwritten (DRHIP_ALLOC_GUARD) */
} drhip_status;

/* ------------------------------------------------------------ runtime --
 * Replaces shp::init/finalize/devices/nprocs/context (shp/init.hpp:16-52)
 * and get_numa_devices/get_duplicated_devices (shp/util.hpp:77-136). */

/* Registers `nsegs` segments on HIP devices dev_ids[0..nsegs) (ids may
 * repeat), creates one non-blocking stream per segment, enables peer access
 * between distinct devices, and allocates per-segment workspaces.  Calling
 * it again re-initialises (finalize + init). */
int drhip_init(const int *dev_ids, int nsegs);
int drhip_finalize(void);
int drhip_device_count(int *count);           /* visible HIP devices */
int drhip_nprocs(int *nsegs);                 /* shp::nprocs() */
int drhip_device_of(int seg, int *dev_id);    /* shp::devices()[seg] */
int drhip_stream(int seg, void **hip_stream); /* the segment's hipStream_t */
int drhip_sync(int seg);                      /* wait for the segment's stream */
int drhip_sync_all(void);
const char *drhip_last_error(void);           /* text of the last failure */
const char *drhip_version(void);
/* HIP graphs of a segment's work (no counterpart in the reference, whose
 * every algorithm call builds new sycl::queues, e.g. reduce.hpp:63): the
 * drhip calls (and RCCL collectives) issued between drhip_graph_begin and
 * drhip_graph_end on seg's stream are captured, not run; drhip_graph_launch
 * replays them on seg's stream with one launch.  For a step repeated with
 * the same buffers and sizes -- e.g. the strong-scaled reduce + scan whose
 * per-rank kernels take ~0.3 ms, where launch gaps are SURVEY.md 7's "per-
 * call overhead <= 10 us" budget.  Every kernel launched by the C-ABI keeps
 * its state on the device (single-pass reduce counters reset by their last
 * block, scan status words re-zeroed by a memset node), so a replay
 * recomputes everything.  Between begin and end, no call may allocate
 * (warm the workspaces with one eager call first) or synchronise.
 * Lifetime: a graph holds raw pointers to seg's workspace and tile-prefix
 * buffer, so from drhip_graph_begin until every graph of seg is destroyed
 * (drhip_graph_destroy) a call that would GROW either buffer fails with
 * DRHIP_ERR_UNSUPPORTED instead of freeing memory a graph still uses.  A
 * drhip_reduce_tiles inside a graph takes effect at drhip_graph_launch: an
 * eager drhip_inclusive_scan_tiles after a replay must name the captured
 * range.  A graph launches only on the segment it was captured on. */
int drhip_graph_begin(int seg);
int drhip_graph_end(int seg, void **graph_exec);
int drhip_graph_launch(int seg, void *graph_exec);
int drhip_graph_destroy(void *graph_exec);

/* ------------------------------------------------------------- memory --
 * device_allocator::allocate/deallocate (shp/allocators.hpp:45-72) and
 * shp::copy/copy_async/fill_async (shp/copy.hpp:19-173), device_ref
 * element access (shp/device_ref.hpp:23-44). */
/* drhip_malloc: device memory on seg's device, valid on every stream and
 * peer device.  Default (DRHIP_ALLOC=cache, read at drhip_init): a caching
 * allocator over hipMalloc -- drhip_free keeps the block, whole, in seg's
 * cache behind fences recorded on every segment stream and the device's NULL
 * stream (no host sync), and drhip_malloc hands it out again for a request
 * of the same size class (powers of two below 1 MiB, 2 MiB multiples above)
 * once every fence has completed; work a caller queued on OTHER streams of
 * its own is not fenced (drain those before freeing memory they use).  The
 * cache is released at drhip_finalize and when hipMalloc runs out of memory.
 * DRHIP_ALLOC=hipmalloc: plain hipMalloc / hipFree (hipFree synchronises the
 * device).  DRHIP_ALLOC=pool: the device's stream-ordered pool
 * (hipMallocAsync), kept for diagnosis only -- on ROCm 7.2 / gfx950 a pool
 * block filled by a copy can read differently from a kernel
 * (profiles/r06_pool_diagnosis.txt; DRHIP_POOL=private|noreuse variants).
 * Every live block is tracked: one the allocator returns overlapping a live
 * block is refused (DRHIP_ERR_ALLOC), and drhip_free refuses
 * (DRHIP_ERR_BAD_ARG) a pointer that is not a live drhip_malloc block.
 * DRHIP_ALLOC_GUARD=1: red zones around every block, checked by drhip_free
 * and drhip_sync (DRHIP_ERR_ALLOC names the block); DRHIP_ALLOC_TRACE=path:
 * one line per allocation / free. */
int drhip_malloc(int seg, size_t bytes, void **ptr);
int drhip_free(int seg, void *ptr);
int drhip_host_alloc(size_t bytes, void **ptr);        /* pinned, device-visible host memory */
int drhip_host_free(void *ptr);
/* Async on the segment stream for device / pinned host buffers; with a
 * pageable host buffer the copy still goes on the segment stream (the
 * runtime stages it; DRHIP_COPY=staged: through a pinned 64 MiB buffer of
 * the segment's) and the call blocks until it has landed. */
int drhip_memcpy_h2d(int seg, void *dst, const void *src, size_t bytes);
int drhip_memcpy_d2h(int seg, void *dst, const void *src, size_t bytes);
int drhip_memcpy_d2d(int seg, void *dst, const void *src, size_t bytes);  /* async, may cross devices */
/* dst[i] = *value_host, i < n, element size 1/2/4/8 bytes (copy.hpp:147-168) */
int drhip_fill(int seg, void *dst, size_t n, const void *value_host, size_t elem_size);
/* dst[i] = start + i (std::iota over a segment; test/gtest/shp/algorithms.cpp:11-19) */
int drhip_iota(int seg, int dtype, void *dst, size_t n, const void *start_host);

/* ------------------------------------------------------- elementwise --
 * Fixed-function forms of shp::for_each (shp/algorithms/for_each.hpp:14-92)
 * for callers that cannot compile user lambdas with hipcc; the C++ layer
 * has a header-only template path for arbitrary callables. */
/* out[i] = op(in[i], scalar)   (out may alias in) */
int drhip_transform_scalar(int seg, int dtype, int op, const void *in, void *out, size_t n,
                           const void *scalar_host);
/* out[i] = op(a[i], b[i]) */
int drhip_transform_binary(int seg, int dtype, int op, const void *a, const void *b, void *out,
                           size_t n);
/* x[i] = -x[i]  (the ForEach test's negate, algorithms.cpp:21-37) */
int drhip_negate(int seg, int dtype, void *x, size_t n);

/* ------------------------------------------------------------ reduce --
 * Replaces the per-segment oneDPL reduce_async of shp::reduce
 * (shp/algorithms/reduce.hpp:22-34,74-78).  *out_acc (ACC, device-visible)
 * = op-reduction of x[0..n); n == 0 writes the identity of op.  One kernel
 * launch: the last block to finish folds the block partials. */
int drhip_reduce(int seg, int dtype, int op, const void *x, size_t n, void *out_acc);
/* Cross-segment combine (shp/algorithms/reduce.hpp:81-83 fold in segment
 * order; inclusive_scan.hpp:108-116 scan of the partials) of w gathered
 * segment results partials[0..w) (ACC values of dtype, device-visible, e.g.
 * the output of drhip_allgather): *result = p[0] op p[1] op ... op p[w-1]
 * and, when rank > 0, *carry = p[0] op ... op p[rank-1] -- both folded left
 * to right by one device thread (floats combine in the reference's order).
 * result / carry nullable; asynchronous on seg's stream. */
int drhip_fold_partials(int seg, int dtype, int op, const void *partials, int w, int rank, void *result,
                        void *carry);
/* transform_reduce / dot: sum_i x[i]*y[i] (examples/shp/dot_product.cpp:11-18,
 * reduce(zip(x,y) | transform(a*b), 0, plus)). */
int drhip_dot(int seg, int dtype, const void *x, const void *y, size_t n, void *out_acc);

/* ------------------------------------------------------------- scan ----
 * Replaces phases 1 and 3 of shp::inclusive_scan
 * (shp/algorithms/inclusive_scan.hpp:77-83 oneDPL inclusive_scan_async,
 * :118-143 for_each_async carry pass) with ONE single-pass decoupled-
 * lookback kernel:
 *     out[i] = carry op init op in[0] op ... op in[i]
 * init_host  (nullable, element type): the reference's piece-0 init (:77-80)
 * carry_host (nullable, ACC):          carry read at call time
 * carry_dev  (nullable, ACC):          carry read by the kernel (device-visible),
 *                                      e.g. the output of an RCCL exchange
 * total_acc  (nullable, ACC):          receives carry op init op (all of in),
 *                                      the value phase 2 (:108-116) scans.
 * Supported ops are commutative, so carry placement (the reference applies
 * op(x, carry), :132-134) is value-identical; fp32 inter-tile carries are
 * kept in fp64.  in == out (in-place) is allowed. */
int drhip_inclusive_scan(int seg, int dtype, int op, const void *in, void *out, size_t n,
                         const void *init_host, const void *carry_host, const void *carry_dev,
                         void *total_acc);
/* The N > 1 step of a reduce + scan in one kernel after the exchange:
 * partials[0..w) are the w gathered segment totals (ACC of dtype, device
 * memory, e.g. drhip_allgather's output); the scan of in[0..n) gets as carry
 * the fold of partials[0..rank) and, if result is not null, *result = the
 * fold of all w (the reduce's answer) -- both folded left to right exactly
 * as drhip_fold_partials does, by tile 0 of the scan kernel, so the step
 * runs one kernel fewer (reduce.hpp:81-83, inclusive_scan.hpp:108-143). */
int drhip_inclusive_scan_gathered(int seg, int dtype, int op, const void *in, void *out, size_t n,
                                  const void *partials, int w, int rank, void *result);
/* Reduce + scan over the SAME range (the C2 step, and the shp scan's piece
 * totals): drhip_reduce_tiles is drhip_reduce (the ACC op-reduction of
 * x[0..n) to *out_acc) that also leaves, in the segment, every scan tile's
 * exclusive prefix; drhip_inclusive_scan_tiles then scans that same range
 * (in == x, same n, dtype, op: checked, DRHIP_ERR_BAD_ARG otherwise) with
 * those prefixes -- no look-back, no status words: a streaming pass.  x must
 * not be written between the two calls (the prefixes describe its contents
 * at the reduce; DRHIP_CHECK_TILES=1 at drhip_init hashes the range at both
 * calls and makes drhip_sync return DRHIP_ERR_BAD_ARG on a change -- a debug
 * mode, 4 B/elem more per call), and another drhip_reduce_tiles on the same
 * segment replaces the prefixes.  Its
 * carry is *carry_dev (nullable) and/or the fold of partials[0..rank) of the
 * w gathered segment totals (nullable; *result = fold of all w, nullable),
 * as drhip_inclusive_scan_gathered (also when n == 0: an empty segment still
 * writes *result).  Bytes: 4 + 8 per element, as a reduce
 * followed by drhip_inclusive_scan; the reduce's tile pass replaces the
 * scan's inter-tile look-back (reduce.hpp:40-88 then inclusive_scan.hpp:
 * 22-148 over one range). */
int drhip_reduce_tiles(int seg, int dtype, int op, const void *x, size_t n, void *out_acc);
int drhip_inclusive_scan_tiles(int seg, int dtype, int op, const void *in, void *out, size_t n,
                               const void *carry_dev, const void *partials, int w, int rank, void *result);

/* ------------------------------------------------------------- gemv ----
 * Replaces the gemv nonzero loop (shp/algorithms/gemv.hpp:45-66) with a
 * CSR-vector SpMV over one row tile:  y[i] += sum_k vals[k] * x[colind[k]]
 * for rows i < m, rowptr/colind int32 (idtype DRHIP_I32) or int64
 * (DRHIP_I64), vals/x/y of vdtype (F32 or F64).  The reference's racy
 * `c_v += a_v*b_v` (:62) becomes one owner per row -- no atomics.
 * colind/vals hold nnz entries; rowptr values index them (0 <= rowptr[i]
 * <= nnz) and every colind entry is a valid column of x: the kernel reads
 * whole 16-byte vectors of colind/vals that may straddle row-tile edges. */
int drhip_spmv_csr(int seg, int vdtype, int idtype, size_t m, size_t nnz, const void *rowptr,
                   const void *colind, const void *vals, const void *x, void *y);
/* Device-side synthetic CSR generator for rows [row0, row0+nrows) of an
 * ncols-wide matrix (kind 0 = banded offsets -4..+5, kind 1 = k random
 * distinct sorted columns).  Same hash definition as oracle.c, so a tile
 * generated here equals orc_csr_gen_*.  rowptr is tile-local (starts at 0).
 * Replaces sparse_matrix::init_random_ (containers/sparse_matrix.hpp:286-336),
 * whose host std::map generator cannot build 2^26-row matrices. */
int drhip_csr_nnz(int kind, size_t row0, size_t nrows, size_t ncols, int k, size_t *nnz);
int drhip_csr_gen(int seg, int kind, size_t row0, size_t nrows, size_t ncols, int k,
                  uint64_t seed, void *rowptr, void *colind, void *vals);
/* Density generator for rows [row0, row0+nrows) of an m x ncols matrix:
 * floor(density*m*ncols) nonzeros in total (util/generate_random.hpp:37),
 * spread evenly over rows, one column per equal-width stratum of each row
 * (distinct, sorted), values U[0,1) (float/double) or {0,1} (integers).
 * Replaces generate_random_csr (util/generate_random.hpp:29-90) as called by
 * sparse_matrix(shape, density[, partition]) (containers/sparse_matrix.hpp:
 * 157-166, 286-336), which ignores density and reseeds every tile with 0.
 * Equals orc_csr_gen_density.  rowptr is tile-local. */
int drhip_csr_density_nnz(size_t row0, size_t nrows, size_t m, size_t ncols, double density, size_t *nnz);
int drhip_csr_gen_density(int seg, int vdtype, int idtype, size_t row0, size_t nrows, size_t m, size_t ncols,
                          double density, uint64_t seed, void *rowptr, void *colind, void *vals);

/* ------------------------------------------------------------- sort ----
 * shp::sort is absent from the reference; defined with
 * std::ranges::sort semantics (ascending, std::less).  LSD radix sort of
 * 4- or 8-byte keys (I32/U32/F32 order-preserving bit transforms).
 * From 256 MiB of 4-byte keys the passes are persistent kernels (a grid of
 * the device's resident capacity, tiles claimed per XCD).  Segments of ONE
 * process sharing a device are serialised by the runtime; sorts from
 * SEPARATE processes must not run on one device at the same time (their
 * resident grids can starve each other until the bounded spin reports
 * DRHIP_ERR_TIMEOUT): run them one after the other, or set
 * DRHIP_SORT_OS_PT=0 (the one-shot kernels) in those processes. */
int drhip_sort_workspace(int seg, int dtype, size_t n, size_t *bytes);
int drhip_sort(int seg, int dtype, void *keys, size_t n, void *tmp, size_t tmp_bytes);
/* Distributed-sort helpers: the regular samples samples[j] = sorted[j *
 * stride] (j < ceil(n / stride)) of a sorted run, and per-bucket counts of a
 * sorted run against nsplit sorted splitters (bucket b = [splitter[b-1],
 * splitter[b])). */
int drhip_sort_sample(int seg, int dtype, const void *sorted, size_t n, size_t stride,
                      void *samples);
int drhip_sort_bucket_counts(int seg, int dtype, const void *sorted, size_t n,
                             const void *splitters, int nsplit, uint64_t *counts);
/* Exact splitting of the distributed sort (host functions, csrc/split.hip;
 * SURVEY.md 8e "sort": one samples allgather, one slices allgather, then
 * the all-to-all).  Keys are radix-order bits widened to uint64.  p ranks
 * with n[i] sorted keys; rank i's regular samples (stride[i], nsamples[i]
 * of them) concatenated in `samples`; nb boundaries g[k] (global sorted
 * ranks, normally the prefix sums of n).  drhip_split_windows writes, for
 * each boundary, a value bracket [lo[k], hi[k]] holding the key of global
 * rank g[k], and win[2 (i nb + k) + {0,1}] = the slice [a, b) of rank i's
 * sorted keys holding every key of that bracket.  drhip_split_exact takes
 * every slice's keys concatenated in (rank, boundary) order and writes
 * split[i (nb + 1) + k] = the number of rank i's keys that go to
 * destinations <= k (split[i (nb + 1) + nb] = n[i]): keys below the
 * boundary key in full, keys equal to it in rank order, so destination k
 * receives exactly g[k] - g[k-1] keys.  Deterministic: every rank computes
 * the same matrix. */
int drhip_split_windows(int p, const uint64_t *n, const uint64_t *stride, const uint64_t *nsamples,
                        const uint64_t *samples, int nb, const uint64_t *g, uint64_t *lo, uint64_t *hi,
                        uint64_t *win);
int drhip_split_exact(int p, const uint64_t *n, int nb, const uint64_t *g, const uint64_t *lo,
                      const uint64_t *hi, const uint64_t *win, const uint64_t *wkeys, uint64_t *split);
/* Destination step of the distributed sort: keys[0, n) holds nruns sorted
 * runs [run_offsets[r], run_offsets[r+1]) (host array, 0 .. n); on return
 * keys is sorted (radix order, as drhip_sort).  Pairwise merge-path rounds,
 * ceil(log2 nruns) passes of one read + one write per key, instead of a
 * second full radix sort; nruns <= 128.  Replaces the per-destination local
 * sort of the sample sort (SURVEY.md 8e "sort": local merge or second radix). */
int drhip_merge_workspace(int seg, int dtype, size_t n, int nruns, size_t *bytes);
int drhip_merge_runs(int seg, int dtype, void *keys, size_t n, const size_t *run_offsets, int nruns, void *tmp,
                     size_t tmp_bytes);
/* The same merge from src (the runs, e.g. where the all_to_all landed) into
 * a separate dst (e.g. the segment itself): the rounds alternate so that the
 * last one writes dst -- no copy of the keys before or after (the
 * distributed sort's destination step moves 8 B/key per round and nothing
 * else).  src, dst key-aligned and not overlapping; same workspace as
 * drhip_merge_runs. */
int drhip_merge_runs_to(int seg, int dtype, const void *src, void *dst, size_t n, const size_t *run_offsets,
                        int nruns, void *tmp, size_t tmp_bytes);

/* ---------------------------------------------------------- stencil ----
 * mhp::transform of a radius-r 1-D stencil over a halo'd segment
 * (mhp/algorithms/cpu_algorithms.hpp:147-161 with the ops of
 * examples/mhp/stencil-1d.cpp:16-19): buffers are [r halo | owned | r halo];
 * for lo <= i < hi:  out[r+i] = sum_{d=-r..r} in[r+i+d].  I32 (wrapping)
 * and F32. */
int drhip_stencil1d(int seg, int dtype, const void *in_buf, void *out_buf, size_t n_owned,
                    int radius, size_t lo, size_t hi);
/* 5-point 2-D stencil on a row block with one halo row above and below:
 * buffers are (rows+2) x nx, row-major; for owned rows r in [rlo, rhi) and
 * columns 1..nx-2:  out = c + n + s + e + w. */
int drhip_stencil2d(int seg, int dtype, const void *in_buf, void *out_buf, size_t nx,
                    size_t rows, size_t rlo, size_t rhi);

/* ------------------------------------------------- RCCL over xGMI -------
 * The reference's cross-rank layer is MPI (mhp communicator,
 * include/dr/details/communicator.hpp:51-56 gather, :97-149 isend/irecv;
 * halo exchange details/halo.hpp:55-137) and, inside shp, peer USM copies.
 * Here every segment may own ONE RCCL communicator; calls are enqueued on
 * the segment's stream (asynchronous, like every other drhip call).
 *   multi-process (one rank per GPU, the mhp model, bench.py at N > 1):
 *     rank 0 drhip_comm_unique_id -> broadcast the 128 bytes by any channel
 *     (MPI_Bcast, torch.distributed store) -> every rank
 *     drhip_comm_init_rank(seg, nranks, rank, id);
 *   single process, many devices (the shp model): drhip_comm_init_all()
 *     builds one communicator per segment (distinct devices only), and a
 *     collective over all segments is issued between
 *     drhip_comm_group_start() / drhip_comm_group_end(). */
#define DRHIP_COMM_ID_BYTES 128
int drhip_comm_unique_id(void *id /* DRHIP_COMM_ID_BYTES */);
int drhip_comm_init_rank(int seg, int nranks, int rank, const void *id);
int drhip_comm_init_all(void);
int drhip_comm_destroy(int seg);
int drhip_comm_rank(int seg, int *rank, int *nranks);
int drhip_comm_group_start(void);
int drhip_comm_group_end(void);
/* shp::reduce partial fold (reduce.hpp:81-83) / scan totals: elementwise
 * allreduce of n values of dtype with op (+, *, min, max). */
int drhip_allreduce(int seg, int dtype, int op, const void *send, void *recv, size_t n);
/* gemv.hpp:30-42 x replication, scan carries, sort samples: recv holds
 * nranks blocks of `bytes` in rank order. */
int drhip_allgather(int seg, const void *send, void *recv, size_t bytes);
/* mhp gather to root (communicator.hpp:51-56, mhp reduce cpu_algorithms.hpp:102-140). */
int drhip_gather(int seg, const void *send, void *recv, size_t bytes, int root);
/* sort exchange: byte counts and offsets per peer; grouped
 * point-to-point sends/receives, zero-byte pairs skipped. */
int drhip_alltoallv(int seg, const void *send, const size_t *send_bytes, const size_t *send_off, void *recv,
                    const size_t *recv_bytes, const size_t *recv_off);
/* lib::span_halo exchange (details/halo.hpp:336-387): buf is
 * [prev halo | owned | next halo] in cells of cell_bytes (a 2-D row block
 * passes one row as a cell).  Sends the first `prev` owned cells to rank-1
 * (tag halo_reverse) and the last `next` owned cells to rank+1 (halo_forward);
 * receives rank-1's into the prev halo and rank+1's into the next halo; ends
 * are skipped unless periodic.  The reference's message pattern only pairs
 * up when prev == next (a send of `prev` cells lands in the neighbour's
 * `next`-cell halo), so prev != next is rejected. */
int drhip_halo_exchange(int seg, void *buf, size_t n_owned, size_t cell_bytes, size_t prev, size_t next,
                        int periodic);

/* ---------------------------------------- flag exchange (no collective) ----
 * The combine of a strong-scaled reduce + inclusive_scan step -- every rank
 * needs the w segment results in segment order (reduce.hpp:81-83,
 * inclusive_scan.hpp:108-116) -- as stores into peers' slots plus a flag
 * instead of an RCCL all_gather.  A rank allocates its slot
 * array (fine-grained device memory, drhip_xchg_alloc), every rank maps
 * every other rank's array (the same pointers in one process with peer
 * access; drhip_ipc_handle / drhip_ipc_open across processes) and
 * drhip_xchg_allgather (one 1-block kernel on seg's stream) posts the
 * value_bytes (4 or 8) at *value (device memory, e.g. drhip_reduce_tiles'
 * ACC result) into slot `rank` of every array and waits until all w values
 * of this exchange have arrived in its own, writing them to gathered[0..w)
 * (value_bytes each) in rank order -- the partials argument of
 * drhip_inclusive_scan_tiles.  Exchanges are counted
 * on the device (graph replays included), so every rank must make the same
 * sequence of exchanges on the same arrays.  peer_slots is a host array of
 * w device pointers with peer_slots[rank] == local_slots.  The w exchange
 * kernels must be able to run at the same time: one participant per device
 * or per process.  Segments that share a device inside one process do not
 * qualify -- the HIP runtime multiplexes their streams onto a few hardware
 * queues, so one segment's waiting kernel can sit in front of another's post
 * (8 duplicated segments hit the spin bound, round 5).  A wait past the
 * spin bound (1-2 s) sets the segment's error word:
 * drhip_sync returns DRHIP_ERR_TIMEOUT. */
#define DRHIP_IPC_HANDLE_BYTES 64
int drhip_xchg_bytes(int w, size_t *bytes);
int drhip_xchg_alloc(int seg, int w, void **slots);
int drhip_xchg_free(int seg, void *slots);
int drhip_xchg_allgather(int seg, void *local_slots, void *const *peer_slots, int w, int rank, const void *value,
                         int value_bytes, void *gathered);
/* Cross-process mapping of device memory (hipIpcGetMemHandle /
 * hipIpcOpenMemHandle): handle is DRHIP_IPC_HANDLE_BYTES of opaque bytes. */
int drhip_ipc_handle(const void *dev_ptr, void *handle);
int drhip_ipc_open(int seg, const void *handle, void **dev_ptr);
int drhip_ipc_close(int seg, void *dev_ptr);

#ifdef __cplusplus
}
#endif
#endif /* DRHIP_H */
