/* c1_mpi_dot.c -- BASELINE config C1 on the CPU, as the reference runs it
 * (MEASUREMENT INFRASTRUCTURE, never the product path): a dot product /
 * transform_reduce over a distributed vector<float> of 2^24 elements on 2
 * MPI ranks.  Each rank owns a block of ceil(n/P) elements
 * (mhp/containers/distributed_vector.hpp:190-207), folds x[i]*y[i] over it
 * serially (std::reduce with the PSTL serial backend,
 * mhp/algorithms/cpu_algorithms.hpp:114-120), MPI_Gather's one float to
 * the root (details/communicator.hpp:51-56, cpu_algorithms.hpp:125) and the
 * root folds the partials (:126-129) -- the vector-add-ref.cpp:30-44
 * MPI pattern.  One warm-up, then the median of `reps` timed runs bracketed
 * by MPI_Barrier + MPI_Wtime, max over ranks.
 *   usage: mpiexec -n 2 c1_mpi_dot [log2n] [reps]                        */
#include <mpi.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static int cmpd(const void *a, const void *b) {
  double x = *(const double *)a, y = *(const double *)b;
  return (x > y) - (x < y);
}

int main(int argc, char **argv) {
  MPI_Init(&argc, &argv);
  int rank, P;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &P);
  const int lg = argc > 1 ? atoi(argv[1]) : 24;
  const int reps = argc > 2 ? atoi(argv[2]) : 7;
  const size_t n = (size_t)1 << lg;
  const size_t blk = (n + P - 1) / P;
  const size_t lo = rank * blk < n ? rank * blk : n, hi = lo + blk < n ? lo + blk : n;
  float *x = malloc((hi - lo + 1) * sizeof(float)), *y = malloc((hi - lo + 1) * sizeof(float));
  uint64_t s = 0x9E3779B97F4A7C15ull * (lo + 1);
  for (size_t i = 0; i < hi - lo; i++) { /* U[0,1) from a 64-bit LCG, per global index block */
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    x[i] = (float)(s >> 40) * (1.0f / 16777216.0f);
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    y[i] = (float)(s >> 40) * (1.0f / 16777216.0f);
  }
  double *t = malloc((reps + 1) * sizeof(double));
  float result = 0.f;
  for (int r = 0; r <= reps; r++) {
    MPI_Barrier(MPI_COMM_WORLD);
    const double t0 = MPI_Wtime();
    float local = 0.f;
    for (size_t i = 0; i < hi - lo; i++) local += x[i] * y[i];
    float *parts = rank == 0 ? malloc(P * sizeof(float)) : NULL;
    MPI_Gather(&local, 1, MPI_FLOAT, parts, 1, MPI_FLOAT, 0, MPI_COMM_WORLD);
    if (rank == 0) {
      result = 0.f;
      for (int k = 0; k < P; k++) result += parts[k];
      free(parts);
    }
    double dt = MPI_Wtime() - t0, mx;
    MPI_Reduce(&dt, &mx, 1, MPI_DOUBLE, MPI_MAX, 0, MPI_COMM_WORLD);
    t[r] = mx;
  }
  if (rank == 0) {
    qsort(t + 1, reps, sizeof(double), cmpd); /* t[0] is the warm-up */
    const double med = t[1 + reps / 2];
    printf("{\"config\": \"C1\", \"workload\": \"mhp dot (transform_reduce) 2^%d f32, %d MPI ranks\", "
           "\"value\": %.6g, \"unit\": \"elements/s\", \"median_s\": %.6g, \"ranks\": %d, \"runs\": %d, "
           "\"check\": %.9g}\n",
           lg, P, (double)n / med, med, P, reps, (double)result);
  }
  free(x);
  free(y);
  free(t);
  MPI_Finalize();
  return 0;
}
