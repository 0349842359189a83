// ipc_probe.hip -- can two processes on this box share device memory for a
// flag hand-off (the combine of the strong-scaled reduce + scan without a
// collective)?  Two processes on ONE GPU (fork before any HIP
// call, no exec): the parent allocates a slot buffer (hipMalloc, or
// fine-grained hipExtMallocWithFlags), exports it with hipIpcGetMemHandle and
// starts a one-block kernel that polls the flag word (bounded: ~2^22 sleeps,
// then it gives up); the child opens the handle (hipIpcOpenMemHandle) and a
// kernel of its own stores {value, flag} into it (payload, release at system
// scope, flag).  Prints one JSON line per allocation kind: open ok, whether
// the parent's poll saw the flag, the value it read, the poll's spins.
// Measurement tool, not product.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <sys/wait.h>
#include <unistd.h>

#define CK(x)                                                                                  \
  do {                                                                                         \
    hipError_t e_ = (x);                                                                       \
    if (e_ != hipSuccess) {                                                                    \
      std::printf("{\"step\": \"%s\", \"error\": \"%s\"}\n", #x, hipGetErrorString(e_));       \
      std::fflush(stdout);                                                                     \
      return 1;                                                                                \
    }                                                                                          \
  } while (0)

__global__ void poll_kernel(unsigned long long *slot, unsigned long long want, unsigned long long *out) {
  if (threadIdx.x != 0) return;
  unsigned spins = 0;
  while (__hip_atomic_load(slot + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != want) {
    if (++spins > (1u << 22)) break;
    __builtin_amdgcn_s_sleep(2);
  }
  out[0] = spins;
  out[1] = __hip_atomic_load(slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void post_kernel(unsigned long long *slot, unsigned long long value, unsigned long long flag) {
  if (threadIdx.x != 0) return;
  __hip_atomic_store(slot, value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(slot + 1, flag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static int child(int rd, int wr) {
  hipIpcMemHandle_t h;
  if (read(rd, &h, sizeof h) != (ssize_t)sizeof h) return 2;
  CK(hipSetDevice(0));
  void *p = nullptr;
  hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  char ok = e == hipSuccess ? 1 : 0;
  if (!ok) std::fprintf(stderr, "child: hipIpcOpenMemHandle: %s\n", hipGetErrorString(e));
  if (ok) {
    usleep(20000); // let the parent's poll start first
    hipLaunchKernelGGL(post_kernel, dim3(1), dim3(64), 0, 0, (unsigned long long *)p, 0x1234ABCDull, 7ull);
    if (hipDeviceSynchronize() != hipSuccess) ok = 0;
    (void)hipIpcCloseMemHandle(p);
  }
  if (write(wr, &ok, 1) != 1) return 2;
  return ok ? 0 : 1;
}

static int parent(int kind, int wr, int rd, pid_t pid) {
  CK(hipSetDevice(0));
  unsigned long long *slot = nullptr, *out = nullptr;
  if (kind == 0) CK(hipMalloc(&slot, 4096));
  else CK(hipExtMallocWithFlags((void **)&slot, 4096, hipDeviceMallocFinegrained));
  CK(hipMemset(slot, 0, 4096));
  CK(hipHostMalloc(&out, 16));
  out[0] = out[1] = ~0ull;
  hipIpcMemHandle_t h;
  hipError_t e = hipIpcGetMemHandle(&h, slot);
  if (e != hipSuccess) {
    std::printf("{\"kind\": \"%s\", \"get_handle\": false, \"error\": \"%s\"}\n", kind ? "finegrained" : "hipMalloc",
                hipGetErrorString(e));
    std::memset(&h, 0, sizeof h);
  }
  hipLaunchKernelGGL(poll_kernel, dim3(1), dim3(64), 0, 0, slot, 7ull, out);
  if (write(wr, &h, sizeof h) != (ssize_t)sizeof h) return 2;
  char ok = 0;
  if (read(rd, &ok, 1) != 1) ok = 0;
  CK(hipDeviceSynchronize());
  int st = 0;
  waitpid(pid, &st, 0);
  std::printf("{\"kind\": \"%s\", \"get_handle\": %s, \"child_open_and_post\": %s, \"poll_saw_flag\": %s, "
              "\"value_ok\": %s, \"poll_spins\": %llu}\n",
              kind ? "finegrained" : "hipMalloc", e == hipSuccess ? "true" : "false", ok ? "true" : "false",
              out[0] <= (1u << 22) ? "true" : "false", out[1] == 0x1234ABCDull ? "true" : "false", out[0]);
  std::fflush(stdout);
  return 0;
}

int main(int argc, char **argv) {
  const int kind = argc > 1 ? std::atoi(argv[1]) : 0;
  int a[2], b[2];
  if (pipe(a) || pipe(b)) return 2;
  std::fflush(stdout);
  const pid_t pid = fork(); // before any HIP call in either process
  if (pid < 0) return 2;
  if (pid == 0) return child(a[0], b[1]);
  return parent(kind, a[1], b[0], pid);
}
