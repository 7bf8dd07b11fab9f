// Probe: a one-shot all-reduce between PROCESSES through IPC-mapped device buffers and epoch flags
// (the transport of parallel/ipc_allreduce in the trainer), run as N processes sharing one GPU.
//   * every rank fills its send buffer (parity = epoch & 1) with a rank/epoch/index pattern,
//   * k_exchange: block 0 publishes flag[me] = epoch (system-scope release), every block waits for
//     all peers' flags >= epoch (system-scope acquire, s_memrealtime timeout), sums the N buffers and
//     checks the result against the closed form; mismatches / timeouts are counted.
// Prints per-epoch time for the exchange vs a no-wait single-process twin of the same kernels.
// Build: hipcc --offload-arch=gfx950 -O3 ipc_probe.hip -o ipc_probe
// Run:   ./ipc_probe <nranks> <elems> <iters> <dir>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>
#include <sys/wait.h>
#include <chrono>
#include <string>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "[rank %d] %s @%d: %s\n", g_rank, #x, __LINE__, hipGetErrorString(e_)); exit(3); } } while (0)

static int g_rank = 0;
constexpr int kMaxRanks = 8;

struct Peers {
  const int64_t* buf[kMaxRanks];
  const unsigned* flag[kMaxRanks];
};

__device__ __forceinline__ int64_t pattern(int r, int e, int64_t i) { return (int64_t)r * 1000003 + (int64_t)e * 7919 + i; }

__global__ void k_fill(int64_t* buf, int64_t n, int rank, int epoch) {
  int64_t* b = buf + (int64_t)(epoch & 1) * n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    b[i] = pattern(rank, epoch, i);
}

__global__ void k_exchange(Peers p, int nr, int me, unsigned* myflag, int epoch, int64_t n, int64_t* out,
                           unsigned* err, int wait) {
  __shared__ int ok;
  if (blockIdx.x == 0 && threadIdx.x == 0)
    __hip_atomic_store(myflag, (unsigned)epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  if (threadIdx.x == 0) {
    int good = 1;
    if (wait) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (int r = 0; r < nr && good; ++r) {
        while (__hip_atomic_load(p.flag[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < (unsigned)epoch) {
          if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) { good = 0; break; }  // 2 s
          __builtin_amdgcn_s_sleep(1);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    }
    ok = good;
  }
  __syncthreads();
  if (!ok) {
    if (threadIdx.x == 0) atomicAdd(err + 1, 1u);
    return;
  }
  const int64_t off = (int64_t)(epoch & 1) * n;
  unsigned bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t acc = 0, want = 0;
    for (int r = 0; r < nr; ++r) {
      acc += p.buf[r][off + i];
      want += pattern(wait ? r : me, epoch, i);
    }
    out[i] = acc;
    bad += acc != want;
  }
  if (bad) atomicAdd(err, bad);
}

static std::string path_of(const char* dir, const char* what, int r) {
  return std::string(dir) + "/" + what + std::to_string(r);
}

static void write_file(const std::string& p, const void* data, size_t n) {
  std::string tmp = p + ".tmp";
  FILE* f = fopen(tmp.c_str(), "wb");
  fwrite(data, 1, n, f);
  fclose(f);
  rename(tmp.c_str(), p.c_str());
}

static void wait_file(const std::string& p, void* data, size_t n) {
  for (int k = 0; k < 200000; ++k) {
    FILE* f = fopen(p.c_str(), "rb");
    if (f) {
      size_t got = data ? fread(data, 1, n, f) : n;
      fclose(f);
      if (got == n) return;
    }
    usleep(100);
  }
  fprintf(stderr, "[rank %d] timeout waiting for %s\n", g_rank, p.c_str());
  exit(4);
}

static int run_rank(int nr, int me, int64_t n, int iters, const char* dir) {
  g_rank = me;
  CHECK(hipSetDevice(0));
  int64_t* buf;
  unsigned* flag;
  CHECK(hipMalloc(&buf, 2 * n * sizeof(int64_t)));
  CHECK(hipExtMallocWithFlags((void**)&flag, 256, hipDeviceMallocUncached));
  CHECK(hipMemset(flag, 0, 256));
  int64_t* out;
  unsigned* err;
  CHECK(hipMalloc(&out, n * sizeof(int64_t)));
  CHECK(hipMalloc(&err, 16));
  CHECK(hipMemset(err, 0, 16));
  hipIpcMemHandle_t h[2];
  CHECK(hipIpcGetMemHandle(&h[0], buf));
  CHECK(hipIpcGetMemHandle(&h[1], flag));
  write_file(path_of(dir, "h", me), h, sizeof(h));
  Peers p{};
  for (int r = 0; r < nr; ++r) {
    if (r == me) {
      p.buf[r] = buf;
      p.flag[r] = flag;
      continue;
    }
    hipIpcMemHandle_t ph[2];
    wait_file(path_of(dir, "h", r), ph, sizeof(ph));
    void* pb;
    void* pf;
    CHECK(hipIpcOpenMemHandle(&pb, ph[0], hipIpcMemLazyEnablePeerAccess));
    CHECK(hipIpcOpenMemHandle(&pf, ph[1], hipIpcMemLazyEnablePeerAccess));
    p.buf[r] = (const int64_t*)pb;
    p.flag[r] = (const unsigned*)pf;
  }
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int grid = (int)std::min<int64_t>((n + 255) / 256, 256);
  // warm-up + timed loop (epochs continue across both)
  int epoch = 0;
  for (int k = 0; k < 20; ++k) {
    ++epoch;
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, s, buf, n, me, epoch);
    hipLaunchKernelGGL(k_exchange, dim3(grid), dim3(256), 0, s, p, nr, me, flag, epoch, n, out, err, 1);
  }
  CHECK(hipStreamSynchronize(s));
  auto t0 = std::chrono::steady_clock::now();
  for (int k = 0; k < iters; ++k) {
    ++epoch;
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, s, buf, n, me, epoch);
    hipLaunchKernelGGL(k_exchange, dim3(grid), dim3(256), 0, s, p, nr, me, flag, epoch, n, out, err, 1);
  }
  CHECK(hipStreamSynchronize(s));
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / iters;
  // the same two kernels without waiting (own buffer only): per-epoch floor -- after every rank has
  // finished reading this rank's buffers
  write_file(path_of(dir, "mid", me), "x", 1);
  for (int r = 0; r < nr; ++r) wait_file(path_of(dir, "mid", r), nullptr, 1);
  auto t1 = std::chrono::steady_clock::now();
  Peers self{};
  self.buf[0] = buf;
  self.flag[0] = flag;
  for (int k = 0; k < iters; ++k) {
    hipLaunchKernelGGL(k_fill, dim3(grid), dim3(256), 0, s, buf, n, me, epoch + 1 + k);
    hipLaunchKernelGGL(k_exchange, dim3(grid), dim3(256), 0, s, self, 1, me, flag + 16, epoch + 1 + k, n, out, err + 2, 0);
  }
  CHECK(hipStreamSynchronize(s));
  const double us0 = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count() / iters;
  unsigned e[4];
  CHECK(hipMemcpy(e, err, 16, hipMemcpyDeviceToHost));
  printf("rank %d/%d elems %lld: exchange %.2f us/epoch, no-wait twin %.2f us/epoch, mismatches %u, timeouts %u, "
         "twin mismatches %u\n", me, nr, (long long)n, us, us0, e[0], e[1], e[2]);
  fflush(stdout);
  // nobody unmaps / frees while a peer may still read: meet on files first
  write_file(path_of(dir, "done", me), "x", 1);
  for (int r = 0; r < nr; ++r) wait_file(path_of(dir, "done", r), nullptr, 1);
  for (int r = 0; r < nr; ++r)
    if (r != me) {
      CHECK(hipIpcCloseMemHandle((void*)p.buf[r]));
      CHECK(hipIpcCloseMemHandle((void*)p.flag[r]));
    }
  return (e[0] || e[1] || e[2]) ? 1 : 0;
}

int main(int argc, char** argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s nranks elems iters dir\n", argv[0]);
    return 2;
  }
  const int nr = atoi(argv[1]);
  const int64_t n = atoll(argv[2]);
  const int iters = atoi(argv[3]);
  const char* dir = argv[4];
  if (nr < 1 || nr > kMaxRanks) return 2;
  // fork the peers BEFORE any HIP call (no HIP state is inherited)
  pid_t kids[kMaxRanks];
  for (int r = 1; r < nr; ++r) {
    pid_t pid = fork();
    if (pid == 0) return run_rank(nr, r, n, iters, dir);
    kids[r] = pid;
  }
  int rc = run_rank(nr, 0, n, iters, dir);
  for (int r = 1; r < nr; ++r) {
    int st = 0;
    waitpid(kids[r], &st, 0);
    if (!WIFEXITED(st) || WEXITSTATUS(st) != 0) rc = 1;
  }
  printf("ipc_probe %s\n", rc == 0 ? "OK" : "FAILED");
  return rc;
}
