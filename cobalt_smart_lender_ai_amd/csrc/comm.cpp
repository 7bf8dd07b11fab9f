// Native RCCL communicator for the GBDT hot path (per-level histogram all-reduce), and the dispatch
// of the cobalt_comm_* entry points over the three communicator kinds (RCCL, in-process loopback,
// IPC one-shot group -- see comm.h).
//
// torch.distributed (backend "nccl" == RCCL on ROCm) bootstraps the process group and ships the
// 128-byte unique id; this file owns a dedicated communicator so the int64 histogram all-reduce
// is enqueued from C++ on the trainer's HIP stream, in the middle of a tree, with no Python in the
// loop (and stays capturable in a hipGraph). RCCL is resolved at run time with dlopen from the
// library PyTorch already loaded, so the process holds exactly one RCCL and one HIP runtime.
// (The reference has no collective layer at all: SURVEY.md §2.5/§2.7.)
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <stdint.h>
#include <string.h>

#include "comm.h"

#define COBALT_API extern "C" __attribute__((visibility("default")))

namespace {

typedef struct { char internal[128]; } UniqueId;
typedef void* Comm;
typedef int Result;
// Enum values from rccl.h (ncclDataType_t / ncclRedOp_t)
constexpr int kInt64 = 4, kUint8 = 1, kFloat32 = 7, kFloat64 = 8, kInt32 = 2;
constexpr int kSum = 0, kMax = 2, kMin = 3;

struct Api {
  void* lib = nullptr;
  Result (*get_unique_id)(UniqueId*) = nullptr;
  Result (*comm_init_rank)(Comm*, int, UniqueId, int) = nullptr;
  Result (*comm_destroy)(Comm) = nullptr;
  Result (*comm_abort)(Comm) = nullptr;
  Result (*all_reduce)(const void*, void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  Result (*all_gather)(const void*, void*, size_t, int, Comm, hipStream_t) = nullptr;
  Result (*broadcast)(const void*, void*, size_t, int, int, Comm, hipStream_t) = nullptr;
  const char* (*error_string)(Result) = nullptr;
  Result (*async_error)(Comm, Result*) = nullptr;  // optional (ncclCommGetAsyncError)
};

Api g_api;
char g_err[512];

template <typename T>
bool sym(T& fn, const char* name) {
  fn = reinterpret_cast<T>(dlsym(g_api.lib, name));
  return fn != nullptr;
}

int dtype_code(int code) {
  // 0 = int64, 1 = uint8, 2 = int32, 3 = float32, 4 = float64
  switch (code) {
    case 0: return kInt64;
    case 1: return kUint8;
    case 2: return kInt32;
    case 3: return kFloat32;
    case 4: return kFloat64;
    default: return -1;
  }
}

}  // namespace

COBALT_API const char* cobalt_comm_last_error() { return g_err; }

void comm_set_error(const char* msg) { snprintf(g_err, sizeof(g_err), "%s", msg); }

static inline void* nccl_of(void* h) { return static_cast<CobaltComm*>(h)->nccl; }
static inline bool is_loop(void* h) { return static_cast<CobaltComm*>(h)->kind == 1; }
static inline bool is_ipc(void* h) { return static_cast<CobaltComm*>(h)->kind == 2; }

COBALT_API int cobalt_comm_load(const char* path) {
  if (g_api.lib) return 0;
  g_api.lib = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!g_api.lib) {
    snprintf(g_err, sizeof(g_err), "dlopen(%s) failed: %s", path, dlerror());
    return -1;
  }
  bool ok = sym(g_api.get_unique_id, "ncclGetUniqueId") && sym(g_api.comm_init_rank, "ncclCommInitRank") &&
            sym(g_api.comm_destroy, "ncclCommDestroy") && sym(g_api.comm_abort, "ncclCommAbort") &&
            sym(g_api.all_reduce, "ncclAllReduce") && sym(g_api.all_gather, "ncclAllGather") &&
            sym(g_api.broadcast, "ncclBroadcast") && sym(g_api.error_string, "ncclGetErrorString");
  if (!ok) {
    snprintf(g_err, sizeof(g_err), "missing RCCL symbol in %s", path);
    return -2;
  }
  sym(g_api.async_error, "ncclCommGetAsyncError");
  return 0;
}

COBALT_API int cobalt_comm_unique_id(void* out128) {
  if (!g_api.lib) return -1;
  UniqueId id;
  Result r = g_api.get_unique_id(&id);
  if (r) { snprintf(g_err, sizeof(g_err), "ncclGetUniqueId: %s", g_api.error_string(r)); return r; }
  memcpy(out128, &id, sizeof(id));
  return 0;
}

COBALT_API int cobalt_comm_init(const void* id128, int nranks, int rank, void** out) {
  if (!g_api.lib) return -1;
  UniqueId id;
  memcpy(&id, id128, sizeof(id));
  Comm c = nullptr;
  Result r = g_api.comm_init_rank(&c, nranks, id, rank);
  if (r) { snprintf(g_err, sizeof(g_err), "ncclCommInitRank: %s", g_api.error_string(r)); return r; }
  *out = new CobaltComm{0, c, nullptr, rank, nranks};
  return 0;
}

COBALT_API int cobalt_comm_destroy(void* comm, int abort) {
  if (!comm) return 0;
  CobaltComm* h = static_cast<CobaltComm*>(comm);
  Result r = 0;
  if (h->kind == 1) {
    loop_release(h);
  } else if (h->kind == 2) {
    ipc_release(h);
  } else if (g_api.lib) {
    r = abort ? g_api.comm_abort(static_cast<Comm>(h->nccl)) : g_api.comm_destroy(static_cast<Comm>(h->nccl));
  }
  delete h;
  return r;
}

// Asynchronous communicator error (a peer died, a network/transport failure): 0 = healthy. Polled by
// the host-side collective watchdog (parallel/dist.py) while it waits on the trainer's stream.
COBALT_API int cobalt_comm_async_error(void* comm) {
  if (comm && is_ipc(comm)) return ipc_error(static_cast<CobaltComm*>(comm));
  if (!comm || is_loop(comm) || !g_api.async_error) return 0;
  Result st = 0;
  Result r = g_api.async_error(static_cast<Comm>(nccl_of(comm)), &st);
  if (r) return r;
  if (st && st != 7 /* ncclInProgress */) {
    snprintf(g_err, sizeof(g_err), "RCCL async error: %s", g_api.error_string(st));
    return st;
  }
  return 0;
}

COBALT_API int cobalt_comm_allreduce_sum_i64(void* comm, int64_t* buf, int64_t count, hipStream_t stream) {
  if (is_loop(comm)) return loop_allreduce(static_cast<CobaltComm*>(comm), buf, count, 0, kSum, stream);
  if (is_ipc(comm)) return ipc_allreduce(static_cast<CobaltComm*>(comm), buf, count, 0, kSum, stream);
  Result r = g_api.all_reduce(buf, buf, (size_t)count, kInt64, kSum, static_cast<Comm>(nccl_of(comm)), stream);
  if (r) snprintf(g_err, sizeof(g_err), "ncclAllReduce: %s", g_api.error_string(r));
  return r;
}

// Generic in-place all-reduce. dtype: 0 int64, 1 uint8, 2 int32, 3 f32, 4 f64; op: 0 sum, 2 max, 3 min.
COBALT_API int cobalt_comm_allreduce(void* comm, void* buf, int64_t count, int dtype, int op, hipStream_t stream) {
  const int dt = dtype_code(dtype);
  if (dt < 0 || (op != kSum && op != kMax && op != kMin)) return -3;
  if (is_loop(comm)) return loop_allreduce(static_cast<CobaltComm*>(comm), buf, count, dtype, op, stream);
  if (is_ipc(comm)) return ipc_allreduce(static_cast<CobaltComm*>(comm), buf, count, dtype, op, stream);
  Result r = g_api.all_reduce(buf, buf, (size_t)count, dt, op, static_cast<Comm>(nccl_of(comm)), stream);
  if (r) snprintf(g_err, sizeof(g_err), "ncclAllReduce: %s", g_api.error_string(r));
  return r;
}

COBALT_API int cobalt_comm_allgather(void* comm, const void* send, void* recv, int64_t count, int dtype,
                                     hipStream_t stream) {
  const int dt = dtype_code(dtype);
  if (dt < 0) return -3;
  if (is_loop(comm)) return loop_allgather(static_cast<CobaltComm*>(comm), send, recv, count, dtype, stream);
  if (is_ipc(comm)) { comm_set_error("ipc: all-gather is not provided by the IPC group"); return -3; }
  Result r = g_api.all_gather(send, recv, (size_t)count, dt, static_cast<Comm>(nccl_of(comm)), stream);
  if (r) snprintf(g_err, sizeof(g_err), "ncclAllGather: %s", g_api.error_string(r));
  return r;
}
