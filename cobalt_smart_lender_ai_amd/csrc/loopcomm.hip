// In-process loopback communicator: N "ranks" that are host threads of ONE process driving ONE
// device, each on its own HIP stream. Test infrastructure for the data-parallel GBDT protocol: a
// 1-GPU box cannot host two RCCL ranks (RCCL refuses duplicate devices), but the trainer's
// multi-rank code path -- per-rank row shards, per-level collectives enqueued mid-tree from C++ --
// runs unchanged against this group, so N-rank training can be checked byte-for-byte against a
// single-rank fit without a multi-GPU node (tests/test_gpu_gbdt.py).
//
// A collective is two host barriers and stream-ordered events: every rank records "my input is
// ready" on its stream, the ranks meet, each stream waits on all the others' events and reduces
// all N buffers (same device, plain loads) into a private staging buffer, records "done reading";
// the ranks meet again, each stream waits for all readers and copies its result back in place.
// Host threads only meet at enqueue time, never wait for the GPU.
#include "comm.h"

#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

struct LoopGroup {
  int n;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool broken = false;
  int refs = 0;
  std::vector<const void*> bufs;
  std::vector<hipEvent_t> ev_in, ev_mid;
  std::vector<void*> tmp;
  std::vector<size_t> tmp_bytes;

  // false when the group is broken: a rank left (its handle was destroyed, e.g. it failed) or the
  // meeting timed out -- every waiter then fails fast instead of hanging
  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const uint64_t g = gen;
    if (++arrived == n) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return true;
    }
    cv.wait_for(lk, std::chrono::seconds(timeout_s), [&] { return gen != g || broken; });
    if (gen != g) return true;  // completed (a rank may have left right after it)
    broken = true;
    cv.notify_all();
    return false;
  }
  int timeout_s = 300;
};

namespace {

constexpr int kMaxLoopRanks = 64;
struct RankPtrs {  // passed by value: no host-to-device upload of the pointer table
  const void* p[kMaxLoopRanks];
};

template <typename T, int OP>
__global__ __launch_bounds__(256) void k_loop_reduce(RankPtrs bufs, int n, int64_t count, T* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x) {
    T acc = static_cast<const T*>(bufs.p[0])[i];
    for (int r = 1; r < n; ++r) {
      const T v = static_cast<const T*>(bufs.p[r])[i];
      acc = OP == 0 ? acc + v : (OP == 2 ? (v > acc ? v : acc) : (v < acc ? v : acc));
    }
    out[i] = acc;
  }
}

template <typename T>
int launch_reduce(const RankPtrs& b, int n, int64_t count, int op, void* out, hipStream_t s) {
  const int grid = (int)std::min<int64_t>((count + 255) / 256, 4096);
  auto o = static_cast<T*>(out);
  if (op == 0) hipLaunchKernelGGL((k_loop_reduce<T, 0>), dim3(grid), dim3(256), 0, s, b, n, count, o);
  else if (op == 2) hipLaunchKernelGGL((k_loop_reduce<T, 2>), dim3(grid), dim3(256), 0, s, b, n, count, o);
  else if (op == 3) hipLaunchKernelGGL((k_loop_reduce<T, 3>), dim3(grid), dim3(256), 0, s, b, n, count, o);
  else return -3;
  return hipGetLastError() == hipSuccess ? 0 : -4;
}

int elem_size(int dtype) {
  switch (dtype) {
    case 0: case 4: return 8;
    case 1: return 1;
    case 2: case 3: return 4;
    default: return -1;
  }
}

// per-rank staging buffer, grown on demand (at least 64 MiB, so a fit never re-allocates)
int ensure_tmp(LoopGroup* g, int rank, size_t bytes) {
  const size_t need = std::max<size_t>(bytes, (size_t)64 << 20);
  if (g->tmp_bytes[rank] >= need) return 0;
  if (g->tmp[rank]) hipFree(g->tmp[rank]);
  g->tmp[rank] = nullptr;
  g->tmp_bytes[rank] = 0;
  if (hipMalloc(&g->tmp[rank], need) != hipSuccess) return -5;
  g->tmp_bytes[rank] = need;
  return 0;
}

}  // namespace

#define COBALT_API extern "C" __attribute__((visibility("default")))

COBALT_API int cobalt_comm_loop_group(int nranks, void** out) {
  if (nranks < 1 || nranks > kMaxLoopRanks) return -3;
  LoopGroup* g = new LoopGroup();
  g->n = nranks;
  g->bufs.assign(nranks, nullptr);
  g->ev_in.assign(nranks, nullptr);
  g->ev_mid.assign(nranks, nullptr);
  g->tmp.assign(nranks, nullptr);
  g->tmp_bytes.assign(nranks, 0);
  for (int r = 0; r < nranks; ++r) {
    if (hipEventCreateWithFlags(&g->ev_in[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g->ev_mid[r], hipEventDisableTiming) != hipSuccess)
      return -5;
  }
  *out = g;
  return 0;
}

COBALT_API int cobalt_comm_loop_rank(void* group, int rank, void** out) {
  LoopGroup* g = static_cast<LoopGroup*>(group);
  if (!g || rank < 0 || rank >= g->n) return -3;
  CobaltComm* c = new CobaltComm{1, nullptr, g, rank, g->n};
  {
    std::lock_guard<std::mutex> lk(g->mu);
    ++g->refs;
  }
  *out = c;
  return 0;
}

// Frees the group once every rank handle has been destroyed (cobalt_comm_destroy).
COBALT_API int cobalt_comm_loop_group_free(void* group) {
  LoopGroup* g = static_cast<LoopGroup*>(group);
  if (!g) return 0;
  {
    std::lock_guard<std::mutex> lk(g->mu);
    if (g->refs) return -6;
  }
  hipDeviceSynchronize();
  for (int r = 0; r < g->n; ++r) {
    if (g->tmp[r]) hipFree(g->tmp[r]);
    hipEventDestroy(g->ev_in[r]);
    hipEventDestroy(g->ev_mid[r]);
  }
  delete g;
  return 0;
}

void loop_release(CobaltComm* c) {
  std::lock_guard<std::mutex> lk(c->group->mu);
  --c->group->refs;
  c->group->broken = true;  // a departed rank can never join another collective
  c->group->cv.notify_all();
}

int loop_allreduce(CobaltComm* c, void* buf, int64_t count, int dtype, int op, hipStream_t stream) {
  LoopGroup* g = c->group;
  const int r = c->rank, n = g->n;
  const int es = elem_size(dtype);
  if (es < 0) return -3;
  if (n == 1 || count == 0) return 0;
  const size_t bytes = (size_t)count * es;
  if (ensure_tmp(g, r, bytes)) { comm_set_error("loopback: staging allocation failed"); return -5; }
  g->bufs[r] = buf;
  hipEventRecord(g->ev_in[r], stream);
  if (!g->barrier()) { comm_set_error("loopback: barrier timed out"); return -7; }
  for (int k = 0; k < n; ++k)
    if (k != r) hipStreamWaitEvent(stream, g->ev_in[k], 0);
  RankPtrs ptrs{};
  for (int k = 0; k < n; ++k) ptrs.p[k] = g->bufs[k];
  int rc;
  switch (dtype) {
    case 0: rc = launch_reduce<int64_t>(ptrs, n, count, op, g->tmp[r], stream); break;
    case 1: rc = launch_reduce<uint8_t>(ptrs, n, count, op, g->tmp[r], stream); break;
    case 2: rc = launch_reduce<int32_t>(ptrs, n, count, op, g->tmp[r], stream); break;
    case 3: rc = launch_reduce<float>(ptrs, n, count, op, g->tmp[r], stream); break;
    default: rc = launch_reduce<double>(ptrs, n, count, op, g->tmp[r], stream); break;
  }
  hipEventRecord(g->ev_mid[r], stream);
  if (!g->barrier()) { comm_set_error("loopback: barrier timed out"); return -7; }
  for (int k = 0; k < n; ++k)
    if (k != r) hipStreamWaitEvent(stream, g->ev_mid[k], 0);
  hipMemcpyAsync(buf, g->tmp[r], bytes, hipMemcpyDeviceToDevice, stream);
  // a third meeting keeps the next collective from re-recording events still being waited on
  if (!g->barrier()) { comm_set_error("loopback: barrier timed out"); return -7; }
  return rc;
}

int loop_allgather(CobaltComm* c, const void* send, void* recv, int64_t count, int dtype, hipStream_t stream) {
  LoopGroup* g = c->group;
  const int r = c->rank, n = g->n;
  const int es = elem_size(dtype);
  if (es < 0) return -3;
  const size_t bytes = (size_t)count * es;
  g->bufs[r] = send;
  hipEventRecord(g->ev_in[r], stream);
  if (!g->barrier()) { comm_set_error("loopback: barrier timed out"); return -7; }
  for (int k = 0; k < n; ++k) {
    if (k != r) hipStreamWaitEvent(stream, g->ev_in[k], 0);
  }
  for (int k = 0; k < n; ++k)
    hipMemcpyAsync(static_cast<char*>(recv) + k * bytes, g->bufs[k], bytes, hipMemcpyDeviceToDevice, stream);
  hipEventRecord(g->ev_mid[r], stream);
  if (!g->barrier()) { comm_set_error("loopback: barrier timed out"); return -7; }
  for (int k = 0; k < n; ++k)
    if (k != r) hipStreamWaitEvent(stream, g->ev_mid[k], 0);
  if (!g->barrier()) { comm_set_error("loopback: barrier timed out"); return -7; }
  return 0;
}
