// One-shot all-reduce between the ranks of ONE node over IPC-mapped device buffers -- the
// data-parallel GBDT's per-level histogram collective without RCCL in the loop (SURVEY.md §2.7:
// "a custom one-shot xGMI all-reduce via IPC peer pointers if RCCL latency dominates").
//
// Every rank exports two send slots (parity = epoch & 1, `cap` bytes each) and an uncached flag word
// through hipIpcGetMemHandle; the handles travel once over the torch process group and every rank
// maps every peer's slots (hipIpcOpenMemHandle). One exchange = ONE kernel on the caller's stream:
//   1. block 0 publishes flag[me] = epoch with a system-scope release (the send slot was written by
//      earlier kernels of the stream, so it is complete and written back at the kernel boundary),
//   2. every block's wave 0 polls all peers' flags at once (lane r <- rank r) until they reach the
//      epoch (system-scope acquire, s_sleep back-off, an s_memrealtime deadline -> sticky error word,
//      mirrored to pinned host memory where the host watchdog polls it),
//   3. out[i] = peer_0[i] (+) ... (+) peer_{n-1}[i] in rank order -- each thread reads the n ranks'
//      elements together, so an 8-GPU exchange pulls from all 7 xGMI links at once instead of the
//      one-link-per-hop pattern of a ring,
//   4. the rank zeroes its OTHER slot for the next exchange's producer (the trainer's histogram
//      reduce accumulates straight into it).
// Slot reuse is safe without a second flag: a peer publishes epoch e only after its exchange e - 1
// (which read this rank's slot of parity e - 1) has finished on its stream, and this rank touches
// that slot again only after it has seen the peer's epoch-e flag.
// The same kernel serves 2-3 processes sharing ONE GPU (tests/test_00gpu_dp_ipc.py), the only
// multi-process configuration a 1-GPU box can run (RCCL refuses two ranks on one device).
#include "comm.h"
#include "common.h"
#include "ipc_device.h"

#include <string.h>
#include <algorithm>
#include <vector>

using cobalt::kWave;

namespace {

struct IpcPeers {  // by value: no pointer-table upload per exchange
  const char* x[kMaxIpcRanks];
  const unsigned* flag[kMaxIpcRanks];
};

template <typename T, int OP>
__device__ __forceinline__ T combine(T a, T b) {
  return OP == 0 ? a + b : (OP == 2 ? (b > a ? b : a) : (b < a ? b : a));
}

// Flag words: [0] = this rank's last published epoch (read by the peers), [kIpcStickyWord] = sticky
// failure (a wait of this rank timed out; later exchanges skip waiting). Both in the uncached
// allocation. The publish / wait protocol itself is ipc_publish / ipc_wait (ipc_device.h).

template <typename T, int OP>
__global__ __launch_bounds__(256) void k_ipc_exchange(IpcPeers p, const unsigned* const* __restrict__ ftab, int n,
                                                      int me, unsigned* myflag, unsigned epoch, int64_t slot_off,
                                                      int64_t count, T* __restrict__ out, int4* __restrict__ zero_dst,
                                                      int64_t zero_vec, unsigned* err_host, uint64_t timeout) {
  if (blockIdx.x == 0) ipc_publish(myflag, epoch);
  if (!ipc_wait(ftab, n, me, myflag, epoch, err_host, timeout)) return;
  const T* src[kMaxIpcRanks];
#pragma unroll
  for (int r = 0; r < kMaxIpcRanks; ++r) src[r] = reinterpret_cast<const T*>(p.x[r < n ? r : 0] + slot_off);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += stride) {
    T v[kMaxIpcRanks];
#pragma unroll
    for (int r = 0; r < kMaxIpcRanks; ++r)
      if (r < n) v[r] = src[r][i];  // all ranks' loads in flight before the first combine
    T acc = v[0];
#pragma unroll
    for (int r = 1; r < kMaxIpcRanks; ++r)
      if (r < n) acc = combine<T, OP>(acc, v[r]);
    out[i] = acc;
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < zero_vec; i += stride)
    zero_dst[i] = make_int4(0, 0, 0, 0);
}

// Decision-table probe (connect self-test of the node-owner path): every rank writes a record whose
// words encode its rank and the round into its table's spare last slot (system-scope stores, the tag
// last) and reads every peer's record back (tag poll + system-scope loads), as the trainer's owners and
// copying ranks do mid-kernel. result: 0 = every peer's record arrived intact, 1 = wrong words, 2 =
// a tag did not arrive before the deadline.
__global__ void k_ipc_dtab_probe(const IpcFusedView* v, unsigned round, unsigned* result) {
  if (threadIdx.x != 0) return;
  const int n = v->n, me = v->me;
  const int64_t slot = (int64_t)(kIpcDecNodes - 1) * kIpcDecStride;
  const unsigned long long tag = 0x5E1F7E57ull ^ ((unsigned long long)round << 32);
  char* mine = v->mydtab + slot;
  for (int w = 0; w < 24; ++w)
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(mine + w * 8),
                       ((unsigned long long)(me + 1) << 40) ^ ((unsigned long long)round << 20) ^ (unsigned long long)w,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __builtin_amdgcn_s_waitcnt(0);
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(mine + 192), tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  unsigned res = 0;
  for (int r = 0; r < n; ++r) {
    if (r == me) continue;
    const char* rec = v->dtab[r] + slot;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    bool ok = true;
    while (__hip_atomic_load(reinterpret_cast<const unsigned long long*>(rec + 192), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM) != tag) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > v->timeout) { ok = false; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok) { res |= 2u; continue; }
    for (int w = 0; w < 24; ++w) {
      const unsigned long long x = __hip_atomic_load(reinterpret_cast<const unsigned long long*>(rec + w * 8),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (x != (((unsigned long long)(r + 1) << 40) ^ ((unsigned long long)round << 20) ^ (unsigned long long)w))
        res |= 1u;
    }
  }
  *result = res;
}

int elem_bytes(int dtype) {
  switch (dtype) {
    case 0: case 4: return 8;
    case 1: return 1;
    case 2: case 3: return 4;
    default: return -1;
  }
}

}  // namespace

struct IpcGroup {
  int rank = 0, n = 1;
  int64_t cap = 0;             // bytes per send slot
  char* xbuf = nullptr;        // [2][cap], exported
  unsigned* flags = nullptr;   // uncached; flags[0] = last published epoch, exported
  char* dtab = nullptr;        // uncached node-owner decision table (kIpcDecBytes), exported: written and
                               // read by the ranks' kernels while they run, so not L2-cacheable memory
  unsigned* err_host = nullptr;  // pinned + mapped: [0] = a wait timed out (sticky)
  unsigned* err_dev = nullptr;
  IpcPeers peers{};
  const char* dpeer[kMaxIpcRanks] = {};  // every rank's decision table (own + mapped peers)
  const unsigned** ftab = nullptr;  // device copy of peers.flag (polled lane-parallel)
  IpcFusedView* views = nullptr;    // device [2]: the group per slot parity (ipc_device_views)
  std::vector<void*> opened;
  unsigned epoch = 0;          // exchanges enqueued so far (identical on every rank)
  uint64_t timeout_ticks = 0;  // s_memrealtime ticks (100 MHz)
};

#define IPC_CK(expr)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (expr);                                                               \
    if (e_ != hipSuccess) {                                                               \
      char m_[256];                                                                       \
      snprintf(m_, sizeof(m_), "ipc: %s failed: %s", #expr, hipGetErrorString(e_));       \
      comm_set_error(m_);                                                                 \
      return (int)e_;                                                                     \
    }                                                                                     \
  } while (0)

// Size of one rank's exported handle blob (send slots + flag word + decision table).
COBALT_API int cobalt_ipc_handle_bytes() { return (int)(3 * sizeof(hipIpcMemHandle_t)); }

// Allocate this rank's send slots (2 x cap_bytes) and flag word on the current device and write their
// IPC handles to handles_out (cobalt_ipc_handle_bytes() bytes). The comm is usable after connect.
COBALT_API int cobalt_ipc_create(int rank, int nranks, int64_t cap_bytes, double timeout_s, void** out,
                                 void* handles_out) {
  if (nranks < 1 || nranks > kMaxIpcRanks || rank < 0 || rank >= nranks || cap_bytes < 16) {
    comm_set_error("ipc: bad rank / size");
    return -3;
  }
  IpcGroup* g = new IpcGroup();
  g->rank = rank;
  g->n = nranks;
  g->cap = (cap_bytes + 255) / 256 * 256;
  g->timeout_ticks = (uint64_t)(std::max(0.001, timeout_s) * 1e8);
  IPC_CK(hipMalloc((void**)&g->xbuf, 2 * g->cap));
  IPC_CK(hipMemset(g->xbuf, 0, 2 * g->cap));
  IPC_CK(hipExtMallocWithFlags((void**)&g->dtab, kIpcDecBytes, hipDeviceMallocUncached));
  IPC_CK(hipMemset(g->dtab, 0, kIpcDecBytes));
  IPC_CK(hipExtMallocWithFlags((void**)&g->flags, 256, hipDeviceMallocUncached));
  IPC_CK(hipMemset(g->flags, 0, 256));
  IPC_CK(hipHostMalloc((void**)&g->err_host, 64, hipHostMallocMapped | hipHostMallocCoherent));
  memset(g->err_host, 0, 64);
  IPC_CK(hipHostGetDevicePointer((void**)&g->err_dev, g->err_host, 0));
  hipIpcMemHandle_t h[3];
  IPC_CK(hipIpcGetMemHandle(&h[0], g->xbuf));
  IPC_CK(hipIpcGetMemHandle(&h[1], g->flags));
  IPC_CK(hipIpcGetMemHandle(&h[2], g->dtab));
  memcpy(handles_out, h, sizeof(h));
  IPC_CK(hipDeviceSynchronize());
  g->peers.x[rank] = g->xbuf;
  g->peers.flag[rank] = g->flags;
  g->dpeer[rank] = g->dtab;
  *out = new CobaltComm{2, nullptr, nullptr, rank, nranks, g};
  return 0;
}

// Map every peer's slots from the gathered handle blobs (nranks x cobalt_ipc_handle_bytes()).
COBALT_API int cobalt_ipc_connect(void* comm, const void* all_handles) {
  CobaltComm* c = static_cast<CobaltComm*>(comm);
  if (!c || c->kind != 2) return -3;
  IpcGroup* g = c->ipc;
  const auto* hs = static_cast<const hipIpcMemHandle_t*>(all_handles);
  for (int r = 0; r < g->n; ++r) {
    if (r == g->rank) continue;
    void* px = nullptr;
    void* pf = nullptr;
    void* pd = nullptr;
    IPC_CK(hipIpcOpenMemHandle(&px, hs[3 * r], hipIpcMemLazyEnablePeerAccess));
    g->opened.push_back(px);
    IPC_CK(hipIpcOpenMemHandle(&pf, hs[3 * r + 1], hipIpcMemLazyEnablePeerAccess));
    g->opened.push_back(pf);
    IPC_CK(hipIpcOpenMemHandle(&pd, hs[3 * r + 2], hipIpcMemLazyEnablePeerAccess));
    g->opened.push_back(pd);
    g->peers.x[r] = static_cast<const char*>(px);
    g->peers.flag[r] = static_cast<const unsigned*>(pf);
    g->dpeer[r] = static_cast<const char*>(pd);
  }
  IPC_CK(hipMalloc((void**)&g->ftab, kMaxIpcRanks * sizeof(unsigned*)));
  IPC_CK(hipMemcpy(g->ftab, g->peers.flag, kMaxIpcRanks * sizeof(unsigned*), hipMemcpyHostToDevice));
  IpcFusedView hv[2] = {};
  for (int p = 0; p < 2; ++p) {
    for (int r = 0; r < g->n; ++r) {
      hv[p].slot[r] = g->peers.x[r] + (int64_t)p * g->cap;
      hv[p].dtab[r] = g->dpeer[r];
    }
    hv[p].mydtab = g->dtab;
    hv[p].ftab = g->ftab;
    hv[p].myflag = g->flags;
    hv[p].err_host = g->err_dev;
    hv[p].n = g->n;
    hv[p].me = g->rank;
    hv[p].timeout = g->timeout_ticks;
  }
  IPC_CK(hipMalloc((void**)&g->views, sizeof(hv)));
  IPC_CK(hipMemcpy(g->views, hv, sizeof(hv), hipMemcpyHostToDevice));
  return 0;
}

// Change the wait deadline (host + device views). Call with no exchange in flight (device idle): the
// connect self-test runs under a short deadline, the training under the long one.
COBALT_API int cobalt_ipc_set_timeout(void* comm, double timeout_s) {
  CobaltComm* c = static_cast<CobaltComm*>(comm);
  if (!c || c->kind != 2) return -3;
  IpcGroup* g = c->ipc;
  g->timeout_ticks = (uint64_t)(std::max(0.001, timeout_s) * 1e8);
  if (g->views) {
    IpcFusedView hv[2];
    IPC_CK(hipMemcpy(hv, g->views, sizeof(hv), hipMemcpyDeviceToHost));
    hv[0].timeout = hv[1].timeout = g->timeout_ticks;
    IPC_CK(hipMemcpy(g->views, hv, sizeof(hv), hipMemcpyHostToDevice));
  }
  return 0;
}

// Decision-table probe of the connect self-test (k_ipc_dtab_probe); every rank calls it with the same
// round. Returns the probe's result word (0 = ok), < 0 on a launch error.
COBALT_API int cobalt_ipc_dtab_selftest(void* comm, unsigned round, hipStream_t stream) {
  CobaltComm* c = static_cast<CobaltComm*>(comm);
  if (!c || c->kind != 2 || !c->ipc->views) return -3;
  unsigned* d_res = nullptr;
  IPC_CK(hipMalloc((void**)&d_res, sizeof(unsigned)));
  hipLaunchKernelGGL(k_ipc_dtab_probe, dim3(1), dim3(64), 0, stream, c->ipc->views, round, d_res);
  unsigned h_res = 0;
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipMemcpyAsync(&h_res, d_res, sizeof(unsigned), hipMemcpyDeviceToHost, stream);
  if (e == hipSuccess) e = hipStreamSynchronize(stream);
  (void)hipFree(d_res);
  if (e != hipSuccess) {
    comm_set_error("ipc: decision-table probe failed to run");
    return -(int)e;
  }
  return (int)h_res;
}

void* ipc_send_buffer(CobaltComm* c) {
  IpcGroup* g = c->ipc;
  return g->xbuf + (int64_t)((g->epoch + 1) & 1u) * g->cap;
}

int64_t ipc_capacity(CobaltComm* c) { return c->ipc->cap; }

int ipc_error(CobaltComm* c) {
  const unsigned e = __atomic_load_n(c->ipc->err_host, __ATOMIC_ACQUIRE);
  if (e) comm_set_error("ipc: a peer did not reach the exchange before the deadline (peer dead or hung)");
  return e ? 6 /* ncclSystemError-like */ : 0;
}

int ipc_zero_send(CobaltComm* c, int64_t bytes, hipStream_t stream) {
  IpcGroup* g = c->ipc;
  if (bytes > g->cap) { comm_set_error("ipc: zero beyond the slot capacity"); return -3; }
  IPC_CK(hipMemsetAsync(ipc_send_buffer(c), 0, (size_t)bytes, stream));
  return 0;
}

template <typename T>
static void launch_exchange(int op, dim3 grid, hipStream_t s, const IpcGroup* g, unsigned epoch, int64_t off,
                            int64_t count, void* out, int4* zd, int64_t zv) {
  T* o = static_cast<T*>(out);
#define IPC_LAUNCH(OPC)                                                                                       \
  hipLaunchKernelGGL((k_ipc_exchange<T, OPC>), grid, dim3(256), 0, s, g->peers, g->ftab, g->n, g->rank, g->flags, epoch, \
                     off, count, o, zd, zv, g->err_dev, g->timeout_ticks)
  if (op == 0) IPC_LAUNCH(0);
  else if (op == 2) IPC_LAUNCH(2);
  else IPC_LAUNCH(3);
#undef IPC_LAUNCH
}

int ipc_exchange(CobaltComm* c, void* out, int64_t count, int dtype, int op, int64_t zero_bytes, hipStream_t stream) {
  IpcGroup* g = c->ipc;
  const int es = elem_bytes(dtype);
  if (es < 0 || (op != 0 && op != 2 && op != 3)) return -3;
  if (count * es > g->cap || zero_bytes > g->cap || zero_bytes % 16 != 0) {
    comm_set_error("ipc: exchange larger than the slot capacity (COBALT_IPC_SLOT_MB)");
    return -3;
  }
  const unsigned e = ++g->epoch;
  const int64_t off = (int64_t)(e & 1u) * g->cap;
  int4* zd = reinterpret_cast<int4*>(g->xbuf + (int64_t)((e + 1) & 1u) * g->cap);
  const int64_t zv = zero_bytes / 16;
  const int64_t work = std::max<int64_t>(count, zv);
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>((work + 255) / 256, 1024)));
  if (!g->ftab) { comm_set_error("ipc: exchange before cobalt_ipc_connect"); return -3; }
  switch (dtype) {
    case 0: launch_exchange<int64_t>(op, grid, stream, g, e, off, count, out, zd, zv); break;
    case 1: launch_exchange<uint8_t>(op, grid, stream, g, e, off, count, out, zd, zv); break;
    case 2: launch_exchange<int32_t>(op, grid, stream, g, e, off, count, out, zd, zv); break;
    case 3: launch_exchange<float>(op, grid, stream, g, e, off, count, out, zd, zv); break;
    default: launch_exchange<double>(op, grid, stream, g, e, off, count, out, zd, zv); break;
  }
  IPC_CK(hipGetLastError());
  return 0;
}

unsigned ipc_next_epoch(CobaltComm* c) { return ++c->ipc->epoch; }

const IpcFusedView* ipc_device_views(CobaltComm* c) { return c->ipc->views; }

// In-place all-reduce of `buf` (generic path: the buffer is first copied into the send slot).
int ipc_allreduce(CobaltComm* c, void* buf, int64_t count, int dtype, int op, hipStream_t stream) {
  const int es = elem_bytes(dtype);
  if (es < 0) return -3;
  if (count * es > c->ipc->cap) {
    comm_set_error("ipc: all-reduce larger than the slot capacity (COBALT_IPC_SLOT_MB)");
    return -3;
  }
  if (c->nranks == 1) return 0;
  IPC_CK(hipMemcpyAsync(ipc_send_buffer(c), buf, (size_t)(count * es), hipMemcpyDeviceToDevice, stream));
  return ipc_exchange(c, buf, count, dtype, op, 0, stream);
}

void ipc_release(CobaltComm* c) {
  IpcGroup* g = c->ipc;
  if (!g) return;
  (void)hipDeviceSynchronize();
  for (void* p : g->opened) (void)hipIpcCloseMemHandle(p);
  if (g->xbuf) (void)hipFree(g->xbuf);
  if (g->flags) (void)hipFree(g->flags);
  if (g->dtab) (void)hipFree(g->dtab);
  if (g->ftab) (void)hipFree(g->ftab);
  if (g->views) (void)hipFree(g->views);
  if (g->err_host) (void)hipHostFree(g->err_host);
  delete g;
  c->ipc = nullptr;
}

// Exchanges enqueued so far (diagnostics / tests).
COBALT_API unsigned cobalt_ipc_epoch(void* comm) {
  CobaltComm* c = static_cast<CobaltComm*>(comm);
  return (c && c->kind == 2) ? c->ipc->epoch : 0u;
}

// ------------------------------------------------------------------------------------------
// Placement probe for ranks sharing one device through CU-masked streams (parallel/cumask.py):
// thread 0 of each block records where the block ran -- the XCC (HW_REG_XCC_ID) and the shader
// engine / array / CU fields of HW_REG_HW_ID -- as xcc << 16 | se << 8 | sh << 4 | cu. A stream whose
// mask leaves an XCC without CUs can never run that XCC's share of a grid (every XCC takes blocks
// round-robin), which is what the probe exposes on the configurations that complete.
namespace {
__global__ __launch_bounds__(64) void k_hw_ids(uint32_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t xcc, hw;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
  const uint32_t cu = (hw >> 8) & 0xFu, sh = (hw >> 12) & 0x1u, se = (hw >> 13) & 0x7u;
  out[blockIdx.x] = (xcc & 0xFu) << 16 | se << 8 | sh << 4 | cu;
}
}  // namespace

COBALT_API int cobalt_hw_ids(hipStream_t stream, int blocks, uint32_t* out) {
  if (blocks <= 0 || !out) return -3;
  hipLaunchKernelGGL(k_hw_ids, dim3(blocks), dim3(64), 0, stream, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
