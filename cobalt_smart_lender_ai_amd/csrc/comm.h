// Communicator handle shared by comm.cpp (RCCL), loopcomm.hip (in-process loopback group) and
// ipccomm.hip (one-shot all-reduce over IPC-mapped peer buffers).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct LoopGroup;
struct IpcGroup;

struct CobaltComm {
  int kind;          // 0 = RCCL communicator, 1 = loopback rank of an in-process group, 2 = IPC group
  void* nccl;        // ncclComm_t (kind 0)
  LoopGroup* group;  // (kind 1)
  int rank, nranks;
  IpcGroup* ipc;     // (kind 2)
};

constexpr int kMaxIpcRanks = 16;
// flag words: [0] = published epoch, [32] = sticky failure (this rank's later waits fail at once),
// [40] = failure notice for the PEERS: a rank whose wait timed out (or that saw a peer's notice) sets it,
// and every peer's next wait sees it and fails too -- so one rank's timeout surfaces as a timeout on
// every rank (instead of the others running on with a stale exchange and reporting a divergence)
constexpr int kIpcStickyWord = 32;
constexpr int kIpcFailWord = 40;

// The IPC group as seen by a kernel that performs the exchange itself (the GBDT split evaluation sums
// the ranks' histogram slots while it reads them), for one slot parity: rank r's send slot, the device
// table of the ranks' flag words, this rank's flag word (+ sticky failure word), the pinned host error
// word and the wait deadline. Two of them (parity 0 / 1) live in device memory for the group's
// lifetime, so a kernel takes one pointer + the epoch instead of a per-launch copy.
// Node-owner decision table (after the two send slots of every rank's exported buffer): per tree node
// one record of 3 Node images (the node and its two children, 64 B each) + an 8-byte epoch tag.
constexpr int kIpcDecStride = 256;
constexpr int kIpcDecNodes = 2048;  // trees of depth <= 10
constexpr int64_t kIpcDecBytes = (int64_t)kIpcDecStride * kIpcDecNodes;

struct IpcFusedView {
  const char* slot[kMaxIpcRanks];
  const char* dtab[kMaxIpcRanks];  // every rank's decision table (peer-mapped)
  char* mydtab;
  const unsigned* const* ftab;
  unsigned* myflag;
  unsigned* err_host;
  int n, me;
  unsigned long long timeout;
};

// dtype: 0 int64, 1 uint8, 2 int32, 3 f32, 4 f64; op: 0 sum, 2 max, 3 min
int loop_allreduce(CobaltComm* c, void* buf, int64_t count, int dtype, int op, hipStream_t stream);
int loop_allgather(CobaltComm* c, const void* send, void* recv, int64_t count, int dtype, hipStream_t stream);
void loop_release(CobaltComm* c);
void comm_set_error(const char* msg);

// IPC group (ipccomm.hip)
int ipc_allreduce(CobaltComm* c, void* buf, int64_t count, int dtype, int op, hipStream_t stream);
int ipc_error(CobaltComm* c);
void ipc_release(CobaltComm* c);
// The buffer the next exchange sends (this rank's IPC-exported slot of parity epoch + 1).
void* ipc_send_buffer(CobaltComm* c);
int64_t ipc_capacity(CobaltComm* c);
// Zero the first `bytes` of the next send buffer (stream-ordered; safe once this rank's previous
// exchange has run: every peer finished reading that slot before it published its own flag).
int ipc_zero_send(CobaltComm* c, int64_t bytes, hipStream_t stream);
// One exchange: publish the send buffer, wait for every peer's, out = sum over ranks (rank order),
// then zero the first `zero_bytes` of the following send buffer.
int ipc_exchange(CobaltComm* c, void* out, int64_t count, int dtype, int op, int64_t zero_bytes, hipStream_t stream);
// Start the next epoch for a kernel that exchanges by itself (publish + wait + sum inside it): returns
// the epoch; the kernel reads ipc_device_views(c)[epoch & 1].
unsigned ipc_next_epoch(CobaltComm* c);
const IpcFusedView* ipc_device_views(CobaltComm* c);
