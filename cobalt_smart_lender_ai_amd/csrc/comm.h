// Communicator handle shared by comm.cpp (RCCL) and loopcomm.hip (in-process loopback group).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct LoopGroup;

struct CobaltComm {
  int kind;          // 0 = RCCL communicator, 1 = loopback rank of an in-process group
  void* nccl;        // ncclComm_t (kind 0)
  LoopGroup* group;  // (kind 1)
  int rank, nranks;
};

// dtype: 0 int64, 1 uint8, 2 int32, 3 f32, 4 f64; op: 0 sum, 2 max, 3 min
int loop_allreduce(CobaltComm* c, void* buf, int64_t count, int dtype, int op, hipStream_t stream);
int loop_allgather(CobaltComm* c, const void* send, void* recv, int64_t count, int dtype, hipStream_t stream);
void loop_release(CobaltComm* c);
void comm_set_error(const char* msg);
