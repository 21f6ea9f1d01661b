// Collective transport of the column-sharded engine (DESIGN.md "Multi-GPU").
//
// Every per-round exchange of the sharded engine goes through this
// interface, stream-ordered on the engine's HIP stream (column layout: O(N)
// allreduce / allgather; row layout adds the senders' rows by alltoallv):
//   RCCL   one process per GPU, RCCL (loaded at run time) over xGMI;
//   LOCAL  ranks are threads of one process (any devices, including G shards
//          on one GPU, which RCCL does not allow): the parity-test transport
//          for the sharded code path, built from hipMemcpyPeerAsync + a
//          reduction kernel + a host barrier.
// world == 1 needs no transport: both calls degenerate to a device copy.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

enum GhDType { GH_DT_U8 = 0, GH_DT_I32 = 1, GH_DT_U64 = 2 };
enum GhROp { GH_OP_SUM = 0, GH_OP_MAX = 1 };

struct GhComm {
  int rank = 0, world = 1;
  std::string err;
  virtual ~GhComm() {}
  // recv[x] = op over ranks of send[x], x < count. send may equal recv.
  virtual int allreduce(const void* send, void* recv, size_t count, GhDType dt, GhROp op,
                        hipStream_t s) = 0;
  // recv[r*bytes .. (r+1)*bytes) = rank r's send; send may alias
  // recv + rank*bytes (in place).
  virtual int allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // Personalized exchange (row layout): send holds one block per
  // destination rank in rank order (sendbytes[r] bytes for rank r), recv
  // receives one block per source rank (recvbytes[r] bytes from rank r) at
  // byte offset recvdispl[r], or in rank order back to back when recvdispl
  // is null. Host arrays of world entries; send and recv must not alias.
  virtual int alltoallv(const void* send, const size_t* sendbytes, void* recv, const size_t* recvbytes,
                        hipStream_t s, const size_t* recvdispl = nullptr) = 0;
  // Ranks that are threads of one process on one device (LOCAL): each
  // publishes a host pointer, its stream's work done; on return 0, all[r] is
  // rank r's pointer, and the caller may read the peers' published objects
  // and their device buffers (its own kernels) until share_done, which waits
  // for every rank's reads. 1: not available on this transport (no rank
  // waited).
  virtual int share(const void* mine, hipStream_t s, const void** all) {
    (void)mine, (void)s, (void)all;
    return 1;
  }
  virtual int share_done(hipStream_t s) {
    (void)s;
    return 0;
  }
};

size_t gh_dtype_size(GhDType dt);

// world == 1 (no transport)
GhComm* gh_comm_single();
// RCCL: id = 128-byte ncclUniqueId from gh_comm_rccl_unique_id on rank 0;
// the caller has selected the rank's device.
GhComm* gh_comm_rccl(int rank, int world, const uint8_t* id, std::string* err);
int gh_comm_rccl_unique_id(uint8_t* id, std::string* err);
// LOCAL: ranks rendezvous on the same key (<= 128 bytes, NUL-terminated)
GhComm* gh_comm_local(int rank, int world, const uint8_t* key, int device, std::string* err);
