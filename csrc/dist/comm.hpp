// Collective layer of the multi-GPU engine (internal header).
//
// Production: RCCL over xGMI, one process per GPU (make_rccl_comm).  Separate
// processes that share a GPU (RCCL refuses that) use the IPC transport
// (make_ipc_comm), which also runs one process per GPU.  The
// engine only ever issues the handful of collectives below, always on a HIP
// stream, so the same engine code also runs over an in-process "local group"
// (make_local_comm): P host threads that share one GPU.  The local group
// moves data with device-to-device copies ordered by HIP events between the
// ranks' streams (the host only rendezvouses to swap buffer pointers and
// events), so stream ordering, overlap and the engine's no-host-sync rounds
// behave as they do over RCCL.  It is test infrastructure (SURVEY.md §4 item
// 5: validate the partition / ownership / exchange logic with P > 1 on a box
// with one GPU); it is never used for a measured multi-GPU number.
//
// Failure handling (the reference aborts the job on any error:
// v2/second_try.cpp:35, v4/mpi_bas.cpp:33, v3/bibfs_cuda_only.cu:6-10):
// `abort()` tears the communicator down so peers blocked in a collective
// return (ncclCommAbort / waking the local group), `check()` surfaces an
// asynchronous RCCL error, and the local group's rendezvous has a timeout.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

namespace bibfs {
namespace dist {

enum class DType { kU32, kU64, kF64 };
enum class ROp { kSum, kMin, kMax };

class Comm {
 public:
  virtual ~Comm() = default;
  virtual int rank() const = 0;
  virtual int size() const = 0;
  virtual const char* name() const = 0;
  // Collectives between group_begin / group_end are issued as one group (RCCL
  // fuses them into one launch); every rank issues the same sequence.
  virtual void group_begin() {}
  virtual void group_end() {}
  // In place, device memory, enqueued on `s`.
  virtual void allreduce(void* buf, size_t count, DType t, ROp op, hipStream_t s) = 0;
  // recv = P consecutive blocks of `bytes` (block r from rank r); device memory.
  virtual void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // Owner-addressed exchange: send = P blocks of `bytes` (block r goes to rank
  // r), recv = P blocks (block r came from rank r); device memory.
  virtual void alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) = 0;
  // The same exchange read in place where the transport can: `peers[r]` (P
  // entries) is set to a device pointer to the block rank r addressed to this
  // rank, readable by work enqueued on `s` until alltoall_release(s); the
  // caller leaves `send` untouched until then.  Default: alltoall into `recv`
  // and point into it.  The local group points straight into the peers' send
  // buffers: no copy at all.
  virtual void alltoall_view(const void* send, void* recv, size_t bytes, hipStream_t s, const void** peers) {
    alltoall(send, recv, bytes, s);
    for (int r = 0; r < size(); ++r) peers[r] = static_cast<const char*>(recv) + (size_t)r * bytes;
  }
  virtual void alltoall_release(hipStream_t s) {}
  // Device-synchronised exchange window (collective: every rank calls it with
  // the same `bytes`).  Each rank gets `bytes` of device memory whose first
  // kWinFlagBytes hold its epoch flag, and device pointers to every peer's
  // window that its kernels may read in place; ranks then order their
  // exchanges by polling the peers' flags on the device, with no host
  // rendezvous.  Only where every rank's memory is mapped on the caller's
  // device and every rank has hardware queues of its own (IPC ranks that
  // share one GPU: one process each).  False: not supported (RCCL; the local
  // group, whose ranks' streams share one process's queues), nothing was
  // allocated.  The window lives as long as the communicator.
  static constexpr int kWinMax = 16;
  static constexpr size_t kWinFlagBytes = 256;
  struct Window {
    void* mine = nullptr;
    const void* peer[kWinMax] = {};
  };
  virtual bool dev_window(size_t bytes, Window& w) { return false; }
  // Throw if the communicator reported an asynchronous error (peer failure).
  virtual void check() {}
  // Abort every outstanding and future collective of this communicator
  // (peers blocked in one return with an error).  Idempotent.
  virtual void abort() = 0;
  virtual bool aborted() const = 0;
  // Watchdog of a transport whose host waits for its peers (ipc).
  virtual void set_timeout(double seconds) {}
};

std::vector<uint8_t> rccl_unique_id();
std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& uid);

// P processes, on one GPU or several, exchanging through IPC-mapped staging
// buffers (ipc_comm.hip).  The id names the group's shared-memory control
// segment; rank 0 makes it (ipc_unique_id) and hands it to the other ranks
// over any channel (MPI_Bcast, torch.distributed), as with an RCCL unique id.
std::vector<uint8_t> ipc_unique_id();
std::unique_ptr<Comm> make_ipc_comm(int rank, int size, const std::vector<uint8_t>& uid, double timeout_s = 120.0);

struct LocalGroup;
// `timeout_s`: a rank waiting longer than this in a rendezvous aborts the group.
std::shared_ptr<LocalGroup> make_local_group(int size, double timeout_s = 120.0);
std::unique_ptr<Comm> make_local_comm(std::shared_ptr<LocalGroup> g, int rank);
// Wake every rank blocked in a local collective with an error (a rank failed).
void abort_local_group(LocalGroup& g);

}  // namespace dist
}  // namespace bibfs
