// Collective layer of the multi-GPU engine (internal header).
//
// Production: RCCL over xGMI, one process per GPU (make_rccl_comm).  The
// engine only ever issues the handful of collectives below, always on a HIP
// stream, so the same engine code also runs over an in-process "local group"
// (make_local_comm): P host threads that share one GPU and exchange through
// host staging.  The local group is test infrastructure (SURVEY.md §4 item 5:
// validate the partition / ownership / exchange logic with P > 1 on a box
// with one GPU); it is never used for a measured number.
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
};

std::vector<uint8_t> rccl_unique_id();
std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& uid);

struct LocalGroup;
std::shared_ptr<LocalGroup> make_local_group(int size);
std::unique_ptr<Comm> make_local_comm(std::shared_ptr<LocalGroup> g, int rank);
// Wake every rank blocked in a local collective with an error (a rank failed).
void abort_local_group(LocalGroup& g);

}  // namespace dist
}  // namespace bibfs
