// Collectives of the multi-GPU engine: RCCL over xGMI (production) and the
// in-process local group (tests).  See comm.hpp.
//
// The reference exchanges every per-level frontier with blocking MPI
// collectives over host arrays (MPI_Allreduce BOR over N
// ints, v4/mpi_bas.cpp:107).  Here every collective is enqueued on a HIP
// stream over device buffers; RCCL has no bitwise-OR reduction, so the engine
// is built on allgather of owned slices plus sum / min / max reductions.
#include "comm.hpp"

#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>

#include "device.hpp"

namespace bibfs {
namespace dist {

#define RCCL_CHECK(expr)                                                                  \
  do {                                                                                    \
    ncclResult_t _r = (expr);                                                             \
    if (_r != ncclSuccess)                                                                \
      throw ::bibfs::Error(std::string("RCCL error ") + ncclGetErrorString(_r) + " at " + \
                           __FILE__ + ":" + std::to_string(__LINE__));                    \
  } while (0)

namespace {

ncclDataType_t nccl_type(DType t) {
  switch (t) {
    case DType::kU32: return ncclUint32;
    case DType::kU64: return ncclUint64;
    default: return ncclFloat64;
  }
}

ncclRedOp_t nccl_op(ROp o) {
  switch (o) {
    case ROp::kSum: return ncclSum;
    case ROp::kMin: return ncclMin;
    default: return ncclMax;
  }
}

size_t type_size(DType t) { return t == DType::kU32 ? 4 : 8; }

class RcclComm final : public Comm {
 public:
  RcclComm(int rank, int size, const std::vector<uint8_t>& uid) : rank_(rank), size_(size) {
    BIBFS_REQUIRE(uid.size() == sizeof(ncclUniqueId), "bad RCCL unique id size");
    ncclUniqueId id;
    std::memcpy(&id, uid.data(), sizeof(id));
    RCCL_CHECK(ncclCommInitRank(&comm_, size, id, rank));
    int count = 0;
    RCCL_CHECK(ncclCommCount(comm_, &count));  // the rank count the communicator itself reports
    BIBFS_REQUIRE(count == size, "RCCL communicator has " + std::to_string(count) + " ranks, expected " +
                                     std::to_string(size));
  }
  ~RcclComm() override {
    if (comm_ && !aborted_) (void)ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* name() const override { return "rccl"; }
  void group_begin() override {
    live();
    RCCL_CHECK(ncclGroupStart());
  }
  void group_end() override { RCCL_CHECK(ncclGroupEnd()); }
  // A one-rank collective is the identity: no RCCL launch (and none of its
  // internal stream hand-offs) on the world-1 path.
  void allreduce(void* buf, size_t count, DType t, ROp op, hipStream_t s) override {
    live();
    if (size_ == 1) return;
    RCCL_CHECK(ncclAllReduce(buf, buf, count, nccl_type(t), nccl_op(op), comm_, s));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    live();
    if (size_ == 1) {
      if (send != recv && bytes) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    if (bytes % 4 == 0)
      RCCL_CHECK(ncclAllGather(send, recv, bytes / 4, ncclUint32, comm_, s));
    else
      RCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
  }
  // One grouped send/recv per peer (RCCL fuses the group into one launch);
  // a message to itself is a device copy.
  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    live();
    const char* sp = static_cast<const char*>(send);
    char* rp = static_cast<char*>(recv);
    if (bytes) HIP_CHECK(hipMemcpyAsync(rp + (size_t)rank_ * bytes, sp + (size_t)rank_ * bytes, bytes,
                                        hipMemcpyDeviceToDevice, s));
    if (size_ == 1) return;
    const bool words = bytes % 4 == 0;
    const size_t count = words ? bytes / 4 : bytes;
    const ncclDataType_t ty = words ? ncclUint32 : ncclUint8;
    RCCL_CHECK(ncclGroupStart());
    for (int r = 0; r < size_; ++r) {
      if (r == rank_) continue;
      RCCL_CHECK(ncclSend(sp + (size_t)r * bytes, count, ty, r, comm_, s));
      RCCL_CHECK(ncclRecv(rp + (size_t)r * bytes, count, ty, r, comm_, s));
    }
    RCCL_CHECK(ncclGroupEnd());
  }
  void check() override {
    live();
    ncclResult_t e = ncclSuccess;
    RCCL_CHECK(ncclCommGetAsyncError(comm_, &e));
    if (e != ncclSuccess && e != ncclInProgress)
      throw Error(std::string("RCCL asynchronous error on rank ") + std::to_string(rank_) + ": " +
                  ncclGetErrorString(e));
  }
  void abort() override {
    if (aborted_.exchange(true)) return;
    (void)ncclCommAbort(comm_);  // outstanding collectives of every rank on this comm return
  }
  bool aborted() const override { return aborted_; }

 private:
  void live() const {
    if (aborted_) throw Error("RCCL communicator was aborted after an earlier failure");
  }
  int rank_, size_;
  ncclComm_t comm_ = nullptr;
  std::atomic<bool> aborted_{false};
};

}  // namespace

// P ranks = P host threads of one process sharing one GPU.  A collective is a
// host rendezvous that swaps {buffer pointer, "ready" event} between the
// ranks; the data then moves with device-to-device copies on each rank's own
// stream, ordered by stream-waits on the other ranks' events -- no stream is
// drained and no byte goes through the host.
struct LocalGroup {
  LocalGroup(int p, double t) : P(p), timeout_s(t), slot((size_t)p) {}
  struct Slot {
    const void* src = nullptr;
    hipEvent_t ready = nullptr;  // recorded after the source bytes are final
    hipEvent_t done = nullptr;   // recorded after this rank copied everyone's bytes
  };
  const int P;
  const double timeout_s;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::atomic<uint64_t> gen_pub{0};  // gen / aborted, readable without the mutex (the spin)
  std::atomic<bool> aborted_pub{false};
  std::vector<Slot> slot;

  // Ranks arrive within microseconds of each other every round: a waiter
  // spins on the generation for up to kSpinUs before it sleeps on the
  // condition variable (a futex wake-up costs more than the round's kernels).
  static constexpr double kSpinUs = 200.0;
  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw Error("local group aborted by another rank");
    const uint64_t g = gen;
    if (++arrived == P) {
      arrived = 0;
      gen_pub.store(++gen, std::memory_order_release);
      cv.notify_all();
      return;
    }
    lk.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t k = 0;; ++k) {
      if (gen_pub.load(std::memory_order_acquire) != g || aborted_pub.load(std::memory_order_acquire)) break;
      if ((k & 255) == 255 &&
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() > kSpinUs)
        break;
    }
    lk.lock();
    const auto deadline = std::chrono::steady_clock::now() + std::chrono::duration<double>(timeout_s);
    if (!cv.wait_until(lk, deadline, [&] { return gen != g || aborted; })) {
      aborted = true;  // a peer never arrived: fail the whole group, not just this rank
      aborted_pub.store(true, std::memory_order_release);
      cv.notify_all();
      throw Error("local group collective timed out after " + std::to_string(timeout_s) + " s");
    }
    if (gen == g) throw Error("local group aborted by another rank");
  }
};

namespace {

template <typename T>
__global__ void k_local_reduce(const T* __restrict__ parts, T* __restrict__ out, size_t count, int P, int op) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < count; i += (size_t)gridDim.x * blockDim.x) {
    T acc = parts[i];
    for (int r = 1; r < P; ++r) {
      const T x = parts[(size_t)r * count + i];
      acc = op == 0 ? acc + x : (op == 1 ? (x < acc ? x : acc) : (x > acc ? x : acc));
    }
    out[i] = acc;
  }
}

class LocalComm final : public Comm {
 public:
  LocalComm(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), rank_(rank) {
    HIP_CHECK(hipEventCreateWithFlags(&ready_, hipEventDisableTiming));
    HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
  }
  ~LocalComm() override {
    if (scratch_) (void)hipFree(scratch_);
    (void)hipEventDestroy(ready_);
    (void)hipEventDestroy(done_);
  }
  int rank() const override { return rank_; }
  int size() const override { return g_->P; }
  const char* name() const override { return "local"; }

  void allreduce(void* buf, size_t count, DType t, ROp op, hipStream_t s) override {
    if (g_->P == 1 || count == 0) return;
    const size_t bytes = count * type_size(t);
    if (scratch_bytes_ < bytes * g_->P) {
      HIP_CHECK(hipStreamSynchronize(s));
      if (scratch_) HIP_CHECK(hipFree(scratch_));
      scratch_bytes_ = std::max<size_t>(bytes * g_->P, 4096);
      HIP_CHECK(hipMalloc(&scratch_, scratch_bytes_));
    }
    exchange(buf, scratch_, bytes, s);
    const int o = op == ROp::kSum ? 0 : (op == ROp::kMin ? 1 : 2);
    const unsigned blocks = (unsigned)std::min<size_t>((count + 255) / 256, 64);
    switch (t) {
      case DType::kU32:
        k_local_reduce<uint32_t><<<blocks, 256, 0, s>>>(static_cast<const uint32_t*>(scratch_),
                                                        static_cast<uint32_t*>(buf), count, g_->P, o);
        break;
      case DType::kU64:
        k_local_reduce<unsigned long long><<<blocks, 256, 0, s>>>(
            static_cast<const unsigned long long*>(scratch_), static_cast<unsigned long long*>(buf), count, g_->P, o);
        break;
      case DType::kF64:
        k_local_reduce<double><<<blocks, 256, 0, s>>>(static_cast<const double*>(scratch_),
                                                      static_cast<double*>(buf), count, g_->P, o);
        break;
    }
    HIP_CHECK(hipGetLastError());
  }

  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (g_->P == 1) {
      if (bytes && send != recv) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    exchange(send, recv, bytes, s);
  }

  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (g_->P == 1) {
      if (bytes && send != recv) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    exchange(send, recv, bytes, s, true);
  }

  // In place: every rank's {send, ready} swapped as in exchange(), then the
  // caller's kernels read the peers' blocks where they are; release records
  // `done` behind them and orders this rank's next writes of its own send
  // buffer after every peer's reads (the second half of exchange()).
  void alltoall_view(const void* send, void* recv, size_t bytes, hipStream_t s, const void** peers) override {
    LocalGroup& G = *g_;
    if (G.P == 1) {
      peers[0] = send;
      return;
    }
    if (aborted_) throw Error("local group communicator was aborted after an earlier failure");
    HIP_CHECK(hipEventRecord(ready_, s));
    {
      std::lock_guard<std::mutex> lk(G.mu);
      G.slot[(size_t)rank_] = {send, ready_, done_};
    }
    G.barrier();
    {
      std::lock_guard<std::mutex> lk(G.mu);
      view_peers_ = G.slot;
    }
    for (int r = 0; r < G.P; ++r) {
      if (r != rank_) HIP_CHECK(hipStreamWaitEvent(s, view_peers_[(size_t)r].ready, 0));
      peers[r] = static_cast<const char*>(view_peers_[(size_t)r].src) + (size_t)rank_ * bytes;
    }
    in_view_ = true;
  }
  void alltoall_release(hipStream_t s) override {
    if (!in_view_) return;
    in_view_ = false;
    LocalGroup& G = *g_;
    HIP_CHECK(hipEventRecord(done_, s));
    G.barrier();  // every rank's reads enqueued and its `done` recorded
    for (int r = 0; r < G.P; ++r)
      if (r != rank_) HIP_CHECK(hipStreamWaitEvent(s, view_peers_[(size_t)r].done, 0));
  }

  // (no dev_window: the ranks' streams share this process's hardware queues,
  // and a claim kernel spinning at the head of one would block the very peer
  // kernel it waits for -- only ranks with queues of their own, the IPC
  // transport's processes, order their exchange on the device)

  void check() override {
    if (g_->aborted_pub.load(std::memory_order_acquire)) throw Error("local group aborted by another rank");
  }

  void abort() override {
    aborted_ = true;
    abort_local_group(*g_);
  }
  bool aborted() const override { return aborted_; }

 private:
  // recv[r] = rank r's src, for every r (addressed: rank r's src block
  // `rank_`); ordered on `s` after every rank's producer work, and every
  // rank's later writes to its src ordered after every copy out of it.
  void exchange(const void* src, void* recv, size_t bytes, hipStream_t s, bool addressed = false) {
    if (aborted_) throw Error("local group communicator was aborted after an earlier failure");
    LocalGroup& G = *g_;
    HIP_CHECK(hipEventRecord(ready_, s));
    {
      std::lock_guard<std::mutex> lk(G.mu);
      G.slot[(size_t)rank_] = {src, ready_, done_};
    }
    G.barrier();  // every rank's {src, ready} published
    std::vector<LocalGroup::Slot> peers;
    {
      std::lock_guard<std::mutex> lk(G.mu);
      peers = G.slot;
    }
    for (int r = 0; r < G.P; ++r) {
      const LocalGroup::Slot& x = peers[(size_t)r];
      if (r != rank_) HIP_CHECK(hipStreamWaitEvent(s, x.ready, 0));
      if (bytes)
        HIP_CHECK(hipMemcpyAsync(static_cast<char*>(recv) + (size_t)r * bytes,
                                 static_cast<const char*>(x.src) + (addressed ? (size_t)rank_ * bytes : 0), bytes,
                                 hipMemcpyDeviceToDevice, s));
    }
    HIP_CHECK(hipEventRecord(done_, s));
    G.barrier();  // every rank's copies enqueued and its `done` recorded
    for (int r = 0; r < G.P; ++r)
      if (r != rank_) HIP_CHECK(hipStreamWaitEvent(s, peers[(size_t)r].done, 0));
    // No third rendezvous: a rank re-records `ready` only before the next
    // collective's first barrier, which every peer reaches after its waits above.
  }

  std::shared_ptr<LocalGroup> g_;
  int rank_;
  hipEvent_t ready_ = nullptr, done_ = nullptr;
  void* scratch_ = nullptr;
  size_t scratch_bytes_ = 0;
  bool aborted_ = false;
  std::vector<LocalGroup::Slot> view_peers_;  // alltoall_view -> alltoall_release
  bool in_view_ = false;
};

}  // namespace

std::vector<uint8_t> rccl_unique_id() {
  ncclUniqueId id;
  RCCL_CHECK(ncclGetUniqueId(&id));
  return std::vector<uint8_t>(reinterpret_cast<uint8_t*>(&id), reinterpret_cast<uint8_t*>(&id) + sizeof(id));
}

std::unique_ptr<Comm> make_rccl_comm(int rank, int size, const std::vector<uint8_t>& uid) {
  BIBFS_REQUIRE(size >= 1 && rank >= 0 && rank < size, "bad RCCL rank / size");
  return std::unique_ptr<Comm>(new RcclComm(rank, size, uid));
}

std::shared_ptr<LocalGroup> make_local_group(int size, double timeout_s) {
  BIBFS_REQUIRE(size >= 1, "local group needs at least one rank");
  BIBFS_REQUIRE(timeout_s > 0, "local group timeout must be positive");
  return std::make_shared<LocalGroup>(size, timeout_s);
}

std::unique_ptr<Comm> make_local_comm(std::shared_ptr<LocalGroup> g, int rank) {
  BIBFS_REQUIRE(g && rank >= 0 && rank < g->P, "bad local-group rank");
  return std::unique_ptr<Comm>(new LocalComm(std::move(g), rank));
}

void abort_local_group(LocalGroup& g) {
  std::lock_guard<std::mutex> lk(g.mu);
  g.aborted = true;
  g.aborted_pub.store(true, std::memory_order_release);
  g.cv.notify_all();
}

}  // namespace dist
}  // namespace bibfs
