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
  }
  ~RcclComm() override {
    if (comm_) (void)ncclCommDestroy(comm_);
  }
  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* name() const override { return "rccl"; }
  void group_begin() override { RCCL_CHECK(ncclGroupStart()); }
  void group_end() override { RCCL_CHECK(ncclGroupEnd()); }
  void allreduce(void* buf, size_t count, DType t, ROp op, hipStream_t s) override {
    RCCL_CHECK(ncclAllReduce(buf, buf, count, nccl_type(t), nccl_op(op), comm_, s));
  }
  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    if (bytes % 4 == 0)
      RCCL_CHECK(ncclAllGather(send, recv, bytes / 4, ncclUint32, comm_, s));
    else
      RCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, comm_, s));
  }

 private:
  int rank_, size_;
  ncclComm_t comm_ = nullptr;
};

}  // namespace

// P ranks = P host threads of one process.  Every collective: drain the
// caller's stream, stage its bytes in the rank's slot, barrier, combine, barrier.
struct LocalGroup {
  explicit LocalGroup(int p) : P(p), slot((size_t)p) {}
  const int P;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t gen = 0;
  bool aborted = false;
  std::vector<std::vector<uint8_t>> slot;

  void barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) throw Error("local group aborted by another rank");
    const uint64_t g = gen;
    if (++arrived == P) {
      arrived = 0;
      ++gen;
      cv.notify_all();
      return;
    }
    cv.wait(lk, [&] { return gen != g || aborted; });
    if (gen == g) throw Error("local group aborted by another rank");
  }
};

namespace {

template <typename T>
void combine(T* acc, const T* x, size_t n, ROp op) {
  for (size_t i = 0; i < n; ++i)
    acc[i] = op == ROp::kSum ? acc[i] + x[i] : (op == ROp::kMin ? std::min(acc[i], x[i]) : std::max(acc[i], x[i]));
}

class LocalComm final : public Comm {
 public:
  LocalComm(std::shared_ptr<LocalGroup> g, int rank) : g_(std::move(g)), rank_(rank) {}
  int rank() const override { return rank_; }
  int size() const override { return g_->P; }
  const char* name() const override { return "local"; }

  void allreduce(void* buf, size_t count, DType t, ROp op, hipStream_t s) override {
    const size_t bytes = count * type_size(t);
    HIP_CHECK(hipStreamSynchronize(s));
    auto& mine = g_->slot[(size_t)rank_];
    mine.resize(bytes);
    if (bytes) HIP_CHECK(hipMemcpy(mine.data(), buf, bytes, hipMemcpyDeviceToHost));
    g_->barrier();
    std::vector<uint8_t> acc(g_->slot[0]);
    for (int r = 1; r < g_->P; ++r) {
      const uint8_t* x = g_->slot[(size_t)r].data();
      switch (t) {
        case DType::kU32:
          combine(reinterpret_cast<uint32_t*>(acc.data()), reinterpret_cast<const uint32_t*>(x), count, op);
          break;
        case DType::kU64:
          combine(reinterpret_cast<uint64_t*>(acc.data()), reinterpret_cast<const uint64_t*>(x), count, op);
          break;
        case DType::kF64:
          combine(reinterpret_cast<double*>(acc.data()), reinterpret_cast<const double*>(x), count, op);
          break;
      }
    }
    g_->barrier();  // every rank has read every slot before any is rewritten
    if (bytes) HIP_CHECK(hipMemcpy(buf, acc.data(), bytes, hipMemcpyHostToDevice));
  }

  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    HIP_CHECK(hipStreamSynchronize(s));
    auto& mine = g_->slot[(size_t)rank_];
    mine.resize(bytes);
    if (bytes) HIP_CHECK(hipMemcpy(mine.data(), send, bytes, hipMemcpyDeviceToHost));
    g_->barrier();
    for (int r = 0; r < g_->P && bytes; ++r)
      HIP_CHECK(hipMemcpy(static_cast<char*>(recv) + (size_t)r * bytes, g_->slot[(size_t)r].data(), bytes,
                          hipMemcpyHostToDevice));
    g_->barrier();
  }

 private:
  std::shared_ptr<LocalGroup> g_;
  int rank_;
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

std::shared_ptr<LocalGroup> make_local_group(int size) {
  BIBFS_REQUIRE(size >= 1, "local group needs at least one rank");
  return std::make_shared<LocalGroup>(size);
}

std::unique_ptr<Comm> make_local_comm(std::shared_ptr<LocalGroup> g, int rank) {
  BIBFS_REQUIRE(g && rank >= 0 && rank < g->P, "bad local-group rank");
  return std::unique_ptr<Comm>(new LocalComm(std::move(g), rank));
}

void abort_local_group(LocalGroup& g) {
  std::lock_guard<std::mutex> lk(g.mu);
  g.aborted = true;
  g.cv.notify_all();
}

}  // namespace dist
}  // namespace bibfs
