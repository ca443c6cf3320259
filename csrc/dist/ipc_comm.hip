// Multi-process collectives over HIP IPC (comm.hpp: make_ipc_comm).
//
// P ranks are P processes.  They may share one GPU -- the reference's own v4
// launch shape, 4 MPI ranks on one machine's GPU (single_machine_bench.sh:9,52;
// v4/Makefile:64 uses 6) -- or sit on different GPUs of a node, where the very
// same loads read peer HBM over xGMI.  RCCL refuses two ranks on one device
// ("Duplicate GPU detected"), so this transport is what runs the partitioned
// engine as separate processes (separate HIP contexts and address spaces,
// cross-process collective order, abort between processes) on a one-GPU box,
// and it is an A/B point against RCCL for the small per-round blocks on a
// multi-GPU node.
//
// Data plane: every rank owns two IPC-exported staging buffers (ping-pong by
// collective index).  A collective copies the rank's payload into its
// staging slot, then ONE kernel on the caller's stream pulls every peer's
// block straight out of the peers' staging buffers (allgather / alltoall) or
// reduces them element-wise (allreduce).  Nothing goes through host memory.
//
// Control plane: a POSIX shared-memory segment (name = the group's unique id)
// with one cache line per rank.  A collective is: stage (one kernel that
// copies and then writes the collective's tag into pinned host memory),
// host-spin on that tag, publish "arrived at collective k", wait until every
// rank arrived at k, launch the pull kernel.  The device
// never spins on another process's work (a waiting rank is a host thread).
// The ping-pong slot makes one rendezvous per collective enough: slot k%2 is
// rewritten at collective k+2, after every peer arrived at k+1, and a peer
// arrives at k+1 only once its pull kernel of collective k has completed.
//
// Failure: abort() raises a flag in the segment that every waiting rank sees;
// a rank that waits past the timeout aborts the group; a waiting rank checks
// that its peers' processes are still alive (a killed rank aborts the group
// within milliseconds instead of at the timeout).
#include "comm.hpp"

#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <thread>

#include "device.hpp"

namespace bibfs {
namespace dist {

namespace {

constexpr int kIpcMax = 16;
constexpr uint64_t kIpcMagic = 0x4942465349504331ull;  // "1CPISFBI"

struct alignas(64) IpcRankSlot {
  std::atomic<uint64_t> arrived;  // collectives this rank has entered
  std::atomic<int32_t> pid;
  int32_t device;
  uint64_t gen[2];                // staging generation per slot (0 = none yet)
  uint64_t cap[2];
  hipIpcMemHandle_t handle[2];
};

struct IpcShm {
  std::atomic<uint64_t> magic;
  int32_t P;
  std::atomic<int32_t> attached;
  std::atomic<int32_t> aborted;   // 0, or 1 + the rank that aborted first
  std::atomic<int32_t> detached;  // ranks that closed their peer mappings (teardown)
  char why[240];
  IpcRankSlot r[kIpcMax];
};

struct IpcSrc {
  const unsigned char* p[kIpcMax];
};

// recv block r <- src.p[r] + off (null = skip: the block is already in place)
__global__ void k_ipc_gather(IpcSrc src, uint64_t off, unsigned char* __restrict__ recv, uint64_t bytes) {
  const int r = blockIdx.y;
  const unsigned char* s = src.p[r];
  if (!s) return;
  s += off;
  unsigned char* d = recv + (uint64_t)r * bytes;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((((uintptr_t)s | (uintptr_t)d | bytes) & 15) == 0) {
    const uint4* s4 = reinterpret_cast<const uint4*>(s);
    uint4* d4 = reinterpret_cast<uint4*>(d);
    for (uint64_t i = t; i < bytes / 16; i += stride) d4[i] = s4[i];
  } else if ((((uintptr_t)s | (uintptr_t)d | bytes) & 3) == 0) {
    const uint32_t* s1 = reinterpret_cast<const uint32_t*>(s);
    uint32_t* d1 = reinterpret_cast<uint32_t*>(d);
    for (uint64_t i = t; i < bytes / 4; i += stride) d1[i] = s1[i];
  } else {
    for (uint64_t i = t; i < bytes; i += stride) d[i] = s[i];
  }
}

// Stage a collective's payload into this rank's exported buffer, then tell the
// host: one workgroup copies, and after a system-scope release (the staged
// bytes reach memory every agent and XCD reads) thread 0 writes the
// collective's tag into pinned host memory, where the host spins -- the stream
// position is seen one PCIe write after it is reached (an event query sees
// it much later).  Larger payloads: hipMemcpyAsync, then this kernel with 0 bytes.
__global__ void k_ipc_stage(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n16,
                            const unsigned char* __restrict__ src_tail, unsigned char* __restrict__ dst_tail,
                            uint32_t tail, uint64_t* host_tag, uint64_t tag) {
  for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = src[i];
  if (threadIdx.x < tail) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(host_tag, tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <typename T>
__global__ void k_ipc_reduce(IpcSrc src, T* out, uint64_t count, int P, int op) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
    T acc = reinterpret_cast<const T*>(src.p[0])[i];
    for (int r = 1; r < P; ++r) {
      const T x = reinterpret_cast<const T*>(src.p[r])[i];
      acc = op == 0 ? acc + x : (op == 1 ? (x < acc ? x : acc) : (x > acc ? x : acc));
    }
    out[i] = acc;  // (this rank's own source may be `out`: element i is read before it is written)
  }
}

size_t tsize(DType t) { return t == DType::kU32 ? 4 : 8; }

bool pid_dead(int pid) {
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0 && errno == ESRCH) return true;
  // a killed rank stays a zombie until its launcher reaps it
  char path[64];
  std::snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char buf[256] = {0};
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  const char* rp = std::strrchr(buf, ')');  // "pid (comm) S ..."
  return n > 0 && rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X');
}

class IpcComm final : public Comm {
 public:
  IpcComm(int rank, int size, const std::string& name, double timeout_s)
      : rank_(rank), size_(size), name_(name), timeout_s_(timeout_s) {
    BIBFS_REQUIRE(size >= 1 && size <= kIpcMax, "ipc comm: 1.." + std::to_string(kIpcMax) + " ranks");
    BIBFS_REQUIRE(rank >= 0 && rank < size, "ipc comm: bad rank");
    BIBFS_REQUIRE(!name.empty() && name[0] == '/' && name.size() < 200, "ipc comm: bad group id");
    HIP_CHECK(hipGetDevice(&device_));
    attach();
    HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_tag_), 64, hipHostMallocDefault));
    *h_tag_ = 0;
    if (const char* e = std::getenv("BIBFS_IPC_STATS")) stats_on_ = e[0] == '1';
  }

  ~IpcComm() override {
    for (int r = 0; r < size_; ++r)
      for (int s = 0; s < 2; ++s)
        if (peer_[r][s].ptr) (void)hipIpcCloseMemHandle(peer_[r][s].ptr);
    if (shm_) {
      // An exported buffer is freed only after every peer unmapped it (or the
      // group failed, or a bounded wait for peers that are gone ran out).
      shm_->detached.fetch_add(1, std::memory_order_acq_rel);
      const auto deadline = clock::now() + std::chrono::seconds(2);
      while (shm_->detached.load(std::memory_order_acquire) < size_ && !aborted() && clock::now() < deadline &&
             peers_alive())
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
    for (auto& x : retired_) (void)hipFree(x.ptr);
    for (int s = 0; s < 2; ++s)
      if (stage_[s]) (void)hipFree(stage_[s]);
    if (done_) (void)hipEventDestroy(done_);
    if (h_tag_) (void)hipHostFree(h_tag_);
    if (stats_on_ && n_coll_)
      std::fprintf(stderr,
                   "[ipc rank %d] %llu collectives: %.2f us mean stream wait, %.2f us mean rendezvous, %.2f us mean "
                   "host time per collective\n",
                   rank_, (unsigned long long)n_coll_, ns_stream_ * 1e-3 / n_coll_, ns_meet_ * 1e-3 / n_coll_,
                   ns_total_ * 1e-3 / n_coll_);
    if (shm_) munmap(shm_, sizeof(IpcShm));
    if (rank_ == 0 && !unlinked_) shm_unlink(name_.c_str());
  }

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* name() const override { return "ipc"; }
  void set_timeout(double s) override {
    if (s > 0) timeout_s_ = s;
  }

  void allreduce(void* buf, size_t count, DType t, ROp op, hipStream_t s) override {
    live();
    if (size_ == 1 || count == 0) return;
    const size_t bytes = count * tsize(t);
    const int slot = enter(buf, bytes, s);
    IpcSrc src = sources(slot);
    src.p[rank_] = static_cast<const unsigned char*>(buf);
    const int o = op == ROp::kSum ? 0 : (op == ROp::kMin ? 1 : 2);
    const unsigned blocks = (unsigned)std::min<size_t>((count + 255) / 256, 64);
    switch (t) {
      case DType::kU32:
        k_ipc_reduce<uint32_t><<<blocks, 256, 0, s>>>(src, static_cast<uint32_t*>(buf), count, size_, o);
        break;
      case DType::kU64:
        k_ipc_reduce<unsigned long long><<<blocks, 256, 0, s>>>(src, static_cast<unsigned long long*>(buf), count,
                                                                size_, o);
        break;
      case DType::kF64:
        k_ipc_reduce<double><<<blocks, 256, 0, s>>>(src, static_cast<double*>(buf), count, size_, o);
        break;
    }
    HIP_CHECK(hipGetLastError());
    leave(s);
  }

  void allgather(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    live();
    if (size_ == 1) {
      if (bytes && send != recv) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    const int slot = enter(send, bytes, s);
    IpcSrc src = sources(slot);
    unsigned char* rp = static_cast<unsigned char*>(recv);
    src.p[rank_] = send == rp + (size_t)rank_ * bytes ? nullptr : static_cast<const unsigned char*>(send);
    pull(src, 0, rp, bytes, s);
    leave(s);
  }

  void alltoall(const void* send, void* recv, size_t bytes, hipStream_t s) override {
    live();
    if (size_ == 1) {
      if (bytes && send != recv) HIP_CHECK(hipMemcpyAsync(recv, send, bytes, hipMemcpyDeviceToDevice, s));
      return;
    }
    // every peer pulls block `peer` of this rank's staged P blocks
    const int slot = enter(send, bytes * (size_t)size_, s);
    IpcSrc src = sources(slot);
    src.p[rank_] = static_cast<const unsigned char*>(send);
    pull(src, (uint64_t)rank_ * bytes, static_cast<unsigned char*>(recv), bytes, s);
    leave(s);
  }

  void check() override {
    live();
    if (!peers_alive()) {
      abort_with("a peer process died");
      throw Error(abort_message());
    }
  }

  void abort() override { abort_with("aborted by rank " + std::to_string(rank_)); }
  bool aborted() const override { return aborted_ || (shm_ && shm_->aborted.load(std::memory_order_acquire) != 0); }

 private:
  struct Peer {
    void* ptr = nullptr;
    uint64_t gen = 0;
  };
  struct Retired {
    void* ptr;
    uint64_t free_after;  // arrived-count every rank must pass first
  };

  using clock = std::chrono::steady_clock;

  void attach() {
    const auto deadline = clock::now() + std::chrono::duration<double>(timeout_s_);
    int fd = -1;
    if (rank_ == 0) {
      fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw Error("ipc comm: shm_open(" + name_ + ") failed: " + std::strerror(errno));
      if (ftruncate(fd, sizeof(IpcShm)) != 0) {
        close(fd);
        shm_unlink(name_.c_str());
        throw Error(std::string("ipc comm: ftruncate failed: ") + std::strerror(errno));
      }
    } else {
      for (;;) {
        fd = shm_open(name_.c_str(), O_RDWR, 0600);
        if (fd >= 0) {
          struct stat st;
          if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(IpcShm)) break;
          close(fd);
          fd = -1;
        } else if (errno != ENOENT) {
          throw Error("ipc comm: shm_open(" + name_ + ") failed: " + std::strerror(errno));
        }
        if (clock::now() > deadline) throw Error("ipc comm: rank 0 never created group " + name_);
        std::this_thread::sleep_for(std::chrono::milliseconds(1));
      }
    }
    void* m = mmap(nullptr, sizeof(IpcShm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (m == MAP_FAILED) {
      if (rank_ == 0) shm_unlink(name_.c_str());
      throw Error(std::string("ipc comm: mmap failed: ") + std::strerror(errno));
    }
    shm_ = static_cast<IpcShm*>(m);  // (fresh segments are zero-filled)
    if (rank_ == 0) {
      shm_->P = size_;
      shm_->magic.store(kIpcMagic, std::memory_order_release);
    } else {
      while (shm_->magic.load(std::memory_order_acquire) != kIpcMagic) {
        if (clock::now() > deadline) throw Error("ipc comm: group " + name_ + " never initialised");
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
      BIBFS_REQUIRE(shm_->P == size_, "ipc comm: group " + name_ + " has " + std::to_string(shm_->P) +
                                          " ranks, this rank expected " + std::to_string(size_));
    }
    IpcRankSlot& me = shm_->r[rank_];
    me.device = device_;
    me.pid.store((int32_t)getpid(), std::memory_order_release);
    shm_->attached.fetch_add(1, std::memory_order_acq_rel);
    while (shm_->attached.load(std::memory_order_acquire) < size_) {
      if (shm_->aborted.load(std::memory_order_acquire)) throw Error(abort_message());
      if (clock::now() > deadline) {
        abort_with("not every rank attached within the timeout");
        throw Error("ipc comm: only " + std::to_string(shm_->attached.load()) + " of " + std::to_string(size_) +
                    " ranks attached to " + name_);
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    if (rank_ == 0) {  // every rank has it mapped: the name is no longer needed (no leak on a crash)
      shm_unlink(name_.c_str());
      unlinked_ = true;
    }
  }

  void live() const {
    if (aborted()) throw Error(abort_message());
  }

  std::string abort_message() const {
    const int who = shm_ ? shm_->aborted.load(std::memory_order_acquire) : 0;
    std::string why = shm_ && who ? std::string(shm_->why, strnlen(shm_->why, sizeof(shm_->why))) : "";
    return "ipc group aborted" + (who ? " (first by rank " + std::to_string(who - 1) + ": " + why + ")" : std::string());
  }

  void abort_with(const std::string& why) {
    aborted_ = true;
    if (!shm_) return;
    int expect = 0;
    if (shm_->aborted.compare_exchange_strong(expect, rank_ + 1, std::memory_order_acq_rel)) {
      std::snprintf(shm_->why, sizeof(shm_->why), "%s", why.c_str());
      std::atomic_thread_fence(std::memory_order_release);
    }
  }

  bool peers_alive() {
    const auto now = clock::now();
    if (now - last_alive_check_ < std::chrono::milliseconds(5)) return true;
    last_alive_check_ = now;
    for (int r = 0; r < size_; ++r)
      if (r != rank_ && pid_dead(shm_->r[r].pid.load(std::memory_order_acquire))) return false;
    return true;
  }

  // Host wait for the stage kernel's tag (this rank's own stream reached the
  // collective), with the group's watchdog.
  void wait_tag(uint64_t tag, hipStream_t s, const clock::time_point& deadline) {
    for (uint64_t spin = 0;; ++spin) {
      if (__atomic_load_n(h_tag_, __ATOMIC_ACQUIRE) == tag) return;
      if ((spin & 1023) == 1023) {
        live();
        const hipError_t q = hipStreamQuery(s);
        if (q != hipSuccess && q != hipErrorNotReady) HIP_CHECK(q);
        if (q == hipSuccess && __atomic_load_n(h_tag_, __ATOMIC_ACQUIRE) != tag)
          throw Error("ipc comm: stream drained without the stage tag");
        if (clock::now() > deadline) {
          abort_with("rank " + std::to_string(rank_) + " timed out waiting for its own stream");
          throw Error("ipc comm: rank " + std::to_string(rank_) + " waited " + std::to_string(timeout_s_) +
                      " s for its stream; group aborted");
        }
        if (spin > (1u << 16)) sched_yield();
      }
    }
  }

  void grow_stage(int slot, size_t bytes) {
    // The old buffer may still be mapped by peers until they see the new
    // generation (at this collective); it is freed after the next rendezvous.
    if (stage_[slot]) retired_.push_back({stage_[slot], seq_ + 1});
    // >= 2 MiB: a small hipMalloc can be a sub-allocation of a larger block,
    // whose IPC handle some runtimes (torch's bundled HIP 7.0) refuse to open
    size_t cap = 2u << 20;
    while (cap < bytes) cap <<= 1;
    HIP_CHECK(hipMalloc(&stage_[slot], cap));
    IpcRankSlot& me = shm_->r[rank_];
    HIP_CHECK(hipIpcGetMemHandle(&me.handle[slot], stage_[slot]));
    me.cap[slot] = cap;
    me.gen[slot] = ++gen_;
    stage_cap_[slot] = cap;
  }

  // Stage `bytes` of `src`, wait for them (and for the previous collective's
  // pull), rendezvous.  Returns the staging slot of this collective.
  int enter(const void* src, size_t bytes, hipStream_t s) {
    const clock::time_point t0 = clock::now();
    const int slot = (int)(seq_ & 1);
    if (bytes > stage_cap_[slot]) grow_stage(slot, bytes);
    // the previous collective's pull must be complete before this rank
    // arrives (peers then rewrite what it read): on another stream, this
    // stream waits for it, so the stage tag below implies it
    if (done_recorded_ && done_stream_ != s) HIP_CHECK(hipStreamWaitEvent(s, done_, 0));
    const uint64_t tag = ++tag_seq_;
    const unsigned char* sc = static_cast<const unsigned char*>(src);
    unsigned char* dc = static_cast<unsigned char*>(stage_[slot]);
    const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(stage_[slot])) & 15) == 0;
    if (bytes <= kStageOneBlock && aligned) {
      k_ipc_stage<<<1, 1024, 0, s>>>(reinterpret_cast<const uint4*>(sc), reinterpret_cast<uint4*>(dc), bytes / 16,
                                     sc + bytes / 16 * 16, dc + bytes / 16 * 16, (uint32_t)(bytes % 16), h_tag_, tag);
    } else {
      if (bytes) HIP_CHECK(hipMemcpyAsync(dc, sc, bytes, hipMemcpyDeviceToDevice, s));
      k_ipc_stage<<<1, 64, 0, s>>>(nullptr, nullptr, 0, nullptr, nullptr, 0, h_tag_, tag);
    }
    HIP_CHECK(hipGetLastError());
    const clock::time_point deadline =
        t0 + std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(timeout_s_));
    wait_tag(tag, s, deadline);
    const clock::time_point t1 = clock::now();
    ++seq_;
    shm_->r[rank_].arrived.store(seq_, std::memory_order_release);
    for (uint64_t spin = 0;; ++spin) {
      int behind = 0;
      for (int r = 0; r < size_; ++r)
        if (shm_->r[r].arrived.load(std::memory_order_acquire) < seq_) ++behind;
      if (!behind) break;
      if ((spin & 127) == 127) {
        live();
        if (!peers_alive()) {
          abort_with("a peer process died while rank " + std::to_string(rank_) + " waited at collective " +
                     std::to_string(seq_));
          throw Error(abort_message());
        }
        if (clock::now() > deadline) {
          abort_with("rank " + std::to_string(rank_) + " timed out at collective " + std::to_string(seq_));
          throw Error("ipc comm: rank " + std::to_string(rank_) + " waited " + std::to_string(timeout_s_) +
                      " s for its peers at collective " + std::to_string(seq_) + "; group aborted");
        }
        if (spin > 2048) sched_yield();
      }
    }
    if (stats_on_) {
      const clock::time_point t2 = clock::now();
      ++n_coll_;
      ns_stream_ += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count();
      ns_meet_ += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t1).count();
      t_enter_ = t0;
    }
    // every rank has passed the rendezvous before this one: buffers retired
    // before it are unmapped everywhere
    for (size_t i = 0; i < retired_.size();) {
      if (retired_[i].free_after < seq_) {
        HIP_CHECK(hipFree(retired_[i].ptr));
        retired_[i] = retired_.back();
        retired_.pop_back();
      } else {
        ++i;
      }
    }
    return slot;
  }

  IpcSrc sources(int slot) {
    IpcSrc src{};
    for (int r = 0; r < size_; ++r) {
      if (r == rank_) continue;
      const IpcRankSlot& ps = shm_->r[r];
      Peer& p = peer_[r][slot];
      if (p.gen != ps.gen[slot]) {
        if (p.ptr) HIP_CHECK(hipIpcCloseMemHandle(p.ptr));
        p.ptr = nullptr;
        hipIpcMemHandle_t h = ps.handle[slot];
        const hipError_t e = hipIpcOpenMemHandle(&p.ptr, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
          p.ptr = nullptr;
          throw Error(std::string("ipc comm: rank ") + std::to_string(rank_) + " cannot map rank " +
                      std::to_string(r) + "'s staging buffer (device " + std::to_string(ps.device) +
                      "): hipIpcOpenMemHandle: " + hipGetErrorString(e));
        }
        p.gen = ps.gen[slot];
      }
      src.p[r] = static_cast<const unsigned char*>(p.ptr);
    }
    return src;
  }

  void pull(const IpcSrc& src, uint64_t off, unsigned char* recv, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    const uint64_t units = (bytes + 15) / 16;
    const unsigned bx = (unsigned)std::min<uint64_t>((units + 255) / 256, 256);
    k_ipc_gather<<<dim3(bx, (unsigned)size_), 256, 0, s>>>(src, off, recv, bytes);
    HIP_CHECK(hipGetLastError());
  }

  void leave(hipStream_t s) {
    HIP_CHECK(hipEventRecord(done_, s));
    done_recorded_ = true;
    done_stream_ = s;
    if (stats_on_)
      ns_total_ += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(clock::now() - t_enter_).count();
  }

  int rank_, size_;
  std::string name_;
  double timeout_s_;
  int device_ = 0;
  IpcShm* shm_ = nullptr;
  bool unlinked_ = false;
  bool aborted_ = false;
  uint64_t seq_ = 0, gen_ = 0;
  void* stage_[2] = {nullptr, nullptr};
  size_t stage_cap_[2] = {0, 0};
  Peer peer_[kIpcMax][2];
  std::vector<Retired> retired_;
  static constexpr size_t kStageOneBlock = 256u << 10;  // one-workgroup stage kernel up to this many bytes
  hipEvent_t done_ = nullptr;
  bool done_recorded_ = false;
  hipStream_t done_stream_ = nullptr;
  uint64_t* h_tag_ = nullptr;  // pinned: the last stage tag the device wrote
  uint64_t tag_seq_ = 0;
  bool stats_on_ = false;      // BIBFS_IPC_STATS=1: per-collective host timings on teardown
  uint64_t n_coll_ = 0, ns_stream_ = 0, ns_meet_ = 0, ns_total_ = 0;
  clock::time_point t_enter_{};
  clock::time_point last_alive_check_{};
};

}  // namespace

std::vector<uint8_t> ipc_unique_id() {
  std::random_device rd;
  const uint64_t x = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
  char buf[96];
  std::snprintf(buf, sizeof(buf), "/bibfs_ipc_%d_%016llx", (int)getpid(), (unsigned long long)x);
  return std::vector<uint8_t>(buf, buf + std::strlen(buf));
}

std::unique_ptr<Comm> make_ipc_comm(int rank, int size, const std::vector<uint8_t>& uid, double timeout_s) {
  return std::unique_ptr<Comm>(new IpcComm(rank, size, std::string(uid.begin(), uid.end()), timeout_s));
}

}  // namespace dist
}  // namespace bibfs
