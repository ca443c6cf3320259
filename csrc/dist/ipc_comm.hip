// Multi-process collectives over HIP IPC (comm.hpp: make_ipc_comm).
//
// P ranks are P processes.  They may share one GPU -- the reference's own v4
// launch shape, 4 MPI ranks on one machine's GPU (single_machine_bench.sh:9,52;
// v4/Makefile:64 uses 6) -- or sit on different GPUs of a node, where the very
// same loads read peer HBM over xGMI (UNVERIFIED: only the one-GPU shape has
// run; test_mpi_bibfs_ipc_transport_across_gpus needs a multi-GPU box).
// RCCL refuses two ranks on one device
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
// Control plane (IpcGroup, ipc_group.cpp -- host-only, CPU-tested): a POSIX
// shared-memory segment (name = the group's unique id) with one cache line per rank.  A collective is: stage (one kernel that
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

#include <sched.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "device.hpp"
#include "ipc_group.hpp"

namespace bibfs {
namespace dist {

namespace {

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

class IpcComm final : public Comm {
 public:
  IpcComm(int rank, int size, const std::string& name, double timeout_s)
      : rank_(rank), size_(size), group_(rank, size, name, timeout_s, current_device()) {
    static_assert(sizeof(hipIpcMemHandle_t) == sizeof(IpcGroup::Blob::handle), "IPC handle size");
    HIP_CHECK(hipEventCreateWithFlags(&done_, hipEventDisableTiming));
    HIP_CHECK(hipHostMalloc(reinterpret_cast<void**>(&h_tag_), 64, hipHostMallocDefault));
    *h_tag_ = 0;
    if (const char* e = std::getenv("BIBFS_IPC_STATS")) stats_on_ = e[0] == '1';
  }

  ~IpcComm() override {
    // A pull kernel of the last collective may still read the peers' mapped
    // buffers (after an abort ~DistBiBfs skips its stream sync): wait for it
    // before unmapping.  Pull kernels never wait on peers, so this is bounded.
    if (done_) (void)hipEventSynchronize(done_);
    for (int r = 0; r < size_; ++r) {
      for (int s = 0; s < 2; ++s)
        if (peer_[r][s].ptr) (void)hipIpcCloseMemHandle(peer_[r][s].ptr);
      if (win_peer_[r]) (void)hipIpcCloseMemHandle(win_peer_[r]);
    }
    // an exported buffer is freed only after every peer unmapped it (or the
    // group failed, or a bounded wait for peers that are gone ran out)
    group_.detach_wait(2.0);
    for (auto& x : retired_) (void)hipFree(x.ptr);
    for (int s = 0; s < 2; ++s)
      if (stage_[s]) (void)hipFree(stage_[s]);
    if (win_) (void)hipFree(win_);
    if (done_) (void)hipEventDestroy(done_);
    if (h_tag_) (void)hipHostFree(h_tag_);
    if (stats_on_ && n_coll_)
      std::fprintf(stderr,
                   "[ipc rank %d] %llu collectives: %.2f us mean stream wait, %.2f us mean rendezvous, %.2f us mean "
                   "host time per collective\n",
                   rank_, (unsigned long long)n_coll_, ns_stream_ * 1e-3 / n_coll_, ns_meet_ * 1e-3 / n_coll_,
                   ns_total_ * 1e-3 / n_coll_);
  }

  int rank() const override { return rank_; }
  int size() const override { return size_; }
  const char* name() const override { return "ipc"; }
  void set_timeout(double s) override { group_.set_timeout(s); }

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

  // In place: the stage and the rendezvous as alltoall, then the caller's
  // kernels read every peer's block straight out of its mapped staging slot
  // (this rank's own block out of `send`) -- no pull kernel, no copy into
  // recv.  alltoall_release records `done` behind those readers, which is
  // what the next collective's stage (same stream) and the peers' rewrite of
  // this slot two collectives later are ordered after.
  void alltoall_view(const void* send, void* recv, size_t bytes, hipStream_t s, const void** peers) override {
    live();
    if (size_ == 1) {
      peers[0] = send;
      return;
    }
    const int slot = enter(send, bytes * (size_t)size_, s);
    const IpcSrc src = sources(slot);
    for (int r = 0; r < size_; ++r)
      peers[r] = (r == rank_ ? static_cast<const unsigned char*>(send) : src.p[r]) + (size_t)rank_ * bytes;
    in_view_ = true;
  }
  void alltoall_release(hipStream_t s) override {
    if (!in_view_) return;
    in_view_ = false;
    leave(s);
  }

  // Every rank exports a window; the handles (with each rank's PCI bus id)
  // move in one allgather, and the peers' windows are mapped.  Only when every
  // rank sits on the caller's GPU: the device-side flag protocol is measured
  // there (cross-GPU windows over xGMI stay off).
  bool dev_window(size_t bytes, Window& w) override {
    live();
    if (size_ > kWinMax) return false;
    if (win_) {  // (one window per communicator: sized once, by the first caller)
      if (bytes > win_bytes_) return false;
      w.mine = win_;
      for (int r = 0; r < size_; ++r) w.peer[r] = r == rank_ ? win_ : win_peer_[r];
      return true;
    }
    struct Blob {
      int32_t ok;
      char pci[28];
      unsigned char handle[64];
    };
    static_assert(sizeof(hipIpcMemHandle_t) <= 64, "IPC handle size");
    Blob me{};
    int dev = 0;
    HIP_CHECK(hipGetDevice(&dev));
    if (hipDeviceGetPCIBusId(me.pci, (int)sizeof me.pci, dev) != hipSuccess) {
      (void)hipGetLastError();
      me.pci[0] = 0;
    }
    size_t cap = 2u << 20;  // (>= 2 MiB: an exportable block, as grow_stage)
    while (cap < bytes) cap <<= 1;
    void* mine = nullptr;
    hipIpcMemHandle_t h;
    if (hipMalloc(&mine, cap) == hipSuccess && hipIpcGetMemHandle(&h, mine) == hipSuccess) {
      HIP_CHECK(hipMemset(mine, 0, cap));
      std::memcpy(me.handle, &h, sizeof h);
      me.ok = me.pci[0] ? 1 : 0;
    } else {
      (void)hipGetLastError();
      if (mine) (void)hipFree(mine);
      mine = nullptr;
    }
    void* d = nullptr;
    HIP_CHECK(hipMalloc(&d, sizeof(Blob) * (size_t)(size_ + 1)));
    std::vector<Blob> all((size_t)size_);
    hipStream_t s = nullptr;
    HIP_CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    HIP_CHECK(hipMemcpy(d, &me, sizeof me, hipMemcpyHostToDevice));
    allgather(d, static_cast<Blob*>(d) + 1, sizeof(Blob), s);
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipMemcpy(all.data(), static_cast<Blob*>(d) + 1, sizeof(Blob) * (size_t)size_, hipMemcpyDeviceToHost));
    HIP_CHECK(hipStreamDestroy(s));
    HIP_CHECK(hipFree(d));
    bool ok = true;
    for (int r = 0; r < size_; ++r)
      ok = ok && all[(size_t)r].ok && std::strncmp(all[(size_t)r].pci, me.pci, sizeof me.pci) == 0;
    if (!ok) {  // every rank sees the same blobs: every rank declines
      if (mine) (void)hipFree(mine);
      return false;
    }
    win_ = mine;
    win_bytes_ = cap;
    for (int r = 0; r < size_; ++r) {
      if (r == rank_) continue;
      std::memcpy(&h, all[(size_t)r].handle, sizeof h);
      HIP_CHECK(hipIpcOpenMemHandle(&win_peer_[r], h, hipIpcMemLazyEnablePeerAccess));
    }
    w.mine = win_;
    for (int r = 0; r < size_; ++r) w.peer[r] = r == rank_ ? win_ : win_peer_[r];
    return true;
  }

  void check() override { group_.check(); }
  void abort() override { group_.abort("aborted by rank " + std::to_string(rank_)); }
  bool aborted() const override { return group_.aborted(); }

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

  static int current_device() {
    int d = 0;
    HIP_CHECK(hipGetDevice(&d));
    return d;
  }

  void live() const {
    if (group_.aborted()) throw Error(group_.abort_message());
  }

  clock::time_point deadline_from(clock::time_point t0) const {
    return t0 + std::chrono::duration_cast<clock::duration>(std::chrono::duration<double>(group_.timeout()));
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
          group_.abort("rank " + std::to_string(rank_) + " timed out waiting for its own stream");
          throw Error("ipc comm: rank " + std::to_string(rank_) + " waited " + std::to_string(group_.timeout()) +
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
    // A block the runtime will not export (seen with 8 ranks on one device:
    // hipIpcGetMemHandle "invalid argument" on a fresh 2 MiB hipMalloc) is
    // held while a larger one is tried -- so the allocator cannot hand the
    // same block back -- and freed once one exports.
    std::vector<void*> refused;
    hipIpcMemHandle_t h;
    for (int attempt = 0;; ++attempt) {
      HIP_CHECK(hipMalloc(&stage_[slot], cap));
      const hipError_t e = hipIpcGetMemHandle(&h, stage_[slot]);
      if (e == hipSuccess) break;
      (void)hipGetLastError();
      refused.push_back(stage_[slot]);
      stage_[slot] = nullptr;
      if (attempt == 5) {
        for (void* p : refused) (void)hipFree(p);
        throw Error(std::string("ipc comm: rank ") + std::to_string(rank_) +
                    " cannot export a staging buffer: hipIpcGetMemHandle: " + hipGetErrorString(e));
      }
      cap <<= 1;
    }
    for (void* p : refused) HIP_CHECK(hipFree(p));
    IpcGroup::Blob& me = group_.mine(slot);
    std::memcpy(me.handle, &h, sizeof(h));
    me.cap = cap;
    me.gen = ++gen_;
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
    const clock::time_point deadline = deadline_from(t0);
    wait_tag(tag, s, deadline);
    const clock::time_point t1 = clock::now();
    ++seq_;
    group_.arrive_and_wait(seq_, deadline);
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
      const IpcGroup::Blob& pb = group_.peer(r, slot);
      Peer& p = peer_[r][slot];
      if (p.gen != pb.gen) {
        if (p.ptr) HIP_CHECK(hipIpcCloseMemHandle(p.ptr));
        p.ptr = nullptr;
        hipIpcMemHandle_t h;
        std::memcpy(&h, pb.handle, sizeof(h));
        const hipError_t e = hipIpcOpenMemHandle(&p.ptr, h, hipIpcMemLazyEnablePeerAccess);
        if (e != hipSuccess) {
          p.ptr = nullptr;
          throw Error(std::string("ipc comm: rank ") + std::to_string(rank_) + " cannot map rank " +
                      std::to_string(r) + "'s staging buffer (device " + std::to_string(group_.peer_device(r)) +
                      "): hipIpcOpenMemHandle: " + hipGetErrorString(e));
        }
        p.gen = pb.gen;
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

  static constexpr size_t kStageOneBlock = 256u << 10;  // one-workgroup stage kernel up to this many bytes
  int rank_, size_;
  IpcGroup group_;
  uint64_t seq_ = 0, gen_ = 0;
  void* stage_[2] = {nullptr, nullptr};
  size_t stage_cap_[2] = {0, 0};
  Peer peer_[kIpcMax][2];
  std::vector<Retired> retired_;
  hipEvent_t done_ = nullptr;
  bool done_recorded_ = false;
  hipStream_t done_stream_ = nullptr;
  uint64_t* h_tag_ = nullptr;  // pinned: the last stage tag the device wrote
  uint64_t tag_seq_ = 0;
  bool stats_on_ = false;      // BIBFS_IPC_STATS=1: per-collective host timings on teardown
  bool in_view_ = false;       // alltoall_view -> alltoall_release
  void* win_ = nullptr;        // dev_window: this rank's exported window and the peers' mapped ones
  size_t win_bytes_ = 0;
  void* win_peer_[kIpcMax] = {};
  uint64_t n_coll_ = 0, ns_stream_ = 0, ns_meet_ = 0, ns_total_ = 0;
  clock::time_point t_enter_{};
};

}  // namespace

std::vector<uint8_t> ipc_unique_id() {
  const std::string n = IpcGroup::make_name();
  return std::vector<uint8_t>(n.begin(), n.end());
}

std::unique_ptr<Comm> make_ipc_comm(int rank, int size, const std::vector<uint8_t>& uid, double timeout_s) {
  return std::unique_ptr<Comm>(new IpcComm(rank, size, std::string(uid.begin(), uid.end()), timeout_s));
}

}  // namespace dist
}  // namespace bibfs
