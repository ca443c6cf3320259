// Control plane of the multi-process IPC transport (ipc_comm.hip): a POSIX
// shared-memory segment through which P processes rendezvous once per
// collective, publish their exported staging buffers, and fail together.
// Host-only (no HIP), so the rendezvous, abort, timeout and dead-peer paths
// are tested on the CPU with real processes (tools/ipc_group_check.cpp).
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <string>

namespace bibfs {
namespace dist {

constexpr int kIpcMax = 16;  // ranks per group

class IpcGroup {
 public:
  // What a rank publishes per staging slot: the exported buffer's IPC handle,
  // its capacity and a generation that changes whenever the buffer does.
  struct Blob {
    uint64_t gen;
    uint64_t cap;
    unsigned char handle[64];
  };

  // Rank 0 creates the segment `name` (a "/..." POSIX shm name, e.g. from
  // make_name()), the others open it; returns once every rank has attached
  // (or throws after timeout_s).  Rank 0 then unlinks the name, so a crash
  // leaks nothing.
  IpcGroup(int rank, int size, const std::string& name, double timeout_s, int device = 0);
  ~IpcGroup();
  IpcGroup(const IpcGroup&) = delete;
  IpcGroup& operator=(const IpcGroup&) = delete;

  static std::string make_name();

  int rank() const { return rank_; }
  int size() const { return size_; }
  void set_timeout(double s) {
    if (s > 0) timeout_s_ = s;
  }
  double timeout() const { return timeout_s_; }

  Blob& mine(int slot);
  const Blob& peer(int r, int slot) const;
  int peer_device(int r) const;

  // Arrive at collective number `seq` (1, 2, ...: every rank the same
  // sequence) and wait until every rank has.  Throws -- after aborting the
  // group -- when the group was aborted, a peer process died, or the wait
  // passed `deadline`.
  void arrive_and_wait(uint64_t seq, std::chrono::steady_clock::time_point deadline);
  uint64_t arrived(int r) const;

  // Abort the group: every rank waiting (or arriving later) throws.  The
  // first reason is kept.  Idempotent.
  void abort(const std::string& why);
  bool aborted() const;
  std::string abort_message() const;
  // Throws if the group was aborted, or (checked at most every 5 ms) a peer
  // process died -- then the group is aborted first.
  void check();
  bool peers_alive();

  // Teardown rendezvous: count this rank out and wait (at most max_s, less
  // if the group failed or a peer is gone) for every rank to do the same --
  // so a rank frees what it exported only after its peers unmapped it.
  void detach_wait(double max_s);

 private:
  struct Shm;
  void attach(int device);
  int rank_, size_;
  std::string name_;
  double timeout_s_;
  Shm* shm_ = nullptr;
  bool unlinked_ = false;
  bool aborted_ = false;
  std::chrono::steady_clock::time_point last_alive_check_{};
};

}  // namespace dist
}  // namespace bibfs
