// IpcGroup: the shared-memory control plane of the IPC transport (see
// ipc_group.hpp and ipc_comm.hip).
#include "ipc_group.hpp"

#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>

#include "bibfs/common.hpp"

namespace bibfs {
namespace dist {

namespace {

constexpr uint64_t kIpcMagic = 0x4942465349504331ull;  // "1CPISFBI"
using clock = std::chrono::steady_clock;

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

}  // namespace

struct alignas(64) IpcRankSlot {
  std::atomic<uint64_t> arrived;  // collectives this rank has entered
  std::atomic<int32_t> pid;
  int32_t device;
  IpcGroup::Blob blob[2];         // per staging slot
};

struct IpcGroup::Shm {
  std::atomic<uint64_t> magic;
  int32_t P;
  std::atomic<int32_t> attached;
  std::atomic<int32_t> aborted;   // 0, or 1 + the rank that aborted first
  std::atomic<int32_t> detached;  // ranks through the teardown rendezvous
  std::atomic<int32_t> why_ready; // `why` is written (after the abort CAS)
  char why[240];
  IpcRankSlot r[kIpcMax];
};

std::string IpcGroup::make_name() {
  std::random_device rd;
  const uint64_t x = ((uint64_t)rd() << 32) ^ rd() ^ (uint64_t)clock::now().time_since_epoch().count();
  char buf[96];
  std::snprintf(buf, sizeof(buf), "/bibfs_ipc_%d_%016llx", (int)getpid(), (unsigned long long)x);
  return buf;
}

IpcGroup::IpcGroup(int rank, int size, const std::string& name, double timeout_s, int device)
    : rank_(rank), size_(size), name_(name), timeout_s_(timeout_s) {
  BIBFS_REQUIRE(size >= 1 && size <= kIpcMax, "ipc group: 1.." + std::to_string(kIpcMax) + " ranks");
  BIBFS_REQUIRE(rank >= 0 && rank < size, "ipc group: bad rank");
  BIBFS_REQUIRE(!name.empty() && name[0] == '/' && name.size() < 200, "ipc group: bad group id");
  BIBFS_REQUIRE(timeout_s > 0, "ipc group: timeout must be positive");
  attach(device);
}

IpcGroup::~IpcGroup() {
  if (shm_) munmap(shm_, sizeof(Shm));
  if (rank_ == 0 && !unlinked_) shm_unlink(name_.c_str());
}

void IpcGroup::attach(int device) {
  const auto deadline = clock::now() + std::chrono::duration_cast<clock::duration>(
                                           std::chrono::duration<double>(timeout_s_));
  int fd = -1;
  if (rank_ == 0) {
    fd = shm_open(name_.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) throw Error("ipc group: shm_open(" + name_ + ") failed: " + std::strerror(errno));
    if (ftruncate(fd, sizeof(Shm)) != 0) {
      const int e = errno;
      close(fd);
      shm_unlink(name_.c_str());
      throw Error(std::string("ipc group: ftruncate failed: ") + std::strerror(e));
    }
  } else {
    for (;;) {
      fd = shm_open(name_.c_str(), O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && (size_t)st.st_size >= sizeof(Shm)) break;
        close(fd);
        fd = -1;
      } else if (errno != ENOENT) {
        throw Error("ipc group: shm_open(" + name_ + ") failed: " + std::strerror(errno));
      }
      if (clock::now() > deadline) throw Error("ipc group: rank 0 never created group " + name_);
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  void* m = mmap(nullptr, sizeof(Shm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  const int e = errno;
  close(fd);
  if (m == MAP_FAILED) {
    if (rank_ == 0) shm_unlink(name_.c_str());
    throw Error(std::string("ipc group: mmap failed: ") + std::strerror(e));
  }
  shm_ = static_cast<Shm*>(m);  // (a fresh segment is zero-filled)
  if (rank_ == 0) {
    shm_->P = size_;
    shm_->magic.store(kIpcMagic, std::memory_order_release);
  } else {
    while (shm_->magic.load(std::memory_order_acquire) != kIpcMagic) {
      if (clock::now() > deadline) throw Error("ipc group: group " + name_ + " never initialised");
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
    BIBFS_REQUIRE(shm_->P == size_, "ipc group: group " + name_ + " has " + std::to_string(shm_->P) +
                                        " ranks, this rank expected " + std::to_string(size_));
  }
  IpcRankSlot& me = shm_->r[rank_];
  me.device = device;
  me.pid.store((int32_t)getpid(), std::memory_order_release);
  shm_->attached.fetch_add(1, std::memory_order_acq_rel);
  while (shm_->attached.load(std::memory_order_acquire) < size_) {
    if (shm_->aborted.load(std::memory_order_acquire)) throw Error(abort_message());
    if (clock::now() > deadline) {
      abort("not every rank attached within the timeout");
      throw Error("ipc group: only " + std::to_string(shm_->attached.load()) + " of " + std::to_string(size_) +
                  " ranks attached to " + name_);
    }
    std::this_thread::sleep_for(std::chrono::microseconds(100));
  }
  if (rank_ == 0) {  // every rank has it mapped: the name is no longer needed
    shm_unlink(name_.c_str());
    unlinked_ = true;
  }
}

IpcGroup::Blob& IpcGroup::mine(int slot) { return shm_->r[rank_].blob[slot]; }
const IpcGroup::Blob& IpcGroup::peer(int r, int slot) const { return shm_->r[r].blob[slot]; }
int IpcGroup::peer_device(int r) const { return shm_->r[r].device; }
uint64_t IpcGroup::arrived(int r) const { return shm_->r[r].arrived.load(std::memory_order_acquire); }

bool IpcGroup::aborted() const { return aborted_ || (shm_ && shm_->aborted.load(std::memory_order_acquire) != 0); }

std::string IpcGroup::abort_message() const {
  const int who = shm_ ? shm_->aborted.load(std::memory_order_acquire) : 0;
  if (who) {  // the first aborter writes its reason right after its CAS
    const auto until = clock::now() + std::chrono::milliseconds(2);
    while (!shm_->why_ready.load(std::memory_order_acquire) && clock::now() < until) std::this_thread::yield();
  }
  const std::string why = shm_ && who ? std::string(shm_->why, strnlen(shm_->why, sizeof(shm_->why))) : "";
  return "ipc group aborted" + (who ? " (first by rank " + std::to_string(who - 1) + ": " + why + ")" : std::string());
}

void IpcGroup::abort(const std::string& why) {
  aborted_ = true;
  if (!shm_) return;
  int expect = 0;
  if (shm_->aborted.compare_exchange_strong(expect, rank_ + 1, std::memory_order_acq_rel)) {
    std::snprintf(shm_->why, sizeof(shm_->why), "%s", why.c_str());
    shm_->why_ready.store(1, std::memory_order_release);
  }
}

bool IpcGroup::peers_alive() {
  const auto now = clock::now();
  if (now - last_alive_check_ < std::chrono::milliseconds(5)) return true;
  last_alive_check_ = now;
  for (int r = 0; r < size_; ++r)
    if (r != rank_ && pid_dead(shm_->r[r].pid.load(std::memory_order_acquire))) return false;
  return true;
}

void IpcGroup::check() {
  if (aborted()) throw Error(abort_message());
  if (!peers_alive()) {
    abort("a peer process died");
    throw Error(abort_message());
  }
}

void IpcGroup::arrive_and_wait(uint64_t seq, clock::time_point deadline) {
  if (aborted()) throw Error(abort_message());
  shm_->r[rank_].arrived.store(seq, std::memory_order_release);
  for (uint64_t spin = 0;; ++spin) {
    int behind = 0;
    for (int r = 0; r < size_; ++r)
      if (shm_->r[r].arrived.load(std::memory_order_acquire) < seq) ++behind;
    if (!behind) return;
    if ((spin & 127) == 127) {
      if (aborted()) throw Error(abort_message());
      if (!peers_alive()) {
        abort("a peer process died while rank " + std::to_string(rank_) + " waited at collective " +
              std::to_string(seq));
        throw Error(abort_message());
      }
      if (clock::now() > deadline) {
        abort("rank " + std::to_string(rank_) + " timed out at collective " + std::to_string(seq));
        throw Error("ipc group: rank " + std::to_string(rank_) + " waited " + std::to_string(timeout_s_) +
                    " s for its peers at collective " + std::to_string(seq) + "; group aborted");
      }
      if (spin > 2048) sched_yield();
    }
  }
}

void IpcGroup::detach_wait(double max_s) {
  if (!shm_) return;
  shm_->detached.fetch_add(1, std::memory_order_acq_rel);
  const auto deadline = clock::now() + std::chrono::duration_cast<clock::duration>(
                                           std::chrono::duration<double>(max_s));
  while (shm_->detached.load(std::memory_order_acquire) < size_ && !aborted() && clock::now() < deadline &&
         peers_alive())
    std::this_thread::sleep_for(std::chrono::microseconds(200));
}

}  // namespace dist
}  // namespace bibfs
