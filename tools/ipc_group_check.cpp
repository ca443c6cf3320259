// ipc_group_check MODE [P] [N]
//
// Host-only check of the IPC transport's control plane (csrc/dist/ipc_group.cpp)
// with P real processes (fork) -- the part of `--comm ipc` that decides
// whether a group of processes makes progress together or fails together:
//   ok     N rendezvous; every rank publishes a per-iteration value in its
//          ping-pong slot and checks every peer's after each rendezvous
//   kill   rank 1 is SIGKILLed mid-run: every other rank must fail fast
//   hang   rank 1 stops arriving: every other rank must time out
//   abort  rank 1 aborts the group: every other rank must fail with its reason
// Prints one JSON line; exit status 0 when every rank behaved as expected.
#include <signal.h>
#include <sys/wait.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../csrc/dist/ipc_group.hpp"

using bibfs::dist::IpcGroup;
using clock_t_ = std::chrono::steady_clock;

// child exit codes
enum { kOk = 0, kThrew = 10, kWrongValue = 20, kNoThrow = 30, kSetupFailed = 40 };

static int run_rank(const std::string& mode, const std::string& name, int r, int P, int N, double timeout_s,
                    int fd) {
  try {
    IpcGroup g(r, P, name, timeout_s);
    const auto t0 = clock_t_::now();
    for (int i = 1; i <= N; ++i) {
      if (r == 1 && i == 3) {
        if (mode == "kill") raise(SIGKILL);
        if (mode == "hang") std::this_thread::sleep_for(std::chrono::duration<double>(3 * timeout_s));
        if (mode == "abort") {
          g.abort("test abort from rank 1");
          return kOk;
        }
      }
      g.mine(i & 1).gen = (uint64_t)i * 100 + r;
      const auto deadline =
          clock_t_::now() + std::chrono::duration_cast<clock_t_::duration>(std::chrono::duration<double>(timeout_s));
      g.arrive_and_wait((uint64_t)i, deadline);
      for (int p = 0; p < P; ++p)
        if (g.peer(p, i & 1).gen != (uint64_t)i * 100 + p) return kWrongValue;
    }
    const double us = std::chrono::duration<double, std::micro>(clock_t_::now() - t0).count() / N;
    if (r == 0) {
      char buf[64];
      const int n = std::snprintf(buf, sizeof buf, "%.3f", us);
      if (write(fd, buf, (size_t)n) < 0) return kSetupFailed;
    }
    g.detach_wait(2.0);
    return (mode == "ok" || r == 1) ? kOk : kNoThrow;
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[rank %d] %s\n", r, e.what());
    const bool ok_msg = (mode == "kill" && std::strstr(e.what(), "died")) ||
                        (mode == "hang" && (std::strstr(e.what(), "timed out") || std::strstr(e.what(), "waited"))) ||
                        (mode == "abort" && std::strstr(e.what(), "test abort from rank 1"));
    return ok_msg ? kThrew : kSetupFailed;
  }
}

int main(int argc, char** argv) {
  if (argc < 2) {
    std::fprintf(stderr, "usage: %s ok|kill|hang|abort [P] [N]\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1];
  const int P = argc > 2 ? std::atoi(argv[2]) : 4;
  const int N = argc > 3 ? std::atoi(argv[3]) : (mode == "ok" ? 20000 : 50);
  const double timeout_s = mode == "hang" ? 1.0 : 30.0;
  const std::string name = IpcGroup::make_name();
  int pfd[2];
  if (pipe(pfd) != 0) return 2;
  const auto t0 = clock_t_::now();
  std::vector<pid_t> kids;
  for (int r = 0; r < P; ++r) {
    const pid_t pid = fork();
    if (pid == 0) {
      close(pfd[0]);
      _exit(run_rank(mode, name, r, P, N, timeout_s, pfd[1]));
    }
    kids.push_back(pid);
  }
  close(pfd[1]);
  std::vector<int> st(P, -1);
  for (int r = 0; r < P; ++r) {
    int s = 0;
    waitpid(kids[r], &s, 0);
    st[r] = WIFEXITED(s) ? WEXITSTATUS(s) : -WTERMSIG(s);
  }
  const double sec = std::chrono::duration<double>(clock_t_::now() - t0).count();
  char us[64] = {0};
  if (read(pfd[0], us, sizeof(us) - 1) < 0) us[0] = 0;
  bool ok = true;
  for (int r = 0; r < P; ++r) {
    if (mode == "ok") ok = ok && st[r] == kOk;
    else if (r == 1) ok = ok && (mode == "kill" ? st[r] == -SIGKILL : st[r] == kOk || st[r] == kThrew);
    else ok = ok && st[r] == kThrew;
  }
  std::printf("{\"mode\": \"%s\", \"ranks\": %d, \"iterations\": %d, \"ok\": %s, \"seconds\": %.3f, "
              "\"us_per_rendezvous\": %s, \"status\": [",
              mode.c_str(), P, N, ok ? "true" : "false", sec, us[0] ? us : "null");
  for (int r = 0; r < P; ++r) std::printf("%s%d", r ? ", " : "", st[r]);
  std::printf("]}\n");
  return ok ? 0 : 1;
}
