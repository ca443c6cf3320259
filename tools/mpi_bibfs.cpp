// mpirun -n <p> mpi_bibfs <graph.bin | gnp:N[:p[:seed]] | rmat:N:M[:seed] | kron:S[:EF[:seed]]> <src> <dst>
//                         [--repeat R] [--warmup W] [--json] [--verify] [--direction auto|topdown|bottomup]
//                         [--comm auto|rccl|ipc] [--timeout S] [--fault RANK:ROUND:MODE]
//
// v4 capability (reference v4/mpi_bas.cpp + v4/comp.cu): multi-GPU
// bidirectional BFS, one MPI rank per GPU.  MPI is used only to bootstrap the
// RCCL communicator (rank 0's unique id is MPI_Bcast) and for the final
// timing reduction; every per-level exchange is RCCL over xGMI.  Each rank
// reads only its shard of the .bin (or generates the graph on its GPU and
// keeps its rows); the reference broadcast the whole edge list and every rank
// expanded the whole frontier (v4/comp.cu:99).
//
// --comm ipc runs the ranks as separate processes over the HIP-IPC transport
// (csrc/dist/ipc_comm.hip), so several ranks may share one GPU -- the
// reference's own single-machine launch, `mpirun -n 4` with every rank on the
// one GPU (single_machine_bench.sh:9,52; v4/Makefile:64 uses -np 6).  The
// default `auto` picks RCCL when every rank on a node has a GPU of its own and
// IPC otherwise.  --fault arms DistBiBfs::inject_fault on one rank (1 throw,
// 2 stall past the timeout, 3 kill the process) to check that the other ranks
// fail instead of hanging.
#include <mpi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "bibfs/dist_engine.hpp"
#include "bibfs/hip_engine.hpp"
#include "cli_common.hpp"

// rank and rank count among the processes of this node
static void node_rank(int* local_rank, int* local_size) {
  MPI_Comm node;
  MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, 0, MPI_INFO_NULL, &node);
  MPI_Comm_rank(node, local_rank);
  MPI_Comm_size(node, local_size);
  MPI_Comm_free(&node);
}

// GPUs of this node without touching the HIP runtime: KFD topology nodes
// with SIMDs (narrowed by ROCR_ / HIP_VISIBLE_DEVICES); 0 when unreadable.
static int host_gpu_count() {
  int n = 0;
  for (int i = 0; i < 256; ++i) {
    const std::string path = "/sys/class/kfd/kfd/topology/nodes/" + std::to_string(i) + "/properties";
    std::FILE* f = std::fopen(path.c_str(), "r");
    if (!f) break;
    char key[64];
    unsigned long long v = 0;
    while (std::fscanf(f, "%63s %llu", key, &v) == 2)
      if (std::strcmp(key, "simd_count") == 0 && v > 0) ++n;
    std::fclose(f);
  }
  for (const char* var : {"ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"})
    if (const char* e = std::getenv(var); e && *e) {
      int listed = 1;
      for (const char* c = e; *c; ++c) listed += *c == ',';
      n = std::min(n, listed);
    }
  return n;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  auto a = cli::parse(argc, argv,
                      {"repeat", "warmup", "side", "direction", "alpha", "beta", "device", "comm", "timeout", "fault"});
  if (a.pos.size() != 3) {
    if (rank == 0) std::fprintf(stderr, "Usage: mpirun -n <p> %s <graph.bin> <src> <dst>\n", argv[0]);
    MPI_Finalize();
    return 1;
  }
  int rc = 0;
  try {
    int local_rank = 0, local_size = 1, max_local = 1, min_local = 1;
    node_rank(&local_rank, &local_size);
    MPI_Allreduce(&local_size, &max_local, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
    MPI_Allreduce(&local_size, &min_local, 1, MPI_INT, MPI_MIN, MPI_COMM_WORLD);
    // The IPC control plane is node-local shared memory and checks peer
    // liveness by local pid, so it needs every rank on one node.
    const bool one_node = min_local == size;
    // Ranks sharing a GPU as processes (IPC): one hardware queue each, set
    // before this process's first HIP call -- with HIP's 4 per process the GPU
    // time-slices the ranks' queues (8 ranks on one GPU: ~140 -> ~2 ms per
    // G(1M) query, profiles/r6_hw_queues_procs.jsonl).
    {
      const std::string want = a.has("comm") ? a.get("comm") : "auto";
      const int hdev = host_gpu_count();
      if (want != "rccl" && one_node && hdev > 0 && max_local > hdev) setenv("GPU_MAX_HW_QUEUES", "1", 1);
    }
    const int ndev = bibfs::gpu_count();
    std::string comm = a.has("comm") ? a.get("comm") : "auto";
    if (comm == "auto") comm = (max_local > ndev && one_node) ? "ipc" : "rccl";
    if (comm != "rccl" && comm != "ipc") throw bibfs::Error("--comm must be auto, rccl or ipc");
    if (comm == "ipc" && !one_node) {
      if (rank == 0)
        std::fprintf(stderr,
                     "--comm ipc needs all %d ranks on one node (this job spans several nodes: %d to %d ranks per "
                     "node); use --comm rccl with at most one rank per GPU\n",
                     size, min_local, max_local);
      MPI_Finalize();
      return 1;
    }
    // RCCL: one rank per GPU (a rank owns a GPU's HBM and its RCCL endpoint).
    // IPC: ranks share the node's GPUs round-robin.  Every rank checks its
    // device and the verdict is agreed on before any rank touches a
    // communicator, so a bad launch fails with one clear message on every rank.
    const int device = a.has("device") ? (int)a.geti("device", 0)
                                       : (comm == "ipc" && ndev > 0 ? local_rank % ndev : local_rank);
    int bad = (device < 0 || device >= ndev) ? 1 : 0, any_bad = 0;
    MPI_Allreduce(&bad, &any_bad, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
    if (any_bad) {
      if (bad && comm == "rccl")
        std::fprintf(stderr,
                     "[rank %d] --comm rccl runs one rank per GPU: this rank maps to device %d but only %d GPU(s) "
                     "are visible (ranks on this node > GPUs); launch at most %d ranks per node, pass --device, "
                     "or use --comm ipc\n",
                     rank, device, ndev, ndev);
      else if (bad)
        std::fprintf(stderr, "[rank %d] no usable GPU for this rank (device %d, %d visible)\n", rank, device, ndev);
      MPI_Finalize();
      return 1;
    }
    std::vector<uint8_t> uid(128);
    if (rank == 0) uid = bibfs::dist_unique_id(comm);
    int len = (int)uid.size();
    MPI_Bcast(&len, 1, MPI_INT, 0, MPI_COMM_WORLD);
    uid.resize((size_t)len);
    MPI_Bcast(uid.data(), len, MPI_BYTE, 0, MPI_COMM_WORLD);
    bibfs::DistBiBfs eng(rank, size, device, uid, comm);
    if (a.has("timeout")) {
      bibfs::DistTuning t = eng.tuning();
      t.timeout_s = a.getd("timeout", 120.0);
      eng.set_tuning(t);
    }
    if (a.has("fault")) {
      auto f = cli::split(a.get("fault"), ':');
      BIBFS_REQUIRE(f.size() == 3, "--fault RANK:ROUND:MODE");
      if (std::atoi(f[0].c_str()) == rank) eng.inject_fault(std::atoi(f[1].c_str()), std::atoi(f[2].c_str()));
    }
    const std::string graph = a.pos[0];
    double tl = MPI_Wtime();
    if (cli::is_spec(graph)) {
      auto f = cli::split(graph, ':');
      if (f[0] == "gnp") {
        uint32_t n = (uint32_t)std::atoll(f.at(1).c_str());
        double p = f.size() > 2 && !f[2].empty() ? std::atof(f[2].c_str()) : bibfs::reference_p(n);
        eng.generate_gnp(n, p, f.size() > 3 ? std::strtoull(f[3].c_str(), nullptr, 10) : 1);
      } else if (f[0] == "rmat") {
        eng.generate_rmat((uint32_t)std::atoll(f.at(1).c_str()), std::strtoull(f.at(2).c_str(), nullptr, 10),
                          f.size() > 3 ? std::strtoull(f[3].c_str(), nullptr, 10) : 1);
      } else {
        int scale = std::atoi(f.at(1).c_str());
        int ef = f.size() > 2 ? std::atoi(f[2].c_str()) : 16;
        eng.generate_rmat(1u << scale, (uint64_t)ef << scale, f.size() > 3 ? std::strtoull(f[3].c_str(), nullptr, 10) : 1);
      }
    } else {
      eng.load_bin(graph);
    }
    eng.barrier();
    tl = MPI_Wtime() - tl;
    const bibfs::vid_t src = (bibfs::vid_t)std::atoll(a.pos[1].c_str());
    const bibfs::vid_t dst = (bibfs::vid_t)std::atoll(a.pos[2].c_str());
    if (src >= eng.n() || dst >= eng.n()) throw bibfs::Error("src/dst must be < N");
    auto opt = cli::options_from(a);
    const int warmup = (int)a.geti("warmup", 2), repeat = (int)std::max(1LL, a.geti("repeat", 5));
    for (int i = 0; i < warmup; ++i) eng.search(src, dst, opt);
    std::vector<double> ts;
    bibfs::SearchResult r;
    for (int i = 0; i < repeat; ++i) {
      eng.barrier();
      r = eng.search(src, dst, opt);
      ts.push_back(eng.allreduce_max(r.total_ms));
    }
    if (rank == 0) {
      const double med = cli::median(ts);
      if (a.has("json")) {
        cli::print_json(r, "hip-dist", graph, eng.n(), eng.m_input(), src, dst, tl * 1e3, 0, med, med, repeat, size);
      } else {
        if (r.found) std::printf("Shortest path length = %lld\n", (long long)r.hops);
        else std::printf("No path found\n");
        std::printf("[Time] MPI+HIP BI-BFS = %.9g s\n", med * 1e-3);
        std::printf("Ranks: %d over %s (%d GPU(s) visible per node)\n", size, eng.backend(), ndev);
        cli::print_path(r);
      }
    }
    if (a.has("verify") && rank == 0) {
      bibfs::EdgeList el = cli::edges_from_spec(graph);
      auto g = bibfs::build_csr(el);
      auto o = bibfs::bfs_oracle(g, src, dst);
      std::string why;
      bool ok = o.hops == r.hops && (!r.found || bibfs::validate_path(g, src, dst, r.hops, r.path, &why));
      std::printf("Verify: %s (oracle hops = %lld)%s%s\n", ok ? "OK" : "MISMATCH", (long long)o.hops,
                  why.empty() ? "" : " ", why.c_str());
      if (!ok) rc = 2;
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[rank %d] %s\n", rank, e.what());
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  MPI_Finalize();
  return rc;
}
