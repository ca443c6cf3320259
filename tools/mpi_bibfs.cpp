// mpirun -n <p> mpi_bibfs <graph.bin | gnp:N[:p[:seed]] | rmat:N:M[:seed] | kron:S[:EF[:seed]]> <src> <dst>
//                         [--repeat R] [--warmup W] [--json] [--verify] [--direction auto|topdown|bottomup]
//
// v4 capability (reference v4/mpi_bas.cpp + v4/comp.cu): multi-GPU
// bidirectional BFS, one MPI rank per GPU.  MPI is used only to bootstrap the
// RCCL communicator (rank 0's unique id is MPI_Bcast) and for the final
// timing reduction; every per-level exchange is RCCL over xGMI.  Each rank
// reads only its shard of the .bin (or generates the graph on its GPU and
// keeps its rows); the reference broadcast the whole edge list and every rank
// expanded the whole frontier (v4/comp.cu:99).
#include <mpi.h>

#include "bibfs/dist_engine.hpp"
#include "bibfs/hip_engine.hpp"
#include "cli_common.hpp"

static int local_rank_from_env(int rank) {
  for (const char* k : {"MPI_LOCALRANKID", "OMPI_COMM_WORLD_LOCAL_RANK", "LOCAL_RANK", "SLURM_LOCALID"}) {
    const char* v = std::getenv(k);
    if (v) return std::atoi(v);
  }
  return rank;
}

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  auto a = cli::parse(argc, argv, {"repeat", "warmup", "side", "direction", "alpha", "beta", "device"});
  if (a.pos.size() != 3) {
    if (rank == 0) std::fprintf(stderr, "Usage: mpirun -n <p> %s <graph.bin> <src> <dst>\n", argv[0]);
    MPI_Finalize();
    return 1;
  }
  int rc = 0;
  try {
    const int device = a.has("device") ? (int)a.geti("device", 0) : local_rank_from_env(rank);
    // One rank per GPU (the reference ran 4-6 ranks on 1-2 GPUs, v4/Makefile:64,
    // README.md:16; here a rank owns a GPU's HBM and its RCCL endpoint).  Every
    // rank checks its device and the verdict is agreed on before any rank
    // touches RCCL, so a bad launch fails with one clear message, not a raw
    // HIP error on some ranks and a hang on the others.
    const int ndev = bibfs::gpu_count();
    int bad = (device < 0 || device >= ndev) ? 1 : 0, any_bad = 0;
    MPI_Allreduce(&bad, &any_bad, 1, MPI_INT, MPI_MAX, MPI_COMM_WORLD);
    if (any_bad) {
      if (bad)
        std::fprintf(stderr,
                     "[rank %d] mpi_bibfs runs one rank per GPU: this rank maps to device %d but only %d GPU(s) "
                     "are visible (ranks on this node > GPUs); launch with at most %d ranks per node or pass "
                     "--device\n",
                     rank, device, ndev, ndev);
      MPI_Finalize();
      return 1;
    }
    std::vector<uint8_t> uid(128);
    if (rank == 0) uid = bibfs::dist_unique_id();
    int len = (int)uid.size();
    MPI_Bcast(&len, 1, MPI_INT, 0, MPI_COMM_WORLD);
    uid.resize((size_t)len);
    MPI_Bcast(uid.data(), len, MPI_BYTE, 0, MPI_COMM_WORLD);
    bibfs::DistBiBfs eng(rank, size, device, uid);
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
