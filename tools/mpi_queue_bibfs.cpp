// mpirun -n <p> mpi_queue_bibfs <graph.bin> <src> <dst> [--repeat R] [--json] [--verify] [--alternate]
//
// C4 capability (reference v2/main-v2.cpp): MPI frontier-list bidirectional BFS
// (Allgatherv of discovered vertices, candidate-min meet rule) on real graphs.
// Rank 0 reads and broadcasts the edge list like the reference (:33-44); each
// rank keeps only its own CSR rows.  Prints the reference lines with the
// CORRECT hop count (the reference printed the number of rounds).
#include "bibfs/mpi_engines.hpp"
#include "cli_common.hpp"

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank, size;
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  auto a = cli::parse(argc, argv, {"repeat", "side"});
  if (a.pos.size() != 3) {
    if (rank == 0) std::fprintf(stderr, "Usage: mpirun -n <p> %s <graph.bin> <src> <dst>\n", argv[0]);
    MPI_Finalize();
    return 1;
  }
  int rc = 0;
  try {
    const bibfs::vid_t src = (bibfs::vid_t)std::atoll(a.pos[1].c_str());
    const bibfs::vid_t dst = (bibfs::vid_t)std::atoll(a.pos[2].c_str());
    double tl = MPI_Wtime();
    bibfs::EdgeList el = cli::is_spec(a.pos[0]) ? cli::edges_from_spec(a.pos[0])
                                                : bibfs::mpi_bcast_edges(MPI_COMM_WORLD, a.pos[0]);
    auto part = bibfs::Partition::block(el.n, rank, size);
    bibfs::Csr full = bibfs::build_csr(el);
    (void)part;
    tl = MPI_Wtime() - tl;
    if (src >= el.n || dst >= el.n) throw bibfs::Error("src/dst must be < N");
    bibfs::SearchOptions opt = cli::options_from(a);
    if (a.has("alternate")) opt.side = bibfs::SidePolicy::kAlternate;
    const int repeat = (int)std::max(1LL, a.geti("repeat", 1));
    std::vector<double> ts;
    bibfs::SearchResult r;
    for (int i = 0; i < repeat; ++i) {
      MPI_Barrier(MPI_COMM_WORLD);
      r = bibfs::mpi_queue_bibfs(MPI_COMM_WORLD, full, src, dst, opt);
      double t = r.search_ms;
      MPI_Allreduce(MPI_IN_PLACE, &t, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD);
      ts.push_back(t);
    }
    if (rank == 0) {
      const double med = cli::median(ts);
      if (a.has("json")) {
        cli::print_json(r, "mpi-queue", a.pos[0], el.n, el.m(), src, dst, tl * 1e3, 0, med, med, repeat, 0);
      } else {
        if (r.found) std::printf("Shortest path length = %lld\n", (long long)r.hops);
        else std::printf("No path found\n");
        std::printf("[Time] bidir-queue BFS = %.9g seconds\n", med * 1e-3);
        cli::print_path(r);
      }
      if (a.has("verify")) {
        auto g = bibfs::build_csr(el);
        auto o = bibfs::bfs_oracle(g, src, dst);
        std::string why;
        bool ok = o.hops == r.hops && (!r.found || bibfs::validate_path(g, src, dst, r.hops, r.path, &why));
        std::printf("Verify: %s (oracle hops = %lld)%s%s\n", ok ? "OK" : "MISMATCH", (long long)o.hops,
                    why.empty() ? "" : " ", why.c_str());
        if (!ok) rc = 2;
      }
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "[rank %d] %s\n", rank, e.what());
    MPI_Abort(MPI_COMM_WORLD, 1);
  }
  MPI_Finalize();
  return rc;
}
