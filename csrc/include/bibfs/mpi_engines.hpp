// CPU distributed engines over MPI (MPICH): the v2 capability.
//  * mpi_bitmap_bibfs: C3 (v2/second_try.cpp) -- replicated uint64 frontier /
//    visited bitmaps merged with MPI_Allreduce(BOR) each half-step, but with
//    block (not cyclic) ownership of the frontier scan, each rank storing only
//    its own CSR rows, the hop count fixed (v2 printed ceil(h/2): it counted
//    rounds), the `||` termination (v2 used `&&`,
//    second_try.cpp:125) and the path recovered from recorded parents instead
//    of a separate full BFS on rank 0 (second_try.cpp:137-162).
//  * mpi_queue_bibfs: C4 (v2/main-v2.cpp) -- replicated frontier LISTS,
//    cyclic split of the frontier (main-v2.cpp:47,89), MPI_Allgather of counts
//    + MPI_Allgatherv of discovered (vertex, parent) pairs (main-v2.cpp:59-69)
//    and the min over intersections of dist_S + dist_T meet rule
//    (main-v2.cpp:73-83) -- on real .bin graphs instead of the hard-coded
//    6-node matrix (main-v2.cpp:15-26).
#pragma once

#include <mpi.h>

#include "bibfs/graph.hpp"
#include "bibfs/result.hpp"

namespace bibfs {

// `rows` = CSR rows of part.lo .. part.hi (build_csr_rows); column ids global.
SearchResult mpi_bitmap_bibfs(MPI_Comm comm, const Csr& rows, const Partition& part, vid_t src, vid_t dst,
                              const SearchOptions& opt = {});

// `g` = full CSR (replicated, as in the reference prototype).
SearchResult mpi_queue_bibfs(MPI_Comm comm, const Csr& g, vid_t src, vid_t dst, const SearchOptions& opt = {});

// rank 0 reads the .bin and broadcasts it (the reference's ingest path,
// v2/second_try.cpp:33-44); other ranks return the same edge list.
EdgeList mpi_bcast_edges(MPI_Comm comm, const std::string& path);

}  // namespace bibfs
