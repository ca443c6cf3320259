// show_matrix [graph.bin]
//
// C6 capability (reference v2/read_in.cpp): dump a legacy dense adjacency
// matrix file (u32 N followed by N*N u8), validating the size against the
// header exactly like the reference (read_in.cpp:14-22).  The default file
// name is graph.bin, as in the reference.
#include <cstdio>

#include "bibfs/io.hpp"

int main(int argc, char** argv) {
  const std::string path = argc > 1 ? argv[1] : "graph.bin";
  try {
    bibfs::DenseMatrix d = bibfs::read_dense(path);
    std::string line;
    for (uint32_t i = 0; i < d.n; ++i) {
      line.clear();
      for (uint32_t j = 0; j < d.n; ++j) {
        line += std::to_string((int)d.a[(size_t)i * d.n + j]);
        line += (j + 1 == d.n) ? '\n' : ' ';
      }
      std::fputs(line.c_str(), stdout);
    }
  } catch (const std::exception& e) {
    std::fprintf(stderr, "%s\n", e.what());
    return 1;
  }
  return 0;
}
