// Graph file I/O: .bin edge lists, .json path sidecars, legacy dense matrices
// and the .csr cache.  See include/bibfs/io.hpp for the format list.
#include "bibfs/io.hpp"

#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cctype>
#include <cstring>
#include <fstream>
#include <sstream>

namespace bibfs {

namespace {

struct MappedFile {
  int fd = -1;
  size_t size = 0;
  const uint8_t* data = nullptr;
  explicit MappedFile(const std::string& path) {
    fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) throw Error("Cannot open " + path);
    struct stat st;
    if (fstat(fd, &st) != 0) {
      ::close(fd);
      throw Error("Cannot stat " + path);
    }
    size = (size_t)st.st_size;
    if (size > 0) {
      void* p = mmap(nullptr, size, PROT_READ, MAP_PRIVATE, fd, 0);
      if (p == MAP_FAILED) {
        ::close(fd);
        throw Error("Cannot mmap " + path);
      }
      madvise(p, size, MADV_SEQUENTIAL);
      data = static_cast<const uint8_t*>(p);
    }
  }
  ~MappedFile() {
    if (data) munmap(const_cast<uint8_t*>(data), size);
    if (fd >= 0) ::close(fd);
  }
  MappedFile(const MappedFile&) = delete;
  MappedFile& operator=(const MappedFile&) = delete;
};

uint32_t load_u32(const uint8_t* p) {
  uint32_t x;
  std::memcpy(&x, p, 4);
  return x;  // little-endian host assumed (x86-64 / the MI355X host)
}

}  // namespace

BinHeader read_bin_header(const std::string& path) {
  std::ifstream in(path, std::ios::binary);
  if (!in) throw Error("Cannot open " + path);
  BinHeader h;
  in.read(reinterpret_cast<char*>(&h.n), 4);
  in.read(reinterpret_cast<char*>(&h.m), 4);
  if (!in) throw Error("Unexpected EOF reading header of " + path);
  return h;
}

EdgeList read_bin(const std::string& path) {
  MappedFile f(path);
  if (f.size < 8) throw Error("Unexpected EOF reading header of " + path);
  EdgeList el;
  el.n = load_u32(f.data);
  const uint32_t m = load_u32(f.data + 4);
  const uint64_t need = 8ULL + 8ULL * m;
  if (f.size < need) {
    throw Error("Unexpected EOF reading edges of " + path + ": header says M = " +
                std::to_string(m) + " (" + std::to_string(need) + " bytes) but file has " +
                std::to_string(f.size) + " bytes");
  }
  el.uv.resize(2ULL * m);
  std::memcpy(el.uv.data(), f.data + 8, 8ULL * m);
  uint32_t bad = 0;
  for (uint64_t i = 0; i < 2ULL * m; ++i) bad |= (el.uv[i] >= el.n);
  if (bad) {
    for (uint64_t i = 0; i < 2ULL * m; ++i)
      if (el.uv[i] >= el.n)
        throw Error("Edge " + std::to_string(i / 2) + " of " + path + " has endpoint " +
                    std::to_string(el.uv[i]) + " >= N = " + std::to_string(el.n));
  }
  return el;
}

EdgeList read_bin_shard(const std::string& path, uint32_t lo, uint32_t hi) {
  MappedFile f(path);
  if (f.size < 8) throw Error("Unexpected EOF reading header of " + path);
  EdgeList el;
  el.n = load_u32(f.data);
  const uint32_t m = load_u32(f.data + 4);
  if (f.size < 8ULL + 8ULL * m) throw Error("Unexpected EOF reading edges of " + path);
  const uint32_t* e = reinterpret_cast<const uint32_t*>(f.data + 8);
  for (uint64_t i = 0; i < m; ++i) {
    uint32_t u = e[2 * i], v = e[2 * i + 1];
    if (u >= el.n || v >= el.n) throw Error("Edge endpoint out of range in " + path);
    if ((u >= lo && u < hi) || (v >= lo && v < hi)) {
      el.uv.push_back(u);
      el.uv.push_back(v);
    }
  }
  return el;
}

void write_bin(const std::string& path, const EdgeList& el) {
  std::ofstream out(path, std::ios::binary);
  if (!out) throw Error("Cannot open " + path + " for writing");
  BIBFS_REQUIRE(el.m() <= 0xFFFFFFFFULL, ".bin header caps M < 2^32");
  uint32_t n = el.n, m = (uint32_t)el.m();
  out.write(reinterpret_cast<const char*>(&n), 4);
  out.write(reinterpret_cast<const char*>(&m), 4);
  out.write(reinterpret_cast<const char*>(el.uv.data()), (std::streamsize)(el.uv.size() * 4));
  if (!out) throw Error("Write failed for " + path);
}

// ---------------------------------------------------------------- JSON sidecar

void write_path_json(const std::string& path, const PathJson& pj) {
  std::ofstream out(path);
  if (!out) throw Error("Cannot open " + path + " for writing");
  // Same key order and indent=2 layout as json.dump(..., indent=2) in
  // graphs/generate_graph.py:61-62.
  out << "{\n  \"source\": " << pj.source << ",\n  \"target\": " << pj.target
      << ",\n  \"hop_count\": ";
  if (pj.hop_count)
    out << *pj.hop_count;
  else
    out << "null";
  out << ",\n  \"nodes\": [";
  if (pj.nodes.empty()) {
    out << "]\n}";
  } else {
    for (size_t i = 0; i < pj.nodes.size(); ++i) out << (i ? ",\n    " : "\n    ") << pj.nodes[i];
    out << "\n  ]\n}";
  }
}

namespace {
struct JsonCursor {
  const std::string& s;
  size_t i = 0;
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  bool eat(char c) {
    ws();
    if (i < s.size() && s[i] == c) {
      ++i;
      return true;
    }
    return false;
  }
  std::string key() {
    ws();
    if (!eat('"')) throw Error("json: expected key");
    size_t b = i;
    while (i < s.size() && s[i] != '"') ++i;
    std::string k = s.substr(b, i - b);
    ++i;
    return k;
  }
  bool null_lit() {
    ws();
    if (s.compare(i, 4, "null") == 0) {
      i += 4;
      return true;
    }
    return false;
  }
  int64_t integer() {
    ws();
    size_t b = i;
    if (i < s.size() && (s[i] == '-' || s[i] == '+')) ++i;
    while (i < s.size() && std::isdigit((unsigned char)s[i])) ++i;
    if (b == i) throw Error("json: expected integer");
    return std::stoll(s.substr(b, i - b));
  }
  void skip_value() {
    ws();
    int depth = 0;
    bool instr = false;
    for (; i < s.size(); ++i) {
      char c = s[i];
      if (instr) {
        if (c == '\\') ++i;
        else if (c == '"') instr = false;
        continue;
      }
      if (c == '"') instr = true;
      else if (c == '[' || c == '{') ++depth;
      else if (c == ']' || c == '}') {
        if (depth == 0) return;
        --depth;
      } else if (c == ',' && depth == 0)
        return;
    }
  }
};
}  // namespace

PathJson read_path_json(const std::string& path) {
  std::ifstream in(path);
  if (!in) throw Error("Cannot open " + path);
  std::stringstream ss;
  ss << in.rdbuf();
  std::string s = ss.str();
  JsonCursor c{s};
  PathJson pj;
  if (!c.eat('{')) throw Error("json: expected object in " + path);
  if (c.eat('}')) return pj;
  do {
    std::string k = c.key();
    if (!c.eat(':')) throw Error("json: expected ':'");
    if (k == "source") pj.source = c.integer();
    else if (k == "target") pj.target = c.integer();
    else if (k == "hop_count") {
      if (c.null_lit()) pj.hop_count.reset();
      else pj.hop_count = c.integer();
    } else if (k == "nodes") {
      if (!c.eat('[')) throw Error("json: expected '['");
      if (!c.eat(']')) {
        do pj.nodes.push_back(c.integer());
        while (c.eat(','));
        if (!c.eat(']')) throw Error("json: expected ']'");
      }
    } else {
      c.skip_value();
    }
  } while (c.eat(','));
  return pj;
}

std::string sidecar_path(const std::string& bin_path) {
  size_t slash = bin_path.find_last_of('/');
  size_t dot = bin_path.find_last_of('.');
  if (dot == std::string::npos || (slash != std::string::npos && dot < slash))
    return bin_path + ".json";
  return bin_path.substr(0, dot) + ".json";
}

// ---------------------------------------------------------------- dense legacy

DenseMatrix read_dense(const std::string& path) {
  MappedFile f(path);
  if (f.size < 4) throw Error("Unexpected EOF reading header of " + path);
  DenseMatrix d;
  d.n = load_u32(f.data);
  const uint64_t expected = 4ULL + (uint64_t)d.n * d.n;
  if (f.size != expected)
    throw Error("Size mismatch: header says N = " + std::to_string(d.n) + " => expected " +
                std::to_string(expected) + " bytes, but file is " + std::to_string(f.size) +
                " bytes.");
  d.a.assign(f.data + 4, f.data + expected);
  return d;
}

void write_dense(const std::string& path, const DenseMatrix& m) {
  std::ofstream out(path, std::ios::binary);
  if (!out) throw Error("Cannot open " + path + " for writing");
  out.write(reinterpret_cast<const char*>(&m.n), 4);
  out.write(reinterpret_cast<const char*>(m.a.data()), (std::streamsize)m.a.size());
}

// ---------------------------------------------------------------- CSR cache

static const char kCsrMagic[8] = {'B', 'B', 'F', 'S', 'C', 'S', 'R', '1'};

void write_csr_cache(const std::string& path, const Csr& g) {
  std::ofstream out(path, std::ios::binary);
  if (!out) throw Error("Cannot open " + path + " for writing");
  uint64_t nnz = g.nnz();
  out.write(kCsrMagic, 8);
  out.write(reinterpret_cast<const char*>(&g.n), 4);
  out.write(reinterpret_cast<const char*>(&g.m_input), 8);
  out.write(reinterpret_cast<const char*>(&nnz), 8);
  out.write(reinterpret_cast<const char*>(g.row_off.data()), (std::streamsize)(8ULL * (g.n + 1ULL)));
  out.write(reinterpret_cast<const char*>(g.col.data()), (std::streamsize)(4ULL * nnz));
  if (!out) throw Error("Write failed for " + path);
}

Csr read_csr_cache(const std::string& path) {
  MappedFile f(path);
  if (f.size < 28 || std::memcmp(f.data, kCsrMagic, 8) != 0) throw Error("Not a .csr cache: " + path);
  Csr g;
  uint64_t nnz;
  std::memcpy(&g.n, f.data + 8, 4);
  std::memcpy(&g.m_input, f.data + 12, 8);
  std::memcpy(&nnz, f.data + 20, 8);
  const uint64_t need = 28 + 8ULL * (g.n + 1ULL) + 4ULL * nnz;
  if (f.size < need) throw Error("Truncated .csr cache: " + path);
  g.row_off.resize(g.n + 1ULL);
  g.col.resize(nnz);
  std::memcpy(g.row_off.data(), f.data + 28, 8ULL * (g.n + 1ULL));
  std::memcpy(g.col.data(), f.data + 28 + 8ULL * (g.n + 1ULL), 4ULL * nnz);
  BIBFS_REQUIRE(g.row_off[g.n] == nnz, "corrupt .csr cache (row_off[n] != nnz)");
  return g;
}

}  // namespace bibfs
