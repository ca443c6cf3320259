// pybind11 bindings: bidirectional_bfs_amd._native
//
// Exposes the native core (formats, generators, CSR, CPU engines, the HIP
// single-GPU engine and the RCCL multi-GPU engine) to Python.  Every search
// call releases the GIL.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>

#include "bibfs/cpu_engine.hpp"
#include "bibfs/dist_engine.hpp"
#include "bibfs/gen.hpp"
#include "bibfs/hip_engine.hpp"
#include "bibfs/io.hpp"

namespace py = pybind11;
using namespace bibfs;

namespace {

template <typename T>
py::array_t<T> to_numpy(const std::vector<T>& v) {
  py::array_t<T> a(v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

template <typename T>
std::vector<T> from_numpy(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
  std::vector<T> v((size_t)a.size());
  if (a.size()) std::memcpy(v.data(), a.data(), v.size() * sizeof(T));
  return v;
}

py::dict stats_dict(const SearchStats& s) {
  py::dict d;
  d["levels"] = s.levels;
  d["edges_inspected"] = s.edges_inspected;
  d["visited"] = s.visited;
  d["grid_levels"] = s.grid_levels;
  d["bottomup_levels"] = s.bottomup_levels;
  d["handoff"] = s.handoff;
  d["lds_ms"] = s.lds_ms;
  d["lds_levels"] = s.lds_levels;
  d["walk_ms"] = s.walk_ms;
  d["probe_edges"] = s.probe_edges;
  d["probe_hit"] = s.probe_hit;
  py::list tr;
  for (const auto& t : s.trace) {
    py::dict x;
    x["side"] = t.side;
    x["depth"] = t.depth;
    x["frontier"] = t.frontier;
    x["edges"] = t.edges;
    x["discovered"] = t.discovered;
    x["mode"] = t.mode;
    tr.append(x);
  }
  d["trace"] = tr;
  return d;
}

// (hops, [path]) -- the serving API's answer, built straight from the vector
py::tuple hops_path(int64_t hops, const std::vector<vid_t>& p) {
  PyObject* l = PyList_New((Py_ssize_t)p.size());
  if (!l) throw py::error_already_set();
  for (size_t i = 0; i < p.size(); ++i) PyList_SET_ITEM(l, (Py_ssize_t)i, PyLong_FromUnsignedLong(p[i]));
  return py::make_tuple(hops, py::reinterpret_steal<py::list>(l));
}

}  // namespace

static py::dict dist_stats_dict(const DistLevelStats& s) {
  py::dict d;
  d["levels"] = s.levels;
  d["rounds"] = s.rounds;
  d["lockstep_rounds"] = s.lockstep_rounds;
  d["sparse_levels"] = s.sparse_levels;
  d["dense_levels"] = s.dense_levels;
  d["overflow_levels"] = s.overflow_levels;
  d["count_syncs"] = s.count_syncs;
  d["host_syncs"] = s.host_syncs;
  d["spec_rounds"] = s.spec_rounds;
  d["plan_polls"] = s.plan_polls;
  d["host_rounds"] = s.host_rounds;
  d["collectives"] = s.collectives;
  d["path_collectives"] = s.path_collectives;
  d["solo_rounds"] = s.solo_rounds;
  d["cont_rounds"] = s.cont_rounds;
  d["pipelined"] = s.pipelined;
  d["dev_sync_rounds"] = s.dev_sync_rounds;
  d["pipe_drains"] = s.pipe_drains;
  d["pipe_retries"] = s.pipe_retries;
  d["exchanged_bytes"] = s.exchanged_bytes;
  d["comm_ms"] = s.comm_ms;
  d["device_ms"] = s.device_ms;
  d["stamped_rounds"] = s.stamped_rounds;
  d["single_engine"] = s.single_engine;
  d["expand_us"] = s.expand_us;
  d["claim_us"] = s.claim_us;
  d["exchange_us"] = s.exchange_us;
  d["status_us"] = s.status_us;
  d["walk_insert_us"] = s.walk_insert_us;
  d["walk_chain_us"] = s.walk_chain_us;
  d["small_expand_rounds"] = s.small_expand_rounds;
  d["small_claim_rounds"] = s.small_claim_rounds;
  d["sx_plan_us"] = s.sx_plan_us;
  d["sx_staging_us"] = s.sx_staging_us;
  d["sx_stage_us"] = s.sx_stage_us;
  d["sx_edges_us"] = s.sx_edges_us;
  d["sx_end_us"] = s.sx_end_us;
  d["sc_claims_us"] = s.sc_claims_us;
  d["sc_end_us"] = s.sc_end_us;
  return d;
}

PYBIND11_MODULE(_native, m) {
  m.doc() = "MI355X-native bidirectional BFS core (HIP/CDNA4 + RCCL)";

  py::register_exception<Error>(m, "BibfsError", PyExc_RuntimeError);

  // ---------------------------------------------------------------- graphs
  py::class_<EdgeList>(m, "EdgeList")
      .def(py::init<>())
      .def_readwrite("n", &EdgeList::n)
      .def_property_readonly("m", &EdgeList::m)
      .def("edges",
           [](const EdgeList& e) {
             py::array_t<uint32_t> a({(py::ssize_t)e.m(), (py::ssize_t)2});
             if (e.m()) std::memcpy(a.mutable_data(), e.uv.data(), e.uv.size() * 4);
             return a;
           })
      .def_static(
          "from_numpy",
          [](uint32_t n, py::array_t<uint32_t, py::array::c_style | py::array::forcecast> uv) {
            EdgeList e;
            e.n = n;
            e.uv = from_numpy<uint32_t>(uv);
            BIBFS_REQUIRE(e.uv.size() % 2 == 0, "edge array must have an even number of entries");
            for (uint32_t x : e.uv) BIBFS_REQUIRE(x < n, "edge endpoint >= n");
            return e;
          },
          py::arg("n"), py::arg("edges"));

  py::class_<Csr>(m, "Csr")
      .def(py::init<>())
      .def_readonly("n", &Csr::n)
      .def_readonly("m_input", &Csr::m_input)
      .def_property_readonly("nnz", &Csr::nnz)
      .def_property_readonly("row_off", [](const Csr& g) { return to_numpy(g.row_off); })
      .def_property_readonly("col", [](const Csr& g) { return to_numpy(g.col); })
      .def("degree", &Csr::degree);

  m.def(
      "build_csr",
      [](const EdgeList& el, bool dedup, bool sort_rows, int threads) {
        CsrOptions o;
        o.dedup = dedup;
        o.sort_rows = sort_rows;
        o.threads = threads;
        return build_csr(el, o);
      },
      py::arg("edges"), py::arg("dedup") = false, py::arg("sort_rows") = false, py::arg("threads") = 0,
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "build_csr_rows",
      [](const EdgeList& el, int rank, int size) {
        return build_csr_rows(el, Partition::block(el.n, rank, size));
      },
      py::arg("edges"), py::arg("rank"), py::arg("size"));
  m.def("csr_to_edges", &csr_to_edges);

  m.def("read_bin", &read_bin, py::call_guard<py::gil_scoped_release>());
  m.def("write_bin", &write_bin, py::call_guard<py::gil_scoped_release>());
  m.def("read_bin_shard", &read_bin_shard);
  m.def("read_csr_cache", &read_csr_cache);
  m.def("write_csr_cache", &write_csr_cache);
  m.def("sidecar_path", &sidecar_path);
  m.def(
      "read_dense",
      [](const std::string& p) {
        DenseMatrix d = read_dense(p);
        py::array_t<uint8_t> a({(py::ssize_t)d.n, (py::ssize_t)d.n});
        if (d.n) std::memcpy(a.mutable_data(), d.a.data(), d.a.size());
        return a;
      });
  m.def("write_dense", [](const std::string& p, py::array_t<uint8_t, py::array::c_style | py::array::forcecast> a) {
    BIBFS_REQUIRE(a.ndim() == 2 && a.shape(0) == a.shape(1), "dense matrix must be square");
    DenseMatrix d;
    d.n = (uint32_t)a.shape(0);
    d.a = from_numpy<uint8_t>(a);
    write_dense(p, d);
  });

  m.def("gen_gnp", &gen_gnp, py::arg("n"), py::arg("p"), py::arg("seed") = 1, py::arg("threads") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("gen_rmat", &gen_rmat, py::arg("n"), py::arg("m"), py::arg("seed") = 1, py::arg("a") = 0.57,
        py::arg("b") = 0.19, py::arg("c") = 0.19, py::arg("threads") = 0,
        py::call_guard<py::gil_scoped_release>());
  m.def("gen_kronecker", &gen_kronecker, py::arg("scale"), py::arg("edgefactor") = 16,
        py::arg("seed") = 1, py::arg("threads") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("reference_p", &reference_p);

  // ---------------------------------------------------------------- search API
  py::enum_<SidePolicy>(m, "SidePolicy")
      .value("SMALLER_EDGES", SidePolicy::kSmallerEdges)
      .value("SMALLER_FRONTIER", SidePolicy::kSmallerFrontier)
      .value("ALTERNATE", SidePolicy::kAlternate);
  py::enum_<Direction>(m, "Direction")
      .value("AUTO", Direction::kAuto)
      .value("TOPDOWN", Direction::kTopDown)
      .value("BOTTOMUP", Direction::kBottomUp);

  py::class_<SearchOptions>(m, "SearchOptions")
      .def(py::init<>())
      .def_readwrite("side", &SearchOptions::side)
      .def_readwrite("direction", &SearchOptions::direction)
      .def_readwrite("alpha", &SearchOptions::alpha)
      .def_readwrite("beta", &SearchOptions::beta)
      .def_readwrite("want_path", &SearchOptions::want_path)
      .def_readwrite("force_grid", &SearchOptions::force_grid)
      .def_readwrite("lockstep", &SearchOptions::lockstep)
      .def_readwrite("trace", &SearchOptions::trace);

  py::class_<SearchResult>(m, "SearchResult")
      .def_readonly("found", &SearchResult::found)
      .def_readonly("hops", &SearchResult::hops)
      .def_readonly("path", &SearchResult::path)
      .def_readonly("meet", &SearchResult::meet)
      .def_readonly("search_ms", &SearchResult::search_ms)
      .def_readonly("total_ms", &SearchResult::total_ms)
      .def_property_readonly("stats", [](const SearchResult& r) { return stats_dict(r.stats); })
      // cheap scalar views (the stats dict is rebuilt on every access)
      .def_property_readonly("levels", [](const SearchResult& r) { return r.stats.levels; })
      .def_property_readonly("edges_inspected", [](const SearchResult& r) { return r.stats.edges_inspected; })
      .def_property_readonly("visited", [](const SearchResult& r) { return r.stats.visited; })
      .def_property_readonly("handoff", [](const SearchResult& r) { return r.stats.handoff; })
      .def("__repr__", [](const SearchResult& r) {
        return "SearchResult(found=" + std::string(r.found ? "True" : "False") +
               ", hops=" + std::to_string(r.hops) + ", search_ms=" + std::to_string(r.search_ms) + ")";
      });

  py::class_<SerialBiBfs>(m, "SerialBiBfs")
      .def(py::init<const Csr&>(), py::keep_alive<1, 2>())
      .def("search", &SerialBiBfs::search, py::arg("src"), py::arg("dst"),
           py::arg("options") = SearchOptions{}, py::call_guard<py::gil_scoped_release>())
      // same lean answer as HipBiBfs.query, so the CPU / GPU serving comparison
      // pays identical Python overhead
      .def("query", [](SerialBiBfs& e, vid_t s, vid_t d) {
        SearchResult r = e.search(s, d);
        return hops_path(r.found ? r.hops : -1, r.path);
      });
  m.def("bfs_oracle", &bfs_oracle, py::call_guard<py::gil_scoped_release>());
  m.def("bfs_distances", [](const Csr& g, vid_t src) { return to_numpy(bfs_distances(g, src)); });
  m.def("validate_path", [](const Csr& g, vid_t src, vid_t dst, int64_t hops, const std::vector<vid_t>& path) {
    std::string why;
    bool ok = validate_path(g, src, dst, hops, path, &why);
    return py::make_tuple(ok, why);
  });

  // ---------------------------------------------------------------- HIP engine
  py::class_<DeviceInfo>(m, "DeviceInfo")
      .def_readonly("name", &DeviceInfo::name)
      .def_readonly("arch", &DeviceInfo::arch)
      .def_readonly("cus", &DeviceInfo::cus)
      .def_readonly("hbm_bytes", &DeviceInfo::hbm_bytes)
      .def_readonly("lds_bytes", &DeviceInfo::lds_bytes);

  py::class_<HipBiBfs>(m, "HipBiBfs")
      .def(py::init<int>(), py::arg("device") = 0)
      .def("load_csr", &HipBiBfs::load_csr, py::call_guard<py::gil_scoped_release>())
      .def("load_edges", &HipBiBfs::load_edges, py::call_guard<py::gil_scoped_release>())
      .def("generate_gnp", &HipBiBfs::generate_gnp, py::arg("n"), py::arg("p"), py::arg("seed") = 1,
           py::call_guard<py::gil_scoped_release>())
      .def("generate_rmat", &HipBiBfs::generate_rmat, py::arg("n"), py::arg("m"), py::arg("seed") = 1,
           py::arg("a") = 0.57, py::arg("b") = 0.19, py::arg("c") = 0.19,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("n", &HipBiBfs::n)
      .def_property_readonly("nnz", &HipBiBfs::nnz)
      .def_property_readonly("m_input", &HipBiBfs::m_input)
      .def_property_readonly("last_build_ms", &HipBiBfs::last_build_ms)
      .def_property_readonly("device_bytes", &HipBiBfs::device_bytes)
      .def_property_readonly("device", &HipBiBfs::device)
      .def("search", &HipBiBfs::search, py::arg("src"), py::arg("dst"), py::arg("options") = SearchOptions{},
           py::call_guard<py::gil_scoped_release>())
      // serving entry point: (hops, path); the GIL is kept (a query is ~10 us)
      .def("query", [](HipBiBfs& e, vid_t s, vid_t d) {
        static thread_local std::vector<vid_t> p;  // reused: no allocation per query
        p.clear();
        const int64_t h = e.query(s, d, &p);
        return hops_path(h, p);
      })
      .def_property_readonly("last_search_ms", &HipBiBfs::last_search_ms)
      .def_property_readonly("last_edges_inspected", &HipBiBfs::last_edges_inspected)
      .def_property_readonly("tiny_engine", &HipBiBfs::tiny_engine)
      .def_property_readonly("tiny_overflows", &HipBiBfs::tiny_overflows)
      .def("set_host_stamps", &HipBiBfs::set_host_stamps)
      .def("host_stamps", [](const HipBiBfs& e) {
        const auto v = e.host_stamps();
        py::dict d;
        d["queries"] = (uint64_t)v[0];
        d["post_us"] = v[1];
        d["wait_first_packet_us"] = v[2];
        d["read_packets_us"] = v[3];
        d["return_us"] = v[4];
        return d;
      })
      .def("release", &HipBiBfs::release, py::call_guard<py::gil_scoped_release>())
      .def("search_batch", &HipBiBfs::search_batch, py::arg("src"), py::arg("dst"),
           py::arg("options") = SearchOptions{}, py::call_guard<py::gil_scoped_release>())
      .def(
          "search_batch_arrays",
          [](HipBiBfs& e, py::array_t<uint32_t, py::array::c_style | py::array::forcecast> src,
             py::array_t<uint32_t, py::array::c_style | py::array::forcecast> dst, const SearchOptions& opt) {
            std::vector<vid_t> s(src.data(), src.data() + src.size()), d(dst.data(), dst.data() + dst.size());
            std::vector<SearchResult> rs;
            {
              py::gil_scoped_release rel;
              rs = e.search_batch(s, d, opt);
            }
            // compact result: hops (-1 = no path), CSR-style paths (offsets + flat vertex list)
            py::array_t<int64_t> hops(rs.size());
            py::array_t<int64_t> off(rs.size() + 1);
            size_t total = 0;
            for (auto& r : rs) total += r.path.size();
            py::array_t<uint32_t> flat(total);
            auto h = hops.mutable_unchecked<1>();
            auto o = off.mutable_unchecked<1>();
            uint32_t* f = flat.mutable_data();
            size_t pos = 0;
            for (size_t i = 0; i < rs.size(); ++i) {
              h(i) = rs[i].hops;
              o(i) = (int64_t)pos;
              std::memcpy(f + pos, rs[i].path.data(), rs[i].path.size() * 4);
              pos += rs[i].path.size();
            }
            o(rs.size()) = (int64_t)pos;
            return py::make_tuple(hops, off, flat);
          },
          py::arg("src"), py::arg("dst"), py::arg("options") = SearchOptions{})
      .def("set_resident", &HipBiBfs::set_resident, py::arg("on"), py::arg("idle_ms") = 200.0,
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("resident", &HipBiBfs::resident)
      .def_property("auto_handoff", &HipBiBfs::auto_handoff, &HipBiBfs::set_auto_handoff)
      .def_property("auto_gate_timeout_us", &HipBiBfs::auto_gate_timeout_us, &HipBiBfs::set_auto_gate_timeout_us)
      .def_property_readonly("auto_gate_misses", &HipBiBfs::auto_gate_misses)
      .def_property("auto_levels", &HipBiBfs::auto_levels, &HipBiBfs::set_auto_levels)
      .def_property("auto_max_degree", &HipBiBfs::auto_max_degree, &HipBiBfs::set_auto_max_degree)
      .def_property("lds_probe_edges", &HipBiBfs::lds_probe_edges, &HipBiBfs::set_lds_probe_edges)
      .def("set_build_flags", &HipBiBfs::set_build_flags, py::arg("wide_offsets") = false,
           py::arg("stream_gen") = false, py::arg("tiny") = true)
      .def_property("batch_edge_cap", &HipBiBfs::batch_edge_cap, &HipBiBfs::set_batch_edge_cap)
      .def_property_readonly("last_batch_fallbacks", &HipBiBfs::last_batch_fallbacks)
      .def("set_batch_tuning", &HipBiBfs::set_batch_tuning, py::arg("lds_first") = -1, py::arg("threads") = 0)
      .def("begin", &HipBiBfs::begin, py::call_guard<py::gil_scoped_release>())
      .def(
          "expand",
          [](HipBiBfs& e, int side, Direction dir) {
            bool met = false;
            uint64_t c;
            {
              py::gil_scoped_release rel;
              c = e.expand(side, &met, dir);
            }
            return py::make_tuple(c, met);
          },
          py::arg("side"), py::arg("direction") = Direction::kTopDown)
      .def("check_meet", &HipBiBfs::check_meet, py::call_guard<py::gil_scoped_release>())
      .def("finish", &HipBiBfs::finish, py::call_guard<py::gil_scoped_release>())
      .def("download_csr", &HipBiBfs::download_csr)
      .def("neighbors", &HipBiBfs::neighbors)
      .def("download_edges", &HipBiBfs::download_edges)
      .def("info", &HipBiBfs::info)
      .def("synchronize", &HipBiBfs::synchronize, py::call_guard<py::gil_scoped_release>());

  // ---------------------------------------------------------------- multi-GPU engine
  m.def("gpu_count", &gpu_count);
  m.def("rccl_unique_id", []() {
    auto id = dist_unique_id();
    return py::bytes(reinterpret_cast<const char*>(id.data()), id.size());
  });
  m.def(
      "dist_unique_id",
      [](const std::string& backend) {
        auto id = dist_unique_id(backend);
        return py::bytes(reinterpret_cast<const char*>(id.data()), id.size());
      },
      py::arg("backend") = "rccl");
  py::class_<DistTuning>(m, "DistTuning")
      .def(py::init<>())
      .def_readwrite("spec_rounds", &DistTuning::spec_rounds)
      .def_readwrite("spec_cap_max", &DistTuning::spec_cap_max)
      .def_readwrite("cap", &DistTuning::cap)
      .def_readwrite("nosync_bytes", &DistTuning::nosync_bytes)
      .def_readwrite("timeout_s", &DistTuning::timeout_s)
      .def_readwrite("walk_max", &DistTuning::walk_max)
      .def_readwrite("solo", &DistTuning::solo)
      .def_readwrite("solo_edges", &DistTuning::solo_edges)
      .def_readwrite("owner_cap", &DistTuning::owner_cap)
      .def_readwrite("pipeline", &DistTuning::pipeline)
      .def_readwrite("dev_sync", &DistTuning::dev_sync)
      .def_readwrite("spec_stall_edges", &DistTuning::spec_stall_edges)
      .def_readwrite("stamps", &DistTuning::stamps)
      .def_readwrite("spill_cap", &DistTuning::spill_cap)
      .def_readwrite("hbm_cap_bytes", &DistTuning::hbm_cap_bytes)
      .def_readwrite("world1_single", &DistTuning::world1_single);
  py::class_<DistLocalFault>(m, "DistLocalFault")
      .def(py::init<>())
      .def_readwrite("rank", &DistLocalFault::rank)
      .def_readwrite("at", &DistLocalFault::at)
      .def_readwrite("mode", &DistLocalFault::mode);
  py::class_<DistBiBfs>(m, "DistBiBfs")
      .def(py::init([](int rank, int size, int device, py::bytes uid, const std::string& backend) {
             std::string s = uid;
             std::vector<uint8_t> id(s.begin(), s.end());
             py::gil_scoped_release rel;
             return new DistBiBfs(rank, size, device, id, backend);
           }),
           py::arg("rank"), py::arg("size"), py::arg("device"), py::arg("unique_id"), py::arg("backend") = "rccl")
      .def_property_readonly("rank", &DistBiBfs::rank)
      .def_property_readonly("size", &DistBiBfs::size)
      .def_property_readonly("n", &DistBiBfs::n)
      .def_property_readonly("m_input", &DistBiBfs::m_input)
      .def_property_readonly("local_nnz", &DistBiBfs::local_nnz)
      .def_property_readonly("shard_bytes", &DistBiBfs::shard_bytes)
      .def_property_readonly("gen_peak_bytes", &DistBiBfs::gen_peak_bytes)
      .def_property_readonly("gen_hbm_peak_bytes", &DistBiBfs::gen_hbm_peak_bytes)
      .def_property_readonly("resident_bytes", &DistBiBfs::resident_bytes)
      .def("validate_path", &DistBiBfs::validate_path, py::arg("src"), py::arg("dst"), py::arg("hops"),
           py::arg("path"), py::call_guard<py::gil_scoped_release>())
      .def("search_unidirectional", &DistBiBfs::search_unidirectional, py::arg("src"), py::arg("dst"),
           py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("lo", &DistBiBfs::lo)
      .def_property_readonly("hi", &DistBiBfs::hi)
      .def("load_edges", &DistBiBfs::load_edges, py::call_guard<py::gil_scoped_release>())
      .def("load_bin", &DistBiBfs::load_bin, py::call_guard<py::gil_scoped_release>())
      .def("generate_gnp", &DistBiBfs::generate_gnp, py::arg("n"), py::arg("p"), py::arg("seed") = 1,
           py::call_guard<py::gil_scoped_release>())
      .def("generate_rmat", &DistBiBfs::generate_rmat, py::arg("n"), py::arg("m"), py::arg("seed") = 1,
           py::arg("a") = 0.57, py::arg("b") = 0.19, py::arg("c") = 0.19,
           py::call_guard<py::gil_scoped_release>())
      .def("search", &DistBiBfs::search, py::arg("src"), py::arg("dst"), py::arg("options") = SearchOptions{},
           py::call_guard<py::gil_scoped_release>())
      // lean serving call, the twin of HipBiBfs.query: (hops, path), hops -1 when unreachable
      .def("query",
           [](DistBiBfs& e, vid_t s, vid_t d) {
             static thread_local std::vector<vid_t> p;  // reused: no allocation per query
             p.clear();
             int64_t h;
             if (e.query_is_local()) {  // world size 1: the single engine's query, GIL kept (~10 us)
               h = e.query(s, d, &p);
             } else {  // a collective: other ranks' Python threads may need the GIL meanwhile
               py::gil_scoped_release rel;
               h = e.query(s, d, &p);
             }
             return hops_path(h, p);
           })
      .def("barrier", &DistBiBfs::barrier, py::call_guard<py::gil_scoped_release>())
      .def("allreduce_max", &DistBiBfs::allreduce_max, py::call_guard<py::gil_scoped_release>())
      .def("release", &DistBiBfs::release, py::call_guard<py::gil_scoped_release>())
      .def("set_tuning", &DistBiBfs::set_tuning, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("tuning", &DistBiBfs::tuning)
      .def("inject_fault", &DistBiBfs::inject_fault, py::arg("at"), py::arg("mode"))
      .def_property_readonly("backend", &DistBiBfs::backend)
      .def_property_readonly("last_stats", [](const DistBiBfs& e) { return dist_stats_dict(e.last_stats()); });
  m.def(
      "dist_local_run",
      [](int ranks, int device, const EdgeList& el, const std::vector<std::pair<vid_t, vid_t>>& queries,
         const SearchOptions& opt, const DistTuning& tuning, const DistLocalFault& fault) {
        std::vector<DistLevelStats> st;
        std::vector<SearchResult> rs;
        {
          py::gil_scoped_release nogil;
          rs = dist_local_run(ranks, device, el, queries, opt, tuning, fault, &st);
        }
        py::list stl;
        for (const auto& x : st) stl.append(dist_stats_dict(x));
        return py::make_tuple(rs, stl);
      },
      py::arg("ranks"), py::arg("device"), py::arg("edges"), py::arg("queries"),
      py::arg("options") = SearchOptions{}, py::arg("tuning") = DistTuning{}, py::arg("fault") = DistLocalFault{});
  m.def(
      "dist_local_generate_run",
      [](int ranks, int device, const std::string& kind, uint32_t n, double arg, uint64_t seed,
         const std::vector<std::pair<vid_t, vid_t>>& queries, const SearchOptions& opt, const DistTuning& tuning,
         int verify) {
        DistLocalTiming t;
        std::vector<SearchResult> rs;
        {
          py::gil_scoped_release nogil;
          rs = dist_local_generate_run(ranks, device, kind, n, arg, seed, queries, opt, &t, tuning, verify);
        }
        py::dict d;
        d["build_ms"] = t.build_ms;
        d["query_ms"] = t.query_ms;
        d["local_nnz"] = t.local_nnz;
        d["shard_bytes"] = t.shard_bytes;
        d["gen_peak_bytes"] = t.gen_peak_bytes;
        d["gen_hbm_peak_bytes"] = t.gen_hbm_peak_bytes;
        d["resident_bytes"] = t.resident_bytes;
        d["path_valid"] = t.path_valid;
        d["uni_hops"] = t.uni_hops;
        py::list st;
        for (const auto& x : t.stats) st.append(dist_stats_dict(x));
        d["stats"] = st;
        return py::make_tuple(rs, d);
      },
      py::arg("ranks"), py::arg("device"), py::arg("kind"), py::arg("n"), py::arg("arg"), py::arg("seed"),
      py::arg("queries"), py::arg("options") = SearchOptions{}, py::arg("tuning") = DistTuning{},
      py::arg("verify") = 0);
}
