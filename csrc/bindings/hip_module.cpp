// Python bindings of the gfx950 SART kernels (module mpi_cuda_sartsolver_amd._lib._sart_hip).
//
// The interface is deliberately ABI-neutral: device pointers and HIP streams are passed as integers
// (torch.Tensor.data_ptr(), torch.cuda.Stream.cuda_stream), so this module links only against the
// HIP runtime and works with any PyTorch-ROCm build. Launch functions never allocate, copy or
// synchronise, so callers may capture them into HIP graphs.
#include <hip/hip_runtime.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>

#include "../engine/comm.hpp"
#include "../engine/engine.hpp"
#include "../engine/geometry.hpp"
#include "../engine/multiframe.hpp"
#include "../kernels/launchers.hpp"

namespace py = pybind11;


template <typename T>
static T* P(uintptr_t p) {
    return reinterpret_cast<T*>(p);
}
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

using f64arr = py::array_t<double, py::array::c_style | py::array::forcecast>;

static py::dict solve_info(const sart::SolveInfo& i) {
    py::dict d;
    d["status"] = i.status;
    d["iterations"] = i.iterations;
    d["convergence"] = i.convergence;
    d["used_fused"] = i.used_fused;
    d["fused_variant"] = i.fused_variant;
    d["fallbacks"] = i.fallbacks;
    d["comm_fallbacks"] = i.comm_fallbacks;
    d["comm"] = std::string(i.comm ? i.comm : "");
    d["nonfinite"] = i.nonfinite;
    d["ms"] = i.ms;
    d["sweeps"] = i.sweeps;
    d["comm_ms"] = i.comm_ms;
    d["warm_from"] = i.warm_from;
    d["warm_iter"] = i.warm_iter;
    d["warm_live"] = i.warm_live;
    return d;
}

static void bind_engine(py::module_& m) {
    py::enum_<sart::ReduceOp>(m, "ReduceOp", py::module_local()).value("SUM", sart::ReduceOp::kSum).value("MAX", sart::ReduceOp::kMax);
    py::class_<sart::Communicator, std::shared_ptr<sart::Communicator>>(m, "Comm")
        .def_property_readonly("rank", [](sart::Communicator& c) { return c.rank(); })
        .def_property_readonly("size", [](sart::Communicator& c) { return c.size(); })
        .def_property_readonly("backend", &sart::Communicator::backend)
        .def_property_readonly("describe", &sart::Communicator::describe)
        .def_property_readonly("setup_seconds", &sart::Communicator::setup_seconds)
        .def("prepare", &sart::Communicator::prepare, py::arg("float_sizes"), py::call_guard<py::gil_scoped_release>())
        .def("check", &sart::Communicator::check)
        .def("device_failed", &sart::Communicator::device_failed)
        .def_property_readonly("degradable", &sart::Communicator::degradable)
        .def("degrade", &sart::Communicator::degrade)
        .def("barrier", [](sart::Communicator& c) { c.host().barrier(); }, py::call_guard<py::gil_scoped_release>())
        .def("abort", &sart::Communicator::abort)
        .def("all_reduce_host",
             [](sart::Communicator& c, f64arr v, sart::ReduceOp op) {
                 py::array_t<double> out(v.size());
                 std::memcpy(out.mutable_data(), v.data(), v.size() * sizeof(double));
                 double* p = out.mutable_data();
                 const size_t n = (size_t)v.size();
                 {
                     py::gil_scoped_release rel;
                     c.host().all_reduce_host(p, n, op);
                 }
                 return out;
             })
        .def("broadcast_bytes",
             [](sart::Communicator& c, py::bytes data, size_t nbytes, int root) {
                 std::string buf(nbytes, '\0');
                 if (c.rank() == root) {
                     const std::string d = data;
                     if (d.size() != nbytes) throw py::value_error("broadcast_bytes: root payload size mismatch");
                     buf = d;
                 }
                 {
                     py::gil_scoped_release rel;
                     c.host().broadcast_host(buf.data(), nbytes, root);
                 }
                 return py::bytes(buf);
             })
        .def("all_reduce_device",
             [](sart::Communicator& c, uintptr_t ptr, size_t n, bool f64, sart::ReduceOp op, uintptr_t stream) {
                 py::gil_scoped_release rel;
                 if (f64)
                     c.all_reduce(P<double>(ptr), n, op, S(stream));
                 else
                     c.all_reduce(P<float>(ptr), n, op, S(stream));
             });
    m.def("local_comm", []() { return std::shared_ptr<sart::Communicator>(sart::make_local_comm()); });
    m.def("staged_comm",
          [](int rank, int size, const std::string& host, int port, double timeout_s) {
              py::gil_scoped_release rel;
              return std::shared_ptr<sart::Communicator>(
                  sart::make_staged_comm(sart::make_tcp_host_comm(rank, size, host, port, timeout_s)));
          },
          py::arg("rank"), py::arg("size"), py::arg("host"), py::arg("port"), py::arg("timeout_s") = 3600.0);
    m.def("rccl_unique_id", []() { return py::bytes(sart::rccl_unique_id()); });
    m.def("rccl_comm",
          [](int device, py::bytes uid, int rank, int size, const std::string& host, int port) {
              const std::string id = uid;
              py::gil_scoped_release rel;
              return std::shared_ptr<sart::Communicator>(
                  sart::make_rccl_comm(device, id, sart::make_tcp_host_comm(rank, size, host, port)));
          });
    m.def("p2p_comm",
          [](int device, std::shared_ptr<sart::Communicator> base) {
              py::gil_scoped_release rel;
              return std::shared_ptr<sart::Communicator>(sart::make_p2p_comm(device, std::move(base)));
          },
          py::arg("device"), py::arg("base"));
    m.def("comm_from_env", [](int device) {
        py::gil_scoped_release rel;
        return std::shared_ptr<sart::Communicator>(sart::comm_from_env(device));
    });

    py::class_<sart::FusedGeometry>(m, "FusedGeometry")
        .def_readonly("K", &sart::FusedGeometry::K)
        .def_readonly("J", &sart::FusedGeometry::J)
        .def_readonly("I", &sart::FusedGeometry::I)
        .def_readonly("grid", &sart::FusedGeometry::grid)
        .def_readonly("variant", &sart::FusedGeometry::variant)
        .def_readonly("T", &sart::FusedGeometry::T)
        .def_readonly("cpl", &sart::FusedGeometry::cpl)
        .def_readonly("kw", &sart::FusedGeometry::kw)
        .def_readonly("xl", &sart::FusedGeometry::xl)
        .def("valid", &sart::FusedGeometry::valid);
    m.def("fused_geometry", &sart::fused_geometry, py::arg("ld"), py::arg("num_cus"), py::arg("variant") = 6,
          py::arg("rows_per_tile") = 0, py::arg("narrow_slabs") = true, py::arg("chip_wide") = true);
    m.def("fused_geometry_bf16_wide", &sart::fused_geometry_bf16_wide, py::arg("ld"), py::arg("num_cus"));
    m.def("fused_fold_tiles", &sart::fused_fold_tiles, py::arg("geometry"), py::arg("nrows_pad"));
    m.def("fused_chain_plan", [](const sart::FusedGeometry& g, int64_t nrows_pad, bool split) {
        const auto p = sart::fused_chain_plan(g, nrows_pad, split);
        return py::make_tuple(p.chain_tiles, p.blocks);
    }, py::arg("geometry"), py::arg("nrows_pad"), py::arg("split_schedule"));
    m.def("fused_split_schedule", &sart::fused_split_schedule, py::arg("T"), py::arg("bf16"));
    m.def("choose_ld", &sart::choose_ld, py::arg("nvoxel"), py::arg("max_waste") = 0.10,
          py::arg("narrow_slabs") = true);

    py::class_<sart::EngineConfig>(m, "EngineConfig")
        .def(py::init<>())
        .def_readwrite("logarithmic", &sart::EngineConfig::logarithmic)
        .def_readwrite("ray_density_threshold", &sart::EngineConfig::ray_density_threshold)
        .def_readwrite("ray_length_threshold", &sart::EngineConfig::ray_length_threshold)
        .def_readwrite("conv_tolerance", &sart::EngineConfig::conv_tolerance)
        .def_readwrite("beta_laplace", &sart::EngineConfig::beta_laplace)
        .def_readwrite("relaxation", &sart::EngineConfig::relaxation)
        .def_readwrite("max_iterations", &sart::EngineConfig::max_iterations)
        .def_readwrite("allow_zero_tolerance", &sart::EngineConfig::allow_zero_tolerance)
        .def_readwrite("check_interval", &sart::EngineConfig::check_interval)
        .def_readwrite("use_fused", &sart::EngineConfig::use_fused)
        .def_readwrite("mf_frames", &sart::EngineConfig::mf_frames)
        .def_readwrite("fused_min_bytes", &sart::EngineConfig::fused_min_bytes)
        .def_readwrite("column_shard", &sart::EngineConfig::column_shard)
        .def_readwrite("col_offset", &sart::EngineConfig::col_offset)
        .def_readwrite("nvoxel_total", &sart::EngineConfig::nvoxel_total)
        .def_readwrite("fused_variant", &sart::EngineConfig::fused_variant)
        .def_readwrite("rows_per_tile", &sart::EngineConfig::rows_per_tile)
        .def_readwrite("fused_schedule", &sart::EngineConfig::fused_schedule)
        .def_readwrite("use_graph", &sart::EngineConfig::use_graph)
        .def_readwrite("time_collectives", &sart::EngineConfig::time_collectives)
        .def_readwrite("rtm_bf16", &sart::EngineConfig::rtm_bf16)
        .def_readwrite("mf_split_a", &sart::EngineConfig::mf_split_a)
        .def_readwrite("fault_inject", &sart::EngineConfig::fault_inject)
        .def_readwrite("fault_nan_sweep", &sart::EngineConfig::fault_nan_sweep)
        .def_readwrite("fused_max_cus", &sart::EngineConfig::fused_max_cus);
    m.def("validate_config", [](const sart::EngineConfig& c) {
        try {
            sart::validate_params(c);
        } catch (const std::invalid_argument& e) {
            throw py::value_error(e.what());
        }
    });

    py::class_<sart::Engine>(m, "Engine")
        .def(py::init([](int device, uintptr_t A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel, int64_t ld,
                         std::shared_ptr<sart::Communicator> comm, const sart::EngineConfig& cfg) {
                 try {
                     return new sart::Engine(device, P<const float>(A), nrows, nrows_pad, nvoxel, ld, comm.get(), cfg);
                 } catch (const std::invalid_argument& e) {
                     throw py::value_error(e.what());
                 }
             }),
             py::keep_alive<1, 8>())
        // sparse shard: device pointers of the CSR (row_ptr, col, val) and CSC (col_ptr, row, cval) arrays (not owned:
        // the caller keeps them alive with the engine)
        .def_static("from_sparse",
                    [](int device, uintptr_t row_ptr, uintptr_t col, uintptr_t val, uintptr_t col_ptr, uintptr_t row,
                       uintptr_t cval, int64_t nnz, int64_t nrows, int64_t nvoxel,
                       std::shared_ptr<sart::Communicator> comm, const sart::EngineConfig& cfg) {
                        sart::SparseRtm s;
                        s.row_ptr = P<const int64_t>(row_ptr);
                        s.col = P<const int32_t>(col);
                        s.val = P<const float>(val);
                        s.col_ptr = P<const int64_t>(col_ptr);
                        s.row = P<const int32_t>(row);
                        s.cval = P<const float>(cval);
                        s.nnz = nnz;
                        const int64_t pp = (nrows + 63) / 64 * 64, ld = (nvoxel + 63) / 64 * 64;
                        try {
                            return new sart::Engine(device, nullptr, nrows, pp, nvoxel, ld, comm.get(), cfg, &s);
                        } catch (const std::invalid_argument& e) {
                            throw py::value_error(e.what());
                        }
                    },
                    py::keep_alive<0, 11>())
        .def("set_laplacian",
             [](sart::Engine& e, py::array_t<int64_t, py::array::c_style | py::array::forcecast> rp,
                py::array_t<int32_t, py::array::c_style | py::array::forcecast> col,
                py::array_t<float, py::array::c_style | py::array::forcecast> val) {
                 e.set_laplacian(rp.data(), col.data(), val.data(), (int64_t)val.size());
             })
        .def("solve",
             [](sart::Engine& e, f64arr g, py::object x0) {
                 if ((int64_t)g.size() != e.nrows())
                     throw py::value_error("measurement has " + std::to_string(g.size()) +
                                           " pixels, the local shard has " + std::to_string(e.nrows()));
                 f64arr x0a;
                 const double* x0p = nullptr;
                 if (!x0.is_none()) {
                     x0a = x0.cast<f64arr>();
                     if ((int64_t)x0a.size() != e.nvoxel())
                         throw py::value_error("Solution vector must be empty or contain nvoxel elements.");
                     x0p = x0a.data();
                 }
                 py::array_t<double> x(e.nvoxel());
                 double* xp = x.mutable_data();
                 const double* gp = g.data();
                 sart::SolveInfo info;
                 {
                     py::gil_scoped_release rel;
                     info = e.solve(gp, x0p, xp);
                 }
                 return py::make_tuple(x, solve_info(info));
             },
             py::arg("g"), py::arg("x0") = py::none())
        .def("forward",
             [](sart::Engine& e, f64arr x) {
                 if ((int64_t)x.size() != e.nvoxel()) throw py::value_error("x must have nvoxel elements");
                 py::array_t<double> f(e.nrows());
                 e.forward(x.data(), f.mutable_data());
                 return f;
             })
        .def_property_readonly("use_fused", &sart::Engine::use_fused)
        .def_property_readonly("geometry", &sart::Engine::geometry)
        .def_property_readonly("num_cus", &sart::Engine::num_cus)
        .def_property_readonly("column_shard", &sart::Engine::column_shard)
        .def_property_readonly("sparse", &sart::Engine::sparse)
        .def_property_readonly("nnz", &sart::Engine::nnz)
        .def_property_readonly("shared_device", &sart::Engine::shared_device)
        .def_property_readonly("ranks_per_device", &sart::Engine::ranks_per_device)
        .def_property_readonly("plan_cus", &sart::Engine::plan_cus)
        .def_property_readonly("nrows", &sart::Engine::nrows)
        .def_property_readonly("nvoxel", &sart::Engine::nvoxel)
        .def_property_readonly("stream", [](const sart::Engine& e) { return reinterpret_cast<uintptr_t>(e.stream()); })
        .def("ray_density", [](const sart::Engine& e) { auto v = e.ray_density(); return py::array_t<double>(v.size(), v.data()); })
        .def("ray_length", [](const sart::Engine& e) { auto v = e.ray_length(); return py::array_t<double>(v.size(), v.data()); })        ;

    py::class_<sart::MultiFrameEngine>(m, "MultiFrameEngine")
        .def(py::init([](int device, uintptr_t A, int64_t nrows, int64_t nrows_pad, int64_t nvoxel, int64_t ld,
                         std::shared_ptr<sart::Communicator> comm, const sart::EngineConfig& cfg) {
                 try {
                     return new sart::MultiFrameEngine(device, P<const void>(A), nrows, nrows_pad, nvoxel, ld,
                                                       comm.get(), cfg);
                 } catch (const std::invalid_argument& e) {
                     throw py::value_error(e.what());
                 }
             }),
             py::keep_alive<1, 8>())
        .def_static("from_sparse",
                    [](int device, uintptr_t row_ptr, uintptr_t col, uintptr_t val, uintptr_t col_ptr, uintptr_t row,
                       uintptr_t cval, int64_t nnz, int64_t nrows, int64_t nvoxel,
                       std::shared_ptr<sart::Communicator> comm, const sart::EngineConfig& cfg) {
                        sart::SparseRtm s;
                        s.row_ptr = P<const int64_t>(row_ptr);
                        s.col = P<const int32_t>(col);
                        s.val = P<const float>(val);
                        s.col_ptr = P<const int64_t>(col_ptr);
                        s.row = P<const int32_t>(row);
                        s.cval = P<const float>(cval);
                        s.nnz = nnz;
                        const int64_t pp = (nrows + 63) / 64 * 64, ld = (nvoxel + 63) / 64 * 64;
                        try {
                            return new sart::MultiFrameEngine(device, nullptr, nrows, pp, nvoxel, ld, comm.get(), cfg,
                                                              &s);
                        } catch (const std::invalid_argument& e) {
                            throw py::value_error(e.what());
                        }
                    },
                    py::keep_alive<0, 11>())
        .def_property_readonly("sparse", &sart::MultiFrameEngine::sparse)
        .def_property_readonly("batch_frames", &sart::MultiFrameEngine::batch_frames)
        .def_property_readonly("split_a", &sart::MultiFrameEngine::split_a)
        .def_property_readonly("forward_split", &sart::MultiFrameEngine::forward_split)
        .def_property_readonly("backproject_split", &sart::MultiFrameEngine::backproject_split)
        .def("set_laplacian",
             [](sart::MultiFrameEngine& e, py::array_t<int64_t, py::array::c_style | py::array::forcecast> rp,
                py::array_t<int32_t, py::array::c_style | py::array::forcecast> col,
                py::array_t<float, py::array::c_style | py::array::forcecast> val) {
                 e.set_laplacian(rp.data(), col.data(), val.data(), (int64_t)val.size());
             })
        .def("solve_batch", [](sart::MultiFrameEngine& e, f64arr g, py::object x0, bool chain, bool record_starts) -> py::tuple {
            if (g.ndim() != 2 || g.shape(1) != e.nrows())
                throw py::value_error("measurements must be [nframes, nrows of the local shard]");
            const int nf = (int)g.shape(0);
            f64arr x0a;
            const double* x0p = nullptr;
            if (!x0.is_none()) {
                x0a = x0.cast<f64arr>();
                if ((int64_t)x0a.size() != e.nvoxel()) throw py::value_error("x0 must have nvoxel elements");
                x0p = x0a.data();
            }
            py::array_t<double> x({(py::ssize_t)nf, (py::ssize_t)e.nvoxel()});
            py::array_t<double> st({(py::ssize_t)(record_starts ? nf : 0), (py::ssize_t)e.nvoxel()});
            double* xp = x.mutable_data();
            double* sp = record_starts ? st.mutable_data() : nullptr;
            const double* gp = g.data();
            std::vector<sart::SolveInfo> infos;
            {
                py::gil_scoped_release rel;
                infos = e.solve_batch(gp, nf, xp, x0p, chain, sp);
            }
            py::list li;
            for (const auto& i : infos) li.append(solve_info(i));
            if (record_starts) return py::make_tuple(x, li, st);
            return py::make_tuple(x, li);
        }, py::arg("g"), py::arg("x0") = py::none(), py::arg("chain") = false, py::arg("record_starts") = false)
        .def_property_readonly("series_stats", [](sart::MultiFrameEngine& e) {
            const auto& s = e.series_stats();
            py::dict d;
            d["frames"] = s.frames;
            d["sweeps"] = s.sweeps;
            d["queued_sweeps"] = s.queued_sweeps;
            d["busy_slot_sweeps"] = s.busy_slot_sweeps;
            d["chained"] = s.chained;
            d["slot_util"] = s.slot_util;
            d["mean_iterations"] = s.mean_iterations;
            d["mean_warm_age"] = s.mean_warm_age;
            d["ms"] = s.ms;
            d["chunk"] = s.chunk;
            d["admit_cap"] = s.admit_cap;
            d["src_age"] = s.src_age;
            d["restarts"] = s.restarts;
            d["src_finished"] = s.src_finished;
            d["lead"] = s.lead;
            d["src_extrap"] = s.src_extrap;
            d["drift"] = s.drift;
            d["host_wait_ms"] = s.host_wait_ms;
            d["host_stage_ms"] = s.host_stage_ms;
            d["host_src_ms"] = s.host_src_ms;
            d["host_deliver_ms"] = s.host_deliver_ms;
            return d;
        });
}

PYBIND11_MODULE(_sart_hip, m) {
    m.doc() = "Hand-written gfx950 (CDNA4) HIP kernels of the SART solver and the native engine";
    bind_engine(m);

    m.def("arch", []() { return std::string("gfx950"); });
    m.def("state_nbytes", []() { return (int)sizeof(sart::SartState); });

    m.def("device_info", [](int dev) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess) throw std::runtime_error("hipGetDeviceProperties failed");
        py::dict d;
        d["name"] = std::string(prop.name);
        d["gcnArchName"] = std::string(prop.gcnArchName);
        d["multiProcessorCount"] = prop.multiProcessorCount;
        d["totalGlobalMem"] = (int64_t)prop.totalGlobalMem;
        d["l2CacheSize"] = prop.l2CacheSize;
        d["clockRate_kHz"] = prop.clockRate;
        d["memoryClockRate_kHz"] = prop.memoryClockRate;
        d["memoryBusWidth"] = prop.memoryBusWidth;
        return d;
    });

    m.def("forward_num_blocks", &sart::forward_num_blocks);
    // bf16: A holds bf16 bit patterns (opt-in storage precision)
    m.def("forward", [](int epi, uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t x,
                        uintptr_t ghat, uintptr_t arow, uintptr_t out_f, uintptr_t out_w, uintptr_t Fpart,
                        uintptr_t st, uintptr_t stream, bool bf16) {
        if (bf16)
            sart::launch_forward(epi, P<const sart::bf16_t>(A), ld, nrows, nrows_pad, P<const float>(x),
                                 P<const float>(ghat), P<const float>(arow), P<float>(out_f), P<float>(out_w),
                                 P<double>(Fpart), P<const sart::SartState>(st), S(stream));
        else
            sart::launch_forward(epi, P<const float>(A), ld, nrows, nrows_pad, P<const float>(x), P<const float>(ghat),
                                 P<const float>(arow), P<float>(out_f), P<float>(out_w), P<double>(Fpart),
                                 P<const sart::SartState>(st), S(stream));
    }, py::arg("epi"), py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("nrows_pad"), py::arg("x"),
       py::arg("ghat"), py::arg("arow"), py::arg("out_f"), py::arg("out_w"), py::arg("Fpart"), py::arg("st"),
       py::arg("stream"), py::arg("bf16") = false);
    m.def("rowsum_f64", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t out, uintptr_t stream, bool bf16) {
        if (bf16)
            sart::launch_rowsum_f64(P<const sart::bf16_t>(A), ld, nrows, P<double>(out), S(stream));
        else
            sart::launch_rowsum_f64(P<const float>(A), ld, nrows, P<double>(out), S(stream));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("out"), py::arg("stream"), py::arg("bf16") = false);
    m.def("backproject_num_splits", &sart::backproject_num_splits, py::arg("ld"), py::arg("nrows"),
          py::arg("elem_bytes") = 4);
    m.def("backproject", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t w, int nsplit, uintptr_t partial,
                            uintptr_t st, uintptr_t stream, bool bf16) {
        if (bf16)
            sart::launch_backproject(P<const sart::bf16_t>(A), ld, nrows, P<const float>(w), nsplit,
                                     P<float>(partial), P<const sart::SartState>(st), S(stream));
        else
            sart::launch_backproject(P<const float>(A), ld, nrows, P<const float>(w), nsplit, P<float>(partial),
                                     P<const sart::SartState>(st), S(stream));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("w"), py::arg("nsplit"), py::arg("partial"),
       py::arg("st"), py::arg("stream"), py::arg("bf16") = false);
    m.def("colsum_f64", [](uintptr_t A, int64_t ld, int64_t nrows, int nsplit, uintptr_t partial, uintptr_t stream,
                           bool bf16) {
        if (bf16)
            sart::launch_colsum_f64(P<const sart::bf16_t>(A), ld, nrows, nsplit, P<double>(partial), S(stream));
        else
            sart::launch_colsum_f64(P<const float>(A), ld, nrows, nsplit, P<double>(partial), S(stream));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("nsplit"), py::arg("partial"), py::arg("stream"),
       py::arg("bf16") = false);
    m.def("f32_to_bf16", [](uintptr_t src, int64_t n, uintptr_t dst, uintptr_t stream) {
        sart::launch_f32_to_bf16(P<const float>(src), n, P<sart::bf16_t>(dst), S(stream));
    });
    m.def("reduce_partials", [](uintptr_t partial, int64_t ld, int nsplit, uintptr_t scale, uintptr_t out,
                                uintptr_t Fpart, int64_t nF, uintptr_t Fout, uintptr_t st, uintptr_t stream) {
        sart::launch_reduce_partials(P<const float>(partial), ld, nsplit, P<const float>(scale), P<float>(out),
                                     P<const double>(Fpart), nF, P<float>(Fout), P<const sart::SartState>(st),
                                     S(stream));
    });
    m.def("reduce_partials_f64", [](uintptr_t partial, int64_t ld, int nsplit, uintptr_t out, uintptr_t stream) {
        sart::launch_reduce_partials_f64(P<const double>(partial), ld, nsplit, P<double>(out), S(stream));
    });
    m.def("prep_rows", [](uintptr_t g, int64_t nrows, int64_t nrows_pad, double inv_s, uintptr_t ray_length,
                          float len_thres, uintptr_t ghat, uintptr_t arow, uintptr_t gpos, uintptr_t wo,
                          uintptr_t stream) {
        sart::launch_prep_rows(P<const double>(g), nrows, nrows_pad, inv_s, P<const float>(ray_length), len_thres,
                               P<float>(ghat), P<float>(arow), P<float>(gpos), P<float>(wo), S(stream));
    });
    m.def("init_solution", [](uintptr_t x, int64_t n, int64_t n_pad, uintptr_t src_f32, uintptr_t src_f64,
                              double scale, uintptr_t stream) {
        sart::launch_init_solution(P<float>(x), n, n_pad, P<const float>(src_f32), P<const double>(src_f64), scale,
                                   S(stream));
    });
    m.def("penalty", [](bool logx, uintptr_t row_ptr, uintptr_t col, uintptr_t val, int64_t n, float beta,
                        uintptr_t x, uintptr_t pen, uintptr_t st, uintptr_t stream) {
        sart::launch_penalty(logx, P<const int64_t>(row_ptr), P<const int32_t>(col), P<const float>(val), n, beta,
                             P<const float>(x), P<float>(pen), P<const sart::SartState>(st), S(stream));
    });
    m.def("decide", [](uintptr_t st, uintptr_t Fslot, uintptr_t stream) {
        sart::launch_decide(P<sart::SartState>(st), P<const float>(Fslot), S(stream));
    });
    m.def("update_linear", [](uintptr_t x, uintptr_t d, uintptr_t pen, int64_t n, uintptr_t st, uintptr_t stream) {
        sart::launch_update_linear(P<float>(x), P<const float>(d), P<const float>(pen), n,
                                   P<const sart::SartState>(st), S(stream));
    });
    m.def("update_log", [](uintptr_t x, uintptr_t O, uintptr_t Fv, uintptr_t pen, float alpha, int64_t n,
                           uintptr_t st, uintptr_t stream) {
        sart::launch_update_log(P<float>(x), P<const float>(O), P<const float>(Fv), P<const float>(pen), alpha, n,
                                P<const sart::SartState>(st), S(stream));
    });
    m.def("state_begin", [](uintptr_t st, double G, double tol, int max_iter, uintptr_t stream) {
        sart::launch_state_begin(P<sart::SartState>(st), G, tol, max_iter, S(stream));
    });
    m.def("synth_matrix", [](uintptr_t A, int64_t ld, int64_t nrows_pad, int64_t nrows, int64_t ncols,
                             int64_t row_offset, uint64_t seed, float lo, float hi, uintptr_t stream,
                             int64_t col_offset, int64_t ncols_total) {
        sart::launch_synth_matrix_block(P<float>(A), ld, nrows_pad, nrows, ncols, row_offset, col_offset,
                                        ncols_total > 0 ? ncols_total : ncols, seed, lo, hi, S(stream));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows_pad"), py::arg("nrows"), py::arg("ncols"), py::arg("row_offset"),
       py::arg("seed"), py::arg("lo"), py::arg("hi"), py::arg("stream"), py::arg("col_offset") = 0,
       py::arg("ncols_total") = 0);
    m.def("synth_vector", [](uintptr_t out, int64_t n, int64_t offset, uint64_t seed, double lo, double hi,
                             uintptr_t stream) {
        sart::launch_synth_vector(P<double>(out), n, offset, seed, lo, hi, S(stream));
    });
    m.def("fused_pick_k", &sart::fused_pick_k);
    m.def("fused_tile_rows", &sart::fused_tile_rows);
    m.def("fused_set_schedule", &sart::fused_set_schedule);
    m.def("fused_get_schedule", &sart::fused_get_schedule);
    m.def("fused_granules", &sart::fused_granules, py::arg("nrows_pad"), py::arg("J"), py::arg("xl") = true);
    m.def("fused_last_schedule", &sart::fused_last_schedule);
    m.def("fused_debug_map", &sart::fused_debug_map);
    m.def("fused_set_trace", [](uintptr_t buf, long long tiles) {
        sart::fused_set_trace(reinterpret_cast<unsigned long long*>(buf), tiles);
    });
    m.def("fused_fpart_per_block", &sart::fused_fpart_per_block);
    m.def("fused_set_debug", &sart::fused_set_debug);
    m.def("fused_debug_stats", &sart::fused_debug_stats);
    m.def("fused_sweep", [](bool logmode, int K, int variant, uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad,
                            uintptr_t x, uintptr_t ghat, uintptr_t arow, uintptr_t partial, uintptr_t Fpart,
                            uintptr_t gran, int I, int J, uintptr_t st, uintptr_t xcnt, uintptr_t stream) {
        sart::launch_fused_sweep(logmode, K, variant, P<const float>(A), ld, nrows, nrows_pad, P<const float>(x),
                                 P<const float>(ghat), P<const float>(arow), P<float>(partial), P<double>(Fpart),
                                 P<uint64_t>(gran), I, J, P<sart::SartState>(st), P<unsigned>(xcnt), S(stream));
    });
    m.def("fused_min_bytes_from_env", &sart::fused_min_bytes_from_env);
    m.def("mf_forward_num_splits", &sart::mf_forward_num_splits, py::arg("ld"), py::arg("nrows_pad"), py::arg("target") = 0);
    m.def("mf_backproject_num_splits", &sart::mf_backproject_num_splits);
    m.def("mf_set_depth", &sart::mf_set_depth);
    m.def("mf_set_rows", &sart::mf_set_rows);
    m.def("mf_set_vox", &sart::mf_set_vox);
    m.def("mf_forward", [](uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t X, int64_t ldx,
                           uintptr_t Fout, int nsplit, uintptr_t stream, int nf) {
        sart::launch_mf_forward(P<const float>(A), ld, nrows, nrows_pad, P<const float>(X), ldx, P<float>(Fout),
                                nsplit, nf, S(stream));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("nrows_pad"), py::arg("X"), py::arg("ldx"),
       py::arg("Fout"), py::arg("nsplit"), py::arg("stream"), py::arg("nf") = 16);
    m.def("mf_backproject_b16_num_splits", &sart::mf_backproject_b16_num_splits, py::arg("ld"), py::arg("nrows"),
          py::arg("a32") = false);
    m.def("mf_backproject_b16_vox_align", &sart::mf_backproject_b16_vox_align, py::arg("ld"), py::arg("a32") = false);
    m.def("mf_forward_x3", [](uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t Xh, uintptr_t Xl,
                              uintptr_t Fout, int nsplit, uintptr_t stream, int nf, bool xblk) {
        sart::launch_mf_forward_x3(P<const float>(A), ld, nrows, nrows_pad, P<const sart::bf16_t>(Xh),
                                   P<const sart::bf16_t>(Xl), P<float>(Fout), nsplit, nf, S(stream), xblk);
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("nrows_pad"), py::arg("Xh"), py::arg("Xl"),
       py::arg("Fout"), py::arg("nsplit"), py::arg("stream"), py::arg("nf"), py::arg("xblk") = false);
    m.def("mf_backproject_x3", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t Wh, uintptr_t Wl, int64_t ldw,
                                  int nsplit, uintptr_t partial, uintptr_t stream, int nf, int64_t v0, int64_t v1) {
        sart::launch_mf_backproject_x3(P<const float>(A), ld, nrows, P<const sart::bf16_t>(Wh),
                                       P<const sart::bf16_t>(Wl), ldw, nsplit, P<float>(partial), nf, S(stream), v0, v1);
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("Wh"), py::arg("Wl"), py::arg("ldw"), py::arg("nsplit"),
       py::arg("partial"), py::arg("stream"), py::arg("nf") = 16, py::arg("v0") = 0, py::arg("v1") = -1);
    m.def("mf_split_x", [](uintptr_t X, int64_t n, uintptr_t hi, uintptr_t lo, uintptr_t stream, bool perm,
                           int64_t ld) {
        sart::launch_mf_split_x(P<const float>(X), n, P<sart::bf16_t>(hi), P<sart::bf16_t>(lo), S(stream), perm, ld);
    }, py::arg("X"), py::arg("n"), py::arg("hi"), py::arg("lo"), py::arg("stream"), py::arg("perm") = false,
       py::arg("ld") = 0);
    m.def("mf_split_w16", [](uintptr_t W, int64_t nrows_pad, int nf, int64_t ldw, uintptr_t w1, uintptr_t w2,
                             uintptr_t wmax, float a_scale, uintptr_t inv_scale, uintptr_t stream) {
        sart::launch_mf_split_w16(P<const float>(W), nrows_pad, nf, ldw, P<uint16_t>(w1), P<uint16_t>(w2),
                                  P<unsigned>(wmax), a_scale, P<float>(inv_scale), S(stream));
    });
    m.def("absmax_pow2_scale", [](uintptr_t A, int64_t n, uintptr_t scratch, uintptr_t stream) {
        return sart::absmax_pow2_scale(P<const float>(A), n, P<unsigned>(scratch), S(stream));
    });
    m.def("mf_backproject_h16", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t W1, uintptr_t W2, int64_t ldw,
                                   int nsplit, uintptr_t partial, uintptr_t stream, int nf, int64_t v0, int64_t v1,
                                   uintptr_t csc, uintptr_t inv_scale) {
        sart::launch_mf_backproject_h16(P<const float>(A), ld, nrows, P<const uint16_t>(W1), P<const uint16_t>(W2), ldw,
                                        nsplit, P<float>(partial), nf, S(stream), v0, v1, P<const float>(csc),
                                        P<const float>(inv_scale));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("W1"), py::arg("W2"), py::arg("ldw"), py::arg("nsplit"),
       py::arg("partial"), py::arg("stream"), py::arg("nf"), py::arg("v0"), py::arg("v1"), py::arg("csc"),
       py::arg("inv_scale"));
    m.def("mf_row_scales", [](uintptr_t A, int64_t ld, int64_t nrows_pad, uintptr_t rsc, uintptr_t stream) {
        sart::launch_mf_row_scales(P<const float>(A), ld, nrows_pad, P<float>(rsc), S(stream));
    });
    m.def("mf_col_scales", [](uintptr_t A, int64_t ld, int64_t nrows_pad, uintptr_t scratch, uintptr_t csc,
                              uintptr_t stream) {
        sart::launch_mf_col_scales(P<const float>(A), ld, nrows_pad, P<unsigned>(scratch), P<float>(csc), S(stream));
    });
    m.def("mf_split_x16", [](uintptr_t X, int64_t ld, int nf, uintptr_t x1, uintptr_t x2, uintptr_t xmax,
                             uintptr_t xinv, uintptr_t stream, bool perm, bool blocked) {
        sart::launch_mf_split_x16(P<const float>(X), ld, nf, P<uint16_t>(x1), P<uint16_t>(x2), P<unsigned>(xmax),
                                  P<float>(xinv), S(stream), perm, blocked);
    }, py::arg("X"), py::arg("ld"), py::arg("nf"), py::arg("x1"), py::arg("x2"), py::arg("xmax"), py::arg("xinv"),
       py::arg("stream"), py::arg("perm") = true, py::arg("blocked") = false);
    m.def("mf_forward_h16", [](uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t X1, uintptr_t X2,
                               uintptr_t Fout, int nsplit, uintptr_t stream, int nf, bool xblk, uintptr_t rsc,
                               uintptr_t xinv) {
        sart::launch_mf_forward_h16(P<const float>(A), ld, nrows, nrows_pad, P<const uint16_t>(X1),
                                    P<const uint16_t>(X2), P<float>(Fout), nsplit, nf, S(stream), xblk,
                                    P<const float>(rsc), P<const float>(xinv));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("nrows_pad"), py::arg("X1"), py::arg("X2"),
       py::arg("Fout"), py::arg("nsplit"), py::arg("stream"), py::arg("nf"), py::arg("xblk"), py::arg("rsc"),
       py::arg("xinv"));
    m.def("mf_split_w", [](uintptr_t W, int64_t nrows_pad, int nf, int64_t ldw, uintptr_t hi, uintptr_t lo,
                           uintptr_t stream, bool three) {
        sart::launch_mf_split_w(P<const float>(W), nrows_pad, nf, ldw, P<sart::bf16_t>(hi), P<sart::bf16_t>(lo),
                                S(stream), three);
    }, py::arg("W"), py::arg("nrows_pad"), py::arg("nf"), py::arg("ldw"), py::arg("hi"), py::arg("lo"),
       py::arg("stream"), py::arg("three") = false);
    m.def("mf_forward_b16", [](uintptr_t A, int64_t ld, int64_t nrows, int64_t nrows_pad, uintptr_t Xh, uintptr_t Xl,
                               uintptr_t Fout, int nsplit, uintptr_t stream, int nf, bool xblk) {
        sart::launch_mf_forward_b16(P<const sart::bf16_t>(A), ld, nrows, nrows_pad, P<const sart::bf16_t>(Xh),
                                    P<const sart::bf16_t>(Xl), P<float>(Fout), nsplit, nf, S(stream), xblk);
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("nrows_pad"), py::arg("Xh"), py::arg("Xl"),
       py::arg("Fout"), py::arg("nsplit"), py::arg("stream"), py::arg("nf"), py::arg("xblk") = false);
    m.def("mf_backproject_b16", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t Wh, uintptr_t Wl, int64_t ldw,
                                   int nsplit, uintptr_t partial, uintptr_t stream, int nf, int64_t v0, int64_t v1) {
        sart::launch_mf_backproject_b16(P<const sart::bf16_t>(A), ld, nrows, P<const sart::bf16_t>(Wh),
                                        P<const sart::bf16_t>(Wl), ldw, nsplit, P<float>(partial), nf, S(stream), v0,
                                        v1);
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("Wh"), py::arg("Wl"), py::arg("ldw"), py::arg("nsplit"),
       py::arg("partial"), py::arg("stream"), py::arg("nf") = 16, py::arg("v0") = 0, py::arg("v1") = -1);
    m.def("mf_backproject", [](uintptr_t A, int64_t ld, int64_t nrows, uintptr_t W, int nsplit, uintptr_t partial,
                               uintptr_t stream, int nf) {
        sart::launch_mf_backproject(P<const float>(A), ld, nrows, P<const float>(W), nsplit, P<float>(partial), nf,
                                    S(stream));
    }, py::arg("A"), py::arg("ld"), py::arg("nrows"), py::arg("W"), py::arg("nsplit"), py::arg("partial"),
       py::arg("stream"), py::arg("nf") = 16);
}
