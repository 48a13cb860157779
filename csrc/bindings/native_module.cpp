// Python bindings of the native host runtime (module mpi_cuda_sartsolver_amd._lib._sart_native):
// CLI/config, time intervals, HDF5 input validation and loaders, composite-image streamer, solution
// writer, voxel grids, fp64 CPU kernels and HDF5 fixture writers. Long-running calls release the GIL
// so the Python driver can prefetch the next frame / RTM block while the GPU works.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "config.hpp"
#include "cpu_kernels.hpp"
#include "cpu_solver.hpp"
#include "sparse_csr.hpp"
#include "host_comm.hpp"
#include "fixtures.hpp"
#include "frames.hpp"
#include "h5.hpp"
#include "inputs.hpp"

namespace py = pybind11;
using namespace sart;

using f32arr = py::array_t<float, py::array::c_style | py::array::forcecast>;
using f64arr = py::array_t<double, py::array::c_style | py::array::forcecast>;
using u64arr = py::array_t<uint64_t, py::array::c_style | py::array::forcecast>;
using u8arr = py::array_t<uint8_t, py::array::c_style | py::array::forcecast>;
using i32arr = py::array_t<int32_t, py::array::c_style | py::array::forcecast>;

template <typename T>
static std::vector<T> vec(const py::array_t<T, py::array::c_style | py::array::forcecast>& a) {
    return std::vector<T>(a.data(), a.data() + a.size());
}

template <typename T>
static py::array_t<T> arr(const std::vector<T>& v) {
    py::array_t<T> out(v.size());
    std::copy(v.begin(), v.end(), out.mutable_data());
    return out;
}

static void check_rows(const py::buffer_info& bi, int64_t P, int64_t V, int64_t ld) {
    if (bi.ndim != 2 || bi.shape[0] < P || bi.shape[1] != ld || ld < V)
        throw std::invalid_argument("matrix must be a C-contiguous float32 array of shape [>=P, ld >= V]");
}

PYBIND11_MODULE(_sart_native, m) {
    m.doc() = "Native C++ runtime of the MI355X SART solver (CLI, HDF5 I/O, CPU kernels)";
    py::register_exception<Error>(m, "NativeError", PyExc_RuntimeError);
    m.def("have_hdf5", &have_hdf5);

    // ---------------------------------------------------------------- config
    py::class_<Config>(m, "Config")
        .def(py::init<>())
        .def_readwrite("input_files", &Config::input_files)
        .def_readwrite("output_file", &Config::output_file)
        .def_readwrite("time_range", &Config::time_range)
        .def_readwrite("laplacian_file", &Config::laplacian_file)
        .def_readwrite("raytransfer_name", &Config::raytransfer_name)
        .def_readwrite("wavelength_threshold", &Config::wavelength_threshold)
        .def_readwrite("ray_density_threshold", &Config::ray_density_threshold)
        .def_readwrite("ray_length_threshold", &Config::ray_length_threshold)
        .def_readwrite("conv_tolerance", &Config::conv_tolerance)
        .def_readwrite("beta_laplace", &Config::beta_laplace)
        .def_readwrite("relaxation", &Config::relaxation)
        .def_readwrite("max_iterations", &Config::max_iterations)
        .def_readwrite("max_cached_frames", &Config::max_cached_frames)
        .def_readwrite("max_cached_solutions", &Config::max_cached_solutions)
        .def_readwrite("logarithmic", &Config::logarithmic)
        .def_readwrite("no_guess", &Config::no_guess)
        .def_readwrite("use_cpu", &Config::use_cpu)
        .def_readwrite("parallel_read", &Config::parallel_read)
        .def_readwrite("resume", &Config::resume)
        .def_readwrite("batch_frames", &Config::batch_frames)
        .def_readwrite("two_pass", &Config::two_pass)
        .def_readwrite("partition_voxels", &Config::partition_voxels)
        .def_readwrite("rtm_bf16", &Config::rtm_bf16)
        .def_readwrite("rtm_format", &Config::rtm_format)
        .def_readwrite("profile_file", &Config::profile_file)
        .def_readwrite("help", &Config::help);
    m.def("parse_arguments", &parse_arguments, py::arg("argv"));
    m.def("usage", &usage);
    m.def("parse_time_intervals", &parse_time_intervals, py::arg("spec"));

    // ---------------------------------------------------------------- input validation
    m.def("categorize_input_files", [](const std::vector<std::string>& files) {
        std::vector<std::string> r, i;
        categorize_input_files(files, r, i);
        return py::make_tuple(r, i);
    });
    m.def("check_group_attribute_consistency", &check_group_attribute_consistency, py::arg("files"),
          py::arg("group"), py::arg("names"), py::arg("integer"));
    m.def("sort_rtm_files", &sort_rtm_files);
    m.def("check_rtm_frame_consistency", &check_rtm_frame_consistency);
    m.def("check_rtm_voxel_consistency", &check_rtm_voxel_consistency);
    m.def("read_rtm_frame_masks", [](const SortedRtmFiles& s) {
        py::dict d;
        for (auto& [k, v] : read_rtm_frame_masks(s)) d[py::str(k)] = arr(v);
        return d;
    });
    m.def("read_rtm_frame_shapes", &read_rtm_frame_shapes);
    m.def("sort_image_files", &sort_image_files);
    m.def("check_rtm_image_consistency", &check_rtm_image_consistency, py::arg("rtm_files"), py::arg("image_files"),
          py::arg("rtm_name"), py::arg("wavelength_threshold"));
    m.def("get_total_rtm_size", &get_total_rtm_size);
    m.def("rtm_has_sparse", &rtm_has_sparse);
    m.def(
        "read_rtm_rows",
        [](const SortedRtmFiles& s, const std::string& name, uint64_t nvoxel, uint64_t r0, uint64_t r1,
           py::array_t<float, py::array::c_style> out) {
            auto bi = out.request(true);
            if (bi.ndim != 2 || (uint64_t)bi.shape[0] < r1 - r0 || (uint64_t)bi.shape[1] < nvoxel)
                throw std::invalid_argument("out must be float32 [rows, ld >= nvoxel]");
            float* ptr = static_cast<float*>(bi.ptr);
            const uint64_t ld = bi.shape[1];
            py::gil_scoped_release nogil;
            read_rtm_rows(s, name, nvoxel, r0, r1, ptr, ld);
        },
        py::arg("sorted_files"), py::arg("rtm_name"), py::arg("nvoxel"), py::arg("row_begin"), py::arg("row_end"),
        py::arg("out"));
    m.def(
        "read_rtm_rows_ptr",
        [](const SortedRtmFiles& s, const std::string& name, uint64_t nvoxel, uint64_t r0, uint64_t r1, uintptr_t ptr,
           uint64_t ld) {
            py::gil_scoped_release nogil;
            read_rtm_rows(s, name, nvoxel, r0, r1, reinterpret_cast<float*>(ptr), ld);
        },
        "Fill a caller-owned (e.g. pinned) host buffer", py::arg("sorted_files"), py::arg("rtm_name"),
        py::arg("nvoxel"), py::arg("row_begin"), py::arg("row_end"), py::arg("ptr"), py::arg("ld"));
    py::class_<RtmReader>(m, "RtmReader")
        .def(py::init<SortedRtmFiles, std::string, uint64_t, uint64_t, uint64_t>(), py::arg("sorted_files"),
             py::arg("rtm_name"), py::arg("nvoxel"), py::arg("col_begin") = 0, py::arg("col_end") = 0)
        .def_property_readonly("ncols", &RtmReader::ncols)
        .def(
            "read_csr",
            [](RtmReader& r, uint64_t r0, uint64_t r1) {
                HostCsr a;
                {
                    py::gil_scoped_release nogil;
                    a = r.read_csr(r0, r1);
                }
                return py::make_tuple(py::array_t<int64_t>(a.ptr.size(), a.ptr.data()),
                                      py::array_t<int32_t>(a.idx.size(), a.idx.data()),
                                      py::array_t<float>(a.val.size(), a.val.data()));
            },
            "Rows [r0, r1) x the column window as CSR (row_ptr, col, value) of the non-zeros", py::arg("row_begin"),
            py::arg("row_end"))
        .def("set_rows_per_read", &RtmReader::set_rows_per_read, py::arg("rows"))
        .def(
            "read_ptr",
            [](RtmReader& r, uint64_t r0, uint64_t r1, uintptr_t ptr, uint64_t ld) {
                py::gil_scoped_release nogil;
                r.read(r0, r1, reinterpret_cast<float*>(ptr), ld);
            },
            "Rows [r0, r1) x the column window into a caller-owned (e.g. pinned) host buffer", py::arg("row_begin"),
            py::arg("row_end"), py::arg("ptr"), py::arg("ld"))
        .def("read", [](RtmReader& r, uint64_t r0, uint64_t r1, py::array_t<float, py::array::c_style> out) {
            auto bi = out.request(true);
            if (bi.ndim != 2 || (uint64_t)bi.shape[0] < r1 - r0 || (uint64_t)bi.shape[1] < r.ncols())
                throw std::invalid_argument("out must be float32 [rows, ld >= ncols]");
            float* ptr = static_cast<float*>(bi.ptr);
            const uint64_t ld = bi.shape[1];
            py::gil_scoped_release nogil;
            r.read(r0, r1, ptr, ld);
        });
    m.def("read_laplacian", [](const std::string& path, uint64_t nvoxel) {
        LaplacianCOO L = read_laplacian(path, nvoxel);
        return py::make_tuple(arr(L.i), arr(L.j), arr(L.value));
    });

    // ---------------------------------------------------------------- frames / output / voxel grid
    py::class_<CompositeImage>(m, "CompositeImage")
        .def(py::init([](std::map<std::string, std::string> files, py::dict masks,
                         std::vector<std::array<double, 4>> intervals, uint64_t npixel, uint64_t offset) {
                 std::map<std::string, std::vector<int32_t>> mm;
                 for (auto item : masks) mm[py::cast<std::string>(item.first)] = vec(py::cast<i32arr>(item.second));
                 return new CompositeImage(std::move(files), std::move(mm), intervals, npixel, offset);
             }),
             py::arg("image_files"), py::arg("frame_masks"), py::arg("time_intervals"), py::arg("npixel"),
             py::arg("offset_pixel") = 0)
        .def_property("max_cache_size", &CompositeImage::max_cache_size, &CompositeImage::set_max_cache_size)
        .def("next_frame",
             [](CompositeImage& c) -> py::object {
                 std::vector<double> f;
                 bool ok;
                 {
                     py::gil_scoped_release nogil;
                     ok = c.next_frame(f);
                 }
                 if (!ok) return py::none();
                 return arr(f);
             })
        .def("frame",
             [](CompositeImage& c, uint64_t i) {
                 std::vector<double> f;
                 {
                     py::gil_scoped_release nogil;
                     f = c.frame(i);
                 }
                 return arr(f);
             })
        .def("frame_time", py::overload_cast<uint64_t>(&CompositeImage::frame_time, py::const_))
        .def("camera_frame_time", py::overload_cast<uint64_t>(&CompositeImage::camera_frame_time, py::const_))
        .def("frame_indices", &CompositeImage::frame_indices)
        .def_property_readonly("nframe", &CompositeImage::nframe)
        .def_property_readonly("npixel", &CompositeImage::npixel)
        .def_property_readonly("offset_pixel", &CompositeImage::offset_pixel)
        .def_property_readonly("current_frame_index", &CompositeImage::current_frame_index);

    py::class_<SolutionWriter>(m, "SolutionWriter")
        .def(py::init<std::string, std::vector<std::string>, uint64_t, uint64_t, bool>(), py::arg("filename"),
             py::arg("camera_names"), py::arg("nvoxel"), py::arg("max_cache_size") = 100, py::arg("append") = false)
        .def("add",
             [](SolutionWriter& w, f64arr sol, int32_t status, double t, std::vector<double> cam_t, int32_t iters) {
                 w.add(vec(sol), status, t, cam_t, iters);
             },
             py::arg("solution"), py::arg("status"), py::arg("time"), py::arg("camera_time"),
             py::arg("iterations") = -1)
        .def("flush", &SolutionWriter::flush)
        .def_property("max_cache_size", &SolutionWriter::max_cache_size, &SolutionWriter::set_max_cache_size)
        .def_property_readonly("pending", &SolutionWriter::pending);
    m.def("read_solution_file", [](const std::string& fn) {
        StoredSolutions s = read_solution_file(fn);
        return py::make_tuple(arr(s.time), arr(s.last_solution), arr(s.status));
    });
    // any numeric dataset as float64 with its shape (tests: every frame of solution/value, solution/iterations)
    m.def("read_dataset_f64", [](const std::string& fn, const std::string& name) {
#ifdef SART_HAVE_HDF5
        std::vector<double> v;
        std::vector<hsize_t> dims;
        {
            SART_H5_LOCK;
            H5Id f = h5_open_file(fn);
            v = h5_read_f64(f, name);
            H5Id d = h5_open_dataset(f, name);
            dims = h5_dims(d);
        }
        std::vector<py::ssize_t> shape(dims.begin(), dims.end());
        py::array_t<double> out(shape);
        std::copy(v.begin(), v.end(), out.mutable_data());
        return out;
#else
        (void)fn;
        (void)name;
        throw Error("built without HDF5 support");
        return py::array_t<double>();
#endif
    });

    py::class_<VoxelGrid>(m, "VoxelGrid")
        .def(py::init<>())
        .def_static("coordinate_system", &VoxelGrid::coordinate_system)
        .def("read", &VoxelGrid::read)
        .def("write", &VoxelGrid::write)
        .def("voxel_index", &VoxelGrid::voxel_index)
        .def("voxel_index_at", &VoxelGrid::voxel_index_at)
        .def_readonly("coordsys", &VoxelGrid::coordsys)
        .def_readonly("nx", &VoxelGrid::nx)
        .def_readonly("ny", &VoxelGrid::ny)
        .def_readonly("nz", &VoxelGrid::nz)
        .def_readonly("nvoxel", &VoxelGrid::nvox)
        .def_readonly("warnings", &VoxelGrid::warnings)
        .def_property_readonly("bounds",
                               [](const VoxelGrid& g) {
                                   return py::make_tuple(g.xmin, g.xmax, g.ymin, g.ymax, g.zmin, g.zmax);
                               })
        .def_property_readonly("voxel_map", [](const VoxelGrid& g) { return arr(g.voxmap); });

    // ---------------------------------------------------------------- CPU kernels
    m.def("cpu_num_threads", &cpu_num_threads);
    m.def("cpu_set_num_threads", &cpu_set_num_threads);
    m.def("cpu_raysums", [](py::array_t<float, py::array::c_style> A, int64_t P, int64_t V) {
        auto bi = A.request();
        check_rows(bi, P, V, bi.ndim == 2 ? bi.shape[1] : 0);
        py::array_t<double> rho(V), ell(P);
        const float* a = static_cast<const float*>(bi.ptr);
        double *r = rho.mutable_data(), *e = ell.mutable_data();
        const int64_t ld = bi.shape[1];
        {
            py::gil_scoped_release nogil;
            cpu_raysums(a, P, V, ld, r, e);
        }
        return py::make_tuple(rho, ell);
    });
    m.def("cpu_forward", [](py::array_t<float, py::array::c_style> A, int64_t P, int64_t V, f64arr x) {
        auto bi = A.request();
        check_rows(bi, P, V, bi.ndim == 2 ? bi.shape[1] : 0);
        if (x.size() < V) throw std::invalid_argument("x too short");
        py::array_t<double> f(P);
        const float* a = static_cast<const float*>(bi.ptr);
        const double* xp = x.data();
        double* fp = f.mutable_data();
        const int64_t ld = bi.shape[1];
        double f2;
        {
            py::gil_scoped_release nogil;
            f2 = cpu_forward(a, P, V, ld, xp, fp);
        }
        return py::make_tuple(f, f2);
    });
    m.def("cpu_backproject", [](py::array_t<float, py::array::c_style> A, int64_t P, int64_t V, f64arr w) {
        auto bi = A.request();
        check_rows(bi, P, V, bi.ndim == 2 ? bi.shape[1] : 0);
        if (w.size() < P) throw std::invalid_argument("w too short");
        py::array_t<double> out(V);
        const float* a = static_cast<const float*>(bi.ptr);
        const double* wp = w.data();
        double* op = out.mutable_data();
        const int64_t ld = bi.shape[1];
        {
            py::gil_scoped_release nogil;
            cpu_backproject(a, P, V, ld, wp, op);
        }
        return out;
    });

    // host CSR of (row, col, value) entries (later duplicates win, zeros dropped) and its transpose (= CSC)
    m.def("csr_from_entries", [](int64_t nrows, int64_t ncols, py::array_t<int64_t, py::array::c_style | py::array::forcecast> r,
                                 py::array_t<int32_t, py::array::c_style | py::array::forcecast> c,
                                 py::array_t<float, py::array::c_style | py::array::forcecast> v) {
        std::vector<int64_t> rows(r.data(), r.data() + r.size());
        std::vector<int32_t> cols(c.data(), c.data() + c.size());
        std::vector<float> vals(v.data(), v.data() + v.size());
        sart::HostCsr a;
        try {
            a = sart::csr_from_entries(nrows, ncols, rows, cols, vals);
        } catch (const std::invalid_argument& e) {
            throw py::value_error(e.what());
        }
        return py::make_tuple(py::array_t<int64_t>(a.ptr.size(), a.ptr.data()),
                              py::array_t<int32_t>(a.idx.size(), a.idx.data()),
                              py::array_t<float>(a.val.size(), a.val.data()));
    });
    m.def("csr_transpose", [](int64_t nrows, int64_t ncols, py::array_t<int64_t, py::array::c_style | py::array::forcecast> ptr,
                              py::array_t<int32_t, py::array::c_style | py::array::forcecast> idx,
                              py::array_t<float, py::array::c_style | py::array::forcecast> val) {
        sart::HostCsr a;
        a.nrows = nrows;
        a.ncols = ncols;
        a.ptr.assign(ptr.data(), ptr.data() + ptr.size());
        a.idx.assign(idx.data(), idx.data() + idx.size());
        a.val.assign(val.data(), val.data() + val.size());
        if ((int64_t)a.ptr.size() != nrows + 1 || a.idx.size() != a.val.size() || a.ptr.back() != (int64_t)a.val.size())
            throw py::value_error("csr_transpose: inconsistent CSR arrays");
        const sart::HostCsr t = sart::csr_transpose(a);
        return py::make_tuple(py::array_t<int64_t>(t.ptr.size(), t.ptr.data()),
                              py::array_t<int32_t>(t.idx.size(), t.idx.data()),
                              py::array_t<float>(t.val.size(), t.val.data()));
    });
    m.def("rtm_sparse_density", &rtm_sparse_density, py::arg("sorted_files"), py::arg("rtm_name"), py::arg("npixel"),
          py::arg("nvoxel"));
    // the RTM rows [r0, r1) of validated inputs as CSR (RtmReader::read_csr)
    m.def("read_rtm_csr", [](const std::vector<std::string>& files, const std::string& rtm_name, uint64_t r0, uint64_t r1) {
        const sart::InputSet in = sart::validate_inputs(files, rtm_name, 50.0);
        sart::RtmReader rd(in.rtm_files, rtm_name, in.nvoxel);
        const sart::HostCsr a = rd.read_csr(r0, r1);
        return py::make_tuple(py::array_t<int64_t>(a.ptr.size(), a.ptr.data()),
                              py::array_t<int32_t>(a.idx.size(), a.idx.data()),
                              py::array_t<float>(a.val.size(), a.val.data()), a.ncols);
    }, py::arg("files"), py::arg("rtm_name") = "with_reflections", py::arg("row_begin"), py::arg("row_end"));

    // one read of A per iteration (the --use_cpu sweep): returns (f, out, sum f^2)
    m.def("cpu_sweep", [](py::array_t<float, py::array::c_style> A, int64_t P, int64_t V, f64arr x, f64arr g, f64arr a,
                          bool logmode) {
        auto bi = A.request();
        check_rows(bi, P, V, bi.ndim == 2 ? bi.shape[1] : 0);
        if (x.size() < V || g.size() < P || a.size() < P) throw std::invalid_argument("vector too short");
        py::array_t<double> f(P), out(V);
        const float* ap = static_cast<const float*>(bi.ptr);
        const double *xp = x.data(), *gp = g.data(), *arow = a.data();
        double *fp = f.mutable_data(), *op = out.mutable_data();
        const int64_t ld = bi.shape[1];
        double f2;
        {
            py::gil_scoped_release nogil;
            f2 = cpu_sweep(ap, P, V, ld, xp, gp, arow, logmode, fp, op);
        }
        return py::make_tuple(f, out, f2);
    });

    // ---------------------------------------------------------------- fixture writers
    m.def(
        "write_rtm_file",
        [](std::string path, std::string camera, double wavelength, uint64_t npixel, uint64_t nvoxel, u8arr mask,
           u64arr vi, u64arr vj, u64arr vk, i32arr vvalue, uint64_t nx, uint64_t ny, uint64_t nz, py::object dense,
           py::object pix, py::object vox, py::object val, std::string rtm_name, std::string coordsys,
           std::vector<double> bounds) {
            RtmFileSpec s;
            s.path = path;
            s.camera_name = camera;
            s.wavelength = wavelength;
            s.npixel = npixel;
            s.nvoxel = nvoxel;
            auto mb = mask.request();
            if (mb.ndim != 2) throw std::invalid_argument("frame mask must be 2-D");
            s.frame_h = mb.shape[0];
            s.frame_w = mb.shape[1];
            s.frame_mask = vec(mask);
            s.vi = vec(vi);
            s.vj = vec(vj);
            s.vk = vec(vk);
            s.vvalue = vec(vvalue);
            s.nx = nx;
            s.ny = ny;
            s.nz = nz;
            s.rtm_name = rtm_name;
            s.coordinate_system = coordsys;
            s.bounds = bounds;
            if (!dense.is_none()) {
                s.sparse = false;
                s.value = vec(py::cast<f32arr>(dense));
            } else {
                s.sparse = true;
                s.pixel_index = vec(py::cast<u64arr>(pix));
                s.voxel_index = vec(py::cast<u64arr>(vox));
                s.value = vec(py::cast<f32arr>(val));
            }
            write_rtm_file(s);
        },
        py::arg("path"), py::arg("camera_name"), py::arg("wavelength"), py::arg("npixel"), py::arg("nvoxel"),
        py::arg("frame_mask"), py::arg("vi"), py::arg("vj"), py::arg("vk"), py::arg("vvalue"), py::arg("nx"),
        py::arg("ny"), py::arg("nz"), py::arg("dense") = py::none(), py::arg("pixel_index") = py::none(),
        py::arg("voxel_index") = py::none(), py::arg("value") = py::none(),
        py::arg("rtm_name") = "with_reflections", py::arg("coordinate_system") = "",
        py::arg("bounds") = std::vector<double>());
    m.def(
        "write_image_file",
        [](std::string path, std::string camera, double wavelength, f64arr time, f64arr frames) {
            auto fb = frames.request();
            if (fb.ndim != 3) throw std::invalid_argument("frames must be [T, H, W]");
            write_image_file(path, camera, wavelength, vec(time), vec(frames), fb.shape[1], fb.shape[2]);
        },
        py::arg("path"), py::arg("camera_name"), py::arg("wavelength"), py::arg("time"), py::arg("frames"));
    m.def(
        "write_synthetic_rtm_file",
        [](std::string path, std::string camera, double wavelength, uint64_t h, uint64_t w, uint64_t nvoxel,
           uint64_t seed, uint64_t nnz_per_row, bool drop_cache, uint64_t block_bytes, std::string rtm_name) {
            py::gil_scoped_release nogil;
            return write_synthetic_rtm_file(path, camera, wavelength, h, w, nvoxel, seed, nnz_per_row, drop_cache,
                                            block_bytes, rtm_name);
        },
        py::arg("path"), py::arg("camera_name"), py::arg("wavelength"), py::arg("h"), py::arg("w"), py::arg("nvoxel"),
        py::arg("seed") = 0, py::arg("nnz_per_row") = 0, py::arg("drop_cache") = false,
        py::arg("block_bytes") = (uint64_t)256 << 20, py::arg("rtm_name") = "with_reflections");
    m.def("synthetic_rtm_value", &synthetic_rtm_value, py::arg("seed"), py::arg("p"), py::arg("v"));
    m.def("synthetic_rtm_voxel", &synthetic_rtm_voxel, py::arg("p"), py::arg("k"), py::arg("nnz_per_row"),
          py::arg("nvoxel"));
    m.def("drop_file_cache", &drop_file_cache, py::arg("path"));
    m.def(
        "write_laplacian_file",
        [](std::string path, uint64_t nvoxel, u64arr i, u64arr j, f32arr v) {
            write_laplacian_file(path, nvoxel, vec(i), vec(j), vec(v));
        },
        py::arg("path"), py::arg("nvoxel"), py::arg("i"), py::arg("j"), py::arg("value"));

    // ---- host collectives and the CPU solver (the --use_cpu path)
    py::enum_<ReduceOp>(m, "ReduceOp", py::module_local()).value("SUM", ReduceOp::kSum).value("MAX", ReduceOp::kMax);
    py::class_<HostComm, std::shared_ptr<HostComm>>(m, "HostComm")
        .def_property_readonly("rank", &HostComm::rank)
        .def_property_readonly("size", &HostComm::size)
        .def_property_readonly("backend", &HostComm::backend)
        .def("barrier", &HostComm::barrier, py::call_guard<py::gil_scoped_release>())
        .def("broadcast_bytes",
             [](HostComm& c, py::bytes data, size_t nbytes, int root) {
                 std::string buf(nbytes, '\0');
                 if (c.rank() == root) {
                     const std::string d = data;
                     if (d.size() != nbytes) throw py::value_error("broadcast_bytes: root payload size mismatch");
                     buf = d;
                 }
                 {
                     py::gil_scoped_release rel;
                     c.broadcast_host(buf.data(), nbytes, root);
                 }
                 return py::bytes(buf);
             })
        .def("all_reduce_host", [](HostComm& c, f64arr v, ReduceOp op) {
            py::array_t<double> out(v.size());
            std::copy(v.data(), v.data() + v.size(), out.mutable_data());
            double* p = out.mutable_data();
            const size_t n = (size_t)v.size();
            {
                py::gil_scoped_release rel;
                c.all_reduce_host(p, n, op);
            }
            return out;
        })
        .def("all_reduce_host_f32", [](HostComm& c, py::array_t<float, py::array::c_style | py::array::forcecast> v,
                                       ReduceOp op) {
            py::array_t<float> out(v.size());
            std::copy(v.data(), v.data() + v.size(), out.mutable_data());
            float* p = out.mutable_data();
            const size_t n = (size_t)v.size();
            {
                py::gil_scoped_release rel;
                c.all_reduce_host(p, n, op);
            }
            return out;
        });
    m.def("local_host_comm", []() { return std::shared_ptr<HostComm>(make_local_host_comm()); });
    m.def("mpi_host_comm", []() { return std::shared_ptr<HostComm>(make_mpi_host_comm()); });
    m.def("mpi_library_version", &mpi_library_version);
    m.def("mpi_launch_detected", &mpi_launch_detected);
    m.def("tcp_host_comm",
          [](int rank, int size, const std::string& host, int port, double timeout_s) {
              py::gil_scoped_release rel;
              return std::shared_ptr<HostComm>(make_tcp_host_comm(rank, size, host, port, timeout_s));
          },
          py::arg("rank"), py::arg("size"), py::arg("host"), py::arg("port"), py::arg("timeout_s") = 3600.0);
    m.def("block_partition", [](uint64_t n, int parts, int part) {
        const Block b = block_partition(n, parts, part);
        return py::make_tuple(b.offset, b.size);
    });

    py::class_<SolverParams>(m, "SolverParams")
        .def(py::init<>())
        .def_readwrite("logarithmic", &SolverParams::logarithmic)
        .def_readwrite("ray_density_threshold", &SolverParams::ray_density_threshold)
        .def_readwrite("ray_length_threshold", &SolverParams::ray_length_threshold)
        .def_readwrite("conv_tolerance", &SolverParams::conv_tolerance)
        .def_readwrite("beta_laplace", &SolverParams::beta_laplace)
        .def_readwrite("relaxation", &SolverParams::relaxation)
        .def_readwrite("max_iterations", &SolverParams::max_iterations)
        .def_readwrite("allow_zero_tolerance", &SolverParams::allow_zero_tolerance);

    py::class_<CpuSolver>(m, "CpuSolver")
        .def(py::init([](py::array A, int64_t P, int64_t V, std::shared_ptr<HostComm> comm, const SolverParams& p,
                         bool gpu_semantics) {
                 py::buffer_info bi = A.request();
                 if (bi.format != py::format_descriptor<float>::format())
                     throw std::invalid_argument("A must be float32");
                 const int64_t ld = bi.ndim == 2 ? bi.shape[1] : V;
                 check_rows(bi, P, V, ld);
                 try {
                     return new CpuSolver(static_cast<const float*>(bi.ptr), P, V, ld, comm.get(), p, gpu_semantics);
                 } catch (const std::invalid_argument& e) {
                     throw py::value_error(e.what());
                 }
             }),
             py::keep_alive<1, 2>(), py::keep_alive<1, 5>())
        .def("set_laplacian",
             [](CpuSolver& s, int64_t n, py::array_t<int64_t, py::array::c_style | py::array::forcecast> rp,
                i32arr col, f32arr val) {
                 Csr c;
                 c.n = n;
                 c.row_ptr.assign(rp.data(), rp.data() + rp.size());
                 c.col.assign(col.data(), col.data() + col.size());
                 c.val.assign(val.data(), val.data() + val.size());
                 s.set_laplacian(c);
             })
        .def("solve",
             [](CpuSolver& s, f64arr g, py::object x0) {
                 f64arr x0a;
                 const double* x0p = nullptr;
                 if (!x0.is_none()) {
                     x0a = x0.cast<f64arr>();
                     x0p = x0a.data();
                 }
                 py::array_t<double> x(s.ray_density().size());
                 double* xp = x.mutable_data();
                 const double* gp = g.data();
                 SolveInfo info;
                 {
                     py::gil_scoped_release rel;
                     info = s.solve(gp, x0p, xp);
                 }
                 py::dict d;
                 d["status"] = info.status;
                 d["iterations"] = info.iterations;
                 d["convergence"] = info.convergence;
                 d["nonfinite"] = info.nonfinite;
                 d["ms"] = info.ms;
                 return py::make_tuple(x, d);
             },
             py::arg("g"), py::arg("x0") = py::none())
        .def("ray_density", [](const CpuSolver& s) { return arr(s.ray_density()); })
        .def("ray_length", [](const CpuSolver& s) { return arr(s.ray_length()); });
}
