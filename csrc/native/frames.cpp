#include "frames.hpp"

#include <algorithm>
#include <future>
#include <cmath>
#include <limits>
#include <numeric>
#include <sstream>

namespace sart {

namespace {
constexpr double kTimeEps = 1e-10;  // reference image.cpp:17
}

// =============================================================================================
// CompositeImage
// =============================================================================================
#ifdef SART_HAVE_HDF5

CompositeImage::CompositeImage(std::map<std::string, std::string> image_files,
                               std::map<std::string, std::vector<int32_t>> frame_masks,
                               const std::vector<std::array<double, 4>>& intervals, uint64_t npixel,
                               uint64_t offset_pixel)
    : files_(std::move(image_files)), masks_(std::move(frame_masks)), npix_(npixel), offset_(offset_pixel) {
    if (npix_ == 0) throw Error("Argument npixel must be positive.");
    SART_H5_LOCK;
    // timelines, cameras in name order (the map order of the mask dictionary)
    std::vector<std::vector<double>> timelines;
    for (const auto& [cam, mask] : masks_) {
        auto it = files_.find(cam);
        if (it == files_.end()) throw Error("No image file for " + cam + " camera.");
        H5Id f = h5_open_file(it->second);
        auto t = h5_read_f64(f, "image/time");
        if (!std::is_sorted(t.begin(), t.end())) throw Error("Image frames are not sorted by time in " + it->second + ".");
        timelines.push_back(std::move(t));
    }
    for (const auto& iv : intervals) {
        std::vector<std::vector<std::pair<double, uint64_t>>> sel(timelines.size());
        bool all = true;
        for (size_t c = 0; c < timelines.size(); ++c) {
            for (uint64_t n = 0; n < timelines[c].size(); ++n)
                if (timelines[c][n] >= iv[0] && timelines[c][n] <= iv[1]) sel[c].push_back({timelines[c][n], n});
            all &= !sel[c].empty();
        }
        // A camera without frames in the interval yields no composite frame there (the reference
        // dereferences front() of an empty selection, image.cpp:119-135).
        if (all && !sel.empty()) build_frames(sel, iv[2], iv[3]);
    }
    if (time_.empty()) throw Error("No composite images can be created for given time intervals.");
    cur_ = time_.size();
}

void CompositeImage::set_max_cache_size(uint64_t v) {
    if (v == 0) throw Error("Attribute max_cache_size must be positive.");
    max_cache_ = v;
}

void CompositeImage::build_frames(const std::vector<std::vector<std::pair<double, uint64_t>>>& sel, double step,
                                  double threshold) {
    double t_lo = sel.front().front().first, t_hi = sel.front().back().first;
    for (const auto& s : sel) {
        t_lo = std::min(t_lo, s.front().first);
        t_hi = std::max(t_hi, s.back().first);
    }
    if (step == 0) {
        if (t_hi - t_lo < kTimeEps) {
            step = 1.0;
        } else {
            // the largest per-camera minimal frame spacing (reference image.cpp:127-136)
            for (const auto& s : sel) {
                double dmin = s.back().first - s.front().first;
                for (size_t n = 1; n < s.size(); ++n) dmin = std::min(dmin, s[n].first - s[n - 1].first);
                step = std::max(step, dmin);
            }
            if (!(step > 0)) step = 1.0;  // every camera has a single frame
        }
    }
    if (threshold == 0) threshold = step;
    t_lo -= step;  // one empty grid point on both sides: no border checks below
    t_hi += step;
    const uint64_t ngrid = (uint64_t)std::llround((t_hi - t_lo) / step) + 1;
    const size_t ncam = sel.size();
    // best candidate per (grid point, camera): (signed offset from the grid time, frame index)
    std::vector<std::pair<double, uint64_t>> best(ngrid * ncam, {1.01 * threshold, 0});
    for (size_t c = 0; c < ncam; ++c) {
        for (const auto& [t, idx] : sel[c]) {
            const int64_t g0 = (int64_t)std::llround((t - t_lo) / step);
            for (int64_t g = g0 - 1; g <= g0 + 1; ++g) {
                if (g < 0 || (uint64_t)g >= ngrid) continue;
                auto& slot = best[(uint64_t)g * ncam + c];
                const double delta = t - t_lo - (double)g * step;
                // '+ eps' prefers the earlier frame when two are equally distant
                if (std::abs(delta) + kTimeEps < std::abs(slot.first)) slot = {delta, idx};
            }
        }
    }
    double last_delta = 0;
    for (uint64_t g = 1; g + 1 < ngrid; ++g) {
        const double tg = t_lo + (double)g * step;
        std::vector<uint64_t> idx;
        std::vector<double> ctime;
        double total = 0;
        for (size_t c = 0; c < ncam; ++c) {
            const auto& slot = best[g * ncam + c];
            if (std::abs(slot.first) > threshold + kTimeEps) break;
            idx.push_back(slot.second);
            ctime.push_back(tg + slot.first);
            total += std::abs(slot.first);
        }
        if (idx.size() != ncam) continue;
        if (indices_.empty() || idx != indices_.back()) {
            indices_.push_back(std::move(idx));
            camera_time_.push_back(std::move(ctime));
            time_.push_back(tg);
        } else if (total + kTimeEps < last_delta) {
            time_.back() = tg;  // same frames, closer grid point (camera times kept, as the reference)
        }
        last_delta = total;
    }
}

void CompositeImage::fill_cache(uint64_t first) {
    SART_H5_LOCK;
    const uint64_t count = std::min<uint64_t>(max_cache_, time_.size() - first);
    cache_.assign(count * npix_, 0.0);
    uint64_t start = 0;  // first global pixel of the current camera
    size_t c = 0;
    for (const auto& [cam, mask] : masks_) {
        const uint64_t nmasked = (uint64_t)std::count_if(mask.begin(), mask.end(), [](int32_t v) { return v != 0; });
        const uint64_t end = start + nmasked;
        if (end > offset_ && start < offset_ + npix_) {
            H5Id f = h5_open_file(files_.at(cam));
            H5Id d = h5_open_dataset(f, "image/frame");
            const auto dims = h5_dims(d);
            const uint64_t fsize = dims.size() == 3 ? dims[1] * dims[2] : 0;
            if (fsize != mask.size()) throw Error("Image frame of " + cam + " does not match its frame mask.");
            const uint64_t m0 = std::max(offset_, start) - start;        // masked-pixel range of this camera
            const uint64_t m1 = std::min(offset_ + npix_, end) - start;  // that falls into the local slice
            const uint64_t dst0 = start + m0 - offset_;
            std::vector<double> full(fsize);
            for (uint64_t n = 0; n < count; ++n) {
                h5_read_frame_f64(d, indices_[first + n][c], full.data(), fsize);
                double* dst = cache_.data() + n * npix_ + dst0;
                uint64_t m = 0;
                for (uint64_t p = 0; p < fsize && m < m1; ++p) {
                    if (!mask[p]) continue;
                    if (m >= m0) *dst++ = full[p];
                    ++m;
                }
            }
        }
        start = end;
        ++c;
        if (start >= offset_ + npix_) break;
    }
    cache_first_ = first;
    cache_count_ = count;
}

std::vector<double> CompositeImage::frame(uint64_t i) {
    if (i >= time_.size())
        throw Error("Index " + std::to_string(i) + " is out of bounds (" + std::to_string(time_.size()) + ").");
    if (!cached(i)) fill_cache(i);
    cur_ = i;
    const double* p = cache_.data() + (i - cache_first_) * npix_;
    return std::vector<double>(p, p + npix_);
}

bool CompositeImage::next_frame(std::vector<double>& out) {
    if (cur_ + 1 == time_.size()) return false;
    out = frame(cur_ == time_.size() ? 0 : cur_ + 1);
    return true;
}

double CompositeImage::frame_time(uint64_t i) const {
    if (i >= time_.size())
        throw Error("Index " + std::to_string(i) + " is out of bounds (" + std::to_string(time_.size()) + ").");
    return time_[i];
}

std::vector<double> CompositeImage::camera_frame_time(uint64_t i) const {
    if (i >= time_.size())
        throw Error("Index " + std::to_string(i) + " is out of bounds (" + std::to_string(time_.size()) + ").");
    return camera_time_[i];
}

// =============================================================================================
// SolutionWriter
// =============================================================================================
SolutionWriter::SolutionWriter(std::string filename, std::vector<std::string> camera_names, uint64_t nvoxel,
                               uint64_t max_cache_size, bool append)
    : filename_(std::move(filename)), cams_(std::move(camera_names)), nvox_(nvoxel), first_(!append) {
    if (nvox_ == 0) throw Error("Argument nvoxel must be positive.");
    set_max_cache_size(max_cache_size);
    cache_.cam_times.resize(cams_.size());
}

SolutionWriter::~SolutionWriter() {
    try {
        flush();
    } catch (...) {
    }
}

void SolutionWriter::set_max_cache_size(uint64_t v) {
    if (v == 0) throw Error("Attribute max_cache_size must be positive.");
    max_cache_ = v;
}

void SolutionWriter::add(const std::vector<double>& solution, int32_t status, double time,
                         const std::vector<double>& camera_time, int32_t iterations) {
    if (solution.size() != nvox_) throw Error("Solution vector must contain nvoxel elements.");
    if (camera_time.size() != cams_.size()) throw Error("One time stamp per camera is required.");
    cache_.solutions.push_back(solution);
    cache_.status.push_back(status);
    cache_.times.push_back(time);
    cache_.iterations.push_back(iterations);
    for (size_t c = 0; c < cams_.size(); ++c) cache_.cam_times[c].push_back(camera_time[c]);
    if (cache_.times.size() >= max_cache_) {  // write in the background (the previous write first)
        if (pending_.valid()) pending_.get();
        pending_ = std::async(std::launch::async, [this, b = take()]() { write(b); });
    }
}

SolutionWriter::Batch SolutionWriter::take() {
    Batch b = std::move(cache_);
    cache_ = Batch{};
    cache_.cam_times.resize(cams_.size());
    return b;
}

namespace {
H5Id create_ext_1d(hid_t grp, const std::string& name, hid_t ftype, hsize_t n, hsize_t chunk) {
    hsize_t dims = n, maxd = H5S_UNLIMITED;
    H5Id sp(H5Screate_simple(1, &dims, &maxd), H5Id::kSpace);
    H5Id pl(H5Pcreate(H5P_DATASET_CREATE), H5Id::kPlist);
    hsize_t ch = std::max<hsize_t>(1, chunk);
    H5Pset_chunk(pl, 1, &ch);
    H5Id ds(H5Dcreate2(grp, name.c_str(), ftype, sp, H5P_DEFAULT, pl, H5P_DEFAULT), H5Id::kDataset);
    if (!ds.valid()) throw Error("Unable to create dataset solution/" + name + ".");
    return ds;
}

void write_1d_at(hid_t ds, hid_t mtype, hsize_t offset, hsize_t n, const void* data) {
    hsize_t newsize = offset + n;
    if (H5Dset_extent(ds, &newsize) < 0) throw Error("Unable to extend a solution dataset.");
    H5Id fsp(H5Dget_space(ds), H5Id::kSpace);
    H5Sselect_hyperslab(fsp, H5S_SELECT_SET, &offset, nullptr, &n, nullptr);
    H5Id msp(H5Screate_simple(1, &n, nullptr), H5Id::kSpace);
    if (H5Dwrite(ds, mtype, msp, fsp, H5P_DEFAULT, data) < 0) throw Error("Unable to write a solution dataset.");
}
}  // namespace

void SolutionWriter::create(uint64_t chunk) {
    SART_H5_LOCK;
    H5Id f = h5_create_file(filename_);
    H5Id g = h5_create_group(f, "solution");
    const hsize_t n = chunk;
    {
        hsize_t dims[2] = {0, nvox_}, maxd[2] = {H5S_UNLIMITED, nvox_}, ch[2] = {1, nvox_};
        H5Id sp(H5Screate_simple(2, dims, maxd), H5Id::kSpace);
        H5Id pl(H5Pcreate(H5P_DATASET_CREATE), H5Id::kPlist);
        H5Pset_chunk(pl, 2, ch);
        double fill = 0;
        H5Pset_fill_value(pl, H5T_NATIVE_DOUBLE, &fill);
        H5Id ds(H5Dcreate2(g, "value", H5T_IEEE_F64LE, sp, H5P_DEFAULT, pl, H5P_DEFAULT), H5Id::kDataset);
        if (!ds.valid()) throw Error("Unable to create dataset solution/value.");
    }
    create_ext_1d(g, "time", H5T_IEEE_F64LE, 0, n);
    for (const auto& cam : cams_) create_ext_1d(g, "time_" + cam, H5T_IEEE_F64LE, 0, n);
    create_ext_1d(g, "status", H5T_STD_I32LE, 0, n);
    create_ext_1d(g, "iterations", H5T_STD_I32LE, 0, n);  // extension: SART updates per frame
}

void SolutionWriter::append(const Batch& b) {
    SART_H5_LOCK;
    H5Id f = h5_open_file(filename_, true);
    H5Id tds = h5_open_dataset(f, "solution/time");
    const hsize_t off = h5_dims(tds)[0];
    const hsize_t n = b.times.size();
    write_1d_at(tds, H5T_NATIVE_DOUBLE, off, n, b.times.data());
    {
        H5Id ds = h5_open_dataset(f, "solution/status");
        write_1d_at(ds, H5T_NATIVE_INT32, off, n, b.status.data());
    }
    if (h5_exists(f, "solution/iterations")) {
        H5Id ds = h5_open_dataset(f, "solution/iterations");
        write_1d_at(ds, H5T_NATIVE_INT32, off, n, b.iterations.data());
    }
    for (size_t c = 0; c < cams_.size(); ++c) {
        H5Id ds = h5_open_dataset(f, "solution/time_" + cams_[c]);
        write_1d_at(ds, H5T_NATIVE_DOUBLE, off, n, b.cam_times[c].data());
    }
    H5Id vds = h5_open_dataset(f, "solution/value");
    hsize_t newsize[2] = {off + n, nvox_};
    if (H5Dset_extent(vds, newsize) < 0) throw Error("Unable to extend solution/value.");
    H5Id fsp(H5Dget_space(vds), H5Id::kSpace);
    hsize_t m = nvox_;
    H5Id msp(H5Screate_simple(1, &m, nullptr), H5Id::kSpace);
    for (hsize_t r = 0; r < n; ++r) {
        hsize_t o[2] = {off + r, 0}, c[2] = {1, nvox_};
        H5Sselect_hyperslab(fsp, H5S_SELECT_SET, o, nullptr, c, nullptr);
        if (H5Dwrite(vds, H5T_NATIVE_DOUBLE, msp, fsp, H5P_DEFAULT, b.solutions[r].data()) < 0)
            throw Error("Unable to write solution/value.");
    }
}

void SolutionWriter::write(const Batch& b) {
    SART_H5_LOCK;
    if (b.times.empty()) return;
    if (first_) create(b.times.size());  // (the reference: chunk size = the first flush's size, solution.cpp:91)
    first_ = false;
    append(b);
}

void SolutionWriter::flush() {
    if (pending_.valid()) pending_.get();  // the background write first (rethrows its error)
    write(take());
}

StoredSolutions read_solution_file(const std::string& filename) {
    SART_H5_LOCK;
    StoredSolutions out;
    h5_quiet();
    if (H5Fis_hdf5(filename.c_str()) <= 0) return out;
    H5Id f = h5_open_file(filename);
    if (!h5_exists(f, "solution/time")) return out;
    out.time = h5_read_f64(f, "solution/time");
    out.status = h5_read_i32(f, "solution/status");
    if (!out.time.empty()) {
        H5Id vds = h5_open_dataset(f, "solution/value");
        const auto dims = h5_dims(vds);
        out.last_solution.resize(dims[1]);
        H5Id fsp(H5Dget_space(vds), H5Id::kSpace);
        hsize_t o[2] = {dims[0] - 1, 0}, c[2] = {1, dims[1]};
        H5Sselect_hyperslab(fsp, H5S_SELECT_SET, o, nullptr, c, nullptr);
        hsize_t m = dims[1];
        H5Id msp(H5Screate_simple(1, &m, nullptr), H5Id::kSpace);
        H5Dread(vds, H5T_NATIVE_DOUBLE, msp, fsp, H5P_DEFAULT, out.last_solution.data());
    }
    return out;
}

// =============================================================================================
// VoxelGrid
// =============================================================================================
int VoxelGrid::coordinate_system(const std::string& filename, const std::string& group) {
    SART_H5_LOCK;
    H5Id f = h5_open_file(filename);
    if (!h5_attr_exists(f, group, "coordinate_system")) return kCartesian;
    std::string cs = h5_attr_string(f, group, "coordinate_system");
    std::transform(cs.begin(), cs.end(), cs.begin(), [](unsigned char c) { return (char)std::tolower(c); });
    return cs == "cylindrical" ? kCylindrical : kCartesian;
}

void VoxelGrid::read(const std::vector<std::string>& filenames, const std::string& group) {
    SART_H5_LOCK;
    if (filenames.empty()) throw Error("VoxelGrid::read needs at least one file.");
    coordsys = coordinate_system(filenames.front(), group);
    {
        H5Id f = h5_open_file(filenames.front());
        nx = h5_attr_u64(f, group, "nx");
        ny = h5_attr_u64(f, group, "ny");
        nz = h5_attr_u64(f, group, "nz");
        auto opt = [&](const char* name, double dflt) {
            return h5_attr_exists(f, group, name) ? h5_attr_double(f, group, name) : dflt;
        };
        xmin = opt("xmin", 0);
        xmax = opt("xmax", 1);
        ymin = opt("ymin", 0);
        ymax = opt("ymax", 1);
        zmin = opt("zmin", 0);
        zmax = opt("zmax", 1);
    }
    voxmap.assign(nx * ny * nz, -1);
    int64_t offset = 0;
    for (const auto& path : filenames) {
        H5Id f = h5_open_file(path);
        const auto i = h5_read_u64(f, group + "/i");
        const auto j = h5_read_u64(f, group + "/j");
        const auto k = h5_read_u64(f, group + "/k");
        const auto v = h5_read_i64(f, group + "/value");
        int64_t vmax = -1;
        for (size_t n = 0; n < v.size(); ++n) {
            const uint64_t flat = i[n] * ny * nz + j[n] * nz + k[n];
            if (flat >= voxmap.size()) throw Error("Voxel map index out of range in " + path + ".");
            voxmap[flat] = (int32_t)(v[n] + offset);
            vmax = std::max(vmax, v[n]);
        }
        // segment offsets follow the rtm/nvoxel attribute (the solver's column layout); the
        // reference derives them from max(value) + 1 (voxelgrid.cpp:94-96), equal for valid files
        const std::string rtm_group = group.substr(0, group.rfind('/'));
        if (!rtm_group.empty() && rtm_group != group && h5_attr_exists(f, rtm_group, "nvoxel"))
            offset += h5_attr_i64(f, rtm_group, "nvoxel");
        else
            offset += vmax + 1;
    }
    nvox = (uint64_t)offset;
    if (coordsys == kCylindrical && std::fmod(360.0, ymax - ymin) > 0.001) {
        std::ostringstream os;
        os << (ymax - ymin) << " is not a divisor of 360.";
        warnings.push_back(os.str());
    }
}

void VoxelGrid::write(const std::string& filename, const std::string& group) const {
    SART_H5_LOCK;
    H5Id f = h5_open_file(filename, true);
    H5Id g = h5_create_group(f, group);
    h5_write_attr_u64(g, "nx", nx);
    h5_write_attr_u64(g, "ny", ny);
    h5_write_attr_u64(g, "nz", nz);
    h5_write_attr_double(g, "xmin", xmin);
    h5_write_attr_double(g, "xmax", xmax);
    h5_write_attr_double(g, "ymin", ymin);
    h5_write_attr_double(g, "ymax", ymax);
    h5_write_attr_double(g, "zmin", zmin);
    h5_write_attr_double(g, "zmax", zmax);
    h5_write_attr_string(g, "coordinate_system", coordsys == kCylindrical ? "cylindrical" : "cartesian");
    std::vector<int32_t> ii, jj, kk, vv;
    for (uint64_t flat = 0; flat < voxmap.size(); ++flat) {
        if (voxmap[flat] < 0) continue;
        ii.push_back((int32_t)(flat / (ny * nz)));
        jj.push_back((int32_t)((flat % (ny * nz)) / nz));
        kk.push_back((int32_t)(flat % nz));
        vv.push_back(voxmap[flat]);
    }
    const std::vector<uint64_t> dims = {ii.size()};
    h5_write_i32(g, "i", dims, ii.data());
    h5_write_i32(g, "j", dims, jj.data());
    h5_write_i32(g, "k", dims, kk.data());
    h5_write_i32(g, "value", dims, vv.data());
}

#endif  // SART_HAVE_HDF5

int32_t VoxelGrid::voxel_index(uint64_t i, uint64_t j, uint64_t k) const {
    if (i >= nx || j >= ny || k >= nz) return -1;
    return voxmap[i * ny * nz + j * nz + k];
}

int32_t VoxelGrid::voxel_index_at(double x, double y, double z) const {
    if (voxmap.empty()) throw Error("Voxel map is not initialized.");
    const double dx = (xmax - xmin) / nx, dy = (ymax - ymin) / ny, dz = (zmax - zmin) / nz;
    double a = x, b = y;
    if (coordsys == kCylindrical) {
        a = std::sqrt(x * x + y * y);
        const double period = ymax - ymin;
        double phi = 180.0 / M_PI * std::atan2(y, x);
        if (phi < 0) phi += 360.0;
        b = std::fmod(phi, period);
        if (a < xmin || a >= xmax || z < zmin || z >= zmax) return -1;
    } else if (x < xmin || x >= xmax || y < ymin || y >= ymax || z < zmin || z >= zmax) {
        return -1;
    }
    const uint64_t i = (uint64_t)((a - xmin) / dx), j = (uint64_t)((b - ymin) / dy), k = (uint64_t)((z - zmin) / dz);
    return voxel_index(i, j, k);
}

}  // namespace sart
