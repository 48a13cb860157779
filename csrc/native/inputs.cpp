#include "inputs.hpp"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <omp.h>
#include <cstdlib>
#include <cmath>
#include <limits>
#include <numeric>
#include <sstream>

namespace sart {

#ifdef SART_HAVE_HDF5

namespace {

std::string fmt_double(double v) {
    std::ostringstream os;
    os << v;
    return os.str();
}

struct VoxelMapData {
    uint64_t nx = 0, ny = 0, nz = 0;
    std::vector<uint64_t> i, j, k;
};

VoxelMapData read_voxel_map_indices(hid_t f) {
    VoxelMapData m;
    m.nx = h5_attr_u64(f, "rtm/voxel_map", "nx");
    m.ny = h5_attr_u64(f, "rtm/voxel_map", "ny");
    m.nz = h5_attr_u64(f, "rtm/voxel_map", "nz");
    m.i = h5_read_u64(f, "rtm/voxel_map/i");
    m.j = h5_read_u64(f, "rtm/voxel_map/j");
    m.k = h5_read_u64(f, "rtm/voxel_map/k");
    if (m.j.size() != m.i.size() || m.k.size() != m.i.size()) throw Error("Inconsistent voxel map index arrays.");
    return m;
}

}  // namespace

void categorize_input_files(const std::vector<std::string>& input_files, std::vector<std::string>& rtm_files,
                            std::vector<std::string>& image_files) {
    SART_H5_LOCK;
    for (const auto& path : input_files) {
        H5Id f = h5_open_file(path);
        if (h5_exists(f, "rtm"))
            rtm_files.push_back(path);
        else if (h5_exists(f, "image"))
            image_files.push_back(path);
        else
            throw Error("The file " + path + " is neither an RTM file nor an image file.");
    }
}

void check_group_attribute_consistency(const std::vector<std::string>& files, const std::string& group,
                                       const std::vector<std::string>& names, bool integer) {
    SART_H5_LOCK;
    if (files.empty()) return;
    std::vector<double> ref_d(names.size());
    std::vector<uint64_t> ref_u(names.size());
    {
        H5Id f = h5_open_file(files.front());
        for (size_t a = 0; a < names.size(); ++a) {
            if (integer)
                ref_u[a] = h5_attr_u64(f, group, names[a]);
            else
                ref_d[a] = h5_attr_double(f, group, names[a]);
        }
    }
    for (size_t n = 1; n < files.size(); ++n) {
        H5Id f = h5_open_file(files[n]);
        for (size_t a = 0; a < names.size(); ++a) {
            bool same;
            std::string sv, sr;
            if (integer) {
                const uint64_t v = h5_attr_u64(f, group, names[a]);
                same = v == ref_u[a];
                sv = std::to_string(v);
                sr = std::to_string(ref_u[a]);
            } else {
                const double v = h5_attr_double(f, group, names[a]);
                same = v == ref_d[a];
                sv = fmt_double(v);
                sr = fmt_double(ref_d[a]);
            }
            if (!same)
                throw Error("Different " + names[a] + " values in " + files[n] + " (" + sv + ") and in " +
                            files.front() + " (" + sr + ").");
        }
    }
}

SortedRtmFiles sort_rtm_files(const std::vector<std::string>& files) {
    SART_H5_LOCK;
    std::map<std::string, std::map<uint64_t, std::string>> by_camera;
    for (const auto& path : files) {
        H5Id f = h5_open_file(path);
        const std::string cam = h5_attr_string(f, "rtm", "camera_name");
        const VoxelMapData m = read_voxel_map_indices(f);
        uint64_t imin = m.nx * m.ny * m.nz;
        for (size_t n = 0; n < m.i.size(); ++n) imin = std::min(imin, m.i[n] * m.ny * m.nz + m.j[n] * m.nz + m.k[n]);
        by_camera[cam][imin] = path;
    }
    SortedRtmFiles out;
    for (auto& [cam, segs] : by_camera) {
        auto& v = out[cam];
        for (auto& [key, path] : segs) v.push_back(path);
    }
    return out;
}

void check_rtm_frame_consistency(const SortedRtmFiles& sorted) {
    SART_H5_LOCK;
    for (const auto& [cam, files] : sorted) {
        if (files.size() < 2) continue;
        std::vector<int32_t> ref;
        std::vector<hsize_t> ref_dims;
        for (size_t n = 0; n < files.size(); ++n) {
            H5Id f = h5_open_file(files[n]);
            H5Id d = h5_open_dataset(f, "rtm/frame_mask");
            const auto dims = h5_dims(d);
            auto mask = h5_read_i32(f, "rtm/frame_mask");
            if (n == 0) {
                ref = std::move(mask);
                ref_dims = dims;
            } else if (mask != ref || dims != ref_dims) {
                throw Error("RTM files for " + cam + " view have different frame masks.");
            }
        }
    }
}

void check_rtm_voxel_consistency(const SortedRtmFiles& sorted) {
    SART_H5_LOCK;
    std::vector<int64_t> ref_map;
    std::string ref_cam;
    for (const auto& [cam, files] : sorted) {
        uint64_t nx, ny, nz;
        {
            H5Id f0 = h5_open_file(files.front());
            nx = h5_attr_u64(f0, "rtm/voxel_map", "nx");
            ny = h5_attr_u64(f0, "rtm/voxel_map", "ny");
            nz = h5_attr_u64(f0, "rtm/voxel_map", "nz");
        }
        std::vector<int64_t> vmap(nx * ny * nz, -1);
        int64_t offset = 0;
        for (const auto& path : files) {
            H5Id f = h5_open_file(path);
            const int64_t nvox = h5_attr_i64(f, "rtm", "nvoxel");
            const VoxelMapData m = read_voxel_map_indices(f);
            const auto value = h5_read_i64(f, "rtm/voxel_map/value");
            if (value.size() != m.i.size()) throw Error("Inconsistent voxel map value array in " + path + ".");
            for (size_t n = 0; n < m.i.size(); ++n) {
                const uint64_t flat = m.i[n] * ny * nz + m.j[n] * nz + m.k[n];
                if (flat >= vmap.size()) throw Error("Voxel map index out of range in " + path + ".");
                if (vmap[flat] >= 0)
                    throw Error("RTM segments for " + cam + " view have overlapping voxel maps at element (" +
                                std::to_string(m.i[n]) + "," + std::to_string(m.j[n]) + "," +
                                std::to_string(m.k[n]) + ").");
                vmap[flat] = value[n] + offset;
            }
            offset += nvox;
        }
        if (ref_map.empty() && ref_cam.empty()) {
            ref_map = std::move(vmap);
            ref_cam = cam;
        } else if (vmap != ref_map) {
            throw Error("RTM files for " + cam + " and " + ref_cam + " views have different voxel maps.");
        }
    }
}

std::map<std::string, std::vector<int32_t>> read_rtm_frame_masks(const SortedRtmFiles& sorted) {
    SART_H5_LOCK;
    std::map<std::string, std::vector<int32_t>> out;
    for (const auto& [cam, files] : sorted) {
        H5Id f = h5_open_file(files.front());
        out[cam] = h5_read_i32(f, "rtm/frame_mask");
    }
    return out;
}

std::map<std::string, std::pair<uint64_t, uint64_t>> read_rtm_frame_shapes(const SortedRtmFiles& sorted) {
    SART_H5_LOCK;
    std::map<std::string, std::pair<uint64_t, uint64_t>> out;
    for (const auto& [cam, files] : sorted) {
        H5Id f = h5_open_file(files.front());
        H5Id d = h5_open_dataset(f, "rtm/frame_mask");
        const auto dims = h5_dims(d);
        if (dims.size() != 2) throw Error("rtm/frame_mask must be 2-D in " + files.front() + ".");
        out[cam] = {dims[0], dims[1]};
    }
    return out;
}

SortedImageFiles sort_image_files(const std::vector<std::string>& files) {
    SART_H5_LOCK;
    SortedImageFiles out;
    for (const auto& path : files) {
        H5Id f = h5_open_file(path);
        const std::string cam = h5_attr_string(f, "image", "camera_name");
        auto it = out.find(cam);
        if (it != out.end())
            throw Error("Image files " + path + " and " + it->second + " share the same diagnostic view: " + cam + ".");
        out[cam] = path;
    }
    return out;
}

void check_rtm_image_consistency(const SortedRtmFiles& rtm, const SortedImageFiles& images,
                                 const std::string& rtm_name, double wavelength_threshold) {
    SART_H5_LOCK;
    for (const auto& kv : rtm)
        if (!images.count(kv.first)) throw Error("No image file for " + kv.first + " camera.");
    for (const auto& kv : images)
        if (!rtm.count(kv.first)) throw Error("No RTM file for " + kv.first + " camera.");
    if (rtm.empty()) return;
    {
        H5Id rf = h5_open_file(rtm.begin()->second.front());
        H5Id imf = h5_open_file(images.begin()->second);
        const double rw = h5_attr_double(rf, "rtm/" + rtm_name, "wavelength");
        const double iw = h5_attr_double(imf, "image", "wavelength");
        if (std::abs(rw - iw) > wavelength_threshold)
            throw Error("RTM wavelength (" + fmt_double(rw) + " nm) is not within " + fmt_double(wavelength_threshold) +
                        " nm threshold from image wavelength (" + fmt_double(iw) + " nm).");
    }
    for (const auto& [cam, files] : rtm) {
        H5Id rf = h5_open_file(files.front());
        H5Id md = h5_open_dataset(rf, "rtm/frame_mask");
        const auto mdims = h5_dims(md);
        H5Id imf = h5_open_file(images.at(cam));
        H5Id fd = h5_open_dataset(imf, "image/frame");
        const auto fdims = h5_dims(fd);
        if (mdims.size() != 2 || fdims.size() != 3 || fdims[1] != mdims[0] || fdims[2] != mdims[1]) {
            const auto s = [](const std::vector<hsize_t>& d, size_t a, size_t b) {
                return (d.size() > std::max(a, b)) ? std::to_string(d[b]) + "x" + std::to_string(d[a]) : std::string("?");
            };
            throw Error("RTM for " + cam + " view was calculated for resolution " + s(mdims, 0, 1) +
                        ", but the camera image has resolution " + s(fdims, 1, 2) + ".");
        }
    }
}

std::pair<uint64_t, uint64_t> get_total_rtm_size(const SortedRtmFiles& sorted) {
    SART_H5_LOCK;
    uint64_t npixel = 0, nvoxel = 0;
    for (const auto& [cam, files] : sorted) {
        H5Id f = h5_open_file(files.front());
        npixel += h5_attr_u64(f, "rtm", "npixel");
    }
    if (!sorted.empty())
        for (const auto& path : sorted.begin()->second) {
            H5Id f = h5_open_file(path);
            nvoxel += h5_attr_u64(f, "rtm", "nvoxel");
        }
    return {npixel, nvoxel};
}

bool rtm_has_sparse(const SortedRtmFiles& sorted, const std::string& rtm_name) {
    SART_H5_LOCK;
    for (const auto& [cam, files] : sorted)
        for (const auto& path : files) {
            H5Id f = h5_open_file(path);
            if (h5_attr_i64(f, "rtm/" + rtm_name, "is_sparse")) return true;
        }
    return false;
}

double rtm_sparse_density(const SortedRtmFiles& sorted, const std::string& rtm_name, uint64_t npixel,
                          uint64_t nvoxel) {
    SART_H5_LOCK;
    double entries = 0.0;
    for (const auto& [cam, files] : sorted)
        for (const auto& path : files) {
            H5Id f = h5_open_file(path);
            if (!h5_attr_i64(f, "rtm/" + rtm_name, "is_sparse")) return -1.0;
            H5Id d = h5_open_dataset(f, "rtm/" + rtm_name + "/value");
            const auto dims = h5_dims(d);
            entries += dims.empty() ? 0.0 : (double)dims[0];
        }
    return npixel && nvoxel ? entries / ((double)npixel * (double)nvoxel) : -1.0;
}

RtmReader::RtmReader(SortedRtmFiles sorted, std::string rtm_name, uint64_t nvoxel, uint64_t col_begin,
                     uint64_t col_end)
    : sorted_(std::move(sorted)), name_(std::move(rtm_name)), nvoxel_(nvoxel), c0_(col_begin),
      c1_(col_end == 0 ? nvoxel : col_end) {
    if (c0_ > c1_ || c1_ > nvoxel_) throw Error("RtmReader: column window outside [0, nvoxel)");
}

const RtmReader::SparseSegment& RtmReader::sparse_segment(int64_t f, const std::string& path, uint64_t nvox_seg) {
    auto it = sparse_.find(path);
    if (it != sparse_.end()) return it->second;
    // read the COO arrays of this segment ONCE and order them by pixel, so every row block finds its
    // entries with a binary search (the reference re-reads and filters the whole arrays per shard,
    // raytransfer.cpp:67-91; a per-block re-read would cost O(blocks x nnz))
    const std::string grp = "rtm/" + name_;
    const auto pix = h5_read_u64(f, grp + "/pixel_index");
    const auto vox = h5_read_u64(f, grp + "/voxel_index");
    const auto val = h5_read_f32(f, grp + "/value");
    if (pix.size() != val.size() || vox.size() != val.size())
        throw Error("Inconsistent sparse RTM arrays in " + path + ".");
    std::vector<size_t> order(val.size());
    for (size_t n = 0; n < order.size(); ++n) {
        if (vox[n] >= nvox_seg) throw Error("Sparse RTM voxel index out of range in " + path + ".");
        order[n] = n;
    }
    std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return pix[a] < pix[b]; });
    SparseSegment seg;
    seg.pix.reserve(order.size());
    seg.vox.reserve(order.size());
    seg.val.reserve(order.size());
    for (size_t n : order) {
        seg.pix.push_back(pix[n]);
        seg.vox.push_back(vox[n]);
        seg.val.push_back(val[n]);
    }
    return sparse_.emplace(path, std::move(seg)).first->second;
}

void RtmReader::read(uint64_t row_begin, uint64_t row_end, float* out, uint64_t ld) {
    SART_H5_LOCK;
    if (row_end <= row_begin) return;
    if (ld < c1_ - c0_) throw Error("read_rtm_rows: ld smaller than the column window");
    const std::string grp = "rtm/" + name_;
    uint64_t start_pixel = 0;
    for (const auto& [cam, files] : sorted_) {
        uint64_t npix;
        {
            H5Id f0 = h5_open_file(files.front());
            npix = h5_attr_u64(f0, "rtm", "npixel");
        }
        const uint64_t cam_end = start_pixel + npix;
        if (cam_end > row_begin && start_pixel < row_end) {
            const uint64_t lr0 = std::max(row_begin, start_pixel) - start_pixel;  // camera-local rows
            const uint64_t lr1 = std::min(row_end, cam_end) - start_pixel;
            uint64_t start_voxel = 0;
            for (const auto& path : files) {
                H5Id f = h5_open_file(path);
                const uint64_t nvox_seg = h5_attr_u64(f, "rtm", "nvoxel");
                if (start_voxel + nvox_seg > nvoxel_) throw Error("RTM segments exceed the total number of voxels.");
                // this segment's columns inside the window [c0, c1): segment-local [s0, s1)
                const uint64_t s0 = std::max(c0_, start_voxel) - start_voxel;
                const uint64_t s1 = std::min(c1_, start_voxel + nvox_seg) > start_voxel
                                        ? std::min(c1_, start_voxel + nvox_seg) - start_voxel
                                        : 0;
                if (s1 > s0) {
                    const uint64_t ocol = start_voxel + s0 - c0_;  // output column of segment column s0
                    if (h5_attr_i64(f, grp, "is_sparse")) {
                        const SparseSegment& seg = sparse_segment(f, path, nvox_seg);
                        auto lo = std::lower_bound(seg.pix.begin(), seg.pix.end(), lr0);
                        auto hi = std::lower_bound(lo, seg.pix.end(), lr1);
                        for (size_t n = (size_t)(lo - seg.pix.begin()); n < (size_t)(hi - seg.pix.begin()); ++n) {
                            const uint64_t v = seg.vox[n];
                            if (v < s0 || v >= s1) continue;
                            const uint64_t row = start_pixel + seg.pix[n] - row_begin;
                            out[row * ld + ocol + (v - s0)] = seg.val[n];
                        }
                    } else {
                        H5Id d = h5_open_dataset(f, grp + "/value");
                        const auto dims = h5_dims(d);
                        if (dims.size() != 2 || dims[0] != npix || dims[1] != nvox_seg)
                            throw Error("Dense RTM dataset in " + path + " has unexpected shape.");
                        // row blocks of <= 64 MiB per hyperslab read, only the window's columns (the reference
                        // reads one whole row per call, raytransfer.cpp:103-109)
                        const uint64_t nc = s1 - s0;
                        const uint64_t rows_per_read =
                            rows_per_read_ ? rows_per_read_ : std::max<uint64_t>(1, (64ull << 20) / (4 * nc));
                        for (uint64_t r = lr0; r < lr1; r += rows_per_read) {
                            const uint64_t n = std::min(rows_per_read, lr1 - r);
                            h5_read_block_f32(d, r, n, s0, nc, out + (start_pixel + r - row_begin) * ld, ld, ocol);
                        }
                    }
                }
                start_voxel += nvox_seg;
            }
        }
        start_pixel = cam_end;
        if (start_pixel >= row_end) break;
    }
}

void read_rtm_rows(const SortedRtmFiles& sorted, const std::string& rtm_name, uint64_t nvoxel, uint64_t row_begin,
                   uint64_t row_end, float* out, uint64_t ld) {
    RtmReader(sorted, rtm_name, nvoxel).read(row_begin, row_end, out, ld);
}

// Bounded-memory CSR reader. Camera by camera (cameras own disjoint row ranges), every voxel segment becomes a CSR
// over the camera's rows of the shard: sparse (COO) datasets by a count pass and a fill pass over hyperslab chunks
// of the three arrays (SART_COO_CHUNK entries, default 1M: 20 MB of buffers) keeping only this shard's rows and
// window columns -- no whole-array read, no global sort, no cache (the reference reads every array whole per rank,
// raytransfer.cpp:67-91) -- and dense datasets from the non-zeros of row blocks. A row's entries are then ordered by
// column (stable: the file order of an entry repeated at the same (row, col) is kept and the LAST one wins, exact
// zeros dropped: csr_from_entries' semantics) and the camera's segments are concatenated row by row (their columns are
// disjoint and ascending). Peak host memory: the CSR built so far plus the current camera's segments (<= 2x the CSR).
HostCsr RtmReader::read_csr(uint64_t row_begin, uint64_t row_end) {
    SART_H5_LOCK;
    const uint64_t nrows = row_end > row_begin ? row_end - row_begin : 0, ncols = c1_ - c0_;
    if (ncols > (uint64_t)INT32_MAX) throw Error("read_csr: more than 2^31 - 1 columns");
    HostCsr out;
    out.nrows = (int64_t)nrows;
    out.ncols = (int64_t)ncols;
    out.ptr.assign(nrows + 1, 0);
    uint64_t chunk = 1ull << 20;
    if (const char* e = std::getenv("SART_COO_CHUNK"); e && *e && std::atoll(e) > 0) chunk = (uint64_t)std::atoll(e);
    const std::string grp = "rtm/" + name_;
    uint64_t start_pixel = 0;
    for (const auto& [cam, files] : sorted_) {
        if (nrows == 0) break;
        uint64_t npix;
        {
            H5Id f0 = h5_open_file(files.front());
            npix = h5_attr_u64(f0, "rtm", "npixel");
        }
        const uint64_t cam_end = start_pixel + npix;
        if (cam_end > row_begin && start_pixel < row_end) {
            const uint64_t lr0 = std::max(row_begin, start_pixel) - start_pixel;
            const uint64_t lr1 = std::min(row_end, cam_end) - start_pixel;
            const uint64_t nr = lr1 - lr0, orow = start_pixel + lr0 - row_begin;  // camera rows, first output row
            std::vector<HostCsr> segs;
            uint64_t start_voxel = 0;
            for (const auto& path : files) {
                H5Id f = h5_open_file(path);
                const uint64_t nvox_seg = h5_attr_u64(f, "rtm", "nvoxel");
                if (start_voxel + nvox_seg > nvoxel_) throw Error("RTM segments exceed the total number of voxels.");
                const uint64_t s0 = std::max(c0_, start_voxel) - start_voxel;
                const uint64_t s1 = std::min(c1_, start_voxel + nvox_seg) > start_voxel
                                        ? std::min(c1_, start_voxel + nvox_seg) - start_voxel
                                        : 0;
                if (s1 > s0) {
                    const uint64_t ocol = start_voxel + s0 - c0_;
                    HostCsr seg;
                    seg.nrows = (int64_t)nr;
                    seg.ncols = (int64_t)ncols;
                    seg.ptr.assign(nr + 1, 0);
                    if (h5_attr_i64(f, grp, "is_sparse")) {
                        H5Id dp = h5_open_dataset(f, grp + "/pixel_index");
                        H5Id dv = h5_open_dataset(f, grp + "/voxel_index");
                        H5Id dx = h5_open_dataset(f, grp + "/value");
                        const auto np = h5_dims(dp), nv = h5_dims(dv), nx = h5_dims(dx);
                        if (np.size() != 1 || nv.size() != 1 || nx.size() != 1 || np[0] != nx[0] || nv[0] != nx[0])
                            throw Error("Inconsistent sparse RTM arrays in " + path + ".");
                        const uint64_t n = nx[0];
                        // SART_LOAD_TRACE=1: the passes' wall times on stderr
                        const bool trace = std::getenv("SART_LOAD_TRACE") != nullptr;
                        double t_read = 0, t_count = 0, t_fill = 0;
                        auto now = [] { return std::chrono::steady_clock::now(); };
                        auto since = [](auto t) { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t).count(); };
                        const auto t_pass1 = now();
                        std::vector<uint64_t> pb(std::min(chunk, n)), vb(std::min(chunk, n));
                        std::vector<float> xb;
                        // pass 1: entries per row of the shard (and the checks of every entry)
                        for (uint64_t o = 0; o < n; o += chunk) {
                            const uint64_t m = std::min(chunk, n - o);
                            auto tr = now();
                            h5_read_range_u64(dp, o, m, pb.data());
                            h5_read_range_u64(dv, o, m, vb.data());
                            t_read += since(tr);
                            for (uint64_t t = 0; t < m; ++t) {
                                if (vb[t] >= nvox_seg) throw Error("Sparse RTM voxel index out of range in " + path + ".");
                                if (pb[t] >= lr0 && pb[t] < lr1 && vb[t] >= s0 && vb[t] < s1) ++seg.ptr[pb[t] - lr0 + 1];
                            }
                        }
                        t_count = since(t_pass1);
                        const auto t_pass2 = now();
                        for (uint64_t r = 0; r < nr; ++r) seg.ptr[r + 1] += seg.ptr[r];
                        seg.idx.resize((size_t)seg.ptr[nr]);
                        seg.val.resize((size_t)seg.ptr[nr]);
                        // pass 2: the entries into their rows, in file order (one thread: a parallel scatter over
                        // row ranges measured no faster, every thread scanning every chunk)
                        std::vector<int64_t> next(seg.ptr.begin(), seg.ptr.end() - 1);
                        xb.resize(std::min(chunk, n));
                        const int nth = std::max(1, std::min(omp_get_max_threads(), 16));
                        for (uint64_t o = 0; o < n && seg.ptr[nr] > 0; o += chunk) {
                            const uint64_t m = std::min(chunk, n - o);
                            auto tr = now();
                            h5_read_range_u64(dp, o, m, pb.data());
                            h5_read_range_u64(dv, o, m, vb.data());
                            h5_read_range_f32(dx, o, m, xb.data());
                            t_read += since(tr);
                            for (uint64_t t = 0; t < m; ++t)
                                if (pb[t] >= lr0 && pb[t] < lr1 && vb[t] >= s0 && vb[t] < s1) {
                                    const int64_t d = next[pb[t] - lr0]++;
                                    seg.idx[(size_t)d] = (int32_t)(ocol + (vb[t] - s0));
                                    seg.val[(size_t)d] = xb[t];
                                }
                        }
                        // per row: ascending columns (stable), the last of repeated (row, col) entries, no zeros --
                        // rows sorted in parallel (1.45 -> 0.25 s for 20M entries on 8 threads), their kept entries
                        // at the start of their own range (kept[r]), then moved down in row order
                        t_fill = since(t_pass2);
                        const auto t_sort = now();
                        std::vector<int64_t> kept(nr, 0);
#pragma omp parallel num_threads(nth)
                        {
                            std::vector<std::pair<int32_t, float>> row;
#pragma omp for schedule(dynamic, 256)
                            for (int64_t r = 0; r < (int64_t)nr; ++r) {
                                row.clear();
                                for (int64_t k = seg.ptr[r]; k < seg.ptr[r + 1]; ++k) row.push_back({seg.idx[k], seg.val[k]});
                                std::stable_sort(row.begin(), row.end(),
                                                 [](const auto& p, const auto& q) { return p.first < q.first; });
                                int64_t w = seg.ptr[r];
                                for (size_t k = 0; k < row.size(); ++k) {
                                    if (k + 1 < row.size() && row[k + 1].first == row[k].first) continue;
                                    if (row[k].second == 0.0f) continue;
                                    seg.idx[(size_t)w] = row[k].first;
                                    seg.val[(size_t)w] = row[k].second;
                                    ++w;
                                }
                                kept[r] = w - seg.ptr[r];
                            }
                        }
                        int64_t w = 0;
                        for (uint64_t r = 0; r < nr; ++r) {
                            const int64_t b = seg.ptr[r];
                            seg.ptr[r] = w;
                            if (b != w)
                                for (int64_t k = 0; k < kept[r]; ++k) {
                                    seg.idx[(size_t)(w + k)] = seg.idx[(size_t)(b + k)];
                                    seg.val[(size_t)(w + k)] = seg.val[(size_t)(b + k)];
                                }
                            w += kept[r];
                        }
                        seg.ptr[nr] = w;
                        if (trace)
                            std::fprintf(stderr, "read_csr %s: %llu entries, pass 1 %.3f s, pass 2 %.3f s (HDF5 reads %.3f s "
                                         "of both), sort + compact %.3f s, %d threads\n", path.c_str(),
                                         (unsigned long long)n, t_count, t_fill, t_read, since(t_sort), nth);
                        seg.idx.resize((size_t)w);
                        seg.val.resize((size_t)w);
                        seg.idx.shrink_to_fit();
                        seg.val.shrink_to_fit();
                    } else {
                        H5Id d = h5_open_dataset(f, grp + "/value");
                        const auto dims = h5_dims(d);
                        if (dims.size() != 2 || dims[0] != npix || dims[1] != nvox_seg)
                            throw Error("Dense RTM dataset in " + path + " has unexpected shape.");
                        const uint64_t nc = s1 - s0;
                        const uint64_t rpr = std::max<uint64_t>(1, (64ull << 20) / (4 * nc));
                        std::vector<float> blk;
                        for (uint64_t r = lr0; r < lr1; r += rpr) {
                            const uint64_t m = std::min(rpr, lr1 - r);
                            blk.assign(m * nc, 0.0f);
                            h5_read_block_f32(d, r, m, s0, nc, blk.data(), nc, 0);
                            for (uint64_t i = 0; i < m; ++i) {
                                for (uint64_t c = 0; c < nc; ++c)
                                    if (blk[i * nc + c] != 0.0f) {
                                        seg.idx.push_back((int32_t)(ocol + c));
                                        seg.val.push_back(blk[i * nc + c]);
                                    }
                                seg.ptr[r - lr0 + i + 1] = (int64_t)seg.val.size();
                            }
                        }
                    }
                    segs.push_back(std::move(seg));
                }
                start_voxel += nvox_seg;
            }
            // the camera's rows: its segments concatenated row by row (one segment into an empty CSR: moved)
            if (segs.size() == 1 && out.idx.empty()) {
                HostCsr& sg = segs.front();
                for (uint64_t r = 0; r < nr; ++r) out.ptr[orow + r + 1] = sg.ptr[r + 1];
                out.idx = std::move(sg.idx);
                out.val = std::move(sg.val);
                start_pixel = cam_end;
                if (start_pixel >= row_end) break;
                continue;
            }
            size_t total = out.idx.size();
            for (const auto& sg : segs) total += sg.idx.size();
            out.idx.reserve(total);
            out.val.reserve(total);
            for (uint64_t r = 0; r < nr; ++r) {
                for (const auto& sg : segs) {
                    out.idx.insert(out.idx.end(), sg.idx.begin() + sg.ptr[r], sg.idx.begin() + sg.ptr[r + 1]);
                    out.val.insert(out.val.end(), sg.val.begin() + sg.ptr[r], sg.val.begin() + sg.ptr[r + 1]);
                }
                out.ptr[orow + r + 1] = (int64_t)out.idx.size();
            }
        }
        start_pixel = cam_end;
        if (start_pixel >= row_end) break;
    }
    // rows of cameras past the files (none for validated inputs) keep the last offset
    for (uint64_t r = 0; r < nrows; ++r) out.ptr[r + 1] = std::max(out.ptr[r + 1], out.ptr[r]);
    return out;
}

LaplacianCOO read_laplacian(const std::string& path, uint64_t expected_nvoxel) {
    SART_H5_LOCK;
    H5Id f = h5_open_file(path);
    LaplacianCOO L;
    L.nvoxel = h5_attr_u64(f, "laplacian", "nvoxel");
    if (L.nvoxel != expected_nvoxel) throw Error("Laplacian and ray-transfer matrices have different number of voxels.");
    auto val = h5_read_f32(f, "laplacian/value");
    auto ii = h5_read_u64(f, "laplacian/i");
    auto jj = h5_read_u64(f, "laplacian/j");
    if (ii.size() != val.size() || jj.size() != val.size()) throw Error("Inconsistent Laplacian arrays in " + path + ".");
    const uint64_t n = L.nvoxel;
    std::vector<uint64_t> flat(val.size());
    for (size_t t = 0; t < val.size(); ++t) {
        if (ii[t] >= n || jj[t] >= n) throw Error("Laplacian index out of range in " + path + ".");
        flat[t] = ii[t] * n + jj[t];
    }
    std::vector<size_t> order(val.size());
    std::iota(order.begin(), order.end(), 0);
    if (!std::is_sorted(flat.begin(), flat.end()))
        std::stable_sort(order.begin(), order.end(), [&](size_t a, size_t b) { return flat[a] < flat[b]; });
    L.i.resize(val.size());
    L.j.resize(val.size());
    L.value.resize(val.size());
    for (size_t t = 0; t < order.size(); ++t) {
        L.i[t] = ii[order[t]];
        L.j[t] = jj[order[t]];
        L.value[t] = val[order[t]];
    }
    return L;
}

InputSet validate_inputs(const std::vector<std::string>& input_files, const std::string& rtm_name,
                         double wavelength_threshold) {
    SART_H5_LOCK;
    std::vector<std::string> rtm, img;
    categorize_input_files(input_files, rtm, img);
    if (rtm.empty()) throw Error("No RTM files given.");
    if (img.empty()) throw Error("No image files given.");
    check_group_attribute_consistency(rtm, "rtm/" + rtm_name, {"wavelength"}, false);
    check_group_attribute_consistency(rtm, "rtm/voxel_map", {"nx", "ny", "nz"}, true);
    InputSet in;
    in.rtm_files = sort_rtm_files(rtm);
    check_rtm_frame_consistency(in.rtm_files);
    check_rtm_voxel_consistency(in.rtm_files);
    check_group_attribute_consistency(img, "image", {"wavelength"}, false);
    in.image_files = sort_image_files(img);
    check_rtm_image_consistency(in.rtm_files, in.image_files, rtm_name, wavelength_threshold);
    const auto sz = get_total_rtm_size(in.rtm_files);
    in.npixel = sz.first;
    in.nvoxel = sz.second;
    in.frame_masks = read_rtm_frame_masks(in.rtm_files);
    for (const auto& kv : in.image_files) in.camera_names.push_back(kv.first);
    in.rtm_name = rtm_name;
    in.has_sparse = rtm_has_sparse(in.rtm_files, rtm_name);
    return in;
}

#else  // !SART_HAVE_HDF5

[[noreturn]] static void nohdf5() { throw Error("built without HDF5 support"); }
void categorize_input_files(const std::vector<std::string>&, std::vector<std::string>&, std::vector<std::string>&) { nohdf5(); }
void check_group_attribute_consistency(const std::vector<std::string>&, const std::string&, const std::vector<std::string>&, bool) { nohdf5(); }
SortedRtmFiles sort_rtm_files(const std::vector<std::string>&) { nohdf5(); }
void check_rtm_frame_consistency(const SortedRtmFiles&) { nohdf5(); }
void check_rtm_voxel_consistency(const SortedRtmFiles&) { nohdf5(); }
std::map<std::string, std::vector<int32_t>> read_rtm_frame_masks(const SortedRtmFiles&) { nohdf5(); }
std::map<std::string, std::pair<uint64_t, uint64_t>> read_rtm_frame_shapes(const SortedRtmFiles&) { nohdf5(); }
SortedImageFiles sort_image_files(const std::vector<std::string>&) { nohdf5(); }
void check_rtm_image_consistency(const SortedRtmFiles&, const SortedImageFiles&, const std::string&, double) { nohdf5(); }
std::pair<uint64_t, uint64_t> get_total_rtm_size(const SortedRtmFiles&) { nohdf5(); }
RtmReader::RtmReader(SortedRtmFiles, std::string, uint64_t, uint64_t, uint64_t) { nohdf5(); }
void RtmReader::read(uint64_t, uint64_t, float*, uint64_t) { nohdf5(); }
HostCsr RtmReader::read_csr(uint64_t, uint64_t) { nohdf5(); }
void read_rtm_rows(const SortedRtmFiles&, const std::string&, uint64_t, uint64_t, uint64_t, float*, uint64_t) { nohdf5(); }
bool rtm_has_sparse(const SortedRtmFiles&, const std::string&) { nohdf5(); }
double rtm_sparse_density(const SortedRtmFiles&, const std::string&, uint64_t, uint64_t) { nohdf5(); }
LaplacianCOO read_laplacian(const std::string&, uint64_t) { nohdf5(); }
InputSet validate_inputs(const std::vector<std::string>&, const std::string&, double) { nohdf5(); }

#endif

}  // namespace sart
