// Writers of input files in the reference HDF5 schema (manual.pdf p.5-8). The reference ships no
// writer and no test data; these produce RTM / image / Laplacian files for the tests, examples and
// synthetic end-to-end benchmarks of the CLI.
#include "fixtures.hpp"

#include <fcntl.h>
#include <unistd.h>

#include <algorithm>

namespace sart {

float synthetic_rtm_value(uint64_t seed, uint64_t p, uint64_t v) {
    uint64_t z = seed * 0x9E3779B97F4A7C15ull + p * 0xBF58476D1CE4E5B9ull + v * 0x94D049BB133111EBull + 1;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (float)((double)(z >> 40) * (1.0 / 16777216.0));  // 24 bits: exact in fp32
}

uint64_t synthetic_rtm_voxel(uint64_t p, uint64_t k, uint64_t nnz_per_row, uint64_t nvoxel) {
    // distinct voxels per pixel (k * stride < nvoxel for k < nnz_per_row), shifted per pixel
    const uint64_t stride = std::max<uint64_t>(1, nvoxel / std::max<uint64_t>(1, nnz_per_row));
    return (p * 7919 + k * stride) % nvoxel;
}

bool drop_file_cache(const std::string& path) {
    const int fd = ::open(path.c_str(), O_RDONLY);
    if (fd < 0) return false;
    (void)::fdatasync(fd);
#ifdef POSIX_FADV_DONTNEED
    (void)::posix_fadvise(fd, 0, 0, POSIX_FADV_DONTNEED);
#endif
    ::close(fd);
    return true;
}

#ifdef SART_HAVE_HDF5

uint64_t write_synthetic_rtm_file(const std::string& path, const std::string& camera_name, double wavelength,
                                  uint64_t h, uint64_t w, uint64_t nvoxel, uint64_t seed, uint64_t nnz_per_row,
                                  bool drop_cache, uint64_t block_bytes, const std::string& rtm_name) {
    if (h == 0 || w == 0 || nvoxel == 0) throw Error("write_synthetic_rtm_file: empty shape");
    if (nnz_per_row > nvoxel) throw Error("write_synthetic_rtm_file: more nonzeros per row than voxels");
    const uint64_t npixel = h * w;
    uint64_t bytes = 0;
    {
        SART_H5_LOCK;
        H5Id f = h5_create_file(path);
        H5Id rtm = h5_create_group(f, "rtm");
        h5_write_attr_string(rtm, "camera_name", camera_name);
        h5_write_attr_u64(rtm, "npixel", npixel);
        h5_write_attr_u64(rtm, "nvoxel", nvoxel);
        {
            H5Id g = h5_create_group(rtm, rtm_name);
            h5_write_attr_double(g, "wavelength", wavelength);
            h5_write_attr_i32(g, "is_sparse", nnz_per_row ? 1 : 0);
            if (nnz_per_row == 0) {
                H5Id d = h5_create_dataset(g, "value", {npixel, nvoxel}, H5T_IEEE_F32LE);
                const uint64_t rows = std::max<uint64_t>(1, std::min<uint64_t>(npixel, block_bytes / (4 * nvoxel)));
                std::vector<float> buf(rows * nvoxel);
                for (uint64_t r0 = 0; r0 < npixel; r0 += rows) {
                    const uint64_t nr = std::min(rows, npixel - r0);
#pragma omp parallel for schedule(static)
                    for (int64_t r = 0; r < (int64_t)nr; ++r)
                        for (uint64_t v = 0; v < nvoxel; ++v)
                            buf[(uint64_t)r * nvoxel + v] = synthetic_rtm_value(seed, r0 + (uint64_t)r, v);
                    h5_write_box(d, {r0, 0}, {nr, nvoxel}, H5T_NATIVE_FLOAT, buf.data());
                }
                bytes = npixel * nvoxel * 4;
            } else {
                const uint64_t nnz = npixel * nnz_per_row;
                H5Id dp = h5_create_dataset(g, "pixel_index", {nnz}, H5T_STD_U64LE);
                H5Id dv = h5_create_dataset(g, "voxel_index", {nnz}, H5T_STD_U64LE);
                H5Id dx = h5_create_dataset(g, "value", {nnz}, H5T_IEEE_F32LE);
                const uint64_t rows = std::max<uint64_t>(1, std::min<uint64_t>(npixel, block_bytes / (20 * nnz_per_row)));
                std::vector<uint64_t> pi(rows * nnz_per_row), vi(rows * nnz_per_row);
                std::vector<float> val(rows * nnz_per_row);
                for (uint64_t r0 = 0; r0 < npixel; r0 += rows) {
                    const uint64_t nr = std::min(rows, npixel - r0);
#pragma omp parallel for schedule(static)
                    for (int64_t r = 0; r < (int64_t)nr; ++r)
                        for (uint64_t k = 0; k < nnz_per_row; ++k) {
                            const uint64_t n = (uint64_t)r * nnz_per_row + k, p = r0 + (uint64_t)r;
                            pi[n] = p;
                            vi[n] = synthetic_rtm_voxel(p, k, nnz_per_row, nvoxel);
                            val[n] = synthetic_rtm_value(seed, p, vi[n]);
                        }
                    const uint64_t n0 = r0 * nnz_per_row, cnt = nr * nnz_per_row;
                    h5_write_box(dp, {n0}, {cnt}, H5T_NATIVE_UINT64, pi.data());
                    h5_write_box(dv, {n0}, {cnt}, H5T_NATIVE_UINT64, vi.data());
                    h5_write_box(dx, {n0}, {cnt}, H5T_NATIVE_FLOAT, val.data());
                }
                bytes = nnz * 20;
            }
        }
        std::vector<uint8_t> mask(npixel, 1);
        h5_write_u8(rtm, "frame_mask", {h, w}, mask.data());
        H5Id vm = h5_create_group(rtm, "voxel_map");
        h5_write_attr_u64(vm, "nx", nvoxel);
        h5_write_attr_u64(vm, "ny", 1);
        h5_write_attr_u64(vm, "nz", 1);
        std::vector<uint64_t> vi(nvoxel), zero(nvoxel, 0);
        std::vector<int32_t> vv(nvoxel);
        for (uint64_t v = 0; v < nvoxel; ++v) {
            vi[v] = v;
            vv[v] = (int32_t)v;
        }
        h5_write_u64(vm, "i", {nvoxel}, vi.data());
        h5_write_u64(vm, "j", {nvoxel}, zero.data());
        h5_write_u64(vm, "k", {nvoxel}, zero.data());
        h5_write_i32(vm, "value", {nvoxel}, vv.data());
    }  // file closed here
    if (drop_cache) (void)drop_file_cache(path);
    return bytes;
}

void write_rtm_file(const RtmFileSpec& s) {
    SART_H5_LOCK;
    H5Id f = h5_create_file(s.path);
    H5Id rtm = h5_create_group(f, "rtm");
    h5_write_attr_string(rtm, "camera_name", s.camera_name);
    h5_write_attr_u64(rtm, "npixel", s.npixel);
    h5_write_attr_u64(rtm, "nvoxel", s.nvoxel);
    {
        H5Id g = h5_create_group(rtm, s.rtm_name);
        h5_write_attr_double(g, "wavelength", s.wavelength);
        h5_write_attr_i32(g, "is_sparse", s.sparse ? 1 : 0);
        if (s.sparse) {
            const std::vector<uint64_t> d = {s.value.size()};
            if (s.pixel_index.size() != s.value.size() || s.voxel_index.size() != s.value.size())
                throw Error("write_rtm_file: inconsistent sparse arrays");
            h5_write_u64(g, "pixel_index", d, s.pixel_index.data());
            h5_write_u64(g, "voxel_index", d, s.voxel_index.data());
            h5_write_f32(g, "value", d, s.value.data());
        } else {
            if (s.value.size() != s.npixel * s.nvoxel) throw Error("write_rtm_file: dense value has the wrong size");
            h5_write_f32(g, "value", {s.npixel, s.nvoxel}, s.value.data());
        }
    }
    if (s.frame_mask.size() != s.frame_h * s.frame_w) throw Error("write_rtm_file: frame mask has the wrong size");
    h5_write_u8(rtm, "frame_mask", {s.frame_h, s.frame_w}, s.frame_mask.data());
    H5Id vm = h5_create_group(rtm, "voxel_map");
    h5_write_attr_u64(vm, "nx", s.nx);
    h5_write_attr_u64(vm, "ny", s.ny);
    h5_write_attr_u64(vm, "nz", s.nz);
    if (s.bounds.size() == 6) {
        const char* names[6] = {"xmin", "xmax", "ymin", "ymax", "zmin", "zmax"};
        for (int k = 0; k < 6; ++k) h5_write_attr_double(vm, names[k], s.bounds[k]);
    }
    if (!s.coordinate_system.empty()) h5_write_attr_string(vm, "coordinate_system", s.coordinate_system);
    const std::vector<uint64_t> d = {s.vi.size()};
    h5_write_u64(vm, "i", d, s.vi.data());
    h5_write_u64(vm, "j", d, s.vj.data());
    h5_write_u64(vm, "k", d, s.vk.data());
    h5_write_i32(vm, "value", d, s.vvalue.data());
}

void write_image_file(const std::string& path, const std::string& camera_name, double wavelength,
                      const std::vector<double>& time, const std::vector<double>& frames, uint64_t h, uint64_t w) {
    SART_H5_LOCK;
    if (frames.size() != time.size() * h * w) throw Error("write_image_file: frames have the wrong size");
    H5Id f = h5_create_file(path);
    H5Id g = h5_create_group(f, "image");
    h5_write_attr_string(g, "camera_name", camera_name);
    h5_write_attr_double(g, "wavelength", wavelength);
    h5_write_f64(g, "time", {time.size()}, time.data());
    h5_write_f64(g, "frame", {time.size(), h, w}, frames.data());
}

void write_laplacian_file(const std::string& path, uint64_t nvoxel, const std::vector<uint64_t>& i,
                          const std::vector<uint64_t>& j, const std::vector<float>& value) {
    SART_H5_LOCK;
    if (i.size() != value.size() || j.size() != value.size()) throw Error("write_laplacian_file: inconsistent arrays");
    H5Id f = h5_create_file(path);
    H5Id g = h5_create_group(f, "laplacian");
    h5_write_attr_u64(g, "nvoxel", nvoxel);
    const std::vector<uint64_t> d = {value.size()};
    h5_write_u64(g, "i", d, i.data());
    h5_write_u64(g, "j", d, j.data());
    h5_write_f32(g, "value", d, value.data());
}

#else
void write_rtm_file(const RtmFileSpec&) { throw Error("built without HDF5 support"); }
void write_image_file(const std::string&, const std::string&, double, const std::vector<double>&,
                      const std::vector<double>&, uint64_t, uint64_t) {
    SART_H5_LOCK;
    throw Error("built without HDF5 support");
}
void write_laplacian_file(const std::string&, uint64_t, const std::vector<uint64_t>&, const std::vector<uint64_t>&,
                          const std::vector<float>&) {
    SART_H5_LOCK;
    throw Error("built without HDF5 support");
}
uint64_t write_synthetic_rtm_file(const std::string&, const std::string&, double, uint64_t, uint64_t, uint64_t,
                                  uint64_t, uint64_t, bool, uint64_t, const std::string&) {
    throw Error("built without HDF5 support");
}
#endif

}  // namespace sart
