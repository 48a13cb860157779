#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "h5.hpp"

namespace sart {

struct RtmFileSpec {
    std::string path, camera_name, rtm_name = "with_reflections", coordinate_system;
    double wavelength = 0;
    uint64_t npixel = 0, nvoxel = 0;
    bool sparse = false;
    std::vector<float> value;  // dense: npixel * nvoxel; sparse: nnz
    std::vector<uint64_t> pixel_index, voxel_index;
    uint64_t frame_h = 0, frame_w = 0;
    std::vector<uint8_t> frame_mask;
    uint64_t nx = 0, ny = 0, nz = 0;
    std::vector<uint64_t> vi, vj, vk;
    std::vector<int32_t> vvalue;
    std::vector<double> bounds;  // empty or {xmin, xmax, ymin, ymax, zmin, zmax}
};

void write_rtm_file(const RtmFileSpec& spec);
void write_image_file(const std::string& path, const std::string& camera_name, double wavelength,
                      const std::vector<double>& time, const std::vector<double>& frames, uint64_t h, uint64_t w);
void write_laplacian_file(const std::string& path, uint64_t nvoxel, const std::vector<uint64_t>& i,
                          const std::vector<uint64_t>& j, const std::vector<float>& value);

// Large synthetic RTM file (load-path benchmarks, multi-GB fixtures) streamed to disk in row blocks of at most
// `block_bytes`, so host memory stays bounded whatever the file size. Frame mask: all ones (h x w = npixel pixels);
// voxel map: nvoxel x 1 x 1. nnz_per_row == 0: dense value[p, v] = synthetic_rtm_value(seed, p, v); else sparse COO
// with nnz_per_row entries per pixel at voxels synthetic_rtm_voxel(p, k, ...). drop_cache: fdatasync, then
// POSIX_FADV_DONTNEED, so a following read comes from the storage device rather than the page cache.
// Returns the bytes of matrix values written.
uint64_t write_synthetic_rtm_file(const std::string& path, const std::string& camera_name, double wavelength,
                                  uint64_t h, uint64_t w, uint64_t nvoxel, uint64_t seed, uint64_t nnz_per_row,
                                  bool drop_cache, uint64_t block_bytes = 256ull << 20,
                                  const std::string& rtm_name = "with_reflections");
float synthetic_rtm_value(uint64_t seed, uint64_t p, uint64_t v);  // in [0, 1)
uint64_t synthetic_rtm_voxel(uint64_t p, uint64_t k, uint64_t nnz_per_row, uint64_t nvoxel);
// fdatasync + POSIX_FADV_DONTNEED of a whole file (no-op where unsupported); false when the file cannot be opened
bool drop_file_cache(const std::string& path);

}  // namespace sart
