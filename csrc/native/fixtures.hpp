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

}  // namespace sart
