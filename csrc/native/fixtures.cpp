// Writers of input files in the reference HDF5 schema (manual.pdf p.5-8). The reference ships no
// writer and no test data; these produce RTM / image / Laplacian files for the tests, examples and
// synthetic end-to-end benchmarks of the CLI.
#include "fixtures.hpp"

namespace sart {

#ifdef SART_HAVE_HDF5

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
#endif

}  // namespace sart
