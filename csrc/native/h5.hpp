// Thin RAII layer over the HDF5 C API (HDF5 >= 1.10).
//
// The reference uses the HDF5 C++ API (H5Cpp.h) everywhere; the C API is used here so the module
// has no C++-ABI dependency on the HDF5 build. Every failure throws sart::Error with the HDF5 path
// that failed, the HDF5 error stack printing is silenced.
#pragma once

#include <cstdint>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

#ifdef SART_HAVE_HDF5
#include <hdf5.h>
#endif

namespace sart {

struct Error : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// The HDF5 library (the conda build is not thread-safe) may be entered by one thread at a time: every
// public entry point of the native runtime that touches HDF5 holds this lock (the drivers read the next
// frame on a helper thread while the solution writer may flush).
std::recursive_mutex& h5_mutex();
#define SART_H5_LOCK std::lock_guard<std::recursive_mutex> sart_h5_lock_(::sart::h5_mutex())

#ifdef SART_HAVE_HDF5

class H5Id {
   public:
    enum Kind { kFile, kGroup, kDataset, kSpace, kAttr, kType, kPlist, kObject };
    H5Id() = default;
    H5Id(hid_t id, Kind k) : id_(id), kind_(k) {}
    H5Id(const H5Id&) = delete;
    H5Id& operator=(const H5Id&) = delete;
    H5Id(H5Id&& o) noexcept : id_(o.id_), kind_(o.kind_) { o.id_ = -1; }
    H5Id& operator=(H5Id&& o) noexcept {
        if (this != &o) {
            reset();
            id_ = o.id_;
            kind_ = o.kind_;
            o.id_ = -1;
        }
        return *this;
    }
    ~H5Id() { reset(); }
    hid_t get() const { return id_; }
    operator hid_t() const { return id_; }
    bool valid() const { return id_ >= 0; }
    void reset();

   private:
    hid_t id_ = -1;
    Kind kind_ = kObject;
};

void h5_quiet();  // disable automatic error-stack printing (once)

H5Id h5_open_file(const std::string& path, bool write = false);
H5Id h5_create_file(const std::string& path);  // truncates
bool h5_exists(hid_t loc, const std::string& path);  // link path exists (every component checked)
bool h5_attr_exists(hid_t loc, const std::string& obj_path, const std::string& name);
H5Id h5_open_group(hid_t loc, const std::string& path);
H5Id h5_open_dataset(hid_t loc, const std::string& path);
std::vector<hsize_t> h5_dims(hid_t dset);

double h5_attr_double(hid_t loc, const std::string& obj, const std::string& name);
uint64_t h5_attr_u64(hid_t loc, const std::string& obj, const std::string& name);
int64_t h5_attr_i64(hid_t loc, const std::string& obj, const std::string& name);
std::string h5_attr_string(hid_t loc, const std::string& obj, const std::string& name);

// Whole-dataset reads converted to the requested memory type.
std::vector<double> h5_read_f64(hid_t loc, const std::string& path);
std::vector<float> h5_read_f32(hid_t loc, const std::string& path);
std::vector<uint64_t> h5_read_u64(hid_t loc, const std::string& path);
std::vector<int64_t> h5_read_i64(hid_t loc, const std::string& path);
std::vector<int32_t> h5_read_i32(hid_t loc, const std::string& path);

// Rows [row0, row0 + nrows) x [0, ncols) of a 2-D float dataset into out (row stride ld floats,
// column offset col0 inside each output row).
void h5_read_rows_f32(hid_t dset, uint64_t row0, uint64_t nrows, uint64_t ncols, float* out, uint64_t ld,
                      uint64_t col0);
// Rows [row0, +nrows) x file columns [fcol0, +ncols) of a 2-D float dataset into out (row stride ld, at
// memory column col0): one hyperslab per call.
void h5_read_block_f32(hid_t dset, uint64_t row0, uint64_t nrows, uint64_t fcol0, uint64_t ncols, float* out,
                       uint64_t ld, uint64_t col0);
// One [1, H, W] slab of a 3-D dataset as doubles.
void h5_read_frame_f64(hid_t dset, uint64_t index, double* out, uint64_t frame_size);
// elements [off, off + n) of a 1-D dataset (hyperslab reads of the sparse RTM's COO arrays in bounded chunks)
void h5_read_range_u64(hid_t dset, uint64_t off, uint64_t n, uint64_t* out);
void h5_read_range_f32(hid_t dset, uint64_t off, uint64_t n, float* out);

// Writers (used by the solution writer, the voxel-map copy and the test-fixture writers).
H5Id h5_create_group(hid_t loc, const std::string& path);
void h5_write_attr_double(hid_t obj, const std::string& name, double v);
void h5_write_attr_u64(hid_t obj, const std::string& name, uint64_t v);
void h5_write_attr_i32(hid_t obj, const std::string& name, int32_t v);
void h5_write_attr_string(hid_t obj, const std::string& name, const std::string& v);
void h5_write_f64(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const double* data);
void h5_write_f32(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const float* data);
void h5_write_u64(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const uint64_t* data);
void h5_write_i32(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const int32_t* data);
void h5_write_u8(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const uint8_t* data);
// Datasets written piecewise (large synthetic fixtures): create with file type `ftype`, then write the box
// [off, off + cnt) from a dense memory block of memory type `mtype`.
H5Id h5_create_dataset(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, hid_t ftype);
void h5_write_box(hid_t dset, const std::vector<uint64_t>& off, const std::vector<uint64_t>& cnt, hid_t mtype,
                  const void* data);

#endif  // SART_HAVE_HDF5

bool have_hdf5();

}  // namespace sart
