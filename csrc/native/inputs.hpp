// Input-file discovery, validation and matrix loaders (HDF5 schema of manual.pdf p.5-8).
//
// Behaviour mirrors the reference validators (reference hdf5files.cpp:20-389, raytransfer.cpp:27-127,
// laplacian.cpp:34-91); errors are reported by throwing sart::Error with the reference's messages
// instead of calling std::exit on one rank.
#pragma once

#include <cstdint>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "h5.hpp"
#include "sparse_csr.hpp"

namespace sart {

// camera name -> RTM files ordered by the minimum flat voxel index of their voxel-map segment
using SortedRtmFiles = std::map<std::string, std::vector<std::string>>;
// camera name -> image file
using SortedImageFiles = std::map<std::string, std::string>;

void categorize_input_files(const std::vector<std::string>& input_files, std::vector<std::string>& rtm_files,
                            std::vector<std::string>& image_files);
// Attributes `names` of group `group` must be identical in every file (double or integer compare).
void check_group_attribute_consistency(const std::vector<std::string>& files, const std::string& group,
                                       const std::vector<std::string>& names, bool integer);
SortedRtmFiles sort_rtm_files(const std::vector<std::string>& files);
void check_rtm_frame_consistency(const SortedRtmFiles& sorted);
void check_rtm_voxel_consistency(const SortedRtmFiles& sorted);
std::map<std::string, std::vector<int32_t>> read_rtm_frame_masks(const SortedRtmFiles& sorted);
std::map<std::string, std::pair<uint64_t, uint64_t>> read_rtm_frame_shapes(const SortedRtmFiles& sorted);
SortedImageFiles sort_image_files(const std::vector<std::string>& files);
void check_rtm_image_consistency(const SortedRtmFiles& rtm, const SortedImageFiles& images,
                                 const std::string& rtm_name, double wavelength_threshold);
std::pair<uint64_t, uint64_t> get_total_rtm_size(const SortedRtmFiles& sorted);

// Streaming reader of the global RTM (cameras concatenated in name order along the rows, voxel segments
// concatenated along the columns), restricted to the column window [col_begin, col_end) (a voxel-column
// shard reads only its block; col_end 0 = nvoxel). read(r0, r1, out, ld) writes rows [r0, r1) x the window
// into out[(r - r0) * ld + (v - col_begin)]: dense datasets as row blocks with one hyperslab per block (only
// the window's columns), sparse (COO) datasets scattered from arrays read ONCE per segment and kept sorted
// by pixel. Rows of `out` must be zero-initialised by the caller when sparse data is present.
class RtmReader {
   public:
    RtmReader(SortedRtmFiles sorted, std::string rtm_name, uint64_t nvoxel, uint64_t col_begin = 0,
              uint64_t col_end = 0);
    void read(uint64_t row_begin, uint64_t row_end, float* out, uint64_t ld);
    // The same rows and columns as a CSR matrix of the non-zero entries (sparse datasets from their COO arrays,
    // dense datasets from the non-zeros of row blocks): what read() would leave in a zeroed dense block, without
    // the dense block (the sparse RTM path, csrc/kernels/sparse.hip).
    HostCsr read_csr(uint64_t row_begin, uint64_t row_end);
    uint64_t ncols() const { return c1_ - c0_; }
    // Dense datasets: rows per hyperslab read (0: blocks of <= 64 MiB; 1: one row per read, the reference's
    // pattern raytransfer.cpp:103-109, kept for load-path comparisons: SART_RTM_ROWS_PER_READ).
    void set_rows_per_read(uint64_t n) { rows_per_read_ = n; }

   private:
    struct SparseSegment {
        std::vector<uint64_t> pix, vox;
        std::vector<float> val;
    };
    const SparseSegment& sparse_segment(int64_t f, const std::string& path, uint64_t nvox_seg);  // f: hid_t
    SortedRtmFiles sorted_;
    std::string name_;
    uint64_t nvoxel_ = 0, c0_ = 0, c1_ = 0, rows_per_read_ = 0;
    std::map<std::string, SparseSegment> sparse_;
};
// One-shot read of whole rows (all columns).
void read_rtm_rows(const SortedRtmFiles& sorted, const std::string& rtm_name, uint64_t nvoxel, uint64_t row_begin,
                   uint64_t row_end, float* out, uint64_t ld);
bool rtm_has_sparse(const SortedRtmFiles& sorted, const std::string& rtm_name);
// Stored entries of all RTM datasets / (npixel x nvoxel) when every dataset is sparse COO; -1 when one is dense.
double rtm_sparse_density(const SortedRtmFiles& sorted, const std::string& rtm_name, uint64_t npixel, uint64_t nvoxel);

// Everything the driver needs to know about the inputs, validated with the same checks in the same order
// as the reference (main.cpp:27-59).
struct InputSet {
    SortedRtmFiles rtm_files;
    SortedImageFiles image_files;
    std::vector<std::string> camera_names;  // sorted by name: global pixel order
    uint64_t npixel = 0, nvoxel = 0;
    std::map<std::string, std::vector<int32_t>> frame_masks;
    std::string rtm_name;
    bool has_sparse = false;
};
InputSet validate_inputs(const std::vector<std::string>& input_files, const std::string& rtm_name,
                         double wavelength_threshold);

struct LaplacianCOO {
    uint64_t nvoxel = 0;
    std::vector<uint64_t> i, j;  // sorted by flat index i * nvoxel + j
    std::vector<float> value;
};
LaplacianCOO read_laplacian(const std::string& path, uint64_t expected_nvoxel);

}  // namespace sart
