// Composite multi-camera frames, solution output and voxel grids (HDF5 schema of manual.pdf p.5-8).
//
// CompositeImage   -- reference image.cpp:20-331: per-camera frame selection inside time intervals,
//                     synchronisation on a step grid within a threshold, masking, local pixel slice,
//                     read-ahead cache of max_cache_size frames.
// SolutionWriter   -- reference solution.cpp:17-180: cached rows, extendible chunked datasets,
//                     create on first flush (truncate) or append (resume), flush on destruction.
// VoxelGrid        -- reference voxelgrid.cpp:19-323: voxel map read/write, Cartesian and
//                     cylindrical point -> voxel lookup.
#pragma once

#include <array>
#include <cstdint>
#include <map>
#include <future>
#include <string>
#include <vector>

#include "h5.hpp"

namespace sart {

class CompositeImage {
   public:
    CompositeImage(std::map<std::string, std::string> image_files,
                   std::map<std::string, std::vector<int32_t>> frame_masks,
                   const std::vector<std::array<double, 4>>& time_intervals, uint64_t npixel, uint64_t offset_pixel);

    uint64_t max_cache_size() const { return max_cache_; }
    void set_max_cache_size(uint64_t v);

    // next composite frame (returns false at the end); the first call yields frame 0
    bool next_frame(std::vector<double>& out);
    std::vector<double> frame(uint64_t i);
    double frame_time(uint64_t i) const;
    double frame_time() const { return frame_time(cur_ == time_.size() ? 0 : cur_); }
    std::vector<double> camera_frame_time(uint64_t i) const;
    std::vector<double> camera_frame_time() const { return camera_frame_time(cur_ == time_.size() ? 0 : cur_); }
    const std::vector<std::vector<uint64_t>>& frame_indices() const { return indices_; }
    uint64_t nframe() const { return time_.size(); }
    uint64_t npixel() const { return npix_; }
    uint64_t offset_pixel() const { return offset_; }
    uint64_t current_frame_index() const { return cur_; }

   private:
    void build_frames(const std::vector<std::vector<std::pair<double, uint64_t>>>& sel, double step, double threshold);
    void fill_cache(uint64_t first);
    bool cached(uint64_t i) const { return i >= cache_first_ && i < cache_first_ + cache_count_; }

    std::map<std::string, std::string> files_;
    std::map<std::string, std::vector<int32_t>> masks_;
    uint64_t npix_, offset_;
    uint64_t cur_ = 0, cache_first_ = 0, cache_count_ = 0, max_cache_ = 100;
    std::vector<double> time_;
    std::vector<std::vector<double>> camera_time_;
    std::vector<std::vector<uint64_t>> indices_;
    std::vector<double> cache_;
};

class SolutionWriter {
   public:
    SolutionWriter(std::string filename, std::vector<std::string> camera_names, uint64_t nvoxel,
                   uint64_t max_cache_size = 100, bool append = false);
    ~SolutionWriter();
    void add(const std::vector<double>& solution, int32_t status, double time, const std::vector<double>& camera_time,
             int32_t iterations = -1);
    void flush();
    uint64_t max_cache_size() const { return max_cache_; }
    void set_max_cache_size(uint64_t v);
    uint64_t pending() const { return cache_.times.size(); }

   private:
    struct Batch {
        std::vector<std::vector<double>> solutions;
        std::vector<double> times;
        std::vector<int32_t> status, iterations;
        std::vector<std::vector<double>> cam_times;  // [camera][frame]
    };
    Batch take();                // the cached frames, leaving the cache empty
    void write(const Batch& b);  // create the file on the first write, then extend the datasets
    void create(uint64_t chunk);
    void append(const Batch& b);
    std::string filename_;
    std::vector<std::string> cams_;
    uint64_t nvox_, max_cache_;
    bool first_;
    Batch cache_;
    // a full cache is written by a background thread (one at a time) while the frame loop continues: the
    // max_cache_size-frame flush no longer stalls the frame that fills the cache (profiles/series_r5_*.jsonl)
    std::future<void> pending_;
};

// (times, last solution, number of stored frames) of an existing solution file; empty if absent.
struct StoredSolutions {
    std::vector<double> time;
    std::vector<double> last_solution;
    std::vector<int32_t> status;
};
StoredSolutions read_solution_file(const std::string& filename);

class VoxelGrid {
   public:
    enum CoordSys { kCartesian = 0, kCylindrical = 1 };
    static int coordinate_system(const std::string& filename, const std::string& group);

    VoxelGrid() = default;
    // segments of one camera, in voxel order; nvoxel_per_segment (rtm/nvoxel) fixes the offsets
    void read(const std::vector<std::string>& filenames, const std::string& group);
    void write(const std::string& filename, const std::string& group) const;
    int32_t voxel_index(uint64_t i, uint64_t j, uint64_t k) const;
    int32_t voxel_index_at(double x, double y, double z) const;

    int coordsys = kCartesian;
    uint64_t nx = 0, ny = 0, nz = 0, nvox = 0;
    double xmin = 0, xmax = 1, ymin = 0, ymax = 1, zmin = 0, zmax = 1;
    std::vector<int32_t> voxmap;
    std::vector<std::string> warnings;
};

}  // namespace sart
