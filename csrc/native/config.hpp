// Command-line configuration of the sartsolver driver.
//
// Same options, short aliases, defaults and validation as the reference CLI (reference
// arguments.cpp:82-251, arguments.hpp:14-33), with an in-tree parser instead of p-ranav/argparse.
// Extensions (not in the reference) are marked: --resume, --batch_frames, --two_pass, --partition_voxels,
// --profile.
#pragma once

#include <array>
#include <string>
#include <vector>

namespace sart {

struct Config {
    std::vector<std::string> input_files;
    std::string output_file = "solution.h5";
    std::string time_range;
    std::string laplacian_file;
    std::string raytransfer_name = "with_reflections";
    double wavelength_threshold = 50.0;
    double ray_density_threshold = 1e-6;
    double ray_length_threshold = 1e-6;
    double conv_tolerance = 1e-5;
    double beta_laplace = 2e-2;
    double relaxation = 1.0;
    int max_iterations = 2000;
    int max_cached_frames = 100;
    int max_cached_solutions = 100;
    bool logarithmic = false;
    bool no_guess = false;
    bool use_cpu = false;
    bool parallel_read = false;
    // extensions
    bool resume = false;        // append to an existing output file, skip frames already solved
    int batch_frames = 1;       // >1: solve independent frames together (MFMA multi-frame path, implies --no_guess)
    bool two_pass = false;      // disable the fused single-pass sweep
    bool partition_voxels = false;
    // GPU single-frame solver: keep the RTM sparse on the device (CSR + CSC, csrc/kernels/sparse.hip) instead of a
    // dense shard. "auto": when every RTM dataset is sparse COO with at most 10 % non-zeros; "dense" / "sparse".
    std::string rtm_format = "auto";
    bool rtm_bf16 = false;      // GPU: store the RTM shard in bf16 (fp32 products and sums)  // GPU: shard the RTM by voxel columns (all pixels per rank) instead of pixel rows
    std::string profile_file;   // JSON timing/telemetry sidecar
    bool help = false;
};

// Throws sart::Error with a usage message on invalid input; --help sets Config::help.
Config parse_arguments(const std::vector<std::string>& argv);
std::string usage();

// "start:stop[:step[:sync_threshold]], ..." -> {start, stop, step, threshold}; empty -> {0, inf, 0, 0}
std::vector<std::array<double, 4>> parse_time_intervals(const std::string& spec);

}  // namespace sart
