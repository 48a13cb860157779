#include "config.hpp"

#include <cerrno>
#include <cstdlib>
#include <functional>
#include <limits>
#include <map>
#include <sstream>

#include "h5.hpp"  // sart::Error

namespace sart {

namespace {

std::string trim(const std::string& s) {
    size_t a = s.find_first_not_of(" \t\n\r"), b = s.find_last_not_of(" \t\n\r");
    return a == std::string::npos ? std::string() : s.substr(a, b - a + 1);
}

double to_double(const std::string& tok, const std::string& opt) {
    const std::string t = trim(tok);
    char* end = nullptr;
    errno = 0;
    const double v = std::strtod(t.c_str(), &end);
    if (t.empty() || end != t.c_str() + t.size() || errno == ERANGE)
        throw Error("Failed to parse '" + tok + "' as a number for " + opt + ".");
    return v;
}

int to_int(const std::string& tok, const std::string& opt) {
    const std::string t = trim(tok);
    char* end = nullptr;
    errno = 0;
    const long v = std::strtol(t.c_str(), &end, 10);
    if (t.empty() || end != t.c_str() + t.size() || errno == ERANGE || v < std::numeric_limits<int>::min() ||
        v > std::numeric_limits<int>::max())
        throw Error("Failed to parse '" + tok + "' as an integer for " + opt + ".");
    return (int)v;
}

std::string fmt(double v) {
    std::ostringstream os;
    os << v;
    return os.str();
}

}  // namespace

std::string usage() {
    return "Usage: sartsolver [options] input_files...\n"
           "Impurity flux reconstruction for ITER: emissivity (MI355X-native SART solver)\n\n"
           "Positional arguments:\n"
           "  input_files                 List of ray transfer matrix and camera image hdf5 files.\n\n"
           "Optional arguments:\n"
           "  -h, --help                  shows help message and exits\n"
           "  -o, --output_file           Filename to save the solution. [default: \"solution.h5\"]\n"
           "  -t, --time_range            Time intervals in s to process in a form: start:stop:(step):(synch_threshold),\n"
           "                              e.g. '20.5:40.1, 45.2:51:15:0.05'. The step and the synchronization threshold\n"
           "                              are optional. [default: \"\"]\n"
           "  -w, --wavelength_threshold  An RTM is considered valid if its wavelength is within this threshold of the\n"
           "                              image wavelength (in nm). [default: 50]\n"
           "  -d, --ray_density_threshold Voxels with ray density lesser than this threshold are ignored. [default: 1e-06]\n"
           "  -r, --ray_length_threshold  Pixels with ray length lesser than this threshold are ignored. [default: 1e-06]\n"
           "  -m, --max_iterations        Maximum number of SART iterations. [default: 2000]\n"
           "  -c, --conv_tolerance        SART convolution relative tolerance. [default: 1e-05]\n"
           "  -l, --laplacian_file        File with laplacian regularization matrix. [default: \"\"]\n"
           "  -b, --beta_laplace          Weight of the regularization factor. [default: 0.02]\n"
           "  -R, --relaxation            Relaxation parameter. [default: 1]\n"
           "  -n, --raytransfer_name      Ray transfer matrix dataset name. [default: \"with_reflections\"]\n"
           "  -L, --logarithmic           Use logarithmic SART solver.\n"
           "  --max_cached_frames         Maximum number of cached image frames. [default: 100]\n"
           "  --max_cached_solutions      Maximum number of cached solutions. [default: 100]\n"
           "  --no_guess                  Do not use solution found on previous time moment as initial guess for the\n"
           "                              next one.\n"
           "  --use_cpu                   Perform all calculations on CPUs.\n"
           "  --parallel_read             Read RTM data in a parallel way (high-IOPS storage optimization).\n"
           "Extensions:\n"
           "  --resume                    Append to an existing output file and skip frames already solved.\n"
           "  --batch_frames N            Solve N frames together on the matrix cores (continuous batching: a\n"
           "                              finished frame's slot takes the next frame, warm-started from the\n"
           "                              latest frame finished before it; cold with --no_guess). This is NOT\n"
           "                              the reference's frame k-1 -> k warm-start chain, so results depend\n"
           "                              on N; N = 1 keeps the reference semantics. [default: 1]\n"
           "  --two_pass                  Use the two-pass projection kernels instead of the fused sweep.\n"
           "  --partition_voxels          Shard the RTM by voxel columns (every GPU holds all pixels of a voxel\n"
           "                              block; all-reduce of A x per iteration) instead of by pixel rows.\n"
           "  --rtm_bf16                  Store the RTM in bf16 on the GPU (half the memory and bytes per sweep;\n"
           "                              products and sums stay fp32).\n"
           "  --rtm_format F              auto | dense | sparse: keep a sparse RTM sparse (CSR + CSC; the GPU\n"
           "                              solvers and the CPU solver, pixel-row shards). auto: when every RTM dataset is\n"
           "                              sparse COO with at most 10 % non-zeros. [default: auto]\n"
           "  --profile FILE              Write per-frame timing/iteration telemetry as JSON lines.\n";
}

Config parse_arguments(const std::vector<std::string>& argv) {
    Config c;
    using Setter = std::function<void(const std::string&, const std::string&)>;
    std::map<std::string, Setter> valued = {
        {"--output_file", [&](const std::string& v, const std::string&) { c.output_file = v; }},
        {"--time_range", [&](const std::string& v, const std::string&) { c.time_range = v; }},
        {"--wavelength_threshold", [&](const std::string& v, const std::string& o) { c.wavelength_threshold = to_double(v, o); }},
        {"--ray_density_threshold", [&](const std::string& v, const std::string& o) { c.ray_density_threshold = to_double(v, o); }},
        {"--ray_length_threshold", [&](const std::string& v, const std::string& o) { c.ray_length_threshold = to_double(v, o); }},
        {"--max_iterations", [&](const std::string& v, const std::string& o) { c.max_iterations = to_int(v, o); }},
        {"--conv_tolerance", [&](const std::string& v, const std::string& o) { c.conv_tolerance = to_double(v, o); }},
        {"--laplacian_file", [&](const std::string& v, const std::string&) { c.laplacian_file = v; }},
        {"--beta_laplace", [&](const std::string& v, const std::string& o) { c.beta_laplace = to_double(v, o); }},
        {"--relaxation", [&](const std::string& v, const std::string& o) { c.relaxation = to_double(v, o); }},
        {"--raytransfer_name", [&](const std::string& v, const std::string&) { c.raytransfer_name = v; }},
        {"--max_cached_frames", [&](const std::string& v, const std::string& o) { c.max_cached_frames = to_int(v, o); }},
        {"--max_cached_solutions", [&](const std::string& v, const std::string& o) { c.max_cached_solutions = to_int(v, o); }},
        {"--batch_frames", [&](const std::string& v, const std::string& o) { c.batch_frames = to_int(v, o); }},
        {"--profile", [&](const std::string& v, const std::string&) { c.profile_file = v; }},
        {"--rtm_format", [&](const std::string& v, const std::string&) { c.rtm_format = v; }},
    };
    std::map<std::string, bool*> flags = {
        {"--logarithmic", &c.logarithmic}, {"--no_guess", &c.no_guess},   {"--use_cpu", &c.use_cpu},
        {"--parallel_read", &c.parallel_read}, {"--resume", &c.resume}, {"--two_pass", &c.two_pass},
        {"--partition_voxels", &c.partition_voxels}, {"--rtm_bf16", &c.rtm_bf16},
    };
    const std::map<std::string, std::string> alias = {
        {"-o", "--output_file"},           {"-t", "--time_range"},          {"-w", "--wavelength_threshold"},
        {"-d", "--ray_density_threshold"}, {"-r", "--ray_length_threshold"}, {"-m", "--max_iterations"},
        {"-c", "--conv_tolerance"},        {"-l", "--laplacian_file"},      {"-b", "--beta_laplace"},
        {"-R", "--relaxation"},            {"-n", "--raytransfer_name"},    {"-L", "--logarithmic"},
    };

    size_t i = 0;
    for (; i < argv.size(); ++i) {
        std::string tok = argv[i];
        if (tok == "-h" || tok == "--help") {
            c.help = true;
            return c;
        }
        if (tok.size() < 2 || tok[0] != '-') break;  // first positional: the rest are input files
        std::string value;
        bool has_value = false;
        const size_t eq = tok.find('=');
        if (tok.rfind("--", 0) == 0 && eq != std::string::npos) {
            value = tok.substr(eq + 1);
            tok = tok.substr(0, eq);
            has_value = true;
        }
        auto a = alias.find(tok);
        const std::string name = a != alias.end() ? a->second : tok;
        if (auto f = flags.find(name); f != flags.end()) {
            if (has_value) throw Error("Option " + name + " does not take a value.\n" + usage());
            *f->second = true;
        } else if (auto v = valued.find(name); v != valued.end()) {
            if (!has_value) {
                if (i + 1 >= argv.size()) throw Error("Too few arguments for " + name + ".\n" + usage());
                value = argv[++i];
            }
            v->second(value, name);
        } else {
            throw Error("Unknown argument: " + argv[i] + "\n" + usage());
        }
    }
    for (; i < argv.size(); ++i) c.input_files.push_back(argv[i]);

    // validation (reference arguments.cpp:184-248)
    if (c.ray_density_threshold < 0)
        throw Error("Argument ray_density_threshold must be >= 0, " + fmt(c.ray_density_threshold) + " given.");
    if (c.ray_length_threshold < 0)
        throw Error("Argument ray_length_threshold must be >= 0, " + fmt(c.ray_length_threshold) + " given.");
    if (c.max_iterations < 1)
        throw Error("Argument max_iterations must be >= 1, " + std::to_string(c.max_iterations) + " given.");
    if (c.conv_tolerance <= 0)
        throw Error("Argument conv_tolerance must be > 0, " + fmt(c.conv_tolerance) + " given.");
    if (c.relaxation <= 0 || c.relaxation > 1.0)
        throw Error("Argument relaxation must be within (0, 1] interval," + fmt(c.relaxation) + " given.");
    if (c.beta_laplace < 0) throw Error("Argument beta_laplace must be positive.");
    if (c.max_cached_frames <= 0) throw Error("Argument max_cached_frames must be positive.");
    if (c.max_cached_solutions <= 0) throw Error("Argument max_cached_solutions must be positive.");
    if (c.batch_frames < 1) throw Error("Argument batch_frames must be >= 1.");
    if (c.partition_voxels && (c.batch_frames > 1 || c.use_cpu))
        throw Error("Argument partition_voxels applies to the single-frame GPU solver only.");
    if (c.rtm_bf16 && (c.use_cpu || c.partition_voxels))
        throw Error("Argument rtm_bf16 applies to the GPU solvers with pixel-row shards only.");
    if (c.rtm_format != "auto" && c.rtm_format != "dense" && c.rtm_format != "sparse")
        throw Error("Argument rtm_format must be auto, dense or sparse, " + c.rtm_format + " given.");
    if (c.rtm_format == "sparse" && (c.partition_voxels || c.rtm_bf16 || (c.use_cpu && c.batch_frames > 1)))
        throw Error("Argument rtm_format sparse applies to fp32 pixel-row shards (and not to CPU batches).");
    if (c.input_files.size() < 2)
        throw Error("At least two input file, one with RTM and one with image, are required, " +
                    std::to_string(c.input_files.size()) + " given.");
    return c;
}

std::vector<std::array<double, 4>> parse_time_intervals(const std::string& spec) {
    std::vector<std::array<double, 4>> out;
    if (spec.empty()) {
        out.push_back({0.0, std::numeric_limits<double>::infinity(), 0.0, 0.0});
        return out;
    }
    std::vector<std::string> pieces;
    {
        size_t pos = 0;
        while (true) {
            const size_t comma = spec.find(',', pos);
            pieces.push_back(spec.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos));
            if (comma == std::string::npos) break;
            pos = comma + 1;
        }
        if (pieces.size() > 1 && pieces.back().empty()) pieces.pop_back();  // trailing ',' is allowed
    }
    for (const auto& piece : pieces) {
        std::vector<std::string> f;
        size_t pos = 0;
        while (pos < piece.size()) {
            const size_t colon = piece.find(':', pos);
            f.push_back(piece.substr(pos, colon == std::string::npos ? std::string::npos : colon - pos));
            pos = colon == std::string::npos ? piece.size() : colon + 1;
        }
        if (f.size() < 2) throw Error("Unable to recognize a time interval in " + piece + ".");
        if (f.size() > 4) throw Error("Too many values in a time interval: " + piece + ".");
        double v[4] = {0, 0, 0, 0};
        for (size_t k = 0; k < f.size(); ++k) {
            // leading blanks are skipped, trailing characters ignored (std::stod semantics)
            const std::string t = f[k];
            char* end = nullptr;
            const char* beg = t.c_str();
            v[k] = std::strtod(beg, &end);
            if (end == beg) throw Error("Unable to convert " + piece + " to the time interval.");
        }
        if (v[0] < 0) throw Error("Time limits must be positive.");
        if (v[1] <= v[0]) throw Error("The upper limit of the time interval must be higher than the lower one.");
        if (v[2] > v[1] - v[0]) throw Error("Time step must be less or equal to the time interval.");
        if (v[3] > v[2]) throw Error("Synchronization threshold must be less or equal to the time step.");
        out.push_back({v[0], v[1], v[2], v[3]});
    }
    return out;
}

}  // namespace sart
