"""CLI/config parser, time intervals and the row partition (reference arguments.cpp, main.cpp:67-68)."""
import math

import pytest

from mpi_cuda_sartsolver_amd.ops import native
from mpi_cuda_sartsolver_amd.parallel.partition import all_blocks, block_partition, row_partition


@pytest.fixture(scope="module")
def n():
    return native()


def test_defaults_match_reference(n):
    c = n.parse_arguments(["a.h5", "b.h5"])
    assert c.output_file == "solution.h5" and c.time_range == "" and c.laplacian_file == ""
    assert c.wavelength_threshold == 50.0 and c.ray_density_threshold == 1e-6 and c.ray_length_threshold == 1e-6
    assert c.max_iterations == 2000 and c.conv_tolerance == 1e-5 and c.beta_laplace == 2e-2 and c.relaxation == 1.0
    assert c.raytransfer_name == "with_reflections" and c.max_cached_frames == 100 and c.max_cached_solutions == 100
    assert not (c.logarithmic or c.no_guess or c.use_cpu or c.parallel_read or c.resume or c.two_pass)
    assert c.batch_frames == 1 and c.input_files == ["a.h5", "b.h5"]


def test_short_and_long_aliases(n):
    c = n.parse_arguments(["-o", "x.h5", "-t", "1:2", "-w", "3", "-d", "0.5", "-r", "0.25", "-m", "7", "-c", "1e-3",
                           "-l", "lap.h5", "-b", "0.1", "-R", "0.5", "-n", "name", "-L", "--no_guess", "--use_cpu",
                           "--parallel_read", "--max_cached_frames", "3", "--max_cached_solutions=4", "f1", "f2", "f3"])
    assert (c.output_file, c.time_range, c.wavelength_threshold) == ("x.h5", "1:2", 3.0)
    assert (c.ray_density_threshold, c.ray_length_threshold, c.max_iterations) == (0.5, 0.25, 7)
    assert (c.conv_tolerance, c.laplacian_file, c.beta_laplace, c.relaxation) == (1e-3, "lap.h5", 0.1, 0.5)
    assert c.raytransfer_name == "name" and c.logarithmic and c.no_guess and c.use_cpu and c.parallel_read
    assert c.max_cached_frames == 3 and c.max_cached_solutions == 4 and c.input_files == ["f1", "f2", "f3"]
    c2 = n.parse_arguments(["--output_file=y.h5", "--relaxation=1", "--batch_frames", "16", "--resume", "a", "b"])
    assert c2.output_file == "y.h5" and c2.batch_frames == 16 and c2.resume
    assert not c2.rtm_bf16 and n.parse_arguments(["--rtm_bf16", "a", "b"]).rtm_bf16
    assert "--rtm_bf16" in n.usage()
    assert c2.rtm_format == "auto" and n.parse_arguments(["--rtm_format", "sparse", "a", "b"]).rtm_format == "sparse"
    assert n.parse_arguments(["--rtm_format=dense", "a", "b"]).rtm_format == "dense" and "--rtm_format" in n.usage()


@pytest.mark.parametrize("argv,msg", [
    (["-d", "-1", "a", "b"], "ray_density_threshold must be >= 0"),
    (["-r", "-1", "a", "b"], "ray_length_threshold must be >= 0"),
    (["-m", "0", "a", "b"], "max_iterations must be >= 1"),
    (["-c", "0", "a", "b"], "conv_tolerance must be > 0"),
    (["-R", "0", "a", "b"], "relaxation must be within (0, 1]"),
    (["-R", "1.5", "a", "b"], "relaxation must be within (0, 1]"),
    (["-b", "-1", "a", "b"], "beta_laplace must be positive"),
    (["--max_cached_frames", "0", "a", "b"], "max_cached_frames must be positive"),
    (["--max_cached_solutions", "0", "a", "b"], "max_cached_solutions must be positive"),
    (["a"], "At least two input file"),
    (["-m", "abc", "a", "b"], "Failed to parse"),
    (["--bogus", "a", "b"], "Unknown argument"),
    (["-m"], "Too few arguments"),
    (["--rtm_bf16", "--use_cpu", "a", "b"], "rtm_bf16 applies to the GPU solvers with pixel-row shards"),
    (["--rtm_bf16", "--partition_voxels", "a", "b"], "rtm_bf16 applies to the GPU solvers with pixel-row shards"),
    (["--rtm_format", "csr", "a", "b"], "rtm_format must be auto, dense or sparse"),
    (["--rtm_format", "sparse", "--batch_frames", "16", "--use_cpu", "a", "b"], "rtm_format sparse applies to fp32"),
    (["--rtm_format", "sparse", "--partition_voxels", "a", "b"], "rtm_format sparse applies to fp32"),
])
def test_validation_errors(n, argv, msg):
    with pytest.raises(RuntimeError, match=msg.replace("(", r"\(").replace(")", r"\)").replace("]", r"\]")):
        n.parse_arguments(argv)


def test_help(n):
    assert n.parse_arguments(["--help"]).help
    assert "--ray_density_threshold" in n.usage()


def test_time_intervals(n):
    assert n.parse_time_intervals("") == [[0.0, math.inf, 0.0, 0.0]]
    assert n.parse_time_intervals("20.5:40.1, 45.2:51:3:0.05,") == [[20.5, 40.1, 0, 0], [45.2, 51, 3, 0.05]]
    assert n.parse_time_intervals("1:2:0.5") == [[1, 2, 0.5, 0]]


@pytest.mark.parametrize("spec,msg", [
    ("5", "Unable to recognize a time interval"),
    ("1:2:0.1:0.05:9", "Too many values"),
    ("-1:2", "Time limits must be positive"),
    ("3:2", "upper limit of the time interval must be higher"),
    ("1:2:5", "Time step must be less or equal"),
    ("1:2:0.1:0.5", "Synchronization threshold must be less or equal"),
    ("a:b", "Unable to convert"),
])
def test_time_interval_errors(n, spec, msg):
    with pytest.raises(RuntimeError, match=msg):
        n.parse_time_intervals(spec)


@pytest.mark.parametrize("npix,nproc", [(10, 3), (7, 7), (1000, 8), (5, 1), (65537, 8)])
def test_row_partition_matches_reference_formula(npix, nproc):
    blocks = all_blocks(npix, nproc)
    assert sum(b.size for b in blocks) == npix
    for r, b in enumerate(blocks):
        off = r * (npix // nproc) + min(r, npix % nproc)
        size = npix // nproc + 1 if r < npix % nproc else npix // nproc
        assert (b.offset, b.size) == (off, size) == (row_partition(npix, nproc, r).offset, size)
    assert all(blocks[i].stop == blocks[i + 1].offset for i in range(nproc - 1))
    with pytest.raises(ValueError):
        block_partition(npix, nproc, nproc)
