"""Solvers and problem data: RTM shard, Laplacian, GPU/CPU SART engines, fp64 oracles."""
