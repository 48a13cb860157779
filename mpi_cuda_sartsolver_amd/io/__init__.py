"""HDF5 inputs/outputs backed by the native C++ module (HDF5 C API)."""
