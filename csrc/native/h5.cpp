#include "h5.hpp"

#include <mutex>

namespace sart {

std::recursive_mutex& h5_mutex() {
    static std::recursive_mutex m;
    return m;
}


bool have_hdf5() {
#ifdef SART_HAVE_HDF5
    return true;
#else
    return false;
#endif
}

#ifdef SART_HAVE_HDF5

void H5Id::reset() {
    if (id_ < 0) return;
    switch (kind_) {
        case kFile: H5Fclose(id_); break;
        case kGroup: H5Gclose(id_); break;
        case kDataset: H5Dclose(id_); break;
        case kSpace: H5Sclose(id_); break;
        case kAttr: H5Aclose(id_); break;
        case kType: H5Tclose(id_); break;
        case kPlist: H5Pclose(id_); break;
        case kObject: H5Oclose(id_); break;
    }
    id_ = -1;
}

void h5_quiet() {
    static std::once_flag once;
    std::call_once(once, [] { H5Eset_auto2(H5E_DEFAULT, nullptr, nullptr); });
}

static void check(herr_t st, const std::string& what) {
    if (st < 0) throw Error("HDF5 error: " + what);
}

H5Id h5_open_file(const std::string& path, bool write) {
    h5_quiet();
    hid_t f = H5Fopen(path.c_str(), write ? H5F_ACC_RDWR : H5F_ACC_RDONLY, H5P_DEFAULT);
    if (f < 0) throw Error("Unable to open HDF5 file " + path + ".");
    return H5Id(f, H5Id::kFile);
}

H5Id h5_create_file(const std::string& path) {
    h5_quiet();
    hid_t f = H5Fcreate(path.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    if (f < 0) throw Error("Unable to create HDF5 file " + path + ".");
    return H5Id(f, H5Id::kFile);
}

bool h5_exists(hid_t loc, const std::string& path) {
    // check every component, H5Lexists requires the intermediate links to exist
    size_t pos = 0;
    while (true) {
        size_t next = path.find('/', pos);
        const std::string part = path.substr(0, next);
        if (!part.empty()) {
            htri_t e = H5Lexists(loc, part.c_str(), H5P_DEFAULT);
            if (e <= 0) return false;
        }
        if (next == std::string::npos) return true;
        pos = next + 1;
    }
}

bool h5_attr_exists(hid_t loc, const std::string& obj_path, const std::string& name) {
    if (!h5_exists(loc, obj_path)) return false;
    htri_t e = H5Aexists_by_name(loc, obj_path.c_str(), name.c_str(), H5P_DEFAULT);
    return e > 0;
}

H5Id h5_open_group(hid_t loc, const std::string& path) {
    hid_t g = H5Gopen2(loc, path.c_str(), H5P_DEFAULT);
    if (g < 0) throw Error("Unable to open HDF5 group " + path + ".");
    return H5Id(g, H5Id::kGroup);
}

H5Id h5_open_dataset(hid_t loc, const std::string& path) {
    hid_t d = H5Dopen2(loc, path.c_str(), H5P_DEFAULT);
    if (d < 0) throw Error("Unable to open HDF5 dataset " + path + ".");
    return H5Id(d, H5Id::kDataset);
}

std::vector<hsize_t> h5_dims(hid_t dset) {
    H5Id sp(H5Dget_space(dset), H5Id::kSpace);
    const int nd = H5Sget_simple_extent_ndims(sp);
    if (nd < 0) throw Error("HDF5 error: unable to query dataset rank");
    std::vector<hsize_t> dims(nd);
    if (nd) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
    return dims;
}

static H5Id open_attr(hid_t loc, const std::string& obj, const std::string& name) {
    hid_t a = H5Aopen_by_name(loc, obj.c_str(), name.c_str(), H5P_DEFAULT, H5P_DEFAULT);
    if (a < 0) throw Error("Unable to open attribute " + name + " of " + obj + ".");
    return H5Id(a, H5Id::kAttr);
}

double h5_attr_double(hid_t loc, const std::string& obj, const std::string& name) {
    H5Id a = open_attr(loc, obj, name);
    double v = 0;
    check(H5Aread(a, H5T_NATIVE_DOUBLE, &v), "reading attribute " + name);
    return v;
}

uint64_t h5_attr_u64(hid_t loc, const std::string& obj, const std::string& name) {
    H5Id a = open_attr(loc, obj, name);
    unsigned long long v = 0;
    check(H5Aread(a, H5T_NATIVE_ULLONG, &v), "reading attribute " + name);
    return (uint64_t)v;
}

int64_t h5_attr_i64(hid_t loc, const std::string& obj, const std::string& name) {
    H5Id a = open_attr(loc, obj, name);
    long long v = 0;
    check(H5Aread(a, H5T_NATIVE_LLONG, &v), "reading attribute " + name);
    return (int64_t)v;
}

std::string h5_attr_string(hid_t loc, const std::string& obj, const std::string& name) {
    H5Id a = open_attr(loc, obj, name);
    H5Id ft(H5Aget_type(a), H5Id::kType);
    if (H5Tget_class(ft) != H5T_STRING) throw Error("Attribute " + name + " of " + obj + " is not a string.");
    if (H5Tis_variable_str(ft) > 0) {
        H5Id mt(H5Tcopy(H5T_C_S1), H5Id::kType);
        H5Tset_size(mt, H5T_VARIABLE);
        H5Tset_cset(mt, H5Tget_cset(ft));
        char* buf = nullptr;
        check(H5Aread(a, mt, &buf), "reading string attribute " + name);
        std::string s = buf ? std::string(buf) : std::string();
        if (buf) H5free_memory(buf);
        return s;
    }
    const size_t n = H5Tget_size(ft);
    std::string s(n, '\0');
    H5Id mt(H5Tcopy(H5T_C_S1), H5Id::kType);
    H5Tset_size(mt, n);
    check(H5Aread(a, mt, s.data()), "reading string attribute " + name);
    const size_t z = s.find('\0');
    if (z != std::string::npos) s.resize(z);
    while (!s.empty() && s.back() == ' ') s.pop_back();  // space-padded fixed strings
    return s;
}

template <typename T>
static std::vector<T> read_all(hid_t loc, const std::string& path, hid_t memtype) {
    H5Id d = h5_open_dataset(loc, path);
    const auto dims = h5_dims(d);
    size_t n = 1;
    for (auto v : dims) n *= v;
    std::vector<T> out(n);
    if (n) check(H5Dread(d, memtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.data()), "reading dataset " + path);
    return out;
}

std::vector<double> h5_read_f64(hid_t loc, const std::string& path) { return read_all<double>(loc, path, H5T_NATIVE_DOUBLE); }
std::vector<float> h5_read_f32(hid_t loc, const std::string& path) { return read_all<float>(loc, path, H5T_NATIVE_FLOAT); }
std::vector<uint64_t> h5_read_u64(hid_t loc, const std::string& path) {
    return read_all<uint64_t>(loc, path, H5T_NATIVE_UINT64);
}
std::vector<int64_t> h5_read_i64(hid_t loc, const std::string& path) { return read_all<int64_t>(loc, path, H5T_NATIVE_INT64); }
std::vector<int32_t> h5_read_i32(hid_t loc, const std::string& path) { return read_all<int32_t>(loc, path, H5T_NATIVE_INT32); }

void h5_read_rows_f32(hid_t dset, uint64_t row0, uint64_t nrows, uint64_t ncols, float* out, uint64_t ld,
                      uint64_t col0) {
    h5_read_block_f32(dset, row0, nrows, 0, ncols, out, ld, col0);
}

void h5_read_block_f32(hid_t dset, uint64_t row0, uint64_t nrows, uint64_t fcol0, uint64_t ncols, float* out,
                       uint64_t ld, uint64_t col0) {
    if (nrows == 0 || ncols == 0) return;
    H5Id fsp(H5Dget_space(dset), H5Id::kSpace);
    hsize_t foff[2] = {row0, fcol0}, fcnt[2] = {nrows, ncols};
    check(H5Sselect_hyperslab(fsp, H5S_SELECT_SET, foff, nullptr, fcnt, nullptr), "selecting RTM rows");
    hsize_t mdims[2] = {nrows, ld};
    H5Id msp(H5Screate_simple(2, mdims, nullptr), H5Id::kSpace);
    hsize_t moff[2] = {0, col0}, mcnt[2] = {nrows, ncols};
    check(H5Sselect_hyperslab(msp, H5S_SELECT_SET, moff, nullptr, mcnt, nullptr), "selecting memory rows");
    check(H5Dread(dset, H5T_NATIVE_FLOAT, msp, fsp, H5P_DEFAULT, out), "reading RTM rows");
}

void h5_read_frame_f64(hid_t dset, uint64_t index, double* out, uint64_t frame_size) {
    H5Id fsp(H5Dget_space(dset), H5Id::kSpace);
    const int nd = H5Sget_simple_extent_ndims(fsp);
    std::vector<hsize_t> dims(nd);
    H5Sget_simple_extent_dims(fsp, dims.data(), nullptr);
    std::vector<hsize_t> off(nd, 0), cnt(dims);
    off[0] = index;
    cnt[0] = 1;
    check(H5Sselect_hyperslab(fsp, H5S_SELECT_SET, off.data(), nullptr, cnt.data(), nullptr), "selecting frame");
    hsize_t m = frame_size;
    H5Id msp(H5Screate_simple(1, &m, nullptr), H5Id::kSpace);
    check(H5Dread(dset, H5T_NATIVE_DOUBLE, msp, fsp, H5P_DEFAULT, out), "reading image frame");
}

static void read_range(hid_t dset, uint64_t off, uint64_t n, hid_t memtype, void* out) {
    if (n == 0) return;
    H5Id fsp(H5Dget_space(dset), H5Id::kSpace);
    hsize_t o = off, c = n;
    check(H5Sselect_hyperslab(fsp, H5S_SELECT_SET, &o, nullptr, &c, nullptr), "selecting a range");
    H5Id msp(H5Screate_simple(1, &c, nullptr), H5Id::kSpace);
    check(H5Dread(dset, memtype, msp, fsp, H5P_DEFAULT, out), "reading a range");
}

void h5_read_range_u64(hid_t dset, uint64_t off, uint64_t n, uint64_t* out) {
    read_range(dset, off, n, H5T_NATIVE_UINT64, out);
}

void h5_read_range_f32(hid_t dset, uint64_t off, uint64_t n, float* out) {
    read_range(dset, off, n, H5T_NATIVE_FLOAT, out);
}

H5Id h5_create_group(hid_t loc, const std::string& path) {
    hid_t g = H5Gcreate2(loc, path.c_str(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT);
    if (g < 0) throw Error("Unable to create HDF5 group " + path + ".");
    return H5Id(g, H5Id::kGroup);
}

static void write_scalar_attr(hid_t obj, const std::string& name, hid_t ftype, hid_t mtype, const void* v) {
    H5Id sp(H5Screate(H5S_SCALAR), H5Id::kSpace);
    if (H5Aexists(obj, name.c_str()) > 0) H5Adelete(obj, name.c_str());
    H5Id a(H5Acreate2(obj, name.c_str(), ftype, sp, H5P_DEFAULT, H5P_DEFAULT), H5Id::kAttr);
    if (!a.valid()) throw Error("Unable to create attribute " + name + ".");
    check(H5Awrite(a, mtype, v), "writing attribute " + name);
}

void h5_write_attr_double(hid_t obj, const std::string& name, double v) {
    write_scalar_attr(obj, name, H5T_IEEE_F64LE, H5T_NATIVE_DOUBLE, &v);
}
void h5_write_attr_u64(hid_t obj, const std::string& name, uint64_t v) {
    write_scalar_attr(obj, name, H5T_STD_U64LE, H5T_NATIVE_UINT64, &v);
}
void h5_write_attr_i32(hid_t obj, const std::string& name, int32_t v) {
    write_scalar_attr(obj, name, H5T_STD_I32LE, H5T_NATIVE_INT32, &v);
}
void h5_write_attr_string(hid_t obj, const std::string& name, const std::string& v) {
    H5Id t(H5Tcopy(H5T_C_S1), H5Id::kType);
    H5Tset_size(t, H5T_VARIABLE);
    const char* p = v.c_str();
    write_scalar_attr(obj, name, t, t, &p);
}

static void write_ds(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, hid_t ftype,
                     hid_t mtype, const void* data) {
    std::vector<hsize_t> d(dims.begin(), dims.end());
    H5Id sp(H5Screate_simple((int)d.size(), d.data(), nullptr), H5Id::kSpace);
    H5Id ds(H5Dcreate2(loc, path.c_str(), ftype, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Id::kDataset);
    if (!ds.valid()) throw Error("Unable to create HDF5 dataset " + path + ".");
    size_t n = 1;
    for (auto v : dims) n *= v;
    if (n) check(H5Dwrite(ds, mtype, H5S_ALL, H5S_ALL, H5P_DEFAULT, data), "writing dataset " + path);
}

void h5_write_f64(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const double* data) {
    write_ds(loc, path, dims, H5T_IEEE_F64LE, H5T_NATIVE_DOUBLE, data);
}
void h5_write_f32(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const float* data) {
    write_ds(loc, path, dims, H5T_IEEE_F32LE, H5T_NATIVE_FLOAT, data);
}
void h5_write_u64(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const uint64_t* data) {
    write_ds(loc, path, dims, H5T_STD_U64LE, H5T_NATIVE_UINT64, data);
}
void h5_write_i32(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const int32_t* data) {
    write_ds(loc, path, dims, H5T_STD_I32LE, H5T_NATIVE_INT32, data);
}
void h5_write_u8(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, const uint8_t* data) {
    write_ds(loc, path, dims, H5T_STD_U8LE, H5T_NATIVE_UINT8, data);
}

H5Id h5_create_dataset(hid_t loc, const std::string& path, const std::vector<uint64_t>& dims, hid_t ftype) {
    std::vector<hsize_t> d(dims.begin(), dims.end());
    H5Id sp(H5Screate_simple((int)d.size(), d.data(), nullptr), H5Id::kSpace);
    H5Id ds(H5Dcreate2(loc, path.c_str(), ftype, sp, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), H5Id::kDataset);
    if (!ds.valid()) throw Error("Unable to create HDF5 dataset " + path + ".");
    return ds;
}

void h5_write_box(hid_t dset, const std::vector<uint64_t>& off, const std::vector<uint64_t>& cnt, hid_t mtype,
                  const void* data) {
    if (off.size() != cnt.size() || off.empty()) throw Error("h5_write_box: bad box");
    size_t n = 1;
    for (auto v : cnt) n *= v;
    if (n == 0) return;
    std::vector<hsize_t> o(off.begin(), off.end()), c(cnt.begin(), cnt.end());
    H5Id fsp(H5Dget_space(dset), H5Id::kSpace);
    check(H5Sselect_hyperslab(fsp, H5S_SELECT_SET, o.data(), nullptr, c.data(), nullptr), "selecting a box");
    H5Id msp(H5Screate_simple((int)c.size(), c.data(), nullptr), H5Id::kSpace);
    check(H5Dwrite(dset, mtype, msp, fsp, H5P_DEFAULT, data), "writing a box");
}

#endif  // SART_HAVE_HDF5

}  // namespace sart
