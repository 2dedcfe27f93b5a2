// datafile.cpp -- RBIN, classic netCDF and netCDF-4/HDF5 readers (see datafile.hpp).
//
// Classic netCDF follows the published file-format specification (header: magic, numrecs, dim_list,
// gatt_list, var_list; big-endian data; record variables interleaved per record).  netCDF-4 files are HDF5
// files whose netCDF variables are the root group's datasets; they are read through the HDF5 C API,
// resolved with dlopen/dlsym from libhdf5 (RRTMGPNN_HDF5_LIB, else the loader path, else the image's
// /opt/conda/lib).  Dimension-scale datasets and variable-length strings (which the reference never reads
// on this path) are skipped.
#include "datafile.hpp"

#include <dlfcn.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <fstream>

#include "internal.hpp"

namespace rrtmgpnn {

std::vector<float> to_float(const DataVar &v)
{
  std::vector<float> out(v.count());
  if (v.dtype == kF32) std::memcpy(out.data(), v.data.data(), out.size() * 4);
  else if (v.dtype == kI32)
    for (size_t i = 0; i < out.size(); i++) out[i] = (float)((const int32_t *)v.data.data())[i];
  return out;
}

std::vector<int> to_int(const DataVar &v)
{
  std::vector<int> out(v.count());
  if (v.dtype == kI32) std::memcpy(out.data(), v.data.data(), out.size() * 4);
  else if (v.dtype == kF32)
    for (size_t i = 0; i < out.size(); i++) out[i] = (int)((const float *)v.data.data())[i];
  return out;
}

// ---------------------------------------------------------------------------------------------
// RBIN: "RBIN" u32 version=1, u32 count, then per entry: char name[64], u32 dtype (0 f32, 1 i32, 2 u8),
// u32 ndim, u32 dims[ndim], data (little endian)
// ---------------------------------------------------------------------------------------------
static int read_rbin(const char *path, DataFile &out)
{
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(RRTMGPNN_ERR_IO, std::string("cannot open ") + path);
  char magic[4];
  uint32_t ver = 0, count = 0;
  f.read(magic, 4);
  f.read((char *)&ver, 4);
  f.read((char *)&count, 4);
  if (!f || std::memcmp(magic, "RBIN", 4) != 0 || ver != 1)
    return fail(RRTMGPNN_ERR_IO, std::string(path) + ": not an RBIN v1 file");
  for (uint32_t e = 0; e < count; e++) {
    char name[64];
    uint32_t dt = 0, nd = 0;
    f.read(name, 64);
    f.read((char *)&dt, 4);
    f.read((char *)&nd, 4);
    if (!f || dt > 2 || nd > 8) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": corrupt entry header");
    DataVar a;
    a.dtype = (int)dt;
    for (uint32_t i = 0; i < nd; i++) {
      uint32_t d = 0;
      f.read((char *)&d, 4);
      a.dims.push_back((int)d);
    }
    a.data.resize(a.count() * (dt == 2 ? 1 : 4));
    f.read(a.data.data(), (std::streamsize)a.data.size());
    if (!f) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": truncated");
    name[63] = 0;
    out.vars[std::string(name)] = std::move(a);
  }
  return RRTMGPNN_OK;
}

// ---------------------------------------------------------------------------------------------
// Classic netCDF (CDF-1, CDF-2 64-bit offsets, CDF-5 64-bit data)
// ---------------------------------------------------------------------------------------------
namespace {

enum NcType { NC_BYTE = 1, NC_CHAR, NC_SHORT, NC_INT, NC_FLOAT, NC_DOUBLE, NC_UBYTE, NC_USHORT, NC_UINT,
              NC_INT64, NC_UINT64 };

int nc_size(int t)
{
  switch (t) {
    case NC_BYTE: case NC_CHAR: case NC_UBYTE: return 1;
    case NC_SHORT: case NC_USHORT: return 2;
    case NC_INT: case NC_FLOAT: case NC_UINT: return 4;
    case NC_DOUBLE: case NC_INT64: case NC_UINT64: return 8;
    default: return 0;
  }
}

struct Cursor {
  const std::vector<unsigned char> &b;
  size_t p = 0;
  bool ok = true;
  int version = 1;
  uint64_t be(int n)
  {
    if (p + n > b.size()) { ok = false; return 0; }
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | b[p + i];
    p += n;
    return v;
  }
  uint64_t u32() { return be(4); }
  uint64_t nonneg() { return be(version == 5 ? 8 : 4); }  // NON_NEG: 8 bytes in CDF-5
  uint64_t offset() { return be(version == 1 ? 4 : 8); }
  std::string name()
  {
    uint64_t n = nonneg();
    if (p + n > b.size()) { ok = false; return ""; }
    std::string s((const char *)&b[p], (size_t)n);
    p += (n + 3) / 4 * 4;
    return s;
  }
  void skip_values(int type, uint64_t n) { p += (n * nc_size(type) + 3) / 4 * 4; }
};

// decode n big-endian values of `type` at src into float or int32 (C casts)
void decode(const unsigned char *src, int type, size_t n, DataVar &v)
{
  const int sz = nc_size(type);
  if (type == NC_CHAR) {
    v.dtype = kChar;
    v.data.assign((const char *)src, (const char *)src + n);
    return;
  }
  const bool integral = type != NC_FLOAT && type != NC_DOUBLE;
  v.dtype = integral ? kI32 : kF32;
  v.data.resize(n * 4);
  for (size_t i = 0; i < n; i++) {
    uint64_t u = 0;
    for (int k = 0; k < sz; k++) u = (u << 8) | src[i * sz + k];
    float f = 0.0f;
    int32_t iv = 0;
    switch (type) {
      case NC_BYTE: iv = (int8_t)u; break;
      case NC_UBYTE: iv = (uint8_t)u; break;
      case NC_SHORT: iv = (int16_t)u; break;
      case NC_USHORT: iv = (uint16_t)u; break;
      case NC_INT: iv = (int32_t)u; break;
      case NC_UINT: iv = (int32_t)(uint32_t)u; break;
      case NC_INT64: iv = (int32_t)(int64_t)u; break;
      case NC_UINT64: iv = (int32_t)u; break;
      case NC_FLOAT: { uint32_t w = (uint32_t)u; std::memcpy(&f, &w, 4); break; }
      case NC_DOUBLE: { double d; std::memcpy(&d, &u, 8); f = (float)d; break; }
    }
    if (integral) std::memcpy(&v.data[i * 4], &iv, 4);
    else std::memcpy(&v.data[i * 4], &f, 4);
  }
}

std::string att_text(const unsigned char *src, int type, uint64_t n)
{
  if (type == NC_CHAR) {
    std::string s((const char *)src, (size_t)n);
    while (!s.empty() && s.back() == '\0') s.pop_back();
    return s;
  }
  return "";  // numeric attributes are not needed on this path
}

}  // namespace

static int read_cdf(const char *path, const std::vector<unsigned char> &buf, DataFile &out)
{
  Cursor c{buf};
  c.version = buf[3];  // magic "CDF" + version byte
  c.p = 4;
  const std::string where = std::string(path) + ": ";
  uint64_t numrecs = c.nonneg();
  if (numrecs == 0xFFFFFFFFull) numrecs = 0;  // STREAMING: no complete records recorded
  struct Dim { std::string name; uint64_t len; };
  std::vector<Dim> dims;
  auto att_list = [&](const std::string &owner) {
    uint64_t tag = c.u32(), n = c.nonneg();
    if (tag == 0) return;
    for (uint64_t i = 0; i < n && c.ok; i++) {
      std::string an = c.name();
      int t = (int)c.u32();
      uint64_t nv = c.nonneg();
      if (c.p + nv * nc_size(t) > buf.size()) { c.ok = false; return; }
      std::string s = att_text(&buf[c.p], t, nv);
      if (t == NC_CHAR) out.atts[owner + ":" + an] = s;
      c.skip_values(t, nv);
    }
  };
  uint64_t tag = c.u32(), n = c.nonneg();
  if (tag == 0x0A)
    for (uint64_t i = 0; i < n && c.ok; i++) {
      std::string dn = c.name();
      dims.push_back({dn, c.nonneg()});
    }
  att_list("");
  struct Var { std::string name; std::vector<uint64_t> dimids; int type; uint64_t vsize, begin; };
  std::vector<Var> vars;
  tag = c.u32();
  n = c.nonneg();
  if (tag == 0x0B)
    for (uint64_t i = 0; i < n && c.ok; i++) {
      Var v;
      v.name = c.name();
      uint64_t nd = c.nonneg();
      for (uint64_t k = 0; k < nd; k++) v.dimids.push_back(c.nonneg());
      att_list(v.name);
      v.type = (int)c.u32();
      v.vsize = c.nonneg();
      v.begin = c.offset();
      vars.push_back(v);
    }
  if (!c.ok) return fail(RRTMGPNN_ERR_IO, where + "corrupt classic netCDF header");
  // record variables: first dimension of length 0 (the unlimited one); records interleave all of them
  uint64_t recsize = 0;
  int nrecvars = 0;
  for (const Var &v : vars)
    if (!v.dimids.empty() && v.dimids[0] < dims.size() && dims[v.dimids[0]].len == 0) {
      recsize += v.vsize;
      nrecvars++;
    }
  for (const Var &v : vars) {
    if (nc_size(v.type) == 0) return fail(RRTMGPNN_ERR_IO, where + v.name + ": unsupported netCDF type");
    DataVar dv;
    bool rec = false;
    size_t per = 1;  // elements per record (or in total for fixed-size variables)
    for (size_t k = 0; k < v.dimids.size(); k++) {
      if (v.dimids[k] >= dims.size()) return fail(RRTMGPNN_ERR_IO, where + v.name + ": bad dimension id");
      uint64_t len = dims[v.dimids[k]].len;
      if (k == 0 && len == 0) {
        rec = true;
        len = numrecs;
      } else {
        per *= (size_t)len;
      }
      dv.dims.push_back((int)len);
    }
    const size_t esz = (size_t)nc_size(v.type);
    std::vector<unsigned char> raw;
    if (!rec) {
      if (v.begin + per * esz > buf.size()) return fail(RRTMGPNN_ERR_IO, where + v.name + ": truncated data");
      raw.assign(buf.begin() + v.begin, buf.begin() + v.begin + per * esz);
    } else {
      // one record variable alone is not padded (special case of the format); otherwise stride = recsize
      const uint64_t stride = nrecvars == 1 ? per * esz : recsize;
      for (uint64_t r = 0; r < numrecs; r++) {
        uint64_t at = v.begin + r * stride;
        if (at + per * esz > buf.size()) return fail(RRTMGPNN_ERR_IO, where + v.name + ": truncated record");
        raw.insert(raw.end(), buf.begin() + at, buf.begin() + at + per * esz);
      }
    }
    decode(raw.data(), v.type, raw.size() / esz, dv);
    out.vars[v.name] = std::move(dv);
  }
  return RRTMGPNN_OK;
}

// ---------------------------------------------------------------------------------------------
// netCDF-4 / HDF5 through the HDF5 C API (run-time bound)
// ---------------------------------------------------------------------------------------------
namespace {

typedef int64_t hid_t;
typedef int herr_t;
typedef int htri_t;
typedef unsigned long long hsize_t;
struct H5GInfo {  // H5G_info_t (HDF5 1.10+): storage type, number of links, max creation order, mounted
  int storage_type;
  hsize_t nlinks;
  int64_t max_corder;
  int mounted;
};
typedef herr_t (*H5AOp)(hid_t, const char *, const void *, void *);

struct H5Api {
  void *lib = nullptr;
  herr_t (*open)();
  hid_t (*Fopen)(const char *, unsigned, hid_t);
  herr_t (*Fclose)(hid_t);
  herr_t (*Eset_auto2)(hid_t, void *, void *);
  herr_t (*Gget_info)(hid_t, H5GInfo *);
  long (*Lget_name_by_idx)(hid_t, const char *, int, int, hsize_t, char *, size_t, hid_t);
  hid_t (*Dopen2)(hid_t, const char *, hid_t);
  herr_t (*Dclose)(hid_t);
  hid_t (*Dget_space)(hid_t);
  hid_t (*Dget_type)(hid_t);
  herr_t (*Dread)(hid_t, hid_t, hid_t, hid_t, hid_t, void *);
  int (*Sget_simple_extent_ndims)(hid_t);
  int (*Sget_simple_extent_dims)(hid_t, hsize_t *, hsize_t *);
  herr_t (*Sclose)(hid_t);
  int (*Tget_class)(hid_t);
  size_t (*Tget_size)(hid_t);
  htri_t (*Tis_variable_str)(hid_t);
  herr_t (*Tclose)(hid_t);
  herr_t (*Aiterate2)(hid_t, int, int, hsize_t *, H5AOp, void *);
  hid_t (*Aopen)(hid_t, const char *, hid_t);
  hid_t (*Aget_type)(hid_t);
  herr_t (*Aread)(hid_t, hid_t, void *);
  herr_t (*Aclose)(hid_t);
  hid_t native_float = -1, native_int = -1;
};

const char *h5_load(H5Api &h)
{
  if (h.lib) return nullptr;
  const char *env = std::getenv("RRTMGPNN_HDF5_LIB");
  const char *cands[] = {env, "libhdf5.so", "libhdf5.so.103", "/opt/conda/lib/libhdf5.so"};
  for (const char *c : cands)
    if (c && (h.lib = dlopen(c, RTLD_NOW | RTLD_LOCAL))) break;
  if (!h.lib) return "netCDF-4 file needs the HDF5 C library (set RRTMGPNN_HDF5_LIB to libhdf5.so)";
  bool ok = true;
  auto sym = [&](const char *n) {
    void *p = dlsym(h.lib, n);
    if (!p) ok = false;
    return p;
  };
#define H5SYM(field, name) h.field = (decltype(h.field))sym(name)
  H5SYM(open, "H5open");
  H5SYM(Fopen, "H5Fopen");
  H5SYM(Fclose, "H5Fclose");
  H5SYM(Eset_auto2, "H5Eset_auto2");
  H5SYM(Gget_info, "H5Gget_info");
  H5SYM(Lget_name_by_idx, "H5Lget_name_by_idx");
  H5SYM(Dopen2, "H5Dopen2");
  H5SYM(Dclose, "H5Dclose");
  H5SYM(Dget_space, "H5Dget_space");
  H5SYM(Dget_type, "H5Dget_type");
  H5SYM(Dread, "H5Dread");
  H5SYM(Sget_simple_extent_ndims, "H5Sget_simple_extent_ndims");
  H5SYM(Sget_simple_extent_dims, "H5Sget_simple_extent_dims");
  H5SYM(Sclose, "H5Sclose");
  H5SYM(Tget_class, "H5Tget_class");
  H5SYM(Tget_size, "H5Tget_size");
  H5SYM(Tis_variable_str, "H5Tis_variable_str");
  H5SYM(Tclose, "H5Tclose");
  H5SYM(Aiterate2, "H5Aiterate2");
  H5SYM(Aopen, "H5Aopen");
  H5SYM(Aget_type, "H5Aget_type");
  H5SYM(Aread, "H5Aread");
  H5SYM(Aclose, "H5Aclose");
#undef H5SYM
  if (!ok || h.open() < 0) {
    dlclose(h.lib);
    h.lib = nullptr;
    return "libhdf5 lacks a required symbol";
  }
  hid_t *nf = (hid_t *)dlsym(h.lib, "H5T_NATIVE_FLOAT_g"), *ni = (hid_t *)dlsym(h.lib, "H5T_NATIVE_INT_g");
  if (!nf || !ni) return "libhdf5 lacks H5T_NATIVE_FLOAT_g / H5T_NATIVE_INT_g";
  h.native_float = *nf;
  h.native_int = *ni;
  h.Eset_auto2(0, nullptr, nullptr);  // no HDF5 error-stack printing: failures are reported here
  return nullptr;
}

H5Api g_h5;

constexpr int kH5Integer = 0, kH5Float = 1, kH5String = 3;

struct AttCollect {
  H5Api *h;
  std::string owner;
  std::map<std::string, std::string> *atts;
};

herr_t collect_att(hid_t loc, const char *name, const void *, void *op)
{
  AttCollect *a = (AttCollect *)op;
  H5Api &h = *a->h;
  hid_t at = h.Aopen(loc, name, 0);
  if (at < 0) return 0;
  hid_t t = h.Aget_type(at);
  if (h.Tget_class(t) == kH5String && h.Tis_variable_str(t) <= 0) {
    size_t n = h.Tget_size(t);
    std::vector<char> s(n + 1, 0);
    if (h.Aread(at, t, s.data()) >= 0) (*a->atts)[a->owner + ":" + name] = std::string(s.data());
  }
  h.Tclose(t);
  h.Aclose(at);
  return 0;
}

}  // namespace

static int read_hdf5(const char *path, DataFile &out)
{
  const std::string where = std::string(path) + ": ";
  if (const char *e = h5_load(g_h5)) return fail(RRTMGPNN_ERR_IO, where + e);
  H5Api &h = g_h5;
  hid_t f = h.Fopen(path, 0u /* H5F_ACC_RDONLY */, 0 /* H5P_DEFAULT */);
  if (f < 0) return fail(RRTMGPNN_ERR_IO, where + "cannot open as HDF5");
  H5GInfo gi{};
  int rc = RRTMGPNN_OK;
  if (h.Gget_info(f, &gi) < 0) rc = fail(RRTMGPNN_ERR_IO, where + "cannot list the root group");
  AttCollect ga{&h, "", &out.atts};
  hsize_t aidx = 0;
  h.Aiterate2(f, 0, 0, &aidx, collect_att, &ga);
  for (hsize_t i = 0; rc == RRTMGPNN_OK && i < gi.nlinks; i++) {
    char name[256];
    if (h.Lget_name_by_idx(f, ".", 0, 0, i, name, sizeof(name), 0) < 0) continue;
    hid_t d = h.Dopen2(f, name, 0);
    if (d < 0) continue;  // a group or another non-dataset object
    hid_t sp = h.Dget_space(d), t = h.Dget_type(d);
    const int cls = h.Tget_class(t);
    const int nd = h.Sget_simple_extent_ndims(sp);
    DataVar v;
    bool keep = nd >= 0 && nd <= 8;
    if (keep) {
      hsize_t dd[8];
      h.Sget_simple_extent_dims(sp, dd, nullptr);
      for (int k = 0; k < nd; k++) v.dims.push_back((int)dd[k]);
    }
    if (keep && (cls == kH5Float || cls == kH5Integer)) {
      v.dtype = cls == kH5Float ? kF32 : kI32;
      v.data.resize(v.count() * 4);
      if (h.Dread(d, cls == kH5Float ? h.native_float : h.native_int, 0, 0, 0, v.data.data()) < 0)
        rc = fail(RRTMGPNN_ERR_IO, where + name + ": read failed");
    } else if (keep && cls == kH5String && h.Tis_variable_str(t) <= 0) {
      const size_t sz = h.Tget_size(t);  // netCDF char variables: fixed strings of one byte
      v.dtype = kChar;
      v.data.resize(v.count() * sz);
      if (sz > 1) v.dims.push_back((int)sz);
      if (h.Dread(d, t, 0, 0, 0, v.data.data()) < 0) rc = fail(RRTMGPNN_ERR_IO, where + name + ": read failed");
    } else {
      keep = false;  // variable-length strings, compounds: not on this path
    }
    if (keep && rc == RRTMGPNN_OK) {
      AttCollect va{&h, name, &out.atts};
      hsize_t idx = 0;
      h.Aiterate2(d, 0, 0, &idx, collect_att, &va);
      // netCDF-4 dimension scales without a coordinate variable are not netCDF variables
      auto it = out.atts.find(std::string(name) + ":NAME");
      const bool dim_only = it != out.atts.end() &&
                            it->second.find("This is a netCDF dimension but not a netCDF variable") == 0;
      if (!dim_only) out.vars[name] = std::move(v);
    }
    h.Tclose(t);
    h.Sclose(sp);
    h.Dclose(d);
  }
  h.Fclose(f);
  return rc;
}

int read_data_file(const char *path, DataFile &out)
{
  if (!path) return fail(RRTMGPNN_ERR_ARGUMENT, "read: null path");
  std::ifstream f(path, std::ios::binary);
  if (!f) return fail(RRTMGPNN_ERR_IO, std::string("cannot open ") + path);
  unsigned char m[8] = {0};
  f.read((char *)m, 8);
  if (std::memcmp(m, "RBIN", 4) == 0) return read_rbin(path, out);
  if (m[0] == 0x89 && std::memcmp(m + 1, "HDF", 3) == 0) return read_hdf5(path, out);
  if (std::memcmp(m, "CDF", 3) == 0 && (m[3] == 1 || m[3] == 2 || m[3] == 5)) {
    f.seekg(0, std::ios::end);
    std::vector<unsigned char> buf((size_t)f.tellg());
    f.seekg(0);
    f.read((char *)buf.data(), (std::streamsize)buf.size());
    if (!f) return fail(RRTMGPNN_ERR_IO, std::string(path) + ": read failed");
    return read_cdf(path, buf, out);
  }
  return fail(RRTMGPNN_ERR_IO, std::string(path) + ": not an RBIN, netCDF or HDF5 file");
}

}  // namespace rrtmgpnn
