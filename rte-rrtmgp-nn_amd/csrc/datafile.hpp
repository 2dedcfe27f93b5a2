// datafile.hpp -- host-side readers for the data files the path consumes:
// RBIN (this repository's flat format, rrtmgpnn/rbin.py), classic netCDF (CDF-1/2/5, parsed here) and
// netCDF-4 (HDF5; the HDF5 C library is loaded at run time with dlopen, so librrtmgpnn.so has no link-time
// dependency on it).  Every variable is read whole into host memory in its file order (C order = the
// reference's Fortran arrays with the dimensions reversed).
#pragma once
#include <map>
#include <string>
#include <vector>

namespace rrtmgpnn {

enum DataType { kF32 = 0, kI32 = 1, kChar = 2 };

struct DataVar {
  int dtype = kF32;        // floating-point variables are converted to float32, integers to int32
  std::vector<int> dims;   // file (C) order
  std::vector<char> data;  // count() elements of 4 bytes (kF32, kI32) or 1 byte (kChar)
  size_t count() const
  {
    size_t n = 1;
    for (int d : dims) n *= (size_t)d;
    return n;
  }
};

struct DataFile {
  std::map<std::string, DataVar> vars;
  std::map<std::string, std::string> atts;  // text attributes: "var:att", global ones as ":att"
  bool has(const std::string &v) const { return vars.count(v) != 0; }
};

// Dispatch on the file's magic bytes: "RBIN", "CDF\x01|\x02|\x05", "\x89HDF".
int read_data_file(const char *path, DataFile &out);

// Element conversions (int <-> float as C casts; chars are not numeric).
std::vector<float> to_float(const DataVar &v);
std::vector<int> to_int(const DataVar &v);

}  // namespace rrtmgpnn
