// NetCDFClassic.h -- the netCDF classic file format (CDF-1 / CDF-2 "64-bit offset", the format of
// the netCDF User's Guide, "File Format Specification") read and written without libnetcdf, which
// this image lacks. It carries the reference's two netCDF files:
//   * the data files the likelihoods read through NetCDFDataFile (src/utils/NetCDFDataFile.cpp:
//     GetDimensionSize / GetValue / GetValues / GetValuesDim2 on a group such as "trial" in
//     pkdata.nc, LikelihoodPopPKTrajectory.cpp:89-204), and
//   * the sampler's output.nc (SampleHandlerNetCDF.cpp:24-110: group "samples" with dims
//     sample_ix / variable / temperature and variables variable_transform, variable_values,
//     log_prior, log_likelihood, weights).
// The reference writes netCDF-4 (HDF5) with groups; classic files have no groups, so a group g's
// dimension or variable n is stored as "g.n", nested groups g/h as "g.h.n" (the name after the last
// '.' is the member; tools/nc_convert.py converts both ways where the netCDF4 Python module is
// installed). NC_STRING variables become NC_CHAR [.., g.<dim>_strlen].
#pragma once
#include <cstdint>
#include <cstdio>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "json.h"

namespace bcm3 {

enum NcType { NcByte = 1, NcChar = 2, NcShort = 3, NcInt = 4, NcFloat = 5, NcDouble = 6 };

constexpr double kNcFillDouble = 9.9692099683868690e+36;  // NC_FILL_DOUBLE
constexpr int32_t kNcFillInt = -2147483647;              // NC_FILL_INT

struct NcAttr {
    std::string name;
    int type = NcChar;
    std::string text;          // NcChar
    std::vector<double> nums;  // numeric types
};

struct NcDim {
    std::string name;
    uint64_t len = 0;  // 0: the record (unlimited) dimension
};

struct NcVar {
    std::string name;
    int type = NcDouble;
    std::vector<int> dims;
    std::vector<NcAttr> attrs;
    uint64_t vsize = 0, begin = 0;  // set by the layout
};

// a file's header: dimensions, global attributes, variables (fixed-size variables only on write)
struct NcHeader {
    int version = 2;
    uint64_t numrecs = 0;
    std::vector<NcDim> dims;
    std::vector<NcAttr> gattrs;
    std::vector<NcVar> vars;

    int AddDim(const std::string& name, uint64_t len);
    int AddVar(const std::string& name, int type, const std::vector<int>& dims);
    int FindVar(const std::string& name) const;
    int FindDim(const std::string& name) const;
    uint64_t NumElements(const NcVar& v) const;  // of one record for record variables
};

size_t NcTypeSize(int type);

// Read: the whole file as the JSON tree the likelihood loaders take,
// {"<group>": {"<var>": {"dims": [dim names], "data": nested arrays}}} -- numbers, NaN for the
// variable's _FillValue, char arrays as strings along their last dimension. The group is the name
// up to the last '.'; names without one go under the group "". Throws JsonError on malformed input.
Json NcClassicRead(const std::string& filename);
bool NcIsClassic(const std::string& filename);

// A likelihood data file (NetCDFDataFile::Open): netCDF classic (NcClassicRead) or the JSON
// sidecar, chosen by the file's magic bytes; a netCDF-4 (HDF5) file goes through libnetcdf when
// it can be loaded at run time, else it is refused with the conversion command. Throws JsonError.
Json LoadDataFile(const std::string& filename);
// netCDF-4 through a run-time loaded libnetcdf (NetCDF4.cpp): same layout as NcClassicRead
bool NcNetCDF4Available(std::string* why);
Json NcNetCDF4Read(const std::string& filename);
// {"dims", "data"} variable records -> their data arrays, for the loaders that index arrays
void UnwrapDataVariables(Json& doc);

// netCDF-4 output through the run-time loaded libnetcdf (NetCDF4.cpp), as the reference writes
// output.nc / sampler_adaptation.nc (NetCDFDataFile::Create, NC_CLOBBER | NC_NETCDF4). Unavailable
// without a libnetcdf that has the writing API, or with BCM3_OUTPUT_FORMAT=classic.
enum { Nc4Double = 6, Nc4UInt = 9, Nc4String = 12 };
bool NcNetCDF4WriteAvailable(std::string* why);
struct NcWriteApi;  // NetCDF4.cpp
class NcNetCDF4Writer {
public:
    bool Create(const std::string& filename);
    int Group(const std::string& path);  // nested groups by '/', created on first use; -1 on error
    int Dim(int grp, const std::string& name, size_t len);
    int Var(int grp, const std::string& name, int type, const std::vector<int>& dims);
    bool PutDouble(int grp, int var, const std::vector<size_t>& start, const std::vector<size_t>& count,
                   const double* data);
    bool PutUInt(int grp, int var, const std::vector<size_t>& start, const std::vector<size_t>& count,
                 const uint32_t* data);
    bool PutStrings(int grp, int var, const std::vector<std::string>& s);
    bool Sync();
    void Close();
    bool IsOpen() const { return nc_ >= 0; }
    ~NcNetCDF4Writer() { Close(); }

private:
    int nc_ = -1;
    std::string filename_;
    std::map<std::string, int> groups_;
    const NcWriteApi* w_ = nullptr;  // the library nc_ belongs to (NetCDF4.cpp), set by Create
};

// Write: a fixed-size (non-record) CDF-2 file. Layout() assigns offsets; Create() writes the
// header and, for the variables of `fill_vars` (all when empty), their fill values; Put()
// writes a hyperslab [start, start+count) in row-major order, converting from double / int32 /
// char. Several processes may write disjoint slabs of the same file: Create(..., false) writes
// identical header bytes, sizes the file exactly and leaves other processes' regions alone.
class NcClassicWriter {
public:
    NcHeader h;
    // fill_vars: the variables to fill (nullptr: all)
    bool Create(const std::string& filename, bool truncate, const std::vector<int>* fill_vars = nullptr);
    bool PutDouble(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count, const double* data);
    bool PutInt(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count, const int32_t* data);
    bool PutChars(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count, const char* data);
    bool Sync();
    void Close();
    ~NcClassicWriter() { Close(); }

private:
    bool Layout();
    std::vector<uint8_t> EncodeHeader() const;
    bool PutRaw(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count,
                const std::vector<uint8_t>& be_bytes);
    bool FillVar(int var);
    int fd_ = -1;
    uint64_t header_size_ = 0, file_size_ = 0;
};

// SampleHandlerNetCDF (SampleHandlerNetCDF.cpp:24-110) over the classic writer: group "samples",
// dims sample_ix [num_samples], temperature [temperatures], variable [names]; sample_ix holds
// 1..n at creation and the 0-based index of every received sample (as the reference writes
// it); values, log prior, log likelihood and weight per (sample, temperature), NC_FILL_DOUBLE
// where nothing was received. `first_temperature` / `own` select the temperature columns this
// process writes (a rank's ladder slice): each rank writes only its own columns of the shared
// file. A process that writes every temperature writes netCDF-4 with the group "samples" instead
// (the reference's own format) when libnetcdf can be loaded (NcNetCDF4WriteAvailable); the shared
// file of a sharded ladder stays classic (HDF5 files take one writer).
class SampleFileWriter {
public:
    bool Initialize(const std::string& filename, size_t num_samples, const std::vector<std::string>& names,
                    const std::vector<int32_t>& transforms, const std::vector<double>& temperatures,
                    size_t first_temperature, size_t own);
    // rows of this process's temperatures (t0 relative to first_temperature): values [own][d]
    bool Write(size_t sample_ix, size_t t0, size_t nt, const double* values, const double* lprior,
               const double* llh, const double* weight);
    bool Sync() { return w4_ ? w4_->Sync() : w_.Sync(); }
    void Close()
    {
        if (w4_) w4_->Close();
        w_.Close();
    }
    bool IsNetCDF4() const { return w4_ != nullptr; }

private:
    // one process writing every temperature: netCDF-4 when libnetcdf can be loaded
    bool InitializeNetCDF4(const std::string& filename, const std::vector<std::string>& names,
                           const std::vector<int32_t>& transforms, const std::vector<double>& temperatures);
    NcClassicWriter w_;
    std::unique_ptr<NcNetCDF4Writer> w4_;
    int g4_ = -1;
    int v_six_ = -1, v_vals_ = -1, v_lp_ = -1, v_llh_ = -1, v_w_ = -1;
    size_t first_ = 0, own_ = 0, d_ = 0, n_ = 0;
};

// NetCDFBundler (src/utils/NetCDFBundler.cpp:34-80) as a whole-file writer: groups of vectors and
// matrices, each with the reference's dimension names (<name>_dim, <name>_dim1 / _dim2) and their
// 1-based coordinate variables; Write() (re)writes the whole file, so records can be added between
// writes (sampler_adaptation.nc grows by one group per adaptation).
class BundleFile {
public:
    void AddVector(const std::string& group, const std::string& name, const std::vector<double>& v);
    void AddVector(const std::string& group, const std::string& name, const std::vector<int32_t>& v);
    void AddMatrix(const std::string& group, const std::string& name, size_t rows, size_t cols,
                   const std::vector<double>& row_major);
    // netCDF-4 with nested groups (adapt<k>/block1) when libnetcdf can be loaded, classic otherwise
    bool Write(const std::string& filename) const;

private:
    bool WriteNetCDF4(const std::string& filename) const;
    struct Item {
        std::string group, name;
        bool is_int = false;
        size_t rows = 0, cols = 0;  // cols == 0: vector
        std::vector<double> d;
        std::vector<int32_t> i;
    };
    std::vector<Item> items_;
};

}  // namespace bcm3
