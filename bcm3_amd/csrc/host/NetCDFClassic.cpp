// NetCDFClassic.cpp -- netCDF classic format reader / writer (see NetCDFClassic.h).
#include "NetCDFClassic.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cmath>
#include <cstring>
#include <fstream>
#include <algorithm>
#include <limits>

#include "log.h"

namespace bcm3 {

namespace {

constexpr uint32_t NC_DIMENSION = 0x0A, NC_VARIABLE = 0x0B, NC_ATTRIBUTE = 0x0C;
constexpr float kNcFillFloat = 9.9692099683868690e+36f;

uint64_t pad4(uint64_t n) { return (n + 3) & ~(uint64_t)3; }

// ---- big-endian encoding
struct Out {
    std::vector<uint8_t> b;
    void u32(uint32_t v)
    {
        for (int s = 24; s >= 0; s -= 8) b.push_back((uint8_t)(v >> s));
    }
    void u64(uint64_t v)
    {
        for (int s = 56; s >= 0; s -= 8) b.push_back((uint8_t)(v >> s));
    }
    void name(const std::string& s)
    {
        u32((uint32_t)s.size());
        b.insert(b.end(), s.begin(), s.end());
        while (b.size() % 4) b.push_back(0);
    }
};

void put_be(uint8_t* p, const void* src, size_t size)
{
    const uint8_t* s = (const uint8_t*)src;
    for (size_t i = 0; i < size; i++) p[i] = s[size - 1 - i];
}

struct In {
    const std::vector<uint8_t>& b;
    size_t p = 0;
    void need(size_t n) const
    {
        if (p + n > b.size()) throw JsonError{"netCDF header truncated"};
    }
    uint32_t u32()
    {
        need(4);
        uint32_t v = ((uint32_t)b[p] << 24) | ((uint32_t)b[p + 1] << 16) | ((uint32_t)b[p + 2] << 8) | b[p + 3];
        p += 4;
        return v;
    }
    uint64_t u64()
    {
        const uint64_t hi = u32();
        return (hi << 32) | u32();
    }
    std::string name()
    {
        const uint32_t n = u32();
        need(pad4(n));
        std::string s((const char*)&b[p], n);
        p += pad4(n);
        return s;
    }
};

double read_value(const uint8_t* p, int type)
{
    uint8_t le[8];
    switch (type) {
    case NcByte: return (double)(int8_t)p[0];
    case NcChar: return (double)p[0];
    case NcShort: {
        put_be(le, p, 2);
        int16_t v;
        std::memcpy(&v, le, 2);
        return v;
    }
    case NcInt: {
        put_be(le, p, 4);
        int32_t v;
        std::memcpy(&v, le, 4);
        return v;
    }
    case NcFloat: {
        put_be(le, p, 4);
        float v;
        std::memcpy(&v, le, 4);
        return v;
    }
    default: {
        put_be(le, p, 8);
        double v;
        std::memcpy(&v, le, 8);
        return v;
    }
    }
}

std::vector<NcAttr> read_attrs(In& in)
{
    std::vector<NcAttr> out;
    const uint32_t tag = in.u32(), n = in.u32();
    if (tag == 0 && n == 0) return out;
    if (tag != NC_ATTRIBUTE) throw JsonError{"netCDF: bad attribute list"};
    for (uint32_t i = 0; i < n; i++) {
        NcAttr a;
        a.name = in.name();
        a.type = (int)in.u32();
        const uint32_t ne = in.u32();
        const size_t sz = NcTypeSize(a.type);
        if (sz == 0) throw JsonError{"netCDF: unknown attribute type"};
        in.need(pad4((uint64_t)ne * sz));
        if (a.type == NcChar) {
            a.text.assign((const char*)&in.b[in.p], ne);
        } else {
            for (uint32_t k = 0; k < ne; k++) a.nums.push_back(read_value(&in.b[in.p + k * sz], a.type));
        }
        in.p += pad4((uint64_t)ne * sz);
        out.push_back(a);
    }
    return out;
}

void write_attrs(Out& o, const std::vector<NcAttr>& attrs)
{
    if (attrs.empty()) {
        o.u32(0);
        o.u32(0);
        return;
    }
    o.u32(NC_ATTRIBUTE);
    o.u32((uint32_t)attrs.size());
    for (auto& a : attrs) {
        o.name(a.name);
        o.u32((uint32_t)a.type);
        if (a.type == NcChar) {
            o.u32((uint32_t)a.text.size());
            o.b.insert(o.b.end(), a.text.begin(), a.text.end());
        } else {
            o.u32((uint32_t)a.nums.size());
            for (double v : a.nums) {
                uint8_t buf[8];
                const size_t sz = NcTypeSize(a.type);
                if (a.type == NcDouble) {
                    put_be(buf, &v, 8);
                } else if (a.type == NcFloat) {
                    const float f = (float)v;
                    put_be(buf, &f, 4);
                } else if (a.type == NcInt) {
                    const int32_t x = (int32_t)v;
                    put_be(buf, &x, 4);
                } else if (a.type == NcShort) {
                    const int16_t x = (int16_t)v;
                    put_be(buf, &x, 2);
                } else {
                    buf[0] = (uint8_t)(int8_t)v;
                }
                o.b.insert(o.b.end(), buf, buf + sz);
            }
        }
        while (o.b.size() % 4) o.b.push_back(0);
    }
}

bool is_fill(double v, int type, const NcVar& var)
{
    for (auto& a : var.attrs)
        if (a.name == "_FillValue" && !a.nums.empty()) return v == a.nums[0];
    switch (type) {
    case NcDouble: return v == kNcFillDouble || v == (double)kNcFillFloat;
    case NcFloat: return v == (double)kNcFillFloat;
    case NcInt: return v == (double)kNcFillInt;
    case NcShort: return v == -32767.0;
    case NcByte: return v == -127.0;
    default: return false;
    }
}

}  // namespace

size_t NcTypeSize(int type)
{
    switch (type) {
    case NcByte:
    case NcChar: return 1;
    case NcShort: return 2;
    case NcInt:
    case NcFloat: return 4;
    case NcDouble: return 8;
    default: return 0;
    }
}

int NcHeader::AddDim(const std::string& name, uint64_t len)
{
    dims.push_back({name, len});
    return (int)dims.size() - 1;
}

int NcHeader::AddVar(const std::string& name, int type, const std::vector<int>& d)
{
    NcVar v;
    v.name = name;
    v.type = type;
    v.dims = d;
    vars.push_back(v);
    return (int)vars.size() - 1;
}

int NcHeader::FindVar(const std::string& name) const
{
    for (size_t i = 0; i < vars.size(); i++)
        if (vars[i].name == name) return (int)i;
    return -1;
}

int NcHeader::FindDim(const std::string& name) const
{
    for (size_t i = 0; i < dims.size(); i++)
        if (dims[i].name == name) return (int)i;
    return -1;
}

uint64_t NcHeader::NumElements(const NcVar& v) const
{
    uint64_t n = 1;
    for (int d : v.dims)
        if (dims[d].len != 0) n *= dims[d].len;
    return n;
}

bool NcIsClassic(const std::string& filename)
{
    std::ifstream f(filename, std::ios::binary);
    char m[4] = {0, 0, 0, 0};
    f.read(m, 4);
    return f && m[0] == 'C' && m[1] == 'D' && m[2] == 'F' && (m[3] == 1 || m[3] == 2);
}

// ---------------------------------------------------------------------------------------------
// reader

Json NcClassicRead(const std::string& filename)
{
    std::ifstream f(filename, std::ios::binary);
    if (!f) throw JsonError{"cannot open " + filename};
    std::vector<uint8_t> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    In in{buf};
    in.need(4);
    if (buf[0] != 'C' || buf[1] != 'D' || buf[2] != 'F' || (buf[3] != 1 && buf[3] != 2))
        throw JsonError{filename + " is not a netCDF classic file"};
    NcHeader h;
    h.version = buf[3];
    in.p = 4;
    const uint32_t nr = in.u32();
    h.numrecs = (nr == 0xFFFFFFFFu) ? 0 : nr;
    {
        const uint32_t tag = in.u32(), n = in.u32();
        if (!(tag == 0 && n == 0)) {
            if (tag != NC_DIMENSION) throw JsonError{"netCDF: bad dimension list"};
            for (uint32_t i = 0; i < n; i++) {
                NcDim d;
                d.name = in.name();
                d.len = in.u32();
                h.dims.push_back(d);
            }
        }
    }
    h.gattrs = read_attrs(in);
    {
        const uint32_t tag = in.u32(), n = in.u32();
        if (!(tag == 0 && n == 0)) {
            if (tag != NC_VARIABLE) throw JsonError{"netCDF: bad variable list"};
            for (uint32_t i = 0; i < n; i++) {
                NcVar v;
                v.name = in.name();
                const uint32_t nd = in.u32();
                for (uint32_t k = 0; k < nd; k++) {
                    const uint32_t id = in.u32();
                    if (id >= h.dims.size()) throw JsonError{"netCDF: bad dimension id"};
                    v.dims.push_back((int)id);
                }
                v.attrs = read_attrs(in);
                v.type = (int)in.u32();
                if (NcTypeSize(v.type) == 0) throw JsonError{"netCDF: unknown variable type"};
                v.vsize = in.u32();
                v.begin = (h.version == 1) ? in.u32() : in.u64();
                h.vars.push_back(v);
            }
        }
    }
    // record layout: the record variables' slabs interleave; recsize = the sum of their vsizes
    // (one record variable: its unpadded size)
    uint64_t recsize = 0;
    int nrecvars = 0;
    for (auto& v : h.vars)
        if (!v.dims.empty() && h.dims[v.dims[0]].len == 0) {
            recsize += v.vsize;
            nrecvars++;
        }
    if (nrecvars == 1)
        for (auto& v : h.vars)
            if (!v.dims.empty() && h.dims[v.dims[0]].len == 0) recsize = h.NumElements(v) * NcTypeSize(v.type);

    Json doc;
    doc.type = Json::Object;
    auto split = [](const std::string& n, std::string& g, std::string& leaf) {
        const size_t dot = n.rfind('.');
        if (dot == std::string::npos) {
            g.clear();
            leaf = n;
        } else {
            g = n.substr(0, dot);
            leaf = n.substr(dot + 1);
        }
    };
    for (auto& v : h.vars) {
        std::string g, leaf;
        split(v.name, g, leaf);
        const bool rec = !v.dims.empty() && h.dims[v.dims[0]].len == 0;
        std::vector<uint64_t> shape;
        for (size_t k = 0; k < v.dims.size(); k++) shape.push_back((k == 0 && rec) ? h.numrecs : h.dims[v.dims[k]].len);
        const size_t sz = NcTypeSize(v.type);
        const uint64_t per_rec = h.NumElements(v);
        // element i (row-major over shape) -> file offset
        auto offset = [&](uint64_t i) -> uint64_t {
            if (!rec) return v.begin + i * sz;
            const uint64_t r = i / per_rec, k = i % per_rec;
            return v.begin + r * recsize + k * sz;
        };
        // every element must lie inside the file: bounds the element count before anything is
        // allocated (a corrupt header cannot ask for more elements than the file has bytes)
        uint64_t total = 1;
        for (auto s : shape) {
            if (s != 0 && total > buf.size() / s) throw JsonError{"netCDF: data beyond end of file"};
            total *= s;
        }
        if (total > 0 && (offset(total - 1) > buf.size() || offset(total - 1) + sz > buf.size()))
            throw JsonError{"netCDF: data beyond end of file"};
        const bool chars = (v.type == NcChar) && !shape.empty();
        const uint64_t inner = chars ? std::max<uint64_t>(shape.back(), 1) : 1;
        std::vector<Json> flat;
        flat.reserve(total / inner);
        for (uint64_t i = 0; i < total; i += inner) {
            Json e;
            if (chars) {
                e.type = Json::String;
                for (uint64_t k = 0; k < inner; k++) {
                    const uint64_t o = offset(i + k);
                    if (o >= buf.size()) throw JsonError{"netCDF: data beyond end of file"};
                    if (buf[o] == 0) break;
                    e.str.push_back((char)buf[o]);
                }
            } else {
                const uint64_t o = offset(i);
                if (o + sz > buf.size()) throw JsonError{"netCDF: data beyond end of file"};
                const double x = read_value(&buf[o], v.type);
                e.type = Json::Number;
                e.num = is_fill(x, v.type, v) ? std::numeric_limits<double>::quiet_NaN() : x;
            }
            flat.push_back(std::move(e));
        }
        // nest along the leading dimensions
        std::vector<uint64_t> outer(shape.begin(), shape.end() - (chars ? 1 : 0));
        Json data;
        if (outer.empty()) {
            data = flat.empty() ? Json() : flat[0];
        } else {
            std::vector<Json> level = std::move(flat);
            for (size_t k = outer.size(); k-- > 1;) {
                std::vector<Json> up;
                const uint64_t m = outer[k];
                for (size_t i = 0; i < level.size(); i += m) {
                    Json a;
                    a.type = Json::Array;
                    a.arr.assign(std::make_move_iterator(level.begin() + i), std::make_move_iterator(level.begin() + i + m));
                    up.push_back(std::move(a));
                }
                level = std::move(up);
            }
            data.type = Json::Array;
            data.arr = std::move(level);
        }
        Json var;
        var.type = Json::Object;
        Json dims;
        dims.type = Json::Array;
        for (size_t k = 0; k < v.dims.size() - (chars ? 1 : 0) && k < v.dims.size(); k++) {
            Json dn;
            dn.type = Json::String;
            std::string dg;
            split(h.dims[v.dims[k]].name, dg, dn.str);
            dims.arr.push_back(dn);
        }
        var.obj["dims"] = dims;
        var.obj["data"] = std::move(data);
        Json& grp = doc.obj[g];
        grp.type = Json::Object;
        grp.obj[leaf] = std::move(var);
    }
    return doc;
}

Json LoadDataFile(const std::string& filename)
{
    std::ifstream f(filename, std::ios::binary);
    if (!f) throw JsonError{"cannot open " + filename};
    unsigned char m[4] = {0, 0, 0, 0};
    f.read((char*)m, 4);
    if (m[0] == 'C' && m[1] == 'D' && m[2] == 'F') return NcClassicRead(filename);
    if (m[0] == 0x89 && m[1] == 'H' && m[2] == 'D' && m[3] == 'F') {
        // netCDF-4: through the system's libnetcdf when it can be loaded (NetCDF4.cpp)
        std::string why;
        if (NcNetCDF4Available(&why)) return NcNetCDF4Read(filename);
        throw JsonError{filename + " is netCDF-4 (HDF5) and " + why + " ($BCM3_LIBNETCDF names it); convert it: "
                                   "python tools/nc_convert.py to-classic " + filename + " <out.nc>"};
    }
    return json_load(filename);
}

void UnwrapDataVariables(Json& doc)
{
    for (auto& g : doc.obj)
        for (auto& v : g.second.obj)
            if (v.second.type == Json::Object) {
                auto it = v.second.obj.find("data");
                if (it != v.second.obj.end()) {
                    Json d = std::move(it->second);
                    v.second = std::move(d);
                }
            }
}

// ---------------------------------------------------------------------------------------------
// writer

std::vector<uint8_t> NcClassicWriter::EncodeHeader() const
{
    Out o;
    o.b = {'C', 'D', 'F', 2};
    o.u32(0);
    if (h.dims.empty()) {
        o.u32(0);
        o.u32(0);
    } else {
        o.u32(NC_DIMENSION);
        o.u32((uint32_t)h.dims.size());
        for (auto& d : h.dims) {
            o.name(d.name);
            o.u32((uint32_t)d.len);
        }
    }
    write_attrs(o, h.gattrs);
    if (h.vars.empty()) {
        o.u32(0);
        o.u32(0);
    } else {
        o.u32(NC_VARIABLE);
        o.u32((uint32_t)h.vars.size());
        for (auto& v : h.vars) {
            o.name(v.name);
            o.u32((uint32_t)v.dims.size());
            for (int d : v.dims) o.u32((uint32_t)d);
            write_attrs(o, v.attrs);
            o.u32((uint32_t)v.type);
            o.u32(v.vsize > 0xFFFFFFFCull ? 0xFFFFFFFFu : (uint32_t)v.vsize);
            o.u64(v.begin);
        }
    }
    return o.b;
}

bool NcClassicWriter::Layout()
{
    h.version = 2;
    h.numrecs = 0;
    for (auto& d : h.dims)
        if (d.len == 0) {
            LOGERROR("netCDF writer: record dimensions are not supported (%s)", d.name.c_str());
            return false;
        }
    for (auto& v : h.vars) v.vsize = pad4(h.NumElements(v) * NcTypeSize(v.type));
    // header size with placeholder offsets, then the data offsets in variable order
    header_size_ = EncodeHeader().size();
    uint64_t off = header_size_;
    for (auto& v : h.vars) {
        v.begin = off;
        off += v.vsize;
    }
    file_size_ = off;
    return true;
}

bool NcClassicWriter::Create(const std::string& filename, bool truncate, const std::vector<int>* fill_vars)
{
    Close();
    if (!Layout()) return false;
    fd_ = ::open(filename.c_str(), O_RDWR | O_CREAT | (truncate ? O_TRUNC : 0), 0644);
    if (fd_ < 0) {
        LOGERROR("Cannot create %s", filename.c_str());
        return false;
    }
    // the header, encoded again with the final offsets
    const std::vector<uint8_t> hb = EncodeHeader();
    if (hb.size() != header_size_ || ::pwrite(fd_, hb.data(), hb.size(), 0) != (ssize_t)hb.size()) {
        LOGERROR("Cannot write the header of %s", filename.c_str());
        return false;
    }
    // a shared file is cut or grown to its final size: every process writes only below it, so
    // this is safe in any order
    struct stat st;
    if (::fstat(fd_, &st) == 0 && (uint64_t)st.st_size != file_size_ && ::ftruncate(fd_, (off_t)file_size_) != 0) {
        LOGERROR("Cannot size %s", filename.c_str());
        return false;
    }
    if (!fill_vars) {
        for (size_t v = 0; v < h.vars.size(); v++)
            if (!FillVar((int)v)) return false;
    } else {
        for (int v : *fill_vars)
            if (!FillVar(v)) return false;
    }
    return true;
}

bool NcClassicWriter::FillVar(int var)
{
    const NcVar& v = h.vars[var];
    const size_t sz = NcTypeSize(v.type);
    uint8_t fill[8] = {0};
    double fv = (v.type == NcDouble) ? kNcFillDouble : (v.type == NcInt) ? (double)kNcFillInt : 0.0;
    for (auto& a : v.attrs)
        if (a.name == "_FillValue" && !a.nums.empty()) fv = a.nums[0];
    if (v.type == NcDouble) {
        put_be(fill, &fv, 8);
    } else if (v.type == NcInt) {
        const int32_t x = (int32_t)fv;
        put_be(fill, &x, 4);
    } else if (v.type == NcFloat) {
        const float x = (float)fv;
        put_be(fill, &x, 4);
    }
    const uint64_t n = h.NumElements(v);
    std::vector<uint8_t> chunk;
    const uint64_t per = 1 << 16;
    chunk.resize(std::min<uint64_t>(n, per) * sz);
    for (size_t i = 0; i < chunk.size(); i += sz) std::memcpy(&chunk[i], fill, sz);
    for (uint64_t i = 0; i < n; i += per) {
        const uint64_t m = std::min<uint64_t>(per, n - i);
        if (::pwrite(fd_, chunk.data(), m * sz, (off_t)(v.begin + i * sz)) != (ssize_t)(m * sz)) return false;
    }
    return true;
}

bool NcClassicWriter::PutRaw(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count,
                             const std::vector<uint8_t>& be)
{
    if (fd_ < 0 || var < 0 || var >= (int)h.vars.size()) return false;
    const NcVar& v = h.vars[var];
    const size_t nd = v.dims.size(), sz = NcTypeSize(v.type);
    if (start.size() != nd || count.size() != nd) return false;
    uint64_t total = 1;
    for (size_t k = 0; k < nd; k++) {
        if (start[k] + count[k] > h.dims[v.dims[k]].len) {
            LOGERROR("netCDF writer: slab out of range for %s", v.name.c_str());
            return false;
        }
        total *= count[k];
    }
    if (be.size() != total * sz) return false;
    if (total == 0) return true;
    if (nd == 0) return ::pwrite(fd_, be.data(), sz, (off_t)v.begin) == (ssize_t)sz;
    // contiguous runs along the last dimension
    const uint64_t run = count[nd - 1];
    std::vector<uint64_t> idx(nd, 0);
    for (uint64_t r = 0; r < total / run; r++) {
        uint64_t lin = 0;
        for (size_t k = 0; k < nd; k++) lin = lin * h.dims[v.dims[k]].len + start[k] + (k + 1 < nd ? idx[k] : 0);
        if (::pwrite(fd_, &be[r * run * sz], run * sz, (off_t)(v.begin + lin * sz)) != (ssize_t)(run * sz)) return false;
        for (size_t k = nd - 1; k-- > 0;) {
            if (++idx[k] < count[k]) break;
            idx[k] = 0;
        }
    }
    return true;
}

bool NcClassicWriter::PutDouble(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count,
                                const double* data)
{
    uint64_t n = 1;
    for (auto c : count) n *= c;
    std::vector<uint8_t> be(n * 8);
    for (uint64_t i = 0; i < n; i++) put_be(&be[i * 8], &data[i], 8);
    return var >= 0 && h.vars[var].type == NcDouble && PutRaw(var, start, count, be);
}

bool NcClassicWriter::PutInt(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count,
                             const int32_t* data)
{
    uint64_t n = 1;
    for (auto c : count) n *= c;
    std::vector<uint8_t> be(n * 4);
    for (uint64_t i = 0; i < n; i++) put_be(&be[i * 4], &data[i], 4);
    return var >= 0 && h.vars[var].type == NcInt && PutRaw(var, start, count, be);
}

bool NcClassicWriter::PutChars(int var, const std::vector<uint64_t>& start, const std::vector<uint64_t>& count,
                               const char* data)
{
    uint64_t n = 1;
    for (auto c : count) n *= c;
    std::vector<uint8_t> be((const uint8_t*)data, (const uint8_t*)data + n);
    return var >= 0 && h.vars[var].type == NcChar && PutRaw(var, start, count, be);
}

bool NcClassicWriter::Sync() { return fd_ >= 0 && ::fsync(fd_) == 0; }

void NcClassicWriter::Close()
{
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
}

// ---------------------------------------------------------------------------------------------
// SampleHandlerNetCDF

bool SampleFileWriter::Initialize(const std::string& filename, size_t num_samples,
                                  const std::vector<std::string>& names, const std::vector<int32_t>& transforms,
                                  const std::vector<double>& temperatures, size_t first_temperature, size_t own)
{
    d_ = names.size();
    n_ = num_samples;
    first_ = first_temperature;
    own_ = own;
    const size_t T = temperatures.size();
    if (d_ == 0 || T == 0 || num_samples == 0 || transforms.size() != d_ || first_ + own_ > T) {
        LOGERROR("SampleFileWriter: inconsistent output geometry");
        return false;
    }
    w4_.reset();
    if (first_ == 0 && own_ == T && NcNetCDF4WriteAvailable(nullptr))
        return InitializeNetCDF4(filename, names, transforms, temperatures);
    size_t strlen_max = 1;
    for (auto& s : names) strlen_max = std::max(strlen_max, s.size());
    NcHeader& h = w_.h;
    h = NcHeader();
    h.gattrs.push_back(NcAttr{"bcm3_groups", NcChar, "samples", {}});
    const int ds = h.AddDim("samples.sample_ix", num_samples);
    const int dv = h.AddDim("samples.variable", d_);
    const int dt = h.AddDim("samples.temperature", T);
    const int dl = h.AddDim("samples.variable_strlen", strlen_max);
    v_six_ = h.AddVar("samples.sample_ix", NcInt, {ds});
    const int v_var = h.AddVar("samples.variable", NcChar, {dv, dl});
    const int v_temp = h.AddVar("samples.temperature", NcDouble, {dt});
    const int v_tr = h.AddVar("samples.variable_transform", NcInt, {dv});
    v_lp_ = h.AddVar("samples.log_prior", NcDouble, {ds, dt});
    v_llh_ = h.AddVar("samples.log_likelihood", NcDouble, {ds, dt});
    v_w_ = h.AddVar("samples.weights", NcDouble, {ds, dt});
    // last: CDF-2 lets only the last variable exceed 4 GiB (long runs x large ladders)
    v_vals_ = h.AddVar("samples.variable_values", NcDouble, {ds, dt, dv});
    for (int v : {v_vals_, v_lp_, v_llh_, v_w_}) h.vars[v].attrs.push_back(NcAttr{"_FillValue", NcDouble, "", {kNcFillDouble}});
    // the process holding temperature 0 writes the shared coordinate variables; every process
    // fills only its own temperature columns (no process truncates: see NcClassicWriter::Create)
    const bool lead = (first_ == 0);
    const std::vector<int> none;
    if (!w_.Create(filename, false, &none)) return false;
    // fill this process's columns in slabs of samples (bounded host memory)
    const size_t chunk = std::max<size_t>(1, (size_t)(1 << 20) / std::max<size_t>(1, own_ * d_));
    std::vector<double> fill(std::min(chunk, n_) * own_ * d_, kNcFillDouble);
    for (size_t s0 = 0; own_ > 0 && s0 < n_; s0 += chunk) {
        const size_t m = std::min(chunk, n_ - s0);
        if (!w_.PutDouble(v_vals_, {s0, first_, 0}, {m, own_, d_}, fill.data()) ||
            !w_.PutDouble(v_lp_, {s0, first_}, {m, own_}, fill.data()) ||
            !w_.PutDouble(v_llh_, {s0, first_}, {m, own_}, fill.data()) ||
            !w_.PutDouble(v_w_, {s0, first_}, {m, own_}, fill.data()))
            return false;
    }
    if (lead) {
        std::vector<int32_t> six(n_);
        for (size_t i = 0; i < n_; i++) six[i] = (int32_t)(i + 1);
        std::vector<char> nm(d_ * strlen_max, 0);
        for (size_t i = 0; i < d_; i++) std::memcpy(&nm[i * strlen_max], names[i].data(), names[i].size());
        if (!w_.PutInt(v_six_, {0}, {n_}, six.data()) || !w_.PutChars(v_var, {0, 0}, {d_, strlen_max}, nm.data()) ||
            !w_.PutDouble(v_temp, {0}, {T}, temperatures.data()) || !w_.PutInt(v_tr, {0}, {d_}, transforms.data()))
            return false;
    }
    return true;
}

// SampleHandlerNetCDF::Initialize (SampleHandlerNetCDF.cpp:24-63) in the reference's own netCDF-4
// layout: group samples; coordinate variables sample_ix (NC_UINT, 1..n), variable (NC_STRING, the
// names), temperature (NC_DOUBLE); variable_transform (NC_UINT); variable_values [sample_ix]
// [temperature][variable], log_prior / log_likelihood / weights [sample_ix][temperature] (NC_DOUBLE,
// the library's default fill where nothing is written)
bool SampleFileWriter::InitializeNetCDF4(const std::string& filename, const std::vector<std::string>& names,
                                         const std::vector<int32_t>& transforms, const std::vector<double>& temperatures)
{
    auto w = std::make_unique<NcNetCDF4Writer>();
    if (!w->Create(filename)) return false;
    const int g = w->Group("samples");
    if (g < 0) return false;
    const size_t T = temperatures.size();
    const int ds = w->Dim(g, "sample_ix", n_), dv = w->Dim(g, "variable", d_), dt = w->Dim(g, "temperature", T);
    if (ds < 0 || dv < 0 || dt < 0) return false;
    const int v_ix = w->Var(g, "sample_ix", Nc4UInt, {ds}), v_names = w->Var(g, "variable", Nc4String, {dv});
    const int v_temp = w->Var(g, "temperature", Nc4Double, {dt});
    const int v_tr = w->Var(g, "variable_transform", Nc4UInt, {dv});
    v_vals_ = w->Var(g, "variable_values", Nc4Double, {ds, dt, dv});
    v_lp_ = w->Var(g, "log_prior", Nc4Double, {ds, dt});
    v_llh_ = w->Var(g, "log_likelihood", Nc4Double, {ds, dt});
    v_w_ = w->Var(g, "weights", Nc4Double, {ds, dt});
    if (v_ix < 0 || v_names < 0 || v_temp < 0 || v_tr < 0 || v_vals_ < 0 || v_lp_ < 0 || v_llh_ < 0 || v_w_ < 0)
        return false;
    std::vector<uint32_t> ix(n_), tr(d_);
    for (size_t i = 0; i < n_; i++) ix[i] = (uint32_t)(i + 1);
    for (size_t i = 0; i < d_; i++) tr[i] = (uint32_t)transforms[i];
    if (!w->PutUInt(g, v_ix, {0}, {n_}, ix.data()) || !w->PutStrings(g, v_names, names) ||
        !w->PutDouble(g, v_temp, {0}, {T}, temperatures.data()) || !w->PutUInt(g, v_tr, {0}, {d_}, tr.data()))
        return false;
    v_six_ = v_ix;
    g4_ = g;
    w4_ = std::move(w);
    return true;
}

bool SampleFileWriter::Write(size_t sample_ix, size_t t0, size_t nt, const double* values, const double* lprior,
                             const double* llh, const double* weight)
{
    if (sample_ix >= n_ || t0 + nt > own_) return false;
    if (w4_) {
        // SampleHandlerNetCDF::ReceiveSample (:75-110): sample_ix[si] = si (the reference's 0-based
        // write over the 1-based coordinate), then the rows of these temperatures
        const uint32_t si = (uint32_t)sample_ix;
        const size_t t = t0;
        return w4_->PutUInt(g4_, v_six_, {sample_ix}, {1}, &si) &&
               w4_->PutDouble(g4_, v_vals_, {sample_ix, t, 0}, {1, nt, d_}, values) &&
               w4_->PutDouble(g4_, v_lp_, {sample_ix, t}, {1, nt}, lprior) &&
               w4_->PutDouble(g4_, v_llh_, {sample_ix, t}, {1, nt}, llh) &&
               w4_->PutDouble(g4_, v_w_, {sample_ix, t}, {1, nt}, weight);
    }
    const size_t t = first_ + t0;
    const int32_t si = (int32_t)sample_ix;
    return (first_ != 0 || w_.PutInt(v_six_, {sample_ix}, {1}, &si)) &&
           w_.PutDouble(v_vals_, {sample_ix, t, 0}, {1, nt, d_}, values) &&
           w_.PutDouble(v_lp_, {sample_ix, t}, {1, nt}, lprior) && w_.PutDouble(v_llh_, {sample_ix, t}, {1, nt}, llh) &&
           w_.PutDouble(v_w_, {sample_ix, t}, {1, nt}, weight);
}

// ---------------------------------------------------------------------------------------------
// NetCDFBundler

void BundleFile::AddVector(const std::string& group, const std::string& name, const std::vector<double>& v)
{
    Item it;
    it.group = group;
    it.name = name;
    it.rows = v.size();
    it.d = v;
    items_.push_back(std::move(it));
}

void BundleFile::AddVector(const std::string& group, const std::string& name, const std::vector<int32_t>& v)
{
    Item it;
    it.group = group;
    it.name = name;
    it.is_int = true;
    it.rows = v.size();
    it.i = v;
    items_.push_back(std::move(it));
}

void BundleFile::AddMatrix(const std::string& group, const std::string& name, size_t rows, size_t cols,
                           const std::vector<double>& row_major)
{
    Item it;
    it.group = group;
    it.name = name;
    it.rows = rows;
    it.cols = cols;
    it.d = row_major;
    items_.push_back(std::move(it));
}

// NetCDFBundler::AddVector / AddMatrix (NetCDFBundler.cpp:34-80) on netCDF-4: per item the
// dimension(s) <name>_dim or <name>_dim1 / _dim2 with NC_UINT coordinate variables 1..n
// (NetCDFDataFile::CreateDimension) and an NC_DOUBLE variable (CreateVariable), in nested groups
bool BundleFile::WriteNetCDF4(const std::string& filename) const
{
    NcNetCDF4Writer w;
    if (!w.Create(filename)) return false;
    auto coord = [&](int g, const std::string& name, size_t n) {
        const int d = w.Dim(g, name, n);
        if (d < 0) return -1;
        const int v = w.Var(g, name, Nc4UInt, {d});
        std::vector<uint32_t> c(n);
        for (size_t k = 0; k < n; k++) c[k] = (uint32_t)(k + 1);
        if (v < 0 || (n && !w.PutUInt(g, v, {0}, {n}, c.data()))) return -1;
        return d;
    };
    for (const Item& it : items_) {
        const int g = w.Group(it.group);
        if (g < 0) return false;
        if (it.cols == 0) {
            const int d = coord(g, it.name + "_dim", it.rows);
            const int v = (d < 0) ? -1 : w.Var(g, it.name, Nc4Double, {d});
            if (v < 0) return false;
            std::vector<double> x = it.d;
            if (it.is_int) x.assign(it.i.begin(), it.i.end());
            if (it.rows && !w.PutDouble(g, v, {0}, {it.rows}, x.data())) return false;
        } else {
            const int d1 = coord(g, it.name + "_dim1", it.rows), d2 = coord(g, it.name + "_dim2", it.cols);
            const int v = (d1 < 0 || d2 < 0) ? -1 : w.Var(g, it.name, Nc4Double, {d1, d2});
            if (v < 0) return false;
            if (it.rows && it.cols && !w.PutDouble(g, v, {0, 0}, {it.rows, it.cols}, it.d.data())) return false;
        }
    }
    w.Close();
    return true;
}

bool BundleFile::Write(const std::string& filename) const
{
    if (NcNetCDF4WriteAvailable(nullptr)) return WriteNetCDF4(filename);
    NcClassicWriter w;
    std::vector<std::string> groups;
    for (auto& it : items_)
        if (std::find(groups.begin(), groups.end(), it.group) == groups.end()) groups.push_back(it.group);
    std::string gl;
    for (auto& g : groups) gl += (gl.empty() ? "" : " ") + g;
    w.h.gattrs.push_back(NcAttr{"bcm3_groups", NcChar, gl, {}});
    // every dimension gets a coordinate variable 1..n (NetCDFDataFile::CreateDimension)
    struct Coord {
        int var;
        size_t n;
    };
    std::vector<Coord> coords;
    std::vector<int> data_vars;
    auto flat = [](const std::string& g, const std::string& n) {
        std::string p = g;
        for (auto& ch : p)
            if (ch == '/') ch = '.';
        return p.empty() ? n : p + "." + n;
    };
    auto dim = [&](const std::string& g, const std::string& n, size_t len) {
        const int d = w.h.AddDim(flat(g, n), len);
        coords.push_back(Coord{w.h.AddVar(flat(g, n), NcInt, {d}), len});
        return d;
    };
    for (auto& it : items_) {
        if (it.cols == 0) {
            const int d = dim(it.group, it.name + "_dim", it.rows);
            data_vars.push_back(w.h.AddVar(flat(it.group, it.name), it.is_int ? NcInt : NcDouble, {d}));
        } else {
            const int d1 = dim(it.group, it.name + "_dim1", it.rows);
            const int d2 = dim(it.group, it.name + "_dim2", it.cols);
            data_vars.push_back(w.h.AddVar(flat(it.group, it.name), NcDouble, {d1, d2}));
        }
    }
    if (!w.Create(filename, true)) return false;
    for (auto& c : coords) {
        std::vector<int32_t> v(c.n);
        for (size_t k = 0; k < c.n; k++) v[k] = (int32_t)(k + 1);
        if (c.n && !w.PutInt(c.var, {0}, {c.n}, v.data())) return false;
    }
    for (size_t k = 0; k < items_.size(); k++) {
        const Item& it = items_[k];
        bool ok = true;
        if (it.cols == 0 && it.rows == 0) continue;
        if (it.cols == 0)
            ok = it.is_int ? w.PutInt(data_vars[k], {0}, {it.rows}, it.i.data())
                           : w.PutDouble(data_vars[k], {0}, {it.rows}, it.d.data());
        else if (it.rows && it.cols)
            ok = w.PutDouble(data_vars[k], {0, 0}, {it.rows, it.cols}, it.d.data());
        if (!ok) return false;
    }
    w.Close();
    return true;
}

}  // namespace bcm3
