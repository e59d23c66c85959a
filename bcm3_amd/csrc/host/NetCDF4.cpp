// NetCDF4.cpp -- netCDF-4 (HDF5-backed) data files through the system's libnetcdf, loaded at run
// time when present (the reference links libnetcdf and reads its data through NetCDFDataFile,
// src/utils/NetCDFDataFile.cpp). Neither libnetcdf nor HDF5 is in this image, so the library is
// dlopen()ed: $BCM3_LIBNETCDF if set, else libnetcdf.so / .so.22 / .so.19 / .so.18 / .so.15 on the
// loader's search path. Without it a netCDF-4 file is refused with the conversion command
// (tools/nc_convert.py), as before. The result has the layout NcClassicRead gives a classic file:
// doc[group][variable] = {"dims": [dimension names], "data": nested values}, nested groups named
// "a.b", the root group "", fill values -> NaN, char arrays -> strings.
// The same library writes the sampler's output.nc and sampler_adaptation.nc as netCDF-4 with real
// groups (NcNetCDF4Writer: nc_create(NC_CLOBBER | NC_NETCDF4) as NetCDFDataFile::Create,
// src/utils/NetCDFDataFile.cpp:117-260) when it is present and has the writing API.
#include <dlfcn.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <mutex>
#include <string>
#include <type_traits>
#include <vector>

#include "NetCDFClassic.h"
#include "log.h"

namespace bcm3 {

// the writing subset (nc_create ... nc_close), resolved separately: a reader-only test double or an
// old library still serves the data files
struct NcWriteApi {
    int (*create)(const char*, int, int*) = nullptr;
    int (*def_grp)(int, const char*, int*) = nullptr;
    int (*def_dim)(int, const char*, size_t, int*) = nullptr;
    int (*def_var)(int, const char*, int, int, const int*, int*) = nullptr;
    int (*put_vara_double)(int, int, const size_t*, const size_t*, const double*) = nullptr;
    int (*put_vara_uint)(int, int, const size_t*, const size_t*, const unsigned int*) = nullptr;
    int (*put_vara_string)(int, int, const size_t*, const size_t*, const char**) = nullptr;
    int (*sync)(int) = nullptr;
    int (*close)(int) = nullptr;
    const char* (*strerror)(int) = nullptr;
    bool ok = false;
};

namespace {

// the subset of the netCDF C API (netcdf.h) this reader calls
struct NcApi {
    int (*open)(const char*, int, int*) = nullptr;
    int (*close)(int) = nullptr;
    int (*inq_grps)(int, int*, int*) = nullptr;
    int (*inq_grpname)(int, char*) = nullptr;
    int (*inq_varids)(int, int*, int*) = nullptr;
    int (*inq_var)(int, int, char*, int*, int*, int*, int*) = nullptr;
    int (*inq_dim)(int, int, char*, size_t*) = nullptr;
    int (*get_var_double)(int, int, double*) = nullptr;
    int (*get_var_text)(int, int, char*) = nullptr;
    int (*get_var_string)(int, int, char**) = nullptr;
    int (*free_string)(size_t, char**) = nullptr;
    int (*inq_att)(int, int, const char*, int*, size_t*) = nullptr;
    int (*get_att_double)(int, int, const char*, double*) = nullptr;
    const char* (*strerror)(int) = nullptr;
    void* handle = nullptr;
    std::string error;
    std::string env;  // $BCM3_LIBNETCDF when the library was loaded
    NcWriteApi write;
};

constexpr int kNcNoWrite = 0, kNcMaxName = 256, kNcMaxDims = 1024, kNcClobber = 0, kNcNetCDF4 = 0x1000;
constexpr int kNcByte = 1, kNcChar = 2, kNcShort = 3, kNcInt = 4, kNcFloat = 5, kNcDouble = 6, kNcString = 12;
constexpr double kFillDouble = 9.9692099683868690e+36, kFillFloat = 9.9692099683868690e+36f;

// loads libnetcdf on first success; a failed attempt is retried on the next call (a later
// $BCM3_LIBNETCDF or install is seen), and a change of $BCM3_LIBNETCDF switches libraries. A
// loaded library is never unloaded and its NcApi never changes: readers and writers that hold it
// (NcNetCDF4Writer pins the write API at Create) keep calling into the library their ids came from.
const NcApi& api()
{
    static std::mutex mu;
    static std::vector<std::unique_ptr<NcApi>> loaded;  // every library loaded so far, never freed
    static const NcApi* cur = nullptr;
    static NcApi failed;  // the last failed attempt (error only)
    std::lock_guard<std::mutex> lock(mu);
    const char* env_now = std::getenv("BCM3_LIBNETCDF");
    const std::string env = env_now ? env_now : "";
    if (cur && cur->env == env) return *cur;
    for (const auto& l : loaded)
        if (l->env == env) return *(cur = l.get());
    std::vector<std::string> names;
    if (!env.empty()) names.push_back(env);
    for (const char* n : {"libnetcdf.so", "libnetcdf.so.22", "libnetcdf.so.19", "libnetcdf.so.18", "libnetcdf.so.15"})
        names.push_back(n);
    void* h = nullptr;
    for (const auto& n : names)
        if ((h = dlopen(n.c_str(), RTLD_NOW | RTLD_LOCAL))) break;
    failed = NcApi();
    if (!h) {
        failed.error = "libnetcdf was not found";
        return failed;
    }
    std::unique_ptr<NcApi> t(new NcApi());
    bool ok = true;
    auto sym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        ok &= fn != nullptr;
    };
    sym(t->open, "nc_open");
    sym(t->close, "nc_close");
    sym(t->inq_grps, "nc_inq_grps");
    sym(t->inq_grpname, "nc_inq_grpname");
    sym(t->inq_varids, "nc_inq_varids");
    sym(t->inq_var, "nc_inq_var");
    sym(t->inq_dim, "nc_inq_dim");
    sym(t->get_var_double, "nc_get_var_double");
    sym(t->get_var_text, "nc_get_var_text");
    sym(t->get_var_string, "nc_get_var_string");
    sym(t->free_string, "nc_free_string");
    sym(t->inq_att, "nc_inq_att");
    sym(t->get_att_double, "nc_get_att_double");
    sym(t->strerror, "nc_strerror");
    if (!ok) {
        dlclose(h);  // nothing holds this handle yet
        failed.error = "the libnetcdf found lacks the netCDF-4 group API";
        return failed;
    }
    t->handle = h;
    t->env = env;
    // the writing subset, resolved once (a reader-only test double or an old library leaves it !ok)
    NcWriteApi& w = t->write;
    bool wok = true;
    auto wsym = [&](auto& fn, const char* name) {
        fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
        wok &= fn != nullptr;
    };
    wsym(w.create, "nc_create");
    wsym(w.def_grp, "nc_def_grp");
    wsym(w.def_dim, "nc_def_dim");
    wsym(w.def_var, "nc_def_var");
    wsym(w.put_vara_double, "nc_put_vara_double");
    wsym(w.put_vara_uint, "nc_put_vara_uint");
    wsym(w.put_vara_string, "nc_put_vara_string");
    wsym(w.sync, "nc_sync");
    wsym(w.close, "nc_close");
    w.strerror = t->strerror;
    w.ok = wok;
    loaded.push_back(std::move(t));
    return *(cur = loaded.back().get());
}

void check(const NcApi& a, int rc, const std::string& what)
{
    if (rc != 0) throw JsonError{"netCDF-4: " + what + ": " + (a.strerror ? a.strerror(rc) : std::to_string(rc))};
}

// nest a flat row-major vector along `shape`
Json nest(std::vector<Json> flat, const std::vector<size_t>& shape)
{
    if (shape.empty()) return flat.empty() ? Json() : flat[0];
    for (size_t k = shape.size(); k-- > 1;) {
        std::vector<Json> up;
        const size_t m = shape[k];
        for (size_t i = 0; i + m <= flat.size() && m > 0; i += m) {
            Json a;
            a.type = Json::Array;
            a.arr.assign(std::make_move_iterator(flat.begin() + i), std::make_move_iterator(flat.begin() + i + m));
            up.push_back(std::move(a));
        }
        flat = std::move(up);
    }
    Json data;
    data.type = Json::Array;
    data.arr = std::move(flat);
    return data;
}

void read_group(const NcApi& a, int grp, const std::string& path, Json& doc)
{
    int nvars = 0;
    check(a, a.inq_varids(grp, &nvars, nullptr), "nc_inq_varids");
    std::vector<int> ids((size_t)nvars);
    if (nvars) check(a, a.inq_varids(grp, &nvars, ids.data()), "nc_inq_varids");
    for (int vid : ids) {
        char name[kNcMaxName + 1] = {0};
        int type = 0, ndims = 0, natts = 0;
        std::vector<int> dimids(kNcMaxDims);
        check(a, a.inq_var(grp, vid, name, &type, &ndims, dimids.data(), &natts), "nc_inq_var");
        std::vector<size_t> shape;
        Json dims;
        dims.type = Json::Array;
        size_t total = 1;
        for (int k = 0; k < ndims; k++) {
            char dn[kNcMaxName + 1] = {0};
            size_t len = 0;
            check(a, a.inq_dim(grp, dimids[k], dn, &len), std::string("nc_inq_dim of ") + name);
            shape.push_back(len);
            total *= len;
            Json d;
            d.type = Json::String;
            d.str = dn;
            dims.arr.push_back(d);
        }
        std::vector<Json> flat;
        if (type == kNcChar && !shape.empty()) {  // the last dimension holds the characters
            std::vector<char> buf(total);
            if (total) check(a, a.get_var_text(grp, vid, buf.data()), std::string("nc_get_var_text of ") + name);
            const size_t inner = std::max<size_t>(shape.back(), 1);
            for (size_t i = 0; i + inner <= buf.size(); i += inner) {
                Json s;
                s.type = Json::String;
                s.str.assign(&buf[i], strnlen(&buf[i], inner));
                flat.push_back(std::move(s));
            }
            shape.pop_back();
            dims.arr.pop_back();
        } else if (type == kNcString) {
            std::vector<char*> buf(total, nullptr);
            if (total) check(a, a.get_var_string(grp, vid, buf.data()), std::string("nc_get_var_string of ") + name);
            for (char* p : buf) {
                Json s;
                s.type = Json::String;
                if (p) s.str = p;
                flat.push_back(std::move(s));
            }
            if (total) a.free_string(total, buf.data());
        } else if (type >= kNcByte && type <= 11) {  // numeric types, converted by the library
            std::vector<double> buf(total);
            if (total) check(a, a.get_var_double(grp, vid, buf.data()), std::string("nc_get_var_double of ") + name);
            // fill values -> NaN: the variable's _FillValue, else the type's default fill
            int at = 0;
            size_t alen = 0;
            double fill = std::numeric_limits<double>::quiet_NaN();
            bool has_fill = a.inq_att(grp, vid, "_FillValue", &at, &alen) == 0 && alen == 1 &&
                            a.get_att_double(grp, vid, "_FillValue", &fill) == 0;
            for (double x : buf) {
                bool is_fill = has_fill ? x == fill
                                        : (type == kNcDouble && (x == kFillDouble || x == (double)kFillFloat)) ||
                                              (type == kNcFloat && x == (double)kFillFloat) ||
                                              (type == kNcInt && x == -2147483647.0) || (type == kNcShort && x == -32767.0) ||
                                              (type == kNcByte && x == -127.0);
                Json e;
                e.type = Json::Number;
                e.num = is_fill ? std::numeric_limits<double>::quiet_NaN() : x;
                flat.push_back(std::move(e));
            }
        } else {
            continue;  // compound / opaque / enum / vlen: not data BCM3 reads
        }
        Json var;
        var.type = Json::Object;
        var.obj["dims"] = dims;
        var.obj["data"] = nest(std::move(flat), shape);
        Json& g = doc.obj[path];
        g.type = Json::Object;
        g.obj[name] = std::move(var);
    }
    int ngrps = 0;
    check(a, a.inq_grps(grp, &ngrps, nullptr), "nc_inq_grps");
    std::vector<int> sub((size_t)ngrps);
    if (ngrps) check(a, a.inq_grps(grp, &ngrps, sub.data()), "nc_inq_grps");
    for (int s : sub) {
        char gn[kNcMaxName + 1] = {0};
        check(a, a.inq_grpname(s, gn), "nc_inq_grpname");
        read_group(a, s, path.empty() ? std::string(gn) : path + "." + gn, doc);
    }
}

const NcWriteApi& wapi() { return api().write; }

bool wcheck(const NcWriteApi& w, int rc, const std::string& what)
{
    if (rc == 0) return true;
    LOGERROR("netCDF-4 output: %s: %s", what.c_str(), w.strerror ? w.strerror(rc) : std::to_string(rc).c_str());
    return false;
}

}  // namespace

bool NcNetCDF4WriteAvailable(std::string* why)
{
    std::string r;
    const bool have = NcNetCDF4Available(&r) && wapi().ok;
    if (why) *why = have ? "" : (r.empty() ? "the libnetcdf found cannot write (nc_create / nc_def_*)" : r);
    if (have) {
        // BCM3_OUTPUT_FORMAT=classic keeps the netCDF classic output even with libnetcdf present
        const char* f = std::getenv("BCM3_OUTPUT_FORMAT");
        if (f && std::string(f) == "classic") {
            if (why) *why = "BCM3_OUTPUT_FORMAT=classic";
            return false;
        }
    }
    return have;
}

// NetCDFDataFile::Create / CreateGroup / CreateDimension / CreateVariable / PutValue(s)
// (src/utils/NetCDFDataFile.cpp:117-260) over the run-time loaded library
bool NcNetCDF4Writer::Create(const std::string& filename)
{
    Close();
    const NcWriteApi& w = wapi();
    if (!w.ok) return false;
    filename_ = filename;
    w_ = &w;  // this file's library until Close, whatever $BCM3_LIBNETCDF does meanwhile
    return wcheck(w, w.create(filename.c_str(), kNcClobber | kNcNetCDF4, &nc_), "nc_create " + filename);
}

int NcNetCDF4Writer::Group(const std::string& path)
{
    if (nc_ < 0) return -1;
    if (path.empty()) return nc_;
    auto it = groups_.find(path);
    if (it != groups_.end()) return it->second;
    const size_t slash = path.rfind('/');
    const int parent = (slash == std::string::npos) ? nc_ : Group(path.substr(0, slash));
    if (parent < 0) return -1;
    int g = -1;
    const std::string name = (slash == std::string::npos) ? path : path.substr(slash + 1);
    if (!wcheck(*w_, w_->def_grp(parent, name.c_str(), &g), "nc_def_grp " + path)) return -1;
    groups_[path] = g;
    return g;
}

int NcNetCDF4Writer::Dim(int grp, const std::string& name, size_t len)
{
    int d = -1;
    return wcheck(*w_, w_->def_dim(grp, name.c_str(), len, &d), "nc_def_dim " + name) ? d : -1;
}

int NcNetCDF4Writer::Var(int grp, const std::string& name, int type, const std::vector<int>& dims)
{
    int v = -1;
    return wcheck(*w_, w_->def_var(grp, name.c_str(), type, (int)dims.size(), dims.data(), &v), "nc_def_var " + name) ? v
                                                                                                                       : -1;
}

bool NcNetCDF4Writer::PutDouble(int grp, int var, const std::vector<size_t>& start, const std::vector<size_t>& count,
                                const double* data)
{
    return wcheck(*w_, w_->put_vara_double(grp, var, start.data(), count.data(), data), "nc_put_vara_double");
}

bool NcNetCDF4Writer::PutUInt(int grp, int var, const std::vector<size_t>& start, const std::vector<size_t>& count,
                              const uint32_t* data)
{
    return wcheck(*w_, w_->put_vara_uint(grp, var, start.data(), count.data(), data), "nc_put_vara_uint");
}

bool NcNetCDF4Writer::PutStrings(int grp, int var, const std::vector<std::string>& s)
{
    std::vector<const char*> p;
    for (auto& x : s) p.push_back(x.c_str());
    const size_t start = 0, count = s.size();
    return wcheck(*w_, w_->put_vara_string(grp, var, &start, &count, p.data()), "nc_put_vara_string");
}

bool NcNetCDF4Writer::Sync() { return nc_ < 0 || wcheck(*w_, w_->sync(nc_), "nc_sync"); }

void NcNetCDF4Writer::Close()
{
    if (nc_ >= 0) wcheck(*w_, w_->close(nc_), "nc_close " + filename_);
    nc_ = -1;
    groups_.clear();
}

bool NcNetCDF4Available(std::string* why)
{
    const NcApi& a = api();
    if (why) *why = a.error;
    return a.handle != nullptr;
}

Json NcNetCDF4Read(const std::string& filename)
{
    const NcApi& a = api();
    if (!a.handle) throw JsonError{a.error};
    int nc = -1;
    check(a, a.open(filename.c_str(), kNcNoWrite, &nc), "nc_open " + filename);
    Json doc;
    doc.type = Json::Object;
    try {
        read_group(a, nc, "", doc);
    } catch (...) {
        a.close(nc);
        throw;
    }
    a.close(nc);
    return doc;
}

}  // namespace bcm3
