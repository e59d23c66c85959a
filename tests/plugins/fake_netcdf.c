/* fake_netcdf.c -- TEST DOUBLE of the system libnetcdf for tests/test_netcdf.py: the subset of the
 * netCDF C API that bcm3_amd/csrc/host/NetCDF4.cpp calls, serving the groups / dimensions /
 * variables of a small text manifest instead of an HDF5 file (neither libnetcdf nor HDF5 is in
 * this image). nc_open checks the HDF5 signature and reads the manifest that follows the first
 * line of the file:
 *   G <parent group> <name>                          group (root = 0, then 1, 2, ... in order)
 *   D <name> <length>                                dimension (ids 0, 1, ... in order)
 *   V <group> <name> <type> <ndims> <dimids...> <has_fill> <fill> <count> <values...>
 * type 6 = double, 9 = unsigned int (values as numbers), 12 = string, 2 = char (values are strings,
 * space-free). The writing calls NetCDF4.cpp makes for the sampler's output files (nc_create,
 * nc_def_grp / _dim / _var, nc_put_vara_double / _uint / _string, nc_sync, nc_close) build the same
 * model in memory and write it back as such a manifest; a value never written is the type's default
 * fill (NC_FILL_DOUBLE 9.969209968386869e36, NC_FILL_UINT 4294967295). Up to MAXF datasets are
 * open at once (the sampler writes output.nc and sampler_adaptation.nc side by side); an ncid is
 * (dataset << 24) | ((group + 1) << 16). Anything else returns an error code. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAXG 64
#define MAXV 256
#define MAXD 128

typedef struct {
    int group, type, ndims, dims[8], has_fill;
    double fill;
    char name[128];
    size_t count;
    double* num;
    char** str;
} Var;

#define MAXF 8
typedef struct {
    int used, writing;
    int ng, nd, nv;
    int gparent[MAXG];
    char gname[MAXG][128];
    char dname[MAXD][128];
    size_t dlen[MAXD];
    Var vars[MAXV];
    char wpath[4096];
} DS;
static DS files[MAXF];

static int gid(int ncid) { return ((ncid >> 16) & 0xff) - 1; }
static DS* ds_of(int ncid)
{
    const int f = ncid >> 24;
    return (f >= 0 && f < MAXF && files[f].used) ? &files[f] : NULL;
}
static int ncid_of(const DS* d, int g) { return (int)((d - files) << 24) | ((g + 1) << 16); }
static DS* ds_new(void)
{
    for (int f = 0; f < MAXF; f++)
        if (!files[f].used) {
            DS* d = &files[f];
            d->used = 1;
            d->writing = 0;
            d->ng = 1;
            d->nd = d->nv = 0;
            d->gparent[0] = -1;
            strcpy(d->gname[0], "/");
            return d;
        }
    return NULL;
}
static void ds_free(DS* d)
{
    for (int i = 0; i < d->nv; i++) {
        free(d->vars[i].num);
        if (d->vars[i].str)
            for (size_t k = 0; k < d->vars[i].count; k++) free(d->vars[i].str[k]);
        free(d->vars[i].str);
    }
    d->used = 0;
}
#define ng (d->ng)
#define nd (d->nd)
#define nv (d->nv)
#define gparent (d->gparent)
#define gname (d->gname)
#define dname (d->dname)
#define dlen (d->dlen)
#define vars (d->vars)
#define writing (d->writing)
#define wpath (d->wpath)

int nc_open(const char* path, int mode, int* ncidp)
{
    (void)mode;
    FILE* f = fopen(path, "rb");
    if (!f) return -31;
    char sig[8];
    if (fread(sig, 1, 8, f) != 8 || memcmp(sig, "\x89HDF\r\n\x1a\n", 8) != 0) {
        fclose(f);
        return -51; /* NC_ENOTNC */
    }
    int c;
    while ((c = fgetc(f)) != EOF && c != '\n') {
    }
    DS* d = ds_new();
    if (!d) {
        fclose(f);
        return -34; /* NC_ENFILE */
    }
    char tag[4];
    while (fscanf(f, "%3s", tag) == 1) {
        if (tag[0] == 'G') {
            if (fscanf(f, "%d %127s", &gparent[ng], gname[ng]) != 2) break;
            ng++;
        } else if (tag[0] == 'D') {
            if (fscanf(f, "%127s %zu", dname[nd], &dlen[nd]) != 2) break;
            nd++;
        } else if (tag[0] == 'V') {
            Var* v = &vars[nv++];
            memset(v, 0, sizeof(*v));
            if (fscanf(f, "%d %127s %d %d", &v->group, v->name, &v->type, &v->ndims) != 4) break;
            for (int k = 0; k < v->ndims; k++)
                if (fscanf(f, "%d", &v->dims[k]) != 1) break;
            if (fscanf(f, "%d %lf %zu", &v->has_fill, &v->fill, &v->count) != 3) break;
            if (v->type == 6 || v->type == 9) {
                v->num = calloc(v->count + 1, sizeof(double));
                for (size_t i = 0; i < v->count; i++) {
                    char tok[64];
                    if (fscanf(f, "%63s", tok) != 1) break;
                    v->num[i] = strtod(tok, NULL); /* "nan" parses to NaN */
                }
            } else {
                v->str = calloc(v->count + 1, sizeof(char*));
                for (size_t i = 0; i < v->count; i++) {
                    char tok[256];
                    if (fscanf(f, "%255s", tok) != 1) break;
                    v->str[i] = strdup(tok);
                }
            }
        }
    }
    fclose(f);
    *ncidp = ncid_of(d, 0);
    return 0;
}

static int write_manifest(DS* d);

int nc_close(int ncid)
{
    DS* d = ds_of(ncid);
    if (!d) return -33; /* NC_EBADID */
    const int r = writing ? write_manifest(d) : 0;
    ds_free(d);
    return r;
}

int nc_inq_grps(int ncid, int* numgrps, int* ncids)
{
    DS* d = ds_of(ncid);
    if (!d) return -33;
    int g = gid(ncid), n = 0;
    for (int i = 1; i < ng; i++)
        if (gparent[i] == g) {
            if (ncids) ncids[n] = ncid_of(d, i);
            n++;
        }
    if (numgrps) *numgrps = n;
    return 0;
}

int nc_inq_grpname(int ncid, char* name)
{
    DS* d = ds_of(ncid);
    if (!d) return -33;
    strcpy(name, gname[gid(ncid)]);
    return 0;
}

static Var* var_of(int ncid, int varid)
{
    DS* d = ds_of(ncid);
    if (!d) return NULL;
    int g = gid(ncid), k = 0;
    for (int i = 0; i < nv; i++)
        if (vars[i].group == g) {
            if (k == varid) return &vars[i];
            k++;
        }
    return NULL;
}

int nc_inq_varids(int ncid, int* nvars, int* varids)
{
    DS* d = ds_of(ncid);
    if (!d) return -33;
    int g = gid(ncid), n = 0;
    for (int i = 0; i < nv; i++)
        if (vars[i].group == g) {
            if (varids) varids[n] = n;
            n++;
        }
    if (nvars) *nvars = n;
    return 0;
}

int nc_inq_var(int ncid, int varid, char* name, int* xtypep, int* ndimsp, int* dimidsp, int* nattsp)
{
    Var* v = var_of(ncid, varid);
    if (!v) return -49; /* NC_ENOTVAR */
    if (name) strcpy(name, v->name);
    if (xtypep) *xtypep = v->type;
    if (ndimsp) *ndimsp = v->ndims;
    if (dimidsp)
        for (int k = 0; k < v->ndims; k++) dimidsp[k] = v->dims[k];
    if (nattsp) *nattsp = v->has_fill;
    return 0;
}

int nc_inq_dim(int ncid, int dimid, char* name, size_t* lenp)
{
    DS* d = ds_of(ncid);
    if (!d) return -33;
    if (dimid < 0 || dimid >= nd) return -46; /* NC_EBADDIM */
    if (name) strcpy(name, dname[dimid]);
    if (lenp) *lenp = dlen[dimid];
    return 0;
}

int nc_get_var_double(int ncid, int varid, double* ip)
{
    Var* v = var_of(ncid, varid);
    if (!v || (v->type != 6 && v->type != 9)) return -56;
    memcpy(ip, v->num, v->count * sizeof(double));
    return 0;
}

int nc_get_var_text(int ncid, int varid, char* ip)
{
    DS* d = ds_of(ncid);
    Var* v = var_of(ncid, varid);
    if (!v || v->type != 2) return -56;
    size_t w = dlen[v->dims[v->ndims - 1]];
    for (size_t i = 0; i < v->count; i++) {
        memset(ip + i * w, 0, w);
        strncpy(ip + i * w, v->str[i], w);
    }
    return 0;
}

int nc_get_var_string(int ncid, int varid, char** ip)
{
    Var* v = var_of(ncid, varid);
    if (!v || v->type != 12) return -56;
    for (size_t i = 0; i < v->count; i++) ip[i] = strdup(v->str[i]);
    return 0;
}

int nc_free_string(size_t len, char** data)
{
    for (size_t i = 0; i < len; i++) free(data[i]);
    return 0;
}

int nc_inq_att(int ncid, int varid, const char* name, int* xtypep, size_t* lenp)
{
    Var* v = var_of(ncid, varid);
    if (!v || strcmp(name, "_FillValue") != 0 || !v->has_fill) return -43; /* NC_ENOTATT */
    if (xtypep) *xtypep = v->type;
    if (lenp) *lenp = 1;
    return 0;
}

int nc_get_att_double(int ncid, int varid, const char* name, double* ip)
{
    Var* v = var_of(ncid, varid);
    if (!v || strcmp(name, "_FillValue") != 0 || !v->has_fill) return -43;
    *ip = v->fill;
    return 0;
}

const char* nc_strerror(int ncerr)
{
    static char buf[64];
    snprintf(buf, sizeof buf, "fake netCDF error %d", ncerr);
    return buf;
}

/* ---- writing ---- */
static size_t var_count(const DS* d, const Var* v)
{
    size_t n = 1;
    for (int k = 0; k < v->ndims; k++) n *= dlen[v->dims[k]];
    return n;
}

int nc_create(const char* path, int cmode, int* ncidp)
{
    if (!(cmode & 0x1000)) return -128; /* only NC_NETCDF4 */
    DS* d = ds_new();
    if (!d) return -34;
    snprintf(wpath, sizeof wpath, "%s", path);
    writing = 1;
    *ncidp = ncid_of(d, 0);
    return 0;
}

int nc_def_grp(int parent_ncid, const char* name, int* new_ncid)
{
    DS* d = ds_of(parent_ncid);
    if (!d || ng >= MAXG) return -1;
    gparent[ng] = gid(parent_ncid);
    snprintf(gname[ng], sizeof gname[ng], "%s", name);
    *new_ncid = ncid_of(d, ng);
    ng++;
    return 0;
}

int nc_def_dim(int ncid, const char* name, size_t len, int* idp)
{
    DS* d = ds_of(ncid);
    if (!d || nd >= MAXD) return -1;
    snprintf(dname[nd], sizeof dname[nd], "%s", name);
    dlen[nd] = len;
    *idp = nd++;
    return 0;
}

int nc_def_var(int ncid, const char* name, int xtype, int ndims, const int* dimidsp, int* varidp)
{
    DS* d = ds_of(ncid);
    if (!d || nv >= MAXV || ndims > 8 || (xtype != 6 && xtype != 9 && xtype != 12)) return -1;
    int g = gid(ncid), k = 0;
    for (int i = 0; i < nv; i++)
        if (vars[i].group == g) k++;
    Var* v = &vars[nv++];
    memset(v, 0, sizeof(*v));
    v->group = g;
    v->type = xtype;
    v->ndims = ndims;
    for (int d = 0; d < ndims; d++) v->dims[d] = dimidsp[d];
    snprintf(v->name, sizeof v->name, "%s", name);
    v->count = var_count(d, v);
    if (xtype == 12) {
        v->str = calloc(v->count + 1, sizeof(char*));
        for (size_t i = 0; i < v->count; i++) v->str[i] = strdup("");
    } else {
        v->num = calloc(v->count + 1, sizeof(double));
        for (size_t i = 0; i < v->count; i++) v->num[i] = (xtype == 6) ? 9.9692099683868690e+36 : 4294967295.0;
    }
    *varidp = k;
    return 0;
}

/* row-major offset of each element of the hyperslab, in order */
static int slab(const DS* d, const Var* v, const size_t* start, const size_t* count, size_t* n, size_t** offs)
{
    size_t total = 1;
    for (int k = 0; k < v->ndims; k++) {
        if (start[k] + count[k] > dlen[v->dims[k]]) return -40; /* NC_EEDGE */
        total *= count[k];
    }
    size_t* o = malloc((total + 1) * sizeof(size_t));
    size_t idx[8] = {0};
    for (size_t e = 0; e < total; e++) {
        size_t off = 0;
        for (int k = 0; k < v->ndims; k++) off = off * dlen[v->dims[k]] + start[k] + idx[k];
        o[e] = off;
        for (int k = v->ndims - 1; k >= 0; k--) {
            if (++idx[k] < count[k]) break;
            idx[k] = 0;
        }
    }
    *n = total;
    *offs = o;
    return 0;
}

int nc_put_vara_double(int ncid, int varid, const size_t* startp, const size_t* countp, const double* op)
{
    Var* v = var_of(ncid, varid);
    size_t n, *o;
    if (!v || v->type != 6) return -56;
    int r = slab(ds_of(ncid), v, startp, countp, &n, &o);
    if (r) return r;
    for (size_t e = 0; e < n; e++) v->num[o[e]] = op[e];
    free(o);
    return 0;
}

int nc_put_vara_uint(int ncid, int varid, const size_t* startp, const size_t* countp, const unsigned int* op)
{
    Var* v = var_of(ncid, varid);
    size_t n, *o;
    if (!v || v->type != 9) return -56;
    int r = slab(ds_of(ncid), v, startp, countp, &n, &o);
    if (r) return r;
    for (size_t e = 0; e < n; e++) v->num[o[e]] = (double)op[e];
    free(o);
    return 0;
}

int nc_put_vara_string(int ncid, int varid, const size_t* startp, const size_t* countp, const char** op)
{
    Var* v = var_of(ncid, varid);
    size_t n, *o;
    if (!v || v->type != 12) return -56;
    int r = slab(ds_of(ncid), v, startp, countp, &n, &o);
    if (r) return r;
    for (size_t e = 0; e < n; e++) {
        free(v->str[o[e]]);
        v->str[o[e]] = strdup(op[e]);
    }
    free(o);
    return 0;
}

static int write_manifest(DS* d)
{
    FILE* f = fopen(wpath, "wb");
    if (!f) return -31;
    static const char sig[] = "\x89HDF\r\n\x1a\n fake netCDF-4 written by tests/plugins/fake_netcdf.c\n";
    fwrite(sig, 1, sizeof sig - 1, f);
    for (int i = 1; i < ng; i++) fprintf(f, "G %d %s\n", gparent[i], gname[i]);
    for (int i = 0; i < nd; i++) fprintf(f, "D %s %zu\n", dname[i], dlen[i]);
    for (int i = 0; i < nv; i++) {
        const Var* v = &vars[i];
        fprintf(f, "V %d %s %d %d", v->group, v->name, v->type, v->ndims);
        for (int k = 0; k < v->ndims; k++) fprintf(f, " %d", v->dims[k]);
        fprintf(f, " 0 0 %zu", v->count);
        for (size_t e = 0; e < v->count; e++) {
            if (v->type == 12)
                fprintf(f, " %s", v->str[e][0] ? v->str[e] : "-");
            else
                fprintf(f, " %.17g", v->num[e]);
        }
        fprintf(f, "\n");
    }
    fclose(f);
    return 0;
}

int nc_sync(int ncid)
{
    DS* d = ds_of(ncid);
    if (!d) return -33;
    return writing ? write_manifest(d) : 0;
}
