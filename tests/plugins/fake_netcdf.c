/* fake_netcdf.c -- TEST DOUBLE of the system libnetcdf for tests/test_netcdf.py: the subset of the
 * netCDF C API that bcm3_amd/csrc/host/NetCDF4.cpp calls, serving the groups / dimensions /
 * variables of a small text manifest instead of an HDF5 file (neither libnetcdf nor HDF5 is in
 * this image). nc_open checks the HDF5 signature and reads the manifest that follows the first
 * line of the file:
 *   G <parent group> <name>                          group (root = 0, then 1, 2, ... in order)
 *   D <name> <length>                                dimension (ids 0, 1, ... in order)
 *   V <group> <name> <type> <ndims> <dimids...> <has_fill> <fill> <count> <values...>
 * type 6 = double (values as numbers), 12 = string, 2 = char (values are strings, space-free).
 * Only the calls the reader makes are implemented; anything else returns an error code. */
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

static int ng, nd, nv;
static int gparent[MAXG];
static char gname[MAXG][128];
static char dname[MAXD][128];
static size_t dlen[MAXD];
static Var vars[MAXV];

static int gid(int ncid) { return ncid / 65536 - 1; }

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
    ng = 1;
    nd = nv = 0;
    gparent[0] = -1;
    strcpy(gname[0], "/");
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
            if (v->type == 6) {
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
    *ncidp = 65536;
    return 0;
}

int nc_close(int ncid) { (void)ncid; return 0; }

int nc_inq_grps(int ncid, int* numgrps, int* ncids)
{
    int g = gid(ncid), n = 0;
    for (int i = 1; i < ng; i++)
        if (gparent[i] == g) {
            if (ncids) ncids[n] = (i + 1) * 65536;
            n++;
        }
    if (numgrps) *numgrps = n;
    return 0;
}

int nc_inq_grpname(int ncid, char* name)
{
    strcpy(name, gname[gid(ncid)]);
    return 0;
}

static Var* var_of(int ncid, int varid)
{
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
    (void)ncid;
    if (dimid < 0 || dimid >= nd) return -46; /* NC_EBADDIM */
    if (name) strcpy(name, dname[dimid]);
    if (lenp) *lenp = dlen[dimid];
    return 0;
}

int nc_get_var_double(int ncid, int varid, double* ip)
{
    Var* v = var_of(ncid, varid);
    if (!v || v->type != 6) return -56;
    memcpy(ip, v->num, v->count * sizeof(double));
    return 0;
}

int nc_get_var_text(int ncid, int varid, char* ip)
{
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
