"""Convert between the reference's netCDF-4 files and the formats libbcm3 reads and writes.

The reference reads its data (pkdata.nc, cellpop data) and writes output.nc through netCDF-4, i.e.
HDF5 with groups (src/utils/NetCDFDataFile.cpp). This image has neither libnetcdf nor HDF5, so
libbcm3 reads netCDF classic files and JSON sidecars and writes output.nc as netCDF classic, with a
group g's dimension or variable n named "g.n" (bcm3_amd/csrc/host/NetCDFClassic.h).

    python tools/nc_convert.py to-classic IN OUT     IN: netCDF-4 (needs netCDF4 or h5py) or JSON sidecar
    python tools/nc_convert.py to-json IN OUT        IN: netCDF classic (scipy) or netCDF-4
    python tools/nc_convert.py to-netcdf4 IN OUT     IN: netCDF classic; OUT for R/load.r (needs netCDF4)

JSON sidecar: {"<group>": {"<var>": {"dims": [...], "data": nested lists}}} (null = NaN); the
plain form {"<group>": {"<var>": nested lists}} is accepted on input.
"""
import json
import math
import sys

import numpy as np

FILL_DOUBLE = 9.9692099683868690e+36


def _is_hdf5(path):
    with open(path, "rb") as f:
        return f.read(4) == b"\x89HDF"


# ---- the in-memory form: {group: {var: (dims, ndarray)}}

def _from_json(path):
    doc = json.load(open(path))
    out = {}
    for g, grp in doc.items():
        coords = {k: len(v) for k, v in grp.items() if isinstance(v, list) and k in ("time", "patients")}
        vars_ = {}
        for name, v in grp.items():
            if isinstance(v, dict) and "data" in v:
                dims, data = list(v["dims"]), v["data"]
            else:
                data = v
                shape = np.shape(np.array(data, dtype=object))
                dims = []
                for k, n in enumerate(shape):
                    hit = [c for c, m in coords.items() if m == n and c not in dims]
                    dims.append(name if (len(shape) == 1 and name in coords) else (hit[0] if hit else f"{name}_d{k}"))
            arr = np.array(data, dtype=object)
            if arr.size and all(isinstance(x, str) for x in arr.reshape(-1)):
                vars_[name] = (dims, arr.astype(str))
            else:
                vars_[name] = (dims, np.array([np.nan if x is None else x for x in arr.reshape(-1)],
                                              dtype=np.float64).reshape(arr.shape))
        out[g] = vars_
    return out


def _from_classic(path):
    from scipy.io import netcdf_file
    out = {}
    with netcdf_file(path, "r", mmap=False) as f:
        for full, v in f.variables.items():
            g, _, name = full.rpartition(".") if "." in full else ("", "", full)
            g = g.replace(".", "/")  # nested groups a.b -> a/b
            dims = [d.rpartition(".")[2] for d in v.dimensions]
            data = np.array(v[:])
            if data.dtype.kind == "S":
                data = np.array([b"".join(r).decode() for r in data.reshape(-1, data.shape[-1])]).reshape(data.shape[:-1])
                dims = dims[:-1]
            elif data.dtype.kind == "f":
                fill = getattr(v, "_FillValue", FILL_DOUBLE)
                data = np.where(data == fill, np.nan, data)
            out.setdefault(g, {})[name] = (dims, data)
    return out


def _from_netcdf4(path):
    try:
        import netCDF4
    except ImportError:
        netCDF4 = None
    out = {}
    if netCDF4 is not None:
        ds = netCDF4.Dataset(path, "r")

        def walk(grp, prefix):
            for name, v in grp.variables.items():
                data = v[:]
                data = np.ma.filled(data, np.nan) if data.dtype.kind == "f" else np.ma.getdata(data)
                out.setdefault(prefix, {})[name] = (list(v.dimensions), np.array(data))
            for gname, sub in grp.groups.items():
                walk(sub, f"{prefix}/{gname}" if prefix else gname)
        walk(ds, "")
        ds.close()
        return out
    try:
        import h5py
    except ImportError:
        sys.exit("reading netCDF-4 needs the netCDF4 or h5py module, neither is installed here")
    with h5py.File(path, "r") as f:
        def visit(name, obj):
            if isinstance(obj, h5py.Dataset):
                g, _, leaf = name.rpartition("/")
                data = obj[()]
                if data.dtype.kind in "SO":
                    data = np.array([x.decode() if isinstance(x, bytes) else str(x) for x in np.ravel(data)]).reshape(np.shape(data))
                elif data.dtype.kind == "f":
                    fill = obj.attrs.get("_FillValue", [FILL_DOUBLE])
                    data = np.where(data == np.ravel(fill)[0], np.nan, data)
                dims = [f"{leaf}_d{k}" for k in range(np.ndim(data))]
                if "DIMENSION_LIST" in obj.attrs:
                    dims = [f[ref[0]].name.rpartition("/")[2] for ref in obj.attrs["DIMENSION_LIST"]]
                out.setdefault(g, {})[leaf] = (dims, data)
        f.visititems(visit)
    return out


def _load(path):
    if _is_hdf5(path):
        return _from_netcdf4(path)
    with open(path, "rb") as f:
        magic = f.read(3)
    return _from_classic(path) if magic == b"CDF" else _from_json(path)


# ---- writers

def _to_classic(doc, path):
    from scipy.io import netcdf_file
    f = netcdf_file(path, "w", version=2)
    groups = [g for g in doc if g]
    if groups:
        f.bcm3_groups = " ".join(groups)
    made = set()
    for g, vars_ in doc.items():
        pre = (g.replace("/", ".") + ".") if g else ""
        for name, (dims, data) in vars_.items():
            dims = list(dims)
            if data.dtype.kind in "US":
                strlen = max([1] + [len(s) for s in data.reshape(-1)])
                chars = np.zeros(data.shape + (strlen,), dtype="S1")
                for i, s in enumerate(data.reshape(-1)):
                    for k, ch in enumerate(s.encode()):
                        chars.reshape(-1, strlen)[i, k] = bytes([ch])
                dims = dims + [f"{name}_strlen"]
                data = chars
            for k, dn in enumerate(dims):
                if pre + dn not in made:
                    f.createDimension(pre + dn, data.shape[k])
                    made.add(pre + dn)
            if data.dtype.kind in "iu":
                v = f.createVariable(pre + name, "i", tuple(pre + d for d in dims))
                v[:] = data.astype(np.int32)
            elif data.dtype.kind == "S":
                v = f.createVariable(pre + name, "c", tuple(pre + d for d in dims))
                v[:] = data
            else:
                v = f.createVariable(pre + name, "d", tuple(pre + d for d in dims))
                v[:] = np.asarray(data, dtype=np.float64)
    f.close()


def _to_json(doc, path):
    def enc(x):
        if isinstance(x, float) and math.isnan(x):
            return None
        return x
    out = {}
    for g, vars_ in doc.items():
        og = out.setdefault(g, {})
        for name, (dims, data) in vars_.items():
            lst = data.tolist()

            def clean(o):
                return [clean(e) for e in o] if isinstance(o, list) else enc(o)
            og[name] = {"dims": list(dims), "data": clean(lst)}
    json.dump(out, open(path, "w"))


def _to_netcdf4(doc, path):
    try:
        import netCDF4
    except ImportError:
        sys.exit("writing netCDF-4 needs the netCDF4 module, which is not installed here")
    ds = netCDF4.Dataset(path, "w", format="NETCDF4")
    for g, vars_ in doc.items():
        grp = ds
        for part in [p for p in g.split("/") if p]:
            grp = grp.groups[part] if part in grp.groups else grp.createGroup(part)
        for name, (dims, data) in vars_.items():
            for k, dn in enumerate(dims):
                if dn not in grp.dimensions:
                    grp.createDimension(dn, data.shape[k])
            if data.dtype.kind == "U":
                v = grp.createVariable(name, str, tuple(dims))
                for i, s in enumerate(data.reshape(-1)):
                    v[np.unravel_index(i, data.shape)] = s
            else:
                v = grp.createVariable(name, data.dtype if data.dtype.kind in "iu" else "f8", tuple(dims),
                                       fill_value=None if data.dtype.kind in "iu" else FILL_DOUBLE)
                v[:] = data
    ds.close()


def main(argv):
    if len(argv) != 4 or argv[1] not in ("to-classic", "to-json", "to-netcdf4"):
        sys.exit(__doc__)
    doc = _load(argv[2])
    {"to-classic": _to_classic, "to-json": _to_json, "to-netcdf4": _to_netcdf4}[argv[1]](doc, argv[3])


if __name__ == "__main__":
    main(sys.argv)
