"""Summarise rocprofv3 PMC passes of bench.py into profiles/ (per-launch HBM traffic + SQ counters).

    python tools/pmc_traffic.py gpurun_out/r01 profiles r01 256

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KB (TCC_EA0 read/write requests x 64 B,
MI355X_MICROARCH.md "HBM / rocprofv3"). The gfx950 x2 correction applies to wide (16 B/lane)
coalesced streaming reads; this kernel's global reads are 8-byte scalar/per-lane loads of the
parameter vector and observations, so FETCH_SIZE is taken as is (stated in the output).
"""
import collections
import csv
import json
import os
import sys

KERNEL = "popk_traj_kernel"


def per_launch(path, counter):
    """mean over the dispatches of the most frequent grid size (the bench's speculative-pair launches;
    the few plain launches of its start and of the issue-rate probe are left out), and that grid"""
    vals = collections.defaultdict(float)
    grid = {}
    for r in csv.DictReader(open(path)):
        if KERNEL in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals[r["Dispatch_Id"]] += float(r["Counter_Value"])
            grid[r["Dispatch_Id"]] = r.get("Grid_Size", "?")
    if not vals:
        return None, 0, None
    g = collections.Counter(grid.values()).most_common(1)[0][0]
    v = [x for d, x in vals.items() if grid[d] == g]
    return sum(v) / len(v), len(v), g


def main():
    src, dst, tag, n = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    fetch_kb, nf, grid = per_launch(os.path.join(src, "pmc_fetch", "pmc_counter_collection.csv"), "FETCH_SIZE")
    write_kb, nw, _ = per_launch(os.path.join(src, "pmc_write", "pmc_counter_collection.csv"), "WRITE_SIZE")
    sq = {}
    sq_path = os.path.join(src, "pmc_sq", "pmc_counter_collection.csv")
    for c in ("SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"):
        sq[c] = per_launch(sq_path, c)[0]
    out = {
        "n": n,
        "kernel": KERNEL,
        "launches_fetch_pass": nf,
        "grid_size": grid,
        "launches_write_pass": nw,
        "fetch_kb_per_launch": fetch_kb,
        "write_kb_per_launch": write_kb,
        "bytes_per_launch": (fetch_kb + write_kb) * 1024.0,
        "fetch_correction": "none (8-byte loads, not 16 B/lane streaming reads)",
        "sq_per_launch": sq,
        "valu_per_wave": sq["SQ_INSTS_VALU"] / sq["SQ_WAVES"] if sq["SQ_WAVES"] else None,
        "salu_per_wave": sq["SQ_INSTS_SALU"] / sq["SQ_WAVES"] if sq["SQ_WAVES"] else None,
    }
    os.makedirs(dst, exist_ok=True)
    with open(os.path.join(dst, f"{tag}_traffic_c3_{n}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
