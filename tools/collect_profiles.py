"""Copy the round-end evidence from gpurun_out/<tag> into profiles/ (tracked).

    python tools/collect_profiles.py r01
"""
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    os.makedirs(dst, exist_ok=True)
    copies = {
        os.path.join(src, "kt", "kt_kernel_stats.csv"): f"{tag}_kernel_stats.csv",
        os.path.join(src, "kt_extras", "kt_kernel_stats.csv"): f"{tag}_kernel_stats_extras.csv",
        os.path.join(src, "smoke.log"): f"{tag}_smoke.log",
        os.path.join(src, "bench.json"): f"{tag}_bench.json",
        os.path.join(src, "ubench_lat.txt"): f"{tag}_ubench_lat.txt",
        os.path.join(src, "ubench_branch.txt"): f"{tag}_ubench_branch.txt",
        os.path.join(src, "probe.log"): f"{tag}_lpw_sweep.txt",
        os.path.join(src, "pytest_gpu.log"): f"{tag}_pytest_gpu.log",
    }
    for a, b in copies.items():
        if os.path.exists(a):
            shutil.copy(a, os.path.join(dst, b))
            print("copied", b)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), src, dst, tag, "256"], check=True,
                   stdout=subprocess.DEVNULL)
    # per-dispatch durations of the BDF kernel by launch size (kernel trace of the bench): the
    # speculative-pair launches are the largest grid; the bench's own HIP-event average is over them
    tr = os.path.join(src, "kt", "kt_kernel_trace.csv")
    if os.path.exists(tr):
        import collections
        import csv
        by = collections.defaultdict(list)
        for r in csv.DictReader(open(tr)):
            if "popk_traj_kernel" in r["Kernel_Name"]:
                by[r.get("Grid_Size_X", r.get("Grid_Size", "?"))].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
        summ = {g: {"dispatches": len(v), "avg_ms": sum(v) / len(v), "min_ms": min(v), "max_ms": max(v)}
                for g, v in by.items()}
        with open(os.path.join(dst, f"{tag}_popk_dispatch_durations.json"), "w") as f:
            json.dump(summ, f, indent=1)
        print("wrote", f"{tag}_popk_dispatch_durations.json")
    # second SQ pass
    import collections
    import csv
    p = os.path.join(src, "pmc_sq2", "pmc_counter_collection.csv")
    if os.path.exists(p):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            if "popk_traj_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        with open(os.path.join(dst, f"{tag}_pmc_sq2.json"), "w") as f:
            json.dump({k: sum(v) / len(v) for k, v in agg.items()}, f, indent=1)
        print("wrote", f"{tag}_pmc_sq2.json")


if __name__ == "__main__":
    main()
