"""Per-launch HBM traffic of the MAC kernels from two rocprofv3 PMC passes -> profiles/pmc_traffic.json.

usage: python tools/pmc_traffic.py <config> <fetch_counter_collection.csv> <write_counter_collection.csv>

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (summed over the agent).  On gfx950 FETCH_SIZE
reports half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section), so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane stores.  bench.py reads the result as
roofline.traffic for the dominant kernel.
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOW = "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE passes of bench.py --steps 2 --warmup 1 (tools/gpu_pmc.sh)"
KERNELS = {"encode_mac": (r"gf_mac_bs<\d+, false", r"gf_mac<\d, false"),
           "decode_mac": (r"gf_mac_bs<\d+, true", r"gf_mac<\d, true")}


def git_head():
    """The commit the measured tree was sent from (gpurun snapshots this working tree);
    NTC_PMC_COMMIT overrides it when the counters are processed after later commits."""
    import subprocess
    if os.environ.get("NTC_PMC_COMMIT"):
        return os.environ["NTC_PMC_COMMIT"]
    try:
        h = subprocess.run(["git", "-C", ROOT, "rev-parse", "--short=12", "HEAD"], capture_output=True,
                           text=True, check=True).stdout.strip()
        dirty = subprocess.run(["git", "-C", ROOT, "status", "--porcelain", "--untracked-files=no", "--",
                                ".", ":!profiles"],
                               capture_output=True, text=True).stdout.strip()
        return h + ("+dirty" if dirty else "")
    except (OSError, subprocess.CalledProcessError):
        return "unknown"


def means(path, counter):
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] != counter:
            continue
        acc[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def pick(table, names):
    for k, v in table.items():
        if any(re.search(n, k) for n in names):
            return v
    return None


def main():
    cfg, fpath, wpath = sys.argv[1:4]
    fetch, write = means(fpath, "FETCH_SIZE"), means(wpath, "WRITE_SIZE")
    out_p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    out = json.load(open(out_p)) if os.path.exists(out_p) else {}
    ent = {}
    for key, names in KERNELS.items():
        f, w = pick(fetch, names), pick(write, names)
        if f is None or w is None:
            continue
        rd, wr = 2 * f * 1024, w * 1024
        ent[key] = int(rd + wr)
        ent[key + "_detail"] = {"read_bytes": int(rd), "write_bytes": int(wr),
                                "FETCH_SIZE_KiB_raw": f, "WRITE_SIZE_KiB": w}
    ent["note"] = ("bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KiB x 1024); FETCH_SIZE doubled "
                   "per the gfx950 correction")
    ent["_commit"] = git_head()
    ent["_how"] = HOW
    out[cfg] = ent
    json.dump(out, open(out_p, "w"), indent=1)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()
