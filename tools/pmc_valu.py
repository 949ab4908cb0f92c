"""VALU-op fraction of the MAC kernels from the SQ passes of tools/gpu_sq.sh -> profiles/pmc_valu.json.

usage: python tools/pmc_valu.py <config> <sq/run_counter_collection.csv> <sq2/run_counter_collection.csv>

Per launch (mean over dispatches; SQ counters are summed over the agent):
  valu_lane_ops_per_byte_mac = 64 * SQ_INSTS_VALU / byte-MACs of the launch
  valu_issue_frac            = SQ_INSTS_VALU * 2 / (1024 SIMDs * GRBM_GUI_ACTIVE / 8)
                               (2 cycles per wave64 VALU op at full issue; GRBM_GUI_ACTIVE is
                               summed over the 8 XCDs)
  wave_cycles_split          = SQ_ACTIVE_INST_ANY / SQ_WAIT_ANY / SQ_WAIT_INST_ANY over SQ_WAVE_CYCLES
bench.py copies the entry of its config into the bench line (roofline.valu_profile).
"""
import collections
import csv
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"encode_mac": (r"gf_mac_bs<\d+, false", r"gf_mac<\d, false"),
           "decode_mac": (r"gf_mac_bs<\d+, true", r"gf_mac<\d, true")}
CONFIGS = {"k128r32s4096": (128, 32, 4096, 4096, 32),   # k, r, S, G, m
           "k32r8s1024": (32, 8, 1024, 4096, 8), "k128r32s1500": (128, 32, 1500, 8192, 32),
           "k1024dense": (1024, 1024, 65536, 1, 1024)}
# config 5: the dense encode and the dense decode (the inverse applied as a combine) are the same
# kernel -- the sliced-source encode MAC -- so one counter entry serves both keys
DENSE_KERNELS = {"encode_mac": (r"gf_mac_bs<16, false, true, false, true>",),
                 "decode_mac": (r"gf_mac_bs<16, false, true, false, true>",)}
HOW = "rocprofv3 --pmc, 2 SQ passes of bench.py --steps 2 --warmup 1 (tools/gpu_pmc.sh)"


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


def means(paths):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for p in paths:
        for row in csv.DictReader(open(p)):
            acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def main():
    cfg, *paths = sys.argv[1:]
    k, r, S, G, m = CONFIGS[cfg]
    table = means(paths)
    out_p = os.path.join(ROOT, "profiles", "pmc_valu.json")
    out = json.load(open(out_p)) if os.path.exists(out_p) else {}
    ent = {}
    for key, names in (DENSE_KERNELS if cfg == "k1024dense" else KERNELS).items():
        cs = next((v for n, v in table.items() if any(re.search(x, n) for x in names)), None)
        if cs is None:
            continue
        macs = G * k * (r if key == "encode_mac" else m) * S
        wc = cs["SQ_WAVE_CYCLES"]
        ent[key] = {
            "SQ_INSTS_VALU": cs["SQ_INSTS_VALU"],
            "SQ_INSTS_SALU": cs["SQ_INSTS_SALU"],
            "valu_lane_ops_per_byte_mac": round(64 * cs["SQ_INSTS_VALU"] / macs, 3),
            "valu_issue_frac": round(cs["SQ_INSTS_VALU"] * 2 / (1024 * cs["GRBM_GUI_ACTIVE"] / 8), 3),
            "wave_cycles_split": {"active": round(cs["SQ_ACTIVE_INST_ANY"] / wc, 3),
                                  "wait_waitcnt": round(cs["SQ_WAIT_ANY"] / wc, 3),
                                  "issue_stall": round(cs["SQ_WAIT_INST_ANY"] / wc, 3)},
        }
    ent["_commit"] = git_head()
    ent["_how"] = HOW
    out[cfg] = ent
    out["note"] = ("SQ PMC passes (tools/gpu_sq.sh, tools/pmc_valu.py); VALU issue slots = 1024 SIMDs x "
                   "(GRBM_GUI_ACTIVE/8) / 2 cycles per wave64 VALU op")
    json.dump(out, open(out_p, "w"), indent=1)
    print(json.dumps(ent, indent=1))


if __name__ == "__main__":
    main()
