"""Per-kernel launch durations of the TIMED steps from a rocprofv3 kernel trace, to set beside the
bench's own HIP-event numbers (bench.py roofline.kernel_ms / kernels_ms).  rocprofv3 --stats
averages every launch of the profiled process, warmup included (the first launches run while the
clocks ramp up); the bench times only the last `--steps` steps.  This takes, per kernel name, the
launches of the last `timed` of `total` steps and prints their time per step next to the
all-launch mean (a split batch launches its MAC twice per step).

usage: python tools/trace_timed.py <run_kernel_trace.csv> --timed 10 --total 50 --skip-last 10
       [--bench <bench log>]
"""
import argparse
import csv
import json
import re


def short(name):
    m = re.search(r"(\w+)(<[^()]*>)?\(", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--timed", type=int, required=True, help="timed steps (the trailing ones)")
    ap.add_argument("--total", type=int, required=True, help="steps in the run (warmup + timed + profiled)")
    ap.add_argument("--skip-last", type=int, default=0, help="trailing steps after the timed ones "
                    "(bench.py's profiled steps)")
    ap.add_argument("--bench", help="bench log whose JSON line to compare against")
    a = ap.parse_args()
    per = {}
    for r in csv.DictReader(open(a.trace)):
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        per.setdefault(short(r["Kernel_Name"]), []).append((int(r["Start_Timestamp"]), d))
    out = {}
    for n, v in per.items():
        v.sort()
        ds = [d for _, d in v]
        if len(ds) < a.total or not n.startswith(("gf_", "decode_plan", "encode_prep", "plan_rows",
                                                     "dense", "slot_pack", "wire_")):
            continue
        lps = len(ds) // a.total                       # launches per step
        end = len(ds) - a.skip_last * lps
        tail = ds[end - a.timed * lps:end]
        out[n] = {"launches": len(ds), "launches_per_step": lps,
                  "mean_all_launches_ms": round(sum(ds) / len(ds), 4),
                  "timed_ms_per_step": round(sum(tail) / a.timed, 4)}
    res = {"kernels": out, "timed_steps": a.timed, "total_steps": a.total}
    if a.bench:
        for line in open(a.bench):
            if line.startswith("{"):
                j = json.loads(line)
                res["bench_kernels_ms"] = j.get("kernels_ms")
                res["bench_roofline_kernel_ms"] = j.get("roofline", {}).get("kernel_ms")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
