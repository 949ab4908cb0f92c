"""Per-kernel mean duration and launches per inversion of the last dense inversion in a rocprofv3
kernel trace (tools/dense_trace.sh).  usage: python tools/dense_trace_summary.py <kernel_trace.csv>"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "dn_init" in r["Kernel_Name"]]
seq = rows[starts[-1]:]
end = next((i for i, r in enumerate(seq) if "dn_gather_inv" in r["Kernel_Name"]), len(seq) - 1)
seq = seq[:end + 1]
per = {}
for r in seq:
    n = r["Kernel_Name"].split("(")[0].split("::")[-1]
    per.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
span = (int(seq[-1]["End_Timestamp"]) - int(seq[0]["Start_Timestamp"])) / 1e3
print({"inversion_us": round(span, 1),
       **{n: {"launches": len(v), "mean_us": round(sum(v) / len(v), 2), "total_us": round(sum(v), 1)}
          for n, v in per.items()}})
