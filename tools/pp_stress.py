"""Randomised per-packet parity sweep (one-off stress, not a test): tools/pp_driver.c through
libntc.so (batched / async / immediate) against the oracle's or_pp_bench on random shapes --
flows, items, payload size, window, repair rate, loss -- packets and deliveries compared by hash.
usage: python tools/pp_stress.py [n_cases] [seed]"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import oracle as O  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    rng = np.random.default_rng(int(sys.argv[2]) if len(sys.argv) > 2 else 5)
    lib = O.lib()
    drv = os.path.join(ROOT, "tests", "_build", "pp_driver")
    bad = 0
    for case in range(n):
        flows = int(rng.integers(1, 48))
        items = int(rng.integers(5, 160))
        size = int(rng.choice([1, 7, 64, 300, 1024, 1500, 4000]))
        window = int(rng.integers(1, 64))
        rate = int(rng.integers(1, 9))
        loss = int(rng.integers(0, 45))
        seed = int(rng.integers(1, 1 << 30))
        mode = str(rng.choice(["batched", "async", "immediate"] if case % 5 == 0 else ["batched", "async"]))
        args = [str(x) for x in (flows, items, size, window, rate, loss, seed)]
        r = subprocess.run([drv, mode] + args, capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            print(json.dumps({"case": case, "mode": mode, "args": args, "error": r.stderr[-300:]}), flush=True)
            bad += 1
            continue
        g = json.loads(r.stdout.strip().splitlines()[-1])
        secs, cnt, hs = (C.c_double * 2)(), (C.c_uint64 * 4)(), (C.c_uint64 * 2)()
        rc = lib.or_pp_bench(flows, items, size, window, rate, loss, C.c_uint64(seed), secs, cnt, hs)
        ok = (rc == 0 and [g["packets"], g["received"], g["deliveries"], g["repairs"]] == list(cnt)
              and g["packets_hash"] == f"{hs[0]:016x}" and g["deliveries_hash"] == f"{hs[1]:016x}")
        bad += not ok
        print(json.dumps({"case": case, "mode": mode, "args": args, "ok": ok}), flush=True)
    print(json.dumps({"cases": n, "failed": bad}), flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
