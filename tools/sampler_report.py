"""Flat and inclusive profile from tools/sampler.c's sample file.

usage: python tools/sampler_report.py [/tmp/ntc_samples.txt] [top N]
Symbols come from `nm -C --defined-only` of each mapped object (text symbols, nearest below).
"""
import bisect
import collections
import subprocess
import sys


def load(path):
    maps, samples = [], []
    for line in open(path):
        if line.startswith("M "):
            f = line[2:].split()
            if len(f) >= 6 and "x" in f[1]:
                lo, hi = (int(x, 16) for x in f[0].split("-"))
                maps.append((lo, hi, int(f[2], 16), f[5]))
        elif line.startswith("S "):
            samples.append([int(x, 16) for x in line[2:].split()])
    return maps, samples


_syms = {}


def symbols(obj):
    if obj not in _syms:
        out = subprocess.run(["nm", "-C", "--defined-only", obj], capture_output=True, text=True).stdout
        tab = []
        for ln in out.splitlines():
            p = ln.split(" ", 2)
            if len(p) == 3 and p[1] in "tTwW":
                tab.append((int(p[0], 16), p[2]))
        tab.sort()
        _syms[obj] = ([a for a, _ in tab], [n for _, n in tab])
    return _syms[obj]


def resolve(maps, pc):
    for lo, hi, off, obj in maps:
        if lo <= pc < hi:
            # PIE / shared objects: file offset of the pc; nm addresses ~ file offsets for text
            a = pc - lo + off
            addrs, names = symbols(obj)
            i = bisect.bisect_right(addrs, a) - 1
            name = names[i] if i >= 0 else "?"
            return f"{obj.rsplit('/', 1)[-1]}:{name[:110]}"
    return "?"


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/ntc_samples.txt"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    maps, samples = load(path)
    self_c, incl_c = collections.Counter(), collections.Counter()
    for s in samples:
        names = [resolve(maps, pc) for pc in s if pc]
        if not names:
            continue
        self_c[names[0]] += 1
        for n in set(names):
            incl_c[n] += 1
    n = len(samples)
    print(f"{n} samples")
    print("-- self --")
    for k, v in self_c.most_common(top):
        print(f"{100 * v / n:6.2f}%  {k}")
    print("-- inclusive (up to 3 frame-pointer callers) --")
    for k, v in incl_c.most_common(top):
        print(f"{100 * v / n:6.2f}%  {k}")


if __name__ == "__main__":
    main()
