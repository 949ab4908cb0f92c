"""Flat and inclusive profile from tools/sampler.c's sample file.

usage: python tools/sampler_report.py [/tmp/ntc_samples.txt] [top N] [obj,obj (resolve with addr2line)]
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
        if not out.strip():                      # stripped: the dynamic symbol table
            out = subprocess.run(["nm", "-C", "-D", "--defined-only", obj], capture_output=True, text=True).stdout
        tab = []
        for ln in out.splitlines():
            p = ln.split(" ", 2)
            if len(p) == 3 and p[1] in "tTwW":
                tab.append((int(p[0], 16), p[2]))
        tab.sort()
        _syms[obj] = ([a for a, _ in tab], [n for _, n in tab])
    return _syms[obj]


_a2l = {}
_segs = {}


def to_vaddr(obj, a):
    """File offset -> link-time address (lld places text at offset + 0x1000 and the like)."""
    if obj not in _segs:
        out = subprocess.run(["readelf", "-lW", obj], capture_output=True, text=True).stdout
        segs = []
        for ln in out.splitlines():
            f = ln.split()
            if f and f[0] == "LOAD":
                segs.append((int(f[1], 16), int(f[2], 16), int(f[4], 16)))
        _segs[obj] = segs
    for off, va, sz in _segs[obj]:
        if off <= a < off + sz:
            return a - off + va
    return a


def addr2line(obj, addrs):
    """Function names of file offsets in obj via addr2line (objects built with -g), cached."""
    todo = sorted({a for a in addrs if (obj, a) not in _a2l})
    if todo:
        out = subprocess.run(["addr2line", "-f", "-C", "-e", obj] + [hex(a) for a in todo],
                             capture_output=True, text=True).stdout.splitlines()
        for i, a in enumerate(todo):
            _a2l[(obj, a)] = out[2 * i] if 2 * i < len(out) else "?"


def resolve(maps, pc, dbg=()):
    for lo, hi, off, obj in maps:
        if lo <= pc < hi:
            a = to_vaddr(obj, pc - lo + off)
            if obj in dbg:
                addr2line(obj, [a])
                name = _a2l[(obj, a)]
            else:
                addrs, names = symbols(obj)
                i = bisect.bisect_right(addrs, a) - 1
                name = names[i] if i >= 0 else "?"
            return f"{obj.rsplit('/', 1)[-1]}:{name[:110]}"
    return "?"


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "/tmp/ntc_samples.txt"
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    maps, samples = load(path)
    dbg = set(sys.argv[3].split(",")) if len(sys.argv) > 3 else set()
    for lo, hi, off, obj in maps:                  # batch the addr2line calls
        if obj in dbg:
            addr2line(obj, [to_vaddr(obj, pc - lo + off) for s in samples for pc in s if lo <= pc < hi])
    self_c, incl_c = collections.Counter(), collections.Counter()
    for s in samples:
        names = [resolve(maps, pc, dbg) for pc in s if pc]
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
