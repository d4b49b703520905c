#!/usr/bin/env python3
"""Static instruction mix of the loops of one kernel in a hipcc -S listing (compile-only, no GPU):
for every loop header the instructions between it and its last back edge, by class.

    python tools/asm_loops.py LISTING.s KERNEL_SUBSTRING
"""
import re
import sys

CLASSES = [("valu", r"\s+v_"), ("salu", r"\s+s_"), ("vmem", r"\s+(buffer|global|flat)_"), ("lds", r"\s+ds_"),
           ("waitcnt", r"\s+s_waitcnt")]


def main():
    lines = open(sys.argv[1]).read().split("\n")
    key = sys.argv[2]
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*:", l) and key in l.split(":")[0])
    end = start
    while "; -- End function" not in lines[end]:
        end += 1
    body = lines[start:end]
    print(body[0].split(":")[0], "lines", len(body))
    for h, l in enumerate(body):
        m = re.search(r"Loop Header: Depth=(\d+)", l)
        if not m:
            continue
        k = h
        while not body[k].startswith(".LBB"):
            k -= 1
        lbl = body[k].split(":")[0]
        backs = [i for i, x in enumerate(body) if i > k and re.search(r"s_c?branch\w*\s+" + re.escape(lbl) + r"\s*$", x)]
        e = max(backs) if backs else k
        seg = body[k:e + 1]
        c = {name: sum(1 for x in seg if re.match(pat, x)) for name, pat in CLASSES}
        print(f"{lbl:12s} depth {m.group(1)} lines {len(seg):5d} " + " ".join(f"{n} {c[n]:5d}" for n, _ in CLASSES))


if __name__ == "__main__":
    main()
