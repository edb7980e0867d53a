"""Compare two tools/isa_dump.sh outputs kernel by kernel: identical instruction streams, or the number of
inserted / deleted instruction lines (difflib over the instruction text with comments stripped) and the
register counts of both builds.

    python tools/isa_compare.py /tmp/isa_before /tmp/isa_after [--filter SUBSTRING] [--show N]
"""
from __future__ import annotations

import argparse
import difflib
import glob
import os
import re


def kernels(path: str) -> dict:
    out = {}
    for f in sorted(glob.glob(os.path.join(path, "*.s"))):
        text = open(f).read()
        meta = dict(re.findall(r"\.name:\s+(\S+)\n(?:.*\n){0,40}?\s+\.vgpr_count:\s+(\d+)", text))
        for m in re.finditer(r"^(_Z\S+):\s*(?:;.*)?$", text, re.M):
            name = m.group(1)
            end = text.find(".Lfunc_end", m.end())
            body = []
            for line in text[m.end():end].split("\n"):
                s = line.split(";")[0].strip()
                if not s or s.startswith(".") or s.endswith(":"):
                    continue
                body.append(re.sub(r"\.LBB\d+_\d+", "L", s))
            out[name] = (body, meta.get(name))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("before")
    ap.add_argument("after")
    ap.add_argument("--filter", default="")
    ap.add_argument("--show", type=int, default=0, help="print the first N differing lines per kernel")
    a = ap.parse_args()
    b, c = kernels(a.before), kernels(a.after)
    same = diff = 0
    for name in sorted(set(b) | set(c)):
        if a.filter not in name:
            continue
        if name not in b or name not in c:
            print(f"{'only in ' + ('after' if name in c else 'before'):14s} {name}")
            continue
        (x, vx), (y, vy) = b[name], c[name]
        if x == y:
            same += 1
            continue
        diff += 1
        sm = difflib.SequenceMatcher(None, x, y, autojunk=False)
        ins = sum(j2 - j1 for t, i1, i2, j1, j2 in sm.get_opcodes() if t in ("insert", "replace"))
        dele = sum(i2 - i1 for t, i1, i2, j1, j2 in sm.get_opcodes() if t in ("delete", "replace"))
        print(f"differs  +{ins:4d} -{dele:4d} lines  vgpr {vx}->{vy}  {name}")
        if a.show:
            shown = 0
            for t, i1, i2, j1, j2 in sm.get_opcodes():
                if t == "equal":
                    continue
                for l in x[i1:i2]:
                    print("    - " + l)
                for l in y[j1:j2]:
                    print("    + " + l)
                shown += 1
                if shown >= a.show:
                    break
    print(f"identical kernels: {same}, differing: {diff}")


if __name__ == "__main__":
    main()
