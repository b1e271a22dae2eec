#!/usr/bin/env python3
# SPDX-License-Identifier: GPL-2.0
"""Static instruction mix of the RX kernel instances' loops (diagnostic):
the gfx950 code object of a file holding the offload bundle (a .o or the
.so) is disassembled, and for each instance the largest loops (backward
branches) are counted by class: valu, salu, lane (v_readlane/v_writelane:
SGPR spills), lds, vmem, wait (s_waitcnt, s_nop).

    python tools/loopstat.py [file] [instance-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kres  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
INSTANCES = {"config2": "ILb0ELi0ELb0ELi64ELb0E", "imix": "ILb0ELi0ELb1ELi128ELb0E",
             "w128": "ILb0ELi0ELb0ELi128ELb0E", "echo": "ILb0ELi0ELb1ELi128ELb1E"}


def kind(l):
    l = l.strip()
    if not l or l[0] in "0<":
        return None
    op = l.split()[0]
    if op.startswith(("v_readlane", "v_writelane")):
        return "lane"
    if op.startswith("v_"):
        return "valu"
    if op.startswith(("s_waitcnt", "s_nop")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "scratch_")):
        return "vmem"
    return "other"


def loops(path, pats, top=3):
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(kres.code_objects(path)[0])
        f.flush()
        txt = subprocess.run([OBJDUMP, "-d", "--symbolize-operands", f.name],
                             capture_output=True, text=True, check=True).stdout
    lines = txt.split("\n")
    starts = [(i, m.group(1)) for i, l in enumerate(lines)
              for m in [re.match(r"^[0-9a-f]+ <(_Z\S+)>:", l)] if m]
    starts.append((len(lines), "END"))
    out = {}
    for (a, name), (b, _) in zip(starts, starts[1:]):
        tag = next((t for t, p in pats.items() if p in name), None)
        if not tag:
            continue
        body = lines[a:b]
        labels = {}
        for j, l in enumerate(body):
            m = re.match(r"^[0-9a-f]+ <(L\d+)>:", l)
            if m:
                labels[m.group(1)] = j
        lp = set()
        for j, l in enumerate(body):
            m = re.search(r"s_(c)?branch\S*\s+(L\d+)", l)
            if m and m.group(2) in labels and labels[m.group(2)] < j:
                lp.add((labels[m.group(2)], j))
        res = []
        for s, e in sorted(lp, key=lambda x: x[1] - x[0], reverse=True)[:top]:
            c = {}
            for l in body[s:e + 1]:
                k = kind(l)
                if k:
                    c[k] = c.get(k, 0) + 1
            res.append((s, e, c))
        tot = {}
        for l in body:
            k = kind(l)
            if k:
                tot[k] = tot.get(k, 0) + 1
        # the tile loop: the first loop (in program order) of more than
        # 500 lines, the outermost of those starting there
        big = sorted((x for x in lp if x[1] - x[0] > 500), key=lambda x: (x[0], x[0] - x[1]))
        tl = None
        if big:
            s, e = big[0]
            c = {}
            for l in body[s:e + 1]:
                k = kind(l)
                if k:
                    c[k] = c.get(k, 0) + 1
            tl = (s, e, c)
        out[tag] = {"total": tot, "loops": res, "tile_loop": tl}
    return out


if __name__ == "__main__":
    path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(kres.LIB), "xdp_rx.o")
    want = sys.argv[2:] or list(INSTANCES)
    r = loops(path, {k: INSTANCES[k] for k in want}, top=6)
    for tag, v in r.items():
        print(tag, "total", v["total"])
        print("   tile loop", v["tile_loop"])
        for s, e, c in v["loops"]:
            print(f"   loop {s}-{e}: {c}")
