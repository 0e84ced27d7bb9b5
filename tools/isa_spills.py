#!/usr/bin/env python3
"""Where a kernel spills: compile nexg_parse.hip to gfx950 assembly and list,
for one kernel, its scratch spill / reload instructions and its barriers in
program order, with the sub-tile loop marked (the basic block range between a
loop header label and its backward branch that holds the loop's barriers).
usage: [NEXG_DEFS="-DX=1 ..."] [NEXG_SRC=file.hip] python tools/isa_spills.py [mangled-kernel-substring]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name = sys.argv[1] if len(sys.argv) > 1 else "k_parse_spanILi6ELi1ELj20480ELi6E"
out = "/tmp/nexg_parse_isa.s"
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950"] + os.environ.get("NEXG_DEFS", "").split() + [
                       "--cuda-device-only", "-S", "-o", out,
                       os.environ.get("NEXG_SRC", os.path.join(ROOT, "nex_amd/csrc/nexg_parse.hip"))],
                      stderr=subprocess.DEVNULL)
s = open(out).read()
start = [m.start() for m in re.finditer(r"^_ZN4nexg\w*:", s, re.M) if name in s[m.start():m.start() + 200]][0]
body = s[start:s.index(".Lfunc_end", start)].split("\n")
labels = {l.split(":")[0]: i for i, l in enumerate(body) if re.match(r"^\.LBB\w+:", l)}
loops = []  # backward branches: (header line, branch line)
for i, l in enumerate(body):
    m = re.match(r"\s+s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        loops.append((labels[m.group(2)], i))
bars = [i for i, l in enumerate(body) if "s_barrier" in l]
spills = [i for i, l in enumerate(body) if "scratch_" in l]
for a, b in loops:
    nb = sum(a <= x <= b for x in bars)
    ns = sum(a <= x <= b for x in spills)
    if nb:
        print(f"loop lines {a}-{b}: {nb} barriers, {ns} scratch ops")
print(f"{len(spills)} scratch ops in {len(body)} lines; barriers at {bars}")
print("scratch op lines:", spills)
