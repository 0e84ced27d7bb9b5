#!/usr/bin/env python3
"""One line per bench JSON (driver or mixprobe logs): the box (PCI address),
the span objects' roofline fractions, shader clocks, per-phase workgroup
cycles and the box's dependent HBM load latency — the data DESIGN.md §6
(round 5) uses to tell where the App. C mix's box dependence comes from.
usage: python tools/mix_summary.py LOG [LOG ...]"""
import json
import sys


def main():
    for path in sys.argv[1:]:
        lines = [l for l in open(path) if l.startswith("{")]
        if not lines:
            continue
        d = json.loads(lines[-1])
        sysfs = d.get("clocks", {}).get("sysfs", {})
        row = {"log": path, "pci": sysfs.get("pci"), "udp64": d.get("roofline", {}).get("frac")}
        for k in ("imix", "malformed", "real_traffic"):
            o = d.get(k)
            if not o:
                continue
            c = o.get("clocks", {})
            sp = c.get("span", {})
            row[k] = {"frac": o.get("roofline", {}).get("frac"),
                      "clock_ghz": sp.get("shader_clock_ghz", {}).get("median"),
                      "wg_cycles": sp.get("workgroup_cycles", {}).get("mean"),
                      "phases": sp.get("phase_cycles"), "hbm_latency": c.get("hbm_latency")}
        print(json.dumps(row))


if __name__ == "__main__":
    main()
