"""Which clocks a measurement ran at (bench.py's per-object `clocks` field).

Two sources, both read without executing anything:

* the kernel itself: `Engine.probe_span_clock` runs the span kernel once in a
  stamped instance (include/nexg.h nexg_probe_span_clock); `span_summary`
  turns its per-workgroup stamps into the shader clock the workgroups ran at
  (shader-clock ticks / 100-MHz real time, MI355X_MICROARCH.md 'DVFS
  give-back' item 6) and the cycles of each phase of a workgroup's life;
* sysfs: the DPM levels the driver reports current for the GPU's PCI device
  (`pp_dpm_sclk`, `pp_dpm_mclk`, `pp_dpm_fclk`), board power and the edge /
  HBM temperatures from hwmon. The guide warns that `pp_dpm_sclk` is not the
  in-kernel clock; it is recorded beside it to tell boxes apart.

Nothing here imports torch at module level.
"""
import glob
import os

#: phases between the stamps of include/nexg.h nexg_probe_span_clock
PHASES = ("start", "subtile_loop", "fast_path", "generic", "stores")


def span_summary(stamps):
    """Per-launch summary of nexg_probe_span_clock stamps ((workgroups, 8)
    int64 numpy array). Workgroups whose stamps are missing or inconsistent
    (a zero, or time running backwards) are dropped."""
    import numpy as np
    s = np.asarray(stamps, dtype=np.int64)
    t, rt = s[:, :6], s[:, 6:8]
    d = np.diff(t, axis=1)
    cyc = t[:, 5] - t[:, 0]
    ticks = rt[:, 1] - rt[:, 0]
    ok = (cyc > 0) & (ticks > 0) & (d >= 0).all(axis=1) & (t > 0).all(axis=1)
    if not ok.any():
        return {"workgroups": int(len(s)), "valid": 0}
    d, cyc, ticks = d[ok], cyc[ok], ticks[ok]
    ghz = cyc / (ticks * 10.0)  # real time ticks at 100 MHz = 10 ns
    mean_cyc = float(cyc.mean())
    return {
        "workgroups": int(len(s)), "valid": int(ok.sum()),
        "shader_clock_ghz": {"median": round(float(np.median(ghz)), 4), "p10": round(float(np.percentile(ghz, 10)), 4),
                             "p90": round(float(np.percentile(ghz, 90)), 4)},
        "workgroup_us": {"mean": round(float(ticks.mean()) / 100.0, 3),
                         "p90": round(float(np.percentile(ticks, 90)) / 100.0, 3)},
        "workgroup_cycles": {"mean": round(mean_cyc, 1), "p90": round(float(np.percentile(cyc, 90)), 1)},
        "phase_cycles": {k: round(float(v), 1) for k, v in zip(PHASES, d.mean(axis=0))},
        "phase_share": {k: round(float(v) / mean_cyc, 4) for k, v in zip(PHASES, d.mean(axis=0))}}


def _read(path):
    try:
        with open(path) as f:
            return f.read()
    except OSError:
        return None


def _current_level(text):
    """The '*'-marked line of a pp_dpm_* file ('1: 2100Mhz *' -> '2100Mhz')."""
    if not text:
        return None
    for line in text.splitlines():
        if line.rstrip().endswith("*"):
            parts = line.split(":", 1)
            return (parts[1] if len(parts) > 1 else parts[0]).replace("*", "").strip()
    return None


def pci_path(device_index=0):
    """sysfs directory of the torch device's PCI function, or None."""
    try:
        import torch
        p = torch.cuda.get_device_properties(device_index)
        dom, bus, dev = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        if bus is None:
            return None
        path = "/sys/bus/pci/devices/%04x:%02x:%02x.0" % (dom or 0, bus, dev or 0)
        return path if os.path.isdir(path) else None
    except Exception:
        return None


def sysfs(device_index=0, path=None):
    """Current DPM levels, power and temperatures of the device (file reads only)."""
    path = path or pci_path(device_index)
    if path is None:
        return {"pci": None}
    r = {"pci": os.path.basename(path)}
    for k in ("sclk", "mclk", "fclk", "socclk"):
        lvl = _current_level(_read(os.path.join(path, f"pp_dpm_{k}")))
        if lvl is not None:
            r[k] = lvl
    for k in ("current_compute_partition", "current_memory_partition"):  # SPX / NPS1 etc.
        v = _read(os.path.join(path, k))
        if v is not None:
            r[k.replace("current_", "")] = v.strip()
    for hw in sorted(glob.glob(os.path.join(path, "hwmon", "hwmon*"))):
        for name, key, scale in (("power1_average", "power_w", 1e-6), ("power1_input", "power_w", 1e-6),
                                 ("power1_cap", "power_cap_w", 1e-6)):
            v = _read(os.path.join(hw, name))
            if v is not None and key not in r:
                try:
                    r[key] = round(int(v.strip()) * scale, 1)
                except ValueError:
                    pass
        for tin in sorted(glob.glob(os.path.join(hw, "temp*_input"))):
            label = (_read(tin.replace("_input", "_label")) or os.path.basename(tin)).strip()
            v = _read(tin)
            try:
                r[f"temp_{label}_c"] = round(int(v.strip()) / 1000.0, 1)
            except (AttributeError, ValueError):
                pass
        v = _read(os.path.join(hw, "freq1_input"))  # sclk in Hz where the driver exposes it
        if v is not None:
            try:
                r["hwmon_sclk_mhz"] = round(int(v.strip()) / 1e6)
            except ValueError:
                pass
    return r


def _mhz_range(counts):
    """{'2100Mhz': n, ...} sample counts -> [min, median, max] MHz (ints)."""
    vals = []
    for k, n in counts.items():
        try:
            vals += [int(str(k).lower().replace("mhz", "").strip())] * int(n)
        except ValueError:
            continue
    if not vals:
        return None
    vals.sort()
    return [vals[0], vals[len(vals) // 2], vals[-1]]


def compact(clk):
    """The short form of a `clocks` object that bench.py's stdout line carries
    (the full form goes to stderr): sysfs sclk / mclk as [min, median, max]
    MHz over the samples, board power [min, max] W; the span kernel's
    median shader clock and its phase shares in PHASES order; the dependent
    HBM load latency [idle, loaded] ns. Keys are documented in DESIGN.md §6."""
    r = {}
    s = clk.get("sysfs") or {}
    for k in ("sclk", "mclk"):
        if isinstance(s.get(k), dict):
            v = _mhz_range(s[k])
            if v is not None:
                r[f"{k}_mhz"] = v
    if isinstance(s.get("power_w"), dict):
        r["power_w"] = [s["power_w"].get("min"), s["power_w"].get("max")]
    sp = clk.get("span")
    if isinstance(sp, dict) and "shader_clock_ghz" in sp:
        r["span_ghz"] = sp["shader_clock_ghz"]["median"]
        r["span_share"] = [round(sp["phase_share"][k], 3) for k in PHASES]
    elif isinstance(sp, dict) and "error" in sp:
        r["span_error"] = str(sp["error"])[:80]
    lat = clk.get("hbm_latency")
    if isinstance(lat, dict):
        r["lat_ns"] = [lat.get("idle_ns"), lat.get("loaded_ns")]
    return r


class Sampler:
    """Samples `sysfs(device_index)` every `period` seconds on a thread while
    a measurement runs (file reads only; the GPU work is not touched), and
    summarises what it saw: each DPM field's levels with their sample counts,
    the power range and the last temperatures."""

    def __init__(self, device_index=0, period=0.02):
        self.device_index, self.period = device_index, period
        self.samples = []
        self._stop = None
        self._thread = None

    def __enter__(self):
        import threading
        path = pci_path(self.device_index)
        if path is None:
            return self
        self._stop = threading.Event()

        def run():
            while not self._stop.is_set():
                self.samples.append(sysfs(path=path))
                self._stop.wait(self.period)
        self._thread = threading.Thread(target=run, daemon=True)
        self._thread.start()
        return self

    def __exit__(self, *exc):
        if self._thread is not None:
            self._stop.set()
            self._thread.join(timeout=5)
        return False

    def summary(self):
        if not self.samples:
            return {"pci": None, "samples": 0}
        r = {"pci": self.samples[0].get("pci"), "samples": len(self.samples)}
        for k in ("sclk", "mclk", "fclk", "socclk", "hwmon_sclk_mhz"):
            seen = {}
            for s in self.samples:
                if k in s:
                    seen[str(s[k])] = seen.get(str(s[k]), 0) + 1
            if seen:
                r[k] = seen
        pw = [s["power_w"] for s in self.samples if "power_w" in s]
        if pw:
            r["power_w"] = {"min": min(pw), "max": max(pw)}
        last = self.samples[-1]
        r.update({k: v for k, v in last.items()
                  if k.startswith("temp_") or k in ("power_cap_w", "compute_partition", "memory_partition")})
        return r
