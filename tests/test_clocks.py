"""CPU: nex_amd/clocks.py — the per-object `clocks` field of bench.py.
span_summary over synthetic nexg_probe_span_clock stamps (include/nexg.h
layout: six s_memtime stamps, two 100-MHz s_memrealtime stamps per
workgroup), and sysfs over a fake PCI device directory."""
import numpy as np

from nex_amd import clocks


def _stamps(n, ghz=2.0, phases=(100, 500, 200, 50, 150), seed=0):
    rng = np.random.default_rng(seed)
    s = np.zeros((n, 8), np.int64)
    t0 = 1_000_000 + rng.integers(0, 1000, n)
    s[:, 0] = t0
    for k, c in enumerate(phases):
        s[:, k + 1] = s[:, k] + c
    total = sum(phases)
    s[:, 6] = 5_000
    s[:, 7] = 5_000 + np.round(total / (ghz * 10.0)).astype(np.int64)  # 10 ns per real-time tick
    return s


def test_span_summary_clock_and_phases():
    s = _stamps(1000, ghz=2.0, phases=(200, 1000, 400, 100, 300))
    r = clocks.span_summary(s)
    assert r["workgroups"] == 1000 and r["valid"] == 1000
    assert abs(r["shader_clock_ghz"]["median"] - 2.0) < 0.01
    assert r["phase_cycles"] == {"start": 200.0, "subtile_loop": 1000.0, "fast_path": 400.0, "generic": 100.0,
                                 "stores": 300.0}
    assert abs(sum(r["phase_share"].values()) - 1.0) < 1e-3
    assert abs(r["workgroup_us"]["mean"] - 2000 / 2.0 / 1000) < 0.02


def test_span_summary_drops_inconsistent_workgroups():
    s = _stamps(10)
    s[3, 2] = s[3, 1] - 1  # time running backwards
    s[5, :] = 0  # never stamped
    r = clocks.span_summary(s)
    assert r["valid"] == 8
    assert clocks.span_summary(np.zeros((4, 8), np.int64)) == {"workgroups": 4, "valid": 0}


def test_sysfs_reads_current_levels(tmp_path):
    (tmp_path / "pp_dpm_sclk").write_text("0: 500Mhz\n1: 1800Mhz\n2: 2400Mhz *\n")
    (tmp_path / "pp_dpm_mclk").write_text("0: 900Mhz\n1: 2000Mhz *\n")
    (tmp_path / "pp_dpm_fclk").write_text("0: 1250Mhz *\n")
    (tmp_path / "current_compute_partition").write_text("SPX\n")
    (tmp_path / "current_memory_partition").write_text("NPS1\n")
    hw = tmp_path / "hwmon" / "hwmon3"
    hw.mkdir(parents=True)
    (hw / "power1_average").write_text("1250000000\n")
    (hw / "power1_cap").write_text("1400000000\n")
    (hw / "temp1_input").write_text("47000\n")
    (hw / "temp1_label").write_text("junction\n")
    (hw / "freq1_input").write_text("2400000000\n")
    r = clocks.sysfs(path=str(tmp_path))
    assert r["sclk"] == "2400Mhz" and r["mclk"] == "2000Mhz" and r["fclk"] == "1250Mhz"
    assert r["compute_partition"] == "SPX" and r["memory_partition"] == "NPS1"
    assert r["power_w"] == 1250.0 and r["power_cap_w"] == 1400.0
    assert r["temp_junction_c"] == 47.0 and r["hwmon_sclk_mhz"] == 2400
