"""tools/pmc_summary.py turns rocprofv3 CSVs into the committed evidence bench.py reads: per-launch
HBM bytes (2 * FETCH_SIZE + WRITE_SIZE, KB), MFMA busy over 1024 SIMDs x GRBM_GUI_ACTIVE / 8, the
LDS-array busy fraction, and the lookup keys per precision mode (the F16 mode's kernels
k_mlp_fwd_h32 / k_wgrad_s, the f16x2 mode's k_wgrad_h).  Synthetic CSVs, CPU only."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(header)
        w.writerows(rows)


def _run(tmp, suffix):
    src, dst = os.path.join(tmp, "src"), os.path.join(tmp, "profiles")
    kernels = {"void nof::k_mlp_fwd_h32<true>(nof::FwdArgs)": 0.5e6, "void nof::k_wgrad_s(nof::WgradArgs)": 0.25e6,
               "void nof::k_wgrad_h(nof::WgradArgs)": 0.25e6}
    _write(os.path.join(src, "trace", "run_kernel_stats.csv"), ["Name", "Calls", "AverageNs"],
           [[k, 10, ns] for k, ns in kernels.items()])
    cyc = 2.0e9 * 0.5e-3  # 0.5 ms at 2.0 GHz
    counters = {"pmc_fetch": [("FETCH_SIZE", 1000.0)], "pmc_write": [("WRITE_SIZE", 500.0)],
                "pmc_clk": [("GRBM_GUI_ACTIVE", 8 * cyc), ("SQ_VALU_MFMA_BUSY_CYCLES", 0.25 * 1024 * cyc)],
                "pmc_lds": [("SQ_LDS_IDX_ACTIVE", 0.5 * 256 * cyc), ("SQ_LDS_BANK_CONFLICT", 0.0)]}
    for d, cs in counters.items():
        _write(os.path.join(src, d, "run_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
               [[k, c, v] for k in kernels for c, v in cs])
    env = dict(os.environ, NOF_PROFILES_DIR=dst)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), src, "t" + suffix, suffix],
                   env=env, check=True, capture_output=True)
    return (json.load(open(os.path.join(dst, f"t{suffix}_pmc.json"))),
            json.load(open(os.path.join(dst, "pmc_traffic.json"))), json.load(open(os.path.join(dst, "pmc_mfma.json"))))


def test_f16_mode_keys_and_fractions(tmp_path):
    per, traffic, busy = _run(str(tmp_path), "_f16")
    fwd = per["k_mlp_fwd_h32<true>"]
    assert fwd["hbm_bytes_per_launch"] == (2 * 1000.0 + 500.0) * 1024
    assert abs(fwd["mfma_busy"] - 0.25) < 1e-4 and abs(fwd["lds_busy"] - 0.5) < 1e-4
    assert abs(fwd["eff_clock_GHz"] - 2.0) < 1e-3  # 0.5 ms dispatch: clock reported
    assert per["k_wgrad_s"]["eff_clock_GHz"] is None  # < 0.3 ms: GRBM quotient not trusted
    assert set(traffic) >= {"mlp_fwd_f16", "wgrad_f16", "wgrad_f16x2"}
    assert busy["mlp_fwd_f16"] == fwd["mfma_busy"]


def test_f16x2_run_keeps_its_weight_gradient_key(tmp_path):
    per, traffic, _ = _run(str(tmp_path), "_f16x2")
    assert traffic["wgrad_f16x2"] == per["k_wgrad_h"]["hbm_bytes_per_launch"]
