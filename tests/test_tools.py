"""CPU: the measurement tools' arithmetic (tools/pmc_traffic.py,
tools/defer_profile.py, tools/check_citations.py) on synthetic rocprofv3 output."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(REPO, "tools")

KR = "void st::dev::k_round<double, 4, 2, 2, 0, 0, 256, true>(double*, double const*)"
KR32 = "void st::dev::k_round<float, 4, 4, 2, 0, 0, 256, true>(float*, float const*)"
KM = "void st::dev::k_mfree<double, 4, 2, 2, true, 256, true>(double const*)"


def _write(path, fields, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=fields)
        w.writeheader()
        w.writerows(rows)


def test_pmc_traffic_corrections(tmp_path):
    n = 1024
    algo_round = 2.0 * n * n * 8
    # FETCH_SIZE counts half of the wide streaming reads on gfx950 (KiB)
    fetch_kib = algo_round / 2 / 2 / 1024
    write_kib = algo_round / 2 / 1024
    pmc = [{"Kernel_Name": KR, "Counter_Value": fetch_kib}] * 4 + [
        {"Kernel_Name": KR, "Counter_Value": 1.0},          # a gated no-op launch: dropped
        {"Kernel_Name": KR32, "Counter_Value": 123.0},      # other dtype: filtered
        {"Kernel_Name": KM, "Counter_Value": n * n * 8 / 2 / 1024}]
    wr = [{"Kernel_Name": KR, "Counter_Value": write_kib}] * 4 + [
        {"Kernel_Name": KR, "Counter_Value": 0.0},
        {"Kernel_Name": KR32, "Counter_Value": 1.0},
        {"Kernel_Name": KM, "Counter_Value": 0.0}]
    trace = [{"Kernel_Name": KR, "Start_Timestamp": 0, "End_Timestamp": 100000}] * 4
    _write(tmp_path / "f.csv", ["Kernel_Name", "Counter_Value"], pmc)
    _write(tmp_path / "w.csv", ["Kernel_Name", "Counter_Value"], wr)
    _write(tmp_path / "t.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], trace)
    out = tmp_path / "o.json"
    subprocess.run([sys.executable, os.path.join(TOOLS, "pmc_traffic.py"), "--workload", "x",
                    "--n", str(n), "--fetch", str(tmp_path / "f.csv"),
                    "--write", str(tmp_path / "w.csv"), "--trace", str(tmp_path / "t.csv"),
                    "--out", str(out)], check=True, capture_output=True)
    d = json.load(open(out))
    e = {x["kernel"]: x for x in d["entries"]}
    assert set(e) == {"k_round", "k_mfree"}
    assert abs(e["k_round"]["traffic_over_algorithmic"] - 1.0) < 1e-12
    assert e["k_round"]["launches_used"] == 4
    assert abs(e["k_round"]["trace_ms_avg"] - 0.1) < 1e-12
    assert abs(e["k_mfree"]["traffic_over_algorithmic"] - 1.0) < 1e-12
    assert d["fused_bytes_per_launch"] == e["k_round"]["hbm_bytes_per_launch"]


def _kflat(np_, store, old=False):
    # k_flat's template arguments as rocprofv3 prints them: NP is the 9th
    # (round 6 on), the 12th in earlier rounds' traces (BLK = 256 the 9th)
    if old:
        return ("void st::dev::k_flat<double, 2, 0, true, 8, false, true, 2, 256, 0, 1, "
                f"{np_}, 1, false, {1 if store else 0}>(double*, double const*)")
    return ("void st::dev::k_flat<double, 2, 0, true, 8, true, 2, 0, "
            f"{np_}, 1, {1 if store else 0}>(double*, double const*)")


def test_kflat_np_parsed_in_both_layouts():
    sys.path.insert(0, TOOLS)
    import defer_profile
    import pmc_traffic
    for old in (False, True):
        for np_ in (0, 3, 5):
            name = _kflat(np_, np_ == 5, old)
            assert pmc_traffic.flat_np(name) == np_
            assert defer_profile.np_of(name) == np_
    assert pmc_traffic.flat_np("void st::dev::k_flat<double, 2, 0, true, 1, true, 2, 0, -1, "
                               "2, -1, false, 2>(double*)") == -1


def test_defer_profile_cycle_and_launch_rows(tmp_path):
    """tools/defer_profile.py summary mode: per-NP averages of k_flat and of
    the k_parts launch that follows each, the cycle sum per round, and the
    per-launch CSV (the trimmed trace the committed summaries cite) holding
    exactly the deferred launches."""
    m, n = 6, 1024
    rows, t = [], 0
    for cyc in range(2):
        for np_ in range(m):
            dur = 2000 if np_ == m - 1 else 1000
            rows.append({"Kernel_Name": _kflat(np_, np_ == m - 1), "Start_Timestamp": t,
                         "End_Timestamp": t + dur})
            t += dur + 10
            rows.append({"Kernel_Name": "void st::dev::k_parts_seg<double, 16, 256>(double const*)",
                         "Start_Timestamp": t, "End_Timestamp": t + 100})
            t += 110
            rows.append({"Kernel_Name": "other_kernel", "Start_Timestamp": t,
                         "End_Timestamp": t + 5})
            t += 10
    _write(tmp_path / "trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    out, lc = tmp_path / "cycle.json", tmp_path / "cycle_launches.csv"
    subprocess.run([sys.executable, os.path.join(TOOLS, "defer_profile.py"), "--n", str(n),
                    "--trace", str(tmp_path / "trace.csv"), "--json", str(out),
                    "--launches", str(lc)], check=True, capture_output=True)
    d = json.load(open(out))
    assert d["trace"] == "cycle_launches.csv" and d["m"] == m
    assert d["k_flat"]["0"]["launches"] == 2 and d["k_flat"]["5"]["avg_ms"] == 0.002
    assert d["cycle_ms_per_round"] == round((5 * 0.0011 + 0.0021) / 6, 5)     # rounded to 10 ns
    launch_rows = list(csv.DictReader(open(lc)))
    assert len(launch_rows) == 2 * m * 2                      # k_flat + k_parts, no others
    assert {r["kernel"] for r in launch_rows} == {"k_flat", "k_parts"}
    assert launch_rows[0]["start_ns"] == "0" and launch_rows[0]["np"] == "0"
    # the committed launches CSV re-summarises to the same figures, with the
    # steady-state medians beside the averages
    out2 = tmp_path / "cycle2.json"
    subprocess.run([sys.executable, os.path.join(TOOLS, "defer_profile.py"), "--n", str(n),
                    "--trace", str(lc), "--json", str(out2)], check=True, capture_output=True)
    d2 = json.load(open(out2))
    assert d2["cycle_ms_per_round"] == d["cycle_ms_per_round"]
    assert d2["k_flat"]["5"]["median_ms"] == 0.002
    assert d2["cycle_ms_per_round_median"] == d["cycle_ms_per_round_median"]


def test_citation_checker_expands_ellipsis_names():
    """tools/check_citations.py reads `name.log, …_X_table.txt` as the full
    name the ellipsis abbreviates (its --rm pass had deleted two
    tables cited that way), and every tracked profile is cited."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import check_citations as cc
    assert cc.expand_ellipsis("r01_sweep_dir_blocks.log", "_blocks_table.txt") == \
        "r01_sweep_dir_blocks_table.txt"
    assert cc.expand_ellipsis("r03_defer_cycle_x.json", "_launches.csv") == \
        "r03_defer_cycle_x_launches.csv"
    pats = cc.cited_patterns()
    assert any(p.startswith("r06_") for p in pats)
    assert cc.uncited() == []


def test_defer_profile_bench_leg_passes(tmp_path):
    """tools/defer_profile.py --bench-leg: a kernel trace of bench.py's own
    deferred leg is cut into passes at k_recip (each pass's deferred_start
    after a fresh load), the warm-up cycles are dropped, each pass's timed
    k_flat + k_parts time per round is taken and the block's figure is the
    median pass - next to the leg's HIP-event passes.  The
    leg's trailing bitwise check (2m rounds) is not a pass."""
    m, cycles, warm = 6, 3, 2
    rows, t = [], 0

    def k(name, d):
        nonlocal t
        rows.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + d})
        t += d + 50

    pass_us = [1000, 1200, 1100]          # per-round k_flat time of each pass's timed cycles
    for p, fl in enumerate(pass_us + [5000]):
        k("void st::dev::k_generate<double>(double*)", 500)
        k("void st::dev::k_recip<double>(double const*, double*, unsigned int)", 10)
        ncyc = warm + cycles if p < 3 else 2
        for c in range(ncyc):
            for np_ in range(m):
                k(_kflat(np_, np_ == m - 1), 3000 if c < warm else fl)
                k("void st::dev::k_parts_seg<double, 16, 256>(double const*)", 100)
    _write(tmp_path / "trace.csv", ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    by = 7.0 / 6.0 * 8192 * 8192 * 8
    leg = {"deferred_writes": {"configs[1] hilbert8192_f64": {
        "stores_every": m, "cycles": cycles, "bytes_per_round": by,
        "ms_per_iteration_passes": [0.0010, 0.0011, 0.0012]}}}
    (tmp_path / "leg.out").write_text("noise\n@@LEG " + json.dumps(leg) + "\n")
    out = tmp_path / "bench_leg.json"
    subprocess.run([sys.executable, os.path.join(TOOLS, "defer_profile.py"), "--kind", "hilbert",
                    "--trace", str(tmp_path / "trace.csv"), "--bench-leg",
                    str(tmp_path / "leg.out"), "--json", str(out)], check=True,
                   capture_output=True)
    b = json.load(open(out))["blocks"]
    assert len(b) == 1 and b[0]["workload"] == "hilbert8192_f64"
    assert b[0]["rocprof_ms_per_round_passes"] == [0.0011, 0.0013, 0.0012]   # k_flat + k_parts
    assert b[0]["rocprof_ms_per_round"] == 0.0012
    assert b[0]["event_ms_per_round"] == 0.0011
    assert b[0]["events_over_rocprof"] == round(0.0011 / 0.0012, 4)
