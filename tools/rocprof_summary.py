"""Summarise a tools/profile.sh directory (rocprofv3 kernel trace + PMC passes) for one kernel
into the JSON bench.py reads (profiles/rocprof_<config>_<path>_<walk>.json).

    python tools/rocprof_summary.py <prof dir> <config> <n_rows> <spp> <path> <walk> <schedule> <out.json>
                                    [kernel substring, default "k_megakernel<false, false, false" (the timed instantiation)]

Per launch of the kernel (averaged over the profiled launches):
  * duration from the kernel trace (trace_kernel_stats.csv);
  * HBM bytes: read = 2 x FETCH_SIZE x 1024 (MI355X_MICROARCH.md §HBM: on gfx950 FETCH_SIZE
    reports half the bytes of wide coalesced reads), write = WRITE_SIZE x 1024;
  * issue and latency: SQ counters (quad-cycle units for SQ_WAVE_CYCLES / SQ_WAIT_ANY /
    SQ_ACTIVE_INST_*, MI355X_MICROARCH.md constants table), lane use per VALU instruction,
    the share of wave time spent waiting, and the VALU issue share of the SIMDs' capacity at
    one wave64 VALU instruction per 2 cycles per SIMD (MI355X_MICROARCH.md §Wave scheduling)
    at the measured effective clock (GRBM_GUI_ACTIVE / 8 XCDs / duration).
"""
import csv
import glob
import json
import os
import sys

N_SIMD = 256 * 4          # MI355X: 256 CUs x 4 SIMDs
VALU_CYCLES = 2           # wave64 VALU instruction issue cost per SIMD at throughput


def counters(d, kname):
    out = {}
    for f in glob.glob(f"{d}/*counter_collection.csv") + glob.glob(f"{d}/*/*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                out.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in out.items()}


def kernel_ms(d, kname):
    for f in glob.glob(f"{d}/trace/*kernel_stats.csv") + glob.glob(f"{d}/*kernel_stats.csv"):
        for r in csv.DictReader(open(f)):
            if kname in r["Name"]:
                return float(r["AverageNs"]) / 1e6, int(r["Calls"])
    raise SystemExit(f"no kernel '{kname}' in the trace of {d}")


def summarise(d, kname):
    ms, calls = kernel_ms(d, kname)
    c = counters(d, kname)
    t = ms / 1e3
    rd = 2 * c["FETCH_SIZE"] * 1024
    wr = c["WRITE_SIZE"] * 1024
    clock = c["GRBM_GUI_ACTIVE"] / 8 / t if "GRBM_GUI_ACTIVE" in c else None
    issue = {
        "valu_insts": c.get("SQ_INSTS_VALU"),
        "waves": c.get("SQ_WAVES"),
        "lanes_per_valu": round(c["SQ_THREAD_CYCLES_VALU"] / c["SQ_ACTIVE_INST_VALU"], 2),
        "wait_frac": round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4),
        "active_inst_frac": round(c["SQ_ACTIVE_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4),
        "clock_ghz": round(clock / 1e9, 3) if clock else None,
    }
    if clock:
        issue["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * VALU_CYCLES / (N_SIMD * t * clock), 4)
    return {
        "kernel": kname, "kernel_avg_ms_rocprof": round(ms, 3), "launches": calls,
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
        "hbm_read_gbs": round(rd / t / 1e9, 3), "hbm_write_gbs": round(wr / t / 1e9, 3),
        "l2_hit_rate": round(c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"]), 5) if "TCC_HIT_sum" in c else None,
        "issue": issue,
        "limiter": (f"divergent VALU issue + latency, not HBM: {issue['lanes_per_valu']} of 64 lanes per VALU "
                    f"instruction, {issue['wait_frac'] * 100:.0f}% of wave time waiting"
                    + (f", VALU issue {issue['valu_issue_frac'] * 100:.0f}% of the SIMDs' capacity at "
                       f"{issue['clock_ghz']} GHz" if clock else "")),
        "counters": c,
    }


if __name__ == "__main__":
    d, config, n_rows, spp, path, walk, schedule, out = sys.argv[1:9]
    kname = sys.argv[9] if len(sys.argv) > 9 else "k_megakernel<false, false, false"
    res = {"config": config, "n_rows": int(n_rows), "spp": int(spp), "path": path, "walk": walk,
           "schedule": schedule, "source": os.path.relpath(d, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}
    res.update(summarise(d, kname))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "counters"}))
