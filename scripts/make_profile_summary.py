#!/usr/bin/env python3
"""Turn a scripts/profile_gpu.sh output dir into the committed profile summary.

  scripts/make_profile_summary.py gpurun_out/prof_<tag> profiles/<round> M K N s

Writes <round>_kernel_stats.csv (rocprofv3 --stats copy), <round>_kernel_trace_tsg.csv
(our dispatches only) and <round>_pmc_summary.json:
  per-kernel counter totals / launch, HBM bytes corrected as MI355X_MICROARCH.md
  (HBM section) prescribes: FETCH_SIZE is KiB and reads 1/2 of a wide (16 B/lane)
  coalesced stream on gfx950 -> read bytes = 2 * FETCH_SIZE * 1024; WRITE_SIZE is
  exact for 16-B-per-lane stores -> write bytes = WRITE_SIZE * 1024.
Dispatches are grouped by (kernel, grid size): the workload's own launches
(the largest grid of a kernel) are reported under the kernel's name, smaller
grids of the same kernel (the host-pointer comp_func pipeline launches M
chunks, bench.py e2e_host_pointers) under "<kernel> [grid G]", so per-launch
figures never mix launch sizes.  The kernel-trace dispatches get the same
split (<round>_kernel_trace_by_grid.json: count and average duration per
grid), with the median and, leaving out the first STEADY_SKIP launches of
each grid (the clock ramp after idle), the steady-state average and median.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

STEADY_SKIP = 30  # launches on the ramping clock (~25 at configs[2], profiles/r02c_clock_ramp.txt)
src, dst = sys.argv[1], sys.argv[2]
M, K, N, s = (int(v) for v in sys.argv[3:7])
os.makedirs(os.path.dirname(dst) or ".", exist_ok=True)
stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
if stats:
    shutil.copy(stats[0], dst + "_kernel_stats.csv")
trace = glob.glob(os.path.join(src, "trace", "*kernel_trace.csv"))
if trace:
    rows = [r for r in csv.DictReader(open(trace[0])) if "tsg" in r["Kernel_Name"]]
    if rows:
        with open(dst + "_kernel_trace_tsg.csv", "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)
        by = collections.defaultdict(list)
        rows.sort(key=lambda r: int(r["Start_Timestamp"]))
        for r in rows:
            by[(r["Kernel_Name"].split("(")[0].replace("void ", "").strip(), int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) * int(r["Grid_Size_Z"]))].append(
                int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        def med(v):
            v = sorted(v)
            return (v[(len(v) - 1) // 2] + v[len(v) // 2]) / 2

        def entry(v):
            # launch order = trace order; the first STEADY_SKIP launches of a
            # grid run on the ramping clock after idle (DESIGN.md 5 "Clock
            # warm-up"): the steady-state figures leave them out
            steady = v[STEADY_SKIP:] if len(v) > 2 * STEADY_SKIP else v
            return {"dispatches": len(v), "avg_us": sum(v) / len(v) / 1e3, "median_us": med(v) / 1e3,
                    "steady_dispatches": len(steady), "steady_avg_us": sum(steady) / len(steady) / 1e3,
                    "steady_median_us": med(steady) / 1e3, "min_us": min(v) / 1e3, "max_us": max(v) / 1e3}

        json.dump({f"{k} [grid {g}]": entry(v) for (k, g), v in sorted(by.items())},
                  open(dst + "_kernel_trace_by_grid.json", "w"), indent=1)

# per (pass, kernel, counter): total and dispatches; a counter collected in
# several passes (GRBM_GUI_ACTIVE) is averaged over them, not summed
tot = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(float)))
disp = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(set)))
for f in sorted(glob.glob(os.path.join(src, "pmc*", "*counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "tsg" not in k or "probe" in k:
            continue
        kn = (k.split("(")[0].replace("void ", "").strip(), int(r["Grid_Size"]))
        tot[kn][r["Counter_Name"]][f] += float(r["Counter_Value"])
        disp[kn][r["Counter_Name"]][f].add(r["Dispatch_Id"])
# the workload's launches: the largest grid of each kernel
biggest = {}
for name, g in tot:
    biggest[name] = max(g, biggest.get(name, 0))
tot = {(name if g == biggest[name] else f"{name} [grid {g}]"): v for (name, g), v in tot.items()}
disp = {(name if g == biggest[name] else f"{name} [grid {g}]"): v for (name, g), v in disp.items()}
out = {"workload": f"{M}x{K}x{N}s{s}", "kernel": None, "kernels": {}, "per_launch_hbm_bytes": {}}
# the plan the library picks for this workload (host only; exactly K N / s
# nonzeros, as the bench's W): bench.py uses these counters only while its
# own call runs the same plan
try:
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "ternary-spgemm_amd"))
    import tspgemm
    out["plan"] = {k: list(v) if isinstance(v, tuple) else v for k, v in tspgemm.call_plan(K, N, K * N // s, M).items()}
except Exception as e:  # noqa: BLE001 -- the summary is still useful without it
    out["plan"] = None
    print("no plan:", e, file=sys.stderr)
for kn, v in tot.items():
    per = {c: sum(x / max(len(disp[kn][c][f]), 1) for f, x in passes.items()) / len(passes)
           for c, passes in v.items()}
    o = {"per_launch": per}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        o["hbm_read_bytes"] = 2 * per["FETCH_SIZE"] * 1024  # guide's gfx950 correction (see the calibration below)
        o["hbm_write_bytes"] = per["WRITE_SIZE"] * 1024
        o["hbm_bytes"] = o["hbm_read_bytes"] + o["hbm_write_bytes"]
    if "GRBM_GUI_ACTIVE" in per:
        o["gpu_cycles_per_xcd"] = per["GRBM_GUI_ACTIVE"] / 8
    # calibration of FETCH_SIZE on THIS kernel: the memory-side read requests
    # by size (TCC_EA0_RDREQ_{32,64,128}B) give the read bytes directly,
    # whatever issued them (LDS-DMA, code-prefetch loads, instruction-cache
    # misses); the ratio to FETCH_SIZE*1024 says whether the guide's x2 holds
    ea = [per.get(f"TCC_EA0_RDREQ_{w}B_sum") for w in (32, 64, 128)]
    if all(v is not None for v in ea):
        o["hbm_read_bytes_by_request_size"] = 32 * ea[0] + 64 * ea[1] + 128 * ea[2]
        if "FETCH_SIZE" in per and per["FETCH_SIZE"]:
            o["read_bytes_over_fetch_size_bytes"] = o["hbm_read_bytes_by_request_size"] / (per["FETCH_SIZE"] * 1024)
        if "WRITE_SIZE" in per:
            # round 6: the traffic bench.py reports -- read bytes
            # by request size + WRITE_SIZE; FETCH_SIZE x 2 stays beside it
            o["hbm_bytes_by_request_size"] = o["hbm_read_bytes_by_request_size"] + per["WRITE_SIZE"] * 1024
    if "SQC_ICACHE_BUSY_CYCLES" in per and "GRBM_GUI_ACTIVE" in per:
        # summed over the instruction caches (one SQC per CU pair: 128 on the chip);
        # GRBM_GUI_ACTIVE over the 8 XCDs
        o["sqc_icache_busy_frac"] = per["SQC_ICACHE_BUSY_CYCLES"] / 128 / (per["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_ACTIVE_INST_VALU" in per and "GRBM_GUI_ACTIVE" in per:
        # a wave64 v_pk_add_f32 occupies its SIMD 4 cycles, a VOP2 v_add_f32 2
        # (the 64-row image's adds) -- 1024 SIMDs
        cyc = 2 if "jit64" in kn else 4
        o["valu_busy_frac"] = cyc * per["SQ_ACTIVE_INST_VALU"] / 1024 / (per["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAIT_INST_ANY" in per and "SQ_WAVE_CYCLES" in per:
        o["wave_time_waiting_for_instructions"] = per["SQ_WAIT_INST_ANY"] / per["SQ_WAVE_CYCLES"]
    if "SQC_ICACHE_HITS" in per and "SQC_ICACHE_REQ" in per and per["SQC_ICACHE_REQ"]:
        o["sqc_icache_hit_rate"] = per["SQC_ICACHE_HITS"] / per["SQC_ICACHE_REQ"]
    if "SQ_LDS_IDX_ACTIVE" in per and "GRBM_GUI_ACTIVE" in per:
        o["lds_util"] = per["SQ_LDS_IDX_ACTIVE"] / (per["GRBM_GUI_ACTIVE"] / 8 * 256)
    out["kernels"][kn] = o
# the workload's TCSC kernel: the longest-running non-staging kernel per launch
# (bench.py's host-pointer leg launches a second kernel on row chunks)
main_kn = max((kn for kn, o in out["kernels"].items() if "transpose" not in kn and "[grid" not in kn and "hbm_bytes" in o),
              key=lambda kn: out["kernels"][kn].get("gpu_cycles_per_xcd", 0), default=None)
if main_kn:
    out["kernel"] = main_kn.split("::")[-1].split("<")[0]
    out["per_launch_hbm_bytes"][out["workload"]] = out["kernels"][main_kn]["hbm_bytes"]
json.dump(out, open(dst + "_pmc_summary.json", "w"), indent=1)
print(json.dumps(out, indent=1)[:3000])
