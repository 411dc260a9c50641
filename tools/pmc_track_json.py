#!/usr/bin/env python3
"""profiles/pmc_tracker.json from a tools/pmc_track.sh run: the batched
tracker's (k_track7 for the default configuration, else k_track_frames_g) instruction mix per Newton iteration and its VALU
issue ceiling (the tracker has no HBM roofline; its bound is
instruction issue and gather latency).

Counters are per dispatch (rocprofv3 --pmc, kernel-trace only); the run's
counted replay (count.json: klt_hip_set_track_count) gives the Newton
iterations -- the 2x2 systems formed, trackFeatures.c:418-455 -- of the same
launches.  GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md), so
a dispatch lasts GRBM/8 cycles on 256 CUs x 4 SIMDs; a wave64 VALU instruction
occupies its SIMD 2 cycles (SIMD-32), which sets the ceiling
  iterations/s <= 1024 SIMDs * clock / (2 * VALU instructions per iteration).
usage: python tools/pmc_track_json.py gpurun_out/<tag> [out.json]
"""
import csv
import glob
import json
import sys

root = sys.argv[1]
out = sys.argv[2] if len(sys.argv) > 2 else "profiles/pmc_tracker.json"
per, names = {}, set()
for path in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if "k_track_frames" not in r["Kernel_Name"] and "k_track7" not in r["Kernel_Name"]:
            continue
        names.add(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0])
        per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in per.items()}
cnt = json.load(open(f"{root}/count.json"))
launches = cnt["frames"] // cnt["chunk"]  # the counted replay: frames / chunk launches
it = cnt["newton_iterations"] / launches  # per launch
cyc = avg["GRBM_GUI_ACTIVE"] / 8.0  # per-XCD cycles of one dispatch
simd_cycles = cyc * 256 * 4
valu = avg["SQ_INSTS_VALU"]
clock_hz = 2.1e9  # sustained shader clock under load (tools: GRBM / wall); nominal 2.4 GHz
res = {
    "kernel": " / ".join(sorted(names)) + " (one wave per feature)",
    "workload": f"{cnt['resolution']}, {cnt['features']} features, {cnt['chunk']}-frame launches, feature table",
    "source": "rocprofv3 --pmc SQ_* / GRBM_GUI_ACTIVE (tools/pmc_track.sh), per dispatch; iterations from the counted replay",
    "newton_iterations_per_launch": it,
    "per_iteration": {k.replace("SQ_INSTS_", "").lower(): avg[k] / it
                      for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH",
                                "SQ_INSTS_SMEM") if k in avg},
    "valu_issue_busy": 2.0 * valu / simd_cycles,
    "wave_time_split": {"active_inst": avg["SQ_ACTIVE_INST_ANY"] / avg["SQ_WAVE_CYCLES"],
                        "wait_memory_or_lds": avg["SQ_WAIT_ANY"] / avg["SQ_WAVE_CYCLES"],
                        "wait_issue": avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]},
    "issue_ceiling_iterations_per_s": 1024 * clock_hz / (2.0 * valu / it),
    "clock_hz_assumed": clock_hz,
    "measured_iterations_per_s": it / (cyc / clock_hz),
}
res["measured_vs_ceiling"] = res["measured_iterations_per_s"] / res["issue_ceiling_iterations_per_s"]
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
