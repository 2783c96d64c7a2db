"""Summarise a tools/profile.sh run into profiles/<round>_<tag>_*.

  kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (as produced)
  pmc.json           per kernel: launches, avg duration (trace), avg FETCH_SIZE /
                     WRITE_SIZE (KiB, as reported) and corrected HBM bytes per launch

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE reports half
the bytes of a wide (16 B/lane) coalesced read -> x2; WRITE_SIZE is exact for
16 B/lane stores.  Both counters are KiB.  All loads/stores of the kernels
summarised here are 16 B/lane (float4) except where noted in DESIGN.md.

A `valu` pass (tools/profile.sh STEPS=valu: SQ_INSTS_VALU, SQ_INSTS_MFMA,
SQ_VALU_MFMA_BUSY_CYCLES, GRBM_GUI_ACTIVE), when present, adds per kernel the
MFMA-busy fraction of the SIMDs' cycles, the VALU lane-instructions per
launch ((SQ_INSTS_VALU - SQ_INSTS_MFMA) x 64: wave-instructions of 64 lanes;
the counter counts MFMAs as VALU) and the effective clock (GRBM_GUI_ACTIVE / 8
XCDs / trace duration), and the whole step's VALU lane-instructions -- bench.py
prices the VALU-bound small configurations (L, z <= 128) with them.

usage: python tools/pmc_summary.py gpurun_out/prof/c4 profiles r01_c4
"""
import csv
import json
import os
import shutil
import sys


def short(name):
    name = name.split("(")[0]
    for pre in ("void ", "mpv::"):
        name = name.replace(pre, "")
    return name.split("<")[0].replace("_kernel", "")


def counters(path, counter):
    agg = {}
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        agg.setdefault(short(r["Kernel_Name"]), []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in agg.items()}


# in-library timing tag (bench.py roofline "kernel") -> kernel name prefix
TAGS = {"probit_fwd": "probit_fwd", "dR_gemm": ("dR16", "dR_gemm"), "bwd_elem": "bwd_elem",
        "noise_philox": "noise_philox"}


def tag_of(kernel):
    for t, pre in TAGS.items():
        if kernel.startswith(pre):
            return t
    return None


def main(src, dst, tag):
    os.makedirs(dst, exist_ok=True)
    stats = os.path.join(src, "trace", "trace_kernel_stats.csv")
    shutil.copy(stats, os.path.join(dst, f"{tag}_kernel_stats.csv"))
    dur = {}
    for r in csv.DictReader(open(stats)):
        k = short(r["Name"])
        if not r["Name"].startswith(("void mpv::", "mpv::")):
            continue
        dur[k] = (int(r["Calls"]), float(r["AverageNs"]) / 1e6)
    # per-launch durations in launch order: the timed steps are the last
    # `timed` launches (bench.py's --steps; the first ones are warm-up)
    timed = int(os.environ.get("TIMED_STEPS", "10"))
    per = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "trace_kernel_trace.csv"))):
        if not r["Kernel_Name"].startswith(("void mpv::", "mpv::")):
            continue
        per.setdefault(short(r["Kernel_Name"]), []).append(
            (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6))
    last = {k: [d for _, d in sorted(v)][-timed:] for k, v in per.items()}
    def opt(step, counter):
        f = os.path.join(src, step, f"{step}_counter_collection.csv")
        return counters(f, counter) if os.path.exists(f) else {}

    fetch = opt("fetch", "FETCH_SIZE")
    write = opt("write", "WRITE_SIZE")
    valu, mfma, grbm = opt("valu", "SQ_INSTS_VALU"), opt("valu", "SQ_INSTS_MFMA"), \
        opt("valu", "GRBM_GUI_ACTIVE")
    mbusy = opt("valu", "SQ_VALU_MFMA_BUSY_CYCLES")
    out = {"source": src, "note": "bytes per launch; fetch corrected x2 (gfx950 FETCH_SIZE "
                                  "reports half of 16B/lane reads)", "kernels": {}}
    for k in sorted(set(fetch) | set(write) | set(valu)):
        f_kib, w_kib = fetch.get(k), write.get(k)
        hbm = None
        if f_kib is not None and w_kib is not None:
            hbm = (2.0 * f_kib + w_kib) * 1024.0
        lt = last.get(k) or []
        out["kernels"][k] = {"launches_traced": dur.get(k, (None,))[0],
                             "avg_ms_trace": dur.get(k, (None, None))[1],
                             "avg_ms_trace_timed_steps": sum(lt) / len(lt) if lt else None,
                             "fetch_size_kib": f_kib, "write_size_kib": w_kib,
                             "hbm_bytes_per_launch": hbm}
        if k in valu:
            lanes = 64.0 * (valu[k] - mfma.get(k, 0.0))
            d = dur.get(k, (None, None))[1]
            out["kernels"][k].update(
                valu_lane_insts_per_launch=lanes, mfma_insts_per_launch=mfma.get(k),
                clock_ghz=(grbm[k] / 8.0 / (d * 1e6) if k in grbm and d else None))
            if k in mbusy and k in grbm:
                # MFMA-busy cycles per SIMD (1024 SIMDs) over the kernel's GPU cycles
                # (GRBM_GUI_ACTIVE summed over the 8 XCDs)
                out["kernels"][k]["mfma_busy_frac"] = mbusy[k] / 1024.0 / (grbm[k] / 8.0)
    # aliases under the timing tags bench.py reports (e.g. probit_fwd16 -> probit_fwd)
    for k in list(out["kernels"]):
        t = tag_of(k)
        if t is not None and t not in out["kernels"]:
            out["kernels"][t] = dict(out["kernels"][k], kernel=k)
    if valu:
        # the whole step: every mpv kernel's VALU lane-instructions per forward launch
        tot = {}
        f = os.path.join(src, "valu", "valu_counter_collection.csv")
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA") and \
                    r["Kernel_Name"].startswith(("void mpv::", "mpv::")):
                sgn = 1.0 if r["Counter_Name"] == "SQ_INSTS_VALU" else -1.0
                tot["all"] = tot.get("all", 0.0) + sgn * 64.0 * float(r["Counter_Value"])
        nfwd = sum(1 for r in csv.DictReader(open(f)) if r["Counter_Name"] == "SQ_INSTS_VALU"
                   and short(r["Kernel_Name"]).startswith("probit_fwd"))
        if nfwd:
            out["valu_lane_insts_per_step"] = tot.get("all", 0.0) / nfwd
    json.dump(out, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
