"""Summarise a tools/profile.sh run into profiles/ (committed evidence).

    python tools/summarize_prof.py gpurun_out/prof1 r03x [config]

writes profiles/<tag>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary) and
profiles/<tag>_pmc.json + profiles/pmc_latest.json: per nart kernel the HBM-side bytes per launch
(FETCH_SIZE x 2 -- on gfx950 FETCH_SIZE counts half the bytes of a wide read, MI355X_MICROARCH.md
HBM section -- plus WRITE_SIZE; both rocprofv3 KiB) and the SQ issue counters: VALU busy
(SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES), SIMD lane utilisation (SQ_THREAD_CYCLES_VALU /
(64 SQ_ACTIVE_INST_VALU)), waiting and issue-stall fractions.  `hbm_bytes_per_launch` is the
corrected sum for the path-tracing launch pair (k_primary + k_render_rq) that bench.py's roofline
times; bench.py reads it only while `hip_source_sha` matches the kernel sources.
"""
import csv
import json
import os
import shutil
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _key(name):
    return name.split("(")[0].replace("void ", "")


def waves_per_simd(vgpr, lds=None):
    """Resident waves per SIMD the kernel's registers allow: 512 VGPRs per SIMD lane in 8-register
    granules, at most 8 waves.  rocprofv3's VGPR_Count is in units of two registers on gfx950
    (k_render_rq's lean build: 84 for 163 VGPRs, kernel descriptor; k_primary: 60 for 113)."""
    try:
        v = 2 * int(vgpr)
    except (TypeError, ValueError):
        return None
    v = max(8, (v + 7) // 8 * 8)
    return min(8, 512 // v)


def _rows(src, kind):
    path = os.path.join(src, kind, "run_counter_collection.csv")
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


def main(src, tag, config="1920x1080x256"):
    prof = os.path.join(REPO, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(prof, tag + "_kernel_stats.csv"))
    per = {}
    # one dispatch per kernel name: the longest (the timed launch, not a probe / counter pass of
    # the same template); counters of the same dispatch id across passes
    for kind in ("fetch", "write", "sq"):
        for r in _rows(src, kind):
            if "nd::" not in r["Kernel_Name"]:
                continue
            k = _key(r["Kernel_Name"])
            d = per.setdefault(k, {"vgpr": r.get("VGPR_Count"), "sgpr": r.get("SGPR_Count"),
                                   "lds": r.get("LDS_Block_Size"), "scratch": r.get("Scratch_Size")})
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
            disp = d.setdefault(kind, {}).setdefault(r["Dispatch_Id"], {"dur": dur})
            disp[r["Counter_Name"]] = disp.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    sys.path.insert(0, REPO)
    from nart_amd.build import hip_source_sha
    out = {"config": config, "profile": tag, "hip_source_sha": hip_source_sha(), "kernels": {},
           "notes": "fetch_bytes_corrected = 2 x FETCH_SIZE (gfx950), write_bytes = WRITE_SIZE; per launch "
                    "(the longest dispatch of each kernel)"}
    for k, d in per.items():
        e = {"vgpr_count": d["vgpr"], "sgpr_count": d["sgpr"], "lds_bytes": d["lds"], "scratch_bytes": d["scratch"]}
        for kind, field in (("fetch", "FETCH_SIZE"), ("write", "WRITE_SIZE")):
            if kind in d:
                top = max(d[kind].values(), key=lambda v: v["dur"])
                e[kind + "_kib"] = top.get(field, 0.0)
                e["duration_ms_" + kind + "_pass"] = top["dur"]
        if "fetch_kib" in e:
            e["fetch_bytes_corrected"] = e["fetch_kib"] * 2048
        if "write_kib" in e:
            e["write_bytes"] = e["write_kib"] * 1024
        if "fetch_bytes_corrected" in e and "write_bytes" in e:
            e["hbm_bytes"] = e["fetch_bytes_corrected"] + e["write_bytes"]
            dur = e.get("duration_ms_fetch_pass") or 1e-9
            e["hbm_gbps"] = e["hbm_bytes"] / (dur * 1e-3) / 1e9
        if "sq" in d:
            top = max(d["sq"].values(), key=lambda v: v["dur"])
            wc = top.get("SQ_WAVE_CYCLES", 0.0) or 1.0
            av = top.get("SQ_ACTIVE_INST_VALU", 0.0)
            e["sq"] = {n: v for n, v in top.items() if n != "dur"}
            e["valu_busy"] = av / wc
            e["lane_utilization"] = top.get("SQ_THREAD_CYCLES_VALU", 0.0) / (64.0 * av) if av else None
            e["wait_any"] = top.get("SQ_WAIT_ANY", 0.0) / wc
            e["wait_inst_any"] = top.get("SQ_WAIT_INST_ANY", 0.0) / wc
            # issue rate: a wave issues at most one instruction per quad-cycle (the
            # SQ counters' unit), so issue_frac = (VALU issue quad-cycles + SALU instructions) / wave
            # quad-cycles is the fraction of the wave's issue slots it used.  simd_valu_frac: the
            # SIMD's VALU pipe, which takes a wave64 instruction every 2 cycles (two per quad-cycle,
            # MI355X_MICROARCH.md), summed over the resident waves
            wps = waves_per_simd(d["vgpr"], d.get("lds"))
            e["waves_per_simd"] = wps
            e["simd_valu_frac"] = min(1.0, av / wc * wps / 2.0) if wps else None
            if "SQ_INSTS_SALU" in top:
                e["issue_frac"] = (av + top["SQ_INSTS_SALU"]) / wc
        out["kernels"][k] = e

    def timed(name, base):
        # k_render_rq<EXT, COUNT, ENV> / k_primary<COUNT, ENV> / k_render_volume_sm<COUNT, WV>:
        # the COUNT == false build is the timed one
        if not name.startswith("nd::" + base + "<"):
            return False
        args = [a.strip() for a in name.split("<", 1)[1].split(">", 1)[0].split(",")]
        return "false" == (args[1] if base == "k_render_rq" else args[0])

    # several timed instantiations can appear (the cost probe, the volume ENV/WV forms): the
    # dominant one is the longest dispatch
    dur = lambda k: out["kernels"][k].get("duration_ms_fetch_pass", 0.0)  # noqa: E731
    rq = sorted([k for k in out["kernels"] if timed(k, "k_render_rq")], key=dur, reverse=True)
    rq = rq or sorted([k for k in out["kernels"] if timed(k, "k_render_volume_sm")], key=dur, reverse=True)
    pr = sorted([k for k in out["kernels"] if timed(k, "k_primary")], key=dur, reverse=True)
    if rq and "hbm_bytes" in out["kernels"][rq[0]]:
        r = out["kernels"][rq[0]]
        out["render_kernel"] = rq[0]
        out["hbm_bytes_per_launch"] = r["hbm_bytes"]
        if pr and "hbm_bytes" in out["kernels"][pr[0]]:
            out["hbm_bytes_per_launch"] += out["kernels"][pr[0]]["hbm_bytes"]
            out["render_kernel"] = pr[0] + " + " + rq[0]
        out["lane_utilization"] = r.get("lane_utilization")
        out["valu_busy"] = r.get("valu_busy")
        out["issue_frac"] = r.get("issue_frac")
        out["simd_valu_frac"] = r.get("simd_valu_frac")
        out["waves_per_simd"] = r.get("waves_per_simd")
    json.dump(out, open(os.path.join(prof, tag + "_pmc.json"), "w"), indent=1)
    # bench.py reads pmc_latest_<config>.json (and pmc_latest.json for the headline C3 config)
    json.dump(out, open(os.path.join(prof, "pmc_latest_%s.json" % config), "w"), indent=1)
    if config == "1920x1080x256":
        json.dump(out, open(os.path.join(prof, "pmc_latest.json"), "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}, indent=1))
    for k, e in out["kernels"].items():
        print("%-44s hbm %8.2f GB  %7.1f GB/s  lane_util %s  valu_busy %s" % (
            k[:44], e.get("hbm_bytes", 0) / 1e9, e.get("hbm_gbps", 0), e.get("lane_utilization"), e.get("valu_busy")))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(sys.argv[3:4]))
