#!/usr/bin/env python3
"""Summarise tools/gpu_profile.sh output: generation-0 transport dispatches
(the transport dispatch that follows each c2d_source_kernel dispatch), their
durations, and the PMC counters of the timed (last) generation-0 dispatch.

FETCH_SIZE / WRITE_SIZE are in KiB summed over the XCDs.  On gfx950
FETCH_SIZE counts wide streaming reads at half their bytes
(MI355X_MICROARCH.md §HBM); both raw and x2-corrected fetch bytes are
reported.  hbm_bytes_per_step = (2*FETCH + WRITE) / packet-steps of that
dispatch (packet-steps from the bench JSON of the same run)."""
import csv
import glob
import json
import os
import sys
from statistics import mean

CLOCK = 2.4e9          # MI355X engine clock
N_SIMD = 1024          # 256 CUs x 4 SIMDs


def find(d, suffix):
    f = glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True)
    return f[0] if f else None


def dispatches(kt_csv):
    rows = list(csv.DictReader(open(kt_csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    return rows


def gen0_ids(rows):
    ids, after_src = [], False
    for r in rows:
        k = r["Kernel_Name"]
        if "c2d_source_kernel" in k:
            after_src = True
        elif ("c2d_transport_kernel" in k or "c2d_bundle_kernel" in k) and after_src:
            ids.append(r["Dispatch_Id"])
            after_src = False
    return ids


def counters(d, did):
    f = find(d, "counter_collection.csv")
    out = {}
    if not f:
        return out
    for r in csv.DictReader(open(f)):
        if r["Dispatch_Id"] == did:
            out[r["Counter_Name"]] = out.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def main(root):
    res = {}
    kt = find(os.path.join(root, "kt"), "kernel_trace.csv")
    if kt:
        rows = dispatches(kt)
        by = {r["Dispatch_Id"]: r for r in rows}
        g0 = gen0_ids(rows)
        dur = [(int(by[i]["End_Timestamp"]) - int(by[i]["Start_Timestamp"])) / 1e6 for i in g0]
        print("generation-0 transport dispatches: %d; ms: %s" % (len(dur), ", ".join("%.3f" % d for d in dur)))
        k = 5
        try:
            k = int(json.load(open(os.path.join(root, "bench_kt.json")))["steps"])
        except Exception:
            pass
        if len(dur) >= k:
            print("mean of the last %d (bench timed steps): %.3f ms" % (k, mean(dur[-k:])))
            res["gen0_ms_timed_mean"] = mean(dur[-k:])
        names = {}
        for r in rows:
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            names.setdefault(n, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        for n, v in sorted(names.items(), key=lambda kv: -sum(kv[1])):
            print("  %-60s n=%4d total=%9.3f ms mean=%8.3f ms" % (n[:60], len(v), sum(v), mean(v)))
        r0 = by[g0[-1]] if g0 else rows[0]
        print("transport launch: grid=%s wg=%s LDS=%s (rocprofv3 fields; its VGPR_Count=%s is a "
              "granule field, the code object's counts follow)" % (
            r0.get("Grid_Size_X"), r0.get("Workgroup_Size_X"), r0.get("LDS_Block_Size"),
            r0.get("VGPR_Count")))
        try:
            sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
            import code_object
            print(code_object.describe(code_object.Path(os.environ.get(
                "C2D_LIBRARY") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                               "compton2d_amd", "libcompton2d.so")), "bundle_kernel"))
        except Exception as e:  # the summary stays useful without the code object
            print("code object registers unavailable: %s" % e)
    for sub in ("fetch", "write", "sq"):
        d = os.path.join(root, sub)
        f = find(d, "kernel_trace.csv")
        if not f:
            continue
        rows = dispatches(f)
        g0 = gen0_ids(rows)
        if not g0:
            continue
        # the timed generation-0 dispatches of that pass (its bench JSON's K)
        bj = os.path.join(root, "bench_%s.json" % sub)
        steps = paths = None
        k = 1
        if os.path.exists(bj):
            try:
                b = json.load(open(bj))
                k = int(b["steps"])
                steps = b["roofline"]["steps_per_launch_avg"] * k
                paths = b["roofline"].get("paths_per_launch_avg")
                paths = paths * k if paths else None
            except Exception:
                steps = paths = None
        ids = g0[-k:]
        by = {r["Dispatch_Id"]: r for r in rows}
        ms = sum((int(by[i]["End_Timestamp"]) - int(by[i]["Start_Timestamp"])) / 1e6 for i in ids)
        c = {}
        for i in ids:
            for kk, v in counters(d, i).items():
                c[kk] = c.get(kk, 0.0) + v
        print("[%s] %d timed dispatches %s: %.3f ms, packet-steps %s, path-steps %s, counters %s"
              % (sub, len(ids), ",".join(ids), ms, steps, paths, c))
        res[sub] = {"ms": ms, "steps": steps, "paths": paths, "launches": len(ids), "counters": c}
    if "fetch" in res and "write" in res and res["fetch"]["steps"] and res["write"]["steps"]:
        fk = res["fetch"]["counters"].get("FETCH_SIZE", 0.0)
        wk = res["write"]["counters"].get("WRITE_SIZE", 0.0)
        fb = fk * 1024.0 * 2.0 / res["fetch"]["steps"]
        wb = wk * 1024.0 / res["write"]["steps"]
        res["hbm_bytes_per_step"] = fb + wb
        print("HBM bytes per packet-step: fetch(x2) %.2f + write %.2f = %.2f" % (fb, wb, fb + wb))
        if res["fetch"]["paths"] and res["write"]["paths"]:
            fpb = fk * 1024.0 * 2.0 / res["fetch"]["paths"]
            wpb = wk * 1024.0 / res["write"]["paths"]
            res["hbm_bytes_per_path"] = fpb + wpb
            res["hbm_gbs_measured"] = (fk * 1024.0 * 2.0 / (res["fetch"]["ms"] * 1e-3) +
                                       wk * 1024.0 / (res["write"]["ms"] * 1e-3)) / 1e9
            print("HBM bytes per lane path-step: fetch(x2) %.2f + write %.2f = %.2f; measured %.0f GB/s"
                  % (fpb, wpb, fpb + wpb, res["hbm_gbs_measured"]))
    # the FP kernel (c2d_fp_kernel<W>, or c2d_fp_fast_kernel<BS> in the fast
    # mode): last dispatch of each pass
    fp = {}
    for sub in ("fetch", "write", "sq"):
        f = find(os.path.join(root, sub), "kernel_trace.csv")
        if not f:
            continue
        rows = [r for r in dispatches(f)
                if "c2d_fp_kernel" in r["Kernel_Name"] or "c2d_fp_fast_kernel" in r["Kernel_Name"]]
        if not rows:
            continue
        r = rows[-1]
        ms = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        c = counters(os.path.join(root, sub), r["Dispatch_Id"])
        fp[sub] = {"ms": ms, "counters": c, "grid": r.get("Grid_Size_X"),
                   "workgroup": r.get("Workgroup_Size_X"), "vgpr": r.get("VGPR_Count"),
                   "lds": r.get("LDS_Block_Size")}
        print("[fp %s] dispatch %s: %.3f ms grid %s wg %s counters %s" % (
            sub, r["Dispatch_Id"], ms, r.get("Grid_Size_X"), r.get("Workgroup_Size_X"), c))
    if "sq" in fp:
        c, ms = fp["sq"]["counters"], fp["sq"]["ms"]
        w = c.get("SQ_WAVE_CYCLES", 0.0)
        waves = int(fp["sq"]["grid"] or 0) // 64
        # a wave64 VALU instruction issues over 4 cycles on a 16-lane SIMD:
        # fraction of the chip's VALU issue slots used during the kernel
        res["fp_valu_issue_frac"] = c.get("SQ_INSTS_VALU", 0.0) * 4.0 / (ms * 1e-3 * CLOCK * N_SIMD)
        res["fp_wait_frac"] = c.get("SQ_WAIT_ANY", 0.0) / w if w else None
        res["fp_waves"] = waves
        res["fp_simd_occupancy"] = waves / float(N_SIMD)
        print("FP kernel: %.3f ms, %d waves (%.2f per SIMD), VALU issue %.3f of the chip, wait_any %.3f" % (
            ms, waves, waves / float(N_SIMD), res["fp_valu_issue_frac"], res["fp_wait_frac"] or 0))
    res["fp"] = fp
    if "sq" in res:
        c = res["sq"]["counters"]
        w = c.get("SQ_WAVE_CYCLES", 0.0)
        if w:
            print("SQ: wait_any %.3f  wait_inst_any %.3f  active_inst_any %.3f  active_valu %.3f" % (
                c.get("SQ_WAIT_ANY", 0) / w, c.get("SQ_WAIT_INST_ANY", 0) / w,
                c.get("SQ_ACTIVE_INST_ANY", 0) / w, c.get("SQ_ACTIVE_INST_VALU", 0) / w))
            st = res["sq"]["steps"]
            pa = res["sq"]["paths"]
            if pa:
                res["valu_wave_insts_per_path"] = c.get("SQ_INSTS_VALU", 0) / pa
                print("per lane path-step: VALU insts %.1f  SALU %.1f  VMEM %.2f" % (
                    64 * c.get("SQ_INSTS_VALU", 0) / pa, 64 * c.get("SQ_INSTS_SALU", 0) / pa,
                    64 * c.get("SQ_INSTS_VMEM", 0) / pa))
            if st:
                res["valu_wave_insts_per_step"] = c.get("SQ_INSTS_VALU", 0) / st
                res["transport_valu_issue_frac"] = (c.get("SQ_INSTS_VALU", 0) * 4.0 /
                                                    (res["sq"]["ms"] * 1e-3 * CLOCK * N_SIMD))
                print("transport VALU issue: %.3f of the chip's VALU slots" % res["transport_valu_issue_frac"])
                print("per packet-step: VALU insts %.1f  SALU %.1f  VMEM %.2f (wave-instructions x64 / steps)" % (
                    64 * c.get("SQ_INSTS_VALU", 0) / st, 64 * c.get("SQ_INSTS_SALU", 0) / st,
                    64 * c.get("SQ_INSTS_VMEM", 0) / st))
    json.dump(res, open(os.path.join(root, "summary.json"), "w"), indent=1)
    return res


def latest(res, workload_key, source):
    """The per-packet-step figures bench.py reads (profiles/pmc_latest.json)."""
    return {"workload_key": workload_key,
            "hbm_bytes_per_step": res.get("hbm_bytes_per_step"),
            "hbm_bytes_per_path": res.get("hbm_bytes_per_path"),
            "hbm_gbs_measured": res.get("hbm_gbs_measured"),
            "valu_wave_insts_per_path": res.get("valu_wave_insts_per_path"),
            "valu_wave_insts_per_step": res.get("valu_wave_insts_per_step"),
            "transport_valu_issue_frac": res.get("transport_valu_issue_frac"),
            "fp_valu_issue_frac": res.get("fp_valu_issue_frac"),
            "fp_wait_frac": res.get("fp_wait_frac"),
            "fp_simd_occupancy": res.get("fp_simd_occupancy"),
            "fp_waves": res.get("fp_waves"),
            "source": source}


if __name__ == "__main__":
    # pmc_summary.py <profile dir> [--latest <workload_key> <source text>]
    r = main(sys.argv[1])
    if len(sys.argv) > 3 and sys.argv[2] == "--latest":
        out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "pmc_latest.json")
        json.dump(latest(r, sys.argv[3], " ".join(sys.argv[4:])), open(out, "w"), indent=1)
