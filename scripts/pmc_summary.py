"""Summarise scripts/pmc.sh output: per-dispatch averages of every counter for the
main optimisation kernel of the C2 bench (largest grid), derived VALU/wait shares,
and HBM bytes per launch (FETCH_SIZE x2 per the gfx950 note of MI355X_MICROARCH.md
§HBM, + WRITE_SIZE).  Writes <outdir>/summary.json; with --commit also
profiles/pmc_traffic.json (read by bench.py for roofline.traffic)."""
import csv, glob, json, os, sys
from collections import defaultdict

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
vals = defaultdict(list)
meta = {}
for f in sorted(glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True)):
    rows = list(csv.DictReader(open(f)))
    rows = [r for r in rows if "rl_optimize_kernel" in r["Kernel_Name"] or "rl_stream_kernel" in r["Kernel_Name"]]
    if not rows:
        continue
    gmax = max(int(r["Grid_Size"]) for r in rows)
    per = defaultdict(lambda: defaultdict(float))
    for r in rows:
        if int(r["Grid_Size"]) != gmax:
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        meta = {"kernel": r["Kernel_Name"], "grid": gmax, "wg": int(r["Workgroup_Size"]),
                "vgpr": int(r["VGPR_Count"]), "sgpr": int(r["SGPR_Count"]), "scratch": int(r["Scratch_Size"])}
    for d, cs in per.items():
        for c, v in cs.items():
            vals[c].append(v)
avg = {c: sum(v) / len(v) for c, v in vals.items()}
res = {"meta": meta, "dispatches": {c: len(v) for c, v in vals.items()}, "per_launch": avg}
g = avg.get
der = {}
if g("SQ_WAVE_CYCLES"):
    wc = g("SQ_WAVE_CYCLES")
    for k in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU"):
        if g(k) is not None:
            der[k + "/WAVE_CYCLES"] = g(k) / wc
if g("SQ_WAVES") and g("SQ_INSTS_VALU"):
    w = g("SQ_WAVES")
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VALU_FMA_F64",
              "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"):
        if g(k) is not None:
            der[k + "_per_wave"] = g(k) / w
if g("GRBM_GUI_ACTIVE"):
    der["gui_active_cycles"] = g("GRBM_GUI_ACTIVE")
f64 = sum(g(k) or 0 for k in ("SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_TRANS_F64"))
if f64:
    # SQ_INSTS_VALU_* count wave-instructions; flops = 64 lanes x (2 for FMA, 1 otherwise)
    der["fp64_flops_per_launch"] = 64 * (2 * (g("SQ_INSTS_VALU_FMA_F64") or 0) + (g("SQ_INSTS_VALU_ADD_F64") or 0)
                                         + (g("SQ_INSTS_VALU_MUL_F64") or 0) + (g("SQ_INSTS_VALU_TRANS_F64") or 0))
if g("FETCH_SIZE") is not None or g("WRITE_SIZE") is not None:
    fetch = (g("FETCH_SIZE") or 0.0) * 1024.0      # rocprofv3 reports KiB
    write = (g("WRITE_SIZE") or 0.0) * 1024.0
    der["fetch_bytes_raw"] = fetch
    der["write_bytes"] = write
    der["hbm_bytes_per_launch"] = 2.0 * fetch + write
res["derived"] = der
json.dump(res, open(os.path.join(out, "summary.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
if g("SQ_INSTS_VALU") and f64:
    der["valu_fp64_share"] = f64 / g("SQ_INSTS_VALU")     # fp64 add/mul/fma/trans of all VALU instructions
if "--commit" in sys.argv and "hbm_bytes_per_launch" in der:
    # profiles/pmc_traffic.json feeds bench.py's roofline; bench.py uses an entry only when its
    # source_sha equals the hash of the kernel sources it runs (bench.source_sha)
    sys.path.insert(0, REPO)
    from bench import source_sha

    p = os.path.join(REPO, "profiles", "pmc_traffic.json")
    os.makedirs(os.path.dirname(p), exist_ok=True)     # (on the GPU box profiles/r0*/ are not uploaded: .gpurunignore)
    d = json.load(open(p)) if os.path.exists(p) else {}
    key = sys.argv[sys.argv.index("--key") + 1] if "--key" in sys.argv else "c2_mincurv"
    prof = sys.argv[sys.argv.index("--profile") + 1] if "--profile" in sys.argv else out
    d[key] = {"hbm_bytes_per_launch": der["hbm_bytes_per_launch"], "fetch_bytes_raw": der["fetch_bytes_raw"],
              "write_bytes": der["write_bytes"], "kernel": meta.get("kernel"), "source_sha": source_sha(),
              "profile": prof, "fp64_flops_per_launch": der.get("fp64_flops_per_launch"),
              "valu_fp64_share": der.get("valu_fp64_share"),
              "note": "rocprofv3 FETCH_SIZE x2 + WRITE_SIZE x1, separate --pmc passes; both factors calibrated at this kernel family's 8-B/lane access width on a 2 GiB array, plain and buffer-resource loads (profiles/r06/fetch_calib.json: read 2.000, write 1.000; the neighbour-load pattern 1.886)"}
    json.dump(d, open(p, "w"), indent=1)
