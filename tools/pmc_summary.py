"""Summarise rocprofv3 --pmc CSVs per kernel (mean counter value per dispatch).

    python tools/pmc_summary.py gpurun_out/pmc [--config c3] [--out profiles/latest_pmc.json]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced streaming reads, so it is
doubled; WRITE_SIZE is exact for 16-B-per-lane streaming stores. The path kernel's reads
are 8-B census codes (an uncalibrated width): its FETCH figure is indicative only.
"""
import argparse
import collections
import csv
import glob
import json

STAGE_OF = {"k_census9x7": "census", "k_census_paths16": "paths8", "k_census_wta16": "wta_lr", "k_census_fused16": "fused", "k_census_tiles": "rectify+census",
            "k_ocv_pixcost": "ocv_cost", "k_ocv_paths": "ocv_paths", "k_ocv_wta": "ocv_wta_lr"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", nargs="?", default="gpurun_out/pmc")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--out", default=None)
    ap.add_argument("--steady-name", default="paths7+up_wta+census",
                    help="bench stage name of the largest-grid fused launch (SGM_UPWTA=0: paths8+wta_lr+census)")
    ap.add_argument("--git", default=None, help="source revision the profiled build came from")
    args = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    grids = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{args.dir}/pass*_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            if "k_census_fused16" in k:      # one fused kernel, launches of different content: split by grid
                k = f"{k}@grid{r['Grid_Size']}"
                grids[k.split("@")[0]].add(int(r["Grid_Size"]))
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    raw = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}
    kernels = {}
    for k, cs in raw.items():
        base = k.split("<")[0].replace("sgm::", "")
        stage = STAGE_OF.get(base)
        if "@grid" in k:
            # the steady-state launch (paths of group k + WTA of k-1 + census of k+1) has the
            # largest grid; the pipeline's ramp launches are reported by grid size
            g = int(k.split("@grid")[1])
            stage = args.steady_name if g == max(grids[k.split("@")[0]]) else f"fused@grid{g}"
        if stage is None or "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = 2.0 * cs["FETCH_SIZE"] * 1024.0
        write = cs["WRITE_SIZE"] * 1024.0
        kernels[stage] = {"kernel": k, "fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                          "hbm_bytes_per_launch": fetch + write,
                          "valu_insts": cs.get("SQ_INSTS_VALU"), "salu_insts": cs.get("SQ_INSTS_SALU"),
                          "lds_insts": cs.get("SQ_INSTS_LDS")}
        if cs.get("SQ_INSTS_VALU") and cs.get("GRBM_GUI_ACTIVE"):
            # launch cycles = GRBM_GUI_ACTIVE / 8 XCDs; VALU issue ~4.2 cycles per wave64
            # instruction per SIMD for the path engine's mix, 1024 SIMDs
            cyc = cs["GRBM_GUI_ACTIVE"] / 8.0
            kernels[stage]["launch_cycles"] = cyc
            kernels[stage]["valu_busy_est"] = cs["SQ_INSTS_VALU"] / 1024.0 * 4.2 / cyc
    out = {"config": args.config, "git": args.git, "source": "rocprofv3 --pmc (tools/pmc.sh), mean per dispatch",
           "kernels": kernels, "raw": raw}
    s = json.dumps(out, indent=1)
    if args.out:
        open(args.out, "w").write(s + "\n")
    print(s)


if __name__ == "__main__":
    main()
