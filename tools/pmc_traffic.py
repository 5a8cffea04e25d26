"""PMC summaries (tools/pmc_summary.py output, one per workload) -> profiles/pmc_traffic.json:
the HBM bytes per step of each kernel family (scan "gemm", "select", "prep", "finalize") that
bench.py reports as roofline.traffic of the dominant kernel (and roofline.scan.traffic).

Correction per /opt/skills/guides/MI355X_MICROARCH.md (HBM section): on gfx950 FETCH_SIZE
counts half the bytes of 16-B/lane streaming reads (global_load and global_load ... lds
alike) -> doubled; WRITE_SIZE is exact for 16-B/lane stores.  Both are in KiB.

Per step = Σ over a family's kernels (mean bytes per dispatch × dispatches) ÷ dispatches of the
workload's once-per-step anchor kernel.

    python tools/pmc_traffic.py KEY summary.json [profiles/pmc_traffic.json]
    KEY: f32 (configs[1] scan3) | c3 (configs[2] hybrid) | c4 | c5 (sharded bf16)
"""
import json
import os
import sys

# kernel families of bench.py's kernels_us_per_step (bb_get_profile) -> kernel name prefixes
FAMILIES = {
    "gemm": ("bb::scan3_kernel", "bb::scan2_kernel", "bb::scan4_kernel", "bb::scan4_dual_kernel",
             "bb::(anonymous namespace)::sq_scan_kernel"),
    "select": ("bb::select_list_kernel", "bb::select_list_dual_kernel", "bb::select_kernel", "bb::select_rr_wave",
               "bb::cand_select_kernel", "bb::cand_select_wave_kernel", "bb::pilot_bound", "bb::(anonymous namespace)::sq_merge_kernel"),
    "prep": ("bb::prep_kernel", "bb::prep2_kernel"),
    "finalize": ("bb::finalize1_kernel", "bb::finalize1_small_kernel", "bb::finalize1_mid_kernel", "bb::finalize_kernel"),
    "rerank": ("bb::rerank_kernel",),
    "pack": ("bb::compact_kernel",),
}
ANCHOR = {"f32": ("bb::select_list_kernel", "bb::select_kernel", "bb::scan3_kernel"), "c3": ("bb::finalize1_mid_kernel", "bb::finalize1_small_kernel", "bb::finalize1_kernel"),
          "c4": ("bb::finalize_kernel", "bb::finalize1_kernel"), "c5": ("bb::finalize_kernel", "bb::finalize1_kernel")}


def main(key, src, dst):
    summ = json.load(open(src))
    try:
        out = json.load(open(dst))
    except Exception:
        out = {}
    anchor = None
    for a in ANCHOR[key]:
        hit = [v["_dispatches"] for k, v in summ.items() if k.startswith(a) and "_dispatches" in v]
        if hit:
            anchor = max(hit)
            break
    if not anchor:
        print("no anchor kernel in", src)
        return
    entry = {}
    for fam, prefixes in FAMILIES.items():
        ks = {k: v for k, v in summ.items() if k.startswith(prefixes) and "FETCH_SIZE" in v and "WRITE_SIZE" in v}
        if not ks:
            continue
        rd = sum(2.0 * v["FETCH_SIZE"] * 1024 * v["_dispatches"] for v in ks.values()) / anchor
        wr = sum(v["WRITE_SIZE"] * 1024 * v["_dispatches"] for v in ks.values()) / anchor
        entry[fam] = {
            "kernels": {k: {"fetch_size_kib": v["FETCH_SIZE"], "write_size_kib": v["WRITE_SIZE"],
                            "dispatches": v["_dispatches"]} for k, v in ks.items()},
            "steps": anchor,
            "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr,
            "hbm_bytes_per_launch": rd + wr,
            "unit_note": f"per step of the {fam} launches",
            "correction": "FETCH_SIZE x2 (gfx950 16-B/lane reads), WRITE_SIZE x1; KiB -> bytes",
            "source": os.path.relpath(src, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}
    out[key] = entry
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({f: e["hbm_bytes_per_launch"] for f, e in entry.items()}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else
         os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_traffic.json"))
